# r04: C3 repeat diagnostic (a one-off deviation in the GPU suite), the C5 full-size byte-exact test with the pass-1
# split, C5 kernel traces and A/B.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u tools/c3_repeat_diag.py 4 > gpurun_out/c3_repeat.log 2>&1
rc=$?; echo "c3diag rc=$rc"; grep -v "^W2026\|^I2026" gpurun_out/c3_repeat.log | tail -14; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider -k c5 --timeout 300 --timeout-method thread > gpurun_out/c5_test.log 2>&1
rc=$?; echo "c5test rc=$rc"; tail -2 gpurun_out/c5_test.log; case $rc in 0) ;; *) exit $rc;; esac
mkdir -p gpurun_out/c5split1
for v in p1split p1nosplit; do
  LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5split1/$v -o run --output-format csv -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 1 > gpurun_out/c5split1/$v.json 2> gpurun_out/c5split1/$v.err
  rc=$?; echo "trace $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
CONFIGS=C5 VARIANTS="p1split p1w8 p1nosplit" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
