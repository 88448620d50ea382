# r04: C5 pass 1 without the fit, one fit kernel -- GPU suite (C5 full size byte-exact), one-stream C5 kernel traces,
# C5 A/B over the walk kernel's occupancy.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
mkdir -p gpurun_out/c5split1
for v in p1split p1nosplit; do
  LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5split1/$v -o run --output-format csv -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 1 > gpurun_out/c5split1/$v.json 2> gpurun_out/c5split1/$v.err
  rc=$?; echo "trace $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
CONFIGS=C5 VARIANTS="p1split p1w8 p1nosplit" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
