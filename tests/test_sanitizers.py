"""Host-code sanitizers: the CPU restatement and the library's host-only hand-eye
code built with -fsanitize=address,undefined and driven once through every entry point
(tests/cpp/sanitize_driver.cpp).  Device code is not sanitized (GPU ASan is unavailable on the
pool); the device kernels are covered by the parity tests."""
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_oracle_and_handeye_under_asan_ubsan(tmp_path):
    from lmsf import synth
    wl = synth.make_workload("C1", n_scans=1, map_points=60_000, n_cols=900, road_length=10.0, radius=30.0)
    org = synth.make_scan(wl.scene, wl.truth[0], 5, n_cols=900, organized=True, clockwise=True)
    files = {"scan": wl.scans[0], "edge": wl.edge_map, "surf": wl.surf_map}
    for k, v in files.items():
        np.ascontiguousarray(v, np.float32).tofile(tmp_path / f"{k}.bin")
    synth.to_pointcloud2(org).tofile(tmp_path / "msg.bin")
    exe = tmp_path / "sanitize_driver"
    oracle = os.path.join(REPO, "oracle")
    srcs = [os.path.join(oracle, f) for f in ("extract.cpp", "kdtree.cpp", "registration.cpp", "saes.cpp", "voxel.cpp",
                                              "ingest.cpp")]
    srcs += [os.path.join(REPO, "lmsf-slam_amd", "csrc", "calib.cpp"), os.path.join(REPO, "tests", "cpp",
                                                                                   "sanitize_driver.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=undefined", "-fopenmp", "-ffp-contract=off", "-I", oracle, "-I",
                    os.path.join(REPO, "include"), *srcs, "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    out = subprocess.run([str(exe), *(str(tmp_path / f"{k}.bin") for k in ("scan", "edge", "surf", "msg")),
                          str(len(org))], capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr[-4000:]
    f = out.stdout.split()
    assert int(f[1]) > 0 and int(f[2]) > 0 and int(f[-1]) == 1, out.stdout
