"""the reference-side PCL adapters (include/lmsf/lmsf_pcl.hpp) executed on the device.

tests/cpp/bin/pcl_adapter_run (built by __graft_entry__.build() against the reference's own plugin bases, included
in place where /root/reference exists; tests/pcl_stubs.py) constructs HipLOAMFeatureProcessor<P, P>(16, 2, 80),
HipPointCloudCommonProcess<P>("filtered") and HipEdgeSurfFeatureRegistration<P>("loam_edge", "loam_surf") on device 0
and drives them only through PointCloudProcessBase<P, P>::Process (processing/process_base.hpp:26-39) and
RegistrationBase<P>::{SetInputSource, SetInputTarget, Solve} (REG/registration_base.hpp:25-34).  Its "loam_edge" /
"loam_surf" / "filtered" clouds equal the oracle's byte for byte and Solve's T (the factory default: the reference's
decay schedule, 10 -> 9 outer iterations) the oracle's to <= 1e-4 m / rad."""
import os
import subprocess

import numpy as np
import pytest

from conftest import mat_err, pose_matrix

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNER = os.path.join(REPO, "tests", "cpp", "bin", "pcl_adapter_run")


def test_pcl_adapters_run_on_device(oracle_mod, small_workload, tmp_path):
    if not os.path.exists(RUNNER):
        pytest.skip("tests/cpp/bin/pcl_adapter_run not built (build() needs the reference headers)")
    wl = small_workload
    paths = []
    for name, arr in (("scan", wl.scans[0]), ("edge", wl.edge_map), ("surf", wl.surf_map)):
        p = tmp_path / f"{name}.bin"
        np.ascontiguousarray(arr, np.float32).tofile(p)
        paths.append(str(p))
    g = wl.guess[0]
    voxel, near, far = 0.5, 2.0, 100.0
    run = subprocess.run([RUNNER, *paths, str(tmp_path), *[repr(float(v)) for v in g], repr(voxel), repr(near), repr(far)],
                         capture_output=True, text=True, timeout=300)
    assert run.returncode == 0 and "constructed 3" in run.stdout, run.stdout + run.stderr
    e, s, _, _ = oracle_mod.extract(wl.scans[0])
    for name, want in (("loam_edge", e), ("loam_surf", s)):
        got = np.fromfile(tmp_path / f"{name}.bin", np.float32).reshape(-1, 4)
        assert got.tobytes() == want.tobytes(), name
    filt = np.fromfile(tmp_path / "filtered.bin", np.float32).reshape(-1, 4)
    want = oracle_mod.common_process(wl.scans[0], voxel_leaf=voxel, distance_near=near, distance_far=far)
    assert filt.tobytes() == want.tobytes()
    t = np.fromfile(tmp_path / "T.bin", np.float64)
    T = np.eye(4)
    T[:3, :3] = t[:9].reshape(3, 3)
    T[:3, 3] = t[9:]
    reg = oracle_mod.Registration()             # CeresEdgeSurfFeatureRegistration defaults: decay from 10
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    ox, otr, ost = reg.solve(g)
    assert ost.outer_iterations == 9
    dt, dr = mat_err(T, pose_matrix(ox))
    assert dt <= 1e-4 and dr <= 1e-4, (dt, dr)
