import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lmsf-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblmsf_hip.so)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    oracle.set_threads(1)
    return oracle


@pytest.fixture(scope="session")
def small_workload():
    """C2-shaped (16 x 4096 VLP-16) scans against a reduced 300k-point map: seconds on the oracle."""
    from lmsf import synth
    return synth.make_workload("C2", n_scans=3, map_points=300_000)


@pytest.fixture(scope="session")
def c2_workload():
    """Full C2 workload (64k-point scans, 1M-point map)."""
    from lmsf import synth
    return synth.make_workload("C2", n_scans=2, map_points=1_000_000)


HDL64_ELEV = np.concatenate([np.linspace(2.0, -8.33, 32), np.linspace(-8.83, -24.33, 32)])


@pytest.fixture(scope="session")
def sequence_workload():
    """10 consecutive 64-beam scans (HDL-64 ring formula, 1024 columns), 10 Hz at 2.5 m/s:
    the tracker builds its own map from the first scan.  A 16-beam first scan is too sparse
    vertically to seed a scan-to-map tracker in this synthetic canyon (it drifts), 64 beams hold."""
    from types import SimpleNamespace
    from lmsf import synth
    scene = synth.make_scene(1001)
    truth = synth.trajectory(10, 3001, step=0.25)
    scans = [synth.make_scan(scene, truth[i], 2001 + 97 * i, n_cols=1024, elev_deg=HDL64_ELEV)
             for i in range(len(truth))]
    # world-frame prior map of the same stretch (multi-stream shared-map tests)
    edge_map, surf_map = synth.make_map(scene, 150_000, 1008, center_x=(0.0, 2.5), radius=35.0)
    return SimpleNamespace(scans=scans, truth=truth, n_scans=64, dt=0.1, edge_map=edge_map, surf_map=surf_map)


def saes_cases():
    """Symmetric 3x3 inputs of the edge fit's eigen-solver: 5-point covariances, near-collinear sets,
    and the special cases of Eigen's algorithm (diagonal, tridiagonal, underflowing m20, repeated)."""
    rng = np.random.default_rng(11)
    out = []
    for _ in range(3000):                   # 5-point covariances, as the edge fit builds them
        P = (rng.normal(size=(5, 3)) * rng.uniform(0.001, 1.0, 3)).astype(np.float32).astype(np.float64)
        c = P.sum(0) / 5.0
        out.append((P - c).T @ (P - c))
    for _ in range(300):                    # nearly collinear points: the accepted-edge regime
        t = rng.uniform(-0.5, 0.5, 5)
        d = rng.normal(size=3)
        P = np.outer(t, d) + rng.normal(scale=1e-3, size=(5, 3))
        c = P.sum(0) / 5.0
        out.append((P - c).T @ (P - c))
    out += [np.diag([3.0, 1.0, 2.0]), np.diag([1.0, 1.0, 1.0]), np.zeros((3, 3)),
            np.array([[2.0, 1.0, 0.0], [1.0, 2.0, 1.0], [0.0, 1.0, 2.0]]),       # already tridiagonal
            np.array([[1.0, 0.0, 1e-170], [0.0, 1.0, 0.0], [1e-170, 0.0, 1.0]]),  # m20^2 underflows
            np.array([[4.0, 2.0, 2.0], [2.0, 4.0, 2.0], [2.0, 2.0, 4.0]]),       # repeated eigenvalue
            np.ones((3, 3)), -np.eye(3), np.diag([1e-300, 1.0, 1e300])]
    return out


def pose_matrix(p):
    from lmsf import synth
    T = np.eye(4)
    T[:3, :3] = synth.quat_to_mat(p[:4])
    T[:3, 3] = p[4:]
    return T


def relative_truth(truth):
    """Ground-truth poses relative to the first scan (the tracker's local frame), 4x4."""
    from lmsf import synth
    mats = []
    for p in truth:
        T = np.eye(4)
        T[:3, :3] = synth.quat_to_mat(p[:4])
        T[:3, 3] = p[4:]
        mats.append(T)
    T0i = np.linalg.inv(mats[0])
    return [T0i @ T for T in mats]


def mat_err(A, B):
    from lmsf import synth
    dt = float(np.linalg.norm(A[:3, 3] - B[:3, 3]))
    return dt, synth.rot_angle_of_matrix(A[:3, :3].T @ B[:3, :3])


def pose_err(a, b):
    from lmsf import synth
    return synth.pose_delta(a, b)


def libm_probe_scan():
    """A 16-ring VLP-16 cylinder (r = 20 m, 1800 columns) with one extra point at index 900 whose
    x*x + y*y is 6400 + 2^-11 in float: inside max_distance 80 with the float sqrt overload, outside
    with the double one (lmsf_config::libm_float)."""
    from lmsf import synth
    rng = np.random.default_rng(3)
    az = np.linspace(0, 2 * np.pi, 1800, endpoint=False)
    rows = []
    for el in synth.VLP16_FIRING_DEG:
        r = 20.0 + rng.normal(0, 0.05, az.size)
        rows.append(np.stack([r * np.cos(az), r * np.sin(az), r * np.tan(np.radians(el)), rng.random(az.size)], 1))
    scan = np.concatenate(rows, 0).astype(np.float32)
    odd = np.array([[80.0, 0.0221, 80.0 * np.tan(np.radians(-15.0)), 0.5]], np.float32)
    return np.concatenate([scan[:900], odd, scan[900:]], 0)


def assert_captured_records(ctx, reg, slot, iters, min_matched=0.2):
    """Records and 5-NN indices the batch path kept after each outer iteration of `slot` (lmsf_batch_capture:
    fresh searches, memo reuses and refits alike) against the oracle's fresh match at the exact pose the GPU
    matched at (REG/FeatureMatch/EdgeFeatureMatch.hpp:38-80, surfFeatureMatch.hpp:37-83).  reg holds the
    slot's scan.  Byte-identical records; equal neighbour indices on every rank found within 1 m.
    Returns the per-iteration count of matched records."""
    matched = []
    for it in range(iters):
        grec, gnn, gpose = ctx.batch_records(slot, it)
        orec, onn = reg.match(gpose)
        assert len(grec) == len(orec), (slot, it)
        found = gnn >= 0
        assert np.array_equal(gnn[found], onn[found]), (slot, it, int((gnn[found] != onn[found]).sum()))
        matched5 = orec["kind"] > 0                              # a record needs the 5 found within 1 m
        assert found[matched5].all(), (slot, it)
        if grec.tobytes() != orec.tobytes():
            diff = np.nonzero((grec.view(np.uint8).reshape(len(grec), -1) !=
                               orec.view(np.uint8).reshape(len(orec), -1)).any(1))[0]
            raise AssertionError(f"slot {slot} outer iteration {it}: {len(diff)} records differ, first {diff[:5]}: "
                                 f"gpu {grec[diff[:2]]} oracle {orec[diff[:2]]}")
        assert matched5.sum() > min_matched * len(orec), (slot, it)
        matched.append(int(matched5.sum()))
    return matched
