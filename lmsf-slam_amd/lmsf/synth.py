"""Synthetic VLP-16-shaped scans and LOAM feature maps (SURVEY.md §8(d) "Synthetic scan generator").

The reference ships no scan data (its one known-answer test reads PCDs that are not in the
repository: src/MultiSensorFusionEstimator3D/src/test/registration/feature_registration_test.cpp:56-60),
so every workload here is procedural and seeded:

* scene   -- ground plane 1.8 m below the sensor, rows of axis-aligned buildings along a road,
             vertical poles (r = 0.15 m, the edge features), a few tilted planes;
* scan    -- analytic ray cast in the VLP-16 firing order (-15, 1, -13, 3, ... 15 deg) inside each
             azimuth column, columns azimuth-major, range noise N(0, 0.01 m), intensity U[0, 1),
             max range 100 m; points in the lidar frame as float32 (x, y, z, intensity);
* map     -- points sampled on the same surfaces ("loam_surf") and along building edges / poles
             ("loam_edge") to an exact total count, world frame, float32;
* poses   -- world <- lidar, stored (qx, qy, qz, qw, tx, ty, tz) like the reference's parameter
             block (REG/ceres_edgeSurfFeatureRegistration.hpp:38-40).

Seeds follow SURVEY.md: config k uses 1000+k (scene), 2000+k (noise), 3000+k (perturbations).
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

VLP16_FIRING_DEG = np.array([-15, 1, -13, 3, -11, 5, -9, 7, -7, 9, -5, 11, -3, 13, -1, 15], dtype=np.float64)
GROUND_Z = -1.8
POLE_R = 0.15
MAX_RANGE = 100.0


@dataclasses.dataclass
class Scene:
    boxes: np.ndarray   # (K, 6) xmin ymin zmin xmax ymax zmax
    poles: np.ndarray   # (P, 4) cx cy zbot ztop
    planes: np.ndarray  # (Q, 14) c(3) n(3) u(3) v(3) hu hv  (bounded rectangles)
    x_range: tuple      # extent of the road used for the trajectory


def _unit(v):
    return v / np.linalg.norm(v)


def make_scene(seed: int, road_length: float = 80.0) -> Scene:
    """Urban canyon along +x: building rows on both sides, poles at the kerbs, a few ramps."""
    rng = np.random.default_rng(seed)
    x0, x1 = -140.0, road_length + 140.0
    boxes = []
    for side in (-1.0, 1.0):
        x = x0
        while x < x1:
            w = rng.uniform(8.0, 22.0)
            d = rng.uniform(8.0, 25.0)
            h = rng.uniform(6.0, 32.0)
            y_near = rng.uniform(9.0, 14.0)
            if side > 0:
                boxes.append([x, y_near, GROUND_Z, x + w, y_near + d, GROUND_Z + h])
            else:
                boxes.append([x, -y_near - d, GROUND_Z, x + w, -y_near, GROUND_Z + h])
            x += w + rng.uniform(0.5, 4.0)
        # second row further back so upward beams hit something
        x = x0
        while x < x1:
            w = rng.uniform(15.0, 40.0)
            h = rng.uniform(20.0, 45.0)
            y_near = rng.uniform(45.0, 60.0)
            d = rng.uniform(10.0, 20.0)
            if side > 0:
                boxes.append([x, y_near, GROUND_Z, x + w, y_near + d, GROUND_Z + h])
            else:
                boxes.append([x, -y_near - d, GROUND_Z, x + w, -y_near, GROUND_Z + h])
            x += w + rng.uniform(1.0, 6.0)
    poles = []
    for side in (-1.0, 1.0):
        x = x0 + rng.uniform(0, 10)
        while x < x1:
            poles.append([x, side * rng.uniform(6.5, 7.5), GROUND_Z, GROUND_Z + rng.uniform(3.0, 8.0)])
            x += rng.uniform(8.0, 18.0)
    planes = []
    for _ in range(6):
        c = np.array([rng.uniform(x0 + 40, x1 - 40), rng.choice([-1, 1]) * rng.uniform(20, 40), GROUND_Z + rng.uniform(1, 4)])
        n = _unit(np.array([rng.uniform(-0.4, 0.4), rng.uniform(-0.4, 0.4), 1.0]))
        u = _unit(np.cross(n, [0.0, 0.0, 1.0]) if abs(n[2]) < 0.99 else np.cross(n, [1.0, 0.0, 0.0]))
        v = np.cross(n, u)
        planes.append(np.concatenate([c, n, u, v, [rng.uniform(3, 8), rng.uniform(3, 8)]]))
    return Scene(np.array(boxes), np.array(poles), np.array(planes), (0.0, road_length))


def trajectory(n: int, seed: int, step: float = 1.0, start_x: float = 0.0) -> np.ndarray:
    """Ground-truth world<-lidar poses, 10 Hz, <= 10 m/s, yaw rate <= 30 deg/s, small roll/pitch."""
    rng = np.random.default_rng(seed)
    poses = np.zeros((n, 7))
    amp, lam = 1.5, 40.0
    for k in range(n):
        x = start_x + k * step
        y = amp * math.sin(x / lam)
        yaw = math.atan(amp / lam * math.cos(x / lam)) + rng.normal(0, 0.01)
        roll, pitch = rng.normal(0, 0.005), rng.normal(0, 0.005)
        poses[k, :4] = quat_from_rpy(roll, pitch, yaw)
        poses[k, 4:] = (x, y, rng.normal(0, 0.02))
    return poses


# ----------------------------------------------------------------------------- pose helpers
def quat_from_rpy(roll, pitch, yaw):
    cr, sr = math.cos(roll / 2), math.sin(roll / 2)
    cp, sp = math.cos(pitch / 2), math.sin(pitch / 2)
    cy, sy = math.cos(yaw / 2), math.sin(yaw / 2)
    w = cr * cp * cy + sr * sp * sy
    x = sr * cp * cy - cr * sp * sy
    y = cr * sp * cy + sr * cp * sy
    z = cr * cp * sy - sr * sp * cy
    return np.array([x, y, z, w])


def quat_to_mat(q):
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([
        aw * bx + ax * bw + ay * bz - az * by,
        aw * by + ay * bw + az * bx - ax * bz,
        aw * bz + az * bw + ax * by - ay * bx,
        aw * bw - ax * bx - ay * by - az * bz,
    ])


def axis_angle_quat(rv):
    th = float(np.linalg.norm(rv))
    if th < 1e-15:
        return np.array([0.0, 0.0, 0.0, 1.0])
    ax = rv / th
    s = math.sin(th / 2)
    return np.array([ax[0] * s, ax[1] * s, ax[2] * s, math.cos(th / 2)])


def perturb(pose, rng, sigma_t=0.1, sigma_r_deg=1.0):
    """Initial guess = ground truth o perturbation (sigma_t 0.1 m, sigma_r 1 deg)."""
    dq = axis_angle_quat(rng.normal(0, math.radians(sigma_r_deg), 3))
    out = np.array(pose, dtype=np.float64).copy()
    out[:4] = quat_mul(pose[:4], dq)
    out[4:] = pose[4:] + rng.normal(0, sigma_t, 3)
    return out


def pose_delta(a, b):
    """(translation error m, rotation error rad) between two (q, t) poses.  The angle is the log map of the
    relative rotation, 2 atan2(|v|, |w|) of r = conj(qa) qb: it resolves angles down to ~1e-16 rad, where
    the acos of a dot product stops at its sqrt(2 eps) ~ 3e-8 floor."""
    dt = float(np.linalg.norm(np.asarray(a[4:]) - np.asarray(b[4:])))
    return dt, rot_angle_between(a[:4], b[:4])


def rot_angle_between(qa, qb):
    """Angle of conj(qa) * qb (quaternions x, y, z, w; normalised here) by 2 atan2(|vec|, |w|)."""
    qa = np.asarray(qa, np.float64) / np.linalg.norm(qa)
    qb = np.asarray(qb, np.float64) / np.linalg.norm(qb)
    ax, ay, az, aw = -qa[0], -qa[1], -qa[2], qa[3]
    bx, by, bz, bw = qb
    w = aw * bw - ax * bx - ay * by - az * bz
    x = aw * bx + ax * bw + ay * bz - az * by
    y = aw * by + ay * bw + az * bx - ax * bz
    z = aw * bz + az * bw + ax * by - ay * bx
    return 2.0 * math.atan2(math.sqrt(x * x + y * y + z * z), abs(w))


def rot_angle_of_matrix(R):
    """Rotation angle of a 3x3 rotation matrix: atan2(|vee(R - R^T)| / 2, (tr R - 1) / 2), accurate at small
    angles (no acos)."""
    R = np.asarray(R, np.float64)
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]) * 0.5
    return float(math.atan2(float(np.linalg.norm(v)), (float(np.trace(R)) - 1.0) * 0.5))


# ----------------------------------------------------------------------------- ray casting
def raycast(scene: Scene, origin: np.ndarray, dirs: np.ndarray, max_range: float = MAX_RANGE) -> np.ndarray:
    """Nearest hit distance along unit world-frame directions (inf when nothing within max_range)."""
    o = origin.astype(np.float64)
    d = dirs.astype(np.float64)
    best = np.full(d.shape[0], np.inf)
    with np.errstate(divide="ignore", invalid="ignore"):
        # ground
        t = (GROUND_Z - o[2]) / d[:, 2]
        ok = (d[:, 2] < 0) & (t > 0)
        best = np.where(ok & (t < best), t, best)
        inv = 1.0 / d
        # boxes / poles farther than max_range from the origin can only give hits that are dropped
        # below (culling them leaves the result bit-identical and halves the cost of a scan)
        gap = np.maximum(np.maximum(scene.boxes[:, :3] - o, o - scene.boxes[:, 3:]), 0.0)
        near_boxes = scene.boxes[np.sqrt((gap ** 2).sum(1)) <= max_range]
        for b in near_boxes:
            t1 = (b[:3] - o) * inv
            t2 = (b[3:] - o) * inv
            tn = np.max(np.minimum(t1, t2), axis=1)
            tf = np.min(np.maximum(t1, t2), axis=1)
            hit = (tn <= tf) & (tn > 1e-6)
            best = np.where(hit & (tn < best), tn, best)
        dxy2 = d[:, 0] ** 2 + d[:, 1] ** 2
        pole_d = np.hypot(scene.poles[:, 0] - o[0], scene.poles[:, 1] - o[1]) - POLE_R if len(scene.poles) else np.zeros(0)
        for p in scene.poles[pole_d <= max_range] if len(scene.poles) else scene.poles:
            ox, oy = o[0] - p[0], o[1] - p[1]
            bq = 2 * (ox * d[:, 0] + oy * d[:, 1])
            cq = ox * ox + oy * oy - POLE_R * POLE_R
            disc = bq * bq - 4 * dxy2 * cq
            sq = np.sqrt(np.maximum(disc, 0))
            tt = (-bq - sq) / (2 * dxy2)
            z = o[2] + tt * d[:, 2]
            hit = (disc > 0) & (tt > 1e-6) & (z >= p[2]) & (z <= p[3])
            best = np.where(hit & (tt < best), tt, best)
        for pl in scene.planes:
            c, n, u, v, hu, hv = pl[0:3], pl[3:6], pl[6:9], pl[9:12], pl[12], pl[13]
            den = d @ n
            tt = ((c - o) @ n) / den
            hp = o[None, :] + tt[:, None] * d - c[None, :]
            hit = (np.abs(den) > 1e-9) & (tt > 1e-6) & (np.abs(hp @ u) <= hu) & (np.abs(hp @ v) <= hv)
            best = np.where(hit & (tt < best), tt, best)
    best[best > max_range] = np.inf
    return best


def scan_directions(n_cols: int, elev_deg: np.ndarray, clockwise: bool = False) -> np.ndarray:
    """Lidar-frame unit rays, azimuth-major, firing order inside each column.  clockwise=True sweeps
    like a Velodyne seen from above (-atan2(y, x) increasing, the direction
    RotaryLidar_preprocessing.hpp:38 assumes)."""
    az = 2 * np.pi * np.arange(n_cols) / n_cols
    if clockwise:
        az = -az
    el = np.radians(elev_deg)
    A, E = np.meshgrid(az, el, indexing="ij")
    d = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], axis=-1)
    return d.reshape(-1, 3)


def make_scan(scene: Scene, pose: np.ndarray, seed: int, n_cols: int = 4096,
              elev_deg: np.ndarray = VLP16_FIRING_DEG, range_noise: float = 0.01,
              organized: bool = False, clockwise: bool = False) -> np.ndarray:
    """One revolution seen from world<-lidar `pose`; returns (N, 4) float32 lidar-frame x y z i.
    organized=True keeps one row per ray (NaN x y z for no return), as a driver's organized cloud."""
    rng = np.random.default_rng(seed)
    dl = scan_directions(n_cols, np.asarray(elev_deg, dtype=np.float64), clockwise)
    R = quat_to_mat(pose[:4])
    dw = dl @ R.T
    r = raycast(scene, np.asarray(pose[4:]), dw)
    keep = np.isfinite(r)
    rr = r[keep] + rng.normal(0, range_noise, int(keep.sum()))
    pts = dl[keep] * rr[:, None]
    if organized:
        out = np.full((dl.shape[0], 4), np.nan, dtype=np.float32)
        out[keep, :3] = pts
        out[:, 3] = rng.random(dl.shape[0])
        return out
    out = np.empty((pts.shape[0], 4), dtype=np.float32)
    out[:, :3] = pts
    out[:, 3] = rng.random(pts.shape[0])
    return out


def to_pointcloud2(points: np.ndarray, point_step: int = 32) -> np.ndarray:
    """sensor_msgs/PointCloud2 data bytes in the velodyne_pointcloud layout (x 0, y 4, z 8,
    intensity 16, ring uint16 20, little endian); returns a uint8 array of n * point_step bytes."""
    n = len(points)
    buf = np.zeros((n, point_step), np.uint8)
    f = np.ascontiguousarray(points[:, :4], dtype="<f4")
    buf[:, 0:12] = f[:, :3].view(np.uint8).reshape(n, 12)
    buf[:, 16:20] = f[:, 3:4].view(np.uint8).reshape(n, 4)
    if point_step >= 22:
        buf[:, 20:22] = (np.arange(n) % 16).astype("<u2").view(np.uint8).reshape(n, 2)
    return buf.reshape(-1)


# ----------------------------------------------------------------------------- maps
def _in_any_footprint(scene, p):
    inside = np.zeros(p.shape[0], dtype=bool)
    for b in scene.boxes:
        inside |= (p[:, 0] > b[0]) & (p[:, 0] < b[3]) & (p[:, 1] > b[1]) & (p[:, 1] < b[4])
    return inside


def make_map(scene: Scene, n_points: int, seed: int, center_x=(0.0, 80.0), radius: float = 100.0,
             edge_frac: float = 0.1, noise: float = 0.005):
    """Edge / surf feature maps (world frame) with exactly n_points in total.

    Surf points are area-weighted on ground, building walls + roofs, pole mantles and tilted
    planes inside the slab |y| <= radius, x in [center_x[0]-radius, center_x[1]+radius]; edge
    points lie along building vertical / roof / foot edges and on pole mantles.
    """
    rng = np.random.default_rng(seed)
    xlo, xhi = center_x[0] - radius, center_x[1] + radius
    ylo, yhi = -radius, radius
    n_edge = int(round(n_points * edge_frac))
    n_surf = n_points - n_edge

    def clip_box(b):
        return np.array([max(b[0], xlo), max(b[1], ylo), b[2], min(b[3], xhi), min(b[4], yhi), b[5]])

    boxes = [clip_box(b) for b in scene.boxes if b[3] > xlo and b[0] < xhi and b[4] > ylo and b[1] < yhi]
    poles = [p for p in scene.poles if xlo <= p[0] <= xhi]
    # --- surf: list of (area, sampler)
    faces = []
    faces.append(((xhi - xlo) * (yhi - ylo), ("ground",)))
    for b in boxes:
        dx, dy, dz = b[3] - b[0], b[4] - b[1], b[5] - b[2]
        faces += [(dy * dz, ("wx", b, b[0])), (dy * dz, ("wx", b, b[3])),
                  (dx * dz, ("wy", b, b[1])), (dx * dz, ("wy", b, b[4])), (dx * dy, ("roof", b))]
    for p in poles:
        faces.append((2 * np.pi * POLE_R * (p[3] - p[2]), ("pole", p)))
    for pl in scene.planes:
        if xlo <= pl[0] <= xhi:
            faces.append((4 * pl[12] * pl[13], ("plane", pl)))
    areas = np.array([f[0] for f in faces])
    counts = rng.multinomial(n_surf, areas / areas.sum())
    surf = []
    for (area, f), c in zip(faces, counts):
        if c == 0:
            continue
        kind = f[0]
        if kind == "ground":
            p = np.stack([rng.uniform(xlo, xhi, c), rng.uniform(ylo, yhi, c), np.full(c, GROUND_Z)], 1)
        elif kind == "wx":
            b = f[1]
            p = np.stack([np.full(c, f[2]), rng.uniform(b[1], b[4], c), rng.uniform(b[2], b[5], c)], 1)
        elif kind == "wy":
            b = f[1]
            p = np.stack([rng.uniform(b[0], b[3], c), np.full(c, f[2]), rng.uniform(b[2], b[5], c)], 1)
        elif kind == "roof":
            b = f[1]
            p = np.stack([rng.uniform(b[0], b[3], c), rng.uniform(b[1], b[4], c), np.full(c, b[5])], 1)
        elif kind == "pole":
            pp = f[1]
            a = rng.uniform(0, 2 * np.pi, c)
            p = np.stack([pp[0] + POLE_R * np.cos(a), pp[1] + POLE_R * np.sin(a), rng.uniform(pp[2], pp[3], c)], 1)
        else:
            pl = f[1]
            su, sv = rng.uniform(-pl[12], pl[12], c), rng.uniform(-pl[13], pl[13], c)
            p = pl[0:3][None] + su[:, None] * pl[6:9][None] + sv[:, None] * pl[9:12][None]
        surf.append(p)
    # ground points under building footprints are redrawn on free ground
    g = surf[0]
    bad = _in_any_footprint(scene, g)
    while bad.any():
        k = int(bad.sum())
        g[bad] = np.stack([rng.uniform(xlo, xhi, k), rng.uniform(ylo, yhi, k), np.full(k, GROUND_Z)], 1)
        bad = _in_any_footprint(scene, g)
    surf = np.concatenate(surf, 0)
    # --- edge: segments
    segs = []
    for b in boxes:
        x0, y0, z0, x1, y1, z1 = b
        for (cx, cy) in ((x0, y0), (x0, y1), (x1, y0), (x1, y1)):
            segs.append(((cx, cy, z0), (cx, cy, z1)))
        for z in (z0, z1):
            segs += [((x0, y0, z), (x1, y0, z)), ((x0, y1, z), (x1, y1, z)),
                     ((x0, y0, z), (x0, y1, z)), ((x1, y0, z), (x1, y1, z))]
    seg_a = np.array([s[0] for s in segs])
    seg_b = np.array([s[1] for s in segs])
    seg_len = np.linalg.norm(seg_b - seg_a, axis=1)
    pole_len = np.array([p[3] - p[2] for p in poles]) if poles else np.zeros(0)
    lens = np.concatenate([seg_len, pole_len])
    counts = rng.multinomial(n_edge, lens / lens.sum())
    edge = []
    ns = len(segs)
    for i, c in enumerate(counts):
        if c == 0:
            continue
        if i < ns:
            t = rng.random(c)
            edge.append(seg_a[i][None] + t[:, None] * (seg_b[i] - seg_a[i])[None])
        else:
            pp = poles[i - ns]
            a = rng.uniform(0, 2 * np.pi, c)
            edge.append(np.stack([pp[0] + POLE_R * np.cos(a), pp[1] + POLE_R * np.sin(a), rng.uniform(pp[2], pp[3], c)], 1))
    edge = np.concatenate(edge, 0)
    surf = surf + rng.normal(0, noise, surf.shape)
    edge = edge + rng.normal(0, noise, edge.shape)
    perm_s = rng.permutation(surf.shape[0])
    perm_e = rng.permutation(edge.shape[0])

    def pack(p):
        out = np.empty((p.shape[0], 4), dtype=np.float32)
        out[:, :3] = p
        out[:, 3] = rng.random(p.shape[0])
        return out

    return pack(edge[perm_e]), pack(surf[perm_s])


def transform_points(pose, pts):
    """World <- lidar transform of float32 xyzi rows (float64 math, float32 out)."""
    R = quat_to_mat(pose[:4])
    out = pts.copy()
    out[:, :3] = (pts[:, :3].astype(np.float64) @ R.T + np.asarray(pose[4:])).astype(np.float32)
    return out


# ----------------------------------------------------------------------------- configs
BEAMS128_DEG = np.linspace(-25.0, 15.0, 128)          # C5: 128 beams evenly in [-25, 15] deg
HDL64_DEG = np.concatenate([np.linspace(2.0, -8.33, 32), np.linspace(-8.83, -24.33, 32)])
# C3 sub-lidar extrinsic primary <- sub (qx qy qz qw tx ty tz),
# config/MultiLidar_system/loam_feature_multi_lidar_system.yaml:73-74 ("PS-Calib")
DUAL_EXTRINSIC = np.array([0.34087, -0.0101817, 0.0147921, 0.945613, 0.0334837, -0.540249, -0.141798])

CONFIGS = {
    # n_cols per revolution, map points, map slab radius, seed index k; elev = beam table,
    # extract = lmsf_config overrides the extraction needs for that beam table
    "C1": dict(n_cols=1800, map_points=200_000, radius=60.0, k=1, elev=VLP16_FIRING_DEG, extract={}),
    "C2": dict(n_cols=4096, map_points=1_000_000, radius=100.0, k=2, elev=VLP16_FIRING_DEG, extract={}),
    "C3": dict(n_cols=4096, map_points=1_000_000, radius=100.0, k=3, elev=VLP16_FIRING_DEG, extract={}),
    "C4": dict(n_cols=4096, map_points=5_000_000, radius=100.0, k=4, elev=VLP16_FIRING_DEG, extract={}),
    "C5": dict(n_cols=2048, map_points=10_000_000, radius=100.0, k=5, elev=BEAMS128_DEG,
               extract=dict(n_scans=128, beam_lo_deg=-25.0, beam_spacing_deg=40.0 / 127)),
}


def unit_extrinsic(x):
    """Normalised copy of a (q, t) pose (the YAML quaternion is rounded to 6 digits)."""
    y = np.array(x, dtype=np.float64)
    y[:4] /= np.linalg.norm(y[:4])
    return y


def compose(a, b):
    """(q, t) poses: a * b."""
    R = quat_to_mat(a[:4])
    out = np.empty(7)
    out[:4] = quat_mul(a[:4], b[:4])
    out[4:] = R @ np.asarray(b[4:]) + np.asarray(a[4:])
    return out


@dataclasses.dataclass
class DualSequence:
    scene: Scene
    truth: np.ndarray        # primary LiDAR world <- lidar poses (q, t)
    extrinsic: np.ndarray    # primary <- sub (q, t), normalised PS-Calib value
    primary: list            # raw scans, primary frame
    sub: list                # raw scans, sub frame


def make_dual_sequence(n: int, n_cols: int = 4096, step: float = 0.5, k: int = 3, start_x: float = 0.0,
                       elev=VLP16_FIRING_DEG) -> DualSequence:
    """C3: two rigidly mounted 16-beam LiDARs (MultiLidar_system config: lidar_num 2, n_scans 16)
    at the reference's PS-Calib extrinsic, 10 Hz frames along the road."""
    scene = make_scene(1000 + k)
    truth = trajectory(n, 3000 + k, step=step, start_x=start_x)
    X = unit_extrinsic(DUAL_EXTRINSIC)
    prim = [make_scan(scene, truth[i], 2000 + k + 97 * i, n_cols=n_cols, elev_deg=elev) for i in range(n)]
    sub = [make_scan(scene, compose(truth[i], X), 2500 + k + 97 * i, n_cols=n_cols, elev_deg=elev) for i in range(n)]
    return DualSequence(scene, truth, X, prim, sub)


@dataclasses.dataclass
class Workload:
    scene: Scene
    edge_map: np.ndarray
    surf_map: np.ndarray
    scans: list
    truth: np.ndarray
    guess: np.ndarray


def make_workload(config: str = "C2", n_scans: int = 4, map_points: int | None = None,
                  n_cols: int | None = None, road_length: float = 80.0, radius: float | None = None) -> Workload:
    """Scene, ground-truth trajectory, perturbed initial guesses, scans and the feature map.
    `radius` / `road_length` shrink the mapped region for small test maps (keeps density)."""
    c = CONFIGS[config]
    k = c["k"]
    scene = make_scene(1000 + k, road_length=80.0)
    truth = trajectory(n_scans, 3000 + k, step=road_length / max(n_scans, 1))
    rng = np.random.default_rng(3000 + k)
    guess = np.stack([perturb(p, rng) for p in truth]) if n_scans else np.zeros((0, 7))
    scans = [make_scan(scene, truth[i], 2000 + k + 97 * i, n_cols=n_cols or c["n_cols"], elev_deg=c["elev"])
             for i in range(n_scans)]
    em, sm = make_map(scene, map_points or c["map_points"], 1000 + k + 7, center_x=(0.0, road_length),
                      radius=radius or c["radius"])
    return Workload(scene, em, sm, scans, truth, guess)
