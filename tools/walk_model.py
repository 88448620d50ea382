"""Candidate counts of the C2 rows-first walk: mode 0 = the kernel's walk (rows nearest
first, a row skipped when its yz-gap bound exceeds the 6th key), 1 = the other 8 rows re-trimmed to the 6th key found
in the own row.  CPU only: python tools/walk_model.py"""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', 'lmsf-slam_amd'))
from lmsf import synth
wl = synth.make_workload("C2", n_scans=1)
M = np.asarray(wl.surf_map)[:, :3].astype(np.float32)
sx = 4
ox, oy, oz = np.floor(M[:,0]*sx).min().astype(int), np.floor(M[:,1]).min().astype(int), np.floor(M[:,2]).min().astype(int)
cx = (np.floor(M[:,0]*sx).astype(int)-ox); cy = np.floor(M[:,1]).astype(int)-oy; cz = np.floor(M[:,2]).astype(int)-oz
nx, ny, nz = cx.max()+1, cy.max()+1, cz.max()+1
lin = (cz*ny+cy)*nx+cx
order = np.argsort(lin, kind='stable'); P = M[order]; L = lin[order]
off = np.searchsorted(L, np.arange(nx*ny*nz+1))
scan = np.asarray(wl.scans[0])[:, :3]
pose = wl.truth[0]
Q = synth.transform_points(pose, scan).astype(np.float32)
rng = np.random.default_rng(0)
Q = Q[rng.choice(len(Q), 4000, replace=False)]
near = [4,1,3,5,7,0,2,6,8]
def rows(w):
    fx, fy, fz = np.floor(w)
    out = []
    for rr in near:
        dyo, dzo = rr%3-1, rr//3-1
        cxs = int(fx*sx)-ox; ccy = int(fy)-oy+dyo; ccz = int(fz)-oz+dzo
        if not (0<=ccy<ny and 0<=ccz<nz): out.append(None); continue
        xa, xb = max(cxs-sx,0), min(cxs+2*sx-1, nx-1)
        ylo, zlo = fy+dyo, fz+dzo
        gy = max(0., ylo-w[1], w[1]-(ylo+1)); gz = max(0., zlo-w[2], w[2]-(zlo+1))
        out.append((ccy, ccz, xa, xb, gy*gy+gz*gz))
    return out
def walk(w, mode):
    R = rows(w); keys = []; cand = 0; d6 = 1.0
    for i, r in enumerate(R):
        if r is None: continue
        ccy, ccz, xa, xb, lb = r
        if lb > d6: continue
        lim = 1.0 + 1e-5
        if mode == 1 and i > 0: lim = min(lim, d6*(1+1e-5))
        if mode == 2: lim = min(lim, d6*(1+1e-5))
        rem = lim - lb
        if rem < 0: continue
        rad = np.sqrt(rem)
        sa = max(xa, int(np.floor((w[0]-rad)*sx))-ox); sb = min(xb, int(np.floor((w[0]+rad)*sx))-ox)
        if sa > sb: continue
        base = (ccz*ny+ccy)*nx
        a, b = off[base+sa], off[base+sb+1]
        cand += b-a
        if b > a:
            d = ((P[a:b]-w)**2).sum(1)
            keys = sorted(list(keys)+list(d[d < 1+1e-5]))[:6]
            if len(keys) == 6: d6 = keys[5]
    return cand
for mode in (0, 1, 2):
    c = [walk(w, mode) for w in Q]
    print(mode, np.mean(c))
