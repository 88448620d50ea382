"""Host-side equivalence checks of the extraction kernels' step-wise loops (k_extract.hip) against the
reference's sequential loops, on random inputs (no GPU):

* the bad-point skip automaton of checkBadEdgePoint (FX/LOAMFeatureProcessor_base.hpp:216-282: events
  1 / 2 skip 5 positions, event 3 disables the 6 points ending at j) walked 64 events per step with the
  step's skips followed in registers (ring_bad_points);
* the greedy edge pick of featureExtractionFromSector (FX:157-195) taken 64 sorted candidates per step,
  the step's picks resolved by "disable the candidates within 5 ring positions" (ring_features_kernel);
* the ascending-only bitonic network on keys alone followed by the index tie fix-up
  (sector_sort_regs), against a (key, index) sort.

The GPU results of the same kernels are compared bit for bit with the oracle in tests/test_gpu_parity.py
(test_extract_*); these tests pin the loop restructurings themselves on many more random cases."""
import random

import pytest

STEP = 64


def automaton_ref(ev, jmax):
    dis, j = set(), 5
    while j <= jmax:
        e = ev[j]
        if e == 1:
            dis.update(range(j - 5, j + 6))
            j += 5
        elif e == 2:
            dis.update(range(j + 1, j + 6))
            j += 5
        else:
            if e == 3:
                dis.update(range(j - 5, j + 1))
            j += 1
    return dis


def automaton_steps(ev, jmax):
    dis, pos = set(), 5
    while pos <= jmax:
        e = [ev[pos + l] if pos + l <= jmax else 0 for l in range(STEP)]
        ev12 = [x in (1, 2) for x in e]
        start = 0
        while True:
            hits = [l for l in range(start, STEP) if ev12[l]]
            f = hits[0] if hits else STEP
            for l in range(start, f):
                if e[l] == 3:
                    dis.update(range(pos + l - 5, pos + l + 1))
            if hits:
                j = pos + f
                dis.update(range(j - 5, j + 6) if e[f] == 1 else range(j + 1, j + 6))
            if not hits:
                pos += STEP
                break
            start = f + 5
            if start >= STEP:
                pos += start
                break
    return dis


def pick_ref(keys, idxs, dis0, thresh, size):
    dis, picks, picked = set(dis0), [], 0
    for i in range(len(keys) - 1, -1, -1):
        ind = idxs[i]
        if ind in dis:
            continue
        if keys[i] <= thresh:
            break
        picked += 1
        if picked > 20:
            break
        picks.append(ind)
        for q in range(1, 6):
            dis.add(min(ind + q, size - 1))
            dis.add(max(ind - q, 0))
    return picks, dis


def pick_steps(keys, idxs, dis0, thresh, size):
    dis, picks, pos, picked = set(dis0), [], len(keys) - 1, 0
    while pos >= 0 and picked < 20:
        cand = [pos - l for l in range(STEP)]
        valid = [c >= 0 for c in cand]
        idx = [idxs[c] if v else -100 for c, v in zip(cand, valid)]
        above = [v and keys[c] > thresh for c, v in zip(cand, valid)]
        m = [a and i not in dis for a, i in zip(above, idx)]
        last = pos < STEP or any(v and not a for v, a in zip(valid, above))
        while any(m) and picked < 20:
            f = m.index(True)
            ind = idx[f]
            picked += 1
            picks.append(ind)
            for q in range(1, 6):
                dis.add(min(ind + q, size - 1))
                dis.add(max(ind - q, 0))
            m = [mm and abs(i - ind) > 5 for mm, i in zip(m, idx)]
        if last:
            break
        pos -= STEP
    return picks, dis


def sort_keys_then_ties(keys, idx):
    n = len(keys)
    npow = 1
    while npow < n:
        npow *= 2
    pad = 2**64 - 1
    k = list(keys) + [pad] * (npow - n)
    d = list(idx) + [0x7FFFFFFF] * (npow - n)
    kk = 2
    while kk <= npow:
        m, jj = kk - 1, kk
        while jj > 1:
            nk, nd = k[:], d[:]
            for i in range(npow):
                p = i ^ m
                if (k[p] < k[i]) if p > i else (k[p] > k[i]):
                    nk[i], nd[i] = k[p], d[p]
            k, d = nk, nd
            jj >>= 1
            m = jj >> 1
        kk <<= 1
    assert all(x == pad for x in k[n:]), "pads stay above n"
    out = d[:n]
    for i in range(n):
        kv = k[i]
        if (i > 0 and k[i - 1] == kv) or (i + 1 < n and k[i + 1] == kv):
            s, e = i, i + 1
            while s > 0 and k[s - 1] == kv:
                s -= 1
            while e < n and k[e] == kv:
                e += 1
            out[s + sum(1 for j in range(s, e) if d[j] < d[i])] = d[i]
    return k[:n], out


@pytest.mark.parametrize("seed", range(4))
def test_automaton_steps_match_sequential(seed):
    rng = random.Random(seed)
    for _ in range(400):
        n = rng.randint(20, 500)
        ev = [rng.choice([0, 0, 0, 0, 1, 2, 3, 3]) for _ in range(n)]
        assert automaton_steps(ev, n - 7) == automaton_ref(ev, n - 7)


@pytest.mark.parametrize("seed", range(4))
def test_pick_steps_match_greedy(seed):
    rng = random.Random(100 + seed)
    for _ in range(300):
        size = rng.randint(30, 700)
        n = rng.randint(1, size - 10)
        s0 = 5 + rng.randint(0, max(0, size - 11 - n))
        pts = list(range(s0, s0 + n))
        rng.shuffle(pts)
        keys = sorted(rng.choice([rng.random(), 0.5]) for _ in range(n))   # ties at the threshold too
        dis0 = set(rng.sample(range(size), rng.randint(0, size // 3)))
        thresh = rng.choice([0.1, 0.5, 0.9, 0.99])
        assert pick_steps(keys, pts, dis0, thresh, size) == pick_ref(keys, pts, dis0, thresh, size)


def test_sector_sort_network_with_ties():
    rng = random.Random(7)
    for t in range(150):
        n = rng.randint(1, 150)
        hi = 8 if t % 2 else 2**40   # many equal keys / distinct keys
        keys = [rng.randrange(hi) for _ in range(n)]
        idx = rng.sample(range(4096), n)
        k, d = sort_keys_then_ties(keys, idx)
        ref = sorted(zip(keys, idx))
        assert k == [a for a, _ in ref] and d == [b for _, b in ref]
