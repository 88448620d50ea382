// Correspondence search and residual evaluation for LOAM edge/surf registration on gfx950.
//
// Replaces, per outer iteration of CeresEdgeSurfFeatureRegistration::Solve
// (REG/ceres_edgeSurfFeatureRegistration.hpp:105-125; REG = src/MultiSensorFusionEstimator3D/
// include/Algorithm/PointClouds/registration):
//   pointAssociateToMap (:235-244)  -> knn_kernel (query = float(q * p + t), double math)
//   KdTreeFLANN::nearestKSearch(5) + sqd[4] < 1.0 (FeatureMatch/EdgeFeatureMatch.hpp:38-40,
//       FeatureMatch/surfFeatureMatch.hpp:37-42) -> knn_kernel over a dense 1 m cell grid
//   PCA line / QR plane fits (EdgeFeatureMatch.hpp:44-80, surfFeatureMatch.hpp:46-82) and the
//       first Ceres evaluation of every factor (ceres_factor/*.hpp) -> fit_eval_kernel
//   later Ceres residual evaluations at LM candidates -> lm_eval_kernel
// Memory roofline: HBM/L2 gather of float4 map points; no MFMA (no dense contraction here).
#include <hip/hip_runtime.h>

#include "devmath.h"
#include "lm_control.h"
#include "lmsf_internal.h"

#pragma clang fp contract(off)

namespace lmsf {

namespace {

// Candidate key = (d2 bits + kKeyBias) << 32 | map index, read as an IEEE double: a positive normal
// double (exponent field 1 .. 0x7fe for every float d2, NaN and inf included), and positive doubles
// order exactly as their bit patterns, so v_min_f64 / v_max_f64 rank (d2, index) lexicographically:
// the top-5 insertion is a 5-step min/max network (10 VALU per candidate, no branches).
constexpr uint32_t kKeyBias = 0x00100000u;
constexpr uint64_t kSentinel = (uint64_t)(0x3f800000u + kKeyBias) << 32;  // key of d2 == 1.0f, idx 0
__device__ __forceinline__ double key_as_double(uint64_t k) { return __longlong_as_double((long long)k); }
__device__ __forceinline__ uint64_t key_bits(double k) { return (uint64_t)__double_as_longlong(k); }
__device__ __forceinline__ float key_d2(double k) { return __uint_as_float((uint32_t)(key_bits(k) >> 32) - kKeyBias); }
// Keys are never NaN, so the min / max need none of the quieting (v_max_f64 x, x, x per operand built
// from bits or carried around a loop) that fmin / fmax get in IEEE mode: 18 -> 11 f64 ops per candidate
// of a 6-key insertion (C2 22.35k -> 22.7-22.8k scans/s, C5 2853 -> 2894-2904 pairs/s, r02).
// LMSF_KEY_ASM = 0 (A/B build): fmin / fmax.  LMSF_KEY_PK = 1 (A/B build): (dx, dy) squared as packed
// f32 pairs, 97 -> 79 VALU per 4 candidates but measured slower (C2 22.1-22.7k, C5 2847-2857).
#ifndef LMSF_KEY_ASM
#define LMSF_KEY_ASM 1
#endif
#ifndef LMSF_KEY_PK
#define LMSF_KEY_PK 0
#endif
// LMSF_TAIL_PAIRS: a row's tail of fewer than RU candidates as straight-line code (a pair, then a last one)
// instead of a one-candidate loop (A/B)
#ifndef LMSF_TAIL_PAIRS
#define LMSF_TAIL_PAIRS 1
#endif
constexpr bool kTailPairs = LMSF_TAIL_PAIRS != 0;
__device__ __forceinline__ double key_min(double a, double b) {
#if LMSF_KEY_ASM
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fmin(a, b);
#endif
}
__device__ __forceinline__ double key_max(double a, double b) {
#if LMSF_KEY_ASM
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fmax(a, b);
#endif
}
#ifndef LMSF_KNN_UNROLL
#define LMSF_KNN_UNROLL 4
#endif
constexpr int kKnnUnroll = LMSF_KNN_UNROLL;   // candidate loads in flight per lane (T = 1 path): 4 measured best (r01: 0.485 ms vs 0.522 at 1, 0.572 at 8 -- 87 VGPRs)
#ifndef LMSF_KNN_ROWS_FIRST
#define LMSF_KNN_ROWS_FIRST 1
#endif
constexpr bool kKnnRowsFirst = LMSF_KNN_ROWS_FIRST != 0;
#ifndef LMSF_KNN_LB_SKIP
#define LMSF_KNN_LB_SKIP 1
#endif
constexpr bool kLbSkip = LMSF_KNN_LB_SKIP != 0;   // rows-first walk: nearest rows first, rows beyond the kept keys skipped
// First-pass radius^2 of the pruned team walk as a multiple of the map's lim1 (its 6th key, the slot memo's, lies
// farther out than the one-lane walk's 5th)
#ifndef LMSF_TEAM_R1X
#define LMSF_TEAM_R1X 2
#endif

template <int T>
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl_xor(lo, m, T);
    hi = __shfl_xor(hi, m, T);
    return ((uint64_t)hi << 32) | lo;
}

// World-frame query of a lidar-frame feature: double transform rounded to float
// (pointAssociateToMap, ceres_...:235-244).
__device__ __forceinline__ float3 associate(const Pose& P, float4 p) {
    d3 w = transform(P, mk((double)p.x, (double)p.y, (double)p.z));
    return make_float3((float)w.x, (float)w.y, (float)w.z);
}

}  // namespace

// Block id -> (query block, scan).  With remap, the 8 XCDs (blocks are dealt round-robin: b and
// b + 8 share one) each walk one contiguous eighth of the logical block range, so the queries an
// XCD has in flight are neighbours along the same rings and reuse that XCD's 4 MB L2.  Speed
// only: the mapping is a bijection and results do not depend on placement.
__device__ __forceinline__ void block_coords(int remap, int gx, int& x, int& b) {
    const int L = blockIdx.x, total = gridDim.x;
    int logical = L;
    if (remap) {
        const int q = total >> 3, r = total & 7, xcd = L & 7, k = L >> 3;
        logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
    }
    b = logical / gx;
    x = logical - b * gx;
}

// LMSF_MEMO_AOS: a search position's 7 memo words in one 32-B record ([B][F][8]) instead of 7 planes ([B][7][F]):
// the listed search writes one partial line per query instead of seven, the memo pass reads it in two 16-B loads
#ifndef LMSF_MEMO_AOS
#define LMSF_MEMO_AOS 1
#endif
constexpr bool kMemoAos = LMSF_MEMO_AOS != 0;
__device__ __forceinline__ size_t memo_idx(size_t b, int j, size_t i, size_t F) {
    return kMemoAos ? (b * F + i) * kMemoStride + j : (b * kMemoWords + j) * F + i;
}

// Field-wise select of two grids: a runtime-selected GridView reference (or a select of whole
// structs) makes the compiler spill the kernel arguments to scratch.
__device__ __forceinline__ GridView pick_grid(bool c, const GridView& a, const GridView& b) {
    GridView r;
    r.ox = c ? a.ox : b.ox;
    r.oy = c ? a.oy : b.oy;
    r.oz = c ? a.oz : b.oz;
    r.nx = c ? a.nx : b.nx;
    r.ny = c ? a.ny : b.ny;
    r.nz = c ? a.nz : b.nz;
    r.off = c ? a.off : b.off;
    r.pts = c ? a.pts : b.pts;
    r.orig = c ? a.orig : b.orig;
    r.n = c ? a.n : b.n;
    r.sx = c ? a.sx : b.sx;
    r.lim1 = c ? a.lim1 : b.lim1;
    r.sy = c ? a.sy : b.sy;
    return r;
}

// The 5-NN walk of one query w (T lanes per query; lane = this lane's index in the team): the kept
// keys of this lane in k (ascending), c27 += the untrimmed 27-cell candidate count when count27.
// RU: candidate loads in flight per row step of the one-lane rows-first walk.  NK: keys kept (5, or 6
// for the fused kernel, whose query memo needs the 6th-nearest distance; the pruned walk prunes with
// the NK-th key, so all NK are exact).
// lim (plain walks): the squared search radius with its rounding margin -- kCullLim for the 1 m match
// radius, smaller when a bound on the NK-th neighbour distance is known (memo misses, match_fit_kernel).
template <int T, bool TWO, bool PRUNE, int RU = kKnnUnroll, int NK = 5>
__device__ __forceinline__ void knn_walk(const GridView& g, const GridView& g2, const float3 w, const int lane,
                                         const int count27, double (&k)[NK], unsigned int& c27,
                                         const float lim = 1.0f + 1e-5f) {
    constexpr int NR = TWO ? 18 : 9;
    constexpr uint32_t kGridBit = 0x80000000u;
    const float fx = floorf(w.x), fy = floorf(w.y), fz = floorf(w.z);
    // A (grid, dy, dz) x-row of 3 cells (3 sx slices) is one contiguous range of the sorted points.
    // With rem = kCullLim - gy^2 - gz^2 (gy, gz: the query's gaps to the row's y and z slabs), only
    // points with |x - qx| <= sqrt(rem) can have d2 < 1, so the row is trimmed to the slices
    // meeting [qx - sqrt(rem), qx + sqrt(rem)] (window edges in double from the exact float query;
    // the kCullLim margin dwarfs float rounding of the gaps, of sqrt and of d2).  c27 counts the
    // untrimmed 27 cells (SURVEY 8(d) accounting).
    constexpr float kCullLim = 1.0f + 1e-5f;
    auto resolve_row = [&](int rr, int& rs, int& rl, float& rlb) {
        rs = 0;
        rl = 0;
        rlb = 0.f;
        const GridView gg = pick_grid(TWO && rr >= 9, g2, g);
        const int gn = gg.n, ox = gg.ox, oy = gg.oy, oz = gg.oz, nx = gg.nx, ny = gg.ny, nz = gg.nz, sx = gg.sx;
        const uint32_t* off = gg.off;
        const int r9 = rr % 9, dyo = (r9 % 3) - 1, dzo = (r9 / 3) - 1;
        const float fxs = fx * (float)sx;
        const bool inside = gn > 0 && fxs >= (float)(ox - 2 * sx) && fxs <= (float)(ox + nx + sx) &&
                            fy >= (float)(oy - 2) && fy <= (float)(oy + ny + 1) &&
                            fz >= (float)(oz - 2) && fz <= (float)(oz + nz + 1);
        if (!inside) return;
        const int cxs = (int)fxs - ox, cy = (int)fy - oy + dyo, cz = (int)fz - oz + dzo;
        const int xa = max(cxs - sx, 0), xb = min(cxs + 2 * sx - 1, nx - 1);
        if (cy < 0 || cy >= ny || cz < 0 || cz >= nz || xa > xb) return;
        const uint32_t* row = off + ((size_t)cz * ny + cy) * nx;
        const float ylo = fy + (float)dyo, zlo = fz + (float)dzo;
        const float gy = fmaxf(0.f, fmaxf(ylo - w.y, w.y - (ylo + 1.f)));
        const float gz = fmaxf(0.f, fmaxf(zlo - w.z, w.z - (zlo + 1.f)));
        rlb = gy * gy + gz * gz;
        const float rem = lim - gy * gy - gz * gz;
        if (rem >= 0.f) {
            const double r = (double)sqrtf(rem);
            const int sa = max(xa, (int)floor(((double)w.x - r) * sx) - ox);
            const int sb = min(xb, (int)floor(((double)w.x + r) * sx) - ox);
            if (sa <= sb) {
                const uint32_t s0 = row[sa], s1 = row[sb + 1];
                rs = (int)s0;
                rl = (int)(s1 - s0);
            }
        }
        if (count27) c27 += row[xb + 1] - row[xa];
    };
    auto consider = [&](const float4 m, uint32_t /*tagged_pos*/) {
#if LMSF_KEY_PK
        // (dx, dy) and their squares as packed pairs (v_pk_add_f32 / v_pk_mul_f32): the same
        // roundings as the scalar expression, one instruction for two
        typedef float f2v __attribute__((ext_vector_type(2)));
        const f2v wxy = {w.x, w.y}, mxy = {m.x, m.y};
        const f2v dxy = wxy - mxy;
        const f2v sq = dxy * dxy;
        const float dz = w.z - m.z;
        const float d2 = (sq.x + sq.y) + dz * dz;
#else
        const float dx = w.x - m.x, dy = w.y - m.y, dz = w.z - m.z;
        const float d2 = dx * dx + dy * dy + dz * dz;
#endif
        double x = key_as_double(((uint64_t)(__float_as_uint(d2) + kKeyBias) << 32) | (uint32_t)__float_as_int(m.w));
#pragma unroll
        for (int i = 0; i < NK; ++i) {
            const double lo = key_min(k[i], x);
            x = key_max(k[i], x);
            k[i] = lo;
        }
    };
    // row rr -> its (grid, dy, dz) geometry; false when the row lies outside the grid
    auto row_geo = [&](int rr, const uint32_t*& row, int& xa, int& xb, float& lb, int& ox, int& sx) {
        const GridView gg = pick_grid(TWO && rr >= 9, g2, g);
        ox = gg.ox;
        sx = gg.sx;
        const int r9 = rr % 9, dyo = (r9 % 3) - 1, dzo = (r9 / 3) - 1;
        const float fxs = fx * (float)gg.sx;
        const bool inside = gg.n > 0 && fxs >= (float)(gg.ox - 2 * gg.sx) && fxs <= (float)(gg.ox + gg.nx + gg.sx) &&
                            fy >= (float)(gg.oy - 2) && fy <= (float)(gg.oy + gg.ny + 1) &&
                            fz >= (float)(gg.oz - 2) && fz <= (float)(gg.oz + gg.nz + 1);
        if (!inside) return false;
        const int cxs = (int)fxs - gg.ox, cy = (int)fy - gg.oy + dyo, cz = (int)fz - gg.oz + dzo;
        xa = max(cxs - gg.sx, 0);
        xb = min(cxs + 2 * gg.sx - 1, gg.nx - 1);
        if (cy < 0 || cy >= gg.ny || cz < 0 || cz >= gg.nz || xa > xb) return false;
        row = gg.off + ((size_t)cz * gg.ny + cy) * gg.nx;
        const float ylo = fy + (float)dyo, zlo = fz + (float)dzo;
        const float gy = fmaxf(0.f, fmaxf(ylo - w.y, w.y - (ylo + 1.f)));
        const float gz = fmaxf(0.f, fmaxf(zlo - w.z, w.z - (zlo + 1.f)));
        lb = gy * gy + gz * gz;
        return true;
    };
    // slices of [xa, xb] meeting [w.x - r, w.x + r], r = sqrt(lim - lb) (empty when lim < lb)
    auto window = [&](float lim, float lb, int xa, int xb, int ox, int sx, int& sa, int& sb) {
        const float rem = lim - lb;
        sa = 1;
        sb = 0;
        if (rem < 0.f) return;
        const double r = (double)sqrtf(rem);
        sa = max(xa, (int)floor(((double)w.x - r) * sx) - ox);
        sb = min(xb, (int)floor(((double)w.x + r) * sx) - ox);
    };
    if constexpr (T == 1 && !PRUNE && kKnnRowsFirst) {
        // all rows resolved first (2 x NR offset loads in one batch, one latency instead of NR), then
        // walked with RU candidate loads in flight
        // Rows are walked nearest first (own row, faces, corners) and a row whose yz-gap^2 lower bound
        // exceeds the current NK-th key is skipped: exact, as in the pruned walk below (every point of the
        // row has fl(d2) >= fl(gy^2 + gz^2) > that key, so it cannot enter the kept NK, ties included).
        int rs_[NR], rl_[NR];
        float lb_[NR];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) resolve_row(rr, rs_[rr], rl_[rr], lb_[rr]);
        constexpr int kNear[9] = {4, 1, 3, 5, 7, 0, 2, 6, 8};
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const int rr = kLbSkip ? kNear[TWO ? i / 2 : i] + ((TWO && (i & 1)) ? 9 : 0) : i;
            if (kLbSkip && lb_[rr] > key_d2(k[NK - 1])) continue;
            const float4* rp = (TWO && rr >= 9) ? g2.pts : g.pts;
            const uint32_t tag = (TWO && rr >= 9) ? kGridBit : 0u;
            const int a = rs_[rr], len = rl_[rr];
            int c = 0;
            for (; c + RU <= len; c += RU) {
                float4 m[RU];
#pragma unroll
                for (int u = 0; u < RU; ++u) m[u] = rp[a + c + u];
#pragma unroll
                for (int u = 0; u < RU; ++u) consider(m[u], (uint32_t)(a + c + u) | tag);
            }
            if constexpr (kTailPairs) {   // the row's tail (< RU) straight-line: a pair, then a last one
                if (c + 2 <= len) {
                    const float4 m0 = rp[a + c], m1 = rp[a + c + 1];
                    consider(m0, (uint32_t)(a + c) | tag);
                    consider(m1, (uint32_t)(a + c + 1) | tag);
                    c += 2;
                }
                if (c < len) consider(rp[a + c], (uint32_t)(a + c) | tag);
            } else {
                for (; c < len; ++c) consider(rp[a + c], (uint32_t)(a + c) | tag);
            }
        }
    } else if constexpr (T == 1 && !PRUNE) {
        // one lane walks its rows; kKnnUnroll loads in flight per step (a row is contiguous: 8 points per
        // 128-B line), so the lane waits once per kKnnUnroll candidates instead of once per candidate.
        // Keys are unique (global index), so the kept top-5 does not depend on the visit order.
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
            const float4* rp = (TWO && rr >= 9) ? g2.pts : g.pts;
            const uint32_t tag = (TWO && rr >= 9) ? kGridBit : 0u;
            int a, len;
            float lbr;
            resolve_row(rr, a, len, lbr);
            int c = 0;
            for (; c + kKnnUnroll <= len; c += kKnnUnroll) {
                float4 m[kKnnUnroll];
#pragma unroll
                for (int u = 0; u < kKnnUnroll; ++u) m[u] = rp[a + c + u];
#pragma unroll
                for (int u = 0; u < kKnnUnroll; ++u) consider(m[u], (uint32_t)(a + c + u) | tag);
            }
            for (; c < len; ++c) consider(rp[a + c], (uint32_t)(a + c) | tag);
        }
    } else if constexpr (T == 1) {
        // Dense maps (PRUNE): the walk prunes with the current 5th-best distance d4 (1.0 until five
        // are held), which is ~0.2 m on a 10M-point map:
        //   pass 1: rows nearest first (own row, 4 faces, 4 corners), each trimmed to the x-window of
        //           radius sqrt(lim1) (lim1 from the map's density, GridView::lim1); rows with yz-gap^2
        //           lb > min(d4, lim1) skipped; scanned rows are marked;
        //   pass 2: every row with lb <= d4, trimmed to the x-window of radius sqrt(d4) minus the
        //           slices pass 1 scanned (recomputed from lim1).
        // Skipping a row whose lb exceeds d4 is exact: float rounding is monotone, so every point of
        // the row has fl(d2) >= fl(gy^2 + gz^2) > d4 (it could not enter the top-5, ties included).
        // x-windows carry the 1e-5 relative margin of kCullLim.  Sparse maps (C2: ~6 points per
        // occupied cell) take the plain walk above: there the extra offset loads cost more than the
        // candidates they save (measured).
        auto scan_range = [&](const float4* rp, uint32_t tag, int a, int len) {
            int c = 0;
            for (; c + RU <= len; c += RU) {
                float4 m[RU];
#pragma unroll
                for (int u = 0; u < RU; ++u) m[u] = rp[a + c + u];
#pragma unroll
                for (int u = 0; u < RU; ++u) consider(m[u], (uint32_t)(a + c + u) | tag);
            }
            for (; c < len; ++c) consider(rp[a + c], (uint32_t)(a + c) | tag);
        };
        constexpr int kOrder[9] = {4, 1, 3, 5, 7, 0, 2, 6, 8};   // own row, faces, corners
        auto row_of = [&](int i) { return kOrder[TWO ? i / 2 : i] + ((TWO && (i & 1)) ? 9 : 0); };
        const float lim1 = g.lim1 * kCullLim;   // both grids of a kind share the first-pass radius
        uint32_t scanned = 0;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const int rr = row_of(i);
            const uint32_t* row;
            int xa, xb, ox, sx;
            float lb;
            if (!row_geo(rr, row, xa, xb, lb, ox, sx)) continue;
            if (count27) c27 += row[xb + 1] - row[xa];
            const float d4 = key_d2(k[NK - 1]);
            if (lb > d4 || lb > lim1) continue;
            int sa, sb;
            window(lim1, lb, xa, xb, ox, sx, sa, sb);
            scanned |= 1u << rr;
            if (sa <= sb) {
                const uint32_t s0 = row[sa];
                scan_range((TWO && rr >= 9) ? g2.pts : g.pts, (TWO && rr >= 9) ? kGridBit : 0u, (int)s0,
                           (int)(row[sb + 1] - s0));
            }
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const int rr = row_of(i);
            const float d4 = key_d2(k[NK - 1]);
            const uint32_t* row;
            int xa, xb, ox, sx;
            float lb;
            if (!row_geo(rr, row, xa, xb, lb, ox, sx)) continue;
            if (lb > d4) continue;
            int sa, sb, ta = 1, tb = 0;
            window(d4 * kCullLim, lb, xa, xb, ox, sx, sa, sb);
            if (scanned & (1u << rr)) window(lim1, lb, xa, xb, ox, sx, ta, tb);
            const float4* rp = (TWO && rr >= 9) ? g2.pts : g.pts;
            const uint32_t tag = (TWO && rr >= 9) ? kGridBit : 0u;
            if (ta > tb) {
                if (sa <= sb) {
                    const uint32_t s0 = row[sa];
                    scan_range(rp, tag, (int)s0, (int)(row[sb + 1] - s0));
                }
            } else {
                const int l1 = min(sb, ta - 1), r0 = max(sa, tb + 1);
                if (sa <= l1) {
                    const uint32_t s0 = row[sa];
                    scan_range(rp, tag, (int)s0, (int)(row[l1 + 1] - s0));
                }
                if (r0 <= sb) {
                    const uint32_t s0 = row[r0];
                    scan_range(rp, tag, (int)s0, (int)(row[sb + 1] - s0));
                }
            }
        }
    } else {
        // lane l resolves rows l, l + T, ...; the team shares them by shuffles
        constexpr int REPS = (NR + T - 1) / T;
        // the team strides over the flattened candidates of the rows' ranges [rs_, rs_ + rl_) (entry rep of lane l:
        // row l + rep T)
        auto walk_rows = [&](const int (&rs_)[REPS], const int (&rl_)[REPS]) {
            int st[NR], pre[NR + 1];
            pre[0] = 0;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                st[r] = __shfl(rs_[r / T], r % T, T);
                pre[r + 1] = pre[r] + __shfl(rl_[r / T], r % T, T);
            }
            const int total = pre[NR];
            // current row r: candidates [rpre, rend) map to pts[rbase + (v - rpre)]
            int r = 0, rpre = 0, rend = pre[1], rbase = st[0];
            const float4* rpts = g.pts;
            uint32_t rtag = 0;
            for (int v = lane; v < total; v += T) {
                while (v >= rend) {
                    ++r;
                    rpre = rend;
                    int e = pre[NR], s0 = st[NR - 1];
#pragma unroll
                    for (int j = NR - 1; j >= 1; --j) {   // static-index selects keep pre[]/st[] in registers
                        e = (r + 1 == j) ? pre[j] : e;
                        s0 = (r == j - 1) ? st[j - 1] : s0;
                    }
                    rend = e;
                    rbase = s0;
                    if (TWO && r == 9) {
                        rpts = g2.pts;
                        rtag = kGridBit;
                    }
                }
                const int pos = rbase + (v - rpre);
                consider(rpts[pos], (uint32_t)pos | rtag);
            }
        };
        int rs_[REPS], rl_[REPS];
        if constexpr (!PRUNE) {
#pragma unroll
            for (int rep = 0; rep < REPS; ++rep) {
                rs_[rep] = 0;
                rl_[rep] = 0;
                float lbr;
                if (lane + rep * T < NR) resolve_row(lane + rep * T, rs_[rep], rl_[rep], lbr);
            }
            walk_rows(rs_, rl_);
        } else {
            // Pruned team walk (dense priors, single-scan launches): pass 1 walks every row meeting the first-pass
            // ball (radius^2 r1 = min(lim1, lim)) trimmed to it; the team's NK-th key d4 (its lanes' lists merged)
            // ends the search when it lies within lim1 (no point outside the scanned ball can displace it) or
            // when the ball was the whole search radius; else pass 2 walks the rows with yz-gap^2 <= d4, trimmed
            // to d4 (kCullLim margin) minus the slices pass 1 scanned -- the one-lane pruned walk's rules, with
            // the bound shared by the team once, between the passes.
            const float l1 = fminf(g.lim1 * (float)LMSF_TEAM_R1X, 1.f);   // the team's first-pass radius^2
            const float r1 = fminf(l1 * kCullLim, lim);
#pragma unroll
            for (int rep = 0; rep < REPS; ++rep) {
                rs_[rep] = 0;
                rl_[rep] = 0;
                const int rr = lane + rep * T;
                const uint32_t* row;
                int xa, xb, ox, sx;
                float lb;
                if (rr < NR && row_geo(rr, row, xa, xb, lb, ox, sx)) {
                    if (count27) c27 += row[xb + 1] - row[xa];
                    int sa, sb;
                    if (lb <= r1) {
                        window(r1, lb, xa, xb, ox, sx, sa, sb);
                        if (sa <= sb) {
                            rs_[rep] = (int)row[sa];
                            rl_[rep] = (int)(row[sb + 1] - row[sa]);
                        }
                    }
                }
            }
            walk_rows(rs_, rl_);
            // the team's NK-th key (a copy of the lists merged: NK rounds of team-min, the owner pops)
            double kk[NK];
#pragma unroll
            for (int j = 0; j < NK; ++j) kk[j] = k[j];
            double kth = kk[0];
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                kth = kk[0];
#pragma unroll
                for (int o = T / 2; o >= 1; o >>= 1) kth = key_min(kth, __shfl_xor(kth, o, T));
                if (key_bits(kk[0]) == key_bits(kth)) {
#pragma unroll
                    for (int j = 0; j + 1 < NK; ++j) kk[j] = kk[j + 1];
                    kk[NK - 1] = key_as_double(kSentinel);
                }
            }
            const float d4 = key_d2(kth);
            if (!(d4 <= l1) && !(lim <= l1 * kCullLim)) {
                const float b2 = fminf(d4 * kCullLim, lim);
                int qs_[REPS], ql_[REPS];   // right-hand segments (left-hand ones in rs_ / rl_)
#pragma unroll
                for (int rep = 0; rep < REPS; ++rep) {
                    rs_[rep] = 0;
                    rl_[rep] = 0;
                    qs_[rep] = 0;
                    ql_[rep] = 0;
                    const int rr = lane + rep * T;
                    const uint32_t* row;
                    int xa, xb, ox, sx;
                    float lb;
                    if (rr < NR && row_geo(rr, row, xa, xb, lb, ox, sx) && !(lb > d4)) {
                        int sa, sb, ta = 1, tb = 0;
                        window(b2, lb, xa, xb, ox, sx, sa, sb);
                        if (lb <= r1) window(r1, lb, xa, xb, ox, sx, ta, tb);
                        if (ta > tb) {
                            if (sa <= sb) {
                                rs_[rep] = (int)row[sa];
                                rl_[rep] = (int)(row[sb + 1] - row[sa]);
                            }
                        } else {
                            const int l1 = min(sb, ta - 1), r0 = max(sa, tb + 1);
                            if (sa <= l1) {
                                rs_[rep] = (int)row[sa];
                                rl_[rep] = (int)(row[l1 + 1] - row[sa]);
                            }
                            if (r0 <= sb) {
                                qs_[rep] = (int)row[r0];
                                ql_[rep] = (int)(row[sb + 1] - row[r0]);
                            }
                        }
                    }
                }
                walk_rows(rs_, rl_);
                walk_rows(qs_, ql_);
            }
        }
    }
}

// One team of T lanes per query.  The 27 cells around the query cell are enumerated as 9
// x-rows (each row = 3 consecutive cells = one contiguous range of the cell-sorted points); the
// team strides over the flattened candidate list with coalesced float4 loads, keeps a per-lane
// sorted top-5 of (d2 bits, map index) keys with d2 < 1 (plus each key's position in the sorted
// array), then merges the lanes' lists.  Output: the 5 neighbour points (w = map index).
// TWO: the map of a kind is split into a static grid (a shared prior map, indices [0, P)) and a
// dynamic grid (the keyframe window, indices P + j): 18 rows, positions tagged with the grid bit.
// Keys carry global indices, so the result equals the search of the concatenation [prior | window].
constexpr float kFullLim = 1.0f + 1e-5f;   // knn_walk's squared radius for the 1 m match radius (+ margin)

// Key of map point m (caller-order index idx) for the query w: the expression of knn_walk's consider().
__device__ __forceinline__ double nn_key(const float3 w, const float4 m, uint32_t idx) {
    const float dx = w.x - m.x, dy = w.y - m.y, dz = w.z - m.z;
    const float d2 = dx * dx + dy * dy + dz * dz;
    return key_as_double(((uint64_t)(__float_as_uint(d2) + kKeyBias) << 32) | idx);
}

__device__ __forceinline__ void key_cswap(double& a, double& b) {
    const double lo = key_min(a, b);
    b = key_max(a, b);
    a = lo;
}

// MEMO (single-scan Ceres-LM launches on sparse maps, T > 1): the team keeps the 6th-nearest key and
// leaves the slot's anchor (w, s6 - s5, s6) beside its 5 neighbour points in nnp; in outer iterations
// > 0 (bv.memo) a query that moved d < (s6 - s5) / 2 still has the same 5 nearest, whose keys are
// recomputed from nnp (points + indices) and sorted: when the order is unchanged nnp already holds this
// search's answer and the walk is skipped (fit_eval refits from it); otherwise the walk covers only
// min(1 m, s6 + d) (match_memo_kernel's argument, DESIGN.md "Query memo").
// SPLIT (r06, tracking contexts with a prior map: outer iteration 0 of a Solve in two launches): 1 walks the prior
// grid only (ge / gs) and leaves the team's NK kept keys in bv.pre_keys -- enqueued before the keyframe window's
// rebuild is joined, so it runs beside that rebuild; 2 walks the window grid only (ge2 / gs2), its lane 0 seeded
// with those keys and every row trimmed to the prior's NK-th key (+ 1e-5, the memo bound's margin: every window
// point that can enter the kept NK lies within it), then the usual merge, neighbours and memo anchor.  Keys carry
// global indices, so the result is the one-launch TWO walk's over [prior | window] exactly.
template <int T, bool TWO, bool PRUNE, bool MEMO = false, int SPLIT = 0>
__global__ __launch_bounds__(256) void knn_kernel(GridView ge, GridView gs, GridView ge2, GridView gs2, BatchView bv,
                                                  int skip_converged, int gx, int remap) {
    constexpr int NK = MEMO ? 6 : 5;
    static_assert(SPLIT == 0 || (!TWO && !PRUNE && T > 1), "split walks: plain team walks of one grid each");
    __shared__ unsigned long long blk_n27;
    __shared__ unsigned int blk_q, blk_r;
#ifdef LMSF_STEP_PROFILE   // diagnostics build: block start / walk start / walk end / end stamps of sampled blocks
    __shared__ unsigned long long kt[4];
    if (threadIdx.x == 0) { kt[0] = wall_clock64(); kt[1] = kt[2] = 0; }
#endif
    stamp_if(bv.stamp_start, blockIdx.x == 0);
    int bx, b;
    block_coords(remap, gx, bx, b);
    if (threadIdx.x == 0) { blk_n27 = 0; blk_q = 0; blk_r = 0; }
    __syncthreads();
    const int ne = bv.n_edge[b], ns = bv.n_surf[b];
    const int team = threadIdx.x / T, lane = threadIdx.x % T;
    // ring order when the features came from the extraction kernels (neighbouring lanes search
    // neighbouring ring points, whose 27-cell blocks overlap in L1), else slot order
    int q = bx * (256 / T) + team;
    bool active;
    if (bv.qslot) {
        active = q < bv.n_pos[b];
        q = active ? bv.qslot[(size_t)b * bv.pos_stride + q] : -1;
        active = active && q >= 0;
    } else {
        active = q < ne + ns;
    }
    active = active && !(skip_converged && bv.st[b].gn_converged);
    if (active) {
        const bool is_edge = q < ne;
        const GridView g = pick_grid(is_edge, ge, gs);
        const GridView g2 = pick_grid(is_edge, ge2, gs2);   // SPLIT 2: the walked window, g the prior
        const Pose P = load_pose(bv.st[b].x);
        const size_t slot = (size_t)b * bv.feat_stride + q;
        const float4 p = bv.feat[slot];
        const float3 w = associate(P, p);
        float4* nn_out = bv.nnp + slot * 5;
        bool reuse = false;
        float lim = kFullLim;
        if (MEMO && bv.memo) {   // every lane of the team decides alike (same loads, same arithmetic)
            const float4 pw = bv.prevw[slot];
            if (pw.w >= 0.f) {
                const double dx = (double)w.x - pw.x, dy = (double)w.y - pw.y, dz = (double)w.z - pw.z;
                const double dd = sqrt(dx * dx + dy * dy + dz * dz);
                const double s6 = (double)__int_as_float(bv.memo_nbr[memo_idx(b, 5, q, bv.feat_stride)]);
                const double r6 = s6 + dd + 1e-5;
                if (r6 < 1.0 && bv.memo_bound) lim = fminf(kFullLim, (float)(r6 * r6) + 1e-5f);
                double k5[5];
                float4 m[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    m[j] = nn_out[j];
                    k5[j] = nn_key(w, m[j], (uint32_t)__float_as_int(m[j].w));
                }
                key_cswap(k5[0], k5[1]); key_cswap(k5[3], k5[4]); key_cswap(k5[2], k5[4]);
                key_cswap(k5[2], k5[3]); key_cswap(k5[0], k5[3]); key_cswap(k5[0], k5[2]);
                key_cswap(k5[1], k5[4]); key_cswap(k5[1], k5[3]); key_cswap(k5[1], k5[2]);
                // the stored 5 are still the 5 nearest when the farthest of them is nearer than any
                // other point can have come (those were >= s6 from w0, so >= s6 - d from w)
                bool same = true;
#pragma unroll
                for (int j = 0; j < 5; ++j) same = same && (uint32_t)key_bits(k5[j]) == (uint32_t)__float_as_int(m[j].w);
                reuse = key_bits(k5[4]) < kSentinel &&
                        (bv.memo_exact ? sqrt((double)key_d2(k5[4])) + dd + 1e-5 < s6   // A/B: r01's gap test
                                       : same && 2.0 * dd + 1e-5 < (double)pw.w);
                if (reuse && !same && lane == 0) {   // a new order of the same set: what the walk would write
#pragma unroll
                    for (int j = 0; j < 5; ++j) {
                        float4 o = m[0];
#pragma unroll
                        for (int i = 1; i < 5; ++i)
                            if ((uint32_t)__float_as_int(m[i].w) == (uint32_t)key_bits(k5[j])) o = m[i];
                        nn_out[j] = o;
                    }
                }
            }
        }
        unsigned int c27 = 0;
#ifdef LMSF_STEP_PROFILE
        if (threadIdx.x == 0) kt[1] = wall_clock64();
#endif
        if (!reuse) {
            const double sentinel = key_as_double(kSentinel);
            double k[NK];   // ascending kept keys
#pragma unroll
            for (int j = 0; j < NK; ++j) k[j] = sentinel;
            if constexpr (SPLIT == 2) {   // the prior's kept keys, in lane 0's list
                const double* pk = bv.pre_keys + slot * 6;
                double pre[NK];
#pragma unroll
                for (int j = 0; j < NK; ++j) pre[j] = pk[j];
                lim = fminf(kFullLim, key_d2(pre[NK - 1]) + 1e-5f);
                if (lane == 0) {
#pragma unroll
                    for (int j = 0; j < NK; ++j) k[j] = pre[j];
                }
                knn_walk<T, false, false, kKnnUnroll, NK>(g2, g2, w, lane, 0, k, c27, lim);
            } else if constexpr (SPLIT == 1) {
                knn_walk<T, false, false, kKnnUnroll, NK>(g, g, w, lane, 0, k, c27, lim);
            } else {
                knn_walk<T, TWO, PRUNE, kKnnUnroll, NK>(g, g2, w, lane, bv.count27, k, c27, lim);
            }
#ifdef LMSF_STEP_PROFILE
            if (threadIdx.x == 0) kt[2] = wall_clock64();
#endif
            // merge: NK rounds of team-min; the owning lane pops its head (keys are unique)
            double res[NK];
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                double mn = k[0];
#pragma unroll
                for (int o = T / 2; o >= 1; o >>= 1) mn = key_min(mn, __shfl_xor(mn, o, T));
                res[i] = mn;
                if (key_bits(k[0]) == key_bits(mn)) {
#pragma unroll
                    for (int j = 0; j + 1 < NK; ++j) k[j] = k[j + 1];
                    k[NK - 1] = sentinel;
                }
            }
            if constexpr (SPLIT == 1) {   // the prior pass leaves its keys; the window pass writes the results
#pragma unroll
                for (int i = 0; i < NK; ++i)
                    if (i % T == lane) bv.pre_keys[slot * 6 + i] = res[i];
            }
            // every rank written (lane i % T writes rank i; teams smaller than 5 write several): the
            // neighbour point (from the caller-order copy, w = its map index), so the fit reads 80
            // contiguous bytes.  Indices below g.n belong to g, the rest to g2 (its points carry P + j).
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                if (SPLIT != 1 && i % T == lane) {
                    float4 o = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
                    const uint64_t kb = key_bits(res[i]);
                    if (kb < kSentinel) {
                        const uint32_t idx = (uint32_t)kb;
                        const bool second = (TWO || SPLIT == 2) && idx >= (uint32_t)g.n;
                        const float4 m = second ? g2.orig[idx - (uint32_t)g.n] : g.orig[idx];
                        o = make_float4(m.x, m.y, m.z, __int_as_float((int)idx));
                    }
                    nn_out[i] = o;
                }
            }
            if (MEMO && SPLIT != 1 && lane == 0) {   // the anchor of this full search
                float gap = -1.f;
                if (key_bits(res[4]) < kSentinel) {
                    const double s6 = sqrt((double)fminf(key_d2(res[NK - 1]), 1.0f));
                    gap = (float)(s6 - sqrt((double)key_d2(res[4])));
                    bv.memo_nbr[memo_idx(b, 5, q, bv.feat_stride)] = __float_as_int((float)s6);
                }
                bv.prevw[slot] = make_float4(w.x, w.y, w.z, gap);
            }
        }
        if (bv.n27) {
            if (c27) atomicAdd(&blk_n27, (unsigned long long)c27);
            if (lane == 0) atomicAdd(&blk_q, 1u);
            if (lane == 0 && reuse) atomicAdd(&blk_r, 1u);
        }
    }
    __syncthreads();
#ifdef LMSF_STEP_PROFILE
    if (threadIdx.x == 0 && (blockIdx.x % 97) == 0)
        printf("knnblk %d %llu %llu %llu %llu\n", blockIdx.x, kt[0], kt[1], kt[2], (unsigned long long)wall_clock64());
#endif
    if (threadIdx.x == 0 && bv.n27 && blk_q) {
        // 64 counter shards on separate 128-B lines: one word serialises ~1e5 block updates
        unsigned long long* shard = bv.n27 + (size_t)(blockIdx.x & (kCounterShards - 1)) * 16;
        atomicAdd(shard, blk_n27);
        atomicAdd(shard + 1, (unsigned long long)blk_q);
        if (blk_r) atomicAdd(shard + 2, (unsigned long long)blk_r);
    }
}

// ---------------------------------------------------------------- fits (double precision)

// EdgeFeatureMatch::Match body after the 5-NN (EdgeFeatureMatch.hpp:44-80).
__device__ bool edge_fit(const float4* np, d3& a, d3& b) {
    d3 pts[5];
    d3 center = mk(0, 0, 0);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float4 p = np[j];
        pts[j] = mk((double)p.x, (double)p.y, (double)p.z);
        center = center + pts[j];
    }
    center = mk(center.x / 5.0, center.y / 5.0, center.z / 5.0);
    double cov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        d3 e = pts[j] - center;
        const double ev[3] = {e.x, e.y, e.z};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) cov[r * 3 + c] = cov[r * 3 + c] + ev[r] * ev[c];
    }
    double d[3], v[9];
    saes3(cov, d, v);   // Eigen::SelfAdjointEigenSolver<Matrix3d> (EdgeFeatureMatch.hpp:63)
    if (!(d[2] > 3 * d[1])) return false;
    const d3 u = mk(v[2], v[5], v[8]);   // eigenvectors().col(2)
    a = smul(0.1, u) + center;
    b = smul(-0.1, u) + center;
    return true;
}

// SurfFeatureMatch::Match body after the 5-NN (surfFeatureMatch.hpp:46-82).
__device__ bool surf_fit(const float4* p, float3 q, d3& n_out, double& D_out, double& gn_res) {
    double A[15], bb[5], x[3];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        A[j * 3 + 0] = p[j].x; A[j * 3 + 1] = p[j].y; A[j * 3 + 2] = p[j].z;
        bb[j] = -1.0;
    }
    colpiv_qr_solve<5, 3>(A, bb, x);
    d3 n = mk(x[0], x[1], x[2]);
    double nn_ = norm(n);
    double D = 1 / nn_;
    double z = sqnorm(n);
    if (z > 0.0) {
        double s = sqrt(z);
        n = mk(n.x / s, n.y / s, n.z / s);
    }
#pragma unroll
    for (int j = 0; j < 5; ++j)
        if (fabs(n.x * (double)p[j].x + n.y * (double)p[j].y + n.z * (double)p[j].z + D) > 0.2) return false;
    const d3 cp = mk((double)q.x, (double)q.y, (double)q.z);
    const float distance = (float)(dot(n, cp) + D);
    gn_res = fabs((double)distance);
    if (distance >= 0) { n_out = n; D_out = D; } else { n_out = mk(-n.x, -n.y, -n.z); D_out = -D; }
    return true;
}

// Block reduction of a kPacket-double packet: wave butterfly, then 4 wave sums in LDS.
// Fixed order -> deterministic.
// The wave step is a transposing butterfly: at distance 32 a lane keeps half of the entries (the
// lower half in lanes 0-31, the upper in 32-63) and adds its partner's copy of them, at 16 half of
// the rest, ... down to distance 2, then one plain step at distance 1: 16 + 8 + 4 + 2 + 1 + 1 = 32
// double shuffles instead of 32 x 6.  Lanes 2e and 2e + 1 end with entry e = (lane >> 1).
template <int H>
__device__ __forceinline__ void butterfly_step(double* P, int lane) {
    const bool upper = (lane & (2 * H)) != 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const double send = upper ? P[i] : P[H + i];
        const double keep = upper ? P[H + i] : P[i];
        P[i] = keep + __shfl_xor(send, 2 * H, 64);
    }
}

__device__ __forceinline__ void block_reduce_packet(double* P, double* out) {
    static_assert(kPacket == 32, "butterfly over 32 entries");
    __shared__ double red[4][kPacket];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    butterfly_step<16>(P, lane);
    butterfly_step<8>(P, lane);
    butterfly_step<4>(P, lane);
    butterfly_step<2>(P, lane);
    butterfly_step<1>(P, lane);
    const double v = P[0] + __shfl_xor(P[0], 1, 64);
    if ((lane & 1) == 0) red[wave][lane >> 1] = v;
    __syncthreads();
    if (threadIdx.x < kPacket) {
        const int i = threadIdx.x;
        out[i] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
    }
}

// Split record store / load (BatchView: rec_p, rec_v, rec_e).
// LMSF_REC44 (default): the record's point is packed to 12 B in rec_p's memory (rec_p then holds
// float3s) and the kind is the position's -- edges come before surfs both in slot order and in the fused path's
// search order -- with a NaN of a payload arithmetic never produces (kRecNone) in v[3] marking an unmatched record (a
// degenerate fit's own NaN stays a matched record, as the oracle evaluates it): an LM
// evaluation then reads 44 B per surf record and 60 B per edge record instead of 48 / 64.  0 (A/B builds): the
// float4 point with the kind in w, whose unmatched records' value arrays are never read.
#ifndef LMSF_REC44
#define LMSF_REC44 1
#endif
struct RecQ { float x, y, z; };
bool rec44_layout() { return LMSF_REC44 != 0; }
__device__ __forceinline__ void store_record(const BatchView& bv, size_t slot, float4 p, int kind, const d3& v0, double v1x,
                                             double v1y, double v1z) {
    if (LMSF_REC44) reinterpret_cast<RecQ*>(bv.rec_p)[slot] = RecQ{p.x, p.y, p.z};
    else bv.rec_p[slot] = make_float4(p.x, p.y, p.z, __int_as_float(kind));
    if (kind != 0) {
        RecV v;
        v.v[0] = v0.x; v.v[1] = v0.y; v.v[2] = v0.z; v.v[3] = v1x;
        bv.rec_v[slot] = v;
        if (kind == LMSF_EDGE) bv.rec_e[slot] = make_double2(v1y, v1z);
    } else if (LMSF_REC44) {
        bv.rec_v[slot].v[3] = __longlong_as_double(kRecNone);
    }
}

// The record at slot (its position `local` in the slot's order, ne edges first): the point with the kind in w,
// and the values in v (unspecified when the kind is 0).  Both loads are issued before either is used.
__device__ __forceinline__ float4 load_record(const BatchView& bv, size_t slot, int local, int ne, RecV& v) {
    v = bv.rec_v[slot];
    if (LMSF_REC44) {
        const RecQ q = reinterpret_cast<const RecQ*>(bv.rec_p)[slot];
        const int kind = __double_as_longlong(v.v[3]) == kRecNone ? 0 : local < ne ? LMSF_EDGE : LMSF_SURF;
        return make_float4(q.x, q.y, q.z, __int_as_float(kind));
    }
    return bv.rec_p[slot];
}

// Residual + Jacobian of one stored record at pose Ps (edge_factor.hpp:33-61, surf_factor.hpp:32-56);
// false when the slot holds no correspondence.
__device__ __forceinline__ bool record_residual(const BatchView& bv, size_t slot, int local, int ne, const Pose& Ps,
                                                double& res, double* J) {
    RecV v;
    const float4 p = load_record(bv, slot, local, ne, v);
    const int kind = __float_as_int(p.w);
    if (kind == 0) return false;
    const d3 pp = mk((double)p.x, (double)p.y, (double)p.z);
    if (kind == LMSF_EDGE) {
        const double2 e = bv.rec_e[slot];
        res = edge_residual(Ps, pp, mk(v.v[0], v.v[1], v.v[2]), mk(v.v[3], e.x, e.y), J);
    } else {
        res = surf_residual(Ps, pp, mk(v.v[0], v.v[1], v.v[2]), v.v[3], J);
    }
    return true;
}

// Line / plane fit of one query from its 5 neighbours, record write, and its Huber-weighted
// normal-equation contribution at the linearisation pose (Ceres' first evaluation).
// np: the 5 neighbour points (w = map index bits, np[4].w < 0: fewer than 5 within the radius); w: the
// query in the map frame (associate(Ps, p)).
__device__ __forceinline__ void fit_query(const BatchView& bv, int solver, size_t slot, bool is_edge, const float4 p,
                                          const float3 w, const float4* np, const Pose& Ps, double* P) {
    {
        int kind = 0;
        d3 v0 = mk(0, 0, 0);
        double v1x = 0.0, v1y = 0.0, v1z = 0.0;
        double gn_grad[3] = {0, 0, 0}, gn_res = 0.0;
        if (__float_as_int(np[4].w) >= 0) {
            if (is_edge) {
                d3 a, bpt;
                if (edge_fit(np, a, bpt)) {
                    kind = LMSF_EDGE;
                    v0 = a;
                    v1x = bpt.x; v1y = bpt.y; v1z = bpt.z;
                    if (solver == LMSF_SOLVER_GN) {  // EdgeCostFactorInfo residuals_ / norm_
                        const d3 cp = mk((double)w.x, (double)w.y, (double)w.z);
                        d3 nu = cross(cp - a, cp - bpt);
                        d3 de = a - bpt;
                        gn_res = norm(nu) / norm(de);
                        d3 gg = cross(de, nu);
                        double gnn = norm(gg);
                        gn_grad[0] = gnn > 0 ? gg.x / gnn : gg.x;
                        gn_grad[1] = gnn > 0 ? gg.y / gnn : gg.y;
                        gn_grad[2] = gnn > 0 ? gg.z / gnn : gg.z;
                    }
                }
            } else {
                d3 n;
                double D;
                if (surf_fit(np, w, n, D, gn_res)) {
                    kind = LMSF_SURF;
                    v0 = n;
                    v1x = D;
                    gn_grad[0] = n.x; gn_grad[1] = n.y; gn_grad[2] = n.z;
                }
            }
        }
        store_record(bv, slot, p, kind, v0, v1x, v1y, v1z);
        if (solver == LMSF_SOLVER_GN) {
            double* gr = bv.gn_rows + slot * 4;
            gr[0] = gn_grad[0]; gr[1] = gn_grad[1]; gr[2] = gn_grad[2]; gr[3] = kind ? gn_res : -1.0;
        } else if (kind != 0) {
            double J[6], res;
            const d3 pp = mk((double)p.x, (double)p.y, (double)p.z);
            if (kind == LMSF_EDGE)
                res = edge_residual(Ps, pp, v0, mk(v1x, v1y, v1z), J);
            else
                res = surf_residual(Ps, pp, v0, v1x, J);
            huber_accumulate(P, res, J);
        }
        // branch-free: a predicated `P[kind ? 29 : 30] += 1` becomes a select of two addresses (scratch)
        P[29] += kind == LMSF_EDGE ? 1.0 : 0.0;
        P[30] += kind == LMSF_SURF ? 1.0 : 0.0;
    }
}

__device__ __forceinline__ void fit_one(const BatchView& bv, int solver, int b, int q, int ne, const Pose& Ps,
                                        double* P) {
    const size_t slot = (size_t)b * bv.feat_stride + q;
    const float4 p = bv.feat[slot];
    // the 5 neighbour points, written contiguously by knn
    float4 np[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) np[j] = bv.nnp[slot * 5 + j];
    fit_query(bv, solver, slot, q < ne, p, associate(Ps, p), np, Ps, P);
}

// FPT queries per thread (block = 256 * FPT queries): one packet reduction per block.
template <int FPT>
__global__ __launch_bounds__(256) void fit_eval_kernel(BatchView bv, int solver) {
    stamp_if(bv.stamp_end, blockIdx.x == 0 && blockIdx.y == 0);
    const int b = blockIdx.y;
    const int ne = bv.n_edge[b], ns = bv.n_surf[b];
    const int nq = ne + ns;
    if (blockIdx.x * 256 * FPT >= nq) return;
    if (solver == LMSF_SOLVER_GN && bv.st[b].gn_converged) return;
    const Pose Ps = load_pose(bv.st[b].x);
    double P[kPacket];
#pragma unroll
    for (int i = 0; i < kPacket; ++i) P[i] = 0.0;
#pragma unroll
    for (int k = 0; k < FPT; ++k) {
        const int q = blockIdx.x * 256 * FPT + k * 256 + threadIdx.x;
        if (q < nq) fit_one(bv, solver, b, q, ne, Ps, P);
    }
    block_reduce_packet(P, bv.partials + ((size_t)b * bv.max_parts + blockIdx.x) * kPacket);
}

// Write-through / L2-bypassing accesses for packets other blocks read inside the same launch (per-XCD L2s are not
// coherent, MI355X_MICROARCH.md): agent-scope atomic stores and loads.
__device__ __forceinline__ void coherent_store_f64(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double coherent_load_f64(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<double*>(p)),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// ---------------------------------------------------------------- single-scan search + fit (tracking, Ceres-LM)
// Single-scan launches (C3 / C4 tracking: one ~63k-query scan) run the 8-lane search, the line / plane fit, the
// record write and the first evaluation in ONE launch (r04: knn_kernel<8> then fit_eval_kernel<1>, the 5
// neighbours handed over through nnp, knn lane utilisation 0.50: the teams of memo-reused queries idled beside
// the walking ones).  A block of 8 waves takes 64 consecutive search positions (featp order: edges then surfs,
// each in ring order; slot order for host features):
//   1. wave 0, one lane per position: its query and the slot memo test (knn_kernel<., MEMO>'s rule); the
//      positions that must walk are listed in LDS by ballot compaction;
//   2. the block's 64 8-lane teams take the listed positions in order (a wave with no entry goes straight to the
//      barrier), walk (knn_walk<8>, 6 keys), merge, and leave the 5 neighbours in LDS and nnp and the anchor;
//   3. waves 1-7 exit (their SIMD slots go to other blocks' walks); wave 0 fits its 64 positions -- neighbours
//      from registers (memo reuse) or LDS (walked) -- writes the records and its packet at the linearisation pose
//      (write-through); the last block of each group of 4 (agent-scope ticket) sums the group's packets in block
//      order into the group packet, so lm_begin / lm_loop read one packet per 256 positions (fit_eval_kernel<1>'s
//      count) and the sums do not depend on which block came last.
// Records and the memo state stay by slot (the single-scan layout lmsf_match / capture read).
#ifndef LMSF_TRACK_FUSED
#define LMSF_TRACK_FUSED 0
#endif
constexpr int kTrackPos = 64;     // search positions per block (one 8-lane team each)
constexpr int kTrackGroup = 4;    // blocks per packet: 256 positions
__host__ __device__ size_t track_ticket_words(size_t feat_stride) { return (feat_stride + kTrackPos * kTrackGroup - 1) / (kTrackPos * kTrackGroup); }

template <bool TWO>
__global__ __launch_bounds__(512) void track_match_kernel(GridView ge, GridView gs, GridView ge2, GridView gs2,
                                                          BatchView bv, unsigned* ticket) {
    constexpr int T = 8, NK = 6;
    __shared__ float4 s_nb[kTrackPos][5];
    __shared__ float4 s_q[kTrackPos];     // listed entries: query (xyz), search radius^2 (w)
    __shared__ int s_pos[kTrackPos];      // listed entries: block lane | is_edge << 8
    __shared__ int s_slot[kTrackPos];     // listed entries: the feature slot
    __shared__ int s_nwalk;
    __shared__ unsigned long long s_n27;
    stamp_if(bv.stamp_start, blockIdx.x == 0 && blockIdx.y == 0);
    const int b = blockIdx.y;
    const int ne = bv.n_edge[b], nq = ne + bv.n_surf[b];
    const int pos0 = blockIdx.x * kTrackPos;
    if (pos0 >= nq) return;   // block-uniform
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t F = bv.feat_stride;
    const Pose P = load_pose(bv.st[b].x);
    // ---- 1. wave 0: the queries, the memo test, the walk list
    bool valid = false, is_edge = false, reuse = false;
    int q = 0;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    float3 w = make_float3(0.f, 0.f, 0.f);
    float4 mo[5];   // a reused position's 5 neighbours in this search's order
    if (wave == 0) {
        const int i = pos0 + lane;
        valid = i < nq;
        if (valid) {
            if (bv.fslot) {
                p = bv.featp[(size_t)b * F + i];
                q = __float_as_int(p.w);
            } else {
                q = i;
                p = bv.feat[(size_t)b * F + i];
            }
            is_edge = q < ne;
            w = associate(P, p);
        }
        const size_t slot = (size_t)b * F + q;
        float lim = kFullLim;
        if (valid && bv.memo) {
            const float4 pw = bv.prevw[slot];
            if (pw.w >= 0.f) {
                const double dx = (double)w.x - pw.x, dy = (double)w.y - pw.y, dz = (double)w.z - pw.z;
                const double dd = sqrt(dx * dx + dy * dy + dz * dz);
                const double s6 = (double)__int_as_float(bv.memo_nbr[memo_idx(b, 5, q, F)]);
                const double r6 = s6 + dd + 1e-5;
                if (r6 < 1.0 && bv.memo_bound) lim = fminf(kFullLim, (float)(r6 * r6) + 1e-5f);
                const float4* nn_in = bv.nnp + slot * 5;
                double k5[5];
                float4 m[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    m[j] = nn_in[j];
                    k5[j] = nn_key(w, m[j], (uint32_t)__float_as_int(m[j].w));
                }
                key_cswap(k5[0], k5[1]); key_cswap(k5[3], k5[4]); key_cswap(k5[2], k5[4]);
                key_cswap(k5[2], k5[3]); key_cswap(k5[0], k5[3]); key_cswap(k5[0], k5[2]);
                key_cswap(k5[1], k5[4]); key_cswap(k5[1], k5[3]); key_cswap(k5[1], k5[2]);
                bool same = true;
#pragma unroll
                for (int j = 0; j < 5; ++j) same = same && (uint32_t)key_bits(k5[j]) == (uint32_t)__float_as_int(m[j].w);
                reuse = key_bits(k5[4]) < kSentinel &&
                        (bv.memo_exact ? sqrt((double)key_d2(k5[4])) + dd + 1e-5 < s6
                                       : same && 2.0 * dd + 1e-5 < (double)pw.w);
#pragma unroll
                for (int j = 0; j < 5; ++j) {   // the set in key order: what the walk would return
                    float4 o = m[0];
#pragma unroll
                    for (int t = 1; t < 5; ++t)
                        if ((uint32_t)__float_as_int(m[t].w) == (uint32_t)key_bits(k5[j])) o = m[t];
                    mo[j] = o;
                }
                if (reuse && !same) {
                    float4* nn_out = bv.nnp + slot * 5;
#pragma unroll
                    for (int j = 0; j < 5; ++j) nn_out[j] = mo[j];
                }
            }
        }
        const bool walk = valid && !reuse;
        const unsigned long long todo = __ballot(walk);
        const int rank = __popcll(todo & ((1ull << lane) - 1ull));
        if (walk) {
            s_q[rank] = make_float4(w.x, w.y, w.z, lim);
            s_pos[rank] = lane | (is_edge ? 256 : 0);
            s_slot[rank] = q;
        }
        if (lane == 0) {
            s_nwalk = __popcll(todo);
            s_n27 = 0ull;
        }
        if (bv.n27) {
            const unsigned long long vm = __ballot(valid), rm = __ballot(reuse);
            if (lane == 0) {
                unsigned long long* shard = bv.n27 + (size_t)((blockIdx.x + blockIdx.y) & (kCounterShards - 1)) * 16;
                atomicAdd(shard + 1, (unsigned long long)__popcll(vm));
                if (rm) atomicAdd(shard + 2, (unsigned long long)__popcll(rm));
            }
        }
    }
    __syncthreads();
    // ---- 2. the listed positions, one 8-lane team each
    const int nwalk = s_nwalk;
    if (wave * (64 / T) < nwalk) {   // wave-uniform: the wave's first team has an entry
        const int team = threadIdx.x / T, tl = threadIdx.x % T;
        if (team < nwalk) {          // team-uniform
            const float4 qe = s_q[team];
            const int pe = s_pos[team];
            const bool edge_q = (pe & 256) != 0;
            const GridView g = pick_grid(edge_q, ge, gs);
            const GridView g2 = pick_grid(edge_q, ge2, gs2);
            const double sentinel = key_as_double(kSentinel);
            double k[NK];
#pragma unroll
            for (int j = 0; j < NK; ++j) k[j] = sentinel;
            unsigned int c27 = 0;
            knn_walk<T, TWO, false, kKnnUnroll, NK>(g, g2, make_float3(qe.x, qe.y, qe.z), tl, bv.count27, k, c27, qe.w);
            double res[NK];
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                double mn = k[0];
#pragma unroll
                for (int o = T / 2; o >= 1; o >>= 1) mn = key_min(mn, __shfl_xor(mn, o, T));
                res[i] = mn;
                if (key_bits(k[0]) == key_bits(mn)) {
#pragma unroll
                    for (int j = 0; j + 1 < NK; ++j) k[j] = k[j + 1];
                    k[NK - 1] = sentinel;
                }
            }
            const int pl = pe & 255;
            const int qs = s_slot[team];
            const size_t slot = (size_t)b * F + qs;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                if (i == tl) {
                    float4 o = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
                    const uint64_t kb = key_bits(res[i]);
                    if (kb < kSentinel) {
                        const uint32_t idx = (uint32_t)kb;
                        const bool second = TWO && idx >= (uint32_t)g.n;
                        const float4 m = second ? g2.orig[idx - (uint32_t)g.n] : g.orig[idx];
                        o = make_float4(m.x, m.y, m.z, __int_as_float((int)idx));
                    }
                    bv.nnp[slot * 5 + i] = o;
                    s_nb[pl][i] = o;
                }
            }
            if (tl == 0) {   // the anchor of this full search
                float gap = -1.f;
                if (key_bits(res[4]) < kSentinel) {
                    const double s6 = sqrt((double)fminf(key_d2(res[NK - 1]), 1.0f));
                    gap = (float)(s6 - sqrt((double)key_d2(res[4])));
                    bv.memo_nbr[memo_idx(b, 5, qs, F)] = __float_as_int((float)s6);
                }
                bv.prevw[slot] = make_float4(qe.x, qe.y, qe.z, gap);
            }
            if (bv.count27 && c27) atomicAdd(&s_n27, (unsigned long long)c27);
        }
    }
    __syncthreads();
    if (wave != 0) return;
    if (bv.n27 && lane == 0 && s_n27)
        atomicAdd(bv.n27 + (size_t)((blockIdx.x + blockIdx.y) & (kCounterShards - 1)) * 16, s_n27);
    // ---- 3. wave 0: the fits, the records, the packet
    double Pk[kPacket];
#pragma unroll
    for (int i = 0; i < kPacket; ++i) Pk[i] = 0.0;
    if (valid) {
        if (!reuse)
#pragma unroll
            for (int j = 0; j < 5; ++j) mo[j] = s_nb[lane][j];
        fit_query(bv, LMSF_SOLVER_CERES_LM, (size_t)b * F + q, is_edge, p, w, mo, P, Pk);
    }
    // the block's packet (wave butterfly: entry e in lane 2e), stored write-through above the group packets
    butterfly_step<16>(Pk, lane);
    butterfly_step<8>(Pk, lane);
    butterfly_step<4>(Pk, lane);
    butterfly_step<2>(Pk, lane);
    butterfly_step<1>(Pk, lane);
    const double v = Pk[0] + __shfl_xor(Pk[0], 1, 64);
    double* blk = bv.partials + ((size_t)b * bv.max_parts + bv.max_parts / 2) * kPacket;   // [ceil(F / 64)] packets
    if ((lane & 1) == 0) coherent_store_f64(blk + (size_t)blockIdx.x * kPacket + (lane >> 1), v);
    __builtin_amdgcn_s_waitcnt(0);   // this wave's packet stores are complete before its ticket
    const int grp = blockIdx.x / kTrackGroup;
    const int nblk = (nq + kTrackPos - 1) / kTrackPos;
    const int members = min(kTrackGroup, nblk - grp * kTrackGroup);
    unsigned* tk = ticket + (size_t)b * track_ticket_words(F) + grp;
    unsigned mine = 0;
    // acq_rel ticket: this block's packet stores are released before its arrival, and the last
    // arrival acquires every earlier member's packet before it sums them
    if (lane == 0) mine = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    mine = __shfl(mine, 0, 64);
    if ((int)mine + 1 != members) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the whole wave, not only lane 0, reads after the acquire
    // the group's last block: its packets summed in block order into the group packet, the ticket re-armed
    if (lane < kPacket) {
        double t = 0.0;
        for (int j = 0; j < members; ++j)
            t += coherent_load_f64(blk + (size_t)(grp * kTrackGroup + j) * kPacket + lane);
        bv.partials[((size_t)b * bv.max_parts + grp) * kPacket + lane] = t;
    }
    if (lane == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

bool track_fused_enabled() {
    static const bool v = ab_int("LMSF_TRACK_FUSED", LMSF_TRACK_FUSED) != 0;
    return v;
}

hipError_t launch_track_match(const GridView& edge, const GridView& surf, const GridView& edge2, const GridView& surf2,
                              const BatchView& bv, unsigned* ticket, hipStream_t s) {
    const dim3 grid((bv.feat_stride + kTrackPos - 1) / kTrackPos, bv.B);
    if (edge2.n > 0 || surf2.n > 0)
        hipLaunchKernelGGL(track_match_kernel<true>, grid, dim3(512), 0, s, edge, surf, edge2, surf2, bv, ticket);
    else
        hipLaunchKernelGGL(track_match_kernel<false>, grid, dim3(512), 0, s, edge, surf, edge2, surf2, bv, ticket);
    return hipGetLastError();
}

// Fused search + fit for batch launches (one lane per query, Ceres-LM solver): the 5-NN walk of
// knn_kernel<1, false, PRUNE>, then fit_query (line / plane fit, record write, Huber-weighted packet
// at the linearisation pose) on the neighbours held in registers -- knn_kernel + fit_eval_kernel
// hand the 5 neighbour points (80 B per query) through memory instead.  Queries run in fslot order:
// edge slots then surf slots, each in ring order, so neighbouring lanes search neighbouring ring
// points and a wave runs one fit kind.  Block x reduces fslot entries [256 x, 256 x + 256): the
// partial count of fit_eval_kernel<1>, so lm_begin reads the same number of packets.
// Wave-level packet reduction (the transposing butterfly of block_reduce_packet without the LDS
// step): entry e lands in lane 2e; out[e] written by that lane.
__device__ __forceinline__ void wave_reduce_packet(double* P, double* out) {
    const int lane = threadIdx.x & 63;
    butterfly_step<16>(P, lane);
    butterfly_step<8>(P, lane);
    butterfly_step<4>(P, lane);
    butterfly_step<2>(P, lane);
    butterfly_step<1>(P, lane);
    const double v = P[0] + __shfl_xor(P[0], 1, 64);
    if ((lane & 1) == 0) out[lane >> 1] = v;
}

// The slot's record values (kind, v0 = a | n, v1 = b | (D, -, -)) -> its residual and Huber-weighted
// packet at the linearisation pose, plus the match counts (fit_query's LM tail).
__device__ __forceinline__ void record_packet(int kind, const float4 p, const d3& v0, double v1x, double v1y, double v1z,
                                              const Pose& Ps, double* P) {
    if (kind != 0) {
        double J[6], res;
        const d3 pp = mk((double)p.x, (double)p.y, (double)p.z);
        if (kind == LMSF_EDGE)
            res = edge_residual(Ps, pp, v0, mk(v1x, v1y, v1z), J);
        else
            res = surf_residual(Ps, pp, v0, v1x, J);
        huber_accumulate(P, res, J);
    }
    P[29] += kind == LMSF_EDGE ? 1.0 : 0.0;
    P[30] += kind == LMSF_SURF ? 1.0 : 0.0;
}

// LMSF_LIN_EVAL (default 1): the batch path's packets at the linearisation pose come from one evaluation
// pass over all records after the matching (lm_eval_kernel<true>, counts included), so the memo pass and the
// search kernel only write records -- no residual / Jacobian / Huber packet or wave reduction in them.  0 (A/B
// builds): the memo pass and the search kernel accumulate the packets themselves, one per wave.
#ifndef LMSF_LIN_EVAL
#define LMSF_LIN_EVAL 1
#endif
constexpr bool kLinEval = LMSF_LIN_EVAL != 0;

// Entries of one memo block's work list per scan: wcount stride.
__host__ __device__ __forceinline__ size_t memo_blocks(size_t feat_stride) { return feat_stride / 256 + 1; }
// LMSF_LIST_ATOMIC: the memo pass lists a scan's searches / refits by wave atomics into one list per scan (needs the
// linearisation pass: the search kernel then forms no packets, so entry order is free); 0: per-block segments in
// position order, found by the search kernel through a prefix scan of the block counts (r02-r03).
#ifndef LMSF_LIST_ATOMIC
#define LMSF_LIST_ATOMIC 1
#endif
constexpr bool kListAtomic = kLinEval && LMSF_LIST_ATOMIC != 0;

#ifndef LMSF_MEMO_WAVES   // waves per SIMD the memo pass is compiled for (A/B)
#define LMSF_MEMO_WAVES 5
#endif
// Query memo pass (outer iterations > 0 of a batch solve, sparse maps): one lane per search position
// i (fslot order).  Position i's last full search left its anchor w0, gap = s6 - s5 and the 5
// neighbour indices.  Every map point's distance to the query changes by at most d = |w - w0|, and
// float d2 / sqrt are within 1e-6 m of exact below 1 m, so with 2 d + 1e-5 < gap the 5 nearest points
// (all within the 1 m radius, the 6th capped there) are still the same 5: a new search returns these
// 5 keys recomputed at w, in key order.  They are recomputed (the consider() expression) and sorted;
// when the order equals the stored one, the new search's result is the stored one and so is the fit
// (line / plane fits depend only on the ordered neighbours; the plane's orientation, which follows the
// sign of n . w + D, is re-tested): only the residual, Jacobian and Huber-weighted packet at the
// linearisation pose are new.  Otherwise the position goes to this block's work list for
// match_fit_kernel<., true>, with a search radius: the 6 nearest points at w0 lie within s6 + d of w,
// so the new 6 nearest do too, and a walk over the rows / x-slices within min(1 m, s6 + d) (+ margin)
// returns the same 6 keys as the full 1 m walk.  One packet per wave at partial index 4 bx + wave.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LMSF_MEMO_WAVES))) void match_memo_kernel(GridView ge, GridView gs, BatchView bv, int gx, int remap) {
    __shared__ int wcnt[8];

    int bx, b;
    block_coords(remap, gx, bx, b);
    const int ne = bv.n_edge[b], nq = ne + bv.n_surf[b];
    if (bx * 256 >= nq) return;   // uniform per block, ahead of the barrier
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t F = bv.feat_stride;
    const Pose Ps = load_pose(bv.st[b].x);
    const int i = bx * 256 + threadIdx.x;
    bool need = i < nq;
    bool refit = false;   // same 5 neighbours in a new order: fit without a walk
    unsigned int n_refit = 0;
    unsigned int n_reused = 0;
    float lim = kFullLim;   // a miss's search radius^2: the 6 nearest at w0 are within s6 + d of w
    double P[kPacket];
#pragma unroll
    for (int e = 0; e < kPacket; ++e) P[e] = 0.0;
    if (need) {
        const size_t pos = (size_t)b * F + i;   // search position: memo state and records live here
        const float4 p = bv.featp[pos];
        const int q = __float_as_int(p.w);
        const float4 pw = bv.prevw[pos];
        // everything the position may need, in flight together (the pass is latency-bound: one round trip
        // for the state instead of three dependent ones -- memo words, then the record)
        int mw[7];
        if constexpr (kMemoAos) {
            const int4 m0 = *reinterpret_cast<const int4*>(bv.memo_nbr + memo_idx(b, 0, i, F));
            const int4 m1 = *reinterpret_cast<const int4*>(bv.memo_nbr + memo_idx(b, 4, i, F));
            mw[0] = m0.x; mw[1] = m0.y; mw[2] = m0.z; mw[3] = m0.w; mw[4] = m1.x; mw[5] = m1.y; mw[6] = m1.z;
        } else {
#pragma unroll
            for (int j = 0; j < 7; ++j) mw[j] = bv.memo_nbr[memo_idx(b, j, i, F)];
        }
        RecV rv;
        const float4 rp = load_record(bv, pos, i, ne, rv);
        if (q >= 0 && q < nq && pw.w >= 0.f) {
            const size_t slot = pos;
            const float3 w = associate(Ps, p);
            const double dx = (double)w.x - pw.x, dy = (double)w.y - pw.y, dz = (double)w.z - pw.z;
            const double dd = sqrt(dx * dx + dy * dy + dz * dz);
            const double s6 = (double)__int_as_float(mw[5]);
            const double r6 = s6 + dd + 1e-5;
            if (r6 < 1.0 && bv.memo_bound) lim = fminf(kFullLim, (float)(r6 * r6) + 1e-5f);
            // every distance moved by at most dd: with 2 dd + 1e-5 below every gap between consecutive
            // neighbours and below s6 - s5, neither the set nor the order of the 5 nearest changed, and a
            // search would return the stored keys -- no re-keying (r01's test, ahead of the exact one)
            const double gord = (double)__int_as_float(mw[6]);
            bool same = bv.memo_order && 2.0 * dd + 1e-5 < gord;
            if (!same && (bv.memo_exact || 2.0 * dd + 1e-5 < (double)pw.w)) {
                const float4* orig = q < ne ? ge.orig : gs.orig;
                uint32_t idx[5];
                double k[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) idx[j] = (uint32_t)mw[j];
#pragma unroll
                for (int j = 0; j < 5; ++j) k[j] = nn_key(w, orig[idx[j]], idx[j]);
                // 5-key sorting network (9 compare-exchanges)
                key_cswap(k[0], k[1]); key_cswap(k[3], k[4]); key_cswap(k[2], k[4]);
                key_cswap(k[2], k[3]); key_cswap(k[0], k[3]); key_cswap(k[0], k[2]);
                key_cswap(k[1], k[4]); key_cswap(k[1], k[3]); key_cswap(k[1], k[2]);
                // all five still inside the radius and still the 5 nearest: the farthest of them is nearer
                // than any other point can have come (those were >= s6 from w0, so >= s6 - d from w)
                const bool inside = key_bits(k[4]) < kSentinel && sqrt((double)key_d2(k[4])) + dd + 1e-5 < s6;
                same = inside;
#pragma unroll
                for (int j = 0; j < 5; ++j) same = same && (uint32_t)key_bits(k[j]) == idx[j];
                refit = inside && !same && bv.memo_refit;
                if (refit) {   // the set's new order is what a search would return: keep it for the fit
#pragma unroll
                    for (int j = 0; j < 5; ++j)
                        bv.memo_nbr[memo_idx(b, j, i, F)] = (int)(uint32_t)key_bits(k[j]);
                    bv.memo_nbr[memo_idx(b, 6, i, F)] = __float_as_int(-1.f);   // gaps are w0's order
                    need = false;
                    n_refit = 1;
                }
            }
            if (same) {
                const int kind = __float_as_int(rp.w);
                d3 v0 = mk(0, 0, 0);
                double v1x = 0.0, v1y = 0.0, v1z = 0.0;
                bool reuse = true;
                if (kind != 0) {
                    const RecV v = rv;
                    v0 = mk(v.v[0], v.v[1], v.v[2]);
                    v1x = v.v[3];
                    if (kind == LMSF_SURF) {
                        // surf_fit keeps its plane (n, D) when (float)(n . w + D) >= 0 and flips it
                        // otherwise; the stored record is that plane up to sign, and negation is exact,
                        // so t = (float)(n_s . w + D_s) = +-(the fit's test): t > 0 -> the stored record
                        // is the fit's answer at w, t < 0 -> its negation; t == 0 is ambiguous (search)
                        const d3 cp = mk((double)w.x, (double)w.y, (double)w.z);
                        const float t = (float)(dot(v0, cp) + v1x);
                        reuse = t != 0.f;
                        if (t < 0.f) {
                            v0 = mk(-v0.x, -v0.y, -v0.z);
                            v1x = -v1x;
                            store_record(bv, slot, p, kind, v0, v1x, 0.0, 0.0);
                        }
                    } else if (!kLinEval) {
                        const double2 e = bv.rec_e[slot];
                        v1y = e.x;
                        v1z = e.y;
                    }
                }
                if (reuse) {
                    if (!kLinEval) record_packet(kind, p, v0, v1x, v1y, v1z, Ps, P);
                    need = false;
                    refit = false;
                    n_reused = 1;
                }
            }
        }
    }
    if (!kLinEval && bx * 256 + wave * 64 < nq)
        wave_reduce_packet(P, bv.partials + ((size_t)b * bv.max_parts + (size_t)bx * 4 + wave) * kPacket);
    const unsigned long long m = __ballot(need), mr = __ballot(refit);
    const unsigned long long below = (1ull << lane) - 1ull;
    if constexpr (kListAtomic) {
        // the scan's searches from the front of its list and its refits from the back, a block's entries placed by
        // one atomic each (counters at wcount[b * memo_blocks(F) + 0 / 1], zeroed before the pass): no block counts
        // for the search kernel to scan, and the entry order does not matter -- no packets downstream.  (One
        // atomic per wave on the scan's counter serialised ~970 waves per address: memo pass 310 vs 201 us.)
        __shared__ int wbase[2];
        if (lane == 0) {
            wcnt[wave] = __popcll(m);
            wcnt[4 + wave] = __popcll(mr);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int* cnt = bv.wcount + (size_t)b * memo_blocks(F);
            const int ts = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3], tr = wcnt[4] + wcnt[5] + wcnt[6] + wcnt[7];
            wbase[0] = ts ? atomicAdd(cnt, ts) : 0;
            wbase[1] = tr ? atomicAdd(cnt + 1, tr) : 0;
        }
        __syncthreads();
        int before = wbase[0], before_r = wbase[1];
#pragma unroll
        for (int w4 = 0; w4 < 4; ++w4) {
            before += w4 < wave ? wcnt[w4] : 0;
            before_r += w4 < wave ? wcnt[4 + w4] : 0;
        }
        if (need) {
            const size_t at = (size_t)b * F + before + __popcll(m & below);
            bv.wl[at] = i;
            bv.wlim[at] = lim;
        }
        if (refit) bv.wl[(size_t)b * F + F - 1 - (before_r + __popcll(mr & below))] = i;
    } else {
        // this block's positions still needing a search, in position order from the front of its segment,
        // and those needing only a refit, in position order from its back (deterministic)
        if (lane == 0) {
            wcnt[wave] = __popcll(m);
            wcnt[4 + wave] = __popcll(mr);
        }
        __syncthreads();
        int before = 0, total = 0, before_r = 0, total_r = 0;
#pragma unroll
        for (int w4 = 0; w4 < 4; ++w4) {
            before += w4 < wave ? wcnt[w4] : 0;
            total += wcnt[w4];
            before_r += w4 < wave ? wcnt[4 + w4] : 0;
            total_r += wcnt[4 + w4];
        }
        if (need) {
            const size_t at = (size_t)b * F + (size_t)bx * 256 + before + __popcll(m & below);
            bv.wl[at] = i;
            bv.wlim[at] = lim;
        }
        if (refit) {
            const int seg = min(256, nq - bx * 256);
            bv.wl[(size_t)b * F + (size_t)bx * 256 + seg - 1 - (before_r + __popcll(mr & below))] = i;
        }
        if (threadIdx.x == 0) bv.wcount[(size_t)b * memo_blocks(F) + bx] = total | (total_r << 16);
    }

    if (bv.n27) {   // accounting runs: queries and reused ones
        unsigned int qn = i < nq ? 1u : 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            qn += __shfl_xor(qn, o, 64);
            n_reused += __shfl_xor(n_reused, o, 64);
            n_refit += __shfl_xor(n_refit, o, 64);
        }
        if (lane == 0) {
            unsigned long long* shard = bv.n27 + (size_t)((blockIdx.x * 4 + wave) & (kCounterShards - 1)) * 16;
            if (qn) atomicAdd(shard + 1, (unsigned long long)qn);
            if (n_reused) atomicAdd(shard + 2, (unsigned long long)n_reused);
            if (n_refit) atomicAdd(shard + 3, (unsigned long long)n_refit);
        }
    }
}

// Fused 5-NN search + fit for batch launches (one lane per query, Ceres-LM solver): the walk of
// knn_walk<1, false, PRUNE>, then the line / plane fit, record write and Huber-weighted packet at the
// linearisation pose on the neighbours held in registers (knn_kernel + fit_eval_kernel hand the 5
// neighbour points through memory instead).  LIST = false: every search position i < nq (edge slots
// then surf slots, each in ring order, so neighbouring lanes search neighbouring ring points and a
// wave runs one fit kind).  LIST = true: only the positions the memo pass listed -- entry e of the
// concatenation of its blocks' lists (each block scans the block counts into LDS and finds its
// entries' blocks by binary search), so the searches fill whole waves.  Sparse maps (!PRUNE) keep
// the 6th-nearest key and leave position i's anchor (w, s6 - s5) and neighbour indices for the memo
// pass; on dense maps (PRUNE) the walk prunes with the last kept key, so it keeps 5 and has no memo
// (C5: keeping a 6th weakens the pruning more than reuse saves, 2568 / 2660 vs 2830 pairs/s, r01).
// One packet per wave at partial index part2_base + 4 bx + wave.
// Waves per SIMD the kernel is compiled for (A/B): 4 = its natural ~120 VGPRs, no scratch.  Forcing 5
// (96 VGPRs, 100 B spill) measured 16.2k scans/s, 6 (80, 168 B) 15.2k, vs 17.0k at 4 (r01).
// Candidate loads in flight per row step of the walk (A/B): 4 (0.472-0.477 ms) beat 2 (0.49), 6
// (0.485), 8 (0.51) and a walk flattened across rows with 4-16 in flight (0.52-0.54) (r01).
#ifndef LMSF_FUSED_UNROLL
#define LMSF_FUSED_UNROLL 4
#endif
#ifndef LMSF_FUSED_WAVES
#define LMSF_FUSED_WAVES 4
#endif
template <bool PRUNE, bool LIST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LMSF_FUSED_WAVES))) void match_fit_kernel(GridView ge, GridView gs, BatchView bv, int gx, int remap) {
    extern __shared__ int soff[];   // LIST: exclusive prefixes of the memo blocks' search / refit counts, 2 x [nblk + 1]
    constexpr bool kMemo = !PRUNE;
    constexpr int kNK = kMemo ? 6 : 5;
    int bx, b;
    block_coords(remap, gx, bx, b);
    const int ne = bv.n_edge[b], nq = ne + bv.n_surf[b];
    const size_t F = bv.feat_stride;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int total = nq, nblk = 0, total_s = nq;
    int* roff = soff;
    if constexpr (LIST && kListAtomic) {   // the scan's list lengths (memo pass atomics)
        const int* cnt = bv.wcount + (size_t)b * memo_blocks(F);
        total_s = cnt[0];
        total = total_s + cnt[1];
    } else if constexpr (LIST) {   // block counts: searches in the low 16 bits, refits in the high 16
        __shared__ int wsum[8];
        nblk = (nq + 255) / 256;
        roff = soff + nblk + 1;
        const int* wc = bv.wcount + (size_t)b * memo_blocks(F);
        const int per = (nblk + 255) / 256;
        const int j0 = threadIdx.x * per;
        int mine = 0, mine_r = 0;
        for (int j = 0; j < per; ++j) {
            const int c = j0 + j < nblk ? wc[j0 + j] : 0;
            mine += c & 0xffff;
            mine_r += c >> 16;
        }
        int incl = mine, incl_r = mine_r;   // wave inclusive scans
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64), tr = __shfl_up(incl_r, o, 64);
            incl += lane >= o ? t : 0;
            incl_r += lane >= o ? tr : 0;
        }
        if (lane == 63) {
            wsum[wave] = incl;
            wsum[4 + wave] = incl_r;
        }
        __syncthreads();
        int run = incl - mine, run_r = incl_r - mine_r;
#pragma unroll
        for (int w4 = 0; w4 < 4; ++w4) {
            run += w4 < wave ? wsum[w4] : 0;
            run_r += w4 < wave ? wsum[4 + w4] : 0;
        }
        for (int j = 0; j < per; ++j) {
            if (j0 + j < nblk) {
                const int c = wc[j0 + j];
                soff[j0 + j] = run;
                roff[j0 + j] = run_r;
                run += c & 0xffff;
                run_r += c >> 16;
            }
        }
        total_s = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        total = total_s + wsum[4] + wsum[5] + wsum[6] + wsum[7];
        if (threadIdx.x == 0) {
            soff[nblk] = total_s;
            roff[nblk] = total - total_s;
        }
        __syncthreads();
    }
    if (bx == 0 && threadIdx.x == 0) bv.n_search[b] = total;   // listed entries (packets), refits included
    if (bx * 256 >= total) return;   // uniform per block, after the last barrier
    const Pose Ps = load_pose(bv.st[b].x);
    const int e = bx * 256 + threadIdx.x;
    unsigned int c27 = 0;
    double P[kPacket];
#pragma unroll
    for (int j = 0; j < kPacket; ++j) P[j] = 0.0;
    if (e < total) {
        int pos = e;
        float lim = kFullLim;
        bool walk = true;
        if constexpr (LIST && kListAtomic) {
            if (e < total_s) {
                const size_t at = (size_t)b * F + e;
                pos = bv.wl[at];
                lim = bv.wlim[at];
            } else {
                pos = bv.wl[(size_t)b * F + F - 1 - (e - total_s)];
                walk = false;
            }
        } else if constexpr (LIST) {   // largest block whose list starts at or before e (empty blocks share offsets)
            const bool rf = e >= total_s;   // refit entries follow the searches
            const int er = rf ? e - total_s : e;
            const int* off = rf ? roff : soff;
            int lo = 0, hi = nblk - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (off[mid] <= er) lo = mid;
                else hi = mid - 1;
            }
            if (!rf) {
                const size_t at = (size_t)b * F + (size_t)lo * 256 + (er - off[lo]);
                pos = bv.wl[at];
                lim = bv.wlim[at];
            } else {
                const int seg = min(256, nq - lo * 256);
                pos = bv.wl[(size_t)b * F + (size_t)lo * 256 + seg - 1 - (er - off[lo])];
                walk = false;
            }
        }
        const size_t ppos = (size_t)b * F + pos;
        const float4 p = bv.featp[ppos];        // the feature at this search position, w = its slot
        const int qq = __float_as_int(p.w);
        const bool is_edge = qq < ne;
        const GridView g = pick_grid(is_edge, ge, gs);
        const size_t slot = (size_t)b * F + qq;   // nnp (lmsf_match diagnostics) stays slot-indexed
        const float3 w = associate(Ps, p);
        const double sentinel = key_as_double(kSentinel);
        double k[kNK];
#pragma unroll
        for (int j = 0; j < kNK; ++j) k[j] = sentinel;
        if (walk) {
#ifndef LMSF_AB_NOWALK   // A/B ablation builds only (tools/build_variant.sh): no search
            knn_walk<1, false, PRUNE, LMSF_FUSED_UNROLL, kNK>(g, g, w, 0, bv.count27, k, c27, lim);
#endif
        } else {   // refit: the memo pass left the 5 neighbours in their order at w (key bits: index only)
#pragma unroll
            for (int j = 0; j < 5; ++j)
                k[j] = key_as_double((uint64_t)(uint32_t)bv.memo_nbr[memo_idx(b, j, pos, F)]);
        }
        if (kMemo && walk) {   // anchor for the memo pass: gap between the 5th and the 6th neighbour (capped at 1 m)
            float gap = -1.f;
            if (key_bits(k[4]) < kSentinel) {
                const double s6 = sqrt((double)fminf(key_d2(k[5]), 1.0f));
                double sj = sqrt((double)key_d2(k[0])), gord = 1.0;
#pragma unroll
                for (int j = 1; j < 5; ++j) {   // the smallest gap between consecutive neighbours
                    const double sn = sqrt((double)key_d2(k[j]));
                    gord = fmin(gord, sn - sj);
                    sj = sn;
                }
                gap = (float)(s6 - sj);
                if constexpr (kMemoAos) {   // the position's 32-B memo record in two 16-B stores
                    int* mp = bv.memo_nbr + memo_idx(b, 0, pos, F);
                    *reinterpret_cast<int4*>(mp) = make_int4((int)(uint32_t)key_bits(k[0]), (int)(uint32_t)key_bits(k[1]),
                                                             (int)(uint32_t)key_bits(k[2]), (int)(uint32_t)key_bits(k[3]));
                    *reinterpret_cast<int4*>(mp + 4) = make_int4((int)(uint32_t)key_bits(k[4]), __float_as_int((float)s6),
                                                                 __float_as_int((float)fmin(gord, s6 - sj)), 0);
                } else {
#pragma unroll
                    for (int j = 0; j < 5; ++j) bv.memo_nbr[memo_idx(b, j, pos, F)] = (int)(uint32_t)key_bits(k[j]);
                    bv.memo_nbr[memo_idx(b, 5, pos, F)] = __float_as_int((float)s6);
                    bv.memo_nbr[memo_idx(b, 6, pos, F)] = __float_as_int((float)fmin(gord, s6 - sj));
                }
            }
            bv.prevw[ppos] = make_float4(w.x, w.y, w.z, gap);
        }
        float4 np[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint64_t kb = key_bits(k[j]);
            np[j] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
            if (kb < kSentinel) {
                const uint32_t idx = (uint32_t)kb;
                const float4 mp = g.orig[idx];
                np[j] = make_float4(mp.x, mp.y, mp.z, __int_as_float((int)idx));
            }
        }
        if (bv.write_nn) {
#pragma unroll
            for (int j = 0; j < 5; ++j) bv.nnp[slot * 5 + j] = np[j];
        }
        int kind = 0;
        d3 v0 = mk(0, 0, 0);
        double v1x = 0.0, v1y = 0.0, v1z = 0.0;
#ifndef LMSF_AB_NOFIT      // A/B ablation builds only: search without the fit
        if (__float_as_int(np[4].w) >= 0) {   // fit_query's LM branch
            if (is_edge) {
                d3 a, bpt;
                if (edge_fit(np, a, bpt)) {
                    kind = LMSF_EDGE;
                    v0 = a;
                    v1x = bpt.x; v1y = bpt.y; v1z = bpt.z;
                }
            } else {
                d3 n;
                double D, gn_res;
                if (surf_fit(np, w, n, D, gn_res)) {
                    kind = LMSF_SURF;
                    v0 = n;
                    v1x = D;
                }
            }
        }
#endif
        store_record(bv, ppos, p, kind, v0, v1x, v1y, v1z);   // records by search position
        if (!kLinEval) record_packet(kind, p, v0, v1x, v1y, v1z, Ps, P);
    }
    if (!kLinEval && bx * 256 + wave * 64 < total)
        wave_reduce_packet(P, bv.partials + ((size_t)b * bv.max_parts + bv.part2_base + (size_t)bx * 4 + wave) * kPacket);
    if (bv.n27) {   // accounting runs: n27 of the searches (+ the queries when there was no memo pass)
        unsigned int qn = (!LIST && e < total) ? 1u : 0u;
        unsigned long long c = c27;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            qn += __shfl_xor(qn, o, 64);
            c += __shfl_xor(c, o, 64);
        }
        if (lane == 0) {
            unsigned long long* shard = bv.n27 + (size_t)((blockIdx.x * 4 + wave) & (kCounterShards - 1)) * 16;
            if (c) atomicAdd(shard, c);
            if (qn) atomicAdd(shard + 1, (unsigned long long)qn);
        }
    }
}

// ---------------------------------------------------------------- dense maps (C5): first pass on a fine grid, pass 2 listed
// The pruned one-lane walk of match_fit_kernel<true, .> ran at lane utilisation 0.53 on C5 (VALU busy 0.94,
// profiles/r03/C5) and scanned ~9x the points inside its first-pass sphere: the 1 m y-z rows of the match-radius
// grid are far wider than the first-pass radius sqrt(lim1) (0.23 m on C5's surf map, tools/c5_walk_model.py).
//   dense_pass1_kernel: one lane per query, its 9 first-pass rows resolved up front (offsets only, one batch of
//     loads) on the map's first-pass grid (FineGrid: y-z cells of 1/sy m holding the first-pass radius, 8
//     x-slices per metre; the 1 m grid when the map has none), then walked one loop per row, nearest rows first,
//     a row entered only while its yz-gap bound is within the current 5th key.  A query whose 5th key is within
//     lim1 is complete (every point nearer than its 5th lies in the scanned ball) and is fitted here; the others
//     go, with their 5th key as the bound, to a work list.
//   dense_pass2_kernel: the listed queries (dense, grid-stride) run a fresh pruned walk on the 1 m grid bounded
//     by that key (the 5 nearest lie within it), then the fit.
// Results are the pruned walk's exactly (keys totally ordered by (d2, index): the kept 5 do not depend on the
// grid or the visit order).  A/B on C5 (profiles/r04/ab_notes.md): this form 3370 pairs/s vs 2967 for r03's
// kernel on one box; re-dealing a block's queries to its waves by pass-1 work (LDS counting sort) 3220, and a
// flattened candidate stream 3261 -- both cost more than the lane balance they bought.
#ifndef LMSF_DENSE_SPLIT
#define LMSF_DENSE_SPLIT 1
#endif

// The line / plane fit of a query's 5 kept keys and its record (match_fit_kernel's tail).
__device__ __forceinline__ void dense_finish(const GridView& g, const BatchView& bv, size_t ppos, const float4 p, bool is_edge,
                                             size_t slot, const float3 w, const double (&k)[5]) {
    float4 np[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const uint64_t kb = key_bits(k[j]);
        np[j] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
        if (kb < kSentinel) {
            const uint32_t idx = (uint32_t)kb;
            const float4 mp = g.orig[idx];
            np[j] = make_float4(mp.x, mp.y, mp.z, __int_as_float((int)idx));
        }
    }
    if (bv.write_nn) {
#pragma unroll
        for (int j = 0; j < 5; ++j) bv.nnp[slot * 5 + j] = np[j];
    }
    int kind = 0;
    d3 v0 = mk(0, 0, 0);
    double v1x = 0.0, v1y = 0.0, v1z = 0.0;
    if (__float_as_int(np[4].w) >= 0) {
        if (is_edge) {
            d3 a, bpt;
            if (edge_fit(np, a, bpt)) {
                kind = LMSF_EDGE;
                v0 = a;
                v1x = bpt.x; v1y = bpt.y; v1z = bpt.z;
            }
        } else {
            d3 n;
            double D, gn_res;
            if (surf_fit(np, w, n, D, gn_res)) {
                kind = LMSF_SURF;
                v0 = n;
                v1x = D;
            }
        }
    }
    store_record(bv, ppos, p, kind, v0, v1x, v1y, v1z);
}

// Row rr (0..8: dy, dz in {-1, 0, 1}) of the pruned walk around w: its offsets row, x-slice span [xa, xb], the
// yz-gap bound lb and the grid's x origin / slices; false outside the grid (knn_walk's row_geo).
// A query's row geometry on a grid, the parts shared by its rows computed once: the x-slice span (3 m of slices
// around floor(w.x)), its cell (y, z), and the yz gaps to the cells R rows away (gy[R + d] for row offset d; the
// same float expressions per row as knn_walk's, so each row's bound lb = gy^2 + gz^2 is bit-identical).
template <int R>
struct DenseQuery {
    bool inside;
    int xa, xb, cy0, cz0;
    float gy[2 * R + 1], gz[2 * R + 1];
    __device__ __forceinline__ DenseQuery(const GridView& gg, const float3 w) {
        // y / z cells of 1 / sy m (sy a power of two: products by sy and 1 / sy are exact)
        const float fsy = (float)gg.sy, h = 1.0f / fsy;
        const float fx = floorf(w.x), fy = floorf(w.y * fsy), fz = floorf(w.z * fsy);
        const float fxs = fx * (float)gg.sx;
        inside = gg.n > 0 && fxs >= (float)(gg.ox - 2 * gg.sx) && fxs <= (float)(gg.ox + gg.nx + gg.sx) &&
                 fy >= (float)(gg.oy - R - 1) && fy <= (float)(gg.oy + gg.ny + R) && fz >= (float)(gg.oz - R - 1) &&
                 fz <= (float)(gg.oz + gg.nz + R);
        const int cxs = inside ? (int)fxs - gg.ox : 0;
        xa = max(cxs - gg.sx, 0);
        xb = min(cxs + 2 * gg.sx - 1, gg.nx - 1);
        inside = inside && xa <= xb;
        cy0 = inside ? (int)fy - gg.oy : 0;
        cz0 = inside ? (int)fz - gg.oz : 0;
#pragma unroll
        for (int d = -R; d <= R; ++d) {
            const float ylo = (fy + (float)d) * h, zlo = (fz + (float)d) * h;
            gy[R + d] = fmaxf(0.f, fmaxf(ylo - w.y, w.y - (ylo + h)));
            gz[R + d] = fmaxf(0.f, fmaxf(zlo - w.z, w.z - (zlo + h)));
        }
    }
    // the gap of offset d as a select chain (a runtime index into gy / gz would put them in scratch)
    __device__ __forceinline__ static float pick(const float (&a)[2 * R + 1], int d) {
        float v = a[0];
#pragma unroll
        for (int j = 1; j <= 2 * R; ++j) v = d == j - R ? a[j] : v;
        return v;
    }
    // row (dyo, dzo): its bound (always) and, when it lies in the grid, its offsets row
    __device__ __forceinline__ float lb(int dyo, int dzo) const {
        const float y = pick(gy, dyo), z = pick(gz, dzo);
        return y * y + z * z;
    }
    __device__ __forceinline__ bool row(const GridView& gg, int dyo, int dzo, const uint32_t*& r) const {
        const int cy = cy0 + dyo, cz = cz0 + dzo;
        if (!inside || cy < 0 || cy >= gg.ny || cz < 0 || cz >= gg.nz) return false;
        r = gg.off + ((size_t)cz * gg.ny + cy) * gg.nx;
        return true;
    }
};

// slices of [xa, xb] meeting [w.x - r, w.x + r], r = sqrt(lim - lb) (sa > sb: empty) -- knn_walk's window
__device__ __forceinline__ void dense_window(const GridView& gg, const float3 w, float lim, float lb, int xa, int xb, int& sa,
                                             int& sb) {
    const float rem = lim - lb;
    sa = 1;
    sb = 0;
    if (rem < 0.f) return;
    const double r = (double)sqrtf(rem);
    sa = max(xa, (int)floor(((double)w.x - r) * gg.sx) - gg.ox);
    sb = min(xb, (int)floor(((double)w.x + r) * gg.sx) - gg.ox);
}

template <int NK>
__device__ __forceinline__ void key_insert(double (&k)[NK], double x) {
#pragma unroll
    for (int i = 0; i < NK; ++i) {
        const double lo = key_min(k[i], x);
        x = key_max(k[i], x);
        k[i] = lo;
    }
}

// One row's candidates [a, a + len) of pts into the kept NK keys k.
template <int NK>
__device__ __forceinline__ void dense_run(double (&k)[NK], const float4* __restrict__ rp, uint32_t a, uint32_t len, const float3 w) {
    uint32_t c = 0;
    for (; c + LMSF_FUSED_UNROLL <= len; c += LMSF_FUSED_UNROLL) {
        float4 m[LMSF_FUSED_UNROLL];
#pragma unroll
        for (int u = 0; u < LMSF_FUSED_UNROLL; ++u) m[u] = rp[a + c + u];
#pragma unroll
        for (int u = 0; u < LMSF_FUSED_UNROLL; ++u) key_insert(k, nn_key(w, m[u], (uint32_t)__float_as_int(m[u].w)));
    }
    if constexpr (kTailPairs) {
        if (c + 2 <= len) {
            const float4 m0 = rp[a + c], m1 = rp[a + c + 1];
            key_insert(k, nn_key(w, m0, (uint32_t)__float_as_int(m0.w)));
            key_insert(k, nn_key(w, m1, (uint32_t)__float_as_int(m1.w)));
            c += 2;
        }
        if (c < len) {
            const float4 m = rp[a + c];
            key_insert(k, nn_key(w, m, (uint32_t)__float_as_int(m.w)));
        }
    } else {
        for (; c < len; ++c) {
            const float4 m = rp[a + c];
            key_insert(k, nn_key(w, m, (uint32_t)__float_as_int(m.w)));
        }
    }
}

constexpr int kDenseRowOrder[9] = {4, 1, 3, 5, 7, 0, 2, 6, 8};   // own row, faces, corners (knn_walk's kOrder)
constexpr float kDenseCull = 1.0f + 1e-5f;                       // knn_walk's kCullLim

// The kept 5 indices (-1: none) in key order, for the fit kernel, in the position's memo record.
template <int NK>
__device__ __forceinline__ void store_kept(const BatchView& bv, int b, int e, size_t F, const double (&k)[NK]) {
    int kid[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) kid[j] = key_bits(k[j]) < kSentinel ? (int)(uint32_t)key_bits(k[j]) : -1;
    if constexpr (kMemoAos) {   // one 32-B record: words 0-3 as one 16-B store
        int* mp = bv.memo_nbr + memo_idx(b, 0, e, F);
        *reinterpret_cast<int4*>(mp) = make_int4(kid[0], kid[1], kid[2], kid[3]);
        mp[4] = kid[4];
    } else {                    // planar A/B layout: word j of position e at memo_idx(b, j, e, F)
#pragma unroll
        for (int j = 0; j < 5; ++j) bv.memo_nbr[memo_idx(b, j, e, F)] = kid[j];
    }
}

// The memo anchor of an exact 6-key search at w (match_fit_kernel's, for the sparse maps' memo pass): the 5
// indices, s6 (capped at 1 m), the smallest consecutive gap, and prevw = (w, s6 - s5); gap -1: fewer than 5.
__device__ __forceinline__ void store_anchor(const BatchView& bv, int b, int pos, size_t F, const float3 w,
                                             const double (&k)[6]) {
    float gap = -1.f;
    if (key_bits(k[4]) < kSentinel) {
        const double s6 = sqrt((double)fminf(key_d2(k[5]), 1.0f));
        double sj = sqrt((double)key_d2(k[0])), gord = 1.0;
#pragma unroll
        for (int j = 1; j < 5; ++j) {
            const double sn = sqrt((double)key_d2(k[j]));
            gord = fmin(gord, sn - sj);
            sj = sn;
        }
        gap = (float)(s6 - sj);
        const int w5 = __float_as_int((float)s6), w6 = __float_as_int((float)fmin(gord, s6 - sj));
        if constexpr (kMemoAos) {
            int* mp = bv.memo_nbr + memo_idx(b, 0, pos, F);
            *reinterpret_cast<int4*>(mp) = make_int4((int)(uint32_t)key_bits(k[0]), (int)(uint32_t)key_bits(k[1]),
                                                     (int)(uint32_t)key_bits(k[2]), (int)(uint32_t)key_bits(k[3]));
            *reinterpret_cast<int4*>(mp + 4) = make_int4((int)(uint32_t)key_bits(k[4]), w5, w6, 0);
        } else {
#pragma unroll
            for (int j = 0; j < 5; ++j) bv.memo_nbr[memo_idx(b, j, pos, F)] = (int)(uint32_t)key_bits(k[j]);
            bv.memo_nbr[memo_idx(b, 5, pos, F)] = w5;
            bv.memo_nbr[memo_idx(b, 6, pos, F)] = w6;
        }
    }
    bv.prevw[(size_t)b * F + pos] = make_float4(w.x, w.y, w.z, gap);
}

template <int NK>
__device__ __forceinline__ void first5(const double (&k)[NK], double (&k5)[5]) {
#pragma unroll
    for (int j = 0; j < 5; ++j) k5[j] = k[j];
}

// Pass 1 of one query on grid g (its kind's first-pass grid, else its 1 m grid): the 9 rows' offsets resolved up front
// (the 18 loads in flight together), each trimmed to the first-pass ball sqrt(lim1), walked nearest row first while
// a row's yz-gap bound is within the current NK-th key.
template <int NK>
__device__ __forceinline__ void dense_first_pass(const GridView& g, const float3 w, int count27, double (&k)[NK],
                                                 unsigned int& c27) {
    uint32_t st_[9], ln_[9];
    float lb_[9];
    const float lim1 = g.lim1 * kDenseCull;
    const DenseQuery<1> dq(g, w);
    const int xa = dq.xa, xb = dq.xb;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        st_[i] = 0;
        ln_[i] = 0;
        const int dyo = (kDenseRowOrder[i] % 3) - 1, dzo = (kDenseRowOrder[i] / 3) - 1;
        const float lb = dq.lb(dyo, dzo);
        lb_[i] = lb;
        const uint32_t* row;
        int sa, sb;
        if (!dq.row(g, dyo, dzo, row)) continue;
        if (count27) c27 += row[xb + 1] - row[xa];
        if (lb > lim1) continue;
        dense_window(g, w, lim1, lb, xa, xb, sa, sb);
        if (sa <= sb) {
            st_[i] = row[sa];
            ln_[i] = row[sb + 1] - st_[i];
        }
    }
    const float4* rp = g.pts;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const uint32_t ln = ln_[i];
        if (!ln || lb_[i] > key_d2(k[NK - 1])) continue;
        dense_run(k, rp, st_[i], ln, w);
    }
}

// NK = 5, or 6 in the outer iteration before the dense memo starts (BatchView::anchor): the 6th-nearest key is then
// exact too (rows pruned with it), and complete queries leave the memo anchor.
template <int NK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LMSF_FUSED_WAVES))) void dense_pass1_kernel(
    GridView ge, GridView gs, GridView fe, GridView fs, BatchView bv, int gx, int remap, unsigned* p2count) {
    int bx, b;
    block_coords(remap, gx, bx, b);
    const int ne = bv.n_edge[b], nq = ne + bv.n_surf[b];
    const size_t F = bv.feat_stride;
    if (bx == 0 && threadIdx.x == 0) bv.n_search[b] = nq;
    if (bx * 256 >= nq) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long below = (1ull << lane) - 1ull;
    const int e = bx * 256 + threadIdx.x;
    const bool valid = e < nq;
    const size_t ppos = (size_t)b * F + (valid ? e : 0);
    const float4 p = bv.featp[ppos];
    const int qq = __float_as_int(p.w);
    const bool is_edge = qq < ne;
    // the first-pass grid of the query's kind (FineGrid), else its 1 m grid
    const GridView g = pick_grid(is_edge, pick_grid(fe.n > 0, fe, ge), pick_grid(fs.n > 0, fs, gs));
    const float3 w = associate(load_pose(bv.st[b].x), p);
    const double sentinel = key_as_double(kSentinel);
    double k[NK];
#pragma unroll
    for (int j = 0; j < NK; ++j) k[j] = sentinel;
    unsigned int c27 = 0;
    if (valid) dense_first_pass(g, w, bv.count27, k, c27);
    // complete (NK-th key within lim1: nothing nearer lies outside the scanned ball) -> fit; else -> pass-2 list
    const bool p2 = valid && key_d2(k[NK - 1]) > g.lim1;
    const unsigned long long m2 = __ballot(p2);
    int base2 = 0;
    if (lane == 0 && m2) base2 = (int)atomicAdd(p2count, (unsigned)__popcll(m2));
    base2 = __shfl(base2, 0, 64);
    if (p2) {   // pass 2 from scratch, bounded by this NK-th key (the NK nearest lie within it)
        const int at = base2 + __popcll(m2 & below);
        bv.wl[at] = (int)((size_t)b * F + e);
        bv.wlim[at] = key_d2(k[NK - 1]);
    } else if (valid) {
        if constexpr (NK == 6) store_anchor(bv, b, e, F, w, k);
        double k5[5];
        first5(k, k5);
        dense_finish(g, bv, ppos, p, is_edge, (size_t)b * F + qq, w, k5);   // g.orig: the caller-order map either way
    }
    if (bv.n27) {   // accounting runs: the 27-cell candidates (of the first-pass grid) and the queries
        unsigned int qn = valid ? 1u : 0u;
        unsigned long long c = c27;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            qn += __shfl_xor(qn, o, 64);
            c += __shfl_xor(c, o, 64);
        }
        if (lane == 0) {
            unsigned long long* shard = bv.n27 + (size_t)((blockIdx.x * 4 + wave) & (kCounterShards - 1)) * 16;
            if (c) atomicAdd(shard, c);
            if (qn) atomicAdd(shard + 1, (unsigned long long)qn);
        }
    }
}

// The listed queries of dense_pass1_kernel (their 5th key beyond lim1): a fresh pruned walk on the 1 m grid,
// rows nearest first, every row and x-window bounded by min(the pass-1 5th key, the current 5th key) -- the 5
// nearest lie within the pass-1 bound, so the walk is exact whichever grid pass 1 searched -- then the fit.
// The 5 x 5 rows of a 0.5 m first-pass grid around the query, nearest ring first: they hold every point within 1 m
// (a row two cells past them is >= 1 m away in y or z), so pass 2 can run there instead of on the 1 m grid.
constexpr int kRing5[25][2] = {{0, 0},  {0, -1}, {-1, 0}, {1, 0},  {0, 1},  {-1, -1}, {1, -1}, {-1, 1}, {1, 1},
                               {0, -2}, {-2, 0}, {2, 0},  {0, 2},  {-1, -2}, {1, -2}, {-2, -1}, {2, -1}, {-2, 1},
                               {2, 1},  {-1, 2}, {1, 2},  {-2, -2}, {2, -2}, {-2, 2}, {2, 2}};
#ifndef LMSF_PASS2_FINE
#define LMSF_PASS2_FINE 1
#endif
#ifndef LMSF_P2_INNER
#define LMSF_P2_INNER 0
#endif
// LMSF_P2_BALL2 (A/B): a pass-2 query whose bound exceeds one first-pass cell first walks the 0.5 m
// ball in pass 1's form (its 3 x 3 rows' offsets up front, windows at 0.25 m^2): when its NK-th key lies within the
// ball it is complete there; else the 25 rows continue bounded by min(bound, NK-th key), the inner rows minus the
// slices the ball scanned (outer iteration 0's displaced queries, which walked up to 1 m at lane utilisation 0.23).
#ifndef LMSF_P2_BALL2
#define LMSF_P2_BALL2 0
#endif

// The bounded pruned walk of pass 2 (and of the dense memo pass's listed searches): the NK nearest of w within
// `bound` (a squared distance at least the true NK-th key's), on the first-pass grid's 5 x 5 rows when the kind has
// one (sy = 2), else the 1 m grid's 3 x 3.
// A bound within one first-pass cell (bound x margin <= (1 / sy)^2) is walked in pass 1's form: the query's 3 x 3 rows
// hold the whole ball (its cell +- one cell of 1 / sy m in y and z, +-1 m of x-slices), their offsets resolved up
// front in one batch of loads, rows entered nearest first while their bound is within the current NK-th key.
// (r05: pass 2 and the dense memo's searches walked the 25 rows one dependent offset pair at a time -- C5 iteration 0
// pass 2 3.4 ms, the memo's listed searches 2.2-5.0 ms per dispatch.)
template <int NK>
__device__ __forceinline__ void dense_ball_walk(const GridView& g, const float3 w, float lim, double (&k)[NK]) {
    uint32_t st_[9], ln_[9];
    float lb_[9];
    const DenseQuery<1> dq(g, w);
    const int xa = dq.xa, xb = dq.xb;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        st_[i] = 0;
        ln_[i] = 0;
        const int dyo = (kDenseRowOrder[i] % 3) - 1, dzo = (kDenseRowOrder[i] / 3) - 1;
        const float lb = dq.lb(dyo, dzo);
        lb_[i] = lb;
        const uint32_t* row;
        int sa, sb;
        if (lb > lim || !dq.row(g, dyo, dzo, row)) continue;
        dense_window(g, w, lim, lb, xa, xb, sa, sb);
        if (sa <= sb) {
            st_[i] = row[sa];
            ln_[i] = row[sb + 1] - st_[i];
        }
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const uint32_t ln = ln_[i];
        if (!ln || lb_[i] > key_d2(k[NK - 1])) continue;
        dense_run(k, g.pts, st_[i], ln, w);
    }
}

template <int NK>
__device__ __forceinline__ const GridView dense_bounded_walk(const GridView& ge, const GridView& gs, const GridView& fe,
                                                             const GridView& fs, bool is_edge, const float3 w, float bound,
                                                             double (&k)[NK]) {
    const GridView gf = pick_grid(is_edge, fe, fs);
    const bool fine = LMSF_PASS2_FINE && gf.n > 0 && gf.sy == 2;
    const GridView g = pick_grid(fine, gf, pick_grid(is_edge, ge, gs));
#pragma unroll
    for (int j = 0; j < NK; ++j) k[j] = key_as_double(kSentinel);
    if (fine && bound * kDenseCull <= 0.25f) {   // within one 0.5 m first-pass cell
        dense_ball_walk(g, w, bound * kDenseCull, k);
        return g;
    }
    if constexpr (LMSF_P2_BALL2) {
        if (fine) {
            constexpr float kBall = 0.25f;   // (1 / sy)^2: the 3 x 3 rows hold every point within 0.5 m
            dense_ball_walk(g, w, kBall * kDenseCull, k);
            if (key_d2(k[NK - 1]) <= kBall) return g;   // every point nearer than the NK-th was in the scanned ball
            const DenseQuery<2> dq(g, w);
            const int xa = dq.xa, xb = dq.xb;
#pragma unroll 1
            for (int i = 0; i < 25; ++i) {
                const float d4 = fminf(bound, key_d2(k[NK - 1]));
                const uint32_t* row;
                int sa, sb;
                const int dyo = kRing5[i][0], dzo = kRing5[i][1];
                const float lb = dq.lb(dyo, dzo);
                if (lb > d4) continue;
                if (!dq.row(g, dyo, dzo, row)) continue;
                dense_window(g, w, d4 * kDenseCull, lb, xa, xb, sa, sb);
                if (sa > sb) continue;
                int ta = 1, tb = 0;   // the ball's slices of an inner row (scanned unless pruned: then lb > d4 here too)
                if (i < 9 && !(lb > kBall * kDenseCull)) dense_window(g, w, kBall * kDenseCull, lb, xa, xb, ta, tb);
                if (ta > tb) {
                    const uint32_t a = row[sa];
                    dense_run(k, g.pts, a, row[sb + 1] - a, w);
                } else {
                    const int l1 = min(sb, ta - 1), r0 = max(sa, tb + 1);
                    if (sa <= l1) {
                        const uint32_t a = row[sa];
                        dense_run(k, g.pts, a, row[l1 + 1] - a, w);
                    }
                    if (r0 <= sb) {
                        const uint32_t a = row[r0];
                        dense_run(k, g.pts, a, row[sb + 1] - a, w);
                    }
                }
            }
            return g;
        }
    }
    // LMSF_P2_INNER (A/B): a larger ball's inner 3 x 3 rows also resolved up front (windows at the bound), then the
    // outer ring's 16 rows one by one (their yz-gap bound is >= 0.25 m^2: pruned once the kept keys are nearer)
    const bool inner = LMSF_P2_INNER && fine;
    if (inner) dense_ball_walk(g, w, bound * kDenseCull, k);
    const float4* rp = g.pts;
    const int nrows = fine ? 25 : 9;
    const DenseQuery<2> dq(g, w);   // the 1 m grid's 3 x 3 rows are its inner ring
    const int xa = dq.xa, xb = dq.xb;
#pragma unroll 1
    for (int i = inner ? 9 : 0; i < nrows; ++i) {
        const float d4 = fminf(bound, key_d2(k[NK - 1]));
        const uint32_t* row;
        int sa, sb;
        const int dyo = fine ? kRing5[i][0] : (kDenseRowOrder[i] % 3) - 1;
        const int dzo = fine ? kRing5[i][1] : (kDenseRowOrder[i] / 3) - 1;
        const float lb = dq.lb(dyo, dzo);
        if (lb > d4) continue;   // ahead of the row's address and offsets
        if (!dq.row(g, dyo, dzo, row)) continue;
        dense_window(g, w, d4 * kDenseCull, lb, xa, xb, sa, sb);
        if (sa > sb) continue;
        const uint32_t a = row[sa];
        dense_run(k, rp, a, row[sb + 1] - a, w);
    }
    return g;
}

// LMSF_P2_SPLITFIT: pass 2 as a walk kernel (no fit: few registers, more waves to hide its row-by-row offset
// latency; the kept 5 indices left in the position's memo record) and a fit kernel over the same list.
// (r05: a team of 2 / 4 / 8 lanes per listed query -- rows dealt to the lanes, the team's bound shared after every
// step -- measured 4,052 / 3,975 / 3,784 vs 4,163 C5 pairs/s for one lane: the shared bound prunes later than one
// lane's own key, and the extra lanes walk rows one lane never enters.  Not kept.)
#ifndef LMSF_P2_SPLITFIT
#define LMSF_P2_SPLITFIT 1
#endif
#ifndef LMSF_P2_WALK_WAVES
#define LMSF_P2_WALK_WAVES 6
#endif
// wl / wlim: the pass-2 list (bv.wl / bv.wlim, or bv.wl2 / bv.wlim2 in the memo iterations, whose per-scan lists
// occupy wl), p2count entries.
template <bool FIT, int NK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FIT ? 3 : LMSF_P2_WALK_WAVES))) void dense_pass2_kernel(
    GridView ge, GridView gs, GridView fe, GridView fs, BatchView bv, const unsigned* p2count, const int* wl,
    const float* wlim) {
    const unsigned count = *p2count;
    const size_t F = bv.feat_stride;
    for (unsigned li = blockIdx.x * 256 + threadIdx.x; li < count; li += gridDim.x * 256) {
        const size_t code = (size_t)(unsigned)wl[li];
        const float bound = wlim[li];
        const int b = (int)(code / F), e = (int)(code - (size_t)b * F);
        const int ne = bv.n_edge[b];
        const size_t ppos = (size_t)b * F + e;
        const float4 p = bv.featp[ppos];
        const int qq = __float_as_int(p.w);
        const bool is_edge = qq < ne;
        const float3 w = associate(load_pose(bv.st[b].x), p);
        double k[NK];
        const GridView g = dense_bounded_walk<NK>(ge, gs, fe, fs, is_edge, w, bound, k);
        if constexpr (FIT) {
            double k5[5];
            first5(k, k5);
            dense_finish(g, bv, ppos, p, is_edge, (size_t)b * F + qq, w, k5);
        } else {   // the kept indices (-1: none) for the fit kernel, in key order
            store_kept(bv, b, e, F, k);
        }
        if constexpr (NK == 6) store_anchor(bv, b, e, F, w, k);   // the same 5 indices, then s6 and the gaps
    }
}

// The fit of dense_pass2_kernel<false>'s queries (same list, same order): the kept 5 from the memo record.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void dense_fit2_kernel(
    GridView ge, GridView gs, BatchView bv, const unsigned* p2count, const int* wl) {
    const unsigned count = *p2count;
    const size_t F = bv.feat_stride;
    for (unsigned li = blockIdx.x * 256 + threadIdx.x; li < count; li += gridDim.x * 256) {
        const size_t code = (size_t)(unsigned)wl[li];
        const int b = (int)(code / F), e = (int)(code - (size_t)b * F);
        const int ne = bv.n_edge[b];
        const size_t ppos = (size_t)b * F + e;
        const float4 p = bv.featp[ppos];
        const int qq = __float_as_int(p.w);
        const bool is_edge = qq < ne;
        const GridView g = pick_grid(is_edge, ge, gs);   // orig: the caller-order map either way
        const float3 w = associate(load_pose(bv.st[b].x), p);
        int kid[5];
        if constexpr (kMemoAos) {
            const int* mp = bv.memo_nbr + memo_idx(b, 0, e, F);
            const int4 m0 = *reinterpret_cast<const int4*>(mp);
            kid[0] = m0.x; kid[1] = m0.y; kid[2] = m0.z; kid[3] = m0.w; kid[4] = mp[4];
        } else {
#pragma unroll
            for (int j = 0; j < 5; ++j) kid[j] = bv.memo_nbr[memo_idx(b, j, e, F)];
        }
        double k[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) k[j] = kid[j] >= 0 ? key_as_double((uint64_t)(uint32_t)kid[j]) : key_as_double(kSentinel);
        dense_finish(g, bv, ppos, p, is_edge, (size_t)b * F + qq, w, k);
    }
}

// ---------------------------------------------------------------- dense maps: the query memo (r05)
// VERDICT r04 #3b: C5 re-associated every feature in all 5 outer iterations.  tools/memo_model.py C5 (oracle kd-tree
// + Ceres trace on one C5 scan): the memo test serves 33% of the queries in outer iteration 2 (reuse 12%, refit 21%),
// 91% in 3 and 99% in 4, and the misses' bounded re-search (radius s6 + d) holds ~6-7 candidates against ~12-14 in
// pass 1's first-pass ball.  So on dense maps too: outer iteration memo_from - 1 runs the two passes with 6 exact keys
// and leaves every position's anchor (store_anchor, the sparse memo's record); iterations >= memo_from run
// match_memo_kernel (unchanged: it reads only the anchors and the records by position), then this kernel over the
// scan's lists: searches walk the first-pass grid's rows bounded by min(1 m, s6 + d) (dense_bounded_walk, 6 keys --
// exact, the 6 nearest at w0 lie within s6 + d of w), refresh the anchor and fit; refits fit the reordered stored 5.
// Records by search position, as every dense pass.
// Grid (G, B): blockIdx.y = scan, its G blocks grid-stride over the scan's lists (r05 first form: one block per 256
// positions, gx * B = 256k blocks on C5, most of them empty past iteration 2 -- ~2 ms per dispatch of block
// launches alone).  As pass 2, a walk kernel (few registers: more waves to hide the walk's latency; the kept 5 and
// the refreshed anchor left in the position's memo record) and a fit kernel over the searches and the refits
// (LMSF_MEMO_SPLITFIT; 0: one kernel, fit inline).
#ifndef LMSF_MEMO_SPLITFIT
#define LMSF_MEMO_SPLITFIT 0
#endif
template <bool FIT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FIT ? 3 : LMSF_P2_WALK_WAVES))) void dense_memo_search_kernel(
    GridView ge, GridView gs, GridView fe, GridView fs, BatchView bv) {
    const int b = blockIdx.y;
    const size_t F = bv.feat_stride;
    const int* cnt = bv.wcount + (size_t)b * memo_blocks(F);
    const int total_s = cnt[0], total = total_s + cnt[1];
    if (blockIdx.x == 0 && threadIdx.x == 0) bv.n_search[b] = total;
    const int ne = bv.n_edge[b];
    const Pose P = load_pose(bv.st[b].x);
    for (int e = blockIdx.x * 256 + threadIdx.x; e < (FIT ? total : total_s); e += gridDim.x * 256) {
        const bool walk = e < total_s;
        const int pos = walk ? bv.wl[(size_t)b * F + e] : bv.wl[(size_t)b * F + F - 1 - (e - total_s)];
        const size_t ppos = (size_t)b * F + pos;
        const float4 p = bv.featp[ppos];
        const int qq = __float_as_int(p.w);
        const bool is_edge = qq < ne;
        const float3 w = associate(P, p);
        if (walk) {
            double k[6];
            const GridView g = dense_bounded_walk<6>(ge, gs, fe, fs, is_edge, w, bv.wlim[(size_t)b * F + e], k);
            if constexpr (FIT) {
                store_anchor(bv, b, pos, F, w, k);
                double k5[5];
                first5(k, k5);
                dense_finish(g, bv, ppos, p, is_edge, (size_t)b * F + qq, w, k5);
            } else {
                store_kept(bv, b, pos, F, k);        // -1s when fewer than 5 were found
                store_anchor(bv, b, pos, F, w, k);   // the same 5 indices, then s6 and the gaps
            }
        } else if constexpr (FIT) {   // refit: the memo pass left the 5 neighbours in their order at w
            double k5[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) k5[j] = key_as_double((uint64_t)(uint32_t)bv.memo_nbr[memo_idx(b, j, pos, F)]);
            dense_finish(pick_grid(is_edge, ge, gs), bv, ppos, p, is_edge, (size_t)b * F + qq, w, k5);
        }
    }
}

// The fit of dense_memo_search_kernel<false>'s searches and of the memo pass's refits: the 5 from the memo record.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void dense_memo_fit_kernel(GridView ge,
                                                                                                    GridView gs,
                                                                                                    BatchView bv) {
    const int b = blockIdx.y;
    const size_t F = bv.feat_stride;
    const int* cnt = bv.wcount + (size_t)b * memo_blocks(F);
    const int total_s = cnt[0], total = total_s + cnt[1];
    const int ne = bv.n_edge[b];
    const Pose P = load_pose(bv.st[b].x);
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
        const int pos = e < total_s ? bv.wl[(size_t)b * F + e] : bv.wl[(size_t)b * F + F - 1 - (e - total_s)];
        const size_t ppos = (size_t)b * F + pos;
        const float4 p = bv.featp[ppos];
        const int qq = __float_as_int(p.w);
        const bool is_edge = qq < ne;
        int kid[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) kid[j] = bv.memo_nbr[memo_idx(b, j, pos, F)];
        double k5[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) k5[j] = kid[j] >= 0 ? key_as_double((uint64_t)(uint32_t)kid[j]) : key_as_double(kSentinel);
        dense_finish(pick_grid(is_edge, ge, gs), bv, ppos, p, is_edge, (size_t)b * F + qq, associate(P, p), k5);
    }
}

// LMSF_MEMO_PASS1 (default 1): the memo pass's listed searches run pass 1 (the first-pass ball, 9 rows resolved up
// front, 6 keys) instead of the walk bounded by min(1 m, s6 + d): a query the ball completes (6th key within lim1) is
// fitted and re-anchored here, the rest go to the pass-2 list in wl2 (bounded by the smaller of its 6th key and
// s6 + d, both at least the true 6th); refits are fitted from the memo record.  (r05: the s6 + d walk took ~2x pass
// 1's time per query -- its balls are larger than the first-pass ball.)
#ifndef LMSF_MEMO_PASS1
#define LMSF_MEMO_PASS1 1
#endif
// The scans' lists flattened: a block first scans the B lists' lengths into LDS (s_pre, B + 1 ints of dynamic LDS),
// then grid-strides over all entries (r05 first form: G blocks per scan, so the scan with the longest list --
// the pair that moved most -- set the kernel's length: ~2x pass 1's time per entry).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LMSF_FUSED_WAVES))) void dense_pass1_listed_kernel(
    GridView ge, GridView gs, GridView fe, GridView fs, BatchView bv, unsigned* p2count) {
    extern __shared__ int s_pre[];
    __shared__ int s_wave[4];
    const size_t F = bv.feat_stride;
    const int B = bv.B;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // s_pre[b] = entries of the lists before scan b, 256 scans per round
    int run = 0;
    for (int b0 = 0; b0 < B; b0 += 256) {
        const int b = b0 + threadIdx.x;
        int c = 0;
        if (b < B) {
            const int* cnt = bv.wcount + (size_t)b * memo_blocks(F);
            c = cnt[0] + cnt[1];
            if (blockIdx.x == 0) bv.n_search[b] = c;
        }
        int inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(inc, o, 64);
            if (lane >= o) inc += t;
        }
        if (lane == 63) s_wave[wave] = inc;
        __syncthreads();
        int before = run;
#pragma unroll
        for (int w4 = 0; w4 < 4; ++w4) before += w4 < wave ? s_wave[w4] : 0;
        if (b < B) s_pre[b] = before + inc - c;
        run += s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
        __syncthreads();
    }
    if (threadIdx.x == 0) s_pre[B] = run;
    __syncthreads();
    const int total_all = s_pre[B];
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int g_e = blockIdx.x * 256 + threadIdx.x; g_e < total_all; g_e += gridDim.x * 256) {
        int lo = 0, hi = B - 1;   // the last scan whose entries start at or before g_e
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_pre[mid] <= g_e) lo = mid;
            else hi = mid - 1;
        }
        const int b = lo, e = g_e - s_pre[b];
        const int total_s = bv.wcount[(size_t)b * memo_blocks(F)];
        const bool walk = e < total_s;
        const int pos = walk ? bv.wl[(size_t)b * F + e] : bv.wl[(size_t)b * F + F - 1 - (e - total_s)];
        const size_t ppos = (size_t)b * F + pos;
        const float4 p = bv.featp[ppos];
        const int qq = __float_as_int(p.w);
        const bool is_edge = qq < bv.n_edge[b];
        const float3 w = associate(load_pose(bv.st[b].x), p);
        const GridView g = pick_grid(is_edge, pick_grid(fe.n > 0, fe, ge), pick_grid(fs.n > 0, fs, gs));
        double k[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) k[j] = key_as_double(kSentinel);
        bool p2 = false;
        if (walk) {
            unsigned int c27 = 0;
            dense_first_pass(g, w, 0, k, c27);
            p2 = key_d2(k[5]) > g.lim1;
        } else {   // refit: the memo pass left the 5 neighbours in their order at w (key bits: index only)
#pragma unroll
            for (int j = 0; j < 5; ++j) k[j] = key_as_double((uint64_t)(uint32_t)bv.memo_nbr[memo_idx(b, j, pos, F)]);
        }
        // the incomplete searches to the pass-2 list (one atomic per wave: its first active lane)
        const unsigned long long act = __ballot(1), m2 = __ballot(p2);
        const int leader = __ffsll((long long)act) - 1;
        int base2 = 0;
        if (lane == leader && m2) base2 = (int)atomicAdd(p2count, (unsigned)__popcll(m2));
        base2 = __shfl(base2, leader, 64);
        if (p2) {
            const int at = base2 + __popcll(m2 & below);
            bv.wl2[at] = (int)ppos;
            bv.wlim2[at] = fminf(key_d2(k[5]), bv.wlim[(size_t)b * F + e]);
        } else {
            if (walk) store_anchor(bv, b, pos, F, w, k);
            double k5[5];
            first5(k, k5);
            dense_finish(g, bv, ppos, p, is_edge, (size_t)b * F + qq, w, k5);
        }
    }
}

// LM candidate evaluation over the fixed correspondences (Ceres re-evaluates the same residual blocks
// at every trial point): one packet per block; the step runs in lm_step_kernel (k_solver.hip).
// kEvalPerThread records per thread.  (Fusing the step into the last block to finish, behind an
// agent-scope ticket with sc1 packet stores, measured slower in r02 on C2 / C3 / C4 -- 20.9k vs 22.1k
// scans/s, 1.95 vs 1.73 ms per C3 frame, 2.12 vs 2.05 ms per C4 scan: the step code capped the
// kernel at 128 VGPRs and its serial step lands on the launch's tail -- and was removed.)
// Records per thread / occupancy (A/B, r02, tools/gpu_eval_ab.sh, C2 512 x 4): 4 records at 4 waves
// (124 VGPRs) 22.69k scans/s; 2 records at 5 waves (96) 21.67-21.86k; 1 record at 6 waves (79) 21.03k --
// fewer bytes in flight per lane and more block packets lose more than the occupancy gains.
#ifndef LMSF_EVAL_WAVES   // waves per SIMD lm_eval_kernel is compiled for (A/B)
#define LMSF_EVAL_WAVES 4
#endif
template <bool COUNT = false>
__device__ __forceinline__ void eval_record(const Pose& Ps, bool valid, const float4 rp, const RecV& v, const double2 e,
                                            double* P) {
    const int kind = __float_as_int(rp.w);
    if (COUNT) {   // match counts (fit_query's P[29] / P[30])
        P[29] += valid && kind == LMSF_EDGE ? 1.0 : 0.0;
        P[30] += valid && kind == LMSF_SURF ? 1.0 : 0.0;
    }
    if (valid && kind != 0) {
        double J[6], res;
        const d3 pp = mk((double)rp.x, (double)rp.y, (double)rp.z);
        if (kind == LMSF_EDGE)
            res = edge_residual(Ps, pp, mk(v.v[0], v.v[1], v.v[2]), mk(v.v[3], e.x, e.y), J);
        else
            res = surf_residual(Ps, pp, mk(v.v[0], v.v[1], v.v[2]), v.v[3], J);
        huber_accumulate(P, res, J);
    }
}

// LIN: the evaluation at the linearisation pose x of the batch path (after the matching; lm_begin reduces
// its packets, match counts included); else at the LM candidate xc of slots that need one.
template <bool LIN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LMSF_EVAL_WAVES))) void lm_eval_kernel(BatchView bv) {
    const int b = blockIdx.y;
    const int nq = bv.n_edge[b] + bv.n_surf[b];
    if (blockIdx.x * kEvalBlock >= nq) return;
    if (!LIN && !bv.st[b].need_eval) return;
    const Pose Ps = load_pose(LIN ? bv.st[b].x : bv.st[b].xc);
    double P[kPacket];
#pragma unroll
    for (int i = 0; i < kPacket; ++i) P[i] = 0.0;
    const size_t base = (size_t)b * bv.feat_stride;
    const int q0 = blockIdx.x * kEvalBlock + threadIdx.x;
    const int ne = bv.n_edge[b];
    auto loc_of = [&](int k) { return q0 + k * 256 < nq ? q0 + k * 256 : 0; };
    auto slot_of = [&](int k) { return base + loc_of(k); };
    auto rec_of = [&](int k, RecV& v) { return load_record(bv, slot_of(k), loc_of(k), ne, v); };
#if LMSF_EVAL_PIPE
    // Software pipeline, one record per step: rec_p / rec_v of record k + 2 and rec_e of record k + 1
    // (edges only; its kind arrived a step earlier) are in flight while record k is evaluated.
    const double2 ez = make_double2(0.0, 0.0);
    RecV v0, v1;
    float4 p0 = rec_of(0, v0), p1 = p0;
    v1 = v0;
    if (kEvalPerThread > 1) p1 = rec_of(1, v1);
    double2 e0 = __float_as_int(p0.w) == LMSF_EDGE ? bv.rec_e[slot_of(0)] : ez;
#pragma unroll
    for (int k = 0; k < kEvalPerThread; ++k) {
        float4 pn = p1;
        RecV vn = v1;
        if (k + 2 < kEvalPerThread) pn = rec_of(k + 2, vn);
        double2 en = ez;
        if (k + 1 < kEvalPerThread && __float_as_int(p1.w) == LMSF_EDGE) en = bv.rec_e[slot_of(k + 1)];
        eval_record<LIN>(Ps, q0 + k * 256 < nq, p0, v0, e0, P);
        p0 = p1; v0 = v1; e0 = en;
        p1 = pn; v1 = vn;
    }
#else
    float4 rp[kEvalPerThread];
    RecV rv[kEvalPerThread];
#pragma unroll
    for (int k = 0; k < kEvalPerThread; ++k) rp[k] = rec_of(k, rv[k]);
#pragma unroll
    for (int k = 0; k < kEvalPerThread; ++k) {
        const bool edge = __float_as_int(rp[k].w) == LMSF_EDGE;
        eval_record<LIN>(Ps, q0 + k * 256 < nq, rp[k], rv[k], edge ? bv.rec_e[slot_of(k)] : make_double2(0.0, 0.0), P);
    }
#endif
    block_reduce_packet(P, bv.partials + ((size_t)b * bv.max_parts + blockIdx.x) * kPacket);
}

// ---------------------------------------------------------------- single-scan LM loop in one launch
// The Ceres LM of one outer iteration (lm_begin + 4 x (lm_eval + lm_step), 9 launches) as one launch for
// contexts whose whole grid is co-resident (tracking: one scan, 128 blocks for 64k feature slots; kLoopMaxBlocks).  Every block keeps
// its own LDS copy of the slot's SolveState and runs the one-lane control on identical inputs (the same
// packets summed in the same order), so all copies stay equal and no block waits for another's step: a
// block evaluates its kLoopBlock records at the candidate, publishes its packet, and one arrive / wait on a
// per-slot counter later every block reduces every packet itself.
//
// Cross-block visibility (MI355X_MICROARCH.md, correctness boundaries: per-XCD L2s are not coherent):
// packets are stored and loaded with agent-scope atomic accesses (write-through / L2-bypassing), every
// storing wave drains its stores before the block's barrier, and the counter is an agent-scope atomic.
// Packets alternate between two buffers by inner iteration, so a block that runs ahead cannot overwrite a
// packet another block still reads.  Every wait is bounded: a block that spins past the limit flags
// err[0] and leaves (the host reports LMSF_ERR_HIP), so no configuration can hang the device.
// sync[2 b] counts arrivals of slot b across launches; sync[2 b + 1] holds the count at the start of the
// next launch (written by block 0 after the last wait of this one).


// Every block of the slot arrives once; returns when all nblk of this barrier have (count reaches target).
__device__ __forceinline__ void slot_barrier(unsigned* cnt, unsigned target, int* err, unsigned spin_limit) {
    __builtin_amdgcn_s_waitcnt(0);   // this wave's packet stores are complete
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while ((int)(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > spin_limit) {
                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

// The packets [p0, p0 + np) of slot b summed in a fixed order into tot (LDS; the same in every block).
__device__ void reduce_coherent(const BatchView& bv, int b, int p0, int np, double* tot) {
    __shared__ double red[4][kPacket];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, e = lane & 31;
    const double* base = bv.partials + ((size_t)b * bv.max_parts + p0) * kPacket;
    // kLoads loads in flight per lane (the packets of one launch: <= 8 * kLoads), summed in a fixed order
    constexpr int kLoads = kLoopMaxBlocks / 8;
    double v[kLoads];
    const int pl = 2 * wave + (lane >> 5);
#pragma unroll
    for (int u = 0; u < kLoads; ++u) {
        const int p = pl + 8 * u;
        v[u] = p < np ? coherent_load_f64(base + (size_t)p * kPacket + e) : 0.0;
    }
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < kLoads; ++u) acc += v[u];
    acc += __shfl_xor(acc, 32, 64);
    if (lane < 32) red[wave][e] = acc;
    __syncthreads();
    if (threadIdx.x < kPacket) {
        const int i = threadIdx.x;
        tot[i] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
    }
    __syncthreads();
}

// LMSF_LOOP_CTL_WAVE: the LM control of the single-scan loop on wave 0 (lm_control.h wv::, bit-identical) instead
// of one lane.
#ifndef LMSF_LOOP_CTL_WAVE
#define LMSF_LOOP_CTL_WAVE 1
#endif
constexpr bool kLoopCtlWave = LMSF_LOOP_CTL_WAVE != 0;
__global__ __launch_bounds__(256) void lm_loop_kernel(BatchView bv, int outer, unsigned* sync, int* err,
                                                      unsigned spin_limit) {
    stamp_if(bv.stamp_end, blockIdx.x == 0 && blockIdx.y == 0);   // the search launch before it has drained
    const int b = blockIdx.y, part = blockIdx.x, nblk = gridDim.x;
    __shared__ SolveState sS;
    __shared__ double tot[kPacket];
#ifdef LMSF_STEP_PROFILE   // diagnostics build (tools/build_variant.sh): phase stamps of slot 0, first and last block
    unsigned long long tp[24];
    int ntp = 0;
    const bool prof = b == 0 && (part == 0 || part == nblk - 1) && threadIdx.x == 0;
#define LOOP_STAMP() do { if (prof && ntp < 24) tp[ntp++] = wall_clock64(); } while (0)
#else
#define LOOP_STAMP() do {} while (0)
#endif
    LOOP_STAMP();
    state_copy(sS, bv.st[b]);
    const int nq = bv.n_edge[b] + bv.n_surf[b];
    // lm_begin: the first evaluation's packets (fit_eval), IterationZero and the first step
    reduce_parts(bv, b, (nq + bv.part_q - 1) / bv.part_q, tot);   // ends with a barrier: sS is in place
    LOOP_STAMP();
    if constexpr (kLoopCtlWave) {
        if (threadIdx.x < 64) wv::lm_begin(sS, tot);
    } else if (threadIdx.x == 0) {
        lm_begin_apply(sS, tot);
    }
    __syncthreads();
    LOOP_STAMP();
    const unsigned base = sync[2 * b + 1];
    unsigned nbar = 0;
    const int pbuf = bv.max_parts / 2;   // packet buffers [pbuf, pbuf + 2 nblk): above the fit packets
    const size_t rbase = (size_t)b * bv.feat_stride;
    for (int i = 0; i < 4; ++i) {
        const int last = i == 3 ? 1 : 0;
        if (!sS.need_eval) {
            if (last && threadIdx.x == 0) finish_outer(sS, outer);
            __syncthreads();
            continue;
        }
        const Pose Ps = load_pose(sS.xc);
        double P[kPacket];
#pragma unroll
        for (int k = 0; k < kPacket; ++k) P[k] = 0.0;
        // lm_eval_kernel's form: the records' loads in flight together, then evaluated
        const int q0 = part * kLoopBlock + threadIdx.x;
        auto loc_at = [&](int k) { return q0 + k * 256 < nq ? q0 + k * 256 : 0; };
        auto rec_at = [&](int k) { return rbase + loc_at(k); };
        float4 rp[kLoopPerThread];
        RecV rv[kLoopPerThread];
#pragma unroll
        for (int k = 0; k < kLoopPerThread; ++k) rp[k] = load_record(bv, rec_at(k), loc_at(k), bv.n_edge[b], rv[k]);
#pragma unroll
        for (int k = 0; k < kLoopPerThread; ++k) {
            const bool edge = __float_as_int(rp[k].w) == LMSF_EDGE;
            eval_record(Ps, q0 + k * 256 < nq, rp[k], rv[k], edge ? bv.rec_e[rec_at(k)] : make_double2(0.0, 0.0), P);
        }
        double* slotp = bv.partials + ((size_t)b * bv.max_parts + pbuf + (i & 1) * nblk + part) * kPacket;
        {   // block packet (block_reduce_packet's order), stored write-through
            __shared__ double red[4][kPacket];
            const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
            butterfly_step<16>(P, lane);
            butterfly_step<8>(P, lane);
            butterfly_step<4>(P, lane);
            butterfly_step<2>(P, lane);
            butterfly_step<1>(P, lane);
            const double v = P[0] + __shfl_xor(P[0], 1, 64);
            if ((lane & 1) == 0) red[wave][lane >> 1] = v;
            __syncthreads();
            if (threadIdx.x < kPacket) {
                const int e = threadIdx.x;
                coherent_store_f64(slotp + e, ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e]);
            }
        }
        LOOP_STAMP();
        ++nbar;
        slot_barrier(&sync[2 * b], base + nbar * (unsigned)nblk, err, spin_limit);
        LOOP_STAMP();
        reduce_coherent(bv, b, pbuf + (i & 1) * nblk, nblk, tot);
        LOOP_STAMP();
        if constexpr (kLoopCtlWave) {
            if (threadIdx.x < 64) wv::lm_step(sS, tot, outer, last);
        } else if (threadIdx.x == 0) {
            lm_step_apply(sS, tot, outer, last);
        }
        __syncthreads();
        LOOP_STAMP();
    }
    if (nbar == 0) {   // no wait yet: make sure every block has read st before block 0 rewrites it
        ++nbar;
        slot_barrier(&sync[2 * b], base + nbar * (unsigned)nblk, err, spin_limit);
    }
    if (part == 0) {
        state_copy(bv.st[b], sS);
        if (threadIdx.x == 0) sync[2 * b + 1] = base + nbar * (unsigned)nblk;
    }
#ifdef LMSF_STEP_PROFILE
    if (prof) {   // x10 ns: begin reduce, begin apply, then per inner iteration eval, barrier, reduce, step
        unsigned d[18];
        for (int j = 0; j < 18; ++j) d[j] = j + 1 < ntp ? (unsigned)(tp[j + 1] - tp[j]) : 0u;
        printf("lm_loop o%d blk%d/%d nq %d: %u %u | %u %u %u %u | %u %u %u %u | %u %u %u %u | %u %u %u %u\n", outer, part,
               nblk, nq, d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], d[10], d[11], d[12], d[13], d[14],
               d[15], d[16], d[17]);
    }
#endif
#undef LOOP_STAMP
}

int lm_loop_blocks(const BatchView& bv) { return (bv.feat_stride + kLoopBlock - 1) / kLoopBlock; }

hipError_t launch_lm_loop(const BatchView& bv, int outer, unsigned* sync, int* err, unsigned spin_limit,
                          hipStream_t s) {
    hipLaunchKernelGGL(lm_loop_kernel, dim3(lm_loop_blocks(bv), bv.B), dim3(256), 0, s, bv, outer, sync, err,
                       spin_limit);
    return hipGetLastError();
}

// Diagnostics: evaluate slot 0's records at an arbitrary pose into partials of slot 0.
__global__ __launch_bounds__(256) void eval_at_kernel(BatchView bv, const double* pose) {
    const int nq = bv.n_edge[0] + bv.n_surf[0];
    if (blockIdx.x * kEvalBlock >= nq) return;
    const Pose Ps = load_pose(pose);
    double P[kPacket];
#pragma unroll
    for (int i = 0; i < kPacket; ++i) P[i] = 0.0;
#pragma unroll
    for (int k = 0; k < kEvalPerThread; ++k) {
        const int q = blockIdx.x * kEvalBlock + k * 256 + threadIdx.x;
        if (q < nq) {
            double J[6], res;
            if (record_residual(bv, (size_t)q, q, bv.n_edge[0], Ps, res, J)) huber_accumulate(P, res, J);
        }
    }
    block_reduce_packet(P, bv.partials + (size_t)blockIdx.x * kPacket);
}

// Record capture (diagnostics, lmsf_batch_capture): one lane per search position (by_pos: records stored
// by position, featp w = its slot) or slot; the record goes out in slot order in the lmsf_record layout
// lmsf_match returns (value fields of unmatched records zero), with the 5 neighbour indices of nnp.
__global__ __launch_bounds__(256) void capture_kernel(BatchView bv, int b, int by_pos, lmsf_record* out, int32_t* nn,
                                                      double* pose) {
    if (blockIdx.x == 0 && threadIdx.x < 7) pose[threadIdx.x] = bv.st[b].x[threadIdx.x];
    const int nq = bv.n_edge[b] + bv.n_surf[b];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nq) return;
    const size_t pos = (size_t)b * bv.feat_stride + i;
    const int q = by_pos ? __float_as_int(bv.featp[pos].w) : i;
    if (q < 0 || q >= nq) return;
    RecV v;
    const float4 p = load_record(bv, pos, i, bv.n_edge[b], v);
    lmsf_record r;
    r.px = p.x;
    r.py = p.y;
    r.pz = p.z;
    r.kind = __float_as_int(p.w);
    r.v0[0] = r.v0[1] = r.v0[2] = 0.0;
    r.v1[0] = r.v1[1] = r.v1[2] = 0.0;
    if (r.kind != 0) {
        r.v0[0] = v.v[0];
        r.v0[1] = v.v[1];
        r.v0[2] = v.v[2];
        r.v1[0] = v.v[3];
        if (r.kind == LMSF_EDGE) {
            const double2 e = bv.rec_e[pos];
            r.v1[1] = e.x;
            r.v1[2] = e.y;
        }
    }
    out[q] = r;
    const float4* np = bv.nnp + ((size_t)b * bv.feat_stride + q) * 5;
#pragma unroll
    for (int j = 0; j < 5; ++j) nn[(size_t)q * 5 + j] = __float_as_int(np[j].w);
}

hipError_t launch_capture(const BatchView& bv, int b, int by_pos, lmsf_record* rec, int32_t* nn, double* pose,
                          hipStream_t s) {
    const dim3 grid((bv.feat_stride + 255) / 256);
    hipLaunchKernelGGL(capture_kernel, grid, dim3(256), 0, s, bv, b, by_pos, rec, nn, pose);
    return hipGetLastError();
}

// Team size and XCD remap are tunables (LMSF_KNN_TEAM = 1 | 2 | 4 | 8 | 16 | 32, LMSF_XCD_REMAP =
// 0 | 1) for A/B measurement.  Default (measured, r01): one lane per query when a launch carries
// >= 2^20 query slots (C2 batch of 64: 10.8k scans/s vs 7.1k at T = 8); 8 lanes per query for
// single-scan tracking launches (63k queries: knn 234 -> 75 us on the 5M-point C4 map, 56 -> 27
// us on the C3 local map), where one lane per query leaves most of the chip idle.
static int knn_team(size_t query_slots) {
    static int forced = [] {
        const int v = ab_int("LMSF_KNN_TEAM", 0);
        return (v == 1 || v == 2 || v == 4 || v == 8 || v == 16 || v == 32) ? v : 0;
    }();
    if (forced) return forced;
    return query_slots >= ((size_t)1 << 20) ? 1 : 8;
}
int knn_team_for(size_t query_slots) { return knn_team(query_slots); }

static int knn_remap() {
    static int r = ab_int("LMSF_XCD_REMAP", 1);
    return r;
}

template <bool TWO>
static void launch_knn_t(int T, bool prune, bool memo, dim3 grid, const GridView& edge, const GridView& surf,
                         const GridView& edge2, const GridView& surf2, const BatchView& bv, int skip_converged, int gx,
                         int remap, hipStream_t s) {
#define LMSF_KNN(TT, PP) hipLaunchKernelGGL((knn_kernel<TT, TWO, PP>), grid, dim3(256), 0, s, edge, surf, edge2, surf2, bv, \
                                            skip_converged, gx, remap)
    // The memo team walk on dense maps: pruned with LMSF_TEAM_PRUNE=1 (A/B; exact, but C4's search launch took 54.6-58
    // vs 52 us unpruned at first-pass radii of 1-8 x lim1: the walks shortened -- slowest team 22-28 vs 34-48 us,
    // r05 block stamps -- but the launch is set by its blocks' start beside the concurrent extraction and by the
    // memo / row-resolution latencies both forms share).
    if (memo && T == 8) {
        static const bool team_prune = ab_int("LMSF_TEAM_PRUNE", 0) != 0;
        if (prune && team_prune)
            hipLaunchKernelGGL((knn_kernel<8, TWO, true, true>), grid, dim3(256), 0, s, edge, surf, edge2, surf2, bv,
                               skip_converged, gx, remap);
        else
            hipLaunchKernelGGL((knn_kernel<8, TWO, false, true>), grid, dim3(256), 0, s, edge, surf, edge2, surf2, bv,
                               skip_converged, gx, remap);
        return;
    }
    switch (T) {
        case 1:
            if (prune)
                LMSF_KNN(1, true);
            else
                LMSF_KNN(1, false);
            break;
        case 2: LMSF_KNN(2, false); break;
        case 4: LMSF_KNN(4, false); break;
        case 8: LMSF_KNN(8, false); break;
        case 32: LMSF_KNN(32, false); break;
        default: LMSF_KNN(16, false); break;
    }
#undef LMSF_KNN
}

// Outer iteration 0 of a single-scan Solve on a prior + window map in two launches (knn_kernel SPLIT): pass 1
// (prior grids edge / surf) or pass 2 (windows edge2 / surf2, seeded from pass 1's keys).  8-lane teams, memo form.
hipError_t launch_knn_split(int pass, const GridView& edge, const GridView& surf, const GridView& edge2,
                            const GridView& surf2, const BatchView& bv, hipStream_t s) {
    const int T = 8, remap = knn_remap();
    const int span = (bv.qslot && bv.pos_stride > bv.feat_stride) ? bv.pos_stride : bv.feat_stride;
    const int gx = (span + (256 / T) - 1) / (256 / T);
    const dim3 grid(gx * bv.B);
    if (pass == 1)
        hipLaunchKernelGGL((knn_kernel<8, false, false, true, 1>), grid, dim3(256), 0, s, edge, surf, edge2, surf2, bv, 0,
                           gx, remap);
    else
        hipLaunchKernelGGL((knn_kernel<8, false, false, true, 2>), grid, dim3(256), 0, s, edge, surf, edge2, surf2, bv, 0,
                           gx, remap);
    return hipGetLastError();
}

hipError_t launch_knn(const GridView& edge, const GridView& surf, const GridView& edge2, const GridView& surf2,
                      const BatchView& bv, int skip_converged, hipStream_t s, bool memo) {
    const int T = knn_team((size_t)bv.feat_stride * bv.B), remap = knn_remap();
    const int span = (bv.qslot && bv.pos_stride > bv.feat_stride) ? bv.pos_stride : bv.feat_stride;
    const int gx = (span + (256 / T) - 1) / (256 / T);
    const dim3 grid(gx * bv.B);
    // the pruned walk when a searched grid is dense (first-pass radius below the match radius)
    const bool prune = (edge.n > 0 && edge.lim1 < 1.f) || (surf.n > 0 && surf.lim1 < 1.f);
    if (edge2.n > 0 || surf2.n > 0)
        launch_knn_t<true>(T, prune, memo, grid, edge, surf, edge2, surf2, bv, skip_converged, gx, remap, s);
    else
        launch_knn_t<false>(T, prune, memo, grid, edge, surf, edge2, surf2, bv, skip_converged, gx, remap, s);
    return hipGetLastError();
}

hipError_t launch_fit_eval(const GridView& edge, const GridView& surf, const BatchView& bv, int solver,
                           hipStream_t s) {
    (void)edge;
    (void)surf;
    const int per_block = 256 * bv.fit_per_thread;
    dim3 grid((bv.feat_stride + per_block - 1) / per_block, bv.B);
    switch (bv.fit_per_thread) {
        case 1: hipLaunchKernelGGL(fit_eval_kernel<1>, grid, dim3(256), 0, s, bv, solver); break;
        case 2: hipLaunchKernelGGL(fit_eval_kernel<2>, grid, dim3(256), 0, s, bv, solver); break;
        default: hipLaunchKernelGGL(fit_eval_kernel<4>, grid, dim3(256), 0, s, bv, solver); break;
    }
    return hipGetLastError();
}

// Queries per thread of fit_eval (LMSF_FIT_PER_THREAD = 1 | 2 | 4, for A/B measurement).  1 (107
// VGPRs, 4 waves/SIMD) since the butterfly packet reduction: C2 16.8k vs 16.5k scans/s at 2 (165 VGPRs).
int fit_per_thread_default() {
    static int v = [] {
        const int x = ab_int("LMSF_FIT_PER_THREAD", 1);
        return (x == 1 || x == 2 || x == 4) ? x : 1;
    }();
    return v;
}

// LMSF_FUSED = 0 | 1 (A/B builds): the fused search + fit for batch launches (default 1).
static bool fused_enabled() {
    static bool v = ab_int("LMSF_FUSED", 1) != 0;
    return v;
}

bool match_fit_applies(const GridView& edge2, const GridView& surf2, const BatchView& bv, int solver) {
    return fused_enabled() && solver == LMSF_SOLVER_CERES_LM && bv.fslot != nullptr && edge2.n == 0 && surf2.n == 0 &&
           bv.fit_per_thread == 1 && knn_team((size_t)bv.feat_stride * bv.B) == 1;
}

bool match_fit_prune(const GridView& edge, const GridView& surf) {
    return (edge.n > 0 && edge.lim1 < 1.f) || (surf.n > 0 && surf.lim1 < 1.f);
}

// bv.memo: run the memo pass first, then search only its work lists (sparse maps only).
hipError_t launch_match_fit(const GridView& edge, const GridView& surf, const BatchView& bv, hipStream_t s,
                            const GridView& fine_edge, const GridView& fine_surf) {
    const int gx = (bv.feat_stride + 255) / 256;
    const dim3 grid(gx * bv.B);
    const int remap = knn_remap();
    if (match_fit_prune(edge, surf)) {
        static const bool split = ab_int("LMSF_DENSE_SPLIT", LMSF_DENSE_SPLIT) != 0;
        if (split && kLinEval && kListAtomic && bv.memo && bv.wcount) {   // dense memo pass + its listed searches
            hipError_t e = hipMemsetAsync(bv.wcount, 0, (size_t)bv.B * memo_blocks(bv.feat_stride) * sizeof(int), s);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(match_memo_kernel, grid, dim3(256), 0, s, edge, surf, bv, gx, remap);
            // ~2048 blocks over all scans (8 per CU), each scan's list grid-strided by its blocks
            const int G = std::max(1, std::min(gx, std::max(4, 2048 / std::max(bv.B, 1))));
            if (LMSF_MEMO_PASS1 && bv.wl2 && bv.p2count && bv.B <= 8192 &&   // (B + 1) ints of LDS; wl2 holds b * F + pos as int
                (size_t)bv.B * bv.feat_stride < ((size_t)1 << 31)) {
                if ((e = hipMemsetAsync(bv.p2count, 0, sizeof(unsigned), s)) != hipSuccess) return e;
                // all scans' entries flattened over ~8 blocks per CU
                hipLaunchKernelGGL(dense_pass1_listed_kernel, dim3(2048), dim3(256), (size_t)(bv.B + 1) * sizeof(int), s,
                                   edge, surf, fine_edge, fine_surf, bv, bv.p2count);
                const unsigned* cnt = bv.p2count;
                hipLaunchKernelGGL((dense_pass2_kernel<false, 6>), dim3(2048), dim3(256), 0, s, edge, surf, fine_edge,
                                   fine_surf, bv, cnt, (const int*)bv.wl2, (const float*)bv.wlim2);
                hipLaunchKernelGGL(dense_fit2_kernel, dim3(2048), dim3(256), 0, s, edge, surf, bv, cnt, (const int*)bv.wl2);
            } else if (LMSF_MEMO_SPLITFIT) {
                hipLaunchKernelGGL(dense_memo_search_kernel<false>, dim3(G, bv.B), dim3(256), 0, s, edge, surf, fine_edge,
                                   fine_surf, bv);
                hipLaunchKernelGGL(dense_memo_fit_kernel, dim3(G, bv.B), dim3(256), 0, s, edge, surf, bv);
            } else {
                hipLaunchKernelGGL(dense_memo_search_kernel<true>, dim3(G, bv.B), dim3(256), 0, s, edge, surf, fine_edge,
                                   fine_surf, bv);
            }
        } else if (split && kLinEval && bv.p2count && (size_t)bv.B * bv.feat_stride < ((size_t)1 << 31)) {
            hipError_t e = hipMemsetAsync(bv.p2count, 0, sizeof(unsigned), s);
            if (e != hipSuccess) return e;
            const unsigned* cnt = bv.p2count;
            // the outer iteration before the memo: 6 exact keys, anchors left for the memo pass
            if (bv.anchor)
                hipLaunchKernelGGL(dense_pass1_kernel<6>, grid, dim3(256), 0, s, edge, surf, fine_edge, fine_surf, bv, gx,
                                   remap, bv.p2count);
            else
                hipLaunchKernelGGL(dense_pass1_kernel<5>, grid, dim3(256), 0, s, edge, surf, fine_edge, fine_surf, bv, gx,
                                   remap, bv.p2count);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
            // grid-stride over the list (~10% of the queries on C5): 8 blocks per CU
            if (LMSF_P2_SPLITFIT) {
                if (bv.anchor)
                    hipLaunchKernelGGL((dense_pass2_kernel<false, 6>), dim3(2048), dim3(256), 0, s, edge, surf, fine_edge,
                                       fine_surf, bv, cnt, (const int*)bv.wl, (const float*)bv.wlim);
                else
                    hipLaunchKernelGGL((dense_pass2_kernel<false, 5>), dim3(2048), dim3(256), 0, s, edge, surf, fine_edge,
                                       fine_surf, bv, cnt, (const int*)bv.wl, (const float*)bv.wlim);
                e = hipGetLastError();
                if (e != hipSuccess) return e;
                hipLaunchKernelGGL(dense_fit2_kernel, dim3(2048), dim3(256), 0, s, edge, surf, bv, cnt, (const int*)bv.wl);
            } else if (bv.anchor) {
                hipLaunchKernelGGL((dense_pass2_kernel<true, 6>), dim3(2048), dim3(256), 0, s, edge, surf, fine_edge,
                                   fine_surf, bv, cnt, (const int*)bv.wl, (const float*)bv.wlim);
            } else {
                hipLaunchKernelGGL((dense_pass2_kernel<true, 5>), dim3(2048), dim3(256), 0, s, edge, surf, fine_edge,
                                   fine_surf, bv, cnt, (const int*)bv.wl, (const float*)bv.wlim);
            }
        } else {
            hipLaunchKernelGGL((match_fit_kernel<true, false>), grid, dim3(256), 0, s, edge, surf, bv, gx, remap);
        }
    } else if (bv.memo) {
        if (kListAtomic) {
            const hipError_t e = hipMemsetAsync(bv.wcount, 0, (size_t)bv.B * memo_blocks(bv.feat_stride) * sizeof(int), s);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(match_memo_kernel, grid, dim3(256), 0, s, edge, surf, bv, gx, remap);
        const size_t lds = kListAtomic ? 0 : 2 * (memo_blocks(bv.feat_stride) + 1) * sizeof(int);
        hipLaunchKernelGGL((match_fit_kernel<false, true>), grid, dim3(256), lds, s, edge, surf, bv, gx, remap);
    } else {
        hipLaunchKernelGGL((match_fit_kernel<false, false>), grid, dim3(256), 0, s, edge, surf, bv, gx, remap);
    }
    return hipGetLastError();
}

hipError_t launch_lm_eval_step(const BatchView& bv, int outer, int is_last, hipStream_t s) {
    dim3 grid((bv.feat_stride + kEvalBlock - 1) / kEvalBlock, bv.B);
    hipLaunchKernelGGL(lm_eval_kernel<false>, grid, dim3(256), 0, s, bv);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_lm_step(bv, outer, is_last, s);
}

bool lin_eval_enabled() { return kLinEval; }

hipError_t launch_lin_eval(const BatchView& bv, hipStream_t s) {
    dim3 grid((bv.feat_stride + kEvalBlock - 1) / kEvalBlock, bv.B);
    hipLaunchKernelGGL(lm_eval_kernel<true>, grid, dim3(256), 0, s, bv);
    return hipGetLastError();
}

hipError_t launch_eval_at(const BatchView& bv, const double* pose_dev, double* out_dev, hipStream_t s) {
    (void)out_dev;
    dim3 grid((bv.feat_stride + kEvalBlock - 1) / kEvalBlock, 1);
    hipLaunchKernelGGL(eval_at_kernel, grid, dim3(256), 0, s, bv, pose_dev);
    return hipGetLastError();
}

}  // namespace lmsf
