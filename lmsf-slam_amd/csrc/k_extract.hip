// LOAM edge / surf feature extraction on gfx950.
//
// Replaces LOAMFeatureProcessorBase::Process (FX/LOAMFeatureProcessor_base.hpp:59-126, FX =
// src/MultiSensorFusionEstimator3D/include/Algorithm/PointClouds/processing/FeatureExtract) and
// reproduces its output exactly: same ring assignment (splitScan :290-343, float/double
// evaluation order of the C++ expressions), same bad-point automaton including the `j += 4`
// skips (checkBadEdgePoint :216-282), same sectors, same greedy edge pick with disable marks
// leaking across sectors (featureExtractionFromSector :145-207), surf points in ascending
// curvature order.  The unstable std::sort of the reference is canonicalised to (c, index).
//
// Kernels (per batch of scans, one HIP stream):
//   ring_count   tiles of kTile raw points: ring id per point, per-tile ring histogram
//   ring_offsets per scan: exclusive scan (ring-major) -> stable ring-ordered positions
//   ring_scatter stable multisplit (wave ballots) into ring order
//   sector_sort  one workgroup per (sector, ring): curvature + register-resident sort by (c, index)
//   ring_features one workgroup per ring: bad-point events + automaton, then the greedy edge picks of the
//                 6 sectors in order on one wave while the other three trail it with the surf compactions;
//                 each feature position's rank in the ring's search order
//   concat       per scan, per ring position: the feature slot (edges of ring 0..N-1 then surfs) and the
//                 fused search's order (fslot / featp), the point written to both
#include <hip/hip_runtime.h>
#include <math.h>

#include <climits>
#include <type_traits>

#include "lmsf_internal.h"

#pragma clang fp contract(off)

namespace lmsf {

namespace {

// The reference's unqualified sqrt / atan2 on float arguments (lmsf_config::libm_float): the double
// versions, or the float overloads (sqrtf; atan2 in double rounded to float).
__device__ __forceinline__ double ref_sqrt(float s, int libm_float) {
    return libm_float ? (double)sqrtf(s) : sqrt((double)s);
}
__device__ __forceinline__ double ref_atan2(float y, float x, int libm_float) {
    const double a = atan2((double)y, (double)x);
    return libm_float ? (double)(float)a : a;
}

__device__ __forceinline__ int ring_of(const ExtractView& ev, float4 p) {
    const float s = p.x * p.x + p.y * p.y;                       // float expression (FX:300-301)
    const double distance = ref_sqrt(s, ev.libm_float);
    if (distance > (double)ev.max_d || distance < (double)ev.min_d) return -1;   // FX:302
    const double angle = atan((double)p.z / distance) * 180 / M_PI;              // FX:307
    const bool bad = isnan(angle);   // int(NaN) is INT_MIN on the reference's x86 host
    const int n = ev.n_scans;
    int id;
    if (n == 16) {
        if (bad) return -1;
        id = (int)((angle + 15) / 2 + 0.5);
        if (id > n - 1 || id < 0) return -1;
    } else if (n == 32) {
        if (bad) return -1;
        id = (int)((angle + 92.0 / 3.0) * 3.0 / 4.0);
        if (id > n - 1 || id < 0) return -1;    // FX:320 lower-bound bug is UB: rejected here
    } else if (n == 64) {
        if (bad) return -1;
        if (angle >= -8.83) id = (int)((2 - angle) * 3.0 + 0.5);
        else id = n / 2 + (int)((-8.83 - angle) * 2.0 + 0.5);
        if (angle > 2 || angle < -24.33 || id > 63 || id < 0) return -1;
    } else if (ev.beam_spacing > 0) {
        if (bad) return -1;
        id = (int)((angle - ev.beam_lo) / ev.beam_spacing + 0.5);
        if (id > n - 1 || id < 0) return -1;
    } else {
        id = 0;  // "wrong scan number" (FX:337-341)
    }
    return id;
}

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

}  // namespace

__global__ __launch_bounds__(256) void ring_count_kernel(ExtractView ev) {
    __shared__ int cnt[kMaxRings];
    const int b = blockIdx.y, t = blockIdx.x;
    const int n = ev.raw_count[b];
    if (t * kTile >= n && t > 0) return;
    for (int r = threadIdx.x; r < ev.n_scans; r += 256) cnt[r] = 0;
    __syncthreads();
    const float4* raw = ev.raw + ev.raw_off[b];
    int8_t* rid = ev.ring_id + (size_t)b * ev.raw_stride;
    for (int k = threadIdx.x; k < kTile; k += 256) {
        const int i = t * kTile + k;
        if (i < n) {
            const int r = ring_of(ev, raw[i]);
            rid[i] = (int8_t)r;
            if (r >= 0) atomicAdd(&cnt[r], 1);
        }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < ev.n_scans; r += 256)
        ev.tile_counts[((size_t)b * kMaxRings + r) * ev.n_tiles + t] = cnt[r];
}

// Exclusive scan of tile_counts in (ring, tile) order, in place -> tile offsets; ring_start.
__global__ __launch_bounds__(256) void ring_offsets_kernel(ExtractView ev) {
    __shared__ int part[256];
    const int b = blockIdx.x;
    const int n = ev.raw_count[b];
    const int nt = max((n + kTile - 1) / kTile, 1);
    const int E = ev.n_scans * nt;
    int* tc = ev.tile_counts + (size_t)b * kMaxRings * ev.n_tiles;
    const int per = (E + 255) / 256;
    const int lo = threadIdx.x * per, hi = min(lo + per, E);
    int s = 0;
    for (int e = lo; e < hi; ++e) s += tc[(e / nt) * ev.n_tiles + (e % nt)];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int i = 0; i < 256; ++i) { int v = part[i]; part[i] = acc; acc += v; }
    }
    __syncthreads();
    int acc = part[threadIdx.x];
    for (int e = lo; e < hi; ++e) {
        int* c = &tc[(e / nt) * ev.n_tiles + (e % nt)];
        const int v = *c;
        *c = acc;
        if (e % nt == 0) ev.ring_start[(size_t)b * (kMaxRings + 1) + e / nt] = acc;
        acc += v;
    }
    if (hi == E && lo < hi) ev.ring_start[(size_t)b * (kMaxRings + 1) + ev.n_scans] = acc;
    if (E == 0 && threadIdx.x == 0) ev.ring_start[(size_t)b * (kMaxRings + 1) + ev.n_scans] = 0;
}

// LMSF_SCATTER_BITS (A/B): the multisplit's in-wave ranking by ring-id bit ballots (1) or by a leader loop over the
// distinct rings of the wave (0, r04).
#ifndef LMSF_SCATTER_BITS
#define LMSF_SCATTER_BITS 1
#endif
constexpr bool kScatterBits = LMSF_SCATTER_BITS != 0;
// LMSF_CONCAT_LDS (A/B): concat_kernel's ring lookup of a position by binary search over the ring starts staged in
// LDS (1) or read from global memory (0, r04: 7 dependent L2 round trips per position on a 128-ring scan).
#ifndef LMSF_CONCAT_LDS
#define LMSF_CONCAT_LDS 1
#endif
// LMSF_SCATTER_LDS (A/B): ring_scatter_kernel stages its tile in LDS in ring-major order and writes each ring's run of
// the tile contiguously for scans of more than kScatterLdsRings rings (1), or stores every point straight to its ring
// position (0, r04: on a column-major 128-beam scan a wave's 64 stores then land in 64 rings, 16 B each).  16-beam
// scans keep the direct stores: a 256-point chunk already writes 16-point runs per ring, and the staging's extra
// pass and 51 KB of LDS made C2's scatter slower (81 -> 104 us per 128 scans).
#ifndef LMSF_SCATTER_LDS
#define LMSF_SCATTER_LDS 1
#endif
constexpr int kScatterLdsRings = 32;

// Stable multisplit of one tile into ring order (input order preserved inside each ring).
template <bool kScatterLds>
__global__ __launch_bounds__(256) void ring_scatter_kernel(ExtractView ev) {
    __shared__ int wcnt[4][kMaxRings];
    __shared__ int running[kMaxRings];
    // kScatterLds: the tile's points in ring-major order (lstart: the tile's exclusive ring prefix), their
    // destinations and source indices
    __shared__ float4 s_pt[kScatterLds ? kTile : 1];
    __shared__ int s_dst[kScatterLds ? kTile : 1], s_src[kScatterLds ? kTile : 1];
    __shared__ int lstart[kMaxRings];
    const int b = blockIdx.y, t = blockIdx.x;
    const int n = ev.raw_count[b];
    if (t * kTile >= n) return;
    const int nt = (n + kTile - 1) / kTile;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int r = threadIdx.x; r < kMaxRings; r += 256) running[r] = 0;
    const float4* raw = ev.raw + ev.raw_off[b];
    const int8_t* rid = ev.ring_id + (size_t)b * ev.raw_stride;
    const int* toff = ev.tile_counts + (size_t)b * kMaxRings * ev.n_tiles;
    float4* out = ev.ring_pts + (size_t)b * ev.raw_stride;
    int* osrc = ev.ring_src + (size_t)b * ev.raw_stride;
    (void)nt;
    int tile_total = 0;
    if constexpr (kScatterLds) {   // the tile's ring counts (lstart as a histogram first), then their prefix
        for (int r = threadIdx.x; r < kMaxRings; r += 256) lstart[r] = 0;
        __syncthreads();
        for (int k = threadIdx.x; k < kTile; k += 256) {
            const int i = t * kTile + k;
            const int r = i < n ? (int)rid[i] : -1;
            if (r >= 0) atomicAdd(&lstart[r], 1);
        }
        __syncthreads();
        if (threadIdx.x < 64) {   // exclusive scan over the rings by one wave
            int acc = 0;
            for (int r0 = 0; r0 < ev.n_scans; r0 += 64) {
                const int r = r0 + lane;
                const int c = r < ev.n_scans ? lstart[r] : 0;
                int x = c;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int y = __shfl_up(x, o, 64);
                    if (lane >= o) x += y;
                }
                if (r < ev.n_scans) lstart[r] = acc + x - c;
                acc += __shfl(x, 63, 64);
            }
            if (lane == 0) wcnt[0][0] = acc;   // the tile's total (wcnt is cleared before its first use below)
        }
        __syncthreads();
        tile_total = wcnt[0][0];
        __syncthreads();
    }
    const int ring_bits = ev.n_scans <= 1 ? 0 : 32 - __clz(ev.n_scans - 1);
    for (int c0 = 0; c0 < kTile; c0 += 256) {
        for (int k = threadIdx.x; k < 4 * kMaxRings; k += 256) wcnt[k / kMaxRings][k % kMaxRings] = 0;
        __syncthreads();
        const int i = t * kTile + c0 + threadIdx.x;
        const int r = i < n ? (int)rid[i] : -1;
        const float4 pt = r >= 0 ? raw[i] : make_float4(0, 0, 0, 0);   // in flight across the rank pass
        int rank = 0;
        if constexpr (kScatterBits) {
            // the lanes of my ring by one ballot per ring-id bit (k_sort.hip's digit ranking): ceil(log2 n_scans)
            // ballots, where the leader loop below takes one round per distinct ring in the wave -- up to 64 on a
            // 128-beam scan stored column by column
            const unsigned long long lt = lanemask_lt(lane);
            unsigned long long peers = __ballot(r >= 0);
            for (int bit = 0; bit < ring_bits; ++bit) {
                const bool set = ((r >> bit) & 1) != 0;
                const unsigned long long m = __ballot(set);
                peers &= set ? m : ~m;
            }
            if (r >= 0) {
                rank = __popcll(peers & lt);
                if ((peers & lt) == 0ull) wcnt[wave][r] = __popcll(peers);
            }
        } else {
            unsigned long long remaining = __ballot(r >= 0);
            while (remaining) {
                const int leader = __ffsll((long long)remaining) - 1;
                const int rl = __shfl(r, leader, 64);
                const unsigned long long m = __ballot(r == rl);
                if (r == rl) rank = __popcll(m & lanemask_lt(lane));
                if (lane == leader) wcnt[wave][rl] = __popcll(m);
                remaining &= ~m;
            }
        }
        __syncthreads();
        if (r >= 0) {
            int base = running[r];
            for (int w = 0; w < wave; ++w) base += wcnt[w][r];
            const int dst = toff[(size_t)r * ev.n_tiles + t] + base + rank;
            if constexpr (kScatterLds) {
                const int lp = lstart[r] + base + rank;
                s_pt[lp] = pt;
                s_dst[lp] = dst;
                s_src[lp] = i;
            } else {
                out[dst] = pt;
                osrc[dst] = i;
            }
        }
        __syncthreads();
        for (int rr = threadIdx.x; rr < ev.n_scans; rr += 256)
            running[rr] += wcnt[0][rr] + wcnt[1][rr] + wcnt[2][rr] + wcnt[3][rr];
        __syncthreads();
    }
    if constexpr (kScatterLds) {   // each ring's run of the tile to consecutive ring positions
        for (int j = threadIdx.x; j < tile_total; j += 256) {
            const int dst = s_dst[j];
            out[dst] = s_pt[j];
            osrc[dst] = s_src[j];
        }
    }
}

// checkBadEdgePoint (FX:216-282) for one ring: per-point events, then the sequential skip
// automaton (next j = j + 5 after event 1 / 2, else j + 1) walked 64 candidates at a time by one
// wave.  dis[] = disabled marks; flag[] is left cleared for reuse as is_edge.
template <int NT>
__device__ void ring_bad_points(const ExtractView& ev, const float4* pts, int size, uint8_t* dis, uint8_t* flag) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int jmax = size - 7;  // checkBadEdgePoint visits j in [5, size - 7]
    if (ev.remove_bad) {
        // events per point in wave chunks of 63: lane l loads point j = base + l (coalesced) and its azimuth,
        // and takes point j + 1's (its angle_after) from lane l + 1 -- one atan2 per point (+ 1 in 63);
        // lane 63 only serves lane 62
#ifndef LMSF_AB_NO_EVENTS   // A/B ablation builds only
        const int wave = tid >> 6;
        for (int base = 5 + 63 * wave; base <= jmax; base += 63 * (NT / 64)) {
            const int j = base + lane;
            const float4 a = pts[min(j, jmax + 1)];   // jmax + 1 = size - 6: a ring point
            const double angle_curr = ref_atan2(a.x, a.y, ev.libm_float);   // atan2(x, y) order (FX:223-224)
            const double angle_after = __shfl_down(angle_curr, 1, 64);
            const float4 c = make_float4(__shfl_down(a.x, 1, 64), __shfl_down(a.y, 1, 64), __shfl_down(a.z, 1, 64), 0.f);
            if (lane < 63 && j <= jmax) {
                double delta_angle = fabs(angle_curr - angle_after);
                if (delta_angle > M_PI) delta_angle = M_PI * 2 - delta_angle;
                uint8_t e = 0;
                if (delta_angle > 0.0175) {
                    e = 1;
                } else {
                    const float sc = a.x * a.x + a.y * a.y + a.z * a.z;
                    const float sa = c.x * c.x + c.y * c.y + c.z * c.z;
                    const double dc = ref_sqrt(sc, ev.libm_float), da = ref_sqrt(sa, ev.libm_float);
                    const double ang = dc < da ? atan2(dc * delta_angle, da - dc) : atan2(da * delta_angle, dc - da);
                    if (ang <= 0.17) e = dc < da ? 2 : 3;
                }
                flag[j] = e;
            }
        }
#else
        for (int j = 5 + tid; j <= jmax; j += NT) flag[j] = 0;
#endif
        __syncthreads();
        // sequential skip automaton (next j = j + 5 after event 1 / 2, else j + 1), 64 at a time
        // one load of 64 events per step; the step's skips are followed in registers (start: the first lane
        // the walk visits in this step)
        if (tid < 64) {
            int pos = 5;
            while (pos <= jmax) {
                const int j = pos + lane;
                const int e = j <= jmax ? (int)flag[j] : 0;
                const unsigned long long ev12 = __ballot(e == 1 || e == 2);
                int start = 0;
                while (true) {
                    const unsigned long long m = ev12 & (~0ull << start);
                    const int f = m ? (__ffsll((long long)m) - 1) : 64;
                    if (lane >= start && lane < f && e == 3) {
#pragma unroll
                        for (int k = 0; k <= 5; ++k) dis[j - k] = 1;
                    }
                    if (lane == f) {
                        if (e == 1) {
#pragma unroll
                            for (int k = -5; k <= 5; ++k) dis[j + k] = 1;
                        } else {
#pragma unroll
                            for (int k = 1; k <= 5; ++k) dis[j + k] = 1;
                        }
                    }
                    if (!m) { pos += 64; break; }
                    start = f + 5;   // the reference's j += 4 and the loop's ++j (FX:231-260)
                    if (start >= 64) { pos += start; break; }
                }
            }
        }
        __syncthreads();
        for (int j = tid; j < size; j += NT) flag[j] = 0;   // reuse as is_edge
        __syncthreads();
    }
}

// Sort of n (key, index) pairs ascending by (key, index), n <= npow = 64 E * 4: keys (non-negative
// doubles, compared as their u64 bit patterns, which order alike) and indices in LDS on entry and exit,
// positions [n, npow) holding pads (key ~0: above every double) on entry.
//   1. A bitonic network in its ascending-only form: merge step kk opens with a "flip" stage (partner
//      i ^ (kk - 1)) and continues with half-cleaners (partner i ^ jj); every comparator puts the smaller
//      key at the lower position, so the pads never leave [n, npow) and a wave whose positions all lie
//      there has nothing to do (n = 650 of a C2 sector: 3 of 4 waves work).  Keys only: equal keys do not
//      swap, so they end up adjacent in some order.
//   2. Runs of equal keys are put in index order (rank by index inside the run), giving the (key, index)
//      order of a comparison sort with the index as tie-break.
// Elements live in registers: wave w owns positions [w * 64E, (w + 1) * 64E), lane l holds
// w * 64E + e * 64 + l (e < E).  A partner that differs in the lane bits only is a shuffle, in the e bits
// (+ lane bits) a register pick (+ shuffle), and only partners in another wave go through LDS.
// Lane exchange x <- x of lane (lane ^ M), M a constant: DPP quad / row permutations where one exists
// (xor 1, 2, 3 within quads; xor 7 / 15 = the half-row / row mirrors), ds_swizzle's xor mode inside 32
// lanes, ds_bpermute across the two halves.
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x) {
    if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // [2,3,0,1]
    else if constexpr (M == 3) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x1B, 0xF, 0xF, false);   // [3,2,1,0]
    else if constexpr (M == 7) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    else if constexpr (M == 15) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false); // row_mirror
    else if constexpr (M < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (M << 10) | 0x1F);
    else return (uint32_t)__shfl_xor((int)x, M, 64);
}

// Stage s of the ascending-only bitonic network of NPOW elements: merge step kk opens with the flip (partner
// mask kk - 1) and continues with the half-cleaners kk/4 .. 1.
constexpr int sort_stage_mask(int npow, int s) {
    for (int kk = 2; kk <= npow; kk <<= 1) {
        for (int m = kk - 1, jj = kk; jj > 1; jj >>= 1, m = jj >> 1) {
            if (s == 0) return m;
            --s;
        }
    }
    return 0;
}
constexpr int sort_stage_count(int npow) {
    int c = 0;
    for (int kk = 2; kk <= npow; kk <<= 1)
        for (int jj = kk; jj > 1; jj >>= 1) ++c;
    return c;
}
constexpr int high_bit(int m) {
    int h = 1;
    while (h * 2 <= m) h *= 2;
    return h;
}

// One compare-exchange stage with the constant partner mask M over the E keys of every lane (positions
// w * 64E + e * 64 + lane): the lower position of each pair keeps the smaller key.
template <int M, int E>
__device__ __forceinline__ void sort_stage(uint64_t (&k)[E], int (&id)[E], uint64_t* key, int* kidx, int w, int lane,
                                           bool active) {
    constexpr int chunk = 64 * E, HB = high_bit(M);
    if constexpr (M >= chunk) {   // partner in another wave: through LDS
        __syncthreads();
        if (active) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                key[w * chunk + e * 64 + lane] = k[e];
                kidx[w * chunk + e * 64 + lane] = id[e];
            }
        }
        __syncthreads();
        if (active) {
            const bool lower = ((w * chunk) & HB) == 0;   // HB >= chunk: a wave bit
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int p = (w * chunk + e * 64 + lane) ^ M;
                const uint64_t ko = key[p];
                const int io = kidx[p];
                const bool take = lower ? ko < k[e] : ko > k[e];
                if (take) { k[e] = ko; id[e] = io; }
            }
        }
    } else if (active) {
        constexpr int ML = M & 63, ME = (M >> 6) & (E - 1);
        uint64_t ko[E];
        int io[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            ko[e] = k[e ^ ME];
            io[e] = id[e ^ ME];
            if constexpr (ML != 0) {
                const uint32_t lo = lane_xor<ML>((uint32_t)ko[e]), hi = lane_xor<ML>((uint32_t)(ko[e] >> 32));
                ko[e] = ((uint64_t)hi << 32) | lo;
                io[e] = (int)lane_xor<ML>((uint32_t)io[e]);
            }
        }
        const bool lane_lower = (lane & HB) == 0;   // used when HB is a lane bit (HB < 64)
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const bool lower = HB < 64 ? lane_lower : ((e * 64) & HB) == 0;
            const bool take = lower ? ko[e] < k[e] : ko[e] > k[e];
            if (take) { k[e] = ko[e]; id[e] = io[e]; }
        }
    }
}

template <int E, int NPOW, int S, int NS = sort_stage_count(NPOW)>
struct SortStages {
    static __device__ __forceinline__ void run(uint64_t (&k)[E], int (&id)[E], uint64_t* key, int* kidx, int w, int lane,
                                               bool active) {
        sort_stage<sort_stage_mask(NPOW, S), E>(k, id, key, kidx, w, lane, active);
        SortStages<E, NPOW, S + 1, NS>::run(k, id, key, kidx, w, lane, active);
    }
};
template <int E, int NPOW, int NS>
struct SortStages<E, NPOW, NS, NS> {
    static __device__ __forceinline__ void run(uint64_t (&)[E], int (&)[E], uint64_t*, int*, int, int, bool) {}
};

template <int E, int NPOW>
__device__ void sector_sort_regs(uint64_t* key, int* kidx, int n) {
    static_assert(NPOW == 4 * 64 * E, "four waves of E keys per lane");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int chunk = 64 * E;
    const bool active = w * chunk < n;
    uint64_t k[E];
    int id[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = w * chunk + e * 64 + lane;
        k[e] = active ? key[i] : ~0ull;
        id[e] = active ? kidx[i] : 0x7fffffff;
    }
    // every stage's partner mask is a compile-time constant: the in-wave / cross-wave choice, the register
    // pick and the lane exchange (DPP / swizzle) are fixed at compile time, no address arithmetic
    SortStages<E, NPOW, 0>::run(k, id, key, kidx, w, lane, active);
    __syncthreads();
    if (active) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = w * chunk + e * 64 + lane;
            key[i] = k[e];
            kidx[i] = id[e];
        }
    }
    __syncthreads();
    // equal keys: rank by index inside the run (positions held in registers until every rank is read)
    constexpr int kPer = (kSortMax + 255) / 256;
    int fix_pos[kPer], fix_id[kPer];
#pragma unroll
    for (int t = 0; t < kPer; ++t) {
        const int i = threadIdx.x + 256 * t;
        fix_pos[t] = -1;
        fix_id[t] = 0;
        if (i < n) {
            const uint64_t kv = key[i];
            if ((i > 0 && key[i - 1] == kv) || (i + 1 < n && key[i + 1] == kv)) {
                int s0 = i, e0 = i + 1;
                while (s0 > 0 && key[s0 - 1] == kv) --s0;
                while (e0 < n && key[e0] == kv) ++e0;
                const int mine = kidx[i];
                int r = 0;
                for (int j = s0; j < e0; ++j) r += kidx[j] < mine;
                fix_pos[t] = s0 + r;
                fix_id[t] = mine;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kPer; ++t)
        if (fix_pos[t] >= 0) kidx[fix_pos[t]] = fix_id[t];
    __syncthreads();
}

// Sector geometry of featureExtractionFromSector (FX:145-156): 6 sectors of a ring of `size`.
__device__ __forceinline__ void sector_bounds(int size, int k, int& s0, int& n) {
    const int sector_length = (size - 10) / 6;          // (int)((total/6) + 0.5) with int division
    s0 = 5 + sector_length * k;
    const int e0 = (k == 5) ? size - 6 : s0 + sector_length - 1;
    n = e0 - s0 + 1;
}

// One workgroup per (sector, ring, scan): curvature (FX:84-94) of the sector's points and their
// register-resident bitonic sort by (c, index); written to sort_key / sort_idx at the sector's
// place in the ring.  The 6 sectors of a ring sort concurrently; only the greedy pick, which
// carries disable marks across sectors, stays sequential (ring_features_kernel).
__global__ __launch_bounds__(256) void sector_sort_kernel(ExtractView ev) {
    __shared__ uint64_t key[kSortMax];
    __shared__ int kidx[kSortMax];
    const int r = blockIdx.x / 6, k = blockIdx.x % 6, b = blockIdx.y;
    const int* rs = ev.ring_start + (size_t)b * (kMaxRings + 1);
    const int start = rs[r];
    const int size = rs[r + 1] - start;
    if (size < 20 || size > kRingMax) return;            // ring_features_kernel reports
    int s0, n;
    sector_bounds(size, k, s0, n);
    if (n > kSortMax) return;
    const float4* pts = ev.ring_pts + (size_t)b * ev.raw_stride + start;
    const int npow = n <= 256 ? 256 : n <= 512 ? 512 : n <= 1024 ? 1024 : 2048;   // the network's size
    for (int i = threadIdx.x; i < npow; i += 256) {
        if (i < n) {
            const int j = s0 + i;
            const float4 m5 = pts[j - 5], m4 = pts[j - 4], m3 = pts[j - 3], m2 = pts[j - 2], m1 = pts[j - 1];
            const float4 p0 = pts[j];
            const float4 q1 = pts[j + 1], q2 = pts[j + 2], q3 = pts[j + 3], q4 = pts[j + 4], q5 = pts[j + 5];
            const float fx = m5.x + m4.x + m3.x + m2.x + m1.x - 10 * p0.x + q1.x + q2.x + q3.x + q4.x + q5.x;
            const float fy = m5.y + m4.y + m3.y + m2.y + m1.y - 10 * p0.y + q1.y + q2.y + q3.y + q4.y + q5.y;
            const float fz = m5.z + m4.z + m3.z + m2.z + m1.z - 10 * p0.z + q1.z + q2.z + q3.z + q4.z + q5.z;
            const double dx = fx, dy = fy, dz = fz;
            key[i] = (uint64_t)__double_as_longlong(dx * dx + dy * dy + dz * dz);
            kidx[i] = j;
        } else {
            key[i] = ~0ull;
            kidx[i] = 0x7fffffff;
        }
    }
    __syncthreads();
    if (npow == 256) sector_sort_regs<1, 256>(key, kidx, n);
    else if (npow == 512) sector_sort_regs<2, 512>(key, kidx, n);
    else if (npow == 1024) sector_sort_regs<4, 1024>(key, kidx, n);
    else sector_sort_regs<8, 2048>(key, kidx, n);
    double* okey = ev.sort_key + (size_t)b * ev.raw_stride + start + s0;
    int* oidx = ev.sort_idx + (size_t)b * ev.raw_stride + start + s0;
    for (int i = threadIdx.x; i < n; i += 256) {
        okey[i] = __longlong_as_double((long long)key[i]);
        oidx[i] = kidx[i];
    }
}

// One workgroup per (ring, scan): bad-point automaton (all waves: events; wave 0: the skip walk), then
// wave 0 runs the greedy edge picks of the 6 sectors in order (FX:157-195; disable marks leak across
// sectors) while waves 1-3 trail it with the surf compactions (FX:197-206), sector k on wave 1 + k % 3
// as soon as wave 0 has published sector k's picks: a sector's surfs are its points not picked in that
// sector, so its compaction needs nothing from later sectors, and its output offset is the earlier
// sectors' point counts minus their picks.  The pick reads the top kPickWin entries of the sector's
// sorted list from an LDS window (the next sector's window is loaded while the current one is picked),
// deeper entries from global memory; no sector is staged whole, so a block needs ~19 KB of LDS.
constexpr int kPickWin = 256;
// Waves per SIMD ring_features_kernel is compiled for (A/B builds; C2, one box, two rounds each: 5 waves
// (82 VGPRs) 26.02k / 26.13k scans/s, 6 (80) 26.08k / 26.09k, 8 (64, 48 B spill) 25.83k / 25.72k).
#ifndef LMSF_RF_WAVES
#define LMSF_RF_WAVES 5
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LMSF_RF_WAVES))) void ring_features_kernel(ExtractView ev) {
    __shared__ uint8_t dis[kRingMax];
    __shared__ uint8_t flag[kRingMax];
    __shared__ double wkey[kPickWin];
    __shared__ int widx[kPickWin];
    __shared__ int sh_e[6];       // edges picked in sector k
    __shared__ int sh_done;       // sectors whose picks are published
    __shared__ int sh_sc[6];      // surfs of sector k (written by its compaction wave)
    const int r = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int* rs = ev.ring_start + (size_t)b * (kMaxRings + 1);
    const int start = rs[r];
    const int size = rs[r + 1] - start;
    int* ecnt = ev.ring_edge_cnt + (size_t)b * kMaxRings;
    int* scnt = ev.ring_surf_cnt + (size_t)b * kMaxRings;
    int* qc = ev.qcode + (size_t)b * ev.raw_stride + start;   // ring position -> ring-local feature code
    if (size < 20 || size > kRingMax) {   // FX:71
        for (int j = tid; j < size; j += 256) qc[j] = -1;
        if (tid == 0) {
            ecnt[r] = 0;
            scnt[r] = 0;
            if (size > kRingMax) atomicOr(ev.error, 1);
        }
        return;
    }
    const float4* pts = ev.ring_pts + (size_t)b * ev.raw_stride + start;
    for (int j = tid; j < size; j += 256) { dis[j] = 0; flag[j] = 0; qc[j] = -1; }
    if (tid == 0) sh_done = 0;
    __syncthreads();
    ring_bad_points<256>(ev, pts, size, dis, flag);   // ends with a barrier; flag cleared (is_edge)
    const double* skey_ring = ev.sort_key + (size_t)b * ev.raw_stride + start;
    const int* sidx_ring = ev.sort_idx + (size_t)b * ev.raw_stride + start;
    int s0_[6], n_[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) sector_bounds(size, k, s0_[k], n_[k]);
    const bool fits = n_[5] <= kSortMax && n_[0] <= kSortMax;   // uniform: sector_sort_kernel's bound
    if (wave == 0) {
        const double thresh = (double)ev.edge_thresh;
        constexpr int kWin = kPickWin / 64;
        double pk[kWin];
        int pi[kWin];
        auto fetch = [&](int k) {   // sector k's window [n - kPickWin, n) into registers
#pragma unroll
            for (int u = 0; u < kWin; ++u) {
                const int i = n_[k] - kPickWin + u * 64 + lane;
                pk[u] = i >= 0 ? skey_ring[s0_[k] + i] : 0.0;
                pi[u] = i >= 0 ? sidx_ring[s0_[k] + i] : 0;
            }
        };
        if (fits) fetch(0);
        int ec = 0;
        for (int k = 0; k < 6 && fits; ++k) {
            const int n = n_[k], wlo = n - kPickWin;   // window: sorted positions [wlo, n)
#pragma unroll
            for (int u = 0; u < kWin; ++u) {
                wkey[u * 64 + lane] = pk[u];
                widx[u * 64 + lane] = pi[u];
            }
            __builtin_amdgcn_wave_barrier();
            if (k < 5) fetch(k + 1);   // in flight during this sector's pick
            const double* skey = skey_ring + s0_[k];
            const int* sidx = sidx_ring + s0_[k];
            auto idx_at = [&](int i) { return i >= wlo ? widx[i - wlo] : sidx[i]; };
            auto key_at = [&](int i) { return i >= wlo ? wkey[i - wlo] : skey[i]; };
            // 64 candidates per step (lane l: sorted position pos - l, descending curvature): one load of
            // their ring indices, keys and disable marks, then the step's picks in registers -- a pick at ring
            // index ind disables the candidates within 5 of it (the marks it writes), so the next pick is the
            // next eligible lane.  Keys at or below the threshold end the sector (sorted: no later candidate
            // is above it), as the reference's break at the first enabled one does (FX:163-165).
            int pos = n - 1, picked = 0;
            const int ec0 = ec;
            while (pos >= 0 && picked < 20) {
                const int cand = pos - lane;
                const bool valid = cand >= 0;
                const int idx = valid ? idx_at(cand) : -100;   // -100: more than 5 from every ring index
                const bool above = valid && key_at(cand) > thresh;
                unsigned long long m = __ballot(above && dis[idx] == 0);
                const bool last = pos < 64 || __ballot(valid && !above) != 0;
                while (m && picked < 20) {
                    const int f = __ffsll((long long)m) - 1;
                    const int ind = __builtin_amdgcn_readlane(idx, f);
                    ++picked;
                    if (lane == 0) {
                        flag[ind] = 1;
                        qc[ind] = ec;   // ring-local edge index: concat_kernel places the point
                    }
                    if (lane >= 1 && lane <= 5) dis[min(ind + lane, size - 1)] = 1;
                    if (lane >= 6 && lane <= 10) dis[max(ind - (lane - 5), 0)] = 1;
                    ++ec;
                    m &= ~__ballot(abs(idx - ind) <= 5);
                }
                if (last) break;
                pos -= 64;
            }
            if (lane == 0) {
                sh_e[k] = ec - ec0;
                __hip_atomic_store(&sh_done, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        if (lane == 0 && !fits) {
            atomicOr(ev.error, 2);
            __hip_atomic_store(&sh_done, 6, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (lane == 0) ecnt[r] = fits ? ec : 0;
    } else if (fits) {
        for (int k = wave - 1; k < 6; k += 3) {
            while (__hip_atomic_load(&sh_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= k)
                __builtin_amdgcn_s_sleep(2);
            int o = 0;   // surfs of the earlier sectors
            for (int k2 = 0; k2 < k; ++k2) o += n_[k2] - sh_e[k2];
            const int n = n_[k];
            const int* sidx = sidx_ring + s0_[k];
            // ascending curvature, 64 positions per step, 4 steps' index loads in flight
            for (int c0 = 0; c0 < n; c0 += 256) {
                int ind[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = c0 + u * 64 + lane;
                    ind[u] = i < n ? sidx[i] : -1;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool keep = ind[u] >= 0 && flag[ind[u]] == 0;
                    const unsigned long long m = __ballot(keep);
                    if (keep) qc[ind[u]] = kQSurf | (o + __popcll(m & lanemask_lt(lane)));   // ring-local surf index
                    o += __popcll(m);
                }
            }
            if (lane == 0) sh_sc[k] = n - sh_e[k];
        }
    }
    __syncthreads();
    if (tid == 0) {
        int sc = 0;
        for (int k = 0; k < 6; ++k) sc += sh_sc[k];
        scnt[r] = fits ? sc : 0;
    }
    if (!fits) return;   // uniform: the ring's counts are 0, concat_kernel ignores its codes
    // Search order inside the ring: every feature position's rank among the ring's features of its kind in
    // ring order, packed into its code (bits 13-25) for concat_kernel, which places the position at its kind's
    // ring base + rank (edges before surfs: the fused search's order).  Positions [5, size - 6] are the
    // sectors': picked (flag) -> edge, else surf.  Block scan over contiguous chunks, (edge, surf) counts
    // packed 16 | 16 bits.
    {
        __shared__ uint32_t wsum[4];
        const int per = (size + 255) / 256;
        const int p0 = min(tid * per, size), p1 = min(p0 + per, size);
        uint32_t cnt = 0;
        for (int p = p0; p < p1; ++p) {
            if (flag[p]) cnt += 1u;
            else if (p >= 5 && p <= size - 6) cnt += 0x10000u;
        }
        uint32_t x = cnt;
#pragma unroll
        for (int o2 = 1; o2 < 64; o2 <<= 1) {
            const uint32_t y = __shfl_up(x, o2, 64);
            if (lane >= o2) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t ex = x - cnt;
        for (int w2 = 0; w2 < wave; ++w2) ex += wsum[w2];
        uint32_t re = ex & 0xffffu, rsf = ex >> 16;
        for (int p = p0; p < p1; ++p) {
            if (flag[p]) qc[p] = qc[p] | (int)(re++ << kQRankShift);
            else if (p >= 5 && p <= size - 6) qc[p] = qc[p] | (int)(rsf++ << kQRankShift);
        }
    }
}

// Concatenate per-ring stages: edges of ring 0..N-1, then surfs of ring 0..N-1 (FX:124-125 order).
__global__ __launch_bounds__(256) void concat_kernel(ExtractView ev) {
    __shared__ int epre[kMaxRings + 1], spre[kMaxRings + 1], srs[kMaxRings + 1];
    const int b = blockIdx.y;
    const int nr = ev.n_scans;
    if (LMSF_CONCAT_LDS)
        for (int r = threadIdx.x; r <= nr; r += 256) srs[r] = ev.ring_start[(size_t)b * (kMaxRings + 1) + r];
#ifdef LMSF_CONCAT_SERIAL   // A/B build: r02 first-half prologue (one thread sums the ring counts)
    if (threadIdx.x == 0) {
        int e = 0, s = 0;
        for (int r = 0; r < nr; ++r) {
            epre[r] = e; spre[r] = s;
            e += ev.ring_edge_cnt[(size_t)b * kMaxRings + r];
            s += ev.ring_surf_cnt[(size_t)b * kMaxRings + r];
        }
        epre[nr] = e; spre[nr] = s;
        if (blockIdx.x == 0) {
            ev.n_edge[b] = e;
            ev.n_surf[b] = s;
        }
    }
    if (false) {
#else
    if (threadIdx.x < 64) {   // ring-count prefixes by one wave: lane r loads ring r's counts, shuffle scan
#endif
        const int r = threadIdx.x;
        int e = 0, s = 0;
        for (int r0 = 0; r0 < nr; r0 += 64) {
            const int ce = r0 + r < nr ? ev.ring_edge_cnt[(size_t)b * kMaxRings + r0 + r] : 0;
            const int cs = r0 + r < nr ? ev.ring_surf_cnt[(size_t)b * kMaxRings + r0 + r] : 0;
            int xe = ce, xs = cs;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int ye = __shfl_up(xe, o, 64), ys = __shfl_up(xs, o, 64);
                if (r >= o) { xe += ye; xs += ys; }
            }
            if (r0 + r < nr) { epre[r0 + r] = e + xe - ce; spre[r0 + r] = s + xs - cs; }
            e += __shfl(xe, 63, 64);
            s += __shfl(xs, 63, 64);
        }
        if (r == 0) {
            epre[nr] = e; spre[nr] = s;
            if (blockIdx.x == 0) {
                ev.n_edge[b] = e;
                ev.n_surf[b] = s;
            }
        }
    }
    __syncthreads();
    const int ne = epre[nr];
    const int* rs = LMSF_CONCAT_LDS ? srs : ev.ring_start + (size_t)b * (kMaxRings + 1);
    // Every feature position of the rings, in ring order: its feature slot (edges of ring 0..N-1, then surfs,
    // each ring's in the reference's emission order -- the ring-local index ring_features_kernel packed into the
    // position's code) and its place in the fused search's order (edges of ring 0..N-1 then surfs, each ring's in
    // ring order: the rank packed into the code).  The point goes to both: feat / feat_src at the slot (FX:124-125
    // order), featp at the search position.  Codes of a ring whose features were dropped (capacity flags) are
    // ignored through the ring counts.
    const int npos = rs[nr];
    if (blockIdx.x == 0 && threadIdx.x == 0) ev.n_pos[b] = npos;
    const int* qc = ev.qcode + (size_t)b * ev.raw_stride;
    int* qs = ev.qslot + (size_t)b * ev.raw_stride;
    int* fs = ev.fslot + (size_t)b * ev.feat_stride;
    float4* fp = ev.featp + (size_t)b * ev.feat_stride;
    float4* feat = ev.feat + (size_t)b * ev.feat_stride;
    int* fsrc = ev.feat_src + (size_t)b * ev.feat_stride;
    const float4* rp = ev.ring_pts + (size_t)b * ev.raw_stride;
    const int* rsrc = ev.ring_src + (size_t)b * ev.raw_stride;
    for (int p = blockIdx.x * 256 + threadIdx.x; p < npos; p += gridDim.x * 256) {
        const int code = qc[p];
        int slot = -1, o = -1;
        if (code >= 0) {
            int lo = 0, hi = nr - 1;  // last ring with rs[r] <= p
            while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (rs[mid] <= p) lo = mid; else hi = mid - 1; }
            const int l = code & kQCodeMask, rank = (code >> kQRankShift) & kQCodeMask;
            if (code & kQSurf) {
                if (l < spre[lo + 1] - spre[lo]) { slot = ne + spre[lo] + l; o = ne + spre[lo] + rank; }
            } else if (l < epre[lo + 1] - epre[lo]) {
                slot = epre[lo] + l;
                o = epre[lo] + rank;
            }
        }
        qs[p] = slot;
        if (slot >= 0 && slot < ev.feat_stride) {
            const float4 q = rp[p];
            feat[slot] = q;
            fsrc[slot] = rsrc[p];
            if (o < ev.feat_stride) {
                fs[o] = slot;
                fp[o] = make_float4(q.x, q.y, q.z, __int_as_float(slot));
            }
        }
    }
}

// concat_kernel's placement with one workgroup per (sector, ring, scan) (LMSF_CONCAT_SECTOR, A/B): a sector's edge
// picks and its surfs each occupy one contiguous range of the ring's emission order (the greedy pick and the surf
// compaction run sector by sector), so the block stages the sector's points in LDS by their emission index and
// writes feat / feat_src as contiguous runs -- where the grid-stride form stores every point to its slot, a wave's
// 64 stores spread over the sector's curvature permutation.  The search-order outputs (fslot / featp, by rank:
// ring order) and qslot (by position) are written directly.  Results are the same placements.
#ifndef LMSF_CONCAT_SECTOR
#define LMSF_CONCAT_SECTOR 1
#endif
constexpr int kCatPer = kSortMax / 256;   // positions per thread (a sector holds at most kSortMax)
constexpr int kCatStage = 1024;           // surfs staged per sector (larger sectors store the rest directly)
__global__ __launch_bounds__(256) void concat_sector_kernel(ExtractView ev) {
    __shared__ float4 s_pt[kCatStage];
    __shared__ int s_src[kCatStage];
    __shared__ float4 e_pt[64];
    __shared__ int e_src[64];
    __shared__ int s_min[2], s_cnt[2];   // [0] edges, [1] surfs: smallest emission index and count in the sector
    __shared__ int pre[4];               // epre[r], epre[r + 1], spre[r], spre[r + 1]
    __shared__ int tot[2];               // ne, ns of the scan
    const int r = blockIdx.x / 6, k = blockIdx.x % 6, b = blockIdx.y;
    const int nr = ev.n_scans;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int* rs = ev.ring_start + (size_t)b * (kMaxRings + 1);
    if (r >= nr) return;
    const int start = rs[r], size = rs[r + 1] - start;
    // this ring's prefixes and the scan's totals: the edge / surf counts of the rings before r (wave 0 / wave 1)
    if (wave < 2) {
        const int* cnt = (wave == 0 ? ev.ring_edge_cnt : ev.ring_surf_cnt) + (size_t)b * kMaxRings;
        int below = 0, all = 0, mine = 0;
        for (int r0 = lane; r0 < nr; r0 += 64) {
            const int c = cnt[r0];
            all += c;
            below += r0 < r ? c : 0;
            mine += r0 == r ? c : 0;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            below += __shfl_xor(below, o, 64);
            all += __shfl_xor(all, o, 64);
            mine += __shfl_xor(mine, o, 64);
        }
        if (lane == 0) {
            pre[2 * wave] = below;
            pre[2 * wave + 1] = below + mine;
            tot[wave] = all;
            s_min[wave] = INT_MAX;
            s_cnt[wave] = 0;
        }
    }
    __syncthreads();
    const int ne = tot[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ev.n_edge[b] = tot[0];
        ev.n_surf[b] = tot[1];
        ev.n_pos[b] = rs[nr];
    }
    int* qs = ev.qslot + (size_t)b * ev.raw_stride + start;
    // positions outside the sectors (and whole rings the features kernel skipped) hold no feature
    bool ring_ok = size >= 20 && size <= kRingMax;
    int s0 = 0, n = 0;
    if (ring_ok) {   // ring_features_kernel's bound: a ring whose first or last sector exceeds kSortMax has no features
        int a0, n0, a5, n5;
        sector_bounds(size, 0, a0, n0);
        sector_bounds(size, 5, a5, n5);
        ring_ok = n0 <= kSortMax && n5 <= kSortMax;
        sector_bounds(size, k, s0, n);
    }
    if (!ring_ok) {
        if (k == 0)
            for (int j = threadIdx.x; j < size; j += 256) qs[j] = -1;
        return;
    }
    if (k == 0)
        for (int j = threadIdx.x; j < s0; j += 256) qs[j] = -1;
    if (k == 5)
        for (int j = s0 + n + threadIdx.x; j < size; j += 256) qs[j] = -1;
    const int* qc = ev.qcode + (size_t)b * ev.raw_stride + start + s0;
    const float4* rp = ev.ring_pts + (size_t)b * ev.raw_stride + start + s0;
    const int* rsrc = ev.ring_src + (size_t)b * ev.raw_stride + start + s0;
    int code[kCatPer];
    int mn[2] = {INT_MAX, INT_MAX}, ct[2] = {0, 0};
#pragma unroll
    for (int u = 0; u < kCatPer; ++u) {
        const int i = threadIdx.x + 256 * u;
        code[u] = i < n ? qc[i] : -1;
        if (code[u] >= 0) {
            const int kind = (code[u] & kQSurf) ? 1 : 0;
            mn[kind] = min(mn[kind], code[u] & kQCodeMask);
            ++ct[kind];
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {   // per wave, then one LDS atomic per wave and kind
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            mn[d] = min(mn[d], __shfl_xor(mn[d], o, 64));
            ct[d] += __shfl_xor(ct[d], o, 64);
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            if (ct[d]) {
                atomicMin(&s_min[d], mn[d]);
                atomicAdd(&s_cnt[d], ct[d]);
            }
        }
    }
    __syncthreads();
    int* fs = ev.fslot + (size_t)b * ev.feat_stride;
    float4* fp = ev.featp + (size_t)b * ev.feat_stride;
    const int ecap = pre[1] - pre[0], scap = pre[3] - pre[2];   // the ring's kept counts (capacity drops)
#pragma unroll
    for (int u = 0; u < kCatPer; ++u) {
        const int i = threadIdx.x + 256 * u;
        if (i >= n) continue;
        const int c = code[u];
        int slot = -1;
        if (c >= 0) {
            const bool surf = (c & kQSurf) != 0;
            const int l = c & kQCodeMask, rank = (c >> kQRankShift) & kQCodeMask;
            const float4 q = rp[i];
            const int src = rsrc[i];
            int o = -1;
            if (surf) {
                if (l < scap) { slot = ne + pre[2] + l; o = ne + pre[2] + rank; }
                if (l - s_min[1] < kCatStage) {
                    s_pt[l - s_min[1]] = q;
                    s_src[l - s_min[1]] = src;
                } else if (slot >= 0 && slot < ev.feat_stride) {   // beyond the staging: stored directly
                    ev.feat[(size_t)b * ev.feat_stride + slot] = q;
                    ev.feat_src[(size_t)b * ev.feat_stride + slot] = src;
                }
            } else {
                if (l < ecap) { slot = pre[0] + l; o = pre[0] + rank; }
                if (l - s_min[0] < 64) {
                    e_pt[l - s_min[0]] = q;
                    e_src[l - s_min[0]] = src;
                }
            }
            if (slot >= 0 && slot < ev.feat_stride && o < ev.feat_stride) {
                fs[o] = slot;
                fp[o] = make_float4(q.x, q.y, q.z, __int_as_float(slot));
            }
        }
        qs[s0 + i] = slot;
    }
    __syncthreads();
    float4* feat = ev.feat + (size_t)b * ev.feat_stride;
    int* fsrc = ev.feat_src + (size_t)b * ev.feat_stride;
    for (int j = threadIdx.x; j < min(s_cnt[1], kCatStage); j += 256) {   // the sector's surfs: s_min .. + count
        const int l = s_min[1] + j;
        const int slot = ne + pre[2] + l;
        if (l < scap && slot < ev.feat_stride) {
            feat[slot] = s_pt[j];
            fsrc[slot] = s_src[j];
        }
    }
    for (int j = threadIdx.x; j < min(s_cnt[0], 64); j += 256) {
        const int l = s_min[0] + j;
        const int slot = pre[0] + l;
        if (l < ecap && slot < ev.feat_stride) {
            feat[slot] = e_pt[j];
            fsrc[slot] = e_src[j];
        }
    }
}

hipError_t launch_extract(const ExtractView& ev, hipStream_t s) {
    hipLaunchKernelGGL(ring_count_kernel, dim3(ev.n_tiles, ev.B), dim3(256), 0, s, ev);
    hipLaunchKernelGGL(ring_offsets_kernel, dim3(ev.B), dim3(256), 0, s, ev);
    if (LMSF_SCATTER_LDS && ev.n_scans > kScatterLdsRings)
        hipLaunchKernelGGL(ring_scatter_kernel<true>, dim3(ev.n_tiles, ev.B), dim3(256), 0, s, ev);
    else
        hipLaunchKernelGGL(ring_scatter_kernel<false>, dim3(ev.n_tiles, ev.B), dim3(256), 0, s, ev);
    hipLaunchKernelGGL(sector_sort_kernel, dim3(ev.n_scans * 6, ev.B), dim3(256), 0, s, ev);
    hipLaunchKernelGGL(ring_features_kernel, dim3(ev.n_scans, ev.B), dim3(256), 0, s, ev);
    // blocks per scan (LMSF_CONCAT_BLOCKS, A/B; default 256: ~one feature and one position per thread)
    static const int cmax = [] {
        const int v = ab_int("LMSF_CONCAT_BLOCKS", 256);
        return v >= 1 && v <= 1024 ? v : 256;
    }();
    const int cblocks = min(cmax, (ev.raw_stride + 255) / 256);
    if (LMSF_CONCAT_SECTOR)
        hipLaunchKernelGGL(concat_sector_kernel, dim3(ev.n_scans * 6, ev.B), dim3(256), 0, s, ev);
    else
        hipLaunchKernelGGL(concat_kernel, dim3(max(cblocks, 1), ev.B), dim3(256), 0, s, ev);
    return hipGetLastError();
}

}  // namespace lmsf
