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
//   sector_sort  one workgroup per (sector, ring): curvature + register-resident bitonic sort
//   ring_features one workgroup per ring: automaton (wave-ballot walk), then per sector in order
//                 {wave-ballot greedy pick over the sorted list, block-scan compaction}
//   concat       per scan: edges (ring order) then surfs (ring order) into the feature array
#include <hip/hip_runtime.h>
#include <math.h>

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

// Stable multisplit of one tile into ring order (input order preserved inside each ring).
__global__ __launch_bounds__(256) void ring_scatter_kernel(ExtractView ev) {
    __shared__ int wcnt[4][kMaxRings];
    __shared__ int running[kMaxRings];
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
    for (int c0 = 0; c0 < kTile; c0 += 256) {
        for (int k = threadIdx.x; k < 4 * kMaxRings; k += 256) wcnt[k / kMaxRings][k % kMaxRings] = 0;
        __syncthreads();
        const int i = t * kTile + c0 + threadIdx.x;
        const int r = i < n ? (int)rid[i] : -1;
        const float4 pt = r >= 0 ? raw[i] : make_float4(0, 0, 0, 0);   // in flight across the rank pass
        int rank = 0;
        unsigned long long remaining = __ballot(r >= 0);
        while (remaining) {
            const int leader = __ffsll((long long)remaining) - 1;
            const int rl = __shfl(r, leader, 64);
            const unsigned long long m = __ballot(r == rl);
            if (r == rl) rank = __popcll(m & lanemask_lt(lane));
            if (lane == leader) wcnt[wave][rl] = __popcll(m);
            remaining &= ~m;
        }
        __syncthreads();
        if (r >= 0) {
            int base = running[r];
            for (int w = 0; w < wave; ++w) base += wcnt[w][r];
            const int dst = toff[(size_t)r * ev.n_tiles + t] + base + rank;
            out[dst] = pt;
            osrc[dst] = i;
        }
        __syncthreads();
        for (int rr = threadIdx.x; rr < ev.n_scans; rr += 256)
            running[rr] += wcnt[0][rr] + wcnt[1][rr] + wcnt[2][rr] + wcnt[3][rr];
        __syncthreads();
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
        for (int j = 5 + tid; j <= jmax; j += NT) {
            const float4 a = pts[j], c = pts[j + 1];
            const double angle_curr = ref_atan2(a.x, a.y, ev.libm_float);   // atan2(x, y) order (FX:223-224)
            const double angle_after = ref_atan2(c.x, c.y, ev.libm_float);
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
        __syncthreads();
        // sequential skip automaton (next j = j + 5 after event 1 / 2, else j + 1), 64 at a time
        if (tid < 64) {
            int pos = 5;
            while (pos <= jmax) {
                const int j = pos + lane;
                const int e = j <= jmax ? (int)flag[j] : 0;
                const unsigned long long m = __ballot(e == 1 || e == 2);
                const int f = m ? (__ffsll((long long)m) - 1) : 64;
                if (lane < f && e == 3) {
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
                pos = m ? pos + f + 5 : pos + 64;
            }
        }
        __syncthreads();
        for (int j = tid; j < size; j += NT) flag[j] = 0;   // reuse as is_edge
        __syncthreads();
    }
}

// Bitonic sort of npow (key, index) pairs ascending by (key, index), keys/indices in LDS on entry
// and exit.  Elements live in registers: wave w owns positions [w * 64E, (w + 1) * 64E), lane l
// holds w * 64E + e * 64 + l (e < E).  A compare-exchange at distance jj < 64 is a lane shuffle,
// 64 <= jj < 64E a swap inside the thread, and only jj >= 64E crosses waves (LDS + barrier):
// 2 of the 55 stages of a 1024-element sort with E = 4, instead of 55 barrier stages.
template <int E>
__device__ void bitonic_sort_regs(double* key, int* kidx, int npow) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int chunk = 64 * E;
    const bool active = w * chunk < npow;
    double k[E];
    int id[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = w * chunk + e * 64 + lane;
        k[e] = active ? key[i] : 0.0;
        id[e] = active ? kidx[i] : 0;
    }
    for (int kk = 2; kk <= npow; kk <<= 1) {
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            if (jj >= chunk) {                         // partner in another wave: through LDS
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
                if (active) {
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int i = w * chunk + e * 64 + lane, ixj = i ^ jj;
                        const double ko = key[ixj];
                        const int io = kidx[ixj];
                        const bool lower = i < ixj;
                        const double ka = lower ? k[e] : ko, kb = lower ? ko : k[e];
                        const int ia = lower ? id[e] : io, ib = lower ? io : id[e];
                        const bool a_gt_b = ka > kb || (ka == kb && ia > ib);
                        const bool up = (i & kk) == 0;
                        if (up == a_gt_b) { k[e] = ko; id[e] = io; }
                    }
                }
            } else if (jj >= 64) {                     // same thread, another register
                const int ej = jj >> 6;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int e2 = e ^ ej;
                    if (e2 > e) {
                        const int i = w * chunk + e * 64 + lane;
                        const bool a_gt_b = k[e] > k[e2] || (k[e] == k[e2] && id[e] > id[e2]);
                        const bool up = (i & kk) == 0;
                        if (up == a_gt_b) {
                            const double tk = k[e]; k[e] = k[e2]; k[e2] = tk;
                            const int ti = id[e]; id[e] = id[e2]; id[e2] = ti;
                        }
                    }
                }
            } else {                                   // same register, another lane
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int i = w * chunk + e * 64 + lane;
                    const double ko = __shfl_xor(k[e], jj, 64);
                    const int io = __shfl_xor(id[e], jj, 64);
                    const bool lower = (lane & jj) == 0;
                    const double ka = lower ? k[e] : ko, kb = lower ? ko : k[e];
                    const int ia = lower ? id[e] : io, ib = lower ? io : id[e];
                    const bool a_gt_b = ka > kb || (ka == kb && ia > ib);
                    const bool up = (i & kk) == 0;
                    if (up == a_gt_b) { k[e] = ko; id[e] = io; }
                }
            }
        }
    }
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
    __shared__ double key[kSortMax];
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
    int npow = 1;
    while (npow < n) npow <<= 1;
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
            key[i] = dx * dx + dy * dy + dz * dz;
            kidx[i] = j;
        } else {
            key[i] = __builtin_huge_val();
            kidx[i] = 0x7fffffff;
        }
    }
    __syncthreads();
    if (npow <= 256) bitonic_sort_regs<1>(key, kidx, npow);
    else if (npow <= 512) bitonic_sort_regs<2>(key, kidx, npow);
    else if (npow <= 1024) bitonic_sort_regs<4>(key, kidx, npow);
    else bitonic_sort_regs<8>(key, kidx, npow);
    double* okey = ev.sort_key + (size_t)b * ev.raw_stride + start + s0;
    int* oidx = ev.sort_idx + (size_t)b * ev.raw_stride + start + s0;
    for (int i = threadIdx.x; i < n; i += 256) {
        okey[i] = key[i];
        oidx[i] = kidx[i];
    }
}

// One workgroup per (ring, scan): bad-point automaton, then per sector in order the greedy edge
// pick over the pre-sorted curvature list and the surf compaction.
__global__ __launch_bounds__(256) void ring_features_kernel(ExtractView ev) {
    __shared__ uint8_t dis[kRingMax];
    __shared__ uint8_t flag[kRingMax];
    __shared__ double key[kSortMax];
    __shared__ int kidx[kSortMax];
    __shared__ int scan_part[256];
    __shared__ int pick[20];
    __shared__ int sh_ec, sh_sc, sh_err;
    constexpr int kSurfPer = 3;   // sector points per thread held in registers by the surf compaction
    const int r = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63;
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
    const int* psrc = ev.ring_src + (size_t)b * ev.raw_stride + start;
    for (int j = tid; j < size; j += 256) { dis[j] = 0; flag[j] = 0; qc[j] = -1; }
    if (tid == 0) { sh_ec = 0; sh_sc = 0; sh_err = 0; }
    __syncthreads();
    ring_bad_points<256>(ev, pts, size, dis, flag);
    const double thresh = (double)ev.edge_thresh;
    float4* estage = ev.edge_stage + ((size_t)b * kMaxRings + r) * kEdgePerRing;
    int* estage_src = ev.edge_stage_src + ((size_t)b * kMaxRings + r) * kEdgePerRing;
    float4* sstage = ev.surf_stage + (size_t)b * ev.raw_stride + start;
    int* sstage_src = ev.surf_stage_src + (size_t)b * ev.raw_stride + start;
    for (int k = 0; k < 6; ++k) {
        int s0, n;
        sector_bounds(size, k, s0, n);
        if (n > kSortMax) {
            if (tid == 0) { atomicOr(ev.error, 2); sh_err = 1; }
            break;
        }
        const double* skey = ev.sort_key + (size_t)b * ev.raw_stride + start + s0;
        const int* sidx = ev.sort_idx + (size_t)b * ev.raw_stride + start + s0;
        for (int i = tid; i < n; i += 256) {
            key[i] = skey[i];
            kidx[i] = sidx[i];
        }
        __syncthreads();
        // greedy edge pick, largest curvature first (FX:157-195), one wave
        if (tid < 64) {
            int pos = n - 1, picked = 0, ec = sh_ec;
            while (pos >= 0) {
                const int cand = pos - lane;
                const bool elig = cand >= 0 && dis[kidx[cand]] == 0;
                const unsigned long long m = __ballot(elig);
                if (!m) { pos -= 64; continue; }
                const int f = __ffsll((long long)m) - 1;
                const double c = key[pos - f];
                const int ind = kidx[pos - f];
                if (c <= thresh) break;
                ++picked;
                if (picked > 20) break;
                if (lane == 0) {
                    pick[picked - 1] = ind;   // staged after the loop: no load -> store round trip per pick
                    flag[ind] = 1;
                    qc[ind] = ec;
                }
                if (lane >= 1 && lane <= 5) dis[min(ind + lane, size - 1)] = 1;
                if (lane >= 6 && lane <= 10) dis[max(ind - (lane - 5), 0)] = 1;
                ++ec;
                pos = pos - f - 1;
            }
            if (lane == 0) sh_ec = ec;
            const int ec0 = ec - min(picked, 20);
            for (int t = lane; t < ec - ec0; t += 64) {
                const int ind = pick[t];
                estage[ec0 + t] = pts[ind];
                estage_src[ec0 + t] = psrc[ind];
            }
        }
        __syncthreads();
        // surf: every sector point not picked as edge, ascending curvature (FX:197-206);
        // contiguous chunk per thread, block prefix from wave scans
        const int per = (n + 255) / 256;
        const int lo = tid * per, hi = min(lo + per, n);
        int cntv = 0;
        for (int i = lo; i < hi; ++i) cntv += flag[kidx[i]] == 0;
        int incl = cntv;
#pragma unroll
        for (int o2 = 1; o2 < 64; o2 <<= 1) {
            const int t = __shfl_up(incl, o2, 64);
            if (lane >= o2) incl += t;
        }
        if (lane == 63) scan_part[tid >> 6] = incl;
        __syncthreads();
        int wbase = 0;
        for (int w2 = 0; w2 < (tid >> 6); ++w2) wbase += scan_part[w2];
        int o = sh_sc + wbase + incl - cntv;
        if (per <= kSurfPer) {   // every point load in flight before the first store
            int ind[kSurfPer];
            float4 sp[kSurfPer];
            int ss[kSurfPer];
#pragma unroll
            for (int u = 0; u < kSurfPer; ++u) {
                const int i = lo + u;
                ind[u] = i < hi && flag[kidx[i]] == 0 ? kidx[i] : -1;
                if (ind[u] >= 0) {
                    sp[u] = pts[ind[u]];
                    ss[u] = psrc[ind[u]];
                }
            }
#pragma unroll
            for (int u = 0; u < kSurfPer; ++u) {
                if (ind[u] >= 0) {
                    sstage[o] = sp[u];
                    sstage_src[o] = ss[u];
                    qc[ind[u]] = kQSurf | o;
                    ++o;
                }
            }
        } else {
            for (int i = lo; i < hi; ++i) {
                const int ind1 = kidx[i];
                if (flag[ind1] == 0) {
                    sstage[o] = pts[ind1];
                    sstage_src[o] = psrc[ind1];
                    qc[ind1] = kQSurf | o;
                    ++o;
                }
            }
        }
        __syncthreads();
        if (tid == 255) sh_sc = o;  // thread 255's running offset is the sector's total
        __syncthreads();
    }
    if (tid == 0) {
        ecnt[r] = sh_err ? 0 : sh_ec;
        scnt[r] = sh_err ? 0 : sh_sc;
    }
}

// Concatenate per-ring stages: edges of ring 0..N-1, then surfs of ring 0..N-1 (FX:124-125 order).
__global__ __launch_bounds__(256) void concat_kernel(ExtractView ev) {
    __shared__ int epre[kMaxRings + 1], spre[kMaxRings + 1];
    const int b = blockIdx.y;
    const int nr = ev.n_scans;
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
    const int ne = epre[nr], ns = spre[nr];
    const int* rs = ev.ring_start + (size_t)b * (kMaxRings + 1);
    float4* feat = ev.feat + (size_t)b * ev.feat_stride;
    int* fsrc = ev.feat_src + (size_t)b * ev.feat_stride;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < ne + ns; i += gridDim.x * 256) {
        if (i < ne) {
            int lo = 0, hi = nr - 1;  // last ring with epre[r] <= i
            while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (epre[mid] <= i) lo = mid; else hi = mid - 1; }
            const size_t src = ((size_t)b * kMaxRings + lo) * kEdgePerRing + (i - epre[lo]);
            feat[i] = ev.edge_stage[src];
            fsrc[i] = ev.edge_stage_src[src];
        } else {
            const int k = i - ne;
            int lo = 0, hi = nr - 1;
            while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (spre[mid] <= k) lo = mid; else hi = mid - 1; }
            const size_t src = (size_t)b * ev.raw_stride + rs[lo] + (k - spre[lo]);
            feat[i] = ev.surf_stage[src];
            fsrc[i] = ev.surf_stage_src[src];
        }
    }
    // The neighbour search's order: the feature slot of every ring position, so that neighbouring
    // lanes search neighbouring points of a ring (slot order puts a sector's surfs in curvature
    // order, spread over ~60 degrees of the ring).  Codes of a ring whose features were dropped
    // (capacity flags) are ignored through the ring counts.
    const int npos = rs[nr];
    if (blockIdx.x == 0 && threadIdx.x == 0) ev.n_pos[b] = npos;
    const int* qc = ev.qcode + (size_t)b * ev.raw_stride;
    int* qs = ev.qslot + (size_t)b * ev.raw_stride;
    for (int p = blockIdx.x * 256 + threadIdx.x; p < npos; p += gridDim.x * 256) {
        int lo = 0, hi = nr - 1;  // last ring with rs[r] <= p
        while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (rs[mid] <= p) lo = mid; else hi = mid - 1; }
        const int code = qc[p];
        int slot = -1;
        if (code >= 0) {
            const int l = code & ~kQSurf;
            if (code & kQSurf) {
                if (l < spre[lo + 1] - spre[lo]) slot = ne + spre[lo] + l;
            } else if (l < epre[lo + 1] - epre[lo]) {
                slot = epre[lo] + l;
            }
        }
        qs[p] = slot;
    }
}

// Stable partition of the search order by kind: fslot = the valid entries of qslot, edge slots
// (slot < n_edge) first, each kind in ring order (the fused search + fit order: neighbouring lanes
// search neighbouring ring points, and a wave runs one fit kind).  One block per (ring, slot): a
// ring's valid positions are exactly its ring_edge_cnt edges and ring_surf_cnt surfs (concat_kernel),
// so ring r writes edges from epre[r] and surfs from n_edge + spre[r]; inside the ring a block-wide
// exclusive scan of the packed (edge, surf) counts (16 bits each) of 8 consecutive positions per
// thread, 2048 positions per chunk.
__global__ __launch_bounds__(256) void order_kernel(ExtractView ev) {
    constexpr int E = 8;
    __shared__ uint32_t wsum[4];
    __shared__ int pre[2];
    const int r = blockIdx.x, b = blockIdx.y;
    const int nr = ev.n_scans;
    if (threadIdx.x < 64) {   // one wave: ring-count prefixes below r
        int e = 0, sc = 0;
        for (int k = threadIdx.x; k < r; k += 64) {
            e += ev.ring_edge_cnt[(size_t)b * kMaxRings + k];
            sc += ev.ring_surf_cnt[(size_t)b * kMaxRings + k];
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            e += __shfl_xor(e, o, 64);
            sc += __shfl_xor(sc, o, 64);
        }
        if (threadIdx.x == 0) { pre[0] = e; pre[1] = sc; }
    }
    __syncthreads();
    if (r >= nr) return;
    const int ne = ev.n_edge[b];
    const int* rs = ev.ring_start + (size_t)b * (kMaxRings + 1);
    const int p0 = rs[r], p1 = rs[r + 1];
    const int* qs = ev.qslot + (size_t)b * ev.raw_stride;
    int* fs = ev.fslot + (size_t)b * ev.feat_stride;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t base_e = (uint32_t)pre[0], base_s = (uint32_t)(ne + pre[1]);
    for (int c0 = p0; c0 < p1; c0 += 256 * E) {
        int v[E];
        uint32_t cnt = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int p = c0 + threadIdx.x * E + e;
            v[e] = p < p1 ? qs[p] : -1;
            if (v[e] >= 0) cnt += v[e] < ne ? 1u : 0x10000u;
        }
        uint32_t x = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t wpre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t t = wsum[w];
            wpre += w < wave ? t : 0u;
            tot += t;
        }
        const uint32_t ex = wpre + x - cnt;
        uint32_t oe = base_e + (ex & 0xffffu), os = base_s + (ex >> 16);
        // all E feature loads first, then the stores (a load after a store to featp, which the compiler
        // cannot prove distinct from feat, would wait for it: E serial round trips per chunk)
        uint32_t o[E];
        float4 f[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            o[e] = v[e] < 0 ? 0xffffffffu : (v[e] < ne ? oe++ : os++);
            f[e] = o[e] < (uint32_t)ev.feat_stride ? ev.feat[(size_t)b * ev.feat_stride + v[e]] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (o[e] < (uint32_t)ev.feat_stride) {
                fs[o[e]] = v[e];
                ev.featp[(size_t)b * ev.feat_stride + o[e]] = make_float4(f[e].x, f[e].y, f[e].z, __int_as_float(v[e]));
            }
        }
        base_e += tot & 0xffffu;
        base_s += tot >> 16;
        __syncthreads();   // wsum is rewritten by the next chunk
    }
}

hipError_t launch_extract(const ExtractView& ev, hipStream_t s) {
    hipLaunchKernelGGL(ring_count_kernel, dim3(ev.n_tiles, ev.B), dim3(256), 0, s, ev);
    hipLaunchKernelGGL(ring_offsets_kernel, dim3(ev.B), dim3(256), 0, s, ev);
    hipLaunchKernelGGL(ring_scatter_kernel, dim3(ev.n_tiles, ev.B), dim3(256), 0, s, ev);
    hipLaunchKernelGGL(sector_sort_kernel, dim3(ev.n_scans * 6, ev.B), dim3(256), 0, s, ev);
    hipLaunchKernelGGL(ring_features_kernel, dim3(ev.n_scans, ev.B), dim3(256), 0, s, ev);
    // blocks per scan (LMSF_CONCAT_BLOCKS, A/B; default 256: ~one feature and one position per thread)
    static const int cmax = [] {
        const int v = ab_int("LMSF_CONCAT_BLOCKS", 256);
        return v >= 1 && v <= 1024 ? v : 256;
    }();
    const int cblocks = min(cmax, (ev.raw_stride + 255) / 256);
    hipLaunchKernelGGL(concat_kernel, dim3(max(cblocks, 1), ev.B), dim3(256), 0, s, ev);
    hipLaunchKernelGGL(order_kernel, dim3(ev.n_scans, ev.B), dim3(256), 0, s, ev);
    return hipGetLastError();
}

}  // namespace lmsf
