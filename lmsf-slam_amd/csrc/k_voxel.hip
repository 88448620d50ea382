// Voxel-grid downsampling (pcl::VoxelGrid, INC/Algorithm/PointClouds/processing/Filter/voxel_grid.hpp:25-34
// via Algorithm::VoxelGridFilter::Filter, filter_base.hpp:34-45), used by the build-defined
// "sliding_Localmap" (the window of keyframes is downsampled per feature kind) and
// exported as lmsf_voxel_filter.
//
// PCL semantics kept: voxel = (int)floor(p * (1/leaf)) in float; voxels emitted in ascending
// linear index (x fastest, then y, then z, relative to the minimum voxel); each output point is
// the centroid of every field of the voxel's points; when div_x*div_y*div_z exceeds INT32_MAX
// PCL refuses ("integer indices would overflow") and returns the input unchanged -- so does this.
// PCL accumulates the centroid in float in std::sort order (unspecified inside a voxel); here the
// sort is a stable radix sort (ties by input index) and sums are double -> deterministic, and the
// CPU oracle (oracle/voxel.cpp) reproduces it bit for bit.
//
// Roofline: HBM-bound byte work (two reads of the cloud for the box and the keys, 4 B keys written and
// 8 B pairs radix-sorted per digit pass, one gather of 16 B per point, 16 B per voxel out) -- at tracker
// window sizes (<1e6 points) latency- and launch-bound instead.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <climits>

#include "lmsf_internal.h"
#include "radix.h"

namespace lmsf {

// A one-workgroup variant for small clouds (box, keys, LDS bitonic sort of (key, index), heads, sums in one
// launch instead of ~13) was bit-exact but slower on the tracker's ~4.5k-point edge window: C4 1.65-1.89
// vs 1.55-1.85 ms/scan, C3 1.68-1.72 vs 1.58-1.62 ms/frame (91 barrier-separated sort stages): removed.
// hipCUB's SortPairs (merge sort below 2^20 items, ~20 launches) and rocprim onesweep (4 x ~25 us + 8
// look-back resets on a ~6e5-point surf window) were replaced by k_sort.hip (r03).
//
// Launches per filter: box partials, keys + digit histograms, the digit passes (radix.h: only those the key
// bound needs run), segments + centroids in one single pass -- 7 (was ~20).  No atomics on shared
// words for the box: each box block writes its partial, and every key block reduces the (L2-resident) partials.

constexpr int kVoxBatch = 8;   // points in flight per thread (independent loads: one memory latency per batch)

__device__ __forceinline__ int vox_coord(float v, float inv) {
    return (int)fminf(fmaxf(floorf(v * inv), -1073741824.f), 1073741824.f);
}

// Map cell of a point (k_map.hip's map_bbox_kernel / map_count_kernel rule): x-slice, row, level.
__device__ __forceinline__ int map_coord(float v, float scale) {
    return (int)fminf(fmaxf(floorf(v * scale), -1073741824.f), 1073741824.f);
}

// part[block][12] = voxel box (lo xyz, hi xyz), map-cell box (lo, hi) of the block's points; block 0 also
// clears the sort's histograms and tile counters for the launches that follow.
__global__ void __launch_bounds__(256) voxel_box_kernel(const float4* pts, int n, float inv, float sx, int* part,
                                                        uint32_t* hist, uint32_t* ctr) {
    if (blockIdx.x == 0) {
        for (int i = threadIdx.x; i < kRadixPasses * kRadixDigits; i += 256) hist[i] = 0u;
        if (threadIdx.x < 16) ctr[threadIdx.x] = 0u;
    }
    int lo[6], hi[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        lo[d] = INT_MAX;
        hi[d] = INT_MIN;
    }
    const int stride = gridDim.x * 256 * kVoxBatch;
    for (int i0 = blockIdx.x * 256 * kVoxBatch + threadIdx.x; i0 < n; i0 += stride) {
        float4 p[kVoxBatch];
#pragma unroll
        for (int u = 0; u < kVoxBatch; ++u) p[u] = pts[min(i0 + u * 256, n - 1)];   // repeats leave the box unchanged
#pragma unroll
        for (int u = 0; u < kVoxBatch; ++u) {
            const int c[6] = {vox_coord(p[u].x, inv), vox_coord(p[u].y, inv), vox_coord(p[u].z, inv),
                              map_coord(p[u].x, sx), map_coord(p[u].y, 1.f), map_coord(p[u].z, 1.f)};
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                lo[d] = min(lo[d], c[d]);
                hi[d] = max(hi[d], c[d]);
            }
        }
    }
    __shared__ int s_lo[6][4], s_hi[6][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 0; d < 6; ++d) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            lo[d] = min(lo[d], __shfl_xor(lo[d], o, 64));
            hi[d] = max(hi[d], __shfl_xor(hi[d], o, 64));
        }
        if (lane == 0) {
            s_lo[d][w] = lo[d];
            s_hi[d][w] = hi[d];
        }
    }
    __syncthreads();
    if (threadIdx.x < 12) {
        const int d = threadIdx.x % 6;
        const bool is_hi = threadIdx.x >= 6;
        int v = is_hi ? INT_MIN : INT_MAX;
        for (int k = 0; k < 4; ++k) v = is_hi ? max(v, s_hi[d][k]) : min(v, s_lo[d][k]);
        // layout: vox lo xyz, vox hi xyz, map lo xyz, map hi xyz
        part[blockIdx.x * 12 + (d < 3 ? (is_hi ? 3 : 0) + d : 6 + (is_hi ? 3 : 0) + d - 3)] = v;
    }
}

// The box of all partials into box[12] (every thread of the block gets it through LDS).
__device__ __forceinline__ void reduce_box(const int* part, int nparts, int* s_box) {
    int v[12];
#pragma unroll
    for (int d = 0; d < 12; ++d) v[d] = (d % 6) < 3 ? INT_MAX : INT_MIN;
    for (int b = threadIdx.x; b < nparts; b += blockDim.x) {
#pragma unroll
        for (int d = 0; d < 12; ++d) {
            const int x = part[b * 12 + d];
            v[d] = (d % 6) < 3 ? min(v[d], x) : max(v[d], x);
        }
    }
#pragma unroll
    for (int d = 0; d < 12; ++d) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const int x = __shfl_xor(v[d], o, 64);
            v[d] = (d % 6) < 3 ? min(v[d], x) : max(v[d], x);
        }
    }
    __shared__ int s_w[12][16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int d = 0; d < 12; ++d) s_w[d][w] = v[d];
    __syncthreads();
    if (threadIdx.x < 12) {
        const int d = threadIdx.x;
        int x = s_w[d][0];
        for (int k = 1; k < nw; ++k) x = (d % 6) < 3 ? min(x, s_w[d][k]) : max(x, s_w[d][k]);
        s_box[d] = x;
    }
    __syncthreads();
}

// Linear voxel keys (x fastest, relative to the minimum voxel) and the digit histograms of the passes the
// key bound needs.  When div_x*div_y*div_z exceeds INT32_MAX PCL refuses and returns the input unchanged:
// every point then gets its own key (its index), so each "voxel" is one point and the centroid pass
// reproduces the input exactly.  Block 0 publishes the key bound and, for the tracker, the map-cell box.
__global__ void __launch_bounds__(256) voxel_key_kernel(const float4* pts, int n, float inv, const int* part,
                                                        int nparts, uint32_t* keys, uint32_t* bound, uint32_t* hist,
                                                        int* map_bb) {
    __shared__ int s_box[12];
    __shared__ uint32_t s_h[kRadixPasses][kRadixDigits];
    for (int i = threadIdx.x; i < kRadixPasses * kRadixDigits; i += 256) (&s_h[0][0])[i] = 0u;
    reduce_box(part, nparts, s_box);
    const int64_t dx = (int64_t)s_box[3] - s_box[0] + 1, dy = (int64_t)s_box[4] - s_box[1] + 1,
                  dz = (int64_t)s_box[5] - s_box[2] + 1;
    const bool overflow = dx * dy * dz > (int64_t)INT32_MAX;
    const uint32_t bnd = overflow ? (uint32_t)n : (uint32_t)(dx * dy * dz);
    const int passes = radix_pass_count(bnd);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *bound = bnd;
        if (map_bb)
            for (int d = 0; d < 6; ++d) map_bb[d] = s_box[6 + d];
    }
    const int stride = gridDim.x * 256 * kVoxBatch;
    for (int i0 = blockIdx.x * 256 * kVoxBatch + threadIdx.x; i0 < n; i0 += stride) {
        float4 p[kVoxBatch];
#pragma unroll
        for (int u = 0; u < kVoxBatch; ++u) p[u] = pts[min(i0 + u * 256, n - 1)];
#pragma unroll
        for (int u = 0; u < kVoxBatch; ++u) {
            const int i = i0 + u * 256;
            if (i >= n) continue;
            uint32_t k = (uint32_t)i;
            if (!overflow) {
                const uint32_t cx = (uint32_t)(vox_coord(p[u].x, inv) - s_box[0]);
                const uint32_t cy = (uint32_t)(vox_coord(p[u].y, inv) - s_box[1]);
                const uint32_t cz = (uint32_t)(vox_coord(p[u].z, inv) - s_box[2]);
                k = (cz * (uint32_t)dy + cy) * (uint32_t)dx + cx;   // < 2^31
            }
            keys[i] = k;
            radix_hist_add(s_h, k, passes);
        }
    }
    radix_hist_commit(s_h, hist, passes);
}

// Segments and centroids in one pass over the sorted pairs (pcl::VoxelGrid's "one output point per run of
// equal voxel indices").  A block takes a tile of kSegTile sorted positions in start order: each thread flags
// the voxel heads (key differs from its predecessor) of 8 consecutive positions, the block scans the counts,
// the tile's first output index comes by look-back (radix.h), and the heads are listed in LDS.  The tile's
// points -- plus a margin past its end, where its last voxel may run on -- are gathered into LDS once,
// coalesced.  Then each thread sums whole voxels from LDS, one voxel per thread: the sums are sequential
// double sums in sorted (= stable input) order, as in the oracle.  A last voxel longer than the margin reads
// its remaining points from HBM.
// (r03: a segment scan + one wave per voxel took 19 + 42 us on a C4 surf window -- 65k mostly latency-bound
// waves for 3e4 voxels; a wave walking its positions in order through readlane, 150-200 us: one point per
// iteration per wave, and the CU's 16 waves contend for its scalar unit.)
constexpr int kSegThreads = 512;
constexpr int kSegPer = kSegTile / kSegThreads;   // 8 positions per thread
constexpr int kSegMargin = 1024;
constexpr int kSegStage = kSegTile + kSegMargin;  // 80 KB of points in LDS

__global__ __launch_bounds__(kSegThreads) void voxel_reduce_kernel(const float4* pts, const uint32_t* ka,
                                                                   const uint32_t* kb, const int* va, const int* vb,
                                                                   int n, const uint32_t* bound, uint32_t* ctr,
                                                                   unsigned long long* st, uint32_t epoch,
                                                                   float4* out, int* nseg, int* map_bb, int* err) {
    __shared__ float4 s_pts[kSegStage];
    __shared__ uint16_t s_head[kSegTile];
    __shared__ uint32_t s_wave[kSegThreads / 64];
    __shared__ int s_tile, s_end;
    __shared__ uint32_t s_before;
    const bool odd = radix_pass_count(*bound) & 1;
    const uint32_t* keys = odd ? kb : ka;
    const int* idx = odd ? vb : va;
    const int tid = threadIdx.x;
    if (tid == 0) {
        s_tile = (int)__hip_atomic_fetch_add(&ctr[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_end = INT_MAX;
    }
    __syncthreads();
    const int tile = s_tile;
    const int tbase = tile * kSegTile;
    const int staged = min(kSegStage, n - tbase);   // positions [tbase, tbase + staged) land in LDS
    // the stage: indices, then points (all loads of a thread in flight together)
    int ix[kSegStage / kSegThreads];
#pragma unroll
    for (int q = 0; q < kSegStage / kSegThreads; ++q) {
        const int i = q * kSegThreads + tid;
        ix[q] = i < staged ? idx[tbase + i] : 0;
    }
    // head flags of 8 consecutive positions
    const int p0 = tbase + tid * kSegPer;
    uint32_t k[kSegPer];
    if (p0 + kSegPer <= n) {
        const uint4 a = *reinterpret_cast<const uint4*>(keys + p0), b = *reinterpret_cast<const uint4*>(keys + p0 + 4);
        k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w; k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < kSegPer; ++j) k[j] = p0 + j < n ? keys[p0 + j] : 0u;
    }
    uint32_t prev = p0 > 0 && p0 < n ? keys[p0 - 1] : 0u;
    // the first head past the tile, within the margin (the end of the tile's last voxel)
    uint32_t mk[kSegMargin / kSegThreads], mp[kSegMargin / kSegThreads];
#pragma unroll
    for (int q = 0; q < kSegMargin / kSegThreads; ++q) {
        const int i = tbase + kSegTile + q * kSegThreads + tid;
        mk[q] = i < n ? keys[i] : 0u;
        mp[q] = i < n ? keys[i - 1] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kSegStage / kSegThreads; ++q) {
        const int i = q * kSegThreads + tid;
        // a sorted index outside the cloud exists only after a look-back fault upstream: never read with it
        if (i < staged) s_pts[i] = pts[(unsigned)ix[q] < (unsigned)n ? ix[q] : 0];
    }
    uint32_t flags = 0, c = 0;
#pragma unroll
    for (int j = 0; j < kSegPer; ++j) {
        const int i = p0 + j;
        const bool h = i < n && (i == 0 || k[j] != prev);
        prev = k[j];
        flags |= (uint32_t)h << j;
        c += h;
    }
#pragma unroll
    for (int q = 0; q < kSegMargin / kSegThreads; ++q) {
        const int i = tbase + kSegTile + q * kSegThreads + tid;
        if (i < n && mk[q] != mp[q]) atomicMin(&s_end, i - tbase);
    }
    uint32_t total;
    const uint32_t excl = block_exclusive_scan<kSegThreads>(c, s_wave, &total);
    uint32_t r = excl;
#pragma unroll
    for (int j = 0; j < kSegPer; ++j)
        if ((flags >> j) & 1u) s_head[r++] = (uint16_t)(p0 + j - tbase);
    if (tid < 64) {   // wave 0: the tile's offset by a 64-wide look-back (64 tiles per round trip)
        uint32_t before = 0;
        if (tile == 0) {
            if (tid == 0) lb_store(st, epoch, kLbInc, total);
        } else {
            if (tid == 0) lb_store(st + tile, epoch, kLbAgg, total);
            before = wave_lookback(st, tile, epoch, err);
            if (tid == 0) lb_store(st + tile, epoch, kLbInc, before + total);
        }
        if (tid == 0) s_before = before;
    }
    if (tid == 0) {
        const uint32_t before = s_before;
        if (tbase + kSegTile >= n) {   // the last tile: the voxel count (0 after a fault: nothing downstream reads)
            const bool ok = (uint64_t)before + total <= (uint64_t)n;
            *nseg = ok ? (int)(before + total) : 0;
            if (map_bb) map_bb[6] = ok ? (int)(before + total) : 0;
        }
        if (s_end == INT_MAX && tbase + kSegStage >= n) s_end = n - tbase;   // runs to the end of the cloud
    }
    __syncthreads();
    const uint32_t before = s_before;
    const int tend = s_end;   // INT_MAX: the last voxel runs past the margin
    if ((uint64_t)before + total > (uint64_t)n) {   // more voxels than points: only after a look-back fault
        if (tid == 0) lb_fault(err, kFaultSegment);
        return;
    }
    for (uint32_t v = tid; v < total; v += kSegThreads) {
        const int a = s_head[v];
        const int b = v + 1 < total ? (int)s_head[v + 1] : tend;
        double sx = 0, sy = 0, sz = 0, sw = 0;
        int i = a;
        const int lim = min(b, staged);
        for (; i + 4 <= lim; i += 4) {   // 4 LDS reads in flight, added in order
            float4 q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) q[u] = s_pts[i + u];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                sx += (double)q[u].x;
                sy += (double)q[u].y;
                sz += (double)q[u].z;
                sw += (double)q[u].w;
            }
        }
        for (; i < lim; ++i) {
            const float4 q = s_pts[i];
            sx += (double)q.x;
            sy += (double)q.y;
            sz += (double)q.z;
            sw += (double)q.w;
        }
        if (b == INT_MAX) {   // past the margin: from HBM until the key changes
            const uint32_t key = keys[tbase + a];
            for (; tbase + i < n && keys[tbase + i] == key; ++i) {
                const int j = idx[tbase + i];
                const float4 q = pts[(unsigned)j < (unsigned)n ? j : 0];
                sx += (double)q.x;
                sy += (double)q.y;
                sz += (double)q.z;
                sw += (double)q.w;
            }
        }
        const double dc = (double)(i - a);
        out[before + v] = make_float4((float)(sx / dc), (float)(sy / dc), (float)(sz / dc), (float)(sw / dc));
    }
}

void VoxelFilter::release() {
    if (last) (void)hipStreamSynchronize(last);
    void* bufs[] = {keys, keys_b, idx, idx_b, part, nseg, scratch};
    for (void* p : bufs) gfree(p, last);
    if (last) (void)hipStreamSynchronize(last);
    *this = VoxelFilter();
}

int VoxelFilter::box_blocks(int n) { return std::max(std::min((n + 256 * kVoxBatch - 1) / (256 * kVoxBatch), 1024), 1); }

hipError_t VoxelFilter::reserve(size_t need, hipStream_t s) {
    if (need <= cap) return hipSuccess;
    const size_t n = std::min(exact ? need : grow_cap(need, cap), (size_t)INT32_MAX);
    // growth: the old buffers may still be read by this filter's last enqueue on another stream (a tracker
    // kind's rebuild takes either aux stream) -- s waits for that stream's work so far, then frees them in order
    hipError_t e = hipSuccess;
    if (cap && last && last != s) {
        hipEvent_t ev;
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
        e = hipEventRecord(ev, last);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, ev, 0);
        (void)hipEventDestroy(ev);   // released once the wait completes
        if (e != hipSuccess) return e;
    }
    void* old[] = {keys, keys_b, idx, idx_b, part, nseg, scratch};
    for (void* p : old) gfree(p, s);
    const bool ex = exact;
    *this = VoxelFilter();
    exact = ex;
    last = s;
#define VALLOC(p, count) if ((e = galloc(&(p), (count), s)) != hipSuccess) return e
    VALLOC(keys, n);
    VALLOC(keys_b, n);
    VALLOC(idx, n);
    VALLOC(idx_b, n);
    VALLOC(part, (size_t)box_blocks((int)n) * 12 + 16);
    VALLOC(nseg, 1);
    VALLOC(scratch, radix_scratch_words(n));
#undef VALLOC
    // look-back words of epoch 0 are older than every sort (radix.h): zeroed on the stream whose kernels read
    // them (a null-stream memset is not ordered before a non-blocking stream's work -- the r04 fault)
    if ((e = hipMemsetAsync(scratch, 0, radix_scratch_words(n) * sizeof(uint32_t), s)) != hipSuccess) return e;
    cap = n;
    return hipSuccess;
}

hipError_t VoxelFilter::enqueue(const float4* in, int n, float leaf, float4* out, int* err, hipStream_t s, int* map_bb,
                                int sx, int inject) {
    if (n <= 0) return hipSuccess;
    hipError_t e = reserve((size_t)n, s);
    if (e != hipSuccess) return e;
    if (last && last != s) {   // the last enqueue ran on another stream: this one follows it (shared workspace)
        hipEvent_t ev;
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
        e = hipEventRecord(ev, last);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, ev, 0);
        (void)hipEventDestroy(ev);
        if (e != hipSuccess) return e;
    }
    last = s;
    if (poisoned) {   // an injected fault left foreign look-back words behind
        if ((e = hipMemsetAsync(scratch, 0, radix_scratch_words(cap) * sizeof(uint32_t), s)) != hipSuccess) return e;
        poisoned = false;
    }
    epoch = next_lookback_epoch();
    const float inv = 1.0f / leaf;
    const RadixScratch rs = radix_scratch(scratch, (size_t)n);
    uint32_t* bound = reinterpret_cast<uint32_t*>(part) + (size_t)box_blocks(cap) * 12;
    const int nb = box_blocks(n);
    hipLaunchKernelGGL(voxel_box_kernel, dim3(nb), dim3(256), 0, s, in, n, inv, (float)sx, part, rs.hist, rs.ctr);
    // keys + histograms: <= 128 blocks (each commits up to 3 x 256 histogram atomics)
    const int kb = std::max(std::min((n + 256 * kVoxBatch - 1) / (256 * kVoxBatch), 128), 1);
    hipLaunchKernelGGL(voxel_key_kernel, dim3(kb), dim3(256), 0, s, in, n, inv, part, nb, keys, bound, rs.hist, map_bb);
    // pass 0 takes the point index as its value
    if ((e = launch_radix_passes(keys, idx, keys_b, idx_b, nullptr, n, bound, rs, epoch, err, inject, s)) != hipSuccess)
        return e;
    if (inject) poisoned = true;
    hipLaunchKernelGGL(voxel_reduce_kernel, dim3((unsigned)seg_tiles((size_t)n)), dim3(kSegThreads), 0, s, in, keys,
                       keys_b, idx, idx_b, n, bound, rs.ctr, rs.seg_state, epoch, out, nseg, map_bb, err);
    return hipGetLastError();
}

hipError_t VoxelFilter::run(const float4* in, int n, float leaf, float4* out, int* n_out, int* err, hipStream_t s) {
    *n_out = 0;
    if (n <= 0) return hipSuccess;
    hipError_t e = enqueue(in, n, leaf, out, err, s);
    if (e != hipSuccess) return e;
    int h[2] = {0, 0};
    if ((e = hipMemcpyAsync(&h[0], nseg, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&h[1], err, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if (h[1]) return hipErrorIllegalState;   // the caller reads and clears the fault word
    *n_out = h[0];
    return hipSuccess;
}

}  // namespace lmsf
