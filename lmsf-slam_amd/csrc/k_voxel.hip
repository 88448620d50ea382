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
// bound needs run), segment starts (one single-pass scan), centroids -- 8 (was ~20).  No atomics on shared
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

// start[s] = first sorted position of voxel s, *nseg = the voxel count (also map_bb[6] for the tracker's
// grid read-back), start[*nseg] = n: head flags (key differs from its predecessor) scanned in one pass --
// 8 consecutive keys per thread, a block scan, the tile offset by look-back (radix.h) over a tile counter.
__global__ void __launch_bounds__(256) voxel_segments_kernel(const uint32_t* ka, const uint32_t* kb, int n,
                                                             const uint32_t* bound, uint32_t* ctr,
                                                             unsigned long long* st, uint32_t epoch, int* start,
                                                             int* nseg, int* map_bb) {
    __shared__ int s_tile;
    __shared__ uint32_t s_wave[4], s_before;
    const uint32_t* keys = radix_pass_count(*bound) & 1 ? kb : ka;
    if (threadIdx.x == 0) s_tile = (int)__hip_atomic_fetch_add(&ctr[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int tile = s_tile;
    const int i0 = tile * kRadixTile + threadIdx.x * 8;
    uint32_t k[8];
    if (i0 + 8 <= n) {
        const uint4 a = *reinterpret_cast<const uint4*>(keys + i0), b = *reinterpret_cast<const uint4*>(keys + i0 + 4);
        k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w; k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) k[j] = i0 + j < n ? keys[i0 + j] : 0u;
    }
    uint32_t prev = i0 > 0 && i0 < n ? keys[i0 - 1] : 0u;
    uint32_t flags = 0, c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = i0 + j;
        const bool h = i < n && (i == 0 || k[j] != prev);
        prev = k[j];
        flags |= (uint32_t)h << j;
        c += h;
    }
    uint32_t total;
    const uint32_t excl = block_exclusive_scan<256>(c, s_wave, &total);
    if (threadIdx.x == 0) {
        if (tile == 0) {
            lb_store(st, epoch, kLbInc, total);
            s_before = 0;
        } else {
            lb_store(st + tile, epoch, kLbAgg, total);
            const uint32_t before = lookback_sum(st, tile, 1, epoch);
            lb_store(st + tile, epoch, kLbInc, before + total);
            s_before = before;
        }
    }
    __syncthreads();
    uint32_t seg = s_before + excl;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if ((flags >> j) & 1u) start[seg++] = i0 + j;
    if (i0 <= n - 1 && n - 1 < i0 + 8) {   // the thread of the last point
        *nseg = (int)seg;
        start[seg] = n;
        if (map_bb) map_bb[6] = (int)seg;
    }
}

// One wave per voxel (grid-stride over the voxels): the wave gathers 64 of the voxel's points at a
// time and every lane adds them in sorted (= input) order through readlane, so the sums are the
// sequential double sums of the thread-per-voxel form while the gathers run 64 wide.  (One lane per
// voxel measured 164 us vs 40 us on a C4 surf window: voxels near the sensor hold hundreds of points
// and a wave waits for its fullest voxel.)
__global__ __launch_bounds__(256) void voxel_mean_kernel(const float4* pts, const int* va, const int* vb,
                                                         const uint32_t* bound, const int* start, const int* nseg,
                                                         float4* out) {
    const int* idx_sorted = radix_pass_count(*bound) & 1 ? vb : va;
    const int lane = threadIdx.x & 63;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    const int ns = *nseg;
    for (int s = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; s < ns; s += nw) {
        const int a = start[s], b = start[s + 1];
        double sx = 0, sy = 0, sz = 0, sw = 0;
        for (int c = a; c < b; c += 64) {
            const int m = min(64, b - c);
            const float4 p = lane < m ? pts[idx_sorted[c + lane]] : make_float4(0.f, 0.f, 0.f, 0.f);
            for (int j = 0; j < m; ++j) {
                sx += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.x), j));
                sy += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.y), j));
                sz += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.z), j));
                sw += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.w), j));
            }
        }
        const double cnt = (double)(b - a);
        if (lane == 0) out[s] = make_float4((float)(sx / cnt), (float)(sy / cnt), (float)(sz / cnt), (float)(sw / cnt));
    }
}

void VoxelFilter::release() {
    void* bufs[] = {keys, keys_b, idx, idx_b, start, part, nseg, scratch};
    for (void* p : bufs) hipFree(p);
    *this = VoxelFilter();
}

int VoxelFilter::box_blocks(int n) { return std::max(std::min((n + 256 * kVoxBatch - 1) / (256 * kVoxBatch), 1024), 1); }

hipError_t VoxelFilter::reserve(size_t need) {
    if (need <= cap) return hipSuccess;
    const size_t n = std::min(grow_cap(need, cap), (size_t)INT32_MAX);
    release();
    hipError_t e;
#define VALLOC(p, bytes) if ((e = hipMalloc((void**)&(p), (bytes))) != hipSuccess) return e
    VALLOC(keys, n * sizeof(uint32_t));
    VALLOC(keys_b, n * sizeof(uint32_t));
    VALLOC(idx, n * sizeof(int));
    VALLOC(idx_b, n * sizeof(int));
    VALLOC(start, (n + 1) * sizeof(int));
    VALLOC(part, (size_t)box_blocks((int)n) * 12 * sizeof(int) + 16 * sizeof(int));
    VALLOC(nseg, sizeof(int));
    VALLOC(scratch, radix_scratch_words(n) * sizeof(uint32_t));
#undef VALLOC
    // look-back words of epoch 0 never match a sort (epochs start at 1)
    if ((e = hipMemset(scratch, 0, radix_scratch_words(n) * sizeof(uint32_t))) != hipSuccess) return e;
    cap = n;
    return hipSuccess;
}

hipError_t VoxelFilter::enqueue(const float4* in, int n, float leaf, float4* out, hipStream_t s, int* map_bb, int sx) {
    if (n <= 0) return hipErrorInvalidValue;
    hipError_t e = reserve((size_t)n);
    if (e != hipSuccess) return e;
    if (++epoch == 0) ++epoch;
    const float inv = 1.0f / leaf;
    const RadixScratch rs = radix_scratch(scratch, (size_t)n);
    uint32_t* bound = reinterpret_cast<uint32_t*>(part) + (size_t)box_blocks(cap) * 12;
    const int nb = box_blocks(n);
    hipLaunchKernelGGL(voxel_box_kernel, dim3(nb), dim3(256), 0, s, in, n, inv, (float)sx, part, rs.hist, rs.ctr);
    // keys + histograms: <= 128 blocks (each commits up to 3 x 256 histogram atomics)
    const int kb = std::max(std::min((n + 256 * kVoxBatch - 1) / (256 * kVoxBatch), 128), 1);
    hipLaunchKernelGGL(voxel_key_kernel, dim3(kb), dim3(256), 0, s, in, n, inv, part, nb, keys, bound, rs.hist, map_bb);
    // pass 0 takes the point index as its value
    if ((e = launch_radix_passes(keys, idx, keys_b, idx_b, nullptr, n, bound, rs, epoch, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(voxel_segments_kernel, dim3((unsigned)rs.tiles), dim3(256), 0, s, keys, keys_b, n, bound, rs.ctr,
                       rs.seg_state, epoch, start, nseg, map_bb);
    // up to one wave per ~4 points (r02: 4096 blocks, 47 vs 40 us on a C4 surf window; the voxel count is on
    // the device and idle waves exit at once)
    hipLaunchKernelGGL(voxel_mean_kernel, dim3(min((n + 15) / 16, 16384)), dim3(256), 0, s, in, idx, idx_b, bound,
                       start, nseg, out);
    return hipGetLastError();
}

hipError_t VoxelFilter::run(const float4* in, int n, float leaf, float4* out, int* n_out, hipStream_t s) {
    *n_out = 0;
    if (n <= 0) return hipSuccess;
    hipError_t e = enqueue(in, n, leaf, out, s);
    if (e != hipSuccess) return e;
    if ((e = hipMemcpyAsync(n_out, nseg, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

}  // namespace lmsf
