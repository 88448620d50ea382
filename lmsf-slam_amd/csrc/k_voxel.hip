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
// Roofline: HBM-bound byte work (one read of the cloud for the bounding box, keys 8 B + index 4 B
// written and radix-sorted, one gather of 16 B per point, 16 B per voxel out).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "bbox.h"
#include "lmsf_internal.h"

namespace lmsf {

// A one-workgroup variant for small clouds (box, keys, LDS bitonic sort of (key, index), heads, sums in one
// launch instead of ~13) was bit-exact but slower on the tracker's ~4.5k-point edge window: C4 1.65-1.89
// vs 1.55-1.85 ms/scan, C3 1.68-1.72 vs 1.58-1.62 ms/frame (91 barrier-separated sort stages): removed.
// hipcub's default dispatch (merge sort below 2^20 items).  Measured on a C4 commit: rocprim onesweep
// (radix_sort_config merge limit 0) took 4 x ~25 us + 8 lookback resets for the ~6e5-point surf window
// (merge sort ~130 us) and 4 x ~18 us for the edge window (merge sort ~25 us): not used.
static hipError_t voxel_sort(void* tmp, size_t& bytes, const uint32_t* k_in, uint32_t* k_out, const int* v_in,
                             int* v_out, int n, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, k_in, k_out, v_in, v_out, n, 0, 31, s);
}

__device__ __forceinline__ int vox_coord(float v, float inv) {
    return (int)fminf(fmaxf(floorf(v * inv), -1073741824.f), 1073741824.f);
}

__global__ void __launch_bounds__(256) voxel_bbox_kernel(const float4* pts, int n, float inv, int* bbox) {
    int lo[3] = {INT_MAX, INT_MAX, INT_MAX}, hi[3] = {INT_MIN, INT_MIN, INT_MIN};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        const int c[3] = {vox_coord(p.x, inv), vox_coord(p.y, inv), vox_coord(p.z, inv)};
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = min(lo[d], c[d]);
            hi[d] = max(hi[d], c[d]);
        }
    }
    block_bbox_commit<256>(lo, hi, bbox);
}

// Linear voxel key from the device-side bounding box (no host round trip).  When div_x*div_y*div_z
// exceeds INT32_MAX PCL refuses and returns the input unchanged: every point then gets its own key
// (its index), so each "voxel" is one point and the centroid pass reproduces the input exactly.
__global__ void voxel_key_kernel(const float4* pts, int n, float inv, const int* bbox, uint32_t* keys, int* idx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t dx = (int64_t)bbox[3] - bbox[0] + 1, dy = (int64_t)bbox[4] - bbox[1] + 1,
                  dz = (int64_t)bbox[5] - bbox[2] + 1;
    idx[i] = i;
    if (dx * dy * dz > (int64_t)INT32_MAX) {
        keys[i] = (uint32_t)i;
        return;
    }
    const float4 p = pts[i];
    const uint32_t cx = (uint32_t)(vox_coord(p.x, inv) - bbox[0]);
    const uint32_t cy = (uint32_t)(vox_coord(p.y, inv) - bbox[1]);
    const uint32_t cz = (uint32_t)(vox_coord(p.z, inv) - bbox[2]);
    keys[i] = (cz * (uint32_t)dy + cy) * (uint32_t)dx + cx;   // < 2^31
}

// start[s] = first sorted position of voxel s (heads scanned into segment ids).
__global__ void voxel_head_kernel(const uint32_t* keys, int n, uint32_t* head) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void voxel_start_kernel(const uint32_t* head, const uint32_t* seg, int n, int* start, int* nseg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (head[i]) start[seg[i]] = i;
    if (i == n - 1) {
        *nseg = (int)(seg[i] + head[i]);
        start[seg[i] + head[i]] = n;
    }
}

// One wave per voxel (grid-stride over the voxels): the wave gathers 64 of the voxel's points at a
// time and every lane adds them in sorted (= input) order through readlane, so the sums are the
// sequential double sums of the thread-per-voxel form while the gathers run 64 wide.  (One lane per
// voxel measured 164 us vs 40 us on a C4 surf window: voxels near the sensor hold hundreds of points
// and a wave waits for its fullest voxel.)
__global__ __launch_bounds__(256) void voxel_mean_kernel(const float4* pts, const int* idx_sorted, const int* start,
                                                         const int* nseg, float4* out) {
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

__global__ void bbox_init_kernel(int* bbox) {
    if (threadIdx.x < 3) bbox[threadIdx.x] = INT_MAX;
    else if (threadIdx.x < 6) bbox[threadIdx.x] = INT_MIN;
}

void VoxelFilter::release() {
    void* bufs[] = {keys, keys_sorted, idx, idx_sorted, head, seg, start, bbox, nseg, tmp, sort_scratch};
    for (void* p : bufs) hipFree(p);
    *this = VoxelFilter();
}

hipError_t VoxelFilter::reserve(size_t need) {
    if (need <= cap) return hipSuccess;
    const size_t n = std::min(grow_cap(need, cap), (size_t)INT32_MAX);
    release();
    hipError_t e;
#define VALLOC(p, bytes) if ((e = hipMalloc((void**)&(p), (bytes))) != hipSuccess) return e
    VALLOC(keys, n * sizeof(uint32_t));
    VALLOC(keys_sorted, n * sizeof(uint32_t));
    VALLOC(idx, n * sizeof(int));
    VALLOC(idx_sorted, n * sizeof(int));
    VALLOC(head, n * sizeof(uint32_t));
    VALLOC(seg, n * sizeof(uint32_t));
    VALLOC(start, (n + 1) * sizeof(int));
    VALLOC(bbox, 8 * sizeof(int));
    VALLOC(nseg, sizeof(int));
    VALLOC(sort_scratch, radix_sort_scratch_words(n) * sizeof(uint32_t));
    size_t sort_b = 0, scan_b = 0;
    voxel_sort(nullptr, sort_b, keys, keys_sorted, idx, idx_sorted, (int)n, nullptr);
    hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, head, seg, (int)n);
    tmp_bytes = sort_b > scan_b ? sort_b : scan_b;
    VALLOC(tmp, tmp_bytes);
#undef VALLOC
    cap = n;
    return hipSuccess;
}

hipError_t VoxelFilter::enqueue(const float4* in, int n, float leaf, float4* out, hipStream_t s) {
    if (n <= 0) return hipErrorInvalidValue;
    hipError_t e = reserve((size_t)n);
    if (e != hipSuccess) return e;
    const float inv = 1.0f / leaf;
    hipLaunchKernelGGL(bbox_init_kernel, dim3(1), dim3(64), 0, s, bbox);
    // >= 16 points per thread, <= 512 blocks: 6 contended atomics per block (as launch_map_bbox)
    hipLaunchKernelGGL(voxel_bbox_kernel, dim3(min(max((n + 4095) / 4096, 1), 512)), dim3(256), 0, s, in, n, inv, bbox);
    const dim3 g((n + 255) / 256), b(256);
    hipLaunchKernelGGL(voxel_key_kernel, g, b, 0, s, in, n, inv, bbox, keys, idx);
    // keys < 2^31: 31 key bits (one host round trip fewer than sizing the sort to the box)
    const uint32_t* ks = keys_sorted;
    const int* is = idx_sorted;
    static const bool radix = ab_int("LMSF_VOXEL_RADIX", 1) != 0;
    if (radix) {   // k_sort.hip: 6 enqueues, in place (r03)
        if ((e = radix_sort_pairs(keys, idx, keys_sorted, idx_sorted, n, sort_scratch, s)) != hipSuccess) return e;
        ks = keys;
        is = idx;
    } else {
        size_t tb = tmp_bytes;
        if ((e = voxel_sort(tmp, tb, keys, keys_sorted, idx, idx_sorted, n, s)) != hipSuccess) return e;
    }
    size_t tb = tmp_bytes;
    hipLaunchKernelGGL(voxel_head_kernel, g, b, 0, s, ks, n, head);
    if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, head, seg, n, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(voxel_start_kernel, g, b, 0, s, head, seg, n, start, nseg);
    // up to one wave per ~4 points (r02: 4096 blocks, 47 vs 40 us on a C4 surf window; the voxel count is on
    // the device and idle waves exit at once)
    hipLaunchKernelGGL(voxel_mean_kernel, dim3(min((n + 15) / 16, 16384)), b, 0, s, in, is, start, nseg, out);
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
