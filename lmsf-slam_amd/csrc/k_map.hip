// Device neighbour index of a LOAM feature map: dense 1 m cell grid with cell-sorted points,
// each cell cut into sx x-slices (the rows the search trims to the query's x-window).
//
// Replaces FeatureMatch::SetSearchTarget -> pcl::KdTreeFLANN::setInputCloud
// (REG/FeatureMatch/FeatureMatchBase.hpp:40-44), rebuilt whenever the local map changes
// (INC/LidarTracker/LidarTrackerLocalMap.hpp:229).  Cell edge = the 1 m match radius
// (search_thresh_ = 1.0, FeatureMatchBase.hpp:29), so every map point with d^2 < 1 to a query
// lies in the 3x3x3 cells around the query's cell; cell = floor(coord) - origin is exact in float.
// Layout in HBM: float4 pts[n] sorted by linear cell (x fastest: the 3 x-neighbours of a cell are
// one contiguous range, and so are the slices of a row), uint32 off[slices + 1]; w of each sorted
// point = its original index.  x-slice = floor(x * sx) (exact: sx is a power of two).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "bbox.h"
#include "lmsf_internal.h"

namespace lmsf {

// bbox[0..5] = slice / row / level box of the first n points; with n_dev (a producer's count still on the
// device, e.g. the voxel filter's) n = min(n, *n_dev); bbox[6] = that n, so one read-back carries both.
__global__ void map_bbox_init_kernel(int* bbox) {
    if (threadIdx.x < 3) bbox[threadIdx.x] = INT_MAX;
    else if (threadIdx.x < 6) bbox[threadIdx.x] = INT_MIN;
}

__global__ void __launch_bounds__(256) map_bbox_kernel(const float4* pts, int n, const int* n_dev, float sx, int* bbox) {
    if (n_dev) n = min(n, *n_dev);
    if (blockIdx.x == 0 && threadIdx.x == 0) bbox[6] = n;
    int lo[3] = {INT_MAX, INT_MAX, INT_MAX}, hi[3] = {INT_MIN, INT_MIN, INT_MIN};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        const float c[3] = {floorf(p.x * sx), floorf(p.y), floorf(p.z)};
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            // coordinates beyond +-2^30 m are clamped (they cannot be matched anyway)
            const int v = (int)fminf(fmaxf(c[d], -1073741824.f), 1073741824.f);
            lo[d] = min(lo[d], v);
            hi[d] = max(hi[d], v);
        }
    }
    block_bbox_commit<256>(lo, hi, bbox);
}

__global__ void map_count_kernel(const float4* pts, int n, float sx, int ox, int oy, int oz, int nx, int ny, int nz,
                                 int* cell, uint32_t* counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[i];
    const int cx = (int)fminf(fmaxf(floorf(p.x * sx), -1073741824.f), 1073741824.f) - ox;
    const int cy = (int)fminf(fmaxf(floorf(p.y), -1073741824.f), 1073741824.f) - oy;
    const int cz = (int)fminf(fmaxf(floorf(p.z), -1073741824.f), 1073741824.f) - oz;
    const int c = (cz * ny + cy) * nx + cx;
    cell[i] = c;
    atomicAdd(&counts[c], 1u);
}

// Number of occupied slices (the map's density statistic that selects the pruned search).
__global__ void __launch_bounds__(256) count_nonzero_kernel(const uint32_t* counts, size_t n, unsigned long long* out) {
    __shared__ unsigned int part[4];
    unsigned int c = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c += counts[i] != 0u;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(part[0] + part[1] + part[2] + part[3]));
}

hipError_t launch_count_nonzero(const uint32_t* counts, size_t n, unsigned long long* out, hipStream_t s) {
    const size_t blocks = std::min<size_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(count_nonzero_kernel, dim3((unsigned)std::max<size_t>(blocks, 1)), dim3(256), 0, s, counts, n, out);
    return hipGetLastError();
}

// Scatter into cell order.  Order inside a cell is arbitrary: the search ranks candidates by the
// total order (d2, original index), so results do not depend on it.
__global__ void map_scatter_kernel(const float4* pts, int n, const int* cell, const uint32_t* off, uint32_t* fill,
                                   float4* sorted, int base) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = cell[i];
    const uint32_t pos = off[c] + atomicAdd(&fill[c], 1u);
    const float4 p = pts[i];
    sorted[pos] = make_float4(p.x, p.y, p.z, __int_as_float(base + i));
}

// pcl::transformPointCloud with an Eigen::Matrix4d (PCL 1.7 transforms.hpp): per point
// out = float(t(r,0) x + t(r,1) y + t(r,2) z + t(r,3)) evaluated in double, fields copied.
// Used by LidarTrackerLocalMap::updateLocalMap (INC/LidarTracker/LidarTrackerLocalMap.hpp:217).
__global__ void transform_kernel(const float4* in, int n, Affine34 M, float4* out) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 p = in[i];
    const double x = p.x, y = p.y, z = p.z;
    float4 o;
    o.x = (float)(M.m[0] * x + M.m[1] * y + M.m[2] * z + M.m[3]);
    o.y = (float)(M.m[4] * x + M.m[5] * y + M.m[6] * z + M.m[7]);
    o.z = (float)(M.m[8] * x + M.m[9] * y + M.m[10] * z + M.m[11]);
    o.w = p.w;
    out[i] = o;
}

hipError_t launch_transform(const float4* in, int n, Affine34 M, float4* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(transform_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, M, out);
    return hipGetLastError();
}

// The keyframe window concatenated in window order (LidarTrackerLocalMap's local map assembly):
// one launch over all slots instead of a device-to-device copy per keyframe.
__global__ void gather_slots_kernel(SlotTable tab, float4* out) {
    const int total = tab.start[tab.n];
    int k = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        while (i >= tab.start[k + 1]) ++k;
        out[i] = tab.src[k][i - tab.start[k]];
    }
}

hipError_t launch_gather_slots(const SlotTable& tab, float4* out, hipStream_t s) {
    const int total = tab.start[tab.n];
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_slots_kernel, dim3(min((total + 255) / 256, 4096)), dim3(256), 0, s, tab, out);
    return hipGetLastError();
}

hipError_t launch_map_bbox(const float4* pts, int n, const int* n_dev, int sx, int* bbox, hipStream_t s) {
    hipLaunchKernelGGL(map_bbox_init_kernel, dim3(1), dim3(64), 0, s, bbox);
    // >= 16 points per thread, <= 512 blocks: each block commits 6 atomics to the same 6 words (512 blocks
    // serialise ~35 us on them, which only a multi-million-point cloud amortises)
    const int blocks = min((n + 4095) / 4096, 512);
    hipLaunchKernelGGL(map_bbox_kernel, dim3(max(blocks, 1)), dim3(256), 0, s, pts, n, n_dev, (float)sx, bbox);
    return hipGetLastError();
}

hipError_t launch_map_count(const float4* pts, int n, int sx, int ox, int oy, int oz, int nx, int ny, int nz,
                            int* cell, uint32_t* counts, hipStream_t s) {
    hipLaunchKernelGGL(map_count_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pts, n, (float)sx, ox, oy, oz, nx,
                       ny, nz, cell, counts);
    return hipGetLastError();
}

hipError_t launch_map_scatter(const float4* pts, int n, const int* cell, const uint32_t* off, uint32_t* fill,
                              float4* sorted, int base, hipStream_t s) {
    hipLaunchKernelGGL(map_scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pts, n, cell, off, fill, sorted,
                       base);
    return hipGetLastError();
}

// out[0..2] = *a, *b, *c: several device words gathered for one read-back
__global__ void pack3_kernel(const int* a, const int* b, const int* c, int* out) {
    if (threadIdx.x == 0) {
        out[0] = *a;
        out[1] = *b;
        out[2] = *c;
    }
}

hipError_t launch_pack3(const int* a, const int* b, const int* c, int* out, hipStream_t s) {
    hipLaunchKernelGGL(pack3_kernel, dim3(1), dim3(64), 0, s, a, b, c, out);
    return hipGetLastError();
}

// counts[0..n) = fill[0..n) = 0 and *occ = 0 (one launch for the three resets of a grid build)
__global__ void grid_clear_kernel(uint32_t* counts, uint32_t* fill, size_t n, unsigned long long* occ) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        counts[i] = 0u;
        fill[i] = 0u;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *occ = 0ull;
}

hipError_t launch_grid_clear(uint32_t* counts, uint32_t* fill, size_t n, unsigned long long* occ, hipStream_t s) {
    const size_t blocks = std::min<size_t>(2048, (n + 255) / 256);
    hipLaunchKernelGGL(grid_clear_kernel, dim3((unsigned)std::max<size_t>(blocks, 1)), dim3(256), 0, s, counts, fill, n, occ);
    return hipGetLastError();
}

hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, size_t n, void* tmp, size_t& tmp_bytes,
                              hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, n, s);
}

}  // namespace lmsf
