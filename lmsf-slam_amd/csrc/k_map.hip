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
#include "radix.h"

namespace lmsf {

// bbox[0..5] = slice / row / level box of the first n points; with n_dev (a producer's count still on the
// device, e.g. the voxel filter's) n = min(n, *n_dev); bbox[6] = that n, so one read-back carries both.
__global__ void map_bbox_init_kernel(int* bbox) {
    if (threadIdx.x < 3) bbox[threadIdx.x] = INT_MAX;
    else if (threadIdx.x < 6) bbox[threadIdx.x] = INT_MIN;
}

__global__ void __launch_bounds__(256) map_bbox_kernel(const float4* pts, int n, const int* n_dev, float sx, float sy, int* bbox) {
    if (n_dev) n = min(n, *n_dev);
    if (blockIdx.x == 0 && threadIdx.x == 0) bbox[6] = n;
    int lo[3] = {INT_MAX, INT_MAX, INT_MAX}, hi[3] = {INT_MIN, INT_MIN, INT_MIN};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        const float c[3] = {floorf(p.x * sx), floorf(p.y * sy), floorf(p.z * sy)};   // sy: 1 (1 m cells) or 2
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

__global__ void map_count_kernel(const float4* pts, int n, float sx, float sy, int ox, int oy, int oz, int nx, int ny,
                                 int nz, int* cell, uint32_t* counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[i];
    const int cx = (int)fminf(fmaxf(floorf(p.x * sx), -1073741824.f), 1073741824.f) - ox;
    const int cy = (int)fminf(fmaxf(floorf(p.y * sy), -1073741824.f), 1073741824.f) - oy;
    const int cz = (int)fminf(fmaxf(floorf(p.z * sy), -1073741824.f), 1073741824.f) - oz;
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
                                   float4* sorted, int base, int* err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = cell[i];
    const uint32_t pos = off[c] + atomicAdd(&fill[c], 1u);
    if (pos >= (uint32_t)n) {   // never written outside the points (radix.h fault checks)
        lb_fault(err, kFaultGridScatter);
        return;
    }
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

// Cross-stream ordering through a device flag instead of an event wait (tracker rebuild fork / join, A/B
// LMSF_FLAG_SYNC): the producer stream ends its work with flag_signal (release: the kernels before it on that stream
// have completed and released their writes at kernel end), the consumer stream runs flag_wait (one wave polling with
// acquire loads) before the work that reads them.  A wait past its bound flags kFaultStreamWait in err and lets the
// stream go on (reported as LMSF_ERR_HIP at the next read-back), so no configuration can hang the device.
__global__ void flag_signal_kernel(uint32_t* flag, uint32_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void flag_wait_kernel(const uint32_t* flag, uint32_t v, int* err, unsigned spin_limit) {
    if (threadIdx.x != 0) return;
    unsigned spins = 0;
    while ((int)(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - v) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > spin_limit) {
            if (err) atomicOr(err, kFaultStreamWait);
            break;
        }
    }
}

hipError_t launch_flag_signal(uint32_t* flag, uint32_t v, hipStream_t s) {
    hipLaunchKernelGGL(flag_signal_kernel, dim3(1), dim3(64), 0, s, flag, v);
    return hipGetLastError();
}

hipError_t launch_flag_wait(const uint32_t* flag, uint32_t v, int* err, hipStream_t s) {
    hipLaunchKernelGGL(flag_wait_kernel, dim3(1), dim3(64), 0, s, flag, v, err, 1u << 24);
    return hipGetLastError();
}

hipError_t launch_transform(const float4* in, int n, Affine34 M, float4* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(transform_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, M, out);
    return hipGetLastError();
}

// The same transform at a pose the device holds (x = qx qy qz qw tx ty tz, a Solve's result): the matrix as the host
// builds it (tracker.cpp R_from_quat, Eigen's toRotationMatrix; t = x[4..6]), then transform_kernel's arithmetic --
// the same bits as launch_transform with the host's copy of that pose.
__global__ void transform_pose_kernel(const float4* in, int n, const double* x, float4* out, int n0, float4* out1) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double qx = x[0], qy = x[1], qz = x[2], qw = x[3];
    const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz, twx = tx * qw, twy = ty * qw, twz = tz * qw;
    const double txx = tx * qx, txy = ty * qx, txz = tz * qx, tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    const double m[12] = {1 - (tyy + tzz), txy - twz, txz + twy, x[4],
                          txy + twz, 1 - (txx + tzz), tyz - twx, x[5],
                          txz - twy, tyz + twx, 1 - (txx + tyy), x[6]};
    const float4 p = in[i];
    const double px = p.x, py = p.y, pz = p.z;
    float4 o;
    o.x = (float)(m[0] * px + m[1] * py + m[2] * pz + m[3]);
    o.y = (float)(m[4] * px + m[5] * py + m[6] * pz + m[7]);
    o.z = (float)(m[8] * px + m[9] * py + m[10] * pz + m[11]);
    o.w = p.w;
    if (i < n0) out[i] = o;
    else out1[i - n0] = o;
}

hipError_t launch_transform_pose2(const float4* in, int n0, int n1, const double* x, float4* out0, float4* out1,
                                  hipStream_t s) {
    const int n = n0 + n1;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(transform_pose_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, x, out0, n0, out1);
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

hipError_t launch_map_bbox(const float4* pts, int n, const int* n_dev, int sx, int* bbox, hipStream_t s, int sy) {
    hipLaunchKernelGGL(map_bbox_init_kernel, dim3(1), dim3(64), 0, s, bbox);
    // >= 16 points per thread, <= 512 blocks: each block commits 6 atomics to the same 6 words (512 blocks
    // serialise ~35 us on them, which only a multi-million-point cloud amortises)
    const int blocks = min((n + 4095) / 4096, 512);
    hipLaunchKernelGGL(map_bbox_kernel, dim3(max(blocks, 1)), dim3(256), 0, s, pts, n, n_dev, (float)sx, (float)sy, bbox);
    return hipGetLastError();
}

hipError_t launch_map_count(const float4* pts, int n, int sx, int ox, int oy, int oz, int nx, int ny, int nz,
                            int* cell, uint32_t* counts, hipStream_t s, int sy) {
    hipLaunchKernelGGL(map_count_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pts, n, (float)sx, (float)sy, ox, oy, oz,
                       nx, ny, nz, cell, counts);
    return hipGetLastError();
}

hipError_t launch_map_scatter(const float4* pts, int n, const int* cell, const uint32_t* off, uint32_t* fill,
                              float4* sorted, int base, int* err, hipStream_t s) {
    hipLaunchKernelGGL(map_scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pts, n, cell, off, fill, sorted,
                       base, err);
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

// ---- device-sized builds (tracker windows): the box and count come from a producer on the device (d_bb:
// box 0..5, count 6), so the grid is built without a host round trip; d_bb[10] = cells + 1 when that exceeds
// the allocation (the host then rebuilds with room), else 0; d_bb[16] = the scan's tile counter.

__device__ __forceinline__ size_t grid_cells(const int* bb) {
    const long long nx = (long long)bb[3] - bb[0] + 1, ny = (long long)bb[4] - bb[1] + 1, nz = (long long)bb[5] - bb[2] + 1;
    if (nx <= 0 || ny <= 0 || nz <= 0) return 0;
    return (size_t)(nx * ny * nz);
}

__global__ void grid_clear_dev_kernel(int* bb, uint32_t* counts, uint32_t* fill, size_t cap) {
    const size_t cells = grid_cells(bb);
    const bool over = bb[6] > 0 && (cells == 0 || cells + 1 > cap);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        bb[10] = over ? (int)min(cells + 1, (size_t)INT_MAX) : 0;
        bb[16] = 0;
    }
    if (over) return;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells + 1; i += stride) {
        counts[i] = 0u;
        fill[i] = 0u;
    }
}

__global__ void map_count_dev_kernel(const float4* pts, const int* bb, float sx, int* cell, uint32_t* counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= bb[6] || bb[10]) return;
    const int ox = bb[0], oy = bb[1], oz = bb[2], nx = bb[3] - ox + 1, ny = bb[4] - oy + 1;
    const float4 p = pts[i];
    const int cx = (int)fminf(fmaxf(floorf(p.x * sx), -1073741824.f), 1073741824.f) - ox;
    const int cy = (int)fminf(fmaxf(floorf(p.y), -1073741824.f), 1073741824.f) - oy;
    const int cz = (int)fminf(fmaxf(floorf(p.z), -1073741824.f), 1073741824.f) - oz;
    const int c = (cz * ny + cy) * nx + cx;
    cell[i] = c;
    atomicAdd(&counts[c], 1u);
}

__global__ void map_scatter_dev_kernel(const float4* pts, const int* bb, const int* cell, const uint32_t* off,
                                       uint32_t* fill, float4* sorted, int base, int* err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= bb[6] || bb[10]) return;
    const int c = cell[i];
    const uint32_t pos = off[c] + atomicAdd(&fill[c], 1u);
    if (pos >= (uint32_t)bb[6]) {   // the offsets came from the look-back scan: checked (radix.h)
        lb_fault(err, kFaultGridScatter);
        return;
    }
    const float4 p = pts[i];
    sorted[pos] = make_float4(p.x, p.y, p.z, __int_as_float(base + i));
}

// off = exclusive scan of counts[0, cells + 1): tiles of 16 consecutive values per thread, block scan, tile
// offset by wave look-back (radix.h) over a tile counter; blocks past the device-side length exit.
constexpr int kScanThreads = 1024, kScanPer = 16, kScanTile = kScanThreads * kScanPer;

__global__ __launch_bounds__(kScanThreads) void scan_dev_kernel(const uint32_t* in, uint32_t* out, int* bb,
                                                                unsigned long long* st, uint32_t epoch, int* err) {
    __shared__ int s_tile;
    __shared__ uint32_t s_wave[kScanThreads / 64], s_before;
    if (bb[10] || bb[6] <= 0) return;
    const size_t len = grid_cells(bb) + 1;
    if (threadIdx.x == 0)
        s_tile = (int)__hip_atomic_fetch_add(reinterpret_cast<unsigned*>(bb + 16), 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int tile = s_tile;
    const size_t base = (size_t)tile * kScanTile;
    if (base >= len) return;   // block-uniform
    const size_t i0 = base + (size_t)threadIdx.x * kScanPer;
    uint32_t v[kScanPer];
    if (i0 + kScanPer <= len) {
#pragma unroll
        for (int q = 0; q < kScanPer / 4; ++q) {
            const uint4 a = *reinterpret_cast<const uint4*>(in + i0 + 4 * q);
            v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kScanPer; ++j) v[j] = i0 + j < len ? in[i0 + j] : 0u;
    }
    uint32_t t = 0;
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) t += v[j];
    uint32_t total;
    uint32_t run = block_exclusive_scan<kScanThreads>(t, s_wave, &total);
    if (threadIdx.x < 64) {
        uint32_t before = 0;
        if (tile == 0) {
            if (threadIdx.x == 0) lb_store(st, epoch, kLbInc, total);
        } else {
            if (threadIdx.x == 0) lb_store(st + tile, epoch, kLbAgg, total);
            before = wave_lookback(st, tile, epoch, err);
            if (threadIdx.x == 0) lb_store(st + tile, epoch, kLbInc, before + total);
        }
        if (threadIdx.x == 0) s_before = before;
    }
    __syncthreads();
    run += s_before;
    if (i0 + kScanPer <= len) {
#pragma unroll
        for (int q = 0; q < kScanPer / 4; ++q) {
            uint4 a;
            a.x = run; run += v[4 * q];
            a.y = run; run += v[4 * q + 1];
            a.z = run; run += v[4 * q + 2];
            a.w = run; run += v[4 * q + 3];
            *reinterpret_cast<uint4*>(out + i0 + 4 * q) = a;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kScanPer; ++j)
            if (i0 + j < len) {
                out[i0 + j] = run;
                run += v[j];
            }
    }
}

size_t grid_scan_tiles(size_t cells_cap) { return (cells_cap + kScanTile - 1) / kScanTile; }

hipError_t launch_grid_build_dev(const float4* orig, int n_max, int sx, int* d_bb, uint32_t* counts, uint32_t* off,
                                 uint32_t* fill, size_t cells_cap, int* cell, float4* sorted, int base,
                                 unsigned long long* scan_state, uint32_t epoch, int* h_bb, hipEvent_t ev_bb,
                                 int* err, hipStream_t s) {
    if (n_max <= 0) return hipSuccess;
    const unsigned cb = (unsigned)std::min<size_t>(2048, (cells_cap + 255) / 256);
    hipLaunchKernelGGL(grid_clear_dev_kernel, dim3(std::max(cb, 1u)), dim3(256), 0, s, d_bb, counts, fill, cells_cap);
    // the box, count and overflow flag are final here: the host reads them while the build goes on
    hipError_t e = hipMemcpyAsync(h_bb, d_bb, 11 * sizeof(int), hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    if ((e = hipEventRecord(ev_bb, s)) != hipSuccess) return e;
    const dim3 g((n_max + 255) / 256), b(256);
    hipLaunchKernelGGL(map_count_dev_kernel, g, b, 0, s, orig, d_bb, (float)sx, cell, counts);
    hipLaunchKernelGGL(scan_dev_kernel, dim3((unsigned)grid_scan_tiles(cells_cap + 1)), dim3(kScanThreads), 0, s,
                       counts, off, d_bb, scan_state, epoch, err);
    hipLaunchKernelGGL(map_scatter_dev_kernel, g, b, 0, s, orig, d_bb, cell, off, fill, sorted, base, err);
    return hipGetLastError();
}

hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, size_t n, void* tmp, size_t& tmp_bytes,
                              hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, n, s);
}

}  // namespace lmsf
