// Scan ingest in front of the feature extraction, on the device:
//   sensor_msgs/PointCloud2 XYZI decode + pcl::removeNaNFromPointCloud
//       (APPS/MultiLidarSLAM_node.cpp:125-132, APPS = src/apps/src),
//   RotaryLidarPreProcess::Process: per-point relative time in the intensity field
//       (INC/Algorithm/PointClouds/processing/Preprocess/RotaryLidar_preprocessing.hpp:31-104,
//        run by MultiLidarSystem::Process, INC/System/ML_System.hpp:130-135),
//   DistanceFilter::Filter (INC/Algorithm/PointClouds/processing/Filter/distance_filter.hpp:24-43).
//
// removeNaN and the distance filter are stable compactions (flag, hipCUB exclusive scan, scatter).
// The rotary pass is a one-way automaton (half_passed flips once): every point is unwrapped in
// the "first half" mode, the first index whose unwrapped angle passes start + pi is found with
// an atomicMin, and the points after it use the "second half" mode.  Angles: -atan2(y, x)
// evaluated in double and rounded to float (the reference's float atan2 is within 1 ulp; the
// CPU oracle uses the same expression); comparisons against the double M_PI expressions and the
// float rel_time formula as in the reference.
//
// Roofline: HBM-bound byte work: point_step bytes read + 16 B written per point, then 16 B read +
// 16 B written per compaction / rotary pass.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "lmsf_internal.h"

namespace lmsf {

__device__ __forceinline__ float load_f32(const uint8_t* p) {
    uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    return __uint_as_float(v);
}

template <bool kAligned>
__global__ void decode_kernel(const uint8_t* data, int n, uint32_t step, int ox, int oy, int oz, int oi,
                              float4* out, uint32_t* keep) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = data + (size_t)i * step;
    float4 v;
    if (kAligned) {
        v.x = *reinterpret_cast<const float*>(p + ox);
        v.y = *reinterpret_cast<const float*>(p + oy);
        v.z = *reinterpret_cast<const float*>(p + oz);
        v.w = oi >= 0 ? *reinterpret_cast<const float*>(p + oi) : 0.f;
    } else {
        v.x = load_f32(p + ox);
        v.y = load_f32(p + oy);
        v.z = load_f32(p + oz);
        v.w = oi >= 0 ? load_f32(p + oi) : 0.f;
    }
    out[i] = v;
    keep[i] = (isfinite(v.x) && isfinite(v.y) && isfinite(v.z)) ? 1u : 0u;   // removeNaNFromPointCloud
}

__global__ void compact_kernel(const float4* in, const uint32_t* keep, const uint32_t* pos, int n, float4* out,
                               int* count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (keep[i]) out[pos[i]] = in[i];
    if (i == n - 1) *count = (int)(pos[i] + keep[i]);
}

__device__ __forceinline__ float neg_atan2(float y, float x) { return (float)(-atan2((double)y, (double)x)); }

// findStartEndAngle (:77-91)
__global__ void rotary_bounds_kernel(const float4* pts, const int* count, float* se, int* first) {
    const int n = *count;
    if (threadIdx.x != 0 || n == 0) return;
    const float start = neg_atan2(pts[0].y, pts[0].x);
    float end = (float)((double)neg_atan2(pts[n - 1].y, pts[n - 1].x) + 2 * M_PI);
    if (end - start > 3 * M_PI) end = (float)((double)end - 2 * M_PI);        // float difference, promoted
    else if (end - start < M_PI) end = (float)((double)end + 2 * M_PI);
    se[0] = start;
    se[1] = end;
    *first = INT_MAX;
}

__device__ __forceinline__ float unwrap_first(float ori, float start) {   // :42-49
    if ((double)ori < (double)start - M_PI / 2) ori = (float)((double)ori + 2 * M_PI);
    else if ((double)ori > (double)start + M_PI * 3 / 2) ori = (float)((double)ori - 2 * M_PI);
    return ori;
}

__global__ void rotary_switch_kernel(const float4* pts, const int* count, const float* se, int* first) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *count) return;
    const float start = se[0];
    const float ori = unwrap_first(neg_atan2(pts[i].y, pts[i].x), start);
    if (ori - start > M_PI) atomicMin(first, i);                   // :50-53, float difference
}

__global__ void rotary_time_kernel(float4* pts, const int* count, const float* se, const int* first, float period) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *count) return;
    const float start = se[0], end = se[1];
    float ori = neg_atan2(pts[i].y, pts[i].x);
    if (i <= *first) {                                             // half_passed still false here
        ori = unwrap_first(ori, start);
    } else {                                                       // :55-66
        ori = (float)((double)ori + 2 * M_PI);
        if ((double)ori < (double)end - M_PI * 3 / 2) ori = (float)((double)ori + 2 * M_PI);
        else if ((double)ori > (double)end + M_PI / 2) ori = (float)((double)ori - 2 * M_PI);
    }
    pts[i].w = (ori - start) / (end - start) * period;             // :67-69, setPoint -> intensity
}

// DistanceFilter: d = |p| (float norm) promoted to double, keep near < d < far
__global__ void distance_flag_kernel(const float4* pts, const int* count, double near_t, double far_t,
                                     uint32_t* keep) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = *count;
    if (i >= n) return;
    const float4 p = pts[i];
    const double d = (double)sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
    keep[i] = (d > near_t && d < far_t) ? 1u : 0u;
}

// Flags over a host-known count (PointCloudCommonProcess stages, common_processing.hpp:87-112)
__global__ void finite_flag_kernel(const float4* pts, int n, uint32_t* keep) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[i];
    keep[i] = (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) ? 1u : 0u;   // removeNaNFromPointCloud
}

__global__ void distance_flag_n_kernel(const float4* pts, int n, double near_t, double far_t, uint32_t* keep) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[i];
    const double d = (double)sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
    keep[i] = (d > near_t && d < far_t) ? 1u : 0u;
}

hipError_t Ingest::compact_flagged(const float4* in, int n, float4* out, int* n_out, hipStream_t s) {
    int* count = scalars;
    hipError_t e;
    size_t tb = tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, keep, pos, n, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(compact_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, keep, pos, n, out, count);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(n_out, count, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

hipError_t Ingest::finite(const float4* in, int n, float4* out, int* n_out, hipStream_t s) {
    *n_out = 0;
    if (n <= 0) return hipSuccess;
    hipError_t e = reserve((size_t)n, 0);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(finite_flag_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, keep);
    return compact_flagged(in, n, out, n_out, s);
}

hipError_t Ingest::distance(const float4* in, int n, double near_t, double far_t, float4* out, int* n_out,
                            hipStream_t s) {
    *n_out = 0;
    if (n <= 0) return hipSuccess;
    hipError_t e = reserve((size_t)n, 0);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(distance_flag_n_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, near_t, far_t, keep);
    return compact_flagged(in, n, out, n_out, s);
}

hipError_t Ingest::reserve(size_t n, size_t raw_bytes) {
    hipError_t e;
    if (raw_bytes > raw_cap) {
        hipFree(raw);
        raw = nullptr;
        const size_t rc = grow_cap(raw_bytes, raw_cap);
        raw_cap = 0;
        if ((e = hipMalloc((void**)&raw, rc)) != hipSuccess) return e;
        raw_cap = rc;
    }
    if (n <= cap) return hipSuccess;
    n = std::min(grow_cap(n, cap), (size_t)INT32_MAX);
    void* bufs[] = {a, b, keep, pos, scalars, tmp};
    for (void* p : bufs) hipFree(p);
    a = b = nullptr;
    keep = pos = nullptr;
    scalars = nullptr;
    tmp = nullptr;
    cap = 0;
#define IALLOC(p, bytes) if ((e = hipMalloc((void**)&(p), (bytes))) != hipSuccess) return e
    IALLOC(a, n * sizeof(float4));
    IALLOC(b, n * sizeof(float4));
    IALLOC(keep, n * sizeof(uint32_t));
    IALLOC(pos, n * sizeof(uint32_t));
    IALLOC(scalars, 16 * sizeof(int));
    size_t tb = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tb, keep, pos, (int)n);
    tmp_bytes = tb;
    IALLOC(tmp, tmp_bytes);
#undef IALLOC
    cap = n;
    return hipSuccess;
}

void Ingest::release() {
    void* bufs[] = {raw, a, b, keep, pos, scalars, tmp};
    for (void* p : bufs) hipFree(p);
    *this = Ingest();
}

hipError_t Ingest::run(const uint8_t* data_dev, int n, uint32_t step, int ox, int oy, int oz, int oi, float period,
                       double near_t, double far_t, float4** result, int* n_out, hipStream_t s) {
    *n_out = 0;
    *result = a;
    if (n <= 0) return hipSuccess;
    const dim3 g((n + 255) / 256), blk(256);
    int* count = scalars;
    int* first = scalars + 1;
    float* se = reinterpret_cast<float*>(scalars + 2);
    const bool aligned = (step % 4 == 0) && (ox % 4 == 0) && (oy % 4 == 0) && (oz % 4 == 0) && (oi < 0 || oi % 4 == 0) &&
                         (reinterpret_cast<uintptr_t>(data_dev) % 4 == 0);
    if (aligned) hipLaunchKernelGGL(decode_kernel<true>, g, blk, 0, s, data_dev, n, step, ox, oy, oz, oi, b, keep);
    else hipLaunchKernelGGL(decode_kernel<false>, g, blk, 0, s, data_dev, n, step, ox, oy, oz, oi, b, keep);
    size_t tb = tmp_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, keep, pos, n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(compact_kernel, g, blk, 0, s, b, keep, pos, n, a, count);
    if (period > 0.f) {
        hipLaunchKernelGGL(rotary_bounds_kernel, dim3(1), dim3(64), 0, s, a, count, se, first);
        hipLaunchKernelGGL(rotary_switch_kernel, g, blk, 0, s, a, count, se, first);
        hipLaunchKernelGGL(rotary_time_kernel, g, blk, 0, s, a, count, se, first, period);
    }
    if (near_t != 0.0 || far_t != 0.0) {
        hipLaunchKernelGGL(distance_flag_kernel, g, blk, 0, s, a, count, near_t, far_t, keep);
        // points beyond the current count carry stale flags: clear them by masking in the scan input
        int hc = 0;
        if ((e = hipMemcpyAsync(&hc, count, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (hc == 0) return hipSuccess;
        tb = tmp_bytes;
        if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, keep, pos, hc, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(compact_kernel, dim3((hc + 255) / 256), blk, 0, s, a, keep, pos, hc, b, count);
        *result = b;
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(n_out, count, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

}  // namespace lmsf
