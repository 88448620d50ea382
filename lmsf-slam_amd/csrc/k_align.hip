// 1-NN alignment fitness: Slam3D::PointCloudAlignmentEvaluate::AlignmentScore
// (REG/alignEvaluate.hpp:55-87), the loop-closure / relocalisation check that reuses the
// neighbour search with k = 1.
//
// Per source point: pcl::transformPointCloud with an Eigen::Matrix4f (float arithmetic, row-wise
// m0 x + m1 y + m2 z + m3, no contraction), nearest target point by squared float distance
// ((dx dx + dy dy) + dz dz, as FLANN's L2), counted when d2 <= inlier_thresh.  Only neighbours
// with d2 <= inlier_thresh matter, so the search visits the cells of the target's 1 m grid whose
// box is within sqrt(thresh) (inflated) of the query (the callers use 0.1 and 1 m^2: loopDetection.hpp:177, :411,
// :451; backend_lifelong.hpp:319).  Sums: per-block fixed-order tree in double, then one ordered
// pass over the block partials (deterministic; the reference sums sequentially -> rel. 1e-12).
#include <hip/hip_runtime.h>

#include "lmsf_internal.h"

namespace lmsf {

constexpr int kAlignBlock = 256;

__device__ __forceinline__ int acell(float v, int o) {
    return (int)fminf(fmaxf(floorf(v), -1073741824.f), 1073741824.f) - o;
}

__global__ void __launch_bounds__(kAlignBlock) align_kernel(GridView g, const float4* src, int n, Affine34f M,
                                                            double thresh, int R, double* part_sum,
                                                            unsigned int* part_cnt) {
#pragma clang fp contract(off)
    __shared__ double ssum[kAlignBlock];
    __shared__ unsigned int scnt[kAlignBlock];
    const int i = blockIdx.x * kAlignBlock + threadIdx.x;
    double v = 0.0;
    unsigned int c = 0;
    if (i < n) {
        const float4 p = src[i];
        const float qx = M.m[0] * p.x + M.m[1] * p.y + M.m[2] * p.z + M.m[3];
        const float qy = M.m[4] * p.x + M.m[5] * p.y + M.m[6] * p.z + M.m[7];
        const float qz = M.m[8] * p.x + M.m[9] * p.y + M.m[10] * p.z + M.m[11];
        const int cy = acell(qy, g.oy), cz = acell(qz, g.oz);
        // rows / cells whose box lies farther than sqrt(lim) are skipped; lim is inflated so that
        // float rounding of d2 can never admit a skipped point
        const double lim = thresh * (1.0 + 1e-5) + 1e-7;
        float best = INFINITY;
        for (int z = max(cz - R, 0); z <= min(cz + R, g.nz - 1); ++z) {
            const double bz = (double)g.oz + z;
            const double ddz = fmax(0.0, fmax(bz - (double)qz, (double)qz - (bz + 1.0)));
            for (int y = max(cy - R, 0); y <= min(cy + R, g.ny - 1); ++y) {
                const double by = (double)g.oy + y;
                const double ddy = fmax(0.0, fmax(by - (double)qy, (double)qy - (by + 1.0)));
                const double rem = lim - ddz * ddz - ddy * ddy;
                if (rem < 0.0) continue;
                const double r = sqrt(rem);       // x-window in slices (g.sx per metre)
                const int x0 = max(0, (int)fmax(floor(((double)qx - r) * g.sx), -1073741824.0) - g.ox);
                const int x1 = min(g.nx - 1, (int)fmin(floor(((double)qx + r) * g.sx), 1073741824.0) - g.ox);
                if (x0 > x1) continue;
                const size_t row = ((size_t)z * g.ny + y) * g.nx;
                const uint32_t a = g.off[row + x0], b = g.off[row + x1 + 1];
                for (uint32_t k = a; k < b; ++k) {
                    const float4 m = g.pts[k];
                    const float dx = qx - m.x, dy = qy - m.y, dz = qz - m.z;
                    const float d2 = dx * dx + dy * dy + dz * dz;
                    best = fminf(best, d2);
                }
            }
        }
        if ((double)best <= thresh) {                 // float distance promoted, as the reference
            v = (double)best;
            c = 1;
        }
    }
    ssum[threadIdx.x] = v;
    scnt[threadIdx.x] = c;
    __syncthreads();
    for (int s = kAlignBlock / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            ssum[threadIdx.x] += ssum[threadIdx.x + s];
            scnt[threadIdx.x] += scnt[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part_sum[blockIdx.x] = ssum[0];
        part_cnt[blockIdx.x] = scnt[0];
    }
}

__global__ void align_final_kernel(const double* part_sum, const unsigned int* part_cnt, int nparts, double* out) {
    if (threadIdx.x != 0) return;
    double s = 0.0;
    unsigned long long c = 0;
    for (int b = 0; b < nparts; ++b) {
        s += part_sum[b];
        c += part_cnt[b];
    }
    out[0] = s;
    out[1] = (double)c;
}

int align_parts(int n) { return (n + kAlignBlock - 1) / kAlignBlock; }

hipError_t launch_align(const GridView& g, const float4* src, int n, const Affine34f& M, double thresh,
                        double* part_sum, unsigned int* part_cnt, double* out2, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    // a point R + 1 cells away has |float dx| >= R > sqrt(thresh): R = floor(sqrt(thresh)) + 1 is
    // exact (R = ceil would miss float distances rounded onto the threshold); rows are culled above
    const int R = thresh < 0.0 ? 0 : (int)floor(sqrt(thresh)) + 1;
    const int nb = align_parts(n);
    hipLaunchKernelGGL(align_kernel, dim3(nb), dim3(kAlignBlock), 0, s, g, src, n, M, thresh, R, part_sum, part_cnt);
    hipLaunchKernelGGL(align_final_kernel, dim3(1), dim3(64), 0, s, part_sum, part_cnt, nb, out2);
    return hipGetLastError();
}

}  // namespace lmsf
