// Block-level integer bounding-box reduction shared by the map-index and voxel kernels: wave
// shuffles, then the block's waves meet in LDS and one lane issues the 6 atomics (one set per
// block instead of one per wave: the per-wave version serialised ~10^4 atomics on 6 words).
#pragma once
#include <hip/hip_runtime.h>
#include <climits>

namespace lmsf {

template <int kBlock>
__device__ __forceinline__ void block_bbox_commit(int lo[3], int hi[3], int* bbox) {
    static_assert(kBlock % 64 == 0 && kBlock <= 1024, "block of whole waves");
    __shared__ int s_lo[3][kBlock / 64], s_hi[3][kBlock / 64];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            lo[d] = min(lo[d], __shfl_xor(lo[d], o, 64));
            hi[d] = max(hi[d], __shfl_xor(hi[d], o, 64));
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            s_lo[d][w] = lo[d];
            s_hi[d][w] = hi[d];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            int a = INT_MAX, b = INT_MIN;
            for (int k = 0; k < kBlock / 64; ++k) {
                a = min(a, s_lo[d][k]);
                b = max(b, s_hi[d][k]);
            }
            atomicMin(&bbox[d], a);
            atomicMax(&bbox[3 + d], b);
        }
    }
}

}  // namespace lmsf
