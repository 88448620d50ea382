// Stable LSD radix sort of (uint32 key < 2^31, int32 value) pairs for the voxel filter (k_voxel.hip).
//
// Why: the tracker rebuilds its keyframe windows with a VoxelGrid every keyframe, and hipCUB's dispatch of a
// ~6e5-pair sort is a merge sort of ~20 dependent launches (~70 us of host enqueue time alone, r03 probe,
// tools/hostcost) on the tracking critical path.  Here: one histogram launch and four single-pass digit
// launches (8-bit digits; one memset clears the counters first) -- 6 enqueues.
//
// Each pass kernel takes tiles of kTile pairs in the order the blocks start (a tile counter, so a block
// only ever waits for tiles whose blocks are already running), ranks its pairs stably per digit (wave ballots
// over the 8 digit bits, waves and rounds in input order), publishes its per-digit tile count, finds the
// count of every earlier tile by decoupled look-back (aggregate / inclusive flags in the top bits, agent-scope
// atomics: the tiles' blocks run on different XCDs), and scatters.  Equal keys keep their input order, so the
// result equals any stable sort of the pairs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>

#include "lmsf_internal.h"

namespace lmsf {

namespace {

constexpr int kSortThreads = 256;
constexpr int kSortRounds = 8;                         // pairs per thread
constexpr int kSortTile = kSortThreads * kSortRounds;  // 2048 pairs per tile
constexpr int kDigits = 256;
constexpr int kPasses = 4;                             // 32 key bits; keys < 2^31 leave the last digit < 128
constexpr uint32_t kFlagAgg = 1u << 30, kFlagInc = 2u << 30, kCountMask = (1u << 30) - 1u;
constexpr unsigned kLookbackSpinLimit = 1u << 26;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// hist[pass][digit] over all n keys (zeroed by the caller's memset).
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(const uint32_t* keys, int n, uint32_t* hist) {
    __shared__ uint32_t h[kPasses][kDigits];
    for (int i = threadIdx.x; i < kPasses * kDigits; i += kSortThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    for (int i = blockIdx.x * kSortThreads + threadIdx.x; i < n; i += gridDim.x * kSortThreads) {
        const uint32_t k = keys[i];
#pragma unroll
        for (int p = 0; p < kPasses; ++p) atomicAdd(&h[p][(k >> (8 * p)) & 255u], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kPasses * kDigits; i += kSortThreads) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(&hist[i], c);
    }
}

__global__ __launch_bounds__(kSortThreads) void radix_pass_kernel(const uint32_t* k_in, const int* v_in, uint32_t* k_out,
                                                                  int* v_out, int n, int shift, const uint32_t* hist,
                                                                  uint32_t* state, uint32_t* tile_ctr) {
    __shared__ uint32_t s_run[kDigits], s_base[kDigits], s_off[kDigits];
    __shared__ uint32_t s_wc[kSortThreads / 64][kDigits];
    __shared__ int s_tile;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = (int)__hip_atomic_fetch_add(tile_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // digit starts of this pass: exclusive scan of the global histogram (Hillis-Steele in LDS)
    s_base[tid] = hist[tid];
    s_run[tid] = 0;
    __syncthreads();
    for (int o = 1; o < kDigits; o <<= 1) {
        const uint32_t v = tid >= o ? s_base[tid - o] : 0u;
        __syncthreads();
        s_base[tid] += v;
        __syncthreads();
    }
    const uint32_t excl_base = s_base[tid] - hist[tid];
    __syncthreads();
    s_base[tid] = excl_base;
    const int tile = s_tile;
    const int base = tile * kSortTile;
    uint32_t key[kSortRounds];
    int val[kSortRounds];
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const int i = base + r * kSortThreads + tid;
        key[r] = i < n ? k_in[i] : 0u;
        val[r] = i < n ? v_in[i] : 0;
    }
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t rank[kSortRounds];
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const int i = base + r * kSortThreads + tid;
        const bool valid = i < n;
        const uint32_t d = (key[r] >> shift) & 255u;
        for (int k = tid; k < (kSortThreads / 64) * kDigits; k += kSortThreads) (&s_wc[0][0])[k] = 0;
        __syncthreads();
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const unsigned long long m = __ballot(((d >> bit) & 1u) != 0u);
            peers &= ((d >> bit) & 1u) ? m : ~m;
        }
        if (valid && (peers & lt) == 0ull) s_wc[wave][d] = (uint32_t)__popcll(peers);   // the lowest lane of its digit
        __syncthreads();
        uint32_t before = s_run[d];
        for (int w = 0; w < wave; ++w) before += s_wc[w][d];
        rank[r] = before + (uint32_t)__popcll(peers & lt);
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < kSortThreads / 64; ++w) add += s_wc[w][tid];
        s_run[tid] += add;
        __syncthreads();
    }
    // publish this tile's counts, then the counts of every earlier tile per digit (decoupled look-back)
    uint32_t* my = state + (size_t)tile * kDigits;
    const uint32_t cnt = s_run[tid];
    st_agent(&my[tid], kFlagAgg | cnt);
    uint32_t excl = 0;
    for (int p = tile - 1; p >= 0; --p) {
        uint32_t v;
        unsigned spins = 0;
        while (((v = ld_agent(&state[(size_t)p * kDigits + tid])) & ~kCountMask) == 0u) {
            if (++spins > kLookbackSpinLimit) break;   // bounded: a broken invariant shows as a wrong sort, not a hang
            __builtin_amdgcn_s_sleep(1);
        }
        excl += v & kCountMask;
        if ((v & ~kCountMask) == kFlagInc) break;
    }
    st_agent(&my[tid], kFlagInc | (excl + cnt));
    s_off[tid] = s_base[tid] + excl;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const int i = base + r * kSortThreads + tid;
        if (i < n) {
            const uint32_t pos = s_off[(key[r] >> shift) & 255u] + rank[r];
            k_out[pos] = key[r];
            v_out[pos] = val[r];
        }
    }
}

}  // namespace

size_t radix_sort_scratch_words(size_t n) {
    const size_t tiles = (n + kSortTile - 1) / kSortTile;
    return (size_t)kPasses * kDigits + kPasses * 16 + (size_t)kPasses * tiles * kDigits;
}

// Sorts (keys, vals) of n pairs in place (the 4 passes ping-pong through k_tmp / v_tmp and end in keys / vals).
// scratch: radix_sort_scratch_words(n) uint32 words.
hipError_t radix_sort_pairs(uint32_t* keys, int* vals, uint32_t* k_tmp, int* v_tmp, int n, uint32_t* scratch,
                            hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const size_t tiles = (size_t)(n + kSortTile - 1) / kSortTile;
    uint32_t* hist = scratch;                           // [4][256]
    uint32_t* ctr = scratch + kPasses * kDigits;        // [4] tile counters, 64 B apart
    uint32_t* state = ctr + kPasses * 16;               // [4][tiles][256]
    hipError_t e = hipMemsetAsync(scratch, 0, radix_sort_scratch_words((size_t)n) * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const int hb = (int)std::min<size_t>((n + 4095) / 4096, 1024);
    hipLaunchKernelGGL(radix_hist_kernel, dim3(hb), dim3(kSortThreads), 0, s, keys, n, hist);
    uint32_t* ki = keys;
    int* vi = vals;
    uint32_t* ko = k_tmp;
    int* vo = v_tmp;
    for (int p = 0; p < kPasses; ++p) {
        hipLaunchKernelGGL(radix_pass_kernel, dim3((unsigned)tiles), dim3(kSortThreads), 0, s, ki, vi, ko, vo, n, 8 * p,
                           hist + p * kDigits, state + (size_t)p * tiles * kDigits, ctr + p * 16);
        std::swap(ki, ko);
        std::swap(vi, vo);
    }
    return hipGetLastError();
}

}  // namespace lmsf
