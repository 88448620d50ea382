// Shared pieces of the single-pass radix sort (k_sort.hip) and its voxel-filter callers (k_voxel.hip):
// scratch layout, the key-bound -> pass-count rule, the block histogram and the decoupled look-back.
//
// Look-back words are 64-bit: the sort's epoch (high 32 bits) | flag (2 bits) | count (30 bits).  A word of an
// older sort reads as "not published", so the state arrays are never cleared (one memset at allocation).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lmsf {

constexpr int kRadixThreads = 1024;                      // 16 waves; digit d's counts and look-back: thread d
constexpr int kRadixRounds = 8;                          // pairs per thread (per wave: 8 rounds of 64)
constexpr int kRadixTile = kRadixThreads * kRadixRounds;  // 8192 pairs per tile (r03: 2048-pair tiles spent
                                                          // ~20 us per pass in look-back round trips on 6e5 pairs)
constexpr int kRadixDigits = 256;
constexpr int kRadixPasses = 4;                           // 8-bit digits of keys < 2^32
constexpr uint32_t kLbAgg = 1u << 30, kLbInc = 2u << 30, kLbCount = (1u << 30) - 1u;
constexpr unsigned kLbSpinLimit = 1u << 24;               // bounded waits: a broken invariant is a wrong result

// Scratch of a sort over up to n pairs (uint32 words): hist[4][256] | ctr[16] | state[4][tiles][256] (u64) |
// seg_state[seg tiles] (u64, the voxel segment pass: tiles of kSegTile positions).
struct RadixScratch {
    uint32_t* hist;
    uint32_t* ctr;                      // [0..3] tile counters of the passes, [4] of the segment scan
    unsigned long long* state;
    unsigned long long* seg_state;
    int tiles;
};

constexpr int kSegTile = 4096;

inline int radix_tiles(size_t n) { return (int)((n + kRadixTile - 1) / kRadixTile); }
inline int seg_tiles(size_t n) { return (int)((n + kSegTile - 1) / kSegTile); }

inline size_t radix_scratch_words(size_t n) {
    const size_t t = (size_t)radix_tiles(n);
    return (size_t)kRadixPasses * kRadixDigits + 16 + 2 * ((size_t)kRadixPasses * t * kRadixDigits + seg_tiles(n));
}

inline RadixScratch radix_scratch(uint32_t* base, size_t n) {
    RadixScratch r;
    r.tiles = radix_tiles(n);
    r.hist = base;
    r.ctr = base + kRadixPasses * kRadixDigits;
    r.state = reinterpret_cast<unsigned long long*>(r.ctr + 16);   // 8-byte aligned: 1040 words in
    r.seg_state = r.state + (size_t)kRadixPasses * r.tiles * kRadixDigits;
    return r;
}

// Digit passes that a sort of keys < bound needs (the rest leave the order unchanged and are skipped):
// 8 bits each, at least one.  Pass p reads buffer A when p is even; the result is in B when the count is odd.
__device__ __forceinline__ int radix_pass_count(uint32_t bound) {
    const int bits = bound <= 1u ? 0 : 32 - __clz((int)(bound - 1u));
    return bits <= 8 ? 1 : (bits + 7) >> 3;
}

__device__ __forceinline__ unsigned long long lb_load(const unsigned long long* p) {
    return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(unsigned long long* p, uint32_t epoch, uint32_t flag, uint32_t count) {
    __hip_atomic_store(p, ((unsigned long long)epoch << 32) | flag | count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum of the counts of tiles [0, tile) from their look-back words st[p * stride]: W predecessors are read at
// once (independent loads in flight: one round trip covers W tiles), summed nearest first until an inclusive
// word; an unpublished word restarts the window there.  The tiles come from a start-order counter, so every
// waited-on tile's block runs.
template <int W>
__device__ __forceinline__ uint32_t lookback_sum(const unsigned long long* st, int tile, size_t stride,
                                                 uint32_t epoch) {
    uint32_t sum = 0;
    int p = tile - 1;
    unsigned spins = 0;
    while (p >= 0) {
        unsigned long long v[W];
#pragma unroll
        for (int j = 0; j < W; ++j) v[j] = p - j >= 0 ? lb_load(st + (size_t)(p - j) * stride) : 0ull;
        int adv = 0;
        bool done = false;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            if (done || adv != j) continue;
            if (p - j < 0) {
                done = true;
                continue;
            }
            const uint32_t lo = (uint32_t)v[j], flag = lo & ~kLbCount;
            if ((uint32_t)(v[j] >> 32) != epoch || flag == 0u) continue;   // not yet published: wait here
            sum += lo & kLbCount;
            adv = j + 1;
            done = flag == kLbInc;
        }
        if (done) break;
        p -= adv;
        if (adv == 0) {
            if (++spins > kLbSpinLimit) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return sum;
}

// Sum of the counts of tiles [0, tile) by one wave: lane j reads tile p - j (64 tiles per round trip), the
// nearest inclusive word ends the walk, the nearest unpublished one resumes it; every lane returns the sum.
__device__ __forceinline__ uint32_t wave_lookback(const unsigned long long* st, int tile, uint32_t epoch) {
    const int lane = threadIdx.x & 63;
    uint32_t sum = 0;
    int p = tile - 1;
    unsigned spins = 0;
    while (p >= 0) {
        const int q = p - lane;
        const unsigned long long v = q >= 0 ? lb_load(st + q) : 0ull;
        const uint32_t lo = (uint32_t)v, flag = lo & ~kLbCount;
        const bool ready = q < 0 || ((uint32_t)(v >> 32) == epoch && flag != 0u);
        const bool inc = q < 0 || (ready && flag == kLbInc);   // before tile 0: an inclusive zero
        const unsigned long long notready = __ballot(!ready), incm = __ballot(inc);
        const unsigned long long stopm = notready | incm;
        const int stop = stopm ? __ffsll((long long)stopm) - 1 : 64;
        const bool stop_inc = stop < 64 && ((incm >> stop) & 1ull);
        uint32_t c = (lane < stop || (lane == stop && stop_inc)) && q >= 0 ? (lo & kLbCount) : 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
        sum += c;
        if (stop_inc) break;
        p -= stop;
        if (stop == 0) {
            if (++spins > kLbSpinLimit) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return sum;
}

// Exclusive scan over the block's threads (kBlock = whole waves, <= 1024) of one value each; *total = the sum.
template <int kBlock>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wave, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint32_t c = s_wave[w];
        before += w < wave ? c : 0u;
        all += c;
    }
    *total = all;
    return before + inc - v;
}

// Adds the digit histograms of one thread's keys of the needed passes to the block's LDS hist, then (after
// the caller's loop) radix_hist_commit adds the non-zero bins to the global hist.
__device__ __forceinline__ void radix_hist_add(uint32_t (*h)[kRadixDigits], uint32_t key, int passes) {
#pragma unroll
    for (int p = 0; p < kRadixPasses; ++p)
        if (p < passes) atomicAdd(&h[p][(key >> (8 * p)) & 255u], 1u);
}

__device__ __forceinline__ void radix_hist_commit(uint32_t (*h)[kRadixDigits], uint32_t* hist, int passes) {
    __syncthreads();
    for (int i = threadIdx.x; i < passes * kRadixDigits; i += blockDim.x) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(&hist[i], c);
    }
}

// The digit passes over (ka, va) <-> (kb, vb) of n pairs whose keys are < *bound (device word), with the
// global histogram of every needed pass already in rs.hist and rs.ctr[0..3] zeroed: kRadixPasses launches.
// Pass 0 takes its values from v0 (nullptr: the pair's index) instead of va.  epoch: non-zero, new per sort.
hipError_t launch_radix_passes(uint32_t* ka, int* va, uint32_t* kb, int* vb, const int* v0, int n,
                               const uint32_t* bound, const RadixScratch& rs, uint32_t epoch, hipStream_t s);

}  // namespace lmsf
