// Shared pieces of the single-pass radix sort (k_sort.hip) and its voxel-filter callers (k_voxel.hip):
// scratch layout, the key-bound -> pass-count rule, the block histogram and the decoupled look-back.
//
// Look-back words are 64-bit: the sort's epoch (high 32 bits) | flag (2 bits) | count (30 bits).  A word of an
// older sort reads as "not published", so the state arrays are never cleared (one memset at allocation, on the
// stream that reads them).  Epochs come from one process-wide counter (next_lookback_epoch), so they never
// restart: a word whose epoch is NEWER than the running sort's was not written by any earlier sort on this
// memory -- it is left over from another allocation (the r04 fault: a null-stream memset not yet done when
// the sort ran) -- and the walk flags kFaultForeignEpoch instead of waiting on it.  A wait that exceeds its
// bound flags kFaultLookbackWait.  Every scatter whose index comes from a look-back sum is bounds-checked by its
// kernel (kFaultRadixScatter / kFaultSegment / kFaultGridScatter).  The flags go to a device word the host reads
// back at the next Solve / batch wait and reports as LMSF_ERR_HIP.
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
// a word of a newer sort than this one (signed distance: the counter may wrap)
__device__ __forceinline__ bool lb_foreign(unsigned long long v, uint32_t epoch) {
    return (int32_t)((uint32_t)(v >> 32) - epoch) > 0;
}

__device__ __forceinline__ void lb_fault(int* err, int bit) {
    if (err) atomicOr(err, bit);
}

__device__ __forceinline__ void lb_store(unsigned long long* p, uint32_t epoch, uint32_t flag, uint32_t count) {
    __hip_atomic_store(p, ((unsigned long long)epoch << 32) | flag | count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum of the counts of tiles [0, tile) by one wave: lane j reads tile p - j (64 tiles per round trip), the
// nearest inclusive word ends the walk, the nearest unpublished one resumes it; every lane returns the sum.
// A foreign word or an exhausted wait ends the walk with the fault flagged in *err (the sum is then unusable).
__device__ __forceinline__ uint32_t wave_lookback(const unsigned long long* st, int tile, uint32_t epoch, int* err) {
    const int lane = threadIdx.x & 63;
    uint32_t sum = 0;
    int p = tile - 1;
    unsigned spins = 0;
    while (p >= 0) {
        const int q = p - lane;
        const unsigned long long v = q >= 0 ? lb_load(st + q) : 0ull;
        if (__ballot(q >= 0 && lb_foreign(v, epoch))) {
            if (lane == 0) lb_fault(err, kFaultForeignEpoch);
            break;
        }
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
            if (++spins > kLbSpinLimit) {
                if (lane == 0) lb_fault(err, kFaultLookbackWait);
                break;
            }
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
// Pass 0 takes its values from v0 (nullptr: the pair's index) instead of va.  epoch: next_lookback_epoch(), new
// per sort.  err: the fault word (radix.h header).  inject (LMSF_OPT_FAULT_INJECT, tests only): 1 = pass 0's tile
// 1 takes a prefix 2^28 too large (an out-of-range scatter), 2 = pass 0's tile 0 publishes a foreign epoch.
hipError_t launch_radix_passes(uint32_t* ka, int* va, uint32_t* kb, int* vb, const int* v0, int n,
                               const uint32_t* bound, const RadixScratch& rs, uint32_t epoch, int* err, int inject,
                               hipStream_t s);

}  // namespace lmsf
