// Stable LSD radix sort of (uint32 key, int32 value) pairs for the voxel filter (k_voxel.hip).
//
// Why: the tracker rebuilds its keyframe windows with a VoxelGrid every keyframe, and hipCUB's dispatch of a
// ~6e5-pair sort is a merge sort of ~20 dependent launches (~70 us of host enqueue time alone, r03 probe,
// tools/hostcost) on the tracking critical path.  Here the caller's key kernel also builds the digit
// histograms (radix.h), and each 8-bit digit is one launch; digits above the key bound are skipped on the
// device (a surf window's keys span ~24 bits: 3 passes).
//
// A pass block (1024 threads) takes a tile of 8192 pairs in block start order (a tile counter, so a block only ever waits
// for tiles whose blocks are already running).  Each wave ranks its own 512 consecutive pairs (8 rounds of
// 64: ballots over the 8 digit bits, running per-digit counts in the wave's LDS row -- no block barrier per
// round), one barrier turns the 16 rows into per-wave prefixes and the tile's digit counts, the counts are
// published and the counts of all earlier tiles found by decoupled look-back (block_lookback: 32 predecessors
// per round trip, agent-scope words, the tiles' blocks run on different XCDs), and the pairs are scattered.  Tile order
// = wave, round, lane = input order, so equal keys keep their input order.
#include <hip/hip_runtime.h>

#include "lmsf_internal.h"
#include "radix.h"

namespace lmsf {

namespace {

constexpr int kLbParts = kRadixThreads / kRadixDigits;   // threads per digit in the look-back (4)
constexpr int kLbWin = 8;                                 // tiles each of them reads per round trip (16: spills)

// Decoupled look-back of the 256 digit counts by the whole block: per round trip, digit d's kLbParts threads
// read kLbWin consecutive predecessor tiles each (32 tiles per round trip, nearest first), and the digit's
// part-0 thread combines the parts in order -- summing up to the first inclusive word, or up to the first
// unpublished one, where the next round resumes.  Returns, to the part-0 thread of each digit, the count of
// the digit in all earlier tiles.  A foreign word (radix.h) ends the digit's walk and an exhausted wait ends all
// of them, both flagged in *err.
__device__ __forceinline__ uint32_t block_lookback(const unsigned long long* state, int tile, uint32_t epoch, int* err) {
    __shared__ uint32_t s_sum[kLbParts][kRadixDigits];
    __shared__ int s_stat[kLbParts][kRadixDigits];
    __shared__ int s_next[kRadixDigits];
    const int d = threadIdx.x & (kRadixDigits - 1), part = threadIdx.x / kRadixDigits;
    if (part == 0) s_next[d] = tile - 1;
    __syncthreads();
    uint32_t before = 0;
    unsigned spins = 0;
    for (;;) {
        const int pd = s_next[d];   // -1: this digit is done
        uint32_t sum = 0;
        int stat = -1;              // -1: all kLbWin ready aggregates; -2: reached an inclusive word or tile 0;
                                    // >= 0: the first unpublished tile
        if (pd >= 0) {
            const int hi = pd - kLbWin * part;
            unsigned long long v[kLbWin];
#pragma unroll
            for (int j = 0; j < kLbWin; ++j) v[j] = hi - j >= 0 ? lb_load(state + (size_t)(hi - j) * kRadixDigits + d) : 0ull;
#pragma unroll
            for (int j = 0; j < kLbWin; ++j) {
                if (stat != -1) continue;
                if (hi - j < 0) {
                    stat = -2;
                    continue;
                }
                if (lb_foreign(v[j], epoch)) {
                    lb_fault(err, kFaultForeignEpoch);
                    stat = -2;
                    continue;
                }
                const uint32_t lo = (uint32_t)v[j], flag = lo & ~kLbCount;
                if ((uint32_t)(v[j] >> 32) != epoch || flag == 0u) {
                    stat = hi - j;
                    continue;
                }
                sum += lo & kLbCount;
                if (flag == kLbInc) stat = -2;
            }
        }
        s_sum[part][d] = sum;
        s_stat[part][d] = stat;
        __syncthreads();
        bool progress = true;
        if (part == 0 && pd >= 0) {
            int next = pd - kLbWin * kLbParts;
            for (int q = 0; q < kLbParts; ++q) {
                before += s_sum[q][d];
                const int sq = s_stat[q][d];
                if (sq == -1) continue;
                next = sq == -2 ? -1 : sq;
                progress = sq != pd;
                break;
            }
            if (next < -1) next = -1;
            s_next[d] = next;
        }
        const int pending = __syncthreads_or(part == 0 && s_next[d] >= 0);
        if (!pending) break;
        if (__syncthreads_or(!progress)) {   // an unpublished nearest tile: wait a little
            if (++spins > kLbSpinLimit) {
                if (threadIdx.x == 0) lb_fault(err, kFaultLookbackWait);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return before;
}

__global__ __launch_bounds__(kRadixThreads) void radix_pass_kernel(uint32_t* ka, int* va, uint32_t* kb, int* vb, const int* v0, int n,
                                                                   int pass, const uint32_t* bound,
                                                                   const uint32_t* hist, uint32_t* ctr,
                                                                   unsigned long long* state, uint32_t epoch,
                                                                   int* err, int inject) {
    if (pass >= radix_pass_count(*bound)) return;   // keys < 2^(8 pass): this digit is 0 for all of them
    const uint32_t* ki = pass & 1 ? kb : ka;
    const int* vi = pass & 1 ? vb : (pass == 0 ? v0 : va);
    uint32_t* ko = pass & 1 ? ka : kb;
    int* vo = pass & 1 ? va : vb;
    const int shift = 8 * pass;
    __shared__ uint32_t s_cnt[kRadixThreads / 64][kRadixDigits];   // per-wave running counts -> wave prefixes
    __shared__ uint32_t s_off[kRadixDigits];
    __shared__ uint32_t s_wave[kRadixThreads / 64];
    __shared__ int s_tile;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = (int)__hip_atomic_fetch_add(&ctr[pass], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = tid; k < (kRadixThreads / 64) * kRadixDigits; k += kRadixThreads) (&s_cnt[0][0])[k] = 0u;
    const uint32_t h = tid < kRadixDigits ? hist[pass * kRadixDigits + tid] : 0u;
    __syncthreads();
    const int tile = s_tile;
    const int base = tile * kRadixTile + wave * (64 * kRadixRounds);
    uint32_t key[kRadixRounds], rank[kRadixRounds];
    int val[kRadixRounds];
#pragma unroll
    for (int r = 0; r < kRadixRounds; ++r) {
        const int i = base + r * 64 + lane;
        key[r] = i < n ? ki[i] : 0u;
        val[r] = i < n ? (vi ? vi[i] : i) : 0;
    }
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int r = 0; r < kRadixRounds; ++r) {
        const bool valid = base + r * 64 + lane < n;
        const uint32_t d = (key[r] >> shift) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const unsigned long long m = __ballot(((d >> bit) & 1u) != 0u);
            peers &= ((d >> bit) & 1u) ? m : ~m;
        }
        // every lane reads its digit's count before the group's lowest lane writes it (one wave: LDS in order)
        const uint32_t prev = s_cnt[wave][d];
        rank[r] = prev + (uint32_t)__popcll(peers & lt);
        if (valid && (peers & lt) == 0ull) s_cnt[wave][d] = prev + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // digit tid: the waves' counts -> per-wave exclusive prefixes, the tile's count
    uint32_t cnt = 0;
    unsigned long long* my = state + (size_t)tile * kRadixDigits + tid;
    if (tid < kRadixDigits) {
#pragma unroll
        for (int w = 0; w < kRadixThreads / 64; ++w) {
            const uint32_t c = s_cnt[w][tid];
            s_cnt[w][tid] = cnt;
            cnt += c;
        }
        // inject 2 (tests): tile 0 publishes a word of a newer epoch, as memory of another allocation would hold
        const uint32_t e0 = inject == 2 && pass == 0 && tile == 0 ? epoch + 0x40000000u : epoch;   // never reached by a real sort
        if (tile > 0) lb_store(my, epoch, kLbAgg, cnt);
        else lb_store(my, e0, kLbInc, cnt);
    }
    uint32_t total;
    const uint32_t digit_base = block_exclusive_scan<kRadixThreads>(h, s_wave, &total);
    uint32_t before = block_lookback(state, tile, epoch, err);
    if (inject == 1 && pass == 0 && tile == 1) before += 1u << 28;   // tests: a stale prefix
    if (tid < kRadixDigits) {
        if (tile > 0) lb_store(my, epoch, kLbInc, before + cnt);
        s_off[tid] = digit_base + before;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRadixRounds; ++r) {
        const int i = base + r * 64 + lane;
        if (i < n) {
            const uint32_t d = (key[r] >> shift) & 255u;
            const uint32_t pos = s_off[d] + s_cnt[wave][d] + rank[r];
            if (pos >= (uint32_t)n) {   // only after a look-back fault: never write outside the pairs
                lb_fault(err, kFaultRadixScatter);
                continue;
            }
            ko[pos] = key[r];
            vo[pos] = val[r];
        }
    }
}

}  // namespace

hipError_t launch_radix_passes(uint32_t* ka, int* va, uint32_t* kb, int* vb, const int* v0, int n,
                               const uint32_t* bound, const RadixScratch& rs, uint32_t epoch, int* err, int inject,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    for (int p = 0; p < kRadixPasses; ++p)
        hipLaunchKernelGGL(radix_pass_kernel, dim3((unsigned)rs.tiles), dim3(kRadixThreads), 0, s, ka, va, kb, vb, v0, n, p,
                           bound, rs.hist, rs.ctr, rs.state + (size_t)p * rs.tiles * kRadixDigits, epoch, err, inject);
    return hipGetLastError();
}

}  // namespace lmsf
