// Internal device/host interfaces of liblmsf_hip.so (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/lmsf/lmsf.h"

namespace lmsf {

constexpr int kMaxOuter = 32;        // trace rows kept per solve
constexpr int kPacket = 32;          // doubles per partial packet (29 used + edge/surf counts)
constexpr int kFitMaxPerThread = 4;  // queries per thread in the fit / first-evaluation kernel (1..4)
constexpr int kFitBlockMax = 256 * kFitMaxPerThread;
#ifndef LMSF_EVAL_PER_THREAD
#define LMSF_EVAL_PER_THREAD 4
#endif
#ifndef LMSF_EVAL_PIPE
#define LMSF_EVAL_PIPE 0
#endif
constexpr int kEvalPerThread = LMSF_EVAL_PER_THREAD;   // records per thread in the LM evaluation kernel
constexpr int kEvalBlock = 256 * kEvalPerThread;
// Records per thread of the single-scan LM loop (lm_loop_kernel; A/B).  2 puts a C3 / C4 scan's evaluation on twice
// the CUs (128 blocks instead of 64 for 64k feature slots): C4 1,371 / 1,385 vs 1,372 / 1,365 scans/s, C3 1,296 /
// 1,330 vs 1,377 / 1,357 frames/s (r05, alternating) -- the evaluation is not what bounds the loop.
#ifndef LMSF_LOOP_PER_THREAD
#define LMSF_LOOP_PER_THREAD 4
#endif
constexpr int kLoopPerThread = LMSF_LOOP_PER_THREAD;
constexpr int kLoopBlock = 256 * kLoopPerThread;
// Workspace growth: when a request exceeds the capacity, allocate 1.5x (a growing or jittering
// request -- the keyframe window, a varying scan size -- then reallocates rarely: hipFree
// synchronises the device and costs ~0.5 ms on the tracking path).
inline size_t grow_cap(size_t need, size_t cap) { return need > cap + cap / 2 ? need : cap + cap / 2; }

// Buffers that grow while other streams may still read the old ones (map grids, the voxel filter's workspace)
// are stream-ordered allocations: a growth allocates the new buffers and frees the old ones on the stream that
// uses them next, which every earlier user is ordered before ("growth"), so no device
// drain and no host wait (r04 drained the whole device -- every context's streams -- per growth).
// The pool of these allocations on the current device (created once, never trims: a freed block stays cached for
// the next growth instead of going back to the driver at every synchronisation).
hipMemPool_t growth_pool();
#ifndef LMSF_GROW_POOL
#define LMSF_GROW_POOL 1   // A/B builds: 0 = the device's default pool
#endif
template <typename T>
hipError_t galloc(T** p, size_t count, hipStream_t s) {
    *p = nullptr;
    const size_t bytes = (count ? count : 1) * sizeof(T);
#if LMSF_GROW_POOL
    hipMemPool_t pool = growth_pool();
    if (!pool) return hipErrorOutOfMemory;
    return hipMallocFromPoolAsync((void**)p, bytes, pool, s);
#else
    return hipMallocAsync((void**)p, bytes, s);
#endif
}
inline void gfree(void* p, hipStream_t s) {
    if (p) (void)hipFreeAsync(p, s);
}

// Device fault word (lmsf_ctx d_error[17]): bits set by the look-back checks (radix.h) and the scatters whose
// index comes from a look-back sum; read back with the LM-loop flag at every Solve / batch wait and reported as
// LMSF_ERR_HIP ("device look-back fault").
constexpr int kFaultRadixScatter = 1;   // a radix digit pass computed a position outside [0, n)
constexpr int kFaultLookbackWait = 2;   // a look-back wait exceeded its bound
constexpr int kFaultForeignEpoch = 4;   // a look-back word newer than the running sort (memory of another allocation)
constexpr int kFaultSegment = 8;        // the voxel segment pass counted more voxels than points
constexpr int kFaultGridScatter = 16;   // a grid scatter computed a position outside [0, n)
constexpr int kFaultStreamWait = 32;    // a cross-stream flag wait exceeded its bound (k_map.hip flag_wait_kernel)
// Look-back epochs: one process-wide counter (never restarts, never 0), shared by every sort and scan.
uint32_t next_lookback_epoch();
constexpr int kRingMax = 8192;       // points per ring handled by the extraction kernel
constexpr int kSortMax = 2048;       // points per sector (ring / 6 + 5, padded to a power of two)
constexpr int kMaxRings = 128;
constexpr int kEdgePerRing = 120;    // 20 per sector x 6 sectors (FX:172)
constexpr int kQSurf = 0x40000000;  // ExtractView::qcode tag of a surf feature
constexpr int kQCodeMask = 0x1fff;  // qcode bits 0-12: ring-local feature index; 13-25: rank in the ring's search order
constexpr int kQRankShift = 13;
static_assert(kRingMax <= kQCodeMask + 1, "ring positions fit the 13-bit code fields");
constexpr int kTile = 2048;          // raw points per ring-split tile
constexpr int kCounterShards = 64;   // candidate / query counters, 16 u64 (128 B) apart
constexpr int kMemoWords = 7;        // memo words per search position: 5 neighbour indices, s6, order gap
constexpr int kMemoStride = 8;       // memo_nbr allocation per search position (the AoS layout's 32-B record)
constexpr int kCaptureIters = 10;    // outer iterations kept per captured slot (lmsf_batch_capture)
// v[3] of an unmatched record (LMSF_REC44, k_match.hip store_record; decoded by lmsf_match / lmsf_batch_records):
// a quiet NaN whose low payload bits no arithmetic on float map points produces (a float NaN widened to double has
// its 29 low bits 0), so a degenerate fit's own NaN stays a matched record
constexpr long long kRecNone = 0x7ff8dead0000beefll;

// Tuning knobs measured by A/B builds.  The shipped library reads no environment:
// ab_int returns the default unless the library was built with -DLMSF_AB (tools/build_variant.sh), which
// lets one build take an override from the environment.  Algorithm switches a caller may legitimately
// want (the query memo and its tests, HIP graphs) are context options instead (lmsf_set_option).
inline int ab_int(const char* name, int def) {
#ifdef LMSF_AB
    const char* e = getenv(name);
    return e ? atoi(e) : def;
#else
    (void)name;
    return def;
#endif
}

// Host-time probes of a diagnostics build (-DLMSF_HOST_PROFILE, tools/build_variant.sh): HPROF(id, name) adds the
// wall time from there to the end of the enclosing block to bucket id; the table is printed to stderr at exit.
// Empty in every other build.
#ifdef LMSF_HOST_PROFILE
}  // namespace lmsf
#include <chrono>
namespace lmsf {
void hprof_add(int id, const char* name, long long ns);
struct HProf {
    int id;
    const char* name;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~HProf() {
        hprof_add(id, name, std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
    }
};
#define HPROF(id, name) HProf hprof_##id{id, name}
#else
#define HPROF(id, name) do {} while (0)
#endif

// Dense cell grid over one feature map: cell = floor(coord) - origin, 1 m cells (the match
// radius: search_thresh_ = 1.0 squared metres, REG/FeatureMatch/FeatureMatchBase.hpp:29).
struct GridView {
    int ox, oy, oz;          // origin: x in slices, y and z in metres
    int nx, ny, nz;          // extent: x in slices (sx per metre), y and z in 1 m cells
    int sx;                  // x-slices per metre (power of two): a 1 m cell = sx consecutive slices
    const uint32_t* off;   // nx*ny*nz + 1 exclusive offsets into pts
    const float4* pts;     // points sorted by cell; w = original index (int bits)
    const float4* orig;    // points in the caller's order (x, y, z, intensity)
    int n;
    float lim1;            // first-pass radius^2 of the pruned one-lane search (m^2); >= 1: sparse grid, plain walk
    int sy;                // y / z cells per metre: 1 (the 1 m grid of every search), 2 (a dense map's first-pass grid)
};

// Per-registration solver state (device resident, one per batch slot).
struct SolveState {
    double x[7];       // accepted pose (qx qy qz qw tx ty tz)
    double xc[7];      // candidate pose awaiting evaluation
    double H[21];
    double g[6];
    double s[6];       // Jacobi scaling, fixed per ceres::Solve
    double cost, radius, decrease, mcc, x_norm, initial_cost;
    int iteration, need_eval, done, term;
    int evals, nmatch, edge_matches, surf_matches;
    int inner_total, evals_total, outer_run, gn_converged;
    int gn_degenerate, pad0, pad1, pad2;
    double gn_map[36];
    double trace[kMaxOuter][7];
};

struct alignas(32) RecV { double v[4]; };

struct BatchView {
    int B;                   // slots in this launch
    int feat_stride;         // features per slot (capacity)
    const float4* feat;      // [B][feat_stride]: edges then surfs
    const int* n_edge;       // [B]
    const int* n_surf;       // [B]
    float4* nnp;             // [B][feat_stride][5] neighbour points (w = map index bits, -1: none)
    int fit_per_thread;      // queries per thread of fit_eval (partials per kFitThreads*fpt queries)
    int part_q;              // queries per partial packet of the first evaluation (lm_begin): 256 * fit_per_thread,
                             // 64 after the fused search + fit (one packet per wave)
    // correspondence records, split so an LM evaluation of a surf record reads 48 B (not 64):
    float4* rec_p;           // [B][feat_stride] lidar-frame point, w = kind (int bits; 0 = none)
    RecV* rec_v;             // [B][feat_stride] surf: n, D; edge: a, b.x
    double2* rec_e;          // [B][feat_stride] edge only: b.y, b.z
    double* partials;        // [B][max_parts][kPacket]
    int max_parts;
    SolveState* st;          // [B]
    unsigned long long* n27; // [kCounterShards][16]: [0] candidates, [1] queries (may be null)
    int count27;             // also accumulate [0] (extra cell-offset loads: diagnostics only)
    double* gn_rows;         // [B][feat_stride][4] grad + residual (GN only)
    double* partials_gn;     // [B][max_parts][kPacket] (GN only)
    const int* qslot;        // [B][pos_stride] feature slot per ring position (the knn order), null: slot order
    const int* n_pos;        // [B] ring positions per slot (with qslot)
    int pos_stride;
    const int* fslot;        // [B][feat_stride] edge slots then surf slots, each in ring order (with qslot)
    const float4* featp;     // [B][feat_stride] feat in fslot order, w = slot bits (the fused path reads these
                             //   coalesced and stores its records by search position, not by slot)
    int write_nn;            // fused search + fit also writes nnp (lmsf_match diagnostics)
    // Query memo of the fused path (outer iterations > 0 of one solve), indexed by search position i
    // (fslot order, so one lane per position reads them coalesced):
    float4* prevw;           // [B][feat_stride] anchor of position i's last full search: map-frame query w0
                             //   and gap = s6 - s5 (s = distance of the k-th neighbour, the 6th capped at
                             //   the 1 m radius); w = -1 when fewer than 5 neighbours were found
    int* memo_nbr;           // [B][feat_stride][kMemoStride] (LMSF_MEMO_AOS; else [B][kMemoWords][feat_stride]) that search's 5 neighbour map indices, nearest
                             //   first, then s6 (float bits), then (batch path) the order gap: min(s6 - s5,
                             //   s(j+1) - s(j)) (float bits; -1 once a refit reordered the indices)
    float* wlim;             // [B][feat_stride] the listed positions' search radius^2 (knn_walk lim)
    int memo;                // 1: match_memo_kernel ran before match_fit_kernel in this outer iteration
    int* wl;                 // [B][feat_stride] per block of the memo pass: the positions still needing a search
                             //   (from the front of the block's segment), then those needing a refit (from its back)
    int* wcount;             // [B][feat_stride / 256 + 1] their counts per memo block: search | refit << 16
    int* n_search;           // [B] positions searched by the last match_fit_kernel (lm_begin's second range)
    int part2_base;          // packet index of match_fit_kernel's first wave packet (memo pass: [0, ceil(nq/64)))
    int fused_parts;         // lm_begin: packets laid out by the fused path (memo pass + search ranges)
    int memo_bound;          // memo misses walk min(1 m, s6 + d) instead of 1 m (LMSF_OPT_MEMO_BOUND, default 1)
    int memo_order;          // memo: consecutive-gap test first (no re-keying when every gap exceeds 2 d)
    int memo_exact;          // memo: the stored 5 are kept when the farthest of them at w is nearer than s6 - d
                             //   (LMSF_MEMO_EXACT, default 1; 0: r01's 2 d < s6 - s5)
    int memo_refit;          // memo hits whose 5 neighbours changed order are refitted without a walk
                             //   (LMSF_MEMO_REFIT, default 1)
    // LMSF_STATS_TIMING, single-scan launches: device wall-clock stamps of one neighbour-search launch,
    // written by knn_kernel's first block at entry (stamp_start) and by the first block of the fit_eval
    // that follows it at entry (stamp_end: it starts once the search has drained); null: none.  Batch
    // launches are timed by stamp kernels (enqueue_register).
    unsigned long long* stamp_start;
    unsigned long long* stamp_end;
    unsigned* p2count;       // dense maps: entries of the pass-2 work list in wl (dense_pass1_kernel)
    int* wl2;                // dense maps: the pass-2 list of the memo iterations (wl holds the memo pass's lists), B F
    float* wlim2;
    int anchor;              // dense maps: this outer iteration keeps 6 exact keys and leaves the memo anchors
                             //   (the one before the dense memo pass starts, k_match.hip dense_memo_search_kernel)
    double* pre_keys;        // [B][feat_stride][6] kept keys of the prior-grid pass (knn_kernel SPLIT 1 -> 2)
};

__device__ __forceinline__ void stamp_if(unsigned long long* at, bool first_block) {
#ifndef LMSF_NO_STAMPS
    if (at && first_block && threadIdx.x == 0) *at = (unsigned long long)wall_clock64();
#else   // A/B build without the clock read: every stamp 0 (the timing line then reads 0)
    if (at && first_block && threadIdx.x == 0) *at = 0ull;
#endif
}


// ---- launchers (each enqueues on `stream`, never synchronises)
// bbox[0..6] = the map box of the first n points (min(n, *n_dev) when n_dev) and that count; resets bbox first.
hipError_t launch_pack3(const int* a, const int* b, const int* c, int* out, hipStream_t s);
hipError_t launch_grid_clear(uint32_t* counts, uint32_t* fill, size_t n, unsigned long long* occ, hipStream_t s);
// sy: y / z cells per metre (1: the 1 m match-radius grid; 2: the dense maps' first-pass grid)
hipError_t launch_map_bbox(const float4* pts, int n, const int* n_dev, int sx, int* bbox, hipStream_t s, int sy = 1);
hipError_t launch_map_count(const float4* pts, int n, int sx, int ox, int oy, int oz, int nx, int ny, int nz,
                            int* cell, uint32_t* counts, hipStream_t s, int sy = 1);
// sorted[] w = base + original index (base > 0 for a keyframe window behind a prior map)
hipError_t launch_map_scatter(const float4* pts, int n, const int* cell, const uint32_t* off, uint32_t* fill,
                              float4* sorted, int base, int* err, hipStream_t s);
hipError_t launch_count_nonzero(const uint32_t* counts, size_t n, unsigned long long* out, hipStream_t s);
// Grid of a window whose box + count a producer left in d_bb (box 0..5, count 6), built on stream s without
// a host round trip (k_map.hip): clear, read-back of d_bb[0..10] into h_bb + ev_bb, count, scan, scatter.
// d_bb[10] != 0: the cells exceed cells_cap (nothing built; the host rebuilds).
size_t grid_scan_tiles(size_t cells_cap);
hipError_t launch_grid_build_dev(const float4* orig, int n_max, int sx, int* d_bb, uint32_t* counts, uint32_t* off,
                                 uint32_t* fill, size_t cells_cap, int* cell, float4* sorted, int base,
                                 unsigned long long* scan_state, uint32_t epoch, int* h_bb, hipEvent_t ev_bb,
                                 int* err, hipStream_t s);
hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, size_t n, void* tmp, size_t& tmp_bytes, hipStream_t s);

// edge2 / surf2: optional second grid per kind (n = 0: none), searched as if concatenated after
// the first (its points carry global indices).
// memo: keep the per-slot anchors (and, with bv.memo, reuse unchanged 5-NN sets) -- 8-lane sparse launches.
hipError_t launch_knn_split(int pass, const GridView& edge, const GridView& surf, const GridView& edge2,
                            const GridView& surf2, const BatchView& bv, hipStream_t s);
hipError_t launch_knn(const GridView& edge, const GridView& surf, const GridView& edge2, const GridView& surf2,
                      const BatchView& bv, int skip_converged, hipStream_t s, bool memo = false);
hipError_t launch_fit_eval(const GridView& edge, const GridView& surf, const BatchView& bv, int solver,
                           hipStream_t s);
// Single-scan Ceres-LM launches: the search, the fit, the records and the first evaluation in one launch
// (k_match.hip track_match_kernel; its packets are fit_eval_kernel<1>'s count, one per 256 positions).  ticket:
// [B][track_ticket_words(F)] counters, zeroed once (the kernel re-arms them).
bool track_fused_enabled();
__host__ __device__ size_t track_ticket_words(size_t feat_stride);
hipError_t launch_track_match(const GridView& edge, const GridView& surf, const GridView& edge2, const GridView& surf2,
                              const BatchView& bv, unsigned* ticket, hipStream_t s);
hipError_t launch_lm_begin(const BatchView& bv, hipStream_t s);
// One LM inner iteration: evaluation at the candidate, then the step control.
hipError_t launch_lm_eval_step(const BatchView& bv, int outer, int is_last, hipStream_t s);
// batch path: packets at the linearisation pose from one pass over the records (lm_begin then reads
// ceil(nq / kEvalBlock) packets per slot); false in A/B builds where the matching kernels accumulate them
bool lin_eval_enabled();
hipError_t launch_lin_eval(const BatchView& bv, hipStream_t s);
// lm_begin + the 4 inner iterations of one outer iteration in one launch (k_match.hip, lm_loop_kernel): for
// launches whose B x lm_loop_blocks blocks are all co-resident (kLoopMaxBlocks).  sync: [2 B] counters
// (zeroed once), err: set when a bounded wait gave up.
constexpr int kLoopMaxBlocks = 128;   // half the CUs: room for other streams' launches beside it
int lm_loop_blocks(const BatchView& bv);
// spin_limit: sleeps a block waits at a barrier before it flags err and leaves (kLoopSpinDefault; 0 in the
// fault-recovery test, LMSF_OPT_LOOP_FAULT_TEST)
constexpr unsigned kLoopSpinDefault = 1u << 24;
hipError_t launch_lm_loop(const BatchView& bv, int outer, unsigned* sync, int* err, unsigned spin_limit, hipStream_t s);
hipError_t launch_lm_step(const BatchView& bv, int outer, int is_last, hipStream_t s);
hipError_t launch_gn_solve(const BatchView& bv, int outer, hipStream_t s);
hipError_t launch_eigen_selftest(int dim, const double* a, int n, double* d, double* v, int* info, hipStream_t s);
int fit_per_thread_default();
int knn_team_for(size_t query_slots);   // lanes per query of a search launch over that many query slots
// Fused 5-NN search + fit + first evaluation (one lane per query, queries in fslot order); false:
// not applicable to this launch (caller runs launch_knn + launch_fit_eval).
bool match_fit_applies(const GridView& edge2, const GridView& surf2, const BatchView& bv, int solver);
// fine_*: a dense map's first-pass grid per kind (n = 0: none; pass 1 then runs on the 1 m grid)
hipError_t launch_match_fit(const GridView& edge, const GridView& surf, const BatchView& bv, hipStream_t s,
                            const GridView& fine_edge = GridView{}, const GridView& fine_surf = GridView{});
bool match_fit_prune(const GridView& edge, const GridView& surf);   // dense map: pruned walk, no memo
// Record capture (lmsf_batch_capture): slot b's records after an outer iteration's matching as lmsf_record
// rows in slot order, its 5 neighbour indices (nnp w bits, -1: none) and the linearisation pose (7 doubles).
// by_pos: records are stored by search position (fused path), else by slot.
hipError_t launch_capture(const BatchView& bv, int b, int by_pos, lmsf_record* rec, int32_t* nn, double* pose,
                          hipStream_t s);
hipError_t launch_state_init(const BatchView& bv, const double* poses, hipStream_t s);
// one slot (bv.B == 1) at a pose passed by value (no host-to-device copy before it)
hipError_t launch_state_init_pose(const BatchView& bv, const double x[7], hipStream_t s);
hipError_t launch_stamp(unsigned long long* out, hipStream_t s);   // wall clock after the stream's prior work
// Standalone evaluation at one pose (diagnostics): packet of slot 0 into out29 (device).
hipError_t launch_eval_at(const BatchView& bv, const double* pose_dev, double* out_dev, hipStream_t s);

// ---- feature extraction (LOAMFeatureProcessorBase::Process)
struct ExtractView {
    int B;
    int raw_stride;              // raw points per slot (capacity)
    const float4* raw;           // scans packed back to back: slot b's raw_count[b] points at raw + raw_off[b]
    const int* raw_count;        // [B]
    const int64_t* raw_off;      // [B]
    int8_t* ring_id;             // [B][raw_stride]  (-1 rejected)
    int n_tiles;                 // tiles per slot (capacity)
    int* tile_counts;            // [B][kMaxRings][n_tiles]
    int* ring_start;             // [B][kMaxRings + 1]
    float4* ring_pts;            // [B][raw_stride] ring-ordered points
    int* ring_src;               // [B][raw_stride] raw index of each ring-ordered point
    double* sort_key;            // [B][raw_stride] per sector at ring_start + sector start: curvature
    int* sort_idx;               //                 ascending (c, index), ring-local indices
    int* ring_edge_cnt;          // [B][kMaxRings]
    int* ring_surf_cnt;          // [B][kMaxRings]
    int* qcode;                  // [B][raw_stride] per ring position: ring-local edge index, kQSurf | surf index, -1; + rank << 13
    int* qslot;                  // [B][raw_stride] per ring position: its feature slot or -1 (the search order)
    int* fslot;                  // [B][feat_stride] qslot's valid entries, edge slots first (stable)
    float4* featp;               // [B][feat_stride] the features in fslot order: xyz, w = slot (int bits)
    int* n_pos;                  // [B] ring positions of the slot (ring_start[n_scans])
    float4* feat;                // [B][feat_stride] output (edges then surfs)
    int* feat_src;               // [B][feat_stride]
    int feat_stride;
    int* n_edge;                 // [B]
    int* n_surf;                 // [B]
    int* error;                  // [1] capacity flags
    // parameters
    int n_scans;
    float min_d, max_d, edge_thresh;
    int remove_bad;
    double beam_lo, beam_spacing;
    int libm_float;              // lmsf_config::libm_float
};
hipError_t launch_extract(const ExtractView& ev, hipStream_t s);

// ---- local map maintenance (tracker.cpp)
struct Affine34 { double m[12]; };   // row-major 3x4 of an Isometry3d matrix
// pcl::transformPointCloud(cloud, out, Matrix4d) per point: float(m00 x + m01 y + m02 z + m03), double math
hipError_t launch_transform(const float4* in, int n, Affine34 M, float4* out, hipStream_t s);
// ... at the pose x[7] (qx qy qz qw tx ty tz) in device memory, its matrix built as the tracker's host code builds it;
// two clouds in one launch: in[0..n0) -> out0, in[n0..n0+n1) -> out1 (a scan's edge and surf features)
hipError_t launch_transform_pose2(const float4* in, int n0, int n1, const double* x, float4* out0, float4* out1,
                                  hipStream_t s);
// flag <- v after the work enqueued on s so far; s waits until flag reaches v (wrap-safe), bounded (err |= kFaultStreamWait)
hipError_t launch_flag_signal(uint32_t* flag, uint32_t v, hipStream_t s);
hipError_t launch_flag_wait(const uint32_t* flag, uint32_t v, int* err, hipStream_t s);
// Concatenation of up to kSlotTable device arrays (kernel-argument table, start[] exclusive prefix).
constexpr int kSlotTable = 32;
struct SlotTable {
    const float4* src[kSlotTable];
    int start[kSlotTable + 1];
    int n;
};
hipError_t launch_gather_slots(const SlotTable& tab, float4* out, hipStream_t s);

// ---- 1-NN alignment fitness (k_align.hip): AlignmentScore (REG/alignEvaluate.hpp:55-87)
struct Affine34f { float m[12]; };   // row-major 3x4 of an Eigen::Matrix4f
int align_parts(int n);
// out2[0] = sum of inlier d2 (double), out2[1] = inlier count; part_* hold align_parts(n) entries
hipError_t launch_align(const GridView& g, const float4* src, int n, const Affine34f& M, double thresh,
                        double* part_sum, unsigned int* part_cnt, double* out2, hipStream_t s);

// pcl::VoxelGrid centroid downsampling on the device (k_voxel.hip); workspace grows on demand.
// run() synchronises the stream (the output count is returned to the host).
// Sort: k_sort.hip / radix.h (7 launches per filter, no host round trip).
struct VoxelFilter {
    uint32_t *keys = nullptr, *keys_b = nullptr, *scratch = nullptr;
    int *idx = nullptr, *idx_b = nullptr, *part = nullptr, *nseg = nullptr;
    uint32_t epoch = 0;   // look-back epoch of the last sort
    size_t cap = 0;
    hipStream_t last = nullptr;    // stream of the last enqueue (the workspace's release is ordered after it)
    bool exact = false;            // grow to the request exactly (LMSF_OPT_GROWTH_TEST: a growth at every increase)
    bool poisoned = false;         // an injected fault (tests) left foreign look-back words: re-zeroed next time
    static int box_blocks(int n);
    // grows on s: new buffers allocated and the old ones freed on s, after the last enqueue's stream (no drain)
    hipError_t reserve(size_t n, hipStream_t s);
    // err: the device fault word (radix.h); run() also returns hipErrorIllegalState when the sort flagged one
    hipError_t run(const float4* in, int n, float leaf, float4* out, int* n_out, int* err, hipStream_t s);
    // run() without the read-back: the voxel count stays on the device in *nseg (no host wait).  map_bb
    // (optional, device): [0..5] = the map-cell box (k_map.hip's rule, sx x-slices per m) of the INPUT
    // points -- it bounds the centroids' box -- and [6] = the voxel count, the grid stage's read-back.
    // inject: LMSF_OPT_FAULT_INJECT (launch_radix_passes)
    hipError_t enqueue(const float4* in, int n, float leaf, float4* out, int* err, hipStream_t s,
                       int* map_bb = nullptr, int sx = 0, int inject = 0);
    void release();                // waits for the last enqueue's stream
};

// PointCloud2 decode + removeNaN + rotary relative time + distance filter (k_ingest.hip).
// run() reads the message from device memory (raw, staged by the caller) and synchronises.
struct Ingest {
    uint8_t* raw = nullptr;
    size_t raw_cap = 0;
    float4 *a = nullptr, *b = nullptr;
    uint32_t *keep = nullptr, *pos = nullptr;
    int* scalars = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0, cap = 0;
    hipError_t reserve(size_t n, size_t raw_bytes);
    hipError_t run(const uint8_t* data_dev, int n, uint32_t step, int ox, int oy, int oz, int oi, float period,
                   double near_t, double far_t, float4** result, int* n_out, hipStream_t s);
    // stable compactions of device points (in != out), synchronising: removeNaN / DistanceFilter
    hipError_t finite(const float4* in, int n, float4* out, int* n_out, hipStream_t s);
    hipError_t distance(const float4* in, int n, double near_t, double far_t, float4* out, int* n_out, hipStream_t s);
    hipError_t compact_flagged(const float4* in, int n, float4* out, int* n_out, hipStream_t s);
    void release();
};

hipStream_t ctx_stream(lmsf_ctx* c);
int ctx_device(const lmsf_ctx* c);
int ctx_feature_capacity(const lmsf_ctx* c);
bool ctx_features_on_device(const lmsf_ctx* c);
lmsf_status ctx_fail(lmsf_ctx* c, lmsf_status code, const char* msg);
// a tracker's deferred-commit completion, run by the context before its map consumers
void ctx_add_settle(lmsf_ctx* c, lmsf_status (*fn)(void*), void* arg);
void ctx_remove_settle(lmsf_ctx* c, void* arg);
// fn(arg) once, inside the next lmsf_solve: after its kernels are enqueued, before its result's read-back and its
// host wait (a tracker's keyframe lookahead); ctx_solved_pose: that Solve's result on the device (x[7]);
// ctx_loop_recoveries: lmsf_kernel_stats' count (a recovered Solve re-ran after the armed call)
// undo(arg): called before a recovery re-run of that Solve (the armed work must not run beside it)
void ctx_arm_post_solve(lmsf_ctx* c, lmsf_status (*fn)(void*), lmsf_status (*undo)(void*), void* arg);
const double* ctx_solved_pose(const lmsf_ctx* c);
int64_t ctx_loop_recoveries(const lmsf_ctx* c);
uint64_t ctx_feature_seq(const lmsf_ctx* c);   // changes whenever slot 0's features do
// map of a kind = [prior | window]: the prior grid is built once (static), the window grid at every
// keyframe commit with indices offset by the prior size; n == 0 clears that part.
lmsf_status ctx_set_prior_device(lmsf_ctx* c, int kind, const float4* d_pts, size_t n);
// the prior-grid pass of the next Solve's outer iteration 0 at pose x, beside a window rebuild (best effort)
lmsf_status ctx_presearch(lmsf_ctx* c, const double x[7]);
lmsf_status ctx_set_window_device(lmsf_ctx* c, int kind, const float4* d_pts, size_t n);
// host wait of the single-scan paths (spins on hipStreamQuery unless LMSF_SPIN_SYNC=0)
hipError_t stream_wait(hipStream_t s);
// the same in two stages on stream s, so several windows share one host wait: stage (no wait; n_dev, on the
// device, bounds the count n_max when the producer's size is not known on the host yet), then -- once s has
// drained -- finish (n_out = the window's point count)
lmsf_status ctx_window_stage(lmsf_ctx* c, int kind, const float4* d_pts, size_t n_max, const int* n_dev, hipStream_t s);
lmsf_status ctx_window_finish(lmsf_ctx* c, int kind, size_t n_max, hipStream_t s, size_t* n_out);
// The window grid's source buffer (>= n_max points) and its box + count words ([0..5] map-cell box, [6] count),
// for a producer that fills both on the stage stream (the tracker's voxel filter); then
// ctx_window_stage(c, kind, nullptr, n_max, nullptr, s) only reads them back.
lmsf_status ctx_window_target(lmsf_ctx* c, int kind, size_t n_max, float4** orig, int** bb, hipStream_t s);
// The window grid's point buffers sized for n points ahead of the first commit (tracker creation).
lmsf_status ctx_window_reserve(lmsf_ctx* c, int kind, size_t n, hipStream_t s);
// ... or, instead of that read-back, the whole grid build on s (no host wait; ctx_window_finish then only
// takes the box read-back and sets the view).
lmsf_status ctx_window_build(lmsf_ctx* c, int kind, size_t n_max, hipStream_t s);
// The window's points in window order (the grid's unsorted source) after a finished commit.
const float4* ctx_window_points(const lmsf_ctx* c, int kind);
int grid_slices();
bool rec44_layout();                    // records with 12-B points, kind by position (k_match.hip LMSF_REC44)
int* ctx_fault_word(lmsf_ctx* c);       // the context's device fault word (d_error[17])
uint64_t ctx_fault_seq(const lmsf_ctx* c);   // device faults reported so far (LMSF_ERR_HIP "device look-back fault")
int ctx_option(const lmsf_ctx* c, int option);
lmsf_status ctx_slot0_features(lmsf_ctx* c, const float4** d_feat, int64_t* ne, int64_t* ns);

}  // namespace lmsf
