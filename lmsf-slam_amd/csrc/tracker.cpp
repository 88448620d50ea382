// Scan-to-local-map tracker on the MI355X registration context.
//
// Restates LidarTrackerLocalMap (INC/LidarTracker/LidarTrackerLocalMap.hpp:42-263, INC =
// src/MultiSensorFusionEstimator3D/include): first scan seeds the local map (:112-122), constant
// velocity prediction `prev * motion_increment` when deltaT is exactly identity (:125-129),
// RegistrationLocalMap (:168-177), motion increment (:133-135), keyframe gate needUpdataLocalMap
// (:239-262: dt > 10 s -> TIME, |dp| > 0.3 m or 2 acos(q.w / |q|) > 0.1 rad -> MOTION; no abs, as :254), and
// updateLocalMap (:205-232: transformPointCloud, add frame, SetInputSource(local map)).
// The local-map class itself is missing from the reference snapshot (factory/Map/LocalMap_factory.hpp);
// "sliding_Localmap" is defined here as a device-resident window of the last W keyframes
// (W = 10, the config's sliding_window.size), VoxelGrid-downsampled per kind (0.2 / 0.4 m).
// Isometry arithmetic follows Eigen's Isometry3d (linear * linear, linear * t + t; inverse = R^T,
// -R^T t) and its quaternion <-> matrix conversions (the Ceres path converts at Solve, ceres_...:103, :128).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "lmsf_internal.h"

using namespace lmsf;

namespace {

struct Iso {
    double R[9];
    double t[3];
};

Iso iso_identity() {
    Iso I;
    for (int i = 0; i < 9; ++i) I.R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    I.t[0] = I.t[1] = I.t[2] = 0.0;
    return I;
}

Iso iso_mul(const Iso& A, const Iso& B) {
    Iso C;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) C.R[3 * i + j] = A.R[3 * i] * B.R[j] + A.R[3 * i + 1] * B.R[3 + j] + A.R[3 * i + 2] * B.R[6 + j];
        C.t[i] = A.R[3 * i] * B.t[0] + A.R[3 * i + 1] * B.t[1] + A.R[3 * i + 2] * B.t[2] + A.t[i];
    }
    return C;
}

Iso iso_inverse(const Iso& A) {
    Iso B;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) B.R[3 * i + j] = A.R[3 * j + i];
    for (int i = 0; i < 3; ++i)
        B.t[i] = (-B.R[3 * i]) * A.t[0] + (-B.R[3 * i + 1]) * A.t[1] + (-B.R[3 * i + 2]) * A.t[2];
    return B;
}

Iso iso_from16(const double* m) {
    Iso T;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T.R[3 * i + j] = m[4 * i + j];
        T.t[i] = m[4 * i + 3];
    }
    return T;
}

void iso_to16(const Iso& T, double* m) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) m[4 * i + j] = T.R[3 * i + j];
        m[4 * i + 3] = T.t[i];
    }
    m[12] = m[13] = m[14] = 0.0;
    m[15] = 1.0;
}

bool is_identity16(const double* m) {   // deltaT.matrix() == Identity().matrix() (exact)
    for (int i = 0; i < 16; ++i)
        if (m[i] != ((i % 5 == 0) ? 1.0 : 0.0)) return false;
    return true;
}

// Eigen::Quaterniond(Matrix3d) (quaternionbase_assign_impl, Shepperd) -> (x, y, z, w)
void quat_from_R(const double* m, double* q) {
    const double tr = m[0] + m[4] + m[8];
    if (tr > 0) {
        double t = std::sqrt(tr + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t;
        q[1] = (m[2] - m[6]) * t;
        q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        double t = std::sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        q[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        q[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    }
}

// Eigen QuaternionBase::toRotationMatrix
void R_from_quat(const double* q, double* R) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// One feature kind's local map: [prior | keyframe W-ring oldest -> newest].  The context keeps two
// neighbour grids per kind: the prior's (built once) and the downsampled window's (rebuilt at each
// commit, indices offset by the prior size), searched together as one map.
struct Window {
    std::vector<float4*> slots;
    std::vector<int> sizes;
    int head = 0, count = 0;
    float4* prior = nullptr;
    size_t prior_n = 0;
    float4* wcat = nullptr;        // keyframes concatenated, input of the voxel filter (leaf > 0)
    float4* concat = nullptr;      // keyframes concatenated, the window itself (leaf <= 0); a filtered window
                                   // is written straight into its grid's source (ctx_window_target)
    size_t concat_cap = 0;
    size_t window_n = 0;
    size_t total = 0;              // prior_n + window_n = GetLocalMap size
    double leaf = 0.0;
    bool dirty = false;
};

}  // namespace

struct lmsf_tracker {
    lmsf_ctx* ctx = nullptr;
    lmsf_tracker_config cfg{};
    bool init = false;
    Iso origin, curr, prev, motion, last_kf;
    double last_kf_time = 0.0;
    Window win[3];
    VoxelFilter voxel[3];       // per kind: the two windows are filtered concurrently
    hipStream_t aux[2] = {nullptr, nullptr};   // the windows' commits (surf, edge), beside the context stream
    hipEvent_t ev_fork = nullptr, ev_join[3] = {nullptr, nullptr, nullptr};
    // LMSF_FLAG_SYNC (A/B): the fork / join orderings through device flags (k_map.hip flag_wait_kernel) instead of
    // event waits, whose cross-queue wake-up measured 20-35 us per hop on the r06 C4 trace.  flags: [0] fork,
    // [kind] join; the values last signalled.
    uint32_t* flags = nullptr;
    uint32_t fork_val = 0, join_val[3] = {0, 0, 0};
    bool fork_flags = false, join_flags[3] = {false, false, false};   // the mode each mark used (its wait uses the same)
    bool counted = false;         // in g_trackers
    bool fin_defer[3] = {false, false, false};   // a worker left this kind's box read-back to commit_finish
    hipStream_t ks[3] = {nullptr, nullptr, nullptr};   // staged commit: stream per kind (null: unchanged)
    size_t nmax[3] = {0, 0, 0};
    bool pending = false;                               // staged, not yet finished
    float4* stage = nullptr;   // host/device keyframe input staged before the transform
    int cap = 0;               // points per keyframe slot
    // Commit worker (lmsf_tracker_commit_map): enqueues the window rebuild on the aux streams from a host
    // thread of its own, so the ~50 launches of a rebuild (~0.6 ms of host API time per C4 step, r03) overlap
    // the caller's next calls instead of preceding them.  `staging`: a job posted and not yet joined.
    // Two workers, one per window kind / aux stream, so the surf and edge rebuilds are enqueued side by side.
    std::thread worker[2];
    std::mutex mu;
    std::condition_variable cv;
    int job[2] = {0, 0};          // kind to stage on aux[i] (0: none)
    bool quit = false, staging = false;
    std::atomic<unsigned> posted{0};   // jobs posted (spinning workers watch it before they sleep on cv)
    lmsf_status job_rc[2] = {LMSF_OK, LMSF_OK};
    size_t fin_n[3] = {0, 0, 0};  // per kind: the window size a worker's grid finish found
    uint64_t fault_seen = 0;      // ctx_fault_seq when the maps were last (re)built
    // Keyframe lookahead (cfg.keyframe_lookahead, r06): when the motion-model prediction already passes the keyframe
    // gate, the Solve's own features are transformed at its result on the device and the window rebuild is posted
    // while the Solve runs (ctx_arm_post_solve), so the rebuild no longer waits for the pose read-back, the caller's
    // decision and the hand-off to the workers.  The caller's keyframe of exactly that pose and those features adopts
    // it; anything else rolls it back (the window state restored, the evicted frame's buffer kept aside, the window
    // grid rebuilt).  Results are the same either way.
    int look = 0;                 // kLookNone / kLookPosted / kLookAdopted
    double look_pose[16];
    bool look_pose_known = false;
    uint64_t look_feat = 0;       // ctx_feature_seq of the features it transformed
    int64_t look_recoveries = 0;  // ctx_loop_recoveries before the Solve (a recovered Solve re-ran after the transform)
    float4* spare[3] = {nullptr, nullptr, nullptr};   // per kind: a slot buffer outside the ring
    struct Undo { bool pushed; int slot, head, count, size; bool dirty; } undo[3] = {};
};

namespace {

lmsf_status fail(lmsf_tracker* t, lmsf_status code, const char* msg) { return ctx_fail(t->ctx, code, msg); }

// Trackers per device.  The flag waits and the keyframe lookahead are used while a tracker is the only one on its
// device (r06 A/B: C4, one tracker per GPU, 1,579 / 1,578 / 1,541 scans/s with both vs 1,475 / 1,477 / 1,433 with
// neither; C3's two trackers on one GPU 1,230 / 1,359 / 1,394 vs 1,346 / 1,369 / 1,374 frames/s): a spinning wait on a
// hardware queue another tracker's streams share holds that tracker's work behind it (4 queues per process).
std::atomic<int> g_trackers[64];
bool sole_tracker(const lmsf_tracker* t) {
    const int d = ctx_device(t->ctx);
    return d < 0 || d >= 64 || g_trackers[d].load(std::memory_order_relaxed) == 1;
}

#ifndef LMSF_FLAG_SYNC
#define LMSF_FLAG_SYNC 1
#endif
// Only with the keyframe lookahead (flags alone measured neutral), so keyframe_lookahead = 0 also restores plain event
// ordering -- e.g. under a tool that serialises kernel dispatches, where a spinning wait could hold its producer back.
bool flag_sync(const lmsf_tracker* t) {
    static const bool on = ab_int("LMSF_FLAG_SYNC", LMSF_FLAG_SYNC) != 0;
    return on && t->cfg.keyframe_lookahead && sole_tracker(t);
}

// The fork point: everything enqueued on the context stream so far (the keyframe transforms) before the rebuilds.
hipError_t fork_mark(lmsf_tracker* t) {
    t->fork_flags = flag_sync(t);
    hipError_t e = hipEventRecord(t->ev_fork, ctx_stream(t->ctx));
    if (e == hipSuccess && t->fork_flags) e = launch_flag_signal(t->flags, ++t->fork_val, ctx_stream(t->ctx));
    return e;
}

hipError_t fork_wait(lmsf_tracker* t, hipStream_t ks) {
    return t->fork_flags ? launch_flag_wait(t->flags, t->fork_val, ctx_fault_word(t->ctx), ks)
                         : hipStreamWaitEvent(ks, t->ev_fork, 0);
}

// The join of one kind's rebuild on ks into the context stream: marked on ks, waited for on the context stream.
hipError_t join_mark(lmsf_tracker* t, int kind, hipStream_t ks) {
    t->join_flags[kind] = t->fork_flags;
    hipError_t e = hipEventRecord(t->ev_join[kind], ks);
    if (e == hipSuccess && t->join_flags[kind]) e = launch_flag_signal(t->flags + kind, ++t->join_val[kind], ks);
    return e;
}

hipError_t join_wait(lmsf_tracker* t, int kind) {
    hipStream_t s = ctx_stream(t->ctx);
    return t->join_flags[kind] ? launch_flag_wait(t->flags + kind, t->join_val[kind], ctx_fault_word(t->ctx), s)
                               : hipStreamWaitEvent(s, t->ev_join[kind], 0);
}

#define TCHK(t, expr)                                               \
    do {                                                            \
        hipError_t e_ = (expr);                                     \
        if (e_ != hipSuccess) return fail((t), LMSF_ERR_HIP, #expr); \
    } while (0)

Affine34 affine(const Iso& T) {
    Affine34 M;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) M.m[4 * i + j] = T.R[3 * i + j];
        M.m[4 * i + 3] = T.t[i];
    }
    return M;
}

// AddFrameForMotion / AddFrameForTime of one kind: pcl::transformPointCloud(cloud, T) into the
// next window slot (evicting the oldest when full).  src is device memory.
lmsf_status push_frame(lmsf_tracker* t, int kind, const float4* src, int64_t n, const Iso& T) {
    if (n == 0) return LMSF_OK;                                   // :213
    if (n > t->cap) return fail(t, LMSF_ERR_CAPACITY, "keyframe larger than the tracker slot capacity");
    Window& w = t->win[kind];
    const int W = (int)w.slots.size();
    int slot;
    if (w.count < W) {
        slot = (w.head + w.count) % W;
        ++w.count;
    } else {                                                      // window full: evict the oldest
        slot = w.head;
        w.head = (w.head + 1) % W;
    }
    TCHK(t, launch_transform(src, (int)n, affine(T), w.slots[slot], ctx_stream(t->ctx)));
    w.sizes[slot] = (int)n;
    w.dirty = true;
    return LMSF_OK;
}

// SetInputSource(GetLocalMap()) (:229) for every kind whose window changed, in two halves.
// commit_stage (no host wait): each changed kind on a stream of its own (surf on aux[0], edge on aux[1],
// both after the keyframe transforms queued on the context stream) gathers its keyframes, voxel-filters
// them and reads the grid's box + count back.  commit_finish: one wait on those streams, the grids sized
// and filled on them, and the context stream joins them before its next search.  The context stream
// stays free in between, so the next scan's extraction runs beside the map rebuild when the caller
// defers the finish (lmsf_tracker_commit_map; settle() completes it at the next tracker call).
// One kind's half of commit_stage on stream ks (after ev_fork).
lmsf_status commit_stage_kind(lmsf_tracker* t, int kind, hipStream_t ks) {
    Window& w = t->win[kind];
    TCHK(t, fork_wait(t, ks));
    const int W = (int)w.slots.size();
    float4* dst = w.leaf > 0 ? w.wcat : w.concat;
    size_t nw = 0;
    for (int i0 = 0; i0 < w.count; i0 += kSlotTable) {         // keyframes in window order
        SlotTable tab{};
        tab.n = std::min(kSlotTable, w.count - i0);
        for (int i = 0; i < tab.n; ++i) {
            const int j = (w.head + i0 + i) % W;
            tab.src[i] = w.slots[j];
            tab.start[i + 1] = tab.start[i] + w.sizes[j];
        }
        TCHK(t, launch_gather_slots(tab, dst + nw, ks));
        nw += (size_t)tab.start[tab.n];
    }
    t->nmax[kind] = nw;
    if (w.leaf > 0 && nw) {
        // VoxelGrid of the window straight into the grid's source, with the grid's box and the voxel count
        // (they stay on the device; the stage only reads them back)
        float4* orig;
        int* bb;
        lmsf_status rc = ctx_window_target(t->ctx, kind, nw, &orig, &bb, ks);
        if (rc) return rc;
        VoxelFilter& vf = t->voxel[kind];
        vf.exact = ctx_option(t->ctx, LMSF_OPT_GROWTH_TEST) != 0;
        TCHK(t, vf.enqueue(w.wcat, (int)nw, (float)w.leaf, orig, ctx_fault_word(t->ctx), ks, bb, grid_slices(),
                           ctx_option(t->ctx, LMSF_OPT_FAULT_INJECT)));
        return ctx_window_build(t->ctx, kind, nw, ks);   // the grid too, without a host round trip
    }
    // only the window's grid is rebuilt; the prior's grid was built once (set_prior_map)
    return ctx_window_stage(t->ctx, kind, w.concat, nw, nullptr, ks);
}

// The aux stream of each changed kind (surf first: the larger window and its sort); returns the count.
int assign_streams(lmsf_tracker* t) {
    int k = 0;
    for (int kind : {LMSF_SURF, LMSF_EDGE}) {
        t->ks[kind] = nullptr;
        t->nmax[kind] = 0;
        if (t->win[kind].dirty) t->ks[kind] = t->aux[k++];
    }
    return k;
}

lmsf_status commit_stage(lmsf_tracker* t) {
    TCHK(t, fork_mark(t));   // the keyframe transforms queued on the context
    assign_streams(t);
    for (int kind : {LMSF_SURF, LMSF_EDGE}) {
        if (!t->ks[kind]) continue;
        lmsf_status rc = commit_stage_kind(t, kind, t->ks[kind]);
        if (rc) return rc;
    }
    t->pending = true;
    return LMSF_OK;
}

// Wait until the workers have enqueued the posted rebuild (no GPU wait); their status.
lmsf_status join_worker(lmsf_tracker* t) {
    if (!t->staging) return LMSF_OK;
    HPROF(8, "join_worker wait");
    std::unique_lock<std::mutex> lk(t->mu);
    t->cv.wait(lk, [t] { return !t->job[0] && !t->job[1]; });
    t->staging = false;
    return t->job_rc[0] ? t->job_rc[0] : t->job_rc[1];
}

// One kind's half of commit_finish on its stage stream: wait for the stage's read-back, enqueue the grid
// build, mark its end for the context stream.
lmsf_status finish_kind(lmsf_tracker* t, int kind, hipStream_t ks) {
    // a device-built grid (filtered windows) is built whole on ks: only its box read-back is left, which the caller's
    // thread takes after the join (commit_finish: the host wait -- then usually over -- stays off the workers, whose
    // long waits behind a lookahead rebuild held the caller's enqueues: r06 host probes, 150 us per prefetch call);
    // a staged window reads its box back here first and builds its grid on ks
    t->fin_defer[kind] = t->win[kind].leaf > 0;
    if (!t->fin_defer[kind]) {
        TCHK(t, stream_wait(ks));
        lmsf_status rc = ctx_window_finish(t->ctx, kind, t->nmax[kind], ks, &t->fin_n[kind]);
        if (rc) return rc;
    }
    TCHK(t, join_mark(t, kind, ks));
    return LMSF_OK;
}

// Worker i: stage, then finish, of the kind posted for aux[i].  Both halves run here, so the two kinds' host
// waits and grid builds proceed side by side (r03 trace: one thread finishing both put the edge grid's
// ~5 launches behind the surf grid's) and the caller's thread only joins.
// Before sleeping on the condition variable a worker polls for LMSF_WORKER_SPIN_US (A/B knob; commits come once per
// scan, ~0.7 ms apart on C4): a condition-variable wake-up put ~25 us between commit_map and the rebuild's first
// kernel (r06 C4 trace).
#ifndef LMSF_WORKER_SPIN_US
#define LMSF_WORKER_SPIN_US 0
#endif
void worker_main(lmsf_tracker* t, int i, int device) {
    hipSetDevice(device);
    static const int spin_us = ab_int("LMSF_WORKER_SPIN_US", LMSF_WORKER_SPIN_US);
    std::unique_lock<std::mutex> lk(t->mu);
    for (;;) {
        if (spin_us > 0 && t->job[i] == 0 && !t->quit) {
            const unsigned seen = t->posted.load(std::memory_order_acquire);
            lk.unlock();
            const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
            while (t->posted.load(std::memory_order_acquire) == seen && std::chrono::steady_clock::now() < until) {
            }
            lk.lock();
        }
        t->cv.wait(lk, [t, i] { return t->job[i] != 0 || t->quit; });
        if (t->quit) return;
        const int kind = t->job[i];
        lk.unlock();
        lmsf_status rc;
        {
            HPROF(9, "worker stage");
            rc = commit_stage_kind(t, kind, t->aux[i]);
        }
        if (!rc) {
            HPROF(10, "worker finish");
            rc = finish_kind(t, kind, t->aux[i]);
        }
        lk.lock();
        t->job_rc[i] = rc;
        t->job[i] = 0;
        t->cv.notify_all();
    }
}

lmsf_status commit_finish(lmsf_tracker* t) {
    hipStream_t s = ctx_stream(t->ctx);
    if (t->staging) {   // the workers staged and finished: apply the sizes, join their streams
        lmsf_status rj = join_worker(t);
        t->pending = false;
        if (rj) return rj;
        for (int kind : {LMSF_SURF, LMSF_EDGE})
            if (t->ks[kind]) TCHK(t, join_wait(t, kind));
        for (int kind : {LMSF_SURF, LMSF_EDGE}) {
            if (!t->ks[kind]) continue;
            if (t->fin_defer[kind]) {   // its box read-back (an over-capacity grid is rebuilt on the context stream,
                                        // after the join)
                t->fin_defer[kind] = false;
                lmsf_status rc = ctx_window_finish(t->ctx, kind, t->nmax[kind], s, &t->fin_n[kind]);
                if (rc) return rc;
            }
            Window& w = t->win[kind];
            w.window_n = t->fin_n[kind];
            w.total = w.prior_n + w.window_n;
            w.dirty = false;
        }
        return LMSF_OK;
    }
    if (!t->pending) return LMSF_OK;
    t->pending = false;
    for (int kind : {LMSF_SURF, LMSF_EDGE})
        if (t->ks[kind] && !(t->win[kind].leaf > 0)) TCHK(t, stream_wait(t->ks[kind]));   // see finish_kind
    for (int kind : {LMSF_SURF, LMSF_EDGE}) {
        Window& w = t->win[kind];
        if (!t->ks[kind]) continue;
        size_t n = 0;
        lmsf_status rc = ctx_window_finish(t->ctx, kind, t->nmax[kind], t->ks[kind], &n);
        if (rc) return rc;
        w.window_n = n;
        w.total = w.prior_n + n;
        w.dirty = false;
        TCHK(t, join_mark(t, kind, t->ks[kind]));
        TCHK(t, join_wait(t, kind));
    }
    return LMSF_OK;
}

lmsf_status commit(lmsf_tracker* t) {
    lmsf_status rc = commit_stage(t);
    if (rc) return rc;
    return commit_finish(t);
}

// The prior-grid pass of the next Solve at the motion-model prediction (:125-129; deltaT given: that delta) -- the pose
// register_pose will pass -- enqueued on the context stream before a pending keyframe rebuild is joined into it, so
// it runs beside the rebuild (api.cpp ctx_presearch).
lmsf_status presearch_prediction(lmsf_tracker* t, const double* deltaT) {
    const Iso pred = (deltaT == nullptr || is_identity16(deltaT)) ? iso_mul(t->prev, t->motion)
                                                                  : iso_mul(t->prev, iso_from16(deltaT));
    double x[7];
    quat_from_R(pred.R, x);
    x[4] = pred.t[0]; x[5] = pred.t[1]; x[6] = pred.t[2];
    return ctx_presearch(t->ctx, x);
}

enum { kLookNone = 0, kLookPosted = 1, kLookAdopted = 2 };

// The posted half of lmsf_tracker_commit_map: each changed kind's rebuild enqueued on its aux stream by its worker
// (A/B builds: on the caller's thread), after everything enqueued on the context stream so far (ev_fork).
lmsf_status post_commit(lmsf_tracker* t) {
    TCHK(t, fork_mark(t));
    if (assign_streams(t) == 0) return LMSF_OK;
    // A/B builds (diagnostics): the rebuild enqueued on the caller's thread instead of the two workers
    static const bool inline_commit = ab_int("LMSF_COMMIT_INLINE", 0) != 0;
    if (inline_commit) {
        for (int i = 0; i < 2; ++i) {
            const int kind = t->ks[LMSF_SURF] == t->aux[i] ? LMSF_SURF : t->ks[LMSF_EDGE] == t->aux[i] ? LMSF_EDGE : 0;
            lmsf_status r = kind ? commit_stage_kind(t, kind, t->aux[i]) : LMSF_OK;
            if (!r && kind) r = finish_kind(t, kind, t->aux[i]);
            t->job_rc[i] = r;
            t->job[i] = 0;
        }
        t->staging = true;
        t->pending = true;
        return LMSF_OK;
    }
    if (!t->worker[0].joinable())
        for (int i = 0; i < 2; ++i) t->worker[i] = std::thread(worker_main, t, i, ctx_device(t->ctx));
    {
        std::lock_guard<std::mutex> lk(t->mu);
        for (int kind : {LMSF_SURF, LMSF_EDGE})
            if (t->ks[kind]) t->job[t->ks[kind] == t->aux[0] ? 0 : 1] = kind;
        t->staging = true;
        t->posted.fetch_add(1u, std::memory_order_release);
    }
    t->cv.notify_all();
    t->pending = true;
    return LMSF_OK;
}

// needUpdataLocalMap (:239-262) of pose T at timestamp: LMSF_UPDATE_TIME / _MOTION / _NONE.
int gate_type(const lmsf_tracker* t, const Iso& T, double timestamp) {
    if (timestamp - t->last_kf_time > t->cfg.time_interval) return LMSF_UPDATE_TIME;
    const Iso d = iso_mul(iso_inverse(t->last_kf), T);
    const double dt = std::sqrt(d.t[0] * d.t[0] + d.t[1] * d.t[1] + d.t[2] * d.t[2]);
    double q[4];
    quat_from_R(d.R, q);
    const double qn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const double angle = std::acos(q[3] / qn) * 2;
    return (dt > t->cfg.threshold_trans || angle > t->cfg.threshold_rot) ? LMSF_UPDATE_MOTION : LMSF_UPDATE_NONE;
}

// The lookahead (ctx_arm_post_solve, inside lmsf_solve before its wait): the context's slot-0 features of each kind
// transformed at the Solve's device-resident result into the spare buffer, which takes the slot push_frame would
// fill, and the rebuild posted.
lmsf_status lookahead_post(void* p) {
    lmsf_tracker* t = static_cast<lmsf_tracker*>(p);
    const float4* feat;
    int64_t ne, ns;
    lmsf_status rc = ctx_slot0_features(t->ctx, &feat, &ne, &ns);
    if (rc) return rc;
    const int64_t cnt[3] = {0, ne, ns};
    if (ne > t->cap || ns > t->cap) return fail(t, LMSF_ERR_CAPACITY, "keyframe larger than the tracker slot capacity");
    float4* dst[3] = {nullptr, nullptr, nullptr};
    for (int kind = LMSF_EDGE; kind <= LMSF_SURF; ++kind) {
        Window& w = t->win[kind];
        auto& u = t->undo[kind];
        u.pushed = false;
        if (cnt[kind] == 0) continue;
        const int W = (int)w.slots.size();
        u = {true, w.count < W ? (w.head + w.count) % W : w.head, w.head, w.count, 0, w.dirty};
        u.size = w.sizes[u.slot];
        if (w.count < W) ++w.count;
        else w.head = (w.head + 1) % W;
        std::swap(w.slots[u.slot], t->spare[kind]);   // the evicted frame stays in the spare buffer until adopted
        dst[kind] = w.slots[u.slot];
        w.sizes[u.slot] = (int)cnt[kind];
        w.dirty = true;
    }
    t->look_feat = ctx_feature_seq(t->ctx);
    t->look_pose_known = false;
    t->look = kLookPosted;   // from here a failure is undone by the caller (solve_current's look_rollback)
    // both kinds in one launch (edges then surfs, as slot 0 holds them); a kind without features writes nothing
    TCHK(t, launch_transform_pose2(feat, (int)ne, (int)ns, ctx_solved_pose(t->ctx), dst[LMSF_EDGE], dst[LMSF_SURF],
                                   ctx_stream(t->ctx)));
    return post_commit(t);
}

// A posted lookahead the caller did not adopt: its rebuild joined, the windows restored, and rebuilt.
lmsf_status look_rollback(lmsf_tracker* t) {
    t->look = kLookNone;
    lmsf_status rc = commit_finish(t);
    if (rc) return rc;
    bool any = false;
    for (int kind = LMSF_EDGE; kind <= LMSF_SURF; ++kind) {
        auto& u = t->undo[kind];
        if (!u.pushed) continue;
        u.pushed = false;
        Window& w = t->win[kind];
        std::swap(w.slots[u.slot], t->spare[kind]);
        w.head = u.head;
        w.count = u.count;
        w.sizes[u.slot] = u.size;
        w.dirty = true;   // the window grid holds the lookahead frame
        any = true;
    }
    return any ? post_commit(t) : LMSF_OK;
}

// A deferred commit completed before anything that reads or rewrites the windows or the map.  A device fault
// reported since the maps were built (a look-back / scatter check in a voxel filter or grid build: a faulted filter
// leaves its window empty, k_voxel.hip) means a grid the context searches may be empty or partial, and that report
// failed only one call: the priors and every window are rebuilt here from the tracker's own copies (the keyframe
// slots are written by the transforms, never by a filter) before anything reads the map again.
lmsf_status settle(lmsf_tracker* t) {
    HPROF(12, "tracker settle");
    if (t->look == kLookPosted) {   // not adopted by the time anything else touches the windows or the map
        lmsf_status rl = look_rollback(t);
        if (rl) return rl;
    }
    t->look = kLookNone;
    lmsf_status rc = commit_finish(t);
    if (rc) return rc;
    const uint64_t seq = ctx_fault_seq(t->ctx);
    if (seq == t->fault_seen) return LMSF_OK;
    t->fault_seen = seq;
    bool any = false;
    for (int kind = LMSF_EDGE; kind <= LMSF_SURF; ++kind) {
        Window& w = t->win[kind];
        if (w.prior_n) {
            rc = ctx_set_prior_device(t->ctx, kind, w.prior, w.prior_n);
            if (rc) return rc;
        }
        if (w.count > 0 || w.prior_n) {
            w.dirty = true;
            any = true;
        }
    }
    return any ? commit(t) : LMSF_OK;
}

// updateLocalMap (:205-232) with the current scan's features (context slot 0).
lmsf_status update_local_map(lmsf_tracker* t, const Iso& T) {
    const float4* feat;
    int64_t ne, ns;
    lmsf_status rc = ctx_slot0_features(t->ctx, &feat, &ne, &ns);
    if (rc) return rc;
    rc = push_frame(t, LMSF_EDGE, feat, ne, T);
    if (rc) return rc;
    rc = push_frame(t, LMSF_SURF, feat + ne, ns, T);
    if (rc) return rc;
    return commit(t);
}

lmsf_status set_features(lmsf_tracker* t, const float* edge, size_t ne, const float* surf, size_t ns) {
    lmsf_status rc = lmsf_set_scan(t->ctx, LMSF_EDGE, edge, ne);
    if (rc) return rc;
    return lmsf_set_scan(t->ctx, LMSF_SURF, surf, ns);
}

// RegistrationLocalMap (:168-177) -> Solve: T -> (q, t) -> T.linear() = q.toRotationMatrix()
lmsf_status register_pose(lmsf_tracker* t, Iso& T, lmsf_solve_stats* st) {
    double x[7];
    quat_from_R(T.R, x);
    x[4] = T.t[0]; x[5] = T.t[1]; x[6] = T.t[2];
    lmsf_status rc = lmsf_solve(t->ctx, x, st);
    if (rc) return rc;
    R_from_quat(x, T.R);
    T.t[0] = x[4]; T.t[1] = x[5]; T.t[2] = x[6];
    return LMSF_OK;
}

}  // namespace

extern "C" {

lmsf_status lmsf_tracker_config_init(lmsf_tracker_config* cfg) {
    if (!cfg) return LMSF_ERR_ARG;
    cfg->window_frames = 10;
    cfg->threshold_trans = 0.3;
    cfg->threshold_rot = 0.1;
    cfg->time_interval = 10.0;
    cfg->manual_map_update = 0;
    cfg->leaf_edge = 0.2;
    cfg->leaf_surf = 0.4;
    cfg->keyframe_lookahead = 1;
    return LMSF_OK;
}

void lmsf_tracker_destroy(lmsf_tracker* t) {
    if (!t) return;
    if (t->counted) g_trackers[ctx_device(t->ctx)].fetch_sub(1);
    hipSetDevice(ctx_device(t->ctx));
    // A deferred commit is completed first (a posted one joined from the workers): its staging already rewrote
    // the context's window grids (points, box read-back), so the context must not keep searching the old sizes
    // and offsets.  If it cannot be completed, the windows are dropped (the context keeps its prior maps).
    if (commit_finish(t) != LMSF_OK)
        for (int kind = LMSF_EDGE; kind <= LMSF_SURF; ++kind) ctx_set_window_device(t->ctx, kind, nullptr, 0);
    if (t->worker[0].joinable()) {
        {
            std::lock_guard<std::mutex> lk(t->mu);
            t->quit = true;
        }
        t->cv.notify_all();
        for (auto& w : t->worker) w.join();
    }
    ctx_remove_settle(t->ctx, t);
    hipStreamSynchronize(ctx_stream(t->ctx));
    for (auto& w : t->win) {
        for (float4* p : w.slots) hipFree(p);
        hipFree(w.concat);
        hipFree(w.wcat);
        hipFree(w.prior);
    }
    for (auto& v : t->voxel) v.release();
    for (hipStream_t a : t->aux)
        if (a) {
            hipStreamSynchronize(a);
            hipStreamDestroy(a);
        }
    if (t->ev_fork) hipEventDestroy(t->ev_fork);
    hipFree(t->flags);
    for (hipEvent_t e : t->ev_join)
        if (e) hipEventDestroy(e);
    hipFree(t->stage);
    for (float4* p : t->spare) hipFree(p);
    delete t;
}

lmsf_status lmsf_tracker_create(lmsf_ctx* ctx, const lmsf_tracker_config* cfg, lmsf_tracker** out) {
    if (!ctx || !cfg || !out || cfg->window_frames < 1 || cfg->leaf_edge < 0 || cfg->leaf_surf < 0) return LMSF_ERR_ARG;
    *out = nullptr;
    lmsf_tracker* t = new lmsf_tracker();
    t->ctx = ctx;
    t->cfg = *cfg;
    t->cfg.keyframe_lookahead = ab_int("LMSF_LOOKAHEAD", cfg->keyframe_lookahead);   // A/B builds: an override
    t->cap = ctx_feature_capacity(ctx);
    if (hipSetDevice(ctx_device(ctx)) != hipSuccess) { delete t; return LMSF_ERR_HIP; }
    // LMSF_AUX_PRIORITY (A/B): the window rebuild's streams at the device's highest priority, so the rebuild -- the
    // critical path between two Solves -- takes CUs ahead of the next Solve's prior-grid pass running beside it
    static const bool aux_hi = ab_int("LMSF_AUX_PRIORITY", 0) != 0;
    int prio_lo = 0, prio_hi = 0;
    if (aux_hi) (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (hipStreamCreateWithPriority(&t->aux[0], hipStreamNonBlocking, aux_hi ? prio_hi : 0) != hipSuccess ||
        hipStreamCreateWithPriority(&t->aux[1], hipStreamNonBlocking, aux_hi ? prio_hi : 0) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_join[LMSF_EDGE], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_join[LMSF_SURF], hipEventDisableTiming) != hipSuccess ||
        hipMalloc((void**)&t->flags, 4 * sizeof(uint32_t)) != hipSuccess ||
        hipMemsetAsync(t->flags, 0, 4 * sizeof(uint32_t), ctx_stream(ctx)) != hipSuccess ||
        hipStreamSynchronize(ctx_stream(ctx)) != hipSuccess) {
        lmsf_tracker_destroy(t);
        return LMSF_ERR_HIP;
    }
    for (int kind = LMSF_EDGE; kind <= LMSF_SURF; ++kind) {
        Window& w = t->win[kind];
        w.slots.assign(cfg->window_frames, nullptr);
        w.sizes.assign(cfg->window_frames, 0);
        for (auto& p : w.slots)
            if (hipMalloc((void**)&p, (size_t)t->cap * sizeof(float4)) != hipSuccess) { lmsf_tracker_destroy(t); return LMSF_ERR_HIP; }
        w.concat_cap = (size_t)t->cap * cfg->window_frames;
        w.leaf = kind == LMSF_EDGE ? cfg->leaf_edge : cfg->leaf_surf;
        if ((w.leaf <= 0 && hipMalloc((void**)&w.concat, w.concat_cap * sizeof(float4)) != hipSuccess) ||
            (w.leaf > 0 && hipMalloc((void**)&w.wcat, w.concat_cap * sizeof(float4)) != hipSuccess)) {
            lmsf_tracker_destroy(t);
            return LMSF_ERR_HIP;
        }
    }
    for (int kind = LMSF_EDGE; kind <= LMSF_SURF; ++kind)
        if (hipMalloc((void**)&t->spare[kind], (size_t)t->cap * sizeof(float4)) != hipSuccess) {
            lmsf_tracker_destroy(t);
            return LMSF_ERR_HIP;
        }
    if (hipMalloc((void**)&t->stage, (size_t)t->cap * sizeof(float4)) != hipSuccess) {
        lmsf_tracker_destroy(t);
        return LMSF_ERR_HIP;
    }
    // A window never exceeds window_frames x the slot capacity: its voxel-filter workspace and grid points are
    // sized for that here, so keyframe commits never grow them (r05: growths inside the first frames -- the window
    // filling up -- cost C3 ~15% over a 20-frame run).  LMSF_OPT_GROWTH_TEST keeps the grow-on-demand path instead.
    if (!ctx_option(ctx, LMSF_OPT_GROWTH_TEST)) {
        const size_t wmax = (size_t)t->cap * (size_t)cfg->window_frames;
        for (int kind = LMSF_EDGE; kind <= LMSF_SURF; ++kind) {
            const bool ok = (t->win[kind].leaf > 0 ? t->voxel[kind].reserve(wmax, ctx_stream(ctx)) == hipSuccess : true) &&
                            ctx_window_reserve(ctx, kind, wmax, ctx_stream(ctx)) == LMSF_OK;
            if (!ok) {
                lmsf_tracker_destroy(t);
                return LMSF_ERR_HIP;
            }
        }
    }
    t->origin = t->curr = t->prev = t->motion = t->last_kf = iso_identity();
    t->fault_seen = ctx_fault_seq(ctx);
    // the context's map consumers (and extractions) settle a deferred commit; with one pending, the next Solve's
    // prior-grid pass is enqueued first so it overlaps the rebuild
    ctx_add_settle(ctx, [](void* p) {
        lmsf_tracker* tk = static_cast<lmsf_tracker*>(p);
        if (tk->init && (tk->pending || tk->staging)) {
            HPROF(7, "settle hook presearch");
            lmsf_status rp = presearch_prediction(tk, nullptr);
            if (rp) return rp;
        }
        return settle(tk);
    }, t);
    const int dev = ctx_device(ctx);
    if (dev >= 0 && dev < 64) {
        g_trackers[dev].fetch_add(1);
        t->counted = true;
    }
    *out = t;
    return LMSF_OK;
}

}  // extern "C"

namespace {

// Solve (:107-160) on the features currently in the context's slot 0.
lmsf_status solve_current(lmsf_tracker* t, double timestamp, double deltaT[16], lmsf_tracker_result* res) {
    HPROF(15, "tracker solve total");
    if (t->init) {   // the prediction below, as register_pose will pass it (a no-op when the settle hook enqueued it)
        lmsf_status rp = presearch_prediction(t, deltaT);
        if (rp) return rp;
    }
    lmsf_status rc0 = settle(t);   // a deferred keyframe commit completes before the search reads the map
    if (rc0) return rc0;
    lmsf_tracker_result r;
    std::memset(&r, 0, sizeof r);
    lmsf_status rc;
    const bool manual = t->cfg.manual_map_update != 0;
    if (!t->init) {                                                   // :112-122
        // the local frame is the first scan's frame (origin = identity, as the reference) unless
        // lmsf_tracker_set_initial_pose placed it in a shared map's frame
        t->curr = t->prev = t->last_kf = t->origin;
        t->motion = iso_identity();
        if (!manual) {
            rc = update_local_map(t, t->origin);
            if (rc) return rc;
        }
        t->last_kf_time = timestamp;
        t->init = true;
        r.initialized = 1;
        r.update_type = LMSF_UPDATE_MOTION;
    } else {
        if (is_identity16(deltaT)) t->curr = iso_mul(t->prev, t->motion);   // :125-129
        else t->curr = iso_mul(t->prev, iso_from16(deltaT));
        // the keyframe lookahead when the prediction already passes the gate (the window rebuild of this scan's
        // features at the Solve's result is posted while the Solve runs)
        const bool look = t->cfg.keyframe_lookahead && sole_tracker(t) && gate_type(t, t->curr, timestamp) != LMSF_UPDATE_NONE;
        if (look) {
            t->look_recoveries = ctx_loop_recoveries(t->ctx);
            // a recovered Solve (lm_loop's bounded wait given up) re-runs only after the lookahead is undone and the
            // restored window rebuilt and joined: the re-run must not search a window being rebuilt
            ctx_arm_post_solve(t->ctx, lookahead_post, [](void* p) { return settle(static_cast<lmsf_tracker*>(p)); }, t);
        }
        rc = register_pose(t, t->curr, &r.solve);                      // :131
        if (t->look == kLookPosted && (rc || ctx_loop_recoveries(t->ctx) != t->look_recoveries)) {
            // a failed Solve, or one re-run after the lookahead read its first result: not a keyframe of this pose
            lmsf_status rl = look_rollback(t);
            if (!rc) rc = rl;
        }
        if (rc) return rc;
        if (t->look == kLookPosted) {
            iso_to16(t->curr, t->look_pose);
            t->look_pose_known = true;
        }
        t->motion = iso_mul(iso_inverse(t->prev), t->curr);             // :133
        iso_to16(t->motion, deltaT);
        t->prev = t->curr;
        const int type = gate_type(t, t->curr, timestamp);             // needUpdataLocalMap (:239-262)
        r.update_type = type;
        if (type) {
            t->last_kf = t->curr;
            t->last_kf_time = timestamp;
            if (!manual) {
                if (t->look == kLookPosted && t->look_feat == ctx_feature_seq(t->ctx)) {
                    t->look = kLookNone;   // updateLocalMap's frame: the lookahead's, completed as commit() would
                    rc = commit_finish(t);
                    if (rc) return rc;
                } else {
                    rc = update_local_map(t, t->curr);
                    if (rc) return rc;
                }
            }
        }
        if (!manual && t->look == kLookPosted) {   // no keyframe after all
            rc = look_rollback(t);
            if (rc) return rc;
        }
    }
    r.local_map_edge = (int64_t)t->win[LMSF_EDGE].total;
    r.local_map_surf = (int64_t)t->win[LMSF_SURF].total;
    if (res) *res = r;
    return LMSF_OK;
}

}  // namespace

extern "C" {

lmsf_status lmsf_tracker_solve(lmsf_tracker* t, const float* edge, size_t n_edge, const float* surf, size_t n_surf,
                               double timestamp, double deltaT[16], lmsf_tracker_result* res) {
    if (!t || !deltaT || (n_edge && !edge) || (n_surf && !surf)) return LMSF_ERR_ARG;
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    lmsf_status rc = set_features(t, edge, n_edge, surf, n_surf);
    if (rc) return rc;
    return solve_current(t, timestamp, deltaT, res);
}

lmsf_status lmsf_tracker_solve_extracted(lmsf_tracker* t, double timestamp, double deltaT[16], lmsf_tracker_result* res) {
    if (!t || !deltaT) return LMSF_ERR_ARG;
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    if (!ctx_features_on_device(t->ctx)) return fail(t, LMSF_ERR_STATE, "no extracted features on the device");
    return solve_current(t, timestamp, deltaT, res);
}

lmsf_status lmsf_tracker_set_initial_pose(lmsf_tracker* t, const double pose[16]) {
    if (!t || !pose) return LMSF_ERR_ARG;
    if (t->init) return fail(t, LMSF_ERR_STATE, "initial pose after the first scan");
    t->origin = iso_from16(pose);
    return LMSF_OK;
}

lmsf_status lmsf_tracker_set_prior_map(lmsf_tracker* t, int32_t kind, const float* xyzi, size_t n) {
    if (!t || (kind != LMSF_EDGE && kind != LMSF_SURF) || (n && !xyzi)) return LMSF_ERR_ARG;
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    {
        lmsf_status rs = settle(t);
        if (rs) return rs;
    }
    Window& w = t->win[kind];
    hipStream_t s = ctx_stream(t->ctx);
    TCHK(t, hipStreamSynchronize(s));
    TCHK(t, hipFree(w.prior));
    w.prior = nullptr;
    w.prior_n = 0;
    if (n) {
        TCHK(t, hipMalloc((void**)&w.prior, n * sizeof(float4)));
        TCHK(t, hipMemcpyAsync(w.prior, xyzi, n * sizeof(float4), hipMemcpyDefault, s));
        w.prior_n = n;
    }
    lmsf_status rc = ctx_set_prior_device(t->ctx, kind, w.prior, n);   // static grid, built once
    if (rc) return rc;
    w.dirty = true;                 // window indices move behind the new prior
    return commit(t);
}

lmsf_status lmsf_tracker_add_keyframe(lmsf_tracker* t, const float* edge, size_t n_edge, const float* surf,
                                      size_t n_surf, const double pose[16]) {
    if (!t || !pose || (n_edge && !edge) || (n_surf && !surf)) return LMSF_ERR_ARG;
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    {
        lmsf_status rs = settle(t);
        if (rs) return rs;
    }
    hipStream_t s = ctx_stream(t->ctx);
    const Iso T = iso_from16(pose);
    const float* src[3] = {nullptr, edge, surf};
    const size_t cnt[3] = {0, n_edge, n_surf};
    for (int kind = LMSF_EDGE; kind <= LMSF_SURF; ++kind) {
        if (cnt[kind] == 0) continue;
        if (cnt[kind] > (size_t)t->cap) return fail(t, LMSF_ERR_CAPACITY, "keyframe larger than the tracker slot capacity");
        // device memory of this GPU is transformed in place; host (or other-device) memory is staged first
        const float4* from = t->stage;
        hipPointerAttribute_t pa;
        if (hipPointerGetAttributes(&pa, src[kind]) == hipSuccess && pa.type == hipMemoryTypeDevice &&
            pa.device == ctx_device(t->ctx))
            from = reinterpret_cast<const float4*>(src[kind]);
        else
            TCHK(t, hipMemcpyAsync(t->stage, src[kind], cnt[kind] * sizeof(float4), hipMemcpyDefault, s));
        (void)hipGetLastError();   // a host pointer's failed attribute query leaves an error behind
        lmsf_status rc = push_frame(t, kind, from, (int64_t)cnt[kind], T);
        if (rc) return rc;
    }
    return LMSF_OK;
}

lmsf_status lmsf_tracker_add_keyframe_extracted(lmsf_tracker* t, const double pose[16]) {
    if (!t || !pose) return LMSF_ERR_ARG;
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    if (t->look == kLookPosted && t->look_pose_known && std::memcmp(pose, t->look_pose, sizeof t->look_pose) == 0 &&
        t->look_feat == ctx_feature_seq(t->ctx)) {
        t->look = kLookAdopted;   // this frame is in the window already, its rebuild posted
        return LMSF_OK;
    }
    {
        lmsf_status rs = settle(t);
        if (rs) return rs;
    }
    if (!ctx_features_on_device(t->ctx)) return fail(t, LMSF_ERR_STATE, "no extracted features on the device");
    const float4* feat;
    int64_t ne, ns;
    lmsf_status rc = ctx_slot0_features(t->ctx, &feat, &ne, &ns);
    if (rc) return rc;
    HPROF(14, "add_keyframe_extracted push");
    const Iso T = iso_from16(pose);
    rc = push_frame(t, LMSF_EDGE, feat, ne, T);
    if (rc) return rc;
    return push_frame(t, LMSF_SURF, feat + ne, ns, T);
}

// Returns once the rebuild is enqueued (commit_stage); the next tracker call completes it (settle), so
// work the caller enqueues on the context in between (the next scan's extraction) runs beside it.
lmsf_status lmsf_tracker_commit_map(lmsf_tracker* t) {
    if (!t) return LMSF_ERR_ARG;
    HPROF(13, "commit_map call");
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    if (t->look == kLookAdopted) {   // the adopted lookahead's rebuild is this commit, posted already
        t->look = kLookNone;
        return LMSF_OK;
    }
    lmsf_status rc = settle(t);
    if (rc) return rc;
    // the keyframe transforms enqueued so far on the context stream, then each changed kind's rebuild enqueued
    // by its worker on its aux stream
    return post_commit(t);
}

lmsf_status lmsf_tracker_register(lmsf_tracker* t, const float* edge, size_t n_edge, const float* surf,
                                  size_t n_surf, double pose[16], lmsf_solve_stats* stats) {
    if (!t || !pose) return LMSF_ERR_ARG;
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    {
        lmsf_status rs = settle(t);
        if (rs) return rs;
    }
    lmsf_status rc = set_features(t, edge, n_edge, surf, n_surf);
    if (rc) return rc;
    Iso T = iso_from16(pose);
    lmsf_solve_stats st;
    rc = register_pose(t, T, &st);
    if (rc) return rc;
    iso_to16(T, pose);
    if (stats) *stats = st;
    return LMSF_OK;
}

lmsf_status lmsf_tracker_register_extracted(lmsf_tracker* t, double pose[16], lmsf_solve_stats* stats) {
    if (!t || !pose) return LMSF_ERR_ARG;
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    {
        lmsf_status rs = settle(t);
        if (rs) return rs;
    }
    if (!ctx_features_on_device(t->ctx)) return fail(t, LMSF_ERR_STATE, "no extracted features on the device");
    Iso T = iso_from16(pose);
    lmsf_solve_stats st;
    lmsf_status rc = register_pose(t, T, &st);
    if (rc) return rc;
    iso_to16(T, pose);
    if (stats) *stats = st;
    return LMSF_OK;
}

lmsf_status lmsf_tracker_pose(const lmsf_tracker* t, double T[16]) {
    if (!t || !T) return LMSF_ERR_ARG;
    iso_to16(t->curr, T);
    return LMSF_OK;
}

lmsf_status lmsf_tracker_local_map(lmsf_tracker* t, int32_t kind, float* out, size_t cap, size_t* n_out) {
    if (!t || (kind != LMSF_EDGE && kind != LMSF_SURF)) return LMSF_ERR_ARG;
    if (hipSetDevice(ctx_device(t->ctx)) != hipSuccess) return LMSF_ERR_HIP;
    lmsf_status rs = settle(t);   // the window sizes of a deferred commit
    if (rs) return rs;
    const Window& w = t->win[kind];
    if (n_out) *n_out = w.total;
    if (!out) return LMSF_OK;
    if (w.total > cap) return fail(t, LMSF_ERR_CAPACITY, "output capacity smaller than the local map");
    hipStream_t s = ctx_stream(t->ctx);
    if (w.prior_n) TCHK(t, hipMemcpyAsync(out, w.prior, w.prior_n * sizeof(float4), hipMemcpyDefault, s));
    if (w.window_n)
        TCHK(t, hipMemcpyAsync(out + 4 * w.prior_n, ctx_window_points(t->ctx, kind), w.window_n * sizeof(float4),
                               hipMemcpyDefault, s));
    TCHK(t, hipStreamSynchronize(s));
    return LMSF_OK;
}

}  // extern "C"
