/*
 * lmsf.h -- C ABI of the MI355X-native LOAM edge/surface registration hot path.
 *
 * Drop-in boundary for LMSF-Slam's feature-based registration plugin
 * (selection string "feature_based", INC/factory/System/ML_SystemFactory.hpp:179-198;
 * INC = src/MultiSensorFusionEstimator3D/include, REG = INC/Algorithm/PointClouds/registration,
 * FX = INC/Algorithm/PointClouds/processing/FeatureExtract).  Every entry point below names the
 * reference interface it replaces.  Plain pointers and sizes only; no exceptions cross the ABI;
 * every call returns an lmsf_status (0 ok, < 0 error, message in lmsf_last_error()).
 *
 * Threading: a context is used by one host thread at a time and owns one HIP stream on one
 * device; distinct contexts may run concurrently (same rule as the reference, where each
 * tracker owns its registration object: INC/System/ML_System.hpp:248-264).
 * Ownership: the library copies every input into device buffers it owns; no caller pointer is
 * retained after a call returns, except by lmsf_batch_load_scans_async (documented there).
 */
#ifndef LMSF_LMSF_H_
#define LMSF_LMSF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t lmsf_status;
#define LMSF_OK 0
#define LMSF_ERR_ARG (-1)       /* bad argument / null pointer */
#define LMSF_ERR_HIP (-2)       /* HIP runtime failure (device missing, OOM, launch error) */
#define LMSF_ERR_NO_MAP (-3)    /* solve before any map was set */
#define LMSF_ERR_CAPACITY (-4)  /* input larger than the context was created for */
#define LMSF_ERR_STATE (-5)     /* call out of order (e.g. copy features before extraction) */

/* feature cloud names of the reference: "loam_edge" / "loam_surf" (FX:124-125) */
#define LMSF_EDGE 1
#define LMSF_SURF 2

#define LMSF_SOLVER_CERES_LM 0  /* CeresEdgeSurfFeatureRegistration (REG/ceres_edgeSurfFeatureRegistration.hpp) */
#define LMSF_SOLVER_GN 1        /* EdgeSurfFeatureRegistration, GN mode (REG/edgeSurfFeatureRegistration.hpp) */

#define LMSF_SCHEDULE_REFERENCE_DECAY 0 /* optimization_count_ 10 -> 9, 8, ... 2 (ceres_...:100-101) */
#define LMSF_SCHEDULE_FIXED 1           /* exactly max_iterations outer iterations per solve */

/* termination of the last inner solve (Ceres TerminationType / GN convergence) */
#define LMSF_TERM_MAX_ITERATIONS 0
#define LMSF_TERM_FUNCTION_TOL 1
#define LMSF_TERM_PARAMETER_TOL 2
#define LMSF_TERM_GRADIENT_TOL 3
#define LMSF_TERM_NO_RESIDUALS 4
#define LMSF_TERM_GN_CONVERGED 5
#define LMSF_TERM_GN_TOO_FEW 6

typedef struct {
    int32_t device;            /* HIP device ordinal */
    int32_t solver;            /* LMSF_SOLVER_* */
    int32_t schedule;          /* LMSF_SCHEDULE_* */
    int32_t max_iterations;    /* initial optimization_count_ (10: ceres_...:46) */
    int32_t max_batch;         /* registrations processed together by lmsf_batch_run */
    int32_t max_scan_points;   /* raw points per scan (capacity) */
    int32_t max_features;      /* edge + surf features per scan (capacity) */
    /* LOAMFeatureProcessorBase(N_SCANS, min_distance, max_distance, edge_thresh, voxel, RemovalBadPoints)
       (FX:36-50); the factory uses (16, 2, 80) (ML_SystemFactory.hpp:196-197). */
    int32_t n_scans;
    float min_distance;
    float max_distance;
    float edge_threshold;
    int32_t remove_bad_points;
    /* build-defined uniform beam model for N_SCANS not in {16, 32, 64} (0 spacing: reference
       behaviour, every point in ring 0, FX:337-341) */
    double beam_lo_deg;
    double beam_spacing_deg;
    /* Which libm overloads the reference's unqualified sqrt / atan2 calls on float arguments bind to
       (FX:223-224 atan2(x, y), FX:247-252 sqrt, FX:300-301 sqrt): 0 = the double versions, as on the
       reference's documented toolchain (README.md:35, ROS kinetic: GCC 5, whose global-scope <math.h>
       declares only double sqrt / atan2); 1 = the float overloads, as with GCC >= 6 once libstdc++'s
       <math.h> wrapper is included (it exports std::sqrt(float) / std::atan2(float, float) to the
       global namespace) -- float atan2 taken as (float)atan2 in double, within glibc atan2f's 1 ulp. */
    int32_t libm_float;
} lmsf_config;

/* One correspondence (64 bytes).  kind 0: none, 1: edge (v0 = a, v1 = b: the two line points of
 * EdgeFeatureMatch.hpp:72-73), 2: surf (v0 = unit normal, v1[0] = D: surfFeatureMatch.hpp:76-82).
 * p is the feature in the lidar frame (the factor's curr_point, ceres_...:148-150). */
typedef struct {
    float px, py, pz;
    int32_t kind;
    double v0[3];
    double v1[3];
} lmsf_record;

typedef struct {
    int32_t outer_iterations;
    int32_t edge_matches;      /* of the last outer iteration */
    int32_t surf_matches;
    int32_t inner_iterations;  /* summed over outer iterations */
    int32_t evaluations;       /* residual passes summed over outer iterations */
    int32_t termination;       /* LMSF_TERM_* of the last outer iteration */
    double initial_cost;       /* of the last outer iteration */
    double final_cost;
} lmsf_solve_stats;

typedef struct {
    int64_t n_edge;
    int64_t n_surf;
} lmsf_feature_counts;

typedef struct lmsf_ctx lmsf_ctx;

/* Defaults: device 0, Ceres-LM, reference decay, 10 iterations, batch 1, VLP-16 (16, 2, 80, 1, true). */
lmsf_status lmsf_config_init(lmsf_config* cfg);

/* Registration object construction: CeresEdgeSurfFeatureRegistration("loam_edge", "loam_surf")
 * (REG/ceres_edgeSurfFeatureRegistration.hpp:45-49) + LOAMFeatureProcessorBase ctor (FX:36-50). */
lmsf_status lmsf_ctx_create(const lmsf_config* cfg, lmsf_ctx** out);
void lmsf_ctx_destroy(lmsf_ctx* ctx);
/* Message of the last error on ctx, copied under the context's error lock; valid until the next call of
 * lmsf_last_error on the same context from any thread (call it from one thread per context). */
const char* lmsf_last_error(const lmsf_ctx* ctx);

/* RegistrationBase::SetInputSource (REG/registration_base.hpp:31; ceres_...:56-71): set the local
 * feature map of one kind and build its device neighbour index.  n == 0 keeps the previous map
 * (ceres_...:60).  xyzi may be host or device memory of the context's GPU (e.g. a map received by
 * an RCCL broadcast). */
lmsf_status lmsf_set_map(lmsf_ctx* ctx, int32_t kind, const float* xyzi, size_t n);

/* RegistrationBase::SetInputTarget (REG/registration_base.hpp:32; ceres_...:73-84): set the
 * current scan's features of one kind (host arrays, copied to the device). */
lmsf_status lmsf_set_scan(lmsf_ctx* ctx, int32_t kind, const float* xyzi, size_t n);

/* SetMaxIteration (ceres_...:86-89). */
lmsf_status lmsf_set_max_iterations(lmsf_ctx* ctx, int32_t n);
/* Outer-iteration schedule: LMSF_SCHEDULE_REFERENCE_DECAY (the reference's per-object
 * optimization_count_ decrement, ceres_...:100-101) or LMSF_SCHEDULE_FIXED (benchmarks). */
lmsf_status lmsf_set_schedule(lmsf_ctx* ctx, int32_t schedule);

/* LOAMFeatureProcessorBase constructor arguments (FX:36-50) + the build's beam model, changeable
 * between extractions (lmsf_config holds the initial values). */
typedef struct {
    int32_t n_scans;           /* 1..128 */
    float min_distance;
    float max_distance;
    float edge_threshold;
    int32_t remove_bad_points;
    double beam_lo_deg;
    double beam_spacing_deg;
    int32_t libm_float;        /* lmsf_config::libm_float */
} lmsf_extract_params;
lmsf_status lmsf_set_extract_params(lmsf_ctx* ctx, const lmsf_extract_params* p);

/* RegistrationBase::Solve (REG/registration_base.hpp:33; ceres_...:96-130).  pose: qx qy qz qw tx
 * ty tz (Eigen storage order of ceres_...:38-40); in = predicted map<-lidar pose, out = refined. */
lmsf_status lmsf_solve(lmsf_ctx* ctx, double pose[7], lmsf_solve_stats* stats);
/* Pose after every outer iteration of the last lmsf_solve (rows of 7 doubles); *n_out = rows. */
lmsf_status lmsf_solve_trace(lmsf_ctx* ctx, double* trace, int32_t cap, int32_t* n_out);

/* PointCloudProcessBase::Process (INC/Algorithm/PointClouds/processing/process_base.hpp:26-39),
 * LOAM implementation FX:59-126: extract "loam_edge" / "loam_surf" from a raw scan.  The features
 * stay device-resident and become the current scan target (as SetInputTarget with the
 * processor's output container) without a host round trip.  xyzi: host or device memory. */
lmsf_status lmsf_extract_features(lmsf_ctx* ctx, const float* xyzi, size_t n, lmsf_feature_counts* counts);

/* The extraction of the NEXT scan, enqueued now on a stream of the context's own so that it runs beside
 * what the context runs meanwhile (normally the current scan's solve): the next lmsf_extract_features call
 * with the same xyzi pointer and n adopts its result instead of extracting again (bitwise the same features:
 * the same kernels on the same input).  The scan must stay unchanged until that call; any other extraction
 * first waits for the prefetch and discards it.  The pipelining of the reference's preprocess and estimate
 * threads (apps/src/MultiLidarOdometry/lidar_lidar_odometry.cpp:281-284: features of scan k+1 are extracted
 * while scan k is registered). */
lmsf_status lmsf_prefetch_features(lmsf_ctx* ctx, const float* xyzi, size_t n);
/* PointCloudCommonProcess<P>(output_name = "filtered")::Process (INC/Algorithm/PointClouds/processing/
 * common_processing.hpp:87-112), the preprocessor of the "sparse_point_plane_icp" scan-to-map mode
 * (INC/factory/System/ML_SystemFactory.hpp:141-178): optional removeNaNFromPointCloud, VoxelGrid
 * (centroids, as lmsf_voxel_filter), then DistanceFilter (float |p| promoted to double, keep
 * near < d < far; distance_filter.hpp:24-43); the outlier filter is not configured on that path.  The
 * "filtered" cloud becomes the current surf target on the device (no edge cloud: the registration is
 * CeresEdgeSurfFeatureRegistration("", "filtered")), as lmsf_extract_features does for the LOAM
 * clouds; lmsf_copy_features(LMSF_SURF) returns it.  Defaults (lmsf_common_params_init) are
 * config/MultiSensorSystem/point_plane_icp_test.yaml:16-24: VoxelGrid 0.5 m, distance 2 .. 100 m,
 * no NaN removal (the constructor's removal_nan = false). */
typedef struct {
    int32_t removal_nan;
    float voxel_leaf;          /* m; 0: no downsampling */
    float distance_near;       /* both 0: no distance filter (DistanceFilter's pass-through) */
    float distance_far;
} lmsf_common_params;
lmsf_status lmsf_common_params_init(lmsf_common_params* p);
lmsf_status lmsf_common_process(lmsf_ctx* ctx, const float* xyzi, size_t n, const lmsf_common_params* p,
                                lmsf_feature_counts* counts);
/* Copy the current features of one kind (xyzi rows, reference emission order) to host or device
 * memory; src (nullable) receives each feature's index in the raw scan. */
lmsf_status lmsf_copy_features(lmsf_ctx* ctx, int32_t kind, float* out, int32_t* src, size_t cap, size_t* n_out);

/* Batch throughput path: n independent registrations against the context's map (the ML_System
 * per-LiDAR loop, INC/System/ML_System.hpp:137-156 + :248-264, run as one device pass).
 * load_scans copies raw scans (concatenated rows, counts[i] points each; host or device memory)
 * into device slots;
 * run extracts features for every slot and registers slot i from poses[i] (in/out). */
lmsf_status lmsf_batch_load_scans(lmsf_ctx* ctx, const float* xyzi, const int64_t* counts, int32_t n);
/* Streaming ingest (the driver callback feeding MultiLidarSystem, APPS/MultiLidarSLAM_node.cpp:126-180):
 * the copy of lmsf_batch_load_scans enqueued on the context's copy stream without blocking, into
 * the raw slots the NEXT lmsf_batch_launch extracts from.  It starts once the previous launch's
 * extraction has read those slots, so it overlaps that launch's registration.  The caller keeps
 * xyzi (page-locked host memory for a truly asynchronous copy) and counts' values unchanged until
 * the lmsf_batch_wait of that next launch returns. */
lmsf_status lmsf_batch_load_scans_async(lmsf_ctx* ctx, const float* xyzi, const int64_t* counts, int32_t n);
/* n may not exceed the scans of the last load (LMSF_ERR_STATE): a load of fewer scans -- including
 * lmsf_extract_features, which loads one scan into slot 0 -- replaces a streamed batch not yet launched. */
lmsf_status lmsf_batch_run(lmsf_ctx* ctx, int32_t n, double* poses, lmsf_solve_stats* stats);
/* Same, but without blocking: poses are read back by lmsf_batch_wait. */
lmsf_status lmsf_batch_launch(lmsf_ctx* ctx, int32_t n, const double* poses);
lmsf_status lmsf_batch_wait(lmsf_ctx* ctx, int32_t n, double* poses, lmsf_solve_stats* stats);
/* Pose after every outer iteration of batch slot `slot` in the last lmsf_batch_wait / lmsf_batch_run
 * (rows of 7 doubles, as lmsf_solve_trace); *n_out = rows. */
lmsf_status lmsf_batch_trace(lmsf_ctx* ctx, int32_t slot, double* trace, int32_t cap, int32_t* n_out);
/* Features of one batch slot after lmsf_batch_run. */
lmsf_status lmsf_batch_copy_features(lmsf_ctx* ctx, int32_t slot, int32_t kind, float* out, int32_t* src,
                                     size_t cap, size_t* n_out);

/* ---- context options (not on the reference surface): algorithm switches of the build.
 * Results do not depend on them (the memo switches are exact, DESIGN.md section 4 "Query memo"); they
 * exist so tests can compare the paths in one process and a caller can rule a path out.  Values 0 | 1;
 * defaults 1 except LMSF_OPT_GRAPH and the testing options (LOOP_FAULT_TEST, GROWTH_TEST, FAULT_INJECT) 0;
 * FAULT_INJECT also takes 2. */
#define LMSF_OPT_QUERY_MEMO 0   /* 1: outer iterations > 0 reuse 5-NN sets that provably did not change */
#define LMSF_OPT_MEMO_REFIT 1   /* 1: a reused set in a new order is refitted without a walk */
#define LMSF_OPT_MEMO_EXACT 2   /* 1: keep the set when its farthest point is nearer than s6 - d (0: 2d < s6 - s5) */
#define LMSF_OPT_MEMO_ORDER 3   /* 1: consecutive-gap test first (no re-keying when every gap exceeds 2d) */
#define LMSF_OPT_MEMO_BOUND 4   /* 1: memo misses walk min(1 m, s6 + d) instead of 1 m */
#define LMSF_OPT_GRAPH 5        /* 1: replay state init + registration as a HIP graph (default 0) */
#define LMSF_OPT_MEMO_SKIP1 6   /* 1: batch launches search outer iteration 1 in full (no memo pass): the first LM
                                 *    solve moves the queries past the memo's gaps, so its pass finds ~nothing
                                 *    (default 1; 0: the memo pass from iteration 1) */
#define LMSF_OPT_LM_LOOP 7      /* 1: single-scan launches run each outer iteration's Ceres LM as one launch when its
                                 *    grid is co-resident (lm_loop_kernel); 0: the 9-launch form (default 1) */
#define LMSF_OPT_LOOP_FAULT_TEST 8 /* 1 (testing only): lm_loop_kernel's bounded waits give up at once, forcing the
                                 *    fault and its recovery -- the Solve re-run on the 9-launch form (default 0) */
#define LMSF_OPT_GROWTH_TEST 9  /* 1 (testing only): map grids and voxel-filter workspaces grow to each request exactly
                                 *    and window grids start at 2^10 cells, so a tracker's buffers are regrown at
                                 *    nearly every keyframe commit (on the commit streams) (default 0) */
#define LMSF_OPT_FAULT_INJECT 10 /* 1 | 2 (testing only): the next voxel filters' first radix pass takes a stale
                                 *    prefix (1: an out-of-range scatter) or meets a foreign look-back word (2); the
                                 *    device checks flag it and the next Solve / batch wait fails with LMSF_ERR_HIP
                                 *    "device look-back fault" (default 0) */
#define LMSF_OPT_COUNT 11
lmsf_status lmsf_set_option(lmsf_ctx* ctx, int32_t option, int32_t value);

/* ---- diagnostics used by the parity tests and the roofline report (not on the reference surface) */
/* Record capture: for the following launches (lmsf_batch_launch / lmsf_batch_run / lmsf_solve), the
 * correspondence records and 5-NN indices of up to LMSF_MAX_CAPTURE batch slots are copied aside on the
 * device after every outer iteration's matching (the first 10), with the pose they were matched at --
 * the records the solver then reads, including those the query memo reused or refitted.  n = 0 stops it.
 * The capture makes the search kernels also store their neighbours (stores only; the same kernels). */
#define LMSF_MAX_CAPTURE 4
lmsf_status lmsf_batch_capture(lmsf_ctx* ctx, const int32_t* slots, int32_t n);
/* Captured rows of `slot` at outer iteration `iter` of the last launch, in slot order (edges then surfs,
 * as lmsf_match): records, neighbour indices (5 per query, -1: rank not found within 1 m; nullable), the
 * linearisation pose (nullable); *n_out = queries.  Host or device memory. */
lmsf_status lmsf_batch_records(lmsf_ctx* ctx, int32_t slot, int32_t iter, lmsf_record* out, int32_t* nn, size_t cap,
                               double pose[7], size_t* n_out);

/* Matching only at a pose: n_edge + n_surf records (edges first) and the 5 neighbour map indices. */
lmsf_status lmsf_match(lmsf_ctx* ctx, const double pose[7], lmsf_record* out, int32_t* nn, size_t cap);
/* Weighted normal-equation packet of the current records at a pose: cost, H (21 upper, row-major),
 * g (6), count -- the quantities the device LM reduces. */
lmsf_status lmsf_eval(lmsf_ctx* ctx, const double pose[7], double out[29]);
/* Device self-test of the restated Eigen 3.3 SelfAdjointEigenSolver the kernels run: n symmetric dim x dim
 * matrices (row-major, lower triangle read; host or device memory) -> ascending eigenvalues d[n][dim],
 * eigenvectors v[n][dim][dim] (row-major, eigenvector i in column i), info[n] (0 Success, 1 NoConvergence).
 * dim 3: the fixed-size Matrix3d path of the edge fit (EdgeFeatureMatch.hpp:63); dim 6: the MatrixXd path
 * of the GN degeneracy test (edgeSurfFeatureRegistration.hpp:282).  Synchronous on the context stream. */
lmsf_status lmsf_eigen_selfadjoint(lmsf_ctx* ctx, int32_t dim, const double* a, size_t n, double* d, double* v,
                                   int32_t* info);
/* Neighbour-search kernel accounting since the last reset: launches, summed device time (ms,
 * HIP events on the context stream), queries, and sum over queries of n27 (map points in the
 * 3x3x3 block of 1 m cells around each query: the algorithmic-byte figure of DESIGN.md).
 * reset mode: LMSF_STATS_TIMING (events, launches, queries) | LMSF_STATS_N27 (n27_sum and
 * queries; costs the search extra cell-offset loads, so it is kept out of timed launches);
 * 0 turns accounting off.  fused_launches: how many of the launches were the fused search + fit
 * kernel (batch launches with the Ceres-LM solver; the fit is then inside the timed launch).
 * reused_queries: queries of those launches (outer iterations > 0) that moved less than half the
 * neighbour-distance gap of their last full search, so their 5-NN set and fit were reused without a
 * search (counted with the queries; DESIGN.md "Query memo"); refit_queries: queries whose 5-NN set was
 * unchanged but reordered, refitted from the memo without a walk. */
#define LMSF_STATS_TIMING 1
#define LMSF_STATS_N27 2
typedef struct {
    int64_t launches;
    double total_ms;
    int64_t queries;
    int64_t n27_sum;
    int64_t fused_launches;
    int64_t reused_queries;
    int64_t refit_queries;
    int64_t loop_recoveries;  /* solves whose single-launch LM loop gave up a bounded wait and were re-run on
                               * the 9-launch form (results as without the fault) */
    int64_t buffer_growths;   /* map-grid buffer growths since the context was created (not reset: the
                               * growth test checks that a tracker's window grids were regrown) */
    int64_t split_searches;   /* Solves whose outer iteration 0 ran in two passes: the prior grids' walk enqueued
                               * beside a tracker's keyframe window rebuild, then the window's (same results) */
    int64_t lookahead_solves; /* Solves during which a tracker's keyframe lookahead was enqueued
                               * (lmsf_tracker_config.keyframe_lookahead) */
} lmsf_kernel_stats;
lmsf_status lmsf_kernel_stats_get(lmsf_ctx* ctx, lmsf_kernel_stats* out);
lmsf_status lmsf_kernel_stats_reset(lmsf_ctx* ctx, int32_t mode);

/* ---- scan-to-local-map tracker: LidarTrackerLocalMap<P, RegistrationBase<P>>
 * (INC/LidarTracker/LidarTrackerLocalMap.hpp:42-263) over one context's registration.
 * The local map implementation is absent from the reference snapshot (factory/Map/LocalMap_factory.hpp,
 * included at :15); the build defines "sliding_Localmap" as a window of the last `window_frames`
 * keyframes per feature kind, concatenated oldest -> newest and VoxelGrid-downsampled (leaf per
 * kind), rebuilt on the device at every keyframe (MOTION and TIME updates both append).  Without
 * the downsampling a 16-beam keyframe's 5-NN sets lie on one ring (degenerate plane fits) and
 * tracking drifts by decimetres per frame.  Poses are row-major 4x4 Isometry3d matrices. */
typedef struct lmsf_tracker lmsf_tracker;
typedef struct {
    int32_t window_frames;     /* keyframes kept per feature map: 10, the LOAM MultiLidar config's
                                  tracker.local_map_type.sliding_window.size
                                  (config/MultiLidar_system/loam_feature_multi_lidar_system.yaml:28-29) */
    double threshold_trans;    /* THRESHOLD_TRANS_ = 0.3 m   (LidarTrackerLocalMap.hpp:65) */
    double threshold_rot;      /* THRESHOLD_ROT_   = 0.1 rad */
    double time_interval;      /* TIME_INTERVAL_   = 10 s */
    int32_t manual_map_update; /* 0 (reference): a keyframe is appended inside solve.  1: solve only
                                  decides (res->update_type, keyframe pose/time); the caller appends
                                  keyframes with lmsf_tracker_add_keyframe and rebuilds once with
                                  lmsf_tracker_commit_map (multi-stream map stitching) */
    double leaf_edge;          /* VoxelGrid leaf of the keyframe window, per kind (build-defined: */
    double leaf_surf;          /* 0.2 / 0.4 m, LOAM's mapping resolutions; 0 = no downsampling) */
    int32_t keyframe_lookahead; /* 1 (default): when the motion-model prediction already passes the keyframe
                                  gate, the window rebuild with this scan's features at the Solve's result is
                                  started on the device while the Solve runs; a keyframe of exactly that pose and
                                  those features (the tracker's own, lmsf_tracker_add_keyframe_extracted with
                                  lmsf_tracker_pose, or the automatic update) adopts it, anything else undoes it.
                                  Results are identical either way.  0 for callers that append other streams'
                                  keyframes first (the lookahead would be undone every time), and under tools that
                                  serialise kernel dispatches (its rebuild is ordered by device-side flag waits) */
} lmsf_tracker_config;

#define LMSF_UPDATE_NONE 0    /* LocalMapUpdataType NO_UPDATA */
#define LMSF_UPDATE_MOTION 1  /* MOTION_UPDATA */
#define LMSF_UPDATE_TIME 2    /* TIME_UPDATA */

typedef struct {
    int32_t initialized;       /* 1 when this call only seeded the local map (first call, :112-122) */
    int32_t update_type;       /* LMSF_UPDATE_* decided by needUpdataLocalMap (:239-262) */
    int64_t local_map_edge;    /* local map sizes after the call */
    int64_t local_map_surf;
    lmsf_solve_stats solve;
} lmsf_tracker_result;

lmsf_status lmsf_tracker_config_init(lmsf_tracker_config* cfg);
/* SetRegistration + SetLocalMap({"loam_edge", "loam_surf"}, "sliding_Localmap") on context ctx. */
lmsf_status lmsf_tracker_create(lmsf_ctx* ctx, const lmsf_tracker_config* cfg, lmsf_tracker** out);
void lmsf_tracker_destroy(lmsf_tracker* t);
/* LidarTrackerLocalMap::Solve (:107-160): features of the current scan, timestamp (s), deltaT
 * in/out (identity in => constant-velocity prediction; out = motion increment). */
lmsf_status lmsf_tracker_solve(lmsf_tracker* t, const float* edge, size_t n_edge, const float* surf, size_t n_surf,
                               double timestamp, double deltaT[16], lmsf_tracker_result* res);
/* RegistrationLocalMap (:168-177): register features against the local map from pose (in/out),
 * no tracker state change (the dual-LiDAR refine of INC/System/ML_System.hpp:303-307). */
lmsf_status lmsf_tracker_register(lmsf_tracker* t, const float* edge, size_t n_edge, const float* surf,
                                  size_t n_surf, double pose[16], lmsf_solve_stats* stats);
/* GetCurrPoseInLocalFrame (:182-185). */
lmsf_status lmsf_tracker_pose(const lmsf_tracker* t, double T[16]);
/* GetLocalMap (:187-195): copy one feature map of the window (prior map first, then keyframes
 * oldest -> newest) to host or device memory. */
lmsf_status lmsf_tracker_local_map(lmsf_tracker* t, int32_t kind, float* out, size_t cap, size_t* n_out);

/* Extensions for the multi-stream configurations (not on the reference surface):
 * solve_extracted = lmsf_tracker_solve on the features lmsf_extract_features left on the device;
 * set_initial_pose = before the first scan: the local frame's pose of the first scan (default
 *                   identity = the reference's "first scan defines the local frame");
 * set_prior_map   = a static map (local frame) kept in front of the keyframe window (shared map
 *                   replicated on every GPU; xyzi host or device memory; index rebuilt at once);
 * add_keyframe    = transform features by pose (local <- lidar) and push them into the window
 *                   (evicting the oldest); any thread's stream may contribute, in a fixed order;
 * commit_map      = rebuild the device neighbour index of every kind the window changed. */
lmsf_status lmsf_tracker_solve_extracted(lmsf_tracker* t, double timestamp, double deltaT[16], lmsf_tracker_result* res);
/* lmsf_tracker_register on the device-extracted features (C3: the sub-LiDAR scan is extracted on
 * the primary tracker's context after its Solve, then registered against the primary local map). */
lmsf_status lmsf_tracker_register_extracted(lmsf_tracker* t, double pose[16], lmsf_solve_stats* stats);
lmsf_status lmsf_tracker_set_initial_pose(lmsf_tracker* t, const double pose[16]);
lmsf_status lmsf_tracker_set_prior_map(lmsf_tracker* t, int32_t kind, const float* xyzi, size_t n);
lmsf_status lmsf_tracker_add_keyframe(lmsf_tracker* t, const float* edge, size_t n_edge, const float* surf,
                                      size_t n_surf, const double pose[16]);
/* add_keyframe of the features lmsf_extract_features left on the context's device (a stream's own
 * keyframe: no copy out and back). */
lmsf_status lmsf_tracker_add_keyframe_extracted(lmsf_tracker* t, const double pose[16]);
/* Rebuilds the local map from the appended keyframes.  Returns once the rebuild is enqueued on the
 * tracker's own streams; the next lmsf_tracker_* call on t completes it, and so does the context's next
 * lmsf_extract_features (after enqueuing the extraction, so the window grids are built beside it); map
 * consumers of the same context (lmsf_solve, lmsf_match, lmsf_batch_launch, lmsf_set_map) complete it
 * first as well. */
lmsf_status lmsf_tracker_commit_map(lmsf_tracker* t);

/* VoxelGridFilter::Filter (INC/Algorithm/PointClouds/processing/Filter/voxel_grid.hpp:25-34,
 * filter_base.hpp:34-45; pcl::VoxelGrid centroids, ascending voxel index, input returned unchanged
 * when the voxel index would overflow int32).  in/out: host or device memory; *n_out = voxels. */
lmsf_status lmsf_voxel_filter(lmsf_ctx* ctx, const float* xyzi, size_t n, float leaf, float* out, size_t cap,
                              size_t* n_out);

/* ---- scan ingest: sensor_msgs/PointCloud2 -> pcl::fromROSMsg +
 * pcl::removeNaNFromPointCloud (src/apps/src/MultiLidarSLAM_node.cpp:125-132) ->
 * RotaryLidarPreProcess::Process (INC/Algorithm/PointClouds/processing/Preprocess/
 * RotaryLidar_preprocessing.hpp:31-104: relative time in the intensity field) ->
 * DistanceFilter::Filter (.../processing/Filter/distance_filter.hpp:24-43, optional). */
typedef struct {
    uint32_t point_step;        /* PointCloud2.point_step (bytes per point) */
    int32_t offset_x, offset_y, offset_z;   /* byte offsets of the FLOAT32 fields */
    int32_t offset_intensity;   /* FLOAT32 intensity offset, -1 = absent (0) */
    int32_t is_bigendian;       /* only little-endian messages are accepted */
    float scan_period;          /* RotaryLidarPreProcess SCAN_PERIOD (0.1 s); <= 0 keeps the intensity */
    float distance_near;        /* DistanceFilter thresholds; both 0 = off (distance_filter.hpp:26-30) */
    float distance_far;
} lmsf_ingest_params;
/* Defaults: velodyne_pointcloud layout (x 0, y 4, z 8, intensity 16, point_step 32), period 0.1, no
 * distance filter. */
lmsf_status lmsf_ingest_params_init(lmsf_ingest_params* p);
/* Decode n points of message data (host or device memory) into xyzi rows at out (host or device
 * memory, cap rows); *n_out = points kept. */
lmsf_status lmsf_ingest_pointcloud2(lmsf_ctx* ctx, const uint8_t* data, size_t n_points, const lmsf_ingest_params* p,
                                    float* out, size_t cap, size_t* n_out);
/* Ingest + lmsf_extract_features in one device pass (the cloud never leaves HBM). */
lmsf_status lmsf_extract_pointcloud2(lmsf_ctx* ctx, const uint8_t* data, size_t n_points, const lmsf_ingest_params* p,
                                     lmsf_feature_counts* counts);

/* ---- 1-NN alignment fitness: Slam3D::PointCloudAlignmentEvaluate (REG/alignEvaluate.hpp:24-95),
 * the loop-closure / relocalisation check (INC/LoopDetection/loopDetection.hpp:176-177, :411, :451;
 * INC/BackEnd/backend_lifelong.hpp:318-319).
 * SetTargetPoints (:42-46): build the target's device neighbour grid (host or device memory). */
lmsf_status lmsf_align_set_target(lmsf_ctx* ctx, const float* xyzi, size_t n);
/* AlignmentScore (:55-87): transform the cloud by relpose (row-major Eigen::Matrix4f, float math),
 * 1-NN squared distance to the target, inliers d2 <= inlier_thresh; *overlap = inliers / n,
 * *score = mean inlier d2 when *overlap > inlier_ratio_thresh, else DBL_MAX (empty cloud: DBL_MAX, 0). */
lmsf_status lmsf_align_score(lmsf_ctx* ctx, const float* xyzi, size_t n, const float relpose[16], double inlier_thresh,
                             double inlier_ratio_thresh, double* score, double* overlap);

/* ---- dual-LiDAR extrinsic initialisation (C3): Algorithm::HandEyeCalibrationBase
 * (INC/Algorithm/calibration/handeye_calibration_base.hpp:36-244) as driven by
 * MultiLidarSystem::process phase 0 (INC/System/ML_System.hpp:268-281).  Host-only arithmetic
 * (no device needed).  Poses are row-major 4x4 inter-frame motions (tracker deltaT outputs). */
typedef struct lmsf_handeye lmsf_handeye;
lmsf_status lmsf_handeye_create(lmsf_handeye** out);
void lmsf_handeye_destroy(lmsf_handeye* h);
/* AddPose (:71-106): *ok = the reference's return value (motion accepted and >= 3 pairs stored). */
lmsf_status lmsf_handeye_add_pose(lmsf_handeye* h, const double primary[16], const double sub[16], int32_t* ok);
/* CalibExRotation (:113-148); singular_values (nullable) = the 4 singular values, descending. */
lmsf_status lmsf_handeye_calib_rotation(lmsf_handeye* h, int32_t* ok, double singular_values[4]);
/* CalibExTranslation (:150-184). */
lmsf_status lmsf_handeye_calib_translation(lmsf_handeye* h, int32_t* ok);
/* GetCalibResult (:187-196): primary <- sub extrinsic. */
lmsf_status lmsf_handeye_result(const lmsf_handeye* h, double T[16], int32_t* ok);
lmsf_status lmsf_handeye_pair_count(const lmsf_handeye* h, int32_t* n);

/* Library version string. */
const char* lmsf_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LMSF_LMSF_H_ */
