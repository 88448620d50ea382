/*
 * lmsf_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of LMSF-Slam's LOAM edge/surface registration hot path, used
 * as the parity checker for the HIP product (tests/, __graft_entry__.smoke(),
 * bench.py cpu_baseline leg only).  Nothing in lmsf-slam_amd/ may include,
 * link or call this library.
 *
 * PARITY STATUS: "parity unpinned" against the real reference.  The reference
 * (PCL KdTreeFLANN, Eigen, Ceres) cannot be compiled in this image (no PCL /
 * FLANN / Eigen / Ceres / ROS headers), it has no golden vectors (its only
 * known-answer test is commented out and reads PCDs that are not in the repo:
 * src/MultiSensorFusionEstimator3D/src/test/registration/feature_registration_test.cpp:56-126),
 * so this restatement is pinned only by independent cross-checks
 * (scipy cKDTree, numpy eigh / lstsq, analytic Jacobians, recovered-transform
 * known-answer tests) committed under tests/golden/.
 *
 * Paths cited below are relative to the reference root; INC = src/MultiSensorFusionEstimator3D/include.
 */
#ifndef LMSF_ORACLE_H_
#define LMSF_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One correspondence; byte-identical layout to lmsf_record in include/lmsf/lmsf.h.
 * kind 0: no match, 1: edge (v0 = a, v1 = b), 2: surf (v0 = unit normal n, v1[0] = D). */
typedef struct {
    float px, py, pz;     /* feature point in the lidar frame (ori_point, ceres_...:148-150, 175-177) */
    int32_t kind;
    double v0[3];
    double v1[3];
} lmsfo_record;

typedef struct {
    int32_t n_scans;          /* N_SCANS_ (LOAMFeatureProcessor_base.hpp:36) */
    float min_distance;       /* 2 in the factory (ML_SystemFactory.hpp:196-197) */
    float max_distance;       /* 80 */
    float edge_threshold;     /* 1 */
    int32_t remove_bad_points;/* true */
    /* Build-defined generalisation for n_scans not in {16,32,64}: uniform beam model
     * scanID = int((angle - beam_lo_deg) / beam_spacing_deg + 0.5).  When
     * beam_spacing_deg <= 0 the reference behaviour is kept (every point -> ring 0,
     * LOAMFeatureProcessor_base.hpp:337-341). */
    double beam_lo_deg;
    double beam_spacing_deg;
    int32_t libm_float;      /* 0: double sqrt / atan2 (GCC 5, kinetic), 1: float overloads (see lmsf.h) */
} lmsfo_extract_params;

/* LOAMFeatureProcessorBase::Process (FX/LOAMFeatureProcessor_base.hpp:59-126).
 * Writes edge / surf points (xyzi, 4 floats each) in the reference emission order,
 * and (optionally) the index of each emitted point in the input array.
 * Returns 0, or -1 when cap is too small. */
int lmsfo_extract(const lmsfo_extract_params* prm, const float* xyzi, int64_t n,
                  float* edge_out, int32_t* edge_src, int64_t* n_edge,
                  float* surf_out, int32_t* surf_src, int64_t* n_surf, int64_t cap);

/* Exact k-NN (FLANN-like single kd-tree, leaf size 15, float L2 without FMA,
 * ties broken by ascending map index). */
typedef struct lmsfo_map lmsfo_map;
lmsfo_map* lmsfo_map_build(const float* xyzi, int64_t n);
void lmsfo_map_free(lmsfo_map* m);
int64_t lmsfo_map_size(const lmsfo_map* m);
/* q: nq points, stride 4 floats. idx/d2: nq*k, sorted ascending; missing -> idx -1, d2 +inf. */
int lmsfo_map_knn(const lmsfo_map* m, const float* q, int64_t nq, int k, int32_t* idx, float* d2);
int lmsfo_brute_knn(const float* map_xyzi, int64_t n, const float* q, int64_t nq, int k,
                    int32_t* idx, float* d2);

/* PointCloud2 decode + removeNaN + rotary relative time + distance filter (oracle/ingest.cpp);
 * out holds up to n points.  Returns the number of points written. */
int64_t lmsfo_ingest(const uint8_t* data, int64_t n, uint32_t step, int32_t ox, int32_t oy, int32_t oz, int32_t oi,
                     float period, float near_t, float far_t, float* out);

/* pcl::VoxelGrid centroid downsampling (oracle/voxel.cpp); out holds up to n points.
 * Returns the number of voxels written. */
int64_t lmsfo_voxel_filter(const float* xyzi, int64_t n, float leaf, float* out);

/* Registration object = CeresEdgeSurfFeatureRegistration (REG/ceres_edgeSurfFeatureRegistration.hpp)
 * or EdgeSurfFeatureRegistration in GN mode (REG/edgeSurfFeatureRegistration.hpp). */
enum { LMSFO_SOLVER_CERES_LM = 0, LMSFO_SOLVER_GN = 1 };
enum { LMSFO_KIND_EDGE = 1, LMSFO_KIND_SURF = 2 };
enum {
    LMSFO_TERM_MAX_ITERATIONS = 0,
    LMSFO_TERM_FUNCTION_TOL = 1,
    LMSFO_TERM_PARAMETER_TOL = 2,
    LMSFO_TERM_GRADIENT_TOL = 3,
    LMSFO_TERM_NO_RESIDUALS = 4,
    LMSFO_TERM_GN_CONVERGED = 5,
    LMSFO_TERM_GN_TOO_FEW = 6
};

typedef struct {
    int32_t outer_iterations;
    int32_t edge_matches;        /* of the last outer iteration */
    int32_t surf_matches;
    int32_t inner_iterations;    /* summed over outer iterations */
    int32_t evaluations;         /* residual evaluations summed over outer iterations */
    int32_t termination;         /* of the last outer iteration */
    double initial_cost;         /* of the last outer iteration */
    double final_cost;
} lmsfo_solve_stats;

typedef struct lmsfo_reg lmsfo_reg;
lmsfo_reg* lmsfo_reg_create(int solver);
void lmsfo_reg_free(lmsfo_reg* r);
/* SetInputSource (map); n == 0 keeps the previous map, as ceres_...:60. */
void lmsfo_reg_set_map(lmsfo_reg* r, int kind, const float* xyzi, int64_t n);
/* SetInputTarget (current scan features). */
void lmsfo_reg_set_scan(lmsfo_reg* r, int kind, const float* xyzi, int64_t n);
void lmsfo_reg_set_max_iterations(lmsfo_reg* r, int n);   /* SetMaxIteration (ceres_...:86-89) */
void lmsfo_reg_set_fixed_schedule(lmsfo_reg* r, int fixed); /* 0: reference decay (ceres_...:100-101) */
/* pose: qx qy qz qw tx ty tz (Eigen storage order, ceres_...:38-40); in = prediction, out = result.
 * trace (nullable): pose after every outer iteration, trace_cap rows of 7. */
int lmsfo_reg_solve(lmsfo_reg* r, double pose[7], double* trace, int trace_cap, lmsfo_solve_stats* st);
/* Matching only, at a given pose: out has n_edge + n_surf records (edges first, then surfs);
 * nn (nullable) receives the 5 map indices per query (-1 when unmatched by kNN). */
int lmsfo_reg_match(lmsfo_reg* r, const double pose[7], lmsfo_record* out, int32_t* nn);
int64_t lmsfo_reg_num_queries(const lmsfo_reg* r);

/* Weighted normal-equation packet at a pose over a record array:
 * out[0] cost (0.5 sum rho), out[1..21] upper-triangular H row-major, out[22..27] g, out[28] count. */
void lmsfo_eval(const lmsfo_record* rec, int64_t n, const double pose[7], double out[29]);

/* PoseSE3Parameterization::Plus (INC/Algorithm/Ceres/Parameterization/PoseSE3Parameterization.hpp:32-46). */
void lmsfo_pose_plus(const double x[7], const double delta[6], double out[7]);

/* Eigen 3.3 SelfAdjointEigenSolver restated (oracle/saes.cpp).  a: n x n row-major symmetric (lower
 * triangle read); d: ascending eigenvalues; v: row-major, eigenvector i in column i.  lmsfo_saes3 is
 * the fixed-size Matrix3d path (EdgeFeatureMatch.hpp:63), lmsfo_saesx the dynamic MatrixXd path
 * (edgeSurfFeatureRegistration.hpp:282), n <= 8.  Returns 0 (Success) or 1 (NoConvergence: unsorted). */
int lmsfo_saes3(const double a[9], double d[3], double v[9]);
int lmsfo_saesx(int n, const double* a, double* d, double* v);

void lmsfo_set_num_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
