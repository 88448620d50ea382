// Device-resident solver control for LOAM registration (one 64-lane workgroup per registration).
//
// Restates, without any host round trip per step, ceres::Solve as configured in
// CeresEdgeSurfFeatureRegistration::Solve (REG/ceres_edgeSurfFeatureRegistration.hpp:107-123:
// TRUST_REGION / LEVENBERG_MARQUARDT, DENSE_QR, max_num_iterations = 4, HuberLoss(0.1),
// PoseSE3Parameterization) on the reduced 6x6 normal equations, and the GN alternative
// EdgeSurfFeatureRegistration::GNOptimization (REG/edgeSurfFeatureRegistration.hpp:218-330).
// Ceres semantics restated (external, Ceres Solver 1.x): jacobi scaling s = 1/(1+sqrt(diag JtJ))
// fixed at the first evaluation; LM diagonal clamp(diag, 1e-6, 1e32)/radius; step valid iff the
// model decrease is positive; parameter tolerance 1e-8, function tolerance 1e-6, gradient
// tolerance 1e-10, min_relative_decrease 1e-3; radius update max(1/3, 1-(2rho-1)^3) on success,
// radius /= mu, mu *= 2 on rejection; initial radius 1e4, max 1e16.
#include <hip/hip_runtime.h>

#include "devmath.h"
#include "lm_control.h"
#include "lmsf_internal.h"

#pragma clang fp contract(off)

namespace lmsf {

struct Pose7 { double x[7]; };

// Initialise slot states from poses (qx qy qz qw tx ty tz): poses [B][7] in device memory, or (p, one slot) a pose
// passed by value -- no upload before the launch
__global__ void state_init_kernel(BatchView bv, const double* poses, Pose7 p) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= bv.B) return;
    SolveState& S = bv.st[b];
    for (int i = 0; i < 7; ++i) S.x[i] = poses ? poses[b * 7 + i] : p.x[i];
    S.inner_total = S.evals_total = S.outer_run = 0;
    S.gn_converged = 0;
    S.done = 1;
    S.need_eval = 0;
    S.iteration = 0;
    S.evals = 0;
    S.term = LMSF_TERM_MAX_ITERATIONS;
    S.initial_cost = S.cost = 0.0;
    S.edge_matches = S.surf_matches = S.nmatch = 0;
}

// After fit_eval: IterationZero (evaluate at x0, jacobi scaling, gradient check) + first step.
// LMSF_CTL_WAVES: waves per SIMD the LM control kernels are compiled for; 0 = the compiler's choice
// (lm_begin 195 VGPRs, lm_step 256).  At 8, lm_begin fits 64 VGPRs (604 B of scratch for its serial lane)
// and finds a slot beside the other contexts' search waves (4 x 121 VGPRs per SIMD) sooner; lm_step
// stays at 256.  A/B on one box (tools/gpu_ab_lib2.sh, C2, alternating): 23.31-23.40k scans/s vs
// 23.14-23.25k at 0; 4 (128 VGPRs, 380 / 576 B scratch) 23.18-23.25k.  C4 within its noise.
#ifndef LMSF_CTL_WAVES
#define LMSF_CTL_WAVES 8
#endif
#if LMSF_CTL_WAVES > 0
#define LMSF_CTL_ATTR __attribute__((amdgpu_waves_per_eu(LMSF_CTL_WAVES)))
#else
#define LMSF_CTL_ATTR
#endif
// LMSF_CTL_MODE (A/B): the batch control kernels' step computation -- 3: on the whole wave (lm_control.h wv::);
// 2: one lane, LDS workspace, rolled loops (no scratch within 64 VGPRs); 1: r03's non-inlined call (868 B of
// scratch); 0: one lane, inlined.
#ifndef LMSF_CTL_MODE
#define LMSF_CTL_MODE 3
#endif
constexpr int kCtlMode = LMSF_CTL_MODE;
__global__ __launch_bounds__(kBeginThreads) LMSF_CTL_ATTR void lm_begin_kernel(BatchView bv) {
    stamp_if(bv.stamp_end, blockIdx.x == 0);   // the search launch before it has drained (single-scan launches)
    const int b = blockIdx.x;
    const int nq = bv.n_edge[b] + bv.n_surf[b];
#ifdef LMSF_STEP_PROFILE
    const unsigned long long t0 = wall_clock64();
#endif
    __shared__ SolveState sS;
    __shared__ double tot[kPacket];
    if (bv.fused_parts) {   // fused path: the memo pass's wave packets (when it ran), then the search's
        reduce_parts(bv, b, bv.memo ? (nq + 63) / 64 : 0, tot, bv.part2_base, (bv.n_search[b] + 63) / 64, &bv.st[b], &sS);
    } else {
        const int fb = bv.part_q;
        reduce_parts(bv, b, (nq + fb - 1) / fb, tot, 0, 0, &bv.st[b], &sS);
    }   // (reduce_parts stages sS and ends with a barrier)
#ifdef LMSF_STEP_PROFILE
    const unsigned long long t1 = wall_clock64();
#endif
    __shared__ double ws[kStepWs];
    if constexpr (kCtlMode == 3) {
        if (threadIdx.x < 64) wv::lm_begin(sS, tot);
    } else if (threadIdx.x == 0) {
        lm_begin_apply<kCtlMode>(sS, tot, ws);
    }
    __syncthreads();
#ifdef LMSF_STEP_PROFILE
    const unsigned long long t2 = wall_clock64();
#endif
    state_copy(bv.st[b], sS);
#ifdef LMSF_STEP_PROFILE
    __syncthreads();
    if (b == 0 && threadIdx.x == 0)
        printf("lm_begin: copy+reduce %llu apply %llu copy-out %llu (x10 ns)\n", t1 - t0, t2 - t1, wall_clock64() - t2);
#endif
}

// After lm_eval_kernel at the candidate: the reduction and lm_step_apply.  kStepThreads: one wave.  Four
// waves sharing the packet loads (A/B r03, tools/gpu_ab_lib.sh, two rounds): C3 1.81 vs 1.52-1.57 ms per
// frame, C4 1.69-1.70 vs 1.64-1.66 ms per scan -- slower: a 4 x 256-VGPR block waits for a whole CU.
#ifndef LMSF_STEP_THREADS
#define LMSF_STEP_THREADS 64
#endif
constexpr int kStepThreads = LMSF_STEP_THREADS;
// LMSF_STEP_RED_U: packet loads in flight per lane in lm_step's reduction (one wave: 61 packets per C2 slot, so 16
// takes two batches where 8 took four)
#ifndef LMSF_STEP_RED_U
#define LMSF_STEP_RED_U 16
#endif
constexpr int kStepRedU = LMSF_STEP_RED_U;
__global__ __launch_bounds__(kStepThreads) void lm_step_kernel(BatchView bv, int outer, int is_last) {
    const int b = blockIdx.x;
    SolveState& S = bv.st[b];
    const int need = S.need_eval, nq = bv.n_edge[b] + bv.n_surf[b];   // one round trip
    if (!need) {
        if (is_last && threadIdx.x == 0) finish_outer(S, outer);
        return;
    }
#ifdef LMSF_STEP_PROFILE   // diagnostics build (tools/build_variant.sh): phase times of slot 0's step
    const unsigned long long t0 = wall_clock64();
#endif
    __shared__ SolveState sS;
    __shared__ double tot[kPacket];
    // the state's copy into LDS rides with the packet loads; ends with a barrier
    reduce_parts<kStepRedU>(bv, b, (nq + kEvalBlock - 1) / kEvalBlock, tot, 0, 0, &S, &sS);
#ifdef LMSF_STEP_PROFILE
    const unsigned long long t1 = wall_clock64();
#endif
    __shared__ double ws[kStepWs];
    if constexpr (kCtlMode == 3) {
        if (threadIdx.x < 64) wv::lm_step(sS, tot, outer, is_last);
    } else if (threadIdx.x == 0) {
        lm_step_apply<kCtlMode>(sS, tot, outer, is_last, ws);
    }
    __syncthreads();
#ifdef LMSF_STEP_PROFILE
    const unsigned long long t2 = wall_clock64();
#endif
    state_copy(S, sS);
#ifdef LMSF_STEP_PROFILE
    __syncthreads();
    if (b == 0 && threadIdx.x == 0)
        printf("lm_step outer %d: copy+reduce %llu apply %llu copy-out %llu (x10 ns)\n", outer, t1 - t0, t2 - t1,
               wall_clock64() - t2);
#endif
}

// ---------------------------------------------------------------- GN (edgeSurfFeatureRegistration)
// gn_accum writes JtJ (upper 21 at [1..21]), JtR ([22..27]) and per-block match counts
// ([29] edge, [30] surf) into partials_gn; fit_eval's own partials carry the per-block counts
// used to rank matches.

__device__ void gn_record_trace(SolveState& S, int outer) {
    if (outer < kMaxOuter)
        for (int i = 0; i < 7; ++i) S.trace[outer][i] = S.x[i];
    S.outer_run = outer + 1;
}

__global__ __launch_bounds__(64) void gn_solve_kernel(BatchView bv, int outer) {
    const int b = blockIdx.x;
    SolveState& S = bv.st[b];
    if (S.gn_converged) return;
    const int nq = bv.n_edge[b] + bv.n_surf[b];
    const int fb = 256 * bv.fit_per_thread;
    const int nparts = (nq + fb - 1) / fb;
    __shared__ double tot[kPacket];
    BatchView g = bv;
    g.partials = bv.partials_gn;
    reduce_parts(g, b, nparts, tot);
    if (threadIdx.x != 0) return;
    S.edge_matches = (int)tot[29];
    S.surf_matches = (int)tot[30];
    const int e16 = (int)(uint16_t)(int)tot[29], s16 = (int)(uint16_t)(int)tot[30];
    S.inner_total += 1;
    if (e16 + s16 < 10) {  // edgeSurf...:221-225: no update this iteration
        S.term = LMSF_TERM_GN_TOO_FEW;
        gn_record_trace(S, outer);
        return;
    }
    double JTJ[36], JTR[6];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) JTJ[i * 6 + j] = tot[1 + (i <= j ? hidx(i, j) : hidx(j, i))];
    for (int i = 0; i < 6; ++i) JTR[i] = tot[22 + i];
    double A[36], nb[6], X[6];
    for (int i = 0; i < 36; ++i) A[i] = JTJ[i];
    for (int i = 0; i < 6; ++i) nb[i] = -JTR[i];
    colpiv_qr_solve<6, 6>(A, nb, X);
    if (outer == 0) {  // degeneracy check at iterCount == 0 (edgeSurf...:280-304)
        double a2[36], d[6], ds[6], Vs[36], V2[36];
        for (int i = 0; i < 36; ++i) a2[i] = JTJ[i];
        saesx<6>(a2, d, Vs);   // SelfAdjointEigenSolver<MatrixXd> (edgeSurf...:282): ascending, sorted
        for (int i = 0; i < 6; ++i) ds[i] = d[i];
        for (int i = 0; i < 36; ++i) V2[i] = Vs[i];
        S.gn_degenerate = 0;
        for (int i = 5; i >= 0; i--) {
            if (ds[i] < 100.0) {
                for (int c = 0; c < 6; ++c) V2[i * 6 + c] = 0.0;   // rows zeroed (:293)
                S.gn_degenerate = 1;
            } else {
                break;
            }
        }
        // Map = V^-1 V2 with V^-1 = V^T (orthogonal eigenvectors; Eigen uses an LU inverse)
        for (int a = 0; a < 6; ++a)
            for (int c = 0; c < 6; ++c) {
                double t = 0.0;
                for (int k = 0; k < 6; ++k) t += Vs[k * 6 + a] * V2[k * 6 + c];
                S.gn_map[a * 6 + c] = t;
            }
    }
    if (S.gn_degenerate) {
        double Y[6];
        for (int a = 0; a < 6; ++a) {
            double t = 0.0;
            for (int k = 0; k < 6; ++k) t += S.gn_map[a * 6 + k] * X[k];
            Y[a] = t;
        }
        for (int a = 0; a < 6; ++a) X[a] = Y[a];
    }
    // t += X[3:6]; q = q * AngleAxis(|dr|/2, dr/|dr|) (edgeSurf...:312-321)
    S.x[4] += X[3]; S.x[5] += X[4]; S.x[6] += X[5];
    const d3 dr = mk(X[0], X[1], X[2]);
    const double drn = norm(dr);
    const d3 axis = drn > 0 ? mk(dr.x / drn, dr.y / drn, dr.z / drn) : dr;
    const double ha = 0.5 * (drn / 2);
    const double sh = sin(ha);
    dq dqq; dqq.x = sh * axis.x; dqq.y = sh * axis.y; dqq.z = sh * axis.z; dqq.w = cos(ha);
    dq q; q.x = S.x[0]; q.y = S.x[1]; q.z = S.x[2]; q.w = S.x[3];
    dq qn = qmul(q, dqq);
    S.x[0] = qn.x; S.x[1] = qn.y; S.x[2] = qn.z; S.x[3] = qn.w;
    const float deltaR = (float)(drn / 2);
    const float deltaT = (float)sqrt(pow(X[3] * 100, 2.0) + pow(X[4] * 100, 2.0) + pow(X[5] * 100, 2.0));
    if (deltaR < 0.0009f && deltaT < 0.05f) {
        S.gn_converged = 1;
        S.term = LMSF_TERM_GN_CONVERGED;
    } else {
        S.term = LMSF_TERM_MAX_ITERATIONS;
    }
    gn_record_trace(S, outer);
}

// GN accumulation: J row = grad^T [-R [p]x, I] (edgeSurf...:255-265) over the first
// (count mod 65536) matches of each kind in query order (uint16_t counters, :58-59).
__global__ __launch_bounds__(256) void gn_accum_kernel(BatchView bv) {
    const int b = blockIdx.y;
    SolveState& S = bv.st[b];
    const int ne = bv.n_edge[b], ns = bv.n_surf[b];
    const int nq = ne + ns;
    const int fb = 256 * bv.fit_per_thread;
    if (blockIdx.x * fb >= nq) return;
    if (S.gn_converged) return;
    __shared__ int wcnt[2][4];
    __shared__ int base_e, base_s;
    __shared__ double red[4][kPacket];
    if (threadIdx.x == 0) {  // matches in earlier blocks (fit_eval's per-block counts)
        double e = 0.0, s = 0.0;
        const double* pb = bv.partials + (size_t)b * bv.max_parts * kPacket;
        for (int p = 0; p < (int)blockIdx.x; ++p) { e += pb[(size_t)p * kPacket + 29]; s += pb[(size_t)p * kPacket + 30]; }
        base_e = (int)e;
        base_s = (int)s;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    double P[kPacket];
    for (int i = 0; i < kPacket; ++i) P[i] = 0.0;
    for (int chunk = 0; chunk < bv.fit_per_thread; ++chunk) {
    const int q = blockIdx.x * fb + chunk * 256 + threadIdx.x;
    const size_t slot = (size_t)b * bv.feat_stride + q;
    const double* gr = bv.gn_rows + slot * 4;
    // unmatched rows carry -1; a matched row's residual is >= 0 or NaN (a degenerate fit, e.g. the edge of two equal
    // points: 0/0), and a NaN row is a match that poisons the normal equations, as in the reference (kind != 0)
    const bool valid = q < nq && !(gr[3] < 0.0);
    const bool is_edge = q < ne;
    __syncthreads();   // previous chunk's wcnt / base reads are complete
    const unsigned long long me = __ballot(valid && is_edge), ms = __ballot(valid && !is_edge);
    if (lane == 0) { wcnt[0][wave] = __popcll(me); wcnt[1][wave] = __popcll(ms); }
    __syncthreads();
    int rank = 0;
    for (int w = 0; w < wave; ++w) rank += is_edge ? wcnt[0][w] : wcnt[1][w];
    rank += __popcll((is_edge ? me : ms) & below) + (is_edge ? base_e : base_s);
    __syncthreads();
    if (threadIdx.x == 0) {
        base_e += wcnt[0][0] + wcnt[0][1] + wcnt[0][2] + wcnt[0][3];
        base_s += wcnt[1][0] + wcnt[1][1] + wcnt[1][2] + wcnt[1][3];
    }
    if (valid && rank < 65536) {
        const float4 p4 = bv.feat[slot];
        const d3 p = mk((double)p4.x, (double)p4.y, (double)p4.z);
        double R[9];
        dq qq; qq.x = S.x[0]; qq.y = S.x[1]; qq.z = S.x[2]; qq.w = S.x[3];
        qmat(qq, R);
        const double sk[9] = {0., -p.z, p.y, p.z, 0., -p.x, -p.y, p.x, 0.};
        double M[9];
        for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c)
                M[a * 3 + c] = (-R[a * 3 + 0]) * sk[0 * 3 + c] + (-R[a * 3 + 1]) * sk[1 * 3 + c] + (-R[a * 3 + 2]) * sk[2 * 3 + c];
        double J[6];
        for (int c = 0; c < 3; ++c) J[c] = gr[0] * M[0 * 3 + c] + gr[1] * M[1 * 3 + c] + gr[2] * M[2 * 3 + c];
        J[3] = gr[0]; J[4] = gr[1]; J[5] = gr[2];
        const double res = gr[3];
        for (int i = 0; i < 6; ++i)
            for (int j = i; j < 6; ++j) P[1 + hidx(i, j)] += J[i] * J[j];
        for (int i = 0; i < 6; ++i) P[22 + i] += J[i] * res;
    }
    if (valid) { if (is_edge) P[29] += 1.0; else P[30] += 1.0; }
    }  // chunk
    for (int i = 0; i < kPacket; ++i) {
        double v = P[i];
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        P[i] = v;
    }
    if (lane == 0)
        for (int i = 0; i < kPacket; ++i) red[wave][i] = P[i];
    __syncthreads();
    if (threadIdx.x < kPacket) {
        const int i = threadIdx.x;
        bv.partials_gn[((size_t)b * bv.max_parts + blockIdx.x) * kPacket + i] =
            ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
    }
}

// Kernel accounting (LMSF_STATS_TIMING): the device's constant-rate wall clock at this point of the
// stream (every earlier kernel of the stream has finished).  Replaces HIP events, whose elapsed time
// is not available for records made by graph nodes on this runtime.
__global__ void stamp_kernel(unsigned long long* out) {
    if (threadIdx.x == 0) out[0] = (unsigned long long)wall_clock64();
}

hipError_t launch_stamp(unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, s, out);
    return hipGetLastError();
}

hipError_t launch_state_init(const BatchView& bv, const double* poses, hipStream_t s) {
    hipLaunchKernelGGL(state_init_kernel, dim3((bv.B + 63) / 64), dim3(64), 0, s, bv, poses, Pose7{});
    return hipGetLastError();
}

hipError_t launch_state_init_pose(const BatchView& bv, const double x[7], hipStream_t s) {
    if (bv.B != 1) return hipErrorInvalidValue;
    Pose7 p;
    for (int i = 0; i < 7; ++i) p.x[i] = x[i];
    hipLaunchKernelGGL(state_init_kernel, dim3(1), dim3(64), 0, s, bv, nullptr, p);
    return hipGetLastError();
}

hipError_t launch_lm_begin(const BatchView& bv, hipStream_t s) {
    hipLaunchKernelGGL(lm_begin_kernel, dim3(bv.B), dim3(kBeginThreads), 0, s, bv);
    return hipGetLastError();
}

hipError_t launch_lm_step(const BatchView& bv, int outer, int is_last, hipStream_t s) {
    hipLaunchKernelGGL(lm_step_kernel, dim3(bv.B), dim3(kStepThreads), 0, s, bv, outer, is_last);
    return hipGetLastError();
}

// Device self-test of the restated SelfAdjointEigenSolver (lmsf_eigen_selfadjoint): one lane per matrix,
// dim 3 = the Matrix3d path of the edge fit, 6 = the MatrixXd path of the GN degeneracy test.
template <int D>
__global__ __launch_bounds__(64) void eigen_selftest_kernel(const double* a, int n, double* d, double* v, int* info) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    double A[D * D], dd[D], V[D * D];
    for (int k = 0; k < D * D; ++k) A[k] = a[(size_t)i * D * D + k];
    int rc;
    if constexpr (D == 3) rc = saes3(A, dd, V);
    else rc = saesx<D>(A, dd, V);
    for (int k = 0; k < D; ++k) d[(size_t)i * D + k] = dd[k];
    for (int k = 0; k < D * D; ++k) v[(size_t)i * D * D + k] = V[k];
    info[i] = rc;
}

hipError_t launch_eigen_selftest(int dim, const double* a, int n, double* d, double* v, int* info, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((n + 63) / 64);
    if (dim == 3) hipLaunchKernelGGL(eigen_selftest_kernel<3>, grid, dim3(64), 0, s, a, n, d, v, info);
    else hipLaunchKernelGGL(eigen_selftest_kernel<6>, grid, dim3(64), 0, s, a, n, d, v, info);
    return hipGetLastError();
}

hipError_t launch_gn_solve(const BatchView& bv, int outer, hipStream_t s) {
    const int fb = 256 * bv.fit_per_thread;
    dim3 grid((bv.feat_stride + fb - 1) / fb, bv.B);
    hipLaunchKernelGGL(gn_accum_kernel, grid, dim3(256), 0, s, bv);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gn_solve_kernel, dim3(bv.B), dim3(64), 0, s, bv, outer);
    return hipGetLastError();
}

}  // namespace lmsf
