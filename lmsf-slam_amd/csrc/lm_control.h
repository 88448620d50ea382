// Device-side Ceres LM control shared by the solver kernels (k_solver.hip) and the fused LM
// evaluation + step kernel (k_match.hip): fixed-order packet reduction, 6x6 Cholesky, the trust-region
// step and the step acceptance, restating ceres::Solve as configured in
// CeresEdgeSurfFeatureRegistration::Solve (REG/ceres_edgeSurfFeatureRegistration.hpp:107-123); see
// k_solver.hip for the Ceres semantics restated.
#pragma once
#include <hip/hip_runtime.h>

#include "devmath.h"
#include "lmsf_internal.h"

namespace lmsf {
constexpr int kBeginThreads = 512;   // lm_begin_kernel block: 8 waves share the packet loads

namespace {

constexpr int kMaxInner = 4;  // options.max_num_iterations (ceres_...:118)

// Sum the packets [0, nparts) and [base2, base2 + n2) of slot b in a fixed order into tot (LDS, valid
// after the closing barrier; entry i summed by thread i, over the waves in wave order).  Wave w, lane l owns entry l % 32 of the packets p = 2 w + l / 32 (mod 2 waves): the
// loads are coalesced and 8 per lane in flight, the two halves add in one shuffle and the waves'
// sums in wave order through LDS.  Every wave of the block loads (lm_begin: kBeginThreads, 1.5k
// packets per slot at C2 -- one wave took 60 us, latency-bound).
// U: loads in flight per lane per batch.  stage_src / stage_dst: the slot's SolveState copied into LDS by the same
// pass, its loads issued ahead of the packet loads (one round trip for both; valid after the closing barrier).
template <int U = 8>
__device__ void reduce_parts(const BatchView& bv, int b, int nparts, double* tot, int base2 = 0, int n2 = 0,
                             const SolveState* stage_src = nullptr, SolveState* stage_dst = nullptr) {
    static_assert(kPacket == 32, "one packet entry per half-wave lane");
    constexpr int kMaxWaves = 16;
    constexpr int kWords = (int)(sizeof(SolveState) / 8);
    constexpr int kStage = 6;   // words per thread (64-thread blocks: sizeof(SolveState) <= 3 KB)
    static_assert(kWords <= 64 * kStage, "SolveState staged by at least one wave");
    __shared__ double red[kMaxWaves][kPacket];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, e = lane & 31;
    long long sw[kStage];
    if (stage_src) {
        const long long* src = reinterpret_cast<const long long*>(stage_src);
#pragma unroll
        for (int j = 0; j < kStage; ++j) {
            const int i = threadIdx.x + j * (int)blockDim.x;
            sw[j] = i < kWords ? src[i] : 0;
        }
    }
    const int nw = min((int)(blockDim.x >> 6), kMaxWaves);
    const int stride = 2 * nw;   // a wave reads two packets per load (one per half-wave)
    double acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = 0.0;
    for (int range = 0; range < 2 && wave < nw; ++range) {   // every thread reaches the barrier
        const int np = range ? n2 : nparts;
        const double* base = bv.partials + ((size_t)b * bv.max_parts + (range ? base2 : 0)) * kPacket;
        // U independent loads in flight per lane, the last batch predicated (a tail of one load per round trip
        // took 7 of lm_step's 11 round trips at C2's 61 packets per slot)
        for (int p = 2 * wave + (lane >> 5); p < np; p += U * stride) {
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = p + u * stride < np ? base[(size_t)(p + u * stride) * kPacket + e] : 0.0;
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += v[u];
        }
    }
    if (stage_src) {
        long long* dst = reinterpret_cast<long long*>(stage_dst);
#pragma unroll
        for (int j = 0; j < kStage; ++j) {
            const int i = threadIdx.x + j * (int)blockDim.x;
            if (i < kWords) dst[i] = sw[j];
        }
    }
    // pairwise tree over the U accumulators (U = 8: ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7)))
#pragma unroll
    for (int h = 1; h < U; h *= 2)
#pragma unroll
        for (int u = 0; u + h < U; u += 2 * h) acc[u] = acc[u] + acc[u + h];
    double v = acc[0];
    v += __shfl_xor(v, 32, 64);
    if (lane < 32 && wave < nw) red[wave][e] = v;
    __syncthreads();
    if (threadIdx.x < kPacket) {
        const int i = threadIdx.x;
        double t = red[0][i];
        for (int w = 1; w < nw; ++w) t += red[w][i];
        tot[i] = t;
    }
    __syncthreads();
}

// A slot's SolveState staged in LDS around the one-lane LM control: every field access of the serial
// step is then an LDS access instead of a dependent global-memory round trip.  Copied in / out by the
// whole block (8-byte words); callers put a barrier between the copy and the lane that uses it.
__device__ __forceinline__ void state_copy(SolveState& dst, const SolveState& src) {
    static_assert(sizeof(SolveState) % 8 == 0, "SolveState copied as 8-byte words");
    const long long* s = reinterpret_cast<const long long*>(&src);
    long long* d = reinterpret_cast<long long*>(&dst);
    for (int i = threadIdx.x; i < (int)(sizeof(SolveState) / 8); i += blockDim.x) d[i] = s[i];
}

__device__ double norm7(const double* x) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 7; ++i) s += x[i] * x[i];
    return sqrt(s);
}

__device__ void pose_plus_lds(const double* x, const double* delta, double* out, double* w);
// grad_max_norm with its Plus in the LDS workspace (MODE 2): ws[0..5] = -g, ws[6..12] = the Plus, ws[13..] its
// matrices
__device__ __forceinline__ double grad_max_norm_lds(const double* x, const double* g, double* ws) {
#pragma unroll 1
    for (int i = 0; i < 6; ++i) ws[i] = -g[i];
    pose_plus_lds(x, ws, ws + 6, ws + 13);
    double m = 0.0;
#pragma unroll 1
    for (int i = 0; i < 7; ++i) m = fmax(m, fabs(x[i] - ws[6 + i]));
    return m;
}

__device__ __forceinline__ double grad_max_norm(const double* x, const double* g) {
    double ng[6], xp[7];
#pragma unroll
    for (int i = 0; i < 6; ++i) ng[i] = -g[i];
    pose_plus(x, ng, xp);
    double m = 0.0;
#pragma unroll
    for (int i = 0; i < 7; ++i) m = fmax(m, fabs(x[i] - xp[i]));
    return m;
}

// Cholesky solve of the 6x6 SPD system in packed lower-triangular storage, in place (A[lidx(i, j)],
// j <= i, becomes L): the arithmetic of the dense version, in 21 doubles instead of 2 x 36 -- the
// one-lane LM control kernels then fit in fewer VGPRs and find a slot beside the search waves sooner.
__device__ __forceinline__ constexpr int lidx(int i, int j) { return i * (i + 1) / 2 + j; }

__device__ __forceinline__ bool chol_solve6(double* A, const double* b, double* x) {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double s = A[lidx(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) s -= A[lidx(j, k)] * A[lidx(j, k)];
        if (!(s > 0.0)) return false;
        const double ljj = sqrt(s);
        A[lidx(j, j)] = ljj;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double t = A[lidx(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) t -= A[lidx(i, k)] * A[lidx(j, k)];
            A[lidx(i, j)] = t / ljj;
        }
    }
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double t = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k) t -= A[lidx(i, k)] * y[k];
        y[i] = t / A[lidx(i, i)];
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double t = y[i];
#pragma unroll
        for (int k = i + 1; k < 6; ++k) t -= A[lidx(k, i)] * x[k];
        x[i] = t / A[lidx(i, i)];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i)
        if (!isfinite(x[i])) return false;
    return true;
}

// ComputeTrustRegionStep + HandleInvalidStep loop: leaves a candidate awaiting evaluation, or
// terminates (max iterations / min radius).
__device__ __forceinline__ void compute_step_body(SolveState& S) {
    while (true) {
        if (S.iteration >= kMaxInner) { S.done = 1; S.term = LMSF_TERM_MAX_ITERATIONS; return; }
        if (S.radius < 1e-32) { S.done = 1; S.term = LMSF_TERM_PARAMETER_TOL; return; }
        ++S.iteration;
        // Hs = D H D (D = diag(s)) and A = Hs + diag(clamp(Hs_ii, 1e-6, 1e32)) / radius, lower triangle
        double A[21], gs[6], nb[6], step[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            gs[i] = S.g[i] * S.s[i];
#pragma unroll
            for (int j = 0; j <= i; ++j) A[lidx(i, j)] = S.H[hidx(j, i)] * S.s[i] * S.s[j];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double hs = S.H[hidx(i, i)] * S.s[i] * S.s[i];
            const double dg = fmin(fmax(hs, 1e-6), 1e32);
            A[lidx(i, i)] = hs + dg / S.radius;
            nb[i] = -gs[i];
        }
        const bool ok = chol_solve6(A, nb, step);
        double mcc = 0.0;
        if (ok) {
            double sg = 0.0, sHs = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                sg += step[i] * gs[i];
                double t = 0.0;
#pragma unroll
                for (int j = 0; j < 6; ++j) t += S.H[i <= j ? hidx(i, j) : hidx(j, i)] * S.s[i] * S.s[j] * step[j];
                sHs += step[i] * t;
            }
            mcc = -(sg + 0.5 * sHs);
        }
        if (!ok || !(mcc > 0.0)) {  // StepIsInvalid == StepRejected(0)
            S.radius = S.radius / S.decrease;
            S.decrease *= 2.0;
            continue;
        }
        double delta[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) delta[i] = step[i] * S.s[i];
        pose_plus(S.x, delta, S.xc);
        S.mcc = mcc;
        S.need_eval = 1;
        return;
    }
}

// CALL: the step computation as a non-inlined call.  lm_step_apply calls it from two places, and the
// inlined copies keep lm_step_kernel at 256 VGPRs + 14 AGPRs (one wave per SIMD, only on a SIMD with at most
// one search wave); as a call it is 84 VGPRs (868 B of stack in the serial lane): 12.4 -> 29 us alone, but
// C2 +0.5-1% (three alternating rounds: 25.67k / 25.93k / 25.68k vs 25.58k / 25.65k / 25.61k scans/s) --
// the batch lm_step waits less for room beside the other contexts' search waves.  The batch lm_begin takes
// the call too (C2 26.14k / 25.88k with it vs 25.85k / 25.84k without); the single-scan lm_loop_kernel keeps
// the inlined form (C4 1,153 / 1,123 vs 1,073 / 1,100 scans/s with the call there as well).
__device__ __noinline__ void compute_step_call(SolveState& S) { compute_step_body(S); }

// The same step with its 6x6 system in an LDS workspace (kStepWs doubles) and the loops rolled: the serial
// lane keeps only a few values in registers, so the control kernels fit 64 VGPRs (they co-reside with four
// search waves per SIMD) with no scratch stack -- the call form above spends its time in 868 B of scratch
// round trips (lm_step 29 us alone vs 12.4 us inlined at 256 VGPRs).  Arithmetic and order are
// compute_step_body's, so the results are bit-identical.
constexpr int kStepWs = 21 + 4 * 6 + 9 + 9 + 7;

// pose_plus (devmath.h) with its 3x3 matrices in the LDS workspace w (25 doubles) and the loops rolled:
// the same operations in the same order.
__device__ void pose_plus_lds(const double* x, const double* delta, double* out, double* w) {
    double* Om = w;
    double* J = w + 9;
    const d3 om = mk(delta[0], delta[1], delta[2]);
    const double theta = norm(om);
    const double half_theta = 0.5 * theta;
    double sin_half, real_factor;
    sincos(half_theta, &sin_half, &real_factor);
    double imag_factor;
    if (theta < 1e-10) {
        const double tsq = theta * theta;
        const double tp4 = tsq * tsq;
        imag_factor = 0.5 - 0.0208333 * tsq + 0.000260417 * tp4;
    } else {
        imag_factor = sin_half / theta;
    }
    dq d;
    d.x = imag_factor * om.x; d.y = imag_factor * om.y; d.z = imag_factor * om.z; d.w = real_factor;
    if (theta < 1e-10) {
        qmat(d, J);
    } else {
        Om[0] = 0.; Om[1] = -om.z; Om[2] = om.y; Om[3] = om.z; Om[4] = 0.; Om[5] = -om.x; Om[6] = -om.y; Om[7] = om.x; Om[8] = 0.;
        double sin_t, cos_t;
        sincos(theta, &sin_t, &cos_t);
        const double c1 = (1 - cos_t) / (theta * theta);
        const double c2 = (theta - sin_t) / cube_rn(theta);
#pragma unroll 1
        for (int i = 0; i < 3; ++i)
#pragma unroll 1
            for (int j = 0; j < 3; ++j) {
                const double o2 = Om[i * 3 + 0] * Om[0 * 3 + j] + Om[i * 3 + 1] * Om[1 * 3 + j] + Om[i * 3 + 2] * Om[2 * 3 + j];
                J[i * 3 + j] = (i == j ? 1.0 : 0.0) + c1 * Om[i * 3 + j] + c2 * o2;
            }
    }
    const d3 up = mk(delta[3], delta[4], delta[5]);
    const d3 dt = mk(J[0] * up.x + J[1] * up.y + J[2] * up.z,
                     J[3] * up.x + J[4] * up.y + J[5] * up.z,
                     J[6] * up.x + J[7] * up.y + J[8] * up.z);
    dq q; q.x = x[0]; q.y = x[1]; q.z = x[2]; q.w = x[3];
    const dq qp = qmul(d, q);
    const d3 tp = rotate(d, mk(x[4], x[5], x[6])) + dt;
    out[0] = qp.x; out[1] = qp.y; out[2] = qp.z; out[3] = qp.w;
    out[4] = tp.x; out[5] = tp.y; out[6] = tp.z;
}
__device__ __noinline__ bool chol_solve6_lds(double* A, const double* b, double* y, double* x) {
#pragma unroll 1
    for (int j = 0; j < 6; ++j) {
        double s = A[lidx(j, j)];
#pragma unroll 1
        for (int k = 0; k < j; ++k) s -= A[lidx(j, k)] * A[lidx(j, k)];
        if (!(s > 0.0)) return false;
        const double ljj = sqrt(s);
        A[lidx(j, j)] = ljj;
#pragma unroll 1
        for (int i = j + 1; i < 6; ++i) {
            double t = A[lidx(i, j)];
#pragma unroll 1
            for (int k = 0; k < j; ++k) t -= A[lidx(i, k)] * A[lidx(j, k)];
            A[lidx(i, j)] = t / ljj;
        }
    }
#pragma unroll 1
    for (int i = 0; i < 6; ++i) {
        double t = b[i];
#pragma unroll 1
        for (int k = 0; k < i; ++k) t -= A[lidx(i, k)] * y[k];
        y[i] = t / A[lidx(i, i)];
    }
#pragma unroll 1
    for (int i = 5; i >= 0; --i) {
        double t = y[i];
#pragma unroll 1
        for (int k = i + 1; k < 6; ++k) t -= A[lidx(k, i)] * x[k];
        x[i] = t / A[lidx(i, i)];
    }
    bool fin = true;
#pragma unroll 1
    for (int i = 0; i < 6; ++i) fin = fin && isfinite(x[i]);
    return fin;
}

__device__ void compute_step_lds(SolveState& S, double* ws) {
    double* A = ws;
    double* gs = ws + 21;
    double* nb = ws + 27;
    double* step = ws + 33;
    double* y = ws + 39;
    while (true) {
        if (S.iteration >= kMaxInner) { S.done = 1; S.term = LMSF_TERM_MAX_ITERATIONS; return; }
        if (S.radius < 1e-32) { S.done = 1; S.term = LMSF_TERM_PARAMETER_TOL; return; }
        ++S.iteration;
#pragma unroll 1
        for (int i = 0; i < 6; ++i) {
            gs[i] = S.g[i] * S.s[i];
#pragma unroll 1
            for (int j = 0; j <= i; ++j) A[lidx(i, j)] = S.H[hidx(j, i)] * S.s[i] * S.s[j];
        }
#pragma unroll 1
        for (int i = 0; i < 6; ++i) {
            const double hs = S.H[hidx(i, i)] * S.s[i] * S.s[i];
            const double dg = fmin(fmax(hs, 1e-6), 1e32);
            A[lidx(i, i)] = hs + dg / S.radius;
            nb[i] = -gs[i];
        }
        const bool ok = chol_solve6_lds(A, nb, y, step);
        double mcc = 0.0;
        if (ok) {
            double sg = 0.0, sHs = 0.0;
#pragma unroll 1
            for (int i = 0; i < 6; ++i) {
                sg += step[i] * gs[i];
                double t = 0.0;
#pragma unroll 1
                for (int j = 0; j < 6; ++j) t += S.H[i <= j ? hidx(i, j) : hidx(j, i)] * S.s[i] * S.s[j] * step[j];
                sHs += step[i] * t;
            }
            mcc = -(sg + 0.5 * sHs);
        }
        if (!ok || !(mcc > 0.0)) {  // StepIsInvalid == StepRejected(0)
            S.radius = S.radius / S.decrease;
            S.decrease *= 2.0;
            continue;
        }
        double* delta = y;   // y is free after the solve
#pragma unroll 1
        for (int i = 0; i < 6; ++i) delta[i] = step[i] * S.s[i];
        pose_plus_lds(S.x, delta, S.xc, ws + 45);
        S.mcc = mcc;
        S.need_eval = 1;
        return;
    }
}

// MODE 0: inlined (registers), 1: non-inlined call, 2: LDS workspace ws (kStepWs doubles), rolled loops
template <int MODE>
__device__ __forceinline__ void compute_step(SolveState& S, double* ws) {
    if constexpr (MODE == 1) compute_step_call(S);
    else if constexpr (MODE == 2) compute_step_lds(S, ws);
    else compute_step_body(S);
}

__device__ void finish_outer(SolveState& S, int outer) {
    if (outer < kMaxOuter)
        for (int i = 0; i < 7; ++i) S.trace[outer][i] = S.x[i];
    S.inner_total += S.iteration;
    S.evals_total += S.evals;
    S.outer_run = outer + 1;
}

// ---------------------------------------------------------------- wave-cooperative LM control (MODE 3)
// The one-lane control above is a chain of dependent operations: ~20 us per step in LDS mode (every access an
// LDS round trip), ~6 us inlined in registers (256 VGPRs).  Here the 64 lanes of one wave share it, each lane
// doing one element's arithmetic in exactly the one-lane order, so the results are bit-identical:
//   * lanes 0..20 hold the packed lower triangle (i, j), lidx(i, j) == lane, of H / the scaled system / L;
//     lanes 0..5 the vectors (s, g, the right-hand side);
//   * Cholesky right-looking: at column k every element (i, j), j > k, subtracts L_ik L_jk -- the same
//     subtractions in the same (ascending k) order as the left-looking loops of chol_solve6; the forward
//     substitution column by column (again ascending k per element); the back substitution (descending rows,
//     ascending k inside a row) on broadcast values;
//   * the Plus of the gradient check (lanes 0..31, at -g) and of the candidate (lanes 32..63, at the step)
//     evaluated side by side in one pass of pose_plus.
// Uniform values are broadcast with readlane (scalar registers), per-lane gathers with ds_bpermute.
namespace wv {
__device__ __forceinline__ double bcast(double v, int src) {   // src: wave-uniform lane index
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double gather(double v, int src) { return __shfl(v, src & 63, 64); }
__device__ __forceinline__ int tri_row(int l) { return (l >= 1) + (l >= 3) + (l >= 6) + (l >= 10) + (l >= 15); }
struct Ctl { double radius, decrease; int iteration; };

// compute_step_body on the wave.  h: this lane's H(i, j) (triangle lanes), sv / gv: s / g of this lane (lanes
// < 6).  True: a candidate step delta (uniform) with model cost change mcc; false: terminated with term.
__device__ __forceinline__ bool compute_step(double h, double sv, double gv, Ctl& c, double delta[6], double& mcc,
                                             int& term) {
    const int lane = __lane_id();
    const bool tri = lane < 21, vec = lane < 6;
    const int ti = tri_row(lane), tj = tri ? lane - ti * (ti + 1) / 2 : 63;
    const double hs = h * gather(sv, ti) * gather(sv, tj);   // Hs = D H D: (H s_i) s_j
    const double gs = gv * sv;
    while (true) {
        if (c.iteration >= kMaxInner) { term = LMSF_TERM_MAX_ITERATIONS; return false; }
        if (c.radius < 1e-32) { term = LMSF_TERM_PARAMETER_TOL; return false; }
        ++c.iteration;
        double a = hs;
        if (tri && ti == tj) a = hs + fmin(fmax(hs, 1e-6), 1e32) / c.radius;
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const double piv = bcast(a, lidx(k, k));
            if (!(piv > 0.0)) { ok = false; break; }
            const double lkk = sqrt(piv);
            if (lane == lidx(k, k)) a = lkk;
            else if (tri && tj == k && ti > k) a = a / lkk;
            const double lik = gather(a, lidx(ti, k)), ljk = gather(a, tri ? lidx(tj, k) : 0);
            if (tri && tj > k) a = a - lik * ljk;
        }
        double st[6];
        if (ok) {
            double t = -gs, y[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                y[k] = bcast(t, k) / bcast(a, lidx(k, k));
                const double lvk = gather(a, vec ? lidx(lane, k) : 0);
                if (vec && lane > k) t = t - lvk * y[k];
            }
#pragma unroll
            for (int i = 5; i >= 0; --i) {
                double u = y[i];
#pragma unroll
                for (int k = i + 1; k < 6; ++k) u -= bcast(a, lidx(k, i)) * st[k];
                st[i] = u / bcast(a, lidx(i, i));
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) ok = ok && isfinite(st[i]);
        }
        mcc = 0.0;
        if (ok) {
            double t = 0.0;   // lane i: sum_j ((H_ij s_i) s_j) step_j
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int r = lane > j ? lane : j, q = lane > j ? j : lane;
                t += gather(h, vec ? lidx(r, q) : 0) * sv * bcast(sv, j) * st[j];
            }
            double sg = 0.0, sHs = 0.0;   // the products step_i gs_i, step_i t_i on broadcast values, in i order
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                sg += st[i] * bcast(gs, i);
                sHs += st[i] * bcast(t, i);
            }
            mcc = -(sg + 0.5 * sHs);
        }
        if (!ok || !(mcc > 0.0)) {   // StepIsInvalid == StepRejected(0)
            c.radius = c.radius / c.decrease;
            c.decrease *= 2.0;
            continue;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) delta[i] = st[i] * bcast(sv, i);
        return true;
    }
}

// The gradient check (if check_grad: max |x - Plus(x, -g)| <= 1e-10 ends the solve) and, unless it ends it,
// the next step -- IterationZero's / HandleSuccessfulStep's tail and StepRejected's re-step.  Updates S's
// control fields from lane 0 (the caller writes nothing else of them afterwards).
__device__ __forceinline__ void grad_then_step(SolveState& S, bool check_grad, const double x[7], double h, double sv,
                                               double gv, Ctl c) {
    const int lane = __lane_id();
    double delta[6] = {0, 0, 0, 0, 0, 0}, mcc = 0.0;
    int term = 0;
    Ctl cs = c;
    const bool stepped = compute_step(h, sv, gv, cs, delta, mcc, term);
    double xo[7];
    double m = 0.0;
    if (check_grad || stepped) {
        double d[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) d[i] = lane < 32 ? -bcast(gv, i) : delta[i];
        pose_plus_inl(x, d, xo);
#pragma unroll
        for (int i = 0; i < 7; ++i) m = fmax(m, fabs(x[i] - xo[i]));
        m = bcast(m, 0);
    }
    if (check_grad && m <= 1e-10) {
        if (lane == 0) { S.done = 1; S.term = LMSF_TERM_GRADIENT_TOL; }
        return;
    }
    if (lane == 0) {
        S.radius = cs.radius;
        S.decrease = cs.decrease;
        S.iteration = cs.iteration;
        if (!stepped) {
            S.done = 1;
            S.term = term;
        } else {
            S.mcc = mcc;
            S.need_eval = 1;
        }
    }
    if (stepped && lane == 32) {
#pragma unroll
        for (int i = 0; i < 7; ++i) S.xc[i] = xo[i];
    }
}

__device__ __forceinline__ double norm7u(const double* x) {   // norm7 of uniform values
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 7; ++i) s += x[i] * x[i];
    return sqrt(s);
}

// lm_step_apply on the wave (S, tot in LDS; all 64 lanes of one wave call it).
__device__ __forceinline__ void lm_step(SolveState& S, const double* tot, int outer, int is_last) {
    const int lane = __lane_id();
    const bool tri = lane < 21, vec = lane < 6;
    const int ti = tri_row(lane), tj = tri ? lane - ti * (ti + 1) / 2 : 0;
    double x[7], xc[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) { x[i] = S.x[i]; xc[i] = S.xc[i]; }
    const double cost = S.cost, mcc = S.mcc, x_norm = S.x_norm;
    Ctl c{S.radius, S.decrease, S.iteration};
    const int evals = S.evals + 1;
    double h = tri ? S.H[hidx(tj, ti)] : 0.0;
    double sv = vec ? S.s[lane] : 0.0, gv = vec ? S.g[lane] : 0.0;
    const double tot_h = tri ? tot[1 + hidx(tj, ti)] : 0.0, tot_g = vec ? tot[22 + lane] : 0.0;
    const double cost_c = isfinite(tot[0]) ? tot[0] : 1.7976931348623157e308;
    double dx[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) dx[i] = x[i] - xc[i];
    if (lane == 0) { S.need_eval = 0; S.evals = evals; }
    bool done = false;
    int term = 0;
    if (norm7u(dx) <= 1e-8 * (x_norm + 1e-8)) {
        done = true;
        term = LMSF_TERM_PARAMETER_TOL;
    } else {
        const double cost_change = cost - cost_c;
        if (fabs(cost_change) <= 1e-6 * cost) {
            done = true;
            term = LMSF_TERM_FUNCTION_TOL;
        } else {
            const double rel = cost_change / mcc;
            if (rel > 1e-3) {
                const double f = 1.0 - cube_rn(2.0 * rel - 1.0);
                c.radius = c.radius / fmax(1.0 / 3.0, f);
                c.radius = fmin(1e16, c.radius);
                c.decrease = 2.0;
#pragma unroll
                for (int i = 0; i < 7; ++i) x[i] = xc[i];
                h = tot_h;
                gv = tot_g;
                if (lane == 0) {
#pragma unroll
                    for (int i = 0; i < 7; ++i) S.x[i] = x[i];
                    S.x_norm = norm7u(x);
                    S.cost = cost_c;
                    S.radius = c.radius;
                    S.decrease = c.decrease;
                }
                if (tri) S.H[hidx(tj, ti)] = h;
                if (vec) S.g[lane] = gv;
                if (c.iteration >= kMaxInner) {
                    done = true;
                    term = LMSF_TERM_MAX_ITERATIONS;
                } else {
                    grad_then_step(S, true, x, h, sv, gv, c);
                }
            } else {
                c.radius = c.radius / c.decrease;
                c.decrease *= 2.0;
                grad_then_step(S, false, x, h, sv, gv, c);
            }
        }
    }
    if (lane == 0) {
        if (done) { S.done = 1; S.term = term; }
        if (is_last) {
            const int it = S.iteration;   // lane 0 wrote it in grad_then_step (same lane: program order)
            if (outer < kMaxOuter)
#pragma unroll
                for (int i = 0; i < 7; ++i) S.trace[outer][i] = x[i];
            S.inner_total += it;
            S.evals_total += evals;
            S.outer_run = outer + 1;
        }
    }
}

// lm_begin_apply on the wave.
__device__ __forceinline__ void lm_begin(SolveState& S, const double* tot) {
    const int lane = __lane_id();
    const bool tri = lane < 21, vec = lane < 6;
    const int ti = tri_row(lane), tj = tri ? lane - ti * (ti + 1) / 2 : 0;
    const double h = tri ? tot[1 + hidx(tj, ti)] : 0.0, gv = vec ? tot[22 + lane] : 0.0;
    const double hjj = vec ? tot[1 + hidx(lane, lane)] : 0.0;
    const int nmatch = (int)tot[28];
    double x[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) x[i] = S.x[i];
    if (lane == 0) {
        S.iteration = 0;
        S.need_eval = 0;
        S.done = 0;
        S.evals = 1;
        S.nmatch = nmatch;
        S.edge_matches = (int)tot[29];
        S.surf_matches = (int)tot[30];
        S.cost = tot[0];
        S.initial_cost = tot[0];
    }
    if (tri) S.H[hidx(tj, ti)] = h;
    if (vec) S.g[lane] = gv;
    if (nmatch == 0) {
        if (lane == 0) { S.done = 1; S.term = LMSF_TERM_NO_RESIDUALS; }
        return;
    }
    const double sv = vec ? 1.0 / (1.0 + sqrt(hjj)) : 0.0;
    if (vec) S.s[lane] = sv;
    if (lane == 0) {
        S.radius = 1e4;
        S.decrease = 2.0;
        S.x_norm = norm7u(x);
    }
    grad_then_step(S, true, x, h, sv, gv, Ctl{1e4, 2.0, 0});
}
}  // namespace wv


// lm_step after the evaluation at the candidate (tot = its reduced packet): step acceptance
// (ParameterToleranceReached, FunctionToleranceReached, IsStepSuccessful, HandleSuccessfulStep /
// StepRejected) + next step; one thread.
template <int MODE = 0>
__device__ __forceinline__ void lm_step_apply(SolveState& S, const double* tot, int outer, int is_last, double* ws = nullptr) {
    S.need_eval = 0;
    ++S.evals;
    const double cost_c = isfinite(tot[0]) ? tot[0] : 1.7976931348623157e308;
    double dx[7];
    for (int i = 0; i < 7; ++i) dx[i] = S.x[i] - S.xc[i];
    if (norm7(dx) <= 1e-8 * (S.x_norm + 1e-8)) {
        S.done = 1;
        S.term = LMSF_TERM_PARAMETER_TOL;
    } else {
        const double cost_change = S.cost - cost_c;
        if (fabs(cost_change) <= 1e-6 * S.cost) {
            S.done = 1;
            S.term = LMSF_TERM_FUNCTION_TOL;
        } else {
            const double rel = cost_change / S.mcc;
            if (rel > 1e-3) {
                const double f = 1.0 - cube_rn(2.0 * rel - 1.0);   // pow(2 rel - 1, 3), correctly rounded
                S.radius = S.radius / fmax(1.0 / 3.0, f);
                S.radius = fmin(1e16, S.radius);
                S.decrease = 2.0;
                for (int i = 0; i < 7; ++i) S.x[i] = S.xc[i];
                S.x_norm = norm7(S.x);
                S.cost = cost_c;
                for (int i = 0; i < 21; ++i) S.H[i] = tot[1 + i];
                for (int i = 0; i < 6; ++i) S.g[i] = tot[22 + i];
                if (S.iteration >= kMaxInner) {
                    S.done = 1;
                    S.term = LMSF_TERM_MAX_ITERATIONS;
                } else if ((MODE == 2 ? grad_max_norm_lds(S.x, S.g, ws) : grad_max_norm(S.x, S.g)) <= 1e-10) {
                    S.done = 1;
                    S.term = LMSF_TERM_GRADIENT_TOL;
                } else {
                    compute_step<MODE>(S, ws);
                }
            } else {
                S.radius = S.radius / S.decrease;
                S.decrease *= 2.0;
                compute_step<MODE>(S, ws);
            }
        }
    }
    if (is_last) finish_outer(S, outer);
}

// IterationZero on the reduced first evaluation (tot) + the first step; one lane, S in LDS.
template <int MODE = 0>
__device__ __forceinline__ void lm_begin_apply(SolveState& S, const double* tot, double* ws = nullptr) {
    S.iteration = 0;
    S.need_eval = 0;
    S.done = 0;
    S.evals = 1;
    S.nmatch = (int)tot[28];
    S.edge_matches = (int)tot[29];
    S.surf_matches = (int)tot[30];
    S.cost = tot[0];
    S.initial_cost = tot[0];
    for (int i = 0; i < 21; ++i) S.H[i] = tot[1 + i];
    for (int i = 0; i < 6; ++i) S.g[i] = tot[22 + i];
    if (S.nmatch == 0) {  // no residual blocks: pose unchanged
        S.done = 1;
        S.term = LMSF_TERM_NO_RESIDUALS;
        return;
    }
    for (int j = 0; j < 6; ++j) S.s[j] = 1.0 / (1.0 + sqrt(S.H[hidx(j, j)]));
    S.radius = 1e4;
    S.decrease = 2.0;
    S.x_norm = norm7(S.x);
    if ((MODE == 2 ? grad_max_norm_lds(S.x, S.g, ws) : grad_max_norm(S.x, S.g)) <= 1e-10) {
        S.done = 1;
        S.term = LMSF_TERM_GRADIENT_TOL;
        return;
    }
    compute_step<MODE>(S, ws);
}

}  // namespace
}  // namespace lmsf
