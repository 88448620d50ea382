// Device-side math of the registration path (gfx950).  Operation order follows the reference's
// Eigen / Ceres expressions literally (cited per function) so that, with FP contraction off,
// IEEE double results agree bit-for-bit with any CPU evaluation of the same expressions.
// REG = src/MultiSensorFusionEstimator3D/include/Algorithm/PointClouds/registration,
// INC = src/MultiSensorFusionEstimator3D/include.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace lmsf {

struct d3 { double x, y, z; };

__device__ __forceinline__ d3 mk(double x, double y, double z) { d3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ d3 operator+(d3 a, d3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ d3 operator-(d3 a, d3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ d3 smul(double s, d3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ d3 cross(d3 a, d3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double sqnorm(d3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ double norm(d3 a) { return sqrt(sqnorm(a)); }

struct dq { double x, y, z, w; };

// Eigen Quaternion::_transformVector: uv = q.vec x v; uv += uv; v + w*uv + q.vec x uv
__device__ __forceinline__ d3 rotate(const dq& q, d3 v) {
    d3 qv = mk(q.x, q.y, q.z);
    d3 uv = cross(qv, v);
    uv = uv + uv;
    d3 c = cross(qv, uv);
    return mk(v.x + q.w * uv.x + c.x, v.y + q.w * uv.y + c.y, v.z + q.w * uv.z + c.z);
}
// Eigen quat_product
__device__ __forceinline__ dq qmul(const dq& a, const dq& b) {
    dq r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}
// Eigen toRotationMatrix
__device__ __forceinline__ void qmat(const dq& q, double R[9]) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

struct Pose { dq q; d3 t; };
__device__ __forceinline__ Pose load_pose(const double* x) {
    Pose p;
    p.q.x = x[0]; p.q.y = x[1]; p.q.z = x[2]; p.q.w = x[3];
    p.t = mk(x[4], x[5], x[6]);
    return p;
}
__device__ __forceinline__ d3 transform(const Pose& P, d3 p) { return rotate(P.q, p) + P.t; }

// x^3 correctly rounded (the value glibc's pow(x, 3) returns; two error-free products, then the double-double
// sum rounded once): 7 VALU instead of ocml pow's ~300 on the serial LM-control lane
__device__ __forceinline__ double cube_rn(double x) {
    const double p = x * x;
    const double pe = fma(x, x, -p);   // x^2 = p + pe exactly
    const double h = p * x;
    const double he = fma(p, x, -h);   // p x = h + he exactly
    return h + (he + pe * x);
}

// Math::GetTransformFromSe3 (INC/Math.hpp:29-72) + PoseSE3Parameterization::Plus
// (INC/Algorithm/Ceres/Parameterization/PoseSE3Parameterization.hpp:32-46).  sin / cos of one argument come
// from one sincos (one range reduction), pow(theta, 3) is cube_rn.
__device__ __forceinline__ void pose_plus_inl(const double* x, const double* delta, double* out) {
    d3 om = mk(delta[0], delta[1], delta[2]);
    d3 up = mk(delta[3], delta[4], delta[5]);
    double theta = norm(om);
    double half_theta = 0.5 * theta;
    double sin_half, real_factor;
    sincos(half_theta, &sin_half, &real_factor);
    double imag_factor;
    if (theta < 1e-10) {
        double tsq = theta * theta;
        double tp4 = tsq * tsq;
        imag_factor = 0.5 - 0.0208333 * tsq + 0.000260417 * tp4;
    } else {
        imag_factor = sin_half / theta;
    }
    dq d;
    d.x = imag_factor * om.x; d.y = imag_factor * om.y; d.z = imag_factor * om.z; d.w = real_factor;
    double J[9];
    if (theta < 1e-10) {
        qmat(d, J);
    } else {
        const double Om[9] = {0., -om.z, om.y, om.z, 0., -om.x, -om.y, om.x, 0.};
        double sin_t, cos_t;
        sincos(theta, &sin_t, &cos_t);
        double c1 = (1 - cos_t) / (theta * theta);
        double c2 = (theta - sin_t) / cube_rn(theta);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                double o2 = Om[i * 3 + 0] * Om[0 * 3 + j] + Om[i * 3 + 1] * Om[1 * 3 + j] + Om[i * 3 + 2] * Om[2 * 3 + j];
                J[i * 3 + j] = (i == j ? 1.0 : 0.0) + c1 * Om[i * 3 + j] + c2 * o2;
            }
    }
    d3 dt = mk(J[0] * up.x + J[1] * up.y + J[2] * up.z,
               J[3] * up.x + J[4] * up.y + J[5] * up.z,
               J[6] * up.x + J[7] * up.y + J[8] * up.z);
    dq q; q.x = x[0]; q.y = x[1]; q.z = x[2]; q.w = x[3];
    dq qp = qmul(d, q);
    d3 tp = rotate(d, mk(x[4], x[5], x[6])) + dt;
    out[0] = qp.x; out[1] = qp.y; out[2] = qp.z; out[3] = qp.w;
    out[4] = tp.x; out[5] = tp.y; out[6] = tp.z;
}
__device__ inline void pose_plus(const double* x, const double* delta, double* out) { pose_plus_inl(x, delta, out); }

// ---------------------------------------------------------------- SelfAdjointEigenSolver (Eigen 3.3)
// Eigen's published algorithm (Eigenvalues/SelfAdjointEigenSolver.h, Tridiagonalization.h, Jacobi.h),
// restated for the two call sites of the reference: the fixed-size Matrix3d edge PCA
// (EdgeFeatureMatch.hpp:63) and the dynamic MatrixXd degeneracy test of the GN variant
// (edgeSurfFeatureRegistration.hpp:282).  compute(): lower triangle scaled into [-1, 1] by its largest
// magnitude, tridiagonalised (3x3: one closed-form Householder step), implicit symmetric QR steps with a
// Wilkinson shift on the trailing unreduced block (deflation |e| <= 2 eps (|d_i| + |d_i+1|) or
// |e| <= DBL_MIN, at most 30 n steps), the rotations accumulated into Q on the right, then a selection
// sort ascending with column swaps (only when converged), eigenvalues scaled back.

// numext::hypot: p = max(|x|, |y|), p sqrt(1 + (min / p)^2)
__device__ __forceinline__ double eigen_hypot(double x, double y) {
    const double ax = fabs(x), ay = fabs(y);
    const double p = ax > ay ? ax : ay;
    const double qp = (ax > ay ? ay : ax) / p;
    return p == 0.0 ? 0.0 : p * sqrt(1.0 + qp * qp);
}

// JacobiRotation<double>::makeGivens(p, q), real case: G = [c s; -s c], G^T [p; q] = [r; 0]
__device__ __forceinline__ void make_givens(double p, double q, double& c, double& s) {
    if (q == 0.0) {
        c = p < 0.0 ? -1.0 : 1.0;
        s = 0.0;
    } else if (p == 0.0) {
        c = 0.0;
        s = q < 0.0 ? 1.0 : -1.0;
    } else if (fabs(p) > fabs(q)) {
        const double t = q / p;
        double u = sqrt(1.0 + t * t);
        if (p < 0.0) u = -u;
        c = 1.0 / u;
        s = -t * c;
    } else {
        const double t = p / q;
        double u = sqrt(1.0 + t * t);
        if (q < 0.0) u = -u;
        s = -1.0 / u;
        c = -t * s;
    }
}

// tridiagonal_qr_step's Wilkinson shift from (diag[end-1], diag[end], sub[end-1])
__device__ __forceinline__ double wilkinson_shift(double da, double db, double e) {
    const double td = (da - db) * 0.5;
    double mu = db;
    if (td == 0.0) {
        mu -= fabs(e);
    } else {
        const double e2 = e * e;
        const double h = eigen_hypot(td, e);
        if (e2 == 0.0)
            mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / h);
        else
            mu -= e2 / (td + (td > 0.0 ? h : -h));
    }
    return mu;
}

// One bulge-chasing rotation of tridiagonal_qr_step at k on (diag[k], diag[k+1], sub[k]): G^T T G.
__device__ __forceinline__ void qr_rotate(double c, double s, double& dk, double& dk1, double& ek) {
    const double sdk = s * dk + c * ek;
    const double dkp1 = s * ek + c * dk1;
    const double nk = c * (c * dk - s * ek) - s * (c * ek - s * dk1);
    dk1 = s * sdk + c * dkp1;
    ek = c * sdk - s * dkp1;
    dk = nk;
}
// Q = Q * G on columns (k, k+1): applyOnTheRight(k, k+1, rot)
__device__ __forceinline__ void q_rotate(double c, double s, double& a, double& b) {
    const double xi = a, yi = b;
    a = c * xi - s * yi;
    b = s * xi + c * yi;
}
__device__ __forceinline__ bool eig_negligible(double e, double da, double db) {
    return fabs(e) <= (fabs(da) + fabs(db)) * (2.0 * 2.220446049250313e-16) || fabs(e) <= 2.2250738585072014e-308;
}

// SelfAdjointEigenSolver<Matrix3d>(A).  A row-major (lower triangle read).  Out: d ascending,
// V row-major with eigenvector i in column i.  Every index static (registers only).  Returns 0
// (Success) or 1 (NoConvergence: left unsorted, as Eigen does).
__device__ inline int saes3(const double* A, double d[3], double V[9]) {
    double m00 = A[0], m10 = A[3], m20 = A[6], m11 = A[4], m21 = A[7], m22 = A[8];
    double scale = 0.0;
    scale = fabs(m00) > scale ? fabs(m00) : scale;
    scale = fabs(m10) > scale ? fabs(m10) : scale;
    scale = fabs(m20) > scale ? fabs(m20) : scale;
    scale = fabs(m11) > scale ? fabs(m11) : scale;
    scale = fabs(m21) > scale ? fabs(m21) : scale;
    scale = fabs(m22) > scale ? fabs(m22) : scale;
    if (scale == 0.0) scale = 1.0;
    m00 /= scale; m10 /= scale; m20 /= scale; m11 /= scale; m21 /= scale; m22 /= scale;
    // tridiagonalization_inplace_selector<MatrixType, 3, false>
    double d0 = m00, d1, d2, e0, e1;
    double q00 = 1.0, q01 = 0.0, q02 = 0.0, q10 = 0.0, q11, q12, q20 = 0.0, q21, q22;
    const double v1norm2 = m20 * m20;
    if (v1norm2 <= 2.2250738585072014e-308) {
        d1 = m11; d2 = m22; e0 = m10; e1 = m21;
        q11 = 1.0; q12 = 0.0; q21 = 0.0; q22 = 1.0;
    } else {
        const double beta = sqrt(m10 * m10 + v1norm2);
        const double inv_beta = 1.0 / beta;
        const double m01 = m10 * inv_beta, m02 = m20 * inv_beta;
        const double q = 2.0 * m01 * m21 + m02 * (m22 - m11);
        d1 = m11 + m02 * q;
        d2 = m22 - m02 * q;
        e0 = beta;
        e1 = m21 - m01 * q;
        q11 = m01; q12 = m02; q21 = m02; q22 = -m01;
    }
    // computeFromTridiagonal_impl
    int end = 2, start = 0, iter = 0;
    while (true) {
        if (start <= 0 && end > 0 && eig_negligible(e0, d0, d1)) e0 = 0.0;
        if (start <= 1 && end > 1 && eig_negligible(e1, d1, d2)) e1 = 0.0;
        if (end == 2 && e1 == 0.0) end = 1;
        if (end == 1 && e0 == 0.0) end = 0;
        if (end == 0) break;
        if (++iter > 90) break;
        start = (end == 2 && e0 != 0.0) ? 0 : end - 1;
        const double mu = end == 2 ? wilkinson_shift(d1, d2, e1) : wilkinson_shift(d0, d1, e0);
        double c, s;
        if (start == 0) {
            make_givens(d0 - mu, e0, c, s);
            qr_rotate(c, s, d0, d1, e0);
            q_rotate(c, s, q00, q01); q_rotate(c, s, q10, q11); q_rotate(c, s, q20, q21);
            if (end == 2) {
                const double z = -s * e1;       // the bulge
                e1 = c * e1;
                make_givens(e0, z, c, s);
                qr_rotate(c, s, d1, d2, e1);
                e0 = c * e0 - s * z;
                q_rotate(c, s, q01, q02); q_rotate(c, s, q11, q12); q_rotate(c, s, q21, q22);
            }
        } else {   // start == 1, end == 2
            make_givens(d1 - mu, e1, c, s);
            qr_rotate(c, s, d1, d2, e1);
            q_rotate(c, s, q01, q02); q_rotate(c, s, q11, q12); q_rotate(c, s, q21, q22);
        }
    }
    const int info = iter > 90 ? 1 : 0;
    if (!info) {
        // i = 0: first index of min(d0, d1, d2); i = 1: min(d1, d2)
        if (d1 < d0 && !(d2 < d1)) {
            double t = d0; d0 = d1; d1 = t;
            t = q00; q00 = q01; q01 = t; t = q10; q10 = q11; q11 = t; t = q20; q20 = q21; q21 = t;
        } else if (d2 < d0 && d2 < d1) {
            double t = d0; d0 = d2; d2 = t;
            t = q00; q00 = q02; q02 = t; t = q10; q10 = q12; q12 = t; t = q20; q20 = q22; q22 = t;
        }
        if (d2 < d1) {
            double t = d1; d1 = d2; d2 = t;
            t = q01; q01 = q02; q02 = t; t = q11; q11 = q12; q12 = t; t = q21; q21 = q22; q22 = t;
        }
    }
    d[0] = d0 * scale; d[1] = d1 * scale; d[2] = d2 * scale;
    V[0] = q00; V[1] = q01; V[2] = q02; V[3] = q10; V[4] = q11; V[5] = q12; V[6] = q20; V[7] = q21; V[8] = q22;
    return info;
}

// SelfAdjointEigenSolver<MatrixXd>(A), N x N (one lane, runtime loops: the GN degeneracy test runs once
// per Solve).  Householder tridiagonalisation (makeHouseholderInPlace, SYMV of the lower triangle,
// rank-2 update) in plain sequential order (Eigen's packet kernels sum in another order: agreement to
// rounding), Q from the Householder sequence, then the same QR iteration and sort as saes3.
template <int N>
__device__ inline int saesx(const double* A, double* d, double* V) {
    double M[N * N];
    double scale = 0.0;
    for (int r = 0; r < N; ++r)
        for (int c = 0; c < N; ++c) {
            M[r * N + c] = c <= r ? A[r * N + c] : 0.0;
            scale = fabs(M[r * N + c]) > scale ? fabs(M[r * N + c]) : scale;
        }
    if (scale == 0.0) scale = 1.0;
    for (int r = 0; r < N; ++r)
        for (int c = 0; c <= r; ++c) M[r * N + c] /= scale;
    double hc[N];
    for (int i = 0; i < N - 1; ++i) {
        const int rem = N - i - 1;
        double* col = M + (i + 1) * N + i;
        const double c0 = col[0];
        double tail = 0.0;
        for (int r = 1; r < rem; ++r) tail += col[r * N] * col[r * N];
        double tau, beta;
        if (tail <= 2.2250738585072014e-308) {
            tau = 0.0;
            beta = c0;
            for (int r = 1; r < rem; ++r) col[r * N] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            for (int r = 1; r < rem; ++r) col[r * N] = col[r * N] / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        col[0] = 1.0;
        double w[N], hv[N];
        for (int r = 0; r < rem; ++r) hv[r] = tau * col[r * N];
        for (int r = 0; r < rem; ++r) {
            double s = 0.0;
            for (int c = 0; c < rem; ++c) {
                const int R = i + 1 + (r > c ? r : c), Cc = i + 1 + (r > c ? c : r);
                s += M[R * N + Cc] * hv[c];
            }
            w[r] = s;
        }
        double dt = 0.0;
        for (int r = 0; r < rem; ++r) dt += w[r] * col[r * N];
        const double alpha = tau * -0.5 * dt;
        for (int r = 0; r < rem; ++r) w[r] += alpha * col[r * N];
        for (int c = 0; c < rem; ++c)
            for (int r = c; r < rem; ++r)
                M[(i + 1 + r) * N + (i + 1 + c)] += (-1.0 * col[c * N]) * w[r] + (-1.0 * w[c]) * col[r * N];
        col[0] = beta;
        hc[i] = tau;
    }
    double dg[N], sb[N];
    for (int i = 0; i < N; ++i) dg[i] = M[i * N + i];
    for (int i = 0; i < N - 1; ++i) sb[i] = M[(i + 1) * N + i];
    for (int r = 0; r < N; ++r)
        for (int c = 0; c < N; ++c) V[r * N + c] = r == c ? 1.0 : 0.0;
    for (int k = N - 2; k >= 0; --k) {
        const int o = k + 1, cs = N - k - 1;
        const double tau = hc[k];
        if (cs == 1) {
            V[o * N + o] *= (1.0 - tau);
        } else if (tau != 0.0) {
            for (int c = o; c < N; ++c) {
                double tmp = 0.0;
                for (int r = 1; r < cs; ++r) tmp += M[(o + r) * N + k] * V[(o + r) * N + c];
                tmp += V[o * N + c];
                V[o * N + c] -= tau * tmp;
                for (int r = 1; r < cs; ++r) V[(o + r) * N + c] -= (tau * M[(o + r) * N + k]) * tmp;
            }
        }
    }
    int end = N - 1, start = 0, iter = 0;
    while (end > 0) {
        for (int i = start; i < end; ++i)
            if (eig_negligible(sb[i], dg[i], dg[i + 1])) sb[i] = 0.0;
        while (end > 0 && sb[end - 1] == 0.0) end--;
        if (end <= 0) break;
        if (++iter > 30 * N) break;
        start = end - 1;
        while (start > 0 && sb[start - 1] != 0.0) start--;
        const double mu = wilkinson_shift(dg[end - 1], dg[end], sb[end - 1]);
        double x = dg[start] - mu, z = sb[start];
        for (int k = start; k < end; ++k) {
            double c, s;
            make_givens(x, z, c, s);
            qr_rotate(c, s, dg[k], dg[k + 1], sb[k]);
            if (k > start) sb[k - 1] = c * sb[k - 1] - s * z;
            x = sb[k];
            if (k < end - 1) {
                z = -s * sb[k + 1];
                sb[k + 1] = c * sb[k + 1];
            }
            for (int r = 0; r < N; ++r) q_rotate(c, s, V[r * N + k], V[r * N + k + 1]);
        }
    }
    const int info = iter > 30 * N ? 1 : 0;
    if (!info) {
        for (int i = 0; i < N - 1; ++i) {
            int k = 0;
            for (int j = 1; j < N - i; ++j)
                if (dg[i + j] < dg[i + k]) k = j;
            if (k > 0) {
                const double t = dg[i]; dg[i] = dg[i + k]; dg[i + k] = t;
                for (int r = 0; r < N; ++r) {
                    const double u = V[r * N + i]; V[r * N + i] = V[r * N + i + k]; V[r * N + i + k] = u;
                }
            }
        }
    }
    for (int i = 0; i < N; ++i) d[i] = dg[i] * scale;
    return info;
}

// ---------------------------------------------------------------- ColPivHouseholderQR solve
// Eigen computeInPlace + _solve_impl restated (surfFeatureMatch.hpp:52, edgeSurf...:272).
// A is MxN row-major in registers (compile-time M, N), b length M, x length N.
template <int M, int N>
__device__ inline void colpiv_qr_solve(double* A, const double* b, double* x) {
    const double eps = 2.220446049250313e-16;
    const double dmin = 2.2250738585072014e-308;
    double cn_upd[N], cn_dir[N], hc[N];
    int perm[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) s += A[i * N + j] * A[i * N + j];
        cn_upd[j] = cn_dir[j] = sqrt(s);
        perm[j] = j;
    }
    double maxcn = cn_upd[0];
#pragma unroll
    for (int j = 1; j < N; ++j) maxcn = fmax(maxcn, cn_upd[j]);
    double thr_helper = (maxcn * eps) * (maxcn * eps) / (double)M;
    const double downdate_thr = 1.4901161193847656e-08;  // sqrt(eps)
    constexpr int SIZE = M < N ? M : N;
    int nonzero = SIZE;
#pragma unroll
    for (int k = 0; k < SIZE; ++k) {
        int big = k;
        double bigv = cn_upd[k];
#pragma unroll
        for (int j = k + 1; j < N; ++j)
            if (cn_upd[j] > bigv) { big = j; bigv = cn_upd[j]; }
        double big_sq = bigv * bigv;
        if (nonzero == SIZE && big_sq < thr_helper * (double)(M - k)) nonzero = k;
        // swap column k <-> big (static indices, runtime predicate)
#pragma unroll
        for (int j = k + 1; j < N; ++j) {
            if (j == big) {
#pragma unroll
                for (int i = 0; i < M; ++i) { double t = A[i * N + k]; A[i * N + k] = A[i * N + j]; A[i * N + j] = t; }
                double t1 = cn_upd[k]; cn_upd[k] = cn_upd[j]; cn_upd[j] = t1;
                double t2 = cn_dir[k]; cn_dir[k] = cn_dir[j]; cn_dir[j] = t2;
                int t3 = perm[k]; perm[k] = perm[j]; perm[j] = t3;
            }
        }
        double c0 = A[k * N + k];
        double tail = 0.0;
#pragma unroll
        for (int i = k + 1; i < M; ++i) tail += A[i * N + k] * A[i * N + k];
        double tau, beta;
        if (tail <= dmin) {
            tau = 0.0;
            beta = c0;
#pragma unroll
            for (int i = k + 1; i < M; ++i) A[i * N + k] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
#pragma unroll
            for (int i = k + 1; i < M; ++i) A[i * N + k] = A[i * N + k] / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        A[k * N + k] = beta;
        hc[k] = tau;
        if (k + 1 < N) {
            if (M - k == 1) {
#pragma unroll
                for (int j = k + 1; j < N; ++j) A[k * N + j] *= (1.0 - tau);
            } else if (tau != 0.0) {
#pragma unroll
                for (int j = k + 1; j < N; ++j) {
                    double tmp = 0.0;
#pragma unroll
                    for (int i = k + 1; i < M; ++i) tmp += A[i * N + k] * A[i * N + j];
                    tmp += A[k * N + j];
                    A[k * N + j] -= tau * tmp;
#pragma unroll
                    for (int i = k + 1; i < M; ++i) A[i * N + j] -= (tau * A[i * N + k]) * tmp;
                }
            }
        }
#pragma unroll
        for (int j = k + 1; j < N; ++j) {
            if (cn_upd[j] != 0.0) {
                double temp = fabs(A[k * N + j]) / cn_upd[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                // at k = 0 both norms are still the one computed value (swapped together): x / x = 1 exactly
                double r = k == 0 ? 1.0 : cn_upd[j] / cn_dir[j];
                double temp2 = temp * r * r;
                if (temp2 <= downdate_thr) {
                    double s = 0.0;
#pragma unroll
                    for (int i = k + 1; i < M; ++i) s += A[i * N + j] * A[i * N + j];
                    cn_dir[j] = sqrt(s);
                    cn_upd[j] = cn_dir[j];
                } else {
                    cn_upd[j] *= sqrt(temp);
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] = 0.0;
    if (nonzero == 0) return;
    double c[M];
#pragma unroll
    for (int i = 0; i < M; ++i) c[i] = b[i];
#pragma unroll
    for (int k = 0; k < SIZE; ++k) {
        if (k < nonzero) {
            double tau = hc[k];
            if (M - k == 1) {
                c[k] *= (1.0 - tau);
            } else if (tau != 0.0) {
                double tmp = 0.0;
#pragma unroll
                for (int i = k + 1; i < M; ++i) tmp += A[i * N + k] * c[i];
                tmp += c[k];
                c[k] -= tau * tmp;
#pragma unroll
                for (int i = k + 1; i < M; ++i) c[i] -= (tau * A[i * N + k]) * tmp;
            }
        }
    }
#pragma unroll
    for (int i = SIZE - 1; i >= 0; --i) {
        if (i < nonzero) {
            c[i] = c[i] / A[i * N + i];
#pragma unroll
            for (int r = 0; r < i; ++r) c[r] -= c[i] * A[r * N + i];
        }
    }
#pragma unroll
    for (int i = 0; i < SIZE; ++i) {
        if (i < nonzero) {
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (perm[i] == j) x[j] = c[i];
        }
    }
}

// ---------------------------------------------------------------- residuals / Jacobians
// Upper-triangular 6x6 index (row-major).
__host__ __device__ constexpr int hidx(int i, int j) { return i * 6 - i * (i - 1) / 2 + (j - i); }

// se3PointEdgeFactor::Evaluate (REG/ceres_factor/edge_factor.hpp:33-61), 6 local columns.
// |nu| == 0 yields NaN in the reference; the Jacobian is zero here (documented deviation).
__device__ __forceinline__ double edge_residual(const Pose& P, d3 p, d3 a, d3 b, double* J) {
    d3 lp = transform(P, p);
    d3 nu = cross(lp - a, lp - b);
    d3 de = a - b;
    double de_norm = norm(de);
    double nu_norm = norm(nu);
    double res = nu_norm / de_norm;
    if (nu_norm > 0) {
        double wx = -nu.x / nu_norm, wy = -nu.y / nu_norm, wz = -nu.z / nu_norm;
        double r0 = wy * de.z + wz * (-de.y);
        double r1 = wx * (-de.z) + wz * de.x;
        double r2 = wx * de.y + wy * (-de.x);
        J[0] = (r1 * (-lp.z) + r2 * lp.y) / de_norm;
        J[1] = (r0 * lp.z + r2 * (-lp.x)) / de_norm;
        J[2] = (r0 * (-lp.y) + r1 * lp.x) / de_norm;
        J[3] = r0 / de_norm;
        J[4] = r1 / de_norm;
        J[5] = r2 / de_norm;
    } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) J[k] = 0.0;
    }
    return res;
}

// se3PointSurfFactor::Evaluate (REG/ceres_factor/surf_factor.hpp:32-56).
__device__ __forceinline__ double surf_residual(const Pose& P, d3 p, d3 n, double D, double* J) {
    d3 lp = transform(P, p);
    double res = dot(n, lp) + D;
    J[0] = n.y * (-lp.z) + n.z * lp.y;
    J[1] = n.x * lp.z + n.z * (-lp.x);
    J[2] = n.x * (-lp.y) + n.y * lp.x;
    J[3] = n.x;
    J[4] = n.y;
    J[5] = n.z;
    return res;
}

// Ceres HuberLoss(0.1) (a = 0.1, b = a*a) + Corrector with rho'' <= 0: r, J scaled by sqrt(rho').
// Accumulates into packet: [0] cost, [1..21] H upper, [22..27] g, [28] count.
__device__ __forceinline__ void huber_accumulate(double* P, double res, const double* J) {
    const double a = 0.1, b = a * a;
    double s = res * res;
    double rho0, rho1;
    if (s > b) {
        double r = sqrt(s);
        rho0 = 2.0 * a * r - b;
        rho1 = fmax(2.2250738585072014e-308, a / r);
    } else {
        rho0 = s;
        rho1 = 1.0;
    }
    double sr = sqrt(rho1);
    double rr = sr * res;
    double JJ[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) JJ[k] = sr * J[k];
    P[0] += 0.5 * rho0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = i; j < 6; ++j) P[1 + hidx(i, j)] += JJ[i] * JJ[j];
#pragma unroll
    for (int i = 0; i < 6; ++i) P[22 + i] += JJ[i] * rr;
    P[28] += 1.0;
}

}  // namespace lmsf
