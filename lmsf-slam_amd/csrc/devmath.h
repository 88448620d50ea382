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

// Math::GetTransformFromSe3 (INC/Math.hpp:29-72) + PoseSE3Parameterization::Plus
// (INC/Algorithm/Ceres/Parameterization/PoseSE3Parameterization.hpp:32-46)
__device__ inline void pose_plus(const double* x, const double* delta, double* out) {
    d3 om = mk(delta[0], delta[1], delta[2]);
    d3 up = mk(delta[3], delta[4], delta[5]);
    double theta = norm(om);
    double half_theta = 0.5 * theta;
    double real_factor = cos(half_theta);
    double imag_factor;
    if (theta < 1e-10) {
        double tsq = theta * theta;
        double tp4 = tsq * tsq;
        imag_factor = 0.5 - 0.0208333 * tsq + 0.000260417 * tp4;
    } else {
        imag_factor = sin(half_theta) / theta;
    }
    dq d;
    d.x = imag_factor * om.x; d.y = imag_factor * om.y; d.z = imag_factor * om.z; d.w = real_factor;
    double J[9];
    if (theta < 1e-10) {
        qmat(d, J);
    } else {
        const double Om[9] = {0., -om.z, om.y, om.z, 0., -om.x, -om.y, om.x, 0.};
        double c1 = (1 - cos(theta)) / (theta * theta);
        double c2 = (theta - sin(theta)) / (pow(theta, 3.0));
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

// ---------------------------------------------------------------- cyclic Jacobi, symmetric NxN
// (SelfAdjointEigenSolver restated; EdgeFeatureMatch.hpp:63).  Compile-time N keeps every index
// static so the matrices live in registers.  Output: d ascending (stable on index), v columns.
template <int N>
__device__ __forceinline__ void jrot(double* m, int i, int j, int k, int l, double s, double tau) {
    double g = m[i * N + j], h = m[k * N + l];
    m[i * N + j] = g - s * (h + g * tau);
    m[k * N + l] = h + s * (g - h * tau);
}

template <int N>
__device__ inline void jacobi_eig(double* a, double* d, double* v) {
    double b[N], z[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int j = 0; j < N; ++j) v[i * N + j] = (i == j) ? 1.0 : 0.0;
        b[i] = d[i] = a[i * N + i];
        z[i] = 0.0;
    }
    for (int sweep = 1; sweep <= 50; ++sweep) {
        double sm = 0.0;
#pragma unroll
        for (int p = 0; p < N - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) sm += fabs(a[p * N + q]);
        if (sm == 0.0) break;
        double tresh = (sweep < 4) ? 0.2 * sm / (N * N) : 0.0;
#pragma unroll
        for (int p = 0; p < N - 1; ++p) {
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                double apq = a[p * N + q];
                double g = 100.0 * fabs(apq);
                if (sweep > 4 && fabs(d[p]) + g == fabs(d[p]) && fabs(d[q]) + g == fabs(d[q])) {
                    a[p * N + q] = 0.0;
                } else if (fabs(apq) > tresh) {
                    double h = d[q] - d[p];
                    double t;
                    if (fabs(h) + g == fabs(h)) {
                        t = apq / h;
                    } else {
                        double theta = 0.5 * h / apq;
                        t = 1.0 / (fabs(theta) + sqrt(1.0 + theta * theta));
                        if (theta < 0.0) t = -t;
                    }
                    double c = 1.0 / sqrt(1 + t * t);
                    double s = t * c;
                    double tau = s / (1.0 + c);
                    h = t * apq;
                    z[p] -= h; z[q] += h; d[p] -= h; d[q] += h;
                    a[p * N + q] = 0.0;
#pragma unroll
                    for (int j = 0; j < p; ++j) jrot<N>(a, j, p, j, q, s, tau);
#pragma unroll
                    for (int j = p + 1; j < q; ++j) jrot<N>(a, p, j, j, q, s, tau);
#pragma unroll
                    for (int j = q + 1; j < N; ++j) jrot<N>(a, p, j, q, j, s, tau);
#pragma unroll
                    for (int j = 0; j < N; ++j) jrot<N>(v, j, p, j, q, s, tau);
                }
            }
        }
#pragma unroll
        for (int p = 0; p < N; ++p) { b[p] += z[p]; d[p] = b[p]; z[p] = 0.0; }
    }
}

// Eigenvalue order of a 3x3 result (ascending, stable on index) without dynamic indexing.
__device__ __forceinline__ void order3(const double* d, int& i0, int& i1, int& i2) {
    // insertion sort of (0,1,2) by d, stable; the values ride along (a0 = d[i0], a1 = d[i1]) so no
    // runtime index touches d (a dynamically indexed array lives in scratch)
    i0 = 0; i1 = 1; i2 = 2;
    double a0 = d[0], a1 = d[1];
    const double a2 = d[2];
    if (a0 > a1) { int t = i0; i0 = i1; i1 = t; double u = a0; a0 = a1; a1 = u; }
    // insert element 2
    if (a1 > a2) {
        i2 = i1;
        if (a0 > a2) { i1 = i0; i0 = 2; } else { i1 = 2; }
    }
}
// Middle and largest value of the stable ascending order of d[0..2] and the largest's index
// (= d[i1], d[i2] of order3), as selects: order3's reference outputs end up in scratch.
__device__ __forceinline__ void top2_of3(const double* d, double& mid, double& big, int& ibig) {
    double a0 = d[0], a1 = d[1];
    int j1 = 1;
    if (a0 > a1) { const double u = a0; a0 = a1; a1 = u; j1 = 0; }
    const double a2 = d[2];
    const bool hi = a1 > a2;   // element 2 inserted below a1
    ibig = hi ? j1 : 2;
    big = hi ? a1 : a2;
    mid = hi ? (a0 > a2 ? a0 : a2) : a1;
}
__device__ __forceinline__ double pick3(const double* a, int i) { return i == 0 ? a[0] : (i == 1 ? a[1] : a[2]); }

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
                double r = cn_upd[j] / cn_dir[j];
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
