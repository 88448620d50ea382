// TEST INFRASTRUCTURE ONLY -- CPU restatement of the registration half of the hot path.
//
// Follows (INC = src/MultiSensorFusionEstimator3D/include, REG = INC/Algorithm/PointClouds/registration):
//   REG/ceres_edgeSurfFeatureRegistration.hpp:96-244  (Solve, addEdge/SurfCostFactor, pointAssociateToMap)
//   REG/FeatureMatch/EdgeFeatureMatch.hpp:33-87        (5-NN + PCA line)
//   REG/FeatureMatch/surfFeatureMatch.hpp:32-88        (5-NN + QR plane)
//   REG/ceres_factor/edge_factor.hpp:33-61, surf_factor.hpp:32-56   (residuals / Jacobians)
//   INC/Algorithm/Ceres/Parameterization/PoseSE3Parameterization.hpp:32-60, INC/Math.hpp:19-72
//   REG/edgeSurfFeatureRegistration.hpp:113-350        (GN variant)
// External algorithms restated from their published descriptions (parity unpinned):
//   Eigen 3 Quaternion::_transformVector / quat_product / toRotationMatrix, ColPivHouseholderQR,
//   SelfAdjointEigenSolver (saes.cpp), Ceres Solver 1.x TrustRegionMinimizer +
//   LevenbergMarquardtStrategy (jacobi_scaling, DENSE_QR restated as normal equations), HuberLoss.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "lmsf_oracle.h"


void lmsfo_map_knn_one(const lmsfo_map* m, const float q[3], int k, int32_t* idx, float* d2);

namespace {

// ---------------------------------------------------------------- small math (Eigen semantics)
struct V3 { double x, y, z; };
inline V3 v3(double x, double y, double z) { return {x, y, z}; }
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline double sqnorm(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline double norm(V3 a) { return std::sqrt(sqnorm(a)); }

struct Quat { double x, y, z, w; };

// Eigen Quaternion::_transformVector: uv = q.vec x v; uv += uv; return v + w*uv + q.vec x uv
inline V3 rotate(const Quat& q, V3 v) {
    V3 qv{q.x, q.y, q.z};
    V3 uv = cross(qv, v);
    uv = add(uv, uv);
    V3 c = cross(qv, uv);
    return {v.x + q.w * uv.x + c.x, v.y + q.w * uv.y + c.y, v.z + q.w * uv.z + c.z};
}
// Eigen quat_product (scalar path)
inline Quat qmul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}
// Eigen QuaternionBase::toRotationMatrix
inline void qmat(const Quat& q, double R[3][3]) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz;       R[0][2] = txz + twy;
    R[1][0] = txy + twz;       R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy;       R[2][1] = tyz + twx;       R[2][2] = 1 - (txx + tyy);
}

inline Quat pose_q(const double* x) { return {x[0], x[1], x[2], x[3]}; }
inline V3 pose_t(const double* x) { return {x[4], x[5], x[6]}; }

// Math::GetTransformFromSe3 (INC/Math.hpp:29-72) + PoseSE3Parameterization::Plus (:32-46)
void pose_plus(const double* x, const double* delta, double* out) {
    V3 omega{delta[0], delta[1], delta[2]};
    V3 ups{delta[3], delta[4], delta[5]};
    double Om[3][3] = {{0., -omega.z, omega.y}, {omega.z, 0., -omega.x}, {-omega.y, omega.x, 0.}};
    double theta = norm(omega);
    double half_theta = 0.5 * theta;
    double imag_factor;
    double real_factor = std::cos(half_theta);
    if (theta < 1e-10) {
        double theta_sq = theta * theta;
        double theta_po4 = theta_sq * theta_sq;
        imag_factor = 0.5 - 0.0208333 * theta_sq + 0.000260417 * theta_po4;
    } else {
        double sin_half_theta = std::sin(half_theta);
        imag_factor = sin_half_theta / theta;
    }
    Quat dq{imag_factor * omega.x, imag_factor * omega.y, imag_factor * omega.z, real_factor};
    double J[3][3];
    if (theta < 1e-10) {
        qmat(dq, J);
    } else {
        double Om2[3][3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Om2[i][j] = Om[i][0] * Om[0][j] + Om[i][1] * Om[1][j] + Om[i][2] * Om[2][j];
        double c1 = (1 - std::cos(theta)) / (theta * theta);
        double c2 = (theta - std::sin(theta)) / (std::pow(theta, 3));
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) J[i][j] = (i == j ? 1.0 : 0.0) + c1 * Om[i][j] + c2 * Om2[i][j];
    }
    V3 dt{J[0][0] * ups.x + J[0][1] * ups.y + J[0][2] * ups.z,
          J[1][0] * ups.x + J[1][1] * ups.y + J[1][2] * ups.z,
          J[2][0] * ups.x + J[2][1] * ups.y + J[2][2] * ups.z};
    Quat q = pose_q(x);
    Quat qp = qmul(dq, q);
    V3 tp = add(rotate(dq, pose_t(x)), dt);
    out[0] = qp.x; out[1] = qp.y; out[2] = qp.z; out[3] = qp.w;
    out[4] = tp.x; out[5] = tp.y; out[6] = tp.z;
}

// ---------------------------------------------------------------- ColPivHouseholderQR solve
// A: m x n row-major (m <= 6, n <= 6, m >= n), b: m.  x: n.  Restates Eigen's computeInPlace +
// _solve_impl (column norms + LAPACK-style downdate, Householder with beta sign rule).
void colpiv_qr_solve(int m, int n, double* A, const double* b, double* x) {
    const double eps = std::numeric_limits<double>::epsilon();
    double cn_upd[6], cn_dir[6], hc[6];
    int transp[6];
    for (int j = 0; j < n; ++j) {
        double s = 0.0;
        for (int i = 0; i < m; ++i) s += A[i * n + j] * A[i * n + j];
        cn_upd[j] = cn_dir[j] = std::sqrt(s);
    }
    double maxcn = cn_upd[0];
    for (int j = 1; j < n; ++j) maxcn = std::max(maxcn, cn_upd[j]);
    double thr_helper = (maxcn * eps) * (maxcn * eps) / (double)m;
    const double downdate_thr = std::sqrt(eps);
    int size = std::min(m, n);
    int nonzero = size;
    for (int k = 0; k < size; ++k) {
        int big = k;
        for (int j = k + 1; j < n; ++j)
            if (cn_upd[j] > cn_upd[big]) big = j;
        double big_sq = cn_upd[big] * cn_upd[big];
        if (nonzero == size && big_sq < thr_helper * (double)(m - k)) nonzero = k;
        transp[k] = big;
        if (k != big) {
            for (int i = 0; i < m; ++i) std::swap(A[i * n + k], A[i * n + big]);
            std::swap(cn_upd[k], cn_upd[big]);
            std::swap(cn_dir[k], cn_dir[big]);
        }
        // makeHouseholderInPlace on A[k:m, k]
        double c0 = A[k * n + k];
        double tail = 0.0;
        for (int i = k + 1; i < m; ++i) tail += A[i * n + k] * A[i * n + k];
        double tau, beta;
        if (tail <= std::numeric_limits<double>::min()) {
            tau = 0.0;
            beta = c0;
            for (int i = k + 1; i < m; ++i) A[i * n + k] = 0.0;
        } else {
            beta = std::sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            for (int i = k + 1; i < m; ++i) A[i * n + k] = A[i * n + k] / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        A[k * n + k] = beta;
        hc[k] = tau;
        // applyHouseholderOnTheLeft to A[k:m, k+1:n]
        if (k + 1 < n) {
            if (m - k == 1) {
                for (int j = k + 1; j < n; ++j) A[k * n + j] *= (1.0 - tau);
            } else if (tau != 0.0) {
                for (int j = k + 1; j < n; ++j) {
                    double tmp = 0.0;
                    for (int i = k + 1; i < m; ++i) tmp += A[i * n + k] * A[i * n + j];
                    tmp += A[k * n + j];
                    A[k * n + j] -= tau * tmp;
                    for (int i = k + 1; i < m; ++i) A[i * n + j] -= (tau * A[i * n + k]) * tmp;
                }
            }
        }
        // column norm downdate
        for (int j = k + 1; j < n; ++j) {
            if (cn_upd[j] != 0.0) {
                double temp = std::fabs(A[k * n + j]) / cn_upd[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                double r = cn_upd[j] / cn_dir[j];
                double temp2 = temp * r * r;
                if (temp2 <= downdate_thr) {
                    double s = 0.0;
                    for (int i = k + 1; i < m; ++i) s += A[i * n + j] * A[i * n + j];
                    cn_dir[j] = std::sqrt(s);
                    cn_upd[j] = cn_dir[j];
                } else {
                    cn_upd[j] *= std::sqrt(temp);
                }
            }
        }
    }
    int perm[6];
    for (int j = 0; j < n; ++j) perm[j] = j;
    for (int k = 0; k < size; ++k) std::swap(perm[k], perm[transp[k]]);
    for (int j = 0; j < n; ++j) x[j] = 0.0;
    if (nonzero == 0) return;
    double c[6];
    for (int i = 0; i < m; ++i) c[i] = b[i];
    for (int k = 0; k < nonzero; ++k) {  // c = Q^T c, H_0 first
        double tau = hc[k];
        if (m - k == 1) {
            c[k] *= (1.0 - tau);
        } else if (tau != 0.0) {
            double tmp = 0.0;
            for (int i = k + 1; i < m; ++i) tmp += A[i * n + k] * c[i];
            tmp += c[k];
            c[k] -= tau * tmp;
            for (int i = k + 1; i < m; ++i) c[i] -= (tau * A[i * n + k]) * tmp;
        }
    }
    for (int i = nonzero - 1; i >= 0; --i) {  // column-oriented back substitution
        c[i] = c[i] / A[i * n + i];
        for (int r = 0; r < i; ++r) c[r] -= c[i] * A[r * n + i];
    }
    for (int i = 0; i < nonzero; ++i) x[perm[i]] = c[i];
}

// ---------------------------------------------------------------- matching
struct Match {
    lmsfo_record rec;
    double gn_grad[3];   // EdgeCostFactorInfo::norm_ / flipped surf normal (GN path)
    double gn_res;       // residuals_ (GN path)
};

inline V3 fpt(const float* p) { return {(double)p[0], (double)p[1], (double)p[2]}; }

// pointAssociateToMap (ceres_...:235-244): double transform, stored back into float members.
inline void associate(const double* x, const float* p, float out[3]) {
    V3 w = add(rotate(pose_q(x), fpt(p)), pose_t(x));
    out[0] = (float)w.x; out[1] = (float)w.y; out[2] = (float)w.z;
}

// EdgeFeatureMatch::Match (EdgeFeatureMatch.hpp:33-87) given the 5 sorted neighbours.
bool edge_fit(const float* mp, const int32_t* nn, const float q[3], Match& m) {
    V3 pts[5];
    V3 center{0, 0, 0};
    for (int j = 0; j < 5; ++j) {
        const float* p = mp + 4 * (size_t)nn[j];
        pts[j] = fpt(p);
        center = add(center, pts[j]);
    }
    center = {center.x / 5.0, center.y / 5.0, center.z / 5.0};
    double cov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < 5; ++j) {
        V3 e = sub(pts[j], center);
        double ev[3] = {e.x, e.y, e.z};
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) cov[r * 3 + c] = cov[r * 3 + c] + ev[r] * ev[c];
    }
    double d[3], v[9];
    lmsfo_saes3(cov, d, v);   // Eigen::SelfAdjointEigenSolver<Matrix3d> (EdgeFeatureMatch.hpp:63, saes.cpp)
    V3 u{v[0 * 3 + 2], v[1 * 3 + 2], v[2 * 3 + 2]};
    if (!(d[2] > 3 * d[1])) return false;
    V3 a = add(mul(0.1, u), center);
    V3 b = add(mul(-0.1, u), center);
    V3 cp = fpt(q);
    V3 nu = cross(sub(cp, a), sub(cp, b));
    V3 de = sub(a, b);
    double de_norm = norm(de);
    m.gn_res = norm(nu) / de_norm;
    V3 g = cross(de, nu);
    double gn = norm(g);
    m.gn_grad[0] = gn > 0 ? g.x / gn : g.x;
    m.gn_grad[1] = gn > 0 ? g.y / gn : g.y;
    m.gn_grad[2] = gn > 0 ? g.z / gn : g.z;
    m.rec.kind = LMSFO_KIND_EDGE;
    m.rec.v0[0] = a.x; m.rec.v0[1] = a.y; m.rec.v0[2] = a.z;
    m.rec.v1[0] = b.x; m.rec.v1[1] = b.y; m.rec.v1[2] = b.z;
    return true;
}

// SurfFeatureMatch::Match (surfFeatureMatch.hpp:32-88) given the 5 sorted neighbours.
bool surf_fit(const float* mp, const int32_t* nn, const float q[3], Match& m) {
    double A[15], b[5];
    for (int j = 0; j < 5; ++j) {
        const float* p = mp + 4 * (size_t)nn[j];
        A[j * 3 + 0] = p[0]; A[j * 3 + 1] = p[1]; A[j * 3 + 2] = p[2];
        b[j] = -1.0;
    }
    double nrm[3];
    colpiv_qr_solve(5, 3, A, b, nrm);
    V3 n{nrm[0], nrm[1], nrm[2]};
    double nn_ = norm(n);
    double D = 1 / nn_;
    double z = sqnorm(n);
    if (z > 0.0) {
        double s = std::sqrt(z);
        n = {n.x / s, n.y / s, n.z / s};
    }
    for (int j = 0; j < 5; ++j) {
        const float* p = mp + 4 * (size_t)nn[j];
        if (std::fabs(n.x * (double)p[0] + n.y * (double)p[1] + n.z * (double)p[2] + D) > 0.2) return false;
    }
    V3 cp = fpt(q);
    float distance = (float)(dot(n, cp) + D);
    m.gn_res = std::fabs(distance);
    if (distance >= 0) {
        m.rec.v0[0] = n.x; m.rec.v0[1] = n.y; m.rec.v0[2] = n.z; m.rec.v1[0] = D;
    } else {
        m.rec.v0[0] = -n.x; m.rec.v0[1] = -n.y; m.rec.v0[2] = -n.z; m.rec.v1[0] = -D;
    }
    m.rec.v1[1] = 0.0; m.rec.v1[2] = 0.0;
    m.gn_grad[0] = m.rec.v0[0]; m.gn_grad[1] = m.rec.v0[1]; m.gn_grad[2] = m.rec.v0[2];
    m.rec.kind = LMSFO_KIND_SURF;
    return true;
}

// ---------------------------------------------------------------- residual packet
inline int hidx(int i, int j) { return i * 6 - i * (i - 1) / 2 + (j - i); }

struct Packet {
    double v[29];
    void clear() { for (int i = 0; i < 29; ++i) v[i] = 0.0; }
};

// Residual and 6-dof Jacobian of one record at pose x (edge_factor.hpp:33-61 / surf_factor.hpp:32-56).
inline bool residual_jacobian(const lmsfo_record& r, const double* x, double& res, double J[6]) {
    V3 p{(double)r.px, (double)r.py, (double)r.pz};
    V3 lp = add(rotate(pose_q(x), p), pose_t(x));
    if (r.kind == LMSFO_KIND_EDGE) {
        V3 a{r.v0[0], r.v0[1], r.v0[2]}, b{r.v1[0], r.v1[1], r.v1[2]};
        V3 nu = cross(sub(lp, a), sub(lp, b));
        V3 de = sub(a, b);
        double de_norm = norm(de);
        double nu_norm = norm(nu);
        res = nu_norm / de_norm;
        // J = -(nu^T/|nu|) * [de]x * [-[lp]x, I] / |de|   (|nu| == 0: NaN in the reference; 0 here)
        if (nu_norm > 0) {
            V3 w{-nu.x / nu_norm, -nu.y / nu_norm, -nu.z / nu_norm};
            // row1 = w^T [de]x,  [de]x = [[0,-dz,dy],[dz,0,-dx],[-dy,dx,0]]
            double r0 = w.y * de.z + w.z * (-de.y);
            double r1 = w.x * (-de.z) + w.z * de.x;
            double r2 = w.x * de.y + w.y * (-de.x);
            // row2 = row1 * [-[lp]x | I],  -[lp]x = [[0,lz,-ly],[-lz,0,lx],[ly,-lx,0]]
            J[0] = (r1 * (-lp.z) + r2 * lp.y) / de_norm;
            J[1] = (r0 * lp.z + r2 * (-lp.x)) / de_norm;
            J[2] = (r0 * (-lp.y) + r1 * lp.x) / de_norm;
            J[3] = r0 / de_norm;
            J[4] = r1 / de_norm;
            J[5] = r2 / de_norm;
        } else {
            for (int k = 0; k < 6; ++k) J[k] = 0.0;
        }
        return true;
    }
    if (r.kind == LMSFO_KIND_SURF) {
        V3 n{r.v0[0], r.v0[1], r.v0[2]};
        res = dot(n, lp) + r.v1[0];
        J[0] = n.y * (-lp.z) + n.z * lp.y;
        J[1] = n.x * lp.z + n.z * (-lp.x);
        J[2] = n.x * (-lp.y) + n.y * lp.x;
        J[3] = n.x;
        J[4] = n.y;
        J[5] = n.z;
        return true;
    }
    return false;
}

// Ceres HuberLoss(0.1) + Corrector (rho'' <= 0 => pure sqrt(rho') scaling).
inline void accumulate(Packet& P, double res, const double J[6]) {
    const double a = 0.1, b = a * a;
    double s = res * res;
    double rho0, rho1;
    if (s > b) {
        double r = std::sqrt(s);
        rho0 = 2.0 * a * r - b;
        rho1 = std::max(std::numeric_limits<double>::min(), a / r);
    } else {
        rho0 = s;
        rho1 = 1.0;
    }
    double sr = std::sqrt(rho1);
    double rr = sr * res;
    double JJ[6];
    for (int k = 0; k < 6; ++k) JJ[k] = sr * J[k];
    P.v[0] += 0.5 * rho0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j) P.v[1 + hidx(i, j)] += JJ[i] * JJ[j];
    for (int i = 0; i < 6; ++i) P.v[22 + i] += JJ[i] * rr;
    P.v[28] += 1.0;
}

int g_threads = 1;

void eval_records(const lmsfo_record* rec, int64_t n, const double* x, Packet& out) {
    out.clear();
    int nt = g_threads;
    if (nt <= 1 || n < 4096) {
        for (int64_t i = 0; i < n; ++i) {
            double res, J[6];
            if (residual_jacobian(rec[i], x, res, J)) accumulate(out, res, J);
        }
        return;
    }
    // fixed chunking by nt (not by the team size OpenMP grants) keeps the sum order reproducible
    std::vector<Packet> part(nt);
    for (auto& p : part) p.clear();
#pragma omp parallel for schedule(static, 1) num_threads(nt)
    for (int t = 0; t < nt; ++t) {
        int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
        for (int64_t i = lo; i < hi; ++i) {
            double res, J[6];
            if (residual_jacobian(rec[i], x, res, J)) accumulate(part[t], res, J);
        }
    }
    for (int t = 0; t < nt; ++t)
        for (int k = 0; k < 29; ++k) out.v[k] += part[t].v[k];
}

// 6x6 SPD solve by Cholesky; returns false when not positive definite.
bool chol_solve6(const double* A, const double* b, double* x) {
    double L[36] = {0};
    for (int j = 0; j < 6; ++j) {
        double s = A[j * 6 + j];
        for (int k = 0; k < j; ++k) s -= L[j * 6 + k] * L[j * 6 + k];
        if (!(s > 0.0)) return false;
        double ljj = std::sqrt(s);
        L[j * 6 + j] = ljj;
        for (int i = j + 1; i < 6; ++i) {
            double t = A[i * 6 + j];
            for (int k = 0; k < j; ++k) t -= L[i * 6 + k] * L[j * 6 + k];
            L[i * 6 + j] = t / ljj;
        }
    }
    double y[6];
    for (int i = 0; i < 6; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t -= L[i * 6 + k] * y[k];
        y[i] = t / L[i * 6 + i];
    }
    for (int i = 5; i >= 0; --i) {
        double t = y[i];
        for (int k = i + 1; k < 6; ++k) t -= L[k * 6 + i] * x[k];
        x[i] = t / L[i * 6 + i];
    }
    for (int i = 0; i < 6; ++i)
        if (!std::isfinite(x[i])) return false;
    return true;
}

double norm7(const double* x) {
    double s = 0.0;
    for (int i = 0; i < 7; ++i) s += x[i] * x[i];
    return std::sqrt(s);
}

double grad_max_norm(const double* x, const double* g) {
    double ng[6], xp[7];
    for (int i = 0; i < 6; ++i) ng[i] = -g[i];
    pose_plus(x, ng, xp);
    double m = 0.0;
    for (int i = 0; i < 7; ++i) m = std::max(m, std::fabs(x[i] - xp[i]));
    return m;
}

struct LmResult { int term; int iterations; int evaluations; double initial_cost, final_cost; };

// ceres::Solve with TRUST_REGION / LEVENBERG_MARQUARDT, max_num_iterations = 4, defaults otherwise
// (ceres_...:107-123).  x is updated in place to the last accepted point.
LmResult ceres_lm(const lmsfo_record* rec, int64_t n, double* x) {
    LmResult R{LMSFO_TERM_MAX_ITERATIONS, 0, 0, 0.0, 0.0};
    const int max_iter = 4;
    const double func_tol = 1e-6, grad_tol = 1e-10, param_tol = 1e-8, min_rel = 1e-3;
    const double min_diag = 1e-6, max_diag = 1e32, max_radius = 1e16, min_radius = 1e-32;
    Packet P;
    eval_records(rec, n, x, P);
    R.evaluations = 1;
    if (P.v[28] == 0.0) { R.term = LMSFO_TERM_NO_RESIDUALS; return R; }
    double cost = P.v[0];
    R.initial_cost = R.final_cost = cost;
    double H[21], g[6], s[6];
    std::memcpy(H, P.v + 1, sizeof H);
    std::memcpy(g, P.v + 22, sizeof g);
    for (int j = 0; j < 6; ++j) s[j] = 1.0 / (1.0 + std::sqrt(H[hidx(j, j)]));
    double radius = 1e4, decrease = 2.0;
    double x_norm = norm7(x);
    int iteration = 0;
    if (grad_max_norm(x, g) <= grad_tol) { R.term = LMSFO_TERM_GRADIENT_TOL; return R; }
    while (true) {
        if (iteration >= max_iter) { R.term = LMSFO_TERM_MAX_ITERATIONS; break; }
        if (radius < min_radius) { R.term = LMSFO_TERM_PARAMETER_TOL; break; }
        ++iteration;
        double A[36], gs[6], step[6], nb[6];
        for (int i = 0; i < 6; ++i) {
            gs[i] = g[i] * s[i];
            for (int j = 0; j < 6; ++j) {
                int a = i <= j ? hidx(i, j) : hidx(j, i);
                A[i * 6 + j] = H[a] * s[i] * s[j];
            }
        }
        double Hs[36];
        std::memcpy(Hs, A, sizeof Hs);
        for (int i = 0; i < 6; ++i) {
            double dg = std::min(std::max(Hs[i * 6 + i], min_diag), max_diag);
            A[i * 6 + i] += dg / radius;
            nb[i] = -gs[i];
        }
        bool ok = chol_solve6(A, nb, step);
        double mcc = 0.0;
        if (ok) {
            double sg = 0.0, sHs = 0.0;
            for (int i = 0; i < 6; ++i) {
                sg += step[i] * gs[i];
                double t = 0.0;
                for (int j = 0; j < 6; ++j) t += Hs[i * 6 + j] * step[j];
                sHs += step[i] * t;
            }
            mcc = -(sg + 0.5 * sHs);
        }
        if (!ok || !(mcc > 0.0)) {  // invalid step: StepIsInvalid == StepRejected(0)
            radius = radius / decrease;
            decrease *= 2.0;
            continue;
        }
        double delta[6], xc[7];
        for (int i = 0; i < 6; ++i) delta[i] = step[i] * s[i];
        pose_plus(x, delta, xc);
        Packet Pc;
        eval_records(rec, n, xc, Pc);
        ++R.evaluations;
        double cost_c = std::isfinite(Pc.v[0]) ? Pc.v[0] : DBL_MAX;
        double dx[7];
        for (int i = 0; i < 7; ++i) dx[i] = x[i] - xc[i];
        if (norm7(dx) <= param_tol * (x_norm + param_tol)) { R.term = LMSFO_TERM_PARAMETER_TOL; break; }
        double cost_change = cost - cost_c;
        if (std::fabs(cost_change) <= func_tol * cost) { R.term = LMSFO_TERM_FUNCTION_TOL; break; }
        double rel = cost_change / mcc;
        if (rel > min_rel) {
            double f = 1.0 - std::pow(2.0 * rel - 1.0, 3);
            radius = radius / std::max(1.0 / 3.0, f);
            radius = std::min(max_radius, radius);
            decrease = 2.0;
            std::memcpy(x, xc, 7 * sizeof(double));
            x_norm = norm7(x);
            cost = cost_c;
            R.final_cost = cost;
            std::memcpy(H, Pc.v + 1, sizeof H);
            std::memcpy(g, Pc.v + 22, sizeof g);
            if (iteration >= max_iter) { R.term = LMSFO_TERM_MAX_ITERATIONS; break; }
            if (grad_max_norm(x, g) <= grad_tol) { R.term = LMSFO_TERM_GRADIENT_TOL; break; }
        } else {
            radius = radius / decrease;
            decrease *= 2.0;
        }
    }
    R.iterations = iteration;
    return R;
}

}  // namespace

// ---------------------------------------------------------------- registration object
struct lmsfo_reg {
    int solver = LMSFO_SOLVER_CERES_LM;
    int optimization_count = 10;   // ceres_...:46 / edgeSurf...:65
    bool fixed = false;
    lmsfo_map* tree[3] = {nullptr, nullptr, nullptr};
    std::vector<float> map_pts[3];
    std::vector<float> scan[3];
    // GN persistent state (edgeSurfFeatureRegistration.hpp:55,61)
    double gn_map[36];
    bool gn_degenerate = false;
    ~lmsfo_reg() {
        for (auto* t : tree) lmsfo_map_free(t);
    }
};

namespace {

void match_all(lmsfo_reg* r, const double* x, std::vector<Match>& out, int32_t* nn_out) {
    const int64_t ne = (int64_t)r->scan[1].size() / 4, ns = (int64_t)r->scan[2].size() / 4;
    out.resize((size_t)(ne + ns));
#pragma omp parallel for schedule(dynamic, 256) num_threads(g_threads)
    for (int64_t i = 0; i < ne + ns; ++i) {
        int kind = i < ne ? 1 : 2;
        const float* p = kind == 1 ? &r->scan[1][4 * (size_t)i] : &r->scan[2][4 * (size_t)(i - ne)];
        Match& m = out[(size_t)i];
        std::memset(&m, 0, sizeof m);
        m.rec.px = p[0]; m.rec.py = p[1]; m.rec.pz = p[2];
        m.rec.kind = 0;
        int32_t nn[5] = {-1, -1, -1, -1, -1};
        if (r->tree[kind] != nullptr && lmsfo_map_size(r->tree[kind]) > 0) {
            float q[3];
            associate(x, p, q);
            float d2[5];
            lmsfo_map_knn_one(r->tree[kind], q, 5, nn, d2);
            // sqd[4] < search_thresh_ (1.0, FeatureMatchBase.hpp:29); fewer than 5 points -> no match
            if (nn[4] >= 0 && d2[4] < 1.0f) {
                if (kind == 1) edge_fit(r->map_pts[1].data(), nn, q, m);
                else surf_fit(r->map_pts[2].data(), nn, q, m);
            }
        }
        if (nn_out)
            for (int j = 0; j < 5; ++j) nn_out[5 * i + j] = nn[j];
    }
}

// GNOptimization (edgeSurfFeatureRegistration.hpp:218-330).  Returns true when converged.
bool gn_step(lmsfo_reg* r, int iterCount, const std::vector<Match>& ms, int64_t ne, double* x, int& term) {
    // uint16_t counters (edgeSurf...:58-59) wrap modulo 65536
    int e_cnt = 0, s_cnt = 0;
    std::vector<const Match*> E, S;
    for (int64_t i = 0; i < (int64_t)ms.size(); ++i) {
        if (ms[i].rec.kind == 0) continue;
        if (i < ne) E.push_back(&ms[i]); else S.push_back(&ms[i]);
    }
    e_cnt = (int)(uint16_t)E.size();
    s_cnt = (int)(uint16_t)S.size();
    if (e_cnt + s_cnt < 10) { term = LMSFO_TERM_GN_TOO_FEW; return false; }
    double R[3][3];
    Quat q = pose_q(x);
    qmat(q, R);
    double JTJ[36] = {0}, JTR[6] = {0};
    for (int i = 0; i < e_cnt + s_cnt; ++i) {
        const Match* m = i < e_cnt ? E[i] : S[i - e_cnt];
        V3 p{(double)m->rec.px, (double)m->rec.py, (double)m->rec.pz};
        double sk[3][3] = {{0., -p.z, p.y}, {p.z, 0., -p.x}, {-p.y, p.x, 0.}};
        double M[3][3];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) M[a][b] = (-R[a][0]) * sk[0][b] + (-R[a][1]) * sk[1][b] + (-R[a][2]) * sk[2][b];
        const double* gr = m->gn_grad;
        double J[6];
        for (int b = 0; b < 3; ++b) J[b] = gr[0] * M[0][b] + gr[1] * M[1][b] + gr[2] * M[2][b];
        J[3] = gr[0]; J[4] = gr[1]; J[5] = gr[2];
        double res = m->gn_res;
        for (int a = 0; a < 6; ++a) {
            for (int b = 0; b < 6; ++b) JTJ[a * 6 + b] += J[a] * J[b];
            JTR[a] += J[a] * res;
        }
    }
    double A[36], nb[6], X[6];
    std::memcpy(A, JTJ, sizeof A);
    for (int a = 0; a < 6; ++a) nb[a] = -JTR[a];
    colpiv_qr_solve(6, 6, A, nb, X);
    if (iterCount == 0) {
        double a2[36], d[6], V[36];
        std::memcpy(a2, JTJ, sizeof a2);
        lmsfo_saesx(6, a2, d, V);   // SelfAdjointEigenSolver<MatrixXd> (edgeSurf...:282, saes.cpp)
        double V2[36];
        std::memcpy(V2, V, sizeof V2);
        r->gn_degenerate = false;
        for (int i = 5; i >= 0; i--) {
            if (d[i] < 100.0) {  // float degeneracy_thresh = 100
                for (int c = 0; c < 6; ++c) V2[i * 6 + c] = 0.0;   // rows zeroed (:293)
                r->gn_degenerate = true;
            } else {
                break;
            }
        }
        // Map = V^-1 * V2 ; V orthogonal => V^-1 = V^T (deviation: Eigen uses an LU inverse)
        for (int a = 0; a < 6; ++a)
            for (int b = 0; b < 6; ++b) {
                double t = 0.0;
                for (int k = 0; k < 6; ++k) t += V[k * 6 + a] * V2[k * 6 + b];
                r->gn_map[a * 6 + b] = t;
            }
    }
    if (r->gn_degenerate) {
        double Y[6];
        for (int a = 0; a < 6; ++a) {
            double t = 0.0;
            for (int k = 0; k < 6; ++k) t += r->gn_map[a * 6 + k] * X[k];
            Y[a] = t;
        }
        std::memcpy(X, Y, sizeof Y);
    }
    x[4] += X[3]; x[5] += X[4]; x[6] += X[5];
    V3 dr{X[0], X[1], X[2]};
    double drn = norm(dr);
    V3 axis = drn > 0 ? V3{dr.x / drn, dr.y / drn, dr.z / drn} : dr;
    double ha = 0.5 * (drn / 2);
    double sh = std::sin(ha);
    Quat dq{sh * axis.x, sh * axis.y, sh * axis.z, std::cos(ha)};
    Quat qn = qmul(q, dq);
    x[0] = qn.x; x[1] = qn.y; x[2] = qn.z; x[3] = qn.w;
    float deltaR = (float)(drn / 2);
    float deltaT = (float)std::sqrt(std::pow(X[3] * 100, 2) + std::pow(X[4] * 100, 2) + std::pow(X[5] * 100, 2));
    if (deltaR < 0.0009f && deltaT < 0.05f) { term = LMSFO_TERM_GN_CONVERGED; return true; }
    term = LMSFO_TERM_MAX_ITERATIONS;
    return false;
}

}  // namespace

extern "C" {

lmsfo_reg* lmsfo_reg_create(int solver) {
    lmsfo_reg* r = new lmsfo_reg();
    r->solver = solver;
    return r;
}
void lmsfo_reg_free(lmsfo_reg* r) { delete r; }

void lmsfo_reg_set_map(lmsfo_reg* r, int kind, const float* xyzi, int64_t n) {
    if (kind != 1 && kind != 2) return;
    if (n <= 0) return;  // empty source ignored (ceres_...:60)
    r->map_pts[kind].assign(xyzi, xyzi + 4 * n);
    lmsfo_map_free(r->tree[kind]);
    r->tree[kind] = lmsfo_map_build(xyzi, n);
}

void lmsfo_reg_set_scan(lmsfo_reg* r, int kind, const float* xyzi, int64_t n) {
    if (kind != 1 && kind != 2) return;
    r->scan[kind].assign(xyzi, xyzi + 4 * (n > 0 ? n : 0));
}

void lmsfo_reg_set_max_iterations(lmsfo_reg* r, int n) { r->optimization_count = n; }
void lmsfo_reg_set_fixed_schedule(lmsfo_reg* r, int fixed) { r->fixed = fixed != 0; }
int64_t lmsfo_reg_num_queries(const lmsfo_reg* r) { return (int64_t)(r->scan[1].size() + r->scan[2].size()) / 4; }

int lmsfo_reg_match(lmsfo_reg* r, const double pose[7], lmsfo_record* out, int32_t* nn) {
    std::vector<Match> ms;
    match_all(r, pose, ms, nn);
    for (size_t i = 0; i < ms.size(); ++i) out[i] = ms[i].rec;
    return 0;
}

int lmsfo_reg_solve(lmsfo_reg* r, double pose[7], double* trace, int trace_cap, lmsfo_solve_stats* st) {
    lmsfo_solve_stats S;
    std::memset(&S, 0, sizeof S);
    const int64_t ne = (int64_t)r->scan[1].size() / 4;
    int iters;
    if (r->solver == LMSFO_SOLVER_CERES_LM) {
        if (!r->fixed && r->optimization_count > 2) r->optimization_count--;   // ceres_...:100-101
        iters = r->optimization_count;
    } else {
        iters = r->optimization_count;  // GN: no decrement (edgeSurf...:127)
    }
    std::vector<Match> ms;
    std::vector<lmsfo_record> recs;
    for (int it = 0; it < iters; ++it) {
        match_all(r, pose, ms, nullptr);
        int ec = 0, sc = 0;
        for (int64_t i = 0; i < (int64_t)ms.size(); ++i)
            if (ms[i].rec.kind != 0) (i < ne ? ec : sc)++;
        S.edge_matches = ec;
        S.surf_matches = sc;
        S.outer_iterations = it + 1;
        if (r->solver == LMSFO_SOLVER_CERES_LM) {
            recs.resize(ms.size());
            for (size_t i = 0; i < ms.size(); ++i) recs[i] = ms[i].rec;
            LmResult L = ceres_lm(recs.data(), (int64_t)recs.size(), pose);
            S.inner_iterations += L.iterations;
            S.evaluations += L.evaluations;
            S.termination = L.term;
            S.initial_cost = L.initial_cost;
            S.final_cost = L.final_cost;
            if (trace && it < trace_cap) std::memcpy(trace + 7 * it, pose, 7 * sizeof(double));
        } else {
            int term = 0;
            bool conv = gn_step(r, it, ms, ne, pose, term);
            S.termination = term;
            S.inner_iterations += 1;
            if (trace && it < trace_cap) std::memcpy(trace + 7 * it, pose, 7 * sizeof(double));
            if (conv) break;
        }
    }
    if (st) *st = S;
    return 0;
}

void lmsfo_eval(const lmsfo_record* rec, int64_t n, const double pose[7], double out[29]) {
    Packet P;
    eval_records(rec, n, pose, P);
    for (int i = 0; i < 29; ++i) out[i] = P.v[i];
}

void lmsfo_pose_plus(const double x[7], const double delta[6], double out[7]) { pose_plus(x, delta, out); }

void lmsfo_set_num_threads(int n) { g_threads = n < 1 ? 1 : n; }

}  // extern "C"
