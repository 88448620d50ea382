// TEST INFRASTRUCTURE ONLY -- CPU restatement of Eigen's SelfAdjointEigenSolver, the symmetric
// eigen-decomposition the reference calls on the hot path:
//   EdgeFeatureMatch.hpp:63               Eigen::SelfAdjointEigenSolver<Eigen::Matrix3d> saes(covMat)
//   edgeSurfFeatureRegistration.hpp:282   Eigen::SelfAdjointEigenSolver<Eigen::MatrixXd> eigensolver(JTJ)
// Eigen is a third-party dependency absent from /root/reference (the reference resolves it with
// find_package(Eigen3), CMakeLists.txt:33).  Pinned version: the Eigen 3.3 series (3.3.4 / 3.3.7, the
// Ubuntu 18.04 / 20.04 system packages of ROS melodic / noetic).  Its published algorithm
// (Eigenvalues/SelfAdjointEigenSolver.h, Eigenvalues/Tridiagonalization.h, Jacobi/Jacobi.h):
//   compute():  mat = lower triangle of A; scale = max |mat|; (scale == 0 -> 1); mat /= scale;
//               tridiagonalization_inplace(mat, diag, subdiag, extractQ = true);
//               computeFromTridiagonal_impl(diag, subdiag, 30, true, mat);  eigenvalues *= scale.
//   tridiagonalization_inplace_selector<Matrix3d, 3, false>: one closed-form Householder step
//               (beta = hypot(m10, m20) by sqrt of the sum of squares), Q = [1 0 0; 0 m01 m02; 0 m02 -m01],
//               or the identity when m20^2 <= DBL_MIN;  dynamic size: Householder reflections
//               (makeHouseholderInPlace, SYMV of the lower triangle, rank-2 update), Q evaluated from the
//               HouseholderSequence (reflectors applied to I on the left, last first).
//   computeFromTridiagonal_impl: sub-diagonal entries with |e| <= 2 eps (|d_i| + |d_i+1|) or
//               |e| <= DBL_MIN set to 0; the trailing unreduced block [start, end] gets one implicit
//               symmetric QR step with Wilkinson shift (tridiagonal_qr_step: makeGivens rotations chasing
//               the bulge, Q = Q * G); at most 30 n steps; then selection sort ascending (first index of
//               the minimum) with column swaps -- only when converged.
// Deviation (documented): the dynamic path evaluates SYMV / dot / rank-2 update / the
// reflector products in plain sequential order; Eigen's vectorised kernels sum in packet order, so the
// 6x6 GN result agrees to rounding, not bit for bit.  The fixed 3x3 path has no such kernel: it is a
// bit-level restatement (the GPU edge fit, devmath.h saes3, follows it operation for operation).
// The 3.4 series changed two details (deflation |e| <= eps sqrt(|d_i| + |d_i+1|), and the QR step
// stops once the bulge z is 0); kinetic's 3.3-beta1 is taken to match 3.3.
#include <cfloat>
#include <cmath>
#include <cstring>
#include <utility>

#include "lmsf_oracle.h"

namespace {

// numext::hypot (MathFunctions.h hypot_impl): p = max(|x|, |y|), qp = min / p, p sqrt(1 + qp^2)
inline double eigen_hypot(double x, double y) {
    const double ax = std::fabs(x), ay = std::fabs(y);
    double p, qp;
    if (ax > ay) { p = ax; qp = ay / p; } else { p = ay; qp = ax / p; }
    if (p == 0.0) return 0.0;
    return p * std::sqrt(1.0 + qp * qp);
}

// JacobiRotation<double>::makeGivens(p, q) (real case): G = [c s; -s c] with G^T [p; q] = [r; 0]
inline void make_givens(double p, double q, double& c, double& s) {
    if (q == 0.0) {
        c = p < 0.0 ? -1.0 : 1.0;
        s = 0.0;
    } else if (p == 0.0) {
        c = 0.0;
        s = q < 0.0 ? 1.0 : -1.0;
    } else if (std::fabs(p) > std::fabs(q)) {
        const double t = q / p;
        double u = std::sqrt(1.0 + t * t);
        if (p < 0.0) u = -u;
        c = 1.0 / u;
        s = -t * c;
    } else {
        const double t = p / q;
        double u = std::sqrt(1.0 + t * t);
        if (q < 0.0) u = -u;
        s = -1.0 / u;
        c = -t * s;
    }
}

// tridiagonal_qr_step<ColMajor>: Q (row-major n x n here) = Q * G_k for each rotation
void tridiagonal_qr_step(double* diag, double* sub, int start, int end, double* Q, int n) {
    const double td = (diag[end - 1] - diag[end]) * 0.5;
    const double e = sub[end - 1];
    double mu = diag[end];
    if (td == 0.0) {
        mu -= std::fabs(e);
    } else {
        const double e2 = e * e;
        const double h = eigen_hypot(td, e);
        if (e2 == 0.0)
            mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / h);
        else
            mu -= e2 / (td + (td > 0.0 ? h : -h));
    }
    double x = diag[start] - mu;
    double z = sub[start];
    for (int k = start; k < end; ++k) {
        double c, s;
        make_givens(x, z, c, s);
        const double sdk = s * diag[k] + c * sub[k];
        const double dkp1 = s * sub[k] + c * diag[k + 1];
        diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
        diag[k + 1] = s * sdk + c * dkp1;
        sub[k] = c * sdk - s * dkp1;
        if (k > start) sub[k - 1] = c * sub[k - 1] - s * z;
        x = sub[k];
        if (k < end - 1) {
            z = -s * sub[k + 1];
            sub[k + 1] = c * sub[k + 1];
        }
        // q.applyOnTheRight(k, k+1, rot): apply_rotation_in_the_plane(col k, col k+1, rot^T)
        for (int i = 0; i < n; ++i) {
            const double xi = Q[i * n + k], yi = Q[i * n + k + 1];
            Q[i * n + k] = c * xi - s * yi;
            Q[i * n + k + 1] = s * xi + c * yi;
        }
    }
}

// computeFromTridiagonal_impl (maxIterations = 30); returns 0 (Success) or 1 (NoConvergence)
int compute_from_tridiagonal(int n, double* diag, double* sub, double* Q) {
    int end = n - 1, start = 0, iter = 0;
    const double consider_as_zero = DBL_MIN;
    const double precision = 2.0 * DBL_EPSILON;
    while (end > 0) {
        for (int i = start; i < end; ++i)
            if (std::fabs(sub[i]) <= (std::fabs(diag[i]) + std::fabs(diag[i + 1])) * precision ||
                std::fabs(sub[i]) <= consider_as_zero)
                sub[i] = 0.0;
        while (end > 0 && sub[end - 1] == 0.0) end--;
        if (end <= 0) break;
        iter++;
        if (iter > 30 * n) break;
        start = end - 1;
        while (start > 0 && sub[start - 1] != 0.0) start--;
        tridiagonal_qr_step(diag, sub, start, end, Q, n);
    }
    if (iter > 30 * n) return 1;
    for (int i = 0; i < n - 1; ++i) {   // diag.segment(i, n-i).minCoeff(&k): first index of the minimum
        int k = 0;
        for (int j = 1; j < n - i; ++j)
            if (diag[i + j] < diag[i + k]) k = j;
        if (k > 0) {
            std::swap(diag[i], diag[i + k]);
            for (int r = 0; r < n; ++r) std::swap(Q[r * n + i], Q[r * n + i + k]);
        }
    }
    return 0;
}

}  // namespace

extern "C" int lmsfo_saes3(const double a[9], double d[3], double v[9]) {
    // mat = A.triangularView<Lower>(); scale = mat.cwiseAbs().maxCoeff()
    double m00 = a[0], m10 = a[3], m20 = a[6], m11 = a[4], m21 = a[7], m22 = a[8];
    double scale = 0.0;
    for (double t : {m00, m10, m20, m11, m21, m22}) scale = std::fabs(t) > scale ? std::fabs(t) : scale;
    if (scale == 0.0) scale = 1.0;
    m00 /= scale; m10 /= scale; m20 /= scale; m11 /= scale; m21 /= scale; m22 /= scale;
    // tridiagonalization_inplace_selector<MatrixType, 3, false>::run
    double diag[3], sub[2];
    diag[0] = m00;
    const double v1norm2 = m20 * m20;
    if (v1norm2 <= DBL_MIN) {
        diag[1] = m11; diag[2] = m22;
        sub[0] = m10; sub[1] = m21;
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        std::memcpy(v, I, sizeof I);
    } else {
        const double beta = std::sqrt(m10 * m10 + v1norm2);
        const double inv_beta = 1.0 / beta;
        const double m01 = m10 * inv_beta;
        const double m02 = m20 * inv_beta;
        const double q = 2.0 * m01 * m21 + m02 * (m22 - m11);
        diag[1] = m11 + m02 * q;
        diag[2] = m22 - m02 * q;
        sub[0] = beta;
        sub[1] = m21 - m01 * q;
        const double Q[9] = {1, 0, 0, 0, m01, m02, 0, m02, -m01};
        std::memcpy(v, Q, sizeof Q);
    }
    const int info = compute_from_tridiagonal(3, diag, sub, v);
    for (int i = 0; i < 3; ++i) d[i] = diag[i] * scale;
    return info;
}

extern "C" int lmsfo_saesx(int n, const double* a, double* d, double* v) {
    if (n < 1 || n > 8) return -1;
    double M[64];
    double scale = 0.0;
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
            M[r * n + c] = c <= r ? a[r * n + c] : 0.0;
            if (std::fabs(M[r * n + c]) > scale) scale = std::fabs(M[r * n + c]);
        }
    if (n == 1) {   // compute(): n == 1 -> eigenvalue = the entry, eigenvector 1
        d[0] = a[0];
        v[0] = 1.0;
        return 0;
    }
    if (scale == 0.0) scale = 1.0;
    for (int r = 0; r < n; ++r)
        for (int c = 0; c <= r; ++c) M[r * n + c] /= scale;
    // Tridiagonalization.h tridiagonalization_inplace(matA, hCoeffs)
    double hc[8];
    for (int i = 0; i < n - 1; ++i) {
        const int rem = n - i - 1;
        double* col = M + (i + 1) * n + i;            // v = M[i+1.., i], stride n
        // makeHouseholderInPlace: c0 stays, the tail becomes the essential part
        const double c0 = col[0];
        double tail = 0.0;
        for (int r = 1; r < rem; ++r) tail += col[r * n] * col[r * n];
        double tau, beta;
        if (tail <= DBL_MIN) {
            tau = 0.0;
            beta = c0;
            for (int r = 1; r < rem; ++r) col[r * n] = 0.0;
        } else {
            beta = std::sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            for (int r = 1; r < rem; ++r) col[r * n] = col[r * n] / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        col[0] = 1.0;
        double w[8], hv[8];
        for (int r = 0; r < rem; ++r) hv[r] = tau * col[r * n];
        // hCoeffs.tail = bottomRightCorner.selfadjointView<Lower>() * (tau v)
        for (int r = 0; r < rem; ++r) {
            double s = 0.0;
            for (int c = 0; c < rem; ++c) {
                const int R = i + 1 + (r > c ? r : c), Cc = i + 1 + (r > c ? c : r);
                s += M[R * n + Cc] * hv[c];
            }
            w[r] = s;
        }
        // hCoeffs.tail += (tau * -0.5 * (hCoeffs.tail . v)) * v
        double dt = 0.0;
        for (int r = 0; r < rem; ++r) dt += w[r] * col[r * n];
        const double alpha = tau * -0.5 * dt;
        for (int r = 0; r < rem; ++r) w[r] += alpha * col[r * n];
        // selfadjointView<Lower>().rankUpdate(v, w, -1): lower += -(v w^T + w v^T)
        for (int c = 0; c < rem; ++c)
            for (int r = c; r < rem; ++r)
                M[(i + 1 + r) * n + (i + 1 + c)] += (-1.0 * col[c * n]) * w[r] + (-1.0 * w[c]) * col[r * n];
        col[0] = beta;
        hc[i] = tau;
    }
    double diag[8], sub[8];
    for (int i = 0; i < n; ++i) diag[i] = M[i * n + i];
    for (int i = 0; i < n - 1; ++i) sub[i] = M[(i + 1) * n + i];
    // Q = HouseholderSequence(M, hc).setLength(n - 1).setShift(1), evaluated: I, then for k = n-2 .. 0
    // the bottom-right (n-k-1) corner gets applyHouseholderOnTheLeft(M[k+2.., k], hc[k])
    double Q[64];
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) Q[r * n + c] = r == c ? 1.0 : 0.0;
    for (int k = n - 2; k >= 0; --k) {
        const int o = k + 1, cs = n - k - 1;
        const double tau = hc[k];
        if (cs == 1) {
            Q[o * n + o] *= (1.0 - tau);
        } else if (tau != 0.0) {
            for (int c = o; c < n; ++c) {
                double tmp = 0.0;
                for (int r = 1; r < cs; ++r) tmp += M[(o + r) * n + k] * Q[(o + r) * n + c];
                tmp += Q[o * n + c];
                Q[o * n + c] -= tau * tmp;
                for (int r = 1; r < cs; ++r) Q[(o + r) * n + c] -= (tau * M[(o + r) * n + k]) * tmp;
            }
        }
    }
    const int info = compute_from_tridiagonal(n, diag, sub, Q);
    for (int i = 0; i < n; ++i) d[i] = diag[i] * scale;
    std::memcpy(v, Q, sizeof(double) * n * n);
    return info;
}
