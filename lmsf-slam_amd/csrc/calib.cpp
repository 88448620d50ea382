// Dual-LiDAR extrinsic initialisation: hand-eye calibration from the two trackers' inter-frame
// motions (AX = XB), host side of the C3 configuration.
//
// Restates Algorithm::HandEyeCalibrationBase (INC/Algorithm/calibration/handeye_calibration_base.hpp,
// INC = src/MultiSensorFusionEstimator3D/include) as called by MultiLidarSystem::process
// (INC/System/ML_System.hpp:268-281):
//   AddPose (:71-106)            screw-motion check, accumulate, keep <= 300 pose pairs (a max-heap
//                                on q.w replaces the smallest rotation once full)
//   checkScrewMotion (:207-242)  |angle_p - angle_s| <= 0.05 and |t_p.axis_p - t_s.axis_s| <= 0.1
//   CalibExRotation (:113-148)   rows L(q_p) - R(q_s) (Math.hpp:79-95), null vector of the stacked
//                                4N x 4 matrix, accepted when the 2nd-smallest singular value > 0.25
//   calibExTranslationNonPlanar  (R_p - I) t = q_x t_s - t_p, least squares (:160-184)
// Eigen's JacobiSVD is replaced by the eigen-decomposition of the 4x4 / 3x3 normal matrices
// (same singular vectors and values up to rounding; parity unpinned as for every Eigen call).
// The reference's checkScrewMotion falls off its end when both accumulated angles are 0 (UB);
// here that case returns false.
#include <cmath>
#include <cstring>
#include <queue>
#include <utility>
#include <vector>

#include "lmsf/lmsf.h"

namespace {

struct Q { double x, y, z, w; };
struct P { Q q; double t[3]; };

Q qmul(const Q& a, const Q& b) {     // Eigen quaternion product a * b
    return {a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
            a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}

Q qnormalized(Q q) {
    const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    return {q.x / n, q.y / n, q.z / n, q.w / n};
}

void cross(const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

void rotate(const Q& q, const double* v, double* out) {   // Eigen _transformVector
    const double qv[3] = {q.x, q.y, q.z};
    double uv[3], uv2[3];
    cross(qv, v, uv);
    for (double& u : uv) u += u;
    cross(qv, uv, uv2);
    for (int i = 0; i < 3; ++i) out[i] = v[i] + q.w * uv[i] + uv2[i];
}

void qmat(const Q& q, double* R) {   // toRotationMatrix
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z, twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x, tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

Q quat_from_R(const double* m) {     // Eigen Quaterniond(Matrix3d)
    double a[4];                     // x, y, z, w
    const double tr = m[0] + m[4] + m[8];
    if (tr > 0) {
        double t = std::sqrt(tr + 1.0);
        a[3] = 0.5 * t;
        t = 0.5 / t;
        a[0] = (m[7] - m[5]) * t;
        a[1] = (m[2] - m[6]) * t;
        a[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        double t = std::sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
        a[i] = 0.5 * t;
        t = 0.5 / t;
        a[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        a[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        a[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    }
    return {a[0], a[1], a[2], a[3]};
}

P identity() { return {{0, 0, 0, 1}, {0, 0, 0}}; }

P from16(const double* T) {          // Pose(const Isometry3d&) (pose.hpp:59-67)
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    return {qnormalized(quat_from_R(R)), {T[3], T[7], T[11]}};
}

P mul(const P& a, const P& b) {      // Pose::operator* (pose.hpp:95-98): q normalised by the ctor
    P c;
    c.q = qnormalized(qmul(a.q, b.q));
    rotate(a.q, b.t, c.t);
    for (int i = 0; i < 3; ++i) c.t[i] += a.t[i];
    return c;
}

void angle_axis(const Q& q, double* angle, double* axis) {   // Eigen AngleAxis(const Quaternion&)
    double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z);
    if (n != 0) {
        *angle = 2 * std::atan2(n, std::fabs(q.w));
        if (q.w < 0) n = -n;
        axis[0] = q.x / n; axis[1] = q.y / n; axis[2] = q.z / n;
    } else {
        *angle = 0;
        axis[0] = 1; axis[1] = 0; axis[2] = 0;
    }
}

// Cyclic Jacobi eigen-decomposition of a symmetric n x n matrix (row-major, destroyed);
// eigenvalues d, eigenvectors in the columns of v.
void jacobi(double* a, int n, double* d, double* v) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) v[i * n + j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) off += a[p * n + q] * a[p * n + q];
        if (off < 1e-300) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = a[p * n + q];
                if (apq == 0) continue;
                const double theta = (a[q * n + q] - a[p * n + p]) / (2 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
                const double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; ++k) {       // A <- A J
                    const double akp = a[k * n + p], akq = a[k * n + q];
                    a[k * n + p] = c * akp - s * akq;
                    a[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {       // A <- J^T A
                    const double apk = a[p * n + k], aqk = a[q * n + k];
                    a[p * n + k] = c * apk - s * aqk;
                    a[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = v[k * n + p], vkq = v[k * n + q];
                    v[k * n + p] = c * vkp - s * vkq;
                    v[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < n; ++i) d[i] = a[i * n + i];
}

constexpr double kEpsR = 0.05, kEpsT = 0.1, kRotCovThre = 0.25;
constexpr size_t kNPose = 300;

using Entry = std::pair<uint16_t, std::pair<P, P>>;
struct RotCmp {   // max-heap on the primary rotation's w (= smallest rotation on top) (:24-31)
    bool operator()(const Entry& r, const Entry& l) const { return l.second.first.q.w > r.second.first.q.w; }
};

}  // namespace

struct lmsf_handeye {
    std::priority_queue<Entry, std::vector<Entry>, RotCmp> heap;
    std::queue<Entry> fresh;
    std::vector<std::pair<P, P>> storage;
    std::vector<double> blocks;   // 16 doubles per stored pair: L(q_p) - R(q_s)
    P acc_p = identity(), acc_s = identity();
    Q ext_q{0, 0, 0, 1};
    double ext_t[3] = {0, 0, 0};
    bool done = false;

    bool check_screw(const P& p, const P& s) {
        double ap, as, xp[3], xs[3];
        angle_axis(p.q, &ap, xp);
        angle_axis(s.q, &as, xs);
        const double r_dis = std::fabs(ap - as);
        const double t_dis = std::fabs((p.t[0] * xp[0] + p.t[1] * xp[1] + p.t[2] * xp[2]) -
                                       (s.t[0] * xs[0] + s.t[1] * xs[1] + s.t[2] * xs[2]));
        if (r_dis > kEpsR || t_dis > kEpsT) {
            acc_p = acc_s = identity();
            return false;
        }
        acc_p = mul(acc_p, p);
        acc_s = mul(acc_s, s);
        double a1, a2, ax[3];
        angle_axis(acc_p.q, &a1, ax);
        angle_axis(acc_s.q, &a2, ax);
        return a1 > 0 || a2 > 0;
    }
};

extern "C" {

lmsf_status lmsf_handeye_create(lmsf_handeye** out) {
    if (!out) return LMSF_ERR_ARG;
    *out = new lmsf_handeye();
    (*out)->storage.reserve(kNPose);
    (*out)->blocks.assign(kNPose * 16, 0.0);
    return LMSF_OK;
}

void lmsf_handeye_destroy(lmsf_handeye* h) { delete h; }

lmsf_status lmsf_handeye_add_pose(lmsf_handeye* h, const double primary[16], const double sub[16], int32_t* ok) {
    if (!h || !primary || !sub || !ok) return LMSF_ERR_ARG;
    *ok = 0;
    if (!h->check_screw(from16(primary), from16(sub))) return LMSF_OK;
    const std::pair<P, P> pr(h->acc_p, h->acc_s);
    if (h->storage.size() < kNPose) {
        const uint16_t idx = (uint16_t)h->storage.size();
        h->fresh.emplace(idx, pr);
        h->heap.emplace(idx, pr);
        h->storage.push_back(pr);
    } else {                                   // replace the smallest rotation (:89-98)
        const uint16_t pos = h->heap.top().first;
        h->storage[pos] = pr;
        h->fresh.emplace(pos, pr);
        h->heap.pop();
        h->heap.emplace(pos, pr);
    }
    h->acc_p = h->acc_s = identity();
    *ok = h->storage.size() >= 3 ? 1 : 0;
    return LMSF_OK;
}

lmsf_status lmsf_handeye_calib_rotation(lmsf_handeye* h, int32_t* ok, double singular_values[4]) {
    if (!h || !ok) return LMSF_ERR_ARG;
    while (!h->fresh.empty()) {
        const Entry e = h->fresh.front();
        h->fresh.pop();
        const Q& a = e.second.first.q;    // primary
        const Q& b = e.second.second.q;   // sub
        const double L[16] = {a.w, -a.x, -a.y, -a.z, a.x, a.w, -a.z, a.y, a.y, a.z, a.w, -a.x, a.z, -a.y, a.x, a.w};
        const double R[16] = {b.w, -b.x, -b.y, -b.z, b.x, b.w, b.z, -b.y, b.y, -b.z, b.w, b.x, b.z, b.y, -b.x, b.w};
        for (int i = 0; i < 16; ++i) h->blocks[(size_t)e.first * 16 + i] = L[i] - R[i];
    }
    double M[16] = {0};                        // Q^T Q over the stored blocks
    for (size_t k = 0; k < h->storage.size(); ++k) {
        const double* B = &h->blocks[k * 16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                for (int r = 0; r < 4; ++r) M[i * 4 + j] += B[r * 4 + i] * B[r * 4 + j];
    }
    double d[4], V[16];
    jacobi(M, 4, d, V);
    int order[4] = {0, 1, 2, 3};              // descending singular values (JacobiSVD order)
    for (int i = 0; i < 4; ++i)
        for (int j = i + 1; j < 4; ++j)
            if (d[order[j]] > d[order[i]]) std::swap(order[i], order[j]);
    double sv[4];
    for (int i = 0; i < 4; ++i) sv[i] = std::sqrt(std::fmax(d[order[i]], 0.0));
    if (singular_values) std::memcpy(singular_values, sv, sizeof sv);
    double x[4];
    for (int i = 0; i < 4; ++i) x[i] = V[i * 4 + order[3]];   // [w, x, y, z]
    if (x[0] < 0)
        for (double& v : x) v = -v;
    *ok = 0;
    if (sv[2] > kRotCovThre) {
        h->ext_q = qnormalized(Q{x[1], x[2], x[3], x[0]});
        *ok = 1;
    }
    return LMSF_OK;
}

lmsf_status lmsf_handeye_calib_translation(lmsf_handeye* h, int32_t* ok) {
    if (!h || !ok) return LMSF_ERR_ARG;
    double AtA[9] = {0}, Atb[3] = {0};
    for (const auto& pr : h->storage) {
        double R[9], qt[3], b[3];
        qmat(pr.first.q, R);
        R[0] -= 1; R[4] -= 1; R[8] -= 1;
        rotate(h->ext_q, pr.second.t, qt);
        for (int i = 0; i < 3; ++i) b[i] = qt[i] - pr.first.t[i];
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j)
                for (int r = 0; r < 3; ++r) AtA[i * 3 + j] += R[r * 3 + i] * R[r * 3 + j];
            for (int r = 0; r < 3; ++r) Atb[i] += R[r * 3 + i] * b[r];
        }
    }
    double d[3], V[9];
    jacobi(AtA, 3, d, V);                      // minimum-norm least squares (JacobiSVD::solve)
    const double dmax = std::fmax(std::fmax(d[0], d[1]), d[2]);
    double x[3] = {0, 0, 0};
    for (int k = 0; k < 3; ++k) {
        if (d[k] <= dmax * 1e-24 || d[k] <= 0) continue;
        double proj = 0;
        for (int r = 0; r < 3; ++r) proj += V[r * 3 + k] * Atb[r];
        for (int r = 0; r < 3; ++r) x[r] += V[r * 3 + k] * proj / d[k];
    }
    std::memcpy(h->ext_t, x, sizeof x);
    h->done = true;
    *ok = 1;
    return LMSF_OK;
}

lmsf_status lmsf_handeye_result(const lmsf_handeye* h, double T[16], int32_t* ok) {
    if (!h || !T || !ok) return LMSF_ERR_ARG;
    *ok = h->done ? 1 : 0;
    if (!h->done) return LMSF_OK;
    double R[9];
    qmat(h->ext_q, R);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[4 * i + j] = R[3 * i + j];
        T[4 * i + 3] = h->ext_t[i];
    }
    T[12] = T[13] = T[14] = 0;
    T[15] = 1;
    return LMSF_OK;
}

lmsf_status lmsf_handeye_pair_count(const lmsf_handeye* h, int32_t* n) {
    if (!h || !n) return LMSF_ERR_ARG;
    *n = (int32_t)h->storage.size();
    return LMSF_OK;
}

}  // extern "C"
