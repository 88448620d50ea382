// lmsf.hpp -- header-only C++ facade over include/lmsf/lmsf.h that mirrors the reference's two
// plugin interfaces on the hot path, with PCL-free stand-in types:
//
//   Algorithm::RegistrationBase<P>          REG/registration_base.hpp:25-34
//     SetInputSource(pair<name, cloud>) / SetInputTarget(FeaturePointCloudContainer) / Solve(T)
//   Algorithm::PointCloudProcessBase<In,Out> INC/Algorithm/PointClouds/processing/process_base.hpp:26-39
//     Process(LidarData const&, CloudContainer&)
//   Slam3D::LidarData / CloudContainer / FeaturePointCloudContainer   INC/Sensor/lidar_data_type.h:29-66
//
// (INC = src/MultiSensorFusionEstimator3D/include, REG = INC/Algorithm/PointClouds/registration.)
// A PCL adapter for the reference build itself (pcl::PointCloud<P>, Eigen::Isometry3d) is shown
// in INTEGRATION.md.  Errors: the reference's Solve/Process return void and only print; here a
// failing call throws lmsf::Error (a C++ caller can catch and fall back to its own path).
#ifndef LMSF_LMSF_HPP_
#define LMSF_LMSF_HPP_

#include <cmath>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "lmsf.h"

namespace lmsf {

struct PointXYZI {
    float x, y, z, intensity;
};
using PointCloud = std::vector<PointXYZI>;
using PointCloudConstPtr = std::shared_ptr<const PointCloud>;
using FeaturePointCloudContainer = std::unordered_map<std::string, PointCloudConstPtr>;

struct LidarData {
    PointCloud point_cloud;
};
struct CloudContainer {
    double time_stamp_ = 0;
    FeaturePointCloudContainer pointcloud_data_;
};

// Rigid transform kept as the reference's parameter block (quaternion x y z w + translation,
// ceres_edgeSurfFeatureRegistration.hpp:38-40), convertible to a row-major 4x4 matrix.
struct Isometry3d {
    double q[4] = {0, 0, 0, 1};
    double t[3] = {0, 0, 0};

    static Isometry3d Identity() { return Isometry3d(); }
    // Eigen QuaternionBase::toRotationMatrix
    void matrix(double m[16]) const {
        const double x = q[0], y = q[1], z = q[2], w = q[3];
        const double tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w;
        const double txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
        const double r[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz),
                             tyz - twx,       txz - twy, tyz + twx, 1 - (txx + tyy)};
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) m[4 * i + j] = r[3 * i + j];
            m[4 * i + 3] = t[i];
        }
        m[12] = m[13] = m[14] = 0;
        m[15] = 1;
    }
    // Eigen quaternion from a rotation matrix (Shepperd's method, as Eigen's assignment)
    static Isometry3d FromMatrix(const double m[16]) {
        Isometry3d T;
        const double tr = m[0] + m[5] + m[10];
        if (tr > 0) {
            double s = std::sqrt(tr + 1.0);
            T.q[3] = 0.5 * s;
            s = 0.5 / s;
            T.q[0] = (m[9] - m[6]) * s;
            T.q[1] = (m[2] - m[8]) * s;
            T.q[2] = (m[4] - m[1]) * s;
        } else {
            int i = 0;
            if (m[5] > m[0]) i = 1;
            if (m[10] > m[5 * i]) i = 2;
            const int j = (i + 1) % 3, k = (i + 2) % 3;
            double s = std::sqrt(m[5 * i] - m[5 * j] - m[5 * k] + 1.0);
            T.q[i] = 0.5 * s;
            s = 0.5 / s;
            T.q[3] = (m[4 * k + j] - m[4 * j + k]) * s;
            T.q[j] = (m[4 * j + i] + m[4 * i + j]) * s;
            T.q[k] = (m[4 * k + i] + m[4 * i + k]) * s;
        }
        T.t[0] = m[3];
        T.t[1] = m[7];
        T.t[2] = m[11];
        return T;
    }
};

class Error : public std::runtime_error {
  public:
    Error(lmsf_status code, const std::string& msg) : std::runtime_error(msg), code(code) {}
    lmsf_status code;
};

namespace detail {
class Ctx {
  public:
    explicit Ctx(const lmsf_config& cfg) {
        lmsf_status rc = lmsf_ctx_create(&cfg, &ctx_);
        if (rc != LMSF_OK) throw Error(rc, "lmsf_ctx_create failed (HIP device or configuration)");
    }
    ~Ctx() { lmsf_ctx_destroy(ctx_); }
    Ctx(const Ctx&) = delete;
    Ctx& operator=(const Ctx&) = delete;
    lmsf_ctx* get() const { return ctx_; }
    void check(lmsf_status rc) const {
        if (rc != LMSF_OK) throw Error(rc, lmsf_last_error(ctx_));
    }

  private:
    lmsf_ctx* ctx_ = nullptr;
};
inline const float* xyzi(const PointCloud& c) { return reinterpret_cast<const float*>(c.data()); }
}  // namespace detail

// ---------------------------------------------------------------- plugin bases (reference names)
template <typename _PointType>
class RegistrationBase {
  public:
    using PointCloudConstPtr = std::shared_ptr<const std::vector<_PointType>>;
    using SourceInput = std::pair<std::string, PointCloudConstPtr>;
    virtual ~RegistrationBase() = default;
    virtual void SetInputSource(SourceInput const& source_input) = 0;
    virtual void SetInputTarget(FeaturePointCloudContainer const& target_input) = 0;
    virtual void Solve(Isometry3d& T) = 0;
};

template <typename _InPointT, typename _OutPointT>
class PointCloudProcessBase {
  public:
    virtual ~PointCloudProcessBase() = default;
    virtual void Process(LidarData const& data_in, CloudContainer& data_out) = 0;
};

// ---------------------------------------------------------------- MI355X implementations
// CeresEdgeSurfFeatureRegistration (solver = LMSF_SOLVER_CERES_LM) or EdgeSurfFeatureRegistration
// GN mode (LMSF_SOLVER_GN) on one device stream.
class EdgeSurfFeatureRegistrationHIP : public RegistrationBase<PointXYZI> {
  public:
    EdgeSurfFeatureRegistrationHIP(std::string const& edge_name, std::string const& surf_name,
                                   int32_t solver = LMSF_SOLVER_CERES_LM, int32_t device = 0,
                                   int32_t max_features = 1 << 17)
        : edge_name_(edge_name), surf_name_(surf_name), ctx_(make_cfg(solver, device, max_features)) {}

    void SetInputSource(SourceInput const& source_input) override {
        if (!source_input.second || source_input.second->empty()) return;  // ceres_...:60
        const int32_t kind = source_input.first == edge_name_ ? LMSF_EDGE
                             : source_input.first == surf_name_ ? LMSF_SURF : 0;
        if (!kind) return;
        ctx_.check(lmsf_set_map(ctx_.get(), kind, detail::xyzi(*source_input.second), source_input.second->size()));
    }
    void SetInputTarget(FeaturePointCloudContainer const& target_input) override {
        auto e = target_input.find(edge_name_);
        if (e != target_input.end() && e->second)
            ctx_.check(lmsf_set_scan(ctx_.get(), LMSF_EDGE, detail::xyzi(*e->second), e->second->size()));
        auto s = target_input.find(surf_name_);
        if (s != target_input.end() && s->second)
            ctx_.check(lmsf_set_scan(ctx_.get(), LMSF_SURF, detail::xyzi(*s->second), s->second->size()));
    }
    void SetMaxIteration(uint16_t n) { ctx_.check(lmsf_set_max_iterations(ctx_.get(), n)); }
    void Solve(Isometry3d& T) override {
        double x[7] = {T.q[0], T.q[1], T.q[2], T.q[3], T.t[0], T.t[1], T.t[2]};
        ctx_.check(lmsf_solve(ctx_.get(), x, &last_stats_));
        for (int i = 0; i < 4; ++i) T.q[i] = x[i];
        for (int i = 0; i < 3; ++i) T.t[i] = x[4 + i];
    }
    const lmsf_solve_stats& LastStats() const { return last_stats_; }
    lmsf_ctx* handle() const { return ctx_.get(); }

  private:
    static lmsf_config make_cfg(int32_t solver, int32_t device, int32_t max_features) {
        lmsf_config c;
        lmsf_config_init(&c);
        c.solver = solver;
        c.device = device;
        c.max_features = max_features;
        c.max_scan_points = max_features;
        return c;
    }
    std::string edge_name_, surf_name_;
    detail::Ctx ctx_;
    lmsf_solve_stats last_stats_{};
};

// LOAMFeatureProcessorBase(N_SCANS, min_distance, max_distance, edge_thresh, surf_voxel_grid_size,
// RemovalBadPoints) (FX/LOAMFeatureProcessor_base.hpp:36-50); outputs "loam_edge" / "loam_surf".
class LOAMFeatureProcessorHIP : public PointCloudProcessBase<PointXYZI, PointXYZI> {
  public:
    LOAMFeatureProcessorHIP(uint16_t N_SCANS, float min_distance = 0, float max_distance = 9999,
                            float edge_thresh = 1, float /*surf_voxel_grid_size: unused by the reference*/ = 0.1f,
                            bool RemovalBadPoints = true, int32_t device = 0, int32_t max_points = 1 << 17)
        : ctx_(make_cfg(N_SCANS, min_distance, max_distance, edge_thresh, RemovalBadPoints, device, max_points)) {}

    void Process(LidarData const& data_in, CloudContainer& data_out) override {
        lmsf_feature_counts fc{};
        ctx_.check(lmsf_extract_features(ctx_.get(), detail::xyzi(data_in.point_cloud), data_in.point_cloud.size(), &fc));
        data_out.pointcloud_data_.insert({"loam_edge", copy(LMSF_EDGE, (size_t)fc.n_edge)});
        data_out.pointcloud_data_.insert({"loam_surf", copy(LMSF_SURF, (size_t)fc.n_surf)});
    }

  private:
    PointCloudConstPtr copy(int32_t kind, size_t n) {
        auto out = std::make_shared<PointCloud>(n);
        size_t got = 0;
        ctx_.check(lmsf_copy_features(ctx_.get(), kind, reinterpret_cast<float*>(out->data()), nullptr, n, &got));
        out->resize(got);
        return out;
    }
    static lmsf_config make_cfg(uint16_t n_scans, float mn, float mx, float et, bool rb, int32_t device, int32_t mp) {
        lmsf_config c;
        lmsf_config_init(&c);
        c.n_scans = n_scans;
        c.min_distance = mn;
        c.max_distance = mx;
        c.edge_threshold = et;
        c.remove_bad_points = rb ? 1 : 0;
        c.device = device;
        c.max_scan_points = mp;
        c.max_features = mp;
        return c;
    }
    detail::Ctx ctx_;
};

}  // namespace lmsf

#endif  // LMSF_LMSF_HPP_
