// lmsf_pcl.hpp -- reference-side adapters: LMSF-Slam's plugin interfaces implemented on the C ABI of
// liblmsf_hip.so (include/lmsf/lmsf.h), for a maintainer to add to the reference build
// (INTEGRATION.md).  Compiled only where PCL and the reference's own headers are on the include path
// (the reference's include root, src/MultiSensorFusionEstimator3D/include); elsewhere this header
// is empty.
//
//   HipEdgeSurfFeatureRegistration<P>   RegistrationBase<P>     (REG/registration_base.hpp:25-34) as
//                                       CeresEdgeSurfFeatureRegistration (REG/ceres_edgeSurfFeatureRegistration.hpp)
//   HipLOAMFeatureProcessor<In, Out>    PointCloudProcessBase   (processing/process_base.hpp:26-39) as
//                                       LOAMFeatureProcessorBase (FX/LOAMFeatureProcessor_base.hpp:36-126)
//   HipPointCloudCommonProcess<P>       PointCloudProcessBase   as PointCloudCommonProcess
//                                       (processing/common_processing.hpp:39-122), the
//                                       "sparse_point_plane_icp" preprocessor
#pragma once

#if defined(__has_include)
#if __has_include(<pcl/point_cloud.h>) && __has_include("Algorithm/PointClouds/registration/registration_base.hpp")
#define LMSF_HAVE_PCL_REFERENCE 1
#endif
#endif

#ifdef LMSF_HAVE_PCL_REFERENCE
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include <lmsf/lmsf.h>

#include "Algorithm/PointClouds/processing/process_base.hpp"
#include "Algorithm/PointClouds/registration/registration_base.hpp"

namespace Algorithm {

namespace lmsf_pcl {
// PointXYZI payload rows (x, y, z, intensity): the layout of every lmsf cloud argument.
template <typename P>
std::vector<float> to_xyzi(pcl::PointCloud<P> const& c) {
    std::vector<float> v(4 * c.size());
    for (size_t i = 0; i < c.size(); ++i) {
        v[4 * i] = c.points[i].x;
        v[4 * i + 1] = c.points[i].y;
        v[4 * i + 2] = c.points[i].z;
        v[4 * i + 3] = c.points[i].intensity;
    }
    return v;
}

template <typename P>
typename pcl::PointCloud<P>::Ptr from_xyzi(std::vector<float> const& v, size_t n) {
    typename pcl::PointCloud<P>::Ptr pc(new pcl::PointCloud<P>());
    pc->resize(n);
    for (size_t i = 0; i < n; ++i) {
        pc->points[i].x = v[4 * i];
        pc->points[i].y = v[4 * i + 1];
        pc->points[i].z = v[4 * i + 2];
        pc->points[i].intensity = v[4 * i + 3];
    }
    return pc;
}

inline lmsf_ctx* make_ctx(lmsf_config const& cfg) {
    lmsf_ctx* c = nullptr;
    if (lmsf_ctx_create(&cfg, &c) != LMSF_OK) throw std::runtime_error("lmsf_ctx_create failed (no HIP device?)");
    return c;
}

// the current features of one kind of a context, as a PCL cloud
template <typename P>
typename pcl::PointCloud<P>::Ptr copy_kind(lmsf_ctx* c, int kind, size_t n) {
    std::vector<float> buf(4 * n);
    size_t got = 0;
    if (n && lmsf_copy_features(c, kind, buf.data(), nullptr, n, &got) != LMSF_OK) got = 0;
    return from_xyzi<P>(buf, got);
}
}  // namespace lmsf_pcl

// RegistrationBase<_PointType> (registration_base.hpp:25-34) on liblmsf_hip.so, with the semantics of
// CeresEdgeSurfFeatureRegistration(edge_name, surf_name): "" disables a kind (the sparse_point_plane_icp
// registration is ("", "filtered"), ML_SystemFactory.hpp:148-150).
template <typename _PointType>
class HipEdgeSurfFeatureRegistration : public RegistrationBase<_PointType> {
    using Base = RegistrationBase<_PointType>;
    std::string edge_name_, surf_name_;
    lmsf_ctx* ctx_ = nullptr;

  public:
    HipEdgeSurfFeatureRegistration(std::string const& edge_name, std::string const& surf_name, int device = 0)
        : edge_name_(edge_name), surf_name_(surf_name) {
        lmsf_config cfg;
        lmsf_config_init(&cfg);
        cfg.device = device;
        ctx_ = lmsf_pcl::make_ctx(cfg);
    }
    ~HipEdgeSurfFeatureRegistration() { lmsf_ctx_destroy(ctx_); }

    void SetInputSource(typename Base::SourceInput const& in) override {   // ceres_...:56-71
        if (in.second->empty()) return;
        const int kind = (!edge_name_.empty() && in.first == edge_name_) ? LMSF_EDGE
                         : (!surf_name_.empty() && in.first == surf_name_) ? LMSF_SURF : 0;
        if (!kind) return;
        auto v = lmsf_pcl::to_xyzi(*in.second);
        if (lmsf_set_map(ctx_, kind, v.data(), in.second->size()) != LMSF_OK)
            std::cout << "lmsf_set_map: " << lmsf_last_error(ctx_) << std::endl;
    }

    void SetInputTarget(FeaturePointCloudContainer<_PointType> const& in) override {   // :73-84
        for (int kind : {LMSF_EDGE, LMSF_SURF}) {
            auto it = in.find(kind == LMSF_EDGE ? edge_name_ : surf_name_);
            if (it == in.end()) continue;
            auto v = lmsf_pcl::to_xyzi(*it->second);
            lmsf_set_scan(ctx_, kind, v.data(), it->second->size());
        }
    }

    void SetMaxIteration(uint16_t const& n) { lmsf_set_max_iterations(ctx_, n); }   // :86-89

    void Solve(Eigen::Isometry3d& T) override {   // :96-130; failure: message, pose unchanged
        Eigen::Quaterniond q(T.rotation());
        double x[7] = {q.x(), q.y(), q.z(), q.w(), T.translation().x(), T.translation().y(), T.translation().z()};
        lmsf_solve_stats st;
        if (lmsf_solve(ctx_, x, &st) != LMSF_OK) {
            std::cout << "lmsf_solve: " << lmsf_last_error(ctx_) << std::endl;
            return;
        }
        T = Eigen::Isometry3d::Identity();
        T.linear() = Eigen::Quaterniond(x[3], x[0], x[1], x[2]).toRotationMatrix();
        T.translation() = Eigen::Vector3d(x[4], x[5], x[6]);
    }

    lmsf_ctx* context() const { return ctx_; }
};

// PointCloudProcessBase<In, Out> (process_base.hpp:26-39) as LOAMFeatureProcessorBase(N_SCANS, min,
// max, edge_thresh, voxel (unused by the reference, FX:48-49), RemovalBadPoints) (FX:36-50).
template <typename _InputPointT, typename _OutputFeatureT>
class HipLOAMFeatureProcessor : public PointCloudProcessBase<_InputPointT, _OutputFeatureT> {
    lmsf_ctx* ctx_ = nullptr;

  public:
    HipLOAMFeatureProcessor(uint16_t N_SCANS, float min_distance = 0, float max_distance = 9999,
                            float edge_thresh = 1, float /*surf_voxel_grid_size*/ = 0.1, bool RemovalBadPoints = true,
                            int device = 0) {
        lmsf_config cfg;
        lmsf_config_init(&cfg);
        cfg.device = device;
        cfg.n_scans = N_SCANS;
        cfg.min_distance = min_distance;
        cfg.max_distance = max_distance;
        cfg.edge_threshold = edge_thresh;
        cfg.remove_bad_points = RemovalBadPoints ? 1 : 0;
        ctx_ = lmsf_pcl::make_ctx(cfg);
    }
    ~HipLOAMFeatureProcessor() { lmsf_ctx_destroy(ctx_); }

    void Process(LidarData<_InputPointT> const& in, CloudContainer<_OutputFeatureT>& out) override {   // FX:59-126
        auto v = lmsf_pcl::to_xyzi(in.point_cloud);
        lmsf_feature_counts fc{0, 0};
        if (lmsf_extract_features(ctx_, v.data(), in.point_cloud.size(), &fc) != LMSF_OK) {
            std::cout << "lmsf_extract_features: " << lmsf_last_error(ctx_) << std::endl;
            return;
        }
        out.pointcloud_data_.insert(std::make_pair("loam_edge", lmsf_pcl::copy_kind<_OutputFeatureT>(ctx_, LMSF_EDGE, fc.n_edge)));
        out.pointcloud_data_.insert(std::make_pair("loam_surf", lmsf_pcl::copy_kind<_OutputFeatureT>(ctx_, LMSF_SURF, fc.n_surf)));
    }
};

// PointCloudCommonProcess<P>(output_name, removal_nan) (common_processing.hpp:39-122): SetVoxelGrid
// ("VoxelGrid" only), SetDistanceFilter, Process -> {output_name: removeNaN? -> VoxelGrid -> distance}.
template <typename _PointType>
class HipPointCloudCommonProcess : public PointCloudProcessBase<_PointType, _PointType> {
    std::string output_name_;
    lmsf_common_params prm_;
    lmsf_ctx* ctx_ = nullptr;

  public:
    HipPointCloudCommonProcess(std::string const& output_name, bool removal_nan = false, int device = 0)
        : output_name_(output_name) {
        lmsf_common_params_init(&prm_);
        prm_.removal_nan = removal_nan ? 1 : 0;
        prm_.voxel_leaf = 0.f;                 // unset until SetVoxelGrid, like the reference's filter
        prm_.distance_near = prm_.distance_far = 0.f;
        lmsf_config cfg;
        lmsf_config_init(&cfg);
        cfg.device = device;
        ctx_ = lmsf_pcl::make_ctx(cfg);
    }
    ~HipPointCloudCommonProcess() { lmsf_ctx_destroy(ctx_); }

    void SetVoxelGrid(std::string const& name, float cell_size) {
        if (name != "VoxelGrid") throw std::invalid_argument("HipPointCloudCommonProcess: VoxelGrid only");
        prm_.voxel_leaf = cell_size;
    }
    void SetDistanceFilter(float const& near_thresh, float const& far_thresh) {
        prm_.distance_near = near_thresh;
        prm_.distance_far = far_thresh;
    }

    void Process(LidarData<_PointType> const& in, CloudContainer<_PointType>& out) override {   // :87-112
        auto v = lmsf_pcl::to_xyzi(in.point_cloud);
        lmsf_feature_counts fc{0, 0};
        if (lmsf_common_process(ctx_, v.data(), in.point_cloud.size(), &prm_, &fc) != LMSF_OK) {
            std::cout << "lmsf_common_process: " << lmsf_last_error(ctx_) << std::endl;
            return;
        }
        out.pointcloud_data_.insert(std::make_pair(output_name_, lmsf_pcl::copy_kind<_PointType>(ctx_, LMSF_SURF, fc.n_surf)));
    }
};

}  // namespace Algorithm
#endif  // LMSF_HAVE_PCL_REFERENCE
