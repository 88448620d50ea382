// Test infrastructure: the reference-side PCL adapters (include/lmsf/lmsf_pcl.hpp) run on a device, driven only
// through the reference's own plugin interfaces -- RegistrationBase<P> (REG/registration_base.hpp:25-34) and
// PointCloudProcessBase<P, P> (processing/process_base.hpp:26-39) -- the way its estimator holds them
// (ML_SystemFactory.hpp: LOAM processor (16, 2, 80), CeresEdgeSurfFeatureRegistration("loam_edge", "loam_surf"),
// the sparse_point_plane_icp preprocessor PointCloudCommonProcess("filtered") with VoxelGrid + DistanceFilter).
// Built by __graft_entry__.build() against the reference headers in place (tests/pcl_stubs.py); run by
// tests/test_gpu_adapters.py, which checks the outputs against the CPU oracle.
//
//   pcl_adapter_run scan.bin edge_map.bin surf_map.bin out_dir qx qy qz qw tx ty tz voxel near far
//   (.bin: float32 x y z intensity rows) -> out_dir/{loam_edge,loam_surf,filtered}.bin, out_dir/T.bin (R row-major,
//   t: 12 doubles), stdout "constructed 3".
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "lmsf/lmsf_pcl.hpp"
#ifndef LMSF_HAVE_PCL_REFERENCE
#error "the adapters were not enabled"
#endif

using P = pcl::PointXYZI;

static pcl::PointCloud<P> read_cloud(const char* path) {
    pcl::PointCloud<P> c;
    FILE* f = std::fopen(path, "rb");
    if (!f) throw std::runtime_error(std::string("cannot open ") + path);
    std::fseek(f, 0, SEEK_END);
    const long bytes = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    c.resize((size_t)bytes / sizeof(P));
    if (c.size() && std::fread(c.points.data(), sizeof(P), c.size(), f) != c.size()) throw std::runtime_error("short read");
    std::fclose(f);
    return c;
}

static void write_cloud(const std::string& path, const pcl::PointCloud<P>& c) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    if (c.size()) std::fwrite(c.points.data(), sizeof(P), c.size(), f);
    std::fclose(f);
}

// The estimator's front end (ML_System: preprocess -> extract -> register) through the base interfaces only.
static void front_end(Algorithm::PointCloudProcessBase<P, P>& extract, Algorithm::PointCloudProcessBase<P, P>& pre,
                      Algorithm::RegistrationBase<P>& reg, const Slam3D::LidarData<P>& scan,
                      const pcl::PointCloud<P>& edge_map, const pcl::PointCloud<P>& surf_map, Eigen::Isometry3d& T,
                      Slam3D::CloudContainer<P>& feats, Slam3D::CloudContainer<P>& filtered) {
    extract.Process(scan, feats);
    pre.Process(scan, filtered);
    reg.SetInputSource(std::make_pair(std::string("loam_edge"),
                                      typename pcl::PointCloud<P>::ConstPtr(new pcl::PointCloud<P>(edge_map))));
    reg.SetInputSource(std::make_pair(std::string("loam_surf"),
                                      typename pcl::PointCloud<P>::ConstPtr(new pcl::PointCloud<P>(surf_map))));
    reg.SetInputTarget(feats.pointcloud_data_);
    reg.Solve(T);
}

int main(int argc, char** argv) {
    if (argc != 15) {
        std::fprintf(stderr, "usage: %s scan edge_map surf_map out_dir qx qy qz qw tx ty tz voxel near far\n", argv[0]);
        return 2;
    }
    try {
        Slam3D::LidarData<P> scan;
        scan.point_cloud = read_cloud(argv[1]);
        const pcl::PointCloud<P> edge_map = read_cloud(argv[2]), surf_map = read_cloud(argv[3]);
        const std::string out = argv[4];
        double x[7];
        for (int i = 0; i < 7; ++i) x[i] = std::atof(argv[5 + i]);
        Algorithm::HipLOAMFeatureProcessor<P, P> fx(16, 2, 80);
        Algorithm::HipPointCloudCommonProcess<P> pre("filtered");
        pre.SetVoxelGrid("VoxelGrid", (float)std::atof(argv[12]));
        pre.SetDistanceFilter((float)std::atof(argv[13]), (float)std::atof(argv[14]));
        Algorithm::HipEdgeSurfFeatureRegistration<P> reg("loam_edge", "loam_surf");
        std::printf("constructed 3\n");
        Eigen::Isometry3d T = Eigen::Isometry3d::Identity();
        T.linear() = Eigen::Quaterniond(x[3], x[0], x[1], x[2]).toRotationMatrix();
        T.translation() = Eigen::Vector3d(x[4], x[5], x[6]);
        Slam3D::CloudContainer<P> feats, filtered;
        front_end(fx, pre, reg, scan, edge_map, surf_map, T, feats, filtered);
        for (const char* name : {"loam_edge", "loam_surf"}) write_cloud(out + "/" + name + ".bin", *feats.pointcloud_data_.at(name));
        write_cloud(out + "/filtered.bin", *filtered.pointcloud_data_.at("filtered"));
        double t[12];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) t[3 * r + c] = T.rotation()(r, c);
        for (int i = 0; i < 3; ++i) t[9 + i] = T.translation().v[i];
        FILE* f = std::fopen((out + "/T.bin").c_str(), "wb");
        if (!f || std::fwrite(t, sizeof(double), 12, f) != 12) throw std::runtime_error("cannot write T.bin");
        std::fclose(f);
    } catch (const std::exception& e) {
        std::printf("refused: %s\n", e.what());
        return 1;
    }
    return 0;
}
