// C++ caller written against the reference's interfaces (RegistrationBase / PointCloudProcessBase),
// linked against liblmsf_hip.so.  Reads a raw scan and two maps from binary files (xyzi float32
// rows), extracts features, registers from a given initial pose, prints the result.
// Used by tests/test_gpu_parity.py::test_cpp_facade (build-only check on CPU in test_abi.py).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <vector>

#include "lmsf/lmsf.hpp"

static std::shared_ptr<lmsf::PointCloud> load(const char* path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    const size_t bytes = (size_t)f.tellg();
    f.seekg(0);
    auto c = std::make_shared<lmsf::PointCloud>(bytes / sizeof(lmsf::PointXYZI));
    f.read(reinterpret_cast<char*>(c->data()), (std::streamsize)bytes);
    return c;
}

int main(int argc, char** argv) {
    if (argc < 12) {
        std::fprintf(stderr, "usage: %s scan edge_map surf_map qx qy qz qw tx ty tz iters\n", argv[0]);
        return 2;
    }
    try {
        lmsf::LidarData scan;
        scan.point_cloud = *load(argv[1]);
        // factory: LOAMFeatureProcessorBase(16, 2, 80) + CeresEdgeSurfFeatureRegistration("loam_edge", "loam_surf")
        std::unique_ptr<lmsf::PointCloudProcessBase<lmsf::PointXYZI, lmsf::PointXYZI>> proc(
            new lmsf::LOAMFeatureProcessorHIP(16, 2, 80));
        std::unique_ptr<lmsf::EdgeSurfFeatureRegistrationHIP> reg(
            new lmsf::EdgeSurfFeatureRegistrationHIP("loam_edge", "loam_surf"));
        lmsf::CloudContainer feats;
        proc->Process(scan, feats);
        reg->SetInputSource({"loam_edge", load(argv[2])});
        reg->SetInputSource({"loam_surf", load(argv[3])});
        reg->SetInputTarget(feats.pointcloud_data_);
        reg->SetMaxIteration((uint16_t)std::atoi(argv[11]));
        lmsf::Isometry3d T;
        for (int i = 0; i < 4; ++i) T.q[i] = std::atof(argv[4 + i]);
        for (int i = 0; i < 3; ++i) T.t[i] = std::atof(argv[8 + i]);
        reg->Solve(T);
        std::printf("%zu %zu %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d\n",
                    feats.pointcloud_data_["loam_edge"]->size(), feats.pointcloud_data_["loam_surf"]->size(),
                    T.q[0], T.q[1], T.q[2], T.q[3], T.t[0], T.t[1], T.t[2], reg->LastStats().outer_iterations);
    } catch (const lmsf::Error& e) {
        std::fprintf(stderr, "lmsf error %d: %s\n", e.code, e.what());
        return 1;
    }
    return 0;
}
