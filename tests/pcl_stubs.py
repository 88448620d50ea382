"""Stand-in PCL / Eigen headers for compiling include/lmsf/lmsf_pcl.hpp's adapters against the reference's own
plugin bases (REG/registration_base.hpp:25-34, processing/process_base.hpp:26-39, Sensor/lidar_data_type.h), which
are included in place from /root/reference -- never copied.  PCL and Eigen are absent from the image; the stubs hold
only what those headers and the adapters touch.  Test infrastructure: used by tests/test_abi.py (the compile test)
and by __graft_entry__.build() (tests/cpp/bin/pcl_adapter_run, the runner tests/test_gpu_adapters.py executes on
the GPU box, where the reference tree is absent)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REF_INCLUDE = "/root/reference/src/MultiSensorFusionEstimator3D/include"

# Minimal stand-ins for the third-party headers the reference's plugin bases include (PCL, Eigen): only what
# registration_base.hpp / process_base.hpp / Sensor/lidar_data_type.h and the adapters touch.  Generated into
# tmp_path by the test; the reference's own headers are included in place, never copied.
_STUB_EIGEN = r"""
#pragma once
#include <cmath>
namespace Eigen {
struct Vector3d {
    double v[3];
    Vector3d() : v{0, 0, 0} {}
    Vector3d(double a, double b, double c) : v{a, b, c} {}
    double& x() { return v[0]; } double& y() { return v[1]; } double& z() { return v[2]; }
    double x() const { return v[0]; } double y() const { return v[1]; } double z() const { return v[2]; }
};
struct Matrix3d {
    double m[9];
    double& operator()(int r, int c) { return m[3 * r + c]; }
    double operator()(int r, int c) const { return m[3 * r + c]; }
    static Matrix3d Identity() { Matrix3d a{{1, 0, 0, 0, 1, 0, 0, 0, 1}}; return a; }
};
struct Matrix4f {
    float m[16];
    static Matrix4f Identity() { Matrix4f a{}; a.m[0] = a.m[5] = a.m[10] = a.m[15] = 1.f; return a; }
};
struct Quaterniond {
    double x_, y_, z_, w_;
    Quaterniond(double w, double x, double y, double z) : x_(x), y_(y), z_(z), w_(w) {}
    explicit Quaterniond(const Matrix3d& R) {   // Eigen's quaternion-from-matrix
        const double tr = R(0, 0) + R(1, 1) + R(2, 2);
        double q[4];
        if (tr > 0) {
            double t = std::sqrt(tr + 1.0); q[3] = 0.5 * t; t = 0.5 / t;
            q[0] = (R(2, 1) - R(1, 2)) * t; q[1] = (R(0, 2) - R(2, 0)) * t; q[2] = (R(1, 0) - R(0, 1)) * t;
        } else {
            int i = 0; if (R(1, 1) > R(0, 0)) i = 1; if (R(2, 2) > R(i, i)) i = 2;
            const int j = (i + 1) % 3, k = (j + 1) % 3;
            double t = std::sqrt(R(i, i) - R(j, j) - R(k, k) + 1.0); q[i] = 0.5 * t; t = 0.5 / t;
            q[3] = (R(k, j) - R(j, k)) * t; q[j] = (R(j, i) + R(i, j)) * t; q[k] = (R(k, i) + R(i, k)) * t;
        }
        x_ = q[0]; y_ = q[1]; z_ = q[2]; w_ = q[3];
    }
    double x() const { return x_; } double y() const { return y_; } double z() const { return z_; }
    double w() const { return w_; }
    Matrix3d toRotationMatrix() const {
        const double tx = 2 * x_, ty = 2 * y_, tz = 2 * z_, twx = tx * w_, twy = ty * w_, twz = tz * w_;
        const double txx = tx * x_, txy = ty * x_, txz = tz * x_, tyy = ty * y_, tyz = tz * y_, tzz = tz * z_;
        Matrix3d R{{1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                    txz - twy, tyz + twx, 1 - (txx + tyy)}};
        return R;
    }
};
struct Isometry3d {
    Matrix3d R = Matrix3d::Identity();
    Vector3d t;
    static Isometry3d Identity() { return Isometry3d(); }
    Matrix3d rotation() const { return R; }
    Matrix3d& linear() { return R; }
    Vector3d& translation() { return t; }
    const Vector3d& translation() const { return t; }
};
}  // namespace Eigen
"""

_STUB_PCL_CLOUD = r"""
#pragma once
#include <cstddef>
#include <memory>
#include <vector>
namespace pcl {
template <typename P>
struct PointCloud {
    std::vector<P> points;
    using Ptr = std::shared_ptr<PointCloud<P>>;
    using ConstPtr = std::shared_ptr<const PointCloud<P>>;
    std::size_t size() const { return points.size(); }
    bool empty() const { return points.empty(); }
    void resize(std::size_t n) { points.resize(n); }
};
}  // namespace pcl
"""

_STUB_PCL_TYPES = r"""
#pragma once
#include <Eigen/Core>   /* pcl/point_types.h brings Eigen in, as the real one does */
namespace pcl {
struct PointXYZI { float x, y, z, intensity; };
}  // namespace pcl
"""


def write_stubs(root):
    """The stand-in headers under `root` (a directory, created)."""
    for rel, text in (("lmsf_stub_eigen.hpp", _STUB_EIGEN),
                      ("eigen3/Eigen/Dense", '#pragma once\n#include "../../lmsf_stub_eigen.hpp"\n'),
                      ("Eigen/Core", '#pragma once\n#include "../lmsf_stub_eigen.hpp"\n'),
                      ("pcl/point_cloud.h", _STUB_PCL_CLOUD),
                      ("pcl/point_types.h", _STUB_PCL_TYPES),
                      ("pcl/kdtree/kdtree_flann.h", "#pragma once\n"),
                      ("pcl/common/transforms.h", "#pragma once\n")):
        p = os.path.join(str(root), rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(text)


def adapter_cmd(stub, src, exe, rpath=None):
    """g++ line of a program using the adapters: reference headers in place, stubs, liblmsf_hip.so."""
    lib_dir = os.path.join(REPO, "lmsf-slam_amd")
    return ["g++", "-std=c++14", "-O1", "-Wall", "-Wextra", "-Werror=suggest-override", "-Werror=overloaded-virtual",
            "-Wno-unused-parameter", "-I", str(stub), "-I", REF_INCLUDE, "-I", os.path.join(REPO, "include"), str(src),
            "-L", lib_dir, "-llmsf_hip", f"-Wl,-rpath,{rpath or lib_dir}", "-o", str(exe)]


RUNNER_SRC = os.path.join(REPO, "tests", "cpp", "pcl_adapter_run.cpp")
RUNNER = os.path.join(REPO, "tests", "cpp", "bin", "pcl_adapter_run")


def build_runner():
    """tests/cpp/bin/pcl_adapter_run (git-ignored, shipped to the GPU box with the tree) when the reference headers
    are present; returns its path or None."""
    if not os.path.isdir(REF_INCLUDE):
        return None
    bin_dir = os.path.dirname(RUNNER)
    stub = os.path.join(bin_dir, "stub")
    write_stubs(stub)
    if (os.path.exists(RUNNER) and os.path.getmtime(RUNNER) >= os.path.getmtime(RUNNER_SRC) and
            os.path.getmtime(RUNNER) >= os.path.getmtime(os.path.join(REPO, "include", "lmsf", "lmsf_pcl.hpp"))):
        return RUNNER
    subprocess.run(adapter_cmd(stub, RUNNER_SRC, RUNNER, rpath="$ORIGIN/../../../lmsf-slam_amd"), check=True)
    return RUNNER
