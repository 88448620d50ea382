// TEST INFRASTRUCTURE ONLY -- CPU restatement of pcl::VoxelGrid::applyFilter (PCL 1.7
// voxel_grid.hpp) as wrapped by Algorithm::VoxelGridFilter (INC/Algorithm/PointClouds/processing/
// Filter/voxel_grid.hpp:25-34, filter_base.hpp:34-45), with the build's determinism choices
// (stable order inside a voxel, double centroid sums) -- see lmsf-slam_amd/csrc/k_voxel.hip.
// Parity vs PCL: unpinned (PCL sums in float in std::sort order).
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <vector>

#include "lmsf_oracle.h"

namespace {

int vox(float v, float inv) {
    const float f = std::floor(v * inv);
    return (int)std::fmin(std::fmax(f, -1073741824.f), 1073741824.f);
}

}  // namespace

extern "C" int64_t lmsfo_voxel_filter(const float* xyzi, int64_t n, float leaf, float* out) {
    if (n <= 0) return 0;
    const float inv = 1.0f / leaf;                 // inverse_leaf_size_ (float)
    std::vector<int> c(3 * (size_t)n);
    int lo[3] = {INT_MAX, INT_MAX, INT_MAX}, hi[3] = {INT_MIN, INT_MIN, INT_MIN};
    for (int64_t i = 0; i < n; ++i)
        for (int d = 0; d < 3; ++d) {
            const int v = vox(xyzi[4 * i + d], inv);
            c[3 * i + d] = v;
            lo[d] = std::min(lo[d], v);
            hi[d] = std::max(hi[d], v);
        }
    const int64_t dx = (int64_t)hi[0] - lo[0] + 1, dy = (int64_t)hi[1] - lo[1] + 1, dz = (int64_t)hi[2] - lo[2] + 1;
    if (dx * dy * dz > (int64_t)INT32_MAX) {      // PCL refuses: output = input
        std::copy(xyzi, xyzi + 4 * n, out);
        return n;
    }
    std::vector<uint64_t> key(n);
    for (int64_t i = 0; i < n; ++i)
        key[i] = ((uint64_t)(c[3 * i + 2] - lo[2]) * dy + (uint64_t)(c[3 * i + 1] - lo[1])) * dx +
                 (uint64_t)(c[3 * i] - lo[0]);
    std::vector<int64_t> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return key[a] < key[b]; });
    int64_t m = 0;
    for (int64_t a = 0; a < n;) {
        int64_t b = a;
        double s[4] = {0, 0, 0, 0};
        while (b < n && key[order[b]] == key[order[a]]) {
            for (int d = 0; d < 4; ++d) s[d] += xyzi[4 * order[b] + d];
            ++b;
        }
        const double cnt = (double)(b - a);
        for (int d = 0; d < 4; ++d) out[4 * m + d] = (float)(s[d] / cnt);
        ++m;
        a = b;
    }
    return m;
}
