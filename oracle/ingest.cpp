// TEST INFRASTRUCTURE ONLY -- CPU restatement of the scan ingest in front of the LOAM extraction:
// pcl::fromROSMsg + pcl::removeNaNFromPointCloud (src/apps/src/MultiLidarSLAM_node.cpp:125-132),
// RotaryLidarPreProcess::Process (INC/Algorithm/PointClouds/processing/Preprocess/
// RotaryLidar_preprocessing.hpp:31-104, sequential, as written) and DistanceFilter::Filter
// (.../processing/Filter/distance_filter.hpp:24-43).  Angles use -atan2 in double rounded to float
// (the library's choice, within 1 ulp of the reference's float atan2).  Parity vs PCL: unpinned.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "lmsf_oracle.h"

namespace {

float f32_at(const uint8_t* p) {
    float v;
    std::memcpy(&v, p, 4);
    return v;
}

float neg_atan2(float y, float x) { return (float)(-std::atan2((double)y, (double)x)); }

}  // namespace

extern "C" int64_t lmsfo_ingest(const uint8_t* data, int64_t n, uint32_t step, int32_t ox, int32_t oy, int32_t oz,
                                int32_t oi, float period, float near_t, float far_t, float* out) {
    std::vector<float> c;
    c.reserve(4 * (size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* p = data + (size_t)i * step;
        const float x = f32_at(p + ox), y = f32_at(p + oy), z = f32_at(p + oz);
        const float in = oi >= 0 ? f32_at(p + oi) : 0.f;
        if (!std::isfinite(x) || !std::isfinite(y) || !std::isfinite(z)) continue;   // removeNaN
        c.insert(c.end(), {x, y, z, in});
    }
    const int64_t m = (int64_t)c.size() / 4;
    if (period > 0.f && m > 0) {
        // findStartEndAngle (:77-91)
        const float start_ori = neg_atan2(c[1], c[0]);
        float end_ori = (float)((double)neg_atan2(c[4 * (m - 1) + 1], c[4 * (m - 1)]) + 2 * M_PI);
        if (end_ori - start_ori > 3 * M_PI) end_ori = (float)((double)end_ori - 2 * M_PI);
        else if (end_ori - start_ori < M_PI) end_ori = (float)((double)end_ori + 2 * M_PI);
        bool half_passed = false;
        for (int64_t i = 0; i < m; ++i) {                                     // :36-70
            float ori = neg_atan2(c[4 * i + 1], c[4 * i]);
            if (!half_passed) {
                if (ori < start_ori - M_PI / 2) ori = (float)((double)ori + 2 * M_PI);
                else if (ori > start_ori + M_PI * 3 / 2) ori = (float)((double)ori - 2 * M_PI);
                if (ori - start_ori > M_PI) half_passed = true;
            } else {
                ori = (float)((double)ori + 2 * M_PI);
                if (ori < end_ori - M_PI * 3 / 2) ori = (float)((double)ori + 2 * M_PI);
                else if (ori > end_ori + M_PI / 2) ori = (float)((double)ori - 2 * M_PI);
            }
            c[4 * i + 3] = (ori - start_ori) / (end_ori - start_ori) * period;
        }
    }
    int64_t k = 0;
    const bool dist = !(near_t == 0.f && far_t == 0.f);
    for (int64_t i = 0; i < m; ++i) {
        const float* q = &c[4 * i];
        if (dist) {
            const double d = (double)std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
            if (!(d > near_t && d < far_t)) continue;
        }
        std::memcpy(out + 4 * k, q, 16);
        ++k;
    }
    return k;
}
