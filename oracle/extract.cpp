// TEST INFRASTRUCTURE ONLY -- CPU restatement of LOAM feature extraction.
// Follows FX/LOAMFeatureProcessor_base.hpp (FX = src/MultiSensorFusionEstimator3D/include/
// Algorithm/PointClouds/processing/FeatureExtract/).  Parity vs the reference: unpinned
// (see lmsf_oracle.h).  Arithmetic follows the reference's C++ evaluation rules literally:
// PointXYZI members are float, so `x*x + y*y` and the 11-point curvature sums are float
// expressions that are only widened to double on assignment.  Unqualified sqrt / atan2 on float
// arguments bind to the double versions on the reference's toolchain (ROS kinetic, GCC 5) and to the
// float overloads with GCC >= 6 when libstdc++'s <math.h> wrapper is in scope: prm.libm_float picks
// (float atan2 as the double atan2 rounded to float, within glibc atan2f's 1 ulp).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "lmsf_oracle.h"


namespace {

struct P4 { float x, y, z, i; };

double ref_sqrt(float s, int libm_float) { return libm_float ? (double)std::sqrt(s) : std::sqrt((double)s); }
double ref_atan2(float y, float x, int libm_float) {
    const double a = std::atan2((double)y, (double)x);
    return libm_float ? (double)(float)a : a;
}

// splitScan ring assignment (FX:290-343).  Returns -1 for rejected points.
int ring_of(const lmsfo_extract_params& prm, const P4& p) {
    float s = p.x * p.x + p.y * p.y;                 // float expression (FX:300-301)
    double distance = ref_sqrt(s, prm.libm_float);
    if (distance > (double)prm.max_distance || distance < (double)prm.min_distance) return -1;  // FX:302
    double angle = std::atan((double)p.z / distance) * 180 / M_PI;                               // FX:307
    int n = prm.n_scans;
    int id = 0;
    if (n == 16) {
        id = (int)((angle + 15) / 2 + 0.5);          // truncation toward zero, as int() (FX:311)
        if (id > n - 1 || id < 0) return -1;
    } else if (n == 32) {
        id = (int)((angle + 92.0 / 3.0) * 3.0 / 4.0); // FX:319
        // FX:320 tests `N_SCANS_ < 0` instead of scanID < 0, so a negative id indexes out of
        // bounds in the reference (UB).  Deviation: such points are rejected.
        if (id > n - 1 || id < 0) return -1;
    } else if (n == 64) {
        if (angle >= -8.83) id = (int)((2 - angle) * 3.0 + 0.5);
        else id = n / 2 + (int)((-8.83 - angle) * 2.0 + 0.5);
        if (angle > 2 || angle < -24.33 || id > 63 || id < 0) return -1;   // FX:332
    } else if (prm.beam_spacing_deg > 0) {
        // Build-defined uniform beam model for other beam counts.
        id = (int)((angle - prm.beam_lo_deg) / prm.beam_spacing_deg + 0.5);
        if (id > n - 1 || id < 0) return -1;
    } else {
        id = 0;                                      // "wrong scan number" (FX:337-341)
    }
    return id;
}

// checkBadEdgePoint (FX:216-282).
void check_bad(const std::vector<P4>& pc, std::vector<int>& dis, int libm_float) {
    int scan_num = (int)pc.size();
    for (int j = 5; j < scan_num - 6; j++) {
        double angle_curr = ref_atan2(pc[j].x, pc[j].y, libm_float);        // atan2(x, y) order
        double angle_after = ref_atan2(pc[j + 1].x, pc[j + 1].y, libm_float);
        double delta_angle = std::fabs(angle_curr - angle_after);
        if (delta_angle > M_PI) delta_angle = M_PI * 2 - delta_angle;
        if (delta_angle > 0.0175) {
            for (int k = -5; k <= 5; ++k) dis[j + k] = 1;
            j = j + 4;
            continue;
        }
        float sc = pc[j].x * pc[j].x + pc[j].y * pc[j].y + pc[j].z * pc[j].z;
        float sa = pc[j + 1].x * pc[j + 1].x + pc[j + 1].y * pc[j + 1].y + pc[j + 1].z * pc[j + 1].z;
        double distance_curr = ref_sqrt(sc, libm_float);
        double distance_after = ref_sqrt(sa, libm_float);
        double angle;
        if (distance_curr < distance_after)
            angle = std::atan2(distance_curr * delta_angle, distance_after - distance_curr);
        else
            angle = std::atan2(distance_after * delta_angle, distance_curr - distance_after);
        if (angle <= 0.17) {
            if (distance_curr < distance_after) {
                for (int k = 1; k <= 5; ++k) dis[j + k] = 1;
                j = j + 4;
            } else {
                for (int k = 0; k <= 5; ++k) dis[j - k] = 1;
            }
        }
    }
}

struct Curv { int id; double value; };

// One ring: FX:69-121 + featureExtractionFromSector (FX:145-207).
void process_ring(const lmsfo_extract_params& prm, const std::vector<P4>& pc, const std::vector<int32_t>& src,
                  std::vector<P4>& edge, std::vector<int32_t>& edge_src,
                  std::vector<P4>& surf, std::vector<int32_t>& surf_src) {
    int size = (int)pc.size();
    if (size < 20) return;
    int total_points = size - 10;
    if (total_points < 6) return;
    int sector_length = (int)((total_points / 6) + 0.5);     // integer division first (FX:74)
    std::vector<int> dis(size, 0), is_edge(size, 0);
    if (prm.remove_bad_points) check_bad(pc, dis, prm.libm_float);
    const double thresh = (double)prm.edge_threshold;
    std::vector<Curv> cc;
    cc.reserve(total_points);
    for (int k = 0; k < 6; k++) {
        int sector_start = 5 + sector_length * k;
        int sector_end = sector_start + sector_length - 1;
        if (k == 5) sector_end = size - 6;
        cc.clear();
        for (int j = sector_start; j <= sector_end; j++) {
            // float expressions, widened on assignment (FX:99-116)
            float fx = pc[j - 5].x + pc[j - 4].x + pc[j - 3].x + pc[j - 2].x + pc[j - 1].x - 10 * pc[j].x
                       + pc[j + 1].x + pc[j + 2].x + pc[j + 3].x + pc[j + 4].x + pc[j + 5].x;
            float fy = pc[j - 5].y + pc[j - 4].y + pc[j - 3].y + pc[j - 2].y + pc[j - 1].y - 10 * pc[j].y
                       + pc[j + 1].y + pc[j + 2].y + pc[j + 3].y + pc[j + 4].y + pc[j + 5].y;
            float fz = pc[j - 5].z + pc[j - 4].z + pc[j - 3].z + pc[j - 2].z + pc[j - 1].z - 10 * pc[j].z
                       + pc[j + 1].z + pc[j + 2].z + pc[j + 3].z + pc[j + 4].z + pc[j + 5].z;
            double dx = fx, dy = fy, dz = fz;
            cc.push_back({j, dx * dx + dy * dy + dz * dz});
        }
        // std::sort is unstable in the reference (FX:152-156); ties are broken here by index,
        // the canonical order the GPU path reproduces.
        std::sort(cc.begin(), cc.end(), [](const Curv& a, const Curv& b) {
            return a.value < b.value || (a.value == b.value && a.id < b.id);
        });
        int picked = 0;
        for (int i = (int)cc.size() - 1; i >= 0; i--) {
            int ind = cc[i].id;
            if (dis[ind] == 0) {
                if (cc[i].value <= thresh) break;
                picked++;
                if (picked <= 20) {
                    edge.push_back(pc[ind]);
                    edge_src.push_back(src[ind]);
                    is_edge[ind] = 1;
                } else {
                    break;
                }
                for (int q = 1; q <= 5; q++) {
                    int nn = ind + q >= size ? size - 1 : ind + q;
                    dis[nn] = 1;
                }
                for (int q = -1; q >= -5; q--) {
                    int nn = ind + q < 0 ? 0 : ind + q;
                    dis[nn] = 1;
                }
            }
        }
        for (int i = 0; i <= (int)cc.size() - 1; i++) {
            int ind = cc[i].id;
            if (is_edge[ind] == 0) {
                surf.push_back(pc[ind]);
                surf_src.push_back(src[ind]);
            }
        }
    }
}

}  // namespace

extern "C" int lmsfo_extract(const lmsfo_extract_params* prm, const float* xyzi, int64_t n,
                             float* edge_out, int32_t* edge_src, int64_t* n_edge,
                             float* surf_out, int32_t* surf_src, int64_t* n_surf, int64_t cap) {
    const int nsc = prm->n_scans;
    if (nsc <= 0) return -2;
    std::vector<std::vector<P4>> rings(nsc);
    std::vector<std::vector<int32_t>> rsrc(nsc);
    const P4* pts = reinterpret_cast<const P4*>(xyzi);
    for (int64_t i = 0; i < n; ++i) {
        int id = ring_of(*prm, pts[i]);
        if (id < 0) continue;
        rings[id].push_back(pts[i]);               // stable: input order within the ring
        rsrc[id].push_back((int32_t)i);
    }
    std::vector<P4> edge, surf;
    std::vector<int32_t> es, ss;
    for (int r = 0; r < nsc; ++r) process_ring(*prm, rings[r], rsrc[r], edge, es, surf, ss);
    *n_edge = (int64_t)edge.size();
    *n_surf = (int64_t)surf.size();
    if ((int64_t)edge.size() > cap || (int64_t)surf.size() > cap) return -1;
    if (edge_out) std::memcpy(edge_out, edge.data(), edge.size() * sizeof(P4));
    if (surf_out) std::memcpy(surf_out, surf.data(), surf.size() * sizeof(P4));
    if (edge_src) std::memcpy(edge_src, es.data(), es.size() * sizeof(int32_t));
    if (surf_src) std::memcpy(surf_src, ss.data(), ss.size() * sizeof(int32_t));
    return 0;
}
