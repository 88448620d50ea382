// C caller of the multi-GPU plumbing (include/lmsf/lmsf_dist.h, liblmsf_dist.so) together with the
// registration ABI (include/lmsf/lmsf.h): the C2 / C4 protocol of one rank.  Rank 0 broadcasts the map
// into device memory, every rank extracts + registers its scan from device-resident inputs, the poses
// are all-gathered, the scan's features go through the keyframe exchange, and the timing max is taken.
// argv: nranks rank id_file scan edge_map surf_map qx qy qz qw tx ty tz iters
// (rank 0 writes the group id to id_file; other ranks wait for it).  Prints one line:
// n_edge n_surf pose[7] gather_ok keyframe_ok max
// Used by tests/test_gpu_parity.py::test_dist_example (one rank on the one-GPU box).
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <thread>
#include <vector>

#include "lmsf/lmsf.h"
#include "lmsf/lmsf_dist.h"

static std::vector<float> load(const char* path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    const size_t bytes = (size_t)f.tellg();
    f.seekg(0);
    std::vector<float> v(bytes / sizeof(float));
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)bytes);
    return v;
}

#define DIE(msg)                                          \
    do {                                                  \
        std::fprintf(stderr, "dist_example: %s\n", msg); \
        return 1;                                         \
    } while (0)
#define HIP(expr)                                 \
    do {                                          \
        if ((expr) != hipSuccess) DIE(#expr);     \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 15) DIE("usage: nranks rank id_file scan edge surf qx qy qz qw tx ty tz iters");
    const int nranks = std::atoi(argv[1]), rank = std::atoi(argv[2]);
    uint8_t id[LMSF_GROUP_ID_BYTES];
    if (rank == 0) {
        if (lmsf_group_unique_id(id) != LMSF_OK) DIE("unique id");
        std::ofstream(argv[3], std::ios::binary).write(reinterpret_cast<const char*>(id), sizeof id);
    } else {
        for (int t = 0; t < 600; ++t) {
            std::ifstream f(argv[3], std::ios::binary);
            if (f.read(reinterpret_cast<char*>(id), sizeof id)) break;
            std::this_thread::sleep_for(std::chrono::milliseconds(100));
        }
    }
    const int device = 0;   // one GPU per process: HIP_VISIBLE_DEVICES / the launcher picks it
    lmsf_group* g = nullptr;
    if (lmsf_group_create(device, nranks, rank, id, &g) != LMSF_OK) DIE("group create");

    // C4: the map replicated from rank 0 into device memory
    std::vector<float> he, hs;
    size_t ne_map = 0, ns_map = 0;
    if (rank == 0) {
        he = load(argv[5]);
        hs = load(argv[6]);
        ne_map = he.size() / 4;
        ns_map = hs.size() / 4;
    }
    size_t cap_e = ne_map, cap_s = ns_map;   // capacities agreed first (a real caller sizes them once)
    double caps[2] = {(double)cap_e, (double)cap_s};
    lmsf_group_max(g, &caps[0]);
    lmsf_group_max(g, &caps[1]);
    cap_e = (size_t)caps[0];
    cap_s = (size_t)caps[1];
    float *d_edge = nullptr, *d_surf = nullptr;
    if (hipMalloc((void**)&d_edge, cap_e * 16) != hipSuccess || hipMalloc((void**)&d_surf, cap_s * 16) != hipSuccess)
        DIE("hipMalloc");
    if (rank == 0) {
        HIP(hipMemcpy(d_edge, he.data(), ne_map * 16, hipMemcpyHostToDevice));
        HIP(hipMemcpy(d_surf, hs.data(), ns_map * 16, hipMemcpyHostToDevice));
    }
    if (lmsf_group_broadcast_cloud(g, 0, d_edge, cap_e, &ne_map) != LMSF_OK) DIE("broadcast edge");
    if (lmsf_group_broadcast_cloud(g, 0, d_surf, cap_s, &ns_map) != LMSF_OK) DIE("broadcast surf");

    lmsf_config cfg;
    lmsf_config_init(&cfg);
    cfg.device = device;
    cfg.schedule = LMSF_SCHEDULE_FIXED;
    cfg.max_iterations = std::atoi(argv[14]);
    cfg.max_scan_points = cfg.max_features = 70000;
    lmsf_ctx* ctx = nullptr;
    if (lmsf_ctx_create(&cfg, &ctx) != LMSF_OK) DIE("ctx create");
    if (lmsf_set_map(ctx, LMSF_EDGE, d_edge, ne_map) != LMSF_OK || lmsf_set_map(ctx, LMSF_SURF, d_surf, ns_map) != LMSF_OK)
        DIE(lmsf_last_error(ctx));

    // C2: this rank's scan, registered; poses all-gathered
    std::vector<float> scan = load(argv[4]);
    lmsf_feature_counts fc;
    if (lmsf_extract_features(ctx, scan.data(), scan.size() / 4, &fc) != LMSF_OK) DIE(lmsf_last_error(ctx));
    double pose[7];
    for (int i = 0; i < 7; ++i) pose[i] = std::atof(argv[7 + i]);
    lmsf_solve_stats st;
    if (lmsf_solve(ctx, pose, &st) != LMSF_OK) DIE(lmsf_last_error(ctx));
    std::vector<double> all((size_t)nranks * 7);
    if (lmsf_group_allgather_poses(g, pose, 1, all.data()) != LMSF_OK) DIE("allgather");
    const int gather_ok = std::memcmp(&all[(size_t)rank * 7], pose, sizeof pose) == 0;

    // C4: this scan's features as a keyframe through the exchange
    const size_t cap = 70000;
    float *d_feat = nullptr, *d_gath = nullptr;
    if (hipMalloc((void**)&d_feat, 2 * cap * 16) != hipSuccess ||
        hipMalloc((void**)&d_gath, (size_t)nranks * 2 * cap * 16) != hipSuccess)
        DIE("hipMalloc");
    HIP(hipMemset(d_feat, 0, 2 * cap * 16));
    size_t got_e = 0, got_s = 0;
    if (lmsf_copy_features(ctx, LMSF_EDGE, d_feat, nullptr, cap, &got_e) != LMSF_OK ||
        lmsf_copy_features(ctx, LMSF_SURF, d_feat + 4 * cap, nullptr, cap, &got_s) != LMSF_OK)
        DIE(lmsf_last_error(ctx));
    double T[16] = {0};
    T[0] = T[5] = T[10] = T[15] = 1.0;
    T[3] = pose[4];
    T[7] = pose[5];
    T[11] = pose[6];
    std::vector<double> info((size_t)nranks * 19);
    int32_t any = 0;
    int64_t rows[2] = {0, 0};
    if (lmsf_group_exchange_keyframes(g, T, 1, (int64_t)got_e, (int64_t)got_s, d_feat, cap, info.data(), d_gath, rows,
                                      &any) != LMSF_OK)
        DIE("keyframe exchange");
    // this rank's rows come back at [rank rows[0], + got_e) and [nranks rows[0] + rank rows[1], + got_s)
    std::vector<float> mine_e(got_e * 4), mine_s(got_s * 4), back_e(got_e * 4), back_s(got_s * 4);
    HIP(hipMemcpy(mine_e.data(), d_feat, mine_e.size() * 4, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(mine_s.data(), d_feat + 4 * cap, mine_s.size() * 4, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(back_e.data(), d_gath + (size_t)rank * rows[0] * 4, back_e.size() * 4, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(back_s.data(), d_gath + ((size_t)nranks * rows[0] + (size_t)rank * rows[1]) * 4, back_s.size() * 4,
                  hipMemcpyDeviceToHost));
    const int kf_ok = any == 1 && rows[0] == (int64_t)got_e && rows[1] == (int64_t)got_s &&
                      info[(size_t)rank * 19 + 17] == (double)got_e && info[(size_t)rank * 19 + 18] == (double)got_s &&
                      std::memcmp(mine_e.data(), back_e.data(), mine_e.size() * 4) == 0 &&
                      std::memcmp(mine_s.data(), back_s.data(), mine_s.size() * 4) == 0;
    double tmax = 1.5 + rank;
    lmsf_group_max(g, &tmax);
    std::printf("%lld %lld %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d %d %.17g\n", (long long)fc.n_edge,
                (long long)fc.n_surf, pose[0], pose[1], pose[2], pose[3], pose[4], pose[5], pose[6], gather_ok, kf_ok,
                tmax);
    HIP(hipFree(d_feat));
    HIP(hipFree(d_gath));
    HIP(hipFree(d_edge));
    HIP(hipFree(d_surf));
    lmsf_ctx_destroy(ctx);
    lmsf_group_destroy(g);
    return 0;
}
