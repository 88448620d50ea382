// Host-code sanitizer run (SURVEY.md §5 "Race detection / sanitizers": ASan/UBSan on the CPU
// restatement).  Built by tests/test_sanitizers.py with -fsanitize=address,undefined from the
// oracle sources (test infrastructure) and the library's host-only hand-eye code
// (lmsf-slam_amd/csrc/calib.cpp); drives every oracle entry point once on files written by the
// test: scan.bin / edge.bin / surf.bin (float32 x y z i rows), msg.bin (PointCloud2 bytes).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lmsf/lmsf.h"
#include "lmsf_oracle.h"

static std::vector<float> load(const char* path) {
    std::vector<float> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    float buf[4096];
    size_t n;
    while ((n = std::fread(buf, sizeof(float), 4096, f)) > 0) v.insert(v.end(), buf, buf + n);
    std::fclose(f);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 6) { std::fprintf(stderr, "usage: scan edge surf msg n_msg\n"); return 2; }
    const std::vector<float> scan = load(argv[1]), edge = load(argv[2]), surf = load(argv[3]);
    const std::vector<float> msgf = load(argv[4]);
    const long n_msg = std::atol(argv[5]);
    const int64_t n = (int64_t)scan.size() / 4;

    lmsfo_extract_params prm{16, 2.f, 80.f, 1.f, 1, 0.0, 0.0};
    std::vector<float> e(4 * n), s(4 * n);
    std::vector<int32_t> ei(n), si(n);
    int64_t ne = 0, ns = 0;
    if (lmsfo_extract(&prm, scan.data(), n, e.data(), ei.data(), &ne, s.data(), si.data(), &ns, n) != 0) return 3;

    lmsfo_set_num_threads(2);
    lmsfo_reg* reg = lmsfo_reg_create(0);
    lmsfo_reg_set_map(reg, 1, edge.data(), (int64_t)edge.size() / 4);
    lmsfo_reg_set_map(reg, 2, surf.data(), (int64_t)surf.size() / 4);
    lmsfo_reg_set_scan(reg, 1, e.data(), ne);
    lmsfo_reg_set_scan(reg, 2, s.data(), ns);
    double pose[7] = {0, 0, 0, 1, 0.05, -0.03, 0.02};
    double trace[32 * 7];
    lmsfo_solve_stats st;
    lmsfo_reg_solve(reg, pose, trace, 32, &st);
    std::vector<lmsfo_record> rec((size_t)(ne + ns));
    std::vector<int32_t> nn((size_t)(ne + ns) * 5);
    lmsfo_reg_match(reg, pose, rec.data(), nn.data());
    double packet[29];
    lmsfo_eval(rec.data(), (int64_t)rec.size(), pose, packet);
    lmsfo_reg_free(reg);
    lmsfo_reg* gn = lmsfo_reg_create(1);
    lmsfo_reg_set_map(gn, 1, edge.data(), (int64_t)edge.size() / 4);
    lmsfo_reg_set_map(gn, 2, surf.data(), (int64_t)surf.size() / 4);
    lmsfo_reg_set_scan(gn, 1, e.data(), ne);
    lmsfo_reg_set_scan(gn, 2, s.data(), ns);
    double pose2[7] = {0, 0, 0, 1, 0.05, -0.03, 0.02};
    lmsfo_reg_solve(gn, pose2, trace, 32, &st);
    lmsfo_reg_free(gn);

    std::vector<float> vox(4 * ns + 4);
    const int64_t nv = lmsfo_voxel_filter(s.data(), ns, 0.4f, vox.data());
    std::vector<float> ing(4 * (size_t)n_msg + 4);
    const int64_t ni = lmsfo_ingest(reinterpret_cast<const uint8_t*>(msgf.data()), n_msg, 32, 0, 4, 8, 16, 0.1f,
                                    3.f, 50.f, ing.data());

    // hand-eye on exact conjugate screw motions B = X^-1 A X (rotation about varied axes)
    lmsf_handeye* h = nullptr;
    lmsf_handeye_create(&h);
    int32_t ok = 0;
    for (int k = 0; k < 12; ++k) {
        const double th = 0.1 + 0.03 * k, ax[3] = {std::sin(1.0 + k), std::cos(2.0 * k), 0.5};
        const double nrm = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
        double A[16] = {0}, B[16];
        const double u[3] = {ax[0] / nrm, ax[1] / nrm, ax[2] / nrm}, c = std::cos(th), sn = std::sin(th);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                A[4 * i + j] = (i == j ? c : 0.0) + (1 - c) * u[i] * u[j] +
                               sn * ((i == 0 && j == 1) ? -u[2] : (i == 0 && j == 2) ? u[1] : (i == 1 && j == 0) ? u[2]
                                     : (i == 1 && j == 2) ? -u[0] : (i == 2 && j == 0) ? -u[1] : (i == 2 && j == 1) ? u[0] : 0.0);
        A[3] = 0.3 * k; A[7] = -0.2; A[11] = 0.1; A[15] = 1;
        for (int i = 0; i < 16; ++i) B[i] = A[i];   // identity extrinsic: B = A
        lmsf_handeye_add_pose(h, A, B, &ok);
        if (ok) {
            double sv[4];
            lmsf_handeye_calib_rotation(h, &ok, sv);
            if (ok) lmsf_handeye_calib_translation(h, &ok);
        }
    }
    double T[16];
    lmsf_handeye_result(h, T, &ok);
    lmsf_handeye_destroy(h);
    std::printf("features %lld %lld outer %d voxels %lld ingest %lld handeye %d\n", (long long)ne, (long long)ns,
                st.outer_iterations, (long long)nv, (long long)ni, ok);
    return 0;
}
