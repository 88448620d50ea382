// liblmsf_dist.so: the multi-GPU exchanges of include/lmsf/lmsf_dist.h on RCCL (one communicator per
// group, its own HIP stream; every call synchronises that stream before returning).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "../../include/lmsf/lmsf_dist.h"

static_assert(sizeof(ncclUniqueId) == LMSF_GROUP_ID_BYTES, "RCCL unique id size");

struct lmsf_group {
    int device = 0, nranks = 1, rank = 0;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    double* d_small = nullptr;        // device staging for host-sized exchanges
    size_t small_cap = 0;             // doubles
};

namespace {

bool ok(hipError_t e) { return e == hipSuccess; }
bool ok(ncclResult_t r) { return r == ncclSuccess; }

#define LCHK(expr)                          \
    do {                                    \
        if (!ok(expr)) return LMSF_ERR_HIP; \
    } while (0)

lmsf_status reserve_small(lmsf_group* g, size_t doubles) {
    if (doubles <= g->small_cap) return LMSF_OK;
    if (g->d_small) LCHK(hipFree(g->d_small));
    g->d_small = nullptr;
    g->small_cap = 0;
    LCHK(hipMalloc((void**)&g->d_small, doubles * sizeof(double)));
    g->small_cap = doubles;
    return LMSF_OK;
}

// all-gather of `count` doubles per rank between host arrays (staged through the device)
lmsf_status allgather_host(lmsf_group* g, const double* mine, size_t count, double* all) {
    lmsf_status rc = reserve_small(g, count * (size_t)(g->nranks + 1));
    if (rc) return rc;
    double* d_in = g->d_small;
    double* d_out = g->d_small + count;
    if (count) {
        LCHK(hipMemcpyAsync(d_in, mine, count * sizeof(double), hipMemcpyHostToDevice, g->stream));
        LCHK(ncclAllGather(d_in, d_out, count, ncclFloat64, g->comm, g->stream));
        LCHK(hipMemcpyAsync(all, d_out, count * g->nranks * sizeof(double), hipMemcpyDeviceToHost, g->stream));
    }
    LCHK(hipStreamSynchronize(g->stream));
    return LMSF_OK;
}

}  // namespace

extern "C" {

lmsf_status lmsf_group_unique_id(uint8_t id[LMSF_GROUP_ID_BYTES]) {
    if (!id) return LMSF_ERR_ARG;
    ncclUniqueId u;
    LCHK(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return LMSF_OK;
}

lmsf_status lmsf_group_create(int32_t device, int32_t nranks, int32_t rank, const uint8_t id[LMSF_GROUP_ID_BYTES],
                              lmsf_group** out) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return LMSF_ERR_ARG;
    *out = nullptr;
    LCHK(hipSetDevice(device));
    lmsf_group* g = new lmsf_group();
    g->device = device;
    g->nranks = nranks;
    g->rank = rank;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    if (!ok(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking)) ||
        !ok(ncclCommInitRank(&g->comm, nranks, u, rank))) {
        lmsf_group_destroy(g);
        return LMSF_ERR_HIP;
    }
    *out = g;
    return LMSF_OK;
}

void lmsf_group_destroy(lmsf_group* g) {
    if (!g) return;
    hipSetDevice(g->device);
    if (g->stream) hipStreamSynchronize(g->stream);
    if (g->comm) ncclCommDestroy(g->comm);
    if (g->d_small) hipFree(g->d_small);
    if (g->stream) hipStreamDestroy(g->stream);
    delete g;
}

int32_t lmsf_group_rank(const lmsf_group* g) { return g ? g->rank : -1; }
int32_t lmsf_group_size(const lmsf_group* g) { return g ? g->nranks : 0; }

lmsf_status lmsf_group_allgather_poses(lmsf_group* g, const double* mine, int32_t n, double* all) {
    if (!g || n < 0 || (n && (!mine || !all))) return LMSF_ERR_ARG;
    LCHK(hipSetDevice(g->device));
    return allgather_host(g, mine, (size_t)n * 7, all);
}

lmsf_status lmsf_group_broadcast_cloud(lmsf_group* g, int32_t root, float* xyzi_dev, size_t cap, size_t* n) {
    if (!g || !n || root < 0 || root >= g->nranks) return LMSF_ERR_ARG;
    LCHK(hipSetDevice(g->device));
    lmsf_status rc = reserve_small(g, 1);
    if (rc) return rc;
    double cnt = g->rank == root ? (double)*n : 0.0;   // < 2^53 rows
    LCHK(hipMemcpyAsync(g->d_small, &cnt, sizeof cnt, hipMemcpyHostToDevice, g->stream));
    LCHK(ncclBroadcast(g->d_small, g->d_small, 1, ncclFloat64, root, g->comm, g->stream));
    LCHK(hipMemcpyAsync(&cnt, g->d_small, sizeof cnt, hipMemcpyDeviceToHost, g->stream));
    LCHK(hipStreamSynchronize(g->stream));
    const size_t rows = (size_t)cnt;
    *n = rows;
    if (rows > cap) return LMSF_ERR_CAPACITY;   // collective: every rank sees the same count first
    if (rows) {
        if (!xyzi_dev) return LMSF_ERR_ARG;
        LCHK(ncclBroadcast(xyzi_dev, xyzi_dev, rows * 4, ncclFloat32, root, g->comm, g->stream));
    }
    LCHK(hipStreamSynchronize(g->stream));
    return LMSF_OK;
}

lmsf_status lmsf_group_exchange_keyframes(lmsf_group* g, const double pose[16], int32_t update_type, int64_t n_edge,
                                          int64_t n_surf, const float* feat_dev, size_t cap, double* info,
                                          float* gathered_dev, int32_t* any) {
    if (!g || !pose || !info || !any || n_edge < 0 || n_surf < 0 || (size_t)n_edge > cap || (size_t)n_surf > cap)
        return LMSF_ERR_ARG;
    LCHK(hipSetDevice(g->device));
    double mine[19];
    std::memcpy(mine, pose, 16 * sizeof(double));
    mine[16] = (double)update_type;
    mine[17] = (double)n_edge;
    mine[18] = (double)n_surf;
    lmsf_status rc = allgather_host(g, mine, 19, info);
    if (rc) return rc;
    *any = 0;
    for (int r = 0; r < g->nranks; ++r)
        if (info[(size_t)r * 19 + 16] != 0.0) *any = 1;
    if (!*any) return LMSF_OK;
    if (!feat_dev || !gathered_dev) return LMSF_ERR_ARG;
    LCHK(ncclAllGather(feat_dev, gathered_dev, 2 * cap * 4, ncclFloat32, g->comm, g->stream));
    LCHK(hipStreamSynchronize(g->stream));
    return LMSF_OK;
}

lmsf_status lmsf_group_max(lmsf_group* g, double* value) {
    if (!g || !value) return LMSF_ERR_ARG;
    LCHK(hipSetDevice(g->device));
    lmsf_status rc = reserve_small(g, 1);
    if (rc) return rc;
    LCHK(hipMemcpyAsync(g->d_small, value, sizeof(double), hipMemcpyHostToDevice, g->stream));
    LCHK(ncclAllReduce(g->d_small, g->d_small, 1, ncclFloat64, ncclMax, g->comm, g->stream));
    LCHK(hipMemcpyAsync(value, g->d_small, sizeof(double), hipMemcpyDeviceToHost, g->stream));
    LCHK(hipStreamSynchronize(g->stream));
    return LMSF_OK;
}

}  // extern "C"
