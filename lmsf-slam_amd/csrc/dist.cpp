// liblmsf_dist.so: the multi-GPU exchanges of include/lmsf/lmsf_dist.h.  One protocol, two transports:
// RCCL (one communicator per group, its own HIP stream; every call synchronises that stream before
// returning) or the caller's own host collectives (lmsf_group_create_transport: MPI, a torch.distributed
// group, ... -- and the CPU tests, which drive this same code over gloo).
//
// Every call is collective and every rank takes the same path through it: argument problems a rank can
// only see locally (a null buffer, a capacity) travel in the first exchange, so all ranks return the same
// error instead of some entering a collective the others skipped.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/lmsf/lmsf_dist.h"

static_assert(sizeof(ncclUniqueId) == LMSF_GROUP_ID_BYTES, "RCCL unique id size");

struct lmsf_group {
    int device = 0, nranks = 1, rank = 0;
    bool custom = false;              // caller-supplied host collectives instead of RCCL
    lmsf_transport tp{};
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    double* d_small = nullptr;        // device staging for host-sized exchanges (RCCL)
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

// all-gather of `count` doubles per rank between host arrays (RCCL: staged through the device)
lmsf_status allgather_host(lmsf_group* g, const double* mine, size_t count, double* all) {
    if (g->custom) {
        if (count && g->tp.allgather(g->tp.user, mine, all, count * sizeof(double)) != 0) return LMSF_ERR_HIP;
        return LMSF_OK;
    }
    LCHK(hipSetDevice(g->device));
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

// all-gather of `count` floats per rank between buffers of the group's memory space (device for RCCL)
lmsf_status allgather_buffers(lmsf_group* g, const float* mine, size_t count, float* all) {
    if (!count) return LMSF_OK;
    if (g->custom) return g->tp.allgather(g->tp.user, mine, all, count * sizeof(float)) == 0 ? LMSF_OK : LMSF_ERR_HIP;
    LCHK(hipSetDevice(g->device));
    LCHK(ncclAllGather(mine, all, count, ncclFloat32, g->comm, g->stream));
    LCHK(hipStreamSynchronize(g->stream));
    return LMSF_OK;
}

lmsf_status broadcast_buffer(lmsf_group* g, float* buf, size_t count, int root) {
    if (!count) return LMSF_OK;
    if (g->custom) return g->tp.broadcast(g->tp.user, buf, count * sizeof(float), root) == 0 ? LMSF_OK : LMSF_ERR_HIP;
    LCHK(hipSetDevice(g->device));
    LCHK(ncclBroadcast(buf, buf, count, ncclFloat32, root, g->comm, g->stream));
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

lmsf_status lmsf_group_create_transport(int32_t nranks, int32_t rank, const lmsf_transport* tp, lmsf_group** out) {
    if (!out || !tp || !tp->allgather || !tp->broadcast || nranks < 1 || rank < 0 || rank >= nranks) return LMSF_ERR_ARG;
    lmsf_group* g = new lmsf_group();
    g->custom = true;
    g->tp = *tp;
    g->nranks = nranks;
    g->rank = rank;
    *out = g;
    return LMSF_OK;
}

void lmsf_group_destroy(lmsf_group* g) {
    if (!g) return;
    if (!g->custom) {
        hipSetDevice(g->device);
        if (g->stream) hipStreamSynchronize(g->stream);
        if (g->comm) ncclCommDestroy(g->comm);
        if (g->d_small) hipFree(g->d_small);
        if (g->stream) hipStreamDestroy(g->stream);
    }
    delete g;
}

int32_t lmsf_group_rank(const lmsf_group* g) { return g ? g->rank : -1; }
int32_t lmsf_group_size(const lmsf_group* g) { return g ? g->nranks : 0; }

lmsf_status lmsf_group_allgather_poses(lmsf_group* g, const double* mine, int32_t n, double* all) {
    if (!g || n < 0 || (n && (!mine || !all))) return LMSF_ERR_ARG;
    return allgather_host(g, mine, (size_t)n * 7, all);
}

lmsf_status lmsf_group_broadcast_cloud(lmsf_group* g, int32_t root, float* xyzi, size_t cap, size_t* n) {
    if (!g || !n || root < 0 || root >= g->nranks) return LMSF_ERR_ARG;
    // one exchange of (rows at the root, this rank's receive capacity; -1: no buffer): every rank then
    // knows the row count and whether every rank can take it
    const double mine[2] = {g->rank == root ? (double)*n : 0.0, xyzi ? (double)cap : -1.0};   // < 2^53 rows
    std::vector<double> all((size_t)2 * g->nranks);
    lmsf_status rc = allgather_host(g, mine, 2, all.data());
    if (rc) return rc;
    const size_t rows = (size_t)all[(size_t)2 * root];
    *n = rows;
    if (rows == 0) return LMSF_OK;
    for (int r = 0; r < g->nranks; ++r) {
        if (all[(size_t)2 * r + 1] < 0.0) return LMSF_ERR_ARG;
        if (all[(size_t)2 * r + 1] < (double)rows) return LMSF_ERR_CAPACITY;
    }
    return broadcast_buffer(g, xyzi, rows * 4, root);
}

lmsf_status lmsf_group_exchange_keyframes(lmsf_group* g, const double pose[16], int32_t update_type, int64_t n_edge,
                                          int64_t n_surf, const float* feat, size_t cap, double* info, float* gathered,
                                          int64_t rows[2], int32_t* any) {
    if (!g || !pose || !info || !any || !rows) return LMSF_ERR_ARG;
    // local argument state travels with the info row, so a bad argument on one rank fails every rank
    const bool args_ok = n_edge >= 0 && n_surf >= 0 && (size_t)n_edge <= cap && (size_t)n_surf <= cap && feat && gathered;
    constexpr int kRow = 21;   // pose[16], update type, n_edge, n_surf, args ok, cap
    double mine[kRow];
    std::memcpy(mine, pose, 16 * sizeof(double));
    mine[16] = (double)update_type;
    mine[17] = (double)n_edge;
    mine[18] = (double)n_surf;
    mine[19] = args_ok ? 1.0 : 0.0;
    mine[20] = (double)cap;
    std::vector<double> all((size_t)kRow * g->nranks);
    lmsf_status rc = allgather_host(g, mine, kRow, all.data());
    if (rc) return rc;
    bool all_ok = true;
    *any = 0;
    rows[0] = rows[1] = 0;
    double min_cap = all[20];
    for (int r = 0; r < g->nranks; ++r) {
        const double* row = &all[(size_t)r * kRow];
        std::memcpy(info + (size_t)r * 19, row, 19 * sizeof(double));
        all_ok = all_ok && row[19] != 0.0;
        min_cap = std::min(min_cap, row[20]);
        if (row[16] != 0.0) {   // the payload is sized by the keyframing ranks' largest counts
            *any = 1;
            rows[0] = std::max(rows[0], (int64_t)row[17]);
            rows[1] = std::max(rows[1], (int64_t)row[18]);
        }
    }
    // every rank sends rows[k] rows of its own buffer: they must fit the smallest one
    if (!all_ok || (double)rows[0] > min_cap || (double)rows[1] > min_cap) {
        *any = 0;
        rows[0] = rows[1] = 0;
        return LMSF_ERR_ARG;
    }
    if (!*any) return LMSF_OK;
    // two gathers at the max counts instead of the padded 2 cap rows: edges [rank][rows[0]], then surfs
    // [rank][rows[1]] behind them
    float* g_edge = gathered;
    float* g_surf = gathered + (size_t)g->nranks * (size_t)rows[0] * 4;
    if (!g->custom) {
        LCHK(hipSetDevice(g->device));
        LCHK(ncclGroupStart());
        // a failed enqueue inside the group still closes it (an early return left the RCCL group open on
        // this rank, misordering its later collectives against the other ranks')
        bool enq = true;
        if (rows[0]) enq = ok(ncclAllGather(feat, g_edge, (size_t)rows[0] * 4, ncclFloat32, g->comm, g->stream));
        if (enq && rows[1])
            enq = ok(ncclAllGather(feat + cap * 4, g_surf, (size_t)rows[1] * 4, ncclFloat32, g->comm, g->stream));
        const bool closed = ok(ncclGroupEnd());
        if (!enq || !closed) return LMSF_ERR_HIP;
        LCHK(hipStreamSynchronize(g->stream));
        return LMSF_OK;
    }
    rc = allgather_buffers(g, feat, (size_t)rows[0] * 4, g_edge);
    if (rc) return rc;
    return allgather_buffers(g, feat + cap * 4, (size_t)rows[1] * 4, g_surf);
}

lmsf_status lmsf_group_max(lmsf_group* g, double* value) {
    if (!g || !value) return LMSF_ERR_ARG;
    std::vector<double> all((size_t)g->nranks);
    lmsf_status rc = allgather_host(g, value, 1, all.data());
    if (rc) return rc;
    *value = *std::max_element(all.begin(), all.end());
    return LMSF_OK;
}

}  // extern "C"
