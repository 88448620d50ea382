/*
 * lmsf_dist.h -- multi-GPU plumbing of the registration hot path for C / C++ callers
 * (liblmsf_dist.so, RCCL over xGMI).
 *
 * The reference runs one MultiLidarSystem per process (INC/System/ML_System.hpp:130-156) and has no
 * multi-device path; the build's scaling protocol -- one process (or thread) per GPU, each with its
 * own lmsf_ctx -- needs three exchanges, the same ones lmsf-slam_amd/lmsf/multi.py runs over
 * torch.distributed for bench.py:
 *   C2 / C5  scans (pairs) sharded with no data-path collective, then an all-gather of the 6-DoF
 *            poses (7 doubles each);
 *   C4       the shared map broadcast from rank 0 once (into device memory, then lmsf_set_map /
 *            lmsf_tracker_set_prior_map from it), and per tracking step an all-gather of every
 *            stream's (pose, keyframe flag, feature counts) followed -- only when some stream
 *            keyframed -- by an all-gather of the feature buffers at the keyframing streams' largest
 *            counts, so every replica appends the same keyframes in rank order.
 * Every call is collective (all ranks, same order) and returns when its result is usable: host
 * results are written, device results are complete on the device.  Every rank takes the same path
 * through a call: an argument problem only one rank can see (a null buffer, a too-small capacity)
 * travels in the call's first exchange, so every rank returns the same error and none is left inside
 * a collective the others skipped.
 *
 * Transports: RCCL (lmsf_group_create; "device" buffers below are device memory of the group's GPU), or
 * the caller's own host collectives (lmsf_group_create_transport; the same buffers are then host
 * memory) -- the same protocol code either way, which is how the CPU tests run it over gloo.
 */
#ifndef LMSF_LMSF_DIST_H_
#define LMSF_LMSF_DIST_H_

#include <stddef.h>
#include <stdint.h>

#include "lmsf.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LMSF_GROUP_ID_BYTES 128

typedef struct lmsf_group lmsf_group;

/* Rank 0 creates the group id and hands it to every rank out of band (a file, the ROS parameter
 * server, MPI, ...). */
lmsf_status lmsf_group_unique_id(uint8_t id[LMSF_GROUP_ID_BYTES]);
/* Join the group as `rank` of `nranks` on HIP device `device` (one device per rank). */
lmsf_status lmsf_group_create(int32_t device, int32_t nranks, int32_t rank, const uint8_t id[LMSF_GROUP_ID_BYTES],
                              lmsf_group** out);
/* Caller-supplied collectives on host memory (MPI, a torch.distributed group, ...); each returns 0 on
 * success.  allgather: bytes_per_rank from send -> recv[nranks][bytes_per_rank] in rank order;
 * broadcast: bytes of buf from root to every rank.  The struct is copied; `user` is passed back. */
typedef struct {
    void* user;
    int32_t (*allgather)(void* user, const void* send, void* recv, size_t bytes_per_rank);
    int32_t (*broadcast)(void* user, void* buf, size_t bytes, int32_t root);
} lmsf_transport;
lmsf_status lmsf_group_create_transport(int32_t nranks, int32_t rank, const lmsf_transport* tp, lmsf_group** out);
void lmsf_group_destroy(lmsf_group* g);
int32_t lmsf_group_rank(const lmsf_group* g);
int32_t lmsf_group_size(const lmsf_group* g);

/* C2 / C5: every rank's n poses (qx qy qz qw tx ty tz, host) -> all[rank][n][7] (host). */
lmsf_status lmsf_group_allgather_poses(lmsf_group* g, const double* mine, int32_t n, double* all);

/* C4: the root's cloud (xyzi rows, *n rows at the root) replicated into every rank's buffer xyzi of cap
 * rows (device memory for RCCL groups); *n = rows on return.  Every rank returns LMSF_ERR_CAPACITY when
 * some rank's cap is too small, LMSF_ERR_ARG when some rank passed no buffer for a non-empty cloud. */
lmsf_status lmsf_group_broadcast_cloud(lmsf_group* g, int32_t root, float* xyzi, size_t cap, size_t* n);

/* C4 keyframe exchange.  In: this rank's pose (4x4 row-major), update type (0: none), feature counts
 * and feat = [edges (cap rows) | surfs (cap rows)] xyzi (device memory for RCCL groups).  Out: info[rank]
 * [19] = (pose[16], update type, n_edge, n_surf) of every rank (host); *any = 1 when some rank keyframed.
 * The feature payload is sized by the keyframing ranks' largest counts, rows[0] = max n_edge and rows[1] =
 * max n_surf over the ranks with a non-zero update type (not by cap): gathered then holds the edges of
 * rank r at rows [r rows[0], r rows[0] + n_edge_r) and its surfs at rows [nranks rows[0] + r rows[1], + n_surf_r)
 * -- (rows[0] + rows[1]) rows per rank on the wire.  gathered must hold nranks (rows[0] + rows[1]) rows;
 * nranks * 2 * cap always does.  Every replica appends rank r's keyframe for r = 0, 1, ... with a non-zero
 * update type: the same keyframes in the same order on every rank.  Counts above cap, a null feat /
 * gathered on any rank, or a maximum count above some rank's cap: LMSF_ERR_ARG on every rank (*any = 0).
 * g, pose, info, rows and any are required. */
lmsf_status lmsf_group_exchange_keyframes(lmsf_group* g, const double pose[16], int32_t update_type, int64_t n_edge,
                                          int64_t n_surf, const float* feat, size_t cap, double* info, float* gathered,
                                          int64_t rows[2], int32_t* any);

/* Max over ranks of a host double (the bench's max-over-ranks timing). */
lmsf_status lmsf_group_max(lmsf_group* g, double* value);

#ifdef __cplusplus
}
#endif

#endif /* LMSF_LMSF_DIST_H_ */
