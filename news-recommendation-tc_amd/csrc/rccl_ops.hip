// rccl_ops.hip -- the multi-GPU exchanges of the recall as C-ABI entry points
// over RCCL (SURVEY.md 8b's nrk_rccl_topk_allgather; config 4, 8e), for a
// caller that binds the C ABI without torch.distributed.  One process per
// GPU: each rank creates its communicator from a unique id rank 0 made
// (nrk_rccl_get_unique_id / nrk_rccl_comm_init, sent between the processes
// by the caller), then calls the exchange entry points on its stream.  The
// Python host path (nrk.dist) drives the same exchanges through
// torch.distributed, whose "nccl" backend is this RCCL.
#include "nrk_common.h"

#include <rccl/rccl.h>

#include <cstring>

namespace nrk {

// hipLaunch-style status mapping: RCCL failures surface as NRK_EHIP
#define NRK_RCCL(call)                                                                              \
    do {                                                                                           \
        const ncclResult_t r_ = (call);                                                            \
        if (r_ != ncclSuccess) {                                                                   \
            ::nrk::set_error(std::string(__func__) + ": " #call ": " + ncclGetErrorString(r_)); \
            return NRK_EHIP;                                                                       \
        }                                                                                          \
    } while (0)

// the same inside ncclGroupStart / ncclGroupEnd: a failing call ends the
// group before returning, so the communicator takes the caller's next call
#define NRK_RCCL_G(call)                                                                            \
    do {                                                                                           \
        const ncclResult_t r_ = (call);                                                            \
        if (r_ != ncclSuccess) {                                                                   \
            (void)ncclGroupEnd();                                                                  \
            ::nrk::set_error(std::string(__func__) + ": " #call ": " + ncclGetErrorString(r_)); \
            return NRK_EHIP;                                                                       \
        }                                                                                          \
    } while (0)

}  // namespace nrk

using namespace nrk;

extern "C" {

int nrk_rccl_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int nrk_rccl_get_unique_id(void* out_id) {
    clear_error();
    NRK_REQUIRE(out_id != nullptr, "null pointer");
    ncclUniqueId id;
    NRK_RCCL(ncclGetUniqueId(&id));
    memcpy(out_id, &id, sizeof(id));
    return NRK_OK;
}

int nrk_rccl_comm_init(void** out_comm, int n_ranks, const void* id, int rank) {
    clear_error();
    NRK_REQUIRE(out_comm && id, "null pointer");
    NRK_REQUIRE(n_ranks >= 1 && rank >= 0 && rank < n_ranks, "rank out of [0, n_ranks)");
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    NRK_RCCL(ncclCommInitRank(&c, n_ranks, uid, rank));
    *out_comm = c;
    return NRK_OK;
}

int nrk_rccl_comm_destroy(void* comm) {
    clear_error();
    if (comm == nullptr) return NRK_OK;
    NRK_RCCL(ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm)));
    return NRK_OK;
}

// Config 4, merge protocol: every rank holds its shard's top-k_in of EVERY
// user (fp64 exact score + GLOBAL row, n_users x k_in); all-gather them into
// gather_exact / gather_rows ([n_ranks][n_users][k_in], caller-owned), then
// nrk_topk_merge (score desc, row asc) -> the final top-k_out of every user
// on every rank (out_exact may be NULL).

int nrk_rccl_topk_allgather(void* comm, const double* in_exact, const int32_t* in_rows, int64_t n_users, int k_in,
                            int k_out, double* gather_exact, int32_t* gather_rows, float* out_scores,
                            int32_t* out_rows, double* out_exact, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(comm != nullptr, "null communicator");
    NRK_REQUIRE(n_users >= 0 && k_in >= 1 && k_out >= 1, "bad sizes");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(in_exact && in_rows && gather_exact && gather_rows && out_scores && out_rows, "null pointer");
    ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
    int n_ranks = 0;
    NRK_RCCL(ncclCommCount(c, &n_ranks));
    hipStream_t s = as_stream(stream);
    const size_t per = (size_t)n_users * (size_t)k_in;
    NRK_RCCL(ncclGroupStart());
    NRK_RCCL_G(ncclAllGather(in_exact, gather_exact, per, ncclFloat64, c, s));
    NRK_RCCL_G(ncclAllGather(in_rows, gather_rows, per, ncclInt32, c, s));
    NRK_RCCL(ncclGroupEnd());
    return nrk_topk_merge(gather_exact, gather_rows, n_ranks, (int64_t)per, n_users, k_in, k_out, out_scores,
                          out_rows, out_exact, stream);
}

// Config 4, owner protocol (nrk.dist.catalog_sharded_owner): the all-gather
// of every rank's per-user bounds (f32 [n_users, m] -> [n_ranks][n_users][m]).
int nrk_rccl_bound_allgather(void* comm, const float* bounds, int64_t n_users, int m, float* out,
                             nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(comm != nullptr, "null communicator");
    NRK_REQUIRE(n_users >= 0 && m >= 1, "bad sizes");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(bounds && out, "null pointer");
    NRK_RCCL(ncclAllGather(bounds, out, (size_t)n_users * m, ncclFloat32, reinterpret_cast<ncclComm_t>(comm),
                           as_stream(stream)));
    return NRK_OK;
}

// Config 4, owner protocol: the fixed-slot band exchange.  cnt [n_ranks *
// per] i32 and ids [n_ranks * per][x_cap] i32 (user block o = rows [o * per,
// (o + 1) * per), padded) go to owner o; out_cnt [n_ranks][per] and out_ids
// [n_ranks][per][x_cap] receive source s's block in slot s (grouped
// point-to-point sends / receives, one pair per peer and buffer).
int nrk_rccl_band_alltoall(void* comm, const int32_t* cnt, const int32_t* ids, int64_t per, int x_cap,
                           int32_t* out_cnt, int32_t* out_ids, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(comm != nullptr, "null communicator");
    NRK_REQUIRE(per >= 0 && x_cap >= 1, "bad sizes");
    if (per == 0) return NRK_OK;
    NRK_REQUIRE(cnt && ids && out_cnt && out_ids, "null pointer");
    ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
    int n_ranks = 0;
    NRK_RCCL(ncclCommCount(c, &n_ranks));
    hipStream_t s = as_stream(stream);
    const size_t pe = (size_t)per * x_cap;
    NRK_RCCL(ncclGroupStart());
    for (int p = 0; p < n_ranks; ++p) {
        NRK_RCCL_G(ncclSend(cnt + (size_t)p * per, (size_t)per, ncclInt32, p, c, s));
        NRK_RCCL_G(ncclRecv(out_cnt + (size_t)p * per, (size_t)per, ncclInt32, p, c, s));
        NRK_RCCL_G(ncclSend(ids + (size_t)p * pe, pe, ncclInt32, p, c, s));
        NRK_RCCL_G(ncclRecv(out_ids + (size_t)p * pe, pe, ncclInt32, p, c, s));
    }
    NRK_RCCL(ncclGroupEnd());
    return NRK_OK;
}

}  // extern "C"
