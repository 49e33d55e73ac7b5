// Test double of RCCL (see rccl/rccl.h): counts calls, tracks the group
// depth and fails the call with a chosen sequence number with
// ncclInvalidArgument.  Host memory only; nothing runs on a GPU.
#include "rccl/rccl.h"

static int g_depth = 0, g_calls = 0, g_fail_at = -1, g_ranks = 2, g_ops = 0;

extern "C" {
void mock_reset(int n_ranks, int fail_at) {
    g_depth = 0;
    g_calls = 0;
    g_ops = 0;
    g_ranks = n_ranks;
    g_fail_at = fail_at;
}
int mock_group_depth(void) { return g_depth; }
int mock_ops(void) { return g_ops; }  // data-path calls that succeeded

const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "invalid argument (mock)"; }
ncclResult_t ncclGetUniqueId(ncclUniqueId*) { return ncclSuccess; }
ncclResult_t ncclCommInitRank(ncclComm_t* c, int, ncclUniqueId, int) {
    *c = reinterpret_cast<ncclComm_t>(0x1);
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t) { return ncclSuccess; }
ncclResult_t ncclCommCount(const ncclComm_t, int* n) {
    *n = g_ranks;
    return ncclSuccess;
}
ncclResult_t ncclGroupStart(void) {
    ++g_depth;
    return ncclSuccess;
}
ncclResult_t ncclGroupEnd(void) {
    if (g_depth == 0) return ncclInvalidUsage;
    --g_depth;
    return ncclSuccess;
}
static ncclResult_t op() {
    if (g_calls++ == g_fail_at) return ncclInvalidArgument;
    ++g_ops;
    return ncclSuccess;
}
ncclResult_t ncclAllGather(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) { return op(); }
ncclResult_t ncclSend(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) { return op(); }
ncclResult_t ncclRecv(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) { return op(); }
}

// the merge that nrk_rccl_topk_allgather runs after its group (ip_topk.hip
// in the product library): a no-op here
#include "../../include/nrk.h"
extern "C" int nrk_topk_merge(const double*, const int32_t*, int, int64_t, int64_t, int, int, float*, int32_t*,
                              double*, nrk_stream_t) {
    return NRK_OK;
}
