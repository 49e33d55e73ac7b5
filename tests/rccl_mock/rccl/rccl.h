// Test double of the RCCL API subset csrc/rccl_ops.hip uses (host only, no
// GPU): tests/test_rccl_errors.py builds rccl_ops.hip against it to drive the
// C-ABI error paths, e.g. a call that fails between ncclGroupStart and
// ncclGroupEnd.  Not the product: libnrk.so links the real librccl.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

typedef enum { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
               ncclInvalidArgument = 4, ncclInvalidUsage = 5 } ncclResult_t;
typedef enum { ncclInt32 = 2, ncclFloat32 = 7, ncclFloat64 = 8 } ncclDataType_t;
typedef struct ncclComm* ncclComm_t;
typedef struct {
    char internal[128];
} ncclUniqueId;

extern "C" {
const char* ncclGetErrorString(ncclResult_t r);
ncclResult_t ncclGetUniqueId(ncclUniqueId* id);
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int n, ncclUniqueId id, int rank);
ncclResult_t ncclCommDestroy(ncclComm_t comm);
ncclResult_t ncclCommCount(const ncclComm_t comm, int* count);
ncclResult_t ncclGroupStart(void);
ncclResult_t ncclGroupEnd(void);
ncclResult_t ncclAllGather(const void* s, void* r, size_t n, ncclDataType_t t, ncclComm_t c, hipStream_t st);
ncclResult_t ncclSend(const void* s, size_t n, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t st);
ncclResult_t ncclRecv(void* r, size_t n, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t st);
}
