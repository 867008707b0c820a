// Multi-GPU exchange over RCCL (xGMI): the one global reduction of
// ParallelDeconvolution::ExecuteParallelRun — the maximum start peak over all
// subimages (cpp/algorithms/parallel_deconvolution.cc:592-603) — plus a sum
// of finished/iteration counters (:622-653). 4-8 bytes per call: latency
// bound, one call per major iteration.
#include <rccl/rccl.h>

#include <cstring>

#include "rdl_internal.h"

#define RDL_NCCL_CHECK(expr)                                                \
  do {                                                                      \
    ncclResult_t _r = (expr);                                               \
    if (_r != ncclSuccess) {                                                \
      ::rdl::SetError(std::string(#expr) + ": " + ncclGetErrorString(_r));  \
      return RDL_ERR_HIP;                                                   \
    }                                                                       \
  } while (0)

extern "C" {

int rdl_comm_id_size(void) { return int(sizeof(ncclUniqueId)); }

int rdl_comm_get_unique_id(void* h_id) {
  RDL_ARG_CHECK(h_id, "NULL argument");
  ncclUniqueId id;
  RDL_NCCL_CHECK(ncclGetUniqueId(&id));
  std::memcpy(h_id, &id, sizeof(id));
  return RDL_OK;
}

int rdl_comm_init(rdl_session* s, int n_ranks, int rank, const void* h_id) {
  RDL_ARG_CHECK(s && h_id, "NULL argument");
  RDL_ARG_CHECK(n_ranks >= 1 && rank >= 0 && rank < n_ranks, "bad rank");
  RDL_HIP_CHECK(hipSetDevice(s->device));
  ncclUniqueId id;
  std::memcpy(&id, h_id, sizeof(id));
  ncclComm_t comm;
  RDL_NCCL_CHECK(ncclCommInitRank(&comm, n_ranks, id, rank));
  s->comm = comm;
  return RDL_OK;
}

int rdl_comm_destroy(rdl_session* s) {
  RDL_ARG_CHECK(s, "NULL argument");
  if (s->comm) {
    ncclCommDestroy(static_cast<ncclComm_t>(s->comm));
    s->comm = nullptr;
  }
  return RDL_OK;
}

int rdl_comm_allreduce_max(rdl_session* s, float* value) {
  RDL_ARG_CHECK(s && value && s->comm, "communicator not initialised");
  float* d = static_cast<float*>(s->d_small);
  RDL_HIP_CHECK(hipMemcpyAsync(d, value, sizeof(float), hipMemcpyHostToDevice,
                               s->stream));
  RDL_NCCL_CHECK(ncclAllReduce(d, d, 1, ncclFloat32, ncclMax,
                               static_cast<ncclComm_t>(s->comm), s->stream));
  RDL_HIP_CHECK(hipMemcpyAsync(value, d, sizeof(float), hipMemcpyDeviceToHost,
                               s->stream));
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}

int rdl_comm_allreduce_sum_u64(rdl_session* s, uint64_t* value) {
  RDL_ARG_CHECK(s && value && s->comm, "communicator not initialised");
  uint64_t* d = static_cast<uint64_t*>(s->d_small);
  RDL_HIP_CHECK(hipMemcpyAsync(d, value, sizeof(uint64_t),
                               hipMemcpyHostToDevice, s->stream));
  RDL_NCCL_CHECK(ncclAllReduce(d, d, 1, ncclUint64, ncclSum,
                               static_cast<ncclComm_t>(s->comm), s->stream));
  RDL_HIP_CHECK(hipMemcpyAsync(value, d, sizeof(uint64_t),
                               hipMemcpyDeviceToHost, s->stream));
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}

}  // extern "C"
