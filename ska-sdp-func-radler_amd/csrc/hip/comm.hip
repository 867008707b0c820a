// Multi-GPU exchange over RCCL (xGMI) for the process-per-GPU split of
// ParallelDeconvolution::ExecuteParallelRun: the global reduction of the
// maximum start peak over all subimages (cpp/algorithms/
// parallel_deconvolution.cc:592-603), a sum of counters (:622-653), and the
// broadcast of each finished subimage's residual/model boxes from the rank
// that deconvolved it (the copy-back of :458-484, applied by every rank in
// subimage order). The reductions are 4-8 bytes (latency bound, once per
// major iteration); the broadcasts move each box once over xGMI.
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

void rdl::CommRelease(rdl_session* s) {
  if (s->comm) {
    ncclCommDestroy(static_cast<ncclComm_t>(s->comm));
    s->comm = nullptr;
  }
}

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
  if (rdl::ShutDown()) return RDL_OK;  // released by rdl_shutdown
  rdl::CommRelease(s);
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

int rdl_comm_allreduce_max_n(rdl_session* s, float* values, size_t n) {
  RDL_ARG_CHECK(s && values && s->comm, "communicator not initialised");
  RDL_ARG_CHECK(n * sizeof(float) <= rdl::kPeakTickets, "too many values");
  if (n == 0) return RDL_OK;
  float* d = static_cast<float*>(s->d_small);
  RDL_HIP_CHECK(hipMemcpyAsync(d, values, n * sizeof(float), hipMemcpyHostToDevice,
                               s->stream));
  RDL_NCCL_CHECK(ncclAllReduce(d, d, n, ncclFloat32, ncclMax,
                               static_cast<ncclComm_t>(s->comm), s->stream));
  RDL_HIP_CHECK(hipMemcpyAsync(values, d, n * sizeof(float), hipMemcpyDeviceToHost,
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

int rdl_comm_broadcast(rdl_session* s, void* d_buf, size_t bytes, int root) {
  RDL_ARG_CHECK(s && s->comm, "communicator not initialised");
  RDL_ARG_CHECK(d_buf || bytes == 0, "NULL buffer");
  if (bytes == 0) return RDL_OK;
  RDL_NCCL_CHECK(ncclBroadcast(d_buf, d_buf, bytes, ncclUint8, root,
                               static_cast<ncclComm_t>(s->comm), s->stream));
  return RDL_OK;
}

int rdl_comm_rank(rdl_session* s, int* rank, int* n_ranks) {
  RDL_ARG_CHECK(s && s->comm && rank && n_ranks, "communicator not initialised");
  RDL_NCCL_CHECK(ncclCommUserRank(static_cast<ncclComm_t>(s->comm), rank));
  RDL_NCCL_CHECK(ncclCommCount(static_cast<ncclComm_t>(s->comm), n_ranks));
  return RDL_OK;
}

}  // extern "C"
