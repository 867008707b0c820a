#include "communicator.h"

#include <algorithm>
#include <stdexcept>
#include <utility>
#include <vector>

#include "device.h"
#include "rdl_hip.h"

namespace radler {

RcclCommunicator::RcclCommunicator(std::shared_ptr<gpu::Session> session, int size,
                                   int rank, const void* unique_id)
    : session_(std::move(session)), size_(size), rank_(rank) {
  if (!session_) throw std::runtime_error("RcclCommunicator: no session");
  if (size < 1 || rank < 0 || rank >= size)
    throw std::runtime_error("RcclCommunicator: bad rank / size");
  gpu::Check(rdl_comm_init(session_->Handle(), size, rank, unique_id), "rdl_comm_init");
}

RcclCommunicator::~RcclCommunicator() {
  if (session_) rdl_comm_destroy(session_->Handle());
}

std::size_t RcclCommunicator::IdSize() { return std::size_t(rdl_comm_id_size()); }

void RcclCommunicator::UniqueId(void* out) {
  gpu::Check(rdl_comm_get_unique_id(out), "rdl_comm_get_unique_id");
}

float RcclCommunicator::AllreduceMax(gpu::Session& s, float value) {
  if (&s != session_.get())
    throw std::runtime_error("RcclCommunicator: collective on a foreign session");
  gpu::Check(rdl_comm_allreduce_max(s.Handle(), &value), "rdl_comm_allreduce_max");
  return value;
}

void RcclCommunicator::AllreduceMax(gpu::Session& s, float* values, std::size_t n) {
  if (&s != session_.get())
    throw std::runtime_error("RcclCommunicator: collective on a foreign session");
  gpu::Check(rdl_comm_allreduce_max_n(s.Handle(), values, n), "rdl_comm_allreduce_max_n");
}

void RcclCommunicator::Broadcast(gpu::Session& s, void* d_buffer, size_t bytes,
                                 int root) {
  if (&s != session_.get())
    throw std::runtime_error("RcclCommunicator: collective on a foreign session");
  gpu::Check(rdl_comm_broadcast(s.Handle(), d_buffer, bytes, root),
             "rdl_comm_broadcast");
}

HostCommunicator::HostCommunicator(int size, int rank, BroadcastFn broadcast,
                                   MaxFn max)
    : size_(size), rank_(rank), broadcast_(std::move(broadcast)), max_(std::move(max)) {
  if (size < 1 || rank < 0 || rank >= size)
    throw std::runtime_error("HostCommunicator: bad rank / size");
  if (!broadcast_ || !max_)
    throw std::runtime_error("HostCommunicator: missing collective callbacks");
}

float HostCommunicator::AllreduceMax(gpu::Session&, float value) {
  return max_(value);
}

void HostCommunicator::Broadcast(gpu::Session& s, void* d_buffer, size_t bytes,
                                 int root) {
  if (bytes == 0) return;
  std::vector<unsigned char> host(bytes);
  if (rank_ == root) s.D2H(host.data(), d_buffer, bytes);  // synchronous
  broadcast_(host.data(), bytes, root);
  if (rank_ != root) s.H2D(d_buffer, host.data(), bytes);
}

std::vector<int> LptOwners(const std::vector<double>& costs, int n_ranks) {
  std::vector<int> owners(costs.size(), 0);
  if (n_ranks <= 1) return owners;
  std::vector<std::size_t> order(costs.size());
  for (std::size_t i = 0; i != order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [&](std::size_t a, std::size_t b) { return costs[a] > costs[b]; });
  std::vector<double> load(std::size_t(n_ranks), 0.0);
  for (std::size_t i : order) {
    int best = 0;
    for (int r = 1; r != n_ranks; ++r)
      if (load[std::size_t(r)] < load[std::size_t(best)]) best = r;
    owners[i] = best;
    load[std::size_t(best)] += costs[i];
  }
  return owners;
}

}  // namespace radler
