// Process-per-GPU communicator for ParallelDeconvolution.
// The reference runs the subimages of a gridded major iteration on the
// threads of one process (cpp/algorithms/parallel_deconvolution.cc:556-654);
// here the subimages can also be shared by the ranks of a job, one process
// per GPU. The exchange needs three operations: the signed maximum of the
// start peaks, a broadcast of each finished subimage's boxes from the rank
// that owns it, and a barrier-free agreement on that ownership (static,
// computed identically by every rank).
#pragma once

#include <cstddef>
#include <functional>
#include <memory>
#include <vector>

namespace radler {
namespace gpu {
class Session;
}

class Communicator {
 public:
  virtual ~Communicator() = default;
  virtual int Rank() const = 0;
  virtual int Size() const = 0;
  /// Maximum of one float over all ranks (every rank gets the result).
  virtual float AllreduceMax(gpu::Session& s, float value) = 0;
  /// Element-wise maximum of n floats over all ranks, in place (a rank
  /// gathers the others' entries by leaving its unknown ones at lowest()).
  virtual void AllreduceMax(gpu::Session& s, float* values, std::size_t n) {
    for (std::size_t i = 0; i != n; ++i) values[i] = AllreduceMax(s, values[i]);
  }
  /// In-place broadcast of `bytes` of device memory on `s`'s device from
  /// `root`. Returns with the data in place (stream ordered on `s`).
  virtual void Broadcast(gpu::Session& s, void* d_buffer, size_t bytes, int root) = 0;
};

/// RCCL over xGMI (rdl_comm_*): rank 0 creates the unique id
/// (rdl_comm_get_unique_id / UniqueId()), the job distributes it, every rank
/// constructs one of these on its own device's session.
class RcclCommunicator final : public Communicator {
 public:
  RcclCommunicator(std::shared_ptr<gpu::Session> session, int size, int rank,
                   const void* unique_id);
  ~RcclCommunicator() override;
  int Rank() const override { return rank_; }
  int Size() const override { return size_; }
  float AllreduceMax(gpu::Session& s, float value) override;
  void AllreduceMax(gpu::Session& s, float* values, std::size_t n) override;
  void Broadcast(gpu::Session& s, void* d_buffer, size_t bytes, int root) override;
  /// A fresh RCCL unique id (rank 0 only), `IdSize()` bytes.
  static std::size_t IdSize();
  static void UniqueId(void* out);

 private:
  std::shared_ptr<gpu::Session> session_;
  int size_, rank_;
};

/// Collectives supplied by the host job (MPI, torch.distributed gloo, ...)
/// on host memory: device buffers are staged through the host. Slower than
/// RCCL; it lets several ranks share one GPU (RCCL refuses that), which is how
/// the distributed path is tested on a one-GPU machine.
class HostCommunicator final : public Communicator {
 public:
  using BroadcastFn = std::function<void(void* data, std::size_t bytes, int root)>;
  using MaxFn = std::function<float(float value)>;
  HostCommunicator(int size, int rank, BroadcastFn broadcast, MaxFn max);
  int Rank() const override { return rank_; }
  int Size() const override { return size_; }
  float AllreduceMax(gpu::Session& s, float value) override;
  void Broadcast(gpu::Session& s, void* d_buffer, size_t bytes, int root) override;
  /// The raw host broadcast (tests of the job-side plumbing).
  void BroadcastHost(void* data, std::size_t bytes, int root) {
    broadcast_(data, bytes, root);
  }
  float AllreduceMaxHost(float value) { return max_(value); }

 private:
  int size_, rank_;
  BroadcastFn broadcast_;
  MaxFn max_;
};

/// The rank that runs subimage `index` in the find-peak pass (round robin:
/// every rank computes the same assignment, no exchange needed).
inline int SubImageOwner(std::size_t index, int n_ranks) {
  return n_ranks <= 1 ? 0 : int(index % std::size_t(n_ranks));
}

/// Owners for the cleaning pass: longest-processing-time-first over the
/// per-subimage cost estimates (every rank holds the same estimates after
/// the find-peak exchange, so every rank computes the same assignment):
/// subimages by decreasing cost (ties: lower index first) each go to the
/// rank with the least assigned cost (ties: lower rank).
std::vector<int> LptOwners(const std::vector<double>& costs, int n_ranks);

}  // namespace radler
