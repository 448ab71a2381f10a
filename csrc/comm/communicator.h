// Communicator interface: one implementation over RCCL (GPU tensors, xGMI) and
// one over TCP (CPU tensors, the no-GPU plumbing and test path).
//
// Parity: the reference reaches collectives through ProcessGroupGloo
// (main.py:50, main.py:65, main.py:90-91). Here the
// process-group object in Python owns one Communicator per device type.
#pragma once

#include <ATen/ATen.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../store/tcp_store.h"

namespace dcp {

enum class ReduceOp : int { SUM = 0, AVG = 1, PRODUCT = 2, MIN = 3, MAX = 4 };

// Handle of an in-flight collective.
class Work {
 public:
  virtual ~Work() = default;
  // True once the collective finished (device-side for RCCL).
  virtual bool is_completed() = 0;
  // Make the caller's current stream wait for completion (GPU: no host block;
  // host backend: blocks the calling thread). Raises on communicator failure.
  virtual void wait() = 0;
  // Block the calling host thread until completion.
  virtual void synchronize() = 0;
  // Elapsed device time in ms between issue and completion, or -1 if unknown.
  virtual double elapsed_ms() { return -1.0; }
  std::vector<at::Tensor> outputs;
};

using WorkPtr = std::shared_ptr<Work>;

class Communicator {
 public:
  Communicator(std::shared_ptr<TCPStore> store, std::string prefix, int rank, int size)
      : store_(std::move(store)), prefix_(std::move(prefix)), rank_(rank), size_(size) {}
  virtual ~Communicator() = default;

  int rank() const { return rank_; }
  int size() const { return size_; }
  virtual std::string backend() const = 0;
  // The rank count the transport itself reports (RCCL: ncclCommCount) — a
  // cross-check of size() for multi-GPU run records.
  virtual int transport_size() const { return size_; }
  // Device-time events on every Work from now on (DCP_COMM_TIMING=1 sets it
  // at construction); a no-op where there are no device events.
  virtual void set_timing(bool) {}

  virtual WorkPtr all_reduce(at::Tensor& t, ReduceOp op) = 0;
  // All-reduce `wire` in place, then write the result into `out` (same numel,
  // any float dtype: the cast back of a compressed collective), ordered before
  // the Work's completion — a compression comm hook returns this Work instead
  // of waiting inside the hook (which would order the compute stream behind
  // every bucket's collective mid-backward). Default: reduce, wait, copy.
  virtual WorkPtr all_reduce_into(at::Tensor& wire, at::Tensor& out, ReduceOp op) {
    auto w = all_reduce(wire, op);
    w->wait();
    out.view(-1).copy_(wire.view(-1));
    return w;
  }
  virtual WorkPtr broadcast(at::Tensor& t, int root) = 0;
  // out: contiguous [size * in.numel()] (any shape with that numel).
  virtual WorkPtr all_gather(at::Tensor& out, const at::Tensor& in) = 0;
  // in: contiguous [size * out.numel()].
  virtual WorkPtr reduce_scatter(at::Tensor& out, const at::Tensor& in, ReduceOp op) = 0;
  // Equal splits: in/out contiguous with numel divisible by size.
  virtual WorkPtr all_to_all(at::Tensor& out, const at::Tensor& in) = 0;
  virtual WorkPtr send(const at::Tensor& t, int dst) = 0;
  virtual WorkPtr recv(at::Tensor& t, int src) = 0;
  virtual WorkPtr barrier() = 0;
  // Tear down without waiting for peers (failure path).
  virtual void abort() {}
  // Collective over this communicator: ranks with the same color >= 0 form a
  // new communicator (rank order by key); color < 0 returns nullptr. The
  // default (host backend) is unsupported: new_group builds a fresh host
  // communicator through the store instead.
  virtual std::shared_ptr<Communicator> split(int color, int key, const std::string& prefix) {
    throw std::runtime_error(backend() + " communicator does not support split()");
  }
  // raw handle of the device stream collectives run on (0 = none / host)
  virtual int64_t stream_handle() const { return 0; }
  // A Work that completes when everything the caller's stream has queued so
  // far has run, ordered through the collective stream exactly like a
  // collective (event edge, deadline tracking, watchdog) but issuing no
  // collective. Backs fault-injection tests of the watchdog → abort path
  // (a stalled caller stream looks like a hung collective). Host backend:
  // nullptr (no device stream).
  virtual std::shared_ptr<Work> stream_fence() { return nullptr; }
  // Long-lived buffer registration with the collective library (RCCL
  // ncclCommRegister: lets its intra-node paths read / write the user buffer
  // directly instead of staging through its own FIFO buffers). Returns a
  // handle id (0: nothing registered — one rank, or a backend without it).
  virtual int64_t register_buffer(const at::Tensor&) { return 0; }
  virtual void deregister_buffer(int64_t) {}
  // Contention emulation of an all-reduce of `t` among `world` ranks on a
  // single GPU (bench.py --emulate-world): `channels` workgroups on the
  // collective stream move the ring all-reduce's 2(world-1)/world × bytes
  // through HBM and hold their CUs for alpha_us + those bytes / busbw_gbps —
  // the footprint the real collective has on this GPU while backward runs.
  // `t` is read, never written. Returns a Work like a collective's.
  virtual std::shared_ptr<Work> emulate_all_reduce(at::Tensor& t, int world, double busbw_gbps, int channels,
                                                   double alpha_us) {
    throw std::runtime_error(backend() + " communicator cannot emulate collectives");
  }
  // Non-empty once the communicator hit an unrecoverable error.
  virtual std::string error() { return {}; }

  // Debug collective fingerprinting: when enabled every
  // collective first checks through the store that all ranks issue the same
  // (op, dtype, numel, root) at the same sequence number, turning a would-be
  // RCCL hang into an error that names the diverging rank.
  void set_debug_fingerprint(bool on) { fingerprint_ = on; }
  bool debug_fingerprint() const { return fingerprint_; }

  // Counters for observability.
  int64_t ops_issued() const { return ops_.load(); }
  int64_t bytes_issued() const { return bytes_.load(); }

 protected:
  void account(const char* op, const at::Tensor& t, int64_t extra = 0);
  void check_fingerprint(const char* op, const at::Tensor& t, int64_t extra);

  std::shared_ptr<TCPStore> store_;
  std::string prefix_;
  int rank_;
  int size_;
  bool fingerprint_ = false;
  int64_t seq_ = 0;
  std::atomic<int64_t> ops_{0};
  std::atomic<int64_t> bytes_{0};
};

// Host (CPU) communicator: full TCP mesh, ring algorithms, one worker thread so
// collectives run asynchronously to the caller (the Reducer overlaps them with
// backward exactly as on GPU).
std::shared_ptr<Communicator> make_host_communicator(std::shared_ptr<TCPStore> store, const std::string& prefix,
                                                     int rank, int size, int64_t timeout_ms);

// RCCL communicator on `device`, comm stream from the torch pool.
std::shared_ptr<Communicator> make_rccl_communicator(std::shared_ptr<TCPStore> store, const std::string& prefix,
                                                     int rank, int size, int device, int64_t timeout_ms);

bool rccl_available();
std::string rccl_version();

}  // namespace dcp
