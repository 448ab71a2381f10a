// RCCL communicator over xGMI: one process per GPU, collectives on a dedicated
// HIP stream (normal priority by default: a high-priority queue pre-empted the
// backward's compute kernels, NOTES §22; DCP_COMM_STREAM_PRIORITY=high opts in),
// ordered against the caller's stream with events, no host synchronisation on
// the hot path.
//
// Parity: the reference's collectives (main.py:50 init, main.py:65 loss
// all-reduce, main.py:90-91 metric all-reduces) went through gloo, staging GPU
// tensors through pinned host memory. This path keeps them on the
// device. Failure detection: a watchdog thread polls
// ncclCommGetAsyncError and per-Work deadlines and aborts the communicator.
#include <ATen/ATen.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <map>

#include <condition_variable>
#include <list>
#include <thread>

#include "../common.h"
#include "../kernels/kernels.h"
#include "communicator.h"

namespace dcp {

namespace {

#define HIP_OK(expr)                                                                          \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    DK_CHECK(_e == hipSuccess, #expr, " failed: ", hipGetErrorString(_e));                    \
  } while (0)

#define NCCL_OK(expr)                                                                         \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    DK_CHECK(_r == ncclSuccess || _r == ncclInProgress, #expr, " failed: ", ncclGetErrorString(_r)); \
  } while (0)

ncclDataType_t to_nccl(at::ScalarType st) {
  switch (st) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kBool: return ncclUint8;
    default: throw Error(str_cat("RCCL: unsupported dtype ", c10::toString(st)));
  }
}

ncclRedOp_t to_nccl(ReduceOp op, at::ScalarType st) {
  switch (op) {
    case ReduceOp::SUM: return ncclSum;
    case ReduceOp::AVG:
      DK_CHECK(at::isFloatingType(st), "ReduceOp.AVG needs a floating dtype");
      return ncclAvg;
    case ReduceOp::PRODUCT: return ncclProd;
    case ReduceOp::MIN: return ncclMin;
    case ReduceOp::MAX: return ncclMax;
  }
  return ncclSum;
}

class RcclCommunicator;

// DCP_COMM_STREAM_PRIORITY=high puts collectives on a high-priority queue
// (default: normal priority, same as the compute stream).
bool comm_stream_high_priority() {
  const char* v = std::getenv("DCP_COMM_STREAM_PRIORITY");
  return v && std::string(v) == "high";
}

class RcclWork : public Work {
 public:
  RcclWork(RcclCommunicator* comm, hipStream_t stream, int device, int64_t timeout_ms, bool timing);
  ~RcclWork() override {
    if (start_) (void)hipEventDestroy(start_);
    if (end_) (void)hipEventDestroy(end_);
  }
  bool is_completed() override;
  void wait() override;
  void synchronize() override;
  double elapsed_ms() override;

  hipEvent_t start_ = nullptr;
  hipEvent_t end_ = nullptr;
  int device_;
  int64_t issued_ms_;
  int64_t timeout_ms_;
  RcclCommunicator* comm_;
};

class RcclCommunicator : public Communicator {
 public:
  RcclCommunicator(std::shared_ptr<TCPStore> store, const std::string& prefix, int rank, int size, int device,
                   int64_t timeout_ms, ncclComm_t existing = nullptr)
      : Communicator(std::move(store), prefix, rank, size),
        device_(device),
        timeout_ms_(timeout_ms),
        stream_(c10::hip::getStreamFromPool(comm_stream_high_priority(), static_cast<c10::DeviceIndex>(device))) {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    if (existing) {
      comm_ = existing;  // produced by ncclCommSplit of a parent communicator
    } else {
      ncclUniqueId id;
      const std::string key = prefix_ + "/rccl/uid";
      if (rank_ == 0) {
        NCCL_OK(ncclGetUniqueId(&id));
        store_->set(key, std::string(reinterpret_cast<const char*>(&id), sizeof(id)));
      } else {
        const std::string v = store_->get(key);
        DK_CHECK(v.size() == sizeof(id), "RCCL unique id has wrong size");
        std::memcpy(&id, v.data(), sizeof(id));
      }
      NCCL_OK(ncclCommInitRank(&comm_, size_, id, rank_));
    }
    const char* t = std::getenv("DCP_COMM_TIMING");
    timing_ = t && std::string(t) == "1";
    const char* h = std::getenv("DCP_SINGLE_RANK_HOP");
    single_rank_hop_ = h && std::string(h) == "1";
    watchdog_ = std::thread([this] { watchdog(); });
  }

  ~RcclCommunicator() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (watchdog_.joinable()) watchdog_.join();
    if (ready_) (void)hipEventDestroy(ready_);
    if (comm_ && !aborted_.load())
      for (auto& kv : regs_) (void)ncclCommDeregister(comm_, kv.second.first);
    regs_.clear();
    if (comm_) {
      if (aborted_.load()) {
        // already aborted
      } else {
        ncclCommDestroy(comm_);
      }
    }
  }

  int64_t stream_handle() const override { return reinterpret_cast<int64_t>(stream_.stream()); }
  std::string backend() const override { return "rccl"; }
  int transport_size() const override {
    int n = -1;
    if (comm_ && !aborted_.load()) NCCL_OK(ncclCommCount(comm_, &n));
    return n;
  }
  void set_timing(bool on) override { timing_ = on; }

  WorkPtr all_reduce(at::Tensor& t, ReduceOp op) override {
    check_tensor(t);
    account("all_reduce", t, static_cast<int>(op));
    return launch({t}, [&](hipStream_t s) {
      if (size_ == 1 && !single_rank_hop_) return;  // identity for every op on one rank (in place)
      NCCL_OK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()),
                            to_nccl(op, t.scalar_type()), comm_, s));
    });
  }

  WorkPtr all_reduce_into(at::Tensor& wire, at::Tensor& out, ReduceOp op) override {
    check_tensor(wire);
    check_tensor(out);
    DK_CHECK(wire.numel() == out.numel(), "all_reduce_into: wire and out sizes differ");
    account("all_reduce", wire, static_cast<int>(op));
    return launch({wire, out}, [&](hipStream_t s) {
      if (size_ > 1 || single_rank_hop_)
        NCCL_OK(ncclAllReduce(wire.data_ptr(), wire.data_ptr(), wire.numel(), to_nccl(wire.scalar_type()),
                              to_nccl(op, wire.scalar_type()), comm_, s));
      // the cast back runs on the collective's stream, before the Work's end event
      c10::hip::HIPStreamGuard g(c10::hip::getStreamFromExternal(s, static_cast<c10::DeviceIndex>(device_)));
      out.view(-1).copy_(wire.view(-1));
    });
  }

  WorkPtr broadcast(at::Tensor& t, int root) override {
    check_tensor(t);
    account("broadcast", t, root);
    return launch({t}, [&](hipStream_t s) {
      if (size_ == 1 && !single_rank_hop_) return;
      NCCL_OK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, s));
    });
  }

  WorkPtr all_gather(at::Tensor& out, const at::Tensor& in) override {
    check_tensor(out);
    check_tensor(in);
    DK_CHECK(out.numel() == in.numel() * size_, "all_gather: out.numel must be size*in.numel");
    account("all_gather", in);
    return launch({out, in}, [&](hipStream_t s) {
      NCCL_OK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), to_nccl(in.scalar_type()), comm_, s));
    });
  }

  WorkPtr reduce_scatter(at::Tensor& out, const at::Tensor& in, ReduceOp op) override {
    check_tensor(out);
    check_tensor(in);
    DK_CHECK(in.numel() == out.numel() * size_, "reduce_scatter: in.numel must be size*out.numel");
    account("reduce_scatter", in, static_cast<int>(op));
    return launch({out, in}, [&](hipStream_t s) {
      NCCL_OK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), to_nccl(in.scalar_type()),
                                to_nccl(op, in.scalar_type()), comm_, s));
    });
  }

  WorkPtr all_to_all(at::Tensor& out, const at::Tensor& in) override {
    check_tensor(out);
    check_tensor(in);
    DK_CHECK(in.numel() == out.numel() && in.numel() % size_ == 0, "all_to_all: bad sizes");
    account("all_to_all", in);
    return launch({out, in}, [&](hipStream_t s) {
      const int64_t m = in.numel() / size_;
      const int64_t bytes = m * in.element_size();
      auto dt = to_nccl(in.scalar_type());
      NCCL_OK(ncclGroupStart());
      for (int p = 0; p < size_; ++p) {
        NCCL_OK(ncclSend(static_cast<const char*>(in.data_ptr()) + p * bytes, m, dt, p, comm_, s));
        NCCL_OK(ncclRecv(static_cast<char*>(out.data_ptr()) + p * bytes, m, dt, p, comm_, s));
      }
      NCCL_OK(ncclGroupEnd());
    });
  }

  WorkPtr send(const at::Tensor& t, int dst) override {
    check_tensor(t);
    ops_.fetch_add(1);
    return launch({t}, [&](hipStream_t s) {
      NCCL_OK(ncclSend(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), dst, comm_, s));
    });
  }

  WorkPtr recv(at::Tensor& t, int src) override {
    check_tensor(t);
    ops_.fetch_add(1);
    return launch({t}, [&](hipStream_t s) {
      NCCL_OK(ncclRecv(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), src, comm_, s));
    });
  }

  WorkPtr emulate_all_reduce(at::Tensor& t, int world, double busbw_gbps, int channels, double alpha_us) override {
    check_tensor(t);
    DK_CHECK(world >= 2 && busbw_gbps > 0 && channels > 0, "emulate_all_reduce: bad parameters");
    const int64_t bytes = t.numel() * t.element_size();
    const double move = 2.0 * (world - 1) / world * static_cast<double>(bytes);
    const double us = alpha_us + move / (busbw_gbps * 1e3);  // GB/s = 1e3 bytes per µs
    if (!emu_scratch_.defined() || emu_scratch_.numel() < bytes)
      emu_scratch_ = at::empty({bytes}, t.options().dtype(at::kByte));
    ops_.fetch_add(1);
    at::Tensor scratch = emu_scratch_;
    return launch({t, scratch}, [&](hipStream_t s) {
      kern::comm_emulate(t.data_ptr(), scratch.data_ptr(), bytes, static_cast<int64_t>(move), channels, us, s);
    });
  }

  int64_t register_buffer(const at::Tensor& t) override {
    check_tensor(t);
    if (size_ == 1 && !single_rank_hop_) return 0;  // no collective ever touches it
    raise_if_error();
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    void* h = nullptr;
    NCCL_OK(ncclCommRegister(comm_, t.data_ptr(), static_cast<size_t>(t.numel()) * t.element_size(), &h));
    std::lock_guard<std::mutex> g(mu_);
    const int64_t id = ++next_reg_;
    regs_[id] = {h, t};  // the tensor keeps the registered memory alive
    return id;
  }

  void deregister_buffer(int64_t id) override {
    std::pair<void*, at::Tensor> r;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = regs_.find(id);
      if (it == regs_.end()) return;
      r = it->second;
      regs_.erase(it);
    }
    if (!aborted_.load()) {
      c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
      (void)ncclCommDeregister(comm_, r.first);
    }
  }

  WorkPtr stream_fence() override {
    ops_.fetch_add(1);
    return launch({}, [](hipStream_t) {});
  }

  WorkPtr barrier() override {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    if (!barrier_buf_.defined())
      barrier_buf_ = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
    auto w = all_reduce(barrier_buf_, ReduceOp::SUM);
    w->synchronize();
    return w;
  }

  void abort() override {
    if (!aborted_.exchange(true) && comm_) ncclCommAbort(comm_);
  }

  // Sub-communicator via ncclCommSplit (collective over this communicator:
  // every rank calls it; color < 0 = not a member -> nullptr). Same xGMI
  // topology discovery and channels as the parent, no new unique-id
  // rendezvous through the store.
  std::shared_ptr<Communicator> split(int color, int key, const std::string& prefix) override {
    raise_if_error();
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    ncclComm_t sub = nullptr;
    NCCL_OK(ncclCommSplit(comm_, color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &sub, nullptr));
    if (color < 0 || sub == nullptr) return nullptr;
    int n = 0, r = 0;
    NCCL_OK(ncclCommCount(sub, &n));
    NCCL_OK(ncclCommUserRank(sub, &r));
    auto c = std::make_shared<RcclCommunicator>(store_, prefix, r, n, device_, timeout_ms_, sub);
    c->set_debug_fingerprint(fingerprint_);
    return c;
  }

  std::string error() override {
    std::lock_guard<std::mutex> g(mu_);
    return error_;
  }

  void raise_if_error() {
    std::lock_guard<std::mutex> g(mu_);
    if (!error_.empty()) throw Error("RCCL communicator failed: " + error_);
  }

  void set_error(const std::string& e) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (error_.empty()) error_ = e;
    }
    abort();
  }

 private:
  void check_tensor(const at::Tensor& t) {
    DK_CHECK(t.is_cuda(), "RCCL communicator needs device tensors");
    DK_CHECK(t.get_device() == device_, "tensor on device ", t.get_device(), " but communicator on ", device_);
    DK_CHECK(t.is_contiguous() || t.is_non_overlapping_and_dense(), "RCCL needs dense tensors");
  }

  template <typename F>
  WorkPtr launch(std::vector<at::Tensor> ts, F&& issue) {
    raise_if_error();
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    hipStream_t caller = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device_)).stream();
    if (size_ == 1 && !single_rank_hop_) {
      // One rank: every collective is an identity (or a local copy issued by
      // `issue` on the caller's stream) — no comm-stream round trip.
      auto work = std::make_shared<RcclWork>(this, caller, device_, timeout_ms_, false);
      issue(caller);
      HIP_OK(hipEventRecord(work->end_, caller));
      work->outputs = std::move(ts);
      return work;
    }
    hipStream_t comm = stream_.stream();
    auto work = std::make_shared<RcclWork>(this, comm, device_, timeout_ms_, timing_);
    // comm stream waits for everything the caller queued so far (producers of ts)
    // (a wait binds to the event's state at call time, so one event is reused)
    if (!ready_) HIP_OK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
    HIP_OK(hipEventRecord(ready_, caller));
    HIP_OK(hipStreamWaitEvent(comm, ready_, 0));
    // The caching allocator must not recycle these blocks until comm is done.
    for (auto& t : ts) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_);
    if (work->start_) HIP_OK(hipEventRecord(work->start_, comm));
    issue(comm);
    HIP_OK(hipEventRecord(work->end_, comm));
    work->outputs = std::move(ts);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(comm, &cap);
    if (cap == hipStreamCaptureStatusNone) {  // captured events are not queryable: no deadline tracking
      std::lock_guard<std::mutex> g(mu_);
      inflight_.push_back(work);
    }
    return work;
  }

  void watchdog() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      cv_.wait_for(lk, Millis(100));
      if (stop_) break;
      if (!error_.empty()) continue;
      // async errors
      ncclResult_t async = ncclSuccess;
      if (comm_ && !aborted_.load() && ncclCommGetAsyncError(comm_, &async) == ncclSuccess &&
          async != ncclSuccess && async != ncclInProgress) {
        error_ = str_cat("async RCCL error: ", ncclGetErrorString(async));
        lk.unlock();
        abort();
        lk.lock();
        continue;
      }
      // deadlines
      const int64_t now = now_ms();
      for (auto it = inflight_.begin(); it != inflight_.end();) {
        auto w = it->lock();
        if (!w) {
          it = inflight_.erase(it);
          continue;
        }
        if (hipEventQuery(w->end_) == hipSuccess) {
          it = inflight_.erase(it);
          continue;
        }
        if (timeout_ms_ > 0 && now - w->issued_ms_ > timeout_ms_) {
          error_ = str_cat("collective timed out after ", now - w->issued_ms_, " ms (timeout ", timeout_ms_,
                           " ms) on rank ", rank_);
          lk.unlock();
          abort();
          lk.lock();
          break;
        }
        ++it;
      }
    }
  }

  int device_;
  int64_t timeout_ms_;
  c10::hip::HIPStream stream_;
  ncclComm_t comm_ = nullptr;
  bool timing_ = false;
  bool single_rank_hop_ = false;
  std::atomic<bool> aborted_{false};
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::string error_;
  std::list<std::weak_ptr<RcclWork>> inflight_;
  std::thread watchdog_;
  at::Tensor barrier_buf_;
  at::Tensor emu_scratch_;
  hipEvent_t ready_ = nullptr;
  std::map<int64_t, std::pair<void*, at::Tensor>> regs_;  // register_buffer handles
  int64_t next_reg_ = 0;
};

RcclWork::RcclWork(RcclCommunicator* comm, hipStream_t, int device, int64_t timeout_ms, bool timing)
    : device_(device), issued_ms_(now_ms()), timeout_ms_(timeout_ms), comm_(comm) {
  HIP_OK(hipEventCreateWithFlags(&end_, timing ? hipEventDefault : hipEventDisableTiming));
  if (timing) HIP_OK(hipEventCreateWithFlags(&start_, hipEventDefault));
}

bool RcclWork::is_completed() {
  comm_->raise_if_error();
  return hipEventQuery(end_) == hipSuccess;
}

void RcclWork::wait() {
  comm_->raise_if_error();
  hipStream_t cur = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device_)).stream();
  HIP_OK(hipStreamWaitEvent(cur, end_, 0));
}

void RcclWork::synchronize() {
  // Poll instead of hipEventSynchronize so a watchdog abort can release us.
  while (true) {
    comm_->raise_if_error();
    hipError_t e = hipEventQuery(end_);
    if (e == hipSuccess) return;
    DK_CHECK(e == hipErrorNotReady, "hipEventQuery failed: ", hipGetErrorString(e));
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

double RcclWork::elapsed_ms() {
  if (!start_) return -1.0;
  if (hipEventQuery(end_) != hipSuccess) return -1.0;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, start_, end_) != hipSuccess) return -1.0;
  return ms;
}

}  // namespace

std::shared_ptr<Communicator> make_rccl_communicator(std::shared_ptr<TCPStore> store, const std::string& prefix,
                                                     int rank, int size, int device, int64_t timeout_ms) {
  return std::make_shared<RcclCommunicator>(std::move(store), prefix, rank, size, device, timeout_ms);
}

bool rccl_available() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

std::string rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return std::to_string(v);
}

}  // namespace dcp
