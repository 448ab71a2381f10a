// Host (CPU) communicator: TCP full mesh + ring collectives on a worker thread.
//
// Parity: ProcessGroupGloo as used by the reference (main.py:50) — it carries
// the CPU-only configuration (BASELINE config #1, world_size=2 on CPU) and
// every multi-process CPU test. GPU tensors handed to it are staged through
// host memory like gloo does (reference-literal "gloo on GPU" variant).
#include <ATen/Dispatch.h>

#include <condition_variable>
#include <deque>
#include <functional>
#include <thread>

#include "../common.h"
#include "../store/socket.h"
#include "communicator.h"

namespace dcp {

namespace {

template <typename T>
inline T apply_op(T a, T b, ReduceOp op) {
  switch (op) {
    case ReduceOp::SUM:
    case ReduceOp::AVG:
      return static_cast<T>(a + b);
    case ReduceOp::PRODUCT:
      return static_cast<T>(a * b);
    case ReduceOp::MIN:
      return b < a ? b : a;
    case ReduceOp::MAX:
      return a < b ? b : a;
  }
  return a;
}

void reduce_into(void* dst, const void* src, int64_t n, at::ScalarType st, ReduceOp op) {
  AT_DISPATCH_ALL_TYPES_AND3(at::kBFloat16, at::kHalf, at::kBool, st, "host_reduce", [&] {
    scalar_t* d = static_cast<scalar_t*>(dst);
    const scalar_t* s = static_cast<const scalar_t*>(src);
    for (int64_t i = 0; i < n; ++i) d[i] = apply_op<scalar_t>(d[i], s[i], op);
  });
}

void divide_by(void* buf, int64_t n, at::ScalarType st, int64_t world) {
  AT_DISPATCH_ALL_TYPES_AND2(at::kBFloat16, at::kHalf, st, "host_avg", [&] {
    scalar_t* d = static_cast<scalar_t*>(buf);
    for (int64_t i = 0; i < n; ++i) d[i] = static_cast<scalar_t>(d[i] / static_cast<scalar_t>(world));
  });
}

class HostWork : public Work {
 public:
  bool is_completed() override {
    std::lock_guard<std::mutex> g(mu);
    return done;
  }
  void wait() override { synchronize(); }
  void synchronize() override {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
    if (!err.empty()) throw Error(err);
    if (post) {
      auto f = std::move(post);
      post = nullptr;
      lk.unlock();
      f();
    }
  }
  void finish(const std::string& e) {
    {
      std::lock_guard<std::mutex> g(mu);
      done = true;
      err = e;
    }
    cv.notify_all();
  }
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::string err;
  std::function<void()> post;  // runs on the waiting thread (e.g. H2D copy-back)
};

class HostCommunicator : public Communicator {
 public:
  HostCommunicator(std::shared_ptr<TCPStore> store, const std::string& prefix, int rank, int size,
                   int64_t timeout_ms)
      : Communicator(std::move(store), prefix, rank, size), timeout_ms_(timeout_ms), peers_(size, -1) {
    connect_mesh();
    worker_ = std::thread([this] { run(); });
  }

  ~HostCommunicator() override {
    {
      std::lock_guard<std::mutex> g(qmu_);
      stop_ = true;
    }
    qcv_.notify_all();
    if (worker_.joinable()) worker_.join();
    for (int fd : peers_)
      if (fd >= 0) ::close(fd);
    if (listen_fd_ >= 0) ::close(listen_fd_);
  }

  std::string backend() const override { return "host"; }

  WorkPtr all_reduce(at::Tensor& t, ReduceOp op) override {
    account("all_reduce", t, static_cast<int>(op));
    return submit({t}, [this, op](std::vector<at::Tensor>& ts) { ring_all_reduce(ts[0], op); });
  }

  WorkPtr broadcast(at::Tensor& t, int root) override {
    account("broadcast", t, root);
    return submit({t}, [this, root](std::vector<at::Tensor>& ts) { do_broadcast(ts[0], root); });
  }

  WorkPtr all_gather(at::Tensor& out, const at::Tensor& in) override {
    DK_CHECK(out.numel() == in.numel() * size_, "all_gather: out.numel must be size*in.numel");
    account("all_gather", in);
    return submit({out, in}, [this](std::vector<at::Tensor>& ts) { ring_all_gather(ts[0], ts[1]); });
  }

  WorkPtr reduce_scatter(at::Tensor& out, const at::Tensor& in, ReduceOp op) override {
    DK_CHECK(in.numel() == out.numel() * size_, "reduce_scatter: in.numel must be size*out.numel");
    account("reduce_scatter", in, static_cast<int>(op));
    return submit({out, in}, [this, op](std::vector<at::Tensor>& ts) { ring_reduce_scatter(ts[0], ts[1], op); });
  }

  WorkPtr all_to_all(at::Tensor& out, const at::Tensor& in) override {
    DK_CHECK(in.numel() == out.numel() && in.numel() % size_ == 0, "all_to_all: bad sizes");
    account("all_to_all", in);
    return submit({out, in}, [this](std::vector<at::Tensor>& ts) { do_all_to_all(ts[0], ts[1]); });
  }

  WorkPtr send(const at::Tensor& t, int dst) override {
    ops_.fetch_add(1);
    return submit({t}, [this, dst](std::vector<at::Tensor>& ts) {
      auto& x = ts[0];
      DK_CHECK(net::send_all(peers_[dst], x.data_ptr(), x.numel() * x.element_size()), "send failed");
    });
  }

  WorkPtr recv(at::Tensor& t, int src) override {
    ops_.fetch_add(1);
    return submit({t}, [this, src](std::vector<at::Tensor>& ts) {
      auto& x = ts[0];
      DK_CHECK(net::recv_all(peers_[src], x.data_ptr(), x.numel() * x.element_size(), timeout_ms_),
                "recv failed: peer closed");
    });
  }

  WorkPtr barrier() override {
    auto t = at::zeros({1}, at::kFloat);
    return all_reduce(t, ReduceOp::SUM);
  }

  std::string error() override {
    std::lock_guard<std::mutex> g(qmu_);
    return error_;
  }

 private:
  using Fn = std::function<void(std::vector<at::Tensor>&)>;

  // CPU tensors run in place (contiguous required). GPU tensors are staged:
  // D2H on the caller thread, collective on the worker, H2D on wait().
  WorkPtr submit(std::vector<at::Tensor> ts, Fn fn) {
    auto w = std::make_shared<HostWork>();
    std::vector<at::Tensor> host(ts.size());
    bool staged = false;
    for (size_t i = 0; i < ts.size(); ++i) {
      if (!ts[i].device().is_cpu()) {
        staged = true;
        host[i] = ts[i].to(at::kCPU).contiguous();
      } else {
        DK_CHECK(ts[i].is_contiguous(), "host communicator needs contiguous tensors");
        host[i] = ts[i];
      }
    }
    if (staged) {
      auto originals = ts;
      auto hs = host;
      w->post = [originals, hs]() mutable {
        for (size_t i = 0; i < originals.size(); ++i)
          if (!originals[i].device().is_cpu()) originals[i].copy_(hs[i]);
      };
    }
    w->outputs = ts;
    {
      std::lock_guard<std::mutex> g(qmu_);
      if (!error_.empty()) throw Error("host communicator is in error state: " + error_);
      queue_.push_back(Task{std::move(host), std::move(fn), w});
    }
    qcv_.notify_one();
    return w;
  }

  struct Task {
    std::vector<at::Tensor> ts;
    Fn fn;
    std::shared_ptr<HostWork> work;
  };

  void run() {
    while (true) {
      Task task;
      {
        std::unique_lock<std::mutex> lk(qmu_);
        qcv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
        if (queue_.empty() && stop_) return;
        task = std::move(queue_.front());
        queue_.pop_front();
      }
      std::string err;
      try {
        if (size_ > 1) task.fn(task.ts);
      } catch (const std::exception& e) {
        err = e.what();
        std::lock_guard<std::mutex> g(qmu_);
        error_ = err;
      }
      task.work->finish(err);
    }
  }

  void connect_mesh() {
    if (size_ == 1) return;
    int port = 0;
    listen_fd_ = net::listen_on("0.0.0.0", 0, &port);
    const std::string me = store_->local_ip() + ":" + std::to_string(port);
    store_->set(prefix_ + "/host/addr/" + std::to_string(rank_), me);
    // Connect to every lower rank; accept every higher rank.
    for (int j = 0; j < rank_; ++j) {
      const std::string addr = store_->get(prefix_ + "/host/addr/" + std::to_string(j));
      const auto colon = addr.rfind(':');
      int fd = net::connect_to(addr.substr(0, colon), std::stoi(addr.substr(colon + 1)), timeout_ms_);
      int32_t r = rank_;
      DK_CHECK(net::send_all(fd, &r, sizeof(r)), "mesh handshake failed");
      net::set_bufsizes(fd, 4 << 20);
      peers_[j] = fd;
    }
    for (int k = rank_ + 1; k < size_; ++k) {
      int fd = net::accept_one(listen_fd_, timeout_ms_);
      int32_t r = -1;
      DK_CHECK(net::recv_all(fd, &r, sizeof(r), timeout_ms_), "mesh handshake failed");
      DK_CHECK(r > rank_ && r < size_ && peers_[r] < 0, "mesh handshake: unexpected rank ", r);
      net::set_bufsizes(fd, 4 << 20);
      peers_[r] = fd;
    }
  }

  int next() const { return (rank_ + 1) % size_; }
  int prev() const { return (rank_ - 1 + size_) % size_; }

  // chunk c of n elements split into size_ parts
  std::pair<int64_t, int64_t> chunk(int64_t n, int c) const {
    const int64_t b = n * c / size_;
    const int64_t e = n * (c + 1) / size_;
    return {b, e - b};
  }

  void ring_reduce_scatter_inplace(char* base, int64_t n, at::ScalarType st, int64_t es, ReduceOp op) {
    std::vector<char> tmp;
    for (int s = 0; s < size_ - 1; ++s) {
      const int sc = ((rank_ - s) % size_ + size_) % size_;
      const int rc = ((rank_ - s - 1) % size_ + size_) % size_;
      auto [sb, sn] = chunk(n, sc);
      auto [rb, rn] = chunk(n, rc);
      tmp.resize(static_cast<size_t>(rn * es));
      net::send_recv(peers_[next()], base + sb * es, sn * es, peers_[prev()], tmp.data(), rn * es, timeout_ms_);
      reduce_into(base + rb * es, tmp.data(), rn, st, op);
    }
  }

  void ring_all_gather_inplace(char* base, int64_t n, int64_t es, int own_chunk_shift) {
    for (int s = 0; s < size_ - 1; ++s) {
      const int sc = ((rank_ + own_chunk_shift - s) % size_ + size_) % size_;
      const int rc = ((rank_ + own_chunk_shift - s - 1) % size_ + size_) % size_;
      auto [sb, sn] = chunk(n, sc);
      auto [rb, rn] = chunk(n, rc);
      net::send_recv(peers_[next()], base + sb * es, sn * es, peers_[prev()], base + rb * es, rn * es,
                     timeout_ms_);
    }
  }

  void ring_all_reduce(at::Tensor& t, ReduceOp op) {
    const int64_t n = t.numel();
    const int64_t es = t.element_size();
    char* base = static_cast<char*>(t.data_ptr());
    ring_reduce_scatter_inplace(base, n, t.scalar_type(), es, op);
    // After reduce-scatter rank r owns the fully reduced chunk (r+1) % size.
    const int own = (rank_ + 1) % size_;
    if (op == ReduceOp::AVG) {
      auto [ob, on] = chunk(n, own);
      divide_by(base + ob * es, on, t.scalar_type(), size_);
    }
    ring_all_gather_inplace(base, n, es, /*own_chunk_shift=*/1);
  }

  void ring_all_gather(at::Tensor& out, const at::Tensor& in) {
    const int64_t es = in.element_size();
    const int64_t m = in.numel();
    char* base = static_cast<char*>(out.data_ptr());
    std::memcpy(base + rank_ * m * es, in.data_ptr(), m * es);
    // Blocks are equal so chunk(n, c) == block c.
    ring_all_gather_inplace(base, m * size_, es, /*own_chunk_shift=*/0);
  }

  void ring_reduce_scatter(at::Tensor& out, const at::Tensor& in, ReduceOp op) {
    const int64_t es = in.element_size();
    const int64_t m = out.numel();
    at::Tensor work = in.clone();
    char* base = static_cast<char*>(work.data_ptr());
    // Shift so that rank r ends owning block r: reduce-scatter ring leaves rank r
    // owning chunk (r+1); run it on the buffer rotated by one block.
    ring_reduce_scatter_rotated(base, m, in.scalar_type(), es, op);
    if (op == ReduceOp::AVG) divide_by(base + rank_ * m * es, m, in.scalar_type(), size_);
    std::memcpy(out.data_ptr(), base + rank_ * m * es, m * es);
  }

  void ring_reduce_scatter_rotated(char* base, int64_t m, at::ScalarType st, int64_t es, ReduceOp op) {
    std::vector<char> tmp(static_cast<size_t>(m * es));
    for (int s = 0; s < size_ - 1; ++s) {
      const int sc = ((rank_ - s - 1) % size_ + size_) % size_;
      const int rc = ((rank_ - s - 2) % size_ + size_) % size_;
      net::send_recv(peers_[next()], base + sc * m * es, m * es, peers_[prev()], tmp.data(), m * es, timeout_ms_);
      reduce_into(base + rc * m * es, tmp.data(), m, st, op);
    }
  }

  void do_broadcast(at::Tensor& t, int root) {
    const size_t bytes = static_cast<size_t>(t.numel() * t.element_size());
    if (rank_ == root) {
      for (int j = 0; j < size_; ++j)
        if (j != root) DK_CHECK(net::send_all(peers_[j], t.data_ptr(), bytes), "broadcast send failed");
    } else {
      DK_CHECK(net::recv_all(peers_[root], t.data_ptr(), bytes, timeout_ms_), "broadcast recv failed");
    }
  }

  void do_all_to_all(at::Tensor& out, const at::Tensor& in) {
    const int64_t es = in.element_size();
    const int64_t m = in.numel() / size_;
    const char* src = static_cast<const char*>(in.data_ptr());
    char* dst = static_cast<char*>(out.data_ptr());
    std::memcpy(dst + rank_ * m * es, src + rank_ * m * es, m * es);
    for (int k = 1; k < size_; ++k) {
      const int to = (rank_ + k) % size_;
      const int from = (rank_ - k + size_) % size_;
      net::send_recv(peers_[to], src + to * m * es, m * es, peers_[from], dst + from * m * es, m * es, timeout_ms_);
    }
  }

  int64_t timeout_ms_;
  int listen_fd_ = -1;
  std::vector<int> peers_;
  std::thread worker_;
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<Task> queue_;
  bool stop_ = false;
  std::string error_;
};

}  // namespace

std::shared_ptr<Communicator> make_host_communicator(std::shared_ptr<TCPStore> store, const std::string& prefix,
                                                     int rank, int size, int64_t timeout_ms) {
  return std::make_shared<HostCommunicator>(std::move(store), prefix, rank, size, timeout_ms);
}

}  // namespace dcp
