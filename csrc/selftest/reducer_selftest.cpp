// Multi-process self-test of the host communicator + Reducer, built with
// ASan/UBSan by tests/test_sanitizers.py (the threaded hook /
// launch / finalize logic and the socket ring collectives under sanitizers).
//
// The parent forks `world` ranks BEFORE any thread exists; each rank builds a
// TCPStore + host communicator, a Reducer over CPU parameters with small
// buckets, and runs backward passes through libtorch autograd:
//   * synced steps: every gradient equals the average of the ranks' local
//     gradients (closed form: d/dp sum(p * c_r) = c_r);
//   * a no_sync step followed by a synced one: local accumulation, then the
//     average of the accumulated sums;
//   * find_unused_parameters with a parameter unused on every rank and one
//     unused on rank 0 only;
//   * bucket rebuild after the first iteration (ready order).
// Exit status 0 and "OK" on success; any mismatch aborts with a message.
#include <sys/socket.h>
#include <sys/wait.h>
#include <netinet/in.h>
#include <unistd.h>

#include <torch/torch.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "comm/communicator.h"
#include "reducer/reducer.h"
#include "store/tcp_store.h"

using dcp::Reducer;
using dcp::ReducerOptions;

namespace {

void check(bool ok, const char* what, int rank) {
  if (!ok) {
    std::fprintf(stderr, "[rank %d] FAILED: %s\n", rank, what);
    std::fflush(stderr);
    std::abort();
  }
}

int free_port() {
  int s = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  ::bind(s, reinterpret_cast<sockaddr*>(&a), sizeof(a));
  socklen_t len = sizeof(a);
  ::getsockname(s, reinterpret_cast<sockaddr*>(&a), &len);
  const int p = ntohs(a.sin_port);
  ::close(s);
  return p;
}

// coefficient of parameter i on rank r (local gradient of sum(p * c))
float coef(int i, int r) { return 0.5f + static_cast<float>(i) + 0.25f * static_cast<float>(r); }

void run(int rank, int world, int port, bool find_unused, bool as_view) {
  auto store = std::make_shared<dcp::TCPStore>("127.0.0.1", port, world, rank == 0, 30000, false);
  const std::string prefix = std::string("asan") + (find_unused ? "u" : "") + (as_view ? "v" : "");
  auto comm = dcp::make_host_communicator(store, prefix, rank, world, 30000);

  torch::manual_seed(0);
  const std::vector<int64_t> numels = {37, 1000, 5, 4096, 64, 300};
  std::vector<at::Tensor> params;
  std::vector<int64_t> bytes, keys;
  for (int64_t n : numels) {
    params.push_back(torch::randn({n}).requires_grad_(true));
    bytes.push_back(n * 4);
    keys.push_back(0);
  }
  // several small buckets so launches interleave with the remaining backward
  auto buckets = dcp::compute_bucket_assignment(bytes, keys, {1024, 8192}, {});
  ReducerOptions o;
  o.find_unused_parameters = find_unused;
  o.gradient_as_bucket_view = as_view;
  o.first_bucket_bytes = 1024;
  o.bucket_bytes_cap = 8192;
  auto red = std::make_shared<Reducer>(params, buckets, comm, o);
  red->register_hooks();

  const int n = static_cast<int>(params.size());
  // unused: param 4 everywhere, param 2 on rank 0 only (find_unused runs)
  auto used = [&](int i) { return !(find_unused && (i == 4 || (i == 2 && rank == 0))); };
  auto forward = [&] {
    at::Tensor loss = torch::zeros({});
    for (int i = 0; i < n; ++i)
      if (used(i)) loss = loss + (params[i] * coef(i, rank)).sum();
    return loss;
  };
  auto expect_avg = [&](int i, float scale) {
    // average over ranks of the local gradient (0 where a rank did not use it)
    float s = 0.f;
    for (int r = 0; r < world; ++r) {
      const bool u = !(find_unused && (i == 4 || (i == 2 && r == 0)));
      s += u ? coef(i, r) : 0.f;
    }
    return scale * s / static_cast<float>(world);
  };
  auto zero_grads = [&] {
    for (auto& p : params)
      if (p.grad().defined()) p.mutable_grad().zero_();
  };

  for (int it = 0; it < 4; ++it) {
    zero_grads();
    at::Tensor loss = forward();
    red->prepare_for_backward({loss}, true);
    loss.backward();
    red->wait_all();
    for (int i = 0; i < n; ++i) {
      if (find_unused && i == 4) {
        check(!params[i].grad().defined() || params[i].grad().abs().max().item<float>() == 0.f,
              "globally unused parameter got a gradient", rank);
        continue;
      }
      check(params[i].grad().defined(), "missing gradient", rank);
      const float want = expect_avg(i, 1.f);
      const float got_max = params[i].grad().max().item<float>(), got_min = params[i].grad().min().item<float>();
      check(std::fabs(got_max - want) < 1e-5f && std::fabs(got_min - want) < 1e-5f, "synced gradient != average",
            rank);
    }
  }
  // no_sync accumulation, then one synced step: average of the summed local grads
  zero_grads();
  {
    at::Tensor loss = forward();
    red->prepare_for_backward({loss}, false);
    loss.backward();
  }
  for (int i = 0; i < n; ++i)
    if (used(i))
      check(std::fabs(params[i].grad().max().item<float>() - coef(i, rank)) < 1e-5f, "no_sync grad not local", rank);
  {
    at::Tensor loss = forward();
    red->prepare_for_backward({loss}, true);
    loss.backward();
    red->wait_all();
  }
  for (int i = 0; i < n; ++i) {
    if (find_unused && i == 4) continue;
    // torch semantics: a parameter used in a no_sync step counts as used
    float s = 0.f;
    for (int r = 0; r < world; ++r) {
      const bool u = !(find_unused && (i == 4 || (i == 2 && r == 0)));
      s += u ? 2.f * coef(i, r) : 0.f;
    }
    const float want = s / static_cast<float>(world);
    check(std::fabs(params[i].grad().max().item<float>() - want) < 1e-4f, "accumulated gradient != average", rank);
  }
  check(red->num_iterations() >= 5, "iteration count", rank);
  comm->barrier()->wait();
}

}  // namespace

int main(int argc, char** argv) {
  const int world = argc > 1 ? std::atoi(argv[1]) : 2;
  for (int cfg = 0; cfg < 4; ++cfg) {
    const bool find_unused = cfg & 1, as_view = cfg & 2;
    const int port = free_port();
    std::vector<pid_t> kids;
    std::fflush(stdout);  // children must not inherit (and re-print) buffered output
    for (int r = 0; r < world; ++r) {
      const pid_t pid = ::fork();
      if (pid == 0) {
        run(r, world, port, find_unused, as_view);
        std::fflush(stdout);
        ::_exit(0);
      }
      kids.push_back(pid);
    }
    for (pid_t k : kids) {
      int st = 0;
      ::waitpid(k, &st, 0);
      if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
        std::fprintf(stderr, "rank process failed (cfg %d, status %d)\n", cfg, st);
        return 1;
      }
    }
    std::printf("cfg find_unused=%d as_view=%d ok\n", find_unused, as_view);
  }
  std::printf("OK\n");
  return 0;
}
