#include "reducer.h"

#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <optional>
#include <thread>
#include <unordered_set>

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <cstdlib>
#include <cstring>

#include "../common.h"
#include "../ops.h"
#include "../trace/trace.h"

namespace dcp {

// ------------------------------------------------------------ planner ----
std::vector<std::vector<int64_t>> compute_bucket_assignment(const std::vector<int64_t>& sizes_bytes,
                                                            const std::vector<int64_t>& keys,
                                                            const std::vector<int64_t>& limits,
                                                            const std::vector<int64_t>& order) {
  DK_CHECK(sizes_bytes.size() == keys.size(), "planner: sizes/keys length mismatch");
  DK_CHECK(!limits.empty(), "planner: empty limit list");
  struct Acc {
    std::vector<int64_t> idx;
    int64_t size = 0;
  };
  std::map<int64_t, Acc> open;
  std::map<int64_t, size_t> limit_it;
  std::vector<std::vector<int64_t>> result;
  const size_t n = order.empty() ? sizes_bytes.size() : order.size();
  for (size_t k = 0; k < n; ++k) {
    const int64_t i = order.empty() ? static_cast<int64_t>(k) : order[k];
    DK_CHECK(i >= 0 && i < static_cast<int64_t>(sizes_bytes.size()), "planner: bad index ", i);
    const int64_t key = keys[i];
    Acc& b = open[key];
    b.idx.push_back(i);
    b.size += sizes_bytes[i];
    size_t& li = limit_it[key];  // value-initialised to 0 on first use
    if (b.size >= limits[li]) {
      result.push_back(std::move(b.idx));
      b = Acc();
      if (li + 1 < limits.size()) ++li;
    }
  }
  for (auto& kv : open)
    if (!kv.second.idx.empty()) result.push_back(std::move(kv.second.idx));
  if (order.empty()) {
    std::sort(result.begin(), result.end(), [](const std::vector<int64_t>& a, const std::vector<int64_t>& b) {
      return *std::min_element(a.begin(), a.end()) < *std::min_element(b.begin(), b.end());
    });
  }
  return result;
}

std::vector<std::vector<int64_t>> split_tail_bucket(std::vector<std::vector<int64_t>> assignment,
                                                    const std::vector<int64_t>& sizes_bytes, int64_t tail_bytes) {
  if (tail_bytes <= 0 || assignment.empty()) return assignment;
  std::vector<int64_t>& last = assignment.back();
  int64_t total = 0;
  for (int64_t i : last) total += sizes_bytes.at(i);
  if (total <= tail_bytes || last.size() < 2) return assignment;
  size_t cut = last.size() - 1;  // the tail takes at least the last-ready parameter
  int64_t tail = sizes_bytes.at(last[cut]);
  while (cut > 1 && tail + sizes_bytes.at(last[cut - 1]) <= tail_bytes) tail += sizes_bytes.at(last[--cut]);
  std::vector<int64_t> t(last.begin() + static_cast<std::ptrdiff_t>(cut), last.end());
  last.resize(cut);
  assignment.push_back(std::move(t));
  return assignment;
}

namespace {

int64_t bucket_key(const at::Tensor& t) {
  return (static_cast<int64_t>(t.scalar_type()) << 32) | (static_cast<int64_t>(t.device().type()) << 16) |
         static_cast<int64_t>(t.device().index() + 1);
}

bool same_layout(const at::Tensor& a, const at::Tensor& b) {
  return a.sizes() == b.sizes() && (a.strides() == b.strides() || (a.is_contiguous() && b.is_contiguous()));
}

}  // namespace

// ------------------------------------------------------------ reducer ----
Reducer::Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
                 std::shared_ptr<Communicator> comm, ReducerOptions opts)
    : params_(std::move(params)), comm_(std::move(comm)), opts_(opts) {
  for (auto& p : params_) {
    DK_CHECK(p.requires_grad(), "Reducer: every parameter must require grad");
    DK_CHECK(p.is_non_overlapping_and_dense(), "Reducer: parameters must be dense");
  }
  ready_.assign(params_.size(), 0);
  unused_.assign(params_.size(), 0);
  used_since_sync_.assign(params_.size(), 0);
  build_buckets(buckets);
  const char* t = std::getenv("DCP_COMM_TIMING");
  timing_ = t && std::strcmp(t, "1") == 0 && !params_.empty() && params_[0].is_cuda();
  const char* ds = std::getenv("DCP_DEBUG_STREAMS");
  check_ = opts_.check_streams || (ds && std::strcmp(ds, "1") == 0);
}

double Reducer::exposed_comm_ms() {
  std::lock_guard<std::mutex> g(mu_);
  if (!timing_ || !ev_recorded_) return -1.0;
  double total = 0.0;
  for (auto& b : buckets_) {
    if (!b.stall_recorded) continue;
    if (hipEventSynchronize(b.stall1) != hipSuccess) return -1.0;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, b.stall0, b.stall1) != hipSuccess) return -1.0;
    total += ms;
  }
  return total;
}

void Reducer::wait_bucket(Bucket& b, hipStream_t cur, bool timed) {
  if (timed) {
    if (!b.stall0) {
      DK_CHECK(hipEventCreate(&b.stall0) == hipSuccess && hipEventCreate(&b.stall1) == hipSuccess,
               "Reducer: event creation failed");
    }
    (void)hipEventRecord(b.stall0, cur);
  }
  if (!b.slice_works.empty()) {
    for (auto& w : b.slice_works)
      if (w) w->wait();
  } else {
    b.work->wait();
  }
  if (timed) {
    (void)hipEventRecord(b.stall1, cur);
    b.stall_recorded = true;
    ev_recorded_ = true;
  }
}

void Reducer::sync_locked(Bucket& b) {
  if (!b.deferred) return;
  hipStream_t cur = nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (b.flat.is_cuda()) {
    cur = c10::hip::getCurrentHIPStream(b.flat.device().index()).stream();
    (void)hipStreamIsCapturing(cur, &cap);
  }
  const bool timed = timing_ && cap == hipStreamCaptureStatusNone;
  if (!b.slice_works.empty()) {
    if (timed) {  // the stall events around the wait on every slice
      wait_bucket(b, cur, true);
      b.timed_work = b.work;
    }
    // only the slices not synced yet (each unpacks its own wire range)
    for (size_t s = 0; s < b.slice_works.size(); ++s) sync_slice_locked(b, s);
    finish_slices(b);
    return;
  }
  wait_bucket(b, cur, timed);
  if (timed) b.timed_work = b.work;
  if (!b.wire.is_same(b.flat)) ops::mt_copy({b.wire}, {b.flat}, 1.0);
  b.work.reset();
  b.deferred = false;
}

void Reducer::sync_slice_locked(Bucket& b, size_t s) {
  if (b.slice_synced[s]) return;
  b.slice_works[s]->wait();
  if (!b.wire.is_same(b.flat)) {
    const int64_t lo = b.slice_bounds[s], n = b.slice_bounds[s + 1] - lo;
    ops::mt_copy({b.wire.narrow(0, lo, n)}, {b.flat.narrow(0, lo, n)}, 1.0);
  }
  b.slice_synced[s] = 1;
}

void Reducer::finish_slices(Bucket& b) {
  for (char c : b.slice_synced)
    if (!c) return;
  b.slice_works.clear();
  b.slice_synced.clear();
  b.work.reset();
  b.deferred = false;
}

std::vector<int64_t> Reducer::bucket_slice_bounds(int64_t k) {
  std::lock_guard<std::mutex> g(mu_);
  DK_CHECK(k >= 0 && k < static_cast<int64_t>(buckets_.size()), "Reducer::bucket_slice_bounds: bad bucket ", k);
  const Bucket& b = buckets_[k];
  if (!b.deferred || b.slice_works.empty()) return {};
  return b.slice_bounds;
}

void Reducer::sync_bucket_slice(int64_t k, int64_t s) {
  std::lock_guard<std::mutex> g(mu_);
  DK_CHECK(k >= 0 && k < static_cast<int64_t>(buckets_.size()), "Reducer::sync_bucket_slice: bad bucket ", k);
  Bucket& b = buckets_[k];
  if (!b.deferred) return;
  if (b.slice_works.empty() || timing_) {  // not sliced, or timed (the stall events span the whole bucket)
    sync_locked(b);
    return;
  }
  DK_CHECK(s >= 0 && s < static_cast<int64_t>(b.slice_works.size()), "Reducer::sync_bucket_slice: bad slice ", s);
  sync_slice_locked(b, static_cast<size_t>(s));
  finish_slices(b);
}

std::vector<int64_t> Reducer::deferred_buckets() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<int64_t> r;
  for (size_t k = 0; k < buckets_.size(); ++k)
    if (buckets_[k].deferred) r.push_back(static_cast<int64_t>(k));
  return r;
}

void Reducer::sync_bucket(int64_t k) {
  std::lock_guard<std::mutex> g(mu_);
  DK_CHECK(k >= 0 && k < static_cast<int64_t>(buckets_.size()), "Reducer::sync_bucket: bad bucket ", k);
  sync_locked(buckets_[k]);
}

void Reducer::sync_all() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& b : buckets_) sync_locked(b);
}

Reducer::~Reducer() {
  for (auto& b : buckets_) {
    if (b.stall0) (void)hipEventDestroy(b.stall0);
    if (b.stall1) (void)hipEventDestroy(b.stall1);
    if (b.ready_ev) (void)hipEventDestroy(b.ready_ev);
  }
  release_registrations();
  if (used_ev_) (void)hipEventDestroy(used_ev_);
  if (bwd_t0_ev_) (void)hipEventDestroy(bwd_t0_ev_);
  for (size_t i = 0; i < grad_accs_.size() && i < hook_handles_.size(); ++i)
    grad_accs_[i]->del_post_hook(hook_handles_[i]);
}

void Reducer::build_buckets(const std::vector<std::vector<int64_t>>& assignment) {
  std::vector<char> seen(params_.size(), 0);
  std::vector<Bucket> out;
  out.reserve(assignment.size());
  where_.assign(params_.size(), {-1, -1});
  for (size_t bi = 0; bi < assignment.size(); ++bi) {
    const auto& idx = assignment[bi];
    DK_CHECK(!idx.empty(), "Reducer: empty bucket");
    Bucket b;
    b.params = idx;
    const at::Tensor& p0 = params_[idx[0]];
    int64_t total = 0;
    for (int64_t i : idx) {
      DK_CHECK(i >= 0 && i < static_cast<int64_t>(params_.size()) && !seen[i], "Reducer: bad bucket index ", i);
      seen[i] = 1;
      DK_CHECK(params_[i].scalar_type() == p0.scalar_type() && params_[i].device() == p0.device(),
                "Reducer: a bucket must be single dtype/device");
      b.offsets.push_back(total);
      total += params_[i].numel();
    }
    b.flat = at::zeros({total}, p0.options().requires_grad(false));
    if (opts_.comm_dtype != at::ScalarType::Undefined && opts_.comm_dtype != p0.scalar_type())
      b.wire = at::empty({total}, b.flat.options().dtype(opts_.comm_dtype));
    else
      b.wire = b.flat;
    for (size_t s = 0; s < idx.size(); ++s) {
      const at::Tensor& p = params_[idx[s]];
      b.views.push_back(b.flat.as_strided(p.sizes(), p.strides(), b.offsets[s]));
      where_[idx[s]] = {static_cast<int64_t>(bi), static_cast<int64_t>(s)};
    }
    b.pending_grads.resize(idx.size());
    b.pending = static_cast<int>(idx.size());
    b.stats.bytes = total * p0.element_size();
    b.stats.num_params = static_cast<int64_t>(idx.size());
    if (opts_.slice_bytes > 0 && 2 * b.stats.bytes > 3 * opts_.slice_bytes) {
      const int64_t n = (b.stats.bytes + opts_.slice_bytes - 1) / opts_.slice_bytes;
      const int64_t al = std::max<int64_t>(1, 256 / static_cast<int64_t>(b.wire.element_size()));
      const int64_t per = ((total + n - 1) / n + al - 1) / al * al;
      for (int64_t lo = 0; lo < total; lo += per) b.slice_bounds.push_back(lo);
      b.slice_bounds.push_back(total);
    }
    out.push_back(std::move(b));
  }
  for (size_t i = 0; i < params_.size(); ++i) DK_CHECK(seen[i], "Reducer: parameter ", i, " not in any bucket");
  release_registrations();
  for (auto& b : buckets_) {
    if (b.stall0) (void)hipEventDestroy(b.stall0);
    if (b.stall1) (void)hipEventDestroy(b.stall1);
    if (b.ready_ev) (void)hipEventDestroy(b.ready_ev);
  }
  buckets_ = std::move(out);
  next_bucket_ = 0;
  if (opts_.register_buckets && comm_)
    for (auto& b : buckets_) {
      const int64_t h = comm_->register_buffer(b.wire);
      if (h) reg_handles_.push_back(h);
    }
}

void Reducer::release_registrations() {
  if (comm_)
    for (int64_t h : reg_handles_) comm_->deregister_buffer(h);
  reg_handles_.clear();
}

void Reducer::register_hooks() {
  std::weak_ptr<Reducer> weak = shared_from_this();
  for (size_t i = 0; i < params_.size(); ++i) {
    auto acc = torch::autograd::impl::grad_accumulator(params_[i]);
    DK_CHECK(acc, "Reducer: parameter ", i, " has no grad accumulator (not a leaf?)");
    const int64_t idx = static_cast<int64_t>(i);
    auto handle = acc->add_post_hook(std::make_unique<torch::autograd::utils::LambdaPostHook>(
        [weak, idx](const torch::autograd::variable_list& outputs, const torch::autograd::variable_list&) {
          if (auto self = weak.lock()) self->autograd_hook(idx);
          return outputs;
        }));
    grad_accs_.push_back(std::move(acc));
    hook_handles_.push_back(handle);
  }
}

void Reducer::set_expect_backward(bool v) {
  std::lock_guard<std::mutex> g(mu_);
  expect_hooks_ = v;
}

void Reducer::set_timing(bool on) {
  std::lock_guard<std::mutex> g(mu_);
  timing_ = on && !params_.empty() && params_[0].is_cuda();
  if (!timing_) ev_recorded_ = false;
}

void Reducer::note_used(const std::vector<int64_t>& indices) {
  std::lock_guard<std::mutex> g(mu_);
  for (int64_t i : indices) {
    DK_CHECK(i >= 0 && i < static_cast<int64_t>(params_.size()), "Reducer::note_used: bad parameter index ", i);
    used_since_sync_[i] = 1;
  }
}

void Reducer::prepare_for_backward(const std::vector<at::Tensor>& outputs, bool require_sync) {
  std::lock_guard<std::mutex> g(mu_);
  DK_CHECK(!finalize_queued_, "Reducer: forward called while a backward reduction is still in progress");
  // a deferred bucket's buffer is still being reduced: order the compute
  // stream (which accumulates the next gradients into it) behind it first
  for (auto& b : buckets_) sync_locked(b);
  expect_hooks_ = require_sync;
  if (!require_sync) return;
  unused_list_.clear();
  std::fill(unused_.begin(), unused_.end(), 0);
  if (!opts_.find_unused_parameters) return;
  if (static_frozen_) {
    unused_list_ = static_unused_;
    for (int64_t u : unused_list_) unused_[u] = 1;
  } else {
    find_unused(outputs);
  }
}

void Reducer::find_unused(const std::vector<at::Tensor>& outputs) {
  // Traverse the autograd graph from the outputs; parameters whose
  // AccumulateGrad node is unreachable get no gradient this iteration.
  std::unordered_set<torch::autograd::Node*> seen;
  std::vector<torch::autograd::Node*> stack;
  for (auto& o : outputs) {
    if (!o.defined() || !o.requires_grad()) continue;
    auto fn = o.grad_fn();
    if (fn) {
      if (seen.insert(fn.get()).second) stack.push_back(fn.get());
    } else {
      auto acc = torch::autograd::impl::try_get_grad_accumulator(o);
      if (acc) seen.insert(acc.get());
    }
  }
  while (!stack.empty()) {
    auto* n = stack.back();
    stack.pop_back();
    for (const auto& e : n->next_edges()) {
      auto* nx = e.function.get();
      if (nx && seen.insert(nx).second) stack.push_back(nx);
    }
  }
  for (size_t i = 0; i < params_.size(); ++i) {
    if (!seen.count(grad_accs_[i].get())) {
      unused_[i] = 1;
      unused_list_.push_back(static_cast<int64_t>(i));
    }
  }
}

void Reducer::autograd_hook(int64_t index) {
  std::lock_guard<std::mutex> g(mu_);
  if (!expect_hooks_) {
    // no_sync micro-step: remember the use (torch marks its local_used_map_
    // before the expect-hooks check), so a parameter used only during
    // accumulation still counts as used at the next synced step.
    if (opts_.find_unused_parameters && params_[index].grad().defined()) used_since_sync_[index] = 1;
    return;
  }
  if (!finalize_queued_) {
    finalize_queued_ = true;
    backward_t0_ms_ = static_cast<double>(now_ms());
    bwd_t0_recorded_ = false;
    if (timing_) {
      hipStream_t cur = c10::hip::getCurrentHIPStream(params_[0].device().index()).stream();
      hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(cur, &cap);
      if (cap == hipStreamCaptureStatusNone) {
        if (!bwd_t0_ev_) DK_CHECK(hipEventCreate(&bwd_t0_ev_) == hipSuccess, "Reducer: event creation failed");
        bwd_t0_recorded_ = hipEventRecord(bwd_t0_ev_, cur) == hipSuccess;
      }
    }
    std::weak_ptr<Reducer> weak = shared_from_this();
    torch::autograd::Engine::get_default_engine().queue_callback([weak] {
      if (auto self = weak.lock()) self->finalize();
    });
  }
  if (opts_.find_unused_parameters && !marked_unused_) {
    marked_unused_ = true;
    // Issued before any bucket on every rank: the collective order matches.
    // A frozen static graph already knows the global map.
    if (!static_frozen_) launch_used_map_reduce();
    for (int64_t u : unused_list_) mark_ready(u, /*unused=*/true);
  }
  mark_ready(index, /*unused=*/false);
  launch_ready_buckets();
}

void Reducer::mark_ready(int64_t i, bool unused) {
  DK_CHECK(!ready_[i], "Reducer: parameter ", i,
            " was marked ready twice in one backward (reentrant backward / shared parameters across "
            "checkpointed regions are not supported; or find_unused_parameters misclassified it)");
  ready_[i] = 1;
  if (record_order_) ready_order_.push_back(i);
  auto [bi, s] = where_[i];
  Bucket& b = buckets_[bi];
  const at::Tensor& view = b.views[s];
  const at::Tensor& grad = params_[i].grad();
  // An unused parameter may still hold gradients accumulated under no_sync:
  // they are packed like any other (torch: mark_variable_ready_dense).
  (void)unused;
  if (!grad.defined()) {
    b.pending_grads[s] = at::Tensor();
    view.zero_();
  } else if (grad.data_ptr() == view.data_ptr() && same_layout(grad, view)) {
    b.pending_grads[s] = at::Tensor();  // accumulated in place (gradient_as_bucket_view)
  } else {
    b.pending_grads[s] = grad;
  }
  --b.pending;
}

void Reducer::launch_ready_buckets() {
  while (next_bucket_ < buckets_.size() && buckets_[next_bucket_].pending == 0) {
    launch(buckets_[next_bucket_]);
    ++next_bucket_;
  }
}

namespace {
bool capturing(const at::Tensor& t) {
  if (!t.is_cuda()) return false;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(c10::hip::getCurrentHIPStream(t.device().index()).stream(), &cap);
  return cap != hipStreamCaptureStatusNone;
}
}  // namespace

void Reducer::launch(Bucket& b) {
  sync_locked(b);  // (a deferred previous reduction must land before this pack)
  // Pack: one multi-tensor launch for every gradient not already in place.
  const bool compressed = !b.wire.is_same(b.flat);
  std::vector<at::Tensor> src, dst;
  for (size_t s = 0; s < b.params.size(); ++s) {
    at::Tensor& g = b.pending_grads[s];
    at::Tensor target = compressed
        ? b.wire.as_strided(b.views[s].sizes(), b.views[s].strides(), b.offsets[s])
        : b.views[s];
    const at::Tensor& from = g.defined() ? g : b.views[s];
    if (!g.defined() && !compressed) continue;  // already in the bucket
    if (same_layout(from, target) && from.is_non_overlapping_and_dense() &&
        (from.is_cuda() || from.device().is_cpu())) {
      src.push_back(from);
      dst.push_back(target);
    } else {
      target.copy_(from);
    }
  }
  if (!src.empty()) {
    // mt_copy needs a single src dtype per call; grads match the bucket dtype
    // except under autocast-free mixed setups, which we copy per tensor.
    bool uniform = true;
    for (auto& t : src) uniform = uniform && t.scalar_type() == src[0].scalar_type();
    if (uniform) {
      ops::mt_copy(src, dst, 1.0);
    } else {
      for (size_t k = 0; k < src.size(); ++k) dst[k].copy_(src[k]);
    }
  }
  for (auto& g : b.pending_grads) g = at::Tensor();
  b.stats.ready_ms = static_cast<double>(now_ms()) - backward_t0_ms_;
  b.ready_recorded = false;
  if (timing_ && bwd_t0_recorded_ && b.flat.is_cuda() && !capturing(b.wire)) {
    if (!b.ready_ev) DK_CHECK(hipEventCreate(&b.ready_ev) == hipSuccess, "Reducer: event creation failed");
    b.ready_recorded =
        hipEventRecord(b.ready_ev, c10::hip::getCurrentHIPStream(b.flat.device().index()).stream()) == hipSuccess;
  }
  trace::Range r("dcp.reducer.bucket_allreduce");
  const bool check = check_ && !capturing(b.wire);
  if (check) {
    // packed-buffer checksum (Σx, Σ|x|), taken BEFORE the bucket's collective
    // is issued: that collective reduces b.wire in place (on the comm stream
    // after an event recorded now, or on the host communicator's worker), so
    // a checksum enqueued after it would race with the reduction
    const at::Tensor w = b.wire.to(at::kDouble);
    b.check_sum = at::stack({w.sum(), w.abs().sum()}).to(at::kFloat);
  }
  b.slice_works.clear();
  b.slice_synced.clear();
  if (comm_hook_) {
    b.work = comm_hook_(b.wire, static_cast<int64_t>(&b - buckets_.data()));
  } else if (!b.slice_bounds.empty()) {
    // oversize bucket: one collective per slice, issued back to back (on the
    // communicator's stream in order; the last one's Work stands for all)
    for (size_t s = 0; s + 1 < b.slice_bounds.size(); ++s) {
      at::Tensor piece = b.wire.narrow(0, b.slice_bounds[s], b.slice_bounds[s + 1] - b.slice_bounds[s]);
      b.slice_works.push_back(comm_->all_reduce(piece, opts_.average ? ReduceOp::AVG : ReduceOp::SUM));
    }
    b.slice_synced.assign(b.slice_works.size(), 0);
    b.work = b.slice_works.back();
  } else {
    b.work = comm_->all_reduce(b.wire, opts_.average ? ReduceOp::AVG : ReduceOp::SUM);
  }
  if (check) {
    // reduced by a collective issued right after the bucket's own
    b.check_work = comm_->all_reduce(b.check_sum, opts_.average ? ReduceOp::AVG : ReduceOp::SUM);
  }
  b.launched = true;
}

void Reducer::finalize() {
  std::lock_guard<std::mutex> g(mu_);
  if (!finalize_queued_) return;
  trace::Range range("dcp.reducer.finalize");
  // Every bucket must have been launched: an unready parameter means the
  // model produced no gradient for it and find_unused_parameters was off.
  std::vector<int64_t> missing;
  for (auto& b : buckets_)
    if (!b.launched)
      for (size_t s = 0; s < b.params.size(); ++s)
        if (!ready_[b.params[s]]) missing.push_back(b.params[s]);
  if (!missing.empty()) {
    // Reset every per-iteration field so the next forward/backward starts
    // clean. Collectives already issued for launched buckets stay issued; if
    // peers did not issue the same ones the communicator's watchdog deadline
    // turns the mismatch into an error instead of a hang.
    reset_iteration_state();
    std::string ids;
    for (size_t k = 0; k < missing.size() && k < 16; ++k) ids += (k ? ", " : "") + std::to_string(missing[k]);
    throw Error(str_cat("Reducer: expected to have finished reduction but parameters [", ids,
                        "] received no gradient. Pass find_unused_parameters=True to DistributedDataParallel "
                        "if parts of the model do not take part in the loss."));
  }

  std::vector<char> global_used;
  if (opts_.find_unused_parameters) {
    if (static_frozen_) {
      global_used = static_global_used_;
    } else {
      global_used = collect_global_used();
      if (opts_.static_graph) {
        static_frozen_ = true;
        static_unused_ = unused_list_;
        const bool all = std::all_of(global_used.begin(), global_used.end(), [](char c) { return c != 0; });
        static_global_used_ = all ? std::vector<char>() : global_used;
      }
    }
  }

  hipStream_t cur = nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (timing_) {
    cur = c10::hip::getCurrentHIPStream(params_[0].device().index()).stream();
    (void)hipStreamIsCapturing(cur, &cap);
  }
  // defer_grad_wait: grads are pointed at their bucket views now (host
  // only), the compute-stream waits are left to the consumer (sync_bucket).
  // Not in an iteration that rebuilds the buckets (the buffers are replaced).
  const bool defer = opts_.defer_grad_wait && opts_.gradient_as_bucket_view && global_used.empty() && !check_ &&
                     !(record_order_ && opts_.rebuild_buckets);
  for (auto& b : buckets_) b.stall_recorded = false;
  for (auto& b : buckets_) {
    if (defer) {
      // every .grad becomes its bucket view (host-only pointer swap, as the
      // waiting path below does): the reduced values land there — or what
      // the deferred-grad hook wraps each view in
      if (deferred_grad_hook_) {
        const int64_t k = static_cast<int64_t>(&b - buckets_.data());
        std::vector<at::Tensor> gs = deferred_grad_hook_(k, b.views);
        DK_CHECK(gs.size() == b.params.size(), "Reducer: deferred-grad hook returned ", gs.size(), " tensors for ",
                 b.params.size(), " parameters");
        for (size_t s = 0; s < b.params.size(); ++s) {
          DK_CHECK(gs[s].data_ptr() == b.views[s].data_ptr() && gs[s].sizes() == b.views[s].sizes(),
                   "Reducer: the deferred-grad hook must return the bucket views themselves (wrapped)");
          params_[b.params[s]].mutable_grad() = gs[s];
        }
      } else {
        for (size_t s = 0; s < b.params.size(); ++s) {
          at::Tensor& grad = params_[b.params[s]].mutable_grad();
          if (!grad.defined() || grad.data_ptr() != b.views[s].data_ptr()) grad = b.views[s];
        }
      }
      b.deferred = true;
      b.launched = false;
      b.pending = static_cast<int>(b.params.size());
      continue;
    }
    wait_bucket(b, cur, timing_ && cap == hipStreamCaptureStatusNone);
    // the collective may still be running (wait() only orders the compute
    // stream): keep the Work, bucket_stats() resolves its events when read
    if (timing_ && cap == hipStreamCaptureStatusNone) b.timed_work = b.work;
    if (check_ && b.check_work) {
      b.check_work->wait();
      // what the compute stream sees now vs what the collective must have produced
      const double seen = b.wire.to(at::kDouble).sum().item<double>();
      const at::Tensor cs = b.check_sum.to(at::kDouble).cpu();
      const double want = cs[0].item<double>(), mag = cs[1].item<double>();
      // rounding of the reduction itself: each of the ~world adds of a ring
      // (plus a hook's cast to its wire dtype) rounds by at most half an ulp,
      // eps/2 of the magnitude summed (a near-zero Σx of large terms is not an
      // ordering error) — bf16 wire eps 7.8e-3, fp32 1.2e-7
      const at::ScalarType wdt =
          comm_hook_ && hook_wire_ != at::ScalarType::Undefined ? hook_wire_ : b.wire.scalar_type();
      const double eps = wdt == at::kBFloat16 ? 7.8125e-3 : wdt == at::kHalf ? 9.77e-4 : 1.19e-7;
      const double tol = (comm_->size() + 1) * 0.5 * eps * mag + 1e-6 * std::max(1.0, std::fabs(want)) +
                         1e-6 * static_cast<double>(b.wire.numel());
      b.check_work.reset();
      if (!(std::fabs(seen - want) <= tol)) {
        const int64_t k = static_cast<int64_t>(&b - buckets_.data());
        reset_iteration_state();
        throw Error(str_cat("Reducer stream-ordering check failed for bucket ", k, " (", b.params.size(),
                            " params): the reduced buffer sums to ", seen, " on the compute stream but the "
                            "reduction of the packed buffers sums to ", want,
                            " — a missing event edge between pack, collective and consumer, or a comm hook "
                            "whose work completed before its result was written"));
      }
    }
    if (!b.wire.is_same(b.flat)) ops::mt_copy({b.wire}, {b.flat}, 1.0);
    std::vector<at::Tensor> src, dst;
    for (size_t s = 0; s < b.params.size(); ++s) {
      const int64_t i = b.params[s];
      at::Tensor& grad = params_[i].mutable_grad();
      const bool used = global_used.empty() || global_used[i];
      if (!grad.defined()) {
        if (used) grad = opts_.gradient_as_bucket_view ? b.views[s] : b.views[s].clone();
        continue;
      }
      // Globally unused: keep the existing (e.g. no_sync-accumulated) gradient
      // untouched (torch: copy_bucket_to_grad with global_unused).
      if (!used && grad.data_ptr() != b.views[s].data_ptr()) continue;
      if (opts_.gradient_as_bucket_view) {
        if (grad.data_ptr() != b.views[s].data_ptr()) grad = b.views[s];
      } else if (same_layout(grad, b.views[s])) {
        src.push_back(b.views[s]);
        dst.push_back(grad);
      } else {
        grad.copy_(b.views[s]);
      }
    }
    if (!src.empty()) ops::mt_copy(src, dst, 1.0);
    b.work.reset();
    b.slice_works.clear();
    b.slice_synced.clear();
    b.launched = false;
    b.pending = static_cast<int>(b.params.size());
  }
  std::fill(ready_.begin(), ready_.end(), 0);
  next_bucket_ = 0;
  finalize_queued_ = false;
  marked_unused_ = false;
  expect_hooks_ = false;
  used_work_.reset();
  ++iterations_;
  if (record_order_) {
    record_order_ = false;
    if (opts_.rebuild_buckets) rebuild_from_ready_order();
  }
}

void Reducer::reset_iteration_state() {
  for (auto& b : buckets_) {
    b.work.reset();
    b.slice_works.clear();
    b.slice_synced.clear();
    b.check_work.reset();
    b.launched = false;
    b.pending = static_cast<int>(b.params.size());
    for (auto& g : b.pending_grads) g = at::Tensor();
  }
  std::fill(ready_.begin(), ready_.end(), 0);
  next_bucket_ = 0;
  finalize_queued_ = false;
  marked_unused_ = false;
  expect_hooks_ = false;
  used_work_.reset();
  if (record_order_) ready_order_.clear();
}

void Reducer::launch_used_map_reduce() {
  const int64_t n = static_cast<int64_t>(params_.size());
  const bool cuda = params_[0].is_cuda();
  if (cuda) {
    hipStream_t cur = c10::hip::getCurrentHIPStream(params_[0].device().index()).stream();
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(cur, &cap);
    DK_CHECK(cap == hipStreamCaptureStatusNone,
              "find_unused_parameters=True cannot be used inside HIP-graph capture (the used-parameter map "
              "is read on the host at the end of every backward)");
  }
  if (!used_host_.defined()) {
    auto host = at::TensorOptions().dtype(at::kInt).pinned_memory(cuda);
    used_host_ = at::empty({n}, host);
    used_back_ = at::empty({n}, host);
    used_dev_ = cuda ? at::empty({n}, params_[0].options().dtype(at::kInt).requires_grad(false)) : used_host_;
    if (cuda) DK_CHECK(hipEventCreateWithFlags(&used_ev_, hipEventDisableTiming) == hipSuccess, "event create");
  }
  // The previous iteration's finalize waited for used_ev_, which follows the
  // H2D copy of used_host_: rewriting it now cannot race that copy.
  int32_t* h = used_host_.data_ptr<int32_t>();
  for (int64_t i = 0; i < n; ++i) h[i] = (!unused_[i] || used_since_sync_[i]) ? 1 : 0;
  std::fill(used_since_sync_.begin(), used_since_sync_.end(), 0);
  if (cuda) used_dev_.copy_(used_host_, /*non_blocking=*/true);
  used_work_ = comm_->all_reduce(used_dev_, ReduceOp::MAX);
  if (!cuda) return;
  // Copy the result back on the comm stream (not the compute stream: the
  // backward keeps running) and remember the point to wait for.
  std::optional<c10::hip::HIPStreamGuard> sg;
  if (const int64_t hs = comm_->stream_handle())
    sg.emplace(c10::hip::getStreamFromExternal(reinterpret_cast<hipStream_t>(hs), params_[0].device().index()));
  used_work_->wait();
  used_back_.copy_(used_dev_, /*non_blocking=*/true);
  hipStream_t s = c10::hip::getCurrentHIPStream(params_[0].device().index()).stream();
  DK_CHECK(hipEventRecord(used_ev_, s) == hipSuccess, "event record");
}

std::vector<char> Reducer::collect_global_used() {
  const size_t n = params_.size();
  std::vector<char> out(n, 1);
  if (!used_work_) launch_used_map_reduce();  // no hook fired (nothing used locally)
  if (params_[0].is_cuda()) {
    // Poll (not hipEventSynchronize) so a communicator abort releases us.
    while (true) {
      if (!comm_->error().empty()) throw Error("Reducer: communicator failed: " + comm_->error());
      hipError_t e = hipEventQuery(used_ev_);
      if (e == hipSuccess) break;
      DK_CHECK(e == hipErrorNotReady, "hipEventQuery failed: ", hipGetErrorString(e));
      std::this_thread::sleep_for(std::chrono::microseconds(10));
    }
    const int32_t* h = used_back_.data_ptr<int32_t>();
    for (size_t i = 0; i < n; ++i) out[i] = h[i] != 0;
  } else {
    used_work_->wait();
    const int32_t* h = used_dev_.data_ptr<int32_t>();
    for (size_t i = 0; i < n; ++i) out[i] = h[i] != 0;
  }
  return out;
}

void Reducer::rebuild_from_ready_order() {
  // Complete the observed order with parameters that produced no gradient.
  std::vector<int64_t> order = ready_order_;
  std::vector<char> in(params_.size(), 0);
  for (int64_t i : order) in[i] = 1;
  for (int64_t i = static_cast<int64_t>(params_.size()) - 1; i >= 0; --i)
    if (!in[i]) order.push_back(i);
  // Adopt rank 0's order everywhere: different orders would mismatch the
  // collective sequence across ranks and hang RCCL.
  at::Tensor t = at::from_blob(order.data(), {static_cast<int64_t>(order.size())}, at::kLong).clone();
  at::Tensor dev = t.to(params_[0].device());
  auto w = comm_->broadcast(dev, 0);
  w->wait();
  w->synchronize();
  at::Tensor back = dev.cpu().contiguous();
  std::memcpy(order.data(), back.data_ptr<int64_t>(), order.size() * sizeof(int64_t));

  std::vector<int64_t> sizes, keys;
  for (auto& p : params_) {
    sizes.push_back(p.numel() * p.element_size());
    keys.push_back(bucket_key(p));
  }
  auto assignment = split_tail_bucket(
      compute_bucket_assignment(sizes, keys, {opts_.first_bucket_bytes, opts_.bucket_bytes_cap}, order), sizes,
      opts_.tail_bucket_bytes);
  if (assignment == bucket_indices()) return;
  // Keep current gradients (bucket views in gradient_as_bucket_view mode).
  std::vector<at::Tensor> old_grads(params_.size());
  for (size_t i = 0; i < params_.size(); ++i) old_grads[i] = params_[i].grad();
  build_buckets(assignment);
  if (opts_.gradient_as_bucket_view) {
    for (size_t i = 0; i < params_.size(); ++i) {
      if (!old_grads[i].defined()) continue;
      auto [bi, s] = where_[i];
      buckets_[bi].views[s].copy_(old_grads[i]);
      params_[i].mutable_grad() = buckets_[bi].views[s];
    }
  }
  ++rebuilds_;
}

void Reducer::wait_all() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& b : buckets_) {
    sync_locked(b);
    if (b.work) b.work->synchronize();
  }
}

std::vector<std::vector<int64_t>> Reducer::bucket_indices() const {
  std::vector<std::vector<int64_t>> r;
  for (auto& b : buckets_) r.push_back(b.params);
  return r;
}

std::vector<int64_t> Reducer::bucket_sizes_bytes() const {
  std::vector<int64_t> r;
  for (auto& b : buckets_) r.push_back(b.stats.bytes);
  return r;
}

std::vector<BucketStats> Reducer::bucket_stats() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<BucketStats> r;
  for (auto& b : buckets_) {
    if (b.timed_work) {
      b.timed_work->synchronize();
      b.stats.comm_ms = b.timed_work->elapsed_ms();
      b.timed_work.reset();
    }
    if (b.ready_recorded && bwd_t0_ev_) {
      float ms = 0.f;
      (void)hipEventSynchronize(b.ready_ev);
      if (hipEventElapsedTime(&ms, bwd_t0_ev_, b.ready_ev) == hipSuccess) b.stats.ready_dev_ms = ms;
      b.ready_recorded = false;
    }
    r.push_back(b.stats);
  }
  return r;
}

std::vector<at::Tensor> Reducer::bucket_buffers() const {
  std::vector<at::Tensor> r;
  for (auto& b : buckets_) r.push_back(b.flat);
  return r;
}

}  // namespace dcp
