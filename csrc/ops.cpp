#include "ops.h"

#include <ATen/Dispatch.h>
#include <ATen/Parallel.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <cmath>
#include <list>
#include <map>
#include <mutex>

#include "common.h"
#include "kernels/kernels.h"

namespace dcp {
namespace ops {

namespace {

kern::DType kdtype(at::ScalarType st) {
  switch (st) {
    case at::kFloat: return kern::F32;
    case at::kBFloat16: return kern::BF16;
    case at::kHalf: return kern::F16;
    default: throw Error(str_cat("multi-tensor kernels: unsupported dtype ", c10::toString(st)));
  }
}

// ---- device table cache --------------------------------------------------
struct TableEntry {
  std::vector<int64_t> key;
  uint64_t hash = 0;        // of key: the lookup compares this first
  at::Tensor dev;
  int n;
  int64_t nchunks;
  at::Tensor host;          // pinned source of the upload (undefined for capture-time entries)
  bool persistent = false;  // read by a captured kernel on every replay: never evicted
};

std::mutex g_cache_mu;
std::list<TableEntry> g_cache;  // MRU at front
// Large enough for every distinct table of a training step: a BERT step runs
// ~60 multi-tensor launches (optimizer chunks, bucket packs); at 32 entries the
// LRU thrashed on that cycle and every launch re-uploaded its table (~110
// pinned H2D copies per step, 0.45 ms of copy kernels on the compute queue).
constexpr size_t kCacheCap = 1024;

uint64_t words_hash(const std::vector<int64_t>& w) {
  uint64_t h = 1469598103934665603ull;
  for (int64_t v : w) {
    h ^= static_cast<uint64_t>(v);
    h *= 1099511628211ull;
    h ^= h >> 29;
  }
  return h;
}
// Evicted pinned upload buffers wait here until the copy that read them has
// finished (raw hipMemcpyAsync: the torch host allocator does not track it).
std::vector<std::pair<hipEvent_t, at::Tensor>> g_graveyard;

void reap_graveyard() {
  for (auto it = g_graveyard.begin(); it != g_graveyard.end();) {
    if (hipEventQuery(it->first) == hipSuccess) {
      (void)hipEventDestroy(it->first);
      it = g_graveyard.erase(it);
    } else {
      ++it;
    }
  }
}

// lists[d][i]: tensor i of list d. All lists must have the same length; rows
// (same i) must have identical numel. Empty tensors are skipped.
TableEntry get_table(const std::vector<const TensorList*>& lists) {
  const size_t depth = lists.size();
  const size_t n_all = lists[0]->size();
  std::vector<size_t> keep;
  keep.reserve(n_all);
  for (size_t i = 0; i < n_all; ++i)
    if ((*lists[0])[i].numel() > 0) keep.push_back(i);
  const int n = static_cast<int>(keep.size());
  std::vector<int64_t> words;
  words.reserve((n + 1) + n + depth * n);
  int64_t chunks = 0;
  for (int k = 0; k < n; ++k) {
    words.push_back(chunks);
    chunks += ((*lists[0])[keep[k]].numel() + kern::kChunk - 1) / kern::kChunk;
  }
  words.push_back(chunks);
  for (int k = 0; k < n; ++k) words.push_back((*lists[0])[keep[k]].numel());
  for (size_t d = 0; d < depth; ++d)
    for (int k = 0; k < n; ++k)
      words.push_back(reinterpret_cast<int64_t>((*lists[d])[keep[k]].data_ptr()));

  std::lock_guard<std::mutex> g(g_cache_mu);
  const auto dev = (*lists[0])[keep.empty() ? 0 : keep[0]].device();
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const hipStream_t st = c10::hip::getCurrentHIPStream(dev.index()).stream();
  (void)hipStreamIsCapturing(st, &cap);
  const bool capturing = cap == hipStreamCaptureStatusActive;
  const uint64_t h = words_hash(words);
  for (auto it = g_cache.begin(); it != g_cache.end(); ++it) {
    if (it->hash == h && it->key == words) {
      // a captured kernel now reads this device table on every replay: it must
      // never be evicted (eviction frees it to the caching allocator, and a
      // later replay would read whatever reused the memory)
      if (capturing) it->persistent = true;
      g_cache.splice(g_cache.begin(), g_cache, it);
      return g_cache.front();
    }
  }
  at::Tensor host;
  at::Tensor d = at::empty({static_cast<int64_t>(words.size())}, at::TensorOptions().dtype(at::kLong).device(dev));
  if (capturing) {
    // copy kernels carrying the words as arguments (stored in the graph): a
    // captured memcpy node is not reliably ordered before the kernel reading
    // the table on replays (the defect behind fused.cpp zeroed_floats)
    kern::copy_words(words.data(), d.data_ptr<int64_t>(), static_cast<int64_t>(words.size()), st);
  } else {
    host = at::empty({static_cast<int64_t>(words.size())}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
    std::memcpy(host.data_ptr(), words.data(), words.size() * sizeof(int64_t));
    DK_CHECK(hipMemcpyAsync(d.data_ptr(), host.data_ptr(), words.size() * sizeof(int64_t), hipMemcpyHostToDevice,
                             st) == hipSuccess,
              "table upload failed");
  }
  TableEntry e{std::move(words), h, d, n, chunks, host, capturing};
  g_cache.push_front(std::move(e));
  // evict the least recently used non-persistent entry (never while capturing:
  // the deferred-free event would itself be captured)
  if (!capturing) {
    reap_graveyard();
    if (g_cache.size() > kCacheCap) {
      for (auto it = std::prev(g_cache.end());; --it) {
        if (!it->persistent) {
          hipEvent_t ev;
          if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess &&
              hipEventRecord(ev, st) == hipSuccess) {
            g_graveyard.emplace_back(ev, it->host);
          }
          g_cache.erase(it);
          break;
        }
        if (it == g_cache.begin()) break;
      }
    }
  }
  return g_cache.front();
}

void check_lists(const std::vector<const TensorList*>& lists, const char* what) {
  const size_t n = lists[0]->size();
  for (auto* l : lists) DK_CHECK(l->size() == n, what, ": tensor lists differ in length");
  for (size_t i = 0; i < n; ++i) {
    const at::Tensor& ref = (*lists[0])[i];
    DK_CHECK(ref.is_non_overlapping_and_dense(), what, ": tensor ", i, " is not dense");
    for (auto* l : lists) {
      const at::Tensor& t = (*l)[i];
      DK_CHECK(t.numel() == ref.numel(), what, ": numel mismatch at ", i);
      DK_CHECK(t.device() == ref.device(), what, ": device mismatch at ", i);
      DK_CHECK(t.strides() == ref.strides() || t.is_contiguous() && ref.is_contiguous(), what,
                ": stride mismatch at ", i, " (memory formats must agree)");
    }
  }
}

bool on_gpu(const TensorList& l) { return !l.empty() && l[0].is_cuda(); }

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

// CPU helper: apply f(i, n, ptrs...) over each row.
template <typename scalar_t>
scalar_t* P(const at::Tensor& t) {
  return static_cast<scalar_t*>(t.data_ptr());
}

}  // namespace

int64_t table_cache_size() {
  std::lock_guard<std::mutex> g(g_cache_mu);
  return static_cast<int64_t>(g_cache.size());
}

// ------------------------------------------------------------------ copy ---
void mt_copy(const TensorList& src, const TensorList& dst, double scale) {
  if (src.empty()) return;
  check_lists({&src, &dst}, "mt_copy");
  if (on_gpu(src)) {
    // One launch per (src dtype, dst dtype) class; buckets are single-dtype.
    const auto sd = src[0].scalar_type(), dd = dst[0].scalar_type();
    for (size_t i = 0; i < src.size(); ++i)
      DK_CHECK(src[i].scalar_type() == sd && dst[i].scalar_type() == dd, "mt_copy: mixed dtypes in one call");
    c10::hip::HIPGuard guard(src[0].device().index());
    auto tab = get_table({&src, &dst});
    kern::mt_copy(kern::TableView{tab.dev.data_ptr<int64_t>(), tab.n}, tab.nchunks, kdtype(sd), kdtype(dd),
                  static_cast<float>(scale), cur_stream(src[0]));
    return;
  }
  for (size_t i = 0; i < src.size(); ++i) {
    if (scale == 1.0) {
      // raw memory-order copy (layouts agree)
      dst[i].as_strided({dst[i].numel()}, {1}).copy_(src[i].as_strided({src[i].numel()}, {1}));
    } else {
      dst[i].as_strided({dst[i].numel()}, {1}).copy_(src[i].as_strided({src[i].numel()}, {1}).mul(scale));
    }
  }
}

// ------------------------------------------------------------------- SGD ---
void fused_sgd(const TensorList& params, const TensorList& grads, const TensorList& bufs, double lr,
               double momentum, double dampening, double weight_decay, bool nesterov, bool maximize,
               bool first_step, double grad_scale) {
  if (params.empty()) return;
  const bool has_buf = momentum != 0.0;
  std::vector<const TensorList*> lists{&params, &grads};
  if (has_buf) lists.push_back(&bufs);
  check_lists(lists, "fused_sgd");
  if (on_gpu(params)) {
    c10::hip::HIPGuard guard(params[0].device().index());
    auto tab = get_table(lists);
    kern::mt_sgd(kern::TableView{tab.dev.data_ptr<int64_t>(), tab.n}, tab.nchunks, kdtype(params[0].scalar_type()),
                 static_cast<float>(lr), static_cast<float>(momentum), static_cast<float>(dampening),
                 static_cast<float>(weight_decay), nesterov, maximize, first_step, has_buf,
                 static_cast<float>(grad_scale), cur_stream(params[0]));
    return;
  }
  for (size_t t = 0; t < params.size(); ++t) {
    AT_DISPATCH_FLOATING_TYPES_AND2(at::kBFloat16, at::kHalf, params[t].scalar_type(), "cpu_sgd", [&] {
      scalar_t* p = P<scalar_t>(params[t]);
      const scalar_t* g = P<scalar_t>(grads[t]);
      scalar_t* b = has_buf ? P<scalar_t>(bufs[t]) : nullptr;
      at::parallel_for(0, params[t].numel(), 16384, [&](int64_t s, int64_t e) {
        for (int64_t i = s; i < e; ++i) {
          float pv = static_cast<float>(p[i]);
          float gv = static_cast<float>(g[i]) * static_cast<float>(grad_scale);
          if (maximize) gv = -gv;
          if (weight_decay != 0.0) gv = gv + static_cast<float>(weight_decay) * pv;
          if (has_buf) {
            float bv = first_step ? gv
                                  : static_cast<float>(momentum) * static_cast<float>(b[i]) +
                                        (1.f - static_cast<float>(dampening)) * gv;
            b[i] = static_cast<scalar_t>(bv);
            gv = nesterov ? gv + static_cast<float>(momentum) * bv : bv;
          }
          p[i] = static_cast<scalar_t>(pv - static_cast<float>(lr) * gv);
        }
      });
    });
  }
}

// ------------------------------------------------------------------ Adam ---
void fused_adam(const TensorList& params, const TensorList& grads, const TensorList& exp_avgs,
                const TensorList& exp_avg_sqs, const TensorList& max_exp_avg_sqs, double lr, double beta1,
                double beta2, double eps, double weight_decay, double step, bool amsgrad, bool decoupled,
                bool maximize, double grad_scale, const TensorList& shadows, const TensorList& steps) {
  if (params.empty()) return;
  std::vector<const TensorList*> lists{&params, &grads, &exp_avgs, &exp_avg_sqs};
  if (amsgrad) lists.push_back(&max_exp_avg_sqs);
  // shadows: optional bf16 copies of fp32 params, rewritten with the updated values
  const bool shadow = !shadows.empty();
  if (shadow) {
    lists.push_back(&shadows);
    for (size_t i = 0; i < shadows.size(); ++i)
      DK_CHECK(shadows[i].scalar_type() == at::kBFloat16 && params[i].scalar_type() == at::kFloat &&
                    shadows[i].is_contiguous() && params[i].is_contiguous(),
                "fused_adam: shadows must be contiguous bf16 copies of contiguous fp32 params");
  }
  check_lists(lists, "fused_adam");
  // capturable mode: one device fp32 step scalar per tensor (already
  // incremented by the caller), appended as an extra table list (the table
  // sizes chunks by list 0 only, so 1-element rows are fine there)
  int step_list = -1;
  if (!steps.empty()) {
    DK_CHECK(steps.size() == params.size() && on_gpu(params), "fused_adam: steps must be one device tensor per param");
    for (auto& t : steps)
      DK_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.numel() == 1 && t.device() == params[0].device(),
                "fused_adam: each step must be a 1-element fp32 tensor on the parameters' device");
    step_list = static_cast<int>(lists.size());
    lists.push_back(&steps);
  }
  const double bc1 = 1.0 - std::pow(beta1, step);
  const double bc2_sqrt = std::sqrt(1.0 - std::pow(beta2, step));
  if (on_gpu(params)) {
    c10::hip::HIPGuard guard(params[0].device().index());
    auto tab = get_table(lists);
    kern::mt_adam(kern::TableView{tab.dev.data_ptr<int64_t>(), tab.n}, tab.nchunks, kdtype(params[0].scalar_type()),
                  static_cast<float>(lr), static_cast<float>(beta1), static_cast<float>(beta2),
                  static_cast<float>(eps), static_cast<float>(weight_decay), static_cast<float>(bc1),
                  static_cast<float>(bc2_sqrt), amsgrad, decoupled, maximize, static_cast<float>(grad_scale),
                  shadow, step_list, cur_stream(params[0]));
    return;
  }
  for (size_t t = 0; t < params.size(); ++t) {
    AT_DISPATCH_FLOATING_TYPES_AND2(at::kBFloat16, at::kHalf, params[t].scalar_type(), "cpu_adam", [&] {
      scalar_t* p = P<scalar_t>(params[t]);
      const scalar_t* g = P<scalar_t>(grads[t]);
      scalar_t* m = P<scalar_t>(exp_avgs[t]);
      scalar_t* v = P<scalar_t>(exp_avg_sqs[t]);
      scalar_t* vm = amsgrad ? P<scalar_t>(max_exp_avg_sqs[t]) : nullptr;
      const float flr = static_cast<float>(lr), b1 = static_cast<float>(beta1), b2 = static_cast<float>(beta2);
      const float feps = static_cast<float>(eps), wd = static_cast<float>(weight_decay);
      at::parallel_for(0, params[t].numel(), 16384, [&](int64_t s, int64_t e) {
        for (int64_t i = s; i < e; ++i) {
          float pv = static_cast<float>(p[i]);
          float gv = static_cast<float>(g[i]) * static_cast<float>(grad_scale);
          if (maximize) gv = -gv;
          if (wd != 0.f) {
            if (decoupled) pv *= (1.f - flr * wd);
            else gv += wd * pv;
          }
          float mv = static_cast<float>(m[i]);
          float vv = static_cast<float>(v[i]);
          mv = mv + (1.f - b1) * (gv - mv);
          vv = b2 * vv + (1.f - b2) * gv * gv;
          float denom;
          if (amsgrad) {
            float mx = std::max(static_cast<float>(vm[i]), vv);
            vm[i] = static_cast<scalar_t>(mx);
            denom = std::sqrt(mx) / static_cast<float>(bc2_sqrt) + feps;
          } else {
            denom = std::sqrt(vv) / static_cast<float>(bc2_sqrt) + feps;
          }
          pv -= (flr / static_cast<float>(bc1)) * (mv / denom);
          p[i] = static_cast<scalar_t>(pv);
          m[i] = static_cast<scalar_t>(mv);
          v[i] = static_cast<scalar_t>(vv);
        }
      });
    });
  }
  for (size_t t = 0; t < shadows.size(); ++t) shadows[t].copy_(params[t]);
}

// -------------------------------------------------------------- Adadelta ---
void fused_adadelta(const TensorList& params, const TensorList& grads, const TensorList& square_avgs,
                    const TensorList& acc_deltas, double lr, double rho, double eps, double weight_decay,
                    bool maximize, double grad_scale) {
  if (params.empty()) return;
  std::vector<const TensorList*> lists{&params, &grads, &square_avgs, &acc_deltas};
  check_lists(lists, "fused_adadelta");
  if (on_gpu(params)) {
    c10::hip::HIPGuard guard(params[0].device().index());
    auto tab = get_table(lists);
    kern::mt_adadelta(kern::TableView{tab.dev.data_ptr<int64_t>(), tab.n}, tab.nchunks,
                      kdtype(params[0].scalar_type()), static_cast<float>(lr), static_cast<float>(rho),
                      static_cast<float>(eps), static_cast<float>(weight_decay), maximize,
                      static_cast<float>(grad_scale), cur_stream(params[0]));
    return;
  }
  for (size_t t = 0; t < params.size(); ++t) {
    AT_DISPATCH_FLOATING_TYPES_AND2(at::kBFloat16, at::kHalf, params[t].scalar_type(), "cpu_adadelta", [&] {
      scalar_t* p = P<scalar_t>(params[t]);
      const scalar_t* g = P<scalar_t>(grads[t]);
      scalar_t* sq = P<scalar_t>(square_avgs[t]);
      scalar_t* ac = P<scalar_t>(acc_deltas[t]);
      const float r = static_cast<float>(rho), e = static_cast<float>(eps);
      at::parallel_for(0, params[t].numel(), 16384, [&](int64_t s, int64_t en) {
        for (int64_t i = s; i < en; ++i) {
          float pv = static_cast<float>(p[i]);
          float gv = static_cast<float>(g[i]) * static_cast<float>(grad_scale);
          if (maximize) gv = -gv;
          if (weight_decay != 0.0) gv += static_cast<float>(weight_decay) * pv;
          float s2 = r * static_cast<float>(sq[i]) + (1.f - r) * gv * gv;
          float stdv = std::sqrt(s2 + e);
          float delta = std::sqrt(static_cast<float>(ac[i]) + e) / stdv * gv;
          float a2 = r * static_cast<float>(ac[i]) + (1.f - r) * delta * delta;
          sq[i] = static_cast<scalar_t>(s2);
          ac[i] = static_cast<scalar_t>(a2);
          p[i] = static_cast<scalar_t>(pv - static_cast<float>(lr) * delta);
        }
      });
    });
  }
}

// ------------------------------------------------------------- grad norm ---
at::Tensor sumsq(const TensorList& tensors) {
  DK_CHECK(!tensors.empty(), "sumsq: empty list");
  if (on_gpu(tensors)) {
    c10::hip::HIPGuard guard(tensors[0].device().index());
    at::Tensor out = at::zeros({2}, at::TensorOptions().dtype(at::kFloat).device(tensors[0].device()));
    // group by dtype
    std::map<at::ScalarType, TensorList> by;
    for (auto& t : tensors) {
      DK_CHECK(t.is_non_overlapping_and_dense(), "sumsq: dense tensors required");
      by[t.scalar_type()].push_back(t);
    }
    for (auto& kv : by) {
      auto tab = get_table({&kv.second});
      kern::mt_sumsq(kern::TableView{tab.dev.data_ptr<int64_t>(), tab.n}, tab.nchunks, kdtype(kv.first),
                     out.data_ptr<float>(), cur_stream(tensors[0]));
    }
    return out;
  }
  double acc = 0.0;
  bool bad = false;
  for (auto& t : tensors) {
    at::Tensor f = t.to(at::kDouble);
    acc += f.pow(2).sum().item<double>();
    bad = bad || !f.isfinite().all().item<bool>();
  }
  at::Tensor out = at::zeros({2}, at::kFloat);
  out[0] = acc;
  out[1] = bad ? 1.0 : 0.0;
  return out;
}

void scale_by(const TensorList& tensors, const at::Tensor& scale) {
  if (tensors.empty()) return;
  if (on_gpu(tensors)) {
    c10::hip::HIPGuard guard(tensors[0].device().index());
    DK_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat, "scale_by: scale must be fp32 on device");
    std::map<at::ScalarType, TensorList> by;
    for (auto& t : tensors) by[t.scalar_type()].push_back(t);
    for (auto& kv : by) {
      auto tab = get_table({&kv.second});
      kern::mt_scale_by(kern::TableView{tab.dev.data_ptr<int64_t>(), tab.n}, tab.nchunks, kdtype(kv.first),
                        scale.data_ptr<float>(), cur_stream(tensors[0]));
    }
    return;
  }
  for (auto& t : tensors) t.mul_(scale.to(t.device()).to(t.scalar_type()));
}

}  // namespace ops
}  // namespace dcp
