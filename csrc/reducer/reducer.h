// Gradient Reducer: bucketing, autograd-hook driven launch of bucket
// all-reduces overlapped with backward, finalize, ready-order rebuild.
//
// Parity: torch's C++ Reducer that the reference gets from
// DistributedDataParallel(model, device_ids=[rank]) (main.py:122, SURVEY §2b
// F6/F7, §3.3). The semantics kept: per-parameter post-accumulate hooks, in-
// order bucket launch while backward continues, finalize at the end of
// backward, gradients averaged over the world, `no_sync`, find_unused_
// parameters, gradient_as_bucket_view, bucket rebuild from the observed
// gradient-ready order (rank 0's order adopted everywhere).
//
// MI355X design: one flat buffer per bucket; pack/unpack are ONE multi-tensor
// HIP launch per bucket (csrc/kernels/multi_tensor.hip) instead of a copy per
// parameter; averaging is folded into RCCL (ncclAvg) so there is no separate
// scale pass; optional bf16 wire compression packs fp32 grads straight into a
// bf16 comm buffer in the same launch.
#pragma once

#include <ATen/ATen.h>
#include <hip/hip_runtime.h>
#include <torch/csrc/autograd/function.h>

#include <functional>
#include <memory>
#include <mutex>
#include <vector>

#include "../comm/communicator.h"

namespace dcp {

// torch-compatible bucket planner (semantics of
// torch.distributed._compute_bucket_assignment_by_size): greedy packing per
// (dtype, device) key under the limit list; `order` empty = natural order and
// buckets sorted by min index, else tensors visited in `order` and buckets kept
// in that order.
std::vector<std::vector<int64_t>> compute_bucket_assignment(const std::vector<int64_t>& sizes_bytes,
                                                            const std::vector<int64_t>& keys,
                                                            const std::vector<int64_t>& limits,
                                                            const std::vector<int64_t>& order);

// xGMI tail bucket: split the LAST bucket of a launch-ordered plan so that
// its final part (the parameters whose gradients are ready last, i.e. the
// suffix of the bucket's ready-ordered list) holds at most `tail_bytes`
// (always >= 1 parameter). The last bucket's all-reduce cannot overlap any
// backward compute, so its size is the exposed communication (NOTES §18).
// No-op when tail_bytes <= 0 or the last bucket already fits.
std::vector<std::vector<int64_t>> split_tail_bucket(std::vector<std::vector<int64_t>> assignment,
                                                    const std::vector<int64_t>& sizes_bytes, int64_t tail_bytes);

struct ReducerOptions {
  bool gradient_as_bucket_view = false;
  bool find_unused_parameters = false;
  bool rebuild_buckets = true;
  int64_t first_bucket_bytes = 1 << 20;
  int64_t bucket_bytes_cap = 25 << 20;
  int64_t tail_bucket_bytes = 0;  // see split_tail_bucket; 0 = torch behaviour
  // at::ScalarType of the wire buffer; Undefined = same as the gradient.
  at::ScalarType comm_dtype = at::ScalarType::Undefined;
  // false -> SUM instead of AVG (for custom hooks that pre-scale).
  bool average = true;
  // register every bucket's wire buffer with the communicator (RCCL
  // ncclCommRegister) for the Reducer's lifetime; released on a rebuild
  bool register_buckets = false;
  // Debug (SURVEY §5.2 "stream-ordering asserts"; also DCP_DEBUG_STREAMS=1):
  // per bucket, a checksum of the packed wire buffer taken on the compute
  // stream right after the pack, all-reduced over the world, must equal the
  // checksum of the buffer the compute stream sees after waiting on the
  // reduction. A missing pack→collective or collective→consumer event edge
  // (or a comm hook that returns before its result is in the buffer) shows up
  // as a mismatch, raised from finalize. Host-syncs once per bucket: debug only.
  bool check_streams = false;
  // Optimizer overlap (gradient_as_bucket_view, no find_unused_parameters):
  // finalize points every .grad at its bucket view but does NOT order the
  // compute stream behind the bucket collectives; the consumer (the fused
  // optimizers, optim/fused.py) calls sync_bucket(k) in launch order right
  // before it updates bucket k's parameters, so the update of the early
  // buckets runs while the last ones are still being reduced. Anything
  // still deferred is synced before the next backward's first pack, by
  // prepare_for_backward and by wait_gradients().
  bool defer_grad_wait = false;
  // Oversize buckets (defer_grad_wait): a bucket of more than 1.5x this many
  // bytes is reduced as ceil(bytes / slice_bytes) collectives over 256-B
  // aligned slices of its buffer, each with its own Work, so a consumer can
  // update the parameter ranges of a slice as soon as that slice lands
  // (sync_bucket_slice) — the ready-last tied embeddings of GPT-2 / BERT are
  // single 147 / 89 MB buckets. 0 = one collective per bucket (torch).
  int64_t slice_bytes = 0;
  // torch's static_graph: the set of parameters that get no gradient is the
  // same every iteration. The first synchronised backward traverses the graph
  // and all-reduces the used map (as find_unused_parameters does); later ones
  // reuse both results — no traversal, no used-map collective, and capturable
  // in a HIP graph. Implies find_unused_parameters semantics.
  bool static_graph = false;
};

struct BucketStats {
  int64_t bytes = 0;
  int64_t num_params = 0;
  double ready_ms = 0;   // host time since backward start when the bucket became ready
  // device time (DCP_COMM_TIMING=1, GPU): from the backward's first gradient
  // hook to the completion of the bucket's pack on the compute stream — when
  // its gradients really exist, which is what overlap depends on (-1: none)
  double ready_dev_ms = -1;
  double comm_ms = -1;   // device time of its collective (when timing enabled)
};

class Reducer : public std::enable_shared_from_this<Reducer> {
 public:
  // (bucket buffer, position of the bucket in this iteration's launch order)
  using CommHook = std::function<WorkPtr(at::Tensor& bucket, int64_t index)>;
  // defer_grad_wait: what a deferred bucket's parameters get as .grad — given
  // the bucket index and its gradient views, the tensors to install (the DDP
  // wrapper hands out views that order every reader behind the reduction:
  // parallel/ddp.py _PendingGrad). Unset: the plain views.
  using DeferredGradHook = std::function<std::vector<at::Tensor>(int64_t index, const std::vector<at::Tensor>& views)>;

  Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
          std::shared_ptr<Communicator> comm, ReducerOptions opts);
  ~Reducer();

  // Must be called once after construction (hooks capture a weak_ptr).
  void register_hooks();

  // Called from DDP forward: expect hooks in the next backward iff require_sync.
  void prepare_for_backward(const std::vector<at::Tensor>& outputs, bool require_sync);
  // Called when a forward ran without a following backward being expected.
  void set_expect_backward(bool v);
  // find_unused_parameters: these parameters got gradient contributions
  // outside a hook this iteration (deferred no_sync segments added into .grad
  // by the DDP wrapper): they count as used, like a no_sync hook would mark them.
  void note_used(const std::vector<int64_t>& indices);

  // Custom comm hook (runs on the autograd thread with the bucket buffer).
  // wire_dtype: the precision the hook's collective carries (a compression
  // hook declares bf16 / fp16; Undefined = the bucket's own dtype) — it sets
  // the rounding the debug stream-ordering check tolerates
  void set_deferred_grad_hook(DeferredGradHook hook) { deferred_grad_hook_ = std::move(hook); }
  void set_comm_hook(CommHook hook, at::ScalarType wire_dtype = at::ScalarType::Undefined) {
    comm_hook_ = std::move(hook);
    hook_wire_ = wire_dtype;
  }

  std::vector<std::vector<int64_t>> bucket_indices() const;
  std::vector<int64_t> bucket_sizes_bytes() const;
  std::vector<BucketStats> bucket_stats();
  // DCP_COMM_TIMING=1 on a GPU: communication NOT hidden behind compute in
  // the last finished iteration = the device time the compute stream stood
  // at its waits on the bucket collectives (summed over buckets; with
  // defer_grad_wait the waits sit between the optimizer's per-bucket
  // updates). -1 when unavailable (timing off, CPU, still in flight).
  double exposed_comm_ms();
  // turn the DCP_COMM_TIMING instrumentation on / off from the next backward
  // (GPU only): e.g. a few diagnostic steps after an untimed-instrumentation
  // benchmark region
  void set_timing(bool on);
  std::vector<int64_t> ready_order() const { return ready_order_; }
  int64_t num_iterations() const { return iterations_; }
  int64_t num_rebuilds() const { return rebuilds_; }
  bool static_frozen() const { return static_frozen_; }
  std::vector<int64_t> static_unused() const { return static_unused_; }
  bool has_rebuilt() const { return rebuilds_ > 0; }
  // Bucket buffers (tests / optimizers that work on flat buffers).
  std::vector<at::Tensor> bucket_buffers() const;
  // Wait for in-flight reductions (used by no_sync exit / destructor paths).
  void wait_all();
  // defer_grad_wait: bucket indices (launch order) whose collective the
  // compute stream has not been ordered behind yet; sync_bucket orders it
  // (and unpacks a compressed wire buffer); sync_all syncs every one.
  std::vector<int64_t> deferred_buckets();
  void sync_bucket(int64_t k);
  void sync_all();
  // slice_bytes: element bounds [0, e1, …, numel] of deferred bucket k's
  // slices when its reduction was issued slice by slice (else empty), and
  // the per-slice sync (slices synced in any order; the bucket stops being
  // deferred once all are)
  std::vector<int64_t> bucket_slice_bounds(int64_t k);
  void sync_bucket_slice(int64_t k, int64_t s);

 private:
  struct Bucket {
    std::vector<int64_t> params;
    std::vector<int64_t> offsets;
    at::Tensor flat;                  // gradient dtype
    at::Tensor wire;                  // == flat, or compressed copy
    std::vector<at::Tensor> views;    // as_strided views matching param layouts
    std::vector<at::Tensor> pending_grads;  // copy mode: grads to pack at launch
    int pending = 0;
    bool launched = false;
    WorkPtr work;
    std::vector<int64_t> slice_bounds;  // slice_bytes: element bounds of the slices (empty: not sliced)
    std::vector<WorkPtr> slice_works;   // this iteration's per-slice collectives (sliced launch)
    std::vector<char> slice_synced;     // deferred: slices the compute stream is ordered behind
    WorkPtr timed_work;  // last finished collective, its elapsed time read lazily (bucket_stats)
    BucketStats stats;
    at::Tensor check_sum;  // check_streams: fp64 [1] checksum of the packed buffer (all-reduced)
    WorkPtr check_work;
    bool deferred = false;  // defer_grad_wait: work kept, compute stream not yet ordered behind it
    hipEvent_t stall0 = nullptr, stall1 = nullptr;  // timing: compute-stream wait on this bucket
    hipEvent_t ready_ev = nullptr;                    // timing: after the bucket's pack (compute stream)
    bool ready_recorded = false;
    bool stall_recorded = false;
  };

  void build_buckets(const std::vector<std::vector<int64_t>>& assignment);
  void autograd_hook(int64_t index);
  void mark_ready(int64_t index, bool unused);
  void launch_ready_buckets();
  void launch(Bucket& b);
  void finalize();
  void rebuild_from_ready_order();
  void find_unused(const std::vector<at::Tensor>& outputs);
  void launch_used_map_reduce();
  std::vector<char> collect_global_used();
  void reset_iteration_state();
  // compute stream waits on b's collective (timed when DCP_COMM_TIMING)
  void wait_bucket(Bucket& b, hipStream_t cur, bool timed);
  void sync_slice_locked(Bucket& b, size_t s);
  void finish_slices(Bucket& b);
  void sync_locked(Bucket& b);

  std::vector<at::Tensor> params_;
  std::shared_ptr<Communicator> comm_;
  std::vector<int64_t> reg_handles_;  // register_buckets handles
  void release_registrations();
  ReducerOptions opts_;
  CommHook comm_hook_;
  DeferredGradHook deferred_grad_hook_;
  at::ScalarType hook_wire_ = at::ScalarType::Undefined;

  std::vector<Bucket> buckets_;
  std::vector<std::pair<int64_t, int64_t>> where_;  // param -> (bucket, slot)
  std::vector<std::shared_ptr<torch::autograd::Node>> grad_accs_;
  std::vector<uintptr_t> hook_handles_;

  std::mutex mu_;
  bool expect_hooks_ = false;
  bool require_sync_ = true;
  bool finalize_queued_ = false;
  bool marked_unused_ = false;
  size_t next_bucket_ = 0;
  std::vector<char> ready_;
  std::vector<char> unused_;
  std::vector<char> used_since_sync_;  // find_unused: got a gradient in a no_sync micro-step
  std::vector<int64_t> unused_list_;
  // static_graph: frozen after the first synchronised backward
  bool static_frozen_ = false;
  std::vector<int64_t> static_unused_;
  std::vector<char> static_global_used_;  // empty = every parameter used somewhere
  std::vector<int64_t> ready_order_;
  bool record_order_ = true;
  int64_t iterations_ = 0;
  int64_t rebuilds_ = 0;
  double backward_t0_ms_ = 0;
  hipEvent_t bwd_t0_ev_ = nullptr;  // timing: the compute stream at the backward's first gradient hook
  bool bwd_t0_recorded_ = false;
  bool timing_ = false;
  bool check_ = false;  // ReducerOptions::check_streams / DCP_DEBUG_STREAMS=1
  bool ev_recorded_ = false;  // timing: some bucket's stall events were recorded
  // find_unused_parameters: per-parameter used flags. Host staging (pinned on
  // GPU) -> device -> async MAX all-reduce issued at the first hook ->
  // async copy back on the comm stream; finalize waits only on that small
  // copy's event (launched early in backward), never on the backward itself.
  at::Tensor used_host_, used_dev_, used_back_;
  WorkPtr used_work_;
  hipEvent_t used_ev_ = nullptr;
};

}  // namespace dcp
