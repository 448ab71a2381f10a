// Python bindings of the native runtime: store, communicators, reducer,
// planner and the multi-tensor / fused kernels.
#include <torch/extension.h>

#include "comm/communicator.h"
#include "common.h"
#include "fused.h"
#include "kernels/gemm_kernels.h"
#include "ops.h"
#include "reducer/reducer.h"

namespace dcp {
namespace stem {
void bind(pybind11::module& m);
}
namespace convnet {
void bind(pybind11::module& m);
}
}  // namespace dcp
#include "trace/trace.h"
#include "store/tcp_store.h"

namespace py = pybind11;
using namespace dcp;

namespace {
// Work whose result is produced by a Python comm hook synchronously.
class DoneWork : public Work {
 public:
  bool is_completed() override { return true; }
  void wait() override {}
  void synchronize() override {}
};
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "distributed_compute_pytorch_amd native runtime (gfx950 / RCCL)";

  static py::exception<TimeoutError> timeout_exc(m, "DistTimeoutError", PyExc_TimeoutError);
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const TimeoutError& e) {
      PyErr_SetString(PyExc_TimeoutError, e.what());
    }
  });

  // ------------------------------------------------------------ store ---
  py::class_<TCPStore, std::shared_ptr<TCPStore>>(m, "TCPStore")
      .def(py::init<const std::string&, int, int, bool, int64_t, bool>(), py::arg("host"), py::arg("port"),
           py::arg("world_size"), py::arg("is_master"), py::arg("timeout_ms") = 1800000,
           py::arg("wait_for_workers") = true, py::call_guard<py::gil_scoped_release>())
      .def("set", [](TCPStore& s, const std::string& k, py::bytes v) {
             std::string val = v;
             py::gil_scoped_release r;
             s.set(k, val);
           })
      .def("get", [](TCPStore& s, const std::string& k) {
             std::string v;
             {
               py::gil_scoped_release r;
               v = s.get(k);
             }
             return py::bytes(v);
           })
      .def("add", &TCPStore::add, py::call_guard<py::gil_scoped_release>())
      .def("check", &TCPStore::check, py::call_guard<py::gil_scoped_release>())
      .def("wait", &TCPStore::wait, py::arg("keys"), py::arg("timeout_ms") = -1,
           py::call_guard<py::gil_scoped_release>())
      .def("delete_key", &TCPStore::delete_key, py::call_guard<py::gil_scoped_release>())
      .def("num_keys", &TCPStore::num_keys, py::call_guard<py::gil_scoped_release>())
      .def("compare_set", [](TCPStore& s, const std::string& k, py::bytes e, py::bytes d) {
             std::string es = e, ds = d, r;
             {
               py::gil_scoped_release g;
               r = s.compare_set(k, es, ds);
             }
             return py::bytes(r);
           })
      .def("barrier", &TCPStore::barrier, py::arg("tag") = "default", py::call_guard<py::gil_scoped_release>())
      .def("local_ip", &TCPStore::local_ip)
      .def_property_readonly("port", &TCPStore::port)
      .def_property_readonly("host", &TCPStore::host)
      .def_property_readonly("world_size", &TCPStore::world_size)
      .def_property("timeout_ms", &TCPStore::timeout_ms, &TCPStore::set_timeout_ms);

  // ------------------------------------------------------ communicator ---
  py::enum_<ReduceOp>(m, "ReduceOp")
      .value("SUM", ReduceOp::SUM)
      .value("AVG", ReduceOp::AVG)
      .value("PRODUCT", ReduceOp::PRODUCT)
      .value("MIN", ReduceOp::MIN)
      .value("MAX", ReduceOp::MAX);

  py::class_<Work, std::shared_ptr<Work>>(m, "Work")
      .def("is_completed", &Work::is_completed)
      .def("wait", &Work::wait, py::call_guard<py::gil_scoped_release>())
      .def("synchronize", &Work::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("elapsed_ms", &Work::elapsed_ms)
      .def_readonly("outputs", &Work::outputs);

  py::class_<Communicator, std::shared_ptr<Communicator>>(m, "Communicator")
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("size", &Communicator::size)
      .def_property_readonly("backend", &Communicator::backend)
      .def_property_readonly("stream_handle", &Communicator::stream_handle)
      .def("all_reduce", &Communicator::all_reduce, py::call_guard<py::gil_scoped_release>())
      .def("all_reduce_into", &Communicator::all_reduce_into, py::arg("wire"), py::arg("out"), py::arg("op"),
           py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &Communicator::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &Communicator::all_gather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &Communicator::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("all_to_all", &Communicator::all_to_all, py::call_guard<py::gil_scoped_release>())
      .def("send", &Communicator::send, py::call_guard<py::gil_scoped_release>())
      .def("recv", &Communicator::recv, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &Communicator::barrier, py::call_guard<py::gil_scoped_release>())
      .def("abort", &Communicator::abort)
      .def("transport_size", &Communicator::transport_size)
      .def("set_timing", &Communicator::set_timing)
      .def("stream_fence", &Communicator::stream_fence, py::call_guard<py::gil_scoped_release>())
      .def("register_buffer", &Communicator::register_buffer, py::arg("tensor"))
      .def("deregister_buffer", &Communicator::deregister_buffer, py::arg("handle"))
      .def("emulate_all_reduce", &Communicator::emulate_all_reduce, py::arg("t"), py::arg("world"),
           py::arg("busbw_gbps"), py::arg("channels"), py::arg("alpha_us") = 20.0,
           py::call_guard<py::gil_scoped_release>())
      .def("split", &Communicator::split, py::arg("color"), py::arg("key"), py::arg("prefix"),
           py::call_guard<py::gil_scoped_release>())
      .def("error", &Communicator::error)
      .def("set_debug_fingerprint", &Communicator::set_debug_fingerprint)
      .def_property_readonly("ops_issued", &Communicator::ops_issued)
      .def_property_readonly("bytes_issued", &Communicator::bytes_issued);

  m.def("make_host_communicator", &make_host_communicator, py::arg("store"), py::arg("prefix"), py::arg("rank"),
        py::arg("size"), py::arg("timeout_ms") = 1800000, py::call_guard<py::gil_scoped_release>());
  m.def("make_rccl_communicator", &make_rccl_communicator, py::arg("store"), py::arg("prefix"), py::arg("rank"),
        py::arg("size"), py::arg("device"), py::arg("timeout_ms") = 1800000,
        py::call_guard<py::gil_scoped_release>());
  m.def("rccl_version", &rccl_version);

  // ----------------------------------------------------------- reducer ---
  m.def("compute_bucket_assignment", &compute_bucket_assignment, py::arg("sizes_bytes"), py::arg("keys"),
        py::arg("limits"), py::arg("order") = std::vector<int64_t>{});

  m.def("split_tail_bucket", &split_tail_bucket, py::arg("assignment"), py::arg("sizes_bytes"),
        py::arg("tail_bytes"));

  py::class_<ReducerOptions>(m, "ReducerOptions")
      .def(py::init<>())
      .def_readwrite("gradient_as_bucket_view", &ReducerOptions::gradient_as_bucket_view)
      .def_readwrite("find_unused_parameters", &ReducerOptions::find_unused_parameters)
      .def_readwrite("rebuild_buckets", &ReducerOptions::rebuild_buckets)
      .def_readwrite("first_bucket_bytes", &ReducerOptions::first_bucket_bytes)
      .def_readwrite("bucket_bytes_cap", &ReducerOptions::bucket_bytes_cap)
      .def_readwrite("tail_bucket_bytes", &ReducerOptions::tail_bucket_bytes)
      .def_readwrite("comm_dtype", &ReducerOptions::comm_dtype)
      .def_readwrite("average", &ReducerOptions::average)
      .def_readwrite("register_buckets", &ReducerOptions::register_buckets)
      .def_readwrite("check_streams", &ReducerOptions::check_streams)
      .def_readwrite("defer_grad_wait", &ReducerOptions::defer_grad_wait)
      .def_readwrite("slice_bytes", &ReducerOptions::slice_bytes)
      .def_readwrite("static_graph", &ReducerOptions::static_graph);

  m.def("trace_enabled", &trace::enabled);
  m.def("trace_push", [](const std::string& n) { trace::push(n.c_str()); });
  m.def("trace_pop", &trace::pop);
  m.def("trace_mark", [](const std::string& n) { trace::mark(n.c_str()); });
  py::class_<BucketStats>(m, "BucketStats")
      .def_readonly("bytes", &BucketStats::bytes)
      .def_readonly("num_params", &BucketStats::num_params)
      .def_readonly("ready_ms", &BucketStats::ready_ms)
      .def_readonly("ready_dev_ms", &BucketStats::ready_dev_ms)
      .def_readonly("comm_ms", &BucketStats::comm_ms);

  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init([](std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
                       std::shared_ptr<Communicator> comm, ReducerOptions opts) {
             auto r = std::make_shared<Reducer>(std::move(params), std::move(buckets), std::move(comm), opts);
             r->register_hooks();
             return r;
           }),
           py::arg("params"), py::arg("buckets"), py::arg("comm"), py::arg("options"))
      .def("prepare_for_backward", &Reducer::prepare_for_backward, py::arg("outputs"), py::arg("require_sync"))
      .def("set_expect_backward", &Reducer::set_expect_backward)
      .def("set_comm_hook", [](Reducer& r, py::object fn, py::object wire_dtype) {
             if (fn.is_none()) {
               r.set_comm_hook(nullptr);
               return;
             }
             at::ScalarType wdt = at::ScalarType::Undefined;
             if (!wire_dtype.is_none()) wdt = torch::python::detail::py_object_to_dtype(wire_dtype);
             auto holder = std::make_shared<py::object>(fn);
             r.set_comm_hook([holder](at::Tensor& bucket, int64_t index) -> WorkPtr {
               py::gil_scoped_acquire g;
               py::object res = (*holder)(bucket, index);
               if (res.is_none()) return std::make_shared<DoneWork>();
               return res.cast<WorkPtr>();
             }, wdt);
           }, py::arg("fn"), py::arg("wire_dtype") = py::none())
      .def("set_deferred_grad_hook", [](Reducer& r, py::object fn) {
             if (fn.is_none()) {
               r.set_deferred_grad_hook(nullptr);
               return;
             }
             auto holder = std::make_shared<py::object>(fn);
             r.set_deferred_grad_hook([holder](int64_t k, const std::vector<at::Tensor>& views) {
               py::gil_scoped_acquire g;
               return (*holder)(k, views).cast<std::vector<at::Tensor>>();
             });
           }, py::arg("fn"))
      .def("bucket_indices", &Reducer::bucket_indices)
      .def("bucket_sizes_bytes", &Reducer::bucket_sizes_bytes)
      .def("bucket_stats", &Reducer::bucket_stats)
      .def("exposed_comm_ms", &Reducer::exposed_comm_ms)
      .def("bucket_buffers", &Reducer::bucket_buffers)
      .def("ready_order", &Reducer::ready_order)
      .def("wait_all", &Reducer::wait_all, py::call_guard<py::gil_scoped_release>())
      .def("deferred_buckets", &Reducer::deferred_buckets)
      .def("sync_bucket", &Reducer::sync_bucket, py::call_guard<py::gil_scoped_release>())
      .def("bucket_slice_bounds", &Reducer::bucket_slice_bounds)
      .def("sync_bucket_slice", &Reducer::sync_bucket_slice, py::call_guard<py::gil_scoped_release>())
      .def("sync_all", &Reducer::sync_all, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("num_iterations", &Reducer::num_iterations)
      .def_property_readonly("num_rebuilds", &Reducer::num_rebuilds)
      .def_property_readonly("static_frozen", &Reducer::static_frozen)
      .def("static_unused", &Reducer::static_unused)
      .def("note_used", &Reducer::note_used)
      .def("set_timing", &Reducer::set_timing);

  // ------------------------------------------------------------- ops ---
  m.def("mt_copy", &ops::mt_copy, py::arg("src"), py::arg("dst"), py::arg("scale") = 1.0);
  m.def("fused_sgd", &ops::fused_sgd);
  m.def("fused_adam", &ops::fused_adam, pybind11::arg("params"), pybind11::arg("grads"), pybind11::arg("exp_avgs"),
        pybind11::arg("exp_avg_sqs"), pybind11::arg("max_exp_avg_sqs"), pybind11::arg("lr"), pybind11::arg("beta1"),
        pybind11::arg("beta2"), pybind11::arg("eps"), pybind11::arg("weight_decay"), pybind11::arg("step"),
        pybind11::arg("amsgrad"), pybind11::arg("decoupled"), pybind11::arg("maximize"),
        pybind11::arg("grad_scale"), pybind11::arg("shadows") = std::vector<at::Tensor>{},
        pybind11::arg("steps") = std::vector<at::Tensor>{});
  m.def("fused_adadelta", &ops::fused_adadelta);
  m.def("sumsq", &ops::sumsq);
  m.def("scale_by", &ops::scale_by);
  m.def("table_cache_size", &ops::table_cache_size);

  m.def("gemm_tune", [](const std::string& k, int v) { kern::gemm_tune(k.c_str(), v); });
  m.def("gemm_pp_splitk", [](int64_t M, int N, int K) { return kern::gemm_pp_splitk(M, N, K); },
        "split-K count gemm_pp uses for this shape (1 = none)");
  m.def("gemm_tune_get", [](const std::string& k) { return kern::gemm_tune_get(k.c_str()); });

  fused::bind(m);
  stem::bind(m);
  convnet::bind(m);
}
