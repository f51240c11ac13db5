// Native RCCL communicator over xGMI: stream-ordered collectives on a dedicated high-priority
// HIP stream, fenced to / from the compute stream with hipEvents.
//
// Reference: every collective in the reference went through ProcessGroupNCCL inside DDP / FSDP or
// explicit torch.distributed calls; there was no comm code of its own.
// MI355X design (SURVEY §2.3 "MI355X-native equivalent"):
//  * the communicator is a raw ncclComm_t (RCCL — the same librccl.so torch loads, so one RCCL
//    per process), bootstrapped from an ncclUniqueId that Python shares through the torchrun
//    TCPStore (env:// rendezvous);
//  * every collective runs on a highest-priority stream from torch's stream pool, so
//    bucket all-reduces / FSDP all-gathers are not starved by compute kernels; the comm stream
//    waits on an event recorded on the caller's current stream (inputs ready), and `wait()` makes
//    the caller's current stream wait on the completion event — the host never blocks;
//  * tensors used on the comm stream are recorded with the caching allocator (recordStream) so a
//    buffer freed by Python is not reused before RCCL is done with it;
//  * grouped launches (ncclGroupStart/End) let a whole bucket list go out as one submission.
#include <rccl/rccl.h>

#include <memory>
#include <string>
#include <vector>

#include <c10/hip/HIPCachingAllocator.h>

#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {
namespace {

#define HYP_CHECK_NCCL(expr)                                                                                 \
  do {                                                                                                       \
    ncclResult_t _r = (expr);                                                                                \
    TORCH_CHECK(_r == ncclSuccess, "hyperion RCCL error: ", ncclGetErrorString(_r), " at ", __FILE__, ":", \
                __LINE__);                                                                                   \
  } while (0)

ncclDataType_t nccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "hyperion RCCL: unsupported dtype ", t.scalar_type());
  }
}

ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  if (op == "avg") return ncclAvg;
  TORCH_CHECK(false, "hyperion RCCL: unknown reduce op ", op);
}

// Completion handle: an event recorded on the comm stream after the collective.
class Work {
 public:
  Work(hipEvent_t ev, int device) : ev_(ev), device_(device) {}
  ~Work() {
    if (ev_) (void)hipEventDestroy(ev_);
  }
  // make the caller's current stream wait for the collective (no host block)
  void wait() {
    const at::DeviceGuard g(at::Device(at::kCUDA, device_));
    HYP_CHECK_HIP(hipStreamWaitEvent(c10::hip::getCurrentHIPStream(device_).stream(), ev_, 0));
  }
  void synchronize() { HYP_CHECK_HIP(hipEventSynchronize(ev_)); }
  bool is_completed() { return hipEventQuery(ev_) == hipSuccess; }

 private:
  hipEvent_t ev_;
  int device_;
};

class RcclComm {
 public:
  RcclComm(const std::string& uid_bytes, int rank, int world, int device) : rank_(rank), world_(world), device_(device) {
    TORCH_CHECK(uid_bytes.size() == sizeof(ncclUniqueId), "bad ncclUniqueId size ", uid_bytes.size());
    ncclUniqueId id;
    memcpy(&id, uid_bytes.data(), sizeof(id));
    const at::DeviceGuard g(at::Device(at::kCUDA, device_));
    // a HIGH-priority stream from torch's own pool: it outlives this communicator, so the caching
    // allocator's recordStream bookkeeping (events recorded on this stream when a tensor used by a
    // collective is freed) can never touch a destroyed stream
    stream_obj_ = c10::hip::getStreamFromPool(/*isHighPriority=*/true, device_);
    stream_ = stream_obj_.stream();
    HYP_CHECK_NCCL(ncclCommInitRank(&comm_, world_, id, rank_));
  }
  ~RcclComm() { destroy(); }

  void destroy() {
    if (comm_) {
      (void)ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
    if (stream_) {
      (void)hipStreamSynchronize(stream_);  // pooled stream: drained, never destroyed
      stream_ = nullptr;
    }
  }

  void abort() {
    if (comm_) {
      (void)ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

  int rank() const { return rank_; }
  int world() const { return world_; }
  int64_t stream_handle() const { return reinterpret_cast<int64_t>(stream_); }

  std::shared_ptr<Work> all_reduce(at::Tensor& t, const std::string& op) {
    check(t);
    begin({t});
    HYP_CHECK_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), comm_, stream_));
    return end();
  }

  std::shared_ptr<Work> all_reduce_coalesced(std::vector<at::Tensor>& ts, const std::string& op) {
    for (auto& t : ts) check(t);
    begin(ts);
    HYP_CHECK_NCCL(ncclGroupStart());
    for (auto& t : ts)
      HYP_CHECK_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), comm_, stream_));
    HYP_CHECK_NCCL(ncclGroupEnd());
    return end();
  }

  std::shared_ptr<Work> reduce_scatter(at::Tensor& out, const at::Tensor& in, const std::string& op) {
    check(out);
    check(in);
    TORCH_CHECK(in.numel() == out.numel() * world_ && in.scalar_type() == out.scalar_type(), "reduce_scatter sizes");
    begin({out, in});
    HYP_CHECK_NCCL(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_dtype(out), nccl_op(op), comm_,
                                     stream_));
    return end();
  }

  std::shared_ptr<Work> all_gather(at::Tensor& out, const at::Tensor& in) {
    check(out);
    check(in);
    TORCH_CHECK(out.numel() == in.numel() * world_ && in.scalar_type() == out.scalar_type(), "all_gather sizes");
    begin({out, in});
    HYP_CHECK_NCCL(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dtype(in), comm_, stream_));
    return end();
  }

  std::shared_ptr<Work> broadcast(at::Tensor& t, int root) {
    check(t);
    begin({t});
    HYP_CHECK_NCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), root, comm_, stream_));
    return end();
  }

  // all-to-all of equal chunks (expert / sequence parallel exchanges) as grouped send/recv
  std::shared_ptr<Work> all_to_all(at::Tensor& out, const at::Tensor& in) {
    check(out);
    check(in);
    TORCH_CHECK(in.numel() == out.numel() && in.numel() % world_ == 0, "all_to_all sizes");
    const int64_t n = in.numel() / world_;
    const int64_t es = in.element_size();
    begin({out, in});
    HYP_CHECK_NCCL(ncclGroupStart());
    for (int p = 0; p < world_; ++p) {
      HYP_CHECK_NCCL(ncclSend(static_cast<const char*>(in.data_ptr()) + p * n * es, n, nccl_dtype(in), p, comm_, stream_));
      HYP_CHECK_NCCL(ncclRecv(static_cast<char*>(out.data_ptr()) + p * n * es, n, nccl_dtype(out), p, comm_, stream_));
    }
    HYP_CHECK_NCCL(ncclGroupEnd());
    return end();
  }

  void barrier() {
    auto t = at::zeros({1}, at::TensorOptions().device(at::Device(at::kCUDA, device_)).dtype(at::kFloat));
    all_reduce(t, "sum")->synchronize();
  }

  std::string async_error() {
    ncclResult_t r = ncclSuccess;
    if (comm_) HYP_CHECK_NCCL(ncclCommGetAsyncError(comm_, &r));
    return r == ncclSuccess ? "" : ncclGetErrorString(r);
  }

 private:
  void check(const at::Tensor& t) const {
    TORCH_CHECK(comm_ != nullptr, "hyperion RCCL communicator is destroyed");
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_, "tensor must live on cuda:", device_);
    TORCH_CHECK(t.is_contiguous(), "collective tensors must be contiguous");
  }

  // comm stream waits for the producer stream; tensors are marked in use by the comm stream
  void begin(std::vector<at::Tensor> ts) {
    const at::DeviceGuard g(at::Device(at::kCUDA, device_));
    auto cur = c10::hip::getCurrentHIPStream(device_);
    hipEvent_t ready;
    HYP_CHECK_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    HYP_CHECK_HIP(hipEventRecord(ready, cur.stream()));
    HYP_CHECK_HIP(hipStreamWaitEvent(stream_, ready, 0));
    HYP_CHECK_HIP(hipEventDestroy(ready));  // destruction is deferred until the wait is satisfied
    for (auto& t : ts) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_obj_);
  }

  std::shared_ptr<Work> end() {
    hipEvent_t done;
    HYP_CHECK_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    HYP_CHECK_HIP(hipEventRecord(done, stream_));
    return std::make_shared<Work>(done, device_);
  }

  ncclComm_t comm_ = nullptr;
  c10::hip::HIPStream stream_obj_ = c10::hip::getDefaultHIPStream();
  hipStream_t stream_ = nullptr;
  int rank_, world_, device_;
};

pybind11::bytes unique_id() {
  ncclUniqueId id;
  HYP_CHECK_NCCL(ncclGetUniqueId(&id));
  return pybind11::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

int version() {
  int v = 0;
  HYP_CHECK_NCCL(ncclGetVersion(&v));
  return v;
}

}  // namespace

void register_comm(pybind11::module& m) {
  namespace py = pybind11;
  m.def("rccl_unique_id", &unique_id, "new ncclUniqueId (bytes) for bootstrap");
  m.def("rccl_version", &version, "RCCL version code");
  py::class_<Work, std::shared_ptr<Work>>(m, "RcclWork")
      .def("wait", &Work::wait, "current stream waits for the collective (no host block)")
      .def("synchronize", &Work::synchronize)
      .def("is_completed", &Work::is_completed);
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, int>(), py::arg("unique_id"), py::arg("rank"), py::arg("world"),
           py::arg("device"))
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("stream_handle", &RcclComm::stream_handle)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("tensor"), py::arg("op") = "sum")
      .def("all_reduce_coalesced", &RcclComm::all_reduce_coalesced, py::arg("tensors"), py::arg("op") = "sum")
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::arg("out"), py::arg("inp"), py::arg("op") = "sum")
      .def("all_gather", &RcclComm::all_gather, py::arg("out"), py::arg("inp"))
      .def("broadcast", &RcclComm::broadcast, py::arg("tensor"), py::arg("root") = 0)
      .def("all_to_all", &RcclComm::all_to_all, py::arg("out"), py::arg("inp"))
      .def("barrier", &RcclComm::barrier)
      .def("async_error", &RcclComm::async_error)
      .def("abort", &RcclComm::abort)
      .def("destroy", &RcclComm::destroy);
}

}  // namespace hypbind
