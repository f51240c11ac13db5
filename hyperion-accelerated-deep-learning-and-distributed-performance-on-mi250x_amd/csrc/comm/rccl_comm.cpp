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
//  * grouped launches (ncclGroupStart/End) let a whole bucket list go out as one submission;
//  * failure instead of a hang (comm/watchdog.h): the communicator is created NONBLOCKING
//    (ncclCommInitRankConfig, blocking=0) so a peer that never joins hits the deadline instead of
//    blocking init forever; every collective's completion event is supervised by a per-communicator
//    watchdog thread against `timeout_s` (the setup(timeout_s) value) together with
//    ncclCommGetAsyncError; on expiry it calls ncclCommAbort (RCCL kernels waiting on a dead peer
//    exit) and every later collective / Work.wait() raises RuntimeError naming the collective.
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "comm/watchdog.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>

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

// "avg" is issued as ncclSum followed by a 1/world scale on the comm stream (scale_avg below), never
// as ncclAvg: the torch-bundled RCCL 2.26.6 leaves the last 4-16 elements of some reduce-scatter
// outputs unwritten under ncclAvg (bf16 132480 / 131392 / 133568 elements, fp32 16704 / 17024 /
// ..., single rank — scripts/rccl_avg_check.py), which corrupted the tail of FSDP flat gradients.
ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum" || op == "avg") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "hyperion RCCL: unknown reduce op ", op);
}

// An owned hipEvent shared between a Work handle and the watchdog's probe.
struct EventBox {
  hipEvent_t ev = nullptr;
  ~EventBox() {
    if (ev) (void)hipEventDestroy(ev);
  }
};

[[noreturn]] void raise_comm_failure(const std::string& why) {
  throw std::runtime_error("hyperion RCCL communicator failed: " + why);
}

// Completion handle: an event recorded on the comm stream after the collective.
class Work {
 public:
  Work(std::shared_ptr<EventBox> ev, int device, std::shared_ptr<hypcomm::Watchdog> wd)
      : ev_(std::move(ev)), device_(device), wd_(std::move(wd)) {}
  // make the caller's current stream wait for the collective (no host block); raises if the
  // communicator has failed (timeout / async error), so a dead peer surfaces at the next wait
  void wait() {
    check_failed();
    const at::DeviceGuard g(at::Device(at::kCUDA, device_));
    HYP_CHECK_HIP(hipStreamWaitEvent(c10::hip::getCurrentHIPStream(device_).stream(), ev_->ev, 0));
  }
  // host wait that stays interruptible by the watchdog (never an unbounded hipEventSynchronize)
  void synchronize() {
    for (;;) {
      check_failed();
      const hipError_t e = hipEventQuery(ev_->ev);
      if (e == hipSuccess) return;
      TORCH_CHECK(e == hipErrorNotReady, "hyperion RCCL: event query failed: ", hipGetErrorString(e));
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  bool is_completed() {
    check_failed();
    return hipEventQuery(ev_->ev) == hipSuccess;
  }

 private:
  void check_failed() const {
    if (wd_ && wd_->failed()) raise_comm_failure(wd_->error());
  }
  std::shared_ptr<EventBox> ev_;
  int device_;
  std::shared_ptr<hypcomm::Watchdog> wd_;
};

class RcclComm {
 public:
  RcclComm(const std::string& uid_bytes, int rank, int world, int device, double timeout_s)
      : rank_(rank), world_(world), device_(device), timeout_s_(timeout_s) {
    TORCH_CHECK(uid_bytes.size() == sizeof(ncclUniqueId), "bad ncclUniqueId size ", uid_bytes.size());
    TORCH_CHECK(timeout_s > 0, "timeout_s must be > 0");
    ncclUniqueId id;
    memcpy(&id, uid_bytes.data(), sizeof(id));
    const at::DeviceGuard g(at::Device(at::kCUDA, device_));
    // a HIGH-priority stream from torch's own pool: it outlives this communicator, so the caching
    // allocator's recordStream bookkeeping (events recorded on this stream when a tensor used by a
    // collective is freed) can never touch a destroyed stream
    stream_obj_ = c10::hip::getStreamFromPool(/*isHighPriority=*/true, device_);
    stream_ = stream_obj_.stream();
    // nonblocking init: returns at once; ncclCommGetAsyncError reports ncclInProgress until every
    // rank has joined, so a missing peer is a deadline, not an infinite block inside RCCL
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&comm_, world_, id, rank_, &cfg);
    settle(r, "ncclCommInitRankConfig");
    const char* act = std::getenv("HYPERION_COMM_ON_TIMEOUT");
    exit_on_fail_ = act != nullptr && std::string(act) == "exit";
    const char* poll = std::getenv("HYPERION_COMM_POLL_MS");
    const double poll_ms = poll ? std::atof(poll) : 2.0;
    wd_ = std::make_shared<hypcomm::Watchdog>(
        timeout_s_, poll_ms > 0 ? poll_ms : 2.0,
        [this]() -> std::string {
          std::lock_guard<std::recursive_mutex> g(mu_);
          if (!comm_) return "";
          ncclResult_t a = ncclSuccess;
          if (ncclCommGetAsyncError(comm_, &a) != ncclSuccess) return "ncclCommGetAsyncError failed";
          return (a == ncclSuccess || a == ncclInProgress) ? "" : ncclGetErrorString(a);
        },
        [this](const std::string& why) { on_failure(why); },
        []() {
          // the watchdog thread must never join (or invalidate) a graph capture that another
          // thread runs in global capture mode: its event queries run in relaxed mode
          hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
          (void)hipThreadExchangeStreamCaptureMode(&mode);
        });
  }
  ~RcclComm() { destroy(); }

  void destroy() {
    if (wd_) wd_->stop();  // no probe may run against a destroyed communicator
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (comm_) {
      if (wd_ && wd_->failed()) {
        (void)ncclCommAbort(comm_);
      } else {
        (void)ncclCommDestroy(comm_);
      }
      comm_ = nullptr;
    }
    if (stream_) {
      if (!(wd_ && wd_->failed())) (void)hipStreamSynchronize(stream_);  // pooled stream: drained, never destroyed
      stream_ = nullptr;
    }
  }

  void abort() {
    if (wd_) wd_->fail("aborted by the caller");
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (comm_) {
      (void)ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

  std::string error() const { return wd_ ? wd_->error() : std::string(); }
  size_t pending() const { return wd_ ? wd_->pending() : 0; }
  double timeout_s() const { return timeout_s_; }

  int rank() const { return rank_; }
  int world() const { return world_; }
  int64_t stream_handle() const { return reinterpret_cast<int64_t>(stream_); }

  // the 1/world of an "avg" (see nccl_op), on the comm stream before the completion event
  void scale_avg(at::Tensor& t, const std::string& op) {
    const int div = avg_div_ > 0 ? avg_div_ : world_;
    if (op != "avg" || div == 1) return;
    const c10::hip::HIPStreamGuard sg(stream_obj_);
    t.mul_(1.0 / div);
  }
  // tests only: the divisor "avg" applies (0 = the world size), so a one-GPU run drives the
  // world > 1 branch of scale_avg (a 2-rank RCCL communicator needs two GPUs)
  void set_avg_divisor(int d) { avg_div_ = d; }

  std::shared_ptr<Work> all_reduce(at::Tensor& t, const std::string& op) {
    check(t);
    std::lock_guard<std::recursive_mutex> g(mu_);
    begin({t});
    settle(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), comm_, stream_),
           "all_reduce");
    scale_avg(t, op);
    return end("all_reduce", t.numel() * t.element_size());
  }

  std::shared_ptr<Work> all_reduce_coalesced(std::vector<at::Tensor>& ts, const std::string& op) {
    for (auto& t : ts) check(t);
    std::lock_guard<std::recursive_mutex> g(mu_);
    begin(ts);
    int64_t bytes = 0;
    HYP_CHECK_NCCL(ncclGroupStart());
    for (auto& t : ts) {
      bytes += t.numel() * t.element_size();
      HYP_CHECK_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), comm_, stream_));
    }
    settle(ncclGroupEnd(), "all_reduce_coalesced");
    for (auto& t : ts) scale_avg(t, op);
    return end("all_reduce_coalesced", bytes);
  }

  std::shared_ptr<Work> reduce_scatter(at::Tensor& out, const at::Tensor& in, const std::string& op) {
    check(out);
    check(in);
    TORCH_CHECK(in.numel() == out.numel() * world_ && in.scalar_type() == out.scalar_type(), "reduce_scatter sizes");
    std::lock_guard<std::recursive_mutex> g(mu_);
    begin({out, in});
    settle(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_dtype(out), nccl_op(op), comm_, stream_),
           "reduce_scatter");
    scale_avg(out, op);
    return end("reduce_scatter", in.numel() * in.element_size());
  }

  std::shared_ptr<Work> all_gather(at::Tensor& out, const at::Tensor& in) {
    check(out);
    check(in);
    TORCH_CHECK(out.numel() == in.numel() * world_ && in.scalar_type() == out.scalar_type(), "all_gather sizes");
    std::lock_guard<std::recursive_mutex> g(mu_);
    begin({out, in});
    settle(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dtype(in), comm_, stream_), "all_gather");
    return end("all_gather", out.numel() * out.element_size());
  }

  std::shared_ptr<Work> broadcast(at::Tensor& t, int root) {
    check(t);
    std::lock_guard<std::recursive_mutex> g(mu_);
    begin({t});
    settle(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), root, comm_, stream_), "broadcast");
    return end("broadcast", t.numel() * t.element_size());
  }

  // all-to-all of equal chunks (expert / sequence parallel exchanges) as grouped send/recv
  std::shared_ptr<Work> all_to_all(at::Tensor& out, const at::Tensor& in) {
    check(out);
    check(in);
    TORCH_CHECK(in.numel() == out.numel() && in.numel() % world_ == 0, "all_to_all sizes");
    const int64_t n = in.numel() / world_;
    const int64_t es = in.element_size();
    std::lock_guard<std::recursive_mutex> g(mu_);
    begin({out, in});
    HYP_CHECK_NCCL(ncclGroupStart());
    for (int p = 0; p < world_; ++p) {
      HYP_CHECK_NCCL(ncclSend(static_cast<const char*>(in.data_ptr()) + p * n * es, n, nccl_dtype(in), p, comm_, stream_));
      HYP_CHECK_NCCL(ncclRecv(static_cast<char*>(out.data_ptr()) + p * n * es, n, nccl_dtype(out), p, comm_, stream_));
    }
    settle(ncclGroupEnd(), "all_to_all");
    return end("all_to_all", in.numel() * es);
  }

  void barrier() {
    auto t = at::zeros({1}, at::TensorOptions().device(at::Device(at::kCUDA, device_)).dtype(at::kFloat));
    all_reduce(t, "sum")->synchronize();
  }

  std::string async_error() {
    std::lock_guard<std::recursive_mutex> g(mu_);
    ncclResult_t r = ncclSuccess;
    if (comm_) HYP_CHECK_NCCL(ncclCommGetAsyncError(comm_, &r));
    return (r == ncclSuccess || r == ncclInProgress) ? "" : ncclGetErrorString(r);
  }

 private:
  void check(const at::Tensor& t) const {
    if (wd_ && wd_->failed()) raise_comm_failure(wd_->error());
    TORCH_CHECK(comm_ != nullptr, "hyperion RCCL communicator is destroyed");
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_, "tensor must live on cuda:", device_);
    TORCH_CHECK(t.is_contiguous(), "collective tensors must be contiguous");
  }

  // A nonblocking communicator may answer ncclInProgress: poll its state to completion, bounded by
  // the timeout (an init whose peers never arrive, a group launch that cannot enqueue).
  void settle(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) {
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s_);
      do {
        if (std::chrono::steady_clock::now() > deadline) {
          const std::string why = std::string(what) + " still in progress after the " + std::to_string(timeout_s_) +
                                  " s timeout (a peer rank never joined)";
          if (wd_) {
            wd_->fail(why);  // runs on_failure: aborts the communicator (recursive lock)
          } else if (comm_) {
            (void)ncclCommAbort(comm_);  // init never completed: no watchdog yet
            comm_ = nullptr;
          }
          raise_comm_failure(why);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
        HYP_CHECK_NCCL(ncclCommGetAsyncError(comm_, &r));
      } while (r == ncclInProgress);
    }
    TORCH_CHECK(r == ncclSuccess, "hyperion RCCL error in ", what, ": ", ncclGetErrorString(r));
  }

  // comm stream waits for the producer stream; tensors are marked in use by the comm stream
  void begin(std::vector<at::Tensor> ts) {
    // (under mu_: the watchdog may have aborted the communicator since the unlocked check())
    if (wd_ && wd_->failed()) raise_comm_failure(wd_->error());
    TORCH_CHECK(comm_ != nullptr, "hyperion RCCL communicator is destroyed");
    const at::DeviceGuard g(at::Device(at::kCUDA, device_));
    auto cur = c10::hip::getCurrentHIPStream(device_);
    hipEvent_t ready;
    HYP_CHECK_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    HYP_CHECK_HIP(hipEventRecord(ready, cur.stream()));
    HYP_CHECK_HIP(hipStreamWaitEvent(stream_, ready, 0));
    HYP_CHECK_HIP(hipEventDestroy(ready));  // destruction is deferred until the wait is satisfied
    for (auto& t : ts) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_obj_);
  }

  std::shared_ptr<Work> end(const char* what, int64_t bytes) {
    auto box = std::make_shared<EventBox>();
    HYP_CHECK_HIP(hipEventCreateWithFlags(&box->ev, hipEventDisableTiming));
    HYP_CHECK_HIP(hipEventRecord(box->ev, stream_));
    ++seq_;
    // a collective recorded into a graph under capture has no host-observable completion: only
    // eagerly issued collectives are supervised
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HYP_CHECK_HIP(hipStreamIsCapturing(stream_, &cs));
    if (wd_ && cs == hipStreamCaptureStatusNone) {
      std::shared_ptr<EventBox> probe_ev = box;
      wd_->watch(
          [probe_ev]() -> int {
            const hipError_t e = hipEventQuery(probe_ev->ev);
            if (e == hipSuccess) return hypcomm::Watchdog::kDone;
            if (e == hipErrorNotReady) return hypcomm::Watchdog::kPending;
            return hypcomm::Watchdog::kFailed;
          },
          std::string(what) + " #" + std::to_string(seq_) + " (" + std::to_string(bytes) + " B, rank " +
              std::to_string(rank_) + "/" + std::to_string(world_) + ")");
    }
    return std::make_shared<Work>(box, device_, wd_);
  }

  // watchdog failure action (runs once, on the watchdog thread)
  void on_failure(const std::string& why) {
    std::fprintf(stderr, "[hyperion] RCCL communicator rank %d/%d: %s -- aborting the communicator\n", rank_, world_,
                 why.c_str());
    std::fflush(stderr);
    {
      std::lock_guard<std::recursive_mutex> g(mu_);
      if (comm_) {
        (void)ncclCommAbort(comm_);
        comm_ = nullptr;
      }
    }
    if (exit_on_fail_) {
      std::fprintf(stderr, "[hyperion] HYPERION_COMM_ON_TIMEOUT=exit: terminating rank %d\n", rank_);
      std::fflush(stderr);
      std::_Exit(75);
    }
  }

  // serialises RCCL calls against the watchdog's abort (recursive: a timed-out settle() fails the
  // watchdog, whose action re-locks to abort)
  mutable std::recursive_mutex mu_;
  ncclComm_t comm_ = nullptr;
  c10::hip::HIPStream stream_obj_ = c10::hip::getDefaultHIPStream();
  hipStream_t stream_ = nullptr;
  int rank_, world_, device_;
  int avg_div_ = 0;
  double timeout_s_;
  bool exit_on_fail_ = false;
  int64_t seq_ = 0;
  std::shared_ptr<hypcomm::Watchdog> wd_;
};

// CPU-testable harness around the SAME Watchdog class: simulated work handles whose completion /
// failure the test drives, and a recorded failure action instead of ncclCommAbort.
class WatchdogSim {
 public:
  WatchdogSim(double timeout_s, double poll_ms) {
    wd_ = std::make_shared<hypcomm::Watchdog>(
        timeout_s, poll_ms,
        [this]() -> std::string {
          std::lock_guard<std::mutex> g(mu_);
          return async_;
        },
        [this](const std::string& why) {
          std::lock_guard<std::mutex> g(mu_);
          ++aborts_;
          last_ = why;
        });
  }
  ~WatchdogSim() { wd_->stop(); }
  int submit(const std::string& what) {
    auto st = std::make_shared<std::atomic<int>>(hypcomm::Watchdog::kPending);
    int id;
    {
      std::lock_guard<std::mutex> g(mu_);
      id = static_cast<int>(ops_.size());
      ops_.push_back(st);
    }
    wd_->watch([st]() -> int { return st->load(); }, what);
    return id;
  }
  void complete(int id) { op(id)->store(hypcomm::Watchdog::kDone); }
  void fail_op(int id) { op(id)->store(hypcomm::Watchdog::kFailed); }
  void set_async_error(const std::string& e) {
    std::lock_guard<std::mutex> g(mu_);
    async_ = e;
  }
  std::string error() const { return wd_->error(); }
  bool failed() const { return wd_->failed(); }
  size_t pending() const { return wd_->pending(); }
  int aborts() const {
    std::lock_guard<std::mutex> g(mu_);
    return aborts_;
  }
  bool drain(double max_s) {
    // bounded drain for tests: poll instead of blocking forever
    const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(max_s);
    while (std::chrono::steady_clock::now() < end) {
      if (wd_->failed()) return false;
      if (wd_->pending() == 0) return true;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return false;
  }

 private:
  std::shared_ptr<std::atomic<int>> op(int id) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(id >= 0 && id < static_cast<int>(ops_.size()), "bad op id");
    return ops_[id];
  }
  mutable std::mutex mu_;
  std::vector<std::shared_ptr<std::atomic<int>>> ops_;
  std::string async_, last_;
  int aborts_ = 0;
  std::shared_ptr<hypcomm::Watchdog> wd_;
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
      .def(py::init<const std::string&, int, int, int, double>(), py::arg("unique_id"), py::arg("rank"),
           py::arg("world"), py::arg("device"), py::arg("timeout_s") = 600.0)
      .def_property_readonly("timeout_s", &RcclComm::timeout_s)
      .def("error", &RcclComm::error, "'' while healthy, else why the communicator failed")
      .def("pending", &RcclComm::pending, "collectives still supervised by the watchdog")
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
      .def("set_avg_divisor", &RcclComm::set_avg_divisor, "tests: the divisor of 'avg' (0 = world size)")
      .def("abort", &RcclComm::abort)
      .def("destroy", &RcclComm::destroy);
  py::class_<WatchdogSim>(m, "WatchdogSim", "CPU harness for the communicator watchdog (tests)")
      .def(py::init<double, double>(), py::arg("timeout_s"), py::arg("poll_ms") = 1.0)
      .def("submit", &WatchdogSim::submit)
      .def("complete", &WatchdogSim::complete)
      .def("fail_op", &WatchdogSim::fail_op)
      .def("set_async_error", &WatchdogSim::set_async_error)
      .def("error", &WatchdogSim::error)
      .def("failed", &WatchdogSim::failed)
      .def("pending", &WatchdogSim::pending)
      .def("aborts", &WatchdogSim::aborts)
      .def("drain", &WatchdogSim::drain, py::arg("max_s"), py::call_guard<py::gil_scoped_release>());
}

}  // namespace hypbind
