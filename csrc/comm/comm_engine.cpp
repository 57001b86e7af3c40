// Native gradient-communication engine: the MI355X replacement for Horovod's C++ core + NCCL
// (reference: hvd.DistributedOptimizer at scripts/train.py:114 and BroadcastGlobalVariablesCallback at
// scripts/train.py:133).
//
// * One RCCL communicator per process (one process per GPU), bootstrapped from an ncclUniqueId that
//   Python passes around through torch's TCPStore — no MPI, no per-step negotiation.
// * A dedicated high-priority HIP stream for collectives. Every collective is ordered after the work
//   already queued on the caller's (compute) stream by an event, so it overlaps with the backward
//   kernels queued after it; `wait_all` makes the compute stream wait for the collectives' events
//   (the host never blocks).
// * Static gradient buckets over ONE flat gradient buffer (the FlatParamStore's main_grad): the
//   backward kernels mark parameters ready in a deterministic order on every rank, so the engine
//   launches bucket b's in-place ncclAllReduce as soon as its last parameter is ready — the role of
//   Horovod's 64 MiB fusion buffer + coordinator, without the coordinator.
// * Optional wire compression (Horovod's hvd.Compression.fp16): a bucket is cast to a bf16 /
//   fp16 shadow on the comm stream, all-reduced in that type (half the xGMI bytes) and cast back into the fp32
//   gradient buffer, all on the comm stream.
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../kernels/launchers.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace hsd {
namespace {

bool dbg() {
  static bool d = getenv("HSD_COMM_DEBUG") != nullptr;
  return d;
}
#define DBG(...) do { if (dbg()) { fprintf(stderr, "[comm] " __VA_ARGS__); fflush(stderr); } } while (0)

#define HIP_OK(x)                                                                       \
  do {                                                                                  \
    hipError_t e__ = (x);                                                               \
    if (e__ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e__) + " at " #x); \
  } while (0)
#define NCCL_OK(x)                                                                      \
  do {                                                                                  \
    ncclResult_t r__ = (x);                                                             \
    if (r__ != ncclSuccess) throw std::runtime_error(std::string("RCCL: ") + ncclGetErrorString(r__) + " at " #x); \
  } while (0)

ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: throw std::runtime_error("CommEngine: unsupported dtype");
  }
}

struct Bucket {
  int64_t start = 0, end = 0;  // element range in the flat buffer
  int nparams = 0;
  int pending = 0;
  bool launched = false;
  hipEvent_t done = nullptr;
  hipEvent_t t_start = nullptr, t_end = nullptr;  // timing events (only with set_timing(true))
};

class CommEngine {
 public:
  CommEngine(int64_t rank, int64_t world, const std::string& uid, int64_t device, bool high_priority)
      : rank_((int)rank), world_((int)world), device_((int)device) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("CommEngine: bad unique id size");
    DBG("ctor rank %d world %d dev %d\n", rank_, world_, device_);
    HIP_OK(hipSetDevice(device_));
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, high_priority ? hi : lo));
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    DBG("stream ok, init comm\n");
    NCCL_OK(ncclCommInitRank(&comm_, world_, id, rank_));
    DBG("comm ok\n");
    HIP_OK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
  }

  ~CommEngine() { close_impl(false); }

  // Drain, then release the communicator (idempotent); the stream and events are left to process teardown (the
  // caching allocator may still hold blocks whose last use was recorded on this stream).
  // Captures: synchronising a stream that is itself being captured is illegal in EVERY capture mode, and the engine's
  // stream is part of a data-parallel whole-step capture once the capture forks it. close() therefore checks its own
  // stream first: inside such a capture it refuses (Python's close() raises; the destructor leaves the communicator to
  // process exit rather than corrupting the graph). When only ANOTHER stream of this thread captures (Python's cyclic
  // collector may run a finaliser in the middle of any capture; train/graph.py also turns it off there), syncing the
  // engine's own stream is legal in relaxed mode only, so the thread's mode is relaxed around the teardown.
  void close() { close_impl(true); }

  bool stream_capturing() const {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return stream_ != nullptr && hipStreamIsCapturing(stream_, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
  }

  void close_impl(bool strict) {
    if (comm_ == nullptr) return;
    if (stream_capturing()) {
      if (strict) {
        throw std::runtime_error("CommEngine.close(): the comm stream is being captured into a HIP graph; close the "
                                 "engine after the capture ends");
      }
      fprintf(stderr, "CommEngine: destroyed while its stream is captured; the communicator is left to process exit\n");
      comm_ = nullptr;
      return;
    }
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    const bool swapped = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
    if (stream_) (void)hipStreamSynchronize(stream_);
    (void)ncclCommDestroy(comm_);
    comm_ = nullptr;  // collectives after close() fail in RCCL (invalid communicator)
    if (swapped) (void)hipThreadExchangeStreamCaptureMode(&mode);
  }

  static std::string unique_id() {
    ncclUniqueId id;
    NCCL_OK(ncclGetUniqueId(&id));
    return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
  }

  int64_t rank() const { return rank_; }
  // the comm stream (the optimizer steps each bucket on it right after the bucket's all-reduce)
  int64_t stream_ptr() const { return reinterpret_cast<int64_t>(stream_); }
  int64_t world() const { return world_; }

  // ---------------------------------------------------------------- one-shot collectives
  // in-place all-reduce SUM of `t` ordered after the caller's stream; with `wait` the caller's stream waits
  // for it before any later work (otherwise call wait_all() before `t` is read or freed).
  void allreduce(torch::Tensor t, bool wait) {
    check(t);
    DBG("allreduce n=%ld\n", (long)t.numel());
    order_after_caller();
    DBG("ordered\n");
    NCCL_OK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), to_nccl(t.scalar_type()), ncclSum, comm_,
                          stream_));
    DBG("launched\n");
    if (!wait) record_stream(t);
    hipEvent_t e = make_event();
    HIP_OK(hipEventRecord(e, stream_));
    if (wait) HIP_OK(hipStreamWaitEvent(caller(), e, 0));
  }

  void broadcast(torch::Tensor t, int64_t root) {
    check(t);
    order_after_caller();
    NCCL_OK(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), to_nccl(t.scalar_type()), (int)root, comm_,
                          stream_));
    hipEvent_t e = make_event();
    HIP_OK(hipEventRecord(e, stream_));
    HIP_OK(hipStreamWaitEvent(caller(), e, 0));
  }

  // ---------------------------------------------------------------- gradient buckets
  // flat: the gradient buffer; ranges: [start, end) element ranges; counts: parameters per bucket;
  // param_bucket[i] = bucket of parameter i.
  void set_buckets(torch::Tensor flat, std::vector<int64_t> starts, std::vector<int64_t> ends,
                   std::vector<int64_t> counts, std::vector<int64_t> param_bucket) {
    check(flat);
    if (starts.size() != ends.size() || starts.size() != counts.size())
      throw std::runtime_error("set_buckets: size mismatch");
    for (auto& b : buckets_) {
      if (b.done) (void)hipEventDestroy(b.done);
      if (b.t_start) (void)hipEventDestroy(b.t_start);
      if (b.t_end) (void)hipEventDestroy(b.t_end);
    }
    buckets_.clear();
    flat_ = flat;
    for (size_t i = 0; i < starts.size(); ++i) {
      Bucket b;
      b.start = starts[i];
      b.end = ends[i];
      b.nparams = (int)counts[i];
      if (b.start < 0 || b.end > flat.numel() || b.start > b.end) throw std::runtime_error("set_buckets: bad range");
      HIP_OK(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
      HIP_OK(hipEventCreate(&b.t_start));
      HIP_OK(hipEventCreate(&b.t_end));
      buckets_.push_back(b);
    }
    param_bucket_.assign(param_bucket.begin(), param_bucket.end());
    begin_step();
  }

  // 0 = none (all-reduce the gradient buffer in place), 1 = bf16 on the wire, 2 = fp16 on the wire
  void set_compression(int64_t mode) {
    if (mode < 0 || mode > 2) throw std::runtime_error("set_compression: mode 0 (none), 1 (bf16) or 2 (fp16)");
    if (mode != 0) {
      if (!flat_.defined()) throw std::runtime_error("set_compression: call set_buckets first");
      for (auto& b : buckets_)  // the 16-B vectorised casts (launch_wire_cast)
        if (b.start % 4 || b.end % 4) throw std::runtime_error("set_compression: bucket ranges must be multiples of 4");
    }
    comp_ = (int)mode;
    if (comp_ != 0) {
      const auto dt = comp_ == 1 ? at::kBFloat16 : at::kHalf;
      if (!shadow_.defined() || shadow_.numel() != flat_.numel() || shadow_.scalar_type() != dt)
        shadow_ = at::empty({flat_.numel()}, flat_.options().dtype(dt));
    }
  }

  // fp16 wire pre-scale for the coming step(s): 1 / gradient-accumulation micro-steps
  void set_prescale(double s) { prescale_ = s > 0.0 ? s : 1.0; }

  void begin_step() {
    for (auto& b : buckets_) {
      b.pending = b.nparams;
      b.launched = false;
    }
    if (timing_) HIP_OK(hipEventRecord(t_begin_, caller()));
  }

  // ---------------------------------------------------------------- overlap timeline
  // With timing on, a step records: t_begin on the compute stream at begin_step, per-bucket start/end
  // around each ncclAllReduce on the comm stream, and t_bwd_end on the compute stream when finish() is
  // called (= every backward kernel queued). Off by default: timing events cost a little per record.
  void set_timing(bool on) {
    if (on && !t_begin_) {
      HIP_OK(hipEventCreate(&t_begin_));
      HIP_OK(hipEventCreate(&t_bwd_end_));
    }
    timing_ = on;
  }

  // {backward_end_ms, [bucket start_ms, end_ms, bytes]...} relative to begin_step of the last timed step
  // (blocks the host until the last bucket has finished; call after the step).
  std::vector<double> timings() {
    if (!timing_ || buckets_.empty()) return {};
    for (auto& b : buckets_)
      if (!b.launched) throw std::runtime_error("timings: step not finished");
    HIP_OK(hipStreamSynchronize(stream_));
    HIP_OK(hipEventSynchronize(t_bwd_end_));
    std::vector<double> out;
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, t_begin_, t_bwd_end_));
    out.push_back(ms);
    for (auto& b : buckets_) {
      float a = 0.f, e = 0.f;
      HIP_OK(hipEventElapsedTime(&a, t_begin_, b.t_start));
      HIP_OK(hipEventElapsedTime(&e, t_begin_, b.t_end));
      out.push_back(a);
      out.push_back(e);
      out.push_back((double)(b.end - b.start) * flat_.element_size());
    }
    return out;
  }

  // a parameter's gradient is complete (its producing kernels are queued on the caller's stream)
  // returns the bucket index launched, or -1
  int64_t mark_ready(int64_t param) {
    if (param < 0 || (size_t)param >= param_bucket_.size()) throw std::runtime_error("mark_ready: bad index");
    Bucket& b = buckets_[param_bucket_[param]];
    if (b.launched) throw std::runtime_error("mark_ready: gradient arrived after its bucket was reduced");
    if (--b.pending == 0) {
      launch(b);
      return param_bucket_[param];
    }
    return -1;
  }

  // launch every bucket not launched yet (unused parameters), then order the caller's stream after
  // all bucket reductions
  void finish() {
    if (timing_) HIP_OK(hipEventRecord(t_bwd_end_, caller()));
    for (auto& b : buckets_)
      if (!b.launched) launch(b);
    for (auto& b : buckets_) HIP_OK(hipStreamWaitEvent(caller(), b.done, 0));
  }

  void wait_all() {
    HIP_OK(hipEventRecord(ready_, stream_));
    HIP_OK(hipStreamWaitEvent(caller(), ready_, 0));
  }

  // every collective is also ordered after the work queued on this stream (e.g. the wgrad side stream)
  void add_dependency_stream(int64_t stream_ptr) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_ptr);
    for (auto d : deps_)
      if (d == s) return;
    hipEvent_t e;
    HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    deps_.push_back(s);
    dep_events_.push_back(e);
  }

  // 0 = the current stream (default); otherwise every caller-side event record / wait uses this stream (a HIP-graph
  // capture). A new caller stream starts with its dependency streams outside the capture (see set_capture_deps).
  void set_caller_stream(int64_t stream_ptr) {
    caller_override_ = reinterpret_cast<hipStream_t>(stream_ptr);
    capture_deps_ = false;
  }

  // Inside a capture: whether the registered dependency streams are branches of it now (the capture forked the wgrad
  // side stream: ops/hip.py side_stream_in_capture). From then on every bucket is ordered after them as in eager
  // steps; before the fork they hold no captured work, and an event of an uncaptured stream is no capture edge.
  void set_capture_deps(bool on) { capture_deps_ = on; }

  int64_t num_buckets() const { return (int64_t)buckets_.size(); }
  int64_t launched_count() const {
    int64_t n = 0;
    for (auto& b : buckets_) n += b.launched ? 1 : 0;
    return n;
  }

 private:
  // the stream the gradients are produced on: the thread's current stream, or the stream set by set_caller_stream
  // (a HIP-graph capture: readiness hooks run on autograd's thread, whose current stream is not the capture stream)
  hipStream_t caller() const {
    return caller_override_ ? caller_override_ : c10::hip::getCurrentHIPStream(device_).stream();
  }

  void check(const torch::Tensor& t) const {
    if (!t.is_cuda() || t.get_device() != device_) throw std::runtime_error("CommEngine: tensor on the wrong device");
    if (!t.is_contiguous()) throw std::runtime_error("CommEngine: tensor must be contiguous");
  }

  void order_after_caller() {
    HIP_OK(hipEventRecord(ready_, caller()));
    HIP_OK(hipStreamWaitEvent(stream_, ready_, 0));
    // gradients may also be produced on registered side streams (the wgrad stream): order after them too. Inside a
    // capture (set_caller_stream) only once the capture has forked them (set_capture_deps): the wgrad branch writes
    // the same main_grad slices this bucket's all-reduce and Adam slice read
    if (caller_override_ && !capture_deps_) return;
    for (size_t i = 0; i < deps_.size(); ++i) {
      HIP_OK(hipEventRecord(dep_events_[i], deps_[i]));
      HIP_OK(hipStreamWaitEvent(stream_, dep_events_[i], 0));
    }
  }

  void record_stream(const torch::Tensor& t) {
    c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(),
                                                c10::hip::getStreamFromExternal(stream_, device_));
  }

  hipEvent_t make_event() {
    // small ring of reusable events for one-shot collectives
    if (extra_.size() < 16) {
      hipEvent_t e;
      HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      extra_.push_back(e);
      return e;
    }
    hipEvent_t e = extra_[next_extra_];
    next_extra_ = (next_extra_ + 1) % extra_.size();
    return e;
  }

  void launch(Bucket& b) {
    order_after_caller();
    const int64_t n = b.end - b.start;
    if (timing_) HIP_OK(hipEventRecord(b.t_start, stream_));
    if (n > 0 && comp_ != 0 && flat_.scalar_type() == at::kFloat) {
      // cast -> all-reduce in 16 bits -> cast back, all ordered on the comm stream
      // one fused HIP pass each way (elementwise.hip launch_wire_cast). fp16 on the wire: pre-scaled by 1/micro-steps
      // so the rank SUM of k accumulated micro-steps stays inside fp16's range (65504), scaled back in fp32 after
      // the all-reduce (exact for powers of two); the 1/world average stays in the optimizer's fp32 grad_scale
      float* src = flat_.data_ptr<float>() + b.start;
      void* wire = static_cast<char*>(shadow_.data_ptr()) + b.start * shadow_.element_size();
      const bool half = comp_ == 2;
      const float pre = half ? (float)prescale_ : 1.0f;
      launch_wire_cast(src, wire, n, true, half, pre, stream_);
      NCCL_OK(ncclAllReduce(wire, wire, (size_t)n, to_nccl(shadow_.scalar_type()), ncclSum, comm_, stream_));
      launch_wire_cast(wire, src, n, false, half, 1.0f / pre, stream_);
    } else if (n > 0) {
      char* base = static_cast<char*>(flat_.data_ptr()) + b.start * flat_.element_size();
      NCCL_OK(ncclAllReduce(base, base, (size_t)n, to_nccl(flat_.scalar_type()), ncclSum, comm_, stream_));
    }
    if (timing_) HIP_OK(hipEventRecord(b.t_end, stream_));
    HIP_OK(hipEventRecord(b.done, stream_));
    b.launched = true;
  }

  int rank_, world_, device_;
  hipStream_t stream_ = nullptr;
  hipStream_t caller_override_ = nullptr;
  bool capture_deps_ = false;
  ncclComm_t comm_ = nullptr;
  hipEvent_t ready_ = nullptr;
  bool timing_ = false;
  hipEvent_t t_begin_ = nullptr, t_bwd_end_ = nullptr;
  std::vector<hipEvent_t> extra_;
  size_t next_extra_ = 0;
  std::vector<Bucket> buckets_;
  std::vector<int64_t> param_bucket_;
  std::vector<hipStream_t> deps_;
  std::vector<hipEvent_t> dep_events_;
  torch::Tensor flat_;
  torch::Tensor shadow_;
  int comp_ = 0;
  double prescale_ = 1.0;
};

}  // namespace

void register_comm(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<CommEngine>(m, "CommEngine")
      .def(py::init([](int64_t rank, int64_t world, py::bytes uid, int64_t device, bool high_priority) {
             return new CommEngine(rank, world, std::string(uid), device, high_priority);
           }),
           py::arg("rank"), py::arg("world"), py::arg("uid"), py::arg("device"), py::arg("high_priority") = true)
      .def_static("unique_id", []() { return py::bytes(CommEngine::unique_id()); })
      .def("allreduce", &CommEngine::allreduce, py::arg("t"), py::arg("wait") = true)
      .def("broadcast", &CommEngine::broadcast, py::arg("t"), py::arg("root") = 0)
      .def("set_buckets", &CommEngine::set_buckets)
      .def("set_compression", &CommEngine::set_compression)
      .def("set_prescale", &CommEngine::set_prescale)
      .def("begin_step", &CommEngine::begin_step)
      .def("set_timing", &CommEngine::set_timing)
      .def("timings", &CommEngine::timings)
      .def("mark_ready", &CommEngine::mark_ready)
      .def("finish", &CommEngine::finish)
      .def("wait_all", &CommEngine::wait_all)
      .def("add_dependency_stream", &CommEngine::add_dependency_stream)
      .def("num_buckets", &CommEngine::num_buckets)
      .def("launched_count", &CommEngine::launched_count)
      .def("stream_ptr", &CommEngine::stream_ptr)
      .def("set_caller_stream", &CommEngine::set_caller_stream)
      .def("set_capture_deps", &CommEngine::set_capture_deps)
      .def("close", &CommEngine::close)
      .def_property_readonly("rank", &CommEngine::rank)
      .def_property_readonly("world", &CommEngine::world);
}

}  // namespace hsd
