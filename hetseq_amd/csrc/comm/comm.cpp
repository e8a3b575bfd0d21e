// Native gradient-communication engine over RCCL.
//
// Reference: the data-parallel gradient exchange is torch DDP's C++ reducer over NCCL
// (controller.py:74-89 wrapping the model, all-reduce hooks fired from loss.backward()
// at optim.py:55-57), with the fast-stat all-reduce issued by c10d (controller.py:294-296).
//
// MI355X design.  One RCCL communicator per data-parallel group, created from a unique id
// that rank 0 publishes through the job's rendezvous (the Python facade), with
//  * a dedicated comm stream at the device's GREATEST priority: the hardware queue of the
//    collectives is scheduled ahead of the GEMM queues, so a bucket's ring kernels start
//    as soon as its gradients exist instead of queueing behind a 700-block GEMM wave;
//  * bucket all-reduces gated by hipEvents recorded on every producer stream (the compute
//    stream and the weight-gradient stream), in place on slices of the flat gradient buffer
//    -- no copies, no host synchronisation;
//  * a consumer-side join (`wait`): the compute stream waits for the comm stream's last
//    event before the optimizer reads the gradients;
//  * a watchdog thread: it polls the outstanding events and the communicator's async error
//    state; an operation older than the collective timeout (a dead or desynchronised peer)
//    or an RCCL error aborts the communicator, so the stuck kernels exit and the next call
//    from Python raises instead of hanging the job (`check`).
// Small collectives (fast-stat vector, parameter broadcast, consistency checksums) run
// in-stream on the caller's stream through the same communicator.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("hetseq comm: ") + what + ": " + hipGetErrorString(e));
}

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("hetseq comm: ") + what + ": " + ncclGetErrorString(r));
}

ncclDataType_t nccl_type(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat64;
    case 3: return ncclInt64;
    case 4: return ncclUint8;
    case 5: return ncclInt32;
  }
  throw std::invalid_argument("hetseq comm: unsupported dtype code");
}

ncclRedOp_t nccl_op(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclMin;
    case 2: return ncclMax;
  }
  throw std::invalid_argument("hetseq comm: unsupported reduction");
}

hipStream_t as_stream(uintptr_t h) { return reinterpret_cast<hipStream_t>(h); }

// Emulated collectives (bench.py --emulate-world): the stand-in kernel of the HIP module
// (csrc/kernels/comm_emul.hip, hetseq_comm_emulation), reached through its address.
typedef void (*EmulFn)(const void* src, int64_t src_bytes, void* scratch, int64_t scratch_bytes, int64_t traffic_bytes,
                       int channels, int64_t hold_ns, hipStream_t st);

size_t elem_size(int code) {
  switch (code) {
    case 0: return 4;
    case 1: return 2;
    case 2: return 8;
    case 3: return 8;
    case 4: return 1;
    case 5: return 4;
  }
  throw std::invalid_argument("hetseq comm: unsupported dtype code");
}

class Comm {
 public:
  // Two-phase construction: the local part (device, comm stream) here, the blocking rendezvous in
  // init() -- so every rank can report a local failure (parallel/comm.py create(), round 1) before
  // any rank enters ncclCommInitRank, which waits for all of them.
  Comm(int nranks, int rank, int device, double timeout_s)
      : nranks_(nranks), rank_(rank), device_(device), timeout_(timeout_s) {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    int least = 0, greatest = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest), "hipStreamCreateWithPriority");
  }
  Comm(py::bytes uid, int nranks, int rank, int device, double timeout_s) : Comm(nranks, rank, device, timeout_s) {
    init(uid);
  }

  void init(py::bytes uid) {
    if (comm_) throw std::logic_error("hetseq comm: init called twice");
    std::string u = uid;
    if (u.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("hetseq comm: bad unique id size");
    ncclUniqueId id;
    std::memcpy(&id, u.data(), sizeof(id));
    hip_check(hipSetDevice(device_), "hipSetDevice");
    {
      py::gil_scoped_release nogil;  // a blocking rendezvous among the ranks
      nccl_check(ncclCommInitRank(&comm_, nranks_, id, rank_), "ncclCommInitRank");
    }
    watchdog_ = std::thread([this] { watch(); });
  }

  ~Comm() { close(false); }

  // What RCCL itself reports for this communicator (ncclCommCount / ncclCommUserRank /
  // ncclCommCuDevice) and the PCI bus id of the HIP device it runs on: bench.py records these per
  // rank, so a multi-GPU result carries proof of N ranks on N distinct devices.
  py::dict identity() {
    if (!comm_) throw std::logic_error("hetseq comm: identity before init");
    int count = 0, user_rank = -1, dev = -1;
    nccl_check(ncclCommCount(comm_, &count), "ncclCommCount");
    nccl_check(ncclCommUserRank(comm_, &user_rank), "ncclCommUserRank");
    nccl_check(ncclCommCuDevice(comm_, &dev), "ncclCommCuDevice");
    char bus[64] = {0};
    hip_check(hipDeviceGetPCIBusId(bus, sizeof(bus), dev), "hipDeviceGetPCIBusId");
    py::dict d;
    d["rccl_count"] = count;
    d["rccl_rank"] = user_rank;
    d["rccl_device"] = dev;
    d["pci_bus_id"] = std::string(bus);
    return d;
  }

  // graceful: destroy the communicator when every operation has completed (all ranks close at
  // the same point); otherwise -- operations still outstanding (a peer died) or process exit --
  // abort it, which never waits for peers.
  void close(bool graceful) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (closed_.load()) return;
      closed_.store(true);
    }
    cv_.notify_all();
    if (watchdog_.joinable()) watchdog_.join();
    if (comm_) {
      if (!aborted_.load()) {  // (an aborted communicator was freed by ncclCommAbort)
        hipSetDevice(device_);
        bool done = true;
        for (auto& p : pending_) done = done && !p.stalled && hipEventQuery(p.ev) == hipSuccess;
        if (graceful && done) {
          hipStreamSynchronize(stream_);
          ncclCommDestroy(comm_);
        } else {
          ncclCommAbort(comm_);
        }
      }
      comm_ = nullptr;
    }
    for (hipEvent_t e : free_) hipEventDestroy(e);
    for (auto& p : pending_) hipEventDestroy(p.ev);
    free_.clear();
    pending_.clear();
    if (stream_) hipStreamDestroy(stream_);
    stream_ = nullptr;
  }

  // In-place all-reduce of [ptr, ptr + count) on the comm stream after every producer stream's
  // work enqueued so far.  Returns immediately.
  void all_reduce_async(uintptr_t ptr, int64_t count, int dtype, int op, std::vector<uintptr_t> producers) {
    check();
    for (uintptr_t s : producers) {
      hipEvent_t e = take_event();
      hip_check(hipEventRecord(e, as_stream(s)), "hipEventRecord(producer)");
      hip_check(hipStreamWaitEvent(stream_, e, 0), "hipStreamWaitEvent(comm)");
      give_event(e);  // recorded + waited: reusable once the comm stream passes it (ordered)
    }
    void* p = reinterpret_cast<void*>(ptr);
    if (emul_) {  // W-rank prediction: ring all-reduce, each rank receives 2(W-1)/W of the bucket
      const int64_t bytes = count * (int64_t)elem_size(dtype);
      emulate(p, bytes, 2 * (emul_world_ - 1) * bytes / emul_world_, stream_);
      return;
    }
    if (snap_dst_) {
      // test mode: copy the bucket as it stands when the collective would read it (the copy is
      // ordered exactly like the all-reduce: on the comm stream, behind the producer events)
      if (ptr < snap_src_ || ptr + (uintptr_t)count * elem_size(dtype) > snap_src_ + snap_bytes_)
        throw std::invalid_argument("hetseq comm: snapshot range outside the registered buffer");
      hip_check(hipMemcpyAsync(reinterpret_cast<void*>(snap_dst_ + (ptr - snap_src_)), p,
                               (size_t)count * elem_size(dtype), hipMemcpyDeviceToDevice, stream_),
                "hipMemcpyAsync(snapshot)");
      track(stream_);
      return;
    }
    {
      std::lock_guard<std::mutex> g(op_mu_);
      check();
      nccl_check(ncclAllReduce(p, p, (size_t)count, nccl_type(dtype), nccl_op(op), comm_, stream_), "ncclAllReduce");
    }
    track(stream_);
  }

  // All-gather of `count` elements per rank into `recv` on the comm stream, ordered after the
  // work enqueued so far on every producer stream (the tied-embedding key / row exchange).
  void all_gather_async(uintptr_t send, uintptr_t recv, int64_t count, int dtype, std::vector<uintptr_t> producers) {
    check();
    for (uintptr_t s : producers) {
      hipEvent_t e = take_event();
      hip_check(hipEventRecord(e, as_stream(s)), "hipEventRecord(producer)");
      hip_check(hipStreamWaitEvent(stream_, e, 0), "hipStreamWaitEvent(comm)");
      give_event(e);
    }
    {
      std::lock_guard<std::mutex> g(op_mu_);
      check();
      nccl_check(ncclAllGather(reinterpret_cast<void*>(send), reinterpret_cast<void*>(recv), (size_t)count,
                               nccl_type(dtype), comm_, stream_),
                 "ncclAllGather");
    }
    track(stream_);
    if (emul_) {  // after the real (1-rank) gather: the other W-1 ranks' rows over the links
      const int64_t bytes = count * (int64_t)elem_size(dtype);
      emulate(reinterpret_cast<void*>(send), bytes, (emul_world_ - 1) * bytes, stream_);
    }
  }

  // The comm stream waits for raw events the caller recorded (a fused backward's per-group
  // readiness, ops/layer_prog.py): the next collective is ordered after exactly that work.
  void wait_events(const std::vector<uintptr_t>& events) {
    check();
    for (uintptr_t e : events)
      hip_check(hipStreamWaitEvent(stream_, reinterpret_cast<hipEvent_t>(e), 0), "hipStreamWaitEvent(events)");
  }

  // Sharded update (parallel/zero.py): in-place reduce-scatter of [ptr, ptr + total) -- rank r keeps
  // the sum of piece r, [ptr + r total / n, ...) -- on the comm stream after every producer stream's work
  // so far; and the in-place all-gather of the updated pieces (each rank's piece r to every rank).
  // `total` is a multiple of the rank count.  Emulated: the bytes one rank of the ring receives,
  // (W-1)/W of the region either way.
  void reduce_scatter_async(uintptr_t ptr, int64_t total, int dtype, int op, std::vector<uintptr_t> producers) {
    check();
    order_after(producers);
    const int64_t bytes = total * (int64_t)elem_size(dtype);
    if (emul_) {
      emulate(reinterpret_cast<void*>(ptr), bytes, (emul_world_ - 1) * bytes / emul_world_, stream_);
      return;
    }
    if (snap_dst_) {  // test mode, as all_reduce_async: the region as the collective would read it
      if (ptr < snap_src_ || ptr + (uintptr_t)bytes > snap_src_ + snap_bytes_)
        throw std::invalid_argument("hetseq comm: snapshot range outside the registered buffer");
      hip_check(hipMemcpyAsync(reinterpret_cast<void*>(snap_dst_ + (ptr - snap_src_)), reinterpret_cast<void*>(ptr),
                               (size_t)bytes, hipMemcpyDeviceToDevice, stream_),
                "hipMemcpyAsync(snapshot)");
      track(stream_);
      return;
    }
    if (total % nranks_) throw std::invalid_argument("hetseq comm: reduce-scatter region not divisible by ranks");
    const int64_t count = total / nranks_;
    char* base = reinterpret_cast<char*>(ptr);
    {
      std::lock_guard<std::mutex> g(op_mu_);
      check();
      nccl_check(ncclReduceScatter(base, base + (int64_t)rank_ * count * (int64_t)elem_size(dtype), (size_t)count,
                                   nccl_type(dtype), nccl_op(op), comm_, stream_),
                 "ncclReduceScatter");
    }
    track(stream_);
  }

  void all_gather_inplace_async(uintptr_t ptr, int64_t total, int dtype, std::vector<uintptr_t> producers) {
    check();
    order_after(producers);
    const int64_t bytes = total * (int64_t)elem_size(dtype);
    if (emul_) {
      emulate(reinterpret_cast<void*>(ptr), bytes, (emul_world_ - 1) * bytes / emul_world_, stream_);
      return;
    }
    if (total % nranks_) throw std::invalid_argument("hetseq comm: all-gather region not divisible by ranks");
    const int64_t count = total / nranks_;
    char* base = reinterpret_cast<char*>(ptr);
    {
      std::lock_guard<std::mutex> g(op_mu_);
      check();
      nccl_check(ncclAllGather(base + (int64_t)rank_ * count * (int64_t)elem_size(dtype), base, (size_t)count,
                               nccl_type(dtype), comm_, stream_),
                 "ncclAllGather");
    }
    track(stream_);
  }

  // Emulation mode (1-rank communicator only): every bucket all-reduce / all-gather on the comm
  // stream becomes the stand-in kernel -- `channels` workgroups moving the bytes a rank of a
  // `world`-rank ring receives and staying resident for latency + bytes / busbw.  world <= 1 ends it.
  void set_emulation(uintptr_t fn, int world, int channels, double busbw_gbs, double latency_us, uintptr_t scratch,
                     int64_t scratch_bytes) {
    if (world > 1 && nranks_ != 1) throw std::invalid_argument("hetseq comm: emulation needs a 1-rank communicator");
    if (world > 1 && (!fn || !scratch || scratch_bytes < 16 || channels < 1 || busbw_gbs <= 0))
      throw std::invalid_argument("hetseq comm: bad emulation parameters");
    emul_ = world > 1 ? reinterpret_cast<EmulFn>(fn) : nullptr;
    emul_world_ = world;
    emul_channels_ = channels;
    emul_busbw_ = busbw_gbs;
    emul_lat_us_ = latency_us;
    emul_scratch_ = scratch;
    emul_scratch_bytes_ = scratch_bytes;
  }

  // Test hook (single-GPU ordering check): while set, all_reduce_async copies each bucket of
  // [src, src + bytes) into the same offset of `dst` on the comm stream instead of reducing it.
  void set_snapshot(uintptr_t dst, uintptr_t src, int64_t bytes) {
    snap_dst_ = dst;
    snap_src_ = src;
    snap_bytes_ = (uintptr_t)bytes;
  }

  // The consumer stream waits for every collective issued on the comm stream so far.
  void wait(uintptr_t consumer) {
    check();
    hipEvent_t e = take_event();
    hip_check(hipEventRecord(e, stream_), "hipEventRecord(comm)");
    hip_check(hipStreamWaitEvent(as_stream(consumer), e, 0), "hipStreamWaitEvent(consumer)");
    give_event(e);
  }

  // In-stream collectives on the caller's stream (small / one-off transfers).
  void all_reduce(uintptr_t ptr, int64_t count, int dtype, int op, uintptr_t stream) {
    check();
    void* p = reinterpret_cast<void*>(ptr);
    if (emul_) {  // (the fast-stat vector: latency-bound at W ranks)
      const int64_t bytes = count * (int64_t)elem_size(dtype);
      emulate(p, bytes, 2 * (emul_world_ - 1) * bytes / emul_world_, as_stream(stream));
      return;
    }
    {
      std::lock_guard<std::mutex> g(op_mu_);
      check();
      nccl_check(ncclAllReduce(p, p, (size_t)count, nccl_type(dtype), nccl_op(op), comm_, as_stream(stream)),
                 "ncclAllReduce");
    }
    track(as_stream(stream));
  }

  void broadcast(uintptr_t ptr, int64_t count, int dtype, int root, uintptr_t stream) {
    check();
    void* p = reinterpret_cast<void*>(ptr);
    {
      std::lock_guard<std::mutex> g(op_mu_);
      check();
      nccl_check(ncclBroadcast(p, p, (size_t)count, nccl_type(dtype), root, comm_, as_stream(stream)),
                 "ncclBroadcast");
    }
    track(as_stream(stream));
  }

  void all_gather(uintptr_t send, uintptr_t recv, int64_t count, int dtype, uintptr_t stream) {
    {
      std::lock_guard<std::mutex> g(op_mu_);
      check();
      nccl_check(ncclAllGather(reinterpret_cast<void*>(send), reinterpret_cast<void*>(recv), (size_t)count,
                               nccl_type(dtype), comm_, as_stream(stream)),
                 "ncclAllGather");
    }
    track(as_stream(stream));
  }

  // The watchdog also covers the work enqueued on `stream` so far (a replayed HIP graph whose
  // collectives were captured: their completion is the replay's).
  void watch_stream(uintptr_t stream) {
    check();
    track(as_stream(stream));
  }

  // Raises if the watchdog aborted the communicator (timeout / async RCCL error).
  void check() {
    if (aborted_.load()) {
      std::lock_guard<std::mutex> g(mu_);
      throw std::runtime_error("hetseq comm: communicator aborted: " + error_);
    }
    if (closed_.load()) throw std::runtime_error("hetseq comm: communicator closed");
  }

  // Test hook: makes the watchdog treat the next `n` operations as stuck (fault injection).
  void inject_stall(int n) { stall_.store(n); }

  int outstanding() {
    std::lock_guard<std::mutex> g(mu_);
    return (int)pending_.size();
  }

  uintptr_t stream() const { return reinterpret_cast<uintptr_t>(stream_); }
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  bool aborted() const { return aborted_.load(); }

 private:
  uintptr_t snap_dst_ = 0, snap_src_ = 0, snap_bytes_ = 0;
  EmulFn emul_ = nullptr;
  int emul_world_ = 1, emul_channels_ = 1;
  double emul_busbw_ = 1.0, emul_lat_us_ = 0.0;
  uintptr_t emul_scratch_ = 0;
  int64_t emul_scratch_bytes_ = 0;

  void emulate(void* src, int64_t src_bytes, int64_t traffic, hipStream_t s) {
    const double ns = emul_lat_us_ * 1e3 + (double)traffic / emul_busbw_;  // bytes / (GB/s) = ns
    emul_(src, src_bytes, reinterpret_cast<void*>(emul_scratch_), emul_scratch_bytes_, traffic, emul_channels_,
          (int64_t)ns, s);
    hip_check(hipGetLastError(), "comm emulation kernel launch");
    track(s);
  }

  void order_after(const std::vector<uintptr_t>& producers) {
    for (uintptr_t s : producers) {
      hipEvent_t e = take_event();
      hip_check(hipEventRecord(e, as_stream(s)), "hipEventRecord(producer)");
      hip_check(hipStreamWaitEvent(stream_, e, 0), "hipStreamWaitEvent(comm)");
      give_event(e);
    }
  }

  struct Pending {
    hipEvent_t ev;
    std::chrono::steady_clock::time_point t0;
    bool stalled;
  };

  hipEvent_t take_event() {
    std::lock_guard<std::mutex> g(mu_);
    if (!free_.empty()) {
      hipEvent_t e = free_.back();
      free_.pop_back();
      return e;
    }
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
  }

  void give_event(hipEvent_t e) {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(e);
  }

  // completion event of the collective just enqueued on `s`, watched by the watchdog.  Not while
  // `s` is being captured into a HIP graph: an event recorded there never completes outside the
  // graph (the replay is watched instead: watch_stream() after each launch).
  void track(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hip_check(hipStreamIsCapturing(s, &cs), "hipStreamIsCapturing");
    if (cs != hipStreamCaptureStatusNone) return;
    hipEvent_t e = take_event();
    hip_check(hipEventRecord(e, s), "hipEventRecord(done)");
    bool stalled = false;
    int n = stall_.load();
    if (n > 0) {
      stall_.store(n - 1);
      stalled = true;
    }
    std::lock_guard<std::mutex> g(mu_);
    pending_.push_back({e, std::chrono::steady_clock::now(), stalled});
  }

  void fail(const std::string& why) {
    std::lock_guard<std::mutex> op(op_mu_);
    {
      std::lock_guard<std::mutex> g(mu_);
      if (aborted_.load()) return;
      error_ = why;
    }
    aborted_.store(true);
    ncclCommAbort(comm_);  // stuck ring kernels exit; the communicator is freed, never used again
  }

  void watch() {
    hipSetDevice(device_);
    std::unique_lock<std::mutex> lk(mu_);
    while (!closed_.load()) {
      cv_.wait_for(lk, std::chrono::milliseconds(20));
      if (closed_.load() || aborted_.load()) break;
      const auto now = std::chrono::steady_clock::now();
      std::string why;
      while (!pending_.empty()) {
        Pending& p = pending_.front();
        if (!p.stalled && hipEventQuery(p.ev) == hipSuccess) {
          free_.push_back(p.ev);
          pending_.pop_front();
          continue;
        }
        const double age = std::chrono::duration<double>(now - p.t0).count();
        if (age > timeout_)
          why = p.stalled ? "collective stalled (injected fault)" : "collective timed out after " + std::to_string(age) + " s";
        break;
      }
      if (why.empty()) {
        ncclResult_t async = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &async) == ncclSuccess && async != ncclSuccess)
          why = std::string("async RCCL error: ") + ncclGetErrorString(async);
      }
      if (!why.empty()) {
        lk.unlock();
        fail(why);
        lk.lock();
      }
    }
  }

  int nranks_, rank_, device_;
  double timeout_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Pending> pending_;
  std::vector<hipEvent_t> free_;
  std::thread watchdog_;
  std::atomic<bool> aborted_{false};
  std::atomic<int> stall_{0};
  std::atomic<bool> closed_{false};
  std::mutex op_mu_;  // enqueue calls vs the watchdog's abort (which frees the communicator)
  std::string error_;
};

py::bytes unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

int rccl_version() {
  int v = 0;
  nccl_check(ncclGetVersion(&v), "ncclGetVersion");
  return v;
}

}  // namespace

PYBIND11_MODULE(_comm, m) {
  m.doc() = "hetseq_amd native RCCL communication engine";
  m.def("unique_id", &unique_id);
  m.def("rccl_version", &rccl_version);
  py::class_<Comm>(m, "Comm")
      .def(py::init<py::bytes, int, int, int, double>(), py::arg("uid"), py::arg("nranks"), py::arg("rank"),
           py::arg("device"), py::arg("timeout_s"))
      .def(py::init<int, int, int, double>(), py::arg("nranks"), py::arg("rank"), py::arg("device"),
           py::arg("timeout_s"))
      .def("init", &Comm::init, py::arg("uid"), "the blocking RCCL rendezvous of a two-phase construction")
      .def("all_reduce_async", &Comm::all_reduce_async, py::arg("ptr"), py::arg("count"), py::arg("dtype"),
           py::arg("op"), py::arg("producers"))
      .def("all_gather_async", &Comm::all_gather_async, py::arg("send"), py::arg("recv"), py::arg("count"),
           py::arg("dtype"), py::arg("producers"))
      .def("wait_events", &Comm::wait_events, py::arg("events"))
      .def("reduce_scatter_async", &Comm::reduce_scatter_async, py::arg("ptr"), py::arg("total"), py::arg("dtype"),
           py::arg("op"), py::arg("producers"))
      .def("all_gather_inplace_async", &Comm::all_gather_inplace_async, py::arg("ptr"), py::arg("total"),
           py::arg("dtype"), py::arg("producers"))
      .def("wait", &Comm::wait, py::arg("consumer"))
      .def("all_reduce", &Comm::all_reduce, py::arg("ptr"), py::arg("count"), py::arg("dtype"), py::arg("op"),
           py::arg("stream"))
      .def("broadcast", &Comm::broadcast, py::arg("ptr"), py::arg("count"), py::arg("dtype"), py::arg("root"),
           py::arg("stream"))
      .def("all_gather", &Comm::all_gather, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
           py::arg("stream"))
      .def("check", &Comm::check)
      .def("identity", &Comm::identity, "RCCL's own count / rank / device and the device's PCI bus id")
      .def("watch_stream", &Comm::watch_stream, py::arg("stream"))
      .def("close", &Comm::close, py::arg("graceful") = true)
      .def("inject_stall", &Comm::inject_stall)
      .def("set_snapshot", &Comm::set_snapshot, py::arg("dst"), py::arg("src"), py::arg("bytes"))
      .def("set_emulation", &Comm::set_emulation, py::arg("fn"), py::arg("world"), py::arg("channels"),
           py::arg("busbw_gbs"), py::arg("latency_us"), py::arg("scratch"), py::arg("scratch_bytes"))
      .def("outstanding", &Comm::outstanding)
      .def_property_readonly("stream", &Comm::stream)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("size", &Comm::size)
      .def_property_readonly("aborted", &Comm::aborted);
}
