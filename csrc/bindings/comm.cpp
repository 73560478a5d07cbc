// tfk_comm: the runtime's own RCCL communicator.
//
// One process per GPU; the chief draws an ncclUniqueId and publishes it through the job's TCP store
// (parallel/tfk_comm.py), every rank calls ncclCommInitRank. Collectives are enqueued on a stream
// the caller chooses (a HIP stream handle; 0 = torch's current stream), so a caller that is
// capturing a hipGraph gets the RCCL kernels as graph nodes -- the training step, gradient buckets
// included, replays as one graph at any world size. No watchdog thread, no work objects: ordering is
// expressed with stream events by the Python layer. abort() (ncclCommAbort) is safe to call from
// the runtime watchdog thread while the main thread is blocked on a wedged collective.
//
// Linked against the librccl.so that torch itself loads (same SONAME, librccl.so.1), so one RCCL
// instance serves both.
#include <rccl/rccl.h>

#include <atomic>
#include <mutex>
#include <string>

#include "bind_util.h"

namespace py = pybind11;

namespace {

void nccl_check(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, "RCCL ", what, " failed: ", ncclGetErrorString(r), " (", (int)r, ")");
}

ncclDataType_t nccl_dtype(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "tfk_comm: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  if (op == "avg") return ncclAvg;
  TORCH_CHECK(false, "tfk_comm: unknown reduction '", op, "' (sum|max|min|prod|avg)");
  return ncclSum;
}

hipStream_t pick_stream(uint64_t s) { return s ? reinterpret_cast<hipStream_t>(s) : cur_stream(); }

void need_comm_tensor(const torch::Tensor& t, int device, const char* name) {
  TORCH_CHECK(t.is_cuda(), "tfk_comm: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.get_device() == device, "tfk_comm: ", name, " is on device ", t.get_device(),
              ", the communicator on ", device);
  TORCH_CHECK(t.is_contiguous(), "tfk_comm: ", name, " must be contiguous");
}

py::bytes unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

int version() {
  int v = 0;
  nccl_check(ncclGetVersion(&v), "ncclGetVersion");
  return v;
}

// The rccl.h this binding was compiled against (ROCm 7.2) is newer than the librccl torch loads
// (ROCm 7.0.x); parallel/tfk_comm.py checks at import that both are the same major family and that
// the runtime has every entry point used here (ncclCommSplit / ncclCommFinalize: >= 2.18).
int header_version() { return NCCL_VERSION_CODE; }

class RcclComm {
 public:
  // Blocks until all nranks have joined (ncclCommInitRank); the GIL is released meanwhile.
  RcclComm(const std::string& uid, int nranks, int rank, int device) : nranks_(nranks), rank_(rank), device_(device) {
    TORCH_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "tfk_comm: unique id must be ", NCCL_UNIQUE_ID_BYTES, " bytes");
    TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "tfk_comm: bad rank ", rank, " of ", nranks);
    ncclUniqueId id;
    memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;
      TORCH_CHECK(hipSetDevice(device) == hipSuccess, "tfk_comm: hipSetDevice(", device, ")");
      r = ncclCommInitRank(&comm_, nranks, id, rank);
    }
    nccl_check(r, "ncclCommInitRank");
  }
  explicit RcclComm(ncclComm_t c, int device) : comm_(c), device_(device) {
    nccl_check(ncclCommCount(c, &nranks_), "ncclCommCount");
    nccl_check(ncclCommUserRank(c, &rank_), "ncclCommUserRank");
  }
  ~RcclComm() {
    // a normal teardown destroys explicitly; a communicator dropped without destroy() is aborted
    // (never blocks in the destructor, e.g. at interpreter exit after a peer died)
    if (comm_ && !gone_.exchange(true)) ncclCommAbort(comm_);
  }

  int rank() const { return rank_; }
  int size() const { return nranks_; }
  int device() const { return device_; }
  bool valid() const { return comm_ != nullptr && !gone_.load(); }

  void all_reduce(torch::Tensor in, torch::Tensor out, const std::string& op, uint64_t stream) {
    live();
    need_comm_tensor(in, device_, "input");
    need_comm_tensor(out, device_, "output");
    TORCH_CHECK(in.numel() == out.numel() && in.scalar_type() == out.scalar_type(), "all_reduce: in/out mismatch");
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // RCCL may block (lazy peer connect): keep the watchdog thread runnable
      r = ncclAllReduce(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), nccl_dtype(in), nccl_op(op), comm_, pick_stream(stream));
    }
    nccl_check(r, "ncclAllReduce");
  }
  void reduce(torch::Tensor in, torch::Tensor out, int root, const std::string& op, uint64_t stream) {
    live();
    need_comm_tensor(in, device_, "input");
    need_comm_tensor(out, device_, "output");
    TORCH_CHECK(in.numel() == out.numel() && in.scalar_type() == out.scalar_type(), "reduce: in/out mismatch");
    check_peer(root);
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // RCCL may block (lazy peer connect): keep the watchdog thread runnable
      r = ncclReduce(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), nccl_dtype(in), nccl_op(op), root, comm_, pick_stream(stream));
    }
    nccl_check(r, "ncclReduce");
  }
  void broadcast(torch::Tensor t, int root, uint64_t stream) {
    live();
    need_comm_tensor(t, device_, "tensor");
    check_peer(root);
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // RCCL may block (lazy peer connect): keep the watchdog thread runnable
      r = ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), root, comm_, pick_stream(stream));
    }
    nccl_check(r, "ncclBroadcast");
  }
  // out holds size() * in.numel() elements (rank-major)
  void all_gather(torch::Tensor out, torch::Tensor in, uint64_t stream) {
    live();
    need_comm_tensor(in, device_, "input");
    need_comm_tensor(out, device_, "output");
    TORCH_CHECK(out.numel() == in.numel() * nranks_ && in.scalar_type() == out.scalar_type(),
                "all_gather: output must hold world * input elements");
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // RCCL may block (lazy peer connect): keep the watchdog thread runnable
      r = ncclAllGather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), nccl_dtype(in), comm_, pick_stream(stream));
    }
    nccl_check(r, "ncclAllGather");
  }
  // in holds size() * out.numel() elements; rank r receives the reduced r-th slice
  void reduce_scatter(torch::Tensor out, torch::Tensor in, const std::string& op, uint64_t stream) {
    live();
    need_comm_tensor(in, device_, "input");
    need_comm_tensor(out, device_, "output");
    TORCH_CHECK(in.numel() == out.numel() * nranks_ && in.scalar_type() == out.scalar_type(),
                "reduce_scatter: input must hold world * output elements");
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // RCCL may block (lazy peer connect): keep the watchdog thread runnable
      r = ncclReduceScatter(in.data_ptr(), out.data_ptr(), (size_t)out.numel(), nccl_dtype(in), nccl_op(op), comm_, pick_stream(stream));
    }
    nccl_check(r, "ncclReduceScatter");
  }
  void all_to_all(torch::Tensor out, torch::Tensor in, uint64_t stream) {
    live();
    need_comm_tensor(in, device_, "input");
    need_comm_tensor(out, device_, "output");
    TORCH_CHECK(in.numel() == out.numel() && in.numel() % nranks_ == 0 && in.scalar_type() == out.scalar_type(),
                "all_to_all: equal in/out, divisible by world");
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // RCCL may block (lazy peer connect): keep the watchdog thread runnable
      r = ncclAllToAll(in.data_ptr(), out.data_ptr(), (size_t)(in.numel() / nranks_), nccl_dtype(in), comm_, pick_stream(stream));
    }
    nccl_check(r, "ncclAllToAll");
  }
  void send(torch::Tensor t, int peer, uint64_t stream) {
    live();
    need_comm_tensor(t, device_, "tensor");
    check_peer(peer);
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // RCCL may block (lazy peer connect): keep the watchdog thread runnable
      r = ncclSend(t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), peer, comm_, pick_stream(stream));
    }
    nccl_check(r, "ncclSend");
  }
  void recv(torch::Tensor t, int peer, uint64_t stream) {
    live();
    need_comm_tensor(t, device_, "tensor");
    check_peer(peer);
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // RCCL may block (lazy peer connect): keep the watchdog thread runnable
      r = ncclRecv(t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), peer, comm_, pick_stream(stream));
    }
    nccl_check(r, "ncclRecv");
  }

  // Sub-communicator (ncclCommSplit): every rank of this communicator must call it, in the same
  // order; ranks passing color < 0 get None.
  std::unique_ptr<RcclComm> split(int color, int key) {
    live();
    ncclComm_t nc = nullptr;
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;
      r = ncclCommSplit(comm_, color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &nc, nullptr);
    }
    nccl_check(r, "ncclCommSplit");
    if (!nc) return nullptr;
    return std::unique_ptr<RcclComm>(new RcclComm(nc, device_));
  }

  // "" while healthy, else the asynchronous error RCCL recorded (peer lost, remote abort ...)
  std::string async_error() {
    if (destroyed_.load()) return std::string();  // orderly teardown (destroy), not a failure
    if (!valid()) return "communicator aborted";
    ncclResult_t e = ncclSuccess;
    nccl_check(ncclCommGetAsyncError(comm_, &e), "ncclCommGetAsyncError");
    return e == ncclSuccess || e == ncclInProgress ? std::string() : std::string(ncclGetErrorString(e));
  }

  // Tear down without waiting for peers: outstanding RCCL kernels of this communicator exit, so a
  // rank whose peer died does not spin on the GPU. Idempotent, callable from any thread.
  void abort() {
    if (!comm_ || gone_.exchange(true)) return;
    py::gil_scoped_release nogil;
    ncclCommAbort(comm_);
  }
  // Orderly teardown (all ranks): finalize outstanding work, then free.
  void destroy() {
    if (!comm_) return;
    destroyed_.store(true);
    if (gone_.exchange(true)) return;
    py::gil_scoped_release nogil;
    ncclCommFinalize(comm_);
    ncclCommDestroy(comm_);
  }

 private:
  void live() const { TORCH_CHECK(valid(), "tfk_comm: communicator was aborted or destroyed"); }
  void check_peer(int p) const { TORCH_CHECK(p >= 0 && p < nranks_, "tfk_comm: peer ", p, " out of range [0,", nranks_, ")"); }

  ncclComm_t comm_ = nullptr;
  int nranks_ = 0, rank_ = 0, device_ = 0;
  std::atomic<bool> gone_{false};
  std::atomic<bool> destroyed_{false};
};

void group_start() { nccl_check(ncclGroupStart(), "ncclGroupStart"); }
void group_end() {
  ncclResult_t r;
  {
    py::gil_scoped_release nogil;
    r = ncclGroupEnd();
  }
  nccl_check(r, "ncclGroupEnd");
}

}  // namespace

void register_comm_ops(py::module& m) {
  m.def("rccl_unique_id", &unique_id);
  m.def("rccl_version", &version);
  m.def("rccl_header_version", &header_version);
  m.def("rccl_group_start", &group_start);
  m.def("rccl_group_end", &group_end);
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, int>(), py::arg("unique_id"), py::arg("nranks"), py::arg("rank"),
           py::arg("device"))
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("device", &RcclComm::device)
      .def_property_readonly("valid", &RcclComm::valid)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("input"), py::arg("output"), py::arg("op") = "sum",
           py::arg("stream") = 0)
      .def("reduce", &RcclComm::reduce, py::arg("input"), py::arg("output"), py::arg("root"), py::arg("op") = "sum",
           py::arg("stream") = 0)
      .def("broadcast", &RcclComm::broadcast, py::arg("tensor"), py::arg("root"), py::arg("stream") = 0)
      .def("all_gather", &RcclComm::all_gather, py::arg("output"), py::arg("input"), py::arg("stream") = 0)
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::arg("output"), py::arg("input"), py::arg("op") = "sum",
           py::arg("stream") = 0)
      .def("all_to_all", &RcclComm::all_to_all, py::arg("output"), py::arg("input"), py::arg("stream") = 0)
      .def("send", &RcclComm::send, py::arg("tensor"), py::arg("peer"), py::arg("stream") = 0)
      .def("recv", &RcclComm::recv, py::arg("tensor"), py::arg("peer"), py::arg("stream") = 0)
      .def("split", &RcclComm::split, py::arg("color"), py::arg("key"))
      .def("async_error", &RcclComm::async_error)
      .def("abort", &RcclComm::abort)
      .def("destroy", &RcclComm::destroy);
}
