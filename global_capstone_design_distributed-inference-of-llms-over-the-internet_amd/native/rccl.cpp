// Direct RCCL communicators for the device data plane (SURVEY §2.4 "RCCL calls ... captured
// inside the per-stage HIP graph"; §7.5 "keep RCCL a thin, separately tested layer").
//
// torch.distributed's ProcessGroupNCCL runs every collective / send / recv on a private stream
// with its own events and a lazily built per-peer communicator: a call cannot be recorded into
// a hipGraph that the executor replays, and the first send to a new peer initialises a
// communicator mid-step.  This module owns the communicator itself (one ncclComm_t per
// channel direction or TP group, initialised eagerly from a unique id exchanged over the
// channel's TCPStore) and enqueues every operation on the CALLER's stream, so
//
//   * a stage's decode graph captures its hidden-state ncclSend right after the last layer
//     (no host launch, no private copy: stream order keeps the next replay from overwriting
//     the buffer until the send has read it), and the receiver's ncclRecv lands straight in
//     the graph's static input;
//   * the tensor-parallel all-reduces after the o / down projections are captured with the
//     rest of the step (torch's all-reduce cannot be replayed from a graph).
//
// The library is the librccl torch itself loaded (dlopen of its path: one RCCL instance in the
// process), resolved by symbol at start-up; nothing here links against ROCm.  Blocking calls
// (communicator init, group end) release the GIL.  Failure handling: ``abort`` (ncclCommAbort)
// releases a stream blocked on a dead peer; ``async_error`` polls the communicator.
#include <dlfcn.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

typedef struct ncclComm* comm_t;
struct UniqueId {
  char internal[128];
};
typedef int result_t;  // ncclResult_t: 0 = ncclSuccess, 7 = ncclInProgress
typedef void* stream_t;  // hipStream_t

struct Api {
  void* lib = nullptr;
  result_t (*get_unique_id)(UniqueId*) = nullptr;
  result_t (*comm_init_rank)(comm_t*, int, UniqueId, int) = nullptr;
  result_t (*all_reduce)(const void*, void*, size_t, int, int, comm_t, stream_t) = nullptr;
  result_t (*all_gather)(const void*, void*, size_t, int, comm_t, stream_t) = nullptr;
  result_t (*send)(const void*, size_t, int, int, comm_t, stream_t) = nullptr;
  result_t (*recv)(void*, size_t, int, int, comm_t, stream_t) = nullptr;
  result_t (*group_start)() = nullptr;
  result_t (*group_end)() = nullptr;
  result_t (*comm_abort)(comm_t) = nullptr;
  result_t (*comm_destroy)(comm_t) = nullptr;
  result_t (*async_error)(comm_t, result_t*) = nullptr;
  const char* (*error_string)(result_t) = nullptr;
  result_t (*get_version)(int*) = nullptr;
};

Api g_api;

template <typename F>
void sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g_api.lib, name));
  if (f == nullptr) throw std::runtime_error(std::string("librccl: missing symbol ") + name);
}

int load(const std::string& path) {
  if (g_api.lib != nullptr) return 0;
  // the copy torch already mapped (RTLD_NOLOAD), else map it now
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
  if (h == nullptr) h = dlopen(path.c_str(), RTLD_NOW);
  if (h == nullptr) throw std::runtime_error(std::string("dlopen ") + path + ": " + dlerror());
  g_api.lib = h;
  sym(g_api.get_unique_id, "ncclGetUniqueId");
  sym(g_api.comm_init_rank, "ncclCommInitRank");
  sym(g_api.all_reduce, "ncclAllReduce");
  sym(g_api.all_gather, "ncclAllGather");
  sym(g_api.send, "ncclSend");
  sym(g_api.recv, "ncclRecv");
  sym(g_api.group_start, "ncclGroupStart");
  sym(g_api.group_end, "ncclGroupEnd");
  sym(g_api.comm_abort, "ncclCommAbort");
  sym(g_api.comm_destroy, "ncclCommDestroy");
  sym(g_api.async_error, "ncclCommGetAsyncError");
  sym(g_api.error_string, "ncclGetErrorString");
  sym(g_api.get_version, "ncclGetVersion");
  int v = 0;
  g_api.get_version(&v);
  return v;
}

void check(result_t r, const char* what) {
  if (r != 0) {
    const char* s = g_api.error_string ? g_api.error_string(r) : "?";
    throw std::runtime_error(std::string(what) + " failed: " + s + " (" + std::to_string(r) + ")");
  }
}

void need() {
  if (g_api.lib == nullptr) throw std::runtime_error("librccl not loaded (call load(path) first)");
}

py::bytes unique_id() {
  need();
  UniqueId id;
  check(g_api.get_unique_id(&id), "ncclGetUniqueId");
  return py::bytes(id.internal, sizeof(id.internal));
}

// One communicator.  Pointers / streams travel as integers (torch's data_ptr() and
// Stream.cuda_stream): no torch headers in this translation unit.
class Comm {
 public:
  Comm(int nranks, int rank, py::bytes uid) : nranks_(nranks), rank_(rank) {
    need();
    std::string s = uid;
    if (s.size() != sizeof(UniqueId)) throw std::invalid_argument("unique id must be 128 bytes");
    UniqueId id;
    std::memcpy(id.internal, s.data(), sizeof(id.internal));
    result_t r;
    {
      py::gil_scoped_release nogil;  // blocks until every rank has joined
      r = g_api.comm_init_rank(&comm_, nranks, id, rank);
    }
    check(r, "ncclCommInitRank");
  }
  ~Comm() { destroy(); }

  void all_reduce(uintptr_t buf, size_t count, int dtype, int op, uintptr_t stream) {
    live();
    check(g_api.all_reduce(reinterpret_cast<void*>(buf), reinterpret_cast<void*>(buf), count, dtype, op, comm_,
                           reinterpret_cast<stream_t>(stream)),
          "ncclAllReduce");
  }
  void all_gather(uintptr_t src, uintptr_t dst, size_t count, int dtype, uintptr_t stream) {
    live();
    check(g_api.all_gather(reinterpret_cast<void*>(src), reinterpret_cast<void*>(dst), count, dtype, comm_,
                           reinterpret_cast<stream_t>(stream)),
          "ncclAllGather");
  }
  // one send and/or one receive, fused into one group (a receive from peer p and a send to p on
  // the same stream must be grouped, or each waits for the other's kernel)
  void send_recv(uintptr_t sbuf, size_t scount, int speer, uintptr_t rbuf, size_t rcount, int rpeer, int dtype,
                 uintptr_t stream) {
    live();
    stream_t st = reinterpret_cast<stream_t>(stream);
    check(g_api.group_start(), "ncclGroupStart");
    result_t r = 0;
    if (scount > 0 && speer >= 0) r = g_api.send(reinterpret_cast<void*>(sbuf), scount, dtype, speer, comm_, st);
    if (r == 0 && rcount > 0 && rpeer >= 0)
      r = g_api.recv(reinterpret_cast<void*>(rbuf), rcount, dtype, rpeer, comm_, st);
    result_t e;
    {
      py::gil_scoped_release nogil;
      e = g_api.group_end();
    }
    check(r, "ncclSend/ncclRecv");
    check(e, "ncclGroupEnd");
  }
  void send(uintptr_t buf, size_t count, int dtype, int peer, uintptr_t stream) {
    send_recv(buf, count, peer, 0, 0, -1, dtype, stream);
  }
  void recv(uintptr_t buf, size_t count, int dtype, int peer, uintptr_t stream) {
    send_recv(0, 0, -1, buf, count, peer, dtype, stream);
  }
  // 0 = healthy; an RCCL error code otherwise (a peer died / the communicator was aborted)
  int async_error() {
    if (comm_ == nullptr) return -1;
    result_t e = 0;
    g_api.async_error(comm_, &e);
    return e;
  }
  void abort() {
    if (comm_ != nullptr) {
      comm_t c = comm_;
      comm_ = nullptr;
      py::gil_scoped_release nogil;
      g_api.comm_abort(c);
    }
  }
  void destroy() {
    if (comm_ != nullptr && g_api.lib != nullptr) {
      comm_t c = comm_;
      comm_ = nullptr;
      g_api.comm_destroy(c);
    }
  }
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  bool alive() const { return comm_ != nullptr; }

 private:
  void live() {
    if (comm_ == nullptr) throw std::runtime_error("RCCL communicator is closed");
  }
  comm_t comm_ = nullptr;
  int nranks_, rank_;
};

}  // namespace

PYBIND11_MODULE(_mpamd_rccl, m) {
  m.doc() = "Direct RCCL communicators on the caller's stream (hipGraph-capturable)";
  m.def("load", &load, py::arg("path"), "map librccl (torch's copy) and resolve the API; returns the version");
  m.def("unique_id", &unique_id);
  // ncclDataType_t / ncclRedOp_t values used by the Python side
  m.attr("UINT8") = 1;
  m.attr("INT32") = 2;
  m.attr("INT64") = 4;
  m.attr("FLOAT16") = 6;
  m.attr("FLOAT32") = 7;
  m.attr("BFLOAT16") = 9;
  m.attr("SUM") = 0;
  m.attr("MAX") = 2;
  py::class_<Comm>(m, "Comm")
      .def(py::init<int, int, py::bytes>(), py::arg("nranks"), py::arg("rank"), py::arg("uid"))
      .def("all_reduce", &Comm::all_reduce)
      .def("all_gather", &Comm::all_gather)
      .def("send", &Comm::send)
      .def("recv", &Comm::recv)
      .def("send_recv", &Comm::send_recv)
      .def("async_error", &Comm::async_error)
      .def("abort", &Comm::abort)
      .def("destroy", &Comm::destroy)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("size", &Comm::size)
      .def_property_readonly("alive", &Comm::alive);
}
