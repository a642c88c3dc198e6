// comm.cpp — collective backends of the coset-sharded prover (see comm.hpp).
#include "comm.hpp"

#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

namespace {

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw CommError(std::string(what) + ": " + hipGetErrorString(e));
}
void nccl_ok(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw CommError(std::string(what) + ": " + ncclGetErrorString(r));
}

// ------------------------------------------------------------------ world 1
struct SelfComm : zkp_comm {
  const char* kind() const override { return "self"; }
  void copy(hipStream_t st, const void* send, void* recv, size_t bytes) {
    if (send != recv && bytes) hip_ok(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, st), "self copy");
  }
  void all_to_all(hipStream_t st, const void* send, void* recv, size_t b) override { copy(st, send, recv, b); }
  void all_gather(hipStream_t st, const void* send, void* recv, size_t b) override { copy(st, send, recv, b); }
};

// ------------------------------------------------------------------ in-process group
// Ranks are host threads (each with its own zkp_ctx and stream, on one or more
// devices). A collective publishes the rank's send pointer, meets the others
// at a barrier, pulls its blocks with device copies, and meets them again so
// no rank reuses its send buffer while a peer is still reading it.
struct LocalGroup {
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  unsigned long long gen = 0;
  bool failed = false;
  std::vector<const void*> ptrs;
  explicit LocalGroup(int w) : world(w), ptrs(w, nullptr) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (failed) throw CommError("a peer rank of the local group failed");
    unsigned long long g = gen;
    if (++arrived == world) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || failed; });
    }
    if (failed) throw CommError("a peer rank of the local group failed");
  }
  void fail() {
    std::lock_guard<std::mutex> lk(mu);
    failed = true;
    cv.notify_all();
  }
};

struct LocalComm : zkp_comm {
  std::shared_ptr<LocalGroup> g;
  const char* kind() const override { return "local"; }
  void exchange(hipStream_t st, const void* send, void* recv, size_t bytes, bool a2a) {
    hip_ok(hipStreamSynchronize(st), "local group: sync before publish");
    g->ptrs[rank] = send;
    g->barrier();
    for (int s = 0; s < world; s++) {
      const char* src = static_cast<const char*>(g->ptrs[s]) + (a2a ? (size_t)rank * bytes : 0);
      char* dst = static_cast<char*>(recv) + (size_t)s * bytes;
      if (src != dst && bytes) hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st), "local group copy");
    }
    hip_ok(hipStreamSynchronize(st), "local group: sync after copy");
    g->barrier();
  }
  void all_to_all(hipStream_t st, const void* send, void* recv, size_t b) override { exchange(st, send, recv, b, true); }
  void all_gather(hipStream_t st, const void* send, void* recv, size_t b) override { exchange(st, send, recv, b, false); }
  void abort() override { g->fail(); }
};

// ------------------------------------------------------------------ RCCL
// Ordering invariant: every collective of a communicator runs on
// the communicator's own stream `cs`, in the order the prover issues them (the
// same program order on every rank). The caller's stream (main, side or copy)
// hands over with an event before the collective and waits for one after it, so
// collectives issued from different prover streams are never in flight on one
// communicator at the same time, whatever RCCL does internally with streams.
struct RcclComm : zkp_comm {
  ncclComm_t c = nullptr;
  hipStream_t cs = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  const char* kind() const override { return "rccl"; }
  void enter(hipStream_t st) {
    hip_ok(hipEventRecord(ev_in, st), "rccl: record on the caller stream");
    hip_ok(hipStreamWaitEvent(cs, ev_in, 0), "rccl: comm stream waits");
  }
  void leave(hipStream_t st) {
    hip_ok(hipEventRecord(ev_out, cs), "rccl: record on the comm stream");
    hip_ok(hipStreamWaitEvent(st, ev_out, 0), "rccl: caller stream waits");
  }
  void all_to_all(hipStream_t st, const void* send, void* recv, size_t b) override {
    enter(st);
    nccl_ok(ncclGroupStart(), "ncclGroupStart");
    for (int s = 0; s < world; s++) {
      nccl_ok(ncclSend(static_cast<const char*>(send) + (size_t)s * b, b, ncclUint8, s, c, cs), "ncclSend");
      nccl_ok(ncclRecv(static_cast<char*>(recv) + (size_t)s * b, b, ncclUint8, s, c, cs), "ncclRecv");
    }
    nccl_ok(ncclGroupEnd(), "ncclGroupEnd");
    leave(st);
  }
  void all_gather(hipStream_t st, const void* send, void* recv, size_t b) override {
    enter(st);
    nccl_ok(ncclAllGather(send, recv, b, ncclUint8, c, cs), "ncclAllGather");
    leave(st);
  }
  void abort() override {
    if (c) (void)ncclCommAbort(c);
    c = nullptr;
  }
  int backend_world() const override {
    int n = -1;
    if (!c || ncclCommCount(c, &n) != ncclSuccess) return -1;
    return n;
  }
  ~RcclComm() override {
    if (c) (void)ncclCommDestroy(c);
    if (cs) (void)hipStreamSynchronize(cs);
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_out) (void)hipEventDestroy(ev_out);
    if (cs) (void)hipStreamDestroy(cs);
  }
};

// ------------------------------------------------------------------ caller transport
// One process per rank, collectives carried by the caller's transport
// (zkp_host_transport: e.g. torch.distributed/gloo, MPI, sockets) through
// pinned host staging: device -> host, the caller's collective, host -> device.
// The exchange points and buffers are exactly those of the RCCL backend.
struct HostComm : zkp_comm {
  zkp_host_transport t{};
  void* stage = nullptr;
  size_t stage_bytes = 0;
  const char* kind() const override { return "host"; }
  char* staging(size_t bytes) {
    if (stage_bytes < bytes) {
      if (stage) (void)hipHostFree(stage);
      stage = nullptr;
      stage_bytes = 0;
      hip_ok(hipHostMalloc(&stage, bytes, hipHostMallocDefault), "host comm staging");
      stage_bytes = bytes;
    }
    return static_cast<char*>(stage);
  }
  void exchange(hipStream_t st, const void* send, void* recv, size_t bytes, bool a2a) {
    const size_t out_b = a2a ? (size_t)world * bytes : bytes, in_b = (size_t)world * bytes;
    char* hs = staging(out_b + in_b);
    char* hr = hs + out_b;
    if (out_b) hip_ok(hipMemcpyAsync(hs, send, out_b, hipMemcpyDeviceToHost, st), "host comm: D2H");
    hip_ok(hipStreamSynchronize(st), "host comm: sync before the transport");
    int rc = a2a ? t.all_to_all(t.user, hs, hr, bytes) : t.all_gather(t.user, hs, hr, bytes);
    if (rc != 0) throw CommError("caller transport failed (status " + std::to_string(rc) + ")");
    if (in_b) hip_ok(hipMemcpyAsync(recv, hr, in_b, hipMemcpyHostToDevice, st), "host comm: H2D");
    hip_ok(hipStreamSynchronize(st), "host comm: sync after H2D");  // staging is reused by the next exchange
  }
  void all_to_all(hipStream_t st, const void* send, void* recv, size_t b) override { exchange(st, send, recv, b, true); }
  void all_gather(hipStream_t st, const void* send, void* recv, size_t b) override { exchange(st, send, recv, b, false); }
  void abort() override {
    if (t.abort) t.abort(t.user);
  }
  ~HostComm() override {
    if (stage) (void)hipHostFree(stage);
  }
};

}  // namespace

zkp_comm* make_host_comm(int world, int rank, const zkp_host_transport& t) {
  auto* c = new HostComm();
  c->rank = rank;
  c->world = world;
  c->t = t;
  return c;
}

zkp_comm* make_self_comm() { return new SelfComm(); }

void make_local_group(int world, zkp_comm** out) {
  auto g = std::make_shared<LocalGroup>(world);
  for (int r = 0; r < world; r++) {
    auto* c = new LocalComm();
    c->rank = r;
    c->world = world;
    c->g = g;
    out[r] = c;
  }
}

void rccl_unique_id(unsigned char id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "NCCL_UNIQUE_ID_BYTES");
  ncclUniqueId u;
  nccl_ok(ncclGetUniqueId(&u), "ncclGetUniqueId");
  memcpy(id, &u, sizeof u);
}

zkp_comm* make_rccl_comm(int device, const unsigned char id[128], int world, int rank) {
  hip_ok(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  auto* c = new RcclComm();
  c->rank = rank;
  c->world = world;
  if (hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming) != hipSuccess) {
    delete c;
    throw CommError("rccl: stream/event creation failed");
  }
  ncclResult_t r = ncclCommInitRank(&c->c, world, u, rank);
  if (r != ncclSuccess) {
    delete c;
    throw CommError(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  return c;
}
