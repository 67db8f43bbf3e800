// executor.cpp -- communicators, transports and the device plan executor of
// libbine_amd.so, plus the C ABI of include/bine_amd.h.
//
// Execution model (one process per GPU, one communicator per process):
//   * compute stream K = the caller's stream: every REDUCE / REDUCE3 / COPY;
//   * comm stream C (the communicator's own, high priority): every exchange,
//     i.e. RCCL ncclSend/ncclRecv inside one ncclGroupStart/End (RCCL P2P over
//     xGMI), or the in-process loopback copies;
//   * hipEvents hand work between the two, only where memory regions overlap
//     (make_schedule, schedule.cpp).  An exchange whose receive feeds the
//     following reduction element-for-element (plan flag BINE_PRIM_PIPELINE --
//     every reduce-scatter step of the Bine schedules) is cut into chunks: the
//     receive of chunk k+1 on C overlaps the reduction of chunk k on K, and the
//     next step's first chunks go out while this step's last ones are reduced.
//     This is the device form of the segmented variant's double-buffered
//     Irecv/Reduce_local loop (libbine_allreduce.c:1218-1253).
//   * workspace (TMP0..2), plans and their schedules are cached per communicator.
#include <execinfo.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <ucontext.h>
#include <rccl/rccl.h>
#include <signal.h>
#include <unistd.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bine_internal.h"
#include "direct.h"

namespace bine {

static thread_local std::string g_err;

static void set_err(const char *fmt, ...) {
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      set_err("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
      return BINE_ERR_HIP;                                                         \
    }                                                                              \
  } while (0)

#define NCCL_TRY(expr)                                                                 \
  do {                                                                                 \
    ncclResult_t r_ = (expr);                                                          \
    if (r_ != ncclSuccess) {                                                           \
      set_err("%s:%d %s -> %s", __FILE__, __LINE__, #expr, ncclGetErrorString(r_));    \
      return BINE_ERR_RCCL;                                                            \
    }                                                                                  \
  } while (0)

// ---------------------------------------------------------------------------
// transports
// ---------------------------------------------------------------------------

struct Transport {
  virtual ~Transport() = default;
  virtual int exchange(const std::vector<XSend> &s, const std::vector<XRecv> &r, hipStream_t st) = 0;
  virtual int vendor_allreduce(const void *, void *, size_t, int, int, hipStream_t) { return BINE_ERR_UNSUPPORTED; }
  virtual int alltoallv(const std::vector<XSend> &, const std::vector<XRecv> &, hipStream_t) {
    return BINE_ERR_UNSUPPORTED;
  }
  virtual void retire() {}
  // device-side transport state that must see every collective's exchanges
  // in one stream order (the direct transport's sequence bases)
  virtual bool stream_ordered() const { return false; }
  // non-success: the transport is unusable (checked before issuing and
  // before a graph replay); _drained: the same after the streams drained,
  // with the transport's full state in the error string
  virtual int health() const { return BINE_SUCCESS; }
  virtual int health_drained() const { return health(); }
  // an exchange whose receives are the leaves of the following tree, the
  // tree evaluated inside the exchange (direct transport, k_dm_move_tree)
  virtual bool tree_ok(const std::vector<XSend> &, const std::vector<XRecv> &, const TreeSpec &) const {
    return false;
  }
  virtual bool defer_ok(const std::vector<XSend> &, const std::vector<XRecv> &, const std::vector<XRecv> &,
                        const TreeSpec &) const {
    return false;
  }
  // DirectState::exchange's tree / deferred-leaves forms
  virtual int exchange_tree(const std::vector<XSend> &, const std::vector<XRecv> &, const TreeSpec *,
                            const std::vector<XRecv> *, const TreeSpec *, hipStream_t) {
    return BINE_ERR_UNSUPPORTED;
  }
};

static bool nccl_type(int dtype, ncclDataType_t *t) {
  switch (dtype) {
    case BINE_INT8: *t = ncclInt8; return true;
    case BINE_UINT8: *t = ncclUint8; return true;
    case BINE_INT32: *t = ncclInt32; return true;
    case BINE_UINT32: *t = ncclUint32; return true;
    case BINE_INT64: *t = ncclInt64; return true;
    case BINE_UINT64: *t = ncclUint64; return true;
    case BINE_FLOAT: *t = ncclFloat32; return true;
    case BINE_DOUBLE: *t = ncclFloat64; return true;
    default: return false;  // 16-bit integers: no RCCL type
  }
}

struct RcclTransport final : Transport {
  ncclComm_t comm = nullptr;
  int rank = 0, size = 1;
  // bine_comm_set_coll_ag: an exchange in which this rank sends ONE buffer to
  // every other rank and receives one equal-sized message from each (the flat
  // allgather phase, the one-shot latency form, the allgather family's flat
  // form) runs as ncclAllGather into `stage`, then the P-1 received blocks are
  // copied to their destinations.  Same bytes in the same places: result bits
  // unchanged.  The test is local but globally consistent: with block sizes
  // b_0..b_{P-1}, rank x matches iff b_y == b_x for every y, i.e. all ranks
  // match or none does.
  bool coll_ag = false;
  void *stage = nullptr;
  size_t stage_bytes = 0;
  uint64_t stage_gen = 0;  // bumped when `stage` moves (graph mode drops graphs holding the old one)
  ~RcclTransport() override {
    if (stage) (void)hipFree(stage);
    if (comm) ncclCommDestroy(comm);
  }
  // *all = 1 iff every rank passes ok = true (an RCCL MIN reduction of one int)
  int agree(bool ok, int *all) {
    int *d = nullptr;
    HIP_TRY(hipMalloc(&d, sizeof(int)));
    int v = ok ? 1 : 0;
    hipError_t e = hipMemcpy(d, &v, sizeof v, hipMemcpyHostToDevice);
    ncclResult_t nr = ncclSuccess;
    if (e == hipSuccess) nr = ncclAllReduce(d, d, 1, ncclInt32, ncclMin, comm, nullptr);
    if (e == hipSuccess && nr == ncclSuccess) e = hipStreamSynchronize(nullptr);
    if (e == hipSuccess && nr == ncclSuccess) e = hipMemcpy(&v, d, sizeof v, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    NCCL_TRY(nr);
    HIP_TRY(e);
    *all = v;
    return BINE_SUCCESS;
  }
  // The RCCL ABI probe at communicator creation (see bine_rccl_abi_check): the
  // enum values this library passes, run through the loaded runtime in one
  // group and checked on the host -- int32 MIN, uint32 MAX, int64 SUM, float
  // SUM, double PROD (ops on data whose result depends on reading the type
  // right), and a uint8 allgather (the exchanges' byte type: a misread element
  // size would move the wrong number of bytes)
  int abi_probe() {
    constexpr int kG = 8;  // bytes each rank contributes to the allgather
    struct Probe {
      int32_t i32[2];
      uint32_t u32;
      int32_t pad;
      int64_t i64;
      float f32;
      int32_t pad2;
      double f64;
      uint8_t g[64 * kG];
    };
    if (size > 64) return BINE_SUCCESS;  // the probe's gather area: up to 64 ranks
    Probe h{};
    h.i32[0] = rank + 1;
    h.i32[1] = -(rank + 1);
    h.u32 = 0x10000u * (uint32_t)rank + 7u;
    h.i64 = ((int64_t)1 << 40) + rank;
    h.f32 = 0.5f + (float)rank;
    h.f64 = rank == 0 ? 3.0 : 1.0;
    uint8_t mine[kG];
    for (int k = 0; k < kG; k++) mine[k] = (uint8_t)(rank * 37 + k * 11 + 1);
    Probe *d = nullptr;
    uint8_t *gs = nullptr;
    HIP_TRY(hipMalloc(&d, sizeof(Probe)));
    hipError_t e = hipMalloc(&gs, kG);
    if (e == hipSuccess) e = hipMemcpy(d, &h, sizeof h, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(gs, mine, kG, hipMemcpyHostToDevice);
    ncclResult_t nr = ncclSuccess;
    if (e == hipSuccess) {
      nr = ncclGroupStart();
      if (nr == ncclSuccess) nr = ncclAllReduce(d->i32, d->i32, 2, ncclInt32, ncclMin, comm, nullptr);
      if (nr == ncclSuccess) nr = ncclAllReduce(&d->u32, &d->u32, 1, ncclUint32, ncclMax, comm, nullptr);
      if (nr == ncclSuccess) nr = ncclAllReduce(&d->i64, &d->i64, 1, ncclInt64, ncclSum, comm, nullptr);
      if (nr == ncclSuccess) nr = ncclAllReduce(&d->f32, &d->f32, 1, ncclFloat32, ncclSum, comm, nullptr);
      if (nr == ncclSuccess) nr = ncclAllReduce(&d->f64, &d->f64, 1, ncclFloat64, ncclProd, comm, nullptr);
      if (nr == ncclSuccess) nr = ncclAllGather(gs, d->g, kG, ncclUint8, comm, nullptr);
      const ncclResult_t ne = ncclGroupEnd();
      if (nr == ncclSuccess) nr = ne;
    }
    if (e == hipSuccess && nr == ncclSuccess) e = hipStreamSynchronize(nullptr);
    Probe o{};
    if (e == hipSuccess && nr == ncclSuccess) e = hipMemcpy(&o, d, sizeof o, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (gs) (void)hipFree(gs);
    NCCL_TRY(nr);
    HIP_TRY(e);
    const int64_t P = size;
    bool ok = o.i32[0] == 1 && o.i32[1] == -(int32_t)P && o.u32 == 0x10000u * (uint32_t)(P - 1) + 7u &&
              o.i64 == P * ((int64_t)1 << 40) + P * (P - 1) / 2 && o.f32 == 0.5f * (float)P + (float)(P * (P - 1) / 2) &&
              o.f64 == 3.0;
    for (int x = 0; ok && x < size; x++)
      for (int k = 0; k < kG; k++) ok = ok && o.g[x * kG + k] == (uint8_t)(x * 37 + k * 11 + 1);
    if (!ok) {
      set_err("RCCL ABI probe failed on rank %d: the runtime reads this library's types / ops differently", rank);
      return BINE_ERR_RCCL;
    }
    return BINE_SUCCESS;
  }
  // how many ranks of this communicator run on this rank's GPU (same host
  // name and PCI bus id): more than one only when processes share a device
  int ranks_on_my_gpu(int device, int *same) {
    char bus[64] = {0}, host[256] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess || !bus[0]) {
      // no bus id: the device UUID, else this rank alone (never a false match)
      (void)hipGetLastError();
      hipUUID u{};
      if (hipDeviceGetUuid(&u, device) == hipSuccess) {
        for (int k = 0; k < 16 && 2 * k + 2 < (int)sizeof bus; k++)
          snprintf(bus + 2 * k, 3, "%02x", (unsigned char)u.bytes[k]);
      } else {
        (void)hipGetLastError();
        snprintf(bus, sizeof bus, "rank-%d", rank);
      }
    }
    gethostname(host, sizeof host - 1);
    uint64_t h = 1469598103934665603ull;  // FNV-1a of "host/bus"
    for (const char *s : {(const char *)host, "/", (const char *)bus})
      for (; *s; s++) h = (h ^ (uint8_t)*s) * 1099511628211ull;
    uint64_t *d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)size * sizeof(uint64_t)));
    hipError_t e = hipMemcpy(d + rank, &h, sizeof h, hipMemcpyHostToDevice);
    ncclResult_t nr = ncclSuccess;
    if (e == hipSuccess) nr = ncclAllGather(d + rank, d, 1, ncclUint64, comm, nullptr);
    if (e == hipSuccess && nr == ncclSuccess) e = hipStreamSynchronize(nullptr);
    std::vector<uint64_t> all((size_t)size);
    if (e == hipSuccess && nr == ncclSuccess) e = hipMemcpy(all.data(), d, all.size() * sizeof(uint64_t),
                                                            hipMemcpyDeviceToHost);
    (void)hipFree(d);
    NCCL_TRY(nr);
    HIP_TRY(e);
    *same = (int)std::count(all.begin(), all.end(), h);
    return BINE_SUCCESS;
  }
  // bine_comm_set_direct: exchanges through mapped peer memory (direct.cpp)
  std::unique_ptr<DirectState> dm;
  bool dm_on = false;
  int dm_wgs = 0;  // workgroups per message of the direct transport (0: BINE_DIRECT_WGS / 128)
  uint64_t key = 0;  // hash of the unique id: names the direct transport's sockets
  bool stream_ordered() const override { return dm_on; }
  // `flags`: also read the per-peer flags (device memory: only once the
  // streams drained, bine_comm_synchronize)
  int health(bool flags) const {
    if (dm_on && dm->poisoned()) {
      set_err("direct transport: a wait timed out; transport disabled: %s", dm->describe(flags).c_str());
      return BINE_ERR_INTERNAL;
    }
    return BINE_SUCCESS;
  }
  int health() const override { return health(false); }
  int health_drained() const override { return health(true); }
  bool allgather_shape(const std::vector<XSend> &s, const std::vector<XRecv> &r) const {
    if (size < 3 || (int)s.size() != size - 1 || (int)r.size() != size - 1) return false;
    const size_t b = s[0].bytes;
    std::vector<char> seen_s((size_t)size, 0), seen_r((size_t)size, 0);
    for (const auto &x : s) {
      if (x.ptr != s[0].ptr || x.bytes != b || x.peer == rank || seen_s[(size_t)x.peer]) return false;
      seen_s[(size_t)x.peer] = 1;
    }
    for (const auto &x : r) {
      if (x.bytes != b || x.peer == rank || seen_r[(size_t)x.peer]) return false;
      seen_r[(size_t)x.peer] = 1;
    }
    return true;
  }
  int allgather(const std::vector<XSend> &s, const std::vector<XRecv> &r, hipStream_t st) {
    const size_t b = s[0].bytes, need = b * (size_t)size;
    if (need > stage_bytes) {
      HIP_TRY(hipStreamSynchronize(st));  // the old area may still be read by enqueued copies
      if (stage) HIP_TRY(hipFree(stage));
      stage = nullptr;
      stage_bytes = 0;
      HIP_TRY(hipMalloc(&stage, need));
      stage_bytes = need;
      stage_gen++;
    }
    static const bool trace = getenv("BINE_TRACE") && atoi(getenv("BINE_TRACE")) != 0;
    if (trace) fprintf(stderr, "[bine r%d] coll_ag ncclAllGather %zu B per rank\n", rank, b);
    NCCL_TRY(ncclAllGather(s[0].ptr, stage, b, ncclUint8, comm, st));
    for (const auto &x : r) {
      const int rc = launch_copy(x.ptr, (const char *)stage + (size_t)x.peer * b, b, st);
      if (rc) return rc;
    }
    return BINE_SUCCESS;
  }
  bool tree_ok(const std::vector<XSend> &s, const std::vector<XRecv> &r, const TreeSpec &t) const override {
    return dm_on && dm && dm->tree_ok(s, r, t);
  }
  bool defer_ok(const std::vector<XSend> &s, const std::vector<XRecv> &r, const std::vector<XRecv> &dl,
                const TreeSpec &t) const override {
    return dm_on && dm && dm->defer_ok(s, r, dl, t);
  }
  int exchange_tree(const std::vector<XSend> &s, const std::vector<XRecv> &r, const TreeSpec *t,
                    const std::vector<XRecv> *dl, const TreeSpec *dt, hipStream_t st) override {
    if (!dm_on) return BINE_ERR_UNSUPPORTED;
    if (int rc = health(false)) return rc;
    return dm->exchange(s, r, st, t, dl, dt);
  }
  int exchange(const std::vector<XSend> &s, const std::vector<XRecv> &r, hipStream_t st) override {
    if (dm_on) {
      if (int rc = health(false)) return rc;
      return dm->exchange(s, r, st);
    }
    if (coll_ag && allgather_shape(s, r)) return allgather(s, r, st);
    NCCL_TRY(ncclGroupStart());
    // the group is always closed, also when posting an operation failed
    ncclResult_t r0 = ncclSuccess;
    for (const auto &x : s)
      if (r0 == ncclSuccess) r0 = ncclSend(x.ptr, x.bytes, ncclUint8, x.peer, comm, st);
    for (const auto &x : r)
      if (r0 == ncclSuccess) r0 = ncclRecv(x.ptr, x.bytes, ncclUint8, x.peer, comm, st);
    const ncclResult_t r1 = ncclGroupEnd();
    NCCL_TRY(r0);
    NCCL_TRY(r1);
    return BINE_SUCCESS;
  }
  // one message to and from every peer as ONE ncclAllToAllv: displacements
  // from the lowest send / receive address (nothing to or from self)
  int alltoallv(const std::vector<XSend> &s, const std::vector<XRecv> &r, hipStream_t st) override {
    std::vector<size_t> sc((size_t)size, 0), sd((size_t)size, 0), rc((size_t)size, 0), rd((size_t)size, 0);
    const char *sb = (const char *)s[0].ptr;
    char *rb = (char *)r[0].ptr;
    for (const auto &x : s) sb = std::min(sb, (const char *)x.ptr);
    for (const auto &x : r) rb = std::min(rb, (char *)x.ptr);
    for (const auto &x : s) {
      sc[(size_t)x.peer] = x.bytes;
      sd[(size_t)x.peer] = (size_t)((const char *)x.ptr - sb);
    }
    for (const auto &x : r) {
      rc[(size_t)x.peer] = x.bytes;
      rd[(size_t)x.peer] = (size_t)((char *)x.ptr - rb);
    }
    static const bool trace = getenv("BINE_TRACE") && atoi(getenv("BINE_TRACE")) != 0;
    if (trace) fprintf(stderr, "[bine r%d] coll_a2a ncclAllToAllv %zu B per peer\n", rank, s[0].bytes);
    NCCL_TRY(ncclAllToAllv(sb, sc.data(), sd.data(), rb, rc.data(), rd.data(), ncclUint8, comm, st));
    return BINE_SUCCESS;
  }
  int vendor_allreduce(const void *s, void *r, size_t n, int dtype, int op, hipStream_t st) override {
    // RCCL has no logical / bitwise reductions: the vendor baseline covers the arithmetic four
    static const ncclRedOp_t ops[4] = {ncclSum, ncclProd, ncclMax, ncclMin};
    ncclDataType_t t;
    if (!nccl_type(dtype, &t) || op < 0 || op > BINE_MIN) return BINE_ERR_ARG;
    NCCL_TRY(ncclAllReduce(s, r, n, t, ops[op], comm, st));
    return BINE_SUCCESS;
  }
};

// In-process peer copies between virtual ranks on one device.  A send posts
// {pointer, ready-event}; the receiver waits for the event on its own stream,
// copies, records done; the sender's stream then waits for done before anything
// that could overwrite the send buffer -- ncclSend/ncclRecv semantics.
struct LoopbackHub {
  struct Post {
    const void *ptr = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr, done = nullptr;
    bool consumed = false;
  };
  int P;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::deque<Post *>> box;  // [src * P + dst]
  std::atomic<int> mismatches{0};
  explicit LoopbackHub(int n) : P(n), box((size_t)n * (size_t)n) {}
};

struct LoopbackTransport final : Transport {
  std::shared_ptr<LoopbackHub> hub;
  int rank;
  std::vector<LoopbackHub::Post *> retired;
  LoopbackTransport(std::shared_ptr<LoopbackHub> h, int r) : hub(std::move(h)), rank(r) {}
  ~LoopbackTransport() override { retire(); }
  void retire() override {  // caller guarantees the streams are idle
    for (auto *p : retired) {
      (void)hipEventDestroy(p->ready);
      (void)hipEventDestroy(p->done);
      delete p;
    }
    retired.clear();
  }
  int exchange(const std::vector<XSend> &s, const std::vector<XRecv> &r, hipStream_t st) override {
    const int P = hub->P;
    std::vector<LoopbackHub::Post *> mine;
    for (const auto &x : s) {
      auto *p = new LoopbackHub::Post;
      p->ptr = x.ptr;
      p->bytes = x.bytes;
      HIP_TRY(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&p->done, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(p->ready, st));
      {
        std::lock_guard<std::mutex> g(hub->mu);
        hub->box[(size_t)rank * (size_t)P + (size_t)x.peer].push_back(p);
      }
      hub->cv.notify_all();
      mine.push_back(p);
    }
    for (const auto &x : r) {
      LoopbackHub::Post *p;
      {
        std::unique_lock<std::mutex> g(hub->mu);
        auto &q = hub->box[(size_t)x.peer * (size_t)P + (size_t)rank];
        hub->cv.wait(g, [&] { return !q.empty(); });
        p = q.front();
        q.pop_front();
      }
      if (p->bytes != x.bytes) hub->mismatches++;
      HIP_TRY(hipStreamWaitEvent(st, p->ready, 0));
      const size_t nb = std::min(p->bytes, x.bytes);
      if (nb) HIP_TRY(hipMemcpyAsync(x.ptr, p->ptr, nb, hipMemcpyDeviceToDevice, st));
      HIP_TRY(hipEventRecord(p->done, st));
      {
        std::lock_guard<std::mutex> g(hub->mu);
        p->consumed = true;
      }
      hub->cv.notify_all();
    }
    for (auto *p : mine) {
      {
        std::unique_lock<std::mutex> g(hub->mu);
        hub->cv.wait(g, [&] { return p->consumed; });
      }
      HIP_TRY(hipStreamWaitEvent(st, p->done, 0));
      retired.push_back(p);
    }
    return BINE_SUCCESS;
  }
};

// the trees plan_dm_trees (below) fuses into exchange launches
struct DmTreePlan {
  std::vector<int> tree_at, host, hosted;
  std::vector<char> defer;
  std::vector<TreeSpec> spec;                // by tree op j
  std::vector<std::vector<XRecv>> leaves;    // by tree op j: exchange i's receives
  bool any = false;   // some tree is fused
  bool solo = false;  // every local op is a fused tree: the whole call on one stream (execute)
};

}  // namespace bine

// ---------------------------------------------------------------------------
// communicator
// ---------------------------------------------------------------------------

struct bine_comm {
  int rank = 0, size = 1, device = 0;
  hipStream_t stream = nullptr;   // default compute stream
  hipStream_t cstream = nullptr;  // comm stream
  std::unique_ptr<bine::Transport> tx;
  std::shared_ptr<bine::LoopbackHub> hub;
  void *tmp[4] = {nullptr, nullptr, nullptr, nullptr};  // TMP0..2, STAGE
  size_t tmp_bytes[4] = {0, 0, 0, 0};
  size_t relay_min_bytes = 0;  // relay mode: smallest relayed part (0: off)
  bool trees = false;          // multi-tree mode (allreduce, P = 4 / 8)
  size_t chunk_bytes = 0;      // pipelining chunk (0: default_chunk_bytes(direct transport on))
  size_t single_stream_bytes = 1 << 20;  // collectives up to this size run on the caller's stream only
  int flat_ag = 0;             // allreduce: one-step all-peers allgather phase (2: cut with the flat RS chunks)
  bool flat_rs = false;        // one-step all-peers reduce-scatter phase + tree kernel
  bool coll_a2a = false;       // all-peers exchanges as ncclAllToAllv (no relay / trees)
  hipStream_t last_user = nullptr;  // caller's stream of the latest collective
  bool used_user = false;
  // stream-ordered transports (the direct transport's device-side sequence
  // bases): every exchange of a call must follow every exchange of the
  // previous call, whichever caller stream that one ran on.  `order_ev` is
  // recorded on the caller's stream at the end of each call (which by then
  // follows all of the call's exchanges, single-stream or not, eager or graph);
  // a call on another stream waits for it before issuing anything.
  hipEvent_t order_ev = nullptr;
  hipStream_t order_stream = nullptr;
  bool order_valid = false;
  // bine_comm_set_graphs: each (plan, buffers, stream) is captured once into a
  // HIP graph -- both streams' work and the event hand-offs between them -- and
  // replayed with one hipGraphLaunch per call (RCCL communicators only)
  bool graphs = false;
  struct GraphEntry { hipGraph_t g = nullptr; hipGraphExec_t x = nullptr; };
  std::map<std::string, GraphEntry> graph_cache;
  uint64_t graph_stage_gen = 0;  // the transport's staging-area generation the cached graphs hold
  std::vector<hipEvent_t> ev;
  size_t ev_next = 0;
  std::map<std::string, std::pair<bine::Plan, bine::Schedule>> plans;
  std::map<std::string, bine::StageRanges> stage_cache;  // host staging ranges per plan key
  std::vector<hipEvent_t> op_ev;  // scratch of execute()
  std::vector<hipEvent_t> stage_ev;  // scratch of execute(): host staging batches
  // scratch of execute(): trees evaluated inside their exchange (plan_dm_trees)
  bool dm_tree = false;  // bine_comm_set_direct_tree
  int dm_tree_wgs = 0;   // its tree workgroups per launch (0: the transport's default)
  // fused-tree plans (plan_dm_trees) per (plan, buffers, dtype, op, settings):
  // a pure function of those, cached so a call's issue path does not redo it
  std::map<std::string, bine::DmTreePlan> tree_cache;
  std::map<std::string, bool> fused_cache;  // fused_for
  int64_t fused_calls = 0;                  // bine_comm_fused_calls
  std::vector<hipEvent_t> tree_ev;
  std::vector<char> tree_pending;
  // per-op device timing of the latest collective (bine_comm_set_profile)
  bool profile = false;
  struct OpTime { hipEvent_t a = nullptr, b = nullptr; int xchg = 0, nprims = 0; uint64_t bytes = 0; };
  std::vector<OpTime> prof;
  size_t prof_n = 0;
  std::vector<bine::XSend> xs;
  std::vector<bine::XRecv> xr;
  std::mutex mu;
  // releases whatever was set up (also after a failed init); the caller has
  // drained the streams (bine_comm_destroy) or never used them (init errors)
  void drop_graphs() {  // caller: no cached graph is still executing
    for (auto &kv : graph_cache) {
      if (kv.second.x) (void)hipGraphExecDestroy(kv.second.x);
      if (kv.second.g) (void)hipGraphDestroy(kv.second.g);
    }
    graph_cache.clear();
  }
  ~bine_comm() {
    (void)hipSetDevice(device);
    drop_graphs();
    tx.reset();
    for (int t = 0; t < 4; t++)
      if (tmp[t]) (void)hipFree(tmp[t]);
    for (auto e : ev) (void)hipEventDestroy(e);
    if (order_ev) (void)hipEventDestroy(order_ev);
    for (auto &p : prof) {
      if (p.a) (void)hipEventDestroy(p.a);
      if (p.b) (void)hipEventDestroy(p.b);
    }
    if (stream) (void)hipStreamDestroy(stream);
    if (cstream) (void)hipStreamDestroy(cstream);
  }
};

namespace bine {

// BINE_SEGV_TRACE=1 (diagnostics): a host-side SIGSEGV / SIGABRT prints the
// native call stack to stderr -- which HIP / RCCL call of which library
// function faulted -- and then passes the signal on to the handler installed
// before (Python's faulthandler prints its frames) or the default action
static struct sigaction g_prev_segv, g_prev_abrt;
static char g_segv_dir[256];  // BINE_SEGV_TRACE_DIR: one file per process instead of stderr
static void put_str(int fd, const char *s) { (void)!write(fd, s, strlen(s)); }
static void put_hex(int fd, const char *label, uint64_t v) {
  char b[32];
  int n = 0;
  b[n++] = '0';
  b[n++] = 'x';
  for (int sh = 60; sh >= 0; sh -= 4) b[n++] = "0123456789abcdef"[(v >> sh) & 15];
  b[n++] = '\n';
  put_str(fd, label);
  (void)!write(fd, b, (size_t)n);
}
static void segv_trace(int sig, siginfo_t *si, void *uc) {
  // async-signal-safe calls only (open / read / write), plus backtrace
  int fd = 2;
  if (g_segv_dir[0]) {
    char path[320];
    char pid[24];
    int n = 0;
    for (long p = (long)getpid(); p > 0; p /= 10) pid[n++] = (char)('0' + p % 10);
    size_t k = strlen(g_segv_dir);
    memcpy(path, g_segv_dir, k);
    memcpy(path + k, "/segv_", 6);
    k += 6;
    while (n > 0) path[k++] = pid[--n];
    memcpy(path + k, ".txt", 5);
    const int f = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (f >= 0) fd = f;
  }
  put_str(fd, sig == SIGSEGV ? "bine: SIGSEGV, native stack:\n" : "bine: SIGABRT, native stack:\n");
  put_hex(fd, "fault address ", (uint64_t)(uintptr_t)(si ? si->si_addr : nullptr));
  if (uc) {
    const greg_t *g = ((ucontext_t *)uc)->uc_mcontext.gregs;
    put_hex(fd, "interrupted pc ", (uint64_t)g[REG_RIP]);
    // a jump / call to a bad address leaves no unwind information at the pc:
    // the words at the stack pointer hold the caller's return address
    put_hex(fd, "sp ", (uint64_t)g[REG_RSP]);
    const uint64_t *sp = (const uint64_t *)g[REG_RSP];
    for (int k = 0; k < 24 && sp; k++) put_hex(fd, "  [sp] ", sp[k]);
    put_hex(fd, "rdi ", (uint64_t)g[REG_RDI]);
    put_hex(fd, "rax ", (uint64_t)g[REG_RAX]);
  }
  void *fr[64];
  backtrace_symbols_fd(fr, backtrace(fr, 64), fd);
  // the load addresses of the runtime libraries, to place the frames
  const int m = open("/proc/self/maps", O_RDONLY);
  if (m >= 0) {
    put_str(fd, "maps (executable segments of HIP / HSA / RCCL / bine):\n");
    char buf[4096], line[512];
    size_t ll = 0;
    ssize_t got;
    while ((got = read(m, buf, sizeof buf)) > 0) {
      for (ssize_t i = 0; i < got; i++) {
        if (ll < sizeof line - 1) line[ll++] = buf[i];
        if (buf[i] != '\n') continue;
        line[ll] = 0;
        if (strstr(line, "r-xp") && (strstr(line, "amdhip") || strstr(line, "hsa-runtime") || strstr(line, "rccl") ||
                                     strstr(line, "bine")))
          (void)!write(fd, line, ll);
        ll = 0;
      }
    }
    close(m);
  }
  if (fd != 2) {
    put_str(2, "bine: fatal signal; native stack written to BINE_SEGV_TRACE_DIR\n");
    close(fd);
  }
  struct sigaction &prev = sig == SIGSEGV ? g_prev_segv : g_prev_abrt;
  sigaction(sig, &prev, nullptr);
  if ((prev.sa_flags & SA_SIGINFO) && prev.sa_sigaction) prev.sa_sigaction(sig, si, uc);
  else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN) prev.sa_handler(sig);
  else raise(sig);
}
static void install_segv_trace() {
  static std::once_flag once;
  std::call_once(once, [] {
    const char *e = getenv("BINE_SEGV_TRACE");
    if (!e || atoi(e) == 0) return;
    if (const char *d = getenv("BINE_SEGV_TRACE_DIR"))
      if (strlen(d) < sizeof g_segv_dir - 32) strcpy(g_segv_dir, d);
    struct sigaction sa {};
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGABRT, &sa, &g_prev_abrt);
  });
}

// BINE_DIRECT_TREE=0: new communicators start with the direct transport's
// fused trees off (bine_comm_set_direct_tree; on by default)
static bool dm_tree_env() {
  static const bool on = !getenv("BINE_DIRECT_TREE") || atoi(getenv("BINE_DIRECT_TREE")) != 0;
  return on;
}

static int comm_setup(bine_comm *c) {
  install_segv_trace();
  c->dm_tree = dm_tree_env();
  HIP_TRY(hipSetDevice(c->device));
  int lo = 0, hi = 0;
  HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  // the comm stream at the highest priority (BINE_COMM_PRIORITY=0: the
  // default priority, a diagnostic for ranks sharing one GPU)
  const char *cp = getenv("BINE_COMM_PRIORITY");
  HIP_TRY(hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, cp && atoi(cp) == 0 ? lo : hi));
  c->ev.resize(1024);
  for (auto &e : c->ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming));
  if (const char *e = getenv("BINE_RELAY_MIN_BYTES")) c->relay_min_bytes = (size_t)strtoull(e, nullptr, 10);
  if (const char *e = getenv("BINE_TREES")) c->trees = atoi(e) != 0;
  if (const char *e = getenv("BINE_FLAT_AG")) c->flat_ag = atoi(e) < 0 ? 0 : std::min(atoi(e), 2);
  if (const char *e = getenv("BINE_FLAT_RS")) c->flat_rs = atoi(e) != 0;
  if (const char *e = getenv("BINE_COLL_A2A")) c->coll_a2a = atoi(e) != 0;
  if (const char *e = getenv("BINE_GRAPHS")) c->graphs = atoi(e) != 0;
  if (const char *e = getenv("BINE_SINGLE_STREAM_BYTES")) c->single_stream_bytes = (size_t)strtoull(e, nullptr, 10);
  return BINE_SUCCESS;
}

// BINE_ROCTX=1: roctx ranges around every collective and every issued op
// (host timeline of rocprofv3 --marker-trace)
static bool roctx_on() {
  static const bool on = getenv("BINE_ROCTX") && atoi(getenv("BINE_ROCTX")) != 0;
  return on;
}

// BINE_TRACE=1: one stderr line per issued op (debugging the issue sequence)
static bool trace_on() {
  static const bool on = getenv("BINE_TRACE") && atoi(getenv("BINE_TRACE")) != 0;
  return on;
}

static hipEvent_t next_event(bine_comm *c) {
  hipEvent_t e = c->ev[c->ev_next];
  c->ev_next = (c->ev_next + 1) % c->ev.size();
  return e;
}

// `dst` waits for all work enqueued so far on `src`
static int stream_join(bine_comm *c, hipStream_t dst, hipStream_t src) {
  hipEvent_t e = next_event(c);
  HIP_TRY(hipEventRecord(e, src));
  HIP_TRY(hipStreamWaitEvent(dst, e, 0));
  return BINE_SUCCESS;
}

// stream-ordered transports: K follows the previous call's exchanges (see
// bine_comm::order_ev); order_end() marks this call's end on K
static int order_begin(bine_comm *c, hipStream_t K) {
  if (c->tx->stream_ordered() && c->order_valid && c->order_stream != K)
    HIP_TRY(hipStreamWaitEvent(K, c->order_ev, 0));
  return BINE_SUCCESS;
}

static int order_end(bine_comm *c, hipStream_t K) {
  if (!c->tx->stream_ordered()) return BINE_SUCCESS;
  HIP_TRY(hipEventRecord(c->order_ev, K));
  c->order_stream = K;
  c->order_valid = true;
  return BINE_SUCCESS;
}

static int ensure_workspace(bine_comm *c, const uint64_t *elems, size_t esz, hipStream_t user) {
  bool grow = false;
  for (int t = 0; t < 4; t++) grow |= elems[t] * esz > c->tmp_bytes[t];
  if (!grow) return BINE_SUCCESS;
  // old buffers may still be read by enqueued work
  HIP_TRY(hipStreamSynchronize(user));
  HIP_TRY(hipStreamSynchronize(c->cstream));
  c->drop_graphs();  // captured graphs hold the old workspace addresses

  for (int t = 0; t < 4; t++) {
    const size_t need = elems[t] * esz;
    if (need <= c->tmp_bytes[t]) continue;
    if (c->tmp[t]) HIP_TRY(hipFree(c->tmp[t]));
    c->tmp[t] = nullptr;
    c->tmp_bytes[t] = 0;
    const size_t alloc = (need + 255) & ~(size_t)255;
    HIP_TRY(hipMalloc(&c->tmp[t], alloc));
    c->tmp_bytes[t] = alloc;
  }
  return BINE_SUCCESS;
}

// BINE_CHUNK_BYTES, else 16 MiB -- 64 MiB over the direct transport, whose
// exchange launches take whole 64 MiB slots (C3 at P = 2 on one GPU: 0.50 ms
// at 64 MiB vs 0.66 at 16, profiles/r4_dm_stamps_p2_sweep2.txt; the node
// model: 0.45 vs 0.47 ms at P = 8).  Bit-identical either way.
static size_t default_chunk_bytes(bool direct) {
  static const char *e = getenv("BINE_CHUNK_BYTES");
  if (e) return (size_t)strtoull(e, nullptr, 10);
  return (size_t)(direct ? 64 : 16) << 20;
}

// ---------------------------------------------------------------------------
// plan execution
// ---------------------------------------------------------------------------

// Issue a schedule (make_schedule): exchanges on the comm stream C, local
// primitives on the caller's stream K, one event per op, and a cross-stream
// wait only where the schedule names one.
// the local primitives of one op: several reductions go out as one batched
// launch (multi-tree rounds), anything else one launch / copy each
template <typename Ptr>
static int run_local(const std::vector<Prim> &prims, Ptr ptr, int dtype, int op, size_t esz, hipStream_t K) {
  const size_t n = prims.size();
  bool batch = n >= 2 && n <= (size_t)kMaxBatch;
  for (const Prim &p : prims) batch = batch && (p.type == BINE_PRIM_REDUCE || p.type == BINE_PRIM_REDUCE3);
  if (batch) {
    const void *a[kMaxBatch], *b[kMaxBatch];
    void *out[kMaxBatch];
    size_t cnt[kMaxBatch];
    for (size_t i = 0; i < n; i++) {
      const Prim &p = prims[i];
      a[i] = ptr(p.src_buf, p.src_off);
      b[i] = p.type == BINE_PRIM_REDUCE ? ptr(p.dst_buf, p.dst_off) : ptr(p.aux_buf, p.aux_off);
      out[i] = ptr(p.dst_buf, p.dst_off);
      cnt[i] = p.count;
    }
    const int rc = launch_reduce_batch((int)n, a, b, out, cnt, dtype, op, K);
    if (rc != BINE_ERR_ARG) return rc;  // ERR_ARG: not co-aligned, one by one below
  }
  for (const Prim &p : prims) {
    int rc = BINE_SUCCESS;
    if (p.type == BINE_PRIM_REDUCE)
      rc = launch_reduce(ptr(p.src_buf, p.src_off), ptr(p.dst_buf, p.dst_off), ptr(p.dst_buf, p.dst_off), p.count,
                         dtype, op, K);
    else if (p.type == BINE_PRIM_REDUCE_TREE) {
      if (p.peer < 2 || p.peer > kMaxLeaves) return BINE_ERR_INTERNAL;
      if (p.pos < 0 || p.pos >= p.peer) return BINE_ERR_INTERNAL;
      const void *leaf[kMaxLeaves];
      for (int j = 0, k = 0; j < p.peer; j++)
        leaf[j] = j == p.pos ? ptr(p.aux_buf, p.aux_off) : ptr(p.src_buf, p.src_off + (uint64_t)k++ * p.count);
      rc = launch_reduce_tree(p.peer, leaf, ptr(p.dst_buf, p.dst_off), p.count, dtype, op, K,
                              (unsigned)p.flags >> 8);
    } else if (p.type == BINE_PRIM_REDUCE3)
      rc = launch_reduce(ptr(p.src_buf, p.src_off), ptr(p.aux_buf, p.aux_off), ptr(p.dst_buf, p.dst_off), p.count,
                         dtype, op, K);
    else
      rc = launch_copy(ptr(p.dst_buf, p.dst_off), ptr(p.src_buf, p.src_off), p.count * esz, K);
    if (rc) return rc;
  }
  return BINE_SUCCESS;
}

// single = true: every op on the caller's stream K in issue order (small
// collectives: no overlap to win, so no cross-stream event edges to pay for)
// bine_comm_set_coll_a2a: an exchange with exactly one message of B bytes to
// and from every other rank.  With relay and multi-tree mode off (settings are
// collective) such exchanges come only from the flat phases, where rank x
// sends peer y the part y evaluates (e_y bytes) and receives e_x from each:
// x matches iff e_y == e_x for all y -- every rank or none.
static bool a2a_shape(const bine_comm *c, const std::vector<XSend> &s, const std::vector<XRecv> &r) {
  const int P = c->size;
  if (!c->coll_a2a || c->hub || c->relay_min_bytes || c->trees || P < 3) return false;  // hub: loopback
  const auto *rt = dynamic_cast<const RcclTransport *>(c->tx.get());
  if (!rt || rt->dm_on) return false;  // direct exchanges have their own path
  if ((int)s.size() != P - 1 || (int)r.size() != P - 1) return false;
  const size_t b = s[0].bytes;
  std::vector<char> ss((size_t)P, 0), rs((size_t)P, 0);
  for (const auto &x : s) {
    if (x.bytes != b || x.peer == c->rank || ss[(size_t)x.peer]) return false;
    ss[(size_t)x.peer] = 1;
  }
  for (const auto &x : r) {
    if (x.bytes != b || x.peer == c->rank || rs[(size_t)x.peer]) return false;
    rs[(size_t)x.peer] = 1;
  }
  return true;
}

// BINE_DIRECT_FUSED=0: small direct-transport collectives issue their
// primitives one by one instead of k_dm_fused
static bool fused_on() {
  static const bool on = !getenv("BINE_DIRECT_FUSED") || atoi(getenv("BINE_DIRECT_FUSED")) != 0;
  return on;
}

// BINE_DIRECT_FUSED_LARGE=0: large direct-transport collectives keep their
// per-exchange launches (k_dm_move / k_dm_move_tree) instead of k_dm_fused
static bool fused_large_on() {
  static const bool on = !getenv("BINE_DIRECT_FUSED_LARGE") || atoi(getenv("BINE_DIRECT_FUSED_LARGE")) != 0;
  return on;
}

// The flat form of a collective over the direct transport as ONE launch
// (k_dm_fused, bine_internal.h DmFusedArgs) when its schedule is
//   ([exchange X_c][REDUCE_TREE over X_c's received blocks + the own leaf])
//   for chunks c = 0 .. C-1, then optionally [exchange AG]
// with exchange AG (the flat allgather) sending the concatenated tree outputs
// to every peer and receiving into the caller's buffer --
// allreduce_bine_bdw_remap / _static / segmented / rabenseifner ... with the
// flat phases, the one-shot bine_lat, and the flat reduce-scatters.  AG's
// sends become the trees' result pushes (piece c = tree c's output, pushed
// from registers, one slot each but the last), its receives are cut into
// slot-sized pieces -- exactly the messages the per-exchange launches move,
// so ranks may choose either form independently.  The kernel's workgroups each own the same slice of
// every message, so it is correct only when no workgroup writes bytes another
// one may still read: the trees' outputs overlap no block the X exchanges
// send, and every piece AG receives is disjoint from the X sends or exactly
// one of them (the same slice then belongs to the same workgroup in both
// phases).  A message of more than one slot, more than kSlots messages to or
// from one peer, more than kMaxFusedTrees chunks or kMaxFusedMsgs messages:
// not this form.  Returns false when the schedule or the arguments do not
// qualify (the caller then issues the primitives).
// ops [o0, o1) of a schedule, indexed from 0
struct OpSpan {
  const SOp *p;
  size_t n;
  const SOp &operator[](size_t i) const { return p[i]; }
  size_t size() const { return n; }
};

// the transport parameters a fused launch is built from (the live
// DirectState, or bine_plan_dm_fused's host-only stand-in)
struct FusedEnv {
  int P = 1, rank = 0;
  const DirectState *d = nullptr;
  uint8_t *own = nullptr;  // the inbox base the kernel addresses (host-only planning: a stand-in)
};

template <typename Ptr>
static bool build_fused(const FusedEnv &e, OpSpan ops, Ptr ptr, size_t esz, int dtype, int op, bool single,
                        DmFusedArgs &a) {
  const size_t nops = ops.size();
  size_t C = 0, i = 0;
  while (i + 1 < nops && ops[i].xchg && !ops[i + 1].xchg) {
    if (ops[i + 1].prims.size() != 1 || ops[i + 1].prims[0].type != BINE_PRIM_REDUCE_TREE) return false;
    C++;
    i += 2;
  }
  const bool ag = i < nops;
  if (C == 0 || C > (size_t)kMaxFusedTrees || (ag && (i + 1 != nops || !ops[i].xchg))) return false;
  const DirectState &d = *e.d;
  const Prim &t0 = ops[1].prims[0];
  if (t0.peer < 2 || t0.peer > kMaxLeaves || t0.pos < 0 || t0.pos >= t0.peer) return false;
  a = DmFusedArgs{};
  a.wgs = single ? d.wgs : d.fused_wgs ? d.fused_wgs : d.tree_wgs;
  a.share = d.share;
  a.rank = e.rank;
  a.slot = d.slot;
  a.own = e.own;
  a.poison_host = d.hpoison_dev;
  a.timeout_ticks = d.timeout_ticks;
  a.slices = d.slice_flags ? 1 : 0;
  a.nl = t0.peer;
  a.pos = t0.pos;
  a.swap = (unsigned)t0.flags >> 8;
  a.nt = (int)C;
  struct Range { const char *lo, *hi; };
  auto overlap = [](Range x, Range y) { return x.lo < y.hi && y.lo < x.hi; };
  std::vector<Range> outs, owns, a_src;
  for (size_t k = 0; k < C; k++) {
    const Prim &t = ops[2 * k + 1].prims[0];
    const uint64_t tb = t.count * esz;
    if (t.peer != a.nl || t.pos != a.pos || ((unsigned)t.flags >> 8) != a.swap || !tb || tb % 16 || tb > d.slot)
      return false;
    DmFusedTree &ft = a.t[k];
    ft.own_leaf = ptr(t.aux_buf, t.aux_off);
    ft.out = ptr(t.dst_buf, t.dst_off);
    ft.nvec = tb / 16;
    outs.push_back({(const char *)ft.out, (const char *)ft.out + tb});
    owns.push_back({(const char *)ft.own_leaf, (const char *)ft.own_leaf + tb});
    for (int j = 0; j < kMaxLeaves; j++) ft.leaf[j] = -1;
  }
  // a tree's own leaf written by ANOTHER chunk's tree: there is
  // no grid barrier between the phases, so that is only safe when the bytes
  // a workgroup reads are the bytes it wrote itself -- the same range cut
  // into the same slices (equal nvec); anything else is not this form
  for (size_t k = 0; k < C; k++)
    for (size_t k2 = 0; k2 < C; k2++)
      if (k2 != k && overlap(owns[k2], outs[k]) &&
          (owns[k2].lo != outs[k].lo || owns[k2].hi != outs[k].hi || a.t[k2].nvec != a.t[k].nvec))
        return false;
  std::vector<int> js((size_t)e.P, 0), jr((size_t)e.P, 0);
  int n = 0;
  auto add = [&](int peer, uint64_t bytes, bool push, const void *src, void *dst) -> bool {
    if (n >= kMaxFusedMsgs || peer < 0 || peer >= e.P || peer == e.rank || bytes > d.slot || !bytes)
      return false;
    int &j = push ? js[(size_t)peer] : jr[(size_t)peer];
    if (j >= dm::kSlots) return false;
    DmMsg &m = a.m[n++];
    m.src = (const uint8_t *)src;
    m.dst = (uint8_t *)dst;
    m.bytes = bytes;
    m.push = push ? 1 : 0;
    m.peer = peer;
    m.j = j++;
    return true;
  };
  // phase A: every X exchange's sends (any source but a tree's output)
  for (size_t k = 0; k < C; k++)
    for (const Prim &x : ops[2 * k].prims)
      if (x.type == BINE_PRIM_SEND) {
        const char *p = ptr(x.src_buf, x.src_off);
        const Range r{p, p + x.count * esz};
        for (const Range &o : outs)
          if (overlap(r, o)) return false;
        if (!add(x.peer, x.count * esz, true, p, nullptr)) return false;
        a_src.push_back(r);
        a.na++;
      }
  // the allgather's sends: the trees' outputs, concatenated, to every peer
  std::vector<int> ag_peers;
  if (ag) {
    for (size_t k = 1; k < C; k++)
      if (outs[k].lo != outs[k - 1].hi) return false;
    for (const Prim &x : ops[nops - 1].prims)
      if (x.type == BINE_PRIM_SEND) {
        if (ptr(x.src_buf, x.src_off) != outs[0].lo || ptr(x.src_buf, x.src_off) + x.count * esz != outs[C - 1].hi)
          return false;
        ag_peers.push_back(x.peer);
      }
  }
  // phases B_c: X_c's receives are tree c's non-own leaves (leaf k of the
  // staging area: the k-th leaf != pos), then the result pushes of piece c
  for (size_t k = 0; k < C; k++) {
    const Prim &t = ops[2 * k + 1].prims[0];
    DmFusedTree &ft = a.t[k];
    ft.b0 = n;
    for (const Prim &x : ops[2 * k].prims)
      if (x.type == BINE_PRIM_RECV) {
        if (x.dst_buf != t.src_buf || x.count != t.count || x.dst_off < t.src_off ||
            (x.dst_off - t.src_off) % t.count)
          return false;
        const uint64_t q = (x.dst_off - t.src_off) / t.count;
        if (q >= (uint64_t)t.peer - 1) return false;
        const int leaf = (int)q < t.pos ? (int)q : (int)q + 1;
        if (ft.leaf[leaf] >= 0) return false;
        ft.leaf[leaf] = (int8_t)n;
        if (!add(x.peer, x.count * esz, false, nullptr, ptr(x.dst_buf, x.dst_off))) return false;
        ft.nb++;
      }
    if (ft.nb != t.peer - 1) return false;
    for (int p : ag_peers) {
      if (!add(p, ft.nvec * 16, true, ft.out, nullptr)) return false;
      ft.nc++;
    }
  }
  // phase D: the allgather's receives, cut into slot-sized pieces -- the
  // rounds DirectState::exchange cuts every message into, so each ordered
  // pair sees the same messages whichever form each side issues
  a.d0 = n;
  if (ag) {
    const uint64_t piece = d.slot;
    for (const Prim &x : ops[nops - 1].prims)
      if (x.type == BINE_PRIM_RECV) {
        char *p = ptr(x.dst_buf, x.dst_off);
        const uint64_t bytes = x.count * esz;
        for (uint64_t off = 0; off < bytes; off += piece) {
          const uint64_t len = std::min<uint64_t>(piece, bytes - off);
          const Range r{p + off, p + off + len};
          for (size_t k = 0; k < C; k++)
            if (overlap(r, outs[k]) || overlap(r, owns[k])) return false;
          for (const Range &y : a_src)
            if (overlap(r, y) && (r.lo != y.lo || r.hi != y.hi)) return false;
          if (len % 16 || !add(x.peer, len, false, nullptr, p + off)) return false;
          a.nd++;
        }
      }
    // our pieces are our trees' outputs: each exactly one slot but the last
    for (size_t k = 0; k + 1 < C; k++)
      if (a.t[k].nvec * 16 != d.slot) return false;
  }
  return dm_fused_check(a, dtype, op) == BINE_SUCCESS;
}

// The call's fused launches: the whole schedule as one k_dm_fused launch, or
// -- a reduce-scatter of more chunks than one launch holds (no allgather
// pieces) -- one launch per kMaxFusedTrees chunks.  Either way every ordered
// pair sees the per-exchange form's messages in its order (chunk by chunk),
// so the ranks' choices need not agree.  Empty: not this form.
template <typename Ptr>
static bool plan_fused_env(const FusedEnv &e, const Schedule &sc, Ptr ptr, size_t esz, int dtype, int op,
                           bool single, std::vector<DmFusedArgs> &out) {
  out.assign(1, DmFusedArgs{});
  const OpSpan all{sc.ops.data(), sc.ops.size()};
  if (build_fused(e, all, ptr, esz, dtype, op, single, out[0])) return true;
  out.clear();
  const size_t n = sc.ops.size();
  if (single || n % 2 || n <= 2 * (size_t)kMaxFusedTrees) return false;
  for (size_t i = 0; i < n; i += 2)  // [X_c][tree_c] pairs only: no allgather exchange at the end
    if (!sc.ops[i].xchg || sc.ops[i + 1].xchg) return false;
  for (size_t o0 = 0; o0 < n; o0 += 2 * kMaxFusedTrees) {
    out.emplace_back();
    const OpSpan g{sc.ops.data() + o0, std::min(n - o0, 2 * (size_t)kMaxFusedTrees)};
    if (!build_fused(e, g, ptr, esz, dtype, op, single, out.back())) {
      out.clear();
      return false;
    }
  }
  return true;
}

// the direct transport is on, other ranks of this communicator share this
// rank's GPU, and BINE_SHARED_GPU_SINGLE_STREAM=1 asks for one stream there
// (opt-in: DESIGN.md 7.2 -- one GPU-suite run with it on showed one digest
// mismatch per rank in the 8-process full-size check, case not captured; the
// rerun passed; not the default until that is explained)
static bool shared_gpu_direct(bine_comm *c) {
  static const bool on = getenv("BINE_SHARED_GPU_SINGLE_STREAM") && atoi(getenv("BINE_SHARED_GPU_SINGLE_STREAM")) != 0;
  auto *rt = dynamic_cast<RcclTransport *>(c->tx.get());
  return on && rt && rt->dm_on && rt->dm && rt->dm->share > 1;
}

template <typename Ptr>
static bool plan_fused(bine_comm *c, const Schedule &sc, Ptr ptr, size_t esz, int dtype, int op, bool single,
                       std::vector<DmFusedArgs> &out) {
  out.clear();
  auto *rt = dynamic_cast<RcclTransport *>(c->tx.get());
  if (!rt || !rt->dm_on || !rt->dm || c->profile || !fused_on() || op < 0 || !dm_fused_supported(dtype, op))
    return false;
  if (!single && !fused_large_on()) return false;
  FusedEnv e;
  e.P = c->size;
  e.rank = c->rank;
  e.d = rt->dm.get();
  e.own = (uint8_t *)rt->dm->own;
  return plan_fused_env(e, sc, ptr, esz, dtype, op, single, out);
}

// k_dm_fused for the call if its schedule qualifies (plan_fused): the
// launches' status, or -1 (the caller issues the primitives)
template <typename Ptr>
static int try_fused(bine_comm *c, const Schedule &sc, Ptr ptr, size_t esz, int dtype, int op, bool single,
                     hipStream_t K) {
  std::vector<DmFusedArgs> v;
  if (!plan_fused(c, sc, ptr, esz, dtype, op, single, v)) return -1;
  auto *rt = dynamic_cast<RcclTransport *>(c->tx.get());
  // as exchange(): a dead transport's launches would exit at once, moving nothing
  if (int rc = rt->health()) return rc;
  for (size_t i = 0; i < v.size(); i++) {
    v[i].stamps = rt->dm->stamps;
    v[i].serial = rt->dm->serial++;
    const int rc = launch_dm_fused(v[i], dtype, op, K);
    if (rc == BINE_ERR_ARG || rc == BINE_ERR_UNSUPPORTED) {
      if (i == 0) return -1;  // not co-aligned etc.: the primitives
      set_err("k_dm_fused: launch %zu of %zu refused after the first ran", i + 1, v.size());
      return BINE_ERR_INTERNAL;
    }
    if (rc) return rc;
  }
  if (!single) c->fused_calls++;
  return BINE_SUCCESS;
}

// Host staging of one call (bine_*_staged): the input buffer comes from
// `in_host` piece by piece on the h2d stream, the output goes back to
// `out_host` piece by piece on the d2h stream (StageRanges)
struct Staging {
  const char *in_host = nullptr;
  char *out_host = nullptr;
  hipStream_t h2d = nullptr, d2h = nullptr;
  const StageRanges *rg = nullptr;
};


// Trees of the flat reduce-scatter over the direct transport, evaluated
// inside an exchange launch instead of as pull copies into the staging area
// plus a separate k_reduce_tree launch (TreeSpec, k_dm_move_tree).  A pair
// [exchange i][...exchanges...][tree j] -- j the first local op after i,
// waiting for i, its non-own leaves exactly i's receives -- is hosted
//   * deferred (preferred): by the NEXT exchange i2 after i, whose first
//     launch pulls i's receives (issued at i without them) and evaluates the
//     tree beside i2's own messages -- tree k then overlaps the pushes of
//     chunk k + 1, as the separate tree launch on the caller's stream did.
//     Needs: i2 = i + 1 before j, or i2 = j + 1 (no op of either stream
//     between the tree's place and its host); i2 neither reads the tree's
//     output nor writes its output or own leaf, nor waits for j; leaves of
//     one slot each; i2 hosts no other tree;
//   * in its own exchange i otherwise (the last chunk's tree): the tree
//     workgroups of round r beside the pushes of round r + 1 (merge 1), or of
//     the one round; its output must overlap no block i sends;
//   * by itself otherwise (the last chunk's tree when its exchange already
//     hosts the previous one): a launch of its own on the comm stream at the
//     tree's place, pulling the leaves in place;
//   * not at all (the unfused form) when none applies.
// Always: the staging buffer is referenced by receives and trees only (no one
// else reads what is no longer written there).  host[j] = the hosting
// exchange, hosted[x] = the tree exchange x evaluates, tree_at[j] = i,
// defer[i]: i's receives are pulled by the host; false: no fused tree at all.
template <typename Ptr>
static bool plan_dm_trees(const Transport &tx, bool on, const Schedule &sc, Ptr ptr, size_t esz, int dtype, int op,
                          DmTreePlan &pl) {
  const size_t n = sc.ops.size();
  pl.tree_at.assign(n, -1);
  pl.host.assign(n, -1);
  pl.hosted.assign(n, -1);
  pl.defer.assign(n, 0);
  pl.spec.resize(n);
  pl.leaves.resize(n);
  if (!tx.stream_ordered() || !on || op < 0) return false;
  auto sends_of = [&](size_t x, std::vector<XSend> &s) {
    s.clear();
    for (const Prim &p : sc.ops[x].prims)
      if (p.type == BINE_PRIM_SEND) s.push_back({p.peer, ptr(p.src_buf, p.src_off), p.count * esz});
  };
  auto recvs_of = [&](size_t x, std::vector<XRecv> &r) {
    r.clear();
    for (const Prim &p : sc.ops[x].prims)
      if (p.type == BINE_PRIM_RECV) r.push_back({p.peer, ptr(p.dst_buf, p.dst_off), p.count * esz});
  };
  auto overlaps = [](const char *a, size_t na, const char *b, size_t nb) { return a < b + nb && b < a + na; };
  // buffers only receives write and only trees read (staging areas)
  bool clean_buf[8];
  for (int b = 0; b < 8; b++) clean_buf[b] = true;
  for (const SOp &o : sc.ops)
    for (const Prim &x : o.prims) {
      const bool tree = x.type == BINE_PRIM_REDUCE_TREE, recv = x.type == BINE_PRIM_RECV;
      auto dirty = [&](int b) { if (b >= 0 && b < 8) clean_buf[b] = false; };
      if (!tree && !recv) dirty(x.src_buf);
      dirty(x.aux_buf);
      if (!recv) dirty(x.dst_buf);
    }
  bool any = false;
  std::vector<XSend> s, s2;
  std::vector<XRecv> r, r2;
  for (size_t i = 0; i < n; i++) {
    if (!sc.ops[i].xchg) continue;
    size_t j = i + 1;
    while (j < n && sc.ops[j].xchg) j++;
    if (j >= n || sc.ops[j].wait != (int64_t)i || sc.ops[j].prims.size() != 1 ||
        sc.ops[j].prims[0].type != BINE_PRIM_REDUCE_TREE)
      continue;
    const Prim &t = sc.ops[j].prims[0];
    // the staging buffer: only receives write it, only trees read it
    if (t.src_buf < 0 || t.src_buf >= 8 || !clean_buf[t.src_buf]) continue;
    TreeSpec ts;
    ts.nl = t.peer;
    ts.pos = t.pos;
    ts.swap = (unsigned)t.flags >> 8;
    ts.own_leaf = ptr(t.aux_buf, t.aux_off);
    ts.out = ptr(t.dst_buf, t.dst_off);
    ts.leaf_bytes = t.count * esz;
    ts.dtype = dtype;
    ts.op = op;
    bool ok = t.peer >= 2;
    for (const Prim &x : sc.ops[i].prims) {
      if (x.type != BINE_PRIM_RECV) continue;
      if (x.dst_buf != t.src_buf || x.count != t.count || x.dst_off < t.src_off || (x.dst_off - t.src_off) % t.count) {
        ok = false;
        break;
      }
      const uint64_t k = (x.dst_off - t.src_off) / t.count;
      if (k >= (uint64_t)t.peer - 1) {
        ok = false;
        break;
      }
      ts.leaf_of_recv.push_back((int)k < t.pos ? (int)k : (int)k + 1);
    }
    if (!ok) continue;
    sends_of(i, s);
    recvs_of(i, r);
    // deferred into the next exchange i2
    size_t i2 = i + 1;
    while (i2 < n && !sc.ops[i2].xchg) i2++;
    bool dfr = i2 < n && ((i2 == i + 1 && i2 < j) || i2 == j + 1) && pl.hosted[i2] < 0 &&
               sc.ops[i2].wait != (int64_t)j;
    if (dfr) {
      sends_of(i2, s2);
      recvs_of(i2, r2);
      for (const XSend &x : s2) dfr = dfr && !overlaps((const char *)x.ptr, x.bytes, ts.out, ts.leaf_bytes);
      for (const XRecv &x : r2)
        dfr = dfr && !overlaps((const char *)x.ptr, x.bytes, ts.out, ts.leaf_bytes) &&
              !overlaps((const char *)x.ptr, x.bytes, ts.own_leaf, ts.leaf_bytes);
      dfr = dfr && tx.defer_ok(s2, r2, r, ts);
    }
    size_t hx = n;
    if (dfr) {
      hx = i2;
      pl.defer[i] = 1;
    } else if (pl.hosted[i] < 0) {
      bool own = true;  // in its own exchange: the output is written while the pushes still read
      for (const XSend &x : s) own = own && !overlaps((const char *)x.ptr, x.bytes, ts.out, ts.leaf_bytes);
      if (own && tx.tree_ok(s, r, ts)) hx = i;
    }
    if (hx == n && tx.defer_ok({}, {}, r, ts)) {
      // no exchange can take it (i already hosts the previous chunk's tree,
      // and nothing follows -- the last chunk): the tree op itself becomes a
      // launch of its own on the comm stream that pulls i's leaves in place
      hx = j;
      pl.defer[i] = 1;
    }
    if (hx == n) continue;
    pl.tree_at[j] = (int)i;
    pl.host[j] = (int)hx;
    pl.hosted[hx] = (int)j;
    pl.leaves[j] = r;
    pl.spec[j] = std::move(ts);
    any = true;
  }
  pl.any = any;
  pl.solo = any;
  for (size_t j = 0; j < n && pl.solo; j++)
    if (!sc.ops[j].xchg && pl.host[j] < 0) pl.solo = false;
  return any;
}

// tp: the call's fused-tree plan (tree_plan_for; null: none).  With tp->solo
// every local op is a tree hosted by an exchange launch, so nothing is left to
// overlap on a second stream: the whole call goes to K -- no cross-stream
// events at all, and graph mode captures it as one branch (§4.3 of DESIGN.md)
static int execute(bine_comm *c, const Schedule &sc, const void *sbuf, void *rbuf, size_t esz, int dtype, int op,
                   hipStream_t K, bool single = false, bool joined = false, const Staging *stg = nullptr,
                   const DmTreePlan *tpl = nullptr, bool fused = false) {
  char *base[6];
  base[BINE_BUF_SBUF] = (char *)sbuf;
  base[BINE_BUF_RBUF] = (char *)rbuf;
  for (int t = 0; t < 3; t++) base[BINE_BUF_TMP0 + t] = (char *)c->tmp[t];
  base[BINE_BUF_STAGE] = (char *)c->tmp[3];
  auto ptr = [&](int buf, uint64_t off) { return base[buf] + off * esz; };
  // over the direct transport, a small collective (and a large one that
  // run_collective found fusable, `fused`) is one launch when its form allows
  if ((single || fused) && !stg) {
    const int rc = try_fused(c, sc, ptr, esz, dtype, op, single, K);
    if (rc >= 0) return rc;
  }
  const bool solo = tpl && tpl->solo && !single && !stg;
  hipStream_t C = single || solo ? K : c->cstream;
  // host staging: the host -> device copies overwrite the device input (and,
  // in place, the output) that the previous call's ops may still read or
  // write: the h2d stream follows K first (K follows the previous call's comm
  // stream and d2h copies -- final_wait / the joins at the end of execute)
  if (stg && stg->in_host)
    if (int rc = stream_join(c, stg->h2d, K)) return rc;
  // stream-ordered transports (direct: sequence bases in device memory) need
  // every exchange of this call after every exchange of the previous one,
  // whichever stream that one used: the comm stream follows K at the start
  // and K follows the comm stream at the end
  const bool ordered = c->tx->stream_ordered() && !single && !solo;
  if ((sc.c_join || ordered) && !single && !solo && !joined) {  // joined: the comm stream already follows K (graph capture)
    int rc = stream_join(c, C, K);
    if (rc) return rc;
  }
  // fused trees: the comm stream follows K again only when K has work of its
  // own since it last did (k_dirty), and K takes up a tree's place lazily --
  // it waits for the newest hosting launch (k_pending) just before its next
  // own op.  With every tree hosted on the comm stream K stays idle, and its
  // joins -- a barrier packet on each stream per chunk -- would only add gaps
  // between the exchange launches
  bool k_dirty = C != K && !(joined || ((sc.c_join || ordered) && !single));
  hipEvent_t k_pending = nullptr;
  std::vector<hipEvent_t> &evs = c->op_ev;
  evs.resize(sc.ops.size());
  const bool prof = c->profile;
  if (prof) {
    if (c->prof.size() < sc.ops.size()) c->prof.resize(sc.ops.size());
    c->prof_n = sc.ops.size();
  }
  // profile events of op i on stream s (begin: its fields and start event)
  auto prof_begin = [&](size_t i, hipStream_t s) -> int {
    const SOp &o = sc.ops[i];
    auto &pt = c->prof[i];
    if (!pt.a) HIP_TRY(hipEventCreate(&pt.a));
    if (!pt.b) HIP_TRY(hipEventCreate(&pt.b));
    pt.xchg = o.xchg ? 1 : 0;
    pt.nprims = (int)o.prims.size();
    pt.bytes = 0;
    for (const Prim &x : o.prims) {  // exchanges: bytes sent; local ops: algorithmic HBM bytes
      if (x.type == BINE_PRIM_SEND) pt.bytes += x.count * esz;
      else if (x.type == BINE_PRIM_REDUCE || x.type == BINE_PRIM_REDUCE3) pt.bytes += 3 * x.count * esz;
      else if (x.type == BINE_PRIM_REDUCE_TREE) pt.bytes += (uint64_t)(x.peer + 1) * x.count * esz;
      else if (x.type == BINE_PRIM_COPY) pt.bytes += 2 * x.count * esz;
    }
    HIP_TRY(hipEventRecord(pt.a, s));
    return BINE_SUCCESS;
  };
  auto prof_end = [&](size_t i, hipStream_t s) -> int {
    HIP_TRY(hipEventRecord(c->prof[i].b, s));
    return BINE_SUCCESS;
  };
  std::vector<XSend> &sends = c->xs;
  std::vector<XRecv> &recvs = c->xr;
  // staging: the input buffer's device copy (SBUF, or RBUF in place) and the
  // h2d batches' events; per stream, the newest batch already waited for
  char *in_dev = sbuf == rbuf ? base[BINE_BUF_RBUF] : base[BINE_BUF_SBUF];
  std::vector<hipEvent_t> &hev = c->stage_ev;
  if (stg) hev.assign(sc.ops.size(), nullptr);
  int64_t h_waited[2] = {-1, -1};
  // trees evaluated inside an exchange launch (direct transport; plan_dm_trees)
  static const DmTreePlan no_trees;
  const DmTreePlan &tp = tpl ? *tpl : no_trees;
  const bool dm_trees = !single && !stg && tpl && tpl->any;
  std::vector<hipEvent_t> &tev = c->tree_ev;
  std::vector<char> &tpend = c->tree_pending;
  if (dm_trees) {
    tev.assign(sc.ops.size(), nullptr);
    tpend.assign(sc.ops.size(), 0);
  }
  for (size_t i = 0; i < sc.ops.size(); i++) {
    const SOp &o = sc.ops[i];
    hipStream_t st = o.xchg ? C : K;
    if (dm_trees && tp.host[i] == (int)i) {
      // a tree hosted by itself: its own launch on the comm stream pulls the
      // leaves in place (after the exchange that was issued without them)
      if (k_dirty && C != K) {
        if (int rj = stream_join(c, C, K)) return rj;
        k_dirty = false;
      }
      static const std::vector<XSend> no_s;
      static const std::vector<XRecv> no_r;
      if (prof)
        if (int rp = prof_begin(i, C)) return rp;
      if (int rc = c->tx->exchange_tree(no_s, no_r, nullptr, &tp.leaves[i], &tp.spec[i], C)) return rc;
      if (prof)
        if (int rp = prof_end(i, C)) return rp;
      tev[i] = next_event(c);
      if (C != K) HIP_TRY(hipEventRecord(tev[i], C));  // (one stream: nothing waits for it)
    }
    if (dm_trees && tp.host[i] >= 0) {
      // profile: a tree inside another exchange's launch has no launch of its
      // own -- a zero-length entry; its time is inside the hosting exchange's
      if (prof && tp.host[i] != (int)i) {
        if (int rp = prof_begin(i, C)) return rp;
        if (int rp = prof_end(i, C)) return rp;
        c->prof[i].nprims = 0;  // nothing launched for it (bine_comm_profile)
        c->prof[i].bytes = 0;
      }
      // this tree runs inside exchange host[i]: K takes up its place in K's
      // order (later local ops follow it as they followed the tree) -- now,
      // or right after the host is issued when that comes next
      if (tev[i]) {
        if (C != K) k_pending = tev[i];
        if (sc.signals[i]) evs[i] = tev[i];
      } else {
        tpend[i] = 1;
      }
      continue;
    }
    if (!o.xchg && k_pending) {  // K's next own op: after every tree hosted so far
      HIP_TRY(hipStreamWaitEvent(K, k_pending, 0));
      k_pending = nullptr;
    }
    if (!o.xchg) k_dirty = true;
    if (trace_on())
      fprintf(stderr, "bine[%d] op %zu/%zu %s wait %lld prims %zu\n", c->rank, i, sc.ops.size(),
              o.xchg ? "xchg" : "local", (long long)o.wait, o.prims.size());
    if (stg && stg->in_host) {
      const StageRanges &g = *stg->rg;
      if (!g.h2d[i].empty()) {
        for (const Ivl &r : g.h2d[i])
          HIP_TRY(hipMemcpyAsync(in_dev + r.first * esz, stg->in_host + r.first * esz, (r.second - r.first) * esz,
                                 hipMemcpyHostToDevice, stg->h2d));
        hev[i] = next_event(c);
        HIP_TRY(hipEventRecord(hev[i], stg->h2d));
      }
      const int64_t w = g.h2d_wait[i];
      int64_t &hw = h_waited[st == K ? 0 : 1];
      if (w > hw) {
        HIP_TRY(hipStreamWaitEvent(st, hev[(size_t)w], 0));
        hw = w;
      }
    }
    if (o.wait >= 0 && !single && !solo) HIP_TRY(hipStreamWaitEvent(st, evs[(size_t)o.wait], 0));
    if (roctx_on()) {
      char lbl[64];
      snprintf(lbl, sizeof lbl, "bine op %zu %s (%zu prims)", i, o.xchg ? "exchange" : "local", o.prims.size());
      roctxRangePushA(lbl);
    }
    if (prof)
      if (int rp = prof_begin(i, st)) return rp;
    int rc = BINE_SUCCESS;
    if (o.xchg) {
      sends.clear();
      recvs.clear();
      for (const Prim &x : o.prims) {
        if (x.type == BINE_PRIM_SEND) sends.push_back({x.peer, ptr(x.src_buf, x.src_off), x.count * esz});
        else recvs.push_back({x.peer, ptr(x.dst_buf, x.dst_off), x.count * esz});
      }
      const int hj = dm_trees ? tp.hosted[i] : -1;
      if (dm_trees && tp.defer[i]) recvs.clear();  // pulled by the next exchange, for its tree
      if (hj >= 0) {
        // the tree reads the own leaf and writes its output where K's earlier
        // ops may still be writing / reading: C follows K first (if K has
        // had any since C last did)
        if (k_dirty && C != K) {
          if (int rj = stream_join(c, C, K)) return rj;
          k_dirty = false;
        }
        const bool own = tp.tree_at[(size_t)hj] == (int)i;
        rc = own ? c->tx->exchange_tree(sends, recvs, &tp.spec[(size_t)hj], nullptr, nullptr, C)
                 : c->tx->exchange_tree(sends, recvs, nullptr, &tp.leaves[(size_t)hj], &tp.spec[(size_t)hj], C);
        if (rc) return rc;
        hipEvent_t e = next_event(c);
        if (C != K) HIP_TRY(hipEventRecord(e, C));
        tev[(size_t)hj] = e;
        if (tpend[(size_t)hj]) {  // the tree's place in K's order came first
          if (C != K) k_pending = e;
          if (sc.signals[(size_t)hj]) evs[(size_t)hj] = e;
        }
      } else {
        rc = a2a_shape(c, sends, recvs) ? c->tx->alltoallv(sends, recvs, C) : c->tx->exchange(sends, recvs, C);
      }
      if (rc) return rc;
    } else {
      rc = run_local(o.prims, ptr, dtype, op, esz, K);
      if (rc) { set_err("local primitive failed (%s)", bine_status_string(rc)); return rc; }
    }
    if (prof)
      if (int rp = prof_end(i, st)) return rp;
    if (roctx_on()) roctxRangePop();
    // an event of the pool may be re-recorded by a later op once the pool
    // wraps: any later record only delays a waiter, never lets it run early.
    // Ops nothing waits for record no event (host cost per op).
    if (sc.signals[i] && !single && !solo) {
      evs[i] = next_event(c);
      HIP_TRY(hipEventRecord(evs[i], st));
    }
    if (stg && stg->out_host && !stg->rg->d2h[i].empty()) {  // pieces of the output this op wrote last
      if (int rc = stream_join(c, stg->d2h, st)) return rc;
      for (const Ivl &r : stg->rg->d2h[i])
        HIP_TRY(hipMemcpyAsync(stg->out_host + r.first * esz, base[BINE_BUF_RBUF] + r.first * esz,
                               (r.second - r.first) * esz, hipMemcpyDeviceToHost, stg->d2h));
    }
  }
  if (stg && stg->out_host) {  // the caller's stream ends after the last copy back
    if (int rc = stream_join(c, K, stg->d2h)) return rc;
  }
  if (k_pending && !ordered) HIP_TRY(hipStreamWaitEvent(K, k_pending, 0));  // (ordered: the join below covers it)
  if (sc.final_wait >= 0 && !single && !solo) HIP_TRY(hipStreamWaitEvent(K, evs[(size_t)sc.final_wait], 0));
  if (ordered) return stream_join(c, K, C);
  return BINE_SUCCESS;
}

// pipelining chunk in elements, kept 16-B aligned (0 = no chunking)
static size_t chunk_elems(size_t chunk_bytes, size_t esz) {
  size_t ch = chunk_bytes / esz;
  if (!ch) return 0;
  const size_t v = 16 / esz;
  return std::max(v, ch / v * v);
}

static std::string plan_key(const PlanArgs &a) {
  std::string k;
  char buf[160];
  snprintf(buf, sizeof buf, "%d|%zu|%zu|%zu|%d|%d|%d|%d|%d|", a.algo, a.count, a.esz, a.segsize, (int)a.in_place,
           a.root, (int)a.flat_ag, (int)a.flat_ag_chunked, (int)a.flat_rs);
  k = buf;
  for (int x : a.rcounts) { k += std::to_string(x); k += ','; }
  return k;
}

// own plan + issue schedule; relay mode needs every rank's plan
static void build(const PlanArgs &args, size_t ch, size_t relay_min_bytes, bool trees, Plan &plan, Schedule &sc) {
  PlanArgs a = args;
  a.flat_chunk = ch;  // the flat reduce-scatter is chunked by the planner itself
  if (trees) plan = make_tree_plan(a);
  if (!trees || plan.status == BINE_ERR_UNSUPPORTED) plan = make_plan(a);
  if (plan.status != BINE_SUCCESS) return;
  SchedCfg cfg;
  cfg.chunk = ch;
  cfg.in_place = a.in_place;
  if (relay_min_bytes && a.P >= 3) {
    cfg.relay_min = std::max<size_t>(1, (relay_min_bytes + a.esz - 1) / a.esz);
    std::vector<Plan> all((size_t)a.P);
    for (int x = 0; x < a.P; x++) {
      PlanArgs b = a;
      b.rank = x;
      all[(size_t)x] = x == a.rank ? plan : make_plan(b);
    }
    make_schedule(plan, &all, a.rank, cfg, sc);
  } else {
    make_schedule(plan, nullptr, a.rank, cfg, sc);
  }
}

// The call's fused-tree plan (plan_dm_trees), cached per (plan, the buffers'
// addresses, dtype, op, the direct transport's settings): null when the call
// has none (no direct transport, trees off, single-stream or staged calls)
static const DmTreePlan *tree_plan_for(bine_comm *c, const std::string &plan_key_s, const Schedule &sc,
                                       const void *sbuf, void *rbuf, size_t esz, int dtype, int op) {
  auto *rt = dynamic_cast<const RcclTransport *>(c->tx.get());
  if (!rt || !rt->dm_on || !rt->dm || !c->dm_tree || op < 0) return nullptr;
  char buf[256];
  snprintf(buf, sizeof buf, "|%p|%p|%p|%p|%p|%p|%d|%d|%zu|%d|%zu|%d", sbuf, rbuf, c->tmp[0], c->tmp[1], c->tmp[2],
           c->tmp[3], dtype, op, esz, rt->dm->merge, rt->dm->slot, rt->dm->tree_wgs);
  const std::string key = plan_key_s + buf;
  auto it = c->tree_cache.find(key);
  if (it == c->tree_cache.end()) {
    if (c->tree_cache.size() >= 256) c->tree_cache.clear();
    char *base[6];
    base[BINE_BUF_SBUF] = (char *)sbuf;
    base[BINE_BUF_RBUF] = (char *)rbuf;
    for (int t = 0; t < 3; t++) base[BINE_BUF_TMP0 + t] = (char *)c->tmp[t];
    base[BINE_BUF_STAGE] = (char *)c->tmp[3];
    auto ptr = [&](int b, uint64_t off) { return base[b] + off * esz; };
    DmTreePlan pl;
    plan_dm_trees(*c->tx, true, sc, ptr, esz, dtype, op, pl);
    it = c->tree_cache.emplace(key, std::move(pl)).first;
  }
  return it->second.any ? &it->second : nullptr;
}

// Whether a large call runs as ONE k_dm_fused launch (build_fused on the
// call's buffers), cached per (plan, buffers, dtype, op, the direct
// transport's settings)
static bool fused_for(bine_comm *c, const std::string &plan_key_s, const Schedule &sc, const void *sbuf, void *rbuf,
                      size_t esz, int dtype, int op) {
  auto *rt = dynamic_cast<const RcclTransport *>(c->tx.get());
  // the large form belongs to the fused-tree setting (bine_comm_set_direct_tree);
  // with it off the per-exchange launches and separate trees stay (A/B)
  if (!rt || !rt->dm_on || !rt->dm || op < 0 || c->profile || !fused_large_on() || !c->dm_tree) return false;
  char buf[256];
  snprintf(buf, sizeof buf, "|%p|%p|%p|%p|%p|%p|%d|%d|%zu|%zu", sbuf, rbuf, c->tmp[0], c->tmp[1], c->tmp[2],
           c->tmp[3], dtype, op, esz, rt->dm->slot);
  const std::string key = plan_key_s + buf;
  auto it = c->fused_cache.find(key);
  if (it == c->fused_cache.end()) {
    if (c->fused_cache.size() >= 256) c->fused_cache.clear();
    char *base[6];
    base[BINE_BUF_SBUF] = (char *)sbuf;
    base[BINE_BUF_RBUF] = (char *)rbuf;
    for (int t = 0; t < 3; t++) base[BINE_BUF_TMP0 + t] = (char *)c->tmp[t];
    base[BINE_BUF_STAGE] = (char *)c->tmp[3];
    auto ptr = [&](int b, uint64_t off) { return base[b] + off * esz; };
    std::vector<DmFusedArgs> v;
    it = c->fused_cache.emplace(key, plan_fused(c, sc, ptr, esz, dtype, op, false, v)).first;
  }
  return it->second;
}

// Graph mode: the first call for a (plan, buffers, dtype, op, stream,
// transport options) key runs eagerly -- RCCL connects to new peers lazily and
// the allgather option sizes its staging area, neither of which may happen
// inside a capture -- and then captures the same execute() on K without
// running it: the comm stream joins the capture through the schedule's event
// hand-offs (c_join forks it from K, final_wait joins it back), and RCCL's
// grouped P2P launches are captured as RCCL supports.  Every later call with
// that key replays the graph with one hipGraphLaunch.  Work and ordering are
// the eager schedule's, so results are bit-identical (GPU tests).
static int run_graph(bine_comm *c, const std::string &plan_key_s, const Schedule &sc, const void *sbuf, void *rbuf,
                     size_t esz, int dtype, int op, hipStream_t K, bool single, const DmTreePlan *tpl, bool fused) {
  const bool one = single || fused || (tpl && tpl->solo);  // the whole call on K: a one-branch graph
  const auto *rt = dynamic_cast<const RcclTransport *>(c->tx.get());
  char buf[192];
  snprintf(buf, sizeof buf, "|%p|%p|%d|%d|%p|%d|%d|%d|%d", sbuf, rbuf, dtype, op, (void *)K, (int)single,
           (int)c->coll_a2a, rt && rt->coll_ag ? 1 : 0, rt && rt->dm_on ? 1 : 0);
  const std::string key = plan_key_s + buf;
  if (int rc = c->tx->health()) return rc;  // a replay would not pass through exchange()'s check
  auto it = c->graph_cache.find(key);
  if (it != c->graph_cache.end()) {
    HIP_TRY(hipGraphLaunch(it->second.x, K));
    return BINE_SUCCESS;
  }
  int rc = execute(c, sc, sbuf, rbuf, esz, dtype, op, K, single, false, nullptr, tpl, fused);  // this call, eagerly
  if (rc) return rc;
  if (rt && rt->stage_gen != c->graph_stage_gen) {
    // the allgather option's staging area moved (freed after a synchronize of
    // the comm stream, which follows every earlier graph launch on K): drop
    // the graphs that still point into the old one
    HIP_TRY(hipStreamSynchronize(K));
    HIP_TRY(hipStreamSynchronize(c->cstream));
    c->drop_graphs();
    c->graph_stage_gen = rt->stage_gen;
  }
  if (c->graph_cache.size() >= 64) {  // bound the cache: drain, then drop every graph
    HIP_TRY(hipStreamSynchronize(K));
    HIP_TRY(hipStreamSynchronize(c->cstream));
    c->drop_graphs();
  }
  // Capture origin: K for single-stream schedules; the COMM stream otherwise,
  // with K forked from it and joined back at the end.  RCCL's captured P2P
  // launches must sit on the capture's origin stream: with K as origin and the
  // comm stream forked in, hipStreamEndCapture segfaulted (RCCL 2.26.6 / HIP
  // 7.0, both capture modes; tools/graph_probe.py, profiles/r2_graph_capture.txt).
  bine_comm::GraphEntry e;
  const hipStream_t O = one ? K : c->cstream;
  HIP_TRY(hipStreamBeginCapture(O, hipStreamCaptureModeThreadLocal));
  if (!one) rc = stream_join(c, K, O);
  if (!rc) rc = execute(c, sc, sbuf, rbuf, esz, dtype, op, K, single, true, nullptr, tpl, fused);
  if (!rc && !one) rc = stream_join(c, O, K);
  const hipError_t ee = hipStreamEndCapture(O, &e.g);
  if (rc || ee != hipSuccess) {
    if (e.g) (void)hipGraphDestroy(e.g);
    if (!rc) set_err("graph capture of the collective failed: %s", hipGetErrorString(ee));
    return rc ? rc : BINE_ERR_HIP;
  }
  const hipError_t ie = hipGraphInstantiate(&e.x, e.g, nullptr, nullptr, 0);
  if (ie != hipSuccess) {
    (void)hipGraphDestroy(e.g);
    set_err("hipGraphInstantiate: %s", hipGetErrorString(ie));
    return BINE_ERR_HIP;
  }
  c->graph_cache.emplace(key, e);
  return BINE_SUCCESS;
}

// Graphs with parallel branches (a two-stream schedule: comm stream + the
// caller's) only on HIP >= 7.2.  The 7.0.51831 runtime torch bundles crashes
// in hipGraphLaunch -> GraphExec::Run -> Graph::UpdateStreams, which skips
// every parallel stream sharing the launch stream's hardware queue and reads
// past the end of its vector when all do (always under GPU_MAX_HW_QUEUES=1);
// libbine-free repro tools/graph_fork_repro.{cpp,py}, symbolised stack and
// disassembly in profiles/r4_graph_fork_repro.txt.  /opt/rocm's 7.2 runtime
// (libbine.so under pico_core) replays the same graph.  On 7.0 a multi-stream
// schedule therefore runs eagerly in graph mode, and so does every schedule
// with RCCL calls in it: RCCL forks streams of its own inside a capture, so
// even a single-stream schedule becomes a graph with parallel branches (the
// 4-process RCCL matrix's graph pass crashed on 7.0 with 1 and with 2 HW
// queues per process; it replays with HIP's default 4, where some parallel
// stream lands on another queue).  What 7.0 captures: single-stream
// schedules over the direct transport (our kernels only, one branch) with at
// least 2 HW queues, and single-stream RCCL schedules with at least 4.
static bool multi_branch_graphs_ok() {
  static const bool v = [] {
    int rt = 0;
    return hipRuntimeGetVersion(&rt) == hipSuccess && rt >= 70200000;
  }();
  return v;
}
// the call makes no RCCL calls: one rank (no exchanges), or its exchanges go
// to the direct transport (not poisoned)
static bool rccl_free(const bine_comm *c) {
  const auto *rt = dynamic_cast<const RcclTransport *>(c->tx.get());
  return c->size == 1 || (rt && rt->dm_on && rt->dm && !rt->dm->poisoned());
}
// HIP's hardware queues per stream priority (GPU_MAX_HW_QUEUES, default 4)
static int hw_queues() {
  static const int v = getenv("GPU_MAX_HW_QUEUES") ? atoi(getenv("GPU_MAX_HW_QUEUES")) : 4;
  return v;
}

// chunk_bytes == kCommChunk: the communicator's setting (bine_comm_set_chunk)
constexpr size_t kCommChunk = ~(size_t)0;
// op of the data-movement collectives (allgather family): no reduction runs
constexpr int kOpNone = -1;

// `stg` (host staging, bine_*_staged): the flat forms are forced on for the
// call (bit-identical; the allgather cut with the reduce-scatter's chunks, so
// the output completes chunk by chunk), never graph-captured
static int run_collective(bine_comm *c, PlanArgs &a, const void *sbuf, void *rbuf, int dtype, int op,
                          size_t chunk_bytes, void *stream, Staging *stg = nullptr) {
  if (!c) return BINE_ERR_ARG;
  if (dtype < 0 || dtype >= BINE_NUM_DTYPES) return BINE_ERR_UNSUPPORTED;
  if (op != kOpNone) {
    if (op < 0 || op >= BINE_NUM_OPS) return BINE_ERR_UNSUPPORTED;
    // (op, type) pairs MPICH's MPI_Reduce_local rejects (MPI_ERR_OP): refused
    // before any exchange, identically on every rank
    if (!bine_op_valid(dtype, op)) return BINE_ERR_ARG;
  }
  std::lock_guard<std::mutex> g(c->mu);
  if (chunk_bytes == kCommChunk) {
    const auto *rt = dynamic_cast<const RcclTransport *>(c->tx.get());
    chunk_bytes = c->chunk_bytes ? c->chunk_bytes : default_chunk_bytes(rt && rt->dm_on);
  }
  HIP_TRY(hipSetDevice(c->device));
  a.P = c->size;
  a.rank = c->rank;
  a.esz = bine_dtype_size(dtype);
  a.in_place = sbuf == BINE_IN_PLACE;
  a.flat_ag = c->flat_ag != 0 || stg;
  a.flat_ag_chunked = c->flat_ag == 2 || stg;
  a.flat_rs = c->flat_rs || stg;
  const size_t ch = chunk_elems(chunk_bytes, a.esz);
  const std::string key = plan_key(a) + "|" + std::to_string(ch) + "|" + std::to_string(c->relay_min_bytes) +
                          (c->trees ? "|T" : "");
  auto it = c->plans.find(key);
  if (it == c->plans.end()) {
    std::pair<Plan, Schedule> v;
    build(a, ch, c->relay_min_bytes, c->trees, v.first, v.second);
    it = c->plans.emplace(key, std::move(v)).first;
  }
  const Plan &plan = it->second.first;
  const Schedule &sc = it->second.second;
  if (plan.status != BINE_SUCCESS) return plan.status;
  hipStream_t K = (hipStream_t)stream;  // NULL = the HIP null stream, as in every HIP / RCCL API
  c->last_user = K;
  c->used_user = true;
  const uint64_t need[4] = {plan.tmp_elems[0], plan.tmp_elems[1], plan.tmp_elems[2], sc.stage_elems};
  int rc = ensure_workspace(c, need, a.esz, K);
  if (rc) return rc;
  uint64_t bytes = (uint64_t)a.count;
  for (int x : a.rcounts) bytes += (uint64_t)x;
  bytes *= a.esz;
  if (roctx_on()) {
    char lbl[96];
    snprintf(lbl, sizeof lbl, "bine %s P=%d count=%zu", bine_algo_name(a.algo), a.P, a.count);
    roctxRangePushA(lbl);
  }
  // one rank: local ops only, so one stream (and a one-branch graph)
  bool single = bytes <= c->single_stream_bytes || c->size == 1;
  if (stg) {
    auto sit = c->stage_cache.find(key);
    if (sit == c->stage_cache.end()) {
      StageRanges g;
      stage_ranges(sc, a.in_place, g);
      sit = c->stage_cache.emplace(key, std::move(g)).first;
    }
    stg->rg = &sit->second;
  }
  const void *src = a.in_place ? rbuf : sbuf;
  const bool fused = !single && !stg && fused_for(c, key, sc, src, rbuf, a.esz, dtype, op);
  const DmTreePlan *tpl = single || stg || fused ? nullptr : tree_plan_for(c, key, sc, src, rbuf, a.esz, dtype, op);
  // ranks sharing ONE GPU over the direct transport (opt-in): a call that
  // would hand its chunks between the comm stream and the caller's stream (no
  // one-launch form, no trees inside the exchanges) runs on the caller's
  // stream alone -- with 8 processes on one GPU those hand-offs cost 100-1,300
  // ms per C3 call, one stream 3-4 ms (DESIGN.md 7.2,
  // profiles/r6_single_stream_shared.txt)
  if (!single && !fused && !tpl && shared_gpu_direct(c)) single = true;
  rc = order_begin(c, K);
  if (rc) {
  } else if (c->graphs && K && !c->hub && !c->profile && !roctx_on() && !trace_on() && !stg &&
             (multi_branch_graphs_ok() ||
              ((single || fused || (tpl && tpl->solo)) && hw_queues() >= (rccl_free(c) ? 2 : 4))))
    rc = run_graph(c, key, sc, src, rbuf, a.esz, dtype, op, K, single, tpl, fused);
  else
    rc = execute(c, sc, src, rbuf, a.esz, dtype, op, K, single, false, stg, tpl, fused);
  if (!rc) rc = order_end(c, K);
  if (roctx_on()) roctxRangePop();
  return rc;
}

}  // namespace bine

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------

using namespace bine;

template <typename F>
static int run_threads(bine_comm_t *comms, int n, int *statuses, F f) {
  std::vector<std::thread> th;
  std::vector<int> st((size_t)n, BINE_SUCCESS);
  for (int r = 0; r < n; r++)
    th.emplace_back([&, r] {
      int rc = f(r);
      if (rc == BINE_SUCCESS) rc = bine_comm_synchronize(comms[r]);
      if (comms[r]->tx) comms[r]->tx->retire();
      st[(size_t)r] = rc;
    });
  for (auto &t : th) t.join();
  int first = BINE_SUCCESS;
  for (int r = 0; r < n; r++) {
    if (statuses) statuses[r] = st[(size_t)r];
    if (first == BINE_SUCCESS) first = st[(size_t)r];
  }
  return first;
}


extern "C" {

const char *bine_status_string(int s) {
  switch (s) {
    case BINE_SUCCESS: return "success";
    case BINE_ERR_ARG: return "invalid argument (reference: MPI_ERR_ARG)";
    case BINE_ERR_SIZE: return "unsupported communicator size (reference: MPI_ERR_SIZE)";
    case BINE_ERR_NO_MEM: return "out of memory";
    case BINE_ERR_HIP: return "HIP runtime error";
    case BINE_ERR_RCCL: return "RCCL error";
    case BINE_ERR_UNSUPPORTED: return "unsupported algorithm, datatype or operator";
    case BINE_ERR_ROOT: return "unsupported root (reference: MPI_ERR_ROOT)";
    case BINE_ERR_COUNT: return "count below the number of ranks (reference: MPI_ERR_COUNT)";
    default: return "internal error";
  }
}

const char *bine_last_error(void) { return g_err.c_str(); }

int bine_op_valid(int dtype, int op) {
  if (dtype < 0 || dtype >= BINE_NUM_DTYPES || op < 0 || op >= BINE_NUM_OPS) return 0;
  const bool pair = dtype >= BINE_FLOAT_INT && dtype <= BINE_SHORT_INT, loc = op == BINE_MAXLOC || op == BINE_MINLOC;
  if (pair != loc) return 0;  // pair types under MAXLOC / MINLOC only, and those ops on pairs only
  if (dtype == BINE_C_FLOAT_COMPLEX || dtype == BINE_C_DOUBLE_COMPLEX) return op == BINE_SUM || op == BINE_PROD;
  if ((op == BINE_BAND || op == BINE_BOR || op == BINE_BXOR) && (dtype == BINE_FLOAT || dtype == BINE_DOUBLE))
    return 0;  // no bitwise ops on floating types
  return 1;
}

size_t bine_dtype_size(int dt) {
  switch (dt) {
    case BINE_INT8: case BINE_UINT8: return 1;
    case BINE_INT16: case BINE_UINT16: return 2;
    case BINE_INT32: case BINE_UINT32: case BINE_FLOAT: return 4;
    case BINE_INT64: case BINE_UINT64: case BINE_DOUBLE: return 8;
    case BINE_FLOAT_INT: case BINE_2INT: case BINE_SHORT_INT: return 8;
    case BINE_DOUBLE_INT: case BINE_LONG_INT: return 16;
    case BINE_C_FLOAT_COMPLEX: return 8;
    case BINE_C_DOUBLE_COMPLEX: return 16;
    default: return 0;
  }
}

static const struct { int algo; const char *coll, *name, *selector; } kAlgos[] = {
    {BINE_AR_RECURSIVEDOUBLING, "allreduce", "recursivedoubling", "recursive_doubling_over"},
    {BINE_AR_RING, "allreduce", "ring", "ring_over"},
    {BINE_AR_RABENSEIFNER, "allreduce", "rabenseifner", "rabenseifner_over"},
    {BINE_AR_BINE_LAT, "allreduce", "bine_lat", "bine_lat_over"},
    {BINE_AR_BINE_BDW_STATIC, "allreduce", "bine_bdw_static", "bine_bdw_static_over"},
    {BINE_AR_BINE_BDW_REMAP, "allreduce", "bine_bdw_remap", "bine_bdw_remap_over"},
    {BINE_AR_BINE_BDW_REMAP_SEGMENTED, "allreduce", "bine_bdw_remap_segmented", "bine_bdw_remap_segmented_over"},
    {BINE_AR_BINE_BLOCK_BY_BLOCK_ANY_EVEN, "allreduce", "bine_block_by_block_any_even", "bine_block_by_block_any_even"},
    {BINE_RS_RECURSIVEHALVING, "reduce_scatter", "recursivehalving", "recursive_halving_over"},
    {BINE_RS_RECURSIVE_DISTANCE_DOUBLING, "reduce_scatter", "recursive_distance_doubling", "recursive_distance_doubling_over"},
    {BINE_RS_RING, "reduce_scatter", "ring", "ring_over"},
    {BINE_RS_BUTTERFLY, "reduce_scatter", "butterfly", "butterfly_over"},
    {BINE_RS_BINE_STATIC, "reduce_scatter", "bine_static", "bine_static_over"},
    {BINE_RS_BINE_SEND_REMAP, "reduce_scatter", "bine_send_remap", "bine_send_remap_over"},
    {BINE_RS_BINE_PERMUTE_REMAP, "reduce_scatter", "bine_permute_remap", "bine_permute_remap_over"},
    {BINE_RS_BINE_BLOCK_BY_BLOCK, "reduce_scatter", "bine_block_by_block", "bine_block_by_block_over"},
    {BINE_RS_BINE_BLOCK_BY_BLOCK_ANY_EVEN, "reduce_scatter", "bine_block_by_block_any_even", "bine_block_by_block_any_even"},
    {BINE_RD_BINE_LAT, "reduce", "bine_lat", "bine_lat_over"},
    {BINE_RD_BINE_BDW, "reduce", "bine_bdw", "bine_bdw_over"},
    // pico_core_utils.c:125-140
    {BINE_AG_K_BRUCK, "allgather", "k_bruck", "k_bruck_over"},
    {BINE_AG_RECURSIVEDOUBLING, "allgather", "recursivedoubling", "recursive_doubling_over"},
    {BINE_AG_RING, "allgather", "ring", "ring_over"},
    {BINE_AG_SPARBIT, "allgather", "sparbit", "sparbit_over"},
    {BINE_AG_BINE_BLOCK_BY_BLOCK_ANY_EVEN, "allgather", "bine_block_by_block_any_even",
     "bine_block_by_block_over_any_even"},
    {BINE_AG_BINE_BLOCK_BY_BLOCK, "allgather", "bine_block_by_block", "bine_block_by_block_over"},
    {BINE_AG_BINE_PERMUTE_STATIC, "allgather", "bine_permute_static", "bine_permute_static_over"},
    {BINE_AG_BINE_SEND_STATIC, "allgather", "bine_send_static", "bine_send_static_over"},
    {BINE_AG_BINE_PERMUTE_REMAP, "allgather", "bine_permute_remap", "bine_permute_remap_over"},
    {BINE_AG_BINE_SEND_REMAP, "allgather", "bine_send_remap", "bine_send_remap_over"},
    {BINE_AG_BINE_2_BLOCKS, "allgather", "bine_2_blocks", "bine_2_blocks_over"},
    {BINE_AG_BINE_2_BLOCKS_DTYPE, "allgather", "bine_2_blocks_dtype", "bine_2_blocks_dtype_over"},
    // pico_core_utils.c:166-174
    {BINE_BC_SCATTER_ALLGATHER, "bcast", "scatter_allgather", "scatter_allgather_over"},
    {BINE_BC_BINE_LAT, "bcast", "bine_lat", "bine_lat_over"},
    {BINE_BC_BINE_LAT_REVERSED, "bcast", "bine_lat_reversed", "bine_lat_reversed_over"},
    {BINE_BC_BINE_LAT_NEW, "bcast", "bine_lat_new", "bine_lat_new_over"},
    {BINE_BC_BINE_LAT_I_NEW, "bcast", "bine_lat_i_new", "bine_lat_i_new_over"},
    {BINE_BC_BINE_BDW_STATIC, "bcast", "bine_bdw_static", "bine_bdw_static_over"},
    {BINE_BC_BINE_BDW_REMAP, "bcast", "bine_bdw_remap", "bine_bdw_remap_over"},
    // pico_core_utils.c:152, :190, :245
    {BINE_A2A_BINE, "alltoall", "bine", "bine_over"},
    {BINE_GA_BINE, "gather", "bine", "bine_over"},
    {BINE_SC_BINE, "scatter", "bine", "bine_over"},
};

int bine_algo_from_name(const char *coll, const char *name) {
  if (!coll || !name) return -1;
  for (const auto &a : kAlgos) {
    if (strcmp(a.coll, coll)) continue;
    std::string full = std::string(a.coll) + "_" + a.name;
    if (!strcmp(name, a.name) || !strcmp(name, a.selector) || full == name) return a.algo;
  }
  return -1;
}

const char *bine_algo_name(int algo) {
  for (const auto &a : kAlgos)
    if (a.algo == algo) return a.name;
  return "unknown";
}

int bine_reduce_local(const void *in, void *inout, size_t count, int dtype, int op, void *stream) {
  return launch_reduce(in, inout, inout, count, dtype, op, stream);
}

int bine_reduce3(const void *a, const void *b, void *out, size_t count, int dtype, int op, void *stream) {
  return launch_reduce(a, b, out, count, dtype, op, stream);
}

int bine_reduce_batch(int n, const void *const *a, const void *const *b, void *const *out, const size_t *count,
                      int dtype, int op, void *stream) {
  return launch_reduce_batch(n, a, b, out, count, dtype, op, stream);
}

int bine_reduce_tree(int nleaves, const void *const *leaves, void *out, size_t count, int dtype, int op,
                     void *stream) {
  if (!leaves || (!out && count)) return BINE_ERR_ARG;
  return launch_reduce_tree(nleaves, leaves, out, count, dtype, op, stream);
}

int bine_copy(void *dst, const void *src, size_t bytes, void *stream) {
  if ((!dst || !src) && bytes) return BINE_ERR_ARG;
  return launch_copy(dst, src, bytes, stream);
}

int bine_fill_pico(void *buf, size_t count, int dtype, uint32_t seed, void *stream) {
  return launch_fill_pico(buf, count, dtype, seed, stream);
}

int bine_checksum(const void *buf, size_t count, int dtype, uint64_t *out, void *stream) {
  if (!bine_dtype_size(dtype) || !out) return BINE_ERR_ARG;
  return launch_checksum(buf, count, dtype, out, stream);
}

int bine_get_unique_id(void *id) {
  static_assert(sizeof(ncclUniqueId) == BINE_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return BINE_SUCCESS;
}

// RCCL ABI pin.  In a torch process the loader resolves
// librccl.so.1 to torch's bundled RCCL (2.26.6 in this image) although the
// library is compiled against ROCm's headers (2.27.7).  What crosses that
// boundary is exactly: the 128-byte ncclUniqueId, the opaque ncclComm_t, the
// ncclResult_t / ncclDataType_t / ncclRedOp_t values below, and the argument
// lists of ncclCommInitRank, ncclSend / ncclRecv, ncclGroupStart / End,
// ncclAllGather, ncclAllToAllv, ncclAllReduce, ncclGetVersion,
// ncclGetErrorString, ncclCommDestroy.  (1) Build time: the static_asserts pin
// the compiled headers to those values -- a header that renumbers any of them
// does not compile.  (2) Version window: both the compiled headers and the
// runtime must lie in the window whose ABI for these items was checked
// (header text: 2.27.3 -- rocprofiler-sdk's copy -- and 2.27.7; runtime 2.26.6
// behaviourally, by the GPU suite's every-type RCCL matrix and the probe
// below); anything outside it is refused (bine_rccl_abi_check, a pure function
// with a CPU test).  (3) At communicator creation one grouped probe (abi_probe)
// runs the types and ops the library passes through the RUNTIME and checks
// the results on the host: a runtime that reads any of them differently fails
// the probe instead of corrupting data later.
static_assert(sizeof(ncclUniqueId) == 128 && NCCL_UNIQUE_ID_BYTES == 128, "ncclUniqueId layout");
static_assert(sizeof(ncclComm_t) == sizeof(void *), "ncclComm_t is an opaque pointer");
static_assert(sizeof(ncclResult_t) == 4 && sizeof(ncclDataType_t) == 4 && sizeof(ncclRedOp_t) == 4,
              "enum sizes");
static_assert(ncclSuccess == 0, "ncclResult_t");
static_assert(ncclInt8 == 0 && ncclUint8 == 1 && ncclInt32 == 2 && ncclUint32 == 3 && ncclInt64 == 4 &&
                  ncclUint64 == 5 && ncclFloat32 == 7 && ncclFloat64 == 8,
              "ncclDataType_t numbering");
static_assert(ncclSum == 0 && ncclProd == 1 && ncclMax == 2 && ncclMin == 3, "ncclRedOp_t numbering");
constexpr int kRcclAbiLo = 22600, kRcclAbiHi = 22799;  // 2.26.0 ... 2.27.99
static_assert(NCCL_VERSION_CODE >= kRcclAbiLo && NCCL_VERSION_CODE <= kRcclAbiHi,
              "compiled against RCCL headers outside the checked ABI window");

int bine_rccl_abi_check(int runtime, int compiled) {
  const bool rt_ok = runtime >= kRcclAbiLo && runtime <= kRcclAbiHi;
  const bool ct_ok = compiled >= kRcclAbiLo && compiled <= kRcclAbiHi;
  if (rt_ok && ct_ok) return BINE_SUCCESS;
  set_err("RCCL ABI skew: runtime %d, headers %d; both must lie in the checked window %d..%d", runtime, compiled,
          kRcclAbiLo, kRcclAbiHi);
  return BINE_ERR_RCCL;
}

int bine_rccl_version(int *runtime, int *compiled) {
  int v = 0;
  NCCL_TRY(ncclGetVersion(&v));
  if (runtime) *runtime = v;
  if (compiled) *compiled = NCCL_VERSION_CODE;
  return BINE_SUCCESS;  // a reporter: the refusal is bine_comm_init_rccl's
}

int bine_comm_init_rccl(bine_comm_t *out, int nranks, int rank, const void *id, int device) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks || !id) return BINE_ERR_ARG;
  {
    int v = 0;
    NCCL_TRY(ncclGetVersion(&v));
    if (int rc0 = bine_rccl_abi_check(v, NCCL_VERSION_CODE)) return rc0;  // the version window: refuses a skewed pair
  }
  auto c = std::make_unique<bine_comm>();
  c->rank = rank;
  c->size = nranks;
  c->device = device;
  int rc = comm_setup(c.get());
  if (rc) return rc;
  auto tx = std::make_unique<RcclTransport>();
  tx->rank = rank;
  tx->size = nranks;
  if (const char *e = getenv("BINE_COLL_AG")) tx->coll_ag = atoi(e) != 0;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  uint64_t h = 1469598103934665603ull;  // FNV-1a of the unique id: names the direct transport's sockets
  for (size_t i = 0; i < sizeof u; i++) h = (h ^ ((const unsigned char *)id)[i]) * 1099511628211ull;
  tx->key = h;
  NCCL_TRY(ncclCommInitRank(&tx->comm, nranks, u, rank));
  if (int rc2 = tx->abi_probe()) return rc2;
  c->tx = std::move(tx);
  *out = c.release();
  return BINE_SUCCESS;
}

int bine_comm_init_loopback(bine_comm_t *comms, int nranks, int device) {
  if (!comms || nranks < 1) return BINE_ERR_ARG;
  auto hub = std::make_shared<LoopbackHub>(nranks);
  for (int r = 0; r < nranks; r++) {
    auto c = std::make_unique<bine_comm>();
    c->rank = r;
    c->size = nranks;
    c->device = device;
    int rc = comm_setup(c.get());
    if (rc) {  // undo the ranks already set up
      for (int k = 0; k < r; k++) {
        delete comms[k];
        comms[k] = nullptr;
      }
      return rc;
    }
    c->hub = hub;
    c->tx = std::make_unique<LoopbackTransport>(hub, r);
    comms[r] = c.release();
  }
  return BINE_SUCCESS;
}

// A host wait with a bound (BINE_SYNC_TIMEOUT_S, default 120 s): a stream that
// does not drain in time is reported by name instead of hanging the caller
// (VERDICT r3 item 3).  The work stays enqueued; the communicator's transport
// state is dumped for a direct transport.
static int sync_bounded(bine_comm *c, hipStream_t s, const char *what) {
  static const double limit = getenv("BINE_SYNC_TIMEOUT_S") ? atof(getenv("BINE_SYNC_TIMEOUT_S")) : 120.0;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return BINE_SUCCESS;
    if (q != hipErrorNotReady) {
      set_err("%s stream: %s", what, hipGetErrorString(q));
      return BINE_ERR_HIP;
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > limit) {
      auto *rt = dynamic_cast<RcclTransport *>(c->tx.get());
      const bool dm = rt && rt->dm_on && rt->dm;
      if (dm) rt->dm->dump();
      set_err("rank %d: the %s stream did not drain within %.0f s (BINE_SYNC_TIMEOUT_S)%s%s", c->rank, what, limit,
              dm ? "; direct transport: " : "", dm ? rt->dm->describe(false).c_str() : "");
      return BINE_ERR_INTERNAL;
    }
    if (el > 2e-3) std::this_thread::sleep_for(std::chrono::microseconds(50));  // spin first: short calls
  }
}

int bine_comm_synchronize(bine_comm_t c) {
  if (!c) return BINE_ERR_ARG;
  HIP_TRY(hipSetDevice(c->device));
  if (int rc = sync_bounded(c, c->stream, "compute")) return rc;
  if (int rc = sync_bounded(c, c->cstream, "comm")) return rc;
  if (c->used_user)
    if (int rc = sync_bounded(c, c->last_user, "caller's")) return rc;
  if (c->hub && c->hub->mismatches.load()) {
    set_err("loopback: %d send/recv size mismatches", c->hub->mismatches.load());
    return BINE_ERR_INTERNAL;
  }
  // a direct-transport wait that timed out inside the calls just drained:
  // they completed without their data, so their completion is an error
  //  -- and stays one until bine_comm_set_direct(1)
  // rebuilds the transport or bine_comm_set_direct(0) leaves it
  return c->tx ? c->tx->health_drained() : BINE_SUCCESS;
}

int bine_comm_destroy(bine_comm_t c) {
  if (!c) return BINE_ERR_ARG;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->cstream);
  delete c;
  return BINE_SUCCESS;
}

int bine_comm_rank(bine_comm_t c) { return c ? c->rank : -1; }
int bine_comm_size(bine_comm_t c) { return c ? c->size : -1; }
int bine_comm_device(bine_comm_t c) { return c ? c->device : -1; }
void *bine_comm_stream(bine_comm_t c) { return c ? (void *)c->stream : nullptr; }

int bine_allreduce(bine_comm_t c, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, int op,
                   size_t segsize, void *stream) {
  if (algo < BINE_AR_RECURSIVEDOUBLING || algo > BINE_AR_BINE_BLOCK_BY_BLOCK_ANY_EVEN) return BINE_ERR_UNSUPPORTED;
  PlanArgs a;
  a.algo = algo;
  a.count = count;
  a.segsize = segsize;
  // segmented: the reference's segment is the pipelining chunk (0 = one chunk)
  size_t chunk = algo == BINE_AR_BINE_BDW_REMAP_SEGMENTED ? segsize : (segsize ? segsize : kCommChunk);
  return run_collective(c, a, sbuf, rbuf, dtype, op, chunk, stream);
}

int bine_reduce_scatter(bine_comm_t c, int algo, const void *sbuf, void *rbuf, const int *rcounts, int dtype,
                        int op, void *stream) {
  if (algo < BINE_RS_RECURSIVEHALVING || algo > BINE_RS_BINE_BLOCK_BY_BLOCK_ANY_EVEN) return BINE_ERR_UNSUPPORTED;
  if (!c || !rcounts) return BINE_ERR_ARG;
  PlanArgs a;
  a.algo = algo;
  a.rcounts.assign(rcounts, rcounts + c->size);
  return run_collective(c, a, sbuf, rbuf, dtype, op, kCommChunk, stream);
}

// host staging: `per` = flat pipeline chunk per block piece, from the bytes one
// exchange round carries over all blocks
// host_sbuf / host_rbuf NULL: that buffer is already on the device (dev_sbuf /
// dev_rbuf are the caller's own) and is not copied -- so a rank whose buffers
// live on the device runs the very schedule its host-buffer peers run
static int run_staged(bine_comm_t c, PlanArgs &a, const void *host_sbuf, void *host_rbuf, void *dev_sbuf,
                      void *dev_rbuf, int dtype, int op, size_t chunk_bytes, void *h2d, void *d2h, void *stream) {
  if (!c || !dev_rbuf) return BINE_ERR_ARG;
  const bool in_place = host_sbuf == BINE_IN_PLACE;
  if (!in_place && !dev_sbuf) return BINE_ERR_ARG;
  Staging g;
  g.in_host = (const char *)(in_place ? host_rbuf : host_sbuf);
  g.out_host = (char *)host_rbuf;
  if ((g.in_host && !h2d) || (g.out_host && !d2h)) return BINE_ERR_ARG;
  g.h2d = (hipStream_t)h2d;
  g.d2h = (hipStream_t)d2h;
  const size_t per = std::max<size_t>((chunk_bytes ? chunk_bytes : (size_t)16 << 20) / (size_t)c->size, 64 << 10);
  return run_collective(c, a, in_place ? BINE_IN_PLACE : dev_sbuf, dev_rbuf, dtype, op, per, stream, &g);
}

int bine_allreduce_staged(bine_comm_t c, int algo, const void *host_sbuf, void *host_rbuf, void *dev_sbuf,
                          void *dev_rbuf, size_t count, int dtype, int op, size_t segsize, size_t chunk_bytes,
                          void *h2d_stream, void *d2h_stream, void *stream) {
  if (algo < BINE_AR_RECURSIVEDOUBLING || algo > BINE_AR_BINE_BLOCK_BY_BLOCK_ANY_EVEN) return BINE_ERR_UNSUPPORTED;
  PlanArgs a;
  a.algo = algo;
  a.count = count;
  a.segsize = segsize;
  return run_staged(c, a, host_sbuf, host_rbuf, dev_sbuf, dev_rbuf, dtype, op, chunk_bytes, h2d_stream,
                    d2h_stream, stream);
}

int bine_reduce_scatter_staged(bine_comm_t c, int algo, const void *host_sbuf, void *host_rbuf, void *dev_sbuf,
                               void *dev_rbuf, const int *rcounts, int dtype, int op, size_t chunk_bytes,
                               void *h2d_stream, void *d2h_stream, void *stream) {
  if (algo < BINE_RS_RECURSIVEHALVING || algo > BINE_RS_BINE_BLOCK_BY_BLOCK_ANY_EVEN) return BINE_ERR_UNSUPPORTED;
  if (!c || !rcounts) return BINE_ERR_ARG;
  PlanArgs a;
  a.algo = algo;
  a.rcounts.assign(rcounts, rcounts + c->size);
  return run_staged(c, a, host_sbuf, host_rbuf, dev_sbuf, dev_rbuf, dtype, op, chunk_bytes, h2d_stream,
                    d2h_stream, stream);
}

int bine_reduce(bine_comm_t c, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, int op, int root,
                void *stream) {
  if (algo != BINE_RD_BINE_LAT && algo != BINE_RD_BINE_BDW) return BINE_ERR_UNSUPPORTED;
  if (!c || root < 0 || root >= c->size) return BINE_ERR_ARG;
  PlanArgs a;
  a.algo = algo;
  a.count = count;
  a.root = root;
  if (c->rank == root && sbuf == BINE_IN_PLACE) {
    // handled by run_collective's in_place mapping
  } else if (sbuf == BINE_IN_PLACE) {
    return BINE_ERR_ARG;
  }
  return run_collective(c, a, sbuf, rbuf, dtype, op, kCommChunk, stream);
}

int bine_allgather(bine_comm_t c, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, void *stream) {
  if (algo < BINE_AG_RECURSIVEDOUBLING || algo > BINE_AG_BINE_2_BLOCKS_DTYPE) return BINE_ERR_UNSUPPORTED;
  PlanArgs a;
  a.algo = algo;
  a.count = count;
  // pure data movement: no operator applies (kOpNone skips the (type, op) check)
  return run_collective(c, a, sbuf, rbuf, dtype, kOpNone, kCommChunk, stream);
}

int bine_bcast(bine_comm_t c, int algo, void *buf, size_t count, int dtype, int root, void *stream) {
  if (algo < BINE_BC_SCATTER_ALLGATHER || algo > BINE_BC_BINE_BDW_REMAP) return BINE_ERR_UNSUPPORTED;
  // the communicator size, then the root, are checked by the planner in the
  // reference's order (libbine_bcast.c:198-210): MPI_ERR_SIZE before
  // MPI_ERR_ROOT, also for count == 0
  if (!c) return BINE_ERR_ARG;
  PlanArgs a;
  a.algo = algo;
  a.count = count;
  a.root = root;
  // in place on `buf`; pure data movement (no operator)
  return run_collective(c, a, BINE_IN_PLACE, buf, dtype, kOpNone, kCommChunk, stream);
}

// gather_bine / scatter_bine / alltoall_bine: `count` elements per block; pure
// data movement (no operator)
int bine_gather(bine_comm_t c, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, int root,
                void *stream) {
  if (algo != BINE_GA_BINE) return BINE_ERR_UNSUPPORTED;
  PlanArgs a;
  a.algo = algo;
  a.count = count;
  a.root = root;
  return run_collective(c, a, sbuf, rbuf, dtype, kOpNone, kCommChunk, stream);
}

int bine_scatter(bine_comm_t c, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, int root,
                 void *stream) {
  if (algo != BINE_SC_BINE) return BINE_ERR_UNSUPPORTED;
  PlanArgs a;
  a.algo = algo;
  a.count = count;
  a.root = root;
  return run_collective(c, a, sbuf, rbuf, dtype, kOpNone, kCommChunk, stream);
}

int bine_alltoall(bine_comm_t c, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, void *stream) {
  if (algo != BINE_A2A_BINE) return BINE_ERR_UNSUPPORTED;
  PlanArgs a;
  a.algo = algo;
  a.count = count;
  return run_collective(c, a, sbuf, rbuf, dtype, kOpNone, kCommChunk, stream);
}

int bine_exchange(bine_comm_t c, int nsend, const int *send_peers, const void *const *sbufs, const size_t *sbytes,
                  int nrecv, const int *recv_peers, void *const *rbufs, const size_t *rbytes, void *stream) {
  if (!c || nsend < 0 || nrecv < 0) return BINE_ERR_ARG;
  if (c->hub) return BINE_ERR_UNSUPPORTED;  // loopback: exchanges block on the host (drivers only)
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<XSend> xs;
  std::vector<XRecv> xr;
  for (int i = 0; i < nsend; i++) {
    if (send_peers[i] < 0 || send_peers[i] >= c->size) return BINE_ERR_ARG;
    if (sbytes[i]) xs.push_back({send_peers[i], sbufs[i], sbytes[i]});
  }
  for (int i = 0; i < nrecv; i++) {
    if (recv_peers[i] < 0 || recv_peers[i] >= c->size) return BINE_ERR_ARG;
    if (rbytes[i]) xr.push_back({recv_peers[i], rbufs[i], rbytes[i]});
  }
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t K = (hipStream_t)stream;
  c->last_user = K;
  c->used_user = true;
  int rc = order_begin(c, K);
  if (!rc) rc = stream_join(c, c->cstream, K);
  if (rc) return rc;
  if ((rc = c->tx->exchange(xs, xr, c->cstream))) return rc;
  if ((rc = stream_join(c, K, c->cstream))) return rc;
  return order_end(c, K);
}

int bine_vendor_allreduce(bine_comm_t c, const void *sbuf, void *rbuf, size_t count, int dtype, int op,
                          void *stream) {
  if (!c) return BINE_ERR_ARG;
  if (c->hub) return BINE_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t K = (hipStream_t)stream;
  c->last_user = K;
  c->used_user = true;
  int rc = stream_join(c, c->cstream, K);
  if (rc) return rc;
  if ((rc = c->tx->vendor_allreduce(sbuf, rbuf, count, dtype, op, c->cstream))) return rc;
  return stream_join(c, K, c->cstream);
}

// ---- loopback drivers --------------------------------------------------------

int bine_loopback_run_allreduce(bine_comm_t *comms, int n, int algo, const void *const *sbufs,
                                void *const *rbufs, size_t count, int dtype, int op, size_t segsize,
                                int *statuses) {
  return run_threads(comms, n, statuses, [&](int r) {
    (void)hipSetDevice(comms[r]->device);
    return bine_allreduce(comms[r], algo, sbufs[r], rbufs[r], count, dtype, op, segsize, comms[r]->stream);  // one stream per virtual rank
  });
}

int bine_loopback_run_reduce_scatter(bine_comm_t *comms, int n, int algo, const void *const *sbufs,
                                     void *const *rbufs, const int *rcounts, int dtype, int op, int *statuses) {
  return run_threads(comms, n, statuses, [&](int r) {
    (void)hipSetDevice(comms[r]->device);
    return bine_reduce_scatter(comms[r], algo, sbufs[r], rbufs[r], rcounts, dtype, op, comms[r]->stream);  // one stream per virtual rank
  });
}

int bine_loopback_run_reduce(bine_comm_t *comms, int n, int algo, const void *const *sbufs, void *const *rbufs,
                             size_t count, int dtype, int op, int root, int *statuses) {
  return run_threads(comms, n, statuses, [&](int r) {
    (void)hipSetDevice(comms[r]->device);
    return bine_reduce(comms[r], algo, sbufs[r], rbufs[r], count, dtype, op, root, comms[r]->stream);  // one stream per virtual rank
  });
}

int bine_loopback_run_allgather(bine_comm_t *comms, int n, int algo, const void *const *sbufs, void *const *rbufs,
                                size_t count, int dtype, int *statuses) {
  return run_threads(comms, n, statuses, [&](int r) {
    (void)hipSetDevice(comms[r]->device);
    return bine_allgather(comms[r], algo, sbufs[r], rbufs[r], count, dtype, comms[r]->stream);  // one stream per virtual rank
  });
}

int bine_loopback_run_bcast(bine_comm_t *comms, int n, int algo, void *const *bufs, size_t count, int dtype,
                            int root, int *statuses) {
  return run_threads(comms, n, statuses, [&](int r) {
    (void)hipSetDevice(comms[r]->device);
    return bine_bcast(comms[r], algo, bufs[r], count, dtype, root, comms[r]->stream);  // one stream per virtual rank
  });
}

int bine_loopback_run_gather(bine_comm_t *comms, int n, int algo, const void *const *sbufs, void *const *rbufs,
                             size_t count, int dtype, int root, int *statuses) {
  return run_threads(comms, n, statuses, [&](int r) {
    (void)hipSetDevice(comms[r]->device);
    return bine_gather(comms[r], algo, sbufs[r], rbufs[r], count, dtype, root, comms[r]->stream);
  });
}

int bine_loopback_run_scatter(bine_comm_t *comms, int n, int algo, const void *const *sbufs, void *const *rbufs,
                              size_t count, int dtype, int root, int *statuses) {
  return run_threads(comms, n, statuses, [&](int r) {
    (void)hipSetDevice(comms[r]->device);
    return bine_scatter(comms[r], algo, sbufs[r], rbufs[r], count, dtype, root, comms[r]->stream);
  });
}

int bine_loopback_run_alltoall(bine_comm_t *comms, int n, int algo, const void *const *sbufs, void *const *rbufs,
                               size_t count, int dtype, int *statuses) {
  return run_threads(comms, n, statuses, [&](int r) {
    (void)hipSetDevice(comms[r]->device);
    return bine_alltoall(comms[r], algo, sbufs[r], rbufs[r], count, dtype, comms[r]->stream);
  });
}

// ---- schedule introspection ------------------------------------------------------

static PlanArgs plan_args(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                          size_t segsize, int in_place) {
  PlanArgs a;
  a.algo = algo;
  a.P = nranks;
  a.rank = rank;
  a.count = count;
  if (rcounts && algo >= BINE_RS_RECURSIVEHALVING && algo <= BINE_RS_BINE_BLOCK_BY_BLOCK_ANY_EVEN)
    a.rcounts.assign(rcounts, rcounts + nranks);
  a.root = root;
  a.esz = esz;
  a.segsize = segsize;
  a.in_place = in_place != 0;
  return a;
}

int64_t bine_plan(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                  size_t segsize, int in_place, bine_prim_t *prims, int64_t cap, uint64_t *tmp_elems) {
  Plan p = make_plan(plan_args(algo, nranks, rank, count, rcounts, root, esz, segsize, in_place));
  if (p.status != BINE_SUCCESS) return -(int64_t)p.status;
  for (int64_t k = 0; k < (int64_t)p.prims.size() && k < cap; k++) prims[k] = p.prims[(size_t)k];
  if (tmp_elems)
    for (int t = 0; t < 3; t++) tmp_elems[t] = p.tmp_elems[t];
  return (int64_t)p.prims.size();
}

int64_t bine_plan_schedule(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                           size_t segsize, int in_place, size_t chunk_bytes, size_t relay_min_bytes, int mode,
                           bine_sched_entry_t *out, int64_t cap, int *c_join, int64_t *final_wait,
                           uint64_t *workspace) {
  if (!esz) return -(int64_t)BINE_ERR_ARG;
  PlanArgs a = plan_args(algo, nranks, rank, count, rcounts, root, esz, segsize, in_place);
  a.flat_ag = (mode & 2) != 0;
  a.flat_rs = (mode & 4) != 0;
  a.flat_ag_chunked = (mode & 8) != 0;
  Plan p;
  Schedule sc;
  build(a, chunk_elems(chunk_bytes, esz), relay_min_bytes, (mode & 1) != 0, p, sc);
  if (p.status != BINE_SUCCESS) return -(int64_t)p.status;
  int64_t n = 0;
  for (size_t i = 0; i < sc.ops.size(); i++)
    for (const Prim &x : sc.ops[i].prims) {
      if (n < cap) out[n] = {(int32_t)i, sc.ops[i].xchg ? 1 : 0, sc.ops[i].wait, x};
      n++;
    }
  if (c_join) *c_join = sc.c_join ? 1 : 0;
  if (final_wait) *final_wait = sc.final_wait;
  if (workspace) {
    for (int t = 0; t < 3; t++) workspace[t] = p.tmp_elems[t];
    workspace[3] = sc.stage_elems;
  }
  return n;
}

// plan_dm_trees' decisions for rank `rank`'s issue schedule, with the
// direct transport's shape rules at `slot` / `merge` and distinct, aligned
// stand-in addresses per buffer (the decisions depend on overlaps within a
// buffer only): host[i] = the exchange whose launch evaluates tree op i (-1:
// not fused), defer[i] = 1 if exchange i's receives are pulled by the next
// exchange.  Returns the number of ops (may exceed cap) or -status.
namespace {
struct PlanOnlyTx final : Transport {
  DirectState d;
  int exchange(const std::vector<XSend> &, const std::vector<XRecv> &, hipStream_t) override {
    return BINE_ERR_UNSUPPORTED;
  }
  bool stream_ordered() const override { return true; }
  bool tree_ok(const std::vector<XSend> &s, const std::vector<XRecv> &r, const TreeSpec &t) const override {
    return d.tree_ok(s, r, t);
  }
  bool defer_ok(const std::vector<XSend> &s, const std::vector<XRecv> &r, const std::vector<XRecv> &dl,
                const TreeSpec &t) const override {
    return d.defer_ok(s, r, dl, t);
  }
};
}  // namespace

int64_t bine_plan_dm_trees(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                           int in_place, size_t chunk_bytes, int mode, size_t slot, int merge, int dtype, int op,
                           int32_t *host, int32_t *defer, int64_t cap) {
  if (!esz || !slot || merge < 0 || merge > 3) return -(int64_t)BINE_ERR_ARG;
  PlanArgs a = plan_args(algo, nranks, rank, count, rcounts, root, esz, 0, in_place);
  a.flat_ag = (mode & 2) != 0;
  a.flat_rs = (mode & 4) != 0;
  a.flat_ag_chunked = (mode & 8) != 0;
  Plan p;
  Schedule sc;
  build(a, chunk_elems(chunk_bytes, esz), 0, (mode & 1) != 0, p, sc);
  if (p.status != BINE_SUCCESS) return -(int64_t)p.status;
  PlanOnlyTx tx;
  tx.d.slot = slot;
  tx.d.merge = merge;
  auto ptr = [&](int buf, uint64_t off) { return (char *)((uintptr_t)(buf + 1) << 40) + off * esz; };
  DmTreePlan pl;
  plan_dm_trees(tx, true, sc, ptr, esz, dtype, op, pl);
  const int64_t n = (int64_t)sc.ops.size();
  for (int64_t i = 0; i < n && i < cap; i++) {
    if (host) host[i] = pl.host[(size_t)i];
    if (defer) defer[i] = pl.defer[(size_t)i];
  }
  return n;
}

int bine_plan_dm_fused(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                       int in_place, size_t chunk_bytes, int mode, size_t slot, int dtype, int op, int small) {
  return (int)bine_plan_dm_fused_msgs(algo, nranks, rank, count, rcounts, root, esz, in_place, chunk_bytes, mode,
                                      slot, dtype, op, small, nullptr, 0, nullptr);
}

int64_t bine_plan_dm_fused_msgs(int algo, int nranks, int rank, size_t count, const int *rcounts, int root,
                                size_t esz, int in_place, size_t chunk_bytes, int mode, size_t slot, int dtype, int op,
                                int small, uint64_t *out, int64_t cap, int64_t *nmsgs) {
  if (!esz || !slot) return -BINE_ERR_ARG;
  PlanArgs a = plan_args(algo, nranks, rank, count, rcounts, root, esz, 0, in_place);
  a.flat_ag = (mode & 2) != 0;
  a.flat_rs = (mode & 4) != 0;
  a.flat_ag_chunked = (mode & 8) != 0;
  Plan p;
  Schedule sc;
  build(a, chunk_elems(chunk_bytes, esz), 0, (mode & 1) != 0, p, sc);
  if (p.status != BINE_SUCCESS) return -p.status;
  if (op < 0 || !dm_fused_supported(dtype, op)) return 0;
  PlanOnlyTx tx;
  tx.d.slot = slot;
  FusedEnv e;
  e.P = nranks;
  e.rank = rank;
  e.d = &tx.d;
  e.own = (uint8_t *)((uintptr_t)15 << 40);  // stand-ins: 4 KiB-aligned, disjoint per buffer
  auto ptr = [&](int buf, uint64_t off) { return (char *)((uintptr_t)(buf + 1) << 40) + off * esz; };
  std::vector<DmFusedArgs> v;
  if (!plan_fused_env(e, sc, ptr, esz, dtype, op, small != 0, v)) v.clear();
  // the launches' messages in the order their sequence numbers are taken
  // (per peer and direction: j order = this order): launch, push, peer, bytes
  int64_t n = 0;
  for (size_t l = 0; l < v.size(); l++)
    for (int i = 0; i < v[l].d0 + v[l].nd; i++, n++)
      if (out && n < cap) {
        uint64_t *o = out + 4 * n;
        o[0] = l;
        o[1] = (uint64_t)v[l].m[i].push;
        o[2] = (uint64_t)v[l].m[i].peer;
        o[3] = v[l].m[i].bytes;
      }
  if (nmsgs) *nmsgs = n;
  return (int64_t)v.size();
}

int64_t bine_plan_stage(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                        size_t segsize, int in_place, size_t chunk_bytes, int mode, int kind, uint64_t *out,
                        int64_t cap) {
  if (!esz || kind < 0 || kind > 2) return -(int64_t)BINE_ERR_ARG;
  PlanArgs a = plan_args(algo, nranks, rank, count, rcounts, root, esz, segsize, in_place);
  a.flat_ag = (mode & 2) != 0;
  a.flat_rs = (mode & 4) != 0;
  a.flat_ag_chunked = (mode & 8) != 0;
  Plan p;
  Schedule sc;
  build(a, chunk_elems(chunk_bytes, esz), 0, (mode & 1) != 0, p, sc);
  if (p.status != BINE_SUCCESS) return -(int64_t)p.status;
  StageRanges g;
  stage_ranges(sc, a.in_place, g);
  int64_t n = 0;
  for (size_t i = 0; i < sc.ops.size(); i++) {
    if (kind == 2) {  // (op, h2d_wait)
      if (n < cap) { out[2 * n] = i; out[2 * n + 1] = (uint64_t)g.h2d_wait[i]; }
      n++;
      continue;
    }
    for (const Ivl &r : kind == 0 ? g.h2d[i] : g.d2h[i]) {  // (op, lo, hi)
      if (n < cap) { out[3 * n] = i; out[3 * n + 1] = r.first; out[3 * n + 2] = r.second; }
      n++;
    }
  }
  return n;
}

int bine_comm_set_trees(bine_comm_t c, int on) {
  if (!c) return BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->trees = on != 0;
  return BINE_SUCCESS;
}

int bine_comm_set_coll_a2a(bine_comm_t c, int on) {
  if (!c) return BINE_ERR_ARG;
  if (!dynamic_cast<RcclTransport *>(c->tx.get())) return BINE_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> g(c->mu);
  c->coll_a2a = on != 0;
  return BINE_SUCCESS;
}

int bine_comm_set_coll_ag(bine_comm_t c, int on) {
  if (!c) return BINE_ERR_ARG;
  auto *r = dynamic_cast<RcclTransport *>(c->tx.get());
  if (!r) return BINE_ERR_UNSUPPORTED;  // loopback: no RCCL collective to use
  std::lock_guard<std::mutex> g(c->mu);
  r->coll_ag = on != 0;
  return BINE_SUCCESS;
}

int bine_comm_set_graphs(bine_comm_t c, int on) {
  if (!c) return BINE_ERR_ARG;
  if (c->hub) return BINE_ERR_UNSUPPORTED;  // loopback exchanges wait on the host: not capturable
  std::lock_guard<std::mutex> g(c->mu);
  if (!on && c->graphs) {
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());  // no cached graph may still run; the caller's streams may be gone
    c->drop_graphs();
  }
  c->graphs = on != 0;
  return BINE_SUCCESS;
}

int64_t bine_comm_fused_calls(bine_comm_t c) {
  if (!c) return -(int64_t)BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return c->fused_calls;
}

int64_t bine_comm_graphs_cached(bine_comm_t c) {
  if (!c) return -(int64_t)BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return (int64_t)c->graph_cache.size();
}

int bine_comm_set_direct(bine_comm_t c, int on) {
  if (!c) return BINE_ERR_ARG;
  auto *r = dynamic_cast<RcclTransport *>(c->tx.get());
  if (!r) return BINE_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  if (on && r->dm) {
    // collective as well once the transport exists: a transport poisoned on
    // any rank (a wait timed out) is rebuilt on every rank -- fresh inboxes,
    // flags and sequence bases.  Every rank's kernels have ended (each waited
    // for its device above, and a timed-out wait ends its launch) before the
    // agreement, so nothing touches the old inboxes when they go.
    int all = 0;
    if (int rc2 = r->agree(!r->dm->poisoned(), &all)) return rc2;
    if (!all) {
      if (trace_on()) fprintf(stderr, "[bine dm r%d] poisoned on some rank: rebuilding\n", c->rank);
      r->dm_on = false;
      c->drop_graphs();  // captured launches carry the old inboxes
      c->tree_cache.clear();
      c->fused_cache.clear();
      r->dm.reset();
    }
  }
  if (on && !r->dm) {  // collective: every rank maps every peer's inbox
    auto d = std::make_unique<DirectState>();
    std::string err;
    int rc = d->init(c->size, c->rank, c->device, err);
    // every step only if every rank got through the previous one (agreed over
    // RCCL), so no rank waits for a peer that has given up
    int all = 0;
    if (trace_on()) fprintf(stderr, "[bine dm r%d] phase 1 rc %d, agreeing\n", c->rank, rc);
    int rc2 = r->agree(rc == BINE_SUCCESS, &all);
    if (!rc2 && all) {
      rc = d->connect_peers(r->key, err);
      rc2 = r->agree(rc == BINE_SUCCESS, &all);
    }
    if (rc2) return rc2;
    if (!all) {
      set_err("direct transport unavailable on some rank: %s", err.empty() ? "(a peer failed)" : err.c_str());
      return BINE_ERR_UNSUPPORTED;
    }
    int same = 1;
    if (int rc3 = r->ranks_on_my_gpu(c->device, &same)) return rc3;
    d->share = same;
    if (r->dm_wgs) d->wgs = r->dm_wgs;
    if (c->dm_tree_wgs) d->tree_wgs = c->dm_tree_wgs;
    r->dm = std::move(d);
  }
  if (on && r->dm->poisoned()) {
    set_err("direct transport: poisoned by an earlier timeout");
    return BINE_ERR_INTERNAL;
  }
  r->dm_on = on != 0;
  return BINE_SUCCESS;
}

int bine_comm_direct_timed_out(bine_comm_t c) {
  if (!c) return -BINE_ERR_ARG;
  auto *r = dynamic_cast<RcclTransport *>(c->tx.get());
  return r && r->dm && r->dm->poisoned() ? 1 : 0;
}

int bine_comm_direct_ping(bine_comm_t c, int peer, int iters, double *us) {
  if (!c || !us || iters < 2 || peer < 0 || peer >= c->size || peer == c->rank) return BINE_ERR_ARG;
  auto *r = dynamic_cast<RcclTransport *>(c->tx.get());
  if (!r || !r->dm_on || !r->dm) return BINE_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  if (int rc = r->health()) return rc;
  // after everything the communicator issued (the probe's flags are its own,
  // but a probe beside a running collective would measure the collective)
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipStreamSynchronize(c->cstream));
  uint64_t ticks = 0;
  if (int rc = r->dm->ping(peer, iters, c->cstream, &ticks)) return rc;
  if (int rc = r->health_drained()) return rc;
  *us = r->dm->clock_khz > 0 ? (double)ticks / (r->dm->clock_khz * 1e3) * 1e6 / (iters - 1) : 0.0;
  return BINE_SUCCESS;
}

int bine_comm_direct_stamps(bine_comm_t c, uint64_t *out, size_t cap, size_t *n, int reset) {
  if (!c || !n || (cap && !out)) return BINE_ERR_ARG;
  auto *r = dynamic_cast<RcclTransport *>(c->tx.get());
  if (!r || !r->dm || !r->dm->stamps) return BINE_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  uint64_t hdr[2];
  HIP_TRY(hipMemcpy(hdr, r->dm->stamps, sizeof hdr, hipMemcpyDeviceToHost));
  *n = (size_t)hdr[0];
  const size_t k = std::min<size_t>({cap, (size_t)hdr[0], (size_t)hdr[1]});
  if (k)
    HIP_TRY(hipMemcpy(out, r->dm->stamps + dm::kStampHdr, k * dm::kStampWords * sizeof(uint64_t),
                      hipMemcpyDeviceToHost));
  if (reset) {
    hdr[0] = 0;
    HIP_TRY(hipMemcpy(r->dm->stamps, hdr, sizeof(uint64_t), hipMemcpyHostToDevice));
  }
  return BINE_SUCCESS;
}

int bine_comm_set_direct_wgs(bine_comm_t c, int wgs) {
  if (!c || wgs < 0 || wgs > 1024) return BINE_ERR_ARG;
  auto *r = dynamic_cast<RcclTransport *>(c->tx.get());
  if (!r) return BINE_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> g(c->mu);
  if (wgs == r->dm_wgs) return BINE_SUCCESS;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // no launch of the old shape may still run
  c->drop_graphs();                 // captured direct launches carry the old grid
  r->dm_wgs = wgs;
  if (r->dm) r->dm->wgs = wgs ? wgs : r->dm->env_wgs;
  return BINE_SUCCESS;
}

int bine_comm_set_direct_tree(bine_comm_t c, int on) {
  if (!c || on < -1 || on > 1024) return BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  const bool v = on < 0 ? dm_tree_env() : on != 0;
  const int w = on > 1 ? on : 0;  // tree workgroups per launch (0: BINE_DIRECT_TREE_WGS / 256)
  if (v == c->dm_tree && w == c->dm_tree_wgs) return BINE_SUCCESS;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  c->drop_graphs();  // captured exchanges carry the other launch structure
  c->dm_tree = v;
  c->dm_tree_wgs = w;
  if (auto *r = dynamic_cast<RcclTransport *>(c->tx.get()))
    if (r->dm) r->dm->tree_wgs = w ? w : r->dm->tree_wgs_env;
  return BINE_SUCCESS;
}

int bine_dropin_defaults(int P, int *flat_rs, int *flat_ag, int *direct) {
  if (P < 1 || !flat_rs || !flat_ag || !direct) return BINE_ERR_ARG;
  auto env = [](const char *k) -> const char * {
    const char *v = getenv(k);
    return v && *v ? v : nullptr;
  };
  const bool literal = env("BINE_LITERAL") && atoi(env("BINE_LITERAL")) != 0;
  *flat_rs = env("BINE_FLAT_RS") ? atoi(env("BINE_FLAT_RS")) != 0 : !literal;
  *flat_ag = env("BINE_FLAT_AG") ? std::max(0, std::min(atoi(env("BINE_FLAT_AG")), 2)) : !literal;
  *direct = P > 1 && (env("BINE_DIRECT") ? atoi(env("BINE_DIRECT")) > 0 : !literal);
  return BINE_SUCCESS;
}

int bine_comm_set_flat_ag(bine_comm_t c, int on) {
  if (!c) return BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (on < 0 || on > 2) return BINE_ERR_ARG;
  c->flat_ag = on;
  return BINE_SUCCESS;
}

int bine_comm_set_profile(bine_comm_t c, int on) {
  if (!c) return BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->profile = on != 0;
  c->prof_n = 0;
  return BINE_SUCCESS;
}

int64_t bine_comm_profile(bine_comm_t c, bine_op_time_t *out, int64_t cap) {
  if (!c) return -(int64_t)BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->prof_n == 0) return 0;
  hipEvent_t first = c->prof[0].a;
  for (size_t i = 0; i < c->prof_n && (int64_t)i < cap; i++) {
    auto &pt = c->prof[i];
    if (hipEventSynchronize(pt.b) != hipSuccess) return -(int64_t)BINE_ERR_HIP;
    float ms = 0.f, st = 0.f;
    if (hipEventElapsedTime(&ms, pt.a, pt.b) != hipSuccess || hipEventElapsedTime(&st, first, pt.a) != hipSuccess)
      return -(int64_t)BINE_ERR_HIP;
    out[i] = {pt.xchg, pt.nprims, pt.bytes, st, ms};
  }
  return (int64_t)c->prof_n;
}

int bine_comm_set_flat_rs(bine_comm_t c, int on) {
  if (!c) return BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->flat_rs = on != 0;
  return BINE_SUCCESS;
}

int bine_comm_set_chunk(bine_comm_t c, size_t bytes) {
  if (!c) return BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->chunk_bytes = bytes;
  return BINE_SUCCESS;
}

int bine_comm_set_relay(bine_comm_t c, size_t min_part_bytes) {
  if (!c) return BINE_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->relay_min_bytes = min_part_bytes;
  return BINE_SUCCESS;
}

int bine_set_reduce_tuning(int unroll, int maxblocks, int nontemporal);

int bine_dm_residency_cap(int cus, int per_cu, int margin, int share) {
  return dm_residency_cap(cus, per_cu, margin, share);
}

int bine_dm_launch_cap(int kind, int dtype, int op, int nl, int share) {
  return dm_launch_cap(kind, dtype, op, nl, share);
}

int bine_dm_fit_residency(int *cw, int n, int *tw, int cap) {
  if ((n > 0 && !cw) || n < 0 || n > kMaxDm) return -1;
  return dm_fit_residency(cw, n, tw, cap);
}

}  // extern "C"
