// mpi_shim.cpp -- libbine.so: the reference's include/libbine.h ABI on top of
// libbine_amd.so (see include/libbine_amd.h for the contract).
//
// Compiled against the same mpi.h as pico_core (MPICH: MPI_Datatype / MPI_Op /
// MPI_Comm are int handles).  The shim owns no algorithm: it maps MPI handles to
// bine_* enums, finds (or creates) the RCCL-backed bine communicator of the
// MPI communicator, stages host buffers through the device, and turns status
// codes into MPI error classes.
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <mutex>
#include <set>
#include <utility>
#include <vector>

#include "bine_amd.h"
#include "libbine_amd.h"

extern "C" {
size_t bine_allreduce_segsize = 0;  // libbine.h:28, written by pico_core (pico_core_utils.c:317)
}

namespace {

struct Entry {
  bine_comm_t comm = nullptr;
  int rank = 0, size = 1;
  // staging for host buffers
  void *dev[2] = {nullptr, nullptr};
  size_t dev_bytes[2] = {0, 0};
  // host->device and device->host copy streams (PCIe is full duplex: the two
  // directions overlap) and the events that hand chunks between them and the
  // collective's stream
  hipStream_t h2d = nullptr, d2h = nullptr;
  std::vector<hipEvent_t> ev;
  size_t ev_next = 0;
  // page-locked bounce buffers for small host buffers (bounce_bytes())
  void *bounce[2] = {nullptr, nullptr};
  size_t bounce_cap[2] = {0, 0};
  // every collective of this communicator runs as kernels end to end (P = 1,
  // or the direct transport): small host buffers may be read and written by
  // those kernels in place (zero_copy_bytes())
  bool kernels_only = false;
};

// Small host buffers MAY go through two page-locked bounce buffers the
// communicator owns: the caller's bytes memcpy'd into
// them (and the result out of them) on the CPU, so the call registers
// nothing.  Measured through the unchanged pico_core (C1, 1 MiB fp32,
// profiles/r6_e2e_c1.txt): 115 us per call at P = 1 against 66 us with the
// per-call hipHostRegister / hipHostUnregister, 488 vs 419 us at P = 4 on one
// GPU -- the two 1 MiB CPU copies cost more than the registration they save
// (as HIP's own pageable staging does: 115 us).  So it is off by default;
// BINE_HOST_BOUNCE_BYTES=<bytes> turns it on for buffers up to that size
// (a host whose memcpy is faster than its page-locking).
size_t bounce_bytes() {
  static const size_t v = getenv("BINE_HOST_BOUNCE_BYTES") ? (size_t)strtoull(getenv("BINE_HOST_BOUNCE_BYTES"),
                                                                              nullptr, 10)
                                                           : 0;
  return v;
}

// bounce buffer `slot` of at least `bytes` (grown on demand, kept); nullptr
// when it cannot be allocated (the call then registers, as a large one)
void *bounce_buf(Entry *e, int slot, size_t bytes) {
  if (e->bounce_cap[slot] < bytes) {
    if (e->bounce[slot]) (void)hipHostFree(e->bounce[slot]);
    e->bounce[slot] = nullptr;
    e->bounce_cap[slot] = 0;
    if (hipHostMalloc(&e->bounce[slot], bytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    e->bounce_cap[slot] = bytes;
  }
  return e->bounce[slot];
}

// Small host buffers in place (zero copy): on a communicator whose
// collectives are kernels end to end (Entry::kernels_only), a call whose
// host buffers are at most this many bytes (BINE_HOST_ZERO_COPY_BYTES,
// default 16 MiB; 0 = off) page-locks them for the call, mapped into the GPU's
// address space, and hands their device addresses to the collective: its
// kernels read the input and write the result over PCIe themselves -- no
// staging copies, no device workspace round trip (C1: one k_dm_fused launch
// instead of copy in, launch, copy out).  Measured through pico_core on one
// GPU (profiles/r6_zero_copy_threshold.txt): faster than staging at 1, 4 and
// 16 MiB per rank for P = 1, 2, 4 (by 10-28 %); from 32 MiB the staging is
// pipelined (into the collective at P > 1) instead.
size_t zero_copy_bytes() {
  static const size_t v = getenv("BINE_HOST_ZERO_COPY_BYTES")
                              ? (size_t)strtoull(getenv("BINE_HOST_ZERO_COPY_BYTES"), nullptr, 10)
                              : (size_t)16 << 20;
  return v;
}

// Host buffers page-locked for ONE call.  A permanent
// registration cache is unsafe in a general MPI library: a buffer freed and
// allocated again at the same address keeps the old registration, whose pages
// the kernel driver invalidated at munmap -- the next copy through it faulted
// the GPU (profiles/r4_host_pin_probe.txt).  So the call's host buffers are
// registered at its start and unregistered before it returns, once every
// stream that copies them has drained (bounded, below).  Measured cost of the
// per-call registration against round 3's permanent one: 10.085 vs 10.066 ms
// for a 256 MiB host round trip (profiles/r4_host_stage_probe.txt).  Memory
// the caller page-locked itself is used as it is.  BINE_HOST_REGISTER=0 keeps
// the buffers pageable (HIP's own staging copies).
bool register_on() {
  static const bool on = !getenv("BINE_HOST_REGISTER") || atoi(getenv("BINE_HOST_REGISTER")) != 0;
  return on;
}

// Host waits of the shim are bounded: a stream that does
// not drain within BINE_SYNC_TIMEOUT_S (default 120 s) makes the call return
// MPI_ERR_OTHER naming the stream, instead of hanging the caller.
double sync_timeout_s() {
  static const double v = getenv("BINE_SYNC_TIMEOUT_S") ? atof(getenv("BINE_SYNC_TIMEOUT_S")) : 120.0;
  return v;
}

int drain(hipStream_t s, const char *what, int rank) {
  const double t0 = MPI_Wtime();
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return MPI_SUCCESS;
    if (q != hipErrorNotReady) {
      fprintf(stderr, "libbine(amd) rank %d: %s stream: %s\n", rank, what, hipGetErrorString(q));
      return MPI_ERR_OTHER;
    }
    const double el = MPI_Wtime() - t0;
    if (el > sync_timeout_s()) {
      fprintf(stderr, "libbine(amd) rank %d: the %s stream did not drain within %.0f s (BINE_SYNC_TIMEOUT_S); "
                      "returning MPI_ERR_OTHER\n", rank, what, sync_timeout_s());
      return MPI_ERR_OTHER;
    }
    if (el > 2e-3) usleep(50);  // spin first: short calls
  }
}

struct CallPins {
  std::vector<std::pair<uintptr_t, uintptr_t>> want, regs;  // [lo, hi), page-rounded
  bool drained = true;  // false: a copy may still read / write the pages (never unregister then)
  unsigned flags = hipHostRegisterDefault;  // hipHostRegisterMapped: kernels address the pages (zero copy)
  void add(const void *p, size_t n) {
    if (!register_on() || !p || p == MPI_IN_PLACE || !n) return;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost) return;  // caller's own
    (void)hipGetLastError();
    const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
    want.emplace_back((uintptr_t)p & ~(pg - 1), ((uintptr_t)p + n + pg - 1) & ~(pg - 1));
  }
  // register the union of the wanted ranges (two buffers may share a page)
  void commit() {
    std::sort(want.begin(), want.end());
    for (size_t i = 0; i < want.size();) {
      uintptr_t lo = want[i].first, hi = want[i].second;
      for (i++; i < want.size() && want[i].first <= hi; i++) hi = std::max(hi, want[i].second);
      if (hipHostRegister((void *)lo, hi - lo, flags) == hipSuccess) regs.emplace_back(lo, hi);
      else (void)hipGetLastError();  // stays pageable: HIP stages those copies itself
    }
  }
  ~CallPins() {
    if (!drained) {
      if (!regs.empty()) fprintf(stderr, "libbine(amd): a stream did not drain; %zu host registrations kept\n",
                                 regs.size());
      return;
    }
    for (const auto &r : regs) (void)hipHostUnregister((void *)r.first);
    (void)hipGetLastError();
  }
  // whether every wanted range got registered (a failed one stays pageable)
  bool covered() const {
    for (const auto &w : want) {
      bool in = false;
      for (const auto &r : regs) in = in || (r.first <= w.first && w.second <= r.second);
      if (!in) return false;
    }
    return true;
  }
};

// the device address of host memory the GPU can address (registered mapped,
// or the caller's own page-locked memory); nullptr if it cannot
void *host_dev_ptr(const void *p) {
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void *>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}

int g_keyval = MPI_KEYVAL_INVALID;
int g_self_keyval = MPI_KEYVAL_INVALID;
std::set<Entry *> g_entries;  // live entries; an attribute may outlive its entry

void release(Entry *e) {
  if (!e) return;
  if (e->comm) {
    bine_comm_synchronize(e->comm);
    bine_comm_destroy(e->comm);
  }
  for (int i = 0; i < 2; i++) {
    if (e->dev[i]) (void)hipFree(e->dev[i]);
    if (e->bounce[i]) (void)hipHostFree(e->bounce[i]);
  }
  if (e->h2d) (void)hipStreamDestroy(e->h2d);
  if (e->d2h) (void)hipStreamDestroy(e->d2h);
  for (auto x : e->ev) (void)hipEventDestroy(x);
  delete e;
}

int comm_delete(MPI_Comm, int, void *val, void *) {
  Entry *e = (Entry *)val;
  if (g_entries.erase(e)) release(e);  // already released if MPI_COMM_SELF went first
  return MPI_SUCCESS;
}

// MPI_Finalize deletes MPI_COMM_SELF's attributes first: release everything
int self_delete(MPI_Comm, int, void *, void *) {
  for (auto *e : g_entries) release(e);
  g_entries.clear();
  return MPI_SUCCESS;
}

int to_mpi(int st) {
  switch (st) {
    case BINE_SUCCESS: return MPI_SUCCESS;
    case BINE_ERR_ARG: return MPI_ERR_ARG;
    case BINE_ERR_SIZE: return MPI_ERR_SIZE;
    case BINE_ERR_NO_MEM: return MPI_ERR_NO_MEM;
    case BINE_ERR_UNSUPPORTED: return MPI_ERR_UNSUPPORTED_OPERATION;
    case BINE_ERR_ROOT: return MPI_ERR_ROOT;
    case BINE_ERR_COUNT: return MPI_ERR_COUNT;
    default:
      fprintf(stderr, "libbine(amd): %s: %s\n", bine_status_string(st), bine_last_error());
      return MPI_ERR_OTHER;
  }
}

int map_dtype(MPI_Datatype d) {
  if (d == MPI_FLOAT) return BINE_FLOAT;
  if (d == MPI_DOUBLE) return BINE_DOUBLE;
  if (d == MPI_INT8_T || d == MPI_SIGNED_CHAR || d == MPI_CHAR) return BINE_INT8;
  if (d == MPI_UINT8_T || d == MPI_UNSIGNED_CHAR || d == MPI_BYTE) return BINE_UINT8;
  if (d == MPI_INT16_T || d == MPI_SHORT) return BINE_INT16;
  if (d == MPI_UINT16_T || d == MPI_UNSIGNED_SHORT) return BINE_UINT16;
  if (d == MPI_INT32_T || d == MPI_INT) return BINE_INT32;
  if (d == MPI_UINT32_T || d == MPI_UNSIGNED) return BINE_UINT32;
  if (d == MPI_INT64_T || d == MPI_LONG || d == MPI_LONG_LONG || d == MPI_AINT || d == MPI_OFFSET || d == MPI_COUNT)
    return BINE_INT64;
  if (d == MPI_C_BOOL) return BINE_UINT8;  // logical ops only (map_op)
  if (d == MPI_UINT64_T || d == MPI_UNSIGNED_LONG || d == MPI_UNSIGNED_LONG_LONG) return BINE_UINT64;
  if (d == MPI_FLOAT_INT) return BINE_FLOAT_INT;
  if (d == MPI_DOUBLE_INT) return BINE_DOUBLE_INT;
  if (d == MPI_LONG_INT) return BINE_LONG_INT;
  if (d == MPI_2INT) return BINE_2INT;
  if (d == MPI_SHORT_INT) return BINE_SHORT_INT;
  if (d == MPI_C_FLOAT_COMPLEX || d == MPI_C_COMPLEX) return BINE_C_FLOAT_COMPLEX;
  if (d == MPI_C_DOUBLE_COMPLEX) return BINE_C_DOUBLE_COMPLEX;
  return -1;
}

// The predefined MPI_Ops MPICH's MPI_Reduce_local applies, and the (op, type)
// pairs it accepts (MPICH 3.3.2, probed with its own MPI_Reduce_local):
// MPI_BYTE only under the bitwise ops, floating types under every op but the
// bitwise ones, the (value, index) pair types under MAXLOC / MINLOC only.
// -1 = MPI_ERR_OP (the reference's MPI_Reduce_local would fail).
int map_op(MPI_Op o, MPI_Datatype d) {
  int r = -1;
  if (o == MPI_SUM) r = BINE_SUM;
  else if (o == MPI_PROD) r = BINE_PROD;
  else if (o == MPI_MAX) r = BINE_MAX;
  else if (o == MPI_MIN) r = BINE_MIN;
  else if (o == MPI_LAND) r = BINE_LAND;
  else if (o == MPI_BAND) r = BINE_BAND;
  else if (o == MPI_LOR) r = BINE_LOR;
  else if (o == MPI_BOR) r = BINE_BOR;
  else if (o == MPI_LXOR) r = BINE_LXOR;
  else if (o == MPI_BXOR) r = BINE_BXOR;
  else if (o == MPI_MAXLOC) r = BINE_MAXLOC;
  else if (o == MPI_MINLOC) r = BINE_MINLOC;
  if (r < 0) return -1;
  const bool bits = r == BINE_BAND || r == BINE_BOR || r == BINE_BXOR;
  if (d == MPI_BYTE) return bits ? r : -1;
  if (d == MPI_C_BOOL) return r == BINE_LAND || r == BINE_LOR || r == BINE_LXOR ? r : -1;
  const int dt = map_dtype(d);
  return dt < 0 || bine_op_valid(dt, r) ? r : -1;  // unknown types are reported as MPI_ERR_TYPE
}

int get_entry(MPI_Comm comm, Entry **out) {
  if (g_keyval == MPI_KEYVAL_INVALID) {
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, comm_delete, &g_keyval, nullptr);
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, self_delete, &g_self_keyval, nullptr);
    MPI_Comm_set_attr(MPI_COMM_SELF, g_self_keyval, nullptr);
  }
  void *val = nullptr;
  int flag = 0;
  MPI_Comm_get_attr(comm, g_keyval, &val, &flag);
  if (flag && val && g_entries.count((Entry *)val)) { *out = (Entry *)val; return MPI_SUCCESS; }
  auto *e = new Entry;
  MPI_Comm_rank(comm, &e->rank);
  MPI_Comm_size(comm, &e->size);
  MPI_Comm local;
  int lrank = 0;
  MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, e->rank, MPI_INFO_NULL, &local);
  MPI_Comm_rank(local, &lrank);
  MPI_Comm_free(&local);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    fprintf(stderr, "libbine(amd): no HIP device visible\n");
    delete e;
    return MPI_ERR_OTHER;
  }
  const char *forced = getenv("BINE_DEVICE");
  const int device = forced ? atoi(forced) : lrank % ndev;
  unsigned char id[BINE_UNIQUE_ID_BYTES] = {0};
  int st = BINE_SUCCESS;
  if (e->rank == 0) st = bine_get_unique_id(id);
  MPI_Bcast(&st, 1, MPI_INT, 0, comm);
  if (st != BINE_SUCCESS) { delete e; return to_mpi(st); }
  MPI_Bcast(id, BINE_UNIQUE_ID_BYTES, MPI_BYTE, 0, comm);
  st = bine_comm_init_rccl(&e->comm, e->size, e->rank, id, device);
  if (st != BINE_SUCCESS) { delete e; return to_mpi(st); }
  // The drop-in's forms (bine_dropin_defaults): the
  // fastest bit-identical ones unless the environment says otherwise -- the
  // flat phases, and exchanges over the direct peer-memory transport instead
  // of RCCL P2P (bine_comm_set_direct; collective, and every rank of a
  // pico_core run sees the same environment).  Setup is agreed over RCCL, so
  // a failure is the same on every rank: then the communicator keeps RCCL.
  int frs = 0, fag = 0, dm = 0;
  if ((st = bine_dropin_defaults(e->size, &frs, &fag, &dm)) == BINE_SUCCESS &&
      (st = bine_comm_set_flat_rs(e->comm, frs)) == BINE_SUCCESS)
    st = bine_comm_set_flat_ag(e->comm, fag);
  if (st != BINE_SUCCESS) {
    bine_comm_destroy(e->comm);
    delete e;
    return to_mpi(st);
  }
  e->kernels_only = e->size == 1;
  if (dm) {
    const int dst = bine_comm_set_direct(e->comm, 1);
    if (dst != BINE_SUCCESS && e->rank == 0)
      fprintf(stderr, "libbine(amd): the direct transport is unavailable (%d: %s); using RCCL P2P\n", dst,
              bine_last_error());
    e->kernels_only = e->kernels_only || dst == BINE_SUCCESS;
  }
  MPI_Comm_set_attr(comm, g_keyval, e);
  g_entries.insert(e);
  *out = e;
  return MPI_SUCCESS;
}

bool on_device(const void *p) {
  if (!p || p == MPI_IN_PLACE) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

int stage(Entry *e, int slot, size_t bytes, void **dev) {
  bytes = std::max<size_t>(bytes, 256);  // a zero-byte buffer still gets an address
  if (e->dev_bytes[slot] < bytes) {
    if (e->dev[slot]) (void)hipFree(e->dev[slot]);
    e->dev[slot] = nullptr;
    e->dev_bytes[slot] = 0;
    if (hipMalloc(&e->dev[slot], bytes) != hipSuccess) return MPI_ERR_NO_MEM;
    e->dev_bytes[slot] = bytes;
  }
  *dev = e->dev[slot];
  return MPI_SUCCESS;
}

int copy_streams(Entry *e) {
  if (e->h2d) return MPI_SUCCESS;
  if (hipStreamCreateWithFlags(&e->h2d, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&e->d2h, hipStreamNonBlocking) != hipSuccess)
    return MPI_ERR_OTHER;
  e->ev.resize(64);
  for (auto &x : e->ev)
    if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) return MPI_ERR_OTHER;
  return MPI_SUCCESS;
}

// `dst` stream waits for everything enqueued so far on `src`
int follow(Entry *e, hipStream_t dst, hipStream_t src) {
  hipEvent_t x = e->ev[e->ev_next];
  e->ev_next = (e->ev_next + 1) % e->ev.size();
  if (hipEventRecord(x, src) != hipSuccess || hipStreamWaitEvent(dst, x, 0) != hipSuccess) return MPI_ERR_OTHER;
  return MPI_SUCCESS;
}

// staging chunk of the pipelined path (BINE_STAGE_CHUNK_BYTES, default 16 MiB)
size_t stage_chunk_bytes() {
  static const size_t v = [] {
    const char *x = getenv("BINE_STAGE_CHUNK_BYTES");
    const size_t b = x ? (size_t)strtoull(x, nullptr, 10) : (size_t)16 << 20;
    return std::max<size_t>(b, 1 << 20) & ~(size_t)255;
  }();
  return v;
}

// the end of a call: every stream that touched the caller's buffers (or the
// communicator's) drained within the bound, then the communicator's own
int finish(Entry *e, CallPins &pins, std::initializer_list<std::pair<hipStream_t, const char *>> streams) {
  for (const auto &x : streams)
    if (int rc = drain(x.first, x.second, e->rank)) {
      pins.drained = false;
      return rc;
    }
  const hipStream_t cs = (hipStream_t)bine_comm_stream(e->comm);
  if (int rc = drain(cs, "communicator", e->rank)) {
    pins.drained = false;
    return rc;
  }
  return to_mpi(bine_comm_synchronize(e->comm));
}

// Run `body(dev_sbuf, dev_rbuf, first_elem, elems, stream)` with host buffers
// staged through the device.  Host->device copies run on the h2d stream,
// device->host copies on the d2h stream, the collective on the communicator's
// stream, chained by events.  `esz` > 0 declares the collective separable by
// element (element i of the result depends only on element i of the inputs --
// P = 1, where every algorithm is the copy, see do_allreduce): then the buffer
// is cut into chunks and chunk k's host->device copy, collective and
// device->host copy are pipelined, so the two PCIe directions and the device
// work overlap.  Otherwise one collective over the whole buffer, between the
// two staged copies.  Every rank calls `body` the same number of times with
// the same counts whatever its buffers are (device buffers: the same chunks,
// uncopied), so ranks with host and with device buffers meet in one
// schedule.
template <typename F>
int with_buffers(Entry *e, const void *sbuf, size_t sbytes, void *rbuf, size_t rbytes, bool read_rbuf, size_t esz,
                 size_t count, F body) {
  hipStream_t st = (hipStream_t)bine_comm_stream(e->comm);
  (void)hipSetDevice(bine_comm_device(e->comm));
  const bool in_place = sbuf == MPI_IN_PLACE;
  const void *ds = sbuf;
  void *dr = rbuf;
  bool stage_s = !in_place && sbuf && sbytes && !on_device(sbuf);
  bool stage_r = rbuf && rbytes && !on_device(rbuf);
  int rc;
  if ((rc = copy_streams(e))) return rc;
  const size_t ch = esz ? stage_chunk_bytes() / esz * esz : 0;
  const size_t total = count * esz;
  const bool piped = ch && total >= 2 * ch && (stage_s || stage_r) && (!stage_s || sbytes == total) &&
                     (!stage_r || rbytes == total);
  // small host buffers: through the communicator's page-locked bounce buffers
  // (nothing registered); the caller's input is copied in on the CPU now
  void *bs = nullptr, *br = nullptr;
  const bool fill_r = stage_r && (in_place || read_rbuf);  // (every earlier call has drained all three streams)
  if (!piped && (stage_s || stage_r) && std::max(stage_s ? sbytes : 0, stage_r ? rbytes : 0) <= bounce_bytes()) {
    bs = stage_s ? bounce_buf(e, 0, sbytes) : nullptr;
    br = stage_r ? bounce_buf(e, 1, rbytes) : nullptr;
    if ((stage_s && !bs) || (stage_r && !br)) bs = br = nullptr;  // no bounce memory: register as a large call
  }
  const bool bounced = bs || br;
  // zero copy: the collective's kernels address the host buffers themselves
  if (!piped && !bounced && e->kernels_only && register_on() && (stage_s || stage_r) &&
      std::max(stage_s ? sbytes : 0, stage_r ? rbytes : 0) <= zero_copy_bytes()) {
    CallPins zp;
    zp.flags = hipHostRegisterMapped;
    if (stage_s) zp.add(sbuf, sbytes);
    if (stage_r) zp.add(rbuf, rbytes);
    zp.commit();
    const void *zs = stage_s ? host_dev_ptr(sbuf) : ds;
    void *zr = stage_r ? host_dev_ptr(rbuf) : dr;
    if (zp.covered() && zs && zr) {
      const int bst = body(in_place ? BINE_IN_PLACE : zs, zr, (size_t)0, count, (void *)st);
      const int rz = finish(e, zp, {{st, "collective"}});
      return bst ? to_mpi(bst) : rz;
    }
    // not addressable: staged as any other call (zp unregisters on return)
  }
  CallPins pins;
  if (stage_s) {
    void *d;
    if ((rc = stage(e, 0, sbytes, &d))) return rc;
    ds = d;
    if (bounced) memcpy(bs, sbuf, sbytes);
    else pins.add(sbuf, sbytes);
  }
  if (stage_r) {
    void *d;
    if ((rc = stage(e, 1, rbytes, &d))) return rc;
    dr = d;
    if (bounced) {
      if (fill_r) memcpy(br, rbuf, rbytes);
    } else {
      pins.add(rbuf, rbytes);
    }
  }
  pins.commit();
  const void *hs = bounced && stage_s ? bs : sbuf;  // the host side of the copies
  void *hr = bounced && stage_r ? br : rbuf;
  auto issue = [&]() -> int {
    if (piped) {
      for (size_t off = 0; off < total; off += ch) {
        const size_t len = std::min(ch, total - off);
        if (stage_s && hipMemcpyAsync((char *)ds + off, (const char *)sbuf + off, len, hipMemcpyHostToDevice,
                                      e->h2d) != hipSuccess)
          return MPI_ERR_OTHER;
        if (fill_r && hipMemcpyAsync((char *)dr + off, (char *)rbuf + off, len, hipMemcpyHostToDevice, e->h2d) !=
                          hipSuccess)
          return MPI_ERR_OTHER;
        if (int r2 = follow(e, st, e->h2d)) return r2;
        const void *cs = in_place ? BINE_IN_PLACE : (const void *)((const char *)ds + off);
        if (int bst = body(cs, (char *)dr + off, off / esz, len / esz, (void *)st)) return to_mpi(bst);
        if (stage_r) {
          if (int r2 = follow(e, e->d2h, st)) return r2;
          if (hipMemcpyAsync((char *)rbuf + off, (char *)dr + off, len, hipMemcpyDeviceToHost, e->d2h) != hipSuccess)
            return MPI_ERR_OTHER;
        }
      }
      return MPI_SUCCESS;
    }
    // unpipelined: copy in, collective, copy out depend on each other in
    // turn, so they share the collective's stream -- no cross-stream event
    // hops (a small call's latency is mostly such hops: C1 end to end)
    if (stage_s && hipMemcpyAsync((void *)ds, hs, sbytes, hipMemcpyHostToDevice, st) != hipSuccess)
      return MPI_ERR_OTHER;
    if (fill_r && hipMemcpyAsync(dr, hr, rbytes, hipMemcpyHostToDevice, st) != hipSuccess)
      return MPI_ERR_OTHER;
    if (int bst = body(in_place ? BINE_IN_PLACE : ds, dr, (size_t)0, count, (void *)st)) return to_mpi(bst);
    if (stage_r && hipMemcpyAsync(hr, dr, rbytes, hipMemcpyDeviceToHost, st) != hipSuccess) return MPI_ERR_OTHER;
    return MPI_SUCCESS;
  };
  rc = issue();
  // drain whatever was issued (also after an error: the registrations must
  // outlive every copy that uses them)
  const int rc2 = finish(e, pins, {{e->h2d, "host-to-device"}, {e->d2h, "device-to-host"}, {st, "collective"}});
  // a bounced result reaches the caller's buffer only from a call that
  // completed (an error leaves rbuf as it was)
  if (!rc && !rc2 && bounced && stage_r) memcpy(rbuf, br, rbytes);
  return rc ? rc : rc2;
}

// The staging pipelined into the collective itself (bine_*_staged): for
// collectives whose result bits follow the whole count's block ownership, so
// they cannot be cut into independent calls.  The core copies each input piece
// in just before the first operation that touches it and each output piece
// back right after its last writer, with the flat forms on (bit-identical) so
// the output completes chunk by chunk.  Chosen from (P, bytes) only -- the
// same on every rank -- and run whatever the buffers are: a device buffer is
// passed as is (NULL host pointer, nothing copied), so every rank issues the
// same schedule.  BINE_STAGE_PIPELINE=0 keeps the serial H2D -> collective ->
// D2H.
bool staged_pipeline_on() {
  static const bool v = !getenv("BINE_STAGE_PIPELINE") || atoi(getenv("BINE_STAGE_PIPELINE")) != 0;
  return v;
}

bool use_staged(const Entry *e, size_t bytes) {
  return e->size > 1 && staged_pipeline_on() && bytes >= 2 * stage_chunk_bytes();
}

template <typename G>
int with_staged(Entry *e, const void *sbuf, size_t sbytes, void *rbuf, size_t rbytes, G body) {
  hipStream_t st = (hipStream_t)bine_comm_stream(e->comm);
  (void)hipSetDevice(bine_comm_device(e->comm));
  const bool in_place = sbuf == MPI_IN_PLACE;
  int rc;
  if ((rc = copy_streams(e))) return rc;
  const bool host_s = !in_place && sbuf && !on_device(sbuf), host_r = rbuf && !on_device(rbuf);
  void *ds = in_place ? nullptr : (void *)sbuf, *dr = rbuf;
  CallPins pins;
  if (host_s) {
    if ((rc = stage(e, 0, sbytes, &ds))) return rc;
    pins.add(sbuf, sbytes);
  }
  if (host_r) {
    if ((rc = stage(e, 1, rbytes, &dr))) return rc;
    pins.add(rbuf, rbytes);
  } else if (!dr) {
    // a rank that receives nothing may pass no rbuf (reduce_scatter with
    // rcounts[rank] == 0): it still issues the schedule its peers issue, so it
    // gets a device placeholder instead of refusing the call on its own
    if ((rc = stage(e, 1, 0, &dr))) return rc;
  }
  pins.commit();
  const void *hs = in_place ? BINE_IN_PLACE : host_s ? sbuf : nullptr;
  const int bst = body(hs, host_r ? rbuf : nullptr, ds, dr, (void *)e->h2d, (void *)e->d2h, (void *)st);
  const int rc2 = finish(e, pins, {{e->h2d, "host-to-device"}, {e->d2h, "device-to-host"}, {st, "collective"}});
  return bst != BINE_SUCCESS ? to_mpi(bst) : rc2;
}

int do_allreduce(int algo, const void *sbuf, void *rbuf, size_t count, MPI_Datatype dtype, MPI_Op op,
                 MPI_Comm comm) {
  const int dt = map_dtype(dtype), o = map_op(op, dtype);
  if (dt < 0) return MPI_ERR_TYPE;
  if (o < 0) return MPI_ERR_OP;
  if (count == 0) return MPI_SUCCESS;
  Entry *e;
  int rc = get_entry(comm, &e);
  if (rc) return rc;
  const size_t esz = bine_dtype_size(dt);
  const size_t bytes = count * esz;
  const size_t seg = bine_allreduce_segsize;
  // Every choice below depends on (P, count, type) only -- never on where a
  // rank's buffers live -- so all ranks issue the same collectives (ADVICE
  // r3).  P = 1: every algorithm is the copy sbuf -> rbuf
  // (libbine_allreduce.c:849-852), separable by element, so the staged path
  // pipelines it as independent chunks.  P > 1: the result bits follow the
  // whole count's block ownership (floating point) -- one collective, with the
  // staging pipelined into it when the buffer is large enough.
  if (use_staged(e, bytes))
    return with_staged(e, sbuf, bytes, rbuf, bytes,
                       [&](const void *hs, void *hr, void *ds, void *dr, void *h2d, void *d2h, void *st) {
                         return bine_allreduce_staged(e->comm, algo, hs, hr, ds, dr, count, dt, o,
                                                      algo == BINE_AR_BINE_BDW_REMAP_SEGMENTED ? seg : 0,
                                                      stage_chunk_bytes(), h2d, d2h, st);
                       });
  return with_buffers(e, sbuf, bytes, rbuf, bytes, false, e->size == 1 ? esz : 0, count,
                      [&](const void *s, void *r, size_t, size_t n, void *st) {
                        return bine_allreduce(e->comm, algo, s, r, n, dt, o,
                                              algo == BINE_AR_BINE_BDW_REMAP_SEGMENTED ? seg : 0, st);
                      });
}

int do_reduce_scatter(int algo, const void *sbuf, void *rbuf, const int rcounts[], MPI_Datatype dtype, MPI_Op op,
                      MPI_Comm comm) {
  const int dt = map_dtype(dtype), o = map_op(op, dtype);
  if (dt < 0) return MPI_ERR_TYPE;
  if (o < 0) return MPI_ERR_OP;
  Entry *e;
  int rc = get_entry(comm, &e);
  if (rc) return rc;
  size_t total = 0;
  for (int i = 0; i < e->size; i++) total += (size_t)rcounts[i];
  const size_t esz = bine_dtype_size(dt);
  const bool in_place = sbuf == MPI_IN_PLACE;
  // MPI_IN_PLACE: the input is the whole rbuf
  const size_t rbytes = (in_place ? total : (size_t)rcounts[e->rank]) * esz;
  if (use_staged(e, total * esz))  // (P, counts, type): the same on every rank
    return with_staged(e, sbuf, total * esz, rbuf, rbytes,
                       [&](const void *hs, void *hr, void *ds, void *dr, void *h2d, void *d2h, void *st) {
                         return bine_reduce_scatter_staged(e->comm, algo, hs, hr, ds, dr, rcounts, dt, o,
                                                           stage_chunk_bytes(), h2d, d2h, st);
                       });
  return with_buffers(e, sbuf, total * esz, rbuf, rbytes, false, 0, total,
                      [&](const void *s, void *r, size_t, size_t, void *st) {
                        return bine_reduce_scatter(e->comm, algo, s, r, rcounts, dt, o, st);
                      });
}

int do_reduce(int algo, const void *sbuf, void *rbuf, size_t count, MPI_Datatype dtype, MPI_Op op, int root,
              MPI_Comm comm) {
  const int dt = map_dtype(dtype), o = map_op(op, dtype);
  if (dt < 0) return MPI_ERR_TYPE;
  if (o < 0) return MPI_ERR_OP;
  if (count == 0) return MPI_SUCCESS;
  Entry *e;
  int rc = get_entry(comm, &e);
  if (rc) return rc;
  const size_t bytes = count * bine_dtype_size(dt);
  void *r = e->rank == root ? rbuf : nullptr;
  return with_buffers(e, sbuf, bytes, r, r ? bytes : 0, false, 0, count,
                      [&](const void *s, void *rr, size_t, size_t, void *st) {
                        return bine_reduce(e->comm, algo, s, rr, count, dt, o, root, st);
                      });
}

// allgather family: pure data movement, so it runs on bytes whatever the type
// bytes one element of `dt` spans in memory (its extent: MPI_DOUBLE_INT's
// padding included, where MPI_Type_size counts 12 of its 16 bytes); 0 for a
// type with a gap in front or holes a byte copy would not preserve
size_t span(MPI_Datatype dt) {
  MPI_Aint lb = 0, ext = 0;
  int sz = 0;
  if (MPI_Type_get_extent(dt, &lb, &ext) != MPI_SUCCESS || MPI_Type_size(dt, &sz) != MPI_SUCCESS) return 0;
  if (lb != 0 || ext <= 0 || sz <= 0) return 0;
  // predefined types only (derived types: MPI_ERR_TYPE, as map_dtype); the
  // pair types' padding is the only gap allowed
  if ((size_t)sz != (size_t)ext && map_dtype(dt) < 0) return 0;
  return (size_t)ext;
}

int do_allgather(int algo, const void *sbuf, size_t scount, MPI_Datatype sdtype, void *rbuf, size_t rcount,
                 MPI_Datatype rdtype, MPI_Comm comm) {
  const size_t rsz = span(rdtype);
  if (!rsz) return MPI_ERR_TYPE;
  const size_t bytes = rcount * rsz;
  if (sbuf != MPI_IN_PLACE) {
    const size_t ssz = span(sdtype);
    if (!ssz) return MPI_ERR_TYPE;
    if (scount * ssz != bytes) return MPI_ERR_ARG;  // unequal block sizes: not supported
  }
  if (bytes == 0) return MPI_SUCCESS;
  Entry *e;
  int rc = get_entry(comm, &e);
  if (rc) return rc;
  return with_buffers(e, sbuf, bytes, rbuf, bytes * (size_t)e->size, false, 0, bytes,
                      [&](const void *s, void *r, size_t, size_t, void *st) {
                        return bine_allgather(e->comm, algo, s, r, bytes, BINE_UINT8, st);
                      });
}

// bcast family: pure data movement on `buf` in place (read on the root,
// written elsewhere), run on bytes whatever the type
int do_bcast(int algo, void *buf, size_t count, MPI_Datatype dtype, int root, MPI_Comm comm) {
  const size_t sz = span(dtype);
  if (!sz) return MPI_ERR_TYPE;
  const size_t bytes = count * sz;
  // count == 0 still goes through the planner: the reference returns
  // MPI_ERR_SIZE / MPI_ERR_ROOT before looking at the count
  // (libbine_bcast.c:198-210)
  Entry *e;
  int rc = get_entry(comm, &e);
  if (rc) return rc;
  // the bandwidth bcasts split the buffer into blocks of ELEMENTS (and refuse
  // count < P, MPI_ERR_COUNT): they run on the type itself when the library
  // has it with this extent, else on bytes with the element count checked
  // here -- the blocks then fall elsewhere, the delivered bytes are the same
  size_t n = bytes;
  int dt = BINE_UINT8;
  if (algo == BINE_BC_SCATTER_ALLGATHER || algo == BINE_BC_BINE_BDW_STATIC || algo == BINE_BC_BINE_BDW_REMAP) {
    const int t = map_dtype(dtype);
    if (t >= 0 && bine_dtype_size(t) == sz) {
      n = count;
      dt = t;
    } else if (e->size > 1 && count < (size_t)e->size && algo != BINE_BC_BINE_BDW_REMAP) {
      return MPI_ERR_COUNT;
    }
  }
  return with_buffers(e, MPI_IN_PLACE, 0, buf, bytes, true, 0, bytes,
                      [&](const void *, void *r, size_t, size_t, void *st) {
                        return bine_bcast(e->comm, algo, r, n, dt, root, st);
                      });
}

// alltoall_bine / gather_bine / scatter_bine: whole blocks of scount elements
// (the reference asserts sendcount == recvcount and one type,
// libbine_gather.c:17, libbine_scatter.c:17-18, libbine_alltoall.c:17-18:
// unequal block sizes are MPI_ERR_ARG here), run on bytes.  gather: rbuf on
// the root only (pico_core passes NULL elsewhere, pico_core_gather_utils.c);
// scatter: sbuf on the root only.
int do_blocks(int algo, const void *sbuf, size_t scount, MPI_Datatype sdtype, void *rbuf, size_t rcount,
              MPI_Datatype rdtype, int root, MPI_Comm comm) {
  Entry *e;
  int rc = get_entry(comm, &e);
  if (rc) return rc;
  const bool has_s = algo != BINE_SC_BINE || e->rank == root;
  const bool has_r = algo != BINE_GA_BINE || e->rank == root;
  const size_t rsz = span(rdtype), ssz = has_s && sbuf != MPI_IN_PLACE ? span(sdtype) : rsz;
  if (!rsz || !ssz) return MPI_ERR_TYPE;
  const size_t bytes = rcount * rsz;
  if (has_s && sbuf != MPI_IN_PLACE && scount * ssz != bytes) return MPI_ERR_ARG;
  if (bytes == 0) return MPI_SUCCESS;
  const size_t P = (size_t)e->size;
  const size_t sbytes = has_s ? (algo == BINE_GA_BINE ? bytes : P * bytes) : 0;
  const size_t rbytes = has_r ? (algo == BINE_SC_BINE ? bytes : P * bytes) : 0;
  return with_buffers(e, has_s ? sbuf : nullptr, sbytes, has_r ? rbuf : nullptr, rbytes, false, 0, bytes,
                      [&](const void *s, void *r, size_t, size_t, void *st) {
                        if (algo == BINE_GA_BINE) return bine_gather(e->comm, algo, s, r, bytes, BINE_UINT8, root, st);
                        if (algo == BINE_SC_BINE) return bine_scatter(e->comm, algo, s, r, bytes, BINE_UINT8, root, st);
                        return bine_alltoall(e->comm, algo, s, r, bytes, BINE_UINT8, st);
                      });
}

}  // namespace

extern "C" {

#define AR(fn, id) \
  int fn(BINE_ALLREDUCE_ARGS) { return do_allreduce(id, sbuf, rbuf, count, dtype, op, comm); }
AR(allreduce_recursivedoubling, BINE_AR_RECURSIVEDOUBLING)
AR(allreduce_ring, BINE_AR_RING)
AR(allreduce_rabenseifner, BINE_AR_RABENSEIFNER)
AR(allreduce_bine_lat, BINE_AR_BINE_LAT)
AR(allreduce_bine_bdw_static, BINE_AR_BINE_BDW_STATIC)
AR(allreduce_bine_bdw_remap, BINE_AR_BINE_BDW_REMAP)
AR(allreduce_bine_bdw_remap_segmented, BINE_AR_BINE_BDW_REMAP_SEGMENTED)
AR(allreduce_bine_block_by_block_any_even, BINE_AR_BINE_BLOCK_BY_BLOCK_ANY_EVEN)
#undef AR

#define RS(fn, id) \
  int fn(BINE_REDUCE_SCATTER_ARGS) { return do_reduce_scatter(id, sbuf, rbuf, rcounts, dtype, op, comm); }
RS(reduce_scatter_recursivehalving, BINE_RS_RECURSIVEHALVING)
RS(reduce_scatter_recursive_distance_doubling, BINE_RS_RECURSIVE_DISTANCE_DOUBLING)
RS(reduce_scatter_ring, BINE_RS_RING)
RS(reduce_scatter_butterfly, BINE_RS_BUTTERFLY)
RS(reduce_scatter_bine_static, BINE_RS_BINE_STATIC)
RS(reduce_scatter_bine_send_remap, BINE_RS_BINE_SEND_REMAP)
RS(reduce_scatter_bine_permute_remap, BINE_RS_BINE_PERMUTE_REMAP)
RS(reduce_scatter_bine_block_by_block, BINE_RS_BINE_BLOCK_BY_BLOCK)
RS(reduce_scatter_bine_block_by_block_any_even, BINE_RS_BINE_BLOCK_BY_BLOCK_ANY_EVEN)
#undef RS

int reduce_bine_lat(BINE_REDUCE_ARGS) { return do_reduce(BINE_RD_BINE_LAT, sbuf, rbuf, count, dtype, op, root, comm); }
int reduce_bine_bdw(BINE_REDUCE_ARGS) { return do_reduce(BINE_RD_BINE_BDW, sbuf, rbuf, count, dtype, op, root, comm); }

#define AG(fn, id) \
  int fn(BINE_ALLGATHER_ARGS) { return do_allgather(id, sbuf, scount, sdtype, rbuf, rcount, rdtype, comm); }
AG(allgather_k_bruck, BINE_AG_K_BRUCK)
AG(allgather_recursivedoubling, BINE_AG_RECURSIVEDOUBLING)
AG(allgather_ring, BINE_AG_RING)
AG(allgather_sparbit, BINE_AG_SPARBIT)
AG(allgather_bine_block_by_block, BINE_AG_BINE_BLOCK_BY_BLOCK)
AG(allgather_bine_block_by_block_any_even, BINE_AG_BINE_BLOCK_BY_BLOCK_ANY_EVEN)
AG(allgather_bine_permute_static, BINE_AG_BINE_PERMUTE_STATIC)
AG(allgather_bine_send_static, BINE_AG_BINE_SEND_STATIC)
AG(allgather_bine_permute_remap, BINE_AG_BINE_PERMUTE_REMAP)
AG(allgather_bine_send_remap, BINE_AG_BINE_SEND_REMAP)
AG(allgather_bine_2_blocks, BINE_AG_BINE_2_BLOCKS)
AG(allgather_bine_2_blocks_dtype, BINE_AG_BINE_2_BLOCKS_DTYPE)
#undef AG

int alltoall_bine(BINE_ALLGATHER_ARGS) {
  return do_blocks(BINE_A2A_BINE, sbuf, scount, sdtype, rbuf, rcount, rdtype, 0, comm);
}
#define BC(fn, id) \
  int fn(BINE_BCAST_ARGS) { return do_bcast(id, buf, count, dtype, root, comm); }
BC(bcast_bine_lat, BINE_BC_BINE_LAT)
BC(bcast_bine_lat_reversed, BINE_BC_BINE_LAT_REVERSED)
BC(bcast_bine_lat_new, BINE_BC_BINE_LAT_NEW)
BC(bcast_bine_lat_i_new, BINE_BC_BINE_LAT_I_NEW)
BC(bcast_scatter_allgather, BINE_BC_SCATTER_ALLGATHER)
BC(bcast_bine_bdw_static, BINE_BC_BINE_BDW_STATIC)
BC(bcast_bine_bdw_remap, BINE_BC_BINE_BDW_REMAP)
#undef BC
int gather_bine(BINE_GATHER_ARGS) {
  return do_blocks(BINE_GA_BINE, sbuf, scount, sdtype, rbuf, rcount, rdtype, root, comm);
}
int scatter_bine(BINE_GATHER_ARGS) {
  return do_blocks(BINE_SC_BINE, sbuf, scount, sdtype, rbuf, rcount, rdtype, root, comm);
}

}  // extern "C"
