// direct.cpp -- the direct peer-memory transport of libbine_amd.so
// (bine_comm_set_direct): exchanges move through device memory every rank
// maps from every peer, without RCCL's FIFOs and channels.
//
// Each rank allocates one "inbox" with the VMM API (hipMemCreate, exportable
// as a POSIX file descriptor), hands the descriptor to every peer over a Unix
// socket (SCM_RIGHTS), and maps every peer's inbox (hipMemImportFromShareable
// Handle + hipMemMap + hipMemSetAccess for its own device): on one node the
// peers' memory is reachable over xGMI by plain loads and stores.
//
// Inbox layout (rank y; offsets in bine_internal.h, namespace dm):
//   flags   ready[x][k] latest sequence number x has published into y's slot k
//           ack[x][k]   latest sequence number of y's slot-k sub-message to x
//                       that x has copied out
//           cnt_push[x][k], cnt_pull[x][k]  arrival counters of k_dm_move (local)
//           poison     nonzero once a wait timed out (the transport is then dead)
//           base_send[x], base_recv[x]  sub-messages to / from x so far (local;
//                       the sequence numbers live here, not on the host)
//           launch counter, peer table (x -> x's inbox as mapped here)
//   data    region[x] = kSlots slots of `slot` bytes, written only by rank x
//
// An exchange (sends / receives of one RCCL-style group) is cut into rounds:
// round r carries sub-message r (at most `slot` bytes) of every message.  Each
// round PUSHES every send -- wait until the receiver has acknowledged the
// slot's previous use (sequence s - kSlots), copy into the receiver's slot
// s % kSlots, publish ready = s in the receiver's inbox -- and PULLS every
// receive -- wait for ready >= s, copy the slot into the destination, publish
// ack = s in the sender's inbox.  One k_dm_move launch carries round r-1's
// pulls together with round r's pushes.  Sequence numbers
// are per ordered pair and monotonic, so flags never need resetting.
// Deadlock freedom: at most kSlots messages per peer per exchange (more are
// refused), so a push waits only for pulls of earlier rounds, which every
// rank has issued before it (rounds of one exchange, and exchanges, are
// issued in the same order everywhere -- the RCCL matching rule the planner
// already obeys).  Both ends cut messages identically (sizes match exactly,
// as RCCL requires).  Every wait has a time limit; a timeout poisons the
// transport and every later launch exits immediately (no hang), and the
// collective reports BINE_ERR_INTERNAL from then on.
//
// The received bytes are copied out of the slot (one extra local pass over
// HBM per received byte -- HBM is ~8x the xGMI rate, so it is not the bound);
// sends read the caller's buffer directly.  Launch arguments hold no
// sequence numbers (the kernel derives every slot and flag from the device-side
// bases), so collectives over this transport can be captured into a graph and
// replayed (bine_comm_set_graphs).
#include <hip/hip_runtime.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "bine_internal.h"
#include "direct.h"

namespace bine {

namespace {

// BINE_TRACE=1: one stderr line per setup step
void step(int rank, const char *what) {
  static const bool on = getenv("BINE_TRACE") && atoi(getenv("BINE_TRACE")) != 0;
  if (on) fprintf(stderr, "[bine dm r%d] %s\n", rank, what);
}

using namespace dm;

int send_fd(int sock, int fd, int rank) {
  iovec io{&rank, sizeof rank};
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  cmsghdr *c = CMSG_FIRSTHDR(&m);
  c->cmsg_level = SOL_SOCKET;
  c->cmsg_type = SCM_RIGHTS;
  c->cmsg_len = CMSG_LEN(sizeof(int));
  memcpy(CMSG_DATA(c), &fd, sizeof fd);
  return sendmsg(sock, &m, 0) == (ssize_t)sizeof rank ? 0 : -1;
}

int recv_fd(int sock, int *rank) {
  iovec io{rank, sizeof *rank};
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  if (recvmsg(sock, &m, MSG_WAITALL) != (ssize_t)sizeof *rank) return -1;
  cmsghdr *c = CMSG_FIRSTHDR(&m);
  if (!c || c->cmsg_type != SCM_RIGHTS) return -1;
  int fd;
  memcpy(&fd, CMSG_DATA(c), sizeof fd);
  return fd;
}

// abstract Unix socket name of rank r for this communicator
sockaddr_un addr_of(uint64_t key, int r, socklen_t *len) {
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  char name[96];
  const int n = snprintf(name, sizeof name, "bine-dm-%016llx-%d", (unsigned long long)key, r);
  a.sun_path[0] = '\0';  // abstract namespace: no file, gone with the process
  memcpy(a.sun_path + 1, name, (size_t)n);
  *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
  return a;
}

}  // namespace

DirectState::~DirectState() {
  if (own || !peer.empty()) (void)hipDeviceSynchronize();  // nothing to wait for when nothing was set up
  for (size_t x = 0; x < peer.size(); x++) {
    if ((int)x == rank || !peer[x]) continue;
    (void)hipMemUnmap(peer[x], total);
    (void)hipMemAddressFree(peer[x], total);
    (void)hipMemRelease(peer_h[x]);
  }
  if (own) {
    (void)hipMemUnmap(own, total);
    (void)hipMemAddressFree(own, total);
    (void)hipMemRelease(own_h);
  }
  if (own_fd >= 0) close(own_fd);
  if (hpoison) (void)hipHostFree(hpoison);
  if (stamps) (void)hipFree(stamps);
  if (ping_out) (void)hipFree(ping_out);
}

static int map_handle(hipMemGenericAllocationHandle_t h, size_t size, int device, void **va, std::string &err) {
  void *p = nullptr;
  hipError_t e = hipMemAddressReserve(&p, size, 0, nullptr, 0);
  step(-1, e == hipSuccess ? "reserved" : "reserve failed");
  if (e == hipSuccess) e = hipMemMap(p, size, 0, h, 0);
  step(-1, e == hipSuccess ? "mapped" : "map failed");
  hipMemAccessDesc d{};
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = device;
  d.flags = hipMemAccessFlagsProtReadWrite;
  if (e == hipSuccess) e = hipMemSetAccess(p, size, &d, 1);
  if (e != hipSuccess) {
    err = std::string("map: ") + hipGetErrorString(e);
    return BINE_ERR_HIP;
  }
  *va = p;
  return BINE_SUCCESS;
}

// Phase 1 (local): allocate, zero the flags, export the descriptor.
int DirectState::init(int P_, int rank_, int device_, std::string &err) {
  P = P_;
  rank = rank_;
  device = device_;
  if (P > kMaxPeers) {
    err = "direct transport: more ranks than the inbox layout holds";
    return BINE_ERR_UNSUPPORTED;
  }
  if (const char *e = getenv("BINE_DIRECT_SLOT_BYTES")) slot = (size_t)strtoull(e, nullptr, 10);
  if (const char *e = getenv("BINE_DIRECT_WGS")) wgs = atoi(e);
  if (const char *e = getenv("BINE_DIRECT_PULL_WGS")) pull_wgs = std::max(0, atoi(e));
  if (const char *e = getenv("BINE_DIRECT_AUTOSCALE")) autoscale = atoi(e) != 0;
  if (const char *e = getenv("BINE_DIRECT_MERGE")) merge = std::min(3, std::max(0, atoi(e)));
  if (const char *e = getenv("BINE_DIRECT_TREE_WGS")) tree_wgs = std::max(1, atoi(e));
  if (const char *e = getenv("BINE_DIRECT_MCAST")) mcast = atoi(e) != 0;
  if (const char *e = getenv("BINE_DIRECT_SLICE_FLAGS")) slice_flags = atoi(e) != 0;
  if (const char *e = getenv("BINE_DIRECT_FUSED_WGS")) fused_wgs = std::max(1, atoi(e));
  tree_wgs_env = tree_wgs;
  if (slot < (1 << 20)) slot = 1 << 20;
  if (slot > ((size_t)1 << 30)) slot = (size_t)1 << 30;  // write-through stores address a slot by 32-bit offsets
  slot = slot / 4096 * 4096;
  if (wgs < 1) wgs = 1;
  env_wgs = wgs;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
  double secs = 10.0;
  if (const char *e = getenv("BINE_DIRECT_TIMEOUT_S")) secs = atof(e);
  timeout_ticks = (uint64_t)(secs * khz * 1000.0);
  clock_khz = khz;
  step(rank, "host word");
  if (hipHostMalloc((void **)&hpoison, kHostBytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&hpoison_dev, hpoison, 0) != hipSuccess) {
    err = "direct transport: no mapped host word";
    return BINE_ERR_NO_MEM;
  }
  memset(hpoison, 0, kHostBytes);
  if (const char *e = getenv("BINE_DIRECT_STAMPS")) {
    const uint64_t cap = strtoull(e, nullptr, 10);
    if (cap) {
      const size_t bytes = (dm::kStampHdr + cap * dm::kStampWords) * sizeof(uint64_t);
      const uint64_t hdr[2] = {0, cap};
      if (hipMalloc((void **)&stamps, bytes) != hipSuccess ||
          hipMemcpy(stamps, hdr, sizeof hdr, hipMemcpyHostToDevice) != hipSuccess) {
        err = "direct transport: no stamps buffer";
        return BINE_ERR_NO_MEM;
      }
    }
  }
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  size_t gran = 0;
  if (hipMemGetAllocationGranularity(&gran, &p, hipMemAllocationGranularityRecommended) != hipSuccess || !gran)
    gran = 2 << 20;
  data_off = kFlagsBytes;
  total = data_off + (size_t)P * kSlots * slot;
  total = (total + gran - 1) / gran * gran;
  step(rank, "hipMemCreate");
  hipError_t e = hipMemCreate(&own_h, total, &p, 0);
  if (e != hipSuccess) { err = std::string("hipMemCreate: ") + hipGetErrorString(e); return BINE_ERR_NO_MEM; }
  step(rank, "map own");
  int rc = map_handle(own_h, total, device, &own, err);
  if (rc) return rc;
  step(rank, "zero flags, export");
  e = hipMemset(own, 0, kFlagsBytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemExportToShareableHandle(&own_fd, own_h, hipMemHandleTypePosixFileDescriptor, 0);
  if (e != hipSuccess) { err = std::string("export: ") + hipGetErrorString(e); return BINE_ERR_HIP; }
  peer.assign((size_t)P, nullptr);
  peer_h.assign((size_t)P, hipMemGenericAllocationHandle_t{});
  ping_count.assign((size_t)P, 0);
  peer[(size_t)rank] = own;
  return BINE_SUCCESS;
}

int dm_fit_residency(int *cw, int n, int *tw, int cap) {
  long tot = tw ? *tw : 0;
  for (int i = 0; i < n; i++) tot += cw[i];
  const int parts = n + (tw && *tw > 0 ? 1 : 0);
  if (cap <= 0 || tot <= cap) return 0;
  if (parts > cap) return -1;
  long sum = 0;
  auto cut = [&](int &v) {
    v = (int)std::max<long>(1, (long)v * cap / tot);
    sum += v;
  };
  for (int i = 0; i < n; i++) cut(cw[i]);
  if (tw && *tw > 0) cut(*tw);
  // the floors of the proportional shares sum to <= cap; the minimum of one
  // per part can push it over: take the excess from the largest parts
  while (sum > cap) {
    int *big = tw && *tw > 0 ? tw : &cw[0];
    for (int i = 0; i < n; i++)
      if (cw[i] > *big) big = &cw[i];
    (*big)--;
    sum--;
  }
  return 1;
}


// Phase 2 (after every rank's phase 1 succeeded -- the caller agrees on that
// over RCCL first, so no rank waits here for a peer that gave up): hand our
// descriptor to every peer, take theirs, map their inboxes.  Every blocking
// step has a time limit.
int DirectState::connect_peers(uint64_t key, std::string &err) {
  if (P == 1) return BINE_SUCCESS;  // no exchanges at P = 1
  int rc = BINE_SUCCESS;
  hipError_t e;

  // descriptor exchange: listen, connect to every peer and send ours, accept
  // every peer's (sends are buffered by the kernel: no ordering deadlock)
  int ls = socket(AF_UNIX, SOCK_STREAM, 0);
  socklen_t len;
  sockaddr_un me = addr_of(key, rank, &len);
  if (ls < 0 || bind(ls, (sockaddr *)&me, len) || listen(ls, P)) {
    err = "direct transport: cannot listen on its Unix socket";
    if (ls >= 0) close(ls);
    return BINE_ERR_INTERNAL;
  }
  const auto t0 = std::chrono::steady_clock::now();
  auto expired = [&] { return std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60); };
  std::vector<int> conns;
  for (int x = 0; x < P && !rc; x++) {
    if (x == rank) continue;
    sockaddr_un pa = addr_of(key, x, &len);
    int s = -1;
    while (true) {
      s = socket(AF_UNIX, SOCK_STREAM, 0);
      if (s >= 0 && connect(s, (sockaddr *)&pa, len) == 0) break;
      if (s >= 0) close(s);
      s = -1;
      if (expired()) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    if (s < 0 || send_fd(s, own_fd, rank)) {
      err = "direct transport: descriptor exchange with a peer failed";
      rc = BINE_ERR_INTERNAL;
    }
    if (s >= 0) conns.push_back(s);
  }
  step(rank, "descriptors sent");
  std::vector<int> fds((size_t)P, -1);
  for (int k = 0; k < P - 1 && !rc; k++) {
    pollfd pf{ls, POLLIN, 0};
    int s = -1;
    while (s < 0 && !expired()) {
      if (poll(&pf, 1, 100) > 0) s = accept(ls, nullptr, nullptr);
    }
    int from = -1;
    const int fd = s >= 0 ? recv_fd(s, &from) : -1;
    if (s >= 0) close(s);
    if (fd < 0 || from < 0 || from >= P || from == rank || fds[(size_t)from] >= 0) {
      err = "direct transport: bad descriptor from a peer";
      rc = BINE_ERR_INTERNAL;
    } else {
      fds[(size_t)from] = fd;
    }
  }
  close(ls);
  for (int s : conns) close(s);
  step(rank, "descriptors received; importing");
  for (int x = 0; x < P && !rc; x++) {
    if (x == rank) continue;
    {
      char b[96];
      snprintf(b, sizeof b, "import from %d (fd %d, %zu B)", x, fds[(size_t)x], total);
      step(rank, b);
    }
    // HIP runtimes disagree on what osHandle is for a POSIX descriptor: the
    // 7.0 runtime torch bundles reads it as a POINTER to the descriptor (the
    // value form segfaults inside it), the 7.2 runtime takes the descriptor
    // VALUE (the pointer form returns hipErrorInvalidValue, harmlessly) --
    // measured, profiles/r2_direct_transport.txt.  So: pointer first, value
    // on failure.
    int fdv = fds[(size_t)x];
    e = hipMemImportFromShareableHandle(&peer_h[(size_t)x], (void *)&fdv, hipMemHandleTypePosixFileDescriptor);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      e = hipMemImportFromShareableHandle(&peer_h[(size_t)x], (void *)(intptr_t)fdv,
                                          hipMemHandleTypePosixFileDescriptor);
    }
    step(rank, e == hipSuccess ? "imported; mapping" : "import failed");
    if (e != hipSuccess) {
      err = std::string("import: ") + hipGetErrorString(e);
      rc = BINE_ERR_HIP;
      break;
    }
    rc = map_handle(peer_h[(size_t)x], total, device, &peer[(size_t)x], err);
  }
  for (int fd : fds)
    if (fd >= 0) close(fd);
  if (rc) return rc;
  // the peer table the kernel reads: x -> x's inbox as mapped in this process
  std::vector<uint64_t> tab((size_t)P);
  for (int x = 0; x < P; x++) tab[(size_t)x] = (uint64_t)(uintptr_t)peer[(size_t)x];
  e = hipMemcpy((char *)own + kPeerTabOff, tab.data(), tab.size() * sizeof(uint64_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    err = std::string("peer table: ") + hipGetErrorString(e);
    return BINE_ERR_HIP;
  }
  return BINE_SUCCESS;
}

// One ready and one ack flag per (pair, slot), and one arrival counter per
// (peer, slot, direction): every flag has one writer at a time and its values
// only grow (a slot's next use waits for the ack of its previous one).  A flag
// per pair would not do: two messages of one launch to the same peer publish
// in either order, and a plain store of the smaller sequence number after the
// larger would move the flag backwards.
static uint64_t rd64(const void *p) {
  uint64_t v = 0;
  (void)hipMemcpy(&v, p, 8, hipMemcpyDeviceToHost);
  return v;
}

void DirectState::dump() const { fprintf(stderr, "[bine dm r%d] %s\n", rank, describe(true).c_str()); }

std::string DirectState::describe(bool flags) const {
  static const char *const kinds[] = {"?", "k_dm_move push", "k_dm_move pull", "k_dm_move push group",
                                      "k_dm_move_tree leaf", "k_dm_fused push", "k_dm_fused pull", "k_dm_ping"};
  std::string s;
  char b[320];
  const volatile uint64_t *h = (const volatile uint64_t *)hpoison;
  if (!h || !(h[0] & 0xffffffffu)) return "no wait timed out";
  const uint64_t kp = h[kRecFirst];
  const uint32_t kind = (uint32_t)(kp >> 8), phase = (uint32_t)(kp & 255);
  if (kind == 0 || kind > kWaitPing) {
    s = "a wait timed out (no record: poisoned by a launch without one)";
  } else {
    const bool push = kind == kWaitMovePush || kind == kWaitGroupPush || kind == kWaitFusedPush;
    const uint64_t peer_ = h[kRecFirst + 2], slot_ = h[kRecFirst + 3], want = h[kRecFirst + 4],
                   seen = h[kRecFirst + 5], ser = h[kRecFirst + 6], wg = h[kRecFirst + 7], ticks = h[kRecFirst + 8];
    char ph[32] = "";
    if (kind >= kWaitFusedPush) {
      if (phase == 0) snprintf(ph, sizeof ph, " (phase A)");
      else if (phase == 15) snprintf(ph, sizeof ph, " (phase D)");
      else snprintf(ph, sizeof ph, " (phase B%u)", phase - 1);
    }
    snprintf(b, sizeof b,
             "rank %d: %s%s, workgroup %llu thread %llu of launch %llu, waited %.3g s for peer %llu's %s of "
             "slot %llu to reach %llu; last seen %llu",
             rank, kinds[kind], ph, (unsigned long long)(wg >> 16), (unsigned long long)(wg & 0xffff),
             (unsigned long long)ser, clock_khz > 0 ? (double)ticks / (clock_khz * 1e3) : 0.0,
             (unsigned long long)peer_, push ? "acknowledgement" : kind == kWaitPing ? "ping answer" : "ready mark", (unsigned long long)slot_,
             (unsigned long long)want, (unsigned long long)seen);
    s = b;
  }
  if (!flags || !own) return s;
  // per peer x, read here and -- through the mapping every rank holds of
  // every peer's inbox -- in x's own inbox: the ready marks x set in our
  // slots 0..3, the sub-messages we have taken from x (our base) against the
  // ones x has sent us (x's base), the acknowledgements x set for our slots,
  // our sends against x's receives, and whether x itself timed out.  Bases
  // advance at a launch's end, so between calls both ends of a pair agree; a
  // disagreement is an accounting fault, a lagging peer a peer that never
  // ran its part.
  auto u = [](uint64_t v) { return (unsigned long long)v; };
  const uint32_t lc = (uint32_t)rd64((char *)own + kLaunchCntOff);
  snprintf(b, sizeof b, "; launch counter %u; per peer x (ready x->us slots 0-3, bases us-recv/x-send, "
                        "ack x->us slots 0-3, bases us-send/x-recv, x poisoned):", lc);
  s += b;
  for (int x = 0; x < P; x++) {
    if (x == rank) continue;
    uint64_t rd[kSlots], ak[kSlots];
    for (int k = 0; k < kSlots; k++) {
      rd[k] = rd64((char *)own + kReadyOff + ((size_t)x * kSlots + k) * kFlagStride);
      ak[k] = rd64((char *)own + kAckOff + ((size_t)x * kSlots + k) * kFlagStride);
    }
    const char *px = x < (int)peer.size() ? (const char *)peer[(size_t)x] : nullptr;
    const uint64_t xs = px ? rd64(px + kBaseSendOff + 8 * (size_t)rank) : ~0ull,
                   xr = px ? rd64(px + kBaseRecvOff + 8 * (size_t)rank) : ~0ull,
                   xp = px ? rd64(px + kPoisonOff) & 0xffffffffu : ~0ull;
    snprintf(b, sizeof b, " %d: r[%llu %llu %llu %llu] %llu/%llu a[%llu %llu %llu %llu] %llu/%llu p%llu;", x,
             u(rd[0]), u(rd[1]), u(rd[2]), u(rd[3]), u(rd64((char *)own + kBaseRecvOff + 8 * (size_t)x)), u(xs),
             u(ak[0]), u(ak[1]), u(ak[2]), u(ak[3]), u(rd64((char *)own + kBaseSendOff + 8 * (size_t)x)), u(xr),
             u(xp));
    s += b;
  }
  return s;
}

int DirectState::ping(int x, int iters, hipStream_t st, uint64_t *ticks) {
  if (x < 0 || x >= P || x == rank || iters < 2) return BINE_ERR_ARG;
  if (!ping_out && hipMalloc((void **)&ping_out, sizeof(uint64_t)) != hipSuccess) return BINE_ERR_NO_MEM;
  DmPingArgs a;
  a.own = (uint8_t *)own;
  a.poison_host = hpoison_dev;
  a.timeout_ticks = timeout_ticks;
  a.base = ping_count[(size_t)x];
  a.out = ping_out;
  a.rank = rank;
  a.peer = x;
  a.iters = iters;
  a.initiator = rank < x;
  a.serial = serial++;
  ping_count[(size_t)x] += (uint64_t)iters;
  if (int rc = launch_dm_ping(a, st)) return rc;
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipMemcpy(ticks, ping_out, sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
    return BINE_ERR_HIP;
  return BINE_SUCCESS;
}

bool DirectState::tree_ok(const std::vector<XSend> &s, const std::vector<XRecv> &r, const TreeSpec &t) const {
  if (!dm_tree_supported(t.dtype, t.op, t.nl) || t.pos < 0 || t.pos >= t.nl || (int)r.size() != t.nl - 1 ||
      (int)t.leaf_of_recv.size() != (int)r.size() || !t.leaf_bytes || t.leaf_bytes % 16 || slot % 16 ||
      ((uintptr_t)t.own_leaf & 15) || ((uintptr_t)t.out & 15) || s.size() + r.size() > (size_t)kMaxDm)
    return false;
  unsigned seen = 1u << t.pos;
  for (size_t i = 0; i < r.size(); i++) {
    const int j = t.leaf_of_recv[i];
    if (j < 0 || j >= t.nl || (seen >> j & 1) || r[i].bytes != t.leaf_bytes) return false;
    seen |= 1u << j;
  }
  return true;
}

bool DirectState::defer_ok(const std::vector<XSend> &s, const std::vector<XRecv> &r,
                           const std::vector<XRecv> &dl, const TreeSpec &t) const {
  if (!tree_ok({}, dl, t) || t.leaf_bytes > slot) return false;
  // the first launch holds the deferred leaves, every send's and (one round,
  // or merge 2) every receive's first sub-message
  size_t maxb = 0;
  for (const auto &x : s) maxb = std::max(maxb, x.bytes);
  for (const auto &x : r) maxb = std::max(maxb, x.bytes);
  const bool pulls_first = merge == 2 || (merge == 3 && maxb <= slot);
  return dl.size() + s.size() + (pulls_first ? r.size() : 0) <= (size_t)kMaxDm;
}

int DirectState::exchange(const std::vector<XSend> &s, const std::vector<XRecv> &r, hipStream_t st,
                          const TreeSpec *tree, const std::vector<XRecv> *dleaves, const TreeSpec *dtree) {
  if (tree && !tree_ok(s, r, *tree)) return BINE_ERR_UNSUPPORTED;
  if (dleaves && (tree || !dtree || !defer_ok(s, r, *dleaves, *dtree))) return BINE_ERR_UNSUPPORTED;
  // more messages to (or from) one peer in one exchange than slots per pair
  // would make a push wait for a pull of the same exchange: refuse
  std::vector<int> ns((size_t)P, 0), nr((size_t)P, 0);
  for (const auto &x : s)
    if (x.peer < 0 || x.peer >= P || ++ns[(size_t)x.peer] > kSlots) return BINE_ERR_UNSUPPORTED;
  for (const auto &x : r)
    if (x.peer < 0 || x.peer >= P || ++nr[(size_t)x.peer] > kSlots) return BINE_ERR_UNSUPPORTED;
  size_t maxb = 0;
  for (const auto &x : s) maxb = std::max(maxb, x.bytes);
  for (const auto &x : r) maxb = std::max(maxb, x.bytes);
  const size_t rounds = (maxb + slot - 1) / slot;
  DmArgs a;
  a.wgs = wgs;
  a.rank = rank;
  a.share = share;
  a.slot = slot;
  a.own = (uint8_t *)own;
  a.poison_host = hpoison_dev;
  a.timeout_ticks = timeout_ticks;
  a.stamps = stamps;
  // j = index of a message among this launch's messages of its kind to / from
  // its peer (the kernel adds it to the device-side base)
  std::vector<int> js((size_t)P, 0), jr((size_t)P, 0);
  // a launch holding leaf pulls (all of one round: tree_ok) evaluates that
  // round's tree in place of copying them
  int tree_round = -1;
  const TreeSpec *ltree = tree;  // the tree of the launch being built
  // the messages that get workgroups of their own: standalone copies and the
  // leaders of push groups (members ride with their leader, leaves with the tree)
  auto index_copies = [&](bool plain) {
    a.ncopy = 0;
    a.ncw = 0;
    for (int i = 0; i < a.nmsg; i++) {
      const DmMsg &m = a.m[i];
      if (m.leaf >= 0 || (m.grp >= 0 && m.grp != i)) continue;
      int members = 1;
      if (m.grp == i)
        for (int q = i + 1; q < a.nmsg; q++) members += a.m[q].grp == i;
      a.cidx[a.ncopy] = i;
      a.cwgs[a.ncopy] = (m.push || !pull_wgs ? a.wgs : pull_wgs) * members;
      a.ncw += a.cwgs[a.ncopy++];
    }
    // a plain k_dm_move launch of few messages (one push and one pull of a
    // Bine step, a rooted collective's single message) would leave most of
    // the GPU idle at `wgs` workgroups each: every copy takes the same whole
    // multiple of its workgroups that the resident capacity allows, keeping
    // at least 64 KiB per workgroup.  The protocol does not care how many
    // workgroups a copy has (each launch counts its own arrivals).  Bounded
    // (ADVICE r5): launches of at most two copies (the measured gains: one
    // push and one pull, a rooted collective's single message), and to half
    // the resident capacity, so a direct launch of this rank in flight on
    // another stream (a tree, a fused call) keeps room beside it.
    if (plain && autoscale && a.ncw > 0 && a.ncopy <= 2) {
      const int cap = dm_launch_cap(0, 0, 0, 0, share) / 2;
      const int k = cap > 0 ? cap / a.ncw : 1;
      if (k > 1) {
        a.ncw = 0;
        for (int c = 0; c < a.ncopy; c++) {
          const uint64_t by = a.m[a.cidx[c]].bytes >> 16;
          const int lim = (int)std::min<uint64_t>((uint64_t)a.cwgs[c] * (uint64_t)k,
                                                  std::max<uint64_t>((uint64_t)a.cwgs[c], by));
          a.cwgs[c] = lim;
          a.ncw += a.cwgs[c];
        }
      }
    }
  };
  auto flush = [&]() -> int {
    int rc;
    a.serial = serial++;
    if (tree_round >= 0) {
      DmTree t;
      t.nl = ltree->nl;
      t.pos = ltree->pos;
      t.swap = ltree->swap;
      t.twgs = tree_wgs;
      const size_t off = (size_t)tree_round * slot, len = std::min(slot, ltree->leaf_bytes - off);
      t.own_leaf = ltree->own_leaf + off;
      t.out = ltree->out + off;
      t.nvec = len / 16;
      for (int j = 0; j < kMaxLeaves; j++) t.leaf_msg[j] = -1;
      for (int i = 0; i < a.nmsg; i++)
        if (a.m[i].leaf >= 0) t.leaf_msg[a.m[i].leaf] = i;
      index_copies(false);
      rc = launch_dm_move_tree(a, t, ltree->dtype, ltree->op, st);
      tree_round = -1;
      ltree = tree;
    } else {
      index_copies(true);
      rc = launch_dm_move(a, st);
    }
    a.nmsg = 0;
    std::fill(js.begin(), js.end(), 0);
    std::fill(jr.begin(), jr.end(), 0);
    return rc;
  };
  // round k's pushes: into the receiver's slot, after its ack of the slot's
  // previous use
  auto pushes = [&](size_t k) -> int {
    for (const auto &x : s) {
      if (x.bytes <= k * slot) continue;
      const size_t off = k * slot, len = std::min(slot, x.bytes - off);
      DmMsg &m = a.m[a.nmsg++];
      m.src = (const uint8_t *)x.ptr + off;
      m.dst = nullptr;
      m.bytes = len;
      m.push = 1;
      m.peer = x.peer;
      m.j = js[(size_t)x.peer]++;
      m.leaf = -1;
      // the same bytes already pushed to another peer in this launch: one
      // group, the source read once (BINE_DIRECT_MCAST=1; default: every push alone)
      m.grp = -1;
      if (mcast) {
        const int me = a.nmsg - 1;
        for (int q = 0; q < me && m.grp < 0; q++)
          if (a.m[q].push && a.m[q].src == m.src && a.m[q].bytes == m.bytes) m.grp = a.m[q].grp;
        if (m.grp < 0) m.grp = me;
      }
      if (a.nmsg == kMaxDm)
        if (int rc = flush()) return rc;
    }
    return BINE_SUCCESS;
  };
  // round k's pulls: out of our own slot once the sender marked it ready
  auto pulls = [&](size_t k) -> int {
    for (size_t i = 0; i < r.size(); i++) {
      const auto &x = r[i];
      if (x.bytes <= k * slot) continue;
      const size_t off = k * slot, len = std::min(slot, x.bytes - off);
      DmMsg &m = a.m[a.nmsg++];
      m.src = nullptr;
      m.dst = (uint8_t *)x.ptr + off;
      m.bytes = len;
      m.push = 0;
      m.peer = x.peer;
      m.j = jr[(size_t)x.peer]++;
      m.grp = -1;
      m.leaf = tree ? tree->leaf_of_recv[i] : -1;
      if (tree) tree_round = (int)k;
      if (a.nmsg == kMaxDm)
        if (int rc = flush()) return rc;
    }
    return BINE_SUCCESS;
  };
  // the deferred leaves (one sub-message each, defer_ok): pulled first --
  // their sender pushed them before anything of this exchange -- and
  // evaluated by the first launch's tree workgroups
  if (dleaves) {
    for (size_t i = 0; i < dleaves->size(); i++) {
      const auto &x = (*dleaves)[i];
      DmMsg &m = a.m[a.nmsg++];
      m.src = nullptr;
      m.dst = (uint8_t *)x.ptr;
      m.bytes = x.bytes;
      m.push = 0;
      m.peer = x.peer;
      m.j = jr[(size_t)x.peer]++;
      m.grp = -1;
      m.leaf = dtree->leaf_of_recv[i];
    }
    tree_round = 0;
    ltree = dtree;
  }
  // merge = 2: launch k carries round k's pushes and then round k's pulls --
  // one launch per round, a pull's workgroups waiting for the peer's push of
  // the same round.  The pushes come first in workgroup order, so they
  // are dispatched before any pull can occupy the chip waiting, and a push
  // waits only for pulls of rounds <= k-1 (issued in earlier launches
  // everywhere): no cycle.  merge = 1: launch k carries round k-1's pulls and
  // round k's pushes.  merge = 0: separate push and pull launches per round.
  // merge = 3 (default): 2 for a one-round exchange (one launch: the latency
  // case, and a pull overlaps the pushes still in flight), 1 for several
  // rounds (the links stay busy while the previous round is copied out)
  if (merge == 2 || (merge == 3 && rounds == 1)) {
    for (size_t k = 0; k < rounds; k++) {
      if (int rc = pushes(k)) return rc;
      if (int rc = pulls(k)) return rc;
      if (int rc = flush()) return rc;
    }
    // a self-hosted tree (no messages of its own, rounds = 0): the launch
    // that pulls the deferred leaves and evaluates the tree
    if (rounds == 0 && a.nmsg) return flush();
    return BINE_SUCCESS;
  }
  for (size_t k = 0; k <= rounds; k++) {
    if (k > 0)
      if (int rc = pulls(k - 1)) return rc;
    if (!merge)
      if (int rc = flush()) return rc;
    if (k < rounds)
      if (int rc = pushes(k)) return rc;
    if (int rc = flush()) return rc;
  }
  return BINE_SUCCESS;
}

}  // namespace bine
