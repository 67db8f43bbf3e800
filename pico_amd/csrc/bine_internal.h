// bine_internal.h -- shared declarations of libbine_amd.so (not installed).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "bine_amd.h"

namespace bine {

// ---- schedule (schedule.cpp) ------------------------------------------------

// One primitive of a per-rank plan (same layout as bine_prim_t).
using Prim = bine_prim_t;

struct Plan {
  std::vector<Prim> prims;
  uint64_t tmp_elems[3] = {0, 0, 0};  // workspace per TMP buffer, elements
  int status = BINE_SUCCESS;          // non-success: the reference's error return
};

struct PlanArgs {
  int algo = -1;
  int P = 1, rank = 0;
  size_t count = 0;                 // allreduce / reduce
  std::vector<int> rcounts;         // reduce_scatter
  int root = 0;                     // reduce
  size_t esz = 4;
  size_t segsize = 0;               // bytes; segmented variant's segment
  bool in_place = false;
  // allreduce (remap / static / rabenseifner, power-of-two P): replace the
  // mirrored allgather by one exchange in which every rank sends its reduced
  // block to every other rank (one hop on every link of a fully connected
  // node); reduce_bine_bdw: the gather tree becomes one step into the root.
  // Pure data movement: result bits unchanged.
  bool flat_ag = false;
  // allreduce remap / static / segmented (power-of-two P), reduce_scatter
  // bine_{permute,send}_remap / bine_static, reduce_bine_bdw, 2 <= P <= 16:
  // replace the log2(P) reduce-scatter steps by one all-peers exchange in which
  // every rank sends each block straight to the rank that computes it, which
  // then evaluates the reference's reduction tree for that block over the P
  // contributions in one REDUCE_TREE (same operands, same association, same
  // operand order: result bits unchanged).  flat_chunk = pipelining chunk in
  // elements (0: one chunk): chunk k's transfer overlaps chunk k-1's tree.
  bool flat_rs = false;
  size_t flat_chunk = 0;
  // with flat_rs and flat_ag (allreduce): the allgather exchange cut with the
  // reduce-scatter's chunks, chunk k's results sent right after chunk k+1's
  // reduce-scatter exchange, so the outputs complete chunk by chunk (the staged
  // host-buffer pipeline copies each chunk back as soon as it is final).  Pure
  // data movement: result bits unchanged.
  bool flat_ag_chunked = false;
};

Plan make_plan(const PlanArgs &a);

// multi-tree mode (trees.cpp): P-1 relabelled instances on P-1 slices; status
// BINE_ERR_UNSUPPORTED when not applicable (only allreduce, P = 4 or 8)
int tree_count(int P);
const int *tree_relabel(int P, int k);  // virtual -> physical rank of instance k
Plan make_tree_plan(const PlanArgs &a);

// schedule math (libbine_utils.h restated for the planner)
int pi(int rank, int step, int P);
uint32_t remap_rank(uint32_t P, uint32_t rank);
uint32_t get_nu(uint32_t rank, uint32_t size);
int log2_ceil(int v);
bool is_pow2(int v);
void static_perm(int P, std::vector<int> &perm);

// ---- issue schedule (schedule.cpp) -------------------------------------------
// A plan turned into device work for two streams: exchange groups go to the
// comm stream, local primitives to the compute stream.  PIPELINE exchanges are
// cut into `chunk` element pieces, each feeding the matching piece of the
// following reduction.  `wait` = index of the op of the OTHER stream this op
// must wait for (the newest one touching overlapping memory), -1 = none; ops of
// one stream are ordered by the stream.

struct SOp {
  bool xchg;
  std::vector<Prim> prims;
  int64_t wait;
};

struct Schedule {
  std::vector<SOp> ops;
  bool c_join = false;        // comm stream waits for the caller's prior work
  int64_t final_wait = -1;    // op of the comm stream the caller's stream waits for at the end
  uint64_t stage_elems = 0;   // BINE_BUF_STAGE workspace (relay mode)
  int relayed_steps = 0;
  std::vector<char> signals;  // op i is waited on (by an op's `wait` or final_wait): record its event
};

struct SchedCfg {
  size_t chunk = 0;       // pipelining chunk, elements (0: none)
  bool in_place = false;
  size_t relay_min = 0;   // relay mode: smallest relayed part, elements (0: off)
};

// Host staging of a schedule (bine_allreduce_staged / bine_reduce_scatter_staged):
// the input buffer (SBUF, or RBUF in place) is copied host -> device piece by
// piece just before the first op that touches each piece, and the output
// (RBUF) device -> host piece by piece right after the op that writes it last.
// h2d[i] = input element ranges first touched by op i (copied before it);
// h2d_wait[i] = the newest op whose h2d batch op i must wait for (-1: none);
// d2h[i] = output element ranges op i writes last (copied after it).
using Ivl = std::pair<uint64_t, uint64_t>;  // [lo, hi) in elements
struct StageRanges {
  std::vector<std::vector<Ivl>> h2d, d2h;
  std::vector<int64_t> h2d_wait;
};
void stage_ranges(const Schedule &sc, bool in_place, StageRanges &out);

// issue.cpp.  `all` = the plans of every rank (same arguments, rank varied);
// needed only for relay mode (null: no relay).
void make_schedule(const Plan &plan, const std::vector<Plan> *all, int rank, const SchedCfg &cfg, Schedule &out);
void make_schedule(const Plan &plan, size_t chunk, bool in_place, Schedule &out);

// ---- transports (executor.cpp, direct.cpp) -------------------------------------
struct XSend { int peer; const void *ptr; size_t bytes; };
struct XRecv { int peer; void *ptr; size_t bytes; };

// ---- kernels (kernels.hip) ----------------------------------------------------
int launch_reduce(const void *a, const void *b, void *out, size_t count, int dtype, int op,
                  void *stream);   // out = b (op) a
// up to kMaxBatch windows in one launch; BINE_ERR_ARG if a window is not
// co-aligned mod 16 B (then launch them one by one)
constexpr int kMaxBatch = 8;
int launch_reduce_batch(int n, const void *const *a, const void *const *b, void *const *out, const size_t *count,
                        int dtype, int op, void *stream);
// out = the reduction tree over nl (2..kMaxLeaves, power of two) leaves in
// tree order:
// level by level (w = 1, 2, 4, ...) v[i] = v[i] (op) v[i + w] for i % 2w == 0
// (v[i + w] (op) v[i] at the levels whose bit is set in `swap`)
constexpr int kMaxLeaves = 16;
int launch_reduce_tree(int nl, const void *const *leaf, void *out, size_t count, int dtype, int op, void *stream,
                       unsigned swap = 0);
// the logical / bitwise ops' instantiations (kernels.hip compiled with
// BINE_OPSET=1); the entry points above forward those ops here
int launch_reduce_logic(const void *a, const void *b, void *out, size_t count, int dtype, int op, void *stream);
int launch_reduce_batch_logic(int n, const void *const *a, const void *const *b, void *const *out,
                              const size_t *count, int dtype, int op, void *stream);
int launch_reduce_tree_logic(int nl, const void *const *leaf, void *out, size_t count, int dtype, int op,
                             void *stream, unsigned swap);
// copy_buffer on the device (k_copy); hipMemcpyAsync when src / dst are not
// co-aligned mod 16 B
int launch_copy(void *dst, const void *src, size_t bytes, void *stream);
int launch_fill_pico(void *buf, size_t count, int dtype, uint32_t seed, void *stream);

// direct peer-memory transport (direct.cpp): one launch moves up to kMaxDm
// messages, `wgs` workgroups each (k_dm_move).  Sequence numbers live in the
// device (per peer and direction, in the rank's own inbox) and every address
// and flag is derived from them in the kernel, so launches carry no host-side
// state and can be captured into a graph and replayed.
constexpr int kMaxDm = 32;
// the inbox layout (bytes from its base): flags region, then the data slots
namespace dm {
constexpr size_t kFlagStride = 128;  // one flag / counter per 128-B line
constexpr size_t kReadyOff = 0, kAckOff = 64 << 10, kCntPushOff = 128 << 10, kCntPullOff = 192 << 10,
                 kPoisonOff = 256 << 10, kBaseSendOff = 260 << 10, kBaseRecvOff = 264 << 10,
                 kLaunchCntOff = 268 << 10, kPeerTabOff = 272 << 10, kPingOff = 288 << 10,
                 kGeomOff = 296 << 10;
// Slice flags of k_dm_fused (round 6): workgroup w of a launch of `wgs`
// workgroups owns slice w of every message (slice(): [n w / wgs, n (w+1) / wgs)
// of its n vectors), so a receiver's workgroup w needs only the SENDER's
// workgroup w to be done with slice w, not the whole message.  Per (ordered
// pair, slot, slice) a ready flag (in the receiver's inbox, set by the sender's
// workgroup w after its stores of slice w were acknowledged) and an ack flag
// (in the sender's inbox, set by the receiver's workgroup w after its reads of
// slice w completed); value = seq << kSliceWgsBits | wgs of the setter's launch
// -- a slice flag stands for slice w only when both ends cut the message with
// the same wgs (the message sizes match by construction).  The whole-message
// flags are still published (the last arriver), so a peer issuing another
// form waits on those.  kGeomOff: per (peer, slot) the sequence number and
// vector count of this rank's last k_dm_fused push into that slot (local), so
// a push can tell whether the receiver's slice acks of the slot's previous use
// cover the bytes it is about to overwrite.
// Layout [w][x][k]: one 128-B line per (slice w, pair x) holds that pair's
// kSlots flags of slice w -- written only by one sender workgroup, polled
// only by one receiver workgroup (flags of different workgroups in one line
// made the phases contend for it: C3 at P = 2 0.385 -> 0.412 ms).
constexpr int kSliceMax = 1024, kSliceWgsBits = 12;
constexpr size_t kSliceLine = 128;
constexpr size_t kSliceReadyOff = 320 << 10,
                 kSliceAckOff = kSliceReadyOff + (size_t)kSliceMax * 64 * kSliceLine,   // x kMaxPeers
                 kFlagsBytes = kSliceAckOff + (size_t)kSliceMax * 64 * kSliceLine;
// the slice flag of (slice w, pair x, slot k) from a region's base
constexpr size_t slice_off(size_t w, size_t x, size_t k) { return (w * 64 + x) * kSliceLine + k * 8; }
constexpr int kSlots = 4;      // slots per ordered pair
constexpr int kMaxPeers = 64;  // P limit of the layout (flag regions: P * kSlots * 128 B <= 64 KiB)
static_assert(kSliceAckOff - kSliceReadyOff == (size_t)kMaxPeers * kSliceMax * kSliceLine &&
                  kFlagsBytes - kSliceAckOff == (size_t)kMaxPeers * kSliceMax * kSliceLine &&
                  kSlots * 8 <= kSliceLine &&
                  kGeomOff + (size_t)kMaxPeers * kSlots * 16 <= kSliceReadyOff && kFlagsBytes % 4096 == 0,
              "inbox layout");
}  // namespace dm
struct DmMsg {
  const uint8_t *src;  // push: the data to send (pull: unused -- the slot)
  uint8_t *dst;        // pull: where the data goes (push: unused -- the peer's slot)
  uint64_t bytes;
  int push;            // 1: into the peer's inbox, 0: out of our own
  int peer;
  int j;               // this launch's j-th message of this kind to / from `peer`: seq = base[peer] + j + 1
  int leaf = -1;       // k_dm_move_tree: >= 0 -- a pull whose slot is a leaf of the launch's tree (read in
                       // place, never copied); -1 -- copied by its own workgroups
  int grp = -1;        // a push of the same bytes to several peers: index in m of the group's leader, whose
                       // workgroups read the source once and store it into every member's slot; -1: alone
};
// Residency: every workgroup of a direct-transport launch
// may wait on a flag that a workgroup of a peer's launch sets.  A launch whose
// workgroups cannot all be resident at once -- together with the launches of
// the other `share` ranks on the same GPU -- can fill the chip with waiters
// whose producers never get a slot: a residency stall (the hardware
// scheduler's time slicing resolves it slowly, or a wait times out).  So every
// launch is cut to fit: its workgroups (each copy entry's cwgs, the tree's
// twgs, the fused kernel's wgs) are scaled so that they sum to at most
// cap = CUs x (resident blocks per CU of the kernel (hipOccupancy...) - margin)
// / share (dm_residency_cap).  The margin (one workgroup per CU,
// BINE_DIRECT_RESIDENCY_MARGIN) is what any other wave on the GPU may hold
// while the spinning ones hold theirs: with 8 ranks on one GPU at the exact
// cap (8 x 160 = 1,280 = 256 CUs x 5) a producer's last workgroups got a slot
// only after the first waiter timed out.
// dm_fit_residency: scale `cw[0..n)` and *tw (null: none) proportionally,
// each >= 1, to sum <= cap.  0: unchanged (already fits or cap <= 0),
// 1: scaled, -1: n parts (+ the tree) alone exceed cap (left unchanged).
int dm_fit_residency(int *cw, int n, int *tw, int cap);
// the cap from the device's CUs, the kernel's resident blocks per CU, the
// margin (blocks per CU left free; never below one resident block per CU)
// and the ranks sharing the GPU; 0 when unknown (cus or per_cu <= 0)
inline int dm_residency_cap(int cus, int per_cu, int margin, int share) {
  if (cus <= 0 || per_cu <= 0) return 0;
  const int per = per_cu - margin >= 1 ? per_cu - margin : 1;
  return cus * per / (share >= 1 ? share : 1);
}
// the cap itself on the current device: kind 0 k_dm_move, 1 k_dm_move_tree for
// (dtype, op, nl), 2 k_dm_fused for (dtype, op); -1: no such kernel, 0: unknown
int dm_launch_cap(int kind, int dtype, int op, int nl, int share);
struct DmArgs {
  int nmsg = 0;
  int wgs = 1;
  int rank = 0;
  int share = 1;                   // ranks of this transport on this GPU (the residency cap's divisor)
  uint64_t slot = 0;               // bytes per slot
  uint8_t *own = nullptr;          // this rank's inbox (flags, counters, sequence bases, peer table)
  uint32_t *poison_host = nullptr; // mapped host word set together with the inbox's poison word
  uint64_t timeout_ticks = 0;      // wall_clock64 ticks
  DmMsg m[kMaxDm];
  int ncopy = 0;                   // messages with workgroups of their own (standalone copies, group leaders):
  int cidx[kMaxDm] = {};           // indices into m, in dispatch order,
  int cwgs[kMaxDm] = {};           // and their workgroups (wgs; wgs x members for a group)
  int ncw = 0;                     // sum of cwgs: the copy workgroups of the launch
  // diagnostics (BINE_DIRECT_STAMPS): per-workgroup wall_clock64 stamps of
  // entry / wait done / copy done, appended to `stamps` (dm::Stamp layout);
  // null: off
  uint64_t *stamps = nullptr;
  uint32_t serial = 0;             // the launch's number (host-side count)
};
namespace dm {
// stamps buffer: [0] records written (atomic), [1] capacity (records), then
// records of 4 words: tag = serial << 32 | kind << 24 | msg << 16 | wg, and the
// workgroup's wall_clock64 at entry, when its wait ended, when its copy (or
// tree) ended.  kind: 0 push, 1 pull, 2 tree, 3 push group
constexpr int kStampHdr = 8, kStampWords = 4;
// The mapped host words (DirectState::hpoison, kHostBytes): word 0's low half
// is the poison flag; 64-bit words kRecFirst .. kRecFirst + kRecWords - 1 hold
// the first timed-out waiter's record (dm_time_out, kernels.hip): kind << 8 |
// phase, rank, peer, slot, sequence number wanted, flag value last seen,
// launch serial, workgroup << 16 | thread, wall_clock64 ticks waited
constexpr int kRecFirst = 1, kRecWords = 9;
constexpr size_t kHostBytes = 128;
// what the waiter was: a push waits for the receiver's acknowledgement of the
// slot's previous use, a pull / leaf for the sender's ready mark
enum WaitKind : uint32_t {
  kWaitMovePush = 1,   // k_dm_move push
  kWaitMovePull = 2,   // k_dm_move pull
  kWaitGroupPush = 3,  // k_dm_move push group (BINE_DIRECT_MCAST)
  kWaitTreeLeaf = 4,   // k_dm_move_tree leaf
  kWaitFusedPush = 5,  // k_dm_fused push (phase 0: A, 1 + c: the allgather pieces of tree c)
  kWaitFusedPull = 6,  // k_dm_fused leaf (phase 1 + c) or allgather pull (phase 15: D)
  kWaitPing = 7,       // k_dm_ping (bine_comm_direct_ping): the peer's answer
};
}  // namespace dm
int launch_dm_move(const DmArgs &a, void *stream);

// The flag latency probe (k_dm_ping, bine_comm_direct_ping): ping flags at
// dm::kPingOff + x * kFlagStride of the inbox of rank y, written by rank x
// (monotonic: sequence numbers base + 1 .. base + iters, base = the pair's
// earlier pings, counted on the host by both ranks alike)
struct DmPingArgs {
  uint8_t *own = nullptr;
  uint32_t *poison_host = nullptr;
  uint64_t timeout_ticks = 0;
  uint64_t base = 0;
  uint64_t *out = nullptr;  // device word: wall_clock64 ticks of round trips 2 .. iters (0: timed out)
  int rank = 0, peer = 0, iters = 0, initiator = 0;
  uint32_t serial = 0;
};
int launch_dm_ping(const DmPingArgs &a, void *stream);

// The flat reduce-scatter's tree evaluated INSIDE the exchange launch that
// receives its leaves (k_dm_move_tree<T, OP, NL>): the launch's copy messages
// (pushes, and pulls that are not leaves) run as in k_dm_move on their
// `wgs` workgroups each; `twgs` further workgroups wait for the leaf pulls'
// ready marks, evaluate the reference's tree (own leaf at `pos`, per-level
// swap bits) reading the received leaves in place in the inbox slots, write
// `out`, and acknowledge every leaf slot -- the pull copy into a staging area
// and the separate tree launch of the unfused form are gone (one HBM pass
// over every received byte less).  Slots, flags, counters and sequence bases
// are k_dm_move's; a leaf pull is counted and acknowledged like a copied one,
// so both ends see the same protocol.
struct DmTree {
  int nl = 0, pos = 0;
  unsigned swap = 0;
  int twgs = 0;                 // tree workgroups (dispatched after the copy workgroups, DmArgs::cidx)
  int leaf_msg[kMaxLeaves] = {};  // tree position -> DmArgs::m index (-1 at pos)
  const void *own_leaf = nullptr;
  void *out = nullptr;
  uint64_t nvec = 0;            // 16-B vectors per leaf and of `out`
};
// BINE_ERR_UNSUPPORTED: no instantiation for (dtype, op, nl) -- the caller
// issues the unfused form
int launch_dm_move_tree(const DmArgs &a, const DmTree &t, int dtype, int op, void *stream);
bool dm_tree_supported(int dtype, int op, int nl);

// A whole flat-form collective in ONE launch over the direct transport
// (k_dm_fused): phase A pushes this rank's blocks (every chunk) into the
// peers' inboxes; then for each chunk c, phase B_c waits for the peers' blocks
// of that chunk and evaluates the reference's reduction tree (the
// REDUCE_TREE primitive: own leaf at `pos`, the received blocks read straight
// out of the inbox slots, `swap` per level) into its `out`, pushing each
// result vector from registers into the peers' slots (the flat allgather's
// piece c); phase D copies the peers' results out of the inbox (absent for
// the one-shot latency form and for reduce-scatters).  Workgroup w handles
// the same 1/wgs slice of every message in every phase, so a workgroup only
// ever reads back what it wrote itself: no grid-wide barrier.  Every wait
// is for a flag that a peer sets in an EARLIER phase, and every workgroup of
// every rank's launch is resident (the residency cut), so the phases
// complete in order.  Messages use the same slots, flags, counters and
// device-side sequence bases as k_dm_move (j = the message's index among
// this launch's messages of its kind to / from its peer, < kSlots: no slot
// is used twice in one launch).
constexpr int kMaxFusedPeers = 15;  // P <= 16
constexpr int kMaxFusedTrees = 4;   // chunks of the tree phase
constexpr int kMaxFusedMsgs = 4 * kMaxFusedPeers;
struct DmFusedTree {
  const void *own_leaf = nullptr;
  void *out = nullptr;
  uint64_t nvec = 0;                   // 16-B vectors per leaf / of out
  int b0 = 0, nb = 0, nc = 0;          // leaves m[b0, b0 + nb), then the pushes of out m[b0 + nb, b0 + nb + nc)
  int8_t leaf[kMaxLeaves] = {};        // leaf j != pos: index in m of the pull carrying it
};
struct DmFusedArgs {
  int wgs = 1, rank = 0;
  int share = 1;                       // as DmArgs::share (wgs is cut to the residency cap)
  uint64_t slot = 0;
  uint8_t *own = nullptr;
  uint32_t *poison_host = nullptr;
  uint64_t timeout_ticks = 0;
  int na = 0, nt = 0, d0 = 0, nd = 0;  // phase A pushes m[0, na); trees t[0, nt); phase D pulls m[d0, d0 + nd)
  DmMsg m[kMaxFusedMsgs];
  int nl = 0, pos = 0;
  unsigned swap = 0;
  DmFusedTree t[kMaxFusedTrees];
  uint64_t *stamps = nullptr;          // DmArgs::stamps: one record per workgroup (kind 4: entry, end of the
  uint32_t serial = 0;                 // first wait, end)
  int slices = 1;                      // per-slice flags (dm::kSliceReadyOff; BINE_DIRECT_SLICE_FLAGS=0: off)
};
// BINE_ERR_UNSUPPORTED: (dtype, op) has no fused instantiation (the caller
// issues the primitives one by one)
int launch_dm_fused(const DmFusedArgs &a, int dtype, int op, void *stream);
int dm_fused_check(const DmFusedArgs &a, int dtype, int op);  // launch_dm_fused's argument check alone
bool dm_fused_supported(int dtype, int op);
int launch_checksum(const void *buf, size_t count, int dtype, uint64_t *out, void *stream);

}  // namespace bine
