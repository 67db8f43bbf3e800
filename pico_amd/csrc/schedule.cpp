// schedule.cpp -- per-rank execution plans of libbine's reduce-family.
//
// The reference interleaves its schedule with MPI calls inside each algorithm
// (libbine_allreduce.c, libbine_reduce_scatter.c, libbine_reduce.c).  Here the
// schedule is computed once, on the host, into an immutable list of primitives
// (SEND / RECV grouped into exchanges, REDUCE, REDUCE3, COPY) over five logical
// buffers (SBUF, RBUF, TMP0..2).  The device executor (executor.cpp) walks the
// list with RCCL P2P on one HIP stream and the CDNA4 reduce kernels on another.
//
// Differences from a literal reading of the reference, all deliberate:
//  * every receive carries the exact element count its matching send carries
//    (RCCL P2P needs equal counts; MPI only bounds them);
//  * messages of zero elements are dropped on both sides;
//  * an exchange with oneself becomes a local COPY;
//  * the first reduce-scatter step of remap/static/segmented reads the send
//    buffer directly (REDUCE3: rbuf = sbuf op recv) instead of copying sbuf to
//    rbuf first (libbine_allreduce.c:849-852) -- same values, one pass of HBM
//    traffic less;
//  * reference defects are not reproduced: the segmented tail that is never
//    reduced (libbine_allreduce.c:1211-1252), the static tmp_buf overflow
//    (:724 vs :749-765), reduce_scatter_butterfly / _bine_block_by_block leaving
//    rbuf untouched at P = 1 (libbine_reduce_scatter.c:585, :1098).
//  * assert()/hang cases of the reference return BINE_ERR_ARG.
#include <algorithm>
#include <array>
#include <cstring>
#include <map>

#include "bine_internal.h"

namespace bine {

// ---------------------------------------------------------------------------
// schedule math (restates libbine_utils.h)
// ---------------------------------------------------------------------------

static int rho(int step) {  // rhos[] of libbine_utils.h:44-45
  int v = 0, p = 1;
  for (int i = 0; i <= step; i++) { v += p; p *= -2; }
  return v;
}

int pi(int rank, int step, int P) {  // libbine_utils.h:129-138
  int d = (rank & 1) == 0 ? (rank + rho(step)) % P : (rank - rho(step)) % P;
  return d < 0 ? d + P : d;
}

bool is_pow2(int v) { return (v & (v - 1)) == 0; }

int log2_ceil(int v) {  // log_2(), libbine_utils.h:279-288
  if (v < 1) return -1;
  int l = 31 - __builtin_clz((unsigned)v);
  return is_pow2(v) ? l : l + 1;
}

static int floor_log2(int v) { return v < 1 ? -1 : 31 - __builtin_clz((unsigned)v); }  // hibit(v, 31)
static int next_pow2(int v) { return v == 0 ? 1 : (int)(1u << (32 - __builtin_clz((unsigned)v))); }
static int pmod(int a, int b) { int r = a % b; return r < 0 ? r + b : r; }
static uint32_t to_nb(int32_t b) { const uint32_t m = 0xAAAAAAAAu; return (m + (uint32_t)b) ^ m; }
static int32_t from_nb(uint32_t n) { const uint32_t m = 0xAAAAAAAAu; return (int32_t)((m ^ n) - m); }
static int nb_min(int n) { int v = 0; for (int i = 1; i < n; i += 2) v -= 1 << i; return v; }
static int nb_max(int n) { int v = 0; for (int i = 0; i < n; i += 2) v += 1 << i; return v; }
static bool nb_fits(int x, int n) { return x >= nb_min(n) && x <= nb_max(n); }
static uint32_t bitrev(uint32_t x) {
  x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
  x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
  x = ((x >> 4) & 0x0f0f0f0fu) | ((x & 0x0f0f0f0fu) << 4);
  x = ((x >> 8) & 0x00ff00ffu) | ((x & 0x00ff00ffu) << 8);
  return (x >> 16) | (x << 16);
}
static uint32_t top_bits(uint32_t x, int n) { return n <= 0 ? 0 : bitrev(x) >> (32 - n); }

// negabinary label of `rank` among P ranks: the (at most two) representable
// values congruent to +-rank mod P (libbine_utils.h:537-570, including its
// decimal-literal tie-break at :564)
static void nb_candidates(uint32_t P, uint32_t rank, uint32_t *a, uint32_t *b, int *nbits) {
  *a = *b = UINT32_MAX;
  int n = log2_ceil((int)P);
  *nbits = n;
  int x = (int)rank, y = (int)rank - (int)P;
  if (rank % 2 == 0) { x = -(int)rank; y = -(int)rank + (int)P; }
  if (nb_fits(x, n)) *a = to_nb(x);
  if (nb_fits(y, n)) *b = to_nb(y);
}

uint32_t remap_rank(uint32_t P, uint32_t rank) {  // libbine_utils.h:572-578
  uint32_t a, b;
  int n;
  nb_candidates(P, rank, &a, &b, &n);
  uint32_t v;
  if (a == UINT32_MAX) v = b;
  else if (b == UINT32_MAX) v = a;
  else {
    int sh = 32 - n;
    uint32_t probe = (uint32_t)(sh < 32 ? (80000000 >> sh) : 80000000);
    v = (a & probe) ? a : b;
  }
  if (v == UINT32_MAX) v = 0;
  return top_bits(v ^ (v >> 1), n);
}

uint32_t get_nu(uint32_t rank, uint32_t size) {  // libbine_utils.h:611-648
  uint32_t a, b;
  int n;
  nb_candidates(size, rank, &a, &b, &n);
  auto nu = [&](uint32_t v) { return top_bits(v ^ (v >> 1), n); };
  if (a == UINT32_MAX && b == UINT32_MAX) return 0;
  if (a == UINT32_MAX) return nu(b);
  if (b == UINT32_MAX) return nu(a);
  return std::min((int)nu(a), (int)nu(b));
}

// libbine_utils_bitmaps.c:10-56 -- final block of each rank in the static
// variants: the remap permutation with every last-step pair in rank order.
void static_perm(int P, std::vector<int> &perm) {
  int n = log2_ceil(P);
  perm.assign((size_t)P, 0);
  for (int r = 0; r < P; r++)
    perm[(size_t)r] = (int)(remap_rank((uint32_t)P, (uint32_t)r) & ~1u) | (r > pi(r, n - 1, P) ? 1 : 0);
}

static int nb_partner(int r, int mask, int P) {  // e.g. libbine_reduce_scatter.c:936-940
  int d = from_nb((uint32_t)((mask << 1) - 1));
  return r % 2 == 0 ? pmod(r + d, P) : pmod(r - d, P);
}

// ---------------------------------------------------------------------------
// plan builder
// ---------------------------------------------------------------------------

enum { SB = BINE_BUF_SBUF, RB = BINE_BUF_RBUF, T0 = BINE_BUF_TMP0, T1 = BINE_BUF_TMP1, T2 = BINE_BUF_TMP2 };

namespace {
struct Builder {
  Plan p;
  int rank;
  int group = 0;
  std::vector<Prim> pend_send, pend_recv;  // current exchange

  explicit Builder(int r) : rank(r) {}

  static Prim mk(int type) { Prim x; std::memset(&x, 0, sizeof x); x.type = type; x.aux_buf = -1; return x; }
  void send(int peer, int buf, uint64_t off, uint64_t n) {
    if (peer < 0 || n == 0) return;
    Prim x = mk(BINE_PRIM_SEND); x.peer = peer; x.src_buf = buf; x.src_off = off; x.count = n;
    pend_send.push_back(x);
  }
  void recv(int peer, int buf, uint64_t off, uint64_t n) {
    if (peer < 0 || n == 0) return;
    Prim x = mk(BINE_PRIM_RECV); x.peer = peer; x.dst_buf = buf; x.dst_off = off; x.count = n;
    pend_recv.push_back(x);
  }
  // close the exchange; `pipeline` marks a {1 send, 1 recv} exchange whose
  // receive is consumed element-for-element by the next REDUCE(3)
  void end(bool pipeline = false) {
    // an exchange with oneself is a local copy (send_remap's final step)
    for (size_t i = 0; i < pend_send.size(); i++) {
      if (pend_send[i].peer != rank) continue;
      for (size_t j = 0; j < pend_recv.size(); j++) {
        if (pend_recv[j].peer != rank) continue;
        copy(pend_send[i].src_buf, pend_send[i].src_off, pend_recv[j].dst_buf, pend_recv[j].dst_off,
             std::min(pend_send[i].count, pend_recv[j].count));
        pend_send.erase(pend_send.begin() + (long)i);
        pend_recv.erase(pend_recv.begin() + (long)j);
        i--;
        break;
      }
    }
    bool pipe = pipeline && pend_send.size() == 1 && pend_recv.size() == 1 &&
                pend_send[0].peer == pend_recv[0].peer;
    for (auto &x : pend_send) { x.group = group; x.flags = pipe ? BINE_PRIM_PIPELINE : 0; p.prims.push_back(x); }
    for (auto &x : pend_recv) { x.group = group; x.flags = pipe ? BINE_PRIM_PIPELINE : 0; p.prims.push_back(x); }
    if (!pend_send.empty() || !pend_recv.empty()) group++;
    pend_send.clear();
    pend_recv.clear();
  }
  void reduce(int in, uint64_t in_off, int io, uint64_t io_off, uint64_t n, bool pipe = false) {
    if (n == 0) return;
    Prim x = mk(BINE_PRIM_REDUCE);
    x.src_buf = in; x.src_off = in_off; x.dst_buf = io; x.dst_off = io_off; x.count = n;
    x.flags = pipe ? BINE_PRIM_PIPELINE : 0;
    p.prims.push_back(x);
  }
  // out = b (op) a
  void reduce3(int a, uint64_t a_off, int b, uint64_t b_off, int out, uint64_t out_off, uint64_t n,
               bool pipe = false) {
    if (n == 0) return;
    Prim x = mk(BINE_PRIM_REDUCE3);
    x.src_buf = a; x.src_off = a_off; x.aux_buf = b; x.aux_off = b_off; x.dst_buf = out;
    x.dst_off = out_off; x.count = n;
    x.flags = pipe ? BINE_PRIM_PIPELINE : 0;
    p.prims.push_back(x);
  }
  void copy(int src, uint64_t src_off, int dst, uint64_t dst_off, uint64_t n) {
    if (n == 0 || (src == dst && src_off == dst_off)) return;
    Prim x = mk(BINE_PRIM_COPY);
    x.src_buf = src; x.src_off = src_off; x.dst_buf = dst; x.dst_off = dst_off; x.count = n;
    p.prims.push_back(x);
  }
  // out = tree over nl leaves: leaf `pos` at (own, own_off), the k-th of the
  // others at (in, in_off + k * n)
  void reduce_tree(int nl, int pos, int own, uint64_t own_off, int in, uint64_t in_off, int out, uint64_t out_off,
                   uint64_t n, unsigned swap = 0) {
    if (n == 0) return;
    Prim x = mk(BINE_PRIM_REDUCE_TREE);
    x.peer = nl;
    x.pos = pos;
    x.flags = (int)(swap << 8);
    x.aux_buf = own; x.aux_off = own_off; x.src_buf = in; x.src_off = in_off;
    x.dst_buf = out; x.dst_off = out_off; x.count = n;
    p.prims.push_back(x);
  }
  void tmp(int t, uint64_t n) {
    uint64_t &s = p.tmp_elems[t - T0];
    s = std::max(s, n);
  }
  void fail(int st) { p.prims.clear(); p.status = st; }
};

// reduction "pipelined" only when the REDUCE directly follows its exchange
constexpr bool PIPE = true;

// ---------------------------------------------------------------------------
// flat reduce-scatter phase (PlanArgs::flat_rs)
// ---------------------------------------------------------------------------
// In a halving reduce-scatter whose step s pairs rank r with peer(r, s), the
// two partners share their window at every step and each keeps
// acc = acc (op) received on its half (every MPI_Reduce_local call of these
// schedules is reduce(received, own accumulator), e.g.
// libbine_allreduce.c:888, libbine_reduce_scatter.c:1034).  So the block rank x
// holds at the end is the binary tree
//     T(x, -1) = input of x,   T(x, s) = T(x, s-1) (op) T(peer(x, s), s-1),
// i.e. over the leaf order L(x, s) = L(x, s-1) ++ L(peer(x, s), s-1), combined
// level by level, left operand = inout.  flat_leaves() returns L(x, steps-1).
// own_first(r, s) = false puts the partner's subtree on the inout side of
// rank r's step-s combine (schedules whose operand order depends on the ranks).
template <typename Peer, typename OwnFirst>
std::vector<int> flat_leaves(int P, int steps, int x, Peer peer, OwnFirst own_first) {
  std::vector<std::vector<int>> L((size_t)P), N((size_t)P);
  for (int r = 0; r < P; r++) L[(size_t)r] = {r};
  for (int s = 0; s < steps; s++) {
    for (int r = 0; r < P; r++) {
      const auto &mine = L[(size_t)r], &o = L[(size_t)peer(r, s)];
      const bool f = own_first(r, s);
      N[(size_t)r] = f ? mine : o;
      N[(size_t)r].insert(N[(size_t)r].end(), f ? o.begin() : mine.begin(), f ? o.end() : mine.end());
    }
    L.swap(N);
  }
  return L[(size_t)x];
}
template <typename Peer>
std::vector<int> flat_leaves(int P, int steps, int x, Peer peer) {
  return flat_leaves(P, steps, x, peer, [](int, int) { return true; });
}

bool flat_rs_fits(const PlanArgs &a) { return a.flat_rs && a.P >= 2 && a.P <= kMaxLeaves && is_pow2(a.P); }

// One all-peers exchange per chunk: this rank sends block x (boff[x], bcnt[x]
// of buffer `src`) to rank x for every x != rank, receives its own block from
// the P-1 others into TMP0 (chunk-major staging, leaf order), and reduces the
// chunk with one REDUCE_TREE into (out, out_off).  `leaves` = the tree of the
// block this rank computes (this rank's own contribution is one of them, not
// necessarily the first: send_remap / static hand the block to another rank).
//
// `ag`: the caller's flat allgather follows (every rank sends the block it
// computed, RB[boff[x], bcnt[x]], to every other).  With
// PlanArgs::flat_ag_chunked that allgather is cut with the same chunks and
// emitted here, chunk k's results leaving right after chunk k+1's
// reduce-scatter exchange (so the comm stream never waits for a tree with
// nothing else to move); returns true when it did (the caller then skips its
// own).  Pure data movement: the same bytes in the same places.
static bool flat_ag_here(const PlanArgs &a, bool ag, int out, uint64_t out_off, uint64_t own_off) {
  return ag && a.flat_ag && a.flat_ag_chunked && out == RB && out_off == own_off;
}

static void flat_ag_chunk(Builder &b, const PlanArgs &a, const std::vector<uint64_t> &boff,
                          const std::vector<uint64_t> &bcnt, uint64_t o, uint64_t ch) {
  const int P = a.P, r = a.rank;
  const uint64_t mine = bcnt[(size_t)r];
  const uint64_t cl = o < mine ? std::min(ch, mine - o) : 0;
  for (int x = 0; x < P; x++)
    if (x != r) b.send(x, RB, boff[(size_t)r] + o, cl);
  for (int x = 0; x < P; x++)
    if (x != r && o < bcnt[(size_t)x]) b.recv(x, RB, boff[(size_t)x] + o, std::min(ch, bcnt[(size_t)x] - o));
  b.end();
}

bool flat_rs(Builder &b, const PlanArgs &a, int src, const std::vector<uint64_t> &boff,
             const std::vector<uint64_t> &bcnt, const std::vector<int> &leaves, int out, uint64_t out_off,
             unsigned swap = 0, bool ag = false) {
  const int P = a.P, r = a.rank;
  uint64_t cmax = 0;
  for (int x = 0; x < P; x++) cmax = std::max(cmax, bcnt[(size_t)x]);
  const uint64_t mine = bcnt[(size_t)r];
  const uint64_t ch = a.flat_chunk ? a.flat_chunk : std::max<uint64_t>(cmax, 1);
  const bool agc = flat_ag_here(a, ag, out, out_off, boff[(size_t)r]);
  b.tmp(T0, (uint64_t)(P - 1) * mine);
  uint64_t k = 0;
  for (; k * ch < cmax; k++) {
    const uint64_t o = k * ch;
    for (int x = 0; x < P; x++)
      if (x != r && o < bcnt[(size_t)x]) b.send(x, src, boff[(size_t)x] + o, std::min(ch, bcnt[(size_t)x] - o));
    const uint64_t base = (uint64_t)(P - 1) * o, cl = o < mine ? std::min(ch, mine - o) : 0;
    int pos = 0, slot = 0;
    for (int j = 0; j < P; j++) {
      if (leaves[(size_t)j] == r) { pos = j; continue; }
      b.recv(leaves[(size_t)j], T0, base + (uint64_t)slot++ * cl, cl);
    }
    b.end();
    if (agc && k > 0) flat_ag_chunk(b, a, boff, bcnt, o - ch, ch);
    b.reduce_tree(P, pos, src, boff[(size_t)r] + o, T0, base, out, out_off + o, cl, swap);
  }
  if (agc && k > 0) flat_ag_chunk(b, a, boff, bcnt, (k - 1) * ch, ch);
  return agc;
}

// The rings' reduction is a chain, not a balanced tree: block b travels the
// ring and every rank folds its own contribution in as the inout side,
// v = x_j (op) v.  Flat form: the same all-peers exchange as flat_rs, then the
// chain folded over the staged leaves (`order` = leaf ranks in chain order,
// this rank's own leaf last) with P-1 pairwise reductions, each on a staged
// slot, the last one into (out, out_off).
bool flat_chain(Builder &b, const PlanArgs &a, int src, const std::vector<uint64_t> &boff,
                const std::vector<uint64_t> &bcnt, const std::vector<int> &order, int out, uint64_t out_off,
                bool ag = false) {
  const int P = a.P, r = a.rank;
  uint64_t cmax = 0;
  for (int x = 0; x < P; x++) cmax = std::max(cmax, bcnt[(size_t)x]);
  const uint64_t mine = bcnt[(size_t)r];
  const uint64_t ch = a.flat_chunk ? a.flat_chunk : std::max<uint64_t>(cmax, 1);
  const bool agc = flat_ag_here(a, ag, out, out_off, boff[(size_t)r]);
  b.tmp(T0, (uint64_t)(P - 1) * mine);
  uint64_t k = 0;
  for (; k * ch < cmax; k++) {
    const uint64_t o = k * ch;
    for (int x = 0; x < P; x++)
      if (x != r && o < bcnt[(size_t)x]) b.send(x, src, boff[(size_t)x] + o, std::min(ch, bcnt[(size_t)x] - o));
    const uint64_t base = (uint64_t)(P - 1) * o, cl = o < mine ? std::min(ch, mine - o) : 0;
    for (int j = 0; j + 1 < P; j++) b.recv(order[(size_t)j], T0, base + (uint64_t)j * cl, cl);
    b.end();
    if (agc && k > 0) flat_ag_chunk(b, a, boff, bcnt, o - ch, ch);
    for (int j = 1; j + 1 < P; j++) b.reduce(T0, base + (uint64_t)(j - 1) * cl, T0, base + (uint64_t)j * cl, cl);
    b.reduce3(T0, base + (uint64_t)(P - 2) * cl, src, boff[(size_t)r] + o, out, out_off + o, cl);
  }
  if (agc && k > 0) flat_ag_chunk(b, a, boff, bcnt, (k - 1) * ch, ch);
  return agc;
}

// ---------------------------------------------------------------------------
// allreduce -- libbine_allreduce.c
// ---------------------------------------------------------------------------

// allreduce_recursivedoubling, :17-135
void ar_recursivedoubling(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const uint64_t n = a.count;
  const int src = a.in_place ? RB : SB;
  if (P == 1) { b.copy(src, 0, RB, 0, n); return; }
  if (flat_rs_fits(a)) {  // one-shot, as allreduce_bine_lat: partners x ^ 2^s, acc = acc (op) received
    std::vector<uint64_t> boff((size_t)P, 0), bcnt((size_t)P, n);
    flat_rs(b, a, src, boff, bcnt, flat_leaves(P, log2_ceil(P), r, [](int x, int s) { return x ^ (1 << s); }), RB, 0);
    return;
  }
  b.tmp(T0, n);
  b.copy(src, 0, T0, 0, n);  // inplacebuf
  int tsend = T0, newrank;
  const int adj = next_pow2(P) >> 1, extra = P - adj;
  if (r < 2 * extra) {
    if (r % 2 == 0) { b.send(r + 1, T0, 0, n); b.end(); newrank = -1; }
    else { b.recv(r - 1, RB, 0, n); b.end(); b.reduce(RB, 0, T0, 0, n); newrank = r >> 1; }
  } else newrank = r - extra;
  for (int dist = 1; dist < adj && newrank >= 0; dist <<= 1) {
    int nr = newrank ^ dist, remote = nr < extra ? nr * 2 + 1 : nr + extra;
    b.send(remote, T0, 0, n); b.recv(remote, RB, 0, n); b.end(PIPE);
    b.reduce(RB, 0, T0, 0, n, PIPE);
  }
  if (r < 2 * extra) {
    if (r % 2 == 0) { b.recv(r + 1, RB, 0, n); b.end(); tsend = RB; }
    else { b.send(r - 1, T0, 0, n); b.end(); }
  }
  if (tsend != RB) b.copy(T0, 0, RB, 0, n);
}

// COLL_BASE_COMPUTE_BLOCKCOUNT, libbine_utils.h:63-69
struct Blocks {
  uint64_t early, late;
  int split;
  Blocks(uint64_t count, int nb) {
    early = late = count / (uint64_t)nb;
    split = (int)(count % (uint64_t)nb);
    if (split) early++;
  }
  uint64_t off(int blk) const { return blk < split ? (uint64_t)blk * early : (uint64_t)blk * late + (uint64_t)split; }
  uint64_t cnt(int blk) const { return blk < split ? early : late; }
  // a run of w blocks starting at `start` (libbine_allreduce.c:749-756)
  uint64_t wcnt(int start, int w) const {
    if (start + w <= split) return (uint64_t)w * early;
    if (start >= split) return (uint64_t)w * late;
    return (uint64_t)w * late + (uint64_t)(split - start);
  }
};

// allreduce_ring, :138-319
void ar_ring(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const uint64_t n = a.count;
  const int src = a.in_place ? RB : SB;
  if (P == 1) { b.copy(src, 0, RB, 0, n); return; }
  if (n < (uint64_t)P) { ar_recursivedoubling(b, a); return; }
  Blocks bl(n, P);
  if (flat_rs_fits(a)) {
    // block y starts at rank y and ends, folded, at rank y - 1: rank r
    // computes block r + 1 from the chain r + 1, r + 2, ..., r + P - 1, r
    std::vector<uint64_t> boff((size_t)P), bcnt((size_t)P);
    for (int x = 0; x < P; x++) { boff[(size_t)x] = bl.off((x + 1) % P); bcnt[(size_t)x] = bl.cnt((x + 1) % P); }
    std::vector<int> order;
    for (int j = 1; j <= P; j++) order.push_back((r + j) % P);
    const bool agd = flat_chain(b, a, src, boff, bcnt, order, RB, boff[(size_t)r], true);
    if (agd) return;
    if (a.flat_ag) {
      for (int x = 0; x < P; x++)
        if (x != r) b.send(x, RB, boff[(size_t)r], bcnt[(size_t)r]);
      for (int x = 0; x < P; x++)
        if (x != r) b.recv(x, RB, boff[(size_t)x], bcnt[(size_t)x]);
      b.end();
      return;
    }
    const int to = (r + 1) % P, from = (r + P - 1) % P;
    for (int k = 0; k < P - 1; k++) {  // :282-304
      const int rf = (r + P - k) % P, sf = (r + 1 + P - k) % P;
      b.send(to, RB, bl.off(sf), bl.cnt(sf)); b.recv(from, RB, bl.off(rf), bl.cnt(rf)); b.end();
    }
    return;
  }
  b.tmp(T0, bl.early); b.tmp(T1, bl.early);
  const int ib[2] = {T0, T1};
  b.copy(src, 0, RB, 0, n);
  const int to = (r + 1) % P, from = (r + P - 1) % P;
  int inbi = 0;
  b.recv(from, ib[inbi], 0, bl.cnt(from)); b.send(to, RB, bl.off(r), bl.cnt(r)); b.end();
  for (int k = 2; k < P; k++) {
    const int prev = (r + P - k + 1) % P, incoming = (r + P - k) % P;
    inbi ^= 1;
    b.reduce(ib[inbi ^ 1], 0, RB, bl.off(prev), bl.cnt(prev));
    b.recv(from, ib[inbi], 0, bl.cnt(incoming)); b.send(to, RB, bl.off(prev), bl.cnt(prev)); b.end();
  }
  const int last = (r + 1) % P;
  b.reduce(ib[inbi], 0, RB, bl.off(last), bl.cnt(last));
  for (int k = 0; k < P - 1; k++) {  // :282-304
    const int rf = (r + P - k) % P, sf = (r + 1 + P - k) % P;
    b.send(to, RB, bl.off(sf), bl.cnt(sf)); b.recv(from, RB, bl.off(rf), bl.cnt(rf)); b.end();
  }
}

// allreduce_rabenseifner, :441-694
void ar_rabenseifner(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const uint64_t n = a.count;
  const int steps = floor_log2(P), adj = 1 << steps, rem = P - adj;
  b.tmp(T0, n);
  // rank x's block after the halving of :553-590 (power-of-two P)
  auto owned = [&](int x, uint64_t *off, uint64_t *cnt) {
    uint64_t ww = n, o = 0;
    for (int mask = 1; mask < adj; mask <<= 1) {
      const int d = x ^ mask;
      if (x < d) ww = ww / 2;
      else { o += ww / 2; ww = ww - ww / 2; }
    }
    *off = o;
    *cnt = ww;
  };
  const bool flat = rem == 0 && flat_rs_fits(a);
  if (!a.in_place && !flat) b.copy(SB, 0, RB, 0, n);
  const uint64_t lh = n / 2, rh = n - lh;
  int vrank;
  bool agd = false;  // flat_rs emitted the chunked allgather
  if (r < 2 * rem) {
    if (r % 2) {
      b.send(r - 1, RB, 0, lh); b.recv(r - 1, T0, lh, rh); b.end(PIPE);
      b.reduce(T0, lh, RB, lh, rh, PIPE);
      b.send(r - 1, RB, lh, rh); b.end();
      vrank = -1;
    } else {
      b.send(r + 1, RB, lh, rh); b.recv(r + 1, T0, 0, lh); b.end(PIPE);
      b.reduce(T0, 0, RB, 0, lh, PIPE);
      b.recv(r + 1, RB, lh, rh); b.end();
      vrank = r / 2;
    }
  } else vrank = r - rem;
  if (vrank != -1) {
    std::vector<uint64_t> ri(steps + 1), si(steps + 1), rc(steps + 1), sc(steps + 1);
    uint64_t w = n;
    int step = 0;
    for (int mask = 1; mask < adj; mask <<= 1) {
      int vdest = vrank ^ mask, dest = vdest < rem ? vdest * 2 : vdest + rem;
      if (r < dest) { rc[step] = w / 2; sc[step] = w - rc[step]; si[step] = ri[step] + rc[step]; }
      else { sc[step] = w / 2; rc[step] = w - sc[step]; ri[step] = si[step] + sc[step]; }
      if (!flat) {
        b.send(dest, RB, si[step], sc[step]); b.recv(dest, T0, ri[step], rc[step]); b.end(PIPE);
        b.reduce(T0, ri[step], RB, ri[step], rc[step], PIPE);
      }
      if (step + 1 < steps) { ri[step + 1] = ri[step]; si[step + 1] = ri[step]; w = rc[step]; step++; }
    }
    if (flat && steps >= 1) {  // partners x ^ 2^s, acc = acc (op) received
      std::vector<uint64_t> boff((size_t)P), bcnt((size_t)P);
      for (int x = 0; x < P; x++) owned(x, &boff[(size_t)x], &bcnt[(size_t)x]);
      agd = flat_rs(b, a, a.in_place ? RB : SB, boff, bcnt,
                    flat_leaves(P, steps, r, [](int x, int s) { return x ^ (1 << s); }), RB, boff[(size_t)r], 0, true);
    }
    if (agd) {
    } else if (a.flat_ag && rem == 0 && steps >= 1) {
      // one all-peers exchange: rank x's block after the halving
      for (int x = 0; x < P; x++)
        if (x != r) b.send(x, RB, ri[steps - 1], rc[steps - 1]);
      for (int x = 0; x < P; x++) {
        if (x == r) continue;
        uint64_t o, c;
        owned(x, &o, &c);
        b.recv(x, RB, o, c);
      }
      b.end();
    } else {
      step = steps - 1;
      for (int mask = adj >> 1; mask > 0; mask >>= 1) {
        int vdest = vrank ^ mask, dest = vdest < rem ? vdest * 2 : vdest + rem;
        b.send(dest, RB, ri[step], rc[step]); b.recv(dest, RB, si[step], sc[step]); b.end();
        step--;
      }
    }
  }
  if (r < 2 * rem) {
    if (r % 2) b.recv(r - 1, RB, 0, n); else b.send(r + 1, RB, 0, n);
    b.end();
  }
}

// allreduce_bine_lat, :321-439
void ar_bine_lat(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const uint64_t n = a.count;
  const int src = a.in_place ? RB : SB;
  if (P == 1) { b.copy(src, 0, RB, 0, n); return; }
  if (flat_rs_fits(a)) {
    // recursive doubling with acc = acc (op) received at every step: rank x's
    // result is the tree T(x) over the partners pi -- a different association
    // on every rank, as in the reference.  One-shot form: every rank sends its
    // whole vector to every other (one hop each) and evaluates its own tree.
    std::vector<uint64_t> boff((size_t)P, 0), bcnt((size_t)P, n);
    flat_rs(b, a, src, boff, bcnt, flat_leaves(P, log2_ceil(P), r, [P](int x, int s) { return pi(x, s, P); }), RB, 0);
    return;
  }
  b.tmp(T0, n);
  b.copy(src, 0, T0, 0, n);
  int tsend = T0;
  const int steps = floor_log2(P), adj = 1 << steps, extra = P - adj;
  const bool pw2 = is_pow2(P);
  int nr = r;
  bool idle = false;
  if (r < 2 * extra) {
    if (r % 2 == 0) { b.send(r + 1, T0, 0, n); b.end(); idle = true; }
    else { b.recv(r - 1, RB, 0, n); b.end(); b.reduce(RB, 0, T0, 0, n); nr = r >> 1; }
  } else nr = r - extra;
  for (int s = 0; s < steps && !idle; s++) {
    int vd = pi(nr, s, adj), dest = pw2 ? vd : (vd < extra ? (vd << 1) + 1 : vd + extra);
    b.send(dest, T0, 0, n); b.recv(dest, RB, 0, n); b.end(PIPE);
    b.reduce(RB, 0, T0, 0, n, PIPE);
  }
  if (r < 2 * extra) {
    if (!idle) b.send(r - 1, T0, 0, n);
    else { b.recv(r + 1, RB, 0, n); tsend = RB; }
    b.end();
  }
  if (tsend != RB) b.copy(T0, 0, RB, 0, n);
}

// allreduce_bine_bdw_static, :696-817
void ar_bine_bdw_static(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const uint64_t n = a.count;
  const int steps = log2_ceil(P);
  if (!is_pow2(P) || steps < 1) { b.fail(BINE_ERR_ARG); return; }
  Blocks bl(n, P);
  std::vector<int> perm;
  static_perm(P, perm);
  auto recv_start = [&](int rank, int s) { int w = P >> (s + 1); return perm[(size_t)rank] & ~(w - 1); };
  b.tmp(T0, bl.wcnt(0, P / 2) + bl.early);
  const bool elide = !a.in_place;  // step 0 reads sbuf, writes rbuf
  int w = P;
  if (flat_rs_fits(a)) {  // rank x computes block perm[x]
    std::vector<uint64_t> boff((size_t)P), bcnt((size_t)P);
    for (int x = 0; x < P; x++) { boff[(size_t)x] = bl.off(perm[(size_t)x]); bcnt[(size_t)x] = bl.wcnt(perm[(size_t)x], 1); }
    const auto leaves = flat_leaves(P, steps, r, [&](int x, int s) { return pi(x, s, P); });
    if (flat_rs(b, a, a.in_place ? RB : SB, boff, bcnt, leaves, RB, boff[(size_t)r], 0, true)) return;
    w = 1;
  }
  for (int s = 0; s < steps && w > 1; s++) {
    w >>= 1;
    const int dest = pi(r, s, P), sb = recv_start(dest, s), rb = recv_start(r, s);
    const int sbuf = (elide && s == 0) ? SB : RB;
    b.send(dest, sbuf, bl.off(sb), bl.wcnt(sb, w)); b.recv(dest, T0, 0, bl.wcnt(rb, w)); b.end(PIPE);
    if (elide && s == 0) b.reduce3(T0, 0, SB, bl.off(rb), RB, bl.off(rb), bl.wcnt(rb, w), PIPE);
    else b.reduce(T0, 0, RB, bl.off(rb), bl.wcnt(rb, w), PIPE);
  }
  if (a.flat_ag) {  // rank x owns block perm[x] after the reduce-scatter
    for (int x = 0; x < P; x++)
      if (x != r) b.send(x, RB, bl.off(perm[(size_t)r]), bl.wcnt(perm[(size_t)r], 1));
    for (int x = 0; x < P; x++)
      if (x != r) b.recv(x, RB, bl.off(perm[(size_t)x]), bl.wcnt(perm[(size_t)x], 1));
    b.end();
    return;
  }
  for (int s = steps - 1; s >= 0; s--) {
    const int dest = pi(r, s, P), sb = recv_start(dest, s), rb = recv_start(r, s);
    b.send(dest, RB, bl.off(rb), bl.wcnt(rb, w)); b.recv(dest, RB, bl.off(sb), bl.wcnt(sb, w)); b.end();
    w <<= 1;
  }
}

// the window rank x of P (power of two) owns after the remap reduce-scatter of
// n elements: the halving recurrence of libbine_allreduce.c:866-885 for x
static void remap_owned(int P, int x, uint64_t n, uint64_t *off, uint64_t *cnt) {
  const int steps = log2_ceil(P);
  const uint32_t vx = remap_rank((uint32_t)P, (uint32_t)x);
  uint64_t w = n, o = 0;
  for (int s = 0; s < steps; s++) {
    const uint32_t vd = remap_rank((uint32_t)P, (uint32_t)pi(x, s, P));
    uint64_t rc;
    if (vx < vd) rc = w / 2;  // lower half kept at offset o
    else { rc = w - w / 2; o += w / 2; }
    w = rc;
  }
  *off = o;
  *cnt = w;
}

// allreduce_bine_bdw_remap (:820-923) and allreduce_bine_bdw_remap_segmented
// (:1093-1308; the non-power-of-two fold of :1148-1169 / :1282-1290, the
// segment pipelining becomes the executor's chunked exchange+reduce overlap)
void ar_bine_remap(Builder &b, const PlanArgs &a, bool segmented) {
  const int P = a.P, r = a.rank;
  const uint64_t n = a.count;
  int steps, adj, extra;
  if (!segmented) {
    steps = log2_ceil(P);
    if (!is_pow2(P) || steps == -1) { b.fail(BINE_ERR_ARG); return; }
    adj = P; extra = 0;
  } else {
    steps = floor_log2(P);
    adj = 1 << steps; extra = P - adj;
  }
  const bool pw2 = extra == 0;
  b.tmp(T0, n - n / 2);
  int nr = r;
  bool idle = false, elide = false;
  if (r < 2 * extra) {
    if (r % 2 == 0) { b.send(r + 1, a.in_place ? RB : SB, 0, n); b.end(); idle = true; }
    else {
      nr = r >> 1;
      if (!a.in_place) {
        b.recv(r - 1, RB, 0, n); b.end();
        b.reduce(SB, 0, RB, 0, n);  // :1158 in = sbuf, inout = received
      } else {
        b.tmp(T1, n);
        b.recv(r - 1, T1, 0, n); b.end();
        b.reduce(RB, 0, T1, 0, n);
        b.copy(T1, 0, RB, 0, n);
      }
    }
  } else {
    nr = r - extra;
    if (!a.in_place) {
      if (steps >= 1) elide = true;
      else b.copy(SB, 0, RB, 0, n);
    }
  }
  if (!idle) {
    std::vector<uint64_t> ri(steps + 1), si(steps + 1), rc(steps + 1), sc(steps + 1);
    std::vector<int> dst(steps + 1);
    uint64_t w = n;
    const uint32_t vrank = remap_rank((uint32_t)adj, (uint32_t)nr);
    const bool flat = pw2 && flat_rs_fits(a);
    bool agd = false;  // flat_rs emitted the chunked allgather
    for (int s = 0; s < steps; s++) {
      const int vd = pi(nr, s, adj);
      dst[s] = pw2 ? vd : (vd < extra ? (vd << 1) + 1 : vd + extra);
      const uint32_t vdest = remap_rank((uint32_t)adj, (uint32_t)vd);
      if (vrank < vdest) { rc[s] = w / 2; sc[s] = w - rc[s]; si[s] = ri[s] + rc[s]; }
      else { sc[s] = w / 2; rc[s] = w - sc[s]; ri[s] = si[s] + sc[s]; }
      const bool first = elide && s == 0;
      if (!flat) {
        b.send(dst[s], first ? SB : RB, si[s], sc[s]); b.recv(dst[s], T0, 0, rc[s]); b.end(PIPE);
        if (first) b.reduce3(T0, 0, SB, ri[s], RB, ri[s], rc[s], PIPE);
        else b.reduce(T0, 0, RB, ri[s], rc[s], PIPE);
      }
      if (s + 1 < steps) { ri[s + 1] = ri[s]; si[s + 1] = ri[s]; w = rc[s]; }
    }
    if (flat && steps >= 1) {  // rank x computes the window remap_owned(x)
      std::vector<uint64_t> boff((size_t)P), bcnt((size_t)P);
      for (int x = 0; x < P; x++) remap_owned(P, x, n, &boff[(size_t)x], &bcnt[(size_t)x]);
      const auto leaves = flat_leaves(P, steps, r, [&](int x, int s) { return pi(x, s, P); });
      agd = flat_rs(b, a, a.in_place ? RB : SB, boff, bcnt, leaves, RB, ri[steps - 1], 0, true);
    }
    if (agd) {
    } else if (a.flat_ag && pw2 && steps >= 1) {
      for (int x = 0; x < P; x++)
        if (x != r) b.send(x, RB, ri[steps - 1], rc[steps - 1]);
      for (int x = 0; x < P; x++) {
        if (x == r) continue;
        uint64_t o, c;
        remap_owned(P, x, n, &o, &c);
        b.recv(x, RB, o, c);
      }
      b.end();
    } else {
      for (int s = steps - 1; s >= 0; s--) {
        b.send(dst[s], RB, ri[s], rc[s]); b.recv(dst[s], RB, si[s], sc[s]); b.end();
      }
    }
  }
  if (r < 2 * extra) {
    if (!idle) b.send(r - 1, RB, 0, n); else b.recv(r + 1, RB, 0, n);
    b.end();
  }
}

// allreduce_bine_block_by_block_any_even, :925-1091
void ar_bine_bbb_any_even(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const uint64_t n = a.count;
  if (P % 2) { b.fail(BINE_ERR_ARG); return; }  // assert(size % 2 == 0), :931
  Blocks bl(n, P);
  if (flat_rs_fits(a)) {
    // power-of-two P: rank x ends the reduce-scatter with block x, reduced
    // as acc = acc (op) received with the negabinary partners (the same trees
    // as the block-by-block reduce-scatter's first levels; tests/test_flat_symbolic.py)
    std::vector<uint64_t> boff((size_t)P), bcnt((size_t)P);
    for (int x = 0; x < P; x++) { boff[(size_t)x] = bl.off(x); bcnt[(size_t)x] = bl.cnt(x); }
    if (flat_rs(b, a, a.in_place ? RB : SB, boff, bcnt,
                flat_leaves(P, log2_ceil(P), r, [P](int x, int s) { return nb_partner(x, 1 << s, P); }), RB,
                boff[(size_t)r], 0, true))
      return;
    if (a.flat_ag) {
      for (int x = 0; x < P; x++)
        if (x != r) b.send(x, RB, boff[(size_t)r], bcnt[(size_t)r]);
      for (int x = 0; x < P; x++)
        if (x != r) b.recv(x, RB, boff[(size_t)x], bcnt[(size_t)x]);
      b.end();
      return;
    }
  } else {
    b.tmp(T0, n);
    if (!a.in_place) b.copy(SB, 0, RB, 0, n);
  }
  const bool flat = flat_rs_fits(a);
  int mask = 1, rstep = log2_ceil(P) - 1;
  std::vector<int> kof((size_t)P, -1);
  for (int blk = 1; blk < P; blk++) kof[(size_t)blk] = 31 - __builtin_clz(get_nu((uint32_t)blk, (uint32_t)P));
  while (mask < P) {
    if (flat) { mask <<= 1; rstep--; continue; }
    const int partner = nb_partner(r, mask, P);
    std::vector<int> got;
    for (int blk = 1; blk < P; blk++) {
      if (kof[(size_t)blk] != rstep) continue;
      int bts, brv;
      if (r % 2 == 0) { bts = pmod(blk + r, P); brv = pmod(partner - blk, P); }
      else { bts = pmod(r - blk, P); brv = pmod(blk + partner, P); }
      if (bts != r) b.send(partner, RB, bl.off(bts), bl.cnt(bts));
      if (brv != partner) { b.recv(partner, T0, bl.off(brv), bl.cnt(brv)); got.push_back(brv); }
    }
    b.end();
    for (int blk : got) b.reduce(T0, bl.off(blk), RB, bl.off(blk), bl.cnt(blk));
    mask <<= 1; rstep--;
  }
  int step = 0;
  mask >>= 1;
  while (mask > 0) {
    const int partner = nb_partner(r, mask, P);
    for (int blk = 1; blk < P; blk++) {
      if (kof[(size_t)blk] != step) continue;
      int bts, brv;
      if (r % 2 == 0) { brv = pmod(blk + r, P); bts = pmod(partner - blk, P); }
      else { brv = pmod(r - blk, P); bts = pmod(blk + partner, P); }
      if (bts != partner) b.send(partner, RB, bl.off(bts), bl.cnt(bts));
      if (brv != r) b.recv(partner, RB, bl.off(brv), bl.cnt(brv));
    }
    b.end();
    mask >>= 1; step++;
  }
}

// ---------------------------------------------------------------------------
// reduce_scatter -- libbine_reduce_scatter.c
// ---------------------------------------------------------------------------

struct Displs {
  std::vector<uint64_t> d;
  uint64_t total = 0;
  uint64_t maxc = 0;
  explicit Displs(const std::vector<int> &rc) {
    d.resize(rc.size());
    for (size_t i = 0; i < rc.size(); i++) {
      d[i] = total;
      total += (uint64_t)rc[i];
      maxc = std::max(maxc, (uint64_t)rc[i]);
    }
  }
};

// flat reduce-scatter of the reduce_scatter variants: block y (displacement
// d[y], rc[y] elements) goes to rank y; the result lands in rbuf, through TMP1
// when in place (rbuf's own blocks are still being sent)
void flat_rs_block(Builder &b, const PlanArgs &a, int src, const std::vector<uint64_t> &d, const std::vector<int> &rc,
                   const std::vector<int> &leaves, unsigned swap = 0) {
  std::vector<uint64_t> cnt(rc.size());
  for (size_t i = 0; i < rc.size(); i++) cnt[i] = (uint64_t)rc[i];
  const uint64_t mine = cnt[(size_t)a.rank];
  if (!a.in_place) { flat_rs(b, a, src, d, cnt, leaves, RB, 0, swap); return; }
  b.tmp(T1, mine);
  flat_rs(b, a, src, d, cnt, leaves, T1, 0, swap);
  b.copy(T1, 0, RB, 0, mine);
}

// reduce_scatter_recursivehalving, :15-257
void rs_recursivehalving(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const auto &rc = a.rcounts;
  Displs ds(rc);
  const uint64_t count = ds.total;
  if (!count) return;
  const int src = a.in_place ? RB : SB;
  if (is_pow2(P) && flat_rs_fits(a)) {  // rank r ends with block r; partners r ^ (P >> (s + 1))
    flat_rs_block(b, a, src, ds.d, rc,
                  flat_leaves(P, log2_ceil(P), r, [P](int x, int s) { return x ^ (P >> (s + 1)); }));
    return;
  }
  b.tmp(T0, count); b.tmp(T1, count);  // recv_buf, result_buf
  b.copy(src, 0, T1, 0, count);
  const int tsz = next_pow2(P) >> 1, rem = P - tsz;
  int tr;
  if (r < 2 * rem) {
    if ((r & 1) == 0) { b.send(r + 1, T1, 0, count); b.end(); tr = -1; }
    else { b.recv(r - 1, T0, 0, count); b.end(); b.reduce(T0, 0, T1, 0, count); tr = r / 2; }
  } else tr = r - rem;
  if (tr >= 0) {
    std::vector<uint64_t> trc((size_t)tsz), tds((size_t)tsz);
    for (int i = 0; i < tsz; i++) trc[(size_t)i] = i < rem ? (uint64_t)rc[2 * i + 1] + (uint64_t)rc[2 * i] : (uint64_t)rc[i + rem];
    for (int i = 0; i + 1 < tsz; i++) tds[(size_t)i + 1] = tds[(size_t)i] + trc[(size_t)i];
    int sidx = 0, ridx = 0, last = tsz;
    for (int mask = tsz >> 1; mask > 0; mask >>= 1) {
      int tp = tr ^ mask, peer = tp < rem ? tp * 2 + 1 : tp + rem;
      uint64_t scn = 0, rcn = 0;
      if (tr < tp) {
        sidx = ridx + mask;
        for (int i = sidx; i < last; i++) scn += trc[(size_t)i];
        for (int i = ridx; i < sidx; i++) rcn += trc[(size_t)i];
      } else {
        ridx = sidx + mask;
        for (int i = sidx; i < ridx; i++) scn += trc[(size_t)i];
        for (int i = ridx; i < last; i++) rcn += trc[(size_t)i];
      }
      const bool pipe = scn > 0 && rcn > 0;
      b.recv(peer, T0, tds[(size_t)ridx], rcn); b.send(peer, T1, tds[(size_t)sidx], scn); b.end(pipe);
      b.reduce(T0, tds[(size_t)ridx], T1, tds[(size_t)ridx], rcn, pipe);
      sidx = ridx;
      last = ridx + mask;
    }
    b.copy(T1, ds.d[(size_t)r], RB, 0, (uint64_t)rc[(size_t)r]);
  }
  if (r < 2 * rem) {
    if ((r & 1) == 0) b.recv(r + 1, RB, 0, (uint64_t)rc[(size_t)r]);
    else b.send(r - 1, T1, ds.d[(size_t)r - 1], (uint64_t)rc[(size_t)r - 1]);
    b.end();
  }
}

// reduce_scatter_recursive_distance_doubling, :259-419
void rs_recursive_distance_doubling(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const auto &rc = a.rcounts;
  const int steps = log2_ceil(P);
  if (!is_pow2(P) || steps == -1) { b.fail(BINE_ERR_ARG); return; }
  Displs ds(rc);
  const uint64_t count = ds.total;
  if (!count) return;
  const int src = a.in_place ? RB : SB;
  if (flat_rs_fits(a)) {
    // rank x computes block inverse_rank(x) (bit reversal, an involution) with
    // partners x ^ 2^s and sends it there: rank y evaluates the tree of
    // inverse_rank(y)
    flat_rs_block(b, a, src, ds.d, rc, flat_leaves(P, steps, (int)top_bits((uint32_t)r, steps),
                                                   [](int x, int s) { return x ^ (1 << s); }));
    return;
  }
  b.tmp(T0, count); b.tmp(T1, count);
  b.copy(src, 0, T1, 0, count);
  int w = P >> 1, dist = 1, sidx = 0, ridx = 0, last = P;
  for (int s = 0; s < steps; s++) {
    const int peer = r ^ dist;
    uint64_t scn = 0, rcn = 0;
    if (r < peer) {
      sidx = ridx + w;
      for (int i = sidx; i < last; i++) scn += (uint64_t)rc[(size_t)i];
      for (int i = ridx; i < sidx; i++) rcn += (uint64_t)rc[(size_t)i];
    } else {
      ridx = sidx + w;
      for (int i = sidx; i < ridx; i++) scn += (uint64_t)rc[(size_t)i];
      for (int i = ridx; i < last; i++) rcn += (uint64_t)rc[(size_t)i];
    }
    const bool pipe = scn > 0 && rcn > 0;
    b.recv(peer, T0, ds.d[(size_t)ridx], rcn); b.send(peer, T1, ds.d[(size_t)sidx], scn); b.end(pipe);
    b.reduce(T0, ds.d[(size_t)ridx], T1, ds.d[(size_t)ridx], rcn, pipe);
    sidx = ridx;
    last = ridx + w;
    w >>= 1; dist <<= 1;
  }
  const int inv = (int)top_bits((uint32_t)r, steps);  // inverse_rank(), libbine_utils.h:580-583
  if (inv != r) {
    b.send(inv, T1, ds.d[(size_t)inv], (uint64_t)rc[(size_t)inv]); b.recv(inv, RB, 0, (uint64_t)rc[(size_t)r]); b.end();
  } else b.copy(T1, ds.d[(size_t)r], RB, 0, (uint64_t)rc[(size_t)r]);
}

// reduce_scatter_ring, :421-572
void rs_ring(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const auto &rc = a.rcounts;
  Displs ds(rc);
  const int src = a.in_place ? RB : SB;
  auto cnt = [&](int i) { return (uint64_t)rc[(size_t)i]; };
  if (P == 1) { b.copy(src, 0, RB, 0, ds.total); return; }
  if (flat_rs_fits(a)) {
    // block r starts at rank r + 1 and ends, folded, at rank r: chain
    // r + 1, ..., r + P - 1, r; in place through TMP1 (rbuf's blocks are still sent)
    std::vector<uint64_t> cnt((size_t)P);
    for (int x = 0; x < P; x++) cnt[(size_t)x] = (uint64_t)rc[(size_t)x];
    std::vector<int> order;
    for (int j = 1; j <= P; j++) order.push_back((r + j) % P);
    if (!a.in_place) { flat_chain(b, a, src, ds.d, cnt, order, RB, 0); return; }
    b.tmp(T1, cnt[(size_t)r]);
    flat_chain(b, a, src, ds.d, cnt, order, T1, 0);
    b.copy(T1, 0, RB, 0, cnt[(size_t)r]);
    return;
  }
  b.tmp(T0, ds.total); b.tmp(T1, ds.maxc); b.tmp(T2, ds.maxc);
  const int ib[2] = {T1, T2};
  b.copy(src, 0, T0, 0, ds.total);
  const int to = (r + 1) % P, from = (r + P - 1) % P;
  int inbi = 0;
  b.recv(from, ib[inbi], 0, cnt((r + P - 2) % P)); b.send(to, T0, ds.d[(size_t)from], cnt(from)); b.end();
  for (int k = 2; k < P; k++) {
    const int prev = (r + P - k) % P, incoming = (r + P - k - 1) % P;
    inbi ^= 1;
    b.reduce(ib[inbi ^ 1], 0, T0, ds.d[(size_t)prev], cnt(prev));
    b.recv(from, ib[inbi], 0, cnt(incoming)); b.send(to, T0, ds.d[(size_t)prev], cnt(prev)); b.end();
  }
  b.reduce(ib[inbi], 0, T0, ds.d[(size_t)r], cnt(r));
  b.copy(T0, ds.d[(size_t)r], RB, 0, cnt(r));
}

// sum_counts, libbine_utils.h:404-410
static uint64_t sum_counts(const std::vector<int> &c, const Displs &ds, int rem, int lo, int hi) {
  lo = lo < rem ? lo * 2 : lo + rem;
  hi = hi < rem ? hi * 2 + 1 : hi + rem;
  return ds.d[(size_t)hi] + (uint64_t)c[(size_t)hi] - ds.d[(size_t)lo];
}

static uint32_t mirror(uint32_t x, int nbits) { return top_bits(x, nbits); }  // :418-426

// reduce_scatter_butterfly, :575-761
void rs_butterfly(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const auto &rc = a.rcounts;
  Displs ds(rc);
  const int src = a.in_place ? RB : SB;
  if (P < 2) { b.copy(src, 0, RB, 0, ds.total); return; }  // the reference returns without copying
  const uint64_t total = ds.total;
  if (is_pow2(P) && flat_rs_fits(a)) {
    // partners x ^ 2^s; every combine keeps the higher rank's accumulator as
    // the inout side (:680-690: reduce(own, received) when rank < peer, then
    // the buffers swap); rank x ends with block mirror(x) and swaps it with
    // rank mirror(x), so rank y evaluates the tree of mirror(y)
    const int L = log2_ceil(P);
    flat_rs_block(b, a, src, ds.d, rc,
                  flat_leaves(P, L, (int)mirror((uint32_t)r, L), [](int x, int s) { return x ^ (1 << s); },
                              [](int x, int s) { return x > (x ^ (1 << s)); }));
    return;
  }
  b.tmp(T0, total); b.tmp(T1, total);
  int ps = T0, pr = T1;
  b.copy(src, 0, ps, 0, total);
  const int pof2 = next_pow2(P) >> 1, rem = P - pof2, l2 = log2_ceil(pof2);
  int vr;
  if (r < 2 * rem) {
    if (r % 2 == 0) { b.send(r + 1, ps, 0, total); b.end(); vr = -1; }
    else { b.recv(r - 1, pr, 0, total); b.end(); b.reduce(pr, 0, ps, 0, total); vr = r / 2; }
  } else vr = r - rem;
  if (vr != -1) {
    int nblocks = pof2, si = 0, ri = 0;
    for (int mask = 1; mask < pof2; mask <<= 1) {
      const int vp = vr ^ mask, peer = vp < rem ? vp * 2 + 1 : vp + rem;
      nblocks /= 2;
      if ((vr & mask) == 0) si += nblocks; else ri += nblocks;
      const uint64_t scn = sum_counts(rc, ds, rem, si, si + nblocks - 1);
      int ix = si < rem ? 2 * si : rem + si;
      const uint64_t sd = ds.d[(size_t)ix];
      const uint64_t rcn = sum_counts(rc, ds, rem, ri, ri + nblocks - 1);
      ix = ri < rem ? 2 * ri : rem + ri;
      const uint64_t rd = ds.d[(size_t)ix];
      const bool pipe = scn > 0 && rcn > 0;
      b.send(peer, ps, sd, scn); b.recv(peer, pr, rd, rcn); b.end(pipe);
      if (vr < vp) { b.reduce(ps, rd, pr, rd, rcn, pipe); std::swap(ps, pr); }
      else b.reduce(pr, rd, ps, rd, rcn, pipe);
      si = ri;
    }
    const int vp = (int)mirror((uint32_t)vr, l2), peer = vp < rem ? vp * 2 + 1 : vp + rem;
    int ix = si < rem ? 2 * si : rem + si;
    if (vp < rem) b.send(peer - 1, ps, ds.d[(size_t)ix], (uint64_t)rc[(size_t)ix]);
    if (vp < rem) ix++;
    if (vp != vr) {
      b.send(peer, ps, ds.d[(size_t)ix], (uint64_t)rc[(size_t)ix]); b.recv(peer, RB, 0, (uint64_t)rc[(size_t)r]);
    }
    b.end();
    if (vp == vr) b.copy(ps, ds.d[(size_t)r], RB, 0, (uint64_t)rc[(size_t)r]);
  } else {
    const int vp = (int)mirror((uint32_t)((r + 1) / 2), l2), peer = vp < rem ? vp * 2 + 1 : vp + rem;
    b.recv(peer, RB, 0, (uint64_t)rc[(size_t)r]); b.end();
  }
}

// reduce_scatter_bine_static, :763-904
void rs_bine_static(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const auto &rc = a.rcounts;
  Displs ds(rc);
  const uint64_t count = ds.total;
  if (!count) return;
  const int steps = log2_ceil(P);
  if (!is_pow2(P) || steps < 1) { b.fail(BINE_ERR_SIZE); return; }
  std::vector<int> perm;
  static_perm(P, perm);
  auto recv_start = [&](int rank, int s) { int w = P >> (s + 1); return perm[(size_t)rank] & ~(w - 1); };
  auto run = [&](int start, int w) {
    uint64_t c = 0;
    for (int i = 0; i < w; i++) c += (uint64_t)rc[(size_t)(start + i)];
    return c;
  };
  const int src = a.in_place ? RB : SB;
  if (flat_rs_fits(a)) {  // rank x computes block perm[x] and sends it to rank perm[x]
    int tx = r;
    for (int j = 0; j < P; j++) if (perm[(size_t)j] == r) { tx = j; break; }
    flat_rs_block(b, a, src, ds.d, rc, flat_leaves(P, steps, tx, [&](int x, int s) { return pi(x, s, P); }));
    return;
  }
  b.tmp(T0, count); b.tmp(T1, count);  // recv_buf, result_buf
  b.copy(src, 0, T1, 0, count);
  int w = P >> 1;
  for (int s = 0; s < steps; s++) {
    const int peer = pi(r, s, P), sb = recv_start(peer, s), rb = recv_start(r, s);
    const uint64_t scn = run(sb, w), rcn = run(rb, w);
    const bool pipe = scn > 0 && rcn > 0;
    b.send(peer, T1, ds.d[(size_t)sb], scn); b.recv(peer, T0, ds.d[(size_t)rb], rcn); b.end(pipe);
    b.reduce(T0, ds.d[(size_t)rb], T1, ds.d[(size_t)rb], rcn, pipe);
    w >>= 1;
  }
  const int target = perm[(size_t)r];
  if (target != r) {
    int sender = -1;
    for (int j = 0; j < P; j++) if (perm[(size_t)j] == r) { sender = j; break; }
    b.send(target, T1, ds.d[(size_t)target], (uint64_t)rc[(size_t)target]);
    b.recv(sender, RB, 0, (uint64_t)rc[(size_t)r]);
    b.end();
  } else b.copy(T1, ds.d[(size_t)r], RB, 0, (uint64_t)rc[(size_t)r]);
}

// reduce_scatter_bine_send_remap (:906-983) / _permute_remap (:985-1063)
void rs_bine_remap(Builder &b, const PlanArgs &a, bool permute) {
  const int P = a.P, r = a.rank;
  const auto &rc = a.rcounts;
  if (!is_pow2(P)) { b.fail(BINE_ERR_ARG); return; }  // the reference hangs
  // permute: block i moves into the slot of block remap(i) (:1008-1011) --
  // defined only for equal blocks (the reference overruns its buffers otherwise)
  if (permute)
    for (int x : rc)
      if (x != rc[0]) { b.fail(BINE_ERR_ARG); return; }
  Displs ds(rc);
  const uint64_t count = ds.total;
  const int src = a.in_place ? RB : SB;
  if (flat_rs_fits(a)) {
    // permute: rank x computes block x with tree T(x); send: rank x computes
    // block remap(x) and sends it to rank remap(x), so rank y's block y has
    // the tree of remap^-1(y)
    int tx = r;
    if (!permute)
      for (int j = 0; j < P; j++) if ((int)remap_rank((uint32_t)P, (uint32_t)j) == r) { tx = j; break; }
    const auto leaves = flat_leaves(P, log2_ceil(P), tx, [&](int x, int s) { return nb_partner(x, 1 << s, P); });
    flat_rs_block(b, a, src, ds.d, rc, leaves);
    return;
  }
  b.tmp(T0, count); b.tmp(T1, count + ds.maxc);  // tmpbuf, resbuf
  if (!permute) b.copy(src, 0, T1, 0, count);
  else
    for (int i = 0; i < P; i++)
      b.copy(src, ds.d[(size_t)i], T1, ds.d[remap_rank((uint32_t)P, (uint32_t)i)], (uint64_t)rc[(size_t)i]);
  const int steps = log2_ceil(P);
  const int me = (int)remap_rank((uint32_t)P, (uint32_t)r);
  int mask = 1, inv = steps >= 1 ? 1 << (steps - 1) : 0;
  auto span = [&](int first, int lastb) { return ds.d[(size_t)lastb] - ds.d[(size_t)first] + (uint64_t)rc[(size_t)lastb]; };
  while (mask < P) {
    const int partner = nb_partner(r, mask, P);
    const int bfm = ~(inv - 1);
    const int sbf = (int)remap_rank((uint32_t)P, (uint32_t)partner) & bfm, sbl = sbf + inv - 1;
    const int rbf = me & bfm, rbl = rbf + inv - 1;
    const uint64_t scn = span(sbf, sbl), rcn = span(rbf, rbl);
    const bool pipe = scn > 0 && rcn > 0;
    b.send(partner, T1, ds.d[(size_t)sbf], scn); b.recv(partner, T0, ds.d[(size_t)rbf], rcn); b.end(pipe);
    b.reduce(T0, ds.d[(size_t)rbf], T1, ds.d[(size_t)rbf], rcn, pipe);
    mask <<= 1; inv >>= 1;
  }
  if (!permute) {  // :966-969, the any-source receive resolved to its one sender
    int sender = r;
    for (int j = 0; j < P; j++) if ((int)remap_rank((uint32_t)P, (uint32_t)j) == r) { sender = j; break; }
    b.send(me, T1, ds.d[(size_t)me], (uint64_t)rc[(size_t)me]);
    b.recv(sender, RB, 0, (uint64_t)rc[(size_t)r]);
    b.end();
  } else b.copy(T1, ds.d[(size_t)me], RB, 0, (uint64_t)rc[(size_t)r]);
}

// reduce_scatter_bine_block_by_block, :1066-1174
void rs_bine_bbb(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const auto &rc = a.rcounts;
  if (!is_pow2(P)) { b.fail(BINE_ERR_ARG); return; }  // the reference hangs
  Displs ds(rc);
  const int src = a.in_place ? RB : SB;
  if (P == 1) { b.copy(src, 0, RB, 0, (uint64_t)rc[0]); return; }  // reference: rbuf untouched
  if (flat_rs_fits(a)) {
    // rank r ends with block r; every step reduces received into its own
    // accumulator except the last, reduce(own, received) (:1143): the top
    // level's operands are swapped
    const int L = log2_ceil(P);
    flat_rs_block(b, a, src, ds.d, rc, flat_leaves(P, L, r, [&](int x, int s) { return nb_partner(x, 1 << s, P); }),
                  1u << (L - 1));
    return;
  }
  std::vector<int> invr((size_t)P);
  for (int i = 0; i < P; i++) invr[remap_rank((uint32_t)P, (uint32_t)i)] = i;
  b.tmp(T0, ds.total); b.tmp(T1, ds.total);  // tmpbuf, resbuf
  b.copy(src, 0, T1, 0, ds.total);
  const int steps = log2_ceil(P);
  const int me = (int)remap_rank((uint32_t)P, (uint32_t)r);
  int mask = 1, inv = 1 << (steps - 1);
  while (mask < P) {
    const bool last = (mask << 1) >= P;
    const int partner = nb_partner(r, mask, P);
    const int bfm = ~(inv - 1);
    const int sbf = (int)remap_rank((uint32_t)P, (uint32_t)partner) & bfm, sbl = sbf + inv - 1;
    const int rbf = me & bfm, rbl = rbf + inv - 1;
    for (int blk = rbf; blk <= rbl; blk++) {
      const int o = invr[(size_t)blk];
      b.recv(partner, last ? RB : T0, last ? 0 : ds.d[(size_t)o], (uint64_t)rc[(size_t)o]);
    }
    for (int blk = sbf; blk <= sbl; blk++) {
      const int o = invr[(size_t)blk];
      b.send(partner, T1, ds.d[(size_t)o], (uint64_t)rc[(size_t)o]);
    }
    b.end();
    for (int blk = rbf; blk <= rbl; blk++) {
      const int o = invr[(size_t)blk];
      if (last) b.reduce(T1, ds.d[(size_t)o], RB, 0, (uint64_t)rc[(size_t)o]);  // :1143
      else b.reduce(T0, ds.d[(size_t)o], T1, ds.d[(size_t)o], (uint64_t)rc[(size_t)o]);
    }
    mask <<= 1; inv >>= 1;
  }
}

// reduce_scatter_bine_block_by_block_any_even, :1176-1298
void rs_bine_bbb_any_even(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const auto &rc = a.rcounts;
  Displs ds(rc);
  const int src = a.in_place ? RB : SB;
  if (P == 1) { b.copy(src, 0, RB, 0, (uint64_t)rc[0]); return; }
  if (P % 2) { b.fail(BINE_ERR_ARG); return; }  // the reference hangs for odd P > 1
  if (flat_rs_fits(a)) {
    // power-of-two P: the trees of reduce_scatter_bine_block_by_block (top
    // level swapped: the last step reduces (own, received), :1265)
    const int L = log2_ceil(P);
    flat_rs_block(b, a, src, ds.d, rc, flat_leaves(P, L, r, [P](int x, int s) { return nb_partner(x, 1 << s, P); }),
                  1u << (L - 1));
    return;
  }
  b.tmp(T0, ds.total); b.tmp(T1, ds.total);
  b.copy(src, 0, T1, 0, ds.total);
  std::vector<int> kof((size_t)P, -1);
  for (int blk = 1; blk < P; blk++) kof[(size_t)blk] = 31 - __builtin_clz(get_nu((uint32_t)blk, (uint32_t)P));
  int mask = 1, rstep = log2_ceil(P) - 1;
  bool done = false;
  while (mask < P) {
    const bool last = (mask << 1) >= P;
    const int partner = nb_partner(r, mask, P);
    std::vector<int> got;
    for (int blk = 1; blk < P; blk++) {
      if (kof[(size_t)blk] != rstep) continue;
      int bts, brv;
      if (r % 2 == 0) { bts = pmod(blk + r, P); brv = pmod(partner - blk, P); }
      else { bts = pmod(r - blk, P); brv = pmod(blk + partner, P); }
      if (bts != r) b.send(partner, T1, ds.d[(size_t)bts], (uint64_t)rc[(size_t)bts]);
      if (brv != partner) {
        got.push_back(brv);
        if (last) { b.recv(partner, RB, 0, (uint64_t)rc[(size_t)brv]); done = true; }
        else b.recv(partner, T0, ds.d[(size_t)brv], (uint64_t)rc[(size_t)brv]);
      }
    }
    b.end();
    for (int blk : got) {
      if (last) b.reduce(T1, ds.d[(size_t)blk], RB, 0, (uint64_t)rc[(size_t)blk]);
      else b.reduce(T0, ds.d[(size_t)blk], T1, ds.d[(size_t)blk], (uint64_t)rc[(size_t)blk]);
    }
    mask <<= 1; rstep--;
  }
  if (!done) b.copy(T1, ds.d[(size_t)r], RB, 0, (uint64_t)rc[(size_t)r]);
}

// ---------------------------------------------------------------------------
// reduce -- libbine_reduce.c
// ---------------------------------------------------------------------------

// reduce_bine_lat, :16-80
void rd_bine_lat(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank, root = a.root;
  const uint64_t n = a.count;
  if (n == 0) return;
  if (!is_pow2(P)) { b.fail(BINE_ERR_SIZE); return; }
  const int src = (a.in_place && r == root) ? RB : SB;
  const int acc = r == root ? RB : T1;
  // partner of rank x at step s (mask 2^s) in the negabinary binomial tree
  auto partner_of = [&](int x, int s) {
    const int bx = (int)to_nb(pmod(x - root, P));
    return pmod(from_nb((uint32_t)(bx ^ ((2 << s) - 1))) + root, P);
  };
  if (flat_rs_fits(a)) {
    // every subtree root that sends at step s has received at every step
    // before (binomial tree), so the root's result is the tree T(root) of the
    // flat reduce-scatter with these partners: every rank sends its whole
    // vector straight to the root (one hop each) and the root evaluates it
    std::vector<uint64_t> boff((size_t)P, 0), bcnt((size_t)P, 0);
    bcnt[(size_t)root] = n;
    flat_rs(b, a, src, boff, bcnt, flat_leaves(P, log2_ceil(P), root, partner_of), RB, 0);
    return;
  }
  b.tmp(T0, n);
  if (r != root) b.tmp(T1, n);
  b.copy(src, 0, acc, 0, n);
  const int vrank = pmod(r - root, P);
  const int bv = (int)to_nb(vrank);
  for (int mask = 1; mask < P; mask <<= 1) {
    const int partner = pmod(from_nb((uint32_t)(bv ^ ((mask << 1) - 1))) + root, P);
    const int ml = (mask << 2) - 1, lsbs = bv & ml;
    const bool eq = lsbs == 0 || lsbs == ml;
    if (!eq || ((mask << 1) >= P && r != root)) { b.send(partner, acc, 0, n); b.end(); break; }
    b.recv(partner, T0, 0, n); b.end(PIPE);
    b.reduce(T0, 0, acc, 0, n, PIPE);
  }
}

// reduce_bine_bdw, :83-222
void rd_bine_bdw(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const uint64_t n = a.count;
  if (a.root != 0) { b.fail(BINE_ERR_ARG); return; }  // assert(root == 0), :86
  if (!is_pow2(P)) { b.fail(BINE_ERR_SIZE); return; }
  const int steps = log2_ceil(P);
  const uint64_t cpr = n / (uint64_t)P;
  const int rem = (int)(n % (uint64_t)P);
  const int src = (a.in_place && r == 0) ? RB : SB;
  const int res = r == 0 ? RB : T1;
  const bool flat = flat_rs_fits(a);
  b.tmp(T0, n);
  if (r != 0) b.tmp(T1, n);
  if (!flat) b.copy(src, 0, res, 0, n);
  const int me = (int)remap_rank((uint32_t)P, (uint32_t)r);
  std::vector<uint64_t> ri(steps + 1), si(steps + 1), rc(steps + 1), sc(steps + 1);
  auto first = [&](int blk) { return cpr * (uint64_t)blk + (uint64_t)std::min(blk, rem); };
  auto span = [&](int f, int l) {
    return cpr * (uint64_t)(l - f + 1) + (uint64_t)(std::min(l, rem) - std::min(f, rem)) + (l < rem ? 1u : 0u);
  };
  int mask = 1, inv = steps >= 1 ? 1 << (steps - 1) : 0, step = 0;
  while (mask < P) {
    const int partner = nb_partner(r, mask, P);
    const int bfm = ~(inv - 1);
    const int sbf = (int)remap_rank((uint32_t)P, (uint32_t)partner) & bfm, sbl = sbf + inv - 1;
    const int rbf = me & bfm, rbl = rbf + inv - 1;
    si[step] = first(sbf); sc[step] = span(sbf, sbl);
    ri[step] = first(rbf); rc[step] = span(rbf, rbl);
    const bool pipe = sc[step] > 0 && rc[step] > 0;
    if (!flat) {
      b.send(partner, res, si[step], sc[step]); b.recv(partner, T0, ri[step], rc[step]); b.end(pipe);
      b.reduce(T0, ri[step], res, ri[step], rc[step], pipe);
    }
    mask <<= 1; inv >>= 1; step++;
  }
  if (flat && steps >= 1) {  // rank x computes block remap(x)
    std::vector<uint64_t> boff((size_t)P), bcnt((size_t)P);
    for (int x = 0; x < P; x++) {
      const int mx = (int)remap_rank((uint32_t)P, (uint32_t)x);
      boff[(size_t)x] = first(mx); bcnt[(size_t)x] = span(mx, mx);
    }
    const auto leaves = flat_leaves(P, steps, r, [&](int x, int s) { return nb_partner(x, 1 << s, P); });
    flat_rs(b, a, src, boff, bcnt, leaves, res, boff[(size_t)r]);
  }
  if (a.flat_ag && steps >= 1) {
    // flat gather: every rank sends its reduced block straight to the root
    // (pure data movement, same bytes as the binomial gather of :167-199)
    if (r != 0) {
      b.send(0, res, first(me), span(me, me));
    } else {
      for (int x = 1; x < P; x++) {
        const int mx = (int)remap_rank((uint32_t)P, (uint32_t)x);
        b.recv(x, res, first(mx), span(mx, mx));
      }
    }
    b.end();
    return;
  }
  mask >>= 1;
  inv = 1;
  step = steps - 1;
  const unsigned recvmask = me ? 1u << (__builtin_ffs(me) - 1) : 0x80000000u;  // :172 (1 << -1 on x86)
  while (mask > 0) {
    const int partner = nb_partner(r, mask, P);
    if ((unsigned)inv & recvmask) { b.send(partner, res, ri[step], rc[step]); b.end(); break; }
    b.recv(partner, res, si[step], sc[step]); b.end();
    mask >>= 1; inv <<= 1; step--;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// allgather -- libbine_allgather.c (pure data movement)
// ---------------------------------------------------------------------------
// count = elements per rank; rbuf holds P blocks of `count`.  Every variant
// writes each block straight to its final place: the permute variants' closing
// reorder_blocks (:628, :797) is folded into the placement of every message
// (a message of consecutive blocks of the reference's layout becomes one run
// per maximal stretch that stays consecutive in the final layout; both ends
// split identically because they see the same block numbers).

namespace {

// messages of one exchange, as (peer, first block, blocks), merged where the
// next message continues the previous one on the same peer
struct Msgs {
  struct M { int peer; int blk; int n; };
  std::vector<M> s, r;
  static void add(std::vector<M> &v, int peer, int blk, int n) {
    if (n <= 0 || peer < 0) return;
    if (!v.empty() && v.back().peer == peer && v.back().blk + v.back().n == blk) { v.back().n += n; return; }
    v.push_back({peer, blk, n});
  }
  void send(int peer, int blk, int n) { add(s, peer, blk, n); }
  void recv(int peer, int blk, int n) { add(r, peer, blk, n); }
  // blocks [blk, blk + n) of a ring of P blocks (wrapping past P)
  void send_wrap(int peer, int blk, int n, int P) {
    const int a = std::min(n, P - blk);
    send(peer, blk, a);
    send(peer, 0, n - a);
  }
  void recv_wrap(int peer, int blk, int n, int P) {
    const int a = std::min(n, P - blk);
    recv(peer, blk, a);
    recv(peer, 0, n - a);
  }
  // blocks [lo, lo + n) of a layout whose block j sits at final block pos[j]
  void send_mapped(int peer, int lo, int n, const std::vector<int> &pos) {
    for (int j = lo; j < lo + n; j++) send(peer, pos[(size_t)j], 1);
  }
  void recv_mapped(int peer, int lo, int n, const std::vector<int> &pos) {
    for (int j = lo; j < lo + n; j++) recv(peer, pos[(size_t)j], 1);
  }
  void flush(Builder &b, uint64_t count) {
    for (auto &m : s) b.send(m.peer, RB, (uint64_t)m.blk * count, (uint64_t)m.n * count);
    for (auto &m : r) b.recv(m.peer, RB, (uint64_t)m.blk * count, (uint64_t)m.n * count);
    b.end();
    s.clear();
    r.clear();
  }
};

// own block into place (COPY_BUFF_DIFF_DT of sbuf)
void ag_own(Builder &b, const PlanArgs &a, int blk) {
  if (!a.in_place) b.copy(SB, 0, RB, (uint64_t)blk * a.count, a.count);
}

}  // namespace

// allgather_recursivedoubling, :18-86 (non-power-of-two: the reference returns
// MPI_SUCCESS without doing anything, :31-34 -- reported as an error here)
void ag_recursivedoubling(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  if (!is_pow2(P)) { b.fail(BINE_ERR_ARG); return; }
  ag_own(b, a, r);
  Msgs m;
  int sbl = r;
  for (int d = 1; d < P; d <<= 1) {
    const int remote = r ^ d;
    m.send(remote, sbl, d);
    if (r < remote) m.recv(remote, sbl + d, d);
    else { m.recv(remote, sbl - d, d); sbl -= d; }
    m.flush(b, a.count);
  }
}

// allgather_k_bruck, radix 2, :88-211.  The reference gathers into a rotated
// layout (block i = rank r+i) and rotates at the end (:185-196); here block i of
// that layout is written at its final place (r+i) mod P from the start.
void ag_k_bruck(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  ag_own(b, a, r);  // in place: the reference moves rbuf[r] to rotated slot 0 = final slot r
  Msgs m;
  for (int d = 1; d < P; d *= 2) {
    const int rc = d <= P / 2 ? d : std::min(d, P - d);
    m.recv_wrap((r + d) % P, (r + d) % P, rc, P);
    m.send_wrap((r - d + P) % P, r, rc, P);
    m.flush(b, a.count);
  }
}

// allgather_ring, :213-270
void ag_ring(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  ag_own(b, a, r);
  Msgs m;
  for (int i = 0; i < P - 1; i++) {
    m.send((r + 1) % P, (r - i + P) % P, 1);
    m.recv((r - 1 + P) % P, (r - i - 1 + P) % P, 1);
    m.flush(b, a.count);
  }
}

// allgather_sparbit, :327-408 (one message per block, in transfer order)
void ag_sparbit(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  ag_own(b, a, r);
  const int L = log2_ceil(P);
  uint32_t d = L >= 1 ? 1u << (L - 1) : 0;
  const uint32_t last_ignore = (uint32_t)__builtin_ctz((unsigned)P);
  const uint32_t ignore = (~((uint32_t)P >> last_ignore) | 1u) << last_ignore;
  int expected = 1;
  Msgs m;
  for (int i = 0; i < L; i++) {
    const int excl = (d & ignore) == d;
    const int to = (r + (int)d) % P, from = (r - (int)d + P) % P;
    for (int t = 0; t < expected - excl; t++) {
      m.s.push_back({to, (r - 2 * t * (int)d + P) % P, 1});        // no merging: one
      m.r.push_back({from, (r - (2 * t + 1) * (int)d + P) % P, 1});  // message per tag
    }
    m.flush(b, a.count);
    d >>= 1;
    expected = (expected << 1) - excl;
  }
}

// get_indexes, libbine_utils.h:142-161
static void tree_blocks(int rank, int step, int n, int P, std::vector<char> &bm) {
  for (int s = step; s < n; s++) {
    const int p = pi(rank, s, P);
    bm[(size_t)p] = 1;
    tree_blocks(p, s + 1, n, P, bm);
  }
}

// allgather_bine_block_by_block, :410-490
void ag_bine_bbb(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank, steps = log2_ceil(P);
  if (!is_pow2(P) || steps < 1) { b.fail(BINE_ERR_ARG); return; }
  ag_own(b, a, r);
  Msgs m;
  std::vector<char> sb((size_t)P), rb((size_t)P);
  for (int step = steps - 1; step >= 0; step--) {
    const int remote = pi(r, step, P);
    std::fill(sb.begin(), sb.end(), 0);
    std::fill(rb.begin(), rb.end(), 0);
    rb[(size_t)pi(r, step, P)] = 1;
    tree_blocks(pi(r, step, P), step + 1, steps, P, rb);
    sb[(size_t)pi(remote, step, P)] = 1;
    tree_blocks(pi(remote, step, P), step + 1, steps, P, sb);
    for (int blk = 0; blk < P; blk++) {
      if (sb[(size_t)blk]) m.send(remote, blk, 1);
      if (rb[(size_t)blk]) m.recv(remote, blk, 1);
    }
    m.flush(b, a.count);
  }
}

// allgather_bine_block_by_block_any_even, :492-561 (memcpy from sbuf even
// in place -> in place is an error here; odd P, P = 1 included, hangs or
// crashes in the reference -> error)
void ag_bine_bbb_any_even(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  if (a.in_place || P % 2) { b.fail(BINE_ERR_ARG); return; }
  ag_own(b, a, r);
  int inv = (int)(1u << ((unsigned)(log2_ceil(P) - 1) & 31u)), step = 0;
  Msgs m;
  while (inv > 0) {
    const int partner = nb_partner(r, inv, P);
    for (int blk = 1; blk < P; blk++) {
      const int k = 31 - __builtin_clz(get_nu((uint32_t)blk, (uint32_t)P));
      if (k != step) continue;
      int btr, bts;
      if (r % 2 == 0) { btr = pmod(blk + r, P); bts = pmod(partner - blk, P); }
      else { btr = pmod(r - blk, P); bts = pmod(blk + partner, P); }
      if (bts != partner) m.send(partner, bts, 1);
      if (btr != r) m.recv(partner, btr, 1);
    }
    m.flush(b, a.count);
    inv >>= 1;
    step++;
  }
}

// allgather_bine_permute_static (:563-640) and _send_static (:642-723).  Static
// tables: recv[r][s] = perm[r] & ~(w-1), send[r][s] = recv[pi(r,s)][s], w = P >> (s+1).
void ag_bine_static(Builder &b, const PlanArgs &a, bool permute) {
  const int P = a.P, r = a.rank, steps = log2_ceil(P);
  if (!is_pow2(P) || steps < 1 || steps > 8) { b.fail(BINE_ERR_ARG); return; }
  if (!permute && a.in_place) { b.fail(BINE_ERR_ARG); return; }  // Sendrecv from MPI_IN_PLACE
  std::vector<int> perm, pos((size_t)P);
  static_perm(P, perm);
  // permute: the reference's block j ends up at final block perm^-1(j); send
  // variant: its layout is already final
  for (int j = 0; j < P; j++) pos[(size_t)(permute ? perm[(size_t)j] : j)] = j;
  auto recv_start = [&](int rank, int s) { const int w = P >> (s + 1); return perm[(size_t)rank] & ~(w - 1); };
  if (permute) {
    if (a.in_place) b.copy(RB, (uint64_t)perm[(size_t)r] * a.count, RB, (uint64_t)r * a.count, a.count);
    else ag_own(b, a, r);
  } else {
    int to = 0;
    for (int j = 0; j < P; j++)
      if (perm[(size_t)j] == r) to = j;
    b.send(to, SB, 0, a.count);
    b.recv(perm[(size_t)r], RB, (uint64_t)perm[(size_t)r] * a.count, a.count);
    b.end();
  }
  Msgs m;
  int w = 1;
  for (int step = steps - 1; step >= 0; step--) {
    const int remote = pi(r, step, P);
    m.send_mapped(remote, recv_start(r, step), w, pos);
    m.recv_mapped(remote, recv_start(remote, step), w, pos);
    m.flush(b, a.count);
    w *= 2;
  }
}

// allgather_bine_permute_remap (:725-809) and _send_remap (:811-890)
void ag_bine_remap(Builder &b, const PlanArgs &a, bool permute) {
  const int P = a.P, r = a.rank, steps = log2_ceil(P);
  if (!is_pow2(P) || steps < 1 || steps > 8) { b.fail(BINE_ERR_ARG); return; }
  if (!permute && a.in_place) { b.fail(BINE_ERR_ARG); return; }
  std::vector<int> remap((size_t)P), pos((size_t)P);
  for (int j = 0; j < P; j++) remap[(size_t)j] = (int)remap_rank((uint32_t)P, (uint32_t)j);
  for (int j = 0; j < P; j++) pos[(size_t)(permute ? remap[(size_t)j] : j)] = j;
  const int vr = remap[(size_t)r];
  if (permute) {
    if (a.in_place) b.copy(RB, (uint64_t)vr * a.count, RB, (uint64_t)r * a.count, a.count);
    else ag_own(b, a, r);
  } else {
    int to = 0;  // get_sender_rec: the rank whose remap is r
    for (int j = 0; j < P; j++)
      if (remap[(size_t)j] == r) to = j;
    b.send(to, SB, 0, a.count);
    b.recv(vr, RB, (uint64_t)vr * a.count, a.count);
    b.end();
  }
  Msgs m;
  int d = 1, sbl = vr;
  for (int step = steps - 1; step >= 0; step--) {
    const int remote = pi(r, step, P), vrem = remap[(size_t)remote];
    m.send_mapped(remote, sbl, d, pos);
    if (vr < vrem) m.recv_mapped(remote, sbl + d, d, pos);
    else { m.recv_mapped(remote, sbl - d, d, pos); sbl -= d; }
    m.flush(b, a.count);
    d <<= 1;
  }
}

// allgather_bine_2_blocks (:892-997; wrap-around part as its own message,
// posted first at both ends) and _2_blocks_dtype (:999-1106; the same bytes
// packed by MPI_Type_indexed -- wrapped head, then main run)
void ag_bine_2_blocks(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank, steps = log2_ceil(P);
  if (!is_pow2(P) || steps < 1) { b.fail(BINE_ERR_ARG); return; }
  ag_own(b, a, r);
  Msgs m;
  int mask = 1, first = r;
  for (int step = 0; step < steps; step++) {
    const int remote = pi(r, step, P), si = first;
    int ri;
    if ((step & 1) == (r & 1)) ri = (si + mask + P) % P;
    else { ri = (si - mask + P) % P; first = ri; }
    const int xr = ri + mask > P ? ri + mask - P : 0, xs = si + mask > P ? si + mask - P : 0;
    m.s.push_back({remote, 0, xs});
    m.r.push_back({remote, 0, xr});
    m.s.push_back({remote, si, mask - xs});
    m.r.push_back({remote, ri, mask - xr});
    m.flush(b, a.count);
    mask <<= 1;
  }
}

// ---------------------------------------------------------------------------
// bcast, libbine_bcast.c: the latency trees.  Whole-buffer messages in RB
// (in place); a rank receives once and then sends at every later step.
// ---------------------------------------------------------------------------

// bcast_bine_lat (:189-279) and _reversed (:281-371): root 0, power-of-two P;
// the step at which each rank receives is found by replaying the tree from
// the root (:221-234), step s of the reversed variant uses pi(., steps-1-s)
void bc_bine_lat(Builder &b, const PlanArgs &a, bool reversed) {
  const int P = a.P, r = a.rank, steps = log2_ceil(P);
  if (!is_pow2(P)) { b.fail(BINE_ERR_SIZE); return; }
  if (a.root != 0) { b.fail(BINE_ERR_ROOT); return; }
  auto peer = [&](int x, int s) { return pi(x, reversed ? steps - s - 1 : s, P); };
  std::vector<char> got((size_t)P);
  got[0] = 1;
  int recv_step = -1;
  for (int s = 0; s < steps && !got[(size_t)r]; s++)
    for (int x = 0; x < P; x++) {
      if (!got[(size_t)x]) continue;
      const int d = peer(x, s);
      got[(size_t)d] = 1;
      if (d == r) { recv_step = s; break; }
    }
  for (int s = 0; s < steps; s++) {
    if (r != 0 && recv_step == s) b.recv(peer(r, s), RB, 0, a.count);
    else if (recv_step < s) b.send(peer(r, s), RB, 0, a.count);
    b.end();
  }
}

// bcast_bine_lat_new (:373-406) and _i_new (:408-452, the same messages with
// non-blocking sends): any root, power-of-two P; negabinary partner per step
void bc_bine_lat_new(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank, steps = log2_ceil(P);
  if (!is_pow2(P)) { b.fail(BINE_ERR_SIZE); return; }
  if (a.root < 0 || a.root >= P) { b.fail(BINE_ERR_ROOT); return; }
  const uint32_t nbm = 0xAAAAAAAAu;
  const int vrank = pmod(r - a.root, P);
  const uint32_t nb = ((uint32_t)vrank + nbm) ^ nbm;  // binary_to_negabinary, libbine_utils.h:509
  bool have = r == a.root;
  for (int mask = steps ? 1 << (steps - 1) : 0; mask > 0; mask >>= 1) {
    const uint32_t lo = ((uint32_t)mask << 1) - 1;
    const int partner = pmod((int32_t)(((nb ^ lo) ^ nbm) - nbm) + a.root, P);  // negabinary_to_binary
    const uint32_t lsbs = nb & lo;
    if (have) b.send(partner, RB, 0, a.count);
    else if (lsbs == 0 || lsbs == lo) { b.recv(partner, RB, 0, a.count); have = true; }
    b.end();
  }
}

// ---------------------------------------------------------------------------
// bcast, libbine_bcast.c: the bandwidth algorithms -- a scatter of the
// root's buffer, then an allgather of the pieces.  In place in RB.
// ---------------------------------------------------------------------------

// bcast_scatter_allgather (:42-187): binomial-tree scatter of blocks of
// sc = ceil(count / P) (vrank v's subtree gets blocks [v, v + lowbit(v))),
// recursive-doubling allgather, and for a non-power-of-two P the forwarding
// of an incomplete partner group's data by recursive halving (:149-169).
// Every count is the size of the data it names, clamped to the buffer: the
// reference computes them in size_t and its counts wrap when a block starts
// past the buffer's end (e.g. count 9 at P = 8), where it then reads past
// the buffer and crashes; here those blocks are empty and the broadcast
// completes (tests/test_bcast.py: every such case delivers the root's
// buffer).
void bc_scatter_allgather(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  if (P < 2) return;
  if (a.count < (uint64_t)P) { b.fail(BINE_ERR_COUNT); return; }
  const uint64_t count = a.count, sc = (count + P - 1) / P;
  const int v = pmod(r - a.root, P);
  auto real = [&](int x) { return pmod(x + a.root, P); };
  // the data of blocks [lo, lo + w) (vranks), clamped to the buffer
  auto span = [&](int64_t lo, int64_t w) -> uint64_t {
    const uint64_t s = std::min<uint64_t>(count, (uint64_t)lo * sc), e = std::min<uint64_t>(count, (uint64_t)(lo + w) * sc);
    return e > s ? e - s : 0;
  };
  int top = 1;
  while (top < P) top <<= 1;
  const int low = v ? (v & -v) : top;  // the scatter's receive step (the root: none)
  if (v) {  // :73-91
    b.recv(real(v - low), RB, (uint64_t)v * sc, span(v, low));
    b.end();
  }
  for (int m = low >> 1; m > 0; m >>= 1)  // :93-106, one blocking send per child
    if (v + m < P) {
      b.send(real(v + m), RB, (uint64_t)(v + m) * sc, span(v + m, m));
      b.end();
    }
  for (int m = 1; m < P; m <<= 1) {  // :117-171
    const int w = v ^ m;
    const int64_t vtr = v / m * m, wtr = (int64_t)w / m * m;
    if (w < P) {
      b.send(real(w), RB, (uint64_t)vtr * sc, span(vtr, m));
      b.recv(real(w), RB, (uint64_t)wtr * sc, span(wtr, m));
      b.end();
    }
    if (wtr + m > P) {
      const int64_t nad = P - vtr - m;
      const uint64_t off = sc * (uint64_t)(vtr + m), fw = span(vtr + m, m);
      for (int rh = m >> 1; rh > 0; rh >>= 1) {
        const int x = v ^ rh;
        const int64_t tr = v / (rh << 1) * (rh << 1);
        if (x > v && v < tr + nad && x >= tr + nad) {
          b.send(real(x), RB, off, fw);
          b.end();
        } else if (x < v && x < tr + nad && v >= tr + nad) {
          b.recv(real(x), RB, off, fw);
          b.end();
        }
      }
    }
  }
}

// bcast_bine_bdw_static (:462-647): the static tables' windows (libbine_utils_
// bitmaps.c, regenerated by static_perm) of w = P >> (s + 1) blocks of the
// COLL_BASE_COMPUTE_BLOCKCOUNT split; a rank receives its window at the step
// the root's pi-tree reaches it (:519-530, replayed in the reference's own
// order) and then forwards at every later step; the allgather mirrors it
void bc_bine_bdw_static(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank, steps = log2_ceil(P);
  if (P < 2) return;
  if (a.count < (uint64_t)P) { b.fail(BINE_ERR_COUNT); return; }
  if (!is_pow2(P)) { b.fail(BINE_ERR_SIZE); return; }
  if (a.root != 0) { b.fail(BINE_ERR_ROOT); return; }
  std::vector<char> got((size_t)P);
  got[0] = 1;
  int recv_step = -1;
  for (int s = 0; s < steps && !got[(size_t)r]; s++)
    for (int x = 0; x < P; x++) {
      if (!got[(size_t)x]) continue;
      const int d = pi(x, s, P);
      got[(size_t)d] = 1;
      if (d == r) { recv_step = s; break; }
    }
  std::vector<int> perm;
  static_perm(P, perm);
  auto rtab = [&](int x, int s) { const int w = P >> (s + 1); return perm[(size_t)x] & ~(w - 1); };
  auto stab = [&](int x, int s) { return rtab(pi(x, s, P), s); };
  const uint64_t small = a.count / P, split = a.count % P, big = small + (split ? 1 : 0);
  auto cnt = [&](int blk, int w) -> uint64_t {
    const uint64_t bb = (uint64_t)blk, ww = (uint64_t)w;
    return bb + ww <= split ? ww * big : bb >= split ? ww * small : ww * small + (split - bb);
  };
  auto off = [&](int blk) -> uint64_t { const uint64_t bb = (uint64_t)blk; return bb <= split ? bb * big : bb * small + split; };
  int w = P >> 1;
  for (int s = 0; s < steps; s++, w >>= 1) {  // :556-587
    if (r != 0 && recv_step == s) { b.recv(pi(r, s, P), RB, off(rtab(r, s)), cnt(rtab(r, s), w)); b.end(); }
    if (recv_step < s) { b.send(pi(r, s, P), RB, off(stab(r, s)), cnt(stab(r, s), w)); b.end(); }
  }
  w = 1;
  for (int s = steps - 1; s >= 0; s--, w <<= 1) {  // :606-632
    const int d = pi(r, s, P);
    if (recv_step != s) b.send(d, RB, off(rtab(r, s)), cnt(rtab(r, s), w));
    if (!(recv_step < s)) b.recv(d, RB, off(stab(r, s)), cnt(stab(r, s), w));
    b.end();
  }
}

// bcast_bine_bdw_remap (:649-760): blocks in remapped (negabinary) order of
// the count / P split with the remainder spread over the first blocks; the
// partner at mask m is rank +- negabinary_to_binary(2m - 1); a rank receives
// once, at the step given by the lowest set bit of its remapped rank, then
// sends; the allgather mirrors it.  Root 0 and power-of-two P only (the
// reference asserts root == 0 and is undefined elsewhere): BINE_ERR_ARG.
void bc_bine_bdw_remap(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank, steps = log2_ceil(P);
  if (P < 2) return;
  if (!is_pow2(P) || a.root != 0) { b.fail(BINE_ERR_ARG); return; }
  const uint64_t per = a.count / P, rem = a.count % P;
  auto displ = [&](int i) { return per * (uint64_t)i + std::min<uint64_t>((uint64_t)i, rem); };
  auto rc = [&](int i) { return per + ((uint64_t)i < rem ? 1 : 0); };
  auto run = [&](int first, int last) { return displ(last) - displ(first) + rc(last); };
  const int rr = (int)remap_rank((uint32_t)P, (uint32_t)r);
  auto partner = [&](int mask) {
    const int d = (int32_t)((((uint32_t)(mask << 1) - 1) ^ 0xAAAAAAAAu) - 0xAAAAAAAAu);  // negabinary_to_binary
    return r % 2 == 0 ? pmod(r + d, P) : pmod(r - d, P);
  };
  int inv = 1 << (steps - 1);
  uint32_t bfm = ~(uint32_t)(inv - 1);  // (unsigned: the mask's shifts below are well defined; remaps are < P)
  const int recv_mask = r == 0 ? inv << 1 : (rr & -rr);
  bool recvd = r == 0;
  int mask = 1;
  for (; mask < P; mask <<= 1, inv >>= 1, bfm >>= 1) {  // :689-716
    const int pt = partner(mask);
    if (recvd) {
      const int sf = (int)(remap_rank((uint32_t)P, (uint32_t)pt) & bfm);
      b.send(pt, RB, displ(sf), run(sf, sf + inv - 1));
      b.end();
    } else if (inv == recv_mask || pt == 0) {
      const int rf = (int)((uint32_t)rr & bfm);
      b.recv(pt, RB, displ(rf), run(rf, rf + inv - 1));
      b.end();
      recvd = true;
    }
  }
  mask >>= 1;
  inv = 1;
  bfm = ~0u;
  for (; mask > 0; mask >>= 1, inv <<= 1, bfm <<= 1) {  // :719-751
    const int pt = partner(mask);
    if (inv != recv_mask) {
      const int sf = (int)((uint32_t)rr & bfm);
      b.send(pt, RB, displ(sf), run(sf, sf + inv - 1));
    }
    if (inv >= recv_mask) {
      const int rf = (int)(remap_rank((uint32_t)P, (uint32_t)pt) & bfm);
      b.recv(pt, RB, displ(rf), run(rf, rf + inv - 1));
    }
    b.end();
  }
}

// ---------------------------------------------------------------------------
// gather_bine / scatter_bine / alltoall_bine (libbine_gather.c, _scatter.c,
// _alltoall.c): whole-block data movement.  No rank's program depends on the
// data it receives, so the planner writes EVERY rank's program in block units
// (a block = `count` elements), matches their messages per ordered pair in
// posting order, runs them on block tags under rendezvous semantics --
// checking bounds, message lengths (a longer message than its receive is
// MPI_ERR_TRUNCATE), progress, and that every block lands where the
// collective puts it -- and emits its own rank's program scaled by `count`,
// each receive carrying its send's exact length.  Where the reference hangs,
// aborts, reads or writes out of bounds or delivers something other than the
// collective (non-power-of-two P; odd roots, and some even ones for scatter:
// tests/golden pins which), the plan is refused -- BINE_ERR_ROOT at a
// power-of-two P, BINE_ERR_SIZE otherwise -- instead of reproducing it.
// ---------------------------------------------------------------------------
namespace {

enum { BS = 0, BR = 1, BT = 2 };  // sbuf, rbuf, the reference's malloc'd temporary

struct BOp {
  int kind;             // 0 copy, 1 send, 2 recv
  int grp;              // send / recv: one blocking MPI call (Sendrecv: both) = one exchange
  int peer;
  int buf;              // send: source; recv / copy: destination
  int64_t off, n;
  int sbuf;             // copy source
  int64_t soff;
};

struct BProg {
  std::vector<BOp> ops;
  int64_t size[3] = {0, 0, 0};  // blocks each buffer holds
  bool crash = false;           // the reference aborts or dereferences NULL
  int ngrp = 0;
  void copy(int sb, int64_t so, int db, int64_t d, int64_t n) { ops.push_back({0, -1, -1, db, d, n, sb, so}); }
  void send(int peer, int b, int64_t off, int64_t n) { ops.push_back({1, ngrp, peer, b, off, n, -1, 0}); }
  void recv(int peer, int b, int64_t off, int64_t n) { ops.push_back({2, ngrp, peer, b, off, n, -1, 0}); }
  void end() { ngrp++; }
};

int64_t pmod64(int64_t a, int64_t b) { int64_t r = a % b; return r < 0 ? r + b : r; }
int nb_partner_root(uint32_t vnb, int mask, int root, int P) {  // e.g. libbine_gather.c:39-40
  return pmod(from_nb(vnb ^ (uint32_t)((mask << 1) - 1)) + root, P);
}

// gather_bine, libbine_gather.c:16-96
void ga_prog(int P, int root, int x, BProg &p) {
  const int G = x == root ? BR : BT;  // non-roots gather into a P-block temporary (:23-26)
  p.size[BS] = 1;
  p.size[G] = P;
  p.copy(BS, 0, G, x, 1);  // :28
  int64_t lo = x, hi = x;
  const uint32_t vnb = to_nb(pmod(x - root, P));
  int ext = x % 2 ? -1 : 1;  // the REAL rank's parity (:33-36)
  for (int mask = 1; mask < P; mask <<= 1) {
    const int partner = nb_partner_root(vnb, mask, root, P);
    const uint32_t mlsb = (uint32_t)(mask << 2) - 1, lsbs = vnb & mlsb;
    if (!(lsbs == 0 || lsbs == mlsb) || ((mask << 1) >= P && x != root)) {  // :45-57
      if (hi >= lo) { p.send(partner, G, lo, hi - lo + 1); p.end(); }  // one blocking call each
      else { p.send(partner, G, lo, P - lo); p.end(); p.send(partner, G, 0, hi + 1); p.end(); }
      return;
    }
    int64_t rs, re;  // :59-69
    if (ext == 1) { rs = (hi + 1) % P; re = (hi + mask) % P; hi = re; }
    else { re = pmod64(lo - 1, P); rs = pmod64(lo - mask, P); lo = rs; }
    if (re >= rs) { p.recv(partner, G, rs, re - rs + 1); p.end(); }  // :70-80, one blocking
    else { p.recv(partner, G, rs, P - rs); p.end(); p.recv(partner, G, 0, re + 1); p.end(); }  // call each
    ext = -ext;
  }
}

// scatter_bine, libbine_scatter.c:14-151
void sc_prog(int P, int root, int x, BProg &p) {
  p.size[BS] = x == root ? P : 0;
  p.size[BR] = 1;
  if (P == 1) { p.copy(BS, 0, BR, 0, 1); return; }  // the reference shifts by -1 here (:57)
  const int L = log2_ceil(P);
  int hd = x % 2 ? -1 : 1;
  if (L % 2 == 0) hd = -hd;  // :38-40
  const uint32_t full = (1u << L) - 1;
  int64_t maxr, minr;  // :49-55
  if (x % 2 == 0) { maxr = ((uint32_t)x + 0x55555555u) & full; minr = ((uint32_t)x - 0xAAAAAAAAu) & full; }
  else { minr = ((uint32_t)x - 0x55555555u) & full; maxr = ((uint32_t)x + 0xAAAAAAAAu) & full; }
  maxr %= P;
  minr %= P;
  int64_t off = x;
  bool recvd = x == root, leaf = false;
  int sb = x == root ? BS : -1;  // the buffer this rank forwards from
  const uint32_t vnb = to_nb(pmod(x - root, P));
  for (int mask = 1 << (L - 1); mask > 0; mask >>= 1, hd = -hd) {
    const int partner = nb_partner_root(vnb, mask, root, P);
    const uint32_t mlsb = (uint32_t)(mask << 1) - 1, lsbs = vnb & mlsb;
    const int64_t ts = minr, te = pmod64(minr + mask - 1, P), bs = pmod64(te + 1, P), be = maxr;  // :75-93
    int64_t ss, se, rs, re;
    if (hd == 1) { ss = bs; se = be; rs = ts; re = te; maxr = pmod64(maxr - mask, P); }
    else { ss = ts; se = te; rs = bs; re = be; minr = pmod64(minr + mask, P); }
    if (recvd) {  // :95-104
      if (sb < 0) { p.crash = true; return; }
      if (se >= ss) { p.send(partner, sb, ss, se - ss + 1); p.end(); }
      else { p.send(partner, sb, ss, P - ss); p.end(); p.send(partner, sb, 0, se + 1); p.end(); }
    } else if (lsbs == 0 || lsbs == mlsb) {  // :105-137
      const int64_t nb = pmod64(re - rs + 1, P);
      int rb = BR;
      if (rs == re) {
        leaf = true;
      } else {
        rb = sb = BT;
        p.size[BT] = nb;
        minr = 0;
        maxr = nb - 1;
        off = pmod64(x - rs, P);
      }
      if (re >= rs) { p.recv(partner, rb, 0, nb); p.end(); }
      else { p.recv(partner, rb, 0, P - rs); p.end(); p.recv(partner, rb, P - rs, re + 1); p.end(); }
      recvd = true;
    }
  }
  if (!leaf) {  // :142-144
    if (sb < 0) { p.crash = true; return; }
    p.copy(sb, off, BR, 0, 1);
  }
}

int remap_distance_doubling(uint32_t num) {  // libbine_utils.h:601-609
  int out = 0;
  while (num > 0) {
    const int k = 31 - __builtin_clz(num);
    out ^= 1 << k;
    num ^= (uint32_t)((1ull << (k + 1)) - 1);
  }
  return out;
}

// alltoall_bine, libbine_alltoall.c:14-147
void a2a_prog(int P, int x, BProg &p) {
  p.size[BS] = p.size[BR] = p.size[BT] = P;
  p.copy(BS, 0, BT, 0, P);  // :50
  const int L = log2_ceil(P);
  std::vector<int> res((size_t)P), nxt;
  for (int i = 0; i < P; i++) res[(size_t)i] = i;
  int nres = P, inv = L ? 1 << (L - 1) : 0;
  uint32_t bfm = ~(uint32_t)(inv - 1);
  for (int mask = 1; mask < P; mask <<= 1, inv >>= 1, bfm >>= 1) {
    const int partner = nb_partner(x, mask, P);  // :59-64
    const int64_t mins = remap_rank((uint32_t)P, (uint32_t)partner) & bfm, maxs = mins + inv - 1;
    int64_t ns = 0, nk = 0;
    nxt.clear();
    for (int i = 0; i < P; i++) {  // :71-94
      const int blk = res[(size_t)(i % nres)];
      const int64_t rb = remap_rank((uint32_t)P, (uint32_t)blk);
      if (rb >= mins && rb <= maxs) {
        p.copy(BT, i, BR, ns++, 1);
      } else {
        if (i != nk) p.copy(BT, i, BT, nk, 1);
        nk++;
        nxt.push_back(blk);
      }
    }
    if (nk != P / 2 || ns != P / 2) { p.crash = true; return; }  // :95-96
    nres /= 2;
    p.send(partner, BR, 0, ns);  // :100-102, one MPI_Sendrecv
    p.recv(partner, BT, P / 2, ns);
    p.end();
    for (int i = 0; i < nres; i++) res[(size_t)i] = nxt[(size_t)i];
  }
  for (int i = 0; i < P; i++) {  // :121-139
    const int rot = x % 2 == 0 ? pmod(i - x, P) : pmod(x - i, P);
    const uint32_t rep = nb_fits(rot, L) ? to_nb(rot) : to_nb(rot - P);
    p.copy(BT, remap_distance_doubling(rep), BR, i, 1);
  }
}

// Runs every rank's program on block tags (tag = source rank * P + block);
// true when all of it completes in bounds and delivers the collective.
bool blocks_run(int algo, int P, int root, std::vector<BProg> &pg, std::vector<std::vector<int>> &match) {
  for (auto &p : pg)
    if (p.crash) return false;
  std::vector<std::array<std::vector<int64_t>, 3>> tag((size_t)P);
  for (int x = 0; x < P; x++)
    for (int b = 0; b < 3; b++) tag[(size_t)x][(size_t)b].assign((size_t)pg[(size_t)x].size[b], -1);
  for (int x = 0; x < P; x++) {
    auto &s = tag[(size_t)x][BS];
    for (int64_t j = 0; j < (int64_t)s.size(); j++)
      s[(size_t)j] = algo == BINE_GA_BINE ? (int64_t)x * P : algo == BINE_SC_BINE ? (int64_t)root * P + j
                                                                                   : (int64_t)x * P + j;
  }
  auto in = [&](int x, int b, int64_t off, int64_t n) {
    return off >= 0 && n >= 0 && off + n <= (int64_t)tag[(size_t)x][(size_t)b].size();
  };
  // match sends and receives per ordered pair, in posting order
  std::map<std::pair<int, int>, std::vector<int>> sq, rq;
  match.assign((size_t)P, {});
  for (int x = 0; x < P; x++) {
    match[(size_t)x].assign(pg[(size_t)x].ops.size(), -1);
    for (int i = 0; i < (int)pg[(size_t)x].ops.size(); i++) {
      const BOp &o = pg[(size_t)x].ops[(size_t)i];
      if (o.kind == 1) sq[{x, o.peer}].push_back(i);
      if (o.kind == 2) rq[{o.peer, x}].push_back(i);
    }
  }
  for (auto &kv : sq) {
    const auto &r = rq[kv.first];
    if (r.size() != kv.second.size()) return false;
    for (size_t k = 0; k < r.size(); k++) {
      const BOp &s = pg[(size_t)kv.first.first].ops[(size_t)kv.second[k]];
      const BOp &v = pg[(size_t)kv.first.second].ops[(size_t)r[k]];
      if (s.n > v.n) return false;  // MPI_ERR_TRUNCATE
      match[(size_t)kv.first.first][(size_t)kv.second[k]] = r[k];
      match[(size_t)kv.first.second][(size_t)r[k]] = kv.second[k];
    }
  }
  for (auto &kv : rq)
    if (sq.find(kv.first) == sq.end() && !kv.second.empty()) return false;
  // rendezvous run: a rank's copies run in order; the messages of its current
  // exchange complete one by one as their peers reach the matching exchange
  std::vector<size_t> pc((size_t)P, 0);
  std::vector<std::vector<char>> done((size_t)P);
  for (int x = 0; x < P; x++) done[(size_t)x].assign(pg[(size_t)x].ops.size(), 0);
  auto grp_at = [&](int x) { const auto &o = pg[(size_t)x].ops; return pc[(size_t)x] < o.size() ? o[pc[(size_t)x]].grp : -2; };
  for (bool moved = true; moved;) {
    moved = false;
    for (int x = 0; x < P; x++) {
      auto &ops = pg[(size_t)x].ops;
      while (pc[(size_t)x] < ops.size()) {
        const BOp &o = ops[pc[(size_t)x]];
        if (o.kind == 0) {
          if (!in(x, o.sbuf, o.soff, o.n) || !in(x, o.buf, o.off, o.n)) return false;
          auto &sv = tag[(size_t)x][(size_t)o.sbuf];
          auto &dv = tag[(size_t)x][(size_t)o.buf];
          std::vector<int64_t> t(sv.begin() + o.soff, sv.begin() + o.soff + o.n);
          std::copy(t.begin(), t.end(), dv.begin() + o.off);
          pc[(size_t)x]++;
          moved = true;
          continue;
        }
        size_t e = pc[(size_t)x];
        while (e < ops.size() && ops[e].kind != 0 && ops[e].grp == o.grp) e++;
        bool all = true;
        for (size_t i = pc[(size_t)x]; i < e; i++) {
          if (done[(size_t)x][i]) continue;
          const BOp &m = ops[i];
          const int j = match[(size_t)x][i];
          const BOp &q = pg[(size_t)m.peer].ops[(size_t)j];
          if (grp_at(m.peer) != q.grp || q.kind == 0) { all = false; continue; }
          const BOp &s = m.kind == 1 ? m : q, &r = m.kind == 1 ? q : m;
          const int sx = m.kind == 1 ? x : m.peer, rx = m.kind == 1 ? m.peer : x;
          if (!in(sx, s.buf, s.off, s.n) || !in(rx, r.buf, r.off, s.n)) return false;
          auto &sv = tag[(size_t)sx][(size_t)s.buf];
          std::copy(sv.begin() + s.off, sv.begin() + s.off + s.n, tag[(size_t)rx][(size_t)r.buf].begin() + r.off);
          done[(size_t)x][i] = done[(size_t)m.peer][(size_t)j] = 1;
          moved = true;
        }
        if (!all) break;
        pc[(size_t)x] = e;
        moved = true;
      }
    }
  }
  for (int x = 0; x < P; x++)
    if (pc[(size_t)x] < pg[(size_t)x].ops.size()) return false;  // a hang
  for (int x = 0; x < P; x++) {
    const auto &rb = tag[(size_t)x][BR];
    if (algo == BINE_GA_BINE && x == root) {
      for (int j = 0; j < P; j++)
        if (rb[(size_t)j] != (int64_t)j * P) return false;
    } else if (algo == BINE_SC_BINE) {
      if (rb[0] != (int64_t)root * P + x) return false;
    } else if (algo == BINE_A2A_BINE) {
      for (int j = 0; j < P; j++)
        if (rb[(size_t)j] != (int64_t)j * P + x) return false;
    }
  }
  return true;
}

}  // namespace

void rooted_blocks(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  if (a.in_place) { b.fail(BINE_ERR_ARG); return; }  // the reference memcpy's from MPI_IN_PLACE
  const bool rooted = a.algo != BINE_A2A_BINE;
  if (rooted && (a.root < 0 || a.root >= P)) { b.fail(BINE_ERR_ROOT); return; }
  std::vector<BProg> pg((size_t)P);
  for (int x = 0; x < P; x++) {
    if (a.algo == BINE_GA_BINE) ga_prog(P, a.root, x, pg[(size_t)x]);
    else if (a.algo == BINE_SC_BINE) sc_prog(P, a.root, x, pg[(size_t)x]);
    else a2a_prog(P, x, pg[(size_t)x]);
  }
  std::vector<std::vector<int>> match;
  if (!blocks_run(a.algo, P, a.root, pg, match)) {
    b.fail(is_pow2(P) && rooted ? BINE_ERR_ROOT : BINE_ERR_SIZE);
    return;
  }
  const uint64_t c = a.count;
  const int map[3] = {SB, RB, T0};
  BProg &me = pg[(size_t)r];
  // runs of block copies that continue each other (alltoall's staging and
  // compaction, its final permutation) become one copy each -- unless the
  // merged source and destination overlap in one buffer (a forward compaction
  // must stay block by block); message matching is by index, so only copies
  // are merged and the send / receive indices are remapped
  {
    std::vector<BOp> ops;
    std::vector<int> idx(me.ops.size());
    for (size_t i = 0; i < me.ops.size(); i++) {
      const BOp &o = me.ops[i];
      if (o.kind == 0 && !ops.empty()) {
        BOp &q = ops.back();
        const bool cont = q.kind == 0 && q.sbuf == o.sbuf && q.buf == o.buf && q.soff + q.n == o.soff &&
                          q.off + q.n == o.off;
        const bool apart = o.sbuf != o.buf || q.soff + q.n + o.n <= q.off || q.off + q.n + o.n <= q.soff;
        if (cont && apart) {
          q.n += o.n;
          idx[i] = -1;
          continue;
        }
      }
      idx[i] = (int)ops.size();
      ops.push_back(o);
    }
    std::vector<int> m2(ops.size(), -1);
    for (size_t i = 0; i < me.ops.size(); i++)
      if (idx[i] >= 0) m2[(size_t)idx[i]] = match[(size_t)r][i];
    me.ops.swap(ops);
    match[(size_t)r].swap(m2);
  }
  if (me.size[BT]) b.tmp(T0, (uint64_t)me.size[BT] * c);
  for (size_t i = 0; i < me.ops.size(); i++) {
    const BOp &o = me.ops[i];
    if (o.kind == 0) {
      b.copy(map[o.sbuf], (uint64_t)o.soff * c, map[o.buf], (uint64_t)o.off * c, (uint64_t)o.n * c);
      continue;
    }
    if (o.kind == 1) {
      b.send(o.peer, map[o.buf], (uint64_t)o.off * c, (uint64_t)o.n * c);
    } else {  // the matching send's exact length
      const BOp &s = pg[(size_t)o.peer].ops[(size_t)match[(size_t)r][i]];
      b.recv(o.peer, map[o.buf], (uint64_t)o.off * c, (uint64_t)s.n * c);
    }
    if (i + 1 == me.ops.size() || me.ops[i + 1].kind == 0 || me.ops[i + 1].grp != o.grp) b.end();
  }
}

// the direct forms (flat_ag): every block straight from its source to its
// destination in one exchange -- one hop on every link of a fully connected
// node; the same bytes land where the literal schedule puts them
void rooted_flat(Builder &b, const PlanArgs &a) {
  const int P = a.P, r = a.rank;
  const uint64_t c = a.count;
  if (a.algo == BINE_GA_BINE) {
    if (r == a.root) {
      b.copy(SB, 0, RB, (uint64_t)r * c, c);
      for (int x = 0; x < P; x++) b.recv(x == r ? -1 : x, RB, (uint64_t)x * c, c);
    } else {
      b.send(a.root, SB, 0, c);
    }
  } else if (a.algo == BINE_SC_BINE) {
    if (r == a.root) {
      b.copy(SB, (uint64_t)r * c, RB, 0, c);
      for (int x = 0; x < P; x++) b.send(x == r ? -1 : x, SB, (uint64_t)x * c, c);
    } else {
      b.recv(a.root, RB, 0, c);
    }
  } else {
    b.copy(SB, (uint64_t)r * c, RB, (uint64_t)r * c, c);
    for (int x = 0; x < P; x++) b.send(x == r ? -1 : x, SB, (uint64_t)x * c, c);
    for (int x = 0; x < P; x++) b.recv(x == r ? -1 : x, RB, (uint64_t)x * c, c);
  }
  b.end();
}

Plan make_plan(const PlanArgs &a) {
  Builder b(a.rank);
  if (a.P < 1 || a.rank < 0 || a.rank >= a.P || a.esz == 0) { b.fail(BINE_ERR_ARG); return b.p; }
  const bool rs = a.algo >= BINE_RS_RECURSIVEHALVING && a.algo <= BINE_RS_BINE_BLOCK_BY_BLOCK_ANY_EVEN;
  if (rs && (int)a.rcounts.size() != a.P) { b.fail(BINE_ERR_ARG); return b.p; }
  const bool bc = a.algo >= BINE_BC_SCATTER_ALLGATHER && a.algo <= BINE_BC_BINE_BDW_REMAP;
  // nothing to move; the bcast trees still return the reference's size / root
  // errors at count 0 (their planners emit no zero-length message)
  if (!rs && !bc && a.count == 0) return b.p;
  switch (a.algo) {
    case BINE_AR_RECURSIVEDOUBLING: ar_recursivedoubling(b, a); break;
    case BINE_AR_RING: ar_ring(b, a); break;
    case BINE_AR_RABENSEIFNER: ar_rabenseifner(b, a); break;
    case BINE_AR_BINE_LAT: ar_bine_lat(b, a); break;
    case BINE_AR_BINE_BDW_STATIC: ar_bine_bdw_static(b, a); break;
    case BINE_AR_BINE_BDW_REMAP: ar_bine_remap(b, a, false); break;
    case BINE_AR_BINE_BDW_REMAP_SEGMENTED: ar_bine_remap(b, a, true); break;
    case BINE_AR_BINE_BLOCK_BY_BLOCK_ANY_EVEN: ar_bine_bbb_any_even(b, a); break;
    case BINE_RS_RECURSIVEHALVING: rs_recursivehalving(b, a); break;
    case BINE_RS_RECURSIVE_DISTANCE_DOUBLING: rs_recursive_distance_doubling(b, a); break;
    case BINE_RS_RING: rs_ring(b, a); break;
    case BINE_RS_BUTTERFLY: rs_butterfly(b, a); break;
    case BINE_RS_BINE_STATIC: rs_bine_static(b, a); break;
    case BINE_RS_BINE_SEND_REMAP: rs_bine_remap(b, a, false); break;
    case BINE_RS_BINE_PERMUTE_REMAP: rs_bine_remap(b, a, true); break;
    case BINE_RS_BINE_BLOCK_BY_BLOCK: rs_bine_bbb(b, a); break;
    case BINE_RS_BINE_BLOCK_BY_BLOCK_ANY_EVEN: rs_bine_bbb_any_even(b, a); break;
    case BINE_RD_BINE_LAT: rd_bine_lat(b, a); break;
    case BINE_RD_BINE_BDW: rd_bine_bdw(b, a); break;
    case BINE_AG_RECURSIVEDOUBLING: ag_recursivedoubling(b, a); break;
    case BINE_AG_K_BRUCK: ag_k_bruck(b, a); break;
    case BINE_AG_RING: ag_ring(b, a); break;
    case BINE_AG_SPARBIT: ag_sparbit(b, a); break;
    case BINE_AG_BINE_BLOCK_BY_BLOCK: ag_bine_bbb(b, a); break;
    case BINE_AG_BINE_BLOCK_BY_BLOCK_ANY_EVEN: ag_bine_bbb_any_even(b, a); break;
    case BINE_AG_BINE_PERMUTE_STATIC: ag_bine_static(b, a, true); break;
    case BINE_AG_BINE_SEND_STATIC: ag_bine_static(b, a, false); break;
    case BINE_AG_BINE_PERMUTE_REMAP: ag_bine_remap(b, a, true); break;
    case BINE_AG_BINE_SEND_REMAP: ag_bine_remap(b, a, false); break;
    case BINE_AG_BINE_2_BLOCKS:
    case BINE_AG_BINE_2_BLOCKS_DTYPE: ag_bine_2_blocks(b, a); break;
    case BINE_BC_BINE_LAT: bc_bine_lat(b, a, false); break;
    case BINE_BC_BINE_LAT_REVERSED: bc_bine_lat(b, a, true); break;
    case BINE_BC_BINE_LAT_NEW:
    case BINE_BC_BINE_LAT_I_NEW: bc_bine_lat_new(b, a); break;
    case BINE_BC_SCATTER_ALLGATHER: bc_scatter_allgather(b, a); break;
    case BINE_BC_BINE_BDW_STATIC: bc_bine_bdw_static(b, a); break;
    case BINE_BC_BINE_BDW_REMAP: bc_bine_bdw_remap(b, a); break;
    case BINE_A2A_BINE:
    case BINE_GA_BINE:
    case BINE_SC_BINE:
      rooted_blocks(b, a);
      if (a.flat_ag && a.P >= 2 && b.p.status == BINE_SUCCESS) {
        Builder f(a.rank);
        rooted_flat(f, a);
        return f.p;
      }
      break;
    default: b.fail(BINE_ERR_UNSUPPORTED); break;
  }
  if (!b.pend_send.empty() || !b.pend_recv.empty()) b.end();
  // flat allgather for the allgather family (out of place): the algorithm's
  // own plan decides the status (the reference's error returns stay); a
  // successful one is replaced by one all-peers exchange that places every
  // block where the algorithm leaves it (rank order) -- pure data movement
  const bool ag = a.algo >= BINE_AG_RECURSIVEDOUBLING && a.algo <= BINE_AG_BINE_2_BLOCKS_DTYPE;
  if (ag && a.flat_ag && !a.in_place && a.P >= 2 && b.p.status == BINE_SUCCESS) {
    Builder f(a.rank);
    const uint64_t n = a.count;
    f.copy(SB, 0, RB, (uint64_t)a.rank * n, n);
    for (int x = 0; x < a.P; x++)
      if (x != a.rank) f.send(x, SB, 0, n);
    for (int x = 0; x < a.P; x++)
      if (x != a.rank) f.recv(x, RB, (uint64_t)x * n, n);
    f.end();
    return f.p;
  }
  return b.p;
}

}  // namespace bine
