// issue.cpp -- turns a per-rank plan (schedule.cpp) into the executor's
// two-stream issue schedule (see Schedule in bine_internal.h).
//
// Three transformations, none of which changes a single value the plan
// computes (each reduction still sees the same operands in the same order):
//
//  1. chunking: an exchange flagged BINE_PRIM_PIPELINE (one send + one receive
//     whose received block is consumed element-for-element by the following
//     REDUCE / REDUCE3) is cut into pieces, each feeding the matching piece of
//     the reduction -- the device form of the segmented variant's
//     Irecv/Reduce_local double buffering (libbine_allreduce.c:1218-1253);
//
//  2. region-based dependencies: every op records which element ranges of which
//     buffer it reads and writes; an op waits only for the newest op of the
//     OTHER stream it conflicts with (RAW / WAR / WAW).  Chunk k+1's transfer
//     overlaps chunk k's reduction, and the next step's first chunks go out
//     while this step's last chunks are still being reduced;
//
//  3. multi-link relay (optional, cfg.relay_min > 0): a Bine step is a
//     permutation -- every rank sends one block to one partner and receives one
//     block from another -- so a literal execution uses ONE of the seven xGMI
//     links of an MI355X per step.  Relay mode splits each chunk of such a step
//     into a direct part and P-2 parts routed over two hops through the other
//     ranks (first hop origin -> relay, second hop relay -> destination, the
//     relay forwarding from a staging buffer one round later).  With direct
//     part 2M/P and relay parts M/P every directed link carries 2M/P per step
//     instead of M on one link: P/2 times less time per step on a fully
//     connected node.  The bytes that land in each receive buffer are the
//     same; only their route differs.  Rounds are lock-step across ranks and
//     every directed link carries at most one first-hop part followed by at
//     most one forwarded part per round, posted in the same order at both ends
//     (RCCL matches sends and receives of a peer pair in posting order).
#include <algorithm>

#include "bine_internal.h"

namespace bine {

namespace {

struct Reg { int b; uint64_t lo, hi; };

struct Rec {
  bool xchg;
  std::vector<Reg> rd, wr;
};

bool hit(const std::vector<Reg> &a, const std::vector<Reg> &b) {
  for (const auto &x : a)
    for (const auto &y : b)
      if (x.b == y.b && x.lo < y.hi && y.lo < x.hi) return true;
  return false;
}

bool is_x(const Prim &p) { return p.type == BINE_PRIM_SEND || p.type == BINE_PRIM_RECV; }

// [start, end) prim index ranges of the exchange groups of a plan
std::vector<std::pair<size_t, size_t>> groups_of(const Plan &pl) {
  std::vector<std::pair<size_t, size_t>> g;
  const auto &pr = pl.prims;
  for (size_t i = 0; i < pr.size();) {
    if (!is_x(pr[i])) { i++; continue; }
    size_t j = i;
    while (j < pr.size() && is_x(pr[j]) && pr[j].group == pr[i].group) j++;
    g.push_back({i, j});
    i = j;
  }
  return g;
}

// one rank's single send / single receive of a permutation step
struct Perm {
  Prim send, recv;
};

bool one_send_one_recv(const Plan &pl, std::pair<size_t, size_t> g, Perm &out) {
  if (g.second - g.first != 2) return false;
  const Prim &a = pl.prims[g.first], &b = pl.prims[g.first + 1];
  if (a.type == b.type) return false;
  out.send = a.type == BINE_PRIM_SEND ? a : b;
  out.recv = a.type == BINE_PRIM_RECV ? a : b;
  return true;
}

Prim mk(int type, int peer, int buf, uint64_t off, uint64_t count) {
  Prim p{};
  p.type = type;
  p.peer = peer;
  if (type == BINE_PRIM_SEND) { p.src_buf = buf; p.src_off = off; }
  else { p.dst_buf = buf; p.dst_off = off; }
  p.count = count;
  return p;
}

Prim slice(const Prim &q, uint64_t o, uint64_t n) {
  Prim x = q;
  x.src_off += o;
  x.dst_off += o;
  x.aux_off += o;
  x.count = n;
  return x;
}

// Relay rounds of one permutation step at rank r.  steps[x] = rank x's
// send/recv of this step.  Optional pipelined reduction q follows chunk by chunk.
void emit_relay(const std::vector<Perm> &steps, int r, size_t ch, size_t relay_min, const Prim *q,
                std::vector<SOp> &ops, uint64_t &stage_elems) {
  const int P = (int)steps.size();
  std::vector<int> to((size_t)P), from((size_t)P);
  for (int x = 0; x < P; x++) {
    to[(size_t)x] = steps[(size_t)x].send.peer;
    from[(size_t)to[(size_t)x]] = x;
  }
  auto S = [&](int x) { return (uint64_t)steps[(size_t)x].send.count; };
  uint64_t cmax = 0;
  for (int x = 0; x < P; x++) cmax = std::max(cmax, S(x));
  const uint64_t cht = ch ? ch : cmax;
  auto nch = [&](int x) { return (S(x) + cht - 1) / cht; };
  auto clen = [&](int x, uint64_t j) { return std::min<uint64_t>(cht, S(x) - j * cht); };
  // relay part size of chunk j of pair x (0: chunk goes direct only)
  auto u_of = [&](int x, uint64_t j) -> uint64_t {
    const uint64_t c = clen(x, j);
    return c >= (uint64_t)relay_min * (uint64_t)P ? c / (uint64_t)P : 0;
  };
  auto d_of = [&](int x, uint64_t j) { return clen(x, j) - (uint64_t)(P - 2) * u_of(x, j); };
  // relays of pair x: ranks other than x and to[x], increasing
  auto relays = [&](int x) {
    std::vector<int> v;
    for (int k = 0; k < P; k++)
      if (k != x && k != to[(size_t)x]) v.push_back(k);
    return v;
  };
  // pairs rank r relays for (x != r, to[x] != r), increasing x -> staging index
  std::vector<int> mine;
  for (int x = 0; x < P; x++)
    if (x != r && to[(size_t)x] != r) mine.push_back(x);
  uint64_t umax = 0;
  for (int x = 0; x < P; x++)
    for (uint64_t j = 0; j < nch(x); j++) umax = std::max(umax, u_of(x, j));
  stage_elems = std::max(stage_elems, 2 * (uint64_t)mine.size() * umax);
  auto stage_off = [&](uint64_t slot, size_t idx) { return (slot * mine.size() + idx) * umax; };

  uint64_t rounds = 0;
  for (int x = 0; x < P; x++) rounds = std::max(rounds, nch(x) + 1);
  const Perm &me = steps[(size_t)r];
  const int qsrc = from[(size_t)r];
  const std::vector<int> my_relays = relays(r), in_relays = relays(qsrc);
  uint64_t reduced = 0;  // pipelined reduction chunks emitted so far
  for (uint64_t j = 0; j < rounds; j++) {
    SOp o{true, {}, -1};
    // sends: direct and first hops of my chunk j, then forwards of chunk j-1
    if (j < nch(r)) {
      const uint64_t base = me.send.src_off + j * cht, d = d_of(r, j), u = u_of(r, j);
      o.prims.push_back(mk(BINE_PRIM_SEND, to[(size_t)r], me.send.src_buf, base, d));
      if (u)
        for (size_t i = 0; i < my_relays.size(); i++)
          o.prims.push_back(mk(BINE_PRIM_SEND, my_relays[i], me.send.src_buf, base + d + i * u, u));
    }
    if (j >= 1)
      for (size_t idx = 0; idx < mine.size(); idx++) {
        const int x = mine[idx];
        if (j - 1 < nch(x) && u_of(x, j - 1))
          o.prims.push_back(mk(BINE_PRIM_SEND, to[(size_t)x], BINE_BUF_STAGE, stage_off((j - 1) % 2, idx),
                               u_of(x, j - 1)));
      }
    // receives: direct part of chunk j, first hops I relay, second hops of chunk j-1
    if (j < nch(qsrc))
      o.prims.push_back(mk(BINE_PRIM_RECV, qsrc, me.recv.dst_buf, me.recv.dst_off + j * cht, d_of(qsrc, j)));
    for (size_t idx = 0; idx < mine.size(); idx++) {
      const int x = mine[idx];
      if (j < nch(x) && u_of(x, j))
        o.prims.push_back(mk(BINE_PRIM_RECV, x, BINE_BUF_STAGE, stage_off(j % 2, idx), u_of(x, j)));
    }
    if (j >= 1 && j - 1 < nch(qsrc) && u_of(qsrc, j - 1)) {
      const uint64_t u = u_of(qsrc, j - 1), base = me.recv.dst_off + (j - 1) * cht + d_of(qsrc, j - 1);
      for (size_t i = 0; i < in_relays.size(); i++)
        o.prims.push_back(mk(BINE_PRIM_RECV, in_relays[i], me.recv.dst_buf, base + i * u, u));
    }
    if (!o.prims.empty()) ops.push_back(std::move(o));
    // chunk j-1 of my receive is complete after round j
    if (q && j >= 1) {
      const uint64_t lo = (j - 1) * cht;
      if (lo < q->count) {
        ops.push_back({false, {slice(*q, lo, std::min<uint64_t>(cht, q->count - lo))}, -1});
        reduced = j;
      }
    }
  }
  if (q)
    for (uint64_t k = reduced; k * cht < q->count; k++)
      ops.push_back({false, {slice(*q, k * cht, std::min<uint64_t>(cht, q->count - k * cht))}, -1});
}

// Pipelined pairs of an exchange group: the group is n {send, recv} pairs
// (n = 1 normally; one per instance in multi-tree plans), each flagged
// PIPELINE, followed by n pipelined REDUCE / REDUCE3, the i-th consuming the
// i-th pair's receive element for element (the planner's contract for the
// flag).  Returns n, 0 if the group is not of that shape.
size_t pipe_pairs(const Plan &pl, std::pair<size_t, size_t> g) {
  const auto &pr = pl.prims;
  const size_t m = g.second - g.first;
  if (m == 0 || m % 2) return 0;
  const size_t n = m / 2;
  if (g.second + n > pr.size()) return 0;
  for (size_t i = 0; i < n; i++) {
    const Prim &x = pr[g.first + 2 * i], &y = pr[g.first + 2 * i + 1];
    if (x.type == y.type || !(x.flags & BINE_PRIM_PIPELINE) || !(y.flags & BINE_PRIM_PIPELINE)) return 0;
    const Prim &q = pr[g.second + i];
    // (the flags alone decide: both ends of a pair must cut it the same way)
    if (!(q.flags & BINE_PRIM_PIPELINE) || (q.type != BINE_PRIM_REDUCE && q.type != BINE_PRIM_REDUCE3)) return 0;
  }
  return n;
}

// chunked (or whole) exchange group g of `pl`; with n pipelined pairs the
// reductions that follow are cut along with it (all pairs advance together,
// one chunk of every pair per exchange)
void emit_direct(const Plan &pl, std::pair<size_t, size_t> g, size_t n, size_t ch, std::vector<SOp> &ops) {
  const auto &pr = pl.prims;
  if (!n || !ch) {
    ops.push_back({true, std::vector<Prim>(pr.begin() + (long)g.first, pr.begin() + (long)g.second), -1});
    return;
  }
  // both ends of a pair derive its chunk count from the same two sizes (my
  // send is the peer's receive and vice versa), so the k-th groups pair up
  std::vector<const Prim *> S(n), R(n), Q(n);
  std::vector<uint64_t> cs(n);  // per pair: `ch` rebalanced so its chunks come out even
  uint64_t rounds = 0;
  for (size_t i = 0; i < n; i++) {
    const Prim &x = pr[g.first + 2 * i], &y = pr[g.first + 2 * i + 1];
    S[i] = x.type == BINE_PRIM_SEND ? &x : &y;
    R[i] = x.type == BINE_PRIM_RECV ? &x : &y;
    Q[i] = &pr[g.second + i];
    const uint64_t m = std::max(S[i]->count, R[i]->count), k = (m + ch - 1) / ch;
    cs[i] = k ? std::min<uint64_t>(ch, ((m + k - 1) / k + 15) / 16 * 16) : ch;
    rounds = std::max(rounds, std::max((S[i]->count + cs[i] - 1) / cs[i], (R[i]->count + cs[i] - 1) / cs[i]));
  }
  for (uint64_t k = 0; k < rounds; k++) {
    SOp x{true, {}, -1};
    for (size_t i = 0; i < n; i++) {
      const uint64_t o = k * cs[i], c = cs[i];
      if (o < S[i]->count) {
        Prim a = *S[i];
        a.src_off += o;
        a.count = std::min<uint64_t>(c, S[i]->count - o);
        x.prims.push_back(a);
      }
      if (o < R[i]->count) {
        Prim a = *R[i];
        a.dst_off += o;
        a.count = std::min<uint64_t>(c, R[i]->count - o);
        x.prims.push_back(a);
      }
    }
    if (!x.prims.empty()) ops.push_back(x);
    // this round's chunk reductions of every pair: one op (one batched launch)
    SOp q{false, {}, -1};
    for (size_t i = 0; i < n; i++) {
      const uint64_t o = k * cs[i];
      if (o < Q[i]->count) q.prims.push_back(slice(*Q[i], o, std::min<uint64_t>(cs[i], Q[i]->count - o)));
    }
    if (!q.prims.empty()) ops.push_back(q);
  }
}

}  // namespace

void make_schedule(const Plan &plan, size_t ch, bool in_place, Schedule &out) {
  SchedCfg cfg;
  cfg.chunk = ch;
  cfg.in_place = in_place;
  make_schedule(plan, nullptr, 0, cfg, out);
}

void make_schedule(const Plan &plan, const std::vector<Plan> *all, int rank, const SchedCfg &cfg, Schedule &out) {
  const size_t ch = cfg.chunk;
  out.ops.clear();
  out.c_join = false;
  out.final_wait = -1;
  out.stage_elems = 0;
  out.relayed_steps = 0;

  // ---- which exchange groups are relayable permutation steps ----
  const auto mg = groups_of(plan);
  std::vector<std::vector<Perm>> perm(mg.size());
  if (cfg.relay_min && all && all->size() >= 3) {
    const int P = (int)all->size();
    std::vector<std::vector<std::pair<size_t, size_t>>> gs((size_t)P);
    bool same = true;
    for (int x = 0; x < P && same; x++) {
      gs[(size_t)x] = groups_of((*all)[(size_t)x]);
      same = gs[(size_t)x].size() == mg.size();
    }
    for (size_t t = 0; same && t < mg.size(); t++) {
      std::vector<Perm> st((size_t)P);
      std::vector<int> hits((size_t)P, 0);
      bool ok = true;
      for (int x = 0; x < P && ok; x++) {
        ok = one_send_one_recv((*all)[(size_t)x], gs[(size_t)x][t], st[(size_t)x]);
        if (!ok) break;
        const int y = st[(size_t)x].send.peer;
        ok = y != x && y >= 0 && y < P;
        if (ok) hits[(size_t)y]++;
      }
      for (int x = 0; x < P && ok; x++) ok = hits[(size_t)x] == 1;
      for (int x = 0; x < P && ok; x++) {
        const Perm &a = st[(size_t)x];
        const Perm &b = st[(size_t)a.send.peer];  // the receiver
        ok = b.recv.peer == x && b.recv.count == a.send.count;
      }
      if (ok) perm[t] = std::move(st);
    }
  }

  // ---- ops in issue order ----
  const auto &pr = plan.prims;
  size_t t = 0;
  for (size_t i = 0; i < pr.size();) {
    if (!is_x(pr[i])) {
      out.ops.push_back({false, {pr[i]}, -1});
      i++;
      continue;
    }
    const auto g = mg[t];
    const size_t npipe = pipe_pairs(plan, g);
    if (!perm[t].empty()) {
      const bool qpipe = (pr[g.first].flags & BINE_PRIM_PIPELINE) && g.second < pr.size() &&
                         (pr[g.second].flags & BINE_PRIM_PIPELINE) &&
                         (pr[g.second].type == BINE_PRIM_REDUCE || pr[g.second].type == BINE_PRIM_REDUCE3);
      emit_relay(perm[t], rank, ch, cfg.relay_min, qpipe ? &pr[g.second] : nullptr, out.ops, out.stage_elems);
      out.relayed_steps++;
      i = g.second + (qpipe ? 1 : 0);
    } else {
      emit_direct(plan, g, npipe, ch, out.ops);
      i = g.second + (ch ? npipe : 0);
    }
    t++;
  }

  // ---- dependencies ----
  auto reg = [&](int buf, uint64_t off, uint64_t n) {
    return Reg{(cfg.in_place && buf == BINE_BUF_SBUF) ? BINE_BUF_RBUF : buf, off, off + n};
  };
  std::vector<Rec> hist;
  hist.reserve(out.ops.size());
  int64_t waited[2] = {-1, -1};  // per stream: newest op of the other stream already waited for
  // bounded scan: past kWindow non-conflicting ops of the other stream, wait
  // for the oldest of them instead, which orders everything older as well
  constexpr int kWindow = 64;
  for (auto &o : out.ops) {
    Rec r;
    r.xchg = o.xchg;
    for (const Prim &p : o.prims) {
      switch (p.type) {
        case BINE_PRIM_SEND: r.rd.push_back(reg(p.src_buf, p.src_off, p.count)); break;
        case BINE_PRIM_RECV: r.wr.push_back(reg(p.dst_buf, p.dst_off, p.count)); break;
        case BINE_PRIM_REDUCE:
          r.rd.push_back(reg(p.src_buf, p.src_off, p.count));
          r.rd.push_back(reg(p.dst_buf, p.dst_off, p.count));
          r.wr.push_back(reg(p.dst_buf, p.dst_off, p.count));
          break;
        case BINE_PRIM_REDUCE3:
          r.rd.push_back(reg(p.src_buf, p.src_off, p.count));
          r.rd.push_back(reg(p.aux_buf, p.aux_off, p.count));
          r.wr.push_back(reg(p.dst_buf, p.dst_off, p.count));
          break;
        case BINE_PRIM_REDUCE_TREE:
          r.rd.push_back(reg(p.aux_buf, p.aux_off, p.count));
          r.rd.push_back(reg(p.src_buf, p.src_off, (uint64_t)(p.peer - 1) * p.count));
          r.wr.push_back(reg(p.dst_buf, p.dst_off, p.count));
          break;
        default:  // COPY
          r.rd.push_back(reg(p.src_buf, p.src_off, p.count));
          r.wr.push_back(reg(p.dst_buf, p.dst_off, p.count));
      }
    }
    // the comm stream first orders itself after the caller's prior work
    if (o.xchg) out.c_join = true;
    const int s = o.xchg ? 1 : 0;
    int64_t dep = -1, oldest = -1;
    int seen = 0;
    for (int64_t j = (int64_t)hist.size() - 1; j > waited[s]; j--) {
      const Rec &h = hist[(size_t)j];
      if (h.xchg == o.xchg) continue;
      if (hit(h.wr, r.rd) || hit(h.wr, r.wr) || hit(h.rd, r.wr)) {
        dep = j;
        break;
      }
      oldest = j;
      if (++seen >= kWindow) {
        for (int64_t k = j - 1; k > waited[s]; k--)
          if (hist[(size_t)k].xchg != o.xchg) {
            dep = oldest;
            break;
          }
        break;
      }
    }
    if (dep >= 0) waited[s] = dep;
    o.wait = dep;
    hist.push_back(std::move(r));
  }
  // the caller's stream ends after the last exchange
  for (int64_t j = (int64_t)out.ops.size() - 1; j >= 0; j--)
    if (out.ops[(size_t)j].xchg) {
      if (j > waited[0]) out.final_wait = j;
      break;
    }
  // only ops something waits for need an event recorded after them
  out.signals.assign(out.ops.size(), 0);
  for (const auto &o : out.ops)
    if (o.wait >= 0) out.signals[(size_t)o.wait] = 1;
  if (out.final_wait >= 0) out.signals[(size_t)out.final_wait] = 1;
}

// ---- host staging -------------------------------------------------------------

namespace {

// element ranges op `o` reads (rd) and writes (wr) in buffer `buf` (SBUF
// counts as RBUF in place, as in the dependency pass above)
void touched(const SOp &o, int buf, bool in_place, std::vector<Ivl> *rd, std::vector<Ivl> *wr) {
  auto add = [&](std::vector<Ivl> *v, int b, uint64_t off, uint64_t n) {
    if (in_place && b == BINE_BUF_SBUF) b = BINE_BUF_RBUF;
    if (v && b == buf && n) v->push_back({off, off + n});
  };
  for (const Prim &p : o.prims) {
    switch (p.type) {
      case BINE_PRIM_SEND: add(rd, p.src_buf, p.src_off, p.count); break;
      case BINE_PRIM_RECV: add(wr, p.dst_buf, p.dst_off, p.count); break;
      case BINE_PRIM_REDUCE:
        add(rd, p.src_buf, p.src_off, p.count);
        add(rd, p.dst_buf, p.dst_off, p.count);
        add(wr, p.dst_buf, p.dst_off, p.count);
        break;
      case BINE_PRIM_REDUCE3:
        add(rd, p.src_buf, p.src_off, p.count);
        add(rd, p.aux_buf, p.aux_off, p.count);
        add(wr, p.dst_buf, p.dst_off, p.count);
        break;
      case BINE_PRIM_REDUCE_TREE:
        add(rd, p.aux_buf, p.aux_off, p.count);
        add(rd, p.src_buf, p.src_off, (uint64_t)(p.peer - 1) * p.count);
        add(wr, p.dst_buf, p.dst_off, p.count);
        break;
      default:  // COPY
        add(rd, p.src_buf, p.src_off, p.count);
        add(wr, p.dst_buf, p.dst_off, p.count);
    }
  }
}

// sorted, disjoint, merged interval set
struct IvlSet {
  std::vector<Ivl> v;
  // pieces of [lo, hi) not in the set
  void minus(uint64_t lo, uint64_t hi, std::vector<Ivl> &out) const {
    auto it = std::upper_bound(v.begin(), v.end(), Ivl{lo, ~(uint64_t)0});
    if (it != v.begin() && std::prev(it)->second > lo) --it;
    uint64_t at = lo;
    for (; it != v.end() && it->first < hi; ++it) {
      if (it->first > at) out.push_back({at, it->first});
      at = std::max(at, it->second);
    }
    if (at < hi) out.push_back({at, hi});
  }
  void add(uint64_t lo, uint64_t hi) {
    if (lo >= hi) return;
    auto it = std::lower_bound(v.begin(), v.end(), Ivl{lo, 0});
    if (it != v.begin() && std::prev(it)->second >= lo) --it;
    auto end = it;
    while (end != v.end() && end->first <= hi) {
      lo = std::min(lo, end->first);
      hi = std::max(hi, end->second);
      ++end;
    }
    it = v.erase(it, end);
    v.insert(it, {lo, hi});
  }
};

void merge_adjacent(std::vector<Ivl> &x) {
  std::sort(x.begin(), x.end());
  std::vector<Ivl> m;
  for (const Ivl &r : x) {
    if (!m.empty() && r.first <= m.back().second) m.back().second = std::max(m.back().second, r.second);
    else m.push_back(r);
  }
  x.swap(m);
}

}  // namespace

void stage_ranges(const Schedule &sc, bool in_place, StageRanges &out) {
  const size_t n = sc.ops.size();
  const int in_buf = in_place ? BINE_BUF_RBUF : BINE_BUF_SBUF;
  out.h2d.assign(n, {});
  out.d2h.assign(n, {});
  out.h2d_wait.assign(n, -1);
  // forward: first touch of every input piece; `who` remembers which op's
  // batch staged each piece (a later toucher waits for that batch)
  IvlSet covered;
  std::vector<std::pair<Ivl, int64_t>> who;
  std::vector<Ivl> rd, wr, fresh;
  for (size_t i = 0; i < n; i++) {
    rd.clear();
    wr.clear();
    touched(sc.ops[i], in_buf, in_place, &rd, &wr);
    rd.insert(rd.end(), wr.begin(), wr.end());
    int64_t w = -1;
    for (const Ivl &r : rd) {
      fresh.clear();
      covered.minus(r.first, r.second, fresh);
      for (const Ivl &f : fresh) {
        covered.add(f.first, f.second);
        out.h2d[i].push_back(f);
        who.push_back({f, (int64_t)i});
        w = (int64_t)i;
      }
      for (const auto &q : who)  // pieces staged by earlier batches
        if (q.first.first < r.second && r.first < q.first.second) w = std::max(w, q.second);
    }
    merge_adjacent(out.h2d[i]);
    out.h2d_wait[i] = w;
  }
  // backward: the last write of every output piece
  IvlSet later;
  for (size_t i = n; i-- > 0;) {
    wr.clear();
    touched(sc.ops[i], BINE_BUF_RBUF, in_place, nullptr, &wr);
    for (const Ivl &r : wr) later.minus(r.first, r.second, out.d2h[i]);
    for (const Ivl &r : wr) later.add(r.first, r.second);
    merge_adjacent(out.d2h[i]);
  }
}

}  // namespace bine
