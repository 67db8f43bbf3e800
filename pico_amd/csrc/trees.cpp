// trees.cpp -- multi-tree mode: the same Bine schedule run as P-1 concurrent
// instances on P-1 slices of the buffer, each instance with its ranks
// relabelled so that, at every step, the P-1 instances pair the ranks along
// P-1 edge-disjoint perfect matchings -- together every xGMI link of a fully
// connected node, each message one hop (option (ii)).
//
// Instance k: virtual rank v (a rank of the reference's schedule) is played by
// physical rank sigma_k[v]; its input is that rank's slice k, so each slice is
// a valid allreduce of all ranks' data (reduce_scatter permute_remap: see
// Mapper below).  The reduction tree of a slice is the
// reference's tree over relabelled ranks: integer results are identical to the
// reference (wrapping SUM/PROD, MAX, MIN are associative and commutative);
// floating-point results differ from the reference only by association order
// and equal, bit for bit, the reference run on the permuted inputs (that is
// how the tests check them).  Opt-in (bine_comm_set_trees): the default path
// stays bit-exact with the reference for every type.
//
// Relabellings: for each step s the images sigma_k(M_s) of the step's matching
// M_s = {{r, pi(r, s)}} must be pairwise edge-disjoint over k.  Found by
// exhaustive search (tools/find_trees.py); tests/test_trees.py re-checks the
// property.
#include <algorithm>

#include "bine_internal.h"

namespace bine {

namespace {

const int kTrees4[3][4] = {{0, 1, 2, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}};
const int kTrees8[7][8] = {{0, 1, 2, 3, 4, 5, 6, 7}, {0, 2, 3, 1, 4, 6, 7, 5}, {0, 3, 1, 6, 2, 5, 7, 4},
                           {0, 4, 7, 2, 5, 1, 6, 3}, {0, 5, 3, 7, 1, 4, 6, 2}, {0, 6, 3, 5, 4, 2, 7, 1},
                           {0, 7, 3, 4, 2, 1, 5, 6}};

const int *relabel(int P, int k) {
  if (P == 4) return kTrees4[k];
  if (P == 8) return kTrees8[k];
  return nullptr;
}

constexpr uint64_t kAlign = 64;  // slice boundaries on 64-element multiples (>= 256 B)

struct Seg {
  std::vector<Prim> pre;    // local primitives before the group
  std::vector<Prim> group;  // the exchange (empty for the trailing locals)
};

std::vector<Seg> segments(const Plan &p) {
  std::vector<Seg> out(1);
  const auto &pr = p.prims;
  for (size_t i = 0; i < pr.size();) {
    if (pr[i].type != BINE_PRIM_SEND && pr[i].type != BINE_PRIM_RECV) {
      out.back().pre.push_back(pr[i++]);
      continue;
    }
    size_t j = i;
    while (j < pr.size() && (pr[j].type == BINE_PRIM_SEND || pr[j].type == BINE_PRIM_RECV) &&
           pr[j].group == pr[i].group)
      j++;
    out.back().group.assign(pr.begin() + (long)i, pr.begin() + (long)j);
    out.emplace_back();
    i = j;
  }
  return out;
}

}  // namespace

int tree_count(int P) { return (P == 4 || P == 8) ? P - 1 : 1; }

const int *tree_relabel(int P, int k) { return relabel(P, k); }

// One instance's plan mapped onto the physical buffers.  Allreduce: slice k is
// the element range [off, off + len) of sbuf and rbuf.  Reduce-scatter
// (permute_remap): slice k is sub-range k of every rank's block; the
// instance's virtual block u is physical block sigma_k[u] (its input is read
// block by block by the algorithm's own initial permutation copy, so the
// relabelling costs no extra pass), its output is sub-range k of the own block.
struct Mapper {
  int kind = 0;                       // 0 allreduce, 1 reduce_scatter
  uint64_t off = 0;                   // allreduce: slice offset
  std::vector<uint64_t> vdisp, vcnt;  // reduce_scatter: virtual block layout
  std::vector<uint64_t> pstart;       // reduce_scatter: physical start of virtual block u
  uint64_t rb_off = 0;                // reduce_scatter: offset in the own output block
  bool ok = true;
  uint64_t sbuf(uint64_t x, uint64_t n) {
    if (kind == 0) return x + off;
    size_t u = (size_t)(std::upper_bound(vdisp.begin(), vdisp.end(), x) - vdisp.begin()) - 1;
    if (x + n > vdisp[u] + vcnt[u]) ok = false;  // must stay inside one block
    return pstart[u] + (x - vdisp[u]);
  }
  uint64_t rbuf(uint64_t x) { return kind == 0 ? x + off : x + rb_off; }
};

Plan make_tree_plan(const PlanArgs &a) {
  Plan out;
  const int P = a.P, T = tree_count(P);
  const bool allreduce = a.algo >= BINE_AR_RECURSIVEDOUBLING && a.algo <= BINE_AR_BINE_BLOCK_BY_BLOCK_ANY_EVEN;
  const bool rs = a.algo == BINE_RS_BINE_PERMUTE_REMAP && !a.in_place && (int)a.rcounts.size() == P;
  bool fit = T >= 2 && (allreduce || rs);
  if (fit && allreduce) fit = a.count >= (uint64_t)T * kAlign;
  if (fit && rs)
    for (int c : a.rcounts) fit = fit && (uint64_t)c >= (uint64_t)T * kAlign;
  if (!fit) {
    out.status = BINE_ERR_UNSUPPORTED;
    return out;
  }
  // slice k of n elements: [k * base, ...), the last one takes the remainder
  auto slice_of = [&](uint64_t n, int k, uint64_t &o, uint64_t &l) {
    const uint64_t base = n / (uint64_t)T / kAlign * kAlign;
    o = (uint64_t)k * base;
    l = k == T - 1 ? n - o : base;
  };
  std::vector<uint64_t> pdisp((size_t)P + 1, 0);
  if (rs)
    for (int j = 0; j < P; j++) pdisp[(size_t)j + 1] = pdisp[(size_t)j] + (uint64_t)a.rcounts[(size_t)j];
  std::vector<std::vector<Seg>> segs((size_t)T);
  uint64_t tbase[3] = {0, 0, 0};
  for (int k = 0; k < T; k++) {
    const int *sig = relabel(P, k);
    int v = 0;
    while (sig[v] != a.rank) v++;
    PlanArgs b = a;
    b.flat_ag = false;  // instances keep their own (mirrored) allgather
    b.flat_rs = false;  // and their own halving steps
    b.rank = v;
    Mapper m;
    if (allreduce) {
      uint64_t l;
      slice_of(a.count, k, m.off, l);
      b.count = l;
    } else {
      m.kind = 1;
      m.vdisp.resize((size_t)P);
      m.vcnt.resize((size_t)P);
      m.pstart.resize((size_t)P);
      uint64_t acc = 0;
      for (int u = 0; u < P; u++) {
        const int j = sig[u];
        uint64_t o, l;
        slice_of((uint64_t)a.rcounts[(size_t)j], k, o, l);
        b.rcounts[(size_t)u] = (int)l;
        m.vdisp[(size_t)u] = acc;
        m.vcnt[(size_t)u] = l;
        m.pstart[(size_t)u] = pdisp[(size_t)j] + o;
        acc += l;
      }
      uint64_t l;
      slice_of((uint64_t)a.rcounts[(size_t)a.rank], k, m.rb_off, l);
    }
    Plan pk = make_plan(b);
    if (pk.status != BINE_SUCCESS) return pk;
    for (auto &x : pk.prims) {
      if (x.type == BINE_PRIM_SEND || x.type == BINE_PRIM_RECV) x.peer = sig[x.peer];
      auto shift = [&](int32_t buf, uint64_t &o) {
        if (buf == BINE_BUF_SBUF) o = m.sbuf(o, x.count);
        else if (buf == BINE_BUF_RBUF) o = m.rbuf(o);
        else if (buf >= BINE_BUF_TMP0 && buf <= BINE_BUF_TMP2) o += tbase[buf - BINE_BUF_TMP0];
      };
      if (x.type != BINE_PRIM_RECV) shift(x.src_buf, x.src_off);
      if (x.type != BINE_PRIM_SEND) shift(x.dst_buf, x.dst_off);
      if (x.type == BINE_PRIM_REDUCE3) shift(x.aux_buf, x.aux_off);
    }
    if (!m.ok) {
      out.status = BINE_ERR_UNSUPPORTED;
      return out;
    }
    for (int t = 0; t < 3; t++) tbase[t] += pk.tmp_elems[t];
    segs[(size_t)k] = segments(pk);
  }
  for (int t = 0; t < 3; t++) out.tmp_elems[t] = tbase[t];
  // merge step by step: every instance's locals before group g, then one
  // exchange holding all instances' group g (the pipelined reductions that
  // follow a group stay in instance order, matching the pairs' order)
  size_t nseg = 0;
  for (const auto &sg : segs) nseg = std::max(nseg, sg.size());
  int gid = 0;
  for (size_t g = 0; g < nseg; g++) {
    for (const auto &sg : segs)
      if (g < sg.size())
        for (const auto &x : sg[g].pre) out.prims.push_back(x);
    bool any = false;
    for (const auto &sg : segs)
      if (g < sg.size())
        for (auto x : sg[g].group) {
          x.group = gid;
          out.prims.push_back(x);
          any = true;
        }
    if (any) gid++;
  }
  return out;
}

}  // namespace bine
