// tools/plan_bounds.cpp -- host-only sweep of the planner and the issue
// scheduler (schedule.cpp, issue.cpp, trees.cpp) built with AddressSanitizer
// and UndefinedBehaviorSanitizer (tests/test_plan_bounds.py builds and runs it;
// no GPU, no HIP runtime).
//
// For every algorithm (reduce family, allgather, bcast, gather / scatter /
// alltoall), P = 1..16, every rank (and roots 0, P / 2, P - 1), ragged and
// even sizes, in and out of place, and every transport setting (flat
// allgather / flat reduce-scatter / multi-tree / relay, chunked or not) it
// checks that each primitive of the plan AND of the issue schedule stays
// inside the buffer it names: SBUF / RBUF as the caller passes them (the MPI
// in-place conventions of each collective), TMP0-2 within the plan's declared
// workspace, STAGE within the schedule's staging area.  An out-of-range
// primitive here would be an out-of-bounds access on the GPU.
//
// Usage: plan_bounds [max_P [algo]]   (prints one summary line; exit 1 on a violation)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "bine_internal.h"

using namespace bine;

namespace {

struct Bounds {
  uint64_t lim[6];
};

long g_checked = 0, g_bad = 0;

void report(const char *what, const PlanArgs &a, const Prim &p, int buf, uint64_t off, uint64_t n, uint64_t lim) {
  if (g_bad++ < 20)
    fprintf(stderr,
            "OUT OF RANGE (%s): algo %d P %d rank %d count %zu in_place %d flat_ag %d flat_rs %d: prim type %d buf %d "
            "[%llu, +%llu) > %llu\n",
            what, a.algo, a.P, a.rank, a.count, (int)a.in_place, (int)a.flat_ag, (int)a.flat_rs, p.type, buf,
            (unsigned long long)off, (unsigned long long)n, (unsigned long long)lim);
}

void range(const char *what, const PlanArgs &a, const Prim &p, int buf, uint64_t off, uint64_t n, const Bounds &b) {
  g_checked++;
  if (n == 0) return;
  if (buf < 0 || buf > BINE_BUF_STAGE || off + n > b.lim[buf] || off + n < off) report(what, a, p, buf, off, n,
                                                                                      buf >= 0 && buf <= 5 ? b.lim[buf] : 0);
}

void check_prim(const char *what, const PlanArgs &a, const Prim &p, const Bounds &b) {
  switch (p.type) {
    case BINE_PRIM_SEND: range(what, a, p, p.src_buf, p.src_off, p.count, b); break;
    case BINE_PRIM_RECV: range(what, a, p, p.dst_buf, p.dst_off, p.count, b); break;
    case BINE_PRIM_REDUCE:
    case BINE_PRIM_COPY:
      range(what, a, p, p.src_buf, p.src_off, p.count, b);
      range(what, a, p, p.dst_buf, p.dst_off, p.count, b);
      break;
    case BINE_PRIM_REDUCE3:
      range(what, a, p, p.src_buf, p.src_off, p.count, b);
      range(what, a, p, p.aux_buf, p.aux_off, p.count, b);
      range(what, a, p, p.dst_buf, p.dst_off, p.count, b);
      break;
    case BINE_PRIM_REDUCE_TREE:
      range(what, a, p, p.src_buf, p.src_off, (uint64_t)(p.peer - 1) * p.count, b);
      range(what, a, p, p.aux_buf, p.aux_off, p.count, b);
      range(what, a, p, p.dst_buf, p.dst_off, p.count, b);
      break;
    default:
      g_checked++;
      report("bad type", a, p, -1, 0, 0, 0);
  }
}

// the caller's buffers in elements, per the collective's MPI signature
Bounds caller_bounds(const PlanArgs &a, const Plan &plan, uint64_t stage) {
  Bounds b{};
  const int fam = a.algo / 16;  // 0 allreduce, 1 reduce_scatter, 2 reduce, 3 allgather, 4 bcast, 5 a2a/gather/scatter
  uint64_t total = 0;
  for (int x : a.rcounts) total += (uint64_t)x;
  uint64_t s = 0, r = 0;
  const uint64_t all = (uint64_t)a.P * a.count;
  if (fam == 0) s = r = a.count;
  else if (fam == 1) { s = total; r = a.in_place ? total : (uint64_t)a.rcounts[(size_t)a.rank]; }
  else if (fam == 2) { s = a.count; r = a.rank == a.root || a.in_place ? a.count : 0; }
  else if (fam == 3) { s = a.count; r = all; }
  else if (fam == 4) s = r = a.count;  // in place on the one buffer
  else if (a.algo == BINE_GA_BINE) { s = a.count; r = a.rank == a.root ? all : 0; }  // rbuf on the root only
  else if (a.algo == BINE_SC_BINE) { s = a.rank == a.root ? all : 0; r = a.count; }  // sbuf on the root only
  else s = r = all;
  // MPI_IN_PLACE: the executor maps SBUF onto the receive buffer (executor.cpp run_collective)
  b.lim[BINE_BUF_SBUF] = a.in_place ? r : s;
  b.lim[BINE_BUF_RBUF] = r;
  for (int t = 0; t < 3; t++) b.lim[BINE_BUF_TMP0 + t] = plan.tmp_elems[t];
  b.lim[BINE_BUF_STAGE] = stage;
  return b;
}

void sweep(PlanArgs a, int trees, size_t chunk, size_t relay_min) {
  a.flat_chunk = chunk;
  Plan plan;
  if (trees) plan = make_tree_plan(a);
  if (!trees || plan.status == BINE_ERR_UNSUPPORTED) plan = make_plan(a);
  if (plan.status != BINE_SUCCESS) return;
  Bounds b = caller_bounds(a, plan, 0);
  for (const Prim &p : plan.prims) check_prim("plan", a, p, b);
  SchedCfg cfg;
  cfg.chunk = chunk;
  cfg.in_place = a.in_place;
  Schedule sc;
  if (relay_min && a.P >= 3) {
    cfg.relay_min = relay_min;
    std::vector<Plan> all((size_t)a.P);
    for (int x = 0; x < a.P; x++) {
      PlanArgs c = a;
      c.rank = x;
      if (trees) all[(size_t)x] = make_tree_plan(c);
      if (!trees || all[(size_t)x].status == BINE_ERR_UNSUPPORTED) all[(size_t)x] = make_plan(c);
    }
    make_schedule(plan, &all, a.rank, cfg, sc);
  } else {
    make_schedule(plan, nullptr, a.rank, cfg, sc);
  }
  b = caller_bounds(a, plan, sc.stage_elems);
  for (const SOp &o : sc.ops)
    for (const Prim &p : o.prims) check_prim("schedule", a, p, b);
}

}  // namespace

int main(int argc, char **argv) {
  const int maxP = argc > 1 ? atoi(argv[1]) : 16;
  const int only = argc > 2 ? atoi(argv[2]) : -1;  // one algorithm id (-1: all)
  const int algos[] = {0, 1, 2, 3, 4, 5, 6, 7, 16, 17, 18, 19, 20, 21, 22, 23, 24, 32, 33,
                       48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 64, 65, 66, 67, 68, 69, 70, 80, 81, 82};
  const size_t counts[] = {0, 1, 13, 1000};
  long plans = 0;
  for (int algo : algos)
    for (int P = 1; P <= maxP && (only < 0 || only == algo); P++)
      for (size_t n : counts)
        for (int rag = 0; rag < 2; rag++)
          for (int ip = 0; ip < 2; ip++)
            for (int mode = 0; mode < 8; mode++)
              for (int rank = 0; rank < P; rank++)
               for (int root : {0, P / 2, P - 1}) {
                const int fam = algo / 16;
                if (rag && fam != 1) continue;  // ragged blocks: reduce_scatter only
                if (ip && fam == 2 && rank != 0) continue;  // in place only at the root (bine_reduce: ERR_ARG)
                if (root && fam < 4) continue;  // rooted sweeps: bcast, gather, scatter
                if (fam == 4 && !ip) continue;  // bcast: in place by definition
                if ((root == P / 2 && P / 2 == 0) || (root == P - 1 && (P - 1 == P / 2 || P - 1 == 0))) continue;
                PlanArgs a;
                a.root = root;
                a.algo = algo;
                a.P = P;
                a.rank = rank;
                a.count = n;
                a.esz = 4;
                a.in_place = ip != 0;
                a.segsize = algo == BINE_AR_BINE_BDW_REMAP_SEGMENTED ? 64 : 0;
                if (fam == 1)
                  for (int x = 0; x < P; x++) a.rcounts.push_back((int)(rag ? (n + 3 * (size_t)x) % 11 : n));
                a.flat_ag = (mode & 1) != 0;
                a.flat_rs = (mode & 2) != 0;
                const int trees = (mode & 4) != 0;
                for (size_t chunk : {(size_t)0, (size_t)5})
                  for (size_t relay : {(size_t)0, (size_t)1}) {
                    sweep(a, trees, chunk, relay);
                    plans++;
                  }
              }
  printf("plan_bounds: %ld plan/schedule builds, %ld ranges checked, %ld out of range\n", plans, g_checked, g_bad);
  return g_bad ? 1 : 0;
}
