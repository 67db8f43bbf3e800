/*
 * op_check.c -- the libbine.h drop-in (pico_amd/lib/libbine.so) against
 * MPICH's OWN collectives, for every operator / type pair whose result does
 * not depend on the reduction order (so the check can be exact, the way
 * pico_core checks integer results, pico_core_utils.c:553-610):
 *   integers      SUM, PROD, MAX, MIN, LAND, LOR, LXOR, BAND, BOR, BXOR
 *   float/double  MAX, MIN, LAND, LOR, LXOR (no NaN in the inputs), and SUM,
 *                 PROD too: the inputs are multiples of 1/4 below 5 in
 *                 magnitude, so every partial sum or product of up to 4 of
 *                 them is exact in float, whatever the order (P <= 4)
 *   pair types    MAXLOC, MINLOC (ties on purpose)
 * through allreduce (Bine bandwidth / latency, ring), reduce_scatter (Bine
 * permute-remap, block-by-block) and reduce (Bine bandwidth), host buffers
 * staged by the shim, compared byte for byte (pair types: field by field;
 * floats: by value)
 * with PMPI_Allreduce / PMPI_Reduce_scatter / PMPI_Reduce.  And the pairs
 * MPICH rejects come back as MPI_ERR_OP.  Then the bcast latency trees
 * (bine_lat, _reversed at root 0; _new, _i_new at every root) vs PMPI_Bcast,
 * four allgathers vs PMPI_Allgather, and gather_bine / scatter_bine /
 * alltoall_bine vs PMPI_Gather / _Scatter / _Alltoall, every type (P a power
 * of two).
 *   usage: mpiexec -n P op_check      (prints "OPCHECK ok <cases>" on rank 0)
 * P a power of two: the remap / block-by-block reduce-scatters report
 * MPI_ERR_ARG elsewhere (the reference hangs there; DESIGN.md deviations).
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libbine_amd.h"

typedef struct { float v; int i; } float_int;
typedef struct { double v; int i; } double_int;
typedef struct { int v; int i; } int2;

typedef struct { const char *name; MPI_Datatype dt; size_t esz; int kind; } type_t;  /* kind 0 int, 1 fp, 2 pair */
typedef struct { const char *name; MPI_Op op; int ints, fps, pairs; } op_t;

static unsigned lcg(unsigned *s) { *s = *s * 1103515245u + 12345u; return (*s >> 8) & 0xFFFFFF; }

/* inputs with zeros (logical ops see both truth values) and small value
 * ranges (MAX / MIN / MAXLOC ties) */
static void fill(void *b, const type_t *t, size_t n, unsigned seed) {
  for (size_t k = 0; k < n; k++) {
    unsigned r = lcg(&seed);
    int zero = r % 5 == 0;
    switch (t->kind) {
      case 0: {
        int64_t v = zero ? 0 : (int64_t)(r % 97) - 40;
        memcpy((char *)b + k * t->esz, &v, t->esz);  /* little endian: low bytes */
        break;
      }
      case 1:
        if (t->esz == 4) ((float *)b)[k] = zero ? (r & 1 ? -0.0f : 0.0f) : (float)(r % 31) * 0.25f - 3.0f;
        else ((double *)b)[k] = zero ? 0.0 : (double)(r % 31) * 0.25 - 3.0;
        break;
      default:
        if (t->dt == MPI_FLOAT_INT) { ((float_int *)b)[k].v = (float)(r % 7); ((float_int *)b)[k].i = (int)(r % 13); }
        else if (t->dt == MPI_DOUBLE_INT) {
          memset((char *)b + k * t->esz, 0, t->esz);
          ((double_int *)b)[k].v = (double)(r % 7); ((double_int *)b)[k].i = (int)(r % 13);
        } else { ((int2 *)b)[k].v = (int)(r % 7); ((int2 *)b)[k].i = (int)(r % 13); }
    }
  }
}

static int same(const void *a, const void *b, const type_t *t, size_t n) {
  if (t->dt == MPI_DOUBLE_INT) {   /* padding is not part of the type map */
    for (size_t k = 0; k < n; k++)
      if (((const double_int *)a)[k].v != ((const double_int *)b)[k].v ||
          ((const double_int *)a)[k].i != ((const double_int *)b)[k].i) return 0;
    return 1;
  }
  if (t->kind == 1) {   /* by value: the sign of a zero under MAX / MIN follows the reduction order
                           (MPICH's tree differs from Bine's; the oracle tests pin the bits) */
    for (size_t k = 0; k < n; k++)
      if (t->esz == 4 ? ((const float *)a)[k] != ((const float *)b)[k]
                      : ((const double *)a)[k] != ((const double *)b)[k]) return 0;
    return 1;
  }
  return memcmp(a, b, n * t->esz) == 0;
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, P;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);
  if (P > 4) {   /* the exactness argument for float SUM / PROD above */
    if (rank == 0) fprintf(stderr, "op_check: P <= 4\n");
    MPI_Finalize();
    return 2;
  }
  const type_t types[] = {{"int8", MPI_INT8_T, 1, 0}, {"uint8", MPI_UNSIGNED_CHAR, 1, 0}, {"int16", MPI_SHORT, 2, 0},
                          {"int32", MPI_INT, 4, 0}, {"uint32", MPI_UNSIGNED, 4, 0}, {"int64", MPI_INT64_T, 8, 0},
                          {"float", MPI_FLOAT, 4, 1}, {"double", MPI_DOUBLE, 8, 1},
                          {"float_int", MPI_FLOAT_INT, sizeof(float_int), 2},
                          {"double_int", MPI_DOUBLE_INT, sizeof(double_int), 2}, {"2int", MPI_2INT, sizeof(int2), 2}};
  const op_t ops[] = {{"sum", MPI_SUM, 1, 1, 0}, {"prod", MPI_PROD, 1, 1, 0}, {"max", MPI_MAX, 1, 1, 0},
                      {"min", MPI_MIN, 1, 1, 0}, {"land", MPI_LAND, 1, 1, 0}, {"lor", MPI_LOR, 1, 1, 0},
                      {"lxor", MPI_LXOR, 1, 1, 0}, {"band", MPI_BAND, 1, 0, 0}, {"bor", MPI_BOR, 1, 0, 0},
                      {"bxor", MPI_BXOR, 1, 0, 0}, {"maxloc", MPI_MAXLOC, 0, 0, 1}, {"minloc", MPI_MINLOC, 0, 0, 1}};
  const size_t counts[] = {1, 7, 1000, 4099};
  int cases = 0, bad = 0;
  for (size_t ti = 0; ti < sizeof types / sizeof *types; ti++) {
    const type_t *t = &types[ti];
    for (size_t oi = 0; oi < sizeof ops / sizeof *ops; oi++) {
      const op_t *o = &ops[oi];
      const int ok_pair = t->kind == 0 ? o->ints : t->kind == 1 ? o->fps : o->pairs;
      for (size_t ci = 0; ci < sizeof counts / sizeof *counts; ci++) {
        const size_t n = counts[ci] * (size_t)P;   /* divisible by P: reduce_scatter blocks */
        char *s = malloc(n * t->esz), *r = calloc(n, t->esz), *w = calloc(n, t->esz);
        fill(s, t, n, 1234u + 77u * (unsigned)rank + (unsigned)(ti * 131 + oi * 17 + ci));
        int *rc = malloc(sizeof(int) * (size_t)P);
        for (int k = 0; k < P; k++) rc[k] = (int)(n / (size_t)P);
        for (int which = 0; which < 6; which++) {
          int e = 0, ew = MPI_SUCCESS;
          size_t on = n;
          memset(r, 0, n * t->esz);
          memset(w, 0, n * t->esz);
          switch (which) {
            case 0: e = allreduce_bine_bdw_remap(s, r, n, t->dt, o->op, MPI_COMM_WORLD); break;
            case 1: e = allreduce_bine_lat(s, r, n, t->dt, o->op, MPI_COMM_WORLD); break;
            case 2: e = allreduce_ring(s, r, n, t->dt, o->op, MPI_COMM_WORLD); break;
            case 3: e = reduce_scatter_bine_permute_remap(s, r, rc, t->dt, o->op, MPI_COMM_WORLD); on = (size_t)rc[rank]; break;
            case 4: e = reduce_scatter_bine_block_by_block(s, r, rc, t->dt, o->op, MPI_COMM_WORLD); on = (size_t)rc[rank]; break;
            default: e = reduce_bine_bdw(s, rank == 0 ? r : NULL, n, t->dt, o->op, 0, MPI_COMM_WORLD);
                     on = rank == 0 ? n : 0;
          }
          if (which <= 2) ew = PMPI_Allreduce(s, w, (int)n, t->dt, o->op, MPI_COMM_WORLD);
          else if (which <= 4) ew = PMPI_Reduce_scatter(s, w, rc, t->dt, o->op, MPI_COMM_WORLD);
          else ew = PMPI_Reduce(s, rank == 0 ? w : NULL, (int)n, t->dt, o->op, 0, MPI_COMM_WORLD);
          int fail;
          if (!ok_pair) fail = e != MPI_ERR_OP;         /* MPICH rejects the pair: so must the drop-in */
          else if (P == 1 && which == 4) fail = 0;      /* the reference leaves rbuf untouched there */
          else fail = e != MPI_SUCCESS || ew != MPI_SUCCESS || (on && !same(r, w, t, on));
          cases++;
          if (fail) {
            bad++;
            size_t k = 0;
            while (k < on && same((char *)r + k * t->esz, (char *)w + k * t->esz, t, 1)) k++;
            if (bad <= 40)
              fprintf(stderr, "rank %d MISMATCH %s %s n=%zu which=%d rc=%d (mpich rc %d) first bad element %zu\n",
                      rank, t->name, o->name, n, which, e, ew, k);
          }
        }
        free(s); free(r); free(w); free(rc);
      }
    }
  }
  /* bcast latency trees vs PMPI_Bcast (any type: pure data movement); the
   * root-0-only variants at root 0, the _new ones at every root */
  typedef int (*bc_fn)(void *, size_t, MPI_Datatype, int, MPI_Comm);
  const struct { const char *name; bc_fn f; int any_root; } bcs[] = {
      {"bine_lat", bcast_bine_lat, 0}, {"bine_lat_reversed", bcast_bine_lat_reversed, 0},
      {"bine_lat_new", bcast_bine_lat_new, 1}, {"bine_lat_i_new", bcast_bine_lat_i_new, 1}};
  for (size_t bi = 0; bi < sizeof bcs / sizeof *bcs; bi++)
    for (size_t ti = 0; ti < sizeof types / sizeof *types; ti++)
      for (size_t ci = 0; ci < sizeof counts / sizeof *counts; ci++)
        for (int root = 0; root < (bcs[bi].any_root ? P : 1); root++) {
          const type_t *t = &types[ti];
          const size_t n = counts[ci];
          char *r = malloc(n * t->esz), *w = malloc(n * t->esz);
          fill(r, t, n, 99u + 13u * (unsigned)rank + (unsigned)(bi * 7 + ti * 3 + ci));
          memcpy(w, r, n * t->esz);
          int e = bcs[bi].f(r, n, t->dt, root, MPI_COMM_WORLD);
          int ew = PMPI_Bcast(w, (int)n, t->dt, root, MPI_COMM_WORLD);
          cases++;
          if (e != MPI_SUCCESS || ew != MPI_SUCCESS || !same(r, w, t, n)) {
            bad++;
            if (bad <= 40)
              fprintf(stderr, "rank %d MISMATCH bcast_%s %s n=%zu root=%d rc=%d (mpich rc %d)\n", rank,
                      bcs[bi].name, t->name, n, root, e, ew);
          }
          free(r); free(w);
        }
  /* allgather (pure data movement, every type incl. the padded pairs) vs PMPI_Allgather */
  typedef int (*ag_fn)(const void *, size_t, MPI_Datatype, void *, size_t, MPI_Datatype, MPI_Comm);
  /* (the Bine allgathers return MPI_ERR_ARG at P = 1, as the reference: golden-pinned) */
  const struct { const char *name; ag_fn f; int p1; } ags[] = {
      {"ring", allgather_ring, 1}, {"bine_block_by_block", allgather_bine_block_by_block, 0},
      {"bine_permute_remap", allgather_bine_permute_remap, 0}, {"k_bruck", allgather_k_bruck, 1}};
  for (size_t ai = 0; ai < sizeof ags / sizeof *ags; ai++)
    for (size_t ti = 0; ti < sizeof types / sizeof *types; ti++)
      for (size_t ci = 0; ci < sizeof counts / sizeof *counts; ci++) {
        if (P == 1 && !ags[ai].p1) continue;
        const type_t *t = &types[ti];
        const size_t n = counts[ci];
        char *s = malloc(n * t->esz), *r = calloc(n * (size_t)P, t->esz), *w = calloc(n * (size_t)P, t->esz);
        fill(s, t, n, 555u + 31u * (unsigned)rank + (unsigned)(ai * 7 + ti * 3 + ci));
        int e = ags[ai].f(s, n, t->dt, r, n, t->dt, MPI_COMM_WORLD);
        int ew = PMPI_Allgather(s, (int)n, t->dt, w, (int)n, t->dt, MPI_COMM_WORLD);
        cases++;
        if (e != MPI_SUCCESS || ew != MPI_SUCCESS || !same(r, w, t, n * (size_t)P)) {
          bad++;
          if (bad <= 40)
            fprintf(stderr, "rank %d MISMATCH allgather_%s %s n=%zu rc=%d (mpich rc %d)\n", rank, ags[ai].name,
                    t->name, n, e, ew);
        }
        free(s); free(r); free(w);
      }
  /* gather_bine / scatter_bine / alltoall_bine (whole blocks, every type) vs
   * PMPI_Gather / PMPI_Scatter / PMPI_Alltoall, at root 0 and P / 2 (even, or
   * P = 2: roots the reference serves); the root-only buffers NULL elsewhere,
   * as pico_core passes them (pico_core_gather_utils.c, _scatter_utils.c) */
  for (int which = 0; which < 3; which++)
    for (size_t ti = 0; ti < sizeof types / sizeof *types; ti++)
      for (size_t ci = 0; ci < sizeof counts / sizeof *counts; ci++)
        for (int ri = 0; ri < (which == 2 || P == 1 ? 1 : 2); ri++) {
          const type_t *t = &types[ti];
          const size_t n = counts[ci], all = n * (size_t)P;
          const int root = ri ? P / 2 : 0;
          const size_t sn = which == 0 ? n : all, rn = which == 1 ? n : all;
          char *s = malloc(sn * t->esz), *r = calloc(rn, t->esz), *w = calloc(rn, t->esz);
          fill(s, t, sn, 777u + 29u * (unsigned)rank + (unsigned)(which * 11 + ti * 3 + ci));
          int e, ew;
          size_t on = rn;
          if (which == 0) {
            e = gather_bine(s, n, t->dt, rank == root ? r : NULL, n, t->dt, root, MPI_COMM_WORLD);
            ew = PMPI_Gather(s, (int)n, t->dt, rank == root ? w : NULL, (int)n, t->dt, root, MPI_COMM_WORLD);
            if (rank != root) on = 0;
          } else if (which == 1) {
            e = scatter_bine(rank == root ? s : NULL, n, t->dt, r, n, t->dt, root, MPI_COMM_WORLD);
            ew = PMPI_Scatter(rank == root ? s : NULL, (int)n, t->dt, w, (int)n, t->dt, root, MPI_COMM_WORLD);
          } else {
            e = alltoall_bine(s, n, t->dt, r, n, t->dt, MPI_COMM_WORLD);
            ew = PMPI_Alltoall(s, (int)n, t->dt, w, (int)n, t->dt, MPI_COMM_WORLD);
          }
          cases++;
          if (e != MPI_SUCCESS || ew != MPI_SUCCESS || (on && !same(r, w, t, on))) {
            bad++;
            if (bad <= 40)
              fprintf(stderr, "rank %d MISMATCH %s %s n=%zu root=%d rc=%d (mpich rc %d)\n", rank,
                      which == 0 ? "gather_bine" : which == 1 ? "scatter_bine" : "alltoall_bine", t->name, n, root,
                      e, ew);
          }
          free(s); free(r); free(w);
        }
  int tot = 0;
  MPI_Allreduce(&bad, &tot, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
  if (rank == 0) printf(tot ? "OPCHECK FAILED %d of %d\n" : "OPCHECK ok %d cases\n", tot ? tot : cases, cases);
  MPI_Finalize();
  return tot ? 1 : 0;
}
