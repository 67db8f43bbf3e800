/*
 * ref_golden.c -- golden-vector capture harness for the REAL reference libbine.
 *
 * TEST INFRASTRUCTURE ONLY.  This program is never shipped and never part of
 * the product path.  It is linked against oracle/_ref/libbine_ref.so, which
 * oracle/Makefile (target `ref`) compiles directly from the reference sources
 * where they lie (/root/reference/libbine/{libbine_allreduce,
 * libbine_reduce_scatter,libbine_reduce,libbine_utils_bitmaps}.c) against the
 * image's MPICH 3.3.2 (/opt/conda).  Run under mpiexec -n P by
 * tools/make_golden.py, it fills each rank's send buffer with pico_core's own
 * distributions (pico_core/pico_core_utils.c:883-928, seed = base + rank instead
 * of time(NULL) + rank so that the vectors are reproducible), calls one libbine
 * entry point (include/libbine.h:30-78) and dumps per-rank input digest, output
 * and return code.
 *
 * usage: ref_golden <outdir> <coll> <algo> <op> <segsize> <rcounts_kind>
 *                   <seed_base> <dtype,dtype,...> <N,N,...>
 *   coll         allreduce | reduce_scatter | reduce | allgather | bcast | fill (dump the inputs)
 *                bcast: in place on each rank's input; rcounts "root<k>" = root k
 *                allgather: N = elements per rank (scount = rcount, same type,
 *                "_inplace": MPI_IN_PLACE, the own block at block `rank` of rbuf;
 *                pico_core_utils.c:511-514), rbuf = P * N zeroed elements
 *                gather / scatter: N = elements per block, root from "root<k>"
 *                (else 0); gather: sbuf N, rbuf P * N on the root only (NULL
 *                elsewhere, as pico_core passes it); scatter: sbuf P * N on the
 *                root only, rbuf N; alltoall: sbuf and rbuf P * N
 *   rcounts_kind even   -> rcounts[i] = N / P  (pico_core_utils.c:535-536)
 *                ragged -> rcounts[i] = N / P + (i % 3)   (exercises displs)
 *                an "_inplace" suffix calls with MPI_IN_PLACE: the input is
 *                copied into rbuf first (reduce: at the root; reduce_scatter:
 *                the whole input, the result read from the start of rbuf)
 *                a "_sparse" suffix (e.g. even_sparse) post-processes the
 *                inputs so that the logical ops and MAX / MIN see zeros, -0.0
 *                and NaN (sparsify() below; tests/golden_util.py repeats it)
 */
#include <math.h>
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libbine.h"

typedef int (*ar_fn)(const void *, void *, size_t, MPI_Datatype, MPI_Op, MPI_Comm);
typedef int (*rs_fn)(const void *, void *, const int *, MPI_Datatype, MPI_Op, MPI_Comm);
typedef int (*rd_fn)(const void *, void *, size_t, MPI_Datatype, MPI_Op, int, MPI_Comm);
typedef int (*ag_fn)(const void *, size_t, MPI_Datatype, void *, size_t, MPI_Datatype, MPI_Comm);
typedef int (*bc_fn)(void *, size_t, MPI_Datatype, int, MPI_Comm);

static ar_fn pick_allreduce(const char *a) {
  if (!strcmp(a, "recursivedoubling")) return allreduce_recursivedoubling;
  if (!strcmp(a, "ring")) return allreduce_ring;
  if (!strcmp(a, "rabenseifner")) return allreduce_rabenseifner;
  if (!strcmp(a, "bine_lat")) return allreduce_bine_lat;
  if (!strcmp(a, "bine_bdw_static")) return allreduce_bine_bdw_static;
  if (!strcmp(a, "bine_bdw_remap")) return allreduce_bine_bdw_remap;
  if (!strcmp(a, "bine_bdw_remap_segmented")) return allreduce_bine_bdw_remap_segmented;
  if (!strcmp(a, "bine_block_by_block_any_even")) return allreduce_bine_block_by_block_any_even;
  return NULL;
}

static rs_fn pick_reduce_scatter(const char *a) {
  if (!strcmp(a, "recursivehalving")) return reduce_scatter_recursivehalving;
  if (!strcmp(a, "recursive_distance_doubling")) return reduce_scatter_recursive_distance_doubling;
  if (!strcmp(a, "ring")) return reduce_scatter_ring;
  if (!strcmp(a, "butterfly")) return reduce_scatter_butterfly;
  if (!strcmp(a, "bine_static")) return reduce_scatter_bine_static;
  if (!strcmp(a, "bine_send_remap")) return reduce_scatter_bine_send_remap;
  if (!strcmp(a, "bine_permute_remap")) return reduce_scatter_bine_permute_remap;
  if (!strcmp(a, "bine_block_by_block")) return reduce_scatter_bine_block_by_block;
  if (!strcmp(a, "bine_block_by_block_any_even")) return reduce_scatter_bine_block_by_block_any_even;
  return NULL;
}

static rd_fn pick_reduce(const char *a) {
  if (!strcmp(a, "bine_lat")) return reduce_bine_lat;
  if (!strcmp(a, "bine_bdw")) return reduce_bine_bdw;
  return NULL;
}

static bc_fn pick_bcast(const char *a) {
  if (!strcmp(a, "bine_lat")) return bcast_bine_lat;
  if (!strcmp(a, "bine_lat_reversed")) return bcast_bine_lat_reversed;
  if (!strcmp(a, "bine_lat_new")) return bcast_bine_lat_new;
  if (!strcmp(a, "bine_lat_i_new")) return bcast_bine_lat_i_new;
  if (!strcmp(a, "scatter_allgather")) return bcast_scatter_allgather;
  if (!strcmp(a, "bine_bdw_static")) return bcast_bine_bdw_static;
  if (!strcmp(a, "bine_bdw_remap")) return bcast_bine_bdw_remap;
  return NULL;
}

static ag_fn pick_allgather(const char *a) {
  if (!strcmp(a, "recursivedoubling")) return allgather_recursivedoubling;
  if (!strcmp(a, "k_bruck")) return allgather_k_bruck;
  if (!strcmp(a, "ring")) return allgather_ring;
  if (!strcmp(a, "sparbit")) return allgather_sparbit;
  if (!strcmp(a, "bine_block_by_block")) return allgather_bine_block_by_block;
  if (!strcmp(a, "bine_block_by_block_any_even")) return allgather_bine_block_by_block_any_even;
  if (!strcmp(a, "bine_permute_static")) return allgather_bine_permute_static;
  if (!strcmp(a, "bine_send_static")) return allgather_bine_send_static;
  if (!strcmp(a, "bine_permute_remap")) return allgather_bine_permute_remap;
  if (!strcmp(a, "bine_send_remap")) return allgather_bine_send_remap;
  if (!strcmp(a, "bine_2_blocks")) return allgather_bine_2_blocks;
  if (!strcmp(a, "bine_2_blocks_dtype")) return allgather_bine_2_blocks_dtype;
  return NULL;
}

/* MPI's {value; int index} pair types, C layout */
typedef struct { float v; int i; } p_float_int;
typedef struct { double v; int i; } p_double_int;
typedef struct { long v; int i; } p_long_int;
typedef struct { int v; int i; } p_2int;
typedef struct { short v; int i; } p_short_int;

static int dtype_of(const char *s, MPI_Datatype *dt, size_t *sz) {
  if (!strcmp(s, "float"))  { *dt = MPI_FLOAT;         *sz = 4; return 0; }
  if (!strcmp(s, "double")) { *dt = MPI_DOUBLE;        *sz = 8; return 0; }
  if (!strcmp(s, "int8"))   { *dt = MPI_INT8_T;        *sz = 1; return 0; }
  if (!strcmp(s, "int16"))  { *dt = MPI_INT16_T;       *sz = 2; return 0; }
  if (!strcmp(s, "int32"))  { *dt = MPI_INT32_T;       *sz = 4; return 0; }
  if (!strcmp(s, "int64"))  { *dt = MPI_INT64_T;       *sz = 8; return 0; }
  if (!strcmp(s, "uint8"))  { *dt = MPI_UNSIGNED_CHAR; *sz = 1; return 0; }
  if (!strcmp(s, "float_int"))  { *dt = MPI_FLOAT_INT;  *sz = sizeof(p_float_int); return 0; }
  if (!strcmp(s, "double_int")) { *dt = MPI_DOUBLE_INT; *sz = sizeof(p_double_int); return 0; }
  if (!strcmp(s, "long_int"))   { *dt = MPI_LONG_INT;   *sz = sizeof(p_long_int); return 0; }
  if (!strcmp(s, "2int"))       { *dt = MPI_2INT;       *sz = sizeof(p_2int); return 0; }
  if (!strcmp(s, "short_int"))  { *dt = MPI_SHORT_INT;  *sz = sizeof(p_short_int); return 0; }
  if (!strcmp(s, "c_float_complex"))  { *dt = MPI_C_FLOAT_COMPLEX;  *sz = 8; return 0; }
  if (!strcmp(s, "c_double_complex")) { *dt = MPI_C_DOUBLE_COMPLEX; *sz = 16; return 0; }
  return -1;
}

static int op_of(const char *s, MPI_Op *op) {
  if (!strcmp(s, "sum"))  { *op = MPI_SUM;  return 0; }
  if (!strcmp(s, "prod")) { *op = MPI_PROD; return 0; }
  if (!strcmp(s, "max"))  { *op = MPI_MAX;  return 0; }
  if (!strcmp(s, "min"))  { *op = MPI_MIN;  return 0; }
  if (!strcmp(s, "land")) { *op = MPI_LAND; return 0; }
  if (!strcmp(s, "band")) { *op = MPI_BAND; return 0; }
  if (!strcmp(s, "lor"))  { *op = MPI_LOR;  return 0; }
  if (!strcmp(s, "bor"))  { *op = MPI_BOR;  return 0; }
  if (!strcmp(s, "lxor")) { *op = MPI_LXOR; return 0; }
  if (!strcmp(s, "bxor")) { *op = MPI_BXOR; return 0; }
  if (!strcmp(s, "maxloc")) { *op = MPI_MAXLOC; return 0; }
  if (!strcmp(s, "minloc")) { *op = MPI_MINLOC; return 0; }
  return -1;
}

/* pico_core has no generator for the pair types: value = rand_r() % 16
 * (halved for floating values: ties and fractions), index = rand_r() % 1000,
 * padding 0 (the oracle's orc_fill draws the same) */
#define FILL_PAIR(T, VT, HALF)                                 \
  do {                                                         \
    T *p = (T *)buf;                                           \
    memset(p, 0, n * sizeof(T));                               \
    for (size_t i = 0; i < n; i++) {                           \
      const int r = rand_r(&seed) % 16;                        \
      p[i].v = HALF ? (VT)r / (VT)2 : (VT)r;                   \
      p[i].i = rand_r(&seed) % 1000;                           \
    }                                                          \
    return;                                                    \
  } while (0)

/* pico_core's generator (pico_core_utils.c:902-923), glibc rand_r. */
static void fill(void *buf, const char *dt, size_t n, unsigned int seed) {
  if (!strcmp(dt, "float_int"))  FILL_PAIR(p_float_int, float, 1);
  if (!strcmp(dt, "double_int")) FILL_PAIR(p_double_int, double, 1);
  if (!strcmp(dt, "long_int"))   FILL_PAIR(p_long_int, long, 0);
  if (!strcmp(dt, "2int"))       FILL_PAIR(p_2int, int, 0);
  if (!strcmp(dt, "short_int"))  FILL_PAIR(p_short_int, short, 0);
  if (!strcmp(dt, "c_float_complex")) {   /* pico_core's fp distribution, re then im */
    for (size_t i = 0; i < 2 * n; i++) ((float *)buf)[i] = (float)rand_r(&seed) / (float)RAND_MAX * 100.0f;
    return;
  }
  if (!strcmp(dt, "c_double_complex")) {
    for (size_t i = 0; i < 2 * n; i++) ((double *)buf)[i] = (double)rand_r(&seed) / (double)RAND_MAX * 100.0;
    return;
  }
  for (size_t i = 0; i < n; i++) {
    if (!strcmp(dt, "int8"))        ((int8_t *)buf)[i] = (int8_t)((rand_r(&seed) % 256) - 128);
    else if (!strcmp(dt, "int16"))  ((int16_t *)buf)[i] = (int16_t)((rand_r(&seed) % 65536) - 32768);
    else if (!strcmp(dt, "int32"))  ((int32_t *)buf)[i] = (int32_t)rand_r(&seed);
    else if (!strcmp(dt, "int64"))  { int64_t hi = (int64_t)rand_r(&seed) << 32; ((int64_t *)buf)[i] = hi | rand_r(&seed); }
    else if (!strcmp(dt, "float"))  ((float *)buf)[i] = (float)rand_r(&seed) / (float)RAND_MAX * 100.0f;
    else if (!strcmp(dt, "double")) ((double *)buf)[i] = (double)rand_r(&seed) / (double)RAND_MAX * 100.0;
    else if (!strcmp(dt, "uint8"))  ((unsigned char *)buf)[i] = (unsigned char)(rand_r(&seed) % 256);
  }
}

/* j = i + rank: zero where j % 3 == 0; floating types also -0.0 where
 * j % 5 == 1 and NaN where j % 11 == 2 (later rules win) */
static void sparsify(void *buf, const char *dt, size_t n, int rank) {
  for (size_t i = 0; i < n; i++) {
    const size_t j = i + (size_t)rank;
    const int z = j % 3 == 0;
    if (!strcmp(dt, "int8"))        { if (z) ((int8_t *)buf)[i] = 0; }
    else if (!strcmp(dt, "int16"))  { if (z) ((int16_t *)buf)[i] = 0; }
    else if (!strcmp(dt, "int32"))  { if (z) ((int32_t *)buf)[i] = 0; }
    else if (!strcmp(dt, "int64"))  { if (z) ((int64_t *)buf)[i] = 0; }
    else if (!strcmp(dt, "uint8"))  { if (z) ((unsigned char *)buf)[i] = 0; }
    else if (!strcmp(dt, "float")) {
      float *f = (float *)buf;
      if (z) f[i] = 0.0f;
      if (j % 5 == 1) f[i] = -0.0f;
      if (j % 11 == 2) f[i] = NAN;
    } else if (!strcmp(dt, "double")) {
      double *f = (double *)buf;
      if (z) f[i] = 0.0;
      if (j % 5 == 1) f[i] = -0.0;
      if (j % 11 == 2) f[i] = NAN;
    } else if (!strcmp(dt, "float_int")) {
      p_float_int *f = (p_float_int *)buf;
      if (z) f[i].v = 0.0f;
      if (j % 5 == 1) f[i].v = -0.0f;
      if (j % 11 == 2) f[i].v = NAN;
    } else if (!strcmp(dt, "double_int")) {
      p_double_int *f = (p_double_int *)buf;
      if (z) f[i].v = 0.0;
      if (j % 5 == 1) f[i].v = -0.0;
      if (j % 11 == 2) f[i].v = NAN;
    } else if (!strcmp(dt, "long_int"))  { if (z) ((p_long_int *)buf)[i].v = 0; }
    else if (!strcmp(dt, "2int"))        { if (z) ((p_2int *)buf)[i].v = 0; }
    else if (!strcmp(dt, "short_int"))   { if (z) ((p_short_int *)buf)[i].v = 0; }
    else if (!strcmp(dt, "c_float_complex")) {
      float *f = (float *)buf + 2 * i;
      if (z) f[0] = f[1] = 0.0f;
      if (j % 5 == 1) f[0] = -0.0f;
      if (j % 7 == 3) f[1] = -0.0f;
    } else if (!strcmp(dt, "c_double_complex")) {
      double *f = (double *)buf + 2 * i;
      if (z) f[0] = f[1] = 0.0;
      if (j % 5 == 1) f[0] = -0.0;
      if (j % 7 == 3) f[1] = -0.0;
    }
  }
}

static int split_csv(char *s, char **out, int max) {
  int n = 0;
  for (char *tok = strtok(s, ","); tok && n < max; tok = strtok(NULL, ",")) out[n++] = tok;
  return n;
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, P;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  if (argc != 10) {
    if (!rank) fprintf(stderr, "bad args\n");
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  const char *outdir = argv[1], *coll = argv[2], *algo = argv[3], *ops = argv[4];
  size_t segsize = (size_t)strtoull(argv[5], NULL, 10);
  const char *rk = argv[6];
  unsigned seed_base = (unsigned)strtoul(argv[7], NULL, 10);
  char *dts[16], *ns[32];
  int ndt = split_csv(argv[8], dts, 16);
  int nn = split_csv(argv[9], ns, 32);
  MPI_Op op;
  if (op_of(ops, &op)) MPI_Abort(MPI_COMM_WORLD, 3);
  const int inplace = strstr(rk, "_inplace") != NULL;
  bine_allreduce_segsize = segsize;

  for (int d = 0; d < ndt; d++) {
    MPI_Datatype dt; size_t esz;
    if (dtype_of(dts[d], &dt, &esz)) MPI_Abort(MPI_COMM_WORLD, 4);
    for (int k = 0; k < nn; k++) {
      size_t N = (size_t)strtoull(ns[k], NULL, 10);
      int *rcounts = (int *)malloc(sizeof(int) * (size_t)P);
      size_t total = N, outn = N;
      if (!strcmp(coll, "reduce_scatter")) {
        total = 0;
        for (int i = 0; i < P; i++) {
          rcounts[i] = (int)(N / (size_t)P) + (!strcmp(rk, "ragged") ? (i % 3) : 0);
          total += (size_t)rcounts[i];
        }
        outn = (size_t)rcounts[rank];
      }
      const int root = !strncmp(rk, "root", 4) ? atoi(rk + 4) : 0;
      if (!strcmp(coll, "allgather") || !strcmp(coll, "alltoall")) outn = N * (size_t)P;
      if (!strcmp(coll, "alltoall") || !strcmp(coll, "scatter")) total = N * (size_t)P;
      if (!strcmp(coll, "gather")) outn = rank == root ? N * (size_t)P : 0;
      void *sbuf = malloc(total * esz + 16);
      void *rbuf = calloc(outn * esz + total * esz + 16, 1);
      fill(sbuf, dts[d], total, seed_base + (unsigned)rank);
      if (strstr(rk, "_sparse")) sparsify(sbuf, dts[d], total, rank);
      int ret = -12345;
      if (!strcmp(coll, "fill")) {           /* pins the input generator itself */
        memcpy(rbuf, sbuf, total * esz);
        ret = 0;
      } else if (!strcmp(coll, "allreduce")) {
        ar_fn f = pick_allreduce(algo);
        if (!f) MPI_Abort(MPI_COMM_WORLD, 5);
        if (inplace) memcpy(rbuf, sbuf, total * esz);
        ret = f(inplace ? MPI_IN_PLACE : sbuf, rbuf, N, dt, op, MPI_COMM_WORLD);
      } else if (!strcmp(coll, "reduce_scatter")) {
        rs_fn f = pick_reduce_scatter(algo);
        if (!f) MPI_Abort(MPI_COMM_WORLD, 5);
        if (inplace) memcpy(rbuf, sbuf, total * esz);
        ret = f(inplace ? MPI_IN_PLACE : sbuf, rbuf, rcounts, dt, op, MPI_COMM_WORLD);
      } else if (!strcmp(coll, "allgather")) {
        ag_fn f = pick_allgather(algo);
        if (!f) MPI_Abort(MPI_COMM_WORLD, 5);
        /* MPI_IN_PLACE: the rank's own block already at block `rank` of rbuf */
        if (inplace) memcpy((char *)rbuf + (size_t)rank * N * esz, sbuf, N * esz);
        ret = f(inplace ? MPI_IN_PLACE : sbuf, N, dt, rbuf, N, dt, MPI_COMM_WORLD);
      } else if (!strcmp(coll, "bcast")) {
        /* in place on every rank's own input; root from "root<k>" (else 0) */
        bc_fn f = pick_bcast(algo);
        if (!f) MPI_Abort(MPI_COMM_WORLD, 5);
        memcpy(rbuf, sbuf, total * esz);
        ret = f(rbuf, N, dt, root, MPI_COMM_WORLD);
      } else if (!strcmp(coll, "gather")) {
        /* pico_core: rbuf only on the root (pico_core_gather_utils.c) */
        ret = gather_bine(sbuf, N, dt, rank == root ? rbuf : NULL, N, dt, root, MPI_COMM_WORLD);
      } else if (!strcmp(coll, "scatter")) {
        /* pico_core: sbuf only on the root (pico_core_scatter_utils.c) */
        ret = scatter_bine(rank == root ? sbuf : NULL, N, dt, rbuf, N, dt, root, MPI_COMM_WORLD);
      } else if (!strcmp(coll, "alltoall")) {
        ret = alltoall_bine(sbuf, N, dt, rbuf, N, dt, MPI_COMM_WORLD);
      } else if (!strcmp(coll, "reduce")) {
        rd_fn f = pick_reduce(algo);
        if (!f) MPI_Abort(MPI_COMM_WORLD, 5);
        /* pico_core passes rbuf = NULL on non-roots (pico_core_reduce_utils.c:24-31) */
        if (inplace && rank == 0) memcpy(rbuf, sbuf, total * esz);
        ret = f(inplace && rank == 0 ? MPI_IN_PLACE : sbuf, rank == 0 ? rbuf : NULL, N, dt, op, 0, MPI_COMM_WORLD);
        if (rank != 0) outn = 0;
      } else {
        MPI_Abort(MPI_COMM_WORLD, 6);
      }
      /* pair types: MPICH moves only the type map's bytes, so the padding of
       * the output holds whatever the buffers held -- zero it (the tests compare
       * the defined bytes) */
      if (outn && (!strcmp(dts[d], "double_int") || !strcmp(dts[d], "long_int")))
        for (size_t k = 0; k < outn; k++) memset((char *)rbuf + k * esz + 12, 0, 4);
      if (outn && !strcmp(dts[d], "short_int"))
        for (size_t k = 0; k < outn; k++) memset((char *)rbuf + k * esz + 2, 0, 2);
      char path[1024];
      snprintf(path, sizeof path, "%s/%s.N%zu.r%d.bin", outdir, dts[d], N, rank);
      FILE *fp = fopen(path, "wb");
      if (!fp) MPI_Abort(MPI_COMM_WORLD, 7);
      int64_t hdr[2] = {ret, (int64_t)outn};
      fwrite(hdr, sizeof hdr, 1, fp);
      if (outn) fwrite(rbuf, esz, outn, fp);
      fclose(fp);
      free(sbuf); free(rbuf); free(rcounts);
      MPI_Barrier(MPI_COMM_WORLD);
    }
  }
  MPI_Finalize();
  return 0;
}
