/*
 * ref_bench.c -- CPU timing harness for the REAL reference libbine.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY.  Used solely by bench.py's cpu_baseline
 * leg (kind "reference"); never part of the product path.  Linked against
 * oracle/_ref/libbine_ref.so, which oracle/Makefile (target `ref`) compiles
 * from the reference sources where they lie, against the image's MPICH 3.3.2
 * (/opt/conda) -- the MPI whose MPI_Reduce_local is libbine's arithmetic
 * (SURVEY.md 8(a) A1).  The built binary travels to the GPU box with the tree;
 * the reference sources do not.
 *
 * usage (under mpiexec -n P):
 *   ref_bench reduce_local <N> <budget_s>
 *       rank 0 times MPI_Reduce_local(in, inout, N, MPI_FLOAT, MPI_SUM) -- the
 *       call libbine makes per step (e.g. libbine_allreduce.c:888) -- on
 *       pico_core's input distribution, as many calls as fit in budget_s.
 *   ref_bench allreduce <algo> <N> <iters> [float|double|int64]
 *       every rank fills N elements (seed 1234 + rank, pico_core_utils.c:
 *       902-923) and calls allreduce_<algo> <iters> times; per iteration the
 *       time is the max over ranks (pico_core.c:133-140), the statistic the
 *       median after dropping the first 20 % (plot/summarize_data.py:24-48).
 *       Also prints the bine_checksum digest of rank 0's output, so bench.py
 *       can compare the REAL reference's result with the GPU's and the
 *       oracle's in the same run.
 *   ref_bench reduce_scatter <algo> <N> <iters>
 *       the same for reduce_scatter_<algo> on N floats per rank, N / P to
 *       every rank (BASELINE config C4's shape); digest of rank 0's block.
 * Prints one JSON object on rank 0.
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libbine.h"

typedef int (*ar_fn)(const void *, void *, size_t, MPI_Datatype, MPI_Op, MPI_Comm);

typedef int (*rs_fn)(const void *, void *, const int[], MPI_Datatype, MPI_Op, MPI_Comm);

static rs_fn pick_reduce_scatter(const char *a) {
  if (!strcmp(a, "bine_permute_remap")) return reduce_scatter_bine_permute_remap;
  if (!strcmp(a, "bine_send_remap")) return reduce_scatter_bine_send_remap;
  if (!strcmp(a, "bine_static")) return reduce_scatter_bine_static;
  if (!strcmp(a, "ring")) return reduce_scatter_ring;
  return NULL;
}

static ar_fn pick_allreduce(const char *a) {
  if (!strcmp(a, "bine_bdw_remap")) return allreduce_bine_bdw_remap;
  if (!strcmp(a, "bine_bdw_static")) return allreduce_bine_bdw_static;
  if (!strcmp(a, "bine_lat")) return allreduce_bine_lat;
  if (!strcmp(a, "ring")) return allreduce_ring;
  if (!strcmp(a, "rabenseifner")) return allreduce_rabenseifner;
  return NULL;
}

/* pico_core's float distribution (pico_core_utils.c:911), glibc rand_r */
static void fill_float(float *buf, size_t n, unsigned int seed) {
  for (size_t i = 0; i < n; i++) buf[i] = (float)rand_r(&seed) / (float)RAND_MAX * 100.0f;
}

/* pico_core's double and int64 distributions (pico_core_utils.c:902-923);
 * the int64's high word drawn first */
static void fill_double(double *buf, size_t n, unsigned int seed) {
  for (size_t i = 0; i < n; i++) buf[i] = (double)rand_r(&seed) / (double)RAND_MAX * 100.0;
}
static void fill_int64(int64_t *buf, size_t n, unsigned int seed) {
  for (size_t i = 0; i < n; i++) {
    const int64_t hi = (int64_t)rand_r(&seed) << 32;
    buf[i] = hi | rand_r(&seed);
  }
}

/* bine_checksum's digest (include/bine_amd.h) of n 32-bit words */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint64_t digest32(const void *buf, size_t n) {
  const uint32_t *w = (const uint32_t *)buf;
  uint64_t acc = 0;
  for (size_t i = 0; i < n; i++) acc += mix64((uint64_t)w[i] + (uint64_t)i * 0x9E3779B97F4A7C15ull);
  return acc;
}

/* ... and of n 64-bit words */
static uint64_t digest64(const void *buf, size_t n) {
  const uint64_t *w = (const uint64_t *)buf;
  uint64_t acc = 0;
  for (size_t i = 0; i < n; i++) acc += mix64(w[i] + (uint64_t)i * 0x9E3779B97F4A7C15ull);
  return acc;
}

static int cmp_double(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return (x > y) - (x < y);
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, P;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  if (argc < 4) {
    if (!rank) fprintf(stderr, "usage: ref_bench reduce_local N budget_s | allreduce algo N iters [dtype] | "
                             "reduce_scatter algo N iters\n");
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  if (!strcmp(argv[1], "reduce_local")) {
    size_t N = (size_t)strtoull(argv[2], NULL, 10);
    double budget = atof(argv[3]);
    if (rank == 0) {
      float *in = malloc(N * sizeof(float)), *io = malloc(N * sizeof(float));
      if (!in || !io) MPI_Abort(MPI_COMM_WORLD, 3);
      fill_float(in, N, 1234);
      fill_float(io, N, 1235);
      MPI_Reduce_local(in, io, (int)N, MPI_FLOAT, MPI_SUM); /* warm */
      int calls = 0;
      double t0 = MPI_Wtime(), el = 0;
      do {
        MPI_Reduce_local(in, io, (int)N, MPI_FLOAT, MPI_SUM);
        calls++;
        el = MPI_Wtime() - t0;
      } while (el < budget && calls < 100000);
      double sum = 0;
      for (size_t i = 0; i < N; i += 4099) sum += io[i];
      printf("{\"mode\": \"reduce_local\", \"N\": %zu, \"calls\": %d, \"seconds\": %.6f, "
             "\"s_per_call\": %.9f, \"checksum\": %.6e}\n", N, calls, el, el / calls, sum);
      free(in); free(io);
    }
  } else if ((!strcmp(argv[1], "allreduce") || !strcmp(argv[1], "reduce_scatter")) && argc >= 5) {
    const int rs = !strcmp(argv[1], "reduce_scatter");
    ar_fn f = rs ? NULL : pick_allreduce(argv[2]);
    rs_fn g = rs ? pick_reduce_scatter(argv[2]) : NULL;
    size_t N = (size_t)strtoull(argv[3], NULL, 10);
    int iters = atoi(argv[4]);
    const char *tn = argc >= 6 ? argv[5] : "float";
    MPI_Datatype dt = !strcmp(tn, "double") ? MPI_DOUBLE : !strcmp(tn, "int64") ? MPI_INT64_T : MPI_FLOAT;
    const size_t esz = dt == MPI_FLOAT ? 4 : 8;
    if ((!f && !g) || iters < 1 || (rs && (dt != MPI_FLOAT || N % (size_t)P))) MPI_Abort(MPI_COMM_WORLD, 4);
    const size_t nout = rs ? N / (size_t)P : N;
    void *sb = malloc(N * esz), *rb = malloc(nout * esz);
    int *rcounts = malloc(sizeof(int) * (size_t)P);
    if (!sb || !rb || !rcounts) MPI_Abort(MPI_COMM_WORLD, 3);
    for (int k = 0; k < P; k++) rcounts[k] = (int)(N / (size_t)P);
    if (dt == MPI_FLOAT) fill_float(sb, N, 1234u + (unsigned)rank);
    else if (dt == MPI_DOUBLE) fill_double(sb, N, 1234u + (unsigned)rank);
    else fill_int64(sb, N, 1234u + (unsigned)rank);
    memset(rb, 0, nout * esz);
    double *t = malloc(sizeof(double) * (size_t)iters);
    int rc = MPI_SUCCESS;
    for (int i = 0; i < iters; i++) {
      MPI_Barrier(MPI_COMM_WORLD);
      double t0 = MPI_Wtime();
      int r = rs ? g(sb, rb, rcounts, dt, MPI_SUM, MPI_COMM_WORLD) : f(sb, rb, N, dt, MPI_SUM, MPI_COMM_WORLD);
      double dtm = MPI_Wtime() - t0;
      if (r != MPI_SUCCESS) rc = r;
      MPI_Allreduce(MPI_IN_PLACE, &dtm, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
      t[i] = dtm;
    }
    int skip = iters / 5, m = iters - skip;
    qsort(t + skip, (size_t)m, sizeof(double), cmp_double);
    double med = (m % 2) ? t[skip + m / 2] : 0.5 * (t[skip + m / 2 - 1] + t[skip + m / 2]);
    if (rank == 0)
      printf("{\"mode\": \"%s\", \"algo\": \"%s\", \"dtype\": \"%s\", \"P\": %d, \"N\": %zu, "
             "\"iters\": %d, \"median_s\": %.9f, \"rc\": %d, \"digest\": \"%llu\"}\n", argv[1], argv[2], tn, P,
             N, iters, med, rc, (unsigned long long)(esz == 4 ? digest32(rb, nout) : digest64(rb, nout)));
    free(sb); free(rb); free(t); free(rcounts);
  } else {
    if (!rank) fprintf(stderr, "unknown mode %s\n", argv[1]);
    MPI_Abort(MPI_COMM_WORLD, 5);
  }
  MPI_Finalize();
  return 0;
}
