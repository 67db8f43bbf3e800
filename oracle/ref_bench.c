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
 *   ref_bench allreduce <algo> <N> <iters>
 *       every rank fills N floats (seed 1234 + rank, pico_core_utils.c:902-923)
 *       and calls allreduce_<algo> <iters> times; per iteration the time is
 *       the max over ranks (pico_core.c:133-140), the statistic the median
 *       after dropping the first 20 % (plot/summarize_data.py:24-48).  Also
 *       prints the bine_checksum digest of rank 0's output, so bench.py can
 *       compare the REAL reference's result with the GPU's in the same run.
 * Prints one JSON object on rank 0.
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libbine.h"

typedef int (*ar_fn)(const void *, void *, size_t, MPI_Datatype, MPI_Op, MPI_Comm);

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
    if (!rank) fprintf(stderr, "usage: ref_bench reduce_local N budget_s | allreduce algo N iters\n");
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
  } else if (!strcmp(argv[1], "allreduce") && argc >= 5) {
    ar_fn f = pick_allreduce(argv[2]);
    size_t N = (size_t)strtoull(argv[3], NULL, 10);
    int iters = atoi(argv[4]);
    if (!f || iters < 1) MPI_Abort(MPI_COMM_WORLD, 4);
    float *sb = malloc(N * sizeof(float)), *rb = malloc(N * sizeof(float));
    if (!sb || !rb) MPI_Abort(MPI_COMM_WORLD, 3);
    fill_float(sb, N, 1234u + (unsigned)rank);
    memset(rb, 0, N * sizeof(float));
    double *t = malloc(sizeof(double) * (size_t)iters);
    int rc = MPI_SUCCESS;
    for (int i = 0; i < iters; i++) {
      MPI_Barrier(MPI_COMM_WORLD);
      double t0 = MPI_Wtime();
      int r = f(sb, rb, N, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
      double dt = MPI_Wtime() - t0;
      if (r != MPI_SUCCESS) rc = r;
      MPI_Allreduce(MPI_IN_PLACE, &dt, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
      t[i] = dt;
    }
    int skip = iters / 5, m = iters - skip;
    qsort(t + skip, (size_t)m, sizeof(double), cmp_double);
    double med = (m % 2) ? t[skip + m / 2] : 0.5 * (t[skip + m / 2 - 1] + t[skip + m / 2]);
    if (rank == 0)
      printf("{\"mode\": \"allreduce\", \"algo\": \"%s\", \"P\": %d, \"N\": %zu, \"iters\": %d, "
             "\"median_s\": %.9f, \"rc\": %d, \"digest\": \"%llu\"}\n", argv[2], P, N, iters, med, rc,
             (unsigned long long)digest32(rb, N));
    free(sb); free(rb); free(t);
  } else {
    if (!rank) fprintf(stderr, "unknown mode %s\n", argv[1]);
    MPI_Abort(MPI_COMM_WORLD, 5);
  }
  MPI_Finalize();
  return 0;
}
