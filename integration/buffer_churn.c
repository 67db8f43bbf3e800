/*
 * buffer_churn.c -- libbine.so's host staging under buffer churn and mixed
 * buffer placement, checked against MPICH's own collectives the way pico_core
 * checks its runs (pico_core_utils.c:553-610: exact for integers; the float
 * inputs here are multiples of 1/4 below 8 in magnitude, so every partial sum
 * of up to 8 of them is exact whatever the order, and the check is exact too).
 *
 *  1. churn: allreduce_bine_bdw_remap on 64 MiB malloc
 *     buffers, free them, malloc the same sizes again (glibc maps them at the
 *     same addresses; reported), write new data, call again -- in and out of
 *     place, float and int64.  After every call the caller's buffers must not
 *     be left page-locked by the library (hipPointerGetAttributes: not a
 *     registered host range), since nothing of the call may outlive it.
 *  2. mixed placement (P >= 2): rank 0's buffers on the device (hipMalloc),
 *     the other ranks' on the host, in ONE call -- allreduce_bine_bdw_remap
 *     and reduce_scatter_bine_permute_remap, float and int64, sizes on both
 *     sides of the shim's pipelining threshold: every rank must issue the same
 *     schedule whatever its buffers are (a rank-dependent choice hangs or
 *     pairs the wrong messages).
 *   usage: mpiexec -n P buffer_churn     (prints "CHURN ok <cases>" on rank 0)
 */
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libbine_amd.h"

static int rank, size, fails, cases;

static void fill(void *b, MPI_Datatype dt, size_t n, unsigned seed) {
  for (size_t k = 0; k < n; k++) {
    seed = seed * 1103515245u + 12345u;
    const int v = (int)((seed >> 8) % 61) - 30;  /* -30 .. 30 */
    if (dt == MPI_FLOAT) ((float *)b)[k] = (float)v * 0.25f;
    else ((int64_t *)b)[k] = (int64_t)v * 1000003 + (int64_t)seed;
  }
}

static int registered(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return a.type == hipMemoryTypeHost;
}

static void report(const char *what, int ok) {
  int all = 0;
  cases++;
  MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
  if (!all) fails++;
  if (rank == 0) printf("%s: %s\n", what, all ? "ok" : "FAILED");
  fflush(stdout);
}

/* one allreduce vs PMPI_Allreduce; dev: this rank's buffers live on the device */
static void check_allreduce(const char *tag, MPI_Datatype dt, size_t n, int in_place, int dev, unsigned seed,
                            void **keep_s, void **keep_r) {
  const size_t esz = dt == MPI_FLOAT ? 4 : 8, bytes = n * esz;
  void *hs = malloc(bytes), *want = malloc(bytes), *got = malloc(bytes);
  fill(hs, dt, n, seed + 7919u * (unsigned)rank);
  PMPI_Allreduce(hs, want, (int)n, dt, MPI_SUM, MPI_COMM_WORLD);
  void *s = NULL, *r = NULL;
  if (dev) {
    if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&r, bytes) != hipSuccess) { report(tag, 0); return; }
    (void)hipMemcpy(in_place ? r : s, hs, bytes, hipMemcpyHostToDevice);
  } else {
    s = keep_s && *keep_s ? *keep_s : malloc(bytes);
    r = keep_r && *keep_r ? *keep_r : malloc(bytes);
    memcpy(in_place ? r : s, hs, bytes);
  }
  const int e = allreduce_bine_bdw_remap(in_place ? MPI_IN_PLACE : s, r, n, dt, MPI_SUM, MPI_COMM_WORLD);
  if (dev) (void)hipMemcpy(got, r, bytes, hipMemcpyDeviceToHost);
  else memcpy(got, r, bytes);
  int ok = e == MPI_SUCCESS && memcmp(got, want, bytes) == 0;
  if (!dev && (registered(s) || registered(r))) {
    if (rank == 0) printf("  %s: a caller buffer is still page-locked after the call\n", tag);
    ok = 0;
  }
  report(tag, ok);
  if (dev) {
    (void)hipFree(s);
    (void)hipFree(r);
  } else if (keep_s) {
    *keep_s = s;
    *keep_r = r;
  } else {
    free(s);
    free(r);
  }
  free(hs);
  free(want);
  free(got);
}

static void check_reduce_scatter(const char *tag, MPI_Datatype dt, size_t block, int dev, unsigned seed) {
  const size_t esz = dt == MPI_FLOAT ? 4 : 8, total = block * (size_t)size;
  void *hs = malloc(total * esz), *want = malloc(block * esz), *got = malloc(block * esz);
  int *rc = malloc(sizeof(int) * (size_t)size);
  for (int i = 0; i < size; i++) rc[i] = (int)block;
  fill(hs, dt, total, seed + 104729u * (unsigned)rank);
  PMPI_Reduce_scatter(hs, want, rc, dt, MPI_SUM, MPI_COMM_WORLD);
  void *s, *r;
  if (dev) {
    if (hipMalloc(&s, total * esz) != hipSuccess || hipMalloc(&r, block * esz) != hipSuccess) { report(tag, 0); return; }
    (void)hipMemcpy(s, hs, total * esz, hipMemcpyHostToDevice);
  } else {
    s = malloc(total * esz);
    r = malloc(block * esz);
    memcpy(s, hs, total * esz);
  }
  const int e = reduce_scatter_bine_permute_remap(s, r, rc, dt, MPI_SUM, MPI_COMM_WORLD);
  if (dev) (void)hipMemcpy(got, r, block * esz, hipMemcpyDeviceToHost);
  else memcpy(got, r, block * esz);
  report(tag, e == MPI_SUCCESS && memcmp(got, want, block * esz) == 0);
  if (dev) {
    (void)hipFree(s);
    (void)hipFree(r);
  } else {
    free(s);
    free(r);
  }
  free(hs);
  free(want);
  free(got);
  free(rc);
}

/* ragged counts with a rank that receives nothing and passes no rbuf (ADVICE
 * r4): the staged path is chosen from the total on every rank, so that rank
 * must still issue the schedule its peers issue instead of refusing the call */
static void check_reduce_scatter_zero(const char *tag, MPI_Datatype dt, size_t block, unsigned seed) {
  const size_t esz = dt == MPI_FLOAT ? 4 : 8;
  int *rc = malloc(sizeof(int) * (size_t)size);
  size_t total = 0;
  for (int i = 0; i < size; i++) total += (size_t)(rc[i] = i == size - 1 ? 0 : (int)block);
  const size_t mine = (size_t)rc[rank];
  void *hs = malloc(total * esz), *want = malloc(block * esz), *got = malloc(block * esz);
  fill(hs, dt, total, seed + 7927u * (unsigned)rank);
  PMPI_Reduce_scatter(hs, want, rc, dt, MPI_SUM, MPI_COMM_WORLD);
  void *r = mine ? malloc(mine * esz) : NULL;
  const int e = reduce_scatter_bine_send_remap(hs, r, rc, dt, MPI_SUM, MPI_COMM_WORLD);
  if (mine) memcpy(got, r, mine * esz);
  report(tag, e == MPI_SUCCESS && (!mine || memcmp(got, want, mine * esz) == 0));
  free(r);
  free(hs);
  free(want);
  free(got);
  free(rc);
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  char tag[160];
  /* 1. churn: the same sizes freed and allocated again between calls */
  const MPI_Datatype dts[2] = {MPI_FLOAT, MPI_INT64_T};
  const char *dn[2] = {"float", "int64"};
  for (int d = 0; d < 2; d++) {
    const size_t n = ((size_t)64 << 20) / (d ? 8 : 4);
    for (int in_place = 0; in_place < 2; in_place++) {
      /* the caller's buffers first, so that they sit above the check's own
       * allocations and a fresh mmap of the same size lands where they were */
      void *s = malloc(n * (d ? 8 : 4)), *r = malloc(n * (d ? 8 : 4));
      snprintf(tag, sizeof tag, "churn %s 64 MiB %s: first buffers", dn[d], in_place ? "in place" : "out of place");
      check_allreduce(tag, dts[d], n, in_place, 0, 11u, &s, &r);
      void *old_s = s, *old_r = r;
      free(s);
      free(r);
      s = malloc(n * (d ? 8 : 4));
      r = malloc(n * (d ? 8 : 4));
      snprintf(tag, sizeof tag, "churn %s 64 MiB %s: freed, malloc'd again (same addresses: %s), new data",
               dn[d], in_place ? "in place" : "out of place", s == old_s && r == old_r ? "yes" : "no");
      check_allreduce(tag, dts[d], n, in_place, 0, 29u, &s, &r);
      free(s);
      free(r);
    }
  }
  /* 2. mixed placement: rank 0 on the device, the others on the host */
  if (size > 1) {
    const size_t sizes[3] = {4099, (size_t)8 << 20, (size_t)40 << 20};  /* bytes / esz below */
    for (int d = 0; d < 2; d++)
      for (int k = 0; k < 3; k++) {
        const size_t n = k == 0 ? sizes[0] : sizes[k] / (d ? 8 : 4);
        snprintf(tag, sizeof tag, "mixed placement allreduce %s n=%zu (rank 0 device, others host)", dn[d], n);
        check_allreduce(tag, dts[d], n, 0, rank == 0, 41u + (unsigned)k, NULL, NULL);
        snprintf(tag, sizeof tag, "mixed placement allreduce %s n=%zu in place", dn[d], n);
        check_allreduce(tag, dts[d], n, 1, rank == 0, 43u + (unsigned)k, NULL, NULL);
        const size_t block = n / (size_t)size + 1;
        snprintf(tag, sizeof tag, "mixed placement reduce_scatter %s block=%zu", dn[d], block);
        check_reduce_scatter(tag, dts[d], block, rank == 0, 47u + (unsigned)k);
      }
  }
  if (size > 1) {
    /* above the staged threshold (2 x 16 MiB in total) and below it */
    const size_t blocks[2] = {((size_t)48 << 20) / 4 / (size_t)(size - 1) + 3, 1001};
    for (int k = 0; k < 2; k++) {
      snprintf(tag, sizeof tag, "reduce_scatter send_remap float block=%zu, last rank 0 elements and no rbuf",
               blocks[k]);
      check_reduce_scatter_zero(tag, MPI_FLOAT, blocks[k], 53u + (unsigned)k);
    }
  }
  if (rank == 0) printf(fails ? "CHURN FAILED %d of %d\n" : "CHURN ok %d\n", fails ? fails : cases, cases);
  MPI_Finalize();
  return fails ? 1 : 0;
}
