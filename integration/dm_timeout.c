/*
 * dm_timeout.c -- libbine.so's error contract when a direct-transport wait
 * times out: the call in which the wait timed out must
 * return an MPI error itself, never MPI_SUCCESS with a wrong rbuf -- pico_core
 * treats any non-success return as fatal (pico_core_utils.h:253-256), so a
 * success here would hide a wrong result from it.
 *
 * Run with BINE_DIRECT=1 (the direct peer-memory transport) and
 * BINE_DIRECT_TIMEOUT_S=1e-7 (every wait gives up at once).  Per rank, on
 * 64 MiB int64 host buffers (exact under any association):
 *   call 1: MPI_ERR_OTHER, or -- on a rank whose waits were all satisfied
 *           before it looked, so its data had arrived -- MPI_SUCCESS with the
 *           result of PMPI_Allreduce;
 *   call 2: an error on every rank (the transport is dead on a rank that
 *           timed out, and its peers wait in vain);
 * and at least one rank's call 1 fails.
 *   usage: mpiexec -n P dm_timeout     (prints "DMTIMEOUT ok" on rank 0)
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libbine_amd.h"

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  const size_t n = (size_t)8 << 20, bytes = n * sizeof(int64_t);
  int64_t *s = malloc(bytes), *r = malloc(bytes), *want = malloc(bytes);
  unsigned seed = 12345u + 7919u * (unsigned)rank;
  for (size_t k = 0; k < n; k++) {
    seed = seed * 1103515245u + 12345u;
    s[k] = (int64_t)seed * 31 - (int64_t)k;
  }
  PMPI_Allreduce(s, want, (int)n, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
  memset(r, 0, bytes);
  const int e1 = allreduce_bine_bdw_remap(s, r, n, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
  const int right = memcmp(r, want, bytes) == 0;
  memset(r, 0, bytes);
  const int e2 = allreduce_bine_bdw_remap(s, r, n, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
  /* this rank: no success with a wrong result, and the second call fails */
  int ok = (e1 != MPI_SUCCESS || right) && e2 != MPI_SUCCESS, all = 0, failed1 = e1 != MPI_SUCCESS, any = 0;
  printf("rank %d: call 1 returned %d (%s), call 2 returned %d\n", rank, e1,
         e1 == MPI_SUCCESS ? (right ? "result right" : "RESULT WRONG") : "error", e2);
  fflush(stdout);
  PMPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
  PMPI_Allreduce(&failed1, &any, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
  if (rank == 0) printf("DMTIMEOUT %s (P = %d)\n", all && any ? "ok" : "FAILED", size);
  free(s);
  free(r);
  free(want);
  MPI_Finalize();
  return all && any ? 0 : 1;
}
