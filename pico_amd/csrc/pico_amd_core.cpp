// pico_amd_core.cpp -- device-resident benchmark driver for the MI355X library
// with pico_core's command line, environment and output files, so the
// reference's campaign scripts and plot/ tooling read its results unchanged
// (SURVEY.md 8(f) rank 3).  Every COLLECTIVE_TYPE of pico_core:
// ALLREDUCE, REDUCE_SCATTER, REDUCE, ALLGATHER, BCAST, GATHER, SCATTER, ALLTOALL.
//
//   mpiexec -n P pico_amd_core <count> <iterations> <algorithm> <dtype>
//
// Interface it follows (reference behaviour, re-implemented):
//   * arguments and dtype names ........ pico_core_utils.c:612-672
//   * COLLECTIVE_TYPE, SEGMENTED/SEGSIZE, OUTPUT_DIR, DATA_DIR, OUTPUT_LEVEL,
//     LOCATION ........................... pico_core_utils.c:20-40, :311-318, :352-402, :809-870
//   * algorithm selector strings ....... pico_core_utils.c:103-249 (resolved with
//     bine_algo_from_name, then called through the libbine.h symbol of libbine.so)
//   * timing: barrier, per-iteration MPI_Wtime around one call, barrier
//     ................................... pico_core_utils.h:243-262
//   * ground truth against PMPI_* of the same MPI, eps for float/double,
//     memcmp otherwise ................... pico_core_utils.c:553-610, :960-992
//   * <count>_<algo>[_<segsize>]_<dtype>.csv (all | summarized) and
//     alloc_<P>_GPU.csv ................. pico_core_utils.c:368-386, :711-785
//
// What differs: buffers live in HBM for the whole run (the CUDA_AWARE flow of
// pico_core.c:63-123, but the send buffer is generated on the device with the
// same rand_r distribution -- bine_fill_pico -- instead of on the host + H2D);
// PICO_SEED=<n> fixes the seed base (default time(NULL), as pico_core).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <sys/stat.h>

#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "bine_amd.h"
#include "libbine_amd.h"

namespace {

struct Dtype { const char *name; MPI_Datatype mpi; int bine; size_t size; };

const Dtype *find_dtype(const char *s) {
  static const Dtype k[] = {
      {"int8", MPI_INT8_T, BINE_INT8, 1},         {"int16", MPI_INT16_T, BINE_INT16, 2},
      {"int32", MPI_INT32_T, BINE_INT32, 4},      {"int64", MPI_INT64_T, BINE_INT64, 8},
      {"int", MPI_INT, BINE_INT32, sizeof(int)},  {"float", MPI_FLOAT, BINE_FLOAT, 4},
      {"double", MPI_DOUBLE, BINE_DOUBLE, 8},     {"char", MPI_CHAR, BINE_INT8, 1},
      {"unsigned_char", MPI_UNSIGNED_CHAR, BINE_UINT8, 1},
  };
  for (const auto &d : k)
    if (!strcmp(s, d.name)) return &d;
  return nullptr;
}

enum Coll { ALLREDUCE, REDUCE_SCATTER, REDUCE, ALLGATHER, BCAST, GATHER, SCATTER, ALLTOALL };

int fail(const char *msg) {
  fprintf(stderr, "pico_amd_core: %s. Aborting...\n", msg);
  return -1;
}

bool file_exists(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}

// |a - b| <= P * base_eps * 100, base 1e-6 (float) / 1e-15 (double), as pico_core
template <typename T>
bool close_enough(const void *a, const void *b, size_t n, double eps) {
  const T *x = (const T *)a, *y = (const T *)b;
  for (size_t i = 0; i < n; i++)
    if (std::fabs((double)x[i] - (double)y[i]) > eps) return false;
  return true;
}

bool same(const void *got, const void *want, size_t n, const Dtype *dt, int P) {
  if (dt->mpi == MPI_FLOAT) return close_enough<float>(got, want, n, P * 1e-6 * 100.0);
  if (dt->mpi == MPI_DOUBLE) return close_enough<double>(got, want, n, P * 1e-15 * 100.0);
  return memcmp(got, want, n * dt->size) == 0;
}

int write_csv(const std::string &path, const char *level, const std::vector<double> &highest,
              const std::vector<double> &all, int P, int iter) {
  if (!strcmp(level, "statistics")) return 0;  // not written by the reference either (:781-784)
  FILE *f = fopen(path.c_str(), "w");
  if (!f) return fail("cannot open the data file");
  const bool every_rank = !strcmp(level, "all");
  fprintf(f, "highest");
  if (every_rank)
    for (int r = 0; r < P; r++) fprintf(f, ",rank%d", r);
  fprintf(f, "\n");
  for (int i = 0; i < iter; i++) {
    fprintf(f, "%" PRId64, (int64_t)(highest[(size_t)i] * 1e9));
    if (every_rank)
      for (int r = 0; r < P; r++) fprintf(f, ",%" PRId64, (int64_t)(all[(size_t)r * (size_t)iter + (size_t)i] * 1e9));
    fprintf(f, "\n");
  }
  fclose(f);
  return 0;
}

int write_alloc(const std::string &path, MPI_Comm comm) {
  int rank, P, len;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &P);
  char host[MPI_MAX_PROCESSOR_NAME];
  MPI_Get_processor_name(host, &len);
  const int W = MPI_MAX_PROCESSOR_NAME + 64;
  std::vector<char> mine((size_t)W, 0), all;
  snprintf(mine.data(), (size_t)W, "%d,%s\n", rank, host);
  if (rank == 0) all.resize((size_t)W * (size_t)P);
  MPI_Gather(mine.data(), W, MPI_CHAR, all.data(), W, MPI_CHAR, 0, comm);
  if (rank == 0) {
    FILE *f = fopen(path.c_str(), "w");
    if (!f) return fail("cannot open the allocation file");
    fprintf(f, "MPI_Rank,allocation\n");
    for (int r = 0; r < P; r++) fprintf(f, "%s", all.data() + (size_t)r * (size_t)W);
    fclose(f);
  }
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  MPI_Comm comm = MPI_COMM_WORLD;
  int rank, P;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &P);
  auto die = [&](const char *m) {
    fail(m);
    MPI_Abort(comm, 1);
    return 1;
  };

  if (argc != 5) return die("usage: pico_amd_core <array_count> <iterations> <algorithm> <dtype>");
  char *end;
  const size_t count = (size_t)strtoll(argv[1], &end, 10);
  if (*end || count == 0) return die("invalid array count");
  const int iter = (int)strtol(argv[2], &end, 10);
  if (*end || iter <= 0) return die("invalid number of iterations");
  const char *algorithm = argv[3];
  const Dtype *dt = find_dtype(argv[4]);
  if (!dt) return die("unknown datatype");

  const char *ct = getenv("COLLECTIVE_TYPE");
  if (!ct) return die("COLLECTIVE_TYPE not set");
  Coll coll;
  const char *cname;
  if (!strcmp(ct, "ALLREDUCE")) { coll = ALLREDUCE; cname = "allreduce"; }
  else if (!strcmp(ct, "REDUCE_SCATTER")) { coll = REDUCE_SCATTER; cname = "reduce_scatter"; }
  else if (!strcmp(ct, "REDUCE")) { coll = REDUCE; cname = "reduce"; }
  else if (!strcmp(ct, "ALLGATHER")) { coll = ALLGATHER; cname = "allgather"; }
  else if (!strcmp(ct, "BCAST")) { coll = BCAST; cname = "bcast"; }
  else if (!strcmp(ct, "GATHER")) { coll = GATHER; cname = "gather"; }
  else if (!strcmp(ct, "SCATTER")) { coll = SCATTER; cname = "scatter"; }
  else if (!strcmp(ct, "ALLTOALL")) { coll = ALLTOALL; cname = "alltoall"; }
  else return die("unknown COLLECTIVE_TYPE");

  const int algo = bine_algo_from_name(cname, algorithm);
  if (algo < 0) return die("unknown algorithm");
  const std::string sym = std::string(cname) + "_" + bine_algo_name(algo);
  void *fn = dlsym(RTLD_DEFAULT, sym.c_str());
  if (!fn) return die("libbine.so does not export the algorithm");

  const char *seg = getenv("SEGMENTED");
  if (seg && !strcmp(seg, "yes")) {
    const char *ss = getenv("SEGSIZE");
    if (!ss) return die("SEGMENTED=yes needs SEGSIZE");
    bine_allreduce_segsize = (size_t)strtoll(ss, nullptr, 10);
  }
  const char *out_dir = getenv("OUTPUT_DIR"), *data_dir = getenv("DATA_DIR"), *level = getenv("OUTPUT_LEVEL");
  const bool save = out_dir && data_dir && level;
  if (save && strcmp(level, "all") && strcmp(level, "statistics") && strcmp(level, "summarized"))
    return die("invalid OUTPUT_LEVEL");

  // ---- buffers in HBM (sizes as pico_core's allocators) ----
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return die("no HIP device visible");
  MPI_Comm local;
  MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &local);
  int lrank;
  MPI_Comm_rank(local, &lrank);
  MPI_Comm_free(&local);
  const char *dev_env = getenv("BINE_DEVICE");
  (void)hipSetDevice(dev_env ? atoi(dev_env) : lrank % ndev);

  // sizes as pico_core's allocators (pico_core_*_utils.c): the root-only
  // buffers (gather's rbuf, scatter's sbuf) are passed as NULL elsewhere;
  // bcast runs in place on the send buffer
  const size_t local_count = count / (size_t)P;
  const size_t s_elems = coll == ALLGATHER || coll == GATHER ? local_count : count;
  const size_t r_elems = coll == REDUCE_SCATTER || coll == SCATTER ? local_count : coll == BCAST ? 0 : count;
  void *sbuf = nullptr, *rbuf = nullptr;
  if (hipMalloc(&sbuf, s_elems * dt->size + 16) != hipSuccess || hipMalloc(&rbuf, r_elems * dt->size + 16) != hipSuccess)
    return die("device allocation failed");
  (void)hipMemset(rbuf, 0, r_elems * dt->size);
  const char *seed_env = getenv("PICO_SEED");
  const uint32_t seed = (uint32_t)(seed_env ? strtoul(seed_env, nullptr, 10) : (unsigned long)time(nullptr)) + (uint32_t)rank;
  if (bine_fill_pico(sbuf, s_elems, dt->bine, seed, nullptr) != BINE_SUCCESS) return die("input generation failed");
  (void)hipDeviceSynchronize();
  std::vector<char> hs(s_elems * dt->size), hr(r_elems * dt->size), gt(r_elems * dt->size);
  (void)hipMemcpy(hs.data(), sbuf, hs.size(), hipMemcpyDeviceToHost);  // the inputs (bcast: overwritten below)

  // ---- timed loop (one barrier before, one after every iteration) ----
  std::vector<int> rcounts((size_t)P, (int)local_count);
  std::vector<double> times((size_t)iter);
  int ret = MPI_SUCCESS;
  MPI_Barrier(comm);
  for (int i = 0; i < iter && ret == MPI_SUCCESS; i++) {
    const double t0 = MPI_Wtime();
    switch (coll) {
      case ALLREDUCE:
        ret = ((int (*)(BINE_ALLREDUCE_ARGS))fn)(sbuf, rbuf, count, dt->mpi, MPI_SUM, comm);
        break;
      case REDUCE_SCATTER:
        ret = ((int (*)(BINE_REDUCE_SCATTER_ARGS))fn)(sbuf, rbuf, rcounts.data(), dt->mpi, MPI_SUM, comm);
        break;
      case REDUCE:
        ret = ((int (*)(BINE_REDUCE_ARGS))fn)(sbuf, rank == 0 ? rbuf : nullptr, count, dt->mpi, MPI_SUM, 0, comm);
        break;
      case ALLGATHER:
        ret = ((int (*)(BINE_ALLGATHER_ARGS))fn)(sbuf, local_count, dt->mpi, rbuf, local_count, dt->mpi, comm);
        break;
      case BCAST:
        ret = ((int (*)(BINE_BCAST_ARGS))fn)(sbuf, count, dt->mpi, 0, comm);
        break;
      case GATHER:
        ret = ((int (*)(BINE_GATHER_ARGS))fn)(sbuf, local_count, dt->mpi, rank == 0 ? rbuf : nullptr, local_count,
                                              dt->mpi, 0, comm);
        break;
      case SCATTER:
        ret = ((int (*)(BINE_GATHER_ARGS))fn)(rank == 0 ? sbuf : nullptr, local_count, dt->mpi, rbuf, local_count,
                                              dt->mpi, 0, comm);
        break;
      case ALLTOALL:
        ret = ((int (*)(BINE_ALLGATHER_ARGS))fn)(sbuf, local_count, dt->mpi, rbuf, local_count, dt->mpi, comm);
        break;
    }
    times[(size_t)i] = MPI_Wtime() - t0;
    MPI_Barrier(comm);
  }
  if (ret != MPI_SUCCESS) {
    fprintf(stderr, "pico_amd_core: %s returned MPI error %d\n", sym.c_str(), ret);
    MPI_Abort(comm, 1);
  }

  // ---- ground truth: PMPI_* of the same MPI on host copies ----
  (void)hipMemcpy(hr.data(), rbuf, hr.size(), hipMemcpyDeviceToHost);
  bool ok = true;
  switch (coll) {
    case ALLREDUCE:
      PMPI_Allreduce(hs.data(), gt.data(), (int)count, dt->mpi, MPI_SUM, comm);
      ok = same(hr.data(), gt.data(), count, dt, P);
      break;
    case REDUCE_SCATTER:
      PMPI_Reduce_scatter(hs.data(), gt.data(), rcounts.data(), dt->mpi, MPI_SUM, comm);
      ok = same(hr.data(), gt.data(), local_count, dt, P);
      break;
    case REDUCE:
      PMPI_Reduce(hs.data(), gt.data(), (int)count, dt->mpi, MPI_SUM, 0, comm);
      ok = rank != 0 || same(hr.data(), gt.data(), count, dt, P);
      break;
    case ALLGATHER:
      PMPI_Allgather(hs.data(), (int)local_count, dt->mpi, gt.data(), (int)local_count, dt->mpi, comm);
      ok = same(hr.data(), gt.data(), local_count * (size_t)P, dt, P);
      break;
    case BCAST: {  // the root's input, broadcast by MPICH, vs every rank's buffer after the run
      std::vector<char> now(hs.size());
      (void)hipMemcpy(now.data(), sbuf, now.size(), hipMemcpyDeviceToHost);
      PMPI_Bcast(hs.data(), (int)count, dt->mpi, 0, comm);
      ok = memcmp(now.data(), hs.data(), hs.size()) == 0;
      break;
    }
    case GATHER:
      PMPI_Gather(hs.data(), (int)local_count, dt->mpi, gt.data(), (int)local_count, dt->mpi, 0, comm);
      ok = rank != 0 || memcmp(hr.data(), gt.data(), count * dt->size) == 0;
      break;
    case SCATTER:
      PMPI_Scatter(hs.data(), (int)local_count, dt->mpi, gt.data(), (int)local_count, dt->mpi, 0, comm);
      ok = memcmp(hr.data(), gt.data(), local_count * dt->size) == 0;
      break;
    case ALLTOALL:
      PMPI_Alltoall(hs.data(), (int)local_count, dt->mpi, gt.data(), (int)local_count, dt->mpi, comm);
      ok = memcmp(hr.data(), gt.data(), count * dt->size) == 0;
      break;
  }
  int all_ok = 0, mine = ok ? 1 : 0;
  PMPI_Allreduce(&mine, &all_ok, 1, MPI_INT, MPI_MIN, comm);
  if (!all_ok) {
    if (rank == 0) fprintf(stderr, "pico_amd_core: results are not valid. Aborting...\n");
    MPI_Abort(comm, 1);
  }

  // ---- max over ranks per iteration, files ----
  std::vector<double> all(rank == 0 ? (size_t)P * (size_t)iter : 0), highest((size_t)iter);
  PMPI_Gather(times.data(), iter, MPI_DOUBLE, all.data(), iter, MPI_DOUBLE, 0, comm);
  PMPI_Reduce(times.data(), highest.data(), iter, MPI_DOUBLE, MPI_MAX, 0, comm);
  if (rank == 0) {
    printf("-----------------------------------------------------------------------------------------------\n");
    printf("   %-30s\n    Last Iter Time: %15" PRId64 "ns     %10zu elements of %s dtype\t%6d iter",
           algorithm, (int64_t)(highest[(size_t)iter - 1] * 1e9), count, dt->name, iter);
    if (bine_allreduce_segsize) printf("\t%8zu segsize", bine_allreduce_segsize);
    printf("\n");
  }
  if (save) {
    char name[256];
    if (bine_allreduce_segsize)
      snprintf(name, sizeof name, "/%zu_%s_%zu_%s.csv", count, algorithm, bine_allreduce_segsize, dt->name);
    else
      snprintf(name, sizeof name, "/%zu_%s_%s.csv", count, algorithm, dt->name);
    if (rank == 0 && write_csv(std::string(data_dir) + name, level, highest, all, P, iter)) MPI_Abort(comm, 1);
    const std::string alloc = std::string(out_dir) + "/alloc_" + std::to_string(P) + "_GPU.csv";
    int need = rank == 0 ? !file_exists(alloc) : 0;
    PMPI_Bcast(&need, 1, MPI_INT, 0, comm);
    if (need && write_alloc(alloc, comm)) MPI_Abort(comm, 1);
  }
  (void)hipFree(sbuf);
  (void)hipFree(rbuf);
  MPI_Barrier(comm);
  MPI_Finalize();
  return 0;
}
