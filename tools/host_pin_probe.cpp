// host_pin_probe.cpp -- what libbine.so's host staging can afford, measured on
// the box (the permanent hipHostRegister range cache).
//
//   1. hipHostRegister + hipHostUnregister cost of a malloc'd (touched)
//      buffer, 1 / 16 / 64 / 256 MiB, median of 5;
//   2. CPU memcpy pageable -> page-locked, 1 / 2 / 4 / 8 threads, 256 MiB;
//   3. hipMemcpyAsync host -> device from pageable vs page-locked memory;
//   (a 4th probe -- a registered 64 MiB malloc buffer freed, malloc'd again and
//   copied through the old registration -- faulted the GPU, "an illegal memory
//   access was encountered", profiles/r4_host_pin_probe.txt; removed: a GPU
//   fault is never re-run)
//
// build: hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/host_pin_probe.cpp -o tools/bin/host_pin_probe -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static void par_memcpy(char *dst, const char *src, size_t n, int threads) {
  std::vector<std::thread> th;
  const size_t per = (n / threads + 4095) & ~(size_t)4095;
  for (int t = 0; t < threads; t++) {
    const size_t lo = std::min(n, per * t), hi = std::min(n, lo + per);
    th.emplace_back([=] { memcpy(dst + lo, src + lo, hi - lo); });
  }
  for (auto &x : th) x.join();
}

int main() {
  CK(hipSetDevice(0));
  const size_t MiB = 1 << 20;
  // 1. register / unregister cost
  for (size_t mb : {1, 16, 64, 256}) {
    const size_t n = mb * MiB;
    std::vector<double> reg, unreg;
    for (int it = 0; it < 5; it++) {
      char *p = (char *)malloc(n);
      memset(p, it, n);
      const double t0 = now();
      CK(hipHostRegister(p, n, hipHostRegisterMapped));
      const double t1 = now();
      CK(hipHostUnregister(p));
      const double t2 = now();
      reg.push_back(t1 - t0);
      unreg.push_back(t2 - t1);
      free(p);
    }
    printf("{\"probe\": \"register\", \"MiB\": %zu, \"register_ms\": %.3f, \"unregister_ms\": %.3f, "
           "\"register_GBps\": %.1f}\n",
           mb, 1e3 * median(reg), 1e3 * median(unreg), n / median(reg) / 1e9);
    fflush(stdout);
  }
  // 2. CPU memcpy pageable -> page-locked
  const size_t N = 256 * MiB;
  char *pg = (char *)malloc(N), *pl = nullptr, *pg2 = (char *)malloc(N);
  memset(pg, 1, N);
  memset(pg2, 2, N);
  CK(hipHostMalloc((void **)&pl, N, 0));
  memset(pl, 3, N);
  for (int th : {1, 2, 4, 8}) {
    std::vector<double> t;
    for (int it = 0; it < 5; it++) {
      const double t0 = now();
      par_memcpy(pl, pg, N, th);
      t.push_back(now() - t0);
    }
    printf("{\"probe\": \"memcpy_to_pinned\", \"threads\": %d, \"GBps\": %.1f}\n", th, N / median(t) / 1e9);
    fflush(stdout);
  }
  // 3. hipMemcpyAsync H2D pageable vs page-locked, and D2H
  char *d = nullptr;
  CK(hipMalloc((void **)&d, N));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int pinned : {0, 1}) {
    char *h = pinned ? pl : pg;
    std::vector<double> t, host_t, t2;
    for (int it = 0; it < 5; it++) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      CK(hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, s));
      const double t1 = now();
      CK(hipStreamSynchronize(s));
      const double t2_ = now();
      CK(hipMemcpyAsync(h, d, N, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      t.push_back(t2_ - t0);
      host_t.push_back(t1 - t0);
      t2.push_back(now() - t2_);
    }
    printf("{\"probe\": \"hipMemcpyAsync\", \"host\": \"%s\", \"h2d_GBps\": %.1f, \"h2d_host_blocked_ms\": %.3f, "
           "\"d2h_GBps\": %.1f}\n",
           pinned ? "page-locked" : "pageable", N / median(t) / 1e9, 1e3 * median(host_t), N / median(t2) / 1e9);
    fflush(stdout);
  }
  return 0;
}
