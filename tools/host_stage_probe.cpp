// host_stage_probe.cpp -- per-call alternatives to libbine.so's permanent
// hipHostRegister cache, timed on the box.  A 256 MiB
// host round trip in 16 MiB chunks, the shape of libbine.so's P = 1 staging
// pipeline (host -> device chunk k on stream A, device -> host chunk k on
// stream B after it): median of 7 calls per strategy.
//   cached   : both host buffers registered once, outside the timing (round 3)
//   whole    : both registered at the start of the call, unregistered at its end
//   chunked  : each 16 MiB piece registered just before its copy is issued,
//              all unregistered at the end of the call
//   pageable : hipMemcpyAsync straight from / to the pageable buffers
//   bounceT  : shim-owned page-locked bounce buffers (2 x 16 MiB per
//              direction), T threads of CPU memcpy between them and the caller
// Every strategy's output is checked against the input.
// build: hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/host_stage_probe.cpp -o tools/bin/host_stage_probe -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
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

static void par_memcpy(char *dst, const char *src, size_t n, int threads) {
  if (threads <= 1) {
    memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (n / threads + 4095) & ~(size_t)4095;
  for (int t = 0; t < threads; t++) {
    const size_t lo = std::min(n, per * t), hi = std::min(n, lo + per);
    if (hi > lo) th.emplace_back([=] { memcpy(dst + lo, src + lo, hi - lo); });
  }
  for (auto &x : th) x.join();
}

int main(int argc, char **argv) {
  const size_t MiB = 1 << 20, N = (argc > 1 ? (size_t)atoi(argv[1]) : 256) * MiB, CH = 16 * MiB;
  const size_t nch = (N + CH - 1) / CH;
  CK(hipSetDevice(0));
  char *src = (char *)malloc(N), *dst = (char *)malloc(N), *dev = nullptr;
  for (size_t i = 0; i < N; i++) src[i] = (char)(i * 131 + 7);
  memset(dst, 0, N);
  CK(hipMalloc((void **)&dev, N));
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(nch);
  for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  char *bin[2], *bout[2];
  for (int i = 0; i < 2; i++) {
    CK(hipHostMalloc((void **)&bin[i], CH, 0));
    CK(hipHostMalloc((void **)&bout[i], CH, 0));
  }
  hipEvent_t bin_ev[2], bout_ev[2];
  for (int i = 0; i < 2; i++) {
    CK(hipEventCreateWithFlags(&bin_ev[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&bout_ev[i], hipEventDisableTiming));
    CK(hipEventRecord(bin_ev[i], A));
    CK(hipEventRecord(bout_ev[i], B));
  }
  auto len_of = [&](size_t k) { return std::min(CH, N - k * CH); };
  // the pipelined round trip through device memory
  auto pipeline = [&](const std::function<void(size_t)> &before) {
    for (size_t k = 0; k < nch; k++) {
      if (before) before(k);
      CK(hipMemcpyAsync(dev + k * CH, src + k * CH, len_of(k), hipMemcpyHostToDevice, A));
      CK(hipEventRecord(ev[k], A));
      CK(hipStreamWaitEvent(B, ev[k], 0));
      CK(hipMemcpyAsync(dst + k * CH, dev + k * CH, len_of(k), hipMemcpyDeviceToHost, B));
    }
    CK(hipStreamSynchronize(A));
    CK(hipStreamSynchronize(B));
  };
  auto bounce = [&](int T) {
    // host -> bounce -> device, device -> bounce -> host, double-buffered
    for (size_t k = 0; k < nch + 1; k++) {
      if (k < nch) {
        const int s = (int)(k % 2);
        CK(hipEventSynchronize(bin_ev[s]));  // the DMA out of this bounce buffer (chunk k - 2) is done
        par_memcpy(bin[s], src + k * CH, len_of(k), T);
        CK(hipMemcpyAsync(dev + k * CH, bin[s], len_of(k), hipMemcpyHostToDevice, A));
        CK(hipEventRecord(bin_ev[s], A));
        CK(hipStreamWaitEvent(B, bin_ev[s], 0));
        CK(hipMemcpyAsync(bout[s], dev + k * CH, len_of(k), hipMemcpyDeviceToHost, B));
        CK(hipEventRecord(bout_ev[s], B));
      }
      if (k > 0) {  // chunk k - 1 back to the caller
        const int s = (int)((k - 1) % 2);
        CK(hipEventSynchronize(bout_ev[s]));
        par_memcpy(dst + (k - 1) * CH, bout[s], len_of(k - 1), T);
      }
    }
  };
  struct Strat {
    std::string name;
    std::function<void()> run;
    bool cached;
  };
  std::vector<std::pair<char *, size_t>> regs;
  std::vector<Strat> strats = {
      {"cached", [&] { pipeline(nullptr); }, true},
      {"whole",
       [&] {
         CK(hipHostRegister(src, N, hipHostRegisterDefault));
         CK(hipHostRegister(dst, N, hipHostRegisterDefault));
         pipeline(nullptr);
         CK(hipHostUnregister(src));
         CK(hipHostUnregister(dst));
       },
       false},
      {"chunked",
       [&] {
         pipeline([&](size_t k) {
           CK(hipHostRegister(src + k * CH, len_of(k), hipHostRegisterDefault));
           CK(hipHostRegister(dst + k * CH, len_of(k), hipHostRegisterDefault));
         });
         for (size_t k = 0; k < nch; k++) {
           CK(hipHostUnregister(src + k * CH));
           CK(hipHostUnregister(dst + k * CH));
         }
       },
       false},
      {"pageable", [&] { pipeline(nullptr); }, false},
      {"bounce1", [&] { bounce(1); }, false},
      {"bounce4", [&] { bounce(4); }, false},
      {"bounce8", [&] { bounce(8); }, false},
  };
  for (auto &s : strats) {
    if (s.cached) {
      CK(hipHostRegister(src, N, hipHostRegisterDefault));
      CK(hipHostRegister(dst, N, hipHostRegisterDefault));
    }
    std::vector<double> t;
    bool ok = true;
    for (int it = 0; it < 7; it++) {
      memset(dst, 0, N);
      CK(hipMemset(dev, 0, N));
      CK(hipDeviceSynchronize());
      const double t0 = now();
      s.run();
      t.push_back(now() - t0);
      ok = ok && memcmp(src, dst, N) == 0;
    }
    if (s.cached) {
      CK(hipHostUnregister(src));
      CK(hipHostUnregister(dst));
    }
    std::sort(t.begin(), t.end());
    printf("{\"strategy\": \"%s\", \"MiB\": %zu, \"ms_median\": %.3f, \"ms_min\": %.3f, \"ms_max\": %.3f, "
           "\"GBps_each_way\": %.1f, \"ok\": %s}\n",
           s.name.c_str(), N / MiB, 1e3 * t[3], 1e3 * t[0], 1e3 * t[6], N / t[3] / 1e9, ok ? "true" : "false");
    fflush(stdout);
  }
  return 0;
}
