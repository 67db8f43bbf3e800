// wt_store_probe.cpp -- what the direct transport's write-through stores cost
// (k_dm_fused runs a C3 call at P = 2 on one GPU at
// 0.65-0.70 of 8 TB/s while its HBM bytes are 1.0015 x the model's).  Every
// byte a rank pushes into a peer's inbox is stored write-through (buffer
// store, aux 19 = sc0 | nt | sc1: kernels.hip st_wt) so that a reader on
// another XCD or GPU sees it once the flag is seen; phase A of k_dm_fused is
// a copy with such stores, phase B a 2-leaf tree whose result goes to `out`
// (non-temporal) and, write-through, to the peer.  This probe times the same
// shapes on hipMalloc memory with non-temporal stores and with write-through
// stores: 256 MiB, full grid (k_copy's shape: 8 vectors per lane) and 512
// grid-strided workgroups with 4 vectors per lane (k_dm_fused's shape at
// P = 2).  Median of 7 x 5 launches; one JSON line per case.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/wt_store_probe.cpp -o tools/bin/wt_store_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
static const size_t kBytes = 256u << 20;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void *base) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  const uint64_t u = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32 |
                     (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)u, (short)0, 0x7fffffff, 0x00020000);
}

template <bool WT>
__device__ __forceinline__ void store(u32x4 *d, __amdgpu_buffer_rsrc_t r, size_t i, u32x4 v) {
  if (WT) __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(i * 16), 0, 19);
  else __builtin_nontemporal_store(v, d + i);
}

// copy: full grid (nwg = 0 shape: one tile of U = 8 per lane) or grid-strided (U = 4)
template <bool WT, int U, bool STRIDED>
__global__ __launch_bounds__(256) void k_cp(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t nvec) {
  const __amdgpu_buffer_rsrc_t r = rsrc(d);
  const size_t stride = STRIDED ? (size_t)gridDim.x * 256 * U : nvec;
  for (size_t b0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; b0 < nvec; b0 += stride) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 256 < nvec) x[u] = __builtin_nontemporal_load(s + b0 + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 256 < nvec) store<WT>(d, r, b0 + u * 256, x[u]);
    if (!STRIDED) break;
  }
}

// phase B at P = 2: out = a + b (non-temporal), and the same vector pushed (WT
// or non-temporal) into a second buffer; grid-strided, U = 4
template <bool WT>
__global__ __launch_bounds__(256) void k_tree2(const u32x4 *__restrict__ a, const u32x4 *__restrict__ b,
                                               u32x4 *__restrict__ out, u32x4 *__restrict__ push, size_t nvec) {
  constexpr int U = 4;
  const __amdgpu_buffer_rsrc_t r = rsrc(push);
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t b0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; b0 < nvec; b0 += stride) {
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 256 < nvec) {
        x[u] = a[b0 + u * 256];
        y[u] = __builtin_nontemporal_load(b + b0 + u * 256);
      }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 256 < nvec) {
        const u32x4 v = x[u] + y[u];
        __builtin_nontemporal_store(v, out + b0 + u * 256);
        store<WT>(push, r, b0 + u * 256, v);
      }
  }
}

template <typename F>
static double time_us(F launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int r = 0; r < 7; r++) {
    CK(hipEventRecord(e0, 0));
    for (int k = 0; k < 5; k++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t / 5);
  }
  std::sort(ms.begin(), ms.end());
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms[3] * 1e3;
}

static void report(const char *name, const char *stores, const char *shape, double us, double bytes) {
  printf("{\"kernel\": \"%s\", \"stores\": \"%s\", \"shape\": \"%s\", \"us\": %.1f, \"TBs\": %.3f, \"frac_8TBs\": %.3f}\n",
         name, stores, shape, us, bytes / (us * 1e-6) / 1e12, bytes / (us * 1e-6) / 8e12);
  fflush(stdout);
}

int main() {
  const size_t nvec = kBytes / 16;
  u32x4 *s, *d, *a2, *p2;
  CK(hipMalloc(&s, kBytes));
  CK(hipMalloc(&d, kBytes));
  CK(hipMalloc(&a2, kBytes));
  CK(hipMalloc(&p2, kBytes));
  for (void *p : {(void *)s, (void *)d, (void *)a2, (void *)p2}) CK(hipMemset(p, 1, kBytes));
  CK(hipDeviceSynchronize());
  const unsigned full = (unsigned)((nvec + 2047) / 2048);
  for (int wt = 0; wt < 2; wt++) {
    const char *st = wt ? "write-through (sc0 nt sc1)" : "non-temporal";
    double us = time_us([&] {
      if (wt) hipLaunchKernelGGL((k_cp<true, 8, false>), dim3(full), dim3(256), 0, 0, s, d, nvec);
      else hipLaunchKernelGGL((k_cp<false, 8, false>), dim3(full), dim3(256), 0, 0, s, d, nvec);
    });
    report("copy", st, "full grid, 8 vectors per lane", us, 2.0 * kBytes);
    us = time_us([&] {
      if (wt) hipLaunchKernelGGL((k_cp<true, 4, true>), dim3(512), dim3(256), 0, 0, s, d, nvec);
      else hipLaunchKernelGGL((k_cp<false, 4, true>), dim3(512), dim3(256), 0, 0, s, d, nvec);
    });
    report("copy", st, "512 workgroups strided, 4 vectors per lane", us, 2.0 * kBytes);
    us = time_us([&] {
      if (wt) hipLaunchKernelGGL(k_tree2<true>, dim3(512), dim3(256), 0, 0, s, a2, d, p2, nvec);
      else hipLaunchKernelGGL(k_tree2<false>, dim3(512), dim3(256), 0, 0, s, a2, d, p2, nvec);
    });
    report("tree2 + push", st, "512 workgroups strided, 4 vectors per lane", us, 4.0 * kBytes);
  }
  return 0;
}
