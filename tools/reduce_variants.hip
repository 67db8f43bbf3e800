// reduce_variants.hip -- on-box exploration of the fp32 SUM reduce kernel shape
// (C2: inout = inout + in, 64 MiB, 4 rotating buffer sets).  Standalone
// program, not part of the library: prints ms/launch and 3*S/t per variant,
// variants interleaved round-robin, median of rounds; plus read-only and copy
// ceilings of the same access pattern.
//   hipcc -O3 --offload-arch=gfx950 -o reduce_variants tools/reduce_variants.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "bine_amd.h"

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ f4 ld(const f4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// BS threads, U vectors per operand per lane, ORDER 0 = interleaved loads,
// 1 = all of a then all of b; TPW tiles per workgroup (contiguous)
template <int BS, int U, int ORDER, int NTA, int NTB, int NTO, int TPW>
__global__ __launch_bounds__(BS) void k_var(const f4 *__restrict__ a, const f4 *b, f4 *out, size_t nvec) {
  const size_t tile = (size_t)BS * U;
  size_t base0 = (size_t)blockIdx.x * tile * TPW + threadIdx.x;
#pragma unroll 1
  for (int t = 0; t < TPW; t++) {
    const size_t base = base0 + (size_t)t * tile;
    if (base + (U - 1) * (size_t)BS >= nvec) {
      for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * BS;
        if (i < nvec) out[i] = b[i] + a[i];
      }
      return;
    }
    f4 x[U], y[U];
    if constexpr (ORDER == 0) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        x[u] = ld<NTA>(a + base + (size_t)u * BS);
        y[u] = ld<NTB>(b + base + (size_t)u * BS);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = ld<NTA>(a + base + (size_t)u * BS);
#pragma unroll
      for (int u = 0; u < U; u++) y[u] = ld<NTB>(b + base + (size_t)u * BS);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const f4 r = y[u] + x[u];
      if constexpr (NTO) __builtin_nontemporal_store(r, out + base + (size_t)u * BS);
      else out[base + (size_t)u * BS] = r;
    }
  }
}

// read-only ceiling: sum both operands, one store per workgroup
template <int BS, int U>
__global__ __launch_bounds__(BS) void k_read2(const f4 *__restrict__ a, const f4 *__restrict__ b, f4 *sink,
                                              size_t nvec) {
  const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
  f4 s = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = base + (size_t)u * BS;
    if (i < nvec) s += __builtin_nontemporal_load(a + i) + b[i];
  }
  if (s.x == 12345.f) sink[threadIdx.x] = s;
}

// copy ceiling: out = a
template <int BS, int U>
__global__ __launch_bounds__(BS) void k_copy(const f4 *__restrict__ a, f4 *out, size_t nvec) {
  const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = base + (size_t)u * BS;
    if (i < nvec) x[u] = __builtin_nontemporal_load(a + i);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = base + (size_t)u * BS;
    if (i < nvec) out[i] = x[u];
  }
}

struct Var {
  std::string name;
  double bytes_per_elem;  // algorithmic bytes per fp32 element
  std::function<void(const f4 *, f4 *, f4 *, size_t, hipStream_t)> run;
};

template <int BS, int U, int ORDER, int NTA, int NTB, int NTO, int TPW>
Var mk(const char *name) {
  return {name, 12.0, [](const f4 *a, f4 *b, f4 *, size_t nvec, hipStream_t s) {
            const size_t tiles = (nvec + (size_t)BS * U - 1) / ((size_t)BS * U);
            const unsigned grid = (unsigned)((tiles + TPW - 1) / TPW);
            hipLaunchKernelGGL((k_var<BS, U, ORDER, NTA, NTB, NTO, TPW>), dim3(grid), dim3(BS), 0, s, a, b, b, nvec);
          }};
}

int main() {
  const size_t N = 16777216, nvec = N / 4;
  const int sets = 4;
  std::vector<f4 *> A(sets), B(sets);
  f4 *sink;
  for (int k = 0; k < sets; k++) {
    CK(hipMalloc(&A[k], N * 4));
    CK(hipMalloc(&B[k], N * 4));
    CK(hipMemset(A[k], 0, N * 4));
    CK(hipMemset(B[k], 0, N * 4));
  }
  CK(hipMalloc(&sink, 1 << 20));
  const bool rnd = getenv("ZERO") == nullptr;
  if (rnd)
    for (int k = 0; k < sets; k++) {  // pico_core's distribution, as bench.py
      bine_fill_pico(A[k], N, BINE_FLOAT, 1234 + 2 * k, nullptr);
      bine_fill_pico(B[k], N, BINE_FLOAT, 1235 + 2 * k, nullptr);
    }
  CK(hipDeviceSynchronize());
  printf("data: %s\n", rnd ? "pico_core rand_r floats" : "zeros");
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<Var> vars = {
      mk<256, 4, 0, 1, 0, 0, 1>("cur  bs256 u4 ilv ntA"),
      mk<256, 4, 1, 1, 0, 0, 1>("bs256 u4 a-then-b ntA"),
      mk<256, 8, 0, 1, 0, 0, 1>("bs256 u8 ilv ntA"),
      mk<256, 8, 1, 1, 0, 0, 1>("bs256 u8 a-then-b ntA"),
      mk<512, 4, 0, 1, 0, 0, 1>("bs512 u4 ilv ntA"),
      mk<512, 2, 0, 1, 0, 0, 1>("bs512 u2 ilv ntA"),
      mk<1024, 2, 0, 1, 0, 0, 1>("bs1024 u2 ilv ntA"),
      mk<256, 4, 0, 1, 1, 0, 1>("bs256 u4 ilv ntA ntB"),
      mk<256, 4, 0, 1, 0, 1, 1>("bs256 u4 ilv ntA ntO"),
      mk<256, 4, 0, 1, 0, 0, 2>("bs256 u4 ilv ntA 2tiles/wg"),
      mk<256, 2, 0, 1, 0, 0, 4>("bs256 u2 ilv ntA 4tiles/wg"),
      mk<128, 8, 0, 1, 0, 0, 1>("bs128 u8 ilv ntA"),
      {"library bine_reduce_local", 12.0,
       [](const f4 *a, f4 *b, f4 *, size_t nv, hipStream_t st) {
         bine_reduce_local(a, b, nv * 4, BINE_FLOAT, BINE_SUM, st);
       }},
      {"read2 (2S read only)", 8.0,
       [](const f4 *a, f4 *b, f4 *sk, size_t nv, hipStream_t st) {
         hipLaunchKernelGGL((k_read2<256, 4>), dim3((unsigned)((nv + 1023) / 1024)), dim3(256), 0, st, a, b, sk, nv);
       }},
      {"copy (S read + S write)", 8.0,
       [](const f4 *a, f4 *b, f4 *, size_t nv, hipStream_t st) {
         hipLaunchKernelGGL((k_copy<256, 4>), dim3((unsigned)((nv + 1023) / 1024)), dim3(256), 0, st, a, b, nv);
       }},
  };
  const int rounds = 7, iters = 40;
  std::vector<std::vector<float>> ms(vars.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (size_t v = 0; v < vars.size(); v++) {
      for (int i = 0; i < 4; i++) vars[v].run(A[i % sets], B[i % sets], sink, nvec, s);
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; i++) vars[v].run(A[i % sets], B[i % sets], sink, nvec, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / iters);
    }
  for (size_t v = 0; v < vars.size(); v++) {
    auto m = ms[v];
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    printf("%-32s ms=%.5f  GB/s=%.1f  (min ms %.5f)\n", vars[v].name.c_str(), med,
           vars[v].bytes_per_elem * N / (med * 1e-3) / 1e9, m[0]);
  }
  return 0;
}
