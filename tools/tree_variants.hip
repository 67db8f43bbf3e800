// tree_variants.hip -- on-box exploration of the flat reduce-scatter's fused
// tree kernel shape at its C3 shape (fp32 SUM, 8 leaves x 16 MiB -> 16 MiB,
// 4 rotating buffer sets = 576 MiB).  Standalone program, not part of the
// library: prints us/launch and (8+1)*S/t per variant, variants interleaved
// round-robin, median of rounds; plus the read-only ceiling of the same 8
// streams.  (The arithmetic is a plain fp32 add here: speed only; the library
// kernel's bits are checked by tests/test_gpu.py.)
//   hipcc -O3 --offload-arch=gfx950 -I include -o tree_variants tools/tree_variants.hip -L pico_amd/lib -lbine_amd
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "bine_amd.h"
// the library's own kernel templates, launched directly (bisects host-side
// launch costs from kernel shape)
#include "../pico_amd/csrc/kernels.hip"

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int NL = 8;
struct Leaves { const f4 *p[NL]; };

template <int NT>
__device__ __forceinline__ f4 ld(const f4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// BS threads, U vectors of every leaf per lane, NT0 / NTL: non-temporal loads
// of leaf 0 / of the others, NTO: non-temporal store, HALF: load + reduce
// leaves 0-3 before loading 4-7 (fewer registers, less in flight), TPW tiles
// per workgroup (grid-stride over contiguous tiles)
template <int BS, int U, int NT0, int NTL, int NTO, int HALF, int TPW>
__global__ __launch_bounds__(BS) void k_tv(Leaves L, f4 *out, size_t nvec) {
  const size_t tile = (size_t)BS * U;
#pragma unroll 1
  for (int t = 0; t < TPW; t++) {
    const size_t base = ((size_t)blockIdx.x * TPW + t) * tile + threadIdx.x;
    if (base >= nvec) return;
    f4 r[U];
    if constexpr (!HALF) {
      f4 v[U][NL];
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int j = 0; j < NL; j++) {
          const size_t i = base + (size_t)u * BS;
          v[u][j] = i < nvec ? (j == 0 ? ld<NT0>(L.p[j] + i) : ld<NTL>(L.p[j] + i)) : f4{0, 0, 0, 0};
        }
#pragma unroll
      for (int u = 0; u < U; u++) {
#pragma unroll
        for (int w = 1; w < NL; w <<= 1)
#pragma unroll
          for (int j = 0; j < NL; j += 2 * w) v[u][j] = v[u][j] + v[u][j + w];
        r[u] = v[u][0];
      }
    } else {
      f4 lo[U];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        f4 v[U][NL / 2];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
          for (int j = 0; j < NL / 2; j++) {
            const size_t i = base + (size_t)u * BS;
            const int jj = h * NL / 2 + j;
            v[u][j] = i < nvec ? (jj == 0 ? ld<NT0>(L.p[jj] + i) : ld<NTL>(L.p[jj] + i)) : f4{0, 0, 0, 0};
          }
#pragma unroll
        for (int u = 0; u < U; u++) {
#pragma unroll
          for (int w = 1; w < NL / 2; w <<= 1)
#pragma unroll
            for (int j = 0; j < NL / 2; j += 2 * w) v[u][j] = v[u][j] + v[u][j + w];
          if (h == 0) lo[u] = v[u][0];
          else r[u] = lo[u] + v[u][0];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + (size_t)u * BS;
      if (i < nvec) {
        if constexpr (NTO) __builtin_nontemporal_store(r[u], out + i);
        else out[i] = r[u];
      }
    }
  }
}

// read-only ceiling of the 8 streams
template <int BS, int U>
__global__ __launch_bounds__(BS) void k_read8(Leaves L, f4 *sink, size_t nvec) {
  const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
  f4 s = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int j = 0; j < NL; j++) {
      const size_t i = base + (size_t)u * BS;
      if (i < nvec) s += __builtin_nontemporal_load(L.p[j] + i);
    }
  if (s.x == 12345.f) sink[threadIdx.x] = s;
}

// read-only ceiling of 8 / 9 streams with U vectors of each in flight per lane
template <int BS, int U, int NS>
__global__ __launch_bounds__(BS) void k_readn(Leaves L, const f4 *extra, f4 *sink, size_t nvec) {
  const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
  f4 s = {0, 0, 0, 0};
  f4 v[U][NS];
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int j = 0; j < NS; j++) {
      const size_t i = base + (size_t)u * BS;
      v[u][j] = i < nvec ? __builtin_nontemporal_load((j < NL ? L.p[j] : extra) + i) : f4{0, 0, 0, 0};
    }
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int j = 0; j < NS; j++) s += v[u][j];
  if (s.x == 12345.f) sink[threadIdx.x] = s;
}

struct Var {
  std::string name;
  double bytes_per_elem;
  std::function<void(const Leaves &, f4 *, f4 *, size_t, hipStream_t)> run;
};

template <int BS, int U, int NT0, int NTL, int NTO, int HALF, int TPW>
Var mk(const char *name) {
  return {name, 4.0 * (NL + 1), [](const Leaves &L, f4 *out, f4 *, size_t nvec, hipStream_t s) {
            const size_t tiles = (nvec + (size_t)BS * U - 1) / ((size_t)BS * U);
            const unsigned grid = (unsigned)((tiles + TPW - 1) / TPW);
            hipLaunchKernelGGL((k_tv<BS, U, NT0, NTL, NTO, HALF, TPW>), dim3(grid), dim3(BS), 0, s, L, out, nvec);
          }};
}

int main() {
  const size_t N = 4194304, nvec = N / 4;
  const int sets = 4;
  std::vector<Leaves> Ls(sets);
  std::vector<f4 *> O(sets);
  f4 *sink;
  for (int k = 0; k < sets; k++) {
    for (int j = 0; j < NL; j++) {
      f4 *p;
      CK(hipMalloc(&p, N * 4));
      bine_fill_pico(p, N, BINE_FLOAT, 5000 + 16 * k + j, nullptr);
      Ls[k].p[j] = p;
    }
    CK(hipMalloc(&O[k], N * 4));
  }
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<Var> vars = {
      {"library bine_reduce_tree", 4.0 * (NL + 1),
       [](const Leaves &L, f4 *out, f4 *, size_t nv, hipStream_t st) {
         bine_reduce_tree(NL, (const void *const *)L.p, out, nv * 4, BINE_FLOAT, BINE_SUM, st);
       }},
      {"library kernel<8,4> direct launch", 4.0 * (NL + 1),
       [](const Leaves &L, f4 *out, f4 *, size_t nv, hipStream_t st) {
         bine::TreeArgs t{};
         for (int j = 0; j < NL; j++) t.leaf[j] = L.p[j];
         t.out = out; t.n = nv * 4; t.nvec = nv; t.head = 0; t.vec = 1;
         hipLaunchKernelGGL((bine::k_reduce_tree<float, BINE_SUM, 8, 4>), dim3((unsigned)(nv / 1024)), dim3(256), 0,
                            st, t);
       }},
      {"library kernel<8,1> direct launch", 4.0 * (NL + 1),
       [](const Leaves &L, f4 *out, f4 *, size_t nv, hipStream_t st) {
         bine::TreeArgs t{};
         for (int j = 0; j < NL; j++) t.leaf[j] = L.p[j];
         t.out = out; t.n = nv * 4; t.nvec = nv; t.head = 0; t.vec = 1;
         hipLaunchKernelGGL((bine::k_reduce_tree<float, BINE_SUM, 8, 1>), dim3((unsigned)(nv / 256)), dim3(256), 0,
                            st, t);
       }},
      {"library kernel<8,2> direct launch", 4.0 * (NL + 1),
       [](const Leaves &L, f4 *out, f4 *, size_t nv, hipStream_t st) {
         bine::TreeArgs t{};
         for (int j = 0; j < NL; j++) t.leaf[j] = L.p[j];
         t.out = out; t.n = nv * 4; t.nvec = nv; t.head = 0; t.vec = 1;
         hipLaunchKernelGGL((bine::k_reduce_tree<float, BINE_SUM, 8, 2>), dim3((unsigned)(nv / 512)), dim3(256), 0,
                            st, t);
       }},
      mk<256, 2, 0, 1, 0, 0, 1>("bs256 u2 ntL"),
      mk<256, 1, 0, 1, 0, 0, 1>("bs256 u1 ntL"),
      mk<256, 4, 0, 1, 0, 0, 1>("bs256 u4 ntL"),
      mk<256, 2, 1, 1, 0, 0, 1>("bs256 u2 ntAll"),
      mk<256, 2, 0, 0, 0, 0, 1>("bs256 u2 no-nt"),
      mk<256, 2, 0, 1, 1, 0, 1>("bs256 u2 ntL ntO"),
      mk<256, 1, 1, 1, 1, 0, 1>("bs256 u1 ntAll ntO"),
      mk<256, 2, 0, 1, 0, 1, 1>("bs256 u2 ntL half"),
      mk<256, 4, 0, 1, 0, 1, 1>("bs256 u4 ntL half"),
      mk<512, 1, 0, 1, 0, 0, 1>("bs512 u1 ntL"),
      mk<512, 2, 0, 1, 0, 0, 1>("bs512 u2 ntL"),
      mk<1024, 1, 0, 1, 0, 0, 1>("bs1024 u1 ntL"),
      mk<128, 2, 0, 1, 0, 0, 1>("bs128 u2 ntL"),
      mk<64, 4, 0, 1, 0, 0, 1>("bs64 u4 ntL"),
      mk<256, 1, 0, 1, 0, 0, 2>("bs256 u1 ntL 2tiles/wg"),
      mk<256, 1, 0, 1, 0, 0, 4>("bs256 u1 ntL 4tiles/wg"),
      {"read8 (8S read only)", 4.0 * NL,
       [](const Leaves &L, f4 *, f4 *sk, size_t nv, hipStream_t st) {
         hipLaunchKernelGGL((k_read8<256, 1>), dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, L, sk, nv);
       }},
      // r3: read-only ceilings with more in flight, and of all 9 streams the
      // tree touches (the output buffer read instead of written)
      {"read8 u2 (8S read only)", 4.0 * NL,
       [](const Leaves &L, f4 *o, f4 *sk, size_t nv, hipStream_t st) {
         hipLaunchKernelGGL((k_readn<256, 2, 8>), dim3((unsigned)((nv + 511) / 512)), dim3(256), 0, st, L, o, sk, nv);
       }},
      {"read8 u4 (8S read only)", 4.0 * NL,
       [](const Leaves &L, f4 *o, f4 *sk, size_t nv, hipStream_t st) {
         hipLaunchKernelGGL((k_readn<256, 4, 8>), dim3((unsigned)((nv + 1023) / 1024)), dim3(256), 0, st, L, o, sk,
                            nv);
       }},
      {"read9 u2 (9S read only)", 4.0 * (NL + 1),
       [](const Leaves &L, f4 *o, f4 *sk, size_t nv, hipStream_t st) {
         hipLaunchKernelGGL((k_readn<256, 2, 9>), dim3((unsigned)((nv + 511) / 512)), dim3(256), 0, st, L, o, sk, nv);
       }},
      {"read9 u4 (9S read only)", 4.0 * (NL + 1),
       [](const Leaves &L, f4 *o, f4 *sk, size_t nv, hipStream_t st) {
         hipLaunchKernelGGL((k_readn<256, 4, 9>), dim3((unsigned)((nv + 1023) / 1024)), dim3(256), 0, st, L, o, sk,
                            nv);
       }},
      mk<256, 4, 0, 1, 1, 0, 1>("bs256 u4 ntL ntO"),
      mk<256, 4, 1, 1, 1, 0, 1>("bs256 u4 ntAll ntO"),
      mk<256, 4, 0, 1, 0, 1, 2>("bs256 u4 ntL half 2tiles/wg"),
  };
  const int rounds = 7, iters = 40;
  std::vector<std::vector<float>> ms(vars.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (size_t v = 0; v < vars.size(); v++) {
      for (int i = 0; i < 4; i++) vars[v].run(Ls[i % sets], O[i % sets], sink, nvec, s);
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; i++) vars[v].run(Ls[i % sets], O[i % sets], sink, nvec, s);
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
    printf("%-32s us=%.2f  GB/s=%.1f  (min us %.2f)\n", vars[v].name.c_str(), med * 1e3,
           vars[v].bytes_per_elem * N / (med * 1e-3) / 1e9, m[0] * 1e3);
  }
  return 0;
}
