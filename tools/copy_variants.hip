// copy_variants.hip -- on-box survey of (1) the device copy shape for the P = 1
// allreduce (libbine_allreduce.c:849-852 copy_buffer, 256 MiB fp32: the N = 1
// headline workload), and (2) the element-wise reduce at the small windows of
// C1 / the tail chunks (256 KiB .. 16 MiB), where launch and ramp cost dominate.
// (3) the C2 reduce with operands staged through LDS by LDS-DMA vs the
// library's register-only kernel.
// Standalone program, not part of the library: variants interleaved
// round-robin, median of rounds, HIP events on the launch stream.
//   hipcc -O3 --offload-arch=gfx950 -I include -o copy_variants tools/copy_variants.hip \
//         -L pico_amd/lib -lbine_amd -Wl,-rpath,pico_amd/lib
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

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ u4 ld(const u4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int NT>
__device__ __forceinline__ void st(u4 v, u4 *p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// one tile of BS * U vectors per workgroup (TPW consecutive tiles), loads first
template <int BS, int U, int NTL, int NTS, int TPW>
__global__ __launch_bounds__(BS) void k_copy_tile(const u4 *__restrict__ a, u4 *__restrict__ o, size_t nvec) {
  const size_t tile = (size_t)BS * U;
#pragma unroll 1
  for (int t = 0; t < TPW; t++) {
    const size_t base = ((size_t)blockIdx.x * TPW + t) * tile + threadIdx.x;
    if (base + (U - 1) * (size_t)BS < nvec) {
      u4 x[U];
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = ld<NTL>(a + base + (size_t)u * BS);
#pragma unroll
      for (int u = 0; u < U; u++) st<NTS>(x[u], o + base + (size_t)u * BS);
    } else {
      for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * BS;
        if (i < nvec) o[i] = a[i];
      }
      return;
    }
  }
}

// XCD-aware tile order (round 2 addition): workgroups are dispatched
// round-robin over the 8 XCDs (blockIdx.x % 8 = XCD); MAP 1 gives each XCD one
// contiguous eighth of the buffer, MAP 2 pairs of adjacent tiles to one XCD
template <int BS, int U, int NTL, int NTS, int MAP>
__global__ __launch_bounds__(BS) void k_copy_xcd(const u4 *__restrict__ a, u4 *__restrict__ o, size_t nvec,
                                                  unsigned ntiles) {
  const size_t tile = (size_t)BS * U;
  const unsigned b = blockIdx.x, x = b % 8, i = b / 8, per = (ntiles + 7) / 8;
  unsigned t = b;
  if constexpr (MAP == 1) t = x * per + i;
  if constexpr (MAP == 2) t = (i / 2) * 16 + x * 2 + (i % 2);
  if (t >= ntiles) return;
  const size_t base = (size_t)t * tile + threadIdx.x;
  if (base + (U - 1) * (size_t)BS < nvec) {
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld<NTL>(a + base + (size_t)u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(v[u], o + base + (size_t)u * BS);
  } else {
    for (int u = 0; u < U; u++) {
      const size_t j = base + (size_t)u * BS;
      if (j < nvec) o[j] = a[j];
    }
  }
}

// grid-strided over a fixed grid (GRID workgroups), U vectors in flight
template <int BS, int U, int NTL, int NTS>
__global__ __launch_bounds__(BS) void k_copy_gs(const u4 *__restrict__ a, u4 *__restrict__ o, size_t nvec) {
  const size_t tile = (size_t)BS * U, stride = (size_t)gridDim.x * tile;
  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  for (; base + (U - 1) * (size_t)BS < nvec; base += stride) {
    u4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = ld<NTL>(a + base + (size_t)u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(x[u], o + base + (size_t)u * BS);
  }
  for (int u = 0; u < U; u++) {
    const size_t i = base + (size_t)u * BS;
    if (i < nvec) o[i] = a[i];
  }
}

// element-wise fp32 SUM, one tile per workgroup (the library's shape), for
// the small-window sweep
template <int BS, int U>
__global__ __launch_bounds__(BS) void k_red(const f4 *__restrict__ a, const f4 *b, f4 *o, size_t nvec) {
  const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
  if (base + (U - 1) * (size_t)BS < nvec) {
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      x[u] = __builtin_nontemporal_load(a + base + (size_t)u * BS);
      y[u] = b[base + (size_t)u * BS];
    }
#pragma unroll
    for (int u = 0; u < U; u++) o[base + (size_t)u * BS] = y[u] + x[u];
  } else {
    for (int u = 0; u < U; u++) {
      const size_t i = base + (size_t)u * BS;
      if (i < nvec) o[i] = b[i] + a[i];
    }
  }
}

// LDS-staged element-wise reduce (north star: "LDS-staged partials"): operand
// `a` (and optionally `b`) arrives through LDS by LDS-DMA
// (global_load_lds_dwordx4, AUX = cache policy: 2 = nt), the other straight
// into registers; each wave reads back only its own lanes' bytes, so
// s_waitcnt vmcnt(0) orders it (no cross-wave barrier needed)
template <int U, int AUX, bool BOTH>
__global__ __launch_bounds__(256) void k_red_lds(const f4 *__restrict__ a, const f4 *b, f4 *o, size_t nvec) {
  __shared__ f4 sa[256 * U];
  __shared__ f4 sb[BOTH ? 256 * U : 1];
  const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  const int w = threadIdx.x >> 6;
  if (base + (U - 1) * 256 >= nvec) {
    for (int u = 0; u < U; u++) {
      const size_t i = base + (size_t)u * 256;
      if (i < nvec) o[i] = b[i] + a[i];
    }
    return;
  }
  typedef __attribute__((address_space(3))) void lds_t;
#pragma unroll
  for (int u = 0; u < U; u++) {
    __builtin_amdgcn_global_load_lds((const void *)(a + base + u * 256), (lds_t *)(sa + u * 256 + w * 64), 16, 0, AUX);
    if constexpr (BOTH)
      __builtin_amdgcn_global_load_lds((const void *)(b + base + u * 256), (lds_t *)(sb + u * 256 + w * 64), 16, 0, 0);
  }
  f4 y[U];
  if constexpr (!BOTH) {
#pragma unroll
    for (int u = 0; u < U; u++) y[u] = b[base + u * 256];
  }
  __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
  for (int u = 0; u < U; u++) {
    const f4 yy = BOTH ? sb[u * 256 + threadIdx.x] : y[u];
    o[base + u * 256] = yy + sa[u * 256 + threadIdx.x];
  }
}

struct Var {
  std::string name;
  std::function<void(int, hipStream_t)> run;  // argument: buffer set
};

static double median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  const int rounds = 7, iters = 20;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));

  // ---- (1) copy, 256 MiB fp32, 2 rotating sets (1 GiB, beyond the Infinity Cache)
  {
    const size_t N = 67108864, nvec = N / 4, bytes = N * 4;
    const int sets = 2;
    std::vector<u4 *> A(sets), O(sets);
    for (int k = 0; k < sets; k++) {
      CK(hipMalloc(&A[k], bytes));
      CK(hipMalloc(&O[k], bytes));
      bine_fill_pico(A[k], N, BINE_FLOAT, 1234 + k, nullptr);
      CK(hipMemset(O[k], 0, bytes));
    }
    CK(hipDeviceSynchronize());
    std::vector<Var> vars;
#define TILE(BS, U, NTL, NTS, TPW)                                                                          \
  vars.push_back({"tile bs" #BS " u" #U " ntl" #NTL " nts" #NTS " tpw" #TPW, [&, nvec](int k, hipStream_t st) { \
                    const size_t tiles = (nvec + (size_t)BS * U - 1) / ((size_t)BS * U);                    \
                    hipLaunchKernelGGL((k_copy_tile<BS, U, NTL, NTS, TPW>), dim3((unsigned)((tiles + TPW - 1) / TPW)), \
                                       dim3(BS), 0, st, A[k], O[k], nvec);                                   \
                  }})
#define GS(BS, U, NTL, NTS, PERCU)                                                                         \
  vars.push_back({"gs bs" #BS " u" #U " ntl" #NTL " nts" #NTS " " #PERCU "/cu", [&, nvec](int k, hipStream_t st) { \
                    hipLaunchKernelGGL((k_copy_gs<BS, U, NTL, NTS>), dim3((unsigned)(ncu * PERCU)), dim3(BS), 0, \
                                       st, A[k], O[k], nvec);                                                \
                  }})
    TILE(256, 4, 1, 0, 1);
    TILE(256, 4, 0, 0, 1);
    TILE(256, 4, 1, 1, 1);
    TILE(256, 4, 0, 1, 1);
    TILE(256, 8, 1, 0, 1);
    TILE(256, 8, 1, 1, 1);
    TILE(256, 2, 1, 0, 1);
    TILE(256, 16, 1, 0, 1);
    TILE(512, 4, 1, 0, 1);
    TILE(512, 8, 1, 0, 1);
    TILE(1024, 4, 1, 0, 1);
    TILE(256, 4, 1, 0, 4);
    GS(256, 4, 1, 0, 8);
    GS(256, 8, 1, 0, 8);
    GS(512, 4, 1, 0, 4);
    GS(256, 4, 1, 1, 8);
    GS(1024, 4, 1, 0, 2);
#define XCD(BS, U, NTL, NTS, MAP)                                                                          \
  vars.push_back({"xcd bs" #BS " u" #U " ntl" #NTL " nts" #NTS " map" #MAP, [&, nvec](int k, hipStream_t st) {  \
                    const unsigned tiles = (unsigned)((nvec + (size_t)BS * U - 1) / ((size_t)BS * U));      \
                    const unsigned grid = MAP == 0 ? tiles : (tiles + 15) / 16 * 16;                       \
                    hipLaunchKernelGGL((k_copy_xcd<BS, U, NTL, NTS, MAP>), dim3(grid), dim3(BS), 0, st, A[k], O[k], \
                                       nvec, tiles);                                                        \
                  }})
    XCD(256, 8, 1, 1, 0);
    XCD(256, 8, 1, 1, 1);
    XCD(256, 8, 1, 1, 2);
    XCD(256, 4, 1, 1, 1);
    vars.push_back({"hipMemcpyAsync D2D", [&](int k, hipStream_t st) {
                      (void)hipMemcpyAsync(O[k], A[k], bytes, hipMemcpyDeviceToDevice, st);
                    }});
    std::vector<std::vector<float>> ms(vars.size());
    for (int r = 0; r < rounds; r++)
      for (size_t v = 0; v < vars.size(); v++) {
        for (int i = 0; i < 2; i++) vars[v].run(i % sets, s);
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; i++) vars[v].run(i % sets, s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms[v].push_back(t / iters);
      }
    printf("== copy 256 MiB fp32 (algorithmic 2*S = %zu B per launch)\n", 2 * bytes);
    for (size_t v = 0; v < vars.size(); v++) {
      const double med = median(ms[v]);
      printf("%-36s us=%9.2f  2S/t GB/s=%8.1f  S/t (algbw) GB/s=%8.1f  min us=%9.2f\n", vars[v].name.c_str(),
             med * 1e3, 2.0 * bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 1e9,
             *std::min_element(ms[v].begin(), ms[v].end()) * 1e3);
    }
    // correctness of every variant on set 0
    std::vector<unsigned> h(N), g(N);
    CK(hipMemcpy(h.data(), A[0], bytes, hipMemcpyDeviceToHost));
    for (size_t v = 0; v < vars.size(); v++) {
      CK(hipMemset(O[0], 0, bytes));
      vars[v].run(0, s);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(g.data(), O[0], bytes, hipMemcpyDeviceToHost));
      if (g != h) printf("MISMATCH %s\n", vars[v].name.c_str());
    }
    for (int k = 0; k < sets; k++) {
      CK(hipFree(A[k]));
      CK(hipFree(O[k]));
    }
  }

  // ---- (2) small-window fp32 SUM reduce: out = b + a, windows 256 KiB .. 16 MiB,
  // 16 rotating windows spread over a 1 GiB region (cold in L2 like a pipeline's)
  {
    const size_t region = (size_t)1 << 30;
    f4 *Ra, *Rb;
    CK(hipMalloc(&Ra, region));
    CK(hipMalloc(&Rb, region));
    bine_fill_pico(Ra, region / 4, BINE_FLOAT, 7, nullptr);
    bine_fill_pico(Rb, region / 4, BINE_FLOAT, 8, nullptr);
    CK(hipDeviceSynchronize());
    const size_t wins[] = {256 << 10, 1 << 20, 4 << 20, 16 << 20};
    for (size_t W : wins) {
      const size_t nvec = W / 16;
      auto off = [&](int k) { return (size_t)k * (region / 16) / sizeof(f4); };
      std::vector<Var> vars;
#define RED(BS, U)                                                                                 \
  vars.push_back({"red bs" #BS " u" #U, [&, nvec](int k, hipStream_t st) {                          \
                    const size_t tiles = (nvec + (size_t)BS * U - 1) / ((size_t)BS * U);            \
                    hipLaunchKernelGGL((k_red<BS, U>), dim3((unsigned)tiles), dim3(BS), 0, st,      \
                                       Ra + off(k), Rb + off(k), Rb + off(k), nvec);               \
                  }})
      RED(256, 4);
      RED(256, 2);
      RED(256, 1);
      RED(128, 1);
      RED(64, 1);
      RED(512, 1);
      vars.push_back({"library bine_reduce_local", [&, nvec](int k, hipStream_t st) {
                        bine_reduce_local(Ra + off(k), Rb + off(k), nvec * 4, BINE_FLOAT, BINE_SUM, st);
                      }});
      std::vector<std::vector<float>> ms(vars.size());
      const int it = 64;
      for (int r = 0; r < rounds; r++)
        for (size_t v = 0; v < vars.size(); v++) {
          for (int i = 0; i < 4; i++) vars[v].run(i % 16, s);
          CK(hipEventRecord(e0, s));
          for (int i = 0; i < it; i++) vars[v].run(i % 16, s);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float t;
          CK(hipEventElapsedTime(&t, e0, e1));
          ms[v].push_back(t / it);
        }
      printf("== reduce window %zu KiB (3*W = %zu B per launch; back-to-back launches, boundary included)\n", W >> 10,
             3 * W);
      for (size_t v = 0; v < vars.size(); v++) {
        const double med = median(ms[v]);
        printf("%-36s us=%8.2f  GB/s=%8.1f\n", vars[v].name.c_str(), med * 1e3, 3.0 * W / (med * 1e-3) / 1e9);
      }
    }
    CK(hipFree(Ra));
    CK(hipFree(Rb));
  }
  // ---- (3) C2 (64 MiB fp32 inout += in, 4 rotating sets): the library's
  // register-only kernel vs LDS-staged variants
  {
    const size_t N = 16777216, nvec = N / 4;
    const int sets = 4;
    std::vector<f4 *> A(sets), B(sets);
    for (int k = 0; k < sets; k++) {
      CK(hipMalloc(&A[k], N * 4));
      CK(hipMalloc(&B[k], N * 4));
      bine_fill_pico(A[k], N, BINE_FLOAT, 1234 + 2 * k, nullptr);
      bine_fill_pico(B[k], N, BINE_FLOAT, 1235 + 2 * k, nullptr);
    }
    CK(hipDeviceSynchronize());
    std::vector<Var> vars;
    vars.push_back({"library bine_reduce_local (registers)", [&](int k, hipStream_t st) {
                      bine_reduce_local(A[k], B[k], N, BINE_FLOAT, BINE_SUM, st);
                    }});
#define LDSV(U, AUX, BOTH)                                                                                     \
  vars.push_back({std::string("lds-dma u" #U " aux" #AUX) + (BOTH ? " +b" : ""), [&](int k, hipStream_t st) { \
                    hipLaunchKernelGGL((k_red_lds<U, AUX, BOTH>), dim3((unsigned)((nvec + 256 * U - 1) / (256 * U))), \
                                       dim3(256), 0, st, A[k], B[k], B[k], nvec);                              \
                  }})
    LDSV(4, 0, false);
    LDSV(4, 2, false);
    LDSV(8, 2, false);
    LDSV(4, 2, true);
    LDSV(2, 2, true);
    std::vector<std::vector<float>> ms(vars.size());
    for (int r = 0; r < rounds; r++)
      for (size_t v = 0; v < vars.size(); v++) {
        for (int i = 0; i < 4; i++) vars[v].run(i % sets, s);
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 40; i++) vars[v].run(i % sets, s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms[v].push_back(t / 40);
      }
    printf("== C2 reduce 64 MiB fp32 (3*S = %zu B per launch): registers vs LDS-staged\n", 3 * N * 4);
    for (size_t v = 0; v < vars.size(); v++) {
      const double med = median(ms[v]);
      printf("%-40s us=%8.2f  GB/s=%8.1f\n", vars[v].name.c_str(), med * 1e3, 3.0 * N * 4 / (med * 1e-3) / 1e9);
    }
    // parity of the LDS variants vs the library on fresh inputs
    std::vector<float> ref(N), got(N);
    for (size_t v = 0; v < vars.size(); v++) {
      bine_fill_pico(A[0], N, BINE_FLOAT, 1234, nullptr);
      bine_fill_pico(B[0], N, BINE_FLOAT, 1235, nullptr);
      vars[v].run(0, s);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(v ? got.data() : ref.data(), B[0], N * 4, hipMemcpyDeviceToHost));
      if (v && got != ref) printf("MISMATCH %s\n", vars[v].name.c_str());
    }
  }
  (void)argc;
  (void)argv;
  return 0;
}
