// residency_probe.cpp -- how many workgroups of k_dm_fused's footprint the GPU
// really keeps resident at once.  The
// direct transport's residency cap (bine_internal.h dm_fit_residency) takes
// CUs x hipOccupancyMaxActiveBlocksPerMultiprocessor / ranks sharing the GPU;
// with 8 ranks on one MI355X that is 1,280 / 8 = 160 workgroups per rank --
// the whole chip, no margin.  If fewer than the nominal count can be resident
// together, every k_dm_fused workgroup of the last rank to get a slot waits
// for a slot that only a waiter can free: a stall until the wait times out.
//
// Probe: N workgroups of 256 threads whose kernel needs 96 VGPRs (k_dm_fused's
// count, forced by a clobber) and a few bytes of LDS, spread over S streams
// (each its own HW queue when GPU_MAX_HW_QUEUES >= S); thread 0 of each
// counts itself in on a device counter and spins (with k_dm_fused's back-off)
// until all N have arrived or a time limit passes.  N completes iff all N are
// resident together.  One JSON line per (S, N); every workgroup exits (the
// limit), so a short capacity shows as a time-out, never as a hang.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/residency_probe.cpp -o tools/bin/residency_probe
#include <hip/hip_runtime.h>

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

__global__ __launch_bounds__(256) void k_resident(unsigned *cnt, unsigned n, unsigned long long ticks,
                                                  unsigned *timed_out) {
  __shared__ int lds_word;
  // k_dm_fused's register footprint: 96 VGPRs
  asm volatile("" ::: "v95");
  if (threadIdx.x == 0) {
    lds_word = 1;
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n) {
      if (wall_clock64() - t0 > ticks) {
        __hip_atomic_fetch_add(timed_out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (lds_word != 1) timed_out[1] = 1;  // keeps the LDS word
}

int main(int argc, char **argv) {
  int khz = 0, cus = 0, occ = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_resident, 256, 0));
  const int nominal = cus * occ;
  const unsigned long long ticks = (unsigned long long)khz * 300;  // 0.3 s
  unsigned *cnt = nullptr, *to = nullptr;
  CK(hipMalloc(&cnt, sizeof(unsigned)));
  CK(hipMalloc(&to, 2 * sizeof(unsigned)));
  std::vector<int> streams_list = {1, 2, 8};
  if (argc > 1) streams_list = {atoi(argv[1])};
  for (int S : streams_list) {
    std::vector<hipStream_t> st((size_t)S);
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int d : {-64, -8, -1, 0, 1, 8}) {
      const int n = nominal + d;
      if (n < S) continue;
      CK(hipMemset(cnt, 0, sizeof(unsigned)));
      CK(hipMemset(to, 0, 2 * sizeof(unsigned)));
      CK(hipDeviceSynchronize());
      // every stream's share launched back to back (k_dm_fused's case: one
      // launch per rank, all ranks' launches in flight together)
      for (int k = 0; k < S; k++) {
        const int share = n / S + (k < n % S ? 1 : 0);
        hipLaunchKernelGGL(k_resident, dim3((unsigned)share), dim3(256), 0, st[(size_t)k], cnt, (unsigned)n, ticks,
                           to);
      }
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      unsigned h[2] = {0, 0}, c = 0;
      CK(hipMemcpy(h, to, sizeof h, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&c, cnt, sizeof c, hipMemcpyDeviceToHost));
      printf("{\"streams\": %d, \"workgroups\": %d, \"nominal\": %d, \"cus\": %d, \"blocks_per_cu\": %d, "
             "\"all_resident\": %s, \"timed_out_workgroups\": %u, \"arrived\": %u}\n",
             S, n, nominal, cus, occ, h[0] == 0 ? "true" : "false", h[0], c);
      fflush(stdout);
    }
    for (auto &s : st) CK(hipStreamDestroy(s));
  }
  return 0;
}
