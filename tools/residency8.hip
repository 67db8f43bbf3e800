// residency8.hip -- the cross-PROCESS form of tools/residency_probe.cpp
// (DESIGN.md 7.2): tools/residency8.py starts P processes on the one GPU,
// each launching its share of N workgroups of k_dm_fused's footprint (256
// threads, 96 VGPRs) that count themselves in on ONE counter in shared
// device memory (a torch tensor passed between the processes) and spin until
// all N arrived or a time limit passes.  N completes iff all N workgroups of
// all P processes are resident together.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 -shared -fPIC tools/residency8.hip -o tools/bin/libresidency8.so
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void k_resident8(unsigned *cnt, unsigned n, unsigned long long ticks,
                                                   unsigned *timed_out) {
  __shared__ int lds_word;
  asm volatile("" ::: "v95");  // k_dm_fused's register footprint
  if (threadIdx.x == 0) {
    lds_word = 1;
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < n) {
      if (wall_clock64() - t0 > ticks) {
        __hip_atomic_fetch_add(timed_out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (lds_word != 1) timed_out[1] = 1;
}

extern "C" int residency8_launch(void *cnt, unsigned n, unsigned blocks, double secs, void *timed_out,
                                 void *stream) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_resident8, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (unsigned *)cnt, n,
                     (unsigned long long)(secs * khz * 1000.0), (unsigned *)timed_out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
