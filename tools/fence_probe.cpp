// fence_probe.cpp -- what the direct transport's per-workgroup protocol costs
// on top of a plain copy (profiles/r4_dm_stamps_p2_sweep.txt
// shows its copy workgroups 4-5x slower per byte than the same grid-strided
// copy alone, profiles/r4_vmm_bw_probe.txt).  One 16 MiB message (the
// transport's slot) copied by W grid-strided workgroups (4 x 16-B vectors per
// lane in flight, non-temporal), each workgroup finishing with
//   none   : nothing (the plain copy)
//   sys    : k_dm_move's ending -- system-scope release fence (buffer_wbl2
//            sc0 sc1 + wait), barrier, thread 0's system-scope atomic add on
//            the message's arrival counter
//   agent  : the same at agent scope
//   count  : the barrier and the atomic add only, no fence
//   acq+sys: sys plus k_dm_move's opening system-scope acquire fence
//   wt     : stores written through to memory (sc0 sc1 nt), then the stores'
//            acknowledgements awaited (vmcnt 0), the barrier and a RELAXED
//            system-scope atomic add: no L2 write-back at all
//   wt+scld: wt with system-coherent loads (sc0 sc1 nt) as well -- what a
//            reader needs to see a peer's written-through data without an
//            acquire invalidation
// Median of 9 x 20 launches back to back on one stream; also W = 4 x 128 and
// two streams each copying its own message concurrently.  One JSON line each.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/fence_probe.cpp -o tools/bin/fence_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

enum { NONE = 0, SYS = 1, AGENT = 2, COUNT = 3, ACQSYS = 4, WT = 5, WTLD = 6 };

// a 16-B store written through to memory (system-coherent: sc0 sc1), non-temporal,
// through a buffer resource (compiler-scheduled; cache policy sc0|sc1|nt = 19)
__device__ __forceinline__ void st_wt(u32x4 *p, u32x4 v) {
  const uint64_t b = (uint64_t)(uintptr_t)p;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)b, (short)0, 16, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, 0, 0, 19);
}
// (round 4's first version had a system-coherent LOAD in inline asm here:
// unsafe -- the compiler does not see the load's pending result and reused
// its registers, which faulted the transport kernels; wt+scld now uses plain
// non-temporal loads)
__device__ __forceinline__ u32x4 ld_sc(const u32x4 *p) { return __builtin_nontemporal_load(p); }

template <int MODE>
__global__ __launch_bounds__(256) void k_msg(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t nvec,
                                             unsigned *cnt) {
  if (MODE == ACQSYS) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  constexpr int U = 4;
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t b0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; b0 < nvec; b0 += stride) {
    u32x4 x[U];
    if (MODE == WTLD) {  // (nvec is a multiple of the tile here)
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = ld_sc(s + b0 + u * 256);
    } else {
#pragma unroll
      for (int u = 0; u < U; u++)
        if (b0 + u * 256 < nvec) x[u] = __builtin_nontemporal_load(s + b0 + u * 256);
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 256 < nvec) {
        if (MODE == WT || MODE == WTLD) st_wt(d + b0 + u * 256, x[u]);
        else __builtin_nontemporal_store(x[u], d + b0 + u * 256);
      }
  }
  if (MODE == NONE) return;
  if (MODE == WT || MODE == WTLD) {
    // written through: wait for the stores' acknowledgements, then count in
    // with a relaxed system-scope atomic -- no L2 write-back
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (MODE == SYS || MODE == ACQSYS) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (MODE == AGENT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (MODE == AGENT) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int MODE>
static void launch(const u32x4 *s, u32x4 *d, size_t nvec, unsigned *cnt, int wgs, hipStream_t st) {
  hipLaunchKernelGGL(k_msg<MODE>, dim3(wgs), dim3(256), 0, st, s, d, nvec, cnt);
}

int main() {
  const size_t B = 16u << 20, nvec = B / 16;
  u32x4 *s[2], *d[2];
  unsigned *cnt;
  for (int i = 0; i < 2; i++) {
    CK(hipMalloc(&s[i], B));
    CK(hipMalloc(&d[i], B));
    CK(hipMemset(s[i], 1, B));
  }
  CK(hipMalloc(&cnt, 4096));
  CK(hipMemset(cnt, 0, 4096));
  hipStream_t st[2];
  for (auto &x : st) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char *names[7] = {"none", "sys", "agent", "count", "acq+sys", "wt", "wt+scld"};
  auto run = [&](int mode, int wgs, int streams) -> double {
    auto one = [&](int i) {
      switch (mode) {
        case NONE: launch<NONE>(s[i], d[i], nvec, cnt + 64 * i, wgs, st[i]); break;
        case SYS: launch<SYS>(s[i], d[i], nvec, cnt + 64 * i, wgs, st[i]); break;
        case AGENT: launch<AGENT>(s[i], d[i], nvec, cnt + 64 * i, wgs, st[i]); break;
        case COUNT: launch<COUNT>(s[i], d[i], nvec, cnt + 64 * i, wgs, st[i]); break;
        case ACQSYS: launch<ACQSYS>(s[i], d[i], nvec, cnt + 64 * i, wgs, st[i]); break;
        case WT: launch<WT>(s[i], d[i], nvec, cnt + 64 * i, wgs, st[i]); break;
        default: launch<WTLD>(s[i], d[i], nvec, cnt + 64 * i, wgs, st[i]); break;
      }
    };
    std::vector<float> ms;
    for (int r = 0; r < 10; r++) {
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(a, st[0]);
      if (streams == 2) (void)hipStreamWaitEvent(st[1], a, 0);
      for (int k = 0; k < 20; k++)
        for (int i = 0; i < streams; i++) one(i);
      if (streams == 2) {
        hipEvent_t j;
        (void)hipEventCreate(&j);
        (void)hipEventRecord(j, st[1]);
        (void)hipStreamWaitEvent(st[0], j, 0);
        (void)hipEventDestroy(j);
      }
      (void)hipEventRecord(b, st[0]);
      (void)hipEventSynchronize(b);
      float t;
      (void)hipEventElapsedTime(&t, a, b);
      if (r) ms.push_back(t / 20);  // first round: warm-up
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
  };
  for (int streams : {1, 2})
    for (int wgs : {32, 128, 512})
      for (int mode = 0; mode < 7; mode++) {
        const double ms = run(mode, wgs, streams);
        printf("{\"ending\": \"%s\", \"workgroups\": %d, \"streams\": %d, \"us_per_message\": %.2f, "
               "\"TBps_rw\": %.3f}\n",
               names[mode], wgs, streams, ms * 1e3, 2.0 * B * streams / (ms * 1e-3) / 1e12);
        fflush(stdout);
      }
  return 0;
}
