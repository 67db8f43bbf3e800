// visibility_probe.cpp -- does a direct-transport flag poll see a flag that
// another workgroup published?
//
// The 8-rank one-GPU rehearsals time out with the waited-for flag IN MEMORY
// at the time-out dump (DirectState::describe after the drain) although its
// producer published it long before: the poll kept reading the old value.
// This probe puts one producer workgroup and C consumer workgroups (spread
// over the XCDs: blocks are dealt round-robin) on the flag, the consumers
// polling BEFORE the producer's store (so whatever caches a poll allocates
// into already hold the old value), the rest of the chip idle -- no
// streaming traffic that would evict a stale line.  The flag lives in a VMM
// allocation (hipMemCreate, as the inboxes), and the producer stores through
// the SAME mapping or through a SECOND mapping of the same memory (how a peer
// process reaches an inbox).  Poll forms: the transport's relaxed
// system-scope load (sc0 sc1), an agent-scope relaxed load (sc1), a relaxed
// system-scope atomic add of 0, and the system-scope load preceded by a
// system-scope acquire fence every iteration.  Per case: how many consumers
// saw the flag within the limit, and the slowest latency.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/visibility_probe.cpp -o tools/bin/visibility_probe
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

enum Poll { kSys = 0, kAgent = 1, kAtomic = 2, kFenced = 3 };

__device__ __forceinline__ uint64_t poll(const uint64_t *p, int kind) {
  switch (kind) {
    case kAgent: return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    case kAtomic:
      return __hip_atomic_fetch_add(const_cast<uint64_t *>(p), (uint64_t)0, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_SYSTEM);
    case kFenced:
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    default: return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// block 0 publishes `val` at `prod` after `delay` ticks; every other block
// polls `cons` (the same flag, maybe through another mapping) until it sees
// val or `limit` ticks pass; out[b] = ticks from the publish to the sighting
// (0: not seen)
__global__ void k_vis(uint64_t *prod, const uint64_t *cons, uint64_t val, unsigned long long delay,
                      unsigned long long limit, int kind, unsigned long long *out, unsigned long long *t_pub) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  if (blockIdx.x == 0) {
    while (wall_clock64() - t0 < delay) __builtin_amdgcn_s_sleep(8);
    const unsigned long long tp = wall_clock64();
    __hip_atomic_store(prod, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(t_pub, tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  unsigned long long seen = 0;
  while (wall_clock64() - t0 < limit) {
    if (poll(cons, kind) >= val) {
      seen = wall_clock64();
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  out[blockIdx.x] = seen;
}

int main() {
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &p, hipMemAllocationGranularityRecommended));
  const size_t sz = gran ? gran : (2 << 20);
  hipMemGenericAllocationHandle_t h;
  CK(hipMemCreate(&h, sz, &p, 0));
  void *va[2] = {nullptr, nullptr};
  hipMemAccessDesc d{};
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  for (auto &v : va) {
    CK(hipMemAddressReserve(&v, sz, 0, nullptr, 0));
    CK(hipMemMap(v, sz, 0, h, 0));
    CK(hipMemSetAccess(v, sz, &d, 1));
  }
  CK(hipMemset(va[0], 0, sz));
  const int blocks = 65;  // 1 producer + 64 consumers: 8 per XCD
  unsigned long long *out = nullptr, *tp = nullptr;
  CK(hipMalloc(&out, blocks * sizeof(unsigned long long)));
  CK(hipMalloc(&tp, sizeof(unsigned long long)));
  const unsigned long long delay = (unsigned long long)khz * 2;   // 2 ms: every consumer polls first
  const unsigned long long limit = (unsigned long long)khz * 200; // 0.2 s
  const char *kinds[] = {"sys (sc0 sc1 load)", "agent (sc1 load)", "atomic add 0 (sys)", "acquire + sys load"};
  uint64_t val = 0;
  for (int alias = 0; alias < 2; alias++)
    for (int kind = 0; kind < 4; kind++)
      for (int rep = 0; rep < 3; rep++) {
        val++;
        CK(hipMemset(out, 0, blocks * sizeof(unsigned long long)));
        uint64_t *flag_c = (uint64_t *)va[0] + 16 * (val % 64);   // a fresh 128-B line each time
        uint64_t *flag_p = (uint64_t *)va[alias] + 16 * (val % 64);
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_vis, dim3(blocks), dim3(64), 0, 0, flag_p, flag_c, val, delay, limit, kind, out, tp);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> h(blocks);
        unsigned long long t_pub = 0;
        CK(hipMemcpy(h.data(), out, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        CK(hipMemcpy(&t_pub, tp, sizeof t_pub, hipMemcpyDeviceToHost));
        int seen = 0;
        double worst = 0;
        for (int b = 1; b < blocks; b++)
          if (h[b]) {
            seen++;
            const double us = (double)(h[b] - t_pub) / (khz * 1e-3);
            if (us > worst) worst = us;
          }
        printf("{\"producer_mapping\": \"%s\", \"poll\": \"%s\", \"rep\": %d, \"consumers\": %d, \"saw_flag\": %d, "
               "\"slowest_us\": %.2f}\n",
               alias ? "second mapping" : "same mapping", kinds[kind], rep, blocks - 1, seen, worst);
        fflush(stdout);
      }
  return 0;
}
