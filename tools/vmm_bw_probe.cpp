// vmm_bw_probe.cpp -- how fast kernels read and write the direct transport's
// kind of memory (k_dm_move / k_dm_move_tree run far below
// k_copy on one GPU).  The transport's inbox is a VMM allocation
// (hipMemCreate, exportable as a POSIX descriptor) mapped by its owner and,
// through the descriptor, by every peer process.  This probe forks BEFORE any
// HIP call; the parent exports an inbox-like allocation, the child imports it
// (a peer's view) and times a 256 MiB copy kernel between:
//   M   hipMalloc memory
//   E   the child's own exportable VMM allocation (an inbox as its owner maps it)
//   I   the parent's allocation imported by the child (a peer's inbox)
//   V   a non-exportable VMM allocation
// with non-temporal and plain loads / stores, on a full grid (8192 x 256, 8
// vectors per lane, k_copy's shape) and on 32 / 128 / 512 grid-strided
// workgroups (the transport's per-message shape).  Median of 7 x 5 launches.
// One JSON line per case.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/vmm_bw_probe.cpp -o tools/bin/vmm_bw_probe
#include <hip/hip_runtime.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

static const size_t kBytes = 256u << 20;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      _exit(2);                                                                            \
    }                                                                                      \
  } while (0)

static int send_fd(int sock, int fd) {
  char b = 0;
  iovec io{&b, 1};
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  cmsghdr *c = CMSG_FIRSTHDR(&m);
  c->cmsg_level = SOL_SOCKET;
  c->cmsg_type = SCM_RIGHTS;
  c->cmsg_len = CMSG_LEN(sizeof(int));
  memcpy(CMSG_DATA(c), &fd, sizeof fd);
  return sendmsg(sock, &m, 0) == 1 ? 0 : -1;
}

static int recv_fd(int sock) {
  char b;
  iovec io{&b, 1};
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  if (recvmsg(sock, &m, 0) != 1) return -1;
  cmsghdr *c = CMSG_FIRSTHDR(&m);
  if (!c || c->cmsg_type != SCM_RIGHTS) return -1;
  int fd;
  memcpy(&fd, CMSG_DATA(c), sizeof fd);
  return fd;
}

static void *map(hipMemGenericAllocationHandle_t h, size_t n) {
  void *p = nullptr;
  CK(hipMemAddressReserve(&p, n, 0, nullptr, 0));
  CK(hipMemMap(p, n, 0, h, 0));
  hipMemAccessDesc d{};
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(p, n, &d, 1));
  return p;
}

static hipMemGenericAllocationHandle_t create(size_t n, bool exportable) {
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  p.requestedHandleType = exportable ? hipMemHandleTypePosixFileDescriptor : hipMemHandleTypeNone;
  hipMemGenericAllocationHandle_t h;
  CK(hipMemCreate(&h, n, &p, 0));
  return h;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// k_copy's shape: one tile of 8 vectors per lane per workgroup (nwg = 0), or
// grid-strided over nwg workgroups with 4 vectors per lane in flight (the
// transport's shape)
template <bool NT>
__global__ __launch_bounds__(256) void k_cp(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t nvec) {
  constexpr int U = 8;
  const size_t b = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 x[U];
#pragma unroll
  for (int u = 0; u < U; u++)
    if (b + u * 256 < nvec) x[u] = NT ? __builtin_nontemporal_load(s + b + u * 256) : s[b + u * 256];
#pragma unroll
  for (int u = 0; u < U; u++)
    if (b + u * 256 < nvec) {
      if (NT) __builtin_nontemporal_store(x[u], d + b + u * 256);
      else d[b + u * 256] = x[u];
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_cp_strided(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t nvec) {
  constexpr int U = 4;
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t b0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; b0 < nvec; b0 += stride) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 256 < nvec) x[u] = NT ? __builtin_nontemporal_load(s + b0 + u * 256) : s[b0 + u * 256];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 256 < nvec) {
        if (NT) __builtin_nontemporal_store(x[u], d + b0 + u * 256);
        else d[b0 + u * 256] = x[u];
      }
  }
}

static double time_copy(void *dst, const void *src, bool nt, int nwg) {
  const size_t nvec = kBytes / 16;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ms;
  auto launch = [&] {
    const u32x4 *s = (const u32x4 *)src;
    u32x4 *d = (u32x4 *)dst;
    if (nwg == 0) {
      const unsigned g = (unsigned)((nvec + 2047) / 2048);
      if (nt) hipLaunchKernelGGL(k_cp<true>, dim3(g), dim3(256), 0, 0, s, d, nvec);
      else hipLaunchKernelGGL(k_cp<false>, dim3(g), dim3(256), 0, 0, s, d, nvec);
    } else {
      if (nt) hipLaunchKernelGGL(k_cp_strided<true>, dim3(nwg), dim3(256), 0, 0, s, d, nvec);
      else hipLaunchKernelGGL(k_cp_strided<false>, dim3(nwg), dim3(256), 0, 0, s, d, nvec);
    }
  };
  launch();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < 7; r++) {
    CK(hipEventRecord(a, 0));
    for (int k = 0; k < 5; k++) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float t;
    CK(hipEventElapsedTime(&t, a, b));
    ms.push_back(t / 5);
  }
  std::sort(ms.begin(), ms.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms[3];
}

int main() {
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv)) return 2;
  const pid_t pid = fork();
  if (pid == 0) {  // child: the measuring process
    close(sv[0]);
    const int fd = recv_fd(sv[1]);
    CK(hipSetDevice(0));
    hipMemGenericAllocationHandle_t hi;
    int fdv = fd;
    hipError_t e = hipMemImportFromShareableHandle(&hi, (void *)(intptr_t)fdv, hipMemHandleTypePosixFileDescriptor);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      CK(hipMemImportFromShareableHandle(&hi, (void *)&fdv, hipMemHandleTypePosixFileDescriptor));
    }
    void *I = map(hi, kBytes);
    void *E = map(create(kBytes, true), kBytes);
    void *V = map(create(kBytes, false), kBytes);
    void *M0, *M1;
    CK(hipMalloc(&M0, kBytes));
    CK(hipMalloc(&M1, kBytes));
    for (void *p : {I, E, V, M0, M1}) CK(hipMemset(p, 1, kBytes));
    CK(hipDeviceSynchronize());
    struct Case { const char *name; void *dst; const void *src; };
    const Case cases[] = {{"M->M", M1, M0}, {"E->M (pull from own inbox)", M1, E}, {"M->E", E, M0},
                          {"I->M (read a peer's inbox)", M1, I}, {"M->I (push into a peer's inbox)", I, M0},
                          {"V->M", M1, V}, {"M->V", V, M0}};
    for (const Case &c : cases)
      for (int nt = 1; nt >= 0; nt--)
        for (int nwg : {0, 32, 128, 512}) {
          if (!nt && nwg) continue;
          const double ms = time_copy(c.dst, c.src, nt != 0, nwg);
          printf("{\"copy\": \"%s\", \"nontemporal\": %s, \"workgroups\": \"%s\", \"us\": %.1f, "
                 "\"TBps_rw\": %.3f}\n",
                 c.name, nt ? "true" : "false", nwg ? std::to_string(nwg).c_str() : "full grid", ms * 1e3,
                 2.0 * kBytes / (ms * 1e-3) / 1e12);
          fflush(stdout);
        }
    char b = 1;
    (void)!write(sv[1], &b, 1);
    _exit(0);
  }
  close(sv[1]);
  CK(hipSetDevice(0));
  hipMemGenericAllocationHandle_t h = create(kBytes, true);
  void *p = map(h, kBytes);
  (void)p;
  int fd = -1;
  CK(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
  if (send_fd(sv[0], fd)) return 2;
  char b;
  (void)!read(sv[0], &b, 1);  // the child is done with our allocation
  int st = 0;
  waitpid(pid, &st, 0);
  return WIFEXITED(st) ? WEXITSTATUS(st) : 3;
}
