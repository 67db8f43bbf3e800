// vmm_ipc_probe.cpp -- can two processes sharing this box's one GPU map the
// same device allocation through the VMM API (hipMemCreate +
// hipMemExportToShareableHandle as a POSIX fd passed over a Unix socket +
// hipMemImportFromShareableHandle + hipMemMap)?  Round 1's legacy
// hipIpcOpenMemHandle path failed here (profiles/r1_ipc_probe.txt); the VMM
// path is what a peer-memory transport would use under the dmabuf IPC mode.
// The process forks BEFORE any HIP call.  Prints one JSON line.
//   hipcc -O2 -o tools/bin/vmm_ipc_probe tools/vmm_ipc_probe.cpp
#include <hip/hip_runtime.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <vector>

static const size_t kBytes = 64u << 20;

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
  if (!c) return -1;
  int fd;
  memcpy(&fd, CMSG_DATA(c), sizeof fd);
  return fd;
}

static hipMemAllocationProp prop() {
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  return p;
}

static void *map(hipMemGenericAllocationHandle_t h, size_t size, int *err) {
  void *va = nullptr;
  hipError_t e = hipMemAddressReserve(&va, size, 0, nullptr, 0);
  if (e == hipSuccess) e = hipMemMap(va, size, 0, h, 0);
  hipMemAccessDesc d{};
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  if (e == hipSuccess) e = hipMemSetAccess(va, size, &d, 1);
  *err = (int)e;
  return e == hipSuccess ? va : nullptr;
}

int main(int argc, char **argv) {
  // "ptr": pass a POINTER to the descriptor as hipMemImportFromShareableHandle's
  // osHandle (some HIP runtimes read it that way) instead of its value
  const bool by_ptr = argc > 1 && !strcmp(argv[1], "ptr");
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv)) return 2;
  const pid_t pid = fork();
  if (pid == 0) {  // peer
    close(sv[0]);
    int fd = recv_fd(sv[1]);
    hipMemGenericAllocationHandle_t h;
    int imp = (int)hipMemImportFromShareableHandle(&h, by_ptr ? (void *)&fd : (void *)(intptr_t)fd,
                                                   hipMemHandleTypePosixFileDescriptor);
    int merr = -1;
    void *va = imp == 0 ? map(h, kBytes, &merr) : nullptr;
    int ok = 0;
    if (va) {
      std::vector<unsigned char> host(kBytes);
      ok = hipMemcpy(host.data(), va, kBytes, hipMemcpyDeviceToHost) == hipSuccess;
      for (size_t i = 0; ok && i < kBytes; i += 4093) ok = host[i] == (unsigned char)(i * 7);
      (void)hipMemset(va, 0x5A, kBytes);
      (void)hipDeviceSynchronize();
    }
    int msg[3] = {imp, merr, ok};
    (void)!write(sv[1], msg, sizeof msg);
    return 0;
  }
  close(sv[1]);
  hipMemAllocationProp p = prop();
  size_t gran = 0;
  (void)hipMemGetAllocationGranularity(&gran, &p, hipMemAllocationGranularityMinimum);
  hipMemGenericAllocationHandle_t h;
  int cr = (int)hipMemCreate(&h, kBytes, &p, 0);
  int fd = -1, ex = -1, merr = -1;
  void *va = nullptr;
  if (cr == 0) ex = (int)hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0);
  if (cr == 0) va = map(h, kBytes, &merr);
  if (va) {
    std::vector<unsigned char> host(kBytes);
    for (size_t i = 0; i < kBytes; i++) host[i] = (unsigned char)(i * 7);
    (void)hipMemcpy(va, host.data(), kBytes, hipMemcpyHostToDevice);
    (void)hipDeviceSynchronize();
  }
  send_fd(sv[0], fd);
  int msg[3] = {-9, -9, -9};
  (void)!read(sv[0], msg, sizeof msg);
  int owner_sees = 0;
  if (va) {
    unsigned char c = 0;
    (void)hipMemcpy(&c, (char *)va + 12345, 1, hipMemcpyDeviceToHost);
    owner_sees = c == 0x5A;
  }
  int st = 0;
  waitpid(pid, &st, 0);
  int rt = 0;
  (void)hipRuntimeGetVersion(&rt);
  printf("{\"hip_runtime\": %d, \"by_ptr\": %d, \"granularity\": %zu, \"create_rc\": %d, \"export_rc\": %d, \"owner_map_rc\": %d, \"peer_import_rc\": %d, "
         "\"peer_map_rc\": %d, \"peer_reads_owner_bytes\": %d, \"owner_sees_peer_writes\": %d, \"peer_exit\": %d}\n",
         rt, (int)by_ptr, gran, cr, ex, merr, msg[0], msg[1], msg[2], owner_sees, WEXITSTATUS(st));
  return 0;
}
