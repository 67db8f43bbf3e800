// graph_fork_repro.cpp -- a libbine-free reproduction of the hipGraphLaunch
// SIGSEGV of round 3.  A graph with two parallel branches
// (stream A forks stream B through an event, each branch runs a kernel, A
// joins B) is captured, instantiated and launched.  The crash recorded in
// libbine (profiles/r4_rs_graph_segv_rank.txt) is a read past the end of the
// parallel-stream vector in hip::Graph::UpdateStreams (called from
// GraphExec::Run <- hipGraphLaunch), reached when every parallel stream shares
// the launch stream's hardware queue -- always the case under
// GPU_MAX_HW_QUEUES=1.  Prints "GRAPH_FORK ok" when the replays ran.
//   hipcc -O2 --offload-arch=gfx950 tools/graph_fork_repro.cpp -o tools/bin/graph_fork_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)

__global__ void k_add(float *x, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += v;
}

int main() {
  const int n = 1 << 20;
  float *x, *y;
  CK(hipMalloc(&x, n * sizeof(float)));
  CK(hipMalloc(&y, n * sizeof(float)));
  CK(hipMemset(x, 0, n * sizeof(float)));
  CK(hipMemset(y, 0, n * sizeof(float)));
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  int rt = 0;
  CK(hipRuntimeGetVersion(&rt));
  const char *q = getenv("GPU_MAX_HW_QUEUES");
  printf("HIP runtime %d, GPU_MAX_HW_QUEUES=%s\n", rt, q ? q : "(default)");
  fflush(stdout);
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(A, hipStreamCaptureModeThreadLocal));
  CK(hipEventRecord(fork, A));
  CK(hipStreamWaitEvent(B, fork, 0));
  hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, B, y, n, 1.0f);
  hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, A, x, n, 2.0f);
  CK(hipEventRecord(join, B));
  CK(hipStreamWaitEvent(A, join, 0));
  CK(hipStreamEndCapture(A, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  printf("captured and instantiated; launching\n");
  fflush(stdout);
  for (int k = 0; k < 3; k++) CK(hipGraphLaunch(ge, A));
  CK(hipStreamSynchronize(A));
  float hx = 0, hy = 0;
  CK(hipMemcpy(&hx, x + 7, sizeof hx, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hy, y + 7, sizeof hy, hipMemcpyDeviceToHost));
  printf("GRAPH_FORK %s (x = %g, y = %g after 3 replays)\n", hx == 6.0f && hy == 3.0f ? "ok" : "WRONG", hx, hy);
  return hx == 6.0f && hy == 3.0f ? 0 : 1;
}
