// Do independent branches of a captured HIP graph run concurrently on MI355X, and does a weight prefetch that
// runs beside a latency-bound kernel make the next weight-streaming kernel faster?
//   busy(64 blocks, ~T us)  : stand-in for the talker decode attention (64 (row, kv head) blocks on 256 CUs)
//   prefetch(nb blocks)     : reads a weight buffer once (plain loads -> allocates in L2 / Infinity Cache)
//   stream(768 blocks)      : a gate-up-sized weight stream (48 MiB, nt loads like the decode GEMV) + tiny output
// Graphs (each replayed over 28 distinct weight buffers, so HBM is cold for every stream):
//   A: busy -> stream                      (serial, as today)
//   B: fork{busy | prefetch(W)} -> stream  (prefetch of the stream's own buffer beside busy)
//   C: busy ; prefetch ; stream in series   (prefetch not overlapped: its own cost)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/graph_overlap.hip -o tools/graph_overlap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

__global__ void busy(unsigned* out, int iters) {
  unsigned x = threadIdx.x + blockIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
  if (x == 12345u) out[0] = x;
}

// every wave reads `per` consecutive 1 KiB pieces, 4 in flight
template <bool NT>
__global__ __launch_bounds__(256) void stream(const u32x4_t* __restrict__ w, unsigned* out, int per) {
  const int lane = threadIdx.x & 63;
  const long long wid = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u32x4_t* p = w + wid * per * 64 + lane;
  unsigned acc = 0;
  for (int c = 0; c < per; c += 4) {
    u32x4_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (NT) v[u] = __builtin_nontemporal_load(p + (long long)(c + u) * 64);
      else v[u] = p[(long long)(c + u) * 64];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[wid] = acc;
}

int main() {
  const size_t bytes = 48u << 20;
  const int NBUF = 28;
  std::vector<u32x4_t*> bufs(NBUF);
  for (auto& b : bufs) { CK(hipMalloc(&b, bytes)); CK(hipMemset(b, 1, bytes)); }
  unsigned* out; CK(hipMalloc(&out, 1 << 20));
  const int per = 16, blocks = (int)(bytes / 1024 / per / 4);  // 768 blocks x 4 waves x 16 KiB
  hipStream_t s0, s1; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t fork, join, e0, e1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int busy_iters : {0, 4000, 8000}) {
    for (int mode = 0; mode < 4; ++mode) {
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
      for (int i = 0; i < NBUF; ++i) {
        if (mode == 1) {  // B: prefetch beside busy
          CK(hipEventRecord(fork, s0));
          CK(hipStreamWaitEvent(s1, fork, 0));
          hipLaunchKernelGGL(busy, dim3(64), dim3(512), 0, s0, out, busy_iters);
          hipLaunchKernelGGL(stream<false>, dim3(blocks), dim3(256), 0, s1, bufs[i], out, per);
          CK(hipEventRecord(join, s1));
          CK(hipStreamWaitEvent(s0, join, 0));
        } else if (mode == 3) {  // D: busy beside an unrelated stream (concurrency check only, no consumer)
          CK(hipEventRecord(fork, s0));
          CK(hipStreamWaitEvent(s1, fork, 0));
          hipLaunchKernelGGL(busy, dim3(64), dim3(512), 0, s0, out, busy_iters);
          hipLaunchKernelGGL(stream<true>, dim3(blocks), dim3(256), 0, s1, bufs[(i + 7) % NBUF], out, per);
          CK(hipEventRecord(join, s1));
          CK(hipStreamWaitEvent(s0, join, 0));
        } else {
          hipLaunchKernelGGL(busy, dim3(64), dim3(512), 0, s0, out, busy_iters);
          if (mode == 2) hipLaunchKernelGGL(stream<false>, dim3(blocks), dim3(256), 0, s0, bufs[i], out, per);
        }
        if (mode != 3) hipLaunchKernelGGL(stream<true>, dim3(blocks), dim3(256), 0, s0, bufs[i], out, per);
      }
      CK(hipStreamEndCapture(s0, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s0)); CK(hipStreamSynchronize(s0));
      CK(hipEventRecord(e0, s0));
      for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s0));
      CK(hipEventRecord(e1, s0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      const char* names[] = {"A busy -> stream", "B fork{busy | prefetch} -> stream", "C busy -> prefetch -> stream",
                             "D fork{busy | other stream}"};
      printf("busy_iters %5d  %-36s %8.2f us per (busy, stream) pair\n", busy_iters, names[mode], ms * 1e3 / (5 * NBUF));
      fflush(stdout);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  }
  printf("done\n");
  return 0;
}
