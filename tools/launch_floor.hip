// Per-launch floor of a graph-captured chain of dependent launches on MI355X: empty kernels of various grid and
// block sizes, and the same with one 4-byte store per block (a dirty line for the end-of-kernel release) or one
// load of a line the previous launch wrote (the dependency the decode chain has).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void empty_k(float* p, int mode) {
  if (mode == 1 && threadIdx.x == 0) p[blockIdx.x * 32] = 1.f;                    // a dirty line per block
  if (mode == 2 && threadIdx.x == 0) {                                              // read the previous writes
    float v = p[((blockIdx.x * 7) % gridDim.x) * 32];
    p[blockIdx.x * 32] = v + 1.f;
  }
}

int main() {
  float* buf; CK(hipMalloc(&buf, 64 << 20)); CK(hipMemset(buf, 0, 64 << 20));
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int N = 200;
  const int grids[] = {1, 8, 64, 256, 512, 1024};
  const int blocks[] = {64, 256, 512, 1024};
  for (int mode = 0; mode < 3; ++mode)
    for (int g : grids)
      for (int b : blocks) {
        hipGraph_t gr; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(empty_k, dim3(g), dim3(b), 0, s, buf, mode);
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("mode %d (%s) grid %5d x block %5d: %6.2f us per launch\n", mode,
               mode == 0 ? "empty" : (mode == 1 ? "store" : "load+store"), g, b, ms * 1e3 / (10 * N));
        fflush(stdout);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(gr));
      }
  return 0;
}
