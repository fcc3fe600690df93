// Which XCD does block b of each launch land on, along a graph-captured chain of launches?  If the round-robin
// offset (the XCD of block 0) carries over from one launch to the next when grids are multiples of 8, a kernel can
// warm the L2 of the XCD on which the NEXT kernel's block b will read its weights (speed only, never correctness).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xcd_probe.hip -o tools/xcd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void who(int* out) {
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    out[blockIdx.x] = (int)(x & 0xF);
  }
}

int main() {
  const int grids[] = {256, 384, 64, 256, 128, 256, 100, 256, 256, 33, 256, 384, 256};
  const int NL = sizeof(grids) / sizeof(grids[0]);
  std::vector<int*> outs(NL);
  for (auto& o : outs) CK(hipMalloc(&o, 4096 * sizeof(int)));
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int mode = 0; mode < 2; ++mode) {
    hipGraph_t g; hipGraphExec_t ge;
    if (mode == 1) CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int rep = 0; rep < (mode == 1 ? 1 : 1); ++rep)
      for (int i = 0; i < NL; ++i) hipLaunchKernelGGL(who, dim3(grids[i]), dim3(256), 0, s, outs[i]);
    if (mode == 1) {
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    for (int trial = 0; trial < 4; ++trial) {
      if (mode == 1) CK(hipGraphLaunch(ge, s));
      else for (int i = 0; i < NL; ++i) hipLaunchKernelGGL(who, dim3(grids[i]), dim3(256), 0, s, outs[i]);
      CK(hipStreamSynchronize(s));
      printf("%s trial %d:", mode ? "graph" : "eager", trial);
      for (int i = 0; i < NL; ++i) {
        std::vector<int> h(grids[i]);
        CK(hipMemcpy(h.data(), outs[i], grids[i] * sizeof(int), hipMemcpyDeviceToHost));
        // XCD of block 0 and whether b -> XCD is (b + off) % 8 for every block
        const int off = h[0];
        bool rr = true;
        for (int b = 0; b < grids[i]; ++b) rr = rr && (h[b] == (b + off) % 8);
        printf(" [G%d x0=%d%s]", grids[i], off, rr ? "" : " !rr");
      }
      printf("\n");
      fflush(stdout);
    }
  }
  return 0;
}
