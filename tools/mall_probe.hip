// Go / no-go probe for an XCD-local code predictor: if every XCD decoded its own batch row, each
// XCD would stream all of the code predictor's weights per step (5 layers + lm_head, ~160 MB bf16), i.e. 8x the
// bytes of today's shared stream, out of the Infinity Cache (MALL).  How fast can 8 XCDs each read the same
// MALL-resident buffer?
//   mode 0 "shared":  256 blocks, block b reads chunk b of the buffer   -> every byte read once chip-wide
//   mode 1 "per-XCD": 256 blocks, block b reads chunk b / 8 (32 chunks) -> blocks b..b+7 sit on 8 XCDs (round-robin
//                     placement), so every XCD reads the whole buffer: 8x the bytes, all from MALL after warm-up
// Buffer 160 MiB (fits the 256 MiB Infinity Cache), 16-byte loads, 8 in flight per lane, 4 waves per block.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mall_probe.hip -o tools/mall_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

__global__ __launch_bounds__(256) void readk(const u32x4_t* __restrict__ buf, unsigned* out, long long chunk16, int mode) {
  const int b = blockIdx.x;
  const long long c = mode == 0 ? b : b / 8;
  const u32x4_t* p = buf + c * chunk16;
  unsigned acc = 0;
  for (long long i = threadIdx.x; i < chunk16; i += 256 * 8) {
    u32x4_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[min(i + u * 256, chunk16 - 1)];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u][0] ^ v[u][3];
  }
  if (acc == 0x9E3779B9u) out[b] = acc;
}

int main() {
  const size_t bytes = 160ull << 20;
  u32x4_t* buf; unsigned* out;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&out, 4096));
  CK(hipMemset(buf, 1, bytes));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {
    const int chunks = mode == 0 ? 256 : 32;
    const long long chunk16 = (long long)(bytes / 16 / chunks);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(readk, dim3(256), dim3(256), 0, 0, buf, out, chunk16, mode);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(readk, dim3(256), dim3(256), 0, 0, buf, out, chunk16, mode);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    const double moved = (double)bytes * (mode == 0 ? 1 : 8);
    printf("mode %d (%s): %.1f us per pass, %.0f MB read chip-wide -> %.2f TB/s\n", mode,
           mode == 0 ? "shared: each byte once" : "per-XCD: every XCD reads all", us, moved / 1e6, moved / us / 1e6);
  }
  return 0;
}
