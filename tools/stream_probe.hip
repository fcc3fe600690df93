// HBM streaming probe: how fast can decode-GEMV-shaped access patterns read a weight buffer on MI355X?
// Each wave reads `per` consecutive 1 KiB fragments (16 B per lane) of its tile, U loads in flight, XORs them and
// writes one dword per lane (vector store).  Buffers cycle through > 600 MB so every launch streams HBM.
// build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

template <int U, bool NT>
__global__ void probe(const u32x4_t* __restrict__ w, unsigned* out, int frags_per_wave) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long wid = (long long)blockIdx.x * (blockDim.x >> 6) + wv;
  const u32x4_t* p = w + wid * frags_per_wave * 64 + lane;
  unsigned acc = 0;
  for (int c = 0; c < frags_per_wave; c += U) {
    u32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = c + u < frags_per_wave ? c + u : frags_per_wave - 1;
      if (NT) v[u] = __builtin_nontemporal_load(p + (long long)k * 64);
      else v[u] = p[(long long)k * 64];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  out[wid * 64 + lane] = acc;
}

template <int U, bool NT>
float run(std::vector<u32x4_t*>& bufs, unsigned* out, size_t bytes, int wpb, int per) {
  const long long waves = bytes / 1024 / per;
  const int blocks = (int)(waves / wpb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((probe<U, NT>), dim3(blocks), dim3(wpb * 64), 0, 0, bufs[i % bufs.size()], out, per);
  hipEventRecord(e0);
  const int reps = 100;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((probe<U, NT>), dim3(blocks), dim3(wpb * 64), 0, 0, bufs[i % bufs.size()], out, per);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

int main() {
  const size_t sizes[] = {8u << 20, 16u << 20, 48u << 20, 24u << 20};
  unsigned* out;
  hipMalloc(&out, 64 << 20);
  for (size_t bytes : sizes) {
    std::vector<u32x4_t*> bufs;
    for (size_t tot = 0; tot < (700u << 20); tot += bytes) {
      u32x4_t* b; hipMalloc(&b, bytes); hipMemset(b, 1, bytes); bufs.push_back(b);
    }
    hipDeviceSynchronize();
    struct Cfg { int wpb, per; };
    const Cfg cfgs[] = {{4, 16}, {4, 8}, {8, 8}, {16, 4}, {8, 16}, {4, 32}, {16, 8}};
    for (auto c : cfgs) {
      if (bytes / 1024 / c.per / c.wpb < 1) continue;
      float t4 = run<4, false>(bufs, out, bytes, c.wpb, c.per);
      float t8 = run<8, false>(bufs, out, bytes, c.wpb, c.per);
      float t8n = run<8, true>(bufs, out, bytes, c.wpb, c.per);
      float t16 = run<16, false>(bufs, out, bytes, c.wpb, c.per);
      printf("%5zu MiB wpb %2d per %2d blocks %6zu: U4 %6.2f us (%5.0f GB/s)  U8 %6.2f (%5.0f)  U8nt %6.2f (%5.0f)  U16 %6.2f (%5.0f)\n",
             bytes >> 20, c.wpb, c.per, bytes / 1024 / c.per / c.wpb, t4, bytes / t4 / 1e3, t8, bytes / t8 / 1e3, t8n,
             bytes / t8n / 1e3, t16, bytes / t16 / 1e3);
      fflush(stdout);
    }
    for (auto b : bufs) hipFree(b);
  }
  return 0;
}
