// Probe: cost of a grid-wide barrier across the 8 XCDs (agent-scope relaxed atomics, sc1 traffic):
// flat single counter vs two-level (per-group counters, last arriver bumps the top counter).
// Every spin loop has a bounded exit so a bug cannot hang the GPU.
#include <hip/hip_runtime.h>
#include <cstdio>

#define LD(p) __hip_atomic_load((p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define ADD(p, v) __hip_atomic_fetch_add((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)

__device__ __forceinline__ void spin_until(unsigned* p, unsigned target) {
  unsigned spins = 0;
  while (LD(p) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1u << 24)) break;
  }
}

// flat: every block increments one counter
__device__ __forceinline__ void bar_flat(unsigned* c, unsigned epoch) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    ADD(c, 1u);
    spin_until(c, epoch * gridDim.x);
  }
  __syncthreads();
}

// two-level: G groups (block % G), group counters 64 words apart; last of a group bumps top
__device__ __forceinline__ void bar_tree(unsigned* c, unsigned epoch, int G) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int g = blockIdx.x % G;
    const unsigned per = (gridDim.x - g + G - 1) / G;  // blocks in group g
    unsigned* top = c;
    unsigned* gc = c + 64 * (1 + g);
    const unsigned old = ADD(gc, 1u);
    if (old + 1 == epoch * per) ADD(top, 1u);
    spin_until(top, epoch * G);
  }
  __syncthreads();
}

__global__ __launch_bounds__(512) void k_bar(unsigned* c, int iters, float* buf, int exchange, int G) {
  const unsigned nb = gridDim.x;
  float acc = 0.f;
  for (int i = 0; i < iters; ++i) {
    if (exchange) {
      const int src = (blockIdx.x + 37 * (i + 1)) % nb;
      acc += LD(buf + (size_t)src * 512 + threadIdx.x);
      __hip_atomic_store(buf + (size_t)blockIdx.x * 512 + threadIdx.x, acc + i, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if (G == 0) bar_flat(c, i + 1);
    else bar_tree(c, i + 1, G);
  }
  if (acc == 12345.f) buf[0] = acc;
}

int main() {
  unsigned* c; float* buf;
  hipMalloc(&c, 64 * 4 * 80); hipMalloc(&buf, 4 << 20);
  hipMemset(buf, 0, 4 << 20);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int nb : {128, 256, 512}) {
    for (int G : {0, 8, 16, 32}) {
      for (int ex = 0; ex < 2; ++ex) {
        const int iters = 2000;
        hipMemset(c, 0, 64 * 4 * 80);
        k_bar<<<nb, 512>>>(c, 10, buf, ex, G);
        hipMemset(c, 0, 64 * 4 * 80);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        k_bar<<<nb, 512>>>(c, iters, buf, ex, G);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        unsigned v = 0;
        (void)hipMemcpy(&v, c, 4, hipMemcpyDeviceToHost);
        printf("blocks=%4d groups=%2d exchange=%d  %7.3f us/barrier  (top %u, expect %u)\n", nb, G, ex,
               ms * 1e3 / iters, v, (unsigned)(G ? G : nb) * iters);
      }
    }
  }
  return 0;
}
