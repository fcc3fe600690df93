// Probe: cost of a grid-wide barrier across the 8 XCDs (agent-scope relaxed atomics, sc1 traffic),
// with and without a per-stage activation exchange.  Host-side timing with hipEvents.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned target) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 26)) break;  // safety exit: never hang the GPU
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(512) void k_bar(unsigned* bar, int iters, float* buf, int exchange) {
  const unsigned nb = gridDim.x;
  float acc = 0.f;
  for (int i = 0; i < iters; ++i) {
    if (exchange) {
      const int src = (blockIdx.x + 37 * (i + 1)) % nb;
      acc += __hip_atomic_load(buf + (size_t)src * 512 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(buf + (size_t)blockIdx.x * 512 + threadIdx.x, acc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    grid_barrier(bar, (unsigned)(i + 1) * nb);
  }
  if (acc == 12345.f) buf[0] = acc;
}

__global__ void k_empty() {}

int main() {
  unsigned* bar; float* buf;
  hipMalloc(&bar, 4); hipMalloc(&buf, 4 << 20);
  hipMemset(buf, 0, 4 << 20);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int nb : {64, 128, 256, 512}) {
    for (int ex = 0; ex < 2; ++ex) {
      const int iters = 2000;
      hipMemset(bar, 0, 4);
      k_bar<<<nb, 512>>>(bar, 10, buf, ex);
      hipMemset(bar, 0, 4);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      k_bar<<<nb, 512>>>(bar, iters, buf, ex);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      unsigned v; hipMemcpy(&v, bar, 4, hipMemcpyDeviceToHost);
      printf("blocks=%4d exchange=%d  %7.3f us/barrier  (counter %u, expect %u)\n", nb, ex, ms * 1e3 / iters, v,
             (unsigned)nb * iters);
    }
  }
  return 0;
}
