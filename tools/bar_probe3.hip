// Prefetch credit of a persistent kernel on a code-predictor-like chain (256 workgroups x 512 threads, one per CU):
// every phase each block streams its 32 KiB weight slice (a 120 MB pool resident in the Infinity Cache, 15 distinct
// phase slices as in 5 layers x 3 GEMVs), reads the 16 KiB activation vector of the previous phase, consumes both and
// publishes its 64 B slice of the next vector.
//   P0 graph    : one kernel per phase, graph-captured chain (weights issued at kernel start, beside the vector)
//   P1 tagged   : persistent, edges = {value, epoch} 8-byte granules; weights of phase i issued at phase start
//   P2 prefetch : persistent + the NEXT phase's weights issued before this phase's edge wait (register ping-pong)
// Every spin is bounded (error flag, no hang).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bar_probe3.hip -o tools/bar_probe3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

__device__ __forceinline__ unsigned long long ld_sc1_64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int NB = 256, VEC = 4096, NSL = 15, WQ = 4;  // WQ x 16 B per thread = 32 KiB per block
constexpr unsigned SPIN_MAX = 1u << 20;

__device__ __forceinline__ void load_w(const u32x4_t* pool, int slice, u32x4_t (&w)[WQ]) {
  const u32x4_t* p = pool + ((size_t)slice * NB + blockIdx.x) * (WQ * 512) + threadIdx.x;
#pragma unroll
  for (int q = 0; q < WQ; ++q) w[q] = p[q * 512];
}
__device__ __forceinline__ float use_w(const u32x4_t (&w)[WQ]) {
  unsigned x = 0;
#pragma unroll
  for (int q = 0; q < WQ; ++q) x ^= w[q][0] ^ w[q][1] ^ w[q][2] ^ w[q][3];
  return (float)(x & 7u);
}

// one phase as its own kernel: weights + the previous vector (plain data, kernel boundary = the edge)
__global__ __launch_bounds__(512) void phase_k(const u32x4_t* pool, const float* vin, float* vout, int ph) {
  u32x4_t w[WQ];
  load_w(pool, ph % NSL, w);
  float s = 0.f;
  for (int i = threadIdx.x; i < VEC; i += 512) s += vin[i];
  s += use_w(w);
  __shared__ float red[8];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x < 16) vout[blockIdx.x * 16 + threadIdx.x] = red[threadIdx.x & 7] * 1e-9f + (float)threadIdx.x;
}

// untracked loads (hipcc inserts no waits for them): the prefetch stays in flight across the polling loop, whose
// compiler waits would otherwise drain it; waited for by an explicit vmcnt(0) naming the registers before use
__device__ __forceinline__ void load_w_asm(const u32x4_t* pool, int slice, u32x4_t (&w)[WQ]) {
  const u32x4_t* p = pool + ((size_t)slice * NB + blockIdx.x) * (WQ * 512) + threadIdx.x;
#pragma unroll
  for (int q = 0; q < WQ; ++q) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(w[q]) : "v"(p + q * 512) : "memory");
}

template <bool PF>
__global__ __launch_bounds__(512) void persist_k(const u32x4_t* pool, unsigned long long* gran, int phases, float* sink,
                                                 unsigned* err) {
  __shared__ float red[8];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  u32x4_t wa[WQ], wb[WQ];
  load_w(pool, 0, wa);
  float acc = 0.f;
  for (int ph = 1; ph <= phases; ++ph) {
    if (PF) load_w_asm(pool, ph % NSL, wb);  // next phase's weights in flight across this edge
    else load_w(pool, (ph - 1) % NSL, wa);
    // edge: read the previous phase's vector (epoch ph - 1; phase 1 reads epoch 0 = the initial zeros)
    float s = 0.f;
    unsigned spins = 0;
    for (int i = tid; i < VEC; i += 512) {
      unsigned long long g;
      while (true) {
        g = ld_sc1_64(gran + i);
        if ((unsigned)(g >> 32) >= (unsigned)(ph - 1)) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > SPIN_MAX) { atomicOr(err, 1u); break; }
      }
      s += __uint_as_float((unsigned)g);
    }
    s += use_w(wa);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) red[w] = s;
    __syncthreads();
    if (tid < 16)
      st_sc1_64(gran + blockIdx.x * 16 + tid,
                ((unsigned long long)ph << 32) | __float_as_uint(red[tid & 7] * 1e-9f + (float)tid));
    acc += red[0];
    __syncthreads();
    if (PF) {
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(wb[0]), "+v"(wb[1]), "+v"(wb[2]), "+v"(wb[3])::"memory");
#pragma unroll
      for (int q = 0; q < WQ; ++q) wa[q] = wb[q];
    }
    if (*(volatile unsigned*)err) break;
  }
  if (acc == 1234.5f) sink[0] = acc;
}

int main() {
  const size_t pool_bytes = (size_t)NSL * NB * WQ * 512 * 16;  // 120 MB
  u32x4_t* pool; CK(hipMalloc(&pool, pool_bytes)); CK(hipMemset(pool, 1, pool_bytes));
  float *va, *vb, *sink; unsigned* err; unsigned long long* gran;
  CK(hipMalloc(&va, VEC * 4)); CK(hipMalloc(&vb, VEC * 4)); CK(hipMalloc(&sink, 4)); CK(hipMalloc(&err, 4));
  CK(hipMalloc(&gran, VEC * 8));
  CK(hipMemset(va, 0, VEC * 4)); CK(hipMemset(vb, 0, VEC * 4));
  hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int n = 600;
  for (int rep = 0; rep < 2; ++rep) {
    {  // P0
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int i = 0; i < n; ++i)
        hipLaunchKernelGGL(phase_k, dim3(NB), dim3(512), 0, st, pool, (i & 1) ? vb : va, (i & 1) ? va : vb, i);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      printf("P0 graph, kernel per phase      : %6.3f us per phase\n", ms * 1e3 / n);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
    for (int pf = 0; pf < 2; ++pf) {
      CK(hipMemset(gran, 0, VEC * 8)); CK(hipMemset(err, 0, 4));
      CK(hipStreamSynchronize(st)); CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, st));
      if (pf) hipLaunchKernelGGL(persist_k<true>, dim3(NB), dim3(512), 0, st, pool, gran, n, sink, err);
      else hipLaunchKernelGGL(persist_k<false>, dim3(NB), dim3(512), 0, st, pool, gran, n, sink, err);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned he; CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
      printf("P%d persistent tagged%s: %6.3f us per phase, err %u\n", pf ? 2 : 1, pf ? " + prefetch" : "           ",
             ms * 1e3 / n, he);
      fflush(stdout);
    }
  }
  printf("done\n");
  return 0;
}
