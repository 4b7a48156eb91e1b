// Does a partially-active wave make LDS atomics cheaper?  ds_add_u64 into a
// 128 KB-wide random address range with A of 64 lanes active per instruction
// (random lanes, re-drawn every iteration).  If the per-instruction cost is
// fixed, useful lane-ops/s fall linearly with A and compacting sparse
// (row, tree) work into full waves pays; if the cost scales with active lanes,
// it does not.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ __launch_bounds__(512) void k(uint32_t* out, int iters, int A, int W, uint32_t seed) {
  __shared__ unsigned long long buf[8192];
  for (int i = threadIdx.x; i < 8192; i += 512) buf[i] = 0;
  __syncthreads();
  uint32_t x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 97u);
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    const int addr = (x >> 8) % W;
    if ((int)((x >> 2) & 63) < A) atomicAdd(&buf[addr], 1ull);
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)buf[threadIdx.x];
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 4096 * 4);
  const int blocks = 256 * 4, iters = 4096;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int As[] = {64, 48, 32, 16, 8, 0};
  const int Ws[] = {1024, 8192};
  for (int wi = 0; wi < 2; ++wi)
    for (int ai = 0; ai < 6; ++ai) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, out, iters, As[ai], Ws[wi], 7u);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep == 1) {
          const double instr = (double)blocks * 8 * iters;
          const double lanes = instr * As[ai];
          printf("ds_add_u64 W=%5d active=%2d/64 : %8.3f ms  %.3e useful lane-ops/s  %.2f instr/clk/CU\n", Ws[wi],
                 As[ai], ms, lanes / (ms * 1e-3), instr / (ms * 1e-3) / 256 / 2.4e9);
        }
      }
    }
  return 0;
}
