// LDS atomic throughput microbenchmark (gfx950).  Each wave issues N atomic
// instructions into a 64 KB LDS buffer with a chosen address pattern; the
// kernel reports LDS-instruction throughput (lane-ops/s) for:
//   f32 ds_add_f32 | u32 ds_add_u32 | u64 ds_add_u64 | write ds_write_b32 |
//   pk  ds_pk_add_bf16 (2 values / lane-op)
// patterns: 0 = random over W words, 1 = lane-unique (lane*4 + it%4), 2 = all lanes same word
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(512) void k(uint32_t* out, int iters, int pattern, int W, uint32_t seed) {
  __shared__ uint32_t buf[16384];
  for (int i = threadIdx.x; i < 16384; i += 512) buf[i] = 0;
  __syncthreads();
  uint32_t x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 97u);
  const int lane = threadIdx.x & 63;
  float facc = 1.0f;
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    int addr;
    if (pattern == 0) addr = (x >> 8) % W;
    else if (pattern == 1) addr = (lane * 4 + (it & 3)) & 16383;
    else addr = 5;
    if (OP == 0) atomicAdd(reinterpret_cast<float*>(&buf[addr]), facc);
    else if (OP == 1) atomicAdd(&buf[addr], 1u);
    else if (OP == 2) atomicAdd(reinterpret_cast<unsigned long long*>(&buf[addr & ~1]), 1ull);
    else buf[addr] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = buf[threadIdx.x];
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 4096 * 4);
  const int blocks = 256 * 4, iters = 4096;
  const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_add_u64", "ds_write_b32"};
  const int Ws[] = {40, 320, 2560, 16384};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int op = 0; op < 4; ++op) {
    for (int pat = 0; pat < 3; ++pat) {
      for (int wi = 0; wi < (pat == 0 ? 4 : 1); ++wi) {
        const int W = Ws[wi];
        for (int rep = 0; rep < 2; ++rep) {
          hipEventRecord(a);
          switch (op) {
            case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(512), 0, 0, out, iters, pat, W, 7u); break;
            case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(512), 0, 0, out, iters, pat, W, 7u); break;
            case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(512), 0, 0, out, iters, pat, W, 7u); break;
            default: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(512), 0, 0, out, iters, pat, W, 7u); break;
          }
          hipEventRecord(b);
          hipEventSynchronize(b);
          float ms;
          hipEventElapsedTime(&ms, a, b);
          if (rep == 1) {
            double lane_ops = (double)blocks * 512 * iters;
            printf("%-13s pattern=%d W=%5d : %8.3f ms  %.3e lane-ops/s  %.2f lane-ops/clk/CU@2.4GHz\n", names[op],
                   pat, pat == 0 ? W : 0, ms, lane_ops / (ms * 1e-3), lane_ops / (ms * 1e-3) / 256 / 2.4e9);
          }
        }
      }
    }
  }
  return 0;
}
