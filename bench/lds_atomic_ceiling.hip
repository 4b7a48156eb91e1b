// LDS atomic ceiling on gfx950 (round 2): conflict-free ds_add_u64 / ds_add_u32 /
// ds_write_b64 issue rates with NO per-op VALU work (the round-1 bench computed a
// random address per op, so it measured its own VALU, not the LDS).  Each lane
// adds into cell (it & 7) * 64 + lane (bank pair = lane % 32): the 8 unrolled ops
// per loop trip carry immediate offsets, so the loop body is LDS instructions
// plus one scalar compare.  Reports LDS wave-instructions per clock per CU.
//   hipcc --offload-arch=gfx950 -O3 bench/lds_atomic_ceiling.hip -o /tmp/lds_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP, int ACTIVE>
__global__ __launch_bounds__(512) void k(uint32_t* out, int iters) {
  __shared__ unsigned long long buf[8 * 64 * 4];
  for (int i = threadIdx.x; i < 8 * 64 * 4; i += 512) buf[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wq = (threadIdx.x >> 6) & 3;
  unsigned long long* p = buf + wq * 512 + lane;
  uint32_t* p32 = reinterpret_cast<uint32_t*>(buf) + wq * 1024 + lane;
  const unsigned long long v = threadIdx.x + 1;
  if (lane < ACTIVE) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (OP == 0) atomicAdd(p + u * 64, v);
        else if (OP == 1) atomicAdd(p32 + u * 64, (uint32_t)v);
        else p[u * 64] = v + it;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)buf[5];
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 8192 * 4);
  const int iters = 2048;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"ds_add_u64", "ds_add_u32", "ds_write_b64"};
  for (int op = 0; op < 3; ++op) {
    for (int act = 0; act < 2; ++act) {
      for (int blocks_per_cu = 1; blocks_per_cu <= 4; blocks_per_cu *= 2) {
        const int blocks = 256 * blocks_per_cu;
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
          (void)hipEventRecord(a);
#define L(O, A) hipLaunchKernelGGL((k<O, A>), dim3(blocks), dim3(512), 0, 0, out, iters)
          if (op == 0) { if (act) L(0, 50); else L(0, 64); }
          else if (op == 1) { if (act) L(1, 50); else L(1, 64); }
          else { if (act) L(2, 50); else L(2, 64); }
          (void)hipEventRecord(b);
          (void)hipEventSynchronize(b);
          (void)hipEventElapsedTime(&ms, a, b);
        }
        const double winstr = (double)blocks * 8 * iters * 8;  // waves x trips x ops
        const double per_cu_clk = winstr / 256.0 / (ms * 1e-3 * 2.4e9);
        printf("%-13s active=%2d blocks/CU=%d : %8.3f ms  %.3f wave-instr/clk/CU  (%.2f clk per instr)\n",
               names[op], act ? 50 : 64, blocks_per_cu, ms, per_cu_clk, 1.0 / per_cu_clk);
      }
    }
  }
  return 0;
}
