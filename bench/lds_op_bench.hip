// Per-instruction cost of the LDS-pipe operations a wave-compacting histogram
// would add (ds_permute_b32 / ds_bpermute_b32 / ds_write_b128 / ds_read_b128)
// next to the ds_add_u64 they would save.  Reports wave-instructions per clock
// per CU (2.4 GHz) with 16 waves per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(512) void k(uint32_t* out, int iters, uint32_t seed) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[16384];
  for (int i = threadIdx.x; i < 16384; i += 512) buf[i] = 0;
  __syncthreads();
  uint32_t x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 97u);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t acc = 0;
  uint4 v4 = make_uint4(x, x + 1, x + 2, x + 3);
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    if (OP == 0) {
      acc += (uint32_t)__builtin_amdgcn_ds_permute((int)((x >> 8) & 63) * 4, (int)(x ^ acc));
    } else if (OP == 1) {
      acc += (uint32_t)__builtin_amdgcn_ds_bpermute((int)((x >> 8) & 63) * 4, (int)(x ^ acc));
    } else if (OP == 2) {
      v4.x ^= x;
      *reinterpret_cast<uint4*>(&buf[(wid * 64 + ((lane + it) & 63)) * 4 & 16383]) = v4;
    } else if (OP == 3) {
      const uint4 r = *reinterpret_cast<const uint4*>(&buf[(wid * 64 + ((lane + (x >> 20)) & 63)) * 4 & 16383]);
      acc += r.x ^ r.w;
    } else if (OP == 4) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&buf[((x >> 8) % 8192) * 2]), 1ull);
    } else {
      acc += buf[(x >> 8) & 16383];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = buf[threadIdx.x] + acc + v4.x;
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 4096 * 4);
  const int blocks = 256 * 2, iters = 8192;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"ds_permute_b32", "ds_bpermute_b32", "ds_write_b128", "ds_read_b128", "ds_add_u64 rand",
                         "ds_read_b32 rand"};
  for (int op = 0; op < 6; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(a);
      switch (op) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(512), 0, 0, out, iters, 7u); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(512), 0, 0, out, iters, 7u); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(512), 0, 0, out, iters, 7u); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(512), 0, 0, out, iters, 7u); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(512), 0, 0, out, iters, 7u); break;
        default: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(512), 0, 0, out, iters, 7u); break;
      }
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (rep == 1) {
        const double instr = (double)blocks * 8 * iters;
        printf("%-18s : %8.3f ms  %.3f wave-instr/clk/CU  (%.1f clk per instr per CU)\n", names[op], ms,
               instr / (ms * 1e-3) / 256 / 2.4e9, 1.0 / (instr / (ms * 1e-3) / 256 / 2.4e9));
      }
    }
  }
  return 0;
}
