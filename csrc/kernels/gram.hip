// K1 gram_xtx — fused [X-s | 1 | y-ys]ᵀ[X-s | 1 | y-ys] on MFMA.
//
// One pass over the row-major feature matrix produces every sufficient
// statistic LinearRegression / standardisation needs (XᵀX, Xᵀy, column sums,
// n, yᵀy) without materialising the augmented matrix.  Reference behaviour:
// LinearRegression "normal" solver, ML 02 - Linear Regression I.py:84-123,
// Labs/ML 02L:68-79.
//
// Mapping (v_mfma_f32_32x32x2_f32, exact f32): the reduction axis of the
// Gram is the ROW axis, so for an output tile (I,J) lane l supplies
//   A[i=l&31][k=l>>5] = Â[k0 + (l>>5)][32I + (l&31)]
//   B[k=l>>5][j=l&31] = Â[k0 + (l>>5)][32J + (l&31)]
// i.e. each half-wave reads 128 contiguous bytes of one row: fully coalesced
// global loads straight into the MFMA operands, no LDS staging needed.
// Each wave owns a contiguous row range and P upper-triangular tiles; the 4
// waves of a block are folded through LDS atomics and each block writes one
// f32 partial slab, reduced deterministically in f64 by gram_reduce_kernel.
//
// bf16 variant: inputs rounded to bf16 and fed to v_mfma_f32_32x32x16_bf16
// through an LDS transpose (ds_read of 8 consecutive rows per lane).  The
// streaming form (gram_bf16s_kernel) reads X once with all tile pairs per
// block; gram_bf16_kernel remains for unaligned / wide inputs.
#include "common.h"
#include <cstdlib>

namespace {

constexpr int kMaxPairs = 160;
struct PairTable {
  int16_t I[kMaxPairs];
  int16_t J[kMaxPairs];
};

__device__ __forceinline__ float aug_val(const float* __restrict__ X, const float* __restrict__ y,
                                         int64_t r, int c, int d, int64_t ldx, float s, bool valid) {
  if (!valid) return 0.f;
  if (c < d) return X[r * ldx + c] - s;
  if (c == d) return 1.f;
  if (c == d + 1 && y != nullptr) return y[r] - s;
  return 0.f;
}

__device__ __forceinline__ float col_shift(const float* __restrict__ shift, float yshift, int c, int d) {
  if (c < d) return shift ? shift[c] : 0.f;
  if (c == d + 1) return yshift;
  return 0.f;
}

template <int P>
__global__ __launch_bounds__(256) void gram_f32_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                       const float* __restrict__ y, const float* __restrict__ shift,
                                                       float yshift, PairTable tab, int npairs,
                                                       float* __restrict__ partial, int64_t rows_per_wave) {
  __shared__ float red[P * 1024];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < P * 1024; i += 256) red[i] = 0.f;

  const int pbase = blockIdx.y * P;
  int ca[P], cb[P];
  float sa[P], sb[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int gp = pbase + p < npairs ? pbase + p : npairs - 1;
    ca[p] = tab.I[gp] * 32 + (lane & 31);
    cb[p] = tab.J[gp] * 32 + (lane & 31);
    sa[p] = col_shift(shift, yshift, ca[p], d);
    sb[p] = col_shift(shift, yshift, cb[p], d);
  }
  f32x16 acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[p][e] = 0.f;

  const int64_t gw = (int64_t)blockIdx.x * 4 + wid;
  const int64_t r0 = gw * rows_per_wave;
  int64_t r1 = r0 + rows_per_wave;
  if (r1 > n) r1 = n;
  const int half = lane >> 5;
  for (int64_t k0 = r0; k0 < r1; k0 += 4) {
    // two MFMA k-steps (4 rows) per iteration: issue all loads first
    const int64_t ra = k0 + half, rb = k0 + 2 + half;
    const bool va = ra < r1, vb = rb < r1;
    float a0[P], b0[P], a1[P], b1[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      a0[p] = aug_val(X, y, ra, ca[p], d, ldx, sa[p], va);
      b0[p] = aug_val(X, y, ra, cb[p], d, ldx, sb[p], va);
      a1[p] = aug_val(X, y, rb, ca[p], d, ldx, sa[p], vb);
      b1[p] = aug_val(X, y, rb, cb[p], d, ldx, sb[p], vb);
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[p], b0[p], acc[p], 0, 0, 0);
      acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[p], b1[p], acc[p], 0, 0, 0);
    }
  }
  __syncthreads();
  const int col = lane & 31;
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * half;
      atomicAdd(&red[p * 1024 + row * 32 + col], acc[p][e]);
    }
  __syncthreads();
  for (int i = threadIdx.x; i < P * 1024; i += 256) {
    const int p = i >> 10;
    if (pbase + p < npairs) partial[((int64_t)blockIdx.x * npairs + pbase + p) * 1024 + (i & 1023)] = red[i];
  }
}

// bf16 inputs / f32 accumulate: 16 rows per MFMA. A 64-row tile of the
// augmented matrix is converted to bf16 and stored TRANSPOSED in LDS
// (tile[c][r], 64 rows -> 128 B per column) so each lane's 8-row fragment of
// one column is one 16-byte ds_read.
template <int P>
__global__ __launch_bounds__(256) void gram_bf16_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                        const float* __restrict__ y, const float* __restrict__ shift,
                                                        float yshift, PairTable tab, int npairs, int Dpad,
                                                        float* __restrict__ partial, int64_t rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // column stride 64 rows * 2 B = 128 B, padded by 16 B to spread banks
  constexpr int kColStride = 72;  // in bf16 elements (144 B)
  uint16_t* tile = reinterpret_cast<uint16_t*>(smem);
  float* red = reinterpret_cast<float*>(smem + (size_t)Dpad * kColStride * 2);
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < P * 1024; i += 256) red[i] = 0.f;
  const int pbase = blockIdx.y * P;
  int ta[P], tb[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int gp = pbase + p < npairs ? pbase + p : npairs - 1;
    ta[p] = tab.I[gp];
    tb[p] = tab.J[gp];
  }
  f32x16 acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[p][e] = 0.f;
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  const int64_t rb0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t rb1 = rb0 + rows_per_block;
  if (rb1 > n) rb1 = n;
  const int half = lane >> 5;
  for (int64_t t0 = rb0; t0 < rb1; t0 += 64) {
    __syncthreads();
    // stage: element e -> (row r = e / Dpad, col c = e % Dpad); coalesced along c
    for (int e = threadIdx.x; e < 64 * Dpad; e += 256) {
      const int r = e / Dpad, c = e - r * Dpad;
      const int64_t gr = t0 + r;
      const float v = aug_val(X, y, gr, c, d, ldx, col_shift(shift, yshift, c, d), gr < rb1);
      const __bf16 b = (__bf16)v;  // RNE, lowers to v_cvt_pk_bf16_f32
      tile[c * kColStride + r] = __builtin_bit_cast(uint16_t, b);
    }
    __syncthreads();
    // each wave takes a 16-row k-slice of the 64-row tile
    const int kr = wid * 16 + 8 * half;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&tile[(ta[p] * 32 + (lane & 31)) * kColStride + kr]);
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(&tile[(tb[p] * 32 + (lane & 31)) * kColStride + kr]);
      acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[p], 0, 0, 0);
    }
  }
  __syncthreads();
  const int col = lane & 31;
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * half;
      atomicAdd(&red[p * 1024 + row * 32 + col], acc[p][e]);
    }
  __syncthreads();
  for (int i = threadIdx.x; i < P * 1024; i += 256) {
    const int p = i >> 10;
    if (pbase + p < npairs) partial[((int64_t)blockIdx.x * npairs + pbase + p) * 1024 + (i & 1023)] = red[i];
  }
}

// Streaming bf16 Gram (d % 4 == 0, 16-byte aligned rows, D <= 160): one pass
// over X with every tile pair in the same block, so X is read exactly once.
//  * rows stream through a double-buffered LDS tile (64 rows, stored column-
//    major as bf16 so a lane's 8-row MFMA fragment is one 16-byte ds_read);
//  * the next tile's float4 loads are issued into registers before the MFMAs
//    on the current tile, and land in the other LDS buffer after them: one
//    __syncthreads per tile;
//  * wave w owns tile pairs w, w+4, ...; its accumulators go straight to the
//    block's partial slab (no cross-wave fold).
// Each thread's (row, column-quad) items are fixed for the whole kernel, so
// their global and LDS offsets are computed once.
template <int PW, int NI>
__global__ __launch_bounds__(256) void gram_bf16s_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                         const float* __restrict__ y,
                                                         const float* __restrict__ shift, float yshift,
                                                         PairTable tab, int npairs, int Dpad,
                                                         float* __restrict__ partial, int64_t rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // 64-row tiles, 4 waves: the next tile's 8 rows x 4 columns per thread are in flight under the current
  // tile's MFMAs.  Measured alternatives (profiles/r2/gram_ab.md): 128-row tiles with 512 threads 1.75 ms,
  // 128-row tiles with 256 threads at one wave per SIMD no faster; this shape 1.54 ms.
  constexpr int kRows = 64;
  constexpr int kCS = kRows + 8;  // column stride in bf16 elements: 36-dword stride, conflict-free fragment reads
  constexpr int kTh = 256;
  uint16_t* buf = reinterpret_cast<uint16_t*>(smem);
  const int tsz = Dpad * kCS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, half = lane >> 5;
  const int d4 = d >> 2;
  // work item = (row octet r8, column quad c4), r8 fastest: a thread loads 8 rows x 4 columns and stores each
  // column's 8 rows as ONE 16-byte ds_write_b128 (a column quad's 8 lanes fill 128 contiguous bytes:
  // conflict-free; 2-byte column-major stores from row-major items were 80 % of the LDS cycles in conflicts)
  constexpr int kOct = kRows / 8;
  const int items = kOct * d4;
  int goff[NI], loff[NI], r8s[NI];
  float4 sh[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int e = tid + kTh * i;
    const bool ok = e < items;
    const int r8 = ok ? (e % kOct) : 0, c4 = ok ? (e / kOct) : 0;
    goff[i] = ok ? (int)(8 * r8 * ldx) + 4 * c4 : -1;
    loff[i] = 4 * c4 * kCS + 8 * r8;
    r8s[i] = r8;
    sh[i] = shift ? *reinterpret_cast<const float4*>(shift + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // zero both buffers once: padding columns d+2..Dpad-1 stay zero forever
  for (int i = tid; i < 2 * tsz / 2; i += kTh) reinterpret_cast<uint32_t*>(buf)[i] = 0u;
  int pr[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j) pr[j] = wid + (kTh / 64) * j;
  f32x16 acc[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;

  const int64_t rb0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t rb1 = rb0 + rows_per_block;
  if (rb1 > n) rb1 = n;
  float4 v[NI][8];
  float yv = 0.f;
// next tile's rows -> registers (rows past rb1 load the shift, i.e. become 0)
#define GRAM_LOAD(T0)                                                                            \
  {                                                                                              \
    const int64_t lim_ = rb1 - (T0);                                                             \
    _Pragma("unroll") for (int i = 0; i < NI; ++i) {                                             \
      _Pragma("unroll") for (int q = 0; q < 8; ++q) {                                            \
        const bool ok_ = goff[i] >= 0 && 8 * r8s[i] + q < lim_;                                  \
        v[i][q] = ok_ ? *reinterpret_cast<const float4*>(X + (T0) * ldx + goff[i] + q * ldx) : sh[i]; \
      }                                                                                          \
    }                                                                                            \
    if (tid < kRows) yv = (y != nullptr && tid < lim_) ? y[(T0) + tid] - yshift : 0.f;           \
  }
// 8 rows of one column component -> one 16-byte store
#define GRAM_COL(i_, comp_, dst_)                                                                \
  {                                                                                              \
    uint32_t w_[4];                                                                              \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) {                                              \
      const uint32_t lo_ = __builtin_bit_cast(uint16_t, (__bf16)(v[i_][2 * q].comp_ - sh[i_].comp_));     \
      const uint32_t hi_ = __builtin_bit_cast(uint16_t, (__bf16)(v[i_][2 * q + 1].comp_ - sh[i_].comp_)); \
      w_[q] = lo_ | (hi_ << 16);                                                                 \
    }                                                                                            \
    *reinterpret_cast<uint4*>(dst_) = uint4{w_[0], w_[1], w_[2], w_[3]};                          \
  }
#define GRAM_STORE(TB, T0)                                                                       \
  {                                                                                              \
    _Pragma("unroll") for (int i = 0; i < NI; ++i) {                                             \
      if (goff[i] >= 0) {                                                                        \
        uint16_t* p_ = (TB) + loff[i];                                                           \
        GRAM_COL(i, x, p_);                                                                      \
        GRAM_COL(i, y, p_ + kCS);                                                                \
        GRAM_COL(i, z, p_ + 2 * kCS);                                                            \
        GRAM_COL(i, w, p_ + 3 * kCS);                                                            \
      }                                                                                          \
    }                                                                                            \
    if (tid < kRows) {                                                                           \
      (TB)[d * kCS + tid] = __builtin_bit_cast(uint16_t, (__bf16)((T0) + tid < rb1 ? 1.f : 0.f)); \
      (TB)[(d + 1) * kCS + tid] = __builtin_bit_cast(uint16_t, (__bf16)yv);                      \
    }                                                                                            \
  }
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  __syncthreads();
  int cur = 0;
  if (rb0 < rb1) {
    GRAM_LOAD(rb0);
    GRAM_STORE(buf, rb0);
  }
  for (int64_t t0 = rb0; t0 < rb1; t0 += kRows) {
    const bool more = t0 + kRows < rb1;
    if (more) GRAM_LOAD(t0 + kRows);
    __syncthreads();
    const uint16_t* tc = buf + cur * tsz;
#pragma unroll
    for (int ks = 0; ks < kRows / 16; ++ks) {
      const int kr = ks * 16 + 8 * half;
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        if (pr[j] >= npairs) continue;
        const int ti = tab.I[pr[j]], tj = tab.J[pr[j]];
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&tc[(ti * 32 + (lane & 31)) * kCS + kr]);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(&tc[(tj * 32 + (lane & 31)) * kCS + kr]);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
      }
    }
    if (more) GRAM_STORE(buf + (cur ^ 1) * tsz, t0 + kRows);
    cur ^= 1;
  }
  const int col = lane & 31;
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    if (pr[j] >= npairs) continue;
    float* dst = partial + ((int64_t)blockIdx.x * npairs + pr[j]) * 1024;
#pragma unroll
    for (int e = 0; e < 16; ++e) dst[((e & 3) + 8 * (e >> 2) + 4 * half) * 32 + col] = acc[j][e];
  }
}
#undef GRAM_LOAD
#undef GRAM_STORE
#undef GRAM_COL

// ---------------------------------------------------------------------------
// Streaming Gram with direct-to-LDS staging (gram_bf16d_kernel; ldx == d, d % 4 == 0, d + 2 <= 128).
// gram_bf16s_kernel above stages the next tile in VGPRs (128 B per thread): 124 VGPRs + 48 accumulators cap
// it at 2 waves per SIMD and ~51 KB of loads in flight per CU -- rocprofv3: 81 % of wave time waiting on
// HBM, 2.6 TB/s.  Here the fp32 rows go HBM -> LDS with global_load_lds_dwordx4 (no VGPRs), NSTAGE = 5
// tiles deep: four 25.6 KB tiles (~100 KB) are in flight per CU while the current tile is converted to the
// transposed bf16 tile and multiplied on MFMA.  Every wave issues exactly kCPW DMA instructions per tile
// (padding chunks re-read a valid address into the stage's spare slots), so the in-order vmcnt wait
// "tile t has landed" is the compile-time count kCPW * (NSTAGE - 1).
// Stage layout: chunks of 1 KB (one wave instruction each): 25 chunks of the tile's 64 x d fp32 rows (d =
// 100: 25 600 B), one chunk whose first 16 lanes carry the 64 labels, spare chunks.
// ---------------------------------------------------------------------------
constexpr int kDRows = 64;
constexpr int kDStages = 5;
constexpr int kDWaves = 4;

// HBM -> LDS DMA issued through inline asm: the compiler's wait-count pass would otherwise treat every LDS read
// of the staging ring as aliasing the in-flight DMA and drain ALL of it (vmcnt(0)) before the conversion,
// serialising the 5-deep pipeline.  The waits are explicit (vmcnt_imm below).  M0 holds the wave's LDS base;
// lane i writes base + i * size.
__device__ __forceinline__ void dma_dwordx4(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(g),
               "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}
__device__ __forceinline__ void dma_dword(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" : : "v"(g),
               "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}

__device__ __forceinline__ constexpr int vmcnt_imm(int n) {
  return (n & 0xF) | (((n >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8);  // wait vmcnt <= n only
}

template <int PW, int CPW>
__global__ __launch_bounds__(256) void gram_bf16d_kernel(const float* __restrict__ X, int64_t n, int d,
                                                         const float* __restrict__ y,
                                                         const float* __restrict__ shift, float yshift,
                                                         PairTable tab, int npairs, int Dpad,
                                                         float* __restrict__ partial, int64_t rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int kCS = kDRows + 8;                 // bf16 column stride (conflict-free fragment reads)
  constexpr int kStageBytes = CPW * kDWaves * 1024;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  char* stage0 = smem;                                                   // [kDStages][kStageBytes]
  uint16_t* tb = reinterpret_cast<uint16_t*>(smem + kDStages * kStageBytes);  // [Dpad][kCS] bf16
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, half = lane >> 5;
  const int d4 = d >> 2;
  const int xchunks = d >> 2;                      // 64 rows x d floats = d / 4 chunks of 1 KB (d % 4 == 0)
  const int64_t rb0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t rb1 = rb0 + rows_per_block;
  if (rb1 > n) rb1 = n;
  const int ntiles = rb0 < rb1 ? (int)((rb1 - rb0 + kDRows - 1) / kDRows) : 0;
  const char* xend = reinterpret_cast<const char*>(X + n * d);
  // one DMA round: this wave's kCPW chunks of tile `ti` into stage `ti % kDStages` (always kCPW instructions)
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  auto issue = [&](int ti) __attribute__((always_inline)) {
    char* st = stage0 + (ti % kDStages) * kStageBytes;
    const int64_t t0 = rb0 + (int64_t)ti * kDRows;
    const char* xt = reinterpret_cast<const char*>(X + t0 * d);
#pragma unroll
    for (int k = 0; k < CPW; ++k) {
      const int c = wid_u + kDWaves * k;           // chunk index (wave-uniform)
      const char* g = reinterpret_cast<const char*>(X);  // spare: any valid address
      const uint32_t la = (uint32_t)(uintptr_t)(lds_ptr)(st + c * 1024);
      if (c == xchunks) {                          // labels: one dword per lane (64 rows)
        if (ti < ntiles && y != nullptr && t0 + lane < n) g = reinterpret_cast<const char*>(y + t0 + lane);
        dma_dword(g, la);
        continue;
      }
      if (ti < ntiles && c < xchunks) {
        const char* p = xt + (int64_t)c * 1024 + lane * 16;
        g = p + 16 <= xend ? p : g;
      }
      dma_dwordx4(g, la);
    }
  };
  // conversion item: (row octet r8, column quad c4); 8 x 25 = 200 items for d = 100, one per thread
  constexpr int kOct = kDRows / 8;
  const int items = kOct * d4;
  const int e = tid;
  const bool cv = e < items;
  const int r8 = cv ? e % kOct : 0, c4 = cv ? e / kOct : 0;
  const float4 sh = (cv && shift) ? *reinterpret_cast<const float4*>(shift + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
  // zero the bf16 tile once: padding columns d + 2 .. Dpad - 1 stay zero
  for (int i = tid; i < Dpad * kCS / 2; i += 256) reinterpret_cast<uint32_t*>(tb)[i] = 0u;
  int pr[PW], TI[PW], TJ[PW];  // tile-pair ids resolved once (indexing the kernarg table in the loop was a
#pragma unroll                // global load per MFMA, and its vmcnt wait drained the DMA)
  for (int j = 0; j < PW; ++j) {
    pr[j] = wid + kDWaves * j;
    TI[j] = pr[j] < npairs ? tab.I[pr[j]] : 0;
    TJ[j] = pr[j] < npairs ? tab.J[pr[j]] : 0;
  }
  f32x16 acc[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  // prologue: tiles 0 .. NSTAGE-2 in flight
#pragma unroll
  for (int s = 0; s < kDStages - 1; ++s) issue(s);
  for (int ti = 0; ti < ntiles; ++ti) {
    issue(ti + kDStages - 1);                      // keeps exactly kCPW * (NSTAGE - 1) newer loads per wave
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(CPW * (kDStages - 1)));  // this wave's chunks of tile ti landed
    __builtin_amdgcn_s_barrier();                  // ... and every other wave's; MFMA(ti - 1) done with tb
    // stage reads through address-space-3 pointers (ds_read, lgkmcnt): generic pointers became flat loads
    // that also count in vmcnt, and every wait for them drained the in-flight DMA
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const f4v* lf4p;
    typedef __attribute__((address_space(3))) const float* lfp;
    const uint32_t sta = (uint32_t)(uintptr_t)(lds_ptr)(stage0 + (ti % kDStages) * kStageBytes);
    const int64_t t0 = rb0 + (int64_t)ti * kDRows;
    const int64_t lim = rb1 - t0;
    if (cv) {
      uint16_t* dst = tb + (4 * c4) * kCS + 8 * r8;
      float4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = 8 * r8 + q;
        const f4v lv = *(lf4p)(uintptr_t)(sta + (uint32_t)((r * d + 4 * c4) * 4));
        v[q] = r < lim ? make_float4(lv.x, lv.y, lv.z, lv.w) : sh;
      }
#define GRAM_D_COL(comp_, off_)                                                                      \
  {                                                                                                  \
    uint32_t w_[4];                                                                                  \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) {                                                  \
      const uint32_t lo_ = __builtin_bit_cast(uint16_t, (__bf16)(v[2 * q].comp_ - sh.comp_));        \
      const uint32_t hi_ = __builtin_bit_cast(uint16_t, (__bf16)(v[2 * q + 1].comp_ - sh.comp_));    \
      w_[q] = lo_ | (hi_ << 16);                                                                     \
    }                                                                                                \
    *reinterpret_cast<uint4*>(dst + (off_)) = uint4{w_[0], w_[1], w_[2], w_[3]};                     \
  }
      GRAM_D_COL(x, 0);
      GRAM_D_COL(y, kCS);
      GRAM_D_COL(z, 2 * kCS);
      GRAM_D_COL(w, 3 * kCS);
#undef GRAM_D_COL
    }
    if (tid < kDRows) {
      const float ly = *(lfp)(uintptr_t)(sta + (uint32_t)(xchunks * 1024 + 4 * tid));
      const float yv = (y != nullptr && tid < lim) ? ly - yshift : 0.f;
      tb[d * kCS + tid] = __builtin_bit_cast(uint16_t, (__bf16)(tid < lim ? 1.f : 0.f));
      tb[(d + 1) * kCS + tid] = __builtin_bit_cast(uint16_t, (__bf16)yv);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0): this wave's tile stores are in LDS
    __builtin_amdgcn_s_barrier();                  // transposed bf16 tile complete
#pragma unroll
    for (int ks = 0; ks < kDRows / 16; ++ks) {
      const int kr = ks * 16 + 8 * half;
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        if (pr[j] >= npairs) continue;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&tb[(TI[j] * 32 + (lane & 31)) * kCS + kr]);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(&tb[(TJ[j] * 32 + (lane & 31)) * kCS + kr]);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));        // drain the spare DMA rounds before the block exits
  const int col = lane & 31;
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    if (pr[j] >= npairs) continue;
    float* dst = partial + ((int64_t)blockIdx.x * npairs + pr[j]) * 1024;
#pragma unroll
    for (int q = 0; q < 16; ++q) dst[((q & 3) + 8 * (q >> 2) + 4 * half) * 32 + col] = acc[j][q];
  }
}

// partial [nblk][npairs][1024] -> out (symmetric fill).  16 threads per element each sum a fixed stride of
// blocks, then a fixed-order LDS tree: deterministic, and 16x the parallelism of one thread per element
// (the serial 1024-block loop took 0.35 ms of a 3.6 ms fit).
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ partial, int nblk, int npairs,
                                                          PairTable tab, int D, double* __restrict__ out) {
  __shared__ double red[16][16];
  const int el = threadIdx.x & 15, part = threadIdx.x >> 4;
  const int64_t idx = (int64_t)blockIdx.x * 16 + el;
  const bool ok = idx < (int64_t)npairs * 1024;
  const int gp = ok ? (int)(idx >> 10) : 0, e = ok ? (int)(idx & 1023) : 0;
  double s = 0.0;
  if (ok)
    for (int b = part; b < nblk; b += 16) s += (double)partial[((int64_t)b * npairs + gp) * 1024 + e];
  red[part][el] = s;
  __syncthreads();
  if (part == 0 && ok) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][el];
    const int i = tab.I[gp] * 32 + (e >> 5), j = tab.J[gp] * 32 + (e & 31);
    if (i < D && j < D) {
      out[(int64_t)i * D + j] = t;
      out[(int64_t)j * D + i] = t;
    }
  }
}

struct GramPlan {
  PairTable tab;
  int npairs, P, ngroups, nblk, D;
  int64_t rows_per_unit;
};

GramPlan make_plan(int64_t n, int d, bool bf16) {
  GramPlan pl{};
  pl.D = d + 2;
  const int T = (pl.D + 31) / 32;
  int k = 0;
  for (int i = 0; i < T; ++i)
    for (int j = i; j < T; ++j) {
      pl.tab.I[k] = (int16_t)i;
      pl.tab.J[k] = (int16_t)j;
      ++k;
    }
  pl.npairs = k;
  const int maxP = bf16 ? 4 : 8;
  pl.ngroups = (k + maxP - 1) / maxP;
  pl.P = (k + pl.ngroups - 1) / pl.ngroups;
  int64_t nb = (n + 8191) / 8192;
  if (nb > 256) nb = 256;
  if (nb < 1) nb = 1;
  pl.nblk = (int)nb;
  if (bf16) {
    int64_t rpb = (n + nb - 1) / nb;
    rpb = (rpb + 63) / 64 * 64;
    pl.rows_per_unit = rpb;
  } else {
    const int64_t waves = nb * 4;
    int64_t rpw = (n + waves - 1) / waves;
    rpw = (rpw + 3) / 4 * 4;
    if (rpw < 4) rpw = 4;
    pl.rows_per_unit = rpw;
  }
  return pl;
}

constexpr int kStreamMaxD = 160;

bool stream_ok(const float* X, int d, int64_t ldx, const float* shift) {
  return d % 4 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(shift) & 15) == 0 && d + 2 <= kStreamMaxD;
}

GramPlan make_stream_plan(int64_t n, int d) {
  GramPlan pl = make_plan(n, d, true);
  pl.ngroups = 1;
  int64_t nb = (n + 4095) / 4096;
  if (nb > 1024) nb = 1024;  // 4 resident blocks x 256 CUs
  if (nb < 1) nb = 1;
  pl.nblk = (int)nb;
  int64_t rpb = (n + nb - 1) / nb;
  pl.rows_per_unit = (rpb + 63) / 64 * 64;
  return pl;
}

template <int PW, int NI>
void launch_stream(const GramPlan& pl, const float* X, int64_t n, int d, int64_t ldx, const float* y,
                   const float* shift, float yshift, float* ws, hipStream_t st) {
  const int Dpad = ((pl.D + 31) / 32) * 32;
  const size_t lds = (size_t)2 * Dpad * (64 + 8) * 2;
  hipLaunchKernelGGL((gram_bf16s_kernel<PW, NI>), dim3(pl.nblk), dim3(256), lds, st, X, n, d, ldx, y, shift, yshift,
                     pl.tab, pl.npairs, Dpad, ws, pl.rows_per_unit);
}

template <int PW>
void launch_stream_ni(const GramPlan& pl, const float* X, int64_t n, int d, int64_t ldx, const float* y,
                      const float* shift, float yshift, float* ws, hipStream_t st) {
  const int ni = (8 * (d / 4) + 255) / 256;
  if (ni <= 1) launch_stream<PW, 1>(pl, X, n, d, ldx, y, shift, yshift, ws, st);
  else launch_stream<PW, 2>(pl, X, n, d, ldx, y, shift, yshift, ws, st);
}

template <int PW, int CPW>
void launch_direct(const GramPlan& pl, const float* X, int64_t n, int d, const float* y, const float* shift,
                   float yshift, float* ws, hipStream_t st) {
  const int Dpad = ((pl.D + 31) / 32) * 32;
  const size_t lds = (size_t)kDStages * CPW * kDWaves * 1024 + (size_t)Dpad * (kDRows + 8) * 2;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gram_bf16d_kernel<PW, CPW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gram_bf16d_kernel<PW, CPW>), dim3(pl.nblk), dim3(256), lds, st, X, n, d, y, shift, yshift,
                     pl.tab, pl.npairs, Dpad, ws, pl.rows_per_unit);
}

// direct-to-LDS streaming plan: one resident block per CU, contiguous rows (ldx == d), d % 4 == 0, and the
// staging ring + bf16 tile within 160 KB (d <= 108: 7 chunk rounds per wave)
bool direct_ok(const float* X, int d, int64_t ldx, const float* shift) {
  return ldx == d && d % 4 == 0 && d + 2 <= 128 && (d / 4 + 1 + kDWaves - 1) / kDWaves <= 7 &&
         (reinterpret_cast<uintptr_t>(X) & 15) == 0 && (reinterpret_cast<uintptr_t>(shift) & 15) == 0;
}

GramPlan make_direct_plan(int64_t n, int d) {
  GramPlan pl = make_plan(n, d, true);
  pl.ngroups = 1;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int64_t nb = (n + 4095) / 4096;
  if (nb > ncu) nb = ncu;
  if (nb < 1) nb = 1;
  pl.nblk = (int)nb;
  const int64_t rpb = (n + nb - 1) / nb;
  pl.rows_per_unit = (rpb + kDRows - 1) / kDRows * kDRows;
  return pl;
}

template <int PW>
void launch_direct_cpw(const GramPlan& pl, const float* X, int64_t n, int d, const float* y, const float* shift,
                       float yshift, float* ws, hipStream_t st) {
  switch ((d / 4 + 1 + kDWaves - 1) / kDWaves) {
    case 1:
    case 2: launch_direct<PW, 2>(pl, X, n, d, y, shift, yshift, ws, st); break;
    case 3: launch_direct<PW, 3>(pl, X, n, d, y, shift, yshift, ws, st); break;
    case 4: launch_direct<PW, 4>(pl, X, n, d, y, shift, yshift, ws, st); break;
    case 5: launch_direct<PW, 5>(pl, X, n, d, y, shift, yshift, ws, st); break;
    case 6: launch_direct<PW, 6>(pl, X, n, d, y, shift, yshift, ws, st); break;
    default: launch_direct<PW, 7>(pl, X, n, d, y, shift, yshift, ws, st); break;
  }
}

template <int P>
void launch_f32(const GramPlan& pl, const float* X, int64_t n, int d, int64_t ldx, const float* y, const float* shift,
                float yshift, float* ws, hipStream_t st) {
  hipLaunchKernelGGL(gram_f32_kernel<P>, dim3(pl.nblk, pl.ngroups), dim3(256), 0, st, X, n, d, ldx, y, shift, yshift,
                     pl.tab, pl.npairs, ws, pl.rows_per_unit);
}
template <int P>
void launch_bf16(const GramPlan& pl, const float* X, int64_t n, int d, int64_t ldx, const float* y,
                 const float* shift, float yshift, float* ws, hipStream_t st) {
  const int Dpad = ((pl.D + 31) / 32) * 32;
  const size_t lds = (size_t)Dpad * 72 * 2 + (size_t)P * 1024 * 4;
  hipLaunchKernelGGL(gram_bf16_kernel<P>, dim3(pl.nblk, pl.ngroups), dim3(256), lds, st, X, n, d, ldx, y, shift,
                     yshift, pl.tab, pl.npairs, Dpad, ws, pl.rows_per_unit);
}

}  // namespace

// Workspace (in floats) needed by cdna_gram for an n×d problem.
CDNA_API int64_t cdna_gram_workspace(int64_t n, int d, int bf16) {
  GramPlan pl = make_plan(n, d, bf16 != 0);
  int64_t w = (int64_t)pl.nblk * pl.npairs * 1024;
  if (bf16 && d + 2 <= kStreamMaxD) {
    GramPlan ps = make_stream_plan(n, d);
    const int64_t w2 = (int64_t)ps.nblk * ps.npairs * 1024;
    if (w2 > w) w = w2;
  }
  return w;
}

// out: (d+2)×(d+2) f64, row-major.  Column d is the all-ones column, column
// d+1 is y (zeros if y == nullptr).  Supports d+2 <= 512 (160 tile pairs).
CDNA_API int cdna_gram(const float* X, int64_t n, int d, int64_t ldx, const float* y, const float* shift, float yshift,
                       double* out, float* ws, int bf16, hipStream_t st) {
  if (d + 2 > 32 * 17) return (int)hipErrorInvalidValue;
  GramPlan pl = make_plan(n, d, bf16 != 0);
  if (pl.npairs > kMaxPairs) return (int)hipErrorInvalidValue;
  if (bf16 && direct_ok(X, d, ldx, shift)) {
    pl = make_direct_plan(n, d);
    switch ((pl.npairs + kDWaves - 1) / kDWaves) {
      case 1: launch_direct_cpw<1>(pl, X, n, d, y, shift, yshift, ws, st); break;
      case 2: launch_direct_cpw<2>(pl, X, n, d, y, shift, yshift, ws, st); break;
      case 3: launch_direct_cpw<3>(pl, X, n, d, y, shift, yshift, ws, st); break;
      default: launch_direct_cpw<4>(pl, X, n, d, y, shift, yshift, ws, st); break;
    }
  } else if (bf16 && stream_ok(X, d, ldx, shift)) {
    pl = make_stream_plan(n, d);
    const int pw = (pl.npairs + 3) / 4;  // 4 waves share the tile pairs
    switch (pw) {
      case 1: launch_stream_ni<1>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 2: launch_stream_ni<2>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 3: launch_stream_ni<3>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      default: launch_stream_ni<4>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
    }
  } else if (bf16) {
    switch (pl.P) {
      case 1: launch_bf16<1>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 2: launch_bf16<2>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 3: launch_bf16<3>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      default: launch_bf16<4>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
    }
  } else {
    switch (pl.P) {
      case 1: launch_f32<1>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 2: launch_f32<2>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 3: launch_f32<3>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 4: launch_f32<4>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 5: launch_f32<5>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 6: launch_f32<6>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      case 7: launch_f32<7>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
      default: launch_f32<8>(pl, X, n, d, ldx, y, shift, yshift, ws, st); break;
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int64_t tot = (int64_t)pl.npairs * 1024;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((tot + 15) / 16)), dim3(256), 0, st, ws, pl.nblk,
                     pl.npairs, pl.tab, pl.D, out);
  return (int)hipGetLastError();
}
