// Histogram tree learning on CDNA4 (SURVEY §2.10 K4 binize, K5 hist_build,
// K7 row_partition, K8 tree_predict).  Shared by DecisionTree*, RandomForest*
// and the XGBoost-style GBDT.
//
// Reference behaviour: MLlib's PLANET-style learner — per-partition split
// statistics for every (node, feature, bin), tree-reduced once per level,
// best split chosen on the driver (ML 06 - Decision Trees.py:96-118,
// Labs/ML 07L:19); maxBins bounds the bin count (ML 07:41).
//
// Data layout (chosen for the histogram kernel, the hot loop):
//   bins   : uint8, feature-group-major  [G = ceil(d/8)][n][8]
//            -> one 8-byte load per (row, group); a wave reads 512 contiguous B
//   node   : int32 [T][n]   active-node id of the row in tree t (-1 = in a leaf)
//   weight : uint8 [T][n]   Poisson bootstrap multiplicity (nullptr = 1)
//   stats  : f32 v0[n], v1[n] (RF regression: 1, y; GBDT: g, h)
// Histogram accumulation is LDS-privatised per block (ds_add_f32), flushed
// once per block with f64 global atomics; blocks are mapped XCD-aware so the
// G feature-group blocks of one row chunk share an XCD's L2 for node/weight
// re-reads.
#include "common.h"
#include <cstdlib>
#include <type_traits>

namespace {

// ---------------------------------------------------------------------------
// K4 binize: raw f32 [n][d] -> uint8 bins [G][n][8]
// continuous: bin = #thresholds strictly below x  (x <= thr[b] goes left of split b)
// categorical (nthr[f] < 0): bin = (int)x
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void binize_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                     const float* __restrict__ thr, const int* __restrict__ nthr,
                                                     int tmax, int use_lds, int miss_on, float miss_val,
                                                     uint64_t* __restrict__ out, int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (d + 7) / 8;
  const int dp = G * 8;
  uint8_t* tile = reinterpret_cast<uint8_t*>(smem);                 // [256][dp]
  float* sthr = reinterpret_cast<float*>(smem + ((256 * dp + 15) / 16) * 16);
  const float* T = thr;
  if (use_lds) {
    for (int i = threadIdx.x; i < d * tmax; i += 256) sthr[i] = thr[i];
    T = sthr;
  }
  __syncthreads();
  for (int64_t r0 = (int64_t)blockIdx.x * 256; r0 < n; r0 += (int64_t)gridDim.x * 256) {
    const int rows = (int)((n - r0) < 256 ? (n - r0) : 256);
    for (int e = threadIdx.x; e < rows * dp; e += 256) {
      const int r = e / dp, f = e - r * dp;
      uint8_t b = 0;
      if (f < d) {
        float x = X[(r0 + r) * ldx + f];
        if (miss_on && (x != x || x == miss_val)) x = -__builtin_inff();
        const int nt = nthr[f];
        if (nt < 0) {
          int c = (int)x;
          b = (uint8_t)(c < 0 ? 0 : (c > 255 ? 255 : c));
        } else {
          const float* tf = T + (int64_t)f * tmax;
          int lo = 0, hi = nt;  // first index with tf[idx] >= x
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (tf[mid] < x) lo = mid + 1; else hi = mid;
          }
          if (x != x) lo = nt;  // NaN -> last bin
          b = (uint8_t)lo;
        }
      }
      tile[r * dp + f] = b;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < rows * G; e += 256) {
      const int g = e / rows, r = e - g * rows;
      out[(int64_t)g * ldo + r0 + r] = *reinterpret_cast<const uint64_t*>(&tile[r * dp + g * 8]);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// binize v2.  v1 (above) spent 55 ms on 1e8 x 100 (profiles/, traced step):
// one thread per (row, feature) element with integer divisions, a
// data-dependent binary-search loop and byte-wide LDS tile writes.  v2 stages a
// tile of rows with coalesced float4 loads, gives each thread (row, 8-feature
// group) tasks so the result is ONE uint64 store (coalesced along rows for a
// fixed group), and runs a fixed-trip branchless search over the LDS
// thresholds (every lane executes the same 6-7 steps; no divergence).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void binize2_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                      const float* __restrict__ thr, const int* __restrict__ nthr,
                                                      int tmax, int rows_per_tile, int steps, int miss_on,
                                                      float miss_val, uint64_t* __restrict__ out,
                                                      uint64_t* __restrict__ rm, int Gs, int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const int G = (d + 7) / 8;
  // [rows_per_tile][dp]: an odd row stride keeps the per-task x reads (lanes = rows) conflict-free; with
  // stride d = 100 (4 banks apart) 8 lanes shared each bank
  const int dp = d | 1;
  float* sx = smf;                                  // [rows_per_tile][dp]
  float* sthr = smf + (size_t)rows_per_tile * dp;   // [d][tmax]
  int* snt = reinterpret_cast<int*>(sthr + (size_t)d * tmax);
  const int tst = tmax;
  for (int i = threadIdx.x; i < d * tmax; i += 256) sthr[i] = thr[i];
  for (int i = threadIdx.x; i < d; i += 256) snt[i] = nthr[i];
  const bool contiguous = ldx == d && (d % 4) == 0;
  // register double buffer: the next tile's float4s are in flight while the
  // current tile is binned (rocprofv3: the single-buffered loop spent 69 % of
  // wave time waiting on memory)
  constexpr int kPre = 8;  // float4 per thread per tile (64 rows x d <= 128 floats x ... / 256 threads)
  float4 pre[kPre];
  const int64_t stride = (int64_t)gridDim.x * rows_per_tile;
  auto fetch = [&](int64_t r0) {
    if (!contiguous || r0 >= n) return;
    const int rows = (int)((n - r0) < rows_per_tile ? (n - r0) : rows_per_tile);
    const float4* src = reinterpret_cast<const float4*>(X + r0 * ldx);
    const int nv = rows * d / 4;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int i = threadIdx.x + k * 256;
      if (i < nv) pre[k] = src[i];
    }
  };
  const bool use_pre = contiguous && rows_per_tile * d / 4 <= kPre * 256;
  if (use_pre) fetch((int64_t)blockIdx.x * rows_per_tile);
  for (int64_t r0 = (int64_t)blockIdx.x * rows_per_tile; r0 < n; r0 += stride) {
    const int rows = (int)((n - r0) < rows_per_tile ? (n - r0) : rows_per_tile);
    __syncthreads();
    if (use_pre) {
      const int nv = rows * d / 4;
#pragma unroll
      for (int k = 0; k < kPre; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < nv) {
          const int e = i * 4, r = e / d, f = e - r * d;  // d % 4 == 0: a float4 never crosses a row
          float* dst = sx + r * dp + f;
          dst[0] = pre[k].x;
          dst[1] = pre[k].y;
          dst[2] = pre[k].z;
          dst[3] = pre[k].w;
        }
      }
    } else if (contiguous) {
      const float4* src = reinterpret_cast<const float4*>(X + r0 * ldx);
      const int nv = rows * d / 4;
      for (int i = threadIdx.x; i < nv; i += 256) {
        const float4 v = src[i];
        const int e = i * 4, r = e / d, f = e - r * d;
        float* dst = sx + r * dp + f;
        dst[0] = v.x;
        dst[1] = v.y;
        dst[2] = v.z;
        dst[3] = v.w;
      }
    } else {
      for (int i = threadIdx.x; i < rows * d; i += 256) {
        const int r = i / d, f = i - r * d;
        sx[r * dp + f] = X[(r0 + r) * ldx + f];
      }
    }
    __syncthreads();
    if (use_pre) fetch(r0 + stride);
    for (int task = threadIdx.x; task < rows * G; task += 256) {
      const int g = task / rows, r = task - g * rows;
      // the 8 searches of a bins word advance in lockstep: 8 independent LDS
      // reads per step instead of one dependent chain per feature (the
      // dependent version left the waves idle on LDS latency)
      float x[8];
      int nt[8], lo[8], toff[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = g * 8 + j < d ? g * 8 + j : d - 1;
        x[j] = sx[r * dp + f];
        // XGBoost missing values (NaN or == missing) -> -inf -> bin 0 (thresholds start at -FLT_MAX)
        if (miss_on && (x[j] != x[j] || x[j] == miss_val)) x[j] = -__builtin_inff();
        nt[j] = g * 8 + j < d ? snt[f] : 0;
        toff[j] = f * tst - 1;
        lo[j] = 0;
      }
#pragma unroll
      for (int s2 = 7; s2 >= 0; --s2) {
        if (s2 >= steps) continue;  // block-uniform
        const int step = 1 << s2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cand = lo[j] + step;
          const float tv = cand <= nt[j] ? sthr[toff[j] + cand] : __builtin_inff();
          lo[j] = tv < x[j] ? cand : lo[j];
        }
      }
      uint64_t word = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint32_t b;
        if (nt[j] < 0) {
          const int c = (int)x[j];
          b = (uint32_t)(c < 0 ? 0 : (c > 255 ? 255 : c));
        } else {
          b = (x[j] != x[j]) ? (uint32_t)nt[j] : (uint32_t)lo[j];
        }
        if (g * 8 + j >= d) b = 0;
        word |= (uint64_t)b << (8 * j);
      }
      out[(int64_t)g * ldo + r0 + r] = word;
      if (rm) {
        // row-major copy [n][Gs] written from the same registers (saves the separate transpose kernel's
        // re-read of the [G][n] bins); the row's padding words are zeroed by its last group's task
        uint64_t* rrow = rm + (r0 + r) * Gs;
        rrow[g] = word;
        if (g == G - 1)
          for (int gp = G; gp < Gs; ++gp) rrow[gp] = 0;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// binize v5 (d <= 128, d % 4 == 0, 16-byte aligned rows).  v4 (git history:
// float4 tasks, skewed +inf-padded tables, 32-row bins tile; 23.8 ms at the
// headline vs 20.9 ms for v5) put the 32 quads
// of one row on the 32 lanes of a ds_read group, so every search step read 32
// different feature tables: the first step was a 4-way bank conflict (feature
// stride 65 = 1 mod 32 banks, 4 features per quad) and the later steps random
// ones.  v5 turns the task around:
//   * a wave owns (tile of 64 rows, group g of 8 features): lane = row, so all
//     lanes of a ds_read group search the SAME 8 tables.  Step s reads at most
//     2^(STEPS-1-s) distinct entries of a table (broadcast), at most 2-way
//     conflicts, and the table offsets are wave-uniform (scalar registers);
//   * the row's two float4s of the group come straight from HBM (the G waves of
//     a block read the same 64 rows together, so the 128-byte lines are shared
//     in L1/L2), the next tile's float4s are loaded before this tile's search
//     (staging the tile through LDS with coalesced loads instead: 29.5 vs
//     19.1 ms, three block barriers per tile);
//   * the column-major word out[g][r] leaves from registers (512-byte runs);
//     the row-major copy goes through a [64][17] u64 LDS tile (odd pitch:
//     conflict-free 8-byte writes) and leaves as 16-byte stores of whole
//     128-byte rows, padding words zeroed once.
// Block = G waves (one per 8-feature group), persistent over row tiles.
// ---------------------------------------------------------------------------
// Block barrier for LDS only: waits for this wave's LDS ops (lgkmcnt 0), not for its global loads in flight.
// __syncthreads() also drains vmcnt, which emptied binize5's register prefetch at every tile.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LUT (binize v6): the threshold search narrowed by a per-feature uniform grid of kLutCells cells over
// [t_0, t_last].  cell(v) = int(clamp((v - t_0) * scale, 0, C - 1)) with the subtraction and the product rounded
// separately (no contraction) is monotone in v, so for x in cell c every threshold of a lower cell is < x and
// every threshold of a higher cell is > x: bin(x) = base[c] + #{thresholds of cell c that are < x}, where base[c] =
// #{t_j : cell(t_j) < c} -- the same count as the binary search, exactly, whatever the rounding.  The grid is
// built in LDS by every block from the device thresholds (no host round trip); the refinement walks the sorted
// table kmax = max thresholds per cell steps (Gaussian-like columns at 40 bins: 1-2) instead of the 6 search
// steps, and falls back to a binary search of the sorted table when kmax > kLutMaxK (heavy-tailed columns).
// C = cells per feature (template; 0 = no LUT).  Gaussian columns at 40 bins: 64 cells (one cell ~ one threshold
// spacing near the centre) leave 2 thresholds in the fullest cells, so every element walks 2 dependent steps;
// 256 cells leave 1.
constexpr int kLutMaxK = 6;

template <int STEPS, int RPL, int C>
__global__ __launch_bounds__(1024) void binize5_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                       const float* __restrict__ thr, const int* __restrict__ nthr,
                                                       int tmax, int miss_on, float miss_val,
                                                       uint64_t* __restrict__ out, uint64_t* __restrict__ rm, int Gs,
                                                       int64_t ldo) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smf5[];
  constexpr int P = 1 << STEPS, RT = 64 * RPL, TP = 17;  // RPL rows per lane
  constexpr bool LUT = C > 0;
  float* sthr = smf5;                                                          // [d][P]
  uint8_t* sbase = reinterpret_cast<uint8_t*>(sthr + (size_t)((d * P + 3) & ~3));  // LUT: [d][C]
  float* sprm = reinterpret_cast<float*>(sbase + (LUT ? (size_t)d * C : 0));        // LUT: [d][2] lo, scale
  uint64_t* tile = reinterpret_cast<uint64_t*>(sprm + (LUT ? (size_t)((2 * d + 3) & ~3) : 0));  // [RT][TP]
  __shared__ int s_kf[LUT ? 128 : 1];  // LUT: largest threshold count of a cell, per feature (d <= 128)
  if (LUT) {
    // sorted thresholds, +inf padded: the refinement reads t[b] for b <= nthr < P
    for (int f = threadIdx.x; f < d; f += blockDim.x) s_kf[f] = 0;
    for (int i = threadIdx.x; i < d * P; i += blockDim.x) {
      const int f = i >> STEPS, q = i & (P - 1);
      sthr[i] = (q < nthr[f] && q < tmax) ? thr[(size_t)f * tmax + q] : __builtin_inff();
    }
    __syncthreads();
    for (int f = threadIdx.x; f < d; f += blockDim.x) {
      const int nt = nthr[f] < tmax ? nthr[f] : tmax;
      float lo = 0.f, sc = 0.f;
      if (nt >= 1) lo = sthr[f * P];
      if (nt >= 3 && lo <= -3.0e38f) lo = sthr[f * P + 1];  // XGBoost's -FLT_MAX missing-value threshold: off-grid
      if (nt >= 2) {
        const float span = sthr[f * P + nt - 1] - lo;
        sc = (float)C / span;
        if (!(sc > 0.f) || !(sc < __builtin_inff())) sc = 0.f;  // one cell: the walk covers every threshold
      }
      sprm[2 * f] = lo;
      sprm[2 * f + 1] = sc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < d * C; e += blockDim.x) {
      const int f = e / C, c = e - f * C;
      const int nt = nthr[f] < tmax ? nthr[f] : tmax;
      const float lo = sprm[2 * f], sc = sprm[2 * f + 1];
      // the thresholds' cells are non-decreasing in j (sorted table, monotone cell map): base = #{cell_j < c} and
      // the cell's count = #{cell_j <= c} - base, two binary searches
      auto cell = [&](int j) { return (int)fminf(fmaxf((sthr[f * P + j] - lo) * sc, 0.f), (float)(C - 1)); };
      int a0 = 0, a1 = nt;  // first j with cell_j >= c
      while (a0 < a1) {
        const int m = (a0 + a1) >> 1;
        if (cell(m) < c) a0 = m + 1; else a1 = m;
      }
      int b0 = a0, b1 = nt;  // first j with cell_j > c
      while (b0 < b1) {
        const int m = (b0 + b1) >> 1;
        if (cell(m) <= c) b0 = m + 1; else b1 = m;
      }
      sbase[e] = (uint8_t)a0;
      if (b0 > a0) atomicMax(&s_kf[f], b0 - a0);
    }
  } else {
    // Table layout by search step: step s (step 2^s) only ever probes cand = (2k + 1) 2^s, so entry cand - 1 is
    // stored at q = P - 2^(STEPS - s) + k -- each step's candidates are consecutive words, and the 32 lanes of a
    // read group hit distinct banks (the plain layout put cand and cand + 32 on one bank: 43 % of the LDS
    // cycles were conflicts).  The last word (cand = P) is never probed.
    for (int i = threadIdx.x; i < d * P; i += blockDim.x) {
      const int f = i >> STEPS, q = i & (P - 1);
      int sg = 0;
      while (sg < STEPS - 1 && q >= P - (P >> (sg + 1))) ++sg;
      const int k = q - (P - (P >> sg));
      const int c = ((2 * k + 1) << sg) - 1;  // threshold index held at q
      sthr[i] = (q < P - 1 && c < nthr[f] && c < tmax) ? thr[(size_t)f * tmax + c] : __builtin_inff();
    }
  }
  if (rm)
    for (int i = threadIdx.x; i < RT * TP; i += blockDim.x) tile[i] = 0ull;  // words g >= G stay 0 (row padding)
  const int G = (d + 7) >> 3;
  const int nth = 64 * G;  // == blockDim.x (not re-read from the dispatch packet inside the tile loop)
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int Q = d >> 2;
  const bool hi_ok = 2 * g + 1 < Q;  // the group's second quad exists
  int nt[8], fb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int f = 8 * g + j < d ? 8 * g + j : d - 1;
    nt[j] = __builtin_amdgcn_readfirstlane(nthr[f]);
    fb[j] = f * P;  // feature f's table
  }
  __syncthreads();
  float llo[8], lsc[8];
  int kmax = 0;
  if (LUT) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 8 * g + j < d ? 8 * g + j : d - 1;
      llo[j] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sprm[2 * f])));
      lsc[j] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sprm[2 * f + 1])));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 8 * g + j < d ? 8 * g + j : d - 1;
      kmax = kmax > s_kf[f] ? kmax : s_kf[f];
    }
    kmax = __builtin_amdgcn_readfirstlane(kmax);  // this wave's 8 features
  }
  const float4* __restrict__ X4 = reinterpret_cast<const float4*>(X);
  const int64_t ldx4 = ldx >> 2;
  const int64_t ntiles = (n + RT - 1) / RT;
  auto search = [&](float (&x)[8]) -> uint64_t {
    int lo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // XGBoost missing values (NaN or == missing) -> -inf -> bin 0 (thresholds start at -FLT_MAX)
      if (miss_on && (x[j] != x[j] || x[j] == miss_val)) x[j] = -__builtin_inff();
      lo[j] = 0;
    }
    if (!LUT) {
#pragma unroll
      for (int s = STEPS - 1; s >= 0; --s) {
        const int step = 1 << s, base = P - (P >> s);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cand = lo[j] + step;  // lo is a multiple of 2^(s+1)
          lo[j] = sthr[fb[j] + base + (lo[j] >> (s + 1))] < x[j] ? cand : lo[j];
        }
      }
    } else if (kmax <= kLutMaxK) {  // wave-uniform
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = fminf(fmaxf((x[j] - llo[j]) * lsc[j], 0.f), (float)(C - 1));
        lo[j] = sbase[(fb[j] >> STEPS) * C + (int)v];
      }
      for (int s = 0; s < kmax; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lo[j] += sthr[fb[j] + lo[j]] < x[j] ? 1 : 0;
      }
    } else {  // many thresholds in one cell: binary search of the sorted table
#pragma unroll
      for (int s = STEPS - 1; s >= 0; --s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lo[j] += sthr[fb[j] + lo[j] + (1 << s) - 1] < x[j] ? (1 << s) : 0;
      }
    }
    uint64_t word = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t b;
      if (nt[j] < 0) {
        const int c = (int)x[j];
        b = (uint32_t)(c < 0 ? 0 : (c > 255 ? 255 : c));
      } else {
        b = (x[j] != x[j]) ? (uint32_t)nt[j] : (uint32_t)lo[j];
      }
      if (8 * g + j >= d) b = 0;
      word |= (uint64_t)b << (8 * j);
    }
    return word;
  };
  // Gs == -10: the "seg10" row layout of seg_hist_lane10_kernel -- ten 12-byte chunks per 128-byte row, chunk s
  // holding features 10 s .. 10 s + 9 in its first 10 bytes (2 zero bytes, 8 zero bytes after chunk 9), so one
  // aligned dwordx3 gather brings a lane its 10 features.  Output dword k of a row = row bytes
  // [10 s + p, 10 s + p + 4) with s = 4k / 12, p = 4k % 12 (an alignbyte of two tile dwords; p = 8 keeps 2 bytes).
  // seg10: a thread's 16-byte chunk c = i & 7 is the same on every trip (the block size 64 G is a multiple of
  // 8), so its four source dword pairs, byte shifts and masks are fixed before the tile loop
  int s10_src[4];
  uint32_t s10_sh[4], s10_mask[4];
  {
    const int c = threadIdx.x & 7;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * c + e, sg = (4 * k) / 12, p = (4 * k) - 12 * sg;
      const int f0 = 10 * sg + p;  // even: the dword pair (f0 >> 2, +1) shifted by 0 or 2 bytes
      s10_src[e] = sg < 10 ? (f0 >> 2) : 0;
      s10_sh[e] = (uint32_t)(f0 & 3);
      s10_mask[e] = sg < 10 ? (p == 8 ? 0xFFFFu : 0xFFFFFFFFu) : 0u;
    }
  }
  auto store_rm = [&](int64_t tl) {
    const int rows = (int)((n - tl * RT) < RT ? (n - tl * RT) : RT);
    for (int i = threadIdx.x; i < RT * 8; i += nth) {
      const int row = i >> 3, c = i & 7;
      if (row < rows) {
        const uint64_t* tr = tile + row * TP + 2 * c;
        uint4 v;
        if (Gs == -10) {
          const uint32_t* td = reinterpret_cast<const uint32_t*>(tile + row * TP);
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            o[e] = __builtin_amdgcn_alignbyte(td[s10_src[e] + 1], td[s10_src[e]], s10_sh[e]) & s10_mask[e];
          v.x = o[0]; v.y = o[1]; v.z = o[2]; v.w = o[3];
          *reinterpret_cast<uint4*>(rm + (tl * RT + row) * 16 + 2 * c) = v;
        } else {
          v.x = (uint32_t)tr[0]; v.y = (uint32_t)(tr[0] >> 32);
          v.z = (uint32_t)tr[1]; v.w = (uint32_t)(tr[1] >> 32);
          *reinterpret_cast<uint4*>(rm + (tl * RT + row) * Gs + 2 * c) = v;
        }
      }
    }
  };
  // Two register sets of RPL rows per lane, each searched and THEN refilled (two tiles ahead): while one set
  // is searched the other's loads are in flight, and no loaded register is copied (a copy of a fresh load --
  // the single-set loop's phi at the back-edge -- costs a vmcnt(0) drain per tile).  Fetches past the last
  // tile re-read the last tile (never stored), so every fetch is unconditional and counted exactly.
  // Before: one set, __syncthreads() (another vmcnt(0) drain) -- 19.1 ms = 3.3 TB/s.
  const int q1 = hi_ok ? 2 * g + 1 : 2 * g;  // no data dependence between the two loads of a row
  const int64_t S = gridDim.x, last = ntiles - 1;
  auto fetch = [&](int64_t tl, float4 (&p0)[RPL], float4 (&p1)[RPL]) {
    tl = tl < last ? tl : last;
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      int64_t r = tl * RT + k * 64 + lane;
      r = r < n ? r : n - 1;
      p0[k] = X4[r * ldx4 + 2 * g];
      p1[k] = X4[r * ldx4 + q1];
    }
  };
  auto body = [&](int64_t tl, const float4 (&p0)[RPL], const float4 (&p1)[RPL]) {
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      float x[8] = {p0[k].x, p0[k].y, p0[k].z, p0[k].w, p1[k].x, p1[k].y, p1[k].z, p1[k].w};
      const uint64_t word = search(x);
      const int64_t r = tl * RT + k * 64 + lane;
      if (r < n) out[(int64_t)g * ldo + r] = word;
      if (rm) tile[(k * 64 + lane) * TP + g] = word;
    }
    if (rm) {
      lds_barrier();
      store_rm(tl);
      lds_barrier();
    }
  };
  float4 a0[RPL], a1[RPL], b0[RPL], b1[RPL];
  fetch(blockIdx.x, a0, a1);
  fetch(blockIdx.x + S, b0, b1);
  for (int64_t tl = blockIdx.x; tl < ntiles; tl += 2 * S) {
    body(tl, a0, a1);
    fetch(tl + 2 * S, a0, a1);
    if (tl + S < ntiles) body(tl + S, b0, b1);  // block-uniform
    fetch(tl + 3 * S, b0, b1);
  }
  (void)G;
}

// ---------------------------------------------------------------------------
// K7 row_partition: move every row of every tree to its child for the level.
// split_feat[id] : -1 -> node became a leaf (row leaves the active set)
// split_bin[id]  : continuous: left iff bin <= split_bin
// cat_off[id]    : >= 0 -> categorical, left iff bit bin of cat_mask[cat_off..+8]
// child[id*2+{0,1}] : next-level active id or -1
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void partition_kernel(const uint64_t* __restrict__ bins, int64_t n, int T,
                                                        int* __restrict__ node, const int* __restrict__ split_feat,
                                                        const int* __restrict__ split_bin,
                                                        const int* __restrict__ cat_off,
                                                        const uint32_t* __restrict__ cat_mask,
                                                        const int* __restrict__ child) {
  const int t = blockIdx.y;
  const uint8_t* b8 = reinterpret_cast<const uint8_t*>(bins);
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    const int64_t o = (int64_t)t * n + r;
    const int id = node[o];
    if (id < 0) continue;
    const int f = split_feat[id];
    if (f < 0) {
      node[o] = -1;
      continue;
    }
    const int bin = b8[((int64_t)(f >> 3) * n + r) * 8 + (f & 7)];
    const int co = cat_off[id];
    bool left;
    if (co >= 0) left = (cat_mask[co * 8 + (bin >> 5)] >> (bin & 31)) & 1u;
    else left = bin <= split_bin[id];
    node[o] = child[id * 2 + (left ? 0 : 1)];
  }
}

// ---------------------------------------------------------------------------
// K8 tree_predict on raw features.  Packed node = int4:
//   continuous : {f, float_bits(thr), left, right}      left iff x <= thr
//   categorical: {-(f+2), mask_off, left, right}        left iff bit (int)x
//   leaf       : {-1, value_off, 0, 0}                  values[value_off .. +K]
// out[r][k] = base[k] + sum_t tree_w[t] * leafval_t(r)[k], all in fp64 (Spark's Double predictions): the leaf
// values, tree weights and sums are doubles, and the sum has ONE fixed order that the host reference
// (kernels.tree_predict on cpu) repeats bit for bit: tree lane q = t % 4 adds its trees in ascending order
// (product rounded, then added: no FMA contraction), then base + lane 0 + lane 1 + lane 2 + lane 3.
// Block = 256 threads = 64 rows x 4 tree lanes; the 64-row tile of X is staged in LDS with coalesced loads.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void predict_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                      const int4* __restrict__ nodes, const int* __restrict__ roots,
                                                      const double* __restrict__ tree_w, int T,
                                                      const double* __restrict__ values,
                                                      const uint32_t* __restrict__ masks, int K,
                                                      const double* __restrict__ base, double* __restrict__ out,
                                                      int n_nodes_lds, int n_vals_lds) {
#pragma clang fp contract(off)
  // LDS: [n_nodes_lds] int4 forest (when it fits), then (when n_vals_lds > 0) the leaf values and tree weights
  // (doubles) and roots, then the X tile [64][d+1] floats, then [4][64][K] double partials.
  // rocprofv3 on the global-node version: 78 % of wave time waiting on the
  // dependent node loads of each root-to-leaf walk; walking an LDS copy of the
  // forest turns each step into a ~100-cycle ds_read_b128.
  extern __shared__ __attribute__((aligned(16))) float sx_all[];
  int4* snodes = reinterpret_cast<int4*>(sx_all);
  double* svals = reinterpret_cast<double*>(sx_all + (size_t)n_nodes_lds * 4);
  const int nv_pad = n_vals_lds > 0 ? ((n_vals_lds + 1) & ~1) + ((T + 1) & ~1) : 0;  // doubles
  double* stw = svals + ((n_vals_lds + 1) & ~1);
  int* sroots = reinterpret_cast<int*>(svals + nv_pad);
  float* sx = reinterpret_cast<float*>(sroots) + (n_vals_lds > 0 ? ((T + 3) & ~3) : 0);
  const int dp = d + 1;
  double* part = reinterpret_cast<double*>(sx + 64 * dp);  // 64 * dp * 4 bytes: a multiple of 8
  const int4* nd_src = n_nodes_lds > 0 ? snodes : nodes;
  for (int i = threadIdx.x; i < n_nodes_lds; i += 256) snodes[i] = nodes[i];
  if (n_vals_lds > 0) {
    for (int i = threadIdx.x; i < n_vals_lds; i += 256) svals[i] = values[i];
    for (int i = threadIdx.x; i < T; i += 256) {
      sroots[i] = roots[i];
      stw[i] = tree_w[i];
    }
    values = svals;
    roots = sroots;
    tree_w = stw;
  }
  const int tl = threadIdx.x >> 6, row = threadIdx.x & 63;
  const bool vec = ldx == d && (d % 4) == 0;
  // register double buffer: the next tile's float4s are in flight while this
  // tile's trees are walked (the single-buffered loop read X at ~1.8 TB/s)
  constexpr int kPre = 8;
  float4 pre[kPre];
  const int64_t stride = (int64_t)gridDim.x * 64;
  const bool use_pre = vec && 64 * d / 4 <= kPre * 256;
  auto fetch = [&](int64_t r0) {
    if (r0 >= n) return;
    const int rows = (int)((n - r0) < 64 ? (n - r0) : 64);
    const float4* src = reinterpret_cast<const float4*>(X + r0 * ldx);
    const int nv = rows * d / 4;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int i = threadIdx.x + k * 256;
      if (i < nv) pre[k] = src[i];
    }
  };
  if (use_pre) fetch((int64_t)blockIdx.x * 64);
  for (int64_t r0 = (int64_t)blockIdx.x * 64; r0 < n; r0 += stride) {
    const int rows = (int)((n - r0) < 64 ? (n - r0) : 64);
    __syncthreads();
    if (use_pre) {
      const int nv = rows * d / 4;
#pragma unroll
      for (int k = 0; k < kPre; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < nv) {
          const int e = i * 4, r = e / d, f = e - r * d;
          float* dst = sx + r * dp + f;
          dst[0] = pre[k].x;
          dst[1] = pre[k].y;
          dst[2] = pre[k].z;
          dst[3] = pre[k].w;
        }
      }
    } else if (vec) {
      const float4* src = reinterpret_cast<const float4*>(X + r0 * ldx);
      const int nv = rows * d / 4;
      for (int i = threadIdx.x; i < nv; i += 256) {
        const float4 v = src[i];
        const int e = i * 4, r = e / d, f = e - r * d;  // d % 4 == 0: a float4 never crosses a row
        float* dst = sx + r * dp + f;
        dst[0] = v.x;
        dst[1] = v.y;
        dst[2] = v.z;
        dst[3] = v.w;
      }
    } else {
      for (int e = threadIdx.x; e < rows * d; e += 256) {
        const int r = e / d, f = e - r * d;
        sx[r * dp + f] = X[(r0 + r) * ldx + f];
      }
    }
    for (int e = threadIdx.x; e < 4 * 64 * K; e += 256) part[e] = 0.0;
    __syncthreads();
    if (use_pre) fetch(r0 + stride);
    if (row < rows) {
      const float* xr = sx + row * dp;
      double* pr = part + (tl * 64 + row) * K;
      // up to 8 of this lane's trees walk in lockstep: independent node
      // reads per level instead of one dependent chain per tree
      constexpr int W = 8;
      for (int tb = tl; tb < T; tb += 4 * W) {
        int4 nv[W];
        bool live[W];
#pragma unroll
        for (int u = 0; u < W; ++u) {
          const int t = tb + 4 * u;
          live[u] = t < T;
          nv[u] = live[u] ? nd_src[roots[t]] : make_int4(-1, 0, 0, 0);
        }
        bool any = true;
        while (any) {
          any = false;
#pragma unroll
          for (int u = 0; u < W; ++u) {
            if (nv[u].x == -1) continue;
            bool left;
            if (nv[u].x >= 0) {
              left = xr[nv[u].x] <= __int_as_float(nv[u].y);
            } else {
              const int c = (int)xr[-nv[u].x - 2];
              left = (c >= 0 && c < 256) ? ((masks[nv[u].y * 8 + (c >> 5)] >> (c & 31)) & 1u) : false;
            }
            nv[u] = nd_src[left ? nv[u].z : nv[u].w];
            any = true;
          }
        }
        // ascending tree order within the lane (t = tb + 4u grows with u, then with tb)
#pragma unroll
        for (int u = 0; u < W; ++u) {
          if (!live[u]) continue;
          const double tw = tree_w[tb + 4 * u];
          const double* v = values + nv[u].y;
          for (int k = 0; k < K; ++k) {
            const double prod = tw * v[k];
            pr[k] = pr[k] + prod;
          }
        }
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < rows * K; e += 256) {
      const int r = e / K, k = e - r * K;
      double sacc = base ? base[k] : 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) sacc = sacc + part[(q * 64 + r) * K + k];
      out[(r0 + r) * K + k] = sacc;
    }
  }
}

// K8 on a heap-laid-out forest (single output, every tree depth <= 12).  Per tree, in int32 words
// (stride 2^(D+2) - 2): the 2^D - 1 internal slots as int2 {feature | -1 pass-through | -(f+2) categorical,
// threshold bits / mask offset} with the children of slot i at 2i+1 / 2i+2, then the 2^D leaf values of depth D
// as doubles.  A leaf shallower than D is stored as pass-through slots (go left) down to its leftmost depth-D
// descendant, which holds its value, so a walk is exactly D branch-uniform steps with no child loads or
// termination test, and ends in the leaf table.  LDS per tree equals the previous int2-per-slot form with fp32
// leaves (20 trees of depth 5: 10 KB), so 4 blocks still fit a CU at d = 100.  Same split semantics as
// predict_kernel: left iff x <= thr (NaN goes right), categorical left iff the category's mask bit is set.
// Sums in fp64 in predict_kernel's order (lane q = t % 4 ascending, then base + lanes 0..3, no contraction).
// (Two register sets refilled two tiles ahead with LDS-only barriers, as in binize5, measured 8.38 vs 7.78 ms at
// 1e8 x 100: kept one set.  predict_heap_binned_kernel's walk -- trees per wave as a template, no per-tree guards --
// measured 11.5 vs 7.8 ms here and was removed.)
__global__ __launch_bounds__(256) void predict_heap_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                           const int* __restrict__ heap, int depth,
                                                           const double* __restrict__ tree_w, int T,
                                                           const uint32_t* __restrict__ masks, double base,
                                                           float* __restrict__ out, double* __restrict__ out_d) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int NI = (1 << depth) - 1;     // internal slots per tree
  const int Wt = 4 * NI + 2;           // int32 words per tree: 2 NI (int2 slots) + 2 (NI + 1) (double leaves)
  int* sheap = reinterpret_cast<int*>(sm);
  double* stw = reinterpret_cast<double*>(sm + (size_t)T * Wt);  // T * Wt is even: 8-byte aligned
  float* sx = reinterpret_cast<float*>(stw + ((T + 1) & ~1));
  const int dp = d + 1;
  double* part = reinterpret_cast<double*>(sx + 64 * dp);
  for (int i = threadIdx.x; i < T * Wt; i += 256) sheap[i] = heap[i];
  for (int i = threadIdx.x; i < T; i += 256) stw[i] = tree_w[i];
  const int tl = threadIdx.x >> 6, row = threadIdx.x & 63;
  const bool vec = ldx == d && (d % 4) == 0;
  constexpr int kPre = 8;
  float4 pre[kPre];
  const int64_t stride = (int64_t)gridDim.x * 64;
  const bool use_pre = vec && 64 * d / 4 <= kPre * 256;
  auto fetch = [&](int64_t r0) {
    if (r0 >= n) return;
    const int rows = (int)((n - r0) < 64 ? (n - r0) : 64);
    const float4* src = reinterpret_cast<const float4*>(X + r0 * ldx);
    const int nv = rows * d / 4;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int i = threadIdx.x + k * 256;
      if (i < nv) pre[k] = src[i];
    }
  };
  if (use_pre) fetch((int64_t)blockIdx.x * 64);
  for (int64_t r0 = (int64_t)blockIdx.x * 64; r0 < n; r0 += stride) {
    const int rows = (int)((n - r0) < 64 ? (n - r0) : 64);
    __syncthreads();
    if (use_pre) {
      const int nv = rows * d / 4;
#pragma unroll
      for (int k = 0; k < kPre; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < nv) {
          const int e = i * 4, r = e / d, f = e - r * d;
          float* dst = sx + r * dp + f;
          dst[0] = pre[k].x;
          dst[1] = pre[k].y;
          dst[2] = pre[k].z;
          dst[3] = pre[k].w;
        }
      }
    } else {
      for (int e = threadIdx.x; e < rows * d; e += 256) {
        const int r = e / d, f = e - r * d;
        sx[r * dp + f] = X[(r0 + r) * ldx + f];
      }
    }
    __syncthreads();
    if (use_pre) fetch(r0 + stride);
    double acc = 0.0;
    if (row < rows) {
      const float* xr = sx + row * dp;
      constexpr int W = 8;
      for (int tb = tl; tb < T; tb += 4 * W) {
        int idx[W];
#pragma unroll
        for (int u = 0; u < W; ++u) idx[u] = 0;
        for (int s = 0; s < depth; ++s) {
#pragma unroll
          for (int u = 0; u < W; ++u) {
            const int t = tb + 4 * u;
            if (t >= T) continue;
            if (!CDNA_DCHECK(idx[u] < NI, 0x7E01u)) idx[u] = 0;  // walk left the internal slots
            const int2 nd = *reinterpret_cast<const int2*>(sheap + t * Wt + 2 * idx[u]);
            if (nd.x >= 0 && !CDNA_DCHECK(nd.x < d, 0x7E02u)) continue;  // split feature outside the row
            if (nd.x >= 0) {
              idx[u] = 2 * idx[u] + (xr[nd.x] <= __int_as_float(nd.y) ? 1 : 2);
            } else if (nd.x < -1) {
              const int c = (int)xr[-nd.x - 2];
              const bool left = (c >= 0 && c < 256) ? ((masks[nd.y * 8 + (c >> 5)] >> (c & 31)) & 1u) : false;
              idx[u] = 2 * idx[u] + (left ? 1 : 2);
            } else {
              idx[u] = 2 * idx[u] + 1;  // pass-through slot of a shallower leaf
            }
          }
        }
#pragma unroll
        for (int u = 0; u < W; ++u) {
          const int t = tb + 4 * u;
          if (t < T) {
            const int j = idx[u] - NI;
            if (!CDNA_DCHECK(j >= 0 && j <= NI, 0x7E03u)) continue;
            const double v = *reinterpret_cast<const double*>(sheap + t * Wt + 2 * NI + 2 * j);
            const double prod = stw[t] * v;
            acc = acc + prod;
          }
        }
      }
    }
    part[tl * 64 + row] = acc;
    __syncthreads();
    if (threadIdx.x < rows) {
      double v = base;
#pragma unroll
      for (int q = 0; q < 4; ++q) v = v + part[q * 64 + threadIdx.x];
      if (out_d)
        out_d[r0 + threadIdx.x] = v;  // the DoubleType prediction column directly
      else
        out[r0 + threadIdx.x] = (float)v;
    }
  }
}

// K8 over the training matrix's own bins: a transform of the very feature tensor a regression forest was fit on
// (models/inference.py ForestPredictor, forest.FitBins) reads the fit's uint8 bins -- 8 bytes per 8 features --
// instead of the fp32 rows.  bins [G][n] u64 words (binize: byte j of word g = feature 8 g + j's bin), thr_up
// [d][Bup] fp32: feature f's bin b -> t_b, the b-th sorted threshold the bins were cut with (+inf for b >= nthr).
// For a threshold v of feature f (every numeric heap slot holds one):  x <= v  <=>  t_bin(x) <= v.  bin(x) =
// #{t_j < x}, so t_bin(x) is the first threshold >= x: x <= t_bin(x) <= v gives x <= v; x <= v = t_b gives
// bin(x) <= b, so t_bin(x) <= t_b; NaN and x > t_last take bin nthr -> +inf and go right, as NaN <= v and x <= v
// are false.  t_b is non-decreasing in b, so t_bin(x) <= v  <=>  bin(x) < k(f, v) = #{b : t_b <= v}:
// heap_to_bins_kernel rewrites every numeric slot's threshold bits as that count once per call, and the walk
// compares bytes -- the same branches as predict_heap_kernel on X, the fp64 sums in its order: bit-identical
// predictions.  Categorical slots are not handled (the host keeps forests with categorical features on the fp32
// path).  (A first version looked t_bin up in an LDS table at every step -- a third dependent LDS read per step:
// 8.94 vs 7.88 ms for the fp32 kernel at 1e8 x 100.)
__global__ __launch_bounds__(256) void heap_to_bins_kernel(const int* __restrict__ heap, int T, int depth,
                                                           const float* __restrict__ thr_up, int Bup, int d,
                                                           int* __restrict__ heap_b) {
  const int NI = (1 << depth) - 1, Wt = 4 * NI + 2;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < T * Wt; i += gridDim.x * 256) {
    const int w = i % Wt;
    int v = heap[i];
    if (w < 2 * NI && (w & 1)) {
      const int f = heap[i - 1];
      if (f >= 0 && f < d) {
        const float t = __int_as_float(v);
        const float* row = thr_up + (size_t)f * Bup;
        int lo = 0, hi = Bup;  // first b with row[b] > t (row non-decreasing, +inf padded)
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (row[mid] <= t) lo = mid + 1; else hi = mid;
        }
        v = lo;
      }
    }
    heap_b[i] = v;
  }
}

// Tile: 64 rows x G words staged in LDS as binize's [g][row] words (one ds_write_b64 per word, contiguous; the
// walk's byte read of feature f = 8 g + j at (g 64 + row) 8 + j meets at most one other lane per bank), the next
// tile's words in registers while this tile walks.  Each wave (tl = wave index) walks trees tl, tl + 4, ... of its
// 64 rows, NT trees at a time with no per-tree guards inside the walk (a tree index past T walks tree T - 1 and is
// not summed), so the five-step chains of its trees interleave.  heap: heap_to_bins_kernel's.
// (PMC of the per-tree-guarded first version: 72 % of wave cycles waiting, 195 SALU + 90 LDS instructions per
// wave and 64-row tile, LDS 24 % bank-conflict cycles: 5.04 ms at 1e8 x 100.)
template <int NT>
__global__ __launch_bounds__(256) void predict_heap_binned_kernel(const uint64_t* __restrict__ bins, int64_t n, int G,
                                                                  int d, const int* __restrict__ heap, int depth,
                                                                  const double* __restrict__ tree_w, int T,
                                                                  double base, float* __restrict__ out,
                                                                  double* __restrict__ out_d) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int NI = (1 << depth) - 1;
  const int Wt = 4 * NI + 2;
  int* sheap = reinterpret_cast<int*>(sm);
  double* stw = reinterpret_cast<double*>(sm + (size_t)T * Wt);
  uint64_t* sb = reinterpret_cast<uint64_t*>(stw + ((T + 1) & ~1));               // [G][64] words
  double* part = reinterpret_cast<double*>(sb + 64 * G);
  for (int i = threadIdx.x; i < T * Wt; i += 256) sheap[i] = heap[i];
  for (int i = threadIdx.x; i < T; i += 256) stw[i] = tree_w[i];
  const int tl = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), row = threadIdx.x & 63;
  constexpr int kPre = 4;  // G <= 16 (d <= 128): 64 G words per tile = at most 4 per thread
  uint64_t pre[kPre];
  const int nw = 64 * G;
  const bool use_pre = nw <= kPre * 256;
  const int64_t stride = (int64_t)gridDim.x * 64;
  auto fetch = [&](int64_t r0) {
    if (r0 >= n) return;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int i = threadIdx.x + k * 256;
      const int64_t r = r0 + (i & 63);
      if (i < nw) pre[k] = r < n ? bins[(int64_t)(i >> 6) * n + r] : 0ull;
    }
  };
  if (use_pre) fetch((int64_t)blockIdx.x * 64);
  for (int64_t r0 = (int64_t)blockIdx.x * 64; r0 < n; r0 += stride) {
    const int rows = (int)((n - r0) < 64 ? (n - r0) : 64);
    __syncthreads();
    if (use_pre) {
#pragma unroll
      for (int k = 0; k < kPre; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < nw) sb[i] = pre[k];
      }
    } else {
      for (int i = threadIdx.x; i < nw; i += 256) {
        const int64_t r = r0 + (i & 63);
        sb[i] = r < n ? bins[(int64_t)(i >> 6) * n + r] : 0ull;
      }
    }
    __syncthreads();
    if (use_pre) fetch(r0 + stride);
    double acc = 0.0;
    if (row < rows) {
      const uint8_t* xb = reinterpret_cast<const uint8_t*>(sb) + row * 8;  // feature f: xb[(f >> 3) * 512 + (f & 7)]
      for (int tb = tl; tb < T; tb += 4 * NT) {
        const int* hp[NT];
        int idx[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int t = tb + 4 * u < T ? tb + 4 * u : T - 1;  // wave-uniform
          hp[u] = sheap + t * Wt;
          idx[u] = 0;
        }
        for (int s = 0; s < depth; ++s) {
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            const int2 nd = *reinterpret_cast<const int2*>(hp[u] + 2 * idx[u]);
            const int f = nd.x < 0 ? 0 : nd.x;
            const int b = xb[(f >> 3) * 512 + (f & 7)];
            // numeric: left iff bin < k; pass-through (-1): left
            idx[u] = 2 * idx[u] + ((nd.x < 0 || b < nd.y) ? 1 : 2);
          }
        }
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int t = tb + 4 * u;
          if (t < T) {
            const int j = idx[u] - NI;
            const double v = *reinterpret_cast<const double*>(hp[u] + 2 * NI + 2 * j);
            const double prod = stw[t] * v;
            acc = acc + prod;
          }
        }
      }
    }
    part[tl * 64 + row] = acc;
    __syncthreads();
    if (threadIdx.x < rows) {
      double v = base;
#pragma unroll
      for (int q = 0; q < 4; ++q) v = v + part[q * 64 + threadIdx.x];
      if (out_d)
        out_d[r0 + threadIdx.x] = v;
      else
        out[r0 + threadIdx.x] = (float)v;
    }
  }
}

// Leaf lookup on binned data (for GBDT training-set margin updates):
// out[r] += scale * value(leaf(r)) for a single tree in the compact
// level-array form used during training (split on bins).
__global__ __launch_bounds__(256) void predict_binned_kernel(const uint64_t* __restrict__ bins, int64_t n,
                                                             const int4* __restrict__ nodes, int root,
                                                             const float* __restrict__ values,
                                                             const uint32_t* __restrict__ masks, float scale,
                                                             float* __restrict__ out) {
  const uint8_t* b8 = reinterpret_cast<const uint8_t*>(bins);
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    int nd = root;
    int4 nv = nodes[nd];
    while (nv.x != -1) {
      bool left;
      if (nv.x >= 0) {
        const int bin = b8[((int64_t)(nv.x >> 3) * n + r) * 8 + (nv.x & 7)];
        left = bin <= nv.y;
      } else {
        const int f = -nv.x - 2;
        const int bin = b8[((int64_t)(f >> 3) * n + r) * 8 + (f & 7)];
        left = (masks[nv.y * 8 + (bin >> 5)] >> (bin & 31)) & 1u;
      }
      nd = left ? nv.z : nv.w;
      nv = nodes[nd];
    }
    out[r] += scale * values[nv.y];
  }
}

inline unsigned grid_for(int64_t n, int per, unsigned cap) {
  int64_t g = (n + per - 1) / per;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace

// miss_on: values that are NaN or equal miss_val are binned as -inf (XGBoost missing-value bin 0).
// rm (optional): also write the row-major copy [n][Gs] (Gs >= G words per row).  Returns 2 when the v1 kernel
// ran instead (rm not written).
// ldo: row stride of out's [G][ldo] word planes (0: n) -- chunks of a streamed fit bin into their row slice of
// the full bins (out = base + row0, ldo = total rows; rm = row-major base + row0).
// grid_mode bit 0: v5 launches exactly the resident blocks (one persistent round) instead of up to 1024.
// (Non-temporal loads of X and stores of the bins measured 29.8 vs 12.5 ms at 1e8 x 100 and were removed.)
CDNA_API int cdna_binize(const float* X, int64_t n, int d, int64_t ldx, const float* thr, const int* nthr, int tmax,
                         int miss_on, float miss_val, uint64_t* out, uint64_t* rm, int Gs, int64_t ldo, int lut,
                         int grid_mode, hipStream_t st) {
  if (ldo <= 0) ldo = n;
  if (ldo < n) return (int)hipErrorInvalidValue;
  // Gs == -10: rm gets the seg10 row layout (d <= 100, 128-byte rows; binize v5 only, see store_rm)
  const bool s10 = rm && Gs == -10;
  if (s10 && d > 100) return (int)hipErrorInvalidValue;
  if (rm && !s10 && Gs < (d + 7) / 8) return (int)hipErrorInvalidValue;
  if (n <= 0) return 0;
  if (d <= 128 && (d % 4) == 0 && (ldx % 4) == 0 && (reinterpret_cast<uintptr_t>(X) % 16) == 0 &&
      (!rm || Gs == 16 || s10)) {
    // v5: wave = (64-row tile, 8-feature group), lanes search the same tables (broadcast LDS reads)
    int steps = 0;
    while ((1 << steps) <= tmax) ++steps;
    if (steps < 4) steps = 4;
    const int G = (d + 7) / 8;
    constexpr int rpl = 1;  // 2 rows per lane (two tiles of registers, a 128-row LDS tile): 18.7 vs 15.4 ms
    // lut = cells per feature of the threshold grid (64 or 256), 0 = binary search only
    const int lut_cells = lut >= 256 ? 256 : (lut > 0 ? 64 : 0);
    const bool use_lut = lut_cells > 0;
    const size_t lds = (size_t)((d * (1 << steps) + 3) & ~3) * 4 + (size_t)64 * rpl * 17 * 8 +
                       (use_lut ? (size_t)d * lut_cells + (size_t)((2 * d + 3) & ~3) * 4 : 0);
    if (steps <= 8 && lds <= 150 * 1024 && (!use_lut || d <= 128)) {
      auto launch = [&](auto kern) {
        if (lds > 64 * 1024)
          (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds);
        unsigned grid = grid_for(n, 64 * rpl, 1024);
        if (grid_mode & 1) {
          const unsigned res = cdna::resident_blocks(reinterpret_cast<const void*>(kern), 64 * G, lds);
          if (res > 0 && res < grid) grid = res;
        }
        hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * G), lds, st, X, n, d, ldx, thr, nthr,
                           tmax > 0 ? tmax : 1, miss_on, miss_val, out, rm, Gs, ldo);
      };
      auto by_steps = [&](auto c_tag) {
        constexpr int CC = decltype(c_tag)::value;
        switch (steps) {
          case 4: launch(binize5_kernel<4, rpl, CC>); break;
          case 5: launch(binize5_kernel<5, rpl, CC>); break;
          case 6: launch(binize5_kernel<6, rpl, CC>); break;
          case 7: launch(binize5_kernel<7, rpl, CC>); break;
          default: launch(binize5_kernel<8, rpl, CC>); break;
        }
      };
      if (lut_cells == 256) by_steps(std::integral_constant<int, 256>{});
      else if (lut_cells == 64) by_steps(std::integral_constant<int, 64>{});
      else by_steps(std::integral_constant<int, 0>{});
      return (int)hipGetLastError();
    }
  }
  const bool rm_wanted = rm != nullptr;
  if (s10) rm = nullptr;  // the fallbacks write the standard layout only: report "rm not written" (2)
  {
    // v2: tile of rows in LDS next to the thresholds (<= 64 KB per block)
    const size_t tb = (size_t)d * (tmax > 0 ? tmax : 1) * 4 + (size_t)d * 4;
    const size_t dp = (size_t)(d | 1);
    // up to 64 KB per block (2+ blocks per CU); large threshold tables (maxBins 256 at d = 100: 100 KB)
    // opt in to 150 KB rather than falling back to v1 (253 ms at 1e8 x 100 x 256 bins)
    const size_t budget = tb + 64 * dp * 4 <= 64 * 1024 ? 64 * 1024 : 150 * 1024;
    // 32-row tiles: 29 KB blocks, 5 per CU (measured 22.6 ms vs 25.1 ms for 64-row tiles at 1e8 x 100 x 40
    // bins)
    int rpt = 32;
    while (rpt > 4 && ((size_t)rpt * dp * 4 + tb > budget || (size_t)rpt * d > 8192)) rpt /= 2;
    if ((size_t)rpt * dp * 4 + tb <= budget) {
      int steps = 0;
      while ((1 << steps) <= tmax) ++steps;
      const size_t lds = (size_t)rpt * dp * 4 + tb;
      if (lds > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(binize2_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(binize2_kernel, dim3(grid_for(n, rpt, 8192)), dim3(256), lds, st, X, n, d, ldx, thr, nthr,
                         tmax > 0 ? tmax : 1, rpt, steps, miss_on, miss_val, out, rm, Gs, ldo);
      const int e = (int)hipGetLastError();
      return e != 0 ? e : (s10 ? 2 : 0);
    }
  }
  const int G = (d + 7) / 8;
  const size_t tile = ((size_t)256 * G * 8 + 15) / 16 * 16;
  const size_t tbytes = (size_t)d * (tmax > 0 ? tmax : 1) * 4;
  const int use_lds = (tile + tbytes) <= 96 * 1024 ? 1 : 0;
  const size_t lds = tile + (use_lds ? tbytes : 0);
  if (tile > 120 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(binize_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), lds, st, X, n, d, ldx, thr, nthr,
                     tmax, use_lds, miss_on, miss_val, out, ldo);
  const int e = (int)hipGetLastError();
  return e != 0 ? e : (rm_wanted ? 2 : 0);
}

CDNA_API int cdna_partition(const uint64_t* bins, int64_t n, int T, int* node, const int* split_feat,
                            const int* split_bin, const int* cat_off, const uint32_t* cat_mask, const int* child,
                            hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  hipLaunchKernelGGL(partition_kernel, dim3(grid_for(n, 256, 2048), T), dim3(256), 0, st, bins, n, T, node,
                     split_feat, split_bin, cat_off, cat_mask, child);
  return (int)hipGetLastError();
}

CDNA_API int cdna_tree_predict(const float* X, int64_t n, int d, int64_t ldx, const int4* nodes, int64_t n_nodes_total,
                               const int* roots, const double* tree_w, int T, const double* values,
                               const uint32_t* masks, int K, const double* base, double* out, int64_t n_values,
                               hipStream_t st) {
  if (n <= 0) return 0;
  const size_t lds0 = (size_t)64 * (d + 1) * 4 + (size_t)4 * 64 * K * 8;
  if (lds0 > 160 * 1024) return (int)hipErrorInvalidValue;
  // forest copy in LDS when it fits next to the tile (<= 64 KB per block keeps 2 blocks / CU)
  int n_nodes = 0, n_vals = 0;
  const size_t room = lds0 < 64 * 1024 ? 64 * 1024 - lds0 : 0;
  n_nodes = n_nodes_total <= (int64_t)(room / 16) ? (int)n_nodes_total : 0;
  const size_t vbytes = (size_t)(((n_values + 1) & ~1) + ((T + 1) & ~1)) * 8 + (size_t)((T + 3) & ~3) * 4;
  if (n_nodes > 0 && n_values > 0 && (size_t)n_nodes * 16 + vbytes <= room) n_vals = (int)n_values;
  const size_t lds = lds0 + (size_t)n_nodes * 16 + (n_vals > 0 ? vbytes : 0);
  hipLaunchKernelGGL(predict_kernel, dim3(grid_for(n, 64, 8192)), dim3(256), lds, st, X, n, d, ldx, nodes, roots,
                     tree_w, T, values, masks, K, base, out, n_nodes, n_vals);
  return (int)hipGetLastError();
}

CDNA_API int cdna_predict_binned_add(const uint64_t* bins, int64_t n, const int4* nodes, int root,
                                     const float* values, const uint32_t* masks, float scale, float* out,
                                     hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(predict_binned_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, bins, n, nodes, root,
                     values, masks, scale, out);
  return (int)hipGetLastError();
}

// heap forest [T][2^(depth+2) - 2] int32 words (predict_heap_kernel), single output; returns
// hipErrorInvalidValue when it does not fit the LDS budget (the caller then uses cdna_tree_predict).
// grid_mode 1: exactly the resident blocks (one persistent round: the heap is staged once per resident block and
// every block walks the same number of 64-row tiles, +-1) instead of up to 8192 blocks.
CDNA_API int cdna_tree_predict_heap(const float* X, int64_t n, int d, int64_t ldx, const int* heap, int depth,
                                    const double* tree_w, int T, const uint32_t* masks, double base, float* out,
                                    double* out_d, int grid_mode, hipStream_t st) {
  if (n <= 0) return 0;
  if (depth < 0 || depth > 12) return (int)hipErrorInvalidValue;
  const size_t wt = ((size_t)4 << depth) - 2;
  const size_t lds = (size_t)T * wt * 4 + (size_t)((T + 1) & ~1) * 8 + (size_t)64 * (d + 1) * 4 + 256 * 8;
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  unsigned grid = grid_for(n, 64, 8192);
  if (grid_mode & 1) {
    const unsigned res = cdna::resident_blocks(reinterpret_cast<const void*>(predict_heap_kernel), 256, lds);
    if (res > 0 && res < grid) grid = res;
  }
  hipLaunchKernelGGL(predict_heap_kernel, dim3(grid), dim3(256), lds, st, X, n, d, ldx, heap,
                     depth, tree_w, T, masks, base, out, out_d);
  return (int)hipGetLastError();
}

// predict_heap_binned_kernel: bins [G][n] u64 (binize's column groups), thr_up [d][Bup] fp32; the heap as
// cdna_tree_predict_heap (numeric and pass-through slots only), heap_b: scratch of the heap's size (the slots
// rewritten as bin counts).  hipErrorInvalidValue when over the LDS budget.
CDNA_API int cdna_tree_predict_heap_binned(const uint64_t* bins, int64_t n, int G, int d, const float* thr_up,
                                           int Bup, const int* heap, int depth, const double* tree_w, int T,
                                           double base, int* heap_b, float* out, double* out_d, hipStream_t st) {
  if (n <= 0) return 0;
  if (depth < 0 || depth > 12 || G < 1 || d < 1 || d > 8 * G || Bup < 1 || Bup > 256) return (int)hipErrorInvalidValue;
  const size_t wt = ((size_t)4 << depth) - 2;
  const size_t lds = (size_t)T * wt * 4 + (size_t)((T + 1) & ~1) * 8 + (size_t)64 * G * 8 + 256 * 8;
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  const int64_t words = (int64_t)T * (int64_t)wt;
  hipLaunchKernelGGL(heap_to_bins_kernel, dim3(grid_for(words, 256, 64)), dim3(256), 0, st, heap, T, depth, thr_up,
                     Bup, d, heap_b);
  const dim3 grid(grid_for(n, 64, 8192));
  // NT = trees per wave and pass: ceil(T / 4) up to 8 (one pass), else passes of 8
  switch ((T + 3) / 4) {
    case 1: hipLaunchKernelGGL(predict_heap_binned_kernel<1>, grid, dim3(256), lds, st, bins, n, G, d, heap_b, depth,
                               tree_w, T, base, out, out_d); break;
    case 2: hipLaunchKernelGGL(predict_heap_binned_kernel<2>, grid, dim3(256), lds, st, bins, n, G, d, heap_b, depth,
                               tree_w, T, base, out, out_d); break;
    case 3: hipLaunchKernelGGL(predict_heap_binned_kernel<3>, grid, dim3(256), lds, st, bins, n, G, d, heap_b, depth,
                               tree_w, T, base, out, out_d); break;
    case 4: hipLaunchKernelGGL(predict_heap_binned_kernel<4>, grid, dim3(256), lds, st, bins, n, G, d, heap_b, depth,
                               tree_w, T, base, out, out_d); break;
    case 5: hipLaunchKernelGGL(predict_heap_binned_kernel<5>, grid, dim3(256), lds, st, bins, n, G, d, heap_b, depth,
                               tree_w, T, base, out, out_d); break;
    case 6: hipLaunchKernelGGL(predict_heap_binned_kernel<6>, grid, dim3(256), lds, st, bins, n, G, d, heap_b, depth,
                               tree_w, T, base, out, out_d); break;
    case 7: hipLaunchKernelGGL(predict_heap_binned_kernel<7>, grid, dim3(256), lds, st, bins, n, G, d, heap_b, depth,
                               tree_w, T, base, out, out_d); break;
    default: hipLaunchKernelGGL(predict_heap_binned_kernel<8>, grid, dim3(256), lds, st, bins, n, G, d, heap_b, depth,
                                tree_w, T, base, out, out_d); break;
  }
  return (int)hipGetLastError();
}

// The last split level of a regression forest written straight into its packed predict heap (depth D: the
// level's nodes sit at depth D - 1, their children are depth-D leaves), so the predict can follow the split
// scan on the GPU while the host turns the same decisions into the forest's node lists.  Per active node a
// (K6 row so[a] = gain, feature, bin, left W, left S, right W, right S, ...): the host's rule -- gain finite,
// > 0 and >= min_gain, node weight >= min_w -- splits it: internal slot key - 1 = (feature, fp32 threshold bits)
// and the two leaf values S / W (0 for an empty child) at depth-D leaf indices 2 key - 2^D, 2 key + 1 - 2^D.
// A node that does not split keeps the heap's pass-through slot and its own value, already in place.
__global__ __launch_bounds__(256) void heap_last_level_kernel(const double* __restrict__ so, int sw, int A,
                                                              const int* __restrict__ a_tree,
                                                              const int* __restrict__ a_key,
                                                              const double* __restrict__ a_w,
                                                              const float* __restrict__ thr, int Bt, int d,
                                                              double min_gain, double min_w, int* __restrict__ heap,
                                                              int D, int T) {
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (a >= A) return;
  const double* s = so + (int64_t)a * sw;
  const double gain = s[0];
  if (!(isfinite(gain) && gain > 0.0 && gain >= min_gain && a_w[a] >= min_w)) return;
  const int f = (int)s[1], b = (int)s[2], t = a_tree[a], k = a_key[a];
  const int NI = (1 << D) - 1;
  if (!CDNA_DCHECK(f >= 0 && f < d && b >= 0 && b < Bt && t >= 0 && t < T && k >= (1 << (D - 1)) && k <= NI,
                   0x4EA1u))
    return;  // a K6 row or heap key outside the tables
  int* h = heap + (int64_t)t * (4 * NI + 2);
  h[2 * (k - 1)] = f;
  h[2 * (k - 1) + 1] = __float_as_int(thr[(int64_t)f * Bt + b]);
  double* leaf = reinterpret_cast<double*>(h + 2 * NI);
  leaf[2 * k - (1 << D)] = s[3] > 0.0 ? s[4] / s[3] : 0.0;
  leaf[2 * k + 1 - (1 << D)] = s[5] > 0.0 ? s[6] / s[5] : 0.0;
}

CDNA_API int cdna_heap_last_level(const double* so, int sw, int A, const int* a_tree, const int* a_key,
                                  const double* a_w, const float* thr, int Bt, int d, double min_gain, double min_w,
                                  int* heap, int D, int T, hipStream_t st) {
  if (A <= 0) return 0;
  if (sw < 7 || D < 1 || D > 12 || T <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(heap_last_level_kernel, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, st, so, sw, A, a_tree,
                     a_key, a_w, thr, Bt, d, min_gain, min_w, heap, D, T);
  return (int)hipGetLastError();
}

CDNA_DEBUG_EXPORT(trees)
