// Single-tree "segment" mode: rows kept sorted by tree node (K5 + K7 for T = 1).
//
// Boosting grows one tree at a time (XGBoost / GBT: SURVEY A6, P9; DecisionTree
// A3).  The multi-tree row-record kernels (hist5.hip) scan EVERY row per pass
// and skip rows outside the pass's slot group; for one tree at depth 7 with
// 256 bins a pass holds 8 of the 64 built nodes, so the level re-reads all rows
// 8 x 13 times (36 ms of a 115 ms tree at 1e8 rows).  Here the active rows are
// a permutation `perm` grouped by node (one contiguous segment per active node)
// with the per-row statistics stored in the same order, so
//   * hist: a block owns (a chunk of ONE node's segment, one 8-feature group):
//     its LDS plane is a single node's 8 x B cells; it gathers the row's 8-bin
//     word through perm and reads the statistics contiguously;
//   * partition: a stable two-pass split of every segment into its children's
//     segments (pass 1 counts left rows per chunk, the host turns the counts
//     into output offsets, pass 2 scatters perm + statistics); rows of nodes
//     that became leaves are dropped, so perm shrinks level by level.
// Counts/sums are the same fixed-point integers as hist5 (bit-reproducible).
#include "common.h"
#include <cstdlib>

namespace {

typedef const __attribute__((address_space(4))) uint64_t cu64;  // constant address space: s_load when uniform
constexpr int kSegThreads = 256;
constexpr int kPackShift = 44;
constexpr int kPackQ = 1 << 23;

// work item: {start in perm, length, slot (hist) / segment (partition)}
struct SegHistArgs {
  const uint64_t* bins;  // [G][n]
  int64_t n;
  int d, B;
  const int* perm;
  const float* v0p;
  const float* v1p;
  const uint8_t* wp;
  const int* work;
  float qs0, qs1;
  unsigned long long* out;  // [S][d][B][2]
  // optional packed item records (flat kernel, REC): row | weight << 31 | (q1 + 2^23) << 39 (see CompactWArgs)
  const uint64_t* rec = nullptr;
  int rs = 0;  // row stride of the row-major bins in 8-byte words (0: G); 16 = one 128-byte line per row
  // 3-class records (kClsSplit): q = 1 (class 1) or 2^22 (class 2), so a block's sum w * q is W1 + 2^22 W2 with
  // W1 < 3 * 2^20 (the cells' 20-bit counts); the flush re-spaces it to W1 + 2^32 W2 so the global int64 sums of
  // many blocks (and ranks) keep the two fields apart
  int cls_split = 0;
};

constexpr int kClsSplit = 22;

// Flush one packed cell's (count, signed sum) into the int64 output: two columns, or for 3-class records
// (cls_split) three -- (W, W1, W2) with W1 = sum mod 2^22, W2 = sum >> 22 -- so the global sums of many blocks and
// ranks need no bound on W1 (round 5 re-spaced the sum to W1 + 2^32 W2 in one column, which required
// n_global * 255 < 2^32, i.e. <= 1.68e7 rows for the packed 3-class path).
__device__ __forceinline__ void flush_packed(const SegHistArgs& a, int64_t cell, unsigned long long cnt,
                                             long long sum) {
  if (a.cls_split) {
    unsigned long long* o = &a.out[cell * 3];
    atomicAdd(o, cnt);
    const long long lo = sum & ((1ll << a.cls_split) - 1ll), hi = sum >> a.cls_split;
    if (lo) atomicAdd(o + 1, (unsigned long long)lo);
    if (hi) atomicAdd(o + 2, (unsigned long long)hi);
  } else {
    unsigned long long* o = &a.out[cell * 2];
    atomicAdd(o, cnt);
    atomicAdd(o + 1, (unsigned long long)sum);
  }
}

// PACKED: one u64 atomic per update (count << 44 | sum of w * (q + 2^23)); the
// host bounds chunk length x max weight below 2^20 so neither field overflows.
// !PACKED: two u64 sums (w * q0, w * q1).
template <bool PACKED, bool HAS_W>
__global__ __launch_bounds__(kSegThreads) void seg_hist_kernel(const SegHistArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long h[];
  const int g = blockIdx.y;
  const int fbase = g * 8;
  const int start = a.work[3 * blockIdx.x], len = a.work[3 * blockIdx.x + 1], slot = a.work[3 * blockIdx.x + 2];
  const int plane = 8 * a.B;
  const int nplanes = PACKED ? 1 : 2;
  for (int i = threadIdx.x; i < plane * nplanes; i += kSegThreads) h[i] = 0ull;
  const int rot = threadIdx.x & 7;
  int fsel[8], fsh[8], foff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int jj = (j + rot) & 7;
    fsel[j] = jj >> 2;
    fsh[j] = (jj & 3) * 8;
    foff[j] = jj * a.B;
  }
  const int valid_f = a.d - fbase;
  const bool all8 = valid_f >= 8;
  const uint32_t fvalid = all8 ? 0xFFu : ((1u << (valid_f > 0 ? valid_f : 0)) - 1u);
  const uint32_t frot = ((fvalid >> rot) | (fvalid << (8 - rot))) & 0xFFu;
  __syncthreads();
  const uint64_t* bg = a.bins + (int64_t)g * a.n;
  const int* pp = a.perm + start;
  constexpr int U = 4;  // rows in flight per thread: perm loads, then gathers, then atomics
  for (int i0 = threadIdx.x; i0 < len; i0 += kSegThreads * U) {
    uint64_t b8[U];
    float x0[U], x1[U];
    uint32_t w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * kSegThreads;
      const bool ok = i < len;
      const int row = ok ? pp[i] : 0;
      b8[u] = ok ? bg[row] : 0ull;
      x1[u] = ok ? a.v1p[start + i] : 0.f;
      x0[u] = (!PACKED && ok) ? a.v0p[start + i] : 0.f;
      w[u] = ok ? (HAS_W ? (uint32_t)a.wp[start + i] : 1u) : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (w[u] == 0u) continue;
      const uint32_t lo = (uint32_t)b8[u], hi = (uint32_t)(b8[u] >> 32);
      int cell[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        cell[j] = foff[j] + (int)__builtin_amdgcn_ubfe(fsel[j] ? hi : lo, (uint32_t)fsh[j], 8u);
      if (PACKED) {
        int q1 = (int)rintf(x1[u] * a.qs1);
        q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
        const unsigned long long add =
            ((unsigned long long)w[u] << kPackShift) + (unsigned long long)w[u] * (unsigned long long)(q1 + kPackQ);
        if (all8) {
#pragma unroll
          for (int j = 0; j < 8; ++j) atomicAdd(h + cell[j], add);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if ((frot >> j) & 1u) atomicAdd(h + cell[j], add);
        }
      } else {
        const long long y0 = (long long)w[u] * (long long)(int)rintf(x0[u] * a.qs0);
        const long long y1 = (long long)w[u] * (long long)(int)rintf(x1[u] * a.qs1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (!all8 && !((frot >> j) & 1u)) continue;
          atomicAdd(h + cell[j], (unsigned long long)y0);
          atomicAdd(h + plane + cell[j], (unsigned long long)y1);
        }
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < plane; c += kSegThreads) {
    const int jj = c / a.B, bn = c - jj * a.B;
    const int f = fbase + jj;
    if (f >= a.d) continue;
    const int64_t cell = ((int64_t)slot * a.d + f) * a.B + bn;
    if (PACKED) {
      const unsigned long long v = h[c];
      if (!v) continue;
      const unsigned long long cnt = v >> kPackShift;
      flush_packed(a, cell, cnt, (long long)(v & ((1ull << kPackShift) - 1ull)) - (long long)kPackQ * (long long)cnt);
    } else {
      unsigned long long* o = &a.out[cell * 2];
      const unsigned long long v0 = h[c], v1 = h[plane + c];
      if (v0) atomicAdd(o, v0);
      if (v1) atomicAdd(o + 1, v1);
    }
  }
}

// Row-major variant: bins_rm[row][G] (a row's 8-bin words contiguous, one
// 128-byte line for up to 16 groups).  At deep levels a node's rows are sparse
// in row order, so the [G][n] layout costs one cache line PER GROUP per row
// (13 lines at d = 100) while only 8 bytes of each are used; here 8 lanes share
// a row (lane & 7 = group within the block's group range) and read its words
// with one coalesced access.  Blocks cover up to 8 groups (128 KB planes at
// B = 256, 1024 threads); rot = row-within-wave spreads LDS banks.
template <bool PACKED, bool HAS_W>
__global__ __launch_bounds__(1024) void seg_hist_rm_kernel(const SegHistArgs a, const uint64_t* __restrict__ bins_rm,
                                                           int G, int ngb) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long h[];
  constexpr int TH = 1024;
  const int g0 = blockIdx.y * ngb;
  const int ng = G - g0 < ngb ? G - g0 : ngb;
  const int start = a.work[3 * blockIdx.x], len = a.work[3 * blockIdx.x + 1], slot = a.work[3 * blockIdx.x + 2];
  const int plane_g = 8 * a.B;
  const int plane = ng * plane_g;
  const int nplanes = PACKED ? 1 : 2;
  for (int i = threadIdx.x; i < plane * nplanes; i += TH) h[i] = 0ull;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int gi = lane & 7, rsub = lane >> 3;
  const bool lane_on = gi < ng;
  const int g = g0 + (lane_on ? gi : 0);
  const int fbase = g * 8;
  const int rot = rsub;
  int fsel[8], fsh[8], foff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int jj = (j + rot) & 7;
    fsel[j] = jj >> 2;
    fsh[j] = (jj & 3) * 8;
    foff[j] = gi * plane_g + jj * a.B;
  }
  const int valid_f = a.d - fbase;
  const bool all8 = valid_f >= 8;
  const uint32_t fvalid = all8 ? 0xFFu : ((1u << (valid_f > 0 ? valid_f : 0)) - 1u);
  const uint32_t frot = ((fvalid >> rot) | (fvalid << (8 - rot))) & 0xFFu;
  __syncthreads();
  constexpr int RPI = TH / 8;  // rows per block iteration
  constexpr int U = 2;
  for (int i0 = wid * 8 + rsub; i0 < len; i0 += RPI * U) {
    uint64_t b8[U];
    float x0[U], x1[U];
    uint32_t w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * RPI;
      const bool ok = i < len && lane_on;
      const int row = ok ? a.perm[start + i] : 0;
      b8[u] = ok ? bins_rm[(int64_t)row * (a.rs ? a.rs : G) + g] : 0ull;
      x1[u] = ok ? a.v1p[start + i] : 0.f;
      x0[u] = (!PACKED && ok) ? a.v0p[start + i] : 0.f;
      w[u] = ok ? (HAS_W ? (uint32_t)a.wp[start + i] : 1u) : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (w[u] == 0u) continue;
      const uint32_t lo = (uint32_t)b8[u], hi = (uint32_t)(b8[u] >> 32);
      int cell[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        cell[j] = foff[j] + (int)__builtin_amdgcn_ubfe(fsel[j] ? hi : lo, (uint32_t)fsh[j], 8u);
      if (PACKED) {
        int q1 = (int)rintf(x1[u] * a.qs1);
        q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
        const unsigned long long add =
            ((unsigned long long)w[u] << kPackShift) + (unsigned long long)w[u] * (unsigned long long)(q1 + kPackQ);
        if (all8) {
#pragma unroll
          for (int j = 0; j < 8; ++j) atomicAdd(h + cell[j], add);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if ((frot >> j) & 1u) atomicAdd(h + cell[j], add);
        }
      } else {
        const long long y0 = (long long)w[u] * (long long)(int)rintf(x0[u] * a.qs0);
        const long long y1 = (long long)w[u] * (long long)(int)rintf(x1[u] * a.qs1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (!all8 && !((frot >> j) & 1u)) continue;
          atomicAdd(h + cell[j], (unsigned long long)y0);
          atomicAdd(h + plane + cell[j], (unsigned long long)y1);
        }
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < plane; c += TH) {
    const int gq = c / plane_g, rem = c - gq * plane_g;
    const int jj = rem / a.B, bn = rem - jj * a.B;
    const int f = (g0 + gq) * 8 + jj;
    if (f >= a.d) continue;
    const int64_t cell = ((int64_t)slot * a.d + f) * a.B + bn;
    if (PACKED) {
      const unsigned long long v = h[c];
      if (!v) continue;
      const unsigned long long cnt = v >> kPackShift;
      flush_packed(a, cell, cnt, (long long)(v & ((1ull << kPackShift) - 1ull)) - (long long)kPackQ * (long long)cnt);
    } else {
      unsigned long long* o = &a.out[cell * 2];
      const unsigned long long v0 = h[c], v1 = h[plane + c];
      if (v0) atomicAdd(o, v0);
      if (v1) atomicAdd(o + 1, v1);
    }
  }
}

// Flat row-major variant (packed statistics, all G groups in one block): the
// lanes of a wave take consecutive (row, group) PAIRS, so with G = 13 groups
// every lane is busy (the 8-lanes-per-row mapping above leaves 3 of every 16
// lanes idle at G = 13, and every idle lane still costs its share of each
// ds_add wave instruction).  A lane's 8 cells are updated in a rotated order;
// the partial last group (d % 8 != 0) masks its missing features per j, so the
// wave issues exactly 8 atomic instructions per pair round.
template <bool HAS_W, bool REC = false>
__global__ __launch_bounds__(1024) void seg_hist_flat_kernel(const SegHistArgs a, const uint64_t* __restrict__ bins_rm,
                                                             int G, int ngb) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long h[];
  constexpr int TH = 1024;
  const int start = a.work[3 * blockIdx.x], len = a.work[3 * blockIdx.x + 1], slot = a.work[3 * blockIdx.x + 2];
  // block y covers groups [g0, g0 + ng) (all of them when they fit 128 KB of LDS; B = 256 needs 2 blocks)
  const int g0 = blockIdx.y * ngb;
  const int ng = G - g0 < ngb ? G - g0 : ngb;
  const int plane_g = 8 * a.B;
  const int plane = ng * plane_g;
  for (int i = threadIdx.x; i < plane; i += TH) h[i] = 0ull;
  const int rot = threadIdx.x & 7;
  __syncthreads();
  const uint32_t total = (uint32_t)len * (uint32_t)ng;
  const uint32_t Gu = (uint32_t)ng;
  constexpr int U = 2;
  for (uint32_t q0 = threadIdx.x; q0 < total; q0 += TH * U) {
    uint64_t b8[U];
    float x1[U];
    uint32_t w[U];
    int g_[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t q = q0 + u * TH;
      const bool ok = q < total;
      const uint32_t i = ok ? q / Gu : 0u;
      const int g = ok ? (int)(q - i * Gu) : 0;  // group within the block's range
      g_[u] = g;
      if (REC) {
        // one 8-byte record per item instead of perm / v1p / wp: fewer, wider loads
        const uint64_t rc = ok ? a.rec[start + i] : 0ull;
        const int row = (int)(rc & 0x7FFFFFFFull);
        b8[u] = ok ? bins_rm[(int64_t)row * (a.rs ? a.rs : G) + g0 + g] : 0ull;
        w[u] = (uint32_t)(rc >> 31) & 0xFFu;
        x1[u] = __int_as_float((int)(uint32_t)(rc >> 39));  // carries q1 + 2^23 (bit pattern, not a float)
      } else {
        const int row = ok ? a.perm[start + i] : 0;
        b8[u] = ok ? bins_rm[(int64_t)row * (a.rs ? a.rs : G) + g0 + g] : 0ull;
        x1[u] = ok ? a.v1p[start + i] : 0.f;
        w[u] = ok ? (HAS_W ? (uint32_t)a.wp[start + i] : 1u) : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int g = g_[u];
      const int valid_f = a.d - (g0 + g) * 8;
      const uint32_t fvalid = w[u] == 0u ? 0u : (valid_f >= 8 ? 0xFFu : ((1u << (valid_f > 0 ? valid_f : 0)) - 1u));
      const uint32_t frot = ((fvalid >> rot) | (fvalid << (8 - rot))) & 0xFFu;
      const uint32_t lo = (uint32_t)b8[u], hi = (uint32_t)(b8[u] >> 32);
      uint32_t qb;  // q1 + 2^23
      if (REC) {
        qb = (uint32_t)__float_as_int(x1[u]);
      } else {
        int q1 = (int)rintf(x1[u] * a.qs1);
        q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
        qb = (uint32_t)(q1 + kPackQ);
      }
      const unsigned long long add =
          ((unsigned long long)w[u] << kPackShift) + (unsigned long long)w[u] * (unsigned long long)qb;
      const int gbase = g * plane_g;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int jj = (j + rot) & 7;
        const int cell = gbase + jj * a.B + (int)__builtin_amdgcn_ubfe(jj >= 4 ? hi : lo, (uint32_t)((jj & 3) * 8), 8u);
        if ((frot >> j) & 1u) atomicAdd(h + cell, add);
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < plane; c += TH) {
    const int gq = c / plane_g, rem = c - gq * plane_g;
    const int jj = rem / a.B, bn = rem - jj * a.B;
    const int f = (g0 + gq) * 8 + jj;
    if (f >= a.d) continue;
    const unsigned long long v = h[c];
    const unsigned long long cnt = v >> kPackShift;
    const long long sum = (long long)(v & ((1ull << kPackShift) - 1ull)) - (long long)kPackQ * (long long)cnt;
    if (!cnt) continue;
    flush_packed(a, ((int64_t)slot * a.d + f) * a.B + bn, cnt, sum);
  }
}

// Lane-feature variant (packed item records, row-major bins).  The flat
// kernel above gives each lane a (row, 8-feature group) pair: its cells are
// (feature, bin) = random bank pairs (rocprofv3: 67 % of LDS cycles bank
// conflicts) and every atomic costs ~12 VALU ops of cell arithmetic (VALU ~72 %
// busy).  Here each 32-lane HALF of a wave takes one item and lane l' of the
// half owns the 4 features of row dword l' (features f0 + 4l' + j):
//   * one dword load per lane brings the item's 4 bins;
//   * the LDS histogram is 4 byte-position planes [j][bin][32] u64, so the
//     cell of (l', j, bin) is j * PLANE + bin * 32 + l': the 32 lanes of a half
//     always hit 32 distinct bank pairs whatever the bins -- conflict-free;
//   * the cell byte address (bin << 8 | l' * 8) is ONE v_perm_b32 of the bins
//     dword and the lane offset, the plane offset j * PLANE * 8 an immediate.
// ~5.5 VALU and 2 ds_add_u64 per item (flat kernel: ~17 and 1.45 with 3x the
// LDS cycles per instruction).  Items past the chunk end load record 0 (weight
// 0: their adds are 0).  Dwords past d carry zero / in-range bins of slots the
// flush skips.
template <int BP>
__global__ __launch_bounds__(512) void seg_hist_lane_kernel(const SegHistArgs a, const uint8_t* __restrict__ bins8,
                                                            int row_bytes) {
  constexpr int TH = 512, NW = TH / 64, U = 16;
  constexpr int PLANE = BP * 32;
  // static: the planes sit at a link-time-known LDS offset, so the cell address needs no base add
  __shared__ __attribute__((aligned(16))) unsigned long long h[4 * PLANE];  // [4][BP][32]
  const int start = a.work[3 * blockIdx.x], len = a.work[3 * blockIdx.x + 1], slot = a.work[3 * blockIdx.x + 2];
  const int f0 = blockIdx.y * 128;
  for (int i = threadIdx.x; i < 4 * PLANE; i += TH) h[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63, half = lane >> 5, lq = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  int dw = (f0 >> 2) + lq;
  const int dmax = (row_bytes >> 2) - 1;
  dw = dw < dmax ? dw : dmax;
  const uint8_t* lbase = bins8 + 4 * dw;
  const uint32_t loff = (uint32_t)lq * 8u;
  // Record loads are unconditional (lane base + immediate offsets): the record buffer carries >= 2U readable
  // records past its end (codes_compact pads it), and a trip past the chunk end zeroes the out-of-range records
  // (row 0, weight 0) before they are used.  U = 16 item pairs per trip: the kernel is bound by the random
  // row-line gathers, so bytes in flight per CU set its speed (U = 8 with the next trip's records prefetched
  // was measured equal).
  // The wave's records are read through the scalar cache (constant address space, wave-uniform addresses:
  // s_load) and each half selects its item -- rocprofv3 had the texture-address unit ~80 % busy with one
  // 64-lane record load per item pair next to the gather; this leaves it the gathers alone (185.2 -> 181.0 ms).
  cu64* crec = (cu64*)(uintptr_t)(a.rec + start);
  for (int i0 = wid * 2 * U; i0 < len; i0 += NW * 2 * U) {
    uint64_t rc[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint64_t ra = crec[i0 + 2 * p], rb = crec[i0 + 2 * p + 1];
      rc[p] = half ? rb : ra;
    }
    if (i0 + 2 * U > len) {  // wave-uniform: the chunk's last trip
#pragma unroll
      for (int p = 0; p < U; ++p)
        if (i0 + 2 * p + half >= len) rc[p] = 0ull;
    }
    uint32_t x[U];
    unsigned long long add[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t lo = (uint32_t)rc[p], hi = (uint32_t)(rc[p] >> 32);
      const uint32_t row = lo & 0x7FFFFFFFu;
      x[p] = *reinterpret_cast<const uint32_t*>(lbase + (uint64_t)row * (uint64_t)row_bytes);
      const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, 31) & 0xFFu;
      const uint32_t qb = hi >> 7;  // q1 + 2^23
      add[p] = ((unsigned long long)(w << (kPackShift - 32)) << 32) + (unsigned long long)w * qb;
    }
#pragma unroll
    for (int p = 0; p < U; ++p) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t off = __builtin_amdgcn_perm(loff, x[p], 0x0C0C0004u | ((uint32_t)j << 8));  // bin<<8 | l'*8
        atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h) + off) + j * PLANE, add[p]);
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 4 * PLANE; c += TH) {
    const int j = c / PLANE, rem = c - j * PLANE;
    const int bn = rem >> 5, l = rem & 31;
    const int f = f0 + 4 * l + j;
    if (bn >= a.B || f >= a.d) continue;
    const unsigned long long v = h[c];
    if (!v) continue;
    const unsigned long long cnt = v >> kPackShift;
    const long long sum = (long long)(v & ((1ull << kPackShift) - 1ull)) - (long long)kPackQ * (long long)cnt;
    flush_packed(a, ((int64_t)slot * a.d + f) * a.B + bn, cnt, sum);
  }
}

// Quarter-wave record histogram for B <= 64 (the forest levels).  rocprofv3 on
// seg_hist_lane_kernel at the headline: texture-address unit ~79 % busy, LDS
// ~44 %, HBM ~2.8 TB/s -- the 64-lane address work of one dword gather per
// item PAIR binds it (moving the record loads to the scalar cache gained only
// 2.7 %).  Here a 16-lane quarter takes one item and lane l' gathers the 8-byte
// word l' of the row (features f0 + 8 l' + j): one dwordx2 gather serves FOUR
// items, half the address work per item.  The two items of a half-wave would
// collide on bank pairs (same l', same bin parity), so each keeps its own copy
// of the cells, interleaved per bin: [8 planes j][BP][2 copies][16 lanes] u64,
// cell byte address bin << 8 | copy << 7 | l' << 3 -- one v_perm_b32 as in the
// lane kernel, and the 32 lanes of a half always hit 32 distinct bank pairs.
// The flush adds the copies.  LDS = BP * 2 KB (80 KB at 40 bins: two
// 1024-thread blocks per CU).
template <int BP>
__global__ __launch_bounds__(1024, 2) void seg_hist_lane8_kernel(const SegHistArgs a, const uint8_t* __restrict__ bins8,
                                                                 int row_bytes) {
  constexpr int TH = 1024, NW = TH / 64, U = 8;
  constexpr int PLANE = BP * 32;  // u64 cells per feature plane j
  __shared__ __attribute__((aligned(16))) unsigned long long h[8 * PLANE];  // [8][BP][2][16]
  const int start = a.work[3 * blockIdx.x], len = a.work[3 * blockIdx.x + 1], slot = a.work[3 * blockIdx.x + 2];
  const int f0 = blockIdx.y * 128;
  if (!CDNA_DCHECK(start >= 0 && len >= 0 && slot >= 0, 0x5E82u)) return;  // corrupt work item
  for (int i = threadIdx.x; i < 8 * PLANE; i += TH) h[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63, qt = lane >> 4, lq = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  int qw = (f0 >> 3) + lq;  // the lane's 8-byte word of the row
  const int qmax = (row_bytes >> 3) - 1;
  qw = qw < qmax ? qw : qmax;
  const uint8_t* lbase = bins8 + 8 * qw;
  const uint32_t loff = (uint32_t)(qt & 1) * 128u + (uint32_t)lq * 8u;  // copy << 7 | l' << 3
  static_assert(4 * U <= 64, "record over-read must stay within REC_PAD");
  // per-quarter vector record loads (scalar-cache records with a 4-way select: 174.6 vs 170.8 ms headline)
  const uint64_t* __restrict__ recp = a.rec + start + qt;
  for (int i0 = wid * 4 * U; i0 < len; i0 += NW * 4 * U) {
    uint64_t rc[U];
#pragma unroll
    for (int p = 0; p < U; ++p) rc[p] = recp[i0 + 4 * p];
    if (i0 + 4 * U > len) {
#pragma unroll
      for (int p = 0; p < U; ++p)
        if (i0 + 4 * p + qt >= len) rc[p] = 0ull;
    }
    uint2 x[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      uint32_t row = (uint32_t)rc[p] & 0x7FFFFFFFu;
      if (!CDNA_DCHECK((int64_t)row < a.n, 0x5E81u)) row = 0u;  // record row outside the bins
      x[p] = *reinterpret_cast<const uint2*>(lbase + (uint64_t)row * (uint64_t)row_bytes);
    }
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t lo = (uint32_t)rc[p], hi = (uint32_t)(rc[p] >> 32);
      const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, 31) & 0xFFu;
      const unsigned long long add = ((unsigned long long)(w << (kPackShift - 32)) << 32) +
                                     (unsigned long long)w * (hi >> 7);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t off = __builtin_amdgcn_perm(loff, j < 4 ? x[p].x : x[p].y, 0x0C0C0004u | ((uint32_t)(j & 3) << 8));
        atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h) + off) + j * PLANE, add);
      }
    }
  }
  __syncthreads();
  // flush: thread -> (plane j, bin, lane l'), both copies summed
  for (int c = threadIdx.x; c < 8 * BP * 16; c += TH) {
    const int l = c & 15, rest = c >> 4;
    const int bn = rest % BP, j = rest / BP;
    const int f = f0 + 8 * l + j;
    if (bn >= a.B || f >= a.d) continue;
    const unsigned long long* cell = h + j * PLANE + bn * 32 + l;
    const unsigned long long v0 = cell[0], v1 = cell[16];
    const unsigned long long cnt = (v0 >> kPackShift) + (v1 >> kPackShift);
    if (!cnt) continue;
    const unsigned long long m = (1ull << kPackShift) - 1ull;
    const long long sum = (long long)((v0 & m) + (v1 & m)) - (long long)kPackQ * (long long)cnt;
    flush_packed(a, ((int64_t)slot * a.d + f) * a.B + bn, cnt, sum);
  }
}

// Six items per wave for 80 < d <= 100, B <= 40 (the headline forest levels).
// The cost of seg_hist_lane8 is its ds_add_u64 wave instructions (~6 LDS
// cycles each: the address and 8-byte data VGPRs move to the LDS at 2 cycles
// per dword, active lanes or not), and at d = 100 its 4 items x 16 lanes x 8
// features offer 512 lane slots for 400 updates (78 %).  Here the bins rows
// are in the "seg10" layout (binize v5, Gs = -10: ten 12-byte chunks of 10
// features per 128-byte row) and each 32-lane half takes THREE items: lane
// l' = 10 c + s (c = item of the half, s = chunk) gathers its item's chunk s
// with one dwordx3 load and makes 10 updates; lanes 30 / 31 of each half add 0.
// 6 items x 100 updates per 10 wave instructions (94 %): 1.67 instead of 2.0
// atomics per item, and one gather instruction per 6 items instead of 4.
// Cells: [10 planes j][BP][32 columns] u64 with column = l' (item c's copy of
// chunk s), so the 32 lanes of a half hit 32 distinct bank pairs whatever the
// bins (cell byte address bin << 8 | l' << 3: one v_perm_b32, as in lane8);
// the flush adds the three copies.  LDS = BP * 2.5 KB (100 KB at 40 bins:
// one 1024-thread block per CU).
template <int BP, int U>
__global__ __launch_bounds__(1024) void seg_hist_lane10_kernel(const SegHistArgs a, const uint8_t* __restrict__ bins8) {
  constexpr int TH = 1024, NW = TH / 64, IPW = 6;
  constexpr int PLANE = BP * 32;  // u64 cells per feature plane j
  __shared__ __attribute__((aligned(16))) unsigned long long h[10 * PLANE];  // [10][BP][32]
  const int start = a.work[3 * blockIdx.x], slot = a.work[3 * blockIdx.x + 2];
  const int len = a.work[3 * blockIdx.x + 1];
  if (!CDNA_DCHECK(start >= 0 && len >= 0 && slot >= 0, 0x5E83u)) return;  // corrupt work item
  for (int i = threadIdx.x; i < 10 * PLANE; i += TH) h[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int c = l32 / 10, s = l32 - 10 * c;  // c = 3: lanes 30 / 31 (no item)
  const bool on = c < 3;
  const int item = half * 3 + (on ? c : 0);
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint8_t* lbase = bins8 + 12 * (on ? s : 0);
  const uint32_t loff = (uint32_t)l32 * 8u;  // column << 3
  static_assert(IPW * U <= 128, "record over-read must stay within REC_PAD");
  const uint64_t* __restrict__ recp = a.rec + start + item;
  // U = 16 items per lane per trip (160 atomics): the trip's record load and gather latencies are exposed
  // once per trip, so the other 15 waves of the CU need ~15 x 160 ds_add_u64 of work to cover them (U = 8:
  // 13.7 ms per level; a two-set software pipeline did not survive the compiler's loop rotation; round 6: the
  // NEXT trip's records prefetched during this trip's atomics, which fits 128 VGPRs only at U = 12 / 8, measured
  // 127.0-127.5 / 128.0-128.3 vs 126.3-126.7 ms per headline step -- the gathers in flight per trip matter more)
  for (int i0 = wid * IPW * U; i0 < len; i0 += NW * IPW * U) {
    uint64_t rc[U];
#pragma unroll
    for (int p = 0; p < U; ++p) rc[p] = recp[i0 + IPW * p];
    if (!on) {
#pragma unroll
      for (int p = 0; p < U; ++p) rc[p] = 0ull;
    } else if (i0 + IPW * U > len) {
#pragma unroll
      for (int p = 0; p < U; ++p)
        if (i0 + IPW * p + item >= len) rc[p] = 0ull;
    }
    uint32_t x0[U], x1[U], x2[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      uint32_t row = (uint32_t)rc[p] & 0x7FFFFFFFu;
      if (!CDNA_DCHECK((int64_t)row < a.n, 0x5E84u)) row = 0u;  // record row outside the bins
      const uint3 v = *reinterpret_cast<const uint3*>(lbase + (uint64_t)row * 128u);
      x0[p] = v.x; x1[p] = v.y; x2[p] = v.z;
    }
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t lo = (uint32_t)rc[p], hi = (uint32_t)(rc[p] >> 32);
      const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, 31) & 0xFFu;
      const unsigned long long add = ((unsigned long long)(w << (kPackShift - 32)) << 32) +
                                     (unsigned long long)w * (hi >> 7);
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const uint32_t src = j < 4 ? x0[p] : (j < 8 ? x1[p] : x2[p]);
        const uint32_t off = __builtin_amdgcn_perm(loff, src, 0x0C0C0004u | ((uint32_t)(j & 3) << 8));
        atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h) + off) + j * PLANE, add);
      }
    }
  }
  __syncthreads();
  // flush: thread -> (plane j, bin, chunk s), the three item copies summed
  for (int e = threadIdx.x; e < 10 * BP * 10; e += TH) {
    const int sc = e % 10, rest = e / 10;
    const int bn = rest % BP, j = rest / BP;
    const int f = 10 * sc + j;
    if (bn >= a.B || f >= a.d) continue;
    const unsigned long long* cell = h + j * PLANE + bn * 32 + sc;
    const unsigned long long v0 = cell[0], v1 = cell[10], v2 = cell[20];
    const unsigned long long cnt = (v0 >> kPackShift) + (v1 >> kPackShift) + (v2 >> kPackShift);
    if (!cnt) continue;
    const unsigned long long m = (1ull << kPackShift) - 1ull;
    const long long sum = (long long)((v0 & m) + (v1 & m) + (v2 & m)) - (long long)kPackQ * (long long)cnt;
    flush_packed(a, ((int64_t)slot * a.d + f) * a.B + bn, cnt, sum);
  }
}

// Levels with at most one built node per tree (level 0: the roots; level 1:
// the smaller child) without item records: the level's records (row, weight,
// quantised label) are the row-order compaction of each tree's codes for that
// node -- 1.26e9 records at level 0 of the headline, written and read back
// once (count + scatter: ~4.3 ms per step at level 0, ~3 ms at level 1).
// Here a work item is (slot, row range), sinfo[slot] = (tree, local node), and
// each wave compacts its own rows' records on the fly into a 256-entry LDS ring: one coalesced 64-row load of
// the tree's codes and labels (the next window's already in flight), a ballot
// and mbcnt rank, one ds_write_b64 per item; then the lane10 trip consumes 96
// ring entries.  The gathers of a wave walk consecutive rows (each line is read
// by ~0.63 x 20 trees: the XCD-aware work order puts the trees of one row chunk
// on one XCD back to back, so the L2 serves most of them).  Same int64 sums as
// the record path (the sums do not depend on the item order).
// DRAW (level 0 of a bootstrapped forest): the rows' Poisson bootstrap weights are drawn here (the same Philox
// uniforms and tabulated CDF as misc.hip poisson_kernel, keyed by global row id) instead of read from the codes,
// and the level's codes (weight << 8 | 0, 0xFF for weight 0) are written for the partition -- no separate draws
// kernel in series ahead of the histogram: the ~100 VALU instructions of a window's Philox calls run in the
// shadow of its ~70 ds_add_u64 (the kernel is LDS-bound, its VALU mostly idle).
struct RootDraw {
  uint64_t seed, offset;  // Philox key, global row id of local row 0
  double rate;
  cdna::PoissonCdf cdf;
};

template <int BP, bool DRAW>
__global__ __launch_bounds__(1024) void seg_hist_lane10_root_kernel(const SegHistArgs a, const uint8_t* __restrict__ bins8,
                                                                    const uint16_t* __restrict__ codes,
                                                                    const float* __restrict__ v1, float qs1,
                                                                    const int* __restrict__ sinfo, int slot0,
                                                                    const RootDraw dr) {
  constexpr int TH = 1024, NW = TH / 64, U = 16, IPW = 6, NI = IPW * U, RING = 256;  // NI - 1 + 64 < RING
  constexpr int PLANE = BP * 32;
  __shared__ __attribute__((aligned(16))) unsigned long long h[10 * PLANE];  // [10][BP][32]
  __shared__ __attribute__((aligned(16))) uint64_t ring[NW][RING];
  const int r0 = a.work[3 * blockIdx.x], len = a.work[3 * blockIdx.x + 1], slot = a.work[3 * blockIdx.x + 2];
  const int tree = sinfo[2 * slot];
  const uint32_t node = (uint32_t)sinfo[2 * slot + 1];
  if (!CDNA_DCHECK(r0 >= 0 && len >= 0 && slot >= slot0 && tree >= 0 && node < 0xFFu && (int64_t)r0 + len <= a.n,
                   0x5E85u)) return;
  for (int i = threadIdx.x; i < 10 * PLANE; i += TH) h[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int c = l32 / 10, s = l32 - 10 * c;
  const bool on = c < 3;
  const int item = half * 3 + (on ? c : 0);
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint8_t* lbase = bins8 + 12 * (on ? s : 0);
  const uint32_t loff = (uint32_t)l32 * 8u;
  const uint16_t* ct = codes + (int64_t)tree * a.n;
  uint16_t* cw_out = DRAW ? const_cast<uint16_t*>(ct) : nullptr;
  uint64_t* rg = ring[wid];
  // the wave's rows: a contiguous 64-aligned share of the block's range
  const int per = ((len + NW - 1) / NW + 63) & ~63;
  int64_t wr = (int64_t)r0 + (int64_t)wid * per;
  const int64_t wend = (int64_t)r0 + len < wr + per ? (int64_t)r0 + len : wr + per;
  uint32_t head = 0u, tail = 0u;  // wave-uniform ring cursors
  uint32_t ncw = 0xFFu;
  float ny = 0.f;
  auto fetch = [&](int64_t r) {
    if (DRAW) {
      const uint32_t w = cdna::poisson_draw(cdna::bootstrap_uniform(dr.seed, dr.offset + (uint64_t)r, tree), dr.cdf,
                                            dr.rate);
      ncw = (w << 8) | (w ? 0u : 0xFFu);
      if (r < wend) cw_out[r] = (uint16_t)ncw;
      else ncw = 0xFFu;
    } else {
      ncw = r < wend ? (uint32_t)ct[r] : 0xFFu;
    }
    ny = r < wend ? v1[r] : 0.f;
  };
  fetch(wr + lane);
  for (;;) {
    while (tail - head < (uint32_t)NI && wr < wend) {  // wave-uniform refill, one 64-row window per round
      const uint32_t cw = ncw;
      const float y = ny;
      const int64_t r = wr + lane;
      wr += 64;
      fetch(wr + lane);
      const bool has = (cw & 0xFFu) == node && (cw >> 8) != 0u;
      const uint64_t m = __builtin_amdgcn_ballot_w64(has);
      if (has) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        int q1 = (int)rintf(y * qs1);
        q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
        rg[(tail + rank) & (RING - 1)] =
            (uint64_t)r | ((uint64_t)(cw >> 8) << 31) | ((uint64_t)(uint32_t)(q1 + kPackQ) << 39);
      }
      tail += (uint32_t)__builtin_popcountll(m);
    }
    const uint32_t avail = tail - head;
    if (avail == 0u) break;  // wave-uniform: rows exhausted and ring drained
    asm volatile("" ::: "memory");  // the ring writes above are issued before the reads below (LDS: in order)
    uint64_t rc[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t k = (uint32_t)(IPW * p + item);
      rc[p] = (on && k < avail) ? rg[(head + k) & (RING - 1)] : 0ull;
    }
    head += avail < (uint32_t)NI ? avail : (uint32_t)NI;
    uint32_t x0[U], x1[U], x2[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t row = (uint32_t)rc[p] & 0x7FFFFFFFu;
      const uint3 v = *reinterpret_cast<const uint3*>(lbase + (uint64_t)row * 128u);
      x0[p] = v.x; x1[p] = v.y; x2[p] = v.z;
    }
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t lo = (uint32_t)rc[p], hi = (uint32_t)(rc[p] >> 32);
      const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, 31) & 0xFFu;
      const unsigned long long add = ((unsigned long long)(w << (kPackShift - 32)) << 32) +
                                     (unsigned long long)w * (hi >> 7);
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const uint32_t src = j < 4 ? x0[p] : (j < 8 ? x1[p] : x2[p]);
        const uint32_t off = __builtin_amdgcn_perm(loff, src, 0x0C0C0004u | ((uint32_t)(j & 3) << 8));
        atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h) + off) + j * PLANE, add);
      }
    }
    asm volatile("" ::: "memory");  // this trip's ring reads are issued before the next refill overwrites
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 10 * BP * 10; e += TH) {
    const int sc = e % 10, rest = e / 10;
    const int bn = rest % BP, j = rest / BP;
    const int f = 10 * sc + j;
    if (bn >= a.B || f >= a.d) continue;
    const unsigned long long* cell = h + j * PLANE + bn * 32 + sc;
    const unsigned long long v0 = cell[0], v1c = cell[10], v2 = cell[20];
    const unsigned long long cnt = (v0 >> kPackShift) + (v1c >> kPackShift) + (v2 >> kPackShift);
    if (!cnt) continue;
    const unsigned long long m = (1ull << kPackShift) - 1ull;
    const long long sum = (long long)((v0 & m) + (v1c & m) + (v2 & m)) - (long long)kPackQ * (long long)cnt;
    flush_packed(a, ((int64_t)(slot - slot0) * a.d + f) * a.B + bn, cnt, sum);
  }
}

// Wide-bin lane variant (80 < B <= 256: XGBoost-style 256-bin boosting).  Four
// [BP][32] u64 planes of 256 bins would need 256 KB of LDS, so a block covers
// 64 features: each 16-lane QUARTER of a wave takes one item and lane l' owns
// the 4 features of row dword l' (one dword gather), so one record load + one
// gather serve four items.  A first version (one item per 32-lane half, two
// features per lane, conflict-free [2][BP][32] planes) had rocprofv3 show the
// texture-address unit ~80 % busy (one record load + one u16 gather per PAIR
// of items) with LDS ~20 % busy; this one halves the address work and costs
// 784.5 -> 670.8 ms per 20 GBDT trees.  Planes [4][BP][16] u64 (128 KB at
// BP = 256, one 1024-thread block per CU); the two items of a half-wave collide
// on a bank pair when their bins at the same l' share parity, so an atomic
// costs ~2 passes -- LDS has the headroom.  The cell byte offset
// bin << 7 | l' << 3 (+ plane) is a bfe and an lshl_or.
// XCD-aware 1-D grid: block b runs on XCD b % 8, and the ny feature blocks of
// chunk c are slots k = (c / 8) * ny + y of XCD c % 8 -- dispatched back to
// back, so the second half of each gathered 128-byte row line hits the L2 the
// first half filled (the x-major 2-D order re-fetched every line: 867 -> 789 ms
// per 20 trees when fixed).
template <int BP, int U>
__global__ __launch_bounds__(1024) void seg_hist_lane4_kernel(const SegHistArgs a, const uint8_t* __restrict__ bins8,
                                                              int row_bytes, int nwork, int ny) {
  constexpr int TH = 1024, NW = TH / 64;
  constexpr int PLANE = BP * 16;
  static_assert(BP == 128 || BP == 256, "four planes of 128 or 256 bins");
  __shared__ __attribute__((aligned(16))) unsigned long long h[4 * PLANE];  // [4][BP][16]
  const int b = blockIdx.x, k = b >> 3;
  const int c = (k / ny) * 8 + (b & 7), fy = k - (k / ny) * ny;
  if (c >= nwork) return;
  const int start = a.work[3 * c], len = a.work[3 * c + 1], slot = a.work[3 * c + 2];
  const int f0 = fy * 64;
  for (int i = threadIdx.x; i < 4 * PLANE; i += TH) h[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63, qt = lane >> 4, lq = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  int dw = (f0 >> 2) + lq;
  const int dmax = (row_bytes >> 2) - 1;
  dw = dw < dmax ? dw : dmax;
  const uint8_t* lbase = bins8 + 4 * dw;
  const uint32_t loff = (uint32_t)lq * 8u;
  // unconditional record loads reach 4U - 1 records past the chunk end: REC_PAD (64) covers U <= 16
  static_assert(4 * U <= 64, "record over-read must stay within REC_PAD");
  // per-quarter vector record loads (scalar-cache records with a 4-way select measured 743.6 vs 671.1 ms per 20
  // GBDT trees: four selects per item and the lgkmcnt drain of the atomics before every trip)
  const uint64_t* __restrict__ recp = a.rec + start + qt;
  for (int i0 = wid * 4 * U; i0 < len; i0 += NW * 4 * U) {
    uint64_t rc[U];
#pragma unroll
    for (int p = 0; p < U; ++p) rc[p] = recp[i0 + 4 * p];
    if (i0 + 4 * U > len) {
#pragma unroll
      for (int p = 0; p < U; ++p)
        if (i0 + 4 * p + qt >= len) rc[p] = 0ull;
    }
    uint32_t x[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t row = (uint32_t)rc[p] & 0x7FFFFFFFu;
      x[p] = *reinterpret_cast<const uint32_t*>(lbase + (uint64_t)row * (uint64_t)row_bytes);
    }
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t lo = (uint32_t)rc[p], hi = (uint32_t)(rc[p] >> 32);
      const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, 31) & 0xFFu;
      const unsigned long long add = ((unsigned long long)(w << (kPackShift - 32)) << 32) +
                                     (unsigned long long)w * (hi >> 7);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t off = (__builtin_amdgcn_ubfe(x[p], 8u * j, 8u) << 7) | loff;  // bin << 7 | l' << 3
        atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h) + off) + j * PLANE, add);
      }
    }
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < 4 * PLANE; cc += TH) {
    const int b_lo = cc & 7, l = (cc >> 3) & 15, j = (cc >> 7) & 3, b_hi = cc >> 9;
    const int bn = b_hi * 8 + b_lo;
    const int f = f0 + 4 * l + j;
    if (bn >= a.B || f >= a.d) continue;
    const unsigned long long v = h[j * PLANE + bn * 16 + l];
    if (!v) continue;
    const unsigned long long cnt = v >> kPackShift;
    const long long sum = (long long)(v & ((1ull << kPackShift) - 1ull)) - (long long)kPackQ * (long long)cnt;
    flush_packed(a, ((int64_t)slot * a.d + f) * a.B + bn, cnt, sum);
  }
}

struct SegPartArgs {
  const uint64_t* bins;
  int64_t n;
  const int* perm;
  const float* v0p;
  const float* v1p;
  const uint8_t* wp;
  const int* work;        // {start, len, seg}
  const int* split_feat;  // [A] (-1: leaf, rows dropped)
  const int* split_bin;
  const int* cat_off;     // [A] (-1: ordered split)
  const uint32_t* cat_mask;  // [*][8]
  const int* left_base;   // [chunks] output offset of this chunk's first left row (-1: child is a leaf)
  const int* right_base;
  int* left_cnt;          // pass 1 output [chunks]
  int* perm_out;
  float* v0_out;
  float* v1_out;
  uint8_t* w_out;
  // implicit_n > 0: level-0 multi-tree entry.  Segment s is tree s over rows
  // [0, n): perm is the identity (row = start + i - s * n), wp is the [T][n]
  // bootstrap weight matrix (indexed like the virtual perm), v0p/v1p are the
  // unpermuted per-row statistics (indexed by row), and weight-0 rows are dropped.
  int64_t implicit_n;
  int* right_cnt;         // pass 1 output [chunks] (rows kept on the right)
};

struct SegRow {
  int row;
  bool keep;
};

__device__ __forceinline__ SegRow seg_row(const SegPartArgs& a, int seg, int64_t idx) {
  if (a.implicit_n > 0) return SegRow{(int)(idx - (int64_t)seg * a.implicit_n), a.wp[idx] != 0};
  return SegRow{a.perm[idx], true};
}

__device__ __forceinline__ bool seg_left(const SegPartArgs& a, int seg, int row) {
  const int f = a.split_feat[seg];
  const int bin = (int)reinterpret_cast<const uint8_t*>(a.bins)[((int64_t)(f >> 3) * a.n + row) * 8 + (f & 7)];
  const int co = a.cat_off[seg];
  return co >= 0 ? ((a.cat_mask[co * 8 + (bin >> 5)] >> (bin & 31)) & 1u) != 0u : bin <= a.split_bin[seg];
}

__global__ __launch_bounds__(kSegThreads) void seg_count_kernel(const SegPartArgs a) {
  const int start = a.work[3 * blockIdx.x], len = a.work[3 * blockIdx.x + 1], seg = a.work[3 * blockIdx.x + 2];
  __shared__ int red[kSegThreads / 64];
  __shared__ int redr[kSegThreads / 64];
  int c = 0, r = 0;
  if (a.split_feat[seg] >= 0)
    for (int i = threadIdx.x; i < len; i += kSegThreads) {
      const SegRow sr = seg_row(a, seg, (int64_t)start + i);
      if (!sr.keep) continue;
      const bool l = seg_left(a, seg, sr.row);
      c += l ? 1 : 0;
      r += l ? 0 : 1;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    r += __shfl_xor(r, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = c;
    redr[threadIdx.x >> 6] = r;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0, sr = 0;
#pragma unroll
    for (int k = 0; k < kSegThreads / 64; ++k) {
      s += red[k];
      sr += redr[k];
    }
    a.left_cnt[blockIdx.x] = s;
    if (a.right_cnt) a.right_cnt[blockIdx.x] = sr;
  }
}

// Stable scatter: rounds of 256 rows; a row's rank among this chunk's left
// (right) rows = ballot prefix within the wave + the earlier waves' totals.
__global__ __launch_bounds__(kSegThreads) void seg_scatter_kernel(const SegPartArgs a) {
  const int start = a.work[3 * blockIdx.x], len = a.work[3 * blockIdx.x + 1], seg = a.work[3 * blockIdx.x + 2];
  if (a.split_feat[seg] < 0) return;
  const int lb = a.left_base[blockIdx.x], rbase = a.right_base[blockIdx.x];
  __shared__ int wl[kSegThreads / 64];
  __shared__ int wr[kSegThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool implicit = a.implicit_n > 0;
  int done_l = 0, done_r = 0;
  for (int i0 = 0; i0 < len; i0 += kSegThreads) {
    const int i = i0 + threadIdx.x;
    const bool ok = i < len;
    const SegRow sr = ok ? seg_row(a, seg, (int64_t)start + i) : SegRow{0, false};
    const int row = sr.row;
    const bool left = sr.keep && seg_left(a, seg, row);
    const bool right = sr.keep && !left;
    const uint64_t m = __builtin_amdgcn_ballot_w64(left);
    const uint64_t mr = __builtin_amdgcn_ballot_w64(right);
    const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const int below_r =
        (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mr >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mr, 0u));
    if (lane == 0) {
      wl[wid] = __builtin_popcountll(m);
      wr[wid] = __builtin_popcountll(mr);
    }
    __syncthreads();
    int before = 0, tot = 0, before_r = 0, tot_r = 0;
#pragma unroll
    for (int k = 0; k < kSegThreads / 64; ++k) {
      before += k < wid ? wl[k] : 0;
      tot += wl[k];
      before_r += k < wid ? wr[k] : 0;
      tot_r += wr[k];
    }
    __syncthreads();
    if (left || right) {
      const int dst = left ? (lb >= 0 ? lb + done_l + before + below : -1)
                           : (rbase >= 0 ? rbase + done_r + before_r + below_r : -1);
      if (dst >= 0) {
        const int64_t src = (int64_t)start + i;
        const int64_t sidx = implicit ? (int64_t)row : src;  // statistics: per row (implicit) or permuted
        a.perm_out[dst] = row;
        a.v1_out[dst] = a.v1p[sidx];
        if (a.v0p) a.v0_out[dst] = a.v0p[sidx];
        if (a.wp) a.w_out[dst] = a.wp[src];
      }
    }
    done_l += tot;
    done_r += tot_r;
  }
}

// ---------------------------------------------------------------------------
// Multi-tree forests keep the dense row records (hist5.hip codes, cheap to
// partition: one coalesced pass) and, before each level >= 1 histogram, gather
// the rows of the nodes that level BUILDS (the smaller sibling of each pair)
// into per-slot segments: perm / statistics / weight, so the segment
// histogram touches only those rows (the codes kernels scan every (row, tree)
// record and idle on the skipped ones: 54 ms vs ~37 ms per level at 1e8 x 20
// trees).  Pass 1 counts rows per slot; the host turns counts into segment
// starts; pass 2 scatters.  Within a wave the rows of one slot are ranked by
// peeling (one ballot per distinct slot in the wave), so the LDS atomics are
// one per (wave, slot), not one per row.  Segment order is block-arbitrary;
// the fixed-point histogram sums do not depend on it.
struct CompactArgs {
  const uint16_t* codes;  // [T][n]  weight << 8 | local node (0xFF = done)
  int64_t n;
  int T, A;
  const int* tfirst;      // [T] first active index of tree t (active order is tree-major)
  const int* build_slot;  // [A] histogram slot of the active node, -1 = not built
  const float* v0;        // [n] or null
  const float* v1;        // [n]
  int* cnt;               // pass 1: [S] row totals; pass 2: [S] write cursors (pre-set to segment starts)
  int* perm_out;
  float* v0_out;
  float* v1_out;
  uint8_t* w_out;
  uint64_t* rec_out;  // optional packed records (see CompactWArgs)
  float qs1;
};

template <bool SCATTER>
__global__ __launch_bounds__(256) void codes_compact_kernel(const CompactArgs a) {
  __shared__ int s_slot[256], s_cnt[256], s_base[256];
  const int t = blockIdx.y;
  const int tf = a.tfirst[t];
  const int nloc = (t + 1 < a.T ? a.tfirst[t + 1] : a.A) - tf;
  for (int i = threadIdx.x; i < 256; i += 256) {
    s_slot[i] = i < nloc ? a.build_slot[tf + i] : -1;
    s_cnt[i] = 0;
  }
  __syncthreads();
  const uint16_t* rec = a.codes + (int64_t)t * a.n;
  const int64_t per = ((a.n + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
  const int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = r0 + per < a.n ? r0 + per : a.n;
  const int lane = threadIdx.x & 63;
  constexpr int U = 8;  // code loads in flight per thread (one dependent load per trip was latency-bound)
  // sweep 1: per-slot counts of this block's range (wave-aggregated LDS atomics)
  for (int64_t rb = r0; rb < r1; rb += 256 * U) {
    uint32_t cu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + u * 256 + threadIdx.x;
      cu[u] = r < r1 ? (uint32_t)rec[r] : 0xFFu;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
    const uint32_t c = cu[u];
    const uint32_t loc = c & 0xFFu;
    // this kernel serves levels with many built nodes per tree (the wave-owned kernel covers <= 16):
    // plain per-lane LDS atomics; peeling one ballot round per distinct node in the wave cost up to 64 rounds
    if (loc != 0xFFu && s_slot[loc] >= 0) atomicAdd(&s_cnt[loc], 1);
    }
  }
  __syncthreads();
  if (!SCATTER) {
    for (int i = threadIdx.x; i < nloc; i += 256)
      if (s_cnt[i]) atomicAdd(&a.cnt[s_slot[i]], s_cnt[i]);
    return;
  }
  for (int i = threadIdx.x; i < nloc; i += 256) {
    s_base[i] = s_cnt[i] ? atomicAdd(&a.cnt[s_slot[i]], s_cnt[i]) : 0;
    s_cnt[i] = 0;
  }
  __syncthreads();
  // sweep 2: scatter (row, statistics, weight) to the slot segments
  for (int64_t rb = r0; rb < r1; rb += 256 * U) {
    uint32_t cu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + u * 256 + threadIdx.x;
      cu[u] = r < r1 ? (uint32_t)rec[r] : 0xFFu;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
    const int64_t r = rb + u * 256 + threadIdx.x;
    const uint32_t c = cu[u];
    const uint32_t loc = c & 0xFFu;
    const int pos = (loc != 0xFFu && s_slot[loc] >= 0) ? s_base[loc] + atomicAdd(&s_cnt[loc], 1) : -1;
    if (pos >= 0) {
      if (a.rec_out) {
        int q1 = (int)rintf(a.v1[r] * a.qs1);
        q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
        a.rec_out[pos] = (uint64_t)r | ((uint64_t)(c >> 8) << 31) | ((uint64_t)(uint32_t)(q1 + kPackQ) << 39);
      } else {
        a.perm_out[pos] = (int)r;
        a.v1_out[pos] = a.v1[r];
        if (a.v0) a.v0_out[pos] = a.v0[r];
        a.w_out[pos] = (uint8_t)(c >> 8);
      }
    }
    }
  }
}

// Node-id twin of codes_compact_kernel for forest levels deeper than the u16 codes reach (binary classification
// below level 8: up to 512 active nodes per tree): node ids int32 [T][n] (global active index, -1 = done) and
// the bootstrap weights uint8 [T][n] in, the level's packed item records (row | w << 31 | (q + 2^23) << 39) out,
// one segment per built slot -- so the deep levels take the same record histograms (seg_hist_lane10) as the
// shallow ones instead of the node-id kernel, which re-read every row once per LDS-sized slot group.
constexpr int kNodeCompactLoc = 1024;  // active nodes per tree
struct NodeCompactArgs {
  const int* node;
  const uint8_t* w;
  int64_t n;
  int T, A;
  const int* tfirst;
  const int* build_slot;  // [A]
  const float* v1;
  int* cnt;               // pass 1: [S] totals; pass 2: [S] write cursors (segment starts)
  uint64_t* rec_out;
  float qs1;
};

template <bool SCATTER>
__global__ __launch_bounds__(256) void node_compact_kernel(const NodeCompactArgs a) {
  __shared__ int s_slot[kNodeCompactLoc], s_cnt[kNodeCompactLoc], s_base[kNodeCompactLoc];
  const int t = blockIdx.y;
  const int tf = a.tfirst[t];
  const int nloc = (t + 1 < a.T ? a.tfirst[t + 1] : a.A) - tf;  // <= kNodeCompactLoc (host-checked)
  for (int i = threadIdx.x; i < kNodeCompactLoc; i += 256) {
    s_slot[i] = i < nloc ? a.build_slot[tf + i] : -1;
    s_cnt[i] = 0;
  }
  __syncthreads();
  const int* nd = a.node + (int64_t)t * a.n;
  const uint8_t* wt = a.w + (int64_t)t * a.n;
  const int64_t per = ((a.n + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
  const int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = r0 + per < a.n ? r0 + per : a.n;
  constexpr int U = 8;
  auto local = [&](int id) -> int {  // the row's local node when it is in a built slot, else -1
    const int l = id - tf;
    return (id >= 0 && l >= 0 && l < nloc && s_slot[l] >= 0) ? l : -1;
  };
  for (int64_t rb = r0; rb < r1; rb += 256 * U) {
    int id[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + u * 256 + threadIdx.x;
      id[u] = r < r1 ? nd[r] : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int l = local(id[u]);
      if (l >= 0) atomicAdd(&s_cnt[l], 1);
    }
  }
  __syncthreads();
  if (!SCATTER) {
    for (int i = threadIdx.x; i < nloc; i += 256)
      if (s_cnt[i]) atomicAdd(&a.cnt[s_slot[i]], s_cnt[i]);
    return;
  }
  for (int i = threadIdx.x; i < nloc; i += 256) {
    s_base[i] = s_cnt[i] ? atomicAdd(&a.cnt[s_slot[i]], s_cnt[i]) : 0;
    s_cnt[i] = 0;
  }
  __syncthreads();
  for (int64_t rb = r0; rb < r1; rb += 256 * U) {
    int id[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + u * 256 + threadIdx.x;
      id[u] = r < r1 ? nd[r] : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + u * 256 + threadIdx.x;
      const int l = local(id[u]);
      if (l < 0) continue;
      const int pos = s_base[l] + atomicAdd(&s_cnt[l], 1);
      int q1 = (int)rintf(a.v1[r] * a.qs1);
      q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
      a.rec_out[pos] = (uint64_t)r | ((uint64_t)wt[r] << 31) | ((uint64_t)(uint32_t)(q1 + kPackQ) << 39);
    }
  }
}

// Wave-owned variant for few built nodes per tree (KB <= 16, every RF level of
// depth <= 5 and the shallow levels of deeper forests).  rocprofv3 on the
// peeling kernel: ~80 wave instructions per 64 records and 71 % of wave time
// waiting (3.8 + 10.3 ms per level at 1e8 x 20 trees).  Here each wave owns a
// fixed contiguous row range and counts its records per built node in
// registers (pass 1 writes [T][waves][KB] counts, no atomics); a device scan
// turns the counts into per-wave output offsets; pass 2 re-reads the range and
// ranks the lanes' records per node with ballots.  Output order is the row
// order: stable and deterministic.
struct CompactWArgs {
  const uint16_t* codes;
  int64_t n;
  int T, A;
  const int* tfirst;
  const int* kmap;        // [A] index of the active node among its tree's built nodes, -1 = not built
  const float* v0;
  const float* v1;
  int64_t per_wave;       // rows per wave (multiple of 256)
  int Wv;                 // waves per tree
  int* wcnt;              // pass 1: [T][Wv][KB] counts
  const int* woff;        // pass 2: [T][Wv][KB] output offsets
  int* perm_out;
  float* v0_out;
  float* v1_out;
  uint8_t* w_out;
  // rec_out != null: one packed record per item instead of perm / v1 / w:
  // row (31 bits) | weight << 31 (8 bits) | (clamp(rint(v1 * qs1), +-2^23) + 2^23) << 39 (25 bits)
  uint64_t* rec_out;
  float qs1;
  const int64_t* kstart;  // pass 2, optional: [T][KB] segment start added to the per-wave offsets
};

// Pass 1: per-(tree, wave, built node) record counts.  rocprofv3 (PMC) on the first version, one compare-add per
// (row, node): VALU-issue bound (KB = 8: 6.2e8 VALU instructions in 2.5e6 cycles, 4 cycles each per SIMD).  Here
// the LDS table maps a local node to a one-hot increment of 8-bit fields packed four to a word, so a row costs
// one table read and NW = KB / 4 adds whatever KB is; the fields are flushed into the per-node counts before they
// can overflow (31 trips x 8 rows per lane <= 255).
template <int KB>
__global__ __launch_bounds__(256) void codes_count_w_kernel(const CompactWArgs a) {
  constexpr int NW = KB > 4 ? KB / 4 : 1;
  __shared__ uint32_t s_oh[256 * NW];
  // XCD-aware block -> (row chunk, tree) map: block b runs on XCD b % 8, and the T blocks of one row chunk are
  // consecutive slots of ONE XCD (the same map as the scatter pass, whose blocks share that XCD's L2 copy of
  // the chunk's labels: v1 is the same for every tree)
  const int nch = (a.Wv + 3) / 4;
  const int xcd = (int)(blockIdx.x & 7u), slot = (int)(blockIdx.x >> 3);
  const int qc = slot / a.T, t = slot - qc * a.T;
  const int chunk = qc * 8 + xcd;
  if (chunk >= nch) return;  // block-uniform
  const int tf = a.tfirst[t];
  const int nloc = (t + 1 < a.T ? a.tfirst[t + 1] : a.A) - tf;
  {
    const int kk = (threadIdx.x < nloc && threadIdx.x < 255) ? a.kmap[tf + threadIdx.x] : -1;
#pragma unroll
    for (int q = 0; q < NW; ++q)
      s_oh[threadIdx.x * NW + q] = (kk >= 0 && (kk >> 2) == q) ? 1u << (8 * (kk & 3)) : 0u;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = chunk * 4 + (threadIdx.x >> 6);
  if (w >= a.Wv) return;
  const int64_t r_begin = (int64_t)w * a.per_wave;
  const int64_t r_end = r_begin + a.per_wave < a.n ? r_begin + a.per_wave : a.n;
  const uint16_t* rec = a.codes + (int64_t)t * a.n;
  const int64_t cb = ((int64_t)t * a.Wv + w) * KB;
  int acc[KB];
  uint32_t pk[NW];
#pragma unroll
  for (int k = 0; k < KB; ++k) acc[k] = 0;
#pragma unroll
  for (int q = 0; q < NW; ++q) pk[q] = 0;
  auto flush = [&]() {
#pragma unroll
    for (int k = 0; k < KB; ++k) acc[k] += (int)((pk[k >> 2] >> (8 * (k & 3))) & 0xFFu);
#pragma unroll
    for (int q = 0; q < NW; ++q) pk[q] = 0;
  };
  // 2 x 4 codes per lane per trip, loaded up front as 8-byte vectors
  const bool vec = (a.n & 3) == 0 && (reinterpret_cast<uintptr_t>(a.codes) & 7u) == 0;
  constexpr int NG = 2;
  int trips = 0;
  for (int64_t rb = r_begin; rb < r_end; rb += 256 * NG) {
    uint32_t cc[NG][4];
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const int64_t r = rb + q * 256 + lane * 4;
      if (vec && r + 3 < r_end) {
        const uint2 c4 = *reinterpret_cast<const uint2*>(rec + r);
        cc[q][0] = c4.x & 0xFFFFu;
        cc[q][1] = c4.x >> 16;
        cc[q][2] = c4.y & 0xFFFFu;
        cc[q][3] = c4.y >> 16;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) cc[q][j] = r + j < r_end ? (uint32_t)rec[r + j] : 0xFFu;
      }
    }
#pragma unroll
    for (int q = 0; q < NG; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int u = 0; u < NW; ++u) pk[u] += s_oh[(cc[q][j] & 0xFFu) * NW + u];
    if (++trips == 31) {
      flush();
      trips = 0;
    }
  }
  flush();
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    int v = acc[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) a.wcnt[cb + k] = v;
  }
}

// Inclusive wave-wide prefix sum in six DPP adds: row_shr 1 / 2 / 4 / 8 scan each 16-lane row, then
// row_bcast:15 carries row 0's total into row 1 (and row 2's into row 3) and row_bcast:31 carries lane 31's
// (rows 0-1) into rows 2-3.  Lanes whose DPP source is out of range or whose row is masked add the old value 0.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
  return v;
}

// Pass 2 with lane-strided rows.  The first version gave each lane 4
// consecutive rows (ranked with 3 ballots per node), so the lanes' output
// positions were ~4 records apart and every 8-byte store instruction spread
// over ~16 partially written 128-byte lines (level-0 scatter: 14 GB in 5.4 ms
// = 2.7 TB/s; all levels 20.5 ms per headline step).  Here trip row j of lane
// l is rb + 64 j + l, and the lanes of one node get consecutive positions, so
// each store instruction writes one contiguous run per node.
//
// Ranking the lanes inside a node (RANK):
//  0  one ballot + mbcnt per node: ~6 VALU instructions per (row slot, node).  PMC: VALU-issue bound at KB = 8
//     (2.5e9 VALU instructions = the whole 3.8 ms of the level's scatter at 4 cycles per wave64 instruction).
//  1  one DPP prefix scan of one-hot 8-bit fields packed four nodes to a word (NW = KB / 4 scans of 6 adds) gives
//     each lane the count of same-node lanes below it; the node cursors live in lanes 0..KB-1 and are read with
//     ds_bpermute.  Cost independent of KB per word; output order is still the row order.
// A third method, per-wave LDS cursors bumped with a returning LDS atomic, measured the same headline step as both
// (131.4 vs 131.1-131.5 ms) and was dropped; so was giving each lane 4 consecutive rows per trip loaded as 8- and
// 16-byte vectors (scatter 9.8 vs 8.9 ms per step).
template <int KB, int RANK>
__global__ __launch_bounds__(256) void codes_scatter_w_kernel(const CompactWArgs a) {
  constexpr int NW = KB > 4 ? KB / 4 : 1;
  __shared__ int s_k[256];
  const int nch = (a.Wv + 3) / 4;
  const int xcd = (int)(blockIdx.x & 7u), slot = (int)(blockIdx.x >> 3);
  const int qc = slot / a.T, t = slot - qc * a.T;
  const int chunk = qc * 8 + xcd;
  if (chunk >= nch) return;  // block-uniform
  const int tf = a.tfirst[t];
  const int nloc = (t + 1 < a.T ? a.tfirst[t + 1] : a.A) - tf;
  s_k[threadIdx.x] = (threadIdx.x < nloc && threadIdx.x < 255) ? a.kmap[tf + threadIdx.x] : -1;
  const int lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  const int w = chunk * 4 + wib;
  const int64_t cb = ((int64_t)t * a.Wv + w) * KB;
  auto start = [&](int k) { return a.woff[cb + k] + (a.kstart ? (int)a.kstart[(int64_t)t * KB + k] : 0); };
  __syncthreads();
  if (w >= a.Wv) return;
  const int64_t r_begin = (int64_t)w * a.per_wave;
  const int64_t r_end = r_begin + a.per_wave < a.n ? r_begin + a.per_wave : a.n;
  const uint16_t* rec = a.codes + (int64_t)t * a.n;
  int acc[RANK == 0 ? KB : 1];
  int cur = 0;  // RANK 1: lane k < KB holds node k's cursor
  if (RANK == 0) {
#pragma unroll
    for (int k = 0; k < KB; ++k) acc[k] = start(k);
  } else {
    cur = lane < KB ? start(lane) : 0;
  }
  constexpr int NJ = 8;
  for (int64_t rb = r_begin; rb < r_end; rb += 64 * NJ) {
    uint32_t cc[NJ];
    float x1[NJ], x0[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int64_t r = rb + j * 64 + lane;
      const bool ok = r < r_end;
      cc[j] = ok ? (uint32_t)rec[r] : 0xFFu;
      x1[j] = ok ? a.v1[r] : 0.f;
      x0[j] = (ok && a.v0) ? a.v0[r] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int kk = s_k[cc[j] & 0xFFu];
      int pos = -1;
      if (RANK == 0) {
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const uint64_t m = __builtin_amdgcn_ballot_w64(kk == k);
          if (m == 0ull) continue;  // wave-uniform
          if (kk == k)
            pos = acc[k] + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          acc[k] += __builtin_popcountll(m);
        }
      } else {
        const int kc = kk < 0 ? 0 : kk;
        const uint32_t one = kk < 0 ? 0u : 1u << (8 * (kc & 3));
        uint32_t below = 0, tot_mine = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          const uint32_t x = (kc >> 2) == q ? one : 0u;
          const uint32_t inc = wave_incl_scan(x);
          if ((kc >> 2) == q) below = inc - x;
          // node totals = lane 63's inclusive fields; lane k < KB takes the field of node k
          const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
          if ((lane >> 2) == q) tot_mine = tot;
        }
        const int base = __builtin_amdgcn_ds_bpermute(kc << 2, cur);
        if (kk >= 0) pos = base + (int)((below >> (8 * (kc & 3))) & 0xFFu);
        cur += (int)((tot_mine >> (8 * (lane & 3))) & 0xFFu);
      }
      if (pos < 0) continue;
      const int64_t r = rb + j * 64 + lane;
      if (a.rec_out) {
        int q1 = (int)rintf(x1[j] * a.qs1);
        q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
        a.rec_out[pos] = (uint64_t)r | ((uint64_t)(cc[j] >> 8) << 31) | ((uint64_t)(uint32_t)(q1 + kPackQ) << 39);
      } else {
        a.perm_out[pos] = (int)r;
        a.v1_out[pos] = x1[j];
        if (a.v0) a.v0_out[pos] = x0[j];
        a.w_out[pos] = (uint8_t)(cc[j] >> 8);
      }
    }
  }
}

// RANK 2 (packed records only): queue first, rank dense.  PMC on RANK 1 put the scatter at 73-85 % VALU issue, and
// a wave instruction costs the same whatever number of its lanes is active -- but at the headline's levels 2-4
// only ~25 % of the (row, tree) slots belong to a built node: 3 of every 4 lanes of every scan, readlane,
// bpermute and record instruction worked for nothing.  Here the wave first queues its built slots in LDS in row
// order -- a lane reads 4 consecutive codes (one 8-byte load) and their labels (one 16-byte load), counts its
// built ones, and one DPP scan of those counts places them (row offset | weight << 16 | node << 24, and the
// label) -- and then drains the queue in DENSE groups of 64 entries that run the RANK 1 node ranking (RANK 0
// ballots for KB <= 2) and build + store the records.  A group ranks in queue order, so the records and their positions are exactly RANK 0 / 1's
// (row order inside each (tree, node, wave) run).  Leftovers (< 64) carry to the next trip; the wave's last group
// is partial.  A/B at the headline (profiles/r6/scatter_queue_ab.md).  LDS: 4 waves x 576 x 8 B = 18 KB per block.
// PF (rank 3): two register sets of codes / labels, each consumed and refilled two trips ahead, so a trip's loads
// are in flight while the previous trip queues and drains (PMC of the one-set loop: 56 % of wave cycles waiting,
// 14 % VALU busy; 8.2 -> 7.7 ms per headline step).
template <int KB, bool PF>
__global__ __launch_bounds__(256) void codes_scatter_q_kernel(const CompactWArgs a) {
  constexpr int NW = KB > 4 ? KB / 4 : 1;
  constexpr int NG = 2;                  // 256-row groups per trip (4 consecutive rows per lane)
  constexpr int QCAP = NG * 256 + 64;
  __shared__ int s_k[256];
  __shared__ uint32_t s_meta[4][QCAP];
  __shared__ float s_x1[4][QCAP];
  const int nch = (a.Wv + 3) / 4;
  const int xcd = (int)(blockIdx.x & 7u), slot = (int)(blockIdx.x >> 3);
  const int qc = slot / a.T, t = slot - qc * a.T;
  const int chunk = qc * 8 + xcd;
  if (chunk >= nch) return;  // block-uniform
  const int tf = a.tfirst[t];
  const int nloc = (t + 1 < a.T ? a.tfirst[t + 1] : a.A) - tf;
  s_k[threadIdx.x] = (threadIdx.x < nloc && threadIdx.x < 255) ? a.kmap[tf + threadIdx.x] : -1;
  const int lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  const int w = chunk * 4 + wib;
  const int64_t cb = ((int64_t)t * a.Wv + w) * KB;
  __syncthreads();
  if (w >= a.Wv) return;
  const int64_t r_begin = (int64_t)w * a.per_wave;
  const int64_t r_end = r_begin + a.per_wave < a.n ? r_begin + a.per_wave : a.n;
  const uint16_t* rec = a.codes + (int64_t)t * a.n;
  uint32_t* qm = s_meta[wib];
  float* qx = s_x1[wib];
  // RANK 1 cursors: lane k < KB holds node k's next output position
  int cur = lane < KB ? a.woff[cb + lane] + (a.kstart ? (int)a.kstart[(int64_t)t * KB + lane] : 0) : 0;
  // one dense group of queue entries [e0, e0 + cnt): rank among same-node entries in queue order, store
  auto drain = [&](int e0, int cnt) {
    const bool ok = lane < cnt;
    const uint32_t meta = ok ? qm[e0 + lane] : 0u;
    const float x1 = ok ? qx[e0 + lane] : 0.f;
    const int kk = ok ? (int)((meta >> 24) & 0xFu) : -1;
    int pos = -1;
    if (KB <= 2) {
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const uint64_t m = __builtin_amdgcn_ballot_w64(kk == k);
        const int base = __builtin_amdgcn_readlane(cur, k);
        if (kk == k)
          pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (lane == k) cur += __builtin_popcountll(m);
      }
    } else {
      const int kc = kk < 0 ? 0 : kk;
      const uint32_t one = kk < 0 ? 0u : 1u << (8 * (kc & 3));
      uint32_t below = 0, tot_mine = 0;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const uint32_t x = (kc >> 2) == q ? one : 0u;
        const uint32_t inc = wave_incl_scan(x);
        if ((kc >> 2) == q) below = inc - x;
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if ((lane >> 2) == q) tot_mine = tot;
      }
      const int base = __builtin_amdgcn_ds_bpermute(kc << 2, cur);
      if (kk >= 0) pos = base + (int)((below >> (8 * (kc & 3))) & 0xFFu);
      cur += (int)((tot_mine >> (8 * (lane & 3))) & 0xFFu);
    }
    if (pos >= 0) {
      int q1 = (int)rintf(x1 * a.qs1);
      q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
      const uint64_t r = (uint64_t)(r_begin + (int64_t)(meta & 0xFFFFu));
      a.rec_out[pos] = r | ((uint64_t)((meta >> 16) & 0xFFu) << 31) | ((uint64_t)(uint32_t)(q1 + kPackQ) << 39);
    }
  };
  const bool vec = (a.n & 3) == 0 && (reinterpret_cast<uintptr_t>(a.codes) & 7u) == 0 &&
                   (reinterpret_cast<uintptr_t>(a.v1) & 15u) == 0;
  int nq = 0;  // wave-uniform queue length
  // one trip = NG x 256 rows: 4 consecutive codes + labels per lane (8-byte / 16-byte loads)
  auto load = [&](int64_t rb, uint32_t (&cc)[NG][4], float (&xl)[NG][4]) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int64_t r = rb + g * 256 + lane * 4;
      if (vec && r + 3 < r_end) {
        const uint2 c4 = *reinterpret_cast<const uint2*>(rec + r);
        cc[g][0] = c4.x & 0xFFFFu;
        cc[g][1] = c4.x >> 16;
        cc[g][2] = c4.y & 0xFFFFu;
        cc[g][3] = c4.y >> 16;
        const float4 x4 = *reinterpret_cast<const float4*>(a.v1 + r);
        xl[g][0] = x4.x;
        xl[g][1] = x4.y;
        xl[g][2] = x4.z;
        xl[g][3] = x4.w;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          cc[g][u] = r + u < r_end ? (uint32_t)rec[r + u] : 0xFFu;
          xl[g][u] = r + u < r_end ? a.v1[r + u] : 0.f;
        }
      }
    }
  };
  auto trip = [&](int64_t rb, const uint32_t (&cc)[NG][4], const float (&xl)[NG][4]) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      int kk[4], cnt = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        kk[u] = s_k[cc[g][u] & 0xFFu];
        cnt += kk[u] >= 0 ? 1 : 0;
      }
      const uint32_t inc = wave_incl_scan((uint32_t)cnt);
      int e = nq + (int)(inc - (uint32_t)cnt);
      const uint32_t off = (uint32_t)(rb + g * 256 + lane * 4 - r_begin);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (kk[u] >= 0) {
          qm[e] = (off + u) | ((cc[g][u] >> 8) << 16) | ((uint32_t)kk[u] << 24);
          qx[e++] = xl[g][u];
        }
      nq += __builtin_amdgcn_readlane((int)inc, 63);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int e0 = 0;
    for (; e0 + 64 <= nq; e0 += 64) drain(e0, 64);
    // the leftover (< 64 entries) moves to the queue front for the next trip
    const int left = nq - e0;
    if (left > 0 && e0 > 0) {
      const uint32_t mv = lane < left ? qm[e0 + lane] : 0u;
      const float xv = lane < left ? qx[e0 + lane] : 0.f;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane < left) {
        qm[lane] = mv;
        qx[lane] = xv;
      }
    }
    nq = left;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  constexpr int64_t TRIP = 256 * NG;
  if (PF) {
    // two register sets, each consumed and then refilled two trips ahead (no register copy at the back-edge):
    // a trip's code / label loads are in flight while the previous trip queues and drains
    uint32_t ca[NG][4], cb2[NG][4];
    float xa[NG][4], xb[NG][4];
    load(r_begin, ca, xa);
    load(r_begin + TRIP, cb2, xb);
    for (int64_t rb = r_begin; rb < r_end; rb += 2 * TRIP) {
      trip(rb, ca, xa);
      load(rb + 2 * TRIP, ca, xa);
      if (rb + TRIP < r_end) trip(rb + TRIP, cb2, xb);  // wave-uniform
      load(rb + 3 * TRIP, cb2, xb);
    }
  } else {
    for (int64_t rb = r_begin; rb < r_end; rb += TRIP) {
      uint32_t cc[NG][4];
      float xl[NG][4];
      load(rb, cc, xl);
      trip(rb, cc, xl);
    }
  }
  if (nq > 0) drain(0, nq);
}

// Per (tree, built node): exclusive prefix of the per-wave counts [T][Wv][KB] in place and the node's total
// (one launch instead of the torch permute / cumsum / subtract / add / cast / permute chain per level).
__global__ __launch_bounds__(256) void wave_scan_kernel(int* __restrict__ wcnt, int Wv, int KB,
                                                        int64_t* __restrict__ tot) {
  const int t = blockIdx.x / KB, k = blockIdx.x - t * KB;
  int* base = wcnt + (int64_t)t * Wv * KB + k;
  const int per = (Wv + 255) / 256;
  const int w0 = threadIdx.x * per;
  int s = 0;
  for (int j = 0; j < per; ++j)
    if (w0 + j < Wv) s += base[(int64_t)(w0 + j) * KB];
  __shared__ int sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan
    const int v = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
    __syncthreads();
    sh[threadIdx.x] += v;
    __syncthreads();
  }
  int run = sh[threadIdx.x] - s;
  for (int j = 0; j < per; ++j) {
    if (w0 + j < Wv) {
      int* p = base + (int64_t)(w0 + j) * KB;
      const int c = *p;
      *p = run;
      run += c;
    }
  }
  if (threadIdx.x == 255) tot[blockIdx.x] = sh[255];
}

// [G][n] 8-feature bin words -> row-major [n][G] (one row's words contiguous),
// staged through LDS so both the reads and the writes are coalesced.
__global__ __launch_bounds__(256) void bins_row_major_kernel(const uint64_t* __restrict__ bins, int64_t n, int G,
                                                             int Gs, uint64_t* __restrict__ out) {
  extern __shared__ uint64_t tile[];  // [256][G] (odd G strides spread the banks)
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int rows = n - r0 < 256 ? (int)(n - r0) : 256;
  for (int g = 0; g < G; ++g)
    if (threadIdx.x < rows) tile[threadIdx.x * G + g] = bins[(int64_t)g * n + r0 + threadIdx.x];
  __syncthreads();
  // output rows are Gs >= G words (Gs = 16 at d <= 128: every row is one aligned 128-byte line, so a
  // gathered row costs one line instead of ~1.8 for 104-byte rows)
  uint64_t* o = out + r0 * Gs;
  for (int i = threadIdx.x; i < rows * Gs; i += 256) {
    const int r = i / Gs, g = i - r * Gs;
    o[i] = g < G ? tile[r * G + g] : 0ull;
  }
}

}  // namespace

namespace {
// Wide-bin (80 < B <= 256) twin of seg_hist_lane10_root_kernel for boosting (GBDT, one tree per round: every
// level-0 / level-1 histogram has one built node per tree): the quarter-wave lane4 histogram (64 features per
// block, XCD-paired feature blocks) fed by per-wave LDS rings of records compacted from the row codes instead
// of a codes_count_w + codes_scatter_w pass.  [4][BP][16] u64 planes (128 KB at 256 bins) + 16 x 128 ring
// entries (16 KB).  All four quarters of a wave add into the same cells: a block's rows x max weight must stay
// below 2^20.
template <int BP, int U>
__global__ __launch_bounds__(1024) void seg_hist_lane4_root_kernel(const SegHistArgs a, const uint8_t* __restrict__ bins8,
                                                                   int row_bytes, int nwork, int ny,
                                                                   const uint16_t* __restrict__ codes,
                                                                   const float* __restrict__ v1, float qs1,
                                                                   const int* __restrict__ sinfo, int slot0) {
  constexpr int TH = 1024, NW = TH / 64, NI = 4 * U, RING = 128;  // NI - 1 + 64 < RING
  constexpr int PLANE = BP * 16;
  static_assert(BP == 128 || BP == 256, "four planes of 128 or 256 bins");
  __shared__ __attribute__((aligned(16))) unsigned long long h[4 * PLANE];  // [4][BP][16]
  __shared__ __attribute__((aligned(16))) uint64_t ring[NW][RING];
  const int b = blockIdx.x, k = b >> 3;
  const int c = (k / ny) * 8 + (b & 7), fy = k - (k / ny) * ny;
  if (c >= nwork) return;
  const int r0 = a.work[3 * c], len = a.work[3 * c + 1], slot = a.work[3 * c + 2];
  const int tree = sinfo[2 * slot];
  const uint32_t node = (uint32_t)sinfo[2 * slot + 1];
  if (!CDNA_DCHECK(r0 >= 0 && len >= 0 && slot >= slot0 && tree >= 0 && node < 0xFFu && (int64_t)r0 + len <= a.n,
                   0x5E86u)) return;
  const int f0 = fy * 64;
  for (int i = threadIdx.x; i < 4 * PLANE; i += TH) h[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63, qt = lane >> 4, lq = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  int dw = (f0 >> 2) + lq;
  const int dmax = (row_bytes >> 2) - 1;
  dw = dw < dmax ? dw : dmax;
  const uint8_t* lbase = bins8 + 4 * dw;
  const uint32_t loff = (uint32_t)lq * 8u;
  const uint16_t* ct = codes + (int64_t)tree * a.n;
  uint64_t* rg = ring[wid];
  const int per = ((len + NW - 1) / NW + 63) & ~63;
  int64_t wr = (int64_t)r0 + (int64_t)wid * per;
  const int64_t wend = (int64_t)r0 + len < wr + per ? (int64_t)r0 + len : wr + per;
  uint32_t head = 0u, tail = 0u;
  uint32_t ncw = 0xFFu;
  float ny_ = 0.f;
  auto fetch = [&](int64_t r) {
    ncw = r < wend ? (uint32_t)ct[r] : 0xFFu;
    ny_ = r < wend ? v1[r] : 0.f;
  };
  fetch(wr + lane);
  for (;;) {
    while (tail - head < (uint32_t)NI && wr < wend) {
      const uint32_t cw = ncw;
      const float y = ny_;
      const int64_t r = wr + lane;
      wr += 64;
      fetch(wr + lane);
      const bool has = (cw & 0xFFu) == node && (cw >> 8) != 0u;
      const uint64_t m = __builtin_amdgcn_ballot_w64(has);
      if (has) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        int q1 = (int)rintf(y * qs1);
        q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
        rg[(tail + rank) & (RING - 1)] =
            (uint64_t)r | ((uint64_t)(cw >> 8) << 31) | ((uint64_t)(uint32_t)(q1 + kPackQ) << 39);
      }
      tail += (uint32_t)__builtin_popcountll(m);
    }
    const uint32_t avail = tail - head;
    if (avail == 0u) break;
    asm volatile("" ::: "memory");
    uint64_t rc[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t kk = (uint32_t)(4 * p + qt);
      rc[p] = kk < avail ? rg[(head + kk) & (RING - 1)] : 0ull;
    }
    head += avail < (uint32_t)NI ? avail : (uint32_t)NI;
    uint32_t x[U];
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t row = (uint32_t)rc[p] & 0x7FFFFFFFu;
      x[p] = *reinterpret_cast<const uint32_t*>(lbase + (uint64_t)row * (uint64_t)row_bytes);
    }
#pragma unroll
    for (int p = 0; p < U; ++p) {
      const uint32_t lo = (uint32_t)rc[p], hi = (uint32_t)(rc[p] >> 32);
      const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, 31) & 0xFFu;
      const unsigned long long add = ((unsigned long long)(w << (kPackShift - 32)) << 32) +
                                     (unsigned long long)w * (hi >> 7);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t off = (__builtin_amdgcn_ubfe(x[p], 8u * j, 8u) << 7) | loff;  // bin << 7 | l' << 3
        atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h) + off) + j * PLANE, add);
      }
    }
    asm volatile("" ::: "memory");
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < 4 * PLANE; cc += TH) {
    const int b_lo = cc & 7, l = (cc >> 3) & 15, j = (cc >> 7) & 3, b_hi = cc >> 9;
    const int bn = b_hi * 8 + b_lo;
    const int f = f0 + 4 * l + j;
    if (bn >= a.B || f >= a.d) continue;
    const unsigned long long v = h[j * PLANE + bn * 16 + l];
    if (!v) continue;
    const unsigned long long cnt = v >> kPackShift;
    const long long sum = (long long)(v & ((1ull << kPackShift) - 1ull)) - (long long)kPackQ * (long long)cnt;
    flush_packed(a, ((int64_t)(slot - slot0) * a.d + f) * a.B + bn, cnt, sum);
  }
}
}  // namespace

// Record histograms straight from the codes (seg_hist_lane10_root_kernel) for levels with <= 1 built node per
// tree: bins in the seg10 row layout, work [nwork][3] {row start, row count, slot}, sinfo [S][2] {tree, local
// node of the slot}; slot s's sums go to out slot s - slot0 (a slot-range slice).  Row counts per work item
// must keep count x max weight / 3 below 2^20 (the packed LDS cells).
// Wide-bin twin (seg_hist_lane4_root_kernel): bins_rm standard row-major rows of row_bytes, 80 < B <= 256.
CDNA_API int cdna_seg_hist_root_wide(const uint8_t* bins_rm, int64_t n, int d, int B, int row_bytes,
                                     const uint16_t* codes, const float* v1, float qs1, const int* work, int nwork,
                                     const int* sinfo, int slot0, unsigned long long* out, int cls3, hipStream_t st) {
  if (nwork <= 0) return 0;
  if (B <= 80 || B > 256 || row_bytes < ((d + 7) / 8) * 8) return (int)hipErrorInvalidValue;
  SegHistArgs a{nullptr, n, d, B, nullptr, nullptr, v1, nullptr, work, 1.f, qs1, out};
  a.cls_split = cls3 ? kClsSplit : 0;
  const int ny = (d + 63) / 64;
  const dim3 grid((unsigned)(((nwork + 7) / 8) * 8 * ny));
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(1024), 0, st, a, bins_rm, row_bytes, nwork, ny, codes, v1, qs1, sinfo, slot0);
  };
  if (B <= 128) launch(seg_hist_lane4_root_kernel<128, 16>);
  else launch(seg_hist_lane4_root_kernel<256, 16>);
  return (int)hipGetLastError();
}

// draw != 0 (level 0, every slot a tree's root): the bootstrap weights of tree sinfo[2 s] are drawn from Philox
// (seed, global row offset + r, rate) and written to codes as the level's row codes (see RootDraw).
CDNA_API int cdna_seg_hist_root(const uint8_t* bins_s10, int64_t n, int d, int B, const uint16_t* codes,
                                const float* v1, float qs1, const int* work, int nwork, const int* sinfo, int slot0,
                                unsigned long long* out, int draw, uint64_t seed, uint64_t offset, double rate,
                                int cls3, hipStream_t st) {
  if (nwork <= 0) return 0;
  if (d > 100 || B > 40 || B < 1) return (int)hipErrorInvalidValue;
  SegHistArgs a{nullptr, n, d, B, nullptr, nullptr, v1, nullptr, work, 1.f, qs1, out};
  a.cls_split = cls3 ? kClsSplit : 0;
  RootDraw dr{seed, offset, rate, cdna::poisson_cdf(draw ? rate : 1.0)};
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nwork), dim3(1024), 0, st, a, bins_s10, codes, v1, qs1, sinfo, slot0, dr);
  };
  if (draw) {
    if (B <= 32) launch(seg_hist_lane10_root_kernel<32, true>);
    else launch(seg_hist_lane10_root_kernel<40, true>);
  } else {
    if (B <= 32) launch(seg_hist_lane10_root_kernel<32, false>);
    else launch(seg_hist_lane10_root_kernel<40, false>);
  }
  return (int)hipGetLastError();
}

// Largest bootstrap weight the draws can produce at this rate (the saturated CDF table's length), -1 when the table
// does not saturate within kCdf entries (no static bound: the caller draws ahead with the weights' max).
CDNA_API int cdna_poisson_max_draw(double rate) {
  const cdna::PoissonCdf cdf = cdna::poisson_cdf(rate);
  if (cdf.T[cdna::kCdf - 1] != 0xFFFFFFFFu) return -1;
  int k = 0;
  while (k < cdna::kCdf && cdf.T[k] != 0xFFFFFFFFu) ++k;
  return k;
}

// mode bit0: packed (no v0; count | sum in one atomic); bit1: per-row weights wp present;
// bit4: `perm` holds packed 8-byte item records (row | w << 31 | (q1 + 2^23) << 39; flat kernel only).
// bit7 (with bit4 and bit2, B <= 256): lane-feature kernels (seg_hist_lane_kernel, B > 80: seg_hist_lane4_kernel).
// bit9 (packed): 3-class records, sums re-spaced to W1 + 2^32 W2 (SegHistArgs::cls_split).
// bit2: bins are row-major [n][G] words (seg_hist_flat_kernel when packed and all groups fit 128 KB of LDS,
// else seg_hist_rm_kernel); bit3: force seg_hist_rm_kernel.
// work: [nwork][3] {start, len, slot}; grid = nwork x ceil(d / 8).
CDNA_API int cdna_seg_hist(int mode, const uint64_t* bins, int64_t n, int d, int B, const int* perm, const float* v0p,
                           const float* v1p, const uint8_t* wp, const int* work, int nwork, float qs0, float qs1,
                           unsigned long long* out, int rm_stride,
                           hipStream_t st) {
  if (nwork <= 0) return 0;
  if (rm_stride != 0 && rm_stride < (d + 7) / 8) return (int)hipErrorInvalidValue;
  SegHistArgs a{bins, n, d, B, perm, v0p, v1p, wp, work, qs0, qs1, out};
  a.rs = rm_stride;
  a.cls_split = (mode & 512) ? kClsSplit : 0;
  const bool packed = (mode & 1) != 0, has_w = (mode & 2) != 0;
  if ((mode & 128) && (mode & 16) && (mode & 4) && packed) {
    // lane-feature kernel: 128 features per block (4 byte planes of BP >= B bins x 32 lanes, BP KB of LDS);
    // 80 < B <= 256: 64 features per block, a quarter-wave per item (seg_hist_lane4_kernel)
    if (B > 256) return (int)hipErrorInvalidValue;
    const int G = (d + 7) / 8;
    a.rec = reinterpret_cast<const uint64_t*>(perm);
    const int row_bytes = (rm_stride ? rm_stride : G) * 8;
    const uint8_t* b8 = reinterpret_cast<const uint8_t*>(bins);
    if (mode & 256) {
      // bins rows in the seg10 layout (binize v5 with Gs = -10): six items per wave
      if (d > 100 || B > 40 || row_bytes != 128) return (int)hipErrorInvalidValue;
      auto launch10 = [&](auto kern) { hipLaunchKernelGGL(kern, dim3((unsigned)nwork), dim3(1024), 0, st, a, b8); };
      if (B <= 32) launch10(seg_hist_lane10_kernel<32, 16>);
      else launch10(seg_hist_lane10_kernel<40, 16>);
      return (int)hipGetLastError();
    }
    if (B > 80) {
      const int ny = (d + 63) / 64;
      const dim3 grid2((unsigned)(((nwork + 7) / 8) * 8 * ny));
      auto launch2 = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid2, dim3(1024), 0, st, a, b8, row_bytes, nwork, ny);
      };
      if (B <= 128) launch2(seg_hist_lane4_kernel<128, 16>);
      else launch2(seg_hist_lane4_kernel<256, 16>);
      return (int)hipGetLastError();
    }
    const dim3 grid((unsigned)nwork, (unsigned)((d + 127) / 128));
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(512), 0, st, a, b8, row_bytes); };
    if (B <= 64) {
      auto launch8 = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(1024), 0, st, a, b8, row_bytes); };
      if (B <= 32) launch8(seg_hist_lane8_kernel<32>);
      else if (B <= 40) launch8(seg_hist_lane8_kernel<40>);
      else launch8(seg_hist_lane8_kernel<64>);
      return (int)hipGetLastError();
    }
    launch(seg_hist_lane_kernel<80>);  // 64 < B <= 80 (B <= 64: the quarter-wave lane8 kernel above)
    return (int)hipGetLastError();
  }
  if ((mode & 16) && !((mode & 4) && packed && (size_t)8 * B * 8 <= 128 * 1024 && !(mode & 8)))
    return (int)hipErrorInvalidValue;
  if ((mode & 4) && packed && (size_t)8 * B * 8 <= 128 * 1024 && !(mode & 8)) {
    // lanes over (row, group) pairs; the groups are split over as few blocks as fit 128 KB of LDS
    const int G = (d + 7) / 8;
    int ngb = (128 * 1024) / (8 * B * 8);
    if (ngb > G) ngb = G;
    const int nblk_g = (G + ngb - 1) / ngb;
    ngb = (G + nblk_g - 1) / nblk_g;  // balance
    const size_t lds = (size_t)ngb * 8 * B * 8;
    auto launch = [&](auto kern) {
      if (lds > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
      hipLaunchKernelGGL(kern, dim3((unsigned)nwork, (unsigned)nblk_g), dim3(1024), lds, st, a, bins, G, ngb);
    };
    if (mode & 16) {  // perm holds packed item records
      a.rec = reinterpret_cast<const uint64_t*>(perm);
      launch(seg_hist_flat_kernel<true, true>);
    } else if (has_w) {
      launch(seg_hist_flat_kernel<true>);
    } else {
      launch(seg_hist_flat_kernel<false>);
    }
    return (int)hipGetLastError();
  }
  if (mode & 4) {  // bins is row-major [n][G]
    const int G = (d + 7) / 8;
    const int cells_max = 16384 / (packed ? 1 : 2);  // 128 KB of u64 planes
    int ngb = cells_max / (8 * B);
    if (ngb > 8) ngb = 8;
    if (ngb < 1) return (int)hipErrorInvalidValue;
    const int nblk_g = (G + ngb - 1) / ngb;
    ngb = (G + nblk_g - 1) / nblk_g;  // balance the group blocks
    const size_t lds = (size_t)ngb * 8 * B * 8 * (packed ? 1 : 2);
    const dim3 grid((unsigned)nwork, (unsigned)nblk_g);
    auto launch = [&](auto kern) {
      if (lds > 64 * 1024)
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kern, grid, dim3(1024), lds, st, a, bins, G, ngb);
    };
    if (packed) {
      if (has_w) launch(seg_hist_rm_kernel<true, true>);
      else launch(seg_hist_rm_kernel<true, false>);
    } else {
      if (has_w) launch(seg_hist_rm_kernel<false, true>);
      else launch(seg_hist_rm_kernel<false, false>);
    }
    return (int)hipGetLastError();
  }
  const size_t lds = (size_t)8 * B * 8 * (packed ? 1 : 2);
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)nwork, (unsigned)((d + 7) / 8));
  if (packed) {
    if (has_w) hipLaunchKernelGGL((seg_hist_kernel<true, true>), grid, dim3(kSegThreads), lds, st, a);
    else hipLaunchKernelGGL((seg_hist_kernel<true, false>), grid, dim3(kSegThreads), lds, st, a);
  } else {
    if (has_w) hipLaunchKernelGGL((seg_hist_kernel<false, true>), grid, dim3(kSegThreads), lds, st, a);
    else hipLaunchKernelGGL((seg_hist_kernel<false, false>), grid, dim3(kSegThreads), lds, st, a);
  }
  return (int)hipGetLastError();
}

// pass 1 (left_cnt / right_cnt, outputs unused) or pass 2 (scatter) of the segment partition.
// implicit_n > 0: level-0 entry of multi-tree segment mode (see SegPartArgs).
CDNA_API int cdna_seg_partition(int pass, const uint64_t* bins, int64_t n, const int* perm, const float* v0p,
                                const float* v1p, const uint8_t* wp, const int* work, int nwork,
                                const int* split_feat, const int* split_bin, const int* cat_off,
                                const uint32_t* cat_mask, const int* left_base, const int* right_base, int* left_cnt,
                                int* perm_out, float* v0_out, float* v1_out, uint8_t* w_out, int64_t implicit_n,
                                int* right_cnt, hipStream_t st) {
  if (nwork <= 0) return 0;
  if (implicit_n > 0 && (perm != nullptr || wp == nullptr)) return (int)hipErrorInvalidValue;
  if (implicit_n <= 0 && perm == nullptr) return (int)hipErrorInvalidValue;
  SegPartArgs a{bins,     n,         perm,       v0p,        v1p,      wp,       work,   split_feat, split_bin,
                cat_off,  cat_mask,  left_base,  right_base, left_cnt, perm_out, v0_out, v1_out,     w_out,
                implicit_n, right_cnt};
  if (pass == 1) hipLaunchKernelGGL(seg_count_kernel, dim3((unsigned)nwork), dim3(kSegThreads), 0, st, a);
  else hipLaunchKernelGGL(seg_scatter_kernel, dim3((unsigned)nwork), dim3(kSegThreads), 0, st, a);
  return (int)hipGetLastError();
}

// Gather the rows of built nodes into slot segments (see CompactArgs).  pass 1: cnt = per-slot
// totals (must be zeroed); pass 2: cnt = per-slot write cursors initialised to the segment starts.
CDNA_API int cdna_codes_compact(int pass, const uint16_t* codes, int64_t n, int T, int A, const int* tfirst,
                                const int* build_slot, const float* v0, const float* v1, int* cnt, int* perm_out,
                                float* v0_out, float* v1_out, uint8_t* w_out, uint64_t* rec_out, float qs1,
                                hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  if (rec_out && (n >= (int64_t)1 << 31 || v0)) return (int)hipErrorInvalidValue;
  CompactArgs a{codes, n, T, A, tfirst, build_slot, v0, v1, cnt, perm_out, v0_out, v1_out, w_out, rec_out, qs1};
  int64_t nb = (n + 4095) / 4096;
  const int per_tree = (int)(nb < 512 ? nb : 512);
  const dim3 grid((unsigned)per_tree, (unsigned)T);
  if (pass == 1) hipLaunchKernelGGL(codes_compact_kernel<false>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(codes_compact_kernel<true>, grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// pass 1: counts into cnt [S]; pass 2: records from the cursors in cnt (segment starts).  Every tree holds at
// most kNodeCompactLoc active nodes (host-checked, else hipErrorInvalidValue).
CDNA_API int cdna_node_compact(int pass, const int* node, const uint8_t* w, int64_t n, int T, int A, const int* tfirst,
                               const int* build_slot, const float* v1, int* cnt, uint64_t* rec_out, float qs1,
                               int max_loc, hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  if (max_loc > kNodeCompactLoc || n >= (int64_t)1 << 31 || (pass == 2 && !rec_out)) return (int)hipErrorInvalidValue;
  NodeCompactArgs a{node, w, n, T, A, tfirst, build_slot, v1, cnt, rec_out, qs1};
  int64_t nb = (n + 4095) / 4096;
  const dim3 grid((unsigned)(nb < 512 ? nb : 512), (unsigned)T);
  if (pass == 1) hipLaunchKernelGGL(node_compact_kernel<false>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(node_compact_kernel<true>, grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// u16 row codes [T, n] (weight << 8 | local node, 255 = done) -> node ids int32 [T, n] (tfirst[t] + local, -1 for
// done or weight 0) and weights uint8 [T, n]: the switch of a deep forest to node ids at level 8, one pass (the
// torch formulation took seven passes over the [T, n] arrays, ~2.3 ms at 20 trees x 1e7 rows).  blockIdx.y = tree;
// four codes per thread (one 8-byte load) when n % 4 == 0.
__global__ __launch_bounds__(256) void codes_to_nodes_kernel(const uint16_t* __restrict__ codes, int64_t n,
                                                             const int* __restrict__ tfirst, int* __restrict__ node,
                                                             uint8_t* __restrict__ w, int vec4) {
  const int t = blockIdx.y;
  const int tf = tfirst[t];
  const uint16_t* c = codes + (int64_t)t * n;
  int* nd = node + (int64_t)t * n;
  uint8_t* wt = w + (int64_t)t * n;
  const int64_t stride = (int64_t)gridDim.x * 256;
  auto one = [&](unsigned v, int& id, unsigned& wv) {
    const unsigned loc = v & 0xFFu;
    wv = (v >> 8) & 0xFFu;
    id = (loc == 0xFFu || wv == 0u) ? -1 : tf + (int)loc;
  };
  if (vec4) {
    const int64_t n4 = n / 4;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n4; q += stride) {
      const uint2 v = reinterpret_cast<const uint2*>(c)[q];
      int i0, i1, i2, i3;
      unsigned w0, w1, w2, w3;
      one(v.x & 0xFFFFu, i0, w0);
      one(v.x >> 16, i1, w1);
      one(v.y & 0xFFFFu, i2, w2);
      one(v.y >> 16, i3, w3);
      reinterpret_cast<int4*>(nd)[q] = int4{i0, i1, i2, i3};
      reinterpret_cast<unsigned*>(wt)[q] = w0 | (w1 << 8) | (w2 << 16) | (w3 << 24);
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    int id;
    unsigned wv;
    one(c[i], id, wv);
    nd[i] = id;
    wt[i] = (uint8_t)wv;
  }
}

CDNA_API int cdna_codes_to_nodes(const uint16_t* codes, int64_t n, int T, const int* tfirst, int* node, uint8_t* w,
                                 hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  if (!codes || !tfirst || !node || !w || T > 65535) return (int)hipErrorInvalidValue;
  const int vec4 = (n % 4 == 0) && ((uintptr_t)codes % 8 == 0) && ((uintptr_t)node % 16 == 0) && ((uintptr_t)w % 4 == 0);
  const int64_t work = vec4 ? n / 4 : n;
  int64_t nb = (work + 255) / 256;
  const dim3 grid((unsigned)(nb < 1024 ? nb : 1024), (unsigned)T);
  hipLaunchKernelGGL(codes_to_nodes_kernel, grid, dim3(256), 0, st, codes, n, tfirst, node, w, vec4);
  return (int)hipGetLastError();
}

CDNA_API int cdna_bins_row_major(const uint64_t* bins, int64_t n, int G, int Gs, uint64_t* out, hipStream_t st) {
  if (n <= 0) return 0;
  if (G <= 0 || G > 32 || Gs < G) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bins_row_major_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), (size_t)256 * G * 8, st,
                     bins, n, G, Gs, out);
  return (int)hipGetLastError();
}

// Wave-owned compaction (KB = max built nodes per tree, <= 16).  pass 1 writes wcnt, pass 2 scatters
// from woff, ranking the lanes of a node with method `rank` (0 / 1: codes_scatter_w_kernel; 2: the queued
// codes_scatter_q_kernel, packed records and per_wave <= 65536 only; all three write identical records).  per_wave must be a multiple of 256; Wv = ceil(n / per_wave).
CDNA_API int cdna_codes_compact_w(int pass, int KB, const uint16_t* codes, int64_t n, int T, int A,
                                  const int* tfirst, const int* kmap, const float* v0, const float* v1,
                                  int64_t per_wave, int Wv, int* wcnt, const int* woff, int* perm_out, float* v0_out,
                                  float* v1_out, uint8_t* w_out, uint64_t* rec_out, float qs1,
                                  const int64_t* kstart, int rank, hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  if (per_wave % 256 != 0 || (int64_t)Wv * per_wave < n) return (int)hipErrorInvalidValue;
  if (rec_out && (n >= (int64_t)1 << 31 || v0)) return (int)hipErrorInvalidValue;
  CompactWArgs a{codes, n, T, A, tfirst, kmap, v0, v1, per_wave, Wv, wcnt, woff, perm_out, v0_out, v1_out, w_out,
                 rec_out, qs1, kstart};
  const int64_t nch = (Wv + 3) / 4;
  const dim3 grid((unsigned)(((nch + 7) / 8) * 8 * T));  // (chunk, tree) pairs, XCD-aware order (kernel)
  if (rank < 0 || rank > 3) return (int)hipErrorInvalidValue;
  // rank 2 / 3 (queued; 3: loads one trip ahead): packed records only, row offsets inside a wave's range in 16 bits
  if (pass == 2 && rank >= 2 && (!rec_out || per_wave > 65536)) return (int)hipErrorInvalidValue;
  auto go = [&](auto k1, auto k2r0, auto k2r1, auto k2q, auto k2qp) {
    if (pass == 1) hipLaunchKernelGGL(k1, grid, dim3(256), 0, st, a);
    else if (rank == 0) hipLaunchKernelGGL(k2r0, grid, dim3(256), 0, st, a);
    else if (rank == 1) hipLaunchKernelGGL(k2r1, grid, dim3(256), 0, st, a);
    else if (rank == 2) hipLaunchKernelGGL(k2q, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k2qp, grid, dim3(256), 0, st, a);
  };
#define CDNA_CW(K) go(codes_count_w_kernel<K>, codes_scatter_w_kernel<K, 0>, codes_scatter_w_kernel<K, 1>, \
                      codes_scatter_q_kernel<K, false>, codes_scatter_q_kernel<K, true>)
  switch (KB) {
    case 1: CDNA_CW(1); break;
    case 2: CDNA_CW(2); break;
    case 4: CDNA_CW(4); break;
    case 8: CDNA_CW(8); break;
    case 16: CDNA_CW(16); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef CDNA_CW
  return (int)hipGetLastError();
}

// In place: wcnt [T][Wv][KB] -> exclusive per-(tree, node) prefix over waves; tot [T][KB] = node totals.
CDNA_API int cdna_wave_scan(int* wcnt, int T, int Wv, int KB, int64_t* tot, hipStream_t st) {
  if (T <= 0 || Wv <= 0 || KB <= 0) return 0;
  hipLaunchKernelGGL(wave_scan_kernel, dim3((unsigned)(T * KB)), dim3(256), 0, st, wcnt, Wv, KB, tot);
  return (int)hipGetLastError();
}

CDNA_DEBUG_EXPORT(seg)
