// K5 hist_build, v4 — exact fixed-point split statistics on INTEGER LDS atomics.
//
// Measured on MI355X (bench/lds_atomic_bench.hip, 1024 x 512 threads, random
// addresses over 40..16384 words):
//     ds_add_f32   0.33 lane-ops / clk / CU
//     ds_add_u32   3.9 - 4.1            (12x)
//     ds_add_u64   3.7 - 3.9            (same words as u32, 64-bit payload)
// Every float-atomic histogram variant (v1/v2/v3) sat at the f32 ceiling, so v4
// accumulates integers:
//   * counts (bootstrap / bag weights are small integers) -> ds_add_u32, exact;
//   * real-valued moments v -> llrint(v * 2^s) in int64 -> ds_add_u64 (two's
//     complement wrap makes signed sums work), with the power-of-two scale s
//     chosen on the host so |sum| < 2^62 over ALL rows (no overflow possible);
//   * per-block partials flush to an int64 global buffer with 64-bit atomics.
// The sums are exact sums of the quantised values, so histograms are
// bit-reproducible regardless of block scheduling or atomic order — a property
// float atomics never had.  Quantisation step = 2^-s ~ max|v| * 2^-27 at
// n = 1e8 (finer than a float32 ulp of max|v|).
//
// Lane mapping, block decode and LDS slot/mask staging follow hist2.hip (v2):
// one block = (8-feature group g, slot group, row chunk); lanes own rows and
// loop over the 8 features of their bins word.  MAP = 1 selects the v3 mapping
// (lane = 8 * row + feature) for A/B measurement.
#include "common.h"

namespace {

struct Hist4Args {
  const uint64_t* bins;
  int64_t n;
  int d, T;
  const int* node;
  const uint8_t* weight;
  const float* v0;
  const float* v1;
  const int* label;
  int C;
  const int* build_slot;
  const uint32_t* feat_mask;
  int mask_words, S, B, SB, K;
  const int* grp;  // [ngroups][5] = s0, t0, t1, id0, id1
  int ngroups, nchunk;
  int64_t rows_per_chunk;
  int id_span_max;
  float qs0, qs1;      // fixed-point scales (powers of two) for v0, v1
  int n64, n32;        // planes held as 64-bit / 32-bit integers in LDS
  unsigned long long* out;  // [S][d][B][K] int64
};

constexpr int kThreads = 512;

__device__ __forceinline__ void lds_add64(unsigned long long* p, long long v) {
  atomicAdd(p, (unsigned long long)v);
}

// MODE 0: moments. V0 = false: plane k0 = sum w (u32), k1 = sum w*q(v1) (u64).
//                  V0 = true : k0 = sum w*q(v0) (u64), k1 = sum w*q(v1) (u64).
// MODE 1: class counts, plane c = sum w over rows with label c (u32).
template <int MODE, bool V0, int MAP>
__global__ __launch_bounds__(kThreads) void hist4_kernel(const Hist4Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  unsigned long long* h64 = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* h32 = reinterpret_cast<uint32_t*>(h64 + (size_t)a.n64 * plane);
  const int hwords = a.n32 * plane;  // 32-bit words of h32
  int* lslot = reinterpret_cast<int*>(h32 + ((hwords + 3) & ~3));
  uint8_t* lmask = reinterpret_cast<uint8_t*>(lslot + a.id_span_max);

  const uint32_t w = cdna::xcd_remap(blockIdx.x, gridDim.x);
  const int g = (int)(w % G);
  const int grp = (int)((w / G) % a.ngroups);
  const int chunk = (int)(w / ((uint32_t)G * a.ngroups));
  const int s0 = a.grp[grp * 5 + 0], t0 = a.grp[grp * 5 + 1], t1 = a.grp[grp * 5 + 2];
  const int id0 = a.grp[grp * 5 + 3], id1 = a.grp[grp * 5 + 4];
  const int span = id1 - id0;
  const bool lds_slot = span <= a.id_span_max;
  const int fbase = g * 8;

  for (int i = threadIdx.x; i < a.n64 * plane; i += kThreads) h64[i] = 0ull;
  for (int i = threadIdx.x; i < hwords; i += kThreads) h32[i] = 0u;
  if (lds_slot)
    for (int i = threadIdx.x; i < span; i += kThreads) lslot[i] = a.build_slot[id0 + i];
  for (int i = threadIdx.x; i < a.SB; i += kThreads) {
    uint32_t m = 0xFFu;
    const int slot = s0 + i;
    if (a.feat_mask != nullptr && slot < a.S)
      m = (a.feat_mask[(int64_t)slot * a.mask_words + (fbase >> 5)] >> (fbase & 31)) & 0xFFu;
    const int valid = a.d - fbase;
    if (valid < 8) m &= (1u << (valid > 0 ? valid : 0)) - 1u;
    lmask[i] = (uint8_t)m;
  }
  __syncthreads();

  const int64_t rb = (int64_t)chunk * a.rows_per_chunk;
  int64_t re = rb + a.rows_per_chunk;
  if (re > a.n) re = a.n;
  const int64_t n = a.n;
  const uint8_t* bins8 = reinterpret_cast<const uint8_t*>(a.bins);
  const int jl = MAP == 1 ? (int)(threadIdx.x & 7) : 0;
  const int64_t rstep = MAP == 1 ? kThreads / 8 : kThreads;
  for (int64_t r = rb + (MAP == 1 ? (threadIdx.x >> 3) : threadIdx.x); r < re; r += rstep) {
    uint64_t b8;
    if (MAP == 1) b8 = bins8[((int64_t)g * n + r) * 8 + jl];
    else b8 = a.bins[(int64_t)g * n + r];
    long long q0 = 1, q1 = 0;
    int c = 0;
    if (MODE == 0) {
      if (V0) q0 = llrintf(a.v0[r] * a.qs0);
      q1 = llrintf(a.v1[r] * a.qs1);
    } else {
      c = a.label[r];
      if (c < 0 || c >= a.C) continue;
    }
    for (int t = t0; t <= t1; t += 4) {
      int ids[4];
      int wt[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int tt = t + k;
        const bool ok = tt <= t1;
        ids[k] = ok ? a.node[(int64_t)tt * n + r] : -1;
        wt[k] = (ok && a.weight) ? (int)a.weight[(int64_t)tt * n + r] : 1;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int id = ids[k];
        if (id < id0 || id >= id1 || wt[k] == 0) continue;
        const int sl = lds_slot ? lslot[id - id0] : a.build_slot[id];
        const int ls = sl - s0;
        if (ls < 0 || ls >= a.SB) continue;
        uint32_t m = lmask[ls];
        const int off = (ls * 8) * a.B;
        const long long y1 = (long long)wt[k] * q1;
        const long long y0 = V0 ? (long long)wt[k] * q0 : 0;
        if (MAP == 1) {
          if (!((m >> jl) & 1u)) continue;
          m = 1u;  // single feature, bin already in the low byte
        }
#pragma unroll
        for (int j = 0; j < (MAP == 1 ? 1 : 8); ++j) {
          if ((m >> j) & 1u) {
            const int idx = off + (MAP == 1 ? jl : j) * a.B + (int)((b8 >> (8 * j)) & 0xFFu);
            if (MODE == 0) {
              if (V0) {
                lds_add64(h64 + idx, y0);
                lds_add64(h64 + plane + idx, y1);
              } else {
                atomicAdd(h32 + idx, (uint32_t)wt[k]);
                lds_add64(h64 + idx, y1);
              }
            } else {
              atomicAdd(h32 + c * plane + idx, (uint32_t)wt[k]);
            }
          }
        }
      }
    }
  }
  __syncthreads();
  // flush: entry e of plane p -> out[slot][f][bin][k]
  const int total = (a.n64 + a.n32) * plane;
  for (int i = threadIdx.x; i < total; i += kThreads) {
    const bool is64 = i < a.n64 * plane;
    const int p = is64 ? i / plane : (i - a.n64 * plane) / plane;
    const int rem = i - (is64 ? p : a.n64 + p) * plane;
    long long v;
    int k;
    if (is64) {
      v = (long long)h64[i];
      k = (MODE == 0 && !V0) ? 1 : p;
    } else {
      v = (long long)h32[i - a.n64 * plane];
      k = p;
    }
    if (v == 0) continue;
    const int ls = rem / (8 * a.B);
    const int jj = (rem / a.B) & 7;
    const int bn = rem % a.B;
    const int f = fbase + jj;
    const int slot = s0 + ls;
    if (f < a.d && slot < a.S)
      atomicAdd(&a.out[(((int64_t)slot * a.d + f) * a.B + bn) * a.K + k], (unsigned long long)v);
  }
}

// ---------------------------------------------------------------------------
// MAP 2: rotated features + software-pipelined row loads.
// rocprofv3 on MAP 0 (1e8 rows, 20 trees): SQ_LDS_BANK_CONFLICT ~ 55 % of
// SQ_LDS_IDX_ACTIVE and SQ_WAIT_ANY ~ 62 % of SQ_WAVE_CYCLES.  Two causes:
//   * every lane of an instruction updates the SAME feature, so 64 rows land
//     on ~40 bins: same-word collisions serialise the atomic.  Here lane l
//     visits feature (j + l) & 7 at step j, so one instruction spreads over
//     8 features x B bins;
//   * each row's loads (bins word, v1, node id + weight per tree) are waited
//     on right before use.  Here the next row's loads are issued before the
//     current row's atomics, hiding HBM/L2 latency behind LDS work.
// ---------------------------------------------------------------------------
template <int MODE, bool V0>
__global__ __launch_bounds__(kThreads) void hist4r_kernel(const Hist4Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  unsigned long long* h64 = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* h32 = reinterpret_cast<uint32_t*>(h64 + (size_t)a.n64 * plane);
  const int hwords = a.n32 * plane;
  int* lslot = reinterpret_cast<int*>(h32 + ((hwords + 3) & ~3));
  uint8_t* lmask = reinterpret_cast<uint8_t*>(lslot + a.id_span_max);

  const uint32_t w = cdna::xcd_remap(blockIdx.x, gridDim.x);
  const int g = (int)(w % G);
  const int grp = (int)((w / G) % a.ngroups);
  const int chunk = (int)(w / ((uint32_t)G * a.ngroups));
  const int s0 = a.grp[grp * 5 + 0], t0 = a.grp[grp * 5 + 1], t1 = a.grp[grp * 5 + 2];
  const int id0 = a.grp[grp * 5 + 3], id1 = a.grp[grp * 5 + 4];
  const int span = id1 - id0;
  const bool lds_slot = span <= a.id_span_max;
  const int fbase = g * 8;
  const int rot = threadIdx.x & 7;

  for (int i = threadIdx.x; i < a.n64 * plane; i += kThreads) h64[i] = 0ull;
  for (int i = threadIdx.x; i < hwords; i += kThreads) h32[i] = 0u;
  if (lds_slot)
    for (int i = threadIdx.x; i < span; i += kThreads) lslot[i] = a.build_slot[id0 + i];
  for (int i = threadIdx.x; i < a.SB; i += kThreads) {
    uint32_t m = 0xFFu;
    const int slot = s0 + i;
    if (a.feat_mask != nullptr && slot < a.S)
      m = (a.feat_mask[(int64_t)slot * a.mask_words + (fbase >> 5)] >> (fbase & 31)) & 0xFFu;
    const int valid = a.d - fbase;
    if (valid < 8) m &= (1u << (valid > 0 ? valid : 0)) - 1u;
    lmask[i] = (uint8_t)m;
  }
  __syncthreads();

  const int64_t rb = (int64_t)chunk * a.rows_per_chunk;
  int64_t re = rb + a.rows_per_chunk;
  if (re > a.n) re = a.n;
  const int64_t n = a.n;
  const int nt_head = t1 - t0 + 1 < 4 ? t1 - t0 + 1 : 4;  // trees whose loads are pipelined

  // row r's inputs, loaded one iteration ahead
  uint64_t b8 = 0;
  float x0 = 1.f, x1 = 0.f;
  int lab = 0;
  int ids[4] = {-1, -1, -1, -1};
  int wt[4] = {0, 0, 0, 0};
  auto load_row = [&](int64_t rr, uint64_t& ob8, float& ox0, float& ox1, int& olab, int* oids, int* owt) {
    ob8 = a.bins[(int64_t)g * n + rr];
    if (MODE == 0) {
      if (V0) ox0 = a.v0[rr];
      ox1 = a.v1[rr];
    } else {
      olab = a.label[rr];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = k < nt_head;
      oids[k] = ok ? a.node[(int64_t)(t0 + k) * n + rr] : -1;
      owt[k] = (ok && a.weight) ? (int)a.weight[(int64_t)(t0 + k) * n + rr] : 1;
    }
  };
  int64_t r = rb + threadIdx.x;
  if (r < re) load_row(r, b8, x0, x1, lab, ids, wt);

  for (; r < re; r += kThreads) {
    // issue the next row's loads first
    uint64_t nb8 = 0;
    float nx0 = 1.f, nx1 = 0.f;
    int nlab = 0;
    int nids[4] = {-1, -1, -1, -1};
    int nwt[4] = {0, 0, 0, 0};
    const int64_t rn = r + kThreads;
    if (rn < re) load_row(rn, nb8, nx0, nx1, nlab, nids, nwt);

    long long q0 = 1, q1 = 0;
    bool row_ok = true;
    if (MODE == 0) {
      if (V0) q0 = llrintf(x0 * a.qs0);
      q1 = llrintf(x1 * a.qs1);
    } else {
      row_ok = lab >= 0 && lab < a.C;
    }
    if (row_ok) {
      for (int t = t0; t <= t1; t += 4) {
        int cid[4], cwt[4];
        if (t == t0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) { cid[k] = ids[k]; cwt[k] = wt[k]; }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int tt = t + k;
            const bool ok = tt <= t1;
            cid[k] = ok ? a.node[(int64_t)tt * n + r] : -1;
            cwt[k] = (ok && a.weight) ? (int)a.weight[(int64_t)tt * n + r] : 1;
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int id = cid[k];
          if (id < id0 || id >= id1 || cwt[k] == 0) continue;
          const int sl = lds_slot ? lslot[id - id0] : a.build_slot[id];
          const int ls = sl - s0;
          if (ls < 0 || ls >= a.SB) continue;
          const uint32_t m = lmask[ls];
          const int off = (ls * 8) * a.B;
          const long long y1 = (long long)cwt[k] * q1;
          const long long y0 = V0 ? (long long)cwt[k] * q0 : 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int jj = (j + rot) & 7;
            if ((m >> jj) & 1u) {
              const int idx = off + jj * a.B + (int)((b8 >> (8 * jj)) & 0xFFu);
              if (MODE == 0) {
                if (V0) {
                  lds_add64(h64 + idx, y0);
                  lds_add64(h64 + plane + idx, y1);
                } else {
                  atomicAdd(h32 + idx, (uint32_t)cwt[k]);
                  lds_add64(h64 + idx, y1);
                }
              } else {
                atomicAdd(h32 + lab * plane + idx, (uint32_t)cwt[k]);
              }
            }
          }
        }
      }
    }
    b8 = nb8;
    x0 = nx0;
    x1 = nx1;
    lab = nlab;
#pragma unroll
    for (int k = 0; k < 4; ++k) { ids[k] = nids[k]; wt[k] = nwt[k]; }
  }
  __syncthreads();
  const int total = (a.n64 + a.n32) * plane;
  for (int i = threadIdx.x; i < total; i += kThreads) {
    const bool is64 = i < a.n64 * plane;
    const int p = is64 ? i / plane : (i - a.n64 * plane) / plane;
    const int rem = i - (is64 ? p : a.n64 + p) * plane;
    long long v;
    int k;
    if (is64) {
      v = (long long)h64[i];
      k = (MODE == 0 && !V0) ? 1 : p;
    } else {
      v = (long long)h32[i - a.n64 * plane];
      k = p;
    }
    if (v == 0) continue;
    const int ls = rem / (8 * a.B);
    const int jj = (rem / a.B) & 7;
    const int bn = rem % a.B;
    const int f = fbase + jj;
    const int slot = s0 + ls;
    if (f < a.d && slot < a.S)
      atomicAdd(&a.out[(((int64_t)slot * a.d + f) * a.B + bn) * a.K + k], (unsigned long long)v);
  }
}

// ---------------------------------------------------------------------------
// FAST (hist4f): the rotated + pipelined kernel with the per-update VALU work
// stripped down.  rocprofv3 on MAP 0: ~30 VALU instructions per (row-wave,
// tree, feature) update — 64-bit variable shifts of the bins word, index
// arithmetic, 64-bit value math and divergent mask tests inside the 8-feature
// loop — and halving the LDS atomics (packed kernel) did NOT speed it up, so
// the loop is issue-bound, not LDS-bound.  Here, per THREAD: the rotated
// feature order, byte selectors and per-feature LDS offsets are constants; per
// ROW: the 8 bin byte-offsets are extracted once (bfe on 32-bit halves) and
// the moment is quantised in 32 bits (the host caps |q| < 2^30); per TREE: the
// 64-bit contribution and the rotated feature mask; per FEATURE: one add, one
// mad and the two atomics (no mask test at all when MASKED = false).
// ---------------------------------------------------------------------------
template <int MODE, bool MASKED>
__global__ __launch_bounds__(kThreads) void hist4f_kernel(const Hist4Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  unsigned long long* h64 = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* h32 = reinterpret_cast<uint32_t*>(h64 + (size_t)a.n64 * plane);
  const int hwords = a.n32 * plane;
  int* lslot = reinterpret_cast<int*>(h32 + ((hwords + 3) & ~3));
  uint8_t* lmask = reinterpret_cast<uint8_t*>(lslot + a.id_span_max);

  const uint32_t w = cdna::xcd_remap(blockIdx.x, gridDim.x);
  const int g = (int)(w % G);
  const int grp = (int)((w / G) % a.ngroups);
  const int chunk = (int)(w / ((uint32_t)G * a.ngroups));
  const int s0 = a.grp[grp * 5 + 0], t0 = a.grp[grp * 5 + 1], t1 = a.grp[grp * 5 + 2];
  const int id0 = a.grp[grp * 5 + 3], id1 = a.grp[grp * 5 + 4];
  const int span = id1 - id0;
  const int fbase = g * 8;
  const int rot = threadIdx.x & 7;

  for (int i = threadIdx.x; i < a.n64 * plane; i += kThreads) h64[i] = 0ull;
  for (int i = threadIdx.x; i < hwords; i += kThreads) h32[i] = 0u;
  for (int i = threadIdx.x; i < span; i += kThreads) lslot[i] = a.build_slot[id0 + i];
  for (int i = threadIdx.x; i < a.SB; i += kThreads) {
    uint32_t m = 0xFFu;
    const int slot = s0 + i;
    if (a.feat_mask != nullptr && slot < a.S)
      m = (a.feat_mask[(int64_t)slot * a.mask_words + (fbase >> 5)] >> (fbase & 31)) & 0xFFu;
    const int valid = a.d - fbase;
    if (valid < 8) m &= (1u << (valid > 0 ? valid : 0)) - 1u;
    lmask[i] = (uint8_t)m;
  }
  // per-thread constants of the rotated feature order
  int fsel[8], fsh[8], foff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int jj = (j + rot) & 7;
    fsel[j] = jj >> 2;              // which 32-bit half of the bins word
    fsh[j] = (jj & 3) * 8;          // byte position inside it
    foff[j] = jj * a.B;             // feature row inside the slot's [8][B] block
  }
  __syncthreads();

  const int64_t rb = (int64_t)chunk * a.rows_per_chunk;
  int64_t re = rb + a.rows_per_chunk;
  if (re > a.n) re = a.n;
  const int64_t n = a.n;
  const int nt_head = t1 - t0 + 1 < 4 ? t1 - t0 + 1 : 4;
  const int slot_cells = 8 * a.B;

  uint64_t b8 = 0;
  float x1 = 0.f;
  int lab = 0;
  int ids[4] = {-1, -1, -1, -1};
  int wt[4] = {0, 0, 0, 0};
  auto load_row = [&](int64_t rr, uint64_t& ob8, float& ox1, int& olab, int* oids, int* owt) {
    ob8 = a.bins[(int64_t)g * n + rr];
    if (MODE == 0) ox1 = a.v1[rr];
    else olab = a.label[rr];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = k < nt_head;
      oids[k] = ok ? a.node[(int64_t)(t0 + k) * n + rr] : -1;
      owt[k] = (ok && a.weight) ? (int)a.weight[(int64_t)(t0 + k) * n + rr] : 1;
    }
  };
  int64_t r = rb + threadIdx.x;
  if (r < re) load_row(r, b8, x1, lab, ids, wt);

  for (; r < re; r += kThreads) {
    uint64_t nb8 = 0;
    float nx1 = 0.f;
    int nlab = 0;
    int nids[4] = {-1, -1, -1, -1};
    int nwt[4] = {0, 0, 0, 0};
    const int64_t rn = r + kThreads;
    if (rn < re) load_row(rn, nb8, nx1, nlab, nids, nwt);

    // per-row: the 8 rotated cell offsets (in cells) and the quantised moment
    const uint32_t lo = (uint32_t)b8, hi = (uint32_t)(b8 >> 32);
    int cell[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      cell[j] = foff[j] + (int)__builtin_amdgcn_ubfe(fsel[j] ? hi : lo, (uint32_t)fsh[j], 8u);
    int q = 0;
    bool row_ok = true;
    if (MODE == 0) q = (int)rintf(x1 * a.qs1);
    else row_ok = lab >= 0 && lab < a.C;
    const uint32_t cbase_lab = MODE == 1 ? (uint32_t)(lab * plane) : 0u;

    if (row_ok) {
      for (int t = t0; t <= t1; t += 4) {
        int cid[4], cwt[4];
        if (t == t0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) { cid[k] = ids[k]; cwt[k] = wt[k]; }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int tt = t + k;
            const bool ok = tt <= t1;
            cid[k] = ok ? a.node[(int64_t)tt * n + r] : -1;
            cwt[k] = (ok && a.weight) ? (int)a.weight[(int64_t)tt * n + r] : 1;
          }
        }
        // all 4 slot-table reads first: one LDS wait instead of one per tree
        // (the wait would otherwise also drain the previous tree's atomics)
        int lsk[4];
        uint32_t mk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool ok = cid[k] >= id0 && cid[k] < id1 && cwt[k] != 0;
          lsk[k] = ok ? lslot[cid[k] - id0] - s0 : -1;
          if (MASKED) mk[k] = (ok && lsk[k] >= 0 && lsk[k] < a.SB) ? lmask[lsk[k]] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int ls = lsk[k];
          if (ls < 0 || ls >= a.SB) continue;
          const uint32_t base = (uint32_t)(ls * slot_cells) + cbase_lab;
          uint32_t mrot = 0xFFu;
          if (MASKED) mrot = ((mk[k] >> rot) | (mk[k] << (8 - rot))) & 0xFFu;
          const uint32_t wv = (uint32_t)cwt[k];
          const long long y1 = (long long)cwt[k] * (long long)q;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (MASKED && !((mrot >> j) & 1u)) continue;
            const uint32_t c = base + (uint32_t)cell[j];
            atomicAdd(h32 + c, wv);
            if (MODE == 0) atomicAdd(h64 + c, (unsigned long long)y1);
          }
        }
      }
    }
    b8 = nb8;
    x1 = nx1;
    lab = nlab;
#pragma unroll
    for (int k = 0; k < 4; ++k) { ids[k] = nids[k]; wt[k] = nwt[k]; }
  }
  __syncthreads();
  const int total = (a.n64 + a.n32) * plane;
  for (int i = threadIdx.x; i < total; i += kThreads) {
    const bool is64 = i < a.n64 * plane;
    const int p = is64 ? i / plane : (i - a.n64 * plane) / plane;
    const int rem = i - (is64 ? p : a.n64 + p) * plane;
    long long v;
    int k;
    if (is64) {
      v = (long long)h64[i];
      k = 1;
    } else {
      v = (long long)h32[i - a.n64 * plane];
      k = p;
    }
    if (v == 0) continue;
    const int ls = rem / (8 * a.B);
    const int jj = (rem / a.B) & 7;
    const int bn = rem % a.B;
    const int f = fbase + jj;
    const int slot = s0 + ls;
    if (f < a.d && slot < a.S)
      atomicAdd(&a.out[(((int64_t)slot * a.d + f) * a.B + bn) * a.K + k], (unsigned long long)v);
  }
}

// ---------------------------------------------------------------------------
// PACKED (regression, integer weights): ONE ds_add_u64 per update instead of
// a u32 count + u64 sum pair.  The LDS word holds
//     count (bits 44..63)  |  sum_r w_r * (q_r + 2^23)  (bits 0..43)
// with q = round(v * 2^s), |q| <= 2^23 (offset-binary, so no borrow crosses
// into the count field).  Every kSpillRows rows the block drains its LDS words
// into per-thread register accumulators (uint32 count, int64 sum), so the
// fields provably never overflow: count <= 255 * 4096 < 2^20 and the sum field
// <= 4096 * 255 * 2^24 < 2^44.  Measured motive: at level 0 the two-atomic
// kernel sustained ~3 of the ~4 LDS atomic lane-ops/clk/CU the hardware gives
// (bench/lds_atomic_bench.hip), so halving the atomics halves the bound.
// ---------------------------------------------------------------------------
constexpr int kPackShift = 44;
constexpr long long kPackQ = 1LL << 23;
constexpr int kSpillIters = 8;  // 8 x 512 rows = 4096 rows between register drains
constexpr int kMaxCells = 16;   // register accumulators per thread -> LDS plane <= 8192 words

__global__ __launch_bounds__(kThreads) void hist4p_kernel(const Hist4Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  unsigned long long* h64 = reinterpret_cast<unsigned long long*>(smem);
  int* lslot = reinterpret_cast<int*>(h64 + plane);
  uint8_t* lmask = reinterpret_cast<uint8_t*>(lslot + a.id_span_max);

  const uint32_t w = cdna::xcd_remap(blockIdx.x, gridDim.x);
  const int g = (int)(w % G);
  const int grp = (int)((w / G) % a.ngroups);
  const int chunk = (int)(w / ((uint32_t)G * a.ngroups));
  const int s0 = a.grp[grp * 5 + 0], t0 = a.grp[grp * 5 + 1], t1 = a.grp[grp * 5 + 2];
  const int id0 = a.grp[grp * 5 + 3], id1 = a.grp[grp * 5 + 4];
  const int span = id1 - id0;
  const bool lds_slot = span <= a.id_span_max;
  const int fbase = g * 8;
  const int rot = threadIdx.x & 7;

  for (int i = threadIdx.x; i < plane; i += kThreads) h64[i] = 0ull;
  if (lds_slot)
    for (int i = threadIdx.x; i < span; i += kThreads) lslot[i] = a.build_slot[id0 + i];
  for (int i = threadIdx.x; i < a.SB; i += kThreads) {
    uint32_t m = 0xFFu;
    const int slot = s0 + i;
    if (a.feat_mask != nullptr && slot < a.S)
      m = (a.feat_mask[(int64_t)slot * a.mask_words + (fbase >> 5)] >> (fbase & 31)) & 0xFFu;
    const int valid = a.d - fbase;
    if (valid < 8) m &= (1u << (valid > 0 ? valid : 0)) - 1u;
    lmask[i] = (uint8_t)m;
  }
  uint32_t acc_c[kMaxCells];
  long long acc_s[kMaxCells];
#pragma unroll
  for (int i = 0; i < kMaxCells; ++i) {
    acc_c[i] = 0u;
    acc_s[i] = 0;
  }
  __syncthreads();

  const int64_t rb = (int64_t)chunk * a.rows_per_chunk;
  int64_t re = rb + a.rows_per_chunk;
  if (re > a.n) re = a.n;
  const int64_t n = a.n;
  const int nt_head = t1 - t0 + 1 < 4 ? t1 - t0 + 1 : 4;

  auto drain = [&]() {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kMaxCells; ++i) {
      const int idx = (int)threadIdx.x + i * kThreads;
      if (idx < plane) {
        const unsigned long long v = h64[idx];
        if (v) {
          const uint32_t c = (uint32_t)(v >> kPackShift);
          acc_c[i] += c;
          acc_s[i] += (long long)(v & ((1ull << kPackShift) - 1ull)) - kPackQ * (long long)c;
          h64[idx] = 0ull;
        }
      }
    }
    __syncthreads();
  };

  uint64_t b8 = 0;
  float x1 = 0.f;
  int ids[4] = {-1, -1, -1, -1};
  int wt[4] = {0, 0, 0, 0};
  auto load_row = [&](int64_t rr, uint64_t& ob8, float& ox1, int* oids, int* owt) {
    ob8 = a.bins[(int64_t)g * n + rr];
    ox1 = a.v1[rr];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = k < nt_head;
      oids[k] = ok ? a.node[(int64_t)(t0 + k) * n + rr] : -1;
      owt[k] = (ok && a.weight) ? (int)a.weight[(int64_t)(t0 + k) * n + rr] : 1;
    }
  };
  if (rb + (int64_t)threadIdx.x < re) load_row(rb + threadIdx.x, b8, x1, ids, wt);

  int iter = 0;
  for (int64_t base = rb; base < re; base += kThreads, ++iter) {
    const int64_t r = base + threadIdx.x;
    const bool live = r < re;
    uint64_t nb8 = 0;
    float nx1 = 0.f;
    int nids[4] = {-1, -1, -1, -1};
    int nwt[4] = {0, 0, 0, 0};
    if (r + kThreads < re) load_row(r + kThreads, nb8, nx1, nids, nwt);
    if (live) {
      long long q = llrintf(x1 * a.qs1);
      q = q > kPackQ ? kPackQ : (q < -kPackQ ? -kPackQ : q);
      const unsigned long long qoff = (unsigned long long)(q + kPackQ);
      for (int t = t0; t <= t1; t += 4) {
        int cid[4], cwt[4];
        if (t == t0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) { cid[k] = ids[k]; cwt[k] = wt[k]; }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int tt = t + k;
            const bool ok = tt <= t1;
            cid[k] = ok ? a.node[(int64_t)tt * n + r] : -1;
            cwt[k] = (ok && a.weight) ? (int)a.weight[(int64_t)tt * n + r] : 1;
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int id = cid[k];
          if (id < id0 || id >= id1 || cwt[k] == 0) continue;
          const int sl = lds_slot ? lslot[id - id0] : a.build_slot[id];
          const int ls = sl - s0;
          if (ls < 0 || ls >= a.SB) continue;
          const uint32_t m = lmask[ls];
          const int off = (ls * 8) * a.B;
          const unsigned long long add =
              ((unsigned long long)cwt[k] << kPackShift) + (unsigned long long)cwt[k] * qoff;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int jj = (j + rot) & 7;
            if ((m >> jj) & 1u) atomicAdd(h64 + off + jj * a.B + (int)((b8 >> (8 * jj)) & 0xFFu), add);
          }
        }
      }
    }
    b8 = nb8;
    x1 = nx1;
#pragma unroll
    for (int k = 0; k < 4; ++k) { ids[k] = nids[k]; wt[k] = nwt[k]; }
    if ((iter + 1) % kSpillIters == 0) drain();  // block-uniform: every thread runs the same iterations
  }
  drain();
#pragma unroll
  for (int i = 0; i < kMaxCells; ++i) {
    const int idx = (int)threadIdx.x + i * kThreads;
    if (idx >= plane || acc_c[i] == 0u) continue;
    const int ls = idx / (8 * a.B);
    const int jj = (idx / a.B) & 7;
    const int bn = idx % a.B;
    const int f = fbase + jj;
    const int slot = s0 + ls;
    if (f < a.d && slot < a.S) {
      unsigned long long* o = &a.out[(((int64_t)slot * a.d + f) * a.B + bn) * 2];
      atomicAdd(o, (unsigned long long)acc_c[i]);
      atomicAdd(o + 1, (unsigned long long)acc_s[i]);
    }
  }
}

template <int MODE, bool V0>
void launch(const Hist4Args& a, unsigned nblk, size_t lds, int map, hipStream_t st) {
  if (map == 1)
    hipLaunchKernelGGL((hist4_kernel<MODE, V0, 1>), dim3(nblk), dim3(kThreads), lds, st, a);
  else if (map == 2)
    hipLaunchKernelGGL((hist4r_kernel<MODE, V0>), dim3(nblk), dim3(kThreads), lds, st, a);
  else
    hipLaunchKernelGGL((hist4_kernel<MODE, V0, 0>), dim3(nblk), dim3(kThreads), lds, st, a);
}

}  // namespace

// Bytes of LDS per (slot x 8 features x bin) for a mode — the host uses this to
// size slot groups.  mode 0 = moments (v0 absent), 4 = moments with v0, 1 = classes.
CDNA_API int cdna_hist4_bytes_per_bin(int mode, int C) {
  if (mode & 1) return 4 * C;
  if (mode & 16) return 8;
  return (mode & 4) ? 16 : 12;
}

// mode bit0: classes; bit1: v3 lane mapping; bit2: v0 present (moments);
// bit3: rotated features + pipelined row loads (MAP 2); bit4: packed single-atomic
// regression kernel (moments without v0; qs1 must keep |v * qs1| <= 2^23);
// bit5: fast rotated kernel (no v0; qs1 must keep |v * qs1| < 2^30 for 32-bit quantisation).
// `out` (int64 [S][d][B][K]) must be zeroed.  Result in fixed point: plane k
// scaled by qs_k (counts unscaled).
CDNA_API int cdna_hist4(int mode, const uint64_t* bins, int64_t n, int d, int T, const int* node,
                        const uint8_t* weight, const float* v0, const float* v1, const int* label, int C,
                        const int* build_slot, const uint32_t* feat_mask, int mask_words, int S, int B, int SB,
                        const int* grp, int ngroups, int nchunk, int id_span_max, float qs0, float qs1,
                        unsigned long long* out, hipStream_t st) {
  if (n <= 0 || S <= 0) return 0;
  Hist4Args a;
  a.bins = bins;
  a.n = n;
  a.d = d;
  a.T = T;
  a.node = node;
  a.weight = weight;
  a.v0 = v0;
  a.v1 = v1;
  a.label = label;
  a.C = C;
  a.build_slot = build_slot;
  a.feat_mask = feat_mask;
  a.mask_words = mask_words;
  a.S = S;
  a.B = B;
  a.SB = SB;
  const bool classes = (mode & 1) != 0, has_v0 = (mode & 4) != 0;
  a.K = classes ? C : 2;
  a.n64 = classes ? 0 : (has_v0 ? 2 : 1);
  a.n32 = classes ? C : (has_v0 ? 0 : 1);
  a.grp = grp;
  a.ngroups = ngroups;
  a.nchunk = nchunk;
  a.rows_per_chunk = (n + nchunk - 1) / nchunk;
  // u32 LDS counts: at most rows_per_chunk * 255 per word
  if (a.rows_per_chunk * 255 >= (int64_t)1 << 32) return (int)hipErrorInvalidValue;
  a.id_span_max = id_span_max;
  a.qs0 = qs0;
  a.qs1 = qs1;
  a.out = out;
  const int G = (d + 7) / 8;
  const size_t plane = (size_t)SB * 8 * B;
  const size_t lds = plane * 8 * a.n64 + ((plane * a.n32 + 3) & ~(size_t)3) * 4 + (size_t)id_span_max * 4 + SB + 16;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  const unsigned nblk = (unsigned)G * ngroups * nchunk;
  const int map = (mode & 2) ? 1 : ((mode & 8) ? 2 : 0);
  if ((mode & 32) && !has_v0) {  // fast rotated kernel (moments without v0, or classes)
    const bool masked = feat_mask != nullptr;
    if (classes) {
      if (masked) hipLaunchKernelGGL((hist4f_kernel<1, true>), dim3(nblk), dim3(kThreads), lds, st, a);
      else hipLaunchKernelGGL((hist4f_kernel<1, false>), dim3(nblk), dim3(kThreads), lds, st, a);
    } else {
      if (masked) hipLaunchKernelGGL((hist4f_kernel<0, true>), dim3(nblk), dim3(kThreads), lds, st, a);
      else hipLaunchKernelGGL((hist4f_kernel<0, false>), dim3(nblk), dim3(kThreads), lds, st, a);
    }
    return (int)hipGetLastError();
  }
  if (mode & 16) {  // packed single-atomic regression kernel
    if (classes || has_v0) return (int)hipErrorInvalidValue;
    if (plane > (size_t)kMaxCells * kThreads) return (int)hipErrorInvalidValue;
    a.n64 = 1;
    a.n32 = 0;
    const size_t lds_p = plane * 8 + (size_t)id_span_max * 4 + SB + 16;
    hipLaunchKernelGGL(hist4p_kernel, dim3(nblk), dim3(kThreads), lds_p, st, a);
    return (int)hipGetLastError();
  }
  if (classes) launch<1, false>(a, nblk, lds, map, st);
  else if (has_v0) launch<0, true>(a, nblk, lds, map, st);
  else launch<0, false>(a, nblk, lds, map, st);
  return (int)hipGetLastError();
}
