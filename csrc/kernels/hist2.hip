// K5 hist_build, v2 — LDS-privatised split statistics for level-wise tree
// learning (moments for variance/XGBoost gain, class counts for gini/entropy).
//
// What v1 (trees.hip) measured on MI355X (rocprofv3, 1e7 x 100, 20 trees):
// 94 % of fit time in the histogram at ~2.3e11 lane-atomics/s.  Causes and
// the v2 fixes:
//   * 256-thread blocks holding 64 KB of LDS -> 2 waves/SIMD, and a chain of
//     DEPENDENT global loads per (row, tree): node id -> build_slot[id] ->
//     feat_mask[slot].  v2: 512-thread blocks, the group's slot map and the
//     feature-mask bytes are staged in LDS once per block, and node ids /
//     bootstrap weights of 4 trees are loaded together (4 loads in flight).
//   * stats interleaved [bin][2] -> one LDS bank per two bins.  v2: one
//     plane per statistic ([k][slot][feat][bin]) so a wave's 64 random bins
//     spread over all 32 banks of ds_add_f32.
//   * blocks of one row chunk scattered over the grid -> node/weight/label
//     re-reads by the G feature-group blocks came from HBM.  v2: decode
//     order (feature group, slot group) fastest and chunk slowest, after the
//     XCD remap, so all blocks reading a chunk run together on one XCD and
//     share its L2.
#include "common.h"

namespace {

struct Hist2Args {
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
  double* out;  // [S][d][B][K]
};

constexpr int kThreads = 512;

template <int MODE>  // 0: moments (planes w*v0, w*v1); 1: class counts (plane = label)
__global__ __launch_bounds__(kThreads) void hist2_kernel(const Hist2Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  const int hsz = a.K * plane;
  float* h = reinterpret_cast<float*>(smem);
  int* lslot = reinterpret_cast<int*>(smem + (((size_t)hsz * 4 + 15) / 16) * 16);
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

  for (int i = threadIdx.x; i < hsz; i += kThreads) h[i] = 0.f;
  if (lds_slot)
    for (int i = threadIdx.x; i < span; i += kThreads) lslot[i] = a.build_slot[id0 + i];
  for (int i = threadIdx.x; i < a.SB; i += kThreads) {
    uint32_t m = 0xFFu;
    const int slot = s0 + i;
    if (a.feat_mask != nullptr && slot < a.S)
      m = (a.feat_mask[(int64_t)slot * a.mask_words + (fbase >> 5)] >> (fbase & 31)) & 0xFFu;
    // features past d never contribute
    const int valid = a.d - fbase;
    if (valid < 8) m &= (1u << (valid > 0 ? valid : 0)) - 1u;
    lmask[i] = (uint8_t)m;
  }
  __syncthreads();

  const int64_t rb = (int64_t)chunk * a.rows_per_chunk;
  int64_t re = rb + a.rows_per_chunk;
  if (re > a.n) re = a.n;
  const int64_t n = a.n;
  for (int64_t r = rb + threadIdx.x; r < re; r += kThreads) {
    const uint64_t b8 = a.bins[(int64_t)g * n + r];
    float x0 = 1.f, x1 = 0.f;
    int c = 0;
    if (MODE == 0) {
      if (a.v0) x0 = a.v0[r];
      x1 = a.v1[r];
    } else {
      c = a.label[r];
      if (c < 0 || c >= a.C) continue;
    }
    for (int t = t0; t <= t1; t += 4) {
      int ids[4];
      float wt[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int tt = t + k;
        const bool ok = tt <= t1;
        ids[k] = ok ? a.node[(int64_t)tt * n + r] : -1;
        wt[k] = (ok && a.weight) ? (float)a.weight[(int64_t)tt * n + r] : 1.f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int id = ids[k];
        if (id < id0 || id >= id1 || wt[k] == 0.f) continue;
        const int sl = lds_slot ? lslot[id - id0] : a.build_slot[id];
        const int ls = sl - s0;
        if (ls < 0 || ls >= a.SB) continue;
        const uint32_t m = lmask[ls];
        float* base = h + (ls * 8) * a.B;
        if (MODE == 0) {
          const float y0 = wt[k] * x0, y1 = wt[k] * x1;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if ((m >> j) & 1u) {
              const int idx = j * a.B + (int)((b8 >> (8 * j)) & 0xFFu);
              atomicAdd(base + idx, y0);
              atomicAdd(base + plane + idx, y1);
            }
          }
        } else {
          float* pc = base + c * plane;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if ((m >> j) & 1u) atomicAdd(pc + j * a.B + (int)((b8 >> (8 * j)) & 0xFFu), wt[k]);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < hsz; i += kThreads) {
    const float v = h[i];
    if (v == 0.f) continue;
    const int k = i / plane;
    const int rem = i - k * plane;
    const int ls = rem / (8 * a.B);
    const int j = (rem / a.B) & 7;
    const int bin = rem % a.B;
    const int f = fbase + j;
    const int slot = s0 + ls;
    if (f < a.d && slot < a.S) atomicAdd(&a.out[(((int64_t)slot * a.d + f) * a.B + bin) * a.K + k], (double)v);
  }
}

// ---------------------------------------------------------------------------
// v3 lane mapping: lane = 8 * row + feature.  Measured on v2 (rocprofv3 PMC,
// 1e7 rows): SQ_LDS_IDX_ACTIVE / SQ_INSTS_LDS ~ 100 LDS cycles per ds_add_f32
// with SQ_LDS_BANK_CONFLICT = 0 — the 64 lanes of one instruction all target
// the same (slot, feature) and only B ~ 40 bins, so several lanes hit the SAME
// word and the atomic unit serialises them.  With 8 rows x 8 features per
// instruction only lanes sharing a feature can collide (8 rows over B bins),
// and the 8 features land 8*B words apart, spreading the banks.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kThreads) void hist3_kernel(const Hist2Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  const int hsz = a.K * plane;
  float* h = reinterpret_cast<float*>(smem);
  int* lslot = reinterpret_cast<int*>(smem + (((size_t)hsz * 4 + 15) / 16) * 16);
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
  const int j = threadIdx.x & 7;       // feature within the group
  const int rl = threadIdx.x >> 3;     // row within the 64-row step

  for (int i = threadIdx.x; i < hsz; i += kThreads) h[i] = 0.f;
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
  constexpr int kRowsPerStep = kThreads / 8;
  for (int64_t r = rb + rl; r < re; r += kRowsPerStep) {
    const int bin = bins8[((int64_t)g * n + r) * 8 + j];
    float x0 = 1.f, x1 = 0.f;
    int c = 0;
    if (MODE == 0) {
      if (a.v0) x0 = a.v0[r];
      x1 = a.v1[r];
    } else {
      c = a.label[r];
      if (c < 0 || c >= a.C) continue;
    }
    for (int t = t0; t <= t1; t += 4) {
      int ids[4];
      float wt[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int tt = t + k;
        const bool ok = tt <= t1;
        ids[k] = ok ? a.node[(int64_t)tt * n + r] : -1;
        wt[k] = (ok && a.weight) ? (float)a.weight[(int64_t)tt * n + r] : 1.f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int id = ids[k];
        if (id < id0 || id >= id1 || wt[k] == 0.f) continue;
        const int sl = lds_slot ? lslot[id - id0] : a.build_slot[id];
        const int ls = sl - s0;
        if (ls < 0 || ls >= a.SB) continue;
        if (!((lmask[ls] >> j) & 1u)) continue;
        float* p = h + (ls * 8 + j) * a.B + bin;
        if (MODE == 0) {
          atomicAdd(p, wt[k] * x0);
          atomicAdd(p + plane, wt[k] * x1);
        } else {
          atomicAdd(p + c * plane, wt[k]);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < hsz; i += kThreads) {
    const float v = h[i];
    if (v == 0.f) continue;
    const int k = i / plane;
    const int rem = i - k * plane;
    const int ls = rem / (8 * a.B);
    const int jj = (rem / a.B) & 7;
    const int bn = rem % a.B;
    const int f = fbase + jj;
    const int slot = s0 + ls;
    if (f < a.d && slot < a.S) atomicAdd(&a.out[(((int64_t)slot * a.d + f) * a.B + bn) * a.K + k], (double)v);
  }
}

}  // namespace

// grp: device int32 [ngroups][5] (s0, t0, t1, id0, id1).  mode 0 = moments
// (K = 2), mode 1 = classes (K = C).  `out` must be zeroed.
CDNA_API int cdna_hist2(int mode, const uint64_t* bins, int64_t n, int d, int T, const int* node,
                        const uint8_t* weight, const float* v0, const float* v1, const int* label, int C,
                        const int* build_slot, const uint32_t* feat_mask, int mask_words, int S, int B, int SB,
                        const int* grp, int ngroups, int nchunk, int id_span_max, double* out, hipStream_t st) {
  if (n <= 0 || S <= 0) return 0;
  Hist2Args a;
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
  a.K = (mode & 1) == 0 ? 2 : C;
  a.grp = grp;
  a.ngroups = ngroups;
  a.nchunk = nchunk;
  a.rows_per_chunk = (n + nchunk - 1) / nchunk;
  a.id_span_max = id_span_max;
  a.out = out;
  const int G = (d + 7) / 8;
  const size_t lds = (((size_t)a.K * SB * 8 * B * 4 + 15) / 16) * 16 + (size_t)id_span_max * 4 + SB + 16;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  const unsigned nblk = (unsigned)G * ngroups * nchunk;
  const bool v3 = (mode & 2) != 0;  // bit 1 selects the 8-rows x 8-features lane mapping
  if ((mode & 1) == 0)
    hipLaunchKernelGGL(v3 ? hist3_kernel<0> : hist2_kernel<0>, dim3(nblk), dim3(kThreads), lds, st, a);
  else
    hipLaunchKernelGGL(v3 ? hist3_kernel<1> : hist2_kernel<1>, dim3(nblk), dim3(kThreads), lds, st, a);
  return (int)hipGetLastError();
}
