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
// loop over the 8 features of their bins word.  (Measured and removed: the v3
// lane = 8 * row + feature mapping, a rotated-feature pipelined variant and a
// packed single-atomic variant -- the fast kernel hist4f below replaced them.)
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
template <int MODE, bool V0>
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
  for (int64_t r = rb + threadIdx.x; r < re; r += kThreads) {
    const uint64_t b8 = a.bins[(int64_t)g * n + r];
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
        const uint32_t m = lmask[ls];
        const int off = (ls * 8) * a.B;
        const long long y1 = (long long)wt[k] * q1;
        const long long y0 = V0 ? (long long)wt[k] * q0 : 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if ((m >> j) & 1u) {
            const int idx = off + j * a.B + (int)((b8 >> (8 * j)) & 0xFFu);
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

template <int MODE, bool V0>
void launch(const Hist4Args& a, unsigned nblk, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((hist4_kernel<MODE, V0>), dim3(nblk), dim3(kThreads), lds, st, a);
}

}  // namespace

// Bytes of LDS per (slot x 8 features x bin) for a mode — the host uses this to
// size slot groups.  mode 0 = moments (v0 absent), 4 = moments with v0, 1 = classes.
CDNA_API int cdna_hist4_bytes_per_bin(int mode, int C) {
  if (mode & 1) return 4 * C;
  return (mode & 4) ? 16 : 12;
}

// mode bit0: classes; bit2: v0 present (moments);
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
  if (classes) launch<1, false>(a, nblk, lds, st);
  else if (has_v0) launch<0, true>(a, nblk, lds, st);
  else launch<0, false>(a, nblk, lds, st);
  return (int)hipGetLastError();
}
