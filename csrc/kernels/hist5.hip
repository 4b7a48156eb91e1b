// K5/K7 on compact row records: hist v5 + partition over uint16 "codes".
//
// v4 (hist4f) loaded, per (row, tree) and per 8-feature block, a 4-byte node id
// and a 1-byte bootstrap weight from two [T][n] arrays: at level 0 with 20
// trees that is 13 feature blocks x 20 x 5 B = 1.3 KB of loads per row, the
// dominant traffic of the kernel (profiles/pmc_hist4_1e8.csv: 62 % of wave
// time waiting on vector memory).  v5 keeps ONE uint16 per (row, tree):
//
//     code = weight << 8 | local        local = node index within its tree's
//                                       active set at this level, 255 = done
//
// stored tree-major ([T][n], like the int32 node ids it replaces) so every
// per-tree load of a wave is one coalesced 128-byte line (a row-major record
// was measured slower at deep levels, where a block touches only 1-2 trees).
// The global active id is tfirst[t] + local (tfirst = first active id of
// tree t, a per-level table).  Rows with zero
// bootstrap weight are "done" from the start and never touch LDS.  The
// histogram inner loop is hist4f's (rotated features, hoisted VALU work,
// batched slot-table reads); the next row's record is prefetched.
#include "common.h"

namespace {

constexpr int kThreads = 512;
constexpr int kMaxTrees = 16;  // trees per block group (host splits larger groups)

struct Hist5Args {
  const uint64_t* bins;  // [G][n] 8 bins per word
  int64_t n;
  int d, T;
  const uint16_t* codes;  // [T][n]
  const int* tfirst;      // [T] first active id of each tree at this level
  const float* v0;
  const float* v1;
  const int* label;
  int C;
  const int* build_slot;  // [A] slot or -1
  const uint32_t* feat_mask;
  int mask_words, S, B, SB, K;
  const int* grp;  // [ngroups][5] = s0, t0, t1, id0, id1
  int ngroups, nchunk;
  int64_t rows_per_chunk;
  float qs0, qs1;
  int n64, n32;
  int drain_iters;          // packed kernel: row iterations between register drains
  unsigned long long* out;  // [S][d][B][K]
};

// MODE 0: moments (count u32 + sum u64, or with V0 two u64 sums); MODE 1: class counts (u32).
template <int MODE, bool MASKED, bool V0, int NT>
__global__ __launch_bounds__(kThreads) void hist5_kernel(const Hist5Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  unsigned long long* h64 = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* h32 = reinterpret_cast<uint32_t*>(h64 + (size_t)a.n64 * plane);
  const int hwords = a.n32 * plane;
  // per-tree local-node -> slot table: lt[k][loc] = slot - s0 or -1 (loc 255 = done)
  int16_t* lt = reinterpret_cast<int16_t*>(h32 + ((hwords + 3) & ~3));
  const uint32_t w = cdna::xcd_remap(blockIdx.x, gridDim.x);
  const int g = (int)(w % G);
  const int grp = (int)((w / G) % a.ngroups);
  const int chunk = (int)(w / ((uint32_t)G * a.ngroups));
  const int s0 = a.grp[grp * 5 + 0], t0 = a.grp[grp * 5 + 1], t1 = a.grp[grp * 5 + 2];
  const int id1 = a.grp[grp * 5 + 4];
  const int nt = t1 - t0 + 1;  // <= kMaxTrees (host-checked)
  uint8_t* lmask = reinterpret_cast<uint8_t*>(lt + NT * 256);
  const int fbase = g * 8;
  const int rot = threadIdx.x & 7;

  for (int i = threadIdx.x; i < a.n64 * plane; i += kThreads) h64[i] = 0ull;
  for (int i = threadIdx.x; i < hwords; i += kThreads) h32[i] = 0u;
  for (int i = threadIdx.x; i < NT * 256; i += kThreads) {
    const int k = i >> 8, loc = i & 255;
    int v = -1;
    const int id = k < nt ? a.tfirst[t0 + k] + loc : 0;
    const int idend = k + 1 < nt ? a.tfirst[t0 + k + 1] : id1;
    if (k < nt && loc != 255 && id < idend) {
      const int sl = a.build_slot[id];
      if (sl >= s0 && sl < s0 + a.SB) v = sl - s0;
    }
    lt[i] = (int16_t)v;
  }
  if (MASKED) {
    for (int i = threadIdx.x; i < a.SB; i += kThreads) {
      const int slot = s0 + i;
      uint32_t m = 0u;
      if (slot < a.S) m = (a.feat_mask[(int64_t)slot * a.mask_words + (fbase >> 5)] >> (fbase & 31)) & 0xFFu;
      const int valid = a.d - fbase;
      if (valid < 8) m &= (1u << (valid > 0 ? valid : 0)) - 1u;
      lmask[i] = (uint8_t)m;
    }
  }
  int fsel[8], fsh[8], foff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int jj = (j + rot) & 7;
    fsel[j] = jj >> 2;
    fsh[j] = (jj & 3) * 8;
    foff[j] = jj * a.B;
  }
  // features beyond d in the last block
  const int valid_f = a.d - fbase;
  uint32_t fvalid = valid_f >= 8 ? 0xFFu : ((1u << (valid_f > 0 ? valid_f : 0)) - 1u);
  const uint32_t frot = ((fvalid >> rot) | (fvalid << (8 - rot))) & 0xFFu;
  __syncthreads();

  const int64_t rb = (int64_t)chunk * a.rows_per_chunk;
  int64_t re = rb + a.rows_per_chunk;
  if (re > a.n) re = a.n;
  const int64_t n = a.n;
  const int slot_cells = 8 * a.B;

  uint64_t b8 = 0;
  float x0 = 1.f, x1 = 0.f;
  int lab = 0;
  uint32_t cd[NT];
  // trees past nt read a valid row (their tables are all -1, so they never add)
  const int64_t tstride = (int64_t)n;
  auto load_row = [&](int64_t rr, uint64_t& ob8, float& ox0, float& ox1, int& olab, uint32_t* ocd) {
    ob8 = a.bins[(int64_t)g * n + rr];
    if (MODE == 0) {
      if (V0) ox0 = a.v0[rr];
      ox1 = a.v1[rr];
    } else {
      olab = a.label[rr];
    }
    const uint16_t* cp = a.codes + (int64_t)t0 * n + rr;
#pragma unroll
    for (int k = 0; k < NT; ++k) ocd[k] = (uint32_t)cp[(k < nt ? k : 0) * tstride];
  };
  int64_t r = rb + threadIdx.x;
  if (r < re) load_row(r, b8, x0, x1, lab, cd);
  else {
#pragma unroll
    for (int k = 0; k < NT; ++k) cd[k] = 0xFFu;
  }

  for (; r < re; r += kThreads) {
    uint64_t nb8 = 0;
    float nx0 = 1.f, nx1 = 0.f;
    int nlab = 0;
    uint32_t ncd[NT];
    const int64_t rn = r + kThreads;
    if (rn < re) load_row(rn, nb8, nx0, nx1, nlab, ncd);
    else {
#pragma unroll
      for (int k = 0; k < NT; ++k) ncd[k] = 0xFFu;
    }

    const uint32_t lo = (uint32_t)b8, hi = (uint32_t)(b8 >> 32);
    int cell[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      cell[j] = foff[j] + (int)__builtin_amdgcn_ubfe(fsel[j] ? hi : lo, (uint32_t)fsh[j], 8u);
    int q0 = 1, q1 = 0;
    bool row_ok = true;
    if (MODE == 0) {
      if (V0) q0 = (int)rintf(x0 * a.qs0);
      q1 = (int)rintf(x1 * a.qs1);
    } else {
      row_ok = lab >= 0 && lab < a.C;
    }
    const uint32_t cbase_lab = MODE == 1 ? (uint32_t)(lab * plane) : 0u;
    if (row_ok) {
      constexpr int KB = NT;  // all slot-table reads of the row first: one LDS wait per row
#pragma unroll
      for (int kb = 0; kb < NT; kb += KB) {
        int lsk[KB];
        uint32_t mk[KB];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          lsk[k] = lt[(kb + k) * 256 + (int)(cd[kb + k] & 0xFFu)];  // -1: done / not built here
          if (MASKED) mk[k] = lmask[lsk[k] < 0 ? 0 : lsk[k]];
        }
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const int ls = lsk[k];
          if (ls < 0) continue;
          const uint32_t wv = cd[kb + k] >> 8;
          const uint32_t base = (uint32_t)(ls * slot_cells) + cbase_lab;
          uint32_t mrot = frot;
          if (MASKED) mrot &= ((mk[k] >> rot) | (mk[k] << (8 - rot))) & 0xFFu;
          const long long y1 = (long long)wv * (long long)q1;
          const long long y0 = V0 ? (long long)wv * (long long)q0 : 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (!((mrot >> j) & 1u)) continue;
            const uint32_t c = base + (uint32_t)cell[j];
            if (MODE == 1) {
              atomicAdd(h32 + c, wv);
            } else if (V0) {
              atomicAdd(h64 + c, (unsigned long long)y0);
              atomicAdd(h64 + plane + c, (unsigned long long)y1);
            } else {
              atomicAdd(h32 + c, wv);
              atomicAdd(h64 + c, (unsigned long long)y1);
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
    for (int k = 0; k < NT; ++k) cd[k] = ncd[k];
  }
  __syncthreads();
  // flush: 64-bit planes first (k = 1 for count+sum moments, k = p with V0), then 32-bit planes
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

// Packed regression variant (measured motive: the two-atomic kernel reaches
// ~3.5 of the ~4 LDS atomic lane-ops/clk/CU at full levels): ONE ds_add_u64
// per update holding count (bits 44..63) | sum of w * (q + 2^23) (bits 0..43).
// Every kPackIters * 512 = 4096 rows the block drains its words into
// per-thread registers (uint32 count, int64 sum), so count <= 255 * 4096 < 2^20
// and the offset sum < 4096 * 255 * 2^24 = 2^44: no field can overflow.
constexpr int kPackShift = 44;
constexpr int kPackQ = 1 << 23;
constexpr int kPackIters = 8;
constexpr int kPackCells = 16;  // plane <= 16 * 512 = 8192 cells (64 KB)

template <bool MASKED, int NT, int TH>
__global__ __launch_bounds__(TH) void hist5p_kernel(const Hist5Args a) {
  // rows between drains: (rows x max weight) < 2^20 keeps both packed fields in range
  const int drain_iters = a.drain_iters;
  constexpr int MODE = 0;
  constexpr bool V0 = false;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  unsigned long long* h64 = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* h32 = reinterpret_cast<uint32_t*>(h64 + (size_t)plane);
  const int hwords = 0;
  // per-tree local-node -> slot table: lt[k][loc] = slot - s0 or -1 (loc 255 = done)
  int16_t* lt = reinterpret_cast<int16_t*>(h32 + ((hwords + 3) & ~3));
  const uint32_t w = cdna::xcd_remap(blockIdx.x, gridDim.x);
  const int g = (int)(w % G);
  const int grp = (int)((w / G) % a.ngroups);
  const int chunk = (int)(w / ((uint32_t)G * a.ngroups));
  const int s0 = a.grp[grp * 5 + 0], t0 = a.grp[grp * 5 + 1], t1 = a.grp[grp * 5 + 2];
  const int id1 = a.grp[grp * 5 + 4];
  const int nt = t1 - t0 + 1;  // <= kMaxTrees (host-checked)
  uint8_t* lmask = reinterpret_cast<uint8_t*>(lt + NT * 256);
  const int fbase = g * 8;
  const int rot = threadIdx.x & 7;

  for (int i = threadIdx.x; i < plane; i += TH) h64[i] = 0ull;
  uint32_t acc_c[kPackCells];
  long long acc_s[kPackCells];
#pragma unroll
  for (int i = 0; i < kPackCells; ++i) {
    acc_c[i] = 0u;
    acc_s[i] = 0;
  }
  for (int i = threadIdx.x; i < hwords; i += TH) h32[i] = 0u;
  for (int i = threadIdx.x; i < NT * 256; i += TH) {
    const int k = i >> 8, loc = i & 255;
    int v = -1;
    const int id = k < nt ? a.tfirst[t0 + k] + loc : 0;
    const int idend = k + 1 < nt ? a.tfirst[t0 + k + 1] : id1;
    if (k < nt && loc != 255 && id < idend) {
      const int sl = a.build_slot[id];
      if (sl >= s0 && sl < s0 + a.SB) v = sl - s0;
    }
    lt[i] = (int16_t)v;
  }
  if (MASKED) {
    for (int i = threadIdx.x; i < a.SB; i += TH) {
      const int slot = s0 + i;
      uint32_t m = 0u;
      if (slot < a.S) m = (a.feat_mask[(int64_t)slot * a.mask_words + (fbase >> 5)] >> (fbase & 31)) & 0xFFu;
      const int valid = a.d - fbase;
      if (valid < 8) m &= (1u << (valid > 0 ? valid : 0)) - 1u;
      lmask[i] = (uint8_t)m;
    }
  }
  int fsel[8], fsh[8], foff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int jj = (j + rot) & 7;
    fsel[j] = jj >> 2;
    fsh[j] = (jj & 3) * 8;
    foff[j] = jj * a.B;
  }
  // features beyond d in the last block
  const int valid_f = a.d - fbase;
  uint32_t fvalid = valid_f >= 8 ? 0xFFu : ((1u << (valid_f > 0 ? valid_f : 0)) - 1u);
  const uint32_t frot = ((fvalid >> rot) | (fvalid << (8 - rot))) & 0xFFu;
  const bool all8 = valid_f >= 8;
  __syncthreads();

  const int64_t rb = (int64_t)chunk * a.rows_per_chunk;
  int64_t re = rb + a.rows_per_chunk;
  if (re > a.n) re = a.n;
  const int64_t n = a.n;
  const int slot_cells = 8 * a.B;

  uint64_t b8 = 0;
  float x0 = 1.f, x1 = 0.f;
  int lab = 0;
  uint32_t cd[NT];
  // trees past nt read a valid row (their tables are all -1, so they never add)
  const int64_t tstride = (int64_t)n;
  auto load_row = [&](int64_t rr, uint64_t& ob8, float& ox0, float& ox1, int& olab, uint32_t* ocd) {
    ob8 = a.bins[(int64_t)g * n + rr];
    if (MODE == 0) {
      if (V0) ox0 = a.v0[rr];
      ox1 = a.v1[rr];
    } else {
      olab = a.label[rr];
    }
    const uint16_t* cp = a.codes + (int64_t)t0 * n + rr;
#pragma unroll
    for (int k = 0; k < NT; ++k) ocd[k] = (uint32_t)cp[(k < nt ? k : 0) * tstride];
  };
  auto drain = [&]() {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPackCells; ++i) {
      const int idx = (int)threadIdx.x + i * TH;
      if (idx < plane) {
        const unsigned long long v = h64[idx];
        if (v) {
          const uint32_t c = (uint32_t)(v >> kPackShift);
          acc_c[i] += c;
          acc_s[i] += (long long)(v & ((1ull << kPackShift) - 1ull)) - (long long)kPackQ * (long long)c;
          h64[idx] = 0ull;
        }
      }
    }
    __syncthreads();
  };
  int64_t r = rb + threadIdx.x;
  if (r < re) load_row(r, b8, x0, x1, lab, cd);
  else {
#pragma unroll
    for (int k = 0; k < NT; ++k) cd[k] = 0xFFu;
  }

  int iter = 0;
  for (int64_t rbase = rb; rbase < re; rbase += TH, r += TH, ++iter) {
    if (r >= re) {
#pragma unroll
      for (int k = 0; k < NT; ++k) cd[k] = 0xFFu;  // tail lanes: no work, but keep the block in step
    }
    uint64_t nb8 = 0;
    float nx0 = 1.f, nx1 = 0.f;
    int nlab = 0;
    uint32_t ncd[NT];
    const int64_t rn = r + TH;
    if (rn < re) load_row(rn, nb8, nx0, nx1, nlab, ncd);
    else {
#pragma unroll
      for (int k = 0; k < NT; ++k) ncd[k] = 0xFFu;
    }

    const uint32_t lo = (uint32_t)b8, hi = (uint32_t)(b8 >> 32);
    int cell[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      cell[j] = foff[j] + (int)__builtin_amdgcn_ubfe(fsel[j] ? hi : lo, (uint32_t)fsh[j], 8u);
    int q1 = (int)rintf(x1 * a.qs1);
    q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
    const unsigned long long qoff = (unsigned long long)(q1 + kPackQ);
    const bool row_ok = true;
    const uint32_t cbase_lab = MODE == 1 ? (uint32_t)(lab * plane) : 0u;
    if (row_ok) {
      constexpr int KB = NT;  // all slot-table reads of the row first: one LDS wait per row
#pragma unroll
      for (int kb = 0; kb < NT; kb += KB) {
        int lsk[KB];
        uint32_t mk[KB];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          lsk[k] = lt[(kb + k) * 256 + (int)(cd[kb + k] & 0xFFu)];  // -1: done / not built here
          if (MASKED) mk[k] = lmask[lsk[k] < 0 ? 0 : lsk[k]];
        }
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const int ls = lsk[k];
          if (ls < 0) continue;
          const uint32_t wv = cd[kb + k] >> 8;
          const uint32_t base = (uint32_t)(ls * slot_cells) + cbase_lab;
          uint32_t mrot = frot;
          if (MASKED) mrot &= ((mk[k] >> rot) | (mk[k] << (8 - rot))) & 0xFFu;
          const unsigned long long add = ((unsigned long long)wv << kPackShift) + (unsigned long long)wv * qoff;
          if (!MASKED && all8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) atomicAdd(h64 + base + (uint32_t)cell[j], add);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              if (!((mrot >> j) & 1u)) continue;
              atomicAdd(h64 + base + (uint32_t)cell[j], add);
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
    for (int k = 0; k < NT; ++k) cd[k] = ncd[k];
    if ((iter + 1) % drain_iters == 0) drain();
  }
  drain();
#pragma unroll
  for (int i = 0; i < kPackCells; ++i) {
    const int idx = (int)threadIdx.x + i * TH;
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



// Wave-compacted packed kernel.  An LDS atomic costs the same whatever
// fraction of the wave is active (profiles/lds_mask_bench_mi355x.txt: 16 clk
// per ds_add_u64 per CU at 64, 32 or 8 active lanes), and (row, tree) work is
// sparse: bootstrap zeros leave 37 % of lanes idle at level 0 and, below it,
// only rows of the smaller child of each sibling pair are built.  So each
// wave queues its active (row, tree) items and issues the 8 feature atomics
// only for full 64-item rounds:
//   * the row's bins word and offset value go once per row-iteration to a
//     per-wave LDS row buffer (two parities, so items of the previous
//     iteration stay readable);
//   * an item is one word (source lane | parity | weight | slot), moved into
//     queue position with one ds_permute_b32 whose destinations form a full
//     permutation (inactive lanes fill the tail positions);
//   * two register slots hold up to 127 pending items; a round drains 64.
// Leftover items of iteration i-1 are flushed (a partial round) at the end
// of iteration i before their row-buffer parity is reused.
template <bool MASKED, int NT, int TH>
__global__ __launch_bounds__(TH) void hist5q_kernel(const Hist5Args a) {
  const int drain_iters = a.drain_iters;
  constexpr int NW = TH / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = (a.d + 7) / 8;
  const int plane = a.SB * 8 * a.B;
  unsigned long long* h64 = reinterpret_cast<unsigned long long*>(smem);
  uint2* rbuf_b = reinterpret_cast<uint2*>(h64 + (size_t)plane);  // [NW][2][64] bins words
  uint32_t* rbuf_q = reinterpret_cast<uint32_t*>(rbuf_b + NW * 128);  // [NW][2][64] q + 2^23
  int16_t* lt = reinterpret_cast<int16_t*>(rbuf_q + NW * 128);
  uint8_t* lmask = reinterpret_cast<uint8_t*>(lt + NT * 256);
  const uint32_t w = cdna::xcd_remap(blockIdx.x, gridDim.x);
  const int g = (int)(w % G);
  const int grp = (int)((w / G) % a.ngroups);
  const int chunk = (int)(w / ((uint32_t)G * a.ngroups));
  const int s0 = a.grp[grp * 5 + 0], t0 = a.grp[grp * 5 + 1], t1 = a.grp[grp * 5 + 2];
  const int id1 = a.grp[grp * 5 + 4];
  const int nt = t1 - t0 + 1;
  const int fbase = g * 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rot = lane & 7;

  for (int i = threadIdx.x; i < plane; i += TH) h64[i] = 0ull;
  uint32_t acc_c[kPackCells];
  long long acc_s[kPackCells];
#pragma unroll
  for (int i = 0; i < kPackCells; ++i) {
    acc_c[i] = 0u;
    acc_s[i] = 0;
  }
  for (int i = threadIdx.x; i < NT * 256; i += TH) {
    const int k = i >> 8, loc = i & 255;
    int v = -1;
    const int id = k < nt ? a.tfirst[t0 + k] + loc : 0;
    const int idend = k + 1 < nt ? a.tfirst[t0 + k + 1] : id1;
    if (k < nt && loc != 255 && id < idend) {
      const int sl = a.build_slot[id];
      if (sl >= s0 && sl < s0 + a.SB) v = sl - s0;
    }
    lt[i] = (int16_t)v;
  }
  if (MASKED) {
    for (int i = threadIdx.x; i < a.SB; i += TH) {
      const int slot = s0 + i;
      uint32_t m = 0u;
      if (slot < a.S) m = (a.feat_mask[(int64_t)slot * a.mask_words + (fbase >> 5)] >> (fbase & 31)) & 0xFFu;
      const int valid = a.d - fbase;
      if (valid < 8) m &= (1u << (valid > 0 ? valid : 0)) - 1u;
      lmask[i] = (uint8_t)m;
    }
  }
  int fsel[8], fsh[8], foff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int jj = (j + rot) & 7;
    fsel[j] = jj >> 2;
    fsh[j] = (jj & 3) * 8;
    foff[j] = jj * a.B;
  }
  const int valid_f = a.d - fbase;
  const uint32_t fvalid = valid_f >= 8 ? 0xFFu : ((1u << (valid_f > 0 ? valid_f : 0)) - 1u);
  const uint32_t frot = ((fvalid >> rot) | (fvalid << (8 - rot))) & 0xFFu;
  const bool all8 = valid_f >= 8;  // block-uniform: no per-feature guards in the atomic rounds
  __syncthreads();

  const int64_t rb = (int64_t)chunk * a.rows_per_chunk;
  int64_t re = rb + a.rows_per_chunk;
  if (re > a.n) re = a.n;
  const int64_t n = a.n;
  const int slot_cells = 8 * a.B;
  uint2* my_b = rbuf_b + wid * 128;
  uint32_t* my_q = rbuf_q + wid * 128;

// one queue round: lanes with VALID take the item in word IT
#define H5Q_ROUND(IT, VALID)                                                                    \
  if (VALID) {                                                                                  \
    const uint32_t it_ = (IT);                                                                  \
    const int src_ = (int)(it_ & 127u);                                                         \
    const uint2 bw_ = my_b[src_];                                                               \
    const unsigned long long qo_ = my_q[src_];                                                  \
    const uint32_t wv_ = (it_ >> 7) & 255u;                                                     \
    const int ls_ = (int)(it_ >> 15);                                                           \
    uint32_t mr_ = frot;                                                                        \
    if (MASKED) {                                                                               \
      const uint32_t mk_ = lmask[ls_];                                                          \
      mr_ &= ((mk_ >> rot) | (mk_ << (8 - rot))) & 0xFFu;                                       \
    }                                                                                           \
    const unsigned long long add_ = ((unsigned long long)wv_ << kPackShift) + wv_ * qo_;        \
    unsigned long long* hb_ = h64 + ls_ * slot_cells;                                           \
    if (!MASKED && all8) {                                                                      \
      _Pragma("unroll") for (int j = 0; j < 8; ++j)                                             \
        atomicAdd(hb_ + foff[j] + (int)__builtin_amdgcn_ubfe(fsel[j] ? bw_.y : bw_.x,           \
                                                               (uint32_t)fsh[j], 8u), add_);    \
    } else {                                                                                    \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                           \
        if ((mr_ >> j) & 1u)                                                                    \
          atomicAdd(hb_ + foff[j] + (int)__builtin_amdgcn_ubfe(fsel[j] ? bw_.y : bw_.x,         \
                                                                 (uint32_t)fsh[j], 8u), add_);  \
      }                                                                                         \
    }                                                                                           \
  }

  auto drain = [&]() {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPackCells; ++i) {
      const int idx = (int)threadIdx.x + i * TH;
      if (idx < plane) {
        const unsigned long long v = h64[idx];
        if (v) {
          const uint32_t c = (uint32_t)(v >> kPackShift);
          acc_c[i] += c;
          acc_s[i] += (long long)(v & ((1ull << kPackShift) - 1ull)) - (long long)kPackQ * (long long)c;
          h64[idx] = 0ull;
        }
      }
    }
    __syncthreads();
  };

  uint64_t b8 = 0;
  float x1 = 0.f;
  uint32_t cd[NT];
  const int64_t tstride = (int64_t)n;
  int64_t r = rb + threadIdx.x;
  if (r < re) {
    b8 = a.bins[(int64_t)g * n + r];
    x1 = a.v1[r];
    const uint16_t* cp = a.codes + (int64_t)t0 * n + r;
#pragma unroll
    for (int k = 0; k < NT; ++k) cd[k] = (uint32_t)cp[(k < nt ? k : 0) * tstride];
  } else {
#pragma unroll
    for (int k = 0; k < NT; ++k) cd[k] = 0xFFu;
  }

  uint32_t qa = 0u, qb = 0u;  // queue slots: positions [0, 64) and [64, 128)
  int cnt = 0, prev = 0, par = 0;
  int iter = 0;
  for (int64_t rbase = rb; rbase < re; rbase += TH, r += TH, ++iter) {
    if (r >= re) {
#pragma unroll
      for (int k = 0; k < NT; ++k) cd[k] = 0xFFu;
    }
    uint64_t nb8 = 0;
    float nx1 = 0.f;
    uint32_t ncd[NT];
    const int64_t rn = r + TH;
    if (rn < re) {
      nb8 = a.bins[(int64_t)g * n + rn];
      nx1 = a.v1[rn];
      const uint16_t* cp = a.codes + (int64_t)t0 * n + rn;
#pragma unroll
      for (int k = 0; k < NT; ++k) ncd[k] = (uint32_t)cp[(k < nt ? k : 0) * tstride];
    } else {
#pragma unroll
      for (int k = 0; k < NT; ++k) ncd[k] = 0xFFu;
    }
    int q1 = (int)rintf(x1 * a.qs1);
    q1 = q1 > kPackQ ? kPackQ : (q1 < -kPackQ ? -kPackQ : q1);
    my_b[par * 64 + lane] = make_uint2((uint32_t)b8, (uint32_t)(b8 >> 32));
    my_q[par * 64 + lane] = (uint32_t)(q1 + kPackQ);
    int lsk[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) lsk[k] = lt[k * 256 + (int)(cd[k] & 0xFFu)];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      const bool act = lsk[k] >= 0;
      const uint64_t mask = __builtin_amdgcn_ballot_w64(act);
      if (mask == 0ull) continue;
      const int m = __builtin_popcountll(mask);
      const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
      const uint32_t item = (uint32_t)(par * 64 + lane) | (((cd[k] >> 8) & 255u) << 7) |
                            ((uint32_t)(act ? lsk[k] : 0) << 15);
      const int pos = act ? rank : m + lane - rank;
      const uint32_t rcv = (uint32_t)__builtin_amdgcn_ds_permute(((cnt + pos) & 63) * 4, (int)item);
      const int rel = (lane - cnt) & 63;
      if (rel < m) {
        if (lane >= cnt) qa = rcv;
        else qb = rcv;
      }
      cnt += m;
      if (cnt >= 64) {
        H5Q_ROUND(qa, true);
        qa = qb;
        cnt -= 64;
        prev = 0;
      }
    }
    if (prev > 0) {  // items of the previous iteration: their row-buffer parity is reused next
      H5Q_ROUND(qa, lane < cnt);
      cnt = 0;
    }
    prev = cnt;
    par ^= 1;
    b8 = nb8;
    x1 = nx1;
#pragma unroll
    for (int k = 0; k < NT; ++k) cd[k] = ncd[k];
    if ((iter + 1) % drain_iters == 0) {
      H5Q_ROUND(qa, lane < cnt);
      cnt = 0;
      prev = 0;
      drain();
    }
  }
  H5Q_ROUND(qa, lane < cnt);
  drain();
#undef H5Q_ROUND
#pragma unroll
  for (int i = 0; i < kPackCells; ++i) {
    const int idx = (int)threadIdx.x + i * TH;
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

// Row-record partition: every row moves, in every tree, from its active node to
// the chosen child (or finishes).  grid.y = tree.  The tree's split table
// (feature, bin, categorical offset, children as next-level LOCAL indices) is
// staged in LDS once per block, and each thread moves 4 consecutive rows with
// one 8-byte code load/store (v1 did 4 dependent global table loads per row:
// 11 ms per level at 1e8 x 20 trees).
__global__ __launch_bounds__(256) void partition5_kernel(const uint64_t* __restrict__ bins, int64_t n, int T, int A,
                                                         uint16_t* __restrict__ codes,
                                                         const int* __restrict__ tfirst,
                                                         const int* __restrict__ tfirst_next,
                                                         const int* __restrict__ split_feat,
                                                         const int* __restrict__ split_bin,
                                                         const int* __restrict__ cat_off,
                                                         const uint32_t* __restrict__ cat_mask,
                                                         const int* __restrict__ child, int rm_row_bytes,
                                                         const float* __restrict__ lv, float eta,
                                                         float* __restrict__ F) {
  __shared__ int s_f[256], s_b[256], s_co[256], s_ch[512];
  const int t = blockIdx.y;
  const int tf = tfirst[t];
  const int nloc = (t + 1 < T ? tfirst[t + 1] : A) - tf;  // <= 255 (host-checked via max depth)
  const int tfn = tfirst_next[t];
  for (int i = threadIdx.x; i < 256; i += 256) {
    if (i < nloc) {
      s_f[i] = split_feat[tf + i];
      s_b[i] = split_bin[tf + i];
      s_co[i] = cat_off[tf + i];
      const int c0 = child[(tf + i) * 2], c1 = child[(tf + i) * 2 + 1];
      s_ch[2 * i] = c0 >= 0 ? c0 - tfn : 0xFF;
      s_ch[2 * i + 1] = c1 >= 0 ? c1 - tfn : 0xFF;
    } else {
      s_f[i] = -1;
    }
  }
  __syncthreads();
  const uint8_t* b8 = reinterpret_cast<const uint8_t*>(bins);
  // rm_row_bytes > 0: bins is the row-major copy [n][G*8] (a row's bytes share 1-2 cache lines, so the
  // up-to-255 different split features of a tree's rows do not each pull a line of their own group);
  // rm_row_bytes < 0: bins is the feature-major byte copy [G*8][n] -- a 64-byte sector serves 64 rows of ONE
  // feature, so a level pulls only the sectors of the features its nodes split on (the [G][n] words pull the
  // sector of a row's 8-feature group for 8 rows: a deep boosting level, every group in use, read ~half of all)
  auto bidx = [&](int64_t r, int f) -> int64_t {
    return rm_row_bytes > 0 ? r * rm_row_bytes + f
                            : (rm_row_bytes < 0 ? (int64_t)f * n + r : ((int64_t)(f >> 3) * n + r) * 8 + (f & 7));
  };
  uint16_t* rec = codes + (int64_t)t * n;
  const int64_t n4 = n / 4;
  // F (boosting margins, optional): a row whose node becomes a leaf here -- a child that is a leaf, or an active
  // node that does not split -- adds eta * its leaf value (lv[2 a + side] / lv[2 A + a], split_decode's table):
  // the same fp32 update, once per row and tree, as predict_binned_kernel's walk after the tree is built
  auto leaf_add = [&](int64_t r, int e) {
    if (F) F[r] += eta * lv[e];
  };
  auto move = [&](int64_t r, uint32_t c) -> uint32_t {
    const uint32_t loc = c & 0xFFu;
    if (loc == 0xFFu) return c;
    const int f = s_f[loc];
    uint32_t nl = 0xFFu;
    if (f >= 0) {
      const int bin = b8[bidx(r, f)];
      const int co = s_co[loc];
      const bool left = co >= 0 ? ((cat_mask[co * 8 + (bin >> 5)] >> (bin & 31)) & 1u) != 0u : bin <= s_b[loc];
      nl = (uint32_t)s_ch[2 * loc + (left ? 0 : 1)];
      if (nl == 0xFFu) leaf_add(r, 2 * (tf + (int)loc) + (left ? 0 : 1));
    } else {
      leaf_add(r, 2 * A + tf + (int)loc);
    }
    return (c & 0xFF00u) | nl;
  };
  uint64_t* rec4 = reinterpret_cast<uint64_t*>(rec);
  const bool aligned = (reinterpret_cast<uintptr_t>(rec) & 7u) == 0;
  if (aligned) {
    // 4 code words (16 rows) per thread per trip: all code loads, then all bin
    // gathers, are issued before any result is consumed (the 1-word loop spent
    // 92 % of wave time waiting on memory)
    constexpr int U = 4;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t q0 = (int64_t)blockIdx.x * 256 + threadIdx.x; q0 < n4; q0 += stride * U) {
      uint64_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = q0 + u * stride < n4 ? rec4[q0 + u * stride] : 0x00FF00FF00FF00FFull;
      int bins_[U][4];
      uint32_t cs[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t c = (uint32_t)(v[u] >> (16 * k)) & 0xFFFFu;
          cs[u][k] = c;
          const uint32_t loc = c & 0xFFu;
          const int f = loc == 0xFFu ? -1 : s_f[loc];
          const int64_t r = (q0 + u * stride) * 4 + k;
          bins_[u][k] = f >= 0 ? (int)b8[bidx(r, f)] : 0;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (q0 + u * stride >= n4) continue;
        if ((v[u] & 0x00FF00FF00FF00FFull) == 0x00FF00FF00FF00FFull) continue;  // all four rows done
        uint64_t o = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t c = cs[u][k];
          const uint32_t loc = c & 0xFFu;
          uint32_t res = c;
          if (loc != 0xFFu) {
            const int f = s_f[loc];
            const int64_t r = (q0 + u * stride) * 4 + k;
            uint32_t nl = 0xFFu;
            if (f >= 0) {
              const int bin = bins_[u][k];
              const int co = s_co[loc];
              const bool left = co >= 0 ? ((cat_mask[co * 8 + (bin >> 5)] >> (bin & 31)) & 1u) != 0u
                                        : bin <= s_b[loc];
              nl = (uint32_t)s_ch[2 * loc + (left ? 0 : 1)];
              if (nl == 0xFFu) leaf_add(r, 2 * (tf + (int)loc) + (left ? 0 : 1));
            } else {
              leaf_add(r, 2 * A + tf + (int)loc);
            }
            res = (c & 0xFF00u) | nl;
          }
          o |= (uint64_t)res << (16 * k);
        }
        rec4[q0 + u * stride] = o;
      }
    }
    for (int64_t r = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256)
      rec[r] = (uint16_t)move(r, rec[r]);
  } else {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256)
      rec[r] = (uint16_t)move(r, rec[r]);
  }
}

// Row-record partition, persistent (partition7).  partition5 (grid.y = tree)
// re-gathers one byte per (row, tree) from the [G][n] planes, so 20 trees pull
// the bins planes through HBM up to 20 times per level (4.7 -> 9.5 ms per level
// at 1e8 x 20 trees as the split features diversify); partition6 fixed that
// but re-staged every split table per 256-row chunk and ran one short pass per
// block (latency-bound, 8 ms flat).  Here ~4 blocks per CU stay resident: the
// level's split tables (all trees) are staged in LDS ONCE per block, and each
// thread owns one row per trip: its G bins words are read with coalesced
// 8-byte loads (once per level), parked in the thread's own LDS column (no
// block barrier), and the row's codes of up to kP7TB trees are all in flight
// before any is moved.
constexpr int kP7MaxA = 1024;
constexpr int kP7MaxT = 64;
constexpr int kP7MaxG = 16;  // MAXG template: 8 / 13 / 16 words per row (registers sized to the row)
constexpr int kP7TB = 24;

// (A variant that also wrote the next level's item records from the partition -- "EMIT", record emission --
// measured 172.7 vs 138.9 ms per headline step and was removed: profiles/r4/emission_ab.md.)
template <int MAXG>
__global__ __launch_bounds__(256, 4) void partition7_kernel(const uint64_t* __restrict__ bins, int64_t n, int G, int T,
                                                         int A, uint16_t* __restrict__ codes,
                                                         const int* __restrict__ tfirst,
                                                         const int* __restrict__ tfirst_next,
                                                         const int* __restrict__ split_feat,
                                                         const int* __restrict__ split_bin,
                                                         const int* __restrict__ cat_off,
                                                         const uint32_t* __restrict__ cat_mask,
                                                         const int* __restrict__ child) {
  extern __shared__ __attribute__((aligned(16))) uint64_t tile7[];  // [G][256]
  // numeric: feature (0xFFFF: leaf) | bin << 16; categorical / bin-set split: feature | cat_off << 16 | 1 << 31
  __shared__ int s_fb[kP7MaxA];
  __shared__ uint8_t s_ch[2 * kP7MaxA];
  __shared__ int s_tf[kP7MaxT];
  __shared__ uint32_t s_gmask;  // the bins words (8-feature groups) some split of the level reads
  if (threadIdx.x == 0) s_gmask = 0u;
  for (int i = threadIdx.x; i < T; i += 256) s_tf[i] = tfirst[i];
  __syncthreads();
  uint32_t gm = 0u;
  for (int i = threadIdx.x; i < A; i += 256) {
    const int f = split_feat[i];
    if (f >= 0 && (f >> 3) < G) gm |= 1u << (f >> 3);
    const int co = cat_off[i];
    s_fb[i] = f < 0 ? 0xFFFF : (co >= 0 ? (f | (co << 16) | (int)0x80000000) : (f | (split_bin[i] << 16)));
    int lo = 0, hi = T - 1;  // the tree of active node i: largest t with tfirst[t] <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tfirst[mid] <= i) lo = mid; else hi = mid - 1;
    }
    const int tfn = tfirst_next[lo];
    const int c0 = child[i * 2], c1 = child[i * 2 + 1];
    s_ch[2 * i] = (uint8_t)(c0 >= 0 ? c0 - tfn : 0xFF);
    s_ch[2 * i + 1] = (uint8_t)(c1 >= 0 ? c1 - tfn : 0xFF);
  }
  if (gm) atomicOr(&s_gmask, gm);
  __syncthreads();
  // only the words some split reads are loaded and parked (shallow levels split on a few of the 13 groups:
  // every skipped word is n x 8 bytes less HBM traffic per level); the mask is block-uniform
  const uint32_t gmask = __builtin_amdgcn_readfirstlane(s_gmask);
  const uint8_t* tb = reinterpret_cast<const uint8_t*>(tile7);
  const int lr = threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * 256;
  // one row: park its bins words in this thread's LDS column (no barrier), move every tree's code
  auto move_row = [&](int64_t r, const uint64_t (&w)[MAXG], const uint32_t (&cc)[kP7TB], bool live) {
    uint32_t c[kP7TB];
#pragma unroll
    for (int u = 0; u < kP7TB; ++u) c[u] = cc[u] & 0xFFFFu;
    if (live) {
#pragma unroll
      for (int g = 0; g < MAXG; ++g)
        if (g < G && ((gmask >> g) & 1u)) tile7[g * 256 + lr] = w[g];
    }
    for (int t0 = 0; t0 < T; t0 += kP7TB) {
      if (t0 > 0 && live) {
#pragma unroll
        for (int u = 0; u < kP7TB; ++u) c[u] = t0 + u < T ? (uint32_t)codes[(int64_t)(t0 + u) * n + r] : 0xFFu;
      }
#pragma unroll
      for (int u = 0; u < kP7TB; ++u) {
        if (t0 + u >= T) break;  // uniform
        const uint32_t loc = c[u] & 0xFFu;
        if (live && loc != 0xFFu) {
          const int id = s_tf[t0 + u] + (int)loc;
          if (CDNA_DCHECK(id >= 0 && id < A, 0x9701u)) {  // code's local node outside the level
            const int fb = s_fb[id];
            const int f = fb & 0xFFFF;
            uint32_t nl = 0xFFu;
            if (f != 0xFFFF && CDNA_DCHECK((f >> 3) < G, 0x9702u)) {
              const int bin = tb[((f >> 3) * 256 + lr) * 8 + (f & 7)];
              const bool left = fb < 0 ? ((cat_mask[((fb >> 16) & 0x7FFF) * 8 + (bin >> 5)] >> (bin & 31)) & 1u) != 0u
                                       : bin <= ((fb >> 16) & 0xFF);
              nl = s_ch[2 * id + (left ? 0 : 1)];
            }
            codes[(int64_t)(t0 + u) * n + r] = (uint16_t)((c[u] & 0xFF00u) | nl);
          }
        }
      }
    }
  };
  auto load_row = [&](int64_t r, uint64_t (&w)[MAXG], uint32_t (&cc)[kP7TB]) {
#pragma unroll
    for (int g = 0; g < MAXG; ++g)
      if (g < G && ((gmask >> g) & 1u)) w[g] = bins[(int64_t)g * n + r];
#pragma unroll
    for (int u = 0; u < kP7TB; ++u) cc[u] = u < T ? (uint32_t)codes[(int64_t)u * n + r] : 0xFFu;
  };
  // software-pipelined: the next trip's bins words and codes are in flight while this row's codes move
  // (the one-stage loop waited on every trip's loads: 82 % of wave time on memory at ~3.8 TB/s, 19.6 ms per
  // headline step; pipelined at 120 VGPRs / 4 waves per SIMD: 13.2 ms).
  int64_t r = (int64_t)blockIdx.x * 256 + lr;
  uint64_t w[MAXG];
  uint32_t cc[kP7TB];
  if (r < n) load_row(r, w, cc);
  const int64_t rw = r - lane;  // the wave's first row this trip
  for (int64_t rb = rw; rb < n; rb += stride, r += stride) {
    uint64_t wn[MAXG];
    uint32_t cn[kP7TB];
    const int64_t rn = r + stride;
    if (rn < n) load_row(rn, wn, cn);
    move_row(r, w, cc, r < n);
#pragma unroll
    for (int g = 0; g < MAXG; ++g) w[g] = wn[g];
#pragma unroll
    for (int u = 0; u < kP7TB; ++u) cc[u] = cn[u];
  }
}

inline unsigned grid_for(int64_t n, int per, unsigned cap) {
  int64_t b = (n + per - 1) / per;
  return (unsigned)(b < (int64_t)cap ? (b < 1 ? 1 : b) : cap);
}

template <int MODE, bool MASKED, bool V0>
void launch5(const Hist5Args& a, int nt_max, unsigned nblk, size_t lds, hipStream_t st) {
  if (nt_max <= 1) hipLaunchKernelGGL((hist5_kernel<MODE, MASKED, V0, 1>), dim3(nblk), dim3(kThreads), lds, st, a);
  else if (nt_max <= 2)
    hipLaunchKernelGGL((hist5_kernel<MODE, MASKED, V0, 2>), dim3(nblk), dim3(kThreads), lds, st, a);
  else if (nt_max <= 4)
    hipLaunchKernelGGL((hist5_kernel<MODE, MASKED, V0, 4>), dim3(nblk), dim3(kThreads), lds, st, a);
  else if (nt_max <= 8)
    hipLaunchKernelGGL((hist5_kernel<MODE, MASKED, V0, 8>), dim3(nblk), dim3(kThreads), lds, st, a);
  else
    hipLaunchKernelGGL((hist5_kernel<MODE, MASKED, V0, 16>), dim3(nblk), dim3(kThreads), lds, st, a);
}

template <typename K>
void go(K kern, unsigned nblk, int th, size_t lds, hipStream_t st, const Hist5Args& a) {
  // blocks above 64 KB of dynamic LDS must opt in (gfx950 has 160 KB per CU)
  if (lds > 64 * 1024) hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(th), lds, st, a);
}

template <bool MASKED, int TH>
void launch5p_t(const Hist5Args& a, int nt_max, unsigned nblk, size_t lds, hipStream_t st) {
  if (nt_max <= 1) go(hist5p_kernel<MASKED, 1, TH>, nblk, TH, lds, st, a);
  else if (nt_max <= 2) go(hist5p_kernel<MASKED, 2, TH>, nblk, TH, lds, st, a);
  else if (nt_max <= 4) go(hist5p_kernel<MASKED, 4, TH>, nblk, TH, lds, st, a);
  else if (nt_max <= 8) go(hist5p_kernel<MASKED, 8, TH>, nblk, TH, lds, st, a);
  else go(hist5p_kernel<MASKED, 16, TH>, nblk, TH, lds, st, a);
}

// 1024-thread blocks hold 16384 packed cells (128 KB): one block per CU with
// the same 16 waves as two 512-thread blocks, but twice the slots per pass.
template <bool MASKED>
void launch5p(const Hist5Args& a, int nt_max, unsigned nblk, size_t lds, bool big, hipStream_t st) {
  if (big) launch5p_t<MASKED, 1024>(a, nt_max, nblk, lds, st);
  else launch5p_t<MASKED, 512>(a, nt_max, nblk, lds, st);
}

template <bool MASKED, int TH>
void launch5q_t(const Hist5Args& a, int nt_max, unsigned nblk, size_t lds, hipStream_t st) {
  if (nt_max <= 1) go(hist5q_kernel<MASKED, 1, TH>, nblk, TH, lds, st, a);
  else if (nt_max <= 2) go(hist5q_kernel<MASKED, 2, TH>, nblk, TH, lds, st, a);
  else if (nt_max <= 4) go(hist5q_kernel<MASKED, 4, TH>, nblk, TH, lds, st, a);
  else if (nt_max <= 8) go(hist5q_kernel<MASKED, 8, TH>, nblk, TH, lds, st, a);
  else go(hist5q_kernel<MASKED, 16, TH>, nblk, TH, lds, st, a);
}

// compacted kernel: always 1024-thread blocks (16 waves per CU; a 512-thread
// block at >128 VGPRs would run 8)
template <bool MASKED>
void launch5q(const Hist5Args& a, int nt_max, unsigned nblk, size_t lds, hipStream_t st) {
  launch5q_t<MASKED, 1024>(a, nt_max, nblk, lds, st);
}

inline int nt_bucket(int nt) { return nt <= 1 ? 1 : nt <= 2 ? 2 : nt <= 4 ? 4 : nt <= 8 ? 8 : 16; }

}  // namespace

CDNA_API int cdna_hist5_max_trees() { return kMaxTrees; }

// mode bit0: classes; bit2: v0 present; bit4: packed single-atomic regression
// (|v * qs1| <= 2^23, plane <= 16384 cells); bit6 (with bit4): wave-compacted
// packed kernel.  grp rows must satisfy t1 - t0 < 16;
// `id_span_max` = max trees per group (sizes the LDS local -> slot tables).
CDNA_API int cdna_hist5(int mode, const uint64_t* bins, int64_t n, int d, int T, const uint16_t* codes,
                        const int* tfirst, const float* v0, const float* v1, const int* label, int C,
                        const int* build_slot, const uint32_t* feat_mask, int mask_words, int S, int B, int SB,
                        const int* grp, int ngroups, int nchunk, int id_span_max, float qs0, float qs1, int wmax,
                        unsigned long long* out, hipStream_t st) {
  if (n <= 0 || S <= 0) return 0;
  Hist5Args a;
  a.bins = bins;
  a.n = n;
  a.d = d;
  a.T = T;
  a.codes = codes;
  a.tfirst = tfirst;
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
  if (a.rows_per_chunk * 255 >= (int64_t)1 << 32) return (int)hipErrorInvalidValue;
  a.qs0 = qs0;
  a.qs1 = qs1;
  a.out = out;
  const int G = (d + 7) / 8;
  const size_t plane = (size_t)SB * 8 * B;
  // id_span_max carries the max trees per group here (local -> slot tables of 256 int16 each)
  const size_t lds = plane * 8 * a.n64 + ((plane * a.n32 + 3) & ~(size_t)3) * 4 +
                     (size_t)nt_bucket(id_span_max) * 512 + SB + 16;
  if (id_span_max > kMaxTrees) return (int)hipErrorInvalidValue;
  if (lds > 160 * 1024 && !(mode & 16)) return (int)hipErrorInvalidValue;
  const unsigned nblk = (unsigned)G * ngroups * nchunk;
  const bool masked = feat_mask != nullptr;
  const int ntm = id_span_max;
  if (mode & 16) {  // packed single-atomic regression
    const bool compact = (mode & 64) != 0;
    const bool big = compact || plane > (size_t)kPackCells * 512;
    {
      const int th = big ? 1024 : 512;
      const int64_t rows_ok = ((int64_t)1 << 20) / (wmax > 0 ? wmax + 1 : 1);  // rows * wmax < 2^20
      a.drain_iters = (int)(rows_ok / th > 0 ? rows_ok / th : 1);
    }
    if (classes || has_v0 || plane > (size_t)kPackCells * 1024) return (int)hipErrorInvalidValue;
    a.n64 = 1;
    a.n32 = 0;
    const size_t rbuf = compact ? (size_t)16 * 128 * 12 : 0;  // per-wave row buffers
    const size_t lds_p = plane * 8 + rbuf + (size_t)nt_bucket(ntm) * 512 + SB + 16;
    if (lds_p > 160 * 1024) return (int)hipErrorInvalidValue;
    if (compact) {
      if (masked) launch5q<true>(a, ntm, nblk, lds_p, st);
      else launch5q<false>(a, ntm, nblk, lds_p, st);
    } else {
      if (masked) launch5p<true>(a, ntm, nblk, lds_p, big, st);
      else launch5p<false>(a, ntm, nblk, lds_p, big, st);
    }
    return (int)hipGetLastError();
  }
  if (classes) {
    if (masked) launch5<1, true, false>(a, ntm, nblk, lds, st);
    else launch5<1, false, false>(a, ntm, nblk, lds, st);
  } else if (has_v0) {
    if (masked) launch5<0, true, true>(a, ntm, nblk, lds, st);
    else launch5<0, false, true>(a, ntm, nblk, lds, st);
  } else {
    if (masked) launch5<0, true, false>(a, ntm, nblk, lds, st);
    else launch5<0, false, false>(a, ntm, nblk, lds, st);
  }
  return (int)hipGetLastError();
}

// Blocks of a partition7 launch over n rows.
static unsigned p7_grid(int64_t n, int G) {
  size_t lds = (size_t)G * 256 * 8;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int per_cu = 0;
  const void* k = G <= 8 ? reinterpret_cast<const void*>(partition7_kernel<8>)
                          : G <= 13 ? reinterpret_cast<const void*>(partition7_kernel<13>)
                                    : reinterpret_cast<const void*>(partition7_kernel<16>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, lds) != hipSuccess || per_cu < 1) per_cu = 2;
  // exactly the resident blocks (one round): a 4-per-CU grid with only 3 resident per CU (LDS) ran a
  // second, quarter-full round
  return grid_for(n, 256, (unsigned)(per_cu * ncu));
}

CDNA_API int cdna_partition7(const uint64_t* bins, int64_t n, int G, int T, int A, uint16_t* codes,
                             const int* tfirst, const int* tfirst_next, const int* split_feat, const int* split_bin,
                             const int* cat_off, const uint32_t* cat_mask, const int* child, hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  if (G <= 0 || G > kP7MaxG || A > kP7MaxA || T > kP7MaxT || G * 8 > 0xFFFF) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)G * 256 * 8;
  const dim3 grid(p7_grid(n, G));
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, bins, n, G, T, A, codes, tfirst, tfirst_next, split_feat,
                       split_bin, cat_off, cat_mask, child);
  };
  if (G <= 8) launch(partition7_kernel<8>);
  else if (G <= 13) launch(partition7_kernel<13>);
  else launch(partition7_kernel<16>);
  return (int)hipGetLastError();
}

// lv / eta / F (optional, F null: off): boosting margins updated by the rows that finish at this level.
CDNA_API int cdna_partition5(const uint64_t* bins, int64_t n, int T, int A, uint16_t* codes, const int* tfirst,
                             const int* tfirst_next, const int* split_feat, const int* split_bin, const int* cat_off,
                             const uint32_t* cat_mask, const int* child, int rm_row_bytes, const float* lv, float eta,
                             float* F, hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  if (F && !lv) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(partition5_kernel, dim3(grid_for(n / 4 + 1, 256, 1024), T), dim3(256), 0, st, bins, n, T, A,
                     codes, tfirst,
                     tfirst_next, split_feat, split_bin, cat_off, cat_mask, child, rm_row_bytes, lv, eta, F);
  return (int)hipGetLastError();
}

CDNA_DEBUG_EXPORT(hist5)
