// K5m: forest level histograms on the matrix cores (v_mfma_i32_16x16x64_i8).
//
// At the shallow levels of a random forest every tree builds at most a few
// nodes and (almost) every row of the shard is in one of them, so the level's
// histograms are one dense GEMM over the rows:
//
//     H[(f, b), (s, j)] = sum_r  onehot[r, (f, b)]  *  limb_j(w_s(r) * q(r))
//
// with M = cells (feature f, bin b), N = (built slot s, statistic limb j), and
// K = rows.  The statistics are the packed fixed-point pair of the LDS-atomic
// kernels (seg.hip): count = sum w and sum = sum w * q, q = clamp(rint(v1 *
// qs1), +-2^23), w = the row's bootstrap weight in slot s's tree if the row is
// in slot s's node, else 0.  |w * q| < 2^30 for w <= 127, so it splits into
// four balanced base-256 int8 limbs; with the count limb that is 5 columns per
// slot.  int32 MFMA accumulators are exact over a block's rows (<= 2^24 rows x
// |limb| <= 128) and the finalize kernel recombines the limbs in int64: the
// result is BIT-IDENTICAL to seg_hist(raw=True) (tests/test_kernels_gpu.py).
//
// Per K-step of 64 rows a wave (one feature) builds its A fragments from 16
// planar bins bytes per lane with 3 SWAR ops per dword (byte == cell), reads
// the shared B fragments (built once per 256-row stage by the whole block into
// a double-buffered, XOR-swizzled LDS tile) and issues BT x NT MFMAs.  No LDS
// atomics, no per-level row compaction: the level costs one pass over the
// planar bins + the row records, ~5x fewer cycles than the atomic histogram at
// 20 trees (profiles/r2/).
//
// Operand maps: lane l supplies A[m = l & 15][k in group l >> 4] and
// B[k in group l >> 4][n = l & 15]; the 16 bytes a lane holds are 16 rows of
// its K group.  A and B use the same (lane group, byte) <-> k assignment, so
// the contraction is exact whatever the hardware's internal K order (verified
// against the int64 reference).  C/D: col = l & 15, row = (l >> 4) * 4 + i.
#include "common.h"

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int kStageRows = 512;   // rows per LDS stage = 8 K-steps of 64 (enough MFMA work per stage to cover
                                  // the next stage's row-record / label / bins loads, issued at its start)
constexpr int kKSteps = kStageRows / 64;
constexpr int kQuads = kStageRows / 4;  // row quads per stage
constexpr int kRowBytes = kStageRows;   // LDS bytes per B column per stage (16-B chunks, low 4 bits swizzled)

struct MfmaHistArgs {
  const uint8_t* bp;      // planar bins [d][ldp]
  int64_t ldp;            // planar row stride (>= n rounded up to 64, 16-B aligned)
  int64_t n;
  int d, B;
  const uint16_t* codes;  // [T][n] row records: weight << 8 | local node (0xFF: done)
  const int* col_tree;    // [NS] tree of slot column group s
  const int* col_loc;     // [NS] local node (within its tree) of slot s
  int NS;                 // slot column groups in this pass (columns 5s .. 5s + 4)
  const float* v1;        // [n] statistic (label)
  float qs1;              // fixed-point scale
  int64_t chunk;          // rows per block (multiple of kStageRows)
  int nchunks, nfg, fpb;  // row chunks, feature groups, features (waves) per block
  unsigned long long* acc;  // [d][BT*16][NT*16] int64 limb sums (zeroed)
};

__device__ __forceinline__ uint32_t eq_bytes(uint32_t v, uint32_t pat) {
  // bins and cells < 128: x = v ^ pat has bytes <= 127, x + 0x7F never carries across bytes and sets
  // bit 7 of a byte iff it is nonzero -> 0x01 in every byte where v == cell (v_xad_u32, shift, v_bfi_b32)
  const uint32_t t = (v ^ pat) + 0x7F7F7F7Fu;
  return ~(t >> 7) & 0x01010101u;
}

// B stage: columns 5s + j (j = 0 count, 1..4 digits of w * q) for the stage's 256 rows, written as dwords of 4
// rows into the swizzled tile: column c, 16-B chunk q of the stage lives at chunk (q ^ (c & 15)).
//
// Digits: x' = w * q + C with C = 0x80808080 lies in [0, 2^32) (|w * q| < 2^30), and its bytes XOR 0x80 are
// signed digits s_j = byte_j(x') - 128 with sum_j 256^j s_j = x' - C = w * q.  A row outside the slot's node
// has w = 0, so x' = C and all its digits are 0: no select, and the byte transpose of 4 rows is 3 v_perm per
// output dword.  Split in two so the global loads of stage s + 1 are in flight under stage s's MFMAs: a thread
// owns row quad rq = tid % 64 of the stage and the slots s = tid / 64 + k * (threads / 64).
constexpr int kMaxSlotsPerThread = 7;  // 25 slots over 512 / kQuads = 4 thread groups

struct StageLoads {
  float v[4];
  uint32_t c[kMaxSlotsPerThread][4];  // raw row records; nothing is combined at load time, so no wait is forced
};

// Unconditional loads at clamped rows (rows past the chunk end are masked in stage_store): no divergent
// branches, so every load of the stage is in flight at once and nothing waits until stage_store.
__device__ __forceinline__ void stage_load(const MfmaHistArgs& a, StageLoads& L, const int (&tk)[kMaxSlotsPerThread],
                                           int64_t r0, int tid) {
  const int rq = tid % kQuads;
  const int64_t row = r0 + 4 * rq;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t rr = row + r < a.n ? row + r : a.n - 1;
    L.v[r] = a.v1[rr];
#pragma unroll
    for (int k = 0; k < kMaxSlotsPerThread; ++k)
      L.c[k][r] = (uint32_t)a.codes[(int64_t)tk[k] * a.n + rr];  // tk = 0 for unused slots (ignored)
  }
}

__device__ __forceinline__ void stage_store(const MfmaHistArgs& a, const StageLoads& L,
                                            const int (&lk)[kMaxSlotsPerThread], uint8_t* bt, int64_t r0,
                                            int64_t r1, int tid, int nth) {
  const int rq = tid % kQuads, s0 = __builtin_amdgcn_readfirstlane(tid / kQuads), sstep = nth / kQuads;
  const int64_t row = r0 + 4 * rq;
  int q[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int v = (int)rintf(L.v[r] * a.qs1);
    q[r] = v > (1 << 23) ? (1 << 23) : (v < -(1 << 23) ? -(1 << 23) : v);
  }
  const int chunk = rq >> 2, within = (rq & 3) * 4;
#pragma unroll
  for (int k = 0; k < kMaxSlotsPerThread; ++k) {
    const int s = s0 + k * sstep;
    if (s >= a.NS) break;
    const uint32_t loc = (uint32_t)lk[k];
    uint32_t x[4], w[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t c = L.c[k][r];
      w[r] = ((c & 0xFFu) == loc && row + r < r1) ? ((c >> 8) & 0xFFu) : 0u;
      x[r] = ((uint32_t)((int)w[r] * q[r]) + 0x80808080u) ^ 0x80808080u;
    }
    uint32_t vals[5];
    vals[0] = w[0] | (w[1] << 8) | (w[2] << 16) | (w[3] << 24);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // byte j of x[0..3] -> bytes 0..3 (v_perm: selector bytes 0-3 pick src1, 4-7 pick src0)
      const uint32_t lo = __builtin_amdgcn_perm(x[1], x[0], (uint32_t)(j | ((4 + j) << 8)) | 0x0C0C0000u);
      const uint32_t hi = __builtin_amdgcn_perm(x[3], x[2], (uint32_t)(j | ((4 + j) << 8)) | 0x0C0C0000u);
      vals[1 + j] = lo | (hi << 16);
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int c = 5 * s + j;
      *reinterpret_cast<uint32_t*>(bt + c * kRowBytes + ((chunk ^ (c & 15)) << 4) + within) = vals[j];
    }
  }
}

template <int BT, int NT>
__global__ __launch_bounds__(512, 2) void hist_mfma_kernel(const MfmaHistArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int NC = NT * 16;
  uint8_t* buf0 = lds;
  uint8_t* buf1 = lds + NC * kRowBytes;
  const int nb = a.nchunks * a.nfg;
  // XCD-aware order: hardware dispatches block b to XCD b % 8; consecutive blocks of one XCD take
  // consecutive logical items, so the feature groups of a row chunk run together on one XCD and share
  // the chunk's row records / labels through its L2
  const int per_x = (int)((gridDim.x + 7) / 8);
  const int logical = (int)(blockIdx.x % 8) * per_x + (int)(blockIdx.x / 8);
  if (logical >= nb) return;
  const int ch = logical / a.nfg, fg = logical - ch * a.nfg;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nth = blockDim.x;
  const int f = fg * a.fpb + wave;
  const bool fok = f < a.d;
  const int64_t c0 = (int64_t)ch * a.chunk;
  const int64_t c1 = (c0 + a.chunk < a.n) ? c0 + a.chunk : a.n;
  // columns past 5 * NS stay zero in both buffers
  for (int i = threadIdx.x; i < 2 * NC * kRowBytes / 16; i += nth) reinterpret_cast<uint4*>(lds)[i] = uint4{0, 0, 0, 0};
  __syncthreads();
  i32x4 acc[BT][NT];
#pragma unroll
  for (int ct = 0; ct < BT; ++ct)
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[ct][u] = i32x4{0, 0, 0, 0};
  const int ncol = lane & 15, kq = lane >> 4;
  uint32_t pat[BT];
#pragma unroll
  for (int ct = 0; ct < BT; ++ct) pat[ct] = (uint32_t)(ct * 16 + ncol) * 0x01010101u;
  const uint8_t* fb = a.bp + (int64_t)(fok ? f : 0) * a.ldp + kq * 16;
  const int nst = (int)((c1 - c0 + kStageRows - 1) / kStageRows);
  // this thread's slots (fixed for the kernel): tree and local node (slots >= NS are loaded and ignored)
  int tk[kMaxSlotsPerThread], lk[kMaxSlotsPerThread];
  {
    const int s0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kQuads), sstep = nth / kQuads;
#pragma unroll
    for (int k = 0; k < kMaxSlotsPerThread; ++k) {
      const int s = s0 + k * sstep;
      tk[k] = s < a.NS ? a.col_tree[s] : 0;
      lk[k] = s < a.NS ? a.col_loc[s] : 0;
    }
  }
  StageLoads L;
  uint4 araw[kKSteps], anext[kKSteps];
  if (nst > 0) {
    stage_load(a, L, tk, c0, threadIdx.x);
#pragma unroll
    for (int ks = 0; ks < kKSteps; ++ks) araw[ks] = *reinterpret_cast<const uint4*>(fb + c0 + ks * 64);
    stage_store(a, L, lk, buf0, c0, c1, threadIdx.x, nth);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int64_t r0 = c0 + (int64_t)st * kStageRows;
    const bool more = st + 1 < nst;
    const uint8_t* cur = (st & 1) ? buf1 : buf0;
    // stage st + 1: global loads in flight under this stage's MFMAs
    if (more) {
      stage_load(a, L, tk, r0 + kStageRows, threadIdx.x);
#pragma unroll
      for (int ks = 0; ks < kKSteps; ++ks) anext[ks] = *reinterpret_cast<const uint4*>(fb + r0 + kStageRows + ks * 64);
    }
    if (fok) {
      // B fragments of K-step ks + 1 are read from LDS while the MFMAs of K-step ks run (LDS latency hidden
      // behind BT * NT MFMAs instead of BT)
      i32x4 bcur[NT], bnxt[NT];
#pragma unroll
      for (int u = 0; u < NT; ++u)
        bcur[u] = *reinterpret_cast<const i32x4*>(cur + (u * 16 + ncol) * kRowBytes + (((0 * 4 + kq) ^ ncol) << 4));
#pragma unroll
      for (int ks = 0; ks < kKSteps; ++ks) {
        if (ks + 1 < kKSteps) {
          const int chunk = (ks + 1) * 4 + kq;
#pragma unroll
          for (int u = 0; u < NT; ++u)
            bnxt[u] = *reinterpret_cast<const i32x4*>(cur + (u * 16 + ncol) * kRowBytes + ((chunk ^ ncol) << 4));
        }
        i32x4 af[BT];
#pragma unroll
        for (int ct = 0; ct < BT; ++ct) {
          af[ct] = i32x4{(int)eq_bytes(araw[ks].x, pat[ct]), (int)eq_bytes(araw[ks].y, pat[ct]),
                         (int)eq_bytes(araw[ks].z, pat[ct]), (int)eq_bytes(araw[ks].w, pat[ct])};
        }
#pragma unroll
        for (int u = 0; u < NT; ++u)
#pragma unroll
          for (int ct = 0; ct < BT; ++ct)
            acc[ct][u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[ct], bcur[u], acc[ct][u], 0, 0, 0);
        if (ks + 1 < kKSteps) {
#pragma unroll
          for (int u = 0; u < NT; ++u) bcur[u] = bnxt[u];
        }
      }
    }
    if (more) {
      stage_store(a, L, lk, (st & 1) ? buf0 : buf1, r0 + kStageRows, c1, threadIdx.x, nth);
#pragma unroll
      for (int ks = 0; ks < kKSteps; ++ks) araw[ks] = anext[ks];
    }
    __syncthreads();
  }
  if (!fok) return;
  const int cols = 5 * a.NS;
#pragma unroll
  for (int ct = 0; ct < BT; ++ct)
#pragma unroll
    for (int u = 0; u < NT; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cell = ct * 16 + kq * 4 + i, col = u * 16 + ncol;
        const int v = acc[ct][u][i];
        if (v != 0 && cell < a.B && col < cols)
          atomicAdd(a.acc + ((int64_t)f * (BT * 16) + cell) * NC + col, (unsigned long long)(long long)v);
      }
}

// [d][BT*16][NC] limb sums -> out[slot][d][B][2] = (count, sum w * q) int64 (every (slot, f, b) once)
__global__ __launch_bounds__(256) void hist_mfma_finalize(const unsigned long long* __restrict__ acc, int d, int B,
                                                          int Bp, int NC, int NS, const int* __restrict__ slot_of,
                                                          long long* __restrict__ out) {
  const int64_t total = (int64_t)NS * d * B;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int s = (int)(i / ((int64_t)d * B));
    const int rem = (int)(i - (int64_t)s * d * B);
    const int f = rem / B, b = rem - f * B;
    const long long* p = reinterpret_cast<const long long*>(acc) + ((int64_t)f * Bp + b) * NC + 5 * s;
    const long long cnt = p[0];
    // signed digits of (w * q + C) ^ 0x80 per byte: sum_j 256^j digit_j = sum w * q
    const long long sum = p[1] + p[2] * 256ll + p[3] * 65536ll + p[4] * 16777216ll;
    long long* o = out + (((int64_t)slot_of[s] * d + f) * B + b) * 2;
    o[0] = cnt;
    o[1] = sum;
  }
}

// Planar bins [d][ldp] from the feature-group layout [G][n][8]: a thread transposes 16 rows x 8 features in
// registers (v_perm byte gathers) and stores 8 x 16 B.
__global__ __launch_bounds__(256) void planar_bins_kernel(const uint64_t* __restrict__ bins, int64_t n, int d,
                                                          int64_t ldp, uint8_t* __restrict__ out) {
  const int G = (d + 7) / 8;
  const int64_t nq = (n + 15) / 16;
  for (int64_t task = (int64_t)blockIdx.x * 256 + threadIdx.x; task < nq * G; task += (int64_t)gridDim.x * 256) {
    const int g = (int)(task / nq);
    const int64_t q = task - (int64_t)g * nq;
    const int64_t r0 = q * 16;
    uint32_t lo[16], hi[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint64_t w = (r0 + r < n) ? bins[(int64_t)g * n + r0 + r] : 0ull;
      lo[r] = (uint32_t)w;
      hi[r] = (uint32_t)(w >> 32);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = g * 8 + j;
      if (f >= d) break;
      const int sh = (j & 3) * 8;
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t v = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) v |= ((((j < 4) ? lo[4 * k + r] : hi[4 * k + r]) >> sh) & 0xFFu) << (8 * r);
        o[k] = v;
      }
      *reinterpret_cast<uint4*>(out + (int64_t)f * ldp + r0) = uint4{o[0], o[1], o[2], o[3]};
    }
  }
}

template <int BT, int NT>
int launch_mfma(const MfmaHistArgs& a, int nblocks, int threads, hipStream_t st) {
  const size_t lds = (size_t)2 * NT * 16 * kRowBytes;
  hipLaunchKernelGGL((hist_mfma_kernel<BT, NT>), dim3(nblocks), dim3(threads), lds, st, a);
  return (int)hipGetLastError();
}

}  // namespace

// Planar copy of the bins (row stride ldp >= n rounded up to 16; rows past n are left unwritten except the
// 16-row tail block: the MFMA kernel reads them under zero weights).
CDNA_API int cdna_planar_bins(const uint64_t* bins, int64_t n, int d, int64_t ldp, uint8_t* out, hipStream_t st) {
  if (n <= 0 || d <= 0) return 0;
  if (ldp < ((n + 15) / 16) * 16 || (ldp % 16) != 0) return (int)hipErrorInvalidValue;
  const int G = (d + 7) / 8;
  const int64_t tasks = ((n + 15) / 16) * G;
  int64_t grid = (tasks + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(planar_bins_kernel, dim3((unsigned)grid), dim3(256), 0, st, bins, n, d, ldp, out);
  return (int)hipGetLastError();
}

// One pass over NS <= 25 slot column groups.  BT / NT: cell / column tiles (the host rounds them up to an
// instantiated pair, cdnaml/ops/kernels.py:_mfma_tiles).  acc: [d][BT*16][NT*16] u64 scratch (zeroed by the
// caller); out: [S][d][B][2] int64, the slots of this pass written by the finalize kernel.  bp: planar bins
// with ldp a multiple of 256 and >= n rounded up to 256 (stages read whole 256-row blocks).
CDNA_API int cdna_hist_mfma(const uint8_t* bp, int64_t ldp, int64_t n, int d, int B, int BT, int NT,
                            const uint16_t* codes, const int* col_tree, const int* col_loc, const int* slot_of,
                            int NS, const float* v1, float qs1, int64_t chunk, int fpb, unsigned long long* acc,
                            long long* out, hipStream_t st) {
  if (NS <= 0 || d <= 0) return 0;
  if (B > BT * 16 || 5 * NS > NT * 16 || B > 128 || fpb != 8 || NS > 25 || chunk % kStageRows != 0 ||
      chunk > (1 << 24) || chunk <= 0) {
    return (int)hipErrorInvalidValue;
  }
  if (ldp % kStageRows != 0 || ldp < ((n + kStageRows - 1) / kStageRows) * kStageRows) return (int)hipErrorInvalidValue;
  MfmaHistArgs a;
  a.bp = bp;
  a.ldp = ldp;
  a.n = n;
  a.d = d;
  a.B = B;
  a.codes = codes;
  a.col_tree = col_tree;
  a.col_loc = col_loc;
  a.NS = NS;
  a.v1 = v1;
  a.qs1 = qs1;
  a.chunk = chunk;
  a.nchunks = (int)((n + chunk - 1) / chunk);
  a.fpb = fpb;
  a.nfg = (d + fpb - 1) / fpb;
  a.acc = acc;
  const int nb = a.nchunks * a.nfg;
  const int grid = ((nb + 7) / 8) * 8;
  const int threads = 64 * fpb;
  int e = 0;
  if (n > 0) {
#define CDNA_MFMA_CASE(bt, nt) \
  if (BT == bt && NT == nt) e = launch_mfma<bt, nt>(a, grid, threads, st); else
#define CDNA_MFMA_BT(bt) CDNA_MFMA_CASE(bt, 2) CDNA_MFMA_CASE(bt, 4) CDNA_MFMA_CASE(bt, 6) CDNA_MFMA_CASE(bt, 7) \
  CDNA_MFMA_CASE(bt, 8)
    CDNA_MFMA_BT(2) CDNA_MFMA_BT(3) CDNA_MFMA_BT(4) { return (int)hipErrorInvalidValue; }
#undef CDNA_MFMA_BT
#undef CDNA_MFMA_CASE
    if (e) return e;
  }
  const int64_t total = (int64_t)NS * d * B;
  int64_t fg = (total + 255) / 256;
  if (fg > 4096) fg = 4096;
  hipLaunchKernelGGL(hist_mfma_finalize, dim3((unsigned)fg), dim3(256), 0, st, acc, d, B, BT * 16, NT * 16, NS,
                     slot_of, out);
  return (int)hipGetLastError();
}
