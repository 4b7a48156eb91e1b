// K5s: feature-subset ("masked") level histograms of a regression forest, with
// the items generated on the fly from the row codes (no compaction pass).
//
// RandomForestRegressor's featureSubsetStrategy="auto" samples m = ceil(d / 3)
// features per node (ML 07 - Random Forests and Hyperparameter Tuning.py:41;
// ML 06 - Decision Trees.py:108-110 for the level histograms).  The full-feature
// path (seg.hip) accumulates all d features of the smaller child and derives
// its sibling by subtraction; its LDS atomics are the headline's floor
// (quarter-wave lane kernel: ~2 ds_add_u64 wave-instructions per item at 100 of
// 128 lane slots, 87 ms per step) and the item records cost a count + scatter
// pass per level (19 ms).  Here every node of the level is built, but only over
// its m sampled features: 34 instead of 100 lane-ops per item, 2.14e11 instead
// of 3.66e11 per headline step.
//
// Work: a block owns (slot group, row chunk).  A slot group is <= NS
// consecutive active nodes (of one or several trees) whose LDS histograms fit
// beside the per-wave staging buffers.  Each wave walks "tasks" = (32-row tile,
// pair of the group's trees): lanes 0-31 decode tree a's codes (weight << 8 |
// local node) of the 32 rows, lanes 32-63 tree b's.  A ballot turns rows with a
// non-zero weight in one of the group's nodes into items, appended to a per-wave
// LDS ring as 16-byte descriptors {LDS addend, slot's histogram offset, v_perm
// feature selector} plus the row id.  Every 32 items form a batch whose
// 128-byte row lines are gathered L2 -> LDS by global_load_lds_dwordx4.
//
// Pipeline (every vector-memory op is an LDS DMA issued by inline asm, so all
// waits are explicit vmcnt counts kept in a wave-uniform counter; no VGPR is
// ever the target of an in-flight load): the next task's codes and labels and
// the next batch's lines are in flight while the current batch is processed
// (two line buffers, two metadata buffers, a 128-entry descriptor ring).
//
// Processing a batch: a 16-lane QUARTER of the wave takes one item (4 items per
// instruction); lane k owns sampled features 16 p + k of the item's node (p =
// feature planes).  The feature id is one v_perm_b32 of the lane's per-slot
// feature bytes with the item's selector; the bin is a byte read of the staged
// line; the LDS cell is [slot][p][bin][16 lanes] u64, so each 16-lane group of
// a ds_add_u64 (one item, 16 distinct k) hits 16 distinct bank pairs whatever
// the bins -- conflict-free.  One descriptor read serves all planes of an item.
// Features 16 P .. m - 1 (tail) are packed densely over the lanes.
//
// The LDS words are the packed count << 44 | sum w (q + 2^23) of the record
// kernels (same quantisation of the label: rintf(v1 * qs1) clamped to 2^23),
// flushed as exact int64 (count, sum w q) into [S][m][B][2] -- the integers the
// full-feature histogram holds for those features, so every split decision and
// every child statistic is bit-identical (power-of-two scales: all fp64 sums
// downstream are exact).
#include "common.h"

namespace {

constexpr int kShift = 44;
constexpr uint32_t kQOff = 1u << 23;
constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kBatch = 32;                 // items (= staged row lines) per batch
constexpr int kRing = 128;                 // descriptor ring entries per wave (4 batch windows)
constexpr int kLineBytes = 128;
constexpr int kMaxPlanes = 7;              // m <= 127
// per-wave LDS layout (bytes)
constexpr int kDescOff = 0;                               // [kRing] x 16 B descriptors
constexpr int kRowOff = kDescOff + kRing * 16;            // [kRing] x u32 row in chunk
constexpr int kLineOff = kRowOff + kRing * 4;             // [2][kBatch][128] staged row lines
constexpr int kMetaOff = kLineOff + 2 * kBatch * kLineBytes;  // [2][512]: codes (2 x 17 dwords), labels (32 f32)
constexpr int kMetaBytes = 512;
constexpr int kWaveLds = kMetaOff + 2 * kMetaBytes;       // 11 776 B

struct SubHistArgs {
  const uint16_t* codes;   // [T][n]
  const float* v1;         // [n]
  const uint8_t* bins_rm;  // [n][128]
  int64_t n;
  int T;
  int B, m, P, TR;         // bins, sampled features, 16-feature planes, tail features (m = 16 P + TR)
  float qs1;
  const int* tfirst;       // [T] slot of each tree's local node 0 (launch slot coordinates)
  const int* groups;       // [G][4] slot range [s0, s1), tree range [t0, t1)
  const uint8_t* feats;    // [S][m] sampled features per slot (ascending)
  int G;
  int64_t chunk_rows;      // multiple of 32
  int nchunks;
  int ns_max;
  int slot_words;          // u64 words per slot = B * m
  unsigned long long* out; // [S][m][B][2] int64 (count, sum w q)
};

__device__ __forceinline__ void dma16(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(g),
               "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}
__device__ __forceinline__ void dma4(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" : : "v"(g),
               "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}

// Wait until at most n of this wave's vector-memory ops are outstanding (n >= 15: vmcnt(15), stricter, still
// correct).  The "memory" clobber keeps the LDS reads of the landed data behind the wait.
__device__ __forceinline__ void wait_vm(int n) {
  n = __builtin_amdgcn_readfirstlane(n);
  switch (n <= 0 ? 0 : (n >= 15 ? 15 : n)) {
#define CDNA_WVM(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    CDNA_WVM(0) CDNA_WVM(1) CDNA_WVM(2) CDNA_WVM(3) CDNA_WVM(4) CDNA_WVM(5) CDNA_WVM(6) CDNA_WVM(7)
    CDNA_WVM(8) CDNA_WVM(9) CDNA_WVM(10) CDNA_WVM(11) CDNA_WVM(12) CDNA_WVM(13) CDNA_WVM(14) CDNA_WVM(15)
#undef CDNA_WVM
  }
}

struct WaveState {
  uint8_t* base;       // this wave's LDS region
  uint32_t base_lds;   // its LDS byte address
  int vm;              // vector-memory ops issued so far (wave-uniform)
};

// Issue the codes + labels of task (row0, trees ta / tb) into metadata buffer mb.
__device__ __forceinline__ void issue_meta(const SubHistArgs& a, WaveState& ws, int mb, int64_t row0, int ta, int tb,
                                           int64_t r1, int lane) {
  const uintptr_t cbeg = (uintptr_t)a.codes;
  const uintptr_t clast = (cbeg + (uintptr_t)(2 * (int64_t)a.T * a.n) - 4) & ~(uintptr_t)3;
  const int t = lane < 17 ? ta : tb;
  const int l = lane < 17 ? lane : lane - 17;
  uintptr_t ad = (cbeg + 2 * ((uintptr_t)t * (uintptr_t)a.n + (uintptr_t)row0)) & ~(uintptr_t)3;
  ad += 4 * (uintptr_t)(lane < 34 ? l : 0);
  ad = ad < clast ? ad : clast;
  const uint32_t meta = ws.base_lds + kMetaOff + mb * kMetaBytes;
  dma4(reinterpret_cast<const void*>(ad), meta);
  const int64_t rl = r1 - 1;
  int64_t rr = row0 + (lane & 31);
  rr = rr < rl ? rr : rl;
  dma4(a.v1 + rr, meta + 256);
  ws.vm += 2;
}

// Gather the lines of ring window w into line buffer lb (items past cnt were padded with a valid row).
__device__ __forceinline__ void issue_lines(const SubHistArgs& a, WaveState& ws, int w, int lb, int64_t r0, int lane) {
  const uint32_t* rows = reinterpret_cast<const uint32_t*>(ws.base + kRowOff);
  const uint32_t dst = ws.base_lds + kLineOff + lb * kBatch * kLineBytes;
#pragma unroll
  for (int i = 0; i < kBatch / 8; ++i) {
    const int j = 32 * w + 8 * i + (lane >> 3);
    const int64_t row = r0 + (int64_t)rows[j];
    dma16(a.bins_rm + row * kLineBytes + (lane & 7) * 16, dst + i * 1024);
  }
  ws.vm += kBatch / 8;
}

// Histogram the 32 items of ring window w, lines in buffer lb.
__device__ __forceinline__ void process(const SubHistArgs& a, unsigned char* __restrict__ hb, const WaveState& ws,
                                        int w, int lb, int lane,
                                        const uint32_t (&fm0)[kMaxPlanes], const uint32_t (&fm1)[kMaxPlanes],
                                        uint32_t tf0, uint32_t tf1, int tj, int tk, int tper) {
  const uint4* desc = reinterpret_cast<const uint4*>(ws.base + kDescOff) + 32 * w;
  const uint8_t* lines = ws.base + kLineOff + lb * kBatch * kLineBytes;
  const int q = lane >> 4, k = lane & 15;
  const uint32_t k8 = (uint32_t)k * 8u;
  const uint32_t pstride = (uint32_t)a.B * 128u;  // bytes per 16-feature plane of a slot
  // main planes: quarter q takes item 4 g + q
#pragma unroll 2
  for (int g = 0; g < kBatch / 4; ++g) {
    const int j = 4 * g + q;
    const uint4 d = desc[j];
    const unsigned long long add = ((unsigned long long)d.y << 32) | d.x;
    const uint32_t cbk = d.z + k8;
    const uint8_t* ln = lines + j * kLineBytes;
    uint32_t bin[kMaxPlanes];
#pragma unroll
    for (int p = 0; p < kMaxPlanes; ++p)
      if (p < a.P) bin[p] = ln[__builtin_amdgcn_perm(fm1[p], fm0[p], d.w)];
#pragma unroll
    for (int p = 0; p < kMaxPlanes; ++p)
      if (p < a.P)
        atomicAdd(reinterpret_cast<unsigned long long*>(hb + (cbk + (uint32_t)p * pstride + bin[p] * 128u)), add);
  }
  // tail features 16 P + kk: lane (tj, tk) takes item j0 + tj, tper items per instruction
  if (a.TR && tj >= 0) {
    const uint32_t toff = (uint32_t)a.P * pstride;
    for (int j0 = 0; j0 < kBatch; j0 += tper) {
      const int j = j0 + tj;
      if (j < kBatch) {
        const uint4 d = desc[j];
        const unsigned long long add = ((unsigned long long)d.y << 32) | d.x;
        const uint32_t bin = lines[j * kLineBytes + __builtin_amdgcn_perm(tf1, tf0, d.w)];
        atomicAdd(reinterpret_cast<unsigned long long*>(hb + (d.z + toff + (bin * (uint32_t)a.TR + (uint32_t)tk) * 8u)),
                  add);
      }
    }
  }
}

__global__ __launch_bounds__(kThreads) void sub_hist_kernel(const SubHistArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int bid = (int)blockIdx.x;
  const int xcd = bid & 7, k8 = bid >> 3;
  const int cl = k8 / a.G, g = k8 - cl * a.G;
  const int chunk = cl * 8 + xcd;  // the G groups of one chunk run back to back on one XCD (shared L2 lines)
  if (chunk >= a.nchunks) return;  // block-uniform
  const int s0 = a.groups[4 * g], s1 = a.groups[4 * g + 1], t0 = a.groups[4 * g + 2], t1 = a.groups[4 * g + 3];
  const int ns = s1 - s0;
  const int64_t r0 = (int64_t)chunk * a.chunk_rows;
  const int64_t r1 = r0 + a.chunk_rows < a.n ? r0 + a.chunk_rows : a.n;

  unsigned long long* H = reinterpret_cast<unsigned long long*>(smem);
  uint8_t* F = smem + (size_t)a.ns_max * a.slot_words * 8;
  unsigned char* wregion = F + ((a.ns_max * a.m + 15) & ~15);
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = (int)(threadIdx.x & 63);
  WaveState ws;
  ws.base = wregion + wid * kWaveLds;
  ws.base_lds = (uint32_t)(uintptr_t)ws.base;
  ws.vm = 0;

  for (int i = threadIdx.x; i < ns * a.slot_words; i += kThreads) H[i] = 0ull;
  for (int i = threadIdx.x; i < ns * a.m; i += kThreads) F[i] = a.feats[(int64_t)s0 * a.m + i];
  // the group's trees' slot bases, in LDS: a global load inside the task loop would make the compiler drain
  // every in-flight DMA (its own vmcnt bookkeeping does not see the inline-asm loads)
  int* TF = reinterpret_cast<int*>(wregion + kWaves * kWaveLds);
  if (threadIdx.x < t1 - t0) TF[threadIdx.x] = a.tfirst[t0 + threadIdx.x];
  __syncthreads();

  // per-lane feature bytes: plane p, lane k -> feature 16 p + k of slots 0-3 (fm0) / 4-7 (fm1); the item's
  // v_perm selector 0x0C0C0C00 | slot picks one byte
  uint32_t fm0[kMaxPlanes], fm1[kMaxPlanes];
  const int k = lane & 15;
#pragma unroll
  for (int p = 0; p < kMaxPlanes; ++p) {
    uint32_t w0 = 0, w1 = 0;
    if (p < a.P) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        w0 |= (b < ns ? (uint32_t)F[b * a.m + 16 * p + k] : 0u) << (8 * b);
        w1 |= (b + 4 < ns ? (uint32_t)F[(b + 4) * a.m + 16 * p + k] : 0u) << (8 * b);
      }
    }
    fm0[p] = w0;
    fm1[p] = w1;
  }
  // tail: lane l -> (item tj, feature 16 P + tk), tper = 64 / TR items per instruction
  int tper = 1, tj = -1, tk = 0;
  uint32_t tf0 = 0, tf1 = 0;
  if (a.TR) {
    tper = 64 / a.TR;
    if (lane < tper * a.TR) {
      tj = lane / a.TR;
      tk = lane - tj * a.TR;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        tf0 |= (b < ns ? (uint32_t)F[b * a.m + 16 * a.P + tk] : 0u) << (8 * b);
        tf1 |= (b + 4 < ns ? (uint32_t)F[(b + 4) * a.m + 16 * a.P + tk] : 0u) << (8 * b);
      }
    }
  }

  const int npair = (t1 - t0 + 1) >> 1;
  const int64_t ntile = (r1 - r0 + 31) >> 5;
  const int64_t ntask = ((ntile - wid + kWaves - 1) / kWaves) * npair;  // this wave's tiles: wid, wid + 8, ...
  const int half = lane >> 5, kr = lane & 31;
  uint4* descs = reinterpret_cast<uint4*>(ws.base + kDescOff);
  uint32_t* rows = reinterpret_cast<uint32_t*>(ws.base + kRowOff);
  int tail = 0;          // ring entries appended
  int formed = 0;        // ring entries in formed batches
  int pend_w = -1, pend_lb = 0, pend_end = 0;  // batch in flight: window, line buffer, vm index after its DMA
  int nbatch = 0;

  int meta_end[2] = {0, 0};
  if (ntask > 0) {
    issue_meta(a, ws, 0, r0 + wid * 32, t0, t0 + 1 < t1 ? t0 + 1 : t0, r1, lane);
    meta_end[0] = ws.vm;
  }
  for (int64_t tau = 0; tau < ntask; ++tau) {
    const int mb = (int)(tau & 1);
    if (tau + 1 < ntask) {
      const int64_t ti = (tau + 1) / npair;
      const int tan = t0 + 2 * (int)(tau + 1 - ti * npair);
      issue_meta(a, ws, mb ^ 1, r0 + (wid + ti * kWaves) * 32, tan, tan + 1 < t1 ? tan + 1 : tan, r1, lane);
      meta_end[mb ^ 1] = ws.vm;
    }
    wait_vm(ws.vm - meta_end[mb]);
    // ---- items of this task
    const int64_t ti = tau / npair;
    const int ta = t0 + 2 * (int)(tau - ti * npair);
    const int64_t row0 = r0 + (wid + ti * kWaves) * 32;
    const int t = half && ta + 1 < t1 ? ta + 1 : ta;
    const bool tok = half ? (ta + 1 < t1) : true;
    const uint8_t* meta = ws.base + kMetaOff + mb * kMetaBytes;
    const uint32_t mis = (uint32_t)((2 * ((uint64_t)t * (uint64_t)a.n + (uint64_t)row0)) & 3u);
    const uint32_t c = *reinterpret_cast<const uint16_t*>(meta + half * 68 + mis + 2 * kr);
    const float x = reinterpret_cast<const float*>(meta + 256)[kr];
    const int64_t rr = row0 + kr;
    const uint32_t loc = c & 0xFFu, wt = c >> 8;
    const int ls = TF[t - t0] + (int)loc - s0;
    const bool ok = rr < r1 && tok && loc != 0xFFu && wt != 0u && ls >= 0 && ls < ns;
    const uint64_t msk = __builtin_amdgcn_ballot_w64(ok);
    if (msk != 0ull) {
      const int pos = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(msk >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)msk, 0u));
      if (ok) {
        int q1 = (int)rintf(x * a.qs1);
        q1 = q1 > (int)kQOff ? (int)kQOff : (q1 < -(int)kQOff ? -(int)kQOff : q1);
        const unsigned long long add =
            ((unsigned long long)wt << kShift) + (unsigned long long)wt * (uint32_t)(q1 + (int)kQOff);
        const int e = (tail + pos) & (kRing - 1);
        descs[e] = make_uint4((uint32_t)add, (uint32_t)(add >> 32),
                              (uint32_t)ls * (uint32_t)a.slot_words * 8u, 0x0C0C0C00u | (uint32_t)ls);
        rows[e] = (uint32_t)(rr - r0);
      }
      tail += __builtin_popcountll(msk);
    }
    // ---- batches: form the next, then histogram the one in flight
    while (tail - formed >= kBatch) {
      const int w = (formed >> 5) & 3, lb = nbatch & 1;
      issue_lines(a, ws, w, lb, r0, lane);
      const int end = ws.vm;
      formed += kBatch;
      ++nbatch;
      if (pend_w >= 0) {
        wait_vm(ws.vm - pend_end);
        process(a, smem, ws, pend_w, pend_lb, lane, fm0, fm1, tf0, tf1, tj, tk, tper);
      }
      pend_w = w;
      pend_lb = lb;
      pend_end = end;
    }
  }
  // ---- the last partial batch: pad to 32 items with zero addends on a valid row, then drain
  if (tail > formed) {
    const int e = formed + lane;
    if (lane < kBatch && e >= tail) {
      descs[e & (kRing - 1)] = make_uint4(0u, 0u, 0u, 0x0C0C0C00u);
      rows[e & (kRing - 1)] = 0u;
    }
    const int w = (formed >> 5) & 3, lb = nbatch & 1;
    issue_lines(a, ws, w, lb, r0, lane);
    const int end = ws.vm;
    formed += kBatch;
    ++nbatch;
    if (pend_w >= 0) {
      wait_vm(ws.vm - pend_end);
      process(a, smem, ws, pend_w, pend_lb, lane, fm0, fm1, tf0, tf1, tj, tk, tper);
    }
    pend_w = w;
    pend_lb = lb;
    pend_end = end;
  }
  if (pend_w >= 0) {
    wait_vm(0);
    process(a, smem, ws, pend_w, pend_lb, lane, fm0, fm1, tf0, tf1, tj, tk, tper);
  }
  __syncthreads();

  // flush: cell -> (slot, sampled feature index, bin), exact int64 (count, sum w q)
  const int main_words = a.P * a.B * 16;
  for (int cidx = threadIdx.x; cidx < ns * a.slot_words; cidx += kThreads) {
    const unsigned long long v = H[cidx];
    if (!v) continue;
    const int ls = cidx / a.slot_words, r = cidx - ls * a.slot_words;
    int kf, bn;
    if (r < main_words) {
      const int p = r / (a.B * 16), rem = r - p * a.B * 16;
      bn = rem >> 4;
      kf = 16 * p + (rem & 15);
    } else {
      const int rem = r - main_words;
      bn = rem / a.TR;
      kf = 16 * a.P + (rem - bn * a.TR);
    }
    const unsigned long long cnt = v >> kShift;
    const long long sum = (long long)(v & ((1ull << kShift) - 1ull)) - (long long)kQOff * (long long)cnt;
    unsigned long long* o = a.out + ((((int64_t)(s0 + ls) * a.m + kf) * a.B + bn) * 2);
    atomicAdd(o, cnt);
    atomicAdd(o + 1, (unsigned long long)sum);
  }
}

}  // namespace

// groups [G][4] (s0, s1, t0, t1) in launch slot coordinates (tfirst too); out [S][m][B][2] zeroed by the caller.
CDNA_API int cdna_sub_hist(const uint16_t* codes, const float* v1, const uint8_t* bins_rm, int64_t n, int row_bytes,
                           int T, int B, int m, float qs1, const int* tfirst, const int* groups, int G,
                           const uint8_t* feats, int ns_max, int64_t chunk_rows, unsigned long long* out,
                           hipStream_t st) {
  if (row_bytes != kLineBytes || B < 1 || B > 256 || m < 1 || m > 16 * kMaxPlanes + 15 || ns_max < 1 ||
      ns_max > 8 || chunk_rows < 32 || (chunk_rows & 31) || chunk_rows > (1 << 20) || T < 1)
    return (int)hipErrorInvalidValue;
  if (n <= 0 || G <= 0) return 0;
  SubHistArgs a;
  a.codes = codes;
  a.v1 = v1;
  a.bins_rm = bins_rm;
  a.n = n;
  a.T = T;
  a.B = B;
  a.m = m;
  a.P = m / 16;
  a.TR = m % 16;
  a.qs1 = qs1;
  a.tfirst = tfirst;
  a.groups = groups;
  a.feats = feats;
  a.G = G;
  a.chunk_rows = chunk_rows;
  a.nchunks = (int)((n + chunk_rows - 1) / chunk_rows);
  a.ns_max = ns_max;
  a.slot_words = B * m;
  a.out = out;
  const size_t lds = (size_t)ns_max * a.slot_words * 8 + (size_t)((ns_max * m + 15) & ~15) + (size_t)kWaves * kWaveLds +
                     64;  // + the group's tree bases
  if (lds > 163840) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&sub_hist_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        163840);
    attr = true;
  }
  const int ncl = (a.nchunks + 7) / 8;
  const int64_t nblk = (int64_t)ncl * 8 * G;
  hipLaunchKernelGGL(sub_hist_kernel, dim3((unsigned)nblk), dim3(kThreads), lds, st, a);
  return (int)hipGetLastError();
}

// LDS bytes one slot of a group takes, and the budget for the group (the host sizes groups with them).
CDNA_API int cdna_sub_hist_slot_bytes(int B, int m) { return B * m * 8 + m; }
CDNA_API int cdna_sub_hist_lds_budget() { return 163840 - kWaves * kWaveLds - 64 - 16; }
