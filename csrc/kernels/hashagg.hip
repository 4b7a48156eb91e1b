// K16 relational operators in LDS-resident hash tables:
//   groupBy(...).agg(count / sum / avg / min / max / first / last), dropDuplicates (first row of every key),
//   and the probe side of equi-joins.  Course flows: Labs/ML 00L - Dedup Lab.py:79-107 (dropDuplicates),
//   ML 01 - Data Cleansing.py:157-160 (groupBy), MLE 01:246-252 (join + groupBy).
//
// Keys arrive as one 64-bit word per row (a column's value bits, or several key columns packed mixed-radix by
// pack_keys_kernel).  Aggregation and dedup are radix-partitioned so that every partition's table lives in LDS:
//
//   hp_hist     pass 1: rows per (partition, block); partition = top bits of mix64(key)       (LDS counters)
//   hp_part     keys, row ids and value columns radix-partitioned (1-2 passes of <= 128 buckets, LDS tile sort)
//   hp_agg      one 1024-thread block per partition: open-addressing table in LDS holding the key, row count,
//               first row (atomicMin) and up to four accumulators (fp64 sum, ordered-u64 min / max, non-null
//               count, last row) per slot; then the occupied slots are written out as groups.  Dedup mode marks
//               each group's first row in a byte mask (1 + output partition); gid mode sweeps the partition's
//               rows again and writes every row's group position.
//
// A partition whose distinct keys do not fit its table reports -1 and the host runs the operator on its sort
// path instead (never at the sizes of the course or of bench_configs.py relational: 1e8 rows need 6.1e3 rows
// per partition at P = 16384, and the table holds 8191 keys).  No global atomics are issued per row: at
// 64 different rows per wave instruction device atomics run at ~0.08 TB/s (MI355X_MICROARCH.md, 'Global float
// atomics'), which alone would cost ~5 ms per 1e8 rows; LDS atomics cost a few cycles.
//
// join_build / join_probe: the build side (the right input, small for the course's dimension joins) is a global
// table of 2x its rows that stays in L2 / MALL; the probe is plain loads, one per left row, writing the matched
// build row (the first one) and the number of build rows with that key.
#include "common.h"

namespace {

constexpr unsigned long long kEmpty = 0x8000000000000000ull;
constexpr unsigned long long kNullVal = 0x7FF4DEADBEEF0001ull;  // scattered value slot of a null (NaNs canonical)
constexpr int kHistThreads = 256;
constexpr int kAggThreads = 1024;
constexpr int kMaxAcc = 4;
constexpr int kMaxCols = 8;

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int part_of(unsigned long long h, int pbits) {
  return pbits == 0 ? 0 : (int)(h >> (64 - pbits));
}

// table position in [0, S) from the low 32 hash bits (S need not be a power of two)
__device__ __forceinline__ int pos_of(unsigned long long h, int S) {
  return (int)(((h & 0xFFFFFFFFull) * (unsigned long long)S) >> 32);
}

// order-preserving map of doubles to u64 (NaN canonical, above +inf, as Spark orders NaN)
__device__ __forceinline__ unsigned long long ord_of(unsigned long long b) {
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// ----------------------------------------------------------------------------------------------- pack_keys
struct PackArgs {
  const void* col[kMaxCols];
  const uint8_t* valid[kMaxCols];
  long long lo[kMaxCols];     // column minimum (code = value - lo + 1; null = 0)
  long long radix[kMaxCols];  // max - min + 2
  int dtype[kMaxCols];        // 0 u8/bool, 1 i16, 2 i32, 3 i64, 4 i8
  int ncols;
  int64_t n;
  long long* out;
};

__device__ __forceinline__ long long load_int(const void* p, int dt, int64_t i) {
  switch (dt) {
    case 0: return (long long)reinterpret_cast<const uint8_t*>(p)[i];
    case 1: return (long long)reinterpret_cast<const int16_t*>(p)[i];
    case 2: return (long long)reinterpret_cast<const int32_t*>(p)[i];
    case 4: return (long long)reinterpret_cast<const int8_t*>(p)[i];
    default: return reinterpret_cast<const long long*>(p)[i];
  }
}

__global__ __launch_bounds__(256) void pack_keys_kernel(const PackArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * 256) {
    long long k = 0;
    for (int c = 0; c < a.ncols; ++c) {
      const bool ok = !a.valid[c] || a.valid[c][i];
      const long long code = ok ? load_int(a.col[c], a.dtype[c], i) - a.lo[c] + 1 : 0;
      k = k * a.radix[c] + code;
    }
    a.out[i] = k;
  }
}

// ------------------------------------------------------------------------------------------- hp_hist / part
// Four keys in flight per thread (the LDS increment of one waits on nothing but its own load).
__global__ __launch_bounds__(kHistThreads) void hp_hist_kernel(const unsigned long long* __restrict__ keys, int64_t n,
                                                               int pbits, int64_t rpb, int* __restrict__ counts) {
  extern __shared__ int s_cnt[];
  const int P = 1 << pbits;
  for (int i = threadIdx.x; i < P; i += kHistThreads) s_cnt[i] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < n ? r0 + rpb : n;
  int64_t r = r0 + threadIdx.x;
  for (; r + 3 * kHistThreads < r1; r += 4 * kHistThreads) {
    unsigned long long k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = keys[r + u * kHistThreads];
#pragma unroll
    for (int u = 0; u < 4; ++u) atomicAdd(&s_cnt[part_of(mix64(k[u]), pbits)], 1);
  }
  for (; r < r1; r += kHistThreads) atomicAdd(&s_cnt[part_of(mix64(keys[r]), pbits)], 1);
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += kHistThreads) counts[(int64_t)i * gridDim.x + blockIdx.x] = s_cnt[i];
}

// Radix partition of (key, row, values) in one or two passes of <= 128 buckets (partition id = top pbits of the
// key hash; pass 0 buckets by its top pbits - 7 bits when pbits > 7, pass 1 by the low 7).  A scattered 8-byte
// store per row into 16384 partitions measured 6.9 ms per 1e8 rows (every store a partial line), so each block
// sorts a tile of rows by bucket in LDS first and writes every bucket's run as consecutive stores; a bucket's
// runs of successive tiles continue at the next address, so the partial lines at run ends complete in L2.
//
// Pass 0 block b reads rows [b * rpb, ...) of the input and writes bucket q's run at cur[q * nblk + b] onward.
// Pass 1 block (p1, g) reads the pass-0 rows of bucket p1 that came from source blocks [g * gs, g * gs + gs) --
// contiguous, since pass 0 stores bucket p1's rows by source block -- and writes partition (p1, p2) at
// offs[(p1 * 128 + p2) * nblk + g * gs] onward, exactly where hp_agg expects that partition's rows.
struct PartArgs {
  int pass;                         // 0: from the original columns, 1: from pass-0 output
  int64_t n;
  int nb;                           // buckets (power of two <= 128)
  int shift;                        // bucket = (mix64(key) >> shift) & (nb - 1); shift 64: one bucket
  int64_t rpb;                      // pass 0: rows per block
  int nblk;                         // blocks of hp_hist
  int gs, groups;                   // pass 1: source blocks per block, blocks per bucket
  const int64_t* cur;               // pass 0: [nb][nblk] output starts; pass 1: offs [P][nblk]
  const int64_t* src;               // pass 1: [P1][nblk] + 1 pass-0 output starts (last entry n)
  const unsigned long long* keys;   // pass 0
  const void* val[kMaxAcc];
  const uint8_t* valid[kMaxAcc];
  int vdtype[kMaxAcc];              // 0 f64, 1 f32, 2 i64, 3 i32, 4 u8/bool, 5 i16, 6 i8
  const unsigned long long* kin;    // pass 1
  const uint32_t* rin;
  const unsigned long long* vin;    // [nv][n]
  int nv;
  int tile;
  unsigned long long* kout;
  uint32_t* rout;
  unsigned long long* vout;         // [nv][n] fp64 bits, kNullVal for nulls
};

template <class A>
__device__ __forceinline__ unsigned long long value_bits(const A& a, int j, int64_t r) {
  if (a.valid[j] && !a.valid[j][r]) return kNullVal;
  double v;
  switch (a.vdtype[j]) {
    case 0: v = reinterpret_cast<const double*>(a.val[j])[r]; break;
    case 1: v = (double)reinterpret_cast<const float*>(a.val[j])[r]; break;
    case 2: v = (double)reinterpret_cast<const long long*>(a.val[j])[r]; break;
    case 3: v = (double)reinterpret_cast<const int*>(a.val[j])[r]; break;
    case 4: v = (double)reinterpret_cast<const uint8_t*>(a.val[j])[r]; break;
    case 5: v = (double)reinterpret_cast<const int16_t*>(a.val[j])[r]; break;
    default: v = (double)reinterpret_cast<const int8_t*>(a.val[j])[r]; break;
  }
  return v != v ? 0x7FF8000000000000ull : (unsigned long long)__double_as_longlong(v);
}

constexpr int kPartThreads = 512;

__global__ __launch_bounds__(kPartThreads) void hp_part_kernel(const PartArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int TILE = a.tile;
  unsigned long long* s_key = reinterpret_cast<unsigned long long*>(smem);        // [TILE]
  unsigned long long* s_val = s_key + TILE;                                        // [nv][TILE]
  uint32_t* s_row = reinterpret_cast<uint32_t*>(s_val + (int64_t)a.nv * TILE);     // [TILE]
  uint8_t* s_bk = reinterpret_cast<uint8_t*>(s_row + TILE);                        // [TILE]
  __shared__ int s_cnt[128], s_start[128];
  __shared__ int64_t s_cur[128];
  int64_t r0, r1;
  if (a.pass == 0) {
    r0 = (int64_t)blockIdx.x * a.rpb;
    r1 = r0 + a.rpb < a.n ? r0 + a.rpb : a.n;
    for (int q = threadIdx.x; q < a.nb; q += kPartThreads) s_cur[q] = a.cur[(int64_t)q * a.nblk + blockIdx.x];
  } else {
    const int p1 = blockIdx.x / a.groups, g = blockIdx.x - p1 * a.groups;
    const int b0 = g * a.gs, b1 = b0 + a.gs < a.nblk ? b0 + a.gs : a.nblk;
    r0 = a.src[(int64_t)p1 * a.nblk + b0];
    r1 = a.src[(int64_t)p1 * a.nblk + b1];
    for (int q = threadIdx.x; q < a.nb; q += kPartThreads)
      s_cur[q] = a.cur[((int64_t)p1 * a.nb + q) * a.nblk + b0];
  }
  constexpr int kPer = 8;  // rows per thread per tile (TILE <= 8 * 512)
  for (int64_t t0 = r0; t0 < r1; t0 += TILE) {
    const int m = (int)(r1 - t0 < TILE ? r1 - t0 : TILE);
    for (int q = threadIdx.x; q < a.nb; q += kPartThreads) s_cnt[q] = 0;
    __syncthreads();
    unsigned long long k[kPer];
    int bk[kPer], rk[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kPartThreads;
      k[u] = 0;
      bk[u] = -1;
      if (i < m) k[u] = a.pass == 0 ? a.keys[t0 + i] : a.kin[t0 + i];
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kPartThreads;
      if (i < m) {
        bk[u] = a.shift >= 64 ? 0 : (int)((mix64(k[u]) >> a.shift) & (unsigned long long)(a.nb - 1));
        rk[u] = atomicAdd(&s_cnt[bk[u]], 1);
      }
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of <= 128 counts by one wave (two per lane)
      const int l = threadIdx.x;
      const int c0 = 2 * l < a.nb ? s_cnt[2 * l] : 0, c1 = 2 * l + 1 < a.nb ? s_cnt[2 * l + 1] : 0;
      int v = c0 + c1;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o);
        if (l >= o) v += y;
      }
      const int ex = v - c0 - c1;
      if (2 * l < a.nb) s_start[2 * l] = ex;
      if (2 * l + 1 < a.nb) s_start[2 * l + 1] = ex + c0;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kPartThreads;
      if (i < m) {
        const int pos = s_start[bk[u]] + rk[u];
        const int64_t r = t0 + i;
        s_key[pos] = k[u];
        s_row[pos] = a.pass == 0 ? (uint32_t)r : a.rin[r];
        s_bk[pos] = (uint8_t)bk[u];
        for (int j = 0; j < a.nv; ++j)
          s_val[(int64_t)j * TILE + pos] = a.pass == 0 ? value_bits(a, j, r) : a.vin[(int64_t)j * a.n + r];
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += kPartThreads) {
      const int q = s_bk[i];
      const int64_t dst = s_cur[q] + (i - s_start[q]);
      if (!CDNA_DCHECK(dst >= 0 && dst < a.n, 0xA501)) continue;
      a.kout[dst] = s_key[i];
      a.rout[dst] = s_row[i];
      for (int j = 0; j < a.nv; ++j) a.vout[(int64_t)j * a.n + dst] = s_val[(int64_t)j * TILE + i];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < a.nb; q += kPartThreads) s_cur[q] += s_cnt[q];
  }
}

// -------------------------------------------------------------------------------------------------- hp_agg
// acc ops: 0 fp64 sum, 1 min, 2 max (ordered u64 of the fp64 value), 3 non-null count, 4 last row (max row id)
struct AggArgs {
  const unsigned long long* kin;
  const uint32_t* rin;
  const unsigned long long* vin;  // [nv][n]
  int64_t n;
  const int64_t* offs;  // [P][nblk]
  int nblk;
  int S;                // LDS table slots (the special EMPTY key uses slot S)
  int cap;              // distinct keys a partition may hold before it reports overflow
  int na;
  int op[kMaxAcc];
  int vcol[kMaxAcc];
  int mode;             // 0 aggregate, 1 dedup (first rows only), 2 aggregate + per-row group positions
  int pout;             // dedup: output partitions (<= 255)
  unsigned long long* gkey;  // [n] group outputs at the partition's row offset
  uint32_t* gcnt;
  uint32_t* gfirst;
  unsigned long long* gacc;  // [na][n]
  int* ngroups;              // [P]: groups of the partition, -1 = overflow
  uint8_t* keep;             // dedup: [n] 1 + output partition of every first row
  int* gpos;                 // mode 2: [n] group position of every row
};

__device__ __forceinline__ unsigned long long acc_init(int op) {
  return op == 1 ? ~0ull : 0ull;
}

__global__ __launch_bounds__(kAggThreads) void hp_agg_kernel(const AggArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = a.S;
  unsigned long long* tk = reinterpret_cast<unsigned long long*>(smem);  // [S + 1]
  unsigned long long* ta = tk + (S + 1);                                 // [na][S + 1]
  uint32_t* tc = reinterpret_cast<uint32_t*>(ta + (int64_t)a.na * (S + 1));  // [S + 1]
  uint32_t* tf = tc + (S + 1);                                                // [S + 1]
  __shared__ int s_nd, s_ovf, s_out;
  const int p = blockIdx.x;
  const int64_t start = a.offs[(int64_t)p * a.nblk];
  const int64_t end = p + 1 < (int)gridDim.x ? a.offs[(int64_t)(p + 1) * a.nblk] : a.n;
  for (int s = threadIdx.x; s <= S; s += kAggThreads) {
    tk[s] = kEmpty;
    tc[s] = 0u;
    tf[s] = 0xFFFFFFFFu;
    for (int j = 0; j < a.na; ++j) ta[(int64_t)j * (S + 1) + s] = acc_init(a.op[j]);
  }
  if (threadIdx.x == 0) {
    s_nd = 0;
    s_ovf = 0;
    s_out = 0;
  }
  __syncthreads();
  const bool agg = a.mode != 1;
  for (int64_t i = start + threadIdx.x; i < end; i += kAggThreads) {
    const unsigned long long k = a.kin[i];
    const uint32_t r = a.rin[i];
    int s = S;
    if (k != kEmpty) {
      int pos = pos_of(mix64(k), S);
      s = -1;
      for (int t = 0; t < S; ++t) {
        const unsigned long long cur = __hip_atomic_load(tk + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == k) {
          s = pos;
          break;
        }
        if (cur == kEmpty) {
          const unsigned long long prev = atomicCAS(tk + pos, kEmpty, k);
          if (prev == kEmpty) {
            if (atomicAdd(&s_nd, 1) >= a.cap) s_ovf = 1;
            s = pos;
            break;
          }
          if (prev == k) {
            s = pos;
            break;
          }
        }
        pos = pos + 1 == S ? 0 : pos + 1;
      }
      if (s < 0) {
        s_ovf = 1;
        continue;
      }
    }
    atomicMin(tf + s, r);
    if (!agg) continue;
    atomicAdd(tc + s, 1u);
    for (int j = 0; j < a.na; ++j) {
      unsigned long long* slot = ta + (int64_t)j * (S + 1) + s;
      const int op = a.op[j];
      if (op == 4) {
        atomicMax(slot, (unsigned long long)r);
        continue;
      }
      const unsigned long long v = a.vin[(int64_t)a.vcol[j] * a.n + i];
      if (v == kNullVal) continue;
      if (op == 0) atomicAdd(reinterpret_cast<double*>(slot), __longlong_as_double((long long)v));
      else if (op == 1) atomicMin(slot, ord_of(v));
      else if (op == 2) atomicMax(slot, ord_of(v));
      else atomicAdd(slot, 1ull);
    }
  }
  __syncthreads();
  if (s_ovf) {
    if (threadIdx.x == 0) a.ngroups[p] = -1;
    return;
  }
  for (int s = threadIdx.x; s <= S; s += kAggThreads) {
    const unsigned long long k = tk[s];
    const bool occ = s < S ? k != kEmpty : tf[s] != 0xFFFFFFFFu;
    if (!occ) continue;
    const int gi = atomicAdd(&s_out, 1);
    const int64_t o = start + gi;
    const uint32_t first = tf[s];
    if (a.mode == 1) {
      a.keep[first] = (uint8_t)(1 + (int)((uint32_t)(mix64(k) >> 16) % (uint32_t)a.pout));
      continue;
    }
    a.gkey[o] = k;
    a.gcnt[o] = tc[s];
    a.gfirst[o] = first;
    for (int j = 0; j < a.na; ++j) a.gacc[(int64_t)j * a.n + o] = ta[(int64_t)j * (S + 1) + s];
    tc[s] = (uint32_t)gi;  // mode 2 reads the group position back
  }
  __syncthreads();
  if (threadIdx.x == 0) a.ngroups[p] = s_out;
  if (a.mode != 2) return;
  for (int64_t i = start + threadIdx.x; i < end; i += kAggThreads) {
    const unsigned long long k = a.kin[i];
    int s = S;
    if (k != kEmpty) {
      int pos = pos_of(mix64(k), S);
      for (int t = 0; t < S && tk[pos] != k; ++t) pos = pos + 1 == S ? 0 : pos + 1;
      s = pos;
    }
    a.gpos[a.rin[i]] = (int)(start + tc[s]);
  }
}

// --------------------------------------------------------------------------------- low-cardinality path
// Few distinct keys (groupBy over 50 values, a handful of categories): partitioning would put all rows of a key
// into one partition and one block.  Instead every block aggregates a contiguous row chunk of the original
// columns into its own LDS table (la_agg) and appends its partial groups to one list; a single block then merges
// the partials (la_merge: counts and sums add, first rows and mins take the min, maxes and last rows the max).
// A chunk with more distinct keys than its table holds stops early and raises the overflow flag; the host then
// runs the partitioned path.
// Once the table has overflowed (cap distinct keys) a probe gives up within 32 steps: without that, every row after
// the overflow walked the whole nearly-full table (4.4 ms per 1e8 high-cardinality rows before the fallback).
__device__ __forceinline__ bool flagged(int* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
}

__device__ __forceinline__ int lds_slot(unsigned long long* tk, int S, unsigned long long k, int cap, int* s_nd,
                                        int* s_ovf) {
  if (k == kEmpty) return S;
  int pos = pos_of(mix64(k), S);
  for (int t = 0; t < S; ++t) {
    if ((t & 31) == 31 && flagged(s_ovf)) return -1;
    const unsigned long long cur = __hip_atomic_load(tk + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == k) return pos;
    if (cur == kEmpty) {
      const unsigned long long prev = atomicCAS(tk + pos, kEmpty, k);
      if (prev == kEmpty) {
        if (atomicAdd(s_nd, 1) >= cap) *s_ovf = 1;
        return pos;
      }
      if (prev == k) return pos;
    }
    pos = pos + 1 == S ? 0 : pos + 1;
  }
  *s_ovf = 1;
  return -1;
}

struct LocalArgs {
  const unsigned long long* keys;
  int64_t n;
  int64_t rpb;
  int S, cap, na;
  int op[kMaxAcc];
  int vcol[kMaxAcc];
  const void* val[kMaxAcc];
  const uint8_t* valid[kMaxAcc];
  int vdtype[kMaxAcc];
  int mode;                  // 0 aggregate, 1 dedup
  int pout;
  unsigned long long* pkey;  // partial groups [pcap]
  uint32_t* pcnt;
  uint32_t* pfirst;
  unsigned long long* pacc;  // [na][pcap]
  int64_t pcap;
  int* total;                // partial groups appended so far
  int* ovf;
  unsigned long long* gkey;  // la_merge output [S + 1]
  uint32_t* gcnt;
  uint32_t* gfirst;
  unsigned long long* gacc;  // [na][S + 1]
  int* ngroups;              // la_merge: groups, -1 = overflow
  uint8_t* keep;
};

struct LdsTable {
  unsigned long long *tk, *ta;
  uint32_t *tc, *tf;
};

__device__ __forceinline__ LdsTable lds_table(unsigned char* smem, int S, int na) {
  LdsTable t;
  t.tk = reinterpret_cast<unsigned long long*>(smem);
  t.ta = t.tk + (S + 1);
  t.tc = reinterpret_cast<uint32_t*>(t.ta + (int64_t)na * (S + 1));
  t.tf = t.tc + (S + 1);
  return t;
}

__device__ __forceinline__ void lds_table_init(const LdsTable& t, int S, int na, const int* op) {
  for (int s = threadIdx.x; s <= S; s += kAggThreads) {
    t.tk[s] = kEmpty;
    t.tc[s] = 0u;
    t.tf[s] = 0xFFFFFFFFu;
    for (int j = 0; j < na; ++j) t.ta[(int64_t)j * (S + 1) + s] = acc_init(op[j]);
  }
}

__global__ __launch_bounds__(kAggThreads) void la_agg_kernel(const LocalArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (__hip_atomic_load(a.ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // another chunk overflowed
  const int S = a.S;
  const LdsTable t = lds_table(smem, S, a.na);
  __shared__ int s_nd, s_ovf, s_out, s_base;
  lds_table_init(t, S, a.na, a.op);
  if (threadIdx.x == 0) {
    s_nd = 0;
    s_ovf = 0;
    s_out = 0;
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * a.rpb;
  const int64_t r1 = r0 + a.rpb < a.n ? r0 + a.rpb : a.n;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kAggThreads) {
    if (flagged(&s_ovf)) break;
    const int s = lds_slot(t.tk, S, a.keys[r], a.cap, &s_nd, &s_ovf);
    if (s < 0) break;
    atomicMin(t.tf + s, (uint32_t)r);
    if (a.mode == 1) continue;
    atomicAdd(t.tc + s, 1u);
    for (int j = 0; j < a.na; ++j) {
      unsigned long long* slot = t.ta + (int64_t)j * (S + 1) + s;
      const int op = a.op[j];
      if (op == 4) {
        atomicMax(slot, (unsigned long long)r);
        continue;
      }
      const unsigned long long v = value_bits(a, a.vcol[j], r);
      if (v == kNullVal) continue;
      if (op == 0) atomicAdd(reinterpret_cast<double*>(slot), __longlong_as_double((long long)v));
      else if (op == 1) atomicMin(slot, ord_of(v));
      else if (op == 2) atomicMax(slot, ord_of(v));
      else atomicAdd(slot, 1ull);
    }
  }
  __syncthreads();
  if (s_ovf) {
    if (threadIdx.x == 0) atomicOr(a.ovf, 1);
    return;
  }
  if (threadIdx.x == 0) s_base = atomicAdd(a.total, s_nd + (t.tf[S] != 0xFFFFFFFFu ? 1 : 0));
  __syncthreads();
  for (int s = threadIdx.x; s <= S; s += kAggThreads) {
    const bool occ = s < S ? t.tk[s] != kEmpty : t.tf[s] != 0xFFFFFFFFu;
    if (!occ) continue;
    const int64_t o = (int64_t)s_base + atomicAdd(&s_out, 1);
    if (!CDNA_DCHECK(o < a.pcap, 0xA502)) continue;
    a.pkey[o] = s < S ? t.tk[s] : kEmpty;
    a.pcnt[o] = t.tc[s];
    a.pfirst[o] = t.tf[s];
    for (int j = 0; j < a.na; ++j) a.pacc[(int64_t)j * a.pcap + o] = t.ta[(int64_t)j * (S + 1) + s];
  }
}

__global__ __launch_bounds__(kAggThreads) void la_merge_kernel(const LocalArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = a.S;
  const LdsTable t = lds_table(smem, S, a.na);
  __shared__ int s_nd, s_ovf, s_out;
  if (__hip_atomic_load(a.ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
    if (threadIdx.x == 0) a.ngroups[0] = -1;
    return;
  }
  lds_table_init(t, S, a.na, a.op);
  if (threadIdx.x == 0) {
    s_nd = 0;
    s_ovf = 0;
    s_out = 0;
  }
  __syncthreads();
  const int64_t total = *a.total;
  for (int64_t e = threadIdx.x; e < total; e += kAggThreads) {
    if (flagged(&s_ovf)) break;
    const int s = lds_slot(t.tk, S, a.pkey[e], S - 1, &s_nd, &s_ovf);
    if (s < 0) break;
    atomicMin(t.tf + s, a.pfirst[e]);
    if (a.mode == 1) continue;
    atomicAdd(t.tc + s, a.pcnt[e]);
    for (int j = 0; j < a.na; ++j) {
      unsigned long long* slot = t.ta + (int64_t)j * (S + 1) + s;
      const unsigned long long v = a.pacc[(int64_t)j * a.pcap + e];
      const int op = a.op[j];
      if (op == 0) atomicAdd(reinterpret_cast<double*>(slot), __longlong_as_double((long long)v));
      else if (op == 1) atomicMin(slot, v);
      else if (op == 2 || op == 4) atomicMax(slot, v);
      else atomicAdd(slot, v);
    }
  }
  __syncthreads();
  if (s_ovf) {
    if (threadIdx.x == 0) a.ngroups[0] = -1;
    return;
  }
  for (int s = threadIdx.x; s <= S; s += kAggThreads) {
    const bool occ = s < S ? t.tk[s] != kEmpty : t.tf[s] != 0xFFFFFFFFu;
    if (!occ) continue;
    const unsigned long long k = s < S ? t.tk[s] : kEmpty;
    const int gi = atomicAdd(&s_out, 1);
    if (a.mode == 1) {
      a.keep[t.tf[s]] = (uint8_t)(1 + (int)((uint32_t)(mix64(k) >> 16) % (uint32_t)a.pout));
      continue;
    }
    a.gkey[gi] = k;
    a.gcnt[gi] = t.tc[s];
    a.gfirst[gi] = t.tf[s];
    for (int j = 0; j < a.na; ++j) a.gacc[(int64_t)j * (S + 1) + gi] = t.ta[(int64_t)j * (S + 1) + s];
  }
  __syncthreads();
  if (threadIdx.x == 0) a.ngroups[0] = s_out;
}

// ------------------------------------------------------------------------------------------ bucket_compact
// dropDuplicates output: the rows whose keep byte is non-zero (1 + output partition), grouped by partition and
// in row order within a partition.  Every wave owns a contiguous row range (no block barriers): pass 1 counts
// its rows per bucket with one ballot per bucket and 64 rows, pass 2 writes each kept row at its bucket's
// running offset + its rank among the wave's lanes (mbcnt).  Up to 16 buckets keep their counters in scalar
// registers; more buckets elect one bucket per step from the active lanes.
template <bool SCATTER>
__global__ __launch_bounds__(256) void bucket_compact_kernel(const uint8_t* __restrict__ keep, int64_t n, int nb,
                                                             int64_t rpw, int* __restrict__ counts,
                                                             const int64_t* __restrict__ offs,
                                                             int64_t* __restrict__ idx) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t r0 = w * rpw;
  const int64_t r1 = r0 + rpw < n ? r0 + rpw : n;
  if (nb <= 16) {
    int64_t c[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) c[q] = SCATTER && q < nb ? offs[(int64_t)q * nw + w] : 0;
    for (int64_t rb = r0; rb < r1; rb += 64) {
      const int64_t r = rb + lane;
      const int b = r < r1 ? (int)keep[r] - 1 : -1;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q >= nb) break;
        const uint64_t m = __builtin_amdgcn_ballot_w64(b == q);
        if (SCATTER && b == q)
          idx[c[q] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = r;
        c[q] += __builtin_popcountll(m);
      }
    }
    if (!SCATTER && lane == 0)
      for (int q = 0; q < nb; ++q) counts[(int64_t)q * nw + w] = (int)c[q];
    return;
  }
  __shared__ int64_t s_c[4][256];
  int64_t* c = s_c[threadIdx.x >> 6];
  for (int q = lane; q < nb; q += 64) c[q] = SCATTER ? offs[(int64_t)q * nw + w] : 0;
  for (int64_t rb = r0; rb < r1; rb += 64) {
    const int64_t r = rb + lane;
    const int b = r < r1 ? (int)keep[r] - 1 : -1;
    bool want = b >= 0;
    while (true) {
      const uint64_t act = __builtin_amdgcn_ballot_w64(want);
      if (!act) break;
      const int lb = __shfl(b, __builtin_ctzll(act));
      const uint64_t m = __builtin_amdgcn_ballot_w64(want && b == lb);
      const int64_t base = c[lb];
      if (SCATTER && want && b == lb)
        idx[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = r;
      if (want && b == lb) want = false;
      if (lane == 0) c[lb] = base + __builtin_popcountll(m);
    }
  }
  if (!SCATTER)
    for (int q = lane; q < nb; q += 64) counts[(int64_t)q * nw + w] = (int)c[q];
}

// ---------------------------------------------------------------------------------------------------- join
__global__ __launch_bounds__(256) void join_build_kernel(const unsigned long long* __restrict__ keys,
                                                         const uint8_t* __restrict__ valid, int64_t n,
                                                         unsigned long long* __restrict__ table, int64_t mask,
                                                         long long* __restrict__ brow, int* __restrict__ bcnt,
                                                         int* __restrict__ overflow) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (valid && !valid[i]) continue;  // null keys never match
    const unsigned long long k = keys[i];
    int64_t h = mask + 1;  // the EMPTY key's own slot
    if (k != kEmpty) {
      h = (int64_t)(mix64(k) & (unsigned long long)mask);
      int64_t found = -1;
      for (int64_t t = 0; t <= mask; ++t) {
        const unsigned long long cur = __hip_atomic_load(table + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == k) {
          found = h;
          break;
        }
        if (cur == kEmpty) {
          const unsigned long long prev = atomicCAS(table + h, kEmpty, k);
          if (prev == kEmpty || prev == k) {
            found = h;
            break;
          }
        }
        h = (h + 1) & mask;
      }
      if (found < 0) {
        atomicOr(overflow, 1);
        continue;
      }
      h = found;
    }
    atomicMin(brow + h, (long long)i);
    atomicAdd(bcnt + h, 1);
  }
}

// Four rows per thread in flight: key loads, first table probes and the build-row loads of four rows are issued
// back to back (one row's dependent chain at a time left the probe at 1.75 ms per 1e8 rows).
__global__ __launch_bounds__(256) void join_probe_kernel(const unsigned long long* __restrict__ keys,
                                                         const uint8_t* __restrict__ valid, int64_t n,
                                                         const unsigned long long* __restrict__ table, int64_t mask,
                                                         const long long* __restrict__ brow,
                                                         const int* __restrict__ bcnt, long long* __restrict__ ri,
                                                         int* __restrict__ cnt, long long* __restrict__ slot) {
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * U) {
    unsigned long long k[U], cur[U];
    int64_t h[U], found[U];
    bool live[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      live[u] = i < n && (!valid || valid[i]);
      k[u] = live[u] ? keys[i] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      found[u] = -1;
      h[u] = 0;
      cur[u] = kEmpty;
      if (live[u]) {
        if (k[u] == kEmpty) {
          found[u] = bcnt[mask + 1] > 0 ? mask + 1 : -1;
          live[u] = false;
        } else {
          h[u] = (int64_t)(mix64(k[u]) & (unsigned long long)mask);
          cur[u] = table[h[u]];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!live[u]) continue;
      for (int64_t t = 0; t <= mask; ++t) {
        if (cur[u] == k[u]) {
          found[u] = h[u];
          break;
        }
        if (cur[u] == kEmpty) break;
        h[u] = (h[u] + 1) & mask;
        cur[u] = table[h[u]];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n) continue;
      ri[i] = found[u] >= 0 ? brow[found[u]] : -1;
      if (cnt) cnt[i] = found[u] >= 0 ? bcnt[found[u]] : 0;
      if (slot) slot[i] = found[u];
    }
  }
}

// Dense join tables: when the build keys span a small range [lo, lo + R) (the course's integer ids, packed
// (user, movie) pairs), the table is direct-addressed -- no hashing, no probing -- and a presence bitmap of
// R bits (125 KB for 1e6 keys: L2-resident) answers the misses without touching the row array.
__global__ __launch_bounds__(256) void join_build_dense_kernel(const long long* __restrict__ keys,
                                                               const uint8_t* __restrict__ valid, int64_t n,
                                                               long long lo, int64_t R, long long* __restrict__ brow,
                                                               int* __restrict__ bcnt, uint32_t* __restrict__ bits) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (valid && !valid[i]) continue;
    const long long f = keys[i] - lo;
    if (!CDNA_DCHECK(f >= 0 && f < R, 0xA503)) continue;
    atomicMin(brow + f, (long long)i);
    atomicAdd(bcnt + f, 1);
    atomicOr(bits + (f >> 5), 1u << (f & 31));
  }
}

__global__ __launch_bounds__(256) void join_probe_dense_kernel(const long long* __restrict__ keys,
                                                               const uint8_t* __restrict__ valid, int64_t n,
                                                               long long lo, int64_t R,
                                                               const long long* __restrict__ brow,
                                                               const int* __restrict__ bcnt,
                                                               const uint32_t* __restrict__ bits,
                                                               long long* __restrict__ ri, int* __restrict__ cnt,
                                                               long long* __restrict__ slot) {
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * U) {
    long long f[U];
    bool hit[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      f[u] = -1;
      if (i < n && (!valid || valid[i])) f[u] = keys[i] - lo;
      if (f[u] >= R) f[u] = -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) hit[u] = f[u] >= 0 && ((bits[f[u] >> 5] >> (f[u] & 31)) & 1u);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n) continue;
      ri[i] = hit[u] ? brow[f[u]] : -1;
      if (cnt) cnt[i] = hit[u] ? bcnt[f[u]] : 0;
      if (slot) slot[i] = hit[u] ? f[u] : -1;
    }
  }
}

// dynamic LDS above 64 KB needs the attribute once per kernel (the LDS tables take up to 160 KB)
void set_lds_limit() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hp_hist_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            65536);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hp_part_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            163840 - 2048);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hp_agg_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            163840 - 64);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&la_agg_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            163840 - 64);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&la_merge_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            163840 - 64);
  done = true;
}

unsigned grid_of(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (unsigned)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

}  // namespace

CDNA_DEBUG_EXPORT(hashagg)

CDNA_API int cdna_pack_keys(int ncols, const void* const* cols, const uint8_t* const* valids, const long long* lo,
                            const long long* radix, const int* dtypes, int64_t n, long long* out, hipStream_t st) {
  if (n <= 0) return 0;
  if (ncols <= 0 || ncols > kMaxCols) return (int)hipErrorInvalidValue;
  PackArgs a{};
  for (int c = 0; c < ncols; ++c) {
    a.col[c] = cols[c];
    a.valid[c] = valids[c];
    a.lo[c] = lo[c];
    a.radix[c] = radix[c];
    a.dtype[c] = dtypes[c];
  }
  a.ncols = ncols;
  a.n = n;
  a.out = out;
  hipLaunchKernelGGL(pack_keys_kernel, dim3(grid_of(n)), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// counts: [P = 2^pbits][nblk] int32, nblk = ceil(n / rpb).
CDNA_API int cdna_hp_hist(const void* keys, int64_t n, int pbits, int64_t rpb, int* counts, hipStream_t st) {
  if (n <= 0) return 0;
  if (pbits < 0 || pbits > 14 || rpb <= 0 || n >= (1ll << 31)) return (int)hipErrorInvalidValue;
  const unsigned nblk = (unsigned)((n + rpb - 1) / rpb);
  set_lds_limit();
  hipLaunchKernelGGL(hp_hist_kernel, dim3(nblk), dim3(kHistThreads), (size_t)4 << pbits, st,
                     reinterpret_cast<const unsigned long long*>(keys), n, pbits, rpb, counts);
  return (int)hipGetLastError();
}

// pass 0 / pass 1 (np1 pass-0 buckets x groups blocks): see PartArgs.  vals / valids / vdtypes: the value columns (pass 0 only).
CDNA_API int cdna_hp_part(int pass, int64_t n, int nb, int shift, int64_t rpb, int nblk, int gs, int groups, int np1,
                          const int64_t* cur, const int64_t* src, const void* keys, int nv, const void* const* vals,
                          const uint8_t* const* valids, const int* vdtypes, const void* kin, const uint32_t* rin,
                          const void* vin, void* kout, uint32_t* rout, void* vout, hipStream_t st) {
  if (n <= 0) return 0;
  if (nb < 1 || nb > 128 || (nb & (nb - 1)) || nv < 0 || nv > kMaxAcc || n >= (1ll << 31) || nblk <= 0 ||
      (pass == 0 && rpb <= 0) || (pass == 1 && (gs <= 0 || groups <= 0 || np1 <= 0)))
    return (int)hipErrorInvalidValue;
  PartArgs a{};
  a.pass = pass;
  a.n = n;
  a.nb = nb;
  a.shift = shift;
  a.rpb = rpb;
  a.nblk = nblk;
  a.gs = gs;
  a.groups = groups;
  a.cur = cur;
  a.src = src;
  a.keys = reinterpret_cast<const unsigned long long*>(keys);
  for (int j = 0; j < nv; ++j) {
    a.val[j] = pass == 0 ? vals[j] : nullptr;
    a.valid[j] = pass == 0 ? valids[j] : nullptr;
    a.vdtype[j] = pass == 0 ? vdtypes[j] : 0;
  }
  a.kin = reinterpret_cast<const unsigned long long*>(kin);
  a.rin = rin;
  a.vin = reinterpret_cast<const unsigned long long*>(vin);
  a.nv = nv;
  a.tile = nv <= 1 ? 4096 : 2048;
  a.kout = reinterpret_cast<unsigned long long*>(kout);
  a.rout = rout;
  a.vout = reinterpret_cast<unsigned long long*>(vout);
  const size_t lds = (size_t)a.tile * (8 + 8 * nv + 4 + 1);
  set_lds_limit();
  const unsigned nblocks = pass == 0 ? (unsigned)nblk : (unsigned)groups * (unsigned)np1;
  hipLaunchKernelGGL(hp_part_kernel, dim3(nblocks), dim3(kPartThreads), lds, st, a);
  return (int)hipGetLastError();
}

CDNA_API int cdna_hp_agg_lds_bytes(int S, int na) { return (S + 1) * (16 + 8 * na); }
CDNA_API int cdna_hp_agg_lds_budget() { return 163840 - 64; }

CDNA_API int cdna_hp_agg(const void* kin, const uint32_t* rin, const void* vin, int64_t n, const int64_t* offs,
                         int pbits, int nblk, int S, int cap, int na, const int* ops, const int* vcols, int mode,
                         int pout, void* gkey, uint32_t* gcnt, uint32_t* gfirst, void* gacc, int* ngroups,
                         uint8_t* keep, int* gpos, hipStream_t st) {
  if (n <= 0) return 0;
  const int lds = cdna_hp_agg_lds_bytes(S, na);
  if (pbits < 0 || pbits > 14 || S < 64 || S > 65536 || cap >= S || na < 0 || na > kMaxAcc || lds > cdna_hp_agg_lds_budget() ||
      mode < 0 || mode > 2 || (mode == 1 && (pout < 1 || pout > 255)) || n >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  AggArgs a{};
  a.kin = reinterpret_cast<const unsigned long long*>(kin);
  a.rin = rin;
  a.vin = reinterpret_cast<const unsigned long long*>(vin);
  a.n = n;
  a.offs = offs;
  a.nblk = nblk;
  a.S = S;
  a.cap = cap;
  a.na = na;
  for (int j = 0; j < na; ++j) {
    a.op[j] = ops[j];
    a.vcol[j] = vcols[j];
  }
  a.mode = mode;
  a.pout = pout;
  a.gkey = reinterpret_cast<unsigned long long*>(gkey);
  a.gcnt = gcnt;
  a.gfirst = gfirst;
  a.gacc = reinterpret_cast<unsigned long long*>(gacc);
  a.ngroups = ngroups;
  a.keep = keep;
  a.gpos = gpos;
  set_lds_limit();
  hipLaunchKernelGGL(hp_agg_kernel, dim3(1u << pbits), dim3(kAggThreads), (size_t)lds, st, a);
  return (int)hipGetLastError();
}

// table: [mask + 2] u64 = EMPTY (slot mask + 1: the EMPTY key); brow: [mask + 2] = INT64_MAX; bcnt: [mask + 2] = 0.
CDNA_API int cdna_join_build(const void* keys, const uint8_t* valid, int64_t n, void* table, int64_t mask,
                             long long* brow, int* bcnt, int* overflow, hipStream_t st) {
  if (n <= 0) return 0;
  if (((mask + 1) & mask) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(join_build_kernel, dim3(grid_of(n)), dim3(256), 0, st,
                     reinterpret_cast<const unsigned long long*>(keys), valid, n,
                     reinterpret_cast<unsigned long long*>(table), mask, brow, bcnt, overflow);
  return (int)hipGetLastError();
}

// ri: [n] first matching build row or -1; cnt (optional): build rows with the key; slot (optional): table slot.
CDNA_API int cdna_join_probe(const void* keys, const uint8_t* valid, int64_t n, const void* table, int64_t mask,
                             const long long* brow, const int* bcnt, long long* ri, int* cnt, long long* slot,
                             hipStream_t st) {
  if (n <= 0) return 0;
  if (((mask + 1) & mask) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(join_probe_kernel, dim3(grid_of(n)), dim3(256), 0, st,
                     reinterpret_cast<const unsigned long long*>(keys), valid, n,
                     reinterpret_cast<const unsigned long long*>(table), mask, brow, bcnt, ri, cnt, slot);
  return (int)hipGetLastError();
}

// Low-cardinality aggregation / dedup: la_agg over nblk = ceil(n / rpb) blocks, then la_merge; ngroups[0] = groups
// (-1: a chunk or the merged table overflowed -> the partitioned path).  total / ovf: two zeroed ints.
CDNA_API int cdna_la_groups(const void* keys, int64_t n, int64_t rpb, int S, int cap, int na, const int* ops,
                            const int* vcols, int nv, const void* const* vals, const uint8_t* const* valids,
                            const int* vdtypes, int mode, int pout, void* pkey, uint32_t* pcnt, uint32_t* pfirst,
                            void* pacc, int64_t pcap, int* total, int* ovf, void* gkey, uint32_t* gcnt,
                            uint32_t* gfirst, void* gacc, int* ngroups, uint8_t* keep, hipStream_t st) {
  if (n <= 0) return 0;
  const int lds = cdna_hp_agg_lds_bytes(S, na);
  if (rpb <= 0 || S < 64 || S > 65536 || cap >= S || na < 0 || na > kMaxAcc || nv < 0 || nv > kMaxAcc ||
      lds > cdna_hp_agg_lds_budget() || mode < 0 || mode > 1 || (mode == 1 && (pout < 1 || pout > 255)) ||
      n >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  const int64_t nblk = (n + rpb - 1) / rpb;
  if (pcap < nblk * (int64_t)(cap + 2)) return (int)hipErrorInvalidValue;
  LocalArgs a{};
  a.keys = reinterpret_cast<const unsigned long long*>(keys);
  a.n = n;
  a.rpb = rpb;
  a.S = S;
  a.cap = cap;
  a.na = na;
  for (int j = 0; j < na; ++j) {
    a.op[j] = ops[j];
    a.vcol[j] = vcols[j];
  }
  for (int j = 0; j < nv; ++j) {
    a.val[j] = vals[j];
    a.valid[j] = valids[j];
    a.vdtype[j] = vdtypes[j];
  }
  a.mode = mode;
  a.pout = pout;
  a.pkey = reinterpret_cast<unsigned long long*>(pkey);
  a.pcnt = pcnt;
  a.pfirst = pfirst;
  a.pacc = reinterpret_cast<unsigned long long*>(pacc);
  a.pcap = pcap;
  a.total = total;
  a.ovf = ovf;
  a.gkey = reinterpret_cast<unsigned long long*>(gkey);
  a.gcnt = gcnt;
  a.gfirst = gfirst;
  a.gacc = reinterpret_cast<unsigned long long*>(gacc);
  a.ngroups = ngroups;
  a.keep = keep;
  set_lds_limit();
  hipLaunchKernelGGL(la_agg_kernel, dim3((unsigned)nblk), dim3(kAggThreads), (size_t)lds, st, a);
  hipLaunchKernelGGL(la_merge_kernel, dim3(1), dim3(kAggThreads), (size_t)lds, st, a);
  return (int)hipGetLastError();
}

// pass 1: counts [nb][nwaves] of the rows with keep = 1 + bucket (nwaves = 4 * ceil(n / (4 * rpw))); pass 2: idx
// from offs (exclusive scan of counts).
CDNA_API int cdna_bucket_compact(int pass, const uint8_t* keep, int64_t n, int nb, int64_t rpw, int* counts,
                                 const int64_t* offs, int64_t* idx, hipStream_t st) {
  if (n <= 0) return 0;
  if (nb < 1 || nb > 255 || rpw <= 0 || (rpw & 63)) return (int)hipErrorInvalidValue;
  const int64_t nw = (n + rpw - 1) / rpw;
  const unsigned nblk = (unsigned)((nw + 3) / 4);
  if (pass == 1)
    hipLaunchKernelGGL(bucket_compact_kernel<false>, dim3(nblk), dim3(256), 0, st, keep, n, nb, rpw, counts, offs, idx);
  else
    hipLaunchKernelGGL(bucket_compact_kernel<true>, dim3(nblk), dim3(256), 0, st, keep, n, nb, rpw, counts, offs, idx);
  return (int)hipGetLastError();
}

// brow [R] = INT64_MAX, bcnt [R] = 0, bits [(R + 31) / 32] = 0 on entry.
CDNA_API int cdna_join_build_dense(const long long* keys, const uint8_t* valid, int64_t n, long long lo, int64_t R,
                                   long long* brow, int* bcnt, uint32_t* bits, hipStream_t st) {
  if (n <= 0) return 0;
  if (R <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(join_build_dense_kernel, dim3(grid_of(n)), dim3(256), 0, st, keys, valid, n, lo, R, brow, bcnt,
                     bits);
  return (int)hipGetLastError();
}

CDNA_API int cdna_join_probe_dense(const long long* keys, const uint8_t* valid, int64_t n, long long lo, int64_t R,
                                   const long long* brow, const int* bcnt, const uint32_t* bits, long long* ri,
                                   int* cnt, long long* slot, hipStream_t st) {
  if (n <= 0) return 0;
  if (R <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(join_probe_dense_kernel, dim3(grid_of(n)), dim3(256), 0, st, keys, valid, n, lo, R, brow, bcnt,
                     bits, ri, cnt, slot);
  return (int)hipGetLastError();
}
