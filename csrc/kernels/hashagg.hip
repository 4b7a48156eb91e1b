// K16 relational operators in LDS-resident hash tables:
//   groupBy(...).agg(count / sum / avg / min / max / first / last), dropDuplicates (first row of every key),
//   and the probe side of equi-joins.  Course flows: Labs/ML 00L - Dedup Lab.py:79-107 (dropDuplicates),
//   ML 01 - Data Cleansing.py:157-160 (groupBy), MLE 01:246-252 (join + groupBy).
//
// Keys arrive as one 64-bit word per row (a column's value bits, or several key columns packed mixed-radix by
// pack_keys_kernel).  Aggregation and dedup are radix-partitioned so that every partition's table lives in LDS:
//
//   hp_hist     pass 1: rows per (partition, block); partition = top bits of mix64(key)       (LDS counters)
//   hp_scatter  pass 2: keys, row ids and value columns copied partition-contiguous            (LDS cursors)
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

// ------------------------------------------------------------------------------------------- hp_hist / scatter
__global__ __launch_bounds__(kHistThreads) void hp_hist_kernel(const unsigned long long* __restrict__ keys, int64_t n,
                                                               int pbits, int64_t rpb, int* __restrict__ counts) {
  extern __shared__ int s_cnt[];
  const int P = 1 << pbits;
  for (int i = threadIdx.x; i < P; i += kHistThreads) s_cnt[i] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < n ? r0 + rpb : n;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kHistThreads) atomicAdd(&s_cnt[part_of(mix64(keys[r]), pbits)], 1);
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += kHistThreads) counts[(int64_t)i * gridDim.x + blockIdx.x] = s_cnt[i];
}

struct ScatterArgs {
  const unsigned long long* keys;
  int64_t n;
  int pbits;
  int64_t rpb;
  const int64_t* offs;  // [P][nblk] exclusive scan of hp_hist's counts
  int nv;
  const void* val[kMaxAcc];
  const uint8_t* valid[kMaxAcc];
  int vdtype[kMaxAcc];  // 0 f64, 1 f32, 2 i64, 3 i32, 4 u8/bool, 5 i16, 6 i8
  unsigned long long* kout;
  uint32_t* rout;
  unsigned long long* vout;  // [nv][n] fp64 bits, kNullVal for nulls
};

__device__ __forceinline__ unsigned long long value_bits(const ScatterArgs& a, int j, int64_t r) {
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

__global__ __launch_bounds__(kHistThreads) void hp_scatter_kernel(const ScatterArgs a) {
  extern __shared__ uint32_t s_cur[];
  const int P = 1 << a.pbits;
  for (int i = threadIdx.x; i < P; i += kHistThreads) s_cur[i] = (uint32_t)a.offs[(int64_t)i * gridDim.x + blockIdx.x];
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * a.rpb;
  const int64_t r1 = r0 + a.rpb < a.n ? r0 + a.rpb : a.n;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kHistThreads) {
    const unsigned long long k = a.keys[r];
    const uint32_t pos = atomicAdd(&s_cur[part_of(mix64(k), a.pbits)], 1u);
    if (!CDNA_DCHECK(pos < (uint64_t)a.n, 0xA501)) continue;
    a.kout[pos] = k;
    a.rout[pos] = (uint32_t)r;
    for (int j = 0; j < a.nv; ++j) a.vout[(int64_t)j * a.n + pos] = value_bits(a, j, r);
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

__global__ __launch_bounds__(256) void join_probe_kernel(const unsigned long long* __restrict__ keys,
                                                         const uint8_t* __restrict__ valid, int64_t n,
                                                         const unsigned long long* __restrict__ table, int64_t mask,
                                                         const long long* __restrict__ brow,
                                                         const int* __restrict__ bcnt, long long* __restrict__ ri,
                                                         int* __restrict__ cnt, long long* __restrict__ slot) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int64_t found = -1;
    if (!valid || valid[i]) {
      const unsigned long long k = keys[i];
      if (k == kEmpty) {
        found = bcnt[mask + 1] > 0 ? mask + 1 : -1;
      } else {
        int64_t h = (int64_t)(mix64(k) & (unsigned long long)mask);
        for (int64_t t = 0; t <= mask; ++t) {
          const unsigned long long cur = table[h];
          if (cur == k) {
            found = h;
            break;
          }
          if (cur == kEmpty) break;
          h = (h + 1) & mask;
        }
      }
    }
    ri[i] = found >= 0 ? brow[found] : -1;
    if (cnt) cnt[i] = found >= 0 ? bcnt[found] : 0;
    if (slot) slot[i] = found;
  }
}

// dynamic LDS above 64 KB needs the attribute once per kernel (hp_agg's table takes up to 160 KB)
void set_lds_limit() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hp_hist_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            65536);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hp_scatter_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hp_agg_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
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

CDNA_API int cdna_hp_scatter(const void* keys, int64_t n, int pbits, int64_t rpb, const int64_t* offs, int nv,
                             const void* const* vals, const uint8_t* const* valids, const int* vdtypes, void* kout,
                             uint32_t* rout, void* vout, hipStream_t st) {
  if (n <= 0) return 0;
  if (pbits < 0 || pbits > 14 || rpb <= 0 || nv < 0 || nv > kMaxAcc || n >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  ScatterArgs a{};
  a.keys = reinterpret_cast<const unsigned long long*>(keys);
  a.n = n;
  a.pbits = pbits;
  a.rpb = rpb;
  a.offs = offs;
  a.nv = nv;
  for (int j = 0; j < nv; ++j) {
    a.val[j] = vals[j];
    a.valid[j] = valids[j];
    a.vdtype[j] = vdtypes[j];
  }
  a.kout = reinterpret_cast<unsigned long long*>(kout);
  a.rout = rout;
  a.vout = reinterpret_cast<unsigned long long*>(vout);
  const unsigned nblk = (unsigned)((n + rpb - 1) / rpb);
  set_lds_limit();
  hipLaunchKernelGGL(hp_scatter_kernel, dim3(nblk), dim3(kHistThreads), (size_t)4 << pbits, st, a);
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
