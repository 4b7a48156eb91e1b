// DataFrame-engine kernels (SURVEY §2.10 K16 hash_partition, K19 compact, K20 col_stats).
//
// K20 col_moments: count / mean / M2 / min / max of every column of a [n][d]
// row-major matrix in ONE pass (describe(), summary(), StandardScaler,
// Summarizer).  A block owns a row chunk and a group of <= 64 columns: lanes
// are (row lane, column), so a wave reads 64 consecutive columns of a row —
// coalesced for the row-major layout — and each lane runs Welford in fp64 over
// its rows.  Lanes of the same column are merged in LDS with Chan's pairwise
// formula; per-block partials [nblk][d][5] are merged on the device the same
// way (cdnaml/ops/kernels.py col_moments), so the result does not depend on
// the block schedule.  Null entries (valid == 0) are skipped, NaNs are values
// (Spark: a NaN in a column makes its mean NaN).
//
// K16 partition_by_dest: stable counting sort of rows by destination rank /
// bucket (the all-to-all shuffle of groupBy / join / dropDuplicates /
// repartition, Spark "shuffle write").  Pass 1 counts each block's rows per
// bucket in LDS; the host-side exclusive scan of [bucket][block] gives every
// block its output offsets; pass 2 re-reads the block's rows and scatters
// their indices in row order (wave ballots rank rows of equal bucket), so the
// permutation equals a stable argsort of dest without a radix sort.
#include "common.h"

namespace {

constexpr int kThreads = 256;

struct Moments {
  double n, mean, m2, mn, mx;
};

__device__ __forceinline__ Moments merge(const Moments& a, const Moments& b) {
  if (a.n == 0.0) return b;
  if (b.n == 0.0) return a;
  Moments r;
  r.n = a.n + b.n;
  const double delta = b.mean - a.mean;
  r.mean = a.mean + delta * (b.n / r.n);
  r.m2 = a.m2 + b.m2 + delta * delta * (a.n * b.n / r.n);
  // Spark orders NaN above every value: min skips NaNs (fmin), max is NaN once any NaN was seen
  r.mn = fmin(a.mn, b.mn);
  r.mx = (a.mx != a.mx || b.mx != b.mx) ? __builtin_nan("") : fmax(a.mx, b.mx);
  return r;
}

template <typename TV>
__global__ __launch_bounds__(kThreads) void col_moments_kernel(const TV* __restrict__ X, int64_t n, int d,
                                                               int64_t ldx, const uint8_t* __restrict__ valid,
                                                               int64_t ldv, int64_t rows_per_block,
                                                               double* __restrict__ part) {
  __shared__ Moments sm[kThreads];
  const int cg = d - (int)blockIdx.y * 64 < 64 ? d - (int)blockIdx.y * 64 : 64;  // columns in this group
  const int rl = kThreads / cg;                                                   // row lanes
  const int c = threadIdx.x % cg, lane_r = threadIdx.x / cg;
  const int col = blockIdx.y * 64 + c;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  Moments m{0.0, 0.0, 0.0, __builtin_inf(), -__builtin_inf()};
  bool nan_seen = false;
  if (lane_r < rl) {
    for (int64_t r = r0 + lane_r; r < r1; r += rl) {
      if (valid && !valid[r * ldv + col]) continue;
      const double x = (double)X[r * ldx + col];
      if (x != x) nan_seen = true;
      m.n += 1.0;
      const double delta = x - m.mean;
      m.mean += delta / m.n;
      m.m2 += delta * (x - m.mean);
      m.mn = fmin(m.mn, x);
      m.mx = fmax(m.mx, x);
    }
  }
  if (nan_seen) m.mx = __builtin_nan("");
  sm[threadIdx.x] = m;
  __syncthreads();
  if (lane_r == 0) {
    Moments acc = sm[c];
    for (int k = 1; k < rl; ++k) acc = merge(acc, sm[k * cg + c]);
    double* o = part + ((int64_t)blockIdx.x * d + col) * 5;
    o[0] = acc.n;
    o[1] = acc.mean;
    o[2] = acc.m2;
    o[3] = acc.mn;
    o[4] = acc.mx;
  }
}

// dest values must lie in [0, W).  counts: [W][nblk] (bucket-major, so one
// flat exclusive scan gives every (bucket, block) its output offset).
template <bool SCATTER>
__global__ __launch_bounds__(kThreads) void partition_dest_kernel(const int* __restrict__ dest, int64_t n, int W,
                                                                  int64_t rows_per_block, int* __restrict__ counts,
                                                                  const int64_t* __restrict__ offsets,
                                                                  int64_t* __restrict__ perm) {
  extern __shared__ int s_cnt[];  // [W] counts (pass 1) / cursors (pass 2)
  const int nblk = gridDim.x;
  for (int i = threadIdx.x; i < W; i += kThreads) s_cnt[i] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  if (!SCATTER) {
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kThreads) atomicAdd(&s_cnt[dest[r]], 1);
    __syncthreads();
    for (int i = threadIdx.x; i < W; i += kThreads) counts[(int64_t)i * nblk + blockIdx.x] = s_cnt[i];
    return;
  }
  // stable: rounds of 256 rows in order; within a round, waves in order; within a wave, lanes in order
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t rb = r0; rb < r1; rb += kThreads) {
    const int64_t r = rb + threadIdx.x;
    const bool ok = r < r1;
    const int b = ok ? dest[r] : -1;
    // waves take turns so earlier waves' rows get lower positions
    for (int w = 0; w < kThreads / 64; ++w) {
      if (wid == w) {
        bool want = ok;
        while (true) {
          const uint64_t act = __builtin_amdgcn_ballot_w64(want);
          if (!act) break;
          const int leader = __builtin_ctzll(act);
          const int lb = __shfl(b, leader);
          const uint64_t m = __builtin_amdgcn_ballot_w64(want && b == lb);
          int base = 0;
          if (lane == leader) {
            base = s_cnt[lb];
            s_cnt[lb] = base + __builtin_popcountll(m);
          }
          base = __shfl(base, leader);
          if (want && b == lb) {
            const int below =
                (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            perm[offsets[(int64_t)lb * nblk + blockIdx.x] + base + below] = r;
            want = false;
          }
        }
      }
      __syncthreads();
    }
  }
}

// K19 compact: indices of the rows whose mask byte is non-zero, in row order
// (filter / handleInvalid="skip" / coldStartStrategy="drop").  Pass 1 counts
// each block's kept rows with wave ballots; the host-side exclusive scan gives
// block offsets; pass 2 writes each kept row's index at offset + rank (rank =
// kept rows of earlier waves of the round + mbcnt within the wave).
template <bool WRITE>
__global__ __launch_bounds__(kThreads) void compact_mask_kernel(const uint8_t* __restrict__ mask, int64_t n,
                                                                int64_t rows_per_block, int* __restrict__ counts,
                                                                const int64_t* __restrict__ offsets,
                                                                int64_t* __restrict__ idx) {
  __shared__ int s_w[kThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  int64_t base = WRITE ? offsets[blockIdx.x] : 0;
  int total = 0;
  for (int64_t rb = r0; rb < r1; rb += kThreads) {
    const int64_t r = rb + threadIdx.x;
    const bool keep = r < r1 && mask[r] != 0;
    const uint64_t m = __builtin_amdgcn_ballot_w64(keep);
    if (lane == 0) s_w[wid] = __builtin_popcountll(m);
    __syncthreads();
    int before = 0, round = 0;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) {
      before += k < wid ? s_w[k] : 0;
      round += s_w[k];
    }
    __syncthreads();
    if (WRITE && keep) {
      const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      idx[base + before + below] = r;
    }
    base += round;
    total += round;
  }
  if (!WRITE && threadIdx.x == 0) counts[blockIdx.x] = total;
}

// K19 gather: out_c[i] = src_c[idx[i]] for up to 8 one-dimensional columns of 1/2/4/8-byte elements in one launch
// (Batch.take behind filter / join / dropDuplicates / groupBy keys).  Eight rows per thread in flight; the
// index loads and the output stores are coalesced, the source loads follow idx.
constexpr int kMaxGather = 8;
struct GatherArgs {
  const int64_t* idx;
  int64_t m;
  int64_t nsrc;  // source rows: an index outside [0, nsrc) reads nothing and writes 0 (never a wild load)
  int nc;
  const void* src[kMaxGather];
  void* dst[kMaxGather];
  int eb[kMaxGather];
};

// eight rows per thread: their index loads, then per column their eight source loads, are issued back to back
template <typename E, int U>
__device__ __forceinline__ void gcols(const void* s, void* d, const int64_t* j, int64_t i0, int64_t stride,
                                      int64_t m) {
  E v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = j[u] >= 0 ? reinterpret_cast<const E*>(s)[j[u]] : E(0);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i0 + u * stride < m) reinterpret_cast<E*>(d)[i0 + u * stride] = v[u];
}

__global__ __launch_bounds__(kThreads) void gather_kernel(const GatherArgs a) {
  constexpr int U = 8;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i0 = (int64_t)blockIdx.x * kThreads + threadIdx.x; i0 < a.m; i0 += stride * U) {
    int64_t j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      j[u] = i0 + u * stride < a.m ? a.idx[i0 + u * stride] : -1;
      if (j[u] >= a.nsrc) {  // always clamped; the checked build also reports it
        (void)CDNA_DCHECK(false, 0xC019u);
        j[u] = -1;
      }
    }
    for (int c = 0; c < a.nc; ++c) {
      switch (a.eb[c]) {
        case 1: gcols<uint8_t, U>(a.src[c], a.dst[c], j, i0, stride, a.m); break;
        case 2: gcols<uint16_t, U>(a.src[c], a.dst[c], j, i0, stride, a.m); break;
        case 4: gcols<uint32_t, U>(a.src[c], a.dst[c], j, i0, stride, a.m); break;
        default: gcols<uint64_t, U>(a.src[c], a.dst[c], j, i0, stride, a.m); break;
      }
    }
  }
}

}  // namespace

CDNA_DEBUG_EXPORT(relational)

// dtype: 0 = f32, 1 = f64.  part: [nblk][d][5] (count, mean, M2, min, max); nblk = ceil(n / rows_per_block).
CDNA_API int cdna_col_moments(int dtype, const void* X, int64_t n, int d, int64_t ldx, const uint8_t* valid,
                              int64_t ldv, int64_t rows_per_block, double* part, hipStream_t st) {
  if (n <= 0 || d <= 0) return 0;
  if (rows_per_block <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((n + rows_per_block - 1) / rows_per_block), (unsigned)((d + 63) / 64));
  if (dtype == 0)
    hipLaunchKernelGGL(col_moments_kernel<float>, grid, dim3(kThreads), 0, st, (const float*)X, n, d, ldx, valid,
                       ldv, rows_per_block, part);
  else
    hipLaunchKernelGGL(col_moments_kernel<double>, grid, dim3(kThreads), 0, st, (const double*)X, n, d, ldx, valid,
                       ldv, rows_per_block, part);
  return (int)hipGetLastError();
}

// pass 1: counts [W][nblk]; pass 2: perm [n] from offsets [W][nblk] (exclusive scan of counts).
CDNA_API int cdna_partition_dest(int pass, const int* dest, int64_t n, int W, int64_t rows_per_block, int* counts,
                                 const int64_t* offsets, int64_t* perm, hipStream_t st) {
  if (n <= 0) return 0;
  if (W <= 0 || W > 8192 || rows_per_block <= 0) return (int)hipErrorInvalidValue;
  const unsigned nblk = (unsigned)((n + rows_per_block - 1) / rows_per_block);
  const size_t lds = (size_t)W * 4;
  if (pass == 1)
    hipLaunchKernelGGL(partition_dest_kernel<false>, dim3(nblk), dim3(kThreads), lds, st, dest, n, W,
                       rows_per_block, counts, offsets, perm);
  else
    hipLaunchKernelGGL(partition_dest_kernel<true>, dim3(nblk), dim3(kThreads), lds, st, dest, n, W, rows_per_block,
                       counts, offsets, perm);
  return (int)hipGetLastError();
}

// K19: pass 1 counts [nblk] kept rows per block; pass 2 writes idx from offsets [nblk] (exclusive scan).
CDNA_API int cdna_compact_mask(int pass, const uint8_t* mask, int64_t n, int64_t rows_per_block, int* counts,
                               const int64_t* offsets, int64_t* idx, hipStream_t st) {
  if (n <= 0) return 0;
  if (rows_per_block <= 0) return (int)hipErrorInvalidValue;
  const unsigned nblk = (unsigned)((n + rows_per_block - 1) / rows_per_block);
  if (pass == 1)
    hipLaunchKernelGGL(compact_mask_kernel<false>, dim3(nblk), dim3(kThreads), 0, st, mask, n, rows_per_block, counts,
                       offsets, idx);
  else
    hipLaunchKernelGGL(compact_mask_kernel<true>, dim3(nblk), dim3(kThreads), 0, st, mask, n, rows_per_block, counts,
                       offsets, idx);
  return (int)hipGetLastError();
}

CDNA_API int cdna_gather(const int64_t* idx, int64_t m, int64_t nsrc, int nc, const void* const* src,
                         void* const* dst, const int* eb, hipStream_t st) {
  if (m <= 0 || nc <= 0) return 0;
  if (nc > kMaxGather) return (int)hipErrorInvalidValue;
  GatherArgs a{};
  a.idx = idx;
  a.m = m;
  a.nsrc = nsrc;
  a.nc = nc;
  for (int c = 0; c < nc; ++c) {
    if (eb[c] != 1 && eb[c] != 2 && eb[c] != 4 && eb[c] != 8) return (int)hipErrorInvalidValue;
    a.src[c] = src[c];
    a.dst[c] = dst[c];
    a.eb[c] = eb[c];
  }
  int64_t g = (m + 8 * kThreads - 1) / (8 * kThreads);
  g = g < 8192 ? (g > 0 ? g : 1) : 8192;
  hipLaunchKernelGGL(gather_kernel, dim3((unsigned)g), dim3(kThreads), 0, st, a);
  return (int)hipGetLastError();
}
