// K3 quantile_bins: per-feature split thresholds from the (global) sample
// (Spark findSplits semantics; reference call sites ML 06 /
// ML 07 maxBins).  One block per feature: the feature's sample column is
// staged in LDS (<= 16384 doubles = 128 KB of the 160 KB), bitonic-sorted
// there (NaN -> +inf, i.e. last), and the block derives
//   nn   = #non-NaN values,  k = #distinct non-NaN values,
//   cand = midpoints between the value at each quantile position and the next
//          larger sample value (the largest value is replaced by the one below
//          it), de-duplicated,
// exactly as cdnaml/models/tree/engine.py:find_thresholds_t does with a
// chain of ~20 small torch ops (each a launch, 1.4 ms of launch gaps per fit).
// The sorted column is also written out so the host can run the categorical /
// few-distinct-values path on the features that need it.
//
// Sort: when the column is exactly fp32 (the engine's samples are rows of the fp32 feature matrix) and holds at
// most kQRadixS values, a rocPRIM block radix sort of 32-bit keys held 12 per thread in registers (4 passes of
// 8 bits) replaces the 105-stage LDS bitonic network over fp64 (275 us -> see profiles/r4/prologue_ab.md at the
// 1e4-row sample of the headline); otherwise the bitonic path.  Both give the same sorted values (-0.0 / +0.0
// aside, which compare equal everywhere downstream).
#include "common.h"
#include <rocprim/block/block_radix_sort.hpp>

namespace {

constexpr int kQThreads = 1024;
constexpr int kQMaxS = 16384;
constexpr int kQItems = 12;
constexpr int kQRadixS = kQThreads * kQItems;  // 12288
using QRadixSort = rocprim::block_radix_sort<float, kQThreads, kQItems>;

__device__ __forceinline__ double nan_to_inf(double v) { return v != v ? __builtin_inf() : v; }

// RADIX: the caller checked s <= kQRadixS; a block whose column is not exactly fp32 still takes the bitonic path
// (then the dynamic LDS must hold P doubles: the launcher sizes it for both).
template <bool RADIX>
__global__ __launch_bounds__(kQThreads) void quantile_kernel(const double* __restrict__ samp, int s, int d,
                                                             int max_bins, double* __restrict__ sorted,
                                                             double* __restrict__ thr, int* __restrict__ nthr,
                                                             int* __restrict__ kdist, float* __restrict__ thr32) {
  extern __shared__ double sv[];  // [P] (radix: the sort's storage first, then [s] sorted values)
  __shared__ int red_nn[kQThreads / 64], red_k[kQThreads / 64];
  __shared__ double cand[256];
  const int f = blockIdx.x;
  int P = 1;
  while (P < s) P <<= 1;
  int nn_loc = 0;
  bool sorted_ok = false;
  if (RADIX) {
    float key[kQItems];
    int inexact = 0;
#pragma unroll
    for (int j = 0; j < kQItems; ++j) {
      const int i = (int)threadIdx.x * kQItems + j;  // blocked: thread t holds values [12 t, 12 t + 12)
      float v = __builtin_inff();
      if (i < s) {
        const double x = samp[(int64_t)i * d + f];
        nn_loc += x == x;
        const double xi = nan_to_inf(x);
        v = (float)xi;
        inexact |= (double)v != xi;
      }
      key[j] = v;
    }
    if (!__syncthreads_or(inexact)) {
      QRadixSort().sort(key, *reinterpret_cast<typename QRadixSort::storage_type*>(sv));
      __syncthreads();  // the storage is reused as sv below
#pragma unroll
      for (int j = 0; j < kQItems; ++j) {
        const int i = (int)threadIdx.x * kQItems + j;
        if (i < s) sv[i] = (double)key[j];
      }
      __syncthreads();
      sorted_ok = true;
    } else {
      nn_loc = 0;  // recounted by the bitonic path's load
    }
  }
  if (!sorted_ok) {
  for (int i = threadIdx.x; i < P; i += kQThreads) {
    double v = __builtin_inf();
    if (i < s) {
      const double x = samp[(int64_t)i * d + f];
      nn_loc += x == x;
      v = nan_to_inf(x);
    }
    sv[i] = v;
  }
  __syncthreads();
  // bitonic sort, ascending
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += kQThreads) {
        const int ij = i ^ j;
        if (ij > i) {
          const double a = sv[i], b = sv[ij];
          const bool up = (i & k) == 0;
          if (up ? (a > b) : (a < b)) {
            sv[i] = b;
            sv[ij] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  }  // bitonic path
  // nn and the distinct count over the first nn (non-NaN) sorted values
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int v_nn = nn_loc;
  for (int o = 32; o > 0; o >>= 1) v_nn += __shfl_xor(v_nn, o);
  if (lane == 0) red_nn[wid] = v_nn;
  __syncthreads();
  int nn = 0;
  for (int w = 0; w < kQThreads / 64; ++w) nn += red_nn[w];
  int k_loc = 0;
  for (int i = threadIdx.x; i < nn; i += kQThreads) k_loc += (i == 0 || sv[i] != sv[i - 1]);
  for (int i = threadIdx.x; i < s; i += kQThreads) sorted[(int64_t)f * s + i] = i < nn ? sv[i] : __builtin_nan("");
  for (int o = 32; o > 0; o >>= 1) k_loc += __shfl_xor(k_loc, o);
  if (lane == 0) red_k[wid] = k_loc;
  __syncthreads();
  int kd = 0;
  for (int w = 0; w < kQThreads / 64; ++w) kd += red_k[w];
  const int nb = max_bins - 1;
  if (kd <= max_bins || nn == 0 || nb < 1) {
    if (threadIdx.x == 0) {
      kdist[f] = kd;
      nthr[f] = 0;
    }
    if (thr32)
      for (int i = threadIdx.x; i < nb; i += kQThreads) thr32[(int64_t)f * nb + i] = 0.f;
    return;  // host path (few distinct values / categorical / empty)
  }
  // the quantile candidates (same operation order as the torch path)
  const double vmax = sv[nn - 1];
  if (threadIdx.x < nb) {
    const int j = threadIdx.x + 1;
    const double tgt = ((double)nn * (double)j) / (double)max_bins;
    int pos = (int)ceil(tgt) - 1;
    pos = pos < 0 ? 0 : (pos > nn - 1 ? nn - 1 : pos);
    double v = sv[pos];
    if (v == vmax) {
      int lo = 0, hi = s;  // first index with sv >= vmax
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sv[mid] < vmax) lo = mid + 1; else hi = mid;
      }
      v = sv[lo > 0 ? lo - 1 : 0];
    }
    int lo = 0, hi = s;  // first index with sv > v
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sv[mid] <= v) lo = mid + 1; else hi = mid;
    }
    const double nx = sv[lo < s ? lo : s - 1];
    cand[threadIdx.x] = (v + nx) / 2.0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0;
    for (int i = 0; i < nb; ++i) {
      const double x = cand[i];
      if (i > 0) {
        const double p = cand[i - 1];
        if (x == p || (x != x && p != p)) continue;
      }
      if (thr32) thr32[(int64_t)f * nb + c] = (float)x;
      thr[(int64_t)f * nb + c++] = x;
    }
    for (int i = c; i < nb; ++i) {
      thr[(int64_t)f * nb + i] = 0.0;
      if (thr32) thr32[(int64_t)f * nb + i] = 0.f;
    }
    nthr[f] = c;
    kdist[f] = kd;
  }
}

}  // namespace

// samp [s][d] fp64 row-major.  Outputs: sorted [d][s], thr [d][max_bins-1], nthr [d], kdist [d] (features with
// kdist <= max_bins need the host path), thr32 (optional) = (float)thr for the binning kernel.  Returns
// hipErrorInvalidValue when s exceeds the LDS capacity.
CDNA_API int cdna_quantile_thresholds(const double* samp, int s, int d, int max_bins, double* sorted, double* thr,
                                      int* nthr, int* kdist, float* thr32, hipStream_t st) {
  if (d <= 0 || s <= 0) return 0;
  if (s > kQMaxS || max_bins < 2 || max_bins > 257) return (int)hipErrorInvalidValue;
  int P = 1;
  while (P < s) P <<= 1;
  const bool radix = s <= kQRadixS;
  size_t lds = (size_t)P * sizeof(double);
  if (radix && lds < sizeof(typename QRadixSort::storage_type)) lds = sizeof(typename QRadixSort::storage_type);
  auto launch = [&](auto kern) {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL(kern, dim3(d), dim3(kQThreads), lds, st, samp, s, d, max_bins, sorted, thr, nthr, kdist,
                       thr32);
  };
  if (radix) launch(quantile_kernel<true>);
  else launch(quantile_kernel<false>);
  return (int)hipGetLastError();
}
