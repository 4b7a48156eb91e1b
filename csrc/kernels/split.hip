// K6 split_scan: best split of every active node from its level histogram, in
// one kernel (PLANET's per-level "find best splits" on the
// driver, ML 06 - Decision Trees.py:96-118).
//
// The torch formulation (prefix sums, gains, masks, argmax over [A, d, B])
// launches ~30 small kernels per tree level, ~0.65 ms of a level at any data
// size -- 3 ms of a 46 ms fit at the 8-GPU strong-scaling point (1.25e7 rows
// per GPU).  Here one block owns one node: a thread per feature sums its bins
// (node totals = the feature with the largest weight, as the torch path),
// then scans them left to right in fp64, evaluating the impurity gain of
// every legal threshold; a block argmax picks the best (gain, feature, bin)
// with ties going to the lowest flat index f * B + b (torch.argmax order).
//
// Regression variance gain and XGBoost's second-order gain (with the
// sparsity-aware missing direction: bin 0 = missing, tried on both sides)
// are covered; categorical features and classification impurities stay on
// the torch path (cdnaml/models/tree/engine.py).
#include "common.h"

namespace {

constexpr int kThreads = 128;

struct SplitArgs {
  const double* H;       // [A][d][B][2]
  const int* nthr;       // [d]  legal thresholds b < nthr[f]
  const uint32_t* mask;  // [A][mw] feature-subset bits (null: all features)
  int mw;
  int A, d, B;
  int kind;              // 0 variance (stats: weight, sum), 1 xgb (stats: hess, grad)
  int missing_bin;       // xgb: bin 0 holds missing values; also try sending them right (left = bins 1..b)
  double min_inst, lambda, gamma, mcw;
  double* out;           // [A][8]: gain, f, b, left0, left1, right0, right1, -
  double* tot_out;       // [A][2] node totals
};

__device__ __forceinline__ double gain_of(const SplitArgs& a, double l0, double l1, double r0, double r1, double t0,
                                          double t1, bool* ok) {
  if (a.kind == 0) {
    const double lo = a.min_inst > 1e-12 ? a.min_inst : 1e-12;
    *ok = l0 >= lo && r0 >= lo;
    const double wl = l0 > 1e-300 ? l0 : 1e-300, wr = r0 > 1e-300 ? r0 : 1e-300, wt = t0 > 1e-300 ? t0 : 1e-300;
    return (l1 * l1 / wl + r1 * r1 / wr - t1 * t1 / wt) / wt;
  }
  *ok = l0 >= a.mcw && r0 >= a.mcw && l0 > 0.0 && r0 > 0.0;
  return 0.5 * (l1 * l1 / (l0 + a.lambda) + r1 * r1 / (r0 + a.lambda) - t1 * t1 / (t0 + a.lambda)) - a.gamma;
}

__global__ __launch_bounds__(kThreads) void split_scan_kernel(const SplitArgs a) {
  __shared__ double s_w[kThreads], s_t0[kThreads], s_t1[kThreads], s_g[kThreads];
  __shared__ int s_f[kThreads], s_k[kThreads];
  const int node = blockIdx.x;
  const double* Hn = a.H + (int64_t)node * a.d * a.B * 2;
  // pass 1: per-feature totals; node totals = those of the feature with the most weight (first on ties)
  double bw = -1.0, b0 = 0.0, b1 = 0.0;
  int bf = 0x7FFFFFFF;
  for (int f = threadIdx.x; f < a.d; f += kThreads) {
    double t0 = 0.0, t1 = 0.0;
    const double* hf = Hn + (int64_t)f * a.B * 2;
    for (int b = 0; b < a.B; ++b) {
      t0 += hf[2 * b];
      t1 += hf[2 * b + 1];
    }
    if (t0 > bw) {
      bw = t0;
      b0 = t0;
      b1 = t1;
      bf = f;
    }
  }
  s_w[threadIdx.x] = bw;
  s_t0[threadIdx.x] = b0;
  s_t1[threadIdx.x] = b1;
  s_f[threadIdx.x] = bf;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const int j = threadIdx.x + o;
      if (s_w[j] > s_w[threadIdx.x] || (s_w[j] == s_w[threadIdx.x] && s_f[j] < s_f[threadIdx.x])) {
        s_w[threadIdx.x] = s_w[j];
        s_t0[threadIdx.x] = s_t0[j];
        s_t1[threadIdx.x] = s_t1[j];
        s_f[threadIdx.x] = s_f[j];
      }
    }
    __syncthreads();
  }
  const double t0 = s_t0[0], t1 = s_t1[0];
  __syncthreads();
  // pass 2: every legal threshold of every (sampled) feature
  // candidate keys: f * B + b (missing rows left with bin 0), then d * B + f * B + b (missing rows right);
  // ties go to the lower key, as torch.argmax over the concatenated gains
  double best = -__builtin_inf();
  int bk = 0x7FFFFFFF;
  const int off2 = a.d * a.B;
  for (int f = threadIdx.x; f < a.d; f += kThreads) {
    if (a.mask && !((a.mask[(int64_t)node * a.mw + (f >> 5)] >> (f & 31)) & 1u)) continue;
    const int lim = a.nthr[f] < 0 ? 0 : a.nthr[f];
    const double* hf = Hn + (int64_t)f * a.B * 2;
    const double m0 = hf[0], m1 = hf[1];  // bin 0 (missing values when missing_bin)
    double l0 = 0.0, l1 = 0.0;
    for (int b = 0; b < a.B && b < lim; ++b) {
      l0 += hf[2 * b];
      l1 += hf[2 * b + 1];
      bool ok;
      const double g = gain_of(a, l0, l1, t0 - l0, t1 - l1, t0, t1, &ok);
      if (ok && g == g && g != __builtin_inf() && g != -__builtin_inf() && g > best) {
        best = g;
        bk = f * a.B + b;
      }
      if (a.missing_bin && b >= 1) {
        const double q0 = l0 - m0, q1 = l1 - m1;
        const double g2 = gain_of(a, q0, q1, t0 - q0, t1 - q1, t0, t1, &ok);
        if (ok && g2 == g2 && g2 != __builtin_inf() && g2 != -__builtin_inf() && g2 > best) {
          best = g2;
          bk = off2 + f * a.B + b;
        }
      }
    }
  }
  s_g[threadIdx.x] = best;
  s_k[threadIdx.x] = bk;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const int j = threadIdx.x + o;
      if (s_g[j] > s_g[threadIdx.x] || (s_g[j] == s_g[threadIdx.x] && s_k[j] < s_k[threadIdx.x])) {
        s_g[threadIdx.x] = s_g[j];
        s_k[threadIdx.x] = s_k[j];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double* o = a.out + (int64_t)node * 8;
    const int k0 = s_k[0];
    const bool found = k0 != 0x7FFFFFFF;
    const bool mr = found && k0 >= off2;
    const int k = mr ? k0 - off2 : k0;
    const int f = found ? k / a.B : 0, b = found ? k - (k / a.B) * a.B : 0;
    double l0 = 0.0, l1 = 0.0;
    if (found) {
      const double* hf = Hn + (int64_t)f * a.B * 2;
      for (int q = 0; q <= b; ++q) {
        l0 += hf[2 * q];
        l1 += hf[2 * q + 1];
      }
      if (mr) {
        l0 -= hf[0];
        l1 -= hf[1];
      }
    }
    o[0] = found ? s_g[0] : -__builtin_inf();
    o[1] = f;
    o[2] = b;
    o[3] = l0;
    o[4] = l1;
    o[5] = t0 - l0;
    o[6] = t1 - l1;
    o[7] = mr ? 1.0 : 0.0;
    a.tot_out[node * 2] = t0;
    a.tot_out[node * 2 + 1] = t1;
  }
}

// Wave-parallel K6 for EXACT histograms (int64 fixed-point sums at power-of-two scales, as every record /
// codes path produces: each prefix sum is an exact dyadic number, so any summation order gives the same bits).
// split_scan_kernel walks a feature's B bins serially in one thread, so a level costs one thread's 2 x B-bin walk
// whatever A is (~155 us per level at B = 256: 1.25 ms of a 24 ms boosting round).  Here a wave owns a feature
// (lane l: bins [R l, R l + R)), 16 waves per node: lane prefix + wave scan, the same gain_of per candidate, and
// the same winner as split_scan_kernel including its tie order -- thread t of that kernel walks features
// t, t + 128, ... in (feature, bin, left-then-right) order and keeps the FIRST candidate of its best gain, then the
// block keeps the lowest key among equal gains; the per-feature first candidates kept here reproduce both steps.
constexpr int kWaveMaxD = 4096;

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int R>
__global__ __launch_bounds__(1024) void split_scan_wave_kernel(const SplitArgs a) {
  __shared__ double s_fg[kWaveMaxD];  // per feature: best legal gain (-inf: none)
  __shared__ int s_fc[kWaveMaxD];     // per feature: its first candidate of that gain, bin << 1 | missing-right
  __shared__ double s_w[16], s_t0[16], s_t1[16], s_g[16];
  __shared__ int s_f[16], s_k[16];
  const int node = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const double* Hn = a.H + (int64_t)node * a.d * a.B * 2;
  // pass 1: per-feature totals; node totals = those of the feature with the most weight (lowest feature on ties)
  double bw = -1.0, b0 = 0.0, b1 = 0.0;
  int bf = 0x7FFFFFFF;
  for (int f = wid; f < a.d; f += 16) {
    const double* hf = Hn + (int64_t)f * a.B * 2;
    double t0 = 0.0, t1 = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int b = lane * R + r;
      if (b < a.B) {
        t0 += hf[2 * b];
        t1 += hf[2 * b + 1];
      }
    }
    t0 = wave_sum_d(t0);
    t1 = wave_sum_d(t1);
    if (t0 > bw) {
      bw = t0;
      b0 = t0;
      b1 = t1;
      bf = f;
    }
  }
  if (lane == 0) {
    s_w[wid] = bw;
    s_t0[wid] = b0;
    s_t1[wid] = b1;
    s_f[wid] = bf;
  }
  __syncthreads();
  double t0 = 0.0, t1 = 0.0;
  {
    double w = -2.0;
    int ff = 0x7FFFFFFF;
    for (int i = 0; i < 16; ++i)
      if (s_w[i] > w || (s_w[i] == w && s_f[i] < ff)) {
        w = s_w[i];
        ff = s_f[i];
        t0 = s_t0[i];
        t1 = s_t1[i];
      }
  }
  // pass 2: every legal threshold; per feature the best gain and its first candidate in the serial walk's order
  for (int f = wid; f < a.d; f += 16) {
    double best = -__builtin_inf();
    int code = 0x7FFFFFFF;
    const bool on = !(a.mask && !((a.mask[(int64_t)node * a.mw + (f >> 5)] >> (f & 31)) & 1u));
    if (on) {
      const int lim = a.nthr[f] < 0 ? 0 : a.nthr[f];
      const double* hf = Hn + (int64_t)f * a.B * 2;
      const double m0 = hf[0], m1 = hf[1];
      double p0[R], p1[R];
      double c0 = 0.0, c1 = 0.0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int b = lane * R + r;
        c0 += b < a.B ? hf[2 * b] : 0.0;
        c1 += b < a.B ? hf[2 * b + 1] : 0.0;
        p0[r] = c0;
        p1[r] = c1;
      }
      // exclusive wave scan of the lane totals
      double e0 = c0, e1 = c1;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double u0 = __shfl_up(e0, o, 64), u1 = __shfl_up(e1, o, 64);
        if (lane >= o) {
          e0 += u0;
          e1 += u1;
        }
      }
      e0 -= c0;
      e1 -= c1;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int b = lane * R + r;
        if (b < a.B && b < lim) {
          const double l0 = e0 + p0[r], l1 = e1 + p1[r];
          bool ok;
          const double g = gain_of(a, l0, l1, t0 - l0, t1 - l1, t0, t1, &ok);
          if (ok && g == g && g != __builtin_inf() && g != -__builtin_inf() && g > best) {
            best = g;
            code = b << 1;
          }
          if (a.missing_bin && b >= 1) {
            const double q0 = l0 - m0, q1 = l1 - m1;
            const double g2 = gain_of(a, q0, q1, t0 - q0, t1 - q1, t0, t1, &ok);
            if (ok && g2 == g2 && g2 != __builtin_inf() && g2 != -__builtin_inf() && g2 > best) {
              best = g2;
              code = (b << 1) | 1;
            }
          }
        }
      }
    }
    // wave: the highest gain, the lowest code (the serial walk's first) among equal gains
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double og = __shfl_xor(best, o, 64);
      const int oc = __shfl_xor(code, o, 64);
      if (og > best || (og == best && oc < code)) {
        best = og;
        code = oc;
      }
    }
    if (lane == 0) {
      s_fg[f] = best;
      s_fc[f] = code;
    }
  }
  __syncthreads();
  // the best gain over the node's features
  double G = -__builtin_inf();
  for (int f = lane; f < a.d; f += 64) G = s_fg[f] > G ? s_fg[f] : G;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(G, o, 64);
    G = og > G ? og : G;
  }
  // split_scan_kernel's thread t (features t, t + 128, ...) keeps its first candidate of gain G; the block keeps the
  // lowest key of those
  const int off2 = a.d * a.B;
  int key = 0x7FFFFFFF;
  if (G != -__builtin_inf() && threadIdx.x < 128) {
    for (int f = threadIdx.x; f < a.d; f += 128)
      if (s_fg[f] == G) {
        const int c = s_fc[f];
        key = (c & 1) ? off2 + f * a.B + (c >> 1) : f * a.B + (c >> 1);
        break;
      }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int ok = __shfl_xor(key, o, 64);
    key = ok < key ? ok : key;
  }
  if (lane == 0) s_k[wid] = key;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int k0 = s_k[0] < s_k[1] ? s_k[0] : s_k[1];
    double* o = a.out + (int64_t)node * 8;
    const bool found = k0 != 0x7FFFFFFF;
    const bool mr = found && k0 >= off2;
    const int k = mr ? k0 - off2 : k0;
    const int f = found ? k / a.B : 0, b = found ? k - (k / a.B) * a.B : 0;
    double l0 = 0.0, l1 = 0.0;
    if (found) {
      const double* hf = Hn + (int64_t)f * a.B * 2;
      for (int q = 0; q <= b; ++q) {
        l0 += hf[2 * q];
        l1 += hf[2 * q + 1];
      }
      if (mr) {
        l0 -= hf[0];
        l1 -= hf[1];
      }
    }
    o[0] = found ? G : -__builtin_inf();
    o[1] = f;
    o[2] = b;
    o[3] = l0;
    o[4] = l1;
    o[5] = t0 - l0;
    o[6] = t1 - l1;
    o[7] = mr ? 1.0 : 0.0;
    a.tot_out[node * 2] = t0;
    a.tot_out[node * 2 + 1] = t1;
  }
}

}  // namespace

// kind: 0 = variance (regression trees), 1 = XGBoost gain (| 0x100: exact histograms, split_scan_wave_kernel).
// out [A][8], tot_out [A][2] (fp64).
CDNA_API int cdna_split_scan(const double* H, const int* nthr, const uint32_t* mask, int mw, int A, int d, int B,
                             int kind, int missing_bin, double min_inst, double lambda, double gamma, double mcw,
                             double* out, double* tot_out, hipStream_t st) {
  if (A <= 0) return 0;
  // kind bit 8: exact histograms (power-of-two fixed point) -> the wave-parallel kernel (B <= 256, d <= 4096)
  const bool wave = (kind & 0x100) != 0;
  kind &= 0xFF;
  if (d <= 0 || B <= 0 || (kind != 0 && kind != 1) || (missing_bin && kind != 1)) return (int)hipErrorInvalidValue;
  if ((int64_t)2 * d * B >= 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  SplitArgs a{H, nthr, mask, mw, A, d, B, kind, missing_bin, min_inst, lambda, gamma, mcw, out, tot_out};
  // (B <= 64: one bin per lane leaves the wave kernel slower than the serial walk -- 29.3 vs 22.8 us per level at
  // B = 40 on the headline's levels)
  if (wave && B > 64 && B <= 256 && d <= kWaveMaxD) {
    if (B <= 128) hipLaunchKernelGGL(split_scan_wave_kernel<2>, dim3((unsigned)A), dim3(1024), 0, st, a);
    else hipLaunchKernelGGL(split_scan_wave_kernel<4>, dim3((unsigned)A), dim3(1024), 0, st, a);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(split_scan_kernel, dim3((unsigned)A), dim3(kThreads), 0, st, a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Level histogram assembly (one launch instead of ~8 small torch ops + 3 copies
// per level): every active node's fp64 moments [A][d][B][K] from the level's
// built histograms Hb [nb][d][B][K] -- exact int64 fixed-point sums (raw = 1:
// stat 0 divided by `scale0`, stat 1 by `scale1`) or fp64 -- and, for the
// larger sibling, parent minus sibling from the previous level's histograms.
// map [A][3] = (build slot or -1, parent position, sibling position).
// Nodes are strided over gridDim.y (any A: deep levels of many trees exceed
// the 65535 limit of one grid dimension).
// ---------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(256) void hist_assemble_kernel(const void* __restrict__ Hb, int raw, double scale0,
                                                            double scale1, const double* __restrict__ prev,
                                                            const int* __restrict__ map, int A, int64_t cells, int K,
                                                            double* __restrict__ H) {
  for (int a = blockIdx.y; a < A; a += gridDim.y) {
    const int slot = map[3 * a], par = map[3 * a + 1], sib = map[3 * a + 2];
    const int src = slot >= 0 ? slot : map[3 * sib];
    for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < cells; c += (int64_t)gridDim.x * 256) {
      const int64_t i = (int64_t)src * cells + c;
      double v = raw ? (double)reinterpret_cast<const long long*>(Hb)[i] : reinterpret_cast<const double*>(Hb)[i];
      if (raw) {
        const int k = (int)(c % K);
        if (k == 0 && scale0 != 1.0) v = v / scale0;
        if (k == 1) v = v / scale1;
      }
      if (slot < 0) v = prev[(int64_t)par * cells + c] - v;
      H[(int64_t)a * cells + c] = v;
    }
  }
}
}  // namespace

CDNA_API int cdna_hist_assemble(const void* Hb, int raw, double scale0, double scale1, const double* prev,
                                const int* map, int A, int64_t cells, int K, double* H, hipStream_t st) {
  if (A <= 0 || cells <= 0) return 0;
  int64_t gx = (cells + 255) / 256;
  if (gx > 64) gx = 64;
  const int gy = A < 65535 ? A : 65535;
  hipLaunchKernelGGL(hist_assemble_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, st, Hb, raw, scale0,
                     scale1, prev, map, A, cells, K, H);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// K6 for classification (Gini / entropy on class counts) and for categorical
// features (regression or classification), one block per node -- the torch
// formulation these replace (cdnaml/models/tree/engine.py _best_splits) ran a
// ~15-op chain per level (ML 06 - Decision Trees.py:79-118: StringIndexer'd
// categoricals; Labs/ML 07L:105-141: RandomForestClassifier grid).
//
// Same decisions as that chain: node totals = the feature with the largest
// weight (first on ties); numeric feature f: thresholds b < nthr[f];
// categorical feature f (nthr[f] < 0): its bins ordered by centroid (mean label
// for regression, P(class 1) for binary, the bin's impurity for multiclass;
// empty bins last, stable), split positions j < (#non-empty bins) - 1, the left
// set = the first j + 1 categories of that order (returned as a 256-bit mask);
// argmax over the flat (feature, position) order.  All sums are exact (counts
// and power-of-two fixed-point moments), so the split statistics match.
// ---------------------------------------------------------------------------
namespace {
constexpr int kExMaxK = 32;   // classes
constexpr int kExMaxB = 256;

struct SplitExArgs {
  const double* H;       // [A][d][B][K]
  const int* nthr;       // [d] (< 0: categorical)
  const uint32_t* mask;  // [A][mw] or null
  int mw;
  int A, d, B, K;
  int kind;              // 0 variance (K == 2), 2 gini, 3 entropy
  double min_inst;
  double* out;           // [A][4 + 2K]: gain, f, b, 0, left[K], right[K]
  double* tot_out;       // [A][K]
  uint32_t* cat_out;     // [A][8] left-category bits (categorical winners)
};

// No FMA contraction in the impurity / gain arithmetic: every product is rounded before it is added, as in the
// torch path (engine.py _impurity_from_counts), so centroid ties and gains agree bit for bit.
__device__ __forceinline__ double impurity_c(const double* c, int K, int kind) {
#pragma clang fp contract(off)
  double W = 0.0;
  for (int i = 0; i < K; ++i) W += c[i];
  const double Wc = W > 1e-300 ? W : 1e-300;
  double s = 0.0;
  if (kind == 2) {
    for (int i = 0; i < K; ++i) {
      const double p = c[i] / Wc;
      s += p * p;
    }
    return 1.0 - s;
  }
  for (int i = 0; i < K; ++i) {
    const double p = c[i] / Wc;
    const double lp = p > 0.0 ? log2(p > 1e-300 ? p : 1e-300) : 0.0;
    s += p * lp;
  }
  return -s;
}

// gain of a (left, right) partition; *ok = both sides carry enough weight
__device__ __forceinline__ double gain_ex(const SplitExArgs& a, const double* l, const double* t, double imp_t,
                                          bool* ok) {
#pragma clang fp contract(off)
  double r[kExMaxK];
  for (int i = 0; i < a.K; ++i) r[i] = t[i] - l[i];
  const double lo = a.min_inst > 1e-12 ? a.min_inst : 1e-12;
  if (a.kind == 0) {
    *ok = l[0] >= lo && r[0] >= lo;
    const double wl = l[0] > 1e-300 ? l[0] : 1e-300, wr = r[0] > 1e-300 ? r[0] : 1e-300;
    const double wt = t[0] > 1e-300 ? t[0] : 1e-300;
    return (l[1] * l[1] / wl + r[1] * r[1] / wr - t[1] * t[1] / wt) / wt;
  }
  double WL = 0.0, WR = 0.0, Wt = 0.0;
  for (int i = 0; i < a.K; ++i) {
    WL += l[i];
    WR += r[i];
    Wt += t[i];
  }
  *ok = WL >= lo && WR >= lo;
  return imp_t - WL / Wt * impurity_c(l, a.K, a.kind) - WR / Wt * impurity_c(r, a.K, a.kind);
}

__device__ __forceinline__ bool better(double g, int k, double bg, int bk) {
  return g > bg || (g == bg && k < bk);
}

__global__ __launch_bounds__(128) void split_scan_ex_kernel(const SplitExArgs a) {
  constexpr int TH = 128;
  __shared__ double s_w[TH];
  __shared__ int s_f[TH];
  __shared__ double s_t[kExMaxK];
  __shared__ double s_g[TH];
  __shared__ int s_k[TH];
  __shared__ double s_cent[kExMaxB];
  __shared__ int s_ord[kExMaxB];
  __shared__ double s_bg;
  __shared__ int s_bk;
  const int node = blockIdx.x;
  const int K = a.K, B = a.B;
  const double* Hn = a.H + (int64_t)node * a.d * B * K;
  // ---- node totals: the first feature with the largest weight
  double bw = -1.0;
  int bf = 0x7FFFFFFF;
  for (int f = threadIdx.x; f < a.d; f += TH) {
    const double* hf = Hn + (int64_t)f * B * K;
    double w = 0.0;
    if (a.kind == 0) {
      for (int b = 0; b < B; ++b) w += hf[b * K];
    } else {
      for (int b = 0; b < B; ++b) {
        double wb = 0.0;
        for (int i = 0; i < K; ++i) wb += hf[b * K + i];
        w += wb;
      }
    }
    if (w > bw) {
      bw = w;
      bf = f;
    }
  }
  s_w[threadIdx.x] = bw;
  s_f[threadIdx.x] = bf;
  __syncthreads();
  for (int o = TH / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const int j = threadIdx.x + o;
      if (s_w[j] > s_w[threadIdx.x] || (s_w[j] == s_w[threadIdx.x] && s_f[j] < s_f[threadIdx.x])) {
        s_w[threadIdx.x] = s_w[j];
        s_f[threadIdx.x] = s_f[j];
      }
    }
    __syncthreads();
  }
  const int tf = s_f[0];
  if (threadIdx.x < K) {
    double v = 0.0;
    const double* hf = Hn + (int64_t)tf * B * K;
    for (int b = 0; b < B; ++b) v += hf[b * K + threadIdx.x];
    s_t[threadIdx.x] = v;
  }
  __syncthreads();
  double t[kExMaxK];
  for (int i = 0; i < K; ++i) t[i] = s_t[i];
  const double imp_t = a.kind == 0 ? 0.0 : impurity_c(t, K, a.kind);
  auto in_mask = [&](int f) {
    return !a.mask || ((a.mask[(int64_t)node * a.mw + (f >> 5)] >> (f & 31)) & 1u) != 0u;
  };
  // ---- numeric features: a thread per feature
  double best = -__builtin_inf();
  int bk = 0x7FFFFFFF;
  for (int f = threadIdx.x; f < a.d; f += TH) {
    if (a.nthr[f] < 0 || !in_mask(f)) continue;
    const int lim = a.nthr[f];
    const double* hf = Hn + (int64_t)f * B * K;
    double l[kExMaxK];
    for (int i = 0; i < K; ++i) l[i] = 0.0;
    for (int b = 0; b < B && b < lim; ++b) {
      for (int i = 0; i < K; ++i) l[i] += hf[b * K + i];
      bool ok;
      const double g = gain_ex(a, l, t, imp_t, &ok);
      if (ok && g == g && g != __builtin_inf() && g != -__builtin_inf() && g > best) {
        best = g;
        bk = f * B + b;
      }
    }
  }
  s_g[threadIdx.x] = best;
  s_k[threadIdx.x] = bk;
  __syncthreads();
  for (int o = TH / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o && better(s_g[threadIdx.x + o], s_k[threadIdx.x + o], s_g[threadIdx.x], s_k[threadIdx.x])) {
      s_g[threadIdx.x] = s_g[threadIdx.x + o];
      s_k[threadIdx.x] = s_k[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    s_bg = s_g[0];
    s_bk = s_k[0];
  }
  __syncthreads();
  // ---- categorical features: the block orders one feature's bins by centroid, then thread 0 scans them
  auto order_bins = [&](int f) {
    const double* hf = Hn + (int64_t)f * B * K;
    for (int b = threadIdx.x; b < B; b += TH) {
      double c = __builtin_inf(), W = 0.0;
      if (a.kind == 0) {
        W = hf[b * K];
        c = hf[b * K + 1] / (W > 1e-300 ? W : 1e-300);
      } else {
        for (int i = 0; i < K; ++i) W += hf[b * K + i];
        c = K == 2 ? hf[b * K + 1] / (W > 1e-300 ? W : 1e-300) : impurity_c(hf + b * K, K, a.kind);
      }
      s_cent[b] = W > 0.0 ? c : __builtin_inf();
    }
    __syncthreads();
    // stable rank sort: position of bin b = #{c < cent[b]} + #{c == cent[b], index < b}
    for (int b = threadIdx.x; b < B; b += TH) {
      const double cb = s_cent[b];
      int r = 0;
      for (int j = 0; j < B; ++j) {
        const double cj = s_cent[j];
        r += (cj < cb || (cj == cb && j < b)) ? 1 : 0;
      }
      s_ord[r] = b;
    }
    __syncthreads();
  };
  for (int f = 0; f < a.d; ++f) {
    if (a.nthr[f] >= 0 || !in_mask(f)) continue;  // block-uniform
    order_bins(f);
    if (threadIdx.x == 0) {
      const double* hf = Hn + (int64_t)f * B * K;
      int ncnt = 0;
      for (int b = 0; b < B; ++b) ncnt += s_cent[b] != __builtin_inf() ? 1 : 0;
      double l[kExMaxK];
      for (int i = 0; i < K; ++i) l[i] = 0.0;
      for (int j = 0; j < B && j < ncnt - 1; ++j) {
        const int b = s_ord[j];
        for (int i = 0; i < K; ++i) l[i] += hf[b * K + i];
        bool ok;
        const double g = gain_ex(a, l, t, imp_t, &ok);
        const int key = f * B + j;
        if (ok && g == g && g != __builtin_inf() && g != -__builtin_inf() && better(g, key, s_bg, s_bk)) {
          s_bg = g;
          s_bk = key;
        }
      }
    }
    __syncthreads();
  }
  // ---- the winner's statistics (and category set)
  const int k0 = s_bk;
  const bool found = k0 != 0x7FFFFFFF;
  const int f = found ? k0 / B : 0, pos = found ? k0 - f * B : 0;
  const bool cat = found && a.nthr[f] < 0;
  if (cat) order_bins(f);
  if (threadIdx.x == 0) {
    double* o = a.out + (int64_t)node * (4 + 2 * K);
    double l[kExMaxK];
    for (int i = 0; i < K; ++i) l[i] = 0.0;
    uint32_t bits[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (found) {
      const double* hf = Hn + (int64_t)f * B * K;
      for (int j = 0; j <= pos; ++j) {
        const int b = cat ? s_ord[j] : j;
        for (int i = 0; i < K; ++i) l[i] += hf[b * K + i];
        if (cat) bits[b >> 5] |= 1u << (b & 31);
      }
    }
    o[0] = found ? s_bg : -__builtin_inf();
    o[1] = f;
    o[2] = pos;
    o[3] = 0.0;
    for (int i = 0; i < K; ++i) {
      o[4 + i] = l[i];
      o[4 + K + i] = t[i] - l[i];
      a.tot_out[(int64_t)node * K + i] = t[i];
    }
    for (int w = 0; w < 8; ++w) a.cat_out[(int64_t)node * 8 + w] = bits[w];
  }
}
}  // namespace

// kind: 0 variance (K = 2), 2 gini, 3 entropy.  out [A][4 + 2K], tot_out [A][K], cat_out [A][8].
CDNA_API int cdna_split_scan_ex(const double* H, const int* nthr, const uint32_t* mask, int mw, int A, int d, int B,
                                int K, int kind, double min_inst, double* out, double* tot_out, uint32_t* cat_out,
                                hipStream_t st) {
  if (A <= 0) return 0;
  if (d <= 0 || B <= 0 || B > kExMaxB || K < 1 || K > kExMaxK || (kind == 0 && K != 2) ||
      (kind != 0 && kind != 2 && kind != 3))
    return (int)hipErrorInvalidValue;
  if ((int64_t)d * B >= 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  SplitExArgs a{H, nthr, mask, mw, A, d, B, K, kind, min_inst, out, tot_out, cat_out};
  hipLaunchKernelGGL(split_scan_ex_kernel, dim3((unsigned)A), dim3(128), 0, st, a);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------- split_decode
// The level's split decisions turned into the partition tables on the device, so the row partition can be
// launched right behind K6 while the decisions travel to the host (the host's copy of the same decode builds the
// forest and the next level's layout in the meantime, instead of the GPU idling through a device -> host ->
// device round trip at every level).  Numeric splits only (no categorical sets, no missing-value direction).
//   can[a]        = gain finite, > 0, >= min_gain, node weight >= 2 min_inst, and the level may split
//   split_feat[a] = can ? feature : -1;  split_bin[a] = can ? bin : 0;  cat_off[a] = -1
//   child[2a + s] = index among the active children (in (node, side) order) or -1 (leaf / no split), a child
//                   being active when its weight >= 2 min_inst and the next level is not the last
//   tfirst_next[t]= active children of the trees before t (nodes are ordered by tree)
namespace {

__global__ __launch_bounds__(1024) void split_decode_kernel(const double* __restrict__ so, int sw,
                                                            const double* __restrict__ tot, int tw,
                                                            const int* __restrict__ a_tree, int A, int T,
                                                            double min_inst, double min_gain, int can_level,
                                                            int leaf_children, int missing_bin,
                                                            int* __restrict__ split_feat,
                                                            int* __restrict__ split_bin, int* __restrict__ cat_off,
                                                            uint32_t* __restrict__ masks,
                                                            int* __restrict__ child, int* __restrict__ pref,
                                                            int* __restrict__ tfirst_next, float* __restrict__ lv,
                                                            int vkind, double lam, const int* __restrict__ catm,
                                                            const int* __restrict__ nthr) {
  __shared__ int s_wave[16];
  __shared__ int s_carry;
  // lv (optional) [3A]: leaf values of the rows' destinations at this level, for the partition's margin update
  // -- lv[2a + s] the value of child s of a splitting node when that child is a leaf, lv[2A + a] the value of an
  // active node that does not split; the host forest's values of the same nodes (engine._leaf_values_v, fp64,
  // then fp32): vkind 1 (xgb) -S / (W + lam), else S / W (0 when W = 0).  Entries no row reads are 0.
  auto leafval = [&](double W, double S) -> float {
    return vkind == 1 ? (float)(-S / (W + lam)) : (float)(W > 0.0 ? S / W : 0.0);
  };
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int base = 0; base < 2 * A; base += 1024) {
    const int e = base + threadIdx.x;
    int flag = 0;
    if (e < 2 * A) {
      const int a = e >> 1, s = e & 1;
      const double g = so[(int64_t)a * sw];
      const double W = tot[(int64_t)a * tw];
      const bool can = can_level && g == g && g != __builtin_inf() && g > 0.0 && g >= min_gain && W >= 2.0 * min_inst;
      if (s == 0) {
        const int b = (int)so[(int64_t)a * sw + 2];
        const int fs = (int)so[(int64_t)a * sw + 1];
        // a categorical winner (nthr < 0): left = split_scan_ex's category bitmask of the node
        const bool cat = can && catm != nullptr && nthr != nullptr && fs >= 0 && nthr[fs] < 0;
        // XGBoost's missing-right splits (bin 0 = missing goes right): the left side is the bin set 1..b
        const bool mr = !cat && can && missing_bin && sw >= 8 && so[(int64_t)a * sw + 7] > 0.5;
        split_feat[a] = can ? fs : -1;
        split_bin[a] = can && !mr && !cat ? b : 0;
        cat_off[a] = (mr || cat) ? a : -1;
        if (cat)
          for (int w = 0; w < 8; ++w) masks[(int64_t)a * 8 + w] = (uint32_t)catm[(int64_t)a * 8 + w];
        else if (mr)
          for (int w = 0; w < 8; ++w) {
            uint32_t m = 0u;
            for (int j = 0; j < 32; ++j) {
              const int c = 32 * w + j;
              if (c >= 1 && c <= b) m |= 1u << j;
            }
            masks[(int64_t)a * 8 + w] = m;
          }
      }
      const double cw = so[(int64_t)a * sw + (s == 0 ? 3 : 5)];
      flag = (can && !(cw < 2.0 * min_inst) && !leaf_children) ? 1 : 0;
      if (lv) {
        lv[e] = (can && !flag) ? leafval(cw, so[(int64_t)a * sw + (s == 0 ? 4 : 6)]) : 0.f;
        if (s == 0) lv[2 * A + a] = can ? 0.f : leafval(W, tot[(int64_t)a * tw + 1]);
      }
    }
    // block exclusive scan of the flags
    const uint64_t m = __builtin_amdgcn_ballot_w64(flag != 0);
    const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (lane == 0) s_wave[wid] = __builtin_popcountll(m);
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < 16; ++w) {
      before += w < wid ? s_wave[w] : 0;
      total += s_wave[w];
    }
    const int ex = s_carry + before + below;
    if (e < 2 * A) {
      child[e] = flag ? ex : -1;
      pref[e] = ex;
    }
    __syncthreads();
    if (threadIdx.x == 0) s_carry += total;
    __syncthreads();
  }
  // the first active node of tree t starts its children at pref[2 * a]; trees without active nodes start where the
  // next tree does
  const int total_children = s_carry;
  for (int t = threadIdx.x; t < T; t += 1024) {
    int lo = 0, hi = A;  // first a with a_tree[a] >= t
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a_tree[mid] < t) lo = mid + 1;
      else hi = mid;
    }
    tfirst_next[t] = lo < A ? pref[2 * lo] : total_children;
  }
}

}  // namespace

// so [A][sw] (gain, feature, bin, left0, left1, right0, right1, ...), tot [A][tw]; pref: [2A] int scratch.
// masks: [A][8] bin sets of missing-right splits and categorical winners (cat_off[a] = a), written only for those
// nodes; catm [A][8] / nthr [d] (optional): split_scan_ex's category bitmasks and the features' threshold counts
// (< 0: categorical).
CDNA_API int cdna_split_decode(const double* so, int sw, const double* tot, int tw, const int* a_tree, int A, int T,
                               double min_inst, double min_gain, int can_level, int leaf_children, int missing_bin,
                               int* split_feat, int* split_bin, int* cat_off, uint32_t* masks, int* child, int* pref,
                               int* tfirst_next, float* lv, int vkind, double lam, const int* catm, const int* nthr,
                               hipStream_t st) {
  if (A <= 0 || T <= 0) return 0;
  if (sw < 7 || tw < 1 || (missing_bin && sw < 8) || (lv && tw < 2)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(split_decode_kernel, dim3(1), dim3(1024), 0, st, so, sw, tot, tw, a_tree, A, T, min_inst,
                     min_gain, can_level, leaf_children, missing_bin, split_feat, split_bin, cat_off, masks, child,
                     pref, tfirst_next, lv, vkind, lam, catm, nthr);
  return (int)hipGetLastError();
}
