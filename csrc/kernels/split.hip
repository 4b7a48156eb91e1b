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

}  // namespace

// kind: 0 = variance (regression trees), 1 = XGBoost gain.  out [A][8], tot_out [A][2] (fp64).
CDNA_API int cdna_split_scan(const double* H, const int* nthr, const uint32_t* mask, int mw, int A, int d, int B,
                             int kind, int missing_bin, double min_inst, double lambda, double gamma, double mcw,
                             double* out, double* tot_out, hipStream_t st) {
  if (A <= 0) return 0;
  if (d <= 0 || B <= 0 || (kind != 0 && kind != 1) || (missing_bin && kind != 1)) return (int)hipErrorInvalidValue;
  if ((int64_t)2 * d * B >= 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  SplitArgs a{H, nthr, mask, mw, A, d, B, kind, missing_bin, min_inst, lambda, gamma, mcw, out, tot_out};
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
// K6 over compact feature-subset histograms (subhist.hip): H [A][m][B][2] exact
// int64 (count, sum w q * s1) of each node's m sampled features feats [A][m]
// (ascending).  Same variance gain, legality and tie order (lowest f * B + b)
// as split_scan_kernel on the full [A][d][B][2] fp64 histogram: the fp64
// values are the same exact integers over a power-of-two scale, so every sum
// below is exact and the decisions and child statistics are bit-identical.
// Node totals: the first sampled feature (every feature's bins hold the same
// total weight).  No hist_assemble pass: the int64 sums are read directly.
// ---------------------------------------------------------------------------
namespace {
struct SplitSubArgs {
  const long long* H;
  const uint8_t* feats;
  const int* nthr;
  int A, m, B;
  double scale1;
  double min_inst;
  double* out;
  double* tot_out;
};

__global__ __launch_bounds__(kThreads) void split_scan_sub_kernel(const SplitSubArgs a) {
  __shared__ double s_g[kThreads];
  __shared__ int s_k[kThreads];
  const int node = blockIdx.x;
  const long long* Hn = a.H + (int64_t)node * a.m * a.B * 2;
  const uint8_t* fl = a.feats + (int64_t)node * a.m;
  double t0 = 0.0, t1 = 0.0;
  for (int b = 0; b < a.B; ++b) {  // every thread: the node totals from sampled feature 0
    t0 += (double)Hn[2 * b];
    t1 += (double)Hn[2 * b + 1] / a.scale1;
  }
  double best = -__builtin_inf();
  int bk = 0x7FFFFFFF;
  SplitArgs g{};
  g.kind = 0;
  g.min_inst = a.min_inst;
  for (int k = threadIdx.x; k < a.m; k += kThreads) {
    const int f = fl[k];
    const int lim = a.nthr[f] < 0 ? 0 : a.nthr[f];
    const long long* hf = Hn + (int64_t)k * a.B * 2;
    double l0 = 0.0, l1 = 0.0;
    for (int b = 0; b < a.B && b < lim; ++b) {
      l0 += (double)hf[2 * b];
      l1 += (double)hf[2 * b + 1] / a.scale1;
      bool ok;
      const double gn = gain_of(g, l0, l1, t0 - l0, t1 - l1, t0, t1, &ok);
      if (ok && gn == gn && gn != __builtin_inf() && gn != -__builtin_inf() && gn > best) {
        best = gn;
        bk = f * a.B + b;
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
    const int f = found ? k0 / a.B : 0, b = found ? k0 - f * a.B : 0;
    double l0 = 0.0, l1 = 0.0;
    if (found) {
      int kk = 0;
      while (kk < a.m && fl[kk] != f) ++kk;
      const long long* hf = Hn + (int64_t)kk * a.B * 2;
      for (int q = 0; q <= b; ++q) {
        l0 += (double)hf[2 * q];
        l1 += (double)hf[2 * q + 1] / a.scale1;
      }
    }
    o[0] = found ? s_g[0] : -__builtin_inf();
    o[1] = f;
    o[2] = b;
    o[3] = l0;
    o[4] = l1;
    o[5] = t0 - l0;
    o[6] = t1 - l1;
    o[7] = 0.0;
    a.tot_out[node * 2] = t0;
    a.tot_out[node * 2 + 1] = t1;
  }
}
}  // namespace

CDNA_API int cdna_split_scan_sub(const long long* H, const uint8_t* feats, const int* nthr, int A, int m, int B,
                                 double scale1, double min_inst, double* out, double* tot_out, hipStream_t st) {
  if (A <= 0) return 0;
  if (m <= 0 || B <= 0 || m > 255 || !(scale1 > 0.0)) return (int)hipErrorInvalidValue;
  SplitSubArgs a{H, feats, nthr, A, m, B, scale1, min_inst, out, tot_out};
  hipLaunchKernelGGL(split_scan_sub_kernel, dim3((unsigned)A), dim3(kThreads), 0, st, a);
  return (int)hipGetLastError();
}
