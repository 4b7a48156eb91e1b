// K15 philox_rng, K13 reg_metrics, K10 kmeans_step, K11 logistic loss/grad,
// K14 auc score histogram.
#include "common.h"

using cdna::kCdf;
using cdna::PoissonCdf;

namespace {

inline unsigned grid_for(int64_t n, int per, unsigned cap) {
  int64_t g = (n + per - 1) / per;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ---------------------------------------------------------------- K15 RNG
__global__ void uniform_kernel(double* __restrict__ out, int64_t n, uint64_t seed, uint64_t offset, uint32_t stream) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = cdna::philox_uniform(seed, offset + (uint64_t)i, stream);
}

// fp32 standard normals for elements offset..offset+n-1 (global element index
// e = row * d + feature, so a table is the same however it is chunked or
// sharded).  One Philox4x32-10 call per quad q = e >> 2 gives two Box-Muller
// pairs: words (0, 1) -> elements 4q, 4q+1 (r cos, r sin), words (2, 3) ->
// 4q+2, 4q+3.  u = (w + 1/2) 2^-32 in fp32: never 0, but w rounds to 24
// significant bits first, so u1 is exactly 1.0 for w >= 2^32 - 128 (2^-25 of
// the draws) and that pair is (0, 0) where exact arithmetic gives a radius of
// at most 2.4e-4; the oracle forms u the same fp32 way.  Hardware log / sin / cos
// (v_log_f32, v_sin_f32, v_cos_f32): HBM-write bound, ~4 B per element, with
// float4 stores when the quad is interior and the output is 16-byte aligned.
// Oracle: cdnaml/ops/philox.py:normal32.
__global__ __launch_bounds__(256) void normal_f32_kernel(float* __restrict__ out, int64_t n, uint64_t seed,
                                                         uint64_t offset, uint32_t stream, int vec) {
  const uint64_t q0 = offset >> 2, q1 = (offset + (uint64_t)n - 1) >> 2;
  constexpr float k2pi = 6.28318530717958647692f, kln2 = 0.69314718055994530942f, s32 = 2.3283064365386963e-10f;
  for (uint64_t q = q0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= q1;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const cdna::u32x4 r = cdna::philox4x32_10(cdna::u32x4{(uint32_t)q, (uint32_t)(q >> 32), stream, 0x4E0Au},
                                              (uint32_t)seed, (uint32_t)(seed >> 32));
    float z[4];
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float u1 = ((float)w[2 * p] + 0.5f) * s32, u2 = ((float)w[2 * p + 1] + 0.5f) * s32;
      const float rad = __fsqrt_rn(-2.f * kln2 * __builtin_amdgcn_logf(u1));
      const float th = k2pi * u2;
      z[2 * p] = rad * __cosf(th);
      z[2 * p + 1] = rad * __sinf(th);
    }
    const int64_t i0 = (int64_t)(4 * q) - (int64_t)offset;  // output index of the quad's first element
    if (vec && i0 >= 0 && i0 + 4 <= n) {
      *reinterpret_cast<float4*>(out + i0) = float4{z[0], z[1], z[2], z[3]};
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i0 + j >= 0 && i0 + j < n) out[i0 + j] = z[j];
    }
  }
}

// Poisson(rate) bootstrap multiplicities for T trees: out[t][i], stream = t + 1
// (rate >= 1 with no bootstrap is handled on the host as all-ones).
// The CDF of poisson_from_uniform's recurrence is tabulated on the host (common.h poisson_cdf): the kernel does
// compares only, no exp / divide.
// One Philox4x32-10 call yields the 32-bit uniforms of 4 consecutive global
// elements (quad q = index >> 2, word = index & 3): 4x fewer Philox rounds
// than one 53-bit double per draw (this kernel shares the GPU with the binning
// kernel it overlaps, so its VALU time is not free).  Bit-identical to
// cdnaml/ops/philox.py:uniform32.  A draw is 8 unrolled integer compares
// against the tabulated CDF (a data-dependent double loop before: k > 7 has
// probability ~1e-5 at rate 1) and an interior quad leaves as one dword store.
__global__ __launch_bounds__(256) void poisson_kernel(uint8_t* __restrict__ out, int T, int64_t n, uint64_t seed,
                                                      uint64_t offset, double rate, PoissonCdf cdf, int packed,
                                                      uint16_t* __restrict__ codes, unsigned* __restrict__ wmax) {
  const int t = blockIdx.y;
  const uint64_t q0 = offset >> 2, q1 = (offset + (uint64_t)n - 1) >> 2;
  uint8_t* o = out + (int64_t)t * n;
  uint16_t* oc = codes + (int64_t)t * n;
  unsigned m = 0u;
  for (uint64_t q = q0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= q1;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const cdna::u32x4 r = cdna::philox4x32_10(cdna::u32x4{(uint32_t)q, (uint32_t)(q >> 32), 0x100u + (uint32_t)t,
                                                          0xB00Fu},
                                              (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
    uint32_t k[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t kk = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) kk += w[j] > cdf.T[i] ? 1u : 0u;
      if (kk == 8u) {
        while (kk < (uint32_t)kCdf && w[j] > cdf.T[kk]) ++kk;
        if (kk == (uint32_t)kCdf) kk = cdna::poisson_from_uniform((double)w[j] * (1.0 / 4294967296.0), rate);
      }
      k[j] = kk > 255u ? 255u : kk;
    }
    const uint64_t g0 = q * 4;
    if (codes) {  // fused row codes (weight << 8 | local node 0, or 0xFF when the weight is 0) + largest weight
#pragma unroll
      for (int j = 0; j < 4; ++j) m = k[j] > m ? k[j] : m;
      uint32_t c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = (k[j] << 8) | (k[j] ? 0u : 0xFFu);
      if (packed && g0 >= offset && g0 + 3 < offset + (uint64_t)n) {
        *reinterpret_cast<uint2*>(oc + (g0 - offset)) = uint2{c[0] | (c[1] << 16), c[2] | (c[3] << 16)};
        continue;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint64_t gi = g0 + j;
        if (gi < offset || gi >= offset + (uint64_t)n) continue;
        oc[gi - offset] = (uint16_t)c[j];
      }
      continue;
    }
    if (packed && g0 >= offset && g0 + 3 < offset + (uint64_t)n) {
      *reinterpret_cast<uint32_t*>(o + (g0 - offset)) = k[0] | (k[1] << 8) | (k[2] << 16) | (k[3] << 24);
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t gi = g0 + j;
      if (gi < offset || gi >= offset + (uint64_t)n) continue;
      o[gi - offset] = (uint8_t)k[j];
    }
  }
  if (codes) {  // one atomic per wave
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned v = (unsigned)__shfl_xor((int)m, off);
      m = v > m ? v : m;
    }
    // most waves find the maximum already there: the read skips their atomic (T x 1024 blocks' worth of
    // same-address atomics serialised in L2 -- ~0.6 ms of the 0.95 ms kernel at 1.25e7 rows x 20 trees)
    if ((threadIdx.x & 63) == 0 && m && m > __hip_atomic_load(wmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(wmax, m);
  }
}

// ------------------------------------------------------- K9 grad / hess
// Per-row gradient and hessian of the boosting objective at the current margin
// F [n][K] (one pass: F, label, weight in; g, h out).  obj: 0 squared error,
// 1 absolute error, 2 pseudo-Huber, 3 Poisson (hessian * exp(max_delta_step
// 0.7), XGBoost), 4 binary logistic, 5 softmax over K classes (label = class
// index).  Same f32 formulas as the torch path in cdnaml/models/xgboost.py.
// gmax (optional, zeroed by the launcher): max |g| as float bits (atomicMax over non-negative float bit patterns;
// a NaN beats +inf), the fixed-point scale's input -- no separate abs + max pass over g per boosting round.
__global__ __launch_bounds__(256) void grad_hess_kernel(const float* __restrict__ F, const float* __restrict__ y,
                                                        const float* __restrict__ w, int64_t n, int K, int obj,
                                                        float* __restrict__ g, float* __restrict__ h,
                                                        int* __restrict__ gmax) {
  int gm = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float yy = y[i];
    const float ww = w ? w[i] : 1.0f;
    if (obj == 5) {
      const float* f = F + i * K;
      float m = f[0];
      for (int k = 1; k < K; ++k) m = fmaxf(m, f[k]);
      float z = 0.0f;
      for (int k = 0; k < K; ++k) z += expf(f[k] - m);
      const int c = (int)yy;
      for (int k = 0; k < K; ++k) {
        const float p = expf(f[k] - m) / z;
        const float gk = (p - (k == c ? 1.0f : 0.0f)) * ww;
        g[i * K + k] = gk;
        h[i * K + k] = fmaxf(2.0f * p * (1.0f - p), 1e-16f) * ww;
        gm = max(gm, __float_as_int(gk) & 0x7FFFFFFF);
      }
      continue;
    }
    const float f = F[i * K];
    float gg, hh;
    if (obj == 0) {
      gg = f - yy;
      hh = 1.0f;
    } else if (obj == 1) {
      const float r = f - yy;
      gg = (float)((r > 0.0f) - (r < 0.0f));
      hh = 1.0f;
    } else if (obj == 2) {
      const float r = f - yy;
      const float sq = sqrtf(1.0f + r * r);
      gg = r / sq;
      hh = 1.0f / (sq * sq * sq);
    } else if (obj == 3) {
      const float e = expf(f);
      gg = e - yy;
      hh = e * 2.0137527074704766f;  // exp(0.7)
    } else {
      const float p = 1.0f / (1.0f + expf(-f));
      gg = p - yy;
      hh = fmaxf(p * (1.0f - p), 1e-16f);
    }
    const float gw = gg * ww;
    g[i] = gw;
    h[i] = hh * ww;
    gm = max(gm, __float_as_int(gw) & 0x7FFFFFFF);
  }
  if (!gmax) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) gm = max(gm, __shfl_xor(gm, o));
  if ((threadIdx.x & 63) == 0 && gm > 0) atomicMax(gmax, gm);
}

// ------------------------------------------------------- K13 reg metrics
// acc: [0]=w [1]=Σw e² [2]=Σw|e| [3]=Σw y [4]=Σw y² [5]=Σw p [6]=Σw p² [7]=Σw y p
__global__ __launch_bounds__(256) void reg_metrics_kernel(const double* __restrict__ y, const double* __restrict__ p,
                                                          const double* __restrict__ w, int64_t n,
                                                          double* __restrict__ acc) {
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double yy = y[i], pp = p[i], ww = w ? w[i] : 1.0;
    const double e = yy - pp;
    s[0] += ww;
    s[1] += ww * e * e;
    s[2] += ww * fabs(e);
    s[3] += ww * yy;
    s[4] += ww * yy * yy;
    s[5] += ww * pp;
    s[6] += ww * pp * pp;
    s[7] += ww * yy * pp;
  }
  __shared__ double red[4][8];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double v = cdna::wave_sum(s[k]);
    if (lane == 0) red[wid][k] = v;
  }
  __syncthreads();
  // per-block partials, summed in block order by reg_metrics_final: deterministic (fp64 atomics made the RMSE of
  // one evaluation differ from the next in the last ulp)
  if (threadIdx.x < 8)
    acc[blockIdx.x * 8 + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                        red[3][threadIdx.x];
}

__global__ void reg_metrics_final(const double* __restrict__ part, int nblk, double* __restrict__ acc) {
  if (threadIdx.x < 8) {
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s += part[b * 8 + threadIdx.x];
    acc[threadIdx.x] = s;
  }
}

// ------------------------------------------------ K14 AUC score histogram
// Scores are mapped into `nb` equal-width buckets over [lo, hi]; per bucket
// the weighted positive and negative counts are accumulated (f64).
__global__ __launch_bounds__(256) void score_hist_kernel(const double* __restrict__ score,
                                                         const double* __restrict__ label, int64_t n, double lo,
                                                         double hi, int nb, double* __restrict__ hist) {
  const double scale = hi > lo ? (double)nb / (hi - lo) : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int b = (int)((score[i] - lo) * scale);
    b = b < 0 ? 0 : (b >= nb ? nb - 1 : b);
    atomicAdd(&hist[b * 2 + (label[i] > 0.5 ? 1 : 0)], 1.0);
  }
}

// -------------------------------------------------------- K10 k-means step
// assign each row to its nearest centre; accumulate per-centre sums/counts
// (LDS-privatised, f64 flush).  centres/sums staged in LDS.  T = float (the
// HBM-bound large-data path; LDS k*d <= 8192) or double (Spark's Double
// vectors at course scale: distances, LDS partial sums and flush all in fp64;
// ds_add_f64 on gfx950; k*d <= 4096).
template <typename T>
__global__ __launch_bounds__(256) void kmeans_kernel(const T* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                     const T* __restrict__ C, int k, int* __restrict__ assign,
                                                     double* __restrict__ sums, double* __restrict__ counts,
                                                     double* __restrict__ cost) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
  T* sc = reinterpret_cast<T*>(smraw);  // [k][d]
  T* ss = sc + k * d;                   // [k][d]
  T* scnt = ss + k * d;                 // [k]
  for (int i = threadIdx.x; i < k * d; i += 256) {
    sc[i] = C[i];
    ss[i] = T(0);
  }
  for (int i = threadIdx.x; i < k; i += 256) scnt[i] = T(0);
  __syncthreads();
  double mycost = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    const T* x = X + r * ldx;
    T best = T(3.4e38);
    int bi = 0;
    for (int c = 0; c < k; ++c) {
      T dist = T(0);
      for (int f = 0; f < d; ++f) {
        const T df = x[f] - sc[c * d + f];
        dist += df * df;
      }
      if (dist < best) {
        best = dist;
        bi = c;
      }
    }
    assign[r] = bi;
    mycost += (double)best;
    if (sums) {
      for (int f = 0; f < d; ++f) atomicAdd(&ss[bi * d + f], x[f]);
      atomicAdd(&scnt[bi], T(1));
    }
  }
  __syncthreads();
  if (sums) {
    for (int i = threadIdx.x; i < k * d; i += 256)
      if (ss[i] != T(0)) atomicAdd(&sums[i], (double)ss[i]);
    for (int i = threadIdx.x; i < k; i += 256)
      if (scnt[i] != T(0)) atomicAdd(&counts[i], (double)scnt[i]);
  }
  if (cost) {
    const double v = cdna::wave_sum(mycost);
    if ((threadIdx.x & 63) == 0) atomicAdd(cost, v);
  }
}

// ------------------------------------------- K11 binary logistic loss/grad
// margin m = x·w + b ; loss += wt*(log1p(exp(m)) - y m) ; grad += wt*(σ(m)-y)·[x, 1]
// One wave per row group; lanes span features (coalesced row reads), the dot
// product is a wave butterfly, gradient accumulates lane-local then is folded
// once per block (f64 global atomics).  grad has d+1 entries (+ intercept).
// Everything past the fp32 feature load is fp64: w, the margin's products and its wave sum (Spark's Double
// margins; the fp32 dot product moved the fitted objective by ~1e-3 relative against the host's fp64 one, and
// L-BFGS at tol 1e-6 then stopped elsewhere).  The kernel stays HBM-bound on the fp32 rows.
// T = double: Spark's Double feature vectors at course scale (the whole margin and gradient exact fp64).
template <typename T>
__global__ __launch_bounds__(256) void logistic_kernel(const T* __restrict__ X, int64_t n, int d, int64_t ldx,
                                                       const double* __restrict__ y, const double* __restrict__ wt,
                                                       const double* __restrict__ w, double b,
                                                       double* __restrict__ grad, double* __restrict__ loss) {
  extern __shared__ __attribute__((aligned(16))) double gsm[];  // [d+1]
  for (int i = threadIdx.x; i <= d; i += 256) gsm[i] = 0.0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wid, nw = (int64_t)gridDim.x * 4;
  constexpr int FPL = 8;  // features per lane handled in registers (d <= 512)
  double gacc[FPL];
  double wl[FPL];
#pragma unroll
  for (int q = 0; q < FPL; ++q) {
    gacc[q] = 0.0;
    const int f = lane + 64 * q;
    wl[q] = f < d ? w[f] : 0.0;
  }
  double gb = 0.0, ls = 0.0;
  for (int64_t r = gw; r < n; r += nw) {
    const T* x = X + r * ldx;
    T xv[FPL];
    double dot = 0.0;
#pragma unroll
    for (int q = 0; q < FPL; ++q) {
      const int f = lane + 64 * q;
      xv[q] = f < d ? x[f] : T(0);
      dot += (double)xv[q] * wl[q];
    }
    const double m = cdna::wave_sum(dot) + b;
    const double yy = y[r], ww = wt ? wt[r] : 1.0;
    const double p = 1.0 / (1.0 + exp(-m));
    const double res = ww * (p - yy);
#pragma unroll
    for (int q = 0; q < FPL; ++q) gacc[q] += res * (double)xv[q];
    if (lane == 0) {
      gb += res;
      ls += ww * ((m > 0 ? m + log1p(exp(-m)) : log1p(exp(m))) - yy * m);
    }
  }
#pragma unroll
  for (int q = 0; q < FPL; ++q) {
    const int f = lane + 64 * q;
    if (f < d) atomicAdd(&gsm[f], gacc[q]);
  }
  if (lane == 0) atomicAdd(&gsm[d], gb);
  __syncthreads();
  for (int i = threadIdx.x; i <= d; i += 256) atomicAdd(&grad[i], gsm[i]);
  if (lane == 0) atomicAdd(loss, ls);
}

}  // namespace

CDNA_API int cdna_uniform(double* out, int64_t n, uint64_t seed, uint64_t offset, uint32_t stream, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(uniform_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, out, n, seed, offset, stream);
  return (int)hipGetLastError();
}

CDNA_API int cdna_normal_f32(float* out, int64_t n, uint64_t seed, uint64_t offset, uint32_t stream,
                             hipStream_t st) {
  if (n <= 0) return 0;
  const int64_t quads = (int64_t)(((offset + (uint64_t)n - 1) >> 2) - (offset >> 2)) + 1;
  const int vec = ((uintptr_t)out % 16 == 0) && (offset % 4 == 0);
  hipLaunchKernelGGL(normal_f32_kernel, dim3(grid_for(quads, 256, 8192)), dim3(256), 0, st, out, n, seed, offset,
                     stream, vec);
  return (int)hipGetLastError();
}

// Level-0 row records from bootstrap weights: code = w << 8 | (w ? 0 : 255)
// (hist5.hip), 16 rows per thread per trip, and the largest weight (drain
// interval of the packed histogram) folded into one atomicMax per block.
__global__ __launch_bounds__(256) void codes_init_kernel(const uint8_t* __restrict__ w, int64_t total,
                                                         uint16_t* __restrict__ codes, unsigned* __restrict__ wmax) {
  unsigned m = 0u;
  const int64_t n16 = total / 16;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n16; q += (int64_t)gridDim.x * 256) {
    const uint4 v = reinterpret_cast<const uint4*>(w)[q];
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
    uint4 o[2];
    uint32_t* ow = reinterpret_cast<uint32_t*>(o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t b0 = (wd[k] >> (16 * h)) & 0xFFu, b1 = (wd[k] >> (16 * h + 8)) & 0xFFu;
        const uint32_t c0 = (b0 << 8) | (b0 ? 0u : 0xFFu), c1 = (b1 << 8) | (b1 ? 0u : 0xFFu);
        ow[2 * k + h] = c0 | (c1 << 16);
        m = max(m, max(b0, b1));
      }
    }
    reinterpret_cast<uint4*>(codes)[2 * q] = o[0];
    reinterpret_cast<uint4*>(codes)[2 * q + 1] = o[1];
  }
  for (int64_t i = n16 * 16 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const uint32_t b = w[i];
    codes[i] = (uint16_t)((b << 8) | (b ? 0u : 0xFFu));
    m = max(m, b);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  __shared__ unsigned red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(wmax, max(max(red[0], red[1]), max(red[2], red[3])));
}

CDNA_API int cdna_codes_init(const uint8_t* w, int64_t total, uint16_t* codes, unsigned* wmax, hipStream_t st) {
  if (total <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(w) & 15) || (reinterpret_cast<uintptr_t>(codes) & 15))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(codes_init_kernel, dim3(grid_for(total / 16 + 1, 256, 4096)), dim3(256), 0, st, w, total, codes,
                     wmax);
  return (int)hipGetLastError();
}

// codes (optional, then out may be null): the row codes [T][n] u16 of the tree engine (codes_init_kernel's
// format) written straight from the draws, and atomicMax of the weights into *wmax (zeroed by the caller) --
// no uint8 weights array, no codes_init pass, no separate max reduction.
CDNA_API int cdna_poisson(uint8_t* out, int T, int64_t n, uint64_t seed, uint64_t offset, double rate,
                          uint16_t* codes, unsigned* wmax, int grid_blocks, hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  if (codes && !wmax) return (int)hipErrorInvalidValue;
  const PoissonCdf cdf = cdna::poisson_cdf(rate);
  // interior quads as dword stores when every tree row starts 4-byte aligned
  const int packed = (offset % 4 == 0) && (n % 4 == 0) &&
                     (codes ? reinterpret_cast<uintptr_t>(codes) % 8 == 0 : reinterpret_cast<uintptr_t>(out) % 4 == 0);
  // grid_blocks > 0 bounds the grid (blocks over all trees; the caller's bound for draws queued beside the fit's
  // prologue on a side stream: a full-chip grid keeps a co-running kernel of 1024-thread blocks -- the quantile
  // sort -- waiting for whole CUs to drain).  Unbounded in series: T x 1024 blocks measured 2.24 ms vs 2.64 ms
  // for 2048 blocks at 1e8 rows x 20 trees (profiles/r4/prologue_ab.md).
  const int max_blocks = grid_blocks;
  unsigned gx = grid_for(n / 4 + 2, 256, 1024);
  if (max_blocks > 0) {
    const unsigned cap = (unsigned)((max_blocks + T - 1) / T);
    gx = gx < cap ? gx : (cap > 0 ? cap : 1u);
  }
  hipLaunchKernelGGL(poisson_kernel, dim3(gx, T), dim3(256), 0, st, out, T, n, seed, offset, rate, cdf, packed, codes,
                     wmax);
  return (int)hipGetLastError();
}

// Row ids r < n whose Philox uniform (seed, offset + r, stream) is below frac -- K.uniform(...) < frac compacted,
// without the n doubles, the mask bytes and the count / scan / write passes (the quantile sample of
// engine._global_sample, ~1e-4 of the rows).  Waves with a kept row claim their slots with one atomicAdd, so
// the ids land in arbitrary order (the caller sorts the <= cap of them); *count (zeroed here) may pass cap,
// then only ids below cap are written and the caller falls back.
__global__ __launch_bounds__(256) void sample_rows_kernel(int64_t n, uint64_t seed, uint64_t offset, uint32_t stream,
                                                          double frac, int64_t* __restrict__ idx, int64_t cap,
                                                          unsigned* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  for (int64_t rb = (int64_t)blockIdx.x * 256; rb < n; rb += (int64_t)gridDim.x * 256) {
    const int64_t r = rb + threadIdx.x;
    const bool keep = r < n && cdna::philox_uniform(seed, offset + (uint64_t)r, stream) < frac;
    const uint64_t m = __builtin_amdgcn_ballot_w64(keep);
    if (m == 0) continue;
    unsigned base = 0u;
    if (lane == 0) base = atomicAdd(count, (unsigned)__builtin_popcountll(m));
    base = (unsigned)__shfl((int)base, 0);
    const unsigned below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (keep && (int64_t)base + below < cap) idx[(int64_t)base + below] = r;
  }
}

// sample_rows_kernel's selection with the kept ids buffered per BLOCK in LDS and claimed with one atomic per block
// on one of 8 counters (the block's blockIdx % 8: its XCD under round-robin placement -- speed only): region r of
// idx [8][rcap] holds counter r's ids.  sample_rows_kernel claims slots with one atomic per wave with a kept row on
// ONE counter: ~10,000 same-address atomics for a 1e4-row sample, serialised at ~11 ns each (108 us of its 116 us
// at 1.25e7 rows).  counts[8] are zeroed by the caller.
__global__ __launch_bounds__(256) void sample_rows_blk_kernel(int64_t n, uint64_t seed, uint64_t offset,
                                                              uint32_t stream, double frac,
                                                              int64_t* __restrict__ idx, int64_t rcap,
                                                              unsigned* __restrict__ counts) {
  constexpr int SB = 1024;
  __shared__ int64_t s_rows[SB];
  __shared__ unsigned s_n, s_base;
  if (threadIdx.x == 0) s_n = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int region = (int)(blockIdx.x & 7u);
  auto flush = [&]() {  // block-uniform
    __syncthreads();
    const unsigned m = s_n;
    if (m) {
      if (threadIdx.x == 0) s_base = atomicAdd(&counts[region], m);
      __syncthreads();
      const unsigned base = s_base;
      for (unsigned i = threadIdx.x; i < m; i += 256)
        if ((int64_t)base + i < rcap) idx[(int64_t)region * rcap + base + i] = s_rows[i];
      __syncthreads();
      if (threadIdx.x == 0) s_n = 0u;
    }
    __syncthreads();
  };
  for (int64_t rb = (int64_t)blockIdx.x * 256; rb < n; rb += (int64_t)gridDim.x * 256) {
    if (s_n + 256u > (unsigned)SB) flush();  // s_n is only written between barriers: the test is block-uniform
    const int64_t r = rb + threadIdx.x;
    const bool keep = r < n && cdna::philox_uniform(seed, offset + (uint64_t)r, stream) < frac;
    const uint64_t mk = __builtin_amdgcn_ballot_w64(keep);
    if (mk) {
      unsigned slot = 0u;
      if (lane == 0) slot = atomicAdd(&s_n, (unsigned)__builtin_popcountll(mk));
      slot = (unsigned)__shfl((int)slot, 0);
      const unsigned below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
      if (keep) s_rows[slot + below] = r;
    }
    __syncthreads();
  }
  flush();
}

// The sampled rows of X as the fp64 quantile sample, straight from sample_rows_blk_kernel's device ids and counts:
// out [cap][d], row i = X[id i] for i < min(total, cap) (ids taken region by region), NaN beyond (the quantile
// kernel sorts NaN last and counts only the non-NaN values, so the padding changes no threshold).  No host round
// trip for the count between the two kernels, and no separate gather / cast launches.
__global__ __launch_bounds__(256) void sample_gather_kernel(const float* __restrict__ X, int64_t ldx, int d,
                                                            const int64_t* __restrict__ idx,
                                                            const unsigned* __restrict__ counts, int64_t rcap,
                                                            int64_t cap, double* __restrict__ out) {
  int64_t pre[9];
  pre[0] = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int64_t c = (int64_t)counts[q] < rcap ? (int64_t)counts[q] : rcap;
    pre[q + 1] = pre[q] + c;
  }
  const int64_t c = pre[8] < cap ? pre[8] : cap;
  const int64_t total = cap * (int64_t)d;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / d;
    const int f = (int)(e - i * d);
    double v = __builtin_nan("");
    if (i < c) {
      int q = 0;
#pragma unroll
      for (int k = 1; k < 8; ++k) q += i >= pre[k] ? 1 : 0;
      v = (double)X[idx[(int64_t)q * rcap + (i - pre[q])] * ldx + f];
    }
    out[e] = v;
  }
}

// Per-node feature subsets (featureSubsetStrategy) as bit words [A, W]: node a keeps the k features with the
// smallest splitmix64(base[a] + f * 0xD6E8FEB86659FD93) -- the host formula of engine.ForestTrainer._feature_masks
// (base[a] = its seed / tree / heap-key mix, computed on the host).  splitmix64 is a bijection and the inputs of a
// node differ, so the k smallest hashes are one well-defined set: the words equal the host's argpartition result.
// One wave per node, the node's d hashes in LDS, each feature's rank by counting smaller hashes (d <= 2048); the
// host version spent up to ~6 ms per deep level on the [A, d] uint64 arrays while the GPU idled.
__device__ __forceinline__ uint64_t splitmix64_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void feature_masks_kernel(const uint64_t* __restrict__ base, int A, int d, int k,
                                                            int W, unsigned* __restrict__ words) {
  extern __shared__ uint64_t fm_hash[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int a = blockIdx.x * 4 + wave;
  uint64_t* h = fm_hash + (size_t)wave * d;
  if (a < A) {
    const uint64_t b = base[a];
    for (int f = lane; f < d; f += 64) h[f] = splitmix64_mix(b + (uint64_t)f * 0xD6E8FEB86659FD93ull);
  }
  __syncthreads();
  if (a >= A) return;
  for (int j = 0; 2 * j < W; ++j) {
    const int f = j * 64 + lane;
    bool sel = false;
    if (f < d) {
      const uint64_t hf = h[f];
      int r = 0;
      for (int g = 0; g < d; ++g) r += h[g] < hf ? 1 : 0;
      sel = r < k;
    }
    const uint64_t m = __ballot(sel);
    if (lane == 0) {
      words[(size_t)a * W + 2 * j] = (unsigned)m;
      if (2 * j + 1 < W) words[(size_t)a * W + 2 * j + 1] = (unsigned)(m >> 32);
    }
  }
}

CDNA_API int cdna_feature_masks(const uint64_t* base, int A, int d, int k, unsigned* words, hipStream_t st) {
  if (A <= 0) return 0;
  if (!base || !words || d <= 0 || d > 2048 || k <= 0 || k > d) return (int)hipErrorInvalidValue;
  const int W = (d + 31) / 32;
  hipLaunchKernelGGL(feature_masks_kernel, dim3((unsigned)((A + 3) / 4)), dim3(256), (size_t)4 * d * 8, st, base, A, d,
                     k, W, words);
  return (int)hipGetLastError();
}

CDNA_API int cdna_sample_rows(int64_t n, uint64_t seed, uint64_t offset, uint32_t stream, double frac, int64_t* idx,
                              int64_t cap, unsigned* count, hipStream_t st) {
  if (!count || (cap > 0 && !idx)) return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(count, 0, sizeof(unsigned), st);
  if (e != hipSuccess || n <= 0) return (int)e;
  hipLaunchKernelGGL(sample_rows_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, n, seed, offset, stream, frac,
                     idx, cap, count);
  return (int)hipGetLastError();
}

// The fused quantile sample: sample_rows_blk_kernel (ids into idx [8][cap], counts [8] zeroed here) then
// sample_gather_kernel (out [cap][d] fp64, NaN-padded).  counts[8] stay on the device for the caller's check.
CDNA_API int cdna_sample_gather(const float* X, int64_t n, int64_t ldx, int d, uint64_t seed, uint64_t offset,
                                uint32_t stream, double frac, int64_t* idx, unsigned* counts, int64_t cap,
                                double* out, hipStream_t st) {
  if (cap <= 0 || d <= 0 || !counts) return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(counts, 0, 8 * sizeof(unsigned), st);
  if (e != hipSuccess) return (int)e;
  if (n > 0)
    hipLaunchKernelGGL(sample_rows_blk_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, n, seed, offset,
                       stream, frac, idx, cap, counts);
  const int64_t total = cap * (int64_t)d;
  hipLaunchKernelGGL(sample_gather_kernel, dim3(grid_for(total, 256, 8192)), dim3(256), 0, st, X, ldx, d, idx, counts,
                     cap, cap, out);
  return (int)hipGetLastError();
}

// fp32 copy of an fp64 column (minus an optional fp64 device shift, subtracted before the rounding) and,
// when amax is given, max |result| as fp32 bits (atomicMax on the int bits: non-negative floats order as their
// bit patterns, and a NaN's (0x7FC00000) beats +inf, so a NaN label surfaces as a NaN maximum).  One pass for
// the forest's label (y.float() + |y|.max() were three full passes) and for the linear fit's shifted label
// (y - mean, then .float(): two).  *amax is zeroed here.
__global__ __launch_bounds__(256) void cast_absmax_kernel(const double* __restrict__ x, int64_t n,
                                                          float* __restrict__ out, int* __restrict__ amax,
                                                          const double* __restrict__ shift) {
  int m = 0;
  const double sh = shift ? shift[0] : 0.0;
  const int64_t n2 = n / 2;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n2; q += (int64_t)gridDim.x * 256) {
    const double2 v = reinterpret_cast<const double2*>(x)[q];
    const float a = (float)(v.x - sh), b = (float)(v.y - sh);
    reinterpret_cast<float2*>(out)[q] = float2{a, b};
    const int ia = __float_as_int(a) & 0x7FFFFFFF, ib = __float_as_int(b) & 0x7FFFFFFF;
    m = max(m, max(ia, ib));
  }
  for (int64_t i = 2 * n2 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float a = (float)(x[i] - sh);
    out[i] = a;
    m = max(m, __float_as_int(a) & 0x7FFFFFFF);
  }
  if (!amax) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0 && m > 0) atomicMax(amax, m);
}

CDNA_API int cdna_cast_absmax(const double* x, int64_t n, float* out, int* amax, const double* shift,
                              hipStream_t st) {
  if (amax) {
    hipError_t e = hipMemsetAsync(amax, 0, sizeof(int), st);
    if (e != hipSuccess) return (int)e;
  }
  if (n <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(x) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 8 != 0)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_absmax_kernel, dim3(grid_for(n / 2 + 1, 256, 512)), dim3(256), 0, st, x, n, out, amax,
                     shift);
  return (int)hipGetLastError();
}

CDNA_API int cdna_reg_metrics(const double* y, const double* p, const double* w, int64_t n, double* part,
                              double* acc, hipStream_t st) {
  if (n <= 0) return 0;
  const unsigned nblk = grid_for(n, 256, 1024);  // part: >= 8 * 1024 doubles of workspace
  hipLaunchKernelGGL(reg_metrics_kernel, dim3(nblk), dim3(256), 0, st, y, p, w, n, part);
  hipLaunchKernelGGL(reg_metrics_final, dim3(1), dim3(64), 0, st, part, (int)nblk, acc);
  return (int)hipGetLastError();
}

CDNA_API int cdna_score_hist(const double* score, const double* label, int64_t n, double lo, double hi, int nb,
                             double* hist, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(score_hist_kernel, dim3(grid_for(n, 256, 1024)), dim3(256), 0, st, score, label, n, lo, hi, nb,
                     hist);
  return (int)hipGetLastError();
}

// f64: X and C are double (else float)
CDNA_API int cdna_kmeans_step(const void* X, int64_t n, int d, int64_t ldx, const void* C, int k, int* assign,
                              double* sums, double* counts, double* cost, int f64, hipStream_t st) {
  if (n <= 0) return 0;
  const size_t lds = (size_t)(2 * k * d + k) * (f64 ? 8 : 4);
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  if (f64)
    hipLaunchKernelGGL(kmeans_kernel<double>, dim3(grid_for(n, 256, 2048)), dim3(256), lds, st,
                       (const double*)X, n, d, ldx, (const double*)C, k, assign, sums, counts, cost);
  else
    hipLaunchKernelGGL(kmeans_kernel<float>, dim3(grid_for(n, 256, 2048)), dim3(256), lds, st,
                       (const float*)X, n, d, ldx, (const float*)C, k, assign, sums, counts, cost);
  return (int)hipGetLastError();
}

CDNA_API int cdna_logistic_grad(const void* X, int64_t n, int d, int64_t ldx, const double* y, const double* wt,
                                const double* w, double b, double* grad, double* loss, int f64, hipStream_t st) {
  if (n <= 0) return 0;
  if (d > 512) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(d + 1) * 8;
  if (f64)
    hipLaunchKernelGGL(logistic_kernel<double>, dim3(grid_for(n, 64, 1024)), dim3(256), lds, st,
                       (const double*)X, n, d, ldx, y, wt, w, b, grad, loss);
  else
    hipLaunchKernelGGL(logistic_kernel<float>, dim3(grid_for(n, 64, 1024)), dim3(256), lds, st,
                       (const float*)X, n, d, ldx, y, wt, w, b, grad, loss);
  return (int)hipGetLastError();
}

CDNA_API int cdna_grad_hess(const float* F, const float* y, const float* w, int64_t n, int K, int obj, float* g,
                            float* h, int* gmax, hipStream_t st) {
  if (gmax) {
    const hipError_t e = hipMemsetAsync(gmax, 0, sizeof(int), st);
    if (e != hipSuccess) return (int)e;
  }
  if (n <= 0) return 0;
  if (obj < 0 || obj > 5 || K < 1 || (obj != 5 && K != 1)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(grad_hess_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, F, y, w, n, K, obj, g, h,
                     gmax);
  return (int)hipGetLastError();
}
