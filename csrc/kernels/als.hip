// K12 ALS normal equations + batched r x r solves.
//
// One ALS half-step solves, for every destination row u (a user, or an item),
//     (Σ_{(u,s) rated} c·v_s v_sᵀ + λ·n_u·I [+ YᵀY]) x_u = Σ c'·v_s
// (MLlib ALS-WR regularisation; implicit prefs use confidence c = 1 + α|r|).
// Reference behaviour: Extra-01 MovieLens ALS, rank 4/12, regParam 0.1,
// nonnegative=True, coldStartStrategy="drop" (E01:136-202).
//
//  * als_accum_kernel: ratings sorted by destination (CSR offsets); one wave per
//    destination row accumulates the r x r Gram and the right-hand side in
//    registers (lane owns entries lane, lane+64, …), loading each source factor
//    row once per rating (broadcast loads).  No [nnz, r, r] temporary.
//  * als_solve_kernel: one wave per system, matrix in LDS.  Right-looking
//    Cholesky + two triangular solves; or (nonnegative) coordinate-descent
//    NNLS, a fixed number of sweeps with wave-reduced dot products.  Systems
//    that are not positive definite report info != 0 and are re-solved by the
//    host with least squares (as the torch path does).
#include "common.h"

namespace {

constexpr int kMaxRank = 32;

template <int EPL>
__global__ __launch_bounds__(64) void als_accum_kernel(int n_dst, const int64_t* __restrict__ off,
                                                       const int* __restrict__ src, const double* __restrict__ rating,
                                                       const double* __restrict__ F, int r, int implicit, double alpha,
                                                       double* __restrict__ A, double* __restrict__ b,
                                                       double* __restrict__ cnt) {
  const int w = blockIdx.x;
  if (w >= n_dst) return;
  const int lane = threadIdx.x;
  const int64_t lo = off[w], hi = off[w + 1];
  const int rr2 = r * r;
  int ei[EPL], ej[EPL];
  double acc[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int e = lane + 64 * k;
    ei[k] = e < rr2 ? e / r : 0;
    ej[k] = e < rr2 ? e - (e / r) * r : 0;
    acc[k] = 0.0;
  }
  double accb = 0.0;
  for (int64_t t = lo; t < hi; ++t) {
    const int s = src[t];
    const double rv = rating[t];
    double ca = 1.0, cb = rv;
    if (implicit) {
      const double c = 1.0 + alpha * fabs(rv);
      ca = c - 1.0;
      cb = rv > 0.0 ? c : 0.0;
    }
    const double* v = F + (int64_t)s * r;
#pragma unroll
    for (int k = 0; k < EPL; ++k) acc[k] += ca * v[ei[k]] * v[ej[k]];
    if (lane < r) accb += cb * v[lane];
  }
  double* Aw = A + (int64_t)w * rr2;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int e = lane + 64 * k;
    if (e < rr2) Aw[e] = acc[k];
  }
  if (lane < r) b[(int64_t)w * r + lane] = accb;
  if (lane == 0) cnt[w] = (double)(hi - lo);
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// M = A[e] + diag_add[e] * I (+ G if non-null), solve M x = b[e].
__global__ __launch_bounds__(64) void als_solve_kernel(int E, int r, const double* __restrict__ A,
                                                       const double* __restrict__ b,
                                                       const double* __restrict__ diag_add,
                                                       const double* __restrict__ G, int nonneg, int sweeps,
                                                       double* __restrict__ x, int* __restrict__ info) {
  __shared__ double M[kMaxRank * kMaxRank];
  __shared__ double y[kMaxRank];
  const int e = blockIdx.x;
  if (e >= E) return;
  const int lane = threadIdx.x;
  const int rr2 = r * r;
  const double da = diag_add[e];
  for (int i = lane; i < rr2; i += 64) {
    const int a = i / r, c = i - (i / r) * r;
    M[i] = A[(int64_t)e * rr2 + i] + (G ? G[i] : 0.0) + (a == c ? da : 0.0);
  }
  if (lane < r) y[lane] = b[(int64_t)e * r + lane];
  __syncthreads();
  if (nonneg) {
    // coordinate descent: x_j = max(0, (b_j - Σ_{k≠j} M_jk x_k) / M_jj)
    double xl = 0.0;  // lane k holds x_k
    for (int it = 0; it < sweeps; ++it) {
      for (int j = 0; j < r; ++j) {
        const double mjj = fmax(M[j * r + j], 1e-12);
        const double part = (lane < r && lane != j) ? M[j * r + lane] * xl : 0.0;
        const double s = wave_sum_d(part);
        const double nv = fmax(0.0, (y[j] - s) / mjj);
        if (lane == j) xl = nv;
      }
    }
    if (lane < r) x[(int64_t)e * r + lane] = xl;
    if (lane == 0) info[e] = 0;
    return;
  }
  // right-looking Cholesky, lower triangle in place
  int bad = 0;
  for (int k = 0; k < r; ++k) {
    const double dkk = M[k * r + k];
    if (!(dkk > 0.0)) bad = 1;
    const double lkk = sqrt(dkk > 0.0 ? dkk : 1.0);
    __syncthreads();
    for (int i = k + 1 + lane; i < r; i += 64) M[i * r + k] /= lkk;
    if (lane == 0) M[k * r + k] = lkk;
    __syncthreads();
    const int m = r - k - 1;
    for (int t = lane; t < m * m; t += 64) {
      const int i = k + 1 + t / m, j = k + 1 + t % m;
      if (j <= i) M[i * r + j] -= M[i * r + k] * M[j * r + k];
    }
    __syncthreads();
  }
  // forward: L z = y (z overwrites y)
  for (int i = 0; i < r; ++i) {
    const double part = lane < i ? M[i * r + lane] * y[lane] : 0.0;
    const double s = wave_sum_d(part);
    __syncthreads();
    if (lane == 0) y[i] = (y[i] - s) / M[i * r + i];
    __syncthreads();
  }
  // backward: Lᵀ x = z
  for (int i = r - 1; i >= 0; --i) {
    const double part = (lane > i && lane < r) ? M[lane * r + i] * y[lane] : 0.0;
    const double s = wave_sum_d(part);
    __syncthreads();
    if (lane == 0) y[i] = (y[i] - s) / M[i * r + i];
    __syncthreads();
  }
  if (lane < r) x[(int64_t)e * r + lane] = y[lane];
  if (lane == 0) info[e] = bad;
}

}  // namespace

CDNA_API int cdna_als_max_rank() { return kMaxRank; }

// Ratings sorted by destination: off[n_dst + 1] CSR offsets, src/rating[nnz].
CDNA_API int cdna_als_accumulate(int n_dst, const int64_t* off, const int* src, const double* rating, const double* F,
                                 int r, int implicit, double alpha, double* A, double* b, double* cnt, hipStream_t st) {
  if (n_dst <= 0) return 0;
  if (r < 1 || r > kMaxRank) return (int)hipErrorInvalidValue;
  const int epl = (r * r + 63) / 64;
  if (epl <= 1)
    hipLaunchKernelGGL(als_accum_kernel<1>, dim3(n_dst), dim3(64), 0, st, n_dst, off, src, rating, F, r, implicit,
                       alpha, A, b, cnt);
  else if (epl <= 4)
    hipLaunchKernelGGL(als_accum_kernel<4>, dim3(n_dst), dim3(64), 0, st, n_dst, off, src, rating, F, r, implicit,
                       alpha, A, b, cnt);
  else
    hipLaunchKernelGGL(als_accum_kernel<16>, dim3(n_dst), dim3(64), 0, st, n_dst, off, src, rating, F, r, implicit,
                       alpha, A, b, cnt);
  return (int)hipGetLastError();
}

CDNA_API int cdna_als_solve(int E, int r, const double* A, const double* b, const double* diag_add, const double* G,
                            int nonneg, int sweeps, double* x, int* info, hipStream_t st) {
  if (E <= 0) return 0;
  if (r < 1 || r > kMaxRank) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(als_solve_kernel, dim3(E), dim3(64), 0, st, E, r, A, b, diag_add, G, nonneg, sweeps, x, info);
  return (int)hipGetLastError();
}
