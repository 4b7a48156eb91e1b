// cdnaml native kernel library — shared device helpers (gfx950 / CDNA4 only).
//
// Every kernel in this library is written for 64-lane wavefronts and launched
// on the caller's HIP stream (the PyTorch current stream).  Host entry points
// are plain `extern "C"` functions so the Python side can bind them with
// ctypes without a torch C++ ABI dependency; they return hipError_t as int.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CDNA_API extern "C" __attribute__((visibility("default")))

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// Checked builds (CDNAML_HIP_DEBUG=1 builds libcdnaml_hip_debug.so with -O1 -g -DCDNA_DEBUG):
// CDNA_DCHECK(cond, code) records the first failed bounds check of a translation unit in a device word and
// evaluates to false, so the caller skips the access instead of faulting the GPU; the host reads and clears the
// word after every call (cdna_debug_status_<unit>, ops/_lib.py) and raises.  Release builds compile it out.
// ---------------------------------------------------------------------------
#ifdef CDNA_DEBUG
static __device__ unsigned int g_cdna_dbg = 0u;
__device__ __forceinline__ bool cdna_dbg_fail(unsigned int code) {
  atomicCAS(&g_cdna_dbg, 0u, code);
  return false;
}
#define CDNA_DCHECK(cond, code) (__builtin_expect(!!(cond), 1) ? true : cdna_dbg_fail(code))
#define CDNA_DEBUG_EXPORT(unit)                                                          \
  CDNA_API unsigned int cdna_debug_status_##unit() {                                     \
    unsigned int v = 0u, z = 0u;                                                         \
    (void)hipDeviceSynchronize();                                                        \
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_cdna_dbg), sizeof(v), 0, hipMemcpyDeviceToHost); \
    if (v) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_cdna_dbg), &z, sizeof(z), 0, hipMemcpyHostToDevice); \
    return v;                                                                            \
  }
#else
#define CDNA_DCHECK(cond, code) true
#define CDNA_DEBUG_EXPORT(unit) \
  CDNA_API unsigned int cdna_debug_status_##unit() { return 0u; }
#endif

namespace cdna {

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG.  Keyed by a 64-bit seed, countered by a
// 64-bit element index plus a 32-bit stream id.  Because the counter is the
// GLOBAL row id, every random column / split mask / bootstrap weight is
// independent of how rows are partitioned across GPUs.
// The host reference in cdnaml/ops/philox.py is bit-identical.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// Uniform double in [0,1) with 53 random bits for element `idx` of `stream`.
__host__ __device__ __forceinline__ double philox_uniform(uint64_t seed, uint64_t idx, uint32_t stream) {
  u32x4 c{(uint32_t)idx, (uint32_t)(idx >> 32), stream, 0x5EEDu};
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  uint64_t bits = ((uint64_t)(r.x >> 5) << 26) | (uint64_t)(r.y >> 6);  // 27 + 26 bits
  return (double)bits * (1.0 / 9007199254740992.0);
}

// Poisson(lambda) draw by CDF inversion (lambda is small: bagging rate).
__host__ __device__ __forceinline__ uint32_t poisson_from_uniform(double u, double lambda) {
  double p = exp(-lambda), F = p;
  uint32_t k = 0;
  while (u > F && k < 255) {
    ++k;
    p *= lambda / (double)k;
    F += p;
  }
  return k;
}

// Tabulated CDF F_0..F_{kCdf-1} of poisson_from_uniform's recurrence (built on the host with the same double
// operations in the same order, so every draw is bit-identical to the loop): u > F_k  <=>  w > floor(F_k 2^32)
// for the 32-bit uniform w = u 2^32, saturated at 2^32 - 1 (never exceeded).
constexpr int kCdf = 32;
struct PoissonCdf {
  uint32_t T[kCdf];
};

inline PoissonCdf poisson_cdf(double rate) {
  PoissonCdf cdf;
  double p = exp(-rate), F = p;
  for (int k = 0; k < kCdf; ++k) {
    const double x = F * 4294967296.0;  // F after k loop iterations, scaled exactly
    cdf.T[k] = x >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)floor(x);
    p *= rate / (double)(k + 1);
    F += p;
  }
  return cdf;
}

// The draw of the 32-bit uniform w: #{k : w > T[k]} (8 unrolled compares, then the rare tail); when the table does
// not saturate within kCdf entries the recurrence itself.
__device__ __forceinline__ uint32_t poisson_draw(uint32_t w, const PoissonCdf& cdf, double rate) {
  uint32_t kk = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) kk += w > cdf.T[i] ? 1u : 0u;
  if (kk == 8u) {
    while (kk < (uint32_t)kCdf && w > cdf.T[kk]) ++kk;
    if (kk == (uint32_t)kCdf) kk = poisson_from_uniform((double)w * (1.0 / 4294967296.0), rate);
  }
  return kk > 255u ? 255u : kk;
}

// Philox stream / constant of the bootstrap draws of tree t (misc.hip poisson_kernel, cdnaml/ops/philox.py)
__device__ __forceinline__ uint32_t bootstrap_uniform(uint64_t seed, uint64_t gi, int t) {
  const uint64_t q = gi >> 2;
  const u32x4 r = philox4x32_10(u32x4{(uint32_t)q, (uint32_t)(q >> 32), 0x100u + (uint32_t)t, 0xB00Fu},
                                (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t j = (uint32_t)(gi & 3u);
  return j == 0 ? r.x : (j == 1 ? r.y : (j == 2 ? r.z : r.w));
}

// XCD-aware bijective block remap (blocks that share an XCD get contiguous work).
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nblk) {
  const uint32_t nx = 8;
  uint32_t q = nblk / nx, r = nblk % nx, x = bid % nx;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / nx;
}

// Blocks that fit the device at once (one "round") for kernel k at this block size / dynamic LDS; 0 when the
// occupancy query fails.  A persistent (grid-stride) launch of exactly this many blocks reads its per-block setup
// (staged tables, LDS clears) once per resident block and has no partial last round.
inline unsigned resident_blocks(const void* k, int threads, size_t lds) {
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, threads, lds) != hipSuccess || per_cu <= 0) return 0;
  return (unsigned)(per_cu * ncu);
}

}  // namespace cdna
