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

// XCD-aware bijective block remap (blocks that share an XCD get contiguous work).
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nblk) {
  const uint32_t nx = 8;
  uint32_t q = nblk / nx, r = nblk % nx, x = bid % nx;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / nx;
}

}  // namespace cdna
