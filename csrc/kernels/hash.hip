// K16 / K17: device hash tables for the relational engine.
//
// K16 hash_insert: dense group ids of int64 keys (groupBy / dropDuplicates / join key codes / distinct).
//   Open addressing with linear probing on a power-of-two table of 8-byte keys (EMPTY = INT64_MIN, a key
//   equal to EMPTY goes to the extra slot P).  One atomicCAS claims an empty slot; every later row with
//   that key only reads it, so low-cardinality keys (10 IoT devices, 7 group values) are L2-resident
//   reads after the first few inserts.  The host turns occupied slots into ranks of the sorted distinct
//   keys, so ids equal torch.unique's inverse (deterministic whatever the insertion race).
//   An insert that probes past `max_probe` raises the overflow flag; the host retries with 2 n slots.
// K16 hash_lookup: the probe side (no inserts): slot of each key or -1.
// K17 dict_encode: Arrow-style strings (int32 offsets + UTF-8 bytes) -> representative row of each distinct
//   string.  Table word = (32-bit hash << 32) | row, claimed by one CAS, so a reader never sees a
//   half-written entry (no spinning on a second word: lanes of one wave cannot wait on each other).  Equal
//   32-bit hashes are resolved by comparing bytes with the representative row, so the encoding is exact.
#include "common.h"

namespace {

constexpr unsigned long long kEmpty = 0x8000000000000000ull;

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void hash_insert_kernel(const unsigned long long* __restrict__ keys, int64_t n,
                                                          unsigned long long* __restrict__ table, int64_t mask,
                                                          int64_t* __restrict__ slot, int max_probe,
                                                          int* __restrict__ overflow) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const unsigned long long k = keys[i];
    if (k == kEmpty) {
      slot[i] = mask + 1;  // the extra slot P
      continue;
    }
    int64_t h = (int64_t)(mix64(k) & (unsigned long long)mask);
    int64_t found = -1;
    for (int p = 0; p < max_probe; ++p) {
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
    slot[i] = found;
    if (found < 0) atomicOr(overflow, 1);
  }
}

__global__ __launch_bounds__(256) void hash_lookup_kernel(const unsigned long long* __restrict__ keys, int64_t n,
                                                          const unsigned long long* __restrict__ table, int64_t mask,
                                                          int has_special, int64_t* __restrict__ slot) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const unsigned long long k = keys[i];
    if (k == kEmpty) {
      slot[i] = has_special ? mask + 1 : -1;
      continue;
    }
    int64_t h = (int64_t)(mix64(k) & (unsigned long long)mask);
    int64_t found = -1;
    for (int64_t p = 0; p <= mask; ++p) {
      const unsigned long long cur = table[h];
      if (cur == k) {
        found = h;
        break;
      }
      if (cur == kEmpty) break;
      h = (h + 1) & mask;
    }
    slot[i] = found;
  }
}

__device__ __forceinline__ unsigned long long str_hash(const uint8_t* p, int len) {
  // FNV-1a over the bytes, then a 64-bit finalizer (table position and stored tag from one value)
  unsigned long long h = 0xCBF29CE484222325ull;
  for (int i = 0; i < len; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
  return mix64(h ^ (unsigned long long)len);
}

__device__ __forceinline__ bool str_eq(const uint8_t* a, int la, const uint8_t* b, int lb) {
  if (la != lb) return false;
  for (int i = 0; i < la; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

__global__ __launch_bounds__(256) void dict_encode_kernel(const int* __restrict__ offs, const uint8_t* __restrict__ data,
                                                          const uint8_t* __restrict__ valid, int64_t n,
                                                          unsigned long long* __restrict__ table, int64_t mask,
                                                          int* __restrict__ rep, int max_probe,
                                                          int* __restrict__ overflow) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (valid && !valid[i]) {  // nulls never become (or match) a representative
      rep[i] = -1;
      continue;
    }
    const int o0 = offs[i], len = offs[i + 1] - o0;
    const unsigned long long h = str_hash(data + o0, len);
    const unsigned long long tag = (h >> 32) | 1ull;  // never 0: the empty word is 0
    const unsigned long long mine = (tag << 32) | (unsigned long long)(uint32_t)i;
    int64_t pos = (int64_t)(h & (unsigned long long)mask);
    int r = -1;
    for (int p = 0; p < max_probe; ++p) {
      unsigned long long cur = __hip_atomic_load(table + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == 0ull) {
        const unsigned long long prev = atomicCAS(table + pos, 0ull, mine);
        if (prev == 0ull) {
          r = (int)i;
          break;
        }
        cur = prev;
      }
      if ((cur >> 32) == tag) {
        const int j = (int)(uint32_t)cur;
        const int q0 = offs[j];
        if (str_eq(data + o0, len, data + q0, offs[j + 1] - q0)) {
          r = j;
          break;
        }
      }
      pos = (pos + 1) & mask;
    }
    rep[i] = r;
    if (r < 0) atomicOr(overflow, 1);
  }
}

// Grouped reductions for few groups (groupBy(...).avg / count / first over 1e8 rows and 50 keys): global
// atomics on a handful of addresses serialise (fp64 adds as CAS loops), so each block accumulates into
// an LDS copy of the G outputs and writes one partial row; the host reduces the [blocks][G] partials.
template <int OP>  // 0: sum of fp64 values (vals == nullptr: count), 1: min of the row index (first row)
__global__ __launch_bounds__(256) void grouped_reduce_kernel(const double* __restrict__ vals,
                                                             const int64_t* __restrict__ gid, int64_t n, int G,
                                                             int64_t rows_per_block, void* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sd = reinterpret_cast<double*>(smem);
  long long* sl = reinterpret_cast<long long*>(smem);
  for (int g = threadIdx.x; g < G; g += 256) {
    if (OP == 0) sd[g] = 0.0;
    else sl[g] = n;
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) {
    const int g = (int)gid[i];
    if (OP == 0) atomicAdd(sd + g, vals ? vals[i] : 1.0);
    else atomicMin(sl + g, (long long)i);
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += 256) {
    if (OP == 0) reinterpret_cast<double*>(partials)[(int64_t)blockIdx.x * G + g] = sd[g];
    else reinterpret_cast<long long*>(partials)[(int64_t)blockIdx.x * G + g] = sl[g];
  }
}

unsigned grid_of(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (unsigned)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

}  // namespace

// table: [mask + 1] u64 initialised to INT64_MIN by the caller; slot: [n] int64 (mask + 1 for the EMPTY key).
CDNA_API int cdna_hash_insert(const void* keys, int64_t n, void* table, int64_t mask, int64_t* slot, int max_probe,
                              int* overflow, hipStream_t st) {
  if (n <= 0) return 0;
  if (((mask + 1) & mask) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(hash_insert_kernel, dim3(grid_of(n)), dim3(256), 0, st,
                     reinterpret_cast<const unsigned long long*>(keys), n,
                     reinterpret_cast<unsigned long long*>(table), mask, slot, max_probe, overflow);
  return (int)hipGetLastError();
}

CDNA_API int cdna_hash_lookup(const void* keys, int64_t n, const void* table, int64_t mask, int has_special,
                              int64_t* slot, hipStream_t st) {
  if (n <= 0) return 0;
  if (((mask + 1) & mask) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(hash_lookup_kernel, dim3(grid_of(n)), dim3(256), 0, st,
                     reinterpret_cast<const unsigned long long*>(keys), n,
                     reinterpret_cast<const unsigned long long*>(table), mask, has_special, slot);
  return (int)hipGetLastError();
}

// table: [mask + 1] u64 zeroed by the caller; rep: [n] int32 representative row of each string (-1: null).
CDNA_API int cdna_dict_encode(const int* offs, const uint8_t* data, const uint8_t* valid, int64_t n, void* table,
                              int64_t mask, int* rep, int max_probe, int* overflow, hipStream_t st) {
  if (n <= 0) return 0;
  if (((mask + 1) & mask) != 0 || n >= (1ll << 31)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(dict_encode_kernel, dim3(grid_of(n)), dim3(256), 0, st, offs, data, valid, n,
                     reinterpret_cast<unsigned long long*>(table), mask, rep, max_probe, overflow);
  return (int)hipGetLastError();
}

// op 0: partials[blocks][G] fp64 sums of vals (nullptr: row counts); op 1: int64 first row per group.
CDNA_API int cdna_grouped_reduce(int op, const double* vals, const int64_t* gid, int64_t n, int G,
                                 int64_t rows_per_block, void* partials, hipStream_t st) {
  if (n <= 0) return 0;
  if (G <= 0 || G > 8192 || rows_per_block <= 0) return (int)hipErrorInvalidValue;
  const unsigned nblk = (unsigned)((n + rows_per_block - 1) / rows_per_block);
  const size_t lds = (size_t)G * 8;
  if (op == 0)
    hipLaunchKernelGGL(grouped_reduce_kernel<0>, dim3(nblk), dim3(256), lds, st, vals, gid, n, G, rows_per_block,
                       partials);
  else
    hipLaunchKernelGGL(grouped_reduce_kernel<1>, dim3(nblk), dim3(256), lds, st, vals, gid, n, G, rows_per_block,
                       partials);
  return (int)hipGetLastError();
}
