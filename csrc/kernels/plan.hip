// Host-side work planning of the record histograms (no device code).
//
// The level loop plans each record-histogram launch on the host between the compaction's segment totals and the
// histogram launch: the rows-per-block chunk (ops/kernels.py _fill_chunk) and the (start, len, slot) work list
// ordered by relative position inside the segments (_seg_work).  In numpy that was ~250 us per level (a dozen small
// array ops, a bisection, a stable argsort), longer than the compaction scatter it overlaps at the 8-GPU shard
// size, so the GPU idled ~22 us per level; here it is a few microseconds.  Same integers and the same item order
// as the numpy versions (tests/test_kernels_cpu.py compares them).
#include <cstdint>
#include <vector>

#include "common.h"

namespace {

int64_t blocks_for(const std::vector<int64_t>& lens, int64_t c) {
  int64_t b = 0;
  for (int64_t l : lens) b += (l + c - 1) / c;
  return b;
}

}  // namespace

// _fill_chunk: lens [k] (segment lengths), chunk = the largest chunk, B = bins, ncu (0: no round fitting),
// mb = the target block count.
CDNA_API int64_t cdna_fill_chunk(const int64_t* lens_in, int k, int64_t chunk, int B, int ncu, int64_t mb) {
  std::vector<int64_t> lens;
  lens.reserve(k > 0 ? k : 0);
  int64_t total = 0;
  for (int i = 0; i < k; ++i) {
    const int64_t l = lens_in[i] > 0 ? lens_in[i] : 0;
    total += l;
    if (l > 0) lens.push_back(l);
  }
  if (mb < 1) mb = 1;
  int64_t want = (total + mb - 1) / mb;
  if (want < 8192) want = 8192;
  const int64_t c0 = chunk < want ? chunk : want;
  if (ncu <= 0 || B > 64 || c0 >= chunk) return c0;
  const int64_t blocks = blocks_for(lens, c0);
  const int64_t R = blocks / ncu, rem = blocks % ncu;
  if (R < 1 || rem == 0 || rem > ncu / 2) return c0;
  const int64_t cap = R * ncu;
  int64_t lo = c0, hi = chunk;
  if (blocks_for(lens, hi) > cap) return c0;
  const int64_t lo2 = (total + cap - 1) / cap;
  if (lo2 > lo) lo = lo2;
  const int64_t nl = (int64_t)lens.size();
  if (cap > nl) {
    const int64_t hi2 = (total + (cap - nl) - 1) / (cap - nl);
    if (hi2 < hi) hi = hi2;
  }
  while (lo < hi) {
    const int64_t mid = (lo + hi) / 2;
    if (blocks_for(lens, mid) <= cap) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// _seg_work: segs [k][3] {start, len, tag} -> out [m][3] int32 {start, len, tag}, chunks of at most `chunk` rows;
// interleave: stable order by key = j * kmax / k_s (chunk j of a k_s-chunk segment).  Returns m, or -m when
// out_cap < m (nothing written).
CDNA_API int64_t cdna_seg_work(const int64_t* segs, int k, int64_t chunk, int interleave, int32_t* out,
                               int64_t out_cap) {
  if (chunk < 1) return 0;
  int64_t m = 0, kmax = 0, nseg = 0;
  for (int i = 0; i < k; ++i) {
    const int64_t len = segs[3 * i + 1];
    if (len <= 0) continue;
    const int64_t ks = (len + chunk - 1) / chunk;
    m += ks;
    if (ks > kmax) kmax = ks;
    ++nseg;
  }
  if (m > out_cap) return -m;
  auto put = [&](int64_t pos, int i, int64_t j) {
    const int64_t start = segs[3 * i], len = segs[3 * i + 1];
    const int64_t rest = len - j * chunk;
    out[3 * pos] = (int32_t)(start + j * chunk);
    out[3 * pos + 1] = (int32_t)(chunk < rest ? chunk : rest);
    out[3 * pos + 2] = (int32_t)segs[3 * i + 2];
  };
  if (!interleave || nseg <= 1) {
    int64_t pos = 0;
    for (int i = 0; i < k; ++i) {
      const int64_t len = segs[3 * i + 1];
      if (len <= 0) continue;
      const int64_t ks = (len + chunk - 1) / chunk;
      for (int64_t j = 0; j < ks; ++j) put(pos++, i, j);
    }
    return m;
  }
  // counting sort by key (stable: segments, then chunks, in order)
  std::vector<int64_t> cnt((size_t)kmax + 1, 0);
  for (int i = 0; i < k; ++i) {
    const int64_t len = segs[3 * i + 1];
    if (len <= 0) continue;
    const int64_t ks = (len + chunk - 1) / chunk;
    for (int64_t j = 0; j < ks; ++j) ++cnt[(size_t)(j * kmax / ks) + 1];
  }
  for (int64_t q = 1; q <= kmax; ++q) cnt[(size_t)q] += cnt[(size_t)q - 1];
  for (int i = 0; i < k; ++i) {
    const int64_t len = segs[3 * i + 1];
    if (len <= 0) continue;
    const int64_t ks = (len + chunk - 1) / chunk;
    for (int64_t j = 0; j < ks; ++j) put(cnt[(size_t)(j * kmax / ks)]++, i, j);
  }
  return m;
}
