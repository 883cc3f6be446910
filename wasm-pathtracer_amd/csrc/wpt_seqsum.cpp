// Exact sequential f32 sum in binade segments (wpt_seqsum.h).
#include "wpt_seqsum.h"

#include <immintrin.h>

#include <cstring>

namespace wpt {
namespace {

constexpr uint32_t kLim = 1u << 24;  // m of a segment stays below this
constexpr size_t kBlockN = 256;      // elements per vector block

inline uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
inline float bitsf(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// s = m * 2^(es - 150), es = max(biased exponent, 1), m < 2^24 (s finite, >= 0)
struct Seg {
  uint32_t es;
  uint32_t m;
};
inline Seg seg_of(float s) {
  const uint32_t b = fbits(s), e = b >> 23, mant = b & 0x7FFFFFu;
  return {e ? e : 1u, e ? (mant | 0x800000u) : mant};
}
// m <= 2^24 (2^24: the next binade's first value, still exact)
inline float seg_val(Seg g) { return bitsf(((g.es - 1u) << 23) + g.m); }

// Increment of element bits b (sign clear, finite) in segment es: v/u
// rounded half up (< 2^24 + 1 unless `big`), `tie` when v/u is exactly
// half-way, `big` when v's exponent exceeds the segment's (v/u >= 2^24: it
// leaves the segment whatever m is).
struct Inc {
  uint32_t inc, tie, big;
};
inline Inc elem(uint32_t b, uint32_t es) {
  const uint32_t ev = b >> 23;
  const uint32_t mv = (b & 0x7FFFFFu) | (ev ? 0x800000u : 0u);
  const int32_t sh = (int32_t)es - (int32_t)(ev ? ev : 1u);
  const uint32_t shc = sh <= 0 ? 0u : (sh > 31 ? 31u : (uint32_t)sh);
  const uint32_t half = (1u << shc) >> 1;
  return {(mv + half) >> shc, shc != 0u && (mv & ((1u << shc) - 1u)) == half, sh < 0};
}

// Elements i0.. in order, one at a time, from s; returns the new s.
inline float slow(const float* v, size_t i0, size_t i1, float s) {
  for (size_t i = i0; i < i1; i++) {
    const uint32_t b = fbits(v[i]);
    if ((fbits(s) | b) >> 31 || (fbits(s) >> 23) == 0xFFu || (b >> 23) == 0xFFu) {  // not the integer form
      s = s + v[i];
      continue;
    }
    Seg g = seg_of(s);
    const Inc e = elem(b, g.es);
    if (e.big || g.m + e.inc >= kLim) {
      s = s + v[i];  // leaves the binade: the f32 add itself
      continue;
    }
    g.m += e.inc;
    if (e.tie && (g.m & 1u)) g.m--;  // half-way (inc rounded up): the even neighbour
    s = seg_val(g);
  }
  return s;
}

// Vector block (AVX2, 8 lanes): with s = m * u in its binade, element v's
// increment times u is r = (v + C) - C, C = 1.5 * 2^23 * u (v + C rounds to
// a multiple of u; exact for 0 <= v < 2^22 u). Multiples of u below 2^24 u
// add exactly in any order, so the block's r sum in 8 lanes is the integer
// sum of its increments. A block whose elements are all in range and none
// half-way (|r - v| == u/2, exactly computed) and whose sum keeps s in the
// binade advances s by that sum; any other block goes element by element.
__attribute__((target("avx2"))) float run_avx2(const float* v, size_t n, float s) {
  size_t i = 0;
  while (i < n) {
    const size_t k = n - i < kBlockN ? n - i : kBlockN;
    const uint32_t sb = fbits(s), es = sb >> 23;
    if (k == kBlockN && !(sb >> 31) && es < 254u) {
      const uint32_t e = es ? es : 1u;              // u = 2^(e - 150)
      const float u = bitsf(e >= 24u ? (e - 23u) << 23 : 1u << (e - 1u));
      const float top = u * 16777216.0f;            // 2^24 u: the binade's end
      const __m256 C = _mm256_set1_ps(u * 12582912.0f);
      const __m256 lim = _mm256_set1_ps(u * 4194304.0f);
      // no element is half-way in the lowest segment (every float is a multiple of 2^-149)
      const __m256 half = _mm256_set1_ps(e > 1u ? u * 0.5f : __builtin_nanf(""));
      const __m256 zero = _mm256_setzero_ps();
      const __m256 absm = _mm256_castsi256_ps(_mm256_set1_epi32(0x7FFFFFFF));
      __m256 acc[4] = {zero, zero, zero, zero}, bad = zero;
      for (size_t j = 0; j < kBlockN; j += 32) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const __m256 x = _mm256_loadu_ps(v + i + j + 8 * q);
          const __m256 r = _mm256_sub_ps(_mm256_add_ps(x, C), C);
          acc[q] = _mm256_add_ps(acc[q], r);
          const __m256 d = _mm256_and_ps(_mm256_sub_ps(r, x), absm);
          const __m256 ok = _mm256_and_ps(
              _mm256_and_ps(_mm256_cmp_ps(x, zero, _CMP_GE_OQ), _mm256_cmp_ps(x, lim, _CMP_LT_OQ)),
              _mm256_cmp_ps(d, half, _CMP_NEQ_UQ));
          bad = _mm256_or_ps(bad, _mm256_xor_ps(ok, _mm256_castsi256_ps(_mm256_set1_epi32(-1))));
        }
      }
      if (_mm256_testz_ps(bad, bad)) {
        // accumulators, lanes, pairs: every partial is a multiple of u below the total
        const __m256 a = _mm256_add_ps(_mm256_add_ps(acc[0], acc[1]), _mm256_add_ps(acc[2], acc[3]));
        __m128 h = _mm_add_ps(_mm256_castps256_ps128(a), _mm256_extractf128_ps(a, 1));
        h = _mm_add_ps(h, _mm_movehl_ps(h, h));
        h = _mm_add_ss(h, _mm_shuffle_ps(h, h, 1));
        const float t = _mm_cvtss_f32(h);
        if (t < top - s) {  // top - s = (2^24 - m) u, exact
          s = s + t;        // (m + t/u) u < 2^24 u: exact
          i += k;
          continue;
        }
      }
    }
    s = slow(v, i, i + k, s);
    i += k;
  }
  return s;
}

// Elements i0.. in order from s (run_avx2 where the CPU has it).
float run_from(const float* v, size_t n, float s) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  return avx2 ? run_avx2(v, n, s) : slow(v, 0, n, s);
}

// Segment exponent of s, or 0 when s is not in the integer form (negative,
// infinite or NaN, or so large that its segment's end overflows).
inline uint32_t seg_e(float s) {
  const uint32_t b = fbits(s), es = b >> 23;
  if ((b >> 31) || es >= 254u) return 0u;
  return es ? es : 1u;
}

ChunkEff chunk_eff(const float* v, size_t n, uint32_t e) {
  ChunkEff f{e, 1u, 0u};
  for (size_t i = 0; i < n; i++) {
    const uint32_t b = fbits(v[i]);
    if ((b >> 31) || (b >> 23) == 0xFFu) { f.ok = 0u; break; }
    const Inc x = elem(b, e);
    if (x.tie || x.big) { f.ok = 0u; break; }
    f.inc += x.inc;
  }
  return f;
}

}  // namespace

float seq_sum_f32(const float* v, size_t n) { return run_from(v, n, 0.0f); }

void seq_sum_effects(const float* v, size_t n, ChunkEff* eff) {
  const size_t nch = (n + kSumChunk - 1) / kSumChunk;
  double p = 0.0;  // f64 prefix of the chunks before chunk j
  for (size_t j = 0; j < nch; j++) {
    const size_t a = j * kSumChunk, b = a + kSumChunk < n ? a + kSumChunk : n;
    ChunkEff* f = eff + 2 * j;
    f[0] = f[1] = ChunkEff{0u, 0u, 0u};
    const uint32_t e0 = seg_e((float)(p * 0.99)), e1 = seg_e((float)(p * 1.01));
    if (e0) f[0] = chunk_eff(v + a, b - a, e0);
    if (e1 && e1 != e0) f[1] = chunk_eff(v + a, b - a, e1);
    for (size_t i = a; i < b; i++) p += (double)v[i];
  }
}

namespace {
const float* fetch_host(void* ctx, size_t j) { return (const float*)ctx + j * kSumChunk; }
}  // namespace

float seq_sum_walk(const float* v, size_t n, const ChunkEff* eff) {
  return seq_sum_walk_fetch(n, eff, fetch_host, (void*)v);
}

float seq_sum_walk_fetch(size_t n, const ChunkEff* eff, ChunkFetch fetch, void* ctx, uint64_t* resummed) {
  const size_t nch = (n + kSumChunk - 1) / kSumChunk;
  float s = 0.0f;
  for (size_t j = 0; j < nch; j++) {
    const size_t a = j * kSumChunk, b = a + kSumChunk < n ? a + kSumChunk : n;
    const uint32_t e = seg_e(s);
    const ChunkEff* f = nullptr;
    if (e) {
      if (eff[2 * j].e == e) f = &eff[2 * j];
      else if (eff[2 * j + 1].e == e) f = &eff[2 * j + 1];
    }
    if (f && f->ok) {
      Seg g = seg_of(s);  // g.es == e: s in the integer form
      if ((uint64_t)g.m + f->inc < kLim) {
        g.m += (uint32_t)f->inc;
        s = seg_val(g);
        continue;
      }
    }
    if (resummed) ++*resummed;
    s = run_from(fetch(ctx, j), b - a, s);  // from the true s, in order
  }
  return s;
}

}  // namespace wpt
