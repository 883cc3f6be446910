// Sequential f32 sum ((0 + v0) + v1) + ... of an adaptive round's pixel
// errors, bit-identical to the reference's loop (sampling_strategy.rs:138-141,
// `mse_sum += mse[..]` in raster order) but without its chain of dependent
// f32 adds (about 4 cycles each: ~0.9 ms per 1080p half, once per round).
//
// While the running sum s stays in one binade [2^(e-127), 2^(e-126)) (or in
// the subnormal range together with the first normal binade), it is m * u
// with an integer m < 2^24 and u = 2^(max(e,1) - 150). Adding a non-negative
// v then rounds the exact m + v/u to the nearest integer, ties to even, so
// the whole chain is integer additions of per-element increments
// round(v/u) — independent of each other except at exact ties, and
// vectorisable. An addition that would leave the binade, a tie, and any
// negative, infinite or NaN element take the plain f32 add, in order. The
// result is the loop's bits for every input (tests/test_seqsum.py).
#pragma once
#include <cstddef>
#include <cstdint>

namespace wpt {
float seq_sum_f32(const float* v, size_t n);

// The same sum from per-chunk effects computed in parallel (the adaptive
// rounds compute them on the GPU, wpt_render.hip k_sum_*): chunk j holds
// elements [j * kSumChunk, (j + 1) * kSumChunk). For a segment exponent e
// (s = m * 2^(e - 150), m < 2^24), a chunk whose elements are all finite,
// non-negative, none half-way and none larger than the segment's range adds
// inc = sum of its elements' increments round(v / u) to m, provided m + inc
// stays below 2^24 (elem() below, per element). Each chunk carries that sum
// for up to two exponents, speculated from the f64 prefix sum of the chunks
// before it (+-1 %). seq_sum_walk runs the chain over the chunks in order: a chunk
// whose computed exponent is s's, flagged ok and keeping s in its binade
// advances s at once; any other chunk is summed from the true s element by
// element. The result is the sequential loop's bits whatever the
// speculation got right (tests/test_seqsum.py).
constexpr uint32_t kSumChunk = 512;
struct ChunkEff {
  uint32_t e;    // segment exponent assumed (0: none)
  uint32_t ok;   // every element in the integer form for e, none half-way
  uint64_t inc;  // sum of the elements' increments in units of u
};
float seq_sum_walk(const float* v, size_t n, const ChunkEff* eff /* [nchunks][2] */);
// The same walk when the elements are not all on the host: fetch(ctx, j)
// returns chunk j's elements, asked only for the chunks the walk re-sums.
typedef const float* (*ChunkFetch)(void* ctx, size_t j);
float seq_sum_walk_fetch(size_t n, const ChunkEff* eff, ChunkFetch fetch, void* ctx, uint64_t* resummed = nullptr);
// host restatement of the per-chunk pass (tests; the GPU computes the same)
void seq_sum_effects(const float* v, size_t n, ChunkEff* eff /* [nchunks][2] */);
}
