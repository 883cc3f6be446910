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
}
