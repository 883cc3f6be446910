"""The adaptive rounds' mse_sum (sampling_strategy.rs:138-141: `mse_sum +=
mse[..]` in raster order, f32) is computed by wpt_seq_sum in binade segments
of integer increments (wpt_seqsum.h). It must be the plain sequential loop's
bits for every input: checked against numpy's sequential add.accumulate on
error-like data, ties, subnormals, zeros, binade-crossing outliers, and the
values that leave the integer form (negative, -0, inf, NaN)."""
import ctypes

import numpy as np
import pytest


def seq(v):
    v = np.ascontiguousarray(v, np.float32)
    with np.errstate(all="ignore"):  # the overflow / inf / NaN cases
        return np.float32(0.0) if len(v) == 0 else np.add.accumulate(v, dtype=np.float32)[-1]


def fast(wpt, v):
    v = np.ascontiguousarray(v, np.float32)
    return np.float32(wpt.lib().wpt_seq_sum(v.ctypes.data_as(ctypes.c_void_p), len(v)))


def same(a, b):
    return np.asarray(a, np.float32).view(np.uint32) == np.asarray(b, np.float32).view(np.uint32) or (
        np.isnan(a) and np.isnan(b))


def test_accumulate_is_sequential():
    """the checker itself: add.accumulate is the left-to-right f32 chain"""
    rng = np.random.default_rng(3)
    v = rng.random(999, dtype=np.float32) * np.float32(1e-3)
    s = np.float32(0.0)
    for x in v:
        s = np.float32(s + x)
    assert same(s, seq(v))


def cases():
    rng = np.random.default_rng(11)
    n = 1036800  # one 1080p screen half
    yield "errors", (rng.exponential(1.0, n) * 1e-4).astype(np.float32)
    yield "uniform", rng.random(n, dtype=np.float32)
    yield "wide", (rng.random(200000) * 2.0 ** rng.integers(-149, 100, 200000)).astype(np.float32)
    yield "subnormal", rng.integers(0, 1 << 23, 50000).astype(np.uint32).view(np.float32)
    pw = np.ldexp(np.ones(100000), -rng.integers(0, 40, 100000)).astype(np.float32)
    pw[rng.random(100000) < 0.25] = 0
    pw[0] = 1.0
    yield "powers_of_two", pw  # a tie at nearly every addition
    yield "few_bits", np.ldexp(rng.integers(0, 16, 100000).astype(np.float64), -rng.integers(0, 30, 100000)).astype(
        np.float32)
    z = np.zeros(70000, np.float32)
    z[rng.integers(0, 70000, 40)] = rng.random(40, dtype=np.float32) * np.float32(1e20)
    yield "zeros_and_outliers", z
    yield "all_zero", np.zeros(5000, np.float32)
    g = rng.random(30000, dtype=np.float32) * np.float32(1e30)
    yield "near_overflow", np.concatenate([g, np.float32([3e38, 3e38, 1.0])])
    neg = rng.random(20000, dtype=np.float32)
    neg[rng.integers(0, 20000, 30)] *= -1
    neg[rng.integers(0, 20000, 30)] = -0.0
    yield "negative", neg
    special = rng.random(20000, dtype=np.float32)
    special[5000] = np.inf
    yield "inf", special.copy()
    special[9000] = np.nan
    yield "nan", special
    for k in (0, 1, 2, 255, 256, 257, 511, 4097):
        yield f"len{k}", rng.random(k, dtype=np.float32) * np.float32(3.0)


@pytest.mark.parametrize("name,v", list(cases()), ids=[c[0] for c in cases()])
def test_seq_sum_bit_exact(wpt, name, v):
    assert same(seq(v), fast(wpt, v)), (name, seq(v), fast(wpt, v))


def test_seq_sum_random_blocks(wpt):
    """many short random arrays mixing the regimes above"""
    rng = np.random.default_rng(5)
    for t in range(300):
        n = int(rng.integers(0, 3000))
        mode = t % 4
        if mode == 0:
            v = rng.exponential(1.0, n) * 10.0 ** rng.integers(-30, 10)
        elif mode == 1:
            v = np.ldexp(rng.integers(0, 64, n).astype(np.float64), -rng.integers(0, 50, n))
        elif mode == 2:
            v = rng.integers(0, 1 << 31, n).astype(np.uint32).view(np.float32).copy()
            v[~np.isfinite(v)] = 1.0
        else:
            v = rng.random(n) * 2.0 ** rng.integers(-140, 120, n)
        with np.errstate(all="ignore"):
            v = v.astype(np.float32)
        assert same(seq(v), fast(wpt, v)), t


# --- the chunked form the adaptive rounds use (wpt_seqsum.h seq_sum_walk):
# per-chunk effects (here by the host restatement; on the GPU by k_sum_* in
# the rounds and in tests/test_gpu_seqsum.py), then the ordered walk.

def chunked(wpt, v):
    v = np.ascontiguousarray(v, np.float32)
    return np.float32(wpt.lib().wpt_seq_sum_chunks(v.ctypes.data_as(ctypes.c_void_p), len(v)))


@pytest.mark.parametrize("name,v", list(cases()), ids=[c[0] for c in cases()])
def test_seq_sum_chunks_bit_exact(wpt, name, v):
    assert same(seq(v), chunked(wpt, v)), (name, seq(v), chunked(wpt, v))


def walk_cases():
    """inputs that defeat the speculation: the running sum crossing binades
    inside and at the edges of 512-element chunks, sums that stay at a power
    of two, ties at chunk starts, and chunks whose prefix estimate is off"""
    rng = np.random.default_rng(17)
    yield "crossings", np.full(40000, np.float32(0.37), np.float32)
    # chunk sums of exactly a power of two, so s lands on binade edges
    yield "edges", np.full(64 * 512, np.float32(1.0 / 512.0), np.float32)
    ramp = (np.arange(200000, dtype=np.float64) * 1e-6).astype(np.float32)
    yield "ramp", ramp
    spikes = (rng.random(100000) * 1e-3).astype(np.float32)
    spikes[::512] = np.float32(1e3)  # one large element at every chunk start
    yield "spikes", spikes
    ties = np.ones(70000, np.float32)
    ties[::7] = np.float32(0.5)
    yield "ties", ties
    big_then_small = np.concatenate([np.float32([1e9]), (rng.random(60000) * 1e2).astype(np.float32)])
    yield "big_then_small", big_then_small
    yield "errors_4k_half", (rng.exponential(1.0, 3840 * 1080) * 1e-4).astype(np.float32)


@pytest.mark.parametrize("name,v", list(walk_cases()), ids=[c[0] for c in walk_cases()])
def test_seq_sum_chunks_walk_cases(wpt, name, v):
    assert same(seq(v), chunked(wpt, v)), (name, seq(v), chunked(wpt, v))
    assert same(seq(v), fast(wpt, v)), name
