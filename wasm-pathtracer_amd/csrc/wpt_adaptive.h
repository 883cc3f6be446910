// wpt_adaptive.h — adaptive sampling kernels (included by wpt_render.hip).
//
// AdaptiveSamplingStrategy (src/graphics/sampling_strategy.rs:77-230) as
// sample ROUNDS, one sequence per screen half (the reference's two
// RenderInstances): round 0 gives every pixel of an adaptive half 4 samples
// (reset, :205-213); each later round first estimates the per-pixel error of
// the current image exactly as next() does (:122-176: clamped mean vs its
// 3x3 and 5x5 Gaussian blurs over the whole viewport, render_target.rs:
// 88-138), then gives the pixel ceil(1 + 32 * scaled_mse) samples. A round of
// a random (non-adaptive) half gives each of its pixels one sample. A round's
// paths are the half's pixels in partition order, each pixel's samples
// consecutive; sample s of pixel p always uses the stream path_seed(seed, p,
// s), so the image does not depend on batching.
#pragma once

// RenderTarget::read_clamped (render_target.rs:75-79, clamp :214-216):
// max(0) then min(1), so a NaN (0/0) reads as 0.
__device__ __forceinline__ V3 read_clamped(const float4* __restrict__ acc, const uint32_t* __restrict__ cnt,
                                           uint32_t i) {
  const float4 a = acc[i];
  const float c = (float)cnt[i];
  return mk(fminf(fmaxf(a.x / c, 0.0f), 1.0f), fminf(fmaxf(a.y / c, 0.0f), 1.0f),
            fminf(fmaxf(a.z / c, 0.0f), 1.0f));
}

// Order-preserving u32 key of a float (every non-NaN value), and back.
__device__ __host__ __forceinline__ uint32_t f_key(uint32_t b) { return b ^ ((b >> 31) ? 0xFFFFFFFFu : 0x80000000u); }
__device__ __host__ __forceinline__ uint32_t f_unkey(uint32_t k) { return k ^ ((k >> 31) ? 0x80000000u : 0xFFFFFFFFu); }

// Per-pixel error of one screen half [x0, x1) x [0, H) (sampling_strategy.rs:
// 138-141): mse = max(|v0 - g3|^2, |v0 - g5|^2), stored in the half's raster
// order. mm = {min key, max key} of the non-NaN errors (:142-144's min / max
// folds with fminf / fmaxf, which skip NaN; min and max do not depend on the
// order), reduced per wave, one atomic each; the caller initialises mm to
// {key(+inf), key(-inf)}, the folds' start values.
// Computed on 16 x 16 pixel tiles: the block first stages the clamped means
// of its tile plus the 2-pixel halo in LDS (each pixel's read_clamped once
// instead of once per tap: 34 taps, 3 divisions each), then every thread runs
// the reference's tap loops (gaussian3 / gaussian5 with read_mul) over LDS,
// in the same order with the same weights (a tap outside the viewport adds
// ZERO with weight 0).
constexpr int kMseTile = 16;
constexpr int kMseHalo = kMseTile + 4;
__global__ void __launch_bounds__(kBlock) k_mse_tiled(const float4* __restrict__ acc, const uint32_t* __restrict__ cnt,
                                                      uint32_t W, uint32_t H, uint32_t x0, uint32_t x1,
                                                      float* __restrict__ mse, uint32_t* __restrict__ bmm) {
  __shared__ float sv[3][kMseHalo * kMseHalo];
  __shared__ uint8_t s_in[kMseHalo * kMseHalo];
  const int tx0 = (int)x0 + (int)blockIdx.x * kMseTile, ty0 = (int)blockIdx.y * kMseTile;
  for (int k = threadIdx.x; k < kMseHalo * kMseHalo; k += kBlock) {
    const int px = tx0 - 2 + k % kMseHalo, py = ty0 - 2 + k / kMseHalo;
    const bool in = px >= 0 && py >= 0 && px < (int)W && py < (int)H;
    V3 v = mk(0.0f, 0.0f, 0.0f);
    if (in) v = read_clamped(acc, cnt, (uint32_t)py * W + (uint32_t)px);
    sv[0][k] = v.x;
    sv[1][k] = v.y;
    sv[2][k] = v.z;
    s_in[k] = in ? 1 : 0;
  }
  __syncthreads();
  const uint32_t rw = x1 - x0;
  const int lx = (int)(threadIdx.x % kMseTile), ly = (int)(threadIdx.x / kMseTile);
  const int x = tx0 + lx, y = ty0 + ly;
  uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
  if (x < (int)x1 && y < (int)H) {
    constexpr float g3[9] = {1, 2, 1, 2, 4, 2, 1, 2, 1};
    constexpr float g5[25] = {1, 4, 6, 4, 1, 4, 16, 24, 16, 4, 6, 24, 36, 24, 6, 4, 16, 24, 16, 4, 1, 4, 6, 4, 1};
    const int c = (ly + 2) * kMseHalo + (lx + 2);
    const V3 v0 = mk(sv[0][c], sv[1][c], sv[2][c]);
    V3 gg[2];
#pragma unroll
    for (int r = 1; r <= 2; r++) {
      const int D = 2 * r + 1;
      float sum = 0.0f;
      V3 a = mk(0.0f, 0.0f, 0.0f);
      for (int vy = 0; vy < D; vy++) {
        for (int vx = 0; vx < D; vx++) {
          const int k = (ly + 2 + vy - r) * kMseHalo + (lx + 2 + vx - r);
          const float m = r == 1 ? g3[vy * 3 + vx] : g5[vy * 5 + vx];
          if (!s_in[k]) {
            a = add(a, mk(0.0f, 0.0f, 0.0f));
            sum += 0.0f;
          } else {
            a = add(a, mk(m * sv[0][k], m * sv[1][k], m * sv[2][k]));
            sum += m;
          }
        }
      }
      gg[r - 1] = mk(a.x / sum, a.y / sum, a.z / sum);
    }
    const V3 d1 = sub(v0, gg[0]), d2 = sub(v0, gg[1]);
    const float m = fmaxf(dot(d1, d1), dot(d2, d2));
    mse[(uint32_t)y * rw + (uint32_t)(x - (int)x0)] = m;
    if (m == m) kmin = kmax = f_key(__float_as_uint(m));
  }
  // min / max keys: waves, then the block, then one pair per block into
  // bmm (k_mm_reduce folds them: one-address atomics from every wave of a
  // 1M-pixel half serialise at the memory side)
  for (int off = 32; off > 0; off >>= 1) {
    kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, off, 64));
    kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, off, 64));
  }
  __shared__ uint32_t s_mm[2][kBlock / 64];
  if ((threadIdx.x & 63u) == 0) {
    s_mm[0][threadIdx.x >> 6] = kmin;
    s_mm[1][threadIdx.x >> 6] = kmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < kBlock / 64; w++) {
      kmin = min(kmin, s_mm[0][w]);
      kmax = max(kmax, s_mm[1][w]);
    }
    const uint32_t b = blockIdx.y * gridDim.x + blockIdx.x;
    bmm[2 * b] = kmin;
    bmm[2 * b + 1] = kmax;
  }
}

// Folds the per-block {min, max} keys of k_mse_tiled into mm.
__global__ void __launch_bounds__(1024) k_mm_reduce(const uint32_t* __restrict__ bmm, uint32_t nb,
                                                    uint32_t* __restrict__ mm) {
  uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
    kmin = min(kmin, bmm[2 * i]);
    kmax = max(kmax, bmm[2 * i + 1]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, off, 64));
    kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, off, 64));
  }
  __shared__ uint32_t s_mm[2][16];
  if ((threadIdx.x & 63u) == 0) {
    s_mm[0][threadIdx.x >> 6] = kmin;
    s_mm[1][threadIdx.x >> 6] = kmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < blockDim.x / 64; w++) {
      kmin = min(kmin, s_mm[0][w]);
      kmax = max(kmax, s_mm[1][w]);
    }
    // no error is a number: the folds' start values, +inf / -inf
    mm[0] = kmin == 0xFFFFFFFFu ? f_key(0x7F800000u) : kmin;
    mm[1] = kmax == 0u ? f_key(0xFF800000u) : kmax;
  }
}

// The adaptive round's mse_sum (sampling_strategy.rs:138-141), the sequential
// f32 sum of a half's errors, from per-chunk effects computed here in
// parallel and walked in order on the host (seq_sum_walk, wpt_seqsum.h: the
// walk re-sums any chunk whose effect does not apply, so the result is the
// loop's bits whatever these kernels speculate). One wave per kSumChunk
// elements. k_sum_chunks: each chunk's f64 sum; k_sum_scan: their exclusive
// prefix (one block); k_sum_eff: per chunk, for the one or two segment
// exponents its start can have (prefix x 0.99 / 1.01), the sum of its
// elements' increments and whether all of them are in the integer form.
__device__ __forceinline__ uint32_t sum_seg_e(float s) {
  const uint32_t b = __float_as_uint(s), es = b >> 23;
  if ((b >> 31) || es >= 254u) return 0u;
  return es ? es : 1u;
}

__global__ void __launch_bounds__(kBlock) k_sum_chunks(const float* __restrict__ v, uint32_t n,
                                                       double* __restrict__ s64) {
  const uint32_t w = (blockIdx.x * kBlock + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
  const uint64_t a = (uint64_t)w * kSumChunk;
  if (a >= n) return;  // wave-uniform
  double s = 0.0;
  for (uint32_t k = lane; k < kSumChunk; k += 64u)
    if (a + k < n) s += (double)v[a + k];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0u) s64[w] = s;
}

__global__ void __launch_bounds__(256) k_sum_scan(double* __restrict__ s64, uint32_t nch) {
  __shared__ double part[256];
  const uint32_t t = threadIdx.x, per = (nch + 255u) / 256u;
  const uint32_t a = t * per, b = min(nch, a + per);
  double acc = 0.0;
  for (uint32_t i = a; i < b; i++) acc += s64[i];
  part[t] = acc;
  __syncthreads();
  if (t == 0u) {
    double r = 0.0;
    for (uint32_t k = 0; k < 256u; k++) {
      const double x = part[k];
      part[k] = r;
      r += x;
    }
  }
  __syncthreads();
  double r = part[t];
  for (uint32_t i = a; i < b; i++) {
    const double x = s64[i];
    s64[i] = r;
    r += x;
  }
}

__global__ void __launch_bounds__(kBlock) k_sum_eff(const float* __restrict__ v, uint32_t n,
                                                    const double* __restrict__ prefix, ChunkEff* __restrict__ eff,
                                                    uint32_t* __restrict__ need) {
  const uint32_t w = (blockIdx.x * kBlock + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
  const uint64_t a = (uint64_t)w * kSumChunk;
  if (a >= n) return;  // wave-uniform
  const double p = prefix[w];
  // the f32 chain drifts from the f64 prefix by far less than 1 % on error
  // data: the one or two exponents within +-1 % of the prefix
  const uint32_t e0 = sum_seg_e((float)(p * 0.99)), e1 = sum_seg_e((float)(p * 1.01));
  // the chunks the host walk will probably re-sum (their elements are copied
  // ahead, k_sum_pack): the first, any whose running sum may cross a binade
  // (its start - 0.2 % and its end + 0.2 % in different ones), any not in the
  // integer form for its candidates
  double cs = 0.0;
  for (uint32_t k = lane; k < kSumChunk; k += 64u)
    if (a + k < n) cs += (double)v[a + k];
  for (int o = 32; o > 0; o >>= 1) cs += __shfl_xor(cs, o, 64);
  bool any_ok = false;
  for (uint32_t c = 0; c < 2u; c++) {
    const uint32_t e = c ? e1 : e0;
    if (e == 0u || (c && e1 == e0)) {
      if (lane == 0u) eff[2 * w + c] = ChunkEff{0u, 0u, 0ull};
      continue;
    }
    unsigned long long inc = 0ull;
    bool ok = true;
    for (uint32_t k = lane; k < kSumChunk; k += 64u) {
      if (a + k >= n) break;
      const uint32_t b = __float_as_uint(v[a + k]);
      if ((b >> 31) || (b >> 23) == 0xFFu) { ok = false; continue; }
      // wpt_seqsum.cpp elem(): round(v / u) half up, the half-way and
      // out-of-segment cases flagged
      const uint32_t ev = b >> 23;
      const uint32_t mv = (b & 0x7FFFFFu) | (ev ? 0x800000u : 0u);
      const int32_t sh = (int32_t)e - (int32_t)(ev ? ev : 1u);
      const uint32_t shc = sh <= 0 ? 0u : (sh > 31 ? 31u : (uint32_t)sh);
      const uint32_t half = (1u << shc) >> 1;
      const bool tie = shc != 0u && (mv & ((1u << shc) - 1u)) == half;
      if (tie || sh < 0) { ok = false; continue; }
      inc += (mv + half) >> shc;
    }
    for (int o = 32; o > 0; o >>= 1) inc += __shfl_xor(inc, o, 64);
    ok = !__any(!ok);
    any_ok = any_ok || ok;
    if (lane == 0u) eff[2 * w + c] = ChunkEff{e, ok ? 1u : 0u, inc};
  }
  if (lane == 0u)
    need[w] = (w == 0u || !any_ok || sum_seg_e((float)(p * 0.998)) != sum_seg_e((float)((p + cs) * 1.002)) ||
               !(cs == cs)) ? 1u : 0u;
}

// One block: the list of chunks k_sum_eff marked (list[0] = their count,
// list[1..] = their indices in order) and the elements of the first
// kSumFetch of them packed into fb (fb[k * kSumChunk ..] = the k-th marked
// chunk), so that one copy brings the walk the chunks it will re-sum.
constexpr uint32_t kSumFetch = 64;
__global__ void __launch_bounds__(1024) k_sum_pack(const float* __restrict__ v, uint32_t n, uint32_t nch,
                                                   const uint32_t* __restrict__ need, uint32_t* __restrict__ list,
                                                   float* __restrict__ fb) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t s_list[kSumFetch];
  __shared__ uint32_t s_total;
  const uint32_t t = threadIdx.x, per = (nch + 1023u) / 1024u;
  const uint32_t a = t * per, b = min(nch, a + per);
  uint32_t c = 0;
  for (uint32_t i = a; i < b; i++) c += need[i];
  part[t] = c;
  __syncthreads();
  if (t == 0u) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < 1024u; k++) {
      const uint32_t x = part[k];
      part[k] = r;
      r += x;
    }
    list[0] = r;
    s_total = r;
  }
  __syncthreads();
  uint32_t pos = part[t];
  for (uint32_t i = a; i < b; i++)
    if (need[i]) {
      list[1 + pos] = i;
      if (pos < kSumFetch) s_list[pos] = i;
      pos++;
    }
  __syncthreads();
  const uint32_t nf = min(s_total, kSumFetch);
  for (uint32_t k = t; k < nf * kSumChunk; k += 1024u) {
    const uint32_t q = k / kSumChunk, e = k % kSumChunk;
    const uint64_t i = (uint64_t)s_list[q] * kSumChunk + e;
    fb[k] = i < n ? v[i] : 0.0f;
  }
}

// Sampling view after a reset (wasm_interface.rs:137-150): cleared to black
// (SimpleRenderTarget::clear keeps alpha, render_target.rs:160-166), then the
// adaptive halves repaint themselves blue (AdaptiveSamplingStrategy::reset,
// sampling_strategy.rs:205-213); a random half's reset is a no-op (:66-70).
// blue_left / blue_right = 1 paints that half blue.
__global__ void __launch_bounds__(kBlock) k_samp_reset(uint8_t* __restrict__ samp, uint32_t W, uint32_t H,
                                                       uint32_t half, uint32_t blue_left, uint32_t blue_right) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= W * H) return;
  const uint32_t x = i % W;
  const bool blue = x < half ? blue_left != 0 : blue_right != 0;
  reinterpret_cast<uchar4*>(samp)[i] = make_uchar4(0, 0, blue ? 255 : 0, 255);
}

// mix_color (sampling_strategy.rs:222-230)
__device__ __forceinline__ V3 mix_color(float v) {
  if (v < 0.5f) {
    const float a = 1.0f - 2.0f * v;
    const V3 g = mk(0.0f * a, 1.0f * a, 0.0f * a);
    const V3 b = mk(0.0f * 2.0f * v, 0.0f * 2.0f * v, 1.0f * 2.0f * v);
    return add(g, b);
  }
  const float a = 1.0f - 2.0f * (v - 0.5f);
  const V3 b = mk(0.0f * a, 0.0f * a, 1.0f * a);
  const V3 r = mk(1.0f * 2.0f * (v - 0.5f), 0.0f * 2.0f * (v - 0.5f), 0.0f * 2.0f * (v - 0.5f));
  return add(b, r);
}

// SimpleRenderTarget::write (render_target.rs:171-177)
__device__ __forceinline__ uchar4 simple_rgba(V3 v) {
  return make_uchar4((uint8_t)(fmaxf(fminf(v.x, 1.0f), 0.0f) * 255.0f), (uint8_t)(fmaxf(fminf(v.y, 1.0f), 0.0f) * 255.0f),
                     (uint8_t)(fmaxf(fminf(v.z, 1.0f), 0.0f) * 255.0f), 255);
}

struct RoundParams {
  uint32_t W, H, npix, half;
  uint32_t which;         // the screen half planned (x < half: 0, else 1); the other half's pixels get 0
  uint32_t adaptive;      // that half's strategy
  uint32_t first;         // round 0: 4 samples per adaptive pixel (reset, :205-213)
  float stats[3];         // {mse_sum, mse_min, mse_max} of the half (host)
};

// Plan one round: samples per partition pixel (c), the pixel's sample count
// so far (base), and the sampling visualisation of adaptive pixels
// (sampling_strategy.rs:148-172). stats = {sum, min, max} per half.
__global__ void __launch_bounds__(kBlock) k_plan_round(RoundParams P, const uint32_t* __restrict__ part_pix,
                                                       const uint32_t* __restrict__ cnt,
                                                       const float* __restrict__ mse_l, const float* __restrict__ mse_r,
                                                       uint32_t* __restrict__ c_out,
                                                       uint32_t* __restrict__ base_out, uint8_t* __restrict__ samp) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p > P.npix) return;
  if (p == P.npix) { c_out[p] = 0u; return; }  // scan sentinel: off[npix] = round total
  const uint32_t pixel = part_pix ? part_pix[p] : p;
  const uint32_t x = pixel % P.W, y = pixel / P.W;
  const uint32_t h = x < P.half ? 0u : 1u;
  base_out[p] = cnt[pixel];
  uint32_t c = h == P.which ? 1u : 0u;
  if (h == P.which && P.adaptive) {
    if (P.first) {
      c = 4u;
    } else {
      const uint32_t x0 = h ? P.half : 0u, rw = h ? P.W - P.half : P.half;
      const float m = (h ? mse_r : mse_l)[y * rw + (x - x0)];
      const float* st = P.stats;
      const float mn = st[1], mx = st[2];
      const float avg = st[0] / (float)(rw * P.H);  // mse_sum / (width*height) as f32
      float scaled = m < avg ? 0.5f * ((m - mn) / (avg - mn)) : 0.5f + 0.5f * ((m - avg) / (mx - avg));
      scaled = fmaxf(fminf(scaled, 1.0f), 0.0f);
      const float spp = ceilf(1.0f + scaled * 32.0f);
      c = spp >= 1.0f ? (uint32_t)spp : 1u;
      const V3 vis = mn == mx ? mk(0.0f, 0.0f, 0.0f) : mix_color(scaled);
      reinterpret_cast<uchar4*>(samp)[pixel] = simple_rgba(vis);
    }
  }
  c_out[p] = c;
}

// Exclusive scan of n u32 (in place), three passes: per-block sums, one block
// scanning the block sums, then each block adds its offset.
constexpr uint32_t kScanPer = 4;
constexpr uint32_t kScanChunk = kBlock * kScanPer;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t& total) {
  __shared__ uint32_t ws[kBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  uint32_t pre = 0;
  total = 0;
  for (int w = 0; w < (int)(kBlock / 64); w++) {
    if (w < wid) pre += ws[w];
    total += ws[w];
  }
  __syncthreads();
  return pre + inc - v;
}

__global__ void __launch_bounds__(kBlock) k_scan_local(uint32_t* __restrict__ a, uint32_t n,
                                                       uint32_t* __restrict__ sums) {
  const uint32_t base = blockIdx.x * kScanChunk + threadIdx.x * kScanPer;
  uint32_t v[kScanPer], t = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; k++) {
    v[k] = base + k < n ? a[base + k] : 0u;
    t += v[k];
  }
  uint32_t total;
  uint32_t off = block_excl_scan(t, total);
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; k++) {
    if (base + k < n) a[base + k] = off;
    off += v[k];
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kBlock) k_scan_sums(uint32_t* __restrict__ sums, uint32_t nb) {
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < nb; c0 += kBlock) {
    const uint32_t i = c0 + threadIdx.x;
    const uint32_t v = i < nb ? sums[i] : 0u;
    uint32_t total;
    const uint32_t e = block_excl_scan(v, total);
    if (i < nb) sums[i] = carry + e;
    carry += total;
  }
}

__global__ void __launch_bounds__(kBlock) k_scan_add(uint32_t* __restrict__ a, uint32_t n,
                                                     const uint32_t* __restrict__ sums) {
  const uint32_t base = blockIdx.x * kScanChunk + threadIdx.x * kScanPer;
  const uint32_t off = sums[blockIdx.x];
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; k++)
    if (base + k < n) a[base + k] += off;
}

// RenderTarget::write per pixel in sample order for a round batch: pidx[i]
// is path i's partition pixel; a pixel's paths are consecutive.
__global__ void __launch_bounds__(kBlock) k_accumulate_round(const uint32_t* __restrict__ part_pix, uint32_t n,
                                                             const uint32_t* __restrict__ pidx,
                                                             const float4* __restrict__ col,
                                                             float4* __restrict__ acc, uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pidx[i];
  if (i > 0 && pidx[i - 1] == p) return;
  const uint32_t pixel = part_pix ? part_pix[p] : p;
  float4 a = acc[pixel];
  uint32_t c = cnt[pixel];
  for (uint32_t j = i; j < n && pidx[j] == p; j++) {
    const float4 v = col[j];
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    c += 1;
  }
  acc[pixel] = a;
  cnt[pixel] = c;
}

// ---------------------------------------------------------------------------
// Several ranks. Rounds are planned over the WHOLE frame on
// every rank: after a frame exchange (wpt_set_exchange) each rank holds every
// pixel's acc/count, so k_mse, the host mse sums and k_plan_round give every
// rank the same global round (pixels in raster order, each pixel's samples
// consecutive). A compute() chunk covers a range [a, b) of that global round;
// a rank traces the part of it that falls on its own pixels.
// ---------------------------------------------------------------------------

// This rank's share of the global round range [a, b): for own pixel p (global
// offsets goff, sample count before the round gbase) the samples whose global
// positions lie in [a, b). c_out[npart] = 0 is the scan sentinel.
__global__ void __launch_bounds__(kBlock) k_plan_slice(const uint32_t* __restrict__ part_pix, uint32_t npart,
                                                       const uint32_t* __restrict__ goff,
                                                       const uint32_t* __restrict__ gbase, uint32_t a, uint32_t b,
                                                       uint32_t* __restrict__ c_out, uint32_t* __restrict__ base_out) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p > npart) return;
  if (p == npart) { c_out[p] = 0u; return; }
  const uint32_t pixel = part_pix[p];
  const uint32_t o0 = goff[pixel], o1 = goff[pixel + 1];
  const uint32_t lo = o0 > a ? o0 : a, hi = o1 < b ? o1 : b;
  c_out[p] = hi > lo ? hi - lo : 0u;
  base_out[p] = gbase[pixel] + (hi > lo ? lo - o0 : 0u);
}

// Exchange payload of one rank: float4 per partition pixel = (acc.xyz, count
// as u32 bits), so counts stay exact past 2^24.
__global__ void __launch_bounds__(kBlock) k_pack_exchange(const uint32_t* __restrict__ part_pix, uint32_t n,
                                                          const float4* __restrict__ acc,
                                                          const uint32_t* __restrict__ cnt, float4* __restrict__ out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = part_pix[i];
  float4 a = acc[p];
  a.w = __uint_as_float(cnt[p]);
  out[i] = a;
}

// Scatter the gathered payloads (rank-major, `slot` entries per rank) into
// the full frame; xidx[i] = pixel of gathered entry i, or ~0 for padding.
__global__ void __launch_bounds__(kBlock) k_unpack_exchange(const uint32_t* __restrict__ xidx, uint32_t n,
                                                            const float4* __restrict__ in, float4* __restrict__ acc,
                                                            uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t px = xidx[i];
  if (px == 0xFFFFFFFFu) return;
  const float4 v = in[i];
  acc[px] = make_float4(v.x, v.y, v.z, 0.0f);
  cnt[px] = __float_as_uint(v.w);
}
