// wpt_stock.h — the adaptive halves' sample stock (included by wpt_render.hip).
//
// A sample's path depends only on (pixel, sample index) (path_seed), and an
// adaptive half's rounds only decide how many of its next samples each pixel
// takes (sampling_strategy.rs:122-176), added in sample order
// (render_target.rs:55-65). So the samples a pixel will take next can be
// traced ahead of the rounds: a ring of `slots` samples per pixel (radiance
// and ray counts), filled by refill batches on the async lanes; a round adds
// its samples from the ring in sample order (k_consume) and traces only the
// ones the ring lacks (its deficit). The image is the same bits; the rounds'
// chain of dependent batches (each drained to its slowest ray) becomes a
// chain of cheap consumptions beside large independent refills.
//
// Per pixel: cnt (samples accumulated) and front (the next sample index to
// trace); samples [cnt, front) are in the ring, done or in flight, and
// front - cnt <= slots. Sample s of pixel p lives at p * slots + s % slots.
// stock_id[slot] = the refill tracing that sample (a round waits for the
// latest refill holding one of its samples). One rank: partition pixel = pixel.
#pragma once

// After a round is planned (off: its offsets per pixel; base: the samples
// each pixel had before it; cnt: the samples it has now, = base unless the
// round is partly added already, after a dropped stock): of its c = base +
// (off[p+1] - off[p]) - cnt samples still to add, the deficit d = max(0, c -
// (front - cnt)), samples front .. front + d - 1, traced by the round itself
// (def_base = front; front += d); bmax[block] = 1 + the latest refill id
// holding the round's other samples (0: none). def_cnt[npix] = 0 is the scan
// sentinel.
__global__ void __launch_bounds__(kBlock) k_stock_plan(uint32_t npix, const uint32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ base,
                                                       const uint32_t* __restrict__ cnt, uint32_t* __restrict__ front,
                                                       const uint32_t* __restrict__ stock_id, uint32_t slots,
                                                       uint32_t* __restrict__ def_cnt, uint32_t* __restrict__ def_base,
                                                       uint32_t* __restrict__ bmax) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  uint32_t id = 0;
  if (p < npix) {
    // the round's own pixels only (the other half's have c = 0 and may have
    // gained samples since this half's plan)
    const uint32_t cr = off[p + 1] - off[p];
    const uint32_t n0 = cnt[p];
    const uint32_t c = cr ? base[p] + cr - n0 : 0u;
    uint32_t d = 0;
    if (c) {
      const uint32_t f = front[p];
      const uint32_t have = min(c, f - n0);
      if (have) id = stock_id[(size_t)p * slots + ((n0 + have - 1u) & (slots - 1u))] + 1u;
      d = c - have;
      def_base[p] = f;
      front[p] = f + d;
    }
    def_cnt[p] = d;
  } else if (p == npix) {
    def_cnt[p] = 0u;
  }
  for (int o = 32; o > 0; o >>= 1) id = max(id, (uint32_t)__shfl_xor((int)id, o, 64));
  __shared__ uint32_t s_m[kBlock / 64];
  if ((threadIdx.x & 63u) == 0) s_m[threadIdx.x >> 6] = id;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < kBlock / 64; w++) id = max(id, s_m[w]);
    bmax[blockIdx.x] = id;
  }
}

// Folds k_stock_plan's per-block maxima into out[0].
__global__ void __launch_bounds__(1024) k_max_reduce(const uint32_t* __restrict__ bmax, uint32_t nb,
                                                     uint32_t* __restrict__ out) {
  uint32_t m = 0;
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) m = max(m, bmax[i]);
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  __shared__ uint32_t s_m[16];
  if ((threadIdx.x & 63u) == 0) s_m[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < blockDim.x / 64; w++) m = max(m, s_m[w]);
    out[0] = m;
  }
}

// A refill, planned after a round (before that round's samples are added):
// pixel list[i] of the half is stocked up to cnt + c + min((ahead * c +
// extra) * q / 1024, slots - c) samples, at most cnt + slots (the ring: the
// round still reads [cnt, cnt + c)); q <= 1024 scales the stock down to the
// positions left in the compute call. Samples front .. front + w - 1
// (rf_base = front, rf_cnt = w) are marked as this refill's (stock_id =
// id); front += w.
__global__ void __launch_bounds__(kBlock) k_refill_plan(const uint32_t* __restrict__ list, uint32_t n,
                                                        const uint32_t* __restrict__ off,
                                                        const uint32_t* __restrict__ cnt, uint32_t* __restrict__ front,
                                                        uint32_t* __restrict__ stock_id, uint32_t slots, uint32_t ahead,
                                                        uint32_t extra, uint32_t q, uint32_t id, uint32_t* __restrict__ rf_cnt,
                                                        uint32_t* __restrict__ rf_base) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) {
    if (i == n) rf_cnt[n] = 0u;  // scan sentinel
    return;
  }
  const uint32_t p = list[i];
  const uint32_t c = off[p + 1] - off[p];
  const uint32_t n0 = cnt[p], f = front[p];
  const uint32_t room = slots > c ? slots - c : 0u;
  const uint64_t want = (uint64_t)n0 + c + min((((uint64_t)ahead * c + extra) * q) >> 10, (uint64_t)room);
  const uint64_t t = min(want, (uint64_t)n0 + slots);
  const uint32_t w = t > f ? (uint32_t)(t - f) : 0u;
  rf_cnt[i] = w;
  rf_base[i] = f;
  for (uint32_t s = f; s != f + w; s++) stock_id[(size_t)p * slots + (s & (slots - 1u))] = id;
  front[p] = f + w;
}

// The tail of a stock batch: path i's radiance and ray counts to its slot.
__global__ void __launch_bounds__(kBlock) k_stock_store(const uint32_t* __restrict__ slot, uint32_t n,
                                                        const float4* __restrict__ col, float4* __restrict__ stock) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) stock[slot[i]] = col[i];
}

// Positions [a, b) of a round (off / base: its offsets and the samples each
// pixel had before it): every pixel adds its samples of the range from the
// ring in sample order (RenderTarget::write, render_target.rs:55-58); the
// consumed samples' rays (col.w of their paths: extension | shadow << 16)
// into per-block partial sums rb[2 * block ..], folded by k_rays_reduce.
__global__ void __launch_bounds__(kBlock) k_consume(uint32_t npix, const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ base, uint32_t a, uint32_t b,
                                                    const float4* __restrict__ stock, uint32_t slots,
                                                    float4* __restrict__ acc, uint32_t* __restrict__ cnt,
                                                    unsigned long long* __restrict__ rb) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  unsigned long long re = 0, rs = 0;
  if (p < npix) {
    const uint32_t p0 = off[p], p1 = off[p + 1];
    const uint32_t o0 = max(a, p0), o1 = min(b, p1);
    if (o1 > o0) {
      float4 A = acc[p];
      uint32_t c = cnt[p];
      const uint32_t s0 = base[p] + (o0 - p0);
      for (uint32_t s = s0; s != s0 + (o1 - o0); s++) {
        const float4 v = stock[(size_t)p * slots + (s & (slots - 1u))];
        A.x += v.x;
        A.y += v.y;
        A.z += v.z;
        c += 1;
        const uint32_t r = __float_as_uint(v.w);
        re += r & 0xFFFFu;
        rs += r >> 16;
      }
      acc[p] = A;
      cnt[p] = c;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    re += __shfl_xor(re, o, 64);
    rs += __shfl_xor(rs, o, 64);
  }
  __shared__ unsigned long long s_r[2][kBlock / 64];
  if ((threadIdx.x & 63u) == 0) {
    s_r[0][threadIdx.x >> 6] = re;
    s_r[1][threadIdx.x >> 6] = rs;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < kBlock / 64; w++) {
      re += s_r[0][w];
      rs += s_r[1][w];
    }
    rb[2 * blockIdx.x] = re;
    rb[2 * blockIdx.x + 1] = rs;
  }
}

// Adds k_consume's per-block ray sums into total[0..1] (the running count
// of consumed rays, read and cleared by the host).
__global__ void __launch_bounds__(1024) k_rays_reduce(const unsigned long long* __restrict__ rb, uint32_t nb,
                                                      unsigned long long* __restrict__ total) {
  unsigned long long re = 0, rs = 0;
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
    re += rb[2 * i];
    rs += rb[2 * i + 1];
  }
  for (int o = 32; o > 0; o >>= 1) {
    re += __shfl_xor(re, o, 64);
    rs += __shfl_xor(rs, o, 64);
  }
  __shared__ unsigned long long s_r[2][16];
  if ((threadIdx.x & 63u) == 0) {
    s_r[0][threadIdx.x >> 6] = re;
    s_r[1][threadIdx.x >> 6] = rs;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < blockDim.x / 64; w++) {
      re += s_r[0][w];
      rs += s_r[1][w];
    }
    total[0] += re;
    total[1] += rs;
  }
}
