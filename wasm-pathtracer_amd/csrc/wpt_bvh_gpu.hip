// wpt_bvh_gpu.hip — level-synchronous BVH2 build (wpt_bvh_gpu.h), the
// reference's binned-SAH algorithm (src/graphics/bvh.rs:103-437) for all
// nodes of a tree level at once.
#include "wpt_bvh_gpu.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <functional>

namespace wpt {

namespace {

constexpr uint32_t kB = 256;
constexpr uint32_t kNB = 16;             // bins (scene.rs:60 rebuild_bvh(16, ..))
constexpr uint32_t kBinWords = 7 * kNB;  // per task: 6 box keys + count per bin

#define BVH_OK(x)                                                               \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      err = std::string("HIP error (BVH build): ") + hipGetErrorString(e_);     \
      return false;                                                             \
    }                                                                           \
  } while (0)

// Order-preserving u32 image of an f32 (min / max through integer atomics).
__device__ __forceinline__ uint32_t okey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float okey_f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

struct BoxF {
  float x0, y0, z0, x1, y1, z1;
};
__device__ __forceinline__ BoxF join(const BoxF& a, const BoxF& o) {  // aabb.rs:90-100
  return BoxF{fminf(a.x0, o.x0), fminf(a.y0, o.y0), fminf(a.z0, o.z0),
              fmaxf(a.x1, o.x1), fmaxf(a.y1, o.y1), fmaxf(a.z1, o.z1)};
}
__device__ __forceinline__ float surface(const BoxF& b) {  // aabb.rs:72-78
  const float xs = b.x1 - b.x0, ys = b.y1 - b.y0, zs = b.z1 - b.z0;
  return 2.0f * (xs * ys + xs * zs + ys * zs);
}
// split_longest_axis (bvh.rs:286-303) on the box subdivide() receives
__device__ __forceinline__ int longest_axis(const float* pb) {
  const float xs = pb[3] - pb[0], ys = pb[4] - pb[1], zs = pb[5] - pb[2];
  return (xs > ys) ? ((xs > zs) ? 0 : 2) : ((ys > zs) ? 1 : 2);
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
  for (int s = 32; s > 0; s >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, s));
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  for (int s = 32; s > 0; s >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, s));
  return v;
}

__global__ void __launch_bounds__(kB) k_iota(uint32_t n, uint32_t* __restrict__ ord) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p < n) ord[p] = p;
}

// Level task l: min / max keys of the centroid coordinate, bin boxes empty.
__global__ void __launch_bounds__(kB) k_level_init(uint32_t ntasks, uint32_t* __restrict__ vmm,
                                                   uint32_t* __restrict__ bins) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i < 2 * ntasks) vmm[i] = (i & 1u) ? 0u : 0xFFFFFFFFu;
  if (i < kBinWords * ntasks) {
    const uint32_t c = (i % kBinWords) % 7u;
    bins[i] = c < 3 ? 0xFFFFFFFFu : 0u;
  }
}

// bin() first loop (bvh.rs:412-424): min / max of the axis coordinate per node.
__global__ void __launch_bounds__(kB) k_minmax(uint32_t n, uint32_t begin, uint32_t end,
                                               const uint32_t* __restrict__ seg, const uint32_t* __restrict__ ord,
                                               const float* __restrict__ loc, const float* __restrict__ tpbox,
                                               uint32_t* __restrict__ vmm) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  const uint32_t t = p < n ? seg[p] : 0xFFFFFFFFu;
  const bool act = p < n && t >= begin && t < end;
  uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
  if (act) {
    const float v = loc[3 * (size_t)ord[p] + longest_axis(tpbox + 6 * (size_t)t)];
    // a NaN coordinate is skipped, as f32::min / max (fminf / fmaxf) skip it
    // on the host (bvh.rs:412-424): the identity keys stay
    if (v == v) kmin = kmax = okey(v);
  }
  const uint64_t am = __ballot(act);
  if (am == 0) return;
  const int first = __ffsll((unsigned long long)am) - 1;
  const uint32_t tl = (uint32_t)__shfl((int)t, first);
  if (__all(!act || t == tl)) {  // the whole wave in one node: one atomic pair
    kmin = wave_min(kmin);
    kmax = wave_max(kmax);
    if ((int)(threadIdx.x & 63u) == first) {
      atomicMin(vmm + 2 * (tl - begin), kmin);
      atomicMax(vmm + 2 * (tl - begin) + 1, kmax);
    }
  } else if (act) {
    atomicMin(vmm + 2 * (t - begin), kmin);
    atomicMax(vmm + 2 * (t - begin) + 1, kmax);
  }
}

// bin() second loop (bvh.rs:426-435) and the bins' boxes and counts. A node
// whose shapes are not binned (one shape, or all centroids equal) puts them
// all in bin 0, whose box is then the node's hull (bvh.rs:397-407).
__global__ void __launch_bounds__(kB) k_bin(uint32_t n, uint32_t begin, uint32_t end,
                                            const uint32_t* __restrict__ seg, const uint32_t* __restrict__ ord,
                                            const float* __restrict__ loc, const float* __restrict__ box,
                                            const float* __restrict__ tpbox, const uint32_t* __restrict__ tcnt,
                                            const uint32_t* __restrict__ vmm, uint32_t* __restrict__ bins,
                                            uint8_t* __restrict__ binid) {
  __shared__ uint32_t sb[kBinWords];
  __shared__ uint32_t s_t;
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  const uint32_t t = p < n ? seg[p] : 0xFFFFFFFFu;
  const bool act = p < n && t >= begin && t < end;
  uint32_t sid = 0;
  uint32_t k[6] = {0, 0, 0, 0, 0, 0};
  if (act) {
    const uint32_t l = t - begin;
    const float vmin = okey_f(vmm[2 * l]), vmax = okey_f(vmm[2 * l + 1]);
    const uint32_t i = ord[p];
    if (tcnt[t] > 1 && vmin != vmax) {
      const float v = loc[3 * (size_t)i + longest_axis(tpbox + 6 * (size_t)t)];
      const float w = (vmax - vmin) / (float)kNB;
      const float q = floorf((v - vmin) / w);
      sid = (q != q || q <= 0.0f) ? 0u : (q >= (float)(kNB - 1) ? kNB - 1 : (uint32_t)q);
    }
    binid[p] = (uint8_t)sid;
    // NaN bounds are skipped as AABB::join's f32::min / max skip them
    // (aabb.rs:90-100): min slots keep their identity ~0, max slots 0
    for (int c = 0; c < 6; c++) {
      const float b = box[6 * (size_t)i + c];
      k[c] = b == b ? okey(b) : (c < 3 ? 0xFFFFFFFFu : 0u);
    }
  }
  if (threadIdx.x == 0) s_t = 0xFFFFFFFFu;
  __syncthreads();
  if (act) atomicMin(&s_t, t);
  __syncthreads();
  const uint32_t tb = s_t;
  const bool uni = __syncthreads_and(!act || t == tb) != 0;
  if (tb == 0xFFFFFFFFu) return;  // no shape of this level in the block
  if (uni) {  // the whole block in one node: privatised bins, one flush
    if (threadIdx.x < kBinWords) sb[threadIdx.x] = (threadIdx.x % 7u) < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    if (act) {
      uint32_t* b = sb + 7 * sid;
      for (int c = 0; c < 3; c++) atomicMin(b + c, k[c]);
      for (int c = 3; c < 6; c++) atomicMax(b + c, k[c]);
      atomicAdd(b + 6, 1u);
    }
    __syncthreads();
    if (threadIdx.x < kBinWords) {
      const uint32_t c = threadIdx.x % 7u, v = sb[threadIdx.x];
      uint32_t* g = bins + (size_t)kBinWords * (tb - begin) + threadIdx.x;
      if (c < 3) { if (v != 0xFFFFFFFFu) atomicMin(g, v); }
      else if (c < 6) { if (v != 0u) atomicMax(g, v); }
      else if (v != 0u) atomicAdd(g, v);
    }
  } else if (act) {
    uint32_t* g = bins + (size_t)kBinWords * (t - begin) + 7 * sid;
    for (int c = 0; c < 3; c++) atomicMin(g + c, k[c]);
    for (int c = 3; c < 6; c++) atomicMax(g + c, k[c]);
    atomicAdd(g + 6, 1u);
  }
}

__device__ __forceinline__ BoxF bin_box(const uint32_t* b) {
  return BoxF{okey_f(b[0]), okey_f(b[1]), okey_f(b[2]), okey_f(b[3]), okey_f(b[4]), okey_f(b[5])};
}

// split (bvh.rs:254-277) with split_axis's bin sweep (:309-370): one thread per
// node of the level. A split appends the two children to the task list.
__global__ void __launch_bounds__(kB) k_decide(uint32_t begin, uint32_t end, const uint32_t* __restrict__ vmm,
                                               const uint32_t* __restrict__ bins, uint32_t* __restrict__ toff,
                                               uint32_t* __restrict__ tcnt, float* __restrict__ tpbox,
                                               float* __restrict__ tbox, uint32_t* __restrict__ tchild,
                                               uint32_t* __restrict__ tsplit, uint32_t* __restrict__ tdepth,
                                               uint32_t* __restrict__ ntask) {
  const uint32_t t = begin + blockIdx.x * kB + threadIdx.x;
  if (t >= end) return;
  const uint32_t l = t - begin;
  const uint32_t* B = bins + (size_t)kBinWords * l;
  const uint32_t cnt = tcnt[t];
  const bool binned = cnt > 1 && okey_f(vmm[2 * l]) != okey_f(vmm[2 * l + 1]);
  BoxF res = bin_box(B);  // bin 0: the hull when nothing was binned
  tchild[t] = 0;
  if (binned) {
    uint32_t lb = 0, rb = kNB - 1;
    BoxF la = bin_box(B), ra = bin_box(B + 7 * rb);
    uint32_t lc = B[6], rc = B[7 * rb + 6];
    BoxF lna = B[7 * 1 + 6] ? join(la, bin_box(B + 7)) : la;
    BoxF rna = B[7 * (rb - 1) + 6] ? join(ra, bin_box(B + 7 * (rb - 1))) : ra;
    uint32_t lnc = lc + B[7 * 1 + 6], rnc = rc + B[7 * (rb - 1) + 6];
    while (lb + 1 < rb) {
      if ((surface(lna) * (float)lnc + surface(ra) * (float)rc) < (surface(la) * (float)lc + surface(rna) * (float)rnc)) {
        lb += 1;
        la = lna;
        lc = lnc;
        if (lb + 1 < rb) {
          const uint32_t* bn = B + 7 * (lb + 1);
          lna = bn[6] ? join(la, bin_box(bn)) : la;
          lnc = lc + bn[6];
        }
      } else {
        rb -= 1;
        ra = rna;
        rc = rnc;
        if (lb + 1 < rb) {
          const uint32_t* bn = B + 7 * (rb - 1);
          rna = bn[6] ? join(ra, bin_box(bn)) : ra;
          rnc = rc + bn[6];
        }
      }
    }
    const float utility = surface(la) * (float)lc + surface(ra) * (float)(cnt - lc);
    const BoxF pa = join(la, ra);
    res = pa;
    if (utility < surface(pa) * (float)cnt) {
      const uint32_t c0 = atomicAdd(ntask, 2u);
      const uint32_t off = toff[t], d = tdepth[t] + 1;
      toff[c0] = off;
      tcnt[c0] = lc;
      toff[c0 + 1] = off + lc;
      tcnt[c0 + 1] = cnt - lc;
      tdepth[c0] = tdepth[c0 + 1] = d;
      const float lv[6] = {la.x0, la.y0, la.z0, la.x1, la.y1, la.z1};
      const float rv[6] = {ra.x0, ra.y0, ra.z0, ra.x1, ra.y1, ra.z1};
      for (int c = 0; c < 6; c++) {
        tpbox[6 * (size_t)c0 + c] = lv[c];
        tpbox[6 * (size_t)(c0 + 1) + c] = rv[c];
      }
      tchild[t] = c0;
      tsplit[t] = lc;
    }
  }
  const float bv[6] = {res.x0, res.y0, res.z0, res.x1, res.y1, res.z1};
  for (int c = 0; c < 6; c++) tbox[6 * (size_t)t + c] = bv[c];
}

// Sort key: a split node's shapes by bin (write_to, bvh.rs:462-470), every
// other range in place (node ranges are disjoint and ordered by offset).
__global__ void __launch_bounds__(kB) k_keys(uint32_t n, uint32_t begin, uint32_t end,
                                             const uint32_t* __restrict__ seg, const uint32_t* __restrict__ toff,
                                             const uint32_t* __restrict__ tchild, const uint8_t* __restrict__ binid,
                                             uint32_t* __restrict__ key) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= n) return;
  const uint32_t t = seg[p];
  const bool split = t >= begin && t < end && tchild[t] != 0;
  key[p] = toff[t] * kNB + (split ? (uint32_t)binid[p] : 0u);
}

// Each shape of a split node joins its left or right child.
__global__ void __launch_bounds__(kB) k_reseg(uint32_t n, uint32_t begin, uint32_t end, uint32_t* __restrict__ seg,
                                              const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tchild,
                                              const uint32_t* __restrict__ tsplit) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= n) return;
  const uint32_t t = seg[p];
  if (t < begin || t >= end || tchild[t] == 0) return;
  seg[p] = p < toff[t] + tsplit[t] ? tchild[t] : tchild[t] + 1;
}

uint32_t blocks(size_t n) { return (uint32_t)std::max<size_t>(1, (n + kB - 1) / kB); }

}  // namespace

BvhGpu::~BvhGpu() {
  release();
  if (ev0_) (void)hipEventDestroy(ev0_);
  if (ev1_) (void)hipEventDestroy(ev1_);
  if (h_ntask_) (void)hipHostFree(h_ntask_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void BvhGpu::release() {
  void* bufs[] = {d_box_, d_loc_, d_ord_[0], d_ord_[1], d_key_[0], d_key_[1], d_seg_, d_bin_, d_toff_,
                  d_tcnt_, d_tchild_, d_tdepth_, d_tsplit_, d_tpbox_, d_tbox_, d_vmm_, d_bins_, d_ntask_, d_tmp_};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  d_box_ = d_loc_ = nullptr;
  d_ord_[0] = d_ord_[1] = d_key_[0] = d_key_[1] = nullptr;
  d_seg_ = nullptr;
  d_bin_ = nullptr;
  d_toff_ = d_tcnt_ = d_tchild_ = d_tdepth_ = d_tsplit_ = nullptr;
  d_tpbox_ = d_tbox_ = nullptr;
  d_vmm_ = d_bins_ = d_ntask_ = nullptr;
  d_tmp_ = nullptr;
  tmp_bytes_ = 0;
  cap_ = 0;
}

bool BvhGpu::reserve(size_t n, std::string& err) {
  if (!stream_) {
    BVH_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    BVH_OK(hipEventCreate(&ev0_));
    BVH_OK(hipEventCreate(&ev1_));
    BVH_OK(hipHostMalloc(&h_ntask_, sizeof(uint32_t)));
  }
  if (n <= cap_) return true;
  release();
  const size_t nt = 2 * n;  // tasks: at most 2n - 1 nodes
  BVH_OK(hipMalloc(&d_box_, sizeof(float) * 6 * n));
  BVH_OK(hipMalloc(&d_loc_, sizeof(float) * 3 * n));
  for (int k = 0; k < 2; k++) {
    BVH_OK(hipMalloc(&d_ord_[k], sizeof(uint32_t) * n));
    BVH_OK(hipMalloc(&d_key_[k], sizeof(uint32_t) * n));
  }
  BVH_OK(hipMalloc(&d_seg_, sizeof(uint32_t) * n));
  BVH_OK(hipMalloc(&d_bin_, n));
  BVH_OK(hipMalloc(&d_toff_, sizeof(uint32_t) * nt));
  BVH_OK(hipMalloc(&d_tcnt_, sizeof(uint32_t) * nt));
  BVH_OK(hipMalloc(&d_tchild_, sizeof(uint32_t) * nt));
  BVH_OK(hipMalloc(&d_tdepth_, sizeof(uint32_t) * nt));
  BVH_OK(hipMalloc(&d_tsplit_, sizeof(uint32_t) * nt));
  BVH_OK(hipMalloc(&d_tpbox_, sizeof(float) * 6 * nt));
  BVH_OK(hipMalloc(&d_tbox_, sizeof(float) * 6 * nt));
  BVH_OK(hipMalloc(&d_vmm_, sizeof(uint32_t) * 2 * n));
  BVH_OK(hipMalloc(&d_bins_, sizeof(uint32_t) * kBinWords * n));
  BVH_OK(hipMalloc(&d_ntask_, sizeof(uint32_t)));
  hipcub::DoubleBuffer<uint32_t> kb(d_key_[0], d_key_[1]), vb(d_ord_[0], d_ord_[1]);
  BVH_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes_, kb, vb, (int)n, 0, 32, stream_));
  BVH_OK(hipMalloc(&d_tmp_, tmp_bytes_));
  cap_ = n;
  return true;
}

bool BvhGpu::build(const float* box, const float* loc, size_t n, std::vector<Node2>& nodes,
                   std::vector<uint32_t>& ord, uint32_t& depth, double& ms_out, std::string& err) {
  nodes.assign(2, Node2{});  // placeholders (bvh.rs:107-109)
  ord.clear();
  depth = 0;
  levels_ = 0;
  last_ms_ = 0.0;
  ms_out = 0.0;
  if (n == 0) return true;
  if (n >= (1u << 27)) {
    err = "GPU BVH build: too many shapes (keys are offset * 16 + bin in 32 bits)";
    return false;
  }
  if (!reserve(n, err)) return false;
  // the root's box: aabb(reps) in order (bvh.rs:117), as the host builder
  float root[6] = {box[0], box[1], box[2], box[3], box[4], box[5]};
  for (size_t i = 1; i < n; i++) {
    for (int c = 0; c < 3; c++) root[c] = fminf(root[c], box[6 * i + c]);
    for (int c = 3; c < 6; c++) root[c] = fmaxf(root[c], box[6 * i + c]);
  }
  const uint32_t nn = (uint32_t)n;
  const uint32_t zero = 0, one = 1;
  BVH_OK(hipEventRecord(ev0_, stream_));
  BVH_OK(hipMemcpyAsync(d_box_, box, sizeof(float) * 6 * n, hipMemcpyHostToDevice, stream_));
  BVH_OK(hipMemcpyAsync(d_loc_, loc, sizeof(float) * 3 * n, hipMemcpyHostToDevice, stream_));
  BVH_OK(hipMemsetAsync(d_seg_, 0, sizeof(uint32_t) * n, stream_));
  k_iota<<<blocks(n), kB, 0, stream_>>>(nn, d_ord_[0]);
  BVH_OK(hipMemcpyAsync(d_toff_, &zero, sizeof(uint32_t), hipMemcpyHostToDevice, stream_));
  BVH_OK(hipMemcpyAsync(d_tcnt_, &nn, sizeof(uint32_t), hipMemcpyHostToDevice, stream_));
  BVH_OK(hipMemcpyAsync(d_tdepth_, &zero, sizeof(uint32_t), hipMemcpyHostToDevice, stream_));
  BVH_OK(hipMemcpyAsync(d_tpbox_, root, sizeof(root), hipMemcpyHostToDevice, stream_));
  BVH_OK(hipMemcpyAsync(d_ntask_, &one, sizeof(uint32_t), hipMemcpyHostToDevice, stream_));
  int bits = 4;
  while (bits < 32 && ((uint64_t)1 << bits) < (uint64_t)n * kNB) bits++;
  int cur = 0;  // d_ord_[cur] holds the current shape order
  uint32_t begin = 0, end = 1;
  while (begin < end) {
    const uint32_t lv = end - begin;
    k_level_init<<<blocks((size_t)kBinWords * lv), kB, 0, stream_>>>(lv, d_vmm_, d_bins_);
    k_minmax<<<blocks(n), kB, 0, stream_>>>(nn, begin, end, d_seg_, d_ord_[cur], d_loc_, d_tpbox_, d_vmm_);
    k_bin<<<blocks(n), kB, 0, stream_>>>(nn, begin, end, d_seg_, d_ord_[cur], d_loc_, d_box_, d_tpbox_, d_tcnt_,
                                         d_vmm_, d_bins_, d_bin_);
    k_decide<<<blocks(lv), kB, 0, stream_>>>(begin, end, d_vmm_, d_bins_, d_toff_, d_tcnt_, d_tpbox_, d_tbox_,
                                             d_tchild_, d_tsplit_, d_tdepth_, d_ntask_);
    BVH_OK(hipGetLastError());
    BVH_OK(hipMemcpyAsync(h_ntask_, d_ntask_, sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
    BVH_OK(hipStreamSynchronize(stream_));
    const uint32_t next = *h_ntask_;
    if (next > 2 * nn) {
      err = "GPU BVH build: task overflow";
      return false;
    }
    if (next > end) {  // some node split: write_to + the children's ranges
      k_keys<<<blocks(n), kB, 0, stream_>>>(nn, begin, end, d_seg_, d_toff_, d_tchild_, d_bin_, d_key_[0]);
      hipcub::DoubleBuffer<uint32_t> kb(d_key_[0], d_key_[1]), vb(d_ord_[cur], d_ord_[cur ^ 1]);
      BVH_OK(hipcub::DeviceRadixSort::SortPairs(d_tmp_, tmp_bytes_, kb, vb, (int)n, 0, bits, stream_));
      if (vb.Current() != d_ord_[cur]) cur ^= 1;
      k_reseg<<<blocks(n), kB, 0, stream_>>>(nn, begin, end, d_seg_, d_toff_, d_tchild_, d_tsplit_);
      BVH_OK(hipGetLastError());
    }
    begin = end;
    end = next;
    levels_++;
  }
  const uint32_t ntask = end;
  std::vector<uint32_t> toff(ntask), tcnt(ntask), tchild(ntask), tdepth(ntask);
  std::vector<float> tbox(6 * (size_t)ntask);
  ord.resize(n);
  BVH_OK(hipMemcpyAsync(ord.data(), d_ord_[cur], sizeof(uint32_t) * n, hipMemcpyDeviceToHost, stream_));
  BVH_OK(hipMemcpyAsync(toff.data(), d_toff_, sizeof(uint32_t) * ntask, hipMemcpyDeviceToHost, stream_));
  BVH_OK(hipMemcpyAsync(tcnt.data(), d_tcnt_, sizeof(uint32_t) * ntask, hipMemcpyDeviceToHost, stream_));
  BVH_OK(hipMemcpyAsync(tchild.data(), d_tchild_, sizeof(uint32_t) * ntask, hipMemcpyDeviceToHost, stream_));
  BVH_OK(hipMemcpyAsync(tdepth.data(), d_tdepth_, sizeof(uint32_t) * ntask, hipMemcpyDeviceToHost, stream_));
  BVH_OK(hipMemcpyAsync(tbox.data(), d_tbox_, sizeof(float) * 6 * ntask, hipMemcpyDeviceToHost, stream_));
  BVH_OK(hipEventRecord(ev1_, stream_));
  BVH_OK(hipStreamSynchronize(stream_));
  float ms = 0.0f;
  BVH_OK(hipEventElapsedTime(&ms, ev0_, ev1_));
  last_ms_ = ms;
  ms_out = ms;
  // the reference's node numbering: a split node's child pair is allocated
  // when subdivide() reaches it, depth first, left before right (bvh.rs:225-231)
  nodes.reserve(2 * (size_t)ntask);
  auto node_of = [&](uint32_t t, uint32_t lf, uint32_t count) {
    const float* b = tbox.data() + 6 * (size_t)t;
    return Node2{{b[0], b[1], b[2]}, {b[3], b[4], b[5]}, lf, count};
  };
  std::function<Node2(uint32_t)> rec = [&](uint32_t t) -> Node2 {
    if (tchild[t] == 0) {
      depth = std::max(depth, tdepth[t]);
      return node_of(t, toff[t], tcnt[t]);
    }
    const size_t left = nodes.size();
    nodes.push_back(Node2{});
    nodes.push_back(Node2{});
    const Node2 a = rec(tchild[t]);
    nodes[left] = a;
    const Node2 b = rec(tchild[t] + 1);
    nodes[left + 1] = b;
    return node_of(t, (uint32_t)left, 0u);
  };
  nodes[0] = rec(0);
  return true;
}

}  // namespace wpt
