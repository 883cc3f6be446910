// wpt_render.hip — gfx950 wavefront path tracer.
//
// Kernels (one launch each per bounce, counts read from HBM, no host sync):
//   k_generate   camera rays + per-path RNG seed           tracer.rs:175-193
//   k_extend     closest hit over planes + BVH2           scene.rs:137-288
//   k_shade      emitter / diffuse bounce / NEE / RR       tracer.rs:237-329
//   k_shadow     NEE shadow query                          scene.rs:104-133
//   k_accumulate acc += colour, in sample order            render_target.rs:55-58
// The BVH2 traversal is the reference's recursive ordered descent restated as
// an iterative stack machine with identical cull / order / tie rules, so the
// closest hit (t, shape id) is bit-identical to the reference's.
#include "wpt_render.h"
#include "wpt_partition.h"
#include "wpt_photon.h"
#include "wpt_quartic.h"
#include "wpt_seqsum.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <thread>
#include <type_traits>

#define HIP_OK(expr)                                                     \
  do {                                                                   \
    hipError_t e_ = (expr);                                              \
    if (e_ != hipSuccess) {                                              \
      err = std::string(#expr " failed: ") + hipGetErrorString(e_);      \
      return false;                                                      \
    }                                                                    \
  } while (0)

// WPT_OPT_LOG lines, stamped with the host's monotonic clock in ms (Python's
// time.monotonic() on Linux: tools/session_rate.py marks its calls with it)
static double wpt_log_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define WPT_LOGF(fmt, ...) fprintf(stderr, "[wpt %.3f] " fmt, wpt_log_ms(), ##__VA_ARGS__)

namespace wpt {

namespace {

constexpr uint32_t kBlock = 256;
// Threads per block of the traversal kernels (k_extend, k_shadow, k_trace,
// k_finish): their LDS stack (kLdsSlots entries per lane) and the LDS
// treelet are per block, so larger blocks hold one treelet for more lanes.
#ifndef WPT_TRAV_BLOCK
#define WPT_TRAV_BLOCK 256
#endif
constexpr uint32_t kTBlock = WPT_TRAV_BLOCK;
// Entries per chunk of the traversal kernels' work feed (WaveFeed; a power
// of two): smaller chunks spread each wave's rays over more of the stream.
// Leaf batching in step() (0 = off; triangle scenes): a lane at a leaf waits
// until WPT_LEAF_BATCH lanes of its wave are at one, unless fewer than
// WPT_LEAF_BATCH_MIN lanes are active. Round 5, same-session C3 (Mray/s):
// 16 / 32 8 431 / 8 466 vs 8 087 / 8 036; 16 / 24 +5.2 %, 24 / 32 +4.9 %,
// 16 / 40 +4.0 %, 8 / 32 +2.3 %, 32 / 48 +0.9 %; without the minimum C5 lost
// 6-13 % (profiles/r05/ab_lb*.jsonl).
#ifndef WPT_LEAF_BATCH
#define WPT_LEAF_BATCH 16
#endif
#ifndef WPT_LEAF_BATCH_MIN
#define WPT_LEAF_BATCH_MIN 32
#endif
// the same for shadow walks (k_shadow, and every walk of the fused k_trace)
#ifndef WPT_LEAF_BATCH_SH
#define WPT_LEAF_BATCH_SH WPT_LEAF_BATCH
#endif
#ifndef WPT_LEAF_BATCH_MIN_SH
#define WPT_LEAF_BATCH_MIN_SH WPT_LEAF_BATCH_MIN
#endif
#ifndef WPT_FEED_CHUNK
#define WPT_FEED_CHUNK 64
#endif
constexpr uint32_t kFeedChunk = WPT_FEED_CHUNK;
static_assert((kFeedChunk & (kFeedChunk - 1u)) == 0u, "feed chunk: a power of two");
#ifndef WPT_SHADE_BLOCK
#define WPT_SHADE_BLOCK 256
#endif
constexpr uint32_t kShadeBlock = WPT_SHADE_BLOCK;
#ifndef WPT_SHADE_GRID_VAR
#define WPT_SHADE_GRID_VAR 1  // k_shade's grid from the launched variant's own occupancy (0: the smallest of all variants)
#endif
// k_shade on triangle scenes without PNEE: 6 waves per SIMD (77 VGPRs, no
// spill; C3 +0.5 %). 7 spills 32 B and gains nothing; the other variants
// would spill and keep the compiler's choice.
#ifndef WPT_PNEE_SHADE_WAVES
#define WPT_PNEE_SHADE_WAVES 6  // PNEE: 80 VGPRs forced (24 B spilled), C5 +1.6 %; 1 = the compiler's 87 VGPRs, 5 waves
#endif
#ifndef WPT_NEE_SHADE_WAVES
#define WPT_NEE_SHADE_WAVES 6  // a floor: its 72 VGPRs give 7 (8 forced: 44 B spilled)
#endif
#define WPT_SHADE_BOUNDS __launch_bounds__(kShadeBlock, TRI_ONLY ? (PNEE ? WPT_PNEE_SHADE_WAVES : WPT_NEE_SHADE_WAVES) : 1)  // k_shade: the waves of a block share one output-append atomic
#ifndef WPT_LDS_SLOTS
#define WPT_LDS_SLOTS 9
#endif
constexpr int kLdsSlots = WPT_LDS_SLOTS;  // traversal stack entries kept in LDS (18 KB per 256-lane block)
// k_extend / k_shadow / k_trace run at 8 waves per SIMD: 9 LDS slots (19.9 KB
// per block: 8 blocks per CU), <= 64 VGPRs and <= 80 SGPRs
// (MI355X_MICROARCH.md residency rule), no spill. This fits because
// wpt_render.hip is compiled without the SLP vectoriser (Makefile): packing
// neighbouring f32 operations into v_pk_* pairs tied registers into aligned
// pairs and cost k_extend 13 VGPRs (72 -> 59), which had held these kernels
// at 7 / 6 waves. Triangle-only scenes only: the other shape kinds (f64 torus
// quartic) would spill hundreds of bytes.
#ifndef WPT_TRACE_WAVES
#define WPT_TRACE_WAVES 8
#endif
// Scenes with other shape kinds (the museum's f64 tori): 6 waves, 80 VGPRs
// (32-48 B more scratch than the compiler's 5 waves; museum +2.9 %)
#ifndef WPT_TRACE_WAVES_ANY
#define WPT_TRACE_WAVES_ANY 6
#endif
#define WPT_TRACE_BOUNDS __launch_bounds__(kTBlock, TRI_ONLY ? WPT_TRACE_WAVES : WPT_TRACE_WAVES_ANY)
// Treelet: the BVH2 node pairs nearest the root (breadth first), copied to
// LDS by every block; a pair's internal child whose own pair is in the treelet
// has its left_first replaced by kTreeFlag | treelet index.
#ifndef WPT_TREE_PAIRS
#define WPT_TREE_PAIRS 23  // fills the 8-blocks-per-CU LDS budget beside the 9-slot stack (round 4: standalone k_extend -1.5 %, C3 4-lane step equal)
#endif
constexpr uint32_t kTreePairs = WPT_TREE_PAIRS;
#ifndef WPT_TRI_BF
#define WPT_TRI_BF 1  // branch-free triangle test (0: early returns; C3 -1.5 %)
#endif
constexpr uint32_t kTreeFlag = 0x20000000u;
#ifndef WPT_LEAF_PEEL
#define WPT_LEAF_PEEL 1  // the first record of a leaf tested outside the leaf loop (triangle scenes; C5 +1.4-1.7 %, C3 +0.4 %)
#endif
constexpr uint32_t kFlagBounced = 1u;   // has_diffuse_bounced
constexpr uint32_t kTypeShift = 2u;     // render type (2 bits)
constexpr uint32_t kOctLdsWords = 6144;  // PNEE octree words k_shade stages in LDS (24 KB per block)
constexpr uint32_t kShadeLights = 16;    // light records k_shade stages in LDS (80 B each)
constexpr uint32_t kDepthShift = 8u;    // bounce depth (10 bits: <= kMaxBounces)
constexpr uint32_t kDepthMask = 0x3FFu;
constexpr uint32_t kShadowShift = 18u;  // shadow rays the path emitted so far (ShadeParams::count_rays)

__device__ __forceinline__ V3 ld3(const float4& a) { return mk(a.x, a.y, a.z); }

// Pins a loaded float4 in registers at this point: its four words come from
// one 16 B load issued here, not re-split and deferred by the compiler.
// One 128-bit operand: the load's own register quad. (Four 32-bit operands,
// the round-3 form, made the compiler copy the words out of the quad: 20-56
// more v_mov per traversal kernel.)
__device__ __forceinline__ void pin4(float4& v) {
  typedef float q4 __attribute__((ext_vector_type(4)));
  q4 t = {v.x, v.y, v.z, v.w};
  asm volatile("" : "+v"(t));
  v = make_float4(t.x, t.y, t.z, t.w);
}

// Path-state stores (generate, shade): read back only by a later kernel (GBs
// of state, far beyond L2/MALL), so they are marked nontemporal.
__device__ __forceinline__ void st_stream(float4* p, float4 v) {
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
  __builtin_nontemporal_store(v.z, &p->z);
  __builtin_nontemporal_store(v.w, &p->w);
}


// ---------------------------------------------------------------------------
// Primitive tests (Tracable::trace_simple). Precomputed per-triangle values
// (n = (v1-v0)x(v2-v0), n·v0, normalize(n)) are the bits the reference
// recomputes per test, so results are identical.
// ---------------------------------------------------------------------------
// Triangle record (4 float4): (v0, n.x) (v1, n.y) (v2, n.z) (normalize(n), n·v0).
// The test is one conjunction of the reference's comparisons (no divergent
// early returns: the traversal loop's exec-mask bookkeeping is about half of
// its instructions). With the SLP vectoriser on it needed 83-97 VGPRs in the
// traversal kernels; without it, 58-67.
__device__ __forceinline__ bool tri_hit_r(const float4& a, const float4& b, const float4& c, const float4& e, V3 o,
                                          V3 d, float& t) {
  // triangle.rs:159-191
  const V3 n = mk(a.w, b.w, c.w);
  const float n_dot_d = dot(n, d);
#if WPT_TRI_BF
  // the same comparisons as one conjunction (no divergent early returns)
  const float tt = (e.w - dot(n, o)) / n_dot_d;
  const V3 nn = mk(e.x, e.y, e.z);
  const V3 pp = add(o, scale(d, tt));
  const V3 v0 = ld3(a), v1 = ld3(b), v2 = ld3(c);
  const bool ok = (int)(n_dot_d != 0.0f) & (int)(tt > 0.0f) &
                  (int)(dot(nn, cross(sub(v1, v0), sub(pp, v0))) + kTriSlack >= 0.0f) &
                  (int)(dot(nn, cross(sub(v2, v1), sub(pp, v1))) + kTriSlack >= 0.0f) &
                  (int)(dot(nn, cross(sub(v0, v2), sub(pp, v2))) + kTriSlack >= 0.0f);
  t = ok ? tt : t;
  return ok;
#else
  if (n_dot_d == 0.0f) return false;
  const float tt = (e.w - dot(n, o)) / n_dot_d;
  if (tt <= 0.0f) return false;
  const V3 nn = mk(e.x, e.y, e.z);
  const V3 pp = add(o, scale(d, tt));
  const V3 v0 = ld3(a), v1 = ld3(b), v2 = ld3(c);
  // is_approx_left_of (triangle.rs:41-45) for the three edges
  if (!(dot(nn, cross(sub(v1, v0), sub(pp, v0))) + kTriSlack >= 0.0f)) return false;
  if (!(dot(nn, cross(sub(v2, v1), sub(pp, v1))) + kTriSlack >= 0.0f)) return false;
  if (!(dot(nn, cross(sub(v0, v2), sub(pp, v2))) + kTriSlack >= 0.0f)) return false;
  t = tt;
  return true;
#endif
}

__device__ __forceinline__ bool tri_hit(const float4* __restrict__ p, V3 o, V3 d, float& t) {
  float4 a = p[0], b = p[1], c = p[2], e = p[3];
  pin4(a);
  pin4(b);
  pin4(c);
  pin4(e);
  return tri_hit_r(a, b, c, e, o, d, t);
}

__device__ __forceinline__ bool plane_hit(float4 pl, V3 o, V3 d, float& t) {  // plane.rs:80-99
  const V3 n = ld3(pl);
  const float n_dot_dir = dot(n, d);
  if (n_dot_dir == 0.0f) return false;
  const float tt = (pl.w - dot(n, o)) / n_dot_dir;
  if (tt <= 0.0f) return false;
  t = tt;
  return true;
}

__device__ __forceinline__ bool sphere_roots(float4 s, V3 o, V3 d, float& t, bool& entering) {
  // sphere.rs:104-131
  const V3 c = ld3(s);
  const float b = 2.0f * dot(d, sub(o, c));
  const float cc = dot(sub(o, c), sub(o, c)) - s.w * s.w;
  const float disc = b * b - 4.0f * cc;
  if (disc < 0.0f) return false;
  const float ds = sqrtf(disc);
  const float t0 = (-b + ds) / 2.0f;
  const float t1 = (-b - ds) / 2.0f;
  float tt = fminf(t0, t1);
  entering = true;
  if (tt <= 0.0f) {
    tt = fmaxf(t0, t1);
    if (tt <= 0.0f) return false;
    entering = false;
  }
  t = tt;
  return true;
}

__device__ __forceinline__ void aarect_slab(float4 a, float4 b, V3 o, V3 d, float* t6, float& tmin, float& tmax) {
  // aa_rect.rs:142-163
  const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
  t6[0] = (a.x - o.x) * ix;
  t6[1] = (a.y - o.x) * ix;
  t6[2] = (a.z - o.y) * iy;
  t6[3] = (a.w - o.y) * iy;
  t6[4] = (b.x - o.z) * iz;
  t6[5] = (b.y - o.z) * iz;
  tmin = fmaxf(fmaxf(fminf(t6[0], t6[1]), fminf(t6[2], t6[3])), fminf(t6[4], t6[5]));
  tmax = fminf(fminf(fmaxf(t6[0], t6[1]), fmaxf(t6[2], t6[3])), fmaxf(t6[4], t6[5]));
}

__device__ __forceinline__ bool aarect_hit(const float4* p, V3 o, V3 d, float& t) {
  float t6[6], tmin, tmax;
  aarect_slab(p[0], p[1], o, d, t6, tmin, tmax);
  if (tmin >= tmax) return false;
  if (tmin > 0.0f) { t = tmin; return true; }
  if (tmax > 0.0f) { t = tmax; return true; }
  return false;
}

// Torus::trace (f64 quartic, wpt_quartic.h) kept out of line: its registers
// and scratch do not weigh on the traversal loops that call it. The record is
// always in global memory (shape records), and the result comes back by value:
// no generic-pointer (flat) loads and stores across the call.
struct TorusHit {
  float t;
  V3 n;  // (0, 1, 0) unless hit
  bool hit;
};
__device__ __noinline__ TorusHit torus_hit(const float4* p, V3 o, V3 d) {
  typedef __attribute__((address_space(1))) const float gf32;
  const gf32* g = (const gf32*)p;
  TorusHit r;
  r.t = 0.0f;
  r.n = mk(0.0f, 1.0f, 0.0f);
  r.hit = torus_trace(mk(g[0], g[1], g[2]), g[3], g[4], o, d, r.t, r.n);
  return r;
}

__device__ __forceinline__ bool prim_hit(uint32_t kind, const float4* p, V3 o, V3 d, float& t) {
  switch (kind) {
    case kTri: return tri_hit(p, o, d, t);
    case kPlane: return plane_hit(p[0], o, d, t);
    case kSphere: { bool e; return sphere_roots(p[0], o, d, t, e); }
    case kTorus: {  // trace_simple = trace().distance (ray.rs:111-117)
      const TorusHit r = torus_hit(p, o, d);
      t = r.t;
      return r.hit;
    }
    default: return aarect_hit(p, o, d, t);
  }
}

// Triangle::trace's normal (triangle.rs:138-153), normalised by Hit::new.
__device__ __forceinline__ V3 tri_normal(const float4* p, V3 d) {
  const V3 n = mk(p[0].w, p[1].w, p[2].w);
  const float n_dot_d = dot(n, d);
  const V3 nn = ld3(p[3]);
  return normalize(n_dot_d > 0.0f ? neg(nn) : nn);
}

// Shape::trace's surface normal at the winning hit (normalised by Hit::new).
__device__ V3 prim_normal(uint32_t kind, const float4* p, V3 o, V3 d, float t) {
  if (kind == kTri) return tri_normal(p, d);
  if (kind == kPlane) {  // plane.rs:45-78
    V3 n = ld3(p[0]);
    if (dot(n, d) > 0.0f) n = neg(n);
    return normalize(n);
  }
  if (kind == kSphere) {  // sphere.rs:49-102
    float tt;
    bool ent = true;
    sphere_roots(p[0], o, d, tt, ent);
    V3 n = divs(sub(add(o, scale(d, t)), ld3(p[0])), p[0].w);
    return normalize(ent ? n : neg(n));
  }
  if (kind == kTorus) return torus_hit(p, o, d).n;  // torus.rs:115-126 (already normalised as Hit::new does)
  // aa_rect.rs:102-135
  float t6[6], tmin, tmax;
  aarect_slab(p[0], p[1], o, d, t6, tmin, tmax);
  V3 n;
  if (tmin > 0.0f) {
    if (tmin == t6[0]) n = mk(-1, 0, 0);
    else if (tmin == t6[1]) n = mk(1, 0, 0);
    else if (tmin == t6[2]) n = mk(0, -1, 0);
    else if (tmin == t6[3]) n = mk(0, 1, 0);
    else if (tmin == t6[4]) n = mk(0, 0, -1);
    else n = mk(0, 0, 1);
  } else {
    if (tmax == t6[0]) n = mk(1, 0, 0);
    else if (tmax == t6[1]) n = mk(-1, 0, 0);
    else if (tmax == t6[2]) n = mk(0, 1, 0);
    else if (tmax == t6[3]) n = mk(0, -1, 0);
    else if (tmax == t6[4]) n = mk(0, 0, 1);
    else n = mk(0, 0, -1);
  }
  return normalize(n);
}

// AABB::hit + aabb_distance (aabb.rs:132-164, scene.rs:393-403): entry
// distance if hit strictly before max_dis, else +inf sentinel (never < max).
__device__ __forceinline__ bool box_entry(float4 a, float4 b, V3 o, V3 inv, float max_dis, float& h) {
  // a = (x_min, y_min, z_min, x_max), b = (y_max, z_max, ..)
  const float tx1 = (a.x - o.x) * inv.x;
  const float tx2 = (a.w - o.x) * inv.x;
  const float ty1 = (a.y - o.y) * inv.y;
  const float ty2 = (b.x - o.y) * inv.y;
  const float tz1 = (a.z - o.z) * inv.z;
  const float tz2 = (b.y - o.z) * inv.z;
  const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
  const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
  // AABB::hit's decisions in two compares: entry hh = max(tmin, 0) (tmin if
  // the ray starts outside, 0 inside); hit iff hh <= tmax and hh < max_dis.
  // The same verdicts as !(tmin > tmax) && (tmin >= 0 || tmax >= 0) &&
  // hh < max_dis: for tmin >= 0, hh <= tmax is !(tmin > tmax); for tmin < 0,
  // it is tmax >= 0 (and tmin <= tmax follows). NaNs: fminf / fmaxf drop a
  // NaN operand, so tmax is NaN only if every axis is, and then tmin is too;
  // a NaN tmin gives hh = 0 in both forms (max returns the number). -0 vs +0
  // for hh = max(-0, 0) is invisible: entries are only ever compared.
  const float hh = fmaxf(tmin, 0.0f);
  h = hh;
  return (hh <= tmax) & (hh < max_dis);
}

// ---------------------------------------------------------------------------
// BVH2 closest-hit traversal (Scene::trace_g, scene.rs:162-288), one ray per
// lane in a persistent kernel. The reference's recursive ordered descent is
// restated as a stack machine with identical rules:
//   * a child is entered iff its AABB::hit entry is strictly before the
//     current closest hit (aabb_distance, scene.rs:393-403);
//   * both hit: the nearer child first, ties to the right child (:244, :261);
//     the other is deferred;
//   * a deferred child is resumed unless the closest hit found since is
//     strictly before its entry (:247, :264) — its entry is recomputed from
//     its box at pop time (same bits), so a stack entry is one u32 in LDS;
//   * a leaf accepts t <= closest-on-entry, strict < inside the leaf, so the
//     later-visited leaf wins ties (trace_shapes_md, :450-472).
// ---------------------------------------------------------------------------
struct Lane {
  V3 o, d, inv;
  float best;
  int32_t best_id;
  uint32_t lf, cnt;  // current node's left_first / count
  int sp;            // traversal stack depth
};

__device__ __forceinline__ V3 inv_dir(V3 d) { return mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); }  // ray.rs:31-33

// Kernel-constant data every ray starting on a lane needs, loaded once per
// block instead of once per ray (a dependent round trip per refill): the
// BVH2 root node (the same address for every ray) and, for scenes with few
// lights, the lights' triangle records in LDS (a shadow ray tests its light
// first; the light id comes from the ray record, so a global load would wait
// behind the ray's own load).
constexpr uint32_t kLdsLights = 8;
typedef __attribute__((address_space(3))) float lds_f32h;
typedef __attribute__((address_space(3))) int32_t lds_i32;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f4v lds_f4v;
__device__ __forceinline__ float4 to_f4(f4v v) { return make_float4(v.x, v.y, v.z, v.w); }
struct Hot {
  float4 root_a, root_b;  // S.nodes[0], S.nodes[1] (root_b.z: the treelet's first pair when there is one)
  const lds_f32h* lrec;   // kLdsLights light prim records (16 floats each); nullptr: more lights than fit
  const lds_i32* lid;     // their shape ids
  const float4* gtree;    // treelet (S.tree_pairs node pairs nearest the root, 4 float4 each) in the
                          // block's LDS, through a generic pointer (expand_pair's one load site)
  __device__ float4 lq(uint32_t k, uint32_t w) const {
    const lds_f32h* p = lrec + 16 * k + 4 * w;
    return make_float4(p[0], p[1], p[2], p[3]);
  }
};

// Fills the block's root registers, LDS treelet and light table (every
// thread of the block calls it).
__device__ __forceinline__ Hot load_hot(const DevScene& S, lds_f32h* lrec, lds_i32* lid, lds_f4v* tree,
                                        const float4* gtree = nullptr) {
  Hot h;
  h.root_a = S.nodes[0];
  h.root_b = S.nodes[1];
  if (kTreePairs > 0) {
    for (uint32_t i = threadIdx.x; i < 4 * S.tree_pairs; i += kTBlock) {
      const float4 v = S.tree[i];
      tree[i] = f4v{v.x, v.y, v.z, v.w};
    }
    if (S.tree_pairs != 0) h.root_b.z = __uint_as_float(S.tree_root_lf);
  }
  h.gtree = gtree;
  const bool fits = S.num_lights <= kLdsLights;
  if (fits && threadIdx.x < 4 * S.num_lights) {
    const uint32_t l = threadIdx.x >> 2, w = threadIdx.x & 3u;
    const uint32_t sid = __float_as_uint(S.lights[5 * l + 1].w);
    const float4 v = S.prims[4 * (size_t)(sid - S.num_inf) + w];
    lrec[4 * threadIdx.x] = v.x;
    lrec[4 * threadIdx.x + 1] = v.y;
    lrec[4 * threadIdx.x + 2] = v.z;
    lrec[4 * threadIdx.x + 3] = v.w;
    if (w == 0) lid[l] = (int32_t)sid;
  }
  __syncthreads();
  h.lrec = fits ? lrec : nullptr;
  h.lid = lid;
  return h;
}

// traverse_bvh_guarded on the root (scene.rs:191-212). False if the root is
// culled. The block's root registers hold the root (load_hot).
template <bool COUNT>
__device__ __forceinline__ bool enter_root(const DevScene& S, const Hot& H, Lane& L, uint32_t& visits,
                                           uint32_t& nbytes) {
  if (COUNT) { visits++; nbytes += 32; }
  const float4 a = H.root_a, b = H.root_b;
  float h;
  if (!box_entry(a, b, L.o, L.inv, L.best, h)) return false;
  L.lf = __float_as_uint(b.z);
  L.cnt = __float_as_uint(b.w);
  L.sp = 0;
  return true;
}

// Traversal stack: deferred far children as (code, exact entry distance).
// The top kLdsSlots entries live in LDS (one u32 + one f32 per lane, lane-
// strided: conflict-free), deeper ones in a per-lane global spill area.
// code: internal child -> its left_first; leaf child -> bit31 | count<<24 |
// first prim (count < 128, first < 2^24); otherwise bit30 | node index.
// LDS pointers typed as such: through a plain (generic) pointer the compiler
// emits flat loads for the pops, which wait on both the vector-memory and the
// LDS counters (measured: flat_load_dword in k_extend's pop).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) float lds_f32;
struct Stack {
  lds_u32* code;
  lds_f32* h;
  uint2* spill;
  uint32_t stride;
  int cap;             // entries available (LDS + spill), sized on the host
  uint32_t* overflow;  // set if a push would exceed cap (the host fails the call)
};

__device__ __forceinline__ uint32_t encode_child(uint32_t lf, uint32_t cnt, uint32_t node) {
  // selects, not branches (no exec-mask bookkeeping in the push path)
  const uint32_t leaf = (cnt < 128u && lf < (1u << 24)) ? (0x80000000u | (cnt << 24) | lf) : (0x40000000u | node);
  return cnt == 0 ? lf : leaf;
}

// Entry k of the stack (LDS slots, then the global spill area).
__device__ __forceinline__ void stack_store(const Stack& st, int k, uint32_t code, float h) {
  if (k < kLdsSlots) {
    st.code[k * kTBlock] = code;
    st.h[k * kTBlock] = h;
  } else {
    st.spill[(size_t)(k - kLdsSlots) * st.stride] = make_uint2(code, __float_as_uint(h));
  }
}

__device__ __forceinline__ void stack_load(const Stack& st, int k, uint32_t& code, float& h) {
  if (k < kLdsSlots) {
    code = st.code[k * kTBlock];
    h = st.h[k * kTBlock];
  } else {
    const uint2 e = st.spill[(size_t)(k - kLdsSlots) * st.stride];
    code = e.x;
    h = __uint_as_float(e.y);
  }
}

// The uniform fast paths below (a ballot, then a scalar branch) spare the wave
// the exec-mask bookkeeping of per-lane branches when no lane needs the rare
// case (C5 k_trace -2.6 %, C3 equal, round 4).
__device__ __forceinline__ void push(Lane& L, const Stack& st, uint32_t code, float h) {
  // wave-uniform fast path: no pushing lane needs the spill area
  if (!__any(L.sp >= kLdsSlots)) {
    st.code[L.sp * kTBlock] = code;
    st.h[L.sp * kTBlock] = h;
    L.sp++;
    return;
  }
  if (L.sp < kLdsSlots) {  // common case first: one LDS write, no further tests
    st.code[L.sp * kTBlock] = code;
    st.h[L.sp * kTBlock] = h;
    L.sp++;
    return;
  }
  if (L.sp >= st.cap) {  // cannot happen with the host's sizing; never write out of bounds
    *st.overflow = 1u;
    return;
  }
  stack_store(st, L.sp, code, h);
  L.sp++;
}

__device__ __forceinline__ void pop_top(Lane& L, const Stack& st, uint32_t& code, float& h) {
  L.sp--;
  stack_load(st, L.sp, code, h);
}

// Resume the deepest deferred child that is not culled: visited unless the
// closest hit found since is strictly before its entry (scene.rs:247, :264).
// Culled entries cost one LDS read. False when the stack is empty.
template <bool COUNT>
__device__ __forceinline__ bool pop(const DevScene& S, Lane& L, const Stack& st, uint32_t& nbytes) {
  while (L.sp > 0) {
    uint32_t code;
    float h;
    if (!__any(L.sp > kLdsSlots)) {  // wave-uniform: every popping lane's top entry is in LDS
      L.sp--;
      code = st.code[L.sp * kTBlock];
      h = st.h[L.sp * kTBlock];
    } else {
      pop_top(L, st, code, h);
    }
    if (!(L.best < h)) {
      if (!__any((code & 0xC0000000u) == 0x40000000u)) {  // no lane resumes a large leaf: selects
        const bool lc = (code & 0x80000000u) != 0;
        L.cnt = lc ? (code >> 24) & 0x7Fu : 0u;
        L.lf = lc ? code & 0xFFFFFFu : code;
        return true;
      }
      if (code & 0x80000000u) {
        L.cnt = (code >> 24) & 0x7Fu;
        L.lf = code & 0xFFFFFFu;
      } else if (code & 0x40000000u) {
        const float4 b = S.nodes[2 * (size_t)(code & 0x3FFFFFFFu) + 1];
        if (COUNT) nbytes += 16;
        L.lf = __float_as_uint(b.z);
        L.cnt = __float_as_uint(b.w);
      } else {
        L.lf = code;
        L.cnt = 0;
      }
      return true;
    }
  }
  return false;
}

// trace_shapes_md over one leaf (scene.rs:450-472) with max_dis = the closest
// hit on entry. Returns false on the SHADOW early exit (occluded).
template <bool SHADOW, bool TRI_ONLY, bool COUNT>
__device__ __forceinline__ bool leaf_test(const DevScene& S, Lane& L, const float4* tp, uint32_t lf, uint32_t cnt,
                                          int32_t light, float early, bool& occluded, uint32_t& visits,
                                          uint32_t& tests) {
  // tp: the records of shapes lf .. lf+cnt-1
  if (COUNT) { visits++; tests += cnt; }
  const float max_dis = L.best;
  bool found = false;
  float lb;  // read only once found (no initial register move)
  bool occ_any = false;
  uint32_t k0 = lf;
#if WPT_LEAF_PEEL
  if (TRI_ONLY) {
    // the first record outside the loop: a leaf holds one shape at least, and
    // most hold exactly one (no loop bookkeeping for them)
    float t;
    const bool hit = tri_hit(tp, L.o, L.d, t);
    const int32_t sid = (int32_t)(S.num_inf + lf);
    if (SHADOW) occ_any = hit && sid != light && t < early;
    found = hit && t <= max_dis;
    lb = t;
    L.best_id = found ? sid : L.best_id;
    k0 = lf + 1;
  }
#endif
  for (uint32_t k = k0; k < lf + cnt; k++) {
    float t;
    const float4* p = tp + 4 * (size_t)(k - lf);
    const bool hit = TRI_ONLY ? tri_hit(p, L.o, L.d, t) : prim_hit(S.kinds[k], p, L.o, L.d, t);
    if (TRI_ONLY) {
      // the exact acceptance as selects (a triangle hit has t > 0, so the
      // reference's 0 < t test is implied). A shadow walk's occluder is
      // noted and acted on after the leaf (an early return inside the loop
      // made the compiler version it: 4-7 % slower, round 4)
      const int32_t sid = (int32_t)(S.num_inf + k);
      if (SHADOW) occ_any = occ_any || (hit && sid != light && t < early);
      const bool acc = hit && t <= max_dis && (!found || t < lb);
      lb = acc ? t : lb;
      L.best_id = acc ? sid : L.best_id;
      found = found || acc;
      continue;
    }
    if (hit) {
      const int32_t sid = (int32_t)(S.num_inf + k);
      if (SHADOW && sid != light && t < early) {
        occluded = true;
        return false;
      }
      if (t <= max_dis && (!found || (0.0f < t && t < lb))) {
        found = true;
        lb = t;
        L.best_id = sid;
      }
    }
  }
  if (SHADOW && occ_any) {  // an occluder in this leaf: the verdict is "occluded" whatever else it holds
    occluded = true;
    return false;
  }
  if (found) L.best = lb;
  return true;
}

// Both children of the lane's current internal node (a BVH2 node pair): hit
// decisions, exact entry distances (box_entry) and the children's
// (left_first, count) words c = {L.lf, L.cnt, R.lf, R.cnt}. (Measured and
// rejected: the pair with its children's bounds interleaved, so that the two
// box tests' subtracts and multiplies issue as 6 + 6 packed f32 operations —
// C3 7 373 / 7 319 vs 7 444 Mray/s for this layout, both without SLP.)
__device__ __forceinline__ void expand_pair(const DevScene& S, const Hot& H, const Lane& L, float lim, bool& hl,
                                            bool& hr, float& ld, float& rd, uint32_t c[4]) {
  float4 la, lb4, ra, rb;
  // one flat load site: the pair from the block's LDS treelet or from the
  // node array, by a per-lane address (no branch between two load paths;
  // C5 k_trace -1.4 %, round 4)
  const float4* q = (kTreePairs > 0 && (L.lf & kTreeFlag)) ? H.gtree + 4 * (L.lf & ~kTreeFlag) : S.nodes + 2 * (size_t)L.lf;
  la = q[0];
  lb4 = q[1];
  ra = q[2];
  rb = q[3];
  // all 64 B in one round trip: the compiler otherwise defers the
  // left_first/count words past the box tests (a second dependent load)
  pin4(la);
  pin4(lb4);
  pin4(ra);
  pin4(rb);
  hl = box_entry(la, lb4, L.o, L.inv, lim, ld);
  hr = box_entry(ra, rb, L.o, L.inv, lim, rd);
  c[0] = __float_as_uint(lb4.z);
  c[1] = __float_as_uint(lb4.w);
  c[2] = __float_as_uint(rb.z);
  c[3] = __float_as_uint(rb.w);
}

// One traversal iteration on the lane's current node. Returns false when the
// traversal is finished. An internal node is expanded (both children's boxes
// in one 64 B load); when the nearer child is a leaf it is tested in the same
// iteration — exactly what the recursion does next — and the farther child
// is resumed by the pop after it unless the hit just found culls it
// (scene.rs:246-256). (Round 3 kept that farther child in registers: more
// VGPRs and branch state; the stack form is 2 % faster on C3, 4.6 % on C5's
// k_trace, round 4.)
// SHADOW: `occluded` is set on the early exit (a non-light shape hit strictly
// before `early` proves the reference's closest hit is an occluder).
template <bool SHADOW, bool TRI_ONLY, bool COUNT, bool LB = true>
__device__ __forceinline__ bool step(const DevScene& S, const Hot& H, Lane& L, const Stack& stk, int32_t light,
                                     float early, bool& occluded, uint32_t& visits, uint32_t& tests,
                                     uint32_t& nbytes) {
  // the farther child of a nearer leaf goes on the stack at its exact entry:
  // the pop after the leaf resumes it iff !(best < entry), the test the
  // recursion makes after the leaf (scene.rs:246-256); no per-lane "then far"
  // state, one leaf-test site
  bool do_pop = false;
  if (L.cnt == 0) {
    if (COUNT) { visits++; nbytes += 64; }
    float ld, rd;
    bool hl, hr;
    uint32_t c[4];
    const uint32_t lf0 = L.lf;
    expand_pair(S, H, L, L.best, hl, hr, ld, rd, c);
    do_pop = !hl && !hr;
    if (!do_pop) {
      const bool left_first = hl && (!hr || ld < rd);  // ties: right first (scene.rs:244)
      if (hl && hr) {
        const uint32_t flf = left_first ? c[2] : c[0], fcnt = left_first ? c[3] : c[1];
        push(L, stk, encode_child(flf, fcnt, left_first ? lf0 + 1 : lf0), left_first ? rd : ld);
      }
      L.lf = left_first ? c[0] : c[2];
      L.cnt = left_first ? c[1] : c[3];
    }
  }
#if WPT_LEAF_BATCH
  // a lane at a leaf waits (no state changes) until WPT_LEAF_BATCH lanes of
  // the wave are at one, or no active lane is left to expand, or fewer than
  // WPT_LEAF_BATCH_MIN lanes are active (a draining wave runs every body at
  // once): the leaf body then runs for more lanes at once. Each lane's own
  // operations are unchanged.
  bool run_leaf = true;
  if (LB && TRI_ONLY) {  // other shape kinds: C2's kernels measured 2-3 % slower with it compiled in
    const uint32_t na = (uint32_t)__popcll(__ballot(true)), nl = (uint32_t)__popcll(__ballot(L.cnt != 0));
    constexpr uint32_t T = SHADOW ? WPT_LEAF_BATCH_SH : WPT_LEAF_BATCH;
    constexpr uint32_t M = SHADOW ? WPT_LEAF_BATCH_MIN_SH : WPT_LEAF_BATCH_MIN;
    run_leaf = na < M || nl == na || nl >= T;
  }
#else
  constexpr bool run_leaf = true;
#endif
  if (L.cnt != 0 && run_leaf) {  // a leaf: resumed, or the nearer child just reached
    if (!leaf_test<SHADOW, TRI_ONLY, COUNT>(S, L, S.prims + 4 * (size_t)L.lf, L.lf, L.cnt, light, early, occluded,
                                            visits, tests))
      return false;
    do_pop = true;
  }
  return do_pop ? pop<COUNT>(S, L, stk, nbytes) : true;
}

// trace_shapes over all shapes (scene.rs:426-445), BVH disabled. TRI_ONLY:
// every shape is a triangle or an (infinite) plane.
template <bool TRI_ONLY>
__device__ void linear_closest(const DevScene& S, V3 o, V3 d, float& best, int32_t& best_id, uint32_t& tests) {
  bool found = false;
  for (uint32_t i = 0; i < S.num_shapes; i++) {
    float t;
    const uint32_t kind = S.all_kinds[i];
    const float4* p = S.all + 4 * (size_t)i;
    const bool h = TRI_ONLY ? (kind == kPlane ? plane_hit(p[0], o, d, t) : tri_hit(p, o, d, t))
                            : prim_hit(kind, p, o, d, t);
    if (h) {
      if (!found || (0.0f < t && t < best)) {
        found = true;
        best = t;
        best_id = (int32_t)i;
      }
    }
  }
  tests += S.num_shapes;
}

// trace_shapes over the infinite shapes (planes) first (scene.rs:165, :173).
__device__ __forceinline__ bool planes_closest(const DevScene& S, V3 o, V3 d, float& best, int32_t& best_id) {
  bool found = false;
  for (uint32_t i = 0; i < S.num_inf; i++) {
    float t;
    if (plane_hit(S.planes[i], o, d, t)) {
      if (!found || (0.0f < t && t < best)) {
        found = true;
        best = t;
        best_id = (int32_t)i;
      }
    }
  }
  return found;
}

#include "wpt_trav4.h"
#include "wpt_adaptive.h"
#include "wpt_stock.h"

// Start an extension ray: planes, then the guarded root (FAST: the BVH4
// fast path; else the reference's BVH2). False = finished.
template <bool TRI_ONLY, bool COUNT, bool FAST>
__device__ __forceinline__ bool begin_extend(const DevScene& S, const Hot& H, Lane& L, V3 o, V3 d, uint32_t& visits,
                                             uint32_t& tests, uint32_t& nbytes) {
  L.o = o;
  L.d = d;
  L.inv = inv_dir(d);
  L.best = __int_as_float(0x7f800000);
  L.best_id = -1;
  if (!S.use_bvh) {
    linear_closest<TRI_ONLY>(S, o, d, L.best, L.best_id, tests);
    if (L.best_id < 0) L.best = __int_as_float(0x7f800000);
    return false;
  }
  planes_closest(S, o, d, L.best, L.best_id);
  if (!S.num_finite) return false;
  return FAST ? enter_root4<COUNT>(H, L, visits, nbytes) : enter_root<COUNT>(S, H, L, visits, nbytes);
}

// Start a shadow ray (Scene::shadow_ray, scene.rs:104-133; origin already
// offset by EPSILON). Sets `early` (the light's own hit distance, capped at
// dir_len) and may finish immediately (occluded or not). False = finished.
template <bool TRI_ONLY, bool COUNT, bool FAST>
__device__ __forceinline__ bool begin_shadow(const DevScene& S, const Hot& H, Lane& L, V3 o, V3 d, float dir_len,
                                             int32_t light, float& early, bool& occluded, uint32_t& visits,
                                             uint32_t& tests, uint32_t& nbytes) {
  L.o = o;
  L.d = d;
  L.inv = inv_dir(d);
  L.best_id = -1;
  occluded = false;
  if (!S.use_bvh) {
    L.best = 0.0f;
    linear_closest<TRI_ONLY>(S, o, d, L.best, L.best_id, tests);
    return false;
  }
  early = dir_len;
  float tl;
  bool lhit;
  uint32_t k = 0;
  if (H.lrec)
    while (k < S.num_lights && H.lid[k] != light) k++;
  if (H.lrec && k < S.num_lights) {
    // the light's triangle from the block's LDS table (lights are triangles:
    // Tracable::pick_random, checked at upload)
    lhit = tri_hit_r(H.lq(k, 0), H.lq(k, 1), H.lq(k, 2), H.lq(k, 3), o, d, tl);
  } else {
    const uint32_t lk = (uint32_t)light - S.num_inf;
    const float4* lp = S.prims + 4 * (size_t)lk;
    lhit = TRI_ONLY ? tri_hit(lp, o, d, tl) : prim_hit(S.kinds[lk], lp, o, d, tl);
  }
  if (lhit) early = fminf(tl, dir_len);
  float pt = __int_as_float(0x7f800000);
  int32_t pid = -1;
  if (planes_closest(S, o, d, pt, pid) && pt < early) {  // a plane is never a light
    occluded = true;
    return false;
  }
  // Closest hits beyond dir_len never occlude, so the search starts capped
  // at dir_len (or at the plane hit, as the reference's max_dis).
  if (pid >= 0 && pt < dir_len) { L.best = pt; L.best_id = pid; }
  else { L.best = dir_len; L.best_id = -1; }
  if (!S.num_finite) return false;
  return FAST ? enter_root4<COUNT>(H, L, visits, nbytes) : enter_root<COUNT>(S, H, L, visits, nbytes);
}

__device__ __forceinline__ bool shadow_verdict(const Lane& L, float dir_len, int32_t light, bool occluded) {
  return occluded || (L.best_id >= 0 && L.best < dir_len && L.best_id != light);
}

struct GenParams {
  uint32_t W, H, npix;
  float w_inv, h_inv, ar;
  float cam[3];
  float cx, sx, cy, sy;  // cos/sin of rot_x, rot_y
  uint32_t seed;
  uint32_t half;         // W / 2
  uint32_t left_type, right_type;
};

// tracer.rs:175-193. Writes the batch's bounce-0 ray stream (path i at i).
// Path k of the progressive order: pixel k mod P, sample k div P; or, with
// rnd_off (a sample round, wpt_adaptive.h, or a stock batch, wpt_stock.h),
// the entry p whose consecutive range [rnd_off[p], rnd_off[p+1]) holds k,
// sample rnd_base[p] + k - rnd_off[p]; entry p is pixel rnd_list[p] when
// given (a stock refill over a half's pixel list), else partition pixel p.
// A stock batch (stock_slots != 0) writes the path's stock slot, pixel x
// slots + sample mod slots, instead of its pixel.
__global__ void __launch_bounds__(kBlock) k_generate(GenParams P, const uint32_t* __restrict__ part_pix, uint64_t k0,
                                                     uint32_t n, uint32_t* __restrict__ pix_out,
                                                     float4* __restrict__ thr,
                                                     float4* __restrict__ col, float4* __restrict__ ro,
                                                     float4* __restrict__ rd, uint32_t* __restrict__ count0,
                                                     const uint32_t* __restrict__ rnd_off,
                                                     const uint32_t* __restrict__ rnd_base,
                                                     const uint32_t* __restrict__ rnd_list, uint32_t stock_slots) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i == 0) *count0 = n;
  if (i >= n) return;
  const uint64_t k = k0 + i;
  uint32_t pl, sample;
  if (rnd_off) {
    uint32_t lo = 0, hi = P.npix;  // largest p with rnd_off[p] <= k
    while (lo + 1u < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((uint64_t)rnd_off[mid] <= k) lo = mid;
      else hi = mid;
    }
    pl = lo;
    sample = rnd_base[lo] + (uint32_t)(k - rnd_off[lo]);
  } else {
    pl = (uint32_t)(k % P.npix);
    sample = (uint32_t)(k / P.npix);
  }
  const uint32_t pixel = rnd_list ? rnd_list[pl] : part_pix ? part_pix[pl] : pl;
  const uint32_t x = pixel % P.W, y = pixel / P.W;
  uint32_t s = path_seed(P.seed, pixel, sample);
  const float fx = (((float)x + xs_next(s)) * P.w_inv - 0.5f) * P.ar;
  const float fy = 0.5f - ((float)y + xs_next(s)) * P.h_inv;
  V3 v = normalize(mk(fx, fy, 0.8f));
  v = mk(v.x, P.cx * v.y - P.sx * v.z, P.sx * v.y + P.cx * v.z);        // rot_x (vec3.rs:108-119)
  v = mk(P.cy * v.x + P.sy * v.z, v.y, (-P.sy) * v.x + P.cy * v.z);     // rot_y (vec3.rs:95-106)
  const uint32_t type = x < P.half ? P.left_type : P.right_type;
  pix_out[i] = stock_slots ? pixel * stock_slots + (sample & (stock_slots - 1u)) : rnd_off ? pl : pixel;
  thr[i] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(type << kTypeShift));
  col[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  ro[i] = make_float4(P.cam[0], P.cam[1], P.cam[2], __uint_as_float(s));  // w: the path's rng state
  rd[i] = make_float4(v.x, v.y, v.z, __uint_as_float(i));                // w: the path's index in the batch
}

template <bool TRI_ONLY>
__device__ __forceinline__ const float4* shape_rec(const DevScene& S, int32_t id, uint32_t& kind) {
  if (!S.use_bvh) { kind = S.all_kinds[id]; return S.all + 4 * (size_t)id; }
  if ((uint32_t)id < S.num_inf) { kind = kPlane; return nullptr; }
  kind = TRI_ONLY ? (uint32_t)kTri : S.kinds[id - S.num_inf];
  return S.prims + 4 * (size_t)(id - S.num_inf);
}

// ---------------------------------------------------------------------------
// PNEE light selection on the frozen octree: PhotonTree::sample
// (photon_tree.rs:81-160) with EmpiricalPDF::sample / bin_prob
// (empirical_pdf.rs:45-75). Nodes do not store bounds; they are re-derived
// top-down with child() exactly as the reference does.
// ---------------------------------------------------------------------------
// find_leaf (max_depth < 0) / find_node_cdf (photon_tree.rs:209-239):
// descend at most max_depth levels or to a leaf; bounds of the node reached.
// The frozen octree as the shade kernel reads it: child / cum either in the
// block's LDS copy (k_shade stages them when they fit) or in global memory;
// generic pointers, so one code path serves both.
template <class CP, class FP>
struct OctViewT {
  CP child;  // first of 8 children per node, 0 = leaf
  FP cum;    // cum_bins, num_lights per node
};
// Global memory, or the block's LDS copy (child array only, or child + CDFs):
// address-space-typed pointers, so LDS reads are ds_read (a generic pointer
// makes them flat loads, which wait for every outstanding memory operation).
using OctG = OctViewT<const uint32_t*, const float*>;
using OctL1 = OctViewT<const lds_u32*, const float*>;
using OctL2 = OctViewT<const lds_u32*, const lds_f32*>;

template <class OV>
__device__ uint32_t oct_find(const DevScene& S, const OV& O, V3 v, int max_depth, float b[6], int& depth) {
  b[0] = b[1] = b[2] = -kPhotonTreeSize;
  b[3] = b[4] = b[5] = kPhotonTreeSize;
  uint32_t node = 0;
  depth = 0;
  while (O.child[node] != 0u && (max_depth < 0 || depth < max_depth)) {
    float nb[6];
    const uint32_t ci = octant(b, v, nb);
    for (int k = 0; k < 6; k++) b[k] = nb[k];
    node = O.child[node] + ci;
    depth++;
  }
  return node;
}

template <class OV>
__device__ __forceinline__ float oct_bin_prob(const DevScene& S, const OV& O, uint32_t node, uint32_t i) {
  const auto c = O.cum + (size_t)node * S.num_lights;
  return i + 1u == S.num_lights ? 1.0f - c[i] : c[i + 1] - c[i];
}

template <class OV>
__device__ __forceinline__ float oct_node_prob(const DevScene& S, const OV& O, V3 v, int depth, uint32_t res) {
  float b[6];
  int d;
  return oct_bin_prob(S, O, oct_find(S, O, v, depth, b, d), res);
}

// per-axis interpolation weights of photon_tree.rs:96-131:
// (weight of own cell, weight of the adjacent cell, direction of the adjacent cell)
__device__ __forceinline__ void oct_axis(float v, float lo, float hi, float& w, float& wadj, float& off) {
  const float size = hi - lo;                  // x_size (aabb.rs:51-53)
  if (v > 0.5f * (lo + hi)) {                  // center (aabb.rs:81-87)
    const float left = (hi - (v - size * 0.5f)) / size;
    w = left;
    wadj = 1.0f - left;
    off = 1.0f;
  } else {
    const float right = ((v + size * 0.5f) - lo) / size;
    w = right;
    wadj = 1.0f - right;
    off = -1.0f;
  }
}

// Lattice form of the octree lookups. Cells at depth d are the cubes of side
// s = 2048 / 2^d on the lattice -1024 + k s; up to depth kOctLattice every
// bound child() computes (0.5 * (lo + hi), powers of two) is exact, so the
// descent's comparisons w < center choose exactly the bits of the index k of
// the cell [lo(k), lo(k+1)) holding w (clamped to the root box), from the
// most significant down. A descent then needs no bound arithmetic: one child
// read and a few integer operations per level.
constexpr int kOctLattice = 20;
#ifndef WPT_OCT_TABLE
#define WPT_OCT_TABLE 1  // 0: the neighbour cells by walks only (A/B builds)
#endif
__device__ __forceinline__ float oct_lo(int32_t k, float s) { return (float)k * s - kPhotonTreeSize; }
// Index at depth d of coordinate w, known to lie within one cell of k0.
__device__ __forceinline__ uint32_t oct_cell(float w, int32_t k0, float s, int d) {
  int32_t k = k0;
  if (w < oct_lo(k, s)) k--;
  else if (!(w < oct_lo(k + 1, s))) k++;
  const int32_t last = (1 << d) - 1;
  return (uint32_t)(k < 0 ? 0 : (k > last ? last : k));
}
// oct_find(max_depth = d) of the point whose depth-d cell is (ix, iy, iz).
template <class OV>
__device__ __forceinline__ uint32_t oct_walk(const OV& O, uint32_t ix, uint32_t iy, uint32_t iz, int d) {
  uint32_t node = 0;
  for (int l = d - 1; l >= 0; l--) {
    const uint32_t c = O.child[node];
    if (c == 0u) break;
    node = c + (((ix >> l) & 1u) << 2) + (((iy >> l) & 1u) << 1) + ((iz >> l) & 1u);
  }
  return node;
}

template <class OV>
__device__ void photon_sample(const DevScene& S, const OV& O, uint32_t& s, V3 v, uint32_t& light, float& pdf) {
  const float sz = kPhotonTreeSize;
  if (v.x < -sz || v.y < -sz || v.z < -sz || v.x > sz || v.y > sz || v.z > sz) {
    light = xs_next_in_range(s, S.num_lights);
    pdf = 1.0f / (float)S.num_lights;
    return;
  }
  float b[6];
  int depth;
  const uint32_t leaf = oct_find(S, O, v, -1, b, depth);
  float wx, wax, xo, wy, way, yo, wz, waz, zo;
  oct_axis(v.x, b[0], b[3], wx, wax, xo);
  oct_axis(v.y, b[1], b[4], wy, way, yo);
  oct_axis(v.z, b[2], b[5], wz, waz, zo);
  const float xs = b[3] - b[0], ys = b[4] - b[1], zs = b[5] - b[2];
  const bool self_x = xs_next(s) <= wx;
  const bool self_y = xs_next(s) <= wy;
  const bool self_z = xs_next(s) <= wz;
  const float ajx = xs * xo, ajy = ys * yo, ajz = zs * zo;
  // the 8 cells of the trilinear mix (corner c: bit 2 x, bit 1 y, bit 0 z
  // shifted by aj), found at v's leaf depth; the sampled cell is the corner
  // picked by the self_* draws (v + A + B + C, with A = x_off * (x_size, 0,
  // 0) etc.: the same f32 sums per component up to the sign of a zero)
  uint32_t corner[8];
  if (depth <= kOctLattice) {
    const int32_t kx = (int32_t)((b[0] + sz) / xs), ky = (int32_t)((b[1] + sz) / ys), kz = (int32_t)((b[2] + sz) / zs);
    const uint32_t ax = oct_cell(v.x + ajx, kx + (int32_t)xo, xs, depth);
    const uint32_t ay = oct_cell(v.y + ajy, ky + (int32_t)yo, ys, depth);
    const uint32_t az = oct_cell(v.z + ajz, kz + (int32_t)zo, zs, depth);
    corner[0] = leaf;
    // the usual case: each shifted coordinate lands in the adjacent cell
    // (clamped to the lattice); then the 8 cells are the leaf's precomputed
    // row for this offset case (build_photons: the same walks on the host)
    const int32_t last = (1 << depth) - 1;
    const auto adj = [&](int32_t k, float off) {
      const int32_t a = k + (int32_t)off;
      return (uint32_t)(a < 0 ? 0 : (a > last ? last : a));
    };
    if (WPT_OCT_TABLE && S.oct_corners && ax == adj(kx, xo) && ay == adj(ky, yo) && az == adj(kz, zo)) {
      const uint32_t ocase = (xo > 0.0f ? 4u : 0u) | (yo > 0.0f ? 2u : 0u) | (zo > 0.0f ? 1u : 0u);
      const uint4* row = reinterpret_cast<const uint4*>(S.oct_corners + 64 * (size_t)leaf + 8 * ocase);
      const uint4 q0 = row[0], q1 = row[1];
      corner[1] = q0.y;
      corner[2] = q0.z;
      corner[3] = q0.w;
      corner[4] = q1.x;
      corner[5] = q1.y;
      corner[6] = q1.z;
      corner[7] = q1.w;
    } else {
#pragma unroll
      for (int c = 1; c < 8; c++)
        corner[c] =
            oct_walk(O, (c & 4) ? ax : (uint32_t)kx, (c & 2) ? ay : (uint32_t)ky, (c & 1) ? az : (uint32_t)kz, depth);
    }
  } else {
    float nb[6];
    int d;
    corner[0] = leaf;
#pragma unroll
    for (int c = 1; c < 8; c++)
      corner[c] = oct_find(S, O, add(v, mk((c & 4) ? ajx : 0.0f, (c & 2) ? ajy : 0.0f, (c & 1) ? ajz : 0.0f)), depth, nb, d);
  }
  // EmpiricalPDF::sample: binary search of one draw in the sampled cell's CDF
  const int pick = (self_x ? 0 : 4) + (self_y ? 0 : 2) + (self_z ? 0 : 1);
  uint32_t node = corner[0];
#pragma unroll
  for (int c = 1; c < 8; c++) node = pick == c ? corner[c] : node;  // selects: corner[] stays in registers
  const auto cum = O.cum + (size_t)node * S.num_lights;
  const float r = xs_next(s);
  uint32_t lo = 0, hi = S.num_lights;
  while (lo + 1u < hi) {
    const uint32_t mid = (lo + hi) / 2u;
    if (cum[mid] <= r) lo = mid;
    else hi = mid;
  }
  light = lo;
  // trilinear mix of the 8 cells' probability of `light` (photon_tree.rs:142-156 order)
  float p = 0.0f;
  p += oct_bin_prob(S, O, corner[0], lo) * wx * wy * wz;
  p += oct_bin_prob(S, O, corner[4], lo) * wax * wy * wz;
  p += oct_bin_prob(S, O, corner[2], lo) * wx * way * wz;
  p += oct_bin_prob(S, O, corner[1], lo) * wx * wy * waz;
  p += oct_bin_prob(S, O, corner[6], lo) * wax * way * wz;
  p += oct_bin_prob(S, O, corner[3], lo) * wx * way * waz;
  p += oct_bin_prob(S, O, corner[5], lo) * wax * wy * waz;
  p += oct_bin_prob(S, O, corner[7], lo) * wax * way * waz;
  pdf = p;
}

// Hit::normal of Shape::trace for the closest hit (id, t) of ray (o, d).
template <bool TRI_ONLY>
__device__ __forceinline__ V3 hit_normal(const DevScene& S, int32_t id, V3 o, V3 d, float t) {
  uint32_t kind;
  const float4* rec = shape_rec<TRI_ONLY>(S, id, kind);
  if (rec) return TRI_ONLY ? tri_normal(rec, d) : prim_normal(kind, rec, o, d, t);
  V3 pn = ld3(S.planes[id]);  // plane.rs:45-78
  if (dot(pn, d) > 0.0f) pn = neg(pn);
  return normalize(pn);
}

// Hit record of an extension ray (read once by the shade kernel).
__device__ __forceinline__ void st_hit(float* t, int32_t* id, float tv, int32_t iv) {
  *t = tv;
  *id = iv;
}

struct ShadeParams {
  int max_depth;
  int debug;
};

// Dense per-bounce streams of the wavefront. The live paths of bounce b are
// entries 0..n_b-1 of a ray stream; k_shade appends the survivors to the next
// bounce's stream and the NEE shadow rays to the shadow stream, so every
// kernel reads and writes contiguous records (no queue indirection). The
// radiance of a path stays at its index in the batch (col[path]).
struct RayStream {
  float4* o;    // origin.xyz, w = the path's xorshift32 state bits
  float4* d;    // direction.xyz, w = the path's index in the batch (bits)
  float4* thr;  // throughput.xyz, w = flags (type, has_diffuse_bounced, depth)
};
struct ShadowStream {
  float4* o;    // origin.xyz (p + dir * EPSILON), w = |q - p|
  float4* d;    // direction.xyz, w = light shape id (bits)
  float4* c;    // NEE contribution.xyz, w = the path's index in the batch (bits)
};

// What one bounce of a path emits: its next extension ray and/or its shadow ray.
struct ShadeOut {
  bool alive, shadow;
  float4 ro, rd, th;
  float4 so, sd, sc;
};

// One bounce of trace_original_color (tracer.rs:237-329) for a path whose
// extension ray (o4, d4) hit shape `id` at t (id < 0: miss):
// emitter / miss termination, cosine-weighted diffuse bounce
// (material.rs:97-126), NEE light pick + Triangle::pick_random
// (triangle.rs:91-114), shadow-ray emission, depth cap, Russian roulette.
// Radiance changes go to col[path]; the path's next ray and its shadow ray to R.
// lq: the light records in the block's LDS (k_shade stages them when there
// are at most kShadeLights), else null: from global memory.
// CR (count rays): a path that ends writes its ray counts to col[path].w
// (extension rays | shadow rays << 16): the sample stock counts a sample's
// rays when a round takes it (wpt_stock.h). A template parameter, so the
// production kernels keep their registers (NEE k_shade at 72 VGPRs).
template <bool TRI_ONLY, bool PNEE, class OV, bool CR = false>
__device__ __forceinline__ void shade_path(const DevScene& S, const OV& O, const ShadeParams& P,
                                           float4* __restrict__ col, float t,
                                           int32_t id, float4 o4, float4 d4, float4 th4, ShadeOut& R,
                                           const lds_f4v* lq = nullptr) {
  const V3 o = ld3(o4), d = ld3(d4);
  const uint32_t path = __float_as_uint(d4.w);
  V3 thr = ld3(th4);
  uint32_t flags = __float_as_uint(th4.w);
  const uint32_t type = (flags >> kTypeShift) & 3u;
  const bool has_nee = type == 1u || type == 2u;
  bool bounced = (flags & kFlagBounced) != 0;
  const uint32_t depth = ((flags >> kDepthShift) & kDepthMask) + 1u;
  // the path's rays when it ends here: its `depth` extension rays and its
  // shadow rays (ShadeParams::count_rays)
  auto end_counts = [&](uint32_t nsh) {
    if constexpr (CR) reinterpret_cast<uint32_t*>(col + path)[3] = depth | (nsh << 16);
  };
  if (id < 0) {
    // miss: color += throughput * background (tracer.rs:325-327). When the
    // product is +0 in every component (black background, finite throughput)
    // the sum is the colour itself (colours are sums of non-negative terms
    // from +0, never -0), so the read-modify-write is skipped.
    const V3 add_c = mulv(thr, mk(S.bg[0], S.bg[1], S.bg[2]));
    if ((__float_as_uint(add_c.x) | __float_as_uint(add_c.y) | __float_as_uint(add_c.z)) != 0u) {
      const float4 c4 = col[path];
      const V3 c = add(ld3(c4), add_c);
      col[path] = make_float4(c.x, c.y, c.z, c4.w);
    }
    end_counts(flags >> kShadowShift);
    return;
  }
  const float4 m = S.mats[id];
  // triangle scenes: the hit normal's loads go out with the material's, one
  // round trip instead of two (pure computation; unused on an emitter)
  V3 nrm = mk(0.0f, 0.0f, 0.0f);
  if (TRI_ONLY) nrm = hit_normal<TRI_ONLY>(S, id, o, d, t);
  const V3 hp = add(o, scale(d, t));  // ray.at (ray.rs:36-38)
  if (m.w != 0.0f) {
    // emissive (tracer.rs:245-254)
    if (P.debug ? !bounced : (!has_nee || !bounced)) {
      const float4 c4 = col[path];
      const V3 c = add(ld3(c4), mulv(thr, ld3(m)));
      col[path] = make_float4(c.x, c.y, c.z, c4.w);
    }
    end_counts(flags >> kShadowShift);
    return;
  }
  if (!TRI_ONLY) nrm = hit_normal<TRI_ONLY>(S, id, o, d, t);
  uint32_t s = __float_as_uint(o4.w);
  // sample_hemisphere (material.rs:97-118)
  const float r1 = xs_next(s);
  const float r2 = xs_next(s);
  const float ang = (2.0f * kPi) * r1;
  const float x = mcos(ang) * sqrtf(1.0f - r2);
  const float y = sqrtf(r2);
  const float z = msin(ang) * sqrtf(1.0f - r2);
  const V3 xn = orthogonal(nrm);
  const V3 zn = cross(nrm, xn);
  const V3 wi = normalize(add(add(scale(xn, x), scale(nrm, y)), scale(zn, z)));
  const float pdf = dot(wi, nrm) / kPi;
  // brdf = Color3(color) / PI (material.rs:120-126; color3.rs:90-95 clamps)
  const float ipi = 1.0f / kPi;
  const V3 brdf = mk(clamp01(ipi * m.x), clamp01(ipi * m.y), clamp01(ipi * m.z));
  const float cos_i = dot(wi, nrm);
  thr = divs(scale(mulv(thr, brdf), cos_i), pdf);
  const V3 no = add(hp, scale(wi, kEpsilon));
  bounced = true;
  if (has_nee && S.num_lights > 0) {
    // tracer.rs:267-313: light pick, uniform (NEE) or from the photon octree
    // (PNEE, tracer.rs:270-273)
    uint32_t li;
    float light_chance;
    if (PNEE && type == 2u) {
      photon_sample(S, O, s, hp, li, light_chance);
    } else {
      li = xs_next_in_range(s, S.num_lights);
      light_chance = 1.0f / (float)S.num_lights;
    }
    float4 L0, L1, L2, L3, L4;
    if (lq) {
      const lds_f4v* q = lq + 5 * li;
      L0 = to_f4(q[0]);
      L1 = to_f4(q[1]);
      L2 = to_f4(q[2]);
      L3 = to_f4(q[3]);
      L4 = to_f4(q[4]);
    } else {
      const float4* L = S.lights + 5 * (size_t)li;
      L0 = L[0];
      L1 = L[1];
      L2 = L[2];
      L3 = L[3];
      L4 = L[4];
    }
    // Triangle::pick_random (triangle.rs:91-114)
    const float q1 = xs_next(s);
    const float q2 = xs_next(s);
    const float q1s = sqrtf(q1);
    const V3 pt = add(add(scale(ld3(L0), 1.0f - q1s), scale(ld3(L1), q1s * (1.0f - q2))), scale(ld3(L2), q2 * q1s));
    V3 ln = ld3(L3);
    if (xs_next(s) > 0.5f) ln = neg(ln);
    const V3 inten = ld3(L4);
    V3 tl = sub(pt, hp);
    const float d2 = dot(tl, tl);
    const float dl = sqrtf(d2);
    tl = divs(tl, dl);
    const float ci = dot(tl, nrm);
    const float co = dot(neg(tl), ln);
    if (ci > 0.0f && co > 0.0f) {
      if (P.debug) {
        const float4 c4 = col[path];
        const V3 c = add(ld3(c4), mulv(thr, inten));
        col[path] = make_float4(c.x, c.y, c.z, c4.w);
      } else {
        const float solid = (L0.w * co) / d2;
        const V3 contrib = scale(scale(scale(mulv(thr, inten), solid), ci), 1.0f / light_chance);
        // Scene::shadow_ray: dir = (q-p)/|q-p|, origin p + dir*EPSILON
        const V3 sorig = add(hp, scale(tl, kEpsilon));
        R.so = make_float4(sorig.x, sorig.y, sorig.z, dl);
        R.sd = make_float4(tl.x, tl.y, tl.z, L1.w);
        R.sc = make_float4(contrib.x, contrib.y, contrib.z, d4.w);
        R.shadow = true;
      }
    }
  }
  const bool capped = P.max_depth > 0 && (int)depth >= P.max_depth;
  if (!capped && depth < (uint32_t)kMaxBounces) {
    // Russian roulette (tracer.rs:318-324)
    const float keep = fmaxf(fminf(fmaxf(fmaxf(thr.x, thr.y), thr.z), 0.9f), 0.1f);
    if (xs_next(s) < keep) {
      thr = scale(thr, 1.0f / keep);
      const uint32_t nsh = (flags >> kShadowShift) + (R.shadow ? 1u : 0u);
      flags = (flags & ~((~0u) << kDepthShift)) | (depth << kDepthShift) | (nsh << kShadowShift) | kFlagBounced;
      R.ro = make_float4(no.x, no.y, no.z, __uint_as_float(s));
      R.rd = make_float4(wi.x, wi.y, wi.z, d4.w);
      R.th = make_float4(thr.x, thr.y, thr.z, __uint_as_float(flags));
      R.alive = true;
    }
  }
  if (!R.alive) end_counts((flags >> kShadowShift) + (R.shadow ? 1u : 0u));
}

// Shade kernel: one bounce of the path loop for paths 0..n-1 of the input
// stream. A block shades 1024 consecutive paths, then appends the survivors
// and the shadow rays in path order: one block-wide scan of the two flags and
// ONE 64-bit atomic add (survivors in the low word, shadow rays in the high
// word) reserves both output ranges. Blocks append in completion order; a
// path's result does not depend on its position, so the frame is the same
// bits for any order (col and the accumulation are indexed by path).
// OCT (PNEE): where photon_sample reads the octree: 0 global memory, 1 the
// child array from LDS, 2 child array and CDFs from LDS (oct_lds_words).
template <bool TRI_ONLY, bool PNEE, int OCT, bool CR = false>
__global__ void WPT_SHADE_BOUNDS k_shade(DevScene S, ShadeParams P, RayStream in, RayStream out,
                                                       ShadowStream sh, float4* __restrict__ col,
                                                       const uint32_t* __restrict__ count, const float* __restrict__ t_in,
                                                       const int32_t* __restrict__ id_in,
                                                       unsigned long long* __restrict__ append) {
  constexpr uint32_t kWaves = kShadeBlock / 64;
  __shared__ uint32_t s_off[2][kWaves];
  __shared__ f4v s_light[5 * kShadeLights];
  const uint32_t n = *count;
  // the light records (5 float4 each) into LDS when they fit: the NEE light
  // pick is then an LDS read instead of a dependent global round trip
  const bool lds_lights = S.num_lights <= kShadeLights;
  if (lds_lights) {
    for (uint32_t k = threadIdx.x; k < 5 * S.num_lights; k += kShadeBlock) {
      const float4 v = S.lights[k];
      s_light[k] = f4v{v.x, v.y, v.z, v.w};
    }
  }
  // PNEE: the frozen octree (child, then the CDFs) into LDS when it fits the
  // dynamic shared memory the launch gave (oct_lds_words; the per-level
  // descents of photon_sample are chains of dependent loads)
  extern __shared__ uint32_t s_oct[];
  if (PNEE && OCT != 0) {
    const uint32_t nc = S.oct_nodes, nw = S.oct_lds_words;
    for (uint32_t k = threadIdx.x; k < nw; k += kShadeBlock)
      s_oct[k] = k < nc ? S.oct_child[k] : __float_as_uint(S.oct_cum[k - nc]);
  }
  __syncthreads();  // the light records and the octree
  using OV = std::conditional_t<OCT == 2, OctL2, std::conditional_t<OCT == 1, OctL1, OctG>>;
  OV O;
  if constexpr (OCT == 2) {
    O.child = (const lds_u32*)s_oct;
    O.cum = (const lds_f32*)(s_oct + S.oct_nodes);
  } else if constexpr (OCT == 1) {
    O.child = (const lds_u32*)s_oct;
    O.cum = S.oct_cum;
  } else {
    O.child = S.oct_child;
    O.cum = S.oct_cum;
  }
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  for (uint32_t i0 = blockIdx.x * kShadeBlock; i0 < n; i0 += gridDim.x * kShadeBlock) {  // block-uniform
    const uint32_t i = i0 + threadIdx.x;
    ShadeOut R;
    R.alive = R.shadow = false;
    if (i < n)
      shade_path<TRI_ONLY, PNEE, OV, CR>(S, O, P, col, t_in[i], id_in[i], in.o[i], in.d[i], in.thr[i], R,
                                     lds_lights ? (const lds_f4v*)s_light : nullptr);
    const uint64_t am = __ballot(R.alive), sm = __ballot(R.shadow);
    if (lane == 0) {
      s_off[0][wid] = (uint32_t)__popcll(am);
      s_off[1][wid] = (uint32_t)__popcll(sm);
    }
    __syncthreads();
    if (wid == 0) {
      const uint32_t a = lane < kWaves ? s_off[0][lane] : 0u, b = lane < kWaves ? s_off[1][lane] : 0u;
      uint32_t ia = a, ib = b;
#pragma unroll
      for (uint32_t k = 1; k < kWaves; k <<= 1) {
        const uint32_t ya = __shfl_up(ia, k, 64), yb = __shfl_up(ib, k, 64);
        if (lane >= k) { ia += ya; ib += yb; }
      }
      unsigned long long base = 0ull;
      if (lane == kWaves - 1) base = atomicAdd(append, (unsigned long long)ia | ((unsigned long long)ib << 32));
      const uint32_t ba = (uint32_t)__shfl((int)(uint32_t)base, (int)(kWaves - 1), 64);
      const uint32_t bb = (uint32_t)__shfl((int)(uint32_t)(base >> 32), (int)(kWaves - 1), 64);
      if (lane < kWaves) {
        s_off[0][lane] = ba + ia - a;
        s_off[1][lane] = bb + ib - b;
      }
    }
    __syncthreads();
    if (R.alive) {
      const uint32_t p = s_off[0][wid] + (uint32_t)__popcll(am & below);
      st_stream(out.o + p, R.ro);
      st_stream(out.d + p, R.rd);
      st_stream(out.thr + p, R.th);
    }
    if (R.shadow) {
      const uint32_t p = s_off[1][wid] + (uint32_t)__popcll(sm & below);
      st_stream(sh.o + p, R.so);
      st_stream(sh.d + p, R.sd);
      st_stream(sh.c + p, R.sc);
    }
    __syncthreads();  // s_off is rewritten by the next iteration
  }
}

// Wave-interleaved work feed of the persistent traversal kernels. The stream
// is cut into kFeedChunk-entry chunks; wave w of W owns chunks w, w+W, w+2W, ... and
// its idle lanes take the wave's next entries in lane order (ballot + prefix
// popcount). No atomics; the wave's lanes share its work, so a lane that
// finishes early takes more rays (only the wave's last chunk has a tail);
// and a refill hands a wave consecutive entries (coherent rays).
struct WaveFeed {
  uint32_t n, v, wave, nwaves;  // v = entries this wave has taken (wave-uniform)
  __device__ WaveFeed(uint32_t n_) : n(n_), v(0) {
    wave = (blockIdx.x * kTBlock + threadIdx.x) >> 6;
    nwaves = (gridDim.x * kTBlock) >> 6;
  }
  static constexpr uint32_t K = kFeedChunk;
  __device__ uint32_t pos(uint32_t k) const { return ((k / K) * nwaves + wave) * K + (k % K); }
  __device__ bool more() const { return pos(v) < n; }
  // entries of the stream this wave has taken (v counts the last refill's
  // positions past n too)
  __device__ uint32_t taken() const { return taken_below(n); }
  // of those, the entries at stream positions below m (m <= n)
  __device__ uint32_t taken_below(uint32_t m) const {
    const uint32_t C = m / K, rem = m % K;
    const uint32_t full = C > wave ? (C - wave - 1u) / nwaves + 1u : 0u;
    const uint32_t part = (rem != 0u && C % nwaves == wave) ? rem : 0u;
    return min(v, full * K + part);
  }
  // Lanes in `take_m` get consecutive entries; returns this lane's stream
  // position (>= n: nothing left).
  __device__ uint32_t take(uint64_t take_m) {
    const uint32_t rank = (uint32_t)__popcll(take_m & ((1ull << (threadIdx.x & 63)) - 1ull));
    const uint32_t p = pos(v + rank);
    v += (uint32_t)__popcll(take_m);
    return p;
  }
};

// ---------------------------------------------------------------------------
// PNEE preprocessing (RenderInstance::preprocess_photons, tracer.rs:126-152)
// for photons k0 .. k0+n-1, each on its own stream photon_seed(seed, k):
// light pick, Triangle::pick_random, Rng::next_hemisphere (rng.rs:50-68) and
// the photon ray; k_extend traces it (Scene::trace); k_photon_hit keeps
// diffuse hits as (hit point + normal*EPSILON, ln·dir * max(I)).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_photon_gen(DevScene S, uint32_t seed, uint32_t k0, uint32_t n,
                                                       float4* __restrict__ ro, float4* __restrict__ rd,
                                                       float4* __restrict__ rec) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t s = photon_seed(seed, k0 + i);
  const uint32_t li = xs_next_in_range(s, S.num_lights);
  const float4* L = S.lights + 5 * (size_t)li;
  const float4 L0 = L[0], L1 = L[1], L2 = L[2], L3 = L[3], L4 = L[4];
  const float q1 = xs_next(s);
  const float q2 = xs_next(s);
  const float q1s = sqrtf(q1);
  const V3 pt = add(add(scale(ld3(L0), 1.0f - q1s), scale(ld3(L1), q1s * (1.0f - q2))), scale(ld3(L2), q2 * q1s));
  V3 ln = ld3(L3);
  if (xs_next(s) > 0.5f) ln = neg(ln);
  float x, y, z;
  do {  // next_hemisphere: rejection sampling of the unit ball
    x = xs_next(s) * 2.0f - 1.0f;
    y = xs_next(s) * 2.0f - 1.0f;
    z = xs_next(s) * 2.0f - 1.0f;
  } while (x * x + y * y + z * z > 1.0f);
  V3 v = normalize(mk(x, y, z));
  if (dot(v, ln) < 0.0f) v = neg(v);
  const V3 o = add(pt, scale(v, kEpsilon));
  ro[i] = make_float4(o.x, o.y, o.z, 0.0f);
  rd[i] = make_float4(v.x, v.y, v.z, 0.0f);
  const float imax = fmaxf(fmaxf(L4.x, L4.y), L4.z);
  rec[i] = make_float4(__uint_as_float(li), dot(ln, v) * imax, 0.0f, 0.0f);
}

template <bool TRI_ONLY>
__global__ void __launch_bounds__(kBlock) k_photon_hit(DevScene S, uint32_t n, const float4* __restrict__ ro,
                                                       const float4* __restrict__ rd, const float* __restrict__ t_in,
                                                       const int32_t* __restrict__ id_in,
                                                       const float4* __restrict__ rec, float4* __restrict__ hit_out,
                                                       uint32_t* __restrict__ light_out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int32_t id = id_in[i];
  const float4 r = rec[i];
  if (id < 0 || S.mats[id].w != 0.0f) {  // miss, or not diffuse (is_diffuse, material.rs:88-93)
    light_out[i] = 0xFFFFFFFFu;
    return;
  }
  const V3 o = ld3(ro[i]), d = ld3(rd[i]);
  const float t = t_in[i];
  const V3 nrm = hit_normal<TRI_ONLY>(S, id, o, d, t);
  const V3 hp = add(add(o, scale(d, t)), scale(nrm, kEpsilon));
  hit_out[i] = make_float4(hp.x, hp.y, hp.z, r.y);
  light_out[i] = __float_as_uint(r.x);
}

// COUNT builds: SIMD use of the traversal loop's two bodies, on a scale that
// cannot exceed 64. Per wave iteration, the lanes about to expand an internal
// node and those about to test a leaf (then pop); a body counts as executed
// when at least one lane runs it. work[10..13] = expand lanes, expand bodies,
// leaf lanes, leaf bodies (summed over the traversal kernels).
// Wave timeline probe (WPT_OPT_PROBE; S.probe null otherwise): per wave of a
// traversal launch its start, the moment its feed ran dry (no rays left to
// take), its end (steady clock) and the rays it took.
__device__ __forceinline__ uint32_t probe_now() { return (uint32_t)wall_clock64(); }
__device__ __forceinline__ void probe_close(const DevScene& S, uint32_t t0, uint32_t t_dry, uint32_t taken) {
  const uint32_t t1 = probe_now();
  if ((threadIdx.x & 63u) == 0u)
    S.probe[(blockIdx.x * kTBlock + threadIdx.x) >> 6] = make_uint4(t0, t_dry ? t_dry : t0, t1, taken);
}

// Work counters (COUNT builds): d_work_ holds kWorkCopies copies of the
// kWorkWords counters; a wave adds its sum (lane 0, one atomic per counter)
// to copy blockIdx % kWorkCopies. Every lane adding to one address (the
// round-4 form) queued ~10 same-address atomics per lane at the memory side:
// the counted C5 k_trace ran 3x the production kernel's time.
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ void work_add_wave(unsigned long long* work, uint32_t c, unsigned long long v) {
  // v already the wave's total (lane 0 adds it)
  if ((threadIdx.x & 63u) == 0u && v) atomicAdd(work + (blockIdx.x & (kWorkCopies - 1u)) * kWorkWords + c, v);
}
__device__ __forceinline__ void work_add(unsigned long long* work, uint32_t c, unsigned long long v) {
  work_add_wave(work, c, wave_sum(v));
}

struct BodyLanes {
  // wave-uniform (from ballots, so kept in SGPRs): loop iterations, live
  // lanes of each ray kind (a: extension, b: shadow), and the two bodies
  uint32_t it = 0, live_a = 0, live_b = 0, ex_lanes = 0, ex_bodies = 0, lf_lanes = 0, lf_bodies = 0;
  __device__ __forceinline__ void count(bool live, bool kind_b, const Lane& L) {
    it++;
    live_a += (uint32_t)__popcll(__ballot(live && !kind_b));
    live_b += (uint32_t)__popcll(__ballot(live && kind_b));
    const uint32_t e = (uint32_t)__popcll(__ballot(live && L.cnt == 0));
    const uint32_t f = (uint32_t)__popcll(__ballot(live && L.cnt != 0));
    ex_lanes += e;
    ex_bodies += e ? 1u : 0u;
    lf_lanes += f;
    lf_bodies += f ? 1u : 0u;
  }
  // lane iterations (64 per wave iteration) and live lane iterations of
  // kind a to words ca, ca + 1 and of kind b to cb, cb + 1 (cb < 0: none)
  __device__ __forceinline__ void flush(unsigned long long* work, int ca, int cb) const {
    work_add_wave(work, ca, 64ull * it);
    work_add_wave(work, ca + 1, live_a);
    if (cb >= 0) {
      work_add_wave(work, cb, 64ull * it);
      work_add_wave(work, cb + 1, live_b);
    }
    work_add_wave(work, 10, ex_lanes);
    work_add_wave(work, 11, ex_bodies);
    work_add_wave(work, 12, lf_lanes);
    work_add_wave(work, 13, lf_bodies);
  }
};

// Persistent closest-hit kernel for extension rays (primary and bounce,
// Scene::trace) over rays 0..n-1 of a dense stream: each lane traces one ray
// at a time; idle lanes take the wave's next rays from its WaveFeed together
// once enough of the wave is idle (refill_lanes). TRAV: 0 the reference's
// BVH2 (exact); 1 the BVH4 fast path (a flagged result re-traced by the exact
// machine on the same lane; fallbacks[0] counts them).
template <bool TRI_ONLY, bool COUNT, int TRAV>
__global__ void WPT_TRACE_BOUNDS k_extend(DevScene S, const float4* __restrict__ ro,
                                                   const float4* __restrict__ rd, const uint32_t* __restrict__ count,
                                                   float* __restrict__ t_out, int32_t* __restrict__ id_out,
                                                   uint2* __restrict__ spill, unsigned long long* work,
                                                   uint32_t* fallbacks) {
  constexpr bool FAST = TRAV == 1;
  __shared__ uint32_t s_code[kLdsSlots * kTBlock];
  __shared__ float s_h[kLdsSlots * kTBlock];
  __shared__ float s_lrec[16 * kLdsLights];
  __shared__ int32_t s_lid[kLdsLights];
  __shared__ f4v s_tree[4 * kTreePairs + 1];
  const uint32_t n = *count;
  const Hot H = load_hot(S, (lds_f32h*)s_lrec, (lds_i32*)s_lid, (lds_f4v*)s_tree, (const float4*)s_tree);
  const uint32_t G = gridDim.x * kTBlock;
  const Stack stk{(lds_u32*)(s_code + threadIdx.x), (lds_f32*)(s_h + threadIdx.x),
                  spill + blockIdx.x * kTBlock + threadIdx.x, G, S.stack_cap, S.overflow};
  uint32_t visits = 0, tests = 0, nbytes = 0;
  WaveFeed feed(n);
  const uint32_t p_t0 = S.probe ? probe_now() : 0u;
  uint32_t p_dry = 0u;
  Lane L;
  uint32_t slot = 0;
  bool live = false;  // a ray is being traversed on this lane
  bool fast = FAST;   // current mode of the lane's ray (BVH4 path)
  bool tie = false, quirk = false, dummy = false;
  BodyLanes bodies;
  const float inf = __int_as_float(0x7f800000);
  for (;;) {
    const uint64_t idle_m = __ballot(!live);
    const uint32_t nidle = (uint32_t)__popcll(idle_m);
    if (nidle != 0 && (nidle >= S.refill_lanes || nidle == 64u) && feed.more()) {
      const uint32_t q0 = feed.take(idle_m);
      const bool got = q0 < n;
      if (S.probe && p_dry == 0u && !feed.more()) p_dry = probe_now();
      if (!live && got) {
        slot = q0;
        fast = FAST;
        tie = quirk = false;
        const float4 o4 = ro[slot], d4 = rd[slot];
        live = begin_extend<TRI_ONLY, COUNT, FAST>(S, H, L, ld3(o4), ld3(d4), visits, tests, nbytes);
        if (!live) st_hit(t_out + slot, id_out + slot, L.best_id >= 0 ? L.best : inf, L.best_id);
      }
    }
    if (!__any(live) && !feed.more()) {
      if (S.probe) probe_close(S, p_t0, p_dry, feed.taken());
      break;
    }
    if (COUNT) bodies.count(live, false, L);
    if (live) {
      const bool more = (FAST && fast)
                            ? step4<false, TRI_ONLY, COUNT>(S, L, stk, -1, 0.0f, dummy, tie, quirk, visits, tests, nbytes)
                            : step<false, TRI_ONLY, COUNT>(S, H, L, stk, -1, 0.0f, dummy, visits, tests, nbytes);
      if (!more) {
        live = false;
        if (FAST && fast && (tie || quirk)) {
          // the reference's order could pick another result: redo exactly
          fast = false;
          atomicAdd(fallbacks, 1u);
          live = begin_extend<TRI_ONLY, COUNT, false>(S, H, L, L.o, L.d, visits, tests, nbytes);
        }
        if (!live) st_hit(t_out + slot, id_out + slot, L.best_id >= 0 ? L.best : inf, L.best_id);
      }
    }
  }
  if (COUNT) {
    work_add(work, 0, visits);
    work_add(work, 1, tests);
    work_add(work, 2, nbytes);
    bodies.flush(work, 6, -1);
  }
}

// NEE contribution of an unoccluded shadow ray: col[path] += c.xyz
// (tracer.rs:304-308; Vec3 AddAssign, vec3.rs:179-184).
__device__ __forceinline__ void add_contribution(float4* __restrict__ col, float4 c) {
  const uint32_t path = __float_as_uint(c.w);
  float4 v = col[path];
  v.x += c.x;
  v.y += c.y;
  v.z += c.z;
  col[path] = v;
}

// Persistent shadow-ray kernel (Scene::shadow_ray) over shadow rays 0..n-1 of
// a dense stream: unoccluded rays add their precomputed NEE contribution to
// their path's colour. With occ_out set (parity hook) it records the
// occlusion verdict instead. TRAV as k_extend (fallbacks[1] counts the
// BVH4 fast path's exact re-traces).
template <bool TRI_ONLY, bool COUNT, int TRAV>
__global__ void WPT_TRACE_BOUNDS k_shadow(DevScene S, const uint32_t* __restrict__ count,
                                                   const float4* __restrict__ so, const float4* __restrict__ sd,
                                                   const float4* __restrict__ sc, float4* __restrict__ col,
                                                   uint8_t* __restrict__ occ_out, uint2* __restrict__ spill,
                                                   unsigned long long* work, uint32_t* fallbacks) {
  constexpr bool FAST = TRAV == 1;
  __shared__ uint32_t s_code[kLdsSlots * kTBlock];
  __shared__ float s_h[kLdsSlots * kTBlock];
  __shared__ float s_lrec[16 * kLdsLights];
  __shared__ int32_t s_lid[kLdsLights];
  __shared__ f4v s_tree[4 * kTreePairs + 1];
  const uint32_t n = *count;
  const Hot H = load_hot(S, (lds_f32h*)s_lrec, (lds_i32*)s_lid, (lds_f4v*)s_tree, (const float4*)s_tree);
  const uint32_t G = gridDim.x * kTBlock;
  const Stack stk{(lds_u32*)(s_code + threadIdx.x), (lds_f32*)(s_h + threadIdx.x),
                  spill + blockIdx.x * kTBlock + threadIdx.x, G, S.stack_cap, S.overflow};
  uint32_t visits = 0, tests = 0, nbytes = 0;
  WaveFeed feed(n);
  const uint32_t p_t0 = S.probe ? probe_now() : 0u;
  uint32_t p_dry = 0u;
  Lane L;
  uint32_t cur = 0;
  float dir_len = 0.0f, early = 0.0f;
  int32_t light = -1;
  bool occluded = false;
  bool live = false;
  bool fast = FAST;
  bool tie = false, quirk = false;
  BodyLanes bodies;
  for (;;) {
    bool finished = false;
    const uint64_t idle_m = __ballot(!live);
    const uint32_t nidle = (uint32_t)__popcll(idle_m);
    if (nidle != 0 && (nidle >= S.refill_lanes_sh || nidle == 64u) && feed.more()) {
      const uint32_t q0 = feed.take(idle_m);
      const bool got = q0 < n;
      if (S.probe && p_dry == 0u && !feed.more()) p_dry = probe_now();
      if (!live && got) {
        cur = q0;
        const float4 o4 = so[cur], d4 = sd[cur];
        dir_len = o4.w;
        light = (int32_t)__float_as_uint(d4.w);
        fast = FAST;
        tie = quirk = false;
        live = begin_shadow<TRI_ONLY, COUNT, FAST>(S, H, L, ld3(o4), ld3(d4), dir_len, light, early, occluded, visits,
                                                   tests, nbytes);
        finished = !live;
      }
    }
    if (!__any(live || finished) && !feed.more()) {
      if (S.probe) probe_close(S, p_t0, p_dry, feed.taken());
      break;
    }
    if (COUNT) bodies.count(live, false, L);
    if (live) {
      const bool more =
          (FAST && fast)
              ? step4<true, TRI_ONLY, COUNT>(S, L, stk, light, early, occluded, tie, quirk, visits, tests, nbytes)
              : step<true, TRI_ONLY, COUNT>(S, H, L, stk, light, early, occluded, visits, tests, nbytes);
      if (!more) {
        live = false;
        finished = true;
        if (FAST && fast && !occluded && (tie || quirk)) {
          // the reference's order could pick another closest shape: redo exactly
          fast = false;
          atomicAdd(fallbacks + 1, 1u);
          if (begin_shadow<TRI_ONLY, COUNT, false>(S, H, L, L.o, L.d, dir_len, light, early, occluded, visits, tests,
                                                   nbytes)) {
            live = true;
            finished = false;
          }
        }
      }
    }
    if (finished) {
      const bool occ = shadow_verdict(L, dir_len, light, occluded);
      if (occ_out) occ_out[cur] = occ ? 1 : 0;
      else if (!occ) add_contribution(col, sc[cur]);
    }
  }
  if (COUNT) {
    work_add(work, 3, visits);
    work_add(work, 4, tests);
    work_add(work, 5, nbytes);
    bodies.flush(work, 8, -1);
  }
}

// Fused traversal of bounce b's extension rays and bounce b-1's shadow rays
// (WPT_FUSED), on the reference's BVH2 (exact). The two sets
// are independent: a shadow ray only adds its contribution to its path's
// colour, and shade(b), the next writer of that colour, runs after this
// kernel, so the reference's order of colour additions holds. One launch per
// bounce instead of two: one pool of rays (fuller refills) and one drain
// instead of two. Feed positions q < n_ext are extension rays, the others
// shadow rays. A shadow-ray step is the extension step plus the early exit;
// extension rays run it with light = -1 and early = -inf, where the exit can
// never fire.
template <bool TRI_ONLY, bool COUNT>
#ifndef WPT_FUSED_WAVES
#define WPT_FUSED_WAVES 8  // k_trace's waves per SIMD (C5 +4 % over its natural 7)
#endif
__global__ void __launch_bounds__(kTBlock, TRI_ONLY ? WPT_FUSED_WAVES : 1) k_trace(DevScene S, const float4* __restrict__ ro,
                                                  const float4* __restrict__ rd, const uint32_t* __restrict__ cnt_ext,
                                                  float* __restrict__ t_out, int32_t* __restrict__ id_out,
                                                  const uint32_t* __restrict__ cnt_sh, const float4* __restrict__ so,
                                                  const float4* __restrict__ sd, const float4* __restrict__ sc,
                                                  float4* __restrict__ col, uint2* __restrict__ spill,
                                                  unsigned long long* work) {
  __shared__ uint32_t s_code[kLdsSlots * kTBlock];
  __shared__ float s_h[kLdsSlots * kTBlock];
  __shared__ float s_lrec[16 * kLdsLights];
  __shared__ int32_t s_lid[kLdsLights];
  __shared__ f4v s_tree[4 * kTreePairs + 1];
  const uint32_t ne = *cnt_ext;
  const uint32_t n = ne + *cnt_sh;
  const Hot H = load_hot(S, (lds_f32h*)s_lrec, (lds_i32*)s_lid, (lds_f4v*)s_tree, (const float4*)s_tree);
  const uint32_t G = gridDim.x * kTBlock;
  const Stack stk{(lds_u32*)(s_code + threadIdx.x), (lds_f32*)(s_h + threadIdx.x),
                  spill + blockIdx.x * kTBlock + threadIdx.x, G, S.stack_cap, S.overflow};
  // work counters (COUNT): per ray in cv/ct/cb, added to its kind at its end
  uint32_t ev = 0, et = 0, eb = 0, sv = 0, st = 0, sb = 0, cv = 0, ct = 0, cb = 0, vmax = 0;
  WaveFeed feed(n);
  const uint32_t p_t0 = S.probe ? probe_now() : 0u;
  uint32_t p_dry = 0u;
  Lane L;
  uint32_t slot = 0;
  bool live = false, is_sh = false, occluded = false;
  BodyLanes bodies;
  float dir_len = 0.0f, early = -__int_as_float(0x7f800000);
  int32_t light = -1;
  const float inf = __int_as_float(0x7f800000);
  for (;;) {
    bool finished = false;
    const uint64_t idle_m = __ballot(!live);
    const uint32_t nidle = (uint32_t)__popcll(idle_m);
    if (nidle != 0 && (nidle >= S.refill_lanes || nidle == 64u) && feed.more()) {
      const uint32_t q0 = feed.take(idle_m);
      const bool got = q0 < n;
      if (!live && got) {
        is_sh = q0 >= ne;
        slot = is_sh ? q0 - ne : q0;
      }
      if (S.probe && p_dry == 0u && !feed.more()) p_dry = probe_now();
      if (!live && got) {
        const float4 o4 = is_sh ? so[slot] : ro[slot];
        const float4 d4 = is_sh ? sd[slot] : rd[slot];
        if (!is_sh) {
          light = -1;
          early = -inf;
          occluded = false;
          live = begin_extend<TRI_ONLY, COUNT, false>(S, H, L, ld3(o4), ld3(d4), cv, ct, cb);
        } else {
          dir_len = o4.w;
          light = (int32_t)__float_as_uint(d4.w);
          live = begin_shadow<TRI_ONLY, COUNT, false>(S, H, L, ld3(o4), ld3(d4), dir_len, light, early, occluded, cv,
                                                      ct, cb);
        }
        finished = !live;
      }
    }
    if (!__any(live || finished) && !feed.more()) {
      if (S.probe) probe_close(S, p_t0, p_dry, feed.taken());
      break;
    }
    if (COUNT) bodies.count(live, is_sh, L);
    if (live) {
      if (!step<true, TRI_ONLY, COUNT>(S, H, L, stk, light, early, occluded, cv, ct, cb)) {
        live = false;
        finished = true;
      }
    }
    if (finished) {
      if (!is_sh) st_hit(t_out + slot, id_out + slot, L.best_id >= 0 ? L.best : inf, L.best_id);
      else if (!shadow_verdict(L, dir_len, light, occluded)) add_contribution(col, sc[slot]);
      if (COUNT) {
        vmax = max(vmax, cv);
        if (is_sh) { sv += cv; st += ct; sb += cb; }
        else { ev += cv; et += ct; eb += cb; }
        cv = ct = cb = 0;
      }
    }
  }
  if (COUNT) {
    // lane iterations of the fused loop go to both kinds: live_a / iterations
    // and live_b / iterations are the shares of lane slots holding each kind
    const unsigned long long wet = wave_sum(et), wst = wave_sum(st), web = wave_sum(eb), wsb = wave_sum(sb);
    work_add(work, 0, ev);
    work_add_wave(work, 1, wet);
    work_add_wave(work, 2, web);
    work_add(work, 3, sv);
    work_add_wave(work, 4, wst);
    work_add_wave(work, 5, wsb);
    // bench.py's bytes of the fused launch: ray record I/O (extension 40 B,
    // shadow 64 B) + node bytes + 64 B per primitive test, from the wave's
    // totals and its ray counts (positions below ne are extension rays)
    const unsigned long long ne_w = feed.taken_below(ne), ns_w = feed.taken() - ne_w;
    work_add_wave(work, 15, 40ull * ne_w + 64ull * ns_w + web + wsb + 64ull * (wet + wst));
    bodies.flush(work, 6, 8);
    // the most node visits of one ray (word 14 holds a maximum, not a sum)
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o));
    if ((threadIdx.x & 63u) == 0u && vmax) atomicMax(work + (blockIdx.x & (kWorkCopies - 1u)) * kWorkWords + 14, (unsigned long long)vmax);
  }
}

// Path-at-a-time tail (the reference's own loop shape, tracer.rs:237-329):
// when an RR-only batch is down to few live paths, the remaining bounces as
// one kernel per bounce cost a full-grid launch and the slowest ray's
// traversal each. k_finish gives each remaining path one lane and runs it to
// its end: closest hit (the exact BVH2 machine), shade_path, the shadow ray
// at once (its contribution is the next colour write of the path, as after
// k_shadow), Russian roulette, repeat. Per path the operations and their
// order are the wavefront's, so col[path] is the same bits. Rays traced are
// counted into counts[kFinishWord], [kFinishWord + 1], the paths into [+ 2]
// and the most bounces one path took into [+ 3]. (Tracing each bounce's
// shadow ray together with the next extension ray, two stacks per lane,
// measured slower: 3 waves/SIMD instead of 4 in the kernel's bulk phase.)
template <bool TRI_ONLY, bool PNEE, bool CR = false>
#ifndef WPT_FINISH_WAVES
#define WPT_FINISH_WAVES 1
#endif
__global__ void __launch_bounds__(kTBlock, TRI_ONLY ? WPT_FINISH_WAVES : 1) k_finish(DevScene S, ShadeParams P, RayStream in,
                                                   const uint32_t* __restrict__ count, float4* __restrict__ col,
                                                   uint2* __restrict__ spill, uint32_t* __restrict__ counters) {
  __shared__ uint32_t s_code[kLdsSlots * kTBlock];
  __shared__ float s_h[kLdsSlots * kTBlock];
  __shared__ float s_lrec[16 * kLdsLights];
  __shared__ int32_t s_lid[kLdsLights];
  __shared__ f4v s_tree[4 * kTreePairs + 1];
  const Hot H = load_hot(S, (lds_f32h*)s_lrec, (lds_i32*)s_lid, (lds_f4v*)s_tree, (const float4*)s_tree);
  const uint32_t n = *count;
  const uint32_t G = gridDim.x * kTBlock;
  const Stack stk{(lds_u32*)(s_code + threadIdx.x), (lds_f32*)(s_h + threadIdx.x),
                  spill + blockIdx.x * kTBlock + threadIdx.x, G, S.stack_cap, S.overflow};
  const OctG O{S.oct_child, S.oct_cum};
  const float inf = __int_as_float(0x7f800000);
  uint32_t nrays = 0, nshadow = 0, npaths = 0, longest = 0, dummy = 0;
  for (uint32_t i = blockIdx.x * kTBlock + threadIdx.x; i < n; i += G) {
    float4 o4 = in.o[i], d4 = in.d[i], th4 = in.thr[i];
    const uint32_t r0 = nrays;
    npaths++;
    for (;;) {
      Lane L;
      bool occ = false;
      nrays++;
      if (begin_extend<TRI_ONLY, false, false>(S, H, L, ld3(o4), ld3(d4), dummy, dummy, dummy))
        while (step<false, TRI_ONLY, false, false>(S, H, L, stk, -1, 0.0f, occ, dummy, dummy, dummy)) {
        }
      ShadeOut R;
      R.alive = R.shadow = false;
      shade_path<TRI_ONLY, PNEE, OctG, CR>(S, O, P, col, L.best_id >= 0 ? L.best : inf, L.best_id, o4, d4, th4, R);
      if (R.shadow) {
        nshadow++;
        const float dir_len = R.so.w, early0 = 0.0f;
        const int32_t light = (int32_t)__float_as_uint(R.sd.w);
        float early = early0;
        bool occluded = false;
        Lane Ls;
        if (begin_shadow<TRI_ONLY, false, false>(S, H, Ls, ld3(R.so), ld3(R.sd), dir_len, light, early, occluded,
                                                 dummy, dummy, dummy))
          while (step<true, TRI_ONLY, false, false>(S, H, Ls, stk, light, early, occluded, dummy, dummy, dummy)) {
          }
        if (!shadow_verdict(Ls, dir_len, light, occluded)) add_contribution(col, R.sc);
      }
      if (!R.alive) break;
      o4 = R.ro;
      d4 = R.rd;
      th4 = R.th;
    }
    longest = max(longest, nrays - r0);
  }
  if (nrays) atomicAdd(counters, nrays);
  if (nshadow) atomicAdd(counters + 1, nshadow);
  if (npaths) {
    atomicAdd(counters + 2, npaths);
    atomicMax(counters + 3, longest);
  }
}

// RenderTarget::write (render_target.rs:55-58): acc += v, count += 1, per
// pixel in increasing sample order (slots j, j+npix, ... are one pixel).
__global__ void __launch_bounds__(kBlock) k_accumulate(const uint32_t* __restrict__ part_pix, uint64_t k0, uint32_t n,
                                                       uint32_t npix, const float4* __restrict__ col,
                                                       float4* __restrict__ acc, uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t lim = n < npix ? n : npix;
  if (i >= lim) return;
  const uint32_t pl = (uint32_t)((k0 + i) % npix);
  const uint32_t pixel = part_pix ? part_pix[pl] : pl;
  float4 a = acc[pixel];
  uint32_t c = cnt[pixel];
  for (uint32_t j = i; j < n; j += npix) {
    const float4 v = col[j];
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    c += 1;
  }
  acc[pixel] = a;
  cnt[pixel] = c;
}

// render_target.rs:62-64: u8 = (clamp(acc/cnt, 0, 1) * 255) as u8
__global__ void k_rgba(const float4* __restrict__ acc, const uint32_t* __restrict__ cnt, uint32_t npix,
                       uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= npix) return;
  const float4 a = acc[i];
  const uint32_t c = cnt[i];
  uchar4 r = make_uchar4(0, 0, 0, 255);
  if (c > 0) {
    const float fc = (float)c;
    r.x = (uint8_t)(fmaxf(fminf(a.x / fc, 1.0f), 0.0f) * 255.0f);
    r.y = (uint8_t)(fmaxf(fminf(a.y / fc, 1.0f), 0.0f) * 255.0f);
    r.z = (uint8_t)(fmaxf(fminf(a.z / fc, 1.0f), 0.0f) * 255.0f);
  }
  reinterpret_cast<uchar4*>(out)[i] = r;
}

__global__ void k_pack_partition(const uint32_t* __restrict__ part_pix, uint32_t n, const float4* __restrict__ acc,
                                 const uint32_t* __restrict__ cnt, float4* __restrict__ out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = part_pix ? part_pix[i] : i;
  float4 a = acc[p];
  a.w = __uint_as_float(cnt[p]);  // count as u32 bits (exact past 2^24), as k_pack_exchange
  out[i] = a;
}

inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }

}  // namespace

// ===========================================================================
// Renderer
// ===========================================================================
// Sample-stock rings outlive their renderer: a session torn down (or a ring
// resized) hands its two ring blocks (42 GB at 1080p) to the next ring on the
// device instead of hipFree. Allocating and freeing blocks that size over and
// over stalled a process for 1-5 s per allocation after a handful of cycles
// (profiles/r06/alloc_cycle.jsonl, mem_cycle*.jsonl). A ring never reads a
// slot before writing it (k_stock_plan reads ids below the frontier only), so
// a reused block's old contents are harmless. At most kRingCacheBlocks are
// kept per process; never freed at exit (the HIP runtime may be gone by then).
namespace {
struct RingBlock {
  int dev;
  void* p;
  size_t bytes;
};
constexpr size_t kRingCacheBlocks = 4;
std::mutex& ring_mu() {
  static std::mutex* m = new std::mutex;
  return *m;
}
std::vector<RingBlock>& ring_cache() {
  static std::vector<RingBlock>* v = new std::vector<RingBlock>;
  return *v;
}
}  // namespace

// A block of at least `bytes` (and at most twice that) on `dev`: a cached one,
// else hipMalloc; when that fails, the device's cached blocks are freed and
// the allocation tried once more.
static hipError_t ring_take(int dev, size_t bytes, void** p, size_t* got) {
  {
    std::lock_guard<std::mutex> g(ring_mu());
    auto& c = ring_cache();
    size_t best = c.size();
    for (size_t i = 0; i < c.size(); i++)
      if (c[i].dev == dev && c[i].bytes >= bytes && c[i].bytes / 2 <= bytes && (best == c.size() || c[i].bytes < c[best].bytes))
        best = i;
    if (best < c.size()) {
      *p = c[best].p;
      *got = c[best].bytes;
      c.erase(c.begin() + best);
      return hipSuccess;
    }
  }
  *got = bytes;
  if (hipMalloc(p, bytes) == hipSuccess) return hipSuccess;
  (void)hipGetLastError();
  {
    std::lock_guard<std::mutex> g(ring_mu());
    auto& c = ring_cache();
    for (size_t i = 0; i < c.size();)
      if (c[i].dev == dev) {
        (void)hipFree(c[i].p);
        c.erase(c.begin() + i);
      } else {
        i++;
      }
  }
  return hipMalloc(p, bytes);
}

// Back to the cache (the caller's work on the block has finished); the oldest
// block is freed past kRingCacheBlocks.
static void ring_give(int dev, void* p, size_t bytes) {
  if (!p) return;
  std::lock_guard<std::mutex> g(ring_mu());
  auto& c = ring_cache();
  c.push_back({dev, p, bytes});
  while (c.size() > kRingCacheBlocks) {
    (void)hipFree(c.front().p);
    c.erase(c.begin());
  }
}

Renderer::Renderer() {}

Renderer::~Renderer() {
  {
    std::string e;
    (void)drain_async(e);
  }
  {
    if (d_stock_ || d_stock_id_) {
      // the rings go back to the cache once nothing reads them (hipFree
      // would have waited for the device the same way)
      if (stream_) (void)hipStreamSynchronize(stream_);
      for (PathSet& L : lanes_) {
        if (L.stream) (void)hipStreamSynchronize(L.stream);
        if (L.lo) (void)hipStreamSynchronize(L.lo);
      }
      ring_give(device_, d_stock_, stock_bytes_[0]);
      ring_give(device_, d_stock_id_, stock_bytes_[1]);
    }
    void* sb[] = {d_front_, d_def_, d_bmax_, d_rays_};
    for (void* q : sb)
      if (q) (void)hipFree(q);
    for (Refill& f : refills_) {
      if (f.off) (void)hipFree(f.off);
      if (f.base) (void)hipFree(f.base);
    }
  }
  if (h_refill_cnt_) (void)hipHostFree(h_refill_cnt_);
  for (auto& re : refill_ev_)
    for (hipEvent_t e : re)
      if (e) (void)hipEventDestroy(e);
  free_rounds();
  free_photons();
  free_scene();
  free_paths();
  if (d_part_pix_) (void)hipFree(d_part_pix_);
  for (uint32_t* p : d_half_pix_)
    if (p) (void)hipFree(p);
  if (d_frame_pix_) (void)hipFree(d_frame_pix_);
  if (d_xidx_) (void)hipFree(d_xidx_);
  if (d_acc_) (void)hipFree(d_acc_);
  if (d_cnt_) (void)hipFree(d_cnt_);
  if (d_rgba_) (void)hipFree(d_rgba_);
  if (d_samp_) (void)hipFree(d_samp_);
  if (d_work_) (void)hipFree(d_work_);
  if (d_probe_) (void)hipFree(d_probe_);
  if (d_fallback_) (void)hipFree(d_fallback_);
  for (PathSet& L : lanes_) {
    if (L.counts) (void)hipFree(L.counts);
    if (L.h_counts) (void)hipHostFree(L.h_counts);
    if (L.spill) (void)hipFree(L.spill);
    if (L.done) (void)hipEventDestroy(L.done);
    if (L.stream && L.stream != stream_) (void)hipStreamDestroy(L.stream);
    if (L.lo) (void)hipStreamDestroy(L.lo);
  }
  for (int k = 0; k < 2; k++) {
    if (d_seam_pix_[k]) (void)hipFree(d_seam_pix_[k]);
    if (d_rest_pix_[k]) (void)hipFree(d_rest_pix_[k]);
  }
  if (h_fill_cnt_) (void)hipHostFree(h_fill_cnt_);
  for (auto& fe : fill_ev_)
    for (hipEvent_t e : fe)
      if (e) (void)hipEventDestroy(e);
  if (ev_main_) (void)hipEventDestroy(ev_main_);
  if (ev_sync_) (void)hipEventDestroy(ev_sync_);
  if (ev_ref_) (void)hipEventDestroy(ev_ref_);
  if (h_word_) (void)hipHostFree(h_word_);
  for (auto& e : ev_pool_)
    if (e) (void)hipEventDestroy(e);
  if (stream_) (void)hipStreamDestroy(stream_);
}

bool Renderer::set_device(int dev, std::string& err) {
  if (device_ == dev && stream_) return true;
  if (stream_) {
    err = "device already selected";
    return false;
  }
  HIP_OK(hipSetDevice(dev));
  device_ = dev;
  HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  HIP_OK(hipDeviceGetAttribute(&ncu_, hipDeviceAttributeMultiprocessorCount, dev));
  HIP_OK(hipEventCreateWithFlags(&ev_main_, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&ev_sync_, hipEventDisableTiming));
  HIP_OK(hipEventCreate(&ev_ref_));
  HIP_OK(hipHostMalloc(&h_word_, sizeof(uint32_t) * 4));
  // every lane's stream is made here (a stream takes a hardware queue only
  // when it first submits work, so unused lanes cost nothing): the lane
  // count can then change per session, up to kMaxLanes
  lanes_made_ = kMaxLanes;
  for (int i = 0; i < kMaxLanes; i++) {
    PathSet& L = lanes_[i];
    if (i == 0) L.stream = stream_;
    else HIP_OK(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&L.done, hipEventDisableTiming));
    HIP_OK(hipMalloc(&L.counts, sizeof(uint32_t) * kCountWords));
    HIP_OK(hipHostMalloc(&L.h_counts, sizeof(uint32_t) * kCountWords));
  }
  bind_lane(0);
  HIP_OK(hipMalloc(&d_work_, sizeof(unsigned long long) * kWorkWords * kWorkCopies));
  HIP_OK(hipMalloc(&d_fallback_, sizeof(uint32_t) * 4));  // [0..1] fallbacks, [2] stack overflow
  HIP_OK(hipMemset(d_fallback_, 0, sizeof(uint32_t) * 4));
  HIP_OK(hipMemset(d_work_, 0, sizeof(unsigned long long) * kWorkWords * kWorkCopies));
  return true;
}

void Renderer::free_scene() {
  for (void* p : scene_bufs_) (void)hipFree(p);
  scene_bufs_.clear();
  scene_ok_ = false;
}

void Renderer::free_lane_paths(PathSet& L) {
  void* bufs[] = {L.pixel, L.col, L.ro[0], L.rd[0], L.thr[0], L.ro[1], L.rd[1], L.thr[1], L.t, L.id, L.so, L.sd, L.sc};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  L.pixel = nullptr;
  L.col = nullptr;
  for (int k = 0; k < 2; k++) L.ro[k] = L.rd[k] = L.thr[k] = nullptr;
  L.t = nullptr;
  L.id = nullptr;
  L.so = L.sd = L.sc = nullptr;
  L.cap = 0;
}

void Renderer::free_paths() {
  for (PathSet& L : lanes_) free_lane_paths(L);
  bind_lane(bound_);
}

void Renderer::bind_lane(int i) {
  const PathSet& L = lanes_[i];
  bound_ = i;
  async_launch_ = false;
  ks_ = L.stream;
  cap_ = L.cap;
  p_pixel_ = L.pixel;
  p_col_ = L.col;
  for (int k = 0; k < 2; k++) {
    p_ro_[k] = L.ro[k];
    p_rd_[k] = L.rd[k];
    p_thr_[k] = L.thr[k];
  }
  p_t_ = L.t; p_id_ = L.id;
  s_o_ = L.so; s_d_ = L.sd; s_c_ = L.sc;
  d_counts_ = L.counts; h_counts_ = L.h_counts;
  d_spill_ = L.spill; spill_cap_ = L.spill_cap;
}

bool Renderer::upload_scene(const HostScene& sc, std::string& err) {
  if (!stream_) { err = "no device"; return false; }
  if (!drain_async(err)) return false;
  stock_drop();
  HIP_OK(hipStreamSynchronize(stream_));
  free_photons();
  free_scene();
  if (sc.num_inf > (uint32_t)kMaxInf && sc.use_bvh) { err = "too many infinite shapes"; return false; }
  if (sc.use_bvh && sc.depth >= (uint32_t)kMaxBvhDepth) { err = "BVH deeper than supported"; return false; }
  const size_t ns = sc.shapes.size();
  const size_t nf = ns - sc.num_inf;
  auto rec = [](const Shape& s, float4* out) {
    memset(out, 0, 4 * sizeof(float4));
    const float* g = s.g;
    if (s.kind == kTri) {
      V3 v0 = mk(g[0], g[1], g[2]), v1 = mk(g[3], g[4], g[5]), v2 = mk(g[6], g[7], g[8]);
      V3 n = cross(sub(v1, v0), sub(v2, v0));  // triangle.rs:164
      V3 nn = normalize(n);                     // triangle.rs:183
      float od = dot(n, v0);                    // triangle.rs:172
      out[0] = make_float4(v0.x, v0.y, v0.z, n.x);
      out[1] = make_float4(v1.x, v1.y, v1.z, n.y);
      out[2] = make_float4(v2.x, v2.y, v2.z, n.z);
      out[3] = make_float4(nn.x, nn.y, nn.z, od);
    } else if (s.kind == kPlane) {
      V3 loc = mk(g[0], g[1], g[2]), n = mk(g[3], g[4], g[5]);
      out[0] = make_float4(n.x, n.y, n.z, dot(n, loc));  // plane.rs:80-99
      out[1] = make_float4(loc.x, loc.y, loc.z, 0.0f);
    } else if (s.kind == kSphere) {
      out[0] = make_float4(g[0], g[1], g[2], g[3]);
    } else if (s.kind == kTorus) {
      out[0] = make_float4(g[0], g[1], g[2], g[3]);  // location, big_r
      out[1] = make_float4(g[4], 0.0f, 0.0f, 0.0f);  // small_r
    } else {
      out[0] = make_float4(g[0], g[1], g[2], g[3]);
      out[1] = make_float4(g[4], g[5], 0.0f, 0.0f);
    }
  };
  std::vector<float4> prims(4 * std::max<size_t>(nf, 1)), all(4 * std::max<size_t>(ns, 1));
  std::vector<uint32_t> kinds(std::max<size_t>(nf, 1)), all_kinds(std::max<size_t>(ns, 1));
  std::vector<float4> mats(std::max<size_t>(ns, 1));
  for (size_t i = 0; i < ns; i++) {
    const Shape& s = sc.shapes[i];
    rec(s, &all[4 * i]);
    all_kinds[i] = s.kind;
    if (i >= sc.num_inf) {
      rec(s, &prims[4 * (i - sc.num_inf)]);
      kinds[i - sc.num_inf] = s.kind;
    }
    mats[i] = make_float4(s.m[0], s.m[1], s.m[2], s.emissive ? 1.0f : 0.0f);
  }
  std::vector<float4> lights(5 * std::max<size_t>(sc.lights.size(), 1));
  for (size_t l = 0; l < sc.lights.size(); l++) {
    const Shape& s = sc.shapes[sc.lights[l]];
    if (s.kind != kTri) { err = "only triangles can be area lights (Tracable::pick_random)"; return false; }
    const float* g = s.g;
    V3 v0 = mk(g[0], g[1], g[2]), v1 = mk(g[3], g[4], g[5]), v2 = mk(g[6], g[7], g[8]);
    // Heron (triangle.rs:70-78)
    float a = len(sub(v0, v1)), b = len(sub(v1, v2)), c = len(sub(v2, v0));
    float sp = (a + b + c) * 0.5f;
    float area = sqrtf(sp * (sp - a) * (sp - b) * (sp - c));
    V3 nn = normalize(cross(sub(v1, v0), sub(v2, v0)));  // triangle.rs:104
    lights[5 * l + 0] = make_float4(v0.x, v0.y, v0.z, area);
    lights[5 * l + 1] = make_float4(v1.x, v1.y, v1.z, u2f(sc.lights[l]));
    lights[5 * l + 2] = make_float4(v2.x, v2.y, v2.z, 0.0f);
    lights[5 * l + 3] = make_float4(nn.x, nn.y, nn.z, 0.0f);
    lights[5 * l + 4] = make_float4(s.m[0], s.m[1], s.m[2], 0.0f);
  }
  const std::vector<Node2>& tree_nodes = sc.nodes;  // the reference BVH2
  std::vector<float4> nodes(2 * tree_nodes.size());
  for (size_t i = 0; i < tree_nodes.size(); i++) {
    const Node2& n = tree_nodes[i];
    nodes[2 * i] = make_float4(n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0]);
    nodes[2 * i + 1] = make_float4(n.bmax[1], n.bmax[2], u2f(n.left_first), u2f(n.count));
  }
  auto up = [&](const void* src, size_t bytes, void** dst) -> bool {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) { err = "hipMalloc failed (scene)"; return false; }
    scene_bufs_.push_back(p);
    if (hipMemcpy(p, src, bytes, hipMemcpyHostToDevice) != hipSuccess) { err = "hipMemcpy failed (scene)"; return false; }
    *dst = p;
    return true;
  };
  DevScene ds{};
  void* p;
  if (!up(nodes.data(), nodes.size() * sizeof(float4), &p)) return false;
  ds.nodes = (const float4*)p;
  {
    // treelet (kTreePairs): pairs taken breadth first from the root's; a pair holding a
    // leaf that the stack cannot encode by itself (encode_child) stays
    // global, so a treelet index is never pushed as a node index
    std::vector<float4> tree;
    uint32_t root_lf = 0;
    const uint32_t root = 0u;
    const bool on = kTreePairs > 0 && sc.use_bvh && !sc.nodes.empty() && tree_nodes[root].count == 0 &&
                    tree_nodes.size() < (size_t)kTreeFlag && treelet_;
    if (on) {
      auto encodable = [&](uint32_t n) {
        return tree_nodes[n].count == 0 || (tree_nodes[n].count < 128u && tree_nodes[n].left_first < (1u << 24));
      };
      std::vector<uint32_t> order;                 // global left_first of each treelet pair
      std::unordered_map<uint32_t, uint32_t> tix;  // global left_first -> treelet index
      std::deque<uint32_t> q{tree_nodes[root].left_first};
      while (!q.empty() && order.size() < kTreePairs) {
        const uint32_t lf = q.front();
        q.pop_front();
        if (!encodable(lf) || !encodable(lf + 1)) continue;
        tix[lf] = (uint32_t)order.size();
        order.push_back(lf);
        for (uint32_t c = lf; c < lf + 2; c++)
          if (tree_nodes[c].count == 0) q.push_back(tree_nodes[c].left_first);
      }
      for (uint32_t t = 0; t < order.size(); t++) {
        for (uint32_t k = 0; k < 4; k++) tree.push_back(nodes[2 * (size_t)order[t] + k]);
        for (uint32_t c = 0; c < 2; c++) {
          const Node2& n = tree_nodes[order[t] + c];
          auto it = tix.find(n.left_first);
          if (n.count == 0 && it != tix.end()) tree[4 * t + 2 * c + 1].z = u2f(kTreeFlag | it->second);
        }
      }
      if (!order.empty() && order[0] == tree_nodes[root].left_first) root_lf = kTreeFlag;
      else tree.clear();
    }
    ds.tree_pairs = (uint32_t)(tree.size() / 4);
    ds.tree_root_lf = root_lf;
    if (tree.empty()) tree.push_back(make_float4(0.f, 0.f, 0.f, 0.f));
    if (!up(tree.data(), tree.size() * sizeof(float4), &p)) return false;
    ds.tree = (const float4*)p;
  }
  if (!up(prims.data(), prims.size() * sizeof(float4), &p)) return false;
  ds.prims = (const float4*)p;
  if (!up(kinds.data(), kinds.size() * sizeof(uint32_t), &p)) return false;
  ds.kinds = (const uint32_t*)p;
  if (!up(all.data(), all.size() * sizeof(float4), &p)) return false;
  ds.all = (const float4*)p;
  if (!up(all_kinds.data(), all_kinds.size() * sizeof(uint32_t), &p)) return false;
  ds.all_kinds = (const uint32_t*)p;
  if (!up(mats.data(), mats.size() * sizeof(float4), &p)) return false;
  ds.mats = (const float4*)p;
  if (!up(lights.data(), lights.size() * sizeof(float4), &p)) return false;
  ds.lights = (const float4*)p;
  // fast-path BVH4 (128 B nodes) and its leaf table
  {
    const size_t n4 = std::max<size_t>(sc.nodes4.size(), 1);
    std::vector<Node4> n4v(n4);
    if (!sc.nodes4.empty()) memcpy(n4v.data(), sc.nodes4.data(), sizeof(Node4) * sc.nodes4.size());
    if (!up(n4v.data(), sizeof(Node4) * n4, &p)) return false;
    ds.nodes4 = (const float4*)p;
    std::vector<uint32_t> lt(std::max<size_t>(sc.leaf_table.size(), 2), 0u);
    std::copy(sc.leaf_table.begin(), sc.leaf_table.end(), lt.begin());
    if (!up(lt.data(), sizeof(uint32_t) * lt.size(), &p)) return false;
    ds.leaf_table = (const uint32_t*)p;
    // WPT_OPT_TRAVERSAL(_SH): 1 the BVH4 fast path (the scene must carry the
    // BVH4: HostScene::want_bvh4), 0 the exact BVH2 stack machine alone.
    // 3 (auto, the default): the BVH4 on BVH scenes with other finite shapes
    // than triangles (the museum's tori: 2 268 vs 1 882 Mray/s, round 5), the
    // BVH2 on triangle scenes (C3 8 136 vs 6 887, C5 2 313 vs 1 711) and the
    // BVH2 kernels' linear scan on scenes without a BVH (C2)
    auto mode = [&](int want) {
      const bool b4 = want == 1 || (want == 3 && !sc.tri_only && sc.use_bvh);
      return (b4 && !sc.nodes4.empty()) ? 1 : 0;
    };
    trav_ext_ = mode(traversal_);
    trav_sh_ = mode(traversal_sh_);
  }
  ds.num_inf = sc.num_inf;
  ds.num_finite = (uint32_t)nf;
  ds.num_shapes = (uint32_t)ns;
  ds.num_lights = (uint32_t)sc.lights.size();
  ds.use_bvh = sc.use_bvh ? 1u : 0u;
  ds.tri_only = sc.tri_only ? 1u : 0u;
  ds.refill_lanes = refill_;
  ds.refill_lanes_sh = refill_sh_;
  for (int k = 0; k < 3; k++) ds.bg[k] = sc.background[k];
  for (uint32_t i = 0; i < sc.num_inf && i < (uint32_t)kMaxInf; i++) ds.planes[i] = all[4 * i];
  ds_ = ds;
  depth_ = sc.depth;
  ds_.stack_cap = (int)std::max<uint32_t>(sc.depth + 2, 3 * sc.depth4 + 4);
  ds_.overflow = d_fallback_ + 2;
  if (!size_grids(err)) return false;
  scene_ok_ = true;
  return true;
}

// wpt_set_option (include/wpt.h WPT_OPT_*). Range checks here; the caller
// re-uploads the scene (traversal, treelet) or re-partitions (pixel tile).
bool Renderer::set_option(int opt, int64_t v, std::string& err) {
  auto range = [&](int64_t lo, int64_t hi) {
    if (v < lo || v > hi) {
      err = "option value out of range";
      return false;
    }
    return true;
  };
  switch (opt) {
    case 1:
    case 2:
      // 0 exact BVH2, 1 BVH4 fast path, 3 auto (per scene); 2 was the fast
      // tree, removed in round 5 (slower on every config)
      if (!range(0, 3) || v == 2) { err = "traversal: 0 (bvh2), 1 (bvh4) or 3 (auto)"; return false; }
      (opt == 1 ? traversal_ : traversal_sh_) = (int)v;
      return true;
    case 3: if (!range(0, 1)) return false; fused_ = v != 0; return true;
    case 4: if (!range(0, (int64_t)1 << 40)) return false; fused_below_ = (uint64_t)v; return true;
    case 5: if (!range(1, kMaxLanes)) return false; small_lanes_ = (int)v; return true;
    case 6: if (!range(0, 4096)) return false; pixel_tile_ = (uint32_t)v; return true;
    case 7:
      if (!range(1, 100)) return false;
      grid_pct_ = (int)v;
      return !stream_ || size_grids(err);
    case 8: if (!range(1, 64)) return false; refill_ = (uint32_t)v; ds_.refill_lanes = refill_; return true;
    case 9: if (!range(1, 64)) return false; refill_sh_ = (uint32_t)v; ds_.refill_lanes_sh = refill_sh_; return true;
    case 10: if (!range(0, 1)) return false; treelet_ = v != 0; return true;
    case 12:
      if (!set_lanes((int)v)) { err = "lanes out of range"; return false; }
      return true;
    case 13: if (!range(0, (int64_t)1 << 32)) return false; finish_below_ = (uint64_t)v; return true;
    case 14:
      if (!range(1, 100)) return false;
      trace_grid_pct_ = (int)v;
      return !stream_ || size_grids(err);
    case 20: if (!range(1, 64)) return false; finish_every_ = (int)v; return true;
    case 23:
      // ring slots per pixel: 0 (off) or a power of two 64 .. 4096
      if (v != 0 && (v < 64 || v > 4096 || (v & (v - 1)) != 0)) { err = "stock: 0 or a power of two 64..4096"; return false; }
      if (!drain_async(err)) return false;
      stock_drop();
      stock_slots_ = (uint32_t)v;
      return true;
    case 25: if (!range(0, 1)) return false; fill_on_ = v != 0; return true;
    case 30: if (!range(0, 64)) return false; stock_ahead_ = (uint32_t)v; return true;
    case 32: if (!range(1, 1024)) return false; stock_every_ = (uint32_t)v; return true;
    case 33: if (!range(0, 64)) return false; stock_extra_ = (uint32_t)v; return true;
    case 31: if (!range(0, 1)) return false; async_oneshot_ = v != 0; return true;
    case 34: if (!range(0, 1)) return false; log_ = (int)v; return true;
    case 35: if (!range(0, 1)) return false; stock_prefill_ = v != 0; return true;
    case 36: if (!range(0, (int64_t)1 << 40)) return false; async_fused_below_ = (uint64_t)v; return true;
    case 26:
      if (!range(0, 1)) return false;
      if (!drain_async(err)) return false;  // a batch keeps its stream
      async_prio_ = (int)v;
      return true;
    case 27: if (!range(0, 100)) return false; async_grid_pct_ = (int)v; return true;
    case 28:
    case 29: err = "read-only option"; return false;
    case 24:
      if (!range(1, kMaxLanes - kAsyncLane0 - 1)) return false;  // the fill lane follows them
      if (!drain_async(err)) return false;
      stock_lanes_ = (int)v;
      refill_lane_ = 0;
      return true;
    case 22:
      if (!range(0, 1 << 20)) return false;
      probe_cap_ = (uint32_t)v;
      probe_used_ = 0;
      probe_meta_.clear();
      if (d_probe_) { (void)hipFree(d_probe_); d_probe_ = nullptr; }
      return true;
    default: err = "unknown option"; return false;
  }
}

bool Renderer::get_option(int opt, int64_t& v) const {
  switch (opt) {
    case 1: v = traversal_; return true;
    case 2: v = traversal_sh_; return true;
    case 3: v = fused_ ? 1 : 0; return true;
    case 4: v = (int64_t)fused_below_; return true;
    case 5: v = small_lanes_; return true;
    case 6: v = pixel_tile_; return true;
    case 7: v = grid_pct_; return true;
    case 8: v = refill_; return true;
    case 9: v = refill_sh_; return true;
    case 10: v = treelet_ ? 1 : 0; return true;
    case 12: v = nlanes_; return true;
    case 13: v = (int64_t)finish_below_; return true;
    case 14: v = trace_grid_pct_; return true;
    case 20: v = finish_every_; return true;
    case 22: v = probe_cap_; return true;
    case 23: v = stock_slots_; return true;
    case 25: v = fill_on_ ? 1 : 0; return true;
    case 30: v = stock_ahead_; return true;
    case 32: v = stock_every_; return true;
    case 33: v = stock_extra_; return true;
    case 31: v = async_oneshot_ ? 1 : 0; return true;
    case 34: v = log_; return true;
    case 35: v = stock_prefill_ ? 1 : 0; return true;
    case 36: v = (int64_t)async_fused_below_; return true;
    case 26: v = async_prio_; return true;
    case 27: v = async_grid_pct_; return true;
    // read-only: what the uploaded scene's traversal kernels run:
    // 0 exact BVH2, 1 BVH4 fast path, 2 linear scan (BVH disabled), -1 no
    // scene; and whether its finite shapes are all triangles
    case 28: v = !scene_ok_ ? -1 : !ds_.use_bvh ? 2 : trav_ext_; return true;
    case 29: v = !scene_ok_ ? -1 : ds_.tri_only ? 1 : 0; return true;
    case 24: v = stock_lanes_; return true;
    default: return false;
  }
}

bool Renderer::set_viewport(uint32_t w, uint32_t h, std::string& err) {
  if (!stream_) { err = "no device"; return false; }
  if (w == 0 || h == 0) { err = "empty viewport"; return false; }
  if (!drain_async(err)) return false;  // async batches read the buffers freed below
  stock_drop();
  HIP_OK(hipStreamSynchronize(stream_));
  w_ = w;
  h_ = h;
  free_rounds();
  if (d_acc_) (void)hipFree(d_acc_);
  if (d_cnt_) (void)hipFree(d_cnt_);
  if (d_rgba_) (void)hipFree(d_rgba_);
  if (d_samp_) (void)hipFree(d_samp_);
  d_acc_ = nullptr; d_cnt_ = nullptr; d_rgba_ = nullptr; d_samp_ = nullptr;
  HIP_OK(hipMalloc(&d_acc_, sizeof(float4) * (size_t)w * h));
  HIP_OK(hipMalloc(&d_cnt_, sizeof(uint32_t) * (size_t)w * h));
  HIP_OK(hipMalloc(&d_rgba_, 4 * (size_t)w * h));
  HIP_OK(hipMalloc(&d_samp_, 4 * (size_t)w * h));
  return set_partition(rank_, nranks_, tile_, err);
}

void Renderer::set_camera(const float cam[5]) { memcpy(cam_, cam, sizeof cam_); }

bool Renderer::set_partition(uint32_t rank, uint32_t nranks, uint32_t tile, std::string& err) {
  if (nranks == 0 || rank >= nranks || tile == 0) { err = "bad partition"; return false; }
  if (!drain_async(err)) return false;  // async batches read the pixel lists freed below
  stock_drop();
  HIP_OK(hipStreamSynchronize(stream_));  // and the main stream's (its frontier copy, a round's kernels)
  rank_ = rank; nranks_ = nranks; tile_ = tile;
  part_pix_.clear();
  if (d_part_pix_) { (void)hipFree(d_part_pix_); d_part_pix_ = nullptr; }
  for (uint32_t*& p : d_half_pix_)
    if (p) { (void)hipFree(p); p = nullptr; }
  for (int k = 0; k < 2; k++) {
    if (d_seam_pix_[k]) { (void)hipFree(d_seam_pix_[k]); d_seam_pix_[k] = nullptr; }
    if (d_rest_pix_[k]) { (void)hipFree(d_rest_pix_[k]); d_rest_pix_[k] = nullptr; }
    seam_npix_[k] = rest_npix_[k] = 0;
  }
  if (d_frame_pix_) { (void)hipFree(d_frame_pix_); d_frame_pix_ = nullptr; }
  half_npix_[0] = half_npix_[1] = 0;
  if (d_xidx_) { (void)hipFree(d_xidx_); d_xidx_ = nullptr; }
  maxpart_ = 0;
  if (w_ && h_ && nranks > 1) {
    tile_partition(w_, h_, rank, nranks, tile, part_pix_);
    if (!part_pix_.empty()) {
      HIP_OK(hipMalloc(&d_part_pix_, sizeof(uint32_t) * part_pix_.size()));
      HIP_OK(hipMemcpy(d_part_pix_, part_pix_.data(), sizeof(uint32_t) * part_pix_.size(), hipMemcpyHostToDevice));
    }
    // frame exchange index: entry j of rank r's gathered slot -> pixel
    std::vector<std::vector<uint32_t>> parts(nranks);
    for (uint32_t r = 0; r < nranks; r++) {
      tile_partition(w_, h_, r, nranks, tile, parts[r]);
      maxpart_ = std::max<uint64_t>(maxpart_, parts[r].size());
    }
    std::vector<uint32_t> xidx((size_t)nranks * maxpart_, 0xFFFFFFFFu);
    for (uint32_t r = 0; r < nranks; r++)
      std::copy(parts[r].begin(), parts[r].end(), xidx.begin() + (size_t)r * maxpart_);
    if (!xidx.empty()) {
      HIP_OK(hipMalloc(&d_xidx_, sizeof(uint32_t) * xidx.size()));
      HIP_OK(hipMemcpy(d_xidx_, xidx.data(), sizeof(uint32_t) * xidx.size(), hipMemcpyHostToDevice));
    }
  } else if (w_ && h_) {
    part_pix_.resize((size_t)w_ * h_);
    for (size_t i = 0; i < part_pix_.size(); i++) part_pix_[i] = (uint32_t)i;  // identity: kernels use nullptr
    // Whole sample rounds run as one batch over a pixel list in tile order
    // (tile_order): the frame's pixels (compute) and each screen half's
    // (compute_half, a non-adaptive half). Either covers the same (pixel,
    // sample) pairs as the raster sequence, so the frame is the same bits;
    // partial rounds keep raster order.
    const uint32_t tile_px = pixel_tile_;
    std::vector<uint32_t> px;
    tile_order(w_, h_, 0, w_, tile_px, px);
    HIP_OK(hipMalloc(&d_frame_pix_, sizeof(uint32_t) * px.size()));
    HIP_OK(hipMemcpy(d_frame_pix_, px.data(), sizeof(uint32_t) * px.size(), hipMemcpyHostToDevice));
    const uint32_t half = w_ / 2;
    for (int hh = 0; hh < 2; hh++) {
      tile_order(w_, h_, hh ? half : 0u, hh ? w_ : half, tile_px, px);
      half_npix_[hh] = (uint32_t)px.size();
      if (!px.empty()) {
        HIP_OK(hipMalloc(&d_half_pix_[hh], sizeof(uint32_t) * px.size()));
        HIP_OK(hipMemcpy(d_half_pix_[hh], px.data(), sizeof(uint32_t) * px.size(), hipMemcpyHostToDevice));
      }
      // the half's seam (the columns within the 5x5 error filter's radius 2
      // of the other half, render_target.rs:112-128) and the rest, each in
      // the same tile order (compute_halves)
      std::vector<uint32_t> seam, rest;
      for (uint32_t p : px) {
        const uint32_t x = p % w_;
        (hh ? x < half + 2 : x + 2 >= half) ? seam.push_back(p) : rest.push_back(p);
      }
      seam_npix_[hh] = (uint32_t)seam.size();
      rest_npix_[hh] = (uint32_t)rest.size();
      if (!seam.empty()) {
        HIP_OK(hipMalloc(&d_seam_pix_[hh], sizeof(uint32_t) * seam.size()));
        HIP_OK(hipMemcpy(d_seam_pix_[hh], seam.data(), sizeof(uint32_t) * seam.size(), hipMemcpyHostToDevice));
      }
      if (!rest.empty()) {
        HIP_OK(hipMalloc(&d_rest_pix_[hh], sizeof(uint32_t) * rest.size()));
        HIP_OK(hipMemcpy(d_rest_pix_[hh], rest.data(), sizeof(uint32_t) * rest.size(), hipMemcpyHostToDevice));
      }
    }
  }
  return reset(err);
}

bool Renderer::reset(std::string& err) {
  // refills in flight belong to the image being dropped
  if (!drain_async(err)) return false;
  next_path_ = 0;
  for (HalfRounds& r : rounds_) r.pos = r.total = r.idx = 0;
  if (!stream_ || !d_acc_) return true;
  k_samp_reset<<<blocks_for((uint64_t)w_ * h_), kBlock, 0, stream_>>>(d_samp_, w_, h_, w_ / 2, adaptive_[0] ? 1u : 0u,
                                                                      adaptive_[1] ? 1u : 0u);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemsetAsync(d_acc_, 0, sizeof(float4) * (size_t)w_ * h_, stream_));
  HIP_OK(hipMemsetAsync(d_cnt_, 0, sizeof(uint32_t) * (size_t)w_ * h_, stream_));
  stock_drop();  // the ring empty: frontier = the (zero) counts
  return true;
}

bool Renderer::ensure_lane(int i, uint64_t n, std::string& err) {
  PathSet& L = lanes_[i];
  if (!L.spill) {
    // the lane's traversal-stack spill, for the largest persistent grid
    const size_t need = spill_slots() * (size_t)std::max<uint32_t>(max_grid(), 1) * kTBlock;
    HIP_OK(hipMalloc(&L.spill, need * sizeof(uint2)));
    L.spill_cap = need;
    if (i == bound_) bind_lane(i);
  }
  if (async_prio_ && i >= kAsyncLane0 && !L.lo) {
    // async batches' low-priority stream (WPT_OPT_ASYNC_PRIO)
    int least = 0, greatest = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_OK(hipStreamCreateWithPriority(&L.lo, hipStreamNonBlocking, least));
  }
  if (n <= L.cap) return true;
  HIP_OK(hipStreamSynchronize(L.stream));
  if (L.lo) HIP_OK(hipStreamSynchronize(L.lo));
  HIP_OK(hipStreamSynchronize(stream_));
  free_lane_paths(L);
  HIP_OK(hipMalloc(&L.pixel, 4 * n));
  HIP_OK(hipMalloc(&L.col, 16 * n));
  for (int k = 0; k < 2; k++) {
    HIP_OK(hipMalloc(&L.ro[k], 16 * n));
    HIP_OK(hipMalloc(&L.rd[k], 16 * n));
    HIP_OK(hipMalloc(&L.thr[k], 16 * n));
  }
  HIP_OK(hipMalloc(&L.t, 4 * n));
  HIP_OK(hipMalloc(&L.id, 4 * n));
  HIP_OK(hipMalloc(&L.so, 16 * n));
  HIP_OK(hipMalloc(&L.sd, 16 * n));
  HIP_OK(hipMalloc(&L.sc, 16 * n));
  L.cap = n;
  bind_lane(bound_);
  return true;
}

bool Renderer::ensure_paths(uint64_t n, std::string& err) { return ensure_lane(0, n, err); }

#define LAUNCH_TIMED(slot, accum, counter, ...)                          \
  do {                                                                   \
    hipEvent_t a_ = nullptr, b_ = nullptr;                               \
    if (time_launches_) {                                                \
      if (!next_event(&a_, err) || !next_event(&b_, err)) return false;  \
      HIP_OK(hipEventRecord(a_, ks_));                                   \
    }                                                                    \
    __VA_ARGS__;                                                         \
    HIP_OK(hipGetLastError());                                           \
    if (time_launches_) {                                                \
      HIP_OK(hipEventRecord(b_, ks_));                                   \
      pending_.push_back(PendingTiming{a_, b_, slot});                   \
    }                                                                    \
  } while (0)

bool Renderer::next_event(hipEvent_t* e, std::string& err) {
  if (ev_used_ == ev_pool_.size()) {
    hipEvent_t x;
    HIP_OK(hipEventCreate(&x));
    ev_pool_.push_back(x);
  }
  *e = ev_pool_[ev_used_++];
  return true;
}

bool Renderer::resolve_timings(std::string& err) {
  // per-launch durations (summed per kernel) and, per kernel, the union of
  // the launch intervals of all lanes measured from the batch's ev_ref_
  std::vector<std::pair<float, float>> iv[kTimedKernels];
  for (const PendingTiming& p : pending_) {
    float ms = 0, t0 = 0, t1 = 0;
    HIP_OK(hipEventElapsedTime(&ms, p.a, p.b));
    HIP_OK(hipEventElapsedTime(&t0, ev_ref_, p.a));
    HIP_OK(hipEventElapsedTime(&t1, ev_ref_, p.b));
    double* acc[kTimedKernels] = {&times_.generate, &times_.extend,     &times_.shade,  &times_.shadow,
                                  &times_.accumulate, &times_.trace, &times_.retrace};
    uint64_t* n[kTimedKernels] = {&times_.n_generate,   &times_.n_extend, &times_.n_shade,  &times_.n_shadow,
                                  &times_.n_accumulate, &times_.n_trace,  &times_.n_retrace};
    *acc[p.slot] += ms;
    *n[p.slot] += 1;
    iv[p.slot].push_back({t0, t1});
  }
  for (int k = 0; k < kTimedKernels; k++) {
    std::sort(iv[k].begin(), iv[k].end());
    double busy = 0, lo = 0, hi = -1e30;
    for (const auto& x : iv[k]) {
      if (x.first > hi) {
        if (hi > lo) busy += hi - lo;
        lo = x.first;
        hi = x.second;
      } else {
        hi = std::max<double>(hi, x.second);
      }
    }
    if (hi > lo) busy += hi - lo;
    times_.busy[k] += busy;
  }
  pending_.clear();
  ev_used_ = 0;
  return true;
}

// Paths a main-lane batch may hold: every lane's slice of it must fit.
uint64_t Renderer::batch_cap() const {
  const int nl = main_lanes();
  uint64_t c = lanes_[0].cap;
  for (int i = 1; i < nl; i++) c = std::min(c, lanes_[i].cap);
  return c * (uint64_t)nl;
}

// Lanes a main batch may use: all of them, or those below the async lanes
// while speculated batches may run there (an adaptive session on one rank).
int Renderer::main_lanes() const {
  const bool async = (stock_slots_ || fill_on_) && nranks_ == 1 && (adaptive_[0] || adaptive_[1]);
  return async ? std::min(nlanes_, kAsyncLane0) : nlanes_;
}

// One lane's count words of a finished batch into st: the rays of bounces
// 0 .. b-1 (bounce 0: k_generate's count, bounce i: the append counter of
// bounce i-1), the shadow rays of each bounce, k_finish's rays and paths.
static void add_counts(Stats& st, const uint32_t* hc, int b, bool stock) {
  // a stock batch's rays count when a round takes its samples (k_consume)
  uint64_t& r = stock ? st.stock_rays : st.rays;
  uint64_t& sr = stock ? st.stock_rays : st.shadow_rays;
  for (int i = 0; i < b; i++) {
    r += i == 0 ? hc[0] : hc[2 + 2 * (i - 1)];
    sr += hc[3 + 2 * i];
  }
  r += hc[kFinishWord];
  sr += hc[kFinishWord + 1];
  st.finish_paths += hc[kFinishWord + 2];
  st.finish_max_bounces = std::max<uint64_t>(st.finish_max_bounces, hc[kFinishWord + 3]);
}

// The per-lane counts of the last main batch (rays, shadow rays, k_finish
// tails) into stats_, once its copies have landed.
bool Renderer::flush_counts(std::string& err) {
  if (!stats_pending_) return true;
  for (int l = 0; l < pend_nl_; l++)
    if (!host_wait(lanes_[l].done, err)) return false;
  for (int l = 0; l < pend_nl_; l++) add_counts(stats_, lanes_[l].h_counts, pend_b_, pend_stock_);
  stats_pending_ = false;
  return true;
}

// A finished async batch's counts (its done events waited for by the caller).
void Renderer::batch_counts(const Batch& B, const uint32_t* hc) {
  for (int i = 0; i < B.nl; i++) add_counts(stats_, hc + (size_t)i * kCountWords, B.b, B.stock);
  stats_.bounces += (uint64_t)B.b;
}

// Lanes, slices and bounce 0 of batch B (k_generate on each lane's stream,
// after the main stream's work so far: reset, round planning, k_spec_plan).
bool Renderer::batch_begin(Batch& B, std::string& err) {
  time_launches_ = profiling_ && !B.async;
  // the mapping: an explicit one (stock batches), half h's current round,
  // or paths k0 .. k0+n-1 of the sequence path k -> (pixel list[k % npix],
  // sample k / npix) over this rank's pixels or over `part` (a screen half)
  const bool round = B.half >= 0 && !B.moff;
  const uint32_t* rnd_off = B.moff ? B.moff : round ? rounds_[B.half].rc : nullptr;
  const uint32_t* rnd_base = B.moff ? B.mbase : round ? rounds_[B.half].rbase : nullptr;
  const uint32_t npix = B.moff ? B.nent : B.part ? B.npix : (uint32_t)part_pix_.size();
  const uint32_t* part = B.part ? B.part : (nranks_ > 1 ? d_part_pix_ : nullptr);
  GenParams G;
  G.W = w_; G.H = h_; G.npix = npix;
  const float fw = (float)w_, fh = (float)h_;
  G.w_inv = 1.0f / fw; G.h_inv = 1.0f / fh; G.ar = fw / fh;  // tracer.rs:167-172
  G.cam[0] = cam_[0]; G.cam[1] = cam_[1]; G.cam[2] = cam_[2];
  G.cx = mcos(cam_[3]); G.sx = msin(cam_[3]);
  G.cy = mcos(cam_[4]); G.sy = msin(cam_[4]);
  G.seed = seed_;
  G.half = w_ / 2;
  G.left_type = (uint32_t)left_type_; G.right_type = (uint32_t)right_type_;
  const uint32_t slots = B.stock ? stock_used_slots_ : 0u;
  for (int i = 0; i <= B.nl; i++) B.off[i] = B.n * (uint64_t)i / (uint64_t)B.nl;
  if (time_launches_) HIP_OK(hipEventRecord(ev_ref_, stream_));
  HIP_OK(hipEventRecord(ev_main_, stream_));
  batch_lanes_ = B.nl;
  for (int i = 0; i < B.nl; i++) {
    const int l = B.lane0 + i;
    bind_batch_lane(B, l);
    if (B.off[i + 1] - B.off[i] > cap_) { bind_lane(0); err = "batch exceeds lane capacity"; return false; }
    if (l != 0) HIP_OK(hipStreamWaitEvent(ks_, ev_main_, 0));  // after reset / round planning on the main stream
    // a low-priority stream after the lane's last main batch (its buffers)
    if (ks_ != lanes_[l].stream) HIP_OK(hipStreamWaitEvent(ks_, lanes_[l].done, 0));
    const uint32_t nn = (uint32_t)(B.off[i + 1] - B.off[i]);
    HIP_OK(hipMemsetAsync(d_counts_, 0, sizeof(uint32_t) * kCountWords, ks_));
    LAUNCH_TIMED(0, generate, n_generate,
                 k_generate<<<blocks_for(nn), kBlock, 0, ks_>>>(G, part, B.k0 + B.off[i], nn, p_pixel_, p_thr_[0],
                                                              p_col_, p_ro_[0], p_rd_[0], d_counts_, rnd_off, rnd_base,
                                                              B.mlist, slots));
  }
  B.maxb = max_depth_ > 0 ? std::min(max_depth_, kMaxBounces) : kMaxBounces;
  // fused: bounce b >= 1 traces its extension rays together with bounce b-1's
  // shadow rays (k_trace); the last bounce's shadow rays follow the loop
  B.fused = (fused_ || B.n < (B.async && async_fused_below_ ? async_fused_below_ : fused_below_)) && trav_ext_ != 1 &&
            trav_sh_ != 1;
  B.pnee = left_type_ == 2 || right_type_ == 2;
  B.b = 0;
  B.finished = false;
  B.state = Batch::kBouncing;
  bind_lane(0);
  return true;
}

// Issues B's bounces until its last one (then its tail) or until a live count
// of an RR-only batch must come back first. block: wait for such counts;
// else return with B in kCountWait when they have not landed yet.
bool Renderer::batch_advance(Batch& B, bool block, std::string& err) {
  const ShadeParams SP{max_depth_, debug_};
  // the bound lane's paths of stream rin, to their end, one lane each
  auto launch_finish = [&](const RayStream& rin, int bb, uint32_t g, bool pn) -> bool {
#define WPT_FIN(T, PN, CR) \
  k_finish<T, PN, CR><<<g, kTBlock, 0, ks_>>>(ds_, SP, rin, ext_count(bb + 1), p_col_, d_spill_, d_counts_ + kFinishWord)
#define WPT_FIN2(T, PN) \
  if (B.stock) WPT_FIN(T, PN, true); \
  else WPT_FIN(T, PN, false)
    if (ds_.tri_only) {
      if (pn) WPT_FIN2(true, true);
      else WPT_FIN2(true, false);
    } else {
      if (pn) WPT_FIN2(false, true);
      else WPT_FIN2(false, false);
    }
#undef WPT_FIN2
#undef WPT_FIN
    HIP_OK(hipGetLastError());
    return true;
  };
  while (B.state == Batch::kBouncing || B.state == Batch::kCountWait) {
    time_launches_ = profiling_ && !B.async;
    batch_lanes_ = B.nl;
    if (B.state == Batch::kCountWait) {
      // the live counts of bounce b = B.b - 1 (RR-only batches): stop once
      // every lane's stream drains; once few paths are left, k_finish runs
      // each of them to its end (one launch instead of one per bounce)
      const int b = B.b - 1;
      uint32_t live[kMaxLanes];
      uint64_t left = 0;
      if (B.async) {
        for (int i = 0; i < B.nl; i++) {
          if (!block) {
            const hipError_t q = hipEventQuery(B.live[i]);
            if (q == hipErrorNotReady) return true;
            HIP_OK(q);
          }
          HIP_OK(hipEventSynchronize(B.live[i]));
        }
        for (int i = 0; i < B.nl; i++) live[i] = B.hl[i];
      } else {
        // the main lanes wait here: first let the async lanes' batches go on
        if (async_pending() && !pump(false, err)) return false;
        time_launches_ = profiling_;
        batch_lanes_ = B.nl;
        for (int i = 0; i < B.nl; i++)
          if (!host_wait_stream(lanes_[B.lane0 + i].stream, err)) return false;
        time_launches_ = profiling_;  // (the waits pump the async lanes)
        batch_lanes_ = B.nl;
        for (int i = 0; i < B.nl; i++) live[i] = lanes_[B.lane0 + i].h_counts[0];
      }
      for (int i = 0; i < B.nl; i++) left += live[i];
      B.state = Batch::kBouncing;
      if (left == 0) break;
      if (left <= finish_below_ && b + 1 < B.maxb) {
        for (int i = 0; i < B.nl; i++) {
          bind_batch_lane(B, B.lane0 + i);
          // bounce b's shadow rays first (fused mode traces them with the
          // next bounce): they are the paths' next colour additions
          if (B.fused && !launch_shadow(sh_count(b), nullptr, err)) { bind_lane(0); return false; }
          if (live[i] == 0) continue;
          const RayStream rin{p_ro_[(b + 1) & 1], p_rd_[(b + 1) & 1], p_thr_[(b + 1) & 1]};
          const uint32_t g =
              (uint32_t)std::min<uint64_t>((live[i] + kTBlock - 1) / kTBlock,
                                           std::min(async_grid(grid_tr_[ds_.tri_only ? 1 : 0], trace_grid_pct_),
                                                    spill_grid()));
          if (!launch_finish(rin, b, g, B.pnee)) { bind_lane(0); return false; }
        }
        B.finished = true;
        break;
      }
      continue;
    }
    if (B.b >= B.maxb) break;
    const int b = B.b;
    cur_bounce_ = b;
    for (int i = 0; i < B.nl; i++) {
      bind_batch_lane(B, B.lane0 + i);
      const uint32_t nn = (uint32_t)(B.off[i + 1] - B.off[i]);
      if (B.fused && b > 0) {
        if (!launch_trace(b, err)) { bind_lane(0); return false; }
      } else if (!launch_extend(p_ro_[b & 1], p_rd_[b & 1], ext_count(b), err)) {
        bind_lane(0);
        return false;
      }
      {
        const RayStream in{p_ro_[b & 1], p_rd_[b & 1], p_thr_[b & 1]};
        const RayStream out{p_ro_[(b + 1) & 1], p_rd_[(b + 1) & 1], p_thr_[(b + 1) & 1]};
        const ShadowStream sh{s_o_, s_d_, s_c_};
        [[maybe_unused]] const uint32_t sgrid =
            std::max<uint32_t>(1, std::min<uint32_t>((nn + kShadeBlock - 1) / kShadeBlock, grid_shade_));
        // the persistent grid of the variant launched: its own occupancy
        // (VGPRs, and the octree's LDS for OC), cached per variant and LDS size
#if WPT_SHADE_GRID_VAR
#define WPT_SHADE_GRID(T, PN, OC, CR)                                                                           \
  const int vi = (CR ? 8 : 0) + (T ? 4 : 0) + (PN ? 1 + OC : 0);                                                \
  const size_t smem = OC ? 4 * (size_t)ds_.oct_lds_words : 0;                                                   \
  if (shade_occ_[vi] == 0 || shade_occ_smem_[vi] != smem) {                                                     \
    int bpc = 0;                                                                                                \
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k_shade<T, PN, OC, CR>, (int)kShadeBlock, smem));  \
    shade_occ_[vi] = (uint32_t)std::max(bpc, 1);                                                                \
    shade_occ_smem_[vi] = smem;                                                                                 \
  }                                                                                                             \
  const uint32_t sg = std::max<uint32_t>(1, std::min<uint32_t>((nn + kShadeBlock - 1) / kShadeBlock,            \
                                                               (uint32_t)ncu_ * shade_occ_[vi]));
#else
#define WPT_SHADE_GRID(T, PN, OC, CR) const uint32_t sg = sgrid;
#endif
#define WPT_SHADE1(T, PN, OC, CR)                                                                                   \
  do {                                                                                                              \
    WPT_SHADE_GRID(T, PN, OC, CR)                                                                                   \
    const uint32_t sgo = async_launch_ && async_oneshot_ ? std::max<uint32_t>(1, (nn + kShadeBlock - 1) / kShadeBlock) \
                                                         : sg;                                                      \
    LAUNCH_TIMED(2, shade, n_shade,                                                                                 \
                 k_shade<T, PN, OC, CR><<<sgo, kShadeBlock, OC ? 4 * ds_.oct_lds_words : 0, ks_>>>(                 \
                     ds_, SP, in, out, sh, p_col_, ext_count(b), p_t_, p_id_, append_ctr(b)));                      \
  } while (0)
// a stock batch's paths write their ray counts (CR)
#define WPT_SHADE(T, PN, OC)              \
  do {                                    \
    if (B.stock) WPT_SHADE1(T, PN, OC, true); \
    else WPT_SHADE1(T, PN, OC, false);    \
  } while (0)
        // PNEE: the octree from LDS when oct_lds_words covers it (child array and CDFs, or the child array)
        const int oc = !B.pnee || ds_.oct_lds_words == 0 ? 0 : (ds_.oct_lds_words > ds_.oct_nodes ? 2 : 1);
        if (ds_.tri_only) {
          if (!B.pnee) WPT_SHADE(true, false, 0);
          else if (oc == 2) WPT_SHADE(true, true, 2);
          else if (oc == 1) WPT_SHADE(true, true, 1);
          else WPT_SHADE(true, true, 0);
        } else {
          if (!B.pnee) WPT_SHADE(false, false, 0);
          else if (oc == 2) WPT_SHADE(false, true, 2);
          else if (oc == 1) WPT_SHADE(false, true, 1);
          else WPT_SHADE(false, true, 0);
        }
#undef WPT_SHADE
#undef WPT_SHADE1
#undef WPT_SHADE_GRID
      }
      if (!B.fused && !launch_shadow(sh_count(b), nullptr, err)) { bind_lane(0); return false; }
    }
    B.b = b + 1;
    if (max_depth_ <= 0 && (b % finish_every_) == finish_every_ - 1) {
      // RR-only mode: the live count of every lane comes back to the host
      for (int i = 0; i < B.nl; i++) {
        bind_batch_lane(B, B.lane0 + i);
        if (B.async) {
          HIP_OK(hipMemcpyAsync(B.hl + i, ext_count(b + 1), sizeof(uint32_t), hipMemcpyDeviceToHost, ks_));
          HIP_OK(hipEventRecord(B.live[i], ks_));
        } else {
          HIP_OK(hipMemcpyAsync(h_counts_, ext_count(b + 1), sizeof(uint32_t), hipMemcpyDeviceToHost, ks_));
        }
      }
      B.state = Batch::kCountWait;
    }
  }
  bind_lane(0);
  return batch_tail(B, err);
}

// B's last shadow rays (fused), its accumulation (or, for a speculated batch,
// the radiance into its slot) and its count words; B is then issued.
bool Renderer::batch_tail(Batch& B, std::string& err) {
  time_launches_ = profiling_ && !B.async;
  batch_lanes_ = B.nl;
  cur_bounce_ = B.b;
  if (B.fused && B.b > 0 && !B.finished) {
    for (int i = 0; i < B.nl; i++) {  // the last bounce's shadow rays
      bind_batch_lane(B, B.lane0 + i);
      if (!launch_shadow(sh_count(B.b - 1), nullptr, err)) { bind_lane(0); return false; }
    }
  }
  const bool round = B.half >= 0 && !B.moff;
  const uint32_t npix = B.part ? B.npix : (uint32_t)part_pix_.size();
  const uint32_t* part = B.part ? B.part : (nranks_ > 1 ? d_part_pix_ : nullptr);
  // in-order accumulation: lane i's slice after lane i-1's (each pixel's
  // samples are summed in sample order, as RenderTarget::write does); a
  // stock batch stores each path into its ring slot instead
  for (int i = 0; i < B.nl; i++) {
    const int l = B.lane0 + i;
    bind_batch_lane(B, l);
    const uint32_t nn = (uint32_t)(B.off[i + 1] - B.off[i]);
    if (i > 0 && !B.stock) HIP_OK(hipStreamWaitEvent(ks_, B.async ? B.done[i - 1] : lanes_[l - 1].done, 0));
    if (B.stock)
      k_stock_store<<<blocks_for(nn), kBlock, 0, ks_>>>(p_pixel_, nn, p_col_, d_stock_);
    else if (round)
      LAUNCH_TIMED(4, accumulate, n_accumulate,
                   k_accumulate_round<<<blocks_for(nn), kBlock, 0, ks_>>>(part, nn, p_pixel_, p_col_, d_acc_, d_cnt_));
    else
      LAUNCH_TIMED(4, accumulate, n_accumulate,
                   k_accumulate<<<blocks_for(std::min<uint64_t>(nn, npix)), kBlock, 0, ks_>>>(
                       part, B.k0 + B.off[i], nn, npix, p_col_, d_acc_, d_cnt_));
    HIP_OK(hipGetLastError());
    // ray statistics from the per-bounce counts (done: after this copy too)
    uint32_t* hc = B.async ? B.hc + (size_t)i * kCountWords : h_counts_;
    HIP_OK(hipMemcpyAsync(hc, d_counts_, sizeof(uint32_t) * kCountWords, hipMemcpyDeviceToHost, ks_));
    HIP_OK(hipEventRecord(B.async ? B.done[i] : lanes_[l].done, ks_));
  }
  bind_lane(0);
  if (!B.async) {
    for (int i = 1; i < B.nl; i++) HIP_OK(hipStreamWaitEvent(stream_, lanes_[B.lane0 + i].done, 0));
    pend_nl_ = B.nl;
    pend_b_ = B.b;
    pend_stock_ = B.stock;
    stats_pending_ = true;
  }
  B.state = Batch::kIssued;
  return true;
}

// Waits for event e; while async batches are queued the host polls and
// pumps them meanwhile (an RR-only async batch issues its next bounces only
// after the host reads its live counts), else it simply blocks.
bool Renderer::host_wait(hipEvent_t e, std::string& err) {
  for (;;) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) HIP_OK(q);
    if (!async_pending()) {
      HIP_OK(hipEventSynchronize(e));
      return true;
    }
    if (!pump(false, err)) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// The same for everything issued on stream s so far.
bool Renderer::host_wait_stream(hipStream_t s, std::string& err) {
  if (!async_pending()) {
    HIP_OK(hipStreamSynchronize(s));
    return true;
  }
  HIP_OK(hipEventRecord(ev_sync_, s));
  return host_wait(ev_sync_, err);
}

// The async lanes: issue the queued batches in order, each as far as its
// live counts allow (block: wait for them).
bool Renderer::pump(bool block, std::string& err) {
  for (auto& q : aq_) {
    while (!q.empty()) {
      Batch& B = *q.front();
      if (B.state == Batch::kNew && !batch_begin(B, err)) return false;
      if (B.state != Batch::kIssued && !batch_advance(B, block, err)) return false;
      if (B.state != Batch::kIssued) break;  // a live count has not landed yet
      q.pop_front();
    }
  }
  bind_lane(0);
  return true;
}

bool Renderer::wait_issued(Batch* B, std::string& err) {
  std::deque<Batch*>& q0 = aq_[B->queue];
  if (B->state == Batch::kNew && std::find(q0.begin(), q0.end(), B) == q0.end()) q0.push_back(B);
  while (B->state != Batch::kIssued) {
    std::deque<Batch*>& q = aq_[B->queue];
    if (q.empty()) { err = "async batch lost"; return false; }
    Batch& H = *q.front();
    if (H.state == Batch::kNew && !batch_begin(H, err)) return false;
    if (!batch_advance(H, true, err)) return false;
    q.pop_front();
  }
  bind_lane(0);
  return true;
}

// Every async batch issued and finished (before a reset, a reallocation or
// the end of the session).
bool Renderer::drain_async(std::string& err) {
  if (!pump(true, err)) return false;
  for (int l = kAsyncLane0; l < lanes_made_; l++) {
    if (lanes_[l].stream) HIP_OK(hipStreamSynchronize(lanes_[l].stream));
    if (lanes_[l].lo) HIP_OK(hipStreamSynchronize(lanes_[l].lo));
  }
  return true;
}

// Lane l's buffers for batch B: on the lane's stream, or for an async batch
// with WPT_OPT_ASYNC_PRIO on its low-priority stream.
void Renderer::bind_batch_lane(const Batch& B, int l) {
  bind_lane(l);
  async_launch_ = B.async;
  async_paths_ = B.off[l - B.lane0 + 1] - B.off[l - B.lane0];
  if (B.async && async_prio_ && lanes_[l].lo) ks_ = lanes_[l].lo;
}

// ---------------------------------------------------------------------------
// The adaptive halves' sample stock (wpt_stock.h)
// ---------------------------------------------------------------------------

// The ring for this viewport (pixels x slots radiance + ray counts, and the
// refill id of each slot), the frontier (= the counts: an empty ring), the
// round deficit and reduction scratch, the refill pool.
bool Renderer::stock_alloc(std::string& err) {
  const uint64_t np = (uint64_t)w_ * h_;
  // WPT_OPT_STOCK slots, fewer for large viewports: slot indices stay below
  // 2^32 and the ring (20 B per slot) below kStockBytes
  uint32_t slots = stock_slots_;
  while (slots > 64 && (np * slots > 0xFFFFFFFFull || np * slots * 20 > kStockBytes)) slots >>= 1;
  if (d_stock_ && stock_cap_ == np * slots && stock_used_slots_ == slots) return true;
  if (np * slots > 0xFFFFFFFFull) { err = "stock: viewport too large for the sample stock (WPT_OPT_STOCK 0)"; return false; }
  // every lane done with the old ring: the async lanes, and the main stream
  // (which waits on the main lanes' last batch: its k_stock_store)
  if (!drain_async(err)) return false;
  HIP_OK(hipStreamSynchronize(stream_));
  ring_give(device_, d_stock_, stock_bytes_[0]);
  ring_give(device_, d_stock_id_, stock_bytes_[1]);
  void* sb[] = {d_front_, d_def_, d_bmax_, d_rays_};
  for (void* q : sb)
    if (q) (void)hipFree(q);
  d_stock_ = nullptr;
  d_stock_id_ = d_front_ = d_def_ = nullptr;
  d_bmax_ = nullptr;
  d_rays_ = nullptr;
  stock_cap_ = 0;
  for (Refill& f : refills_) {
    if (f.off) (void)hipFree(f.off);
    if (f.base) (void)hipFree(f.base);
    f = Refill();
  }
  const uint64_t nb = np / kBlock + 2;
  HIP_OK(ring_take(device_, sizeof(float4) * np * slots, (void**)&d_stock_, &stock_bytes_[0]));
  HIP_OK(ring_take(device_, sizeof(uint32_t) * np * slots, (void**)&d_stock_id_, &stock_bytes_[1]));
  HIP_OK(hipMalloc(&d_front_, sizeof(uint32_t) * np));
  HIP_OK(hipMalloc(&d_def_, sizeof(uint32_t) * (2 * np + 2)));
  HIP_OK(hipMalloc(&d_bmax_, sizeof(uint32_t) * nb + 16));
  HIP_OK(hipMalloc(&d_rays_, sizeof(unsigned long long) * (2 + 2 * nb)));
  HIP_OK(hipMemsetAsync(d_rays_, 0, sizeof(unsigned long long) * 2, stream_));
  HIP_OK(hipMemcpyAsync(d_front_, d_cnt_, sizeof(uint32_t) * np, hipMemcpyDeviceToDevice, stream_));
  for (Refill& f : refills_) {
    HIP_OK(hipMalloc(&f.off, sizeof(uint32_t) * (np + 1)));
    HIP_OK(hipMalloc(&f.base, sizeof(uint32_t) * (np + 1)));
  }
  if (!h_refill_cnt_) {
    HIP_OK(hipHostMalloc(&h_refill_cnt_, sizeof(uint32_t) * kMaxRefill * kRefillChunks * (kCountWords + 1)));
    for (auto& re : refill_ev_)
      for (hipEvent_t& e : re) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  stock_cap_ = np * slots;
  stock_used_slots_ = slots;
  round_need_[0] = round_need_[1] = 0;
  return true;
}

// Empties the ring: the frontier back to the counts (callers drained the
// async lanes first, so no refill is in flight).
void Renderer::stock_drop() {
  // a round partly added keeps its plan: the rest of its samples is traced
  // again as a deficit before it goes on (stock_round with the counts so far)
  for (int h = 0; h < 2; h++) stock_redo_[h] = rounds_[h].pos < rounds_[h].total;
  std::string e;
  for (Refill& f : refills_) {
    if (f.live) (void)refill_count(f, true, e);
    f.live = false;
  }
  round_need_[0] = round_need_[1] = 0;
  if (d_front_ && d_cnt_ && stock_cap_ == (uint64_t)w_ * h_ * stock_used_slots_)
    (void)hipMemcpyAsync(d_front_, d_cnt_, sizeof(uint32_t) * (size_t)w_ * h_, hipMemcpyDeviceToDevice, stream_);
}

// After half h's round is planned: its deficit (pixels whose stock lacks
// samples of the round) traced into the ring on the main lanes now, and
// every stock_every_ rounds a refill of the half's pixels queued on the next
// stock lane, sized down to the `left` positions this compute call still
// gives the half after this round (the stock tapers at the end of a call).
// round_need_[h] = the latest refill holding the round's samples.
bool Renderer::stock_round(int h, uint64_t left, std::string& err) {
  const auto t0 = std::chrono::steady_clock::now();
  struct Tally {
    std::chrono::steady_clock::time_point t0;
    uint64_t& us;
    ~Tally() { us += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count(); }
  } tally{t0, stats_.stock_us};
  if (!stock_alloc(err)) return false;
  HalfRounds& R = rounds_[h];
  const uint32_t npix = (uint32_t)part_pix_.size(), slots = stock_used_slots_;
  const uint32_t nh = half_npix_[h];
  const uint32_t nb = blocks_for((uint64_t)npix + 1);
  uint32_t* def_cnt = d_def_;
  uint32_t* def_base = d_def_ + npix + 1;
  uint32_t* bmax = d_bmax_;
  uint32_t* need = d_bmax_ + nb;
  stock_redo_[h] = false;
  k_stock_plan<<<nb, kBlock, 0, stream_>>>(npix, R.rc, R.rbase, d_cnt_, d_front_, d_stock_id_, slots, def_cnt, def_base,
                                           bmax);
  k_max_reduce<<<1, 1024, 0, stream_>>>(bmax, nb, need);
  auto scan = [&](uint32_t* a, uint32_t n) {
    const uint32_t sb = (n + kScanChunk - 1) / kScanChunk;
    k_scan_local<<<sb, kBlock, 0, stream_>>>(a, n, d_scan_sums_);
    k_scan_sums<<<1, kBlock, 0, stream_>>>(d_scan_sums_, sb);
    k_scan_add<<<sb, kBlock, 0, stream_>>>(a, n, d_scan_sums_);
  };
  scan(def_cnt, npix + 1);
  // the refill, sized by the positions of later rounds in this call
  Refill* F = nullptr;
  const uint64_t after = left > R.total ? left - R.total : 0;
  const uint32_t q = refill_scale(h, stock_ahead_, after);
  if (nh && d_half_pix_[h] && (R.idx - 1) % stock_every_ == 0 && q > 0) {
    if (!(F = refill_slot(err))) return false;
    refill_plan(*F, h, stock_ahead_, q);
  }
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(h_word_, def_cnt + npix, sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipMemcpyAsync(h_word_ + 1, need, sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  if (F) HIP_OK(hipMemcpyAsync(h_word_ + 2, F->off + nh, sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  if (!host_wait_stream(stream_, err)) return false;
  const uint32_t dt = h_word_[0], wt = F ? h_word_[2] : 0u;
  round_need_[h] = h_word_[1];
  if (log_)
    WPT_LOGF("stock_round h=%d idx=%u pos=%lu total=%lu left=%lu deficit=%u need=%u refill=%u q=%u\n", h, R.idx,
            (unsigned long)R.pos, (unsigned long)R.total, (unsigned long)left, dt, h_word_[1], wt, q);
  stats_.stock_traced += dt;
  stats_.stock_deficit += dt;
  if (dt) {
    // the deficit, traced now on the main lanes into the ring
    Batch M;
    M.moff = def_cnt;
    M.mbase = def_base;
    M.nent = npix;
    M.stock = true;
    // in batches the main lanes hold (they are sized for this call's budget)
    const uint64_t cap = std::max<uint64_t>(batch_cap(), 1);
    for (uint64_t k0 = 0; k0 < dt; k0 += cap)
      if (!run_batch(k0, std::min<uint64_t>(cap, dt - k0), -1, err, nullptr, 0, &M)) return false;
  }
  if (wt && !refill_issue(*F, h, wt, err)) return false;
  return true;
}

// q (of 1024) scaling a refill of half h with lookahead `ahead` to the
// `after` positions the call still gives the half's later rounds.
uint32_t Renderer::refill_scale(int h, uint32_t ahead, uint64_t after) const {
  const uint64_t expect = (uint64_t)ahead * rounds_[h].total + (uint64_t)stock_extra_ * half_npix_[h];
  return expect <= after ? 1024u : (uint32_t)(after * 1024 / std::max<uint64_t>(expect, 1));
}

// A refill pool entry: a free one, else the oldest once it is done.
Renderer::Refill* Renderer::refill_slot(std::string& err) {
  Refill* F = nullptr;
  for (Refill& f : refills_)
    if (!f.live) return &f;
  for (Refill& f : refills_)
    if (!F || f.id < F->id) F = &f;
  if (!refill_count(*F, true, err)) return nullptr;
  F->live = false;
  return F;
}

// k_refill_plan of half h into F (its counts scanned into offsets), from the
// counts of the half's current round (c per pixel: the predictor).
void Renderer::refill_plan(Refill& F, int h, uint32_t ahead, uint32_t q) {
  const uint32_t nh = half_npix_[h];
  k_refill_plan<<<blocks_for((uint64_t)nh + 1), kBlock, 0, stream_>>>(d_half_pix_[h], nh, rounds_[h].rc, d_cnt_,
                                                                      d_front_, d_stock_id_, stock_used_slots_, ahead,
                                                                      stock_extra_, q, refill_id_, F.off, F.base);
  const uint32_t n = nh + 1, sb = (n + kScanChunk - 1) / kScanChunk;
  k_scan_local<<<sb, kBlock, 0, stream_>>>(F.off, n, d_scan_sums_);
  k_scan_sums<<<1, kBlock, 0, stream_>>>(d_scan_sums_, sb);
  k_scan_add<<<sb, kBlock, 0, stream_>>>(F.off, n, d_scan_sums_);
}

// F's wt planned samples onto the next stock lane, in chunks its lane holds.
bool Renderer::refill_issue(Refill& F, int h, uint64_t wt, std::string& err) {
  const uint32_t nh = half_npix_[h];
  const int l = kAsyncLane0 + refill_lane_;
  refill_lane_ = (refill_lane_ + 1) % stock_lanes_;
  // batches of 2^25 paths, larger when a refill would need more than
  // kRefillChunks of them (4K viewports: ~1 G samples per refill)
  const uint64_t chunk = std::max(std::min<uint64_t>(wt, kRefillChunk), (wt + kRefillChunks - 1) / kRefillChunks);
  if (chunk > 0xFFFFFFFFull || (wt + chunk - 1) / chunk > (uint64_t)kRefillChunks) {
    err = "stock refill too large";
    return false;
  }
  if (lanes_[l].cap < chunk && !drain_async(err)) return false;
  if (!ensure_lane(l, chunk, err)) return false;
  if (async_oneshot_ && lanes_[l].spill_cap < spill_slots() * (size_t)oneshot_grid(chunk) * kTBlock &&
      (!drain_async(err) || !ensure_spill(l, oneshot_grid(chunk), err)))
    return false;
  F.id = refill_id_++;
  if (log_) WPT_LOGF("refill id=%u h=%d n=%lu lane=%d\n", F.id, h, (unsigned long)wt, l);
  F.live = true;
  F.counted = false;
  F.chunks.clear();
  const size_t pool = (size_t)(&F - refills_);
  for (uint64_t k0 = 0; k0 < wt; k0 += chunk) {
    F.chunks.emplace_back();
    Batch& B = F.chunks.back();
    const size_t ci = F.chunks.size() - 1;
    B.k0 = k0;
    B.n = std::min<uint64_t>(chunk, wt - k0);
    B.moff = F.off;
    B.mbase = F.base;
    B.mlist = d_half_pix_[h];
    B.nent = nh;
    B.stock = true;
    B.async = true;
    B.queue = 0;
    B.lane0 = l;
    B.nl = 1;
    B.hc = h_refill_cnt_ + (pool * kRefillChunks + ci) * (kCountWords + 1);
    B.hl = B.hc + kCountWords;
    B.done[0] = refill_ev_[pool][2 * ci];
    B.live[0] = refill_ev_[pool][2 * ci + 1];
    aq_[0].push_back(&B);
  }
  stats_.stock_traced += wt;
  return pump(false, err);
}

// At the start of a compute call: half h's stock refilled from the counts of
// its last planned round (the predictor of its next ones), sized to the
// `budget` positions this call gives it, as refills of growing lookahead
// (its next rounds wait only for the first, small one). The half's refills
// then run on the async lanes while the other half's work goes on.
bool Renderer::stock_prefill(int h, uint64_t budget, std::string& err) {
  if (!stock_active(h) || rounds_[h].idx == 0 || rounds_[h].total == 0 || !half_npix_[h] || !d_half_pix_[h])
    return true;
  if (!stock_alloc(err)) return false;
  const uint32_t la[3] = {2u, std::min(8u, stock_ahead_), stock_ahead_};
  uint32_t prev = 0;
  for (uint32_t ahead : la) {
    if (ahead <= prev) continue;
    prev = ahead;
    const uint32_t q = refill_scale(h, ahead, budget);
    if (q == 0) break;
    Refill* F = refill_slot(err);
    if (!F) return false;
    refill_plan(*F, h, ahead, q);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(h_word_ + 2, F->off + half_npix_[h], sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
    if (!host_wait_stream(stream_, err)) return false;
    const uint32_t wt = h_word_[2];
    if (log_) WPT_LOGF("prefill h=%d ahead=%u q=%u refill=%u\n", h, ahead, q, wt);
    if (wt && !refill_issue(*F, h, wt, err)) return false;
  }
  return true;
}

// Positions [a, b) of half h's current round, added from the ring once the
// refills holding its samples are done (the deficit went ahead of it on the
// main stream).
bool Renderer::stock_consume(int h, uint64_t a, uint64_t b, std::string& err) {
  HalfRounds& R = rounds_[h];
  const uint32_t need = round_need_[h];
  bool waited = false;
  for (Refill& f : refills_) {
    if (!f.live || !need || f.id > need - 1) continue;
    for (Batch& c : f.chunks) {
      if (!wait_issued(&c, err)) return false;
      const hipError_t q = hipEventQuery(c.done[0]);
      if (q == hipErrorNotReady) waited = true;
      else HIP_OK(q);
      HIP_OK(hipStreamWaitEvent(stream_, c.done[0], 0));
    }
  }
  if (waited && a == rounds_[h].pos) stats_.stock_waits++;
  if (log_ && waited) WPT_LOGF("consume h=%d waits on a refill in flight (need=%u)\n", h, need);
  const uint32_t npix = (uint32_t)part_pix_.size();
  const uint32_t nb = blocks_for(npix);
  if (log_) WPT_LOGF("consume h=%d [%lu, %lu) need=%u\n", h, (unsigned long)a, (unsigned long)b, need);
  k_consume<<<nb, kBlock, 0, stream_>>>(npix, R.rc, R.rbase, (uint32_t)a, (uint32_t)b, d_stock_, stock_used_slots_,
                                         d_acc_, d_cnt_, d_rays_ + 2);
  k_rays_reduce<<<1, 1024, 0, stream_>>>(d_rays_ + 2, nb, d_rays_);
  HIP_OK(hipGetLastError());
  stats_.stock_consumed += b - a;
  return true;
}

// Refill f's batches' counts into stats_ once they are done (block: wait).
bool Renderer::refill_count(Refill& f, bool block, std::string& err) {
  if (f.counted) return true;
  for (Batch& c : f.chunks) {
    if (c.state != Batch::kIssued) {
      if (!block) return true;
      if (!wait_issued(&c, err)) return false;
    }
    if (block) {
      HIP_OK(hipEventSynchronize(c.done[0]));
    } else {
      const hipError_t q = hipEventQuery(c.done[0]);
      if (q == hipErrorNotReady) return true;
      HIP_OK(q);
    }
  }
  for (const Batch& c : f.chunks) batch_counts(c, c.hc);
  f.counted = true;
  return true;
}

// The rays of the samples the rounds took (k_consume) into stats_, and the
// counts of the refills done by now.
bool Renderer::stock_flush(std::string& err) {
  for (Refill& f : refills_)
    if (f.live && !refill_count(f, false, err)) return false;
  if (!d_rays_) return true;
  unsigned long long r[2];
  HIP_OK(hipMemcpyAsync(r, d_rays_, sizeof r, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipMemsetAsync(d_rays_, 0, sizeof r, stream_));
  if (!host_wait_stream(stream_, err)) return false;
  stats_.rays += r[0];
  stats_.shadow_rays += r[1];
  stats_.stock_rays_used += r[0] + r[1];
  return true;
}

// Paths k0 .. k0+n-1 of half h's rest-of-half sequence (path k -> (rest[k %
// nrest], sample k / nrest)) on the fill lane, as async batches of at most
// 2^25 paths; their counts land in stats_ at drain_fill.
bool Renderer::issue_fill(int h, uint64_t k0, uint64_t n, std::string& err) {
  if (!h_fill_cnt_) {
    HIP_OK(hipHostMalloc(&h_fill_cnt_, sizeof(uint32_t) * kMaxFill * (kCountWords + 1)));
    for (auto& fe : fill_ev_)
      for (hipEvent_t& e : fe) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const uint64_t chunk = std::min<uint64_t>(n, 1ull << 25);
  const int l = fill_lane();
  if (lanes_[l].cap < chunk && !drain_fill(err)) return false;
  if (!ensure_lane(l, chunk, err)) return false;
  if (async_oneshot_ && lanes_[l].spill_cap < spill_slots() * (size_t)oneshot_grid(chunk) * kTBlock &&
      (!drain_fill(err) || !ensure_spill(l, oneshot_grid(chunk), err)))
    return false;
  for (uint64_t done = 0; done < n;) {
    if (nfill_ == kMaxFill && !drain_fill(err)) return false;
    const uint64_t m = std::min(chunk, n - done);
    Batch& B = fill_[nfill_];
    B = Batch();
    B.k0 = k0 + done;
    B.n = m;
    B.part = d_rest_pix_[h];
    B.npix = rest_npix_[h];
    B.async = true;
    B.queue = 1;
    B.lane0 = l;
    B.nl = 1;
    B.hc = h_fill_cnt_ + (size_t)nfill_ * (kCountWords + 1);
    B.hl = B.hc + kCountWords;
    B.done[0] = fill_ev_[nfill_][0];
    B.live[0] = fill_ev_[nfill_][1];
    nfill_++;
    aq_[1].push_back(&B);
    done += m;
  }
  return pump(false, err);
}

// Every filler batch issued and finished; their rays and paths into stats_.
bool Renderer::drain_fill(std::string& err) {
  for (int i = 0; i < nfill_; i++) {
    Batch& B = fill_[i];
    if (!wait_issued(&B, err)) return false;
    HIP_OK(hipEventSynchronize(B.done[0]));
    batch_counts(B, B.hc);
    stats_.paths += B.n;
    stats_.fill_paths += B.n;
  }
  nfill_ = 0;
  return true;
}

// compute(n)'s two halves (wasm_interface.rs:374-379: n/2 positions of the
// left half's sequence, then n - n/2 of the right half's). With one random
// and one adaptive half on one rank, the random half's whole rounds of this
// call do not depend on the image, and the adaptive half's rounds read the
// random half only in its seam columns (the 5x5 filter's radius 2,
// render_target.rs:112-128, sampling_strategy.rs:138-141). So the random
// half's rest pixels are traced on the fill lane beside the adaptive half's
// rounds, and its seam pixels on the main lanes where the reference's order
// puts them relative to the adaptive half's plans: before them when the
// random half is the left one, after them when it is the right one. Each
// pixel keeps its samples in sample order; the frame is the same bits.
bool Renderer::compute_halves(uint64_t nl, uint64_t nr, std::string& err) {
  int R = -1;
  if (fill_on_ && nranks_ == 1 && adaptive_[0] != adaptive_[1]) R = adaptive_[0] ? 1 : 0;
  const uint64_t nR = R == 0 ? nl : nr;
  const uint64_t nh = R >= 0 ? half_npix_[R] : 0;
  if (R < 0 || nh == 0 || rounds_[R].pos != rounds_[R].total || nR < nh || !d_seam_pix_[R] || !d_rest_pix_[R] ||
      (uint64_t)rounds_[R].idx + nR / nh > 0xFFFFFFFFull)
    return compute_half(0, nl, err) && compute_half(1, nr, err);
  HalfRounds& RR = rounds_[R];
  const uint64_t k = nR / nh, rem = nR - k * nh;
  const uint64_t ns = seam_npix_[R], nrest = rest_npix_[R];
  auto seam = [&]() -> bool {
    // the seam's k whole rounds on the main lanes, in batches they hold
    const uint64_t cap = std::max<uint64_t>(batch_cap() / ns * ns, ns);
    for (uint64_t d = 0; d < k * ns;) {
      const uint64_t m = std::min(cap, k * ns - d);
      if (!run_batch((uint64_t)RR.idx * ns + d, m, -1, err, d_seam_pix_[R], (uint32_t)ns)) return false;
      d += m;
    }
    return true;
  };
  if (R == 0) {
    if (!seam() || !issue_fill(0, (uint64_t)RR.idx * nrest, k * nrest, err)) return false;
    RR.idx += (uint32_t)k;
    // a partial round after the whole ones: raster order, after the filler
    if (rem && (!drain_fill(err) || !compute_half(0, rem, err))) return false;
    if (!compute_half(1, nr, err)) return false;
  } else {
    if (!issue_fill(1, (uint64_t)RR.idx * nrest, k * nrest, err)) return false;
    if (!compute_half(0, nl, err) || !seam()) return false;
    RR.idx += (uint32_t)k;
    if (rem && (!drain_fill(err) || !compute_half(1, rem, err))) return false;
  }
  return drain_fill(err);
}

bool Renderer::run_batch(uint64_t k0, uint64_t n, int half, std::string& err, const uint32_t* part_pix,
                         uint32_t part_n, const Batch* map) {
  if (log_) WPT_LOGF("run_batch k0=%lu n=%lu half=%d stock=%d\n", (unsigned long)k0, (unsigned long)n, half,
                    map && map->stock ? 1 : 0);
  if (!flush_counts(err)) return false;  // the previous batch's counts, before its h_counts are reused
  if (async_pending() && !pump(false, err)) return false;
  Batch B;
  B.k0 = k0;
  B.n = n;
  B.half = half;
  B.part = part_pix;
  B.npix = part_n;
  if (map) {  // an explicit mapping (a round's stock deficit)
    B.moff = map->moff;
    B.mbase = map->mbase;
    B.mlist = map->mlist;
    B.nent = map->nent;
    B.stock = map->stock;
  }
  // the batch is cut into contiguous slices, one per lane (small batches: one
  // lane); each slice is a sub-range of the path (or round-position) sequence
  // small batches (adaptive sample rounds) run on at most small_lanes_ lanes
  // when their slices fit the lanes' capacity
  const int lanes = main_lanes();
  int nlb = lanes;
  if (n < fused_below_ && small_lanes_ < lanes) {
    uint64_t cmin = lanes_[0].cap;
    for (int i = 1; i < small_lanes_; i++) cmin = std::min(cmin, lanes_[i].cap);
    if ((n + small_lanes_ - 1) / small_lanes_ <= cmin) nlb = small_lanes_;
  }
  B.nl = (n < (uint64_t)nlb * kMinLanePaths && n <= lanes_[0].cap) ? 1 : nlb;
  B.lane0 = 0;
  if (!batch_begin(B, err)) return false;
  while (B.state != Batch::kIssued)
    if (!batch_advance(B, true, err)) return false;
  time_launches_ = false;
  if (profiling_) {
    for (int i = 0; i < B.nl; i++) HIP_OK(hipStreamSynchronize(lanes_[i].stream));
    if (!resolve_timings(err)) return false;
  }
  // the batch's counts (returning before they land, so that an adaptive
  // round's planning queues behind its batch, measured neutral on C5:
  // profiles/r05/ab_deferred_sync.jsonl)
  if (!flush_counts(err)) return false;
  const int b = B.b;
  if (profiling_) {
    times_.logical[0] += 1;
    times_.logical[1] += B.fused ? 1u : (uint64_t)b;
    times_.logical[2] += (uint64_t)b;
    times_.logical[3] += B.fused ? 1u : (uint64_t)b;
    times_.logical[4] += 1;
    times_.logical[5] += B.fused ? (uint64_t)(b - 1) : 0u;
  }
  stats_.bounces += (uint64_t)b;
  if (!B.stock) stats_.paths += n;  // a stock batch's samples count when a round takes them
  if (log_) WPT_LOGF("batch done n=%lu bounces=%d finished=%d\n", (unsigned long)n, b, B.finished ? 1 : 0);
  return true;
}

// n positions of screen half h's round sequence. With several ranks the
// sequence is the whole frame's (every rank calls with the same n) and this
// rank traces the positions that fall on its own pixels.
bool Renderer::compute_half(int h, uint64_t n, std::string& err) {
  if (log_) WPT_LOGF("compute_half h=%d n=%lu pos=%lu total=%lu redo=%d\n", h, (unsigned long)n,
                    (unsigned long)rounds_[h].pos, (unsigned long)rounds_[h].total, stock_redo_[h] ? 1 : 0);
  const uint32_t half = w_ / 2;
  if ((h == 0 ? half : w_ - half) == 0) return true;  // an empty half (width 1) takes no samples
  const uint64_t bsz = std::min<uint64_t>(std::max<uint64_t>(batch_, 1), 0xFFFFFFFFull);
  HalfRounds& R = rounds_[h];
  uint64_t done = 0;
  while (done < n) {
    if (!adaptive_[h] && nranks_ == 1 && R.pos == R.total && half_npix_[h] != 0) {
      // whole rounds of a non-adaptive half do not depend on the image: a
      // round gives each of the half's pixels (raster order) one sample, and
      // at a round boundary every one of them holds R.idx samples, so rounds
      // R.idx .. R.idx+k-1 are paths R.idx*nh .. of the half's uniform sequence
      const uint64_t nh = half_npix_[h];
      const uint64_t cap = std::min(batch_cap(), bsz) / nh * nh;
      const uint64_t m = std::min((n - done) / nh * nh, cap);
      if (m != 0) {
        if (!run_batch((uint64_t)R.idx * nh, m, -1, err, d_half_pix_[h], (uint32_t)nh)) return false;
        R.idx += (uint32_t)(m / nh);
        done += m;
        continue;
      }
    }
    if (R.pos == R.total && (!plan_round(h, err) || (stock_active(h) && !stock_round(h, n - done, err)))) return false;
    if (nranks_ > 1) {
      const uint64_t m = std::min(std::min(bsz, n - done), R.total - R.pos);
      uint64_t local = 0;
      if (!plan_slice(h, R.pos, R.pos + m, local, err)) return false;
      if (local && !run_batch(0, local, h, err)) return false;
      R.pos += m;
      done += m;
    } else {
      const uint64_t m = std::min(std::min(std::min(batch_cap(), bsz), n - done), R.total - R.pos);
      if (stock_active(h)) {
        // positions [pos, pos + m) added from the sample stock (the round's
        // deficit was traced into it when the round was planned, or again
        // after the stock was dropped)
        if (stock_redo_[h] && !stock_round(h, n - done + R.pos, err)) return false;
        if (!stock_consume(h, R.pos, R.pos + m, err)) return false;
        stats_.paths += m;
      } else if (!run_batch(R.pos, m, h, err)) {
        return false;
      }
      R.pos += m;
      done += m;
    }
  }
  return true;
}

// Two random halves on one rank: when both stand at a round boundary with the
// same rounds done and this call gives each of them the same k whole rounds
// (an even width and n a multiple of the frame), the halves' rounds are the
// frame's rounds k: one batch sequence over the whole frame in tile order
// (path j -> (frame pixel j mod P, sample idx + j div P)), the same (pixel,
// sample) pairs as two per-half sequences. Otherwise merged = false.
bool Renderer::merge_random_halves(uint64_t nl, uint64_t nr, bool& merged, std::string& err) {
  merged = false;
  HalfRounds& A = rounds_[0];
  HalfRounds& B = rounds_[1];
  const uint64_t n0 = half_npix_[0], n1 = half_npix_[1];
  const uint64_t npix = part_pix_.size();
  if (!d_frame_pix_ || n0 == 0 || n1 == 0 || A.pos != A.total || B.pos != B.total || A.idx != B.idx) return true;
  if (nl % n0 != 0 || nr % n1 != 0 || nl / n0 != nr / n1 || nl == 0) return true;
  const uint64_t bsz = std::min<uint64_t>(std::max<uint64_t>(batch_, 1), 0xFFFFFFFFull);
  const uint64_t cap = std::min(batch_cap(), bsz) / npix * npix;
  if (cap == 0) return true;  // batches smaller than a round: the per-half path
  const uint64_t k = nl / n0;
  if ((uint64_t)A.idx + k > 0xFFFFFFFFull) { err = "sample index overflow"; return false; }
  uint64_t done = 0;
  while (done < k * npix) {
    const uint64_t m = std::min(cap, k * npix - done);
    if (!run_batch((uint64_t)A.idx * npix + done, m, -1, err, d_frame_pix_, (uint32_t)npix)) return false;
    done += m;
  }
  A.idx += (uint32_t)k;
  B.idx += (uint32_t)k;
  merged = true;
  return true;
}

bool Renderer::compute(uint64_t num_paths, std::string& err) {
  if (!scene_ok_) { err = "no scene"; return false; }
  if (!d_acc_ || part_pix_.empty()) { err = "no viewport"; return false; }
  if (num_paths == 0) return true;
  const uint64_t npix = part_pix_.size();
  // a batch never holds more than 2^32 paths; keep sample index < 2^32
  const uint64_t bsz = std::min<uint64_t>(std::max<uint64_t>(batch_, 1), 0xFFFFFFFFull);
  if ((left_type_ == 2 || right_type_ == 2) && !build_photons(err)) return false;
  {
    // every lane holds its slice of a full batch; a batch too small to split
    // runs on lane 0 alone
    const int ml = main_lanes();  // (the async lanes are sized by issue_spec)
    const uint64_t want = std::min(bsz, num_paths);
    const uint64_t per = (want + ml - 1) / ml;
    for (int i = 0; i < ml; i++)
      if (!ensure_lane(i, (i == 0 && want < (uint64_t)ml * kMinLanePaths) ? want : per, err)) return false;
  }
  uint64_t done = num_paths;
  if (adaptive_[0] || adaptive_[1] || nranks_ == 1) {
    // as the reference's compute (wasm_interface.rs:374-379): n/2 positions
    // of the left half's sequence, then n - n/2 of the right half's
    const uint64_t nl = num_paths / 2;
    bool merged = false;
    if (!adaptive_[0] && !adaptive_[1] && !merge_random_halves(nl, num_paths - nl, merged, err)) return false;
    if (!merged) {
      if (stock_prefill_ && (!stock_prefill(0, nl, err) || !stock_prefill(1, num_paths - nl, err))) return false;
      if (!compute_halves(nl, num_paths - nl, err)) return false;
    }
  } else {
    // several ranks with random halves: n paths over this rank's partition
    done = 0;
  }
  while (done < num_paths) {
    const uint64_t n = std::min(std::min(batch_cap(), bsz), num_paths - done);
    if ((next_path_ + n) / npix > 0xFFFFFFFFull) { err = "sample index overflow"; return false; }
    const bool whole = nranks_ == 1 && d_frame_pix_ && next_path_ % npix == 0 && n % npix == 0;
    if (!(whole ? run_batch(next_path_, n, -1, err, d_frame_pix_, (uint32_t)npix) : run_batch(next_path_, n, -1, err)))
      return false;
    next_path_ += n;
    done += n;
  }
  // every lane's work of this call done (an adaptive round's batch returns
  // without waiting): the readbacks below go through the null stream
  if (!flush_counts(err)) return false;
  {
    uint32_t fb[4];
    HIP_OK(hipMemcpy(fb, d_fallback_, sizeof fb, hipMemcpyDeviceToHost));
    HIP_OK(hipMemset(d_fallback_, 0, sizeof fb));
    stats_.fallback_ext += fb[0];
    stats_.fallback_sh += fb[1];
    if (fb[2]) { err = "traversal stack overflow (results invalid)"; return false; }
  }
  if (!stock_flush(err)) return false;
  if (async_pending() && !pump(false, err)) return false;
  if (counting_) {
    unsigned long long wc[kWorkWords * kWorkCopies], w[kWorkWords] = {};
    HIP_OK(hipMemcpy(wc, d_work_, sizeof wc, hipMemcpyDeviceToHost));
    HIP_OK(hipMemset(d_work_, 0, sizeof wc));
    for (uint32_t i = 0; i < kWorkWords * kWorkCopies; i++)
      w[i % kWorkWords] = i % kWorkWords == 14 ? std::max(w[14], wc[i]) : w[i % kWorkWords] + wc[i];  // 14: a maximum
    stats_.node_visits += w[0] + w[3];
    stats_.prim_tests += w[1] + w[4];
    stats_.ext_visits += w[0];
    stats_.ext_tests += w[1];
    stats_.ext_node_bytes += w[2];
    stats_.sh_visits += w[3];
    stats_.sh_tests += w[4];
    stats_.sh_node_bytes += w[5];
    stats_.ext_lane_iters += w[6];
    stats_.ext_live_iters += w[7];
    stats_.sh_lane_iters += w[8];
    stats_.sh_live_iters += w[9];
    stats_.trace_bytes += w[15];
    stats_.max_ray_visits = std::max<uint64_t>(stats_.max_ray_visits, w[14]);
    stats_.ex_body_lanes += w[10];
    stats_.ex_bodies += w[11];
    stats_.lf_body_lanes += w[12];
    stats_.lf_bodies += w[13];
  }
  return true;
}

bool Renderer::sync(std::string& err) {
  if (!drain_async(err)) return false;  // every launch of the session done, the async lanes' too
  for (Refill& f : refills_)
    if (f.live && !refill_count(f, true, err)) return false;
  if (stream_) HIP_OK(hipStreamSynchronize(stream_));
  return flush_counts(err);
}

bool Renderer::results_rgba(uint8_t* out, std::string& err) {
  const uint32_t np = w_ * h_;
  k_rgba<<<blocks_for(np), kBlock, 0, stream_>>>(d_acc_, d_cnt_, np, d_rgba_);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(out, d_rgba_, 4 * (size_t)np, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  return true;
}

bool Renderer::read_radiance(float* acc3, uint32_t* cnt, std::string& err) {
  const size_t np = (size_t)w_ * h_;
  std::vector<float4> a(np);
  HIP_OK(hipMemcpyAsync(a.data(), d_acc_, sizeof(float4) * np, hipMemcpyDeviceToHost, stream_));
  if (cnt) HIP_OK(hipMemcpyAsync(cnt, d_cnt_, sizeof(uint32_t) * np, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  for (size_t i = 0; i < np; i++) {
    acc3[3 * i] = a[i].x;
    acc3[3 * i + 1] = a[i].y;
    acc3[3 * i + 2] = a[i].z;
  }
  return true;
}

bool Renderer::copy_partition(float* dev_dst, std::string& err) {
  const uint32_t n = (uint32_t)part_pix_.size();
  k_pack_partition<<<blocks_for(n), kBlock, 0, stream_>>>(nranks_ > 1 ? d_part_pix_ : nullptr, n, d_acc_, d_cnt_,
                                                          (float4*)dev_dst);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(stream_));
  return true;
}

// Launch one bounce of the extend kernel over rays (ro, rd) 0..*cnt-1 with
// the scene's traversal (trav_ext_: 0 exact BVH2, 1 BVH4 fast path). Hits go
// to the bound lane's t / id.
bool Renderer::launch_extend(const float4* ro, const float4* rd, const uint32_t* cnt, std::string& err) {
  const int v = (ds_.tri_only ? 1 : 0) | (counting_ ? 2 : 0) | (trav_ext_ << 2);
  const int full = batch_lanes_ == 1 ? kTravVariants : 0;
  const uint32_t g = std::min(async_grid(grid_ext_[v + full], 100), spill_grid());
  ds_.probe = probe_slot(1, g);
#define WPT_EXT(T, C, F) \
  k_extend<T, C, F><<<g, kTBlock, 0, ks_>>>(ds_, ro, rd, cnt, p_t_, p_id_, d_spill_, d_work_, d_fallback_)
  switch (v) {
    case 0: LAUNCH_TIMED(1, extend, n_extend, WPT_EXT(false, false, 0)); break;
    case 1: LAUNCH_TIMED(1, extend, n_extend, WPT_EXT(true, false, 0)); break;
    case 2: LAUNCH_TIMED(1, extend, n_extend, WPT_EXT(false, true, 0)); break;
    case 3: LAUNCH_TIMED(1, extend, n_extend, WPT_EXT(true, true, 0)); break;
    case 4: LAUNCH_TIMED(1, extend, n_extend, WPT_EXT(false, false, 1)); break;
    case 5: LAUNCH_TIMED(1, extend, n_extend, WPT_EXT(true, false, 1)); break;
    case 6: LAUNCH_TIMED(1, extend, n_extend, WPT_EXT(false, true, 1)); break;
    default: LAUNCH_TIMED(1, extend, n_extend, WPT_EXT(true, true, 1)); break;
  }
#undef WPT_EXT
  ds_.probe = nullptr;
  return true;
}

// The bound lane's shadow stream, rays 0..*cnt-1 (trav_sh_ as launch_extend).
bool Renderer::launch_shadow(const uint32_t* cnt, uint8_t* occ_out, std::string& err) {
  const int v = (ds_.tri_only ? 1 : 0) | (counting_ ? 2 : 0) | (trav_sh_ << 2);
  const int full = batch_lanes_ == 1 ? kTravVariants : 0;
  const uint32_t g = std::min(async_grid(grid_sh_[v + full], 100), spill_grid());
  ds_.probe = probe_slot(3, g);
#define WPT_SH(T, C, F)                                                                                        \
  k_shadow<T, C, F><<<g, kTBlock, 0, ks_>>>(ds_, cnt, s_o_, s_d_, s_c_, p_col_, occ_out, d_spill_, d_work_, \
                                           d_fallback_)
  switch (v) {
    case 0: LAUNCH_TIMED(3, shadow, n_shadow, WPT_SH(false, false, 0)); break;
    case 1: LAUNCH_TIMED(3, shadow, n_shadow, WPT_SH(true, false, 0)); break;
    case 2: LAUNCH_TIMED(3, shadow, n_shadow, WPT_SH(false, true, 0)); break;
    case 3: LAUNCH_TIMED(3, shadow, n_shadow, WPT_SH(true, true, 0)); break;
    case 4: LAUNCH_TIMED(3, shadow, n_shadow, WPT_SH(false, false, 1)); break;
    case 5: LAUNCH_TIMED(3, shadow, n_shadow, WPT_SH(true, false, 1)); break;
    case 6: LAUNCH_TIMED(3, shadow, n_shadow, WPT_SH(false, true, 1)); break;
    default: LAUNCH_TIMED(3, shadow, n_shadow, WPT_SH(true, true, 1)); break;
  }
#undef WPT_SH
  ds_.probe = nullptr;
  return true;
}

// Bounce b's extension rays and bounce b-1's shadow rays of the bound lane
// in one launch (exact BVH2; the fused form never runs the BVH4 fast path).
bool Renderer::launch_trace(int b, std::string& err) {
  const int v = (ds_.tri_only ? 1 : 0) | (counting_ ? 2 : 0);
  const uint32_t g = std::min(async_grid(grid_tr_[v], trace_grid_pct_, 2), spill_grid());  // extension + shadow rays
  const float4* ro = p_ro_[b & 1];
  const float4* rd = p_rd_[b & 1];
  const uint32_t* ce = ext_count(b);
  const uint32_t* cs = sh_count(b - 1);
  ds_.probe = probe_slot(5, g);
#define WPT_TR(T, C) \
  k_trace<T, C><<<g, kTBlock, 0, ks_>>>(ds_, ro, rd, ce, p_t_, p_id_, cs, s_o_, s_d_, s_c_, p_col_, d_spill_, d_work_)
  switch (v) {
    case 0: LAUNCH_TIMED(5, trace, n_trace, WPT_TR(false, false)); break;
    case 1: LAUNCH_TIMED(5, trace, n_trace, WPT_TR(true, false)); break;
    case 2: LAUNCH_TIMED(5, trace, n_trace, WPT_TR(false, true)); break;
    default: LAUNCH_TIMED(5, trace, n_trace, WPT_TR(true, true)); break;
  }
#undef WPT_TR
  ds_.probe = nullptr;
  (void)err;
  return true;
}

// The wave-timeline record of the next traversal launch (kernel 1 extend, 3
// shadow, 5 trace) of `grid` blocks, or null when probing is off or full.
uint4* Renderer::probe_slot(int kernel, uint32_t grid) {
  if (probe_used_ >= probe_cap_) return nullptr;
  const uint32_t waves = grid * (kTBlock / 64);
  if (!d_probe_) {
    probe_waves_ = max_grid() * (kTBlock / 64);
    // entries are addressed with 32-bit offsets (meta's first entry) and the
    // buffer stays below 4 GB
    const uint64_t cap_max = (1ull << 28) / std::max<uint32_t>(probe_waves_, 1);
    probe_cap_ = (uint32_t)std::min<uint64_t>(probe_cap_, cap_max);
    if (hipMalloc(&d_probe_, sizeof(uint4) * (size_t)probe_waves_ * probe_cap_) != hipSuccess) {
      d_probe_ = nullptr;
      probe_cap_ = 0;
      return nullptr;
    }
  }
  if (waves > probe_waves_) return nullptr;
  const uint32_t first = probe_used_ * probe_waves_;
  probe_meta_.insert(probe_meta_.end(), {(uint32_t)kernel, (uint32_t)bound_, (uint32_t)cur_bounce_, waves, first});
  probe_used_++;
  return d_probe_ + first;
}

bool Renderer::probe_read(std::vector<uint32_t>& meta, std::vector<uint4>& rec, double& ticks_per_us,
                          std::string& err) {
  HIP_OK(hipDeviceSynchronize());
  int khz = 0;
  HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_ < 0 ? 0 : device_));
  ticks_per_us = khz / 1000.0;
  meta = probe_meta_;
  rec.assign((size_t)probe_used_ * probe_waves_, make_uint4(0, 0, 0, 0));
  if (probe_used_) HIP_OK(hipMemcpy(rec.data(), d_probe_, sizeof(uint4) * rec.size(), hipMemcpyDeviceToHost));
  probe_used_ = 0;
  probe_meta_.clear();
  return true;
}

// Traversal-stack entries per lane beyond the LDS slots (the spill area holds
// this many x grid x kTBlock: Stack::spill, stride = the launch's threads).
size_t Renderer::spill_slots() const {
  return (size_t)ds_.stack_cap > (size_t)kLdsSlots ? (size_t)ds_.stack_cap - kLdsSlots : 1;
}

// The most blocks a traversal launch on the bound lane may have: what its
// spill area holds. Every launch is clamped to it (a smaller persistent grid
// loops over more feed chunks, the same bits).
uint32_t Renderer::spill_grid() const {
  return (uint32_t)std::min<size_t>(spill_cap_ / (spill_slots() * kTBlock), 0xFFFFFFFFu);
}

// Lane l's spill area for grids of `grid` blocks (one-shot async grids).
bool Renderer::ensure_spill(int l, uint32_t grid, std::string& err) {
  PathSet& L = lanes_[l];
  const size_t need = spill_slots() * (size_t)grid * kTBlock;
  if (need <= L.spill_cap) return true;
  HIP_OK(hipStreamSynchronize(L.stream));
  if (L.lo) HIP_OK(hipStreamSynchronize(L.lo));
  if (L.spill) (void)hipFree(L.spill);
  L.spill = nullptr;
  L.spill_cap = 0;
  HIP_OK(hipMalloc(&L.spill, need * sizeof(uint2)));
  L.spill_cap = need;
  bind_lane(bound_);
  return true;
}

// The largest persistent traversal grid of any variant (spill and probe sizes).
uint32_t Renderer::max_grid() const {
  uint32_t g = 0;
  for (uint32_t x : grid_ext_) g = std::max(g, x);
  for (uint32_t x : grid_sh_) g = std::max(g, x);
  for (uint32_t x : grid_tr_) g = std::max(g, x);
  return g;
}

bool Renderer::size_grids(std::string& err) {
  int bpc = 0;
#define WPT_OCC(arr, idx, K)                                                      \
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, K, (int)kTBlock, 0)); \
  arr[idx] = (uint32_t)std::max(1, ncu_ * (bpc > 0 ? bpc : 1) * pct / 100);
  // The separate extend / shadow kernels (whole-frame batches, 4 concurrent
  // lanes) get persistent grids of half the resident capacity, so two lanes'
  // traversal kernels run side by side instead of one filling the GPU and the
  // next one's blocks starting only as its blocks drain (C3 +4.5 % with 4
  // lanes); the fused k_trace of small batches keeps full grids.
  // One-lane batches (wpt_set_lanes(1), tiny batches) use every resident
  // slot: [8 + v] (a half grid left half the GPU idle there).
  for (int full = 0; full < 2; full++) {
    const int pct = full ? 100 : grid_pct_;
    const int o = full ? kTravVariants : 0;
    WPT_OCC(grid_ext_, o + 0, (k_extend<false, false, 0>));
    WPT_OCC(grid_ext_, o + 1, (k_extend<true, false, 0>));
    WPT_OCC(grid_ext_, o + 2, (k_extend<false, true, 0>));
    WPT_OCC(grid_ext_, o + 3, (k_extend<true, true, 0>));
    WPT_OCC(grid_ext_, o + 4, (k_extend<false, false, 1>));
    WPT_OCC(grid_ext_, o + 5, (k_extend<true, false, 1>));
    WPT_OCC(grid_ext_, o + 6, (k_extend<false, true, 1>));
    WPT_OCC(grid_ext_, o + 7, (k_extend<true, true, 1>));
    WPT_OCC(grid_sh_, o + 0, (k_shadow<false, false, 0>));
    WPT_OCC(grid_sh_, o + 1, (k_shadow<true, false, 0>));
    WPT_OCC(grid_sh_, o + 2, (k_shadow<false, true, 0>));
    WPT_OCC(grid_sh_, o + 3, (k_shadow<true, true, 0>));
    WPT_OCC(grid_sh_, o + 4, (k_shadow<false, false, 1>));
    WPT_OCC(grid_sh_, o + 5, (k_shadow<true, false, 1>));
    WPT_OCC(grid_sh_, o + 6, (k_shadow<false, true, 1>));
    WPT_OCC(grid_sh_, o + 7, (k_shadow<true, true, 1>));
  }
  const int pct = trace_grid_pct_;
  WPT_OCC(grid_tr_, 0, (k_trace<false, false>));
  WPT_OCC(grid_tr_, 1, (k_trace<true, false>));
  WPT_OCC(grid_tr_, 2, (k_trace<false, true>));
  WPT_OCC(grid_tr_, 3, (k_trace<true, true>));
#undef WPT_OCC
  {
    // k_shade: 1024-lane blocks; the smallest occupancy of its variants
    int m = 1 << 30;
#define WPT_SHOCC(...)                                                                                    \
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, __VA_ARGS__, (int)kShadeBlock, 0)); \
  m = std::min(m, bpc);
    WPT_SHOCC(k_shade<true, false, 0>)
    WPT_SHOCC(k_shade<true, true, 0>)
    WPT_SHOCC(k_shade<true, true, 1>)
    WPT_SHOCC(k_shade<true, true, 2>)
    WPT_SHOCC(k_shade<false, false, 0>)
    WPT_SHOCC(k_shade<false, true, 0>)
    WPT_SHOCC(k_shade<false, true, 1>)
    WPT_SHOCC(k_shade<false, true, 2>)
#undef WPT_SHOCC
    grid_shade_ = (uint32_t)(ncu_ * std::max(m, 1));
  }
  // global spill area for stack entries beyond the LDS slots
  const uint32_t gmax = max_grid();
  // exact BVH2 stack <= BVH2 depth; fast BVH4 stack <= 3 pushes per level
  const size_t slots = spill_slots();
  const size_t need = slots * (size_t)gmax * kTBlock;
  // every lane that has a spill area (a lane gets one when a batch first
  // sizes it, ensure_lane: ADVICE r5, not all kMaxLanes up front), re-sized
  // for a deeper scene
  for (int i = 0; i < lanes_made_; i++) {
    PathSet& L = lanes_[i];
    if (L.spill && need > L.spill_cap) {
      HIP_OK(hipStreamSynchronize(L.stream));
      if (L.spill) (void)hipFree(L.spill);
      L.spill = nullptr;
      HIP_OK(hipMalloc(&L.spill, need * sizeof(uint2)));
      L.spill_cap = need;
    }
  }
  bind_lane(bound_);
  return true;
}

void Renderer::free_rounds() {
  void* bufs[] = {d_scan_sums_, d_mse_[0], d_mse_[1], d_gsums_, d_bmm_};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  for (HalfRounds& r : rounds_) {
    void* rb[] = {r.rc, r.rbase, r.gc, r.gbase};
    for (void* p : rb)
      if (p) (void)hipFree(p);
    r = HalfRounds();
  }
  for (float*& h : h_mse_)
    if (h) { (void)hipHostFree(h); h = nullptr; }
  void* dbufs[] = {d_s64_, d_eff_, d_need_, d_list_, d_fb_};
  for (void* p : dbufs)
    if (p) (void)hipFree(p);
  void* hbufs[] = {h_eff_, h_list_, h_fb_};
  for (void* p : hbufs)
    if (p) (void)hipHostFree(p);
  d_s64_ = nullptr;
  d_eff_ = nullptr;
  d_need_ = nullptr;
  d_list_ = nullptr;
  d_fb_ = nullptr;
  h_eff_ = nullptr;
  h_list_ = nullptr;
  h_fb_ = nullptr;
  d_scan_sums_ = nullptr;
  d_mse_[0] = d_mse_[1] = nullptr;
  d_gsums_ = nullptr;
  d_bmm_ = nullptr;
  round_cap_ = 0;
}

// Next sample round of screen half h (wpt_adaptive.h): an adaptive half's
// error estimate from the current image, then samples per pixel (the other
// half's pixels get none), prefix offsets and the round length.
// The walk's re-summed chunks: from the packed copy when k_sum_pack marked
// them (the list is ascending, as the walk asks), else copied on demand.
struct SumFetch {
  const uint32_t* list;  // count, then the marked chunks
  const float* fb;       // the first kSumFetch marked chunks' elements
  const float* dev;      // the errors on the device
  float* host;           // host scratch of the same layout
  hipStream_t stream;
  size_t n;              // elements (the last chunk may be short)
  uint32_t pos;
  bool ok;
  uint64_t fetched = 0;  // chunks copied on demand
  static const float* get(void* c, size_t j) {
    SumFetch& F = *(SumFetch*)c;
    const uint32_t cnt = F.list[0];
    while (F.pos < cnt && F.list[1 + F.pos] < j) F.pos++;
    if (F.pos < cnt && F.pos < kSumFetch && F.list[1 + F.pos] == j) return F.fb + (size_t)F.pos * kSumChunk;
    // not packed: this chunk alone, now
    F.fetched++;
    const size_t a = j * kSumChunk, len = std::min<size_t>(kSumChunk, F.n - a);
    F.ok = F.ok && hipMemcpyAsync(F.host + a, F.dev + a, sizeof(float) * len, hipMemcpyDeviceToHost, F.stream) ==
                       hipSuccess &&
           hipStreamSynchronize(F.stream) == hipSuccess;
    return F.host + j * kSumChunk;
  }
};

bool Renderer::plan_round(int h, std::string& err) {
  struct Tally {
    std::chrono::steady_clock::time_point t0;
    uint64_t& us;
    ~Tally() { us += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count(); }
  } tally{std::chrono::steady_clock::now(), stats_.plan_us};
  if (log_) WPT_LOGF("plan h=%d idx=%u\n", h, rounds_[h].idx);
  const uint32_t npix = (uint32_t)part_pix_.size();
  const uint32_t np = w_ * h_;
  if (round_cap_ != (uint64_t)npix + 1 || (nranks_ > 1 && !rounds_[0].gc)) {
    // (re)allocate the round buffers; the halves' positions and round counts
    // stay (a non-adaptive half may have run whole rounds without a plan)
    HalfRounds keep[2] = {rounds_[0], rounds_[1]};
    free_rounds();
    for (int k = 0; k < 2; k++) {
      rounds_[k].total = keep[k].total;
      rounds_[k].pos = keep[k].pos;
      rounds_[k].idx = keep[k].idx;
    }
    const uint32_t nb = (std::max(npix, np) + 1 + kScanChunk - 1) / kScanChunk;
    HIP_OK(hipMalloc(&d_scan_sums_, sizeof(uint32_t) * (nb + 1)));
    // per half: np errors, then the {min, max} keys k_mse reduces
    HIP_OK(hipMalloc(&d_mse_[0], sizeof(float) * (np + 2)));
    HIP_OK(hipMalloc(&d_mse_[1], sizeof(float) * (np + 2)));
    // per-tile {min, max} keys of k_mse_tiled (a half's tiles)
    HIP_OK(hipMalloc(&d_bmm_, sizeof(uint32_t) * 2 * ((w_ / kMseTile + 2) * (h_ / kMseTile + 1))));
    HIP_OK(hipHostMalloc(&h_mse_[0], sizeof(float) * (np + 2)));
    HIP_OK(hipHostMalloc(&h_mse_[1], sizeof(float) * (np + 2)));
    const size_t nch = ((size_t)np + kSumChunk - 1) / kSumChunk + 1;
    HIP_OK(hipMalloc(&d_s64_, sizeof(double) * nch));
    HIP_OK(hipMalloc(&d_eff_, sizeof(ChunkEff) * 2 * nch));
    HIP_OK(hipHostMalloc(&h_eff_, sizeof(ChunkEff) * 2 * nch));
    HIP_OK(hipMalloc(&d_need_, sizeof(uint32_t) * nch));
    HIP_OK(hipMalloc(&d_list_, sizeof(uint32_t) * (nch + 1)));
    HIP_OK(hipMalloc(&d_fb_, sizeof(float) * kSumFetch * kSumChunk));
    HIP_OK(hipHostMalloc(&h_list_, sizeof(uint32_t) * (nch + 1)));
    HIP_OK(hipHostMalloc(&h_fb_, sizeof(float) * kSumFetch * kSumChunk));
    for (HalfRounds& r : rounds_) {
      HIP_OK(hipMalloc(&r.rc, sizeof(uint32_t) * (npix + 1)));
      HIP_OK(hipMalloc(&r.rbase, sizeof(uint32_t) * (npix + 1)));
      if (nranks_ > 1) {
        HIP_OK(hipMalloc(&r.gc, sizeof(uint32_t) * (np + 1)));
        HIP_OK(hipMalloc(&r.gbase, sizeof(uint32_t) * (np + 1)));
      }
    }
    if (nranks_ > 1) {
      const uint32_t gb = (np + 1 + kScanChunk - 1) / kScanChunk;
      HIP_OK(hipMalloc(&d_gsums_, sizeof(uint32_t) * (gb + 1)));
    }
    round_cap_ = (uint64_t)npix + 1;
  }
  HalfRounds& R = rounds_[h];
  const uint32_t half = w_ / 2;
  RoundParams RP;
  for (int k = 0; k < 3; k++) RP.stats[k] = 0.0f;
  const bool estimate = adaptive_[h] && R.idx > 0;
  if (estimate && nranks_ > 1 && !exchange_frame(err)) return false;
  if (estimate) {
    // per-pixel error, min and max on the GPU; mse_sum on the host: the
    // reference's sequential f32 sum in raster order, in binade segments of
    // integer increments (wpt_seqsum.h) instead of one dependent add chain
    const uint32_t x0 = h ? half : 0u, x1 = h ? w_ : half;
    const uint32_t cnt = (x1 - x0) * h_;
    uint32_t* mm = reinterpret_cast<uint32_t*>(d_mse_[h] + np);
    const dim3 tiles((x1 - x0 + kMseTile - 1) / kMseTile, (h_ + kMseTile - 1) / kMseTile);
    // the errors' sum: chunk effects on the device, walked on the host; the
    // chunks the walk will likely re-sum come with them (k_sum_pack), any
    // other one it re-sums is fetched on demand (SumFetch)
    const uint32_t nch = (cnt + kSumChunk - 1) / kSumChunk;
    if (cnt) {
      k_mse_tiled<<<tiles, kBlock, 0, stream_>>>(d_acc_, d_cnt_, w_, h_, x0, x1, d_mse_[h], d_bmm_);
      k_mm_reduce<<<1, 1024, 0, stream_>>>(d_bmm_, tiles.x * tiles.y, mm);
      const uint32_t wb = (uint32_t)(((uint64_t)nch * 64u + kBlock - 1) / kBlock);
      k_sum_chunks<<<wb, kBlock, 0, stream_>>>(d_mse_[h], cnt, d_s64_);
      k_sum_scan<<<1, 256, 0, stream_>>>(d_s64_, nch);
      k_sum_eff<<<wb, kBlock, 0, stream_>>>(d_mse_[h], cnt, d_s64_, d_eff_, d_need_);
      k_sum_pack<<<1, 1024, 0, stream_>>>(d_mse_[h], cnt, nch, d_need_, d_list_, d_fb_);
      HIP_OK(hipMemcpyAsync(h_eff_, d_eff_, sizeof(ChunkEff) * 2 * nch, hipMemcpyDeviceToHost, stream_));
      HIP_OK(hipMemcpyAsync(h_list_, d_list_, sizeof(uint32_t) * (nch + 1), hipMemcpyDeviceToHost, stream_));
      HIP_OK(hipMemcpyAsync(h_fb_, d_fb_, sizeof(float) * kSumFetch * kSumChunk, hipMemcpyDeviceToHost, stream_));
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(h_mse_[h] + np, mm, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
    if (!host_wait_stream(stream_, err)) return false;  // the async lanes go on while the host waits
    // sampling_strategy.rs:138-141, bit for bit (wpt_seqsum.h)
    SumFetch F{h_list_, h_fb_, d_mse_[h], h_mse_[h], stream_, (size_t)cnt, 0u, true};
    const float sum = cnt ? seq_sum_walk_fetch(cnt, h_eff_, SumFetch::get, &F, &stats_.sum_resummed) : 0.0f;
    stats_.sum_fetched += F.fetched;
    stats_.sum_chunks += nch;
    if (!F.ok) { err = "error sum: chunk copy failed"; return false; }
    uint32_t keys[2];
    memcpy(keys, h_mse_[h] + np, sizeof keys);
    RP.stats[0] = sum;
    keys[0] = f_unkey(keys[0]);
    keys[1] = f_unkey(keys[1]);
    memcpy(&RP.stats[1], &keys[0], sizeof(float));  // min, max (:142-144)
    memcpy(&RP.stats[2], &keys[1], sizeof(float));
  }
  RP.W = w_; RP.H = h_; RP.half = half;
  RP.which = (uint32_t)h;
  RP.adaptive = adaptive_[h] ? 1u : 0u;
  RP.first = R.idx == 0 ? 1u : 0u;
  // one rank: the round over its pixels (= the frame); several ranks: the
  // global round over the whole frame, sliced per compute chunk (plan_slice)
  const bool global = nranks_ > 1;
  const uint32_t pn = global ? np : npix;
  uint32_t* rc = global ? R.gc : R.rc;
  uint32_t* rbase = global ? R.gbase : R.rbase;
  uint32_t* sums = global ? d_gsums_ : d_scan_sums_;
  RP.npix = pn;
  k_plan_round<<<blocks_for((uint64_t)pn + 1), kBlock, 0, stream_>>>(RP, nullptr, d_cnt_, d_mse_[0], d_mse_[1], rc,
                                                                     rbase, d_samp_);
  HIP_OK(hipGetLastError());
  const uint32_t n = pn + 1;
  const uint32_t nb = (n + kScanChunk - 1) / kScanChunk;
  k_scan_local<<<nb, kBlock, 0, stream_>>>(rc, n, sums);
  k_scan_sums<<<1, kBlock, 0, stream_>>>(sums, nb);
  k_scan_add<<<nb, kBlock, 0, stream_>>>(rc, n, sums);
  HIP_OK(hipGetLastError());
  // (a word of its own: the lanes' pinned counts may still hold the last
  // batch's, read at the next flush_counts)
  HIP_OK(hipMemcpyAsync(h_word_, rc + pn, sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  if (!host_wait_stream(stream_, err)) return false;
  R.total = h_word_[0];
  R.pos = 0;
  R.idx++;
  if (log_) WPT_LOGF("planned h=%d idx=%u total=%lu\n", h, R.idx, (unsigned long)R.total);
  return true;
}

bool Renderer::seq_sum_device(const float* v, uint64_t n, float& out, std::string& err) {
  // plan_round's path on host data: the same kernels, copies and walk
  if (n >= (1ull << 32)) { err = "too many elements"; return false; }
  const uint32_t cnt = (uint32_t)n, nch = (cnt + kSumChunk - 1) / kSumChunk;
  out = 0.0f;
  if (!cnt) return true;
  float *dv = nullptr, *dfb = nullptr;
  double* ds = nullptr;
  ChunkEff* de = nullptr;
  uint32_t *dn = nullptr, *dl = nullptr;
  std::vector<ChunkEff> he(2 * (size_t)nch);
  std::vector<uint32_t> hl(nch + 1);
  std::vector<float> hfb((size_t)kSumFetch * kSumChunk), scratch((size_t)nch * kSumChunk);
  bool ok = hipMalloc(&dv, sizeof(float) * (size_t)nch * kSumChunk) == hipSuccess &&
            hipMalloc(&ds, sizeof(double) * nch) == hipSuccess &&
            hipMalloc(&de, sizeof(ChunkEff) * 2 * nch) == hipSuccess &&
            hipMalloc(&dn, sizeof(uint32_t) * nch) == hipSuccess &&
            hipMalloc(&dl, sizeof(uint32_t) * (nch + 1)) == hipSuccess &&
            hipMalloc(&dfb, sizeof(float) * kSumFetch * kSumChunk) == hipSuccess;
  if (ok) {
    const uint32_t wb = (uint32_t)(((uint64_t)nch * 64u + kBlock - 1) / kBlock);
    ok = hipMemcpyAsync(dv, v, sizeof(float) * cnt, hipMemcpyHostToDevice, stream_) == hipSuccess;
    k_sum_chunks<<<wb, kBlock, 0, stream_>>>(dv, cnt, ds);
    k_sum_scan<<<1, 256, 0, stream_>>>(ds, nch);
    k_sum_eff<<<wb, kBlock, 0, stream_>>>(dv, cnt, ds, de, dn);
    k_sum_pack<<<1, 1024, 0, stream_>>>(dv, cnt, nch, dn, dl, dfb);
    ok = ok && hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(he.data(), de, sizeof(ChunkEff) * 2 * nch, hipMemcpyDeviceToHost, stream_) == hipSuccess &&
         hipMemcpyAsync(hl.data(), dl, sizeof(uint32_t) * (nch + 1), hipMemcpyDeviceToHost, stream_) == hipSuccess &&
         hipMemcpyAsync(hfb.data(), dfb, sizeof(float) * hfb.size(), hipMemcpyDeviceToHost, stream_) == hipSuccess &&
         hipStreamSynchronize(stream_) == hipSuccess;
    if (ok) {
      SumFetch F{hl.data(), hfb.data(), dv, scratch.data(), stream_, (size_t)cnt, 0u, true};
      out = seq_sum_walk_fetch(cnt, he.data(), SumFetch::get, &F);
      ok = F.ok;
    }
  }
  void* bufs[] = {dv, dfb, ds, de, dn, dl};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  if (!ok) { err = "device sum failed"; return false; }
  return true;
}

// Round boundary over several ranks: pack this rank's partition, let the
// caller's exchange all-gather every rank's, scatter them into the frame.
bool Renderer::exchange_frame(std::string& err) {
  if (!xfn_ || !xlocal_ || !xall_) { err = "adaptive sampling over several ranks needs wpt_set_exchange"; return false; }
  if (xslot_ < maxpart_) { err = "exchange slot smaller than the largest partition"; return false; }
  const uint32_t n = (uint32_t)part_pix_.size();
  if (n) {
    k_pack_exchange<<<blocks_for(n), kBlock, 0, stream_>>>(d_part_pix_, n, d_acc_, d_cnt_, xlocal_);
    HIP_OK(hipGetLastError());
  }
  HIP_OK(hipStreamSynchronize(stream_));
  if (xfn_(xuser_) != 0) { err = "frame exchange failed"; return false; }
  return unpack_ranks(xall_, xslot_, err);
}

// The other ranks' packed partitions (rank-major, `slot` float4 per rank, the
// wpt_copy_partition layout) scattered into this rank's frame.
bool Renderer::unpack_ranks(const float4* gathered, uint64_t slot, std::string& err) {
  if (nranks_ < 2) return true;
  if (slot < maxpart_) { err = "slot smaller than the largest partition"; return false; }
  // the index map is per maxpart_ entries, so unpack rank by rank
  for (uint32_t r = 0; r < nranks_; r++) {
    if (r == rank_) continue;
    k_unpack_exchange<<<blocks_for(maxpart_), kBlock, 0, stream_>>>(d_xidx_ + (size_t)r * maxpart_,
                                                                     (uint32_t)maxpart_, gathered + (size_t)r * slot,
                                                                     d_acc_, d_cnt_);
    HIP_OK(hipGetLastError());
  }
  HIP_OK(hipStreamSynchronize(stream_));
  return true;
}

// This rank's share of positions [a, b) of half h's global round: per own
// pixel the count and first sample index, scanned into the half's rc (the
// round mapping k_generate / k_accumulate_round read); `local` = paths to trace.
bool Renderer::plan_slice(int h, uint64_t a, uint64_t b, uint64_t& local, std::string& err) {
  HalfRounds& R = rounds_[h];
  const uint32_t npix = (uint32_t)part_pix_.size();
  k_plan_slice<<<blocks_for((uint64_t)npix + 1), kBlock, 0, stream_>>>(d_part_pix_, npix, R.gc, R.gbase, (uint32_t)a,
                                                                      (uint32_t)b, R.rc, R.rbase);
  HIP_OK(hipGetLastError());
  const uint32_t n = npix + 1;
  const uint32_t nb = (n + kScanChunk - 1) / kScanChunk;
  k_scan_local<<<nb, kBlock, 0, stream_>>>(R.rc, n, d_scan_sums_);
  k_scan_sums<<<1, kBlock, 0, stream_>>>(d_scan_sums_, nb);
  k_scan_add<<<nb, kBlock, 0, stream_>>>(R.rc, n, d_scan_sums_);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(h_word_, R.rc + npix, sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  local = h_word_[0];
  return true;
}

bool Renderer::fill_sampling_blue(std::string& err) {
  if (!d_samp_) return true;
  k_samp_reset<<<blocks_for((uint64_t)w_ * h_), kBlock, 0, stream_>>>(d_samp_, w_, h_, w_ / 2, 1u, 1u);
  HIP_OK(hipGetLastError());
  return true;
}

bool Renderer::sampling_rgba(uint8_t* out, std::string& err) {
  if (!d_samp_) { err = "no viewport"; return false; }
  HIP_OK(hipMemcpyAsync(out, d_samp_, 4 * (size_t)w_ * h_, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  return true;
}

void Renderer::free_photons() {
  if (d_oct_child_) (void)hipFree(d_oct_child_);
  if (d_oct_cum_) (void)hipFree(d_oct_cum_);
  if (d_oct_corners_) (void)hipFree(d_oct_corners_);
  d_oct_child_ = nullptr;
  d_oct_cum_ = nullptr;
  d_oct_corners_ = nullptr;
  ds_.oct_child = nullptr;
  ds_.oct_cum = nullptr;
  ds_.oct_corners = nullptr;
  ds_.oct_nodes = 0;
  ds_.oct_lds_words = 0;
  photons_ok_ = false;
}

// RenderInstance::compute's photon phase (tracer.rs:103-123, 126-152): shoot
// photons k = 0, 1, 2, ... (per-photon streams) in rounds of 2^20 on the GPU,
// insert the diffuse hits on the host in photon order until kPhotonsNeeded
// are stored (the photons of the last round past that point count as not
// shot), freeze the tree and upload it. A scene whose photons (almost) never
// reach a diffuse surface stops after 64 x kPhotonsNeeded shots with the
// photons it has (the reference would keep shooting, tracing no paths).
bool Renderer::build_photons(std::string& err) {
  batch_lanes_ = 1;  // lane 0 alone: full-capacity traversal grids
  if (photons_ok_) return true;
  free_photons();
  PhotonTree tree(ds_.num_lights);
  photons_shot_ = photons_stored_ = 0;
  if (ds_.num_lights > 0) {
    const uint32_t R = 1u << 20;
    if (!ensure_paths(R, err)) return false;
    std::vector<float4> hit(R);
    std::vector<uint32_t> lid(R);
    const bool prof = profiling_, cnt = counting_;
    profiling_ = counting_ = false;
    const uint64_t max_shots = 64ull * kPhotonsNeeded;
    bool ok = true;
    while (ok && tree.num_photons() < kPhotonsNeeded && photons_shot_ < max_shots) {
      const uint32_t k0 = (uint32_t)photons_shot_;
      k_photon_gen<<<blocks_for(R), kBlock, 0, stream_>>>(ds_, seed_, k0, R, p_ro_[0], p_rd_[0], p_thr_[0]);
      HIP_OK(hipGetLastError());
      h_counts_[0] = R;
      HIP_OK(hipMemcpyAsync(d_counts_, h_counts_, 4, hipMemcpyHostToDevice, stream_));
      ok = launch_extend(p_ro_[0], p_rd_[0], d_counts_, err);
      if (!ok) break;
      if (ds_.tri_only)
        k_photon_hit<true><<<blocks_for(R), kBlock, 0, stream_>>>(ds_, R, p_ro_[0], p_rd_[0], p_t_, p_id_, p_thr_[0], p_col_, p_pixel_);
      else
        k_photon_hit<false><<<blocks_for(R), kBlock, 0, stream_>>>(ds_, R, p_ro_[0], p_rd_[0], p_t_, p_id_, p_thr_[0], p_col_, p_pixel_);
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(hit.data(), p_col_, sizeof(float4) * R, hipMemcpyDeviceToHost, stream_));
      HIP_OK(hipMemcpyAsync(lid.data(), p_pixel_, sizeof(uint32_t) * R, hipMemcpyDeviceToHost, stream_));
      HIP_OK(hipStreamSynchronize(stream_));
      uint32_t used = R;
      for (uint32_t i = 0; i < R; i++) {
        if (lid[i] != 0xFFFFFFFFu) {
          tree.insert(lid[i], mk(hit[i].x, hit[i].y, hit[i].z), hit[i].w);
          if (tree.num_photons() >= kPhotonsNeeded) { used = i + 1; break; }
        }
      }
      photons_shot_ += used;
    }
    profiling_ = prof;
    counting_ = cnt;
    if (!ok) return false;
  }
  photons_stored_ = tree.num_photons();
  stats_.photon_rays += photons_shot_;
  stats_.photons += photons_stored_;
  tree.freeze(oct_child_, oct_cum_);
  HIP_OK(hipMalloc(&d_oct_child_, sizeof(uint32_t) * oct_child_.size()));
  HIP_OK(hipMemcpy(d_oct_child_, oct_child_.data(), sizeof(uint32_t) * oct_child_.size(), hipMemcpyHostToDevice));
  if (!oct_cum_.empty()) {
    HIP_OK(hipMalloc(&d_oct_cum_, sizeof(float) * oct_cum_.size()));
    HIP_OK(hipMemcpy(d_oct_cum_, oct_cum_.data(), sizeof(float) * oct_cum_.size(), hipMemcpyHostToDevice));
  }
  ds_.oct_child = d_oct_child_;
  ds_.oct_cum = d_oct_cum_;
  ds_.oct_nodes = (uint32_t)oct_child_.size();
  {
    // photon_sample's neighbour cells, per leaf and offset case (xo, yo, zo
    // = -1 / +1 per axis: bits 2, 1, 0 of the case): the walks oct_walk does
    // on the device, from the leaf's lattice index (depth <= kOctLattice)
    const size_t nn = oct_child_.size();
    std::vector<uint32_t> corners(64 * nn, 0u);
    auto walk = [&](uint32_t ix, uint32_t iy, uint32_t iz, int d) {
      uint32_t node = 0;
      for (int l = d - 1; l >= 0; l--) {
        const uint32_t c = oct_child_[node];
        if (c == 0u) break;
        node = c + (((ix >> l) & 1u) << 2) + (((iy >> l) & 1u) << 1) + ((iz >> l) & 1u);
      }
      return node;
    };
    struct Item {
      uint32_t node;
      int d;
      uint32_t kx, ky, kz;
    };
    std::vector<Item> todo{{0u, 0, 0u, 0u, 0u}};
    while (!todo.empty()) {
      const Item it = todo.back();
      todo.pop_back();
      const uint32_t c0 = oct_child_[it.node];
      if (c0 != 0u) {
        if (it.d < kOctLattice)
          for (uint32_t j = 0; j < 8; j++)
            todo.push_back({c0 + j, it.d + 1, 2 * it.kx + ((j >> 2) & 1u), 2 * it.ky + ((j >> 1) & 1u),
                            2 * it.kz + (j & 1u)});
        continue;
      }
      const int64_t last = ((int64_t)1 << it.d) - 1;
      auto adj = [&](uint32_t k, int off) {
        const int64_t a = (int64_t)k + off;
        return (uint32_t)(a < 0 ? 0 : (a > last ? last : a));
      };
      for (uint32_t oc = 0; oc < 8; oc++) {
        const uint32_t ax = adj(it.kx, (oc & 4u) ? 1 : -1), ay = adj(it.ky, (oc & 2u) ? 1 : -1),
                       az = adj(it.kz, (oc & 1u) ? 1 : -1);
        uint32_t* row = corners.data() + 64 * (size_t)it.node + 8 * oc;
        row[0] = it.node;
        for (uint32_t c = 1; c < 8; c++)
          row[c] = walk((c & 4u) ? ax : it.kx, (c & 2u) ? ay : it.ky, (c & 1u) ? az : it.kz, it.d);
      }
    }
    HIP_OK(hipMalloc(&d_oct_corners_, sizeof(uint32_t) * corners.size()));
    HIP_OK(hipMemcpy(d_oct_corners_, corners.data(), sizeof(uint32_t) * corners.size(), hipMemcpyHostToDevice));
    ds_.oct_corners = d_oct_corners_;
  }
  {
    // k_shade's LDS copy of the tree (dynamic shared memory, 6 blocks per CU
    // must still fit): child and CDFs, else the child array alone, else none
    const size_t nodes = oct_child_.size(), all = nodes + oct_cum_.size();
    ds_.oct_lds_words = all <= kOctLdsWords ? (uint32_t)all : nodes <= kOctLdsWords ? (uint32_t)nodes : 0u;
  }
  photons_ok_ = true;
  return true;
}

bool Renderer::photon_tree(std::vector<uint32_t>& child, std::vector<float>& cum, uint64_t& shot, uint64_t& stored,
                           std::string& err) {
  if (!scene_ok_) { err = "no scene"; return false; }
  if (!build_photons(err)) return false;
  child = oct_child_;
  cum = oct_cum_;
  shot = photons_shot_;
  stored = photons_stored_;
  return true;
}

bool Renderer::trace_rays(size_t n, const float* rays, float* t_out, int32_t* id_out, std::string& err) {
  batch_lanes_ = 1;  // lane 0 alone: full-capacity traversal grids
  if (!scene_ok_) { err = "no scene"; return false; }
  if (n == 0) return true;
  if (n > 0xFFFFFFFFull) { err = "too many rays"; return false; }
  if (!ensure_paths(n, err)) return false;
  std::vector<float4> o(n), d(n);
  for (size_t i = 0; i < n; i++) {
    const float* r = rays + 6 * i;
    o[i] = make_float4(r[0], r[1], r[2], 0.0f);
    d[i] = make_float4(r[3], r[4], r[5], 0.0f);
  }
  const uint32_t nn = (uint32_t)n;
  HIP_OK(hipMemcpyAsync(p_ro_[0], o.data(), 16 * n, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipMemcpyAsync(p_rd_[0], d.data(), 16 * n, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipMemcpyAsync(d_counts_, &nn, 4, hipMemcpyHostToDevice, stream_));
  const bool prof = profiling_;
  profiling_ = false;
  const bool ok = launch_extend(p_ro_[0], p_rd_[0], d_counts_, err);
  profiling_ = prof;
  if (!ok) return false;
  HIP_OK(hipMemcpyAsync(t_out, p_t_, 4 * n, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipMemcpyAsync(id_out, p_id_, 4 * n, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  return true;
}

// Parity hook: the production shadow kernel on caller-given (p, q, light);
// the shadow ray is formed as Scene::shadow_ray does (scene.rs:105-108).
bool Renderer::shadow_rays(size_t n, const float* pq, const int32_t* light, uint8_t* occ, std::string& err) {
  batch_lanes_ = 1;  // lane 0 alone: full-capacity traversal grids
  if (!scene_ok_) { err = "no scene"; return false; }
  if (n == 0) return true;
  if (n > 0xFFFFFFFFull) { err = "too many rays"; return false; }
  for (size_t i = 0; i < n; i++)
    if (light[i] < (int32_t)ds_.num_inf || light[i] >= (int32_t)ds_.num_shapes) { err = "light id out of range"; return false; }
  if (!ensure_paths(n, err)) return false;
  std::vector<float4> o(n), d(n);
  for (size_t i = 0; i < n; i++) {
    const float* r = pq + 6 * i;
    const V3 p = mk(r[0], r[1], r[2]), q = mk(r[3], r[4], r[5]);
    V3 dir = sub(q, p);
    const float dl = len(dir);
    dir = divs(dir, dl);
    const V3 org = add(p, scale(dir, kEpsilon));
    o[i] = make_float4(org.x, org.y, org.z, dl);
    d[i] = make_float4(dir.x, dir.y, dir.z, u2f((uint32_t)light[i]));
  }
  uint8_t* dq = nullptr;
  HIP_OK(hipMalloc(&dq, n));
  const uint32_t nn = (uint32_t)n;
  HIP_OK(hipMemcpyAsync(s_o_, o.data(), 16 * n, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipMemcpyAsync(s_d_, d.data(), 16 * n, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipMemcpyAsync(d_counts_, &nn, 4, hipMemcpyHostToDevice, stream_));
  const bool prof = profiling_;
  profiling_ = false;
  const bool ok = launch_shadow(d_counts_, dq, err);
  profiling_ = prof;
  if (ok) {
    HIP_OK(hipMemcpyAsync(occ, dq, n, hipMemcpyDeviceToHost, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
  }
  (void)hipFree(dq);
  return ok;
}

}  // namespace wpt
