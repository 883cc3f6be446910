// wpt_math.h — f32 math of the path-tracing core, compiled for both the host
// (scene build, BVH build) and gfx950 (kernels).
//
// Every operation restates the reference's exact f32 op order so that GPU
// results are bitwise those of the reference semantics:
//   Vec3 ops          src/math/vec3.rs:6-190
//   orthogonal        src/math/vec3.rs:37-54
//   rot_x / rot_y     src/math/vec3.rs:95-119
//   xorshift32 Rng    src/rng.rs:19-47
//   Color3 clamping   src/graphics/color3.rs:32-38
// Build flags: -ffp-contract=off (no FMA contraction), no fast-math,
// correctly-rounded f32 '/' and sqrt (HIP default), IEEE min/max.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define WPT_HD __host__ __device__ __forceinline__
#else
#define WPT_HD inline
#endif

namespace wpt {

static constexpr float kEpsilon = 0.0002f;            // src/math/mod.rs:11
static constexpr float kPi = 3.14159274101257324f;    // std::f32::consts::PI
static constexpr float kTriSlack = 0.1f * kEpsilon;   // triangle.rs:44,58

struct V3 {
  float x, y, z;
};
WPT_HD V3 mk(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
WPT_HD V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
WPT_HD V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
WPT_HD V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
WPT_HD V3 scale(V3 a, float m) { return mk(m * a.x, m * a.y, m * a.z); }       // Vec3*f32 and f32*Vec3
WPT_HD V3 mulv(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
WPT_HD V3 divs(V3 a, float d) { return mk(a.x / d, a.y / d, a.z / d); }
WPT_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
WPT_HD float len(V3 a) { return sqrtf(dot(a, a)); }
WPT_HD V3 normalize(V3 a) { return scale(a, 1.0f / len(a)); }
WPT_HD V3 cross(V3 s, V3 t) {
  return mk(s.y * t.z - s.z * t.y, s.z * t.x - s.x * t.z, s.x * t.y - s.y * t.x);
}
WPT_HD V3 orthogonal(V3 s) {
  if (fabsf(s.z) > 0.1f) {
    return normalize(mk(1.0f, 1.0f, -(s.x * 1.0f + s.y * 1.0f) / s.z));
  } else if (fabsf(s.x) > 0.1f) {
    return normalize(mk(-(s.y * 1.0f + s.z * 1.0f) / s.x, 1.0f, 1.0f));
  } else {
    return normalize(mk(1.0f, -(s.x * 1.0f + s.z * 1.0f) / s.y, 1.0f));
  }
}
WPT_HD float clamp01(float x) { return fminf(1.0f, fmaxf(0.0f, x)); }

// ---------------------------------------------------------------------------
// sin/cos: the reference's `f32::sin/cos` lower to the `libm` crate (a port of
// musl's sinf/cosf) on wasm32. Restated from musl's published algorithm
// (double-precision __sindf/__cosdf kernels, quadrant branches, medium
// __rem_pio2f reduction) so host and device produce identical bits.
// ---------------------------------------------------------------------------
WPT_HD double k_sindf(double x) {
  const double S1 = -0x15555554cbac77.0p-55, S2 = 0x111110896efbb2.0p-59,
               S3 = -0x1a00f9e2cae774.0p-65, S4 = 0x16cd878c3b46a7.0p-71;
  double z = x * x, w = z * z, r = S3 + z * S4, s = z * x;
  return (x + s * (S1 + z * S2)) + s * w * r;
}
WPT_HD double k_cosdf(double x) {
  const double C0 = -0x1ffffffd0c5e81.0p-54, C1 = 0x155553e1053a42.0p-57,
               C2 = -0x16c087e80f1e27.0p-62, C3 = 0x199342e0ee5069.0p-68;
  double z = x * x, w = z * z, r = C2 + z * C3;
  return ((1.0 + z * C0) + w * C1) + (w * z) * r;
}
WPT_HD int rem_pio2f(float x, double* y) {
  const double toint = 1.5 / 2.220446049250313080847e-16, pio4 = 0x1.921fb6p-1,
               invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079631090164184570e+00,
               pio2_1t = 1.58932547735281966916e-08;
  double fn = (double)x * invpio2 + toint - toint;
  int n = (int)fn;
  *y = x - fn * pio2_1 - fn * pio2_1t;
  if (*y < -pio4) { n--; fn--; *y = x - fn * pio2_1 - fn * pio2_1t; }
  else if (*y > pio4) { n++; fn++; *y = x - fn * pio2_1 - fn * pio2_1t; }
  return n;
}
WPT_HD uint32_t f2u(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
WPT_HD float u2f(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }

WPT_HD float msin(float x) {
  const double p1 = 1.57079632679489661923, p2 = 2 * p1, p3 = 3 * p1, p4 = 4 * p1;
  double xd = (double)x;
  uint32_t ix = f2u(x);
  bool sign = (ix >> 31) != 0;
  ix &= 0x7fffffffu;
  if (ix <= 0x3f490fdau) {
    if (ix < 0x39800000u) return x;
    return (float)k_sindf(xd);
  }
  if (ix <= 0x407b53d1u) {
    if (ix <= 0x4016cbe3u) return sign ? -(float)k_cosdf(xd + p1) : (float)k_cosdf(xd - p1);
    return (float)k_sindf(sign ? -(xd + p2) : -(xd - p2));
  }
  if (ix <= 0x40e231d5u) {
    if (ix <= 0x40afeddfu) return sign ? (float)k_cosdf(xd + p3) : -(float)k_cosdf(xd - p3);
    return (float)k_sindf(sign ? xd + p4 : xd - p4);
  }
  if (ix >= 0x7f800000u) return x - x;
  double y;
  int n = rem_pio2f(x, &y);
  switch (n & 3) {
    case 0: return (float)k_sindf(y);
    case 1: return (float)k_cosdf(y);
    case 2: return (float)k_sindf(-y);
    default: return -(float)k_cosdf(y);
  }
}
WPT_HD float mcos(float x) {
  const double p1 = 1.57079632679489661923, p2 = 2 * p1, p3 = 3 * p1, p4 = 4 * p1;
  double xd = (double)x;
  uint32_t ix = f2u(x);
  bool sign = (ix >> 31) != 0;
  ix &= 0x7fffffffu;
  if (ix <= 0x3f490fdau) {
    if (ix < 0x39800000u) return 1.0f;
    return (float)k_cosdf(xd);
  }
  if (ix <= 0x407b53d1u) {
    if (ix > 0x4016cbe3u) return -(float)k_cosdf(sign ? xd + p2 : xd - p2);
    return sign ? (float)k_sindf(xd + p1) : (float)k_sindf(p1 - xd);
  }
  if (ix <= 0x40e231d5u) {
    if (ix > 0x40afeddfu) return (float)k_cosdf(sign ? xd + p4 : xd - p4);
    return sign ? (float)k_sindf(-xd - p3) : (float)k_sindf(xd - p3);
  }
  if (ix >= 0x7f800000u) return x - x;
  double y;
  int n = rem_pio2f(x, &y);
  switch (n & 3) {
    case 0: return (float)k_cosdf(y);
    case 1: return (float)k_sindf(-y);
    case 2: return -(float)k_cosdf(y);
    default: return (float)k_sindf(y);
  }
}

// ---------------------------------------------------------------------------
// xorshift32 (rng.rs:40-47) and next() (rng.rs:19-21).
// ---------------------------------------------------------------------------
WPT_HD uint32_t xs_next_u32(uint32_t& s) {
  uint32_t x = s;
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  s = x;
  return x;
}
WPT_HD float xs_next(uint32_t& s) { return (float)xs_next_u32(s) * (1.0f / (float)0xFFFFFFFFu); }
// rng.rs:25-38 for low = 0 (draws nothing when high == 1)
WPT_HD uint32_t xs_next_in_range(uint32_t& s, uint32_t high) {
  if (high <= 1u) return 0u;
  float f = xs_next(s);
  if (f == 1.0f) return high - 1u;
  float v = floorf(f * (float)high);
  return (v != v || v <= 0.0f) ? 0u : (uint32_t)v;
}

// Per-path stream seed (build-defined).
WPT_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu;
  h ^= h >> 13; h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
WPT_HD uint32_t path_seed(uint32_t frame_seed, uint32_t pixel, uint32_t sample) {
  uint32_t h = fmix32(frame_seed ^ 0x9e3779b9u);
  h = fmix32(h ^ pixel);
  h = fmix32(h ^ (sample * 0x27d4eb2fu + 0x165667b1u));
  return h == 0u ? 0x6d2b79f5u : h;
}
// Stream of photon k (PNEE preprocessing, tracer.rs:126-152): a separate
// domain of the same hash (build-defined, like path_seed).
WPT_HD uint32_t photon_seed(uint32_t frame_seed, uint32_t k) {
  return path_seed(frame_seed ^ 0x50484f54u, k, 0xffffffffu);
}

}  // namespace wpt
