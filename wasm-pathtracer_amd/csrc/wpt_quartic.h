// wpt_quartic.h — Torus::trace (src/graphics/primitives/torus.rs:56-127) in
// f64, host and device.
//
// The reference solves the torus quartic with `roots 0.0.4`
// find_roots_quartic (a crates.io dependency absent from the reference tree;
// parity UNPINNED). It is restated here from the crate's
// published algorithm: normalise, depress (x = y - a3/4), Ferrari with the
// largest root of the resolvent cubic (Cardano / trigonometric form), and the
// cancellation-avoiding quadratic formula; root sets are kept sorted without
// duplicates (Roots::add_new_root). The reference is a WASM build, where
// Rust's f64 cbrt / acos / cos come from the musl port (compiler-builtins
// libm), so those are restated from musl (FreeBSD msun) as well: the GPU and
// the oracle then compute the same bits.
#pragma once
#include <stdint.h>
#include <string.h>

#include "wpt_math.h"

namespace wpt {

WPT_HD uint64_t d2u(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
WPT_HD double u2d(uint64_t u) {
  double x;
  memcpy(&x, &u, 8);
  return x;
}

// musl src/math/cbrt.c
WPT_HD double m64_cbrt(double x) {
  const uint32_t B1 = 715094163, B2 = 696219795;
  const double P0 = 1.87595182427177009643, P1 = -1.88497979543377169875, P2 = 1.621429720105354466140,
               P3 = -0.758397934778766047437, P4 = 0.145996192886612446982;
  uint64_t ui = d2u(x);
  uint32_t hx = (uint32_t)(ui >> 32) & 0x7fffffffu;
  if (hx >= 0x7ff00000u) return x + x;
  if (hx < 0x00100000u) {
    ui = d2u(x * 0x1p54);
    hx = (uint32_t)(ui >> 32) & 0x7fffffffu;
    if (hx == 0) return x;
    hx = hx / 3 + B2;
  } else {
    hx = hx / 3 + B1;
  }
  ui &= 1ull << 63;
  ui |= (uint64_t)hx << 32;
  double t = u2d(ui);
  double r = (t * t) * (t / x);
  t = t * ((P0 + r * (P1 + r * P2)) + ((r * r) * r) * (P3 + r * P4));
  ui = d2u(t);
  ui = (ui + 0x80000000ull) & 0xffffffffc0000000ull;
  t = u2d(ui);
  const double s = t * t;
  r = x / s;
  const double w = t + t;
  r = (r - t) / (w + r);
  return t + t * r;
}

// musl src/math/__cos.c, __sin.c
WPT_HD double m64_kcos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
               C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double z = x * x;
  double w = z * z;
  const double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  const double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}
WPT_HD double m64_ksin(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
               S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double z = x * x;
  const double w = z * z;
  const double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  const double v = z * x;
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

// musl src/math/__rem_pio2.c for |x| < 2^20 * pi/2 (the cubic's angles are
// within [-pi, pi]); larger arguments return n = 0, y = NaN.
WPT_HD int m64_rem_pio2(double x, double* y) {
  const double toint = 1.5 / 2.220446049250313080847e-16, pio4 = 0x1.921fb54442d18p-1,
               invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
               pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
               pio2_3t = 8.47842766036889956997e-32;
  const uint64_t ui = d2u(x);
  const int sign = (int)(ui >> 63);
  const uint32_t ix = (uint32_t)(ui >> 32) & 0x7fffffffu;
  double z, w, t, r, fn;
  int n;
  if (ix <= 0x400f6a7au) {
    if ((ix & 0xfffffu) == 0x921fbu) goto medium;
    if (ix <= 0x4002d97cu) {
      if (!sign) {
        z = x - pio2_1;
        y[0] = z - pio2_1t;
        y[1] = (z - y[0]) - pio2_1t;
        return 1;
      }
      z = x + pio2_1;
      y[0] = z + pio2_1t;
      y[1] = (z - y[0]) + pio2_1t;
      return -1;
    }
    if (!sign) {
      z = x - 2 * pio2_1;
      y[0] = z - 2 * pio2_1t;
      y[1] = (z - y[0]) - 2 * pio2_1t;
      return 2;
    }
    z = x + 2 * pio2_1;
    y[0] = z + 2 * pio2_1t;
    y[1] = (z - y[0]) + 2 * pio2_1t;
    return -2;
  }
  if (ix <= 0x401c463bu) {
    if (ix <= 0x4015fdbcu) {
      if (ix == 0x4012d97cu) goto medium;
      if (!sign) {
        z = x - 3 * pio2_1;
        y[0] = z - 3 * pio2_1t;
        y[1] = (z - y[0]) - 3 * pio2_1t;
        return 3;
      }
      z = x + 3 * pio2_1;
      y[0] = z + 3 * pio2_1t;
      y[1] = (z - y[0]) + 3 * pio2_1t;
      return -3;
    }
    if (ix == 0x401921fbu) goto medium;
    if (!sign) {
      z = x - 4 * pio2_1;
      y[0] = z - 4 * pio2_1t;
      y[1] = (z - y[0]) - 4 * pio2_1t;
      return 4;
    }
    z = x + 4 * pio2_1;
    y[0] = z + 4 * pio2_1t;
    y[1] = (z - y[0]) + 4 * pio2_1t;
    return -4;
  }
  if (ix >= 0x413921fbu) {
    y[0] = y[1] = x - x + __builtin_nan("");
    return 0;
  }
medium:
  fn = x * invpio2 + toint - toint;
  n = (int32_t)fn;
  r = x - fn * pio2_1;
  w = fn * pio2_1t;
  if (r - w < -pio4) {
    n--;
    fn--;
    r = x - fn * pio2_1;
    w = fn * pio2_1t;
  } else if (r - w > pio4) {
    n++;
    fn++;
    r = x - fn * pio2_1;
    w = fn * pio2_1t;
  }
  y[0] = r - w;
  {
    const int ex = (int)(ix >> 20);
    int ey = (int)((d2u(y[0]) >> 52) & 0x7ff);
    if (ex - ey > 16) {
      t = r;
      w = fn * pio2_2;
      r = t - w;
      w = fn * pio2_2t - ((t - r) - w);
      y[0] = r - w;
      ey = (int)((d2u(y[0]) >> 52) & 0x7ff);
      if (ex - ey > 49) {
        t = r;
        w = fn * pio2_3;
        r = t - w;
        w = fn * pio2_3t - ((t - r) - w);
        y[0] = r - w;
      }
    }
  }
  y[1] = (r - y[0]) - w;
  return n;
}

// musl src/math/cos.c
WPT_HD double m64_cos(double x) {
  const uint32_t ix = (uint32_t)(d2u(x) >> 32) & 0x7fffffffu;
  if (ix <= 0x3fe921fbu) {
    if (ix < 0x3e46a09eu) return 1.0;
    return m64_kcos(x, 0);
  }
  if (ix >= 0x7ff00000u) return x - x;
  double y[2];
  const unsigned n = (unsigned)m64_rem_pio2(x, y);
  switch (n & 3u) {
    case 0: return m64_kcos(y[0], y[1]);
    case 1: return -m64_ksin(y[0], y[1], 1);
    case 2: return -m64_kcos(y[0], y[1]);
    default: return m64_ksin(y[0], y[1], 1);
  }
}

// musl src/math/acos.c
WPT_HD double m64_acos_R(double z) {
  const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01, pS2 = 2.01212532134862925881e-01,
               pS3 = -4.00555345006794114027e-02, pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
               qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00, qS3 = -6.88283971605453293030e-01,
               qS4 = 7.70381505559019352791e-02;
  const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  return p / q;
}
WPT_HD double m64_acos(double x) {
  const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
  const uint64_t ui = d2u(x);
  const uint32_t hx = (uint32_t)(ui >> 32), ix = hx & 0x7fffffffu;
  if (ix >= 0x3ff00000u) {
    const uint32_t lx = (uint32_t)ui;
    if (((ix - 0x3ff00000u) | lx) == 0) {
      if (hx >> 31) return 2 * pio2_hi + 0x1p-120;
      return 0;
    }
    return 0 / (x - x);
  }
  if (ix < 0x3fe00000u) {
    if (ix <= 0x3c600000u) return pio2_hi + 0x1p-120;
    return pio2_hi - (x - (pio2_lo - x * m64_acos_R(x * x)));
  }
  if (hx >> 31) {
    const double z = (1.0 + x) * 0.5;
    const double s = sqrt(z);
    const double w = m64_acos_R(z) * s - pio2_lo;
    return 2 * (pio2_hi - (s + w));
  }
  const double z = (1.0 - x) * 0.5;
  const double s = sqrt(z);
  const double df = u2d(d2u(s) & 0xffffffff00000000ull);
  const double c = (z - df * df) / (s + df);
  const double w = m64_acos_R(z) * s + c;
  return 2 * (df + w);
}

// roots::Roots<f64>: an ascending set of at most 4 roots (add_new_root keeps
// it sorted and drops duplicates).
// Every access below uses a constant index (selects, unrolled loops), so the
// set stays in registers; a loop with a variable index put it, and the
// solver's temporaries, in per-lane scratch memory (128 B in torus_hit).
struct Roots4 {
  double r[4] = {0.0, 0.0, 0.0, 0.0};  // defined even where unused: the selects read every slot
  int n = 0;
  // the element at a variable index i < n
  WPT_HD double at(int i) const { return i == 0 ? r[0] : i == 1 ? r[1] : i == 2 ? r[2] : r[3]; }
  WPT_HD void add(double x) {
    // the reference loop: scan while r[i] <= x (not greater), returning on an
    // equal element, and insert before the first greater one
    int pos = n;
    if (n > 3 && r[3] > x) pos = 3;
    if (n > 2 && r[2] > x) pos = 2;
    if (n > 1 && r[1] > x) pos = 1;
    if (n > 0 && r[0] > x) pos = 0;
    const bool dup = (pos > 0 && r[0] == x) || (pos > 1 && r[1] == x) || (pos > 2 && r[2] == x) ||
                     (pos > 3 && r[3] == x);
    if (dup || n == 4) return;
    const double r3 = pos == 3 ? x : (pos < 3 ? r[2] : r[3]);
    const double r2 = pos == 2 ? x : (pos < 2 ? r[1] : r[2]);
    const double r1 = pos == 1 ? x : (pos < 1 ? r[0] : r[1]);
    const double r0 = pos == 0 ? x : r[0];
    r[0] = r0;
    r[1] = r1;
    r[2] = r2;
    r[3] = r3;
    n++;
  }
};

// roots::find_roots_linear / find_roots_quadratic
WPT_HD Roots4 q_linear(double a1, double a0) {
  Roots4 o;
  if (a1 == 0.0) {
    if (a0 == 0.0) o.add(0.0);  // Roots::One([0]) for the identity
  } else {
    o.add(-a0 / a1);
  }
  return o;
}
WPT_HD Roots4 q_quadratic(double a2, double a1, double a0) {
  if (a2 == 0.0) return q_linear(a1, a0);
  Roots4 o;
  const double disc = a1 * a1 - 4.0 * a2 * a0;
  if (disc < 0.0) return o;
  const double a2x2 = 2.0 * a2;
  if (disc == 0.0) {
    o.add(-a1 / a2x2);
    return o;
  }
  const double sq = sqrt(disc);
  double same, diff;
  if (a1 < 0.0) { same = -a1 + sq; diff = -a1 - sq; }
  else { same = -a1 - sq; diff = -a1 + sq; }
  double x1, x2;
  if (fabs(same) > fabs(a2x2)) {
    const double a0x2 = 2.0 * a0;
    if (fabs(diff) > fabs(a2x2)) { x1 = a0x2 / same; x2 = a0x2 / diff; }
    else { x1 = a0x2 / same; x2 = same / a2x2; }
  } else {
    x1 = diff / a2x2;
    x2 = same / a2x2;
  }
  if (x1 < x2) { o.add(x1); o.add(x2); }
  else { o.add(x2); o.add(x1); }
  return o;
}
// roots::find_roots_biquadratic
WPT_HD Roots4 q_biquadratic(double a4, double a2, double a0) {
  if (a4 == 0.0) return q_quadratic(a2, 0.0, a0);
  Roots4 o;
  const Roots4 q = q_quadratic(a4, a2, a0);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i >= q.n) break;
    const double x = q.r[i];
    if (x > 0.0) {
      const double sx = sqrt(x);
      o.add(-sx);
      o.add(sx);
    } else if (x == 0.0) {
      o.add(0.0);
    }
  }
  return o;
}
// roots::find_roots_cubic_normalized: x^3 + a2 x^2 + a1 x + a0
WPT_HD Roots4 q_cubic_normalized(double a2, double a1, double a0) {
  const double two_third_pi = 2.0943951023931953;
  const double q = (3.0 * a1 - a2 * a2) / 9.0;
  const double r = (9.0 * a2 * a1 - 27.0 * a0 - 2.0 * a2 * a2 * a2) / 54.0;
  const double q3 = q * q * q;
  const double d = q3 + r * r;
  const double a2_div_3 = a2 / 3.0;
  Roots4 o;
  if (d < 0.0) {
    const double phi_3 = m64_acos(r / sqrt(-q3)) / 3.0;
    const double sqrt_q_2 = 2.0 * sqrt(-q);
    o.add(sqrt_q_2 * m64_cos(phi_3) - a2_div_3);
    o.add(sqrt_q_2 * m64_cos(phi_3 - two_third_pi) - a2_div_3);
    o.add(sqrt_q_2 * m64_cos(phi_3 + two_third_pi) - a2_div_3);
  } else {
    const double sqrt_d = sqrt(d);
    const double s = m64_cbrt(r + sqrt_d);
    const double t = m64_cbrt(r - sqrt_d);
    if (s == t) {
      if (s + t == 0.0) {
        o.add(s + t - a2_div_3);
      } else {
        o.add(s + t - a2_div_3);
        o.add(-(s + t) / 2.0 - a2_div_3);
      }
    } else {
      o.add(s + t - a2_div_3);
    }
  }
  return o;
}
// roots::find_roots_cubic_depressed: x^3 + a1 x + a0
WPT_HD Roots4 q_cubic_depressed(double a1, double a0) {
  if (a1 == 0.0) {
    Roots4 o;
    o.add(-m64_cbrt(a0));
    return o;
  }
  if (a0 == 0.0) {
    Roots4 o = q_quadratic(1.0, 0.0, a1);
    o.add(0.0);
    return o;
  }
  return q_cubic_normalized(0.0, a1, a0);
}
// roots::find_roots_cubic
WPT_HD Roots4 q_cubic(double a3, double a2, double a1, double a0) {
  if (a3 == 0.0) return q_quadratic(a2, a1, a0);
  if (a2 == 0.0) return q_cubic_depressed(a1 / a3, a0 / a3);
  if (a3 == 1.0) return q_cubic_normalized(a2, a1, a0);
  const double d = 18.0 * a3 * a2 * a1 * a0 - 4.0 * a2 * a2 * a2 * a0 + a2 * a2 * a1 * a1 -
                   4.0 * a3 * a1 * a1 * a1 - 27.0 * a3 * a3 * a0 * a0;
  const double d0 = a2 * a2 - 3.0 * a3 * a1;
  if (d == 0.0) {
    Roots4 o;
    if (d0 == 0.0) {
      o.add(-a2 / (a3 * 3.0));
    } else {
      o.add((9.0 * a3 * a0 - a2 * a1) / (d0 * 2.0));
      o.add((4.0 * a3 * a2 * a1 - 9.0 * a3 * a3 * a0 - a2 * a2 * a2) / (a3 * d0));
    }
    return o;
  }
  return q_cubic_normalized(a2 / a3, a1 / a3, a0 / a3);
}
// roots::find_roots_quartic_depressed: x^4 + a2 x^2 + a1 x + a0 (Ferrari,
// largest root of the resolvent cubic)
WPT_HD Roots4 q_quartic_depressed(double a2, double a1, double a0) {
  if (a1 == 0.0) return q_biquadratic(1.0, a2, a0);
  if (a0 == 0.0) {
    Roots4 o = q_cubic_normalized(0.0, a2, a1);
    o.add(0.0);
    return o;
  }
  const double a2_pow_2 = a2 * a2;
  const double a1_div_2 = a1 / 2.0;
  const double b2 = a2 * 5.0 / 2.0;
  const double b1 = 2.0 * a2_pow_2 - a0;
  const double b0 = (a2_pow_2 * a2 - a2 * a0 - a1_div_2 * a1_div_2) / 2.0;
  const Roots4 res = q_cubic_normalized(b2, b1, b0);
  Roots4 o;
  if (res.n == 0) return o;
  const double y = res.at(res.n - 1);
  const double a2_plus_2y = a2 + 2.0 * y;
  if (a2_plus_2y > 0.0) {
    const double sq = sqrt(a2_plus_2y);
    const double q0a = a2 + y - a1_div_2 / sq;
    const double q0b = a2 + y + a1_div_2 / sq;
    o = q_quadratic(1.0, sq, q0a);
    const Roots4 o2 = q_quadratic(1.0, -sq, q0b);
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (i < o2.n) o.add(o2.r[i]);
  }
  return o;
}
// roots::find_roots_quartic: a4 x^4 + a3 x^3 + a2 x^2 + a1 x + a0
WPT_HD Roots4 q_quartic(double a4, double a3, double a2, double a1, double a0) {
  if (a4 == 0.0) return q_cubic(a3, a2, a1, a0);
  if (a0 == 0.0) {
    Roots4 o = q_cubic(a4, a3, a2, a1);
    o.add(0.0);
    return o;
  }
  if (a1 == 0.0 && a3 == 0.0) return q_biquadratic(a4, a2, a0);
  const double a34 = a3 / a4, a24 = a2 / a4, a14 = a1 / a4, a04 = a0 / a4;
  const double a34_pow_2 = a34 * a34;
  const double p = a24 - 3.0 * a34_pow_2 / 8.0;
  const double q = a34_pow_2 * a34 / 8.0 - a34 * a24 / 2.0 + a14;
  const double r = a04 - a34 * a14 / 4.0 + a24 * a34_pow_2 / 16.0 - 3.0 * a34_pow_2 * a34_pow_2 / 256.0;
  const Roots4 d = q_quartic_depressed(p, q, r);
  Roots4 o;
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (i < d.n) o.add(d.r[i] - a34 / 4.0);
  return o;
}

// Torus::trace (torus.rs:56-127) for a torus at `c` (big radius R, small r)
// lying flat in the x/z plane. Returns false on a miss; else the f32 distance
// and the (normalised, ray-facing as Hit::new gives it) normal.
WPT_HD bool torus_trace(V3 c, float big_r, float small_r, V3 o, V3 dir, float& t_out, V3& n_out) {
  const double a = (double)big_r, b = (double)small_r;
  const V3 dv = sub(o, c);
  const double dx = dv.x, dy = dv.y, dz = dv.z;
  const double ex = dir.x, ey = dir.y, ez = dir.z;
  const double g = 4.0 * a * a * (ex * ex + ez * ez);
  const double h = 8.0 * a * a * (dx * ex + dz * ez);
  const double i = 4.0 * a * a * (dx * dx + dz * dz);
  const double j = ex * ex + ey * ey + ez * ez;
  const double k = 2.0 * (dx * ex + dy * ey + dz * ez);
  const double l = dx * dx + dy * dy + dz * dz + a * a - b * b;
  const Roots4 rt = q_quartic(j * j, 2.0 * j * k, 2.0 * j * l + k * k - g, 2.0 * k * l - h, l * l - i);
  // fix_positive (torus.rs:131-141): keep roots >= 0.0001, in order; the
  // closest of them (fmin over numbers: order-free) and their count
  int np = 0;
  double closest = 0.0;
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const bool keep = m < rt.n && rt.r[m] >= 0.0001;
    closest = keep ? (np == 0 ? rt.r[m] : fmin(closest, rt.r[m])) : closest;
    np += keep ? 1 : 0;
  }
  if (np == 0) return false;
  const double px = (double)dv.x + (double)dir.x * closest;
  const double py = (double)dv.y + (double)dir.y * closest;
  const double pz = (double)dv.z + (double)dir.z * closest;
  const double alpha = 1.0 - a / sqrt(px * px + pz * pz);
  V3 nn = normalize(mk((float)(alpha * px), (float)py, (float)(alpha * pz)));  // Vec3::unit
  if (np % 2 == 1) nn = neg(nn);  // inside the torus
  t_out = (float)closest;
  n_out = normalize(nn);  // Hit::new
  return true;
}

}  // namespace wpt
