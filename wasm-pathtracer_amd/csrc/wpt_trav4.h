// wpt_trav4.h — fast-path BVH4 closest hit (included by wpt_render.hip).
//
// The BVH4 is the reference's BVH2 collapsed two levels at a time (same
// boxes, bit for bit). It is traversed nearest-first with INCLUSIVE culling
// (a box is entered when its entry <= closest hit so far), four child slab
// tests per node and leaf children tested on the spot. This order differs
// from the reference's recursive BVH2 descent (scene.rs:218-288), so two
// conditions are tracked under which the reference could return a different
// (t, shape id):
//   tie   — another shape (or the plane that seeded the search) is hit at
//           exactly the winning t: the reference breaks ties by visit order;
//   quirk — the winning t is below its leaf box's entry distance (possible
//           only through rounding): the reference's strict culling could then
//           skip it. Entry distances never decrease from parent to child box
//           (the slab test is monotone in the bounds), so the leaf's entry
//           bounds every ancestor's.
// Without either, every ancestor box of the winner has entry <= t_win <=
// the reference's closest-so-far, so the reference visits the winner too and
// finds no smaller t: both results agree exactly. A flagged ray is re-traced
// with the exact BVH2 stack machine (step()), so results stay bit-identical.
#pragma once

// AABB::hit (aabb.rs:132-164) on four SoA boxes with inclusive culling.
__device__ __forceinline__ void slab4(const float4& xn, const float4& xx, const float4& yn, const float4& yx,
                                      const float4& zn, const float4& zx, V3 o, V3 inv, float best, float (&e)[4],
                                      bool (&hit)[4]) {
  const float xmn[4] = {xn.x, xn.y, xn.z, xn.w}, xmx[4] = {xx.x, xx.y, xx.z, xx.w};
  const float ymn[4] = {yn.x, yn.y, yn.z, yn.w}, ymx[4] = {yx.x, yx.y, yx.z, yx.w};
  const float zmn[4] = {zn.x, zn.y, zn.z, zn.w}, zmx[4] = {zx.x, zx.y, zx.z, zx.w};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const float tx1 = (xmn[k] - o.x) * inv.x;
    const float tx2 = (xmx[k] - o.x) * inv.x;
    const float ty1 = (ymn[k] - o.y) * inv.y;
    const float ty2 = (ymx[k] - o.y) * inv.y;
    const float tz1 = (zmn[k] - o.z) * inv.z;
    const float tz2 = (zmx[k] - o.z) * inv.z;
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    const float h = tmin >= 0.0f ? tmin : 0.0f;
    hit[k] = !(tmin > tmax) && (tmin >= 0.0f || tmax >= 0.0f) && !(best < h);
    e[k] = h;
  }
}

// Candidate accept with tie / quirk tracking (e_leaf = the leaf box entry).
__device__ __forceinline__ void accept4(Lane& L, float t, int32_t sid, float e_leaf, bool& tie, bool& quirk) {
  if (t < L.best) {
    L.best = t;
    L.best_id = sid;
    tie = false;
    quirk = t < e_leaf;
  } else if (t == L.best && sid != L.best_id) {
    tie = true;
  }
}

__device__ __forceinline__ void cas_desc(float& ea, uint32_t& ca, float& eb, uint32_t& cb) {
  const bool sw = ea < eb;
  const float te = sw ? eb : ea, tb = sw ? ea : eb;
  const uint32_t tc = sw ? cb : ca, tcb = sw ? ca : cb;
  ea = te; eb = tb; ca = tc; cb = tcb;
}

// Resume the nearest deferred BVH4 node not culled (inclusive); false if empty.
__device__ __forceinline__ bool pop4(Lane& L, const Stack& st) {
  while (L.sp > 0) {
    uint32_t code;
    float h;
    pop_top(L, st, code, h);
    if (!(L.best < h)) {
      L.lf = code;
      return true;
    }
  }
  return false;
}

// Fast path start: the reference's root guard with inclusive culling.
template <bool COUNT>
__device__ __forceinline__ bool enter_root4(const Hot& H, Lane& L, uint32_t& visits, uint32_t& nbytes) {
  if (COUNT) { visits++; nbytes += 32; }
  const float4 a = H.root_a, b = H.root_b;
  const float tx1 = (a.x - L.o.x) * L.inv.x, tx2 = (a.w - L.o.x) * L.inv.x;
  const float ty1 = (a.y - L.o.y) * L.inv.y, ty2 = (b.x - L.o.y) * L.inv.y;
  const float tz1 = (a.z - L.o.z) * L.inv.z, tz2 = (b.y - L.o.z) * L.inv.z;
  const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
  const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
  const float h = tmin >= 0.0f ? tmin : 0.0f;
  if (tmin > tmax || !(tmin >= 0.0f || tmax >= 0.0f) || L.best < h) return false;
  L.lf = 0;
  L.cnt = 0;
  L.sp = 0;
  return true;
}

// One BVH4 node visit. Returns false when the traversal is finished (stack
// empty, or the SHADOW early exit: a non-light shape hit strictly before
// `early` and not below its leaf entry — the reference then provably finds an
// occluder).
template <bool SHADOW, bool TRI_ONLY, bool COUNT>
__device__ __forceinline__ bool step4(const DevScene& S, Lane& L, const Stack& stk, int32_t light, float early,
                                      bool& occluded, bool& tie, bool& quirk, uint32_t& visits, uint32_t& tests,
                                      uint32_t& nbytes) {
  const float4* nd = S.nodes4 + 8 * (size_t)L.lf;
  if (COUNT) { visits++; nbytes += 128; }
  float4 xn = nd[0], xx = nd[1], yn = nd[2], yx = nd[3], zn = nd[4], zx = nd[5];
  float4 chf = nd[6];
  pin4(xn);
  pin4(xx);
  pin4(yn);
  pin4(yx);
  pin4(zn);
  pin4(zx);
  pin4(chf);
  const uint4 ch = make_uint4(__float_as_uint(chf.x), __float_as_uint(chf.y), __float_as_uint(chf.z),
                              __float_as_uint(chf.w));
  const uint32_t code[4] = {ch.x, ch.y, ch.z, ch.w};
  float e[4];
  bool hit[4];
  slab4(xn, xx, yn, yx, zn, zx, L.o, L.inv, L.best, e, hit);
  // leaf children first (order is free on the fast path); one test site,
  // driven by the bitmask of hit leaf children
  uint32_t leaves = 0;
#pragma unroll
  for (int k = 0; k < 4; k++)
    leaves |= (hit[k] && code[k] != kChildEmpty && (code[k] & 0x80000000u)) ? (1u << k) : 0u;
  while (leaves) {
    const int k = __builtin_ctz(leaves);
    leaves &= leaves - 1;
    const uint32_t ck = k == 0 ? code[0] : k == 1 ? code[1] : k == 2 ? code[2] : code[3];
    const float ek = k == 0 ? e[0] : k == 1 ? e[1] : k == 2 ? e[2] : e[3];
    uint32_t first, cnt;
    if ((ck & 0xC0000000u) == 0xC0000000u) {
      const uint32_t q = ck & 0x3FFFFFFFu;
      first = S.leaf_table[2 * q];
      cnt = S.leaf_table[2 * q + 1];
    } else {
      first = ck & 0xFFFFFFu;
      cnt = (ck >> 24) & 0x3Fu;
    }
    if (COUNT) tests += cnt;
    for (uint32_t p = first; p < first + cnt; p++) {
      float t;
      const float4* pr = S.prims + 4 * (size_t)p;
      const bool h = TRI_ONLY ? tri_hit(pr, L.o, L.d, t) : prim_hit(S.kinds[p], pr, L.o, L.d, t);
      if (h) {
        const int32_t sid = (int32_t)(S.num_inf + p);
        if (SHADOW && sid != light && t < early && !(t < ek)) {
          occluded = true;
          return false;
        }
        accept4(L, t, sid, ek, tie, quirk);
      }
    }
  }
  // internal children still in range, nearest first
  float ce[4];
  uint32_t cc[4];
  int m = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const bool cand = hit[k] && code[k] != kChildEmpty && !(code[k] & 0x80000000u) && !(L.best < e[k]);
    ce[k] = cand ? e[k] : -__int_as_float(0x7f800000);
    cc[k] = code[k];
    m += cand ? 1 : 0;
  }
  if (m == 0) return pop4(L, stk);
  // sort descending by entry (5-comparator network); candidates first
  cas_desc(ce[0], cc[0], ce[1], cc[1]);
  cas_desc(ce[2], cc[2], ce[3], cc[3]);
  cas_desc(ce[0], cc[0], ce[2], cc[2]);
  cas_desc(ce[1], cc[1], ce[3], cc[3]);
  cas_desc(ce[1], cc[1], ce[2], cc[2]);
  // push the farther ones (popped nearest-first), continue with the nearest
  if (m > 1) push(L, stk, cc[0], ce[0]);
  if (m > 2) push(L, stk, cc[1], ce[1]);
  if (m > 3) push(L, stk, cc[2], ce[2]);
  L.lf = m == 1 ? cc[0] : m == 2 ? cc[1] : m == 3 ? cc[2] : cc[3];
  return true;
}

