// tree_eval.cpp — CPU model of the two traversals on a C3-like ray population.
//
// Builds scene 2 over the seeded triangle cloud (scenes.py triangle_cloud), the
// reference BVH2 (wpt_scene.cpp) and the fast tree (wpt_fasttree.cpp), traces
// primary rays of the C3 camera and up to 7 diffuse bounces plus one NEE
// shadow ray per bounce, and for every ray
//   * runs the exact ordered BVH2 descent (scene.rs:218-288, as step() does),
//   * runs the fast traversal (nearest first, inclusive culling, tie and
//     reference-leaf checks) and compares unflagged results with the exact one,
// counting node visits / triangle tests the way the kernels' COUNT builds do.
// Build: make -C tools tree_eval   (tools/Makefile)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <string>
#include <chrono>

#include "wpt_fasttree.h"
#include "wpt_scene.h"

using namespace wpt;

namespace {

struct F4 { float x, y, z, w; };

static std::vector<float> triangle_cloud(size_t n, uint64_t seed) {
  uint64_t state = seed;
  auto next = [&]() {
    state += 0x9E3779B97F4A7C15ull;
    uint64_t z = state;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
  };
  std::vector<float> out(9 * n);
  for (size_t i = 0; i < n; i++) {
    double cx = next() * 5 - 2.5, cy = next() * 5 - 2.5, cz = next() * 5;
    for (int k = 0; k < 3; k++) {
      out[9 * i + 3 * k + 0] = (float)(cx + next() * 0.5);
      out[9 * i + 3 * k + 1] = (float)(cy + next() * 0.5);
      out[9 * i + 3 * k + 2] = (float)(cz + next() * 0.5);
    }
  }
  return out;
}

struct Scene {
  const HostScene* sc;
  std::vector<F4> prims;  // 4 per finite shape
  std::vector<F4> planes;  // (n, n·loc)
};

bool tri_hit(const F4* r, V3 o, V3 d, float& t) {
  const V3 n = mk(r[0].w, r[1].w, r[2].w);
  const float n_dot_d = dot(n, d);
  const float tt = (r[3].w - dot(n, o)) / n_dot_d;
  const V3 nn = mk(r[3].x, r[3].y, r[3].z);
  const V3 pp = add(o, scale(d, tt));
  const V3 v0 = mk(r[0].x, r[0].y, r[0].z), v1 = mk(r[1].x, r[1].y, r[1].z), v2 = mk(r[2].x, r[2].y, r[2].z);
  const bool ok = (n_dot_d != 0.0f) && (tt > 0.0f) && (dot(nn, cross(sub(v1, v0), sub(pp, v0))) + kTriSlack >= 0.0f) &&
                  (dot(nn, cross(sub(v2, v1), sub(pp, v1))) + kTriSlack >= 0.0f) &&
                  (dot(nn, cross(sub(v0, v2), sub(pp, v2))) + kTriSlack >= 0.0f);
  if (ok) t = tt;
  return ok;
}

bool box_entry(const Node2& n, V3 o, V3 inv, float max_dis, float& h) {
  const float tx1 = (n.bmin[0] - o.x) * inv.x, tx2 = (n.bmax[0] - o.x) * inv.x;
  const float ty1 = (n.bmin[1] - o.y) * inv.y, ty2 = (n.bmax[1] - o.y) * inv.y;
  const float tz1 = (n.bmin[2] - o.z) * inv.z, tz2 = (n.bmax[2] - o.z) * inv.z;
  const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
  const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
  const float hh = tmin >= 0.0f ? tmin : 0.0f;
  h = hh;
  return !(tmin > tmax) && (tmin >= 0.0f || tmax >= 0.0f) && (hh < max_dis);
}
// inclusive: entered when entry <= max_dis
bool box_entry_incl(const Node2& n, V3 o, V3 inv, float max_dis, float& h) {
  const bool hit = box_entry(n, o, inv, __builtin_inff(), h);
  return hit && !(max_dis < h);
}

struct Count { uint64_t visits = 0, tests = 0; };

// --- exact: the reference's recursive ordered descent ------------------------
struct Exact {
  const Scene& S;
  V3 o, d, inv;
  float best;
  int32_t id;
  bool shadow;
  int32_t light;
  float early;
  bool occluded;
  Count c;

  bool leaf(const Node2& n) {  // false: shadow early exit
    c.visits++;
    c.tests += n.count;
    const float max_dis = best;
    bool found = false;
    float lb = 0.0f;
    for (uint32_t k = n.left_first; k < n.left_first + n.count; k++) {
      float t;
      if (tri_hit(&S.prims[4 * k], o, d, t)) {
        const int32_t sid = (int32_t)(S.sc->num_inf + k);
        if (shadow && sid != light && t < early) { occluded = true; return false; }
        if (t <= max_dis && (!found || (0.0f < t && t < lb))) { found = true; lb = t; id = sid; }
      }
    }
    if (found) best = lb;
    return true;
  }
  bool visit(uint32_t k) {
    const Node2& n = S.sc->nodes[k];
    return n.count ? leaf(n) : inner(n);
  }
  bool inner(const Node2& n) {
    c.visits++;
    const Node2& l = S.sc->nodes[n.left_first];
    const Node2& r = S.sc->nodes[n.left_first + 1];
    float ld, rd;
    const bool hl = box_entry(l, o, inv, best, ld), hr = box_entry(r, o, inv, best, rd);
    if (hl && hr) {
      if (ld < rd) {
        if (!visit(n.left_first)) return false;
        if (!(best < rd)) return visit(n.left_first + 1);
      } else {
        if (!visit(n.left_first + 1)) return false;
        if (!(best < ld)) return visit(n.left_first);
      }
      return true;
    }
    if (hl) return visit(n.left_first);
    if (hr) return visit(n.left_first + 1);
    return true;
  }
  void run() {
    c.visits++;
    float h;
    if (!box_entry(S.sc->nodes[0], o, inv, best, h)) return;
    visit(0);
  }
};

// --- fast: nearest first over the fast tree -----------------------------------
struct Fast {
  const Scene& S;
  const FastTree& T;
  V3 o, d, inv;
  float best;
  int32_t id;      // plane index (< num_inf), -1, or num_inf + leaf slot
  bool tie = false;
  bool shadow;
  int32_t light;
  float early;
  bool occluded = false;
  Count c;

  int32_t sid_of(int32_t x) const {
    return x < (int32_t)S.sc->num_inf ? x : (int32_t)(S.sc->num_inf + T.refs[x - S.sc->num_inf]);
  }
  bool ref_leaf_ok(uint32_t prim, float t) const {
    float h;
    return box_entry(S.sc->nodes[T.ref_leaf[prim]], o, inv, __builtin_inff(), h) && !(t < h);
  }
  void run() {
    c.visits++;
    float h;
    if (!box_entry_incl(T.nodes[0], o, inv, best, h)) return;
    std::vector<std::pair<uint32_t, float>> st;
    uint32_t cur = 0;
    for (;;) {
      const Node2& n = T.nodes[cur];
      bool next = false;
      if (n.count) {
        c.visits++;
        c.tests += n.count;
        for (uint32_t s = n.left_first; s < n.left_first + n.count; s++) {
          const uint32_t prim = T.refs[s];
          float t;
          if (!tri_hit(&S.prims[4 * prim], o, d, t)) continue;
          const int32_t slot_id = (int32_t)(S.sc->num_inf + s);
          if (shadow && t < early) {
            const int32_t sid = (int32_t)(S.sc->num_inf + prim);
            if (sid != light && ref_leaf_ok(prim, t)) { occluded = true; return; }
          }
          if (t < best) { best = t; id = slot_id; tie = false; }
          else if (t == best && (getenv("SLOTTIE") ? id != slot_id : (id < 0 || sid_of(id) != sid_of(slot_id)))) tie = true;
        }
      } else {
        c.visits++;
        const Node2& l = T.nodes[n.left_first];
        const Node2& r = T.nodes[n.left_first + 1];
        float ld, rd;
        const bool hl = box_entry_incl(l, o, inv, best, ld), hr = box_entry_incl(r, o, inv, best, rd);
        if (hl && hr) {
          const bool lf = ld <= rd;
          st.push_back({lf ? n.left_first + 1 : n.left_first, lf ? rd : ld});
          cur = lf ? n.left_first : n.left_first + 1;
          next = true;
        } else if (hl || hr) {
          cur = hl ? n.left_first : n.left_first + 1;
          next = true;
        }
      }
      if (next) continue;
      bool got = false;
      while (!st.empty()) {
        auto e = st.back();
        st.pop_back();
        if (!(best < e.second)) { cur = e.first; got = true; break; }
      }
      if (!got) return;
    }
  }
  // the verdict on the fast result: true = must be re-traced exactly
  mutable int why = 0;
  bool flagged() const {
    if (occluded) return false;
    if (tie) { why = 1; return true; }
    why = 2;
    if (id >= (int32_t)S.sc->num_inf) return !ref_leaf_ok(T.refs[id - S.sc->num_inf], best);
    return false;
  }
};

uint32_t rng_next(uint32_t& s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }
float rnd(uint32_t& s) { return (float)rng_next(s) * (1.0f / 4294967296.0f); }

}  // namespace

int main(int argc, char** argv) {
  size_t ntri = argc > 1 ? (size_t)atol(argv[1]) : 100000;
  int stride = argc > 2 ? atoi(argv[2]) : 4;
  FastTreeOptions opt;
  if (argc > 3) opt.bins = atoi(argv[3]);
  if (argc > 4) opt.max_leaf = atoi(argv[4]);
  if (argc > 5) opt.c_trav = (float)atof(argv[5]);
  if (argc > 6) opt.spatial = atoi(argv[6]) != 0;
  if (argc > 7) opt.alpha = (float)atof(argv[7]);
  if (argc > 8) opt.margin_log2 = atoi(argv[8]);
  if (argc > 9) opt.omax_mult = (float)atof(argv[9]);
  if (argc > 10) opt.dup_budget = (float)atof(argv[10]);
  if (argc > 11) opt.sp_bins = atoi(argv[11]);
  std::vector<float> mesh = triangle_cloud(ntri, 0x5EED);
  HostScene sc;
  std::string err;
  if (!build_scene(2, mesh, sc, err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
  FastTree T;
  if (!build_fast_tree(sc, opt, T, err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
  size_t leaves = 0;
  for (size_t k = 0; k < T.nodes.size(); k++) leaves += (k != 1 && T.nodes[k].count) ? 1 : 0;
  printf("ref: %zu nodes depth %u | fast: %zu nodes, %zu leaves, %zu refs (%.3fx), depth %u, sah %.2f, margin %.2e, build %.0f ms\n",
         sc.nodes.size(), sc.depth, T.nodes.size(), leaves, T.refs.size(), (double)T.refs.size() / (sc.shapes.size() - sc.num_inf),
         T.depth, T.sah, T.margin, T.ms);
  Scene S;
  S.sc = &sc;
  const size_t nf = sc.shapes.size() - sc.num_inf;
  S.prims.resize(4 * nf);
  for (size_t i = 0; i < nf; i++) {
    const float* g = sc.shapes[sc.num_inf + i].g;
    V3 v0 = mk(g[0], g[1], g[2]), v1 = mk(g[3], g[4], g[5]), v2 = mk(g[6], g[7], g[8]);
    V3 n = cross(sub(v1, v0), sub(v2, v0));
    V3 nn = normalize(n);
    float od = dot(n, v0);
    S.prims[4 * i + 0] = {v0.x, v0.y, v0.z, n.x};
    S.prims[4 * i + 1] = {v1.x, v1.y, v1.z, n.y};
    S.prims[4 * i + 2] = {v2.x, v2.y, v2.z, n.z};
    S.prims[4 * i + 3] = {nn.x, nn.y, nn.z, od};
  }
  for (uint32_t i = 0; i < sc.num_inf; i++) {
    const float* g = sc.shapes[i].g;
    V3 loc = mk(g[0], g[1], g[2]), n = mk(g[3], g[4], g[5]);
    S.planes.push_back({n.x, n.y, n.z, dot(n, loc)});
  }
  auto planes = [&](V3 o, V3 d, float& best, int32_t& id) {
    bool found = false;
    for (uint32_t i = 0; i < sc.num_inf; i++) {
      const V3 n = mk(S.planes[i].x, S.planes[i].y, S.planes[i].z);
      const float nd = dot(n, d);
      if (nd == 0.0f) continue;
      const float t = (S.planes[i].w - dot(n, o)) / nd;
      if (t <= 0.0f) continue;
      if (!found || (0.0f < t && t < best)) { found = true; best = t; id = (int32_t)i; }
    }
  };
  const uint32_t W = 1920, H = 1080;
  const float cam[5] = {-0.9f, 5.4f, 0.4f, 0.58f, 0.0f};
  const float cx = mcos(cam[3]), sx = msin(cam[3]), cy = mcos(cam[4]), sy = msin(cam[4]);
  Count ce, cf, se, sf;
  uint64_t n_ext = 0, n_sh = 0, flags_ext = 0, flags_sh = 0, mism = 0, far_o = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t y = 0; y < H; y += stride) {
    for (uint32_t x = 0; x < W; x += stride) {
      uint32_t s = (y * W + x) * 2654435761u + 12345u;
      if (!s) s = 1;
      const float fx = (((float)x + rnd(s)) * (1.0f / W) - 0.5f) * ((float)W / (float)H);
      const float fy = 0.5f - ((float)y + rnd(s)) * (1.0f / H);
      V3 v = normalize(mk(fx, fy, 0.8f));
      v = mk(v.x, cx * v.y - sx * v.z, sx * v.y + cx * v.z);
      v = mk(cy * v.x + sy * v.z, v.y, (-sy) * v.x + cy * v.z);
      V3 o = mk(cam[0], cam[1], cam[2]), d = v;
      for (int b = 0; b < 8; b++) {
        const V3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        Exact E{S, o, d, inv, __builtin_inff(), -1, false, -1, 0.0f, false, {}};
        planes(o, d, E.best, E.id);
        E.run();
        Fast F{S, T, o, d, inv, __builtin_inff(), -1, false, false, -1, 0.0f, false, {}};
        planes(o, d, F.best, F.id);
        const bool ofar = !(fabsf(o.x) <= T.omax && fabsf(o.y) <= T.omax && fabsf(o.z) <= T.omax);
        if (!ofar) F.run();
        n_ext++;
        ce.visits += E.c.visits; ce.tests += E.c.tests;
        cf.visits += F.c.visits; cf.tests += F.c.tests;
        if (ofar) { far_o++; flags_ext++; cf.visits += E.c.visits; cf.tests += E.c.tests; }
        else if (F.flagged()) flags_ext++;
        else if (F.best != E.best || F.sid_of(F.id) != E.id) {
          if (mism < 10) printf("MISMATCH ext: fast %.9g %d exact %.9g %d\n", F.best, F.sid_of(F.id), E.best, E.id);
          mism++;
        }
        if (E.id < 0) break;
        // hit: normal, bounce
        const V3 hp = add(o, scale(d, E.best));
        V3 nrm;
        if (E.id < (int32_t)sc.num_inf) {
          nrm = mk(S.planes[E.id].x, S.planes[E.id].y, S.planes[E.id].z);
        } else {
          const F4* r = &S.prims[4 * (E.id - sc.num_inf)];
          nrm = mk(r[3].x, r[3].y, r[3].z);
          if (sc.shapes[E.id].emissive) break;
        }
        if (dot(nrm, d) > 0.0f) nrm = neg(nrm);
        // NEE shadow ray to a random point of a random light
        {
          const uint32_t li = rng_next(s) % (uint32_t)sc.lights.size();
          const float* g = sc.shapes[sc.lights[li]].g;
          float q1 = rnd(s), q2 = rnd(s), q1s = sqrtf(q1);
          V3 pt = add(add(scale(mk(g[0], g[1], g[2]), 1.0f - q1s), scale(mk(g[3], g[4], g[5]), q1s * (1.0f - q2))),
                      scale(mk(g[6], g[7], g[8]), q2 * q1s));
          V3 tl = sub(pt, hp);
          const float dl = len(tl);
          tl = scale(tl, 1.0f / dl);
          if (dot(tl, nrm) > 0.0f) {
            const V3 so = add(hp, scale(tl, kEpsilon));
            const V3 sinv = mk(1.0f / tl.x, 1.0f / tl.y, 1.0f / tl.z);
            const int32_t light = (int32_t)sc.lights[li];
            // early: the light's own hit distance capped at dir_len
            float early = dl, tlh;
            if (tri_hit(&S.prims[4 * (light - sc.num_inf)], so, tl, tlh)) early = fminf(tlh, dl);
            float pt2 = __builtin_inff();
            int32_t pid = -1;
            planes(so, tl, pt2, pid);
            n_sh++;
            if (!(pid >= 0 && pt2 < early)) {
              const float b0 = (pid >= 0 && pt2 < dl) ? pt2 : dl;
              const int32_t i0 = (pid >= 0 && pt2 < dl) ? pid : -1;
              Exact Es{S, so, tl, sinv, b0, i0, true, light, early, false, {}};
              Es.run();
              Fast Fs{S, T, so, tl, sinv, b0, i0, false, true, light, early, false, {}};
              const bool sfar = !(fabsf(so.x) <= T.omax && fabsf(so.y) <= T.omax && fabsf(so.z) <= T.omax);
              if (!sfar) Fs.run();
              se.visits += Es.c.visits; se.tests += Es.c.tests;
              sf.visits += Fs.c.visits; sf.tests += Fs.c.tests;
              auto verdict = [&](bool occ, float bt, int32_t bid) { return occ || (bid >= 0 && bt < dl && bid != light); };
              const bool ve = verdict(Es.occluded, Es.best, Es.id);
              if (sfar) { sf.visits += Es.c.visits; sf.tests += Es.c.tests; }
              if (sfar || Fs.flagged()) { flags_sh++; if (!sfar && flags_sh < 6) printf("shadow flag why %d fast %.9g id %d exact %.9g %d occ %d/%d dl %.9g early %.9g light %d\n", Fs.why, Fs.best, Fs.sid_of(Fs.id), Es.best, Es.id, Fs.occluded, Es.occluded, dl, early, light); }
              else if (verdict(Fs.occluded, Fs.best, Fs.id < 0 ? -1 : Fs.sid_of(Fs.id)) != ve) {
                if (mism < 10) printf("MISMATCH shadow\n");
                mism++;
              }
            }
          }
        }
        // cosine bounce
        const float r1 = rnd(s), r2 = rnd(s);
        const float ang = 2.0f * kPi * r1;
        const float lx = cosf(ang) * sqrtf(1.0f - r2), ly = sqrtf(r2), lz = sinf(ang) * sqrtf(1.0f - r2);
        const V3 xn = orthogonal(nrm), zn = cross(nrm, xn);
        const V3 wi = normalize(add(add(scale(xn, lx), scale(nrm, ly)), scale(zn, lz)));
        o = add(hp, scale(wi, kEpsilon));
        d = wi;
      }
    }
  }
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("extension rays %lu: exact %.2f visits %.2f tests | fast %.2f visits %.2f tests | flagged %.2e (origin %lu)\n",
         (unsigned long)n_ext, (double)ce.visits / n_ext, (double)ce.tests / n_ext, (double)cf.visits / n_ext,
         (double)cf.tests / n_ext, (double)flags_ext / n_ext, (unsigned long)far_o);
  printf("shadow rays %lu: exact %.2f visits %.2f tests | fast %.2f visits %.2f tests | flagged %.2e\n",
         (unsigned long)n_sh, (double)se.visits / n_sh, (double)se.tests / n_sh, (double)sf.visits / n_sh,
         (double)sf.tests / n_sh, (double)flags_sh / n_sh);
  printf("mismatches %lu  (%.1f s)\n", (unsigned long)mism, sec);
  return mism ? 2 : 0;
}
