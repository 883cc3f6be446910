// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see ref_core.h header).
// BVH2 build (src/graphics/bvh.rs:103-437) and scene queries with the
// recursive ordered BVH2 traversal (src/graphics/scene.rs:104-472).
// ============================================================================
#include "ref_scene.h"

#include <functional>
#include <limits>

namespace ref {

namespace {

// bvh.rs:85-89
struct ShapeRep {
  ShapeP shape;
  Vec3 location;
  AABB bounds;
};

// bvh.rs:397-407
bool reps_aabb(const ShapeRep* s, size_t n, AABB* out) {
  if (n == 0) return false;
  AABB res = s[0].bounds;
  for (size_t i = 1; i < n; i++) res = aabb_join(res, s[i].bounds);
  *out = res;
  return true;
}

struct Bins {  // bvh.rs:440-476
  std::vector<std::vector<ShapeRep>> bins;
  explicit Bins(size_t n) : bins(n) {}
  void clear() { for (auto& b : bins) b.clear(); }
  void write_to(ShapeRep* dst) const {
    size_t i = 0;
    for (auto& b : bins)
      for (auto& v : b) dst[i++] = v;
  }
};

// bvh.rs:412-437
bool bin(const ShapeRep* xs, size_t n, int axis, Bins& dst) {
  auto f = [axis](const ShapeRep& s) { return axis == 0 ? s.location.x : axis == 1 ? s.location.y : s.location.z; };
  float min_v = f(xs[0]), max_v = f(xs[0]);
  for (size_t i = 1; i < n; i++) {
    float v = f(xs[i]);
    min_v = fminf(min_v, v);
    max_v = fmaxf(max_v, v);
  }
  if (min_v == max_v) return false;
  size_t num_bins = dst.bins.size();
  dst.clear();
  float segment_width = (max_v - min_v) / (float)num_bins;
  for (size_t i = 0; i < n; i++) {
    float v = f(xs[i]);
    float q = floorf((v - min_v) / segment_width);
    size_t sid = (q != q || q <= 0.0f) ? 0 : (q >= 1.8e19f ? (size_t)-1 : (size_t)q);  // saturating `as usize`
    if (sid > num_bins - 1) sid = num_bins - 1;
    dst.bins[sid].push_back(xs[i]);
  }
  return true;
}

// bvh.rs:309-370
bool split_axis(const ShapeRep* shapes, size_t n, int axis, Bins& b, AABB* lo, AABB* ro, size_t* idx) {
  size_t num_bins = b.bins.size();
  if (n <= 1) return false;
  if (!bin(shapes, n, axis, b)) return false;
  size_t l = 0, r = num_bins - 1;
  AABB l_aabb, r_aabb, tmp;
  reps_aabb(b.bins[l].data(), b.bins[l].size(), &l_aabb);
  reps_aabb(b.bins[r].data(), b.bins[r].size(), &r_aabb);
  size_t l_cnt = b.bins[l].size(), r_cnt = b.bins[r].size();
  AABB ln_aabb = reps_aabb(b.bins[l + 1].data(), b.bins[l + 1].size(), &tmp) ? aabb_join(l_aabb, tmp) : l_aabb;
  AABB rn_aabb = reps_aabb(b.bins[r - 1].data(), b.bins[r - 1].size(), &tmp) ? aabb_join(r_aabb, tmp) : r_aabb;
  size_t ln_cnt = l_cnt + b.bins[l + 1].size();
  size_t rn_cnt = r_cnt + b.bins[r - 1].size();
  while (l + 1 < r) {
    if ((aabb_surface(ln_aabb) * (float)ln_cnt + aabb_surface(r_aabb) * (float)r_cnt) <
        (aabb_surface(l_aabb) * (float)l_cnt + aabb_surface(rn_aabb) * (float)rn_cnt)) {
      l += 1;
      l_aabb = ln_aabb;
      l_cnt = ln_cnt;
      if (l + 1 < r) {
        ln_aabb = reps_aabb(b.bins[l + 1].data(), b.bins[l + 1].size(), &tmp) ? aabb_join(l_aabb, tmp) : l_aabb;
        ln_cnt = l_cnt + b.bins[l + 1].size();
      }
    } else {
      r -= 1;
      r_aabb = rn_aabb;
      r_cnt = rn_cnt;
      if (l + 1 < r) {
        rn_aabb = reps_aabb(b.bins[r - 1].data(), b.bins[r - 1].size(), &tmp) ? aabb_join(r_aabb, tmp) : r_aabb;
        rn_cnt = r_cnt + b.bins[r - 1].size();
      }
    }
  }
  *lo = l_aabb;
  *ro = r_aabb;
  *idx = l_cnt;
  return true;
}

// bvh.rs:282-303
bool split_longest_axis(const ShapeRep* s, size_t n, const AABB& p, Bins& b, AABB* lo, AABB* ro, size_t* idx) {
  float x_size = p.x_max - p.x_min, y_size = p.y_max - p.y_min, z_size = p.z_max - p.z_min;
  int axis;
  if (x_size > y_size) axis = (x_size > z_size) ? 0 : 2;
  else axis = (y_size > z_size) ? 1 : 2;
  return split_axis(s, n, axis, b, lo, ro, idx);
}

// bvh.rs:254-277. Returns true on DoSplit.
bool split(ShapeRep* s, size_t n, const AABB& parent, Bins& b, size_t* idx, AABB* lo, AABB* ro, AABB* leaf) {
  if (n <= 1) {
    reps_aabb(s, n, leaf);
    return false;
  }
  AABB l, r;
  size_t index;
  if (split_longest_axis(s, n, parent, b, &l, &r, &index)) {
    float utility = aabb_surface(l) * (float)index + aabb_surface(r) * (float)(n - index);
    AABB pa = aabb_join(l, r);
    float parent_utility = aabb_surface(pa) * (float)n;
    if (utility < parent_utility) {
      b.write_to(s);
      *idx = index; *lo = l; *ro = r;
      return true;
    }
    *leaf = pa;
    return false;
  }
  reps_aabb(s, n, leaf);
  return false;
}

// bvh.rs:215-239
BVHNode subdivide(std::vector<BVHNode>& dst, ShapeRep* shapes, size_t offset, size_t length, const AABB& parent, Bins& b) {
  size_t si;
  AABB l, r, leaf;
  if (split(shapes + offset, length, parent, b, &si, &l, &r, &leaf)) {
    size_t left_id = dst.size();
    dst.push_back(BVHNode{aabb_empty(), 0, 0});
    dst.push_back(BVHNode{aabb_empty(), 0, 0});
    BVHNode ln = subdivide(dst, shapes, offset, si, l, b);
    dst[left_id] = ln;
    BVHNode rn = subdivide(dst, shapes, offset + si, length - si, r, b);
    dst[left_id + 1] = rn;
    return BVHNode{aabb_join(l, r), (uint32_t)left_id, 0};
  }
  return BVHNode{leaf, (uint32_t)offset, (uint32_t)length};
}

}  // namespace

// bvh.rs:103-125 with shape_reps (:376-394)
size_t build_bvh(std::vector<ShapeP>& shapes, size_t num_bins, std::vector<BVHNode>& dst) {
  size_t num_inf = 0;
  std::vector<ShapeRep> reps;
  reps.reserve(shapes.size());
  for (size_t i = 0; i < shapes.size(); i++) {
    ShapeP s = shapes[i];
    AABB bd;
    Vec3 loc;
    if (s->aabb(&bd) && s->location(&loc)) {
      reps.push_back(ShapeRep{s, loc, bd});
    } else {
      std::swap(shapes[num_inf], shapes[i]);
      num_inf++;
    }
  }
  dst.clear();
  dst.push_back(BVHNode{aabb_empty(), 0, 0});
  dst.push_back(BVHNode{aabb_empty(), 0, 0});
  if (reps.empty()) return num_inf;
  Bins bins(num_bins);
  AABB all;
  reps_aabb(reps.data(), reps.size(), &all);
  BVHNode root = subdivide(dst, reps.data(), 0, reps.size(), all, bins);
  dst[0] = root;
  for (size_t i = 0; i < reps.size(); i++) shapes[i + num_inf] = reps[i].shape;
  return num_inf;
}

namespace {
bool verify_bounds(const std::vector<ShapeP>& shapes, size_t num_inf, const std::vector<BVHNode>& bvh, size_t i) {
  const BVHNode& n = bvh[i];
  if (n.count == 0) {
    size_t li = n.left_first;
    if (!verify_bounds(shapes, num_inf, bvh, li) || !verify_bounds(shapes, num_inf, bvh, li + 1)) return false;
    AABB b = aabb_join(bvh[li].bounds, bvh[li + 1].bounds);
    return aabb_contains(n.bounds, b);
  }
  for (size_t k = num_inf + n.left_first; k < num_inf + n.left_first + n.count; k++) {
    AABB b;
    if (!shapes[k]->aabb(&b) || !aabb_contains(n.bounds, b)) return false;
  }
  return true;
}
void verify_contains(std::vector<bool>& c, const std::vector<BVHNode>& bvh, size_t i) {
  if (bvh[i].count == 0) {
    verify_contains(c, bvh, bvh[i].left_first);
    verify_contains(c, bvh, bvh[i].left_first + 1);
  } else {
    for (uint32_t k = bvh[i].left_first; k < bvh[i].left_first + bvh[i].count; k++) c[k] = true;
  }
}
}  // namespace

// bvh.rs:128-194
bool verify_bvh(const std::vector<ShapeP>& shapes, size_t num_inf, const std::vector<BVHNode>& bvh) {
  if (shapes.size() == num_inf) return true;
  bool a = verify_bounds(shapes, num_inf, bvh, 0);
  std::vector<bool> c(shapes.size() - num_inf, false);
  verify_contains(c, bvh, 0);
  for (bool x : c) a = a && x;
  return a;
}

// ---------------------------------------------------------------------------
// Scene queries
// ---------------------------------------------------------------------------
namespace {
struct Res {
  bool ok;
  float t;
  size_t id;
};
const Res NONE{false, 0.0f, 0};

// scene.rs:426-445
Res trace_shapes(const Ray& ray, const ShapeP* shapes, size_t n) {
  Res best = NONE;
  for (size_t i = 0; i < n; i++) {
    float nd;
    if (shapes[i]->trace_simple(ray, &nd)) {
      if (best.ok) {
        if (0.0f < nd && nd < best.t) best = Res{true, nd, i};
      } else {
        best = Res{true, nd, i};
      }
    }
  }
  return best;
}

// scene.rs:450-472
Res trace_shapes_md(const Ray& ray, const ShapeP* shapes, size_t n, float max_dis) {
  Res best = NONE;
  for (size_t i = 0; i < n; i++) {
    float nd;
    if (shapes[i]->trace_simple(ray, &nd)) {
      if (nd <= max_dis) {
        if (best.ok) {
          if (0.0f < nd && nd < best.t) best = Res{true, nd, i};
        } else {
          best = Res{true, nd, i};
        }
      }
    }
  }
  return best;
}

// scene.rs:393-403
bool aabb_distance(const Ray& ray, const AABB& b, float max_dis, float* out) {
  float h;
  if (aabb_hit(b, ray, &h) && h < max_dis) {
    *out = h;
    return true;
  }
  return false;
}

// scene.rs:406-422 (prefers b on ties)
Res closest(Res a, Res b) {
  if (a.ok) {
    if (b.ok) return (a.t < b.t) ? a : b;
    return a;
  }
  return b;
}

struct Trav {
  const Ray& ray;
  size_t num_inf;
  const std::vector<BVHNode>& bvh;
  const std::vector<ShapeP>& shapes;

  // scene.rs:218-288
  Res traverse(size_t node_i, float max_dis, size_t* visits) const {
    const BVHNode& node = bvh[node_i];
    if (node.count != 0) {
      size_t off = node.left_first, size = node.count;
      Res r = trace_shapes_md(ray, &shapes[num_inf + off], size, max_dis);
      *visits += 1;
      if (r.ok) return Res{true, r.t, num_inf + off + r.id};
      return NONE;
    }
    size_t li = node.left_first;
    float left_dis, right_dis;
    if (aabb_distance(ray, bvh[li].bounds, max_dis, &left_dis)) {
      if (aabb_distance(ray, bvh[li + 1].bounds, max_dis, &right_dis)) {
        if (left_dis < right_dis) {
          size_t ld = 0;
          Res tl = traverse(li, max_dis, &ld);
          if (tl.ok) {
            if (tl.t < right_dis) {
              *visits += 1 + ld;
              return tl;
            }
            size_t rd = 0;
            Res tr = traverse(li + 1, tl.t, &rd);
            *visits += 1 + ld + rd;
            return tr.ok ? tr : tl;
          }
          size_t rd = 0;
          Res tr = traverse(li + 1, max_dis, &rd);
          *visits += 1 + ld + rd;
          return tr;
        } else {
          size_t rd = 0;
          Res tr = traverse(li + 1, max_dis, &rd);
          if (tr.ok) {
            if (tr.t < left_dis) {
              *visits += 1 + rd;
              return tr;
            }
            size_t ld = 0;
            Res tl = traverse(li, tr.t, &ld);
            *visits += 1 + ld + rd;
            return tl.ok ? tl : tr;
          }
          size_t ld = 0;
          Res tl = traverse(li, max_dis, &ld);
          *visits += 1 + ld + rd;
          return tl;
        }
      }
      size_t ld = 0;
      Res tl = traverse(li, max_dis, &ld);
      *visits += ld + 1;
      return tl;
    }
    size_t rd = 0;
    Res tr = guarded(li + 1, max_dis, &rd);
    *visits += rd + 1;
    return tr;
  }

  // scene.rs:191-212
  Res guarded(size_t node_i, float max_dis, size_t* visits) const {
    float h;
    if (aabb_hit(bvh[node_i].bounds, ray, &h)) {
      if (h < max_dis) {
        size_t d = 0;
        Res r = traverse(node_i, max_dis, &d);
        *visits += d + 1;
        return r;
      }
    }
    *visits += 1;
    return NONE;
  }
};
}  // namespace

void Scene::init(Color3 bg, std::vector<ShapeP> s) {
  background = bg;
  shapes = std::move(s);
  num_inf = build_bvh(shapes, 16, bvh);  // scene.rs:60 rebuild_bvh(16, false)
  kind = BVH_2;
  lights.clear();
  for (size_t i = 0; i < shapes.size(); i++)
    if (shapes[i]->is_emissive()) lights.push_back(i);  // scene.rs:62-66
}

size_t Scene::trace_g(const Ray& ray, float* t, size_t* id, bool* found) const {
  Res r;
  size_t visits = 0;
  bool has_finite = shapes.size() > num_inf;
  if (kind == BVH_2) {
    Trav tv{ray, num_inf, bvh, shapes};
    Res h1 = trace_shapes(ray, shapes.data(), num_inf);
    if (h1.ok) {
      Res h2 = has_finite ? tv.guarded(0, h1.t, &visits) : NONE;
      r = closest(h1, h2);
    } else {
      r = has_finite ? tv.guarded(0, std::numeric_limits<float>::infinity(), &visits) : NONE;
    }
  } else {
    r = trace_shapes(ray, shapes.data(), shapes.size());
  }
  *found = r.ok;
  *t = r.t;
  *id = r.id;
  return visits;
}

size_t Scene::trace(const Ray& ray, Hit* hit, bool* ok, size_t* id_out) const {
  float t;
  size_t id;
  bool found;
  size_t d = trace_g(ray, &t, &id, &found);
  *ok = false;
  if (found) {
    *ok = shapes[id]->trace(ray, hit);
    if (id_out) *id_out = id;
  }
  return d;
}

size_t Scene::shadow_ray(Vec3 p, Vec3 q, long light_shape, bool* occluded) const {
  Vec3 dir = q - p;
  float dir_len = len(dir);
  dir = dir / dir_len;
  Ray ray = make_ray(p + dir * EPSILON, dir);
  float t;
  size_t id;
  bool found;
  size_t d = trace_g(ray, &t, &id, &found);
  *occluded = false;
  if (found && t < dir_len) {
    if (light_shape >= 0) *occluded = (id != (size_t)light_shape);
    else *occluded = true;
  }
  return d;
}

}  // namespace ref
