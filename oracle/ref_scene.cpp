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

// ---------------------------------------------------------------------------
// bvh4.rs:121-281
// ---------------------------------------------------------------------------
namespace {
using Memo = std::vector<std::vector<float>>;  // Vec<Option<Vec<f32>>>: empty = None

bool is_leaf(const BVHNode& n) { return n.count != 0; }

// r_cost (bvh4.rs:244-281)
float r_cost(Memo& memo, const std::vector<BVHNode>& bvh, size_t node_i, size_t cutsize) {
  const float t_cost = 1.0f;
  const size_t max_childs = 4;
  if (is_leaf(bvh[node_i])) return t_cost;
  const size_t node_left_i = bvh[node_i].left_first;
  const size_t node_right_i = node_left_i + 1;
  if (memo[node_i].empty()) {
    std::vector<float> cost(max_childs, INFINITY);
    for (size_t t = 2; t < max_childs + 1; t++) {
      for (size_t i = 1; i < t; i++) {
        const float r = r_cost(memo, bvh, node_left_i, i) + r_cost(memo, bvh, node_right_i, t - i);
        cost[t - 1] = fminf(cost[t - 1], r);
      }
      cost[0] = fminf(cost[0], t_cost + cost[t - 1]);
    }
    memo[node_i] = cost;
  }
  const std::vector<float>& m = memo[node_i];
  if (cutsize == 0) return 0.0f;
  float cut_min = m[0];
  for (size_t i = 1; i < cutsize; i++) cut_min = fminf(cut_min, m[i]);
  return cut_min;
}

// node_flat_cost (bvh4.rs:228-240)
float node_flat_cost(const Memo& memo, const std::vector<BVHNode>& bvh, size_t node_i, size_t cutsize) {
  if (is_leaf(bvh[node_i])) return 1.0f;
  if (memo[node_i].empty()) return INFINITY;
  const std::vector<float>& m = memo[node_i];
  float cut_min = m[0];
  for (size_t i = 1; i < cutsize; i++) cut_min = fminf(cut_min, m[i]);
  return cut_min;
}

// find_t (bvh4.rs:189-205)
size_t find_t(const std::vector<BVHNode>& bvh, const Memo& memo, size_t node_i, size_t cutsize) {
  if (is_leaf(bvh[node_i])) return 1;
  const std::vector<float>& m = memo[node_i];
  size_t t_min = 1;
  float t_min_val = m[0];
  for (size_t t = 2; t < cutsize + 1; t++) {
    if (m[t - 1] < t_min_val) {
      t_min = t;
      t_min_val = m[t - 1];
    }
  }
  return t_min;
}

// find_i (bvh4.rs:210-224)
size_t find_i(const std::vector<BVHNode>& bvh, const Memo& memo, size_t l, size_t r, size_t t) {
  size_t i_min = 1;
  float i_min_val = node_flat_cost(memo, bvh, l, 1) + node_flat_cost(memo, bvh, r, t - 1);
  for (size_t i = 2; i < t; i++) {
    const float v = node_flat_cost(memo, bvh, l, i) + node_flat_cost(memo, bvh, r, t - i);
    if (v < i_min_val) {
      i_min = i;
      i_min_val = v;
    }
  }
  return i_min;
}

// AABBx4::extract_hull (aabb.rs) over the first n boxes
AABB hull(const AABB* b, size_t n) {
  AABB h = b[0];
  for (size_t i = 1; i < n; i++) h = aabb_join(h, b[i]);
  return h;
}

// collapse_with (bvh4.rs:127-185)
std::vector<std::pair<AABB, int32_t>> collapse_with(BVH4& dst, const std::vector<BVHNode>& bvh, const Memo& memo,
                                                    size_t node_i, size_t cutsize) {
  if (is_leaf(bvh[node_i])) {
    // F4 fix: the shape range goes to the leaf list instead of count << 27
    dst.leaves.push_back({bvh[node_i].left_first, bvh[node_i].count});
    return {{bvh[node_i].bounds, -(int32_t)dst.leaves.size()}};
  }
  const size_t node_left_i = bvh[node_i].left_first;
  const size_t node_right_i = node_left_i + 1;
  const size_t t = find_t(bvh, memo, node_i, cutsize);
  if (t == 1) {
    const size_t index = dst.nodes.size();
    dst.nodes.push_back(BVHNode4{});
    const size_t i_min = find_i(bvh, memo, node_left_i, node_right_i, 4);
    const auto lcs = collapse_with(dst, bvh, memo, node_left_i, i_min);
    const auto rcs = collapse_with(dst, bvh, memo, node_right_i, 4 - i_min);
    BVHNode4 n{};
    size_t j = 0;
    for (const auto& e : lcs) { n.children[j] = e.second; n.child_bounds[j] = e.first; j++; }
    for (const auto& e : rcs) { n.children[j] = e.second; n.child_bounds[j] = e.first; j++; }
    n.num_children = (uint32_t)(lcs.size() + rcs.size());
    dst.nodes[index] = n;
    return {{hull(n.child_bounds, n.num_children), (int32_t)index}};
  }
  const size_t i_min = find_i(bvh, memo, node_left_i, node_right_i, t);
  auto c1 = collapse_with(dst, bvh, memo, node_left_i, i_min);
  const auto c2 = collapse_with(dst, bvh, memo, node_right_i, t - i_min);
  c1.insert(c1.end(), c2.begin(), c2.end());
  return c1;
}
}  // namespace

// BVHNode4::collapse (bvh4.rs:37-70)
BVH4 collapse_bvh4(const std::vector<BVHNode>& bvh2) {
  BVH4 dst;
  if (bvh2.empty()) return dst;
  Memo memo(bvh2.size());
  r_cost(memo, bvh2, 0, 4);
  const auto res = collapse_with(dst, bvh2, memo, 0, 4);
  if (res.size() > 1 || res[0].second < 0) {
    // the root is not a kept node (or is a leaf, where the reference's assert
    // would panic): rebuild with a placeholder root holding the results
    dst.nodes.clear();
    dst.leaves.clear();
    dst.nodes.push_back(BVHNode4{});
    const auto res2 = collapse_with(dst, bvh2, memo, 0, 4);
    BVHNode4 n{};
    for (size_t i = 0; i < res2.size(); i++) {
      n.child_bounds[i] = res2[i].first;
      n.children[i] = res2[i].second;
    }
    n.num_children = (uint32_t)res2.size();
    dst.nodes[0] = n;
  }
  return dst;
}

}  // namespace ref
