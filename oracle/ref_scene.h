// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see ref_core.h header).
// Restates src/graphics/{ray,aabb,bvh,scene}.rs and primitives/ of
// sourcedennis/wasm-pathtracer in the reference's own structure: shapes behind
// a virtual `Tracable` interface (AoS, heap objects), recursive BVH2 build and
// recursive ordered BVH2 traversal.
// ============================================================================
#pragma once
#include <memory>
#include <vector>
#include "ref_core.h"
#include "ref_quartic.h"

namespace ref {

// ray.rs:22-33
struct Ray {
  Vec3 origin, dir, inv_dir;
};
inline Ray make_ray(Vec3 o, Vec3 d) { return Ray{o, d, v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z)}; }
inline Vec3 ray_at(const Ray& r, float t) { return r.origin + t * r.dir; }  // ray.rs:37-39

// material.rs:16-20 / 70-75
struct Material {
  bool emissive = false;
  Color3 color{0, 0, 0};   // Diffuse
  Vec3 intensity{0, 0, 0}; // Emissive
};
inline Material diffuse(Color3 c) { Material m; m.emissive = false; m.color = c; return m; }
inline Material emissive(Vec3 i) { Material m; m.emissive = true; m.intensity = i; return m; }

// ray.rs:46-62 (normal normalised by Hit::new)
struct Hit {
  float distance;
  Vec3 normal;
  Material mat;
  bool is_entering;
};
inline Hit make_hit(float t, Vec3 n, const Material& m, bool ent) { return Hit{t, normalize(n), m, ent}; }

// aabb.rs:11-18
struct AABB {
  float x_min, y_min, z_min, x_max, y_max, z_max;
};
inline AABB aabb_empty() { return AABB{0, 0, 0, 0, 0, 0}; }
inline float aabb_surface(const AABB& b) {  // aabb.rs:72-78
  float xs = b.x_max - b.x_min, ys = b.y_max - b.y_min, zs = b.z_max - b.z_min;
  return 2.0f * (xs * ys + xs * zs + ys * zs);
}
inline Vec3 aabb_center(const AABB& b) {  // aabb.rs:81-87
  return v3(0.5f * (b.x_min + b.x_max), 0.5f * (b.y_min + b.y_max), 0.5f * (b.z_min + b.z_max));
}
inline AABB aabb_join(const AABB& a, const AABB& o) {  // aabb.rs:90-100
  return AABB{fminf(a.x_min, o.x_min), fminf(a.y_min, o.y_min), fminf(a.z_min, o.z_min),
              fmaxf(a.x_max, o.x_max), fmaxf(a.y_max, o.y_max), fmaxf(a.z_max, o.z_max)};
}
inline bool aabb_contains(const AABB& s, const AABB& o) {  // aabb.rs:113-120
  return o.x_min >= s.x_min && o.y_min >= s.y_min && o.z_min >= s.z_min && o.x_max <= s.x_max &&
         o.y_max <= s.y_max && o.z_max <= s.z_max;
}
// aabb.rs:132-164. Returns false for None.
inline bool aabb_hit(const AABB& b, const Ray& ray, float* out) {
  float invdx = ray.inv_dir.x, invdy = ray.inv_dir.y, invdz = ray.inv_dir.z;
  float tx1 = (b.x_min - ray.origin.x) * invdx;
  float tx2 = (b.x_max - ray.origin.x) * invdx;
  float ty1 = (b.y_min - ray.origin.y) * invdy;
  float ty2 = (b.y_max - ray.origin.y) * invdy;
  float tz1 = (b.z_min - ray.origin.z) * invdz;
  float tz2 = (b.z_max - ray.origin.z) * invdz;
  float txmin = fminf(tx1, tx2), tymin = fminf(ty1, ty2), tzmin = fminf(tz1, tz2);
  float txmax = fmaxf(tx1, tx2), tymax = fmaxf(ty1, ty2), tzmax = fmaxf(tz1, tz2);
  float tmin = fmaxf(fmaxf(txmin, tymin), tzmin);
  float tmax = fminf(fminf(txmax, tymax), tzmax);
  if (tmin > tmax) return false;
  if (tmin >= 0.0f) { *out = tmin; return true; }
  if (tmax >= 0.0f) { *out = 0.0f; return true; }
  return false;
}

// ---------------------------------------------------------------------------
// Tracable (ray.rs:69-121): the reference's shape plugin interface.
// ---------------------------------------------------------------------------
struct PickResult {
  Vec3 point, normal, intensity;
};
struct Tracable {
  virtual ~Tracable() {}
  virtual bool aabb(AABB* out) const = 0;             // Bounded::aabb
  virtual bool location(Vec3* out) const {            // Bounded::location (ray.rs:69-88)
    AABB b;
    if (!aabb(&b)) return false;
    *out = aabb_center(b);
    return true;
  }
  virtual bool is_emissive() const = 0;
  virtual float surface_area() const { return 0.0f; }  // reference panics
  virtual PickResult pick_random(Rng&) const { return PickResult{{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}; }
  virtual bool trace_simple(const Ray& r, float* t) const = 0;
  virtual bool trace(const Ray& r, Hit* h) const = 0;
  virtual int kind() const = 0;  // 0 tri, 1 plane, 2 sphere, 3 aarect, 4 torus (for fixture dumps)
};
typedef std::shared_ptr<Tracable> ShapeP;

// triangle.rs:41-45
inline bool is_approx_left_of(Vec3 v0, Vec3 v1, Vec3 n, Vec3 p) {
  Vec3 edge = v1 - v0;
  Vec3 v0p = p - v0;
  return dot(n, cross(edge, v0p)) + 0.1f * EPSILON >= 0.0f;
}

// triangle.rs:11-192
struct Triangle : Tracable {
  Vec3 v0, v1, v2;
  Material mat;
  Triangle(Vec3 a, Vec3 b, Vec3 c, Material m) : v0(a), v1(b), v2(c), mat(m) {}
  int kind() const override { return 0; }
  bool aabb(AABB* out) const override {  // :48-66
    float x_min = fminf(fminf(v0.x, v1.x), v2.x);
    float y_min = fminf(fminf(v0.y, v1.y), v2.y);
    float z_min = fminf(fminf(v0.z, v1.z), v2.z);
    float x_max = fmaxf(fmaxf(v0.x, v1.x), v2.x);
    float y_max = fmaxf(fmaxf(v0.y, v1.y), v2.y);
    float z_max = fmaxf(fmaxf(v0.z, v1.z), v2.z);
    const float e = 0.1f * EPSILON;
    *out = AABB{x_min - e, y_min - e, z_min - e, x_max + e, y_max + e, z_max + e};
    return true;
  }
  bool is_emissive() const override { return mat.emissive; }
  float surface_area() const override {  // :70-78 (Heron)
    float a = dis(v0, v1), b = dis(v1, v2), c = dis(v2, v0);
    float s = (a + b + c) * 0.5f;
    return sqrtf(s * (s - a) * (s - b) * (s - c));
  }
  PickResult pick_random(Rng& rng) const override {  // :91-114
    float r1 = rng.next();
    float r2 = rng.next();
    float r1_sqrt = sqrtf(r1);
    Vec3 p_hit = (1.0f - r1_sqrt) * v0 + (r1_sqrt * (1.0f - r2)) * v1 + (r2 * r1_sqrt) * v2;
    Vec3 n = normalize(cross(v1 - v0, v2 - v0));
    if (rng.next() > 0.5f) n = -n;
    if (mat.emissive) return PickResult{p_hit, n, mat.intensity};
    return PickResult{{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  }
  bool trace_simple(const Ray& ray, float* tout) const override {  // :159-191
    Vec3 n = cross(v1 - v0, v2 - v0);
    float n_dot_d = dot(n, ray.dir);
    if (n_dot_d == 0.0f) return false;
    float orig_dis = dot(n, v0);
    float t = (orig_dis - dot(n, ray.origin)) / n_dot_d;
    if (t <= 0.0f) return false;
    n = normalize(n);
    Vec3 p = ray_at(ray, t);
    if (is_approx_left_of(v0, v1, n, p) && is_approx_left_of(v1, v2, n, p) && is_approx_left_of(v2, v0, n, p)) {
      *tout = t;
      return true;
    }
    return false;
  }
  bool trace(const Ray& ray, Hit* h) const override {  // :116-157
    Vec3 n = cross(v1 - v0, v2 - v0);
    float n_dot_d = dot(n, ray.dir);
    if (n_dot_d == 0.0f) return false;
    float orig_dis = dot(n, v0);
    float t = (orig_dis - dot(n, ray.origin)) / n_dot_d;
    if (t <= 0.0f) return false;
    n = normalize(n);
    Vec3 p = ray_at(ray, t);
    if (is_approx_left_of(v0, v1, n, p) && is_approx_left_of(v1, v2, n, p) && is_approx_left_of(v2, v0, n, p)) {
      if (n_dot_d > 0.0f) *h = make_hit(t, -n, mat, false);
      else *h = make_hit(t, n, mat, true);
      return true;
    }
    return false;
  }
};

// plane.rs:10-100 (infinite; never in the BVH)
struct Plane : Tracable {
  Vec3 loc, normal;
  Material mat;
  Plane(Vec3 l, Vec3 n, Material m) : loc(l), normal(n), mat(m) {}
  int kind() const override { return 1; }
  bool aabb(AABB*) const override { return false; }
  bool location(Vec3*) const override { return false; }
  bool is_emissive() const override { return mat.emissive; }
  bool trace_simple(const Ray& ray, float* tout) const override {  // :272-291
    float n_dot_dir = dot(normal, ray.dir);
    if (n_dot_dir == 0.0f) return false;
    float o_distance = dot(normal, loc);
    float t = (o_distance - dot(normal, ray.origin)) / n_dot_dir;
    if (t <= 0.0f) return false;
    *tout = t;
    return true;
  }
  bool trace(const Ray& ray, Hit* h) const override {  // :237-269
    Vec3 nn = normal;
    float n_dot_dir = dot(nn, ray.dir);
    if (n_dot_dir == 0.0f) return false;
    float o_distance = dot(nn, loc);
    float t = (o_distance - dot(nn, ray.origin)) / n_dot_dir;
    if (t <= 0.0f) return false;
    if (n_dot_dir > 0.0f) nn = -nn;
    *h = make_hit(t, nn, mat, true);
    return true;
  }
};

// sphere.rs:10-132
struct Sphere : Tracable {
  Vec3 loc;
  float radius;
  Material mat;
  Sphere(Vec3 l, float r, Material m) : loc(l), radius(r), mat(m) {}
  int kind() const override { return 2; }
  bool location(Vec3* o) const override { *o = loc; return true; }
  bool aabb(AABB* out) const override {
    *out = AABB{loc.x - radius, loc.y - radius, loc.z - radius, loc.x + radius, loc.y + radius, loc.z + radius};
    return true;
  }
  bool is_emissive() const override { return mat.emissive; }
  // shared root finding of sphere.rs:49-102 / :104-131
  bool roots(const Ray& ray, float* tout, bool* entering) const {
    float a = 1.0f;
    float b = 2.0f * dot(ray.dir, ray.origin - loc);
    float c = dot(ray.origin - loc, ray.origin - loc) - radius * radius;
    float d = b * b - 4.0f * a * c;
    if (d < 0.0f) return false;
    float d_sqrt = sqrtf(d);
    float t0 = (-b + d_sqrt) / (2.0f * a);
    float t1 = (-b - d_sqrt) / (2.0f * a);
    float t = fminf(t0, t1);
    *entering = true;
    if (t <= 0.0f) {
      t = fmaxf(t0, t1);
      if (t <= 0.0f) return false;
      *entering = false;
    }
    *tout = t;
    return true;
  }
  bool trace_simple(const Ray& ray, float* tout) const override {
    bool ent;
    return roots(ray, tout, &ent);
  }
  bool trace(const Ray& ray, Hit* h) const override {
    float t;
    bool ent;
    if (!roots(ray, &t, &ent)) return false;
    Vec3 normal = (ray_at(ray, t) - loc) / radius;
    if (!ent) normal = -normal;
    *h = make_hit(t, normal, mat, ent);
    return true;
  }
};

// torus.rs:8-127 (f64 quartic, ref_quartic.h; parity unpinned: roots 0.0.4)
struct Torus : Tracable {
  Vec3 loc;
  float big_r, small_r;
  Material mat;
  Torus(Vec3 l, float a, float b, Material m) : loc(l), big_r(a), small_r(b), mat(m) {}
  int kind() const override { return 4; }
  bool location(Vec3* o) const override { *o = loc; return true; }
  bool aabb(AABB* out) const override {  // :26-50
    float r = big_r + small_r;
    *out = AABB{loc.x - r, loc.y - small_r, loc.z - r, loc.x + r, loc.y + small_r, loc.z + r};
    return true;
  }
  bool is_emissive() const override { return mat.emissive; }
  bool trace_simple(const Ray& ray, float* tout) const override {  // ray.rs:111-117 default
    Hit h;
    if (!trace(ray, &h)) return false;
    *tout = h.distance;
    return true;
  }
  bool trace(const Ray& ray, Hit* h) const override {
    float t;
    Vec3 n;
    bool ent;
    if (!torus_trace(loc, big_r, small_r, ray.origin, ray.dir, &t, &n, &ent)) return false;
    *h = Hit{t, n, mat, ent};  // n is already Hit::new-normalised
    return true;
  }
};

// aa_rect.rs:8-175
struct AARect : Tracable {
  float x_min, x_max, y_min, y_max, z_min, z_max;
  Material mat;
  AARect(float a, float b, float c, float d, float e, float f, Material m)
      : x_min(a), x_max(b), y_min(c), y_max(d), z_min(e), z_max(f), mat(m) {}
  int kind() const override { return 3; }
  bool location(Vec3* o) const override {
    *o = v3(0.5f * (x_min + x_max), 0.5f * (y_min + y_max), 0.5f * (z_min + z_max));
    return true;
  }
  bool aabb(AABB* out) const override {
    *out = AABB{x_min, y_min, z_min, x_max, y_max, z_max};
    return true;
  }
  bool is_emissive() const override { return mat.emissive; }
  void slab(const Ray& ray, float* t6, float* tmin, float* tmax) const {
    float invdx = 1.0f / ray.dir.x, invdy = 1.0f / ray.dir.y, invdz = 1.0f / ray.dir.z;
    t6[0] = (x_min - ray.origin.x) * invdx;
    t6[1] = (x_max - ray.origin.x) * invdx;
    t6[2] = (y_min - ray.origin.y) * invdy;
    t6[3] = (y_max - ray.origin.y) * invdy;
    t6[4] = (z_min - ray.origin.z) * invdz;
    t6[5] = (z_max - ray.origin.z) * invdz;
    float txmin = fminf(t6[0], t6[1]), tymin = fminf(t6[2], t6[3]), tzmin = fminf(t6[4], t6[5]);
    float txmax = fmaxf(t6[0], t6[1]), tymax = fmaxf(t6[2], t6[3]), tzmax = fmaxf(t6[4], t6[5]);
    *tmin = fmaxf(fmaxf(txmin, tymin), tzmin);
    *tmax = fminf(fminf(txmax, tymax), tzmax);
  }
  bool trace_simple(const Ray& ray, float* tout) const override {
    float t6[6], tmin, tmax;
    slab(ray, t6, &tmin, &tmax);
    if (tmin >= tmax) return false;
    if (tmin > 0.0f) { *tout = tmin; return true; }
    if (tmax > 0.0f) { *tout = tmax; return true; }
    return false;
  }
  bool trace(const Ray& ray, Hit* h) const override {
    float t6[6], tmin, tmax;
    slab(ray, t6, &tmin, &tmax);
    if (tmin >= tmax) return false;
    if (tmin > 0.0f) {
      Vec3 n;
      if (tmin == t6[0]) n = v3(-1, 0, 0);
      else if (tmin == t6[1]) n = v3(1, 0, 0);
      else if (tmin == t6[2]) n = v3(0, -1, 0);
      else if (tmin == t6[3]) n = v3(0, 1, 0);
      else if (tmin == t6[4]) n = v3(0, 0, -1);
      else n = v3(0, 0, 1);
      *h = make_hit(tmin, n, mat, true);
      return true;
    }
    if (tmax > 0.0f) {
      Vec3 n;
      if (tmax == t6[0]) n = v3(1, 0, 0);
      else if (tmax == t6[1]) n = v3(-1, 0, 0);
      else if (tmax == t6[2]) n = v3(0, 1, 0);
      else if (tmax == t6[3]) n = v3(0, -1, 0);
      else if (tmax == t6[4]) n = v3(0, 0, 1);
      else n = v3(0, 0, -1);
      *h = make_hit(tmax, n, mat, false);
      return true;
    }
    return false;
  }
};

// ---------------------------------------------------------------------------
// BVH2 — src/graphics/bvh.rs
// ---------------------------------------------------------------------------
struct BVHNode {  // bvh.rs:14-20 (32 B, align 32)
  AABB bounds;
  uint32_t left_first;
  uint32_t count;
};

// Builds the BVH over `shapes` (reordering them exactly as the reference:
// infinite shapes first, then the finite shapes in leaf order). Returns num_inf.
size_t build_bvh(std::vector<ShapeP>& shapes, size_t num_bins, std::vector<BVHNode>& out);
bool verify_bvh(const std::vector<ShapeP>& shapes, size_t num_inf, const std::vector<BVHNode>& bvh);

// ---------------------------------------------------------------------------
// BVH4 collapse — src/graphics/bvh4.rs:37-281 (dead in the reference's live
// path; the layout the north_star names). The DP tree cut is
// restated as written; the leaf encoding is the F4 fix: the reference packs
// `count << 27` and decodes `& 0x3` (bvh4.rs:135, :322), which loses leaves of
// 4+ shapes, so a leaf child here is -(1 + index) into `leaves` (first, count).
// ---------------------------------------------------------------------------
struct BVHNode4 {       // bvh4.rs:17-26
  AABB child_bounds[4];
  int32_t children[4];  // >= 0: node index; < 0: leaf -(1 + leaf index)
  uint32_t num_children;
};
struct BVH4 {
  std::vector<BVHNode4> nodes;                        // root at 0
  std::vector<std::pair<uint32_t, uint32_t>> leaves;  // (first shape, count) after the infinite shapes
};
// BVHNode4::collapse (bvh4.rs:37-70) of a BVH2 built by build_bvh.
BVH4 collapse_bvh4(const std::vector<BVHNode>& bvh2);

// ---------------------------------------------------------------------------
// Scene — src/graphics/scene.rs
// ---------------------------------------------------------------------------
enum BvhKind { BVH_NONE = 0, BVH_2 = 2 };

struct Scene {
  Color3 background{0, 0, 0};
  std::vector<size_t> lights;  // LightEnum::Area(shape index)
  std::vector<ShapeP> shapes;
  std::vector<BVHNode> bvh;
  size_t num_inf = 0;
  BvhKind kind = BVH_2;

  // scene.rs:43-69: builds the BVH2 (reordering shapes), then collects lights
  void init(Color3 bg, std::vector<ShapeP> s);
  void disable_bvh() { kind = BVH_NONE; }  // scene.rs:99-101

  // trace_g (scene.rs:162-184). Returns node visits; sets *hit_found.
  size_t trace_g(const Ray& ray, float* t, size_t* id, bool* hit_found) const;
  // scene.rs:137-144
  size_t trace(const Ray& ray, Hit* hit, bool* ok, size_t* id_out = nullptr) const;
  // scene.rs:104-133
  size_t shadow_ray(Vec3 p, Vec3 q, long light_shape, bool* occluded) const;
};

}  // namespace ref
