// wpt_scene.cpp — scene catalogue and the reference-exact BVH2 builder.
//
// The builder restates src/graphics/bvh.rs:103-437 over index arrays instead
// of Rc clones: 16 bins on the centroid of the parent box's longest axis, the
// greedy two-pointer bin sweep (bvh.rs:328-367), the SAH acceptance test
// (bvh.rs:264-268), infinite shapes moved to the front (bvh.rs:376-394) and
// the post-build shape reorder (bvh.rs:119-121) that also fixes the light order.
#include "wpt_scene.h"

#include <algorithm>
#include <cmath>

#include <algorithm>
#include <cstring>

namespace wpt {

namespace {

struct Box {
  float x0, y0, z0, x1, y1, z1;  // x_min,y_min,z_min,x_max,y_max,z_max (aabb.rs:11-18)
};
inline Box join(const Box& a, const Box& o) {  // aabb.rs:90-100
  return Box{fminf(a.x0, o.x0), fminf(a.y0, o.y0), fminf(a.z0, o.z0),
             fmaxf(a.x1, o.x1), fmaxf(a.y1, o.y1), fmaxf(a.z1, o.z1)};
}
inline float surface(const Box& b) {  // aabb.rs:72-78
  float xs = b.x1 - b.x0, ys = b.y1 - b.y0, zs = b.z1 - b.z0;
  return 2.0f * (xs * ys + xs * zs + ys * zs);
}

// Bounded::aabb / location for each primitive.
bool shape_bounds(const Shape& s, Box* b, V3* loc) {
  switch (s.kind) {
    case kTri: {  // triangle.rs:48-66, location = aabb centre (ray.rs:69-88)
      const float* g = s.g;
      const float e = kTriSlack;
      b->x0 = fminf(fminf(g[0], g[3]), g[6]) - e;
      b->y0 = fminf(fminf(g[1], g[4]), g[7]) - e;
      b->z0 = fminf(fminf(g[2], g[5]), g[8]) - e;
      b->x1 = fmaxf(fmaxf(g[0], g[3]), g[6]) + e;
      b->y1 = fmaxf(fmaxf(g[1], g[4]), g[7]) + e;
      b->z1 = fmaxf(fmaxf(g[2], g[5]), g[8]) + e;
      *loc = mk(0.5f * (b->x0 + b->x1), 0.5f * (b->y0 + b->y1), 0.5f * (b->z0 + b->z1));
      return true;
    }
    case kSphere: {  // sphere.rs:31-42
      float x = s.g[0], y = s.g[1], z = s.g[2], r = s.g[3];
      *b = Box{x - r, y - r, z - r, x + r, y + r, z + r};
      *loc = mk(x, y, z);
      return true;
    }
    case kAARect: {  // aa_rect.rs:42-61
      const float* g = s.g;
      *b = Box{g[0], g[2], g[4], g[1], g[3], g[5]};
      *loc = mk(0.5f * (g[0] + g[1]), 0.5f * (g[2] + g[3]), 0.5f * (g[4] + g[5]));
      return true;
    }
    case kTorus: {  // torus.rs:26-50
      const float* g = s.g;
      const float r = g[3] + g[4];
      *b = Box{g[0] - r, g[1] - g[4], g[2] - r, g[0] + r, g[1] + g[4], g[2] + r};
      *loc = mk(g[0], g[1], g[2]);
      return true;
    }
    default:  // plane.rs:30-36: infinite
      return false;
  }
}

struct Builder {
  std::vector<V3> loc;
  std::vector<Box> box;
  std::vector<uint32_t> ord;                 // rep order (indices into loc/box)
  std::vector<std::vector<uint32_t>> bins;   // BinResult (bvh.rs:440-476)
  std::vector<Node2>& dst;

  explicit Builder(std::vector<Node2>& d) : bins(16), dst(d) {}

  bool hull(const uint32_t* ix, size_t n, Box* out) const {  // bvh.rs:397-407
    if (n == 0) return false;
    Box r = box[ix[0]];
    for (size_t i = 1; i < n; i++) r = join(r, box[ix[i]]);
    *out = r;
    return true;
  }
  float coord(uint32_t i, int axis) const { return axis == 0 ? loc[i].x : axis == 1 ? loc[i].y : loc[i].z; }

  bool bin(const uint32_t* xs, size_t n, int axis) {  // bvh.rs:412-437
    float min_v = coord(xs[0], axis), max_v = min_v;
    for (size_t i = 1; i < n; i++) {
      float v = coord(xs[i], axis);
      min_v = fminf(min_v, v);
      max_v = fmaxf(max_v, v);
    }
    if (min_v == max_v) return false;
    const size_t nb = bins.size();
    for (auto& b : bins) b.clear();
    float w = (max_v - min_v) / (float)nb;
    for (size_t i = 0; i < n; i++) {
      float q = floorf((coord(xs[i], axis) - min_v) / w);
      size_t sid = (q != q || q <= 0.0f) ? 0 : (q >= 1.8e19f ? ~(size_t)0 : (size_t)q);
      if (sid > nb - 1) sid = nb - 1;
      bins[sid].push_back(xs[i]);
    }
    return true;
  }
  bool bin_hull(size_t k, Box* out) const { return hull(bins[k].data(), bins[k].size(), out); }

  // bvh.rs:309-370
  bool split_axis(const uint32_t* xs, size_t n, int axis, Box* lo, Box* ro, size_t* idx) {
    const size_t nb = bins.size();
    if (n <= 1 || !bin(xs, n, axis)) return false;
    size_t l = 0, r = nb - 1;
    Box la, ra, t;
    bin_hull(l, &la);
    bin_hull(r, &ra);
    size_t lc = bins[l].size(), rc = bins[r].size();
    Box lna = bin_hull(l + 1, &t) ? join(la, t) : la;
    Box rna = bin_hull(r - 1, &t) ? join(ra, t) : ra;
    size_t lnc = lc + bins[l + 1].size(), rnc = rc + bins[r - 1].size();
    while (l + 1 < r) {
      if ((surface(lna) * (float)lnc + surface(ra) * (float)rc) < (surface(la) * (float)lc + surface(rna) * (float)rnc)) {
        l += 1; la = lna; lc = lnc;
        if (l + 1 < r) { lna = bin_hull(l + 1, &t) ? join(la, t) : la; lnc = lc + bins[l + 1].size(); }
      } else {
        r -= 1; ra = rna; rc = rnc;
        if (l + 1 < r) { rna = bin_hull(r - 1, &t) ? join(ra, t) : ra; rnc = rc + bins[r - 1].size(); }
      }
    }
    *lo = la; *ro = ra; *idx = lc;
    return true;
  }

  // bvh.rs:215-239 + split (bvh.rs:254-277) + split_longest_axis (:282-303)
  Node2 subdivide(size_t off, size_t n, const Box& parent, uint32_t depth, uint32_t* max_depth) {
    uint32_t* xs = ord.data() + off;
    Box leaf;
    if (n > 1) {
      float xsz = parent.x1 - parent.x0, ysz = parent.y1 - parent.y0, zsz = parent.z1 - parent.z0;
      int axis = (xsz > ysz) ? ((xsz > zsz) ? 0 : 2) : ((ysz > zsz) ? 1 : 2);
      Box l, r;
      size_t si;
      if (split_axis(xs, n, axis, &l, &r, &si)) {
        float utility = surface(l) * (float)si + surface(r) * (float)(n - si);
        Box pa = join(l, r);
        if (utility < surface(pa) * (float)n) {
          size_t i = 0;  // tmp_bins.write_to(shapes)
          for (auto& b : bins)
            for (uint32_t v : b) xs[i++] = v;
          size_t left_id = dst.size();
          dst.push_back(Node2{});
          dst.push_back(Node2{});
          Node2 ln = subdivide(off, si, l, depth + 1, max_depth);
          dst[left_id] = ln;
          Node2 rn = subdivide(off + si, n - si, r, depth + 1, max_depth);
          dst[left_id + 1] = rn;
          Box jb = join(l, r);
          return Node2{{jb.x0, jb.y0, jb.z0}, {jb.x1, jb.y1, jb.z1}, (uint32_t)left_id, 0u};
        }
        leaf = pa;
      } else {
        hull(xs, n, &leaf);
      }
    } else {
      hull(xs, n, &leaf);
    }
    if (depth > *max_depth) *max_depth = depth;
    return Node2{{leaf.x0, leaf.y0, leaf.z0}, {leaf.x1, leaf.y1, leaf.z1}, (uint32_t)off, (uint32_t)n};
  }
};

}  // namespace

Shape make_triangle(V3 a, V3 b, V3 c, bool emissive, V3 m) {
  Shape s{};
  s.kind = kTri;
  float g[9] = {a.x, a.y, a.z, b.x, b.y, b.z, c.x, c.y, c.z};
  memcpy(s.g, g, sizeof g);
  s.emissive = emissive;
  s.m[0] = m.x; s.m[1] = m.y; s.m[2] = m.z;
  return s;
}
Shape make_plane(V3 loc, V3 n, bool emissive, V3 m) {
  Shape s{};
  s.kind = kPlane;
  float g[6] = {loc.x, loc.y, loc.z, n.x, n.y, n.z};
  memcpy(s.g, g, sizeof g);
  s.emissive = emissive;
  s.m[0] = m.x; s.m[1] = m.y; s.m[2] = m.z;
  return s;
}
Shape make_sphere(V3 c, float r, bool emissive, V3 m) {
  Shape s{};
  s.kind = kSphere;
  s.g[0] = c.x; s.g[1] = c.y; s.g[2] = c.z; s.g[3] = r;
  s.emissive = emissive;
  s.m[0] = m.x; s.m[1] = m.y; s.m[2] = m.z;
  return s;
}
Shape make_aarect(float x0, float x1, float y0, float y1, float z0, float z1, bool emissive, V3 m) {
  Shape s{};
  s.kind = kAARect;
  float g[6] = {x0, x1, y0, y1, z0, z1};
  memcpy(s.g, g, sizeof g);
  s.emissive = emissive;
  s.m[0] = m.x; s.m[1] = m.y; s.m[2] = m.z;
  return s;
}
Shape make_torus(V3 loc, float big_r, float small_r, bool emissive, V3 m) {
  Shape s{};
  s.kind = kTorus;
  s.g[0] = loc.x; s.g[1] = loc.y; s.g[2] = loc.z; s.g[3] = big_r; s.g[4] = small_r;
  s.emissive = emissive;
  s.m[0] = m.x; s.m[1] = m.y; s.m[2] = m.z;
  return s;
}


namespace {
uint32_t leaf_code(HostScene& sc, uint32_t first, uint32_t count) {
  if (count < 128u && first < (1u << 24)) return 0x80000000u | (count << 24) | first;
  const uint32_t k = (uint32_t)(sc.leaf_table.size() / 2);
  sc.leaf_table.push_back(first);
  sc.leaf_table.push_back(count);
  return 0xC0000000u | k;
}

// One BVH4 node for BVH2 node n2 (internal): its children, each internal
// child replaced by its own two children (up to 4 entries).
uint32_t collapse4(HostScene& sc, uint32_t n2, uint32_t level) {
  if (level > sc.depth4) sc.depth4 = level;
  const uint32_t idx = (uint32_t)sc.nodes4.size();
  sc.nodes4.push_back(Node4{});
  uint32_t kids[4];
  int nk = 0;
  const Node2& n = sc.nodes[n2];
  if (n.count != 0) {
    kids[nk++] = n2;  // a leaf root: one leaf child
  } else {
    for (uint32_t c = n.left_first; c <= n.left_first + 1; c++) {
      const Node2& cn = sc.nodes[c];
      if (cn.count == 0) {
        kids[nk++] = cn.left_first;
        kids[nk++] = cn.left_first + 1;
      } else {
        kids[nk++] = c;
      }
    }
  }
  uint32_t codes[4] = {kChildEmpty, kChildEmpty, kChildEmpty, kChildEmpty};
  for (int k = 0; k < nk; k++) {
    const Node2& kn = sc.nodes[kids[k]];
    codes[k] = kn.count != 0 ? leaf_code(sc, kn.left_first, kn.count) : collapse4(sc, kids[k], level + 1);
  }
  Node4& out = sc.nodes4[idx];  // (re-fetched: the vector may have grown)
  for (int k = 0; k < 4; k++) {
    if (k < nk) {
      const Node2& kn = sc.nodes[kids[k]];
      out.xmin[k] = kn.bmin[0]; out.ymin[k] = kn.bmin[1]; out.zmin[k] = kn.bmin[2];
      out.xmax[k] = kn.bmax[0]; out.ymax[k] = kn.bmax[1]; out.zmax[k] = kn.bmax[2];
    } else {  // empty slot: a box no ray enters
      out.xmin[k] = out.ymin[k] = out.zmin[k] = 1.0f;
      out.xmax[k] = out.ymax[k] = out.zmax[k] = -1.0f;
    }
    out.child[k] = codes[k];
    out.pad[k] = 0;
  }
  return idx;
}
}  // namespace

void build_bvh4(HostScene& sc) {
  sc.nodes4.clear();
  sc.leaf_table.clear();
  sc.depth4 = 0;
  if (sc.shapes.size() > sc.num_inf) collapse4(sc, 0, 0);
}

void scene_init(HostScene& sc, std::vector<Shape> shapes, const float bg[3]) {
  sc.background[0] = bg[0]; sc.background[1] = bg[1]; sc.background[2] = bg[2];
  sc.use_bvh = true;
  sc.nodes.clear();
  // shape_reps (bvh.rs:376-394): infinite shapes swapped to the front in order.
  Builder b(sc.nodes);
  std::vector<Shape> finite;
  uint32_t num_inf = 0;
  for (size_t i = 0; i < shapes.size(); i++) {
    Box bx;
    V3 lc;
    if (shape_bounds(shapes[i], &bx, &lc)) {
      b.loc.push_back(lc);
      b.box.push_back(bx);
      finite.push_back(shapes[i]);
    } else {
      std::swap(shapes[num_inf], shapes[i]);
      num_inf++;
    }
  }
  sc.num_inf = num_inf;
  sc.nodes.push_back(Node2{});  // placeholders (bvh.rs:107-109)
  sc.nodes.push_back(Node2{});
  sc.depth = 0;
  sc.shapes.assign(shapes.begin(), shapes.begin() + num_inf);
  if (!finite.empty()) {
    b.ord.resize(finite.size());
    for (size_t i = 0; i < finite.size(); i++) b.ord[i] = (uint32_t)i;
    for (auto& bn : b.bins) bn.reserve(finite.size());
    Box all;
    b.hull(b.ord.data(), b.ord.size(), &all);
    uint32_t maxd = 0;
    Node2 root = b.subdivide(0, finite.size(), all, 0, &maxd);
    sc.nodes[0] = root;
    sc.depth = maxd;
    for (uint32_t i : b.ord) sc.shapes.push_back(finite[i]);  // bvh.rs:119-121
  }
  sc.tri_only = true;
  for (size_t i = num_inf; i < sc.shapes.size(); i++)
    if (sc.shapes[i].kind != kTri) sc.tri_only = false;
  sc.lights.clear();
  for (size_t i = 0; i < sc.shapes.size(); i++)
    if (sc.shapes[i].emissive) sc.lights.push_back((uint32_t)i);  // scene.rs:62-66
  build_bvh4(sc);
}

namespace {
V3 clamp_color(float r, float g, float b) { return mk(clamp01(r), clamp01(g), clamp01(b)); }  // Color3::new

// museum_lights (scenes.rs:57-68): two emissive quads beside a torus
void museum_lights(std::vector<Shape>& s, float x, float y, V3 color) {
  V3 lc1 = mk(x - 1.0f, 0.0f, y + 2.8f), lc2 = mk(x + 1.0f, 0.0f, y + 2.8f);
  V3 lc3 = mk(x + 1.0f, 1.0f, y + 2.5f), lc4 = mk(x - 1.0f, 1.0f, y + 2.5f);
  s.push_back(make_triangle(lc3, lc2, lc1, true, color));
  s.push_back(make_triangle(lc4, lc3, lc1, true, color));
  lc1 = mk(x - 1.0f, 0.0f, y - 2.8f); lc2 = mk(x + 1.0f, 0.0f, y - 2.8f);
  lc3 = mk(x + 1.0f, 1.0f, y - 2.5f); lc4 = mk(x - 1.0f, 1.0f, y - 2.5f);
  s.push_back(make_triangle(lc3, lc2, lc1, true, color));
  s.push_back(make_triangle(lc4, lc3, lc1, true, color));
}

void push_bunny_light(std::vector<Shape>& s) {  // scenes.rs:85-95
  V3 lc1 = mk(-1.0f, 7.0f, 0.0f), lc2 = mk(1.0f, 7.0f, 0.0f), lc3 = mk(1.0f, 7.0f, 2.0f), lc4 = mk(-1.0f, 7.0f, 2.0f);
  s.push_back(make_triangle(lc3, lc2, lc1, true, mk(16.0f, 16.0f, 16.0f)));
  s.push_back(make_triangle(lc4, lc3, lc1, true, mk(16.0f, 16.0f, 16.0f)));
}
}  // namespace

bool build_scene(int scene_id, const std::vector<float>& mesh, HostScene& sc, std::string& err) {
  std::vector<Shape> s;
  const float black[3] = {0, 0, 0};  // Color3::BLACK (scenes.rs:110)
  if (scene_id == 2) {
    s.push_back(make_plane(mk(0.0f, -1.0f, 0.0f), mk(0.0f, 1.0f, 0.0f), false, clamp_color(1.0f, 1.0f, 1.0f)));
    s.push_back(make_plane(mk(0.0f, 0.0f, 13.0f), mk(0.0f, 0.0f, -1.0f), false, clamp_color(0.8f, 1.0f, 0.8f)));
    // Mesh::Triangled built by notify_mesh_loaded (wasm_interface.rs:300-311)
    size_t nt = mesh.size() / 9;
    V3 mat = clamp_color(1.0f, 0.4f, 0.4f);
    for (size_t i = 0; i < nt; i++) {
      const float* a = mesh.data() + 9 * i;
      V3 tr = mk(0.0f, 0.0f, 5.0f);
      V3 p0 = add(scale(mk(a[0], a[1], a[2]), 0.5f), tr);
      V3 p1 = add(scale(mk(a[3], a[4], a[5]), 0.5f), tr);
      V3 p2 = add(scale(mk(a[6], a[7], a[8]), 0.5f), tr);
      s.push_back(make_triangle(p0, p1, p2, false, mat));
    }
    push_bunny_light(s);
    scene_init(sc, s, black);
    return true;
  }
  if (scene_id == 100) {  // C1 box (build-defined from reference primitives)
    V3 white = clamp_color(0.8f, 0.8f, 0.8f);
    s.push_back(make_plane(mk(0.0f, -1.0f, 0.0f), mk(0.0f, 1.0f, 0.0f), false, white));
    s.push_back(make_plane(mk(0.0f, 3.0f, 0.0f), mk(0.0f, -1.0f, 0.0f), false, white));
    s.push_back(make_plane(mk(0.0f, 0.0f, 4.0f), mk(0.0f, 0.0f, -1.0f), false, white));
    s.push_back(make_plane(mk(-2.0f, 0.0f, 0.0f), mk(1.0f, 0.0f, 0.0f), false, clamp_color(0.75f, 0.25f, 0.25f)));
    s.push_back(make_plane(mk(2.0f, 0.0f, 0.0f), mk(-1.0f, 0.0f, 0.0f), false, clamp_color(0.25f, 0.75f, 0.25f)));
    s.push_back(make_aarect(-1.2f, -0.2f, -1.0f, 0.8f, 1.8f, 2.8f, false, white));
    s.push_back(make_aarect(0.3f, 1.3f, -1.0f, -0.2f, 0.6f, 1.6f, false, white));
    V3 a = mk(-0.5f, 2.99f, 1.5f), b = mk(0.5f, 2.99f, 1.5f), c = mk(0.5f, 2.99f, 2.5f), d = mk(-0.5f, 2.99f, 2.5f);
    s.push_back(make_triangle(c, b, a, true, mk(8.0f, 8.0f, 8.0f)));
    s.push_back(make_triangle(d, c, a, true, mk(8.0f, 8.0f, 8.0f)));
    scene_init(sc, s, black);
    return true;
  }
  if (scene_id == 101) {  // C2 spheres + planes, no BVH
    s.push_back(make_plane(mk(0.0f, -1.0f, 0.0f), mk(0.0f, 1.0f, 0.0f), false, clamp_color(1.0f, 1.0f, 1.0f)));
    s.push_back(make_plane(mk(0.0f, 0.0f, 13.0f), mk(0.0f, 0.0f, -1.0f), false, clamp_color(0.8f, 1.0f, 0.8f)));
    uint32_t g = 0xC2C2C2C2u;
    for (int i = 0; i < 16; i++) {
      float x = xs_next(g) * 6.0f - 3.0f;
      float z = xs_next(g) * 5.0f + 4.0f;
      float r = 0.3f + xs_next(g) * 0.7f;
      float cr = 0.3f + 0.7f * xs_next(g), cg = 0.3f + 0.7f * xs_next(g), cb = 0.3f + 0.7f * xs_next(g);
      s.push_back(make_sphere(mk(x, -1.0f + r, z), r, false, clamp_color(cr, cg, cb)));
    }
    push_bunny_light(s);
    scene_init(sc, s, black);
    sc.use_bvh = false;
    return true;
  }
  if (scene_id == 0) {  // setup_scene_museum (scenes.rs:15-55)
    V3 grey = clamp_color(0.7f, 0.7f, 0.7f);
    s.push_back(make_plane(mk(0.0f, -1.0f, 0.0f), mk(0.0f, 1.0f, 0.0f), false, grey));
    const float xs[9] = {-16.0f, -12.0f, -8.0f, -4.0f, 0.0f, 4.0f, 8.0f, 12.0f, 16.0f};
    V3 colors[9] = {clamp_color(1.0f, 0.3f, 0.3f), clamp_color(0.0f, 1.0f, 1.0f), clamp_color(0.3f, 0.3f, 1.0f),
                    clamp_color(1.0f, 0.0f, 0.0f), clamp_color(0.0f, 1.0f, 0.0f), clamp_color(0.0f, 0.0f, 1.0f),
                    clamp_color(1.0f, 0.0f, 1.0f), clamp_color(1.0f, 1.0f, 0.0f), clamp_color(0.3f, 1.0f, 0.3f)};
    uint32_t rng = 0xBABABEBEu;  // Rng::new, two draws (scenes.rs:30-32)
    (void)xs_next(rng);
    (void)xs_next(rng);
    const float ys[3] = {-7.5f, 0.0f, 7.5f};
    for (float y : ys) {
      for (int i = 0; i < 9; i++) {
        s.push_back(make_torus(mk(xs[i], -0.5f, y), 1.3f, 0.3f, false, clamp_color(1.0f, 1.0f, 1.0f)));
        museum_lights(s, xs[i], y, scale(colors[i], 2.5f));  // Color3::to_vec3() * 2.5
      }
      for (uint32_t i = 0; i < 9; i++) {  // Rng::shuffle (rng.rs:70-75)
        const uint32_t j = xs_next_in_range(rng, 9);
        V3 t = colors[i];
        colors[i] = colors[j];
        colors[j] = t;
      }
    }
    const float wx[8] = {-14.0f, -10.0f, -6.0f, -2.0f, 2.0f, 6.0f, 10.0f, 14.0f};
    for (float x : wx) s.push_back(make_aarect(x - 0.1f, x + 0.1f, -1.0f, 2.0f, -20.0f, 20.0f, false, grey));
    s.push_back(make_aarect(-20.0f, 20.0f, -1.0f, 2.0f, 3.75f - 0.1f, 3.75f + 0.1f, false, grey));
    s.push_back(make_aarect(-20.0f, 20.0f, -1.0f, 2.0f, -3.75f - 0.1f, -3.75f + 0.1f, false, grey));
    scene_init(sc, s, black);
    return true;
  }
  err = "Invalid scene";  // wasm_interface.rs:396
  return false;
}

}  // namespace wpt
