// wpt_scene.cpp — scene catalogue and the reference-exact BVH2 builder.
//
// The builder restates src/graphics/bvh.rs:103-437 over index arrays instead
// of Rc clones: 16 bins on the centroid of the parent box's longest axis, the
// greedy two-pointer bin sweep (bvh.rs:328-367), the SAH acceptance test
// (bvh.rs:264-268), infinite shapes moved to the front (bvh.rs:376-394) and
// the post-build shape reorder (bvh.rs:119-121) that also fixes the light order.
#include "wpt_scene.h"

#include <algorithm>
#include <chrono>
#include <cmath>
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
  // inline: count in bits 24-29 (bit 30 set marks a leaf-table index)
  if (count < 64u && first < (1u << 24)) return 0x80000000u | (count << 24) | first;
  const uint32_t k = (uint32_t)(sc.leaf_table.size() / 2);
  sc.leaf_table.push_back(first);
  sc.leaf_table.push_back(count);
  return 0xC0000000u | k;
}

// BVH4 by the reference's DP tree cut (bvh4.rs:37-281). best[n][t-1] = the
// fewest box tests (t_cost 1 per box) of BVH2 subtree n when it is replaced by
// at most... exactly t nodes (t = 1: kept as one node with up to 4 children);
// costs are small integers in f32, so the sums are exact and the
// first-minimum tie rules of find_t / find_i (bvh4.rs:189-224) pick the same
// cut as the reference. Computed bottom-up (children follow their parent in
// the BVH2 array, so a reverse sweep sees children first).
struct Collapse4 {
  HostScene& sc;
  std::vector<float> best;  // 4 per BVH2 node (internal nodes only)
  explicit Collapse4(HostScene& s) : sc(s), best(4 * s.nodes.size(), INFINITY) {}

  bool leaf(uint32_t n) const { return sc.nodes[n].count != 0; }
  // node_flat_cost / r_cost once memoised: min over replacing n by 1..k nodes
  float flat(uint32_t n, uint32_t k) const {
    if (leaf(n)) return 1.0f;
    float m = best[4 * n];
    for (uint32_t i = 1; i < k; i++) m = fminf(m, best[4 * n + i]);
    return m;
  }
  void costs() {
    for (size_t n = sc.nodes.size(); n-- > 0;) {
      if (n == 1 || leaf((uint32_t)n)) continue;  // node 1 is the unused slot (bvh.rs:108-109)
      const uint32_t l = sc.nodes[n].left_first, r = l + 1;
      float* c = &best[4 * n];
      for (uint32_t t = 2; t <= 4; t++) {
        for (uint32_t i = 1; i < t; i++) c[t - 1] = fminf(c[t - 1], flat(l, i) + flat(r, t - i));
        c[0] = fminf(c[0], 1.0f + c[t - 1]);
      }
    }
  }
  uint32_t pick_t(uint32_t n, uint32_t cut) const {  // find_t
    if (leaf(n)) return 1;
    uint32_t t = 1;
    for (uint32_t k = 2; k <= cut; k++)
      if (best[4 * n + k - 1] < best[4 * n + t - 1]) t = k;
    return t;
  }
  uint32_t pick_i(uint32_t l, uint32_t r, uint32_t t) const {  // find_i
    uint32_t i = 1;
    float v = flat(l, 1) + flat(r, t - 1);
    for (uint32_t k = 2; k < t; k++) {
      const float w = flat(l, k) + flat(r, t - k);
      if (w < v) { i = k; v = w; }
    }
    return i;
  }
  struct Entry { float b[6]; uint32_t code; };
  // collapse_with: the entries (box, child code) that replace subtree n
  void cut(uint32_t n, uint32_t cutsize, std::vector<Entry>& out, uint32_t level) {
    const Node2& nd = sc.nodes[n];
    if (leaf(n)) {
      out.push_back(Entry{{nd.bmin[0], nd.bmin[1], nd.bmin[2], nd.bmax[0], nd.bmax[1], nd.bmax[2]},
                          leaf_code(sc, nd.left_first, nd.count)});
      return;
    }
    const uint32_t l = nd.left_first, r = l + 1;
    const uint32_t t = pick_t(n, cutsize);
    if (t == 1) {
      out.push_back(Entry{{0, 0, 0, 0, 0, 0}, make_node(n, level)});
      const Node4& k = sc.nodes4[out.back().code];
      hull_of(k, out.back().b);
      return;
    }
    const uint32_t i = pick_i(l, r, t);
    cut(l, i, out, level);
    cut(r, t - i, out, level);
  }
  // a kept node: its slot first (pre-order, as dst.push before the recursion)
  uint32_t make_node(uint32_t n, uint32_t level) {
    if (level > sc.depth4) sc.depth4 = level;
    const uint32_t idx = (uint32_t)sc.nodes4.size();
    sc.nodes4.push_back(Node4{});
    const uint32_t l = sc.nodes[n].left_first, r = l + 1;
    const uint32_t i = pick_i(l, r, 4);
    std::vector<Entry> kids;
    cut(l, i, kids, level + 1);
    cut(r, 4 - i, kids, level + 1);
    fill(idx, kids);
    return idx;
  }
  void fill(uint32_t idx, const std::vector<Entry>& kids) {
    Node4& o = sc.nodes4[idx];
    for (int k = 0; k < 4; k++) {
      if (k < (int)kids.size()) {
        const float* b = kids[k].b;
        o.xmin[k] = b[0]; o.ymin[k] = b[1]; o.zmin[k] = b[2];
        o.xmax[k] = b[3]; o.ymax[k] = b[4]; o.zmax[k] = b[5];
        o.child[k] = kids[k].code;
      } else {  // unused slot: skipped by its code
        o.xmin[k] = o.ymin[k] = o.zmin[k] = 0.0f;
        o.xmax[k] = o.ymax[k] = o.zmax[k] = 0.0f;
        o.child[k] = kChildEmpty;
      }
      o.pad[k] = 0;
    }
  }
  // AABBx4::extract_hull: the union of the used child boxes
  static void hull_of(const Node4& k, float* b) {
    b[0] = k.xmin[0]; b[1] = k.ymin[0]; b[2] = k.zmin[0];
    b[3] = k.xmax[0]; b[4] = k.ymax[0]; b[5] = k.zmax[0];
    for (int c = 1; c < 4 && k.child[c] != kChildEmpty; c++) {
      b[0] = fminf(b[0], k.xmin[c]); b[1] = fminf(b[1], k.ymin[c]); b[2] = fminf(b[2], k.zmin[c]);
      b[3] = fmaxf(b[3], k.xmax[c]); b[4] = fmaxf(b[4], k.ymax[c]); b[5] = fmaxf(b[5], k.zmax[c]);
    }
  }
};
}  // namespace

void build_bvh4(HostScene& sc) {
  sc.nodes4.clear();
  sc.leaf_table.clear();
  sc.depth4 = 0;
  if (sc.shapes.size() <= sc.num_inf) return;
  Collapse4 c(sc);
  c.costs();
  // BVHNode4::collapse (bvh4.rs:37-70): the root is kept as node 0 when the
  // cut keeps it; otherwise (or for a leaf root) node 0 is a placeholder
  // holding the root's replacement entries
  if (!c.leaf(0) && c.pick_t(0, 4) == 1) {
    c.make_node(0, 0);
    return;
  }
  sc.nodes4.push_back(Node4{});
  std::vector<Collapse4::Entry> kids;
  c.cut(0, 4, kids, 1);
  c.fill(0, kids);
}

bool scene_init(HostScene& sc, std::vector<Shape> shapes, const float bg[3], Bvh2Builder* gpu, std::string* err) {
  sc.background[0] = bg[0]; sc.background[1] = bg[1]; sc.background[2] = bg[2];
  sc.use_bvh = true;
  sc.nodes.clear();
  // shape_reps (bvh.rs:376-394): infinite shapes swapped to the front in order.
  Builder b(sc.nodes);
  std::vector<Shape> finite;
  finite.reserve(shapes.size());
  b.loc.reserve(shapes.size());
  b.box.reserve(shapes.size());
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
  sc.shapes.reserve(shapes.size());
  sc.shapes.assign(shapes.begin(), shapes.begin() + num_inf);
  sc.bvh_on_gpu = false;
  sc.bvh_ms = 0.0;
  if (!finite.empty() && gpu && finite.size() >= gpu->min_shapes) {
    static_assert(sizeof(Box) == 6 * sizeof(float) && sizeof(V3) == 3 * sizeof(float), "packed boxes");
    std::string e;
    if (!gpu->build(&b.box[0].x0, &b.loc[0].x, finite.size(), sc.nodes, b.ord, sc.depth, sc.bvh_ms, e)) {
      if (err) *err = e;
      return false;
    }
    sc.bvh_on_gpu = true;
    for (uint32_t i : b.ord) sc.shapes.push_back(finite[i]);  // bvh.rs:119-121
  } else if (!finite.empty()) {
    const auto t0 = std::chrono::steady_clock::now();
    b.ord.resize(finite.size());
    for (size_t i = 0; i < finite.size(); i++) b.ord[i] = (uint32_t)i;
    for (auto& bn : b.bins) bn.reserve(finite.size());
    Box all;
    b.hull(b.ord.data(), b.ord.size(), &all);
    uint32_t maxd = 0;
    Node2 root = b.subdivide(0, finite.size(), all, 0, &maxd);
    sc.nodes[0] = root;
    sc.depth = maxd;
    sc.bvh_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (uint32_t i : b.ord) sc.shapes.push_back(finite[i]);  // bvh.rs:119-121
  }
  sc.tri_only = true;
  for (size_t i = num_inf; i < sc.shapes.size(); i++)
    if (sc.shapes[i].kind != kTri) sc.tri_only = false;
  sc.lights.clear();
  for (size_t i = 0; i < sc.shapes.size(); i++)
    if (sc.shapes[i].emissive) sc.lights.push_back((uint32_t)i);  // scene.rs:62-66
  sc.nodes4.clear();
  sc.leaf_table.clear();
  sc.depth4 = 0;
  if (sc.want_bvh4 == 1 || (sc.want_bvh4 == 2 && !sc.tri_only && sc.use_bvh)) build_bvh4(sc);
  return true;
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

bool build_scene(int scene_id, const std::vector<float>& mesh, HostScene& sc, std::string& err, Bvh2Builder* gpu) {
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
    if (!scene_init(sc, std::move(s), black, gpu, &err)) return false;
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
    if (!scene_init(sc, std::move(s), black, gpu, &err)) return false;
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
    if (!scene_init(sc, std::move(s), black, gpu, &err)) return false;
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
    if (!scene_init(sc, std::move(s), black, gpu, &err)) return false;
    return true;
  }
  err = "Invalid scene";  // wasm_interface.rs:396
  return false;
}

}  // namespace wpt
