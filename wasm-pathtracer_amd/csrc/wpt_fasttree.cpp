// wpt_fasttree.cpp — SAH + SBVH build of the fast path's traversal tree
// (wpt_fasttree.h). Nothing here decides a result: the tree only has to hold
// every triangle hit point inside its leaf boxes (conservative boxes, below);
// which shape wins is settled by the traversal's tie / reference-leaf checks
// and, for flagged rays, by the exact BVH2 machine (wpt_render.hip).
#include "wpt_fasttree.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <thread>

namespace wpt {

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

struct DBox {
  double lo[3] = {kInf, kInf, kInf};
  double hi[3] = {-kInf, -kInf, -kInf};
  bool empty() const { return !(lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2]); }
  void grow(const DBox& b) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  void grow(const double* p) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  double area() const {
    if (empty()) return 0.0;
    const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
    return 2.0 * (x * y + x * z + y * z);
  }
};

inline DBox meet(const DBox& a, const DBox& b) {
  DBox r;
  for (int k = 0; k < 3; k++) {
    r.lo[k] = std::max(a.lo[k], b.lo[k]);
    r.hi[k] = std::min(a.hi[k], b.hi[k]);
  }
  return r;
}

// The region Triangle::trace_simple accepts, as a planar polygon: the three
// edge tests dot(nn, cross(e_i, p - v_i)) + slack >= 0 are q_i·(p - v_i) >=
// -slack with q_i = nn × e_i (a·(b×c) = (a×b)·c), i.e. the triangle with each
// edge line pushed out by slack / |q_i|. Its vertices: the meeting points of
// neighbouring pushed-out lines, in the plane through the vertex normal to nn.
struct Poly {
  double v[3][3];
};

bool solve3(const double a[3][3], const double b[3], double x[3]) {
  const double det = a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) -
                     a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
                     a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
  if (!(std::fabs(det) > 0.0) || !std::isfinite(det)) return false;
  for (int c = 0; c < 3; c++) {
    double m[3][3];
    for (int r = 0; r < 3; r++)
      for (int k = 0; k < 3; k++) m[r][k] = k == c ? b[r] : a[r][k];
    const double dc = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
                      m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                      m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    x[c] = dc / det;
    if (!std::isfinite(x[c])) return false;
  }
  return true;
}

// 0: ok; 1: never hit (the record's n is zero: n·d == 0 for every d);
// 2: not supported (non-finite data, or no bounded offset region)
int offset_triangle(const Shape& s, Poly& P) {
  const float* g = s.g;
  for (int k = 0; k < 9; k++)
    if (!std::isfinite(g[k])) return 2;
  // the record's normals, computed as the upload does (wpt_render.hip rec())
  const V3 v0 = mk(g[0], g[1], g[2]), v1 = mk(g[3], g[4], g[5]), v2 = mk(g[6], g[7], g[8]);
  const V3 n = cross(sub(v1, v0), sub(v2, v0));
  if (n.x == 0.0f && n.y == 0.0f && n.z == 0.0f) return 1;
  if (!std::isfinite(n.x) || !std::isfinite(n.y) || !std::isfinite(n.z)) return 2;
  const V3 nnf = normalize(n);
  if (!std::isfinite(nnf.x) || !std::isfinite(nnf.y) || !std::isfinite(nnf.z)) return 2;
  const double nn[3] = {nnf.x, nnf.y, nnf.z};
  const double v[3][3] = {{g[0], g[1], g[2]}, {g[3], g[4], g[5]}, {g[6], g[7], g[8]}};
  double q[3][3], c[3];
  for (int i = 0; i < 3; i++) {
    const double* a = v[i];
    const double* b = v[(i + 1) % 3];
    const double e[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    q[i][0] = nn[1] * e[2] - nn[2] * e[1];
    q[i][1] = nn[2] * e[0] - nn[0] * e[2];
    q[i][2] = nn[0] * e[1] - nn[1] * e[0];
    c[i] = q[i][0] * a[0] + q[i][1] * a[1] + q[i][2] * a[2] - (double)kTriSlack;
  }
  for (int i = 0; i < 3; i++) {  // vertex i: edges i-1 and i meet there
    const int j = (i + 2) % 3;
    const double A[3][3] = {{q[j][0], q[j][1], q[j][2]}, {q[i][0], q[i][1], q[i][2]}, {nn[0], nn[1], nn[2]}};
    const double B[3] = {c[j], c[i], nn[0] * v[i][0] + nn[1] * v[i][1] + nn[2] * v[i][2]};
    if (!solve3(A, B, P.v[i])) return 2;
  }
  return 0;
}

float down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return f;
}
float up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
  return f;
}

struct Ref {
  uint32_t prim;
  DBox b;
};

struct Bin {
  DBox b;
  uint32_t n = 0, enter = 0, exit = 0;
};

// Convex polygon (a clipped hit region) and its cut by an axis plane.
struct PolyN {
  int n = 0;
  double v[16][3];
};
void to_polyn(const Poly& P, PolyN& Q) {
  Q.n = 3;
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) Q.v[i][k] = P.v[i][k];
}
void box_of(const PolyN& P, DBox& b) {
  b = DBox();
  for (int i = 0; i < P.n; i++) b.grow(P.v[i]);
}
// L = P ∩ {x_axis <= c}, R = P ∩ {x_axis >= c}
void cut(const PolyN& P, int axis, double c, PolyN& L, PolyN& R) {
  L.n = R.n = 0;
  for (int i = 0; i < P.n; i++) {
    const double* p = P.v[i];
    const double* q = P.v[(i + 1) % P.n];
    const bool pl = p[axis] <= c, pr = p[axis] >= c;
    if (pl && L.n < 16) { for (int k = 0; k < 3; k++) L.v[L.n][k] = p[k]; L.n++; }
    if (pr && R.n < 16) { for (int k = 0; k < 3; k++) R.v[R.n][k] = p[k]; R.n++; }
    if ((p[axis] < c && q[axis] > c) || (p[axis] > c && q[axis] < c)) {
      const double t = (c - p[axis]) / (q[axis] - p[axis]);
      double x[3];
      for (int k = 0; k < 3; k++) x[k] = p[k] + t * (q[k] - p[k]);
      x[axis] = c;
      if (L.n < 16) { for (int k = 0; k < 3; k++) L.v[L.n][k] = x[k]; L.n++; }
      if (R.n < 16) { for (int k = 0; k < 3; k++) R.v[R.n][k] = x[k]; R.n++; }
    }
  }
}
// P clipped to box B (6 cuts); empty polygon if nothing of P lies in B
void clip_to(const Poly& P, const DBox& B, PolyN& out) {
  PolyN a, l, r;
  to_polyn(P, a);
  for (int axis = 0; axis < 3 && a.n; axis++) {
    cut(a, axis, B.lo[axis], l, r);
    a = r;
    if (!a.n) break;
    cut(a, axis, B.hi[axis], l, r);
    a = l;
  }
  out = a;
}

// Output of one subtree build: nodes (a subtree root at `root`), leaf slots.
struct Ctx {
  std::vector<Node2> nodes;
  std::vector<uint32_t> refs;
  uint32_t depth = 0;
  int64_t budget = 0;  // further references spatial splits may still add
};

struct Task {
  uint32_t idx;  // node index in the top context
  uint32_t depth;
  std::vector<Ref> refs;
};

struct Builder {
  const FastTreeOptions& o;
  const std::vector<Poly>& poly;
  double margin = 0.0;
  double root_area = 1.0;
  // top-level pass: subtrees at depth par_depth with at least par_min
  // references become tasks built in parallel
  uint32_t par_depth = 0;
  size_t par_min = ~(size_t)0;
  std::vector<Task>* tasks = nullptr;

  Builder(const FastTreeOptions& opt, const std::vector<Poly>& p) : o(opt), poly(p) {}

  // Best object split (centroid bins) over the three axes: cost, axis, bin
  // boundary (left = bins 0..pos), the children's boxes, centroid bounds.
  bool object_split(const std::vector<Ref>& refs, double& cost, int& axis, int& pos, DBox& lb, DBox& rb,
                    DBox& cb) const {
    const int B = o.bins;
    cb = DBox();
    for (const Ref& r : refs) {
      double c[3];
      for (int k = 0; k < 3; k++) c[k] = 0.5 * (r.b.lo[k] + r.b.hi[k]);
      cb.grow(c);
    }
    bool found = false;
    std::vector<Bin> bins(B);
    std::vector<DBox> lbx(B), rbx(B);
    std::vector<uint32_t> lc(B), rc(B);
    for (int a = 0; a < 3; a++) {
      const double ext = cb.hi[a] - cb.lo[a];
      if (!(ext > 0.0)) continue;
      bins.assign(B, Bin());
      const double sc = B / ext;
      for (const Ref& r : refs) {
        const double c = 0.5 * (r.b.lo[a] + r.b.hi[a]);
        int k = (int)((c - cb.lo[a]) * sc);
        k = std::min(std::max(k, 0), B - 1);
        bins[k].b.grow(r.b);
        bins[k].n++;
      }
      DBox acc;
      uint32_t cnt = 0;
      for (int k = 0; k < B; k++) {
        acc.grow(bins[k].b);
        cnt += bins[k].n;
        lbx[k] = acc;
        lc[k] = cnt;
      }
      acc = DBox();
      cnt = 0;
      for (int k = B - 1; k >= 0; k--) {
        acc.grow(bins[k].b);
        cnt += bins[k].n;
        rbx[k] = acc;
        rc[k] = cnt;
      }
      for (int k = 0; k + 1 < B; k++) {
        if (lc[k] == 0 || rc[k + 1] == 0) continue;
        const double c = lbx[k].area() * lc[k] + rbx[k + 1].area() * rc[k + 1];
        if (!found || c < cost) {
          found = true;
          cost = c;
          axis = a;
          pos = k;
          lb = lbx[k];
          rb = rbx[k + 1];
        }
      }
    }
    return found;
  }

  // Best spatial split: bins over the node box; a reference spanning several
  // bins is its hit region clipped to its box, cut at each bin plane.
  bool spatial_split(const std::vector<Ref>& refs, const DBox& nb, double& cost, int& axis, double& plane,
                     uint32_t& nl, uint32_t& nr) const {
    const int B = o.sp_bins;
    bool found = false;
    std::vector<Bin> bins(B);
    std::vector<DBox> lbx(B);
    std::vector<uint32_t> lc(B);
    for (int a = 0; a < 3; a++) {
      const double lo = nb.lo[a], ext = nb.hi[a] - nb.lo[a];
      if (!(ext > 0.0)) continue;
      bins.assign(B, Bin());
      const double sc = B / ext;
      auto bin_of = [&](double x) { return std::min(std::max((int)((x - lo) * sc), 0), B - 1); };
      auto edge = [&](int k) { return k >= B ? nb.hi[a] : lo + ext * k / B; };
      for (const Ref& r : refs) {
        const int b0 = bin_of(r.b.lo[a]), b1 = bin_of(r.b.hi[a]);
        bins[b0].enter++;
        bins[b1].exit++;
        if (b0 == b1) {
          bins[b0].b.grow(r.b);
          continue;
        }
        PolyN q, l, rr;
        clip_to(poly[r.prim], r.b, q);
        for (int k = b0; k < b1 && q.n; k++) {
          cut(q, a, edge(k + 1), l, rr);
          if (l.n) {
            DBox bx;
            box_of(l, bx);
            bins[k].b.grow(meet(bx, r.b));
          }
          q = rr;
        }
        if (q.n) {
          DBox bx;
          box_of(q, bx);
          bins[b1].b.grow(meet(bx, r.b));
        }
      }
      DBox acc;
      uint32_t cnt = 0;
      for (int k = 0; k < B; k++) {
        acc.grow(bins[k].b);
        cnt += bins[k].enter;
        lbx[k] = acc;
        lc[k] = cnt;
      }
      acc = DBox();
      cnt = 0;
      for (int k = B - 1; k >= 1; k--) {
        acc.grow(bins[k].b);
        cnt += bins[k].exit;
        const uint32_t ln = lc[k - 1];
        if (ln == 0 || cnt == 0) continue;
        const double c = lbx[k - 1].area() * ln + acc.area() * cnt;
        if (!found || c < cost) {
          found = true;
          cost = c;
          axis = a;
          plane = edge(k);
          nl = ln;
          nr = cnt;
        }
      }
    }
    return found;
  }

  // Writes node `idx` of `C` (children allocated as an adjacent pair before
  // the recursion, as bvh.rs:225-231 does). Internal boxes are filled by
  // fix_boxes() once every subtree exists.
  void build(Ctx& C, uint32_t idx, std::vector<Ref>& refs, uint32_t depth) {
    if (tasks && depth == par_depth && refs.size() >= par_min) {
      tasks->push_back(Task{idx, depth, std::move(refs)});
      return;
    }
    DBox nb;
    for (const Ref& r : refs) nb.grow(r.b);
    const size_t n = refs.size();
    const double area = nb.area();
    double obj_cost = 0.0, sp_cost = 0.0;
    int obj_axis = 0, obj_pos = 0, sp_axis = 0;
    double sp_plane = 0.0;
    uint32_t sp_nl = 0, sp_nr = 0;
    DBox olb, orb, cb;
    bool obj = false, sp = false;
    if (n > 1 && depth < 120) {
      obj = object_split(refs, obj_cost, obj_axis, obj_pos, olb, orb, cb);
      const DBox ov = meet(olb, orb);
      const bool try_sp = o.spatial && C.budget > 0 && (!obj || ov.area() > o.alpha * root_area);
      if (try_sp) sp = spatial_split(refs, nb, sp_cost, sp_axis, sp_plane, sp_nl, sp_nr);
      if (sp && (sp_nl >= n && sp_nr >= n)) sp = false;  // no progress
    }
    const double leaf_cost = o.c_isect * (double)n * area;
    bool use_sp = sp && (!obj || sp_cost < obj_cost);
    const double best = o.c_trav * area + o.c_isect * (use_sp ? sp_cost : obj_cost);
    const bool split = (obj || sp) && (n > (size_t)o.max_leaf || best < leaf_cost);
    if (!split) {
      make_leaf(C, idx, refs, depth);
      return;
    }
    std::vector<Ref> L, R;
    L.reserve(n);
    R.reserve(n);
    if (use_sp) {
      const int a = sp_axis;
      for (const Ref& r : refs) {
        if (r.b.hi[a] <= sp_plane) {
          L.push_back(r);
        } else if (r.b.lo[a] >= sp_plane) {
          R.push_back(r);
        } else {
          PolyN q, l, rr;
          clip_to(poly[r.prim], r.b, q);
          cut(q, a, sp_plane, l, rr);
          DBox bx;
          if (l.n) {
            box_of(l, bx);
            bx = meet(bx, r.b);
            bx.hi[a] = std::min(bx.hi[a], sp_plane);
            if (!bx.empty()) L.push_back(Ref{r.prim, bx});
          }
          if (rr.n) {
            box_of(rr, bx);
            bx = meet(bx, r.b);
            bx.lo[a] = std::max(bx.lo[a], sp_plane);
            if (!bx.empty()) R.push_back(Ref{r.prim, bx});
          }
        }
      }
      if (L.empty() || R.empty() || (L.size() >= n && R.size() >= n)) {
        L.clear();
        R.clear();
        use_sp = false;
        if (!obj) {
          make_leaf(C, idx, refs, depth);
          return;
        }
      }
    }
    if (use_sp) C.budget -= (int64_t)(L.size() + R.size()) - (int64_t)n;
    if (!use_sp) {
      const int a = obj_axis;
      const double lo = cb.lo[a], sc = o.bins / (cb.hi[a] - cb.lo[a]);
      for (const Ref& r : refs) {
        const double c = 0.5 * (r.b.lo[a] + r.b.hi[a]);
        const int k = std::min(std::max((int)((c - lo) * sc), 0), o.bins - 1);
        (k <= obj_pos ? L : R).push_back(r);
      }
    }
    std::vector<Ref>().swap(refs);
    const uint32_t left = (uint32_t)C.nodes.size();
    C.nodes.push_back(Node2{});
    C.nodes.push_back(Node2{});
    C.nodes[idx].left_first = left;
    C.nodes[idx].count = 0;
    build(C, left, L, depth + 1);
    std::vector<Ref>().swap(L);
    build(C, left + 1, R, depth + 1);
  }

  void make_leaf(Ctx& C, uint32_t idx, const std::vector<Ref>& refs, uint32_t depth) const {
    Node2 nd;
    for (int k = 0; k < 3; k++) {
      nd.bmin[k] = std::numeric_limits<float>::infinity();
      nd.bmax[k] = -std::numeric_limits<float>::infinity();
    }
    for (const Ref& r : refs) {
      for (int k = 0; k < 3; k++) {
        nd.bmin[k] = std::min(nd.bmin[k], down(r.b.lo[k] - margin));
        nd.bmax[k] = std::max(nd.bmax[k], up(r.b.hi[k] + margin));
      }
    }
    nd.left_first = (uint32_t)C.refs.size();
    nd.count = (uint32_t)refs.size();
    for (const Ref& r : refs) C.refs.push_back(r.prim);
    C.nodes[idx] = nd;
    C.depth = std::max(C.depth, depth);
  }
};

// Internal boxes as the union of the children's (children always follow
// their parent in the array, so a reverse sweep sees them first).
void fix_boxes(std::vector<Node2>& nodes) {
  for (size_t k = nodes.size(); k-- > 0;) {
    Node2& n = nodes[k];
    if (k == 1 || n.count != 0) continue;
    const Node2& a = nodes[n.left_first];
    const Node2& b = nodes[n.left_first + 1];
    for (int i = 0; i < 3; i++) {
      n.bmin[i] = std::min(a.bmin[i], b.bmin[i]);
      n.bmax[i] = std::max(a.bmax[i], b.bmax[i]);
    }
  }
}

}  // namespace

bool build_fast_tree(const HostScene& sc, const FastTreeOptions& opt, FastTree& ft, std::string& err) {
  const auto t0 = std::chrono::steady_clock::now();
  ft = FastTree();
  if (!sc.use_bvh || !sc.tri_only || sc.shapes.size() <= sc.num_inf || sc.nodes.empty()) {
    err = "fast tree: triangle scenes with a BVH only";
    return false;
  }
  if (opt.bins < 2 || opt.max_leaf < 1) {
    err = "fast tree: bad options";
    return false;
  }
  const size_t nf = sc.shapes.size() - sc.num_inf;
  std::vector<Poly> poly(nf);
  std::vector<Ref> refs;
  refs.reserve(nf);
  double R = 1.0;
  for (size_t i = 0; i < nf; i++) {
    const int st = offset_triangle(sc.shapes[sc.num_inf + i], poly[i]);
    if (st == 2) {
      err = "fast tree: a triangle without a bounded hit region";
      return false;
    }
    if (st == 1) continue;  // never hit: left out of the tree
    Ref r;
    r.prim = (uint32_t)i;
    for (int k = 0; k < 3; k++) r.b.grow(poly[i].v[k]);
    for (int k = 0; k < 3; k++) R = std::max(R, std::max(std::fabs(r.b.lo[k]), std::fabs(r.b.hi[k])));
    refs.push_back(r);
  }
  // Margin and origin bound: every rounding error between the
  // exact line point o + t·d and what the f32 slab and triangle tests see is
  // a few units in the last place of max|o_i| + max|p_i| <= omax + R, times
  // small constants; margin = R / 2^13 is over 100 times that with omax = 8R.
  ft.margin = (float)std::ldexp(R, -opt.margin_log2);
  ft.omax = (float)(opt.omax_mult * R);
  // reference leaf of every finite shape (bvh.rs leaves hold contiguous ranges)
  ft.ref_leaf.assign(nf, 0u);
  for (size_t k = 0; k < sc.nodes.size(); k++) {
    const Node2& n = sc.nodes[k];
    if (k == 1 || n.count == 0) continue;
    for (uint32_t i = n.left_first; i < n.left_first + n.count && i < nf; i++) ft.ref_leaf[i] = (uint32_t)k;
  }
  Builder b(opt, poly);
  b.margin = ft.margin;
  {
    DBox all;
    for (const Ref& r : refs) all.grow(r.b);
    b.root_area = std::max(all.area(), 1e-30);
  }
  if (refs.empty()) {
    err = "fast tree: no triangle can be hit";
    ft = FastTree();
    return false;
  }
  // top levels serially; subtrees of >= 4096 references at depth 5 as
  // parallel tasks (each its own node and slot arrays, spliced in after)
  Ctx top;
  top.nodes.resize(2);  // root 0, node 1 unused (bvh.rs:108-109)
  top.budget = (int64_t)(opt.dup_budget * (double)refs.size());
  std::vector<Task> tasks;
  b.tasks = &tasks;
  b.par_depth = 6;
  b.par_min = std::max<size_t>(256, refs.size() / 512);
  b.build(top, 0, refs, 0);
  b.tasks = nullptr;
  if (getenv("WPT_FT_DEBUG"))
    fprintf(stderr, "fast tree: serial top %.0f ms, %zu tasks\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), tasks.size());
  std::vector<Ctx> sub(tasks.size());
  {
    // the budget left after the top levels, shared by the tasks in proportion
    // to their references (deterministic: the same tree for any thread count)
    size_t tot = 0;
    for (const Task& t : tasks) tot += t.refs.size();
    for (size_t t = 0; t < tasks.size(); t++)
      sub[t].budget = tot ? (int64_t)((double)std::max<int64_t>(top.budget, 0) * tasks[t].refs.size() / tot) : 0;
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t t; (t = next.fetch_add(1)) < tasks.size();) {
        sub[t].nodes.resize(1);
        b.build(sub[t], 0, tasks[t].refs, tasks[t].depth);
      }
    };
    const unsigned nt = std::max(1u, std::min<unsigned>(16, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned i = 1; i < nt && i < tasks.size(); i++) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
  }
  ft.nodes = std::move(top.nodes);
  ft.refs = std::move(top.refs);
  ft.depth = top.depth;
  for (size_t t = 0; t < tasks.size(); t++) {
    const Ctx& c = sub[t];
    const uint32_t nbase = (uint32_t)ft.nodes.size() - 1;  // local node k >= 1 -> nbase + k
    const uint32_t rbase = (uint32_t)ft.refs.size();
    for (size_t k = 0; k < c.nodes.size(); k++) {
      Node2 n = c.nodes[k];
      if (n.count) n.left_first += rbase;
      else n.left_first += nbase;
      if (k == 0) ft.nodes[tasks[t].idx] = n;
      else ft.nodes.push_back(n);
    }
    ft.refs.insert(ft.refs.end(), c.refs.begin(), c.refs.end());
    ft.depth = std::max(ft.depth, c.depth);
  }
  fix_boxes(ft.nodes);
  // SAH of the result, per unit root area (expansions c_trav, tests c_isect)
  {
    auto area = [](const Node2& n) {
      const double x = (double)n.bmax[0] - n.bmin[0], y = (double)n.bmax[1] - n.bmin[1],
                   z = (double)n.bmax[2] - n.bmin[2];
      return 2.0 * (x * y + x * z + y * z);
    };
    const double ra = area(ft.nodes[0]);
    double s = 0.0;
    for (size_t k = 0; k < ft.nodes.size(); k++) {
      if (k == 1) continue;
      const Node2& n = ft.nodes[k];
      s += (n.count == 0 ? opt.c_trav : opt.c_isect * n.count) * area(n) / ra;
    }
    ft.sah = s;
  }
  ft.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return true;
}

}  // namespace wpt
