// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see ref_core.h header).
// Restates src/data/photon_tree.rs (PhotonTree / Octree, child()) and
// src/math/empirical_pdf.rs (EmpiricalPDF with its lazily recomputed CDF),
// structured like the reference: a recursive octree of Node / Leaf cells.
// ============================================================================
#pragma once
#include <memory>
#include <vector>

#include "ref_scene.h"

namespace ref {

// empirical_pdf.rs:10-93
struct EmpiricalPDF {
  std::vector<float> bins, cum_bins;
  bool has_updated_bins = true;
  explicit EmpiricalPDF(size_t n = 0) : bins(n, 1.0f), cum_bins(n, 0.0f) {}
  void add(size_t bin, float v) {  // :37-41
    bins[bin] += v;
    has_updated_bins = true;
  }
  void recheck_cdf() {  // :79-93
    if (!has_updated_bins) return;
    float bin_sum = 0.0f;
    for (float p : bins) bin_sum += p;
    cum_bins[0] = 0.0f;
    for (size_t i = 1; i < bins.size(); i++) cum_bins[i] = cum_bins[i - 1] + bins[i - 1] / bin_sum;
    has_updated_bins = false;
  }
  size_t sample(Rng& rng) {  // :44-62
    recheck_cdf();
    float r = rng.next();
    size_t low = 0, high = bins.size();
    while (low + 1 < high) {
      size_t mid = (low + high) / 2;
      if (cum_bins[mid] <= r) low = mid;
      else high = mid;
    }
    return low;
  }
  float bin_prob(size_t i) {  // :65-75
    recheck_cdf();
    return i + 1 == cum_bins.size() ? 1.0f - cum_bins[i] : cum_bins[i + 1] - cum_bins[i];
  }
};

struct Box6 {
  float x_min, y_min, z_min, x_max, y_max, z_max;
  Vec3 center() const { return v3(0.5f * (x_min + x_max), 0.5f * (y_min + y_max), 0.5f * (z_min + z_max)); }
  float x_size() const { return x_max - x_min; }
  float y_size() const { return y_max - y_min; }
  float z_size() const { return z_max - z_min; }
};

// photon_tree.rs:224-243
inline size_t octree_child(const Box6& b, Vec3 v, Box6* out) {
  Vec3 c = b.center();
  size_t i = (v.x < c.x ? 0 : 4) + (v.y < c.y ? 0 : 2) + (v.z < c.z ? 0 : 1);
  out->x_min = v.x < c.x ? b.x_min : c.x;
  out->x_max = v.x < c.x ? c.x : b.x_max;
  out->y_min = v.y < c.y ? b.y_min : c.y;
  out->y_max = v.y < c.y ? c.y : b.y_max;
  out->z_min = v.z < c.z ? b.z_min : c.z;
  out->z_max = v.z < c.z ? c.z : b.z_max;
  return i;
}

struct PhotonValue {
  size_t light;
  Vec3 loc;
  float intensity;
};

// Octree (photon_tree.rs:36-45, 168-239)
struct Octree {
  bool leaf = true;
  EmpiricalPDF cdf;
  std::vector<std::unique_ptr<Octree>> children;
  std::vector<PhotonValue> values;
  explicit Octree(size_t nl) : cdf(nl) {}

  void insert(size_t nl, Box6 b, size_t light, Vec3 loc, float intensity, int depth = 0) {
    cdf.add(light, intensity);
    if (!leaf) {
      Box6 cb;
      size_t ci = octree_child(b, loc, &cb);
      children[ci]->insert(nl, cb, light, loc, intensity, depth + 1);
      return;
    }
    values.push_back(PhotonValue{light, loc, intensity});
    // > MAX_PHOTONS_IN_CELL (1024): becomes a fresh Node over 8 empty leaves
    // (the depth guard only stops the reference's endless split of > 1024
    // coincident photons)
    if (values.size() > 1024 && depth < 120) {
      std::vector<PhotonValue> vals;
      vals.swap(values);
      leaf = false;
      cdf = EmpiricalPDF(nl);
      for (int i = 0; i < 8; i++) children.push_back(std::make_unique<Octree>(nl));
      for (const PhotonValue& v : vals) insert(nl, b, v.light, v.loc, v.intensity, depth);
    }
  }
  Octree* find_leaf(Box6 b, size_t depth, Vec3 loc, Box6* out_b, size_t* out_depth) {  // :209-220
    if (!leaf) {
      Box6 cb;
      size_t ci = octree_child(b, loc, &cb);
      return children[ci]->find_leaf(cb, depth + 1, loc, out_b, out_depth);
    }
    *out_b = b;
    *out_depth = depth;
    return this;
  }
  EmpiricalPDF& find_node_cdf(Box6 b, size_t depth, Vec3 loc) {  // :225-239
    if (!leaf) {
      if (depth == 0) return cdf;
      Box6 cb;
      size_t ci = octree_child(b, loc, &cb);
      return children[ci]->find_node_cdf(cb, depth - 1, loc);
    }
    return cdf;
  }
  // after the photon phase: compute every CDF once (what the lazy
  // recheck_cdf would do on first use; no bin changes afterwards)
  void freeze() {
    cdf.recheck_cdf();
    for (auto& c : children) c->freeze();
  }
  // pre-order walk (node, then children 0..7): leaf flag + cum_bins
  void dump(std::vector<uint8_t>& leafs, std::vector<float>& cum) const {
    leafs.push_back(leaf ? 1 : 0);
    cum.insert(cum.end(), cdf.cum_bins.begin(), cdf.cum_bins.end());
    for (const auto& c : children) c->dump(leafs, cum);
  }
};

// PhotonTree (photon_tree.rs:18-160)
struct PhotonTree {
  size_t num_lights;
  std::unique_ptr<Octree> root;
  float size = 1024.0f;
  size_t num_photons = 0;
  uint64_t shot = 0;
  explicit PhotonTree(size_t nl) : num_lights(nl), root(std::make_unique<Octree>(nl)) {}
  Box6 bounds() const { return Box6{-size, -size, -size, size, size, size}; }
  void insert(size_t light, Vec3 loc, float intensity) {  // :60-76 (the bounds check never rejects)
    root->insert(num_lights, bounds(), light, loc, intensity);
    num_photons++;
  }
  // :81-160
  void sample(Rng& rng, Vec3 v, size_t* light, float* pdf) {
    if (v.x < -size || v.y < -size || v.z < -size || v.x > size || v.y > size || v.z > size) {
      *light = rng.next_in_range(0, num_lights);
      *pdf = 1.0f / (float)num_lights;
      return;
    }
    Box6 self_bounds = bounds();
    Box6 b;
    size_t depth;
    root->find_leaf(self_bounds, 0, v, &b, &depth);
    float wx, wax, xo, wy, way, yo, wz, waz, zo;
    if (v.x > b.center().x) {
      float lw = (b.x_max - (v.x - b.x_size() * 0.5f)) / b.x_size();
      wx = lw; wax = 1.0f - lw; xo = 1.0f;
    } else {
      float rw = ((v.x + b.x_size() * 0.5f) - b.x_min) / b.x_size();
      wx = rw; wax = 1.0f - rw; xo = -1.0f;
    }
    if (v.y > b.center().y) {
      float lw = (b.y_max - (v.y - b.y_size() * 0.5f)) / b.y_size();
      wy = lw; way = 1.0f - lw; yo = 1.0f;
    } else {
      float rw = ((v.y + b.y_size() * 0.5f) - b.y_min) / b.y_size();
      wy = rw; way = 1.0f - rw; yo = -1.0f;
    }
    if (v.z > b.center().z) {
      float lw = (b.z_max - (v.z - b.z_size() * 0.5f)) / b.z_size();
      wz = lw; waz = 1.0f - lw; zo = 1.0f;
    } else {
      float rw = ((v.z + b.z_size() * 0.5f) - b.z_min) / b.z_size();
      wz = rw; waz = 1.0f - rw; zo = -1.0f;
    }
    bool sx = rng.next() <= wx;
    bool sy = rng.next() <= wy;
    bool sz = rng.next() <= wz;
    Vec3 zero = v3(0.0f, 0.0f, 0.0f);
    Vec3 sampled_v = v + (sx ? zero : xo * v3(b.x_size(), 0.0f, 0.0f)) +
                     (sy ? zero : yo * v3(0.0f, b.y_size(), 0.0f)) + (sz ? zero : zo * v3(0.0f, 0.0f, b.z_size()));
    size_t res = root->find_node_cdf(self_bounds, depth, sampled_v).sample(rng);
    float ajx = b.x_size() * xo, ajy = b.y_size() * yo, ajz = b.z_size() * zo;
    auto prob = [&](Vec3 p) { return root->find_node_cdf(self_bounds, depth, p).bin_prob(res); };
    float p = 0.0f;
    p += prob(v) * wx * wy * wz;
    p += prob(v + v3(ajx, 0.0f, 0.0f)) * wax * wy * wz;
    p += prob(v + v3(0.0f, ajy, 0.0f)) * wx * way * wz;
    p += prob(v + v3(0.0f, 0.0f, ajz)) * wx * wy * waz;
    p += prob(v + v3(ajx, ajy, 0.0f)) * wax * way * wz;
    p += prob(v + v3(0.0f, ajy, ajz)) * wx * way * waz;
    p += prob(v + v3(ajx, 0.0f, ajz)) * wax * wy * waz;
    p += prob(v + v3(ajx, ajy, ajz)) * wax * way * waz;
    *light = res;
    *pdf = p;
  }
};

}  // namespace ref
