// wpt_photon.h — PNEE light-selection octree (host build, device layout).
//
// Restates src/data/photon_tree.rs and src/math/empirical_pdf.rs: an octree
// over [-1024, 1024]^3 whose every node carries an empirical PDF over the
// lights (bins start at 1.0, photons add their intensity); a leaf splits
// once it holds more than 1024 photons, re-inserting them in order into a
// fresh internal node. Photons are inserted in photon order on the host, so
// every bin sum is accumulated in the reference's order. After the 300k
// photons (tracer.rs:104) the tree is frozen: the CDFs (recheck_cdf,
// empirical_pdf.rs:79-93) are computed once and flattened for the GPU.
#pragma once
#include <stdint.h>

#include <vector>

#include "wpt_math.h"

namespace wpt {

constexpr uint32_t kPhotonsNeeded = 300000;    // tracer.rs:104
constexpr size_t kMaxPhotonsInCell = 1024;     // photon_tree.rs:31
constexpr float kPhotonTreeSize = 1024.0f;     // photon_tree.rs:55

struct PhotonRec {
  uint32_t light;
  V3 loc;
  float intensity;
};

class PhotonTree {
 public:
  explicit PhotonTree(uint32_t num_lights = 0);
  // PhotonTree::insert (photon_tree.rs:60-76); the reference's bounds check
  // can never reject (its && chain), so every photon is inserted.
  void insert(uint32_t light, V3 loc, float intensity);
  // Frozen device layout: child[i] = first of 8 children (0: leaf; the root
  // is never a child), cum[i * num_lights + b] = cum_bins of node i.
  void freeze(std::vector<uint32_t>& child, std::vector<float>& cum) const;
  uint32_t num_lights() const { return num_lights_; }
  size_t num_nodes() const { return nodes_.size(); }
  size_t num_photons() const { return inserted_; }

 private:
  struct Node {
    uint32_t child = 0;              // 0 = leaf
    std::vector<float> bins;         // EmpiricalPDF::bins
    std::vector<PhotonRec> values;   // leaf photons, insertion order
  };
  void insert_at(uint32_t node, const float bounds[6], const PhotonRec& p, int depth);
  uint32_t num_lights_;
  size_t inserted_ = 0;
  std::vector<Node> nodes_;
};

// child() (photon_tree.rs:224-243): octant index and bounds of `v` in `b`
// (x_min,y_min,z_min,x_max,y_max,z_max).
WPT_HD uint32_t octant(const float b[6], V3 v, float out[6]) {
  const float cx = 0.5f * (b[0] + b[3]), cy = 0.5f * (b[1] + b[4]), cz = 0.5f * (b[2] + b[5]);
  const uint32_t i = (v.x < cx ? 0u : 4u) + (v.y < cy ? 0u : 2u) + (v.z < cz ? 0u : 1u);
  out[0] = v.x < cx ? b[0] : cx;
  out[3] = v.x < cx ? cx : b[3];
  out[1] = v.y < cy ? b[1] : cy;
  out[4] = v.y < cy ? cy : b[4];
  out[2] = v.z < cz ? b[2] : cz;
  out[5] = v.z < cz ? cz : b[5];
  return i;
}

}  // namespace wpt
