// wpt_photon.cpp — host build of the PNEE octree (see wpt_photon.h).
#include "wpt_photon.h"

namespace wpt {

PhotonTree::PhotonTree(uint32_t num_lights) : num_lights_(num_lights) {
  nodes_.resize(1);
  nodes_[0].bins.assign(num_lights_, 1.0f);  // EmpiricalPDF::new (empirical_pdf.rs:22-28)
}

void PhotonTree::insert(uint32_t light, V3 loc, float intensity) {
  const float b[6] = {-kPhotonTreeSize, -kPhotonTreeSize, -kPhotonTreeSize,
                      kPhotonTreeSize,  kPhotonTreeSize,  kPhotonTreeSize};
  insert_at(0, b, PhotonRec{light, loc, intensity}, 0);
  inserted_++;
}

// Octree::insert (photon_tree.rs:171-206). `depth` only guards the split:
// more than 1024 photons at one point would make the reference recurse
// without end; here such a cell stops splitting below depth 120.
void PhotonTree::insert_at(uint32_t node, const float bounds[6], const PhotonRec& p, int depth) {
  nodes_[node].bins[p.light] += p.intensity;  // EmpiricalPDF::add
  if (nodes_[node].child != 0) {
    float cb[6];
    const uint32_t ci = octant(bounds, p.loc, cb);
    insert_at(nodes_[node].child + ci, cb, p, depth + 1);
    return;
  }
  nodes_[node].values.push_back(p);
  if (nodes_[node].values.size() > kMaxPhotonsInCell && depth < 120) {
    // split: a fresh internal node (bins = 1.0) over 8 empty leaves, then
    // every photon of the cell re-inserted in order
    std::vector<PhotonRec> vals;
    vals.swap(nodes_[node].values);
    const uint32_t first = (uint32_t)nodes_.size();
    nodes_.resize(nodes_.size() + 8);
    for (uint32_t c = 0; c < 8; c++) nodes_[first + c].bins.assign(num_lights_, 1.0f);
    nodes_[node].child = first;
    nodes_[node].bins.assign(num_lights_, 1.0f);
    for (const PhotonRec& v : vals) insert_at(node, bounds, v, depth);
  }
}

// EmpiricalPDF::recheck_cdf (empirical_pdf.rs:79-93), once per node.
void PhotonTree::freeze(std::vector<uint32_t>& child, std::vector<float>& cum) const {
  child.resize(nodes_.size());
  cum.assign(nodes_.size() * num_lights_, 0.0f);
  for (size_t i = 0; i < nodes_.size(); i++) {
    child[i] = nodes_[i].child;
    const std::vector<float>& b = nodes_[i].bins;
    float sum = 0.0f;
    for (float v : b) sum += v;
    float* c = cum.data() + i * num_lights_;
    if (num_lights_ == 0) continue;
    c[0] = 0.0f;
    for (uint32_t k = 1; k < num_lights_; k++) c[k] = c[k - 1] + b[k - 1] / sum;
  }
}

}  // namespace wpt
