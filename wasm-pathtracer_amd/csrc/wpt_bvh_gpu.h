// wpt_bvh_gpu.h — BVH2 build on the GPU, bit-identical to the host build.
//
// The reference builds its BVH2 top-down and recursively (src/graphics/
// bvh.rs:103-437): per node, 16 bins on the centroid of the parent box's
// longest axis, the greedy two-pointer bin sweep (:328-367), the SAH
// acceptance test (:264-268) and `write_to`, a stable reorder of the node's
// shapes by bin (:462-470). Every step is a function of the node's own shapes
// only, so all nodes of one tree level are built at once:
//   k_minmax  per shape: min / max centroid coordinate of its node (atomics on
//             order-preserving u32 keys; min / max do not depend on order)
//   k_bin     per shape: its bin (the reference's f32 arithmetic), per-(node,
//             bin) box and count (LDS-privatised for blocks inside one node)
//   k_decide  per node: the bin sweep and SAH test; a split appends the two
//             children to the next level
//   sort      stable radix sort of (node offset * 16 + bin, shape) pairs: the
//             split nodes' write_to, every other range unchanged
//   k_reseg   per shape: its node on the next level
// After the last level the node records are copied back and numbered in the
// reference's depth-first allocation order (bvh.rs:225-231) on the host.
// Results: nodes and the shape order bit-identical to the host build (zero
// signs aside: a box bound of ±0 may carry the other sign, which no box test
// can tell apart), checked by tests/test_gpu_bvh_build.py.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "wpt_scene.h"

namespace wpt {

class BvhGpu : public Bvh2Builder {
 public:
  BvhGpu() = default;
  ~BvhGpu() override;
  BvhGpu(const BvhGpu&) = delete;
  BvhGpu& operator=(const BvhGpu&) = delete;
  // box: 6 floats per shape (x_min, y_min, z_min, x_max, y_max, z_max),
  // loc: 3 floats per shape, in rep order. Fills nodes (placeholders at 0 and
  // 1, root at 0), the shapes' BVH order and the depth, as the host Builder.
  bool build(const float* box, const float* loc, size_t n, std::vector<Node2>& nodes, std::vector<uint32_t>& ord,
             uint32_t& depth, double& ms, std::string& err) override;
  double last_ms() const { return last_ms_; }  // device time of the last build (levels + sorts)
  uint32_t last_levels() const { return levels_; }

 private:
  bool reserve(size_t n, std::string& err);
  void release();
  hipStream_t stream_ = nullptr;
  size_t cap_ = 0;
  float* d_box_ = nullptr;
  float* d_loc_ = nullptr;
  uint32_t* d_ord_[2] = {nullptr, nullptr};
  uint32_t* d_key_[2] = {nullptr, nullptr};
  uint32_t* d_seg_ = nullptr;
  uint8_t* d_bin_ = nullptr;
  // per task (at most 2n - 1): range, parent box, result
  uint32_t* d_toff_ = nullptr;
  uint32_t* d_tcnt_ = nullptr;
  uint32_t* d_tchild_ = nullptr;  // first child task (0: leaf)
  uint32_t* d_tdepth_ = nullptr;
  uint32_t* d_tsplit_ = nullptr;  // left count of a split task
  float* d_tpbox_ = nullptr;      // 6 per task: the box subdivide() receives
  float* d_tbox_ = nullptr;       // 6 per task: the node's box
  // per task of the current level
  uint32_t* d_vmm_ = nullptr;     // 2 per task: ordered keys of min / max centroid
  uint32_t* d_bins_ = nullptr;    // 16 x 7 per task: box keys (6) and count
  uint32_t* d_ntask_ = nullptr;   // task counter
  uint32_t* h_ntask_ = nullptr;   // pinned mirror
  void* d_tmp_ = nullptr;
  size_t tmp_bytes_ = 0;
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
  double last_ms_ = 0.0;
  uint32_t levels_ = 0;
};

}  // namespace wpt
