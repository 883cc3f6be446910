// wpt_fasttree.h — the traversal tree of the fast path.
//
// The reference's BVH2 (bvh.rs:103-437: 16 bins on the longest axis, greedy
// two-pointer sweep) decides the closest hit's tie order, so the exact stack
// machine must walk it. The fast path walks a better tree instead — binned SAH
// over all three axes plus SBVH spatial splits (a triangle may sit in several
// leaves) — nearest first with inclusive culling, and hands a ray to the exact
// machine only when the reference's order could matter (a tie at the winning
// t, or the winner's REFERENCE leaf box entered after t_win).
//
// What makes that sound is that the fast tree's boxes are conservative: a
// leaf box holds every point at which Triangle::trace_simple (triangle.rs:
// 159-191, with its 0.1·EPSILON edge slack) can report a hit, with a margin
// that covers the f32 rounding of the hit point and of the slab test. Then a
// leaf holding a triangle hit at t is entered whenever the closest hit so far
// is >= t, so the fast traversal returns the minimum t over ALL triangles (and
// sees every shape tied at it). Box per triangle: the triangle with each edge
// pushed out by EPSILON_slack / |edge| (the region the three edge tests
// accept, solved in f64), clipped to its spatial-split cell, then grown by
// `margin` and rounded outward to f32.
//
// The guarantee needs |ray origin| <= omax (max-norm): the rounding of the hit
// point grows with |o| + |hit point|. Rays starting farther out are traced by
// the exact machine directly.
#pragma once
#include <string>
#include <vector>

#include "wpt_scene.h"

namespace wpt {

struct FastTreeOptions {
  int bins = 32;           // SAH bins per axis (object splits)
  int sp_bins = 16;        // ... and for spatial splits
  int max_leaf = 1;        // larger nodes are always split when a split exists (1: one triangle per leaf,
  float c_trav = 0.0f;     // SAH cost of a node-pair expansion ...   with c_trav 0 the fastest measured)
  float c_isect = 1.0f;    // ... and of one triangle test
  bool spatial = true;     // SBVH spatial splits
  float alpha = 1e-5f;     // try spatial splits when the best object split's child overlap / root area exceeds this
  float dup_budget = 0.3f;  // spatial splits stop once they added this many references per triangle
  int margin_log2 = 13;    // leaf boxes grow by R / 2^margin_log2 (R: max |coordinate| of the hit regions)
  float omax_mult = 8.0f;  // rays with max|o_i| <= omax_mult * R take the fast path
};

struct FastTree {
  std::vector<Node2> nodes;      // BVH2 layout of HostScene::nodes: root 0, node 1 unused, pairs adjacent
  std::vector<uint32_t> refs;    // leaf slots: finite shape index (shape index - num_inf), duplicates allowed
  std::vector<uint32_t> ref_leaf;  // per finite shape: its leaf in the reference BVH2 (HostScene::nodes index)
  uint32_t depth = 0;
  float margin = 0.0f;           // growth of every leaf box (scene units)
  float omax = 0.0f;             // rays with max|o_i| > omax go to the exact machine
  double sah = 0.0;              // SAH cost (per unit root area) of the tree
  double ms = 0.0;               // build time
};

// Builds the fast tree over sc's finite shapes (triangle-only scenes with the
// BVH enabled). False with `err` set when the scene is not eligible (other
// shape kinds, non-finite vertices, a degenerate offset region): the exact
// machine then traces every ray.
bool build_fast_tree(const HostScene& sc, const FastTreeOptions& opt, FastTree& ft, std::string& err);

}  // namespace wpt
