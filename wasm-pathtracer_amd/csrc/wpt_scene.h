// wpt_scene.h — host-side scene model of the path-tracing core.
//
// Scenes are assembled exactly like the reference's scene catalogue
// (src/scenes.rs:71-111, mesh transform src/wasm_interface.rs:300-311), the
// BVH2 is built by the reference's binned-SAH algorithm (src/graphics/bvh.rs:
// 103-437) so that node layout, leaf ranges and the shape/light order are
// bit-identical to the reference, and the result is flattened into the
// device layout consumed by the HIP kernels (see DESIGN.md §Data layout).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

#include "wpt_math.h"

namespace wpt {

enum ShapeKind : uint32_t { kTri = 0, kPlane = 1, kSphere = 2, kAARect = 3, kTorus = 4 };

// One reference `Tracable` (src/graphics/ray.rs:91-121) as plain data.
struct Shape {
  uint32_t kind;
  float g[12];        // tri: v0,v1,v2 | plane: loc,normal | sphere: c,r | aarect: xmin,xmax,ymin,ymax,zmin,zmax
                      // | torus: loc, big_r, small_r
  bool emissive;
  float m[3];         // diffuse colour (already Color3-clamped) or emissive intensity
};

// BVHNode (src/graphics/bvh.rs:14-20): 32 bytes, children adjacent.
struct Node2 {
  float bmin[3];
  float bmax[3];      // stored as x_min,y_min,z_min,x_max,y_max,z_max
  uint32_t left_first;
  uint32_t count;
};
static_assert(sizeof(Node2) == 32, "BVHNode is 32 bytes");

// Fast-path BVH4 node (128 B): the BVH2 collapsed two levels at a time, child
// boxes are the BVH2 node boxes (bit-identical), stored SoA for 4-wide slab
// tests. child code: kChildEmpty, internal -> node4 index, leaf ->
// bit31 | count<<24 | first prim (count < 64, first < 2^24) or
// bit31|bit30 | leaf-table index for larger leaves.
struct Node4 {
  float xmin[4], xmax[4], ymin[4], ymax[4], zmin[4], zmax[4];
  uint32_t child[4];
  uint32_t pad[4];
};
static_assert(sizeof(Node4) == 128, "Node4 is 128 bytes");
constexpr uint32_t kChildEmpty = 0xFFFFFFFFu;

struct HostScene {
  std::vector<Shape> shapes;      // reordered as the reference: infinite first, then BVH leaf order
  uint32_t num_inf = 0;
  std::vector<Node2> nodes;       // root at 0, node 1 unused (bvh.rs:108-109)
  std::vector<uint32_t> lights;   // LightEnum::Area(shape index) in shape order (scene.rs:62-66)
  bool use_bvh = true;            // false = Scene::disable_bvh (scene.rs:99-101)
  float background[3] = {0, 0, 0};
  uint32_t depth = 0;             // BVH2 depth (edges root→deepest leaf)
  bool tri_only = true;           // every finite shape is a triangle
  std::vector<Node4> nodes4;      // fast-path BVH4 (root at 0)
  std::vector<uint32_t> leaf_table;  // (first, count) pairs for leaves that do not fit a child code
  uint32_t depth4 = 0;               // BVH4 depth (levels below the root node)
  int want_bvh4 = 1;  // set before building: collapse the BVH4 (the bvh4 traversal reads it): 0 no, 1 yes, 2 unless triangle-only or without a BVH
  bool bvh_on_gpu = false;           // the BVH2 came from a Bvh2Builder (the GPU build)
  double bvh_ms = 0.0;               // BVH2 build time (host wall clock, or the GPU build's device time)
};

// A BVH2 builder that replaces the host one (the GPU build, wpt_bvh_gpu.h)
// for scenes with at least min_shapes finite shapes: the shapes' boxes (6
// floats: x_min, y_min, z_min, x_max, y_max, z_max) and centroids (3 floats)
// in rep order in; nodes (placeholders at 0 and 1), the BVH order of the
// shapes and the depth out, identical to the host build.
struct Bvh2Builder {
  virtual ~Bvh2Builder() = default;
  virtual bool build(const float* box, const float* loc, size_t n, std::vector<Node2>& nodes,
                     std::vector<uint32_t>& ord, uint32_t& depth, double& ms, std::string& err) = 0;
  size_t min_shapes = 0;
};

// Collapse the BVH2 into the fast-path BVH4 (fills nodes4 / leaf_table).
void build_bvh4(HostScene& sc);

// Shape constructors (primitives/*.rs new()).
Shape make_triangle(V3 a, V3 b, V3 c, bool emissive, V3 m);
Shape make_plane(V3 loc, V3 normal, bool emissive, V3 m);
Shape make_sphere(V3 c, float r, bool emissive, V3 m);
Shape make_aarect(float x0, float x1, float y0, float y1, float z0, float z1, bool emissive, V3 m);
Shape make_torus(V3 loc, float big_r, float small_r, bool emissive, V3 m);

// Scene::new (scene.rs:43-69): build the BVH2 over `shapes` with 16 bins
// (reordering them), collect the emissive shapes as area lights.
// With `gpu` set (and enough shapes) the BVH2 comes from it; false if it fails.
bool scene_init(HostScene& sc, std::vector<Shape> shapes, const float bg[3], Bvh2Builder* gpu = nullptr,
                std::string* err = nullptr);

// Scene catalogue. ids: 0 = museum (scenes.rs:15-68), 2 = display_obj over
// mesh slot 1 (scenes.rs:71-111);
// 100 = C1 box, 101 = C2 spheres+planes with the BVH disabled (build-defined
// configs). `mesh` holds mesh slot 1's vertices (may be empty).
// Returns false (and sets err) for ids the core does not implement.
bool build_scene(int scene_id, const std::vector<float>& mesh, HostScene& sc, std::string& err,
                 Bvh2Builder* gpu = nullptr);

}  // namespace wpt
