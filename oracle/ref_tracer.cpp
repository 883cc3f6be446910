// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see ref_core.h header).
// Restates the integrator (src/tracer.rs:156-330), the render target
// (src/render_target.rs:55-77), the scene catalogue (src/scenes.rs:71-111 and
// the mesh transform of src/wasm_interface.rs:300-311) and the build-defined
// config scenes (C1 box, C2 spheres), plus a C API for ctypes.
// ============================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>
#include <limits>

#include "ref_photon.h"
#include "ref_scene.h"

namespace ref {

enum RenderType { NO_NEE = 0, NORMAL_NEE = 1, PNEE = 2 };  // tracer.rs:29-33

struct Camera {  // tracer.rs:16-26
  Vec3 location;
  float rot_x, rot_y;
};

struct PathStats {
  uint64_t rays = 0;         // every trace_g call (primary + extension + shadow)
  uint64_t shadow_rays = 0;
  uint64_t node_visits = 0;  // num_bvh_hits (tracer.rs:40)
};

// tracer.rs:224-330. `max_depth` == 0 is the reference's unbounded loop
// (paths end on miss / emitter / Russian roulette only); a
// positive cap is the build-defined config depth: the path stops after the
// shading (incl. NEE) of its max_depth-th hit.
Vec3 trace_original_color(const Scene& scene, const Ray& original, Rng& rng, RenderType option,
                          bool is_debug_photons, int max_depth, PathStats& st, PhotonTree* photons = nullptr) {
  bool has_nee = option == NORMAL_NEE || option == PNEE;
  Vec3 color = v3(0, 0, 0);
  Vec3 throughput = v3(1, 1, 1);
  Ray ray = original;
  bool has_diffuse_bounced = false;
  for (int depth = 1;; depth++) {
    Hit hit;
    bool ok;
    st.node_visits += scene.trace(ray, &hit, &ok);
    st.rays++;
    if (!ok) {
      color += throughput * to_vec3(scene.background);  // :325-327
      return color;
    }
    Vec3 hit_point = ray_at(ray, hit.distance);
    if (hit.mat.emissive) {  // :245-254
      if (is_debug_photons) {
        if (!has_diffuse_bounced) color += throughput * hit.mat.intensity;
      } else if (!has_nee || !has_diffuse_bounced) {
        color += throughput * hit.mat.intensity;
      }
      return color;
    }
    // :256-263 diffuse bounce (material.rs:97-126)
    Vec3 nrm = hit.normal;
    float r1 = rng.next();
    float r2 = rng.next();
    float ang = (2.0f * PI) * r1;
    float x = ref_cosf(ang) * sqrtf(1.0f - r2);
    float y = sqrtf(r2);
    float z = ref_sinf(ang) * sqrtf(1.0f - r2);
    Vec3 x_normal = orthogonal(nrm);
    Vec3 z_normal = cross(nrm, x_normal);
    Vec3 wi = normalize(x * x_normal + y * nrm + z * z_normal);
    float pdf = dot(wi, nrm) / PI;
    Color3 brdf = hit.mat.color / PI;
    float cos_i = dot(wi, hit.normal);
    throughput = throughput * to_vec3(brdf) * cos_i / pdf;
    ray = make_ray(hit_point + wi * EPSILON, wi);
    has_diffuse_bounced = true;

    if (has_nee && !scene.lights.empty()) {  // :267-313
      size_t num_lights = scene.lights.size();
      size_t light_id;
      float light_chance;
      if (option == PNEE) {  // :270-273
        photons->sample(rng, hit_point, &light_id, &light_chance);
      } else {
        light_id = rng.next_in_range(0, num_lights);
        light_chance = 1.0f / (float)num_lights;
      }
      size_t light_shape_id = scene.lights[light_id];
      const Tracable& light_shape = *scene.shapes[light_shape_id];
      PickResult pk = light_shape.pick_random(rng);
      Vec3 to_light = pk.point - hit_point;
      float d2 = len_sq(to_light);
      to_light = to_light / sqrtf(d2);
      float cos_i2 = dot(to_light, hit.normal);
      float cos_o = dot(-to_light, pk.normal);
      if (cos_i2 > 0.0f && cos_o > 0.0f) {
        if (is_debug_photons) {
          color += throughput * pk.intensity;
        } else {
          bool occluded;
          st.node_visits += scene.shadow_ray(hit_point, pk.point, (long)light_shape_id, &occluded);
          st.rays++;
          st.shadow_rays++;
          if (!occluded) {
            float solid_angle = (light_shape.surface_area() * cos_o) / d2;
            color += throughput * pk.intensity * solid_angle * cos_i2 * (1.0f / light_chance);
          }
        }
      }
    }
    if (max_depth > 0 && depth >= max_depth) return color;
    // :318-324 Russian roulette
    float keep = fmaxf(fminf(fmaxf(fmaxf(throughput.x, throughput.y), throughput.z), 0.9f), 0.1f);
    if (rng.next() < keep) {
      throughput = throughput * (1.0f / keep);
    } else {
      return color;
    }
  }
}

// RenderInstance::preprocess_photons (tracer.rs:126-152) until 300000
// photons are stored (tracer.rs:104-123), photon k on the stream
// photon_seed(seed, k) (build-defined). Photons are traced in parallel
// chunks and inserted in photon order. Stops after 64 x 300000 shots.
void shoot_photons(const Scene& scene, uint32_t seed, int threads, PhotonTree& tree) {
  const size_t needed = 300000;
  const uint64_t max_shots = 64ull * needed;
  if (scene.lights.empty()) return;
  struct Rec { bool ok; size_t light; Vec3 loc; float val; };
  const size_t chunk = 1 << 16;
  std::vector<Rec> recs(chunk);
  uint64_t k0 = 0;
  if (threads < 1) threads = 1;
  while (tree.num_photons < needed && k0 < max_shots) {
    std::atomic<size_t> next(0);
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < chunk;) {
        Rng rng;
        rng.state = photon_seed(seed, (uint32_t)(k0 + i));
        Rec r{false, 0, v3(0, 0, 0), 0.0f};
        size_t light_id = rng.next_in_range(0, scene.lights.size());
        const Tracable& ls = *scene.shapes[scene.lights[light_id]];
        PickResult pk = ls.pick_random(rng);
        Vec3 light_normal = rng.next_hemisphere(pk.normal);
        Ray ray = make_ray(pk.point + light_normal * EPSILON, light_normal);
        Hit hit;
        bool ok;
        scene.trace(ray, &hit, &ok);
        if (ok && !hit.mat.emissive) {
          Vec3 I = pk.intensity;
          r = Rec{true, light_id, ray_at(ray, hit.distance) + hit.normal * EPSILON,
                  dot(pk.normal, light_normal) * fmaxf(fmaxf(I.x, I.y), I.z)};
        }
        recs[i] = r;
      }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    size_t used = chunk;
    for (size_t i = 0; i < chunk; i++) {
      if (!recs[i].ok) continue;
      tree.insert(recs[i].light, recs[i].loc, recs[i].val);
      if (tree.num_photons >= needed) { used = i + 1; break; }
    }
    k0 += used;
  }
  tree.shot = k0;
}

// tracer.rs:178-193: camera ray for pixel (x,y) with two jitter draws.
inline Ray camera_ray(const Camera& cam, size_t x, size_t y, float w_inv, float h_inv, float ar, Rng& rng) {
  float fx = (((float)x + rng.next()) * w_inv - 0.5f) * ar;
  float fy = 0.5f - ((float)y + rng.next()) * h_inv;
  Vec3 pixel = v3(fx, fy, 0.8f);
  Vec3 dir = rot_y(rot_x(normalize(pixel), cam.rot_x), cam.rot_y);
  return make_ray(cam.location, dir);
}

// ---------------------------------------------------------------------------
// Scenes
// ---------------------------------------------------------------------------
// wasm_interface.rs:300-311: mesh triangles scaled by 0.5, translated +z 5,
// diffuse (1, 0.4, 0.4).
std::vector<ShapeP> mesh_triangles(const float* v, size_t num_vertices) {
  std::vector<ShapeP> ts;
  Material mat = diffuse(color3(1.0f, 0.4f, 0.4f));
  size_t nt = num_vertices / 3;
  for (size_t i = 0; i < nt; i++) {
    const float* a = v + 9 * i;
    Vec3 p0 = v3(a[0], a[1], a[2]) * 0.5f, p1 = v3(a[3], a[4], a[5]) * 0.5f, p2 = v3(a[6], a[7], a[8]) * 0.5f;
    Vec3 tr = v3(0.0f, 0.0f, 5.0f);
    ts.push_back(std::make_shared<Triangle>(p0 + tr, p1 + tr, p2 + tr, mat));
  }
  return ts;
}

// scenes.rs:99-108 light quad (intensity 16) at y = 7
void push_bunny_light(std::vector<ShapeP>& s) {
  Vec3 lc1 = v3(-1.0f, 7.0f, 0.0f), lc2 = v3(1.0f, 7.0f, 0.0f), lc3 = v3(1.0f, 7.0f, 2.0f), lc4 = v3(-1.0f, 7.0f, 2.0f);
  s.push_back(std::make_shared<Triangle>(lc3, lc2, lc1, emissive(v3(16.0f, 16.0f, 16.0f))));
  s.push_back(std::make_shared<Triangle>(lc4, lc3, lc1, emissive(v3(16.0f, 16.0f, 16.0f))));
}

// scene ids: 2 = display_obj(bunny slot) (scenes.rs:71-111); 100 = C1 box;
// 101 = C2 spheres+planes (BVH disabled). Returns false for unsupported ids.
bool build_scene(int scene_id, const float* mesh, size_t nverts, Scene& sc) {
  std::vector<ShapeP> s;
  if (scene_id == 2) {
    s.push_back(std::make_shared<Plane>(v3(0.0f, -1.0f, 0.0f), v3(0.0f, 1.0f, 0.0f), diffuse(color3(1.0f, 1.0f, 1.0f))));
    s.push_back(std::make_shared<Plane>(v3(0.0f, 0.0f, 13.0f), v3(0.0f, 0.0f, -1.0f), diffuse(color3(0.8f, 1.0f, 0.8f))));
    if (mesh && nverts >= 3) {
      std::vector<ShapeP> ts = mesh_triangles(mesh, nverts);
      s.insert(s.end(), ts.begin(), ts.end());
    }
    push_bunny_light(s);
    sc.init(color3(0, 0, 0), s);
    return true;
  }
  if (scene_id == 100) {  // C1: build-defined box from reference primitives
    Material white = diffuse(color3(0.8f, 0.8f, 0.8f));
    s.push_back(std::make_shared<Plane>(v3(0.0f, -1.0f, 0.0f), v3(0.0f, 1.0f, 0.0f), white));
    s.push_back(std::make_shared<Plane>(v3(0.0f, 3.0f, 0.0f), v3(0.0f, -1.0f, 0.0f), white));
    s.push_back(std::make_shared<Plane>(v3(0.0f, 0.0f, 4.0f), v3(0.0f, 0.0f, -1.0f), white));
    s.push_back(std::make_shared<Plane>(v3(-2.0f, 0.0f, 0.0f), v3(1.0f, 0.0f, 0.0f), diffuse(color3(0.75f, 0.25f, 0.25f))));
    s.push_back(std::make_shared<Plane>(v3(2.0f, 0.0f, 0.0f), v3(-1.0f, 0.0f, 0.0f), diffuse(color3(0.25f, 0.75f, 0.25f))));
    s.push_back(std::make_shared<AARect>(-1.2f, -0.2f, -1.0f, 0.8f, 1.8f, 2.8f, white));
    s.push_back(std::make_shared<AARect>(0.3f, 1.3f, -1.0f, -0.2f, 0.6f, 1.6f, white));
    Vec3 a = v3(-0.5f, 2.99f, 1.5f), b = v3(0.5f, 2.99f, 1.5f), c = v3(0.5f, 2.99f, 2.5f), d = v3(-0.5f, 2.99f, 2.5f);
    s.push_back(std::make_shared<Triangle>(c, b, a, emissive(v3(8.0f, 8.0f, 8.0f))));
    s.push_back(std::make_shared<Triangle>(d, c, a, emissive(v3(8.0f, 8.0f, 8.0f))));
    sc.init(color3(0, 0, 0), s);
    return true;
  }
  if (scene_id == 101) {  // C2: spheres + planes, linear scan (disable_bvh)
    s.push_back(std::make_shared<Plane>(v3(0.0f, -1.0f, 0.0f), v3(0.0f, 1.0f, 0.0f), diffuse(color3(1.0f, 1.0f, 1.0f))));
    s.push_back(std::make_shared<Plane>(v3(0.0f, 0.0f, 13.0f), v3(0.0f, 0.0f, -1.0f), diffuse(color3(0.8f, 1.0f, 0.8f))));
    Rng g;
    g.state = 0xC2C2C2C2u;
    for (int i = 0; i < 16; i++) {
      float x = g.next() * 6.0f - 3.0f;
      float z = g.next() * 5.0f + 4.0f;
      float r = 0.3f + g.next() * 0.7f;
      float cr = 0.3f + 0.7f * g.next(), cg = 0.3f + 0.7f * g.next(), cb = 0.3f + 0.7f * g.next();
      s.push_back(std::make_shared<Sphere>(v3(x, -1.0f + r, z), r, diffuse(color3(cr, cg, cb))));
    }
    push_bunny_light(s);
    sc.init(color3(0, 0, 0), s);
    sc.disable_bvh();
    return true;
  }
  if (scene_id == 0) {  // setup_scene_museum (scenes.rs:15-55)
    Material grey = diffuse(color3(0.7f, 0.7f, 0.7f));
    s.push_back(std::make_shared<Plane>(v3(0.0f, -1.0f, 0.0f), v3(0.0f, 1.0f, 0.0f), grey));
    const float xs[9] = {-16.0f, -12.0f, -8.0f, -4.0f, 0.0f, 4.0f, 8.0f, 12.0f, 16.0f};
    std::vector<Color3> colors = {color3(1.0f, 0.3f, 0.3f), color3(0.0f, 1.0f, 1.0f), color3(0.3f, 0.3f, 1.0f),
                                  color3(1.0f, 0.0f, 0.0f), color3(0.0f, 1.0f, 0.0f), color3(0.0f, 0.0f, 1.0f),
                                  color3(1.0f, 0.0f, 1.0f), color3(1.0f, 1.0f, 0.0f), color3(0.3f, 1.0f, 0.3f)};
    Rng rng;  // Rng::new (0xBABABEBE), two draws
    rng.next();
    rng.next();
    for (float y : {-7.5f, 0.0f, 7.5f}) {
      for (int i = 0; i < 9; i++) {
        s.push_back(std::make_shared<Torus>(v3(xs[i], -0.5f, y), 1.3f, 0.3f, diffuse(color3(1.0f, 1.0f, 1.0f))));
        // museum_lights (scenes.rs:57-68)
        Vec3 col = to_vec3(colors[i]) * 2.5f;
        float x = xs[i];
        for (float zs : {2.8f, -2.8f}) {
          float zi = zs > 0 ? 2.5f : -2.5f;
          Vec3 lc1 = v3(x - 1.0f, 0.0f, y + zs), lc2 = v3(x + 1.0f, 0.0f, y + zs);
          Vec3 lc3 = v3(x + 1.0f, 1.0f, y + zi), lc4 = v3(x - 1.0f, 1.0f, y + zi);
          s.push_back(std::make_shared<Triangle>(lc3, lc2, lc1, emissive(col)));
          s.push_back(std::make_shared<Triangle>(lc4, lc3, lc1, emissive(col)));
        }
      }
      for (size_t i = 0; i < colors.size(); i++) std::swap(colors[i], colors[rng.next_in_range(0, colors.size())]);
    }
    for (float x : {-14.0f, -10.0f, -6.0f, -2.0f, 2.0f, 6.0f, 10.0f, 14.0f})
      s.push_back(std::make_shared<AARect>(x - 0.1f, x + 0.1f, -1.0f, 2.0f, -20.0f, 20.0f, grey));
    s.push_back(std::make_shared<AARect>(-20.0f, 20.0f, -1.0f, 2.0f, 3.75f - 0.1f, 3.75f + 0.1f, grey));
    s.push_back(std::make_shared<AARect>(-20.0f, 20.0f, -1.0f, 2.0f, -3.75f - 0.1f, -3.75f + 0.1f, grey));
    sc.init(color3(0, 0, 0), s);
    return true;
  }
  return false;
}

}  // namespace ref

// ============================================================================
// C API (ctypes). Test infrastructure only.
// ============================================================================
using namespace ref;

struct OracleHandle {
  Scene scene;
  std::unique_ptr<PhotonTree> photons;  // PNEE tree for photon_seed_of
  uint32_t photon_seed_of = 0;
  PhotonTree* photon_tree(uint32_t seed, int threads) {
    if (!photons || photon_seed_of != seed) {
      photons = std::make_unique<PhotonTree>(scene.lights.size());
      shoot_photons(scene, seed, threads, *photons);
      photons->root->freeze();
      photon_seed_of = seed;
    }
    return photons.get();
  }
};

extern "C" {

void* oracle_new(int scene_id, const float* mesh_vertices, size_t num_vertices) {
  OracleHandle* h = new OracleHandle();
  if (!build_scene(scene_id, mesh_vertices, num_vertices, h->scene)) {
    delete h;
    return nullptr;
  }
  return h;
}

void oracle_free(void* p) { delete (OracleHandle*)p; }

size_t oracle_num_shapes(void* p) { return ((OracleHandle*)p)->scene.shapes.size(); }
size_t oracle_num_inf(void* p) { return ((OracleHandle*)p)->scene.num_inf; }
size_t oracle_num_nodes(void* p) { return ((OracleHandle*)p)->scene.bvh.size(); }
size_t oracle_num_lights(void* p) { return ((OracleHandle*)p)->scene.lights.size(); }
int oracle_bvh_kind(void* p) { return (int)((OracleHandle*)p)->scene.kind; }

// Node dump: 8 u32 words per node (6 f32 bounds bits, left_first, count).
void oracle_get_nodes(void* p, uint32_t* out) {
  const auto& bvh = ((OracleHandle*)p)->scene.bvh;
  for (size_t i = 0; i < bvh.size(); i++) {
    memcpy(out + 8 * i, &bvh[i].bounds, 24);
    out[8 * i + 6] = bvh[i].left_first;
    out[8 * i + 7] = bvh[i].count;
  }
}

// BVH4 collapse (bvh4.rs:37-281, F4 leaf fix) of the scene's BVH2. Returns the
// node count; fills (if out) 37 u32 per node: num_children, then per child
// slot {kind (0 empty, 1 node, 2 leaf), node index | first shape, leaf count,
// 6 f32 bounds bits (x_min, y_min, z_min, x_max, y_max, z_max)}.
size_t oracle_bvh4(void* p, uint32_t* out) {
  const auto& bvh = ((OracleHandle*)p)->scene.bvh;
  if (bvh.empty() || ((OracleHandle*)p)->scene.num_inf == ((OracleHandle*)p)->scene.shapes.size()) return 0;
  const BVH4 b4 = collapse_bvh4(bvh);
  if (out) {
    for (size_t i = 0; i < b4.nodes.size(); i++) {
      const BVHNode4& n = b4.nodes[i];
      uint32_t* o = out + 37 * i;
      memset(o, 0, 37 * sizeof(uint32_t));
      o[0] = n.num_children;
      for (uint32_t k = 0; k < n.num_children; k++) {
        uint32_t* e = o + 1 + 9 * k;
        if (n.children[k] >= 0) {
          e[0] = 1;
          e[1] = (uint32_t)n.children[k];
        } else {
          const auto& l = b4.leaves[(size_t)(-n.children[k] - 1)];
          e[0] = 2;
          e[1] = l.first;
          e[2] = l.second;
        }
        memcpy(e + 3, &n.child_bounds[k], 24);
      }
    }
  }
  return b4.nodes.size();
}

// Shape dump: per shape 12 floats of geometry + kind (as float) + emissive flag
// (16 floats per shape: geom[12], kind, emissive, pad, pad).
void oracle_get_shapes(void* p, float* out) {
  const auto& sh = ((OracleHandle*)p)->scene.shapes;
  for (size_t i = 0; i < sh.size(); i++) {
    float* o = out + 16 * i;
    memset(o, 0, 16 * sizeof(float));
    const Tracable* t = sh[i].get();
    if (auto tr = dynamic_cast<const Triangle*>(t)) {
      float g[9] = {tr->v0.x, tr->v0.y, tr->v0.z, tr->v1.x, tr->v1.y, tr->v1.z, tr->v2.x, tr->v2.y, tr->v2.z};
      memcpy(o, g, sizeof g);
    } else if (auto pl = dynamic_cast<const Plane*>(t)) {
      float g[6] = {pl->loc.x, pl->loc.y, pl->loc.z, pl->normal.x, pl->normal.y, pl->normal.z};
      memcpy(o, g, sizeof g);
    } else if (auto sp = dynamic_cast<const Sphere*>(t)) {
      float g[4] = {sp->loc.x, sp->loc.y, sp->loc.z, sp->radius};
      memcpy(o, g, sizeof g);
    } else if (auto to = dynamic_cast<const Torus*>(t)) {
      float g[5] = {to->loc.x, to->loc.y, to->loc.z, to->big_r, to->small_r};
      memcpy(o, g, sizeof g);
    } else if (auto ar = dynamic_cast<const AARect*>(t)) {
      float g[6] = {ar->x_min, ar->x_max, ar->y_min, ar->y_max, ar->z_min, ar->z_max};
      memcpy(o, g, sizeof g);
    }
    o[12] = (float)t->kind();
    o[13] = t->is_emissive() ? 1.0f : 0.0f;
  }
}

int oracle_verify_bvh(void* p) {
  const Scene& s = ((OracleHandle*)p)->scene;
  return verify_bvh(s.shapes, s.num_inf, s.bvh) ? 1 : 0;
}

// Closest-hit dump (scene.rs:162-184): for each ray (origin, dir as 6 floats)
// writes t (or +inf) and shape id (or -1) and node visits.
void oracle_trace_rays(void* p, size_t n, const float* rays, float* t_out, int32_t* id_out, uint32_t* visits) {
  const Scene& s = ((OracleHandle*)p)->scene;
  for (size_t i = 0; i < n; i++) {
    const float* r = rays + 6 * i;
    Ray ray = make_ray(v3(r[0], r[1], r[2]), v3(r[3], r[4], r[5]));
    float t;
    size_t id;
    bool f;
    size_t v = s.trace_g(ray, &t, &id, &f);
    t_out[i] = f ? t : std::numeric_limits<float>::infinity();
    id_out[i] = f ? (int32_t)id : -1;
    if (visits) visits[i] = (uint32_t)v;
  }
}

// Shadow query (scene.rs:104-133): p, q as 6 floats + light shape id.
void oracle_shadow_rays(void* p, size_t n, const float* pq, const int32_t* light, uint8_t* occluded) {
  const Scene& s = ((OracleHandle*)p)->scene;
  for (size_t i = 0; i < n; i++) {
    const float* r = pq + 6 * i;
    bool occ;
    s.shadow_ray(v3(r[0], r[1], r[2]), v3(r[3], r[4], r[5]), (long)light[i], &occ);
    occluded[i] = occ ? 1 : 0;
  }
}

// Per-path-RNG render: for every pixel p of the W×H viewport
// that belongs to this call (x in [x0,x1), y = y0, y0+row_step, .. < y1) and every sample s
// in [s0, s0+spp), traces the path with rng seeded path_seed(seed, p, s) and
// accumulates acc[p] += color in sample order (render_target.rs:55-58).
// Pixels with x < W/2 use left_type, others right_type (wasm_interface.rs:78,
// :90-94). cam = {x,y,z,rot_x,rot_y}. acc is W*H*3 floats (accumulated into),
// stats = {rays, shadow_rays, node_visits}. Runs on `threads` host threads
// (pixel-interleaved rows, independent paths: bitwise identical for any count).
void oracle_render(void* p, uint32_t W, uint32_t H, const float* cam, int left_type, int right_type,
                   int max_depth, uint32_t frame_seed, uint32_t s0, uint32_t spp, uint32_t x0, uint32_t y0,
                   uint32_t x1, uint32_t y1, uint32_t row_step, int threads, float* acc, uint64_t* stats,
                   int light_debug) {
  const Scene& s = ((OracleHandle*)p)->scene;
  Camera c{v3(cam[0], cam[1], cam[2]), cam[3], cam[4]};
  const bool dbg = light_debug != 0;  // is_light_debug -> is_debug_photons (wasm_interface.rs:198-199)
  float fw = (float)W, fh = (float)H;
  float w_inv = 1.0f / fw, h_inv = 1.0f / fh, ar = fw / fh;
  if (threads < 1) threads = 1;
  PhotonTree* photons = (left_type == PNEE || right_type == PNEE) && !s.lights.empty()
                            ? ((OracleHandle*)p)->photon_tree(frame_seed, threads) : nullptr;
  std::vector<PathStats> st(threads);
  if (row_step < 1) row_step = 1;
  std::atomic<uint32_t> next_row(0);
  auto work = [&](int tid) {
    for (;;) {
      uint64_t y64 = (uint64_t)y0 + (uint64_t)next_row.fetch_add(1) * row_step;
      if (y64 >= y1) break;
      uint32_t y = (uint32_t)y64;
      for (uint32_t x = x0; x < x1; x++) {
        uint32_t pix = y * W + x;
        RenderType rt = (RenderType)(x < W / 2 ? left_type : right_type);
        for (uint32_t k = 0; k < spp; k++) {
          Rng rng;
          rng.state = path_seed(frame_seed, pix, s0 + k);
          Ray ray = camera_ray(c, x, y, w_inv, h_inv, ar, rng);
          Vec3 col = trace_original_color(s, ray, rng, rt, dbg, max_depth, st[tid], photons);
          float* a = acc + 3 * (size_t)pix;
          a[0] += col.x;
          a[1] += col.y;
          a[2] += col.z;
        }
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; t++) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  if (stats) {
    stats[0] = stats[1] = stats[2] = 0;
    for (auto& x : st) {
      stats[0] += x.rays;
      stats[1] += x.shadow_rays;
      stats[2] += x.node_visits;
    }
  }
}

// Reference execution model (mode A): ONE sequential xorshift32
// stream (rng.rs:11) shared by pixel selection and paths, RandomSamplingStrategy
// (sampling_strategy.rs:56-59) on each viewport half, `compute(n)` splitting
// n/2 left and the rest right (wasm_interface.rs:374-379). acc (W*H*3) and cnt
// (W*H) are accumulated into; rng_state is in/out.
void oracle_reference_compute(void* p, uint32_t W, uint32_t H, const float* cam, int left_type,
                              int right_type, int max_depth, uint32_t* rng_state, size_t num_samples,
                              float* acc, uint32_t* cnt, uint64_t* stats) {
  const Scene& s = ((OracleHandle*)p)->scene;
  Camera c{v3(cam[0], cam[1], cam[2]), cam[3], cam[4]};
  float fw = (float)W, fh = (float)H;
  float w_inv = 1.0f / fw, h_inv = 1.0f / fh, ar = fw / fh;
  Rng rng;
  rng.state = *rng_state;
  PathStats st;
  size_t left_width = W / 2;
  size_t n_left = num_samples / 2;
  struct Half { size_t x, w, n; int type; } halves[2] = {
      {0, left_width, n_left, left_type}, {left_width, W - left_width, num_samples - n_left, right_type}};
  for (auto& hv : halves) {
    for (size_t i = 0; i < hv.n; i++) {
      size_t px = hv.x + rng.next_in_range(0, hv.w);
      size_t py = rng.next_in_range(0, H);
      Ray ray = camera_ray(c, px, py, w_inv, h_inv, ar, rng);
      Vec3 col = trace_original_color(s, ray, rng, (RenderType)hv.type, false, max_depth, st);
      size_t pix = py * W + px;
      acc[3 * pix] += col.x;
      acc[3 * pix + 1] += col.y;
      acc[3 * pix + 2] += col.z;
      cnt[pix] += 1;
    }
  }
  *rng_state = rng.state;
  if (stats) {
    stats[0] = st.rays;
    stats[1] = st.shadow_rays;
    stats[2] = st.node_visits;
  }
}

// PNEE tree for `seed` (built on first use): pre-order leaf flags and
// cum_bins (num_lights per node); returns the node count, fills counts[2] =
// photons shot, stored. Pass NULL buffers to query the size.
size_t oracle_photon_tree(void* p, uint32_t seed, int threads, uint8_t* leafs, float* cum, uint64_t* counts) {
  PhotonTree* t = ((OracleHandle*)p)->photon_tree(seed, threads);
  std::vector<uint8_t> l;
  std::vector<float> c;
  t->root->dump(l, c);
  if (leafs) memcpy(leafs, l.data(), l.size());
  if (cum) memcpy(cum, c.data(), sizeof(float) * c.size());
  if (counts) { counts[0] = t->shot; counts[1] = t->num_photons; }
  return l.size();
}

// ---------------------------------------------------------------------------
// Adaptive sampling (sampling_strategy.rs:77-230) in the build-defined ROUND
// schedule of the GPU core (wasm-pathtracer_amd/csrc/wpt_adaptive.h), one
// sequence per screen half as the reference's two RenderInstances
// (wasm_interface.rs:90-94): compute(n) advances the left half's sequence by
// n/2 positions, then the right half's by n - n/2 (:374-379). Round 0 of an
// adaptive half = 4 samples per pixel, later rounds ceil(1 + 32 * scaled_mse)
// from the current image; a round of a random half = 1 sample per pixel; a
// round's paths are the half's pixels in raster order, each pixel's samples
// consecutive, sample s of pixel p on stream path_seed(seed, p, s).
// ---------------------------------------------------------------------------
struct AdaptiveSession {
  OracleHandle* h;
  uint32_t W, H;
  Camera cam;
  int type[2], adaptive[2], max_depth;
  uint32_t seed;
  std::vector<float> acc;       // W*H*3 (RenderTarget::acc_buffer)
  std::vector<uint32_t> cnt;    // acc_count
  std::vector<uint8_t> samp;    // SimpleRenderTarget (sampling view)
  struct Rounds {
    std::vector<uint32_t> off, base;   // per pixel: prefix offsets of the round's samples, samples before it
    uint64_t total = 0, pos = 0;
    uint32_t idx = 0;
  } rounds[2];
  PathStats st;

  // render_target.rs:75-79 / 214-216
  Vec3 read_clamped(uint32_t x, uint32_t y) const {
    size_t i = (size_t)W * y + x;
    float n = (float)cnt[i];
    Vec3 v = v3(acc[3 * i] / n, acc[3 * i + 1] / n, acc[3 * i + 2] / n);
    return v3(fminf(fmaxf(v.x, 0.0f), 1.0f), fminf(fmaxf(v.y, 0.0f), 1.0f), fminf(fmaxf(v.z, 0.0f), 1.0f));
  }
  // render_target.rs:131-138
  void read_mul(int x, int y, float mul, float* m, Vec3* res) const {
    if (x < 0 || y < 0 || x >= (int)W || y >= (int)H) { *m = 0.0f; *res = v3(0, 0, 0); return; }
    *m = mul;
    *res = mul * read_clamped((uint32_t)x, (uint32_t)y);
  }
  // render_target.rs:88-128
  Vec3 gauss(int x, int y, int r) const {
    static const float G3[9] = {1, 2, 1, 2, 4, 2, 1, 2, 1};
    static const float G5[25] = {1, 4, 6, 4, 1, 4, 16, 24, 16, 4, 6, 24, 36, 24, 6, 4, 16, 24, 16, 4, 1, 4, 6, 4, 1};
    int d = 2 * r + 1;
    float sum = 0.0f;
    Vec3 a = v3(0, 0, 0);
    for (int vy = 0; vy < d; vy++)
      for (int vx = 0; vx < d; vx++) {
        float m;
        Vec3 res;
        read_mul(x + vx - r, y + vy - r, r == 1 ? G3[vy * 3 + vx] : G5[vy * 5 + vx], &m, &res);
        a += res;
        sum += m;
      }
    return v3(a.x / sum, a.y / sum, a.z / sum);
  }
  static Vec3 mix_color(float v) {  // sampling_strategy.rs:222-230
    if (v < 0.5f) return v3(0, 1, 0) * (1.0f - 2.0f * v) + v3(0, 0, 1) * 2.0f * v;
    return v3(0, 0, 1) * (1.0f - 2.0f * (v - 0.5f)) + v3(1, 0, 0) * 2.0f * (v - 0.5f);
  }
  void plan_round(int hh) {
    size_t np = (size_t)W * H;
    std::vector<uint32_t> c(np, 0);
    uint32_t half = W / 2;
    uint32_t x0 = hh ? half : 0, rw = hh ? W - half : half;
    Rounds& R = rounds[hh];
    if (!adaptive[hh]) {  // RandomSamplingStrategy stand-in: one sample per pixel of the half
      for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = x0; x < x0 + rw; x++) c[(size_t)y * W + x] = 1;
    } else if (R.idx == 0) {  // reset (:198-219): 4 samples per pixel
      for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = x0; x < x0 + rw; x++) c[(size_t)y * W + x] = 4;
    } else {
      // next() (:122-176)
      std::vector<float> mse((size_t)rw * H);
      float mse_sum = 0.0f, mse_min = INFINITY, mse_max = -INFINITY;
      for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < rw; x++) {
          Vec3 v0 = read_clamped(x0 + x, y);
          Vec3 v1 = gauss((int)(x0 + x), (int)y, 1);
          Vec3 v2 = gauss((int)(x0 + x), (int)y, 2);
          float m = fmaxf(len_sq(v0 - v1), len_sq(v0 - v2));
          mse[(size_t)y * rw + x] = m;
          mse_sum += m;
          mse_min = fminf(mse_min, m);
          mse_max = fmaxf(mse_max, m);
        }
      float mse_avg = mse_sum / (float)(rw * H);
      for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < rw; x++) {
          float m = mse[(size_t)y * rw + x];
          float scaled = m < mse_avg ? 0.5f * ((m - mse_min) / (mse_avg - mse_min))
                                     : 0.5f + 0.5f * ((m - mse_avg) / (mse_max - mse_avg));
          scaled = fmaxf(fminf(scaled, 1.0f), 0.0f);
          size_t pix = (size_t)y * W + x0 + x;
          c[pix] = (uint32_t)ceilf(1.0f + scaled * 32.0f);
          Vec3 vis = mse_min == mse_max ? v3(0, 0, 0) : mix_color(scaled);
          samp[4 * pix] = (uint8_t)(fmaxf(fminf(vis.x, 1.0f), 0.0f) * 255.0f);
          samp[4 * pix + 1] = (uint8_t)(fmaxf(fminf(vis.y, 1.0f), 0.0f) * 255.0f);
          samp[4 * pix + 2] = (uint8_t)(fmaxf(fminf(vis.z, 1.0f), 0.0f) * 255.0f);
        }
    }
    R.off.assign(np + 1, 0);
    R.base.assign(np, 0);
    for (size_t p = 0; p < np; p++) {
      R.off[p + 1] = R.off[p] + c[p];
      R.base[p] = cnt[p];
    }
    R.total = R.off[np];
    R.pos = 0;
    R.idx++;
  }
  // n positions of half hh's sequence
  void compute_half(int hh, uint64_t n, int threads, PhotonTree* photons) {
    if ((hh ? W - W / 2 : W / 2) == 0) return;  // an empty half takes no samples
    float fw = (float)W, fh = (float)H;
    float w_inv = 1.0f / fw, h_inv = 1.0f / fh, ar = fw / fh;
    Rounds& R = rounds[hh];
    while (n > 0) {
      if (R.pos == R.total) plan_round(hh);
      uint64_t m = std::min<uint64_t>(n, R.total - R.pos);
      uint64_t k0 = R.pos, k1 = R.pos + m;
      const std::vector<uint32_t>& off = R.off;
      // pixels whose sample ranges intersect [k0, k1)
      size_t p0 = std::upper_bound(off.begin(), off.end(), (uint32_t)k0) - off.begin() - 1;
      std::atomic<size_t> next(p0);
      std::vector<PathStats> sts(threads < 1 ? 1 : threads);
      auto work = [&](int tid) {
        for (size_t p; (p = next.fetch_add(1)) < (size_t)W * H && off[p] < k1;) {
          uint32_t x = (uint32_t)(p % W), y = (uint32_t)(p / W);
          RenderType rt = (RenderType)(x < W / 2 ? type[0] : type[1]);
          uint64_t a = std::max<uint64_t>(off[p], k0), b = std::min<uint64_t>(off[p + 1], k1);
          for (uint64_t k = a; k < b; k++) {
            Rng rng;
            rng.state = path_seed(seed, (uint32_t)p, R.base[p] + (uint32_t)(k - off[p]));
            Ray ray = camera_ray(cam, x, y, w_inv, h_inv, ar, rng);
            Vec3 col = trace_original_color(h->scene, ray, rng, rt, false, max_depth, sts[tid], photons);
            acc[3 * p] += col.x;
            acc[3 * p + 1] += col.y;
            acc[3 * p + 2] += col.z;
            cnt[p] += 1;
          }
        }
      };
      std::vector<std::thread> pool;
      for (int t = 1; t < (int)sts.size(); t++) pool.emplace_back(work, t);
      work(0);
      for (auto& th : pool) th.join();
      for (auto& x : sts) { st.rays += x.rays; st.shadow_rays += x.shadow_rays; st.node_visits += x.node_visits; }
      R.pos += m;
      n -= m;
    }
  }
  void compute(uint64_t n, int threads) {
    PhotonTree* photons = (type[0] == PNEE || type[1] == PNEE) && !h->scene.lights.empty()
                              ? h->photon_tree(seed, threads) : nullptr;
    const uint64_t nl = n / 2;
    compute_half(0, nl, threads, photons);
    compute_half(1, n - nl, threads, photons);
  }
};

void* oracle_adaptive_new(void* p, uint32_t W, uint32_t H, const float* cam, int left_type, int right_type,
                          int left_adaptive, int right_adaptive, int max_depth, uint32_t seed) {
  AdaptiveSession* a = new AdaptiveSession();
  a->h = (OracleHandle*)p;
  a->W = W;
  a->H = H;
  a->cam = Camera{v3(cam[0], cam[1], cam[2]), cam[3], cam[4]};
  a->type[0] = left_type;
  a->type[1] = right_type;
  a->adaptive[0] = left_adaptive;
  a->adaptive[1] = right_adaptive;
  a->max_depth = max_depth;
  a->seed = seed;
  a->acc.assign((size_t)W * H * 3, 0.0f);
  a->cnt.assign((size_t)W * H, 0);
  a->samp.assign((size_t)W * H * 4, 0);
  // the sampling view after update_settings (wasm_interface.rs:185-201):
  // cleared, then the adaptive halves' reset paints them blue (:205-213)
  for (size_t i = 0; i < (size_t)W * H; i++) {
    const int hh = (i % W) < W / 2 ? 0 : 1;
    a->samp[4 * i + 2] = a->adaptive[hh] ? 255 : 0;
    a->samp[4 * i + 3] = 255;
  }
  return a;
}
void oracle_adaptive_compute(void* a, uint64_t n, int threads) { ((AdaptiveSession*)a)->compute(n, threads); }
void oracle_adaptive_read(void* a, float* acc, uint32_t* cnt, uint8_t* samp) {
  AdaptiveSession* s = (AdaptiveSession*)a;
  if (acc) memcpy(acc, s->acc.data(), sizeof(float) * s->acc.size());
  if (cnt) memcpy(cnt, s->cnt.data(), sizeof(uint32_t) * s->cnt.size());
  if (samp) memcpy(samp, s->samp.data(), s->samp.size());
}
void oracle_adaptive_free(void* a) { delete (AdaptiveSession*)a; }

// Torus::trace (torus.rs:56-127) alone, for n rays {ox,oy,oz,dx,dy,dz}: t,
// normal xyz, and flags (bit0 hit, bit1 is_entering) per ray.
void oracle_torus_trace(const float* loc, float big_r, float small_r, const float* rays, size_t n, float* t,
                        float* nrm, uint8_t* flags) {
  const Vec3 c = v3(loc[0], loc[1], loc[2]);
  for (size_t i = 0; i < n; i++) {
    const float* r = rays + 6 * i;
    float tt = 0.0f;
    Vec3 nn = v3(0, 0, 0);
    bool ent = false;
    const bool hit = torus_trace(c, big_r, small_r, v3(r[0], r[1], r[2]), v3(r[3], r[4], r[5]), &tt, &nn, &ent);
    t[i] = hit ? tt : 0.0f;
    nrm[3 * i] = nn.x;
    nrm[3 * i + 1] = nn.y;
    nrm[3 * i + 2] = nn.z;
    flags[i] = (uint8_t)((hit ? 1 : 0) | (ent ? 2 : 0));
  }
}

// Math KAT hooks (golden vectors).
float oracle_sinf(float x) { return ref_sinf(x); }
float oracle_cosf(float x) { return ref_cosf(x); }
void oracle_rng_floats(uint32_t seed, size_t n, float* out) {
  Rng r;
  r.state = seed;
  for (size_t i = 0; i < n; i++) out[i] = r.next();
}
void oracle_rng_u32(uint32_t seed, size_t n, uint32_t* out) {
  Rng r;
  r.state = seed;
  for (size_t i = 0; i < n; i++) out[i] = r.next_u32();
}
uint32_t oracle_path_seed(uint32_t f, uint32_t p, uint32_t s) { return path_seed(f, p, s); }

// Single-shape intersection KATs: kind 0 tri(9), 1 plane(6), 2 sphere(4),
// 3 aarect(6), 4 torus(5); returns 1 and t on hit.
int oracle_shape_trace(int kind, const float* g, const float* ray6, float* t_out, float* n_out) {
  std::shared_ptr<Tracable> sh;
  Material m = diffuse(color3(1, 1, 1));
  if (kind == 0) sh = std::make_shared<Triangle>(v3(g[0], g[1], g[2]), v3(g[3], g[4], g[5]), v3(g[6], g[7], g[8]), m);
  else if (kind == 1) sh = std::make_shared<Plane>(v3(g[0], g[1], g[2]), v3(g[3], g[4], g[5]), m);
  else if (kind == 2) sh = std::make_shared<Sphere>(v3(g[0], g[1], g[2]), g[3], m);
  else if (kind == 4) sh = std::make_shared<Torus>(v3(g[0], g[1], g[2]), g[3], g[4], m);
  else sh = std::make_shared<AARect>(g[0], g[1], g[2], g[3], g[4], g[5], m);
  Ray r = make_ray(v3(ray6[0], ray6[1], ray6[2]), v3(ray6[3], ray6[4], ray6[5]));
  float t;
  if (!sh->trace_simple(r, &t)) return 0;
  Hit h;
  if (sh->trace(r, &h) && n_out) {
    n_out[0] = h.normal.x; n_out[1] = h.normal.y; n_out[2] = h.normal.z;
  }
  *t_out = t;
  return 1;
}

// AABB::hit KAT (aabb.rs:132-164): returns 1 and the distance on hit.
int oracle_aabb_hit(const float* box6, const float* ray6, float* out) {
  AABB b{box6[0], box6[1], box6[2], box6[3], box6[4], box6[5]};
  Ray r = make_ray(v3(ray6[0], ray6[1], ray6[2]), v3(ray6[3], ray6[4], ray6[5]));
  return aabb_hit(b, r, out) ? 1 : 0;
}

}  // extern "C"
