// wpt_api.cpp — the C ABI (include/wpt.h), mirroring src/wasm_interface.rs.
//
// The reference keeps one global session (`static mut CONFIG`,
// wasm_interface.rs:62) holding meshes, textures, the render target, the
// scene, the camera and two RenderInstances (left/right viewport halves).
// Here the session holds the same host-side state plus one wpt::Renderer
// that owns the GPU side; every reference `panic!` becomes a WPT_ERR_* code.
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/wpt.h"
#include "wpt_bvh_gpu.h"
#include "wpt_comm.h"
#include "wpt_obj.h"
#include "wpt_partition.h"
#include "wpt_render.h"
#include "wpt_seqsum.h"

using namespace wpt;

namespace {

struct Session {
  std::map<uint32_t, std::vector<float>> preload;   // Mesh::Preload (mesh.rs:8-13)
  std::map<uint32_t, std::vector<float>> meshes;    // Mesh::Triangled, as raw vertex triples
  std::map<uint32_t, std::vector<uint8_t>> textures;
  uint32_t scene_id = 0;
  HostScene scene;
  Renderer renderer;
  uint32_t width = 0, height = 0;
  float cam[5] = {0, 0, 0, 0, 0};
  // the reference's initial settings (wasm_interface.rs:90-94): left half
  // NormalNEE with random sampling, right half PNEE with adaptive sampling
  int left_type = WPT_NORMAL_NEE, right_type = WPT_PNEE, light_debug = 0;
  bool left_adaptive = false, right_adaptive = true;
  int max_depth = 0;
  uint32_t seed = 0xBABABEBEu;
  std::vector<uint8_t> rgba;       // RenderTarget.result (render_target.rs:10)
  std::vector<uint8_t> sampling;   // host copy of the SimpleRenderTarget (sampling visualisation)
  // multi-GPU (wpt_set_comm): the RCCL communicator, the packed partition of
  // this rank and the gathered partitions of all ranks (rank-major)
  Comm* comm = nullptr;
  float4* comm_send = nullptr;
  float4* comm_recv = nullptr;
  uint64_t comm_slot = 0;
  // or a caller's transport (wpt_set_transport) over caller-owned buffers
  wpt_transport_fn xfer = nullptr;
  void* xfer_user = nullptr;
  float4* xfer_send = nullptr;
  float4* xfer_recv = nullptr;
  uint64_t xfer_slot = 0;
  BvhGpu bvh_gpu;  // the GPU BVH2 build (wpt_bvh_gpu.h) for large scenes
  // wpt_probe_read's snapshot between its size query and its fill call
  std::vector<uint32_t> probe_meta;
  std::vector<uint4> probe_rec;
  double probe_tpu = 0.0;
  bool probe_taken = false;
  ~Session() { drop_comm(); }
  void drop_comm() {
    if (comm || xfer) renderer.set_exchange(nullptr, nullptr, nullptr, nullptr, 0);
    xfer = nullptr;
    xfer_user = nullptr;
    xfer_send = xfer_recv = nullptr;
    xfer_slot = 0;
    comm_destroy(comm);
    comm = nullptr;
    if (comm_send) (void)hipFree(comm_send);
    if (comm_recv) (void)hipFree(comm_recv);
    comm_send = comm_recv = nullptr;
    comm_slot = 0;
  }
};

Session* g_session = nullptr;
bool size_comm(Session& s);  // communicator buffers for the current partition (below)
int g_device = 0;
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// The mesh slot a scene displays (scenes.rs:16 MESH_BUNNY_HIGH = 1; the
// reference's notify_mesh_loaded maps scene 1/2/3 to mesh 0/1/2, :317-321).
int mesh_for_scene(uint32_t scene_id) {
  if (scene_id == 1) return 0;
  if (scene_id == 2) return 1;
  if (scene_id == 3) return 2;
  return -1;
}

// Where a scene's BVH2 is built (WPT_OPT_BVH_BUILD): 1 = host, 2 = GPU,
// 0 = the GPU for scenes of at least kGpuBvhShapes finite shapes (the same
// tree either way).
constexpr size_t kGpuBvhShapes = 65536;
int g_bvh_build = 0;
Bvh2Builder* scene_builder(BvhGpu& gpu) {
  if (g_bvh_build == 1) return nullptr;
  gpu.min_shapes = g_bvh_build == 2 ? 0 : kGpuBvhShapes;
  return &gpu;
}
// Options set with no session: the defaults of every later wpt_init.
std::map<int, int64_t> g_default_opts;

int rebuild_scene(Session& s, uint32_t scene_id) {
  std::string err;
  HostScene sc;
  // the BVH4 only feeds the fast-path traversal (WPT_OPT_TRAVERSAL(_SH))
  sc.want_bvh4 = s.renderer.wants_bvh4();
  static const std::vector<float> empty;
  int mid = mesh_for_scene(scene_id);
  const std::vector<float>* mesh = &empty;
  if (mid >= 0) {
    auto it = s.meshes.find((uint32_t)mid);
    if (it != s.meshes.end()) mesh = &it->second;
  }
  if (!build_scene((int)scene_id, *mesh, sc, err, scene_builder(s.bvh_gpu))) {
    if (err.rfind("HIP error", 0) == 0 || err.rfind("GPU BVH", 0) == 0) return fail(WPT_ERR_DEVICE, err);
    return fail(scene_id == 0 ? WPT_ERR_UNSUPPORTED : WPT_ERR_INVALID_SCENE, err);
  }
  if (!s.renderer.upload_scene(sc, err)) return fail(WPT_ERR_DEVICE, err);
  s.scene = std::move(sc);
  s.scene_id = scene_id;
  return WPT_OK;
}

int reset_session(Session& s) {  // wasm_interface.rs:137-150
  std::string err;
  if (!s.renderer.reset(err)) return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

bool valid_type(uint32_t t) { return t <= 2u; }

}  // namespace

extern "C" {

const char* wpt_last_error(void) { return g_err.c_str(); }

int wpt_set_device(int device) {
  if (g_session) return fail(WPT_ERR_ALREADY_INIT, "device must be chosen before init");
  if (device < 0) return fail(WPT_ERR_INVALID_ARG, "bad device");
  g_device = device;
  return WPT_OK;
}

int wpt_init(uint32_t width, uint32_t height, uint32_t scene_id, float cam_x, float cam_y, float cam_z,
             float cam_rot_x, float cam_rot_y) {
  if (g_session) return fail(WPT_ERR_ALREADY_INIT, "Cannot init again");
  if (width == 0 || height == 0) return fail(WPT_ERR_INVALID_ARG, "empty viewport");
  std::unique_ptr<Session> s(new Session());
  std::string err;
  if (!s->renderer.set_device(g_device, err)) return fail(WPT_ERR_DEVICE, err);
  s->width = width;
  s->height = height;
  float cam[5] = {cam_x, cam_y, cam_z, cam_rot_x, cam_rot_y};
  memcpy(s->cam, cam, sizeof cam);
  s->renderer.set_camera(cam);
  s->renderer.set_types(s->left_type, s->right_type, s->light_debug);
  s->renderer.set_adaptive(s->left_adaptive, s->right_adaptive);
  s->renderer.set_options(s->max_depth, s->seed, 0);
  for (const auto& o : g_default_opts)
    if (!s->renderer.set_option(o.first, o.second, err)) return fail(WPT_ERR_INVALID_ARG, err);
  if (!s->renderer.set_viewport(width, height, err)) return fail(WPT_ERR_DEVICE, err);
  int rc = rebuild_scene(*s, scene_id);
  if (rc != WPT_OK) return rc;
  s->rgba.assign((size_t)width * height * 4, 0);
  s->sampling.assign((size_t)width * height * 4, 0);
  // both strategies' constructors paint their halves blue (sampling_strategy.rs:42-51, :205-213)
  if (!s->renderer.fill_sampling_blue(err)) return fail(WPT_ERR_DEVICE, err);
  g_session = s.release();
  return WPT_OK;
}

const uint8_t* wpt_results(uint32_t is_show_sampling) {
  if (!g_session) { fail(WPT_ERR_NOT_INIT, "init not called"); return nullptr; }
  Session& s = *g_session;
  std::string err;
  if (is_show_sampling == 1) {
    if (!s.renderer.sampling_rgba(s.sampling.data(), err)) { fail(WPT_ERR_DEVICE, err); return nullptr; }
    return s.sampling.data();
  }
  if (!s.renderer.results_rgba(s.rgba.data(), err)) { fail(WPT_ERR_DEVICE, err); return nullptr; }
  return s.rgba.data();
}

int wpt_update_scene(uint32_t scene_id) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  int rc = rebuild_scene(*g_session, scene_id);
  if (rc != WPT_OK) return rc;
  return reset_session(*g_session);
}

int wpt_update_settings(uint32_t left_type, uint32_t right_type, uint32_t is_left_adaptive, uint32_t is_right_adaptive,
                        uint32_t is_light_debug) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (!valid_type(left_type) || !valid_type(right_type)) return fail(WPT_ERR_INVALID_ARG, "Invalid RenderType magic number");
  Session& s = *g_session;
  s.left_type = (int)left_type;
  s.right_type = (int)right_type;
  s.light_debug = is_light_debug == 1 ? 1 : 0;
  s.left_adaptive = is_left_adaptive == 1;
  s.right_adaptive = is_right_adaptive == 1;
  s.renderer.set_types(s.left_type, s.right_type, s.light_debug);
  s.renderer.set_adaptive(s.left_adaptive, s.right_adaptive);
  // new strategies, then target and sampling view cleared and the instances
  // reset (wasm_interface.rs:185-201): random halves black, adaptive blue
  return reset_session(s);
}

int wpt_update_viewport(uint32_t width, uint32_t height) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (width == 0 || height == 0) return fail(WPT_ERR_INVALID_ARG, "empty viewport");
  Session& s = *g_session;
  std::string err;
  if (!s.renderer.set_viewport(width, height, err)) return fail(WPT_ERR_DEVICE, err);
  s.width = width;
  s.height = height;
  s.rgba.assign((size_t)width * height * 4, 0);
  s.sampling.assign((size_t)width * height * 4, 0);
  if (s.comm && !size_comm(s)) return fail(WPT_ERR_DEVICE, "hipMalloc failed (communicator buffers)");
  return WPT_OK;  // set_viewport reset the session (wasm_interface.rs:219-232)
}

int wpt_update_camera(float cam_x, float cam_y, float cam_z, float cam_rot_x, float cam_rot_y) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  Session& s = *g_session;
  float cam[5] = {cam_x, cam_y, cam_z, cam_rot_x, cam_rot_y};
  memcpy(s.cam, cam, sizeof cam);
  s.renderer.set_camera(cam);
  return reset_session(s);
}

int wpt_allocate_mesh(uint32_t id, uint32_t num_vertices) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  g_session->preload[id].assign((size_t)num_vertices * 3, 0.0f);
  return WPT_OK;
}

int wpt_parse_obj(const char* text, size_t len, const float* scale, float* out, uint64_t capacity,
                  uint64_t* num_vertices) {
  if (!text && len) return fail(WPT_ERR_INVALID_ARG, "null text");
  std::vector<float> v;
  std::string err;
  if (!parse_obj(text, len, v, err)) return fail(WPT_ERR_INVALID_ARG, err);
  if (scale) scale_vertices(v, scale);
  if (num_vertices) *num_vertices = v.size() / 3;
  if (out) {
    if (capacity < v.size() / 3) return fail(WPT_ERR_INVALID_ARG, "output too small");
    std::memcpy(out, v.data(), v.size() * sizeof(float));
  }
  return WPT_OK;
}

int wpt_load_obj(uint32_t id, const char* text, size_t len, const float* scale, uint64_t* num_vertices) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (!text && len) return fail(WPT_ERR_INVALID_ARG, "null text");
  std::vector<float> v;
  std::string err;
  if (!parse_obj(text, len, v, err)) return fail(WPT_ERR_INVALID_ARG, err);
  if (scale) scale_vertices(v, scale);
  if (num_vertices) *num_vertices = v.size() / 3;
  g_session->preload[id] = std::move(v);  // as allocate_mesh + mesh_vertices
  return WPT_OK;
}

float* wpt_mesh_vertices(uint32_t id) {
  if (!g_session) { fail(WPT_ERR_NOT_INIT, "init not called"); return nullptr; }
  auto it = g_session->preload.find(id);
  if (it == g_session->preload.end()) { fail(WPT_ERR_NO_MESH, "Mesh not allocated"); return nullptr; }
  return it->second.data();
}

int wpt_notify_mesh_loaded(uint32_t id) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  Session& s = *g_session;
  auto it = s.preload.find(id);
  if (it != s.preload.end()) {
    // wasm_interface.rs:300-311: num_triangles = len/3 (vertices), the
    // ×0.5 / +z5 transform is applied when the scene is assembled.
    std::vector<float> v = std::move(it->second);
    v.resize((v.size() / 9) * 9);
    s.meshes[id] = std::move(v);
    s.preload.erase(it);
  }
  if (mesh_for_scene(s.scene_id) == (int)id) {
    int rc = wpt_update_scene(s.scene_id);
    return rc == WPT_OK ? 1 : rc;
  }
  return 0;
}

uint8_t* wpt_allocate_texture(uint32_t id, uint32_t width, uint32_t height) {
  if (!g_session) { fail(WPT_ERR_NOT_INIT, "init not called"); return nullptr; }
  auto& t = g_session->textures[id];
  t.assign((size_t)width * height * 3, 0);
  return t.data();
}

int wpt_notify_texture_loaded(uint32_t) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  return 0;  // textures are never sampled (material.rs:53-60)
}

int wpt_compute(size_t num_samples) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  std::string err;
  if (!g_session->renderer.compute((uint64_t)num_samples, err)) return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

int wpt_set_render_options(int32_t max_depth, uint32_t frame_seed, uint64_t batch_paths) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (max_depth < 0) return fail(WPT_ERR_INVALID_ARG, "max_depth < 0");
  Session& s = *g_session;
  s.max_depth = max_depth;
  s.seed = frame_seed;
  s.renderer.set_options(max_depth, frame_seed, batch_paths);
  return reset_session(s);
}

int wpt_set_partition(uint32_t rank, uint32_t nranks, uint32_t tile) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  std::string err;
  if (!g_session->renderer.set_partition(rank, nranks, tile, err)) return fail(WPT_ERR_INVALID_ARG, err);
  return WPT_OK;
}

int64_t wpt_partition_pixels(uint32_t* out) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  int64_t n = g_session->renderer.part_pixels();
  if (out) {
    const std::vector<uint32_t>& l = g_session->renderer.part_list();
    memcpy(out, l.data(), sizeof(uint32_t) * l.size());
  }
  return n;
}

int64_t wpt_tile_partition(uint32_t width, uint32_t height, uint32_t rank, uint32_t nranks, uint32_t tile,
                           uint32_t* out) {
  if (nranks == 0 || rank >= nranks || tile == 0) return fail(WPT_ERR_INVALID_ARG, "bad partition");
  std::vector<uint32_t> l;
  wpt::tile_partition(width, height, rank, nranks, tile, l);
  if (out) memcpy(out, l.data(), sizeof(uint32_t) * l.size());
  return (int64_t)l.size();
}

int64_t wpt_photon_tree(uint32_t* child, float* cum, uint64_t* shot_stored) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  std::vector<uint32_t> c;
  std::vector<float> f;
  uint64_t shot = 0, stored = 0;
  std::string err;
  if (!g_session->renderer.photon_tree(c, f, shot, stored, err)) return fail(WPT_ERR_DEVICE, err);
  if (child) memcpy(child, c.data(), sizeof(uint32_t) * c.size());
  if (cum) memcpy(cum, f.data(), sizeof(float) * f.size());
  if (shot_stored) { shot_stored[0] = shot; shot_stored[1] = stored; }
  return (int64_t)c.size();
}

int wpt_read_radiance(float* acc3, uint32_t* cnt) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (!acc3) return fail(WPT_ERR_INVALID_ARG, "null buffer");
  std::string err;
  if (!g_session->renderer.read_radiance(acc3, cnt, err)) return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

int wpt_copy_partition(void* device_dst) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  std::string err;
  if (!g_session->renderer.copy_partition((float*)device_dst, err)) return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

int wpt_set_exchange(wpt_exchange_fn fn, void* user, void* local_dev, void* gathered_dev, uint64_t slot) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (fn && (!local_dev || !gathered_dev)) return fail(WPT_ERR_INVALID_ARG, "null exchange buffer");
  if (fn && slot < g_session->renderer.exchange_slot()) return fail(WPT_ERR_INVALID_ARG, "exchange slot too small");
  g_session->renderer.set_exchange(fn, user, local_dev, gathered_dev, slot);
  return WPT_OK;
}

int64_t wpt_exchange_slot(void) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  return (int64_t)g_session->renderer.exchange_slot();
}

// ---- RCCL communicator ------------------------------------------
namespace {
// wpt_set_exchange callback of a communicator session: the library has
// packed this rank's partition into comm_send; all-gather every rank's.
int comm_exchange(void* user) {
  Session& s = *(Session*)user;
  std::string err;
  if (!comm_allgather(s.comm, s.comm_send, s.comm_recv, s.comm_slot, s.renderer.stream(), err)) {
    g_err = err;
    return 1;
  }
  return 0;
}
// The communicator's send / receive buffers sized for this rank's partition
// and the largest one (they grow with the viewport: wpt_update_viewport keeps
// the partition), registered as the adaptive rounds' frame exchange.
bool size_comm(Session& s) {
  uint64_t slot = std::max<uint64_t>(s.renderer.exchange_slot(), s.renderer.part_pixels());
  if (slot == 0) slot = 1;
  if (slot > s.comm_slot) {
    if (s.comm_send) (void)hipFree(s.comm_send);
    if (s.comm_recv) (void)hipFree(s.comm_recv);
    s.comm_send = s.comm_recv = nullptr;
    s.comm_slot = 0;
    if (hipMalloc(&s.comm_send, sizeof(float4) * slot) != hipSuccess ||
        hipMalloc(&s.comm_recv, sizeof(float4) * slot * comm_size(s.comm)) != hipSuccess)
      return false;
    s.comm_slot = slot;
  }
  // adaptive rounds exchange the frame over the communicator
  s.renderer.set_exchange(comm_exchange, &s, s.comm_send, s.comm_recv, s.comm_slot);
  return true;
}
}  // namespace

int wpt_comm_unique_id(void* out) {
  if (!out) return fail(WPT_ERR_INVALID_ARG, "null id buffer");
  std::string err;
  if (!comm_unique_id(out, err)) return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

int wpt_set_comm(uint32_t rank, uint32_t nranks, uint32_t tile, const void* unique_id) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (!unique_id || nranks == 0 || rank >= nranks || tile == 0) return fail(WPT_ERR_INVALID_ARG, "bad communicator");
  Session& s = *g_session;
  s.drop_comm();
  std::string err;
  if (!s.renderer.set_partition(rank, nranks, tile, err)) return fail(WPT_ERR_INVALID_ARG, err);
  if (hipSetDevice(g_device) != hipSuccess) return fail(WPT_ERR_DEVICE, "hipSetDevice failed");
  s.comm = comm_create(rank, nranks, unique_id, err);
  if (!s.comm) return fail(WPT_ERR_DEVICE, err);
  if (!size_comm(s)) {
    s.drop_comm();
    return fail(WPT_ERR_DEVICE, "hipMalloc failed (communicator buffers)");
  }
  return WPT_OK;
}

int wpt_gather_frame(uint32_t root) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  Session& s = *g_session;
  if (s.xfer) {
    // the caller's transport: pack, let it move the rank-major buffers, unpack
    std::string err;
    const Renderer& r = s.renderer;
    if (root >= r.nranks()) return fail(WPT_ERR_INVALID_ARG, "bad root");
    if (s.xfer_slot < r.exchange_slot()) return fail(WPT_ERR_INVALID_ARG, "transport slot smaller than the largest partition");
    if (!s.renderer.copy_partition((float*)s.xfer_send, err)) return fail(WPT_ERR_DEVICE, err);
    if (s.xfer(s.xfer_user, WPT_XFER_GATHER, root) != 0) return fail(WPT_ERR_DEVICE, "transport gather failed");
    if (r.rank() == root && !s.renderer.unpack_ranks(s.xfer_recv, s.xfer_slot, err)) return fail(WPT_ERR_DEVICE, err);
    return WPT_OK;
  }
  if (!s.comm) return fail(WPT_ERR_INVALID_ARG, "no communicator (wpt_set_comm / wpt_set_transport)");
  if (root >= comm_size(s.comm)) return fail(WPT_ERR_INVALID_ARG, "bad root");
  if (!size_comm(s)) return fail(WPT_ERR_DEVICE, "hipMalloc failed (communicator buffers)");
  std::string err;
  if (!s.renderer.copy_partition((float*)s.comm_send, err)) return fail(WPT_ERR_DEVICE, err);
  if (!comm_gather(s.comm, s.comm_send, s.comm_recv, s.comm_slot, root, s.renderer.stream(), err))
    return fail(WPT_ERR_DEVICE, err);
  if (comm_rank(s.comm) == root && !s.renderer.unpack_ranks(s.comm_recv, s.comm_slot, err))
    return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

namespace {
// adaptive rounds' frame exchange through the caller's transport
int xfer_exchange(void* user) {
  Session& s = *(Session*)user;
  return s.xfer(s.xfer_user, WPT_XFER_ALLGATHER, 0);
}
}  // namespace

int wpt_set_transport(wpt_transport_fn fn, void* user, void* send_dev, void* recv_dev, uint64_t slot) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  Session& s = *g_session;
  if (!fn) {
    // unregister the transport only (an RCCL communicator, if any, stays)
    if (s.xfer) {
      s.renderer.set_exchange(nullptr, nullptr, nullptr, nullptr, 0);
      s.xfer = nullptr;
      s.xfer_user = nullptr;
      s.xfer_send = s.xfer_recv = nullptr;
      s.xfer_slot = 0;
    }
    return WPT_OK;
  }
  // validate first: a rejected registration leaves the session as it was
  if (!send_dev || !recv_dev) return fail(WPT_ERR_INVALID_ARG, "null transport buffer");
  if (slot < s.renderer.exchange_slot() || slot < s.renderer.part_pixels())
    return fail(WPT_ERR_INVALID_ARG, "transport slot smaller than the largest partition");
  s.drop_comm();  // a transport replaces the RCCL communicator (include/wpt.h)
  s.xfer = fn;
  s.xfer_user = user;
  s.xfer_send = (float4*)send_dev;
  s.xfer_recv = (float4*)recv_dev;
  s.xfer_slot = slot;
  s.renderer.set_exchange(xfer_exchange, &s, send_dev, recv_dev, slot);
  return WPT_OK;
}

int64_t wpt_gather_plan(uint32_t rank, uint32_t nranks, uint32_t root, uint64_t slot, uint64_t* out) {
  if (nranks == 0 || rank >= nranks || root >= nranks) return fail(WPT_ERR_INVALID_ARG, "bad rank");
  std::vector<XferOp> ops;
  gather_plan(rank, nranks, root, slot, ops);
  if (out)
    for (size_t i = 0; i < ops.size(); i++) {
      out[4 * i] = ops[i].peer;
      out[4 * i + 1] = ops[i].offset;
      out[4 * i + 2] = ops[i].count;
      out[4 * i + 3] = ops[i].recv ? 1u : 0u;
    }
  return (int64_t)ops.size();
}

float wpt_seq_sum(const float* v, uint64_t n) { return wpt::seq_sum_f32(v, (size_t)n); }

float wpt_seq_sum_chunks(const float* v, uint64_t n) {
  std::vector<wpt::ChunkEff> eff(2 * ((size_t)n / wpt::kSumChunk + 1));
  wpt::seq_sum_effects(v, (size_t)n, eff.data());
  return wpt::seq_sum_walk(v, (size_t)n, eff.data());
}

int wpt_seq_sum_device(const float* v, uint64_t n, float* out) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (!out || (n && !v)) return fail(WPT_ERR_INVALID_ARG, "null pointer");
  std::string err;
  if (!g_session->renderer.seq_sum_device(v, n, *out, err)) return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

int wpt_comm_destroy(void) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  g_session->drop_comm();
  return WPT_OK;
}

int wpt_stats(uint64_t* out, size_t n) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  std::string err;
  if (!g_session->renderer.flush_counts(err)) return fail(WPT_ERR_DEVICE, err);
  const Stats& st = g_session->renderer.stats();
  uint64_t v[40] = {st.paths,          st.rays,           st.shadow_rays,    st.node_visits,  st.prim_tests,
                    st.bounces,        st.ext_visits,     st.ext_tests,      st.ext_node_bytes, st.sh_visits,
                    st.sh_tests,       st.sh_node_bytes,  st.fallback_ext,   st.fallback_sh,  st.ext_lane_iters,
                    st.ext_live_iters, st.sh_lane_iters,  st.sh_live_iters,  st.photon_rays,  st.photons,
                    st.sum_chunks,     st.sum_resummed,   st.sum_fetched,    st.stock_consumed, st.fill_paths,
                    st.trace_bytes,    st.finish_paths,   st.finish_max_bounces, st.max_ray_visits,
                    st.ex_body_lanes,  st.ex_bodies,      st.lf_body_lanes,  st.lf_bodies,    st.stock_traced,
                    st.stock_deficit,  st.stock_waits,    st.plan_us,        st.stock_us,
                    st.stock_rays,     st.stock_rays_used};
  for (size_t i = 0; i < n && i < 40; i++) out[i] = v[i];
  return WPT_OK;
}

int wpt_kernel_times(double* out, size_t n) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  const KernelTimes& t = g_session->renderer.times();
  double v[28] = {t.generate, (double)t.n_generate, t.extend, (double)t.n_extend, t.shade, (double)t.n_shade,
                  t.shadow, (double)t.n_shadow, t.accumulate, (double)t.n_accumulate, t.trace, (double)t.n_trace};
  for (int k = 0; k < 6; k++) {
    v[12 + 2 * k] = t.busy[k];
    v[13 + 2 * k] = (double)t.logical[k];
  }
  v[24] = t.retrace;
  v[25] = (double)t.n_retrace;
  v[26] = t.busy[6];
  v[27] = (double)t.logical[6];
  for (size_t i = 0; i < n && i < 28; i++) out[i] = v[i];
  return WPT_OK;
}

int wpt_set_counting(int on) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  g_session->renderer.set_counting(on != 0);
  return WPT_OK;
}

int wpt_scene_build_info(double* out) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (!out) return fail(WPT_ERR_INVALID_ARG, "null argument");
  out[0] = g_session->scene.bvh_ms;
  out[1] = g_session->scene.bvh_on_gpu ? 1.0 : 0.0;
  return WPT_OK;
}

int wpt_set_lanes(int32_t n) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  if (!g_session->renderer.set_lanes(n)) return fail(WPT_ERR_INVALID_ARG, "lanes out of range");
  return WPT_OK;
}

int wpt_set_option(int32_t option, int64_t value) {
  if (option == WPT_OPT_BVH_BUILD) {
    if (value < 0 || value > 2) return fail(WPT_ERR_INVALID_ARG, "option value out of range");
    g_bvh_build = (int)value;  // the next scene build
    return WPT_OK;
  }
  std::string err;
  if (!g_session) {
    if (option == WPT_OPT_DEFAULTS) {  // back to the built-in defaults
      g_default_opts.clear();
      g_bvh_build = 0;
      return WPT_OK;
    }
    // validated against a scratch renderer's ranges, applied at wpt_init
    if (option == WPT_OPT_LANES && (value < 1 || value > kMaxLanes)) return fail(WPT_ERR_INVALID_ARG, "lanes out of range");
    if (option != WPT_OPT_LANES && option != WPT_OPT_GRID_PCT) {
      Renderer probe;
      if (!probe.set_option(option, value, err)) return fail(WPT_ERR_INVALID_ARG, err);
    } else if (option == WPT_OPT_GRID_PCT && (value < 1 || value > 100)) {
      return fail(WPT_ERR_INVALID_ARG, "option value out of range");
    }
    g_default_opts[option] = value;
    return WPT_OK;
  }
  Session& s = *g_session;
  int64_t prev = 0;
  const bool had = s.renderer.get_option(option, prev);
  if (!s.renderer.set_option(option, value, err)) return fail(WPT_ERR_INVALID_ARG, err);
  if (Renderer::scene_option(option)) {
    // the device scene carries the traversal's nodes: re-upload it; if that
    // fails, the option goes back to its previous value
    const int rc = rebuild_scene(s, s.scene_id);
    if (rc != WPT_OK) {
      const std::string keep = g_err;
      std::string e2;
      if (had) (void)s.renderer.set_option(option, prev, e2);
      g_err = keep;
      return rc;
    }
    return reset_session(s);
  }
  if (option == WPT_OPT_PIXEL_TILE && s.renderer.nranks() == 1) {
    // the tile order only shapes a one-rank partition (several ranks keep
    // their tiles: nothing to redo)
    if (!s.renderer.set_partition(s.renderer.rank(), s.renderer.nranks(), s.renderer.tile(), err))
      return fail(WPT_ERR_DEVICE, err);
  }
  return WPT_OK;
}

int64_t wpt_probe_read(uint32_t* meta, uint32_t* rec, uint64_t* rec_entries, double* ticks_per_us) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  Session& s = *g_session;
  std::string err;
  if (!meta || !rec) {
    // the size query takes the snapshot (the session keeps it); the fill
    // call below copies it out (no function-static buffers)
    if (!s.renderer.probe_read(s.probe_meta, s.probe_rec, s.probe_tpu, err)) return fail(WPT_ERR_DEVICE, err);
    s.probe_taken = true;
    if (rec_entries) *rec_entries = s.probe_rec.size();
    if (ticks_per_us) *ticks_per_us = s.probe_tpu;
    return (int64_t)(s.probe_meta.size() / 5);
  }
  // fill: *rec_entries holds rec's capacity in entries; meta must hold 5 x
  // the launches the size query returned
  if (!s.probe_taken) return fail(WPT_ERR_INVALID_ARG, "probe: call with meta = rec = NULL first (size query)");
  if (!rec_entries || *rec_entries < s.probe_rec.size())
    return fail(WPT_ERR_INVALID_ARG, "probe: rec smaller than the size query's entries");
  std::memcpy(meta, s.probe_meta.data(), s.probe_meta.size() * sizeof(uint32_t));
  std::memcpy(rec, s.probe_rec.data(), s.probe_rec.size() * sizeof(uint4));
  *rec_entries = s.probe_rec.size();
  if (ticks_per_us) *ticks_per_us = s.probe_tpu;
  const int64_t n = (int64_t)(s.probe_meta.size() / 5);
  s.probe_meta.clear();
  s.probe_rec.clear();
  s.probe_taken = false;
  return n;
}

int wpt_get_option(int32_t option, int64_t* value) {
  if (!value) return fail(WPT_ERR_INVALID_ARG, "null argument");
  if (option == WPT_OPT_BVH_BUILD) { *value = g_bvh_build; return WPT_OK; }
  if (!g_session) {
    auto it = g_default_opts.find(option);
    if (it != g_default_opts.end()) { *value = it->second; return WPT_OK; }
    Renderer probe;
    if (!probe.get_option(option, *value)) return fail(WPT_ERR_INVALID_ARG, "unknown option");
    return WPT_OK;
  }
  if (!g_session->renderer.get_option(option, *value)) return fail(WPT_ERR_INVALID_ARG, "unknown option");
  return WPT_OK;
}

int wpt_set_profiling(int on) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  g_session->renderer.set_profiling(on != 0);
  return WPT_OK;
}

int wpt_clear_stats(void) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  g_session->renderer.clear_stats();
  return WPT_OK;
}

int wpt_sync(void) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  std::string err;
  if (!g_session->renderer.sync(err)) return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

int wpt_bvh_depth(void) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  return (int)g_session->renderer.bvh_depth();
}

int wpt_trace_rays(size_t n, const float* rays, float* t_out, int32_t* id_out) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  std::string err;
  if (!g_session->renderer.trace_rays(n, rays, t_out, id_out, err)) return fail(WPT_ERR_DEVICE, err);
  return WPT_OK;
}

int wpt_shadow_rays(size_t n, const float* pq, const int32_t* light, uint8_t* occluded) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  std::string err;
  if (!g_session->renderer.shadow_rays(n, pq, light, occluded, err)) return fail(WPT_ERR_INVALID_ARG, err);
  return WPT_OK;
}

int wpt_shutdown(void) {
  if (!g_session) return fail(WPT_ERR_NOT_INIT, "init not called");
  delete g_session;
  g_session = nullptr;
  return WPT_OK;
}

// ---- host-only inspection ---------------------------------------------------
void* wpt_debug_scene_new(int32_t scene_id, const float* mesh_vertices, size_t num_vertices) {
  std::vector<float> mesh;
  if (mesh_vertices && num_vertices) mesh.assign(mesh_vertices, mesh_vertices + ((num_vertices / 3) * 9));
  HostScene* sc = new HostScene();
  std::string err;
  if (!build_scene(scene_id, mesh, *sc, err)) {
    delete sc;
    fail(WPT_ERR_INVALID_SCENE, err);
    return nullptr;
  }
  return sc;
}

void* wpt_debug_scene_new_gpu(int32_t scene_id, const float* mesh_vertices, size_t num_vertices) {
  // one builder for the process, on the device wpt_set_device chose; never
  // freed (its buffers would outlive the HIP runtime at exit)
  static BvhGpu* gpu = nullptr;
  const hipError_t he = hipSetDevice(g_device);
  if (he != hipSuccess) {
    fail(WPT_ERR_DEVICE, std::string("hipSetDevice failed: ") + hipGetErrorString(he));
    return nullptr;
  }
  if (!gpu) gpu = new BvhGpu();
  gpu->min_shapes = 0;
  std::vector<float> mesh;
  if (mesh_vertices && num_vertices) mesh.assign(mesh_vertices, mesh_vertices + ((num_vertices / 3) * 9));
  HostScene* sc = new HostScene();
  std::string err;
  if (!build_scene(scene_id, mesh, *sc, err, gpu)) {
    delete sc;
    fail(err.rfind("HIP error", 0) == 0 || err.rfind("GPU BVH", 0) == 0 ? WPT_ERR_DEVICE : WPT_ERR_INVALID_SCENE,
         err);
    return nullptr;
  }
  return sc;
}

int wpt_debug_scene_build_info(void* h, double* out) {
  if (!h || !out) return fail(WPT_ERR_INVALID_ARG, "null argument");
  const HostScene* sc = (const HostScene*)h;
  out[0] = sc->bvh_ms;
  out[1] = sc->bvh_on_gpu ? 1.0 : 0.0;
  return WPT_OK;
}

int wpt_debug_scene_info(void* h, uint64_t* out) {
  const HostScene* sc = (const HostScene*)h;
  if (!sc) return fail(WPT_ERR_INVALID_ARG, "null scene");
  uint64_t v[8] = {sc->shapes.size(), sc->num_inf, sc->nodes.size(), sc->lights.size(), sc->depth,
                   sc->use_bvh ? 1u : 0u, sc->tri_only ? 1u : 0u, sc->nodes4.size()};
  memcpy(out, v, sizeof v);
  return WPT_OK;
}

int wpt_debug_scene_nodes(void* h, uint32_t* out) {
  const HostScene* sc = (const HostScene*)h;
  if (!sc) return fail(WPT_ERR_INVALID_ARG, "null scene");
  for (size_t i = 0; i < sc->nodes.size(); i++) {
    const Node2& n = sc->nodes[i];
    float b[6] = {n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0], n.bmax[1], n.bmax[2]};
    memcpy(out + 8 * i, b, sizeof b);
    out[8 * i + 6] = n.left_first;
    out[8 * i + 7] = n.count;
  }
  return WPT_OK;
}

int wpt_debug_scene_nodes4(void* h, uint32_t* out) {
  const HostScene* sc = (const HostScene*)h;
  if (!sc) return fail(WPT_ERR_INVALID_ARG, "null scene");
  for (size_t i = 0; i < sc->nodes4.size(); i++) {
    const Node4& n = sc->nodes4[i];
    uint32_t* o = out + 37 * i;
    memset(o, 0, 37 * sizeof(uint32_t));
    for (int k = 0; k < 4; k++) {
      const uint32_t c = n.child[k];
      if (c == kChildEmpty) continue;
      o[0]++;
      uint32_t* e = o + 1 + 9 * k;
      if (!(c & 0x80000000u)) {
        e[0] = 1;
        e[1] = c;
      } else {
        e[0] = 2;
        if ((c & 0xC0000000u) == 0xC0000000u) {
          e[1] = sc->leaf_table[2 * (c & 0x3FFFFFFFu)];
          e[2] = sc->leaf_table[2 * (c & 0x3FFFFFFFu) + 1];
        } else {
          e[1] = c & 0xFFFFFFu;
          e[2] = (c >> 24) & 0x3Fu;
        }
      }
      const float b[6] = {n.xmin[k], n.ymin[k], n.zmin[k], n.xmax[k], n.ymax[k], n.zmax[k]};
      memcpy(e + 3, b, sizeof b);
    }
  }
  return WPT_OK;
}

int wpt_debug_scene_shapes(void* h, float* out) {
  const HostScene* sc = (const HostScene*)h;
  if (!sc) return fail(WPT_ERR_INVALID_ARG, "null scene");
  for (size_t i = 0; i < sc->shapes.size(); i++) {
    const Shape& s = sc->shapes[i];
    float* o = out + 16 * i;
    memcpy(o, s.g, sizeof s.g);
    o[12] = (float)s.kind;
    o[13] = s.emissive ? 1.0f : 0.0f;
    o[14] = 0.0f;
    o[15] = 0.0f;
  }
  return WPT_OK;
}

int wpt_debug_scene_lights(void* h, uint32_t* out) {
  const HostScene* sc = (const HostScene*)h;
  if (!sc) return fail(WPT_ERR_INVALID_ARG, "null scene");
  for (size_t i = 0; i < sc->lights.size(); i++) out[i] = sc->lights[i];
  return WPT_OK;
}

void wpt_debug_scene_free(void* h) { delete (HostScene*)h; }

}  // extern "C"
