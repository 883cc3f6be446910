/*
 * wpt.h — C ABI of the MI355X path-tracing core (libwpt.so).
 *
 * Drop-in boundary for sourcedennis/wasm-pathtracer's `src/wasm_interface.rs`
 * (the only FFI surface of the reference: primitive-only `#[wasm_bindgen]`
 * free functions over one global session). Each `wpt_<name>` below replaces
 * the reference export `<name>` cited next to it, with the same argument
 * meaning. Where the reference `panic!`s (a WASM trap) these functions return
 * a negative WPT_ERR_* status instead; wpt_last_error() gives the message.
 * Pointers returned to the caller stay owned by the library, valid until the
 * next init / viewport / scene / mesh change, as in the reference.
 *
 * Additions (no reference counterpart) are grouped at the end: render
 * options (depth cap, seed), multi-GPU pixel partition, f32 radiance access
 * for parity, statistics and kernel timings.
 *
 * Threading: like the reference (Rc/RefCell, one instance per worker) the
 * session is single-threaded; call from one host thread per process.
 */
#ifndef WPT_H
#define WPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (the reference panics instead) */
#define WPT_OK 0
#define WPT_ERR_NOT_INIT (-1)      /* "init not called"      wasm_interface.rs:131 */
#define WPT_ERR_ALREADY_INIT (-2)  /* "Cannot init again"    wasm_interface.rs:75  */
#define WPT_ERR_INVALID_SCENE (-3) /* "Invalid scene"        wasm_interface.rs:396 */
#define WPT_ERR_INVALID_ARG (-4)   /* "Invalid RenderType magic number" :212, bad sizes */
#define WPT_ERR_UNSUPPORTED (-5)   /* feature not in this core (e.g. a scene whose build is unsupported) */
#define WPT_ERR_DEVICE (-6)        /* HIP runtime error */
#define WPT_ERR_NO_MESH (-7)       /* "Mesh not allocated"   wasm_interface.rs:281 */

/* render types (wasm_interface.rs:207-214) */
#define WPT_NO_NEE 0
#define WPT_NORMAL_NEE 1
#define WPT_PNEE 2

/* ---- reference exports (src/wasm_interface.rs) ------------------------- */

/* init(width, height, scene_id, cam_x, cam_y, cam_z, cam_rot_x, cam_rot_y)
 * wasm_interface.rs:67-113. Scene ids: 0 = museum (scenes.rs:15-68), 2 = bunny
 * scene (mesh slot 1), plus the build-defined configs 100 (C1 box) and 101 (C2
 * spheres, BVH disabled). Initial settings as the reference's (:90-94): left
 * half NormalNEE with random sampling, right half PNEE with adaptive
 * sampling; the sampling view starts blue. */
int wpt_init(uint32_t width, uint32_t height, uint32_t scene_id, float cam_x, float cam_y, float cam_z,
             float cam_rot_x, float cam_rot_y);

/* results(is_show_sampling) -> *const u8 — wasm_interface.rs:120-134.
 * RGBA8, width*height*4 bytes, re-quantised as render_target.rs:62-64.
 * is_show_sampling = 1: the sampling view (SimpleRenderTarget). Every reset
 * (settings, viewport, camera, scene, render options) clears it to black and
 * the adaptive halves repaint themselves blue, as reset() / update_scene() /
 * update_settings() do in the reference (wasm_interface.rs:137-201). */
const uint8_t* wpt_results(uint32_t is_show_sampling);

/* update_scene(scene_id) — wasm_interface.rs:154-169 */
int wpt_update_scene(uint32_t scene_id);

/* update_settings(left_type, right_type, is_left_adaptive, is_right_adaptive,
 * is_light_debug) — wasm_interface.rs:173-204 */
int wpt_update_settings(uint32_t left_type, uint32_t right_type, uint32_t is_left_adaptive,
                        uint32_t is_right_adaptive, uint32_t is_light_debug);

/* update_viewport(width, height) — wasm_interface.rs:219-232 */
int wpt_update_viewport(uint32_t width, uint32_t height);

/* update_camera(x, y, z, rot_x, rot_y) — wasm_interface.rs:239-248 */
int wpt_update_camera(float cam_x, float cam_y, float cam_z, float cam_rot_x, float cam_rot_y);

/* allocate_mesh(id, num_vertices) — wasm_interface.rs:259-270 */
int wpt_allocate_mesh(uint32_t id, uint32_t num_vertices);

/* mesh_vertices(id) -> *mut Vec3 — wasm_interface.rs:275-287.
 * Packed f32 x,y,z per vertex, filled by the caller. NULL if not allocated. */
float* wpt_mesh_vertices(uint32_t id);

/* notify_mesh_loaded(id) -> bool — wasm_interface.rs:293-329.
 * Returns 1 if the active scene uses the mesh and was rebuilt, 0 if not. */
int wpt_notify_mesh_loaded(uint32_t id);
/* Mesh ingestion (the reference client's side of allocate_mesh /
 * mesh_vertices): parses OBJ text as src_ts/client/obj_parser.ts:3-51 does
 * (wasm-pathtracer_amd/csrc/wpt_obj.h: 'v' and triangular 'f' only, fields
 * split on single spaces, JavaScript parseFloat / parseInt) into mesh slot
 * `id` as a triangle soup, then scales it per axis if `scale` is non-null
 * (index.ts:216-220 uses (8, 8, -8) for the bunny). *num_vertices = 3 per
 * face. Call wpt_notify_mesh_loaded(id) next, as after mesh_vertices.
 * WPT_ERR_INVALID_ARG on a non-triangular face (the reference throws). */
int wpt_load_obj(uint32_t id, const char* text, size_t len, const float* scale, uint64_t* num_vertices);
/* The same parse without a session (host only): *num_vertices always; the
 * vertices (3 floats each) into `out` when it is non-null and holds
 * `capacity` vertices. */
int wpt_parse_obj(const char* text, size_t len, const float* scale, float* out, uint64_t capacity,
                  uint64_t* num_vertices);

/* allocate_texture(id, width, height) -> *mut (u8,u8,u8) — wasm_interface.rs:335-352 */
uint8_t* wpt_allocate_texture(uint32_t id, uint32_t width, uint32_t height);

/* notify_texture_loaded(id) -> bool (always false) — wasm_interface.rs:358-366 */
int wpt_notify_texture_loaded(uint32_t id);

/* compute(num_samples) — wasm_interface.rs:374-384 (RenderInstance::compute,
 * tracer.rs:103-123). Traces num_samples paths; pixels left of width/2 use
 * left_type, the others right_type.
 * As the reference (two RenderInstances, :377-379), each screen half has its
 * own sample sequence and gets n/2 (left) and n - n/2 (right) of the n
 * samples, on one rank whatever the strategies.
 * Deliberate differences (build-defined):
 *  - pixel order: a random half takes one sample per pixel per round in
 *    raster order (the reference picks pixels at random); whole rounds are
 *    traced in 8x8 tiles (the same (pixel, sample) pairs). An adaptive half
 *    takes AdaptiveSamplingStrategy's rounds (4 per pixel, then ceil(1 + 32
 *    scaled_mse)) in raster order instead of LIFO-shuffled order.
 *  - several ranks (wpt_set_partition / wpt_set_comm): with random halves
 *    compute(n) traces n paths over this rank's pixel list in partition order
 *    (path k -> pixel k mod P, sample k div P: per-GPU work fixed); with an
 *    adaptive half n positions of the GLOBAL per-half sequences (the same n
 *    on every rank).
 *  - RNG: each path has its own xorshift32 stream path_seed(seed, pixel,
 *    sample) with the reference's draw order inside the path.
 *  - PNEE: the 300000 photons are shot once, before the first path, on
 *    per-photon streams, and both halves share the one tree; the reference
 *    spends compute ticks on photons (32 per tick, tracer.rs:103-123) and
 *    builds one tree per half, so its first compute calls trace fewer paths. */
int wpt_compute(size_t num_samples);

/* ---- additions ---------------------------------------------------------- */

/* Last error message (thread-local to the session). */
const char* wpt_last_error(void);

/* Select the HIP device before wpt_init (default: 0). */
int wpt_set_device(int device);

/* Depth cap (0 = the reference's unbounded Russian-roulette loop), frame seed
 * for the per-path xorshift32 streams (default 0xBABABEBE, rng.rs:11) and the
 * number of paths resident per wavefront batch (0 = keep). Resets accumulation. */
int wpt_set_render_options(int32_t max_depth, uint32_t frame_seed, uint64_t batch_paths);

/* Multi-GPU partition: square tiles of `tile` px in raster order, tile t is
 * rendered by rank t % nranks; a rank's pixels are listed tile by tile, 8x8
 * sub-tiles in raster order inside a tile. Resets accumulation. */
int wpt_set_partition(uint32_t rank, uint32_t nranks, uint32_t tile);

/* Number of pixels of this rank's partition; fills `out` (may be NULL) with
 * their viewport indices (y*width+x) in partition order. */
int64_t wpt_partition_pixels(uint32_t* out);

/* Host-only (no session, no GPU): the pixel list wpt_set_partition would give
 * rank `rank` of `nranks` on a width x height viewport; returns its length. */
int64_t wpt_tile_partition(uint32_t width, uint32_t height, uint32_t rank, uint32_t nranks, uint32_t tile,
                           uint32_t* out);

/* PNEE photon octree (photon_tree.rs), built on first use: shoots photons
 * k = 0,1,... on per-photon streams until 300000 are stored (tracer.rs:104),
 * inserts them in photon order, freezes the CDFs. Returns the node count;
 * fills (each may be NULL) child[node] (first of 8 children, 0 = leaf),
 * cum[node * num_lights + light] (cum_bins) and shot_stored[2]. */
int64_t wpt_photon_tree(uint32_t* child, float* cum, uint64_t* shot_stored);

/* Accumulated radiance: acc3 = width*height*3 f32 (sum over samples, as
 * RenderTarget.acc_buffer), cnt = width*height u32 (acc_count). */
int wpt_read_radiance(float* acc3, uint32_t* cnt);

/* Device-to-device copy of this rank's partition as float4 (acc.xyz, count)
 * into `device_dst` (partition_pixels * 16 bytes, same device). */
int wpt_copy_partition(void* device_dst);

/* Adaptive sampling over several ranks. A round's error
 * estimate reads every pixel's radiance, including the 2-pixel halo of
 * gaussian5 (render_target.rs:112-128) across tile borders, so at each round
 * boundary the ranks exchange their partitions: the library packs its own
 * (float4 per partition pixel: acc.xyz, sample count as u32 bits) into
 * `local_dev` and calls fn(user), which must all-gather the `slot`-float4
 * buffers of all ranks, rank-major, into `gathered_dev` (nranks * slot float4,
 * same device), synchronised, and return 0 (non-zero aborts compute). Every
 * rank then plans the same global round over the whole frame.
 * With adaptive halves and several ranks, compute(n) advances the GLOBAL
 * round sequence by n positions (every rank passes the same n) and each rank
 * traces the positions on its own pixels; the union of the partitions is then
 * bitwise the single-rank frame after compute(n). fn = NULL unregisters. */
typedef int (*wpt_exchange_fn)(void* user);
int wpt_set_exchange(wpt_exchange_fn fn, void* user, void* local_dev, void* gathered_dev, uint64_t slot);
/* float4 entries per rank the exchange needs (the largest partition). */
int64_t wpt_exchange_slot(void);

/* Multi-GPU over RCCL (the reference has no collective, its
 * README intends pixel partitions over 8 workers, README.md:87). One process
 * per GPU. Rank 0 makes a 128-byte id with wpt_comm_unique_id and the host
 * hands it to every rank (any channel); every rank then calls wpt_set_comm
 * (collective): its partition = tiles of `tile` px dealt round-robin
 * (wpt_set_partition), plus an RCCL communicator. compute() then traces only
 * the rank's pixels with no communication; with adaptive halves the ranks
 * exchange the frame at round boundaries over the communicator
 * (ncclAllGather), so every rank must pass the same n to compute().
 * wpt_gather_frame(root) (collective): every rank's partition into the root's
 * frame (grouped ncclSend / ncclRecv over xGMI); results() / read_radiance()
 * on the root then return the whole image. */
int wpt_comm_unique_id(void* out128);
int wpt_set_comm(uint32_t rank, uint32_t nranks, uint32_t tile, const void* unique_id128);
int wpt_gather_frame(uint32_t root);
int wpt_comm_destroy(void);
/* A caller's transport instead of RCCL (another collective library, a host
 * staging path, a test harness). After wpt_set_partition(rank, nranks, tile),
 * register fn with two device buffers of this rank's device: send_dev (slot
 * float4) and recv_dev (nranks * slot float4, rank-major), slot >=
 * wpt_exchange_slot(). The library packs this rank's partition into send_dev
 * (float4 per partition pixel: acc.xyz, count as u32 bits; the device is
 * synchronised) and calls fn(user, op, root):
 *   WPT_XFER_GATHER    (wpt_gather_frame): every rank's send_dev into root's
 *                      recv_dev at slot offset r * slot (gather plan below);
 *   WPT_XFER_ALLGATHER (adaptive round boundaries): the same into every rank's.
 * fn returns 0 once the data is in place (non-zero fails the call); the root
 * then unpacks recv_dev into its frame. Registering a transport replaces
 * (destroys) an RCCL communicator set with wpt_set_comm; a registration the
 * call rejects changes nothing. fn = NULL unregisters the transport only;
 * wpt_set_comm and wpt_comm_destroy drop it. */
#define WPT_XFER_GATHER 0
#define WPT_XFER_ALLGATHER 1
typedef int (*wpt_transport_fn)(void* user, int32_t op, uint32_t root);
int wpt_set_transport(wpt_transport_fn fn, void* user, void* send_dev, void* recv_dev, uint64_t slot);
/* Host-only: the point-to-point transfers of a rooted gather as rank `rank`
 * posts them (what wpt_gather_frame runs over RCCL: grouped ncclSend /
 * ncclRecv): out[4i..4i+3] = {peer, float4 offset in root's buffer, float4
 * count, 1 = receive / 0 = send}; returns the count (nranks - 1 at the root,
 * 1 elsewhere, 0 for one rank). */
int64_t wpt_gather_plan(uint32_t rank, uint32_t nranks, uint32_t root, uint64_t slot, uint64_t* out);
/* Host-only: the sequential f32 sum ((0 + v[0]) + v[1]) + ... bit for bit,
 * as the adaptive rounds compute the reference's mse_sum
 * (sampling_strategy.rs:138-141) — exposed for its tests. */
float wpt_seq_sum(const float* v, uint64_t n);
/* Host-only: the same sum from per-chunk effects (wpt_seqsum.h: the chunks'
 * effects by the host restatement, then the ordered walk the adaptive rounds
 * run) — exposed for its tests. */
float wpt_seq_sum_chunks(const float* v, uint64_t n);
/* The same sum with the chunk effects computed on the session's device
 * (k_sum_chunks / k_sum_scan / k_sum_eff, as every adaptive round does), the
 * walk on the host: *out = the sum. For its tests; needs wpt_init. */
int wpt_seq_sum_device(const float* v, uint64_t n, float* out);

/* stats: out[0..39] = paths, rays (primary+extension), shadow rays, BVH node
 * visits, primitive tests, bounce iterations, then per kernel (extend, shadow):
 * node visits, primitive tests, node bytes fetched, then the fast-path rays
 * re-traced by the exact traversal (extend, shadow), then traversal-loop
 * iterations summed over lanes and those with a live ray (extend, shadow),
 * then PNEE photon rays shot and photons stored (tracer.rs:126-152), then
 * the adaptive rounds' error sums: chunks walked, chunks re-summed element
 * by element, and of those the ones copied on demand; then the samples
 * adaptive rounds took from the sample stock (WPT_OPT_STOCK; a sample's
 * rays count when a round takes it) and the paths of a random half traced on
 * the fill lane (WPT_OPT_FILL), then
 * the algorithmic bytes of the fused extend + shadow launches, then the paths
 * RR-only batches handed to k_finish and the most bounces one of them took,
 * then the most node visits of one ray in a fused k_trace launch, then
 * the traversal loop's body SIMD use: lanes about to expand an internal node
 * summed over wave iterations, the iterations in which any lane did, and the
 * same for leaf tests (lanes / bodies <= 64); out[33] = samples traced
 * into the stock (refills and round deficits), out[34] = of those the
 * rounds' deficits, out[35] = rounds that waited for a refill still in
 * flight, out[36..37] = host microseconds in round planning and in the
 * stock's round step, out[38] = rays traced into the stock (extension +
 * shadow; rays and shadow rays count a stocked sample's when a round takes it),
 * out[39] = of rays + shadow rays, those of samples taken from the stock.
 * Visit/test/byte/iteration counts are only gathered with counting on. */
int wpt_stats(uint64_t* out, size_t n);
/* per-kernel device time (profiling on): out[0..11] = {ms, launches} ×
 * {generate, extend, shade, shadow, accumulate, trace (fused extend +
 * shadow)}, summed over launches; the lanes' launches overlap, so
 * out[12..23] = {busy ms, logical launches} per kernel: the union of its
 * launch intervals, and launches counted once per bounce (generate /
 * accumulate: once per batch); out[24..27] = 0 (were the round-4 fast tree's
 * re-trace drains). */
int wpt_kernel_times(double* out, size_t n);
int wpt_set_counting(int on);
int wpt_set_profiling(int on);
/* Concurrent lanes (slices of a batch traced on their own HIP streams) of
 * the next compute calls: 1 .. 8 (default 4). 1 serialises the kernels and
 * gives its traversal kernels the whole GPU (multi-lane batches use
 * WPT_OPT_GRID_PCT of it), so wpt_kernel_times then gives their standalone
 * times. The frame is bit-identical for any count. */
int wpt_set_lanes(int32_t n);
/* Launch configuration (no environment variable changes it; the built-in
 * defaults are the measured production settings). With no
 * session it sets the default of every later wpt_init (WPT_OPT_DEFAULTS
 * restores the built-in ones); with a session it changes that session only
 * (scene / partition rebuilt where the option shapes them, accumulation reset
 * then). The frame is bit-identical for every setting. */
#define WPT_OPT_DEFAULTS 0       /* no session: forget every default set so far (value ignored) */
#define WPT_OPT_TRAVERSAL 1      /* extension rays: 0 exact BVH2, 1 BVH4 fast path + exact re-trace, 3 auto (default: BVH4 on scenes with
                                    other shapes than triangles, else BVH2); 2 (the fast tree) was removed in round 5 */
#define WPT_OPT_TRAVERSAL_SH 2   /* shadow rays: the same choice */
#define WPT_OPT_FUSED 3          /* 1: every batch traces bounce b's extension + b-1's shadow rays in one launch */
#define WPT_OPT_FUSED_BELOW 4    /* batches below this many paths run fused (default 2^24) */
#define WPT_OPT_SMALL_LANES 5    /* lane cap of those small batches (default 2) */
#define WPT_OPT_PIXEL_TILE 6     /* whole sample rounds traced in tiles of this many px (default 8; 0 raster) */
#define WPT_OPT_GRID_PCT 7       /* traversal grids of multi-lane batches, % of resident capacity (default 50) */
#define WPT_OPT_REFILL 8         /* idle lanes of a wave before it takes new extension rays (default 12) */
#define WPT_OPT_REFILL_SH 9      /* the same for shadow rays (default 16) */
#define WPT_OPT_TREELET 10       /* LDS treelet of the BVH2's top node pairs (default 1) */
#define WPT_OPT_BVH_BUILD 11     /* BVH2 build: 0 GPU for >= 65536 finite shapes (default), 1 host, 2 GPU */
#define WPT_OPT_LANES 12         /* as wpt_set_lanes (1..8, default 4; one HIP stream each: more lanes than the process has hardware queues (GPU_MAX_HW_QUEUES, 4 by default) share them) */
#define WPT_OPT_FINISH_BELOW 13  /* RR-only batches: once at most this many paths live, one kernel runs each to its end (default 262144; 0 never) */
#define WPT_OPT_TRACE_GRID_PCT 14 /* grid of the fused k_trace (small batches), % of resident capacity (default 75) */
/* 15-19 and 21 (the fast tree's build and drain options) were removed in round 5 */
#define WPT_OPT_FINISH_EVERY 20  /* RR-only batches: bounces between reads of the live count (a host round trip; default 4) */
#define WPT_OPT_PROBE 22         /* record the wave timelines of the next N traversal launches (wpt_probe_read; default 0 = off) */
#define WPT_OPT_STOCK 23         /* adaptive halves (one rank): per-pixel ring of this many samples traced ahead of the rounds
                                    by refill batches on the async lanes; a round adds its samples from it in sample order
                                    and traces only what it lacks (0 off, or a power of two 64..4096; default 1024, halved
                                    while pixels x slots exceed 2^32 or the ring 48 GB) */
#define WPT_OPT_STOCK_LANES 24   /* async lanes the refills rotate over, 1..5 (default 2) */
#define WPT_OPT_FILL 25          /* one random + one adaptive half (the reference's init defaults): the random half's whole
                                    rounds outside its 2 seam columns run on the fill lane beside the adaptive half's
                                    rounds (default 0: slower than the main lanes once the stock is on) */
#define WPT_OPT_ASYNC_PRIO 26    /* 1: those async batches on low-priority streams (default 0) */
#define WPT_OPT_ASYNC_GRID_PCT 27 /* their persistent traversal grids, % of the resident capacity (0: the main batches';
                                    default 100) */
#define WPT_OPT_STOCK_AHEAD 30   /* a refill stocks a pixel to c + min(ahead * c + extra, slots - c) samples past its count,
                                    c = its samples in the round just planned (default 40) */
#define WPT_OPT_STOCK_EVERY 32   /* a refill after every this many rounds of a half (default 3) */
#define WPT_OPT_STOCK_EXTRA 33   /* see WPT_OPT_STOCK_AHEAD (default 8) */
#define WPT_OPT_ASYNC_ONESHOT 31 /* 1: async batches' traversal grids cover every ray (one feed chunk per wave), so their blocks
                                    retire with their rays instead of holding CUs for a whole bounce (default 0) */
#define WPT_OPT_STOCK_PREFILL 35 /* 1: each compute call first refills the adaptive halves' stock from their last round's
                                    counts, sized to the call's budget (default 1) */
#define WPT_OPT_ASYNC_FUSED_BELOW 36 /* async batches (stock refills, filler) below this many paths run the fused k_trace
                                      (0: WPT_OPT_FUSED_BELOW; default 2^26) */
#define WPT_OPT_LOG 34           /* 1: host steps of adaptive rounds / the stock to stderr (debugging; default 0) */
#define WPT_OPT_SCENE_TRAVERSAL 28 /* read-only (wpt_get_option): what the session's scene runs: 0 exact BVH2, 1 BVH4, 2 linear
                                      scan (BVH disabled), -1 no scene */
#define WPT_OPT_SCENE_TRI_ONLY 29  /* read-only: 1 if the scene's finite shapes are all triangles (-1 no scene) */
int wpt_set_option(int32_t option, int64_t value);
/* Wave timelines of the traversal launches recorded since WPT_OPT_PROBE was
 * set (measurement only; the probe costs a clock read per wave and per feed
 * refill, results are the same bits). Returns the launches recorded; with
 * meta and rec non-NULL fills meta[5i..5i+4] = {kernel (1 extend, 3 shadow,
 * 5 fused trace), lane, bounce, waves, first entry} and rec[4e..4e+3] =
 * {start, the moment the wave's work feed ran dry, end, rays taken} per wave
 * entry e (steady-clock ticks, ticks_per_us of them per microsecond), then
 * restarts the recording. Call it first with meta = rec = NULL (the size
 * query: it takes the snapshot and sets *rec_entries to the entries rec must
 * hold), then with buffers: *rec_entries = rec's capacity in entries, meta
 * of 5 x the launches the query returned. */
int64_t wpt_probe_read(uint32_t* meta, uint32_t* rec, uint64_t* rec_entries, double* ticks_per_us);
int wpt_get_option(int32_t option, int64_t* value);
/* The active scene's BVH2 build: out[0] = build ms (host wall clock, or the
 * GPU build's device time incl. its copies), out[1] = 1 if it was built on
 * the GPU. Scenes with >= 65536 finite shapes are built on the GPU
 * (wpt_bvh_gpu.h, bvh.rs:103-437 level by level, the same tree);
 * WPT_OPT_BVH_BUILD forces either. */
int wpt_scene_build_info(double* out);
int wpt_clear_stats(void);
int wpt_sync(void);
/* BVH2 depth of the active scene. */
int wpt_bvh_depth(void);

/* Parity hooks: closest hit (Scene::trace_g, scene.rs:162-184) for n rays
 * {ox,oy,oz,dx,dy,dz}; t = +inf and id = -1 on a miss. Shadow query
 * (Scene::shadow_ray, scene.rs:104-133) for {p.xyz, q.xyz} and light shape ids. */
int wpt_trace_rays(size_t n, const float* rays, float* t_out, int32_t* id_out);
int wpt_shadow_rays(size_t n, const float* pq, const int32_t* light, uint8_t* occluded);

/* Tear the session down (the reference never does); allows a new wpt_init.
 * The sample stock's two ring blocks (about 42 GB at 1080p) stay with the
 * process for the next session's ring on the device (at most 4 blocks);
 * they are freed when an allocation would otherwise fail. */
int wpt_shutdown(void);

/* Host-only scene inspection (no GPU): builds a scene like wpt_init would and
 * exposes the reordered shapes and the BVH2 nodes for structural parity. */
void* wpt_debug_scene_new(int32_t scene_id, const float* mesh_vertices, size_t num_vertices);
/* out[0..7] = shapes, infinite shapes, nodes, lights, BVH depth, use_bvh, tri_only, BVH4 nodes */
int wpt_debug_scene_info(void* h, uint64_t* out);
/* The BVH4 (bvh4.rs:37-281 DP tree cut, F4 leaf fix): 37 u32 per node =
 * num_children, then per child slot {kind (0 empty, 1 node, 2 leaf), node
 * index | first shape, leaf count, 6 f32 bounds bits}. */
int wpt_debug_scene_nodes4(void* h, uint32_t* out);
/* 8 u32 per node: 6 f32 bounds bits (x_min,y_min,z_min,x_max,y_max,z_max), left_first, count */
int wpt_debug_scene_nodes(void* h, uint32_t* out);
/* 16 f32 per shape: geometry[12], kind, emissive, material rgb[...] packed as in wpt_scene.h */
int wpt_debug_scene_shapes(void* h, float* out);
int wpt_debug_scene_lights(void* h, uint32_t* out);
void wpt_debug_scene_free(void* h);
/* The same scene with its BVH2 built on the GPU (the device of
 * wpt_set_device, default 0) whatever its size; same accessors. */
void* wpt_debug_scene_new_gpu(int32_t scene_id, const float* mesh_vertices, size_t num_vertices);
/* out[0] = BVH2 build ms, out[1] = 1 if built on the GPU. */
int wpt_debug_scene_build_info(void* h, double* out);

#ifdef __cplusplus
}
#endif

#endif /* WPT_H */
