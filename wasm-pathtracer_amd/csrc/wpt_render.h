// wpt_render.h — the wavefront renderer behind the C ABI.
//
// One Renderer per process/GPU. It owns the device copy of the scene, the
// accumulation buffers of its pixel partition and the per-path SoA state of
// the wavefront pipeline (generate → [extend → shade → shadow]* → accumulate),
// replacing RenderInstance::compute_rays + trace_original_color
// (src/tracer.rs:156-330) for a whole batch of paths at once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <algorithm>
#include <deque>
#include <vector>

#include "wpt_scene.h"
#include "wpt_seqsum.h"

namespace wpt {

constexpr int kMaxInf = 16;       // infinite shapes (planes) kept in the kernel argument block
constexpr int kMaxBvhDepth = 4096;  // traversal stack: LDS slots + global spill sized from the BVH depth
constexpr int kMaxBounces = 512;  // hard cap for the RR-only (unbounded) mode

// Read-only scene view passed by value to the kernels.
struct DevScene {
  const float4* nodes;      // BVH2: 2 float4 per node (bounds, left_first, count)
  const float4* tree;       // LDS treelet source: 4 float4 per node pair (wpt_render.hip kTreePairs)
  uint32_t tree_pairs, tree_root_lf;
  const float4* prims;      // 4 float4 per finite shape (shape index - num_inf)
  const uint32_t* kinds;    // ShapeKind per finite shape
  const float4* all;        // 4 float4 per shape, every shape (linear scan, BVH disabled)
  const uint32_t* all_kinds;
  const float4* mats;       // per shape: rgb (colour or intensity), w = 1 if emissive
  const float4* lights;     // 5 float4 per light: (v0,area) (v1,shape id) (v2,-) (n,-) (I,-)
  const float4* nodes4;     // fast-path BVH4: 8 float4 (128 B) per node (wpt_scene.h Node4)
  const uint32_t* leaf_table;
  uint32_t num_inf, num_finite, num_shapes, num_lights;
  uint32_t use_bvh, tri_only;
  uint32_t refill_lanes;     // persistent kernels refill idle lanes once this many are idle
  uint32_t refill_lanes_sh;  // (the same for the shadow kernel)
  int stack_cap;             // traversal stack entries per lane (LDS slots + spill)
  uint32_t* overflow;        // device flag: a traversal stack would have overflowed
  const uint32_t* oct_child;  // PNEE octree (wpt_photon.h): first child per node, 0 = leaf
  const float* oct_cum;       // frozen cum_bins, num_lights per node
  const uint32_t* oct_corners;  // per node x 8 offset cases: the 8 cells of the trilinear mix (null: walk them)
  uint32_t oct_nodes;         // 0: no tree (PNEE paths then cannot run)
  uint32_t oct_lds_words;     // words of the tree k_shade copies to LDS: nodes (child) [+ nodes * lights (cum)], 0 = none
  float bg[3];
  float4 planes[kMaxInf];   // infinite shapes: (normal.xyz, normal·location)
  // wave timeline probe (WPT_OPT_PROBE) of this launch, or null: per wave of
  // the grid {start, feed ran dry, end (steady clock ticks), rays taken}
  uint4* probe;
};

struct Stats {
  uint64_t paths = 0;
  uint64_t rays = 0;          // primary + extension (extend launches)
  uint64_t shadow_rays = 0;
  uint64_t node_visits = 0;   // only when counting is enabled
  uint64_t prim_tests = 0;
  uint64_t bounces = 0;       // bounce iterations executed
  // per-kernel work split (counting on): extend / shadow
  uint64_t ext_visits = 0, ext_tests = 0, ext_node_bytes = 0;
  uint64_t sh_visits = 0, sh_tests = 0, sh_node_bytes = 0;
  uint64_t fallback_ext = 0, fallback_sh = 0;  // fast-path rays re-traced exactly (tie / quirk)
  // traversal-loop bodies (counting on): lanes that expand an internal node /
  // test a leaf per wave iteration, and the iterations in which each body ran
  uint64_t ex_body_lanes = 0, ex_bodies = 0, lf_body_lanes = 0, lf_bodies = 0;
  // traversal loop iterations summed over lanes, and those with a live ray
  // (counting on): live/lane = SIMD occupancy of the traversal loop
  uint64_t ext_lane_iters = 0, ext_live_iters = 0, sh_lane_iters = 0, sh_live_iters = 0;
  // PNEE preprocessing (tracer.rs:126-152): photon rays shot, photons stored
  uint64_t photon_rays = 0, photons = 0;
  // algorithmic bytes of the fused extend + shadow launches (counting on),
  // with bench.py's per-ray formula
  uint64_t trace_bytes = 0;
  uint64_t max_ray_visits = 0;  // the most node visits of one ray in a fused k_trace (counting on)
  // adaptive rounds' error sums: chunks walked, re-summed element by element,
  // and of those copied on demand (not packed by k_sum_pack)
  uint64_t sum_chunks = 0, sum_resummed = 0, sum_fetched = 0;
  // RR-only tails run by k_finish: paths handed over, and the most bounces
  // one of them still took (the tail's length)
  uint64_t finish_paths = 0, finish_max_bounces = 0;
  // adaptive halves' sample stock (wpt_stock.h): samples traced into it
  // (refills and round deficits) and samples the rounds took from it; a
  // random half's paths traced on the fill lane
  uint64_t stock_traced = 0, stock_consumed = 0, fill_paths = 0;
  // of those: traced by the rounds themselves (their deficits), and rounds
  // whose samples were not all traced when the round wanted them; host time
  // (us) in round planning and in the stock's round step
  uint64_t stock_deficit = 0, stock_waits = 0, plan_us = 0, stock_us = 0;
  uint64_t stock_rays = 0;  // rays traced into the stock (they count in rays / shadow_rays when consumed)
  uint64_t stock_rays_used = 0;  // of rays + shadow_rays: those of samples taken from the stock
};

// Kernel-time accumulators (ms), filled when profiling is on.
// The lanes' launches of one kernel overlap in time: busy[k] = the union of
// kernel k's launch intervals (time during which at least one of its launches
// was in flight), logical[k] = launches counted once per batch step (generate /
// accumulate: one per batch; extend / shade / shadow: one per bounce).
// trace = the fused extend + shadow kernel (k_trace).
// retrace: unused since round 5 (the fast tree's drains; kept so that
// wpt_kernel_times keeps its layout, always 0).
constexpr int kTimedKernels = 7;
struct KernelTimes {
  double generate = 0, extend = 0, shade = 0, shadow = 0, accumulate = 0, trace = 0, retrace = 0;
  uint64_t n_extend = 0, n_shadow = 0, n_shade = 0, n_generate = 0, n_accumulate = 0, n_trace = 0, n_retrace = 0;
  double busy[kTimedKernels] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t logical[kTimedKernels] = {0, 0, 0, 0, 0, 0, 0};
};

// One lane of the wavefront: the dense streams of a slice of a batch, its own
// stream, counters and traversal-stack spill area. A batch is split over the
// lanes and their kernels run concurrently, so one lane's per-bounce launch
// tails (persistent kernels draining) are filled by the other lanes' work;
// only the in-order accumulation is chained lane after lane.
//
// Per path of the slice: the ray streams of two consecutive bounces (ping-
// pong: bounce b reads ray[b & 1], its survivors are appended to
// ray[(b + 1) & 1]), the hit record of bounce b's rays, the shadow stream of
// one bounce, and the radiance (and pixel) at the path's batch index.
//
// counts (u32): [0] = bounce 0's ray count (k_generate), then per bounce b a
// 64-bit append counter at u32 index 2 + 2b: low word = rays of bounce b + 1,
// high word = shadow rays emitted at bounce b (k_shade adds both at once).
constexpr int kMaxLanes = 8;  // streams made per session (lanes used: nlanes_)
constexpr uint64_t kMinLanePaths = 1024;  // smaller batches run on one lane
// after the per-bounce words: rays and shadow rays traced by k_finish (the
// path-at-a-time tail of RR-only batches)
constexpr size_t kFinishWord = 2 + 2 * (size_t)kMaxBounces;
constexpr size_t kCountWords = kFinishWord + 4;  // k_finish: rays, shadow rays, paths, longest path (bounces)
constexpr uint32_t kWorkWords = 16;   // device work counters (COUNT builds), see d_work_
constexpr uint32_t kWorkCopies = 64;  // copies of them, one per blockIdx % 64 (spreads the atomics)
struct PathSet {
  hipStream_t stream = nullptr;  // lane 0: the renderer's main stream
  hipStream_t lo = nullptr;      // async batches with WPT_OPT_ASYNC_PRIO: a low-priority stream (lazily made)
  hipEvent_t done = nullptr;     // recorded after the lane's accumulation
  uint64_t cap = 0;
  uint32_t* pixel = nullptr;     // per path: pixel (round batches: partition pixel index)
  float4* col = nullptr;         // per path: radiance
  float4* ro[2] = {nullptr, nullptr};
  float4* rd[2] = {nullptr, nullptr};
  float4* thr[2] = {nullptr, nullptr};
  float* t = nullptr;
  int32_t* id = nullptr;
  float4 *so = nullptr, *sd = nullptr, *sc = nullptr;
  uint32_t* counts = nullptr;    // kCountWords, see above
  uint32_t* h_counts = nullptr;  // pinned mirror
  uint2* spill = nullptr;
  size_t spill_cap = 0;
};

// One batch of the wavefront in flight: its path mapping, its lanes and how
// far its launches are issued. A batch on the main lanes is issued and waited
// for at once (run_batch). An asynchronous batch runs on the async lanes
// (lanes kAsyncLane0 ..) beside the main lanes' work: a refill of the
// adaptive halves' sample stock (wpt_stock.h), or a random half's whole
// rounds under an adaptive half's rounds (the filler); pump() issues it piece
// by piece, because an RR-only batch's launches depend on live counts read
// back every finish_every bounces.
constexpr int kAsyncLane0 = 2;
struct Batch {
  enum State { kNew, kBouncing, kCountWait, kIssued };
  // positions k0 .. k0+n-1 of: half h's current round (half >= 0), the
  // explicit mapping below (moff != null), or the uniform sequence path k ->
  // (part[k % npix], k / npix)
  uint64_t k0 = 0, n = 0;
  int half = -1;
  const uint32_t* part = nullptr;
  uint32_t npix = 0;
  // explicit mapping (k_generate): entry p covers positions [moff[p],
  // moff[p+1]) with samples mbase[p] ..; entry p is pixel mlist[p] (or the
  // partition pixel p); a stock batch stores its radiance into the ring
  const uint32_t* moff = nullptr;
  const uint32_t* mbase = nullptr;
  const uint32_t* mlist = nullptr;
  uint32_t nent = 0;
  bool stock = false;
  bool async = false;
  int queue = 0;      // async: 0 stock refills, 1 a random half's filler (each its own lanes, in order)
  int lane0 = 0, nl = 1;
  uint64_t off[kMaxLanes + 1] = {};
  bool fused = false, pnee = false;
  int maxb = 0, b = 0;  // bounce cap, next bounce to issue
  bool finished = false;  // the tail ran as k_finish
  State state = kNew;
  hipEvent_t done[kMaxLanes] = {};  // async: per lane, its slice done
  hipEvent_t live[kMaxLanes] = {};  // async RR-only: the live count landed in hl
  uint32_t* hc = nullptr;           // async: pinned nl x kCountWords, the final counts
  uint32_t* hl = nullptr;           // async: pinned nl live-count words
};

class Renderer {
 public:
  Renderer();
  ~Renderer();
  bool set_device(int dev, std::string& err);
  bool upload_scene(const HostScene& sc, std::string& err);
  bool set_viewport(uint32_t w, uint32_t h, std::string& err);
  void set_camera(const float cam[5]);
  void set_types(int left, int right, int debug) { left_type_ = left; right_type_ = right; debug_ = debug; }
  // AdaptiveSamplingStrategy per screen half (wpt_adaptive.h); takes effect
  // with the next reset
  void set_adaptive(bool left, bool right) { adaptive_[0] = left; adaptive_[1] = right; }
  bool adaptive() const { return adaptive_[0] || adaptive_[1]; }
  // sampling view (results(1), the SimpleRenderTarget): the whole view blue
  // (both strategies' constructors at init, sampling_strategy.rs:42-51,
  // :205-213); reset() clears it and repaints the adaptive halves blue
  bool fill_sampling_blue(std::string& err);
  bool sampling_rgba(uint8_t* out, std::string& err);
  void set_options(int max_depth, uint32_t seed, uint64_t batch) {
    if (seed != seed_) photons_ok_ = false;  // the photon streams derive from the frame seed
    max_depth_ = max_depth; seed_ = seed; if (batch) batch_ = batch;
  }
  // PNEE: shoot photons until kPhotonsNeeded are stored, build + freeze the
  // octree on the host, upload it. Done lazily by compute() when a half of
  // the screen renders PNEE; `photon_tree` exposes the frozen tree.
  bool build_photons(std::string& err);
  bool photon_tree(std::vector<uint32_t>& child, std::vector<float>& cum, uint64_t& shot, uint64_t& stored,
                   std::string& err);
  bool set_partition(uint32_t rank, uint32_t nranks, uint32_t tile, std::string& err);
  bool reset(std::string& err);                 // clears accumulation + path counter
  bool compute(uint64_t num_paths, std::string& err);
  bool sync(std::string& err);
  bool results_rgba(uint8_t* host_out, std::string& err);
  bool read_radiance(float* acc3, uint32_t* cnt, std::string& err);
  bool copy_partition(float* dev_dst, std::string& err);   // compact (acc.xyz,cnt) of own pixels
  // Frame exchange of adaptive rounds over several ranks (wpt_set_exchange):
  // fn(user) all-gathers every rank's `slot` float4 at local_dev into
  // gathered_dev (rank-major). exchange_slot() = largest partition.
  using ExchangeFn = int (*)(void*);
  void set_exchange(ExchangeFn fn, void* user, void* local_dev, void* gathered_dev, uint64_t slot) {
    xfn_ = fn; xuser_ = user; xlocal_ = (float4*)local_dev; xall_ = (float4*)gathered_dev; xslot_ = slot;
  }
  uint64_t exchange_slot() const { return maxpart_; }
  uint32_t rank() const { return rank_; }
  uint32_t nranks() const { return nranks_; }
  uint32_t tile() const { return tile_; }
  bool unpack_ranks(const float4* gathered, uint64_t slot, std::string& err);
  bool trace_rays(size_t n, const float* rays, float* t_out, int32_t* id_out, std::string& err);
  bool shadow_rays(size_t n, const float* pq, const int32_t* light, uint8_t* occ, std::string& err);
  // the recorded wave timelines (WPT_OPT_PROBE), then recording restarts
  bool probe_read(std::vector<uint32_t>& meta, std::vector<uint4>& rec, double& ticks_per_us, std::string& err);
  void set_counting(bool on) { counting_ = on; }
  void set_profiling(bool on) { profiling_ = on; }
  // concurrent lanes of the next batches (1..the count made at set_device);
  // one lane serialises the kernels (their standalone times)
  bool set_lanes(int n) {
    if (n < 1 || n > lanes_made_) return false;
    nlanes_ = n;
    return true;
  }
  int lanes() const { return nlanes_; }
  // true if `opt` shapes the device scene (re-uploaded when it changes)
  static bool scene_option(int opt) { return opt == 1 || opt == 2 || opt == 10; }
  // Launch configuration (wpt_set_option, include/wpt.h WPT_OPT_*). No
  // environment variable changes it: the defaults below are the measured
  // production settings. Options that shape the device scene
  // (traversal, treelet) take effect at the next upload_scene, the pixel tile
  // at the next set_partition; the caller (wpt_api.cpp) re-runs those.
  bool set_option(int opt, int64_t v, std::string& err);
  bool get_option(int opt, int64_t& v) const;
  // the scene build's BVH4 collapse (HostScene::want_bvh4): 1 always
  // (traversal bvh4), 2 for scenes with other shapes than triangles (auto)
  int wants_bvh4() const {
    return (traversal_ == 1 || traversal_sh_ == 1) ? 1 : (traversal_ == 3 || traversal_sh_ == 3) ? 2 : 0;
  }
  // the adaptive rounds' sum path on host data (tests): chunk effects on the
  // device, the walk on the host
  bool seq_sum_device(const float* v, uint64_t n, float& out, std::string& err);
  const Stats& stats() const { return stats_; }
  const KernelTimes& times() const { return times_; }
  void clear_stats() {
    std::string e;
    (void)flush_counts(e);  // a batch still in flight must not land in the cleared counters
    stats_ = Stats();
    times_ = KernelTimes();
  }
  bool flush_counts(std::string& err);  // the last batch's per-lane counts into stats_ (waits for them)
  uint32_t width() const { return w_; }
  uint32_t height() const { return h_; }
  uint32_t part_pixels() const { return (uint32_t)part_pix_.size(); }
  const std::vector<uint32_t>& part_list() const { return part_pix_; }
  hipStream_t stream() const { return stream_; }
  uint32_t bvh_depth() const { return depth_; }

 private:
  bool ensure_paths(uint64_t n, std::string& err);   // lane 0 holds >= n paths
  bool ensure_lane(int i, uint64_t n, std::string& err);
  void free_lane_paths(PathSet& L);
  void bind_lane(int i);  // the p_*/q_/s_* views, counts, spill and kernel stream ks_ = lane i's
  // half < 0: progressive paths k0.. over the partition; half 0/1: positions
  // k0.. of that screen half's current sample round
  bool run_batch(uint64_t k0, uint64_t n, int half, std::string& err, const uint32_t* part_pix = nullptr,
                 uint32_t part_n = 0, const Batch* map = nullptr);
  // the Batch state machine: lanes and generate; bounces until done or a
  // live-count read is pending (block: wait for it); the tail
  bool batch_begin(Batch& B, std::string& err);
  bool batch_advance(Batch& B, bool block, std::string& err);
  bool batch_tail(Batch& B, std::string& err);
  void batch_counts(const Batch& B, const uint32_t* hc);  // a finished async batch's counts into stats_
  // async lanes: issue queued batches as far as they go (block: the head to
  // its end); wait until one is issued; issue and wait for all of them
  bool pump(bool block, std::string& err);
  bool wait_issued(Batch* B, std::string& err);
  bool drain_async(std::string& err);
  bool host_wait(hipEvent_t e, std::string& err);          // pumps the async lanes while it waits
  bool host_wait_stream(hipStream_t s, std::string& err);
  hipEvent_t ev_sync_ = nullptr;
  uint64_t batch_cap() const;
  int main_lanes() const;  // lanes of main batches (below the async lanes in adaptive sessions)
  bool compute_half(int h, uint64_t n, std::string& err);
  bool merge_random_halves(uint64_t nl, uint64_t nr, bool& merged, std::string& err);
  bool plan_round(int h, std::string& err);
  bool exchange_frame(std::string& err);
  bool plan_slice(int h, uint64_t a, uint64_t b, uint64_t& local, std::string& err);
  void free_rounds();
  bool launch_extend(const float4* ro, const float4* rd, const uint32_t* cnt, std::string& err);
  bool launch_shadow(const uint32_t* cnt, uint8_t* occ_out, std::string& err);
  bool launch_trace(int b, std::string& err);
  bool size_grids(std::string& err);
  uint32_t max_grid() const;
  size_t spill_slots() const;
  uint32_t spill_grid() const;
  bool ensure_spill(int l, uint32_t grid, std::string& err);
  // one-shot grid of a slice of `paths` (fused: 2 rays per path), its spill
  // area capped at 1 GiB (beyond it the grid is clamped: partly persistent)
  uint32_t oneshot_grid(uint64_t paths) const {
    const uint64_t g = (2 * paths + 255) / 256;
    const uint64_t gmax = (1ull << 30) / (sizeof(uint2) * 256 * spill_slots());
    return (uint32_t)std::max<uint64_t>(1, std::min(g, gmax));
  }
  void free_scene();
  void free_paths();
  void free_photons();
  // Sample rounds, per screen half: as the reference's two RenderInstances
  // (wasm_interface.rs:90-94, :374-379), each half has its own strategy and
  // its own sequence of sample positions, and compute(n) advances the left
  // half's sequence by n/2 and the right half's by n - n/2. An adaptive half's
  // rounds are AdaptiveSamplingStrategy's (wpt_adaptive.h); a random half's
  // round gives each of its pixels one sample.
  bool adaptive_[2] = {false, false};
  struct HalfRounds {
    uint64_t total = 0, pos = 0;    // positions in the current round / taken
    uint32_t idx = 0;               // rounds planned since the reset
    uint32_t* rc = nullptr;         // samples per partition pixel -> (scan) offsets, [npix] = total
    uint32_t* rbase = nullptr;      // samples of the pixel before the round
    // several ranks: the round is planned over the whole frame (global
    // offsets gc, bases gbase); rc / rbase then hold this rank's slice
    uint32_t* gc = nullptr;
    uint32_t* gbase = nullptr;
  } rounds_[2];
  uint64_t round_cap_ = 0;
  uint32_t* d_scan_sums_ = nullptr;
  uint32_t* d_gsums_ = nullptr;
  float* d_mse_[2] = {nullptr, nullptr};
  uint32_t* d_bmm_ = nullptr;       // per-tile {min, max} error keys of a half
  float* h_mse_[2] = {nullptr, nullptr};  // pinned copies of the per-pixel errors (host sum)
  // the errors' sequential sum: per-chunk f64 sums / prefixes and chunk
  // effects on the device (k_sum_*), the effects' pinned copy for the walk
  double* d_s64_ = nullptr;
  ChunkEff* d_eff_ = nullptr;
  ChunkEff* h_eff_ = nullptr;
  uint32_t* d_need_ = nullptr;    // per chunk: the walk will likely re-sum it
  uint32_t* d_list_ = nullptr;    // those chunks: count, then their indices
  float* d_fb_ = nullptr;         // the elements of the first kSumFetch of them
  uint32_t* h_list_ = nullptr;
  float* h_fb_ = nullptr;
  // The sample stock of adaptive halves (wpt_stock.h, WPT_OPT_STOCK): a ring
  // of stock_slots_ samples per pixel (radiance + ray counts) and the id of
  // the refill tracing each, the frontier per pixel, the consumed rays; the
  // refills in flight (a pool; each one async batch on one stock lane, in
  // turn); the round's deficit offsets.
  uint32_t stock_slots_ = 1024;  // WPT_OPT_STOCK (power of two; 0: off): at most, see stock_alloc
  int stock_lanes_ = 2;         // WPT_OPT_STOCK_LANES: async lanes the refills rotate over
  uint32_t stock_ahead_ = 40;   // WPT_OPT_STOCK_AHEAD: a refill stocks ahead * c + extra samples per pixel
                                // (40 vs 24 at a refill every 3 rounds: C5 +2.7 %, init defaults equal,
                                // profiles/r06/ab_stock_ahead40_*.jsonl)
  uint32_t stock_extra_ = 8;    // WPT_OPT_STOCK_EXTRA
  uint32_t stock_every_ = 3;    // WPT_OPT_STOCK_EVERY: a refill after every this many rounds of a half
                                // (3 vs 2: C5 +1.3 %, init defaults +0.4 %, profiles/r06/ab_stock_every3.jsonl)
  float4* d_stock_ = nullptr;
  uint32_t* d_stock_id_ = nullptr;
  size_t stock_bytes_[2] = {0, 0};   // the two ring blocks' sizes (cached blocks may be larger)
  uint32_t* d_front_ = nullptr;
  uint32_t* d_def_ = nullptr;        // [npix + 1] deficit counts -> offsets, then [npix] bases
  uint32_t* d_bmax_ = nullptr;       // per-block maxima / ray sums scratch
  unsigned long long* d_rays_ = nullptr;  // [2] consumed rays (extension, shadow), + scratch
  uint64_t stock_cap_ = 0;           // pixels x slots the ring holds (0: not allocated)
  uint32_t stock_used_slots_ = 0;
  static constexpr int kMaxRefill = 8;
  static constexpr uint64_t kStockBytes = 48ull << 30;  // the ring's HBM at most (1080p: 1024 slots, 42 GB)
  static constexpr int kRefillChunks = 8;                 // async batches of one refill (at most)
  static constexpr uint64_t kRefillChunk = 1ull << 25;    // paths per batch
  struct Refill {
    uint32_t id = 0;
    bool live = false;
    bool counted = false;      // its batches' counts are in stats_ (stock_rays, bounces)
    uint32_t* off = nullptr;   // [n + 1] counts -> offsets over the half's list
    uint32_t* base = nullptr;  // [n] first sample per pixel
    std::deque<Batch> chunks;  // its batches (stable addresses: the queue points at them)
  };
  Refill refills_[kMaxRefill];
  hipEvent_t refill_ev_[kMaxRefill][2 * kRefillChunks] = {};
  uint32_t* h_refill_cnt_ = nullptr;  // pinned [kMaxRefill][kRefillChunks][kCountWords + 1]
  uint32_t refill_id_ = 0;            // ids of the session's refills, in issue order
  int refill_lane_ = 0;               // the stock lane of the next refill
  uint32_t round_need_[2] = {0, 0};   // per half: 1 + the refill its current round's samples wait for (0: none)
  bool stock_redo_[2] = {false, false};
  int log_ = 0;  // WPT_OPT_LOG: host steps of the adaptive rounds and async lanes to stderr (debugging)  // per half: the stock was dropped while its round was partly added
  bool stock_active(int h) const { return stock_slots_ != 0 && nranks_ == 1 && adaptive_[h]; }
  bool stock_alloc(std::string& err);
  void stock_drop();                     // forget the ring (reset, reallocation)
  bool stock_round(int h, uint64_t left, std::string& err);   // after half h's round is planned: deficit + refill
  bool stock_consume(int h, uint64_t a, uint64_t b, std::string& err);
  bool stock_flush(std::string& err);    // consumed rays into stats_, finished refills' counts
  bool refill_count(Refill& f, bool block, std::string& err);
  uint32_t refill_scale(int h, uint32_t ahead, uint64_t after) const;
  Refill* refill_slot(std::string& err);
  void refill_plan(Refill& F, int h, uint32_t ahead, uint32_t q);
  bool refill_issue(Refill& F, int h, uint64_t wt, std::string& err);
  bool stock_prefill(int h, uint64_t budget, std::string& err);  // at a compute call's start
  bool stock_prefill_ = true;  // WPT_OPT_STOCK_PREFILL
  bool pend_stock_ = false;              // the last main batch traced stock samples (its rays count when consumed)
  std::deque<Batch*> aq_[2];  // per queue: async batches not yet fully issued, in order
  // A random half's whole rounds traced beside the adaptive half's rounds
  // (WPT_OPT_FILL, compute_halves): its pixels outside the seam (the two
  // columns the other half's 5x5 error filter reads, render_target.rs:112-128)
  // run on the fill lane; the seam columns on the main lanes.
  bool fill_on_ = false;  // measured slower than tracing the random half on the main lanes with the stock on (profiles/r06)
  int async_prio_ = 0;       // WPT_OPT_ASYNC_PRIO: async batches on low-priority streams
  // the async batches (stock refills) run the fused k_trace up to 2^26 paths
  // on grids of the whole resident capacity: C5 +1.4 %, init defaults +1.9 %
  // same-session (profiles/r06/ab_async_fused_grid.jsonl)
  int async_grid_pct_ = 100;  // WPT_OPT_ASYNC_GRID_PCT: their traversal grids, % of resident capacity (0: the main batches')
  uint64_t async_fused_below_ = 1ull << 26;  // WPT_OPT_ASYNC_FUSED_BELOW: async batches below this many paths run fused (0: fused_below)
  bool async_launch_ = false;  // the launch being issued belongs to an async batch
  uint32_t* d_seam_pix_[2] = {nullptr, nullptr};
  uint32_t* d_rest_pix_[2] = {nullptr, nullptr};
  uint32_t seam_npix_[2] = {0, 0}, rest_npix_[2] = {0, 0};
  static constexpr int kMaxFill = 8;
  Batch fill_[kMaxFill];
  int nfill_ = 0;
  hipEvent_t fill_ev_[kMaxFill][2] = {};
  uint32_t* h_fill_cnt_ = nullptr;  // pinned [kMaxFill][kCountWords + 1]
  bool async_pending() const { return !aq_[0].empty() || !aq_[1].empty(); }
  int fill_lane() const { return kAsyncLane0 + stock_lanes_; }
  bool issue_fill(int h, uint64_t k0, uint64_t n, std::string& err);
  bool drain_fill(std::string& err);
  bool compute_halves(uint64_t nl, uint64_t nr, std::string& err);
  // the traversal grid of a launch: the main batches' persistent grid g (of
  // base_pct % of the resident capacity); for an async batch a share of it
  // (WPT_OPT_ASYNC_GRID_PCT), or with WPT_OPT_ASYNC_ONESHOT one block per
  // kTBlock of the most rays the launch can see (rays_per_path x the slice):
  // every wave takes at most one feed chunk, so its blocks retire as soon
  // as their rays end and free the CUs for the main lanes' next kernel
  uint32_t async_grid(uint32_t g, int base_pct, uint32_t rays_per_path = 1) const {
    if (!async_launch_) return g;
    if (async_oneshot_) return std::max<uint32_t>(1u, (uint32_t)((async_paths_ * rays_per_path + 255) / 256));
    return async_grid_pct_ > 0 ? std::max<uint32_t>(1u, (uint32_t)((uint64_t)g * async_grid_pct_ / base_pct)) : g;
  }
  bool async_oneshot_ = false;  // WPT_OPT_ASYNC_ONESHOT
  uint64_t async_paths_ = 0;    // paths of the bound async slice
  void bind_batch_lane(const Batch& B, int l);  // bind_lane(l), on the async stream for async batches
  bool time_launches_ = false;  // LAUNCH_TIMED: the main lanes' launches when profiling
  uint8_t* d_samp_ = nullptr;       // sampling visualisation RGBA8 (allocated with the viewport)
  ExchangeFn xfn_ = nullptr;
  void* xuser_ = nullptr;
  float4* xlocal_ = nullptr;
  float4* xall_ = nullptr;
  uint64_t xslot_ = 0;
  uint64_t maxpart_ = 0;             // largest partition over all ranks
  uint32_t* d_xidx_ = nullptr;       // gathered entry -> pixel (~0: padding), nranks * maxpart_
  bool photons_ok_ = false;
  uint64_t photons_shot_ = 0, photons_stored_ = 0;
  std::vector<uint32_t> oct_child_;
  std::vector<float> oct_cum_;
  uint32_t* d_oct_child_ = nullptr;
  float* d_oct_cum_ = nullptr;
  uint32_t* d_oct_corners_ = nullptr;

  int device_ = -1;
  int ncu_ = 256;
  uint2* d_spill_ = nullptr;       // traversal-stack spill (entries beyond the LDS slots)
  size_t spill_cap_ = 0;
  // persistent grids per kernel variant (tri_only + 2 count + 4 traversal):
  // [0..7] multi-lane batches (grid_pct_ of the resident capacity), [8..15]
  // one-lane batches (all of it); k_trace: tri_only + 2 count
  static constexpr int kTravVariants = 8;
  uint32_t grid_ext_[2 * kTravVariants] = {};
  uint32_t grid_sh_[2 * kTravVariants] = {};
  uint32_t grid_tr_[4] = {};
  uint32_t grid_shade_ = 512;      // k_shade blocks (kShadeBlock lanes each) resident on the chip (the least occupied variant)
  uint32_t shade_occ_[16] = {};  // per k_shade variant (x ray counting): resident blocks per CU (0: not yet queried)
  size_t shade_occ_smem_[16] = {};  // ... for this dynamic LDS size
  bool fused_ = false;             // WPT_OPT_FUSED: bounce b's extension + bounce b-1's shadow rays in one k_trace for every batch
  // batches below this many paths (adaptive sample rounds) always run fused:
  // one launch per bounce drains one pool of rays instead of two (WPT_OPT_FUSED_BELOW)
  uint64_t fused_below_ = 1ull << 24;
  int small_lanes_ = 2;           // WPT_OPT_SMALL_LANES: lane cap for batches below fused_below_ (C5 +3-4 %, init defaults +1 % vs 3)
  int traversal_ = 3, traversal_sh_ = 3;  // WPT_OPT_TRAVERSAL(_SH): 0 exact BVH2, 1 BVH4 fast path, 3 auto (per scene)
  int trav_ext_ = 0, trav_sh_ = 0;        // what the uploaded scene runs (0 the exact BVH2, 1 the BVH4 fast path)
  bool treelet_ = true;            // WPT_OPT_TREELET: LDS treelet of the BVH2's top node pairs
  // WPT_OPT_PIXEL_TILE: whole-round batches in tiles of this many px (0: raster);
  // 4 x 4 vs 8 x 8 is within noise (profiles/r06/ab_pixel_tile.jsonl)
  uint32_t pixel_tile_ = 8;
  int grid_pct_ = 50;              // WPT_OPT_GRID_PCT: persistent traversal grids of multi-lane batches, % of resident capacity
#ifndef WPT_TRACE_GRID_PCT
#define WPT_TRACE_GRID_PCT 75  // C5 +0.6 % over 100 (profiles/r05/ab_trace_grid75.jsonl)
#endif
  int trace_grid_pct_ = WPT_TRACE_GRID_PCT;  // WPT_OPT_TRACE_GRID_PCT: the same for the fused k_trace (small batches)
  uint32_t refill_ = 12, refill_sh_ = 16;  // WPT_OPT_REFILL(_SH): idle lanes before a wave refills
  uint64_t finish_below_ = 1u << 18;  // WPT_OPT_FINISH_BELOW: RR-only batches hand their last paths to k_finish (0: never)
  int finish_every_ = 4;           // WPT_OPT_FINISH_EVERY: bounces between the RR-only batches' live-count reads
  int batch_lanes_ = 1;            // lanes of the batch being launched (1: full-capacity traversal grids)
  // WPT_OPT_PROBE: wave timelines of the next probe_cap_ traversal launches
  // (probe_read); meta per launch {kernel, lane, bounce, waves, first entry}
  uint32_t probe_cap_ = 0, probe_waves_ = 0, probe_used_ = 0;
  uint4* d_probe_ = nullptr;
  std::vector<uint32_t> probe_meta_;
  int cur_bounce_ = 0;
  uint4* probe_slot(int kernel, uint32_t grid);
  uint32_t* d_fallback_ = nullptr; // [2] rays re-traced exactly (extend, shadow)
  hipStream_t stream_ = nullptr;
  hipStream_t ks_ = nullptr;       // stream of the bound lane (kernel launches of a batch)
  PathSet lanes_[kMaxLanes];
  int lanes_made_ = 0;
  bool stats_pending_ = false;     // the last batch's counts not yet read (flush_counts)
  int pend_nl_ = 0, pend_b_ = 0;
  int nlanes_ = 4;                 // wpt_set_lanes (1..kMaxLanes); 4 with half-GPU traversal grids (C3 +4.5 % over 3 lanes at full grids)
  int bound_ = 0;
  hipEvent_t ev_main_ = nullptr;   // lanes > 0 wait for the main stream's prior work
  hipEvent_t ev_ref_ = nullptr;    // profiling: time origin of a batch's launch intervals
  std::vector<void*> scene_bufs_;
  DevScene ds_{};
  uint32_t depth_ = 0;
  bool scene_ok_ = false;

  uint32_t w_ = 0, h_ = 0;
  float cam_[5] = {0, 0, 0, 0, 0};
  int left_type_ = 1, right_type_ = 1, debug_ = 0;
  int max_depth_ = 0;
  uint32_t seed_ = 0xBABABEBEu;
  uint64_t batch_ = 1ull << 27;  // 134M paths (~19 GB of path state): per-bounce tails amortised

  uint32_t rank_ = 0, nranks_ = 1, tile_ = 16;
  std::vector<uint32_t> part_pix_;
  uint32_t* d_part_pix_ = nullptr;
  uint32_t* d_half_pix_[2] = {nullptr, nullptr};  // one rank: each screen half's pixels, tile order
  uint32_t* d_frame_pix_ = nullptr;                // one rank: the frame's pixels, tile order
  uint32_t half_npix_[2] = {0, 0};
  uint64_t next_path_ = 0;

  float4* d_acc_ = nullptr;
  uint32_t* d_cnt_ = nullptr;
  uint8_t* d_rgba_ = nullptr;

  // streams of the bound lane (views into lanes_[bound_]; cap_ = that lane's
  // capacity)
  uint64_t cap_ = 0;
  uint32_t* p_pixel_ = nullptr;
  float4* p_col_ = nullptr;
  float4* p_ro_[2] = {nullptr, nullptr};
  float4* p_rd_[2] = {nullptr, nullptr};
  float4* p_thr_[2] = {nullptr, nullptr};
  float* p_t_ = nullptr;
  int32_t* p_id_ = nullptr;
  float4* s_o_ = nullptr;
  float4* s_d_ = nullptr;
  float4* s_c_ = nullptr;
  uint32_t* d_counts_ = nullptr;   // kCountWords (PathSet::counts)
  unsigned long long* d_work_ = nullptr;  // [kWorkCopies][kWorkWords] extend visits/tests/node bytes, shadow visits/tests/node bytes, ...
  uint32_t* h_counts_ = nullptr;   // pinned mirror
  uint32_t* h_word_ = nullptr;     // pinned scratch of the round planning (a round's path count)
  // count words of the bound lane: rays of bounce b, shadow rays of bounce b,
  // k_shade's append counter of bounce b
  uint32_t* ext_count(int b) const { return b == 0 ? d_counts_ : d_counts_ + 2 + 2 * (b - 1); }
  uint32_t* sh_count(int b) const { return d_counts_ + 3 + 2 * b; }
  unsigned long long* append_ctr(int b) const { return reinterpret_cast<unsigned long long*>(d_counts_ + 2 + 2 * b); }

  bool counting_ = false;
  bool profiling_ = false;
  Stats stats_;
  KernelTimes times_;
  struct PendingTiming {
    hipEvent_t a, b;
    int slot;
  };
  bool next_event(hipEvent_t* e, std::string& err);
  bool resolve_timings(std::string& err);
  std::vector<hipEvent_t> ev_pool_;
  size_t ev_used_ = 0;
  std::vector<PendingTiming> pending_;
};

}  // namespace wpt
