// ctx_internal.h — the fr_ctx context (device memory, streams, frame slots) shared by the C ABI in
// context.cpp and the multi-GPU group in group.cpp. Not part of the public interface (include/fovrt.h).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/fovrt.h"
#include "fr_device.h"
#include "scene.h"

#define FR_MAX_SHARD_RANKS 64  // ranks per view (an owner is one byte of the tile map)

namespace fr {
void launch_gbuffer(const DevScene&, const FrameUniforms&, f4*, f4*, f4*, f4*, f4*, uint8_t*, DevStats*, hipStream_t);
void launch_shade_paths(const DevScene&, const FrameUniforms&, const uint32_t*, const uint32_t*, uint32_t, const f4*,
                        const f4*, uint32_t*, f4*, unsigned long long*, DevStats*, f4*, uint32_t*, uint32_t, uint32_t,
                        uint32_t, f4*, hipStream_t);
size_t shade_item_store_f4();
void launch_sample_setup(const FrameUniforms&, const uint32_t*, const uint32_t*, uint32_t, const f4*, const f4*,
                         const unsigned long long*, f4*, uint32_t*, hipStream_t);
void launch_shade_resolve(const FrameUniforms&, const uint32_t*, const uint32_t*, uint32_t, const f4*, const f4*,
                          const f4*, unsigned long long*, f4*, f4*, uint32_t*, uint32_t, f4*, hipStream_t);
size_t shade_counter_words();
size_t shade_fx_slots(uint32_t max_active, int spp, uint32_t handoff);
void launch_carry_history(const FrameUniforms&, const uint8_t*, const f4*, const f4*, f4*, f4*, unsigned long long*,
                          hipStream_t);
void launch_sampling(const FrameUniforms&, const DevScene&, const f4*, const f4*, const f4*, f4*, const f4*,
                     const f4*, f4*, uint8_t*, const uint8_t*, unsigned long long*, uint32_t*, int, uint8_t*, uint32_t*,
                     bool, uint32_t*, hipStream_t);
size_t logpolar_inv_words(int W, int H);
void launch_owner_counts(const FrameUniforms&, const uint32_t*, uint32_t*, hipStream_t);
void launch_mask_words(const uint8_t*, const uint8_t*, int, int, unsigned long long*, uint32_t*, hipStream_t);
void launch_compaction(int, int, const unsigned long long*, const uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                       uint32_t*, hipStream_t);
size_t compaction_tiles(int W, int H);
void launch_shard_pack(const FrameUniforms&, const f4*, f4*, hipStream_t);
void launch_logpolar(const f4*, f4*, f4*, int, int, f2, hipStream_t);
void launch_composite(const f4*, int, int, int, f4*, hipStream_t);
void launch_shard_unpack(const FrameUniforms&, int, const f4*, f4*, hipStream_t);
void launch_shard_pack_active(const uint32_t*, const uint32_t*, uint32_t, const f4*, f4*, uint32_t*, hipStream_t);
// the history validity rings of a still-camera group (k_trace.hip): FR_VRING pixels inside each tile
void launch_vring_pack(const f4*, int, int, int, const int32_t*, int, uint32_t*, hipStream_t);
void launch_vring_unpack(const uint32_t*, int, int, int, const int32_t*, int, f4*, hipStream_t);
void launch_shard_unpack_active(const FrameUniforms&, const f4*, const uint32_t*, uint32_t, uint32_t, const f4*, const f4*, f4*,
                                f4*, hipStream_t);
const u2* launch_jfa(const f4*, u2*, u2*, f4*, f4*, const float*, int, int, f4*, f4*, bool, hipStream_t);
void launch_jfa_coord(const u2*, const f4*, f4*, int, int, hipStream_t);
void launch_sibson(const f4*, const f4*, f4*, int, int, hipStream_t);
void launch_sibson_runs(const f4*, const u2*, const f4*, f4*, f4*, f4*, uint32_t*, uint32_t*, f4*, int, int, bool, bool,
                        bool, hipStream_t);
int sibson_prefix_blocks(int W);
size_t sibson_strip_words(int W, int H);
size_t sibson_rowp_texels(int W, int H);
struct BvhWork;
bool gpu_build_bvh(BvhWork**, const f3*, int, BvhNode*, TriGeo*, int32_t*, int*, int*, int*, hipStream_t, std::string&);
void bvh_work_free(BvhWork*);
bool bvh_work_prepare(BvhWork**, int, hipStream_t, std::string&);
bool bvh_builder_warm(BvhWork*, hipStream_t, std::string&);
#ifdef FR_STAMPS
void launch_trace_queries(const DevScene&, const f4*, uint32_t, f4*, uint32_t*, hipStream_t, int);
void diag_record_queries(f4*, uint32_t, hipStream_t);
uint32_t diag_recorded_queries(hipStream_t);
void diag_sample_trace(uint32_t*, uint32_t, uint32_t*, uint32_t, hipStream_t);
#endif
void launch_pullpush(const f4*, f4*, f4*, f4*, f4*, int, int, hipStream_t);
void launch_atrous(const f4*, const f4*, const f4*, f4*, int, int, float, float, float, float, hipStream_t);
int pp_size(int W, int H);
size_t pp_snap_count(int S);
}  // namespace fr

using fr::f2;
using fr::f3;
using fr::u2;
using fr::f4;
using fr::BvhNode;
using fr::TriGeo;
using fr::TriShade;
using fr::DevMaterial;
using fr::DevTexture;
using fr::DevScene;
using fr::DevStats;
using fr::FrameUniforms;
using fr::HostScene;
using fr::Bvh;


enum Phys {
  P_POSITION, P_NORMAL, P_DEPTH_A, P_DEPTH_B, P_DIFFUSE, P_WEIGHT, P_HIST_A, P_HIST_B, P_SHADING, P_EXTRA,
  P_JFA_COORD, P_JFA_COLOR, P_SIBSON, P_PULLPUSH, P_ATROUS_A, P_ATROUS_B, P_LOGPOLAR, P_LOGPOLAR_INV,
  // frame-slot copies of the buffers the reconstruction reads (POSITION, NORMAL, SHADING) and of
  // WEIGHT (read by the trace half's tail); slot 0 is the plain entry above
  P_POSITION_B, P_NORMAL_B, P_SHADING_B, P_WEIGHT_B,
  P_POSITION_C, P_NORMAL_C, P_SHADING_C, P_WEIGHT_C,
  P_COUNT
};

struct fr_ctx {
  fr_config cfg;
  std::string asset_dir;
  std::string err;
  int W = 0, H = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // reconstruction chain 2: pull-push -> A-Trous
  hipStream_t stream3 = nullptr;  // reconstruction chain 1: JFA -> Sibson
  hipStream_t stream4 = nullptr;  // entry 3's carry of the inactive pixels, beside the megakernel
  hipStream_t stream5 = nullptr;  // front stages of a pipelined frame (entries 0-2), beside the previous megakernel
  // Invariant for stream5: its front stages wait only for the slot events (ev_recon, ev_trace), not for
  // earlier work on `stream`, although they overwrite shared buffers (gclass, DIFFUSE, EXTRA, depth,
  // ballots, counts, lp_cache). So every ABI call that enqueues on `stream` outside a pipelined frame
  // goes through join_recon, which sets stream_dirty, and the next pipelined frame's front stages then
  // wait for `stream` once (frame_half).
  bool stream_dirty = true;
  // Frame pipelining: frame N's reconstruction (stream3 + stream2) runs while later frames trace.
  // The buffers the reconstruction reads (POSITION, NORMAL, SHADING) rotate over `nslots` frame
  // slots (`slot` = the current frame's); a frame's front stages wait for the reconstruction that
  // last read their slot (ev_recon). The front stages of a pipelined frame (G-buffer, sampling,
  // compaction) run on stream5 while the previous frame's megakernel still runs on `stream`: they
  // read nothing entry 3 writes. What entry 3's tail reads of them (WEIGHT, mask, active list, ray
  // count) rotates with the slot as well; the front of a frame waits for the trace half that last
  // read its slot (ev_trace), and entry 3 of a frame waits for its own front (ev_front).
  static constexpr int MAX_SLOTS = 3;
  int nslots = 3;
  int slot = 0;
  bool recon_pending[MAX_SLOTS] = {};
  bool front_pending = false;
  bool trace_pending[MAX_SLOTS] = {};
  hipEvent_t ev_front = nullptr, ev_trace[MAX_SLOTS] = {}, ev_recon[MAX_SLOTS] = {};
  // latency mode: the end of the slot's JumpFlooding (or of its trace half when the chain is not run here)
  hipEvent_t ev_jfa[MAX_SLOTS] = {};
  bool jfa_pending[MAX_SLOTS] = {};
  // latency mode's schedule: per slot, timing events at the front stages' start and end, the JumpFlooding's
  // end and the reconstruction's end; the last completed frame's front and Sibson (JFA end -> end) times
  hipEvent_t lat_ev[MAX_SLOTS][4] = {};
  bool lat_rec[MAX_SLOTS] = {}, lat_arm = false;
  float lat_front_ms = 0.0f, lat_sib_ms = 0.0f;
  float lat_front_hist[8] = {};  // the last frames' front-stage spans: their minimum is the uncontended one
  int lat_front_n = 0;
  // Tile sharding (fr_set_shard_plan): tile -> (owner << 24 | index among the owner's tiles) on the
  // device (FrameUniforms::shard_map), and the owners on the host. With sharding on, the front stages
  // also count every rank's active pixels from the unfolded mask (bcount per 16x16 block ->
  // owner_counts_p[slot]) and copy them to pinned host memory (h_counts, ev_counts[slot]): a group
  // sizes its transfers from them without a collective (every rank computes the same full mask).
  uint32_t* shard_map = nullptr;
  f4* shade_radiance = nullptr;    // a sharded rank's traced pixels' (tone-mapped radiance, 1), active order
  std::vector<uint8_t> shard_owner;
  uint32_t* bcount = nullptr;
  uint32_t* owner_counts_p[MAX_SLOTS] = {};
  uint32_t* h_counts = nullptr;  // MAX_SLOTS x FR_MAX_SHARD_RANKS, pinned
  hipEvent_t ev_counts[MAX_SLOTS] = {};
  bool counts_valid[MAX_SLOTS] = {};  // a front stage under the current plan recorded ev_counts[slot]
  // Tile-local front stages (fr_set_front_local): per 8x8 pixel tile, does this rank's sampling read
  // it (front_need, device; FrameUniforms::front_need while on); front_need_px = their pixel count.
  bool front_local = false;
  uint8_t* front_need = nullptr;
  std::vector<uint8_t> front_need_h;
  uint32_t front_need_px = 0;
  int pipeline_mode = 0;            // FR_PIPELINE_THROUGHPUT / FR_PIPELINE_LATENCY (fr_set_pipeline_mode)
  int recon_chains = 3;             // reconstruction chains this context runs: 1 JFA -> Sibson, 2 pull-push -> A-Trous
  hipEvent_t recon_gate = nullptr;  // when set, chain 2 (pull-push -> A-Trous) waits for it (a group's
                                    // composite reads the last A-Trous image)
  uint8_t* mask_p[MAX_SLOTS] = {};
  uint32_t* active_p[MAX_SLOTS] = {};
  uint32_t* ray_count_p[MAX_SLOTS] = {};
  HostScene scene;
  Bvh bvh;
  // device scene
  BvhNode* d_nodes = nullptr;
  f3* d_pos = nullptr;  // world-space vertices, 3 per triangle (the GPU builder's input)
  TriGeo* d_tri = nullptr;
  int32_t* d_prim = nullptr;
  // the GPU builder's target arrays (swapped with the current tree after a successful build) and its scratch
  BvhNode* spare_nodes = nullptr;
  TriGeo* spare_tri = nullptr;
  int32_t* spare_prim = nullptr;
  fr::BvhWork* bvh_work = nullptr;
  bool tree_full_cap = false;  // d_nodes / d_tri / d_prim hold one entry per triangle (a device-built tree)
  TriShade* d_shade = nullptr;
  std::vector<void*> d_tex;
  bool tex_packing = true;  // textures in their densest exact storage (pack_texture); FOVRT_TEX_PACKING=0: RGBA32F
  bool sib_strip = true;    // Sibson's big discs by k_sibson_strip (default; FOVRT_SIB_STRIP=0: k_sibson_wide)
  DevMaterial* d_mats = nullptr;
  DevTexture* d_texs = nullptr;
  DevScene dsc;
  // image buffers
  f4* img[P_COUNT] = {};
  int depth_cur = P_DEPTH_A, depth_cache = P_DEPTH_B;
  int hist_cur = P_HIST_A, hist_cache = P_HIST_B;
  int atrous_out = P_ATROUS_A;
  uint8_t* mask = nullptr;  // mask_p[slot]
  uint8_t* gclass = nullptr;
  uint8_t* lp_cache = nullptr;  // log-polar mask for (lp_gaze, lp_mode); recomputed when either changes
  uint32_t* lp_inv = nullptr;   // the inverse log-polar map of every (u, v) of that gaze (k_logpolar_inv)
  f2 lp_gaze{-1e30f, -1e30f};
  int lp_mode = -1;
  unsigned long long* words = nullptr;
  uint32_t* counts = nullptr;
  uint32_t* offsets = nullptr;  // per (class, block) local prefix
  uint32_t* tiles = nullptr;
  uint32_t* ray_count = nullptr;  // ray_count_p[slot]
  uint32_t* active = nullptr;     // active_p[slot]
  uint32_t* shade_ctr = nullptr;  // sharded chunk counters of the shading work queue
  f4* samples = nullptr;          // one radiance value per (active pixel, camera sample): 16 B, or 32 B fixed point
  unsigned long long* sample_help = nullptr;  // fixed-point shares of the lanes that took over items, 32 B per sample
  f4* item_store = nullptr;     // the megakernel's refraction item stacks (shade_item_store_f4)
  f4* aux = nullptr;              // per active pixel: NDC position, r1, r2 (k_sample_setup): aux_p[aux_i]
  uint32_t* aux_seed = nullptr;   // per active pixel: the seed after the two draws: aux_seed_p[aux_i]
  // Early sample setup (frame_half, latency mode): a frame's k_sample_setup runs on the front stream right after its
  // compaction, into the other of two aux buffers, from the history validity bits (hvalid, one per pixel) the previous
  // frame's k_carry_history computed. hvalid_fresh: those bits describe HISTORY_CACHE as the next frame will read it
  // (cleared by anything else that writes the history).
  f4* aux_p[2] = {};
  uint32_t* aux_seed_p[2] = {};
  int aux_i = 0;
  unsigned long long* hvalid = nullptr;
  bool hvalid_fresh = false;
  bool setup_early = false;  // this frame's setup was enqueued by its front stages
  bool early_setup = true;   // FOVRT_EARLY_SETUP=0: every setup on the context stream before its megakernel
  u2 *jfa_a = nullptr, *jfa_b = nullptr;  // JFA state ping-pong (seed coord texel + alpha flags)
  uint32_t chunk_refr = 0;  // fixed refraction-class chunk of the megakernel (FOVRT_SHADE_CHUNK_REFR), 0 adaptive
  uint32_t xcd_bands = 1;   // megakernel queue: per-XCD class bands (FOVRT_SHADE_XCD_BANDS=0: interleaved chunks)
  uint32_t handoff = 1;     // megakernel tail handoff (FOVRT_SHADE_HANDOFF): 0 never, 1 small launches, 2 always
  float* ftab = nullptr;  // texel-centre coordinates ((x + 0.5) / W, x < W; then (y + 0.5) / H)
  f4 *pull = nullptr, *push = nullptr, *snap = nullptr;
  f4 *sib_prefix = nullptr, *sib_blocks = nullptr;  // Sibson run form: per-row block prefix sums + block totals
  uint32_t* sib_wide = nullptr;  // Sibson run form: wide-disc pixel lists (two counts, then W*H indices)
  uint32_t* sib_strips = nullptr;  // Sibson run form: k_sibson_strip's strip list and flags (sibson_strip_words)
  f4* sib_rowp = nullptr;          // Sibson strip kernel: whole-row prefix sums (sibson_rowp_texels)
  bool sib_prefix_fresh = false;  // the last JFA wrote them with JFA_COLOR (cleared when JFA_COLOR / JFA_COORD are
                                  // written or handed out, fr_get_buffer)
  const u2* jfa_final = nullptr;  // that JFA's final state (the seeds k_sibson_runs reads while the prefix is fresh)
  // JumpFlooding leaves JFA_COORD unwritten (the run form reads the seeds from jfa_final): while jfa_coord_owed,
  // materialize_jfa writes it (k_jfa_coord, from jfa_final and JFA_COLOR) before anything reads it or writes JFA_COLOR.
  bool jfa_coord_owed = false;
  bool lazy_jfa_outputs = true;  // FOVRT_JFA_LAZY_OUTPUTS=0: every JumpFlooding writes JFA_COORD
  int pp_S = 0;
  DevStats* stats = nullptr;
  FrameUniforms U;
  uint32_t accum = 0;
  bool light_pending = false;
  bool compacted = false;
  bool mask_dirty = false;
  hipEvent_t ev[24] = {};  // 0-15 stage timing; 16 fork; 17 chain-2 join; 20-22 chain-1 timing
  bool time_kernels = false;  // fr_frame with timing: also time the path-trace kernel alone
  // Live timing of entry 3 inside pipelined (untimed) frames: a ring of event quadruples recorded on
  // the context stream around carry_history / k_shade_paths / resolve (fr_kernel_timing); a slot is
  // harvested (its elapsed times summed) before it is reused and by fr_kernel_times.
  static constexpr int KT_RING = 32;
  hipEvent_t kt_ev[KT_RING][4] = {};
  bool kt_on = false;
  int kt_next = 0, kt_pending = 0;
  uint32_t kt_frames = 0;
  double kt_stage_ms = 0.0, kt_kernel_ms = 0.0;
  // Frame clock of pipelined frames (fr_frame_clock): per frame, an event where its G-buffer may start
  // (on the front stream, after the slot waits) and one after both reconstruction chains (stream3).
  // latency = start -> end of one frame (gaze sample to finished image on the GPU), interval = end of
  // the previous frame -> end of this one. Harvested like kt_ev.
  static constexpr int FC_RING = 16;
  hipEvent_t fc_ev[FC_RING][2] = {};
  bool fc_on = false;
  int fc_next = 0, fc_pending = 0;
  hipEvent_t fc_ref = nullptr;  // recorded when the clock is enabled: every time is read against it
  double fc_prev_end = -1.0;    // the previous harvested frame's end (ms after fc_ref)
  int fc_cur = -1;              // the ring entry of the frame being enqueued
  bool fc_arm = false;          // frame_half: this enqueue_geometry starts a whole frame
  std::vector<float> fc_latency, fc_interval;
  // scene export copies
  std::vector<const float*> tex_ptrs;
  std::vector<int32_t> tex_dims, mat_pairs;
};


// Internal helpers of context.cpp used by group.cpp (same semantics as the ABI calls they back).
namespace fri {
int fail(fr_ctx* c, int code, const std::string& msg);
int check_launch(fr_ctx* c);
void join_recon(fr_ctx* c);
// one frame half on the context; trace / recon as fr_trace_frame / fr_reconstruct_frame (recon runs the
// chains in c->recon_chains)
int frame_half(fr_ctx* c, fr_frame_timing* t, bool trace, bool recon);
int P_shd(const fr_ctx* c);
int P_wgt(const fr_ctx* c);
}  // namespace fri
