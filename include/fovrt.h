/* fovrt.h — C ABI of the MI355X-native foveated path-tracing + reconstruction engine.
 *
 * Drop-in boundary for the reference's hot path (ohseokkwon/Foveated-Rendering-using-Ray-Tracing).
 * Every entry point replaces one call of the reference's frame loop (FR/main.cpp:253-358); the
 * reference interface each one replaces is cited next to it ("FR/" = "Foveated Rendering using
 * Ray Tracing/"). Conventions:
 *   - every function returns FR_OK (0) or a negative fr_status; no exceptions cross the ABI;
 *   - fr_last_error(ctx) (or fr_last_error(NULL) after a failed fr_create) describes the failure;
 *   - the context owns all device memory (allocated in fr_create, freed in fr_destroy); per-frame
 *     calls never allocate; views returned by fr_get_buffer are borrowed and stay valid until the
 *     next call that writes that buffer, or fr_destroy;
 *   - one context per device, one host thread per context (calls are serialised, not re-entrant);
 *   - image buffers are row-major W x H with row 0 = bottom row (the OptiX launch index y and the
 *     GL texture t of the reference agree on this), RGBA32F unless the view says otherwise.
 */
#ifndef FOVRT_H
#define FOVRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: fr_config.abi_version; fr_set_gaze takes the cursor (cursorPosCallback) and fr_reset_gaze; the
 *    sparse shard calls take the slab size; fr_set_shard_plan / fr_shard_plan; the fr_group_* calls. */
#define FOVRT_ABI_VERSION 2

typedef enum fr_status {
  FR_OK = 0,
  FR_E_INVALID = -1,     /* bad argument / unknown buffer id */
  FR_E_HIP = -2,         /* HIP runtime error (no device, launch failure) */
  FR_E_NOMEM = -3,       /* device allocation failed */
  FR_E_IO = -4,          /* asset file missing or malformed */
  FR_E_STATE = -5,       /* call out of order (e.g. shading before sampling) */
  FR_E_UNSUPPORTED = -6  /* configuration outside what the engine implements */
} fr_status;

typedef enum fr_scene_preset {
  FR_SCENE_BOX = 0,      /* ground + refractive box               (configs[0]) */
  FR_SCENE_BUNNY = 1,    /* ground + box + bunny + reflective earth (configs[1], configs[2]) */
  FR_SCENE_VOKSELIA = 2  /* all five models of FR/PathTracer.cpp:582-595 */
} fr_scene_preset;

typedef enum fr_mask_mode {
  FR_MASK_SALIENCY = 0,   /* masked_sampling (FR/cuda/samplingStep.cu:222), the reference default */
  FR_MASK_LOGPOLAR = 1,   /* log-polar round trip (FR/cuda/samplingStep.cu:180-182) */
  FR_MASK_UNIFORM2X2 = 2, /* x%2==0 && y%2==0 (FR/PathTracer.cpp:526-533), non-foveated */
  FR_MASK_ALL = 3,        /* every pixel traced */
  FR_MASK_LOGPOLAR_SIGNED = 4 /* log-polar round trip with signed pixel differences: the 10% foveal
                               * density BASELINE.json quotes (the literal uint2 arithmetic of
                               * samplingStep.cu:182 wraps negative differences, halving it) */
} fr_mask_mode;

typedef struct fr_config {
  int abi_version;            /* FOVRT_ABI_VERSION (fr_config_default sets it; fr_create rejects others) */
  int width, height;          /* FR/main.cpp:127-135 (argv W H), default 1024 x 1024 */
  int scene;                  /* fr_scene_preset */
  int mask_mode;              /* fr_mask_mode */
  int spp;                    /* 1, 2, 4 or 8 (reference: 1, FR/cuda/fov_path_trace_camera.cu:117) */
  int diffuse_max_depth;      /* g_diffuse_max_depth (FR/gui.cpp:26), default 1 */
  int refraction_max_depth;   /* min(refraction_maxdepth, max_depth) = 100 in the reference; default 16 */
  float light_power;          /* g_light_Power (FR/gui.cpp:21), default 810 */
  int optimize;               /* g_isOptimize (FR/gui.cpp:16): run the compaction (entry 2) */
  int atrous_iterations;      /* ATrous::render count (FR/main.cpp:355), default 1 */
  int write_extra;            /* write the saliency heat-map buffer (extra_buffer) */
  int device;                 /* HIP device ordinal */
  int texture_mode;           /* 0: reference assets from asset_dir (error if missing); 1: procedural */
  int detail;                 /* procedural mesh detail (0 = preset default) */
  int mesh_mode;              /* 0: the reference's .obj meshes where present under asset_dir, procedural
                               * stand-ins otherwise; 1: procedural only; 2: .obj required (FR_E_IO) */
  int bvh_builder;            /* 0: host binned SAH (default); 1: GPU LBVH (k_bvh.hip), the builder of
                               * fr_rebuild_bvh / fr_set_positions; both give identical frames */
  int sibson_mode;            /* 0 (default): run form, each row of a pixel's disc summed from per-row prefix
                               * sums (same taps as sibsonFS.glsl:30-44, rounding-level differences, ~1e-6);
                               * 1: per tap in the shader's order (bit-exact against the oracle) */
  const char* asset_dir;      /* directory holding CedarCity.hdr, grid.ppm, bunny/bunny.PPM, ... */
} fr_config;

/* Per-frame camera uniforms (PathTracer::update_optix_variables, FR/PathTracer.cpp:774-820).
 * Matrices are row-major "math" matrices: v' = M v. */
typedef struct fr_camera {
  float eye[3];
  float prev_eye[3];
  float inv_vp[16];   /* device "mvp"      = inverse(P * V)           (:786-787) */
  float prev_vp[16];  /* device "prev_mvp" = P * V of the previous frame (:789-790) */
  float up[3];
  float target[3];
  float gaze[2];      /* (g_gaze.x, H - g_gaze.y) */
} fr_camera;

/* glm-style camera pose (FR/Camera.cpp): position, unit quaternion (w, x, y, z), perspective. */
typedef struct fr_camera_pose {
  float pos[3];
  float rot[4];       /* glm::quat (w, x, y, z) */
  float fovy_deg;     /* 45 (FR/main.cpp:207) */
  float znear, zfar;  /* 0.1, 500.1 */
  float aspect;       /* viewport w / h */
} fr_camera_pose;

typedef enum fr_buffer_id {
  /* PathTracer::TextureName order (FR/PathTracer.h:13-31) */
  FR_BUF_POSITION = 0,
  FR_BUF_NORMAL = 1,
  FR_BUF_DEPTH = 2,
  FR_BUF_DIFFUSE = 3,
  FR_BUF_WEIGHT = 4,
  FR_BUF_THREAD = 5,        /* compacted active-pixel list (u32 pixel index, ray_count entries) */
  FR_BUF_HISTORY = 6,
  FR_BUF_SHADING = 7,
  FR_BUF_EXTRA = 8,
  /* reconstruction outputs (JumpFlooding / Sibson / PullPush / ATrous GL textures) */
  FR_BUF_JFA_COORD = 9,
  FR_BUF_JFA_COLOR = 10,
  FR_BUF_SIBSON = 11,
  FR_BUF_PULLPUSH = 12,
  FR_BUF_ATROUS = 13,
  /* temporal state (OptiX ping-pong partners) */
  FR_BUF_DEPTH_CACHE = 14,
  FR_BUF_HISTORY_CACHE = 15,
  FR_BUF_MASK = 16,         /* u8 usingRay per pixel */
  FR_BUF_LOGPOLAR = 17,     /* LogPolarTransform::logPolarTex  (forward image, W/4 x H/4 used) */
  FR_BUF_LOGPOLAR_INVERSE = 18, /* LogPolarTransform::ilogPolarTex */
  FR_BUF_GCLASS = 19,       /* u8 primary-hit class of the last G-buffer: 0 refraction, 1 reflection, 2 diffuse,
                             * 3 miss (the megakernel's class-major work order; diagnostics) */
  FR_BUF_COUNT = 20
} fr_buffer_id;

typedef enum fr_format { FR_FMT_RGBA32F = 0, FR_FMT_U32 = 1, FR_FMT_U8 = 2 } fr_format;

typedef struct fr_buffer_view {
  void* device_ptr;
  int width, height;   /* elements; THREAD: width = capacity, height = 1 */
  size_t pitch_bytes;  /* bytes per row */
  size_t bytes;        /* total bytes */
  int format;          /* fr_format */
} fr_buffer_view;

typedef struct fr_stats {
  uint64_t gbuffer_primary;   /* entry-0 camera rays */
  uint64_t primary;           /* entry-3 camera rays (ray_count * spp) */
  uint64_t shadow;            /* shadow rays (light samples) */
  uint64_t diffuse_bounce;    /* diffuse GI bounces */
  uint64_t mirror;            /* reflection-material mirror rays */
  uint64_t refraction;        /* refraction-material transmitted rays */
  uint64_t reflection;        /* refraction-material reflected rays */
  uint64_t truncated;         /* refraction nodes cut by refraction_max_depth */
  uint64_t overflow;          /* work items dropped (explicit stack full) */
  uint64_t segments;          /* sum of all traced ray segments */
  uint64_t diag[6];           /* diagnostic build (-DFR_STAMPS) only, else 0: megakernel cycle stamps
                                 [total, refill, shade, traversal], node visits, wave traversal steps */
} fr_stats;

typedef struct fr_frame_timing {
  /* stage names of PrintMSTimes (FR/main.cpp:260-358); milliseconds measured with HIP events */
  float geometry_ms, sampling_ms, optimize_ms, shading_ms;
  float jfa_ms, sibson_ms, pullpush_ms, atrous_ms;
  float total_ms;
  uint32_t ray_count;
  float shade_paths_ms; /* the path-trace megakernel alone (inside shading_ms) */
} fr_frame_timing;

typedef struct fr_ctx fr_ctx;

int fr_config_default(fr_config* cfg);
const char* fr_version(void);
int fr_abi_version(void);  /* FOVRT_ABI_VERSION of the library */

/* PathTracer::initialize(w, h) (FR/PathTracer.cpp:41-78) + the renderer constructors
 * (FR/main.cpp:152-159). */
int fr_create(const fr_config* cfg, fr_ctx** out);
int fr_destroy(fr_ctx* ctx);
const char* fr_last_error(fr_ctx* ctx);

/* Camera (FR/Camera.cpp): glm-compatible helpers. */
int fr_camera_look_at(fr_camera_pose* pose, const float target[3], const float up[3]);  /* :73-83 */
int fr_camera_matrices(const fr_camera_pose* pose, float view[16], float proj[16]);      /* :139-181, row-major */
int fr_camera_uniforms(const fr_camera_pose* cur, const fr_camera_pose* prev, int width, int height,
                       fr_camera* out);  /* update_optix_variables' host math, gaze = screen centre */
int fr_preset_camera(int scene, float eye[3], float target[3]);  /* FR/main.cpp:189-209 */

/* PathTracer::init_camera / update_optix_variables (FR/PathTracer.cpp:606-632, 774-820) */
int fr_set_camera(fr_ctx* ctx, const fr_camera* cam);
int fr_set_light_power(fr_ctx* ctx, float power);          /* g_light_changed path, :103-116 */
int fr_set_diffuse_max_depth(fr_ctx* ctx, int depth);      /* :800-806 */
int fr_reset_accumulation(fr_ctx* ctx);                    /* tracer->m_accumFrame = 0 (FR/main.cpp:248) */
int fr_accum_frame(fr_ctx* ctx, uint32_t* frame);          /* public m_accumFrame */

/* The four OptiX launches (FR/PathTracer.cpp:85-230). Synchronous; *ms = elapsed milliseconds. */
int fr_geometry_launch(fr_ctx* ctx, float* ms);   /* entry 0 g_buffer_trace */
int fr_sampling_launch(fr_ctx* ctx, float* ms);   /* entry 1 sampling_step */
int fr_optimize_launch(fr_ctx* ctx, float* ms);   /* entry 2 warp_sort x3 -> ray_count */
int fr_shading_launch(fr_ctx* ctx, float* ms);    /* entry 3 ray_trace + history/depth swaps */
int fr_ray_count(fr_ctx* ctx, uint32_t* count);   /* m_context["ray_count"] read-back (FR/main.cpp:288-299) */
int fr_gaze_target(fr_ctx* ctx, float xyz[3]);    /* m_context["gaze_target"] read-back (:278-287) */

/* GL reconstruction passes; *elapsed_ns like GL_TIME_ELAPSED (NULL allowed). */
int fr_jfa_render(fr_ctx* ctx, int in_buffer, uint64_t* elapsed_ns);            /* JumpFlooding::render */
int fr_sibson_render(fr_ctx* ctx, uint64_t* elapsed_ns);                        /* SibsonInterpolation::render */
int fr_pullpush_render(fr_ctx* ctx, int in_buffer, uint64_t* elapsed_ns);       /* PullPushInterpolation::render */
int fr_atrous_render(fr_ctx* ctx, int count, int pos_buffer, int nrm_buffer, int col_buffer,
                     uint64_t* elapsed_ns);                                     /* ATrous::render */

/* LogPolarTransform::render (FR/Log_Polar_Transform.cpp:40-106) of any RGBA32F buffer around the
 * current gaze: forward image -> FR_BUF_LOGPOLAR, round trip -> FR_BUF_LOGPOLAR_INVERSE. */
int fr_logpolar_render(fr_ctx* ctx, int in_buffer, uint64_t* elapsed_ns);
/* Final composite of nviews rendered views (e.g. the two eyes gathered to one GPU over RCCL):
 * device `views` = nviews consecutive W x H RGBA32F images -> device `out` = (nviews * W) x H,
 * view v in columns [v W, (v+1) W) (renderAll's side-by-side display, FR/main.cpp:26-113). */
int fr_composite_views(fr_ctx* ctx, const void* views, int nviews, void* out, size_t out_bytes);
/* Gaze input, the reference's GLFW callbacks. fr_set_gaze is cursorPosCallback (FR/gui.cpp:48-66): the
 * cursor (xpos, ypos) in window coordinates (y down) sets the Win32 POINT g_gaze = ((LONG)xpos,
 * (LONG)(ypos * adjust_scale)), adjust_scale = 1 in full screen (g_fullScreen) and 1.25 in a window
 * (:51-56); fr_reset_gaze is framebufferSizeCallback's g_gaze = (w / 2, h / 2) (:32-35). The kernels use
 * (g_gaze.x, H - g_gaze.y) (FR/PathTracer.cpp:795) from the next launch on; fr_set_camera's gaze
 * replaces it too. */
int fr_set_gaze(fr_ctx* ctx, double xpos, double ypos, int fullscreen);
int fr_reset_gaze(fr_ctx* ctx);

/* The whole main.cpp loop body (update -> 0 -> 1 -> 2 -> 3 -> JFA -> SI -> PPI -> AT). With timing == NULL
 * nothing is synchronised and consecutive frames pipeline: frame N's reconstruction (JFA -> Sibson and
 * pull-push -> A-Trous, on two internal streams) runs while frame N+1's trace half runs on the context
 * stream; POSITION / NORMAL / SHADING alternate between two buffers by frame parity for this. Every
 * other call (stage launches, buffer access, fr_synchronize) first orders itself after the pending
 * reconstruction, so results are those of the sequential loop. With timing != NULL the frame is
 * synchronised and per-stage HIP-event times are returned. */
int fr_frame(fr_ctx* ctx, fr_frame_timing* timing);
/* How untimed fr_frame calls overlap (the reference's loop is serial, FR/main.cpp:253-373, so its
 * gaze-to-image latency is its frame time):
 *   FR_PIPELINE_THROUGHPUT (default): the host enqueues frames back to back; frame N+1's front stages
 *     (entries 0-2) run beside frame N's path trace and frame N's reconstruction beside frame N+1's trace
 *     half, up to the context's frame slots in flight (highest frames per second, latency ~2-3 frames);
 *   FR_PIPELINE_LATENCY: one trace half in flight: fr_frame first waits (on the host) for the previous
 *     frame's path trace to finish, so the gaze the caller set just before the call is sampled when the
 *     GPU can start the frame; the previous frame's reconstruction overlaps this frame's front stages
 *     (G-buffer, sampling, compaction) and ends before its path trace starts (latency ~ 1.2 serial
 *     frames, throughput above the serial loop's).
 * Results are identical in both modes. */
#define FR_PIPELINE_THROUGHPUT 0
#define FR_PIPELINE_LATENCY 1
int fr_set_pipeline_mode(fr_ctx* ctx, int mode);
/* Which reconstruction chains fr_frame / fr_reconstruct_frame run on this context: bit 0 JumpFlooding ->
 * Sibson, bit 1 pull-push -> A-Trous (default 3, both; a group's split reconstruction sets 1 and 2 on
 * the two reconstruction ranks of a view). */
int fr_set_recon_chains(fr_ctx* ctx, int chains);
/* How entry 3 sums a camera sample's radiance: 0 fp32 in the oracle's depth-first order,
 * 1 (default) by frame size (fixed point below 64 pixel-samples per megakernel lane, fp32 above), 2 32.32
 * fixed point with the tail handoff (idle lanes take pending refraction items of busy ones; the value does
 * not depend on which lane traces an item). The forms differ by rounding only (<= 1e-4). Synchronises. */
int fr_set_sample_sum(fr_ctx* ctx, int mode);
int fr_trace_frame(fr_ctx* ctx, fr_frame_timing* timing);        /* update -> entries 0..3 only */
int fr_reconstruct_frame(fr_ctx* ctx, fr_frame_timing* timing);  /* JFA -> SI -> PPI -> AT only */
int fr_synchronize(fr_ctx* ctx);

/* Tile sharding of one view across ranks (BASELINE configs[3]): screen tiles of
 * tile x tile pixels, tile t = ty * ceil(W / tile) + tx traced by rank t % count (round robin, so
 * the dense foveal tiles spread over all ranks). Every rank computes the full G-buffer and sampling
 * mask and traces only its own tiles' active pixels; the compositing rank unpacks the other ranks'
 * tiles of SHADING and runs the reconstruction half. Exact for a static camera (history is
 * per-tile); with a moving camera also exchange HISTORY_CACHE the same way. count = 1 restores the
 * whole screen. Slabs are device buffers of fr_shard_texels() RGBA32F texels (T*T per owned tile,
 * owned tiles in increasing order); pack/unpack synchronise the context stream. (fr_group_* below
 * runs all of this, RCCL included, behind one call per frame.) */
int fr_set_shard(fr_ctx* ctx, int rank, int count, int tile);
/* Explicit tile owners: owner[t] (< count) traces tile t (ntiles = ceil(W/tile) * ceil(H/tile)). */
int fr_set_shard_plan(fr_ctx* ctx, int rank, int count, int tile, const uint8_t* owner, size_t ntiles);
/* Host only (no device): deals the ntiles tiles of a W x H screen over count ranks in proportion to
 * weights[0..count-1] (>= 0, not all 0) by smooth weighted round robin in raster order, so every rank
 * gets its share of the dense foveal tiles. weights NULL = equal. Writes owner[0..ntiles-1]. */
int fr_shard_plan(int width, int height, int tile, int count, const float* weights, uint8_t* owner, size_t ntiles);
/* Active pixels of every rank of the view in the last front stages (sampling + compaction), counted
 * on this rank from its own full mask: the pixels rank r traces and sends. Synchronises the front. */
int fr_shard_counts(fr_ctx* ctx, uint32_t* counts, int n);
/* Tile-local front stages for a tracing rank of a static camera (on = 1; needs count > 1 in the shard
 * plan): the G-buffer runs only on this rank's tiles plus the 4-pixel halo the saliency stencil reads
 * (and on the gaze pixel's 8x8 tile), and the sampling mask, compaction and the history carry only on
 * this rank's tiles. Its traced pixels are unchanged; every other pixel of its buffers is unspecified,
 * and fr_shard_counts reports 0 for the other ranks. The reprojection reads the previous frame at the
 * same pixel only while the camera is still, so a moving camera needs on = 0 (the default). A new shard
 * plan keeps the setting (and recomputes the tiles); a whole-screen plan turns it off. */
int fr_set_front_local(fr_ctx* ctx, int on);
/* The same with the tiles dealt over ranks first_tracer .. count-1 only (tile t to rank
 * first_tracer + t % (count - first_tracer)); ranks below first_tracer trace nothing. first_tracer = 1
 * leaves the view's compositing rank 0 to the G-buffer and the reconstruction half, which no other
 * rank can share (JFA's reach, the global pull-push pyramid). fr_set_shard = first_tracer 0. */
int fr_set_shard_ex(fr_ctx* ctx, int rank, int count, int tile, int first_tracer);
/* Sparse SHADING gather (SURVEY §8(e) "sparse variant"): a tracing rank packs only the pixels its last
 * trace half shaded, as capacity x 16 B of (tone-mapped radiance, 1) texels followed by capacity x 4 B of
 * pixel indices (slab_bytes >= 20 x capacity, else FR_E_INVALID); *count returns their number
 * (FR_E_INVALID when it exceeds capacity: size capacity from fr_ray_count). A receiving rank, after its own
 * trace half (which carries every other pixel's history), adds each entry's reprojected history from its
 * own history, as the shading resolve does, and scatters the sums into HISTORY_CACHE and SHADING (indices
 * outside the screen are skipped; the sender's own history is not used: a tile-edge pixel's reprojection
 * can round into another rank's tiles). ~10x less than the tile slabs at a 10 % mask. Exact for a
 * static camera when the compositing rank receives; with a moving camera when every rank receives
 * every other rank's pixels each frame (its reprojection then reads a complete history). Both
 * synchronise the context stream. */
int fr_shard_pack_active(fr_ctx* ctx, void* device_slab, size_t slab_bytes, uint32_t capacity, uint32_t* count);
int fr_shard_unpack_active(fr_ctx* ctx, const void* device_slab, size_t slab_bytes, uint32_t capacity,
                           uint32_t count);
/* fr_shard_unpack_active without the synchronisation: enqueued on the context stream after the work
 * already there (the slab must stay valid until that work has run, e.g. until fr_synchronize). */
int fr_shard_unpack_active_enqueue(fr_ctx* ctx, const void* device_slab, size_t slab_bytes, uint32_t capacity,
                                   uint32_t count);
int fr_shard_texels(fr_ctx* ctx, size_t* texels);
int fr_shard_pack(fr_ctx* ctx, int buffer_id, void* device_slab, size_t bytes);
int fr_shard_unpack(fr_ctx* ctx, int buffer_id, int src_rank, const void* device_slab, size_t bytes);

/* ---- Multi-GPU groups (SURVEY §8(b) Threading, §8(e)) --------------------------------------------
 * The reference is single-GPU; this is how frames shard over the GPUs of a node. A group is R ranks
 * (one fr_ctx each, all created with the same fr_config apart from .device) rendering V views (eyes) of
 * G = R / V ranks: rank r renders view r / G as view rank r % G (view v's camera is set on its ranks'
 * contexts with fr_set_camera as usual). In a view the screen tiles are dealt over the ranks by weight
 * (fr_shard_plan). Every rank runs the front stages (G-buffer, sampling mask, compaction) and traces its
 * own tiles' active pixels; each traced pixel (20 B: radiance texel + pixel index) goes to the view's
 * reconstruction ranks, which run JumpFlooding -> Sibson (view rank 0) and pull-push -> A-Trous (view
 * rank 1 with split_recon, else rank 0 as well); the composite is bit-identical to the one-GPU frame.
 * That gather is the path's only exchange (JFA's reach and the pull-push pyramid are global); it uses
 * RCCL ncclSend/ncclRecv over xGMI, sized on every rank from its own full mask (fr_shard_counts), so
 * there is no control collective and no host synchronisation beyond each rank's own front stages. With
 * moving_camera every rank receives every other rank's pixels instead (reprojection reads across
 * tiles). The optional composite gathers each view's A-Trous image to rank 0 (the stereo pair of
 * BASELINE configs[4], side by side, renderAll FR/main.cpp:26-113).
 * Ranks live either in one process (ctxs[0..n-1], any devices, rccl_comm NULL: device-to-device
 * copies; n = R) or one per process (n = 1, rccl_comm = an ncclComm_t of R ranks whose rank is this
 * context's: fr_rccl_comm_init, or the caller's own). */
#define FR_GROUP_MAX_VIEW_RANKS 16
typedef struct fr_group fr_group;
typedef struct fr_group_config {
  int views;               /* V >= 1, divides R */
  int tile;                /* screen tile edge, a multiple of 16 (default 128) */
  int split_recon;         /* 1 (default): the two reconstruction chains on view ranks 0 and 1 when G >= 2 */
  int moving_camera;       /* 1: every rank receives every other rank's traced pixels (default 0) */
  int composite;           /* 1: every frame, the views' A-Trous images side by side on rank 0 */
  float recon_cost[2];     /* the reconstruction work of view ranks 0 and 1 as a fraction of one frame's
                              trace work (default 0.5, 0.17: JFA + Sibson, pull-push + A-Trous at 4K);
                              the tiles are dealt so that every rank's total is level (water filling) */
  float weights[FR_GROUP_MAX_VIEW_RANKS];  /* explicit tracing weights per view rank; all 0 = from recon_cost */
  int sample_sum;          /* fr_set_sample_sum on every rank when G >= 2 (default 2: fixed point with the tail
                              handoff, which shortens a tracer's small launch; the view then equals a one-GPU
                              frame in that form); -1 leaves the contexts as they are */
  int front_local;         /* 1 (default): with a still camera, ranks that only trace run their front stages
                              on their own tiles plus halo (fr_set_front_local); ignored with moving_camera */
  int jfa_ranks;           /* view ranks that take JumpFlooding -> Sibson in turns, one frame each: view rank 0,
                              then 2, 3, ... (they all receive every traced pixel; the chain keeps no state
                              across frames). 0 (default) = auto: 2 when G >= 6 with split_recon, else 1 */
} fr_group_config;
int fr_group_config_default(fr_group_config* cfg);
/* RCCL bootstrap for callers without their own: rank 0 creates the 128-byte unique id, every rank
 * passes it (sent by any means) to fr_rccl_comm_init on its own device. */
int fr_rccl_unique_id(void* id128);
int fr_rccl_comm_init(const void* id128, int nranks, int rank, int device, void** comm);
int fr_rccl_comm_destroy(void* comm);
int fr_group_create(fr_ctx* const* ctxs, int n, void* rccl_comm, const fr_group_config* cfg, fr_group** out);
/* One frame of every local rank (update -> 0 -> 1 -> 2 -> 3, exchange, JFA -> SI and PPI -> AT on the
 * reconstruction ranks, the composite). timing == NULL: nothing is synchronised beyond the front stages'
 * counts, and consecutive frames pipeline. timing != NULL (n timings, one per local rank): the frame is
 * synchronised and each rank's stage times are returned (reconstruction stages 0 on other ranks). */
int fr_group_frame(fr_group* g, fr_frame_timing* timing);
/* Final composite (the group must have composite = 1): copies the last frame's (V * W) x H RGBA32F image
 * from rank 0 to device memory `out` of rank 0's device (bytes >= V * W * H * 16); synchronises. */
int fr_group_composite(fr_group* g, void* out, size_t bytes);
/* Roles of local rank i: *view, *view_rank, *chains (bit 0 JFA -> Sibson, bit 1 pull-push -> A-Trous
 * run here) and *tiles, the number of screen tiles it traces. */
int fr_group_rank_info(fr_group* g, int i, int* view, int* view_rank, int* chains, int* tiles);
/* Host only (no device): the tile plan fr_group_create would deal for one view of ranks_per_view ranks
 * (cfg NULL = fr_group_config_default): owner[t] = the view rank tracing tile t. */
int fr_group_plan(int width, int height, int ranks_per_view, const fr_group_config* cfg, uint8_t* owner, size_t ntiles);
/* Where the last frame's outputs of a view are: the global rank holding its JFA / Sibson images (the
 * rank whose turn it was, see jfa_ranks) and the one holding its pull-push / A-Trous images. */
int fr_group_output_ranks(fr_group* g, int view, int* jfa_rank, int* atrous_rank);
/* The tile plan of the views: owner[t] = the view rank that traces tile t (ntiles = ceil(W/tile) *
 * ceil(H/tile); all 0 when G = 1). */
int fr_group_tile_owners(fr_group* g, uint8_t* owner, size_t ntiles);
int fr_group_synchronize(fr_group* g);
int fr_group_destroy(fr_group* g);  /* the contexts trace the whole screen again */
const char* fr_group_last_error(void);  /* the failure of the calling thread's last fr_group_* / fr_rccl_* call */


/* GPU BVH builder (the reference's OptiX acceleration rebuild,
 * FR/PathTracer.cpp:590-602 rtAccelerationCreate(ctx, "Trbvh")). fr_rebuild_bvh re-indexes the
 * current triangles on the device (LBVH: Morton sort + Karras hierarchy, collapsed into the
 * engine's four-wide nodes); *ms = its wall time. fr_set_positions replaces the world-space
 * vertex positions (host array, 9 floats per triangle, the scene's triangle order) and rebuilds;
 * shading normals, texture coordinates and materials are kept. */
int fr_rebuild_bvh(fr_ctx* ctx, float* ms);
int fr_set_positions(fr_ctx* ctx, const float* xyz, size_t ntris);
/* Buffer access (PathTracer::get_texture, FR/PathTracer.cpp:337-374; rtBufferMap). */
int fr_get_buffer(fr_ctx* ctx, int id, fr_buffer_view* view);
int fr_read_buffer(fr_ctx* ctx, int id, void* host, size_t bytes);
int fr_write_buffer(fr_ctx* ctx, int id, const void* host, size_t bytes);
int fr_copy_buffer(fr_ctx* ctx, int id, void* device_dst, size_t bytes);  /* device-to-device, synchronous */
/* Snapshot / restore of the temporal state a frame hands to the next (the reference keeps it in
 * the history / depth ping-pong, FR/PathTracer.cpp:226-238, and in the push atlas carried across frames,
 * FR/PullPushInterpolation.cpp:57-58): HISTORY_CACHE / HISTORY, DEPTH_CACHE / DEPTH, the pull and push atlases
 * and the push snapshot texels, m_accumFrame (with a pending light reset), the light emission, the diffuse
 * depth and the last camera / gaze uniforms. fr_snapshot_bytes gives the size; fr_snapshot copies it to host
 * memory after all pending work; fr_restore loads it into a context of the same size, spp and scene
 * (FR_E_INVALID otherwise), so the next frame equals the one that followed the snapshot, bit for bit. */
int fr_snapshot_bytes(fr_ctx* ctx, size_t* bytes);
int fr_snapshot(fr_ctx* ctx, void* host, size_t bytes);
int fr_restore(fr_ctx* ctx, const void* host, size_t bytes);

int fr_get_stats(fr_ctx* ctx, fr_stats* stats);
int fr_reset_stats(fr_ctx* ctx);

/* Live timing of entry 3 inside pipelined frames (no synchronisation added): after
 * fr_kernel_timing(ctx, 1) every shading stage records HIP events on the context stream around
 * itself and around the path-trace megakernel; fr_kernel_times returns the number of stages timed
 * since and their summed milliseconds (what rocprofv3 --kernel-trace reports for k_shade_paths).
 * fr_kernel_timing(ctx, 0) stops and clears. */
typedef struct fr_stage_times {
  uint32_t frames;
  double shading_ms;      /* carry_history + k_shade_paths + k_shade_resolve, summed */
  double shade_paths_ms;  /* k_shade_paths alone, summed */
} fr_stage_times;
int fr_kernel_timing(fr_ctx* ctx, int enable);
int fr_kernel_times(fr_ctx* ctx, fr_stage_times* out);

/* Frame clock of fr_frame (no synchronisation added beyond a ring of 16 frames): after
 * fr_frame_clock(ctx, 1) every fr_frame records a HIP event where its G-buffer may start (after the
 * waits for its frame slot) and one after both of its reconstruction chains. fr_frame_clock_read
 * returns, per frame since, the latency (start -> end: the gaze the frame samples to its finished
 * Sibson and A-Trous images, on the GPU) and the interval between consecutive frames' ends (the frame
 * time a display sees), in milliseconds; *n_latency / *n_interval receive the counts (at most cap each).
 * The reference's frame time is the serial sum of its stage timers (FR/main.cpp:368-373).
 * fr_frame_clock(ctx, 0) stops and clears. */
int fr_frame_clock(fr_ctx* ctx, int enable);
int fr_frame_clock_read(fr_ctx* ctx, float* latency_ms, float* interval_ms, int cap, int* n_latency, int* n_interval);

/* Scene inspection (host copies owned by the context; valid until fr_destroy). */
typedef struct fr_scene_arrays {
  int num_tris;
  const float* pos;      /* 9 floats per triangle (p0, p1, p2) */
  const float* nrm;      /* 9 floats per triangle */
  const float* uv;       /* 6 floats per triangle */
  const int32_t* flags;  /* material | 0x100 has_normals | 0x200 has_uv */
  int num_materials;
  const int32_t* materials;  /* (type, texture) pairs: 0 diffuse, 1 reflection, 2 refraction */
  int num_textures;
  const int32_t* tex_dims;   /* (w, h) pairs */
  const float* const* tex_data;  /* RGBA32F, row 0 = bottom */
  int envmap;
  float light[15];       /* position, v1, v2, normal, emission */
  float bbox[6];         /* min, max */
  int bvh_nodes, bvh_depth;  /* four-wide nodes, levels */
  int bvh_max_stack;        /* deepest traversal stack the tree can need (<= 24) */
} fr_scene_arrays;
int fr_scene_export(fr_ctx* ctx, fr_scene_arrays* out);

/* Host-only scene construction (no device needed): the same presets fr_create builds, for
 * inspection, asset checks and CPU-side validation. */
typedef struct fr_scene fr_scene;
int fr_scene_create(const fr_config* cfg, fr_scene** out);
int fr_scene_get_arrays(fr_scene* scene, fr_scene_arrays* out);
int fr_scene_destroy(fr_scene* scene);

#ifdef __cplusplus
}
#endif
#endif /* FOVRT_H */
