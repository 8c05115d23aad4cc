// context.cpp — fr_ctx: device memory, stage orchestration and the C ABI of include/fovrt.h.
//
// Host-side counterpart of PathTracer (FR/PathTracer.cpp) and of the GL pass classes
// (FR/JumpFlooding.cpp, FR/SibsonInterpolation.cpp, FR/PullPushInterpolation.cpp, FR/ATrous.cpp):
// one HIP stream per context, every buffer allocated once in fr_create, zero host copies between
// stages (the reference's PBO->texture copies, FR/PathTracer.cpp:253-305, disappear).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <chrono>
#include "ctx_internal.h"
#include <immintrin.h>
#include <sched.h>

namespace {
// Host-side waits of the latency mode poll (a blocking wait woke the host up to milliseconds late). The spin
// pauses between queries, yields the core every 64 polls (RCCL proxy threads or other ranks' host threads may
// share it), and gives up after a deadline instead of spinning forever on an event that never completes.
constexpr float kPollDeadlineMs = 10000.0f;
inline void cpu_relax() { _mm_pause(); }
hipError_t poll_event(hipEvent_t ev, float deadline_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t n = 1;; n++) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
    if ((n & 63u) == 0) {
      if (std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count() > deadline_ms)
        return hipErrorNotReady;
      sched_yield();
    } else {
      cpu_relax();
    }
  }
}
}  // namespace

using namespace fr;

static thread_local std::string g_create_error;

namespace {

int fail(fr_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg; else g_create_error = msg;
  return code;
}

#define HIP_TRY(ctx, expr)                                                                                 \
  do {                                                                                                     \
    hipError_t e_ = (expr);                                                                                \
    if (e_ != hipSuccess) return fail(ctx, FR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T>
hipError_t dalloc(T** p, size_t count) {
  hipError_t e = hipMalloc((void**)p, count * sizeof(T) + 16);
  if (e != hipSuccess) return e;
  return hipMemset(*p, 0, count * sizeof(T) + 16);
}

int check_launch(fr_ctx* c) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(c, FR_E_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return FR_OK;
}

// ---- glm-compatible camera math (FR/Camera.cpp; glm 0.9.x, GLM_FORCE_RADIANS) --------------
struct Q { float w, x, y, z; };
f3 qrot(Q q, f3 v) {  // glm::operator*(quat, vec3)
  f3 qv = mk3(q.x, q.y, q.z);
  f3 uv = cross(qv, v);
  f3 uuv = cross(qv, uv);
  return v + ((uv * q.w) + uuv) * 2.0f;
}
Q quat_cast(const float m[3][3]) {  // glm::quat_cast(mat3), m[col][row]
  float fx = m[0][0] - m[1][1] - m[2][2];
  float fy = m[1][1] - m[0][0] - m[2][2];
  float fz = m[2][2] - m[0][0] - m[1][1];
  float fw = m[0][0] + m[1][1] + m[2][2];
  int bi = 0;
  float fb = fw;
  if (fx > fb) { fb = fx; bi = 1; }
  if (fy > fb) { fb = fy; bi = 2; }
  if (fz > fb) { fb = fz; bi = 3; }
  float bv = sqrtf(fb + 1.0f) * 0.5f;
  float mult = 0.25f / bv;
  switch (bi) {
    case 0: return Q{bv, (m[1][2] - m[2][1]) * mult, (m[2][0] - m[0][2]) * mult, (m[0][1] - m[1][0]) * mult};
    case 1: return Q{(m[1][2] - m[2][1]) * mult, bv, (m[0][1] + m[1][0]) * mult, (m[2][0] + m[0][2]) * mult};
    case 2: return Q{(m[2][0] - m[0][2]) * mult, (m[0][1] + m[1][0]) * mult, bv, (m[1][2] + m[2][1]) * mult};
    default: return Q{(m[0][1] - m[1][0]) * mult, (m[2][0] + m[0][2]) * mult, (m[1][2] + m[2][1]) * mult, bv};
  }
}
Q qnormalize(Q q) {
  float len = sqrtf(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  if (len <= 0.0f) return Q{1, 0, 0, 0};
  float inv = 1.0f / len;
  return Q{q.w * inv, q.x * inv, q.y * inv, q.z * inv};
}
// column-major glm mat4 helpers: M[c][r]
struct M4 { float m[4][4]; };
M4 glm_lookat(f3 eye, f3 center, f3 up) {
  f3 f = normalize(center - eye);
  f3 s = normalize(cross(f, up));
  f3 u = cross(s, f);
  M4 r = {};
  r.m[0][0] = s.x; r.m[1][0] = s.y; r.m[2][0] = s.z;
  r.m[0][1] = u.x; r.m[1][1] = u.y; r.m[2][1] = u.z;
  r.m[0][2] = -f.x; r.m[1][2] = -f.y; r.m[2][2] = -f.z;
  r.m[3][0] = -dot(s, eye); r.m[3][1] = -dot(u, eye); r.m[3][2] = dot(f, eye);
  r.m[3][3] = 1.0f;
  return r;
}
M4 glm_perspective(float fovy, float aspect, float zn, float zf) {
  float t = tanf(fovy / 2.0f);
  M4 r = {};
  r.m[0][0] = 1.0f / (aspect * t);
  r.m[1][1] = 1.0f / t;
  r.m[2][2] = -(zf + zn) / (zf - zn);
  r.m[2][3] = -1.0f;
  r.m[3][2] = -(2.0f * zf * zn) / (zf - zn);
  return r;
}
M4 glm_mul(const M4& a, const M4& b) {  // glm mat4 * mat4
  M4 r;
  for (int c = 0; c < 4; c++)
    for (int k = 0; k < 4; k++)
      r.m[c][k] = a.m[0][k] * b.m[c][0] + a.m[1][k] * b.m[c][1] + a.m[2][k] * b.m[c][2] + a.m[3][k] * b.m[c][3];
  return r;
}
void pose_matrices(const fr_camera_pose* p, M4& V, M4& P) {
  Q q{p->rot[0], p->rot[1], p->rot[2], p->rot[3]};
  f3 pos = mk3(p->pos[0], p->pos[1], p->pos[2]);
  f3 front = qrot(q, mk3(0, 0, -1));
  f3 upv = qrot(q, mk3(0, 1, 0));
  V = glm_lookat(pos, pos + front, upv);
  P = glm_perspective(p->fovy_deg * 0.01745329251994329576923690768489f, p->aspect, p->znear, p->zfar);
}
void to_rowmajor(const M4& a, float out[16]) {
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) out[r * 4 + c] = a.m[c][r];
}
bool invert_rowmajor(const float in[16], float out[16]) {  // Gauss-Jordan in f64, rounded once
  double a[4][8];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 8; c++) a[r][c] = c < 4 ? in[r * 4 + c] : (c - 4 == r ? 1.0 : 0.0);
  for (int c = 0; c < 4; c++) {
    int piv = c;
    for (int r = c + 1; r < 4; r++) if (fabs(a[r][c]) > fabs(a[piv][c])) piv = r;
    if (a[piv][c] == 0.0) return false;
    if (piv != c) for (int k = 0; k < 8; k++) std::swap(a[c][k], a[piv][k]);
    double d = a[c][c];
    for (int k = 0; k < 8; k++) a[c][k] /= d;
    for (int r = 0; r < 4; r++) {
      if (r == c) continue;
      double f = a[r][c];
      for (int k = 0; k < 8; k++) a[r][k] -= f * a[c][k];
    }
  }
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) out[r * 4 + c] = (float)a[r][c + 4];
  return true;
}

// Sums the elapsed times of ring slot i (its last event is synchronised first).
void kt_harvest(fr_ctx* c, int i) {
  hipEventSynchronize(c->kt_ev[i][3]);
  float a = 0.0f, b = 0.0f;
  hipEventElapsedTime(&a, c->kt_ev[i][0], c->kt_ev[i][3]);
  hipEventElapsedTime(&b, c->kt_ev[i][1], c->kt_ev[i][2]);
  c->kt_stage_ms += a;
  c->kt_kernel_ms += b;
  c->kt_frames++;
}

// One frame of the frame clock (fr_frame_clock): its latency, and its interval after the previous frame.
void fc_harvest(fr_ctx* c, int i) {
  hipEventSynchronize(c->fc_ev[i][1]);
  float s = 0.0f, e = 0.0f;
  hipEventElapsedTime(&s, c->fc_ref, c->fc_ev[i][0]);
  hipEventElapsedTime(&e, c->fc_ref, c->fc_ev[i][1]);
  c->fc_latency.push_back(e - s);
  if (c->fc_prev_end >= 0.0) c->fc_interval.push_back((float)(e - c->fc_prev_end));
  c->fc_prev_end = e;
}

float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0.0f;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
extern "C" {

const char* fr_version(void) { return "fovrt 0.2 (gfx950)"; }
int fr_abi_version(void) { return FOVRT_ABI_VERSION; }

int fr_config_default(fr_config* c) {
  if (!c) return FR_E_INVALID;
  memset(c, 0, sizeof(*c));
  c->abi_version = FOVRT_ABI_VERSION;
  c->width = 1024; c->height = 1024;
  c->scene = FR_SCENE_BUNNY;
  c->mask_mode = FR_MASK_SALIENCY;
  c->spp = 1;
  c->diffuse_max_depth = 1;
  c->refraction_max_depth = 16;
  c->light_power = 810.0f;
  c->optimize = 1;
  c->atrous_iterations = 1;
  c->write_extra = 1;
  c->device = 0;
  c->texture_mode = 0;
  c->detail = 0;
  c->mesh_mode = 0;
  c->asset_dir = nullptr;
  return FR_OK;
}

const char* fr_last_error(fr_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int fr_preset_camera(int scene, float eye[3], float target[3]) {
  f3 e, t;
  preset_camera(scene, e, t);
  eye[0] = e.x; eye[1] = e.y; eye[2] = e.z;
  target[0] = t.x; target[1] = t.y; target[2] = t.z;
  return FR_OK;
}

int fr_camera_look_at(fr_camera_pose* pose, const float target[3], const float up[3]) {
  if (!pose || !target) return FR_E_INVALID;
  f3 pos = mk3(pose->pos[0], pose->pos[1], pose->pos[2]);
  f3 tg = mk3(target[0], target[1], target[2]);
  f3 u = up ? mk3(up[0], up[1], up[2]) : mk3(0, 1, 0);
  f3 z = normalize(pos - tg);
  f3 x = normalize(cross(u, z));
  f3 y = normalize(cross(z, x));
  float m[3][3] = {{x.x, x.y, x.z}, {y.x, y.y, y.z}, {z.x, z.y, z.z}};
  Q q = qnormalize(quat_cast(m));
  pose->rot[0] = q.w; pose->rot[1] = q.x; pose->rot[2] = q.y; pose->rot[3] = q.z;
  return FR_OK;
}

int fr_camera_matrices(const fr_camera_pose* pose, float view[16], float proj[16]) {
  if (!pose) return FR_E_INVALID;
  M4 V, P;
  pose_matrices(pose, V, P);
  if (view) to_rowmajor(V, view);
  if (proj) to_rowmajor(P, proj);
  return FR_OK;
}

int fr_camera_uniforms(const fr_camera_pose* cur, const fr_camera_pose* prev, int width, int height, fr_camera* out) {
  if (!cur || !out || width <= 0 || height <= 0) return FR_E_INVALID;
  if (!prev) prev = cur;
  M4 V, P, PV, pV, pP, pPV;
  pose_matrices(cur, V, P);
  PV = glm_mul(P, V);
  pose_matrices(prev, pV, pP);
  pPV = glm_mul(pP, pV);
  float rm[16];
  to_rowmajor(PV, rm);
  if (!invert_rowmajor(rm, out->inv_vp)) return FR_E_INVALID;
  to_rowmajor(pPV, out->prev_vp);
  for (int k = 0; k < 3; k++) { out->eye[k] = cur->pos[k]; out->prev_eye[k] = prev->pos[k]; }
  Q q{cur->rot[0], cur->rot[1], cur->rot[2], cur->rot[3]};
  f3 up = qrot(q, mk3(0, 1, 0));
  out->up[0] = up.x; out->up[1] = up.y; out->up[2] = up.z;
  f3 fr = qrot(q, mk3(0, 0, -1));
  out->target[0] = cur->pos[0] + fr.x; out->target[1] = cur->pos[1] + fr.y; out->target[2] = cur->pos[2] + fr.z;
  // g_gaze = (w/2, h/2) ints (FR/gui.cpp:34-35); gaze = (g_gaze.x, H - g_gaze.y) (FR/PathTracer.cpp:795)
  out->gaze[0] = (float)(width / 2);
  out->gaze[1] = (float)(height - height / 2);
  return FR_OK;
}

// GPU build over c->d_pos (k_bvh.hip) into the spare arrays, which become the scene's tree when every
// step succeeded (the old tree becomes the spare). No allocation after the first rebuild, no read-back
// of the tree: the host keeps its node count, stack need and depth (fr_scene_export).
static int gpu_rebuild(fr_ctx* c) {
  const int nt = c->scene.num_tris();
  if (!c->spare_nodes) {  // (a failed re-allocation below left none)
    if (hipMalloc((void**)&c->spare_nodes, (size_t)std::max(nt, 1) * sizeof(BvhNode)) != hipSuccess ||
        hipMalloc((void**)&c->spare_tri, (size_t)std::max(nt, 1) * sizeof(TriGeo)) != hipSuccess ||
        hipMalloc((void**)&c->spare_prim, (size_t)std::max(nt, 1) * sizeof(int32_t)) != hipSuccess) {
      c->err = "GPU BVH: device allocation failed";
      return FR_E_NOMEM;
    }
  }
  int nn = 0, max_stack = 0, depth = 0;
  std::string err;
  if (!gpu_build_bvh(&c->bvh_work, c->d_pos, nt, c->spare_nodes, c->spare_tri, c->spare_prim, &nn, &max_stack, &depth,
                     c->stream, err)) {
    c->err = err;
    return FR_E_HIP;
  }
  if (max_stack > FR_BVH_STACK) {
    c->err = "GPU BVH needs a traversal stack deeper than FR_BVH_STACK";
    return FR_E_UNSUPPORTED;
  }
  std::swap(c->d_nodes, c->spare_nodes);
  std::swap(c->d_tri, c->spare_tri);
  std::swap(c->d_prim, c->spare_prim);
  if (!c->tree_full_cap) {
    // the replaced tree was sized for the host builder's node count (or there was none): the next spare
    // needs room for any device-built tree (at most one node per triangle)
    if (c->spare_nodes) { hipFree(c->spare_nodes); hipFree(c->spare_tri); hipFree(c->spare_prim); }
    c->spare_nodes = nullptr; c->spare_tri = nullptr; c->spare_prim = nullptr;
    c->tree_full_cap = true;
    if (hipMalloc((void**)&c->spare_nodes, (size_t)std::max(nt, 1) * sizeof(BvhNode)) != hipSuccess ||
        hipMalloc((void**)&c->spare_tri, (size_t)std::max(nt, 1) * sizeof(TriGeo)) != hipSuccess ||
        hipMalloc((void**)&c->spare_prim, (size_t)std::max(nt, 1) * sizeof(int32_t)) != hipSuccess) {
      hipFree(c->spare_nodes); hipFree(c->spare_tri); hipFree(c->spare_prim);
      c->spare_nodes = nullptr; c->spare_tri = nullptr; c->spare_prim = nullptr;  // allocated again next time
    }
  }
  c->dsc.nodes = c->d_nodes; c->dsc.tri_geo = c->d_tri; c->dsc.tri_prim = c->d_prim;
  Bvh b;
  b.root_count = 0; b.max_stack = max_stack; b.max_depth = depth;
  b.gpu_nodes = nn;
  b.host_nodes = 0;
  c->bvh = std::move(b);
  return FR_OK;
}

// The densest exact storage of a host texture (DevTexture): FR_TEX_UNORM8 when every channel of every
// texel is (float)b / 255.0f, FR_TEX_RGBE when every texel is m * 2^(e - 136) with alpha 1 (load_hdr's
// decoding), else FR_TEX_F32. Each candidate is decoded back here with the loaders' own formulas and
// must reproduce every float bit for bit.
static int pack_texture(const HostTexture& t, std::vector<uint32_t>& out) {
  const size_t n = t.data.size();
  auto same = [](float a, float b) { return std::memcmp(&a, &b, sizeof(float)) == 0; };
  out.resize(n);
  bool unorm = true;
  for (size_t i = 0; i < n && unorm; i++) {
    const float v[4] = {t.data[i].x, t.data[i].y, t.data[i].z, t.data[i].w};
    uint32_t word = 0;
    for (int c = 0; c < 4; c++) {
      const long b = std::lrint((double)v[c] * 255.0);
      if (b < 0 || b > 255 || !same((float)b / 255.0f, v[c])) { unorm = false; break; }
      word |= (uint32_t)b << (8 * c);
    }
    out[i] = word;
  }
  if (unorm) return FR_TEX_UNORM8;
  for (size_t i = 0; i < n; i++) {
    const float v[3] = {t.data[i].x, t.data[i].y, t.data[i].z};
    if (!same(t.data[i].w, 1.0f)) return FR_TEX_F32;
    const float M = std::max(v[0], std::max(v[1], v[2]));
    uint32_t word = 0;
    if (M > 0.0f) {
      int ex = 0;
      std::frexp(M, &ex);
      const int k = ex - 8, e = k + 136;  // M / 2^k in [128, 256)
      if (e < 1 || e > 255) return FR_TEX_F32;
      const float f = std::ldexp(1.0f, e - 136);
      for (int c = 0; c < 3; c++) {
        const float m = std::ldexp(v[c], -k);
        if (!(m >= 0.0f && m <= 255.0f) || m != std::floor(m) || !same((float)(int)m * f, v[c])) return FR_TEX_F32;
        word |= (uint32_t)m << (8 * c);
      }
      word |= (uint32_t)e << 24;
    } else if (!(same(v[0], 0.0f) && same(v[1], 0.0f) && same(v[2], 0.0f))) {
      return FR_TEX_F32;
    }
    out[i] = word;
  }
  return FR_TEX_RGBE;
}

int fr_create(const fr_config* cfg_in, fr_ctx** out) {
  if (!out) return fail(nullptr, FR_E_INVALID, "out is NULL");
  *out = nullptr;
  fr_config cfg;
  if (cfg_in) cfg = *cfg_in; else fr_config_default(&cfg);
  if (cfg.abi_version != FOVRT_ABI_VERSION)
    return fail(nullptr, FR_E_INVALID, "fr_config.abi_version != FOVRT_ABI_VERSION (initialise it with fr_config_default)");
  if (cfg.width <= 0 || cfg.height <= 0 || cfg.width > 32767 || cfg.height > 32767)
    return fail(nullptr, FR_E_INVALID, "width/height out of range (1..32767)");
  if (!(cfg.spp == 1 || cfg.spp == 2 || cfg.spp == 4 || cfg.spp == 8))
    return fail(nullptr, FR_E_UNSUPPORTED, "spp must be 1, 2, 4 or 8");
  if (cfg.mask_mode < 0 || cfg.mask_mode > 4) return fail(nullptr, FR_E_INVALID, "bad mask_mode");
  if (cfg.mesh_mode < 0 || cfg.mesh_mode > 2) return fail(nullptr, FR_E_INVALID, "bad mesh_mode");
  if (cfg.scene < 0 || cfg.scene > 2) return fail(nullptr, FR_E_INVALID, "bad scene preset");
  if (cfg.refraction_max_depth < 0 || cfg.refraction_max_depth > 100) return fail(nullptr, FR_E_INVALID, "bad refraction_max_depth");
  if (cfg.sibson_mode < 0 || cfg.sibson_mode > 1) return fail(nullptr, FR_E_INVALID, "bad sibson_mode");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(nullptr, FR_E_HIP, "no HIP device available");
  if (cfg.device < 0 || cfg.device >= ndev) return fail(nullptr, FR_E_INVALID, "device ordinal out of range");

  fr_ctx* c = new fr_ctx();
  c->cfg = cfg;
  c->asset_dir = cfg.asset_dir ? cfg.asset_dir : "assets";
  c->cfg.asset_dir = nullptr;
  c->W = cfg.width; c->H = cfg.height;
  auto bail = [&](int code) { g_create_error = c->err; fr_destroy(c); return code; };
  if (hipSetDevice(cfg.device) != hipSuccess) { c->err = "hipSetDevice failed"; return bail(FR_E_HIP); }
  // Stream priorities (FOVRT_STREAM_PRIORITY, A/B knob): 0 (default) all streams at the default
  // priority; 1 trace half (context stream, carry, front stages) high, reconstruction low; 2 the
  // reconstruction high, the trace half low; 3 only the front stages high; 4 JumpFlooding -> Sibson high,
  // pull-push -> A-Trous and the front stages low.
  static const int prio_mode = [] {
    const char* v = getenv("FOVRT_STREAM_PRIORITY");
    return v ? atoi(v) : 0;
  }();
  int lo = 0, hi = 0;
  if (prio_mode) hipDeviceGetStreamPriorityRange(&lo, &hi);
  const int p_trace = prio_mode == 1 ? hi : prio_mode == 2 ? lo : 0;
  const int p_recon = prio_mode == 1 ? lo : prio_mode == 2 ? hi : 0;
  const int p_front = prio_mode == 1 || prio_mode == 3 ? hi : prio_mode == 2 || prio_mode == 4 ? lo : 0;
  const int p_jfa = prio_mode == 4 ? hi : p_recon, p_pp = prio_mode == 4 ? lo : p_recon;
  // CU masks (FOVRT_RECON_CUS = R, A/B knob, 0 = off): the two reconstruction streams run on R CUs spread evenly
  // over the device's CU mask (every XCD); FOVRT_CU_DISJOINT=1 also keeps the trace streams off those CUs.
  static const int recon_cus = [] { const char* v = getenv("FOVRT_RECON_CUS"); return v ? atoi(v) : 0; }();
  static const int cu_disjoint = [] { const char* v = getenv("FOVRT_CU_DISJOINT"); return v ? atoi(v) : 0; }();
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg.device);
  const bool masked = recon_cus > 0 && recon_cus < ncu;
  std::vector<uint32_t> m_recon((size_t)(ncu + 31) / 32, 0u), m_trace((size_t)(ncu + 31) / 32, 0u);
  if (masked) {
    for (int i = 0; i < recon_cus; i++) {
      const int b = (int)((int64_t)i * ncu / recon_cus);
      m_recon[(size_t)b / 32] |= 1u << (b % 32);
    }
    for (int b = 0; b < ncu; b++)
      if (!cu_disjoint || !(m_recon[(size_t)b / 32] & (1u << (b % 32)))) m_trace[(size_t)b / 32] |= 1u << (b % 32);
  }
  auto mk = [&](hipStream_t* st, int prio, bool recon) {
    if (!masked) return hipStreamCreateWithPriority(st, hipStreamNonBlocking, prio);
    std::vector<uint32_t>& m = recon ? m_recon : m_trace;
    return hipExtStreamCreateWithCUMask(st, (uint32_t)m.size(), m.data());
  };
  if (mk(&c->stream, p_trace, false) != hipSuccess || mk(&c->stream2, p_pp, true) != hipSuccess ||
      mk(&c->stream3, p_jfa, true) != hipSuccess || mk(&c->stream4, p_trace, false) != hipSuccess ||
      mk(&c->stream5, p_front, false) != hipSuccess) {
    c->err = "stream create failed";
    return bail(FR_E_HIP);
  }
  for (auto& e : c->ev) hipEventCreate(&e);
  hipEventCreateWithFlags(&c->ev_front, hipEventDisableTiming);
  for (auto& e : c->ev_trace) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& e : c->ev_recon) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& e : c->ev_jfa) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& row : c->lat_ev) for (auto& e : row) hipEventCreate(&e);
  for (auto& e : c->ev_counts) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  if (const char* v = getenv("FOVRT_SHADE_CHUNK_REFR")) c->chunk_refr = (uint32_t)std::max(0, atoi(v));
  if (const char* v = getenv("FOVRT_SHADE_XCD_BANDS")) c->xcd_bands = atoi(v) != 0;
  if (const char* v = getenv("FOVRT_SHADE_HANDOFF")) c->handoff = (uint32_t)std::min(std::max(atoi(v), 0), 2);
  if (const char* v = getenv("FOVRT_TEX_PACKING")) c->tex_packing = atoi(v) != 0;  // A/B knob: 0 = RGBA32F textures
  if (const char* v = getenv("FOVRT_JFA_LAZY_OUTPUTS")) c->lazy_jfa_outputs = atoi(v) != 0;  // A/B knob
  if (const char* v = getenv("FOVRT_EARLY_SETUP")) c->early_setup = atoi(v) != 0;            // A/B knob
  if (const char* v = getenv("FOVRT_SIB_STRIP")) c->sib_strip = atoi(v) != 0;      // A/B knob: 0 = k_sibson_wide for the big discs
  {  // FOVRT_SLOTS: frame slots of the pipelined loop (2 or 3; A/B knob)
    const char* v = getenv("FOVRT_SLOTS");
    if (v) c->nslots = std::max(2, std::min(fr_ctx::MAX_SLOTS, atoi(v)));
  }

  std::string err;
  if (!build_preset_scene(cfg.scene, c->asset_dir, cfg.texture_mode, cfg.light_power, cfg.detail, c->scene, err,
                          cfg.mesh_mode)) {
    c->err = "scene: " + err;
    return bail(FR_E_IO);
  }
  if (cfg.bvh_builder < 0 || cfg.bvh_builder > 1) { c->err = "bad bvh_builder"; return bail(FR_E_INVALID); }
  if (cfg.bvh_builder == 0) {
    build_bvh(c->scene, c->bvh);
    if (c->bvh.max_stack > FR_BVH_STACK) {
      c->err = "BVH needs a traversal stack deeper than FR_BVH_STACK";
      return bail(FR_E_UNSUPPORTED);
    }
  }
  const HostScene& s = c->scene;
  const int nt = s.num_tris();
  std::vector<TriShade> shade(nt);
  for (int i = 0; i < nt; i++) {
    TriShade& t = shade[i];
    f3 n0 = s.nrm[3 * i], n1 = s.nrm[3 * i + 1], n2 = s.nrm[3 * i + 2];
    f2 t0 = s.uv[3 * i], t1 = s.uv[3 * i + 1], t2 = s.uv[3 * i + 2];
    t.n0 = mk4(n0, t0.x); t.n1 = mk4(n1, t0.y); t.n2 = mk4(n2, t1.x);
    t.t = mk4(t1.y, t2.x, t2.y, bitsf((uint32_t)s.flags[i]));
  }
  auto up = [&](auto** dst, const auto& vec) -> bool {
    using T = typename std::remove_reference<decltype(vec)>::type::value_type;
    if (dalloc((T**)dst, vec.size()) != hipSuccess) return false;
    return hipMemcpy(*dst, vec.data(), vec.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(&c->d_shade, shade) || !up(&c->d_pos, s.pos)) {
    c->err = "device allocation (scene) failed";
    return bail(FR_E_NOMEM);
  }
  // The tree arrays hold one entry per triangle (room for any device-built tree), and the GPU builder's
  // spare arrays and scratch exist from the start: fr_rebuild_bvh allocates nothing (hipMalloc / hipFree
  // in a rebuild cost ~10-20 ms and synchronise the device).
  {
    const size_t cap = (size_t)std::max(nt, 1);
    if (hipMalloc((void**)&c->d_nodes, std::max(cap, c->bvh.nodes.size()) * sizeof(BvhNode)) != hipSuccess ||
        hipMalloc((void**)&c->d_tri, cap * sizeof(TriGeo)) != hipSuccess ||
        hipMalloc((void**)&c->d_prim, cap * sizeof(int32_t)) != hipSuccess ||
        hipMalloc((void**)&c->spare_nodes, cap * sizeof(BvhNode)) != hipSuccess ||
        hipMalloc((void**)&c->spare_tri, cap * sizeof(TriGeo)) != hipSuccess ||
        hipMalloc((void**)&c->spare_prim, cap * sizeof(int32_t)) != hipSuccess) {
      c->err = "device allocation (scene) failed";
      return bail(FR_E_NOMEM);
    }

    c->tree_full_cap = c->bvh.nodes.size() <= cap;
    std::string werr;
    if (nt >= 3 && !bvh_work_prepare(&c->bvh_work, nt, c->stream, werr)) { c->err = werr; return bail(FR_E_NOMEM); }
  }
  if (cfg.bvh_builder == 0) {
    if (hipMemcpy(c->d_nodes, c->bvh.nodes.data(), c->bvh.nodes.size() * sizeof(BvhNode), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_tri, c->bvh.tri_geo.data(), c->bvh.tri_geo.size() * sizeof(TriGeo), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_prim, c->bvh.tri_prim.data(), c->bvh.tri_prim.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess) {
      c->err = "device copy (scene) failed";
      return bail(FR_E_HIP);
    }
  } else if (int rc = gpu_rebuild(c)) {
    return bail(rc);
  }
  // The host-built tree's arrays go now, right after their upload, not in the first rebuild. Freeing them
  // (tens of MB, the upload's DMA source) there cost that rebuild 2-6 ms of munmap, and the next GPU
  // submission waited another 7-20 ms before its first kernel started (rocprofv3: the GPU idle with the
  // work queued; profiles/r05_rebuild): the first two rebuilds of every context took 9 and 21 ms
  // (BENCH_r04 bvh.rebuild_ms) instead of 0.8. Here the cost lands in fr_create, which synchronises.
  if (cfg.bvh_builder == 0) {
    c->bvh.host_nodes = (int)c->bvh.nodes.size();
    std::vector<BvhNode>().swap(c->bvh.nodes);
    std::vector<TriGeo>().swap(c->bvh.tri_geo);
    std::vector<int32_t>().swap(c->bvh.tri_prim);
  }
  if (nt >= 3) {
    // the GPU builder's code object is loaded now (HIP loads a module at its first launch: 3-5 ms)
    std::string werr;
    if (!bvh_builder_warm(c->bvh_work, c->stream, werr)) { c->err = werr; return bail(FR_E_HIP); }
  }
  // (the uploads above are synchronous hipMemcpy calls; the builder warm-up ran on c->stream: wait for this
  // context's stream only, not for other contexts or groups rendering on the device)
  if (hipStreamSynchronize(c->stream) != hipSuccess) { c->err = "stream synchronisation (scene) failed"; return bail(FR_E_HIP); }
  DevScene& d = c->dsc;
  memset(&d, 0, sizeof(d));
  d.nodes = c->d_nodes; d.tri_geo = c->d_tri; d.tri_prim = c->d_prim; d.shade = c->d_shade;
  d.root_count = 0; d.num_tris = nt;
  c->d_tex.resize(s.texs.size(), nullptr);
  std::vector<DevTexture> htex(s.texs.size());
  for (size_t i = 0; i < s.texs.size(); i++) {
    std::vector<uint32_t> packed;
    const int kind = c->tex_packing ? pack_texture(s.texs[i], packed) : FR_TEX_F32;
    htex[i] = DevTexture{nullptr, nullptr, s.texs[i].w, s.texs[i].h, kind};
    if (kind == FR_TEX_F32) {
      f4* p = nullptr;
      if (!up(&p, s.texs[i].data)) { c->err = "device allocation (texture) failed"; return bail(FR_E_NOMEM); }
      c->d_tex[i] = p;
      htex[i].data = p;
    } else {
      uint32_t* p = nullptr;
      if (!up(&p, packed)) { c->err = "device allocation (texture) failed"; return bail(FR_E_NOMEM); }
      c->d_tex[i] = p;
      htex[i].packed = p;
    }
  }
  if (!up(&c->d_mats, s.mats) || !up(&c->d_texs, htex)) { c->err = "device allocation (materials) failed"; return bail(FR_E_NOMEM); }
  d.mats = c->d_mats;
  d.texs = c->d_texs;
  d.envmap = s.envmap;
  d.light_position = s.light_position; d.light_v1 = s.light_v1; d.light_v2 = s.light_v2;
  d.light_normal = s.light_normal; d.light_emission = s.light_emission;
  d.light_area = lengthc(cross(s.light_v1, s.light_v2));  // as diffuse.ptx:725-736 computes A (contracted length)
  d.bbox_min = s.bbox_min; d.bbox_max = s.bbox_max;
  d.scene_epsilon = 1.e-3f;

  const size_t N = (size_t)c->W * c->H;
  for (int i = 0; i < P_COUNT; i++)
    if (dalloc(&c->img[i], N) != hipSuccess) { c->err = "device allocation (images) failed"; return bail(FR_E_NOMEM); }
  const size_t nblocks = (size_t)((c->W + 15) / 16) * ((c->H + 15) / 16);
  const size_t nwords = nblocks * 16;  // 4 waves x 4 classes per 16x16 block
  c->pp_S = pp_size(c->W, c->H);
  const size_t atlas = (size_t)c->pp_S * (c->pp_S + c->pp_S / 2);
  if (compaction_tiles(c->W, c->H) > 1024) { c->err = "screen too large for the compaction scan"; return bail(FR_E_UNSUPPORTED); }
  for (int k = 0; k < c->nslots; k++)
    if (dalloc(&c->mask_p[k], N) != hipSuccess || dalloc(&c->ray_count_p[k], 4) != hipSuccess ||
        dalloc(&c->active_p[k], N) != hipSuccess) {
      c->err = "device allocation (work buffers) failed";
      return bail(FR_E_NOMEM);
    }
  c->mask = c->mask_p[0]; c->ray_count = c->ray_count_p[0]; c->active = c->active_p[0];
  for (int k = 0; k < fr_ctx::MAX_SLOTS; k++)
    if (dalloc(&c->owner_counts_p[k], FR_MAX_SHARD_RANKS) != hipSuccess) {
      c->err = "device allocation (work buffers) failed";
      return bail(FR_E_NOMEM);
    }
  if (dalloc(&c->bcount, nblocks) != hipSuccess ||
      hipHostMalloc((void**)&c->h_counts, sizeof(uint32_t) * fr_ctx::MAX_SLOTS * FR_MAX_SHARD_RANKS) != hipSuccess) {
    c->err = "allocation (shard counts) failed";
    return bail(FR_E_NOMEM);
  }
  memset(c->h_counts, 0, sizeof(uint32_t) * fr_ctx::MAX_SLOTS * FR_MAX_SHARD_RANKS);
  if (dalloc(&c->gclass, N) != hipSuccess || dalloc(&c->lp_cache, N) != hipSuccess ||
      dalloc(&c->lp_inv, logpolar_inv_words(c->W, c->H)) != hipSuccess || dalloc(&c->words, nwords) != hipSuccess ||
      dalloc(&c->counts, 4 * nblocks) != hipSuccess || dalloc(&c->offsets, 4 * nblocks) != hipSuccess ||
      dalloc(&c->tiles, 1024) != hipSuccess || dalloc(&c->jfa_a, N) != hipSuccess || dalloc(&c->jfa_b, N) != hipSuccess ||
      dalloc(&c->pull, atlas) != hipSuccess || dalloc(&c->push, atlas) != hipSuccess ||
      dalloc(&c->snap, pp_snap_count(c->pp_S)) != hipSuccess || dalloc(&c->stats, 1) != hipSuccess ||
      dalloc(&c->shade_ctr, shade_counter_words()) != hipSuccess || dalloc(&c->samples, std::max(N * cfg.spp, 2 * shade_fx_slots((uint32_t)N, cfg.spp, c->handoff))) != hipSuccess ||
      dalloc(&c->sample_help, std::max<size_t>(4 * shade_fx_slots((uint32_t)N, cfg.spp, c->handoff), 1)) != hipSuccess ||
      dalloc(&c->aux_p[0], N) != hipSuccess || dalloc(&c->aux_seed_p[0], N) != hipSuccess ||
      dalloc(&c->aux_p[1], N) != hipSuccess || dalloc(&c->aux_seed_p[1], N) != hipSuccess ||
      dalloc(&c->hvalid, N / 64 + 1) != hipSuccess ||
      hipMalloc((void**)&c->item_store, shade_item_store_f4() * sizeof(f4)) != hipSuccess ||
      (cfg.sibson_mode == 0 && (dalloc(&c->sib_prefix, (size_t)(c->W + 1) * c->H) != hipSuccess ||
                                dalloc(&c->sib_blocks, (size_t)sibson_prefix_blocks(c->W) * c->H) != hipSuccess ||
                                hipMalloc((void**)&c->sib_wide, ((size_t)c->W * c->H + 2) * sizeof(uint32_t)) != hipSuccess ||
                                hipMalloc((void**)&c->sib_strips, sibson_strip_words(c->W, c->H) * sizeof(uint32_t)) != hipSuccess ||
                                dalloc(&c->sib_rowp, sibson_rowp_texels(c->W, c->H)) != hipSuccess))) {
    c->err = "device allocation (work buffers) failed";
    return bail(FR_E_NOMEM);
  }
  c->aux = c->aux_p[0];
  c->aux_seed = c->aux_seed_p[0];
  {  // texel centres in texture coordinates, IEEE-correctly-rounded division as in the kernels
    std::vector<float> ft((size_t)c->W + c->H);
    for (int x = 0; x < c->W; x++) ft[x] = ((float)x + 0.5f) / (float)c->W;
    for (int y = 0; y < c->H; y++) ft[(size_t)c->W + y] = ((float)y + 0.5f) / (float)c->H;
    if (!up(&c->ftab, ft)) { c->err = "device allocation (work buffers) failed"; return bail(FR_E_NOMEM); }
  }
  // Default camera: the preset pose, prev = current.
  FrameUniforms& U = c->U;
  memset(&U, 0, sizeof(U));
  U.width = c->W; U.height = c->H;
  U.screen = mk2((float)c->W, (float)c->H);
  U.diffuse_max_depth = cfg.diffuse_max_depth;
  U.reflection_max_depth = 4;
  U.refraction_max_depth = cfg.refraction_max_depth;
  U.spp = cfg.spp;
  U.sqrt_spp = (int)floor(sqrt((double)cfg.spp) + 1e-9);
  U.mask_mode = cfg.mask_mode;
  U.shard_rank = 0; U.shard_count = 1; U.shard_tile = 128; U.shard_tiles_x = (c->W + 127) / 128; U.shard_map = nullptr;
  U.front_need = nullptr; U.front_pixels = 0;
  {
    fr_camera_pose pose;
    float eye[3], tgt[3], upv[3] = {0, 1, 0};
    fr_preset_camera(cfg.scene, eye, tgt);
    memcpy(pose.pos, eye, sizeof(eye));
    pose.rot[0] = 1; pose.rot[1] = pose.rot[2] = pose.rot[3] = 0;
    pose.fovy_deg = 45.0f; pose.znear = 0.1f; pose.zfar = 500.1f;
    pose.aspect = (float)c->W / (float)c->H;
    fr_camera_look_at(&pose, tgt, upv);
    fr_camera cam;
    fr_camera_uniforms(&pose, &pose, c->W, c->H, &cam);
    fr_set_camera(c, &cam);
  }
  if (hipDeviceSynchronize() != hipSuccess) { c->err = "device sync failed"; return bail(FR_E_HIP); }
  *out = c;
  return FR_OK;
}

int fr_destroy(fr_ctx* c) {
  if (!c) return FR_E_INVALID;
  hipSetDevice(c->cfg.device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->stream2) hipStreamSynchronize(c->stream2);
  if (c->stream3) hipStreamSynchronize(c->stream3);
  if (c->stream4) hipStreamSynchronize(c->stream4);
  if (c->stream5) hipStreamSynchronize(c->stream5);
  auto fr = [](void* p) { if (p) hipFree(p); };
  fr(c->d_nodes); fr(c->d_tri); fr(c->d_prim); fr(c->d_shade); fr(c->d_pos);
  fr(c->spare_nodes); fr(c->spare_tri); fr(c->spare_prim);
  if (c->bvh_work) bvh_work_free(c->bvh_work);
  for (auto p : c->d_tex) fr(p);
  fr(c->d_mats); fr(c->d_texs);
  for (auto p : c->img) fr(p);
  for (int k = 0; k < fr_ctx::MAX_SLOTS; k++) { fr(c->mask_p[k]); fr(c->ray_count_p[k]); fr(c->active_p[k]); fr(c->owner_counts_p[k]); }
  fr(c->bcount); fr(c->shard_map); fr(c->front_need); fr(c->shade_radiance);
  if (c->h_counts) hipHostFree(c->h_counts);
  for (auto e : c->ev_counts) if (e) hipEventDestroy(e);
  fr(c->gclass); fr(c->lp_cache); fr(c->lp_inv); fr(c->words); fr(c->counts); fr(c->offsets); fr(c->tiles); fr(c->shade_ctr); fr(c->samples); fr(c->sample_help); fr(c->aux_p[0]); fr(c->aux_p[1]); fr(c->aux_seed_p[0]); fr(c->aux_seed_p[1]); fr(c->hvalid); fr(c->item_store); fr(c->jfa_a); fr(c->jfa_b); fr(c->ftab);
  fr(c->pull); fr(c->push); fr(c->snap); fr(c->stats); fr(c->sib_prefix); fr(c->sib_blocks); fr(c->sib_wide); fr(c->sib_strips); fr(c->sib_rowp);
  for (auto e : c->ev) if (e) hipEventDestroy(e);
  if (c->ev_front) hipEventDestroy(c->ev_front);
  for (auto e : c->ev_trace) if (e) hipEventDestroy(e);
  for (auto e : c->ev_recon) if (e) hipEventDestroy(e);
  for (auto e : c->ev_jfa) if (e) hipEventDestroy(e);
  for (auto& row : c->lat_ev) for (auto e : row) if (e) hipEventDestroy(e);
  for (auto& q : c->kt_ev)
    for (auto e : q) if (e) hipEventDestroy(e);
  for (auto& q : c->fc_ev)
    for (auto e : q) if (e) hipEventDestroy(e);
  if (c->fc_ref) hipEventDestroy(c->fc_ref);
  if (c->stream) hipStreamDestroy(c->stream);
  if (c->stream2) hipStreamDestroy(c->stream2);
  if (c->stream3) hipStreamDestroy(c->stream3);
  if (c->stream4) hipStreamDestroy(c->stream4);
  if (c->stream5) hipStreamDestroy(c->stream5);
  delete c;
  return FR_OK;
}

int fr_set_camera(fr_ctx* c, const fr_camera* cam) {
  if (!c || !cam) return FR_E_INVALID;
  FrameUniforms& U = c->U;
  memcpy(U.inv_vp.m, cam->inv_vp, sizeof(U.inv_vp.m));
  memcpy(U.prev_vp.m, cam->prev_vp, sizeof(U.prev_vp.m));
  U.eye = mk3(cam->eye[0], cam->eye[1], cam->eye[2]);
  U.prev_eye = mk3(cam->prev_eye[0], cam->prev_eye[1], cam->prev_eye[2]);
  if (!std::isfinite(cam->gaze[0]) || !std::isfinite(cam->gaze[1])) return fail(c, FR_E_INVALID, "fr_set_camera: gaze not finite");
  U.gaze = mk2(cam->gaze[0], cam->gaze[1]);
  return FR_OK;
}

int fr_set_light_power(fr_ctx* c, float power) {
  if (!c) return FR_E_INVALID;
  c->dsc.light_emission = mk3(power);
  c->light_pending = true;
  return FR_OK;
}

int fr_set_diffuse_max_depth(fr_ctx* c, int depth) {
  if (!c || depth < 0) return FR_E_INVALID;
  c->U.diffuse_max_depth = depth;
  return FR_OK;
}

int fr_reset_accumulation(fr_ctx* c) {
  if (!c) return FR_E_INVALID;
  c->accum = 0;
  return FR_OK;
}

int fr_accum_frame(fr_ctx* c, uint32_t* f) {
  if (!c || !f) return FR_E_INVALID;
  *f = c->accum;
  return FR_OK;
}

static int slotted(const fr_ctx* c, int p0, int pb) { return c->slot == 0 ? p0 : pb + 4 * (c->slot - 1); }
static int P_pos(const fr_ctx* c) { return slotted(c, P_POSITION, P_POSITION_B); }
static int P_nrm(const fr_ctx* c) { return slotted(c, P_NORMAL, P_NORMAL_B); }
static int P_shd(const fr_ctx* c) { return slotted(c, P_SHADING, P_SHADING_B); }
static int P_wgt(const fr_ctx* c) { return slotted(c, P_WEIGHT, P_WEIGHT_B); }

// The context stream waits for every reconstruction still in flight (before any call that reads or
// writes what the reconstruction uses, or hands buffers to the caller).
static void join_recon(fr_ctx* c) {
  c->stream_dirty = true;  // the caller is about to enqueue on `stream` outside a pipelined frame
  for (int k = 0; k < fr_ctx::MAX_SLOTS; k++)
    if (c->recon_pending[k]) { hipStreamWaitEvent(c->stream, c->ev_recon[k], 0); c->recon_pending[k] = false; }
  if (c->front_pending) { hipStreamWaitEvent(c->stream, c->ev_front, 0); c->front_pending = false; }
}

// fs: the stream of the front stages (entries 0-2): `stream`, or stream5 in a pipelined frame.
static int enqueue_geometry(fr_ctx* c, hipStream_t fs) {
  // a new frame: move to the next slot, once the reconstruction that read it has finished
  c->slot = (c->slot + 1) % c->nslots;
  c->setup_early = false;
  const int sl = c->slot;
  c->mask = c->mask_p[sl]; c->active = c->active_p[sl]; c->ray_count = c->ray_count_p[sl];
  if (c->recon_pending[sl]) {
    hipStreamWaitEvent(fs, c->ev_recon[sl], 0);  // entry 3 on `stream` waits for fs (ev_front)
    c->recon_pending[sl] = false;
  }
  if (fs != c->stream && c->trace_pending[sl]) {
    hipStreamWaitEvent(fs, c->ev_trace[sl], 0);
    c->trace_pending[sl] = false;
  }
  if (c->lat_arm) hipEventRecord(c->lat_ev[sl][0], fs);
  if (c->fc_arm) {  // fr_frame_clock: where this frame's G-buffer (the first stage to read the gaze) may start
    const int i = c->fc_next;
    if (c->fc_pending == fr_ctx::FC_RING) { fc_harvest(c, i); c->fc_pending--; }
    c->fc_cur = i;
    c->fc_next = (i + 1) % fr_ctx::FC_RING;
    c->fc_pending++;
    hipEventRecord(c->fc_ev[i][0], fs);
  }
  // frame = m_accumFrame++ ; a light change resets the counter afterwards (FR/PathTracer.cpp:99-116)
  c->U.frame = c->accum++;
  if (c->light_pending) { c->light_pending = false; c->accum = 0; }
  if (c->U.frame < 1) {  // d_buffer_init (g_buffer_trace_camera.cu:73-82)
    const size_t bytes = (size_t)c->W * c->H * sizeof(f4);
    hipMemsetAsync(c->img[c->hist_cur], 0, bytes, c->stream);
    hipMemsetAsync(c->img[c->hist_cache], 0, bytes, c->stream);
  }
  if (c->front_local) {  // the primaries this G-buffer traces: the needed tiles and the gaze pixel's
    const int t8 = gaze_tile8(c->U);
    const int tx8 = (c->W + 7) / 8;
    const uint32_t gw = (uint32_t)std::min(8, c->W - (t8 % tx8) * 8), gh = (uint32_t)std::min(8, c->H - (t8 / tx8) * 8);
    c->U.front_pixels = c->front_need_px + (c->front_need_h[t8] ? 0u : gw * gh);
  }
  launch_gbuffer(c->dsc, c->U, c->img[P_pos(c)], c->img[P_nrm(c)], c->img[c->depth_cur], c->img[P_DIFFUSE],
                 c->img[P_wgt(c)], c->gclass, c->stats, fs);
  c->compacted = false;
  return check_launch(c);
}

static int enqueue_sampling(fr_ctx* c, hipStream_t fs) {
  c->mask_dirty = false;
  const bool lp = c->U.mask_mode == FR_MASK_LOGPOLAR || c->U.mask_mode == FR_MASK_LOGPOLAR_SIGNED;
  const bool lp_refresh = lp && (c->lp_mode != c->U.mask_mode || c->lp_gaze.x != c->U.gaze.x ||
                                 c->lp_gaze.y != c->U.gaze.y);
  if (lp_refresh) { c->lp_mode = c->U.mask_mode; c->lp_gaze = c->U.gaze; }
  launch_sampling(c->U, c->dsc, c->img[P_pos(c)], c->img[c->depth_cur], c->img[c->depth_cache], c->img[P_wgt(c)],
                  c->img[P_nrm(c)], c->img[P_DIFFUSE], c->img[P_EXTRA], c->mask, c->gclass, c->words, c->counts,
                  c->cfg.write_extra, c->lp_cache, c->lp_inv, lp_refresh, c->U.shard_count > 1 ? c->bcount : nullptr, fs);
  if (c->U.shard_count > 1) {
    // every rank's active count of this frame (fr_shard_counts, the group's transfer sizes), to pinned
    // host memory with its own event: reading it waits for this frame's front stages only
    launch_owner_counts(c->U, c->bcount, c->owner_counts_p[c->slot], fs);
    hipMemcpyAsync(c->h_counts + (size_t)c->slot * FR_MAX_SHARD_RANKS, c->owner_counts_p[c->slot],
                   sizeof(uint32_t) * FR_MAX_SHARD_RANKS, hipMemcpyDeviceToHost, fs);
    hipEventRecord(c->ev_counts[c->slot], fs);
    c->counts_valid[c->slot] = true;
  }
  c->compacted = false;
  return check_launch(c);
}

static int enqueue_optimize(fr_ctx* c, hipStream_t fs) {
  if (c->mask_dirty) {
    launch_mask_words(c->mask, c->gclass, c->W, c->H, c->words, c->counts, fs);
    c->mask_dirty = false;
  }
  launch_compaction(c->W, c->H, c->words, c->counts, c->offsets, c->tiles, c->ray_count, c->active, fs);
  c->compacted = true;
  return check_launch(c);
}

static int enqueue_shading(fr_ctx* c) {
  if (!c->compacted) {  // g_isOptimize = 0: the active list is still needed by this design
    int rc = enqueue_optimize(c, c->stream);
    if (rc) return rc;
  }
  if (c->front_pending) {  // a pipelined frame: entry 3 waits for its own front stages
    hipStreamWaitEvent(c->stream, c->ev_front, 0);
    c->front_pending = false;
  }
  hipEvent_t* kt = nullptr;
  if (c->kt_on) {
    const int i = c->kt_next;
    if (c->kt_pending == fr_ctx::KT_RING) { kt_harvest(c, i); c->kt_pending--; }
    kt = c->kt_ev[i];
    c->kt_next = (i + 1) % fr_ctx::KT_RING;
    c->kt_pending++;
    hipEventRecord(kt[0], c->stream);
  }
  // this frame's sample setup: enqueued by its front stages into the other aux buffer (frame_half), or here
  if (c->setup_early) {
    c->aux_i ^= 1;
    c->aux = c->aux_p[c->aux_i];
    c->aux_seed = c->aux_seed_p[c->aux_i];
  }
  const bool early = c->setup_early;
  c->setup_early = false;
  // The inactive pixels' history carry (HBM-bound) touches no buffer k_shade_paths reads or writes:
  // it runs on stream4 beside the latency-bound megakernel and joins before the resolve. In latency mode, with one
  // untiled view, it also writes the validity bits of the history this frame leaves (the next frame's early setup).
  const bool hv = c->pipeline_mode == FR_PIPELINE_LATENCY && c->early_setup && c->U.shard_count <= 1 && !c->U.front_need;
  hipEventRecord(c->ev[11], c->stream);
  hipStreamWaitEvent(c->stream4, c->ev[11], 0);
  launch_carry_history(c->U, c->mask, c->img[P_wgt(c)], c->img[c->hist_cache], c->img[c->hist_cur],
                       c->img[P_shd(c)], hv ? c->hvalid : nullptr, c->stream4);
  hipEventRecord(c->ev[12], c->stream4);
  const uint32_t N = (uint32_t)((size_t)c->W * c->H);
  if (!early)
    launch_sample_setup(c->U, c->active, c->ray_count, N, c->img[P_wgt(c)], c->img[c->hist_cache], nullptr, c->aux,
                        c->aux_seed, c->stream);
  if (c->time_kernels) hipEventRecord(c->ev[9], c->stream);
  if (kt) hipEventRecord(kt[1], c->stream);
  launch_shade_paths(c->dsc, c->U, c->active, c->ray_count, N, c->img[P_wgt(c)], c->img[c->hist_cache],
                     c->shade_ctr, c->samples, c->sample_help, c->stats, c->aux, c->aux_seed, c->chunk_refr,
                     c->xcd_bands, c->handoff, c->item_store, c->stream);
  if (c->time_kernels) hipEventRecord(c->ev[10], c->stream);
  if (kt) hipEventRecord(kt[2], c->stream);
  hipStreamWaitEvent(c->stream, c->ev[12], 0);
  launch_shade_resolve(c->U, c->active, c->ray_count, N, c->img[P_wgt(c)], c->img[c->hist_cache], c->samples,
                       c->sample_help, c->img[c->hist_cur], c->img[P_shd(c)], c->shade_ctr, c->handoff,
                       c->U.shard_count > 1 ? c->shade_radiance : nullptr, c->stream);
  if (kt) hipEventRecord(kt[3], c->stream);
  // this slot's WEIGHT / mask / active list are free for the front stages of frame + nslots after this
  hipEventRecord(c->ev_trace[c->slot], c->stream);
  c->trace_pending[c->slot] = true;
  int rc = check_launch(c);
  // swapBuffer("history_cache", "history_buffer"); swapBuffer("depth_cache", "depth_buffer") (:226-227)
  std::swap(c->hist_cur, c->hist_cache);
  c->hvalid_fresh = hv;
  std::swap(c->depth_cur, c->depth_cache);
  return rc;
}

// JFA_COORD owed by the last JumpFlooding (launch_jfa with outputs = false), written on `s`, which the caller has
// ordered after that JumpFlooding (from its final state and JFA_COLOR: nothing but the next JumpFlooding or a write of
// JFA_COLOR changes those).
static void materialize_jfa(fr_ctx* c, hipStream_t s) {
  if (!c->jfa_coord_owed) return;
  launch_jfa_coord(c->jfa_final, c->img[P_JFA_COLOR], c->img[P_JFA_COORD], c->W, c->H, s);
  c->jfa_coord_owed = false;
}
static void join_recon(fr_ctx* c);
// the same from an ABI call (on the context stream, after the pending reconstruction)
static void materialize_jfa_now(fr_ctx* c) {
  if (!c->jfa_coord_owed) return;
  join_recon(c);
  materialize_jfa(c, c->stream);
}

static int resolve(fr_ctx* c, int id, int* phys) {
  // JFA_COORD read by a caller or a pass outside the frame chain, or JFA_COLOR about to be written: JFA_COORD is
  // written first when owed
  if (id == FR_BUF_JFA_COORD || id == FR_BUF_JFA_COLOR) materialize_jfa_now(c);
  switch (id) {
    case FR_BUF_POSITION: *phys = P_pos(c); return FR_OK;
    case FR_BUF_NORMAL: *phys = P_nrm(c); return FR_OK;
    case FR_BUF_DEPTH: *phys = c->depth_cur; return FR_OK;
    case FR_BUF_DEPTH_CACHE: *phys = c->depth_cache; return FR_OK;
    case FR_BUF_DIFFUSE: *phys = P_DIFFUSE; return FR_OK;
    case FR_BUF_WEIGHT: *phys = P_wgt(c); return FR_OK;
    case FR_BUF_HISTORY: *phys = c->hist_cur; return FR_OK;
    case FR_BUF_HISTORY_CACHE: *phys = c->hist_cache; return FR_OK;
    case FR_BUF_SHADING: *phys = P_shd(c); return FR_OK;
    case FR_BUF_EXTRA: *phys = P_EXTRA; return FR_OK;
    case FR_BUF_JFA_COORD: *phys = P_JFA_COORD; return FR_OK;
    case FR_BUF_JFA_COLOR: *phys = P_JFA_COLOR; return FR_OK;
    case FR_BUF_SIBSON: *phys = P_SIBSON; return FR_OK;
    case FR_BUF_PULLPUSH: *phys = P_PULLPUSH; return FR_OK;
    case FR_BUF_ATROUS: *phys = c->atrous_out; return FR_OK;
    case FR_BUF_LOGPOLAR: *phys = P_LOGPOLAR; return FR_OK;
    case FR_BUF_LOGPOLAR_INVERSE: *phys = P_LOGPOLAR_INV; return FR_OK;
    default: return FR_E_INVALID;
  }
}

// JFA_COORD is written only when something asks for it (materialize_jfa: a caller's read, copy or view of a JFA
// output, a pass reading one, a write of JFA_COLOR). Sibson's run form takes the seeds from the final state and a frame
// reads nothing else of it: 133 MB less per 4K frame. (FOVRT_JFA_LAZY_OUTPUTS=0: always written.)
static int enqueue_jfa(fr_ctx* c, int in_buffer, hipStream_t stream = nullptr) {
  int p;
  if (resolve(c, in_buffer, &p)) return fail(c, FR_E_INVALID, "jfa: bad input buffer");
  const bool run_form = c->cfg.sibson_mode == 0;
  const bool lazy = run_form && c->lazy_jfa_outputs;
  c->jfa_final = launch_jfa(c->img[p], c->jfa_a, c->jfa_b, c->img[P_JFA_COORD], c->img[P_JFA_COLOR], c->ftab, c->W,
                            c->H, run_form ? c->sib_prefix : nullptr, run_form ? c->sib_blocks : nullptr, !lazy,
                            stream ? stream : c->stream);
  c->jfa_coord_owed = lazy;
  c->sib_prefix_fresh = run_form;
  return check_launch(c);
}
static int enqueue_sibson(fr_ctx* c, hipStream_t stream = nullptr) {
  if (c->cfg.sibson_mode == 1) {  // per tap, bit-exact against the oracle (reads JFA_COORD)
    materialize_jfa(c, stream ? stream : c->stream);
    launch_sibson(c->img[P_JFA_COORD], c->img[P_JFA_COLOR], c->img[P_SIBSON], c->W, c->H, stream ? stream : c->stream);
  } else {  // run form (default): exact tap sets, rounding-level differences
    launch_sibson_runs(c->img[P_JFA_COORD], c->jfa_final, c->img[P_JFA_COLOR], c->sib_prefix, c->sib_blocks, c->sib_rowp, c->sib_wide,
                       c->sib_strips, c->img[P_SIBSON], c->W, c->H, c->sib_prefix_fresh, c->sib_strip, c->jfa_coord_owed,
                       stream ? stream : c->stream);
  }
  return check_launch(c);
}
static int enqueue_pullpush(fr_ctx* c, int in_buffer, hipStream_t stream = nullptr) {
  int p;
  if (resolve(c, in_buffer, &p)) return fail(c, FR_E_INVALID, "pullpush: bad input buffer");
  launch_pullpush(c->img[p], c->pull, c->push, c->snap, c->img[P_PULLPUSH], c->W, c->H, stream ? stream : c->stream);
  return check_launch(c);
}
static int enqueue_atrous(fr_ctx* c, int count, int pos, int nrm, int col, hipStream_t stream = nullptr) {
  if (!stream) stream = c->stream;
  int pp, pn, pc;
  if (count < 1 || resolve(c, pos, &pp) || resolve(c, nrm, &pn) || resolve(c, col, &pc))
    return fail(c, FR_E_INVALID, "atrous: bad arguments");
  if (pc == P_ATROUS_A || pc == P_ATROUS_B) return fail(c, FR_E_INVALID, "atrous: colour input aliases the output");
  float c_phi = 1.f, n_phi = 1.f, p_phi = 1.f;
  int sw = 1;
  launch_atrous(c->img[pp], c->img[pn], c->img[pc], c->img[P_ATROUS_A], c->W, c->H, c_phi, n_phi, p_phi, (float)sw, stream);
  bool usingA = true;
  for (int k = 1; k < count; k++) {  // FR/ATrous.cpp:90-113
    c_phi *= 1.0f; n_phi *= 0.5f; p_phi *= 1.0f; sw *= 2;
    if (usingA) launch_atrous(c->img[pp], c->img[pn], c->img[P_ATROUS_A], c->img[P_ATROUS_B], c->W, c->H, c_phi, n_phi, p_phi, (float)sw, stream);
    else launch_atrous(c->img[pp], c->img[pn], c->img[P_ATROUS_B], c->img[P_ATROUS_A], c->W, c->H, c_phi, n_phi, p_phi, (float)sw, stream);
    usingA = !usingA;
  }
  c->atrous_out = usingA ? P_ATROUS_A : P_ATROUS_B;
  return check_launch(c);
}

static int timed(fr_ctx* c, const std::function<int()>& f, float* ms) {
  hipSetDevice(c->cfg.device);
  join_recon(c);
  hipEventRecord(c->ev[0], c->stream);
  int rc = f();
  if (rc) return rc;
  hipEventRecord(c->ev[1], c->stream);
  hipError_t e = hipEventSynchronize(c->ev[1]);
  if (e != hipSuccess) return fail(c, FR_E_HIP, std::string("stage failed: ") + hipGetErrorString(e));
  if (ms) *ms = elapsed(c->ev[0], c->ev[1]);
  return FR_OK;
}

int fr_geometry_launch(fr_ctx* c, float* ms) { if (!c) return FR_E_INVALID; return timed(c, [&] { return enqueue_geometry(c, c->stream); }, ms); }
int fr_sampling_launch(fr_ctx* c, float* ms) { if (!c) return FR_E_INVALID; return timed(c, [&] { return enqueue_sampling(c, c->stream); }, ms); }
int fr_optimize_launch(fr_ctx* c, float* ms) { if (!c) return FR_E_INVALID; return timed(c, [&] { return enqueue_optimize(c, c->stream); }, ms); }
int fr_shading_launch(fr_ctx* c, float* ms) { if (!c) return FR_E_INVALID; return timed(c, [&] { return enqueue_shading(c); }, ms); }

static int ns_timed(fr_ctx* c, std::function<int()> f, uint64_t* ns) {
  float ms = 0;
  int rc = timed(c, f, &ms);
  if (ns) *ns = (uint64_t)((double)ms * 1e6);
  return rc;
}
int fr_jfa_render(fr_ctx* c, int in_buffer, uint64_t* ns) { if (!c) return FR_E_INVALID; return ns_timed(c, [&] { return enqueue_jfa(c, in_buffer); }, ns); }
int fr_sibson_render(fr_ctx* c, uint64_t* ns) { if (!c) return FR_E_INVALID; return ns_timed(c, [&] { return enqueue_sibson(c); }, ns); }
int fr_pullpush_render(fr_ctx* c, int in_buffer, uint64_t* ns) { if (!c) return FR_E_INVALID; return ns_timed(c, [&] { return enqueue_pullpush(c, in_buffer); }, ns); }
static int enqueue_logpolar(fr_ctx* c, int in_buffer) {
  int p;
  if (resolve(c, in_buffer, &p)) return fail(c, FR_E_INVALID, "logpolar: bad input buffer");
  if (p == P_LOGPOLAR || p == P_LOGPOLAR_INV) return fail(c, FR_E_INVALID, "logpolar: input is one of its outputs");
  launch_logpolar(c->img[p], c->img[P_LOGPOLAR], c->img[P_LOGPOLAR_INV], c->W, c->H, c->U.gaze, c->stream);
  return check_launch(c);
}
int fr_logpolar_render(fr_ctx* c, int in_buffer, uint64_t* ns) {
  if (!c) return FR_E_INVALID;
  return ns_timed(c, [&] { return enqueue_logpolar(c, in_buffer); }, ns);
}

static int buffer_view(fr_ctx* c, int id, fr_buffer_view* v);
int fr_copy_buffer(fr_ctx* c, int id, void* dst, size_t bytes) {
  fr_buffer_view v;
  int rc = buffer_view(c, id, &v);
  if (rc) return rc;
  if (!dst || bytes > v.bytes) return fail(c, FR_E_INVALID, "copy_buffer: size");
  hipSetDevice(c->cfg.device);
  HIP_TRY(c, hipMemcpyAsync(dst, v.device_ptr, bytes, hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}

int fr_composite_views(fr_ctx* c, const void* views, int nviews, void* out, size_t out_bytes) {
  if (!c || !views || !out || nviews < 1) return FR_E_INVALID;
  const size_t need = (size_t)nviews * c->W * c->H * sizeof(f4);
  if (out_bytes < need) return fail(c, FR_E_INVALID, "fr_composite_views: output smaller than nviews * W * H * 16");
  join_recon(c);
  hipSetDevice(c->cfg.device);
  launch_composite((const f4*)views, nviews, c->W, c->H, (f4*)out, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}

// g_gaze is a Win32 POINT (LONG x, y; FR/gui.h:14) and the cursor a double: the assignment truncates
// toward zero (clamped to the LONG range here, where C++ leaves it undefined)
static long to_long(double v) { return (long)std::max(-2147483648.0, std::min(2147483647.0, std::trunc(v))); }
static void set_g_gaze(fr_ctx* c, long gx, long gy) {
  // m_context["gaze"] = (float(g_gaze.x), float(g_screenSize.cy - g_gaze.y)) (FR/PathTracer.cpp:795); off-window
  // cursors are kept as given (the log-polar mask and the gaze distance are defined for any gaze); the two
  // texel reads at the gaze clamp to the screen (k_sampling, fr_gaze_target)
  c->U.gaze = mk2((float)gx, (float)((long)c->H - gy));
}
int fr_set_gaze(fr_ctx* c, double xpos, double ypos, int fullscreen) {
  // cursorPosCallback (FR/gui.cpp:48-66): adjust_scale = g_fullScreen ? 1 : 1.25 (:51-56);
  // g_gaze.x = xpos; g_gaze.y = ypos * adjust_scale (:65-66, and :59-60 on the first call)
  if (!c || !std::isfinite(xpos) || !std::isfinite(ypos)) return FR_E_INVALID;
  const float adjust_scale = fullscreen ? 1.0f : 1.25f;
  set_g_gaze(c, to_long(xpos), to_long(ypos * adjust_scale));
  return FR_OK;
}
int fr_reset_gaze(fr_ctx* c) {
  // framebufferSizeCallback (FR/gui.cpp:32-35): g_gaze = (w / 2, h / 2), integer division
  if (!c) return FR_E_INVALID;
  set_g_gaze(c, c->W / 2, c->H / 2);
  return FR_OK;
}

int fr_atrous_render(fr_ctx* c, int count, int pos, int nrm, int col, uint64_t* ns) {
  if (!c) return FR_E_INVALID;
  return ns_timed(c, [&] { return enqueue_atrous(c, count, pos, nrm, col); }, ns);
}

// Frame halves: the trace half (update -> entries 0..3) and the reconstruction half (JFA -> SI ->
// PPI -> AT). fr_frame runs both; a tile-sharded view runs the trace half on every rank and the
// reconstruction half on the rank that composites (after fr_shard_unpack of the other ranks' tiles).
static int frame_half(fr_ctx* c, fr_frame_timing* t, bool trace, bool recon) {
  if (!c) return FR_E_INVALID;
  hipSetDevice(c->cfg.device);
  hipEvent_t* ev = c->ev;
  int rc;
  // fr_frame_clock: a frame that fails after enqueue_geometry reserved its ring entry gives the entry
  // back (it would never get its end event)
  struct FcGuard {
    fr_ctx* c;
    ~FcGuard() {
      if (c->fc_cur < 0) return;
      c->fc_next = c->fc_cur;
      c->fc_pending--;
      c->fc_cur = -1;
    }
  } fc_guard{c};
  if (t) hipEventRecord(ev[0], c->stream);
  if (trace) {
    // untimed frames pipeline: the front stages go to stream5 and overlap the previous frame's
    // entry 3 (timed frames keep every stage on `stream`, one after the other)
    hipStream_t fs = t ? c->stream : c->stream5;
    const bool latency = !t && c->pipeline_mode == FR_PIPELINE_LATENCY;
    const int prev = c->slot;  // the previous frame's slot
    if (latency && (c->jfa_pending[prev] || c->trace_pending[prev])) {
      // one frame ahead at most: the host waits until the previous frame's JumpFlooding has ended (its
      // path trace, when this context does not run that chain), then samples the gaze and enqueues this
      // frame, whose front stages (G-buffer, sampling, compaction) overlap the previous frame's Sibson
      // and pull-push -> A-Trous; its path trace starts after them (below)
      // (polled: a blocking wait woke the host up to milliseconds late, and the GPU idled meanwhile)
      hipEvent_t w = c->jfa_pending[prev] ? c->ev_jfa[prev] : c->ev_trace[prev];
      hipError_t e;
      if ((e = poll_event(w, kPollDeadlineMs)) != hipSuccess)
        return fail(c, FR_E_HIP, e == hipErrorNotReady ? std::string("frame failed: the previous frame did not complete within the poll deadline")
                                                        : std::string("frame failed: ") + hipGetErrorString(e));
      // Just in time: the front stages should end about when the previous frame's Sibson does (its path
      // trace waits for both). A completed frame's times estimate the two; when its Sibson took longer than
      // half its front stages, the host waits the difference more (an eye-tracked gaze's big discs: 2-5 ms of
      // Sibson against ~1.3 ms of front stages), so the gaze is sampled that much later.
      for (int k = 0; k < c->nslots; k++) {
        if (!c->lat_rec[k] || hipEventQuery(c->lat_ev[k][3]) != hipSuccess) continue;
        float f = 0.0f, sb = 0.0f;
        if (hipEventElapsedTime(&f, c->lat_ev[k][0], c->lat_ev[k][1]) == hipSuccess &&
            hipEventElapsedTime(&sb, c->lat_ev[k][2], c->lat_ev[k][3]) == hipSuccess) {
          // The front stages' span is the smallest of the last eight: a front stage that overlapped the
          // previous Sibson ran slower, and estimating from it started the next front stages earlier still (into
          // more of that Sibson: a feedback that held the eye-tracked circle's fronts at ~4 ms instead of ~1)
          c->lat_front_hist[c->lat_front_n++ & 7] = f;
          c->lat_front_ms = f;
          for (int j = 1; j < std::min(8, c->lat_front_n); j++)
            c->lat_front_ms = std::min(c->lat_front_ms, c->lat_front_hist[(c->lat_front_n - 1 - j) & 7]);
          c->lat_sib_ms = sb;
        }
        c->lat_rec[k] = false;
      }
      // Only half of the front stages' span is overlapped: the big discs' strip kernel fills every CU, and a
      // front stage started further into it ran ~4 ms instead of ~1, with its gaze sampled that much earlier
      // (eye-tracked circle latency p99 16.2 -> 12.6 ms at 142 fps; C3 p50 6.15 -> 5.81 ms; overlapping none:
      // p99 12.5 ms at 139 fps, the serial loop's rate). A short Sibson (no big discs: below kLatShortSibMs) takes the
      // whole span: the front stages then end with it without slowing down (4K bunny centred 186.0 -> 189.3 fps at
      // latency p50 5.72 -> 5.79 ms, 4K vokselia 233.1 -> 235.2 fps; profiles/r06_lat_overlap_*). FOVRT_LAT_OVERLAP:
      // one percentage for every frame instead (A/B knob).
      constexpr float kLatShortSibMs = 1.5f;
      static const float ovl_env = [] { const char* v = getenv("FOVRT_LAT_OVERLAP"); return v ? atoi(v) / 100.0f : -1.0f; }();
      const float ovl = ovl_env >= 0.0f ? ovl_env : c->lat_sib_ms < kLatShortSibMs ? 1.0f : 0.5f;
      const float delay_ms = c->jfa_pending[prev] ? c->lat_sib_ms - ovl * c->lat_front_ms : 0.0f;
      if (delay_ms > 0.05f) {
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count() < delay_ms &&
               hipEventQuery(c->ev_recon[prev]) == hipErrorNotReady) {
          cpu_relax();
        }
      }
      c->jfa_pending[prev] = false;
    }
    if (!t && c->stream_dirty) {
      // the front stages overwrite buffers (gclass, DIFFUSE, EXTRA, depth, ballots, counts, lp_cache) that
      // work enqueued on `stream` by other calls may still read: order them after it explicitly
      hipEventRecord(c->ev[18], c->stream);
      hipStreamWaitEvent(fs, c->ev[18], 0);
    }
    c->stream_dirty = false;
    c->fc_arm = c->fc_on && recon;  // whole frames only (a group's trace half has no end of its own)
    c->lat_arm = latency && recon;
    rc = enqueue_geometry(c, fs);
    c->fc_arm = false;
    if (rc) { c->lat_arm = false; return rc; }
    if (t) hipEventRecord(ev[1], c->stream);
    if ((rc = enqueue_sampling(c, fs))) return rc;
    if (t) hipEventRecord(ev[2], c->stream);
    if ((rc = enqueue_optimize(c, fs))) return rc;
    if (t) hipEventRecord(ev[3], c->stream);
    if (latency && fs != c->stream && c->hvalid_fresh && c->U.shard_count <= 1 && !c->U.front_need && c->early_setup) {
      // Early sample setup (latency mode): from the validity bits of the previous frame's history (its carry, ev[12])
      // instead of the history itself, so it runs here with the front stages, and this frame's megakernel starts as
      // soon as the previous frame's reconstruction ends (the setup sat between them on the context stream, ~0.1 ms
      // on the CUs the reconstruction had just filled). Into the aux buffer the previous megakernel does not read.
      // (Throughput mode keeps the setup after the resolve: there the megakernel then started beside the previous
      // frame's reconstruction burst and ran 3.9 -> 4.1 ms, 240 -> 232 fps; profiles/r06_early_setup_ab.txt.)
      hipStreamWaitEvent(fs, c->ev[12], 0);
      const int o = c->aux_i ^ 1;
      launch_sample_setup(c->U, c->active, c->ray_count, (uint32_t)((size_t)c->W * c->H), c->img[P_wgt(c)], nullptr,
                          c->hvalid, c->aux_p[o], c->aux_seed_p[o], fs);
      if ((rc = check_launch(c))) return rc;
      c->setup_early = true;
    }
    if (!t) {
      hipEventRecord(c->ev_front, fs);
      c->front_pending = true;
    }
    if (c->lat_arm) hipEventRecord(c->lat_ev[c->slot][1], fs);
    // latency mode: this frame's path trace starts after the previous frame's reconstruction. The
    // megakernel fills every CU, so a reconstruction running beside it waited for it to end and then
    // delayed this frame's own reconstruction (pipelined latency p50 10-12 ms against a 5.6 ms frame).
    if (latency && c->recon_pending[prev]) hipStreamWaitEvent(c->stream, c->ev_recon[prev], 0);
    c->time_kernels = t != nullptr;
    rc = enqueue_shading(c);
    c->time_kernels = false;
    if (rc) return rc;
  } else if (t) {
    for (int i = 1; i <= 3; i++) hipEventRecord(ev[i], c->stream);
    hipEventRecord(ev[9], c->stream);
    hipEventRecord(ev[10], c->stream);
  }
  if (t) hipEventRecord(ev[4], c->stream);
  if (recon) {
    // The reconstruction of this frame's shading runs on its own streams, so the next frame's trace
    // half (on `stream`) overlaps it. Two independent chains read the shading: JFA -> Sibson
    // (stream3) and pull-push -> A-Trous (stream2; atFS binds the JFA texture but never reads it,
    // FR/shader/atFS.glsl:40-90). Both resolve their inputs now, at this frame's slot.
    // (a group's reconstruction rank may run only one of the chains: c->recon_chains)
    hipEventRecord(ev[16], c->stream);
    hipStreamWaitEvent(c->stream3, ev[16], 0);
    hipStreamWaitEvent(c->stream2, ev[16], 0);
    if (t) hipEventRecord(ev[20], c->stream3);
    if ((c->recon_chains & 1) && (rc = enqueue_jfa(c, FR_BUF_SHADING, c->stream3))) return rc;
    if (t) hipEventRecord(ev[21], c->stream3);
    if (c->pipeline_mode == FR_PIPELINE_LATENCY && (c->recon_chains & 1)) {
      hipEventRecord(c->ev_jfa[c->slot], c->stream3);
      c->jfa_pending[c->slot] = true;
      if (c->lat_arm) hipEventRecord(c->lat_ev[c->slot][2], c->stream3);
    }
    if ((c->recon_chains & 1) && (rc = enqueue_sibson(c, c->stream3))) return rc;
    if (t) hipEventRecord(ev[22], c->stream3);
    if (c->recon_gate) hipStreamWaitEvent(c->stream2, c->recon_gate, 0);
    if (t) hipEventRecord(ev[13], c->stream2);
    if ((c->recon_chains & 2) && (rc = enqueue_pullpush(c, FR_BUF_SHADING, c->stream2))) return rc;
    if (t) hipEventRecord(ev[14], c->stream2);
    if ((c->recon_chains & 2) && (rc = enqueue_atrous(c, c->cfg.atrous_iterations, FR_BUF_POSITION, FR_BUF_NORMAL,
                                                      FR_BUF_PULLPUSH, c->stream2))) return rc;
    if (t) hipEventRecord(ev[15], c->stream2);
    hipEventRecord(ev[17], c->stream2);
    hipStreamWaitEvent(c->stream3, ev[17], 0);
    hipEventRecord(c->ev_recon[c->slot], c->stream3);  // this slot's buffers are free again after this
    c->recon_pending[c->slot] = true;
    if (c->lat_arm && (c->recon_chains & 1)) {
      hipEventRecord(c->lat_ev[c->slot][3], c->stream3);
      c->lat_rec[c->slot] = true;
    }
    c->lat_arm = false;
    if (c->fc_cur >= 0) {  // fr_frame_clock: both chains of this frame are done
      hipEventRecord(c->fc_ev[c->fc_cur][1], c->stream3);
      c->fc_cur = -1;
    }
    if (t) join_recon(c);
  }
  if (t) {
    hipEventRecord(ev[8], c->stream);
    hipError_t e = hipEventSynchronize(ev[8]);
    if (e != hipSuccess) return fail(c, FR_E_HIP, std::string("frame failed: ") + hipGetErrorString(e));
    t->geometry_ms = elapsed(ev[0], ev[1]);
    t->sampling_ms = elapsed(ev[1], ev[2]);
    t->optimize_ms = elapsed(ev[2], ev[3]);
    t->shading_ms = elapsed(ev[3], ev[4]);
    t->jfa_ms = recon ? elapsed(ev[20], ev[21]) : 0.0f;
    t->sibson_ms = recon ? elapsed(ev[21], ev[22]) : 0.0f;
    t->pullpush_ms = recon ? elapsed(ev[13], ev[14]) : 0.0f;
    t->atrous_ms = recon ? elapsed(ev[14], ev[15]) : 0.0f;
    t->total_ms = elapsed(ev[0], ev[8]);
    t->shade_paths_ms = elapsed(ev[9], ev[10]);
    hipMemcpy(&t->ray_count, c->ray_count, 4, hipMemcpyDeviceToHost);
  }
  return FR_OK;
}

int fr_frame(fr_ctx* c, fr_frame_timing* t) { return frame_half(c, t, true, true); }
int fr_set_pipeline_mode(fr_ctx* c, int mode) {
  if (!c) return FR_E_INVALID;
  if (mode != FR_PIPELINE_THROUGHPUT && mode != FR_PIPELINE_LATENCY)
    return fail(c, FR_E_INVALID, "fr_set_pipeline_mode: FR_PIPELINE_THROUGHPUT (0) or FR_PIPELINE_LATENCY (1)");
  c->pipeline_mode = mode;
  return FR_OK;
}
int fr_set_sample_sum(fr_ctx* c, int mode) {
  if (!c) return FR_E_INVALID;
  if (mode < 0 || mode > 2) return fail(c, FR_E_INVALID, "fr_set_sample_sum: mode 0 (fp32), 1 (by frame size) or 2 (fixed point)");
  if ((uint32_t)mode == c->handoff) return FR_OK;
  join_recon(c);
  hipSetDevice(c->cfg.device);
  HIP_TRY(c, hipDeviceSynchronize());
  // the fixed-point form keeps 32-B sample records and a 32-B help record per sample
  const size_t N = (size_t)c->W * c->H;
  const size_t need_s = std::max(N * c->cfg.spp, 2 * shade_fx_slots((uint32_t)N, c->cfg.spp, (uint32_t)mode));
  const size_t need_h = std::max<size_t>(4 * shade_fx_slots((uint32_t)N, c->cfg.spp, (uint32_t)mode), 1);
  const size_t have_s = std::max(N * c->cfg.spp, 2 * shade_fx_slots((uint32_t)N, c->cfg.spp, c->handoff));
  const size_t have_h = std::max<size_t>(4 * shade_fx_slots((uint32_t)N, c->cfg.spp, c->handoff), 1);
  if (need_s > have_s) {
    hipFree(c->samples); c->samples = nullptr;
    if (dalloc(&c->samples, need_s) != hipSuccess) return fail(c, FR_E_NOMEM, "fr_set_sample_sum: allocation failed");
  }
  if (need_h > have_h) {
    hipFree(c->sample_help); c->sample_help = nullptr;
    if (dalloc(&c->sample_help, need_h) != hipSuccess) return fail(c, FR_E_NOMEM, "fr_set_sample_sum: allocation failed");
  }
  c->handoff = (uint32_t)mode;
  return FR_OK;
}

int fr_shard_unpack_active_enqueue(fr_ctx* c, const void* slab, size_t slab_bytes, uint32_t capacity, uint32_t count) {
  if (!c || !slab) return FR_E_INVALID;
  if (count > capacity) return fail(c, FR_E_INVALID, "fr_shard_unpack_active: count above capacity");
  if (slab_bytes < (size_t)capacity * 20) return fail(c, FR_E_INVALID, "fr_shard_unpack_active: slab smaller than 20 * capacity");
  hipSetDevice(c->cfg.device);
  const f4* vals = (const f4*)slab;
  const uint32_t* idx = (const uint32_t*)((const char*)slab + (size_t)capacity * sizeof(f4));
  launch_shard_unpack_active(c->U, vals, idx, count, (uint32_t)((size_t)c->W * c->H), c->img[P_wgt(c)],
                             c->img[c->hist_cur], c->img[c->hist_cache], c->img[P_shd(c)], c->stream);
  c->hvalid_fresh = false;
  // the unpack reads the slot's WEIGHT: the front stages of frame + nslots (stream5 waits for ev_trace[slot])
  // may overwrite it only after this launch
  hipEventRecord(c->ev_trace[c->slot], c->stream);
  c->trace_pending[c->slot] = true;
  return check_launch(c);
}

int fr_set_recon_chains(fr_ctx* c, int chains) {
  if (!c) return FR_E_INVALID;
  if (chains < 0 || chains > 3) return fail(c, FR_E_INVALID, "fr_set_recon_chains: chains is a mask of bits 0 and 1");
  c->recon_chains = chains;
  return FR_OK;
}
int fr_trace_frame(fr_ctx* c, fr_frame_timing* t) { return frame_half(c, t, true, false); }
int fr_reconstruct_frame(fr_ctx* c, fr_frame_timing* t) { return frame_half(c, t, false, true); }

int fr_shard_plan(int W, int H, int tile, int count, const float* weights, uint8_t* owner, size_t ntiles) {
  if (W <= 0 || H <= 0 || tile < 16 || tile % 16 || count < 1 || count > FR_MAX_SHARD_RANKS || !owner)
    return fail(nullptr, FR_E_INVALID, "fr_shard_plan: need W, H > 0, tile a multiple of 16, 1 <= count <= 64");
  const size_t nt = (size_t)((W + tile - 1) / tile) * ((H + tile - 1) / tile);
  if (ntiles != nt) return fail(nullptr, FR_E_INVALID, "fr_shard_plan: ntiles != ceil(W/tile) * ceil(H/tile)");
  std::vector<double> w(count, 1.0);
  double sum = count;
  if (weights) {
    sum = 0.0;
    for (int r = 0; r < count; r++) {
      if (!(weights[r] >= 0.0f) || !std::isfinite(weights[r])) return fail(nullptr, FR_E_INVALID, "fr_shard_plan: bad weight");
      w[r] = weights[r];
      sum += w[r];
    }
    if (sum <= 0.0) return fail(nullptr, FR_E_INVALID, "fr_shard_plan: all weights are 0");
  }
  // smooth weighted round robin (raster order): every step each rank earns its weight, the richest
  // rank (lowest rank on ties) takes the tile and pays the total
  std::vector<double> cur(count, 0.0);
  for (size_t t = 0; t < nt; t++) {
    int best = -1;
    for (int r = 0; r < count; r++) {
      if (w[r] <= 0.0) continue;
      cur[r] += w[r];
      if (best < 0 || cur[r] > cur[best]) best = r;
    }
    cur[best] -= sum;
    owner[t] = (uint8_t)best;
  }
  return FR_OK;
}

static int update_front_need(fr_ctx* c);

int fr_set_shard_plan(fr_ctx* c, int rank, int count, int tile, const uint8_t* owner, size_t ntiles) {
  if (!c) return FR_E_INVALID;
  if (count < 1 || count > FR_MAX_SHARD_RANKS || rank < 0 || rank >= count || tile < 16 || tile % 16 || tile > 4096)
    return fail(c, FR_E_INVALID, "fr_set_shard: need 0 <= rank < count <= 64 and tile a multiple of 16 in 16..4096");
  const int tx = (c->W + tile - 1) / tile, ty = (c->H + tile - 1) / tile;
  const size_t nt = (size_t)tx * ty;
  if (count > 1 && (!owner || ntiles != nt))
    return fail(c, FR_E_INVALID, "fr_set_shard_plan: owner must hold ceil(W/tile) * ceil(H/tile) entries");
  std::vector<uint32_t> map(nt, 0);
  std::vector<uint32_t> next(count, 0);
  if (count > 1)
    for (size_t t = 0; t < nt; t++) {
      if (owner[t] >= count) return fail(c, FR_E_INVALID, "fr_set_shard_plan: owner out of range");
      map[t] = (uint32_t)owner[t] << 24 | next[owner[t]]++;
    }
  join_recon(c);
  hipSetDevice(c->cfg.device);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream5));
  // the new map is complete before the old one goes: a failed allocation or copy leaves the previous
  // plan (map, owners, uniforms) in force
  uint32_t* new_map = nullptr;
  if (count > 1) {
    // a sharded rank's traced radiance (k_shade_resolve, active order): what it sends (fr_shard_pack_active)
    if (!c->shade_radiance && dalloc(&c->shade_radiance, (size_t)c->W * c->H) != hipSuccess) {
      c->shade_radiance = nullptr;
      return fail(c, FR_E_NOMEM, "fr_set_shard_plan: device allocation failed, previous plan kept");
    }
    if (hipMalloc((void**)&new_map, nt * sizeof(uint32_t)) != hipSuccess)
      return fail(c, FR_E_NOMEM, "fr_set_shard_plan: device allocation failed, previous plan kept");
    if (hipMemcpy(new_map, map.data(), nt * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
      hipFree(new_map);
      return fail(c, FR_E_HIP, "fr_set_shard_plan: device copy failed, previous plan kept");
    }
  }
  if (c->shard_map) hipFree(c->shard_map);
  c->shard_map = new_map;
  c->shard_owner.clear();
  if (count > 1) c->shard_owner.assign(owner, owner + nt);
  // counts of the previous plan are stale (fr_shard_counts refuses until a front stage ran under this one)
  for (bool& v : c->counts_valid) v = false;
  memset(c->h_counts, 0, sizeof(uint32_t) * fr_ctx::MAX_SLOTS * FR_MAX_SHARD_RANKS);
  c->U.shard_rank = rank;
  c->U.shard_count = count;
  c->U.shard_tile = tile;
  c->U.shard_tiles_x = tx;
  c->U.shard_map = c->shard_map;
  c->compacted = false;
  if (count == 1) c->front_local = false;
  return update_front_need(c);
}

// The 8x8 tiles a tile-local front computes: an owned 16x16 block's saliency cells (origins 4 px apart)
// read taps 4 px beyond their origin, so block b's stencil covers pixels [16b - 4, 16b + 16] on each
// axis. The left half of block k is read by blocks k-1 and k, the right half by k and k+1.
static int update_front_need(fr_ctx* c) {
  if (!c->front_local) {
    c->U.front_need = nullptr;
    return FR_OK;
  }
  const int tx8 = (c->W + 7) / 8, ty8 = (c->H + 7) / 8;
  const int bx = (c->W + 15) / 16, by = (c->H + 15) / 16;
  const int T = c->U.shard_tile;
  auto owned = [&](int X, int Y) {
    if (X < 0 || Y < 0 || X >= bx || Y >= by) return false;
    return c->shard_owner[(size_t)((Y * 16) / T) * c->U.shard_tiles_x + (X * 16) / T] == c->U.shard_rank;
  };
  c->front_need_h.assign((size_t)tx8 * ty8, 0);
  c->front_need_px = 0;
  for (int j = 0; j < ty8; j++)
    for (int i = 0; i < tx8; i++) {
      const int X = i >> 1, Y = j >> 1, dx = (i & 1) ? 1 : -1, dy = (j & 1) ? 1 : -1;
      const bool need = owned(X, Y) || owned(X + dx, Y) || owned(X, Y + dy) || owned(X + dx, Y + dy);
      if (!need) continue;
      c->front_need_h[(size_t)j * tx8 + i] = 1;
      c->front_need_px += (uint32_t)(std::min(8, c->W - i * 8) * std::min(8, c->H - j * 8));
    }
  if (!c->front_need) HIP_TRY(c, hipMalloc((void**)&c->front_need, c->front_need_h.size()));
  HIP_TRY(c, hipMemcpy(c->front_need, c->front_need_h.data(), c->front_need_h.size(), hipMemcpyHostToDevice));
  c->U.front_need = c->front_need;
  return FR_OK;
}

int fr_set_front_local(fr_ctx* c, int on) {
  if (!c) return FR_E_INVALID;
  if (on != 0 && on != 1) return fail(c, FR_E_INVALID, "fr_set_front_local: on is 0 or 1");
  if (on && c->U.shard_count <= 1) return fail(c, FR_E_STATE, "fr_set_front_local: needs a shard plan with count > 1");
  if ((bool)on == c->front_local) return FR_OK;
  join_recon(c);
  hipSetDevice(c->cfg.device);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream5));
  c->front_local = on != 0;
  c->compacted = false;
  return update_front_need(c);
}

int fr_set_shard_ex(fr_ctx* c, int rank, int count, int tile, int first_tracer) {
  if (!c) return FR_E_INVALID;
  if (first_tracer < 0 || (count > 1 && first_tracer >= count) || (count == 1 && first_tracer != 0))
    return fail(c, FR_E_INVALID, "fr_set_shard_ex: need 0 <= first_tracer < count (at least one tracing rank)");
  if (count < 1 || tile < 16 || tile % 16) return fail(c, FR_E_INVALID, "fr_set_shard: need count >= 1 and tile a multiple of 16");
  const size_t nt = (size_t)((c->W + tile - 1) / tile) * ((c->H + tile - 1) / tile);
  std::vector<uint8_t> owner(nt);
  for (size_t t = 0; t < nt; t++) owner[t] = (uint8_t)(first_tracer + t % (size_t)(count - first_tracer));
  return fr_set_shard_plan(c, rank, count, tile, owner.data(), nt);
}
int fr_set_shard(fr_ctx* c, int rank, int count, int tile) { return fr_set_shard_ex(c, rank, count, tile, 0); }

int fr_shard_counts(fr_ctx* c, uint32_t* counts, int n) {
  if (!c || !counts || n < 1) return FR_E_INVALID;
  if (c->U.shard_count <= 1) return fail(c, FR_E_STATE, "fr_shard_counts: call fr_set_shard with count > 1 first");
  if (!c->counts_valid[c->slot])
    return fail(c, FR_E_STATE, "fr_shard_counts: no front stage has run under the current shard plan");
  HIP_TRY(c, hipEventSynchronize(c->ev_counts[c->slot]));
  for (int r = 0; r < n; r++) counts[r] = r < c->U.shard_count ? c->h_counts[(size_t)c->slot * FR_MAX_SHARD_RANKS + r] : 0;
  return FR_OK;
}

int fr_shard_texels(fr_ctx* c, size_t* texels) {
  if (!c || !texels) return FR_E_INVALID;
  const int T = c->U.shard_count > 1 ? c->U.shard_tile : 0;
  if (!T) { *texels = (size_t)c->W * c->H; return FR_OK; }
  // the largest tile count of any rank (slabs of every rank have one size)
  std::vector<size_t> per(c->U.shard_count, 0);
  for (uint8_t o : c->shard_owner) per[o]++;
  size_t mx = 0;
  for (size_t v : per) mx = std::max(mx, v);
  *texels = std::max<size_t>(mx, 1) * (size_t)T * T;
  return FR_OK;
}

static int shard_io(fr_ctx* c, int id, int rank, void* slab, size_t bytes, bool pack) {
  if (!c || !slab) return FR_E_INVALID;
  if (c->U.shard_count <= 1) return fail(c, FR_E_STATE, "fr_shard_*: call fr_set_shard with count > 1 first");
  if (rank < 0 || rank >= c->U.shard_count) return fail(c, FR_E_INVALID, "fr_shard_unpack: bad source rank");
  join_recon(c);
  int p;
  if (resolve(c, id, &p)) return fail(c, FR_E_INVALID, "fr_shard_*: buffer is not an RGBA32F image");
  size_t texels = 0;
  fr_shard_texels(c, &texels);
  if (bytes < texels * sizeof(f4)) return fail(c, FR_E_INVALID, "fr_shard_*: slab smaller than fr_shard_texels * 16");
  hipSetDevice(c->cfg.device);
  if (pack) launch_shard_pack(c->U, c->img[p], (f4*)slab, c->stream);
  else launch_shard_unpack(c->U, rank, (const f4*)slab, c->img[p], c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}
int fr_shard_pack(fr_ctx* c, int id, void* slab, size_t bytes) {
  return shard_io(c, id, c ? c->U.shard_rank : 0, slab, bytes, true);
}
int fr_shard_unpack(fr_ctx* c, int id, int src_rank, const void* slab, size_t bytes) {
  return shard_io(c, id, src_rank, const_cast<void*>(slab), bytes, false);
}

int fr_shard_pack_active(fr_ctx* c, void* slab, size_t slab_bytes, uint32_t capacity, uint32_t* count) {
  if (!c || !slab || !count) return FR_E_INVALID;
  if (c->U.shard_count <= 1) return fail(c, FR_E_STATE, "fr_shard_*: call fr_set_shard with count > 1 first");
  if (slab_bytes < (size_t)capacity * 20) return fail(c, FR_E_INVALID, "fr_shard_pack_active: slab smaller than 20 * capacity");
  join_recon(c);
  hipSetDevice(c->cfg.device);
  HIP_TRY(c, hipMemcpyAsync(count, c->ray_count, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (*count > capacity) return fail(c, FR_E_INVALID, "fr_shard_pack_active: capacity below the active pixel count");
  f4* vals = (f4*)slab;
  uint32_t* idx = (uint32_t*)((char*)slab + (size_t)capacity * sizeof(f4));
  launch_shard_pack_active(c->active, c->ray_count, capacity, c->shade_radiance, vals, idx, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}

int fr_shard_unpack_active(fr_ctx* c, const void* slab, size_t slab_bytes, uint32_t capacity, uint32_t count) {
  if (!c || !slab) return FR_E_INVALID;
  if (count > capacity) return fail(c, FR_E_INVALID, "fr_shard_unpack_active: count above capacity");
  if (slab_bytes < (size_t)capacity * 20) return fail(c, FR_E_INVALID, "fr_shard_unpack_active: slab smaller than 20 * capacity");
  join_recon(c);
  hipSetDevice(c->cfg.device);
  const f4* vals = (const f4*)slab;
  const uint32_t* idx = (const uint32_t*)((const char*)slab + (size_t)capacity * sizeof(f4));
  launch_shard_unpack_active(c->U, vals, idx, count, (uint32_t)((size_t)c->W * c->H), c->img[P_wgt(c)],
                             c->img[c->hist_cur], c->img[c->hist_cache], c->img[P_shd(c)], c->stream);
  c->hvalid_fresh = false;
  int rc = check_launch(c);
  if (rc) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}

int fr_synchronize(fr_ctx* c) {
  if (!c) return FR_E_INVALID;
  join_recon(c);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}

int fr_ray_count(fr_ctx* c, uint32_t* n) {
  if (!c || !n) return FR_E_INVALID;
  join_recon(c);
  HIP_TRY(c, hipMemcpyAsync(n, c->ray_count, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}

int fr_gaze_target(fr_ctx* c, float xyz[3]) {
  // gaze_target[0] = position_buffer[make_uint2(gaze)] (samplingStep.cu:184)
  if (!c || !xyz) return FR_E_INVALID;
  join_recon(c);
  // same texel as the sampling kernel's focal-depth read: saturating conversion, clamped to the screen
  const uint32_t gx = std::min(f2u_sat(c->U.gaze.x), (uint32_t)c->W - 1), gy = std::min(f2u_sat(c->U.gaze.y), (uint32_t)c->H - 1);
  f4 v;
  HIP_TRY(c, hipMemcpyAsync(&v, c->img[P_pos(c)] + (size_t)gy * c->W + gx, sizeof(f4), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  xyz[0] = v.x; xyz[1] = v.y; xyz[2] = v.z;
  return FR_OK;
}

int fr_get_buffer(fr_ctx* c, int id, fr_buffer_view* v) {
  const bool owed = c && c->jfa_coord_owed && (id == FR_BUF_JFA_COLOR || id == FR_BUF_JFA_COORD);
  const int rc = buffer_view(c, id, v);
  // a view handed out after its image was written on demand: that write is complete when the call returns (the
  // caller may read through the pointer on any stream)
  if (rc == FR_OK && owed) HIP_TRY(c, hipStreamSynchronize(c->stream));
  // the caller may write the JFA outputs through the view: Sibson then derives its seeds and row prefix sums
  // from them again instead of from the JFA run's own state
  if (rc == FR_OK && (id == FR_BUF_JFA_COLOR || id == FR_BUF_JFA_COORD)) c->sib_prefix_fresh = false;
  // ... and the history: the next frame's sample setup then reads it, not the validity bits of what the last frame left
  if (rc == FR_OK && (id == FR_BUF_HISTORY || id == FR_BUF_HISTORY_CACHE)) c->hvalid_fresh = false;
  return rc;
}

static int buffer_view(fr_ctx* c, int id, fr_buffer_view* v) {
  if (!c || !v) return FR_E_INVALID;
  join_recon(c);  // later work on the context stream is ordered after the reconstruction
  const size_t N = (size_t)c->W * c->H;
  if (id == FR_BUF_THREAD) {
    *v = fr_buffer_view{c->active, (int)N, 1, N * 4, N * 4, FR_FMT_U32};
    return FR_OK;
  }
  if (id == FR_BUF_MASK) {
    *v = fr_buffer_view{c->mask, c->W, c->H, (size_t)c->W, N, FR_FMT_U8};
    return FR_OK;
  }
  if (id == FR_BUF_GCLASS) {
    *v = fr_buffer_view{c->gclass, c->W, c->H, (size_t)c->W, N, FR_FMT_U8};
    return FR_OK;
  }
  int p;
  if (resolve(c, id, &p)) return fail(c, FR_E_INVALID, "unknown buffer id");
  *v = fr_buffer_view{c->img[p], c->W, c->H, (size_t)c->W * sizeof(f4), N * sizeof(f4), FR_FMT_RGBA32F};
  return FR_OK;
}

int fr_read_buffer(fr_ctx* c, int id, void* host, size_t bytes) {
  fr_buffer_view v;
  int rc = buffer_view(c, id, &v);
  if (rc) return rc;
  if (!host || bytes > v.bytes) return fail(c, FR_E_INVALID, "read_buffer: size");
  HIP_TRY(c, hipMemcpyAsync(host, v.device_ptr, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}

int fr_write_buffer(fr_ctx* c, int id, const void* host, size_t bytes) {
  fr_buffer_view v;
  int rc = buffer_view(c, id, &v);
  if (rc) return rc;
  if (!host || bytes > v.bytes) return fail(c, FR_E_INVALID, "write_buffer: size");
  HIP_TRY(c, hipMemcpyAsync(v.device_ptr, host, bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  // Sibson's row prefix sums (and the JFA state it reads its seeds from) no longer match these
  if (id == FR_BUF_JFA_COLOR || id == FR_BUF_JFA_COORD) c->sib_prefix_fresh = false;
  if (id == FR_BUF_HISTORY || id == FR_BUF_HISTORY_CACHE) c->hvalid_fresh = false;
  if (id == FR_BUF_MASK) {
    // a host-written mask must also drive the compaction: rebuild the wave ballots from it
    c->compacted = false;
    c->mask_dirty = true;
  }
  return FR_OK;
}

// ---- Snapshot / restore of the temporal state (deterministic multi-frame golden tests) ----
// What a frame carries into the next one: the history and depth ping-pong pairs (FR/PathTracer.cpp:226-238),
// the pull / push atlases and the push pass's snapshot texels (the push reads the previous frame's atlas,
// FR/PullPushInterpolation.cpp:57-58), the m_accumFrame counter with its pending light reset, the light
// emission, and the camera / gaze uniforms of the last update. Everything else a frame reads it writes first.
// Layout: a fixed header, then the buffers in the order below (cache before current of each pair).
namespace {
constexpr uint32_t kSnapMagic = 0x4E535246u;  // "FRSN"
constexpr uint32_t kSnapVersion = 1;
struct SnapHeader {
  uint32_t magic, version;
  int32_t width, height, pp_S, spp, scene, mask_mode;
  uint32_t accum, light_pending;
  float light_emission[3];
  int32_t diffuse_max_depth;
  float inv_vp[16], prev_vp[16], eye[3], prev_eye[3], gaze[2];
  uint64_t payload_bytes;
};
struct SnapPart {
  void* dev;
  size_t bytes;
};
constexpr int kSnapParts = 7;
struct SnapParts {
  SnapPart p[kSnapParts];
  const SnapPart* begin() const { return p; }
  const SnapPart* end() const { return p + kSnapParts; }
};
SnapParts snap_parts(fr_ctx* c) {
  const size_t img = (size_t)c->W * c->H * sizeof(f4);
  const size_t atlas = (size_t)c->pp_S * (c->pp_S + c->pp_S / 2) * sizeof(f4);
  return SnapParts{{{c->img[c->hist_cache], img}, {c->img[c->hist_cur], img}, {c->img[c->depth_cache], img},
                    {c->img[c->depth_cur], img}, {c->pull, atlas}, {c->push, atlas},
                    {c->snap, pp_snap_count(c->pp_S) * sizeof(f4)}}};
}
size_t snap_total(fr_ctx* c) {
  size_t n = sizeof(SnapHeader);
  for (const SnapPart& p : snap_parts(c)) n += p.bytes;
  return n;
}
}  // namespace

int fr_snapshot_bytes(fr_ctx* c, size_t* bytes) {
  if (!c || !bytes) return FR_E_INVALID;
  *bytes = snap_total(c);
  return FR_OK;
}

int fr_snapshot(fr_ctx* c, void* host, size_t bytes) {
  if (!c) return FR_E_INVALID;
  const size_t need = snap_total(c);
  if (!host || bytes < need) return fail(c, FR_E_INVALID, "snapshot: buffer smaller than fr_snapshot_bytes");
  join_recon(c);
  hipSetDevice(c->cfg.device);
  SnapHeader h{};
  h.magic = kSnapMagic; h.version = kSnapVersion;
  h.width = c->W; h.height = c->H; h.pp_S = c->pp_S; h.spp = c->U.spp; h.scene = c->cfg.scene;
  h.mask_mode = c->U.mask_mode;
  h.accum = c->accum; h.light_pending = c->light_pending ? 1u : 0u;
  h.light_emission[0] = c->dsc.light_emission.x; h.light_emission[1] = c->dsc.light_emission.y;
  h.light_emission[2] = c->dsc.light_emission.z;
  h.diffuse_max_depth = c->U.diffuse_max_depth;
  memcpy(h.inv_vp, &c->U.inv_vp, sizeof(h.inv_vp));
  memcpy(h.prev_vp, &c->U.prev_vp, sizeof(h.prev_vp));
  memcpy(h.eye, &c->U.eye, sizeof(h.eye));
  memcpy(h.prev_eye, &c->U.prev_eye, sizeof(h.prev_eye));
  memcpy(h.gaze, &c->U.gaze, sizeof(h.gaze));
  h.payload_bytes = need - sizeof(SnapHeader);
  char* out = static_cast<char*>(host);
  memcpy(out, &h, sizeof(h));
  size_t off = sizeof(h);
  for (const SnapPart& p : snap_parts(c)) {
    HIP_TRY(c, hipMemcpyAsync(out + off, p.dev, p.bytes, hipMemcpyDeviceToHost, c->stream));
    off += p.bytes;
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FR_OK;
}

int fr_restore(fr_ctx* c, const void* host, size_t bytes) {
  if (!c) return FR_E_INVALID;
  const size_t need = snap_total(c);
  if (!host || bytes < need) return fail(c, FR_E_INVALID, "restore: buffer smaller than fr_snapshot_bytes");
  SnapHeader h;
  memcpy(&h, host, sizeof(h));
  if (h.magic != kSnapMagic || h.version != kSnapVersion) return fail(c, FR_E_INVALID, "restore: not a fovrt snapshot");
  if (h.width != c->W || h.height != c->H || h.pp_S != c->pp_S || h.spp != c->U.spp || h.scene != c->cfg.scene ||
      h.payload_bytes != need - sizeof(SnapHeader))
    return fail(c, FR_E_INVALID, "restore: snapshot of another configuration (size, spp or scene differ)");
  join_recon(c);
  hipSetDevice(c->cfg.device);
  const char* in = static_cast<const char*>(host);
  size_t off = sizeof(h);
  for (const SnapPart& p : snap_parts(c)) {
    HIP_TRY(c, hipMemcpyAsync(p.dev, in + off, p.bytes, hipMemcpyHostToDevice, c->stream));
    off += p.bytes;
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->accum = h.accum;
  c->light_pending = h.light_pending != 0;
  c->dsc.light_emission = mk3(h.light_emission[0], h.light_emission[1], h.light_emission[2]);
  c->U.diffuse_max_depth = h.diffuse_max_depth;
  c->U.mask_mode = h.mask_mode;
  memcpy(&c->U.inv_vp, h.inv_vp, sizeof(h.inv_vp));
  memcpy(&c->U.prev_vp, h.prev_vp, sizeof(h.prev_vp));
  memcpy(&c->U.eye, h.eye, sizeof(h.eye));
  memcpy(&c->U.prev_eye, h.prev_eye, sizeof(h.prev_eye));
  memcpy(&c->U.gaze, h.gaze, sizeof(h.gaze));
  c->lp_gaze = f2{-1e30f, -1e30f};  // the log-polar mask cache is recomputed for the restored gaze
  c->lp_mode = -1;
  c->sib_prefix_fresh = false;
  c->hvalid_fresh = false;
  return FR_OK;
}

int fr_rebuild_bvh(fr_ctx* c, float* ms) {
  if (!c) return FR_E_INVALID;
  join_recon(c);
  hipSetDevice(c->cfg.device);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = gpu_rebuild(c);
  if (ms) *ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

static_assert(sizeof(f3) == 3 * sizeof(float), "f3 must be three packed floats");
int fr_set_positions(fr_ctx* c, const float* xyz, size_t ntris) {
  if (!c || !xyz) return FR_E_INVALID;
  if (ntris != (size_t)c->scene.num_tris()) return fail(c, FR_E_INVALID, "fr_set_positions: triangle count differs");
  for (size_t i = 0; i < ntris * 9; i++)
    if (!std::isfinite(xyz[i])) return fail(c, FR_E_INVALID, "fr_set_positions: position not finite");
  join_recon(c);
  hipSetDevice(c->cfg.device);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  // the BVH is built from the device copy; the context commits the new positions (host mirror,
  // bounding box) only once the rebuild succeeded, and puts the old device copy back otherwise
  const size_t bytes = ntris * 9 * sizeof(float);
  HIP_TRY(c, hipMemcpy(c->d_pos, xyz, bytes, hipMemcpyHostToDevice));
  if (const int rc = gpu_rebuild(c)) {
    const std::string why = c->err;
    if (hipMemcpy(c->d_pos, c->scene.pos.data(), bytes, hipMemcpyHostToDevice) != hipSuccess)
      return fail(c, FR_E_HIP, "fr_set_positions: rebuild failed (" + why + ") and the old positions could not be restored");
    return fail(c, rc, "fr_set_positions: rebuild failed, scene unchanged: " + why);
  }
  memcpy(c->scene.pos.data(), xyz, bytes);
  // bbox_min / bbox_max (the depth-saliency theta of k_sampling) follow the geometry, as the
  // reference's scene AABB does at load time (FR/PathTracer.cpp:601-602,663)
  f3 lo = mk3(INFINITY), hi = mk3(-INFINITY);
  for (const f3& v : c->scene.pos) {
    lo = mk3(fminf(lo.x, v.x), fminf(lo.y, v.y), fminf(lo.z, v.z));
    hi = mk3(fmaxf(hi.x, v.x), fmaxf(hi.y, v.y), fmaxf(hi.z, v.z));
  }
  c->scene.bbox_min = c->dsc.bbox_min = lo;
  c->scene.bbox_max = c->dsc.bbox_max = hi;
  return FR_OK;
}

#ifdef FR_STAMPS
// Diagnostic probe (libfovrt_diag.so only, not part of the ABI): one shading launch (geometry /
// sampling / optimize must have run) with per-sample records (queries, traversal steps, start, end;
// s_memrealtime ticks) and per-wave records (start, refill dry, end, samples), copied to the host.
extern "C" int fr_diag_sample_trace(fr_ctx* c, uint32_t* srec, uint32_t scap, uint32_t* wrec, uint32_t wcap) {
  if (!c || !srec || !wrec) return FR_E_INVALID;
  join_recon(c);
  hipSetDevice(c->cfg.device);
  uint32_t *ds = nullptr, *dw = nullptr;
  HIP_TRY(c, hipMalloc(&ds, (size_t)scap * 16));
  HIP_TRY(c, hipMalloc(&dw, (size_t)wcap * 16));
  hipMemsetAsync(ds, 0, (size_t)scap * 16, c->stream);
  hipMemsetAsync(dw, 0, (size_t)wcap * 16, c->stream);
  diag_sample_trace(ds, scap, dw, wcap, c->stream);
  int rc = enqueue_shading(c);
  diag_sample_trace(nullptr, 0, nullptr, 0, c->stream);
  hipStreamSynchronize(c->stream);
  if (!rc) {
    HIP_TRY(c, hipMemcpy(srec, ds, (size_t)scap * 16, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(wrec, dw, (size_t)wcap * 16, hipMemcpyDeviceToHost));
  }
  hipFree(ds);
  hipFree(dw);
  return rc;
}

// Diagnostic probe (libfovrt_diag.so only, not part of the ABI): records every query of one shading
// launch (geometry / sampling / optimize must have run), then traces the recorded stream with
// k_trace_queries. out = {queries, best ms of 5 runs, shadow queries, ms of the stream partitioned by
// kind, ms of its closest-hit part (specialised kernel), ms of its shadow part (specialised kernel)}.
extern "C" int fr_diag_trace_queries(fr_ctx* c, float* out) {
  if (!c || !out) return FR_E_INVALID;
  join_recon(c);
  hipSetDevice(c->cfg.device);
  const uint32_t cap = 48u << 20;
  f4 *rec = nullptr, *hits = nullptr;
  uint32_t* ctr = nullptr;
  HIP_TRY(c, hipMalloc(&rec, (size_t)cap * 32));
  HIP_TRY(c, hipMalloc(&hits, (size_t)cap * 16));
  HIP_TRY(c, hipMalloc(&ctr, 4));
  diag_record_queries(rec, cap, c->stream);
  int rc = enqueue_shading(c);
  if (rc) return rc;
  uint32_t n = std::min(diag_recorded_queries(c->stream), cap);
  diag_record_queries(nullptr, 0, c->stream);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  // best of 5 runs of fn() on the context stream
  auto timeit = [&](auto fn) {
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(a, c->stream);
      fn();
      hipEventRecord(b, c->stream);
      hipStreamSynchronize(c->stream);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    return best;
  };
  const float t_mixed = timeit([&] { launch_trace_queries(c->dsc, rec, n, hits, ctr, c->stream, 0); });
  // the same stream partitioned by kind (closest-hit first, then shadow; order within a kind kept)
  std::vector<f4> d((size_t)n * 2), part;
  HIP_TRY(c, hipMemcpy(d.data(), rec, (size_t)n * 32, hipMemcpyDeviceToHost));
  part.reserve(d.size());
  for (int pass = 0; pass < 2; pass++)
    for (uint32_t i = 0; i < n; i++)
      if ((d[2 * (size_t)i + 1].w != 0.0f) == (pass == 1)) { part.push_back(d[2 * (size_t)i]); part.push_back(d[2 * (size_t)i + 1]); }
  size_t shadow = 0;
  for (uint32_t i = 0; i < n; i++) shadow += d[2 * (size_t)i + 1].w != 0.0f;
  if (const char* path = getenv("FOVRT_DIAG_DUMP")) {  // every 16th query (o, tmax, d, any) for offline BVH studies
    if (FILE* f = fopen(path, "wb")) {
      for (uint32_t i = 0; i < n; i += 16) fwrite(&d[2 * (size_t)i], sizeof(f4), 2, f);
      fclose(f);
    }
  }
  const uint32_t nc = n - (uint32_t)shadow;
  HIP_TRY(c, hipMemcpy(rec, part.data(), (size_t)n * 32, hipMemcpyHostToDevice));
  const float t_sorted = timeit([&] { launch_trace_queries(c->dsc, rec, n, hits, ctr, c->stream, 0); });
  const float t_closest = timeit([&] { launch_trace_queries(c->dsc, rec, nc, hits, ctr, c->stream, 1); });
  const float t_shadow =
      timeit([&] { launch_trace_queries(c->dsc, rec + 2 * (size_t)nc, (uint32_t)shadow, hits, ctr, c->stream, 2); });
  out[3] = t_sorted;
  out[4] = t_closest;
  out[5] = t_shadow;
  const float best = t_mixed;
  out[0] = (float)n;
  out[1] = best;
  out[2] = (float)shadow;
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFree(rec);
  hipFree(hits);
  hipFree(ctr);
  return check_launch(c);
}
#endif

int fr_get_stats(fr_ctx* c, fr_stats* s) {
  if (!c || !s) return FR_E_INVALID;
  DevStats d;
  HIP_TRY(c, hipMemcpyAsync(&d, c->stats, sizeof(d), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  s->gbuffer_primary = d.gbuffer_primary; s->primary = d.primary; s->shadow = d.shadow;
  s->diffuse_bounce = d.diffuse_bounce; s->mirror = d.mirror; s->refraction = d.refraction;
  s->reflection = d.reflection; s->truncated = d.truncated; s->overflow = d.bvh_overflow;
  for (int i = 0; i < 6; i++) s->diag[i] = d.pad[i];
  s->segments = d.gbuffer_primary + d.primary + d.shadow + d.diffuse_bounce + d.mirror + d.refraction + d.reflection;
  return FR_OK;
}

// Test hook (not part of include/fovrt.h): the host build of the bound JFA and Sibson use.
float fr__sqrt_le_bound(float s) { return sqrt_le_bound(s); }

// Diagnostic hook (not part of include/fovrt.h): the last Sibson pass's list counts: strips (k_sibson_strip),
// wide[0] and wide[1] (k_sibson_wide's two lists).
int fr__sibson_counts(fr_ctx* c, uint32_t* out3) {
  if (!c || !out3 || !c->sib_strips) return FR_E_INVALID;
  hipSetDevice(c->cfg.device);
  HIP_TRY(c, hipDeviceSynchronize());
  HIP_TRY(c, hipMemcpy(out3, c->sib_strips, sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(out3 + 1, c->sib_wide, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return FR_OK;
}

// Test hook (not part of include/fovrt.h): pack_texture on n RGBA32F texels; returns the FR_TEX_* kind
// and writes the packed words (n of them) for the packed kinds.
int fr__pack_texture(const float* rgba, int n, uint32_t* out) {
  if (!rgba || n < 0 || !out) return -1;
  HostTexture t;
  t.w = n; t.h = 1;
  t.data.resize((size_t)n);
  memcpy(t.data.data(), rgba, sizeof(f4) * (size_t)n);
  std::vector<uint32_t> packed;
  const int kind = pack_texture(t, packed);
  if (kind != FR_TEX_F32) memcpy(out, packed.data(), sizeof(uint32_t) * (size_t)n);
  return kind;
}

int fr_kernel_timing(fr_ctx* c, int enable) {
  if (!c) return FR_E_INVALID;
  if (enable && !c->kt_ev[0][0])
    for (auto& q : c->kt_ev)
      for (auto& e : q) HIP_TRY(c, hipEventCreate(&e));
  c->kt_on = enable != 0;
  c->kt_next = c->kt_pending = 0;
  c->kt_frames = 0;
  c->kt_stage_ms = c->kt_kernel_ms = 0.0;
  return FR_OK;
}

int fr_frame_clock(fr_ctx* c, int enable) {
  if (!c) return FR_E_INVALID;
  hipSetDevice(c->cfg.device);
  if (enable && !c->fc_ref) {
    HIP_TRY(c, hipEventCreate(&c->fc_ref));
    for (auto& q : c->fc_ev)
      for (auto& e : q) HIP_TRY(c, hipEventCreate(&e));
  }
  if (c->fc_pending) HIP_TRY(c, hipDeviceSynchronize());  // nothing recorded stays in flight across a reset
  c->fc_on = enable != 0;
  c->fc_next = c->fc_pending = 0;
  c->fc_cur = -1;
  c->fc_prev_end = -1.0;
  c->fc_latency.clear();
  c->fc_interval.clear();
  if (c->fc_on) HIP_TRY(c, hipEventRecord(c->fc_ref, c->stream));
  return FR_OK;
}

int fr_frame_clock_read(fr_ctx* c, float* latency_ms, float* interval_ms, int cap, int* n_latency, int* n_interval) {
  if (!c || cap < 0 || (cap > 0 && (!latency_ms || !interval_ms)) || !n_latency || !n_interval) return FR_E_INVALID;
  hipSetDevice(c->cfg.device);
  for (; c->fc_pending > 0; c->fc_pending--)
    fc_harvest(c, (c->fc_next - c->fc_pending + fr_ctx::FC_RING) % fr_ctx::FC_RING);
  *n_latency = (int)std::min<size_t>(c->fc_latency.size(), (size_t)cap);
  *n_interval = (int)std::min<size_t>(c->fc_interval.size(), (size_t)cap);
  if (*n_latency) memcpy(latency_ms, c->fc_latency.data(), sizeof(float) * *n_latency);
  if (*n_interval) memcpy(interval_ms, c->fc_interval.data(), sizeof(float) * *n_interval);
  return FR_OK;
}

int fr_kernel_times(fr_ctx* c, fr_stage_times* out) {
  if (!c || !out) return FR_E_INVALID;
  for (; c->kt_pending > 0; c->kt_pending--)
    kt_harvest(c, (c->kt_next - c->kt_pending + fr_ctx::KT_RING) % fr_ctx::KT_RING);
  out->frames = c->kt_frames;
  out->shading_ms = c->kt_stage_ms;
  out->shade_paths_ms = c->kt_kernel_ms;
  return FR_OK;
}

int fr_reset_stats(fr_ctx* c) {
  if (!c) return FR_E_INVALID;
  HIP_TRY(c, hipMemsetAsync(c->stats, 0, sizeof(DevStats), c->stream));
  return FR_OK;
}

}  // extern "C"

namespace fri {
int fail(fr_ctx* c, int code, const std::string& msg) { return ::fail(c, code, msg); }
int check_launch(fr_ctx* c) { return ::check_launch(c); }
void join_recon(fr_ctx* c) { ::join_recon(c); }
int frame_half(fr_ctx* c, fr_frame_timing* t, bool trace, bool recon) { return ::frame_half(c, t, trace, recon); }
int P_shd(const fr_ctx* c) { return ::P_shd(c); }
int P_wgt(const fr_ctx* c) { return ::P_wgt(c); }
}  // namespace fri

struct fr_scene {
  HostScene scene;
  Bvh bvh;
  std::string err;
  std::vector<const float*> tex_ptrs;
  std::vector<int32_t> tex_dims, mat_pairs;
};

static void fill_arrays(const HostScene& s, const Bvh& bvh, f3 emission, std::vector<int32_t>& mat_pairs,
                        std::vector<int32_t>& tex_dims, std::vector<const float*>& tex_ptrs, fr_scene_arrays* o) {
  memset(o, 0, sizeof(*o));
  o->num_tris = s.num_tris();
  o->pos = &s.pos[0].x; o->nrm = &s.nrm[0].x; o->uv = &s.uv[0].x; o->flags = s.flags.data();
  mat_pairs.clear();
  for (auto& m : s.mats) { mat_pairs.push_back(m.type); mat_pairs.push_back(m.tex); }
  o->num_materials = (int)s.mats.size();
  o->materials = mat_pairs.data();
  tex_dims.clear(); tex_ptrs.clear();
  for (auto& t : s.texs) { tex_dims.push_back(t.w); tex_dims.push_back(t.h); tex_ptrs.push_back(&t.data[0].x); }
  o->num_textures = (int)s.texs.size();
  o->tex_dims = tex_dims.data();
  o->tex_data = tex_ptrs.data();
  o->envmap = s.envmap;
  const f3 L[5] = {s.light_position, s.light_v1, s.light_v2, s.light_normal, emission};
  for (int i = 0; i < 5; i++) { o->light[3 * i] = L[i].x; o->light[3 * i + 1] = L[i].y; o->light[3 * i + 2] = L[i].z; }
  o->bbox[0] = s.bbox_min.x; o->bbox[1] = s.bbox_min.y; o->bbox[2] = s.bbox_min.z;
  o->bbox[3] = s.bbox_max.x; o->bbox[4] = s.bbox_max.y; o->bbox[5] = s.bbox_max.z;
  o->bvh_nodes = bvh.gpu_nodes >= 0 ? bvh.gpu_nodes : bvh.host_nodes ? bvh.host_nodes : (int)bvh.nodes.size();
  o->bvh_depth = bvh.max_depth;
  o->bvh_max_stack = bvh.max_stack;
}

extern "C" {

int fr_scene_export(fr_ctx* c, fr_scene_arrays* o) {
  if (!c || !o) return FR_E_INVALID;
  fill_arrays(c->scene, c->bvh, c->dsc.light_emission, c->mat_pairs, c->tex_dims, c->tex_ptrs, o);
  return FR_OK;
}

int fr_scene_create(const fr_config* cfg_in, fr_scene** out) {
  if (!out) return fail(nullptr, FR_E_INVALID, "out is NULL");
  *out = nullptr;
  fr_config cfg;
  if (cfg_in) cfg = *cfg_in; else fr_config_default(&cfg);
  if (cfg.scene < 0 || cfg.scene > 2) return fail(nullptr, FR_E_INVALID, "bad scene preset");
  if (cfg.mesh_mode < 0 || cfg.mesh_mode > 2) return fail(nullptr, FR_E_INVALID, "bad mesh_mode");
  fr_scene* sc = new fr_scene();
  std::string err;
  if (!build_preset_scene(cfg.scene, cfg.asset_dir ? cfg.asset_dir : "assets", cfg.texture_mode, cfg.light_power,
                          cfg.detail, sc->scene, err, cfg.mesh_mode)) {
    delete sc;
    return fail(nullptr, FR_E_IO, "scene: " + err);
  }
  build_bvh(sc->scene, sc->bvh);
  *out = sc;
  return FR_OK;
}

int fr_scene_get_arrays(fr_scene* sc, fr_scene_arrays* o) {
  if (!sc || !o) return FR_E_INVALID;
  fill_arrays(sc->scene, sc->bvh, sc->scene.light_emission, sc->mat_pairs, sc->tex_dims, sc->tex_ptrs, o);
  return FR_OK;
}

int fr_scene_destroy(fr_scene* sc) {
  if (!sc) return FR_E_INVALID;
  delete sc;
  return FR_OK;
}

}  // extern "C"
