// fovrt.hpp — header-only C++ facades over the fovrt C ABI (include/fovrt.h) that keep the reference's
// class names, method names and argument order, so a main.cpp-shaped frame loop
// (FR/main.cpp:152-358) drives the MI355X engine with only type changes:
//
//   reference (CUDA/OptiX + GL)                      here
//   ------------------------------------------------ -------------------------------------------------
//   GLuint (texture name)                            fovrt::Texture (a buffer id of the context)
//   tracer->m_context["gaze_target"] + rtBufferMap   tracer->gaze_target()
//   tracer->m_context["ray_count"] + rtBufferMap     tracer->ray_count()
//   const GLuint* query, GLuint64* elapsed, int* done  same parameters; query is ignored, elapsed is the
//                                                    pass time in ns (HIP events), done is set to 1
//   optix::Exception                                 fovrt::Error (thrown by the facade, never by the ABI)
//
// FR/ = "/root/reference/Foveated Rendering using Ray Tracing/". The facades own nothing on the device:
// the fr_ctx of the PathTracer owns every buffer, the pass objects only name its outputs.
#pragma once

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "fovrt.h"

namespace fovrt {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc, fr_ctx* ctx, const char* what) {
  if (rc != FR_OK) {
    const char* msg = fr_last_error(ctx);
    throw Error(rc, std::string(what) + ": " + (msg ? msg : "error"));
  }
}

// A GL texture name of the reference = a buffer id of the context here.
struct Texture {
  int id = -1;
  constexpr Texture() = default;
  constexpr explicit Texture(int i) : id(i) {}
  constexpr operator int() const { return id; }
};

using vec3 = std::array<float, 3>;
using quat = std::array<float, 4>;  // (w, x, y, z) like glm::quat
using mat4 = std::array<float, 16>; // row-major, v' = M v

// Camera (FR/Camera.h, FR/Camera.cpp): the subset the frame loop uses, glm-compatible math.
class Camera {
 public:
  enum ProjMode { PM_Perspective, PM_Ortho_Height, PM_Ortho_Width, PM_Ortho };

  Camera() {
    pose_.pos[0] = pose_.pos[1] = pose_.pos[2] = 0.0f;
    pose_.rot[0] = 1.0f; pose_.rot[1] = pose_.rot[2] = pose_.rot[3] = 0.0f;
    pose_.fovy_deg = 45.0f; pose_.znear = 0.1f; pose_.zfar = 500.1f; pose_.aspect = 1.0f;
    prev_ = pose_;
  }
  void setScreen(float w, float h) { screen_[0] = w; screen_[1] = h; }          // FR/Camera.cpp:18-21
  void setViewport(float, float, float w, float h) { pose_.aspect = w / h; }  // :23-27 (aspect = w / h)
  void setProjectMode(ProjMode mode, float fov_deg, float n, float f) {
    if (mode != PM_Perspective) throw Error(FR_E_UNSUPPORTED, "only PM_Perspective is used by the frame loop");
    pose_.fovy_deg = fov_deg; pose_.znear = n; pose_.zfar = f;
  }
  void setPosition(const vec3& p) { for (int i = 0; i < 3; i++) pose_.pos[i] = p[i]; }
  void setRotation(const quat& q) { for (int i = 0; i < 4; i++) pose_.rot[i] = q[i]; }
  void setTarget(const vec3& t) { target_ = t; }  // FR/Camera.cpp: stores the target only
  void lookAt(const vec3& target, const vec3& up = {0.0f, 1.0f, 0.0f}) {  // FR/Camera.cpp:73-83
    check(fr_camera_look_at(&pose_, target.data(), up.data()), nullptr, "Camera::lookAt");
    target_ = target;
  }
  vec3 getPosition() const { return {pose_.pos[0], pose_.pos[1], pose_.pos[2]}; }
  vec3 getTarget() const { return target_; }
  quat getRotation() const { return {pose_.rot[0], pose_.rot[1], pose_.rot[2], pose_.rot[3]}; }
  mat4 getVMat() const { mat4 v, p; check(fr_camera_matrices(&pose_, v.data(), p.data()), nullptr, "getVMat"); return v; }
  mat4 getPMat() const { mat4 v, p; check(fr_camera_matrices(&pose_, v.data(), p.data()), nullptr, "getPMat"); return p; }
  void setPrevState() { prev_ = pose_; has_prev_ = true; }  // FR/Camera.cpp:234-241

  // the uniforms update_optix_variables derives (FR/PathTracer.cpp:774-820)
  fr_camera uniforms(int width, int height) const {
    fr_camera c;
    check(fr_camera_uniforms(&pose_, has_prev_ ? &prev_ : &pose_, width, height, &c), nullptr, "Camera uniforms");
    for (int i = 0; i < 3; i++) c.target[i] = target_[i];
    return c;
  }
  const fr_camera_pose& pose() const { return pose_; }

 private:
  fr_camera_pose pose_{};
  fr_camera_pose prev_{};
  bool has_prev_ = false;
  vec3 target_{0.0f, 0.0f, 0.0f};
  float screen_[2] = {0.0f, 0.0f};
};

class PathTracer;

// `tracer->m_accumFrame` reads the frame counter; `tracer->m_accumFrame = 0` resets accumulation
// (FR/main.cpp:248, the only assignment the reference makes).
class AccumFrame {
 public:
  explicit AccumFrame(fr_ctx* const* ctx) : ctx_(ctx) {}
  operator unsigned int() const {
    uint32_t f = 0;
    check(fr_accum_frame(*ctx_, &f), *ctx_, "m_accumFrame");
    return f;
  }
  AccumFrame& operator=(unsigned int v) {
    if (v != 0) throw Error(FR_E_UNSUPPORTED, "m_accumFrame can only be reset to 0");
    check(fr_reset_accumulation(*ctx_), *ctx_, "m_accumFrame = 0");
    return *this;
  }

 private:
  fr_ctx* const* ctx_;
};

// PathTracer (FR/PathTracer.h:10-110): the four launches, texture access and frame counter.
class PathTracer {
 public:
  enum TextureName { POSITION, NORMAL, DEPTH, DIFFUSE, WEIGHT, THREAD, HISTORY, SHADING, EXTRA };

  PathTracer() { fr_config_default(&cfg_); }  // cfg.abi_version = FOVRT_ABI_VERSION
  explicit PathTracer(const fr_config& cfg) : cfg_(cfg) {}
  PathTracer(const PathTracer&) = delete;
  PathTracer& operator=(const PathTracer&) = delete;
  virtual ~PathTracer() { if (ctx_) fr_destroy(ctx_); }

  bool initialize(int width, int height) {  // FR/PathTracer.cpp:41-78
    cfg_.width = width; cfg_.height = height;
    if (ctx_) { fr_destroy(ctx_); ctx_ = nullptr; }
    if (fr_create(&cfg_, &ctx_) != FR_OK) { error_ = fr_last_error(nullptr); ctx_ = nullptr; return false; }
    return true;
  }
  const std::string& initialize_error() const { return error_; }
  void init_camera(const Camera& camera) { update_optix_variables(camera); }  // :606-632
  void update_optix_variables(const Camera& camera) {                        // :774-820
    fr_camera c = camera.uniforms(cfg_.width, cfg_.height);
    check(fr_set_camera(ctx(), &c), ctx_, "update_optix_variables");
  }
  float geometry_launch() { float ms = 0; check(fr_geometry_launch(ctx(), &ms), ctx_, "geometry_launch"); return ms; }
  float sampling_launch() { float ms = 0; check(fr_sampling_launch(ctx(), &ms), ctx_, "sampling_launch"); return ms; }
  float optimize_launch() { float ms = 0; check(fr_optimize_launch(ctx(), &ms), ctx_, "optimize_launch"); return ms; }
  float shading_launch() { float ms = 0; check(fr_shading_launch(ctx(), &ms), ctx_, "shading_launch"); return ms; }

  Texture get_texture(TextureName name) const { return Texture((int)name); }  // :337-374

  vec3 gaze_target() {  // m_context["gaze_target"] (FR/main.cpp:278-287)
    vec3 g;
    check(fr_gaze_target(ctx(), g.data()), ctx_, "gaze_target");
    return g;
  }
  float rebuild_bvh() {  // GPU LBVH over the current triangles (fr_rebuild_bvh), wall ms
    float ms = 0.0f;
    check(fr_rebuild_bvh(ctx(), &ms), ctx_, "rebuild_bvh");
    return ms;
  }
  void set_positions(const float* xyz, size_t ntris) {  // moved vertices + GPU rebuild (fr_set_positions)
    check(fr_set_positions(ctx(), xyz, ntris), ctx_, "set_positions");
  }
  // cursorPosCallback (FR/gui.cpp:48-66): the cursor in window coordinates (y down); adjust_scale 1.25
  // in a window, 1 in full screen (g_fullScreen)
  void set_gaze(double xpos, double ypos, bool fullscreen = false) {
    check(fr_set_gaze(ctx(), xpos, ypos, fullscreen ? 1 : 0), ctx_, "set_gaze");
  }
  void reset_gaze() { check(fr_reset_gaze(ctx()), ctx_, "reset_gaze"); }  // framebufferSizeCallback (:32-35)
  unsigned int ray_count() {  // m_context["ray_count"] (FR/main.cpp:288-299)
    uint32_t n = 0;
    check(fr_ray_count(ctx(), &n), ctx_, "ray_count");
    return n;
  }

  // beyond the reference: whole-frame enqueue, buffer reads, statistics
  fr_frame_timing frame() { fr_frame_timing t{}; check(fr_frame(ctx(), &t), ctx_, "frame"); return t; }
  std::vector<float> read_rgba(Texture t) {
    std::vector<float> v((size_t)cfg_.width * cfg_.height * 4);
    check(fr_read_buffer(ctx(), t.id, v.data(), v.size() * sizeof(float)), ctx_, "read_rgba");
    return v;
  }
  fr_stats stats() { fr_stats s{}; check(fr_get_stats(ctx(), &s), ctx_, "stats"); return s; }
  // temporal state (history / depth pairs, pull-push atlases, m_accumFrame, camera) to host memory and back
  std::vector<uint8_t> snapshot() {
    size_t n = 0;
    check(fr_snapshot_bytes(ctx(), &n), ctx_, "snapshot");
    std::vector<uint8_t> v(n);
    check(fr_snapshot(ctx(), v.data(), v.size()), ctx_, "snapshot");
    return v;
  }
  void restore(const std::vector<uint8_t>& v) { check(fr_restore(ctx(), v.data(), v.size()), ctx_, "restore"); }
  // live per-launch HIP-event timing of the shading stage (off by default)
  void kernel_timing(bool on) { check(fr_kernel_timing(ctx(), on ? 1 : 0), ctx_, "kernel_timing"); }
  fr_stage_times kernel_times() { fr_stage_times t{}; check(fr_kernel_times(ctx(), &t), ctx_, "kernel_times"); return t; }
  // FR_PIPELINE_THROUGHPUT (frames back to back) or FR_PIPELINE_LATENCY (one trace half in flight)
  void set_pipeline_mode(int mode) { check(fr_set_pipeline_mode(ctx(), mode), ctx_, "set_pipeline_mode"); }
  // per-frame latency and display interval of pipelined frames (fr_frame_clock), in ms
  void frame_clock(bool on) { check(fr_frame_clock(ctx(), on ? 1 : 0), ctx_, "frame_clock"); }
  void frame_clock_read(std::vector<float>& latency_ms, std::vector<float>& interval_ms, int cap = 65536) {
    latency_ms.resize((size_t)cap);
    interval_ms.resize((size_t)cap);
    int nl = 0, ni = 0;
    check(fr_frame_clock_read(ctx(), latency_ms.data(), interval_ms.data(), cap, &nl, &ni), ctx_, "frame_clock_read");
    latency_ms.resize((size_t)nl);
    interval_ms.resize((size_t)ni);
  }
  fr_ctx* ctx() const {
    if (!ctx_) throw Error(FR_E_STATE, "PathTracer used before initialize()");
    return ctx_;
  }
  const fr_config& config() const { return cfg_; }

  AccumFrame m_accumFrame{&ctx_};

 private:
  fr_config cfg_{};
  fr_ctx* ctx_ = nullptr;
  std::string error_;
};

// GL pass classes (FR/JumpFlooding.h, FR/SibsonInterpolation.h, FR/PullPushInterpolation.h,
// FR/ATrous.h). They read the screen size from the tracer's context instead of g_screenSize.
namespace detail {
inline void finish(uint64_t ns, uint64_t* elapsed, int* done) {
  if (elapsed) *elapsed = ns;
  if (done) *done = 1;
}
}  // namespace detail

// GBuffer (FR/GBuffer.h:27-64): the reference constructs it and calls render() every frame
// (FR/main.cpp:153,255), but its constructor never builds the FBO, VAO or shader (FR/GBuffer.cpp:11-26)
// and nothing reads its textures; the G-buffer that feeds the path is OptiX entry 0
// (PathTracer::geometry_launch). The facade keeps those lines compiling: render() does no work and
// reports 0 ns, and the texture names are the "no texture" 0 of an unbuilt FBO.
class GBuffer {
 public:
  GBuffer() = default;
  void render(const unsigned* /*query*/ = nullptr, uint64_t* elapsed_time = nullptr, int* done = nullptr) {
    detail::finish(0, elapsed_time, done);
  }
  void BindBuffers() {}
  void resetFrameCount() {}
  void resetShader() {}
  void genScene() {}
  void loadMesh(const char*) {}
  void setupMesh() {}
  const Texture positionTex{};
  const Texture normalTex{};
  const Texture depthTex{};
  const unsigned fbo = 0;
};

class JumpFlooding {
 public:
  explicit JumpFlooding(PathTracer& t) : t_(t) {}
  void render(Texture rt, const unsigned* /*query*/ = nullptr, uint64_t* elapsed_time = nullptr, int* done = nullptr) {
    uint64_t ns = 0;
    check(fr_jfa_render(t_.ctx(), rt.id, &ns), t_.ctx(), "JumpFlooding::render");
    detail::finish(ns, elapsed_time, done);
  }
  void resetShader() {}
  const Texture coordTex{FR_BUF_JFA_COORD};
  const Texture colorTex{FR_BUF_JFA_COLOR};

 private:
  PathTracer& t_;
};

class LogPolarTransform {  // FR/Log_Polar_Transform.h
 public:
  explicit LogPolarTransform(PathTracer& t) : t_(t) {}
  void render(Texture pt, const unsigned* = nullptr, uint64_t* elapsed_time = nullptr, int* done = nullptr) {
    uint64_t ns = 0;
    check(fr_logpolar_render(t_.ctx(), pt.id, &ns), t_.ctx(), "LogPolarTransform::render");
    detail::finish(ns, elapsed_time, done);
  }
  void resetShader() {}
  const Texture logPolarTex{FR_BUF_LOGPOLAR};
  const Texture ilogPolarTex{FR_BUF_LOGPOLAR_INVERSE};

 private:
  PathTracer& t_;
};

class SibsonInterpolation {
 public:
  explicit SibsonInterpolation(PathTracer& t) : t_(t) {}
  void render(Texture coord, Texture color, const unsigned* = nullptr, uint64_t* elapsed_time = nullptr,
              int* done = nullptr) {
    if (coord.id != FR_BUF_JFA_COORD || color.id != FR_BUF_JFA_COLOR)
      throw Error(FR_E_INVALID, "SibsonInterpolation::render takes JumpFlooding's coordTex/colorTex");
    uint64_t ns = 0;
    check(fr_sibson_render(t_.ctx(), &ns), t_.ctx(), "SibsonInterpolation::render");
    detail::finish(ns, elapsed_time, done);
  }
  void resetShader() {}
  const Texture outputTex{FR_BUF_SIBSON};

 private:
  PathTracer& t_;
};

class PullPushInterpolation {
 public:
  explicit PullPushInterpolation(PathTracer& t) : t_(t) {}
  void render(Texture sparse, const unsigned* = nullptr, uint64_t* elapsed_time = nullptr, int* done = nullptr) {
    uint64_t ns = 0;
    check(fr_pullpush_render(t_.ctx(), sparse.id, &ns), t_.ctx(), "PullPushInterpolation::render");
    detail::finish(ns, elapsed_time, done);
  }
  void resetShader() {}
  const Texture outputTex{FR_BUF_PULLPUSH};

 private:
  PathTracer& t_;
};

class ATrous {
 public:
  explicit ATrous(PathTracer& t) : t_(t) {}
  // rtTex and frame are accepted and unused, as in atFS.glsl (FR/ATrous.cpp:47-132)
  void render(int count, Texture positionTex, Texture normalTex, Texture inColorTex, Texture /*rtTex*/ = Texture(),
              int /*frame*/ = 0, const unsigned* = nullptr, uint64_t* elapsed_time = nullptr, int* done = nullptr) {
    uint64_t ns = 0;
    check(fr_atrous_render(t_.ctx(), count, positionTex.id, normalTex.id, inColorTex.id, &ns), t_.ctx(),
          "ATrous::render");
    detail::finish(ns, elapsed_time, done);
  }
  const Texture colorTex{FR_BUF_ATROUS};

 private:
  PathTracer& t_;
};

// Multi-GPU group (fr_group_*): one object per process; ranks = the local tracers (in-process copies)
// or this process's tracer in an RCCL communicator.
class Group {
 public:
  Group(std::vector<PathTracer*> tracers, void* rccl_comm, const fr_group_config& cfg) {
    std::vector<fr_ctx*> c;
    for (PathTracer* t : tracers) c.push_back(t->ctx());
    check(fr_group_create(c.data(), (int)c.size(), rccl_comm, &cfg, &g_), nullptr, "fr_group_create");
    n_ = (int)c.size();
  }
  Group(const Group&) = delete;
  Group& operator=(const Group&) = delete;
  ~Group() { if (g_) fr_group_destroy(g_); }
  void frame() { check(fr_group_frame(g_, nullptr), nullptr, "fr_group_frame"); }
  std::vector<fr_frame_timing> frame_timed() {
    std::vector<fr_frame_timing> t((size_t)n_);
    check(fr_group_frame(g_, t.data()), nullptr, "fr_group_frame");
    return t;
  }
  void composite(void* device_out, size_t bytes) { check(fr_group_composite(g_, device_out, bytes), nullptr, "fr_group_composite"); }
  void synchronize() { check(fr_group_synchronize(g_), nullptr, "fr_group_synchronize"); }
  fr_group* handle() const { return g_; }

 private:
  fr_group* g_ = nullptr;
  int n_ = 0;
};

}  // namespace fovrt
