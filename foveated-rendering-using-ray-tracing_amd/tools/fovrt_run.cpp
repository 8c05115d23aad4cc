// fovrt_run — headless C++ driver of the reference's frame loop (FR/main.cpp:227-362) on the C++
// facades (include/fovrt.hpp): the same object construction, camera set-up, launch order, gaze /
// ray-count read-backs and per-stage timing line as the reference, without a window.
//
//   fovrt_run [W H] [--scene box|bunny|vokselia] [--mask saliency|logpolar|uniform|all|logpolar10]
//             [--spp N] [--dmd N] [--frames N] [--assets DIR] [--procedural] [--dump BUFFER FILE.pfm]
//
// --dump writes one buffer (e.g. ATROUS, SHADING, SIBSON) after the last frame as a little-endian
// RGB PFM (row 0 = bottom, as PFM stores it), the image-dump replacement of saveBMP24
// (FR/gui.cpp:315-355).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fovrt.hpp"

using namespace fovrt;

static int buffer_id(const std::string& n) {
  static const char* names[] = {"POSITION", "NORMAL", "DEPTH", "DIFFUSE", "WEIGHT", "THREAD", "HISTORY", "SHADING",
                                "EXTRA", "JFA_COORD", "JFA_COLOR", "SIBSON", "PULLPUSH", "ATROUS"};
  for (int i = 0; i < (int)(sizeof(names) / sizeof(names[0])); i++)
    if (n == names[i]) return i;
  return -1;
}

static bool write_pfm(const char* path, const std::vector<float>& rgba, int w, int h) {
  FILE* f = fopen(path, "wb");
  if (!f) return false;
  fprintf(f, "PF\n%d %d\n-1.0\n", w, h);
  std::vector<float> row((size_t)w * 3);
  for (int y = 0; y < h; y++) {
    for (int x = 0; x < w; x++)
      for (int c = 0; c < 3; c++) row[(size_t)x * 3 + c] = rgba[((size_t)y * w + x) * 4 + c];
    fwrite(row.data(), sizeof(float), row.size(), f);
  }
  return fclose(f) == 0;
}

int main(int argc, char** argv) {
  fr_config cfg;
  fr_config_default(&cfg);
  cfg.width = 1024; cfg.height = 1024;
  cfg.scene = FR_SCENE_BUNNY;
  cfg.mask_mode = FR_MASK_LOGPOLAR_SIGNED;
  cfg.spp = 4; cfg.diffuse_max_depth = 3;
  int frames = 10;
  std::string dump_buf, dump_path, assets = "assets";
  int pos = 0;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> const char* { if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", a.c_str()); exit(2); } return argv[++i]; };
    if (a == "--scene") { std::string s = next(); cfg.scene = s == "box" ? FR_SCENE_BOX : s == "vokselia" ? FR_SCENE_VOKSELIA : FR_SCENE_BUNNY; }
    else if (a == "--mask") {
      std::string m = next();
      cfg.mask_mode = m == "saliency" ? FR_MASK_SALIENCY : m == "logpolar" ? FR_MASK_LOGPOLAR : m == "uniform" ? FR_MASK_UNIFORM2X2
                    : m == "all" ? FR_MASK_ALL : FR_MASK_LOGPOLAR_SIGNED;
    }
    else if (a == "--spp") cfg.spp = atoi(next());
    else if (a == "--dmd") cfg.diffuse_max_depth = atoi(next());
    else if (a == "--frames") frames = atoi(next());
    else if (a == "--assets") assets = next();
    else if (a == "--procedural") cfg.texture_mode = 1;
    else if (a == "--dump") { dump_buf = next(); dump_path = next(); }
    else if (pos == 0) { cfg.width = atoi(a.c_str()); pos++; }
    else if (pos == 1) { cfg.height = atoi(a.c_str()); pos++; }
    else { fprintf(stderr, "unknown argument %s\n", a.c_str()); return 2; }
  }
  cfg.asset_dir = assets.c_str();

  // object construction (FR/main.cpp:152-159)
  PathTracer* tracer = new PathTracer(cfg);
  JumpFlooding* g_JFRenderer = new JumpFlooding(*tracer);
  PullPushInterpolation* g_PPIRenderer = new PullPushInterpolation(*tracer);
  SibsonInterpolation* g_SIRenderer = new SibsonInterpolation(*tracer);
  ATrous* g_ATRenderer = new ATrous(*tracer);
  if (!tracer->initialize(cfg.width, cfg.height)) {
    fprintf(stderr, "initialize failed: %s\n", tracer->initialize_error().c_str());
    return 1;
  }
  // camera (FR/main.cpp:185-209): the preset pose of the scene
  Camera g_camera;
  vec3 eye, target;
  fr_preset_camera(cfg.scene, eye.data(), target.data());
  g_camera.setRotation({1.0f, 0.0f, 0.0f, 0.0f});
  g_camera.setPosition(eye);
  g_camera.lookAt(target);
  g_camera.setProjectMode(Camera::PM_Perspective, 45, 0.1f, 500.1f);
  g_camera.setScreen((float)cfg.width, (float)cfg.height);
  g_camera.setViewport(0, 0, (float)cfg.width, (float)cfg.height);
  tracer->init_camera(g_camera);

  try {
    for (int f = 0; f < frames; f++) {
      // loop body (FR/main.cpp:253-358)
      std::string text;
      char buf[96];
      tracer->update_optix_variables(g_camera);
      float g = tracer->geometry_launch();
      float s = tracer->sampling_launch();
      float o = tracer->optimize_launch();
      float sh = tracer->shading_launch();
      vec3 gaze_target = tracer->gaze_target();
      unsigned trace_sample = tracer->ray_count();
      Texture pos_t = tracer->get_texture(PathTracer::POSITION);
      Texture norm_t = tracer->get_texture(PathTracer::NORMAL);
      Texture shading_tex = tracer->get_texture(PathTracer::SHADING);
      uint64_t jf = 0, si = 0, pp = 0, at = 0;
      int done = 0;
      g_JFRenderer->render(shading_tex, nullptr, &jf, &done);
      Texture jfa_tex = g_JFRenderer->colorTex, jfa_coord_tex = g_JFRenderer->coordTex;
      g_SIRenderer->render(jfa_coord_tex, jfa_tex, nullptr, &si, &done);
      g_PPIRenderer->render(shading_tex, nullptr, &pp, &done);
      Texture ppi_tex = g_PPIRenderer->outputTex;
      g_ATRenderer->render(1, pos_t, norm_t, ppi_tex, jfa_tex, (int)(unsigned)tracer->m_accumFrame, nullptr, &at, &done);
      g_camera.setPrevState();
      // the PrintMSTimes line (FR/main.cpp:21-24, 260-374), in fractional ms
      snprintf(buf, sizeof(buf), "Geometry, %.3f, Sampling, %.3f, Optimize, %.3f, Shading, %.3f, ", g, s, o, sh);
      text += buf;
      snprintf(buf, sizeof(buf), "ray count, %u, (%%), %.3f, ", trace_sample,
               100.0 * trace_sample / ((double)cfg.width * cfg.height));
      text += buf;
      snprintf(buf, sizeof(buf), "JPA, %.3f, SI, %.3f, PPI, %.3f, AT, %.3f", jf / 1e6, si / 1e6, pp / 1e6, at / 1e6);
      text += buf;
      printf("frame %d, %s, gaze_target, %.4f %.4f %.4f\n", f, text.c_str(), gaze_target[0], gaze_target[1],
             gaze_target[2]);
    }
    if (!dump_buf.empty()) {
      int id = buffer_id(dump_buf);
      if (id < 0 || id == FR_BUF_THREAD) { fprintf(stderr, "cannot dump %s\n", dump_buf.c_str()); return 2; }
      std::vector<float> img = tracer->read_rgba(Texture(id));
      if (!write_pfm(dump_path.c_str(), img, cfg.width, cfg.height)) { fprintf(stderr, "write failed\n"); return 1; }
    }
  } catch (const Error& e) {
    fprintf(stderr, "fovrt error %d: %s\n", e.code, e.what());
    return 1;
  }
  delete g_ATRenderer; delete g_SIRenderer; delete g_PPIRenderer; delete g_JFRenderer; delete tracer;
  return 0;
}
