// scene.h — host-side scene assembly for the fovrt path tracer.
//
// Mirrors PathTracer::init_geometry / createGeometry / load_obj (FR/PathTracer.cpp:559-772): five
// models with baked transforms, three material kinds, one parallelogram light, a lat-long
// environment map. The reference's meshes (*.obj) are not in its repository
// (ROOT/.gitignore:52), so each model is a deterministic procedural stand-in.
#pragma once
#include <string>
#include <vector>
#include "fr_device.h"

namespace fr {

struct HostTexture {
  int w = 0, h = 0;
  std::vector<f4> data;  // row 0 = bottom
};

struct HostScene {
  // Triangle soup in world space (transforms baked, as sutil::loadMesh does).
  std::vector<f3> pos;        // 3 per triangle
  std::vector<f3> nrm;        // 3 per triangle (valid when flags & FR_SHADE_HAS_NORMALS)
  std::vector<f2> uv;         // 3 per triangle (valid when flags & FR_SHADE_HAS_UV)
  std::vector<int32_t> flags; // 1 per triangle: material | has_normals | has_uv
  std::vector<DevMaterial> mats;
  std::vector<HostTexture> texs;
  int envmap = -1;
  f3 light_position, light_v1, light_v2, light_normal, light_emission;
  f3 bbox_min, bbox_max;
  std::vector<std::string> model_names;
  std::vector<int> model_tri_count;

  int num_tris() const { return (int)flags.size(); }
};

struct Bvh {
  std::vector<BvhNode> nodes;
  std::vector<TriGeo> tri_geo;    // leaf order
  std::vector<int32_t> tri_prim;  // leaf order -> primitive
  int root_count = 0;             // >0 when the root itself is a leaf
  int max_depth = 0;
  int max_stack = 0;              // deepest traversal stack any root-to-leaf path can need
  int gpu_nodes = -1;             // node count of a device-built tree (its arrays stay on the device)
  int host_nodes = 0;             // node count of a host-built tree whose arrays were released after the upload
};

enum ScenePreset { PRESET_BOX = 0, PRESET_BUNNY = 1, PRESET_VOKSELIA = 2 };

// Builds a preset. texture_mode 0: load the reference assets from asset_dir (error if missing);
// 1: deterministic procedural textures (same sizes), for asset-free tests.
// mesh_mode 0: the reference's OBJ meshes where present under asset_dir, procedural stand-ins
// otherwise; 1: procedural only; 2: OBJ required.
bool build_preset_scene(int preset, const std::string& asset_dir, int texture_mode, float light_power,
                        int detail, HostScene& out, std::string& err, int mesh_mode = 0);

bool load_ppm(const std::string& path, HostTexture& tex, std::string& err);
bool load_hdr(const std::string& path, HostTexture& tex, std::string& err);
bool load_png(const std::string& path, HostTexture& tex, std::string& err);

// Binned-SAH binary BVH over the soup collapsed into four-wide nodes; conservative (inflated)
// child boxes.
void build_bvh(const HostScene& s, Bvh& out);

// Camera presets (FR/main.cpp:189-209): eye and look-at target.
void preset_camera(int preset, f3& eye, f3& target);

}  // namespace fr
