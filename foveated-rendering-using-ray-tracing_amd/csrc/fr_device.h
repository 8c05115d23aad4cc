// fr_device.h — device-resident data layout of the fovrt hot path (shared by host builders and
// the gfx950 kernels). Everything here is plain-old-data that lives in HBM for the lifetime of a
// context; kernels receive the small descriptor structs by value.
#pragma once
#include "fr_math.h"

namespace fr {

#define FR_BVH_STACK 24  // per-lane traversal stack entries (LDS; one per BVH level)
#define FR_VRING 2       // history validity ring inside each tile of a still-camera group (k_vring_pack)

enum MaterialType : int32_t { MATL_DIFFUSE = 0, MATL_REFLECTION = 1, MATL_REFRACTION = 2 };

// Four-wide BVH node: the boxes of all four children, SoA by axis (two 64-byte lines per visit).
// child[k] >= 0 with count[k] == 0  -> inner node index
// count[k] > 0                      -> leaf: triangles [child[k], child[k]+count[k]) of tri_geo
// count[k] < 0                      -> empty slot (box lo = +inf, hi = -inf; never hit)
struct alignas(16) BvhNode {
  f4 lox, hix;  // child k's x slab in component k
  f4 loy, hiy;
  f4 loz, hiz;
  int32_t child[4];
  int32_t count[4];
};
static_assert(sizeof(BvhNode) == 128, "BvhNode must be two 64-byte lines");

// Leaf-ordered triangle, pre-differenced exactly as optix::intersect_triangle does at run time
// (e0 = p1 - p0, e1 = p0 - p2, n = cross(e1, e0); optixu_math_namespace.h, PTX
// FR/cuda/triangle_mesh.ptx:380-430). Three 16-B loads per candidate triangle.
struct alignas(16) TriGeo {
  f4 a;  // p0.x p0.y p0.z e0.x
  f4 b;  // e0.y e0.z e1.x e1.y
  f4 c;  // e1.z n.x  n.y  n.z
};

// Per-primitive shading attributes, fetched once per closest hit (and per refractive any-hit).
// flags = material index | (has_normals << 8) | (has_uv << 9)
struct alignas(16) TriShade {
  f4 n0;  // n0.xyz, t0.x
  f4 n1;  // n1.xyz, t0.y
  f4 n2;  // n2.xyz, t1.x
  f4 t;   // t1.y, t2.x, t2.y, bits(flags)
};
#define FR_SHADE_HAS_NORMALS 0x100
#define FR_SHADE_HAS_UV 0x200

// Texel storage, the densest exact form per texture (context.cpp, pack_texture): RGBA32F; RGBA8 when
// every channel is exactly b / 255.0f (the 8-bit PPM / PNG textures sutil::loadTexture reads as
// normalised bytes); RGBE when every texel is (m * 2^(e - 136), alpha 1) (the Radiance .hdr environment
// map, FR/PathTracer.cpp:454-455). Decoding is exact (tex_texel, k_trace.hip): a lookup returns the
// RGBA32F texel bit for bit, from a quarter of the bytes.
enum { FR_TEX_F32 = 0, FR_TEX_UNORM8 = 1, FR_TEX_RGBE = 2 };
struct DevTexture {
  const f4* data;          // FR_TEX_F32: row 0 = bottom (v = 0), RGBA, normalised float
  const uint32_t* packed;  // FR_TEX_UNORM8 / FR_TEX_RGBE: r | g << 8 | b << 16 | (a or e) << 24
  int32_t w, h;
  int32_t kind;
};

struct DevMaterial {
  int32_t type;
  int32_t tex;
};

#define FR_MAX_TEXTURES 8
#define FR_MAX_MATERIALS 8

// Packed fp32 (v_pk_add_f32 / v_pk_mul_f32, two values per lane). Every element goes through
// exactly the operations of its scalar form, in the same order, so results are bit-identical.
typedef float v2f __attribute__((ext_vector_type(2)));
FR_HD v2f v2(float a, float b) {
  v2f r;
  r.x = a;
  r.y = b;
  return r;
}
FR_HD v2f v2s(float a) { return v2(a, a); }

struct DevScene {
  const BvhNode* nodes;
  const TriGeo* tri_geo;
  const int32_t* tri_prim;  // leaf order -> original primitive index
  const TriShade* shade;    // by original primitive index
  int32_t root_count;       // >0: the whole scene is one leaf; else root is node 0
  int32_t num_tris;
  const DevMaterial* mats;  // device arrays (divergent indexing stays out of the kernarg segment)
  const DevTexture* texs;
  int32_t envmap;           // texture index of the lat-long environment map
  // ParallelogramLight (FR/PathTracer.cpp:564-579)
  f3 light_position, light_v1, light_v2, light_normal, light_emission;
  float light_area;         // length(cross(v1, v2))
  f3 bbox_min, bbox_max;
  float scene_epsilon;      // 1e-3 (FR/PathTracer.cpp:474)
};

// Per-frame uniforms (FR/PathTracer.cpp:85-116, 774-820).
struct FrameUniforms {
  mat4 inv_vp;              // "mvp" on the device: inverse(P*V), row-major
  mat4 prev_vp;             // "prev_mvp": P*V of the previous frame, row-major
  f3 eye, prev_eye;
  f2 gaze;                  // (g_gaze.x, H - g_gaze.y)
  f2 screen;                // (W, H)
  int32_t width, height;
  uint32_t frame;           // m_accumFrame before the post-increment
  int32_t diffuse_max_depth;
  int32_t reflection_max_depth;   // 4 (FR/PathTracer.cpp:724)
  int32_t refraction_max_depth;   // min(refraction_maxdepth=100, max_depth=100), capped
  int32_t spp;
  int32_t sqrt_spp;
  int32_t mask_mode;
  // screen-tile sharding of one view across ranks (fr_set_shard_plan): tile t = ty * tiles_x + tx is
  // traced by rank shard_map[t] >> 24, and is that rank's (shard_map[t] & 0xFFFFFF)-th tile (its slot
  // in a packed tile slab); shard_count 1 = the whole screen (shard_map unused)
  int32_t shard_rank, shard_count, shard_tile, shard_tiles_x;
  const uint32_t* shard_map;
  // tile-local front stages (fr_set_front_local, a tracing rank of a static-camera group): the G-buffer
  // runs on the 8x8 pixel tiles with front_need[t] != 0 (this rank's tiles plus the saliency stencil's
  // halo) and on the gaze pixel's tile; k_sampling and the carry only on this rank's tiles. front_pixels
  // = the G-buffer pixels that traces (the primary-ray count). Null = the whole screen.
  const uint8_t* front_need;
  uint32_t front_pixels;
};

// The 8x8 tile of the gaze pixel (its depth sets the saliency focus in k_sampling; the clamp is
// k_sampling's).
FR_HD int gaze_tile8(const FrameUniforms& U) {
  uint32_t gx = f2u_sat(U.gaze.x), gy = f2u_sat(U.gaze.y);
  gx = gx < (uint32_t)U.width - 1 ? gx : (uint32_t)U.width - 1;
  gy = gy < (uint32_t)U.height - 1 ? gy : (uint32_t)U.height - 1;
  return (int)((gy >> 3) * (uint32_t)((U.width + 7) >> 3) + (gx >> 3));
}

// XCD-aware block order: blocks b, b+8, b+16, ... share an XCD (and its L2), so hand each of the 8
// such classes one contiguous run of tiles (row-major bands of the image) instead of every 8th tile.
// Bijective for any block count. Returns the tile index for 2-D grid block (bx, by).
FR_DEV uint32_t xcd_tile(uint32_t bx, uint32_t by, uint32_t gx, uint32_t gy) {
  const uint32_t nwg = gx * gy, bid = by * gx + bx;
  const uint32_t q = nwg / 8, r = nwg % 8, k = bid % 8, i = bid / 8;
  return k * q + (k < r ? k : r) + i;
}

FR_DEV int shard_owner(const FrameUniforms& U, int t) { return (int)(U.shard_map[t] >> 24); }
FR_DEV int shard_tile_of(const FrameUniforms& U, int x, int y) {
  return (y / U.shard_tile) * U.shard_tiles_x + x / U.shard_tile;
}
FR_DEV bool shard_owns(const FrameUniforms& U, int x, int y) {
  if (U.shard_count <= 1) return true;
  return shard_owner(U, shard_tile_of(U, x, y)) == U.shard_rank;
}

// Ray-segment statistics, accumulated with one atomic per wave.
struct DevStats {
  unsigned long long gbuffer_primary;
  unsigned long long primary;
  unsigned long long shadow;
  unsigned long long diffuse_bounce;
  unsigned long long mirror;
  unsigned long long refraction;
  unsigned long long reflection;
  unsigned long long truncated;   // refraction nodes that hit the depth cap
  unsigned long long bvh_overflow;
  unsigned long long pad[7];
};

}  // namespace fr
