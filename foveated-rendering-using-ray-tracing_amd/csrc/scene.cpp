// scene.cpp — procedural stand-ins for the reference's five models, texture loaders, SAH BVH.
//
// Reference: PathTracer::init_geometry (FR/PathTracer.cpp:559-603), load_obj (:676-772),
// createGeometry (:634-674). Transforms and materials are the reference's; geometry is generated
// deterministically (seed 20180920) because the .obj files were never committed upstream.
#include "scene.h"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <tuple>
#include <map>
#include <sstream>

namespace fr {

namespace {

constexpr uint32_t kSeed = 20180920u;

float hash01(uint32_t a, uint32_t b) { return (float)(tea16(a ^ kSeed, b) & 0xFFFFFF) / 16777216.0f; }

struct Mesh {
  std::vector<f3> v, n;
  std::vector<f2> uv;
  std::vector<int32_t> idx;  // 3 per triangle
  bool has_n = false, has_uv = false;
};

// transform: p' = translate + scale * p (uniform scale), computed in float like optix::Matrix4x4;
// normals by the inverse transpose, n' = n / scale, not renormalised (sutil loadMesh with a
// load_xform; shading normalises after interpolation, FR/cuda/triangle_mesh.cu:82-91).
void bake(Mesh& m, f3 t, float s) {
  for (auto& p : m.v) p = mk3(s * p.x + t.x, s * p.y + t.y, s * p.z + t.z);
  if (m.has_n)
    for (auto& n : m.n) n = mk3(n.x / s, n.y / s, n.z / s);
}

void add_mesh(HostScene& sc, const Mesh& m, int material, const char* name) {
  int before = sc.num_tris();
  for (size_t k = 0; k + 2 < m.idx.size(); k += 3) {
    int i0 = m.idx[k], i1 = m.idx[k + 1], i2 = m.idx[k + 2];
    f3 a = m.v[i0], b = m.v[i1], c = m.v[i2];
    f3 cr = cross(b - a, c - a);
    float area = length(cr);
    if (!(area > 0.0f) || std::isinf(area)) continue;  // mesh_bounds invalidates these (triangle_mesh.cu:132-137)
    sc.pos.push_back(a); sc.pos.push_back(b); sc.pos.push_back(c);
    if (m.has_n) { sc.nrm.push_back(m.n[i0]); sc.nrm.push_back(m.n[i1]); sc.nrm.push_back(m.n[i2]); }
    else { sc.nrm.push_back(mk3(0.f)); sc.nrm.push_back(mk3(0.f)); sc.nrm.push_back(mk3(0.f)); }
    if (m.has_uv) { sc.uv.push_back(m.uv[i0]); sc.uv.push_back(m.uv[i1]); sc.uv.push_back(m.uv[i2]); }
    else { sc.uv.push_back(mk2(0, 0)); sc.uv.push_back(mk2(0, 0)); sc.uv.push_back(mk2(0, 0)); }
    sc.flags.push_back(material | (m.has_n ? FR_SHADE_HAS_NORMALS : 0) | (m.has_uv ? FR_SHADE_HAS_UV : 0));
    for (f3 p : {a, b, c}) {
      sc.bbox_min = mk3(fminf(sc.bbox_min.x, p.x), fminf(sc.bbox_min.y, p.y), fminf(sc.bbox_min.z, p.z));
      sc.bbox_max = mk3(fmaxf(sc.bbox_max.x, p.x), fmaxf(sc.bbox_max.y, p.y), fmaxf(sc.bbox_max.z, p.z));
    }
  }
  sc.model_names.push_back(name);
  sc.model_tri_count.push_back(sc.num_tris() - before);
}

// Ground quad: 20 x 20 units in the xz plane, grid.ppm tiled once per unit.
Mesh make_ground() {
  Mesh m;
  m.v = {mk3(-10, 0, -10), mk3(-10, 0, 10), mk3(10, 0, 10), mk3(10, 0, -10)};
  m.n = {mk3(0, 1, 0), mk3(0, 1, 0), mk3(0, 1, 0), mk3(0, 1, 0)};
  m.uv = {mk2(0, 20), mk2(0, 0), mk2(20, 0), mk2(20, 20)};
  m.idx = {0, 1, 2, 0, 2, 3};  // CCW seen from +y: normal cross(p1-p0, p2-p0) = +y
  m.has_n = m.has_uv = true;
  return m;
}

// Axis-aligned cube, x,z in [-50,50], y in [0,100] (object units of the 100-unit box.obj).
Mesh make_cube() {
  Mesh m;
  const f3 nrm[6] = {mk3(1, 0, 0), mk3(-1, 0, 0), mk3(0, 1, 0), mk3(0, -1, 0), mk3(0, 0, 1), mk3(0, 0, -1)};
  for (int f = 0; f < 6; f++) {
    f3 n = nrm[f];
    f3 u = fabsf(n.y) > 0.5f ? mk3(1, 0, 0) : mk3(0, 1, 0);
    f3 v = cross(n, u);
    f3 c = mk3(50 * n.x, 50 + 50 * n.y, 50 * n.z);
    int base = (int)m.v.size();
    const float su[4] = {-1, 1, 1, -1}, sv[4] = {-1, -1, 1, 1};
    for (int k = 0; k < 4; k++) {
      m.v.push_back(c + u * (50.0f * su[k]) + v * (50.0f * sv[k]));
      m.n.push_back(n);
      m.uv.push_back(mk2(0.5f * (su[k] + 1.0f), 0.5f * (sv[k] + 1.0f)));
    }
    // u x v = n, so (c-u-v, c+u-v, c+u+v) is CCW around n.
    int q[6] = {0, 1, 2, 0, 2, 3};
    for (int k : q) m.idx.push_back(base + k);
  }
  m.has_n = m.has_uv = true;
  return m;
}

// Displaced icosphere standing in for the Stanford bunny: radius ~2 object units, base at y = 0.
Mesh make_blob(int subdiv) {
  std::vector<f3> v;
  std::vector<int32_t> f;
  const float t = (1.0f + sqrtf(5.0f)) * 0.5f;
  f3 base[12] = {mk3(-1, t, 0), mk3(1, t, 0), mk3(-1, -t, 0), mk3(1, -t, 0), mk3(0, -1, t), mk3(0, 1, t),
                 mk3(0, -1, -t), mk3(0, 1, -t), mk3(t, 0, -1), mk3(t, 0, 1), mk3(-t, 0, -1), mk3(-t, 0, 1)};
  for (auto& p : base) v.push_back(normalize(p));
  int tris[60] = {0, 11, 5, 0, 5, 1, 0, 1, 7, 0, 7, 10, 0, 10, 11, 1, 5, 9, 5, 11, 4, 11, 10, 2, 10, 7, 6, 7, 1, 8,
                  3, 9, 4, 3, 4, 2, 3, 2, 6, 3, 6, 8, 3, 8, 9, 4, 9, 5, 2, 4, 11, 6, 2, 10, 8, 6, 7, 9, 8, 1};
  f.assign(tris, tris + 60);
  for (int s = 0; s < subdiv; s++) {
    std::map<uint64_t, int> mid;
    auto midpoint = [&](int a, int b) {
      uint64_t key = a < b ? ((uint64_t)a << 32 | (uint32_t)b) : ((uint64_t)b << 32 | (uint32_t)a);
      auto it = mid.find(key);
      if (it != mid.end()) return it->second;
      f3 p = normalize((v[a] + v[b]) * 0.5f);
      v.push_back(p);
      return mid[key] = (int)v.size() - 1;
    };
    std::vector<int32_t> nf;
    nf.reserve(f.size() * 4);
    for (size_t k = 0; k < f.size(); k += 3) {
      int a = f[k], b = f[k + 1], c = f[k + 2];
      int ab = midpoint(a, b), bc = midpoint(b, c), ca = midpoint(c, a);
      int add[12] = {a, ab, ca, b, bc, ab, c, ca, bc, ab, bc, ca};
      nf.insert(nf.end(), add, add + 12);
    }
    f.swap(nf);
  }
  // Deterministic low-frequency displacement (a lumpy body) plus two "ears".
  const int K = 12;
  f3 fk[K];
  float ak[K], pk[K];
  for (int k = 0; k < K; k++) {
    fk[k] = mk3(hash01(k, 1) * 2 - 1, hash01(k, 2) * 2 - 1, hash01(k, 3) * 2 - 1) * (2.0f + 4.0f * hash01(k, 4));
    ak[k] = 0.03f + 0.05f * hash01(k, 5);
    pk[k] = 6.2831853f * hash01(k, 6);
  }
  Mesh m;
  m.v.resize(v.size());
  m.uv.resize(v.size());
  const f3 ear0 = normalize(mk3(-0.3f, 1.0f, 0.25f)), ear1 = normalize(mk3(0.3f, 1.0f, 0.25f));
  for (size_t i = 0; i < v.size(); i++) {
    f3 d = v[i];
    double r = 1.0;
    for (int k = 0; k < K; k++) r += ak[k] * sin((double)dot(fk[k], d) + pk[k]);
    double e0 = dot(d, ear0), e1 = dot(d, ear1);
    r += 0.6 * pow(fmax(0.0, e0), 40.0) + 0.6 * pow(fmax(0.0, e1), 40.0);
    f3 p = d * (float)(2.0 * r);
    p.y = p.y * 0.9f + 1.9f;  // squash slightly, rest on y ~ 0
    m.v[i] = p;
    m.uv[i] = mk2((float)(0.5 + atan2((double)d.z, (double)d.x) / (2.0 * M_PI)),
                  (float)(0.5 + asin(fmax(-1.0, fmin(1.0, (double)d.y))) / M_PI));
  }
  m.idx = f;
  // Outward winding: the icosahedron table is CCW-outward; smooth area-weighted normals (double).
  std::vector<double> acc(v.size() * 3, 0.0);
  for (size_t k = 0; k < f.size(); k += 3) {
    f3 a = m.v[f[k]], b = m.v[f[k + 1]], c = m.v[f[k + 2]];
    f3 n = cross(b - a, c - a);
    for (int j = 0; j < 3; j++) {
      acc[f[k + j] * 3 + 0] += n.x; acc[f[k + j] * 3 + 1] += n.y; acc[f[k + j] * 3 + 2] += n.z;
    }
  }
  m.n.resize(v.size());
  for (size_t i = 0; i < v.size(); i++) {
    double x = acc[i * 3], y = acc[i * 3 + 1], z = acc[i * 3 + 2];
    double l = sqrt(x * x + y * y + z * z);
    m.n[i] = l > 0 ? mk3((float)(x / l), (float)(y / l), (float)(z / l)) : mk3(0, 1, 0);
  }
  m.has_n = m.has_uv = true;
  return m;
}

// UV sphere of radius 50 (earth.obj stand-in), analytic normals.
Mesh make_sphere(int slices, int stacks) {
  Mesh m;
  for (int j = 0; j <= stacks; j++) {
    double th = M_PI * j / stacks;
    for (int i = 0; i <= slices; i++) {
      double ph = 2.0 * M_PI * i / slices;
      f3 d = mk3((float)(sin(th) * cos(ph)), (float)cos(th), (float)(sin(th) * sin(ph)));
      m.v.push_back(d * 50.0f);
      m.n.push_back(d);
      m.uv.push_back(mk2((float)i / slices, 1.0f - (float)j / stacks));
    }
  }
  for (int j = 0; j < stacks; j++)
    for (int i = 0; i < slices; i++) {
      int a = j * (slices + 1) + i, b = a + slices + 1;
      // outward: (a, a+1, b) is CCW seen from outside for this parameterisation
      int q[6] = {a, a + 1, b, a + 1, b + 1, b};
      for (int k : q) m.idx.push_back(k);
    }
  m.has_n = m.has_uv = true;
  // Fix winding per triangle to be outward (robust to the parameterisation's handedness).
  for (size_t k = 0; k < m.idx.size(); k += 3) {
    f3 a = m.v[m.idx[k]], b = m.v[m.idx[k + 1]], c = m.v[m.idx[k + 2]];
    f3 n = cross(b - a, c - a);
    if (dot(n, a + b + c) < 0) std::swap(m.idx[k + 1], m.idx[k + 2]);
  }
  return m;
}

// Minecraft-style voxel terrain standing in for vokselia_spawn.obj (identity transform).
Mesh make_voxels(int G, float cell) {
  Mesh m;
  auto height = [&](int x, int z) -> int {
    if (x < 0 || z < 0 || x >= G || z >= G) return 0;
    double h = 0;
    for (int o = 0; o < 4; o++) {
      double fr = (0.02 + 0.03 * hash01(o, 11)) * (1 << o);
      double ph = 6.2831853 * hash01(o, 12), ph2 = 6.2831853 * hash01(o, 13);
      h += (3.0 / (1 << o)) * (sin(x * fr + ph) * cos(z * fr * 1.3 + ph2) + 1.0);
    }
    return (int)h;
  };
  const float x0 = -0.5f * G * cell;
  auto quad = [&](f3 c, f3 u, f3 v, f3 n, float tile_u, float tile_v) {
    int base = (int)m.v.size();
    const float su[4] = {-1, 1, 1, -1}, sv[4] = {-1, -1, 1, 1};
    for (int k = 0; k < 4; k++) {
      m.v.push_back(c + u * (0.5f * cell * su[k]) + v * (0.5f * cell * sv[k]));
      m.n.push_back(n);
      m.uv.push_back(mk2(tile_u + 0.0625f * 0.5f * (su[k] + 1.0f), tile_v + 0.0625f * 0.5f * (sv[k] + 1.0f)));
    }
    int q[6] = {0, 1, 2, 0, 2, 3};
    for (int k : q) m.idx.push_back(base + k);
  };
  for (int z = 0; z < G; z++)
    for (int x = 0; x < G; x++) {
      int h = height(x, z);
      float cx = x0 + (x + 0.5f) * cell, cz = x0 + (z + 0.5f) * cell;
      float top = h * cell;
      int kind = h > 6 ? 2 : (h > 2 ? 0 : 1);  // stone / grass / dirt tiles of the atlas
      float tu = 0.0625f * kind, tv = 0.9375f;
      quad(mk3(cx, top, cz), mk3(0, 0, 1), mk3(1, 0, 0), mk3(0, 1, 0), tu, tv);
      const int dx[4] = {1, -1, 0, 0}, dz[4] = {0, 0, 1, -1};
      for (int s = 0; s < 4; s++) {
        int hn = height(x + dx[s], z + dz[s]);
        for (int y = hn; y < h; y++) {
          f3 n = mk3((float)dx[s], 0, (float)dz[s]);
          f3 c = mk3(cx + 0.5f * cell * dx[s], (y + 0.5f) * cell, cz + 0.5f * cell * dz[s]);
          f3 u = mk3(0, 1, 0);
          f3 v = cross(n, u);
          quad(c, v, u, n, 0.0625f * 3, tv);  // u' x v' must equal n: v x u = -(u x v) = n
        }
      }
    }
  for (size_t k = 0; k < m.idx.size(); k += 3) {  // enforce winding == stored normal
    f3 a = m.v[m.idx[k]], b = m.v[m.idx[k + 1]], c = m.v[m.idx[k + 2]];
    if (dot(cross(b - a, c - a), m.n[m.idx[k]]) < 0) std::swap(m.idx[k + 1], m.idx[k + 2]);
  }
  m.has_n = m.has_uv = true;
  return m;
}

HostTexture procedural_texture(int w, int h, uint32_t salt) {
  HostTexture t;
  t.w = w; t.h = h;
  t.data.resize((size_t)w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int c = ((x / 8) + (y / 8)) & 1;
      float r = (float)((tea16(x + salt, y) & 255)) / 255.0f;
      t.data[(size_t)y * w + x] = mk4(c ? 0.9f : 0.2f + 0.3f * r, c ? 0.8f : 0.4f, c ? 0.7f : 0.6f * r + 0.1f, 1.0f);
    }
  return t;
}

HostTexture procedural_env(int w, int h) {
  HostTexture t;
  t.w = w; t.h = h;
  t.data.resize((size_t)w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      float v = (y + 0.5f) / h;
      float sky = v > 0.5f ? 0.4f + 1.6f * (v - 0.5f) : 0.15f;
      float sun = ((x - w / 3) * (x - w / 3) + (y - 3 * h / 4) * (y - 3 * h / 4)) < 64 ? 40.0f : 0.0f;
      t.data[(size_t)y * w + x] = mk4(sky * 0.6f + sun, sky * 0.75f + sun, sky + sun, 1.0f);
    }
  return t;
}

HostTexture white1x1() {
  HostTexture t;
  t.w = t.h = 1;
  t.data.push_back(mk4(1.0f, 1.0f, 1.0f, 1.0f));  // sutil default colour make_float3(1.0f)
  return t;
}

bool file_exists(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  return (bool)f;
}

}  // namespace

// --------------------------------------------------------------------------------------------
// Texture loaders. Orientation: row 0 of HostTexture is the BOTTOM of the image (v = 0), i.e.
// images are flipped on load as sutil's loaders do for OpenGL-convention lookups.
// --------------------------------------------------------------------------------------------

static bool read_token(std::istream& in, std::string& tok) {
  tok.clear();
  int c;
  while ((c = in.get()) != EOF) {
    if (c == '#') { while ((c = in.get()) != EOF && c != '\n') {} continue; }
    if (!isspace(c)) { tok.push_back((char)c); break; }
  }
  while ((c = in.peek()) != EOF && !isspace(c)) { tok.push_back((char)in.get()); }
  return !tok.empty();
}

// Wavefront OBJ (what sutil::loadMesh reads for the reference's models, FR/PathTracer.cpp:582-595):
// v / vt / vn / f with v, v/vt, v//vn, v/vt/vn corners, 1-based or negative (relative) indices,
// polygons fan-triangulated; other statements (o, g, s, usemtl, mtllib, ...) are ignored: the
// reference binds one material program and texture per model (FR/PathTracer.cpp:676-772).
// Normals / texcoords are kept when every face corner has them.
static bool load_obj(const std::string& path, Mesh& m, std::string& err) {
  std::ifstream f(path);
  if (!f) { err = "cannot open " + path; return false; }
  std::vector<f3> V, N;
  std::vector<f2> T;
  std::map<std::tuple<int, int, int>, int32_t> corner;
  std::vector<std::tuple<int, int, int>> verts;
  bool all_n = true, all_t = true;
  m = Mesh();
  std::string line;
  int lineno = 0;
  auto fix = [](int i, size_t n) { return i > 0 ? i - 1 : (i < 0 ? (int)n + i : -1); };
  while (std::getline(f, line)) {
    lineno++;
    std::istringstream ls(line);
    std::string tag;
    if (!(ls >> tag) || tag[0] == '#') continue;
    if (tag == "v") { float x, y, z; ls >> x >> y >> z; V.push_back(mk3(x, y, z)); }
    else if (tag == "vn") { float x, y, z; ls >> x >> y >> z; N.push_back(mk3(x, y, z)); }
    else if (tag == "vt") { float u = 0, v = 0; ls >> u >> v; T.push_back(mk2(u, v)); }
    else if (tag == "f") {
      std::vector<int32_t> poly;
      std::string c;
      while (ls >> c) {
        int vi = 0, ti = 0, ni = 0;
        size_t s1 = c.find('/');
        vi = atoi(c.substr(0, s1).c_str());
        if (s1 != std::string::npos) {
          size_t s2 = c.find('/', s1 + 1);
          std::string ts = c.substr(s1 + 1, s2 == std::string::npos ? std::string::npos : s2 - s1 - 1);
          if (!ts.empty()) ti = atoi(ts.c_str());
          if (s2 != std::string::npos) ni = atoi(c.substr(s2 + 1).c_str());
        }
        int a = fix(vi, V.size()), b = ti ? fix(ti, T.size()) : -1, d = ni ? fix(ni, N.size()) : -1;
        if (a < 0 || a >= (int)V.size() || b >= (int)T.size() || d >= (int)N.size() || (ti && b < 0) || (ni && d < 0)) {
          err = path + ":" + std::to_string(lineno) + ": face index out of range";
          return false;
        }
        all_t = all_t && b >= 0;
        all_n = all_n && d >= 0;
        auto key = std::make_tuple(a, b, d);
        auto it = corner.find(key);
        if (it == corner.end()) {
          it = corner.emplace(key, (int32_t)verts.size()).first;
          verts.push_back(key);
        }
        poly.push_back(it->second);
      }
      for (size_t k = 1; k + 1 < poly.size(); k++) {
        m.idx.push_back(poly[0]); m.idx.push_back(poly[k]); m.idx.push_back(poly[k + 1]);
      }
    }
  }
  m.has_n = all_n && !verts.empty();
  m.has_uv = all_t && !verts.empty();
  for (auto& k : verts) {
    m.v.push_back(V[std::get<0>(k)]);
    m.n.push_back(m.has_n ? N[std::get<2>(k)] : mk3(0.0f));
    m.uv.push_back(m.has_uv ? T[std::get<1>(k)] : mk2(0.0f, 0.0f));
  }
  if (m.idx.empty()) { err = path + ": no faces"; return false; }
  return true;
}

bool load_ppm(const std::string& path, HostTexture& tex, std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in) { err = "cannot open " + path; return false; }
  std::string magic, sw, sh, sm;
  if (!read_token(in, magic) || !read_token(in, sw) || !read_token(in, sh) || !read_token(in, sm)) {
    err = "bad PPM header: " + path; return false;
  }
  int w = atoi(sw.c_str()), h = atoi(sh.c_str()), maxv = atoi(sm.c_str());
  if (w <= 0 || h <= 0 || maxv <= 0 || maxv > 255 || (magic != "P6" && magic != "P3")) {
    err = "unsupported PPM: " + path; return false;
  }
  std::vector<unsigned char> raw((size_t)w * h * 3);
  if (magic == "P6") {
    in.get();  // single whitespace after maxval
    in.read((char*)raw.data(), raw.size());
    if ((size_t)in.gcount() != raw.size()) { err = "truncated PPM: " + path; return false; }
  } else {
    std::string tok;
    for (size_t i = 0; i < raw.size(); i++) {
      if (!read_token(in, tok)) { err = "truncated PPM: " + path; return false; }
      raw[i] = (unsigned char)atoi(tok.c_str());
    }
  }
  tex.w = w; tex.h = h;
  tex.data.resize((size_t)w * h);
  const float scale = (float)maxv;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const unsigned char* p = &raw[((size_t)(h - 1 - y) * w + x) * 3];
      tex.data[(size_t)y * w + x] = mk4((float)p[0] / scale, (float)p[1] / scale, (float)p[2] / scale, 1.0f);
    }
  return true;
}

bool load_hdr(const std::string& path, HostTexture& tex, std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in) { err = "cannot open " + path; return false; }
  std::string line;
  bool rgbe = false;
  while (std::getline(in, line)) {
    if (line.empty()) break;
    if (line.find("FORMAT=32-bit_rle_rgbe") != std::string::npos) rgbe = true;
  }
  if (!rgbe) { err = "not an RGBE .hdr: " + path; return false; }
  if (!std::getline(in, line)) { err = "missing resolution line: " + path; return false; }
  char ya[4] = {0}, xa[4] = {0};
  int h = 0, w = 0;
  if (sscanf(line.c_str(), "%2s %d %2s %d", ya, &h, xa, &w) != 4 || std::string(ya) != "-Y" || std::string(xa) != "+X") {
    err = "unsupported HDR orientation: " + line; return false;
  }
  std::vector<unsigned char> img((size_t)w * h * 4);
  std::vector<unsigned char> scan((size_t)w * 4);
  for (int y = 0; y < h; y++) {
    unsigned char hdr4[4];
    in.read((char*)hdr4, 4);
    if (!in) { err = "truncated HDR: " + path; return false; }
    if (w >= 8 && w < 32768 && hdr4[0] == 2 && hdr4[1] == 2 && ((hdr4[2] << 8) | hdr4[3]) == w) {
      for (int c = 0; c < 4; c++) {
        int x = 0;
        while (x < w) {
          int n = in.get();
          if (n == EOF) { err = "truncated HDR RLE: " + path; return false; }
          if (n > 128) {
            n -= 128;
            int v = in.get();
            for (int k = 0; k < n && x < w; k++) scan[(x++) * 4 + c] = (unsigned char)v;
          } else {
            for (int k = 0; k < n && x < w; k++) scan[(x++) * 4 + c] = (unsigned char)in.get();
          }
        }
      }
    } else {  // flat scanline
      memcpy(&scan[0], hdr4, 4);
      in.read((char*)&scan[4], (w - 1) * 4);
    }
    memcpy(&img[(size_t)y * w * 4], scan.data(), (size_t)w * 4);
  }
  tex.w = w; tex.h = h;
  tex.data.resize((size_t)w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const unsigned char* p = &img[((size_t)(h - 1 - y) * w + x) * 4];
      float f = p[3] == 0 ? 0.0f : ldexpf(1.0f, (int)p[3] - 136);  // m * 2^(e-128-8)
      tex.data[(size_t)y * w + x] = mk4(p[0] * f, p[1] * f, p[2] * f, 1.0f);
    }
  return true;
}

bool load_png(const std::string& path, HostTexture& tex, std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in) { err = "cannot open " + path; return false; }
  std::vector<unsigned char> file((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (file.size() < 8 || memcmp(file.data(), sig, 8) != 0) { err = "not a PNG: " + path; return false; }
  size_t p = 8;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = 0, interlace = 0;
  std::vector<unsigned char> idat;
  auto be32 = [&](size_t o) { return (uint32_t)file[o] << 24 | (uint32_t)file[o + 1] << 16 | (uint32_t)file[o + 2] << 8 | file[o + 3]; };
  while (p + 8 <= file.size()) {
    uint32_t len = be32(p);
    std::string type((const char*)&file[p + 4], 4);
    if (p + 12 + len > file.size()) break;
    const unsigned char* d = &file[p + 8];
    if (type == "IHDR") {
      w = be32(p + 8); h = be32(p + 12); depth = d[8]; ctype = d[9]; interlace = d[12];
    } else if (type == "IDAT") {
      idat.insert(idat.end(), d, d + len);
    } else if (type == "IEND") break;
    p += 12 + len;
  }
  int ch = ctype == 6 ? 4 : (ctype == 2 ? 3 : 0);
  if (!w || !h || depth != 8 || ch == 0 || interlace) { err = "unsupported PNG (need 8-bit RGB/RGBA, no interlace): " + path; return false; }
  size_t stride = (size_t)w * ch;
  std::vector<unsigned char> raw((stride + 1) * h);
  uLongf rl = raw.size();
  if (uncompress(raw.data(), &rl, idat.data(), idat.size()) != Z_OK || rl != raw.size()) { err = "PNG inflate failed: " + path; return false; }
  std::vector<unsigned char> img(stride * h);
  for (uint32_t y = 0; y < h; y++) {
    int ft = raw[y * (stride + 1)];
    const unsigned char* src = &raw[y * (stride + 1) + 1];
    unsigned char* dst = &img[y * stride];
    const unsigned char* up = y ? &img[(y - 1) * stride] : nullptr;
    for (size_t i = 0; i < stride; i++) {
      int a = i >= (size_t)ch ? dst[i - ch] : 0, b = up ? up[i] : 0, c = (up && i >= (size_t)ch) ? up[i - ch] : 0;
      int v = src[i];
      switch (ft) {
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: { int pp = a + b - c, pa = abs(pp - a), pb = abs(pp - b), pc = abs(pp - c);
                  v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c); break; }
        default: break;
      }
      dst[i] = (unsigned char)v;
    }
  }
  tex.w = (int)w; tex.h = (int)h;
  tex.data.resize((size_t)w * h);
  for (uint32_t y = 0; y < h; y++)
    for (uint32_t x = 0; x < w; x++) {
      const unsigned char* q = &img[(size_t)(h - 1 - y) * stride + x * ch];
      tex.data[(size_t)y * w + x] = mk4(q[0] / 255.0f, q[1] / 255.0f, q[2] / 255.0f, ch == 4 ? q[3] / 255.0f : 1.0f);
    }
  return true;
}

void preset_camera(int preset, f3& eye, f3& target) {
  switch (preset) {
    case PRESET_BOX: eye = mk3(-3.5f, 1.2f, 3.5f); target = mk3(-3.5f, 0.7f, 1.2f); break;
    case PRESET_BUNNY: eye = mk3(0.5f, 2.4f, 4.9f); target = mk3(-0.2f, 0.92f, 0.46f); break;  // FR/main.cpp:203
    default: eye = mk3(-0.123401f, 8.361134f, -0.223597f); target = mk3(-3.992834f, -155.545700f, 6.774422f);  // :191
  }
}

bool build_preset_scene(int preset, const std::string& asset_dir, int texture_mode, float light_power, int detail,
                        HostScene& sc, std::string& err, int mesh_mode) {
  sc = HostScene();
  sc.bbox_min = mk3(INFINITY);
  sc.bbox_max = mk3(-INFINITY);
  // ParallelogramLight (FR/PathTracer.cpp:564-579)
  sc.light_position = mk3(343.0f, 548.6f, 227.0f);
  sc.light_v1 = mk3(-130.0f, 0.0f, 0.0f);
  sc.light_v2 = mk3(0.0f, 0.0f, 105.0f);
  sc.light_normal = normalize(cross(sc.light_v1, sc.light_v2));
  sc.light_emission = mk3(light_power);

  auto tex = [&](const std::string& rel, int pw, int ph, uint32_t salt, int& out) -> bool {
    HostTexture t;
    if (texture_mode == 1) t = procedural_texture(pw, ph, salt);
    else {
      std::string path = asset_dir + "/" + rel;
      std::string ext = rel.substr(rel.find_last_of('.') + 1);
      for (auto& c : ext) c = (char)tolower(c);
      bool ok = ext == "ppm" ? load_ppm(path, t, err) : ext == "hdr" ? load_hdr(path, t, err) : load_png(path, t, err);
      if (!ok) return false;
    }
    out = (int)sc.texs.size();
    sc.texs.push_back(std::move(t));
    return true;
  };
  // Environment map: CedarCity.hdr (FR/PathTracer.cpp:454-455)
  if (texture_mode == 1) { sc.envmap = (int)sc.texs.size(); sc.texs.push_back(procedural_env(1600, 800)); }
  else if (!tex("CedarCity.hdr", 1600, 800, 0, sc.envmap)) return false;

  int t_grid = -1, t_bunny = -1, t_white = -1, t_vox = -1;
  if (!tex("grid.ppm", 64, 64, 1, t_grid)) return false;
  t_white = (int)sc.texs.size();
  sc.texs.push_back(white1x1());  // earth: texture "none" -> default (1,1,1) (FR/PathTracer.cpp:593)

  // The reference's meshes (FR/PathTracer.cpp:582-595) when they are present under asset_dir
  // (mesh_mode 0) or required (2); the deterministic procedural stand-in otherwise (0) or always (1).
  auto mesh = [&](const char* rel, Mesh& m, const std::function<Mesh()>& procedural) -> bool {
    const std::string path = asset_dir + "/" + rel;
    if (mesh_mode != 1 && (mesh_mode == 2 || file_exists(path))) return load_obj(path, m, err);
    m = procedural();
    return true;
  };
  auto mat = [&](int type, int texid) {
    sc.mats.push_back(DevMaterial{type, texid});
    return (int)sc.mats.size() - 1;
  };
  // model 0: ground (diffuse, grid.ppm, translate(0,-0.05,0))
  {
    Mesh g;
    if (!mesh("ground.obj", g, make_ground)) return false;
    bake(g, mk3(0.0f, -0.05f, 0.0f), 1.0f);
    add_mesh(sc, g, mat(MATL_DIFFUSE, t_grid), "ground");
  }
  // model 1: vokselia_spawn (diffuse, identity)
  if (preset == PRESET_VOKSELIA) {
    if (texture_mode == 1) { t_vox = (int)sc.texs.size(); sc.texs.push_back(procedural_texture(256, 256, 7)); }
    else if (!tex("vokselia_spawn/vokselia_spawn.png", 0, 0, 0, t_vox)) return false;
    int G = detail > 0 ? 96 * detail : 320;
    Mesh v;
    if (!mesh("vokselia_spawn/vokselia_spawn.obj", v, [&] { return make_voxels(G, 0.125f); })) return false;
    add_mesh(sc, v, mat(MATL_DIFFUSE, t_vox), "vokselia_spawn");
  }
  // model 2: box (refraction, grid.ppm per the code, translate(-3.5,0.2,1.2)*scale(0.01))
  {
    Mesh b;
    if (!mesh("box/box.obj", b, make_cube)) return false;
    bake(b, mk3(-3.5f, 0.2f, 1.2f), 0.01f);
    add_mesh(sc, b, mat(MATL_REFRACTION, t_grid), "box");
  }
  // model 3: bunny (refraction, bunny.ppm, translate(-1.5,0.2,1.2)*scale(0.25))
  if (preset != PRESET_BOX) {
    if (!tex("bunny/bunny.PPM", 1024, 1024, 3, t_bunny)) return false;
    int sub = detail > 0 ? std::min(detail + 3, 7) : 6;
    Mesh bn;
    if (!mesh("bunny/bunny.obj", bn, [&] { return make_blob(sub); })) return false;
    bake(bn, mk3(-1.5f, 0.2f, 1.2f), 0.25f);
    add_mesh(sc, bn, mat(MATL_REFRACTION, t_bunny), "bunny");
    // model 4: earth (reflection, white, translate(0,1,0)*scale(0.01))
    Mesh e;
    if (!mesh("earth/earth.obj", e, [] { return make_sphere(64, 32); })) return false;
    bake(e, mk3(0.0f, 1.0f, 0.0f), 0.01f);
    add_mesh(sc, e, mat(MATL_REFLECTION, t_white), "earth");
  }
  if ((int)sc.texs.size() > FR_MAX_TEXTURES || (int)sc.mats.size() > FR_MAX_MATERIALS) { err = "too many textures/materials"; return false; }
  return true;
}

// --------------------------------------------------------------------------------------------
// Binned SAH BVH
// --------------------------------------------------------------------------------------------
namespace {
struct Box {
  f3 lo = mk3(INFINITY), hi = mk3(-INFINITY);
  void grow(f3 p) {
    lo = mk3(fminf(lo.x, p.x), fminf(lo.y, p.y), fminf(lo.z, p.z));
    hi = mk3(fmaxf(hi.x, p.x), fmaxf(hi.y, p.y), fmaxf(hi.z, p.z));
  }
  void grow(const Box& b) { grow(b.lo); grow(b.hi); }
  float area() const {
    f3 d = hi - lo;
    if (d.x < 0) return 0;
    return 2.0f * (d.x * d.y + d.y * d.z + d.z * d.x);
  }
};
float inflate_lo(float v) { return v - (1e-5f + 4e-7f * fabsf(v)); }
float inflate_hi(float v) { return v + (1e-5f + 4e-7f * fabsf(v)); }

struct Builder {
  const HostScene& s;
  std::vector<Box> tb;
  std::vector<f3> cen;
  std::vector<int32_t> ids;
  Bvh& out;
  static constexpr int kMaxBins = 64, kMaxDepth = 30;
  int kLeaf = 2, kBins = 16;  // leaf size and SAH bins (FOVRT_BVH_LEAF / FOVRT_BVH_BINS override, for tuning)
  int kSplit = 0;             // FOVRT_BVH_SPLIT: 0 binned on the widest centroid axis; 1 binned on all three
                              // axes; 2 exact sweep over the sorted centroids of all three axes
  Builder(const HostScene& sc, Bvh& o) : s(sc), out(o) {
    if (const char* v = getenv("FOVRT_BVH_LEAF")) kLeaf = std::max(1, std::min(8, atoi(v)));
    if (const char* v = getenv("FOVRT_BVH_BINS")) kBins = std::max(2, std::min(kMaxBins, atoi(v)));
    if (const char* v = getenv("FOVRT_BVH_SPLIT")) kSplit = std::max(0, std::min(2, atoi(v)));
  }
  static float axis_of(f3 c, int a) { return a == 0 ? c.x : a == 1 ? c.y : c.z; }
  // Exact SAH sweep on all three axes: sorts [b, e) by the best axis and returns the split point.
  int split_sweep(int b, int e) {
    const int n = e - b;
    std::vector<float> right(n);
    float best = INFINITY;
    int best_axis = -1, best_i = -1;
    std::vector<int32_t> tmp(ids.begin() + b, ids.begin() + e);
    for (int a = 0; a < 3; a++) {
      std::sort(tmp.begin(), tmp.end(), [&](int x, int y) {
        const float kx = axis_of(cen[x], a), ky = axis_of(cen[y], a);
        return kx < ky || (kx == ky && x < y);
      });
      Box r;
      for (int i = n - 1; i >= 1; i--) { r.grow(tb[tmp[i]]); right[i] = r.area(); }
      Box l;
      for (int i = 1; i < n; i++) {
        l.grow(tb[tmp[i - 1]]);
        const float c = l.area() * i + right[i] * (n - i);
        if (c < best) { best = c; best_axis = a; best_i = i; }
      }
    }
    if (best_axis < 0) return -1;
    std::sort(ids.begin() + b, ids.begin() + e, [&](int x, int y) {
      const float kx = axis_of(cen[x], best_axis), ky = axis_of(cen[y], best_axis);
      return kx < ky || (kx == ky && x < y);
    });
    return b + best_i;
  }
  // Binned SAH on all three axes.
  int split_binned3(int b, int e, const Box& cb) {
    float best = INFINITY;
    int best_axis = -1, best_k = -1;
    for (int a = 0; a < 3; a++) {
      const float lo = axis_of(cb.lo, a), ex = axis_of(cb.hi, a) - lo;
      if (!(ex > 0.0f)) continue;
      Box bins[kMaxBins];
      int cnt[kMaxBins] = {0};
      for (int i = b; i < e; i++) {
        int k = (int)((axis_of(cen[ids[i]], a) - lo) / ex * kBins);
        k = k < 0 ? 0 : (k >= kBins ? kBins - 1 : k);
        cnt[k]++; bins[k].grow(tb[ids[i]]);
      }
      float ra[kMaxBins]; int rn[kMaxBins];
      Box r; int nr = 0;
      for (int k = kBins - 1; k >= 1; k--) { if (cnt[k]) { r.grow(bins[k]); nr += cnt[k]; } ra[k] = r.area(); rn[k] = nr; }
      Box l; int nl = 0;
      for (int k = 1; k < kBins; k++) {
        if (cnt[k - 1]) { l.grow(bins[k - 1]); nl += cnt[k - 1]; }
        if (!nl || !rn[k]) continue;
        const float c = l.area() * nl + ra[k] * rn[k];
        if (c < best) { best = c; best_axis = a; best_k = k; }
      }
    }
    if (best_axis < 0) return -1;
    const float lo = axis_of(cb.lo, best_axis), ex = axis_of(cb.hi, best_axis) - lo;
    return (int)(std::partition(ids.begin() + b, ids.begin() + e, [&](int id) {
             int k = (int)((axis_of(cen[id], best_axis) - lo) / ex * kBins);
             k = k < 0 ? 0 : (k >= kBins ? kBins - 1 : k);
             return k < best_k;
           }) - ids.begin());
  }

  Box range_box(int b, int e) const { Box bx; for (int i = b; i < e; i++) bx.grow(tb[ids[i]]); return bx; }

  void emit_leaf(int b, int e, int32_t& child, int32_t& count) {
    child = (int32_t)out.tri_prim.size();
    count = e - b;
    for (int i = b; i < e; i++) out.tri_prim.push_back(ids[i]);
  }
  // Splits [b,e) and returns the split point; returns -1 if it should be a leaf.
  int split(int b, int e, int depth) {
    int n = e - b;
    if (n <= kLeaf || depth >= kMaxDepth) return -1;
    Box cb;
    for (int i = b; i < e; i++) cb.grow(cen[ids[i]]);
    f3 ext = cb.hi - cb.lo;
    int axis = ext.x > ext.y ? (ext.x > ext.z ? 0 : 2) : (ext.y > ext.z ? 1 : 2);
    float lo = axis == 0 ? cb.lo.x : axis == 1 ? cb.lo.y : cb.lo.z;
    float ex = axis == 0 ? ext.x : axis == 1 ? ext.y : ext.z;
    auto key = [&](int id) { f3 c = cen[id]; return axis == 0 ? c.x : axis == 1 ? c.y : c.z; };
    int mid = -1;
    if (kSplit == 2) {
      mid = split_sweep(b, e);
    } else if (kSplit == 1) {
      mid = split_binned3(b, e, cb);
    } else if (ex > 0.0f) {
      Box bins[kMaxBins];
      int cnt[kMaxBins] = {0};
      auto bin_of = [&](int id) { int k = (int)((key(id) - lo) / ex * kBins); return k < 0 ? 0 : (k >= kBins ? kBins - 1 : k); };
      for (int i = b; i < e; i++) { int k = bin_of(ids[i]); cnt[k]++; bins[k].grow(tb[ids[i]]); }
      float best = INFINITY;
      int best_k = -1;
      for (int k = 1; k < kBins; k++) {
        Box l, r; int nl = 0, nr = 0;
        for (int j = 0; j < k; j++) { if (cnt[j]) { l.grow(bins[j]); nl += cnt[j]; } }
        for (int j = k; j < kBins; j++) { if (cnt[j]) { r.grow(bins[j]); nr += cnt[j]; } }
        if (!nl || !nr) continue;
        float c = l.area() * nl + r.area() * nr;
        if (c < best) { best = c; best_k = k; }
      }
      if (best_k > 0) {
        mid = (int)(std::partition(ids.begin() + b, ids.begin() + e, [&](int id) { return bin_of(id) < best_k; }) - ids.begin());
      }
    }
    if (mid <= b || mid >= e) {  // degenerate: median split on the axis
      mid = b + n / 2;
      std::nth_element(ids.begin() + b, ids.begin() + mid, ids.begin() + e,
                       [&](int x, int y) { return key(x) < key(y) || (key(x) == key(y) && x < y); });
    }
    return mid;
  }
  // Binary build: node i has children (box2[2i+k], child2[2i+k], count2[2i+k]), k = 0, 1.
  std::vector<Box> box2;
  std::vector<int32_t> child2, count2;
  int new_node2() {
    box2.resize(box2.size() + 2); child2.resize(child2.size() + 2); count2.resize(count2.size() + 2);
    return (int)child2.size() / 2 - 1;
  }
  void build_node(int ni, int b, int mid, int e, int depth) {
    int ranges[2][2] = {{b, mid}, {mid, e}};
    for (int k = 0; k < 2; k++) {
      int cb = ranges[k][0], ce = ranges[k][1];
      box2[2 * ni + k] = range_box(cb, ce);
      int sp = split(cb, ce, depth + 1);
      if (sp < 0) {
        int32_t c, cnt;
        emit_leaf(cb, ce, c, cnt);
        child2[2 * ni + k] = c; count2[2 * ni + k] = cnt;
      } else {
        int child = new_node2();
        child2[2 * ni + k] = child; count2[2 * ni + k] = 0;
        build_node(child, cb, sp, ce, depth + 1);
      }
    }
  }
  // Collapse into four-wide nodes: repeatedly open the largest-area inner entry until four entries.
  // The inner children of a node are stored contiguously, so one traversal stack entry (the base
  // index + the near-to-far order of the remaining children) covers a whole level.
  struct Entry { Box box; int32_t child, count; };
  void collapse(const std::vector<Entry>& seed, int ni, int depth, int stack_need) {
    std::vector<Entry> ents = seed;
    while (ents.size() < 4) {
      int best = -1; float ba = -1.0f;
      for (size_t i = 0; i < ents.size(); i++)
        if (ents[i].count == 0 && ents[i].box.area() > ba) { ba = ents[i].box.area(); best = (int)i; }
      if (best < 0) break;
      int n2 = ents[best].child;
      ents.erase(ents.begin() + best);
      for (int k = 0; k < 2; k++) ents.push_back(Entry{box2[2 * n2 + k], child2[2 * n2 + k], count2[2 * n2 + k]});
    }
    out.max_depth = std::max(out.max_depth, depth);
    int inner = 0;
    for (auto& e : ents) inner += e.count == 0;
    const int need = stack_need + (inner > 1 ? 1 : 0);
    out.max_stack = std::max(out.max_stack, need);
    const int base = (int)out.nodes.size();
    out.nodes.resize(out.nodes.size() + inner);
    BvhNode& nd = out.nodes[ni];
    float* LX = &nd.lox.x; float* HX = &nd.hix.x;
    float* LY = &nd.loy.x; float* HY = &nd.hiy.x;
    float* LZ = &nd.loz.x; float* HZ = &nd.hiz.x;
    int r = 0;
    for (int k = 0; k < 4; k++) {
      if (k >= (int)ents.size()) {
        LX[k] = LY[k] = LZ[k] = INFINITY; HX[k] = HY[k] = HZ[k] = -INFINITY;
        nd.child[k] = 0; nd.count[k] = -1;
        continue;
      }
      const Box& bx = ents[k].box;
      LX[k] = inflate_lo(bx.lo.x); HX[k] = inflate_hi(bx.hi.x);
      LY[k] = inflate_lo(bx.lo.y); HY[k] = inflate_hi(bx.hi.y);
      LZ[k] = inflate_lo(bx.lo.z); HZ[k] = inflate_hi(bx.hi.z);
      nd.count[k] = ents[k].count;
      nd.child[k] = ents[k].count == 0 ? base + r++ : ents[k].child;
    }
    r = 0;
    for (int k = 0; k < (int)ents.size(); k++) {
      if (ents[k].count != 0) continue;
      int n2 = ents[k].child;
      std::vector<Entry> sub = {Entry{box2[2 * n2], child2[2 * n2], count2[2 * n2]},
                                Entry{box2[2 * n2 + 1], child2[2 * n2 + 1], count2[2 * n2 + 1]}};
      collapse(sub, base + r++, depth + 1, need);
    }
  }
  void run() {
    int n = s.num_tris();
    tb.resize(n); cen.resize(n); ids.resize(n);
    for (int i = 0; i < n; i++) {
      Box b; b.grow(s.pos[3 * i]); b.grow(s.pos[3 * i + 1]); b.grow(s.pos[3 * i + 2]);
      tb[i] = b;
      cen[i] = (b.lo + b.hi) * 0.5f;
      ids[i] = i;
    }
    out.nodes.clear(); out.tri_prim.clear(); out.max_depth = 0; out.max_stack = 0; out.root_count = 0;
    box2.clear(); child2.clear(); count2.clear();
    int sp = split(0, n, 0);
    std::vector<Entry> root;
    if (sp < 0) {  // tiny scene: the root holds one leaf
      int32_t c, cnt; emit_leaf(0, n, c, cnt);
      root.push_back(Entry{range_box(0, n), c, cnt});
    } else {
      int r = new_node2();
      build_node(r, 0, sp, n, 0);
      root.push_back(Entry{box2[0], child2[0], count2[0]});
      root.push_back(Entry{box2[1], child2[1], count2[1]});
    }
    out.nodes.resize(1);
    collapse(root, 0, 0, 0);
    // Re-lay the triangles so that the leaf children of every node are one contiguous range in slot
    // order: a traversal step tests its node's hit leaves in a single loop.
    {
      std::vector<int32_t> prim;
      prim.reserve(out.tri_prim.size());
      for (auto& nd : out.nodes)
        for (int k = 0; k < 4; k++)
          if (nd.count[k] > 0) {
            const int first = (int)prim.size();
            for (int j = 0; j < nd.count[k]; j++) prim.push_back(out.tri_prim[nd.child[k] + j]);
            nd.child[k] = first;
          }
      out.tri_prim.swap(prim);
    }
    out.tri_geo.resize(out.tri_prim.size());
    for (size_t i = 0; i < out.tri_prim.size(); i++) {
      int p = out.tri_prim[i];
      f3 p0 = s.pos[3 * p], p1 = s.pos[3 * p + 1], p2 = s.pos[3 * p + 2];
      f3 e0 = p1 - p0, e1 = p0 - p2, nn = cross(e1, e0);
      out.tri_geo[i].a = mk4(p0.x, p0.y, p0.z, e0.x);
      out.tri_geo[i].b = mk4(e0.y, e0.z, e1.x, e1.y);
      out.tri_geo[i].c = mk4(e1.z, nn.x, nn.y, nn.z);
    }
  }
};
}  // namespace

void build_bvh(const HostScene& s, Bvh& out) {
  Builder b(s, out);
  b.run();
}

}  // namespace fr
