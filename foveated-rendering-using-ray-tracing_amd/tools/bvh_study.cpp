// bvh_study — offline study of BVH layouts on a recorded megakernel query stream (diagnostic tool,
// not part of the library). It replays the queries through a host copy of the engine's traversal
// (k_trace.hip trav_step: same node order, same leaf-range steps) and reports, per query:
//   steps      trav_step calls (one node visit and / or one triangle pair each),
//   visits     node visits,
//   tris       triangles tested, and how many of them lie in a leaf whose box the ray hit,
//   wave64     the mean over waves of 64 consecutive queries of the longest query's steps
//              (the wave-uniform traversal loop runs until its slowest lane is done).
// Queries: the diagnostic build's dump (FOVRT_DIAG_DUMP, every 16th query of one 4K bunny frame:
// f4 (o, tmax), f4 (d, any)). Builder knobs are the library's environment variables.
//   bvh_study <queries.bin> [scene=1] [asset_dir=assets]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "../csrc/scene.h"

using namespace fr;

namespace {

struct Stats {
  double steps = 0, visits = 0, tris = 0, useful = 0, wave_steps = 0, hits = 0;
  size_t n = 0;
};

struct Sim {
  const Bvh& b;
  const HostScene& s;
  bool mask_tris;  // test only the triangles of hit leaves (FOVRT_STUDY_MASK=1)

  static float fma_(float a, float b, float c) { return std::fma(a, b, c); }

  // slab4 of k_trace.hip
  void slab4(const BvhNode& nd, f3 o, f3 inv, float tmin, float tmax, float key[4]) const {
    const float* LX = &nd.lox.x; const float* HX = &nd.hix.x;
    const float* LY = &nd.loy.x; const float* HY = &nd.hiy.x;
    const float* LZ = &nd.loz.x; const float* HZ = &nd.hiz.x;
    const float oix = -o.x * inv.x, oiy = -o.y * inv.y, oiz = -o.z * inv.z;
    for (int k = 0; k < 4; k++) {
      const float x0 = fma_(LX[k], inv.x, oix), x1 = fma_(HX[k], inv.x, oix);
      const float y0 = fma_(LY[k], inv.y, oiy), y1 = fma_(HY[k], inv.y, oiy);
      const float z0 = fma_(LZ[k], inv.z, oiz), z1 = fma_(HZ[k], inv.z, oiz);
      const float n = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), tmin));
      const float f = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tmax));
      key[k] = n <= f ? n : INFINITY;
    }
  }

  bool tri_test(const TriGeo& g, f3 o, f3 d, float tmin, float tmax, float& t) const {
    f3 p0 = mk3(g.a.x, g.a.y, g.a.z), e0 = mk3(g.a.w, g.b.x, g.b.y), e1 = mk3(g.b.z, g.b.w, g.c.x);
    f3 n = mk3(g.c.y, g.c.z, g.c.w);
    f3 e2 = (1.0f / dot(n, d)) * (p0 - o);
    f3 i = cross(d, e2);
    const float beta = dot(i, e1), gamma = dot(i, e0);
    t = dot(n, e2);
    return (t < tmax) & (t > tmin) & (beta >= 0.0f) & (gamma >= 0.0f) & (beta + gamma <= 1.0f);
  }

  // One query; returns steps. Mirrors trav_step (leaf-step form, one pair per step).
  int query(f3 o, f3 d, float tmin, float tmax, bool any, Stats& st) const {
    f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    float best = tmax;
    int node = 0, steps = 0;
    int tlo = 0, thi = 0, mbase = 0;
    uint32_t tmask = 0;  // triangles of hit leaves: bit j -> triangle mbase + j
    int stack[64];
    int sp = 0;
    while (true) {
      steps++;
      if (tlo >= thi) {
        const BvhNode& nd = b.nodes[node];
        st.visits++;
        float key[4];
        slab4(nd, o, inv, tmin, best, key);
        int lo = 0x7FFFFFFF, hi = 0;
        for (int k = 0; k < 4; k++)
          if (key[k] != INFINITY && nd.count[k] > 0) { lo = std::min(lo, nd.child[k]); hi = std::max(hi, nd.child[k] + nd.count[k]); }
        tlo = lo; thi = hi; mbase = lo; tmask = 0;
        for (int k = 0; k < 4; k++)
          if (key[k] != INFINITY && nd.count[k] > 0)
            for (int j = 0; j < nd.count[k]; j++) tmask |= 1u << (nd.child[k] + j - lo);
        int c[4]; float kk[4];
        int m = 0;
        for (int k = 0; k < 4; k++) if (nd.count[k] == 0 && key[k] != INFINITY) { c[m] = nd.child[k]; kk[m] = key[k]; m++; }
        for (int a = 0; a < m; a++) for (int q = a + 1; q < m; q++) if (kk[q] < kk[a]) { std::swap(kk[q], kk[a]); std::swap(c[q], c[a]); }
        if (m) {
          for (int a = m - 1; a >= 1; a--) stack[sp++] = c[a];
          node = c[0];
        } else if (sp == 0) {
          node = -1;
        } else {
          node = stack[--sp];
        }
      }
      if (tlo < thi) {
        int tested = 0;
        while (tlo < thi && tested < 2) {
          const int j = tlo++;
          const bool in = (tmask >> (j - mbase)) & 1u;
          if (mask_tris && !in) continue;
          tested++;
          st.tris++;
          st.useful += in;
          float t;
          if (tri_test(b.tri_geo[j], o, d, tmin, any ? tmax : best, t)) {
            if (!any) {
              best = std::min(best, t);
            } else {
              const int prim = b.tri_prim[j];
              const int mat = s.flags[prim] & 0xff;
              if (s.mats[mat].type != MATL_REFRACTION) { st.hits++; return steps; }
            }
          }
        }
        if (mask_tris && tlo < thi && !((tmask >> (tlo - mbase)) >> 0)) tlo = thi;  // no hit-leaf triangle left
      }
      if (tlo >= thi && node < 0) {
        if (!any && best < tmax) st.hits++;
        return steps;
      }
    }
  }
};

// ---- generic-width study tree: the engine's binned SAH binary build, collapsed to `width` children
// per node (largest-area inner entry opened first), leaf children in one contiguous triangle range.
struct GBox {
  f3 lo = mk3(INFINITY), hi = mk3(-INFINITY);
  void grow(f3 p) { lo = mk3(fminf(lo.x, p.x), fminf(lo.y, p.y), fminf(lo.z, p.z)); hi = mk3(fmaxf(hi.x, p.x), fmaxf(hi.y, p.y), fmaxf(hi.z, p.z)); }
  void grow(const GBox& b) { grow(b.lo); grow(b.hi); }
  float area() const { f3 d = hi - lo; return d.x < 0 ? 0.0f : 2.0f * (d.x * d.y + d.y * d.z + d.z * d.x); }
};
struct GNode { std::vector<GBox> box; std::vector<int> child, count; };
struct GTree {
  std::vector<GNode> nodes;
  std::vector<int> prim;  // leaf order
};
struct GBuilder {
  const HostScene& s;
  int width, leaf = 2, bins = 16;
  std::vector<GBox> tb; std::vector<f3> cen; std::vector<int> ids;
  struct B2 { GBox box[2]; int child[2], count[2]; };
  std::vector<B2> bin;
  std::vector<int> lprim;
  GTree out;
  int split(int b, int e) {
    const int n = e - b;
    if (n <= leaf) return -1;
    GBox cb; for (int i = b; i < e; i++) cb.grow(cen[ids[i]]);
    f3 ext = cb.hi - cb.lo;
    int axis = ext.x > ext.y ? (ext.x > ext.z ? 0 : 2) : (ext.y > ext.z ? 1 : 2);
    auto key = [&](int id) { f3 c = cen[id]; return axis == 0 ? c.x : axis == 1 ? c.y : c.z; };
    const float lo = axis == 0 ? cb.lo.x : axis == 1 ? cb.lo.y : cb.lo.z, ex = axis == 0 ? ext.x : axis == 1 ? ext.y : ext.z;
    int mid = -1;
    if (ex > 0) {
      GBox bx[64]; int cnt[64] = {0};
      auto bof = [&](int id) { int k = (int)((key(id) - lo) / ex * bins); return k < 0 ? 0 : k >= bins ? bins - 1 : k; };
      for (int i = b; i < e; i++) { int k = bof(ids[i]); cnt[k]++; bx[k].grow(tb[ids[i]]); }
      float best = INFINITY; int bk = -1;
      for (int k = 1; k < bins; k++) {
        GBox l, r; int nl = 0, nr = 0;
        for (int j = 0; j < k; j++) if (cnt[j]) { l.grow(bx[j]); nl += cnt[j]; }
        for (int j = k; j < bins; j++) if (cnt[j]) { r.grow(bx[j]); nr += cnt[j]; }
        if (!nl || !nr) continue;
        float c = l.area() * nl + r.area() * nr;
        if (c < best) { best = c; bk = k; }
      }
      if (bk > 0) mid = (int)(std::partition(ids.begin() + b, ids.begin() + e, [&](int id) { return bof(id) < bk; }) - ids.begin());
    }
    if (mid <= b || mid >= e) { mid = b + n / 2; std::nth_element(ids.begin() + b, ids.begin() + mid, ids.begin() + e, [&](int x, int y) { return key(x) < key(y) || (key(x) == key(y) && x < y); }); }
    return mid;
  }
  int build2(int b, int e, int sp) {  // returns binary node index
    int ni = (int)bin.size(); bin.emplace_back();
    int r[2][2] = {{b, sp}, {sp, e}};
    for (int k = 0; k < 2; k++) {
      GBox bx; for (int i = r[k][0]; i < r[k][1]; i++) bx.grow(tb[ids[i]]);
      bin[ni].box[k] = bx;
      int s2 = split(r[k][0], r[k][1]);
      if (s2 < 0) { bin[ni].child[k] = (int)lprim.size(); bin[ni].count[k] = r[k][1] - r[k][0]; for (int i = r[k][0]; i < r[k][1]; i++) lprim.push_back(ids[i]); }
      else { int c = build2(r[k][0], r[k][1], s2); bin[ni].child[k] = c; bin[ni].count[k] = 0; }
    }
    return ni;
  }
  struct E { GBox box; int child, count; };
  void collapse(std::vector<E> ents, int gi) {
    while ((int)ents.size() < width) {
      int best = -1; float ba = -1;
      for (size_t i = 0; i < ents.size(); i++) if (ents[i].count == 0 && ents[i].box.area() > ba) { ba = ents[i].box.area(); best = (int)i; }
      if (best < 0) break;
      int n2 = ents[best].child; ents.erase(ents.begin() + best);
      for (int k = 0; k < 2; k++) ents.push_back(E{bin[n2].box[k], bin[n2].child[k], bin[n2].count[k]});
    }
    int inner = 0; for (auto& e : ents) inner += e.count == 0;
    int base = (int)out.nodes.size(); out.nodes.resize(out.nodes.size() + inner);
    GNode nd; int r = 0;
    for (auto& e : ents) { nd.box.push_back(e.box); nd.count.push_back(e.count); nd.child.push_back(e.count == 0 ? base + r++ : e.child); }
    out.nodes[gi] = nd;
    r = 0;
    for (auto& e : ents) if (e.count == 0) {
      int n2 = e.child;
      collapse({E{bin[n2].box[0], bin[n2].child[0], bin[n2].count[0]}, E{bin[n2].box[1], bin[n2].child[1], bin[n2].count[1]}}, base + r++);
    }
  }
  GTree run() {
    int n = s.num_tris(); tb.resize(n); cen.resize(n); ids.resize(n);
    for (int i = 0; i < n; i++) { GBox b; b.grow(s.pos[3 * i]); b.grow(s.pos[3 * i + 1]); b.grow(s.pos[3 * i + 2]); tb[i] = b; cen[i] = (b.lo + b.hi) * 0.5f; ids[i] = i; }
    int r = build2(0, n, split(0, n));
    out.nodes.resize(1);
    collapse({E{bin[r].box[0], bin[r].child[0], bin[r].count[0]}, E{bin[r].box[1], bin[r].child[1], bin[r].count[1]}}, 0);
    for (auto& nd : out.nodes)  // leaf children of a node: one contiguous range
      for (size_t k = 0; k < nd.child.size(); k++)
        if (nd.count[k] > 0) { int f = (int)out.prim.size(); for (int j = 0; j < nd.count[k]; j++) out.prim.push_back(lprim[nd.child[k] + j]); nd.child[k] = f; }
    return out;
  }
};

// Traversal over a generic tree with the engine's step semantics (a step = one node visit and / or
// one triangle pair).
int gquery(const GTree& t, const HostScene& s, f3 o, f3 d, float tmin, float tmax, bool any, Stats& st) {
  f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float best = tmax;
  int node = 0, steps = 0, tlo = 0, thi = 0, sp = 0;
  int stack[256];
  auto tri = [&](int j, float& tt) {
    int p = t.prim[j];
    f3 p0 = s.pos[3 * p], p1 = s.pos[3 * p + 1], p2 = s.pos[3 * p + 2];
    f3 e0 = p1 - p0, e1 = p0 - p2, n = cross(e1, e0);
    f3 e2 = (1.0f / dot(n, d)) * (p0 - o);
    f3 i = cross(d, e2);
    float beta = dot(i, e1), gamma = dot(i, e0);
    tt = dot(n, e2);
    return (tt < (any ? tmax : best)) & (tt > tmin) & (beta >= 0.0f) & (gamma >= 0.0f) & (beta + gamma <= 1.0f);
  };
  while (true) {
    steps++;
    if (tlo >= thi) {
      const GNode& nd = t.nodes[node];
      st.visits++;
      int lo = 0x7FFFFFFF, hi = 0, m = 0;
      int c[16]; float kk[16];
      for (size_t k = 0; k < nd.box.size(); k++) {
        const GBox& b = nd.box[k];
        float x0 = (b.lo.x - o.x) * inv.x, x1 = (b.hi.x - o.x) * inv.x, y0 = (b.lo.y - o.y) * inv.y, y1 = (b.hi.y - o.y) * inv.y;
        float z0 = (b.lo.z - o.z) * inv.z, z1 = (b.hi.z - o.z) * inv.z;
        float nn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), tmin));
        float ff = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), best));
        if (!(nn <= ff * 1.00001f + 1e-6f)) continue;
        if (nd.count[k] > 0) { lo = std::min(lo, nd.child[k]); hi = std::max(hi, nd.child[k] + nd.count[k]); }
        else { c[m] = nd.child[k]; kk[m] = nn; m++; }
      }
      tlo = lo; thi = hi;
      for (int a = 0; a < m; a++) for (int q = a + 1; q < m; q++) if (kk[q] < kk[a]) { std::swap(kk[q], kk[a]); std::swap(c[q], c[a]); }
      if (m) { for (int a = m - 1; a >= 1; a--) stack[sp++] = c[a]; node = c[0]; }
      else if (sp == 0) node = -1;
      else node = stack[--sp];
    }
    if (tlo < thi) {
      for (int u = 0; u < 2 && tlo < thi; u++) {
        float tt; st.tris++;
        if (tri(tlo++, tt)) {
          if (!any) best = std::min(best, tt);
          else if (s.mats[s.flags[t.prim[tlo - 1]] & 0xff].type != MATL_REFRACTION) return steps;
        }
      }
    }
    if (tlo >= thi && node < 0) return steps;
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: bvh_study queries.bin [scene] [asset_dir]\n"); return 2; }
  const int scene = argc > 2 ? atoi(argv[2]) : 1;
  const std::string assets = argc > 3 ? argv[3] : "assets";
  FILE* f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 1; }
  std::vector<f4> q;
  f4 buf[2];
  while (fread(buf, sizeof(f4), 2, f) == 2) { q.push_back(buf[0]); q.push_back(buf[1]); }
  fclose(f);
  HostScene s;
  std::string err;
  if (!build_preset_scene(scene, assets, 0, 810.0f, 0, s, err, 0)) { fprintf(stderr, "scene: %s\n", err.c_str()); return 1; }
  Bvh b;
  const auto t0 = std::chrono::steady_clock::now();
  build_bvh(s, b);
  const double build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (const char* wv = getenv("FOVRT_STUDY_WIDTH")) {  // generic-width study tree instead of the engine's
    GBuilder gb{s, atoi(wv)};
    GTree t = gb.run();
    Stats g[2];
    double tot = 0;
    const size_t nq = q.size() / 2;
    for (size_t i = 0; i < nq; i++) {
      const f4 a = q[2 * i], d = q[2 * i + 1];
      const bool any = d.w != 0.0f;
      const int st = gquery(t, s, mk3(a.x, a.y, a.z), mk3(d.x, d.y, d.z), 1e-3f, a.w, any, g[any]);
      g[any].steps += st; g[any].n++; tot += st;
    }
    printf("width %d: nodes %zu\n", gb.width, t.nodes.size());
    for (int k = 0; k < 2; k++)
      printf("  %-7s steps %6.2f visits %6.2f tris %6.2f\n", k ? "shadow" : "closest", g[k].steps / g[k].n, g[k].visits / g[k].n, g[k].tris / g[k].n);
    printf("  all     steps %6.2f visits %6.2f tris %6.2f\n", tot / nq, (g[0].visits + g[1].visits) / nq, (g[0].tris + g[1].tris) / nq);
    return 0;
  }
  const char* mv = getenv("FOVRT_STUDY_MASK");
  Sim sim{b, s, mv && atoi(mv) != 0};
  Stats st[2];  // closest, shadow
  const size_t nq = q.size() / 2;
  std::vector<int> steps(nq);
  for (size_t i = 0; i < nq; i++) {
    const f4 a = q[2 * i], d = q[2 * i + 1];
    const bool any = d.w != 0.0f;
    Stats& S = st[any];
    steps[i] = sim.query(mk3(a.x, a.y, a.z), mk3(d.x, d.y, d.z), 1e-3f, a.w, any, S);
    S.steps += steps[i];
    S.n++;
  }
  double wave = 0;
  size_t nw = 0;
  for (size_t i = 0; i + 64 <= nq; i += 64, nw++) {
    int m = 0;
    for (size_t k = i; k < i + 64; k++) m = std::max(m, steps[k]);
    wave += m;
  }
  double tot_steps = st[0].steps + st[1].steps;
  printf("nodes %zu tris %zu max_stack %d build %.0f ms | queries %zu (shadow %zu)\n", b.nodes.size(), b.tri_geo.size(),
         b.max_stack, build_ms, nq, st[1].n);
  for (int k = 0; k < 2; k++) {
    const Stats& S = st[k];
    printf("  %-7s steps %6.2f visits %6.2f tris %6.2f (in hit leaves %5.1f%%) hits %5.1f%%\n", k ? "shadow" : "closest",
           S.steps / S.n, S.visits / S.n, S.tris / S.n, 100.0 * S.useful / std::max(1.0, S.tris), 100.0 * S.hits / S.n);
  }
  const double visits = st[0].visits + st[1].visits, tris = st[0].tris + st[1].tris;
  printf("  all     steps %6.2f visits %6.2f tris %6.2f | wave64 max-steps %6.2f (lane util %.2f)\n", tot_steps / nq,
         visits / nq, tris / nq, wave / nw, tot_steps / nq / (wave / nw));
  printf("  cost model (VALU ~130/visit + 50/tri): %.0f per query\n", (130 * visits + 50 * tris) / nq);
  if (getenv("FOVRT_STUDY_HIST")) {  // steps histogram (closest / shadow) and the share of steps in the tail
    std::vector<size_t> hc(256), hs(256);
    for (size_t i = 0; i < nq; i++) (q[2 * i + 1].w != 0.0f ? hs : hc)[std::min(steps[i], 255)]++;
    double cum = 0;
    for (int k = 1; k < 256; k++) {
      if (!hc[k] && !hs[k]) continue;
      cum += (double)k * (hc[k] + hs[k]);
      printf("    steps %3d: closest %7zu shadow %7zu  cum steps %5.1f%%\n", k, hc[k], hs[k], 100.0 * cum / tot_steps);
    }
  }
  return 0;
}
