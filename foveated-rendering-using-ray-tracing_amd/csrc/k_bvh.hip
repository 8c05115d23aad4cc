// k_bvh.hip — the GPU BVH builder: a linear BVH (Morton order, Karras 2012
// hierarchy) built on the device and collapsed into the engine's four-wide nodes, so that a scene
// whose triangles move can be re-indexed every frame without a host round trip.
//
// The output has exactly the layout the host binned-SAH builder (scene.cpp) produces and the
// traversal (k_trace.hip) relies on:
//   - BvhNode: four SoA child slabs, inflated by the host's inflate_lo/hi, empty slots +-inf/-1;
//   - the inner children of a node are contiguous (one traversal stack entry per level);
//   - the leaf children of a node own one contiguous triangle range (the union-span leaf test);
//   - leaves hold at most two triangles; TriGeo is computed with the host's operations.
// Traversal results do not depend on the tree (closest hit ties -> lowest primitive index, shadow
// transmittance in f64), so a frame rendered over this BVH equals the host-built one.
//
// Steps: primitive boxes + centroid bounds -> 30-bit Morton codes -> radix sort (hipCUB) -> Karras
// binary hierarchy -> bottom-up boxes (one atomic per internal node) -> level-synchronous collapse
// into four-wide nodes (the host's rule: open the largest-area inner entry until four) -> per-node
// leaf triangle counts, exclusive scan, triangle relayout.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "fr_device.h"

namespace fr {
namespace {

constexpr int kLeafMax = 2;  // triangles per leaf (the host builder's default)

FR_DEV uint32_t expand_bits(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

// float <-> unsigned with the same order (for atomicMin / atomicMax on floats)
FR_DEV uint32_t ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
FR_DEV float unord(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u); }

FR_DEV float inflate_lo_d(float v) { return v - (1e-5f + 4e-7f * fabsf(v)); }  // scene.cpp inflate_lo
FR_DEV float inflate_hi_d(float v) { return v + (1e-5f + 4e-7f * fabsf(v)); }

FR_DEV float area_of(f4 lo, f4 hi) {
  const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
  if (dx < 0) return 0.0f;
  return 2.0f * (dx * dy + dy * dz + dz * dx);
}

FR_DEV float wave_min(float v) {
  for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
FR_DEV float wave_max(float v) {
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Primitive boxes and the centroid bounds (cb[0..2] = min, cb[3..5] = max, order-mapped).
__global__ void k_prim_boxes(const f3* __restrict__ pos, int n, f4* __restrict__ blo, f4* __restrict__ bhi,
                             uint32_t* __restrict__ cb) {
  f3 cmin = mk3(INFINITY), cmax = mk3(-INFINITY);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const f3 a = pos[3 * i], b = pos[3 * i + 1], c = pos[3 * i + 2];
    const f3 lo = mk3(fminf(fminf(a.x, b.x), c.x), fminf(fminf(a.y, b.y), c.y), fminf(fminf(a.z, b.z), c.z));
    const f3 hi = mk3(fmaxf(fmaxf(a.x, b.x), c.x), fmaxf(fmaxf(a.y, b.y), c.y), fmaxf(fmaxf(a.z, b.z), c.z));
    blo[i] = mk4(lo, 0.0f);
    bhi[i] = mk4(hi, 0.0f);
    const f3 ce = (lo + hi) * 0.5f;
    cmin = mk3(fminf(cmin.x, ce.x), fminf(cmin.y, ce.y), fminf(cmin.z, ce.z));
    cmax = mk3(fmaxf(cmax.x, ce.x), fmaxf(cmax.y, ce.y), fmaxf(cmax.z, ce.z));
  }
  const float r[6] = {wave_min(cmin.x), wave_min(cmin.y), wave_min(cmin.z),
                      wave_max(cmax.x), wave_max(cmax.y), wave_max(cmax.z)};
  if ((threadIdx.x & 63) == 0) {
    for (int k = 0; k < 3; k++) atomicMin(&cb[k], ord(r[k]));
    for (int k = 3; k < 6; k++) atomicMax(&cb[k], ord(r[k]));
  }
}

__global__ void k_morton(const f4* __restrict__ blo, const f4* __restrict__ bhi, int n, const uint32_t* __restrict__ cb,
                         uint32_t* __restrict__ codes, int32_t* __restrict__ ids) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const f3 cmin = mk3(unord(cb[0]), unord(cb[1]), unord(cb[2]));
  const f3 cmax = mk3(unord(cb[3]), unord(cb[4]), unord(cb[5]));
  const f4 lo = blo[i], hi = bhi[i];
  const f3 ce = (xyz(lo) + xyz(hi)) * 0.5f;
  auto q = [](float c, float a, float b) {
    const float e = b - a;
    const float t = e > 0.0f ? (c - a) / e : 0.5f;
    return (uint32_t)fminf(fmaxf(t * 1024.0f, 0.0f), 1023.0f);
  };
  codes[i] = (expand_bits(q(ce.x, cmin.x, cmax.x)) << 2) | (expand_bits(q(ce.y, cmin.y, cmax.y)) << 1) |
             expand_bits(q(ce.z, cmin.z, cmax.z));
  ids[i] = i;
}

// Karras' delta with the index as the tie-breaker of equal codes.
FR_DEV int kdelta(const uint32_t* __restrict__ codes, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint32_t a = codes[i], b = codes[j];
  if (a == b) return 32 + __clz((uint32_t)(i ^ j));
  return __clz(a ^ b);
}

// Internal node i of the binary tree (ids: internal [0, n-1), leaf k -> n-1+k).
__global__ void k_karras(const uint32_t* __restrict__ codes, int n, int2* __restrict__ child, int* __restrict__ parent,
                         int2* __restrict__ range) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const int d = kdelta(codes, n, i, i + 1) - kdelta(codes, n, i, i - 1) >= 0 ? 1 : -1;
  const int dmin = kdelta(codes, n, i, i - d);
  int lmax = 2;
  while (kdelta(codes, n, i, i + lmax * d) > dmin) lmax *= 2;
  int l = 0;
  for (int t = lmax / 2; t >= 1; t /= 2)
    if (kdelta(codes, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = kdelta(codes, n, i, j);
  int s = 0, t = l;
  do {
    t = (t + 1) >> 1;
    if (kdelta(codes, n, i, i + (s + t) * d) > dnode) s += t;
  } while (t > 1);
  const int gamma = i + s * d + min(d, 0);
  const int first = min(i, j), last = max(i, j);
  const int left = first == gamma ? n - 1 + gamma : gamma;
  const int right = last == gamma + 1 ? n - 1 + gamma + 1 : gamma + 1;
  child[i] = int2{left, right};
  parent[left] = i;
  parent[right] = i;
  range[i] = int2{first, last};
  if (i == 0) parent[0] = -1;
}

FR_DEV f4 load_agent(const f4* p) {
  const float* q = reinterpret_cast<const float*>(p);
  return mk4(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
             __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
             __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0.0f);
}

// Bottom-up boxes: a leaf walks to the root; the first arrival at a node stops, the second (which
// then sees both children) writes the union and continues.
__global__ void k_boxes_up(int n, const int32_t* __restrict__ ids, const f4* __restrict__ blo, const f4* __restrict__ bhi,
                           const int* __restrict__ parent, const int2* __restrict__ child, f4* nlo, f4* nhi,
                           uint32_t* __restrict__ arrivals) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  int node = parent[n - 1 + k];
  while (node >= 0) {
    if (__hip_atomic_fetch_add(&arrivals[node], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    const int2 c = child[node];
    f4 lo = mk4(INFINITY, INFINITY, INFINITY, 0.0f), hi = mk4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
    for (int side = 0; side < 2; side++) {
      const int e = side ? c.y : c.x;
      f4 a, b;
      if (e >= n - 1) { a = blo[ids[e - (n - 1)]]; b = bhi[ids[e - (n - 1)]]; }
      else { a = load_agent(nlo + e); b = load_agent(nhi + e); }
      lo = mk4(fminf(lo.x, a.x), fminf(lo.y, a.y), fminf(lo.z, a.z), 0.0f);
      hi = mk4(fmaxf(hi.x, b.x), fmaxf(hi.y, b.y), fmaxf(hi.z, b.z), 0.0f);
    }
    float* pl = reinterpret_cast<float*>(nlo + node);
    float* ph = reinterpret_cast<float*>(nhi + node);
    for (int q = 0; q < 3; q++) {
      __hip_atomic_store(pl + q, (&lo.x)[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ph + q, (&hi.x)[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    node = parent[node];
  }
}

struct CollapseItem {
  int bin;   // binary node id
  int slot;  // its four-wide node
  int need;  // traversal stack entries on the path to it
};

struct BinTree {
  int n;
  const int2* child;
  const int2* range;
  const f4 *nlo, *nhi, *blo, *bhi;
  const int32_t* ids;
  FR_DEV bool is_leaf(int e) const { return e >= n - 1 || range[e].y - range[e].x + 1 <= kLeafMax; }
  FR_DEV int first(int e) const { return e >= n - 1 ? e - (n - 1) : range[e].x; }
  FR_DEV int size(int e) const { return e >= n - 1 ? 1 : range[e].y - range[e].x + 1; }
  FR_DEV f4 lo(int e) const { return e >= n - 1 ? blo[ids[e - (n - 1)]] : nlo[e]; }
  FR_DEV f4 hi(int e) const { return e >= n - 1 ? bhi[ids[e - (n - 1)]] : nhi[e]; }
};

// One level of the collapse: every item becomes a four-wide node; its inner children are allocated
// contiguously and become the next level's items. Leaf entries keep their sorted-order range for
// now (k_emit_leaves relays them out).
__global__ void k_collapse(BinTree T, const CollapseItem* __restrict__ cur, const uint32_t* __restrict__ ncur,
                           CollapseItem* __restrict__ next, uint32_t* __restrict__ nnext, uint32_t* __restrict__ node_ctr,
                           BvhNode* __restrict__ nodes, uint32_t* __restrict__ max_stack, uint32_t* __restrict__ levels) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nc = *ncur;
  if (i == 0 && nc) atomicAdd(levels, 1u);
  if (i >= nc) return;
  const CollapseItem it = cur[i];
  int e[4];
  int ne = 2;
  e[0] = T.child[it.bin].x;
  e[1] = T.child[it.bin].y;
  while (ne < 4) {  // open the inner entry of largest area (scene.cpp collapse)
    int best = -1;
    float ba = -1.0f;
    for (int k = 0; k < ne; k++)
      if (!T.is_leaf(e[k])) {
        const float a = area_of(T.lo(e[k]), T.hi(e[k]));
        if (a > ba) { ba = a; best = k; }
      }
    if (best < 0) break;
    const int2 c = T.child[e[best]];
    for (int k = best; k + 1 < ne; k++) e[k] = e[k + 1];
    e[ne - 1] = c.x;
    e[ne] = c.y;
    ne++;
  }
  int inner = 0;
  for (int k = 0; k < ne; k++) inner += !T.is_leaf(e[k]);
  const int need = it.need + (inner > 1 ? 1 : 0);
  atomicMax(max_stack, (uint32_t)need);
  const int base = inner ? (int)atomicAdd(node_ctr, (uint32_t)inner) : 0;
  BvhNode nd;
  float* LX = &nd.lox.x; float* HX = &nd.hix.x;
  float* LY = &nd.loy.x; float* HY = &nd.hiy.x;
  float* LZ = &nd.loz.x; float* HZ = &nd.hiz.x;
  int r = 0;
  for (int k = 0; k < 4; k++) {
    if (k >= ne) {
      LX[k] = LY[k] = LZ[k] = INFINITY;
      HX[k] = HY[k] = HZ[k] = -INFINITY;
      nd.child[k] = 0;
      nd.count[k] = -1;
      continue;
    }
    const f4 lo = T.lo(e[k]), hi = T.hi(e[k]);
    LX[k] = inflate_lo_d(lo.x); HX[k] = inflate_hi_d(hi.x);
    LY[k] = inflate_lo_d(lo.y); HY[k] = inflate_hi_d(hi.y);
    LZ[k] = inflate_lo_d(lo.z); HZ[k] = inflate_hi_d(hi.z);
    if (T.is_leaf(e[k])) {
      nd.child[k] = T.first(e[k]);
      nd.count[k] = T.size(e[k]);
    } else {
      nd.child[k] = base + r;
      nd.count[k] = 0;
      next[atomicAdd(nnext, 1u)] = CollapseItem{e[k], base + r, need};
      r++;
    }
  }
  nodes[it.slot] = nd;
}

__global__ void k_leaf_counts(const BvhNode* __restrict__ nodes, int nn, uint32_t* __restrict__ cnt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  uint32_t s = 0;
  for (int k = 0; k < 4; k++) s += nodes[i].count[k] > 0 ? (uint32_t)nodes[i].count[k] : 0u;
  cnt[i] = s;
}

// Leaf children of node i -> one contiguous range starting at off[i]; TriGeo with the host's
// operations (scene.cpp: e0 = p1 - p0, e1 = p0 - p2, n = cross(e1, e0)).
__global__ void k_emit_leaves(BvhNode* __restrict__ nodes, int nn, const uint32_t* __restrict__ off,
                              const int32_t* __restrict__ ids, const f3* __restrict__ pos, TriGeo* __restrict__ tri,
                              int32_t* __restrict__ prim) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  uint32_t o = off[i];
  for (int k = 0; k < 4; k++) {
    const int cnt = nodes[i].count[k];
    if (cnt <= 0) continue;
    const int first = nodes[i].child[k];
    nodes[i].child[k] = (int)o;
    for (int j = 0; j < cnt; j++, o++) {
      const int p = ids[first + j];
      prim[o] = p;
      const f3 p0 = pos[3 * p], p1 = pos[3 * p + 1], p2 = pos[3 * p + 2];
      const f3 e0 = p1 - p0, e1 = p0 - p2, nn3 = cross(e1, e0);
      tri[o].a = mk4(p0.x, p0.y, p0.z, e0.x);
      tri[o].b = mk4(e0.y, e0.z, e1.x, e1.y);
      tri[o].c = mk4(e1.z, nn3.x, nn3.y, nn3.z);
    }
  }
}

template <typename T>
hipError_t alloc(T** p, size_t n) {
  return hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T));
}

}  // namespace

// Scratch of the builder, kept by the context between rebuilds (no allocation, no hipFree, which would
// synchronise the whole device, in a rebuild once it exists).
struct BvhWork {
  int cap = 0;
  f4 *blo = nullptr, *bhi = nullptr, *nlo = nullptr, *nhi = nullptr;
  uint32_t *cb = nullptr, *codes = nullptr, *codes_s = nullptr, *arrivals = nullptr, *ctr = nullptr, *cnt = nullptr,
           *off = nullptr;
  int32_t *ids = nullptr, *ids_s = nullptr;
  int2 *child = nullptr, *range = nullptr;
  int* parent = nullptr;
  CollapseItem *qa = nullptr, *qb = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  uint32_t* host = nullptr;  // pinned: ncur, node count, max stack, levels
};

void bvh_work_free(BvhWork* w) {
  if (!w) return;
  for (void* p : {(void*)w->blo, (void*)w->bhi, (void*)w->nlo, (void*)w->nhi, (void*)w->cb, (void*)w->codes,
                  (void*)w->codes_s, (void*)w->ids, (void*)w->ids_s, (void*)w->child, (void*)w->range, (void*)w->parent,
                  (void*)w->arrivals, (void*)w->ctr, (void*)w->qa, (void*)w->qb, (void*)w->cnt, (void*)w->off, w->tmp})
    if (p) hipFree(p);
  if (w->host) hipHostFree(w->host);
  delete w;
}

static bool bvh_work_reserve(BvhWork*& w, int n, hipStream_t s, std::string& err) {
  if (w && w->cap >= n) return true;
  bvh_work_free(w);
  w = new BvhWork();
  if (alloc(&w->blo, n) || alloc(&w->bhi, n) || alloc(&w->nlo, n) || alloc(&w->nhi, n) || alloc(&w->cb, 6) ||
      alloc(&w->codes, n) || alloc(&w->codes_s, n) || alloc(&w->ids, n) || alloc(&w->ids_s, n) || alloc(&w->child, n) ||
      alloc(&w->range, n) || alloc(&w->parent, 2 * n) || alloc(&w->arrivals, n) || alloc(&w->ctr, 8) ||
      alloc(&w->qa, n) || alloc(&w->qb, n) || alloc(&w->cnt, n) || alloc(&w->off, n) ||
      hipHostMalloc((void**)&w->host, 8 * sizeof(uint32_t)) != hipSuccess) {
    err = "GPU BVH builder: device allocation failed";
    bvh_work_free(w);
    w = nullptr;
    return false;
  }
  size_t sort_bytes = 0, scan_bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, w->codes, w->codes_s, w->ids, w->ids_s, n, 0, 30, s);
  hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, w->cnt, w->off, n, s);
  w->tmp_bytes = std::max(sort_bytes, scan_bytes);
  if (hipMalloc(&w->tmp, w->tmp_bytes) != hipSuccess) {
    err = "GPU BVH builder: scratch allocation failed";
    bvh_work_free(w);
    w = nullptr;
    return false;
  }
  w->cap = n;
  return true;
}

bool bvh_work_prepare(BvhWork** w, int n, hipStream_t s, std::string& err) { return bvh_work_reserve(*w, n, s, err); }

// One launch from this module (k_build_init on the workspace), so that its code object is loaded at
// context creation rather than in the first rebuild.
__global__ void k_build_init(uint32_t* __restrict__ cb, CollapseItem* __restrict__ qa, uint32_t* __restrict__ ctr);
bool bvh_builder_warm(BvhWork* w, hipStream_t s, std::string& err) {
  if (!w) return true;
  hipLaunchKernelGGL(k_build_init, dim3(1), dim3(64), 0, s, w->cb, w->qa, w->ctr);
  if (hipGetLastError() != hipSuccess) { err = "GPU BVH builder: launch failed"; return false; }
  return true;
}

// The builder's small initial values in one launch (they were three pageable host-to-device copies, which
// go through the runtime's staging path: the first rebuilds of a context took 6-15 ms instead of 0.8-2).
// cb: the scene box accumulators (min: +bits, max: 0); qa[0]: the root item; ctr: node_ctr, max_stack, ncur,
// nnext, levels.
__global__ void k_build_init(uint32_t* __restrict__ cb, CollapseItem* __restrict__ qa, uint32_t* __restrict__ ctr) {
  const int t = threadIdx.x;
  if (t < 6) cb[t] = t < 3 ? 0xFFFFFFFFu : 0u;
  if (t < 5) ctr[t] = t == 0 || t == 2 ? 1u : 0u;
  if (t == 0) qa[0] = CollapseItem{0, 0, 0};
}

// Builds the four-wide BVH of n triangles (pos: 3 vertices per triangle, device) into the caller's
// nodes / tri / prim (device, n entries each) with the workspace *work (created or grown here, kept
// by the caller). Returns false with err set on failure. num_nodes, max_stack and depth (levels of
// the four-wide tree below the root) describe the result. The collapse runs its levels in batches of
// launches that skip themselves once the level queue is empty, with one host read per batch.
bool gpu_build_bvh(BvhWork** work, const f3* pos, int n, BvhNode* nodes, TriGeo* tri, int32_t* prim, int* num_nodes,
                   int* max_stack, int* depth, hipStream_t s, std::string& err) {
  if (n < 3) { err = "GPU BVH builder needs at least 3 triangles"; return false; }
  // FOVRT_BVH_PHASES=1: host time of each phase (each followed by a stream sync) on stderr, a diagnostic
  static const bool phases = [] { const char* v = getenv("FOVRT_BVH_PHASES"); return v && atoi(v) != 0; }();
  // (host time, and the GPU time between events recorded at the phase boundaries)
  auto t_last = std::chrono::steady_clock::now();
  hipEvent_t ev_last = nullptr;
  auto phase = [&](const char* name) {
    if (!phases) return;
    using clk = std::chrono::steady_clock;
    const auto a0 = clk::now();
    hipEvent_t ev = nullptr;
    hipEventCreate(&ev);
    const auto a1 = clk::now();
    hipEventRecord(ev, s);
    const auto a2 = clk::now();
    hipStreamSynchronize(s);
    const auto t = clk::now();
    auto ms = [](clk::time_point x, clk::time_point y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    if (!strcmp(name, "entry"))
      fprintf(stderr, "bvh entry api: create %.3f record %.3f sync %.3f ms\n", ms(a0, a1), ms(a1, a2), ms(a2, t));
    float gms = 0.0f;
    if (ev_last) { hipEventElapsedTime(&gms, ev_last, ev); hipEventDestroy(ev_last); }
    fprintf(stderr, "bvh phase %-10s %8.3f ms host %8.3f ms gpu\n", name,
            std::chrono::duration<double, std::milli>(t - t_last).count(), gms);
    t_last = t;
    ev_last = ev;
    if (!strcmp(name, "emit")) { hipEventDestroy(ev_last); ev_last = nullptr; }
  };
  phase("entry");
  if (!bvh_work_reserve(*work, n, s, err)) return false;
  BvhWork& w = **work;
  hipLaunchKernelGGL(k_build_init, dim3(1), dim3(64), 0, s, w.cb, w.qa, w.ctr);
  const int B = 256, G = (n + B - 1) / B;
  hipLaunchKernelGGL(k_prim_boxes, dim3(std::min(G, 2048)), dim3(B), 0, s, pos, n, w.blo, w.bhi, w.cb);
  hipLaunchKernelGGL(k_morton, dim3(G), dim3(B), 0, s, w.blo, w.bhi, n, w.cb, w.codes, w.ids);
  phase("morton");
  size_t tb = w.tmp_bytes;
  hipcub::DeviceRadixSort::SortPairs(w.tmp, tb, w.codes, w.codes_s, w.ids, w.ids_s, n, 0, 30, s);
  phase("sort");
  hipLaunchKernelGGL(k_karras, dim3(G), dim3(B), 0, s, w.codes_s, n, w.child, w.parent, w.range);
  hipMemsetAsync(w.arrivals, 0, (size_t)n * sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_boxes_up, dim3(G), dim3(B), 0, s, n, w.ids_s, w.blo, w.bhi, w.parent, w.child, w.nlo, w.nhi,
                     w.arrivals);
  phase("karras");
  BinTree T{n, w.child, w.range, w.nlo, w.nhi, w.blo, w.bhi, w.ids_s};
  // (qa[0] = the root item and ctr = {1, 0, 1, 0, 0}: k_build_init)
  const int kBatch = 8;
  int launched = 0;
  CollapseItem *qa = w.qa, *qb = w.qb;
  for (;;) {
    for (int b = 0; b < kBatch; b++) {
      hipMemsetAsync(w.ctr + 3, 0, sizeof(uint32_t), s);
      // a level holds at most n items (one per inner node of the binary tree)
      hipLaunchKernelGGL(k_collapse, dim3(G), dim3(B), 0, s, T, qa, w.ctr + 2, qb, w.ctr + 3, w.ctr, nodes, w.ctr + 1,
                         w.ctr + 4);
      hipMemcpyAsync(w.ctr + 2, w.ctr + 3, sizeof(uint32_t), hipMemcpyDeviceToDevice, s);
      std::swap(qa, qb);
    }
    launched += kBatch;
    hipMemcpyAsync(w.host, w.ctr, 5 * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) { err = "GPU BVH builder: kernel failure"; return false; }
    if (w.host[2] == 0) break;
    if (launched >= 64) { err = "GPU BVH builder: collapse did not terminate"; return false; }
  }
  phase("collapse");
  *num_nodes = (int)w.host[0];
  *max_stack = (int)w.host[1];
  *depth = (int)w.host[4] - 1;
  const int nn = *num_nodes, GN = (nn + B - 1) / B;
  hipLaunchKernelGGL(k_leaf_counts, dim3(GN), dim3(B), 0, s, nodes, nn, w.cnt);
  tb = w.tmp_bytes;
  hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.cnt, w.off, nn, s);
  phase("scan");
  hipLaunchKernelGGL(k_emit_leaves, dim3(GN), dim3(B), 0, s, nodes, nn, w.off, w.ids_s, pos, tri, prim);
  if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess) {
    err = "GPU BVH builder: kernel failure";
    return false;
  }
  phase("emit");
  return true;
}

}  // namespace fr
