// group.cpp — multi-GPU groups (include/fovrt.h fr_group_*): tile sharding of a view over ranks, the
// sparse gather of traced pixels to the reconstruction ranks over RCCL (xGMI), split reconstruction
// chains and the final composite of the views (SURVEY §8(b) Threading row, §8(e)).
//
// The reference is single-GPU (one OptiX context, FR/PathTracer.cpp:403-414; its frame loop
// FR/main.cpp:227-462). A group runs that loop on R ranks at once: every rank enqueues its trace half
// (entries 0-3 on its own tiles), the traced pixels travel to the ranks that reconstruct, and those
// run JumpFlooding -> Sibson and pull-push -> A-Trous on their own streams while the next frame traces.
// Transfer sizes come from each rank's own full sampling mask (fr_shard_counts: every rank computes the
// same mask), so the only host wait per frame is for the rank's own front stages.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ctx_internal.h"

namespace {

thread_local std::string g_group_error;

int gfail(int code, const std::string& msg) {
  g_group_error = msg;
  return code;
}

struct GroupRank {
  fr_ctx* c = nullptr;
  int rank = 0, view = 0, vrank = 0;
  int chains = 0;  // bit 0 JFA -> Sibson, bit 1 pull-push -> A-Trous
  int tiles = 0;
  hipStream_t comm = nullptr;  // transfers and the unpack inputs (on the context's device)
  // sparse slabs: [k] double buffers by frame parity; one receive slab per view rank (null for self)
  char* send[2] = {};
  std::vector<char*> recv[2];
  hipEvent_t ev_packed = nullptr, ev_comm[2] = {}, ev_unpacked[2] = {}, ev_out = nullptr, ev_sent_out = nullptr;
  bool comm_pending[2] = {}, unpacked_pending[2] = {};
  uint32_t n[FR_GROUP_MAX_VIEW_RANKS] = {};  // this frame's active pixels of every view rank
  // history validity rings (still camera, k_vring_pack): the tile list grouped by owner (device), this
  // rank's packed ring bits and one receive slab per other view rank, double-buffered by frame parity
  int32_t* tiles_dev = nullptr;
  uint32_t* vsend[2] = {};
  std::vector<uint32_t*> vrecv[2];
  // composite (rank 0): the views' A-Trous images and the side-by-side result
  f4* comp_stack = nullptr;
  f4* comp_out = nullptr;
};

}  // namespace

struct fr_group {
  std::vector<GroupRank> loc;
  int R = 1, V = 1, G = 1;
  int W = 0, H = 0;
  ncclComm_t comm = nullptr;  // null: every rank is local (device-to-device copies)
  fr_group_config cfg;
  std::vector<uint8_t> owner;       // tile -> view rank (the same plan in every view)
  std::vector<int> tiles_per_vrank;
  std::vector<int> tile_off;        // view rank s's tiles: tiles_dev[tile_off[s] .. tile_off[s + 1])
  int jfa_ranks = 1;                // view ranks taking JFA -> Sibson in turns (fr_group_config.jfa_ranks)
  uint64_t frame = 0;
  bool composite_done = false;
};

namespace {

int view_of(const fr_group* g, int rank) { return rank / g->G; }
int rank_of(const fr_group* g, int view, int vrank) { return view * g->G + vrank; }
// The view ranks that take JumpFlooding -> Sibson in turns (one frame each): view rank 0, then 2, 3, ...
// (view rank 1 runs pull-push -> A-Trous, whose push atlas carries state from frame to frame).
int chains_for(int G, bool split, int jfa_ranks, int vrank) {
  if (G == 1) return 3;
  if (vrank == 0) return split ? 1 : 3;
  if (vrank == 1 && split) return 2;
  return vrank >= 2 && vrank <= jfa_ranks ? 1 : 0;
}
int chains_of(const fr_group* g, int vrank) { return chains_for(g->G, g->cfg.split_recon != 0, g->jfa_ranks, vrank); }
// fr_group_config.jfa_ranks, with 0 = auto resolved
int jfa_ranks_for(int G, const fr_group_config& cfg) {
  return cfg.jfa_ranks ? cfg.jfa_ranks : (cfg.split_recon && G >= 6 ? 2 : 1);
}
// The view rank whose turn it is to run JumpFlooding -> Sibson on frame f.
int jfa_turn(const fr_group* g, uint64_t f) {
  const int k = (int)(f % (uint64_t)g->jfa_ranks);
  return k == 0 ? 0 : k + 1;
}
// The view rank whose A-Trous image is the view's output (the composite's source).
int output_vrank(const fr_group* g) { return g->G >= 2 && g->cfg.split_recon ? 1 : 0; }
// Does view rank r receive view rank s's traced pixels?
bool receives(const fr_group* g, int r, int s) {
  if (r == s) return false;
  return g->cfg.moving_camera ? true : chains_of(g, r) != 0;
}

// Does view rank r take the other ranks' history validity rings? A pure tracer of a still camera: it holds
// the history of its own tiles only, and its seeds read the validity of the pixels around them.
bool vring_receiver(const fr_group* g, int r) {
  // (FOVRT_GROUP_VRING=0: no rings, a diagnostic that shows what they fix)
  static const bool on = [] { const char* v = getenv("FOVRT_GROUP_VRING"); return !v || atoi(v) != 0; }();
  return on && g->G > 1 && !g->cfg.moving_camera && chains_of(g, r) == 0 && g->tiles_per_vrank[r] > 0;
}
bool vring_sender(const fr_group* g, int s) {
  if (g->G == 1 || g->cfg.moving_camera || !g->tiles_per_vrank[s]) return false;
  for (int r = 0; r < g->G; r++)
    if (r != s && vring_receiver(g, r)) return true;
  return false;
}
size_t vring_words(const fr_group* g, int s) { return (size_t)g->tiles_per_vrank[s] * (FR_VRING * g->cfg.tile / 8); }

// Water filling: rank r carries recon work c[r] (in units of one frame's trace work) and gets a trace share
// s[r] = max(0, lambda - c[r]) with sum s = 1, so that every loaded rank ends at lambda.
void level_weights(const std::vector<double>& c, std::vector<float>& w) {
  const int n = (int)c.size();
  std::vector<double> sorted(c);
  std::sort(sorted.begin(), sorted.end());
  double lambda = 0.0, acc = 0.0;
  for (int k = 1; k <= n; k++) {
    acc += sorted[k - 1];
    lambda = (1.0 + acc) / k;
    if (k == n || lambda <= sorted[k]) break;
  }
  w.assign(n, 0.0f);
  for (int r = 0; r < n; r++) w[r] = (float)std::max(0.0, lambda - c[r]);
}

// The tile plan of a view of G ranks (fr_group_plan): explicit weights, or water filling on the
// reconstruction loads followed by the sliver rule.
int group_plan(int W, int H, int G, const fr_group_config& cfg, uint8_t* owner, size_t ntiles) {
  std::vector<float> w(G, 0.0f);
  bool explicit_w = false;
  for (int r = 0; r < G; r++) explicit_w |= cfg.weights[r] != 0.0f;
  if (explicit_w) {
    for (int r = 0; r < G; r++) w[r] = cfg.weights[r];
  } else {
    const int m = jfa_ranks_for(G, cfg);
    std::vector<double> cost(G, 0.0);
    for (int r = 0; r < G; r++) {
      const int ch = chains_for(G, cfg.split_recon != 0, m, r);
      cost[r] = ((ch & 1) ? cfg.recon_cost[0] / m : 0.0) + ((ch & 2) ? cfg.recon_cost[1] : 0.0);
    }
    level_weights(cost, w);
    // a rank left with a sliver of the tiles would still pay a whole launch's critical path (the
    // longest refraction trees of a dense foveal tile take ~2 ms however few tiles there are), on top
    // of its reconstruction chain: slivers below a fifth of the largest share go to the others
    const float wmax = *std::max_element(w.begin(), w.end());
    for (float& x : w) if (x < 0.2f * wmax) x = 0.0f;
  }
  if (int rc = fr_shard_plan(W, H, cfg.tile, G, w.data(), owner, ntiles))
    return gfail(rc, std::string("group plan: ") + fr_last_error(nullptr));
  return FR_OK;
}

int rccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return FR_OK;
  return gfail(FR_E_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

// One batch of point-to-point transfers of the frame (every local rank's sends and receives).
struct Xfer {
  int src, dst;  // global ranks
  const void* sbuf;
  void* rbuf;
  size_t bytes;
};

// Enqueues the batch: RCCL (one rank per process) as one ncclGroup of sends and receives on the comm
// streams; in-process ranks as peer copies on the receiver's comm stream after the sender's ev_packed.
int run_xfers(fr_group* g, const std::vector<Xfer>& xs, bool sender_packed) {
  if (xs.empty()) return FR_OK;
  if (g->comm) {
    GroupRank& L = g->loc[0];
    hipSetDevice(L.c->cfg.device);
    if (int rc = rccl_check(ncclGroupStart(), "ncclGroupStart")) return rc;
    for (const Xfer& x : xs) {
      if (x.src == L.rank && x.dst == L.rank) continue;  // never generated
      ncclResult_t r = x.src == L.rank ? ncclSend(x.sbuf, x.bytes, ncclChar, x.dst, g->comm, L.comm)
                                       : ncclRecv(x.rbuf, x.bytes, ncclChar, x.src, g->comm, L.comm);
      if (r != ncclSuccess) {
        ncclGroupEnd();
        return rccl_check(r, x.src == L.rank ? "ncclSend" : "ncclRecv");
      }
    }
    return rccl_check(ncclGroupEnd(), "ncclGroupEnd");
  }
  for (const Xfer& x : xs) {
    GroupRank& S = g->loc[x.src];
    GroupRank& D = g->loc[x.dst];
    hipSetDevice(D.c->cfg.device);
    if (sender_packed) hipStreamWaitEvent(D.comm, S.ev_packed, 0);
    if (hipMemcpyPeerAsync(x.rbuf, D.c->cfg.device, x.sbuf, S.c->cfg.device, x.bytes, D.comm) != hipSuccess)
      return gfail(FR_E_HIP, "group: peer copy failed");
  }
  return FR_OK;
}

void free_rank(GroupRank& L) {
  if (!L.c) return;
  hipSetDevice(L.c->cfg.device);
  if (L.comm) hipStreamSynchronize(L.comm);
  for (int k = 0; k < 2; k++) {
    if (L.send[k]) hipFree(L.send[k]);
    for (char* p : L.recv[k]) if (p) hipFree(p);
    if (L.vsend[k]) hipFree(L.vsend[k]);
    for (uint32_t* p : L.vrecv[k]) if (p) hipFree(p);
    if (L.ev_comm[k]) hipEventDestroy(L.ev_comm[k]);
    if (L.ev_unpacked[k]) hipEventDestroy(L.ev_unpacked[k]);
  }
  if (L.ev_packed) hipEventDestroy(L.ev_packed);
  if (L.ev_out) hipEventDestroy(L.ev_out);
  if (L.ev_sent_out) hipEventDestroy(L.ev_sent_out);
  if (L.tiles_dev) hipFree(L.tiles_dev);
  if (L.comp_stack) hipFree(L.comp_stack);
  if (L.comp_out) hipFree(L.comp_out);
  if (L.comm) hipStreamDestroy(L.comm);
}

// Every local rank's part of one frame's sparse exchange (after its trace half): pack, transfer, unpack.
int exchange(fr_group* g) {
  const int k = (int)(g->frame & 1);
  const size_t T2 = (size_t)g->cfg.tile * g->cfg.tile;
  // counts of this frame (each rank's own front stages only)
  for (GroupRank& L : g->loc) {
    hipSetDevice(L.c->cfg.device);
    if (int rc = fr_shard_counts(L.c, L.n, g->G)) return gfail(rc, std::string("group: ") + fr_last_error(L.c));
    for (int s = 0; s < g->G; s++)
      if (L.n[s] > (size_t)g->tiles_per_vrank[s] * T2) return gfail(FR_E_STATE, "group: active count above the rank's tiles");
  }
  // pack this rank's traced pixels: (radiance, 1) texels, then their pixel indices (n x 20 B)
  for (GroupRank& L : g->loc) {
    const uint32_t n = L.n[L.vrank];
    bool any_receiver = false;
    for (int r = 0; r < g->G; r++) any_receiver |= receives(g, r, L.vrank);
    if (!n || !any_receiver) continue;
    hipSetDevice(L.c->cfg.device);
    // send[k] was last read by the transfers of frame - 2
    if (g->comm) {
      if (L.comm_pending[k]) hipStreamWaitEvent(L.c->stream, L.ev_comm[k], 0);
    } else {
      for (GroupRank& D : g->loc)
        if (D.comm_pending[k]) hipStreamWaitEvent(L.c->stream, D.ev_comm[k], 0);
    }
    f4* vals = (f4*)L.send[k];
    uint32_t* idx = (uint32_t*)(L.send[k] + (size_t)n * sizeof(f4));
    fr::launch_shard_pack_active(L.c->active, L.c->ray_count, n, L.c->shade_radiance, vals, idx, L.c->stream);
    if (int rc = fri::check_launch(L.c)) return gfail(rc, fr_last_error(L.c));
    hipEventRecord(L.ev_packed, L.c->stream);
    // The slot's active list and ray count are released to the front stages of frame + nslots (stream5
    // waits for ev_trace[slot]) only once this pack has read them: enqueue_shading recorded ev_trace
    // before the pack was queued, and the pack may still wait for frame - 2's transfers (ev_comm).
    hipEventRecord(L.c->ev_trace[L.c->slot], L.c->stream);
    L.c->trace_pending[L.c->slot] = true;
    if (g->comm) hipStreamWaitEvent(L.comm, L.ev_packed, 0);
  }
  // the history validity rings of this frame's history (after the trace half: resolve and carry)
  for (GroupRank& L : g->loc) {
    if (!vring_sender(g, L.vrank)) continue;
    hipSetDevice(L.c->cfg.device);
    if (g->comm) {
      if (L.comm_pending[k]) hipStreamWaitEvent(L.c->stream, L.ev_comm[k], 0);
    } else {
      for (GroupRank& D : g->loc)
        if (D.comm_pending[k]) hipStreamWaitEvent(L.c->stream, D.ev_comm[k], 0);
    }
    fr::launch_vring_pack(L.c->img[L.c->hist_cache], g->W, g->H, g->cfg.tile, L.tiles_dev + g->tile_off[L.vrank],
                          g->tiles_per_vrank[L.vrank], L.vsend[k], L.c->stream);
    if (int rc = fri::check_launch(L.c)) return gfail(rc, fr_last_error(L.c));
    hipEventRecord(L.ev_packed, L.c->stream);
    if (g->comm) hipStreamWaitEvent(L.comm, L.ev_packed, 0);
  }
  // receive slabs of frame - 2 must have been unpacked
  for (GroupRank& L : g->loc)
    if (L.unpacked_pending[k]) {
      hipSetDevice(L.c->cfg.device);
      hipStreamWaitEvent(L.comm, L.ev_unpacked[k], 0);
    }
  std::vector<Xfer> xs;
  for (GroupRank& L : g->loc) {
    const int v = L.view;
    for (int s = 0; s < g->G; s++) {
      for (int r = 0; r < g->G; r++) {
        if (!receives(g, r, s) || !L.n[s]) continue;
        const int src = rank_of(g, v, s), dst = rank_of(g, v, r);
        if (src != L.rank && dst != L.rank) continue;
        if (!g->comm && src != L.rank) continue;  // in-process: each pair once, from the sender's side
        const size_t bytes = (size_t)L.n[s] * 20;
        const GroupRank* D = g->comm ? &L : &g->loc[dst];
        xs.push_back({src, dst, g->comm ? (src == L.rank ? L.send[k] : nullptr) : L.send[k],
                      dst == D->rank ? D->recv[k][s] : nullptr, bytes});
      }
    }
  }
  for (GroupRank& L : g->loc) {
    const int v = L.view;
    for (int s = 0; s < g->G; s++) {
      for (int r = 0; r < g->G; r++) {
        if (r == s || !vring_receiver(g, r) || !vring_sender(g, s)) continue;
        const int src = rank_of(g, v, s), dst = rank_of(g, v, r);
        if (src != L.rank && dst != L.rank) continue;
        if (!g->comm && src != L.rank) continue;
        const GroupRank* D = g->comm ? &L : &g->loc[dst];
        xs.push_back({src, dst, g->comm ? (src == L.rank ? L.vsend[k] : nullptr) : L.vsend[k],
                      dst == D->rank ? D->vrecv[k][s] : nullptr, vring_words(g, s) * sizeof(uint32_t)});
      }
    }
  }
  if (int rc = run_xfers(g, xs, true)) return rc;
  for (GroupRank& L : g->loc) {
    hipSetDevice(L.c->cfg.device);
    hipEventRecord(L.ev_comm[k], L.comm);
    L.comm_pending[k] = true;
  }
  // a pure tracer writes the other ranks' validity rings into this frame's history (its next frame's seeds)
  for (GroupRank& L : g->loc) {
    if (!vring_receiver(g, L.vrank)) continue;
    hipSetDevice(L.c->cfg.device);
    hipStreamWaitEvent(L.c->stream, L.ev_comm[k], 0);
    for (int s = 0; s < g->G; s++)
      if (s != L.vrank && vring_sender(g, s))
        fr::launch_vring_unpack(L.vrecv[k][s], g->W, g->H, g->cfg.tile, L.tiles_dev + g->tile_off[s],
                                g->tiles_per_vrank[s], L.c->img[L.c->hist_cache], L.c->stream);
    L.c->hvalid_fresh = false;  // (the history no longer matches the validity bits of this frame's carry)
    if (int rc = fri::check_launch(L.c)) return gfail(rc, fr_last_error(L.c));
    hipEventRecord(L.ev_unpacked[k], L.c->stream);
    L.unpacked_pending[k] = true;
  }
  // scatter the received pixels into HISTORY_CACHE and SHADING (after this rank's own trace half)
  const uint32_t npix = (uint32_t)((size_t)g->W * g->H);
  for (GroupRank& L : g->loc) {
    bool any = false;
    for (int s = 0; s < g->G; s++) any |= receives(g, L.vrank, s) && L.n[s];
    if (!any) continue;
    hipSetDevice(L.c->cfg.device);
    hipStreamWaitEvent(L.c->stream, L.ev_comm[k], 0);
    for (int s = 0; s < g->G; s++) {
      if (!receives(g, L.vrank, s) || !L.n[s]) continue;
      const f4* vals = (const f4*)L.recv[k][s];
      const uint32_t* idx = (const uint32_t*)(L.recv[k][s] + (size_t)L.n[s] * sizeof(f4));
      fr::launch_shard_unpack_active(L.c->U, vals, idx, L.n[s], npix, L.c->img[fri::P_wgt(L.c)], L.c->img[L.c->hist_cur],
                                     L.c->img[L.c->hist_cache], L.c->img[fri::P_shd(L.c)], L.c->stream);
    }
    L.c->hvalid_fresh = false;
    if (int rc = fri::check_launch(L.c)) return gfail(rc, fr_last_error(L.c));
    hipEventRecord(L.ev_unpacked[k], L.c->stream);
    L.unpacked_pending[k] = true;
    // the unpack reads the slot's WEIGHT (the history gather): the slot goes back to the front stages of
    // frame + nslots (stream5 waits for ev_trace[slot]) only after it, as after the pack above
    hipEventRecord(L.c->ev_trace[L.c->slot], L.c->stream);
    L.c->trace_pending[L.c->slot] = true;
  }
  return FR_OK;
}

// The views' A-Trous images to rank 0 (after this frame's reconstruction), then side by side.
int composite(fr_group* g) {
  const size_t img = (size_t)g->W * g->H * sizeof(f4);
  const int ov = output_vrank(g);
  std::vector<Xfer> xs;
  GroupRank* root = nullptr;
  for (GroupRank& L : g->loc) if (L.rank == 0) root = &L;
  for (GroupRank& L : g->loc) {
    if (L.vrank != ov) continue;
    hipSetDevice(L.c->cfg.device);
    hipStreamWaitEvent(L.comm, L.c->ev_recon[L.c->slot], 0);  // this frame's A-Trous is written
    if (!g->comm) hipEventRecord(L.ev_packed, L.comm);
    const f4* src = L.c->img[L.c->atrous_out];
    if (L.rank == 0) {
      hipMemcpyAsync(L.comp_stack + (size_t)L.view * g->W * g->H, src, img, hipMemcpyDeviceToDevice, L.comm);
    } else if (g->comm) {
      xs.push_back({L.rank, 0, src, nullptr, img});
    } else {
      xs.push_back({L.rank, 0, src, root->comp_stack + (size_t)L.view * g->W * g->H, img});
    }
  }
  if (root && g->comm)
    for (int v = 0; v < g->V; v++) {
      const int src = rank_of(g, v, ov);
      if (src != 0) xs.push_back({src, 0, nullptr, root->comp_stack + (size_t)v * g->W * g->H, img});
    }
  if (int rc = run_xfers(g, xs, !g->comm)) return rc;
  // the next frame's A-Trous (stream2) overwrites an output image only after it left: with RCCL the
  // send is on the output rank's comm stream, in-process the copy is on rank 0's
  if (g->comm) {
    for (GroupRank& L : g->loc) {
      if (L.vrank != ov) continue;
      hipSetDevice(L.c->cfg.device);
      hipEventRecord(L.ev_sent_out, L.comm);
      L.c->recon_gate = L.ev_sent_out;
    }
  } else {
    hipSetDevice(root->c->cfg.device);
    hipEventRecord(root->ev_sent_out, root->comm);
    for (GroupRank& L : g->loc)
      if (L.vrank == ov) L.c->recon_gate = root->ev_sent_out;
  }
  if (root) {
    hipSetDevice(root->c->cfg.device);
    fr::launch_composite(root->comp_stack, g->V, g->W, g->H, root->comp_out, root->comm);
    if (int rc = fri::check_launch(root->c)) return gfail(rc, fr_last_error(root->c));
    hipEventRecord(root->ev_out, root->comm);
    g->composite_done = true;
  }
  return FR_OK;
}

}  // namespace

extern "C" {

int fr_group_config_default(fr_group_config* cfg) {
  if (!cfg) return FR_E_INVALID;
  memset(cfg, 0, sizeof(*cfg));
  cfg->views = 1;
  cfg->tile = 128;
  cfg->split_recon = 1;
  cfg->recon_cost[0] = 0.5f;
  cfg->recon_cost[1] = 0.17f;
  cfg->sample_sum = 2;
  cfg->front_local = 1;
  cfg->jfa_ranks = 0;
  return FR_OK;
}

int fr_rccl_unique_id(void* id128) {
  if (!id128) return FR_E_INVALID;
  ncclUniqueId id;
  if (int rc = rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId")) return rc;
  memcpy(id128, &id, sizeof(id));
  return FR_OK;
}

int fr_rccl_comm_init(const void* id128, int nranks, int rank, int device, void** comm) {
  if (!id128 || !comm || nranks < 1 || rank < 0 || rank >= nranks) return FR_E_INVALID;
  if (hipSetDevice(device) != hipSuccess) return gfail(FR_E_HIP, "fr_rccl_comm_init: hipSetDevice failed");
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclComm_t c = nullptr;
  if (int rc = rccl_check(ncclCommInitRank(&c, nranks, id, rank), "ncclCommInitRank")) return rc;
  *comm = c;
  return FR_OK;
}

int fr_rccl_comm_destroy(void* comm) {
  if (!comm) return FR_E_INVALID;
  return rccl_check(ncclCommDestroy((ncclComm_t)comm), "ncclCommDestroy");
}

int fr_group_destroy(fr_group* g) {
  if (!g) return FR_E_INVALID;
  for (GroupRank& L : g->loc) {
    if (L.c) {
      hipSetDevice(L.c->cfg.device);
      fr_synchronize(L.c);
      L.c->recon_gate = nullptr;
      L.c->recon_chains = 3;
      fr_set_shard_plan(L.c, 0, 1, 128, nullptr, 0);  // the whole screen again
    }
    free_rank(L);
  }
  delete g;
  return FR_OK;
}

int fr_group_create(fr_ctx* const* ctxs, int n, void* rccl_comm, const fr_group_config* cfg_in, fr_group** out) {
  if (!out) return gfail(FR_E_INVALID, "fr_group_create: out is NULL");
  *out = nullptr;
  if (!ctxs || n < 1) return gfail(FR_E_INVALID, "fr_group_create: need n >= 1 contexts");
  fr_group_config cfg;
  if (cfg_in) cfg = *cfg_in; else fr_group_config_default(&cfg);
  int R = n, my_rank = 0;
  if (rccl_comm) {
    if (n != 1) return gfail(FR_E_INVALID, "fr_group_create: with an RCCL communicator, one context per process");
    if (int rc = rccl_check(ncclCommCount((ncclComm_t)rccl_comm, &R), "ncclCommCount")) return rc;
    if (int rc = rccl_check(ncclCommUserRank((ncclComm_t)rccl_comm, &my_rank), "ncclCommUserRank")) return rc;
  }
  if (cfg.views < 1 || R % cfg.views) return gfail(FR_E_INVALID, "fr_group_create: views must divide the ranks");
  const int G = R / cfg.views;
  if (G > FR_GROUP_MAX_VIEW_RANKS) return gfail(FR_E_UNSUPPORTED, "fr_group_create: more than 16 ranks per view");
  if (cfg.tile < 16 || cfg.tile % 16 || cfg.tile > 4096) return gfail(FR_E_INVALID, "fr_group_create: tile must be a multiple of 16");
  if (cfg.sample_sum < -1 || cfg.sample_sum > 2) return gfail(FR_E_INVALID, "fr_group_create: sample_sum is -1, 0, 1 or 2");
  for (int i = 0; i < n; i++)
    if (!ctxs[i] || ctxs[i]->W != ctxs[0]->W || ctxs[i]->H != ctxs[0]->H || ctxs[i]->cfg.spp != ctxs[0]->cfg.spp)
      return gfail(FR_E_INVALID, "fr_group_create: every context needs the same width, height and spp");
  fr_group* g = new fr_group();
  g->cfg = cfg;
  g->R = R; g->V = cfg.views; g->G = G;
  g->W = ctxs[0]->W; g->H = ctxs[0]->H;
  g->comm = (ncclComm_t)rccl_comm;
  if (cfg.jfa_ranks < 0 || cfg.jfa_ranks > 1 + std::max(0, G - 2) || (cfg.jfa_ranks > 1 && !cfg.split_recon)) {
    delete g;
    return gfail(FR_E_INVALID, "fr_group_create: jfa_ranks is 0 (auto) or 1 .. G - 1, and above 1 only with split_recon");
  }
  g->jfa_ranks = jfa_ranks_for(G, cfg);
  auto bail = [&](int rc) { fr_group_destroy(g); return rc; };
  // the tile plan (the same in every view)
  const int T = cfg.tile;
  const size_t ntiles = (size_t)((g->W + T - 1) / T) * ((g->H + T - 1) / T);
  g->tiles_per_vrank.assign(G, 0);
  if (G > 1) {
    g->owner.resize(ntiles);
    if (int rc = group_plan(g->W, g->H, G, cfg, g->owner.data(), ntiles)) return bail(rc);
    for (uint8_t o : g->owner) g->tiles_per_vrank[o]++;
  }
  std::vector<int32_t> tiles_by_owner;
  g->tile_off.assign(G + 1, 0);
  for (int o = 0; o < G && G > 1; o++) {
    g->tile_off[o] = (int)tiles_by_owner.size();
    for (size_t t = 0; t < ntiles; t++)
      if (g->owner[t] == o) tiles_by_owner.push_back((int32_t)t);
  }
  g->tile_off[G] = (int)tiles_by_owner.size();
  g->loc.resize(n);
  for (int i = 0; i < n; i++) {
    GroupRank& L = g->loc[i];
    L.c = ctxs[i];
    L.rank = rccl_comm ? my_rank : i;
    L.view = view_of(g, L.rank);
    L.vrank = L.rank % G;
    L.chains = chains_of(g, L.vrank);
    L.tiles = G > 1 ? g->tiles_per_vrank[L.vrank] : (int)ntiles;
    fr_ctx* c = L.c;
    hipSetDevice(c->cfg.device);
    if (G > 1) {
      if (int rc = fr_set_shard_plan(c, L.vrank, G, T, g->owner.data(), ntiles))
        return bail(gfail(rc, std::string("fr_group_create: ") + fr_last_error(c)));
    } else if (int rc = fr_set_shard_plan(c, 0, 1, T, nullptr, 0)) {
      return bail(gfail(rc, std::string("fr_group_create: ") + fr_last_error(c)));
    }
    c->recon_chains = L.chains;
    if (G > 1 && cfg.sample_sum >= 0)
      if (int rc = fr_set_sample_sum(c, cfg.sample_sum)) return bail(gfail(rc, std::string("fr_group_create: ") + fr_last_error(c)));
    // a tracer of a still camera needs the front stages of its own tiles only (it receives nothing)
    if (G > 1 && L.chains == 0 && cfg.front_local && !cfg.moving_camera)
      if (int rc = fr_set_front_local(c, 1)) return bail(gfail(rc, std::string("fr_group_create: ") + fr_last_error(c)));
    if (hipStreamCreateWithFlags(&L.comm, hipStreamNonBlocking) != hipSuccess) return bail(gfail(FR_E_HIP, "group: stream"));
    hipEventCreateWithFlags(&L.ev_packed, hipEventDisableTiming);
    hipEventCreateWithFlags(&L.ev_out, hipEventDisableTiming);
    hipEventCreateWithFlags(&L.ev_sent_out, hipEventDisableTiming);
    const size_t T2 = (size_t)T * T;
    for (int k = 0; k < 2; k++) {
      hipEventCreateWithFlags(&L.ev_comm[k], hipEventDisableTiming);
      hipEventCreateWithFlags(&L.ev_unpacked[k], hipEventDisableTiming);
      L.recv[k].assign(G, nullptr);
      if (G == 1) continue;
      bool sends = false;
      for (int r = 0; r < G; r++) sends |= receives(g, r, L.vrank);
      if (sends && L.tiles && hipMalloc((void**)&L.send[k], (size_t)L.tiles * T2 * 20) != hipSuccess)
        return bail(gfail(FR_E_NOMEM, "group: send slab"));
      for (int s = 0; s < G; s++)
        if (receives(g, L.vrank, s) && g->tiles_per_vrank[s] &&
            hipMalloc((void**)&L.recv[k][s], (size_t)g->tiles_per_vrank[s] * T2 * 20) != hipSuccess)
          return bail(gfail(FR_E_NOMEM, "group: receive slab"));
    }
    if (G > 1 && !cfg.moving_camera) {
      if (hipMalloc((void**)&L.tiles_dev, tiles_by_owner.size() * sizeof(int32_t)) != hipSuccess ||
          hipMemcpy(L.tiles_dev, tiles_by_owner.data(), tiles_by_owner.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess)
        return bail(gfail(FR_E_NOMEM, "group: tile list"));
      for (int k = 0; k < 2; k++) {
        L.vrecv[k].assign(G, nullptr);
        if (vring_sender(g, L.vrank) && hipMalloc((void**)&L.vsend[k], vring_words(g, L.vrank) * sizeof(uint32_t)) != hipSuccess)
          return bail(gfail(FR_E_NOMEM, "group: validity ring slab"));
        for (int s2 = 0; s2 < G; s2++)
          if (s2 != L.vrank && vring_receiver(g, L.vrank) && vring_sender(g, s2) &&
              hipMalloc((void**)&L.vrecv[k][s2], vring_words(g, s2) * sizeof(uint32_t)) != hipSuccess)
            return bail(gfail(FR_E_NOMEM, "group: validity ring slab"));
      }
    }
    if (cfg.composite && L.rank == 0) {
      const size_t img = (size_t)g->W * g->H;
      if (hipMalloc((void**)&L.comp_stack, img * g->V * sizeof(f4)) != hipSuccess ||
          hipMalloc((void**)&L.comp_out, img * g->V * sizeof(f4)) != hipSuccess)
        return bail(gfail(FR_E_NOMEM, "group: composite buffers"));
    }
  }
  *out = g;
  return FR_OK;
}

int fr_group_frame(fr_group* g, fr_frame_timing* t) {
  if (!g) return FR_E_INVALID;
  const int n = (int)g->loc.size();
  // 1. every local rank's trace half (front stages on their own stream; entry 3 on its own tiles)
  for (int i = 0; i < n; i++) {
    GroupRank& L = g->loc[i];
    hipSetDevice(L.c->cfg.device);
    if (int rc = fri::frame_half(L.c, t ? &t[i] : nullptr, true, false))
      return gfail(rc, std::string("group trace half: ") + fr_last_error(L.c));
  }
  // 2. the traced pixels to the ranks that reconstruct (and, with a moving camera, to every rank)
  if (g->G > 1)
    if (int rc = exchange(g)) return rc;
  // 3. the reconstruction chains of this frame on their ranks
  const int turn = jfa_turn(g, g->frame);
  for (int i = 0; i < n; i++) {
    GroupRank& L = g->loc[i];
    const int run = g->G > 1 && L.vrank != turn ? (L.chains & ~1) : L.chains;
    if (!run) continue;
    hipSetDevice(L.c->cfg.device);
    L.c->recon_chains = run;
    fr_frame_timing rt{};
    if (int rc = fri::frame_half(L.c, t ? &rt : nullptr, false, true))
      return gfail(rc, std::string("group reconstruction: ") + fr_last_error(L.c));
    if (t) {
      t[i].jfa_ms = rt.jfa_ms; t[i].sibson_ms = rt.sibson_ms;
      t[i].pullpush_ms = rt.pullpush_ms; t[i].atrous_ms = rt.atrous_ms;
      t[i].total_ms += rt.total_ms;
    }
  }
  // 4. the final composite of the views on rank 0
  if (g->cfg.composite)
    if (int rc = composite(g)) return rc;
  g->frame++;
  if (t)
    if (int rc = fr_group_synchronize(g)) return rc;
  return FR_OK;
}

int fr_group_synchronize(fr_group* g) {
  if (!g) return FR_E_INVALID;
  for (GroupRank& L : g->loc) {
    hipSetDevice(L.c->cfg.device);
    if (hipStreamSynchronize(L.comm) != hipSuccess) return gfail(FR_E_HIP, "group: transfer failed");
    if (int rc = fr_synchronize(L.c)) return gfail(rc, fr_last_error(L.c));
  }
  if (g->comm) {
    ncclResult_t async = ncclSuccess;
    ncclCommGetAsyncError(g->comm, &async);
    if (async != ncclSuccess) return rccl_check(async, "RCCL");
  }
  return FR_OK;
}

int fr_group_composite(fr_group* g, void* out, size_t bytes) {
  if (!g || !out) return FR_E_INVALID;
  if (!g->cfg.composite) return gfail(FR_E_STATE, "fr_group_composite: the group was created without composite");
  for (GroupRank& L : g->loc) {
    if (L.rank != 0) continue;
    const size_t need = (size_t)g->V * g->W * g->H * sizeof(f4);
    if (bytes < need) return gfail(FR_E_INVALID, "fr_group_composite: output smaller than V * W * H * 16");
    if (!g->composite_done) return gfail(FR_E_STATE, "fr_group_composite: no frame yet");
    hipSetDevice(L.c->cfg.device);
    hipStreamWaitEvent(L.comm, L.ev_out, 0);
    if (hipMemcpyAsync(out, L.comp_out, need, hipMemcpyDeviceToDevice, L.comm) != hipSuccess ||
        hipStreamSynchronize(L.comm) != hipSuccess)
      return gfail(FR_E_HIP, "fr_group_composite: copy failed");
    return FR_OK;
  }
  return gfail(FR_E_STATE, "fr_group_composite: rank 0 is not local");
}

int fr_group_rank_info(fr_group* g, int i, int* view, int* view_rank, int* chains, int* tiles) {
  if (!g || i < 0 || i >= (int)g->loc.size()) return FR_E_INVALID;
  const GroupRank& L = g->loc[i];
  if (view) *view = L.view;
  if (view_rank) *view_rank = L.vrank;
  if (chains) *chains = L.chains;
  if (tiles) *tiles = L.tiles;
  return FR_OK;
}

int fr_group_plan(int width, int height, int ranks_per_view, const fr_group_config* cfg_in, uint8_t* owner,
                  size_t ntiles) {
  if (!owner || width <= 0 || height <= 0) return gfail(FR_E_INVALID, "fr_group_plan: bad arguments");
  fr_group_config cfg;
  if (cfg_in) cfg = *cfg_in; else fr_group_config_default(&cfg);
  const int G = ranks_per_view;
  if (G < 1 || G > FR_GROUP_MAX_VIEW_RANKS) return gfail(FR_E_INVALID, "fr_group_plan: 1 <= ranks_per_view <= 16");
  if (cfg.tile < 16 || cfg.tile % 16) return gfail(FR_E_INVALID, "fr_group_plan: tile must be a multiple of 16");
  if (cfg.jfa_ranks < 0 || cfg.jfa_ranks > 1 + std::max(0, G - 2) || (cfg.jfa_ranks > 1 && !cfg.split_recon))
    return gfail(FR_E_INVALID, "fr_group_plan: jfa_ranks is 0 (auto) or 1 .. G - 1, and above 1 only with split_recon");
  const size_t nt = (size_t)((width + cfg.tile - 1) / cfg.tile) * ((height + cfg.tile - 1) / cfg.tile);
  if (ntiles != nt) return gfail(FR_E_INVALID, "fr_group_plan: ntiles != ceil(W/tile) * ceil(H/tile)");
  if (G == 1) {
    memset(owner, 0, nt);
    return FR_OK;
  }
  return group_plan(width, height, G, cfg, owner, nt);
}

int fr_group_output_ranks(fr_group* g, int view, int* jfa_rank, int* atrous_rank) {
  if (!g || view < 0 || view >= g->V) return FR_E_INVALID;
  if (!g->frame) return gfail(FR_E_STATE, "fr_group_output_ranks: no frame yet");
  if (jfa_rank) *jfa_rank = rank_of(g, view, g->G > 1 ? jfa_turn(g, g->frame - 1) : 0);
  if (atrous_rank) *atrous_rank = rank_of(g, view, output_vrank(g));
  return FR_OK;
}

int fr_group_tile_owners(fr_group* g, uint8_t* owner, size_t ntiles) {
  if (!g || !owner) return FR_E_INVALID;
  const int T = g->cfg.tile;
  const size_t nt = (size_t)((g->W + T - 1) / T) * ((g->H + T - 1) / T);
  if (ntiles != nt) return gfail(FR_E_INVALID, "fr_group_tile_owners: ntiles != ceil(W/tile) * ceil(H/tile)");
  for (size_t t = 0; t < nt; t++) owner[t] = g->G > 1 ? g->owner[t] : 0;
  return FR_OK;
}

const char* fr_group_last_error(void) { return g_group_error.c_str(); }

}  // extern "C"
