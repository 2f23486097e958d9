// pp2_shards.cpp -- single-process row-shard groups (pp2_shard_group_*).
//
// One host thread drives the row shards of one grid, each a pp2_ctx on its own
// stream (and device, or all on one device).  Every step runs phase-wise:
//   1. each shard waits for its neighbours' previous step, then copies their
//      boundary rows into its halo rows (device-to-device / peer copies);
//   2. each shard runs its local kernels (the same launches as unsharded);
//   3. the shards' partial belief masses are combined in rank order on shard
//      0's stream and copied back to every shard.
// This is the RCCL path of pp2_runtime.cpp (ncclSend/ncclRecv halo rows +
// ncclAllReduce of the mass) with a different transport, so it exercises the
// same shard geometry, halo semantics and mass bookkeeping on one GPU.
#include <algorithm>
#include <vector>

#include "pp2_ctx.h"

using namespace pp2rt;

struct pp2_shard_group {
  std::vector<pp2_ctx*> ctx;
  std::vector<hipEvent_t> ev_done, ev_local;
  hipEvent_t ev_total = nullptr;
  float* d_gather = nullptr;  // on shard 0's device: n masses + total
};

namespace {

int wait_neighbours(pp2_shard_group* g) {
  const int n = (int)g->ctx.size();
  for (int r = 0; r < n; ++r) {
    DeviceGuard dg(g->ctx[r]->device);
    if (r > 0) HIPCHK(hipStreamWaitEvent(g->ctx[r]->stream, g->ev_done[r - 1], 0));
    if (r < n - 1) HIPCHK(hipStreamWaitEvent(g->ctx[r]->stream, g->ev_done[r + 1], 0));
  }
  return PP2_OK;
}

// k halo rows per side: the neighbours' owned rows [rows-k, rows) / [0, k)
// into this shard's halo rows [-k, 0) / [rows, rows+k).
int exchange_local(pp2_shard_group* g, std::initializer_list<HaloKind> kinds, int k = 1) {
  const int n = (int)g->ctx.size();
  for (int r = 0; r < n; ++r) {
    pp2_ctx* c = g->ctx[r];
    DeviceGuard dg(c->device);
    for (HaloKind kd : kinds) {
      const Planes& P = halo_planes(c, kd);
      const size_t bytes = (size_t)k * P.v.rs * sizeof(float);
      if (r > 0) {
        pp2_ctx* up = g->ctx[r - 1];
        const Planes& Q = halo_planes(up, kd);
        HIPCHK(hipMemcpyAsync(P.v.p - k * P.v.rs, Q.v.p + (long long)(up->g.rows - k) * Q.v.rs,
                              bytes, hipMemcpyDefault, c->stream));
      }
      if (r < n - 1) {
        const Planes& Q = halo_planes(g->ctx[r + 1], kd);
        HIPCHK(hipMemcpyAsync(P.v.p + (long long)c->g.rows * P.v.rs, Q.v.p, bytes,
                              hipMemcpyDefault, c->stream));
      }
    }
  }
  return PP2_OK;
}

// Global mass = sum of shard masses in rank order, written to every shard.
int combine_mass(pp2_shard_group* g) {
  const int n = (int)g->ctx.size();
  pp2_ctx* c0 = g->ctx[0];
  for (int r = 0; r < n; ++r) {
    DeviceGuard dg(g->ctx[r]->device);
    HIPCHK(hipEventRecord(g->ev_local[r], g->ctx[r]->stream));
  }
  {
    DeviceGuard dg(c0->device);
    for (int r = 0; r < n; ++r) {
      HIPCHK(hipStreamWaitEvent(c0->stream, g->ev_local[r], 0));
      pp2_ctx* c = g->ctx[r];
      HIPCHK(hipMemcpyAsync(g->d_gather + r, c->bsum + c->bcur, sizeof(float),
                            hipMemcpyDefault, c0->stream));
    }
    HIPCHK(pp2::launch_sum_ordered(c0->stream, g->d_gather, n, g->d_gather + n));
    HIPCHK(hipEventRecord(g->ev_total, c0->stream));
  }
  for (int r = 0; r < n; ++r) {
    pp2_ctx* c = g->ctx[r];
    DeviceGuard dg(c->device);
    HIPCHK(hipStreamWaitEvent(c->stream, g->ev_total, 0));
    HIPCHK(hipMemcpyAsync(c->bsum + c->bcur, g->d_gather + n, sizeof(float),
                          hipMemcpyDefault, c->stream));
  }
  return PP2_OK;
}

int mark_done(pp2_shard_group* g) {
  for (size_t r = 0; r < g->ctx.size(); ++r) {
    DeviceGuard dg(g->ctx[r]->device);
    HIPCHK(hipEventRecord(g->ev_done[r], g->ctx[r]->stream));
  }
  return PP2_OK;
}

int check_group(pp2_shard_group* g) {
  if (!g || g->ctx.empty()) return set_err(PP2_EINVAL, "null shard group");
  for (pp2_ctx* c : g->ctx) CHECK(check_model(c));
  return PP2_OK;
}

}  // namespace

extern "C" {

int pp2_shard_group_destroy(pp2_shard_group* g);

int pp2_shard_group_create(pp2_shard_group** out, pp2_ctx* const* ctxs, int n) {
  if (!out || !ctxs || n < 1) return set_err(PP2_EINVAL, "bad shard group arguments");
  *out = nullptr;
  int next_row = 0, grows = -1, width = -1;
  for (int r = 0; r < n; ++r) {
    pp2_ctx* c = ctxs[r];
    CHECK(check_ctx(c));
    if (c->group || c->nranks > 1)
      return set_err(PP2_ESTATE, "context %d already belongs to a group / RCCL comm", r);
    if (grows < 0) { grows = c->g.grows; width = c->g.width; }
    if (c->g.grows != grows || c->g.width != width || c->g.row0 != next_row)
      return set_err(PP2_EINVAL, "contexts are not consecutive row shards of one grid");
    next_row += c->g.rows;
  }
  if (next_row != grows) return set_err(PP2_EINVAL, "shards do not cover the grid");
  pp2_shard_group* g = new pp2_shard_group();
  g->ctx.assign(ctxs, ctxs + n);
  g->ev_done.assign(n, nullptr);
  g->ev_local.assign(n, nullptr);
  auto fail = [&](int s) {
    pp2_shard_group_destroy(g);
    return s;
  };
  // peer access between the shards' devices (a no-op on one device)
  for (int r = 0; r < n; ++r)
    for (int q = 0; q < n; ++q) {
      const int a = ctxs[r]->device, b = ctxs[q]->device;
      if (a == b) continue;
      DeviceGuard dg(a);
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
        hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
          return fail(set_err(PP2_EHIP, "peer access %d->%d: %s", a, b, hipGetErrorString(e)));
        (void)hipGetLastError();
      }
    }
  for (int r = 0; r < n; ++r) {
    DeviceGuard dg(ctxs[r]->device);
    if (hipEventCreateWithFlags(&g->ev_done[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_local[r], hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(g->ev_done[r], ctxs[r]->stream) != hipSuccess)
      return fail(set_err(PP2_EHIP, "shard group events"));
  }
  {
    DeviceGuard dg(ctxs[0]->device);
    if (hipEventCreateWithFlags(&g->ev_total, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&g->d_gather, (pp2::kVecRec * n + 1) * sizeof(float)) != hipSuccess)
      return fail(set_err(PP2_ENOMEM, "shard group scratch"));
  }
  int min_rows = ctxs[0]->g.rows;
  for (int r = 0; r < n; ++r) min_rows = std::min(min_rows, ctxs[r]->g.rows);
  for (int r = 0; r < n; ++r) {
    ctxs[r]->group = g;
    ctxs[r]->grank = r;
    ctxs[r]->group_size = n;
    ctxs[r]->min_shard_rows = min_rows;
    ctxs[r]->kdepth_max = std::max(1, std::min(std::min(ctxs[r]->g.halo, kMaxNormBlock), min_rows));
    ctxs[r]->kdepth = ctxs[r]->kdepth_max;
    ctxs[r]->res_e_dict = -1;
    break_pipeline(ctxs[r]);
  }
  *out = g;
  return PP2_OK;
}

int pp2_shard_group_destroy(pp2_shard_group* g) {
  if (!g) return PP2_OK;
  (void)pp2_shard_group_synchronize(g);
  for (size_t r = 0; r < g->ctx.size(); ++r) {
    DeviceGuard dg(g->ctx[r]->device);
    if (g->ev_done[r]) (void)hipEventDestroy(g->ev_done[r]);
    if (g->ev_local[r]) (void)hipEventDestroy(g->ev_local[r]);
    if (g->ctx[r]->group == g) {
      g->ctx[r]->group = nullptr;
      g->ctx[r]->group_size = 0;
      g->ctx[r]->res_e_dict = -1;
      if (g->ctx[r]->d_vec) (void)hipFree(g->ctx[r]->d_vec);
      g->ctx[r]->d_vec = nullptr;
    }
  }
  if (!g->ctx.empty()) {
    DeviceGuard dg(g->ctx[0]->device);
    if (g->ev_total) (void)hipEventDestroy(g->ev_total);
    if (g->d_gather) (void)hipFree(g->d_gather);
  }
  delete g;
  return PP2_OK;
}

int pp2_shard_group_synchronize(pp2_shard_group* g) {
  if (!g) return set_err(PP2_EINVAL, "null shard group");
  for (pp2_ctx* c : g->ctx) {
    DeviceGuard dg(c->device);
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  for (pp2_ctx* c : g->ctx) CHECK(check_ctx_settled(c));
  return PP2_OK;
}

// The RCCL row-shard loop step (pp2_runtime.cpp blocked_loop_step) with
// device copies as the transport: a block starts by refreshing the halo rows
// of b and J kdepth rows deep, and its first step divides by the global mass
// (times 2^96) and the others by 1; step i computes a view kdepth-1-i rows
// wider per side.  (The group also combines the mass after every step, so a
// shard's bsum always holds the global mass for reads.)
// Every shard of the group at the same halo depth and block phase (a
// per-shard PP2_TUNE_HALO_DEPTH or pipeline restart breaks that).
static int check_in_step(pp2_shard_group* g) {
  pp2_ctx* c0 = g->ctx[0];
  for (pp2_ctx* c : g->ctx)
    if (c->kdepth != c0->kdepth || c->kstep != c0->kstep)
      return set_err(PP2_ESTATE, "shards of the group are out of step (halo depth differs?)");
  return PP2_OK;
}

int pp2_shard_group_loop_step(pp2_shard_group* g, uint8_t u, uint8_t z) {
  CHECK(check_group(g));
  if (u > 8 || z > 15) return set_err(PP2_EINVAL, "action %u / observation %u out of range", u, z);
  CHECK(check_in_step(g));
  pp2_ctx* c0 = g->ctx[0];
  const int K = c0->kdepth;
  CHECK(wait_neighbours(g));
  const bool start = c0->kstep == 0;
  if (start) CHECK(exchange_local(g, {HALO_BELIEF, HALO_VALUE}, K));
  for (pp2_ctx* c : g->ctx) {
    DeviceGuard dg(c->device);
    const int bc = c->bcur, bn = bc ^ 1;
    int nparts = 0;
    CHECK(loop_launch(c, K - 1 - c->kstep, u, z, nullptr, 0, start ? c->bsum + bc : nullptr,
                      nullptr, &nparts, start ? kBlockScale : 1.0f));
    HIPCHK(pp2::launch_sum_finalize(c->stream, c->pbuf[bn], nparts, c->bsum + bn));
    c->pending[bc] = c->pending[bn] = false;
    c->bcur = bn;
    c->jcur ^= 1;
    c->kstep = (c->kstep + 1) % K;
  }
  CHECK(combine_mass(g));
  return mark_done(g);
}

// Two loop steps of a halo block on every shard in one launch each
// (pp2rt::pair_launch on the view of step kstep + 1; step kstep is computed
// one row deeper from the halo), the mass combined after the pair.
static int group_loop_pair(pp2_shard_group* g, uint8_t u1, uint8_t z1, uint8_t u2, uint8_t z2) {
  pp2_ctx* c0 = g->ctx[0];
  const int K = c0->kdepth;
  CHECK(wait_neighbours(g));
  const bool start = c0->kstep == 0;
  if (start) CHECK(exchange_local(g, {HALO_BELIEF, HALO_VALUE}, K));
  for (pp2_ctx* c : g->ctx) {
    DeviceGuard dg(c->device);
    const int bc = c->bcur, bn = bc ^ 1;
    int nparts = 0;
    CHECK(pair_launch(c, K - 2 - c->kstep, true, u1, z1, u2, z2, nullptr, 0, nullptr,
                      start ? c->bsum + bc : nullptr, start ? kBlockScale : 1.0f, &nparts));
    HIPCHK(pp2::launch_sum_finalize(c->stream, c->pbuf[bn], nparts, c->bsum + bn));
    c->pending[bc] = c->pending[bn] = false;
    c->bcur = bn;
    c->jcur ^= 1;
    c->kstep = (c->kstep + 2) % K;
  }
  CHECK(combine_mass(g));
  return mark_done(g);
}

// {mass, shift} of every shard into every shard's d_vec: each posts its slot,
// shard 0's stream gathers the slots in rank order, every shard copies the
// whole vector back (the RCCL path's all-reduce).
static int group_share_vec(pp2_shard_group* g) {
  const int n = (int)g->ctx.size();
  for (int r = 0; r < n; ++r) {
    pp2_ctx* c = g->ctx[r];
    DeviceGuard dg(c->device);
    CHECK(shard_post_mass(c, n, r));
    HIPCHK(hipEventRecord(g->ev_local[r], c->stream));
  }
  pp2_ctx* c0 = g->ctx[0];
  {
    DeviceGuard dg(c0->device);
    for (int r = 0; r < n; ++r) {
      HIPCHK(hipStreamWaitEvent(c0->stream, g->ev_local[r], 0));
      HIPCHK(hipMemcpyAsync(g->d_gather + pp2::kVecRec * r, g->ctx[r]->d_vec + pp2::kVecRec * r,
                            pp2::kVecRec * sizeof(float), hipMemcpyDefault, c0->stream));
    }
    HIPCHK(hipEventRecord(g->ev_total, c0->stream));
  }
  for (int r = 0; r < n; ++r) {
    pp2_ctx* c = g->ctx[r];
    DeviceGuard dg(c->device);
    HIPCHK(hipStreamWaitEvent(c->stream, g->ev_total, 0));
    HIPCHK(hipMemcpyAsync(c->d_vec, g->d_gather, pp2::kVecRec * n * sizeof(float),
                          hipMemcpyDefault, c->stream));
  }
  return PP2_OK;
}

// pp2_loop_run's resident shard path for a group (pp2_runtime.cpp
// shard_loop_resident with device copies as the transport): blocks of m <= e
// steps, each after the {mass, shift} exchange + rebase and e halo rows, then
// the closing exchange + rebase.  Resident launches of the shards run one at
// a time per device (the runtime's gate), each on the whole GPU.
static int group_loop_resident(pp2_shard_group* g, int e, int n, const uint8_t* us,
                               const uint8_t* zs) {
  for (int i = 0; i < n; ++i)
    if (us[i] > 8 || zs[i] > 15)
      return set_err(PP2_EINVAL, "action %u / observation %u out of range", us[i], zs[i]);
  const int ns = (int)g->ctx.size();
  for (pp2_ctx* c : g->ctx) break_pipeline(c);
  for (int i = 0; i < n;) {
    const int m = std::min(e, n - i);
    CHECK(wait_neighbours(g));
    const bool pend = g->ctx[0]->pending[g->ctx[0]->bcur];
    if (pend) CHECK(group_share_vec(g));
    CHECK(exchange_local(g, {HALO_BELIEF, HALO_VALUE}, e));
    if (pend) {  // the neighbours have copied our rows before we rebase them
      CHECK(mark_done(g));
      CHECK(wait_neighbours(g));
    }
    for (int r = 0; r < ns; ++r) {
      pp2_ctx* c = g->ctx[r];
      DeviceGuard dg(c->device);
      if (pend) CHECK(shard_rebase(c, ns, r, -e, c->g.rows + e));
      CHECK(shard_resident_launch(c, e, m, us + i, zs + i));
    }
    CHECK(mark_done(g));
    i += m;
  }
  CHECK(group_share_vec(g));
  for (int r = 0; r < ns; ++r) {
    pp2_ctx* c = g->ctx[r];
    DeviceGuard dg(c->device);
    CHECK(shard_rebase(c, ns, r, 0, c->g.rows));
    break_pipeline(c);
  }
  return mark_done(g);
}

int pp2_shard_group_loop_run(pp2_shard_group* g, int n, const uint8_t* us, const uint8_t* zs) {
  CHECK(check_group(g));
  if (n < 0 || (n > 0 && (!us || !zs))) return set_err(PP2_EINVAL, "bad trajectory");
  CHECK(check_in_step(g));
  if (n >= 2) {
    int e = 1 << 30;  // the deepest halo every shard can run
    for (pp2_ctx* c : g->ctx) e = std::min(e, shard_resident_e(c));
    bool ok = e > 0;
    for (pp2_ctx* c : g->ctx) ok = ok && shard_resident_ready(c, e);
    if (ok) return group_loop_resident(g, e, n, us, zs);
  }
  for (int i = 0; i < n;) {
    pp2_ctx* c0 = g->ctx[0];
    bool pair = i + 1 < n && c0->kstep + 2 <= c0->kdepth;
    for (pp2_ctx* c : g->ctx) pair = pair && pairs_apply(c);
    if (pair) {
      for (int k = 0; k < 2; ++k)
        if (us[i + k] > 8 || zs[i + k] > 15)
          return set_err(PP2_EINVAL, "action %u / observation %u out of range", us[i + k],
                         zs[i + k]);
      CHECK(group_loop_pair(g, us[i], zs[i], us[i + 1], zs[i + 1]));
      i += 2;
    } else {
      CHECK(pp2_shard_group_loop_step(g, us[i], zs[i]));
      ++i;
    }
  }
  return PP2_OK;
}

int pp2_shard_group_belief_update(pp2_shard_group* g, uint8_t u, uint8_t z) {
  CHECK(check_group(g));
  CHECK(wait_neighbours(g));
  CHECK(exchange_local(g, {HALO_BELIEF}));
  for (pp2_ctx* c : g->ctx) {
    DeviceGuard dg(c->device);
    CHECK(belief_update_impl(c, u, z, false));
  }
  CHECK(combine_mass(g));
  return mark_done(g);
}

int pp2_shard_group_mdp_sweep(pp2_shard_group* g, int n) {
  CHECK(check_group(g));
  if (n < 0) return set_err(PP2_EINVAL, "negative sweep count");
  for (int i = 0; i < n; ++i) {
    CHECK(wait_neighbours(g));
    CHECK(exchange_local(g, {HALO_VALUE}));
    for (pp2_ctx* c : g->ctx) {
      DeviceGuard dg(c->device);
      CHECK(mdp_sweep_once(c));
    }
    CHECK(mark_done(g));
  }
  return PP2_OK;
}

int pp2_shard_group_fib_sweep(pp2_shard_group* g, int n) {
  CHECK(check_group(g));
  if (n < 0) return set_err(PP2_EINVAL, "negative sweep count");
  for (int i = 0; i < n; ++i) {
    CHECK(wait_neighbours(g));
    CHECK(exchange_local(g, {HALO_FIB}));
    for (pp2_ctx* c : g->ctx) {
      DeviceGuard dg(c->device);
      CHECK(fib_sweep_once(c));
    }
    CHECK(mark_done(g));
  }
  return PP2_OK;
}

int pp2_shard_group_mdp_solve(pp2_shard_group* g, int max_sweeps, int* sweeps,
                              double* final_norm) {
  CHECK(check_group(g));
  for (pp2_ctx* c : g->ctx) CHECK(pp2_mdp_reset(c));
  CHECK(mark_done(g));
  const double max_cost = 5.0 / (1.0 - (double)g->ctx[0]->gamma);
  int total = 0;
  double norm = 0.0;
  do {
    CHECK(pp2_shard_group_mdp_sweep(g, 100));
    total += 100;
    float m = 0.0f;
    for (pp2_ctx* c : g->ctx) {
      DeviceGuard dg(c->device);
      float mr = 0.0f;
      CHECK(absdiff_local_max(c, c->J[c->jcur], c->Jsnap, &mr));
      m = std::max(m, mr);
    }
    norm = (double)m;
    if (max_sweeps > 0 && total >= max_sweeps) break;
  } while (norm > max_cost * 1e-3);
  if (sweeps) *sweeps = total;
  if (final_norm) *final_norm = norm;
  return PP2_OK;
}

}  // extern "C"
