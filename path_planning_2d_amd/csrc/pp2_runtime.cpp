// pp2_runtime.cpp -- the C ABI of libpp2_hip.so (include/pp2.h).
//
// Owns device memory, streams and the drivers around the gfx950 kernels
// (pp2_kernels.hip).  Replaces the reference's dev_*/host_* globals and the
// allocate/free/generate/load/save free functions (see pp2.h for per-entry
// citations).  Errors are returned as pp2_status with a thread-local message;
// nothing here exits the process.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cfloat>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "pp2_ctx.h"

using pp2::Geom;
using pp2::PlaneSet;

namespace pp2rt {

thread_local std::string g_last_error;

int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}


int alloc_planes(pp2_ctx* c, Planes* P, int K, int halo) {
  if (halo < 0) halo = c->g.halo;
  const long long rs = (long long)K * c->g.wp;
  P->K = K;
  P->floats = (size_t)(2 * kGuard) + (size_t)(c->g.rows + 2 * halo) * rs;
  HIPCHK(hipMalloc(&P->alloc, P->floats * sizeof(float)));
  HIPCHK(hipMemsetAsync(P->alloc, 0, P->floats * sizeof(float), c->stream));
  P->v.p = P->alloc + kGuard + (long long)halo * rs;  // skip the top halo rows
  P->v.rs = rs;
  P->v.ps = c->g.wp;
  return PP2_OK;
}

void free_planes(Planes* P) {
  if (P->alloc) (void)hipFree(P->alloc);
  P->alloc = nullptr;
}

int ensure_staging(pp2_ctx* c, size_t bytes) {
  if (c->staging_bytes >= bytes) return PP2_OK;
  if (c->staging) HIPCHK(hipFree(c->staging));
  c->staging = nullptr;
  c->staging_bytes = 0;
  HIPCHK(hipMalloc(&c->staging, bytes));
  c->staging_bytes = bytes;
  return PP2_OK;
}

// Every entry point: a null check, then the journalled resident launch is
// verified (and re-run if it timed out) before the call reads or builds on
// its outputs; a shard whose resident run was lost refuses until its state
// is set again.
int check_ctx_settled(pp2_ctx* c) {
  if (!c) return set_err(PP2_EINVAL, "null context");
  return resident_settle(c);
}
int check_ctx(pp2_ctx* c) {
  CHECK(check_ctx_settled(c));
  if (c->lost_belief || c->lost_values)
    return set_err(PP2_ESTATE, "a resident shard run of this context timed out: set the %s again",
                   c->lost_belief && c->lost_values ? "belief and values (pp2_belief_set, "
                   "pp2_mdp_reset)" : c->lost_belief ? "belief (pp2_belief_set)" :
                   "values (pp2_mdp_reset)");
  return PP2_OK;
}

int check_model(pp2_ctx* c) {
  CHECK(check_ctx(c));
  if (!c->model_ready)
    return set_err(PP2_ESTATE, "model not generated or uploaded");
  return PP2_OK;
}

size_t owned_cells(const pp2_ctx* c) { return (size_t)c->g.rows * c->g.width; }

const Planes& halo_planes(pp2_ctx* c, HaloKind k) {
  switch (k) {
    case HALO_BELIEF: return c->b[c->bcur];
    case HALO_VALUE: return c->J[c->jcur];
    default: return c->fib[c->fcur];
  }
}

// Every RCCL operation of a context is issued in host order (the same on
// every rank) on cst(c): by default the compute stream itself, so a block
// start costs no cross-stream hand-off; with PP2_TUNE_COMM_STREAM 1 a
// dedicated comm stream, entered and left through events.
hipStream_t cst(const pp2_ctx* c) { return c->use_comm_stream ? c->comm_stream : c->stream; }

// With PP2_TUNE_COMM_TIMING, a round's begin event is recorded on cst(c)
// after the enter hand-off and its end event before the leave hand-off, so
// the pair brackets the RCCL group alone (including the wait for the peers).
static int comm_time_mark(pp2_ctx* c, bool begin) {
  if (!c->comm_timing || !c->comm) return PP2_OK;
  if (begin) {
    c->comm_open = c->comm_nev < pp2_ctx::kCommTimed;
    if (!c->comm_open) {
      ++c->comm_dropped;
      return PP2_OK;
    }
    if (c->comm_ev.empty()) {
      c->comm_ev.assign(2 * pp2_ctx::kCommTimed, nullptr);
      for (hipEvent_t& e : c->comm_ev) HIPCHK(hipEventCreate(&e));
    }
    HIPCHK(hipEventRecord(c->comm_ev[2 * c->comm_nev], cst(c)));
    return PP2_OK;
  }
  if (!c->comm_open) return PP2_OK;
  HIPCHK(hipEventRecord(c->comm_ev[2 * c->comm_nev + 1], cst(c)));
  ++c->comm_nev;
  c->comm_open = false;
  return PP2_OK;
}

int comm_enter(pp2_ctx* c) {
  if (c->use_comm_stream) {
    HIPCHK(hipEventRecord(c->ev_enter, c->stream));
    HIPCHK(hipStreamWaitEvent(c->comm_stream, c->ev_enter, 0));
  }
  return comm_time_mark(c, true);
}

int comm_leave(pp2_ctx* c) {
  CHECK(comm_time_mark(c, false));
  if (!c->use_comm_stream) return PP2_OK;
  HIPCHK(hipEventRecord(c->ev_leave, c->comm_stream));
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_leave, 0));
  return PP2_OK;
}

// k halo rows up and down for each state kind, in one RCCL group
// (multi-process shards): owned rows [0, k) and [rows-k, rows) go to the
// neighbours' halo rows [rows, rows+k) and [-k, 0).  With records, the same
// group also sends this rank's {mass, shift, lost} record of d_vec to every
// other rank and receives theirs (the shard all-reduce as point-to-point
// messages, so that a resident block start costs ONE RCCL round: the halo
// rows travel unrebased and the rebase after the group scales them by their
// owner's shift).  Within a group the messages between two ranks match in
// issue order, which is the same on both sides: the record first, then the
// kinds' rows.  Shards of a single-process group exchange through the
// pp2_shard_group_* drivers.
int exchange_halos_k(pp2_ctx* c, std::initializer_list<HaloKind> kinds, int k,
                     bool records = false) {
  if (c->group)
    return set_err(PP2_ESTATE, "context belongs to a shard group: drive it with pp2_shard_group_*");
  if (!c->comm) {
    if (c->nranks > 1) return set_err(PP2_ESTATE, "sharded context without RCCL comm");
    return PP2_OK;
  }
  CHECK(comm_enter(c));
  NCCLCHK(ncclGroupStart());
  if (records) {
    const int R = pp2::kVecRec;
    for (int q = 0; q < c->nranks; ++q) {
      if (q == c->rank) continue;
      NCCLCHK(ncclSend(c->d_vec + R * c->rank, R, ncclFloat, q, c->comm, cst(c)));
      NCCLCHK(ncclRecv(c->d_vec + R * q, R, ncclFloat, q, c->comm, cst(c)));
    }
  }
  for (HaloKind kd : kinds) {
    const Planes* P = &halo_planes(c, kd);
    float* p = P->v.p;
    const long long rs = P->v.rs;
    const size_t n = (size_t)k * rs;
    if (c->rank > 0) {
      NCCLCHK(ncclSend(p, n, ncclFloat, c->rank - 1, c->comm, cst(c)));
      NCCLCHK(ncclRecv(p - k * rs, n, ncclFloat, c->rank - 1, c->comm, cst(c)));
    }
    if (c->rank < c->nranks - 1) {
      NCCLCHK(ncclSend(p + (long long)(c->g.rows - k) * rs, n, ncclFloat, c->rank + 1, c->comm,
                       cst(c)));
      NCCLCHK(ncclRecv(p + (long long)c->g.rows * rs, n, ncclFloat, c->rank + 1, c->comm,
                       cst(c)));
    }
  }
  NCCLCHK(ncclGroupEnd());
  return comm_leave(c);
}

int exchange_halos(pp2_ctx* c, std::initializer_list<HaloKind> kinds) {
  return exchange_halos_k(c, kinds, 1);
}

int allreduce_mass(pp2_ctx* c, float* d) {
  if (!c->comm) return PP2_OK;
  CHECK(comm_enter(c));
  NCCLCHK(ncclAllReduce(d, d, 1, ncclFloat, ncclSum, c->comm, cst(c)));
  return comm_leave(c);
}

int absdiff_local_max(pp2_ctx* c, const Planes& cur, const Planes& snap, float* out);

// max |cur - snap| over owned cells/planes (global over RCCL shards); snap := cur.
int absdiff_max(pp2_ctx* c, const Planes& cur, const Planes& snap, double* out) {
  float m = 0.0f;
  CHECK(absdiff_local_max(c, cur, snap, &m));
  if (c->nranks > 1) {
    HIPCHK(hipMemcpyAsync(c->rpartials, &m, sizeof(float), hipMemcpyHostToDevice, c->stream));
    CHECK(comm_enter(c));
    NCCLCHK(ncclAllReduce(c->rpartials, c->rpartials, 1, ncclFloat, ncclMax, c->comm,
                          cst(c)));
    CHECK(comm_leave(c));
    HIPCHK(hipMemcpyAsync(&m, c->rpartials, sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  *out = (double)m;
  return PP2_OK;
}

int create_impl(pp2_ctx** out, int device, uint32_t grows, uint32_t width,
                uint32_t row_begin, uint32_t row_end, const uint8_t* map,
                int32_t gx, int32_t gy, float gamma, bool shard) {
  if (!out) return set_err(PP2_EINVAL, "out is null");
  *out = nullptr;
  if (!map) return set_err(PP2_EINVAL, "map is null");
  if (grows == 0 || width == 0 || row_begin >= row_end || row_end > grows)
    return set_err(PP2_EINVAL, "bad geometry %ux%u rows [%u,%u)", grows, width,
                   row_begin, row_end);
  if (!(gamma > 0.0f && gamma < 1.0f))
    return set_err(PP2_EINVAL, "discount factor %g not in (0,1)", (double)gamma);
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return set_err(PP2_EINVAL, "device %d out of range (%d devices)", device, ndev);
  DeviceGuard dg(device);

  pp2_ctx* c = new pp2_ctx();
  c->device = device;
  c->g.rows = (int)(row_end - row_begin);
  c->g.width = (int)width;
  c->g.wp = (int)((width + 3u) & ~3u);
  c->g.row0 = (int)row_begin;
  c->g.grows = (int)grows;
  c->g.halo = shard ? kShardHalo : 1;  // shards: room for deep halo exchanges
  c->dense_halo = std::min(c->g.halo, kDenseHalo);
  c->gx = gx;
  c->gy = gy;
  c->gamma = gamma;
  auto fail = [&](int s) {
    pp2_destroy(c);
    return s;
  };
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess)
    return fail(set_err(PP2_EHIP, "hipStreamCreate failed"));
  c->stream = c->own_stream;
  if (hipDeviceGetAttribute(&c->ncus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    c->ncus = 0;

  // the map rows the model generation reads: the shard's rows and halo rows
  // plus one more per side (a shard keeps its window, not the whole map)
  const long long mlo = std::max(0LL, (long long)row_begin - c->g.halo - 1);
  const long long mhi = std::min((long long)grows, (long long)row_end + c->g.halo + 1);
  const size_t map_bytes = (size_t)(mhi - mlo) * width;
  if (hipMalloc(&c->d_map_alloc, map_bytes) != hipSuccess)
    return fail(set_err(PP2_ENOMEM, "hipMalloc map (%zu B)", map_bytes));
  c->d_map = c->d_map_alloc - mlo * (long long)width;  // indexed by global row
  if (hipMemcpyAsync(c->d_map_alloc, map + mlo * (long long)width, map_bytes,
                     hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return fail(set_err(PP2_EHIP, "map upload"));

  int s = PP2_OK;
  const int dh = c->dense_halo;
  if ((s = alloc_planes(c, &c->T, 81, dh)) || (s = alloc_planes(c, &c->L, 16, dh)) ||
      (s = alloc_planes(c, &c->R, 9, dh)) || (s = alloc_planes(c, &c->C, 9, dh)) ||
      (s = alloc_planes(c, &c->b[0], 1)) || (s = alloc_planes(c, &c->b[1], 1)) ||
      (s = alloc_planes(c, &c->J[0], 1)) || (s = alloc_planes(c, &c->J[1], 1)) ||
      (s = alloc_planes(c, &c->Jsnap, 1)) || (s = alloc_planes(c, &c->fib[0], 9, dh)) ||
      (s = alloc_planes(c, &c->fib[1], 9, dh)) || (s = alloc_planes(c, &c->fibsnap, 9, dh)))
    return fail(s);
  const size_t abytes = (size_t)c->g.rows * c->g.wp + 16;
  if (hipMalloc(&c->A, abytes) != hipSuccess ||
      hipMemsetAsync(c->A, 0, abytes, c->stream) != hipSuccess)
    return fail(set_err(PP2_ENOMEM, "hipMalloc actions"));
  if (hipMalloc(&c->bsum, 4 * sizeof(float)) != hipSuccess)
    return fail(set_err(PP2_ENOMEM, "hipMalloc bsum"));
  const float ones[4] = {1.0f, 1.0f, 1.0f, 1.0f};
  if (hipMemcpyAsync(c->bsum, ones, sizeof ones, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return fail(set_err(PP2_EHIP, "bsum init"));
  Geom gext = c->g;  // extended-domain loop launches cover rows + 2 halo
  gext.rows += 2 * gext.halo;
  c->partials_cap = pp2::mass_partials(gext, 1) + 4;
  if (hipMalloc(&c->pbuf[0], c->partials_cap * sizeof(float)) != hipSuccess ||
      hipMalloc(&c->pbuf[1], c->partials_cap * sizeof(float)) != hipSuccess ||
      hipMalloc(&c->rpartials, c->partials_cap * sizeof(float)) != hipSuccess)
    return fail(set_err(PP2_ENOMEM, "hipMalloc partials"));
  if (hipStreamSynchronize(c->stream) != hipSuccess)
    return fail(set_err(PP2_EHIP, "create sync"));
  *out = c;
  return PP2_OK;
}

int download_planes(pp2_ctx* c, const Planes& P, float* host, const float* divide_by) {
  const size_t n = owned_cells(c) * P.K;
  CHECK(ensure_staging(c, n * sizeof(float)));
  HIPCHK(pp2::launch_pack(c->stream, c->g, P.K, P.v, (float*)c->staging, divide_by));
  HIPCHK(hipMemcpyAsync(host, c->staging, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return PP2_OK;
}

int upload_planes(pp2_ctx* c, Planes& P, const float* host) {
  const size_t n = owned_cells(c) * P.K;
  CHECK(ensure_staging(c, n * sizeof(float)));
  HIPCHK(hipMemcpyAsync(c->staging, host, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
  HIPCHK(pp2::launch_unpack(c->stream, c->g, P.K, (const float*)c->staging, P.v));
  HIPCHK(hipStreamSynchronize(c->stream));
  return PP2_OK;
}

int write_text(const std::string& path, const std::vector<float>& v, int per_line) {
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return set_err(PP2_EIO, "cannot open %s for writing: %s", path.c_str(), strerror(errno));
  for (size_t i = 0; i < v.size(); ++i) {
    fprintf(f, "%15.8f", v[i]);
    if ((i + 1) % per_line == 0) fprintf(f, "\n");
  }
  if (fclose(f) != 0) return set_err(PP2_EIO, "write %s failed", path.c_str());
  return PP2_OK;
}

int read_text(const std::string& path, std::vector<float>& v) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return set_err(PP2_EIO, "cannot open %s: %s", path.c_str(), strerror(errno));
  for (size_t i = 0; i < v.size(); ++i)
    if (fscanf(f, "%f ", &v[i]) != 1) {
      fclose(f);
      return set_err(PP2_EIO, "%s: data dimension is not set properly (element %zu)",
                     path.c_str(), i);
    }
  fclose(f);
  return PP2_OK;
}

int read_actions(const std::string& path, std::vector<uint8_t>& v) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return set_err(PP2_EIO, "cannot open %s: %s", path.c_str(), strerror(errno));
  for (size_t i = 0; i < v.size(); ++i) {
    unsigned a = 0;
    if (fscanf(f, "%u", &a) != 1 || a > 8) {
      fclose(f);
      return set_err(PP2_EIO, "%s: data dimension is not set properly (action %zu)",
                     path.c_str(), i);
    }
    v[i] = (uint8_t)a;
  }
  fclose(f);
  return PP2_OK;
}

std::string join(const char* dir, const char* name) {
  std::string d = dir ? dir : ".";
  if (d.empty()) d = ".";
  if (d.back() != '/') d += '/';
  return d + name;
}

bool coded_active(const pp2_ctx* c) {
  return c->use_coded && c->dict_n > 0 && c->cpt == 4 && (!c->dict_sparse || c->belief_sparse_ok);
}

// +0 <= v < +inf (sign bit clear, not inf or NaN)
static bool finite_nonneg(float v) {
  uint32_t bits;
  std::memcpy(&bits, &v, 4);
  return bits < 0x7f800000u;
}

// Dictionary of the distinct per-cell model tuples (T, C, L) over rows
// [-1, rows]: GPU hash per cell, first-appearance numbering on the host, GPU
// gather of one representative per entry, then a bitwise check of every cell
// against its entry.  More than kDictMax entries or any mismatch (a hash
// collision) leaves dict_n = 0, i.e. the dense kernels.
int build_model_dict(pp2_ctx* c, const Planes* mT, const Planes* mL, const Planes* mR,
                     const Planes* mC);
int build_model_dict(pp2_ctx* c) { return build_model_dict(c, &c->T, &c->L, &c->R, &c->C); }

// (mT .. mC: the dense model over rows [-g.halo, rows + g.halo) -- the
// context's planes, or pp2_model_generate's transient full-halo copy)
int build_model_dict(pp2_ctx* c, const Planes* mT, const Planes* mL, const Planes* mR,
                     const Planes* mC) {
  c->dict_n = 0;
  c->res_e_dict = -1;  // shard_resident_e: recomputed (collectively) on the next run
  ++c->agree_gen;      // ... and agreed again (pp2_loop_run)
  const long long n = (long long)(c->g.rows + 2 * c->g.halo) * c->g.wp;
  break_pipeline(c);
  if (!c->code_alloc) {
    if (hipMalloc(&c->code_alloc, (size_t)(n + 2 * kGuard) * sizeof(uint16_t)) != hipSuccess ||
        hipMalloc(&c->d_dict, (size_t)pp2::kDictMax * pp2::kDictRow * sizeof(float)) != hipSuccess ||
        hipMalloc(&c->d_rows, ((size_t)pp2::kDictMax * pp2::kDictTC + 4) * sizeof(float)) != hipSuccess ||
        hipMalloc(&c->d_dl, (size_t)pp2::kDictMax * 16 * sizeof(float)) != hipSuccess ||
        hipMalloc(&c->d_tu, ((size_t)9 * pp2::kDictMax * 9 + 4) * sizeof(float)) != hipSuccess ||
        hipMalloc(&c->d_rfact, ((size_t)pp2::kResTab + pp2::kDictMax / 4 + 4) * sizeof(float)) !=
            hipSuccess)
      return set_err(PP2_ENOMEM, "hipMalloc model dictionary");
    HIPCHK(hipMemsetAsync(c->code_alloc, 0, (size_t)(n + 2 * kGuard) * sizeof(uint16_t), c->stream));
    c->d_code = c->code_alloc + kGuard + (long long)c->g.halo * c->g.wp;
  }
  uint64_t* d_hash = nullptr;
  int* d_aux = nullptr;
  if (hipMalloc(&d_hash, (size_t)n * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&d_aux, (size_t)(pp2::kDictMax + 1) * sizeof(int)) != hipSuccess) {
    (void)hipFree(d_hash);
    return set_err(PP2_ENOMEM, "hipMalloc dictionary scratch");
  }
  struct Free {
    void* a;
    void* b;
    ~Free() { (void)hipFree(a); (void)hipFree(b); }
  } fr{d_hash, d_aux};
  std::vector<uint64_t> h((size_t)n);
  HIPCHK(pp2::launch_dict_hash(c->stream, c->g, mT->v, mC->v, mR->v, mL->v, d_hash));
  HIPCHK(hipMemcpyAsync(h.data(), d_hash, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  std::vector<uint16_t> code((size_t)n);
  std::vector<int> reps;
  std::unordered_map<uint64_t, int> ids;
  ids.reserve(1024);
  uint64_t last_h = 0;
  int last_id = -1;
  for (long long i = 0; i < n; ++i) {
    if (last_id >= 0 && h[i] == last_h) { code[i] = (uint16_t)last_id; continue; }
    auto it = ids.find(h[i]);
    int id;
    if (it == ids.end()) {
      if ((int)reps.size() >= pp2::kDictMax) return PP2_OK;  // too many patterns: dense path
      id = (int)reps.size();
      ids.emplace(h[i], id);
      reps.push_back((int)i);
    } else {
      id = it->second;
    }
    code[i] = (uint16_t)id;
    last_h = h[i];
    last_id = id;
  }
  const int E = (int)reps.size();
  const int zero = 0;
  HIPCHK(hipMemcpyAsync(c->code_alloc + kGuard, code.data(), (size_t)n * sizeof(uint16_t),
                        hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(d_aux, reps.data(), E * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(d_aux + pp2::kDictMax, &zero, sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIPCHK(pp2::launch_dict_gather(c->stream, c->g, mT->v, mC->v, mR->v, mL->v, d_aux, E,
                                 c->d_dict));
  HIPCHK(pp2::launch_dict_verify(c->stream, c->g, mT->v, mC->v, mR->v, mL->v,
                                 c->code_alloc + kGuard, c->d_dict, d_aux + pp2::kDictMax));
  int bad = 1;
  std::vector<float> dh((size_t)E * pp2::kDictRow);
  HIPCHK(hipMemcpyAsync(&bad, d_aux + pp2::kDictMax, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(dh.data(), c->d_dict, dh.size() * sizeof(float), hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (bad) return PP2_OK;
  bool t_finite = true;
  for (int e = 0; e < E && t_finite; ++e)
    for (int a = 0; a < 9; ++a)
      for (int i = 0; i < 9; ++i)
        if (!std::isfinite(dh[(size_t)e * pp2::kDictRow + a * 10 + i])) t_finite = false;
  // the resident kernels hand over beliefs and values with a tag bit in the
  // sign bit: every T and L entry finite and >= +0 keeps every belief so
  // (values: C >= +0, the sparse rows' precondition below)
  bool tl_nonneg = true;
  for (int e = 0; e < E && tl_nonneg; ++e) {
    for (int a = 0; a < 9; ++a)
      for (int i = 0; i < 9; ++i)
        if (!finite_nonneg(dh[(size_t)e * pp2::kDictRow + a * 10 + i])) tl_nonneg = false;
    for (int z = 0; z < 16; ++z)
      if (!finite_nonneg(dh[(size_t)e * pp2::kDictRow + pp2::kDictL + z])) tl_nonneg = false;
  }
  // LDS-layout rows: sparse when every T entry off the base-kernel support is
  // +0.0 (always so for generated models), else the full [a][T..,C] rows
  // They also drop the T == 0 terms of the Bellman backup, which equals the
  // dense fmaf chain only while every partial cost stays finite and never -0:
  // every dictionary C finite and >= +0 (J then starts at +0 and stays finite
  // below max C / (1 - gamma)), 0 <= gamma < 1.  Otherwise the full rows
  // (no term dropped) keep coded == dense bit for bit.
  const float gam = c->gamma;
  bool sparse = gam >= 0.0f && gam < 1.0f;
  double cmax = 0.0;
  for (int e = 0; e < E && sparse; ++e)
    for (int a = 0; a < 9; ++a) {
      const float cv = dh[(size_t)e * pp2::kDictRow + a * 10 + 9];
      if (!finite_nonneg(cv)) { sparse = false; break; }
      cmax = std::max(cmax, (double)cv);
    }
  if (sparse && cmax / (1.0 - (double)gam) >= 0.5 * (double)FLT_MAX) sparse = false;
  for (int e = 0; e < E && sparse; ++e)
    for (int a = 0; a < 9 && sparse; ++a)
      for (int i = 0; i < 9; ++i) {
        bool in = false;
        for (int j = 0; j < pp2::kSupN[a]; ++j) in |= pp2::kSup[a][j] == i;
        uint32_t bits;
        std::memcpy(&bits, &dh[(size_t)e * pp2::kDictRow + a * 10 + i], 4);
        if (!in && bits != 0) { sparse = false; break; }
      }
  // Factored sweep rows (pp2_internal.h): per action the distinct (gT support
  // quad, C_a) pairs, at most kFactK of them, else the full rows.  The classes
  // are keyed on the raw T quad as well, so that a class also fixes the belief
  // gather's T (the resident loop's QR table; gT = fl(gamma * T) does not
  // determine T in general).
  std::vector<uint32_t> fact_iw((size_t)E * 4, 0u);
  std::vector<float> fact_qt(9 * pp2::kFactK * 4, 0.0f), fact_ct(9 * pp2::kFactK * 4, 0.0f);
  std::vector<float> rfact((size_t)pp2::kResTab + pp2::kDictMax / 4 + 4, 0.0f);
  for (int a = 0; a < 9 && sparse; ++a) {
    std::vector<std::array<uint32_t, 9>> pairs;
    for (int e = 0; e < E && sparse; ++e) {
      const float* src = &dh[(size_t)e * pp2::kDictRow];
      float q[4] = {0.0f, 0.0f, 0.0f, 0.0f}, r[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      for (int j = 0; j < pp2::kSupN[a]; ++j) {
        r[j] = src[a * 10 + pp2::kSup[a][j]];
        q[j] = gam * r[j];
      }
      std::array<uint32_t, 9> key;
      std::memcpy(key.data(), q, 16);
      std::memcpy(&key[4], &src[a * 10 + 9], 4);
      std::memcpy(&key[5], r, 16);
      size_t k = std::find(pairs.begin(), pairs.end(), key) - pairs.begin();
      if (k == pairs.size()) {
        if ((int)k >= pp2::kFactK) { sparse = false; break; }
        pairs.push_back(key);
        std::memcpy(&fact_qt[(a * pp2::kFactK + k) * 4], q, 16);
        std::memcpy(&fact_ct[(a * pp2::kFactK + k) * 4], &key[4], 4);
        std::memcpy(&rfact[pp2::kResQR + (a * pp2::kFactK + k) * 4], r, 16);
      }
      fact_iw[(size_t)e * 4 + a / 4] |= (uint32_t)(16 * k) << (8 * (a % 4));
    }
  }
  // L classes: the distinct 16-vectors (L_0..L_15 bits) of the entries
  bool rfact_ok = sparse;
  {
    std::vector<std::array<uint32_t, 16>> lcls;
    uint8_t* lx = reinterpret_cast<uint8_t*>(&rfact[pp2::kResLX]);
    for (int e = 0; e < E && rfact_ok; ++e) {
      std::array<uint32_t, 16> key;
      std::memcpy(key.data(), &dh[(size_t)e * pp2::kDictRow + pp2::kDictL], 64);
      size_t k = std::find(lcls.begin(), lcls.end(), key) - lcls.begin();
      if (k == lcls.size()) {
        if ((int)k >= pp2::kResLK) { rfact_ok = false; break; }
        lcls.push_back(key);
        for (int z = 0; z < 16; ++z)
          std::memcpy(&rfact[pp2::kResLT + z * pp2::kResLK + k], &key[z], 4);
      }
      lx[e] = (uint8_t)(4 * k);
    }
  }
  const int tw = pp2::tu_width(sparse);
  const int es = (E + 3) & ~3;  // L_z column stride (16-B aligned columns)
  std::vector<float> rows((size_t)pp2::rows_floats(E, sparse) + 4, 0.0f),
      dl((size_t)16 * es, 0.0f);
  if (sparse) {
    std::memcpy(&rows[pp2::kFactQT], fact_qt.data(), fact_qt.size() * sizeof(float));
    std::memcpy(&rows[pp2::kFactCT], fact_ct.data(), fact_ct.size() * sizeof(float));
    std::memcpy(&rows[pp2::kFactIW], fact_iw.data(), fact_iw.size() * sizeof(uint32_t));
  }
  const size_t tstride = ((size_t)E * tw + 3) & ~(size_t)3;  // 16-B aligned per action
  std::vector<float> tu(9 * tstride, 0.0f);
  for (int e = 0; e < E; ++e) {
    const float* src = &dh[(size_t)e * pp2::kDictRow];
    for (int a = 0; a < 9; ++a) {
      // full sweep rows hold fl(gamma * T) (the dense sweep's per-cell product)
      if (!sparse) {
        float* dst = &rows[(size_t)e * pp2::kDictTC];
        for (int i = 0; i < 9; ++i) dst[a * 10 + i] = gam * src[a * 10 + i];
        dst[a * 10 + 9] = src[a * 10 + 9];
      }
      // belief gather: raw T of action a
      float* t = &tu[a * tstride + (size_t)e * tw];
      if (sparse)
        for (int j = 0; j < pp2::kSupN[a]; ++j) t[j] = src[a * 10 + pp2::kSup[a][j]];
      else
        for (int i = 0; i < 9; ++i) t[i] = src[a * 10 + i];
    }
    for (int z = 0; z < 16; ++z) dl[(size_t)z * es + e] = src[pp2::kDictL + z];
  }
  HIPCHK(hipMemcpyAsync(c->d_rows, rows.data(), rows.size() * sizeof(float),
                        hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_dl, dl.data(), dl.size() * sizeof(float), hipMemcpyHostToDevice,
                        c->stream));
  HIPCHK(hipMemcpyAsync(c->d_tu, tu.data(), tu.size() * sizeof(float), hipMemcpyHostToDevice,
                        c->stream));
  HIPCHK(hipMemcpyAsync(c->d_rfact, rfact.data(), rfact.size() * sizeof(float),
                        hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->dict_sparse = sparse;
  c->dict_t_finite = t_finite;
  c->dict_tl_nonneg = tl_nonneg;
  c->dict_rfact = rfact_ok;
  c->dict_n = E;
  return PP2_OK;
}

int mdp_sweep_once(pp2_ctx* c) {
  const int jn = c->jcur ^ 1;
  break_pipeline(c);  // the deep halo rows of J are stale after a sweep
  if (coded_active(c)) {
    HIPCHK(pp2::launch_mdp_sweep_coded(c->stream, c->g, c->gamma, c->d_code, c->d_rows,
                                       c->dict_n, c->dict_sparse, c->J[c->jcur].v.p,
                                       c->J[jn].v.p, c->A));
    c->jcur = jn;
    return PP2_OK;
  }
  HIPCHK(pp2::launch_mdp_sweep(c->stream, c->g, c->cpt, c->gamma, c->T.v, c->C.v,
                               c->J[c->jcur].v.p, c->J[jn].v.p, c->A, c->nt_streams));
  c->jcur = jn;
  return PP2_OK;
}

int fib_sweep_once(pp2_ctx* c) {
  const int fn = c->fcur ^ 1;
  // the support-only kernels drop fmaf(0 * L, alpha, s) terms, which equal s
  // only for finite alphas (uploaded alphas may not be)
  HIPCHK(pp2::launch_fib_sweep(c->stream, c->g, c->gamma, c->T.v, c->L.v, c->R.v,
                               c->fib[c->fcur].v, c->fib[fn].v,
                               c->use_coded && c->dict_n > 0 && c->dict_sparse &&
                                   c->fib_finite));
  c->fcur = fn;
  ++c->fib_version;
  return PP2_OK;
}

// max |cur - snap| over this shard (snap := cur); synchronises.
int absdiff_local_max(pp2_ctx* c, const Planes& cur, const Planes& snap, float* out) {
  int np = 0;
  HIPCHK(pp2::launch_absdiff_max(c->stream, c->g, cur.K, cur.v, snap.v,
                                 c->rpartials, &np));
  std::vector<float> h(np);
  HIPCHK(hipMemcpyAsync(h.data(), c->rpartials, np * sizeof(float),
                        hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float m = 0.0f;
  for (float v : h) m = std::max(m, v);
  *out = m;
  return PP2_OK;
}

}  // namespace pp2rt

using namespace pp2rt;

int pp2rt::ensure_mass(pp2_ctx* c) {
  const int bc = c->bcur;
  if (!c->pending[bc]) return PP2_OK;
  if (c->shift_pending && c->comm) {  // a shard-resident run's mass: rebase as well
    CHECK(shard_post_mass(c, c->nranks, c->rank));
    CHECK(comm_enter(c));
    NCCLCHK(ncclAllReduce(c->d_vec, c->d_vec, pp2::kVecRec * c->nranks, ncclFloat, ncclSum, c->comm,
                          cst(c)));
    CHECK(comm_leave(c));
    return shard_rebase(c, c->nranks, c->rank, 0, c->g.rows);
  }
  HIPCHK(pp2::launch_sum_finalize(c->stream, c->pbuf[bc], c->pcount[bc], c->bsum + bc));
  c->pending[bc] = false;
  return allreduce_mass(c, c->bsum + bc);  // global mass (RCCL shards)
}

void pp2rt::break_pipeline(pp2_ctx* c) { c->kstep = 0; }

// One belief update of planes b_in -> b_out (the context's geometry) divided
// by *mass, its mass partials (mass_partials(g, cpt) of them) into partials:
// on a coded model the coded fused kernel without its sweep (code and b in,
// b' out: 10 B per cell instead of the dense planes' 48), else
// k_belief_update -- the same arithmetic and partial layout either way.
int pp2rt::launch_belief(pp2_ctx* c, const float* b_in, float* b_out, uint8_t u, uint8_t z,
                         const float* mass, float* partials) {
  if (coded_active(c)) {
    HIPCHK(pp2::launch_loop_step_coded(
        c->stream, c->g, c->gamma, c->d_code, c->d_rows,
        c->d_dl + (size_t)z * ((c->dict_n + 3) & ~3),
        c->d_tu + (size_t)u * (((size_t)c->dict_n * pp2::tu_width(c->dict_sparse) + 3) & ~(size_t)3),
        c->dict_n, c->dict_sparse, b_in, b_out, u, nullptr, 0, mass, nullptr, partials, nullptr,
        nullptr, nullptr, 0, c->g.rows, 1.0f));
    return PP2_OK;
  }
  HIPCHK(pp2::launch_belief_update(c->stream, c->g, c->cpt, c->T.v, c->L.v, b_in, b_out, u, z,
                                   mass, partials));
  return PP2_OK;
}

// Belief update alone (k_belief_update), mass finalised eagerly.
int pp2rt::belief_update_impl(pp2_ctx* c, uint8_t u, uint8_t z, bool fuse_with_sweep) {
  if (fuse_with_sweep) return loop_step_fused(c, u, z, true);
  if (u > 8 || z > 15) return set_err(PP2_EINVAL, "action %u / observation %u out of range", u, z);
  CHECK(ensure_mass(c));
  break_pipeline(c);
  const int bn = c->bcur ^ 1;
  const int nparts = pp2::mass_partials(c->g, c->cpt);
  CHECK(launch_belief(c, c->b[c->bcur].v.p, c->b[bn].v.p, u, z, c->bsum + c->bcur, c->pbuf[bn]));
  HIPCHK(pp2::launch_sum_finalize(c->stream, c->pbuf[bn], nparts, c->bsum + bn));
  c->pending[bn] = false;
  CHECK(allreduce_mass(c, c->bsum + bn));
  c->bcur = bn;
  return PP2_OK;
}

// One fused north-star step over the owned rows extended by e rows each side
// (a "view": every plane pointer moves up e rows and the view has rows + 2e
// rows, so the kernels read the halo rows as ordinary neighbours).  Only the
// owned rows [e, e + rows) of the view add to the belief mass and store
// actions.  Reads b[bcur], J[jcur]; writes b[bcur^1], J[jcur^1], A and the new
// belief's mass partials into pbuf[bcur^1].
int pp2rt::loop_launch(pp2_ctx* c, int e, uint8_t u, uint8_t z, const float* in_partials,
                       int in_n, const float* in_sum, float* in_sum_out, int* nparts,
                       float scale) {
  const int bc = c->bcur, bn = bc ^ 1, jc = c->jcur, jn = jc ^ 1;
  Geom g = c->g;
  g.rows += 2 * e;
  g.row0 -= e;
  g.halo -= e;
  const long long wp = g.wp;
  auto up = [e](PlaneSet P) {
    P.p -= (long long)e * P.rs;
    return P;
  };
  const float* b_in = c->b[bc].v.p - e * wp;
  float* b_out = c->b[bn].v.p - e * wp;
  const float* J_in = c->J[jc].v.p - e * wp;
  float* J_out = c->J[jn].v.p - e * wp;
  uint8_t* A = c->A - e * wp;  // only owned rows are stored
  if (coded_active(c)) {
    HIPCHK(pp2::launch_loop_step_coded(c->stream, g, c->gamma, c->d_code - e * wp, c->d_rows,
                                       c->d_dl + (size_t)z * ((c->dict_n + 3) & ~3),
                                       c->d_tu + (size_t)u * (((size_t)c->dict_n * pp2::tu_width(c->dict_sparse) + 3) & ~(size_t)3),
                                       c->dict_n, c->dict_sparse, b_in, b_out, u, in_partials,
                                       in_n, in_sum, in_sum_out, c->pbuf[bn], J_in, J_out, A,
                                       e, e + c->g.rows, scale));
    *nparts = pp2::mass_partials(g, 4);
  } else {
    HIPCHK(pp2::launch_loop_step(c->stream, g, c->cpt, c->gamma, up(c->T.v), up(c->L.v),
                                 up(c->C.v), b_in, b_out, u, z, in_partials, in_n, in_sum,
                                 in_sum_out, c->pbuf[bn], J_in, J_out, A, c->nt_streams, e,
                                 e + c->g.rows, scale));
    *nparts = pp2::mass_partials(g, c->cpt);
  }
  return PP2_OK;
}

// One fused north-star step of an unsharded context (k_loop_step).  The input
// mass is reduced inside the kernel when still pending; the output mass stays
// pending (eager_mass = false) or is finalised right away.
int pp2rt::loop_step_fused(pp2_ctx* c, uint8_t u, uint8_t z, bool eager_mass) {
  if (u > 8 || z > 15) return set_err(PP2_EINVAL, "action %u / observation %u out of range", u, z);
  const int bc = c->bcur, bn = bc ^ 1, jn = c->jcur ^ 1;
  const bool pend = c->pending[bc];
  int nparts = 0;
  CHECK(loop_launch(c, 0, u, z, pend ? c->pbuf[bc] : nullptr, c->pcount[bc], c->bsum + bc,
                    pend ? c->bsum + bc : nullptr, &nparts));
  c->pending[bc] = false;
  c->pcount[bn] = nparts;
  c->pending[bn] = true;
  c->bcur = bn;
  c->jcur = jn;
  if (eager_mass) CHECK(ensure_mass(c));
  return PP2_OK;
}

// One loop step in normalisation blocks.  Steps come in
// blocks of `depth`.  A block starts by finalising the exact (global) mass of
// the current belief; its first step divides by that mass times 2^96 (exact)
// and the others by 1, so the in-kernel reduction of the previous step's
// partials drops out of all but the first step of a block.  RCCL shards also refresh their halo
// rows of b and J `depth` rows deep at the block start (one RCCL group), and
// step i computes a view depth-1-i rows wider than the owned rows per side,
// so nothing crosses ranks until the next block.
static int blocked_loop_step(pp2_ctx* c, uint8_t u, uint8_t z) {
  if (u > 8 || z > 15) return set_err(PP2_EINVAL, "action %u / observation %u out of range", u, z);
  const bool shard = c->comm != nullptr;
  const int depth = shard ? c->kdepth : c->norm_block;
  const int bc = c->bcur, bn = bc ^ 1, jn = c->jcur ^ 1;
  const bool start = c->kstep == 0;
  // unsharded coded context: a pending mass is reduced inside the block-start
  // launch (stored to bsum[bc]) instead of by a separate k_sum_finalize
  const bool fold = start && !shard && c->pending[bc] && coded_active(c);
  if (start && !fold) {
    CHECK(ensure_mass(c));
    if (shard) CHECK(exchange_halos_k(c, {HALO_BELIEF, HALO_VALUE}, depth));
  }
  int nparts = 0;
  CHECK(loop_launch(c, shard ? depth - 1 - c->kstep : 0, u, z, fold ? c->pbuf[bc] : nullptr,
                    fold ? c->pcount[bc] : 0, start && !fold ? c->bsum + bc : nullptr,
                    fold ? c->bsum + bc : nullptr, &nparts, start ? kBlockScale : 1.0f));
  c->pending[bc] = false;
  c->pcount[bn] = nparts;
  c->pending[bn] = true;
  c->bcur = bn;
  c->jcur = jn;
  c->kstep = (c->kstep + 1) % depth;
  return PP2_OK;
}

// Two steps of the current normalisation / halo block in one launch
// (k_loop_pair_coded): the same state transitions as two blocked_loop_step
// calls.  Applies to a context with a sparse coded model when the block has
// two steps left: unsharded, or an RCCL row shard, whose launch covers step
// 2's extended view (depth - 2 - kstep rows per side) and computes step 1
// one row deeper from the halo.
bool pp2rt::pairs_apply(pp2_ctx* c) {
  const int depth = (c->comm || c->group) ? c->kdepth : c->norm_block;
  return c->step_pairs && depth >= 2 && coded_active(c) && c->dict_sparse &&
         pp2::loop_pair_fits(c->g, c->dict_n, true) &&
         (c->step_pairs == 2 || pp2::loop_pair_pays(c->g));
}
static bool can_pair(pp2_ctx* c) {
  const int depth = c->comm ? c->kdepth : c->norm_block;
  return !c->group && c->kstep + 2 <= depth && pairs_apply(c);
}

// One k_loop_pair_coded launch for steps kstep, kstep + 1 of a block.  Row
// shards (e >= 0 rows of view extension: step 2's view, step 1 one row
// deeper from the halo) store actions and mass only for their own rows.
int pp2rt::pair_launch(pp2_ctx* c, int e, bool shard, uint8_t u1, uint8_t z1, uint8_t u2,
                       uint8_t z2, const float* in_partials, int in_n, float* in_sum_out,
                       const float* in_sum, float scale, int* nparts) {
  const int bc = c->bcur, bn = bc ^ 1, jc = c->jcur;
  Geom g = c->g;
  g.rows += 2 * e;
  g.row0 -= e;
  g.halo -= e;
  const long long sh = (long long)e * g.wp;
  const size_t es = (size_t)((c->dict_n + 3) & ~3);
  const size_t ts = ((size_t)c->dict_n * pp2::tu_width(true) + 3) & ~(size_t)3;
  HIPCHK(pp2::launch_loop_pair_coded(
      c->stream, g, c->gamma, c->d_code - sh, c->d_rows, c->d_dl + z1 * es, c->d_dl + z2 * es,
      c->d_tu + u1 * ts, c->d_tu + u2 * ts, c->dict_n, u1, u2, c->b[bc].v.p - sh,
      c->b[bn].v.p - sh, c->J[jc].v.p - sh, c->J[jc ^ 1].v.p - sh, c->A - sh, c->pbuf[bn],
      in_partials, in_n, in_sum_out, in_sum, scale, e, e + c->g.rows, shard));
  *nparts = pp2::mass_partials(g, 4);
  return PP2_OK;
}

// Two steps of the current normalisation / halo block in one launch
// (k_loop_pair_coded): the same state transitions as two blocked_loop_step
// calls.  Applies to a context with a sparse coded model when the block has
// two steps left: unsharded, or an RCCL row shard, whose launch covers step
// 2's extended view (depth - 2 - kstep rows per side) and computes step 1
// one row deeper from the halo.
static int loop_pair(pp2_ctx* c, uint8_t u1, uint8_t z1, uint8_t u2, uint8_t z2) {
  for (int i = 0; i < 2; ++i) {
    const uint8_t u = i ? u2 : u1, z = i ? z2 : z1;
    if (u > 8 || z > 15) return set_err(PP2_EINVAL, "action %u / observation %u out of range", u, z);
  }
  const bool shard = c->comm != nullptr;
  const int depth = shard ? c->kdepth : c->norm_block;
  const int bc = c->bcur, bn = bc ^ 1;
  const bool start = c->kstep == 0;
  // unsharded: a block start with the mass still pending reduces it inside
  // the launch (and stores it to bsum[bc]) instead of a separate
  // k_sum_finalize; shards finalise the global mass and refresh the halo
  const bool fold = start && !shard && c->pending[bc];
  if (start && shard) {
    CHECK(ensure_mass(c));
    CHECK(exchange_halos_k(c, {HALO_BELIEF, HALO_VALUE}, depth));
  }
  int nparts = 0;
  CHECK(pair_launch(c, shard ? depth - 2 - c->kstep : 0, shard, u1, z1, u2, z2,
                    fold ? c->pbuf[bc] : nullptr, fold ? c->pcount[bc] : 0,
                    fold ? c->bsum + bc : nullptr, start && !fold ? c->bsum + bc : nullptr,
                    start ? kBlockScale : 1.0f, &nparts));
  c->pending[bc] = false;
  c->pcount[bn] = nparts;
  c->pending[bn] = true;
  c->bcur = bn;
  c->jcur ^= 1;
  c->kstep = (c->kstep + 2) % depth;
  return PP2_OK;
}

// ---------------------------------------------------------------- resident loop
static void resident_free_buffers(pp2_ctx* c) {
  for (void* p : {(void*)c->res_sync, (void*)c->res_ring, (void*)c->res_xch, (void*)c->res_tmax,
                  (void*)c->res_out})
    if (p) (void)hipFree(p);
  c->res_sync = nullptr;
  c->res_ring = nullptr;
  c->res_xch = nullptr;
  c->res_tmax = nullptr;
  c->res_out = nullptr;
  c->res_ntiles = 0;
}

static void resident_free(pp2_ctx* c) {
  resident_free_buffers(c);
  c->res_ok = false;
  c->res_plan_e = -1;
  c->res_view_e = -1;
  c->sol_ok = false;
  c->sol_plan_e = -1;
}

// The pinned words the kernels write ({sweeps, norm bits, error word}, then
// the journalled launches' error words); kept across plan changes.
static bool resident_host_words(pp2_ctx* c) {
  if (!c->res_host) {
    const size_t b = (pp2_ctx::kResHostChain + pp2_ctx::kResidentChain) * sizeof(unsigned);
    if (hipHostMalloc(&c->res_host, b, hipHostMallocDefault) != hipSuccess) {
      c->res_host = nullptr;
      return false;
    }
    std::memset(c->res_host, 0, b);
  }
  return true;
}

// Sync words, partial ring, exchange rows and solve scratch for plan p (both
// resident kernels share them and the epoch counters; a plan with another
// tile count reallocates and restarts the epochs).  The ring holds the
// partials of the largest view a shard can launch.
static bool resident_buffers(pp2_ctx* c, const pp2::ResidentPlan& p) {
  if (!resident_host_words(c)) return false;
  if (c->res_sync && c->res_ntiles == p.ntiles) return true;
  resident_free_buffers(c);
  Geom gext = c->g;
  gext.rows += 2 * gext.halo;
  const size_t sync_b = (size_t)pp2::kResidentSyncWords * sizeof(unsigned);
  const size_t ring_b = (size_t)pp2::kResidentRing * pp2::mass_partials(gext, 4) * sizeof(float);
  // two exchange regions: the loop kernel's (b and J granules) and the
  // sweep kernel's (J alone), each with its own slot-use counts, so that a
  // granule's stale content is always the previous use of its own slot
  const size_t xch_b = 2 * pp2::resident_xch_floats(c->g, p.ntiles) * sizeof(float);
  const size_t tmax_b = (size_t)2 * p.ntiles * sizeof(float);
  if (hipMalloc(&c->res_sync, sync_b) != hipSuccess || hipMalloc(&c->res_ring, ring_b) != hipSuccess ||
      hipMalloc(&c->res_xch, xch_b) != hipSuccess || hipMalloc(&c->res_tmax, tmax_b) != hipSuccess ||
      hipMalloc(&c->res_out, 4 * sizeof(int)) != hipSuccess ||
      hipMemsetAsync(c->res_sync, 0, sync_b, c->stream) != hipSuccess ||
      hipMemsetAsync(c->res_ring, 0, ring_b, c->stream) != hipSuccess ||
      hipMemsetAsync(c->res_xch, 0, xch_b, c->stream) != hipSuccess) {
    (void)hipGetLastError();
    resident_free_buffers(c);
    return false;
  }
  c->res_ntiles = p.ntiles;
  c->res_loop_tc = 0;  // fresh (zero) exchange rows: any tile layout may start
  c->res_slot[0] = c->res_slot[1] = c->res_slot[2] = c->res_slot[3] = 0;
  c->res_arrive = 0;
  return true;
}

// CUs the resident plans may use (PP2_TUNE_RESIDENT_CUS narrows it: tests of
// the fall-back-before-launch path).
static int resident_cus(const pp2_ctx* c) {
  return c->res_cus > 0 ? std::min(c->res_cus, c->ncus) : c->ncus;
}

// A shard's view: its owned rows extended by e rows per side.
static Geom view_geom(const pp2_ctx* c, int e) {
  Geom g = c->g;
  g.rows += 2 * e;
  g.row0 -= e;
  g.halo -= e;
  return g;
}

// The model conditions of the resident kernels: a sparse coded model with
// finite T (the kernel's zero-padded edges multiply T by +0) and the class
// tables.
static bool resident_model_ok(const pp2_ctx* c) {
  return c->resident && coded_active(c) && c->dict_sparse && c->dict_t_finite &&
         c->dict_tl_nonneg && c->dict_rfact &&
         c->norm_block <= pp2::kResidentRing - 2 && c->ncus > 0;
}

// Whether a loop plan exists for view extension e (0: an unsharded grid),
// with no allocation: the eligibility query of pp2_loop_steps_per_launch.
static bool resident_plan_for(pp2_ctx* c, int e) {
  if (c->res_plan_e != c->dict_n || c->res_view_e != e) {
    c->res_plan_e = c->dict_n;
    c->res_view_e = e;
    c->res_ok = false;
    pp2::ResidentPlan p;
    if (!pp2::resident_plan(view_geom(c, e), c->dict_n, resident_cus(c), &p, c->res_tc_pref,
                            e > 0 && e % 4 == 0 && c->g.rows % 4 == 0))
      return false;
    c->res_plan = p;
    c->res_ok = true;
  }
  return c->res_ok;
}

// Whether pp2_loop_run takes the tile-resident loop (pp2_resident.hip) on an
// unsharded context, allocating the plan's buffers.
static bool resident_ready(pp2_ctx* c) {
  if (c->comm || c->group || !resident_model_ok(c)) return false;
  return resident_plan_for(c, 0) && resident_buffers(c, c->res_plan);
}

// Whether pp2_mdp_solve runs as resident sweeps (k_sweep_resident): the
// resident loop's conditions minus the belief's, and a plan for J alone.
static bool solve_plan_ok(pp2_ctx* c) {
  if (!c->resident || c->comm || c->group || !coded_active(c) || !c->dict_sparse ||
      c->ncus <= 0)  // (values >= +0 finite: the sparse rows' precondition)
    return false;
  if (c->sol_plan_e != c->dict_n) {
    c->sol_plan_e = c->dict_n;
    c->sol_ok = false;
    pp2::ResidentPlan p;
    if (!pp2::solve_plan(c->g, c->dict_n, resident_cus(c), &p)) return false;
    c->sol_plan = p;
    c->sol_ok = true;
  }
  return c->sol_ok;
}
static bool solve_ready(pp2_ctx* c) { return solve_plan_ok(c) && resident_buffers(c, c->sol_plan); }

// Resident launches of all contexts of this process on one device run one at
// a time: a launch on another stream than the previous one is ordered after
// everything queued so far on that stream (an event recorded there at this
// point), so two contexts never hold part of the CUs each and wait for the
// rest.  No event per launch: two per launch cost ~8 us of GPU time each
// (profiles/r03/resident_launch_events.txt).  (Work of other processes can
// still delay tiles: the kernels' bounded waits and resident_settle cover it.)
struct ResidentGate {
  std::mutex m;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;  // stream of the last resident launch, null: none pending
};
static ResidentGate& resident_gate(int device) {
  static ResidentGate gates[64];
  return gates[device & 63];
}

template <class F>
static int gated_launch(pp2_ctx* c, F launch) {
  ResidentGate& g = resident_gate(c->device);
  std::lock_guard<std::mutex> lk(g.m);
  if (g.last && g.last != c->stream) {
    if (!g.ev) HIPCHK(hipEventCreateWithFlags(&g.ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(g.ev, g.last));
    HIPCHK(hipStreamWaitEvent(c->stream, g.ev, 0));
  }
  HIPCHK(launch());
  g.last = c->stream;
  return PP2_OK;
}

// A stream leaves the gate (the context is destroyed or moves to another
// stream): drained first, so nothing queued on it needs ordering any more.
static void resident_gate_forget(pp2_ctx* c, hipStream_t s) {
  ResidentGate& g = resident_gate(c->device);
  std::lock_guard<std::mutex> lk(g.m);
  if (g.last == s) {
    (void)hipStreamSynchronize(s);
    g.last = nullptr;
  }
}

// Exchange-slot uses of a launch: the prologue's publish into slot 1, then
// one per published step t (slot t & 1) for t < published.  region 0: the
// loop kernel's exchange rows, 1: the sweep kernel's.
static void count_slot_uses(pp2_ctx* c, int region, int published) {
  c->res_slot[2 * region + 1] += 1u + (unsigned)(published / 2);
  c->res_slot[2 * region] += (unsigned)((published + 1) / 2);
}
static float* sweep_xch(pp2_ctx* c) {
  return c->res_xch + pp2::resident_xch_floats(c->g, c->res_ntiles);
}

// Journal a resident launch about to be enqueued; returns its pinned error
// word (the caller settles first when kResidentChain launches are queued).
static unsigned* journal(pp2_ctx* c, int kind, int n, const uint8_t* us, const uint8_t* zs) {
  c->journal.emplace_back();
  auto& j = c->journal.back();
  j.kind = kind;
  j.n = n;
  j.bcur = c->bcur;
  j.jcur = c->jcur;
  j.kstep = c->kstep;
  for (int i = 0; i < 2; ++i) {
    j.pending[i] = c->pending[i];
    j.pcount[i] = c->pcount[i];
  }
  if (us) j.us.assign(us, us + n);
  if (zs) j.zs.assign(zs, zs + n);
  unsigned* eh = c->res_host + pp2_ctx::kResHostChain + (c->journal.size() - 1);
  *eh = 0u;
  return eh;
}


// Verify the journalled resident launches before anything reads their
// outputs (every C-ABI entry point calls this through check_ctx, except the
// resident runs that queue behind them).  If a launch's waits timed out (a
// tile never got a CU), its outputs are garbage but its inputs are intact
// (b, J went to the other buffers), and the launches queued behind it exited
// without a store: restore the state before the failed launch and re-run it
// and every later one with the launch-per-step kernels, which give the same
// bits; the context stays on them (PP2_TUNE_RESIDENT 1 re-enables the
// resident kernels).  A row shard cannot re-run alone (its RCCL partners
// have moved on): it reports the loss instead, and its belief and values
// stay unusable until pp2_belief_set / pp2_mdp_reset.
int pp2rt::resident_settle(pp2_ctx* c) {
  if (c->journal.empty()) return PP2_OK;
  DeviceGuard dg(c->device);
  std::vector<pp2_ctx::ResidentJournal> q;
  q.swap(c->journal);
  HIPCHK(hipStreamSynchronize(c->stream));
  volatile unsigned* eh = c->res_host + pp2_ctx::kResHostChain;
  size_t bad = q.size();
  for (size_t i = 0; i < q.size(); ++i) {
    if (eh[i] != 0u && bad == q.size()) bad = i;
    eh[i] = 0u;
  }
  if (bad == q.size()) return PP2_OK;
  ++c->res_fallbacks;
  resident_free(c);  // the failed run's epochs and counters are inconsistent
  c->resident = 0;
  const auto& j = q[bad];
  c->bcur = j.bcur;
  c->jcur = j.jcur;
  c->kstep = j.kstep;
  for (int i = 0; i < 2; ++i) {
    c->pending[i] = j.pending[i];
    c->pcount[i] = j.pcount[i];
  }
  for (size_t i = bad; i < q.size(); ++i) {
    const auto& e = q[i];
    if (e.kind == 1) {
      CHECK(loop_run_launches(c, e.n, e.us.data(), e.zs.data()));
    } else if (e.kind == 2) {
      for (int k = 0; k < e.n; ++k) CHECK(mdp_sweep_once(c));
    } else {
      c->lost_belief = c->lost_values = true;
      return set_err(PP2_EHIP, "resident shard run: a workgroup wait timed out (the GPU was "
                     "shared with another process?); this shard's belief and values are lost -- "
                     "set them again (pp2_belief_set, pp2_mdp_reset); the context now uses "
                     "per-step launches");
    }
  }
  return PP2_OK;
}

// Whether a resident loop run (kind 1) or sweeps (kind 2) can be enqueued
// behind the unverified launches without touching the resident buffers
// (no plan change, no allocation): the chained entry points' test.
static bool resident_chainable(pp2_ctx* c, int kind) {
  if (c->journal.empty() || (int)c->journal.size() >= pp2_ctx::kResidentChain || c->comm ||
      c->group || !c->model_ready || !c->res_sync)
    return false;
  if (kind == 1)
    return resident_model_ok(c) && resident_plan_for(c, 0) && c->res_ntiles == c->res_plan.ntiles;
  return solve_plan_ok(c) && c->res_ntiles == c->sol_plan.ntiles;
}

// pp2_mdp_solve's driver (reset, then blocks of 100 sweeps until the
// inf-norm change of a block is <= max_cost * 1e-3 or max_sweeps is reached)
// on resident sweeps: <= 20 blocks per launch, the decision taken in-kernel;
// one host read of {sweeps, norm} per launch.  Returns 1 (not an error) when
// a launch timed out: the caller solves again on per-sweep launches.
static int solve_resident(pp2_ctx* c, int max_sweeps, double thresh, int* sweeps,
                          double* final_norm) {
  const pp2::ResidentPlan& p = c->sol_plan;
  const int cap_total = max_sweeps > 0 ? (max_sweeps + pp2::kSolveBlock - 1) / pp2::kSolveBlock : 0;
  int blocks = 0, total = 0;
  float norm = 0.0f;
  for (;;) {
    pp2::SweepRun a{};
    a.g = c->g;
    a.gamma = c->gamma;
    a.E = c->dict_n;
    a.code = c->d_code;
    a.rows = c->d_rows;
    a.j_in = c->J[c->jcur].v.p;
    a.j_out = c->J[c->jcur ^ 1].v.p;
    a.snap = c->Jsnap.v.p;
    a.A = c->A;
    a.xch = sweep_xch(c);
    a.sync = c->res_sync;
    a.err_host = c->res_host + 2;
    a.tile_max = c->res_tmax;
    a.res = c->res_out;
    a.slot_use[0] = c->res_slot[2];
    a.slot_use[1] = c->res_slot[3];
    a.arrive_base = c->res_arrive;
    a.rt = p.rt;
    a.ntiles = p.ntiles;
    a.max_blocks = 20;
    a.cap_blocks = cap_total ? cap_total - blocks : 0;
    a.thresh = thresh;
    a.nsweeps = 0;
    a.stall_tile = c->res_stall_tile;
    CHECK(gated_launch(c, [&] { return pp2::launch_sweep_resident(c->stream, p, a); }));
    ++c->sol_launches;
    HIPCHK(hipMemcpyAsync(c->res_host, c->res_out, 2 * sizeof(int), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));  // one sync for the result and the error word
    volatile unsigned* eh = c->res_host + 2;
    if (*eh != 0u) {
      *eh = 0u;
      ++c->res_fallbacks;
      resident_free(c);
      c->resident = 0;
      return 1;
    }
    int res[2];
    std::memcpy(res, c->res_host, sizeof(res));
    const int done = res[0];
    if (done <= 0 || done % pp2::kSolveBlock != 0)
      return set_err(PP2_EHIP, "resident MDP solve returned %d sweeps", done);
    std::memcpy(&norm, &res[1], sizeof(float));
    total += done;
    blocks += done / pp2::kSolveBlock;
    count_slot_uses(c, 1, done);  // every sweep publishes
    c->res_arrive += (unsigned)(done / pp2::kSolveBlock * p.ntiles);
    c->jcur ^= 1;
    if (cap_total && blocks >= cap_total) break;
    if (!((double)norm > thresh)) break;
  }
  if (sweeps) *sweeps = total;
  if (final_norm) *final_norm = (double)norm;
  return PP2_OK;
}

// The fields of a loop run shared by the unsharded and shard launches.  A
// plan with another tile layout than the previous loop launch (same tile
// count: whole-row vs 2-D tiles) finds granules of the old layout in its
// exchange rows, whose tag bits could match: the loop region is cleared and
// its slot uses restart, as in freshly allocated buffers.
static int run_common(pp2_ctx* c, const pp2::ResidentPlan& p, pp2::ResidentRun& a) {
  const int layout = p.tc + (p.tr ? 16 : 0);  // (transposed tiles: another granule layout)
  if (c->res_loop_tc != 0 && c->res_loop_tc != layout) {
    HIPCHK(hipMemsetAsync(c->res_xch, 0,
                          pp2::resident_xch_floats(c->g, c->res_ntiles) * sizeof(float), c->stream));
    c->res_slot[0] = c->res_slot[1] = 0;
  }
  c->res_loop_tc = layout;
  a.gamma = c->gamma;
  a.E = c->dict_n;
  a.rows = c->d_rows;
  a.rfact = c->d_rfact;
  a.xch = c->res_xch;
  a.rt = p.rt;
  a.tc = p.tc;
  a.ntiles = p.ntiles;
  a.ring = c->res_ring;
  a.sync = c->res_sync;
  a.slot_use[0] = c->res_slot[0];
  a.slot_use[1] = c->res_slot[1];
  a.arrive_base = c->res_arrive;
  a.stall_tile = c->res_stall_tile;
  return PP2_OK;
}

// n loop steps in ceil(n / kResidentMaxSteps) resident launches, with the
// state transitions of n blocked_loop_step calls (the pending mass of the
// final belief, kstep) -- except that b and J end in the other ping-pong
// buffer of their inputs whatever the parity of n.
static int loop_resident(pp2_ctx* c, int n, const uint8_t* us, const uint8_t* zs) {
  for (int i = 0; i < n; ++i)
    if (us[i] > 8 || zs[i] > 15)
      return set_err(PP2_EINVAL, "action %u / observation %u out of range", us[i], zs[i]);
  const int depth = c->norm_block;
  const int nparts = pp2::mass_partials(c->g, 4);
  std::unique_ptr<pp2::ResidentRun> run(new pp2::ResidentRun());
  pp2::ResidentRun& a = *run;
  for (int i = 0; i < n;) {
    if ((int)c->journal.size() >= pp2_ctx::kResidentChain) {
      CHECK(resident_settle(c));
      if (!resident_ready(c)) return loop_run_launches(c, n - i, us + i, zs + i);
    }
    const pp2::ResidentPlan& p = c->res_plan;
    const int m = std::min(n - i, pp2::kResidentMaxSteps);
    const int bc = c->bcur, jc = c->jcur;
    const bool start0 = c->kstep == 0;
    const bool fold = start0 && c->pending[bc];
    CHECK(run_common(c, p, a));
    a.g = c->g;
    a.code = c->d_code;
    a.b_in = c->b[bc].v.p;
    a.j_in = c->J[jc].v.p;
    a.b_out = c->b[bc ^ 1].v.p;
    a.j_out = c->J[jc ^ 1].v.p;
    a.A = c->A;
    a.n = m;
    a.kstep0 = c->kstep;
    a.depth = depth;
    a.nparts = nparts;
    a.own0 = 0;
    a.own1 = c->g.rows;
    a.shard = 0;
    a.bscale = depth == 1 ? 1.0f : kBlockScale;
    a.in_partials = fold ? c->pbuf[bc] : nullptr;
    a.in_n = c->pcount[bc];
    a.in_sum_out = fold ? c->bsum + bc : nullptr;
    a.in_sum = start0 && !fold ? c->bsum + bc : nullptr;
    a.out_partials = c->pbuf[bc ^ 1];
    a.scale_out = nullptr;
    for (int k = 0; k < m; ++k) a.uz[k] = (uint8_t)(us[i + k] | (zs[i + k] << 4));
    a.err_host = journal(c, 1, m, us + i, zs + i);
    CHECK(gated_launch(c, [&] { return pp2::launch_loop_resident(c->stream, p, a); }));
    ++c->res_launches;
    int arrivals = 0;
    for (int t = 0; t + 1 < m; ++t) arrivals += (c->kstep + t + 1) % depth == 0;
    count_slot_uses(c, 0, m - 1);  // the last step publishes nothing
    c->res_arrive += (unsigned)(arrivals * p.ntiles);
    c->pending[bc] = false;
    c->pending[bc ^ 1] = true;
    c->pcount[bc ^ 1] = nparts;
    c->bcur = bc ^ 1;
    c->jcur = jc ^ 1;
    c->kstep = (c->kstep + m) % depth;
    i += m;
  }
  return PP2_OK;
}

// pp2_mdp_sweep(n) on resident sweeps: n sweeps in one launch (no checks),
// the J of the last sweep in J[jcur ^ 1], A of the last sweep.
static int sweeps_resident(pp2_ctx* c, int n) {
  if ((int)c->journal.size() >= pp2_ctx::kResidentChain) {
    CHECK(resident_settle(c));
    if (!solve_ready(c)) {
      for (int i = 0; i < n; ++i) CHECK(mdp_sweep_once(c));
      return PP2_OK;
    }
  }
  const pp2::ResidentPlan& p = c->sol_plan;
  pp2::SweepRun a{};
  a.g = c->g;
  a.gamma = c->gamma;
  a.E = c->dict_n;
  a.code = c->d_code;
  a.rows = c->d_rows;
  a.j_in = c->J[c->jcur].v.p;
  a.j_out = c->J[c->jcur ^ 1].v.p;
  a.snap = c->Jsnap.v.p;  // read, not written (no checks)
  a.A = c->A;
  a.xch = sweep_xch(c);
  a.sync = c->res_sync;
  a.tile_max = c->res_tmax;
  a.res = c->res_out;
  a.slot_use[0] = c->res_slot[2];
  a.slot_use[1] = c->res_slot[3];
  a.arrive_base = c->res_arrive;
  a.rt = p.rt;
  a.ntiles = p.ntiles;
  a.max_blocks = 1;
  a.nsweeps = n;
  a.stall_tile = c->res_stall_tile;
  a.err_host = journal(c, 2, n, nullptr, nullptr);
  CHECK(gated_launch(c, [&] { return pp2::launch_sweep_resident(c->stream, p, a); }));
  ++c->sol_launches;
  count_slot_uses(c, 1, n);
  c->jcur ^= 1;
  return PP2_OK;
}

// ------------------------------------------------ row shards on the resident loop
// DESIGN.md §6.  A pp2_loop_run of n steps on a row shard runs in blocks of
// m <= the resident halo depth: each block refreshes m halo rows of b and J
// from the neighbours, then ONE resident launch runs the m steps on the view
// extended by m rows per side.  Its first step divides by the global mass
// (times 2^96); its later block starts scale by powers of two from the
// shard's own mass; the next exchange rebases every shard to a common power
// of two, where the global mass is known again.  The call ends rebased, with
// the global mass finalised (the state of the per-step paths), and the halo
// pipeline restarted.

// Deepest resident halo this shard may use: the halo allocation, the smallest
// shard (rows come from the immediate neighbour), PP2_TUNE_RESIDENT_HALO.
static int shard_resident_depth(const pp2_ctx* c) {
  int k = std::min(c->g.halo, std::max(1, c->min_shard_rows));
  if (c->res_halo > 0) k = std::min(k, c->res_halo);
  return k;
}

// The view extension e of this shard's resident runs (0: none fits): the
// deepest halo whose view still has a co-resident plan.  Every launch of a
// run uses this view and exchanges e halo rows, whatever its step count m <=
// e (the rows beyond m go stale without reaching the owned rows), so the plan
// and its buffers stay fixed across calls.
int pp2rt::shard_resident_e(pp2_ctx* c) {
  if (!(c->comm || c->group) || !resident_model_ok(c)) return 0;
  if (c->res_e_dict == c->dict_n) return c->res_e;
  int e = shard_resident_depth(c);
  pp2::ResidentPlan p;
  auto plan = [&](int ee, pp2::ResidentPlan* q) {
    return pp2::resident_plan(view_geom(c, ee), c->dict_n, resident_cus(c), q, c->res_tc_pref,
                              ee % 4 == 0 && c->g.rows % 4 == 0);
  };
  for (; e >= 1; --e)
    if (plan(e, &p)) break;
  // Without a requested halo: half the depth while that gives tiles of fewer
  // rows (fewer waves per CU).  A step of the resident kernel is the tile's
  // compute chain, which shrinks with the waves per CU (2048^2 / 8 ranks: e =
  // 128's 4 x 1024 tiles 4.90 us per step, e = 64's 3 x 1024 tiles 4.46),
  // while the halved depth adds one RCCL round per e steps (<= 0.5 us per
  // step at e >= 64 and 30 us per round; profiles/r04/ab_sweep_ao.txt).
  if (e > 0 && c->res_halo == 0 && c->res_tc_pref != 3) {
    pp2::ResidentPlan q;
    while (e / 2 >= 64 && plan(e / 2, &q) && q.rt < p.rt) {
      e /= 2;
      p = q;
    }
  }
  c->res_e_dict = c->dict_n;
  c->res_e = e;
  return e;
}

bool pp2rt::shard_resident_ready(pp2_ctx* c, int e) {
  if (e < 1 || e > shard_resident_e(c)) return false;
  if (!resident_plan_for(c, e) || !resident_buffers(c, c->res_plan)) return false;
  if (!c->d_shift) {
    if (hipMalloc(&c->d_shift, sizeof(int)) != hipSuccess) {
      c->d_shift = nullptr;
      return false;
    }
  }
  if (!c->d_vec) {
    const int nr = c->group ? c->group_size : c->nranks;
    if (hipMalloc(&c->d_vec, (size_t)pp2::kVecRec * nr * sizeof(float)) != hipSuccess) {
      c->d_vec = nullptr;
      return false;
    }
  }
  return true;
}

// {mass, shift} of this shard's pending belief into its slot of d_vec.
int pp2rt::shard_post_mass(pp2_ctx* c, int nranks, int rank) {
  const int bc = c->bcur;
  // an RCCL shard's sticky resident error word rides the all-reduce, so a run
  // lost on any rank is marked lost on every rank (shard_rebase)
  const unsigned* err = c->comm && c->res_sync ? c->res_sync + pp2::kResidentSyncErr : nullptr;
  HIPCHK(pp2::launch_shard_mass_vec(c->stream, c->pbuf[bc], c->pcount[bc],
                                    c->shift_pending ? c->d_shift : nullptr, c->d_vec, nranks,
                                    rank, err));
  return PP2_OK;
}

// Rebase rows [r0, r1) of the current belief after the vector is complete and
// take the global mass: the state of a finalised, common-scale belief.
int pp2rt::shard_rebase(pp2_ctx* c, int nranks, int rank, int r0, int r1) {
  const int bc = c->bcur;
  // the error slot marks this rank's latest journalled launch as failed
  // (resident_settle then reports the loss, as on the rank that timed out)
  unsigned* eh = c->comm && c->res_sync && !c->journal.empty()
                     ? c->res_host + pp2_ctx::kResHostChain + (c->journal.size() - 1)
                     : nullptr;
  HIPCHK(pp2::launch_shard_rebase(c->stream, c->d_vec, nranks, rank, c->b[bc].v.p, c->g.wp, r0,
                                  r1, c->g.rows, c->bsum + bc, eh));
  c->pending[bc] = false;
  c->shift_pending = false;
  return PP2_OK;
}

// One resident launch of m <= e steps on the view extended by e rows (the
// halo rows e deep and the global mass are in place).
int pp2rt::shard_resident_launch(pp2_ctx* c, int e, int m, const uint8_t* us, const uint8_t* zs) {
  if ((int)c->journal.size() >= pp2_ctx::kResidentChain) CHECK(resident_settle(c));
  if (m < 1 || m > e || !shard_resident_ready(c, e))
    return set_err(PP2_ESTATE, "shard resident plan lost");
  const pp2::ResidentPlan& p = c->res_plan;
  // (transposed tiles: the kernel's grid is the view transposed, HBM is not)
  const Geom gv = p.tr ? pp2::transposed_geom(view_geom(c, e)) : view_geom(c, e);
  const long long sh = (long long)e * c->g.wp;
  const int bc = c->bcur, jc = c->jcur;
  const int nparts = pp2::mass_partials(gv, 4);
  const int depth = std::min(c->norm_block, pp2::kResidentRing - 2);
  std::unique_ptr<pp2::ResidentRun> run(new pp2::ResidentRun());
  pp2::ResidentRun& a = *run;
  CHECK(run_common(c, p, a));
  a.g = gv;
  a.code = c->d_code - sh;
  a.b_in = c->b[bc].v.p - sh;
  a.j_in = c->J[jc].v.p - sh;
  a.b_out = c->b[bc ^ 1].v.p - sh;
  a.j_out = c->J[jc ^ 1].v.p - sh;
  a.A = c->A - sh;  // only owned rows are stored
  a.n = m;
  a.kstep0 = 0;
  a.depth = depth;
  a.nparts = nparts;
  a.own0 = e;
  a.own1 = e + c->g.rows;
  a.ows = c->g.wp;
  a.shard = c->shard_lag ? 2 : 1;
  a.red_lds = a.shard == 2 && nparts <= pp2::kResRedFloats &&
              p.lds + (size_t)pp2::kResRedFloats * sizeof(float) <= pp2::kDictLdsMaxBytes;
  a.bscale = kBlockScale;
  a.in_partials = nullptr;
  a.in_n = 0;
  a.in_sum_out = nullptr;
  a.in_sum = c->bsum + bc;
  a.out_partials = c->pbuf[bc ^ 1];
  a.scale_out = c->d_shift;
  for (int k = 0; k < m; ++k) a.uz[k] = (uint8_t)(us[k] | (zs[k] << 4));
  a.err_host = journal(c, 3, m, nullptr, nullptr);
  CHECK(gated_launch(c, [&] { return pp2::launch_loop_resident(c->stream, p, a); }));
  ++c->res_launches;
  int arrivals = 0;
  for (int t = 0; t + 1 < m; ++t) arrivals += (t + 1) % depth == 0;
  count_slot_uses(c, 0, m - 1);
  c->res_arrive += (unsigned)(arrivals * p.ntiles);
  c->pending[bc] = false;
  c->pending[bc ^ 1] = true;
  c->pcount[bc ^ 1] = nparts;
  c->shift_pending = true;
  c->bcur = bc ^ 1;
  c->jcur = jc ^ 1;
  c->kstep = 0;
  return PP2_OK;
}

// The RCCL shard's resident run: blocks of m <= e steps, each after ONE RCCL
// round -- the exchange of e halo rows, grouped (with a pending mass) with the
// point-to-point {mass, shift, lost} records, then the rebase -- and the
// closing all-reduce of the records and rebase: n / e + 1 rounds per call.
static int shard_allreduce_vec(pp2_ctx* c) {
  CHECK(comm_enter(c));
  NCCLCHK(ncclAllReduce(c->d_vec, c->d_vec, pp2::kVecRec * c->nranks, ncclFloat, ncclSum, c->comm,
                        cst(c)));
  return comm_leave(c);
}

static int shard_loop_resident(pp2_ctx* c, int e, int n, const uint8_t* us, const uint8_t* zs) {
  for (int i = 0; i < n; ++i)
    if (us[i] > 8 || zs[i] > 15)
      return set_err(PP2_EINVAL, "action %u / observation %u out of range", us[i], zs[i]);
  break_pipeline(c);
  // (no settle between blocks: a shard cannot re-run alone, and a timed-out
  // block leaves the sticky error words set for the settle after the call)
  for (int i = 0; i < n;) {
    const int m = std::min(e, n - i);
    if (c->pending[c->bcur]) {
      // one RCCL round: the records and the (unrebased) halo rows together
      CHECK(shard_post_mass(c, c->nranks, c->rank));
      CHECK(exchange_halos_k(c, {HALO_BELIEF, HALO_VALUE}, e, true));
      CHECK(shard_rebase(c, c->nranks, c->rank, -e, c->g.rows + e));
    } else {
      CHECK(exchange_halos_k(c, {HALO_BELIEF, HALO_VALUE}, e));
    }
    CHECK(shard_resident_launch(c, e, m, us + i, zs + i));
    i += m;
  }
  // close: the global mass at a common scale, the state of the per-step paths
  CHECK(shard_post_mass(c, c->nranks, c->rank));
  CHECK(shard_allreduce_vec(c));
  CHECK(shard_rebase(c, c->nranks, c->rank, 0, c->g.rows));
  break_pipeline(c);
  return PP2_OK;
}

static int loop_step_impl(pp2_ctx* c, uint8_t u, uint8_t z) {
  if (c->comm || c->norm_block > 1) return blocked_loop_step(c, u, z);  // RCCL shard or blocks
  return loop_step_fused(c, u, z, false);
}

// The launch-per-step (or per-pair) body of pp2_loop_run; also re-runs a
// resident launch that timed out (resident_settle).
int pp2rt::loop_run_launches(pp2_ctx* c, int n, const uint8_t* us, const uint8_t* zs) {
  for (int i = 0; i < n;) {
    if (i + 1 < n && can_pair(c)) {
      CHECK(loop_pair(c, us[i], zs[i], us[i + 1], zs[i + 1]));
      i += 2;
    } else {
      CHECK(loop_step_impl(c, us[i], zs[i]));
      ++i;
    }
  }
  return PP2_OK;
}

// =========================================================================== C ABI
extern "C" {

int pp2_abi_version(void) { return PP2_ABI_VERSION; }

const char* pp2_status_string(int s) {
  switch (s) {
    case PP2_OK: return "ok";
    case PP2_EINVAL: return "invalid argument";
    case PP2_EHIP: return "HIP error";
    case PP2_EIO: return "I/O error";
    case PP2_ENOMEM: return "out of memory";
    case PP2_ESTATE: return "invalid state";
    case PP2_ERCCL: return "RCCL error";
    default: return "unknown status";
  }
}

const char* pp2_last_error(void) { return g_last_error.c_str(); }

// Diagnostic (tests/test_gpu_shards.py, not part of pp2.h): the device bytes
// a context's grid-sized buffers hold -- every plane set, the code plane,
// the actions and the map window (the fixed-size buffers aside).
int pp2_debug_context_bytes(pp2_ctx* c, unsigned long long* bytes) {
  if (!c || !bytes) return set_err(PP2_EINVAL, "null argument");
  unsigned long long b = 0;
  for (const Planes* P : {&c->T, &c->L, &c->R, &c->C, &c->b[0], &c->b[1], &c->J[0], &c->J[1],
                          &c->Jsnap, &c->fib[0], &c->fib[1], &c->fibsnap})
    b += (unsigned long long)P->floats * sizeof(float);
  if (c->code_alloc)
    b += ((unsigned long long)(c->g.rows + 2 * c->g.halo) * c->g.wp + 2 * kGuard) * sizeof(uint16_t);
  b += (unsigned long long)c->g.rows * c->g.wp + 16;  // actions
  const long long mlo = std::max(0LL, (long long)c->g.row0 - c->g.halo - 1);
  const long long mhi =
      std::min((long long)c->g.grows, (long long)c->g.row0 + c->g.rows + c->g.halo + 1);
  b += (unsigned long long)(mhi - mlo) * c->g.width;
  *bytes = b;
  return PP2_OK;
}

int pp2_comm_rounds(pp2_ctx* c, int* rounds, long long* untimed, float* round_us,
                    int max_rounds) {
  CHECK(check_ctx_settled(c));
  if (!rounds) return set_err(PP2_EINVAL, "rounds is null");
  if (max_rounds > 0 && !round_us) return set_err(PP2_EINVAL, "round_us is null");
  DeviceGuard dg(c->device);
  if (c->comm_stream) HIPCHK(hipStreamSynchronize(c->comm_stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *rounds = c->comm_nev;
  if (untimed) *untimed = c->comm_dropped;
  for (int i = 0; i < c->comm_nev && i < max_rounds; ++i)
    HIPCHK(hipEventElapsedTime(&round_us[i], c->comm_ev[2 * i], c->comm_ev[2 * i + 1]));
  for (int i = 0; i < c->comm_nev && i < max_rounds; ++i) round_us[i] *= 1e3f;
  c->comm_nev = 0;
  c->comm_dropped = 0;
  return PP2_OK;
}

int pp2_device_count(int* count) {
  if (!count) return set_err(PP2_EINVAL, "count is null");
  *count = 0;
  HIPCHK(hipGetDeviceCount(count));
  return PP2_OK;
}

int pp2_create(pp2_ctx** out, int device, uint32_t height, uint32_t width,
               const uint8_t* map, int32_t gx, int32_t gy, float gamma) {
  return create_impl(out, device, height, width, 0, height, map, gx, gy, gamma, false);
}

int pp2_create_shard(pp2_ctx** out, int device, uint32_t global_height,
                     uint32_t width, uint32_t row_begin, uint32_t row_end,
                     const uint8_t* global_map, int32_t gx, int32_t gy,
                     float gamma) {
  return create_impl(out, device, global_height, width, row_begin, row_end,
                     global_map, gx, gy, gamma, true);
}

int pp2_destroy(pp2_ctx* c) {
  if (!c) return PP2_OK;
  DeviceGuard dg(c->device);
  if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
  pbvi_free(c);
  if (c->stream && c->stream != c->own_stream) (void)hipStreamSynchronize(c->stream);
  resident_gate_forget(c, c->stream);
  if (c->own_stream) resident_gate_forget(c, c->own_stream);
  if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  for (hipEvent_t e : {c->ev_enter, c->ev_leave})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->comm_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
  for (Planes* P : {&c->T, &c->L, &c->R, &c->C, &c->b[0], &c->b[1], &c->J[0],
                    &c->J[1], &c->Jsnap, &c->fib[0], &c->fib[1], &c->fibsnap})
    free_planes(P);
  if (c->d_map_alloc) (void)hipFree(c->d_map_alloc);
  if (c->A) (void)hipFree(c->A);
  if (c->bsum) (void)hipFree(c->bsum);
  for (float* pb : c->pbuf)
    if (pb) (void)hipFree(pb);
  if (c->rpartials) (void)hipFree(c->rpartials);
  if (c->staging) (void)hipFree(c->staging);
  if (c->code_alloc) (void)hipFree(c->code_alloc);
  resident_free(c);
  if (c->res_host) (void)hipHostFree(c->res_host);
  if (c->d_shift) (void)hipFree(c->d_shift);
  if (c->d_vec) (void)hipFree(c->d_vec);
  for (float* p : {c->d_dict, c->d_rows, c->d_dl, c->d_tu, c->d_rfact})
    if (p) (void)hipFree(p);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return PP2_OK;
}

int pp2_set_stream(pp2_ctx* c, void* s) {
  CHECK(check_ctx_settled(c));
  DeviceGuard dg(c->device);
  resident_gate_forget(c, c->stream);
  c->stream = s ? (hipStream_t)s : c->own_stream;
  return PP2_OK;
}

int pp2_synchronize(pp2_ctx* c) {
  CHECK(check_ctx_settled(c));
  DeviceGuard dg(c->device);
  if (c->comm_stream) HIPCHK(hipStreamSynchronize(c->comm_stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return PP2_OK;
}

int pp2_get_geometry(pp2_ctx* c, uint32_t* rows, uint32_t* width,
                     uint32_t* row_stride, uint32_t* row_begin) {
  CHECK(check_ctx(c));
  if (rows) *rows = (uint32_t)c->g.rows;
  if (width) *width = (uint32_t)c->g.width;
  if (row_stride) *row_stride = (uint32_t)c->g.wp;
  if (row_begin) *row_begin = (uint32_t)c->g.row0;
  return PP2_OK;
}

int pp2_set_tuning(pp2_ctx* c, int key, int value) {
  CHECK(check_ctx_settled(c));
  // a shard's resident eligibility may change: agree again (not for the
  // measurement knob, which changes nothing the ranks agree on)
  if (key != PP2_TUNE_COMM_TIMING) ++c->agree_gen;
  switch (key) {
    case PP2_TUNE_CELLS_PER_LANE: return pp2_set_cells_per_lane(c, value);
    case PP2_TUNE_NT_STREAMS: c->nt_streams = value != 0; return PP2_OK;
    case PP2_TUNE_CODED_MODEL: c->use_coded = value != 0; return PP2_OK;
    case PP2_TUNE_RESIDENT:
      if (value < 0 || value > 1) return set_err(PP2_EINVAL, "resident %d not in [0, 1]", value);
      c->resident = value;
      c->res_e_dict = -1;
      return PP2_OK;
    case PP2_TUNE_RESIDENT_STALL:
      if (value < -1) return set_err(PP2_EINVAL, "stall tile %d < -1", value);
      c->res_stall_tile = value;
      return PP2_OK;
    case PP2_TUNE_RESIDENT_CUS:
      if (value < 0) return set_err(PP2_EINVAL, "resident CUs %d < 0", value);
      c->res_cus = value;
      c->res_plan_e = c->sol_plan_e = c->res_e_dict = -1;
      return PP2_OK;
    case PP2_TUNE_RESIDENT_TILE_COLS:
      if (value < 0 || value > 3) return set_err(PP2_EINVAL, "tile columns %d not in [0, 3]", value);
      c->res_tc_pref = value;
      c->res_plan_e = c->res_e_dict = -1;
      return PP2_OK;
    case PP2_TUNE_RESIDENT_HALO:
      if (value < 0 || value > c->g.halo)
        return set_err(PP2_EINVAL, "resident halo %d not in [0, %d]", value, c->g.halo);
      c->res_halo = value;
      c->res_e_dict = -1;
      return PP2_OK;
    case PP2_TUNE_SHARD_LAG:
      if (value < 0 || value > 1) return set_err(PP2_EINVAL, "shard lag %d not in [0, 1]", value);
      c->shard_lag = value;
      return PP2_OK;
    case PP2_TUNE_STEP_PAIRS:
      if (value < 0 || value > 2) return set_err(PP2_EINVAL, "step pairs %d not in [0, 2]", value);
      c->step_pairs = value;
      return PP2_OK;
    case PP2_TUNE_NORM_BLOCK:
      if (value < 1 || value > kMaxNormBlock)
        return set_err(PP2_EINVAL, "normalisation block %d not in [1, %d]", value, kMaxNormBlock);
      c->norm_block = value;
      break_pipeline(c);
      return PP2_OK;
    case PP2_TUNE_COMM_STREAM:
      if (c->comm_stream) HIPCHK(hipStreamSynchronize(c->comm_stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      c->use_comm_stream = value != 0;
      return PP2_OK;
    case PP2_TUNE_COMM_TIMING:
      if (value < 0 || value > 1) return set_err(PP2_EINVAL, "comm timing %d not in [0, 1]", value);
      c->comm_timing = value != 0;
      c->comm_nev = 0;
      c->comm_dropped = 0;
      c->comm_open = false;
      return PP2_OK;
    case PP2_TUNE_HALO_DEPTH:
      if (value < 1 || value > c->kdepth_max)
        return set_err(PP2_EINVAL, "halo depth %d not in [1, %d]", value, c->kdepth_max);
      c->kdepth = value;
      break_pipeline(c);
      return PP2_OK;
    default: return set_err(PP2_EINVAL, "unknown tuning key %d", key);
  }
}

int pp2_set_cells_per_lane(pp2_ctx* c, int cpt) {
  CHECK(check_ctx(c));
  if (cpt != 1 && cpt != 2 && cpt != 4)
    return set_err(PP2_EINVAL, "cells per lane must be 1, 2 or 4 (got %d)", cpt);
  c->cpt = cpt;
  ++c->agree_gen;  // cpt decides coded_active, hence a shard's resident eligibility
  return PP2_OK;
}

// ---------------------------------------------------------------- model
int pp2_model_generate(pp2_ctx* c) {
  CHECK(check_ctx(c));
  DeviceGuard dg(c->device);
  if (c->dense_halo >= c->g.halo) {
    HIPCHK(pp2::launch_model_gen(c->stream, c->g, c->d_map, c->gx, c->gy, c->T.v,
                                 c->L.v, c->R.v, c->C.v));
    c->model_ready = true;
    return build_model_dict(c);
  }
  // A shard with deep halo rows: the model over rows [-g.halo, rows +
  // g.halo) into a transient full-halo copy, the code plane built from it,
  // then rows [-dense_halo, rows + dense_halo) kept in the context's planes
  // (contiguous: [row][plane][x])
  Planes t[4];
  struct Free {
    Planes* t;
    ~Free() { for (int i = 0; i < 4; ++i) free_planes(&t[i]); }
  } fr{t};
  const int K[4] = {81, 16, 9, 9};
  for (int i = 0; i < 4; ++i) CHECK(alloc_planes(c, &t[i], K[i], c->g.halo));
  HIPCHK(pp2::launch_model_gen(c->stream, c->g, c->d_map, c->gx, c->gy, t[0].v, t[1].v, t[2].v,
                               t[3].v));
  Planes* dst[4] = {&c->T, &c->L, &c->R, &c->C};
  const int dh = c->dense_halo;
  for (int i = 0; i < 4; ++i)
    HIPCHK(hipMemcpyAsync(dst[i]->v.p - (long long)dh * dst[i]->v.rs,
                          t[i].v.p - (long long)dh * t[i].v.rs,
                          (size_t)(c->g.rows + 2 * dh) * t[i].v.rs * sizeof(float),
                          hipMemcpyDeviceToDevice, c->stream));
  c->model_ready = true;
  const int s = build_model_dict(c, &t[0], &t[1], &t[2], &t[3]);
  HIPCHK(hipStreamSynchronize(c->stream));  // (before the transient planes go)
  return s;
}

int pp2_model_dict_info(pp2_ctx* c, int* entries, int* active) {
  CHECK(check_ctx(c));
  if (entries) *entries = c->dict_n;
  if (active) *active = coded_active(c) ? 1 : 0;
  return PP2_OK;
}

int pp2_model_download(pp2_ctx* c, float* T, float* L, float* R, float* C) {
  CHECK(check_model(c));
  DeviceGuard dg(c->device);
  if (T) CHECK(download_planes(c, c->T, T, nullptr));
  if (L) CHECK(download_planes(c, c->L, L, nullptr));
  if (R) CHECK(download_planes(c, c->R, R, nullptr));
  if (C) CHECK(download_planes(c, c->C, C, nullptr));
  return PP2_OK;
}

int pp2_model_upload(pp2_ctx* c, const float* T, const float* L, const float* R,
                     const float* C) {
  CHECK(check_ctx(c));
  if (c->nranks > 1 || c->g.rows != c->g.grows)
    return set_err(PP2_EINVAL, "model upload is only supported on unsharded contexts");
  DeviceGuard dg(c->device);
  if (!c->model_ready && !(T && L && R && C))
    return set_err(PP2_EINVAL, "first upload needs all of T, L, R, C");
  if (T) CHECK(upload_planes(c, c->T, T));
  if (L) CHECK(upload_planes(c, c->L, L));
  if (R) CHECK(upload_planes(c, c->R, R));
  if (C) CHECK(upload_planes(c, c->C, C));
  c->model_ready = true;
  if (c->dense_halo >= c->g.halo) return build_model_dict(c);
  // A whole-grid shard context (rows == grows, its own RCCL rank or none):
  // its dense planes hold dense_halo < g.halo halo rows, but the dictionary
  // build walks rows [-g.halo, rows + g.halo).  Build it from transient
  // full-halo copies: rows [-dense_halo, rows + dense_halo) from the context,
  // the rest zero -- the off-grid rows, which is what they are here.
  Planes t[4];
  struct Free {
    Planes* t;
    ~Free() { for (int i = 0; i < 4; ++i) free_planes(&t[i]); }
  } fr{t};
  Planes* src[4] = {&c->T, &c->L, &c->R, &c->C};
  const int dh = c->dense_halo;
  for (int i = 0; i < 4; ++i) {
    CHECK(alloc_planes(c, &t[i], src[i]->K, c->g.halo));
    HIPCHK(hipMemcpyAsync(t[i].v.p - (long long)dh * t[i].v.rs,
                          src[i]->v.p - (long long)dh * src[i]->v.rs,
                          (size_t)(c->g.rows + 2 * dh) * t[i].v.rs * sizeof(float),
                          hipMemcpyDeviceToDevice, c->stream));
  }
  const int s = build_model_dict(c, &t[0], &t[1], &t[2], &t[3]);
  HIPCHK(hipStreamSynchronize(c->stream));  // (before the transient planes go)
  return s;
}

int pp2_model_save(pp2_ctx* c, const char* dir) {
  CHECK(check_model(c));
  const size_t n = owned_cells(c);
  std::vector<float> T(n * 81), L(n * 16), R(n * 9);
  CHECK(pp2_model_download(c, T.data(), L.data(), R.data(), nullptr));
  CHECK(write_text(join(dir, "model_data_trans_prob"), T, 9));
  CHECK(write_text(join(dir, "model_data_meas_prob"), L, 16));
  CHECK(write_text(join(dir, "model_data_stage_reward"), R, 9));
  return PP2_OK;
}

int pp2_model_load(pp2_ctx* c, const char* dir) {
  CHECK(check_ctx(c));
  const size_t n = owned_cells(c);
  std::vector<float> T(n * 81), L(n * 16), R(n * 9), Cc(n * 9);
  CHECK(read_text(join(dir, "model_data_trans_prob"), T));
  CHECK(read_text(join(dir, "model_data_meas_prob"), L));
  CHECK(read_text(join(dir, "model_data_stage_reward"), R));
  // The MDP cost is not part of the POMDP files; keep/derive it on device.
  if (!c->model_ready) CHECK(pp2_model_generate(c));
  return pp2_model_upload(c, T.data(), L.data(), R.data(), nullptr);
}

// ---------------------------------------------------------------- belief
int pp2_belief_set(pp2_ctx* c, const float* b) {
  CHECK(check_ctx_settled(c));
  if (!b) return set_err(PP2_EINVAL, "belief is null");
  ++c->agree_gen;  // (after a lost shard run: every rank agrees again)
  DeviceGuard dg(c->device);
  break_pipeline(c);
  CHECK(upload_planes(c, c->b[c->bcur], b));
  bool ok = true;
  for (size_t i = 0; i < (size_t)c->g.rows * c->g.width && ok; ++i) ok = finite_nonneg(b[i]);
  c->belief_sparse_ok = ok;
  c->pending[c->bcur] = false;
  const float one = 1.0f;
  HIPCHK(hipMemcpyAsync(c->bsum + c->bcur, &one, sizeof one, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->lost_belief = false;  // only once the new belief is in place
  return PP2_OK;
}

int pp2_belief_get(pp2_ctx* c, float* b) {
  CHECK(check_ctx(c));
  if (!b) return set_err(PP2_EINVAL, "belief is null");
  DeviceGuard dg(c->device);
  CHECK(ensure_mass(c));
  return download_planes(c, c->b[c->bcur], b, c->bsum + c->bcur);
}

int pp2_belief_get_raw(pp2_ctx* c, float* b, float* mass) {
  CHECK(check_ctx(c));
  DeviceGuard dg(c->device);
  if (b) CHECK(download_planes(c, c->b[c->bcur], b, nullptr));
  if (mass) CHECK(pp2_belief_mass(c, mass));
  return PP2_OK;
}

int pp2_belief_mass(pp2_ctx* c, float* mass) {
  CHECK(check_ctx(c));
  if (!mass) return set_err(PP2_EINVAL, "mass is null");
  DeviceGuard dg(c->device);
  CHECK(ensure_mass(c));
  HIPCHK(hipMemcpyAsync(mass, c->bsum + c->bcur, sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return PP2_OK;
}

int pp2_belief_update(pp2_ctx* c, uint8_t u, uint8_t z) {
  CHECK(check_model(c));
  DeviceGuard dg(c->device);
  CHECK(exchange_halos(c, {HALO_BELIEF}));
  return belief_update_impl(c, u, z, false);
}

// ---------------------------------------------------------------- MDP
int pp2_mdp_reset(pp2_ctx* c) {
  CHECK(check_ctx_settled(c));
  ++c->agree_gen;
  DeviceGuard dg(c->device);
  for (Planes* P : {&c->J[0], &c->J[1], &c->Jsnap})
    HIPCHK(hipMemsetAsync(P->alloc, 0, P->floats * sizeof(float), c->stream));
  HIPCHK(hipMemsetAsync(c->A, 0, (size_t)c->g.rows * c->g.wp, c->stream));
  c->jcur = 0;
  break_pipeline(c);
  c->lost_values = false;  // only once the values are reset
  return PP2_OK;
}

int pp2_mdp_sweep(pp2_ctx* c, int n) {
  if (!c) return set_err(PP2_EINVAL, "null context");
  if (n < 0) return set_err(PP2_EINVAL, "negative sweep count");
  DeviceGuard dg(c->device);
  // resident sweeps queue behind unverified resident launches (resident_settle)
  if (n >= 2 && resident_chainable(c, 2)) {
    break_pipeline(c);
    return sweeps_resident(c, n);
  }
  CHECK(check_model(c));
  if (n >= 2 && solve_ready(c)) {
    break_pipeline(c);  // the loop's deep halo rows of J are stale after sweeps
    return sweeps_resident(c, n);
  }
  for (int i = 0; i < n; ++i) {
    CHECK(exchange_halos(c, {HALO_VALUE}));
    CHECK(mdp_sweep_once(c));
  }
  return PP2_OK;
}

int pp2_mdp_solve(pp2_ctx* c, int max_sweeps, int* sweeps, double* final_norm) {
  CHECK(check_model(c));
  DeviceGuard dg(c->device);
  CHECK(pp2_mdp_reset(c));
  // double max_optimal_cost = 5.0/(1.0-discount_factor) (path_planning_2d.cu:221)
  const double max_cost = 5.0 / (1.0 - (double)c->gamma);
  if (solve_ready(c)) {
    break_pipeline(c);  // J changes: the loop's deep halo rows are stale
    const int s = solve_resident(c, max_sweeps, max_cost * 1e-3, sweeps, final_norm);
    if (s != 1) return s;
    // a launch timed out (resident_settle's case): solve again from J = 0 on
    // per-sweep launches
    CHECK(pp2_mdp_reset(c));
  }
  int total = 0;
  double norm = 0.0;
  do {
    CHECK(pp2_mdp_sweep(c, 100));
    total += 100;
    CHECK(absdiff_max(c, c->J[c->jcur], c->Jsnap, &norm));
    if (max_sweeps > 0 && total >= max_sweeps) break;
  } while (norm > max_cost * 1e-3);
  if (sweeps) *sweeps = total;
  if (final_norm) *final_norm = norm;
  return PP2_OK;
}

int pp2_mdp_get(pp2_ctx* c, float* J, uint8_t* A) {
  CHECK(check_ctx(c));
  DeviceGuard dg(c->device);
  if (J) CHECK(download_planes(c, c->J[c->jcur], J, nullptr));
  if (A) {
    const size_t n = owned_cells(c);
    CHECK(ensure_staging(c, n));
    HIPCHK(pp2::launch_pack_u8(c->stream, c->g, c->A, (uint8_t*)c->staging));
    HIPCHK(hipMemcpyAsync(A, c->staging, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  return PP2_OK;
}

// ---------------------------------------------------------------- north star
int pp2_loop_step(pp2_ctx* c, uint8_t u, uint8_t z) {
  CHECK(check_model(c));
  DeviceGuard dg(c->device);
  if (c->group)
    return set_err(PP2_ESTATE, "context belongs to a shard group: drive it with pp2_shard_group_*");
  return loop_step_impl(c, u, z);
}

// A query: plans (host arithmetic and the occupancy API), allocates nothing.
int pp2_loop_steps_per_launch(pp2_ctx* c, int* steps) {
  CHECK(check_ctx(c));
  if (!steps) return set_err(PP2_EINVAL, "steps is null");
  DeviceGuard dg(c->device);
  if (c->comm || c->group) {
    const int e = shard_resident_e(c);
    *steps = e > 0 ? e : pairs_apply(c) ? 2 : 1;
  } else {
    *steps = resident_model_ok(c) && resident_plan_for(c, 0) ? pp2::kResidentMaxSteps
             : pairs_apply(c) ? 2 : 1;
  }
  return PP2_OK;
}

int pp2_resident_tiling(pp2_ctx* c, int* tiles, int* rows_per_tile, int* tile_cols) {
  CHECK(check_ctx(c));
  DeviceGuard dg(c->device);
  int e = 0;
  bool ok;
  if (c->comm || c->group) {
    e = shard_resident_e(c);
    ok = e > 0 && resident_plan_for(c, e);
  } else {
    ok = resident_model_ok(c) && resident_plan_for(c, 0);
  }
  if (tiles) *tiles = ok ? c->res_plan.ntiles : 0;
  if (rows_per_tile) *rows_per_tile = ok ? c->res_plan.rt : 0;
  if (tile_cols) *tile_cols = ok ? (c->res_plan.tr ? 3 : c->res_plan.tc) : 0;
  return PP2_OK;
}

int pp2_resident_status(pp2_ctx* c, int* fallbacks, int* enabled) {
  CHECK(check_ctx_settled(c));
  if (fallbacks) *fallbacks = c->res_fallbacks;
  if (enabled) *enabled = c->resident;
  return PP2_OK;
}

int pp2_resident_launches(pp2_ctx* c, int* loop_launches, int* solve_launches) {
  CHECK(check_ctx_settled(c));
  if (loop_launches) *loop_launches = c->res_launches;
  if (solve_launches) *solve_launches = c->sol_launches;
  return PP2_OK;
}

// The ranks' smallest v (a blocking 1-int all-reduce): RCCL shards agree on
// their communication pattern before a run takes the resident path, since
// eligibility (the model, the belief's sign pattern, allocations) is local.
static int agree_min(pp2_ctx* c, int* v) {
  if (c->nranks <= 1) return PP2_OK;
  int* d = reinterpret_cast<int*>(c->rpartials);
  HIPCHK(hipMemcpyAsync(d, v, sizeof(int), hipMemcpyHostToDevice, c->stream));
  CHECK(comm_enter(c));
  NCCLCHK(ncclAllReduce(d, d, 1, ncclInt32, ncclMin, c->comm, cst(c)));
  CHECK(comm_leave(c));
  HIPCHK(hipMemcpyAsync(v, d, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return PP2_OK;
}

int pp2_loop_run(pp2_ctx* c, int n, const uint8_t* us, const uint8_t* zs) {
  if (!c) return set_err(PP2_EINVAL, "null context");
  if (n < 0 || (n > 0 && (!us || !zs))) return set_err(PP2_EINVAL, "bad trajectory");
  DeviceGuard dg(c->device);
  // a resident run queues behind unverified resident launches (no host sync
  // between back-to-back runs; resident_settle verifies them all)
  if (n >= 2 && resident_chainable(c, 1)) return loop_resident(c, n, us, zs);
  CHECK(check_model(c));
  if (c->group)
    return set_err(PP2_ESTATE, "context belongs to a shard group: drive it with pp2_shard_group_*");
  if (n >= 2 && c->comm) {
    // The ranks agree on e (a blocking all-reduce) only when something that
    // decides it may have changed since the last agreement: the model or a
    // tuning, events every rank of an SPMD program goes through together, so
    // the generation counts stay equal across ranks and all of them agree,
    // or none (a 20-step call saves one RCCL round trip and a host sync).
    int e;
    if (c->agree_done != c->agree_gen) {
      e = shard_resident_e(c);
      if (e > 0 && !shard_resident_ready(c, e)) e = 0;
      CHECK(agree_min(c, &e));
      c->agreed_e = e;
      c->agree_done = c->agree_gen;
    } else {
      e = c->agreed_e;
    }
    if (e > 0) {
      // every generation bump that can change eligibility makes the ranks
      // agree again above; a cached e that is no longer ready here would
      // leave this rank alone off the resident path (a collective mismatch)
      if (!shard_resident_ready(c, e))
        return set_err(PP2_ESTATE, "the ranks agreed on a %d-row resident halo that this "
                       "shard can no longer run (changed without a model build, tuning or "
                       "belief/value reset on every rank)", e);
      return shard_loop_resident(c, e, n, us, zs);
    }
  }
  if (n >= 2 && resident_ready(c)) return loop_resident(c, n, us, zs);
  return loop_run_launches(c, n, us, zs);
}

// ---------------------------------------------------------------- FIB
int pp2_fib_reset(pp2_ctx* c) {
  CHECK(check_ctx(c));
  DeviceGuard dg(c->device);
  for (Planes* P : {&c->fib[0], &c->fib[1], &c->fibsnap})
    HIPCHK(hipMemsetAsync(P->alloc, 0, P->floats * sizeof(float), c->stream));
  c->fcur = 0;
  c->fib_finite = true;
  ++c->fib_version;
  return PP2_OK;
}

int pp2_fib_sweep(pp2_ctx* c, int n) {
  CHECK(check_model(c));
  if (n < 0) return set_err(PP2_EINVAL, "negative sweep count");
  DeviceGuard dg(c->device);
  for (int i = 0; i < n; ++i) {
    CHECK(exchange_halos(c, {HALO_FIB}));
    CHECK(fib_sweep_once(c));
  }
  return PP2_OK;
}

int pp2_fib_solve(pp2_ctx* c, int max_sweeps, int* sweeps, float* final_norm) {
  CHECK(check_model(c));
  DeviceGuard dg(c->device);
  CHECK(pp2_fib_reset(c));
  int total = 0;
  double norm = 0.0;
  do {
    CHECK(pp2_fib_sweep(c, 10));
    total += 10;
    CHECK(absdiff_max(c, c->fib[c->fcur], c->fibsnap, &norm));
    if (max_sweeps > 0 && total >= max_sweeps) break;
  } while ((float)norm > 0.01f);
  if (sweeps) *sweeps = total;
  if (final_norm) *final_norm = (float)norm;
  return PP2_OK;
}

int pp2_fib_get(pp2_ctx* c, float* alphas) {
  CHECK(check_ctx(c));
  if (!alphas) return set_err(PP2_EINVAL, "alphas is null");
  DeviceGuard dg(c->device);
  return download_planes(c, c->fib[c->fcur], alphas, nullptr);
}

int pp2_fib_set(pp2_ctx* c, const float* alphas) {
  CHECK(check_ctx(c));
  if (!alphas) return set_err(PP2_EINVAL, "alphas is null");
  DeviceGuard dg(c->device);
  ++c->fib_version;
  const size_t n = owned_cells(c) * 9;
  c->fib_finite = true;
  for (size_t i = 0; i < n && c->fib_finite; ++i)
    if (!std::isfinite(alphas[i])) c->fib_finite = false;
  return upload_planes(c, c->fib[c->fcur], alphas);
}

// saveFibDataToFile / loadFibDataFromFile (fast_informed_bound_cuda.cu:343-394):
// dir/fib_alphas holds one cell per line (9 "%15.8f" values), dir/fib_actions
// the 9 actions {0..8} as "%10u" lines.
int pp2_fib_save(pp2_ctx* c, const char* dir) {
  CHECK(check_ctx(c));
  std::vector<float> al(owned_cells(c) * 9);
  CHECK(pp2_fib_get(c, al.data()));
  CHECK(write_text(join(dir, "fib_alphas"), al, 9));
  const std::string path = join(dir, "fib_actions");
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return set_err(PP2_EIO, "cannot open %s for writing", path.c_str());
  for (unsigned u = 0; u < 9; ++u) fprintf(f, "%10u\n", u);
  if (fclose(f) != 0) return set_err(PP2_EIO, "write %s failed", path.c_str());
  return PP2_OK;
}

int pp2_fib_load(pp2_ctx* c, const char* dir) {
  CHECK(check_ctx(c));
  std::vector<float> al(owned_cells(c) * 9);
  CHECK(read_text(join(dir, "fib_alphas"), al));
  std::vector<uint8_t> act(9);
  CHECK(read_actions(join(dir, "fib_actions"), act));
  for (int u = 0; u < 9; ++u)
    if (act[u] != u)
      return set_err(PP2_EIO, "fib_actions: alpha %d is labelled action %u (expected %d)", u,
                     act[u], u);
  return pp2_fib_set(c, al.data());
}

// ---------------------------------------------------------------- shards
int pp2_rccl_unique_id(uint8_t id[PP2_RCCL_ID_BYTES]) {
  if (!id) return set_err(PP2_EINVAL, "id is null");
  static_assert(sizeof(ncclUniqueId) == PP2_RCCL_ID_BYTES, "RCCL id size");
  ncclUniqueId uid;
  NCCLCHK(ncclGetUniqueId(&uid));
  memcpy(id, &uid, sizeof uid);
  return PP2_OK;
}

int pp2_shard_comm_init(pp2_ctx* c, const uint8_t id[PP2_RCCL_ID_BYTES],
                        int nranks, int rank) {
  CHECK(check_ctx(c));
  if (!id || nranks < 1 || rank < 0 || rank >= nranks)
    return set_err(PP2_EINVAL, "bad rank %d / nranks %d", rank, nranks);
  DeviceGuard dg(c->device);
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  if (!c->comm_stream) {
    HIPCHK(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&c->ev_enter, &c->ev_leave})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  NCCLCHK(ncclCommInitRank(&c->comm, nranks, uid, rank));
  c->nranks = nranks;
  c->rank = rank;
  // loop halo depth: no deeper than the halo allocation or any shard's rows
  int* d = nullptr;
  int rows = c->g.rows;
  HIPCHK(hipMalloc(&d, sizeof(int)));
  HIPCHK(hipMemcpyAsync(d, &rows, sizeof(int), hipMemcpyHostToDevice, c->stream));
  CHECK(comm_enter(c));
  NCCLCHK(ncclAllReduce(d, d, 1, ncclInt32, ncclMin, c->comm, cst(c)));
  CHECK(comm_leave(c));
  HIPCHK(hipMemcpyAsync(&rows, d, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipFree(d));
  c->min_shard_rows = rows;
  c->kdepth_max = std::max(1, std::min(std::min(c->g.halo, kMaxNormBlock), rows));
  c->kdepth = c->kdepth_max;
  c->res_e_dict = -1;
  break_pipeline(c);
  return PP2_OK;
}

}  // extern "C"
