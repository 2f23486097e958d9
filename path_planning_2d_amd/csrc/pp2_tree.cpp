// pp2_tree.cpp -- online QV-tree planner (C ABI pp2_planner_*, include/pp2.h).
//
// Host tree logic restates QNode / VNode / SearchTree
// (include/path_planning_2d/search_tree.h:31-165,
//  src/pomdp/search_tree_cuda.cu:161-626) and the plan step of
// PomdpPathPlanning2d::beliefCallback (src/pomdp/path_planning_2d.cu:199-241).
// What changes is where the per-cell work runs: one VNode::expand issues one
// batched device pass (pp2::launch_expand) that scores every (action,
// observation) child at once, while the host draws the reference's samples;
// beliefs are materialised on the device only for nodes that get expanded.
// Host arithmetic is plain fp32 (built with -ffp-contract=off), as the
// reference's x86 host code.
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <set>
#include <vector>

#include <rocrand/rocrand_xorwow.h>

#include "pp2_ctx.h"
#include "pp2_pbvi_internal.h"
#include "pp2_rand.h"

using namespace pp2rt;

namespace {

using pp2rt::GlibcRand;

// cuRAND XORWOW as curand_init(seed, subsequence, 0) seeds it (CUDA 8
// curand_kernel.h: salted seed halves, then skipahead by subsequence * 2^67);
// the 2^67 jump comes from rocRAND's precomputed XORWOW jump matrices.
struct CurandXorwow : rocrand_device::xorwow_engine {
  CurandXorwow(uint64_t seed, uint64_t subsequence)
      : rocrand_device::xorwow_engine(0ULL, 0ULL, 0ULL) {
    const uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    const uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    m_state.d = 6615241u + t1 + t0;
    m_state.x[0] = 123456789u + t0;
    m_state.x[1] = 362436069u ^ t0;
    m_state.x[2] = 521288629u + t1;
    m_state.x[3] = 88675123u ^ t1;
    m_state.x[4] = 5783321u + t0;
    discard_subsequence(subsequence);
  }
};

inline float curand_uniform_of(uint32_t x) {
  const float inv = 2.3283064e-10f;  // CURAND_2POW32_INV
  return fmaf((float)x, inv, inv / 2.0f);
}

struct QNode;

struct VNode {
  uint8_t observation = 0;
  float weight = 0.0f;
  QNode* parent = nullptr;
  std::vector<QNode*> children;
  float upper_bound = FLT_MAX;
  float lower_bound = -FLT_MAX;
  float heuristic = FLT_MIN;
  VNode* vnode_to_expand = nullptr;
  uint32_t depth = 0;
  int slot = -1;  // device belief slot, -1 = not materialised
};

struct QNode {
  uint8_t action = 0;
  VNode* parent = nullptr;
  std::vector<VNode*> children;
  float upper_bound = FLT_MAX;
  float lower_bound = -FLT_MAX;
  float heuristic = FLT_MIN;
  float reward = 0.0f;
  VNode* vnode_to_expand = nullptr;
  uint32_t depth = 1;
};

struct Slot {
  Planes b;               // the belief in plane geometry (reference_order 0)
  float* mass = nullptr;  // device scalar: unnormalised mass of b
  float* row = nullptr;   // reference_order 1: the normalised belief, a dense row
};

constexpr int kStatsPerChild = 10;
// grids up to this many cells run the reference-order sums as walked chains
// (k_chain_walk; its LDS holds n terms, pp2_pbvi_host.hip kWalkMax)
constexpr long long kSeqChainMax = 8192;

constexpr int kStatsFloats = 16 * 9 * kStatsPerChild;

// The x-ordered fp32 prefix sum of a belief: the cdf the QNode constructor
// samples states from (search_tree_cuda.cu:176-183), one serial chain.
// Adding a zero cell leaves the running sum bit-identical, so a 16-cell block
// without a set bit only copies the sum forward (PP2_CDF_SKIP=0 turns that off).
struct Cdf {
  std::vector<float> v;
  bool skip = true;

  void build(const float* b, size_t n) {
    v.resize(n);
    float* c = v.data();
    float acc = 0.0f;
    size_t i = 0;
    if (skip)
      for (; i + 16 <= n; i += 16) {
        uint32_t bits[16], any = 0;
        std::memcpy(bits, b + i, sizeof bits);
        for (int t = 0; t < 16; ++t) any |= bits[t];
        if (!any) {
          for (int t = 0; t < 16; ++t) c[i + t] = acc;
          continue;
        }
        for (int t = 0; t < 16; ++t) {
          acc = acc + b[i + t];
          c[i + t] = acc;
        }
      }
    for (; i < n; ++i) {
      acc = acc + b[i];
      c[i] = acc;
    }
  }
};

}  // namespace

struct pp2_planner {
  pp2_ctx* ctx = nullptr;
  pp2_planner_params prm{};
  float gamma = 0.95f;
  float lb_const = 0.0f;
  int W = 0;
  size_t n = 0;
  std::vector<float> hT, hL;    // host copies (reference layouts) for sampling
  std::vector<float> u1, u2;    // the curand_uniform pairs every QNode sees
  GlibcRand rng;

  std::vector<Slot> slots;
  std::vector<int> free_slots;
  std::vector<void*> arenas;    // reference order: slot rows and masses, a chunk of slots each
  Planes P;                     // 9 prediction planes (scratch)
  float* d_rpart = nullptr;     // tiles * 9
  float* d_spart = nullptr;     // tiles * 16 * 90
  float* d_bpart = nullptr;     // belief-update / dots partials
  // Results the host reads back live in coherent pinned host memory, and the
  // kernels that produce them store there directly (d_* = the device view of
  // h_*): no copy engine between a kernel and the host's wait on it.
  float* h_out = nullptr;       // [9 rewards | 1440 stats | 10 dots | 1 mass]
  float* d_out = nullptr;
  float* h_belief = nullptr;    // normalised belief, dense (the sampling cdf's input)
  float* d_dense = nullptr;
  hipEvent_t ev_belief = nullptr;
  hipEvent_t ev_done = nullptr;  // an expansion's last device work (cheaper to wait on than the stream)
  Cdf cdf;                      // the expanded belief's cdf (host sampling)

  // lower_bound_mode 1: PBVI leaf bounds (evaluatePbviCpu) of all 144
  // (observation, action) children per expansion, as one split-x MFMA GEMM
  // of the materialised children against the context's alpha vectors.
  bool pbvi = false;
  int lb_S = 0, lb_Sp = 0, lb_ld = 0, lb_split = 1;
  float* d_parent = nullptr;    // [ld] the expanded belief, unnormalised
  float* d_children = nullptr;  // [256][ld] its 144 children, row z*9 + a
  float* d_lbpart = nullptr;    // [lb_split][256][Sp] split-x partial dots
  float* d_lbdots = nullptr;    // [256][Sp]
  int* d_lbidx = nullptr;
  float* h_lbv = nullptr;       // pinned: max_k <row, alpha_k>
  float* d_lbv = nullptr;
  int* d_srow = nullptr;
  uint8_t *d_us = nullptr, *d_zs = nullptr;

  // reference_order: node beliefs are dense rows stored normalised exactly
  // as the reference's host normalises them, and every grid-wide sum equals
  // the reference's x-ordered fp32 chain (pp2_fchain.hip; the PBVI leaf dots
  // k_pair_chain).
  bool ref = false;
  // grids of n <= PP2_SEQ_CHAIN_MAX cells (default kSeqChainMax; 0 = off):
  // the sums as sequential chains, one wave per chain whose lanes form the
  // terms into LDS and whose lane 0 walks them (launch_pair_seq_small,
  // launch_row_cdf_seq: k_chain_walk), one launch per chain set instead of
  // the exact parallel chain sets' three.  The reference node's 100 x 40
  // plan step: p50 2.54 vs 3.34-3.51 ms (profiles/r05/chain_walk_ab.txt).
  bool seq = false;
  // larger grids up to 65536 cells (PP2_FX=0: off): each chain set as ONE
  // launch, a workgroup per chain (pp2::launch_fx, launch_fx_cdf_sample)
  bool fx = false;
  // reference order: a node row for each of the 144 children, acquired before
  // an expansion is enqueued; the kept children's rows are stored straight
  // into theirs by the expansion's kernels (no store after the host's wait)
  std::vector<int> pre;
  // PP2_FX_STAMPS=1 (diagnostics): the fused kernels' phase clocks, 8 per
  // workgroup, summed per kernel and phase, printed when the planner goes
  unsigned long long* d_stamps = nullptr;
  double fx_phase[4][8] = {};
  double fx_count[4][4] = {};  // walk steps, fallback chunks, stash misses, predicted chunks
  long long fx_groups[4] = {}, fx_sets = 0;
  int ref_ld = 0;               // dense row length (multiple of 64, zero tail)
  float* d_rrows = nullptr;     // [9][ld] R[.][a]
  float* d_frows = nullptr;     // [9][ld] FIB alphas[.][i]
  float* d_lrows = nullptr;     // [16][ld] L[.][z]
  float* d_pred = nullptr;      // [9][ld] the expanded belief's predictions
  float* d_csum = nullptr;      // [144] the children's masses (accumulate)
  float* d_cdf = nullptr;       // the expanded belief's running sums
  float* d_sub = nullptr;       // and every 16th cell's (n <= 65536; else null)
  float* h_r = nullptr;         // pinned: the expansion's rand() values [9][N]
  float* d_r = nullptr;
  float *d_u1 = nullptr, *d_u2 = nullptr;  // the curand uniforms [N]
  int* h_counts = nullptr;      // pinned: observation counts [9][16]
  int* d_counts = nullptr;
  int* d_klist = nullptr;       // the kept children z * 9 + a, and their number
  int* d_kcount = nullptr;
  pp2::FcScratch scr_main, scr_side;  // chain-set scratch of the two streams
  // the kept children's FIB dots (FC_KEPT): their chunk sums on main right
  // after the samples (beside the children's walk), then their tables and
  // walk once the masses are in; the rewards' own scratch (the FIB sums read
  // scr_side's chunk sums)
  pp2::FcScratch scr_fib, scr_rew;
  hipStream_t side2 = nullptr;  // (spare)
  hipEvent_t ev_csum = nullptr, ev_fsum = nullptr;
  // PP2_PLAN_EVENTS=1: timing events at the expansion's phase ends (device
  // time from the expansion's start on main), summed over expansions
  bool pev = false;
  hipEvent_t tev[10] = {};
  double tev_sum[10] = {};
  long long tev_n = 0;
  float** h_rowptr = nullptr;   // pinned, mapped: the 144 children's node rows
  float** d_rowptr = nullptr;
  float** d_rowdev = nullptr;   // device: the same, published by k_tree_sample
  uint16_t* d_cmask = nullptr;  // the kept children's FIB candidates (launch_fib_cands)
  bool fib_cands = false;       // PP2_FIB_CANDS=1: the FIB chains below another skipped
  bool row_first = false;       // PP2_ROW_FIRST=1: the cdf chain enqueued before the predictions
  bool fib_unit = true;         // PP2_FIB_UNIT=0: the FIB sums wait for the children's chunk sums
  bool host_join = true;        // PP2_HOST_JOIN=0: main joins side on the device
  bool kids_first = false;      // PP2_KIDS_FIRST=1: the children's launches ahead of the cdf chain's
  // reference order, PBVI leaves: every row's candidate alphas (those whose
  // exact chain can reach the row's maximum, from the split-x GEMM's
  // approximate dots and a rigorous bound) as one exact chain set (FC_LIST)
  pp2::FcScratch scr_pbvi;      // its scratch (reserved when it fits; else k_pair_chain)
  float* d_lbapprox = nullptr;  // [256][Sp] approximate dots
  float* d_amax = nullptr;      // [Sp] max |alpha_i|
  uint32_t* d_aflag = nullptr;  // [Sp] alpha_i's sign flags
  unsigned astats_version = 0;  // the context's pbvi_version d_amax / d_aflag are from
  int2* d_plist = nullptr;      // [144 S] candidate (row, alpha) pairs
  int* d_pcount = nullptr;
  int* h_pstat = nullptr;       // pinned: candidates of the last set (PP2_PBVI_STATS)
  long long stat_cands = 0, stat_rows = 0, stat_sets = 0;
  // PP2_PLAN_TIMING=1: host time per expansion (us): enqueue (first launch ..
  // the wait), the tree work after the wait .. store_children enqueued, and
  // the time from there to the next expansion's first launch
  bool timing = false;
  bool spin = true;             // wait_event: poll (PP2_SPIN_WAIT)
  double t_enq = 0, t_post = 0, t_between = 0;
  double t_pa = 0, t_pb = 0;  // (t_post: .. the nodes' first row read, .. the nodes built)
  double t_mark[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // (enqueue phases, tmark())
  // (plan steps: entry .. the first expansion, the last expansion .. return,
  // the caller's time between steps)
  double t_upd = 0, t_tail = 0, t_out = 0;
  long long t_steps = 0;
  std::chrono::steady_clock::time_point t_ret_step{};
  long long t_n = 0;
  std::chrono::steady_clock::time_point t_last_store{};
  unsigned frows_version = 0;   // the context's fib_version d_frows was packed from (0: never)
  hipStream_t side = nullptr;   // reward chains beside the child chains
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_kids = nullptr;
  hipEvent_t ev_kept = nullptr;  // the kept children's rows are stored (main -> side)
  float* d_rsum = nullptr;      // [256] row sums
  float* h_rout = nullptr;      // pinned: [9 rewards | 256 x 9 FIB dots]
  float* d_rout = nullptr;

  VNode* root = nullptr;
  uint32_t n_vnodes = 0, n_qnodes = 0, expansions = 0;
  // deleted nodes, kept for reuse (an expansion builds ~50: malloc / free
  // per node cost the host several us per expansion)
  std::vector<VNode*> vpool;
  std::vector<QNode*> qpool;
};

namespace {

constexpr int kOutRewards = 0;
constexpr int kOutStats = 9;
constexpr int kOutDots = 9 + kStatsFloats;
constexpr int kOutMass = kOutDots + kStatsPerChild;
constexpr int kOutFloats = kOutMass + 1;

// `count` floats of coherent pinned host memory and their device view.
bool host_mapped(size_t count, float** host, float** dev) {
  if (hipHostMalloc((void**)host, count * sizeof(float),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return false;
  std::memset(*host, 0, count * sizeof(float));
  return hipHostGetDevicePointer((void**)dev, *host, 0) == hipSuccess;
}

// Reference order: slots come in chunks of rows from one allocation (one
// hipMalloc and one memset per chunk, not per kept child: every kept child
// of an expansion takes a row), about 64 MB per chunk, 4 to 64 rows.
int grow_ref_slots(pp2_planner* p) {
  const size_t row = (size_t)p->ref_ld * sizeof(float);
  const size_t nrows = std::min<size_t>(64, std::max<size_t>(4, ((size_t)64 << 20) / row));
  const size_t bytes = nrows * (row + 64);
  char* base = nullptr;
  HIPCHK(hipMalloc(&base, bytes));
  p->arenas.push_back(base);
  HIPCHK(hipMemsetAsync(base, 0, bytes, p->ctx->stream));  // the rows' zero tails past n
  for (size_t r = 0; r < nrows; ++r) {
    Slot s;
    s.row = reinterpret_cast<float*>(base + r * row);
    s.mass = reinterpret_cast<float*>(base + nrows * row + r * 64);
    p->slots.push_back(s);
    p->free_slots.push_back((int)p->slots.size() - 1);
  }
  // hand out the chunk's first rows first
  std::reverse(p->free_slots.end() - (long)nrows, p->free_slots.end());
  return PP2_OK;
}

int acquire_slot(pp2_planner* p, int* out) {
  if (p->free_slots.empty()) {
    if (p->ref) {
      CHECK(grow_ref_slots(p));
    } else {
      Slot s;
      CHECK(alloc_planes(p->ctx, &s.b, 1));
      HIPCHK(hipMalloc(&s.mass, 64));
      p->slots.push_back(s);
      p->free_slots.push_back((int)p->slots.size() - 1);
    }
  }
  *out = p->free_slots.back();
  p->free_slots.pop_back();
  return PP2_OK;
}

void release_slot(pp2_planner* p, int s) {
  if (s >= 0) p->free_slots.push_back(s);
}

void delete_vnode_only(pp2_planner* p, VNode* v) {
  release_slot(p, v->slot);
  --p->n_vnodes;
  p->vpool.push_back(v);
}

void delete_qnode_only(pp2_planner* p, QNode* q) {
  --p->n_qnodes;
  p->qpool.push_back(q);
}

// A node as freshly constructed, from the pool when it has one (the
// children vectors keep their capacity)
QNode* alloc_qnode(pp2_planner* p) {
  ++p->n_qnodes;
  if (p->qpool.empty()) return new QNode();
  QNode* q = p->qpool.back();
  p->qpool.pop_back();
  std::vector<VNode*> keep;
  keep.swap(q->children);
  *q = QNode();
  keep.clear();
  q->children.swap(keep);
  return q;
}

void delete_subtree(pp2_planner* p, VNode* v);

void delete_subtree(pp2_planner* p, QNode* q) {
  for (VNode* v : q->children)
    if (v) delete_subtree(p, v);
  delete_qnode_only(p, q);
}

void delete_subtree(pp2_planner* p, VNode* v) {
  for (QNode* q : v->children)
    if (q) delete_subtree(p, q);
  delete_vnode_only(p, v);
}

VNode* new_vnode(pp2_planner* p, uint8_t z, float w, QNode* parent) {
  VNode* v;
  if (p->vpool.empty()) {
    v = new VNode();
  } else {
    v = p->vpool.back();
    p->vpool.pop_back();
    std::vector<QNode*> keep;
    keep.swap(v->children);
    *v = VNode();
    keep.clear();
    v->children.swap(keep);
  }
  v->observation = z;
  v->weight = w;
  v->parent = parent;
  v->vnode_to_expand = v;  // VNode ctor (search_tree_cuda.cu:385)
  ++p->n_vnodes;
  return v;
}

// The FIB upper bound of a belief with FIB values f_i = dots_i / mass
// (evaluateFibCpu: std::max_element -> first maximum).
float fib_upper(const float* dots, float mass) {
  float best = dots[0] / mass;
  for (int i = 1; i < 9; ++i) {
    const float v = dots[i] / mass;
    if (best < v) best = v;
  }
  return best;
}

// max_k <row r, alpha_k> for rows [0, nrows) of d_rows (ld floats each) into
// h_lbv[r] (asynchronous; the caller synchronises the stream).
int pbvi_row_max(pp2_planner* p, const float* d_rows, int nrows) {
  pp2_ctx* c = p->ctx;
  const float* al = nullptr;
  int S = 0, Sp = 0, ld = 0;
  CHECK(pbvi_alphas(c, &al, &S, &Sp, &ld));
  if (S != p->lb_S || ld != p->lb_ld)
    return set_err(PP2_ESTATE, "PBVI alpha vectors changed size since the planner was created");
  const int Mp = (nrows + pp2::kGemmTile - 1) / pp2::kGemmTile * pp2::kGemmTile;
  const long long sstride = (long long)Mp * Sp;
  HIPCHK(pp2::launch_gemm_nt(c->stream, d_rows, al, p->d_lbpart, Mp, Sp, ld, 1, 0, 0,
                             p->lb_split, sstride));
  HIPCHK(pp2::launch_sum_splits(c->stream, p->d_lbpart, p->lb_split, sstride, (int)sstride,
                                p->d_lbdots));
  HIPCHK(pp2::launch_argmax_rows(c->stream, p->d_lbdots, nrows, S, Sp, p->d_lbidx, p->d_lbv));
  return PP2_OK;
}

// QNode::update (search_tree_cuda.cu:251-286)
void qnode_update(pp2_planner* p, QNode* q) {
  float ub_rtg = 0.0f, lb_rtg = 0.0f;
  for (VNode* v : q->children) {
    ub_rtg += v->upper_bound * v->weight;
    lb_rtg += v->lower_bound * v->weight;
  }
  q->upper_bound = q->reward + p->gamma * ub_rtg;
  q->lower_bound = q->reward + p->gamma * lb_rtg;
  q->heuristic = 0.0f;
  for (VNode* v : q->children) {
    const float h = p->gamma * v->weight * v->heuristic;
    if (h > q->heuristic) {
      q->heuristic = h;
      q->vnode_to_expand = v->vnode_to_expand;
    }
  }
  uint32_t child_depth = 0;
  for (VNode* v : q->children)
    if (v->depth > child_depth) {
      child_depth = v->depth;
      q->depth = child_depth + 1;
    }
}

// VNode::update (search_tree_cuda.cu:397-435)
void vnode_update(VNode* v) {
  size_t ui = 0, li = 0;
  for (size_t i = 1; i < v->children.size(); ++i) {
    if (v->children[ui]->upper_bound < v->children[i]->upper_bound) ui = i;
    if (v->children[li]->lower_bound < v->children[i]->lower_bound) li = i;
  }
  v->upper_bound = v->children[ui]->upper_bound;
  v->lower_bound = v->children[li]->lower_bound;
  v->heuristic = -FLT_MAX;
  for (QNode* q : v->children) {
    if (q->upper_bound <= v->lower_bound) continue;
    if (q->heuristic > v->heuristic) {
      v->heuristic = q->heuristic;
      v->vnode_to_expand = q->vnode_to_expand;
    }
  }
  uint32_t child_depth = 0;
  for (QNode* q : v->children)
    if (q->depth > child_depth) {
      child_depth = q->depth;
      v->depth = child_depth + 1;
    }
}

// ---------------------------------------------------------------- reference order
constexpr int kRefOutFloats = 9 + 256 * 9;

// K planes of `src` -> K dense rows of p->ref_ld floats (zero tails stay 0).
int pack_rows(pp2_planner* p, pp2::PlaneSet src, int K, float* dst) {
  pp2_ctx* c = p->ctx;
  for (int k = 0; k < K; ++k) {
    pp2::PlaneSet v = src;
    v.p += (long long)k * src.ps;
    HIPCHK(pp2::launch_pack(c->stream, c->g, 1, v, dst + (size_t)k * p->ref_ld, nullptr));
  }
  return PP2_OK;
}

// The FIB alphas as 9 dense rows, repacked when they changed.
// Whether T is +0 off every action's base-kernel support on every cell (the
// coded model's bitwise-verified sparse dictionary): the predictions read the
// support taps only.
static bool tree_sparse_t(const pp2_ctx* c) { return c->dict_n > 0 && c->dict_sparse; }

int ref_frows(pp2_planner* p) {
  pp2_ctx* c = p->ctx;
  if (p->frows_version != c->fib_version) {
    CHECK(pack_rows(p, c->fib[c->fcur].v, 9, p->d_frows));
    p->frows_version = c->fib_version;
  }
  return PP2_OK;
}

// evaluatePbviCpu (first maximum over the alphas, x-ordered dots) of `rows`
// dense normalised beliefs into h_lbv[r]; with a device list (klist,
// kcount), of the listed rows only (the kept children of an expansion; the
// other rows' h_lbv are stale).  Asynchronous.
int ref_pbvi_bounds(pp2_planner* p, const float* d_rows, int rows, const int* klist = nullptr,
                    const int* kcount = nullptr, hipStream_t st = nullptr) {
  pp2_ctx* c = p->ctx;
  if (!st) st = c->stream;
  const float* al = nullptr;
  int S = 0, Sp = 0, ald = 0;
  CHECK(pbvi_alphas(c, &al, &S, &Sp, &ald));
  if (S != p->lb_S || ald != p->ref_ld)
    return set_err(PP2_ESTATE, "PBVI alpha vectors changed size since the planner was created");
  if (p->scr_pbvi.chains > 0) {
    // candidates: approximate dots by the split-x f32 MFMA GEMM (d_rows
    // holds Mp rows), then the alphas whose chain can reach each row's
    // maximum (pp2_fchain.hip k_pbvi_cands), then their exact chains
    if (p->astats_version != c->pbvi_version) {
      HIPCHK(pp2::launch_alpha_stats(st, al, S, (int)p->n, p->ref_ld, p->d_amax,
                                     p->d_aflag));
      p->astats_version = c->pbvi_version;
    }
    const int Mp = (rows + pp2::kGemmTile - 1) / pp2::kGemmTile * pp2::kGemmTile;
    const long long sstride = (long long)Mp * Sp;
    HIPCHK(pp2::launch_gemm_nt(st, d_rows, al, p->d_lbpart, Mp, Sp, p->ref_ld, 1, 0, 0,
                               p->lb_split, sstride));
    HIPCHK(pp2::launch_sum_splits(st, p->d_lbpart, p->lb_split, sstride, (int)sstride,
                                  p->d_lbapprox));
    HIPCHK(hipMemsetAsync(p->d_pcount, 0, sizeof(int), st));
    pp2::PbviCandArgs ca;
    ca.rows = d_rows;
    ca.row_stride = p->ref_ld;
    ca.n = (int)p->n;
    ca.klist = klist;
    ca.kcount = kcount;
    ca.nrows = rows;
    ca.approx = p->d_lbapprox;
    ca.lda = Sp;
    ca.amax = p->d_amax;
    ca.aflag = p->d_aflag;
    ca.S = S;
    // the GEMM's fmaf chains of kchunk terms and its ordered split sum
    // (launch_gemm_nt's kchunk), the reference's chain of n adds, 1 % slack
    const long long kchunk = pp2::gemm_kchunk(p->ref_ld, p->lb_split);
    ca.c_rel = (float)((double)((long long)p->n + kchunk + p->lb_split + 8) * 0x1p-24 * 1.01);
    ca.exact = p->d_lbdots;
    ca.lde = S;
    ca.plist = p->d_plist;
    ca.pcount = p->d_pcount;
    HIPCHK(pp2::launch_pbvi_cands(st, ca));
    pp2::FcArgs a;
    a.n = (int)p->n;
    a.ld = p->ref_ld;
    a.row = d_rows;
    a.row_stride = p->ref_ld;
    a.partners = al;
    a.plist = p->d_plist;
    a.gcount = p->d_pcount;
    a.out = p->d_lbdots;
    a.ldo = S;
    p->scr_pbvi.attach(&a);
    HIPCHK(pp2::launch_fchain(st, pp2::FC_LIST, 0, rows * S, a));
    if (p->h_pstat) {
      HIPCHK(hipMemcpyAsync(p->h_pstat, p->d_pcount, sizeof(int), hipMemcpyDeviceToHost,
                            st));
      ++p->stat_sets;
    }
  } else {
    // one sequential chain per lane (grids whose chain-set scratch is too big)
    HIPCHK(pp2::launch_pair_chain(st, pp2::PAIR_DOT, d_rows, rows, al, S, p->ref_ld,
                                  (int)p->n, p->d_lbdots, S, klist, kcount));
  }
  HIPCHK(pp2::launch_argmax_rows(st, p->d_lbdots, rows, S, S, p->d_lbidx, p->d_lbv));
  return PP2_OK;
}

// evaluatePbviCpu of one dense normalised row into h_lbv[0] (no-op without
// PBVI leaves).  Asynchronous.
int ref_row_pbvi(pp2_planner* p, const float* row) {
  if (!p->pbvi) return PP2_OK;
  if (p->scr_pbvi.chains > 0) {
    // the candidate GEMM reads a whole tile of rows: the row into row 0 of
    // d_children (scratch between expansions)
    HIPCHK(hipMemcpyAsync(p->d_children, row, (size_t)p->ref_ld * sizeof(float),
                          hipMemcpyDeviceToDevice, p->ctx->stream));
    row = p->d_children;
  }
  return ref_pbvi_bounds(p, row, 1);
}

// The VNode constructor's bounds of one dense normalised row
// (search_tree_cuda.cu:368-388): evaluateFibCpu's 9 dots into h_rout[9 ..
// 17], evaluatePbviCpu into h_lbv[0].  Asynchronous.
int ref_row_bounds(pp2_planner* p, const float* row) {
  pp2_ctx* c = p->ctx;
  CHECK(ref_frows(p));
  if (p->seq) {
    HIPCHK(pp2::launch_pair_seq_small(c->stream, pp2::PAIR_DOT, row, 1, p->d_frows, 9, p->ref_ld,
                                      (int)p->n, p->d_rout + 9, 9));
    return ref_row_pbvi(p, row);
  }
  if (p->fx) {
    pp2::FxArgs a;
    a.n = (int)p->n;
    a.ld = p->ref_ld;
    a.row = row;
    a.partners = p->d_frows;
    a.out = p->d_rout + 9;
    a.ldo = 9;
    HIPCHK(pp2::launch_fx(c->stream, pp2::FX_ROW, 9, 1, a));
    return ref_row_pbvi(p, row);
  }
  pp2::FcArgs a;
  a.n = (int)p->n;
  a.ld = p->ref_ld;
  a.row = row;
  a.partners = p->d_frows;
  a.out = p->d_rout + 9;
  a.ldo = 9;
  p->scr_main.attach(&a);
  HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_ROW, 9, 1, a));
  return ref_row_pbvi(p, row);
}

// The children `cs` (c = z * 9 + a) of the expanded belief, normalised, into
// the rows `dst` (the QNode constructor's renormalised child beliefs).
int ref_store_children(pp2_planner* p, const int* cs, float* const* dst, int count) {
  pp2_ctx* c = p->ctx;
  for (int i0 = 0; i0 < count; i0 += 144) {
    pp2::FcStoreList L;
    L.n = std::min(144, count - i0);
    for (int r = 0; r < L.n; ++r) {
      L.child[r] = cs[i0 + r];
      L.dst[r] = dst[i0 + r];
    }
    HIPCHK(pp2::launch_store_children(c->stream, L, p->d_pred, p->d_lrows, p->d_csum, (int)p->n,
                                      p->ref_ld));
  }
  return PP2_OK;
}

// std::max_element of evaluateFibCpu's 9 values (first maximum).
float first_max9(const float* v) {
  float best = v[0];
  for (int i = 1; i < 9; ++i)
    if (best < v[i]) best = v[i];
  return best;
}

// Device copy of a VNode's belief, recomputed from its parent VNode's
// (always materialised: it was expanded) as the QNode constructor's update:
// cudaBayesBeliefUpdate + renormalisation (search_tree_cuda.cu:213-231).
int materialize(pp2_planner* p, VNode* v) {
  if (v->slot >= 0) return PP2_OK;
  if (p->ref)  // every reference-order VNode gets its row when it is created
    return set_err(PP2_ESTATE, "reference-order VNode without a belief row");
  if (!v->parent || !v->parent->parent)
    return set_err(PP2_ESTATE, "cannot materialise a detached VNode");
  VNode* pv = v->parent->parent;
  CHECK(materialize(p, pv));
  int s = -1;
  CHECK(acquire_slot(p, &s));
  pp2_ctx* c = p->ctx;
  const Slot& ps = p->slots[pv->slot];
  const Slot& ns = p->slots[s];
  CHECK(launch_belief(c, ps.b.v.p, ns.b.v.p, v->parent->action, v->observation, ps.mass,
                      p->d_bpart));
  HIPCHK(pp2::launch_sum_finalize(c->stream, p->d_bpart, pp2::mass_partials(c->g, c->cpt),
                                  ns.mass));
  v->slot = s;
  return PP2_OK;
}

// Root VNode from a belief already in slot `s`: FIB/LB evaluation of the
// VNode constructor (search_tree_cuda.cu:368-388).
int make_root(pp2_planner* p, int s, uint8_t z, VNode** out) {
  pp2_ctx* c = p->ctx;
  const Slot& sl = p->slots[s];
  if (p->ref) {
    // the slot's row holds the normalised belief
    CHECK(ref_row_bounds(p, sl.row));
    HIPCHK(hipEventRecord(p->ev_done, c->stream));
    HIPCHK(hipEventSynchronize(p->ev_done));
    if (p->h_pstat) {
      p->stat_cands += *p->h_pstat;
      ++p->stat_rows;
    }
    VNode* v = new_vnode(p, z, 0.0f, nullptr);
    v->slot = s;
    v->upper_bound = first_max9(p->h_rout + 9);
    v->lower_bound = p->pbvi ? p->h_lbv[0] : p->lb_const;
    v->heuristic = v->upper_bound - v->lower_bound;
    *out = v;
    return PP2_OK;
  }
  HIPCHK(pp2::launch_belief_dots(c->stream, c->g, c->cpt, sl.b.v.p, c->fib[c->fcur].v,
                                 p->d_bpart, p->d_out + kOutDots, sl.mass,
                                 p->d_out + kOutMass));
  if (p->pbvi) {
    HIPCHK(pp2::launch_pack(c->stream, c->g, 1, sl.b.v, p->d_children, nullptr));
    CHECK(pbvi_row_max(p, p->d_children, 1));
  }
  HIPCHK(hipEventRecord(p->ev_done, c->stream));
  HIPCHK(hipEventSynchronize(p->ev_done));
  VNode* v = new_vnode(p, z, 0.0f, nullptr);
  v->slot = s;
  v->upper_bound = fib_upper(p->h_out + kOutDots + 1, p->h_out[kOutMass]);
  // evaluatePbviCpu on the normalised belief: max_k <b, alpha_k> / mass
  v->lower_bound = p->pbvi ? p->h_lbv[0] / p->h_out[kOutMass] : p->lb_const;
  v->heuristic = v->upper_bound - v->lower_bound;
  *out = v;
  return PP2_OK;
}

// QNode::forwardSampling + the unique-observation count of the QNode
// constructor (search_tree_cuda.cu:176-196, :311-366) for action a, given
// the fp32 prefix sum `cdf` of the QNode's belief.
void sample_observations(pp2_planner* p, const float* cdf, size_t n, uint8_t a,
                         std::vector<uint8_t>& zs, std::vector<float>& freq) {
  const uint32_t N = p->prm.sample_num;
  std::vector<uint8_t> obs(N);
  for (uint32_t j = 0; j < N; ++j) {
    const float r = (float)p->rng.next() / ((float)RAND_MAX + 1.0f);
    size_t s1 = (size_t)(std::lower_bound(cdf, cdf + n, r) - cdf);
    // find_if(x >= r) runs off the end when rounding leaves cdf.back() < r;
    // the reference then reads past its arrays.  Take the last cell with mass.
    if (s1 >= n) {
      s1 = n - 1;
      while (s1 > 0 && cdf[s1] == cdf[s1 - 1]) --s1;
    }
    float td[9];
    const float* tp = p->hT.data() + s1 * 81 + (size_t)a * 9;
    for (int i = 0; i < 9; ++i) td[i] = tp[i];
    for (int i = 1; i < 9; ++i) td[i] += td[i - 1];
    uint32_t s2i = 0;
    for (uint32_t i = 0; i < 9; ++i)
      if (p->u1[j] <= td[i]) {
        s2i = i;
        break;
      }
    const uint32_t s2 = (uint32_t)s1 + (s2i / 3 - 1) * (uint32_t)p->W + (s2i % 3 - 1);
    float ld[16];
    const float* lp = p->hL.data() + (size_t)s2 * 16;
    for (int i = 0; i < 16; ++i) ld[i] = lp[i];
    for (int i = 1; i < 16; ++i) ld[i] += ld[i - 1];
    uint8_t o = 0;
    for (uint8_t i = 0; i < 16; ++i)
      if (p->u2[j] <= ld[i]) {
        o = i;
        break;
      }
    obs[j] = o;
  }
  std::set<uint8_t> uniq(obs.begin(), obs.end());
  zs.assign(uniq.begin(), uniq.end());
  freq.resize(zs.size());
  for (size_t i = 0; i < zs.size(); ++i)
    freq[i] = (float)std::count(obs.begin(), obs.end(), zs[i]) / (float)N;
}

// VNode::expand (search_tree_cuda.cu:437-450) with the 9 QNode constructors
// (:161-242) batched.
int expand_vnode_ref(pp2_planner* p, VNode* v);

int expand_vnode(pp2_planner* p, VNode* v) {
  if (p->ref) return expand_vnode_ref(p, v);
  pp2_ctx* c = p->ctx;
  CHECK(materialize(p, v));
  const Slot& sl = p->slots[v->slot];
  const size_t n = p->n;
  // normalised belief -> host (for the state samples), then the batched
  // scoring pass runs on the device while the host samples
  HIPCHK(pp2::launch_pack(c->stream, c->g, 1, sl.b.v, p->d_dense, sl.mass, p->d_out + kOutMass));
  HIPCHK(hipEventRecord(p->ev_belief, c->stream));
  HIPCHK(pp2::launch_expand(c->stream, c->g, c->cpt, c->T.v, sl.b.v.p, c->R.v, c->L.v,
                            c->fib[c->fcur].v, p->P.v, p->d_rpart, p->d_spart,
                            p->d_out + kOutRewards, p->d_out + kOutStats));
  if (p->pbvi) {
    HIPCHK(pp2::launch_pack(c->stream, c->g, 1, sl.b.v, p->d_parent, nullptr));
    HIPCHK(pp2::launch_pbvi_update(c->stream, c->g, c->T.v, c->L.v, p->d_parent, p->lb_ld,
                                   p->d_srow, p->d_us, p->d_zs, 144, p->d_children));
    CHECK(pbvi_row_max(p, p->d_children, 144));
  }
  HIPCHK(hipEventRecord(p->ev_done, c->stream));
  HIPCHK(hipEventSynchronize(p->ev_belief));

  p->cdf.build(p->h_belief, n);
  std::vector<uint8_t> zs[9];
  std::vector<float> fq[9];
  for (uint8_t a = 0; a < 9; ++a) sample_observations(p, p->cdf.v.data(), n, a, zs[a], fq[a]);
  HIPCHK(hipEventSynchronize(p->ev_done));

  for (QNode* q : v->children)
    if (q) delete_subtree(p, q);
  v->children.assign(9, nullptr);
  const float mass = p->h_out[kOutMass];
  const float* stats = p->h_out + kOutStats;
  for (uint8_t a = 0; a < 9; ++a) {
    QNode* q = alloc_qnode(p);
    q->action = a;
    q->parent = v;
    q->reward = p->h_out[kOutRewards + a] / mass;
    for (size_t k = 0; k < zs[a].size(); ++k) {
      const uint8_t z = zs[a][k];
      const float* st = stats + ((size_t)z * 9 + a) * kStatsPerChild;
      VNode* cv = new_vnode(p, z, fq[a][k], q);
      cv->upper_bound = fib_upper(st + 1, st[0]);
      cv->lower_bound = p->pbvi ? p->h_lbv[z * 9 + a] / st[0] : p->lb_const;
      cv->heuristic = cv->upper_bound - cv->lower_bound;
      q->children.push_back(cv);
    }
    qnode_update(p, q);
    v->children[a] = q;
  }
  vnode_update(v);
  ++p->expansions;
  return PP2_OK;
}

// PP2_FX_STAMPS: the stamp rows of the four fused kernels of an expansion
// (cdf + samples 1, children 144, rewards 9, kept dots 1296)
constexpr int kFxStampOff[5] = {0, 1, 145, 154, 1450};
constexpr int kFxStampWGs = 1450;

void fx_stamps_collect(pp2_planner* p) {
  std::vector<unsigned long long> h((size_t)kFxStampWGs * 8);
  if (hipMemcpy(h.data(), p->d_stamps, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost) !=
      hipSuccess)
    return;
  for (int k = 0; k < 4; ++k) {
    unsigned long long first = ~0ull, last = 0;
    for (int b = kFxStampOff[k]; b < kFxStampOff[k + 1]; ++b) {
      const unsigned long long* t = &h[(size_t)b * 8];
      if (!t[0]) continue;  // (an inactive workgroup)
      ++p->fx_groups[k];
      const int np = k == 0 ? 6 : 4;
      for (int ph = 0; ph < np; ++ph)
        if (t[ph + 1] >= t[ph]) p->fx_phase[k][ph] += (double)(t[ph + 1] - t[ph]) * 0.01;
      for (int c = 0; c < 4; ++c) p->fx_count[k][c] += (double)((t[7] >> (10 * c)) & 1023u);
      if (k > 0) {  // the walker's shader clocks in steps / fallbacks (k_fx_chain)
        p->fx_phase[k][5] += (double)t[5];
        p->fx_phase[k][6] += (double)t[6];
      }
      first = std::min(first, t[0]);
      last = std::max(last, t[np]);
    }
    if (last > first) p->fx_phase[k][7] += (double)(last - first) * 0.01;
  }
  ++p->fx_sets;
}

void fx_stamps_print(pp2_planner* p) {
  if (!p->d_stamps || !p->fx_sets) return;
  const char* names[4] = {"cdf+samples", "children", "rewards", "kept dots"};
  for (int k = 0; k < 4; ++k) {
    const double g = p->fx_groups[k] ? (double)p->fx_groups[k] : 1.0;
    std::fprintf(stderr,
                 "fx %-11s: %6.1f workgroups/set; per workgroup us: A %.2f B %.2f C %.2f walk %.2f"
                 " cdf %.2f samples %.2f (chains: step / fallback kclk); set span %.2f us; per"
                 " chain: steps %.1f fallbacks %.1f misses %.1f predicted %.1f\n",
                 names[k], g / (double)p->fx_sets, p->fx_phase[k][0] / g, p->fx_phase[k][1] / g,
                 p->fx_phase[k][2] / g, p->fx_phase[k][3] / g,
                 k ? p->fx_phase[k][5] / g / 1e3 : p->fx_phase[k][4] / g,
                 k ? p->fx_phase[k][6] / g / 1e3 : p->fx_phase[k][5] / g,
                 p->fx_phase[k][7] / (double)p->fx_sets,
                 p->fx_count[k][0] / g, p->fx_count[k][1] / g, p->fx_count[k][2] / g,
                 p->fx_count[k][3] / g);
  }
}

// The host's wait for an expansion: a poll of the event (PP2_SPIN_WAIT=1,
// the default) -- the blocking wait's wake-up is a scheduler round trip on
// the plan step's critical path -- or hipEventSynchronize (0).
hipError_t wait_event(pp2_planner* p, hipEvent_t ev) {
  if (!p->spin) return hipEventSynchronize(ev);
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
  }
}

// VNode::expand in reference order.  Every grid-wide sum of the reference's
// 9 QNode constructors (search_tree_cuda.cu:161-242) is formed on the device
// with the bits of its x-ordered fp32 host chain (pp2_fchain.hip), and the
// samples are drawn there with the host's rand() values:
//   side stream: the 9 action predictions, the 144 children's accumulate
//     (:225-227; child (a, z) = cudaBayesBeliefUpdate(b, a, z)), then the 9
//     rewards inner_product(b, R[.][a]) (:168-173);
//   main stream: the expanded belief's running sums (:176-183) and the 9 x N
//     samples (forwardSampling, :311-366) with the kept children; once the
//     masses are in, the kept children normalised (:228-229) into their rows
//     of d_children and their evaluateFibCpu dots (:378).
// One host wait per expansion.  The kept children's rows are stored into
// their nodes' slots afterwards, queued ahead of anything that reads them.
int expand_vnode_ref(pp2_planner* p, VNode* v) {
  pp2_ctx* c = p->ctx;
  if (v->slot < 0) return set_err(PP2_ESTATE, "reference-order VNode without a belief row");
  using clk = std::chrono::steady_clock;
  const clk::time_point t_begin = p->timing ? clk::now() : clk::time_point{};
  if (p->timing && p->t_n > 0)
    p->t_between += std::chrono::duration<double, std::micro>(t_begin - p->t_last_store).count();
  const float* brow = p->slots[v->slot].row;
  const size_t n = p->n;
  const int ld = p->ref_ld;
  const uint32_t N = p->prm.sample_num;
  clk::time_point t_prev = t_begin;
  auto tmark = [&](int i) {  // (PP2_PLAN_TIMING: host time of the enqueue phases)
    if (!p->timing) return;
    const clk::time_point t = clk::now();
    p->t_mark[i] += std::chrono::duration<double, std::micro>(t - t_prev).count();
    t_prev = t;
  };
  auto tev = [&](int i, hipStream_t st) {  // (PP2_PLAN_EVENTS)
    if (p->pev) (void)hipEventRecord(p->tev[i], st);
  };
  CHECK(ref_frows(p));
  // the rand() values of the 9 QNode constructors, in the reference's order
  for (uint32_t a = 0; a < 9; ++a)
    for (uint32_t j = 0; j < N; ++j)
      p->h_r[a * N + j] = (float)p->rng.next() / ((float)RAND_MAX + 1.0f);
  {
    // a row for each of the 144 children, before anything is enqueued (a new
    // chunk of rows is zeroed on the main stream); the kept ones are stored
    // straight into theirs, the others go back after the wait
    p->pre.assign(144, -1);
    for (int cc = 0; cc < 144; ++cc) CHECK(acquire_slot(p, &p->pre[cc]));
  }
  tmark(0);
  // side waits for main's work so far (brow and the previous stores in
  // place) -- unless main is idle (the usual case right after the previous
  // expansion's wait): a stream query costs the host less than the fork
  const hipError_t mq = hipStreamQuery(c->stream);
  if (mq == hipErrorNotReady) {
    HIPCHK(hipEventRecord(p->ev_fork, c->stream));
    HIPCHK(hipStreamWaitEvent(p->side, p->ev_fork, 0));
  } else {
    HIPCHK(mq);
  }
  tmark(1);
  tev(0, c->stream);
  // main: the expanded belief's running sums (cdf chain: tables, walk, cdf,
  // then the samples).  PP2_ROW_FIRST=1 enqueues them first, before the side
  // stream's predictions and children (a rocprofv3 trace shows 30 us less
  // per expansion; without the profiler the plan step is 0.40 against 0.39
  // ms: opt-in, tools/ab_row_first.sh)
  pp2::FcArgs rowc;
  rowc.n = (int)n;
  rowc.ld = ld;
  rowc.row = brow;
  rowc.out = p->d_rsum;
  rowc.cdf = p->d_cdf;
  rowc.sub = p->seq ? nullptr : p->d_sub;  // (the sampler's first search)
  const bool row_first = !p->fx && !p->seq && p->row_first;
  if (!p->fx) p->scr_main.attach(&rowc);
  if (row_first) {
    HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_ROW, 0, 1, rowc, pp2::FC_TABLES));
    HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_ROW, 0, 1, rowc, pp2::FC_DRIVE));
    tev(3, c->stream);
  }
  // The two streams' launches are interleaved phase by phase, so that
  // neither waits for the host to enqueue the other's (a launch costs the
  // host several us): predictions (side), the cdf chain's tables (main), the
  // children's tables (side), the cdf driver and running sums (main), the
  // children's driver (side), the samples (main); the rewards last (side).
  HIPCHK(pp2::launch_tree_pred(p->side, c->g, c->T.v, brow, ld, p->d_pred, tree_sparse_t(c)));
  tev(1, p->side);
  tmark(2);
  if (p->fx) {
    // main: the expanded belief's running sums and the 9 x N samples (one
    // launch); side: the 144 children's masses, then the 9 rewards (a launch
    // each); main: the kept children normalised into their rows and their
    // FIB dots (one launch)
    pp2::FxArgs cd;
    cd.n = (int)n;
    cd.ld = ld;
    cd.row = brow;
    cd.out = p->d_rsum;
    cd.cdf = p->d_cdf;
    if (p->d_stamps) {
      HIPCHK(hipMemsetAsync(p->d_stamps, 0, kFxStampWGs * 8 * sizeof(unsigned long long),
                            c->stream));
      cd.stamps = p->d_stamps + 8 * kFxStampOff[0];
    }
    pp2::SampleArgs sa;
    sa.g = c->g;
    sa.T = c->T.v;
    sa.L = c->L.v;
    sa.n = (int)n;
    sa.N = (int)N;
    sa.r = p->d_r;
    sa.u1 = p->d_u1;
    sa.u2 = p->d_u2;
    sa.counts = p->d_counts;
    sa.klist = p->d_klist;
    sa.kcount = p->d_kcount;
    HIPCHK(pp2::launch_fx_cdf_sample(c->stream, cd, sa));
    pp2::FxArgs ch;
    ch.n = (int)n;
    ch.ld = ld;
    ch.pred = p->d_pred;
    ch.lrows = p->d_lrows;
    ch.out = p->d_csum;
    ch.ldo = 1;
    if (p->d_stamps) ch.stamps = p->d_stamps + 8 * kFxStampOff[1];
    HIPCHK(pp2::launch_fx(p->side, pp2::FX_CHILD, 0, 144, ch));
    HIPCHK(hipEventRecord(p->ev_kids, p->side));
    pp2::FxArgs r;
    r.n = (int)n;
    r.ld = ld;
    r.row = brow;
    r.partners = p->d_rrows;
    r.out = p->d_rout;
    r.ldo = 9;
    if (p->d_stamps) r.stamps = p->d_stamps + 8 * kFxStampOff[2];
    HIPCHK(pp2::launch_fx(p->side, pp2::FX_ROW, 9, 1, r));
    HIPCHK(hipStreamWaitEvent(c->stream, p->ev_kids, 0));
    // the kept children normalised (one division per cell, here only) into
    // their rows of d_children and their node rows, then their FIB dots
    pp2::FcRowTable rt;
    rt.use = 1;
    for (int cc = 0; cc < 144; ++cc) rt.p[cc] = p->slots[p->pre[cc]].row;
    HIPCHK(pp2::launch_store_kept(c->stream, p->d_klist, p->d_kcount, p->d_pred, p->d_lrows,
                                  p->d_csum, p->d_children, (int)n, ld, &rt));
    pp2::FxArgs kd;
    kd.n = (int)n;
    kd.ld = ld;
    kd.row = p->d_children;
    kd.row_stride = ld;
    kd.partners = p->d_frows;
    kd.glist = p->d_klist;
    kd.gcount = p->d_kcount;
    kd.out = p->d_rout + 9;
    kd.ldo = 9;
    if (p->d_stamps) kd.stamps = p->d_stamps + 8 * kFxStampOff[3];
    HIPCHK(pp2::launch_fx(c->stream, pp2::FX_ROW, 9, 144, kd));
    if (p->pbvi) {
      HIPCHK(hipEventRecord(p->ev_kept, c->stream));
      HIPCHK(hipStreamWaitEvent(p->side, p->ev_kept, 0));
      CHECK(ref_pbvi_bounds(p, p->d_children, 144, p->d_klist, p->d_kcount, p->side));
    }
  }
  if (p->seq) {
    // main: the expanded belief's running sums; side: the 144 children's
    // masses, then the 9 rewards -- sequential chains (small grid)
    HIPCHK(pp2::launch_row_cdf_seq(c->stream, brow, (int)n, p->d_cdf, p->d_rsum));
    HIPCHK(pp2::launch_pair_seq_small(p->side, pp2::PAIR_CHILD, p->d_lrows, 16, p->d_pred, 9, ld,
                                      (int)n, p->d_csum, 9));
    HIPCHK(hipEventRecord(p->ev_kids, p->side));
    HIPCHK(pp2::launch_pair_seq_small(p->side, pp2::PAIR_DOT, brow, 1, p->d_rrows, 9, ld, (int)n,
                                      p->d_rout, 9));
  }
  if (!p->fx) {
    pp2::FcArgs& cd = rowc;  // main: the expanded belief's running sums
    pp2::FcArgs ch;  // side: the 144 children's masses
    ch.n = (int)n;
    ch.ld = ld;
    ch.pred = p->d_pred;
    ch.lrows = p->d_lrows;
    ch.out = p->d_csum;
    ch.ldo = 1;
    p->scr_side.attach(&ch);
    // the kept children's FIB dots (evaluateFibCpu) of their normalised rows
    pp2::FcArgs kd;
    kd.n = (int)n;
    kd.ld = ld;
    kd.pred = p->d_pred;
    kd.lrows = p->d_lrows;
    kd.partners = p->d_frows;
    kd.msum = ch.csum;  // (sums: masses from the children's chunk sums)
    kd.out = p->d_rout + 9;
    kd.ldo = 9;
    p->scr_fib.attach(&kd);
    if (!p->seq) {
      // (PP2_KIDS_FIRST=1: each phase's children launch before the cdf
      // chain's)
      const bool kids_first = p->kids_first && !row_first;
      if (!row_first && !kids_first)
        HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_ROW, 0, 1, cd, pp2::FC_TABLES));
      HIPCHK(pp2::launch_fchain(p->side, pp2::FC_CHILD, 0, 144, ch, pp2::FC_TABLES));
      if (!p->fib_unit)
        HIPCHK(hipEventRecord(p->ev_csum, p->side));  // (the children's chunk sums)
      tev(2, p->side);
      if (kids_first) HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_ROW, 0, 1, cd, pp2::FC_TABLES));
      tmark(3);
      if (!row_first && !kids_first) {
        HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_ROW, 0, 1, cd, pp2::FC_DRIVE));
        tev(3, c->stream);
      }
      HIPCHK(pp2::launch_fchain(p->side, pp2::FC_CHILD, 0, 144, ch, pp2::FC_DRIVE));
      tev(4, p->side);
      HIPCHK(hipEventRecord(p->ev_kids, p->side));  // (the children's masses)
      if (kids_first) {
        HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_ROW, 0, 1, cd, pp2::FC_DRIVE));
        tev(3, c->stream);
      }
      tmark(4);
    }
    {
      pp2::SampleArgs sa;
      sa.g = c->g;
      sa.T = c->T.v;
      sa.L = c->L.v;
      sa.cdf = p->d_cdf;
      sa.n = (int)n;
      sa.N = (int)N;
      sa.r = p->d_r;
      sa.u1 = p->d_u1;
      sa.u2 = p->d_u2;
      sa.counts = p->d_counts;
      sa.klist = p->d_klist;
      sa.kcount = p->d_kcount;
      sa.sub = cd.sub;
      sa.cst = cd.cst;
      // (the 144 children's node rows, acquired above, published to the
      // device in the sampler's arguments for the FIB tables that store them)
      pp2::FcRowTable rt;
      rt.use = 1;
      for (int cc = 0; cc < 144; ++cc) rt.p[cc] = p->slots[p->pre[cc]].row;
      if (!p->seq) {
        sa.rows = &rt;
        sa.rows_out = p->d_rowdev;
      }
      HIPCHK(pp2::launch_tree_sample(c->stream, sa));
      tev(5, c->stream);
      tmark(8);
    }
    const bool sumtab = pp2::fc_sumtab_active();
    kd.glist = p->d_klist;
    kd.gcount = p->d_kcount;
    if (!p->seq && !sumtab) {
      // main, beside the children's walk: the kept children's FIB chunk sums
      // (their masses approximated by the children's chunk sums; waiting
      // for the walk here instead, one cross-stream wait fewer, started the
      // sums ~12 us after the samples)
      // (PP2_FIB_UNIT, default: the sums of the unnormalised cells, which
      // need nothing from side -- no cross-stream wait -- and which the
      // tables scale by 1 / mass)
      if (p->fib_unit) {
        kd.kept_unit = 1;
      } else {
        HIPCHK(hipStreamWaitEvent(c->stream, p->ev_csum, 0));
      }
      HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_KEPT, 9, 144, kd, pp2::FC_SUMS));
      tev(6, c->stream);
    }
    // (side: the 9 rewards, off the critical path, are enqueued after the
    // kept children's FIB launches: each launch ahead of those costs the
    // critical chain its host time)
    tmark(5);
    HIPCHK(hipStreamWaitEvent(c->stream, p->ev_kids, 0));
    // the node rows acquired for the 144 children: the kept ones are stored
    // straight into theirs
    for (int cc = 0; cc < 144; ++cc) p->h_rowptr[cc] = p->slots[p->pre[cc]].row;
    if (p->seq) {
      // main: the kept children (sampled on this stream), normalised by their
      // masses (side) into their rows of d_children and their node rows
      pp2::FcRowTable rt;
      rt.use = 1;
      for (int cc = 0; cc < 144; ++cc) rt.p[cc] = p->h_rowptr[cc];
      HIPCHK(pp2::launch_store_kept(c->stream, p->d_klist, p->d_kcount, p->d_pred, p->d_lrows,
                                    p->d_csum, p->d_children, (int)n, ld, &rt));
    } else {
      // main: the kept children's FIB tables -- which store their normalised
      // rows (d_children, node rows) on the way -- then their walk
      // (with k_fc_sumtab: the sums too, in the same launch, exact masses)
      kd.mass = p->d_csum;
      kd.kept_rows = p->d_children;
      kd.rowptr = p->d_rowdev;
      // only the first maximum of a child's 9 dots is kept: the chains
      // certainly below another (their sums against the exact masses) are
      // neither tabled nor walked (-inf)
      if (p->fib_cands && !sumtab) {
        HIPCHK(pp2::launch_fib_cands(c->stream, kd, p->d_cmask));
        kd.cmask = p->d_cmask;
      }
      HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_KEPT, 9, 144, kd,
                                sumtab ? pp2::FC_TABLES : pp2::FC_TAB));
      tev(7, c->stream);
    }
    tmark(6);
    // the kept children's rows are in place: their PBVI dots (evaluatePbviCpu,
    // the long chains) may start on side
    if (p->pbvi) HIPCHK(hipEventRecord(p->ev_kept, c->stream));
    if (p->seq) {  // main: the kept children's FIB dots (evaluateFibCpu), sequential chains
      HIPCHK(pp2::launch_pair_seq_small(c->stream, pp2::PAIR_DOT, p->d_children, 144, p->d_frows, 9,
                                        ld, (int)n, p->d_rout + 9, 9, p->d_klist, p->d_kcount));
    } else {
      HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_KEPT, 9, 144, kd, pp2::FC_DRIVE));
      tev(8, c->stream);
      // side: the 9 rewards inner_product(b, R[.][a])
      pp2::FcArgs r;
      r.n = (int)n;
      r.ld = ld;
      r.row = brow;
      r.partners = p->d_rrows;
      r.out = p->d_rout;
      r.ldo = 9;
      p->scr_rew.attach(&r);
      HIPCHK(pp2::launch_fchain(p->side, pp2::FC_ROW, 9, 1, r));
      tev(9, p->side);
    }
    // side: the PBVI dots, beside main's FIB dots
    if (p->pbvi) {
      HIPCHK(hipStreamWaitEvent(p->side, p->ev_kept, 0));
      CHECK(ref_pbvi_bounds(p, p->d_children, 144, p->d_klist, p->d_kcount, p->side));
    }
  }  // (!p->fx)
  HIPCHK(hipEventRecord(p->ev_join, p->side));  // (the rewards, the PBVI dots)
  // (PP2_HOST_JOIN, default: the host waits for both streams' last events;
  // else main waits for side's on the device, one cross-stream wait more)
  if (!p->host_join) HIPCHK(hipStreamWaitEvent(c->stream, p->ev_join, 0));
  HIPCHK(hipEventRecord(p->ev_done, c->stream));
  tmark(7);
  const clk::time_point t_enq = p->timing ? clk::now() : clk::time_point{};
  HIPCHK(wait_event(p, p->ev_done));
  if (p->host_join) HIPCHK(wait_event(p, p->ev_join));
  const clk::time_point t_ret = p->timing ? clk::now() : clk::time_point{};
  // the device-written host rows (counts, rewards and FIB dots, PBVI bounds)
  // are cache misses: request every line at once, not one miss at a time
  // in the loop below
  for (int i = 0; i < 144; i += 16) __builtin_prefetch(p->h_counts + i);
  for (int i = 0; i < kRefOutFloats; i += 16) __builtin_prefetch(p->h_rout + i);
  if (p->pbvi)
    for (int i = 0; i < 144; i += 16) __builtin_prefetch(p->h_lbv + i);
  if (p->h_pstat) p->stat_cands += *p->h_pstat;
  if (p->d_stamps) fx_stamps_collect(p);
  if (p->pev && !p->fx && !p->seq) {
    for (int i = 1; i < 10; ++i) {
      float ms = 0.0f;
      if (hipEventElapsedTime(&ms, p->tev[0], p->tev[i]) == hipSuccess) p->tev_sum[i] += 1e3 * ms;
    }
    ++p->tev_n;
  }
  if (p->timing) {
    volatile float sink = p->h_rout[9 + 9 * 143] + (float)p->h_counts[143];
    (void)sink;
    p->t_pa += std::chrono::duration<double, std::micro>(clk::now() - t_ret).count();
  }

  for (QNode* q : v->children)
    if (q) delete_subtree(p, q);
  v->children.assign(9, nullptr);
  long long kept = 0;
  for (uint8_t a = 0; a < 9; ++a) {
    QNode* q = alloc_qnode(p);
    q->action = a;
    q->parent = v;
    q->reward = p->h_rout[a];
    int nk = 0;
    for (uint8_t z = 0; z < 16; ++z) nk += p->h_counts[a * 16 + z] != 0;
    q->children.reserve(nk);  // (one allocation, not a growth sequence)
    for (uint8_t z = 0; z < 16; ++z) {  // std::set order
      const int cnt = p->h_counts[a * 16 + z];
      if (!cnt) continue;
      const int row = z * 9 + a;
      VNode* cv = new_vnode(p, z, (float)cnt / (float)N, q);
      ++kept;
      cv->upper_bound = first_max9(p->h_rout + 9 + 9 * row);
      cv->lower_bound = p->pbvi ? p->h_lbv[row] : p->lb_const;
      cv->heuristic = cv->upper_bound - cv->lower_bound;
      cv->slot = p->pre[row];  // (its row is stored there already)
      p->pre[row] = -1;
      q->children.push_back(cv);
    }
    qnode_update(p, q);
    v->children[a] = q;
  }
  if (p->timing) p->t_pb += std::chrono::duration<double, std::micro>(clk::now() - t_ret).count();
  for (int& sl : p->pre) {  // the rows of the children not kept go back
    if (sl >= 0) release_slot(p, sl);
    sl = -1;
  }
  p->stat_rows += kept;
  vnode_update(v);
  ++p->expansions;
  if (p->timing) {
    p->t_last_store = clk::now();
    p->t_enq += std::chrono::duration<double, std::micro>(t_enq - t_begin).count();
    p->t_post += std::chrono::duration<double, std::micro>(p->t_last_store - t_ret).count();
    ++p->t_n;
  }
  return PP2_OK;
}

// SearchTree::expand (search_tree_cuda.cu:490-508)
int tree_expand(pp2_planner* p) {
  VNode* vte = p->root->vnode_to_expand;
  if (!vte)
    return set_err(PP2_ESTATE, "no expandable node (all heuristics are zero)");
  CHECK(expand_vnode(p, vte));
  VNode* v = vte;
  while (v->parent != nullptr) {
    QNode* q = v->parent;
    qnode_update(p, q);
    VNode* pv = q->parent;
    vnode_update(pv);
    v = pv;
  }
  return PP2_OK;
}

// SearchTree::update (search_tree_cuda.cu:548-626)
int tree_update(pp2_planner* p, uint8_t a, uint8_t z) {
  VNode* root = p->root;
  QNode* root_q = nullptr;
  for (QNode* q : root->children) {
    if (q->action == a) root_q = q;
    else delete_subtree(p, q);
  }
  root->children.clear();
  VNode* root_v = nullptr;
  if (root_q) {
    for (VNode* v : root_q->children) {
      if (v->observation == z) root_v = v;
      else delete_subtree(p, v);
    }
    root_q->children.clear();
  }
  if (root_v) {
    CHECK(materialize(p, root_v));  // from the old root, before it goes
    delete_qnode_only(p, root_q);
    delete_vnode_only(p, root);
    root_v->parent = nullptr;
    p->root = root_v;
    return PP2_OK;
  }
  // No such child (or the root was never expanded -- the reference
  // dereferences a null QNode there): a fresh root from the updated belief.
  int s = -1;
  CHECK(acquire_slot(p, &s));
  pp2_ctx* c = p->ctx;
  const Slot& os = p->slots[root->slot];
  const Slot& ns = p->slots[s];
  if (p->ref) {
    // (search_tree_cuda.cu:586-612) update, accumulate, divide: the child
    // (a, z) of the old root's row, as an expansion forms it
    const int cz = z * 9 + a;
    HIPCHK(pp2::launch_tree_pred(c->stream, c->g, c->T.v, os.row, p->ref_ld, p->d_pred,
                                 tree_sparse_t(c)));
    if (p->seq) {
      HIPCHK(pp2::launch_pair_seq_small(c->stream, pp2::PAIR_CHILD,
                                        p->d_lrows + (size_t)z * p->ref_ld, 1,
                                        p->d_pred + (size_t)a * p->ref_ld, 1, p->ref_ld, (int)p->n,
                                        p->d_csum + cz, 1));
    } else if (p->fx) {
      pp2::FxArgs fa;
      fa.n = (int)p->n;
      fa.ld = p->ref_ld;
      fa.pred = p->d_pred;
      fa.lrows = p->d_lrows;
      fa.g0 = cz;
      fa.out = p->d_csum;
      fa.ldo = 1;
      HIPCHK(pp2::launch_fx(c->stream, pp2::FX_CHILD, 0, 1, fa));
    } else {
      pp2::FcArgs fa;
      fa.n = (int)p->n;
      fa.ld = p->ref_ld;
      fa.pred = p->d_pred;
      fa.lrows = p->d_lrows;
      fa.g0 = cz;
      fa.out = p->d_csum;
      fa.ldo = 1;
      p->scr_main.attach(&fa);
      HIPCHK(pp2::launch_fchain(c->stream, pp2::FC_CHILD, 0, 1, fa));
    }
    float* dst = ns.row;
    CHECK(ref_store_children(p, &cz, &dst, 1));
  } else {
    CHECK(launch_belief(c, os.b.v.p, ns.b.v.p, a, z, os.mass, p->d_bpart));
    HIPCHK(pp2::launch_sum_finalize(c->stream, p->d_bpart, pp2::mass_partials(c->g, c->cpt),
                                    ns.mass));
  }
  VNode* nv = nullptr;
  CHECK(make_root(p, s, 0, &nv));
  if (root_q) delete_qnode_only(p, root_q);
  delete_vnode_only(p, root);
  p->root = nv;
  return PP2_OK;
}

}  // namespace

extern "C" {

int pp2_planner_default_params(pp2_planner_params* prm) {
  if (!prm) return set_err(PP2_EINVAL, "params is null");
  prm->max_search_tree_depth = 50;
  prm->max_online_iteration = 15;
  prm->lower_bound_mode = 0;
  prm->rand_seed = 1;
  prm->rand_skip = 0;
  prm->sample_num = 50;
  prm->curand_seed = 1234;
  prm->reference_order = 1;  // bit-exact with the reference's host arithmetic (the drop-in)
  return PP2_OK;
}

int pp2_curand_uniforms(uint64_t seed, int n, float* u1, float* u2) {
  if (n < 0 || (n > 0 && (!u1 || !u2))) return set_err(PP2_EINVAL, "bad arguments");
  for (int i = 0; i < n; ++i) {
    CurandXorwow g(seed, (uint64_t)i);
    u1[i] = curand_uniform_of(g.next());
    u2[i] = curand_uniform_of(g.next());
  }
  return PP2_OK;
}

int pp2_planner_destroy(pp2_planner* p);

int pp2_planner_create(pp2_planner** out, pp2_ctx* c, const pp2_planner_params* prm) {
  if (!out) return set_err(PP2_EINVAL, "out is null");
  *out = nullptr;
  CHECK(check_model(c));
  if (c->nranks > 1 || c->g.rows != c->g.grows)
    return set_err(PP2_EINVAL, "the QV-tree planner needs an unsharded context");
  pp2_planner_params d;
  pp2_planner_default_params(&d);
  if (!prm) prm = &d;
  if (prm->lower_bound_mode != 0 && prm->lower_bound_mode != 1)
    return set_err(PP2_EINVAL, "lower_bound_mode %d not supported (0 = constant, 1 = PBVI)",
                   prm->lower_bound_mode);
  const float* pal = nullptr;
  int pS = 0, pSp = 0, pld = 0;
  if (prm->lower_bound_mode == 1 && pbvi_alphas(c, &pal, &pS, &pSp, &pld) != PP2_OK)
    return set_err(PP2_ESTATE, "lower_bound_mode 1 needs PBVI alpha vectors (pp2_pbvi_solve "
                   "or pp2_pbvi_set)");
  if (prm->sample_num == 0) return set_err(PP2_EINVAL, "sample_num must be > 0");
  if (prm->reference_order != 0 && prm->reference_order != 1)
    return set_err(PP2_EINVAL, "reference_order must be 0 or 1");
  DeviceGuard dg(c->device);
  pp2_planner* p = new pp2_planner();
  p->ctx = c;
  p->prm = *prm;
  p->gamma = c->gamma;
  // search_tree_cuda.cu:383 (commented fallback): -5.0f / (1.0f - gamma)
  p->lb_const = -5.0f / (1.0f - p->gamma);
  p->W = c->g.width;
  p->n = owned_cells(c);
  auto fail = [&](int s) {
    pp2_planner_destroy(p);
    return s;
  };
  p->hT.resize(p->n * 81);
  p->hL.resize(p->n * 16);
  int s = pp2_model_download(c, p->hT.data(), p->hL.data(), nullptr, nullptr);
  if (s) return fail(s);
  p->u1.resize(prm->sample_num);
  p->u2.resize(prm->sample_num);
  pp2_curand_uniforms(prm->curand_seed, (int)prm->sample_num, p->u1.data(), p->u2.data());
  {
    const char* e = getenv("PP2_CDF_SKIP");
    p->cdf.skip = !(e && e[0] == '0');
  }
  p->rng.seed(prm->rand_seed);
  for (uint64_t k = 0; k < prm->rand_skip; ++k) (void)p->rng.next();
  const int tiles1 = pp2::cells_grid(c->g, 1);
  if ((s = alloc_planes(c, &p->P, 9))) return fail(s);
  if (hipMalloc(&p->d_rpart, (size_t)tiles1 * 9 * sizeof(float)) != hipSuccess ||
      hipMalloc(&p->d_spart, (size_t)tiles1 * kStatsFloats * sizeof(float)) != hipSuccess ||
      hipMalloc(&p->d_bpart, (size_t)(tiles1 + 1) * kStatsPerChild * sizeof(float)) != hipSuccess ||
      !host_mapped(kOutFloats, &p->h_out, &p->d_out) ||
      !host_mapped(p->n, &p->h_belief, &p->d_dense) ||
      hipEventCreateWithFlags(&p->ev_belief, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_kids, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_kept, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_csum, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_fsum, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&p->side, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&p->side2, hipStreamNonBlocking) != hipSuccess)
    return fail(set_err(PP2_ENOMEM, "planner scratch allocation failed"));
  p->ref = prm->reference_order == 1;
  {
    const char* e = getenv("PP2_SEQ_CHAIN_MAX");
    const long long lim = e && *e ? atoll(e) : kSeqChainMax;
    p->seq = p->ref && (long long)p->n <= lim;
  }
  // dense rows of the children / PBVI / reference-order passes: the PBVI
  // alphas' row length, else the cells rounded up to 64
  const int row_ld = prm->lower_bound_mode == 1 ? pld : (int)((p->n + 63) / 64 * 64);
  p->ref_ld = row_ld;
  {
    const char* e = getenv("PP2_FX");
    // (opt-in: on the 256^2 plan step the fused sets run 0.56-0.57 ms p50
    // against 0.45-0.47 for the three-launch sets with k_fc_walk,
    // tools/ab_planner.sh)
    p->fx = p->ref && !p->seq && pp2::fx_fits((int)p->n, row_ld) && e && e[0] == '1';
    const char* d = getenv("PP2_FX_STAMPS");
    if (p->fx && d && d[0] == '1' &&
        hipMalloc(&p->d_stamps, kFxStampWGs * 8 * sizeof(unsigned long long)) != hipSuccess)
      return fail(set_err(PP2_ENOMEM, "planner stamps allocation failed"));
  }
  if (prm->lower_bound_mode == 1) {
    p->pbvi = true;
    p->lb_S = pS;
    p->lb_Sp = pSp;
    p->lb_ld = pld;
    // split x so that the 144-row product fills the chip (>= 768 workgroups)
    const int tiles = (256 / pp2::kGemmTile) * (pSp / pp2::kGemmTile);
    p->lb_split = std::max(1, std::min((768 + tiles - 1) / tiles, pld / 64));
    const size_t rows = (size_t)256 * pld, dots = (size_t)256 * pSp;
    std::vector<int> srow(144, 0);
    std::vector<uint8_t> us(144), zs(144);
    for (int k = 0; k < 144; ++k) {
      us[k] = (uint8_t)(k % 9);
      zs[k] = (uint8_t)(k / 9);
    }
    if (hipMalloc(&p->d_parent, (size_t)pld * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_children, rows * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_lbpart, (size_t)p->lb_split * dots * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_lbdots, dots * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_lbidx, 256 * sizeof(int)) != hipSuccess ||
        hipMalloc(&p->d_srow, 144 * sizeof(int)) != hipSuccess ||
        hipMalloc(&p->d_us, 144) != hipSuccess || hipMalloc(&p->d_zs, 144) != hipSuccess ||
        !host_mapped(256, &p->h_lbv, &p->d_lbv))
      return fail(set_err(PP2_ENOMEM, "planner PBVI scratch allocation failed"));
    if (hipMemsetAsync(p->d_parent, 0, (size_t)pld * sizeof(float), c->stream) != hipSuccess ||
        hipMemsetAsync(p->d_children, 0, rows * sizeof(float), c->stream) != hipSuccess ||
        hipMemcpyAsync(p->d_srow, srow.data(), 144 * sizeof(int), hipMemcpyHostToDevice,
                       c->stream) != hipSuccess ||
        hipMemcpyAsync(p->d_us, us.data(), 144, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(p->d_zs, zs.data(), 144, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return fail(set_err(PP2_EHIP, "planner PBVI scratch initialisation failed"));
  }
  if (p->ref) {
    const size_t rows = (size_t)256 * row_ld;
    if ((!p->d_parent && hipMalloc(&p->d_parent, (size_t)row_ld * sizeof(float)) != hipSuccess) ||
        (!p->d_children && hipMalloc(&p->d_children, rows * sizeof(float)) != hipSuccess) ||
        (!p->d_srow && hipMalloc(&p->d_srow, 144 * sizeof(int)) != hipSuccess) ||
        (!p->d_us && hipMalloc(&p->d_us, 144) != hipSuccess) ||
        (!p->d_zs && hipMalloc(&p->d_zs, 144) != hipSuccess) ||
        hipMalloc(&p->d_rrows, (size_t)9 * row_ld * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_frows, (size_t)9 * row_ld * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_rsum, 256 * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_lrows, (size_t)16 * row_ld * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_pred, (size_t)9 * row_ld * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_csum, 144 * sizeof(float)) != hipSuccess ||
        !host_mapped(kRefOutFloats, &p->h_rout, &p->d_rout) ||
        hipMalloc(&p->d_cdf, (size_t)row_ld * sizeof(float)) != hipSuccess ||
        (p->n <= 65536 && hipMalloc(&p->d_sub, (p->n + 15) / 16 * sizeof(float)) != hipSuccess) ||
        !host_mapped(9 * (size_t)prm->sample_num, &p->h_r, &p->d_r) ||
        hipMalloc(&p->d_u1, (size_t)prm->sample_num * sizeof(float)) != hipSuccess ||
        hipMalloc(&p->d_u2, (size_t)prm->sample_num * sizeof(float)) != hipSuccess ||
        !host_mapped(144, reinterpret_cast<float**>(&p->h_counts),
                     reinterpret_cast<float**>(&p->d_counts)) ||
        hipMalloc(&p->d_klist, 144 * sizeof(int)) != hipSuccess ||
        hipMalloc(&p->d_kcount, sizeof(int)) != hipSuccess ||
        !p->scr_main.reserve((int)p->n, 144 * 9) || !p->scr_side.reserve((int)p->n, 144) ||
        !p->scr_fib.reserve((int)p->n, 144 * 9) || !p->scr_rew.reserve((int)p->n, 9) ||
        !host_mapped(2 * 144, reinterpret_cast<float**>(&p->h_rowptr),
                     reinterpret_cast<float**>(&p->d_rowptr)) ||
        hipMalloc(&p->d_rowdev, 144 * sizeof(float*)) != hipSuccess ||
        hipMalloc(&p->d_cmask, 144 * sizeof(uint16_t)) != hipSuccess)
      return fail(set_err(PP2_ENOMEM, "planner reference-order scratch allocation failed"));
    std::vector<int> srow(144, 0);
    std::vector<uint8_t> us(144), zs(144);
    for (int k = 0; k < 144; ++k) {
      us[k] = (uint8_t)(k % 9);
      zs[k] = (uint8_t)(k / 9);
    }
    if (hipMemsetAsync(p->d_parent, 0, (size_t)row_ld * sizeof(float), c->stream) != hipSuccess ||
        hipMemsetAsync(p->d_children, 0, rows * sizeof(float), c->stream) != hipSuccess ||
        hipMemsetAsync(p->d_rrows, 0, (size_t)9 * row_ld * sizeof(float), c->stream) !=
            hipSuccess ||
        hipMemsetAsync(p->d_frows, 0, (size_t)9 * row_ld * sizeof(float), c->stream) !=
            hipSuccess ||
        hipMemcpyAsync(p->d_srow, srow.data(), 144 * sizeof(int), hipMemcpyHostToDevice,
                       c->stream) != hipSuccess ||
        hipMemcpyAsync(p->d_us, us.data(), 144, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(p->d_zs, zs.data(), 144, hipMemcpyHostToDevice, c->stream) != hipSuccess)
      return fail(set_err(PP2_EHIP, "planner reference-order scratch initialisation failed"));
    if (hipMemsetAsync(p->d_lrows, 0, (size_t)16 * row_ld * sizeof(float), c->stream) !=
            hipSuccess ||
        hipMemsetAsync(p->d_pred, 0, (size_t)9 * row_ld * sizeof(float), c->stream) != hipSuccess)
      return fail(set_err(PP2_EHIP, "planner reference-order scratch initialisation failed"));
    if (hipMemcpyAsync(p->d_u1, p->u1.data(), p->u1.size() * sizeof(float),
                       hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(p->d_u2, p->u2.data(), p->u2.size() * sizeof(float),
                       hipMemcpyHostToDevice, c->stream) != hipSuccess)
      return fail(set_err(PP2_EHIP, "planner reference-order scratch initialisation failed"));
    if ((s = pack_rows(p, c->R.v, 9, p->d_rrows))) return fail(s);
    if ((s = pack_rows(p, c->L.v, 16, p->d_lrows))) return fail(s);
    if ((s = grow_ref_slots(p))) return fail(s);  // the first chunk of node rows
    if (p->pbvi) {
      // opt-in (PP2_PBVI_FCHAIN=1): the PBVI leaf bounds' candidate chain
      // set, scratch for every (row, alpha) pair when that stays <= 1 GiB
      // (12 B per chain and chunk).  Default: the lane-per-chain pair chains
      // (measured faster: PBVI alphas lie so close together that 50-300 of
      // 500 stay candidates per row)
      const long long chains = 144LL * p->lb_S;
      const long long bytes = chains * pp2::fc_chunks((int)p->n) * 12LL;
      const char* e = getenv("PP2_PBVI_FCHAIN");
      if (e && e[0] == '1' && bytes <= (1LL << 30)) {
        if (!p->scr_pbvi.reserve((int)p->n, (int)chains) ||
            hipMalloc(&p->d_lbapprox, (size_t)256 * p->lb_Sp * sizeof(float)) != hipSuccess ||
            hipMalloc(&p->d_amax, (size_t)p->lb_Sp * sizeof(float)) != hipSuccess ||
            hipMalloc(&p->d_aflag, (size_t)p->lb_Sp * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&p->d_plist, (size_t)chains * sizeof(int2)) != hipSuccess ||
            hipMalloc(&p->d_pcount, sizeof(int)) != hipSuccess)
          return fail(set_err(PP2_ENOMEM, "planner PBVI chain scratch allocation failed"));
        const char* st = getenv("PP2_PBVI_STATS");
        if (st && st[0] == '1' && hipHostMalloc((void**)&p->h_pstat, sizeof(int)) != hipSuccess)
          return fail(set_err(PP2_ENOMEM, "planner stats allocation failed"));
      }
    }
  }
  {
    const char* tm = getenv("PP2_PLAN_TIMING");
    p->timing = tm && tm[0] == '1';
    const char* sw = getenv("PP2_SPIN_WAIT");
    p->spin = !(sw && sw[0] == '0');
    const char* fc = getenv("PP2_FIB_CANDS");
    p->fib_cands = fc && fc[0] == '1';
    const char* pe = getenv("PP2_PLAN_EVENTS");
    if (pe && pe[0] == '1') {
      p->pev = true;
      for (hipEvent_t& e : p->tev)
        if (hipEventCreate(&e) != hipSuccess) return fail(set_err(PP2_EHIP, "planner timing events"));
    }
    const char* fu = getenv("PP2_FIB_UNIT");
    p->fib_unit = !(fu && fu[0] == '0');
    const char* hj = getenv("PP2_HOST_JOIN");
    p->host_join = !(hj && hj[0] == '0');
    const char* kf = getenv("PP2_KIDS_FIRST");
    p->kids_first = kf && kf[0] == '1';
    const char* rf = getenv("PP2_ROW_FIRST");
    p->row_first = rf && rf[0] == '1';
  }
  *out = p;
  return PP2_OK;
}

int pp2_planner_reset(pp2_planner* p) {
  if (!p) return set_err(PP2_EINVAL, "null planner");
  if (p->root) delete_subtree(p, p->root);
  p->root = nullptr;
  return PP2_OK;
}

int pp2_planner_destroy(pp2_planner* p) {
  if (!p) return PP2_OK;
  DeviceGuard dg(p->ctx->device);
  (void)hipStreamSynchronize(p->ctx->stream);
  fx_stamps_print(p);
  if (p->d_stamps) (void)hipFree(p->d_stamps);
  pp2_planner_reset(p);
  for (VNode* v : p->vpool) delete v;
  for (QNode* q : p->qpool) delete q;
  for (Slot& s : p->slots) {
    free_planes(&s.b);
    if (s.mass && !p->ref) (void)hipFree(s.mass);
  }
  for (void* a : p->arenas) (void)hipFree(a);
  free_planes(&p->P);
  for (float* d : {p->d_rpart, p->d_spart, p->d_bpart, p->d_parent, p->d_children,
                   p->d_lbpart, p->d_lbdots, p->d_rrows, p->d_frows, p->d_rsum, p->d_lrows,
                   p->d_pred, p->d_csum, p->d_lbapprox, p->d_amax})
    if (d) (void)hipFree(d);
  for (void* d : {(void*)p->d_aflag, (void*)p->d_plist, (void*)p->d_pcount, (void*)p->d_rowdev,
                   (void*)p->d_cmask})
    if (d) (void)hipFree(d);
  if (p->pev && p->tev_n > 0) {
    static const char* names[10] = {"start", "pred", "children tables", "row walk+cdf",
                                    "children walk", "sample", "FIB sums", "FIB tables",
                                    "FIB walk", "rewards"};
    fprintf(stderr, "pp2 planner: device us from an expansion's start (main), mean of %lld:",
            p->tev_n);
    for (int i = 1; i < 10; ++i) fprintf(stderr, " %s %.1f;", names[i], p->tev_sum[i] / p->tev_n);
    fprintf(stderr, "\n");
  }
  for (hipEvent_t e : p->tev)
    if (e) (void)hipEventDestroy(e);
  if (p->timing && p->t_n > 0)
    fprintf(stderr, "pp2 planner: %lld expansions, host us per expansion: enqueue %.1f, "
            "after the wait .. children stored %.1f, .. next expansion %.1f; kept children "
            "per expansion %.1f (after the wait: first rows read %.1f, nodes built %.1f)\n",
            p->t_n, p->t_enq / p->t_n, p->t_post / p->t_n,
            p->t_between / (p->t_n > 1 ? p->t_n - 1 : 1), (double)p->stat_rows / (double)p->t_n,
            p->t_pa / p->t_n, p->t_pb / p->t_n);
  if (p->timing && p->t_steps > 1)
    fprintf(stderr, "pp2 planner: per plan step us: entry .. first expansion %.1f, last "
            "expansion .. return %.1f, the caller between steps %.1f\n", p->t_upd / p->t_steps,
            p->t_tail / p->t_steps, p->t_out / (p->t_steps - 1));
  if (p->timing && p->t_n > 0)
    fprintf(stderr, "pp2 planner: enqueue phases us: rand+slots %.1f, fork %.1f, pred %.1f, tables "
            "%.1f, drives %.1f, sample %.1f, FIB sums %.1f, FIB tables %.1f, FIB walk+rewards+join "
            "%.1f\n",
            p->t_mark[0] / p->t_n, p->t_mark[1] / p->t_n, p->t_mark[2] / p->t_n,
            p->t_mark[3] / p->t_n, p->t_mark[4] / p->t_n, p->t_mark[8] / p->t_n,
            p->t_mark[5] / p->t_n, p->t_mark[6] / p->t_n, p->t_mark[7] / p->t_n);
  if (p->h_pstat) {
    if (p->stat_sets > 0)
      fprintf(stderr, "pp2 planner: PBVI candidate chains %lld over %lld rows in %lld sets "
              "(%.2f per row of %d alphas)\n", p->stat_cands, p->stat_rows, p->stat_sets,
              p->stat_rows ? (double)p->stat_cands / (double)p->stat_rows : 0.0, p->lb_S);
    (void)hipHostFree(p->h_pstat);
  }
  if (p->h_rout) (void)hipHostFree(p->h_rout);
  if (p->h_r) (void)hipHostFree(p->h_r);
  if (p->h_counts) (void)hipHostFree(p->h_counts);
  if (p->h_rowptr) (void)hipHostFree(p->h_rowptr);
  for (void* d : {(void*)p->d_cdf, (void*)p->d_sub, (void*)p->d_u1, (void*)p->d_u2, (void*)p->d_klist,
                  (void*)p->d_kcount})
    if (d) (void)hipFree(d);
  for (void* d : {(void*)p->d_lbidx, (void*)p->d_srow, (void*)p->d_us, (void*)p->d_zs})
    if (d) (void)hipFree(d);
  if (p->h_lbv) (void)hipHostFree(p->h_lbv);
  if (p->h_out) (void)hipHostFree(p->h_out);
  if (p->h_belief) (void)hipHostFree(p->h_belief);
  if (p->ev_belief) (void)hipEventDestroy(p->ev_belief);
  if (p->ev_done) (void)hipEventDestroy(p->ev_done);
  for (hipEvent_t e : {p->ev_fork, p->ev_join, p->ev_kids, p->ev_kept, p->ev_csum, p->ev_fsum})
    if (e) (void)hipEventDestroy(e);
  for (hipStream_t st : {p->side, p->side2}) {
    if (!st) continue;
    (void)hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
  }
  delete p;
  return PP2_OK;
}

int pp2_planner_step(pp2_planner* p, uint8_t action, uint8_t observation,
                     const float* belief, uint8_t* new_action, float* new_value) {
  if (!p) return set_err(PP2_EINVAL, "null planner");
  using clk = std::chrono::steady_clock;
  const clk::time_point t_in = p->timing ? clk::now() : clk::time_point{};
  if (p->timing && p->t_steps > 0)
    p->t_out += std::chrono::duration<double, std::micro>(t_in - p->t_ret_step).count();
  pp2_ctx* c = p->ctx;
  DeviceGuard dg(c->device);
  if (!p->root) {
    if (!belief) return set_err(PP2_EINVAL, "first plan step needs a belief");
    // new SearchTree(msg->belief) (path_planning_2d.cu:212-213)
    int s = -1;
    CHECK(acquire_slot(p, &s));
    if (p->ref)
      HIPCHK(hipMemcpyAsync(p->slots[s].row, belief, p->n * sizeof(float), hipMemcpyHostToDevice,
                            c->stream));
    else
      CHECK(upload_planes(c, p->slots[s].b, belief));
    const float one = 1.0f;
    HIPCHK(hipMemcpyAsync(p->slots[s].mass, &one, sizeof one, hipMemcpyHostToDevice, c->stream));
    CHECK(make_root(p, s, 0, &p->root));
  } else {
    if (action > 8 || observation > 15)
      return set_err(PP2_EINVAL, "action %u / observation %u out of range", action, observation);
    CHECK(tree_update(p, action, observation));
  }
  // while (getDepth() < max_search_tree_depth &&
  //        update_counter++ < max_online_iteration) expand();   (:219-223)
  int counter = 0;
  if (p->timing) p->t_upd += std::chrono::duration<double, std::micro>(clk::now() - t_in).count();
  while (p->root->depth < (uint32_t)p->prm.max_search_tree_depth &&
         counter++ < p->prm.max_online_iteration)
    CHECK(tree_expand(p));
  const clk::time_point t_loop = p->timing ? clk::now() : clk::time_point{};
  // SearchTree::getOptimalAction (search_tree_cuda.cu:510-524)
  uint8_t a = 0;
  float r = -FLT_MAX;
  for (const QNode* q : p->root->children)
    if (q->upper_bound > r) {
      r = q->upper_bound;
      a = q->action;
    }
  if (new_action) *new_action = a;
  if (new_value) *new_value = r;
  if (p->timing) {
    p->t_ret_step = clk::now();
    p->t_tail += std::chrono::duration<double, std::micro>(p->t_ret_step - t_loop).count();
    ++p->t_steps;
  }
  return PP2_OK;
}

int pp2_planner_info(pp2_planner* p, pp2_tree_info* info) {
  if (!p || !info) return set_err(PP2_EINVAL, "null argument");
  memset(info, 0, sizeof *info);
  info->total_vnodes = p->n_vnodes;
  info->total_qnodes = p->n_qnodes;
  info->expansions = p->expansions;
  const VNode* r = p->root;
  if (!r) return PP2_OK;
  info->depth = r->depth;
  info->root_upper_bound = r->upper_bound;
  info->root_lower_bound = r->lower_bound;
  info->root_heuristic = r->heuristic;
  info->n_root_children = (uint32_t)r->children.size();
  for (size_t a = 0; a < r->children.size() && a < 9; ++a) {
    const QNode* q = r->children[a];
    info->q_upper_bound[a] = q->upper_bound;
    info->q_lower_bound[a] = q->lower_bound;
    info->q_reward[a] = q->reward;
    info->q_heuristic[a] = q->heuristic;
    info->q_depth[a] = q->depth;
    info->q_nchildren[a] = (uint32_t)q->children.size();
    for (size_t k = 0; k < q->children.size() && k < 16; ++k) {
      info->q_obs[a][k] = q->children[k]->observation;
      info->q_weight[a][k] = q->children[k]->weight;
      info->v_upper_bound[a][k] = q->children[k]->upper_bound;
      info->v_lower_bound[a][k] = q->children[k]->lower_bound;
    }
  }
  return PP2_OK;
}

}  // extern "C"
