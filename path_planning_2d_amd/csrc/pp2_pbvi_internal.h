// pp2_pbvi_internal.h -- launchers of the PBVI kernels (private).
//
// Flat row layout: a belief / alpha vector is one row of `ld` floats (cell
// idx = y*W + x, ld = hw rounded up to kPbviChunk, pad cells 0); a set of S
// rows is padded to Sp = round_up(S, kGemmTile) rows, pad rows 0.
//
// Two translation units, split by whose arithmetic they restate:
//   pp2_pbvi_dev.hip  (FTZ, like the reference's nvcc --use_fast_math device
//                      code): the batched belief update and Gamma_ao;
//   pp2_pbvi_host.hip (IEEE denormals, like the reference's x86 host code and
//                      cuBLAS): sums, prefix sums, divisions, L1 distances,
//                      inner products, the sampler and the MFMA GEMM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pp2_internal.h"

namespace pp2 {

constexpr int kPbviChunk = 64;  // x-chunk of the pair kernel and the GEMM (ld multiple)
constexpr int kGemmTile = 128;  // GEMM tile rows / cols (Sp multiple)

enum PairOp { PAIR_L1 = 0, PAIR_DOT = 1, PAIR_CHILD = 2 };
enum RowMode { ROW_SUM = 0, ROW_CDF = 1 };

// ---- pp2_pbvi_dev.hip
// out[c] = cudaBayesBeliefUpdate(src[src_row[c]], us[c], zs[c]) (unnormalised)
hipError_t launch_pbvi_update(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet L,
                              const float* src, int ld, const int* src_row, const uint8_t* us,
                              const uint8_t* zs, int n, float* out);
// G[(a-a0)*16 + o][k][x] = cudaComputeGammaOA(a, o) of alpha k, for
// a0 <= a < a1, o < 16, k < S (rows k >= S and cells x >= hw are left
// untouched); ostride = floats between consecutive (a, o) slices.
hipError_t launch_pbvi_gamma_ao(hipStream_t st, const Geom& g, float gamma, PlaneSet T,
                                PlaneSet L, const float* alpha, int ld, int S, int a0, int a1,
                                float* G, long long ostride);

// ---- pp2_pbvi_host.hip
// ROW_SUM: sums[r] = ((A[r][0] + A[r][1]) + ...) over x < n (std::accumulate);
// ROW_CDF: cdf[r][x] = the running sums (std::partial_sum), and sums[r].
hipError_t launch_rows_seq(hipStream_t st, int mode, const float* A, int ld, int rows, int n,
                           float* sums, float* cdf);
// The same sums and dots for few chains (<= a few thousand): one chain per
// lane, rows streamed through an LDS ring (k_lane_chains), ~7x faster at hw
// 65536 when the chains, not the bytes, are the limit.  Bit-identical results.
// launch_lane_dots: out[i*ldo + j] = inner_product(A[i], B[j]), nb < 16.
hipError_t launch_lane_sums(hipStream_t st, const float* A, int ld, int rows, int n, float* sums);
hipError_t launch_lane_dots(hipStream_t st, const float* A, int na, const float* B, int nb,
                            int ld, int n, float* out, int ldo);
// A[r][x] /= sums[r], x < n
hipError_t launch_rows_div(hipStream_t st, float* A, int ld, int rows, int n,
                           const float* sums);
// out[r] = inner_product(A[r % amod], B[r]) (x-ordered, multiply then add)
hipError_t launch_rows_dot(hipStream_t st, const float* A, int amod, const float* B, int ld,
                           int rows, int n, float* out);
// out[i*ldo + j] = x-ordered sum over x < n of |A[i][x] - B[j][x]| (PAIR_L1)
// or A[i][x] * B[j][x] (PAIR_DOT, multiply then add), i < na, j < nb.  With
// a device row list (alist, acount): the rows alist[i], i < min(na, *acount),
// of A, results in out rows alist[i] (the other rows of out untouched).
hipError_t launch_pair_chain(hipStream_t st, int op, const float* A, int na, const float* B,
                             int nb, int ld, int n, float* out, int ldo,
                             const int* alist = nullptr, const int* acount = nullptr);
// The reference-order planner's sums on small grids, sequentially, one chain
// per lane, one wave per block (latency-bound chains: each block on a CU of
// its own): PAIR_DOT as launch_pair_chain; PAIR_CHILD: the term
// fl_ftz(B[j][x] * fl_ftz(A[i][x])) (a child's unnormalised belief, A = L
// rows, B = prediction rows).
hipError_t launch_pair_seq_small(hipStream_t st, int op, const float* A, int na, const float* B,
                                 int nb, int ld, int n, float* out, int ldo,
                                 const int* alist = nullptr, const int* acount = nullptr);
// The planner's PBVI leaf dots (PAIR_DOT, n >= 1024) with the child rows
// handed to the products by DPP broadcasts (pp2_pbvi_dots.hip); the same
// arguments and results as launch_pair_chain.  Needs na * ld < 2^29.
hipError_t launch_pair_dot_bq(hipStream_t st, const float* A, int na, const float* B, int nb, int ld, int n,
                              float* out, int ldo, const int* alist, const int* acount);
// cdf[x] = the running sums of row[0 .. n), *sum = the last (std::partial_sum)
hipError_t launch_row_cdf_seq(hipStream_t st, const float* row, int n, float* cdf, float* sum);
// The three draws of generateBeliefSet per (belief i, action a): state from
// cdf row i, next state from T[s][a][:], observation from L[ns][:].
hipError_t launch_pbvi_sample(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet L,
                              const float* cdf, int ld, int rows, const float* rnd,
                              uint8_t* z_out, int* s_out);
// per belief i < n: m[a] = min_j l1[(9i+a)*ldo + j] (j < nset), best_a[i] =
// first argmax of m, best_l1[i] = m[best_a]
hipError_t launch_pbvi_pick(hipStream_t st, const float* l1, int ldo, int n, int nset,
                            float* best_l1, int* best_a);
// C[z][s][i][k] = x-ordered fmaf chain over the split-s range of x of
// A[i][x] * B[z][k][x] (v_mfma_f32_32x32x2_f32); Mp, Np multiples of
// kGemmTile, ld of kPbviChunk.  ksplit = 1: the chain over all x from 0.
hipError_t launch_gemm_nt(hipStream_t st, const float* A, const float* B, float* C, int Mp,
                          int Np, int ld, int batch, long long bstride, long long cstride,
                          int ksplit, long long sstride);
// x-cells per split of launch_gemm_nt (each split's chain length): the
// planner's PBVI candidate bound (k_pbvi_cands) prices its rounding from it
int gemm_kchunk(int ld, int ksplit);
// out[r] = first argmax over k < n of C[r*ldc + k]
hipError_t launch_argmax_rows(hipStream_t st, const float* C, int rows, int n, int ldc,
                              int* out, float* vmax);
// for a0 <= a < a1: Ga[a][i][x] = R[x][a] + G[(a-a0)16 + 0][k*][x] + ... +
// G[(a-a0)16 + 15][k*][x], k* = kstar[((a-a0)16 + o) * kstride + i];
// Ga's action slices are gstride floats apart, like G's (a, o) slices.
hipError_t launch_pbvi_gamma_a(hipStream_t st, const Geom& g, PlaneSet R, const float* G,
                               long long gstride, int ld, int S, int a0, int a1,
                               const int* kstar, int kstride, float* Ga);
// action of belief i = first argmax_a V[a*Sp + i]; alpha_out[i] = Ga[action][i]
hipError_t launch_pbvi_select(hipStream_t st, const float* V, const float* Ga, int Sp, int S,
                              int ld, float* alpha_out, uint8_t* actions);
// split-K partial sums C[s][r][k] -> out[r][k], s ascending
hipError_t launch_sum_splits(hipStream_t st, const float* C, int splits, long long sstride,
                             int n, float* out);

// ---- pp2_fchain.hip (IEEE): the reference-order planner's grid-wide fp32
// sums, each equal to the reference's x-ordered chain, computed in parallel
// (pp2_fchain.h).  Group g < groups (or < *gcount) has id = glist[g] (or g0 +
// g) and K chains (K = 0: one chain of the base terms; K = 9: term i = base *
// partners[i][x], multiply then add):
//   FC_ROW:   base = row[id * row_stride + x]
//   FC_CHILD: base = fl_ftz(pred[id % 9][x] * L[id / 9][x]) -- the unnormalised
//             child of action id % 9 and observation id / 9
//   FC_LIST:  (K = 0) group g < *gcount is the chain of the pair plist[g] =
//             (row r, partner i): inner_product(row[r], partners[i]), terms
//             fl(row[r][x] * partners[i][x]) (evaluatePbviCpu) -- out[r * ldo + i]
// out[id * ldo + i] = the chain's sum; with cdf (FC_ROW, K = 0, one group)
// also every running sum, cdf[x] (std::partial_sum).  Scratch: FcScratch.
//   FC_KEPT:  (K = 9) group g's id c < 144 is a child of the expansion: its
//             normalised belief fl(ftz(pred[c % 9][x] * ftz(L_{c / 9}[x])) / m_c)
//             (search_tree_cuda.cu:228-229) times partner i: the FIB dots of
//             the kept children.  Sums phase: m_c approximate (msum: the
//             children set's chunk sums) over any group list; tables phase:
//             m_c = mass[c] exact, and each chunk's normalised cells written
//             to kept_rows[c] (and rowptr[c]); the drive walks kept_rows.
//             Scratch chains are indexed by c (by_id), so the phases may run
//             over different group lists.
enum FcBase { FC_ROW = 0, FC_CHILD = 1, FC_LIST = 2, FC_KEPT = 3 };
constexpr int kFcMaxCells = 1 << 28;
constexpr int kFcSegChunks = 4;  // chunks per k_fc_sums / k_fc_tables workgroup (1 per wave)
inline __host__ __device__ int fc_chunks(int n) { return (n + 255) / 256; }
inline __host__ __device__ int fc_segments(int n) {
  return (fc_chunks(n) + kFcSegChunks - 1) / kFcSegChunks;
}
struct FcArgs {
  int n = 0, ld = 0;
  const float* row = nullptr;
  long long row_stride = 0;
  const float* pred = nullptr;   // [9][ld]
  const float* lrows = nullptr;  // [16][ld]
  const float* partners = nullptr;  // [K][ld]
  int g0 = 0;
  const int* glist = nullptr;    // device: group -> id
  const int* gcount = nullptr;   // device: active groups
  float* out = nullptr;
  int ldo = 1;
  float* cdf = nullptr;
  float* sub = nullptr;          // with cdf (optional): the running sum at every 16th cell's end
  // scratch (FcScratch::attach)
  float* csum = nullptr;         // [chains][chunks] approximate chunk sums
  uint32_t* cflag = nullptr;     // [chains][segments] sign flags
  uint2* tab = nullptr;          // [chains][chunks] chunk entries
  int2* cst = nullptr;           // [chunks + 1] chunk start states (cdf)
  uint4* plan = nullptr;         // [chains][chunks][2] crossing plans of predicted chunks (optional)
  unsigned long long* agg = nullptr;  // [chains][segments] k_fc_sumtab's published segment sums
  unsigned epoch = 0;            // (set by launch_fchain: the tag of this launch's agg entries)
  int max_chains = 0, max_chunks = 0;
  int* stats = nullptr;          // diagnostics: driver {iterations, fallbacks, exact rounds, stash hits}
  const int2* plist = nullptr;   // FC_LIST: device (row, partner) pairs, *gcount of them
  int ngroups = 0;               // (set by launch_fchain: the launch's group count)
  // FC_KEPT
  const float* mass = nullptr;   // [144] the children's exact masses (tables, drive)
  const float* msum = nullptr;   // [144][chunks] the children's approximate chunk sums (sums)
  float* kept_rows = nullptr;    // [144][ld] normalised kept children (written by tables)
  float* const* rowptr = nullptr;  // optional device [144]: their node rows too
  int by_id = 0;                 // scratch chain index (id * K + i) instead of (g * K + i)
  // FC_KEPT: the sums pass runs with mass 1 (needs neither mass nor msum);
  // the tables scale its running sums by 1 / mass
  int kept_unit = 0;
  // K = 9, by_id: chain i of group id is tabled and walked only when bit i of
  // cmask[id] is set (launch_fib_cands); the others' out entries hold -inf
  const uint16_t* cmask = nullptr;
};
// The kept children's FIB candidates (evaluateFibCpu keeps only the first
// maximum of the 9 dots): after an FC_KEPT sums pass (a's csum / cflag / msum,
// by id) and with the exact masses (a.mass), each chain's |dot| is bounded;
// bit i of cmask[id] is set unless chain i's dot is certainly below another's,
// whose out[id * ldo + i] is set to -inf.  glist / gcount: the kept children.
hipError_t launch_fib_cands(hipStream_t st, const FcArgs& a, uint16_t* cmask);
// Device scratch of one stream's chain sets (a set may not overlap another
// set using the same scratch).
struct FcScratch {
  float* csum = nullptr;
  uint32_t* cflag = nullptr;
  uint2* tab = nullptr;
  int2* cst = nullptr;
  uint4* plan = nullptr;
  unsigned long long* agg = nullptr;
  int chains = 0, chunks = 0;
  FcScratch() = default;
  FcScratch(const FcScratch&) = delete;
  FcScratch& operator=(const FcScratch&) = delete;
  ~FcScratch() { release(); }
  bool reserve(int n, int max_chains);
  void release();
  void attach(FcArgs* a) const;
};
// phases (bit mask): 1 = the chunk sums and tables, 2 = the driver (and the
// running sums): a caller may enqueue other work between the two, with the
// same FcArgs and scratch.
// FC_SUMS / FC_TAB split FC_TABLES (FC_KEPT: the sums early, over every
// child, on another stream)
enum : int { FC_TABLES = 1, FC_DRIVE = 2, FC_ALL = 3, FC_SUMS = 4, FC_TAB = 8 };
hipError_t launch_fchain(hipStream_t st, int base, int K, int groups, const FcArgs& a,
                         int phases = FC_ALL);
// whether sums + tables run as one launch (k_fc_sumtab; PP2_FC_SUMTAB)
bool fc_sumtab_active();
// forwardSampling of the 9 actions from the expanded belief's running sums
// cdf[n]: r[9 * N] the host's rand() values (action-major), u1 / u2 [N] the
// curand uniforms; counts[a * 16 + z] and the kept children z * 9 + a.
struct SampleArgs {
  Geom g;
  PlaneSet T, L;
  const float* cdf = nullptr;
  int n = 0, N = 0;
  const float* r = nullptr;
  const float* u1 = nullptr;
  const float* u2 = nullptr;
  int* counts = nullptr;  // [144]
  int* klist = nullptr;   // [144]
  int* kcount = nullptr;
  // optional (the chain set's running sums): the 16-cell ends (FcArgs::sub)
  // and the chunk start states, whose entry [chunks] holds the sign flags
  const float* sub = nullptr;
  const int2* cst = nullptr;
  // optional: a table of row pointers to publish to the device on the way
  // (*rows, carried in the kernel's arguments, into rows_out[144])
  const struct FcRowTable* rows = nullptr;
  float** rows_out = nullptr;
};
hipError_t launch_tree_sample(hipStream_t st, const SampleArgs& s);
// Fused chain sets (pp2_fchain.hip, round 6): the same sums as launch_fchain,
// equal bit for bit, in ONE launch per set -- a workgroup of 1024 threads per
// chain holds the chain's terms in registers through the chunk sums, the
// tables and the walk -- for n <= 65536 cells and a row stride ld % 64 == 0
// (fx_fits).  Group g < groups (or < *gcount) has id = glist[g] (or g0 + g)
// and K chains (0, or 9 partners), out[id * ldo + i]:
//   FX_ROW    K 0 / 9: row[id * row_stride + x] (* partners[i][x])
//   FX_CHILD  K 0: fl_ftz(pred[id % 9][x] * L[id / 9][x]) (the children's masses)
//   FX_KEPT   K 9: b[x] = that / sums[id] (the normalised child) * partners[i][x]
//             (evaluateFibCpu of the kept children); the workgroups of partner
//             0 also store b into rows_out + id * ld (if set) and dst[id] (use_dst)
enum FxBase { FX_ROW = 0, FX_CHILD = 1, FX_KEPT = 2 };
struct FxArgs {
  int n = 0, ld = 0;
  const float* row = nullptr;
  long long row_stride = 0;
  const float* pred = nullptr;      // [9][ld]
  const float* lrows = nullptr;     // [16][ld]
  const float* partners = nullptr;  // [K][ld]
  const float* sums = nullptr;      // FX_KEPT: the children's masses [144]
  int g0 = 0;
  const int* glist = nullptr;
  const int* gcount = nullptr;
  float* out = nullptr;
  int ldo = 1;
  float* cdf = nullptr;             // launch_fx_cdf_sample: every running sum
  float* rows_out = nullptr;        // FX_KEPT: the normalised children [144][ld]
  int use_dst = 0;
  float* dst[144] = {};             // FX_KEPT: and child c's row at dst[c]
  unsigned long long* stamps = nullptr;  // diagnostics: s_memrealtime at the phase ends, 8 per workgroup
  int ngroups = 0;                  // (set by the launcher)
};
bool fx_fits(int n, int ld);
hipError_t launch_fx(hipStream_t st, int base, int K, int groups, const FxArgs& a);
// The expanded belief's cdf and forwardSampling in one launch (FX_ROW, K 0,
// row a.row): out[0] = its sum, cdf[x], and s.counts / s.klist / s.kcount as
// launch_tree_sample from that cdf.
hipError_t launch_fx_cdf_sample(hipStream_t st, const FxArgs& a, const SampleArgs& s);
// The planner's PBVI leaf bounds in reference order (pp2_fchain.hip): per
// alpha, max |alpha[x]| and its sign flags; then per row the alphas whose
// exact chain can reach the maximum, from approximate dots and a rigorous
// error bound -- the candidates into plist (+= *pcount), every other entry
// of exact[r * lde + i] set to -inf.
hipError_t launch_alpha_stats(hipStream_t st, const float* al, int S, int n, int ld, float* amax,
                              uint32_t* aflag);
struct PbviCandArgs {
  const float* rows = nullptr;   // the rows (beliefs): row r at rows + r * row_stride
  long long row_stride = 0;
  int n = 0;                     // chain length (cells)
  const int* klist = nullptr;    // rows klist[q], q < *kcount (or q < nrows)
  const int* kcount = nullptr;
  int nrows = 0;                 // grid rows (max rows)
  const float* approx = nullptr; // approximate dots [r * lda + i]
  int lda = 0;
  const float* amax = nullptr;   // launch_alpha_stats
  const uint32_t* aflag = nullptr;
  int S = 0;
  float c_rel = 0.0f;            // (n + kchunk + splits + 8) * 2^-24, with slack
  float* exact = nullptr;        // [r * lde + i]
  int lde = 0;
  int2* plist = nullptr;
  int* pcount = nullptr;
};
hipError_t launch_pbvi_cands(hipStream_t st, const PbviCandArgs& c);
// dst[r][x] = fl_ftz(pred[c % 9][x] * L[c / 9][x]) / sums[c], c = child[r], x < n.
struct FcStoreList {
  int n = 0;
  int child[144];
  float* dst[144];
};
hipError_t launch_store_children(hipStream_t st, const FcStoreList& L, const float* pred,
                                 const float* lrows, const float* sums, int n, int ld);
// The same for the children listed on the device (klist[r], r < *kcount, at
// most 144): child c into dst + c * ld.
// rows (optional): child c's row also into rows->p[c] (the planner's node rows)
struct FcRowTable {
  int use = 0;
  float* p[144] = {};
};
// the kept children's dense rows src + c * ld into rows->p[c] (n cells)
hipError_t launch_copy_kept(hipStream_t st, const int* klist, const int* kcount, const float* src,
                            int n, int ld, const FcRowTable* rows);
hipError_t launch_store_kept(hipStream_t st, const int* klist, const int* kcount,
                             const float* pred, const float* lrows, const float* sums, float* dst,
                             int n, int ld, const FcRowTable* rows = nullptr);

// ---- pp2_pbvi_dev.hip (FTZ): the 9 action predictions of cudaBayesBeliefUpdate
// before the likelihood product: pred[u][idx] = sum_s T[sidx][u][8-s] * b[sidx]
// (fmaf chain, s ascending, in-grid neighbours), b a dense row; sparse: T is
// +0 off each action's base-kernel support (the coded model's check), so
// only the support taps are read.
hipError_t launch_tree_pred(hipStream_t st, const Geom& g, PlaneSet T, const float* b, int ld,
                            float* pred, bool sparse);

}  // namespace pp2
