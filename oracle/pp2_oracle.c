/*
 * pp2_oracle.c -- CPU restatement of path_planning_2d's hot path.
 * TEST INFRASTRUCTURE ONLY; parity unpinned by reference tests (none exist).
 * See pp2_oracle.h for the contract and the citation root.
 *
 * Compile with -ffp-contract=off: every fused multiply-add below is an
 * explicit fmaf() standing for an nvcc contraction in the reference device
 * code; everything else must stay a separately rounded mul / add.
 */
#include "pp2_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline float ftzf(float x, int on) {
  return (on && fabsf(x) < FLT_MIN) ? copysignf(0.0f, x) : x;
}

/* 3x3 local map, out-of-range = occupied
 * (model_generation_cuda.cu:313-324, path_planning_2d_cuda.cu:185-196) */
static void local_map3(int H, int W, const uint8_t* map, int x, int y,
                       uint8_t lm[9]) {
  int i = 0;
  for (int oy = -1; oy < 2; ++oy)
    for (int ox = -1; ox < 2; ++ox, ++i) {
      int nx = x + ox, ny = y + oy;
      lm[i] = (nx < 0 || nx >= W || ny < 0 || ny >= H)
                  ? 1 : map[(size_t)ny * W + nx];
    }
}

/* base motion kernel for action u (model_generation_cuda.cu:175-211) */
static void base_kernel(int u, float tp[9]) {
  for (int i = 0; i < 9; ++i) tp[i] = 0.0f;
  switch (u) {
    case 0: tp[0] = 0.7f; tp[1] = 0.1f; tp[3] = 0.1f; tp[4] = 0.1f; break;
    case 1: tp[0] = 0.1f; tp[1] = 0.7f; tp[2] = 0.1f; tp[4] = 0.1f; break;
    case 2: tp[1] = 0.1f; tp[2] = 0.7f; tp[4] = 0.1f; tp[5] = 0.1f; break;
    case 3: tp[0] = 0.1f; tp[3] = 0.7f; tp[4] = 0.1f; tp[6] = 0.1f; break;
    case 4: tp[4] = 1.0f; break;
    case 5: tp[2] = 0.1f; tp[4] = 0.1f; tp[5] = 0.7f; tp[8] = 0.1f; break;
    case 6: tp[3] = 0.1f; tp[4] = 0.1f; tp[6] = 0.7f; tp[7] = 0.1f; break;
    case 7: tp[4] = 0.1f; tp[6] = 0.1f; tp[7] = 0.7f; tp[8] = 0.1f; break;
    case 8: tp[4] = 0.1f; tp[5] = 0.1f; tp[7] = 0.1f; tp[8] = 0.7f; break;
  }
}

/* POMDP cudaTransitionProbability (model_generation_cuda.cu:161-236):
 * naive copy BEFORE the occupied-neighbour shift and the trap override. */
static void trans_pomdp(int u, const uint8_t lm[9], float tp[9], float nv[9]) {
  base_kernel(u, tp);
  memcpy(nv, tp, sizeof(float) * 9);
  for (int i = 0; i < 9; ++i)
    if (lm[i] == 1 && i != 4) { tp[4] += tp[i]; tp[i] = 0.0f; }
  if (lm[4] == 1) {
    for (int i = 0; i < 9; ++i) tp[i] = 0.0f;
    tp[4] = 1.0f;
  }
}

/* MDP cudaTransitionProbability (path_planning_2d_cuda.cu:76-150):
 * trap override FIRST, then naive copy, then the shift. */
static void trans_mdp(int u, const uint8_t lm[9], float tp[9], float nv[9]) {
  base_kernel(u, tp);
  if (lm[4] == 1) {
    for (int i = 0; i < 9; ++i) tp[i] = 0.0f;
    tp[4] = 1.0f;
  }
  memcpy(nv, tp, sizeof(float) * 9);
  for (int i = 0; i < 9; ++i)
    if (lm[i] == 1 && i != 4) { tp[4] += tp[i]; tp[i] = 0.0f; }
}

/* cudaMeasurementLikelihood (model_generation_cuda.cu:238-264):
 * m = cells {1 up, 3 left, 5 right, 7 down}; the constants are doubles
 * narrowed to float; product left to right in fp32. */
static void meas_lik(const uint8_t lm[9], float L[16]) {
  const uint8_t m[4] = {lm[1], lm[3], lm[5], lm[7]};
  for (int i = 0; i < 16; ++i) {
    float l0 = (((i >> 0) & 1) == m[0]) ? (float)0.98 : (float)0.02;
    float l1 = (((i >> 1) & 1) == m[1]) ? (float)0.98 : (float)0.02;
    float l2 = (((i >> 2) & 1) == m[2]) ? (float)0.98 : (float)0.02;
    float l3 = (((i >> 3) & 1) == m[3]) ? (float)0.98 : (float)0.02;
    L[i] = l0 * l1 * l2 * l3;
  }
}

void orc_cell_model(int H, int W, const uint8_t* map, int x, int y, int gx,
                    int gy, float* T81, float* L16, float* R9, float* C9) {
  uint8_t lm[9];
  local_map3(H, W, map, x, y, lm);
  float tp[81], nv[81];
  if (T81 || R9) {
    for (int u = 0; u < 9; ++u) trans_pomdp(u, lm, tp + 9 * u, nv + 9 * u);
    if (T81) memcpy(T81, tp, sizeof tp);
    if (R9) {
      /* cudaStageReward (model_generation_cuda.cu:266-296) */
      float mr[9];
      for (int i = 0; i < 9; ++i) mr[i] = (lm[i] == 1) ? -2.0f : -1.0f;
      for (int u = 0; u < 9; ++u) {
        float s = 0.0f;
        for (int i = 0; i < 9; ++i) s = fmaf(mr[i], nv[9 * u + i], s);
        R9[u] = s;
      }
      R9[4] = ((unsigned)x != (unsigned)gx || (unsigned)y != (unsigned)gy)
                  ? -2.0f : 0.0f;
    }
  }
  if (C9) {
    /* cudaStageCost (path_planning_2d_cuda.cu:152-172) with the MDP naive T */
    for (int u = 0; u < 9; ++u) trans_mdp(u, lm, tp + 9 * u, nv + 9 * u);
    float mc[9];
    for (int i = 0; i < 9; ++i) mc[i] = (lm[i] == 1) ? 2.0f : 1.0f;
    for (int u = 0; u < 9; ++u) {
      float s = 0.0f;
      for (int i = 0; i < 9; ++i) s = fmaf(mc[i], nv[9 * u + i], s);
      C9[u] = s;
    }
    C9[4] = ((unsigned)x != (unsigned)gx || (unsigned)y != (unsigned)gy)
                ? 2.0f : 0.0f;
  }
  if (L16) meas_lik(lm, L16);
}

void orc_model_pomdp(int H, int W, const uint8_t* map, int gx, int gy,
                     float* T, float* L, float* R) {
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      size_t idx = (size_t)y * W + x;
      orc_cell_model(H, W, map, x, y, gx, gy, T ? T + 81 * idx : NULL,
                     L ? L + 16 * idx : NULL, R ? R + 9 * idx : NULL, NULL);
    }
}

void orc_model_mdp(int H, int W, const uint8_t* map, int gx, int gy,
                   float* T, float* C) {
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      size_t idx = (size_t)y * W + x;
      uint8_t lm[9];
      float tp[81], nv[81];
      local_map3(H, W, map, x, y, lm);
      for (int u = 0; u < 9; ++u) trans_mdp(u, lm, tp + 9 * u, nv + 9 * u);
      if (T) memcpy(T + 81 * idx, tp, sizeof tp);
      if (C) orc_cell_model(H, W, map, x, y, gx, gy, NULL, NULL, NULL,
                            C + 9 * idx);
    }
}

/* ---- belief ---------------------------------------------------------------- */
void orc_belief_update_rows(int H, int W, const float* T, const float* L,
                            const float* b_in, int u, int z, float* b_out,
                            int ftz, int y0, int y1) {
  for (int y = y0; y < y1; ++y)
    for (int x = 0; x < W; ++x) {
      float lt[9] = {0}, lb[9] = {0};
      int s = 0;
      for (int oy = -1; oy < 2; ++oy)
        for (int ox = -1; ox < 2; ++ox, ++s) {
          int sx = x + ox, sy = y + oy;
          if (sx < 0 || sx >= W || sy < 0 || sy >= H) continue;
          size_t sidx = (size_t)sy * W + sx;
          lt[s] = T[81 * sidx + 9 * u + (8 - s)];
          lb[s] = b_in[sidx];
        }
      float p = 0.0f;
      for (s = 0; s < 9; ++s)
        p = ftzf(fmaf(ftzf(lt[s], ftz), ftzf(lb[s], ftz), p), ftz);
      size_t idx = (size_t)y * W + x;
      p = ftzf(p * ftzf(L[16 * idx + z], ftz), ftz);
      b_out[idx] = p;
    }
}

void orc_belief_update(int H, int W, const float* T, const float* L,
                       const float* b_in, int u, int z, float* b_out, int ftz) {
  orc_belief_update_rows(H, W, T, L, b_in, u, z, b_out, ftz, 0, H);
}

float orc_sum_seq(size_t n, const float* b) {
  float s = 0.0f;
  for (size_t i = 0; i < n; ++i) s = s + b[i];
  return s;
}

double orc_sum_f64(size_t n, const float* b) {
  double s = 0.0;
  for (size_t i = 0; i < n; ++i) s += (double)b[i];
  return s;
}

float orc_normalize_seq(size_t n, float* b) {
  float s = orc_sum_seq(n, b);
  for (size_t i = 0; i < n; ++i) b[i] /= s;
  return s;
}

double orc_normalize_f64(size_t n, float* b) {
  double s = orc_sum_f64(n, b);
  for (size_t i = 0; i < n; ++i) b[i] = (float)((double)b[i] / s);
  return s;
}

/* ---- MDP ------------------------------------------------------------------- */
void orc_mdp_sweep_rows(int H, int W, float gamma, const float* T,
                        const float* C, const float* J_in, float* J_out,
                        uint8_t* A, int y0, int y1) {
  for (int y = y0; y < y1; ++y)
    for (int x = 0; x < W; ++x) {
      size_t idx = (size_t)y * W + x;
      float jn[9] = {0};
      int i = 0;
      for (int oy = -1; oy < 2; ++oy)
        for (int ox = -1; ox < 2; ++ox, ++i) {
          int nx = x + ox, ny = y + oy;
          if (nx >= 0 && nx < W && ny >= 0 && ny < H)
            jn[i] = J_in[(size_t)ny * W + nx];
        }
      float best = FLT_MAX;
      uint8_t arg = 0;
      const float* tp = T + 81 * idx;
      for (int u = 0; u < 9; ++u) {
        float cost = C[9 * idx + u];
        for (i = 0; i < 9; ++i)
          cost = fmaf(gamma * tp[9 * u + i], jn[i], cost);
        if (cost < best) { best = cost; arg = (uint8_t)u; }
      }
      J_out[idx] = best;
      if (A) A[idx] = arg;
    }
}

void orc_mdp_sweep(int H, int W, float gamma, const float* T, const float* C,
                   const float* J_in, float* J_out, uint8_t* A) {
  orc_mdp_sweep_rows(H, W, gamma, T, C, J_in, J_out, A, 0, H);
}

/* ---- CPU baseline: loop steps row-partitioned over threads ---------------- */
/* The north-star loop step (belief update, renormalisation, Bellman sweep)
 * with the rows of every phase split across nthreads pthreads -- the
 * "std::thread row-partitioned" CPU mode of SURVEY.md §8(d).  Per-thread
 * partial sums are combined in thread order.  Timing baseline only. */
typedef struct {
  int H, W, y0, y1, u, z, phase;
  float gamma, inv;
  const float *T, *L, *C, *b, *J;
  float *bo, *Jo, sum;
  uint8_t* A;
} orc_loop_job;

static void* orc_loop_worker(void* arg) {
  orc_loop_job* j = (orc_loop_job*)arg;
  if (j->phase == 0) {
    orc_belief_update_rows(j->H, j->W, j->T, j->L, j->b, j->u, j->z, j->bo, 1, j->y0, j->y1);
    orc_mdp_sweep_rows(j->H, j->W, j->gamma, j->T, j->C, j->J, j->Jo, j->A, j->y0, j->y1);
    float s = 0.0f;
    for (size_t i = (size_t)j->y0 * j->W; i < (size_t)j->y1 * j->W; ++i) s = s + j->bo[i];
    j->sum = s;
  } else {
    for (size_t i = (size_t)j->y0 * j->W; i < (size_t)j->y1 * j->W; ++i) j->bo[i] *= j->inv;
  }
  return NULL;
}

int orc_loop_run_mt(int H, int W, float gamma, const float* T, const float* L, const float* C,
                    float* b, float* bo, float* J, float* Jo, uint8_t* A, int nsteps,
                    const uint8_t* us, const uint8_t* zs, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if (nthreads > H) nthreads = H;
  pthread_t th[256];
  orc_loop_job job[256];
  for (int step = 0; step < nsteps; ++step) {
    for (int phase = 0; phase < 2; ++phase) {
      float inv = 0.0f;
      if (phase == 1) {
        float s = 0.0f;
        for (int t = 0; t < nthreads; ++t) s = s + job[t].sum;
        inv = 1.0f / s;
      }
      for (int t = 0; t < nthreads; ++t) {
        orc_loop_job* j = &job[t];
        j->H = H; j->W = W; j->u = us[step]; j->z = zs[step]; j->phase = phase;
        j->y0 = (int)((long long)H * t / nthreads);
        j->y1 = (int)((long long)H * (t + 1) / nthreads);
        j->gamma = gamma; j->inv = inv;
        j->T = T; j->L = L; j->C = C; j->b = b; j->J = J; j->bo = bo; j->Jo = Jo; j->A = A;
        if (pthread_create(&th[t], NULL, orc_loop_worker, j) != 0) return -1;
      }
      for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    }
    float* tb = b; b = bo; bo = tb;
    float* tj = J; J = Jo; Jo = tj;
  }
  return nsteps;
}

int orc_mdp_solve(int H, int W, float gamma, const float* T, const float* C,
                  float* J, uint8_t* A, int max_sweeps, double* final_norm) {
  size_t n = (size_t)H * W;
  float* J2 = (float*)calloc(n, sizeof(float));
  float* prev = (float*)calloc(n, sizeof(float));
  memset(J, 0, n * sizeof(float));
  int total = 0;
  double norm = 0.0;
  /* double max_optimal_cost = 5.0/(1.0-discount_factor) (path_planning_2d.cu:221) */
  const double max_cost = 5.0 / (1.0 - (double)gamma);
  do {
    for (int i = 0; i < 50; ++i) {
      orc_mdp_sweep(H, W, gamma, T, C, J, J2, A);
      orc_mdp_sweep(H, W, gamma, T, C, J2, J, A);
    }
    total += 100;
    float m = 0.0f; /* cv::absdiff + minMaxIdx on CV_32F */
    for (size_t k = 0; k < n; ++k) {
      float d = fabsf(prev[k] - J[k]);
      if (d > m) m = d;
    }
    norm = (double)m;
    memcpy(prev, J, n * sizeof(float));
    if (max_sweeps > 0 && total >= max_sweeps) break;
  } while (norm > max_cost * 1e-3);
  free(J2);
  free(prev);
  if (final_norm) *final_norm = norm;
  return total;
}

/* ---- FIB ------------------------------------------------------------------- */
void orc_fib_sweep(int H, int W, float gamma, const float* T, const float* L,
                   const float* R, const float* a_in, float* a_out) {
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      size_t idx = (size_t)y * W + x;
      float lm[144] = {0}, la[81] = {0};
      int i = 0;
      for (int oy = -1; oy < 2; ++oy)
        for (int ox = -1; ox < 2; ++ox, ++i) {
          int nx = x + ox, ny = y + oy;
          if (nx < 0 || nx >= W || ny < 0 || ny >= H) continue;
          size_t nidx = (size_t)ny * W + nx;
          memcpy(lm + 16 * i, L + 16 * nidx, 16 * sizeof(float));
          memcpy(la + 9 * i, a_in + 9 * nidx, 9 * sizeof(float));
        }
      for (int a = 0; a < 9; ++a) {
        const float* tp = T + 81 * idx + 9 * a;
        float reward = R[9 * idx + a];
        float rtg = 0.0f;
        for (int o = 0; o < 16; ++o) {
          float tm[9];
          for (int sp = 0; sp < 9; ++sp) tm[sp] = tp[sp] * lm[sp * 16 + o];
          float rtgo = -FLT_MAX;
          for (int ap = 0; ap < 9; ++ap) {
            float s = 0.0f;
            for (int sp = 0; sp < 9; ++sp) s = fmaf(tm[sp], la[sp * 9 + ap], s);
            if (rtgo < s) rtgo = s;
          }
          rtg = rtg + rtgo;
        }
        a_out[9 * idx + a] = fmaf(gamma, rtg, reward);
      }
    }
}

int orc_fib_solve(int H, int W, float gamma, const float* T, const float* L,
                  const float* R, float* alphas, int max_sweeps,
                  float* final_norm) {
  size_t n = (size_t)H * W * 9;
  float* a2 = (float*)calloc(n, sizeof(float));
  float* prev = (float*)calloc(n, sizeof(float));
  memset(alphas, 0, n * sizeof(float));
  int total = 0;
  float norm = 0.0f;
  do {
    for (int i = 0; i < 5; ++i) {
      orc_fib_sweep(H, W, gamma, T, L, R, alphas, a2);
      orc_fib_sweep(H, W, gamma, T, L, R, a2, alphas);
    }
    total += 10;
    norm = 0.0f;
    for (size_t k = 0; k < n; ++k) {
      float d = fabsf(prev[k] - alphas[k]);
      if (d > norm) norm = d;
    }
    memcpy(prev, alphas, n * sizeof(float));
    if (max_sweeps > 0 && total >= max_sweeps) break;
  } while (norm > 0.01f);
  free(a2);
  free(prev);
  if (final_norm) *final_norm = norm;
  return total;
}

/* ---- leaves ---------------------------------------------------------------- */
void orc_fib_eval(size_t n, const float* b, const float* alphas, float* value,
                  uint8_t* action) {
  /* evaluateFibCpu (fast_informed_bound_cuda.cu:278-297): nine x-ordered
   * fp32 inner_products, walked side by side (independent chains) */
  float v[9] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  for (size_t k = 0; k < n; ++k) {
    const float bk = b[k];
    for (int i = 0; i < 9; ++i) v[i] = v[i] + bk * alphas[9 * k + i];
  }
  int best = 0; /* std::max_element: first maximum */
  for (int i = 1; i < 9; ++i)
    if (v[best] < v[i]) best = i;
  *value = v[best];
  *action = (uint8_t)best; /* host_fib_actions = {0..8} */
}

/* evaluatePbviCpu (point_based_value_iteration_cuda.cu:678-699): per alpha
 * one x-ordered fp32 inner_product, then the first maximum.  Eight alphas'
 * chains are walked side by side (independent chains, each still added in
 * x order: the same bits, without the add latency of a single chain). */
void orc_pbvi_eval(size_t n, const float* b, int S, const float* alphas,
                   const uint8_t* actions, float* value, uint8_t* action) {
  int best = 0;
  float bv = 0.0f;
  int i = 0;
  for (; i + 8 <= S; i += 8) {
    const float* al = alphas + (size_t)i * n;
    float s[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (size_t k = 0; k < n; ++k) {
      const float bk = b[k];
      for (int m = 0; m < 8; ++m) s[m] = s[m] + bk * al[(size_t)m * n + k];
    }
    for (int m = 0; m < 8; ++m)
      if (i + m == 0 || bv < s[m]) { bv = s[m]; best = i + m; }
  }
  for (; i < S; ++i) {
    float s = 0.0f;
    const float* al = alphas + (size_t)i * n;
    for (size_t k = 0; k < n; ++k) s = s + b[k] * al[k];
    if (i == 0 || bv < s) { bv = s; best = i; }
  }
  *value = bv;
  *action = actions ? actions[best] : 0;
}

float orc_reward_dot(size_t n, const float* b, const float* R, int a) {
  float s = 0.0f;
  for (size_t k = 0; k < n; ++k) s = s + b[k] * R[9 * k + a];
  return s;
}

/* ---- simulator filter (dummy_simulator.cpp) --------------------------------- */
/* DummySimulator::transitionProbability (:440-522): OOB neighbours and
 * grid_map>0 neighbours shift to self; no trap override. */
static void sim_trans(int H, int W, const uint8_t* map, int x, int y, int u,
                      float tp[9]) {
  base_kernel(u, tp);
  int i = 0;
  for (int oy = -1; oy < 2; ++oy)
    for (int ox = -1; ox < 2; ++ox, ++i) {
      int px = x + ox, py = y + oy;
      if (px < 0 || px >= W || py < 0 || py >= H) {
        tp[4] += tp[i]; tp[i] = 0.0f; continue;
      }
      if (map[(size_t)py * W + px] > 0 && i != 4) {
        tp[4] += tp[i]; tp[i] = 0.0f; continue;
      }
    }
}

void orc_sim_predict(int H, int W, const uint8_t* map, const float* b, int u,
                     float* out) {
  size_t n = (size_t)H * W;
  for (size_t i = 0; i < n; ++i) out[i] = 0.0f;
  static const int ox[9] = {-1, 0, 1, -1, 0, 1, -1, 0, 1};
  static const int oy[9] = {-1, -1, -1, 0, 0, 0, 1, 1, 1};
  for (int y = 0, idx = 0; y < H; ++y)
    for (int x = 0; x < W; ++x, ++idx) {
      if (b[idx] == 0.0f) continue;
      float tp[9];
      sim_trans(H, W, map, x, y, u, tp);
      for (int i = 0; i < 9; ++i) {
        int px = x + ox[i], py = y + oy[i];
        if (px < 0 || px >= W || py < 0 || py >= H) continue;
        size_t p = (size_t)py * W + px;
        out[p] = out[p] + b[idx] * tp[i];
      }
    }
  float s = 0.0f;
  for (size_t i = 0; i < n; ++i) s = s + out[i];
  for (size_t i = 0; i < n; ++i) out[i] /= s;
}

void orc_sim_correct(int H, int W, const uint8_t* map, const float* b, int z,
                     float* out) {
  static const int ox[4] = {0, -1, 1, 0};
  static const int oy[4] = {-1, 0, 0, 1};
  size_t n = (size_t)H * W;
  float s = 0.0f;
  for (int y = 0, idx = 0; y < H; ++y)
    for (int x = 0; x < W; ++x, ++idx) {
      if (b[idx] == 0.0f) { out[idx] = 0.0f; continue; }
      float l = 1.0f;
      for (int i = 0; i < 4; ++i) {
        int mx = x + ox[i], my = y + oy[i];
        uint8_t m = (mx < 0 || mx >= W || my < 0 || my >= H)
                        ? 1 : map[(size_t)my * W + mx];
        l *= (m == ((z >> i) & 1)) ? 0.98f : 0.02f;
      }
      out[idx] = l * b[idx];
      s = s + out[idx];
    }
  for (size_t i = 0; i < n; ++i) out[i] /= s;
}

/* ---- glibc rand() ----------------------------------------------------------- */
/* glibc srandom_r/random_r, TYPE_3 (degree 31, separation 3). */
void orc_rand_seed(orc_rand_state* s, uint32_t seed) {
  int32_t st[31];
  int64_t word = (int32_t)(seed == 0 ? 1 : seed);
  st[0] = (int32_t)word;
  for (int i = 1; i < 31; ++i) {
    int64_t hi = word / 127773, lo = word % 127773;
    word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    st[i] = (int32_t)word;
  }
  for (int i = 0; i < 31; ++i) s->r[i] = st[i];
  s->f = 3; /* fptr = &state[SEP_3] */
  s->b = 0; /* rptr = &state[0] */
  for (int i = 0; i < 310; ++i) (void)orc_rand_next(s);
}

int32_t orc_rand_next(orc_rand_state* s) {
  uint32_t val = (uint32_t)s->r[s->f] + (uint32_t)s->r[s->b];
  s->r[s->f] = (int32_t)val;
  int32_t out = (int32_t)(val >> 1);
  if (++s->f >= 31) { s->f = 0; ++s->b; }
  else if (++s->b >= 31) s->b = 0;
  return out;
}

/* ---- cuRAND XORWOW ---------------------------------------------------------- */
/* State x[5] evolves linearly over GF(2); d is a Weyl sequence.  A subsequence
 * is 2^67 draws (curand_init docs), so skipahead_sequence(k) = M^(k*2^67). */
typedef struct { uint32_t c[160][5]; } gf2mat; /* column j = M e_j */

static void xw_step(uint32_t v[5]) {
  uint32_t t = v[0] ^ (v[0] >> 2);
  v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
  v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}

static void gf2_apply(const gf2mat* m, const uint32_t v[5], uint32_t out[5]) {
  uint32_t r[5] = {0, 0, 0, 0, 0};
  for (int j = 0; j < 160; ++j)
    if ((v[j >> 5] >> (j & 31)) & 1u)
      for (int w = 0; w < 5; ++w) r[w] ^= m->c[j][w];
  memcpy(out, r, sizeof r);
}

static void gf2_mul(const gf2mat* a, const gf2mat* b, gf2mat* out) {
  gf2mat t;
  for (int j = 0; j < 160; ++j) gf2_apply(a, b->c[j], t.c[j]);
  *out = t;
}

void orc_curand_xorwow(uint64_t seed, uint64_t subsequence, uint64_t offset,
                       int n, uint32_t* out) {
  /* _curand_init_scratch (CUDA 8 curand_kernel.h) */
  uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
  uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
  uint32_t t0 = 1099087573u * s0;
  uint32_t t1 = 2591861531u * s1;
  uint32_t d = 6615241u + t1 + t0;
  uint32_t v[5] = {123456789u + t0, 362436069u ^ t0, 521288629u + t1,
                   88675123u ^ t1, 5783321u + t0};
  if (subsequence) {
    static gf2mat* J = NULL; /* M^(2^67), built once */
    if (!J) {
      gf2mat* m = (gf2mat*)malloc(sizeof(gf2mat));
      for (int j = 0; j < 160; ++j) {
        uint32_t e[5] = {0, 0, 0, 0, 0};
        e[j >> 5] = 1u << (j & 31);
        xw_step(e);
        memcpy(m->c[j], e, sizeof e);
      }
      for (int k = 0; k < 67; ++k) gf2_mul(m, m, m);
      J = m;
    }
    /* M^(k*2^67) v by binary powering of J */
    gf2mat* p = (gf2mat*)malloc(sizeof(gf2mat));
    *p = *J;
    uint64_t k = subsequence;
    while (k) {
      if (k & 1) gf2_apply(p, v, v);
      k >>= 1;
      if (k) gf2_mul(p, p, p);
    }
    free(p);
  }
  for (uint64_t k = 0; k < offset; ++k) { xw_step(v); d += 362437u; }
  for (int i = 0; i < n; ++i) {
    xw_step(v);
    d += 362437u;
    out[i] = v[4] + d;
  }
}

float orc_curand_uniform(uint32_t x) {
  const float inv = 2.3283064e-10f; /* CURAND_2POW32_INV */
  return fmaf((float)x, inv, inv / 2.0f);
}

/* ---- synthetic inputs --------------------------------------------------------- */
uint64_t orc_splitmix64_next(uint64_t* s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

static double u01(uint64_t* s) {
  return (double)(orc_splitmix64_next(s) >> 11) * 0x1.0p-53;
}

void orc_synth_map(int H, int W, uint64_t seed, double p_occ, uint8_t* map) {
  uint64_t s = seed;
  size_t n = (size_t)H * W;
  for (size_t i = 0; i < n; ++i) map[i] = (u01(&s) < p_occ) ? 1 : 0;
}

int orc_synth_goal(int H, int W, const uint8_t* map, int* gx, int* gy) {
  int x0 = W - 6 < 0 ? W - 1 : W - 6;
  int y0 = H - 6 < 0 ? H - 1 : H - 6;
  for (int y = y0; y >= 0; --y)
    for (int x = x0; x >= 0; --x)
      if (map[(size_t)y * W + x] == 0) { *gx = x; *gy = y; return 0; }
  return -1;
}

int orc_synth_trajectory(int H, int W, const uint8_t* map, int gx, int gy,
                         uint64_t seed, int n, uint8_t* us, uint8_t* zs,
                         int32_t* states) {
  /* start: free cell nearest the centre (squared distance, row-major ties) */
  int cx = W / 2, cy = H / 2, sx = -1, sy = -1;
  long best = -1;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      if (map[(size_t)y * W + x]) continue;
      long d = (long)(x - cx) * (x - cx) + (long)(y - cy) * (y - cy);
      if (best < 0 || d < best) { best = d; sx = x; sy = y; }
    }
  if (sx < 0) return -1;
  uint64_t s = seed;
  int x = sx, y = sy;
  for (int k = 0; k < n; ++k) {
    int u = (int)(u01(&s) * 9.0);
    if (u > 8) u = 8;
    float T81[81], L16[16];
    orc_cell_model(H, W, map, x, y, gx, gy, T81, NULL, NULL, NULL);
    double r = u01(&s), c = 0.0;
    int j = 4;
    for (int i = 0; i < 9; ++i) {
      c += T81[9 * u + i];
      if (T81[9 * u + i] > 0.0f && r < c) { j = i; break; }
    }
    x += j % 3 - 1;
    y += j / 3 - 1;
    orc_cell_model(H, W, map, x, y, gx, gy, NULL, L16, NULL, NULL);
    r = u01(&s);
    c = 0.0;
    int z = 15;
    for (int i = 0; i < 16; ++i) {
      c += L16[i];
      if (r < c) { z = i; break; }
    }
    us[k] = (uint8_t)u;
    zs[k] = (uint8_t)z;
    if (states) states[k] = y * W + x;
  }
  return 0;
}
