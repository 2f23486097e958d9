/*
 * pp2_oracle_tree.c -- CPU restatement of the QV-tree online planner.
 * TEST INFRASTRUCTURE ONLY (see pp2_oracle.h).  Parity unpinned by reference
 * tests (none exist); follows, with every node holding its own host belief
 * exactly like the reference:
 *   QNode / VNode / SearchTree  include/path_planning_2d/search_tree.h:31-165
 *   QNode ctor / update          src/pomdp/search_tree_cuda.cu:161-286
 *   forwardSampling              :84-147, :311-366
 *   VNode ctor / update / expand :368-450
 *   SearchTree expand / update   :490-626
 *   plan step                    src/pomdp/path_planning_2d.cu:199-241
 * Lower bound: the reference's commented constant fallback -5/(1-gamma)
 * (search_tree_cuda.cu:382-383); upper bound evaluateFibCpu.
 */
#include <float.h>
#include <stdlib.h>
#include <string.h>

#include "pp2_oracle.h"

typedef struct OQ OQ;
typedef struct OV OV;

struct OV {
  float* belief;
  uint8_t observation;
  float weight;
  OQ* parent;
  OQ* children[9];
  int nchildren;
  float ub, lb, heuristic;
  OV* vte;
  uint32_t depth;
};

struct OQ {
  float* belief;
  uint8_t action;
  OV* parent;
  OV* children[16];
  int nchildren;
  float ub, lb, heuristic, reward;
  OV* vte;
  uint32_t depth;
};

struct orc_planner {
  int H, W;
  size_t n;
  const float *T, *L, *R, *alphas;
  float gamma, lb_const;
  int max_depth, max_iter;
  int accurate; /* 1: fp64 accumulation of sums/dots (accuracy reference) */
  uint32_t sample_num;
  float* u1;
  float* u2;
  orc_rand_state rng;
  int pbvi_S;                 /* > 0: PBVI lower bounds (evaluatePbviCpu, :379) */
  const float* pbvi_alphas;   /* [S][hw] */
  const uint8_t* pbvi_actions;
  OV* root;
  uint32_t n_vnodes, n_qnodes, expansions;
};

static OV* ov_new(orc_planner* p, const float* b, uint8_t z, float w, OQ* parent) {
  OV* v = (OV*)calloc(1, sizeof(OV));
  v->belief = (float*)malloc(p->n * sizeof(float));
  memcpy(v->belief, b, p->n * sizeof(float));
  v->observation = z;
  v->weight = w;
  v->parent = parent;
  uint8_t dummy;
  if (p->accurate) {
    double f[9] = {0};
    for (size_t k = 0; k < p->n; ++k)
      for (int i = 0; i < 9; ++i) f[i] += (double)v->belief[k] * p->alphas[9 * k + i];
    int best = 0;
    for (int i = 1; i < 9; ++i) if ((float)f[best] < (float)f[i]) best = i;
    v->ub = (float)f[best];
  } else {
    orc_fib_eval(p->n, v->belief, p->alphas, &v->ub, &dummy);
  }
  if (p->pbvi_S > 0) {
    if (p->accurate) {
      float best = 0.0f;
      for (int k = 0; k < p->pbvi_S; ++k) {
        double d = 0.0;
        const float* al = p->pbvi_alphas + (size_t)k * p->n;
        for (size_t x = 0; x < p->n; ++x) d += (double)v->belief[x] * al[x];
        if (k == 0 || best < (float)d) best = (float)d;
      }
      v->lb = best;
    } else {
      orc_pbvi_eval(p->n, v->belief, p->pbvi_S, p->pbvi_alphas, p->pbvi_actions, &v->lb, &dummy);
    }
  } else {
    v->lb = p->lb_const;
  }
  v->heuristic = v->ub - v->lb;
  v->vte = v;
  v->depth = 0;
  ++p->n_vnodes;
  return v;
}

static void oq_update(orc_planner* p, OQ* q) {
  float ur = 0.0f, lr = 0.0f;
  for (int i = 0; i < q->nchildren; ++i) {
    ur = ur + q->children[i]->ub * q->children[i]->weight;
    lr = lr + q->children[i]->lb * q->children[i]->weight;
  }
  q->ub = q->reward + p->gamma * ur;
  q->lb = q->reward + p->gamma * lr;
  q->heuristic = 0.0f;
  for (int i = 0; i < q->nchildren; ++i) {
    OV* v = q->children[i];
    float h = p->gamma * v->weight * v->heuristic;
    if (h > q->heuristic) { q->heuristic = h; q->vte = v->vte; }
  }
  uint32_t cd = 0;
  for (int i = 0; i < q->nchildren; ++i)
    if (q->children[i]->depth > cd) { cd = q->children[i]->depth; q->depth = cd + 1; }
}

static void ov_update(OV* v) {
  int ui = 0, li = 0;
  for (int i = 1; i < v->nchildren; ++i) {
    if (v->children[ui]->ub < v->children[i]->ub) ui = i;
    if (v->children[li]->lb < v->children[i]->lb) li = i;
  }
  v->ub = v->children[ui]->ub;
  v->lb = v->children[li]->lb;
  v->heuristic = -FLT_MAX;
  for (int i = 0; i < v->nchildren; ++i) {
    OQ* q = v->children[i];
    if (q->ub <= v->lb) continue;
    if (q->heuristic > v->heuristic) { v->heuristic = q->heuristic; v->vte = q->vte; }
  }
  uint32_t cd = 0;
  for (int i = 0; i < v->nchildren; ++i)
    if (v->children[i]->depth > cd) { cd = v->children[i]->depth; v->depth = cd + 1; }
}

static void forward_sampling(orc_planner* p, const float* b, uint8_t a, uint8_t* obs) {
  size_t n = p->n;
  float* cdf = (float*)malloc(n * sizeof(float));
  float acc = 0.0f;
  for (size_t i = 0; i < n; ++i) { acc = acc + b[i]; cdf[i] = acc; }
  for (uint32_t j = 0; j < p->sample_num; ++j) {
    float r = (float)orc_rand_next(&p->rng) / ((float)2147483647 + 1.0f);
    size_t s1 = n; /* find_if(x >= r) */
    for (size_t i = 0; i < n; ++i)
      if (cdf[i] >= r) { s1 = i; break; }
    if (s1 >= n) { /* same clamp as the product (reference reads out of bounds) */
      s1 = n - 1;
      while (s1 > 0 && cdf[s1] == cdf[s1 - 1]) --s1;
    }
    float td[9];
    for (int i = 0; i < 9; ++i) td[i] = p->T[s1 * 81 + 9 * a + i];
    for (int i = 1; i < 9; ++i) td[i] += td[i - 1];
    uint32_t s2 = 0;
    for (uint32_t i = 0; i < 9; ++i)
      if (p->u1[j] <= td[i]) { s2 = i; break; }
    s2 = (uint32_t)s1 + (s2 / 3 - 1) * (uint32_t)p->W + (s2 % 3 - 1);
    float ld[16];
    for (int i = 0; i < 16; ++i) ld[i] = p->L[(size_t)s2 * 16 + i];
    for (int i = 1; i < 16; ++i) ld[i] += ld[i - 1];
    uint8_t o = 0;
    for (uint8_t i = 0; i < 16; ++i)
      if (p->u2[j] <= ld[i]) { o = i; break; }
    obs[j] = o;
  }
  free(cdf);
}

static OQ* oq_new(orc_planner* p, const float* b, uint8_t a, OV* parent) {
  OQ* q = (OQ*)calloc(1, sizeof(OQ));
  q->belief = (float*)malloc(p->n * sizeof(float));
  memcpy(q->belief, b, p->n * sizeof(float));
  q->action = a;
  q->parent = parent;
  q->ub = FLT_MAX;
  q->lb = -FLT_MAX;
  q->heuristic = FLT_MIN;
  q->depth = 1;
  ++p->n_qnodes;
  if (p->accurate) {
    double r = 0.0;
    for (size_t k = 0; k < p->n; ++k) r += (double)q->belief[k] * p->R[9 * k + a];
    q->reward = (float)r;
  } else {
    q->reward = orc_reward_dot(p->n, q->belief, p->R, a);
  }
  uint8_t* obs = (uint8_t*)malloc(p->sample_num);
  forward_sampling(p, q->belief, a, obs);
  int count[16] = {0};
  for (uint32_t j = 0; j < p->sample_num; ++j) ++count[obs[j]];
  free(obs);
  float* out = (float*)malloc(p->n * sizeof(float));
  for (int z = 0; z < 16; ++z) { /* std::set: ascending */
    if (!count[z]) continue;
    float w = (float)count[z] / (float)p->sample_num;
    orc_belief_update(p->H, p->W, p->T, p->L, q->belief, a, z, out, 1);
    if (p->accurate) orc_normalize_f64(p->n, out);
    else orc_normalize_seq(p->n, out);
    q->children[q->nchildren++] = ov_new(p, out, (uint8_t)z, w, q);
  }
  free(out);
  oq_update(p, q);
  return q;
}

static void delete_ov(orc_planner* p, OV* v);
static void delete_oq(orc_planner* p, OQ* q) {
  for (int i = 0; i < q->nchildren; ++i) delete_ov(p, q->children[i]);
  free(q->belief);
  free(q);
  --p->n_qnodes;
}
static void delete_ov(orc_planner* p, OV* v) {
  for (int i = 0; i < v->nchildren; ++i) delete_oq(p, v->children[i]);
  free(v->belief);
  free(v);
  --p->n_vnodes;
}

static void ov_expand(orc_planner* p, OV* v) {
  for (int i = 0; i < v->nchildren; ++i) delete_oq(p, v->children[i]);
  v->nchildren = 9;
  for (uint8_t a = 0; a < 9; ++a) v->children[a] = oq_new(p, v->belief, a, v);
  ov_update(v);
  ++p->expansions;
}

static int tree_expand(orc_planner* p) {
  OV* vte = p->root->vte;
  if (!vte) return -1;
  ov_expand(p, vte);
  OV* v = vte;
  while (v->parent) {
    OQ* q = v->parent;
    oq_update(p, q);
    OV* pv = q->parent;
    ov_update(pv);
    v = pv;
  }
  return 0;
}

static void tree_update(orc_planner* p, uint8_t a, uint8_t z) {
  OV* root = p->root;
  OQ* rq = NULL;
  for (int i = 0; i < root->nchildren; ++i) {
    if (root->children[i]->action == a) rq = root->children[i];
    else delete_oq(p, root->children[i]);
  }
  root->nchildren = 0;
  OV* rv = NULL;
  if (rq) {
    for (int i = 0; i < rq->nchildren; ++i) {
      if (rq->children[i]->observation == z) rv = rq->children[i];
      else delete_ov(p, rq->children[i]);
    }
    rq->nchildren = 0;
  }
  if (rv) {
    free(rq->belief); free(rq); --p->n_qnodes;
    free(root->belief); free(root); --p->n_vnodes;
    rv->parent = NULL;
    p->root = rv;
    return;
  }
  float* cur = (float*)malloc(p->n * sizeof(float));
  orc_belief_update(p->H, p->W, p->T, p->L, root->belief, a, z, cur, 1);
  if (p->accurate) orc_normalize_f64(p->n, cur);
  else orc_normalize_seq(p->n, cur);
  OV* nv = ov_new(p, cur, 0, 0.0f, NULL);
  free(cur);
  if (rq) { free(rq->belief); free(rq); --p->n_qnodes; }
  free(root->belief); free(root); --p->n_vnodes;
  p->root = nv;
}

orc_planner* orc_planner_create(int H, int W, const float* T, const float* L,
                                const float* R, const float* alphas, float gamma,
                                int max_depth, int max_iter, uint32_t rand_seed,
                                uint32_t sample_num, uint64_t curand_seed,
                                int accurate) {
  orc_planner* p = (orc_planner*)calloc(1, sizeof(orc_planner));
  p->accurate = accurate;
  p->H = H; p->W = W; p->n = (size_t)H * W;
  p->T = T; p->L = L; p->R = R; p->alphas = alphas;
  p->gamma = gamma;
  p->lb_const = -5.0f / (1.0f - gamma);
  p->max_depth = max_depth; p->max_iter = max_iter;
  p->sample_num = sample_num;
  p->u1 = (float*)malloc(sample_num * sizeof(float));
  p->u2 = (float*)malloc(sample_num * sizeof(float));
  for (uint32_t j = 0; j < sample_num; ++j) {
    uint32_t x[2];
    orc_curand_xorwow(curand_seed, j, 0, 2, x);
    p->u1[j] = orc_curand_uniform(x[0]);
    p->u2[j] = orc_curand_uniform(x[1]);
  }
  orc_rand_seed(&p->rng, rand_seed);
  return p;
}

void orc_planner_set_pbvi(orc_planner* p, int S, const float* alphas, const uint8_t* actions) {
  p->pbvi_S = S;
  p->pbvi_alphas = alphas;
  p->pbvi_actions = actions;
}

void orc_planner_skip_rand(orc_planner* p, uint64_t n) {
  for (uint64_t k = 0; k < n; ++k) (void)orc_rand_next(&p->rng);
}

void orc_planner_reset(orc_planner* p) {
  if (p->root) delete_ov(p, p->root);
  p->root = NULL;
}

void orc_planner_destroy(orc_planner* p) {
  if (!p) return;
  orc_planner_reset(p);
  free(p->u1); free(p->u2);
  free(p);
}

int orc_planner_step(orc_planner* p, uint8_t a, uint8_t z, const float* belief,
                     uint8_t* new_action, float* new_value) {
  if (!p->root) {
    if (!belief) return -1;
    p->root = ov_new(p, belief, 0, 0.0f, NULL);
  } else {
    tree_update(p, a, z);
  }
  int counter = 0;
  while (p->root->depth < (uint32_t)p->max_depth && counter++ < p->max_iter)
    if (tree_expand(p) != 0) return -2;
  uint8_t best = 0;
  float r = -FLT_MAX;
  for (int i = 0; i < p->root->nchildren; ++i)
    if (p->root->children[i]->ub > r) { r = p->root->children[i]->ub; best = p->root->children[i]->action; }
  *new_action = best;
  *new_value = r;
  return 0;
}

void orc_planner_info(orc_planner* p, orc_tree_info* info) {
  memset(info, 0, sizeof *info);
  info->total_vnodes = p->n_vnodes;
  info->total_qnodes = p->n_qnodes;
  info->expansions = p->expansions;
  OV* r = p->root;
  if (!r) return;
  info->depth = r->depth;
  info->root_upper_bound = r->ub;
  info->root_lower_bound = r->lb;
  info->root_heuristic = r->heuristic;
  info->n_root_children = (uint32_t)r->nchildren;
  for (int a = 0; a < r->nchildren; ++a) {
    OQ* q = r->children[a];
    info->q_upper_bound[a] = q->ub;
    info->q_lower_bound[a] = q->lb;
    info->q_reward[a] = q->reward;
    info->q_heuristic[a] = q->heuristic;
    info->q_depth[a] = q->depth;
    info->q_nchildren[a] = (uint32_t)q->nchildren;
    for (int k = 0; k < q->nchildren; ++k) {
      info->q_obs[a][k] = q->children[k]->observation;
      info->q_weight[a][k] = q->children[k]->weight;
      info->v_upper_bound[a][k] = q->children[k]->ub;
      info->v_lower_bound[a][k] = q->children[k]->lb;
    }
  }
}
