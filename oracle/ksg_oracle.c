/*
 * ksg_oracle.c — CPU restatement of the kube-scheduler generic scheduler
 * (smarterclayton/kubernetes v0.13.0-dev) over the interned inputs of
 * include/kschedgpu.h.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the checker for the HIP path and the
 * `cpu_baseline` leg of bench.py. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may load liboracle.so. The product library
 * (kubernetes_amd/libkschedgpu.so) never links or calls it.
 *
 * Parity pinning: the restatement is checked against the golden vectors
 * transcribed from the reference's own Go tests (tests/golden/, via the
 * object-level model oracle/ref_model.py and the Python ingest), see
 * tests/test_oracle_golden.py and tests/test_oracle_crosscheck.py. The Go
 * stdlib math/rand stream is not reproducible here (no Go toolchain); the
 * tie-break source is the injected splitmix64 stream.
 *
 * Two modes that must agree bit-for-bit (tests/test_oracle_crosscheck.py):
 *   faithful    — the reference's cost structure: every Schedule regroups all
 *                 placed pods by host (MapPodsToMachines, predicates.go:354-375),
 *                 runs each predicate per node rescanning that node's pods,
 *                 re-derives every priority from the pod list, builds a
 *                 HostPriorityList and sorts it (generic_scheduler.go:84-96).
 *   incremental — per-node totals/bitsets updated on commit, closed forms.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/kschedgpu.h"

typedef struct {
  uint64_t uid;
  uint32_t host;
  int64_t cpu, mem;
  uint32_t *keys_port, n_port;
  uint32_t *keys_pd, n_pd;
  uint32_t *svcs, n_svcs;
  uint64_t seq;
  int alive;
  int64_t scalar[KSG_MAX_SCALAR]; /* extension: extended resource requests */
} opod;

typedef struct orc {
  ksg_config cfg;
  int faithful;
  /* cluster */
  uint32_t N, n_pairs, S;
  int64_t *cap_c, *cap_m;
  uint32_t **node_pairs; /* per node list */
  uint32_t *node_np;
  uint32_t *pair_keys;   /* label-key id (KSG_PAIR_INVALID stripped) */
  uint8_t *pair_bad;     /* SelectorFromSet would reject the pair (selector.go:654-668) */
  /* placed pods, in insertion order (the lister order we canonicalize to) */
  opod *pods;
  uint32_t n_pods, cap_pods;
  uint64_t seq;
  /* incremental state */
  int64_t *used_c, *used_m;
  uint32_t *key_ref; /* max_conflict_keys x N refcounts */
  int32_t *svc_cnt;  /* S x N */
  int32_t *svc_max, *svc_total;
  /* pending begin */
  int pending;
  ksg_pod pend;
  uint32_t *pend_ids;
  size_t pend_n_ids;
  uint64_t pend_k;
  int64_t pend_M;
  int64_t *scores; /* N */
  uint8_t *fails;  /* N */
  /* extensions (include/kschedgpu.h; later kube-scheduler semantics, parity unpinned) */
  int ext_on;
  ksg_ext_config ext;
  int64_t *scap, *sused;  /* [n_scalar][N] */
  uint32_t **ntaint, *nnt; /* per node taint ids */
  ksg_pod_ext pend_ext;
  /* the node-sharded TaintToleration step (orc_evaluate_ext_tmax): the max soft-taint count
   * over every shard's filtered nodes, supplied by the caller; -1: computed here */
  int32_t tmax_given;
} orc;

#define NONE_SCORE (-0x7fffffffffffffffLL - 1)

/* ------------------------------------------------------------------ utils */
static uint64_t splitmix_next(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* Go int arithmetic wraps (two's complement): combinedScores[host] +=
 * score * weight (generic_scheduler.go:145-159) with weight a Go int */
static int64_t go_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static int64_t go_mul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

static int64_t go_div(int64_t a, int64_t b) {
  if (b == -1) return (int64_t)(0ULL - (uint64_t)a);
  return a / b;
}

/* calculateScore, priorities.go:27-37 (Go int64: wrapping multiply) */
static int64_t calculate_score(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  int64_t diff = (int64_t)((uint64_t)capacity - (uint64_t)requested);
  int64_t prod = (int64_t)((uint64_t)diff * 10ULL);
  return go_div(prod, capacity);
}

/* int(10 * (float32(num) / float32(den))), spreading.go:79-83,156-160 */
static int64_t frac10_f32(int64_t num, int64_t den) {
  volatile float a = (float)num;
  volatile float b = (float)den;
  volatile float q = a / b;
  volatile float s = 10.0f * q;
  return (int64_t)s;
}

static int node_has_key(const orc *o, uint32_t n, uint32_t key) {
  for (uint32_t i = 0; i < o->node_np[n]; ++i)
    if (o->pair_keys[o->node_pairs[n][i]] == key) return 1;
  return 0;
}

static int node_has_pair(const orc *o, uint32_t n, uint32_t pair) {
  if (pair == 0) return 0;
  for (uint32_t i = 0; i < o->node_np[n]; ++i)
    if (o->node_pairs[n][i] == pair) return 1;
  return 0;
}

/* pair id of the node's value for label key, or -1 */
static int32_t node_pair_for_key(const orc *o, uint32_t n, uint32_t key) {
  int32_t pr = -1;
  for (uint32_t i = 0; i < o->node_np[n]; ++i)
    if (o->pair_keys[o->node_pairs[n][i]] == key) pr = (int32_t)o->node_pairs[n][i];
  return pr;
}

static int pod_in_service(const opod *p, uint32_t s) {
  for (uint32_t i = 0; i < p->n_svcs; ++i)
    if (p->svcs[i] == s) return 1;
  return 0;
}

/* --------------------------------------------------------------- lifecycle */
orc *orc_create(const ksg_config *cfg, int faithful) {
  orc *o = (orc *)calloc(1, sizeof(orc));
  o->cfg = *cfg;
  if (o->cfg.max_conflict_keys == 0) o->cfg.max_conflict_keys = 1024;
  o->faithful = faithful;
  o->tmax_given = -1;
  return o;
}

static void free_pods(orc *o) {
  for (uint32_t i = 0; i < o->n_pods; ++i) {
    free(o->pods[i].keys_port);
    free(o->pods[i].keys_pd);
    free(o->pods[i].svcs);
  }
  free(o->pods);
  o->pods = NULL;
  o->n_pods = o->cap_pods = 0;
}

static void free_ext(orc *o) {
  if (o->ntaint)
    for (uint32_t n = 0; n < o->N; ++n) free(o->ntaint[n]);
  free(o->ntaint);
  free(o->nnt);
  free(o->scap);
  free(o->sused);
  o->ntaint = NULL;
  o->nnt = NULL;
  o->scap = o->sused = NULL;
}

static void free_cluster(orc *o) {
  free_ext(o);
  for (uint32_t n = 0; n < o->N; ++n) free(o->node_pairs[n]);
  free(o->node_pairs);
  free(o->node_np);
  free(o->cap_c);
  free(o->cap_m);
  free(o->pair_keys);
  free(o->pair_bad);
  free(o->used_c);
  free(o->used_m);
  free(o->key_ref);
  free(o->svc_cnt);
  free(o->svc_max);
  free(o->svc_total);
  free(o->scores);
  free(o->fails);
  free_pods(o);
  o->node_pairs = NULL;
  o->node_np = NULL;
  o->cap_c = o->cap_m = NULL;
  o->pair_keys = NULL;
  o->pair_bad = NULL;
  o->used_c = o->used_m = NULL;
  o->key_ref = NULL;
  o->svc_cnt = o->svc_max = o->svc_total = NULL;
  o->scores = NULL;
  o->fails = NULL;
}

void orc_destroy(orc *o) {
  if (!o) return;
  free_cluster(o);
  free(o->pend_ids);
  free(o);
}

int orc_set_cluster(orc *o, const ksg_node *nodes, uint32_t n_nodes, const uint32_t *node_pairs,
                    uint32_t n_node_pairs, const uint32_t *pair_keys, uint32_t n_pairs,
                    uint32_t n_services) {
  (void)n_node_pairs;
  free_cluster(o);
  if (n_pairs == 0) n_pairs = 1;
  o->N = n_nodes;
  o->n_pairs = n_pairs;
  o->S = n_services;
  size_t NN = n_nodes ? n_nodes : 1;
  o->cap_c = (int64_t *)calloc(NN, 8);
  o->cap_m = (int64_t *)calloc(NN, 8);
  o->node_pairs = (uint32_t **)calloc(NN, sizeof(uint32_t *));
  o->node_np = (uint32_t *)calloc(NN, 4);
  o->pair_keys = (uint32_t *)calloc(n_pairs, 4);
  o->pair_bad = (uint8_t *)calloc(n_pairs, 1);
  o->pair_keys[0] = 0xffffffffu;
  for (uint32_t p = 1; p < n_pairs; ++p) {
    o->pair_keys[p] = pair_keys[p] & ~KSG_PAIR_INVALID;
    o->pair_bad[p] = (pair_keys[p] & KSG_PAIR_INVALID) != 0;
  }
  for (uint32_t n = 0; n < n_nodes; ++n) {
    o->cap_c[n] = nodes[n].cap_milli_cpu;
    o->cap_m[n] = nodes[n].cap_memory;
    o->node_np[n] = nodes[n].n_labels;
    o->node_pairs[n] = (uint32_t *)calloc(nodes[n].n_labels ? nodes[n].n_labels : 1, 4);
    memcpy(o->node_pairs[n], node_pairs + nodes[n].label_off, (size_t)nodes[n].n_labels * 4);
  }
  o->used_c = (int64_t *)calloc(NN, 8);
  o->used_m = (int64_t *)calloc(NN, 8);
  o->key_ref = (uint32_t *)calloc((size_t)o->cfg.max_conflict_keys * NN, 4);
  o->svc_cnt = (int32_t *)calloc((size_t)(n_services ? n_services : 1) * NN, 4);
  o->svc_max = (int32_t *)calloc(n_services ? n_services : 1, 4);
  o->svc_total = (int32_t *)calloc(n_services ? n_services : 1, 4);
  o->scores = (int64_t *)calloc(NN, 8);
  o->fails = (uint8_t *)calloc(NN, 1);
  o->seq = 0;
  o->pending = 0;
  return KSG_OK;
}

/* ------------------------------------------------------------- pod store */
static uint32_t *dup_ids(const uint32_t *ids, uint32_t off, uint32_t n) {
  uint32_t *r = (uint32_t *)malloc((n ? n : 1) * 4);
  if (n) memcpy(r, ids + off, (size_t)n * 4);
  return r;
}

static int32_t ext_count(const orc *o, uint32_t s, uint32_t host) {
  int32_t c = 0;
  for (uint32_t i = 0; i < o->n_pods; ++i)
    if (o->pods[i].alive && o->pods[i].host == host && pod_in_service(&o->pods[i], s)) ++c;
  return c;
}

static void recompute_svc_max(orc *o, uint32_t s) {
  /* maxCount over all hosts incl. hosts not in the node list (spreading.go:73-80) */
  int32_t m = 0;
  for (uint32_t n = 0; n < o->N; ++n)
    if (o->svc_cnt[(size_t)s * o->N + n] > m) m = o->svc_cnt[(size_t)s * o->N + n];
  for (uint32_t i = 0; i < o->n_pods; ++i) {
    const opod *p = &o->pods[i];
    if (p->alive && p->host >= o->N && pod_in_service(p, s)) {
      int32_t c = ext_count(o, s, p->host);
      if (c > m) m = c;
    }
  }
  o->svc_max[s] = m;
}

int orc_add_pod_ext(orc *o, uint32_t host_id, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids);
int orc_add_pod(orc *o, uint32_t host_id, const ksg_pod *p, const uint32_t *ids) {
  return orc_add_pod_ext(o, host_id, p, NULL, ids);
}

int orc_add_pod_ext(orc *o, uint32_t host_id, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids) {
  if (o->n_pods == o->cap_pods) {
    o->cap_pods = o->cap_pods ? o->cap_pods * 2 : 256;
    o->pods = (opod *)realloc(o->pods, (size_t)o->cap_pods * sizeof(opod));
  }
  opod *q = &o->pods[o->n_pods++];
  q->uid = p->uid;
  q->host = host_id;
  q->cpu = p->milli_cpu;
  q->mem = p->memory;
  q->keys_port = dup_ids(ids, p->ports_off, p->n_ports);
  q->n_port = p->n_ports;
  q->keys_pd = dup_ids(ids, p->pds_off, p->n_pds);
  q->n_pd = p->n_pds;
  q->svcs = dup_ids(ids, p->svcs_off, p->n_svcs);
  q->n_svcs = p->n_svcs;
  q->seq = ++o->seq;
  q->alive = 1;
  for (int r = 0; r < KSG_MAX_SCALAR; ++r) q->scalar[r] = (e && o->ext_on && (uint32_t)r < o->ext.n_scalar) ? e->scalar[r] : 0;
  if (host_id < o->N && o->sused)
    for (uint32_t r = 0; r < o->ext.n_scalar; ++r)
      o->sused[(size_t)r * o->N + host_id] = (int64_t)((uint64_t)o->sused[(size_t)r * o->N + host_id] + (uint64_t)q->scalar[r]);
  if (host_id < o->N) {
    o->used_c[host_id] = (int64_t)((uint64_t)o->used_c[host_id] + (uint64_t)q->cpu);
    o->used_m[host_id] = (int64_t)((uint64_t)o->used_m[host_id] + (uint64_t)q->mem);
    for (uint32_t i = 0; i < q->n_port; ++i) o->key_ref[(size_t)q->keys_port[i] * o->N + host_id]++;
    for (uint32_t i = 0; i < q->n_pd; ++i) o->key_ref[(size_t)q->keys_pd[i] * o->N + host_id]++;
  }
  for (uint32_t i = 0; i < q->n_svcs; ++i) {
    uint32_t s = q->svcs[i];
    int32_t v;
    if (host_id < o->N)
      v = ++o->svc_cnt[(size_t)s * o->N + host_id];
    else
      v = ext_count(o, s, host_id);
    if (v > o->svc_max[s]) o->svc_max[s] = v;
    o->svc_total[s]++;
  }
  return KSG_OK;
}

int orc_remove_pod(orc *o, uint64_t uid) {
  for (uint32_t i = 0; i < o->n_pods; ++i) {
    opod *q = &o->pods[i];
    if (!q->alive || q->uid != uid) continue;
    q->alive = 0;
    uint32_t h = q->host;
    if (h < o->N && o->sused)
      for (uint32_t r = 0; r < o->ext.n_scalar; ++r)
        o->sused[(size_t)r * o->N + h] = (int64_t)((uint64_t)o->sused[(size_t)r * o->N + h] - (uint64_t)q->scalar[r]);
    if (h < o->N) {
      o->used_c[h] = (int64_t)((uint64_t)o->used_c[h] - (uint64_t)q->cpu);
      o->used_m[h] = (int64_t)((uint64_t)o->used_m[h] - (uint64_t)q->mem);
      for (uint32_t k = 0; k < q->n_port; ++k) o->key_ref[(size_t)q->keys_port[k] * o->N + h]--;
      for (uint32_t k = 0; k < q->n_pd; ++k) o->key_ref[(size_t)q->keys_pd[k] * o->N + h]--;
    }
    for (uint32_t k = 0; k < q->n_svcs; ++k) {
      uint32_t s = q->svcs[k];
      if (h < o->N) o->svc_cnt[(size_t)s * o->N + h]--;
      o->svc_total[s]--;
      recompute_svc_max(o, s);
    }
    return KSG_OK;
  }
  return KSG_ERR_ARG;
}

/* first service peer = earliest-added live pod matching service s
 * (canonical order for nsServicePods[0], predicates.go:293) */
static const opod *first_peer(const orc *o, uint32_t s) {
  const opod *best = NULL;
  for (uint32_t i = 0; i < o->n_pods; ++i) {
    const opod *p = &o->pods[i];
    if (p->alive && pod_in_service(p, s) && (!best || p->seq < best->seq)) best = p;
  }
  return best;
}

/* ------------------------------------------------------- pod-level context */
typedef struct {
  const ksg_pod *p;
  const uint32_t *ids;
  int32_t req_aff[KSG_MAX_AFF];
  int error;
  const ksg_pod_ext *ext; /* extensions (NULL: none) */
} pctx;

/* ---------------------------------------------------------- extensions
 * Not in the reference; the published kube-scheduler v1.10 algorithms,
 * restated (parity unpinned): PodToleratesNodeTaints (an untolerated
 * NoSchedule / NoExecute taint fails the node), PodFitsResources'
 * ScalarResources (allocatable < requested + request fails), TaintToleration
 * priority (untolerated PreferNoSchedule taints, NormalizeReduce(10, reverse))
 * and BalancedResourceAllocation (float64, over the same requested totals as
 * LeastRequested here). */
static int node_has_taint(const orc *o, uint32_t n, uint32_t t) {
  for (uint32_t i = 0; i < o->nnt[n]; ++i)
    if (o->ntaint[n][i] == t) return 1;
  return 0;
}

/* used: the node's extended-resource requests (per resource) */
static int ext_fail_code(const orc *o, const pctx *c, uint32_t n, const int64_t *used) {
  if (!o->ext_on || !c->ext) return KSG_FAIL_NONE;
  if (o->ext.filters & KSG_EXT_TAINTS)
    for (uint32_t i = 0; i < c->ext->n_hard; ++i)
      if (node_has_taint(o, n, c->ids[c->ext->hard_off + i])) return KSG_FAIL_TAINTS;
  if (o->ext.filters & KSG_EXT_SCALAR)
    for (uint32_t r = 0; r < o->ext.n_scalar; ++r) {
      int64_t req = c->ext->scalar[r];
      if (req > 0 && o->scap[(size_t)r * o->N + n] < (int64_t)((uint64_t)used[r] + (uint64_t)req)) return KSG_FAIL_SCALAR;
    }
  return KSG_FAIL_NONE;
}

static int64_t balanced_score(int64_t tc, int64_t cc, int64_t tm, int64_t cm) {
  volatile double fc = cc == 0 ? 1.0 : (double)tc / (double)cc;
  volatile double fm = cm == 0 ? 1.0 : (double)tm / (double)cm;
  if (fc >= 1.0 || fm >= 1.0) return 0;
  volatile double diff = fabs(fc - fm);
  volatile double one_minus = 1.0 - diff;
  volatile double v = one_minus * 10.0;
  return (int64_t)v;
}

static int32_t soft_taints(const orc *o, const pctx *c, uint32_t n) {
  int32_t k = 0;
  for (uint32_t i = 0; i < c->ext->n_soft; ++i) k += node_has_taint(o, n, c->ids[c->ext->soft_off + i]);
  return k;
}

/* the extension priorities over the filtered nodes; tc/tm: requested totals incl. the pod */
static void ext_prioritize(const orc *o, const pctx *c, const uint8_t *fails, int64_t *score, const int64_t *tc,
                           const int64_t *tm) {
  if (!o->ext_on) return;
  if (o->ext.w_balanced)
    for (uint32_t n = 0; n < o->N; ++n)
      if (!fails[n]) score[n] = go_add(score[n], go_mul(o->ext.w_balanced, balanced_score(tc[n], o->cap_c[n], tm[n], o->cap_m[n])));
  if (o->ext.w_taint_toleration && c->ext) {
    int32_t mx = 0;
    if (o->tmax_given >= 0)
      mx = o->tmax_given;
    else
      for (uint32_t n = 0; n < o->N; ++n)
        if (!fails[n]) {
          int32_t k = soft_taints(o, c, n);
          if (k > mx) mx = k;
        }
    for (uint32_t n = 0; n < o->N; ++n)
      if (!fails[n]) {
        int64_t v = mx == 0 ? 10 : 10 - (10 * (int64_t)soft_taints(o, c, n)) / mx;
        score[n] = go_add(score[n], go_mul(o->ext.w_taint_toleration, v));
      }
  } else if (o->ext.w_taint_toleration) {
    for (uint32_t n = 0; n < o->N; ++n)
      if (!fails[n]) score[n] = go_add(score[n], go_mul(o->ext.w_taint_toleration, 10));
  }
}

static int ext_prio_on(const orc *o) { return o->ext_on && (o->ext.w_taint_toleration || o->ext.w_balanced); }

/* CheckServiceAffinity (predicates.go:257-324) for every ServiceAffinity
 * predicate at once: req_aff[j] = the value label j must have (pair id), the
 * pod's own nodeSelector value first (:261-271), else the first service peer's
 * node's (:274-307); then SelectorFromSet's trap per predicate (:311-315,
 * labels.go:60-61, selector.go:654-668): a predicate whose affinity map holds
 * an invalid (key, value) matches every node, so its labels stay required only
 * through the predicates that are valid. req_aff[j] < 0: no requirement. */
static void resolve_affinity(const orc *o, pctx *c) {
  c->error = 0;
  for (int j = 0; j < KSG_MAX_AFF; ++j) c->req_aff[j] = -1;
  if (!(o->cfg.predicates & KSG_PRED_SERVICEAFFINITY)) return;
  const uint32_t J = o->cfg.n_aff_labels;
  int all_given = 1;
  for (uint32_t j = 0; j < J; ++j) {
    c->req_aff[j] = c->p->aff_pair[j];
    if (c->p->aff_pair[j] == -1) all_given = 0; /* KSG_AFF_INVALID: given (invalid) */
  }
  if (!all_given && c->p->service >= 0) {
    const opod *peer = first_peer(o, (uint32_t)c->p->service);
    if (peer) {
      if (peer->host >= o->N) {
        c->error = 1; /* GetNodeInfo(peer's Status.Host) fails, predicates.go:293-296 */
        return;
      }
      for (uint32_t j = 0; j < J; ++j)
        if (c->req_aff[j] == -1) {
          int32_t pr = node_pair_for_key(o, peer->host, o->cfg.aff_key[j]);
          c->req_aff[j] = (pr > 0 && o->pair_bad[pr]) ? KSG_AFF_INVALID : pr;
        }
    }
  }
  /* one predicate per group; n_aff_groups == 0: one predicate over every label */
  uint32_t ng = o->cfg.n_aff_groups, masks[KSG_MAX_AFF_GROUPS];
  for (uint32_t g = 0; g < ng; ++g) masks[g] = o->cfg.aff_group_mask[g];
  if (ng == 0) {
    ng = 1;
    masks[0] = (1u << J) - 1u;
  }
  uint32_t active = 0;
  for (uint32_t g = 0; g < ng; ++g) {
    int trapped = 0;
    for (uint32_t j = 0; j < J; ++j)
      if (((masks[g] >> j) & 1u) && c->req_aff[j] == KSG_AFF_INVALID) trapped = 1;
    if (!trapped) active |= masks[g];
  }
  for (uint32_t j = 0; j < J; ++j)
    if (!((active >> j) & 1u)) c->req_aff[j] = -1;
}

/* ================================================================ FAITHFUL */
/* MapPodsToMachines: group every placed pod by Status.Host (predicates.go:354-375) */
typedef struct {
  uint32_t **lists; /* per node: indices into o->pods */
  uint32_t *len;
} machine_map;

static void map_pods_to_machines(const orc *o, machine_map *m) {
  m->len = (uint32_t *)calloc(o->N ? o->N : 1, 4);
  for (uint32_t i = 0; i < o->n_pods; ++i)
    if (o->pods[i].alive && o->pods[i].host < o->N) m->len[o->pods[i].host]++;
  m->lists = (uint32_t **)calloc(o->N ? o->N : 1, sizeof(uint32_t *));
  for (uint32_t n = 0; n < o->N; ++n) m->lists[n] = (uint32_t *)malloc((m->len[n] ? m->len[n] : 1) * 4);
  uint32_t *fillc = (uint32_t *)calloc(o->N ? o->N : 1, 4);
  for (uint32_t i = 0; i < o->n_pods; ++i)
    if (o->pods[i].alive && o->pods[i].host < o->N) {
      uint32_t h = o->pods[i].host;
      m->lists[h][fillc[h]++] = i;
    }
  free(fillc);
}

static void free_machine_map(const orc *o, machine_map *m) {
  for (uint32_t n = 0; n < o->N; ++n) free(m->lists[n]);
  free(m->lists);
  free(m->len);
}

/* PodFitsPorts / getUsedPorts (predicates.go:326-350) */
static int f_fits_ports(const orc *o, const pctx *c, const machine_map *m, uint32_t n) {
  for (uint32_t w = 0; w < c->p->n_ports; ++w) {
    uint32_t want = c->ids[c->p->ports_off + w];
    for (uint32_t e = 0; e < m->len[n]; ++e) {
      const opod *q = &o->pods[m->lists[n][e]];
      for (uint32_t k = 0; k < q->n_port; ++k)
        if (q->keys_port[k] == want) return 0;
    }
  }
  return 1;
}

/* NoDiskConflict / isVolumeConflict (predicates.go:52-83) */
static int f_no_disk_conflict(const orc *o, const pctx *c, const machine_map *m, uint32_t n) {
  for (uint32_t v = 0; v < c->p->n_pds; ++v) {
    uint32_t pd = c->ids[c->p->pds_off + v];
    for (uint32_t e = 0; e < m->len[n]; ++e) {
      const opod *q = &o->pods[m->lists[n][e]];
      for (uint32_t k = 0; k < q->n_pd; ++k)
        if (q->keys_pd[k] == pd) return 0;
    }
  }
  return 1;
}

/* PodFitsResources / CheckPodsExceedingCapacity (predicates.go:104-145): greedy */
static int f_fits_resources(const orc *o, const pctx *c, const machine_map *m, uint32_t n) {
  if (c->p->milli_cpu == 0 && c->p->memory == 0) return 1;
  int64_t totalC = o->cap_c[n], totalM = o->cap_m[n];
  int64_t reqC = 0, reqM = 0;
  for (uint32_t e = 0; e <= m->len[n]; ++e) {
    int64_t pc, pm;
    if (e < m->len[n]) {
      const opod *q = &o->pods[m->lists[n][e]];
      pc = q->cpu;
      pm = q->mem;
    } else {
      pc = c->p->milli_cpu;
      pm = c->p->memory;
    }
    int fitsC = totalC == 0 || (int64_t)((uint64_t)totalC - (uint64_t)reqC) >= pc;
    int fitsM = totalM == 0 || (int64_t)((uint64_t)totalM - (uint64_t)reqM) >= pm;
    if (!fitsC || !fitsM) return 0; /* exceeding non-empty */
    reqC = (int64_t)((uint64_t)reqC + (uint64_t)pc);
    reqM = (int64_t)((uint64_t)reqM + (uint64_t)pm);
  }
  return 1;
}

/* PodSelectorMatches (predicates.go:161-179) */
static int f_selector(const orc *o, const pctx *c, uint32_t n) {
  for (uint32_t i = 0; i < c->p->n_sel; ++i)
    if (!node_has_pair(o, n, c->ids[c->p->sel_off + i])) return 0;
  return 1;
}

/* CheckNodeLabelPresence (predicates.go:215-229), AND over LabelsPresence predicates */
static int f_labels_presence(const orc *o, uint32_t n) {
  for (uint32_t q = 0; q < o->cfg.n_presence; ++q)
    for (uint32_t i = 0; i < o->cfg.presence_n_keys[q]; ++i) {
      int exists = node_has_key(o, n, o->cfg.presence_keys[q][i]);
      if ((exists && !o->cfg.presence_flag[q]) || (!exists && o->cfg.presence_flag[q])) return 0;
    }
  return 1;
}

static int f_service_affinity(const orc *o, const pctx *c, uint32_t n) {
  for (uint32_t j = 0; j < o->cfg.n_aff_labels; ++j)
    if (c->req_aff[j] >= 0 && !node_has_pair(o, n, (uint32_t)c->req_aff[j])) return 0;
  return 1;
}

static int faithful_fail_code(const orc *o, const pctx *c, const machine_map *m, uint32_t n) {
  uint32_t P = o->cfg.predicates;
  if ((P & KSG_PRED_HOSTNAME) && c->p->host != -1 && (int32_t)n != c->p->host) return KSG_FAIL_HOSTNAME;
  if ((P & KSG_PRED_LABELSPRESENCE) && o->cfg.n_presence && !f_labels_presence(o, n))
    return KSG_FAIL_LABELSPRESENCE;
  if ((P & KSG_PRED_MATCHNODESELECTOR) && !f_selector(o, c, n)) return KSG_FAIL_MATCHNODESELECTOR;
  if ((P & KSG_PRED_NODISKCONFLICT) && !f_no_disk_conflict(o, c, m, n)) return KSG_FAIL_NODISKCONFLICT;
  if ((P & KSG_PRED_PODFITSPORTS) && !f_fits_ports(o, c, m, n)) return KSG_FAIL_PODFITSPORTS;
  if ((P & KSG_PRED_PODFITSRESOURCES) && !f_fits_resources(o, c, m, n)) return KSG_FAIL_PODFITSRESOURCES;
  if ((P & KSG_PRED_SERVICEAFFINITY) && !f_service_affinity(o, c, n)) return KSG_FAIL_SERVICEAFFINITY;
  if (o->ext_on && c->ext) {
    int64_t used[KSG_MAX_SCALAR] = {0};
    for (uint32_t e = 0; e < m->len[n]; ++e)
      for (uint32_t r = 0; r < o->ext.n_scalar; ++r)
        used[r] = (int64_t)((uint64_t)used[r] + (uint64_t)o->pods[m->lists[n][e]].scalar[r]);
    return ext_fail_code(o, c, n, used);
  }
  return KSG_FAIL_NONE;
}

/* prioritizeNodes over the filtered nodes (generic_scheduler.go:136-165).
 * score[n] valid where fails[n]==0. Returns 0 if the HostPriorityList is empty. */
static int faithful_prioritize(orc *o, const pctx *c, const uint8_t *fails, int64_t *score) {
  const ksg_config *cf = &o->cfg;
  uint32_t nfilt = 0;
  for (uint32_t n = 0; n < o->N; ++n) nfilt += fails[n] == 0;
  if (cf->n_priority_configs == 0 && !ext_prio_on(o)) { /* EqualPriority */
    for (uint32_t n = 0; n < o->N; ++n) score[n] = 1;
    return nfilt > 0;
  }
  int any = ext_prio_on(o);
  for (uint32_t n = 0; n < o->N; ++n) score[n] = 0;
  if (ext_prio_on(o)) { /* extensions: requested totals by regrouping, as LeastRequested does */
    machine_map m;
    map_pods_to_machines(o, &m);
    int64_t *tc = (int64_t *)calloc(o->N ? o->N : 1, 8), *tm = (int64_t *)calloc(o->N ? o->N : 1, 8);
    for (uint32_t n = 0; n < o->N; ++n) {
      for (uint32_t e = 0; e < m.len[n]; ++e) {
        tc[n] = (int64_t)((uint64_t)tc[n] + (uint64_t)o->pods[m.lists[n][e]].cpu);
        tm[n] = (int64_t)((uint64_t)tm[n] + (uint64_t)o->pods[m.lists[n][e]].mem);
      }
      tc[n] = (int64_t)((uint64_t)tc[n] + (uint64_t)c->p->milli_cpu);
      tm[n] = (int64_t)((uint64_t)tm[n] + (uint64_t)c->p->memory);
    }
    free_machine_map(o, &m);
    ext_prioritize(o, c, fails, score, tc, tm);
    free(tc);
    free(tm);
  }
  if (cf->w_least_requested) { /* LeastRequestedPriority, priorities.go:43-91 */
    any = 1;
    machine_map m;
    map_pods_to_machines(o, &m);
    for (uint32_t n = 0; n < o->N; ++n) {
      if (fails[n]) continue;
      int64_t tc = 0, tm = 0;
      for (uint32_t e = 0; e < m.len[n]; ++e) {
        const opod *q = &o->pods[m.lists[n][e]];
        tc = (int64_t)((uint64_t)tc + (uint64_t)q->cpu);
        tm = (int64_t)((uint64_t)tm + (uint64_t)q->mem);
      }
      tc = (int64_t)((uint64_t)tc + (uint64_t)c->p->milli_cpu);
      tm = (int64_t)((uint64_t)tm + (uint64_t)c->p->memory);
      int64_t cs = calculate_score(tc, o->cap_c[n]);
      int64_t ms = calculate_score(tm, o->cap_m[n]);
      score[n] = go_add(score[n], go_mul(cf->w_least_requested, ((cs + ms) / 2)));
    }
    free_machine_map(o, &m);
  }
  if (cf->w_service_spreading) { /* CalculateSpreadPriority, spreading.go:37-86 */
    any = 1;
    int32_t *counts = (int32_t *)calloc(o->N ? o->N : 1, 4);
    int32_t maxCount = 0;
    if (c->p->service >= 0) {
      uint32_t s = (uint32_t)c->p->service;
      /* counts by Status.Host over all hosts (incl. unknown ones) */
      for (uint32_t i = 0; i < o->n_pods; ++i) {
        const opod *q = &o->pods[i];
        if (!q->alive || !pod_in_service(q, s)) continue;
        int32_t cnt;
        if (q->host < o->N)
          cnt = ++counts[q->host];
        else {
          cnt = 0;
          for (uint32_t k = 0; k <= i; ++k)
            if (o->pods[k].alive && o->pods[k].host == q->host && pod_in_service(&o->pods[k], s)) ++cnt;
        }
        if (cnt > maxCount) maxCount = cnt;
      }
    }
    for (uint32_t n = 0; n < o->N; ++n) {
      if (fails[n]) continue;
      int64_t sc = maxCount > 0 ? frac10_f32((int64_t)maxCount - counts[n], maxCount) : 10;
      score[n] = go_add(score[n], go_mul(cf->w_service_spreading, sc));
    }
    free(counts);
  }
  for (uint32_t a = 0; a < cf->n_anti; ++a) { /* CalculateAntiAffinityPriority, spreading.go:104-168 */
    if (!cf->w_anti[a]) continue;
    any = 1;
    int32_t *podCounts = (int32_t *)calloc(o->n_pairs, 4); /* by pair id of the label value */
    int64_t nsp = 0;
    if (c->p->service >= 0) {
      uint32_t s = (uint32_t)c->p->service;
      for (uint32_t i = 0; i < o->n_pods; ++i) {
        const opod *q = &o->pods[i];
        if (!q->alive || !pod_in_service(q, s)) continue;
        nsp++;
        if (q->host < o->N && !fails[q->host]) { /* labeledMinions built from filtered nodes */
          int32_t pr = node_pair_for_key(o, q->host, cf->anti_key[a]);
          if (pr >= 0) podCounts[pr]++;
        }
      }
    }
    for (uint32_t n = 0; n < o->N; ++n) {
      if (fails[n]) continue;
      int32_t pr = node_pair_for_key(o, n, cf->anti_key[a]);
      int64_t sc = 0;
      if (pr >= 0) sc = nsp > 0 ? frac10_f32(nsp - podCounts[pr], nsp) : 10;
      score[n] = go_add(score[n], go_mul(cf->w_anti[a], sc));
    }
    free(podCounts);
  }
  for (uint32_t q = 0; q < cf->n_label_pref; ++q) { /* CalculateNodeLabelPriority, priorities.go:109-134 */
    if (!cf->w_pref[q]) continue;
    any = 1;
    for (uint32_t n = 0; n < o->N; ++n) {
      if (fails[n]) continue;
      int exists = node_has_key(o, n, cf->pref_key[q]);
      int ok = (exists && cf->pref_presence[q]) || (!exists && !cf->pref_presence[q]);
      score[n] = go_add(score[n], go_mul(cf->w_pref[q], (ok ? 10 : 0)));
    }
  }
  if (cf->w_equal) {
    any = 1;
    for (uint32_t n = 0; n < o->N; ++n)
      if (!fails[n]) score[n] = go_add(score[n], cf->w_equal);
  }
  return any && nfilt > 0;
}

/* ============================================================= INCREMENTAL */
static int incr_fail_code(const orc *o, const pctx *c, uint32_t n) {
  uint32_t P = o->cfg.predicates;
  if ((P & KSG_PRED_HOSTNAME) && c->p->host != -1 && (int32_t)n != c->p->host) return KSG_FAIL_HOSTNAME;
  if ((P & KSG_PRED_LABELSPRESENCE) && o->cfg.n_presence && !f_labels_presence(o, n))
    return KSG_FAIL_LABELSPRESENCE;
  if ((P & KSG_PRED_MATCHNODESELECTOR) && !f_selector(o, c, n)) return KSG_FAIL_MATCHNODESELECTOR;
  if (P & KSG_PRED_NODISKCONFLICT)
    for (uint32_t i = 0; i < c->p->n_pds; ++i)
      if (o->key_ref[(size_t)c->ids[c->p->pds_off + i] * o->N + n]) return KSG_FAIL_NODISKCONFLICT;
  if (P & KSG_PRED_PODFITSPORTS)
    for (uint32_t i = 0; i < c->p->n_ports; ++i)
      if (o->key_ref[(size_t)c->ids[c->p->ports_off + i] * o->N + n]) return KSG_FAIL_PODFITSPORTS;
  if ((P & KSG_PRED_PODFITSRESOURCES) && !(c->p->milli_cpu == 0 && c->p->memory == 0)) {
    int fc = o->cap_c[n] == 0 || (int64_t)((uint64_t)o->cap_c[n] - (uint64_t)o->used_c[n]) >= c->p->milli_cpu;
    int fm = o->cap_m[n] == 0 || (int64_t)((uint64_t)o->cap_m[n] - (uint64_t)o->used_m[n]) >= c->p->memory;
    if (!(fc && fm)) return KSG_FAIL_PODFITSRESOURCES;
  }
  if ((P & KSG_PRED_SERVICEAFFINITY) && !f_service_affinity(o, c, n)) return KSG_FAIL_SERVICEAFFINITY;
  if (o->ext_on && c->ext) {
    int64_t used[KSG_MAX_SCALAR] = {0};
    for (uint32_t r = 0; r < o->ext.n_scalar; ++r) used[r] = o->sused[(size_t)r * o->N + n];
    return ext_fail_code(o, c, n, used);
  }
  return KSG_FAIL_NONE;
}

/* ext_dcount (n_anti x n_pairs, or NULL): ServiceAntiAffinity's domain counts
 * supplied by the caller (the sum of the node shards' partial counts, as a
 * sharded scan receives them from its all-reduce) instead of computed here */
static int incr_prioritize(orc *o, const pctx *c, const uint8_t *fails, int64_t *score, const int32_t *ext_dcount) {
  const ksg_config *cf = &o->cfg;
  uint32_t nfilt = 0;
  for (uint32_t n = 0; n < o->N; ++n) nfilt += fails[n] == 0;
  if (cf->n_priority_configs == 0 && !ext_prio_on(o)) {
    for (uint32_t n = 0; n < o->N; ++n) score[n] = 1;
    return nfilt > 0;
  }
  int any = cf->w_least_requested || cf->w_service_spreading || cf->w_equal || ext_prio_on(o);
  for (uint32_t q = 0; q < cf->n_label_pref; ++q) any |= cf->w_pref[q] != 0;
  for (uint32_t a = 0; a < cf->n_anti; ++a) any |= cf->w_anti[a] != 0;
  int32_t s = c->p->service;
  int32_t maxc = s >= 0 ? o->svc_max[s] : 0;
  int64_t tot = s >= 0 ? o->svc_total[s] : 0;
  /* anti-affinity domain counts over filtered labelled nodes */
  int32_t *dcount[KSG_MAX_ANTI] = {0};
  for (uint32_t a = 0; a < cf->n_anti; ++a) {
    if (!cf->w_anti[a]) continue;
    if (ext_dcount) {
      dcount[a] = (int32_t *)ext_dcount + (size_t)a * o->n_pairs;
      continue;
    }
    dcount[a] = (int32_t *)calloc(o->n_pairs, 4);
    if (s >= 0)
      for (uint32_t n = 0; n < o->N; ++n) {
        if (fails[n]) continue;
        int32_t pr = node_pair_for_key(o, n, cf->anti_key[a]);
        if (pr >= 0) dcount[a][pr] += o->svc_cnt[(size_t)s * o->N + n];
      }
  }
  for (uint32_t n = 0; n < o->N; ++n) {
    if (fails[n]) continue;
    int64_t sc = 0;
    if (cf->w_least_requested) {
      int64_t tc = (int64_t)((uint64_t)o->used_c[n] + (uint64_t)c->p->milli_cpu);
      int64_t tm = (int64_t)((uint64_t)o->used_m[n] + (uint64_t)c->p->memory);
      sc = go_add(sc, go_mul(cf->w_least_requested, ((calculate_score(tc, o->cap_c[n]) + calculate_score(tm, o->cap_m[n])) / 2)));
    }
    if (cf->w_service_spreading) {
      int32_t cnt = s >= 0 ? o->svc_cnt[(size_t)s * o->N + n] : 0;
      sc = go_add(sc, go_mul(cf->w_service_spreading, (maxc > 0 ? frac10_f32((int64_t)maxc - cnt, maxc) : 10)));
    }
    for (uint32_t a = 0; a < cf->n_anti; ++a) {
      if (!cf->w_anti[a]) continue;
      int32_t pr = node_pair_for_key(o, n, cf->anti_key[a]);
      int64_t v = 0;
      if (pr >= 0) v = tot > 0 ? frac10_f32(tot - dcount[a][pr], tot) : 10;
      sc = go_add(sc, go_mul(cf->w_anti[a], v));
    }
    for (uint32_t q = 0; q < cf->n_label_pref; ++q) {
      if (!cf->w_pref[q]) continue;
      int exists = node_has_key(o, n, cf->pref_key[q]);
      int ok = (exists && cf->pref_presence[q]) || (!exists && !cf->pref_presence[q]);
      sc = go_add(sc, go_mul(cf->w_pref[q], (ok ? 10 : 0)));
    }
    sc = go_add(sc, cf->w_equal);
    score[n] = sc;
  }
  if (ext_prio_on(o)) {
    int64_t *tc = (int64_t *)calloc(o->N ? o->N : 1, 8), *tm = (int64_t *)calloc(o->N ? o->N : 1, 8);
    for (uint32_t n = 0; n < o->N; ++n) {
      tc[n] = (int64_t)((uint64_t)o->used_c[n] + (uint64_t)c->p->milli_cpu);
      tm[n] = (int64_t)((uint64_t)o->used_m[n] + (uint64_t)c->p->memory);
    }
    ext_prioritize(o, c, fails, score, tc, tm);
    free(tc);
    free(tm);
  }
  if (!ext_dcount)
    for (uint32_t a = 0; a < cf->n_anti; ++a) free(dcount[a]);
  return any && nfilt > 0;
}

/* ============================================================== Schedule */
/* evaluate: fills o->fails / o->scores; returns 1 if the priority list is
 * non-empty, 0 if empty, <0 on error */
static int evaluate_ext(orc *o, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids) {
  pctx c;
  c.p = p;
  c.ids = ids;
  c.ext = e;
  resolve_affinity(o, &c);
  if (c.error) return KSG_ERR_NOPEER;
  if (o->faithful) {
    machine_map m;
    map_pods_to_machines(o, &m);
    for (uint32_t n = 0; n < o->N; ++n) o->fails[n] = (uint8_t)faithful_fail_code(o, &c, &m, n);
    free_machine_map(o, &m);
    return faithful_prioritize(o, &c, o->fails, o->scores);
  }
  for (uint32_t n = 0; n < o->N; ++n) o->fails[n] = (uint8_t)incr_fail_code(o, &c, n);
  return incr_prioritize(o, &c, o->fails, o->scores, NULL);
}
static int evaluate(orc *o, const ksg_pod *p, const uint32_t *ids) { return evaluate_ext(o, p, NULL, ids); }

typedef struct {
  int64_t score;
  uint32_t rank;
} hp;

/* HostPriorityList.Less (types.go:42-47) under sort.Reverse: score desc, host desc */
static int hp_cmp_desc(const void *a, const void *b) {
  const hp *x = (const hp *)a, *y = (const hp *)b;
  if (x->score != y->score) return x->score > y->score ? -1 : 1;
  return x->rank > y->rank ? -1 : (x->rank < y->rank ? 1 : 0);
}

/* selectHost / getBestHosts: returns ties count; *best_rank_for(ix) resolves later */
static uint64_t count_ties(orc *o, int64_t *M) {
  int64_t best = NONE_SCORE;
  for (uint32_t n = 0; n < o->N; ++n)
    if (!o->fails[n] && o->scores[n] > best) best = o->scores[n];
  uint64_t k = 0;
  for (uint32_t n = 0; n < o->N; ++n)
    if (!o->fails[n] && o->scores[n] == best) k++;
  *M = best;
  return k;
}

static int32_t pick(orc *o, uint64_t ix) {
  if (o->faithful) { /* sort.Sort(sort.Reverse(priorityList)) then hosts[ix] */
    uint32_t cnt = 0;
    hp *list = (hp *)malloc((o->N ? o->N : 1) * sizeof(hp));
    for (uint32_t n = 0; n < o->N; ++n)
      if (!o->fails[n]) list[cnt++] = (hp){o->scores[n], n};
    qsort(list, cnt, sizeof(hp), hp_cmp_desc);
    int32_t r = (int32_t)list[ix].rank;
    free(list);
    return r;
  }
  int64_t M;
  count_ties(o, &M);
  uint64_t seen = 0;
  for (int64_t n = (int64_t)o->N - 1; n >= 0; --n)
    if (!o->fails[n] && o->scores[n] == M) {
      if (seen == ix) return (int32_t)n;
      seen++;
    }
  return -1;
}

static void commit(orc *o, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids, uint32_t node) {
  orc_add_pod_ext(o, node, p, e, ids);
}

int orc_evaluate(orc *o, const ksg_pod *p, const uint32_t *ids, uint8_t *fail_out, int64_t *score_out) {
  if (o->N == 0) return KSG_NONODES;
  int r = evaluate(o, p, ids);
  if (r < 0) return r;
  if (fail_out) memcpy(fail_out, o->fails, o->N);
  if (score_out)
    for (uint32_t n = 0; n < o->N; ++n) score_out[n] = o->fails[n] ? 0 : o->scores[n];
  return KSG_OK;
}

/* The node-sharded ServiceAntiAffinity step, restated (ksg_runtime.cpp
 * scan_exchange): a shard [lo, hi) sums, per anti priority a and label pair pr,
 * the pod's service count over its FILTERED nodes labelled pr
 * (spreading.go:118-139, over the shard's nodes only) into
 * out[a * n_pairs + pr] (int32, wrapping as ncclSum); the shards' partials are
 * all-reduced and every shard scores with the sum (orc_evaluate_counts). */
int orc_domain_counts(orc *o, const ksg_pod *p, const uint32_t *ids, uint32_t lo, uint32_t hi, int32_t *out) {
  const ksg_config *cf = &o->cfg;
  memset(out, 0, (size_t)(cf->n_anti ? cf->n_anti : 1) * o->n_pairs * 4);
  pctx c;
  c.p = p;
  c.ids = ids;
  c.ext = NULL;
  resolve_affinity(o, &c);
  if (c.error) return KSG_ERR_NOPEER;
  const int32_t s = p->service;
  if (s < 0) return KSG_OK;
  if (hi > o->N) hi = o->N;
  for (uint32_t n = lo; n < hi; ++n) {
    if (incr_fail_code(o, &c, n)) continue;
    for (uint32_t a = 0; a < cf->n_anti; ++a) {
      if (!cf->w_anti[a]) continue;
      const int32_t pr = node_pair_for_key(o, n, cf->anti_key[a]);
      if (pr >= 0) {
        uint32_t *slot = (uint32_t *)&out[(size_t)a * o->n_pairs + pr];
        *slot += (uint32_t)o->svc_cnt[(size_t)s * o->N + n];
      }
    }
  }
  return KSG_OK;
}

/* orc_evaluate (incremental mode) with the domain counts supplied */
int orc_evaluate_counts(orc *o, const ksg_pod *p, const uint32_t *ids, const int32_t *dcount, uint8_t *fail_out,
                        int64_t *score_out) {
  if (o->N == 0) return KSG_NONODES;
  pctx c;
  c.p = p;
  c.ids = ids;
  c.ext = NULL;
  resolve_affinity(o, &c);
  if (c.error) return KSG_ERR_NOPEER;
  for (uint32_t n = 0; n < o->N; ++n) o->fails[n] = (uint8_t)incr_fail_code(o, &c, n);
  (void)incr_prioritize(o, &c, o->fails, o->scores, dcount);
  if (fail_out) memcpy(fail_out, o->fails, o->N);
  if (score_out)
    for (uint32_t n = 0; n < o->N; ++n) score_out[n] = o->fails[n] ? 0 : o->scores[n];
  return KSG_OK;
}

/* The node-sharded TaintTolerationPriority step, restated (ksg_runtime.cpp scan_exchange,
 * and the window path's count pass + all-reduce): NormalizeReduce's max is over every
 * filtered node (parity unpinned: no reference code, kschedgpu.h "extensions"), so a
 * shard [lo, hi) reports the max untolerated soft-taint count over ITS filtered nodes
 * (*out), the shards' maxima are all-reduced (max) and every shard scores with the
 * result (orc_evaluate_ext_tmax). */
int orc_taint_max(orc *o, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids, uint32_t lo, uint32_t hi,
                  int32_t *out) {
  *out = 0;
  pctx c;
  c.p = p;
  c.ids = ids;
  c.ext = e;
  resolve_affinity(o, &c);
  if (c.error) return KSG_ERR_NOPEER;
  if (hi > o->N) hi = o->N;
  for (uint32_t n = lo; n < hi; ++n) {
    if (incr_fail_code(o, &c, n)) continue;
    int32_t k = e ? soft_taints(o, &c, n) : 0;
    if (k > *out) *out = k;
  }
  return KSG_OK;
}

/* orc_evaluate_ext (incremental mode) with TaintTolerationPriority's max supplied */
int orc_evaluate_ext_tmax(orc *o, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids, int32_t tmax,
                          uint8_t *fail_out, int64_t *score_out) {
  if (o->N == 0) return KSG_NONODES;
  const int faithful = o->faithful;
  o->faithful = 0;
  o->tmax_given = tmax;
  int r = evaluate_ext(o, p, e, ids);
  o->tmax_given = -1;
  o->faithful = faithful;
  if (r < 0) return r;
  if (fail_out) memcpy(fail_out, o->fails, o->N);
  if (score_out)
    for (uint32_t n = 0; n < o->N; ++n) score_out[n] = o->fails[n] ? 0 : o->scores[n];
  return KSG_OK;
}

int orc_schedule_begin_ext(orc *o, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids, size_t n_ids,
                           int64_t *max_score, uint32_t *tie_count, uint8_t *fail_codes);
int orc_schedule_begin(orc *o, const ksg_pod *p, const uint32_t *ids, size_t n_ids, int64_t *max_score,
                       uint32_t *tie_count, uint8_t *fail_codes) {
  return orc_schedule_begin_ext(o, p, NULL, ids, n_ids, max_score, tie_count, fail_codes);
}

int orc_schedule_begin_ext(orc *o, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids, size_t n_ids,
                           int64_t *max_score, uint32_t *tie_count, uint8_t *fail_codes) {
  o->pending = 0;
  if (o->N == 0) return KSG_NONODES;
  int r = evaluate_ext(o, p, e, ids);
  if (r < 0) return r;
  if (fail_codes) memcpy(fail_codes, o->fails, o->N);
  int64_t M = 0;
  uint64_t k = r ? count_ties(o, &M) : 0;
  if (max_score) *max_score = k ? M : 0;
  if (tie_count) *tie_count = (uint32_t)k;
  if (!k) return KSG_NOFIT;
  o->pending = 1;
  o->pend = *p;
  free(o->pend_ids);
  o->pend_ids = (uint32_t *)malloc((n_ids ? n_ids : 1) * 4);
  if (n_ids) memcpy(o->pend_ids, ids, n_ids * 4);
  o->pend_n_ids = n_ids;
  o->pend_k = k;
  o->pend_M = M;
  memset(&o->pend_ext, 0, sizeof o->pend_ext);
  if (e) o->pend_ext = *e;
  return KSG_OK;
}

int orc_schedule_commit(orc *o, uint32_t tie_index, int32_t *out_node) {
  if (!o->pending || tie_index >= o->pend_k) return KSG_ERR_STATE;
  int32_t node = pick(o, tie_index);
  o->pending = 0;
  if (node < 0) return KSG_ERR_STATE;
  commit(o, &o->pend, &o->pend_ext, o->pend_ids, (uint32_t)node);
  if (out_node) *out_node = node;
  return KSG_OK;
}

/* the same loop the device runs: begin, draw Int63 iff something fits, commit */
int orc_schedule_batch_ext(orc *o, const ksg_pod *pods, const ksg_pod_ext *exts, uint32_t n, const uint32_t *ids,
                           uint32_t n_ids, uint64_t *rng_state, int32_t *out_nodes);
int orc_schedule_batch(orc *o, const ksg_pod *pods, uint32_t n, const uint32_t *ids, uint32_t n_ids,
                       uint64_t *rng_state, int32_t *out_nodes) {
  return orc_schedule_batch_ext(o, pods, NULL, n, ids, n_ids, rng_state, out_nodes);
}

int orc_schedule_batch_ext(orc *o, const ksg_pod *pods, const ksg_pod_ext *exts, uint32_t n, const uint32_t *ids,
                           uint32_t n_ids, uint64_t *rng_state, int32_t *out_nodes) {
  (void)n_ids;
  for (uint32_t i = 0; i < n; ++i) {
    if (o->N == 0) {
      out_nodes[i] = KSG_OUT_NONODES;
      continue;
    }
    const ksg_pod_ext *e = exts ? exts + i : NULL;
    int r = evaluate_ext(o, pods + i, e, ids);
    if (r < 0) {
      out_nodes[i] = KSG_OUT_ERROR;
      continue;
    }
    int64_t M = 0;
    uint64_t k = r ? count_ties(o, &M) : 0;
    if (!k) {
      out_nodes[i] = KSG_OUT_NOFIT;
      continue;
    }
    uint64_t rr = splitmix_next(rng_state) >> 1;
    int32_t node = pick(o, rr % k);
    commit(o, pods + i, e, ids, (uint32_t)node);
    out_nodes[i] = node;
  }
  return KSG_OK;
}

int orc_evaluate_ext(orc *o, const ksg_pod *p, const ksg_pod_ext *e, const uint32_t *ids, uint8_t *fail_out,
                     int64_t *score_out) {
  if (o->N == 0) return KSG_NONODES;
  int r = evaluate_ext(o, p, e, ids);
  if (r < 0) return r;
  if (fail_out) memcpy(fail_out, o->fails, o->N);
  if (score_out)
    for (uint32_t n = 0; n < o->N; ++n) score_out[n] = o->fails[n] ? 0 : o->scores[n];
  return KSG_OK;
}

void orc_set_extensions(orc *o, const ksg_ext_config *e) {
  o->ext = *e;
  o->ext_on = e->filters || e->w_taint_toleration || e->w_balanced || e->n_scalar;
}

/* after orc_set_cluster: allocatable of each extended resource, taints per node */
void orc_set_node_ext(orc *o, const int64_t *scalar_cap, const uint32_t *taint_off, const uint32_t *taint_n,
                      const uint32_t *taint_ids) {
  free_ext(o);
  const size_t NN = o->N ? o->N : 1, ns = o->ext.n_scalar ? o->ext.n_scalar : 1;
  o->scap = (int64_t *)calloc(ns * NN, 8);
  o->sused = (int64_t *)calloc(ns * NN, 8);
  if (scalar_cap) memcpy(o->scap, scalar_cap, (size_t)o->ext.n_scalar * o->N * 8);
  o->ntaint = (uint32_t **)calloc(NN, sizeof(uint32_t *));
  o->nnt = (uint32_t *)calloc(NN, 4);
  for (uint32_t n = 0; n < o->N; ++n) {
    o->nnt[n] = taint_n ? taint_n[n] : 0;
    o->ntaint[n] = (uint32_t *)malloc((o->nnt[n] ? o->nnt[n] : 1) * 4);
    for (uint32_t i = 0; i < o->nnt[n]; ++i) o->ntaint[n][i] = taint_ids[taint_off[n] + i];
  }
}

void orc_read_requested(orc *o, int64_t *c, int64_t *m) {
  if (c) memcpy(c, o->used_c, (size_t)o->N * 8);
  if (m) memcpy(m, o->used_m, (size_t)o->N * 8);
}

/* the extended-resource usage [n_scalar][N] (ksg_read_ext_used) */
void orc_read_ext_used(orc *o, int64_t *used) {
  if (used && o->sused) memcpy(used, o->sused, (size_t)o->ext.n_scalar * o->N * 8);
}

/* ====================================================== kubelet admission */
/* handleNotFittingPods' scheduler checks (pkg/kubelet/kubelet.go:1716-1771) over
 * the ksg_admission_set layout: PodMatchesNodeLabels (predicates.go:161-167),
 * then CheckPodsExceedingCapacity (predicates.go:104-124) greedily in the given
 * order over the pods that matched. mode bit 1: capacity, bit 2: selector. */
void orc_admit_pods(const ksg_admission_set *sets, uint32_t n_sets, const ksg_pod *pods, uint32_t n_pods,
                    const uint32_t *ids, const uint32_t *pairs, int mode, uint8_t *out) {
  for (uint32_t i = 0; i < n_pods; ++i) out[i] = KSG_ADMIT_OK;
  for (uint32_t s = 0; s < n_sets; ++s) {
    const ksg_admission_set *st = &sets[s];
    int64_t totalC = st->cap_milli_cpu, totalM = st->cap_memory, reqC = 0, reqM = 0;
    for (uint32_t i = st->pod_off; i < st->pod_off + st->n_pods; ++i) {
      const ksg_pod *p = &pods[i];
      uint8_t code = KSG_ADMIT_OK;
      if (mode & 2) {
        for (uint32_t k = 0; k < p->n_sel; ++k) {
          uint32_t want = ids[p->sel_off + k];
          int found = 0;
          for (uint32_t l = 0; l < st->n_labels; ++l)
            if (want != 0 && pairs[st->label_off + l] == want) found = 1;
          if (!found) {
            code = KSG_ADMIT_NODESELECTOR;
            break;
          }
        }
      }
      if ((mode & 1) && code == KSG_ADMIT_OK) {
        int fitsC = totalC == 0 || (int64_t)((uint64_t)totalC - (uint64_t)reqC) >= p->milli_cpu;
        int fitsM = totalM == 0 || (int64_t)((uint64_t)totalM - (uint64_t)reqM) >= p->memory;
        if (fitsC && fitsM) {
          reqC = (int64_t)((uint64_t)reqC + (uint64_t)p->milli_cpu);
          reqM = (int64_t)((uint64_t)reqM + (uint64_t)p->memory);
        } else {
          code = KSG_ADMIT_CAPACITY;
        }
      }
      out[i] = code;
    }
  }
}

/* ====================================== incremental mode, node-sharded threads */
/* The strong CPU design point (SURVEY.md 8(d) "CPU timing" ii): the incremental
 * restatement with every pod's node loop split over `nthreads` threads (contiguous
 * node-rank shards, like the GPU shards); per pod, thread 0 resolves the pod's
 * context, every thread filters/scores its shard and reports its max and tie count,
 * thread 0 merges (selectHost: global max, ties in descending rank, one Int63 draw per
 * success) and commits. Two spin barriers per pod. Configurations with
 * ServiceAntiAffinity (a cross-shard domain-count reduction) run single-threaded.
 * Extensions (parity unpinned): the filters and BalancedAllocation are per node;
 * TaintToleration's NormalizeReduce max over the filtered nodes takes a third
 * barrier (every shard's max untolerated soft-taint count) before the scores. */
#include <pthread.h>
#include <stdatomic.h>

typedef struct {
  orc *o;
  const ksg_pod *pods;
  const ksg_pod_ext *exts; /* extension records (NULL: none) */
  const uint32_t *ids;
  uint32_t n;
  uint64_t *rng;
  int32_t *out;
  int T;
  int any;        /* some priority has a weight (else the HostPriorityList is empty) */
  pctx c;         /* the current pod (thread 0 writes it before barrier A) */
  int skip;
  int32_t maxc;
  int64_t *tmax;  /* per thread: local max score (NONE_SCORE: nothing fits) */
  uint64_t *tcnt; /* per thread: nodes at it */
  int32_t *tsoft; /* per thread: max untolerated soft-taint count over its filtered nodes */
  int32_t *soft;  /* per node: the pod's untolerated soft taints (TaintToleration) */
  atomic_int bar_count, bar_sense;
} mt_job;

typedef struct {
  mt_job *j;
  int t;
} mt_arg;

static void mt_barrier(mt_job *j, int *sense) {
  *sense = !*sense;
  if (atomic_fetch_add_explicit(&j->bar_count, 1, memory_order_acq_rel) == j->T - 1) {
    atomic_store_explicit(&j->bar_count, 0, memory_order_relaxed);
    atomic_store_explicit(&j->bar_sense, *sense, memory_order_release);
  } else {
    while (atomic_load_explicit(&j->bar_sense, memory_order_acquire) != *sense) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    }
  }
}

/* incr_prioritize's per-node score without ServiceAntiAffinity */
static int64_t mt_score(const orc *o, const pctx *c, int32_t maxc, uint32_t n) {
  const ksg_config *cf = &o->cfg;
  if (cf->n_priority_configs == 0 && !ext_prio_on(o)) return 1; /* EqualPriority fallback */
  int64_t sc = 0;
  if (cf->w_least_requested) {
    int64_t tc = (int64_t)((uint64_t)o->used_c[n] + (uint64_t)c->p->milli_cpu);
    int64_t tm = (int64_t)((uint64_t)o->used_m[n] + (uint64_t)c->p->memory);
    sc = go_add(sc, go_mul(cf->w_least_requested, ((calculate_score(tc, o->cap_c[n]) + calculate_score(tm, o->cap_m[n])) / 2)));
  }
  if (cf->w_service_spreading) {
    int32_t s = c->p->service;
    int32_t cnt = s >= 0 ? o->svc_cnt[(size_t)s * o->N + n] : 0;
    sc = go_add(sc, go_mul(cf->w_service_spreading, (maxc > 0 ? frac10_f32((int64_t)maxc - cnt, maxc) : 10)));
  }
  for (uint32_t q = 0; q < cf->n_label_pref; ++q) {
    if (!cf->w_pref[q]) continue;
    int exists = node_has_key(o, n, cf->pref_key[q]);
    int ok = (exists && cf->pref_presence[q]) || (!exists && !cf->pref_presence[q]);
    sc = go_add(sc, go_mul(cf->w_pref[q], (ok ? 10 : 0)));
  }
  if (o->ext_on && o->ext.w_balanced) { /* ext_prioritize's per-node term */
    int64_t tc = (int64_t)((uint64_t)o->used_c[n] + (uint64_t)c->p->milli_cpu);
    int64_t tm = (int64_t)((uint64_t)o->used_m[n] + (uint64_t)c->p->memory);
    sc = go_add(sc, go_mul(o->ext.w_balanced, balanced_score(tc, o->cap_c[n], tm, o->cap_m[n])));
  }
  return go_add(sc, cf->w_equal);
}

static void *mt_worker(void *argp) {
  mt_arg *a = (mt_arg *)argp;
  mt_job *j = a->j;
  orc *o = j->o;
  const int t = a->t;
  const uint32_t lo = (uint32_t)(((uint64_t)o->N * t) / j->T), hi = (uint32_t)(((uint64_t)o->N * (t + 1)) / j->T);
  int sense = 0;
  for (uint32_t i = 0; i < j->n; ++i) {
    if (t == 0) {
      j->skip = 0;
      j->c.p = j->pods + i;
      j->c.ids = j->ids;
      j->c.ext = j->exts ? j->exts + i : NULL;
      resolve_affinity(o, &j->c);
      if (j->c.error) {
        j->out[i] = KSG_OUT_ERROR;
        j->skip = 1;
      }
      const int32_t s = j->pods[i].service;
      j->maxc = s >= 0 ? o->svc_max[s] : 0;
    }
    mt_barrier(j, &sense); /* A: the pod's context is ready */
    /* TaintToleration with a toleration record: the max over every shard's filtered nodes first */
    const int taint_w = !j->skip && o->ext_on && o->ext.w_taint_toleration;
    const int taint_norm = taint_w && j->c.ext;
    if (taint_norm) {
      int32_t mx = 0;
      for (uint32_t n = lo; n < hi; ++n) {
        const int f = incr_fail_code(o, &j->c, n);
        o->fails[n] = (uint8_t)f;
        if (f) continue;
        j->soft[n] = soft_taints(o, &j->c, n);
        if (j->soft[n] > mx) mx = j->soft[n];
      }
      j->tsoft[t] = mx;
      mt_barrier(j, &sense); /* C: every shard's max soft-taint count */
    }
    if (!j->skip) {
      int64_t best = NONE_SCORE;
      uint64_t k = 0;
      int32_t mx = 0;
      if (taint_norm)
        for (int g = 0; g < j->T; ++g)
          if (j->tsoft[g] > mx) mx = j->tsoft[g];
      for (uint32_t n = lo; n < hi; ++n) {
        const int f = taint_norm ? o->fails[n] : incr_fail_code(o, &j->c, n);
        o->fails[n] = (uint8_t)f;
        if (f) continue;
        int64_t sc = mt_score(o, &j->c, j->maxc, n);
        if (taint_w) { /* NormalizeReduce(10, reverse); no record: every node 10 */
          const int64_t v = !taint_norm || mx == 0 ? 10 : 10 - (10 * (int64_t)j->soft[n]) / mx;
          sc = go_add(sc, go_mul(o->ext.w_taint_toleration, v));
        }
        o->scores[n] = sc;
        if (sc > best) {
          best = sc;
          k = 1;
        } else if (sc == best) {
          ++k;
        }
      }
      j->tmax[t] = best;
      j->tcnt[t] = k;
    }
    mt_barrier(j, &sense); /* B: every shard reported */
    if (t == 0 && !j->skip) {
      int64_t M = NONE_SCORE;
      uint64_t k = 0;
      for (int g = 0; g < j->T; ++g)
        if (j->tcnt[g] && j->tmax[g] > M) M = j->tmax[g];
      for (int g = 0; g < j->T; ++g)
        if (j->tcnt[g] && j->tmax[g] == M) k += j->tcnt[g];
      if (!j->any) k = 0; /* every weight 0: empty HostPriorityList (generic_scheduler.go:149-151) */
      if (k == 0) {
        j->out[i] = KSG_OUT_NOFIT;
      } else {
        uint64_t ix = (splitmix_next(j->rng) >> 1) % k; /* rand.Int() % len(ties) */
        int32_t node = -1;
        for (int g = j->T - 1; g >= 0 && node < 0; --g) { /* ties in descending rank */
          if (!j->tcnt[g] || j->tmax[g] != M) continue;
          if (ix >= j->tcnt[g]) {
            ix -= j->tcnt[g];
            continue;
          }
          const uint32_t glo = (uint32_t)(((uint64_t)o->N * g) / j->T), ghi = (uint32_t)(((uint64_t)o->N * (g + 1)) / j->T);
          for (int64_t n = (int64_t)ghi - 1; n >= (int64_t)glo; --n)
            if (!o->fails[n] && o->scores[n] == M) {
              if (ix == 0) {
                node = (int32_t)n;
                break;
              }
              --ix;
            }
        }
        commit(o, j->pods + i, j->exts ? j->exts + i : NULL, j->ids, (uint32_t)node);
        j->out[i] = node;
      }
    }
  }
  return NULL;
}

int orc_schedule_batch_mt_ext(orc *o, const ksg_pod *pods, const ksg_pod_ext *exts, uint32_t n, const uint32_t *ids,
                              uint32_t n_ids, uint64_t *rng_state, int32_t *out_nodes, int nthreads);
int orc_schedule_batch_mt(orc *o, const ksg_pod *pods, uint32_t n, const uint32_t *ids, uint32_t n_ids,
                          uint64_t *rng_state, int32_t *out_nodes, int nthreads) {
  return orc_schedule_batch_mt_ext(o, pods, NULL, n, ids, n_ids, rng_state, out_nodes, nthreads);
}

int orc_schedule_batch_mt_ext(orc *o, const ksg_pod *pods, const ksg_pod_ext *exts, uint32_t n, const uint32_t *ids,
                              uint32_t n_ids, uint64_t *rng_state, int32_t *out_nodes, int nthreads) {
  if (nthreads <= 1 || o->faithful || o->cfg.n_anti > 0 || o->N == 0 || (uint32_t)nthreads > o->N)
    return orc_schedule_batch_ext(o, pods, exts, n, ids, n_ids, rng_state, out_nodes);
  mt_job j;
  memset(&j, 0, sizeof j);
  j.o = o;
  j.exts = o->ext_on ? exts : NULL;
  j.pods = pods;
  j.ids = ids;
  j.n = n;
  j.rng = rng_state;
  j.out = out_nodes;
  j.T = nthreads;
  const ksg_config *cf = &o->cfg;
  j.any = cf->n_priority_configs == 0 || cf->w_least_requested || cf->w_service_spreading || cf->w_equal;
  for (uint32_t q = 0; q < cf->n_label_pref; ++q) j.any |= cf->w_pref[q] != 0;
  j.any |= ext_prio_on(o);
  j.tmax = (int64_t *)calloc((size_t)nthreads, 8);
  j.tcnt = (uint64_t *)calloc((size_t)nthreads, 8);
  j.tsoft = (int32_t *)calloc((size_t)nthreads, 4);
  j.soft = (int32_t *)calloc((size_t)o->N, 4);
  atomic_init(&j.bar_count, 0);
  atomic_init(&j.bar_sense, 0);
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  mt_arg *args = (mt_arg *)calloc((size_t)nthreads, sizeof(mt_arg));
  for (int t = 0; t < nthreads; ++t) {
    args[t].j = &j;
    args[t].t = t;
    if (t) pthread_create(&th[t], NULL, mt_worker, &args[t]);
  }
  mt_worker(&args[0]);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(args);
  free(j.tmax);
  free(j.tcnt);
  free(j.tsoft);
  free(j.soft);
  return KSG_OK;
}
