/* Per-call latency of the drop-in per-pod path, from C: what a cgo caller of
 * algorithm.ScheduleAlgorithm.Schedule (generic_scheduler.go:62-96) sees per
 * pod through ksg_schedule_begin + ksg_schedule_commit, with
 * no Python in the loop.
 *
 * Workload: config 2's shape: N nodes of 4 cpu / 16 GiB,
 * DefaultProvider (PodFitsPorts, PodFitsResources, NoDiskConflict,
 * MatchNodeSelector, HostName; LeastRequested 1, ServiceSpreading 1), pods of
 * 100-500 milli-cpu / 128-640 MiB in 8 services, one host port on every 16th
 * pod; splitmix64 draws as in ksg_schedule_batch.
 *
 * Prints one JSON line: per-pod latency percentiles (us), pods/s, the begin
 * and commit calls' own medians, and whether the resident server
 * (ksg_serve.hip) served them (KSG_SERVE=0: kernels launched per call).
 * usage: dropin_latency [n_nodes=5000] [n_pods=4000] [warmup=200] [want_fail=0] [ext=0] [policy=0]
 * policy 1: config 4's shape (ServiceAffinity on region, ServiceAntiAffinity on zone with
 * weight 1, plus the defaults; 4 regions x 2 zones, labels on every node). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/kschedgpu.h"

static uint64_t sm_next(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static double now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

#define CHECK(call)                                                               \
  do {                                                                            \
    int rc_ = (call);                                                             \
    if (rc_ != KSG_OK) {                                                          \
      fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, ctx ? ksg_last_error(ctx) : ""); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t n_nodes = argc > 1 ? (uint32_t)atoi(argv[1]) : 5000;
  const uint32_t n_pods = argc > 2 ? (uint32_t)atoi(argv[2]) : 4000;
  const uint32_t warmup = argc > 3 ? (uint32_t)atoi(argv[3]) : 200;
  const int want_fail = argc > 4 ? atoi(argv[4]) : 0;
  /* 1: extensions (taints + one extended resource, the filters); 2: the same + TaintToleration */
  const int ext_mode = argc > 5 ? atoi(argv[5]) : 0;
  const int policy = argc > 6 ? atoi(argv[6]) : 0;
  const uint32_t n_svc = 8;
  ksg_ctx* ctx = NULL;

  ksg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.predicates = KSG_PRED_PODFITSPORTS | KSG_PRED_PODFITSRESOURCES | KSG_PRED_NODISKCONFLICT |
                   KSG_PRED_MATCHNODESELECTOR | KSG_PRED_HOSTNAME;
  cfg.n_priority_configs = 2;
  cfg.w_least_requested = 1;
  cfg.w_service_spreading = 1;
  cfg.max_conflict_keys = 64;
  if (policy == 1) {  /* label key 0 = region (pairs 1..4), key 1 = zone (pairs 5..12) */
    cfg.predicates |= KSG_PRED_SERVICEAFFINITY;
    cfg.n_aff_labels = 1;
    cfg.aff_key[0] = 0;
    cfg.n_anti = 1;
    cfg.anti_key[0] = 1;
    cfg.w_anti[0] = 1;
    cfg.n_priority_configs = 3;
  }
  CHECK(ksg_create(&cfg, 0, &ctx));
  if (ext_mode) {
    ksg_ext_config e;
    memset(&e, 0, sizeof e);
    e.filters = KSG_EXT_TAINTS | KSG_EXT_SCALAR;
    e.w_taint_toleration = ext_mode == 2 ? 1 : 0;
    e.n_scalar = 1;
    e.max_taints = 4;
    CHECK(ksg_set_extensions(ctx, &e));
  }

  ksg_node* nodes = calloc(n_nodes, sizeof *nodes);
  for (uint32_t i = 0; i < n_nodes; ++i) {
    nodes[i].cap_milli_cpu = 4000;
    nodes[i].cap_memory = 16LL << 30;
  }
  uint32_t pair_keys[13] = {0};
  uint32_t* npairs = NULL;
  uint32_t n_np = 0, n_pk = 1;
  if (policy == 1) {
    for (uint32_t p = 1; p <= 4; ++p) pair_keys[p] = 0;
    for (uint32_t p = 5; p <= 12; ++p) pair_keys[p] = 1;
    n_pk = 13;
    npairs = calloc(2 * (size_t)n_nodes, sizeof *npairs);
    for (uint32_t i = 0; i < n_nodes; ++i) {
      const uint32_t zone = i % 8;
      nodes[i].label_off = n_np;
      nodes[i].n_labels = 2;
      npairs[n_np++] = 1 + zone / 2;
      npairs[n_np++] = 5 + zone;
    }
  }
  CHECK(ksg_set_cluster(ctx, nodes, n_nodes, npairs, n_np, pair_keys, n_pk, n_svc));
  if (ext_mode) {  /* 8 GPUs per node; every 5th node carries taint 1 (hard for the pods that do not tolerate it) */
    int64_t* gcap = calloc(n_nodes, sizeof *gcap);
    uint32_t* toff = calloc(n_nodes, sizeof *toff);
    uint32_t* tn = calloc(n_nodes, sizeof *tn);
    uint32_t* tid = calloc(n_nodes, sizeof *tid);
    uint32_t nt = 0;
    for (uint32_t i = 0; i < n_nodes; ++i) {
      gcap[i] = 8;
      toff[i] = nt;
      if (i % 5 == 0) tid[nt++] = 1, tn[i] = 1;
    }
    CHECK(ksg_set_node_ext(ctx, n_nodes, gcap, toff, tn, tid, nt));
  }

  const uint32_t total = warmup + n_pods;
  ksg_pod* pods = calloc(total, sizeof *pods);
  uint32_t* ids = calloc(3 * (size_t)total, sizeof *ids);  /* pod i's list: ids + 3i: port key, service, taint */
  ksg_pod_ext* pext = calloc(total, sizeof *pext);
  uint64_t gen = 12345;
  for (uint32_t i = 0; i < total; ++i) {
    ksg_pod* p = &pods[i];
    p->uid = i + 1;
    p->milli_cpu = 100 + (int64_t)(sm_next(&gen) % 5) * 100;
    p->memory = (128LL << 20) * (int64_t)(1 + sm_next(&gen) % 5);
    p->host = -1;
    p->service = (int32_t)(sm_next(&gen) % n_svc);
    ids[3 * i] = (uint32_t)(i % 32);  /* host-port conflict key */
    ids[3 * i + 1] = (uint32_t)p->service;
    ids[3 * i + 2] = 1;  /* the taint it does not tolerate (every third pod) */
    pext[i].scalar[0] = (i % 4 == 0) ? 1 : 0;
    pext[i].hard_off = 2;
    pext[i].n_hard = (i % 3 == 0) ? 1 : 0;
    p->ports_off = 0;
    p->n_ports = (i % 16 == 0) ? 1 : 0;
    p->svcs_off = 1;
    p->n_svcs = 1;
    for (int j = 0; j < KSG_MAX_AFF; ++j) p->aff_pair[j] = -1;
  }

  double* lat = calloc(n_pods, sizeof *lat);
  double* lat_b = calloc(n_pods, sizeof *lat_b);
  double* lat_c = calloc(n_pods, sizeof *lat_c);
  uint8_t* fails = calloc(n_nodes, 1);
  uint64_t rng = 0x5eed;
  uint32_t placed = 0, nofit = 0;
  double t_all = 0.0;
  for (uint32_t i = 0; i < total; ++i) {
    int64_t best = 0;
    uint32_t ties = 0;
    int32_t node = KSG_OUT_NOFIT;
    const double t0 = now_us();
    const int rb = ext_mode ? ksg_schedule_begin_ext(ctx, &pods[i], &pext[i], ids + 3 * (size_t)i, &best, &ties,
                                                     want_fail ? fails : NULL)
                            : ksg_schedule_begin(ctx, &pods[i], ids + 3 * (size_t)i, &best, &ties, want_fail ? fails : NULL);
    if (rb != KSG_OK && rb != KSG_NOFIT) CHECK(rb);
    const double tb = now_us();
    if (ties > 0) {
      const uint64_t r = sm_next(&rng) >> 1;  /* rand.Int() */
      CHECK(ksg_schedule_commit(ctx, (uint32_t)(r % ties), &node));
    }
    const double t1 = now_us();
    if (i >= warmup) {
      lat[i - warmup] = t1 - t0;
      lat_b[i - warmup] = tb - t0;
      lat_c[i - warmup] = t1 - tb;
      t_all += t1 - t0;
      if (node >= 0) ++placed;
      else ++nofit;
    }
  }
  qsort(lat, n_pods, sizeof *lat, cmp_d);
  qsort(lat_b, n_pods, sizeof *lat_b, cmp_d);
  qsort(lat_c, n_pods, sizeof *lat_c, cmp_d);
  uint64_t sv[4] = {0, 0, 0, 0};
  ksg_serve_stats(ctx, sv);
#define PCT(q) lat[(size_t)((q) * (n_pods - 1))]
  printf("{\"metric\": \"drop-in per-pod latency (ksg_schedule_begin + ksg_schedule_commit, C caller)\", "
         "\"nodes\": %u, \"pods\": %u, \"warmup\": %u, \"placed\": %u, \"nofit\": %u, "
         "\"us_p50\": %.2f, \"us_p90\": %.2f, \"us_p99\": %.2f, \"us_max\": %.2f, \"us_mean\": %.2f, "
         "\"pods_per_s\": %.1f, \"want_fail\": %d, \"ext\": %d, \"policy\": %d, \"begin_us_p50\": %.2f, \"commit_us_p50\": %.2f, "
         "\"served\": {\"eligible\": %d, \"launches\": %llu, \"requests\": %llu}, \"histogram_us\": {\"edges\": [5, 10, 20, 40, 80, 160, 320], \"counts\": [",
         n_nodes, n_pods, warmup, placed, nofit, PCT(0.5), PCT(0.9), PCT(0.99), lat[n_pods - 1],
         t_all / n_pods, n_pods / (t_all * 1e-6), want_fail, ext_mode, policy, lat_b[n_pods / 2], lat_c[n_pods / 2], (int)sv[3],
         (unsigned long long)sv[0], (unsigned long long)sv[1]);
  const double edges[] = {5, 10, 20, 40, 80, 160, 320, 1e30};
  size_t k = 0;
  for (int b = 0; b < 8; ++b) {
    size_t c = 0;
    while (k < n_pods && lat[k] < edges[b]) ++k, ++c;
    printf("%s%zu", b ? ", " : "", c);
  }
  printf("]}}\n");
  ksg_destroy(ctx);
  free(lat);
  free(lat_b);
  free(lat_c);
  free(fails);
  free(ids);
  free(pods);
  free(nodes);
  return 0;
}
