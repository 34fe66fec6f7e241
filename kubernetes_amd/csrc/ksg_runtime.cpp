// ksg_runtime.cpp — host runtime of libkschedgpu.so: the C ABI in
// include/kschedgpu.h, the device-state mirror, and the RCCL exchange.
//
// Reference behaviour mirrored here (under /root/reference):
//   genericScheduler.Schedule / selectHost     pkg/scheduler/generic_scheduler.go:54-96
//   MapPodsToMachines (pods keyed by Status.Host)  pkg/scheduler/predicates.go:354-375
//   SimpleModeler.AssumePod / listPods        plugin/pkg/scheduler/modeler.go:77-139
//   ServiceSpread maxCount over all hosts     pkg/scheduler/spreading.go:72-80
//
// The library keeps a host mirror of the mutable per-node state (requested
// totals, conflict-key reference counts, per-service pod counts and peers) so
// ksg_remove_pod can undo exactly; the device copy is authoritative for
// scheduling and is patched from the mirror. All scheduling decisions run in
// the HIP kernels (ksg_kernels.hip); there is no CPU evaluation path.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "ksg_internal.h"
#include "ksg_shard.h"


hipError_t ksg_launch_batch(int R, bool anti, const KsgDev& d, const ksg_pod* pods,
                            const uint32_t* ids, uint32_t n, uint64_t* rng, int32_t* out,
                            hipStream_t st, const ksg_pod_ext* ext = nullptr);
hipError_t ksg_launch_scan(int R, bool anti, const KsgDev& d, const ksg_pod* pods,
                           const uint32_t* ids, int mode, int phase, uint8_t* fail_out,
                           int64_t* score_out, uint8_t* record, int32_t* dpart,
                           const int32_t* dglobal, hipStream_t st, const ksg_pod_ext* ext = nullptr);
hipError_t ksg_launch_win_eval(const KsgDev& d, int mode, const ksg_pod* batch, const uint32_t* ids,
                               const KsgWinRun* run, uint32_t wcap, KsgWinSum* sums, uint64_t* wbits, int32_t* wmax,
                               uint32_t ostride, int32_t* dcnt, uint64_t* wfit, int32_t* dmb, uint64_t* wbz,
                               uint32_t dz, hipStream_t st, const ksg_pod_ext* exts = nullptr,
                               int32_t* tmax = nullptr, uint64_t* psoft = nullptr, int32_t* thist = nullptr);
hipError_t ksg_launch_zonemap(uint32_t n_nodes, const int32_t* anti_domain, uint32_t d0, uint32_t nw,
                              uint64_t* zmap, hipStream_t st);
hipError_t ksg_launch_win_t0(const KsgDev& d, uint32_t wcap, const KsgWinRun* run, const KsgWinXchg& x,
                             hipStream_t st);
uint32_t ksg_win_t0_stride(const KsgDev& d);
hipError_t ksg_launch_win_resolve(const KsgDev& d, uint32_t wcap, KsgWinRun* run, const KsgWinSum* sums,
                                  const KsgWinXchg& x, uint64_t* rng, int32_t* out, hipStream_t st);
bool ksg_win_fused_ok(const KsgDev& d);
uint32_t ksg_win_fused_groups(const KsgDev& d, uint32_t wcap);
hipError_t ksg_launch_win_fused(const KsgDev& d, uint32_t wcap, KsgWinRun* run, const KsgWinSum* sums,
                                const KsgWinXchg& x, uint64_t* rng, int32_t* out, const KsgFused& f, uint32_t grid,
                                hipStream_t st);
uint32_t ksg_win_max_window(const KsgDev& d);
hipError_t ksg_launch_decide(const KsgDev& d, const ksg_pod* pods, const uint32_t* ids,
                             const uint8_t* records, uint32_t rec_bytes, uint32_t world,
                             const uint32_t* shard_wlo, int mode, uint64_t tie_index,
                             uint64_t* rng, int32_t* out, uint32_t out_idx, int64_t* summary,
                             hipStream_t st, const ksg_pod_ext* ext = nullptr);
hipError_t ksg_launch_static(const KsgStaticCfg& sc, uint32_t n_nodes, const ksg_node* nodes,
                             const uint32_t* node_pairs, const uint32_t* pair_keys,
                             const int32_t* dom_of_pair, uint32_t n_pairs, uint32_t nw,
                             uint64_t* static_fit, int64_t* static_score, int32_t* anti_domain,
                             int32_t* aff_pair, unsigned long long* pairmap, hipStream_t st);
hipError_t ksg_launch_patch(const KsgPatch* patches, uint32_t n, hipStream_t st);
hipError_t ksg_launch_static_terms(const KsgStaticCfg& sc, uint32_t n_nodes, const ksg_node* nodes,
                                   const uint32_t* node_pairs, const uint32_t* pair_keys, uint32_t n_pairs, uint32_t nw,
                                   uint64_t* fit, int64_t* score, hipStream_t st);
hipError_t ksg_launch_static_fold(uint64_t* static_fit, int64_t* static_score, const uint64_t* xfit,
                                  const int64_t* xscore, uint32_t nw, uint32_t n, int own_fit, int own_score,
                                  hipStream_t st);
hipError_t ksg_launch_serve(int R, bool anti, bool ext, const KsgDev& d, const KsgSrvArgs& a, hipStream_t st);
hipError_t ksg_launch_serve_grid(int npt, bool ext, const KsgDev& d, const KsgSrvArgs& a, hipStream_t st);
hipError_t ksg_launch_admit(const ksg_admission_set* sets, uint32_t n_sets, const ksg_pod* pods,
                            const uint32_t* ids, const uint32_t* pairs, int mode, uint8_t* out, hipStream_t st);

namespace {

struct PodRec {
  uint32_t host;
  int64_t cpu, mem;
  int64_t scalar[KSG_MAX_SCALAR];  // extension: extended resource requests
  std::vector<uint32_t> keys;  // ports + PDs
  std::vector<uint32_t> svcs;
  uint64_t seq;
};

constexpr uint32_t kMaxNodesPerShard = KSG_R_MAX * KSG_NT;
// the fused window launch's control block: two KsgWinRun slots, then the pod groups'
// counters uint32[2][kFctlGroups][8] (a window of up to 4 x kFctlGroups pods)
constexpr uint32_t kFctlGroups = 1024;
constexpr size_t kFctlRuns = 2 * sizeof(KsgWinRun);
constexpr size_t kFctlBytes = kFctlRuns + (size_t)2 * kFctlGroups * 8 * sizeof(uint32_t);

// Timing-only events: no system-scope fence when they complete. A default
// hipEventRecord writes back and invalidates the caches, which costs the
// stream time between the window kernels and evicts the node state the next
// kernel reads from L2 (KSG_EVENT_FENCE=1 restores the default for A/B).
const unsigned kTimingEvent =
    (getenv("KSG_EVENT_FENCE") && atoi(getenv("KSG_EVENT_FENCE"))) ? hipEventDefault : hipEventDisableSystemFence;

}  // namespace

struct ksg_ctx {
  ksg_config cfg{};
  int device = 0, rank = 0, world = 1;
  hipStream_t st = nullptr;
  ncclComm_t comm = nullptr;
  bool xchg = false;
  double ppw_est = 0.0;  // pods resolved per window (window path round sizing)
  // windows per round = margin x (pods left) / ppw_est + 1 (KSG_ROUND_MARGIN): the
  // launches past the batch's end cost ~8 us each, a second round a host round trip
  double round_margin = 1.0;
  // pinned staging for the per-call uploads / small read-backs (a pageable
  // hipMemcpyAsync is a staged, effectively synchronous copy)
  uint8_t* h_up = nullptr;
  size_t h_up_cap = 0;
  uint8_t* h_dn = nullptr;
  size_t h_dn_cap = 0;  // exchange path: world > 1, or a 1-rank RCCL communicator
  // host-staged exchange (ksg_set_allgather) for sharded contexts without RCCL
  ksg_allgather_fn xfn = nullptr;
  void* xuser = nullptr;
  uint8_t *h_xsend = nullptr, *h_xrecv = nullptr;
  size_t h_xsend_cap = 0, h_xrecv_cap = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // the batch path's waits spin on this event (KSG_SPIN_WAIT=0: hipStreamSynchronize)
  hipEvent_t ev_wait = nullptr;
  bool spin_wait = true;
  double last_ms = 0.0;
  std::string err;

  // cluster
  bool have_cluster = false;
  // a batch failed after its device work was enqueued: the device may hold some
  // of its commits and the host mirror none, so every call fails until
  // ksg_set_cluster uploads the cluster again
  bool diverged = false;
  uint32_t N = 0, nw = 0, n_pairs = 0, S = 0, D = 0;
  uint32_t lo = 0, hi = 0, wlo = 0, nwords = 0, nwords_max = 0;
  std::vector<uint32_t> shard_wlo_h;
  int R = 1;
  size_t lds = 0;
  KsgDev dev{};
  std::vector<void*> cluster_allocs;
  uint32_t* d_shard_wlo = nullptr;

  // scratch
  ksg_pod* d_pods = nullptr;
  size_t pods_cap = 0;
  uint32_t* d_ids = nullptr;
  size_t ids_cap = 0;
  uint8_t* d_fail = nullptr;
  int64_t* d_score = nullptr;
  uint8_t* d_rec_send = nullptr;
  uint8_t* d_rec_recv = nullptr;
  uint32_t rec_bytes = 0;
  int32_t* d_dpart = nullptr;
  int32_t* d_dglobal = nullptr;
  int32_t* d_out = nullptr;
  size_t out_cap = 0;
  uint64_t* d_rng = nullptr;
  int64_t* d_summary = nullptr;
  // the per-pod path (begin / commit / evaluate): the pod and its id list in
  // one device buffer (one copy in), and the decide kernel's summary and chosen
  // node written straight into pinned host memory (no copy out)
  uint8_t* d_one = nullptr;
  size_t one_cap = 0;
  const ksg_pod* one_pod = nullptr;
  const uint32_t* one_ids = nullptr;
  uint8_t* h_map = nullptr;  // pinned, coherent: [0, 32) summary int64[3], [32, 36) node
  uint8_t* d_map = nullptr;  // its device address
  KsgPatch* d_patch = nullptr;
  size_t patch_cap = 0;
  uint64_t* d_draws = nullptr;  // ksg_schedule_batch_draws: the caller's rand.Int() values
  size_t draws_cap = 0;
  uint64_t draw_tmp = 0;
  uint8_t* d_admit = nullptr;  // kubelet admission: sets, pods, ids, pairs, codes (one buffer)
  size_t admit_cap = 0;
  std::vector<KsgPatch> patches;

  // host mirror
  std::vector<int64_t> used_c, used_m;
  // max over nodes of used_c / used_m for use_window: raised by each mirror add,
  // recomputed after anything else changes them (a removal, a negative total)
  int64_t mu_max = 0;
  bool mu_neg = false, mu_dirty = true;
  std::unordered_map<uint64_t, uint32_t> key_ref;  // (key << 32) | node
  std::vector<int32_t> svc_cnt;                    // S*N
  std::vector<std::unordered_map<uint32_t, int32_t>> svc_ext;
  std::vector<int32_t> svc_max, svc_total, svc_peer;
  std::vector<int32_t> h_aff_pair;  // [affinity label][node] (ServiceAffinity, one rank; ksg_set_cluster)
  std::vector<std::map<uint64_t, uint32_t>> svc_members;  // seq -> host
  std::unordered_map<uint64_t, PodRec> pods;
  uint64_t seq = 0;

  // window (speculative) path
  uint32_t window = 128;        // 0 = exact one-pod-at-a-time kernel
  // HIP events around every ev_stride-th window launch (phase A and resolver;
  // KSG_KERNEL_EVENTS=N: every N-th, 0: none). An event between two dependent
  // launches lengthens the gap between them, so a sample of the windows is timed
  // and the per-launch mean scaled to all launches (ksg_last_batch_kernel_ms).
  uint32_t ev_stride = 4;
  uint32_t ev_phase = 0;  // which launches of a round are timed; advances every round
  KsgWinSum* d_winsum = nullptr;
  uint8_t* d_xsend = nullptr;   // phase A block of this shard (KsgWinXchg layout)
  uint8_t* d_xrecv = nullptr;   // all-gathered blocks of every shard (world > 1)
  uint8_t* d_t0img = nullptr;   // the plain resolver's T0 images, one per window pod
  size_t t0img_cap = 0;
  int32_t* d_dcnt = nullptr;     // [W][D] per-pod anti-affinity domain counts (phase A pre-pass)
  int32_t* d_dmb = nullptr;      // [W][D+1] re-rank: best score without the anti term per domain row
  uint64_t* d_zmap = nullptr;    // [D+1][nw] re-rank: nodes of each domain row (cluster allocation)
  size_t win_cap = 0, xsend_cap = 0, xrecv_cap = 0, dcnt_cap = 0, dmb_cap = 0;
  int32_t* d_etmax = nullptr;    // [W] extension scores: TaintToleration max per window pod (count pass)
  int32_t* d_ethist = nullptr;   // [W][KSG_TBINS] ... the histogram of its soft-taint counts
  size_t ethist_cap = 0;
  uint64_t* d_epsoft = nullptr;  // [W] ... the pods' untolerated soft taints as masks
  size_t etmax_cap = 0, epsoft_cap = 0;
  KsgWinRun* d_run = nullptr;      // progress of the window chain (device)
  KsgWinRun* h_run = nullptr;      // pinned host copy
  uint32_t last_stats[4] = {0, 0, 0, 0};  // windows, stops (service scalar), stops (ties exhausted)
  std::vector<hipEvent_t> wev;     // event pairs around the chained window kernels
  double last_kms[3] = {0, 0, 0};  // phase A ms, phase B ms, launches (window path)
  double last_t0ms = 0;            // ... and between them: the exchange (sharded) and the T0 images
  double last_wsum = 0;            // window capacity W summed over the launches
  bool dbg_fail_next = false;      // KSG_DEBUG & 16384: the next window batch fails after its device work
  uint32_t dbg_corrupt = 0;        // KSG_DEBUG bits 22 / 23: corrupt the next COMMIT / BEGIN request's layout
  bool win_d1 = true;              // phase A's single-commit drop bitmaps (KSG_WIN_D1=0: off; ksg_plain.hip)
  // the fused window launch (KsgFused, ksg_plain.hip): one launch per window on one rank without
  // ServiceAntiAffinity or extensions (KSG_FUSED=0: phase A, T0 images and resolver apart)
  bool win_fused = true;
  uint32_t fused_grid = 0;          // its blocks: one per CU (KSG_FUSED_GRID overrides)
  // ... up to this many 64-node words per shard (KSG_FUSED_MAX_WORDS; 65,536 nodes): past them the
  // scoring blocks, one per CU under the resolver's LDS, are too few waves to hide phase A's load
  // latency (config 5, 100k nodes, same box: 255k fused against 385k apart; 45k nodes: 492k fused
  // against 465k, profiles/r6_fused_threshold.json)
  uint32_t fused_max_words = 1024;
  uint8_t* d_fctl = nullptr;        // KsgWinRun[2], then the counters uint32[2][groups][8]
  uint8_t* h_fctl = nullptr;        // pinned: the round's first slot and zeroed counters
  double last_hus[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // host us per phase of the last batch (ksg_last_batch_host_us)
  double totals[24] = {};  // ksg_batch_totals: the per-batch diagnostics summed over batches
  int64_t max_cap = 0, min_cap = 0;

  // Commits of the last ksg_schedule_batch not yet replayed into the host
  // mirror: replayed while the next batch runs on the device, or before any
  // call that reads the mirror (flush_deferred).
  std::vector<ksg_pod> dfr_pods;
  std::vector<uint32_t> dfr_ids;
  std::vector<int32_t> dfr_out;
  std::unordered_set<uint64_t> dfr_uids;
  int64_t dfr_sum = 0;   // sum of the deferred pods' requests (cpu + memory), capped
  bool dfr_neg = false;  // a deferred pod has a negative request

  // extensions (ksg_set_extensions; exact kernels, one rank, parity unpinned)
  bool ext_on = false;
  ksg_ext_config ext{};
  std::vector<int64_t> sc_used;  // [n_scalar][N] host mirror of scalar_used
  std::unordered_map<uint64_t, std::array<int64_t, KSG_MAX_SCALAR>> ext_scalar;  // uid -> requests
  const ksg_pod_ext* cur_ext = nullptr;  // the _ext entry point's records for this call
  ksg_pod_ext* d_pext = nullptr;         // device copy (batch) / the single pod's (d_one_ext)
  size_t pext_cap = 0;
  ksg_pod_ext* d_one_ext = nullptr;

  // the resident drop-in server (ksg_serve.hip): begin / commit as requests in
  // mapped host memory instead of launches, copies and stream syncs
  bool srv_enabled = true;      // KSG_SERVE=0: the launch-per-call path
  bool srv_running = false;     // a server kernel may be resident on `st`
  KsgSrvBox* srv_box = nullptr;   // pinned, coherent, mapped
  KsgSrvBox* srv_dbox = nullptr;  // its device address
  uint8_t* srv_fail = nullptr;    // fail codes of the shard's nodes (mapped)
  uint8_t* srv_dfail = nullptr;
  size_t srv_fail_cap = 0;
  uint32_t srv_seq = 0;         // last request posted
  uint64_t srv_idle_us = 20000; // the server returns after this long without a request
  bool pend_srv = false;        // the pending begin was served by the server
  uint32_t srv_bhdr[KSG_SRV_HDR_DW] = {};  // that begin's header (its payload layout)
  std::vector<uint64_t> srv_tw;  // its tie words (node lo + 64 i + b), the commit picks from them
  uint32_t srv_unacked = 0;      // a COMMIT posted without waiting for its answer (0: none)
  uint32_t srv_served = 0;       // every request up to this one was served
  uint32_t srv_last_ctl = 0;     // the last control request posted
  bool srv_pext_on = false;      // the pending begin's extension record (its commit carries it)
  ksg_pod_ext srv_pext{};
  uint64_t srv_launches = 0;
  bool srv_grid_on = true;       // KSG_SERVE_GRID=0: the one-workgroup server at every size
  uint32_t srv_npt4_min = 16384;  // KSG_SERVE_GRID_NPT4_MIN: past this many nodes 4 nodes per thread
  uint32_t srv_grid_min = 0;
  bool srv_grid_ext = true;  // KSG_SERVE_GRID_EXT=0: extension contexts on the one-workgroup server  // KSG_SERVE_GRID_MIN: shards above this many nodes take the grid server
                              // (it beats the one-workgroup server at 500 nodes already: 7.2 vs 10.9 us)
  KsgSrvGrid* srv_grid = nullptr;  // its device state (+ the fail codes)
  size_t srv_grid_cap = 0;
  uint32_t srv_epoch = 0;
  bool srv_stamps = false;      // KSG_SERVE_STAMPS=1: sum the server's per-stage cycles of each begin
  int64_t srv_grid_opts = -1;   // KSG_SERVE_GRID_OPTS (KsgSrvArgs.grid_opts; -1: by size)
  bool srv_debug = false;
  unsigned __int128 static_mag = 0;  // max |score| of the terms ksg_set_static_terms added
  // the node labels on the device (ksg_add_static_config evaluates more static terms from them)
  const ksg_node* d_lbl_nodes = nullptr;
  const uint32_t* d_lbl_pairs = nullptr;
  const uint32_t* d_lbl_keys = nullptr;
  bool srv_trace = false;       // KSG_SERVE_TRACE=1: every post, wait and relaunch to stderr       // KSG_SERVE_DEBUG=1: the grid server's stage markers, reported on a fault
  double srv_stage[6] = {};     // (printed by ksg_destroy)
  uint64_t srv_stamped = 0;

  // begin/commit
  bool pending = false;
  uint64_t pending_k = 0;
  ksg_pod pend{};
  std::vector<uint32_t> pend_ids;

  // Every entry point holds `mu`, so reflector threads may call ksg_add_pod /
  // ksg_remove_pod while the scheduling thread schedules. Updates that arrive
  // between ksg_schedule_begin and its commit are queued (validated first) and
  // applied, in arrival order, when the pending pod is committed or abandoned:
  // between pods, never inside one (SURVEY.md 8(b) "Threading").
  std::recursive_mutex mu;
  struct Queued {
    bool add;
    uint32_t host;
    ksg_pod pod;
    std::vector<uint32_t> ids;
    uint64_t uid;
  };
  std::vector<Queued> upd_q;
  std::unordered_set<uint64_t> q_added, q_removed;
};

#define KSG_LOCK(c) std::lock_guard<std::recursive_mutex> ksg_lock_((c)->mu)

namespace {

int fail(ksg_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(c, x)                                                                 \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess)                                                            \
      return fail((c), KSG_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #x,          \
                  hipGetErrorString(e_));                                            \
  } while (0)

#define NCCLCHK(c, x)                                                                \
  do {                                                                               \
    ncclResult_t r_ = (x);                                                           \
    if (r_ != ncclSuccess)                                                           \
      return fail((c), KSG_ERR_RCCL, "%s:%d %s: %s", __FILE__, __LINE__, #x,         \
                  ncclGetErrorString(r_));                                           \
  } while (0)

template <typename T>
int dalloc(ksg_ctx* c, T** p, size_t count, std::vector<void*>* owner) {
  void* q = nullptr;
  HIPCHK(c, hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)));
  HIPCHK(c, hipMemsetAsync(q, 0, std::max<size_t>(count, 1) * sizeof(T), c->st));
  *p = static_cast<T*>(q);
  if (owner) owner->push_back(q);
  return KSG_OK;
}

void free_cluster(ksg_ctx* c) {
  for (void* p : c->cluster_allocs) (void)hipFree(p);
  c->cluster_allocs.clear();
  c->have_cluster = false;
}

int grow(ksg_ctx* c, void** p, size_t* cap, size_t need, size_t elem) {
  if (need <= *cap && *p) return KSG_OK;
  size_t nc = std::max<size_t>(need, std::max<size_t>(*cap * 2, 64));
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  HIPCHK(c, hipMalloc(p, nc * elem));
  *cap = nc;
  return KSG_OK;
}

int pick_R(uint32_t shard_nodes) {
  const uint32_t r = (shard_nodes + KSG_NT - 1) / KSG_NT;
  int R = 1;
  while ((uint32_t)R < r) R <<= 1;
  return R;
}

// ---- patches: host-mirror deltas applied on the device in order ----------
void patch32(ksg_ctx* c, const void* addr, int32_t v) {
  c->patches.push_back(KsgPatch{(uint64_t)(uintptr_t)addr, (uint64_t)(uint32_t)v, 0, 0});
}
void patch64(ksg_ctx* c, const void* addr, int64_t v) {
  c->patches.push_back(KsgPatch{(uint64_t)(uintptr_t)addr, (uint64_t)v, 1, 0});
}
void patch_or(ksg_ctx* c, const void* addr, uint64_t v) {
  c->patches.push_back(KsgPatch{(uint64_t)(uintptr_t)addr, v, 2, 0});
}
void patch_andnot(ksg_ctx* c, const void* addr, uint64_t v) {
  c->patches.push_back(KsgPatch{(uint64_t)(uintptr_t)addr, v, 3, 0});
}

int srv_flush_patches(ksg_ctx* c);

int flush_patches(ksg_ctx* c) {
  if (c->patches.empty()) return KSG_OK;
  if (c->srv_running) return srv_flush_patches(c);
  int rc = grow(c, (void**)&c->d_patch, &c->patch_cap, c->patches.size(), sizeof(KsgPatch));
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_patch, c->patches.data(), c->patches.size() * sizeof(KsgPatch),
                           hipMemcpyHostToDevice, c->st));
  HIPCHK(c, ksg_launch_patch(c->d_patch, (uint32_t)c->patches.size(), c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));  // host vector is reused
  c->patches.clear();
  return KSG_OK;
}

int32_t peer_code(ksg_ctx* c, uint32_t s) {
  if (c->svc_members[s].empty()) return -1;
  const uint32_t h = c->svc_members[s].begin()->second;
  return h < c->N ? (int32_t)h : -2;
}

int32_t recompute_max(ksg_ctx* c, uint32_t s) {
  int32_t m = 0;
  const int32_t* row = c->svc_cnt.data() + (size_t)s * c->N;
  for (uint32_t n = 0; n < c->N; ++n) m = std::max(m, row[n]);
  for (auto& kv : c->svc_ext[s]) m = std::max(m, kv.second);
  return m;
}

// Mirror update for one pod placed on host h. emit=false when the device has
// already applied the same delta (batch commit).
int mirror_add(ksg_ctx* c, uint32_t h, const ksg_pod* p, const uint32_t* ids, bool emit) {
  if (c->pods.count(p->uid)) return fail(c, KSG_ERR_ARG, "duplicate pod uid %llu", (unsigned long long)p->uid);
  PodRec r;
  r.host = h;
  r.cpu = p->milli_cpu;
  r.mem = p->memory;
  r.seq = ++c->seq;
  for (uint32_t i = 0; i < p->n_ports; ++i) r.keys.push_back(ids[p->ports_off + i]);
  for (uint32_t i = 0; i < p->n_pds; ++i) r.keys.push_back(ids[p->pds_off + i]);
  for (uint32_t i = 0; i < p->n_svcs; ++i) r.svcs.push_back(ids[p->svcs_off + i]);
  for (uint32_t k : r.keys)
    if (k >= c->cfg.max_conflict_keys)
      return fail(c, KSG_ERR_CAPACITY, "conflict key %u >= max_conflict_keys %u", k, c->cfg.max_conflict_keys);
  for (uint32_t s : r.svcs)
    if (s >= c->S) return fail(c, KSG_ERR_ARG, "service %u >= n_services %u", s, c->S);
  for (uint32_t q = 0; q < KSG_MAX_SCALAR; ++q) r.scalar[q] = 0;
  if (c->ext_on && c->ext.n_scalar) {  // extension: the pod's extended resource requests
    auto it = c->ext_scalar.find(p->uid);
    if (it != c->ext_scalar.end())
      for (uint32_t q = 0; q < c->ext.n_scalar; ++q) r.scalar[q] = it->second[q];
    if (h < c->N)
      for (uint32_t q = 0; q < c->ext.n_scalar; ++q) {
        if (!r.scalar[q]) continue;
        int64_t& u = c->sc_used[(size_t)q * c->N + h];
        u = (int64_t)((uint64_t)u + (uint64_t)r.scalar[q]);
        if (emit) patch64(c, c->dev.scalar_used + (size_t)q * c->N + h, u);
      }
  }
  if (h < c->N) {
    c->used_c[h] = (int64_t)((uint64_t)c->used_c[h] + (uint64_t)r.cpu);
    c->used_m[h] = (int64_t)((uint64_t)c->used_m[h] + (uint64_t)r.mem);
    if (c->mu_neg || c->used_c[h] < 0 || c->used_m[h] < 0) c->mu_dirty = true;
    else c->mu_max = std::max(c->mu_max, std::max(c->used_c[h], c->used_m[h]));
    if (emit) {
      patch64(c, c->dev.used_cpu + h, c->used_c[h]);
      patch64(c, c->dev.used_mem + h, c->used_m[h]);
    }
    for (uint32_t k : r.keys) {
      const uint32_t ref = ++c->key_ref[((uint64_t)k << 32) | h];
      if (ref == 1 && emit) patch_or(c, c->dev.keymap + (size_t)k * c->nw + (h >> 6), 1ULL << (h & 63));
    }
  }
  for (uint32_t s : r.svcs) {
    int32_t v;
    if (h < c->N) {
      v = ++c->svc_cnt[(size_t)s * c->N + h];
      if (emit) patch32(c, c->dev.svc_cnt + (size_t)s * c->N + h, v);
      if (emit && v == 1) patch_or(c, c->dev.svc_bits + (size_t)s * c->nw + (h >> 6), 1ULL << (h & 63));
    } else {
      v = ++c->svc_ext[s][h];
    }
    if (v > c->svc_max[s]) {
      c->svc_max[s] = v;
      if (emit) patch32(c, c->dev.svc_max + s, v);
    }
    ++c->svc_total[s];
    if (emit) patch32(c, c->dev.svc_total + s, c->svc_total[s]);
    c->svc_members[s][r.seq] = h;
    const int32_t pc = peer_code(c, s);
    if (pc != c->svc_peer[s]) {
      c->svc_peer[s] = pc;
      if (emit) patch32(c, c->dev.svc_peer + s, pc);
    }
  }
  c->pods.emplace(p->uid, std::move(r));
  return KSG_OK;
}

void reset_mirror(ksg_ctx* c) {
  c->used_c.assign(c->N, 0);
  c->mu_dirty = true;
  c->used_m.assign(c->N, 0);
  c->sc_used.assign((size_t)c->ext.n_scalar * c->N, 0);
  c->ext_scalar.clear();
  c->key_ref.clear();
  c->svc_cnt.assign((size_t)c->S * c->N, 0);
  c->svc_ext.assign(c->S, {});
  c->svc_max.assign(c->S, 0);
  c->svc_total.assign(c->S, 0);
  c->svc_peer.assign(c->S, -1);
  c->svc_members.assign(c->S, {});
  c->pods.clear();
  c->seq = 0;
  c->patches.clear();
  c->pending = false;
  c->pend_srv = false;
  c->upd_q.clear();
  c->q_added.clear();
  c->q_removed.clear();
}

int check_pod(ksg_ctx* c, const ksg_pod* p, const uint32_t* ids, size_t n_ids) {
  auto in = [&](uint32_t off, uint32_t n) { return (size_t)off + n <= n_ids; };
  if (!in(p->ports_off, p->n_ports) || !in(p->pds_off, p->n_pds) || !in(p->sel_off, p->n_sel) ||
      !in(p->svcs_off, p->n_svcs))
    return fail(c, KSG_ERR_ARG, "pod id list out of range");
  if (p->host < -2 || p->host >= (int32_t)c->N) return fail(c, KSG_ERR_ARG, "pod host %d out of range", p->host);
  if (p->service < -1 || p->service >= (int32_t)c->S) return fail(c, KSG_ERR_ARG, "pod service out of range");
  for (uint32_t i = 0; i < p->n_ports; ++i)
    if (ids[p->ports_off + i] >= c->cfg.max_conflict_keys) return fail(c, KSG_ERR_CAPACITY, "port key out of range");
  for (uint32_t i = 0; i < p->n_pds; ++i)
    if (ids[p->pds_off + i] >= c->cfg.max_conflict_keys) return fail(c, KSG_ERR_CAPACITY, "pd key out of range");
  for (uint32_t i = 0; i < p->n_sel; ++i)
    if (ids[p->sel_off + i] >= c->n_pairs) return fail(c, KSG_ERR_ARG, "selector pair out of range");
  for (uint32_t i = 0; i < p->n_svcs; ++i)
    if (ids[p->svcs_off + i] >= c->S) return fail(c, KSG_ERR_ARG, "service id out of range");
  for (uint32_t j = 0; j < c->cfg.n_aff_labels; ++j)
    if (p->aff_pair[j] >= (int32_t)c->n_pairs || p->aff_pair[j] < KSG_AFF_INVALID)
      return fail(c, KSG_ERR_ARG, "affinity pair out of range");
  return KSG_OK;
}

// upload one pod + its id list into the single-pod scratch slots
int grow_host(ksg_ctx* c, uint8_t** p, size_t* cap, size_t need);

int upload_pods(ksg_ctx* c, const ksg_pod* pods, uint32_t n, const uint32_t* ids, size_t n_ids) {
  int rc = grow(c, (void**)&c->d_pods, &c->pods_cap, n, sizeof(ksg_pod));
  if (rc) return rc;
  rc = grow(c, (void**)&c->d_ids, &c->ids_cap, std::max<size_t>(n_ids, 1), sizeof(uint32_t));
  if (rc) return rc;
  // every caller synchronises the stream before it returns, so the staging
  // buffer is free again at the next call
  const size_t pb = (size_t)n * sizeof(ksg_pod), ib = n_ids * sizeof(uint32_t);
  if ((rc = grow_host(c, &c->h_up, &c->h_up_cap, pb + ib))) return rc;
  memcpy(c->h_up, pods, pb);
  if (n_ids) memcpy(c->h_up + pb, ids, ib);
  HIPCHK(c, hipMemcpyAsync(c->d_pods, c->h_up, pb, hipMemcpyHostToDevice, c->st));
  if (n_ids) HIPCHK(c, hipMemcpyAsync(c->d_ids, c->h_up + pb, ib, hipMemcpyHostToDevice, c->st));
  return KSG_OK;
}

// the single-pod APIs: pod + ids staged contiguously, one copy into d_one;
// one_pod / one_ids point into it until the next single-pod upload
int upload_one(ksg_ctx* c, const ksg_pod* pod, const uint32_t* ids, size_t n_ids) {
  const size_t pb = (sizeof(ksg_pod) + 15) & ~(size_t)15, ib = std::max<size_t>(n_ids, 1) * sizeof(uint32_t);
  // (extensions: the pod's ksg_pod_ext after the ids, all-zero for the plain entry points)
  const size_t eo = (pb + ib + 15) & ~(size_t)15, eb = c->ext_on ? sizeof(ksg_pod_ext) : 0;
  int rc = grow(c, (void**)&c->d_one, &c->one_cap, eo + eb, 1);
  if (rc) return rc;
  if ((rc = grow_host(c, &c->h_up, &c->h_up_cap, eo + eb))) return rc;
  memcpy(c->h_up, pod, sizeof(ksg_pod));
  if (n_ids) memcpy(c->h_up + pb, ids, n_ids * sizeof(uint32_t));
  if (eb) {
    if (c->cur_ext) memcpy(c->h_up + eo, c->cur_ext, eb);
    else memset(c->h_up + eo, 0, eb);
  }
  HIPCHK(c, hipMemcpyAsync(c->d_one, c->h_up, eb ? eo + eb : pb + (n_ids ? n_ids * sizeof(uint32_t) : 0),
                           hipMemcpyHostToDevice, c->st));
  c->one_pod = reinterpret_cast<const ksg_pod*>(c->d_one);
  c->one_ids = reinterpret_cast<const uint32_t*>(c->d_one + pb);
  c->d_one_ext = eb ? reinterpret_cast<ksg_pod_ext*>(c->d_one + eo) : nullptr;
  return KSG_OK;
}

int ensure_map(ksg_ctx* c) {
  if (c->h_map) return KSG_OK;
  HIPCHK(c, hipHostMalloc((void**)&c->h_map, 64, hipHostMallocCoherent));
  void* dp = nullptr;
  HIPCHK(c, hipHostGetDevicePointer(&dp, c->h_map, 0));
  c->d_map = static_cast<uint8_t*>(dp);
  return KSG_OK;
}

size_t pod_ids_extent(const ksg_pod* p) {
  size_t e = 0;
  e = std::max<size_t>(e, (size_t)p->ports_off + p->n_ports);
  e = std::max<size_t>(e, (size_t)p->pds_off + p->n_pds);
  e = std::max<size_t>(e, (size_t)p->sel_off + p->n_sel);
  e = std::max<size_t>(e, (size_t)p->svcs_off + p->n_svcs);
  return e;
}
// ... and the extension record's taint lists (the single-pod _ext entry points)
size_t call_ids_extent(const ksg_ctx* c, const ksg_pod* p) {
  size_t e = pod_ids_extent(p);
  if (c->cur_ext) {
    e = std::max<size_t>(e, (size_t)c->cur_ext->hard_off + c->cur_ext->n_hard);
    e = std::max<size_t>(e, (size_t)c->cur_ext->soft_off + c->cur_ext->n_soft);
  }
  return e;
}

// the shard records decide reads: all-gathered (exchange path) or this rank's own
uint8_t* rec_buf(ksg_ctx* c) { return c->xchg ? c->d_rec_recv : c->d_rec_send; }

bool anti_on(const ksg_ctx* c) { return c->cfg.n_anti > 0 && c->dev.n_domains_total > 0; }

// ---- cross-rank exchange: RCCL over xGMI, or the caller's host transport ----
int grow_host(ksg_ctx* c, uint8_t** p, size_t* cap, size_t need) {
  if (*cap >= need) return KSG_OK;
  // geometric: a pinned (re)allocation costs ~0.2 ms (hipHostFree synchronises)
  const size_t nc = std::max<size_t>(need, std::max<size_t>(*cap * 2, 4096));
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  HIPCHK(c, hipHostMalloc((void**)p, nc, hipHostMallocDefault));
  *cap = nc;
  return KSG_OK;
}

// recv[g * bytes, (g + 1) * bytes) = rank g's send, on c->st
int allgather(ksg_ctx* c, const void* dsend, void* drecv, size_t bytes) {
  if (c->comm) {
    NCCLCHK(c, ncclAllGather(dsend, drecv, bytes, ncclUint8, c->comm, c->st));
    return KSG_OK;
  }
  if (!c->xfn) return fail(c, KSG_ERR_STATE, "sharded context has neither an RCCL communicator nor ksg_set_allgather");
  int rc;
  if ((rc = grow_host(c, &c->h_xsend, &c->h_xsend_cap, bytes)) ||
      (rc = grow_host(c, &c->h_xrecv, &c->h_xrecv_cap, bytes * c->world)))
    return rc;
  HIPCHK(c, hipMemcpyAsync(c->h_xsend, dsend, bytes, hipMemcpyDeviceToHost, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  if ((rc = c->xfn(c->xuser, c->h_xsend, c->h_xrecv, (uint64_t)bytes)) != 0)
    return fail(c, KSG_ERR_RCCL, "allgather callback returned %d", rc);
  HIPCHK(c, hipMemcpyAsync(drecv, c->h_xrecv, bytes * c->world, hipMemcpyHostToDevice, c->st));
  return KSG_OK;
}

int allreduce_sum_i32(ksg_ctx* c, const int32_t* dsend, int32_t* drecv, uint32_t n) {
  if (c->comm) {
    NCCLCHK(c, ncclAllReduce(dsend, drecv, n, ncclInt32, ncclSum, c->comm, c->st));
    return KSG_OK;
  }
  if (!c->xfn) return fail(c, KSG_ERR_STATE, "sharded context has neither an RCCL communicator nor ksg_set_allgather");
  const size_t bytes = (size_t)n * 4;
  int rc;
  if ((rc = grow_host(c, &c->h_xsend, &c->h_xsend_cap, bytes)) ||
      (rc = grow_host(c, &c->h_xrecv, &c->h_xrecv_cap, bytes * (c->world + 1))))
    return rc;
  HIPCHK(c, hipMemcpyAsync(c->h_xsend, dsend, bytes, hipMemcpyDeviceToHost, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  if ((rc = c->xfn(c->xuser, c->h_xsend, c->h_xrecv, (uint64_t)bytes)) != 0)
    return fail(c, KSG_ERR_RCCL, "allgather callback returned %d", rc);
  int32_t* all = reinterpret_cast<int32_t*>(c->h_xrecv);
  int32_t* sum = all + (size_t)n * c->world;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t acc = 0;  // wrapping, as ncclSum on int32
    for (int g = 0; g < c->world; ++g) acc += (uint32_t)all[(size_t)g * n + i];
    sum[i] = (int32_t)acc;
  }
  HIPCHK(c, hipMemcpyAsync(drecv, sum, bytes, hipMemcpyHostToDevice, c->st));
  return KSG_OK;
}

int allreduce_max_i32(ksg_ctx* c, const int32_t* dsend, int32_t* drecv, uint32_t n) {
  if (c->comm) {
    NCCLCHK(c, ncclAllReduce(dsend, drecv, n, ncclInt32, ncclMax, c->comm, c->st));
    return KSG_OK;
  }
  if (!c->xfn) return fail(c, KSG_ERR_STATE, "sharded context has neither an RCCL communicator nor ksg_set_allgather");
  const size_t bytes = (size_t)n * 4;
  int rc;
  if ((rc = grow_host(c, &c->h_xsend, &c->h_xsend_cap, bytes)) ||
      (rc = grow_host(c, &c->h_xrecv, &c->h_xrecv_cap, bytes * (c->world + 1))))
    return rc;
  HIPCHK(c, hipMemcpyAsync(c->h_xsend, dsend, bytes, hipMemcpyDeviceToHost, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  if ((rc = c->xfn(c->xuser, c->h_xsend, c->h_xrecv, (uint64_t)bytes)) != 0)
    return fail(c, KSG_ERR_RCCL, "allgather callback returned %d", rc);
  int32_t* all = reinterpret_cast<int32_t*>(c->h_xrecv);
  int32_t* mx = all + (size_t)n * c->world;
  for (uint32_t i = 0; i < n; ++i) {
    int32_t m = all[i];
    for (int g = 1; g < c->world; ++g) m = std::max(m, all[(size_t)g * n + i]);
    mx[i] = m;
  }
  HIPCHK(c, hipMemcpyAsync(drecv, mx, bytes, hipMemcpyHostToDevice, c->st));
  return KSG_OK;
}

// one pod through scan [+ the normalised terms' all-reduces] + record all-gather (device
// only). On a sharded context ServiceAntiAffinity's domain counts and the extension
// TaintTolerationPriority's max are over every shard's filtered nodes: a first pass writes
// this shard's part (dpart: the counts, then the max), the all-reduces combine them (sum,
// max) and the full pass reads the result (dglobal). dext: the pod's extension record.
int scan_exchange(ksg_ctx* c, const ksg_pod* dpod, const uint32_t* dids, int mode, uint8_t* fail_out,
                  int64_t* score_out, const ksg_pod_ext* dext) {
  const bool anti = anti_on(c);
  const bool tt = dext != nullptr && c->ext.w_taint_toleration != 0;
  if ((anti || tt) && c->xchg) {
    HIPCHK(c, ksg_launch_scan(c->R, anti, c->dev, dpod, dids, mode, 1, nullptr, nullptr, c->d_rec_send,
                              c->d_dpart, nullptr, c->st, dext));
    const uint32_t D = c->dev.n_domains_total;
    int rc = anti ? allreduce_sum_i32(c, c->d_dpart, c->d_dglobal, D) : KSG_OK;
    if (!rc && tt) rc = allreduce_max_i32(c, c->d_dpart + D, c->d_dglobal + D, 1);
    if (rc) return rc;
    HIPCHK(c, ksg_launch_scan(c->R, anti, c->dev, dpod, dids, mode, 2, fail_out, score_out, c->d_rec_send,
                              nullptr, c->d_dglobal, c->st, dext));
  } else {
    HIPCHK(c, ksg_launch_scan(c->R, anti, c->dev, dpod, dids, mode, 0, fail_out, score_out, c->d_rec_send,
                              nullptr, nullptr, c->st, dext));
  }
  if (mode == KSG_MODE_BEGIN) {
    if (c->xchg) {
      int rc = allgather(c, c->d_rec_send, c->d_rec_recv, c->rec_bytes);
      if (rc) return rc;
    }  // (one rank: decide reads the record where the scan wrote it, rec_buf)
  }
  return KSG_OK;
}

// The window path needs scores that commits can only lower (see ksg_window.hip):
// non-negative LeastRequested / ServiceSpreading weights and int64 totals far
// from wrapping (ServiceAntiAffinity is handled by its count pass and stops).
// The resolver walks the whole node set on every rank (state is replicated).
KsgDev full_geometry(const ksg_ctx* c) {
  KsgDev f = c->dev;
  f.lo = 0;
  f.hi = c->N;
  f.wlo = 0;
  f.nwords = c->nw;
  return f;
}

bool use_window(ksg_ctx* c, const ksg_pod* pods, uint32_t n) {
  if (c->window == 0 || c->nw > 32 * 64 || ksg_win_max_window(full_geometry(c)) < 8) return false;
  // extensions: PodToleratesNodeTaints is static per (pod, node); extended
  // resources only shrink under commits and the resolver re-checks them on the
  // window's committed nodes like cpu / memory. With TaintToleration /
  // BalancedAllocation scores the resolver re-scores the committed nodes (a
  // BalancedAllocation score can RISE: ksg_plain.hip's risers and joiners); the
  // TaintToleration term needs the node taints as one mask (max_taints <= 64).
  // ServiceAntiAffinity, negative requests and requests past 2^16 take the exact
  // kernels.
  if (c->ext_on) {
    // ServiceAntiAffinity with the extensions: the window path only for the static filters —
    // PodToleratesNodeTaints, and extended resources no pod of the batch requests (a zero request
    // fits whatever the node's usage) — with both extension scores off: the anti-affinity
    // resolvers re-check nothing extension-specific on the window's committed nodes
    if (anti_on(c)) {
      if (c->ext.w_taint_toleration != 0 || c->ext.w_balanced != 0) return false;
      if (c->cur_ext)
        for (uint32_t i = 0; i < n; ++i)
          for (uint32_t r = 0; r < c->ext.n_scalar; ++r)
            if (c->cur_ext[i].scalar[r] != 0) return false;
    }
    if (c->ext.w_taint_toleration != 0 && !c->dev.ntaint) return false;
    if (c->cur_ext)
      for (uint32_t i = 0; i < n; ++i)
        for (uint32_t r = 0; r < c->ext.n_scalar; ++r)
          if (c->cur_ext[i].scalar[r] < 0 || c->cur_ext[i].scalar[r] > KSG_WIN_XREQ_BOUND) return false;
  }
  // int64 combined scores
  if (c->dev.wide) return false;
  // monotonicity under commits needs non-negative pod-dependent weights
  if (c->cfg.w_least_requested < 0 || c->cfg.w_service_spreading < 0) return false;
  // lr_win (ksg_device.h) is exact for 0 <= capacity, requested totals <= 2^49
  const int64_t lim = KSG_WIN_LR_BOUND;
  if (c->max_cap > lim || c->min_cap < 0) return false;
  if (c->mu_dirty) {
    c->mu_max = 0;
    c->mu_neg = false;
    for (uint32_t i = 0; i < c->N; ++i) {
      c->mu_neg |= c->used_c[i] < 0 || c->used_m[i] < 0;
      c->mu_max = std::max<int64_t>(c->mu_max, std::max<int64_t>(c->used_c[i], c->used_m[i]));
    }
    c->mu_dirty = false;
  }
  if (c->mu_neg) return false;
  const int64_t mu = c->mu_max;
  // commits not yet in the mirror (non-negative: checked by the caller) only add
  int64_t sum = c->dfr_sum;
  for (uint32_t i = 0; i < n; ++i) {
    if (pods[i].milli_cpu < 0 || pods[i].memory < 0) return false;
    sum += std::min<int64_t>(pods[i].milli_cpu + pods[i].memory, lim);
    if (sum > lim) return false;
  }
  return mu + sum <= lim;
}

// |combined score| bound of a weight set: 10 * sum |w| over the score-10
// priorities + |w_equal| (+ the extensions'), exact in 128 bits
unsigned __int128 score_bound(const ksg_config& cf, int64_t w_taint, int64_t w_bal) {
  auto mag = [](int64_t w) -> unsigned __int128 { return w < 0 ? (unsigned __int128)(0 - (uint64_t)w) : (unsigned __int128)w; };
  unsigned __int128 b = 10 * (mag(cf.w_least_requested) + mag(cf.w_service_spreading) + mag(w_taint) + mag(w_bal)) +
                        mag(cf.w_equal);
  for (uint32_t a = 0; a < cf.n_anti; ++a) b += 10 * mag(cf.w_anti[a]);
  for (uint32_t q = 0; q < cf.n_label_pref; ++q) b += 10 * mag(cf.w_pref[q]);
  return b;
}

int cluster_ok(ksg_ctx* c) {
  if (!c->have_cluster) return fail(c, KSG_ERR_STATE, "ksg_set_cluster not called");
  if (c->diverged)
    return fail(c, KSG_ERR_STATE, "device state diverged from the host mirror (a batch failed after its device work "
                "started, or the drop-in server rejected a commit): call ksg_set_cluster");
  return KSG_OK;
}

void drop_deferred(ksg_ctx* c) {
  c->dfr_pods.clear();
  c->dfr_ids.clear();
  c->dfr_out.clear();
  c->dfr_uids.clear();
  c->dfr_sum = 0;
  c->dfr_neg = false;
}

int flush_deferred(ksg_ctx* c) {
  int rc = KSG_OK;
  for (size_t i = 0; i < c->dfr_out.size() && rc == KSG_OK; ++i)
    if (c->dfr_out[i] >= 0) rc = mirror_add(c, (uint32_t)c->dfr_out[i], &c->dfr_pods[i], c->dfr_ids.data(), false);
  drop_deferred(c);
  return rc;
}

int ensure_out(ksg_ctx* c, size_t n) { return grow(c, (void**)&c->d_out, &c->out_cap, n, sizeof(int32_t)); }

// Waits for the stream's work so far. The batch path's host thread has nothing
// left to do at this point, so it polls an event instead of sleeping in
// hipStreamSynchronize, whose wake-up lands on the per-batch critical path.
int wait_device(ksg_ctx* c) {
  if (!c->spin_wait || !c->ev_wait) {
    HIPCHK(c, hipStreamSynchronize(c->st));
    return KSG_OK;
  }
  HIPCHK(c, hipEventRecord(c->ev_wait, c->st));
  hipError_t e;
  while ((e = hipEventQuery(c->ev_wait)) == hipErrorNotReady) {
  }
  if (e != hipSuccess) return fail(c, KSG_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(e));
  return KSG_OK;
}

// ---- the resident drop-in server (ksg_serve.hip) ------------------------------
// the grid server: plain configurations (no ServiceAntiAffinity, no extensions)
// past srv_grid_min nodes, one scan workgroup per 256 nodes (<= 255)
// nodes per thread of the grid server's scan workgroups
uint32_t srv_npt(const ksg_ctx* c) { return c->hi - c->lo > c->srv_npt4_min ? 4u : 1u; }

bool srv_grid(const ksg_ctx* c) {
  const uint32_t n = c->hi - c->lo, per = KSG_GSRV_NT * srv_npt(c);
  // (extensions: the filters and BalancedAllocation are per node; TaintToleration normalises over
  // the filtered set: the scan workgroups exchange their maxima through device memory)
  // (ServiceAntiAffinity: the domain counts likewise, up to KSG_GSRV_MAXD domains, without extensions)
  return c->srv_grid_on && !(anti_on(c) && (c->ext_on || c->dev.n_domains_total > KSG_GSRV_MAXD)) &&
         !(c->ext_on && !c->srv_grid_ext) &&
         n > c->srv_grid_min &&
         (n + per - 1) / per <= KSG_GSRV_MAXW;
}

bool srv_eligible(const ksg_ctx* c) {
  return c->srv_enabled && c->world == 1 && !c->xchg && (c->R <= KSG_SRV_MAX_R || srv_grid(c)) && !c->dev.wide &&
         c->N > 0;
}

int srv_alloc(ksg_ctx* c) {
  if (!c->srv_box) {
    HIPCHK(c, hipHostMalloc((void**)&c->srv_box, sizeof(KsgSrvBox), hipHostMallocCoherent | hipHostMallocMapped));
    memset(c->srv_box, 0, sizeof(KsgSrvBox));
    void* dp = nullptr;
    HIPCHK(c, hipHostGetDevicePointer(&dp, c->srv_box, 0));
    c->srv_dbox = static_cast<KsgSrvBox*>(dp);
  }
  return KSG_OK;
}

// (Re)launches the server on the stream, offering every request after the last
// one answered. A COMMIT is posted without waiting for its answer, so the host's
// srv_served may lag the server's: the response block names the last request the
// server answered, and a server answers a request only once it will complete it
// (the one-workgroup server applies a COMMIT's delta after answering it, before
// it reads the next request or returns). Relaunching at srv_served alone would
// offer an answered COMMIT again and apply its delta twice.
int srv_launch(ksg_ctx* c) {
  if (int rc = srv_alloc(c)) return rc;
  const uint32_t r0 = __atomic_load_n(&c->srv_box->resp[0], __ATOMIC_ACQUIRE);
  if ((int32_t)(r0 - c->srv_served) > 0) c->srv_served = r0;
  const uint32_t start_seq = c->srv_served;
  const size_t nf = ((size_t)(c->hi - c->lo) + 3 & ~(size_t)3) + 64;  // (the grid server stores 4 codes at a time)
  if (c->srv_fail_cap < nf) {
    if (c->srv_fail) (void)hipHostFree(c->srv_fail);
    c->srv_fail = nullptr;
    c->srv_fail_cap = 0;
    HIPCHK(c, hipHostMalloc((void**)&c->srv_fail, nf, hipHostMallocCoherent | hipHostMallocMapped));
    void* dp = nullptr;
    HIPCHK(c, hipHostGetDevicePointer(&dp, c->srv_fail, 0));
    c->srv_dfail = static_cast<uint8_t*>(dp);
    c->srv_fail_cap = nf;
  }
  KsgSrvArgs a{c->srv_dbox, c->srv_dfail, start_seq, (uint64_t)c->srv_idle_us * 100,
               (c->srv_stamps ? 1u : 0u) | (c->srv_debug ? 2u : 0u),
               nullptr, 0, ++c->srv_epoch, 0};
  if (srv_grid(c)) {
    const uint32_t n = c->hi - c->lo;
    const size_t need = sizeof(KsgSrvGrid);
    if (c->srv_grid_cap < need) {
      if (c->srv_grid) (void)hipFree(c->srv_grid);
      c->srv_grid = nullptr;
      c->srv_grid_cap = 0;
      HIPCHK(c, hipMalloc((void**)&c->srv_grid, need));
      HIPCHK(c, hipMemsetAsync(c->srv_grid, 0, need, c->st));
      c->srv_grid_cap = need;
    }
    a.grid = c->srv_grid;
    const uint32_t npt = srv_npt(c);
    a.n_workers = (n + KSG_GSRV_NT * npt - 1) / (KSG_GSRV_NT * npt);
    // past 64 scan workgroups their polls of the host block crowd the link: each sleeps ~0.2 us
    // more between polls (measured: 50,000 nodes 73 -> 38 us per pod; no gain at 15,000)
    a.grid_opts = c->srv_grid_opts >= 0 ? (uint32_t)c->srv_grid_opts : a.n_workers > 64 ? 0x10u : 0u;
    HIPCHK(c, ksg_launch_serve_grid((int)npt, c->ext_on, c->dev, a, c->st));
  } else {
    HIPCHK(c, ksg_launch_serve(c->R, anti_on(c), c->ext_on, c->dev, a, c->st));
  }
  c->srv_running = true;
  ++c->srv_launches;
  return KSG_OK;
}

// Waits until request `seq` is answered: its response, or (a grid server's
// BEGIN, parts > 0) that many parts. A server that returned (idle) before it saw
// the request is relaunched to serve it.
int srv_wait(ksg_ctx* c, uint32_t seq, uint32_t parts) {
  const uint32_t* rs = c->srv_box->resp;
  auto done = [&]() {
    if (!parts) return (int32_t)(__atomic_load_n(&rs[0], __ATOMIC_ACQUIRE) - seq) >= 0;  // (answered in order)
    for (uint32_t q = 0; q < parts; ++q)
      if (__atomic_load_n(&c->srv_box->part[q].seq, __ATOMIC_ACQUIRE) != seq ||
          __atomic_load_n(&c->srv_box->part[q].stamp[3], __ATOMIC_ACQUIRE) != seq)  // (both ends of the store)
        return false;
    return true;
  };
  auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0, relaunches = 0;
  while (!done()) {
    if ((++spins & 255) != 0) continue;
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (us < 20.0) continue;
    const hipError_t q = hipStreamQuery(c->st);
    if (q == hipSuccess) {  // the server returned without serving `seq`
      if (done()) break;
      if (++relaunches > 3) return fail(c, KSG_ERR_HIP, "drop-in server exits without serving request %u", seq);
      c->srv_running = false;
      if (c->srv_trace) fprintf(stderr, "srv relaunch start %u (waiting %u)\n", c->srv_served, seq);
      if (int rc = srv_launch(c)) return rc;  // (every request after the last answered one is offered again)
      t0 = std::chrono::steady_clock::now();
    } else if (q != hipErrorNotReady) {
      c->srv_running = false;
      std::string marks;
      if (c->srv_debug)  // where each workgroup was (seq:stage), leader first
        for (int i = 0; i < 12; ++i) {
          const uint32_t m = __atomic_load_n(&c->srv_box->dbg[i], __ATOMIC_RELAXED);
          marks += " " + std::to_string(m >> 8) + ":" + std::to_string(m & 255);
        }
      return fail(c, KSG_ERR_HIP, "drop-in server: %s (request %u%s)", hipGetErrorString(q), seq, marks.c_str());
    } else if (us > 5e6) {
      return fail(c, KSG_ERR_HIP, "drop-in server did not answer request %u in 5 s", seq);
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  if ((int32_t)(seq - c->srv_served) > 0) c->srv_served = seq;  // (and every request before it)
  return KSG_OK;
}

// The control block is free once the server has read the last COMMIT (posted
// without waiting for its answer): before the host writes a control request.
int srv_settle(ksg_ctx* c) {
  if (!c->srv_unacked) return KSG_OK;
  const uint32_t u = c->srv_unacked;
  c->srv_unacked = 0;
  if ((int32_t)(c->srv_served - u) < 0)
    if (int rc = srv_wait(c, u, 0)) return rc;
  // resp[KSG_SRV_RESP_REJECTED]: the last request the server rejected, written before its
  // response (later BEGIN answers overwrite resp[0..3], not this word). The host mirror
  // already holds the commit's pod and the device does not: the context is diverged.
  if (__atomic_load_n(&c->srv_box->resp[KSG_SRV_RESP_REJECTED], __ATOMIC_ACQUIRE) == u) {
    c->diverged = true;
    return fail(c, KSG_ERR_STATE, "drop-in server rejected commit request %u (ksg_set_cluster resyncs)", u);
  }
  return KSG_OK;
}

// Posts request ++srv_seq (header dwords hdr[0..KSG_SRV_HDR_DW); the payload
// chunks were written by the caller): a BEGIN into `req`, a control request into
// `creq` once the last COMMIT there was read. A BEGIN carries the last control
// request before it (ARG).
int srv_post(ksg_ctx* c, const uint32_t* hdr_in, uint32_t* seq_out) {
  if (!c->srv_running) {
    if (int rc = srv_launch(c)) return rc;
  }
  const bool ctl = hdr_in[KSG_SRVH_KIND] != KSG_SRV_BEGIN;
  if (ctl) {
    if (int rc = srv_settle(c)) return rc;
  }
  uint32_t hdr[KSG_SRV_HDR_DW];
  memcpy(hdr, hdr_in, sizeof hdr);
  if (!ctl) hdr[KSG_SRVH_ARG] = c->srv_last_ctl;
  if (c->dbg_corrupt) {
    const uint32_t bit = hdr[KSG_SRVH_KIND] == KSG_SRV_COMMIT ? 1u : hdr[KSG_SRVH_KIND] == KSG_SRV_BEGIN ? 2u : 0u;
    if (c->dbg_corrupt & bit) {
      hdr[KSG_SRVH_IDS_AT] = KSG_SRV_PAY_DW + 1;  // (past the payload: req_bad)
      c->dbg_corrupt &= ~bit;
    }
  }
  const uint32_t seq = ++c->srv_seq;
  if (ctl) c->srv_last_ctl = seq;
  if (c->srv_trace)
    fprintf(stderr, "srv post %u kind %u arg %u served %u\n", seq, hdr[KSG_SRVH_KIND], hdr[KSG_SRVH_ARG], c->srv_served);
  uint32_t* req = ctl ? c->srv_box->creq : c->srv_box->req;
  for (uint32_t i = 0; i < KSG_SRV_HDR_DW; ++i) req[4 * (i / KSG_SRV_CHUNK_DW) + i % KSG_SRV_CHUNK_DW] = hdr[i];
  std::atomic_thread_fence(std::memory_order_release);  // data, then tags (x86: stores stay in order)
  for (uint32_t q = 0; q < KSG_SRV_CHUNKS; ++q) __atomic_store_n(&req[4 * q + 3], seq, __ATOMIC_RELEASE);
  *seq_out = seq;
  return KSG_OK;
}

// Posts a request and waits for its response {seq, a, b, c}.
int srv_call(ksg_ctx* c, const uint32_t* hdr, uint32_t* resp4) {
  uint32_t seq = 0;
  if (int rc = srv_post(c, hdr, &seq)) return rc;
  if (int rc = srv_wait(c, seq, 0)) return rc;
  const uint32_t* rs = c->srv_box->resp;
  for (int i = 0; i < 4; ++i) resp4[i] = __atomic_load_n(&rs[i], __ATOMIC_RELAXED);
  if (c->srv_stamps && hdr[KSG_SRVH_KIND] == KSG_SRV_BEGIN && __atomic_load_n(&rs[10], __ATOMIC_RELAXED) == seq) {
    for (int i = 0; i < 6; ++i) c->srv_stage[i] += (int32_t)__atomic_load_n(&rs[4 + i], __ATOMIC_RELAXED);
    ++c->srv_stamped;
  }
  return KSG_OK;
}

// A BEGIN on either server: {k | ~0u (no peer) | KSG_SRV_BADREQ, max} and the
// tie words into srv_tw. The grid server's parts are merged here.
int srv_begin(ksg_ctx* c, const uint32_t* hdr, uint32_t* resp4) {
  const uint32_t n = c->hi - c->lo, nwd = (n + 63) / 64;
  if (!srv_grid(c)) {
    if (int rc = srv_call(c, hdr, resp4)) return rc;
    if (resp4[1] != KSG_SRV_BADREQ && resp4[1] != ~0u && resp4[1] > 0)
      c->srv_tw.assign(c->srv_box->ties, c->srv_box->ties + nwd);
    return KSG_OK;
  }
  const uint32_t npt = srv_npt(c), G = (n + KSG_GSRV_NT * npt - 1) / (KSG_GSRV_NT * npt), NWG = 4 * npt;
  uint32_t seq = 0;
  if (int rc = srv_post(c, hdr, &seq)) return rc;
  if (int rc = srv_wait(c, seq, G)) return rc;
  const KsgSrvPart* pt = c->srv_box->part;
  int32_t M = KSG_S32_NONE;
  uint32_t err = 0;
  for (uint32_t q = 0; q < G; ++q) {
    M = std::max(M, pt[q].max);
    err |= pt[q].err;
  }
  uint32_t k = 0;
  c->srv_tw.assign((size_t)G * NWG, 0);
  if (M != KSG_S32_NONE)
    for (uint32_t q = 0; q < G; ++q)
      if (pt[q].max == M) {
        k += pt[q].cnt;
        const uint64_t* tw = npt == 1 ? pt[q].tie : c->srv_box->part_tie + (size_t)q * KSG_GSRV_TIEW;
        for (uint32_t r = 0; r < NWG; ++r) c->srv_tw[(size_t)q * NWG + r] = tw[r];
      }
  c->srv_tw.resize(nwd);
  if (c->srv_stamps) {  // worker 0: masks + loads, eval + publish (100-MHz ticks)
    c->srv_stage[0] += (int32_t)(pt[0].stamp[1] - pt[0].stamp[0]);
    c->srv_stage[1] += (int32_t)(pt[0].stamp[2] - pt[0].stamp[1]);  // (stamp[3]: the sequence number)
    ++c->srv_stamped;
  }
  resp4[0] = seq;
  resp4[1] = (err & 2) ? KSG_SRV_BADREQ : err ? ~0u : k;
  if (c->srv_trace) fprintf(stderr, "srv begin %u max %d k %u err %u\n", seq, M, k, err);
  const int64_t m64 = M;
  resp4[2] = (uint32_t)(uint64_t)m64;
  resp4[3] = (uint32_t)((uint64_t)m64 >> 32);
  return KSG_OK;
}

// the t-th set bit (ascending) of the tie words -> node offset, -1 if none
int64_t srv_pick(const std::vector<uint64_t>& tw, uint64_t t) {
  uint64_t acc = 0;
  for (size_t i = 0; i < tw.size(); ++i) {
    const uint64_t pc = (uint64_t)__builtin_popcountll(tw[i]);
    if (t < acc + pc) {
      uint64_t w = tw[i];
      for (uint64_t j = acc; j < t; ++j) w &= w - 1;  // drop the lower set bits
      return (int64_t)(i * 64 + (uint64_t)__builtin_ctzll(w));
    }
    acc += pc;
  }
  return -1;
}

// Ends the resident server so other work can use the stream.
int srv_stop(ksg_ctx* c) {
  if (!c->srv_running) return KSG_OK;
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = srv_settle(c)) return rc;  // (the last commit is applied first)
  if (hipStreamQuery(c->st) != hipSuccess) {
    uint32_t hdr[KSG_SRV_HDR_DW] = {KSG_SRV_EXIT};
    uint32_t r[4];
    if (int rc = srv_call(c, hdr, r)) return rc;
  }
  c->srv_running = false;
  // (a pending begin served by the server stays pending: its commit picks the node from
  // srv_tw on the host and posts the COMMIT to a relaunched server)
  HIPCHK(c, hipStreamSynchronize(c->st));
  return KSG_OK;
}

int srv_flush_patches(ksg_ctx* c) {
  if (int rc = srv_alloc(c)) return rc;
  size_t at = 0;
  while (at < c->patches.size()) {
    const uint32_t n = (uint32_t)std::min<size_t>(c->patches.size() - at, KSG_SRV_PATCHES);
    memcpy(c->srv_box->patch, c->patches.data() + at, (size_t)n * sizeof(KsgPatch));
    uint32_t hdr[KSG_SRV_HDR_DW] = {KSG_SRV_PATCH};
    hdr[KSG_SRVH_NPATCH] = n;
    uint32_t r[4];
    if (int rc = srv_call(c, hdr, r)) return rc;
    at += n;
  }
  c->patches.clear();
  return KSG_OK;
}

// The pod, its ids [0, n_ids) and (extensions) its record as the request
// payload; false if it does not fit the block + ext area.
bool srv_put_pod(ksg_ctx* c, const ksg_pod* pod, const uint32_t* ids, size_t n_ids, const ksg_pod_ext* ext,
                 uint32_t* hdr, bool ctl = false) {
  const uint32_t pod_dw = (uint32_t)(sizeof(ksg_pod) / 4), ext_dw = (uint32_t)(sizeof(ksg_pod_ext) / 4);
  const uint32_t ids_at = pod_dw;
  const uint32_t ext_at = (ids_at + (uint32_t)n_ids + 1) & ~1u;  // 8-byte aligned
  const uint64_t paydw = ext ? (uint64_t)ext_at + ext_dw : (uint64_t)ids_at + n_ids;
  if (paydw > KSG_SRV_PAY_DW) return false;
  uint32_t* req = ctl ? c->srv_box->creq : c->srv_box->req;
  uint32_t* xa = ctl ? c->srv_box->cext : c->srv_box->ext;
  auto put = [&](uint32_t i, uint32_t v) {  // payload dword i
    if (i < KSG_SRV_INLINE_DW) {
      const uint32_t j = KSG_SRV_HDR_DW + i;
      req[4 * (j / KSG_SRV_CHUNK_DW) + j % KSG_SRV_CHUNK_DW] = v;
    } else {
      xa[i - KSG_SRV_INLINE_DW] = v;
    }
  };
  const uint32_t* pw = reinterpret_cast<const uint32_t*>(pod);
  for (uint32_t i = 0; i < pod_dw; ++i) put(i, pw[i]);
  for (uint32_t i = 0; i < n_ids; ++i) put(ids_at + i, ids[i]);
  if (ext) {
    const uint32_t* ew = reinterpret_cast<const uint32_t*>(ext);
    for (uint32_t i = 0; i < ext_dw; ++i) put(ext_at + i, ew[i]);
  }
  hdr[KSG_SRVH_PAYDW] = (uint32_t)paydw;
  hdr[KSG_SRVH_IDS_AT] = ids_at;
  hdr[KSG_SRVH_EXT_AT] = ext_at;
  if (ext) hdr[KSG_SRVH_FLAGS] |= KSG_SRVF_EXT;
  return true;
}

}  // namespace

extern "C" {

int ksg_shard_range(uint32_t n_nodes, int rank, int world, uint32_t* lo, uint32_t* hi) {
  if (world < 1 || rank < 0 || rank >= world || !lo || !hi) return KSG_ERR_ARG;
  uint32_t a, b;
  ksg_shard_words((n_nodes + 63) / 64, (uint32_t)rank, (uint32_t)world, &a, &b);
  *lo = std::min(a * 64, n_nodes);
  *hi = std::min(b * 64, n_nodes);
  return KSG_OK;
}

int ksg_merge_records(const void* records, uint32_t rec_bytes, uint32_t world, uint32_t n_nodes,
                      int empty_priorities, uint64_t* rng_state, uint64_t tie_index, int32_t* out_node,
                      int64_t* max_score, uint64_t* tie_count) {
  if (!records || world < 1 || rec_bytes < sizeof(KsgRecordHdr) || !out_node) return KSG_ERR_ARG;
  const uint8_t* rec = static_cast<const uint8_t*>(records);
  const KsgMerged m = ksg_merge_summary(rec, rec_bytes, world, empty_priorities);
  if (max_score) *max_score = m.max_score;
  if (tie_count) *tie_count = m.tie_count;
  *out_node = -1;
  if (m.error) return KSG_ERR_NOPEER;
  if (m.tie_count == 0) return KSG_NOFIT;
  const uint64_t ix = rng_state ? (ksg_splitmix_next(rng_state) >> 1) % m.tie_count : tie_index % m.tie_count;
  uint64_t lix = 0, kg = 0;
  const int32_t g = ksg_merge_owner(rec, rec_bytes, world, m.max_score, ix, &lix, &kg);
  if (g < 0) return KSG_ERR_ARG;
  uint32_t a, b;
  ksg_shard_words((n_nodes + 63) / 64, (uint32_t)g, world, &a, &b);
  const uint32_t nwords = (rec_bytes - (uint32_t)sizeof(KsgRecordHdr)) / 8;
  const uint64_t* words = reinterpret_cast<const uint64_t*>(rec + (size_t)g * rec_bytes + sizeof(KsgRecordHdr));
  // the lix-th tie from the top = the (kg-1-lix)-th set bit from the bottom
  uint64_t target = kg - 1 - lix;
  for (uint32_t w = 0; w < std::min(nwords, b - a); ++w) {
    uint64_t x = words[w];
    const uint32_t cnt = (uint32_t)__builtin_popcountll(x);
    if (target >= cnt) {
      target -= cnt;
      continue;
    }
    for (; target; --target) x &= x - 1;
    *out_node = (int32_t)((a + w) * 64 + (uint32_t)__builtin_ctzll(x));
    return *out_node < (int32_t)n_nodes ? KSG_OK : KSG_ERR_ARG;
  }
  return KSG_ERR_ARG;  // record's count and bitmap disagree
}

int ksg_nccl_unique_id(void* out128) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return KSG_ERR_RCCL;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  memcpy(out128, &id, sizeof id);
  return KSG_OK;
}

static int create_impl(const ksg_config* cfg, int device, int rank, int world, const void* nccl_id,
                       ksg_ctx** out) {
  if (!cfg || !out || world < 1 || rank < 0 || rank >= world) return KSG_ERR_ARG;
  if (cfg->n_anti > KSG_MAX_ANTI || cfg->n_label_pref > KSG_MAX_LABEL_PREF ||
      cfg->n_presence > KSG_MAX_PRESENCE || cfg->n_aff_labels > KSG_MAX_AFF ||
      cfg->n_aff_groups > KSG_MAX_AFF_GROUPS)
    return KSG_ERR_ARG;
  for (uint32_t g = 0; g < cfg->n_aff_groups; ++g)
    if (cfg->aff_group_mask[g] >> cfg->n_aff_labels) return KSG_ERR_ARG;  // a label the config lacks
  for (uint32_t q = 0; q < cfg->n_presence; ++q)
    if (cfg->presence_n_keys[q] > KSG_MAX_PRESENCE_KEYS) return KSG_ERR_ARG;
  ksg_ctx* c = new ksg_ctx();
  c->cfg = *cfg;
  if (c->cfg.max_conflict_keys == 0) c->cfg.max_conflict_keys = 1024;
  if (c->cfg.max_domains == 0) c->cfg.max_domains = 4096;
  c->device = device;
  c->rank = rank;
  c->world = world;
  auto bail = [&](int rc) {
    if (rc != KSG_OK) {
      fprintf(stderr, "ksg_create: %s\n", c->err.c_str());
      delete c;
    }
    return rc;
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return bail(fail(c, KSG_ERR_HIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e)));
  if ((e = hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&c->ev0, kTimingEvent)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&c->ev1, kTimingEvent)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&c->ev_wait, hipEventDisableTiming)) != hipSuccess)
    return bail(fail(c, KSG_ERR_HIP, "stream/event: %s", hipGetErrorString(e)));
  c->spin_wait = !(getenv("KSG_SPIN_WAIT") && atoi(getenv("KSG_SPIN_WAIT")) == 0);
  c->srv_enabled = !(getenv("KSG_SERVE") && atoi(getenv("KSG_SERVE")) == 0);
  c->srv_stamps = getenv("KSG_SERVE_STAMPS") && atoi(getenv("KSG_SERVE_STAMPS")) != 0;
  c->srv_debug = getenv("KSG_SERVE_DEBUG") && atoi(getenv("KSG_SERVE_DEBUG")) != 0;
  c->srv_trace = getenv("KSG_SERVE_TRACE") && atoi(getenv("KSG_SERVE_TRACE")) != 0;
  if (const char* go = getenv("KSG_SERVE_GRID_OPTS")) c->srv_grid_opts = (int64_t)strtoul(go, nullptr, 0);
  if (const char* iu = getenv("KSG_SERVE_IDLE_US")) c->srv_idle_us = (uint64_t)std::max(atoll(iu), 1LL);
  c->srv_grid_on = !(getenv("KSG_SERVE_GRID") && atoi(getenv("KSG_SERVE_GRID")) == 0);
  if (const char* gm = getenv("KSG_SERVE_GRID_MIN")) c->srv_grid_min = (uint32_t)std::max(atoi(gm), 0);
  if (const char* g4 = getenv("KSG_SERVE_GRID_NPT4_MIN")) c->srv_npt4_min = (uint32_t)std::max(atoi(g4), 0);
  c->srv_grid_ext = !(getenv("KSG_SERVE_GRID_EXT") && atoi(getenv("KSG_SERVE_GRID_EXT")) == 0);
  if (const char* rm = getenv("KSG_ROUND_MARGIN")) c->round_margin = std::min(std::max(atof(rm), 0.5), 4.0);
  // The exchange path (shard scan, all-gather of per-shard records, replicated
  // resolve) runs for world > 1, and for a 1-rank RCCL communicator when the caller
  // passes an nccl_id with world == 1 (RCCL itself exercised on a single GPU).
  c->xchg = world > 1 || nccl_id != nullptr;
  if (c->xchg) {
    if (world > KSG_MAX_WORLD) return bail(fail(c, KSG_ERR_ARG, "world %d > %d", world, KSG_MAX_WORLD));
    if (nccl_id) {  // else: the caller installs a host transport with ksg_set_allgather
      ncclUniqueId id;
      memcpy(&id, nccl_id, sizeof id);
      ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
      if (r != ncclSuccess) return bail(fail(c, KSG_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r)));
    }
  }
  int rc;
  if (const char* wenv = getenv("KSG_WINDOW")) c->window = (uint32_t)atoi(wenv);
  if (const char* kev = getenv("KSG_KERNEL_EVENTS")) c->ev_stride = (uint32_t)std::max(atoi(kev), 0);
  if ((rc = dalloc(c, &c->d_rng, 1, nullptr)) || (rc = dalloc(c, &c->d_summary, 4, nullptr)) ||
      (rc = dalloc(c, &c->d_run, 1, nullptr)))
    return bail(rc);
  if ((e = hipHostMalloc((void**)&c->h_run, sizeof(KsgWinRun), hipHostMallocDefault)) != hipSuccess)
    return bail(fail(c, KSG_ERR_HIP, "hipHostMalloc: %s", hipGetErrorString(e)));
  c->win_fused = !(getenv("KSG_FUSED") && atoi(getenv("KSG_FUSED")) == 0);
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 16) cus = 0;
    c->fused_grid = (uint32_t)cus;
    if (const char* fg = getenv("KSG_FUSED_GRID")) c->fused_grid = (uint32_t)std::min(std::max(atoi(fg), 9), 4096);
    if (c->fused_grid == 0) c->win_fused = false;
    if (const char* fw = getenv("KSG_FUSED_MAX_WORDS")) c->fused_max_words = (uint32_t)std::max(atoi(fw), 0);
  }
  if ((e = hipMalloc((void**)&c->d_fctl, kFctlBytes)) != hipSuccess ||
      (e = hipHostMalloc((void**)&c->h_fctl, kFctlBytes, hipHostMallocDefault)) != hipSuccess)
    return bail(fail(c, KSG_ERR_HIP, "fused window control: %s", hipGetErrorString(e)));
  memset(c->h_fctl, 0, kFctlBytes);
  *out = c;
  return KSG_OK;
}

int ksg_create(const ksg_config* cfg, int device, ksg_ctx** out) {
  return create_impl(cfg, device, 0, 1, nullptr, out);
}

int ksg_create_sharded(const ksg_config* cfg, int device, int rank, int world, const void* nccl_id,
                       ksg_ctx** out) {
  return create_impl(cfg, device, rank, world, nccl_id, out);
}

int ksg_destroy(ksg_ctx* c) {
  if (!c) return KSG_OK;
  if (c->dev.dbgbuf) {  // debug stamps (KSG_DEBUG & 8): cycles/64 per resolver section
    int32_t h[32];
    (void)hipMemcpy(h, c->dev.dbgbuf, sizeof h, hipMemcpyDeviceToHost);
    fprintf(stderr, "ksg stamps (x64 cycles, committer wave): ring-wait %d head %d recheck-last-slot %d "
            "wait-checkers %d select %d commit %d | drop-path pods %d unpredicted commits %d\n",
            h[0], h[1], h[2], h[3], h[4], h[5], h[7], h[8]);
    fprintf(stderr, "ksg ring-wait split: first 4 pods of each window %d, later pods %d\n", h[10], h[11]);
    fprintf(stderr, "ksg producers (sum over waves): slot-wait %d loads %d draw-wait %d stage %d\n", h[12], h[13],
            h[14], h[15]);
    fprintf(stderr, "ksg stamps raw:");
    for (int q = 0; q < 32; ++q) fprintf(stderr, " %d", h[q]);
    fprintf(stderr, "\n");
  }
  {
    KSG_LOCK(c);  // waits for a call in flight on another thread
    (void)hipSetDevice(c->device);
    (void)srv_stop(c);
  }
  if (c->srv_stamped && srv_grid(c)) {
    const double n = (double)c->srv_stamped;
    fprintf(stderr, "ksg grid serve stamps (10-ns ticks per begin, %llu begins, scan workgroup 0): request seen -> "
            "masks + loads done %.1f, -> eval + part stored %.1f\n",
            (unsigned long long)c->srv_stamped, c->srv_stage[0] / n, c->srv_stage[1] / n);
  } else if (c->srv_stamped) {
    const double n = (double)c->srv_stamped;
    fprintf(stderr, "ksg serve stamps (s_memtime cycles per begin, %llu begins): to-LDS %.0f check %.0f resolve %.0f "
            "scan %.0f reduce %.0f fail-codes %.0f\n", (unsigned long long)c->srv_stamped, c->srv_stage[0] / n,
            c->srv_stage[1] / n, c->srv_stage[2] / n, c->srv_stage[3] / n, c->srv_stage[4] / n, c->srv_stage[5] / n);
  }
  (void)hipSetDevice(c->device);
  if (c->st) (void)hipStreamSynchronize(c->st);
  free_cluster(c);
  void* scratch[] = {c->d_pods, c->d_ids, c->d_fail, c->d_score, c->d_rec_send, c->d_rec_recv, c->d_dpart,
                     c->d_dglobal, c->d_out, c->d_rng, c->d_summary, c->d_patch, c->d_shard_wlo,
                     c->d_winsum, c->d_xsend, c->d_xrecv, c->d_run, c->d_dcnt, c->d_admit, c->d_one,
                     c->d_t0img, c->d_draws, c->d_etmax, c->d_epsoft, c->d_ethist};
  for (void* p : scratch)
    if (p) (void)hipFree(p);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->h_xsend) (void)hipHostFree(c->h_xsend);
  if (c->h_run) (void)hipHostFree(c->h_run);
  if (c->h_fctl) (void)hipHostFree(c->h_fctl);
  if (c->d_fctl) (void)hipFree(c->d_fctl);
  if (c->h_up) (void)hipHostFree(c->h_up);
  if (c->h_dn) (void)hipHostFree(c->h_dn);
  if (c->h_map) (void)hipHostFree(c->h_map);
  if (c->srv_box) (void)hipHostFree(c->srv_box);
  if (c->srv_grid) (void)hipFree(c->srv_grid);
  if (c->srv_fail) (void)hipHostFree(c->srv_fail);
  if (c->h_xrecv) (void)hipHostFree(c->h_xrecv);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev_wait) (void)hipEventDestroy(c->ev_wait);
  for (auto& e : c->wev)
    if (e) (void)hipEventDestroy(e);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
  return KSG_OK;
}

const char* ksg_last_error(ksg_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ksg_set_cluster(ksg_ctx* c, const ksg_node* nodes, uint32_t n_nodes, const uint32_t* node_pairs,
                    uint32_t n_node_pairs, const uint32_t* pair_keys, uint32_t n_pairs, uint32_t n_services) {
  if (!c) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->st));
  if (n_nodes && !nodes) return fail(c, KSG_ERR_ARG, "nodes == NULL");
  if (n_pairs == 0) n_pairs = 1;  // pair 0 always exists (empty)
  for (uint32_t i = 0; i < n_nodes; ++i) {
    if ((size_t)nodes[i].label_off + nodes[i].n_labels > n_node_pairs)
      return fail(c, KSG_ERR_ARG, "node %u label range out of bounds", i);
    for (uint32_t k = 0; k < nodes[i].n_labels; ++k)
      if (node_pairs[nodes[i].label_off + k] >= n_pairs || node_pairs[nodes[i].label_off + k] == 0)
        return fail(c, KSG_ERR_ARG, "node %u has invalid pair id", i);
  }
  free_cluster(c);
  drop_deferred(c);
  c->diverged = false;
  c->ppw_est = 0.0;
  c->N = n_nodes;
  c->nw = (n_nodes + 63) / 64;
  c->n_pairs = n_pairs;
  c->S = n_services;
  // shard by 64-node words
  c->shard_wlo_h.resize(c->world);
  c->nwords_max = 0;
  uint32_t max_shard_nodes = 0;
  for (int g = 0; g < c->world; ++g) {
    uint32_t a, b;
    ksg_shard_words(c->nw, (uint32_t)g, (uint32_t)c->world, &a, &b);
    c->shard_wlo_h[g] = a;
    c->nwords_max = std::max(c->nwords_max, b - a);
    max_shard_nodes = std::max(max_shard_nodes, std::min(b * 64, n_nodes) - std::min(a * 64, n_nodes));
    if (g == c->rank) {
      c->wlo = a;
      c->nwords = b - a;
      c->lo = std::min(a * 64, n_nodes);
      c->hi = std::min(b * 64, n_nodes);
    }
  }
  if (max_shard_nodes > kMaxNodesPerShard)
    return fail(c, KSG_ERR_CAPACITY, "shard of %u nodes exceeds %u (use more GPUs)", max_shard_nodes,
                kMaxNodesPerShard);
  c->R = pick_R(std::max<uint32_t>(max_shard_nodes, 1));

  // anti-affinity domains: dense index of each pair whose key is the label
  std::vector<int32_t> dom_of_pair((size_t)std::max<uint32_t>(c->cfg.n_anti, 1) * n_pairs, -1);
  c->D = 0;
  KsgDev& d = c->dev;
  d = KsgDev{};
  for (uint32_t a = 0; a < c->cfg.n_anti; ++a) {
    d.anti_dom_off[a] = c->D;
    uint32_t nd = 0;
    for (uint32_t p = 1; p < n_pairs; ++p)
      if ((pair_keys[p] & ~KSG_PAIR_INVALID) == c->cfg.anti_key[a]) dom_of_pair[(size_t)a * n_pairs + p] = (int32_t)nd++;
    c->D += nd;
  }
  if (c->D > c->cfg.max_domains)
    return fail(c, KSG_ERR_CAPACITY, "%u anti-affinity domains > max_domains %u", c->D, c->cfg.max_domains);
  c->lds = (size_t)c->D * sizeof(int32_t);

  auto* owner = &c->cluster_allocs;
  int rc;
  int64_t *cap_c, *cap_m;
  double *inv_c, *inv_m;
  uint64_t *sfit, *keymap, *pairmap;
  int64_t* sscore;
  int32_t *anti_dom, *aff_pair;
  int64_t* gscore = nullptr;  // (int32 or int64 scores: sized for int64)
  const size_t NN = std::max<uint32_t>(n_nodes, 1);
  if ((rc = dalloc(c, &cap_c, NN, owner)) || (rc = dalloc(c, &cap_m, NN, owner)) ||
      (rc = dalloc(c, &inv_c, NN, owner)) || (rc = dalloc(c, &inv_m, NN, owner)) ||
      (rc = dalloc(c, &d.used_cpu, NN, owner)) || (rc = dalloc(c, &d.used_mem, NN, owner)) ||
      (rc = dalloc(c, &sfit, std::max<uint32_t>(c->nw, 1), owner)) ||
      (rc = dalloc(c, &sscore, NN, owner)) ||
      (rc = dalloc(c, &keymap, (size_t)c->cfg.max_conflict_keys * std::max<uint32_t>(c->nw, 1), owner)) ||
      (rc = dalloc(c, &pairmap, (size_t)n_pairs * std::max<uint32_t>(c->nw, 1), owner)) ||
      (rc = dalloc(c, &d.svc_cnt, (size_t)std::max<uint32_t>(n_services, 1) * NN, owner)) ||
      (rc = dalloc(c, &d.svc_bits, (size_t)std::max<uint32_t>(n_services, 1) * std::max<uint32_t>(c->nw, 1), owner)) ||
      (rc = dalloc(c, &d.svc_max, std::max<uint32_t>(n_services, 1), owner)) ||
      (rc = dalloc(c, &d.svc_total, std::max<uint32_t>(n_services, 1), owner)) ||
      (rc = dalloc(c, &d.svc_peer, std::max<uint32_t>(n_services, 1), owner)) ||
      (rc = dalloc(c, &anti_dom, (size_t)std::max<uint32_t>(c->cfg.n_anti, 1) * NN, owner)) ||
      (rc = dalloc(c, &aff_pair, (size_t)std::max<uint32_t>(c->cfg.n_aff_labels, 1) * NN, owner)) ||
      (c->R > KSG_R_LDS / 2 && (rc = dalloc(c, &gscore, (size_t)c->R * KSG_NT, owner))))
    return rc;
  if (n_services) HIPCHK(c, hipMemsetAsync(d.svc_peer, 0xff, n_services * sizeof(int32_t), c->st));

  // upload nodes + static tables
  std::vector<int64_t> hc(NN, 0), hm(NN, 0);
  c->max_cap = 0;
  c->min_cap = 0;
  for (uint32_t i = 0; i < n_nodes; ++i) {
    hc[i] = nodes[i].cap_milli_cpu;
    hm[i] = nodes[i].cap_memory;
    c->max_cap = std::max<int64_t>(c->max_cap, std::max<int64_t>(std::llabs(hc[i]), std::llabs(hm[i])));
    c->min_cap = std::min<int64_t>(c->min_cap, std::min<int64_t>(hc[i], hm[i]));
  }
  HIPCHK(c, hipMemcpyAsync(cap_c, hc.data(), NN * 8, hipMemcpyHostToDevice, c->st));
  HIPCHK(c, hipMemcpyAsync(cap_m, hm.data(), NN * 8, hipMemcpyHostToDevice, c->st));
  // correctly rounded on host and device alike (lr_inv10, ksg_device.h)
  std::vector<double> ic(NN, 0.0), im(NN, 0.0);
  for (uint32_t i = 0; i < n_nodes; ++i) {
    ic[i] = hc[i] > 0 ? 10.0 / (double)hc[i] : 0.0;
    im[i] = hm[i] > 0 ? 10.0 / (double)hm[i] : 0.0;
  }
  HIPCHK(c, hipMemcpyAsync(inv_c, ic.data(), NN * 8, hipMemcpyHostToDevice, c->st));
  HIPCHK(c, hipMemcpyAsync(inv_m, im.data(), NN * 8, hipMemcpyHostToDevice, c->st));
  ksg_node* dn = nullptr;
  uint32_t *dnp = nullptr, *dpk = nullptr;
  int32_t* ddom = nullptr;
  std::vector<void*> tmp;
  // (the node labels stay with the cluster: ksg_add_static_config reads them)
  if ((rc = dalloc(c, &dn, NN, owner)) || (rc = dalloc(c, &dnp, std::max<uint32_t>(n_node_pairs, 1), owner)) ||
      (rc = dalloc(c, &dpk, n_pairs, owner)) || (rc = dalloc(c, &ddom, dom_of_pair.size(), &tmp)))
    return rc;
  c->d_lbl_nodes = dn;
  c->d_lbl_pairs = dnp;
  c->d_lbl_keys = dpk;
  if (n_nodes) HIPCHK(c, hipMemcpyAsync(dn, nodes, n_nodes * sizeof(ksg_node), hipMemcpyHostToDevice, c->st));
  if (n_node_pairs)
    HIPCHK(c, hipMemcpyAsync(dnp, node_pairs, n_node_pairs * 4, hipMemcpyHostToDevice, c->st));
  std::vector<uint32_t> pk(n_pairs, 0xffffffffu);
  if (pair_keys)
    for (uint32_t p = 1; p < n_pairs; ++p) pk[p] = pair_keys[p];
  HIPCHK(c, hipMemcpyAsync(dpk, pk.data(), n_pairs * 4, hipMemcpyHostToDevice, c->st));
  HIPCHK(c, hipMemcpyAsync(ddom, dom_of_pair.data(), dom_of_pair.size() * 4, hipMemcpyHostToDevice, c->st));
  KsgStaticCfg sc{};
  sc.n_presence = c->cfg.n_presence;
  memcpy(sc.presence_n_keys, c->cfg.presence_n_keys, sizeof sc.presence_n_keys);
  memcpy(sc.presence_keys, c->cfg.presence_keys, sizeof sc.presence_keys);
  memcpy(sc.presence_flag, c->cfg.presence_flag, sizeof sc.presence_flag);
  sc.n_pref = c->cfg.n_label_pref;
  memcpy(sc.pref_key, c->cfg.pref_key, sizeof sc.pref_key);
  memcpy(sc.pref_presence, c->cfg.pref_presence, sizeof sc.pref_presence);
  memcpy(sc.w_pref, c->cfg.w_pref, sizeof sc.w_pref);
  sc.w_equal = c->cfg.w_equal;
  sc.n_anti = c->cfg.n_anti;
  memcpy(sc.anti_key, c->cfg.anti_key, sizeof sc.anti_key);
  sc.n_aff = c->cfg.n_aff_labels;
  memcpy(sc.aff_key, c->cfg.aff_key, sizeof sc.aff_key);
  HIPCHK(c, ksg_launch_static(sc, n_nodes, dn, dnp, dpk, ddom, n_pairs, c->nw, sfit, sscore, anti_dom, aff_pair,
                              (unsigned long long*)pairmap, c->st));
  // (ServiceAffinity: a host copy of each node's pair per affinity label, so the drop-in server's
  // BEGIN carries a pod's requirements already resolved from its service's first peer)
  c->h_aff_pair.clear();
  if ((c->cfg.predicates & KSG_PRED_SERVICEAFFINITY) && c->cfg.n_aff_labels > 0 && c->world == 1) {
    c->h_aff_pair.resize((size_t)c->cfg.n_aff_labels * NN);
    HIPCHK(c, hipMemcpyAsync(c->h_aff_pair.data(), aff_pair, c->h_aff_pair.size() * sizeof(int32_t),
                             hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
  }
  // ServiceAntiAffinity re-rank (one anti priority, one rank, few domains, an
  // LDS count per service): the nodes of each domain row, row D = unlabelled
  c->d_zmap = nullptr;
  uint32_t rr_dz = 0;
  if (c->cfg.n_anti == 1 && c->cfg.w_anti[0] != 0 && c->D > 0 && c->D + 1 <= KSG_RR_MAXZ && c->world == 1 &&
      n_services <= KSG_RR_MAXSVC && !(getenv("KSG_DEBUG") && (atoi(getenv("KSG_DEBUG")) & 2048))) {
    rr_dz = c->D + 1;
    if ((rc = dalloc(c, &c->d_zmap, (size_t)rr_dz * std::max<uint32_t>(c->nw, 1), owner))) return rc;
    HIPCHK(c, ksg_launch_zonemap(n_nodes, anti_dom, c->D, c->nw, c->d_zmap, c->st));
  }
  HIPCHK(c, hipStreamSynchronize(c->st));
  for (void* p : tmp) (void)hipFree(p);

  d.n_nodes = n_nodes;
  d.nw = c->nw;
  d.lo = c->lo;
  d.hi = c->hi;
  d.wlo = c->wlo;
  d.nwords = c->nwords;
  d.n_pairs = n_pairs;
  d.n_services = n_services;
  d.max_keys = c->cfg.max_conflict_keys;
  d.n_domains_total = c->D;
  d.rr_dz = rr_dz;
  d.preds = c->cfg.predicates;
  d.n_aff = (c->cfg.predicates & KSG_PRED_SERVICEAFFINITY) ? c->cfg.n_aff_labels : 0;
  // ServiceAffinity predicates (label groups); none given: one over every label
  d.n_aff_groups = c->cfg.n_aff_groups;
  for (uint32_t g = 0; g < d.n_aff_groups; ++g) d.aff_group_mask[g] = c->cfg.aff_group_mask[g];
  if (d.n_aff_groups == 0 && d.n_aff > 0) {
    d.n_aff_groups = 1;
    d.aff_group_mask[0] = (1u << d.n_aff) - 1u;
  }
  // (extension priorities count as priority configs)
  const bool ext_prio = c->ext_on && (c->ext.w_taint_toleration || c->ext.w_balanced);
  d.equal_fallback = c->cfg.n_priority_configs == 0 && !ext_prio;
  // prioritizeNodes skips weight-0 configs; if every config has weight 0 the
  // HostPriorityList is empty and Schedule returns *FitError.
  bool any_weight = c->cfg.w_least_requested || c->cfg.w_service_spreading || c->cfg.w_equal || ext_prio;
  for (uint32_t a = 0; a < c->cfg.n_anti; ++a) any_weight |= c->cfg.w_anti[a] != 0;
  for (uint32_t q = 0; q < c->cfg.n_label_pref; ++q) any_weight |= c->cfg.w_pref[q] != 0;
  d.empty_priorities = (!d.equal_fallback && !any_weight) ? 1 : 0;
  // int64 combined scores (exact kernels) once a |score| could reach KSG_SCORE_BOUND
  d.wide = score_bound(c->cfg, c->ext.w_taint_toleration, c->ext.w_balanced) >= (unsigned __int128)KSG_SCORE_BOUND;
  c->static_mag = 0;  // (ksg_set_static_terms' terms end with the node list they were built for)
  d.w_lr = c->cfg.w_least_requested;
  d.w_spread = c->cfg.w_service_spreading;
  d.n_anti = 0;
  for (uint32_t a = 0; a < c->cfg.n_anti; ++a) {
    d.w_anti[a] = c->cfg.w_anti[a];
    if (c->cfg.w_anti[a]) d.n_anti = a + 1;
  }
  if (d.n_anti == 0) d.n_domains_total = 0;
  bool any_pref = false;
  for (uint32_t q = 0; q < c->cfg.n_label_pref; ++q) any_pref |= c->cfg.w_pref[q] != 0;
  d.has_static_score = (c->cfg.w_equal != 0 || any_pref) ? 1 : 0;
  d.dbg = getenv("KSG_DEBUG") ? atoi(getenv("KSG_DEBUG")) : 0;
  // KSG_DEBUG bit 22 / 23: the next COMMIT / BEGIN posted to the resident server carries an
  // out-of-range payload layout (tests/test_gpu_serve.py: the server must reject it, not fault)
  c->dbg_corrupt = ((uint32_t)d.dbg >> 22) & 3u;
  c->win_d1 = !(getenv("KSG_WIN_D1") && atoi(getenv("KSG_WIN_D1")) == 0);
  if (d.dbg & (8 | 32 | 64)) {  // (32: the plain resolver's inconsistency record, ksg_plain.hip; 64: phase-A stamps)
    (void)hipMalloc(&d.dbgbuf, KSG_DEBUG_COUNTER_WORDS * sizeof(int32_t));
    (void)hipMemset(d.dbgbuf, 0, KSG_DEBUG_COUNTER_WORDS * sizeof(int32_t));
  }
  d.has_static_fit = ((c->cfg.predicates & KSG_PRED_LABELSPRESENCE) && c->cfg.n_presence > 0) ? 1 : 0;
  d.cap_cpu = cap_c;
  d.cap_mem = cap_m;
  d.inv10_cpu = inv_c;
  d.inv10_mem = inv_m;
  d.static_fit = sfit;
  d.static_score = sscore;
  d.keymap = keymap;
  d.pairmap = pairmap;
  d.anti_domain = anti_dom;
  d.aff_pair = aff_pair;
  d.score_scratch = gscore;
  if (c->ext_on) {  // extensions: extended resources (allocatable, requested) and taint bitmaps
    int64_t *scap = nullptr, *sused = nullptr;
    uint64_t* tmap = nullptr;
    const size_t nsr = std::max<uint32_t>(c->ext.n_scalar, 1);
    if ((rc = dalloc(c, &scap, nsr * NN, owner)) || (rc = dalloc(c, &sused, nsr * NN, owner)) ||
        (rc = dalloc(c, &tmap, (size_t)std::max<uint32_t>(c->ext.max_taints, 1) * std::max<uint32_t>(c->nw, 1), owner)))
      return rc;
    d.ext_filters = c->ext.filters;
    d.w_taint = c->ext.w_taint_toleration;
    d.w_bal = c->ext.w_balanced;
    d.n_scalar = c->ext.n_scalar;
    d.scalar_cap = scap;
    d.scalar_used = sused;
    d.taintmap = tmap;
    d.ntaint = nullptr;
    if (c->ext.max_taints <= 64) {  // (the window path's TaintToleration term: one mask per node)
      uint64_t* ntm = nullptr;
      if ((rc = dalloc(c, &ntm, NN, owner))) return rc;
      d.ntaint = ntm;
    }
  }
  c->lds = (size_t)d.n_domains_total * sizeof(int32_t);

  // scratch sized for the shard
  c->rec_bytes = (uint32_t)(sizeof(KsgRecordHdr) + (size_t)std::max<uint32_t>(c->nwords_max, 1) * 8);
  if (c->d_rec_send) (void)hipFree(c->d_rec_send);
  if (c->d_rec_recv) (void)hipFree(c->d_rec_recv);
  if (c->d_fail) (void)hipFree(c->d_fail);
  if (c->d_score) (void)hipFree(c->d_score);
  if (c->d_dpart) (void)hipFree(c->d_dpart);
  if (c->d_dglobal) (void)hipFree(c->d_dglobal);
  if (c->d_shard_wlo) (void)hipFree(c->d_shard_wlo);
  c->d_rec_send = c->d_rec_recv = c->d_fail = nullptr;
  c->d_score = nullptr;
  c->d_dpart = c->d_dglobal = nullptr;
  c->d_shard_wlo = nullptr;
  if ((rc = dalloc(c, &c->d_rec_send, c->rec_bytes, nullptr)) ||
      (rc = dalloc(c, &c->d_rec_recv, (size_t)c->rec_bytes * c->world, nullptr)) ||
      (rc = dalloc(c, &c->d_fail, NN, nullptr)) || (rc = dalloc(c, &c->d_score, NN, nullptr)) ||
      (rc = dalloc(c, &c->d_dpart, (size_t)c->dev.n_domains_total + 1, nullptr)) ||  // (+ the TaintToleration max)
      (rc = dalloc(c, &c->d_dglobal, (size_t)c->dev.n_domains_total + 1, nullptr)) ||
      (rc = dalloc(c, &c->d_shard_wlo, c->world, nullptr)))
    return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_shard_wlo, c->shard_wlo_h.data(), c->world * 4, hipMemcpyHostToDevice, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  reset_mirror(c);
  c->have_cluster = true;
  return KSG_OK;
}

int ksg_set_static_terms(ksg_ctx* c, const uint64_t* fit_words, const int64_t* score, int score_weighted) {
  if (!c || (!fit_words && !score)) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (int rs = cluster_ok(c)) return rs;
  if (c->pending) return fail(c, KSG_ERR_STATE, "schedule_begin pending");
  // (a node failing the extra fit words reports KSG_FAIL_LABELSPRESENCE: the config must name it)
  if (fit_words && !(c->cfg.predicates & KSG_PRED_LABELSPRESENCE))
    return fail(c, KSG_ERR_ARG, "ksg_set_static_terms: fit words need KSG_PRED_LABELSPRESENCE in the config");
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  HIPCHK(c, hipSetDevice(c->device));
  const uint32_t N = c->N, nw = (N + 63) / 64;
  if (N == 0) return KSG_OK;
  // a combined score stays int32 on the fast paths only while every |score| < 2^30
  unsigned __int128 mag = 0;
  if (score)
    for (uint32_t n = 0; n < N; ++n) {
      const unsigned __int128 m = score[n] < 0 ? (unsigned __int128)(0 - (uint64_t)score[n]) : (unsigned __int128)score[n];
      mag = std::max(mag, m);
    }
  uint8_t* tmp = nullptr;
  const size_t fb = fit_words ? (size_t)nw * 8 : 0, sb = score ? (size_t)N * 8 : 0;
  HIPCHK(c, hipMalloc((void**)&tmp, fb + sb));
  if (fit_words) HIPCHK(c, hipMemcpyAsync(tmp, fit_words, fb, hipMemcpyHostToDevice, c->st));
  if (score) HIPCHK(c, hipMemcpyAsync(tmp + fb, score, sb, hipMemcpyHostToDevice, c->st));
  KsgDev& d = c->dev;
  HIPCHK(c, ksg_launch_static_fold(const_cast<uint64_t*>(d.static_fit), const_cast<int64_t*>(d.static_score),
                                   fit_words ? reinterpret_cast<const uint64_t*>(tmp) : nullptr,
                                   score ? reinterpret_cast<const int64_t*>(tmp + fb) : nullptr, nw, N,
                                   d.has_static_fit, d.has_static_score, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  (void)hipFree(tmp);
  if (fit_words) d.has_static_fit = 1;
  if (score) {
    d.has_static_score = 1;
    c->static_mag += mag;
    if (score_weighted) d.empty_priorities = 0;
  }
  d.wide = score_bound(c->cfg, c->ext.w_taint_toleration, c->ext.w_balanced) + c->static_mag >=
           (unsigned __int128)KSG_SCORE_BOUND;
  return KSG_OK;
}

int ksg_add_static_config(ksg_ctx* c, const ksg_config* extra) {
  if (!c || !extra) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (int rs = cluster_ok(c)) return rs;
  if (c->pending) return fail(c, KSG_ERR_STATE, "schedule_begin pending");
  if (extra->n_presence > KSG_MAX_PRESENCE || extra->n_label_pref > KSG_MAX_LABEL_PREF)
    return fail(c, KSG_ERR_ARG, "ksg_add_static_config: more terms than the config's slots");
  for (uint32_t q = 0; q < extra->n_presence; ++q)
    if (extra->presence_n_keys[q] > KSG_MAX_PRESENCE_KEYS)
      return fail(c, KSG_ERR_ARG, "ksg_add_static_config: presence predicate %u has too many keys", q);
  // (a node failing the extra predicates reports KSG_FAIL_LABELSPRESENCE: the config must name it)
  if (extra->n_presence && !(c->cfg.predicates & KSG_PRED_LABELSPRESENCE))
    return fail(c, KSG_ERR_ARG, "ksg_add_static_config: LabelsPresence terms need KSG_PRED_LABELSPRESENCE in the config");
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  HIPCHK(c, hipSetDevice(c->device));
  const uint32_t N = c->N, nw = (N + 63) / 64;
  if (N == 0 || (extra->n_presence == 0 && extra->n_label_pref == 0)) return KSG_OK;
  KsgStaticCfg sc{};  // (the terms only: no EqualPriority, anti-affinity domains or affinity pairs)
  sc.n_presence = extra->n_presence;
  memcpy(sc.presence_n_keys, extra->presence_n_keys, sizeof sc.presence_n_keys);
  memcpy(sc.presence_keys, extra->presence_keys, sizeof sc.presence_keys);
  memcpy(sc.presence_flag, extra->presence_flag, sizeof sc.presence_flag);
  sc.n_pref = extra->n_label_pref;
  memcpy(sc.pref_key, extra->pref_key, sizeof sc.pref_key);
  memcpy(sc.pref_presence, extra->pref_presence, sizeof sc.pref_presence);
  memcpy(sc.w_pref, extra->w_pref, sizeof sc.w_pref);
  // |the pass's score| <= 10 x sum |w| (Go-int weights: a wrapped sum is still bounded by it)
  unsigned __int128 mag = 0;
  bool weighted = false;
  for (uint32_t q = 0; q < extra->n_label_pref; ++q) {
    const int64_t w = extra->w_pref[q];
    mag += (unsigned __int128)(w < 0 ? 0 - (uint64_t)w : (uint64_t)w) * 10u;
    weighted |= w != 0;
  }
  const bool do_fit = extra->n_presence > 0, do_score = extra->n_label_pref > 0;
  const size_t fb = (size_t)nw * 8;
  // the scratch pair, freed on every path out (an error return included)
  struct Scratch {
    uint8_t* p = nullptr;
    ~Scratch() {
      if (p) (void)hipFree(p);
    }
  } tmp;
  HIPCHK(c, hipMalloc((void**)&tmp.p, fb + (size_t)N * 8));
  uint64_t* xfit = reinterpret_cast<uint64_t*>(tmp.p);
  int64_t* xscore = reinterpret_cast<int64_t*>(tmp.p + fb);
  KsgDev& d = c->dev;
  HIPCHK(c, ksg_launch_static_terms(sc, N, c->d_lbl_nodes, c->d_lbl_pairs, c->d_lbl_keys, c->n_pairs, nw, xfit, xscore,
                                    c->st));
  HIPCHK(c, ksg_launch_static_fold(const_cast<uint64_t*>(d.static_fit), const_cast<int64_t*>(d.static_score),
                                   do_fit ? xfit : nullptr, do_score ? xscore : nullptr, nw, N, d.has_static_fit,
                                   d.has_static_score, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  if (do_fit) d.has_static_fit = 1;
  if (do_score) {
    d.has_static_score = 1;
    c->static_mag += mag;
    if (weighted) d.empty_priorities = 0;
  }
  d.wide = score_bound(c->cfg, c->ext.w_taint_toleration, c->ext.w_balanced) + c->static_mag >=
           (unsigned __int128)KSG_SCORE_BOUND;
  return KSG_OK;
}

static int add_pod_impl(ksg_ctx* c, uint32_t host_id, const ksg_pod* pod, const uint32_t* ids) {
  if (int rc0 = flush_deferred(c)) return rc0;
  if (int rs = cluster_ok(c)) return rs;
  int rc = check_pod(c, pod, ids, pod_ids_extent(pod));
  if (rc) return rc;
  rc = mirror_add(c, host_id, pod, ids, true);
  if (rc) return rc;
  if (c->patches.size() > 4096) return flush_patches(c);
  return KSG_OK;
}

static int remove_pod_impl(ksg_ctx* c, uint64_t uid) {
  if (c->diverged) return cluster_ok(c);
  if (int rc0 = flush_deferred(c)) return rc0;
  auto it = c->pods.find(uid);
  if (it == c->pods.end()) return fail(c, KSG_ERR_ARG, "unknown pod uid %llu", (unsigned long long)uid);
  PodRec r = std::move(it->second);
  c->pods.erase(it);
  const uint32_t h = r.host;
  if (c->ext_on) c->ext_scalar.erase(uid);
  if (h < c->N) {
    c->used_c[h] = (int64_t)((uint64_t)c->used_c[h] - (uint64_t)r.cpu);
    c->used_m[h] = (int64_t)((uint64_t)c->used_m[h] - (uint64_t)r.mem);
    c->mu_dirty = true;
    patch64(c, c->dev.used_cpu + h, c->used_c[h]);
    patch64(c, c->dev.used_mem + h, c->used_m[h]);
    if (c->ext_on)
      for (uint32_t q = 0; q < c->ext.n_scalar; ++q) {
        if (!r.scalar[q]) continue;
        int64_t& u = c->sc_used[(size_t)q * c->N + h];
        u = (int64_t)((uint64_t)u - (uint64_t)r.scalar[q]);
        patch64(c, c->dev.scalar_used + (size_t)q * c->N + h, u);
      }
    for (uint32_t k : r.keys) {
      auto kit = c->key_ref.find(((uint64_t)k << 32) | h);
      if (kit != c->key_ref.end() && --kit->second == 0) {
        c->key_ref.erase(kit);
        patch_andnot(c, c->dev.keymap + (size_t)k * c->nw + (h >> 6), 1ULL << (h & 63));
      }
    }
  }
  for (uint32_t s : r.svcs) {
    int32_t before;
    if (h < c->N) {
      int32_t& v = c->svc_cnt[(size_t)s * c->N + h];
      before = v--;
      patch32(c, c->dev.svc_cnt + (size_t)s * c->N + h, v);
      if (v == 0) patch_andnot(c, c->dev.svc_bits + (size_t)s * c->nw + (h >> 6), 1ULL << (h & 63));
    } else {
      auto& m = c->svc_ext[s];
      before = m[h]--;
      if (m[h] == 0) m.erase(h);
    }
    if (before == c->svc_max[s]) {
      c->svc_max[s] = recompute_max(c, s);
      patch32(c, c->dev.svc_max + s, c->svc_max[s]);
    }
    --c->svc_total[s];
    patch32(c, c->dev.svc_total + s, c->svc_total[s]);
    c->svc_members[s].erase(r.seq);
    const int32_t pc = peer_code(c, s);
    if (pc != c->svc_peer[s]) {
      c->svc_peer[s] = pc;
      patch32(c, c->dev.svc_peer + s, pc);
    }
  }
  if (c->patches.size() > 4096) return flush_patches(c);
  return KSG_OK;
}

// apply the updates queued while a schedule_begin was pending (c->mu held)
static int apply_queued(ksg_ctx* c) {
  std::vector<ksg_ctx::Queued> q;
  q.swap(c->upd_q);
  c->q_added.clear();
  c->q_removed.clear();
  for (auto& u : q) {
    const int rc = u.add ? add_pod_impl(c, u.host, &u.pod, u.ids.data()) : remove_pod_impl(c, u.uid);
    if (rc) return rc;
  }
  return KSG_OK;
}

int ksg_add_pod(ksg_ctx* c, uint32_t host_id, const ksg_pod* pod, const uint32_t* ids) {
  if (!c || !pod) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (c->ext_on && !c->cur_ext) c->ext_scalar.erase(pod->uid);  // (plain entry point: no extension requests)
  HIPCHK(c, hipSetDevice(c->device));  // reflector threads: patches flush on this context's device
  if (!c->pending) return add_pod_impl(c, host_id, pod, ids);
  if (int rs = cluster_ok(c)) return rs;
  const size_t ext = pod_ids_extent(pod);
  int rc = check_pod(c, pod, ids, ext);
  if (rc) return rc;
  const bool live = c->pods.count(pod->uid) && !c->q_removed.count(pod->uid);
  if (live || c->q_added.count(pod->uid) || pod->uid == c->pend.uid)
    return fail(c, KSG_ERR_ARG, "duplicate pod uid %llu", (unsigned long long)pod->uid);
  c->upd_q.push_back({true, host_id, *pod, std::vector<uint32_t>(ids, ids + ext), pod->uid});
  c->q_added.insert(pod->uid);
  c->q_removed.erase(pod->uid);
  return KSG_OK;
}

int ksg_remove_pod(ksg_ctx* c, uint64_t uid) {
  if (!c) return KSG_ERR_ARG;
  KSG_LOCK(c);
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->pending) return remove_pod_impl(c, uid);
  const bool live = (c->pods.count(uid) && !c->q_removed.count(uid)) || c->q_added.count(uid);
  if (!live) return fail(c, KSG_ERR_ARG, "unknown pod uid %llu", (unsigned long long)uid);
  c->upd_q.push_back({false, 0, ksg_pod{}, {}, uid});
  c->q_added.erase(uid);
  c->q_removed.insert(uid);
  return KSG_OK;
}

int ksg_schedule_begin(ksg_ctx* c, const ksg_pod* pod, const uint32_t* ids, int64_t* max_score,
                       uint32_t* tie_count, uint8_t* fail_codes) {
  if (!c || !pod) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (int rc0 = flush_deferred(c)) return rc0;
  if (int rs = cluster_ok(c)) return rs;
  HIPCHK(c, hipSetDevice(c->device));
  if (c->pending) {  // the previous begin was abandoned: its queued updates apply now
    c->pending = false;
    c->pend_srv = false;
    if (int rq = apply_queued(c)) return rq;
  }
  if (c->N == 0) return KSG_NONODES;
  if (c->ext_on && !c->cur_ext) c->ext_scalar.erase(pod->uid);  // (plain entry point: no extension requests)
  const size_t ext = call_ids_extent(c, pod);
  int rc = check_pod(c, pod, ids, ext);
  if (rc) return rc;
  if (srv_eligible(c)) {  // the resident server: one request, no launch / copy / stream sync
    uint32_t hdr[KSG_SRV_HDR_DW] = {KSG_SRV_BEGIN};
    if ((rc = srv_alloc(c))) return rc;
    // (an all-zero record for the plain entry point of an extensions context)
    static const ksg_pod_ext zero_ext{};
    const ksg_pod_ext* xr = c->ext_on ? (c->cur_ext ? c->cur_ext : &zero_ext) : nullptr;
    // ServiceAffinity (predicates.go:257-324): the labels the pod's nodeSelector does not give come
    // from its service's first peer's node; resolved here from the host mirror (svc_peer, kept equal
    // to the device's) so the scan workgroups skip that dependent chain (pod_resolve then finds
    // every requirement given; an unlabelled peer leaves -1, which it resolves to the same -1)
    ksg_pod rp;
    const ksg_pod* sp = pod;
    if (!c->h_aff_pair.empty() && pod->service >= 0 && (uint32_t)pod->service < c->S) {
      const int32_t peer = c->svc_peer[pod->service];
      bool given = true;
      for (uint32_t j = 0; j < c->cfg.n_aff_labels && j < KSG_MAX_AFF; ++j) given = given && pod->aff_pair[j] != -1;
      if (!given && peer >= 0 && (uint32_t)peer < c->N) {
        rp = *pod;
        for (uint32_t j = 0; j < c->cfg.n_aff_labels && j < KSG_MAX_AFF; ++j)
          if (rp.aff_pair[j] == -1) rp.aff_pair[j] = c->h_aff_pair[(size_t)j * c->N + (uint32_t)peer];
        sp = &rp;
      }
    }
    if (srv_put_pod(c, sp, ids, ext, xr, hdr)) {
      if ((rc = flush_patches(c)) || (!c->srv_running && (rc = srv_flush_patches(c)))) return rc;
      if (fail_codes) hdr[KSG_SRVH_FLAGS] |= KSG_SRVF_WANT_FAIL;
      uint32_t r[4];
      if ((rc = srv_begin(c, hdr, r))) return rc;
      // (the last COMMIT was served before this BEGIN: a rejected one diverged the context)
      if ((rc = srv_settle(c))) return rc;
      if (r[1] == KSG_SRV_BADREQ) return fail(c, KSG_ERR_STATE, "drop-in server rejected begin request");
      if (r[1] == ~0u) return fail(c, KSG_ERR_NOPEER, "service affinity peer is not on a known node");
      if (fail_codes) memcpy(fail_codes, c->srv_fail, (size_t)(c->hi - c->lo));
      const int64_t m = (int64_t)((uint64_t)r[2] | ((uint64_t)r[3] << 32));
      if (max_score) *max_score = r[1] > 0 ? m : 0;
      if (tie_count) *tie_count = r[1];
      if (r[1] == 0) return KSG_NOFIT;
      c->pending = true;
      c->pending_k = r[1];
      c->pend = *pod;
      c->pend_ids.assign(ids, ids + ext);
      c->pend_srv = true;
      memcpy(c->srv_bhdr, hdr, sizeof hdr);
      c->srv_pext_on = xr != nullptr;
      if (xr) c->srv_pext = *xr;
      return KSG_OK;
    }
  }
  if ((rc = srv_stop(c))) return rc;
  if ((rc = flush_patches(c))) return rc;
  if ((rc = ensure_map(c)) || (rc = upload_one(c, pod, ids, ext))) return rc;
  if ((rc = scan_exchange(c, c->one_pod, c->one_ids, KSG_MODE_BEGIN, fail_codes ? c->d_fail : nullptr, nullptr,
                          c->ext_on ? c->d_one_ext : nullptr)))
    return rc;
  HIPCHK(c, ksg_launch_decide(c->dev, c->one_pod, c->one_ids, rec_buf(c), c->rec_bytes, c->world,
                              c->d_shard_wlo, 0, 0, c->d_rng, nullptr, 0, reinterpret_cast<int64_t*>(c->d_map),
                              c->st));
  int64_t summ[3];
  const size_t nf = fail_codes ? (size_t)(c->hi - c->lo) : 0;
  if (nf) {
    if ((rc = grow_host(c, &c->h_dn, &c->h_dn_cap, nf))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->h_dn, c->d_fail, nf, hipMemcpyDeviceToHost, c->st));
  }
  HIPCHK(c, hipStreamSynchronize(c->st));
  memcpy(summ, c->h_map, sizeof summ);
  if (nf) memcpy(fail_codes, c->h_dn, nf);
  if (summ[2]) return fail(c, KSG_ERR_NOPEER, "service affinity peer is not on a known node");
  if (max_score) *max_score = summ[1] > 0 ? summ[0] : 0;
  if (tie_count) *tie_count = (uint32_t)summ[1];
  if (summ[1] == 0) return KSG_NOFIT;
  c->pending = true;
  c->pending_k = (uint64_t)summ[1];
  c->pend = *pod;
  c->pend_ids.assign(ids, ids + ext);
  return KSG_OK;
}

// the device half of a commit: decide the tie_index-th tie and apply AssumePod's delta
static int commit_on_device(ksg_ctx* c, uint32_t tie_index, int32_t* node) {
  HIPCHK(c, hipSetDevice(c->device));
  if (c->pend_srv) {  // served by the resident server
    c->pend_srv = false;
    // the tie_index-th tie from the top (generic_scheduler.go:88-95) from the begin's tie words
    const int64_t off = srv_pick(c->srv_tw, c->pending_k - 1 - tie_index);
    if (off < 0 || off >= (int64_t)(c->hi - c->lo)) return fail(c, KSG_ERR_STATE, "commit selected no node");
    *node = (int32_t)(c->lo + (uint32_t)off);
    // AssumePod's delta: one control request carrying the pod, not waited for (the next
    // BEGIN's scan waits on the device until it is applied)
    uint32_t hdr[KSG_SRV_HDR_DW] = {KSG_SRV_COMMIT};
    if (int rc = srv_settle(c)) return rc;  // (the control block is free)
    if (!srv_put_pod(c, &c->pend, c->pend_ids.data(), c->pend_ids.size(), c->srv_pext_on ? &c->srv_pext : nullptr,
                     hdr, true))
      return fail(c, KSG_ERR_STATE, "pending pod does not fit the request block");
    hdr[KSG_SRVH_ARG] = (uint32_t)*node;
    if (c->srv_trace) fprintf(stderr, "srv commit node %d\n", *node);
    uint32_t seq = 0;
    if (int rc = srv_post(c, hdr, &seq)) return rc;
    c->srv_unacked = seq;
    return KSG_OK;
  }
  int rc = ensure_map(c);
  if (rc) return rc;
  if ((rc = srv_stop(c))) return rc;
  // the pending pod is still in d_one (begin's upload; nothing re-uploads before the commit)
  HIPCHK(c, ksg_launch_decide(c->dev, c->one_pod, c->one_ids, rec_buf(c), c->rec_bytes, c->world,
                              c->d_shard_wlo, 2, tie_index, c->d_rng, reinterpret_cast<int32_t*>(c->d_map + 32), 0,
                              c->d_summary, c->st, c->ext_on ? c->d_one_ext : nullptr));
  HIPCHK(c, hipStreamSynchronize(c->st));
  memcpy(node, c->h_map + 32, 4);
  if (*node < 0) return fail(c, KSG_ERR_STATE, "commit selected no node (%d)", *node);
  return KSG_OK;
}

int ksg_schedule_commit(ksg_ctx* c, uint32_t tie_index, int32_t* out_node) {
  if (!c) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (!c->pending) return fail(c, KSG_ERR_STATE, "no schedule_begin pending");
  if (tie_index >= c->pending_k) return fail(c, KSG_ERR_ARG, "tie_index %u >= tie_count %llu", tie_index,
                                             (unsigned long long)c->pending_k);
  int32_t node = -1;
  int rc = commit_on_device(c, tie_index, &node);
  c->pending = false;
  if (rc == KSG_OK) rc = mirror_add(c, (uint32_t)node, &c->pend, c->pend_ids.data(), false);
  c->pend.uid = ~0ULL;
  // the updates queued while the begin was pending apply now, whatever the outcome
  const int rq = apply_queued(c);
  if (rc) return rc;
  if (rq) return rq;
  if (out_node) *out_node = node;
  return KSG_OK;
}

int ksg_schedule_batch(ksg_ctx* c, const ksg_pod* pods, uint32_t n, const uint32_t* ids, uint32_t n_ids,
                       uint64_t* rng_state, int32_t* out_nodes) {
  if (!c || (n && (!pods || !out_nodes)) || !rng_state) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (c->pending) return fail(c, KSG_ERR_STATE, "schedule_begin pending");
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  if (int rs = cluster_ok(c)) return rs;
  HIPCHK(c, hipSetDevice(c->device));
  c->last_ms = 0.0;
  if (n == 0) return KSG_OK;
  if (c->N == 0) {
    for (uint32_t i = 0; i < n; ++i) out_nodes[i] = KSG_OUT_NONODES;
    return KSG_OK;
  }
  // host time per phase (ksg_last_batch_host_us)
  for (double& v : c->last_hus) v = 0.0;
  auto t_last = std::chrono::steady_clock::now();
  auto hphase = [&](int k) {
    const auto t = std::chrono::steady_clock::now();
    c->last_hus[k] += std::chrono::duration<double, std::micro>(t - t_last).count();
    t_last = t;
  };
  for (uint32_t i = 0; i < n; ++i) {
    int rc = check_pod(c, pods + i, ids, n_ids);
    if (rc) return rc;
    if (c->pods.count(pods[i].uid) || c->dfr_uids.count(pods[i].uid))
      return fail(c, KSG_ERR_ARG, "pod %u: duplicate uid", i);
  }
  hphase(0);
  int rc;
  if (c->dfr_neg && (rc = flush_deferred(c))) return rc;
  if ((rc = flush_patches(c))) return rc;
  if ((rc = upload_pods(c, pods, n, ids, n_ids))) return rc;
  if ((rc = ensure_out(c, n))) return rc;
  // the placements and the generator state come back through pinned staging
  // (a pageable copy-out blocks the host until the stream drains); the window
  // path enqueues them with each round, which usually ends the batch, so the
  // host waits for the device once per batch
  const size_t dn_rng = ((size_t)n * 4 + 7) & ~(size_t)7;
  if ((rc = grow_host(c, &c->h_dn, &c->h_dn_cap, dn_rng + 8))) return rc;
  bool tail_queued = false;
  auto enqueue_tail = [&]() -> int {
    HIPCHK(c, hipEventRecord(c->ev1, c->st));
    HIPCHK(c, hipMemcpyAsync(c->h_dn, c->d_out, (size_t)n * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipMemcpyAsync(c->h_dn + dn_rng, c->d_rng, 8, hipMemcpyDeviceToHost, c->st));
    return KSG_OK;
  };
  // Host work that overlaps the device: the previous batch's mirror replay, then
  // this batch's deferred-replay inputs (pods, ids, every uid: the few pods that
  // find no node are taken out again after the wait)
  // (stashed into locals: they become the context's deferred replay only when
  // the batch succeeds; a failure after the device work started leaves the
  // context diverged until ksg_set_cluster)
  bool stashed = false, dup_any = false;
  std::vector<ksg_pod> st_pods;
  std::vector<uint32_t> st_ids;
  std::unordered_set<uint64_t> st_uids;
  auto overlap_work = [&]() -> int {
    if (stashed) return KSG_OK;
    int rc2 = flush_deferred(c);
    if (rc2) return rc2;
    hphase(4);
    st_pods.assign(pods, pods + n);
    st_ids.assign(ids, ids + n_ids);
    st_uids.swap(c->dfr_uids);  // (empty after the flush: keeps its buckets)
    st_uids.reserve(2 * (size_t)n);
    for (uint32_t i = 0; i < n; ++i) dup_any |= !st_uids.insert(pods[i].uid).second;
    stashed = true;
    hphase(7);
    return KSG_OK;
  };
  struct DivergeGuard {
    ksg_ctx* c;
    bool armed = false;
    ~DivergeGuard() {
      if (armed) {
        drop_deferred(c);
        c->diverged = true;
      }
    }
  } guard{c};
  if (c->dev.dbg & 16384) c->dbg_fail_next = true;  // KSG_DEBUG & 16384: fail the batch after its device work
  guard.armed = true;  // device work from here on
  HIPCHK(c, hipMemcpyAsync(c->d_rng, rng_state, 8, hipMemcpyHostToDevice, c->st));
  HIPCHK(c, hipEventRecord(c->ev0, c->st));
  c->last_stats[0] = c->last_stats[1] = c->last_stats[2] = c->last_stats[3] = 0;
  c->last_kms[0] = c->last_kms[1] = c->last_kms[2] = c->last_t0ms = 0;
  c->last_wsum = 0;
  hphase(1);
  const ksg_pod_ext* dext = nullptr;
  if (c->ext_on) {  // extensions: each pod's record (all-zero for the plain entry point)
    if ((rc = grow(c, (void**)&c->d_pext, &c->pext_cap, n, sizeof(ksg_pod_ext)))) return rc;
    if (c->cur_ext) {
      HIPCHK(c, hipMemcpyAsync(c->d_pext, c->cur_ext, (size_t)n * sizeof(ksg_pod_ext), hipMemcpyHostToDevice, c->st));
    } else {
      HIPCHK(c, hipMemsetAsync(c->d_pext, 0, (size_t)n * sizeof(ksg_pod_ext), c->st));
    }
    dext = c->d_pext;
  }
  if (use_window(c, pods, n)) {
    // Window path. Phase A scores the window on this rank's shard; with world > 1
    // the per-word results are all-gathered once per window (not per pod) and
    // every rank runs the same resolver over the whole replicated node state, so
    // every rank commits the same pods to the same nodes.
    const KsgDev full = full_geometry(c);
    uint32_t W = std::min(c->window, ksg_win_max_window(full));
    // Phase A scores all W pods of a window whatever the resolver gets through.
    // Where windows stop early (ServiceAntiAffinity: every ~13 pods on config 4)
    // the capacity follows the pods per window measured on earlier batches: 3x
    // that, in pod groups of 8, at least 16. (A sharded context keeps W: every
    // rank must size its launches alike, and its estimate restarts each batch.)
    if (!c->xchg && c->ppw_est > 0.0) {
      const uint32_t want = ((uint32_t)std::ceil(3.0 * c->ppw_est) + 7u) & ~7u;
      W = std::min(W, std::max<uint32_t>(want, 16u));
    }
    KsgWinXchg x{};
    x.exts = dext;  // (extensions: the filters, and the scores when esc)
    x.ostride = std::max<uint32_t>(c->nwords_max, 1);
    x.wcap = W;
    x.world = (uint32_t)c->world;
    for (int g = 0; g < c->world; ++g) {
      uint32_t a, b;
      ksg_shard_words(c->nw, (uint32_t)g, (uint32_t)c->world, &a, &b);
      x.wlo[g] = a;
      x.nw[g] = b - a;
    }
    const bool anti = anti_on(c);
    const bool rr = anti && c->dev.rr_dz != 0 && c->d_zmap;  // ServiceAntiAffinity re-rank
    const size_t fit_off = ((size_t)W * x.ostride * 12 + 7) & ~(size_t)7;
    // (the domain counts are zeroed once here, then by each resolver for the next window)
    x.fit_off = anti ? (uint32_t)fit_off : 0u;
    x.b_off = rr ? (uint32_t)(fit_off + (size_t)W * x.ostride * 8) : 0u;
    // extension scores on the plain resolver: the pods' fit bitmaps at the same offset
    const bool esc = c->ext_on && (c->ext.w_taint_toleration != 0 || c->ext.w_balanced != 0);
    const bool etm = esc && c->ext.w_taint_toleration != 0;  // (the TaintToleration count pass)
    x.esc = esc ? 1u : 0u;
    x.efit_off = esc ? (uint32_t)fit_off : 0u;
    // the plain resolver without extensions up to 16,384 nodes (its ring holds the bitmaps):
    // phase A's single-commit drop bitmaps at the same offset
    const bool d1 = !anti && !dext && c->win_d1 && c->nw <= 4 * 64;
    x.d1 = d1 ? 1u : 0u;
    x.d1_off = d1 ? (uint32_t)fit_off : 0u;
    x.blk = ((rr                  ? fit_off + (size_t)W * x.ostride * 16
              : anti || esc || d1 ? fit_off + (size_t)W * x.ostride * 8
                                  : (size_t)W * x.ostride * 12) +
             255) & ~(size_t)255;
    if (esc) {
      if ((rc = grow(c, (void**)&c->d_etmax, &c->etmax_cap, W, sizeof(int32_t))) ||
          (rc = grow(c, (void**)&c->d_ethist, &c->ethist_cap, (size_t)W * KSG_TBINS, sizeof(int32_t))) ||
          (rc = grow(c, (void**)&c->d_epsoft, &c->epsoft_cap, W, sizeof(uint64_t))))
        return rc;
      // (zero once here; each resolver zeroes them again for the next window's count pass)
      HIPCHK(c, hipMemsetAsync(c->d_etmax, 0, (size_t)W * sizeof(int32_t), c->st));
      HIPCHK(c, hipMemsetAsync(c->d_ethist, 0, (size_t)W * KSG_TBINS * sizeof(int32_t), c->st));
      x.tmax = c->d_etmax;
      x.thist = c->d_ethist;
      x.psoft = c->d_epsoft;
    }
    const size_t dcnt_n = (size_t)W * std::max<uint32_t>(c->D, 1);
    if (anti) {
      if ((rc = grow(c, (void**)&c->d_dcnt, &c->dcnt_cap, dcnt_n, sizeof(int32_t)))) return rc;
      HIPCHK(c, hipMemsetAsync(c->d_dcnt, 0, dcnt_n * sizeof(int32_t), c->st));
      x.dcnt = c->d_dcnt;
      x.dcnt_n = (uint32_t)dcnt_n;
    }
    if (rr) {  // (the resolver resets the row bests to KSG_S32_NONE and the B counts to 0 for the next window)
      const size_t dmb_n = (size_t)W * c->dev.rr_dz;  // [W][dz] row bests, then [W][dz] B nodes per row
      if ((rc = grow(c, (void**)&c->d_dmb, &c->dmb_cap, 2 * dmb_n, sizeof(int32_t)))) return rc;
      HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)c->d_dmb, (int)0x80000000, dmb_n, c->st));
      HIPCHK(c, hipMemsetAsync(c->d_dmb + dmb_n, 0, dmb_n * sizeof(int32_t), c->st));
      x.rr = 1;
      x.dz = c->dev.rr_dz;
      x.dmb = c->d_dmb;
      x.zmap = c->d_zmap;
    }
    if ((rc = grow(c, (void**)&c->d_winsum, &c->win_cap, W, sizeof(KsgWinSum)))) return rc;
    if ((rc = grow(c, (void**)&c->d_xsend, &c->xsend_cap, x.blk, 1))) return rc;
    if (c->xchg && (rc = grow(c, (void**)&c->d_xrecv, &c->xrecv_cap, x.blk * c->world, 1))) return rc;
    x.buf = c->xchg ? c->d_xrecv : c->d_xsend;
    const bool plain = !anti;  // the plain resolver reads T0 images
    if (plain) {
      x.img_stride = ksg_win_t0_stride(full);
      if ((rc = grow(c, (void**)&c->d_t0img, &c->t0img_cap, (size_t)W * x.img_stride, 1))) return rc;
      x.img = c->d_t0img;
    }
    // one launch per window (KsgFused): one rank, no ServiceAntiAffinity, no extensions
    const uint32_t fgroups = plain && !c->xchg && !dext && c->win_fused && full.nwords <= c->fused_max_words &&
                                     ksg_win_fused_ok(full)
                                 ? ksg_win_fused_groups(full, W) : 0u;
    const bool fused = fgroups > 0 && fgroups <= kFctlGroups;
    KsgWinRun* const fruns = reinterpret_cast<KsgWinRun*>(c->d_fctl);
    uint32_t* const fcnt = reinterpret_cast<uint32_t*>(c->d_fctl + kFctlRuns);
    uint64_t* wbits = reinterpret_cast<uint64_t*>(c->d_xsend);
    int32_t* wmax = reinterpret_cast<int32_t*>(c->d_xsend + (size_t)W * x.ostride * 8);
    // Windows are chained on the device: each kernel reads the window's start
    // from d_run (written by the previous resolver), so the host enqueues a
    // round of windows and synchronises once per round, not once per window.
    // Windows per round: from the pods per window the previous rounds resolved
    // (windows stop early on service / exhaustion / slot events, e.g. every ~13
    // pods with ServiceAntiAffinity), 10% over; launches past the batch's end
    // return at once. Fewer rounds = fewer host synchronisations per batch.
    // A sharded context issues one collective per launch, so every rank must
    // enqueue the same number of launches: its estimate starts fresh each batch
    // and follows only this batch's progress, which every rank resolves alike.
    double ppw_est = c->xchg ? 0.0 : c->ppw_est;
    auto round_k = [&](uint32_t left) -> uint32_t {
      const double ppw = ppw_est > 0.0 ? std::min<double>(std::max(ppw_est, 1.0), (double)W) : 0.8 * W;
      const double k = std::ceil((double)left / ppw * c->round_margin) + 1.0;
      return (uint32_t)std::min(k, 8192.0);
    };
    uint32_t pos = 0, K = round_k(n);
    c->last_kms[0] = c->last_kms[1] = c->last_kms[2] = c->last_t0ms = 0;
    c->last_wsum = 0;
    hphase(2);
    while (pos < n) {
      if (c->wev.size() < 3 * (size_t)K + 1) {
        const size_t old = c->wev.size();
        c->wev.resize(3 * (size_t)K + 1, nullptr);
        for (size_t i = old; i < c->wev.size(); ++i) HIPCHK(c, hipEventCreateWithFlags(&c->wev[i], kTimingEvent));
      }
      // the sampled launches rotate from round to round (launches k with
      // (k + ev_off) % es == 0), so every position in a round, the no-op
      // launches after the batch's end included, is timed equally often
      const uint32_t es = std::min(c->ev_stride, K);  // (a short round still times one launch)
      const uint32_t ev_off = es ? c->ev_phase++ % es : 0u;
      *c->h_run = KsgWinRun{pos, n, 0, 0, {0, 0, 0, 0}};
      if (fused) {  // slot 0 and both counter sets (the launches zero the next set as they go)
        *reinterpret_cast<KsgWinRun*>(c->h_fctl) = *c->h_run;
        HIPCHK(c, hipMemcpyAsync(c->d_fctl, c->h_fctl, kFctlRuns + (size_t)2 * fgroups * 8 * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, c->st));
      } else {
        HIPCHK(c, hipMemcpyAsync(c->d_run, c->h_run, sizeof(KsgWinRun), hipMemcpyHostToDevice, c->st));
      }
      HIPCHK(c, hipEventRecord(c->wev[0], c->st));
      for (uint32_t k = 0; k < K; ++k) {
        // HIP events on this stream around the sampled launches (per-kernel device time)
        const bool evk = es && (k + ev_off) % es == 0;
        // (launch k: events 3k before phase A, 3k+1 after it, 3k+2 before the resolver, 3k+3 =
        // the next launch's 3(k+1) after it; the fused launch: 3k before it, 3k+3 after it)
        if (evk && k > 0) HIPCHK(c, hipEventRecord(c->wev[3 * k], c->st));
        if (fused) {
          // the counter rows: fgroups per set, set k & 1 (the host zeroed both for launch 0; each
          // launch's block 0 zeroes the other set for the next launch)
          KsgFused f{c->d_pods, c->d_ids, fruns + ((k + 1) & 1), fcnt, k & 1u, fgroups};
          HIPCHK(c, ksg_launch_win_fused(full, W, fruns + (k & 1), c->d_winsum, x, c->d_rng, c->d_out, f,
                                         c->fused_grid, c->st));
          if (evk) HIPCHK(c, hipEventRecord(c->wev[3 * k + 3], c->st));
          continue;
        }
        if (anti) {
          // ServiceAntiAffinity: the pods' per-domain counts over their filtered nodes first
          // (into d_dcnt, zero: the previous resolver cleared it)
          HIPCHK(c, ksg_launch_win_eval(c->dev, 1, c->d_pods, c->d_ids, c->d_run, W, c->d_winsum, wbits, wmax,
                                        x.ostride, c->d_dcnt, nullptr, x.dmb, nullptr, x.dz, c->st, dext));
          if (c->xchg && (rc = allreduce_sum_i32(c, c->d_dcnt, c->d_dcnt, (uint32_t)dcnt_n))) return rc;
        }
        if (etm) {  // TaintToleration: each pod's max soft-taint count over its filtered nodes first
          HIPCHK(c, ksg_launch_win_eval(c->dev, 3, c->d_pods, c->d_ids, c->d_run, W, c->d_winsum, wbits, wmax,
                                        x.ostride, nullptr, nullptr, nullptr, nullptr, 0, c->st, dext, x.tmax,
                                        x.psoft, x.thist));
          // sharded: over every shard's filtered nodes (the max, and the histogram of soft
          // counts whose bin at the max the resolver's normalisation stop reads)
          if (c->xchg && ((rc = allreduce_max_i32(c, x.tmax, x.tmax, W)) ||
                          (rc = allreduce_sum_i32(c, x.thist, x.thist, W * KSG_TBINS))))
            return rc;
        }
        HIPCHK(c, ksg_launch_win_eval(c->dev, anti ? 2 : 0, c->d_pods, c->d_ids, c->d_run, W, c->d_winsum, wbits,
                                      wmax, x.ostride, c->d_dcnt,
                                      (anti || esc || d1) ? reinterpret_cast<uint64_t*>(c->d_xsend + fit_off) : nullptr,
                                      x.dmb, rr ? reinterpret_cast<uint64_t*>(c->d_xsend + x.b_off) : nullptr, x.dz,
                                      c->st, dext, x.tmax, x.psoft));
        if (evk) HIPCHK(c, hipEventRecord(c->wev[3 * k + 1], c->st));
        if (c->xchg && (rc = allgather(c, c->d_xsend, c->d_xrecv, x.blk))) return rc;
        if (plain) HIPCHK(c, ksg_launch_win_t0(full, W, c->d_run, x, c->st));
        if (evk) HIPCHK(c, hipEventRecord(c->wev[3 * k + 2], c->st));
        HIPCHK(c, ksg_launch_win_resolve(full, W, c->d_run, c->d_winsum, x, c->d_rng, c->d_out, c->st));
        if (evk) HIPCHK(c, hipEventRecord(c->wev[3 * k + 3], c->st));
      }
      HIPCHK(c, hipMemcpyAsync(c->h_run, fused ? fruns + (K & 1) : c->d_run, sizeof(KsgWinRun), hipMemcpyDeviceToHost,
                               c->st));
      if ((rc = enqueue_tail())) return rc;
      hphase(3);
      if ((rc = overlap_work())) return rc;  // the host mirror catches up while the device works
      if ((rc = wait_device(c))) return rc;
      hphase(5);
      const KsgWinRun r = *c->h_run;
      if (r.windows > 0 && r.pos > pos) {  // pods per window, smoothed over rounds and batches
        const double ppw = (double)(r.pos - pos) / (double)r.windows;
        ppw_est = ppw_est > 0.0 ? 0.5 * ppw_est + 0.5 * ppw : ppw;
        if (!c->xchg) c->ppw_est = ppw_est;
      }
      // the sampled launches (every one of the round's launches is a sampling
      // candidate, including the ones after the batch was done, which return at
      // once, so the mean matches a kernel trace of the run), scaled to all K
      double ea = 0.0, eb = 0.0, et = 0.0;
      uint32_t nt = 0;
      for (uint32_t k = es ? (es - ev_off) % es : 0u; es && k < K; k += es) {
        float a = 0.f, t0 = 0.f, b = 0.f;
        if (fused) {  // (one kernel: its whole time is the resolver's, phase A runs inside it)
          HIPCHK(c, hipEventElapsedTime(&b, c->wev[3 * k], c->wev[3 * k + 3]));
        } else {
          HIPCHK(c, hipEventElapsedTime(&a, c->wev[3 * k], c->wev[3 * k + 1]));
          HIPCHK(c, hipEventElapsedTime(&t0, c->wev[3 * k + 1], c->wev[3 * k + 2]));
          HIPCHK(c, hipEventElapsedTime(&b, c->wev[3 * k + 2], c->wev[3 * k + 3]));
        }
        ea += a;
        et += t0;
        eb += b;
        ++nt;
      }
      if (nt) {
        c->last_kms[0] += ea * K / nt;
        c->last_kms[1] += eb * K / nt;
        c->last_t0ms += et * K / nt;
      }
      c->last_kms[2] += K;
      c->last_wsum += (double)W * K;
      c->last_stats[0] += r.windows;
      for (int q = 1; q <= 3; ++q) c->last_stats[q] += r.stops[q];
      if (c->dbg_fail_next) {
        c->dbg_fail_next = false;
        return fail(c, KSG_ERR_STATE, "window resolver: injected failure (KSG_DEBUG & 16384) at pod %u", r.pos);
      }
      if (r.halt == KSG_HALT_HANG) return fail(c, KSG_ERR_STATE, "window resolver: ring wait timed out at pod %u", r.pos);
      if (r.halt == KSG_HALT_BAD)
        return fail(c, KSG_ERR_STATE,
                    "window resolver: selection outside T0 at pod %u (inconsistent prefixes or drop positions: a bug, "
                    "or stale verdicts under the KSG_DEBUG timing switches)", r.pos);
      if (r.halt == KSG_HALT_BADCOUNT || r.pos < pos || r.pos > n)
        return fail(c, KSG_ERR_STATE, "window resolver: bad progress (halt %u, pos %u -> %u)", r.halt, pos, r.pos);
      pos = r.pos;
      tail_queued = pos >= n && r.halt != KSG_HALT_OVERSIZE;  // (the copies saw the finished batch)
      if (r.halt == KSG_HALT_OVERSIZE) {
        // a pod whose id lists exceed the window record: the exact per-pod path
        if (!c->xchg) {
          HIPCHK(c, ksg_launch_batch(c->R, anti, c->dev, c->d_pods + pos, c->d_ids, 1, c->d_rng,
                                     c->d_out + pos, c->st, dext ? dext + pos : nullptr));
        } else {
          if ((rc = scan_exchange(c, c->d_pods + pos, c->d_ids, KSG_MODE_BEGIN, nullptr, nullptr,
                                  dext ? dext + pos : nullptr)))
            return rc;
          HIPCHK(c, ksg_launch_decide(c->dev, c->d_pods + pos, c->d_ids, rec_buf(c), c->rec_bytes, c->world,
                                      c->d_shard_wlo, 1, 0, c->d_rng, c->d_out, pos, c->d_summary, c->st,
                                      dext ? dext + pos : nullptr));
        }
        pos += 1;
        ++c->last_stats[3];
      }
      // next round (rare: stops shortened this round's windows): the rest at W/2 pods per window
      K = round_k(n - std::min(pos, n));
      hphase(2);
    }
  } else if (!c->xchg) {
    HIPCHK(c, ksg_launch_batch(c->R, anti_on(c), c->dev, c->d_pods, c->d_ids, n, c->d_rng, c->d_out, c->st, dext));
  } else {
    for (uint32_t i = 0; i < n; ++i) {
      if ((rc = scan_exchange(c, c->d_pods + i, c->d_ids, KSG_MODE_BEGIN, nullptr, nullptr, dext ? dext + i : nullptr)))
        return rc;
      HIPCHK(c, ksg_launch_decide(c->dev, c->d_pods + i, c->d_ids, rec_buf(c), c->rec_bytes, c->world,
                                  c->d_shard_wlo, 1, 0, c->d_rng, c->d_out, i, c->d_summary, c->st,
                                  dext ? dext + i : nullptr));
    }
  }
  if (!tail_queued) {
    if ((rc = enqueue_tail())) return rc;
    hphase(3);
    if ((rc = overlap_work())) return rc;
    if ((rc = wait_device(c))) return rc;
    hphase(6);
  }
  memcpy(out_nodes, c->h_dn, (size_t)n * 4);
  memcpy(rng_state, c->h_dn + dn_rng, 8);
  float ms = 0.f;
  HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->last_ms = ms;
  // the device applied every commit; the host mirror replays them later
  // (flush_deferred), overlapped with the next batch's device work
  if (!stashed) {  // (overlap_work ran on every path that reaches here)
    return fail(c, KSG_ERR_STATE, "internal: batch replay inputs missing");
  }
  guard.armed = false;
  if (c->ext_on && !c->cur_ext)  // (plain entry point: the pods carry no extension requests)
    for (uint32_t i = 0; i < n; ++i) c->ext_scalar.erase(pods[i].uid);
  c->dfr_pods.swap(st_pods);
  c->dfr_ids.swap(st_ids);
  c->dfr_uids.swap(st_uids);
  c->dfr_out.assign(out_nodes, out_nodes + n);
  for (uint32_t i = 0; i < n; ++i)  // the uids of the pods that found no node are free again
    if (out_nodes[i] < 0 && !dup_any) c->dfr_uids.erase(pods[i].uid);
  if (dup_any) {  // a uid repeats within the batch: an error iff two placed pods share it
    for (uint32_t i = 0; i < n; ++i) c->dfr_uids.erase(pods[i].uid);
    for (uint32_t i = 0; i < n; ++i)
      if (out_nodes[i] >= 0 && !c->dfr_uids.insert(pods[i].uid).second)  // (mirror_add reports it at the replay)
        return fail(c, KSG_ERR_ARG, "pod %u: duplicate uid within the batch", i);
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (out_nodes[i] < 0) continue;
    if (pods[i].milli_cpu < 0 || pods[i].memory < 0) c->dfr_neg = true;
    else c->dfr_sum = std::min<int64_t>(c->dfr_sum + std::min<int64_t>(pods[i].milli_cpu + pods[i].memory,
                                                                        KSG_WIN_LR_BOUND), KSG_WIN_LR_BOUND + 1);
  }
  hphase(7);
  double* t = c->totals;  // (layout: ksg_batch_totals in kschedgpu.h)
  t[0] += 1;
  t[1] += c->last_ms;
  for (int q = 0; q < 3; ++q) t[2 + q] += c->last_kms[q];
  t[17] += c->last_wsum;
  t[18] += c->last_t0ms;
  for (int q = 0; q < 4; ++q) t[5 + q] += c->last_stats[q];
  for (int q = 0; q < 8; ++q) t[9 + q] += c->last_hus[q];
  return KSG_OK;
}

int ksg_evaluate(ksg_ctx* c, const ksg_pod* pod, const uint32_t* ids, uint8_t* fail_out, int64_t* score_out) {
  if (!c || !pod) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (c->pending) return fail(c, KSG_ERR_STATE, "schedule_begin pending");
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  if (int rc0 = flush_deferred(c)) return rc0;
  if (int rs = cluster_ok(c)) return rs;
  HIPCHK(c, hipSetDevice(c->device));
  if (c->N == 0) return KSG_NONODES;
  const size_t ext = call_ids_extent(c, pod);
  int rc = check_pod(c, pod, ids, ext);
  if (rc) return rc;
  if ((rc = flush_patches(c))) return rc;
  if ((rc = upload_one(c, pod, ids, ext))) return rc;
  // errors surface through the BEGIN record, so run BEGIN first for the flag
  if ((rc = scan_exchange(c, c->one_pod, c->one_ids, KSG_MODE_BEGIN, nullptr, nullptr, c->ext_on ? c->d_one_ext : nullptr)))
    return rc;
  HIPCHK(c, ksg_launch_decide(c->dev, c->one_pod, c->one_ids, rec_buf(c), c->rec_bytes, c->world,
                              c->d_shard_wlo, 0, 0, c->d_rng, nullptr, 0, c->d_summary, c->st));
  if ((rc = scan_exchange(c, c->one_pod, c->one_ids, KSG_MODE_EVAL, c->d_fail, c->d_score, c->ext_on ? c->d_one_ext : nullptr)))
    return rc;
  int64_t summ[3];
  HIPCHK(c, hipMemcpyAsync(summ, c->d_summary, sizeof summ, hipMemcpyDeviceToHost, c->st));
  const size_t ns = c->hi - c->lo;
  if (fail_out && ns) HIPCHK(c, hipMemcpyAsync(fail_out, c->d_fail, ns, hipMemcpyDeviceToHost, c->st));
  if (score_out && ns) HIPCHK(c, hipMemcpyAsync(score_out, c->d_score, ns * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  if (summ[2]) return fail(c, KSG_ERR_NOPEER, "service affinity peer is not on a known node");
  return KSG_OK;
}

int ksg_set_allgather(ksg_ctx* c, ksg_allgather_fn fn, void* user) {
  if (!c) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (c->comm) return fail(c, KSG_ERR_STATE, "context already exchanges over RCCL");
  c->xfn = fn;
  c->xuser = user;
  return KSG_OK;
}

int ksg_set_window(ksg_ctx* c, uint32_t window) {
  if (!c) return KSG_ERR_ARG;
  KSG_LOCK(c);
  c->window = window;
  c->ppw_est = 0.0;
  return KSG_OK;
}

int ksg_last_batch_stats(ksg_ctx* c, uint32_t* stats4) {
  if (!c || !stats4) return KSG_ERR_ARG;
  KSG_LOCK(c);
  for (int i = 0; i < 4; ++i) stats4[i] = c->last_stats[i];
  return KSG_OK;
}

int ksg_last_batch_kernel_ms(ksg_ctx* c, double* out3) {
  if (!c || !out3) return KSG_ERR_ARG;
  KSG_LOCK(c);
  for (int i = 0; i < 3; ++i) out3[i] = c->last_kms[i];
  return KSG_OK;
}

int ksg_batch_totals(ksg_ctx* c, double* out24) {
  if (!c || !out24) return KSG_ERR_ARG;
  KSG_LOCK(c);
  for (int k = 0; k < 24; ++k) out24[k] = c->totals[k];
  return KSG_OK;
}

int ksg_last_batch_host_us(ksg_ctx* c, double* out8) {
  if (!c || !out8) return KSG_ERR_ARG;
  KSG_LOCK(c);
  for (int k = 0; k < 8; ++k) out8[k] = c->last_hus[k];
  return KSG_OK;
}

int ksg_serve_stats(ksg_ctx* c, uint64_t* out4) {
  if (!c || !out4) return KSG_ERR_ARG;
  KSG_LOCK(c);
  out4[0] = c->srv_launches;
  out4[1] = c->srv_seq;
  out4[2] = c->srv_running ? 1 : 0;
  out4[3] = srv_eligible(c) ? (srv_grid(c) ? 2 : 1) : 0;
  return KSG_OK;
}

int ksg_debug_counters(ksg_ctx* c, int32_t* out, uint32_t n_words) {
  if (!c || (!out && n_words)) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  if (!c->dev.dbgbuf) return fail(c, KSG_ERR_STATE, "debug counters need KSG_DEBUG=8 at ksg_create");
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipStreamSynchronize(c->st));
  int32_t words[KSG_DEBUG_COUNTER_WORDS];
  HIPCHK(c, hipMemcpy(words, c->dev.dbgbuf, sizeof(words), hipMemcpyDeviceToHost));
  for (uint32_t k = 0; k < n_words; ++k) out[k] = k < KSG_DEBUG_COUNTER_WORDS ? words[k] : 0;
  return KSG_OK;
}

int ksg_last_batch_ms(ksg_ctx* c, double* ms) {
  if (!c || !ms) return KSG_ERR_ARG;
  KSG_LOCK(c);
  *ms = c->last_ms;
  return KSG_OK;
}

int ksg_shard(ksg_ctx* c, uint32_t* lo, uint32_t* hi) {
  if (!c) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (lo) *lo = c->lo;
  if (hi) *hi = c->hi;
  return KSG_OK;
}

int ksg_read_requested(ksg_ctx* c, int64_t* milli_cpu, int64_t* memory) {
  if (!c || !c->have_cluster) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  HIPCHK(c, hipSetDevice(c->device));
  int rc = flush_patches(c);
  if (rc) return rc;
  if (c->N) {
    if (milli_cpu) HIPCHK(c, hipMemcpyAsync(milli_cpu, c->dev.used_cpu, c->N * 8, hipMemcpyDeviceToHost, c->st));
    if (memory) HIPCHK(c, hipMemcpyAsync(memory, c->dev.used_mem, c->N * 8, hipMemcpyDeviceToHost, c->st));
  }
  HIPCHK(c, hipStreamSynchronize(c->st));
  return KSG_OK;
}

// ---- kubelet admission (ksg_admit.hip) ------------------------------------
static int admit_impl(ksg_ctx* c, int mode, const ksg_admission_set* sets, uint32_t n_sets, const ksg_pod* pods,
                      uint32_t n_pods, const uint32_t* ids, uint32_t n_ids, const uint32_t* pairs, uint32_t n_pairs,
                      uint8_t* out) {
  if (!c || (n_sets && !sets) || (n_pods && (!pods || !out))) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  for (uint32_t s = 0; s < n_sets; ++s) {
    if ((uint64_t)sets[s].pod_off + sets[s].n_pods > n_pods)
      return fail(c, KSG_ERR_ARG, "admission set %u: pods out of range", s);
    if ((mode & KSG_ADMIT_MODE_SELECTOR) && (uint64_t)sets[s].label_off + sets[s].n_labels > n_pairs)
      return fail(c, KSG_ERR_ARG, "admission set %u: labels out of range", s);
  }
  if (mode & KSG_ADMIT_MODE_SELECTOR) {
    if ((n_ids && !ids) || (n_pairs && !pairs)) return fail(c, KSG_ERR_ARG, "admission: ids / pairs == NULL");
    for (uint32_t i = 0; i < n_pods; ++i)
      if ((uint64_t)pods[i].sel_off + pods[i].n_sel > n_ids)
        return fail(c, KSG_ERR_ARG, "pod %u: nodeSelector ids out of range", i);
  }
  // each pod in at most one set (one kernel lane per set writes its pods' results)
  std::vector<uint8_t> in_set(n_pods, 0);
  for (uint32_t s = 0; s < n_sets; ++s)
    for (uint32_t k = 0; k < sets[s].n_pods; ++k)
      if (in_set[sets[s].pod_off + k]++)
        return fail(c, KSG_ERR_ARG, "admission sets %u and an earlier one share pod %u", s, sets[s].pod_off + k);
  for (uint32_t i = 0; i < n_pods; ++i) out[i] = KSG_ADMIT_OK;  // pods in no set
  if (n_sets == 0 || n_pods == 0) return KSG_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const bool sel = (mode & KSG_ADMIT_MODE_SELECTOR) != 0;
  const size_t b_sets = (size_t)n_sets * sizeof(ksg_admission_set), b_pods = (size_t)n_pods * sizeof(ksg_pod);
  const size_t b_ids = sel ? (size_t)n_ids * 4 : 0, b_pairs = sel ? (size_t)n_pairs * 4 : 0;
  const size_t o_pods = (b_sets + 15) & ~(size_t)15, o_ids = o_pods + ((b_pods + 15) & ~(size_t)15);
  const size_t o_pairs = o_ids + ((b_ids + 15) & ~(size_t)15), o_out = o_pairs + ((b_pairs + 15) & ~(size_t)15);
  const size_t total = o_out + n_pods;
  int rc;
  if ((rc = grow(c, (void**)&c->d_admit, &c->admit_cap, total, 1))) return rc;
  if ((rc = grow_host(c, &c->h_up, &c->h_up_cap, o_out))) return rc;
  memcpy(c->h_up, sets, b_sets);
  memcpy(c->h_up + o_pods, pods, b_pods);
  if (b_ids) memcpy(c->h_up + o_ids, ids, b_ids);
  if (b_pairs) memcpy(c->h_up + o_pairs, pairs, b_pairs);
  HIPCHK(c, hipMemcpyAsync(c->d_admit, c->h_up, o_out, hipMemcpyHostToDevice, c->st));
  HIPCHK(c, ksg_launch_admit(reinterpret_cast<const ksg_admission_set*>(c->d_admit), n_sets,
                             reinterpret_cast<const ksg_pod*>(c->d_admit + o_pods),
                             reinterpret_cast<const uint32_t*>(c->d_admit + o_ids),
                             reinterpret_cast<const uint32_t*>(c->d_admit + o_pairs), mode, c->d_admit + o_out, c->st));
  if ((rc = grow_host(c, &c->h_dn, &c->h_dn_cap, n_pods))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->h_dn, c->d_admit + o_out, n_pods, hipMemcpyDeviceToHost, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  // pods outside every set keep KSG_ADMIT_OK; the kernel wrote the others
  for (uint32_t i = 0; i < n_pods; ++i)
    if (in_set[i]) out[i] = c->h_dn[i];
  return KSG_OK;
}

// ---- extensions (include/kschedgpu.h; parity unpinned) ----------------------
int ksg_set_extensions(ksg_ctx* c, const ksg_ext_config* e) {
  if (!c || !e) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (c->have_cluster) return fail(c, KSG_ERR_STATE, "ksg_set_extensions: call before ksg_set_cluster");
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  if ((e->filters & ~(KSG_EXT_TAINTS | KSG_EXT_SCALAR)) || e->n_scalar > KSG_MAX_SCALAR)
    return fail(c, KSG_ERR_ARG, "extensions: bad filters / n_scalar");
  c->ext = *e;
  c->ext_on = e->filters || e->w_taint_toleration || e->w_balanced || e->n_scalar;
  return KSG_OK;
}

int ksg_set_node_ext(ksg_ctx* c, uint32_t n_nodes, const int64_t* scalar_cap, const uint32_t* taint_off,
                     const uint32_t* taint_n, const uint32_t* taint_ids, uint32_t n_taint_ids) {
  if (!c) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (c->pending) return fail(c, KSG_ERR_STATE, "schedule_begin pending");
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  if (!c->ext_on) return fail(c, KSG_ERR_STATE, "ksg_set_node_ext: extensions are off");
  if (!c->have_cluster || n_nodes != c->N) return fail(c, KSG_ERR_ARG, "ksg_set_node_ext: node count != cluster");
  if (int rc0 = flush_deferred(c)) return rc0;
  if (!c->pods.empty()) return fail(c, KSG_ERR_STATE, "ksg_set_node_ext: call before adding pods");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t NN = std::max<uint32_t>(c->N, 1);
  if (c->ext.n_scalar && n_nodes) {
    if (!scalar_cap) return fail(c, KSG_ERR_ARG, "ksg_set_node_ext: scalar_cap missing");
    HIPCHK(c, hipMemcpyAsync(const_cast<int64_t*>(c->dev.scalar_cap), scalar_cap, (size_t)c->ext.n_scalar * n_nodes * 8,
                             hipMemcpyHostToDevice, c->st));
  }
  std::vector<uint64_t> tm((size_t)std::max<uint32_t>(c->ext.max_taints, 1) * std::max<uint32_t>(c->nw, 1), 0);
  if (taint_off && taint_n)
    for (uint32_t n = 0; n < n_nodes; ++n)
      for (uint32_t i = 0; i < taint_n[n]; ++i) {
        if ((size_t)taint_off[n] + i >= n_taint_ids || !taint_ids) return fail(c, KSG_ERR_ARG, "taint list out of range");
        const uint32_t t = taint_ids[taint_off[n] + i];
        if (t >= c->ext.max_taints) return fail(c, KSG_ERR_CAPACITY, "taint id %u >= max_taints", t);
        tm[(size_t)t * c->nw + (n >> 6)] |= 1ULL << (n & 63);
      }
  HIPCHK(c, hipMemcpyAsync(const_cast<uint64_t*>(c->dev.taintmap), tm.data(), tm.size() * 8, hipMemcpyHostToDevice,
                           c->st));
  if (c->dev.ntaint) {  // the same taints as one mask per node (taint ids < 64)
    std::vector<uint64_t> ntm(std::max<uint32_t>(n_nodes, 1), 0);
    if (taint_off && taint_n)
      for (uint32_t n = 0; n < n_nodes; ++n)
        for (uint32_t i = 0; i < taint_n[n]; ++i) ntm[n] |= 1ULL << (taint_ids[taint_off[n] + i] & 63);
    HIPCHK(c, hipMemcpyAsync(const_cast<uint64_t*>(c->dev.ntaint), ntm.data(), ntm.size() * 8, hipMemcpyHostToDevice,
                             c->st));
  }
  HIPCHK(c, hipMemsetAsync(c->dev.scalar_used, 0, (size_t)std::max<uint32_t>(c->ext.n_scalar, 1) * NN * 8, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  c->sc_used.assign((size_t)c->ext.n_scalar * c->N, 0);
  return KSG_OK;
}

int ksg_read_ext_used(ksg_ctx* c, int64_t* used) {
  if (!c || !used || !c->have_cluster) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (!c->ext_on) return fail(c, KSG_ERR_STATE, "ksg_read_ext_used: extensions are off");
  if (int rs_ = srv_stop(c)) return rs_;  // (the resident server leaves the stream)
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = flush_patches(c)) return rc;
  const size_t nb = (size_t)c->ext.n_scalar * c->N * 8;
  if (nb) HIPCHK(c, hipMemcpyAsync(used, c->dev.scalar_used, nb, hipMemcpyDeviceToHost, c->st));
  HIPCHK(c, hipStreamSynchronize(c->st));
  return KSG_OK;
}

// validate a pod's extension record against the call's id array and record its
// extended-resource requests by uid (the host mirror's AssumePod/remove)
static int check_ext_range(ksg_ctx* c, const ksg_pod_ext* e, size_t n_ids) {
  if ((size_t)e->hard_off + e->n_hard > n_ids || (size_t)e->soft_off + e->n_soft > n_ids)
    return fail(c, KSG_ERR_ARG, "extension taint list out of range");
  return KSG_OK;
}
static int note_ext(ksg_ctx* c, const ksg_pod* p, const ksg_pod_ext* e, size_t n_ids) {
  if (int rc = check_ext_range(c, e, n_ids)) return rc;
  std::array<int64_t, KSG_MAX_SCALAR> sc{};
  bool any = false;
  for (uint32_t q = 0; q < c->ext.n_scalar; ++q) {
    sc[q] = e->scalar[q];
    any |= sc[q] != 0;
  }
  if (any) c->ext_scalar[p->uid] = sc;
  else c->ext_scalar.erase(p->uid);
  return KSG_OK;
}
// a taint list is a set: TaintTolerationPriority counts each untolerated taint of the node once,
// and the window path counts a soft list as a bit mask while the exact kernels count its entries,
// so a repeated id would make the answer depend on the path
static bool has_repeat(const uint32_t* v, uint32_t n) {
  if (n <= 64) {
    for (uint32_t i = 1; i < n; ++i)
      for (uint32_t j = 0; j < i; ++j)
        if (v[i] == v[j]) return true;
    return false;
  }
  std::vector<uint32_t> s(v, v + n);
  std::sort(s.begin(), s.end());
  return std::adjacent_find(s.begin(), s.end()) != s.end();
}
static int check_taint_ids(ksg_ctx* c, const ksg_pod_ext* e, const uint32_t* ids) {
  for (uint32_t i = 0; i < e->n_hard; ++i)
    if (ids[e->hard_off + i] >= c->ext.max_taints) return fail(c, KSG_ERR_CAPACITY, "taint id out of range");
  for (uint32_t i = 0; i < e->n_soft; ++i)
    if (ids[e->soft_off + i] >= c->ext.max_taints) return fail(c, KSG_ERR_CAPACITY, "taint id out of range");
  if ((e->n_hard && has_repeat(ids + e->hard_off, e->n_hard)) || (e->n_soft && has_repeat(ids + e->soft_off, e->n_soft)))
    return fail(c, KSG_ERR_ARG, "a taint id repeats in the pod's hard or soft list (each list is a set)");
  return KSG_OK;
}

int ksg_add_pod_ext(ksg_ctx* c, uint32_t host_id, const ksg_pod* pod, const ksg_pod_ext* ext, const uint32_t* ids) {
  if (!c || !pod) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (ext && !c->ext_on) return fail(c, KSG_ERR_STATE, "extensions are off");
  if (c->ext_on) {
    const ksg_pod_ext z{};
    const ksg_pod_ext* e = ext ? ext : &z;
    const size_t n_ids = std::max(pod_ids_extent(pod), std::max<size_t>((size_t)e->hard_off + e->n_hard,
                                                                         (size_t)e->soft_off + e->n_soft));
    if (int rc = note_ext(c, pod, e, n_ids)) return rc;
  }
  c->cur_ext = ext;
  const int rc = ksg_add_pod(c, host_id, pod, ids);
  c->cur_ext = nullptr;
  return rc;
}

int ksg_schedule_batch_draws(ksg_ctx* c, const ksg_pod* pods, uint32_t n, const uint32_t* ids, uint32_t n_ids,
                             const uint64_t* draws, uint32_t n_draws, uint32_t* draws_used, int32_t* out_nodes) {
  if (!c || (n && (!pods || !out_nodes || !draws)) || !draws_used) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (n_draws < n) return fail(c, KSG_ERR_ARG, "%u draws for %u pods: one per pod that may find a node", n_draws, n);
  for (uint32_t k = 0; k < n; ++k)
    if (draws[k] > (uint64_t)INT64_MAX) return fail(c, KSG_ERR_ARG, "draw %u is not a rand.Int() value", k);
  *draws_used = 0;
  if (c->pending) return fail(c, KSG_ERR_STATE, "schedule_begin pending");
  if (n == 0) return ksg_schedule_batch(c, pods, 0, ids, n_ids, &c->draw_tmp, out_nodes);
  HIPCHK(c, hipSetDevice(c->device));
  if (int rs_ = srv_stop(c)) return rs_;
  if (int rc = grow(c, (void**)&c->d_draws, &c->draws_cap, n, sizeof(uint64_t))) return rc;
  HIPCHK(c, hipMemcpy(c->d_draws, draws, (size_t)n * sizeof(uint64_t), hipMemcpyHostToDevice));
  c->dev.draws = c->d_draws;  // (the generator state is now the index of the next value)
  uint64_t state = 0;
  const int rc = ksg_schedule_batch(c, pods, n, ids, n_ids, &state, out_nodes);
  c->dev.draws = nullptr;
  if (rc == KSG_OK) *draws_used = (uint32_t)state;
  return rc;
}

// A rejected Bind in batch mode (scheduler.go:107-112: no AssumePod for pod k, its rand.Int()
// already drawn at generic_scheduler.go:94, pod k + 1 scheduled against the state without it).
// The batch committed pods 0..n-1 in order, so undoing the commits of pods n-1 down to k leaves
// exactly the state after pods 0..k-1; pods k+1..n-1 are then re-batched by the caller with the
// draws they had consumed put back (a splitmix64 state is stepped back over them instead).
int ksg_batch_unwind(ksg_ctx* c, const ksg_pod* pods, const int32_t* out_nodes, uint32_t n, uint32_t k,
                     uint64_t* rng_state, uint32_t* draws_kept) {
  if (!c || !pods || !out_nodes || !draws_kept || k >= n) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (c->pending) return fail(c, KSG_ERR_STATE, "schedule_begin pending");
  if (out_nodes[k] < 0) return fail(c, KSG_ERR_ARG, "pod %u found no node: there was no Bind to reject", k);
  if (int rs = cluster_ok(c)) return rs;
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc0 = flush_deferred(c)) return rc0;  // (the batch's commits into the host mirror)
  // (validate every uid before removing any: a failed call changes nothing)
  for (uint32_t i = k; i < n; ++i)
    if (out_nodes[i] >= 0 && !c->pods.count(pods[i].uid))
      return fail(c, KSG_ERR_ARG, "pod %u (uid %llu) is not a committed pod of this context", i,
                  (unsigned long long)pods[i].uid);
  uint32_t kept = 0, back = 0;
  for (uint32_t i = 0; i <= k; ++i) kept += out_nodes[i] >= 0 ? 1u : 0u;
  for (uint32_t i = n; i-- > k;) {  // newest first
    if (out_nodes[i] < 0) continue;
    if (i > k) ++back;
    if (int rc = remove_pod_impl(c, pods[i].uid)) return rc;
  }
  if (rng_state) *rng_state -= (uint64_t)back * ksg_rng_step(nullptr);
  *draws_kept = kept;
  return flush_patches(c);
}

int ksg_schedule_batch_ext(ksg_ctx* c, const ksg_pod* pods, const ksg_pod_ext* ext, uint32_t n, const uint32_t* ids,
                           uint32_t n_ids, uint64_t* rng_state, int32_t* out_nodes) {
  if (!c || (n && (!pods || !out_nodes)) || !rng_state) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (ext && !c->ext_on) return fail(c, KSG_ERR_STATE, "extensions are off");
  // validate the whole batch first; each placed pod's extended-resource requests
  // are recorded (for the host mirror's deferred replay) only once the batch
  // succeeded, and the pods that found no node leave no entry
  if (c->ext_on && ext)
    for (uint32_t i = 0; i < n; ++i) {
      if (int rc = check_ext_range(c, ext + i, n_ids)) return rc;
      if (int rc = check_taint_ids(c, ext + i, ids)) return rc;
    }
  c->cur_ext = ext;
  const int rc = ksg_schedule_batch(c, pods, n, ids, n_ids, rng_state, out_nodes);
  c->cur_ext = nullptr;
  if (rc == KSG_OK && c->ext_on && ext)
    for (uint32_t i = 0; i < n; ++i) {
      if (out_nodes[i] >= 0) (void)note_ext(c, pods + i, ext + i, n_ids);
      else c->ext_scalar.erase(pods[i].uid);
    }
  return rc;
}

int ksg_schedule_begin_ext(ksg_ctx* c, const ksg_pod* pod, const ksg_pod_ext* ext, const uint32_t* ids,
                           int64_t* max_score, uint32_t* tie_count, uint8_t* fail_codes) {
  if (!c || !pod) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (ext && !c->ext_on) return fail(c, KSG_ERR_STATE, "extensions are off");
  c->cur_ext = ext;
  int rc = KSG_OK;
  if (ext) {
    const size_t n_ids = call_ids_extent(c, pod);
    if (!(rc = check_ext_range(c, ext, n_ids)) && !(rc = check_taint_ids(c, ext, ids))) rc = note_ext(c, pod, ext, n_ids);
  }
  if (!rc) rc = ksg_schedule_begin(c, pod, ids, max_score, tie_count, fail_codes);
  c->cur_ext = nullptr;
  return rc;
}

int ksg_evaluate_ext(ksg_ctx* c, const ksg_pod* pod, const ksg_pod_ext* ext, const uint32_t* ids, uint8_t* fail_out,
                     int64_t* score_out) {
  if (!c || !pod) return KSG_ERR_ARG;
  KSG_LOCK(c);
  if (ext && !c->ext_on) return fail(c, KSG_ERR_STATE, "extensions are off");
  c->cur_ext = ext;
  int rc = ext ? check_taint_ids(c, ext, ids) : KSG_OK;
  if (!rc) rc = ksg_evaluate(c, pod, ids, fail_out, score_out);
  c->cur_ext = nullptr;
  return rc;
}

int ksg_check_pods_exceeding_capacity(ksg_ctx* c, const ksg_admission_set* sets, uint32_t n_sets,
                                      const ksg_pod* pods, uint32_t n_pods, uint8_t* fits) {
  const int rc = admit_impl(c, KSG_ADMIT_MODE_CAPACITY, sets, n_sets, pods, n_pods, nullptr, 0, nullptr, 0, fits);
  if (rc == KSG_OK)
    for (uint32_t i = 0; i < n_pods; ++i) fits[i] = fits[i] == KSG_ADMIT_OK;
  return rc;
}

int ksg_pod_matches_node_labels(ksg_ctx* c, const ksg_admission_set* sets, uint32_t n_sets, const ksg_pod* pods,
                                uint32_t n_pods, const uint32_t* ids, uint32_t n_ids, const uint32_t* pairs,
                                uint32_t n_pairs, uint8_t* matches) {
  const int rc = admit_impl(c, KSG_ADMIT_MODE_SELECTOR, sets, n_sets, pods, n_pods, ids, n_ids, pairs, n_pairs,
                            matches);
  if (rc == KSG_OK)
    for (uint32_t i = 0; i < n_pods; ++i) matches[i] = matches[i] == KSG_ADMIT_OK;
  return rc;
}

int ksg_admit_pods(ksg_ctx* c, const ksg_admission_set* sets, uint32_t n_sets, const ksg_pod* pods, uint32_t n_pods,
                   const uint32_t* ids, uint32_t n_ids, const uint32_t* pairs, uint32_t n_pairs, uint8_t* codes) {
  return admit_impl(c, KSG_ADMIT_MODE_SELECTOR | KSG_ADMIT_MODE_CAPACITY, sets, n_sets, pods, n_pods, ids, n_ids,
                    pairs, n_pairs, codes);
}

}  // extern "C"
