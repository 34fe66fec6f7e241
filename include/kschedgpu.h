/*
 * kschedgpu.h — C ABI of libkschedgpu.so, the MI355X-native Filter/Score pass of
 * the kube-scheduler generic scheduler (smarterclayton/kubernetes v0.13.0-dev).
 *
 * What this ABI replaces (reference file:line, all under /root/reference):
 *   algorithm.Scheduler.Schedule(pod, minionLister)      pkg/scheduler/scheduler.go:25-27
 *     implemented by genericScheduler.Schedule           pkg/scheduler/generic_scheduler.go:54-80
 *       findNodesThatFit                                 pkg/scheduler/generic_scheduler.go:100-128
 *       prioritizeNodes                                  pkg/scheduler/generic_scheduler.go:136-165
 *       selectHost / getBestHosts                        pkg/scheduler/generic_scheduler.go:84-96,167-177
 *   SystemModeler.AssumePod (the commit)                 plugin/pkg/scheduler/scheduler.go:42-47,115-118
 *   NewGenericScheduler(predicates, prioritizers, ...)   pkg/scheduler/generic_scheduler.go:197-204
 *     built by ConfigFactory.CreateFromKeys              plugin/pkg/scheduler/factory/factory.go:107-172
 *
 * Conventions
 *   - Strings never cross this ABI. The caller (the Go cgo shim, or the Python
 *     mirror in kubernetes_amd/) interns node names, label (key,value) pairs,
 *     label keys, host ports, GCE PD names and services to dense ids.
 *   - Node "rank" = index of the node in byte-wise ascending name order. The
 *     reference's tie order (score desc, host name desc; types.go:42-47) is
 *     therefore "rank desc".
 *   - All input arrays are caller-owned and copied before return. Output
 *     buffers are caller-allocated.
 *   - Return codes: KSG_OK (0); KSG_NOFIT (1) = *FitError; KSG_NONODES (2) =
 *     "no minions available to schedule pods"; negative = internal error, see
 *     ksg_last_error(). There is NO CPU fallback inside this library: every
 *     predicate/priority evaluation runs in HIP kernels on the GPU.
 *   - One scheduling thread per context (the reference calls Schedule from one
 *     goroutine, plugin/pkg/scheduler/scheduler.go:86-88). Every entry point
 *     holds the context's mutex, so other threads (the reflectors feeding the
 *     scheduled-pod store, factory.go:126-145) may call ksg_add_pod /
 *     ksg_remove_pod at any time: between pods they apply at once (a batch in
 *     flight finishes first); between ksg_schedule_begin and its commit they
 *     are validated, queued and applied in arrival order right after the
 *     commit (or when the begin is abandoned by the next begin).
 */
#ifndef KSCHEDGPU_H_
#define KSCHEDGPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSG_ABI_VERSION 3

/* ---- return codes ---------------------------------------------------- */
#define KSG_OK 0
#define KSG_NOFIT 1          /* generic_scheduler.go:72-77  *FitError              */
#define KSG_NONODES 2        /* generic_scheduler.go:59-61  no minions available   */
#define KSG_ERR_ARG (-1)
#define KSG_ERR_HIP (-2)
#define KSG_ERR_CAPACITY (-3)
#define KSG_ERR_STATE (-4)
#define KSG_ERR_NOPEER (-5)  /* predicates.go:293-296: service peer's host is not a known node */
#define KSG_ERR_RCCL (-6)

/* out_nodes[] codes of ksg_schedule_batch (>= 0 is a node rank) */
#define KSG_OUT_NOFIT (-1)
#define KSG_OUT_ERROR (-2)
#define KSG_OUT_NONODES (-3)

/* ---- predicates (FitPredicate registry names, factory/plugins.go:63-117) */
#define KSG_PRED_PODFITSPORTS      (1u << 0) /* predicates.go:326-350 */
#define KSG_PRED_PODFITSRESOURCES  (1u << 1) /* predicates.go:94-145  */
#define KSG_PRED_NODISKCONFLICT    (1u << 2) /* predicates.go:52-83   */
#define KSG_PRED_MATCHNODESELECTOR (1u << 3) /* predicates.go:161-179 */
#define KSG_PRED_HOSTNAME          (1u << 4) /* predicates.go:181-186 */
#define KSG_PRED_SERVICEAFFINITY   (1u << 5) /* predicates.go:231-324 (policy) */
#define KSG_PRED_LABELSPRESENCE    (1u << 6) /* predicates.go:188-229 (policy) */

/* fail codes written per node by ksg_schedule_begin/ksg_evaluate:
 * 0 = fits, otherwise the first failing predicate in this fixed order. */
#define KSG_FAIL_NONE 0
#define KSG_FAIL_HOSTNAME 1
#define KSG_FAIL_LABELSPRESENCE 2
#define KSG_FAIL_MATCHNODESELECTOR 3
#define KSG_FAIL_NODISKCONFLICT 4
#define KSG_FAIL_PODFITSPORTS 5
#define KSG_FAIL_PODFITSRESOURCES 6
#define KSG_FAIL_SERVICEAFFINITY 7

#define KSG_MAX_ANTI 64          /* ServiceAntiAffinity priorities (policy)      */
#define KSG_MAX_LABEL_PREF 32    /* LabelPreference priorities (policy)          */
#define KSG_MAX_PRESENCE 16      /* LabelsPresence predicates (policy)           */
#define KSG_MAX_PRESENCE_KEYS 16 /* labels per LabelsPresence predicate          */
#define KSG_MAX_AFF 16          /* ServiceAffinity labels (union of predicates) */
#define KSG_MAX_AFF_GROUPS 32   /* ServiceAffinity predicates (label groups)    */

/* Label pair flag in ksg_set_cluster's pair_keys[p]: the pair's key fails
 * IsQualifiedName or its value fails IsValidLabelValue (pkg/util/validation.go),
 * so a selector built from it by SelectorFromSet is the empty selector that
 * matches every node (pkg/labels/selector.go:654-668). The key id is
 * pair_keys[p] & ~KSG_PAIR_INVALID. */
#define KSG_PAIR_INVALID 0x80000000u
/* ksg_pod.aff_pair[j]: the pod's nodeSelector gives ServiceAffinity label j
 * an invalid value (or label j's key is invalid). */
#define KSG_AFF_INVALID (-2)

/* Scheduler configuration: the compiled form of map[string]FitPredicate +
 * []PriorityConfig that NewGenericScheduler receives (factory.go:149).
 * Any Policy the reference accepts fits: weights are int64 and the list caps
 * above are well past what a Policy names in practice (the reference registers
 * any number, plugins.go:81-183); factory.compile reports a Policy beyond them. */
typedef struct ksg_config {
  uint32_t predicates;          /* KSG_PRED_* bitmask                                   */
  uint32_t n_priority_configs;  /* len(priorityConfigs); 0 => EqualPriority fallback
                                   (generic_scheduler.go:141-143)                       */
  /* Priority weights are Go ints (plugin/pkg/scheduler/api/types.go:46: int64 on
   * the reference's platform) and combined scores wrap like Go's int
   * (generic_scheduler.go:145-159). While 10 * sum|w| + |w_equal| < 2^30 the
   * window path runs with int32 scores (any number of ServiceAntiAffinity
   * priorities, any shard size up to 131,072 nodes); otherwise every batch takes
   * the exact kernels with int64 (wrapping) combined scores. */
  int64_t w_least_requested;    /* LeastRequestedPriority weight, 0 = absent/skipped    */
  int64_t w_service_spreading;  /* ServiceSpreadingPriority weight                       */
  int64_t w_equal;              /* EqualPriority weight (DefaultProvider: 0, skipped)    */
  uint32_t n_anti;              /* ServiceAntiAffinity priorities                        */
  uint32_t anti_key[KSG_MAX_ANTI];   /* label-key id of each                           */
  int64_t w_anti[KSG_MAX_ANTI];
  uint32_t n_label_pref;        /* LabelPreference priorities                            */
  uint32_t pref_key[KSG_MAX_LABEL_PREF];
  uint32_t pref_presence[KSG_MAX_LABEL_PREF];
  int64_t w_pref[KSG_MAX_LABEL_PREF];
  uint32_t n_presence;          /* LabelsPresence predicates                             */
  uint32_t presence_n_keys[KSG_MAX_PRESENCE];
  uint32_t presence_keys[KSG_MAX_PRESENCE][KSG_MAX_PRESENCE_KEYS];
  uint32_t presence_flag[KSG_MAX_PRESENCE];
  uint32_t n_aff_labels;        /* ServiceAffinity: label-key ids (union over predicates) */
  uint32_t aff_key[KSG_MAX_AFF];
  uint32_t max_conflict_keys;   /* capacity for interned host-port + GCE-PD ids          */
  uint32_t max_domains;         /* capacity for anti-affinity label values (pair ids)    */
  /* ServiceAffinity predicates: bit j of aff_group_mask[g] = aff label j belongs
   * to predicate g. Each predicate builds its own selector, so SelectorFromSet's
   * invalid-value trap empties one predicate's selector, not the others'
   * (predicates.go:311-315). n_aff_groups == 0: one predicate over every label. */
  uint32_t n_aff_groups;
  uint32_t aff_group_mask[KSG_MAX_AFF_GROUPS];
} ksg_config;

/* One node, rank-ordered. Capacity is node.Spec.Capacity converted with
 * Quantity.MilliValue (cpu) / Value (memory) (resource_helpers.go:29-42). */
typedef struct ksg_node {
  int64_t cap_milli_cpu;
  int64_t cap_memory;
  uint32_t label_off;   /* offset into node_pairs[] of this node's label pair ids */
  uint32_t n_labels;
} ksg_node;

/* One pod (pending or existing). Variable-length lists are (offset, count)
 * into a caller-supplied uint32 id array passed alongside. */
typedef struct ksg_pod {
  uint64_t uid;         /* caller-unique id (namespace/name) for ksg_remove_pod     */
  int64_t milli_cpu;    /* getResourceRequest: sum of container Limits cpu (milli)  */
  int64_t memory;       /* ... and memory (bytes) (predicates.go:94-102)            */
  int32_t host;         /* Spec.Host: -1 empty, -2 names no node, else node rank    */
  int32_t service;      /* services[0] of GetPodServices, -1 none                   */
  uint32_t ports_off, n_ports;  /* conflict-key ids of HostPorts != 0               */
  uint32_t pds_off, n_pds;      /* conflict-key ids of GCE PD names                 */
  uint32_t sel_off, n_sel;      /* nodeSelector pair ids; 0 = pair no node has;
                                   n_sel == 0 => selector matches everything        */
  uint32_t svcs_off, n_svcs;    /* every service whose selector matches the pod     */
  int32_t aff_pair[KSG_MAX_AFF];/* ServiceAffinity: pair id of the pod's own
                                   nodeSelector value for aff label j; -1 = the pod
                                   does not specify it; 0 = value no node has;
                                   KSG_AFF_INVALID = an invalid value            */
} ksg_pod;

typedef struct ksg_ctx ksg_ctx;

/* Create a context on HIP device `device`. Single-GPU form. */
int ksg_create(const ksg_config* cfg, int device, ksg_ctx** out);

/* Node-sharded form: `world` (<= 16) processes, one per GPU, each owning the
 * node ranks of its run of 64-node words (ksg_shard_range). Node state is
 * replicated; filter/score evaluation is sharded. Window path: the shards'
 * per-word results for a window of pods are all-gathered once per window and
 * every rank resolves the window identically. Per-pod path (begin/commit,
 * ServiceAntiAffinity): the shard records are all-gathered per pod. `nccl_id`
 * is the 128-byte ncclUniqueId from rank 0 (RCCL over xGMI), or NULL to use a
 * host transport installed with ksg_set_allgather. world == 1 with an nccl_id
 * runs the same exchange path over a 1-rank RCCL communicator. */
int ksg_create_sharded(const ksg_config* cfg, int device, int rank, int world,
                       const void* nccl_id, ksg_ctx** out);
/* Host transport for a sharded context created with nccl_id == NULL: the
 * library calls fn(user, send, recv, bytes) with host buffers and fn must
 * all-gather `bytes` from every rank into recv, rank-major (world * bytes),
 * returning 0 on success. Every rank must make the same sequence of calls.
 * This is how a caller that owns its own transport (or a test that runs
 * several ranks on one GPU, where RCCL refuses duplicate devices) drives the
 * same sharded kernels; with an RCCL communicator the exchange stays on the
 * device stream. */
typedef int (*ksg_allgather_fn)(void* user, const void* send, void* recv, uint64_t bytes);
int ksg_set_allgather(ksg_ctx* ctx, ksg_allgather_fn fn, void* user);
/* Fill a fresh ncclUniqueId (128 bytes) for ksg_create_sharded on rank 0. */
int ksg_nccl_unique_id(void* out128);

int ksg_destroy(ksg_ctx* ctx);
const char* ksg_last_error(ksg_ctx* ctx);

/* Replace the node set (MinionLister.List()). Resets all pod state.
 * pair_keys[p] = label-key id of label pair p, | KSG_PAIR_INVALID for a pair
 * SelectorFromSet would reject (pair 0 is reserved: "no node has it").
 * node_pairs holds each node's label pair ids. */
int ksg_set_cluster(ksg_ctx* ctx, const ksg_node* nodes, uint32_t n_nodes,
                    const uint32_t* node_pairs, uint32_t n_node_pairs,
                    const uint32_t* pair_keys, uint32_t n_pairs,
                    uint32_t n_services);

/* Existing / assumed pods (SimpleModeler.AssumePod + scheduled-pod store).
 * host_id < n_nodes is a node rank (Status.Host); host_id >= n_nodes is a host
 * that is not in the node list (still counted by ServiceSpreading's maxCount,
 * spreading.go:73-80). */
int ksg_add_pod(ksg_ctx* ctx, uint32_t host_id, const ksg_pod* pod, const uint32_t* ids);
int ksg_remove_pod(ksg_ctx* ctx, uint64_t uid);

/* Static node terms beyond the config's fixed slots (more LabelsPresence
 * predicates or keys than KSG_MAX_PRESENCE x KSG_MAX_PRESENCE_KEYS, more
 * LabelPreference priorities than KSG_MAX_LABEL_PREF): the caller evaluates
 * them per node from the node labels and folds them in after ksg_set_cluster
 * (they end with that node list: call again after the next one).
 * fit_words (optional): ceil(n_nodes / 64) words in node-rank order, bit n%64
 * of word n/64 set iff node n passes every extra LabelsPresence predicate
 * (CheckNodeLabelPresence, predicates.go:194-229); a node that fails gets
 * KSG_FAIL_LABELSPRESENCE. score (optional): n_nodes Go-int sums of weight x
 * CalculateNodeLabelPriority (priorities.go:98-134) over the extra priorities,
 * added to every node's combined score with Go's wrap; score_weighted != 0
 * when any of them has a nonzero weight (the HostPriorityList is then not
 * empty). The config's predicates must include KSG_PRED_LABELSPRESENCE and its
 * n_priority_configs count the extra priorities. No reference counterpart (the
 * reference's registry takes any number of them: plugins.go:81-117, 145-183). */
int ksg_set_static_terms(ksg_ctx* ctx, const uint64_t* fit_words, const int64_t* score, int score_weighted);
/* The same static terms evaluated on the device from the node labels of the last
 * ksg_set_cluster, one slot pass per call: `extra`'s LabelsPresence slots
 * (n_presence, presence_n_keys, presence_keys, presence_flag) and LabelPreference
 * slots (n_label_pref, pref_key, pref_presence, w_pref) are evaluated per node
 * (ksg_static_kernel) and folded in like ksg_set_static_terms' arrays; every other
 * field of `extra` is ignored. Call it as often as the policy needs (each pass
 * holds up to KSG_MAX_PRESENCE predicates of KSG_MAX_PRESENCE_KEYS keys and
 * KSG_MAX_LABEL_PREF priorities); the terms end with the node list. */
int ksg_add_static_config(ksg_ctx* ctx, const ksg_config* extra);

/* Split Schedule: begin evaluates every node and reports the best combined
 * score and the number of nodes tied at it (0 => KSG_NOFIT). The caller draws
 * r = rand.Int() iff tie_count > 0 and calls commit(r % tie_count), which picks
 * the tie_index-th tie in descending name order (generic_scheduler.go:88-95)
 * and applies AssumePod's delta. fail_codes (optional, n_nodes bytes) gets the
 * per-node KSG_FAIL_* code to rebuild FailedPredicateMap.
 * On one rank (int32 scores; plain shards up to 261,120 nodes, others up to
 * 16,384) both calls are served by a resident kernel polling mapped host memory
 * (ksg_serve.hip): no kernel launch, copy or stream synchronisation per call.
 * begin returns the pod's tie words with its answer, and commit picks the node
 * from them on the host and returns at once: AssumePod's delta is applied on
 * the device before any later call reads device state (a rejected commit is
 * reported by the next call). The server returns after KSG_SERVE_IDLE_US
 * (default 20,000) without a request and is relaunched by the next one; any
 * other entry point that needs the device stops it first. KSG_SERVE=0 in the
 * environment at ksg_create: kernels launched per call. */
int ksg_schedule_begin(ksg_ctx* ctx, const ksg_pod* pod, const uint32_t* ids,
                       int64_t* max_score, uint32_t* tie_count, uint8_t* fail_codes);
int ksg_schedule_commit(ksg_ctx* ctx, uint32_t tie_index, int32_t* out_node);

/* Schedule n pods in order, committing each before the next, entirely on the
 * device. Tie-break source: splitmix64 with state *rng_state; one Int63 draw
 * (next() >> 1) per successful schedule only (generic_scheduler.go:94).
 * out_nodes[i] = node rank or KSG_OUT_*. *rng_state is advanced. */
int ksg_schedule_batch(ksg_ctx* ctx, const ksg_pod* pods, uint32_t n,
                       const uint32_t* ids, uint32_t n_ids,
                       uint64_t* rng_state, int32_t* out_nodes);

/* ksg_schedule_batch with the caller's own random source: draws[k] is the
 * k-th rand.Int() value the caller's generator would return (e.g. a Go
 * *rand.Rand's next n Int()s, n_draws >= n). Pod i that finds a node uses the
 * next unused value, exactly as n sequential Schedule calls would
 * (generic_scheduler.go:94); *draws_used = how many were used (the caller keeps
 * the rest for its next call). The sequential path's stream is reproduced:
 * no splitmix64. Every rank of a sharded context passes the same values. */
int ksg_schedule_batch_draws(ksg_ctx* ctx, const ksg_pod* pods, uint32_t n, const uint32_t* ids,
                             uint32_t n_ids, const uint64_t* draws, uint32_t n_draws, uint32_t* draws_used,
                             int32_t* out_nodes);

/* Bind rejected in batch mode. The reference binds each pod before it schedules
 * the next: a rejected Bind means no AssumePod for that pod, but its rand.Int()
 * was already drawn (plugin/pkg/scheduler/scheduler.go:93-118,
 * pkg/scheduler/generic_scheduler.go:94). A batch committed every placement on
 * the device, so when the caller binds pods[0..n) of the last batch in order and
 * pod k's Bind (out_nodes[k] >= 0) is rejected, this call undoes the commits of
 * pods k..n-1 (newest first), leaving the state of pods 0..k-1 committed.
 * *draws_kept = the draws pods 0..k consumed (pod k's stays consumed): with
 * ksg_schedule_batch_draws the caller puts draws[*draws_kept .. draws_used) back
 * at the front of its FIFO; rng_state (optional, ksg_schedule_batch's splitmix64
 * state) is stepped back over the draws of pods k+1..n-1. The caller then
 * re-batches pods k+1..n-1. pods / out_nodes are the last batch's arrays; every
 * rank of a sharded context makes the same call. KSG_ERR_ARG (nothing changed)
 * when k >= n, pod k found no node, or a placed pod's uid is not committed. */
int ksg_batch_unwind(ksg_ctx* ctx, const ksg_pod* pods, const int32_t* out_nodes, uint32_t n, uint32_t k,
                     uint64_t* rng_state, uint32_t* draws_kept);

/* Introspection (HostPriorityList): per-node fail code and combined score for
 * a pod, without committing. score_out[i] is meaningful where fail_out[i]==0. */
int ksg_evaluate(ksg_ctx* ctx, const ksg_pod* pod, const uint32_t* ids,
                 uint8_t* fail_out, int64_t* score_out);

/* Batch execution strategy. window > 0 (default 128, env KSG_WINDOW): pods
 * are filtered/scored a window at a time against one snapshot on all CUs and
 * then resolved in order by one workgroup (exact; see ksg_window.hip);
 * ServiceAntiAffinity adds a per-window domain-count pass. window = 0: the
 * persistent one-pod-at-a-time kernel. Both give identical results; a batch
 * takes the window path only where it is exact (non-negative LeastRequested /
 * ServiceSpreading weights, capacities and requested totals within 2^49, at
 * most 2048 node words). */
int ksg_set_window(ksg_ctx* ctx, uint32_t window);
/* Window statistics of the last ksg_schedule_batch: stats4[0] = windows
 * (snapshots), [1] = windows ended because a service scalar changed, [2] =
 * windows ended because every snapshot tie of a pod got worse, [3] = windows
 * ended by the per-node window cache filling up or an oversized pod. */
int ksg_last_batch_stats(ksg_ctx* ctx, uint32_t* stats4);

/* Device time (ms) of the last ksg_schedule_batch's kernels, from HIP events
 * recorded on the stream the kernels ran on. */
int ksg_last_batch_ms(ksg_ctx* ctx, double* ms);

/* Window path of the last ksg_schedule_batch: out3[0] = device ms in the
 * snapshot-scoring kernel(s) (ksg_win_score_kernel, its count passes and, on a
 * sharded context, the count passes' all-reduces; not the all-gather or the
 * T0-image kernel: ksg_batch_totals [18]), out3[1] = device ms in the
 * resolver (ksg_win_plain_kernel, or with ServiceAntiAffinity
 * ksg_win_resolve2_kernel / ksg_win_resolve_kernel; the fused window launch of
 * one plain rank scores the window inside the resolver's launch, so its whole
 * time is here and out3[0] is 0), out3[2] = resolver launches (windows are
 * chained on the device, so a round may end with launches that find the batch
 * done and return at once); from HIP events recorded on the context's stream
 * around every 4th launch of a round, the sampled positions rotating from round
 * to round (KSG_KERNEL_EVENTS=N in the environment at context creation: every
 * N-th, 0: none), the sampled launches' mean scaled to all launches: an event
 * between two dependent launches lengthens the gap between them. */
int ksg_last_batch_kernel_ms(ksg_ctx* ctx, double* out3);

/* Host time (microseconds, steady clock) of the last ksg_schedule_batch by
 * phase: out8[0] validation (pod checks, duplicate uids), [1] upload (pending
 * patches, pod copy-in), [2] window setup and round sizing, [3] enqueueing the
 * launches and copies, [4] the host-mirror replay of the previous batch
 * (overlapped with the device), [5] waiting for the device at the end of each
 * window round (the placements' copy-out rides with it), [6] waiting for a
 * separate copy-out (exact path, or a round that did not finish the batch),
 * [7] the deferred-replay bookkeeping. No reference counterpart (diagnostics). */
int ksg_last_batch_host_us(ksg_ctx* ctx, double* out8);

/* The per-batch diagnostics above summed over every successful
 * ksg_schedule_batch since the context was created, so a caller can read them
 * once around a run instead of after each batch: out24[0] batches, [1] device
 * ms (ksg_last_batch_ms), [2..4] ksg_last_batch_kernel_ms, [5..8]
 * ksg_last_batch_stats, [9..16] ksg_last_batch_host_us, [17] the window
 * capacity (pods phase A scores per launch) summed over the window-path
 * launches, [18] device ms between phase A and the resolver (the sharded
 * all-gather and the T0-image kernel, ksg_win_t0_kernel; the count passes'
 * all-reduces are in [2]; sampled like ksg_last_batch_kernel_ms), [19..23] zero. */
int ksg_batch_totals(ksg_ctx* ctx, double* out24);

/* Diagnostics: the window resolver's per-stage clock counters (s_memtime
 * cycles / 64, summed over every window since the context was created) for a
 * context created with KSG_DEBUG=8 in the environment (layout: DESIGN.md
 * section 4, "resolver stages"). The library holds KSG_DEBUG_COUNTER_WORDS
 * words; it copies min(n_words, KSG_DEBUG_COUNTER_WORDS) of them into out and
 * zero-fills the rest of out (ABI version 3: version 2's form took no length
 * and wrote 64 words into a buffer its parameter name said held 32).
 * KSG_ERR_STATE when not enabled. */
#define KSG_DEBUG_COUNTER_WORDS 64
int ksg_debug_counters(ksg_ctx* ctx, int32_t* out, uint32_t n_words);

/* Diagnostics of the resident begin/commit server: out4[0] kernel launches,
 * [1] requests served (begin, commit, patch, exit), [2] 1 while resident,
 * [3] 1 when this context uses the one-workgroup server, 2 the grid server
 * (one scan workgroup per 256 nodes; every plain shard by default,
 * KSG_SERVE_GRID=0 / KSG_SERVE_GRID_MIN), 0 none. No reference counterpart. */
int ksg_serve_stats(ksg_ctx* ctx, uint64_t* out4);

/* ---- node sharding (multi-GPU) ------------------------------
 * Nodes are split into contiguous runs of 64-node words in name-rank order.
 * Per pod every shard produces one record: this header followed by the shard's
 * tie bitmap (uint64 words, bit j of word w = node 64*(shard_first_word+w)+j
 * scores max_score). The winner rule over all records is the reference's
 * selectHost (generic_scheduler.go:84-96): global max, k = sum of the shards'
 * counts at the max, ix = Int63() % k, ix-th tie counted from the highest name
 * rank. ksg_schedule_batch/begin/commit apply it on the device after an RCCL
 * all-gather; these two host functions expose the same rule (same code) for a
 * caller that exchanges records over its own transport. */
typedef struct ksg_shard_record {
  int64_t max_score;  /* INT64_MIN if nothing fits in the shard */
  uint64_t tie_count; /* nodes of the shard at max_score */
  int32_t error;      /* nonzero: the pod errors (ServiceAffinity peer not a node) */
  int32_t pad;
  uint64_t pad2;
} ksg_shard_record;

/* Node range [lo, hi) of shard `rank` of `world` over n_nodes rank-ordered nodes. */
int ksg_shard_range(uint32_t n_nodes, int rank, int world, uint32_t* lo, uint32_t* hi);

/* Merge `world` records of rec_bytes each (header + ceil-words tie bitmap).
 * rng_state != NULL: draw Int63 from the splitmix64 stream only if k > 0 (as the
 * batch path); else use tie_index % k (as ksg_schedule_commit). Returns KSG_OK
 * with *out_node = global node rank, KSG_NOFIT (no draw), or KSG_ERR_NOPEER.
 * empty_priorities: the config has priority configs but all weights are 0. */
int ksg_merge_records(const void* records, uint32_t rec_bytes, uint32_t world, uint32_t n_nodes,
                      int empty_priorities, uint64_t* rng_state, uint64_t tie_index, int32_t* out_node,
                      int64_t* max_score, uint64_t* tie_count);

/* Node shard owned by this context: [lo, hi). */
int ksg_shard(ksg_ctx* ctx, uint32_t* lo, uint32_t* hi);

/* Copy the committed per-node requested totals (sum of limits of all pods on
 * the node) back to the host, for state checks. */
int ksg_read_requested(ksg_ctx* ctx, int64_t* milli_cpu, int64_t* memory);

/* ---- kubelet admission -------------------------------
 * The node agent re-checks its own pods with the scheduler's predicates
 * (handleNotFittingPods, pkg/kubelet/kubelet.go:1716-1771):
 *   checkNodeSelectorMatching -> PodMatchesNodeLabels          predicates.go:161-167
 *   checkCapacityExceeded     -> CheckPodsExceedingCapacity on
 *                                the pods sorted by creation    predicates.go:104-124
 * These entry points check many nodes' admission sets in one device pass. They
 * use only the context's device and stream (no ksg_set_cluster needed) and do
 * not touch its scheduling state. The caller orders each set's pods (creation
 * order for the capacity check) and interns node label pairs and nodeSelector
 * pairs in one id space (0 = a pair no node has). */
typedef struct ksg_admission_set {
  int64_t cap_milli_cpu;  /* CapacityFromMachineInfo (kubelet/util.go:48-58): NumCores*1000 */
  int64_t cap_memory;     /* ... MemoryCapacity (bytes); 0 = unlimited, as in the reference */
  uint32_t pod_off, n_pods;     /* this set's pods: pods[pod_off, pod_off + n_pods)   */
  uint32_t label_off, n_labels; /* the node's label pair ids: pairs[label_off, ...)   */
} ksg_admission_set;

#define KSG_ADMIT_OK 0
#define KSG_ADMIT_NODESELECTOR 1  /* "nodeSelectorMismatching" (kubelet.go:1757-1763) */
#define KSG_ADMIT_CAPACITY 2      /* "capacityExceeded" (kubelet.go:1765-1770)        */

/* CheckPodsExceedingCapacity per set, greedy in the given order: fits[i] = 1
 * (fitting) or 0 (notFitting); only fitting pods accumulate. */
int ksg_check_pods_exceeding_capacity(ksg_ctx* ctx, const ksg_admission_set* sets, uint32_t n_sets,
                                      const ksg_pod* pods, uint32_t n_pods, uint8_t* fits);
/* PodMatchesNodeLabels: matches[i] = 1 iff every nodeSelector pair of pod i
 * (ids[sel_off, sel_off + n_sel)) is one of its set's node label pairs. */
int ksg_pod_matches_node_labels(ksg_ctx* ctx, const ksg_admission_set* sets, uint32_t n_sets,
                                const ksg_pod* pods, uint32_t n_pods, const uint32_t* ids, uint32_t n_ids,
                                const uint32_t* pairs, uint32_t n_pairs, uint8_t* matches);
/* Both, in the kubelet's order: codes[i] = KSG_ADMIT_NODESELECTOR for a pod
 * whose selector does not match, else the capacity check over the matching pods
 * only (KSG_ADMIT_CAPACITY or KSG_ADMIT_OK). */
int ksg_admit_pods(ksg_ctx* ctx, const ksg_admission_set* sets, uint32_t n_sets, const ksg_pod* pods,
                   uint32_t n_pods, const uint32_t* ids, uint32_t n_ids, const uint32_t* pairs, uint32_t n_pairs,
                   uint8_t* codes);

/* ---- extensions beyond this reference vintage ----
 * BASELINE.json's configs name node taints / pod tolerations, extended (scalar)
 * resources and BalancedResourceAllocation. smarterclayton/kubernetes v0.13 has
 * none of them, so their semantics follow the published later kube-scheduler
 * (v1.10: algorithm/predicates PodToleratesNodeTaints and PodFitsResources'
 * ScalarResources, priorities TaintTolerationPriority + NormalizeReduce and
 * BalancedResourceAllocation) and PARITY IS UNPINNED (no reference to run or
 * table to check against; the C restatement oracle/ksg_oracle.c is the checker).
 * Off unless ksg_set_extensions enables them. On a node-sharded context the node
 * state is replicated as usual and TaintTolerationPriority's NormalizeReduce max
 * (over every shard's filtered nodes) is all-reduced (max) before the scores, per
 * window on the window path and per pod on the per-pod path. Batches take the
 * speculative-window path (otherwise the exact one-pod-at-a-time kernels) unless
 *   - a pod's extended-resource request is outside [0, 2^16], or
 *   - the config has a ServiceAntiAffinity priority and either extension score
 *     is on or a pod of the batch requests an extended resource (with both
 *     scores off and no requests the filters are static per (pod, node) and the
 *     anti-affinity window path takes them, round 6), or
 *   - TaintToleration scores (w_taint_toleration != 0) with max_taints > 64 (the
 *     window path counts a node's taints as one 64-bit mask),
 * on top of the window path's general conditions (ksg_set_window). The reference's
 * own predicates and priorities are unchanged. */
#define KSG_EXT_TAINTS (1u << 0) /* PodToleratesNodeTaints: NoSchedule / NoExecute taints */
#define KSG_EXT_SCALAR (1u << 1) /* extended resources: allocatable >= used + request    */
#define KSG_FAIL_TAINTS 8        /* fail codes after the reference's seven             */
#define KSG_FAIL_SCALAR 9
#define KSG_MAX_SCALAR 4         /* extended resource kinds (e.g. GPU counts)          */

typedef struct ksg_ext_config {
  uint32_t filters;            /* KSG_EXT_* bitmask                                     */
  int32_t w_taint_toleration;  /* TaintTolerationPriority weight (0 = off)              */
  int32_t w_balanced;          /* BalancedResourceAllocation weight (0 = off)           */
  uint32_t n_scalar;           /* extended resource kinds in use (<= KSG_MAX_SCALAR)    */
  uint32_t max_taints;         /* interned taint ids are < max_taints                   */
} ksg_ext_config;

/* Per pod, alongside its ksg_pod. The caller interns each distinct node taint
 * (key, value, effect) and lists the ones the pod's tolerations do NOT tolerate
 * (Toleration.ToleratesTaint: effect empty or equal, key empty or equal,
 * operator Exists or value equal): hard = effect NoSchedule or NoExecute,
 * soft = effect PreferNoSchedule against the tolerations whose effect is empty
 * or PreferNoSchedule. Lists are (offset, count) into the call's id array; each
 * list is a set (a taint id repeated in one list is rejected with KSG_ERR_ARG:
 * TaintTolerationPriority counts each untolerated taint of a node once). */
typedef struct ksg_pod_ext {
  int64_t scalar[KSG_MAX_SCALAR]; /* extended resource requests (0: not requested)   */
  uint32_t hard_off, n_hard;
  uint32_t soft_off, n_soft;
} ksg_pod_ext;

/* Enable extensions; call before ksg_set_cluster (every rank of a sharded
 * context alike; KSG_ERR_ARG for n_scalar > KSG_MAX_SCALAR). */
int ksg_set_extensions(ksg_ctx* ctx, const ksg_ext_config* ext);
/* Per node, after ksg_set_cluster: scalar_cap[r * n_nodes + n] = allocatable of
 * resource r (0: none), node n's taint ids taint_ids[taint_off[n], + taint_n[n]).
 * Resets the extended-resource usage (re-add pods with ksg_add_pod_ext). */
int ksg_set_node_ext(ksg_ctx* ctx, uint32_t n_nodes, const int64_t* scalar_cap, const uint32_t* taint_off,
                     const uint32_t* taint_n, const uint32_t* taint_ids, uint32_t n_taint_ids);
/* The pod-taking entry points with each pod's extension record (ext[i] goes
 * with pods[i]); the plain forms use an all-zero record. */
int ksg_add_pod_ext(ksg_ctx* ctx, uint32_t host_id, const ksg_pod* pod, const ksg_pod_ext* ext,
                    const uint32_t* ids);
int ksg_schedule_batch_ext(ksg_ctx* ctx, const ksg_pod* pods, const ksg_pod_ext* ext, uint32_t n,
                           const uint32_t* ids, uint32_t n_ids, uint64_t* rng_state, int32_t* out_nodes);
int ksg_schedule_begin_ext(ksg_ctx* ctx, const ksg_pod* pod, const ksg_pod_ext* ext, const uint32_t* ids,
                           int64_t* max_score, uint32_t* tie_count, uint8_t* fail_codes);
int ksg_evaluate_ext(ksg_ctx* ctx, const ksg_pod* pod, const ksg_pod_ext* ext, const uint32_t* ids,
                     uint8_t* fail_out, int64_t* score_out);
/* Copy the committed extended-resource usage back to the host, for state checks:
 * used[r * n_nodes + n] = the requests of resource r of every pod on node n
 * (the extended-resource counterpart of ksg_read_requested). */
int ksg_read_ext_used(ksg_ctx* ctx, int64_t* used);

#ifdef __cplusplus
}
#endif
#endif /* KSCHEDGPU_H_ */
