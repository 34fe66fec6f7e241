// ksg_internal.h — layout shared by the host runtime (ksg_runtime.cpp) and the
// CDNA4 kernels (ksg_kernels.hip). Not part of the public ABI.
//
// HBM layout (all node-indexed arrays are indexed by node rank; bitmaps are
// node-major bit vectors of nw = ceil(N/64) uint64 words, bit n%64 of word n/64):
//
//   cap_cpu[N], cap_mem[N]        int64   static   node.Spec.Capacity (milli / bytes)
//   inv10_cpu[N], inv10_mem[N]    f64     static   10.0 / capacity (window path's LeastRequested)
//   used_cpu[N], used_mem[N]      int64   mutable  sum of limits of ALL pods on node
//   static_fit[nw]                uint64  static   AND of LabelsPresence predicates
//   static_score[N]               int64   static   sum of w * score of pod-independent
//                                                  priorities (EqualPriority, LabelPreference)
//   keymap[K][nw]                 uint64  mutable  conflict key (host port / GCE PD) in use
//   pairmap[P][nw]                uint64  static   node carries label pair p (p=0: empty)
//   svc_cnt[S][N]                 int32   mutable  pods matching service s on node
//   svc_bits[S][nw]               uint64  mutable  svc_cnt[s][n] > 0
//   svc_max[S], svc_total[S]      int32   mutable  ServiceSpreading maxCount / #pods
//   svc_peer[S]                   int32   mutable  first service peer's node (-1 none,
//                                                  -2 not a known node)
//   anti_domain[A][N]             int32   static   dense value index of anti label, -1
//   aff_pair[J][N]                int32   static   pair id of node's value of aff label j
//                                                  (-1 none, KSG_AFF_INVALID: SelectorFromSet
//                                                  would reject the (key, value))
#pragma once
#include <stdint.h>
#include "../../include/kschedgpu.h"

#define KSG_NT 1024          // threads of the single-workgroup scan kernels
#define KSG_NWAVE (KSG_NT / 64)
#define KSG_R_LDS 32         // largest R whose per-node scores fit the LDS (R * 4 KiB)
#define KSG_R_MAX 128        // nodes per thread of the exact kernels: shards up to 131072 nodes

#define KSG_MODE_EVAL 0      // write fail codes + scores for every node
#define KSG_MODE_BEGIN 1     // write {M, k, tie words} record (+ optional fail codes)

// score sentinels for nodes that do not fit (int64 records / int32 LDS scores)
#define KSG_SCORE_NONE (-0x7fffffffffffffffLL - 1)
#define KSG_S32_NONE ((int32_t)0x80000000)
// combined scores: int32 on the window path, which the host takes only while no
// |score| can reach this bound; int64 and wrapping like Go's int on the exact
// kernels otherwise (KsgDev.wide)
#define KSG_SCORE_BOUND (1LL << 30)
// anti-affinity priorities whose node domains phase A keeps in registers (the
// rest, up to the policy's KSG_MAX_ANTI, are loaded where they are used)
#define KSG_WIN_MAX_ANTI 4
// largest capacity / requested total the window path accepts (lr_win's bound,
// ksg_device.h)
#define KSG_WIN_LR_BOUND (1LL << 49)
// largest extended resource request the window path takes (a window's deltas
// then fit int32: <= 4096 x 2^16)
#define KSG_WIN_XREQ_BOUND (1LL << 16)

struct KsgDev {
  // cluster geometry
  uint32_t n_nodes, nw;
  uint32_t lo, hi;            // evaluated node shard [lo, hi); lo % 64 == 0
  uint32_t wlo, nwords;       // shard's first word and word count
  uint32_t n_pairs, n_services, max_keys, n_domains_total;
  // config (compiled)
  uint32_t preds;
  int64_t w_lr, w_spread;
  uint32_t n_anti;
  int64_t w_anti[KSG_MAX_ANTI];
  uint32_t anti_dom_off[KSG_MAX_ANTI];
  uint32_t n_aff;
  uint32_t n_aff_groups;      // ServiceAffinity predicates (>= 1 when n_aff > 0)
  uint32_t aff_group_mask[KSG_MAX_AFF_GROUPS];  // aff labels of each predicate
  int32_t equal_fallback;     // no priority configs: every fitting node scores 1
  int32_t empty_priorities;   // configs present but all weights 0: always FitError
  int32_t has_static_score;
  int32_t has_static_fit;
  int32_t dbg;                // debug switches (KSG_DEBUG env), 0 in production
  int32_t wide;               // int64 combined scores (exact kernels only)
  uint32_t rr_dz;             // ServiceAntiAffinity re-rank: domain rows (0: off; ksg_window.hip)
  int32_t* dbgbuf;            // KSG_DEBUG & 4: per-pod resolver trace
  // arrays
  const int64_t* cap_cpu;
  const int64_t* cap_mem;
  const double* inv10_cpu;    // 10.0 / cap (0 if cap <= 0): lr_win's reciprocal, static
  const double* inv10_mem;
  int64_t* used_cpu;
  int64_t* used_mem;
  const uint64_t* draws;  // ksg_schedule_batch_draws: the caller's rand.Int() values (else splitmix64)
  const uint64_t* static_fit;
  const int64_t* static_score;
  uint64_t* keymap;
  const uint64_t* pairmap;
  int32_t* svc_cnt;
  uint64_t* svc_bits;         // [S][nw] node holds pods of service s (svc_cnt > 0): phase A
                              // loads a count only where its bit is set
  int32_t* svc_max;
  int32_t* svc_total;
  int32_t* svc_peer;
  const int32_t* anti_domain;
  const int32_t* aff_pair;
  void* score_scratch;        // exact kernels with R > the LDS bound: per-node scores in HBM, not LDS
  // extensions beyond the reference (ksg_set_extensions; exact kernels only, parity unpinned)
  uint32_t ext_filters;       // KSG_EXT_*
  int32_t w_taint, w_bal;     // TaintTolerationPriority, BalancedResourceAllocation weights
  uint32_t n_scalar;          // extended resource kinds
  const int64_t* scalar_cap;  // [n_scalar][N] allocatable
  int64_t* scalar_used;       // [n_scalar][N] requested by the pods on the node (mutable)
  const uint64_t* taintmap;   // [max_taints][nw] nodes carrying taint t
  // per node, its taint ids as a bitmask (max_taints <= 64; else nullptr): the window
  // path's TaintToleration term counts a pod's untolerated soft taints as one popcount
  const uint64_t* ntaint;
};

// static-table configuration (LabelsPresence, EqualPriority, LabelPreference,
// anti-affinity and ServiceAffinity label keys)
struct KsgStaticCfg {
  uint32_t n_presence;
  uint32_t presence_n_keys[KSG_MAX_PRESENCE];
  uint32_t presence_keys[KSG_MAX_PRESENCE][KSG_MAX_PRESENCE_KEYS];
  uint32_t presence_flag[KSG_MAX_PRESENCE];
  uint32_t n_pref;
  uint32_t pref_key[KSG_MAX_LABEL_PREF];
  uint32_t pref_presence[KSG_MAX_LABEL_PREF];
  int64_t w_pref[KSG_MAX_LABEL_PREF];
  int64_t w_equal;
  uint32_t n_anti;
  uint32_t anti_key[KSG_MAX_ANTI];
  uint32_t n_aff;
  uint32_t aff_key[KSG_MAX_AFF];
};

// window path, phase A output per pod (see ksg_window.hip). Everything phase B
// needs for one pod in one 192-byte record, so the sequential resolver streams
// one record per pod instead of chasing the pod descriptor and id lists.
#define KSG_WIN_INLINE 24
#define KSG_WIN_SUM_AFF 4
struct KsgWinSum {
  int32_t m0;          // best combined score at the snapshot (KSG_S32_NONE: nothing fits)
  uint32_t k0;         // nodes at m0 (bits of the pod's T0 bitmap)
  int32_t error;       // ServiceAffinity peer on an unknown node
  int32_t service;     // primary service
  int32_t host;        // PodFitsHost target
  int32_t spread_max;  // svc_max[primary] at the snapshot
  int32_t svc_total;   // svc_total[primary] at the snapshot
  uint32_t n_inline;   // total list entries; > KSG_WIN_INLINE: lists read from pods/ids
  int64_t milli_cpu;
  int64_t memory;
  int32_t req_aff[KSG_WIN_SUM_AFF];  // resolved ServiceAffinity pairs (the first KSG_WIN_SUM_AFF; unread by the resolvers)
  uint16_t n_ports, n_pds, n_sel, n_svcs;
  uint32_t xmask;      // extensions: the extended resource kinds the pod requests (bit r: scalar[r] > 0)
  uint32_t ids[KSG_WIN_INLINE];  // ports, pds, sel, svcs (in that order)
  int32_t xreq[4];     // extensions: the extended resource requests (the window path takes <= 2^16)
  uint32_t pad2;
};
static_assert(sizeof(KsgWinSum) == 192, "KsgWinSum layout");
#define KSG_WIN_SUM_DWORDS (sizeof(KsgWinSum) / 4)

// Where the resolver finds phase A's per-word results (ksg_window.hip). Phase A
// on each rank writes one block for its shard: best-score bitmaps
// uint64[wcap][ostride], then best scores int32[wcap][ostride] (then, with
// ServiceAntiAffinity, fit bitmaps uint64[wcap][ostride] at fit_off), row =
// window pod, column = word of the shard. With world > 1 the blocks are all-gathered
// rank-major (block g at buf + g * blk); global word w lives in the block of
// the rank whose [wlo, wlo + nw) holds it.
#define KSG_MAX_WORLD 16
struct KsgWinXchg {
  const uint8_t* buf;
  uint64_t blk;       // bytes per rank block
  uint32_t ostride;   // words per row (>= every shard's word count)
  uint32_t wcap;      // rows per block (window capacity)
  uint32_t world;
  uint32_t fit_off;   // ServiceAntiAffinity: byte offset in a block of the fit bitmaps
                      // uint64[wcap][ostride] (nodes the pod fits at the snapshot), else 0
  uint32_t wlo[KSG_MAX_WORLD], nw[KSG_MAX_WORLD];
  // ServiceAntiAffinity: the window's per-(pod, domain) counts the count pass
  // accumulates; the resolver zeroes them for the next window's count pass (its
  // score pass has read them), so no per-window fill is enqueued
  int32_t* dcnt;
  uint32_t dcnt_n;
  // ServiceAntiAffinity re-rank (one anti priority, one rank): a pod whose
  // service had commits earlier in the window is re-ranked per label domain
  // instead of ending the window. Phase A's count pass also writes, per (pod,
  // domain row), the best score without the anti term over the pod's filtered
  // nodes (dmb, int32[wcap][dz]; row dz-1 = unlabelled nodes), and the score pass
  // the bitmap of filtered nodes at their row's best (uint64[wcap][ostride] at
  // b_off) and how many of them each row holds (dmb's second half, int32[wcap][dz]);
  // zmap = uint64[dz][nw], the nodes of each domain row. The resolver resets the row
  // bests to KSG_S32_NONE and the counts to 0 for the next window.
  // the plain resolver (no ServiceAntiAffinity): per window pod, its T0 image
  // (ksg_plain.hip, ksg_win_t0_kernel) at img + pod * img_stride
  uint8_t* img;
  // extensions (taints, extended resources; scoring extensions off): the batch's
  // ksg_pod_ext records (pod pos + i of the window at exts[pos + i]), else nullptr
  const ksg_pod_ext* exts;
  uint32_t img_stride;
  // extensions with scores (TaintToleration / BalancedAllocation on the window path):
  // esc != 0; phase A also writes each pod's fit bitmap (uint64[wcap][ostride] at efit_off
  // in a block: non-T0 committed nodes whose score may rise need "fit at the snapshot"),
  // its untolerated soft taints as a mask (psoft[pod]) and, in the count pass, the
  // TaintToleration normalisation max over its filtered nodes (tmax[pod], zeroed by the
  // resolver for the next window)
  uint32_t esc;
  uint32_t efit_off;
  // the plain resolver without extensions, shards of up to 4 x 64 node words per lane
  // (16,384 nodes): d1 != 0, phase A also writes per (pod i, word) the bitmap of the nodes that
  // would stop scoring as they do (drop) for pod i if pod i-1 were committed there as the
  // node's first commit of the window (uint64[wcap][ostride] at d1_off in a block); the
  // committer answers "does commit i-1's node drop for pod i" from it for such a node
  // (ksg_plain.hip, x_fast)
  uint32_t d1;
  uint32_t d1_off;
  int32_t* tmax;
  uint64_t* psoft;
  // ... and the count pass's histogram of the pods' soft-taint counts over their filtered
  // nodes (int32[wcap][KSG_TBINS]): thist[pod][tmax] nodes hold the max, so the max falls
  // only once that many committed nodes at it stopped fitting (zeroed like tmax)
  int32_t* thist;
  uint32_t rr;        // re-rank on (else a service's commit ends the window)
  uint32_t dz;        // domain rows: anti domains + 1 (<= KSG_RR_MAXZ)
  uint32_t b_off;     // byte offset in a block of the best-per-domain bitmaps
  int32_t* dmb;
  const uint64_t* zmap;
};
#define KSG_TBINS 65       // soft-taint counts 0..64 (taint ids < 64 on the window path)
#define KSG_RR_MAXZ 32     // domain rows the re-rank handles (one lane each)
#define KSG_RR_MAXSVC 4096 // services (an LDS count per service)

// Device-side progress of a chain of windows (ksg_window.hip): the host enqueues
// several windows back to back and each kernel reads where the previous one
// stopped, so there is no host round trip between windows.
#define KSG_HALT_OVERSIZE 4  // pod `pos` needs the exact per-pod path
#define KSG_HALT_BADCOUNT 8  // resolver reported an impossible count (a bug)
#define KSG_HALT_HANG 9      // a ring/draw wait timed out (a bug)
#define KSG_HALT_BAD 10      // the resolver's selection left T0 / the shard (KSG_STOP_BAD)
struct KsgWinRun {
  uint32_t pos;       // first pod of the next window
  uint32_t n;         // pods in the batch
  uint32_t halt;      // KSG_HALT_*: later windows of the chain do nothing
  uint32_t windows;   // windows resolved
  uint32_t stops[4];  // windows ended early, by stop reason 1..3
};

// The fused window launch (ksg_plain.hip, ksg_win_plain_kernel<..., FUSED>): one
// launch per window instead of phase A + T0 images + resolver. Block 0 resolves
// the window; blocks 1.. score it (ksg_score.h, outputs write-through) in pod-group
// order, and after each (pod group, word group) task add 1 to cnt[set][group][xcd
// shard]; a resolver producer waits for the 8 shards of its pod's group to sum to
// the word groups, then builds the pod's T0 image itself. The run record has two
// slots: launch k reads slot k & 1 and its block 0 writes the outcome into slot
// (k + 1) & 1 (a scoring block still starting up never reads the window's own
// outcome), and zeroes counter set (k + 1) & 1 for launch k + 1.
struct KsgFused {
  const ksg_pod* batch;  // the batch's pods and id lists (device)
  const uint32_t* ids;
  KsgWinRun* run_out;    // slot (k + 1) & 1
  uint32_t* cnt;         // uint32[2][ngroups][8]
  uint32_t set;          // k & 1
  uint32_t ngroups;      // counter rows per set (>= pod groups in a window)
};

// one record of the per-pod winner exchange (all-gathered across ranks)
typedef ksg_shard_record KsgRecordHdr;  // public layout (include/kschedgpu.h)
// followed by nwords_max uint64 tie words (bit set = node at max_score)

// ksg_admit_kernel modes (ksg_admit.hip)
#define KSG_ADMIT_MODE_CAPACITY 1
#define KSG_ADMIT_MODE_SELECTOR 2

struct KsgPatch {
  uint64_t addr;   // device address
  uint64_t value;
  uint32_t width;  // op: 0 store32, 1 store64, 2 or64, 3 andnot64
  uint32_t pad;
};

// ---- the resident drop-in server (ksg_serve.hip) ---------------------------
// ksg_schedule_begin / ksg_schedule_commit talk to one resident workgroup
// through pinned, host-coherent memory mapped into the device (KsgSrvBox): no
// kernel launch, copy or stream synchronisation per call.
//
// Request block: KSG_SRV_CHUNKS chunks of 16 B that the server reads with ONE
// 16-B-per-lane wave load per poll. Dwords 0..2 of a chunk carry data, dword 3
// the request's sequence number (its tag). The host writes every data dword,
// then every tag; x86 stores become visible in program order and a 16-B read
// is one PCIe read, so a chunk whose tag matches was read after its data (and
// after the `ext` payload) landed. Data dwords, in order: the header
// (KSG_SRV_HDR_DW), then the payload's first KSG_SRV_INLINE_DW dwords; the
// rest of the payload is at `ext`, read once the block matched. Payload: the
// ksg_pod, its id list, its ksg_pod_ext (extensions).
#define KSG_SRV_CHUNKS 64
#define KSG_SRV_CHUNK_DW 3
#define KSG_SRV_HDR_DW 8
#define KSG_SRV_INLINE_DW (KSG_SRV_CHUNKS * KSG_SRV_CHUNK_DW - KSG_SRV_HDR_DW)
#define KSG_SRV_EXT_DW 4096
#define KSG_SRV_PAY_DW (KSG_SRV_INLINE_DW + KSG_SRV_EXT_DW)
#define KSG_SRV_PATCHES 4096
#define KSG_SRV_MAX_R 16  // nodes per thread the server takes (shards up to 16384 nodes)
enum {
  KSG_SRV_BEGIN = 1,   // scan the payload's pod: its tie words into `ties`, then respond
                       // {seq, k | ~0u on error, max lo, max hi} (the grid server: `part`, below)
  KSG_SRV_COMMIT = 2,  // AssumePod of the payload's pod on node `arg` (the host picked it from the
                       // begin's tie words): {seq, node}; not waited for by the host
  KSG_SRV_PATCH = 3,   // apply `n_patch` patches from `patch` in order, reload cached totals: {seq}
  KSG_SRV_EXIT = 4,    // respond {seq} and return
};
// header dwords
// ARG: COMMIT the node; BEGIN the last control request posted before it (its scan waits until
// that one is applied: the grid server's scan workgroups)
enum { KSG_SRVH_KIND = 0, KSG_SRVH_ARG, KSG_SRVH_RSV, KSG_SRVH_FLAGS, KSG_SRVH_PAYDW, KSG_SRVH_IDS_AT,
       KSG_SRVH_EXT_AT, KSG_SRVH_NPATCH };
#define KSG_SRV_BADREQ 0xFFFFFFFEu  // response: the payload's layout, ids or node are out of range
#define KSG_SRV_RESP_REJECTED 12  // resp[12]: the last request answered KSG_SRV_BADREQ (sticky; written first)
#define KSG_SRVF_WANT_FAIL 1u  // BEGIN: write the fail code of every node to `fail`
#define KSG_SRVF_EXT 2u        // the payload carries a ksg_pod_ext at EXT_AT
// The grid server (ksg_serve_grid_kernel): a leader workgroup plus one scan
// workgroup per 256 nodes. Each scan workgroup reads a BEGIN from the host
// block itself, scans its nodes and writes its part (best score, count, tie
// words; fail codes into `fail`) straight into host memory, the sequence number
// last; the host merges the parts. The leader serves COMMIT / PATCH / EXIT and
// answers each once it is applied, so a BEGIN posted after that answer scans
// the state it left.
#define KSG_GSRV_NT 256
#define KSG_GSRV_MAXW 255  // scan workgroups: shards up to 65,280 nodes (261,120 at 4 nodes per thread)
#define KSG_GSRV_TIEW 16   // tie words of a scan workgroup at 4 nodes per thread
#define KSG_GSRV_MAXD 64   // ServiceAntiAffinity label domains (all anti priorities) the grid server takes
struct alignas(64) KsgSrvPart {
  uint32_t seq;     // the BEGIN this part answers (its 16-B store comes last)
  int32_t max;      // best score over the workgroup's nodes (KSG_S32_NONE: none fits)
  uint32_t cnt;     // its nodes at max
  uint32_t err;     // 1: the pod's ServiceAffinity peer is on an unknown node; 2: a bad request
  uint64_t tie[4];  // its nodes at max, one word per 64
  uint32_t stamp[4];  // KSG_SERVE_STAMPS wall-clock ticks: request seen, masks + loads done, stored; then seq again
};
// Two request blocks: `req` (+ `ext`) carries BEGIN, `creq` (+ `cext`) the control
// requests COMMIT / PATCH / EXIT, so the host posts the next BEGIN while the server
// may still be reading a COMMIT. Sequence numbers count both.
struct KsgSrvBox {
  uint32_t req[KSG_SRV_CHUNKS * 4];
  uint32_t creq[KSG_SRV_CHUNKS * 4];
  uint32_t cext[KSG_SRV_EXT_DW];
  uint32_t resp[16];  // {seq, a, b, c}: one 16-B store
  uint32_t ext[KSG_SRV_EXT_DW];
  KsgPatch patch[KSG_SRV_PATCHES];
  uint32_t dbg[256];  // KSG_SERVE_DEBUG: the last stage each workgroup of the server reached (seq << 8 | stage)
  uint64_t ties[KSG_SRV_MAX_R * 16];  // the one-workgroup server's tie words of the last BEGIN
  KsgSrvPart part[KSG_GSRV_MAXW];     // the grid server's parts of the last BEGIN
  uint64_t part_tie[KSG_GSRV_MAXW * KSG_GSRV_TIEW];  // ... their tie words at 4 nodes per thread
};
struct KsgSrvGrid {
  uint32_t quit;     // == the launch's epoch: the scan workgroups return
  uint32_t applied;  // the last control request the leader applied (a BEGIN waits for its ARG)
  uint32_t pad[14];
  // (extensions) TaintToleration: each scan workgroup's max untolerated soft-taint count over its
  // filtered nodes, tagged with the BEGIN's sequence number (seq << 32 | max): every workgroup
  // reads all of them (the normalisation max over the whole shard) before it scores
  uint64_t tmx[KSG_GSRV_MAXW];
  // ServiceAntiAffinity: each scan workgroup's counts of the pod's service pods on its filtered
  // labelled nodes, per domain, tagged likewise ([workgroup][domain]: seq << 32 | count)
  uint64_t dcx[KSG_GSRV_MAXW * KSG_GSRV_MAXD];
};
struct KsgSrvArgs {
  KsgSrvBox* box;        // device address of the mapped box
  uint8_t* fail;         // device address of the mapped fail-code area (shard nodes)
  uint32_t start_seq;    // the server serves start_seq + 1, + 2, ...
  uint64_t idle_ticks;   // returns after this long without a request (wall_clock64: 100 MHz)
  uint32_t stamps;       // bit 0, KSG_SERVE_STAMPS: per-stage s_memtime cycles of each BEGIN in resp[4..9];
                         // bit 1, KSG_SERVE_DEBUG: stage markers in box->dbg
  KsgSrvGrid* grid;      // the grid server's device state (nullptr: the one-workgroup server)
  uint32_t n_workers;    // its scan workgroups
  uint32_t epoch;        // its launch number
  uint32_t grid_opts;    // scan workgroups' polling: bits 0-7 extra sleeps, KSG_GSRV_POLL1
};
#define KSG_GSRV_POLL1 256u  // poll chunk 0 alone until its tag moves

#ifdef __HIP__
#define KSG_HD __host__ __device__
#else
#define KSG_HD
#endif

// Tie-break source: splitmix64; Int63() = next() >> 1.
static inline KSG_HD uint64_t ksg_splitmix_next(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
// ... or the caller's own rand.Int() values, drawn ahead (ksg_schedule_batch_draws):
// the state is then the index of the next value. state advance per draw:
static inline KSG_HD uint64_t ksg_rng_step(const uint64_t* draws) { return draws ? 1ULL : 0x9E3779B97F4A7C15ULL; }
// the draw at state s (the state before it): rand.Int() (generic_scheduler.go:94)
static inline KSG_HD uint64_t ksg_rng_draw(const uint64_t* draws, uint64_t s) {
  if (draws) return draws[s];
  return ksg_splitmix_next(&s) >> 1;
}
