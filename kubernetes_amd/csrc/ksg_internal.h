// ksg_internal.h — layout shared by the host runtime (ksg_runtime.cpp) and the
// CDNA4 kernels (ksg_kernels.hip). Not part of the public ABI.
//
// HBM layout (all node-indexed arrays are indexed by node rank; bitmaps are
// node-major bit vectors of nw = ceil(N/64) uint64 words, bit n%64 of word n/64):
//
//   cap_cpu[N], cap_mem[N]        int64   static   node.Spec.Capacity (milli / bytes)
//   used_cpu[N], used_mem[N]      int64   mutable  sum of limits of ALL pods on node
//   static_fit[nw]                uint64  static   AND of LabelsPresence predicates
//   static_score[N]               int32   static   sum of w * score of pod-independent
//                                                  priorities (EqualPriority, LabelPreference)
//   keymap[K][nw]                 uint64  mutable  conflict key (host port / GCE PD) in use
//   pairmap[P][nw]                uint64  static   node carries label pair p (p=0: empty)
//   svc_cnt[S][N]                 int32   mutable  pods matching service s on node
//   svc_max[S], svc_total[S]      int32   mutable  ServiceSpreading maxCount / #pods
//   svc_peer[S]                   int32   mutable  first service peer's node (-1 none,
//                                                  -2 not a known node)
//   anti_domain[A][N]             int32   static   dense value index of anti label, -1
//   aff_pair[J][N]                int32   static   pair id of node's value of aff label j
#pragma once
#include <stdint.h>
#include "../../include/kschedgpu.h"

#define KSG_NT 1024          // threads of the single-workgroup scan kernels
#define KSG_NWAVE (KSG_NT / 64)

#define KSG_MODE_EVAL 0      // write fail codes + scores for every node
#define KSG_MODE_BEGIN 1     // write {M, k, tie words} record (+ optional fail codes)

// score sentinel for nodes that do not fit
#define KSG_SCORE_NONE (-0x7fffffffffffffffLL - 1)

struct KsgDev {
  // cluster geometry
  uint32_t n_nodes, nw;
  uint32_t lo, hi;            // evaluated node shard [lo, hi); lo % 64 == 0
  uint32_t wlo, nwords;       // shard's first word and word count
  uint32_t n_pairs, n_services, max_keys, n_domains_total;
  // config (compiled)
  uint32_t preds;
  int32_t w_lr, w_spread;
  uint32_t n_anti;
  int32_t w_anti[KSG_MAX_ANTI];
  uint32_t anti_dom_off[KSG_MAX_ANTI];
  uint32_t n_aff;
  int32_t equal_fallback;     // no priority configs: every fitting node scores 1
  int32_t empty_priorities;   // configs present but all weights 0: always FitError
  int32_t has_static_score;
  int32_t has_static_fit;
  // arrays
  const int64_t* cap_cpu;
  const int64_t* cap_mem;
  int64_t* used_cpu;
  int64_t* used_mem;
  const uint64_t* static_fit;
  const int32_t* static_score;
  uint64_t* keymap;
  const uint64_t* pairmap;
  int32_t* svc_cnt;
  int32_t* svc_max;
  int32_t* svc_total;
  int32_t* svc_peer;
  const int32_t* anti_domain;
  const int32_t* aff_pair;
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
  int32_t w_pref[KSG_MAX_LABEL_PREF];
  int32_t w_equal;
  uint32_t n_anti;
  uint32_t anti_key[KSG_MAX_ANTI];
  uint32_t n_aff;
  uint32_t aff_key[KSG_MAX_AFF];
};

// one record of the per-pod winner exchange (all-gathered across ranks)
struct KsgRecordHdr {
  int64_t max_score;   // KSG_SCORE_NONE if nothing fits in this shard
  uint64_t tie_count;  // nodes of this shard at max_score
  int32_t error;       // nonzero: pod errors (ServiceAffinity peer missing)
  int32_t pad;
  uint64_t pad2;
};
// followed by nwords_max uint64 tie words (bit set = node at max_score)

struct KsgPatch {
  uint64_t addr;   // device address
  uint64_t value;
  uint32_t width;  // op: 0 store32, 1 store64, 2 or64, 3 andnot64
  uint32_t pad;
};

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
