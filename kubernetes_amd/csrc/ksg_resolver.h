// ksg_resolver.h — pieces shared by the window path's in-order resolvers
// (phase B): the resolver record's dword offsets, the ring and slot records,
// the LDS polling primitives, the drop tests against a committed node, and the
// select helpers. Included by ksg_window.hip (phase A, the anti-affinity
// resolvers) and ksg_plain.hip (the resolver of every other configuration).
#pragma once
#include "ksg_device.h"

#include <algorithm>

// dword offsets inside KsgWinSum (lane j of the resolver holds dword j)
#define WS_ERR 2
#define WS_SVC 3
#define WS_HOST 4
#define WS_SMAX 5
#define WS_STOT 6
#define WS_NINL 7
#define WS_CPU 8
#define WS_MEM 10
#define WS_AFF 12
#define WS_NPP 16
#define WS_NSS 17
#define WS_XM 18   // extended resource kinds the pod requests (extensions)
#define WS_IDS 19
#define WS_XREQ 43 // its extended resource requests (4 dwords)

// threads of the resolver workgroup: 8 waves
// (16 waves for P <= 8 measured no faster than 8: the chain, not the producers, limits)
__host__ __device__ constexpr uint32_t win_res_nt(uint32_t P) { return P <= 8 ? 512u : 512u; }
#define KSG_RES_C0 2                                  // first checker wave (0: committer, 1: scribe)
#define KSG_RES_NCHK 2                                // checker waves
#define KSG_RES_P0 (KSG_RES_C0 + KSG_RES_NCHK)        // first producer wave
#define KSG_RES_NPW (KSG_RES_NT / 64 - KSG_RES_P0)    // producer waves (KSG_RES_NT: in the kernel)
// ring entries: 16, or 4 when the T0 words of an entry are large (P > 8: more than 32k nodes)
__host__ __device__ constexpr uint32_t win_ring(uint32_t P) { return P <= 8 ? 16u : 4u; }
// the register-slot resolver without ServiceAntiAffinity: an entry holds T0 (8 B)
// and its in-row prefixes (2 B) per word, so larger shards keep a longer ring
__host__ __device__ constexpr uint32_t win2_ring(uint32_t P, bool anti) {
  return anti || P <= 8 ? win_ring(P) : P == 16 ? 8u : 5u;
}
// Shards past 32k nodes (P > 8): the re-rank's per-domain node bitmaps (one P * 512 B bitmap per
// domain row) are read from their HBM copy (x.zmap, L2-resident: rows x words x 8 B) instead of
// LDS; past 64k nodes (P > 16) the pod's fit-at-the-snapshot and best-per-row (B) bitmaps are
// read from phase A's output rows (x.buf, one row per window pod) instead of ring copies. T0 and
// the drop bitmap stay in LDS (the committer reads them every pod).
__host__ __device__ constexpr bool win2_zg(uint32_t P) { return P > 8; }
__host__ __device__ constexpr bool win2_zg_words(uint32_t nwords) { return nwords > 8 * 64; }  // (P > 8)
__host__ __device__ constexpr bool win2_fg(uint32_t P) { return P > 16; }
#define KSG_SLOT_KEYS 8
#define KSG_SLOT_SVCS 12
#define KSG_MAX_SLOTS (64 * KSG_RES_NCHK)
#define KSG_NO_SLOT 0xffffu
#define KSG_NO_NODE 0xffffffffu

struct alignas(16) I64x2 {
  int64_t c, m;
};
struct alignas(16) F64x2 {
  double c, m;
};
struct alignas(16) SlotMeta {
  uint32_t node;    // shard offset of the node
  uint32_t nk, ns;  // conflict keys / service entries added by the window
  uint32_t smask;   // OR of 1 << (service & 31) over the service entries
};
struct alignas(16) RingHdr {
  int32_t m0;
  uint32_t k0;
  uint64_t r;          // Int63 draw of the pod
  uint32_t ready;      // pod index + 1 once the entry is complete
  uint32_t drawable;
  int32_t pred;        // (r mod k0)-th tie of T0 from the top (shard offset), -1: none
  uint32_t pad;
  int64_t cap_c, cap_m, used_c, used_m;  // snapshot of pred
  double inv_c, inv_m;                   // 10 / capacity of pred
  uint64_t psoft;                        // (extension scores) the pod's untolerated soft taints (mask)
  int32_t tmax;                          // ... its TaintToleration max over its filtered nodes
  int32_t tcnt;                          // ... and how many of them hold it
  // (plain resolver) the pod's scalars the committer branches on, staged so its head reads two
  // words instead of the record's lanes: the service, and flags -- bit 0 no draw (error / nothing
  // fit), 1 the previous pod is of this pod's service, 2 lists longer than the record / a slot,
  // bits 8..15 conflict keys, 16..23 services, 24..31 selector pairs (each capped at 255)
  int32_t ps;
  uint32_t pfl;
};
struct alignas(16) RingSvc {  // per service entry t of the pod (t < n_svcs)
  int32_t cnt[KSG_SLOT_SVCS];   // svc_cnt[sv][pred] at the snapshot
  int32_t max[KSG_SLOT_SVCS];   // svc_max[sv]
  int32_t peer[KSG_SLOT_SVCS];  // svc_peer[sv]
  int32_t pad[4];
};
struct alignas(16) WinCtl {
  uint32_t consumed;    // pods the committer is done with (ring entries free)
  uint32_t stop;        // the window ended early: every other wave exits
  uint32_t draw_next;   // next pod allowed to take a draw index
  uint32_t draw_count;  // draws of pods [0, draw_next)
  uint32_t sel_seq;     // pods the committer has selected a node for
  uint32_t xs_slot;     // slot the last selected pod commits into (KSG_NO_SLOT: none)
  uint32_t xs_nslots;   // slots in use once that pod is committed
  uint32_t pad0;
  uint32_t chk_seq[KSG_RES_NCHK];     // pods checker c is done with
  uint32_t chk_cnt[KSG_RES_NCHK][2];  // checker c's drops for the pod of parity p
  uint32_t chk_stop[KSG_RES_NCHK][2]; // checker c: the pod's anti-affinity domain counts changed
  uint32_t order_seq;                 // orders the committer has issued (one per pod)
  uint32_t scribe_done;               // orders the scribe has written into the slots
  uint32_t n_peer;                    // services given their first peer in the window
  uint32_t pad[1];
};
// One pod's outcome, handed from the committer to the scribe (two buffers, by
// pod parity). The scribe reads the pod itself from its ring entry.
struct alignas(16) WinOrder {
  uint32_t kind;     // 0: no commit (error / no fit), 1: commit
  uint32_t slot, node;
  int32_t out;       // placement (node rank or KSG_OUT_*)
  uint32_t e;        // ring entry of the pod
  uint32_t in_c;     // the slot existed before this commit
  uint32_t is_pred;  // the node is the producer's predicted node (its snapshot is staged)
  uint32_t pad;
};

// byte offsets of the resolver's dynamic LDS arrays (host and device agree)
struct WinLdsOff {
  uint32_t ctl, r_hdr, r_t0, r_rec, r_mod, r_svc, r_fit;  // ring
  uint32_t s_meta, s_cap, s_snp, s_dl, s_inv;          // slots
  uint32_t keys, svcs, scnt;
  uint32_t peer, out, flag, peerset, drop, ord;
  // re-rank (dz > 0): ring B words, per-row best scores and domain counts;
  // the domain rows' node words; window commits per service; the checkers'
  // per-row count additions by pod parity
  uint32_t r_b, r_mb, r_dc, zm, nsv, dca;
  uint32_t total;
};

__host__ __device__ constexpr uint32_t win_al16(size_t x) { return (uint32_t)((x + 15) & ~(size_t)15); }

__host__ __device__ inline WinLdsOff win_lds_offsets(uint32_t P, uint32_t nflag, uint32_t W, bool anti,
                                                     uint32_t dz = 0, uint32_t nsvc = 0) {
  WinLdsOff o;
  const uint32_t KSG_RING = win_ring(P);
  uint32_t at = 0;
  o.ctl = at;     at += win_al16(sizeof(WinCtl));
  o.r_hdr = at;   at += win_al16((size_t)KSG_RING * sizeof(RingHdr));
  o.r_t0 = at;    at += win_al16((size_t)KSG_RING * P * 64 * 8);
  o.r_rec = at;   at += win_al16((size_t)KSG_RING * KSG_WIN_SUM_DWORDS * 4);
  o.r_mod = at;   at += win_al16((size_t)KSG_RING * 64 * 4);
  o.r_svc = at;   at += win_al16((size_t)KSG_RING * sizeof(RingSvc));
  // fit bitmaps (anti-affinity; past 64k nodes read from phase A's rows instead, win2_fg)
  o.r_fit = at;   at += anti && !win2_fg(P) ? win_al16((size_t)KSG_RING * P * 64 * 8) : 0u;
  o.s_meta = at;  at += win_al16((size_t)KSG_MAX_SLOTS * sizeof(SlotMeta));
  o.s_cap = at;   at += win_al16((size_t)KSG_MAX_SLOTS * sizeof(I64x2));
  o.s_snp = at;   at += win_al16((size_t)KSG_MAX_SLOTS * sizeof(I64x2));
  o.s_dl = at;    at += win_al16((size_t)KSG_MAX_SLOTS * sizeof(I64x2));
  o.s_inv = at;   at += win_al16((size_t)KSG_MAX_SLOTS * sizeof(F64x2));
  o.keys = at;    at += win_al16((size_t)KSG_MAX_SLOTS * KSG_SLOT_KEYS * 4);
  o.svcs = at;    at += win_al16((size_t)KSG_MAX_SLOTS * KSG_SLOT_SVCS * 4);
  o.scnt = at;    at += win_al16((size_t)KSG_MAX_SLOTS * KSG_SLOT_SVCS * 4);
  o.peer = at;    at += win_al16((size_t)W * 2 * 4);
  o.out = at;     at += win_al16((size_t)W * 4);
  o.flag = at;    at += win_al16((size_t)nflag * 4);
  o.peerset = at; at += win_al16((size_t)nflag * 4);
  o.drop = at;    at += win_al16((size_t)2 * P * 64 * 8);
  o.ord = at;     at += win_al16((size_t)2 * sizeof(WinOrder));
  o.r_b = at;     at += dz ? win_al16((size_t)KSG_RING * P * 64 * 8) : 0u;
  o.r_mb = at;    at += dz ? win_al16((size_t)KSG_RING * KSG_RR_MAXZ * 4) : 0u;
  o.r_dc = at;    at += dz ? win_al16((size_t)KSG_RING * KSG_RR_MAXZ * 4) : 0u;
  o.zm = at;      at += win_al16((size_t)dz * P * 64 * 8);
  o.nsv = at;     at += dz ? win_al16((size_t)nsvc * 4) : 0u;
  o.dca = at;     at += dz ? win_al16((size_t)KSG_RES_NCHK * 2 * KSG_RR_MAXZ * 4) : 0u;
  o.total = at;
  return o;
}

#define KSG_STOP_SERVICE 1
#define KSG_STOP_EXHAUSTED 2
#define KSG_STOP_SLOT 3
#define KSG_STOP_OVERSIZE 4
#define KSG_STOP_HANG 9        // a ring/draw wait exceeded KSG_SPIN_LIMIT polls (a bug): the host fails
#define KSG_STOP_BAD 10        // a selection outside T0 / the shard (inconsistent prefixes or drop positions:
                               // a bug, or stale verdicts under the KSG_DEBUG timing switches): the host fails
#define KSG_SPIN_LIMIT (1u << 22)
// KSG_DEBUG bits that select a resolver's debug instantiation: 16..19 the per-role delay
// skews (interleaving tests), 24..27 the plain resolver's timing switches. Bits 20..23 are
// not resolver switches (22 / 23: the runtime's request-corruption hook for the resident
// server's rejection test), so setting them never changes which resolver build runs.
#define KSG_DBG_SKEW_MASK 0x000f0000u
#define KSG_DBG_RESOLVER_MASK 0x0f0f0000u

// a global-address-space load: global_load (vmcnt only), not flat_load, whose
// lgkmcnt share would make every later LDS wait also wait for it
template <typename T>
__device__ __forceinline__ T gld(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
__device__ __forceinline__ void lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
// the resolvers' rare exits (stops, hangs, error records): laid out off the hot path, so the
// common pod falls through without taken branches (each costs an instruction-buffer refill)
#define KSG_UNLIKELY(c) __builtin_expect(!!(c), 0)
__device__ __forceinline__ uint32_t ld_acq(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// a sequence post publishing data THIS wave wrote to LDS before it: the LDS runs one wave's
// instructions in issue order, so the data lands before the post without the release's
// lgkmcnt(0) wait (which also waits for every LDS read in flight: an LDS round trip on the
// chain). Readers poll with ld_rlx and read the data in the same round (in order too). A post
// that publishes global memory, or another wave's writes, takes st_rel. (-DKSG_POST_RELEASE:
// st_rel everywhere, for A/B runs)
__device__ __forceinline__ void st_post(uint32_t* p, uint32_t v) {
#ifdef KSG_POST_RELEASE
  st_rel(p, v);
#else
  asm volatile("" ::: "memory");  // (the compiler keeps the data stores ahead of the post)
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
}
// polling: relaxed LDS loads issue back to back under one lgkmcnt wait (an
// acquire load waits for each), then one LDS-only acquire once the wait is over
// (no vmcnt wait on the poller's loads in flight)
__device__ __forceinline__ uint32_t ld_rlx(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void acq_lds() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
// a polled word as a wave-uniform (scalar) value: the wait loops branch on
// SCC instead of juggling the exec mask
__device__ __forceinline__ uint32_t ld_u(uint32_t* p) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_rlx(p));
}

// The target-th set bit (ascending, 0-based) of the P-word-per-lane bitmap
// `bits` (lane l owns words l*P + q), given each lane's popcount `cl` and its
// inclusive prefix `incl`. Wave-uniform result: the word-major bit offset.
template <int P>
__device__ __forceinline__ uint32_t select_in_lanes(const uint64_t (&bits)[P], uint32_t cl, uint32_t incl,
                                                    uint32_t target, uint32_t lane) {
  const uint32_t excl = incl - cl;
  const int ol = (int)__builtin_ctzll(__ballot(excl <= target && target < incl));
  // the owner lane's words, in scalar registers; then the bit by mbcnt rank
  uint32_t local = target - (uint32_t)__builtin_amdgcn_readlane((int)excl, ol);
  uint64_t wsel = 0;
  uint32_t qsel = 0;
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const uint64_t wq = readlane64(bits[q], ol);
    const uint32_t pc = __popcll(wq);
    if (qsel == (uint32_t)q) {
      if (local < pc) {
        wsel = wq;
      } else {
        local -= pc;
        qsel = q + 1;
      }
    }
  }
  const uint32_t rank =
      __builtin_amdgcn_mbcnt_hi((uint32_t)(wsel >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wsel, 0u));
  const uint32_t bsel = (uint32_t)__builtin_ctzll(__ballot(((wsel >> lane) & 1ULL) && rank == local));
  return ((uint32_t)ol * P + qsel) * 64 + bsel;
}

// The same for a q-major bitmap (lane l holds words q*64 + l): given each
// lane's bits below it in row q (ex[q]) and the bits below each row (rowex,
// wave-uniform, ascending), the target-th set bit (ascending) as a bit offset.
template <int P>
__device__ __forceinline__ uint32_t select_qmajor(const uint64_t (&bits)[P], const uint32_t (&ex)[P],
                                                  const uint32_t (&rowex)[P], uint32_t target, uint32_t lane) {
  uint32_t qs = 0;
#pragma unroll
  for (int q = 1; q < P; ++q)
    if (rowex[q] <= target) qs = q;  // (an empty row has the next row's prefix)
  uint64_t w = 0;
  uint32_t e = 0, rb = 0;
#pragma unroll
  for (int q = 0; q < P; ++q)
    if ((uint32_t)q == qs) {
      w = bits[q];
      e = ex[q];
      rb = rowex[q];
    }
  const uint32_t loc = target - rb;
  const uint32_t ls = (uint32_t)__builtin_ctzll(__ballot(e <= loc && loc < e + (uint32_t)__popcll(w)));
  const uint64_t ws = readlane64(w, (int)ls);
  const uint32_t lw = loc - (uint32_t)__builtin_amdgcn_readlane((int)e, (int)ls);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(ws >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ws, 0u));
  const uint32_t bsel = (uint32_t)__builtin_ctzll(__ballot(((ws >> lane) & 1ULL) && rank == lw));
  return (qs * 64 + ls) * 64 + bsel;
}

// LDS views of the slots (structure of arrays by slot index)
struct WinSlots {
  SlotMeta* meta;
  I64x2 *cap, *snp, *dl;
  F64x2* inv;
  uint32_t* keys;
  uint32_t* svcs;
  int32_t* scnt;
};

// The pod-side inputs of a re-check (wave-uniform, read from the pod's record).
struct PodView {
  int64_t req_c, req_m;
  bool zero_req;
  uint32_t n_ports, n_pds, nk;
  int32_t s, smax;
  uint32_t xm;  // extended resource kinds requested (extensions; 0 otherwise)
};

// Does slot `sl` (a snapshot tie of the pod) score below M0 once the window's
// deltas are applied? The node fit the pod at the snapshot; only those deltas
// (requested totals, keys, service counts) can change that. `rec` is this
// lane's dword of the pod's record (the pod's key ids are read from it).
__device__ __forceinline__ bool slot_drops(const KsgDev& d, const WinSlots& S, uint32_t sl, const PodView& pv,
                                           uint32_t rec, bool res_on, bool ports_on, bool disk_on,
                                           bool spread_on) {
  const I64x2 cap = S.cap[sl], snp = S.snp[sl], dl = S.dl[sl];
  const SlotMeta me = S.meta[sl];
  const int64_t now_c = (int64_t)((uint64_t)snp.c + (uint64_t)dl.c);
  const int64_t now_m = (int64_t)((uint64_t)snp.m + (uint64_t)dl.m);
  bool drop = false;
  if (res_on && !pv.zero_req) {  // PodFitsResources (predicates.go:127-145)
    const bool fc = cap.c == 0 || cap.c - now_c >= pv.req_c;
    const bool fm = cap.m == 0 || cap.m - now_m >= pv.req_m;
    drop = !(fc && fm);
  }
  if (pv.nk && !drop && me.nk) {  // PodFitsPorts / NoDiskConflict against the window's keys
    const uint32_t* ks = S.keys + (size_t)sl * KSG_SLOT_KEYS;
    for (uint32_t a = 0; a < me.nk; ++a) {
      const uint32_t key = ks[a];
      if (ports_on)
        for (uint32_t b = 0; b < pv.n_ports; ++b)
          drop |= (uint32_t)__builtin_amdgcn_readlane(rec, WS_IDS + b) == key;
      if (disk_on)
        for (uint32_t b = 0; b < pv.n_pds; ++b)
          drop |= (uint32_t)__builtin_amdgcn_readlane(rec, WS_IDS + pv.n_ports + b) == key;
    }
  }
  if (!drop && d.w_lr) {  // LeastRequested (priorities.go:43-76) can only fall as requested grows
    const F64x2 iv = S.inv[sl];
    const int32_t lr_now = lr_win(now_c + pv.req_c, cap.c, iv.c) + lr_win(now_m + pv.req_m, cap.m, iv.m);
    const int32_t lr_snap = lr_win(snp.c + pv.req_c, cap.c, iv.c) + lr_win(snp.m + pv.req_m, cap.m, iv.m);
    drop = (lr_now >> 1) != (lr_snap >> 1);
  }
  if (!drop && spread_on && pv.s >= 0 && ((me.smask >> (pv.s & 31)) & 1u)) {
    // ServiceSpreading (spreading.go:72-86) under an unchanged maxCount
    const uint32_t* sv = S.svcs + (size_t)sl * KSG_SLOT_SVCS;
    const int32_t* sc = S.scnt + (size_t)sl * KSG_SLOT_SVCS;
    int32_t delta = 0, snapc = 0;
    for (uint32_t a = 0; a < me.ns; ++a)
      if (sv[a] == (uint32_t)pv.s) {
        snapc = sc[a];
        ++delta;
      }
    if (delta)
      drop = frac10_f32((int64_t)pv.smax - snapc - delta, pv.smax) != frac10_f32((int64_t)pv.smax - snapc, pv.smax);
  }
  return drop;
}

// ServiceAntiAffinity: a node the pod fitted at the snapshot that it no longer
// fits (the window's commits took its resources or a key) leaves the pod's
// filtered set; if the node is labelled and holds pods of the pod's service,
// the pod's per-domain counts and so the scores of a whole domain change
// (spreading.go:130-151): not a monotone change, the window must end there.
__device__ __forceinline__ bool anti_counts_move(const KsgDev& d, uint32_t node, int32_t s) {
  bool labelled = false;
  for (uint32_t a = 0; a < d.n_anti && !labelled; ++a)
    if (d.w_anti[a] != 0 && d.anti_domain[(size_t)a * d.n_nodes + d.lo + node] >= 0) labelled = true;
  return labelled && d.svc_cnt[(size_t)s * d.n_nodes + d.lo + node] > 0;
}

// The resource and key parts of the filter against slot sl's current state
// (the static parts cannot change in a window).
__device__ __forceinline__ bool slot_fits_now(const WinSlots& S, uint32_t sl, const PodView& pv, uint32_t rec,
                                              bool res_on, bool ports_on, bool disk_on) {
  const I64x2 cap = S.cap[sl], snp = S.snp[sl], dl = S.dl[sl];
  const int64_t now_c = (int64_t)((uint64_t)snp.c + (uint64_t)dl.c);
  const int64_t now_m = (int64_t)((uint64_t)snp.m + (uint64_t)dl.m);
  bool fit = true;
  if (res_on && !pv.zero_req)
    fit = (cap.c == 0 || cap.c - now_c >= pv.req_c) && (cap.m == 0 || cap.m - now_m >= pv.req_m);
  const uint32_t nk = S.meta[sl].nk;
  if (fit && pv.nk && nk) {
    const uint32_t* ks = S.keys + (size_t)sl * KSG_SLOT_KEYS;
    for (uint32_t a = 0; a < nk; ++a) {
      const uint32_t key = ks[a];
      if (ports_on)
        for (uint32_t b = 0; b < pv.n_ports; ++b) fit &= (uint32_t)__builtin_amdgcn_readlane(rec, WS_IDS + b) != key;
      if (disk_on)
        for (uint32_t b = 0; b < pv.n_pds; ++b)
          fit &= (uint32_t)__builtin_amdgcn_readlane(rec, WS_IDS + pv.n_ports + b) != key;
    }
  }
  return fit;
}

__device__ __forceinline__ PodView pod_view(uint32_t rec) {
  PodView pv;
  const uint32_t npp = __builtin_amdgcn_readlane(rec, WS_NPP);
  pv.req_c = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rec, WS_CPU) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rec, WS_CPU + 1) << 32));
  pv.req_m = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rec, WS_MEM) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rec, WS_MEM + 1) << 32));
  pv.zero_req = pv.req_c == 0 && pv.req_m == 0;
  pv.n_ports = npp & 0xffff;
  pv.n_pds = npp >> 16;
  pv.nk = pv.n_ports + pv.n_pds;
  pv.s = (int32_t)__builtin_amdgcn_readlane(rec, WS_SVC);
  pv.smax = (int32_t)__builtin_amdgcn_readlane(rec, WS_SMAX);
  pv.xm = (uint32_t)__builtin_amdgcn_readlane(rec, WS_XM);
  return pv;
}

// per-slot list table: [0, 8) conflict keys, [8, 20) service ids, [20, 32) the
// services' counts on the node at the snapshot (written by the owner checker).
// Row stride 36 dwords (144 B, 16-byte aligned): a checker wave reads its 64
// rows with ds_read_b128, whose 16-lane groups then start at 16 distinct
// multiples of 4 banks mod 64 and cover every bank once (a 32-dword stride put
// all 32 lanes of a ds_read_b32 group on one bank: a 32-way conflict per entry)
#define KSG_CL_KEY 0
#define KSG_CL_SV 8
#define KSG_CL_SC 20
#define KSG_CL_W 36

// A checker lane's slot row in registers: eight 16-byte LDS reads issued
// together, then the list scans run on registers (one dependent LDS read per
// list entry before)
struct SlotRow {
  uint32_t w[32];
  __device__ __forceinline__ void load(const uint32_t* row) {
    const uint4* p = reinterpret_cast<const uint4*>(row);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 q = p[k];
      w[4 * k] = q.x;
      w[4 * k + 1] = q.y;
      w[4 * k + 2] = q.z;
      w[4 * k + 3] = q.w;
    }
  }
  // the row's entries of service s among the first ns (cnt) and their snapshot count
  __device__ __forceinline__ void svc(uint32_t ns, uint32_t s, int32_t& snapc, int32_t& cnt) const {
    snapc = 0;
    cnt = 0;
#pragma unroll
    for (int a = 0; a < KSG_SLOT_SVCS; ++a)
      if ((uint32_t)a < ns && w[KSG_CL_SV + a] == s) {
        snapc = (int32_t)w[KSG_CL_SC + a];
        ++cnt;
      }
  }
  // PodFitsPorts / NoDiskConflict: one of the pod's keys (record lanes WS_IDS..) among the
  // row's first nk keys
  __device__ __forceinline__ bool key_hit(uint32_t nk, uint32_t rec, uint32_t pod_nk, uint32_t n_ports, bool ports_on,
                                          bool disk_on) const {
    bool hit = false;
    for (uint32_t b = 0; b < pod_nk; ++b) {
      if (!(b < n_ports ? ports_on : disk_on)) continue;
      const uint32_t kb = (uint32_t)__builtin_amdgcn_readlane((int)rec, (int)(WS_IDS + b));
#pragma unroll
      for (int a = 0; a < KSG_SLOT_KEYS; ++a) hit |= (uint32_t)a < nk && w[KSG_CL_KEY + a] == kb;
    }
    return hit;
  }
};

// One slot in a checker lane's registers.
struct RegSlot {
  uint32_t node;  // shard offset; ~0u: the lane owns no slot yet
  int64_t cap_c, cap_m, snp_c, snp_m, dl_c, dl_m;
  double inv_c, inv_m;
  uint32_t nk, ns, smask;  // list lengths as of the commits this checker applied
  uint32_t row;            // (ServiceAntiAffinity re-rank) the node's domain row, ~0u unlabelled
  uint32_t xk;             // (extensions) extended resource kinds the window's commits requested here
  int32_t xh[4];           // (extensions) allocatable - requested at the snapshot, clamped to int32
  int32_t xdl[4];          // (extensions) the window's requests here (<= 4096 x 2^16)
  int32_t sst;             // (extension scores) the node's static score
  uint64_t ntm;            // (extension scores) the node's taints (mask)
};

// Extension scores on the window path (BalancedAllocation can RISE on a committed
// node; TaintToleration's term is static per (pod, node) while its normalisation
// max holds): the change of a committed node's score for a pod between the
// snapshot and now. The static and TaintToleration terms cancel; LeastRequested,
// ServiceSpreading (frac_* = the spreading scores) and BalancedAllocation move.
// (The definitions: ksg_plain.hip's checkers and x-checker compute these sums inline from
// terms they share, the x-checker lane-parallel; tests pin both against the restatement.)
__device__ __forceinline__ int64_t es_delta(const KsgDev& d, int64_t req_c, int64_t req_m, int64_t cap_c,
                                            int64_t cap_m, double inv_c, double inv_m, int64_t snp_c, int64_t snp_m,
                                            int64_t now_c, int64_t now_m, int64_t frac_snap, int64_t frac_now) {
  int64_t dl = 0;
  const int64_t tcn = (int64_t)((uint64_t)now_c + (uint64_t)req_c), tmn = (int64_t)((uint64_t)now_m + (uint64_t)req_m);
  const int64_t tcs = (int64_t)((uint64_t)snp_c + (uint64_t)req_c), tms = (int64_t)((uint64_t)snp_m + (uint64_t)req_m);
  if (d.w_lr)
    dl += (int64_t)d.w_lr * ((int64_t)((lr_win_nb(tcn, cap_c, inv_c) + lr_win_nb(tmn, cap_m, inv_m)) >> 1) -
                             (int64_t)((lr_win_nb(tcs, cap_c, inv_c) + lr_win_nb(tms, cap_m, inv_m)) >> 1));
  if (d.w_spread) dl += (int64_t)d.w_spread * (frac_now - frac_snap);
  if (d.w_bal) dl += (int64_t)d.w_bal * (balanced_score(tcn, cap_c, tmn, cap_m) - balanced_score(tcs, cap_c, tms, cap_m));
  return dl;
}
// ... and a node's whole score for the pod at the snapshot (phase A's sum: static,
// LeastRequested, ServiceSpreading, BalancedAllocation, TaintToleration)
__device__ __forceinline__ int64_t es_snap_score(const KsgDev& d, int64_t req_c, int64_t req_m, int64_t cap_c,
                                                 int64_t cap_m, double inv_c, double inv_m, int64_t snp_c,
                                                 int64_t snp_m, int64_t frac_snap, int32_t sst, int32_t soft,
                                                 int32_t tmax) {
  int64_t s = sst;
  const int64_t tcs = (int64_t)((uint64_t)snp_c + (uint64_t)req_c), tms = (int64_t)((uint64_t)snp_m + (uint64_t)req_m);
  if (d.w_lr) s += (int64_t)d.w_lr * ((lr_win_nb(tcs, cap_c, inv_c) + lr_win_nb(tms, cap_m, inv_m)) >> 1);
  if (d.w_spread) s += (int64_t)d.w_spread * frac_snap;
  if (d.w_bal) s += (int64_t)d.w_bal * balanced_score(tcs, cap_c, tms, cap_m);
  if (d.w_taint) s += (int64_t)d.w_taint * (d.ntaint ? taint_score(soft, tmax) : 10);
  return s;
}
// allocatable - requested of an extended resource at the snapshot, clamped to
// int32: with a window's deltas <= 2^28 and requests <= 2^16 every fit test
// h - delta >= request decides as the unclamped one does
__device__ __forceinline__ int32_t xhead(int64_t cap, int64_t used) {
  const int64_t h = (int64_t)((uint64_t)cap - (uint64_t)used);
  return h > 0x7fffffffLL ? 0x7fffffff : h < -0x80000000LL ? (int32_t)0x80000000 : (int32_t)h;
}
