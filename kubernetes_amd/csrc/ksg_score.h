// ksg_score.h — phase A of the window path: one wave scores one 64-node word of
// the shard for a group of window pods against one snapshot (predicates.go:127-186,
// 326-350 for the filters; priorities.go:27-76 and spreading.go:24-168 for the
// scores). Two callers:
//   ksg_win_score_kernel (ksg_window.hip) — its own launch between windows;
//   ksg_win_plain_kernel<FUSED> (ksg_plain.hip) — the worker blocks of the fused
//     window launch, which score the window while block 0 resolves it (WT: every
//     output the resolver reads is stored write-through, sc1, so the resolver's
//     CU, on any XCD, reads it with sc1 loads after the group's counter is full).
#pragma once
#include "ksg_resolver.h"

#define KSG_SC_NT 256  // phase A: 4 waves, one 64-node word each
// phase A: pods per wave. 4 below 512 words per shard (32k nodes): the grid has
// (words / 4) x (W / PG) workgroups, too few to cover the latency at 8 pods per
// wave (config 2: 320 workgroups on 256 CUs); 8 above, where the grid is large
// and the node state each wave loads is shared by more pods
#define KSG_PG_SMALL 4
#define KSG_PG_LARGE 8
#define KSG_PG_WORDS 512


// ---------------------------------------------------------------------------
// phase A
// ---------------------------------------------------------------------------
// MODE 0: filter + score. With ServiceAntiAffinity (calculateAntiAffinityPriority,
// spreading.go:104-168) a pod's score on a node depends on the pod's service
// counts summed per label domain over every node that passes its filters, so
// phase A runs twice: MODE 1 only sums those domain counts (dcnt[pod][domain],
// all-reduced over the ranks when sharded), MODE 2 scores with the
// anti-affinity term and also writes each pod's fit bitmap (the resolver needs
// to know which committed nodes the pod fitted at the snapshot).
#define KSG_WIN_PLAIN 0
#define KSG_WIN_COUNT 1
#define KSG_WIN_ANTI 2
// extensions with TaintToleration scoring: a count pass first, the pod's max count of
// untolerated PreferNoSchedule taints over its filtered nodes (NormalizeReduce's max)
#define KSG_WIN_TMAX 3
// EXT: the extensions' filters (PodToleratesNodeTaints: static per (pod, node);
// extended resources: allocatable >= used + request, monotone under commits
// like cpu / memory), MODE PLAIN only
#ifdef KSG_PA_WAVES  // (A/B builds: an occupancy floor for phase A)
#define KSG_PA_ATTR __attribute__((amdgpu_waves_per_eu(KSG_PA_WAVES, 8)))
#else
#define KSG_PA_ATTR
#endif

// a phase-A output store: plain, or write-through (agent scope: global_store ... sc1)
template <bool WT, typename T>
__device__ __forceinline__ void st_out(T* p, T v) {
  if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// One wave: word w of the shard, window pods [p0, p0 + KSG_PG) of the window
// starting at batch pod pos. WT: outputs stored write-through (the fused launch);
// the pods' resolver records are then staged in rec_lds (KSG_PG x 192 B of this
// wave's LDS) and copied out as sc1 dword stores.
template <int MODE, int KSG_PG, bool EXT, bool WT>
__device__ __forceinline__ void win_score_wave(const KsgDev& d, const ksg_pod* __restrict__ batch,
                                               const uint32_t* __restrict__ ids, uint32_t pos, uint32_t n_batch,
                                               uint32_t wcap, uint32_t w, uint32_t p0,
                                               KsgWinSum* __restrict__ sums, uint64_t* __restrict__ wbits,
                                               int32_t* __restrict__ wmax, uint32_t ostride,
                                               int32_t* __restrict__ dcnt, uint64_t* __restrict__ wfit,
                                               int32_t* __restrict__ dmb, uint64_t* __restrict__ wbz, uint32_t dz,
                                               const ksg_pod_ext* __restrict__ exts, int32_t* __restrict__ tmax,
                                               uint64_t* __restrict__ psoft, int32_t* __restrict__ thist,
                                               uint32_t* rec_lds) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n_pods = min(wcap, n_batch - pos);
  const ksg_pod* __restrict__ pods = batch + pos;
  // the wave of local word 0 also writes the pods' resolver records, so it runs
  // even on a rank whose shard is empty (every rank resolves every pod)
  if ((w >= d.nwords && w != 0) || p0 >= n_pods) return;  // wave-uniform
  const bool has_word = w < d.nwords;
  const uint32_t np = min((uint32_t)KSG_PG, n_pods - p0);
  // KSG_DEBUG & 64: per-wave phase-A stamps into dbgbuf[48..50] (cycles / 16): the loads (to
  // the scoring loop, every load landed), scoring + stores, the wave count (tools/pa_stamps.py;
  // a diagnostic: the vmcnt(0) it adds before the loop changes the schedule)
  const bool pst = (d.dbg & 64) && d.dbgbuf;
  const uint64_t ts0 = pst ? __builtin_amdgcn_s_memtime() : 0ULL;
  uint64_t ts1 = 0;
  const uint32_t gw = d.wlo + w;  // global word
  const uint32_t n = gw * 64 + lane;
  const bool valid = has_word && n < d.hi;
  const uint64_t shard_m = __ballot(valid);  // nodes of the shard in this word
  const uint32_t P = d.preds;

  // ---- node state, once per wave (read-only while phase A runs)
  int64_t capc = 0, capm = 0, usedc = 0, usedm = 0;
  int32_t sst = 0;  // (|static score| < 2^30 on this path)
  if (valid) {
    capc = d.cap_cpu[n];
    capm = d.cap_mem[n];
    usedc = d.used_cpu[n];
    usedm = d.used_mem[n];
    if (d.has_static_score) sst = (int32_t)d.static_score[n];  // (window path: |score| < KSG_SCORE_BOUND)
  }
  const double inv_c = lr_inv10(capc), inv_m = lr_inv10(capm);
  // extended resources of this lane's node
  const bool xs_on = EXT && (d.ext_filters & KSG_EXT_SCALAR) && d.n_scalar > 0;
  int64_t xcap[KSG_MAX_SCALAR], xuse[KSG_MAX_SCALAR];
#pragma unroll
  for (int r = 0; r < KSG_MAX_SCALAR; ++r) {
    const bool on = xs_on && valid && (uint32_t)r < d.n_scalar;
    xcap[r] = on ? d.scalar_cap[(size_t)r * d.n_nodes + n] : 0;
    xuse[r] = on ? d.scalar_used[(size_t)r * d.n_nodes + n] : 0;
  }

  // extension scores: TaintToleration counts a pod's untolerated soft taints on this lane's
  // node as popcount(node taint mask & pod soft mask) (taint ids < 64 on this path)
  const bool tt = EXT && d.w_taint != 0 && d.ntaint != nullptr;
  const uint64_t ntm = (tt && valid) ? d.ntaint[n] : 0ULL;

  // ---- lane j < np: pod p0+j's context and its fit word for this node word
  uint64_t fm = 0;
  uint64_t ps = 0;   // lane j: pod j's untolerated soft taints (mask)
  int32_t tmj = 0;   // lane j: its TaintToleration max (score pass)
  int64_t rc = 0, rm = 0;
  int32_t svc = -1, smax = 0, zr = 0;
  PodCtx c;
  // lane j < np: pod j's list lengths (ports, pds, sel, svcs) and offsets, for its record
  uint32_t q_n[4] = {0, 0, 0, 0}, q_off[4] = {0, 0, 0, 0};
  int64_t xreq[KSG_MAX_SCALAR] = {0, 0, 0, 0};  // lane j: pod j's extended resource requests
  uint32_t xmask = 0;
  if (lane < np) {
    const ksg_pod& p = pods[p0 + lane];
    pod_resolve<false>(d, p, ids, c);
    if constexpr (EXT) {
      const ksg_pod_ext& pe = exts[pos + p0 + lane];
      if (xs_on)
#pragma unroll
        for (int r = 0; r < KSG_MAX_SCALAR; ++r)
          if ((uint32_t)r < d.n_scalar) {
            xreq[r] = pe.scalar[r];
            xmask |= xreq[r] > 0 ? 1u << r : 0u;
          }
      if (tt) {
        for (uint32_t t = 0; t < pe.n_soft; ++t) ps |= 1ULL << (ids[pe.soft_off + t] & 63);
        if (MODE == KSG_WIN_PLAIN && tmax) tmj = tmax[p0 + lane];
      }
    }
    if (w == 0) {
      q_n[0] = p.n_ports; q_n[1] = p.n_pds; q_n[2] = p.n_sel; q_n[3] = p.n_svcs;
      q_off[0] = p.ports_off; q_off[1] = p.pds_off; q_off[2] = p.sel_off; q_off[3] = p.svcs_off;
    }
    uint64_t m = shard_m;
    if (!has_word) m = 0;  // (no bitmap word to read)
    else if (d.has_static_fit) m &= d.static_fit[gw];  // LabelsPresence (predicates.go:215-229)
    if ((P & KSG_PRED_HOSTNAME) && c.host != -1) {  // PodFitsHost (predicates.go:181-186)
      m &= (c.host >= 0 && (uint32_t)c.host >> 6 == gw) ? (1ULL << (c.host & 63)) : 0ULL;
    }
    if (has_word) {
    if (P & KSG_PRED_MATCHNODESELECTOR)  // PodMatchesNodeLabels (predicates.go:161-167)
      for (uint32_t t = 0; t < c.n_sel; ++t) m &= d.pairmap[(size_t)c.sel[t] * d.nw + gw];
    if (P & KSG_PRED_NODISKCONFLICT)  // NoDiskConflict (predicates.go:73-83)
      for (uint32_t t = 0; t < c.n_pds; ++t) m &= ~d.keymap[(size_t)c.pds[t] * d.nw + gw];
    if (P & KSG_PRED_PODFITSPORTS)  // PodFitsPorts (predicates.go:326-338)
      for (uint32_t t = 0; t < c.n_ports; ++t) m &= ~d.keymap[(size_t)c.ports[t] * d.nw + gw];
    if (P & KSG_PRED_SERVICEAFFINITY) {  // CheckServiceAffinity (predicates.go:257-324)
#pragma unroll
      for (uint32_t j = 0; j < KSG_MAX_AFF; ++j)
        if (j < d.n_aff && c.req_aff[j] >= 0) m &= d.pairmap[(size_t)c.req_aff[j] * d.nw + gw];
    }
    if constexpr (EXT) {  // PodToleratesNodeTaints: an untolerated NoSchedule / NoExecute taint
      const ksg_pod_ext& pe = exts[pos + p0 + lane];
      if (d.ext_filters & KSG_EXT_TAINTS)
        for (uint32_t t = 0; t < pe.n_hard; ++t) m &= ~d.taintmap[(size_t)ids[pe.hard_off + t] * d.nw + gw];
    }
    }
    fm = m;
    rc = c.req_cpu;
    rm = c.req_mem;
    zr = c.zero_req;
    svc = c.svc;
    smax = c.spread_max;
  }

  // ---- (plain, no extensions, wfit given: the single-commit drop bitmap, KsgWinXchg.d1) lane j:
  // pod p0+j-1's requests and whether a conflict key of pod p0+j that its predicates check is
  // one of pod p0+j-1's keys (a node that took pod p0+j-1 then conflicts for pod p0+j)
  const bool d1_on = MODE == KSG_WIN_PLAIN && !EXT && wfit != nullptr;
  int64_t prc = 0, prm = 0;
  bool pkey = false;
  if (d1_on && lane < np && p0 + lane > 0) {
    const ksg_pod& q = pods[p0 + lane - 1];
    const ksg_pod& p = pods[p0 + lane];
    prc = q.milli_cpu;
    prm = q.memory;
    const uint32_t nq = q.n_ports + q.n_pds, np_ = p.n_ports + p.n_pds;
    for (uint32_t b = 0; b < np_; ++b) {
      if (!(b < p.n_ports ? (P & KSG_PRED_PODFITSPORTS) : (P & KSG_PRED_NODISKCONFLICT))) continue;
      const uint32_t kb = b < p.n_ports ? ids[p.ports_off + b] : ids[p.pds_off + (b - p.n_ports)];
      for (uint32_t a = 0; a < nq; ++a)
        pkey |= (a < q.n_ports ? ids[q.ports_off + a] : ids[q.pds_off + (a - q.n_ports)]) == kb;
    }
  }

  // ---- per-pod service counts of this lane's node, all issued up front: the
  // service's node word first (svc_bits, one 8-byte load per wave), then a count
  // only where the node holds pods of the service (most counts are 0)
  const bool need_cnt = d.w_spread != 0 || MODE != KSG_WIN_PLAIN;
  uint64_t sbw[KSG_PG];
#pragma unroll
  for (int j = 0; j < KSG_PG; ++j) {
    const int32_t s = __builtin_amdgcn_readlane(svc, j);
    sbw[j] = (need_cnt && has_word && (uint32_t)j < np && s >= 0) ? d.svc_bits[(size_t)s * d.nw + gw] : 0ULL;
  }
  int32_t cnt[KSG_PG];
#pragma unroll
  for (int j = 0; j < KSG_PG; ++j) {
    const int32_t s = __builtin_amdgcn_readlane(svc, j);
    cnt[j] = (valid && ((sbw[j] >> lane) & 1ULL)) ? d.svc_cnt[(size_t)s * d.n_nodes + n] : 0;
  }

  // anti-affinity label domains of this lane's node (dense per priority, -1 unlabelled)
  int32_t dom[KSG_WIN_MAX_ANTI];
#pragma unroll
  for (int a = 0; a < KSG_WIN_MAX_ANTI; ++a)
    dom[a] = (MODE != KSG_WIN_PLAIN && valid && (uint32_t)a < d.n_anti && d.w_anti[a] != 0)
                 ? d.anti_domain[(size_t)a * d.n_nodes + n]
                 : -1;
  int32_t tot = 0;  // svc_total of each pod's service (lane j)
  if (MODE == KSG_WIN_ANTI && lane < np) tot = c.svc_total;
  // ServiceAntiAffinity term of every pod of the group on this lane's node
  // (CalculateAntiAffinityPriority, spreading.go:152-166): the count loads are
  // all issued before the first use, not one L2 round trip per pod
  int64_t aterm[KSG_PG];
  if constexpr (MODE == KSG_WIN_ANTI) {
    int32_t pcs[KSG_PG][KSG_WIN_MAX_ANTI];
#pragma unroll
    for (int j = 0; j < KSG_PG; ++j)
#pragma unroll
      for (int a = 0; a < KSG_WIN_MAX_ANTI; ++a)
        pcs[j][a] = ((uint32_t)j < np && dom[a] >= 0)
                        ? dcnt[(size_t)(p0 + j) * d.n_domains_total + d.anti_dom_off[a] + dom[a]]
                        : 0;
#pragma unroll
    for (int j = 0; j < KSG_PG; ++j) {
      const int32_t tj = __builtin_amdgcn_readlane(tot, j);
      int64_t s = 0;
#pragma unroll
      for (int a = 0; a < KSG_WIN_MAX_ANTI; ++a)
        if (dom[a] >= 0)  // unlabelled nodes score 0
          s += (int64_t)d.w_anti[a] * (tj > 0 ? frac10_f32((int64_t)tj - pcs[j][a], tj) : 10);
      aterm[j] = s;
    }
    // priorities past the first KSG_WIN_MAX_ANTI (policies with more): their domain and counts
    // loaded here, one priority at a time
    for (uint32_t a = KSG_WIN_MAX_ANTI; a < d.n_anti; ++a) {
      if (d.w_anti[a] == 0) continue;
      const int32_t da = valid ? d.anti_domain[(size_t)a * d.n_nodes + n] : -1;
      int32_t pc[KSG_PG];
#pragma unroll
      for (int j = 0; j < KSG_PG; ++j)
        pc[j] = ((uint32_t)j < np && da >= 0) ? dcnt[(size_t)(p0 + j) * d.n_domains_total + d.anti_dom_off[a] + da] : 0;
#pragma unroll
      for (int j = 0; j < KSG_PG; ++j) {
        const int32_t tj = __builtin_amdgcn_readlane(tot, j);
        if (da >= 0) aterm[j] += (int64_t)d.w_anti[a] * (tj > 0 ? frac10_f32((int64_t)tj - pc[j], tj) : 10);
      }
    }
  }
  // re-rank (dmb != nullptr): this node's domain row for the first anti priority
  // (dz - 1: unlabelled), and in the score pass each pod's best score without
  // the anti term over its filtered nodes of that row (the count pass's max)
  const int32_t zrow = (dmb && valid) ? (dom[0] >= 0 ? dom[0] : (int32_t)dz - 1) : -1;
  int32_t mbz[KSG_PG];
  if constexpr (MODE == KSG_WIN_ANTI) {
#pragma unroll
    for (int j = 0; j < KSG_PG; ++j)
      mbz[j] = ((uint32_t)j < np && zrow >= 0) ? dmb[(size_t)(p0 + j) * dz + zrow] : KSG_S32_NONE;
  }

  if (pst) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ts1 = __builtin_amdgcn_s_memtime();
  }
  // ---- score every pod of the group on this word
  const int32_t w_lr = (int32_t)d.w_lr, w_spread = (int32_t)d.w_spread;  // (|w| < 2^30 / 10 on this path)
  int32_t my_max = KSG_S32_NONE;
  uint64_t my_bits = 0, my_fit = 0, my_bz = 0;
  const bool res_on = (P & KSG_PRED_PODFITSRESOURCES) != 0;
#pragma unroll
  for (int j = 0; j < KSG_PG; ++j) {
    if ((uint32_t)j < np) {
      const uint64_t fmj = readlane64(fm, j);
      const int64_t rcj = (int64_t)readlane64((uint64_t)rc, j);
      const int64_t rmj = (int64_t)readlane64((uint64_t)rm, j);
      bool fit = (fmj >> lane) & 1ULL;
      if (res_on && !__builtin_amdgcn_readlane(zr, j)) {
        // CheckPodsExceedingCapacity over existing+pod in closed form (predicates.go:104-145)
        const bool fc = capc == 0 || (int64_t)((uint64_t)capc - (uint64_t)usedc) >= rcj;
        const bool fmm = capm == 0 || (int64_t)((uint64_t)capm - (uint64_t)usedm) >= rmj;
        fit = fit && fc && fmm;
      }
      if constexpr (EXT) {  // PodFitsResources' extended resources: allocatable >= used + request
        if (xs_on)
#pragma unroll
          for (int r = 0; r < KSG_MAX_SCALAR; ++r) {
            const int64_t q = (int64_t)readlane64((uint64_t)xreq[r], j);
            if ((uint32_t)r < d.n_scalar && q > 0 && xcap[r] < (int64_t)((uint64_t)xuse[r] + (uint64_t)q)) fit = false;
          }
      }
      if constexpr (MODE == KSG_WIN_TMAX) {  // the pod's max soft-taint count over its filtered nodes
        const int32_t soft = fit ? __popcll(ntm & readlane64(ps, j)) : 0;
        const int32_t mx = wave_total_max(soft);
        if (lane == 0 && mx > 0) atomicMax(tmax + p0 + j, mx);
        // ... and how many filtered nodes hold each count (one atomic per distinct count)
        uint64_t pend = __ballot(fit);
        while (pend) {
          const int32_t v = __builtin_amdgcn_readlane(soft, (int)__builtin_ctzll(pend));
          const uint64_t mine = __ballot(fit && soft == v);
          if (lane == 0) atomicAdd(thist + (size_t)(p0 + j) * KSG_TBINS + v, (int32_t)__popcll(mine));
          pend &= ~mine;
        }
        continue;
      }
      if constexpr (MODE == KSG_WIN_COUNT) {
        if (dmb) {
          // re-rank: the best score without the anti term per domain row (the
          // same sum the score pass forms), one atomic max per (wave, row)
          int32_t bs = KSG_S32_NONE;
          if (fit) {
            int64_t s = sst;
            if (d.w_lr) {
              const int64_t tc = (int64_t)((uint64_t)usedc + (uint64_t)rcj);
              const int64_t tm = (int64_t)((uint64_t)usedm + (uint64_t)rmj);
              s += (int64_t)d.w_lr * ((lr_win(tc, capc, inv_c) + lr_win(tm, capm, inv_m)) >> 1);
            }
            if (d.w_spread) {
              const int32_t mx = __builtin_amdgcn_readlane(smax, j);
              s += (int64_t)d.w_spread * (mx > 0 ? frac10_f32((int64_t)mx - cnt[j], mx) : 10);
            }
            bs = (int32_t)s;
          }
          uint64_t zp = __ballot(fit && zrow >= 0);
          while (zp) {
            const int32_t zz = __builtin_amdgcn_readlane(zrow, (int)__builtin_ctzll(zp));
            const bool mine = ((zp >> lane) & 1ULL) && zrow == zz;
            const int32_t mx = wave_total_max(mine ? bs : KSG_S32_NONE);
            if (lane == 0) atomicMax(dmb + (size_t)(p0 + j) * dz + zz, mx);
            zp &= ~__ballot(mine);
          }
        }
        // the pod's service pods on filtered labelled nodes, per domain
        // (calculateAntiAffinityPriority, spreading.go:130-151): summed over the
        // wave one domain at a time, one atomic per (wave, domain)
        const int32_t cj = fit ? cnt[j] : 0;
#pragma unroll
        for (int a = 0; a < KSG_WIN_MAX_ANTI; ++a) {
          uint64_t pend = __ballot(cj != 0 && dom[a] >= 0);
          while (pend) {
            const int32_t dd = __builtin_amdgcn_readlane(dom[a], (int)__builtin_ctzll(pend));
            const bool mine = ((pend >> lane) & 1ULL) && dom[a] == dd;
            const uint32_t sum = wave_total_add(mine ? (uint32_t)cj : 0u);
            if (lane == 0) atomicAdd(dcnt + (size_t)(p0 + j) * d.n_domains_total + d.anti_dom_off[a] + dd, (int32_t)sum);
            pend &= ~__ballot(mine);
          }
        }
        for (uint32_t a = KSG_WIN_MAX_ANTI; a < d.n_anti; ++a) {  // (priorities past the first few)
          if (d.w_anti[a] == 0) continue;
          const int32_t da = valid ? d.anti_domain[(size_t)a * d.n_nodes + n] : -1;
          uint64_t pend = __ballot(cj != 0 && da >= 0);
          while (pend) {
            const int32_t dd = __builtin_amdgcn_readlane(da, (int)__builtin_ctzll(pend));
            const bool mine = ((pend >> lane) & 1ULL) && da == dd;
            const uint32_t sum = wave_total_add(mine ? (uint32_t)cj : 0u);
            if (lane == 0) atomicAdd(dcnt + (size_t)(p0 + j) * d.n_domains_total + d.anti_dom_off[a] + dd, (int32_t)sum);
            pend &= ~__ballot(mine);
          }
        }
        continue;
      }
      if (MODE == KSG_WIN_ANTI || (EXT && wfit != nullptr)) {  // (extension scores: non-T0 slots' fit)
        const uint64_t fb = __ballot(fit);
        if (lane == (uint32_t)j) my_fit = fb;
      }
      int32_t base = KSG_S32_NONE;  // (re-rank) the score without the anti term
      int32_t sc = KSG_S32_NONE;
      if (fit) {
        if (d.equal_fallback) {
          sc = 1;  // EqualPriority (generic_scheduler.go:141-143,180-195)
        } else {
          // int32 arithmetic: the window path runs only while 10 x the summed |weights| plus the
          // static score stay below KSG_SCORE_BOUND = 2^30 (KsgDev.wide: the exact kernels), so
          // every term and partial sum here fits and the int64 sum would be the same
          int32_t s = sst;
          if (d.w_lr) {  // calculateOccupancy (priorities.go:43-76)
            const int64_t tc = (int64_t)((uint64_t)usedc + (uint64_t)rcj);
            const int64_t tm = (int64_t)((uint64_t)usedm + (uint64_t)rmj);
            s += w_lr * ((lr_win(tc, capc, inv_c) + lr_win(tm, capm, inv_m)) >> 1);
          }
          if (d.w_spread) {  // CalculateSpreadPriority (spreading.go:72-86)
            const int32_t mx = __builtin_amdgcn_readlane(smax, j);
            // (no count on this node: (mx - 0) / mx = 1 exactly, 10; the f32 divide only where
            // a lane of the wave holds pods of the service)
            int32_t ss = 10;
            if (mx > 0 && cnt[j] != 0) ss = frac10_i32(mx - cnt[j], mx);
            s += w_spread * ss;
          }
          if constexpr (EXT) {  // extension scores (parity unpinned; the exact kernels' terms)
            if (d.w_bal) {  // BalancedResourceAllocation, float64 op for op
              const int64_t tc = (int64_t)((uint64_t)usedc + (uint64_t)rcj);
              const int64_t tm = (int64_t)((uint64_t)usedm + (uint64_t)rmj);
              s += d.w_bal * (int32_t)balanced_score(tc, capc, tm, capm);
            }
            if (tt)  // TaintToleration: NormalizeReduce(10, reverse) over the filtered nodes
              s += d.w_taint * (int32_t)taint_score(__popcll(ntm & readlane64(ps, j)), __builtin_amdgcn_readlane(tmj, j));
            else if (d.w_taint)
              s += d.w_taint * 10;
          }
          base = s;
          if constexpr (MODE == KSG_WIN_ANTI) s += (int32_t)aterm[j];  // (computed above)
          sc = s;
        }
      }
      if (d1_on) {
        // the x-checker's verdict (ksg_plain.hip) on this node for this pod if pod p0+j-1 were the
        // node's first commit of the window: it no longer fits (resources, a shared key) or its
        // LeastRequested term fell; the node's service entries cannot change it when pod p0+j-1
        // is of another service (the committer takes this bitmap only then)
        bool dr = false;
        if (fit) {
          const int64_t pcj = (int64_t)readlane64((uint64_t)prc, j), pmj = (int64_t)readlane64((uint64_t)prm, j);
          const int64_t nowc = (int64_t)((uint64_t)usedc + (uint64_t)pcj), nowm = (int64_t)((uint64_t)usedm + (uint64_t)pmj);
          if (res_on && !__builtin_amdgcn_readlane(zr, j))  // PodFitsResources (predicates.go:127-145)
            dr = !((capc == 0 || capc - nowc >= rcj) && (capm == 0 || capm - nowm >= rmj));
          if (d.w_lr) {  // LeastRequested (priorities.go:43-76)
            const int32_t lr_now = lr_win(nowc + rcj, capc, inv_c) + lr_win(nowm + rmj, capm, inv_m);
            const int32_t lr_snap = lr_win(usedc + rcj, capc, inv_c) + lr_win(usedm + rmj, capm, inv_m);
            dr |= (lr_now >> 1) != (lr_snap >> 1);
          }
          dr |= __builtin_amdgcn_readlane((int)pkey, j) != 0;
        }
        const uint64_t db = __ballot(dr);
        if (lane == (uint32_t)j) my_fit = db;
      }
      int32_t m = wave_total_max(sc);
      if (d.empty_priorities) m = KSG_S32_NONE;  // prioritizeNodes returns nothing
      const uint64_t b = __ballot(m != KSG_S32_NONE && sc == m);
      if (lane == (uint32_t)j) {
        my_max = m;
        my_bits = b;
      }
      if constexpr (MODE == KSG_WIN_ANTI) {
        if (dmb) {  // filtered nodes at their domain row's best score without the anti term
          const uint64_t bz = __ballot(fit && zrow >= 0 && base == mbz[j]);
          if (lane == (uint32_t)j) my_bz = bz;
          // ... and, past 32k nodes per shard (win2_zg: the resolver keeps no row bitmaps in LDS
          // to count them over), how many per row (dmb's second half, [wcap][dz] int32, zeroed by
          // the resolver for the next window), one atomic per (wave, row)
          if (win2_zg_words(d.nwords))
          for (uint64_t pend = bz; pend;) {
            const int32_t zz = __builtin_amdgcn_readlane(zrow, (int)__builtin_ctzll(pend));
            const uint64_t mine = __ballot(zrow == zz) & pend;
            if (lane == 0) atomicAdd(dmb + (size_t)wcap * dz + (size_t)(p0 + j) * dz + zz, (int32_t)__popcll(mine));
            pend &= ~mine;
          }
        }
      }
    }
  }
  if constexpr (MODE == KSG_WIN_COUNT || MODE == KSG_WIN_TMAX) return;
  if (lane < np && has_word) {
    st_out<WT>(wmax + (size_t)(p0 + lane) * ostride + w, my_max);
    st_out<WT>(wbits + (size_t)(p0 + lane) * ostride + w, my_bits);
    if constexpr (MODE == KSG_WIN_ANTI) {
      wfit[(size_t)(p0 + lane) * ostride + w] = my_fit;
      if (dmb) wbz[(size_t)(p0 + lane) * ostride + w] = my_bz;
    }
    if constexpr (EXT)
      if (wfit) wfit[(size_t)(p0 + lane) * ostride + w] = my_fit;
    if (d1_on) st_out<WT>(wfit + (size_t)(p0 + lane) * ostride + w, my_fit);  // (the single-commit drop bitmap)
  }
  if constexpr (EXT)
    if (psoft && w == 0 && lane < np) psoft[p0 + lane] = ps;
  if (pst && lane == 0) {
    const uint64_t ts2 = __builtin_amdgcn_s_memtime();
    atomicAdd(d.dbgbuf + 48, (int32_t)((ts1 - ts0) >> 4));
    atomicAdd(d.dbgbuf + 49, (int32_t)((ts2 - ts1) >> 4));
    atomicAdd(d.dbgbuf + 50, 1);
  }

  // ---- the resolver's record of each pod (one wave per pod group)
  if (w == 0) {
    if (lane < np) {
      const ksg_pod& p = pods[p0 + lane];
      // (WT: staged in this wave's LDS, copied out write-through below)
      KsgWinSum* S = (WT ? reinterpret_cast<KsgWinSum*>(rec_lds) : sums + p0) + lane;
      S->m0 = 0;
      S->k0 = 0;
      S->error = c.error;
      S->service = c.svc;
      S->host = c.host;
      S->spread_max = c.spread_max;
      S->svc_total = c.svc_total;
      S->n_inline = p.n_ports + p.n_pds + p.n_sel + p.n_svcs;
      S->milli_cpu = c.req_cpu;
      S->memory = c.req_mem;
#pragma unroll
      for (int j = 0; j < KSG_WIN_SUM_AFF; ++j) S->req_aff[j] = c.req_aff[j];
      S->n_ports = (uint16_t)p.n_ports;
      S->n_pds = (uint16_t)p.n_pds;
      S->n_sel = (uint16_t)p.n_sel;
      S->n_svcs = (uint16_t)p.n_svcs;
      S->xmask = xmask;
#pragma unroll
      for (int r = 0; r < 4; ++r) S->xreq[r] = r < KSG_MAX_SCALAR ? (int32_t)xreq[r] : 0;
    }
    // the pods' inline id lists: lane t takes entry t of every pod of the group,
    // all loads issued before the first store (not one pod's round trip after
    // another's)
    uint32_t v[KSG_PG], ninl[KSG_PG];
#pragma unroll
    for (int j = 0; j < KSG_PG; ++j) {
      const uint32_t a = __builtin_amdgcn_readlane(q_n[0], j), b = __builtin_amdgcn_readlane(q_n[1], j);
      const uint32_t e = __builtin_amdgcn_readlane(q_n[2], j), f = __builtin_amdgcn_readlane(q_n[3], j);
      ninl[j] = (uint32_t)j < np ? a + b + e + f : 0u;
      uint32_t t = lane, idx;
      if (t < a) idx = __builtin_amdgcn_readlane(q_off[0], j) + t;
      else if ((t -= a) < b) idx = __builtin_amdgcn_readlane(q_off[1], j) + t;
      else if ((t -= b) < e) idx = __builtin_amdgcn_readlane(q_off[2], j) + t;
      else idx = __builtin_amdgcn_readlane(q_off[3], j) + (t - e);
      v[j] = (lane < KSG_WIN_INLINE && lane < ninl[j]) ? ids[idx] : 0u;
    }
#pragma unroll
    for (int j = 0; j < KSG_PG; ++j)
      if (lane < KSG_WIN_INLINE && lane < ninl[j]) (WT ? reinterpret_cast<KsgWinSum*>(rec_lds) : sums + p0)[j].ids[lane] = v[j];
    if constexpr (WT) {
      // one wave's LDS accesses complete in issue order: the staged records read back whole,
      // then stored dword by dword, write-through
      asm volatile("" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < KSG_PG; ++j)
        if ((uint32_t)j < np && lane < KSG_WIN_SUM_DWORDS)
          st_out<true>(reinterpret_cast<uint32_t*>(sums + p0 + j) + lane, rec_lds[j * KSG_WIN_SUM_DWORDS + lane]);
    }
  }
}
