// ksg_window.hip — speculative window path for the Filter/Score pass.
//
// The reference schedules pods strictly one after another: pod i+1 sees pod i's
// AssumePod (plugin/pkg/scheduler/scheduler.go:115-118). The window path keeps
// that exact sequential semantics while moving almost all of the work off the
// sequential chain:
//
//  phase A (ksg_win_eval_kernel, one 256-thread workgroup per pod, all CUs):
//    every pod of a window is filtered and scored against ONE snapshot of the
//    node state; per pod it stores the best score M0, the tie count k0, the tie
//    bitmap T0 (bit n = node n scores M0) and two spreading scalars.
//  phase B (ksg_win_resolve_kernel, one wave): walks the window in order and
//    reproduces the sequential result from the snapshot. For a "clean" pod —
//    one whose service scalars (ServiceSpreading maxCount, ServiceAffinity
//    peer) no earlier pod of the window changed — a commit can only make the
//    committed node WORSE (requested totals grow: LeastRequested falls and
//    PodFitsResources can flip to false; host ports / PDs only get added;
//    service counts grow under a fixed maxCount), and every other node is
//    untouched. So the sequential max is still M0 unless all of T0 was made
//    worse, and the sequential tie set is T0 minus the nodes committed earlier
//    in the window (set C) whose re-evaluated score dropped. Phase B re-scores
//    only T0 ∩ C, draws the same Int63 the reference draws, selects the ix-th
//    tie in descending name order, commits, and continues. A pod that is not
//    clean, or whose whole T0 dropped, ends the window; the host starts the next
//    window (new snapshot) at that pod. Results are bit-identical to the
//    one-pod-at-a-time path (tests/test_gpu_parity.py compares both).
//
// ServiceAntiAffinity changes a service-wide scalar on every commit and is
// served by the exact per-pod kernel instead (ksg_kernels.hip).
#include "ksg_device.h"

#define KSG_WIN_NT 256
#define KSG_WIN_NWAVE (KSG_WIN_NT / 64)

// dword offsets inside KsgWinSum (lane j of the resolver holds dword j)
#define WS_M0 0
#define WS_K0 1
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
#define WS_IDS 19

// phase A: one workgroup per pod of the window. The node state is read-only
// while phase A runs, so every load is a plain (cacheable) load.
__global__ __launch_bounds__(KSG_WIN_NT) void ksg_win_eval_kernel(KsgDev d, const ksg_pod* __restrict__ pods,
                                                                 const uint32_t* __restrict__ ids,
                                                                 KsgWinSum* __restrict__ sums,
                                                                 uint64_t* __restrict__ t0words) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int32_t* s_sc = reinterpret_cast<int32_t*>(smem);  // one score per node of the shard
  __shared__ int32_t s_red[KSG_WIN_NWAVE];
  __shared__ uint32_t s_cnt[KSG_WIN_NWAVE];

  const uint32_t i = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t bit = 1ULL << lane;
  const ksg_pod& p = pods[i];
  PodCtx c;
  pod_resolve<false>(d, p, ids, c);
  KsgWinSum* S = sums + i;
  uint64_t* T0 = t0words + (size_t)i * d.nwords;
  int32_t M = KSG_S32_NONE;
  uint32_t k = 0;
  if (!c.error) {
    const bool need_cnt = d.w_spread != 0 && c.svc >= 0;
    const uint32_t span = d.nwords * 64;
    int32_t m = KSG_S32_NONE;
    for (uint32_t off = tid; off < span; off += KSG_WIN_NT) {
      const uint32_t n = d.lo + off;
      const uint32_t wi = (d.lo >> 6) + (off >> 6);
      int32_t sc = KSG_S32_NONE;
      if (n < d.hi) {
        const int64_t capc = d.cap_cpu[n], capm = d.cap_mem[n];
        const int64_t usedc = (d.dbg & 2) ? ld_mut(d.used_cpu + n) : d.used_cpu[n];
        const int64_t usedm = (d.dbg & 2) ? ld_mut(d.used_mem + n) : d.used_mem[n];
        const int32_t cnt = need_cnt ? d.svc_cnt[(size_t)c.svc * d.n_nodes + n] : 0;
        if (node_fail<false>(d, c, n, wi, bit, capc, capm, usedc, usedm) == KSG_FAIL_NONE)
          sc = (int32_t)node_score(d, c, n, capc, capm, usedc, usedm, cnt);
      }
      s_sc[off] = sc;
      m = sc > m ? sc : m;
    }
    m = wave_max_i32(m);
    if (lane == 0) s_red[wave] = m;
    __syncthreads();
    M = s_red[0];
#pragma unroll
    for (int w = 1; w < KSG_WIN_NWAVE; ++w) M = s_red[w] > M ? s_red[w] : M;
    if (d.empty_priorities) M = KSG_S32_NONE;
    uint32_t cntk = 0;
    for (uint32_t off = tid; off < span; off += KSG_WIN_NT) {
      const uint64_t b = __ballot(M != KSG_S32_NONE && s_sc[off] == M);
      if (lane == 0) T0[off >> 6] = b;
      cntk += __popcll(b);
    }
    if (lane == 0) s_cnt[wave] = cntk;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < KSG_WIN_NWAVE; ++w) k += s_cnt[w];
  }
  // the record phase B streams for this pod
  const uint32_t ninl = p.n_ports + p.n_pds + p.n_sel + p.n_svcs;
  if (tid < KSG_WIN_INLINE && tid < ninl) {
    uint32_t t = tid, v;
    if (t < p.n_ports) v = ids[p.ports_off + t];
    else if ((t -= p.n_ports) < p.n_pds) v = ids[p.pds_off + t];
    else if ((t -= p.n_pds) < p.n_sel) v = ids[p.sel_off + t];
    else v = ids[p.svcs_off + (t - p.n_sel)];
    S->ids[tid] = v;
  }
  if (tid == 0) {
    S->m0 = M;
    S->k0 = M == KSG_S32_NONE ? 0 : k;
    S->error = c.error;
    S->service = c.svc;
    S->host = c.host;
    S->spread_max = c.spread_max;
    S->svc_total = c.svc_total;
    S->n_inline = ninl;
    S->milli_cpu = c.req_cpu;
    S->memory = c.req_mem;
#pragma unroll
    for (int j = 0; j < KSG_MAX_AFF; ++j) S->req_aff[j] = c.req_aff[j];
    S->n_ports = (uint16_t)p.n_ports;
    S->n_pds = (uint16_t)p.n_pds;
    S->n_sel = (uint16_t)p.n_sel;
    S->n_svcs = (uint16_t)p.n_svcs;
  }
}

// list entries straight from the record register (readlane: uniform index;
// v_readlane ignores EXEC, so it is safe inside divergent code)
struct RecLists {
  uint32_t rec, o_pd, o_sel;
  __device__ __forceinline__ uint32_t port(uint32_t i) const { return __builtin_amdgcn_readlane(rec, WS_IDS + i); }
  __device__ __forceinline__ uint32_t pd(uint32_t i) const { return __builtin_amdgcn_readlane(rec, WS_IDS + o_pd + i); }
  __device__ __forceinline__ uint32_t sel(uint32_t i) const { return __builtin_amdgcn_readlane(rec, WS_IDS + o_sel + i); }
};

// Per-window cache of a node committed in the window (set C). The node state in
// HBM stays a pristine snapshot while the window resolves; the window's deltas
// live here and are written back once, at the end of the window.
#define KSG_SLOT_KEYS 8
#define KSG_SLOT_SVCS 12
struct WinSlot {
  int64_t cap_c, cap_m, snap_c, snap_m;  // snapshot capacity / requested totals
  int64_t dc, dm;                        // requested added by the window
  uint32_t node, nk, ns, pad;
  uint32_t keys[KSG_SLOT_KEYS];          // conflict keys added by the window
  uint32_t svcs[KSG_SLOT_SVCS];          // one entry per committed pod x service
  int32_t scnt[KSG_SLOT_SVCS];           // svc_cnt[svcs[a]][node] at the snapshot
};

__host__ __device__ constexpr uint32_t win_even(uint32_t x) { return (x + 1) & ~1u; }
__host__ __device__ constexpr size_t win_lds_fixed(uint32_t P, uint32_t nflag, uint32_t nshard) {
  return (size_t)P * 64 * 8 + (size_t)win_even(nflag) * 4 * 2 + (((size_t)nshard * 2 + 15) & ~(size_t)15);
}
__host__ __device__ constexpr size_t win_lds_per_slot() { return sizeof(WinSlot) + 4 + 8 + 1; }

#define KSG_STOP_SERVICE 1
#define KSG_STOP_EXHAUSTED 2
#define KSG_STOP_SLOT 3
#define KSG_STOP_OVERSIZE 4

__device__ __forceinline__ int64_t rl64(int64_t v, int lane) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane)) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane) << 32));
}

// phase B: one wave resolves the window sequentially. P = words of T0 per lane.
template <int P>
__global__ __launch_bounds__(64) void ksg_win_resolve_kernel(KsgDev d, const ksg_pod* __restrict__ pods,
                                                            const uint32_t* __restrict__ ids, uint32_t n_pods,
                                                            const KsgWinSum* __restrict__ sums,
                                                            const uint64_t* __restrict__ t0words,
                                                            uint64_t* rng_io, int32_t* __restrict__ out,
                                                            uint32_t* stat_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t lane = threadIdx.x;
  const uint32_t nflag = (d.n_services + 31) / 32;
  const uint32_t nshard = d.hi - d.lo;
  uint64_t* s_cmask = reinterpret_cast<uint64_t*>(smem);               // nodes committed in this window
  uint32_t* s_flag = reinterpret_cast<uint32_t*>(s_cmask + P * 64);    // services whose scalars changed
  uint32_t* s_peerset = s_flag + win_even(nflag);                      // services whose peer the window set
  uint16_t* s_slot_of = reinterpret_cast<uint16_t*>(s_peerset + win_even(nflag));
  WinSlot* s_slots = reinterpret_cast<WinSlot*>(reinterpret_cast<char*>(s_slot_of) +
                                                (((size_t)nshard * 2 + 15) & ~(size_t)15));
  uint32_t* s_peer = reinterpret_cast<uint32_t*>(s_slots + n_pods);    // (service, node) pairs
  uint32_t* s_list = s_peer + 2 * n_pods;                              // candidate node offsets
  uint8_t* s_dflag = reinterpret_cast<uint8_t*>(s_list + n_pods);      // candidate dropped?
  for (uint32_t w = lane; w < P * 64u; w += 64) s_cmask[w] = 0;
  for (uint32_t w = lane; w < 2 * win_even(nflag); w += 64) s_flag[w] = 0;
  const bool spread_on = d.w_spread != 0;
  const bool aff_on = (d.preds & KSG_PRED_SERVICEAFFINITY) && d.n_aff > 0;
  const bool res_on = (d.preds & KSG_PRED_PODFITSRESOURCES) != 0;
  const bool ports_on = (d.preds & KSG_PRED_PODFITSPORTS) != 0;
  const bool disk_on = (d.preds & KSG_PRED_NODISKCONFLICT) != 0;
  uint64_t rng = *rng_io;
  uint32_t resolved = n_pods, reason = 0, n_slots = 0, n_peer = 0;

  // pending snapshot loads of the last commit, retired at the next pod
  bool p_active = false, p_new = false;
  uint32_t p_slot = 0, p_base = 0, p_nsv = 0, p_node = 0;
  int64_t p_v = 0;                     // lanes 0..3: cap_c, cap_m, used_c, used_m
  int32_t p_cnt = 0, p_max = 0, p_peer = 0;  // service lanes 32+t
  auto retire = [&]() {
    if (!p_active) return;
    WinSlot& S = s_slots[p_slot];
    if (p_new) {
      const int64_t cc = rl64(p_v, 0), cm = rl64(p_v, 1), uc = rl64(p_v, 2), um = rl64(p_v, 3);
      if (lane == 0) {
        S.cap_c = cc;
        S.cap_m = cm;
        S.snap_c = uc;
        S.snap_m = um;
      }
    }
    const uint32_t t = lane - 32;
    bool changed = false;
    uint32_t sv = 0;
    if (lane >= 32 && t < p_nsv) {
      const uint32_t a = p_base + t;
      sv = S.svcs[a];
      uint32_t before = 0;  // in-window commits of sv on this node before this one
      for (uint32_t b = 0; b < a; ++b) before += S.svcs[b] == sv;
      S.scnt[a] = p_cnt;
      if (spread_on && p_cnt + (int32_t)before + 1 > p_max) changed = true;  // maxCount rises
      if (p_peer == -1 && !((s_peerset[sv >> 5] >> (sv & 31)) & 1u)) changed |= aff_on;
    }
    // first commit of a service with no peer yet: record the peer (ballot, lane 0 applies)
    uint64_t pm = __ballot(lane >= 32 && t < p_nsv && p_peer == -1);
    while (pm) {
      const uint32_t b = __builtin_ctzll(pm);
      pm &= pm - 1;
      const uint32_t fsv = (uint32_t)__builtin_amdgcn_readlane((int)sv, (int)b);
      const bool fresh = !((s_peerset[fsv >> 5] >> (fsv & 31)) & 1u);  // same LDS word for all lanes
      if (fresh) {
        if (lane == 0) {
          s_peerset[fsv >> 5] |= 1u << (fsv & 31);
          s_peer[2 * n_peer] = fsv;
          s_peer[2 * n_peer + 1] = p_node;
        }
        ++n_peer;
      }
    }
    uint64_t fm = __ballot(changed);
    while (fm) {
      const uint32_t b = __builtin_ctzll(fm);
      fm &= fm - 1;
      const uint32_t fsv = (uint32_t)__builtin_amdgcn_readlane((int)sv, (int)b);
      if (lane == 0) s_flag[fsv >> 5] |= 1u << (fsv & 31);
    }
    p_active = false;
  };

  // software pipeline: pod i+1's record and T0 words load while pod i resolves
  const uint32_t* recs = reinterpret_cast<const uint32_t*>(sums);
  uint32_t rec = (n_pods > 0 && lane < KSG_WIN_SUM_DWORDS) ? recs[lane] : 0u;
  uint64_t tw[P], twn[P];
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const uint32_t w = q * 64 + lane;
    tw[q] = (n_pods > 0 && w < d.nwords) ? t0words[w] : 0ULL;
  }
  uint64_t t_last = 0, t_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool stamp = (d.dbg & 8) != 0;
#define KSG_STAMP(k)                                     \
  if (stamp) {                                           \
    const uint64_t t_now = __builtin_amdgcn_s_memtime(); \
    t_acc[k] += t_now - t_last;                          \
    t_last = t_now;                                      \
  }
  if (stamp) t_last = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < n_pods; ++i) {
    uint32_t recn = 0;
    if (i + 1 < n_pods) {
      if (lane < KSG_WIN_SUM_DWORDS) recn = recs[(size_t)(i + 1) * KSG_WIN_SUM_DWORDS + lane];
      const uint64_t* nx = t0words + (size_t)(i + 1) * d.nwords;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const uint32_t w = q * 64 + lane;
        twn[q] = w < d.nwords ? nx[w] : 0ULL;
      }
    }
    KSG_STAMP(0)
    retire();
    KSG_STAMP(1)
    const int32_t m0 = (int32_t)__builtin_amdgcn_readlane(rec, WS_M0);
    const uint32_t k0 = __builtin_amdgcn_readlane(rec, WS_K0);
    const int32_t s = (int32_t)__builtin_amdgcn_readlane(rec, WS_SVC);
    if (s >= 0 && (spread_on || aff_on) && ((s_flag[s >> 5] >> (s & 31)) & 1u)) {
      resolved = i;  // a service scalar this pod reads changed in the window
      reason = KSG_STOP_SERVICE;
      break;
    }
    if (__builtin_amdgcn_readlane(rec, WS_ERR)) {
      if (lane == 0) out[i] = KSG_OUT_ERROR;
    } else if (m0 == KSG_S32_NONE || k0 == 0) {
      if (lane == 0) out[i] = KSG_OUT_NOFIT;  // nothing fit at the snapshot; commits only remove fits
    } else {
      const uint32_t npp = __builtin_amdgcn_readlane(rec, WS_NPP), nss = __builtin_amdgcn_readlane(rec, WS_NSS);
      PodCtx c;
      // readlane returns int: widen through uint32_t (no sign extension of the low dword)
      c.req_cpu = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rec, WS_CPU) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rec, WS_CPU + 1) << 32));
      c.req_mem = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rec, WS_MEM) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rec, WS_MEM + 1) << 32));
      c.zero_req = c.req_cpu == 0 && c.req_mem == 0;
      c.spread_max = (int32_t)__builtin_amdgcn_readlane(rec, WS_SMAX);
      c.n_ports = npp & 0xffff;
      c.n_pds = npp >> 16;
      c.n_sel = nss & 0xffff;
      const uint32_t n_svcs = nss >> 16;
      const uint32_t nk = c.n_ports + c.n_pds;
      if (__builtin_amdgcn_readlane(rec, WS_NINL) > KSG_WIN_INLINE || nk > KSG_SLOT_KEYS ||
          n_svcs > KSG_SLOT_SVCS) {
        // lists longer than the record / a slot: the exact per-pod kernel takes it
        resolved = i;
        reason = i == 0 ? KSG_STOP_OVERSIZE : KSG_STOP_SLOT;
        break;
      }
      const RecLists RL{rec, c.n_ports, c.n_ports + c.n_pds};
      KSG_STAMP(6)

      // ---- candidates: snapshot ties committed earlier in this window (T0 ∩ C),
      //      compacted so that 64 lanes re-check 64 of them at a time
      uint32_t cnt = 0;
      uint64_t dmr[P];
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const uint32_t w = q * 64 + lane;
        cnt += __popcll(tw[q] & (w < d.nwords ? s_cmask[w] : 0ULL));
        dmr[q] = 0;
      }
      const uint32_t incl = wave_incl_scan_u32(cnt, lane);
      const uint32_t total = __shfl(incl, 63, 64);
      if (stamp) t_acc[7] += total * 64;
      if (total) {
        uint32_t pos = incl - cnt;
#pragma unroll
        for (int q = 0; q < P; ++q) {
          const uint32_t w = q * 64 + lane;
          uint64_t x = tw[q] & (w < d.nwords ? s_cmask[w] : 0ULL);
          while (x) {
            s_list[pos++] = w * 64 + __builtin_ctzll(x);
            x &= x - 1;
          }
        }
        for (uint32_t base = 0; base < total; base += 64) {
          const uint32_t t = base + lane;
          if (t < total) {
            // the node fit the pod at the snapshot; only the window's deltas can change that
            const WinSlot& S = s_slots[s_slot_of[s_list[t]]];
            const int64_t now_c = (int64_t)((uint64_t)S.snap_c + (uint64_t)S.dc);
            const int64_t now_m = (int64_t)((uint64_t)S.snap_m + (uint64_t)S.dm);
            bool drop = false;
            if (res_on && !c.zero_req) {  // PodFitsResources
              const bool fc = S.cap_c == 0 || (int64_t)((uint64_t)S.cap_c - (uint64_t)now_c) >= c.req_cpu;
              const bool fm = S.cap_m == 0 || (int64_t)((uint64_t)S.cap_m - (uint64_t)now_m) >= c.req_mem;
              drop = !(fc && fm);
            }
            for (uint32_t a = 0; a < S.nk && !drop; ++a) {  // PodFitsPorts / NoDiskConflict
              const uint32_t key = S.keys[a];
              if (ports_on)
                for (uint32_t b = 0; b < c.n_ports; ++b) drop |= RL.port(b) == key;
              if (disk_on)
                for (uint32_t b = 0; b < c.n_pds; ++b) drop |= RL.pd(b) == key;
            }
            if (!drop && d.w_lr) {  // LeastRequested can only fall as requested grows
              const int64_t lr_now = lr_calc((int64_t)((uint64_t)now_c + (uint64_t)c.req_cpu), S.cap_c) +
                                     lr_calc((int64_t)((uint64_t)now_m + (uint64_t)c.req_mem), S.cap_m);
              const int64_t lr_snap = lr_calc((int64_t)((uint64_t)S.snap_c + (uint64_t)c.req_cpu), S.cap_c) +
                                      lr_calc((int64_t)((uint64_t)S.snap_m + (uint64_t)c.req_mem), S.cap_m);
              drop = lr_now / 2 != lr_snap / 2;
            }
            if (!drop && spread_on && s >= 0) {  // ServiceSpreading under an unchanged maxCount
              int32_t delta = 0, snapc = 0;
              for (uint32_t a = 0; a < S.ns; ++a)
                if (S.svcs[a] == (uint32_t)s) {
                  snapc = S.scnt[a];
                  ++delta;
                }
              if (delta) {
                const int64_t mx = c.spread_max;
                drop = frac10_f32(mx - snapc - delta, mx) != frac10_f32(mx - snapc, mx);
              }
            }
            s_dflag[t] = drop ? 1 : 0;
          }
        }
        // each lane rebuilds the dropped bits of its own T0 words: its candidates
        // sit at [incl - cnt, incl) of the list in bit order
        uint32_t idx = incl - cnt;
#pragma unroll
        for (int q = 0; q < P; ++q) {
          const uint32_t w = q * 64 + lane;
          uint64_t x = tw[q] & (w < d.nwords ? s_cmask[w] : 0ULL);
          while (x) {
            const uint32_t b = __builtin_ctzll(x);
            x &= x - 1;
            if (s_dflag[idx++]) dmr[q] |= 1ULL << b;
          }
        }
      }
      KSG_STAMP(2)
      uint32_t dropped = 0;
      uint64_t live[P];
#pragma unroll
      for (int q = 0; q < P; ++q) {
        live[q] = tw[q] & ~dmr[q];
        dropped += __popcll(dmr[q]);
      }
      dropped = wave_sum_u32(dropped);
      const uint64_t k = (uint64_t)k0 - dropped;
      if (k == 0) {
        resolved = i;  // every snapshot tie got worse: needs a fresh snapshot
        reason = KSG_STOP_EXHAUSTED;
        break;
      }
      const uint64_t rng_before = rng;
      const uint64_t r = ksg_splitmix_next(&rng) >> 1;  // rand.Int() (generic_scheduler.go:94)
      const uint64_t target = k - 1 - (r % k);           // ix-th host in descending name order
      uint64_t acc = 0;
      int32_t win = -1;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const uint32_t cq = __popcll(live[q]);
        const uint32_t iq = wave_incl_scan_u32(cq, lane);
        const uint32_t tot = __shfl(iq, 63, 64);
        if (win < 0 && target < acc + tot) {
          const uint32_t excl = iq - cq;
          int32_t cand = -1;
          if (acc + excl <= target && target < acc + iq)
            cand = (int32_t)(d.lo + (q * 64 + lane) * 64 + select_bit(live[q], (uint32_t)(target - acc - excl)));
          const uint64_t own = __ballot(cand >= 0);
          win = __shfl(cand, (int)__builtin_ctzll(own), 64);
        }
        acc += tot;
      }
      KSG_STAMP(3)
      const uint32_t wn = (uint32_t)win;
      const uint32_t woff = wn - d.lo;
      const bool in_c = (s_cmask[woff >> 6] >> (woff & 63)) & 1ULL;
      const uint32_t slot = in_c ? s_slot_of[woff] : n_slots;
      WinSlot& S = s_slots[slot];
      if (in_c && (S.nk + nk > KSG_SLOT_KEYS || S.ns + n_svcs > KSG_SLOT_SVCS)) {
        rng = rng_before;  // this pod is redone (with the same draw) in the next window
        resolved = i;
        reason = KSG_STOP_SLOT;
        break;
      }
      // ---- AssumePod into the window cache; HBM is written back at window end
      const uint32_t base_ns = in_c ? S.ns : 0u;
      if (!in_c) {
        ++n_slots;
        // snapshot loads, retired at the next pod
        if (lane == 0) p_v = d.cap_cpu[wn];
        else if (lane == 1) p_v = d.cap_mem[wn];
        else if (lane == 2) p_v = d.used_cpu[wn];
        else if (lane == 3) p_v = d.used_mem[wn];
      }
      const uint32_t t32 = lane - 32;
      // every lane takes part in the shuffle (bpermute reads inactive lanes as garbage)
      const uint32_t idx_sv = WS_IDS + nk + c.n_sel + (t32 < n_svcs ? t32 : 0u);
      const uint32_t my_sv = (uint32_t)__shfl(rec, (int)(idx_sv < 64 ? idx_sv : 0u), 64);
      if (lane >= 32 && t32 < n_svcs) {
        const uint32_t sv = my_sv;
        p_cnt = d.svc_cnt[(size_t)sv * d.n_nodes + wn];
        p_max = d.svc_max[sv];
        p_peer = d.svc_peer[sv];
      }
      if (lane == 0) {
        if (!in_c) {
          S.node = wn;
          S.nk = 0;
          S.ns = 0;
          S.dc = 0;
          S.dm = 0;
          s_slot_of[woff] = (uint16_t)slot;
          s_cmask[woff >> 6] |= 1ULL << (wn & 63);
        }
        S.dc = (int64_t)((uint64_t)S.dc + (uint64_t)c.req_cpu);
        S.dm = (int64_t)((uint64_t)S.dm + (uint64_t)c.req_mem);
        for (uint32_t t = 0; t < nk; ++t) S.keys[S.nk++] = t < c.n_ports ? RL.port(t) : RL.pd(t - c.n_ports);
        for (uint32_t t = 0; t < n_svcs; ++t) S.svcs[S.ns++] = __builtin_amdgcn_readlane(rec, WS_IDS + nk + c.n_sel + t);
        out[i] = win;
      }
      p_active = true;
      p_new = !in_c;
      p_slot = slot;
      p_base = base_ns;
      p_nsv = n_svcs;
      p_node = wn;
      KSG_STAMP(4)
    }
    rec = recn;
#pragma unroll
    for (int q = 0; q < P; ++q) tw[q] = twn[q];
    KSG_STAMP(5)
  }
  retire();
  if (stamp && lane == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(d.dbgbuf + k, (int32_t)(t_acc[k] / 64));
#undef KSG_STAMP

  // ---- write the window's deltas back to HBM (the next snapshot) -------------
  for (uint32_t t = lane; t < n_slots; t += 64) {
    const WinSlot& S = s_slots[t];
    const uint32_t n = S.node;
    d.used_cpu[n] = (int64_t)((uint64_t)S.snap_c + (uint64_t)S.dc);
    d.used_mem[n] = (int64_t)((uint64_t)S.snap_m + (uint64_t)S.dm);
    for (uint32_t a = 0; a < S.nk; ++a)
      __hip_atomic_fetch_or(d.keymap + (size_t)S.keys[a] * d.nw + (n >> 6), 1ULL << (n & 63), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t a = 0; a < S.ns; ++a) {
      const uint32_t sv = S.svcs[a];
      bool first = true;
      int32_t count = 0;
      for (uint32_t b = 0; b < S.ns; ++b) {
        if (S.svcs[b] == sv) {
          if (b < a) first = false;
          ++count;
        }
      }
      __hip_atomic_fetch_add(d.svc_total + sv, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (first) {
        const int32_t fin = S.scnt[a] + count;
        d.svc_cnt[(size_t)sv * d.n_nodes + n] = fin;
        __hip_atomic_fetch_max(d.svc_max + sv, fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  for (uint32_t t = lane; t < n_peer; t += 64) {
    const uint32_t sv = s_peer[2 * t];
    int32_t expect = -1;
    __hip_atomic_compare_exchange_strong(d.svc_peer + sv, &expect, (int32_t)s_peer[2 * t + 1], __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (lane == 0) {
    *rng_io = rng;
    stat_out[0] = resolved;
    stat_out[1] = reason;
  }
}

hipError_t ksg_launch_win_eval(const KsgDev& d, const ksg_pod* pods, const uint32_t* ids, uint32_t n,
                               KsgWinSum* sums, uint64_t* t0words, hipStream_t st) {
  const size_t lds = (size_t)d.nwords * 64 * sizeof(int32_t);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(ksg_win_eval_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 8 * 1024);
    (void)hipGetLastError();  // do not leave a sticky error behind
    attr_set = true;
  }
  hipLaunchKernelGGL(ksg_win_eval_kernel, dim3(n), dim3(KSG_WIN_NT), lds, st, d, pods, ids, sums, t0words);
  return hipGetLastError();
}

// largest window the resolver's LDS holds for this shard (slots + candidate list)
uint32_t ksg_win_max_window(const KsgDev& d) {
  const uint32_t P = (d.nwords + 63) / 64;
  const size_t fixed = win_lds_fixed(P < 1 ? 1 : P, (d.n_services + 31) / 32, d.hi - d.lo);
  const size_t budget = 150 * 1024;
  if (fixed >= budget) return 0;
  const size_t n = (budget - fixed) / win_lds_per_slot();
  return (uint32_t)(n > 4096 ? 4096 : n);
}

hipError_t ksg_launch_win_resolve(const KsgDev& d, const ksg_pod* pods, const uint32_t* ids, uint32_t n,
                                  const KsgWinSum* sums, const uint64_t* t0words, uint64_t* rng, int32_t* out,
                                  uint32_t* stat, hipStream_t st) {
  const uint32_t P = (d.nwords + 63) / 64;
#define KSG_RES_CASE(PP)                                                                                  \
  if (P <= PP) {                                                                                          \
    static bool once = false;                                                                             \
    if (!once) {                                                                                          \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(ksg_win_resolve_kernel<PP>),               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 8 * 1024);       \
      (void)hipGetLastError();                                                                            \
      once = true;                                                                                        \
    }                                                                                                     \
    const size_t lds = win_lds_fixed(PP, (d.n_services + 31) / 32, d.hi - d.lo) + (size_t)n * win_lds_per_slot(); \
    hipLaunchKernelGGL(ksg_win_resolve_kernel<PP>, dim3(1), dim3(64), lds, st, d, pods, ids, n, sums, t0words, \
                       rng, out, stat);                                                                   \
    return hipGetLastError();                                                                             \
  }
  KSG_RES_CASE(1)
  KSG_RES_CASE(2)
  KSG_RES_CASE(4)
  KSG_RES_CASE(8)
#undef KSG_RES_CASE
  return hipErrorInvalidValue;
}
