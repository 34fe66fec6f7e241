// ksg_serve.hip — the resident drop-in server behind ksg_schedule_begin /
// ksg_schedule_commit (include/kschedgpu.h).
//
// The reference schedules one pod per call: scheduleOne (plugin/pkg/scheduler/
// scheduler.go:86-118) calls genericScheduler.Schedule (pkg/scheduler/
// generic_scheduler.go:54-96), which filters and scores every node and draws
// random.Int() only when some node fits. The C ABI splits that call in two
// (begin: filter + score + {max, tie count}; commit: the caller's tie index →
// node + AssumePod's delta) so the caller keeps its own *rand.Rand.
//
// Launching kernels per call costs more than the work (round 2: scan + decide
// launches, a copy in and two stream syncs, 42 us per pod at 5,000 nodes). Here
// one workgroup of KSG_NT threads stays resident between calls and serves
// requests from pinned host memory mapped into the device (KsgSrvBox,
// ksg_internal.h):
//   * wave 0 polls the 1-KB request block with one 16-B-per-lane load per
//     round trip; a request is complete when every 16-B chunk carries its
//     sequence number, so the pod travels with the poll that finds it;
//   * BEGIN: the exact one-pod scan of ksg_batch_kernel (ksg_exact.h) over the
//     node state in HBM (capacity and requested totals cached in registers for
//     R <= 2), the block max and tie ballots into LDS; the response
//     {seq, tie count, max} is one 16-B store into host memory;
//   * COMMIT: the ix-th tie from the top (generic_scheduler.go:88-95) from the
//     tie words still in LDS, the node's response first, then AssumePod's delta
//     (commit_pod_wave) before the next request is read. A COMMIT for a begin
//     whose scan is no longer in LDS (a new server instance) rescans the pod
//     the host left in the block;
//   * PATCH: the host mirror's queued deltas (ksg_add_pod / ksg_remove_pod),
//     applied in order by one lane, then the cached totals reloaded;
//   * after idle_ticks without a request the kernel returns; the host relaunches
//     it with the next request (every wait has that exit).
// No stream operation can run while the server is resident: every other entry
// point stops it first (KSG_SRV_EXIT), see ksg_runtime.cpp srv_stop.
#include <hip/hip_runtime.h>
#include "ksg_internal.h"

#include "ksg_device.h"
#include "ksg_exact.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef KSG_SRV_G
#define KSG_SRV_G 2  // nodes per thread whose loads the plain scan issues together
#endif

// host-memory access: system scope (no cache keeps a stale copy)
__device__ __forceinline__ u32x4 sys_ld16(const uint32_t* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void sys_st16(uint32_t* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t sys_ld32(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t sys_ld64(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void respond(const KsgSrvArgs& a, uint32_t seq, uint32_t x, uint32_t y, uint32_t z) {
  u32x4 v;
  v.x = seq;
  v.y = x;
  v.z = y;
  v.w = z;
  sys_st16(a.box->resp, v);
}

// A BEGIN / COMMIT request's payload layout in range: no request can make the
// server read outside its LDS copy of the request (the ids' values are checked
// by the host, check_pod). Wave-uniform, every thread computes it.
__device__ __forceinline__ bool req_bad(const KsgDev& d, const uint32_t* s_req) {
  const uint32_t paydw = s_req[KSG_SRVH_PAYDW], ids_at = s_req[KSG_SRVH_IDS_AT], ext_at = s_req[KSG_SRVH_EXT_AT];
  const bool has_ext = (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_EXT) != 0;
  constexpr uint32_t pod_dw = sizeof(ksg_pod) / 4, ext_dw = sizeof(ksg_pod_ext) / 4;
  if (paydw > KSG_SRV_PAY_DW || ids_at < pod_dw || ids_at > paydw ||
      (has_ext && ((ext_at & 1u) || ext_at < ids_at || (uint64_t)ext_at + ext_dw > paydw)))
    return true;
  const ksg_pod& p = *reinterpret_cast<const ksg_pod*>(s_req + KSG_SRV_HDR_DW);
  const uint64_t nid = (has_ext ? ext_at : paydw) - ids_at;
  bool bad = (uint64_t)p.ports_off + p.n_ports > nid || (uint64_t)p.pds_off + p.n_pds > nid ||
             (uint64_t)p.sel_off + p.n_sel > nid || (uint64_t)p.svcs_off + p.n_svcs > nid ||
             p.host < -2 || p.host >= (int32_t)d.n_nodes || p.service < -1 || p.service >= (int32_t)d.n_services;
  if (has_ext) {
    const ksg_pod_ext& e = *reinterpret_cast<const ksg_pod_ext*>(s_req + KSG_SRV_HDR_DW + ext_at);
    bad |= (uint64_t)e.hard_off + e.n_hard > nid || (uint64_t)e.soft_off + e.n_soft > nid;
  }
  return bad;
}

// calculateScore (priorities.go:27-37) through the f64 reciprocal (lr_win)
// where that form is exact, lr_calc elsewhere
__device__ __forceinline__ int32_t lr_fast(int64_t req, int64_t cap, double inv10) {
  if (cap > 0 && cap <= KSG_WIN_LR_BOUND && req >= 0 && req <= KSG_WIN_LR_BOUND) return lr_win(req, cap, inv10);
  return (int32_t)lr_calc(req, cap);
}

// Filter + score of the shard for one pod without ServiceAntiAffinity or
// extensions, shaped for latency (each dependent L2 round trip costs ~1.3k
// cycles on the server's one CU; node_fail_l's early returns chain one per
// predicate and per list entry):
//  1. one thread per 64-node word folds the word of every predicate bitmap the
//     pod touches (LabelsPresence, nodeSelector pairs, PD and host-port keys,
//     ServiceAffinity pairs) into five masks in LDS, issuing up to 8 row loads
//     before waiting;
//  2. every thread takes G of its nodes at a time, issues all their loads
//     (requested and capacity totals, 10 / capacity, static score, service
//     count), then tests and scores them against the word masks.
// Same fail code order (node_fail_l) and score (node_score) as every other
// kernel. The server takes only int32-score contexts (|combined score| <
// 2^30, no wrap), so the sum is int32; LeastRequested goes through lr_fast and
// ServiceSpreading's int(10 * float32(max - cnt) / float32(max)) through the
// pod's table s_tab[cnt] (cnt < n_tab; the direct form past it).
enum { WM_LP = 0, WM_SEL, WM_PD, WM_PORT, WM_AFF, WM_N };

__device__ __forceinline__ void word_masks(const KsgDev& d, const PodCtx& c, uint32_t q, uint64_t* s_wm,
                                           uint32_t nwq) {
  const uint32_t P = d.preds;
  const uint32_t wi = (d.lo >> 6) + q;
  const uint32_t n_sel = (P & KSG_PRED_MATCHNODESELECTOR) ? c.n_sel : 0;
  const uint32_t n_pd = (P & KSG_PRED_NODISKCONFLICT) ? c.n_pds : 0;
  const uint32_t n_port = (P & KSG_PRED_PODFITSPORTS) ? c.n_ports : 0;
  uint32_t n_aff = 0;
  if (P & KSG_PRED_SERVICEAFFINITY)
#pragma unroll
    for (uint32_t j = 0; j < KSG_MAX_AFF; ++j) n_aff += (j < d.n_aff && c.req_aff[j] >= 0) ? 1u : 0u;
  const uint32_t e1 = n_sel, e2 = e1 + n_pd, e3 = e2 + n_port, total = e3 + n_aff;
  uint64_t m_lp = d.has_static_fit ? d.static_fit[wi] : ~0ULL, m_sel = ~0ULL, m_pd = 0, m_port = 0, m_aff = ~0ULL;
  for (uint32_t e0 = 0; e0 < total; e0 += 8) {
    uint64_t x[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
      const uint32_t e = e0 + i;
      x[i] = 0;
      if (e < total) {
        uint32_t id;
        const uint64_t* base = d.pairmap;
        if (e < e1) {
          id = c.sel[e];
        } else if (e < e2) {
          id = c.pds[e - e1];
          base = d.keymap;
        } else if (e < e3) {
          id = c.ports[e - e2];
          base = d.keymap;
        } else {  // the (e - e3)-th ServiceAffinity requirement
          const uint32_t k = e - e3;
          uint32_t seen = 0;
          id = 0;
#pragma unroll
          for (uint32_t j = 0; j < KSG_MAX_AFF; ++j)
            if (j < d.n_aff && c.req_aff[j] >= 0) {
              if (seen == k) id = (uint32_t)c.req_aff[j];
              ++seen;
            }
        }
        x[i] = ld_mut(base + (size_t)id * d.nw + wi);  // (keymap is mutable; one load form for all rows)
      }
    }
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
      const uint32_t e = e0 + i;
      if (e < e1) m_sel &= x[i];
      else if (e < e2) m_pd |= x[i];
      else if (e < e3) m_port |= x[i];
      else if (e < total) m_aff &= x[i];
    }
  }
  s_wm[WM_LP * nwq + q] = m_lp;
  s_wm[WM_SEL * nwq + q] = m_sel;
  s_wm[WM_PD * nwq + q] = m_pd;
  s_wm[WM_PORT * nwq + q] = m_port;
  s_wm[WM_AFF * nwq + q] = m_aff;
}

template <int R, bool REG, int G>
__device__ __forceinline__ int32_t serve_scan_plain(const KsgDev& d, const PodCtx& c, uint32_t tid, uint32_t wave,
                                                    uint64_t bit, int32_t* s_score, uint8_t* fail_out,
                                                    const int64_t* rcapc, const int64_t* rcapm,
                                                    const int64_t* rusedc, const int64_t* rusedm,
                                                    const int32_t* s_tab, int32_t n_tab, uint64_t* s_wm) {
  constexpr uint32_t NWQ = R * KSG_NWAVE;  // words of the shard a thread's nodes can fall in
  const uint32_t nwq = min(NWQ, (d.hi - d.lo + 63) >> 6);
  if (tid < nwq) word_masks(d, c, tid, s_wm, NWQ);
  const uint32_t P = d.preds;
  const bool need_cnt = d.w_spread != 0 && c.svc >= 0 && !d.equal_fallback;
  const bool res_on = (P & KSG_PRED_PODFITSRESOURCES) && !c.zero_req;
  int32_t m = KSG_S32_NONE;
  __syncthreads();
#pragma unroll 1
  for (int j0 = 0; j0 < R; j0 += G) {
    if (d.lo + (uint32_t)j0 * KSG_NT >= d.hi) break;  // (uniform) the rest of the shard is empty
    int64_t capc[G], capm[G], usedc[G], usedm[G];
    double invc[G], invm[G];
    int32_t cnt[G], ss[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t j = j0 + g;
      const uint32_t n = d.lo + j * KSG_NT + tid;
      const uint32_t nn = n < d.hi ? n : d.lo;
      if constexpr (REG) {
        capc[g] = rcapc[j];
        capm[g] = rcapm[j];
        usedc[g] = rusedc[j];
        usedm[g] = rusedm[j];
      } else {
        capc[g] = d.cap_cpu[nn];
        capm[g] = d.cap_mem[nn];
        usedc[g] = ld_mut(d.used_cpu + nn);
        usedm[g] = ld_mut(d.used_mem + nn);
      }
      invc[g] = d.w_lr ? d.inv10_cpu[nn] : 0.0;
      invm[g] = d.w_lr ? d.inv10_mem[nn] : 0.0;
      ss[g] = d.has_static_score ? (int32_t)d.static_score[nn] : 0;
      cnt[g] = need_cnt ? ld_mut(d.svc_cnt + (size_t)c.svc * d.n_nodes + nn) : 0;
    }
    // branch-free per node: every predicate's verdict, the first failing one
    // by selects, the score computed for every node and kept where it fits
    // (branches serialise each wave on its LDS / compare chain)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t j = j0 + g;
      const uint32_t n = d.lo + j * KSG_NT + tid;
      const uint32_t q = j * KSG_NWAVE + wave;
      const uint64_t w_lp = s_wm[WM_LP * NWQ + q], w_sel = s_wm[WM_SEL * NWQ + q], w_pd = s_wm[WM_PD * NWQ + q],
                     w_port = s_wm[WM_PORT * NWQ + q], w_aff = s_wm[WM_AFF * NWQ + q];
      const bool host_bad = (P & KSG_PRED_HOSTNAME) && c.host != -1 && (int32_t)n != c.host;
      const bool res_bad = res_on && !((capc[g] == 0 || (int64_t)((uint64_t)capc[g] - (uint64_t)usedc[g]) >= c.req_cpu) &&
                                       (capm[g] == 0 || (int64_t)((uint64_t)capm[g] - (uint64_t)usedm[g]) >= c.req_mem));
      int f = (w_aff & bit) ? KSG_FAIL_NONE : KSG_FAIL_SERVICEAFFINITY;
      f = res_bad ? KSG_FAIL_PODFITSRESOURCES : f;
      f = (w_port & bit) ? KSG_FAIL_PODFITSPORTS : f;
      f = (w_pd & bit) ? KSG_FAIL_NODISKCONFLICT : f;
      f = (w_sel & bit) ? f : KSG_FAIL_MATCHNODESELECTOR;
      f = (w_lp & bit) ? f : KSG_FAIL_LABELSPRESENCE;
      f = host_bad ? KSG_FAIL_HOSTNAME : f;
      int32_t s = ss[g];
      if (d.w_lr) {
        const int64_t tc = (int64_t)((uint64_t)usedc[g] + (uint64_t)c.req_cpu);
        const int64_t tm = (int64_t)((uint64_t)usedm[g] + (uint64_t)c.req_mem);
        s += (int32_t)d.w_lr * ((lr_fast(tc, capc[g], invc[g]) + lr_fast(tm, capm[g], invm[g])) / 2);
      }
      if (d.w_spread) {
        int32_t sp = 10;
        if (c.spread_max > 0) {
          const uint32_t ct = (uint32_t)cnt[g] < (uint32_t)n_tab ? (uint32_t)cnt[g] : 0u;
          sp = s_tab[ct];
          if ((uint32_t)cnt[g] >= (uint32_t)n_tab)  // (past the table: rare)
            sp = (int32_t)frac10_f32((int64_t)c.spread_max - cnt[g], c.spread_max);
        }
        s += (int32_t)d.w_spread * sp;
      }
      s = d.equal_fallback ? 1 : s;  // EqualPriority (generic_scheduler.go:141-143,180-195)
      const bool valid = n < d.hi;
      if (fail_out && valid) fail_out[n - d.lo] = (uint8_t)f;
      const int32_t sc = (valid && f == KSG_FAIL_NONE) ? s : KSG_S32_NONE;
      s_score[j * KSG_NT + tid] = sc;
      m = sc > m ? sc : m;
    }
  }
  // (the groups past the shard's end, skipped above, score nothing)
#pragma unroll 1
  for (int j = 0; j < R; ++j)
    if (d.lo + (uint32_t)(j - j % G) * KSG_NT >= d.hi) s_score[j * KSG_NT + tid] = KSG_S32_NONE;
  return m;
}

template <int R, bool ANTI, bool EXT, bool REG>
__global__ __launch_bounds__(KSG_NT) void ksg_serve_kernel(KsgDev d, KsgSrvArgs a) {
  using SC = int32_t;
  using T = ScoreT<SC>;
  static_assert(R <= KSG_SRV_MAX_R, "server shard too large");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // dynamic LDS: scores, anti-affinity domain counts, the TaintToleration max,
  // fail codes, the request (header + payload)
  SC* s_score = reinterpret_cast<SC*>(smem);
  int32_t* s_dcount = reinterpret_cast<int32_t*>(s_score + R * KSG_NT);
  int32_t* s_tmax = s_dcount + d.n_domains_total;
  uint8_t* s_fail = reinterpret_cast<uint8_t*>(smem) + (((size_t)R * KSG_NT * sizeof(SC) +
                                                         (size_t)d.n_domains_total * 4 + 16 + 15) & ~(size_t)15);
  uint32_t* s_req = reinterpret_cast<uint32_t*>(s_fail + (size_t)R * KSG_NT);
  int32_t* s_tab = reinterpret_cast<int32_t*>(s_req + KSG_SRV_HDR_DW + KSG_SRV_PAY_DW);  // ServiceSpreading table
  uint64_t* s_wm = reinterpret_cast<uint64_t*>(s_tab + KSG_NT);  // the pod's word masks [WM_N][R * 16]
  __shared__ uint64_t s_tie[R * KSG_NWAVE];
  __shared__ SC s_wmax[KSG_NWAVE];
  __shared__ uint32_t s_wcnt[KSG_NWAVE];
  __shared__ uint32_t s_kind;
  __shared__ int32_t s_winner;
  __shared__ KsgPatch s_pt[64];

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t bit = 1ULL << lane;

  int64_t rcapc[REG ? R : 1], rcapm[REG ? R : 1], rusedc[REG ? R : 1], rusedm[REG ? R : 1];
  auto load_totals = [&]() {
    if constexpr (REG) {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const uint32_t n = d.lo + j * KSG_NT + tid;
        const bool v = n < d.hi;
        rcapc[j] = v ? d.cap_cpu[n] : 0;
        rcapm[j] = v ? d.cap_mem[n] : 0;
        rusedc[j] = v ? ld_mut(d.used_cpu + n) : 0;
        rusedm[j] = v ? ld_mut(d.used_mem + n) : 0;
      }
    }
  };
  load_totals();

  // KsgSrvArgs.stamps: s_memtime at the stages of each BEGIN (thread 0), written
  // to resp[4..11] before the response (ksg_runtime.cpp sums them)
  uint64_t st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto stamp = [&](int i) {
    if (a.stamps && tid == 0) st_[i] = __builtin_amdgcn_s_memtime();
  };
  uint32_t seq = a.start_seq + 1;
  uint32_t pend = 0;    // the begin whose scan (M, k, s_tie) is in LDS; 0: none
  SC M = T::none;
  uint32_t k = 0;
  bool err = false;

  // filter + score the pod in s_req into s_score / s_tie (every thread)
  auto scan = [&](bool want_fail) {
    const uint32_t* pay = s_req + KSG_SRV_HDR_DW;
    const ksg_pod& p = *reinterpret_cast<const ksg_pod*>(pay);
    const uint32_t* ids = pay + s_req[KSG_SRVH_IDS_AT];
    const ksg_pod_ext* ext = (EXT && (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_EXT))
                                 ? reinterpret_cast<const ksg_pod_ext*>(pay + s_req[KSG_SRVH_EXT_AT])
                                 : nullptr;
    PodCtx c;
    pod_resolve(d, p, ids, c);
    c.ext = ext;
    err = c.error != 0;
    stamp(3);
    if (err) {
      M = T::none;
      k = 0;
      return;
    }
    if (ANTI || ext) {
      for (uint32_t q = tid; q < d.n_domains_total; q += KSG_NT) s_dcount[q] = 0;
      if (tid == 0) *s_tmax = 0;
      __syncthreads();
    }
    SC m;
    if constexpr (!ANTI && !EXT) {
      // the pod's ServiceSpreading scores by count (counts never exceed max)
      int32_t n_tab = 0;
      if (d.w_spread && c.svc >= 0 && c.spread_max > 0 && !d.equal_fallback) {
        n_tab = c.spread_max >= KSG_NT ? KSG_NT : c.spread_max + 1;
        if ((int32_t)tid < n_tab) s_tab[tid] = (int32_t)frac10_f32((int64_t)c.spread_max - (int32_t)tid, c.spread_max);
        __syncthreads();
      }
      m = serve_scan_plain<R, REG, (R < KSG_SRV_G ? R : KSG_SRV_G)>(d, c, tid, wave, bit, s_score,
                                                                    want_fail ? s_fail : nullptr, rcapc, rcapm,
                                                                    rusedc, rusedm, s_tab, n_tab, s_wm);
    }
    else
      m = scan_pod<R, ANTI, REG, SC, (R <= 8)>(d, c, tid, wave, bit, s_score, s_dcount, nullptr, rcapc, rcapm, rusedc,
                                               rusedm, want_fail ? s_fail : nullptr, ext ? s_tmax : nullptr);
    stamp(4);
    uint64_t kk;
    reduce_ties<R, SC>(d, m, tid, lane, wave, s_score, s_wmax, s_wcnt, s_tie, M, kk);
    stamp(5);
    k = M == T::none ? 0 : (uint32_t)kk;
  };

  for (;;) {
    __syncthreads();  // every wave is done with the previous request's LDS
    // ---- wave 0 waits for request `seq`: every chunk's tag equal to it ----
    if (wave == 0) {
      const uint64_t t0 = wall_clock64();
      u32x4 v;
      bool ok = false;
      for (;;) {
        v = sys_ld16(a.box->req + lane * 4);
        if (__ballot(v.w != seq) == 0) {
          ok = true;
          break;
        }
        if (wall_clock64() - t0 > a.idle_ticks) break;
      }
      if (ok) {
        s_req[lane * KSG_SRV_CHUNK_DW + 0] = v.x;
        s_req[lane * KSG_SRV_CHUNK_DW + 1] = v.y;
        s_req[lane * KSG_SRV_CHUNK_DW + 2] = v.z;
      }
      if (lane == 0) s_kind = ok ? v.x : 0u;  // chunk 0's first dword is the header's kind
      stamp(0);
    }
    __syncthreads();
    stamp(1);
    const uint32_t kind = s_kind;
    if (kind == 0 || kind > KSG_SRV_EXIT) break;  // idle: return (the host relaunches)
    if (kind == KSG_SRV_EXIT) {
      if (tid == 0) respond(a, seq, 0, 0, 0);
      break;
    }
    if (kind == KSG_SRV_PATCH) {
      // in order by one lane, as ksg_patch_kernel; 64 patches per round trip
      const uint32_t np = s_req[KSG_SRVH_NPATCH];
      if (wave == 0) {
        for (uint32_t base = 0; base < np; base += 64) {
          if (base + lane < np) {
            const KsgPatch* src = a.box->patch + base + lane;
            KsgPatch pt;
            pt.addr = sys_ld64(&src->addr);
            pt.value = sys_ld64(&src->value);
            pt.width = sys_ld32(&src->width);
            s_pt[lane] = pt;
          }
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
          if (lane == 0) {
            const uint32_t m = min(64u, np - base);
            for (uint32_t q = 0; q < m; ++q) {
              const KsgPatch pt = s_pt[q];
              switch (pt.width) {
                case 0: *reinterpret_cast<uint32_t*>(pt.addr) = (uint32_t)pt.value; break;
                case 1: *reinterpret_cast<uint64_t*>(pt.addr) = pt.value; break;
                case 2: *reinterpret_cast<uint64_t*>(pt.addr) |= pt.value; break;
                case 3: *reinterpret_cast<uint64_t*>(pt.addr) &= ~pt.value; break;
              }
            }
          }
          __builtin_amdgcn_wave_barrier();
        }
        drain_stores();
      }
      __syncthreads();
      load_totals();  // (agent-scope loads: L2 holds the patched values)
      pend = 0;
      if (tid == 0) respond(a, seq, 0, 0, 0);
      ++seq;
      continue;
    }
    // ---- BEGIN / COMMIT: the pod's payload beyond the block ----
    const bool begin = kind == KSG_SRV_BEGIN;
    const bool rescan = begin || pend != s_req[KSG_SRVH_BSEQ];
    if (rescan) {
      const uint32_t paydw = min(s_req[KSG_SRVH_PAYDW], (uint32_t)KSG_SRV_PAY_DW);
      if (paydw > KSG_SRV_INLINE_DW) {
        for (uint32_t t = tid; t < paydw - KSG_SRV_INLINE_DW; t += KSG_NT)
          s_req[KSG_SRV_HDR_DW + KSG_SRV_INLINE_DW + t] = sys_ld32(a.box->ext + t);
        __syncthreads();
      }
    }
    const bool bad = req_bad(d, s_req);
    stamp(2);
    if (bad) {  // (never, unless the host side has a bug)
      if (tid == 0) respond(a, seq, KSG_SRV_BADREQ, 0, 0);
      pend = 0;
      ++seq;
      continue;
    }
    if (rescan) {
      const bool want_fail = begin && (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_WANT_FAIL);
      scan(want_fail);
      pend = begin ? seq : s_req[KSG_SRVH_BSEQ];
      if (begin) {
        if (want_fail && !err) {  // the shard's fail codes into host memory, then the response
          const uint32_t nb = d.hi - d.lo;
          for (uint32_t t = tid * 4; t < nb; t += KSG_NT * 4) {
            if (t + 4 <= nb) {
              *reinterpret_cast<volatile uint32_t*>(a.fail + t) = *reinterpret_cast<const uint32_t*>(s_fail + t);
            } else {
              for (uint32_t u = t; u < nb; ++u) reinterpret_cast<volatile uint8_t*>(a.fail)[u] = s_fail[u];
            }
          }
          drain_stores();
          __syncthreads();
        }
        if (tid == 0) {
          if (a.stamps) {  // stage cycles: request seen->LDS, check, resolve, scan, reduce, fail codes
            stamp(6);
            u32x4 x0, x1;
            x0.x = (uint32_t)(st_[1] - st_[0]);
            x0.y = (uint32_t)(st_[2] - st_[1]);
            x0.z = (uint32_t)(st_[3] - st_[2]);
            x0.w = (uint32_t)(st_[4] - st_[3]);
            x1.x = (uint32_t)(st_[5] - st_[4]);
            x1.y = (uint32_t)(st_[6] - st_[5]);
            x1.z = seq;
            x1.w = 0;
            sys_st16(a.box->resp + 4, x0);
            sys_st16(a.box->resp + 8, x1);
          }
          const int64_t m64 = (int64_t)M;
          respond(a, seq, err ? ~0u : k, (uint32_t)(uint64_t)m64, (uint32_t)((uint64_t)m64 >> 32));
        }
        ++seq;
        continue;
      }
    }
    // ---- COMMIT: the tie_index-th tie from the top, then AssumePod's delta ----
    const uint32_t tie = s_req[KSG_SRVH_TIE];
    if (wave == 0) {
      int32_t win = -1;
      if (!err && k > 0 && tie < k) win = select_tie(s_tie, R * KSG_NWAVE, (uint64_t)(k - 1 - tie), lane, d.lo);
      if (lane == 0) {
        respond(a, seq, (uint32_t)win, 0, 0);
        s_winner = win;
      }
      if (win >= 0) {
        const uint32_t* pay = s_req + KSG_SRV_HDR_DW;
        const ksg_pod& p = *reinterpret_cast<const ksg_pod*>(pay);
        const uint32_t* ids = pay + s_req[KSG_SRVH_IDS_AT];
        const ksg_pod_ext* ext = (EXT && (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_EXT))
                                     ? reinterpret_cast<const ksg_pod_ext*>(pay + s_req[KSG_SRVH_EXT_AT])
                                     : nullptr;
        commit_pod_wave(d, p, ids, (uint32_t)win, lane, ext);
      }
      drain_stores();
    }
    __syncthreads();
    if constexpr (REG) {
      const int32_t w = s_winner;
      if (w >= 0) {
        const ksg_pod& p = *reinterpret_cast<const ksg_pod*>(s_req + KSG_SRV_HDR_DW);
        const uint32_t off = (uint32_t)w - d.lo;
        const uint32_t jw = off / KSG_NT, tw = off % KSG_NT;
#pragma unroll
        for (int j = 0; j < R; ++j)
          if ((uint32_t)j == jw && tid == tw) {
            rusedc[j] = (int64_t)((uint64_t)rusedc[j] + (uint64_t)p.milli_cpu);
            rusedm[j] = (int64_t)((uint64_t)rusedm[j] + (uint64_t)p.memory);
          }
      }
    }
    pend = 0;
    ++seq;
  }
}

// ---- launch wrapper --------------------------------------------------------
size_t ksg_serve_lds(int R, const KsgDev& d) {
  return (((size_t)R * KSG_NT * sizeof(int32_t) + (size_t)d.n_domains_total * 4 + 16 + 15) & ~(size_t)15) +
         (size_t)R * KSG_NT + (size_t)(KSG_SRV_HDR_DW + KSG_SRV_PAY_DW) * 4 + (size_t)KSG_NT * 4 +
         (size_t)WM_N * R * KSG_NWAVE * 8;
}

template <int R, bool ANTI, bool EXT>
static hipError_t launch_serve_t(const KsgDev& d, const KsgSrvArgs& a, hipStream_t st) {
  constexpr bool REG = R <= 2;  // (R = 4, 8 with cached totals spill at 1024 threads)
  static bool once = ((void)hipFuncSetAttribute(reinterpret_cast<const void*>(ksg_serve_kernel<R, ANTI, EXT, REG>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 8 * 1024),
                      (void)hipGetLastError(), true);
  (void)once;
  hipLaunchKernelGGL((ksg_serve_kernel<R, ANTI, EXT, REG>), dim3(1), dim3(KSG_NT), ksg_serve_lds(R, d), st, d, a);
  return hipGetLastError();
}

template <bool ANTI, bool EXT>
static hipError_t launch_serve_a(int R, const KsgDev& d, const KsgSrvArgs& a, hipStream_t st) {
  switch (R) {
    case 1: return launch_serve_t<1, ANTI, EXT>(d, a, st);
    case 2: return launch_serve_t<2, ANTI, EXT>(d, a, st);
    case 4: return launch_serve_t<4, ANTI, EXT>(d, a, st);
    case 8: return launch_serve_t<8, ANTI, EXT>(d, a, st);
    case 16: return launch_serve_t<16, ANTI, EXT>(d, a, st);
  }
  return hipErrorInvalidValue;
}

// anti: ServiceAntiAffinity priorities; ext: a context with extensions (ksg_set_extensions)
hipError_t ksg_launch_serve(int R, bool anti, bool ext, const KsgDev& d, const KsgSrvArgs& a, hipStream_t st) {
  if (ext) return anti ? launch_serve_a<true, true>(R, d, a, st) : launch_serve_a<false, true>(R, d, a, st);
  return anti ? launch_serve_a<true, false>(R, d, a, st) : launch_serve_a<false, false>(R, d, a, st);
}
