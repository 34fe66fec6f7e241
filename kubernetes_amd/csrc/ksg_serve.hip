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
// two 16-B loads in flight together (the one-workgroup server polls both request blocks)
__device__ __forceinline__ void sys_ld16x2(const uint32_t* p, const uint32_t* q, u32x4& v, u32x4& u) {
  asm volatile("global_load_dwordx4 %0, %2, off sc0 sc1\n\tglobal_load_dwordx4 %1, %3, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=&v"(v), "=&v"(u) : "v"(p), "v"(q) : "memory");
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
// A rejected request: its sequence number into resp[KSG_SRV_RESP_REJECTED] before the
// response (a COMMIT is not waited for, and later answers overwrite resp[0..3]; the host
// checks this word when it settles the COMMIT)
__device__ __forceinline__ void respond_rejected(const KsgSrvArgs& a, uint32_t seq) {
  u32x4 r;
  r.x = seq;
  r.y = r.z = r.w = 0;
  sys_st16(a.box->resp + KSG_SRV_RESP_REJECTED, r);
  respond(a, seq, KSG_SRV_BADREQ, 0, 0);
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
enum { WM_LP = 0, WM_SEL, WM_PD, WM_PORT, WM_AFF, WM_TAINT, WM_N };

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
  // (extensions: the pod's untolerated NoSchedule / NoExecute taints, taintmap rows)
  const uint32_t n_taint = (c.ext && (d.ext_filters & KSG_EXT_TAINTS)) ? c.ext->n_hard : 0;
  const uint32_t e1 = n_sel, e2 = e1 + n_pd, e3 = e2 + n_port, e4 = e3 + n_aff, total = e4 + n_taint;
  uint64_t m_lp = d.has_static_fit ? d.static_fit[wi] : ~0ULL, m_sel = ~0ULL, m_pd = 0, m_port = 0, m_aff = ~0ULL;
  uint64_t m_taint = 0;
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
        } else if (e >= e4) {
          id = c.ids[c.ext->hard_off + (e - e4)];
          base = d.taintmap;
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
      else if (e < e4) m_aff &= x[i];
      else if (e < total) m_taint |= x[i];
    }
  }
  s_wm[WM_LP * nwq + q] = m_lp;
  s_wm[WM_SEL * nwq + q] = m_sel;
  s_wm[WM_PD * nwq + q] = m_pd;
  s_wm[WM_PORT * nwq + q] = m_port;
  s_wm[WM_AFF * nwq + q] = m_aff;
  s_wm[WM_TAINT * nwq + q] = m_taint;
}

// One node of the plain scan, branch-free: every predicate's verdict from the
// word masks and the resource totals, the first failing one by selects
// (node_fail_l's order), the score computed regardless (node_score; int32, the
// server's contexts keep |score| < 2^30) and kept by the caller where f == 0.
__device__ __forceinline__ int32_t eval_node(const KsgDev& d, const PodCtx& c, uint32_t n, uint64_t bit,
                                             const uint64_t* s_wm, uint32_t nwq, uint32_t q, bool res_on,
                                             int64_t capc, int64_t capm, int64_t usedc, int64_t usedm, double invc,
                                             double invm, int32_t ss, int32_t cnt, const int32_t* s_tab,
                                             int32_t n_tab, int& f) {
  const uint32_t P = d.preds;
  const uint64_t w_lp = s_wm[WM_LP * nwq + q], w_sel = s_wm[WM_SEL * nwq + q], w_pd = s_wm[WM_PD * nwq + q],
                 w_port = s_wm[WM_PORT * nwq + q], w_aff = s_wm[WM_AFF * nwq + q];
  const bool host_bad = (P & KSG_PRED_HOSTNAME) && c.host != -1 && (int32_t)n != c.host;
  const bool res_bad = res_on && !((capc == 0 || (int64_t)((uint64_t)capc - (uint64_t)usedc) >= c.req_cpu) &&
                                   (capm == 0 || (int64_t)((uint64_t)capm - (uint64_t)usedm) >= c.req_mem));
  int fx = KSG_FAIL_NONE;  // extensions (node_fail_l's order: after the reference's predicates)
  if (c.ext) {
    if ((d.ext_filters & KSG_EXT_SCALAR) && n < d.hi)
      for (uint32_t r = 0; r < d.n_scalar; ++r) {
        const int64_t req = c.ext->scalar[r];
        if (req > 0) {
          const int64_t cap = d.scalar_cap[(size_t)r * d.n_nodes + n];
          const int64_t used = ld_mut(d.scalar_used + (size_t)r * d.n_nodes + n);
          if (cap < (int64_t)((uint64_t)used + (uint64_t)req)) fx = KSG_FAIL_SCALAR;
        }
      }
    if (s_wm[WM_TAINT * nwq + q] & bit) fx = KSG_FAIL_TAINTS;
  }
  f = (w_aff & bit) ? fx : KSG_FAIL_SERVICEAFFINITY;
  f = res_bad ? KSG_FAIL_PODFITSRESOURCES : f;
  f = (w_port & bit) ? KSG_FAIL_PODFITSPORTS : f;
  f = (w_pd & bit) ? KSG_FAIL_NODISKCONFLICT : f;
  f = (w_sel & bit) ? f : KSG_FAIL_MATCHNODESELECTOR;
  f = (w_lp & bit) ? f : KSG_FAIL_LABELSPRESENCE;
  f = host_bad ? KSG_FAIL_HOSTNAME : f;
  int32_t s = ss;
  if (d.w_lr) {
    const int64_t tc = (int64_t)((uint64_t)usedc + (uint64_t)c.req_cpu);
    const int64_t tm = (int64_t)((uint64_t)usedm + (uint64_t)c.req_mem);
    s += (int32_t)d.w_lr * ((lr_fast(tc, capc, invc) + lr_fast(tm, capm, invm)) / 2);
  }
  if (d.w_spread) {
    int32_t sp = 10;
    if (c.spread_max > 0) {
      const uint32_t ct = (uint32_t)cnt < (uint32_t)n_tab ? (uint32_t)cnt : 0u;
      sp = s_tab[ct];
      if ((uint32_t)cnt >= (uint32_t)n_tab)  // (past the table: rare)
        sp = (int32_t)frac10_f32((int64_t)c.spread_max - cnt, c.spread_max);
    }
    s += (int32_t)d.w_spread * sp;
  }
  if (c.ext && d.w_bal) {  // extension: BalancedResourceAllocation (int32: the score bound covers it)
    const int64_t tc = (int64_t)((uint64_t)usedc + (uint64_t)c.req_cpu);
    const int64_t tm = (int64_t)((uint64_t)usedm + (uint64_t)c.req_mem);
    s += (int32_t)d.w_bal * (int32_t)balanced_score(tc, capc, tm, capm);
  }
  return d.equal_fallback ? 1 : s;  // EqualPriority (generic_scheduler.go:141-143,180-195)
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
      int f;
      const int32_t s = eval_node(d, c, n, bit, s_wm, NWQ, q, res_on, capc[g], capm[g], usedc[g], usedm[g], invc[g],
                                  invm[g], ss[g], cnt[g], s_tab, n_tab, f);
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
    if ((a.stamps & 1u) && tid == 0) st_[i] = __builtin_amdgcn_s_memtime();
  };
  uint32_t seq = a.start_seq + 1;
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
    // ---- wave 0 waits for request `seq` in either block: every chunk's tag equal to it ----
    if (wave == 0) {
      const uint64_t t0 = wall_clock64();
      u32x4 v, u;
      uint32_t got = 0;  // 1: the BEGIN block, 2: the control block
      for (;;) {
        sys_ld16x2(a.box->req + lane * 4, a.box->creq + lane * 4, v, u);
        if (__ballot(v.w != seq) == 0) {
          got = 1;
          break;
        }
        if (__ballot(u.w != seq) == 0) {
          got = 2;
          v = u;
          break;
        }
        if (wall_clock64() - t0 > a.idle_ticks) break;
      }
      if (got) {
        s_req[lane * KSG_SRV_CHUNK_DW + 0] = v.x;
        s_req[lane * KSG_SRV_CHUNK_DW + 1] = v.y;
        s_req[lane * KSG_SRV_CHUNK_DW + 2] = v.z;
      }
      if (lane == 0) s_kind = got ? v.x : 0u;  // chunk 0's first dword is the header's kind
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
      if (tid == 0) respond(a, seq, 0, 0, 0);
      ++seq;
      continue;
    }
    // ---- BEGIN / COMMIT: the pod's payload beyond the block (read before any answer: the host
    // writes the next request's once it has one) ----
    const bool begin = kind == KSG_SRV_BEGIN;
    {
      const uint32_t paydw = min(s_req[KSG_SRVH_PAYDW], (uint32_t)KSG_SRV_PAY_DW);
      const uint32_t* xa = begin ? a.box->ext : a.box->cext;
      if (paydw > KSG_SRV_INLINE_DW) {
        for (uint32_t t = tid; t < paydw - KSG_SRV_INLINE_DW; t += KSG_NT)
          s_req[KSG_SRV_HDR_DW + KSG_SRV_INLINE_DW + t] = sys_ld32(xa + t);
        __syncthreads();
      }
    }
    const uint32_t node = s_req[KSG_SRVH_ARG];
    const bool bad = req_bad(d, s_req) || (!begin && (node < d.lo || node >= d.hi));
    stamp(2);
    if (bad) {  // (never, unless the host side has a bug)
      if (tid == 0) respond_rejected(a, seq);
      ++seq;
      continue;
    }
    if (begin) {
      const bool want_fail = (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_WANT_FAIL) != 0;
      scan(want_fail);
      const bool put_fail = want_fail && !err, put_ties = !err && k > 0;
      if (put_fail) {  // the shard's fail codes into host memory
        const uint32_t nb = d.hi - d.lo;
        for (uint32_t t = tid * 4; t < nb; t += KSG_NT * 4) {
          if (t + 4 <= nb) {
            *reinterpret_cast<volatile uint32_t*>(a.fail + t) = *reinterpret_cast<const uint32_t*>(s_fail + t);
          } else {
            for (uint32_t u = t; u < nb; ++u) reinterpret_cast<volatile uint8_t*>(a.fail)[u] = s_fail[u];
          }
        }
      }
      if (put_ties) {  // the tie words (the host picks the commit's node from them)
        const uint32_t nwd = min((uint32_t)(R * KSG_NWAVE), (d.hi - d.lo + 63) >> 6);
        for (uint32_t i = tid * 2; i < nwd; i += KSG_NT * 2) {
          u32x4 v;
          v.x = (uint32_t)s_tie[i];
          v.y = (uint32_t)(s_tie[i] >> 32);
          v.z = (uint32_t)s_tie[i + 1];
          v.w = (uint32_t)(s_tie[i + 1] >> 32);
          sys_st16(reinterpret_cast<uint32_t*>(a.box->ties + i), v);
        }
      }
      if (put_fail || put_ties) {  // ... before the response
        drain_stores();
        __syncthreads();
      }
      if (tid == 0) {
        if (a.stamps & 1u) {  // stage cycles: request seen->LDS, check, resolve, scan, reduce, fail codes
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
    // ---- COMMIT: AssumePod's delta on the host's node (answered first: requests are served in order) ----
    if (wave == 0) {
      if (lane == 0) respond(a, seq, node, 0, 0);
      const uint32_t* pay = s_req + KSG_SRV_HDR_DW;
      const ksg_pod& p = *reinterpret_cast<const ksg_pod*>(pay);
      const uint32_t* ids = pay + s_req[KSG_SRVH_IDS_AT];
      const ksg_pod_ext* ext = (EXT && (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_EXT))
                                   ? reinterpret_cast<const ksg_pod_ext*>(pay + s_req[KSG_SRVH_EXT_AT])
                                   : nullptr;
      commit_pod_wave(d, p, ids, node, lane, ext);
      drain_stores();
    }
    if constexpr (REG) {
      const ksg_pod& p = *reinterpret_cast<const ksg_pod*>(s_req + KSG_SRV_HDR_DW);
      const uint32_t off = node - d.lo;
      const uint32_t jw = off / KSG_NT, tw = off % KSG_NT;
#pragma unroll
      for (int j = 0; j < R; ++j)
        if ((uint32_t)j == jw && tid == tw) {
          rusedc[j] = (int64_t)((uint64_t)rusedc[j] + (uint64_t)p.milli_cpu);
          rusedm[j] = (int64_t)((uint64_t)rusedm[j] + (uint64_t)p.memory);
        }
    }
    ++seq;
  }
}

// ============================================================================
// The grid server: the scan spread over one workgroup per 256 nodes.
//
// The one-workgroup server is VALU-bound on its CU (16 waves x R nodes of
// ~250 instructions each: ~11 us of begin at 5,000 nodes). Here workgroups
// 1..G each own 256 nodes (one per thread) and serve BEGIN: each reads the
// request from the host block itself, so the pod reaches all of them in the
// same round trip, filters and scores its nodes, and writes its part {max,
// count, 4 tie words} and its nodes' fail codes straight into host memory,
// the part's sequence number last. The host merges the parts (the max, the
// count at it) and picks a commit's node from their tie words
// (generic_scheduler.go:88-95): the begin path has no device-side hand-off.
// Workgroup 0 (the leader) serves COMMIT (AssumePod's delta), PATCH and EXIT
// and answers each once it is applied and drained, so a BEGIN the host posts
// after that answer scans the state it left (every scan load of mutable state
// is an sc1 load). Both kinds of workgroup take any request newer than the
// last one they saw and skip the kinds they do not serve.
// ============================================================================
__device__ __forceinline__ void agent_st32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void agent_st64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The `applied` protocol between the leader and the scan workgroups (write the
// invariant down, or use release / acquire). INVARIANT: every access to mutable node state
// on either side is an agent-scope atomic (sc1: the leader's stores and read-modify-writes in
// commit_pod_wave / the patch loop, the scan workgroups' ld_mut loads), so it is served at the
// device's coherence point and no L1 / L2 copy can be stale. The leader drains its stores
// (s_waitcnt vmcnt(0): each one acknowledged at that point) before it stores `applied` = the
// request's sequence number; a scan workgroup polls `applied` (ld_mut) until it covers the
// BEGIN's ARG (the last control request the host posted before it), and only after the
// workgroup barrier that follows (a compiler barrier too) issues its loads of mutable state
// (requested totals, keymap rows, service counts, extended-resource usage). A plain (non-sc1)
// load of mutable state anywhere in the scan would break it. Agent-scope release / acquire
// would not need the invariant, but on gfx950 they are an L2 write-back (buffer_wbl2 sc1) and
// an L2 invalidate (buffer_inv sc1) per request: measured, 15,000 nodes 11.4 -> 22.1 us per pod.
__device__ __forceinline__ void st_applied(const KsgSrvArgs& a, uint32_t seq) {
  agent_st32(&a.grid->applied, seq);
}
// scan workgroups' backstop beyond the leader's idle limit (wall_clock64 ticks, 100 MHz: 10 ms)
#define KSG_GSRV_WAIT 1000000ull
#define KSG_GSRV_ANTI_REG 2  // anti priorities whose node domains a scan thread keeps in registers
// KSG_SERVE_DEBUG: workgroup `slot` reached `stage` of request `seq` (host memory, read after a fault)
__device__ __forceinline__ void grid_mark(const KsgSrvArgs& a, uint32_t slot, uint32_t seq, uint32_t stage) {
  if (a.stamps & 2u)
    __hip_atomic_store(a.box->dbg + slot, (seq << 8) | stage, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// wave 0: the next request in the host block (every tag equal to one sequence
// number > last) into s_req. -> its kind (0: none before the limit / told to quit)
__device__ __forceinline__ uint32_t grid_poll(const KsgSrvArgs& a, const uint32_t* blk, uint32_t lane, uint32_t last,
                                              bool worker, uint64_t limit, uint32_t* s_req, uint32_t& seq_out) {
  const uint64_t t0 = wall_clock64();
  bool armed = !worker || !(a.grid_opts & KSG_GSRV_POLL1);
  for (uint32_t it = 0;; ++it) {
    // (KSG_GSRV_POLL1: a scan workgroup reads chunk 0 alone until its tag moves, then the block)
    const u32x4 v = sys_ld16(blk + (armed ? lane * 4 : 0));
    const uint32_t t = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.w);
    if (!armed) {
      if ((int32_t)(t - last) > 0) {
        armed = true;
        continue;
      }
    } else if (__ballot(v.w != t) == 0 && (int32_t)(t - last) > 0) {
      s_req[lane * KSG_SRV_CHUNK_DW + 0] = v.x;
      s_req[lane * KSG_SRV_CHUNK_DW + 1] = v.y;
      s_req[lane * KSG_SRV_CHUNK_DW + 2] = v.z;
      seq_out = t;
      return (uint32_t)__builtin_amdgcn_readfirstlane((int)v.x);
    }
    if (worker) {  // (every 8th poll looks at `quit`; a short sleep spares the link)
      if ((it & 7) == 7 && ld_mut(&a.grid->quit) == a.epoch) return 0;
      __builtin_amdgcn_s_sleep(2);
      for (uint32_t z = 0; z < (a.grid_opts & 255u); ++z) __builtin_amdgcn_s_sleep(8);
    }
    if (wall_clock64() - t0 > limit) return 0;
  }
}

// the payload beyond the block (every thread; the caller synchronises)
__device__ __forceinline__ void grid_load_ext(const uint32_t* xa, uint32_t* s_req, uint32_t tid) {
  const uint32_t paydw = min(s_req[KSG_SRVH_PAYDW], (uint32_t)KSG_SRV_PAY_DW);
  if (paydw > KSG_SRV_INLINE_DW)
    for (uint32_t t = tid; t < paydw - KSG_SRV_INLINE_DW; t += KSG_GSRV_NT)
      s_req[KSG_SRV_HDR_DW + KSG_SRV_INLINE_DW + t] = sys_ld32(xa + t);
}

// NPT nodes per thread: 256 x NPT nodes per scan workgroup (NPT = 4 past
// KSG_SERVE_GRID_NPT4_MIN nodes: a quarter of the pollers on the link)
template <int NPT, bool EXT>
__global__ __launch_bounds__(KSG_GSRV_NT) void ksg_serve_grid_kernel(KsgDev d, KsgSrvArgs a) {
  constexpr uint32_t NODES = NPT * KSG_GSRV_NT, NW = NODES / 64, NWV = KSG_GSRV_NT / 64;
  __shared__ __attribute__((aligned(16))) uint32_t s_req[KSG_SRV_HDR_DW + KSG_SRV_PAY_DW];
  __shared__ int32_t s_tab[KSG_NT];
  __shared__ uint64_t s_wm[WM_N * NW];
  __shared__ int32_t s_wmax[NWV];
  __shared__ uint32_t s_wcnt[NW];
  __shared__ uint64_t s_tw[NW];
  __shared__ uint32_t s_kind, s_seq, s_ready;
  __shared__ KsgPatch s_pt[64];
  __shared__ int32_t s_tmw[NWV], s_gtm;  // (extensions) TaintToleration maxima: per wave, over the shard
  __shared__ int32_t s_dc[KSG_GSRV_MAXD], s_dtot[KSG_GSRV_MAXD];  // anti-affinity domain counts: here, over the shard

  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t bit = 1ULL << lane;
  uint32_t last = a.start_seq;

  if (blockIdx.x > 0) {
    // ======================= scan workgroup w: BEGIN =======================
    const uint32_t w = blockIdx.x - 1;
    KsgDev dw = d;  // this workgroup's nodes: [lo, hi) of the shard
    dw.lo = d.lo + w * NODES;
    dw.hi = min(d.hi, dw.lo + NODES);
    // this thread's nodes: dw.lo + j * 256 + tid (word j * 4 + wave, bit lane)
    uint32_t nn[NPT];
    bool valid[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const uint32_t n = dw.lo + j * KSG_GSRV_NT + tid;
      valid[j] = n < dw.hi;
      nn[j] = valid[j] ? n : dw.lo;
    }
    KsgSrvPart* hp = a.box->part + w;
    for (;;) {
      __syncthreads();
      if (wave == 0) {
        uint32_t t = 0;
        // (the leader returns first and raises `quit`; the limit is a backstop)
        const uint32_t kind = grid_poll(a, a.box->req, lane, last, true, 4 * a.idle_ticks + KSG_GSRV_WAIT, s_req, t);
        if (lane == 0) {
          s_kind = kind;
          s_seq = t;
        }
      }
      __syncthreads();
      const uint32_t kind = s_kind, T = s_seq;
      if (kind == 0 || kind >= KSG_SRV_EXIT) return;
      last = T;
      if (kind != KSG_SRV_BEGIN) continue;
      const uint64_t ts_seen = wall_clock64();
      if (tid == 0) grid_mark(a, 1 + w, T, 1);
      // the loads of the nodes' static data in flight with the payload's
      int64_t capc[NPT], capm[NPT], usedc[NPT], usedm[NPT];
      double invc[NPT], invm[NPT];
      int32_t ss[NPT], cnt[NPT];
      // ServiceAntiAffinity: the nodes' label domains of the first KSG_GSRV_ANTI_REG anti priorities
      // (static), in flight with the rest
      int32_t domr[NPT][KSG_GSRV_ANTI_REG];
#pragma unroll
      for (int j = 0; j < NPT; ++j) {
        capc[j] = d.cap_cpu[nn[j]];
        capm[j] = d.cap_mem[nn[j]];
        invc[j] = d.w_lr ? d.inv10_cpu[nn[j]] : 0.0;
        invm[j] = d.w_lr ? d.inv10_mem[nn[j]] : 0.0;
        ss[j] = d.has_static_score ? (int32_t)d.static_score[nn[j]] : 0;
#pragma unroll
        for (int q = 0; q < KSG_GSRV_ANTI_REG; ++q)
          domr[j][q] = (uint32_t)q < d.n_anti && d.n_domains_total > 0 ? d.anti_domain[(size_t)q * d.n_nodes + nn[j]] : -1;
      }
      grid_load_ext(a.box->ext, s_req, tid);
      if (wave == 0) {  // the control requests posted before this BEGIN are applied (commits it must see)
        const uint32_t after = s_req[KSG_SRVH_ARG];
        const uint64_t t0 = wall_clock64();
        while ((int32_t)(ld_mut(&a.grid->applied) - after) < 0) {
          if (wall_clock64() - t0 > KSG_GSRV_WAIT || ld_mut(&a.grid->quit) == a.epoch) {
            if (lane == 0) s_kind = 0;  // (the leader left: this launch cannot serve it)
            break;
          }
        }
      }
      __syncthreads();
      if (s_kind == 0) return;
      // mutable state only from here on (issued after `applied` covers the BEGIN's ARG)
#pragma unroll
      for (int j = 0; j < NPT; ++j) {
        usedc[j] = ld_mut(d.used_cpu + nn[j]);
        usedm[j] = ld_mut(d.used_mem + nn[j]);
      }
      const bool want_fail = (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_WANT_FAIL) != 0;
      int32_t sc[NPT];
#pragma unroll
      for (int j = 0; j < NPT; ++j) sc[j] = KSG_S32_NONE;
      uint32_t err = 0;
      if (req_bad(d, s_req)) {
        err = 2;
      } else {
        const uint32_t* pay = s_req + KSG_SRV_HDR_DW;
        const ksg_pod& p = *reinterpret_cast<const ksg_pod*>(pay);
        const uint32_t* ids = pay + s_req[KSG_SRVH_IDS_AT];
        // ServiceAntiAffinity (spreading.go:104-168): the pod's service pods on the shard's filtered
        // labelled nodes per domain, summed over the scan workgroups before any node is scored
        // (the host keeps the grid to <= KSG_GSRV_MAXD domains and no extensions)
        const bool anti_g = d.n_anti > 0 && d.n_domains_total > 0 && !d.equal_fallback;
        const bool need_cnt = (d.w_spread || anti_g) && p.service >= 0 && !d.equal_fallback;
        if (anti_g)
          for (uint32_t k = tid; k < d.n_domains_total; k += KSG_GSRV_NT) s_dc[k] = 0;  // (the barrier below)
#pragma unroll
        for (int j = 0; j < NPT; ++j)
          cnt[j] = need_cnt ? ld_mut(d.svc_cnt + (size_t)p.service * d.n_nodes + nn[j]) : 0;
        PodCtx c;
        pod_resolve(d, p, ids, c);
        // (extensions: the filters, BalancedAllocation and TaintToleration, whose normalisation max
        // is exchanged across the scan workgroups through grid->tmx)
        c.ext = (EXT && (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_EXT))
                    ? reinterpret_cast<const ksg_pod_ext*>(pay + s_req[KSG_SRVH_EXT_AT])
                    : nullptr;
        if (tid == 0) grid_mark(a, 1 + w, T, 3);
        if (c.error) {
          err = 1;
        } else {
          // the word masks' row loads in flight with pod_resolve's service loads, then the table
          const uint32_t nwq = (dw.hi - dw.lo + 63) >> 6;
          if (tid < nwq) word_masks(dw, c, tid, s_wm, NW);
          int32_t n_tab = 0;
          if (need_cnt && c.spread_max > 0) {
            n_tab = c.spread_max >= KSG_NT ? KSG_NT : c.spread_max + 1;
            for (int32_t t = (int32_t)tid; t < n_tab; t += KSG_GSRV_NT)
              s_tab[t] = (int32_t)frac10_f32((int64_t)c.spread_max - t, c.spread_max);
          }
          __syncthreads();  // (the word masks and the table)
          if (tid == 0) grid_mark(a, 1 + w, T, 4);
          if ((a.stamps & 1u) && tid == 0) s_ready = (uint32_t)wall_clock64();
          const bool res_on = (d.preds & KSG_PRED_PODFITSRESOURCES) && !c.zero_req;
          // (extensions) TaintTolerationPriority (ksg_exact.h scan_pod): the node's count of the
          // pod's untolerated PreferNoSchedule taints, normalised by the max over the shard's
          // filtered nodes (NormalizeReduce(10, reverse)) -- a max across the scan workgroups
          const bool ttg = EXT && c.ext != nullptr && d.w_taint != 0 && !d.equal_fallback;
          uint64_t psoft = 0;  // (taint ids < 64 with the per-node masks: the pod's soft ids as a mask)
          if (ttg && d.ntaint)
            for (uint32_t t = 0; t < c.ext->n_soft; ++t) psoft |= 1ULL << (c.ids[c.ext->soft_off + t] & 63);
          int32_t soft[NPT];
#pragma unroll
          for (int j = 0; j < NPT; ++j) {
            int f;
            const uint32_t n = dw.lo + j * KSG_GSRV_NT + tid;
            const int32_t s = eval_node(d, c, n, bit, s_wm, NW, j * NWV + wave, res_on, capc[j], capm[j], usedc[j],
                                        usedm[j], invc[j], invm[j], ss[j], cnt[j], s_tab, n_tab, f);
            sc[j] = (valid[j] && f == KSG_FAIL_NONE) ? s : KSG_S32_NONE;
            if (anti_g && sc[j] != KSG_S32_NONE && cnt[j] != 0) {
#pragma unroll
              for (int q = 0; q < KSG_GSRV_ANTI_REG; ++q)  // (compile-time indices: the domains stay in registers)
                if ((uint32_t)q < d.n_anti && domr[j][q] >= 0) atomicAdd(&s_dc[d.anti_dom_off[q] + domr[j][q]], cnt[j]);
              for (uint32_t q = KSG_GSRV_ANTI_REG; q < d.n_anti; ++q) {
                const int32_t dom = d.anti_domain[(size_t)q * d.n_nodes + nn[j]];
                if (dom >= 0) atomicAdd(&s_dc[d.anti_dom_off[q] + dom], cnt[j]);
              }
            }
            soft[j] = !ttg ? 0
                      : d.ntaint ? __popcll(d.ntaint[nn[j]] & psoft)
                                 : soft_taints(d, c, nn[j] >> 6, 1ULL << (nn[j] & 63));
            if (want_fail) {  // four nodes' codes per dword, straight into host memory
              const uint32_t fb = valid[j] ? (uint32_t)f : 0u;
              const uint32_t b0 = __shfl(fb, (int)((lane * 4 + 0) & 63), 64), b1 = __shfl(fb, (int)((lane * 4 + 1) & 63), 64);
              const uint32_t b2 = __shfl(fb, (int)((lane * 4 + 2) & 63), 64), b3 = __shfl(fb, (int)((lane * 4 + 3) & 63), 64);
              const uint32_t off = j * KSG_GSRV_NT + wave * 64 + lane * 4;
              if (lane < 16 && dw.lo + off < dw.hi)  // (shard-relative; the area is 4-padded)
                *reinterpret_cast<volatile uint32_t*>(a.fail + w * NODES + off) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
            }
          }
          if (anti_g) {
            __syncthreads();  // (every node's counts in s_dc)
            if (wave == 0) {
              const uint32_t D = d.n_domains_total, G = a.n_workers;
              if (lane < D) agent_st64(&a.grid->dcx[(size_t)w * KSG_GSRV_MAXD + lane], ((uint64_t)T << 32) | (uint32_t)s_dc[lane]);
              // lane k sums domain k over every scan workgroup's counts, tagged with this BEGIN
              const uint64_t tq = wall_clock64();
              int32_t tot = 0;
              bool ok = true;
              for (;;) {
                bool all = true;
                tot = 0;
                if (lane < D)
                  for (uint32_t q = 0; q < G; ++q) {
                    const uint64_t v = __hip_atomic_load(&a.grid->dcx[(size_t)q * KSG_GSRV_MAXD + lane], __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                    all = all && (uint32_t)(v >> 32) == T;
                    tot += (int32_t)(uint32_t)v;
                  }
                if (__ballot(!all) == 0) break;
                if (wall_clock64() - tq > KSG_GSRV_WAIT || ld_mut(&a.grid->quit) == a.epoch) {
                  ok = false;  // (a workgroup left: this launch cannot serve the BEGIN)
                  break;
                }
              }
              // each domain's term, int(10 * float32(n - count) / float32(n)) (10 when n == 0), once
              const int64_t tot_n = c.svc_total;
              if (lane < D) s_dtot[lane] = tot_n > 0 ? (int32_t)frac10_f32(tot_n - tot, tot_n) : 10;
              if (lane == 0 && !ok) s_kind = 0;
            }
            __syncthreads();
            if (s_kind == 0) return;
            // (anti_term from the per-domain terms: unlabelled nodes score 0, spreading.go:164-166)
#pragma unroll
            for (int j = 0; j < NPT; ++j) {
              int32_t at = 0;
#pragma unroll
              for (int q = 0; q < KSG_GSRV_ANTI_REG; ++q)
                if ((uint32_t)q < d.n_anti && domr[j][q] >= 0)
                  at += (int32_t)d.w_anti[q] * s_dtot[d.anti_dom_off[q] + domr[j][q]];
              for (uint32_t q = KSG_GSRV_ANTI_REG; q < d.n_anti; ++q) {
                const int32_t dom = d.anti_domain[(size_t)q * d.n_nodes + nn[j]];
                at += dom >= 0 ? (int32_t)d.w_anti[q] * s_dtot[d.anti_dom_off[q] + dom] : 0;
              }
              if (sc[j] != KSG_S32_NONE) sc[j] += at;
            }
          }
          if (ttg) {
            int32_t lm = 0;
#pragma unroll
            for (int j = 0; j < NPT; ++j) lm = sc[j] != KSG_S32_NONE ? max(lm, soft[j]) : lm;
            lm = wave_max_i32(lm);
            if (lane == 0) s_tmw[wave] = lm;
            __syncthreads();
            if (wave == 0) {
              int32_t wmx = s_tmw[0];
#pragma unroll
              for (uint32_t q = 1; q < NWV; ++q) wmx = max(wmx, s_tmw[q]);
              if (lane == 0) agent_st64(&a.grid->tmx[w], ((uint64_t)T << 32) | (uint32_t)wmx);
              // every scan workgroup's, tagged with this BEGIN (lane q reads workgroups q, q + 64, ...)
              const uint32_t G = a.n_workers;
              const uint64_t tq = wall_clock64();
              int32_t gm = 0;
              bool ok = true;
              for (;;) {
                bool all = true;
                int32_t mx = 0;
                for (uint32_t q = lane; q < G; q += 64) {
                  const uint64_t v = __hip_atomic_load(&a.grid->tmx[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                  all = all && (uint32_t)(v >> 32) == T;
                  mx = max(mx, (int32_t)(uint32_t)v);
                }
                if (__ballot(!all) == 0) {
                  gm = wave_max_i32(mx);
                  break;
                }
                if (wall_clock64() - tq > KSG_GSRV_WAIT || ld_mut(&a.grid->quit) == a.epoch) {
                  ok = false;  // (a workgroup left: this launch cannot serve the BEGIN)
                  break;
                }
              }
              if (lane == 0) {
                s_gtm = gm;
                if (!ok) s_kind = 0;
              }
            }
            __syncthreads();
            if (s_kind == 0) return;
            const int32_t gtm = s_gtm;
#pragma unroll
            for (int j = 0; j < NPT; ++j)
              if (sc[j] != KSG_S32_NONE) sc[j] += d.w_taint * taint_score_i32(soft[j], gtm);
          }
        }
      }
      // the part: best score, count and tie words of these nodes
      int32_t m = sc[0];
#pragma unroll
      for (int j = 1; j < NPT; ++j) m = max(m, sc[j]);
      const int32_t wm = wave_total_max(m);
      if (lane == 0) s_wmax[wave] = wm;
      __syncthreads();
      int32_t M = s_wmax[0];
#pragma unroll
      for (uint32_t q = 1; q < NWV; ++q) M = max(M, s_wmax[q]);
      if (d.empty_priorities) M = KSG_S32_NONE;  // all weights 0: an empty HostPriorityList
#pragma unroll
      for (int j = 0; j < NPT; ++j) {
        const uint64_t tb = __ballot(M != KSG_S32_NONE && sc[j] == M);
        if (lane == 0) {
          s_tw[j * NWV + wave] = tb;
          s_wcnt[j * NWV + wave] = (uint32_t)__popcll(tb);
        }
      }
      drain_stores();  // (this wave's fail-code stores)
      __syncthreads();
      if constexpr (NPT == 1) {
        if (tid < 4) {  // the part: one 64-B store of 4 lanes, the sequence number at both ends
          uint32_t k = 0;
#pragma unroll
          for (uint32_t q = 0; q < NW; ++q) k += s_wcnt[q];
          const uint32_t r = (tid == 1 || tid == 2) ? tid - 1 : 0u;  // (lanes 1, 2: the tie words)
          const uint64_t t0 = s_tw[2 * r], t1 = s_tw[2 * r + 1];
          u32x4 v;
          v.x = tid == 0 ? T : tid == 3 ? (uint32_t)ts_seen : (uint32_t)t0;
          v.y = tid == 0 ? (uint32_t)M : tid == 3 ? s_ready : (uint32_t)(t0 >> 32);
          v.z = tid == 0 ? k : tid == 3 ? (uint32_t)wall_clock64() : (uint32_t)t1;
          v.w = tid == 0 ? err : tid == 3 ? T : (uint32_t)(t1 >> 32);
          sys_st16(reinterpret_cast<uint32_t*>(hp) + 4 * tid, v);
          if (tid == 0) grid_mark(a, 1 + w, T, 6);
        }
      } else {
        if (tid < NW / 2) {  // the tie words (acknowledged), then the header line
          u32x4 v;
          v.x = (uint32_t)s_tw[2 * tid];
          v.y = (uint32_t)(s_tw[2 * tid] >> 32);
          v.z = (uint32_t)s_tw[2 * tid + 1];
          v.w = (uint32_t)(s_tw[2 * tid + 1] >> 32);
          sys_st16(reinterpret_cast<uint32_t*>(a.box->part_tie + (size_t)w * KSG_GSRV_TIEW + 2 * tid), v);
        }
        if (tid < 4) {
          uint32_t k = 0;
#pragma unroll
          for (uint32_t q = 0; q < NW; ++q) k += s_wcnt[q];
          u32x4 v;
          v.x = tid == 0 ? T : tid == 3 ? (uint32_t)ts_seen : 0u;
          v.y = tid == 0 ? (uint32_t)M : tid == 3 ? s_ready : 0u;
          v.z = tid == 0 ? k : tid == 3 ? (uint32_t)wall_clock64() : 0u;
          v.w = tid == 0 ? err : tid == 3 ? T : 0u;
          sys_st16(reinterpret_cast<uint32_t*>(hp) + 4 * tid, v);
          if (tid == 0) grid_mark(a, 1 + w, T, 6);
        }
      }
    }
  }

  // ======================= the leader: COMMIT, PATCH, EXIT =======================
  last = ld_mut(&a.grid->applied);  // (a control request newer than that one is still to apply)
  for (;;) {
    __syncthreads();
    if (wave == 0) {
      uint32_t t = 0;
      const uint32_t kind = grid_poll(a, a.box->creq, lane, last, false, a.idle_ticks, s_req, t);
      if (lane == 0) {
        s_kind = kind;
        s_seq = t;
      }
    }
    __syncthreads();
    const uint32_t kind = s_kind, T = s_seq;
    if (kind == 0 || kind > KSG_SRV_EXIT) {  // idle: the scan workgroups return too
      if (tid == 0) agent_st32(&a.grid->quit, a.epoch);
      return;
    }
    last = T;
    if (tid == 0) grid_mark(a, 0, T, 0x10 + kind);
    if (kind == KSG_SRV_EXIT) {  // (applied too: the next launch's leader skips it)
      if (tid == 0) {
        st_applied(a, T);
        agent_st32(&a.grid->quit, a.epoch);
        drain_stores();
        respond(a, T, 0, 0, 0);
      }
      return;
    }
    if (kind != KSG_SRV_PATCH && kind != KSG_SRV_COMMIT) continue;  // (never: BEGINs use the other block)
    if (kind == KSG_SRV_PATCH) {  // in order by one lane, agent scope (the scan workgroups read them)
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
                case 0: agent_st32(reinterpret_cast<uint32_t*>(pt.addr), (uint32_t)pt.value); break;
                case 1: agent_st64(reinterpret_cast<uint64_t*>(pt.addr), pt.value); break;
                case 2:
                  __hip_atomic_fetch_or(reinterpret_cast<uint64_t*>(pt.addr), pt.value, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
                  break;
                case 3:
                  __hip_atomic_fetch_and(reinterpret_cast<uint64_t*>(pt.addr), ~pt.value, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
                  break;
              }
            }
          }
          __builtin_amdgcn_wave_barrier();
        }
        drain_stores();
        if (lane == 0) {
          st_applied(a, T);
          respond(a, T, 0, 0, 0);
        }
      }
      continue;
    }
    // ---- COMMIT: AssumePod's delta on the host's node, then `applied` ----
    grid_load_ext(a.box->cext, s_req, tid);
    __syncthreads();
    const uint32_t node = s_req[KSG_SRVH_ARG];
    const bool bad = req_bad(d, s_req) || node < d.lo || node >= d.hi;
    if (wave == 0) {
      if (!bad) {
        const uint32_t* pay = s_req + KSG_SRV_HDR_DW;
        const ksg_pod& p = *reinterpret_cast<const ksg_pod*>(pay);
        const uint32_t* ids = pay + s_req[KSG_SRVH_IDS_AT];
        const ksg_pod_ext* ext = (EXT && (s_req[KSG_SRVH_FLAGS] & KSG_SRVF_EXT))
                                     ? reinterpret_cast<const ksg_pod_ext*>(pay + s_req[KSG_SRVH_EXT_AT])
                                     : nullptr;
        commit_pod_wave(d, p, ids, node, lane, ext);
        drain_stores();
      }
      if (lane == 0) {
        st_applied(a, T);  // (a bad one too: the BEGINs after it must not wait forever)
        if (bad) respond_rejected(a, T);
        else respond(a, T, node, 0, 0);
      }
    }
  }
}

hipError_t ksg_launch_serve_grid(int npt, bool ext, const KsgDev& d, const KsgSrvArgs& a, hipStream_t st) {
  const dim3 g(a.n_workers + 1), b(KSG_GSRV_NT);
  if (npt == 4 && ext) hipLaunchKernelGGL((ksg_serve_grid_kernel<4, true>), g, b, 0, st, d, a);
  else if (npt == 4) hipLaunchKernelGGL((ksg_serve_grid_kernel<4, false>), g, b, 0, st, d, a);
  else if (ext) hipLaunchKernelGGL((ksg_serve_grid_kernel<1, true>), g, b, 0, st, d, a);
  else hipLaunchKernelGGL((ksg_serve_grid_kernel<1, false>), g, b, 0, st, d, a);
  return hipGetLastError();
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
