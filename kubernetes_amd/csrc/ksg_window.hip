// ksg_window.hip — speculative window path for the Filter/Score pass.
//
// The reference schedules pods strictly one after another: pod i+1 sees pod i's
// AssumePod (plugin/pkg/scheduler/scheduler.go:115-118). The window path keeps
// that exact sequential semantics while moving almost all of the work off the
// sequential chain:
//
//  phase A (ksg_win_score_kernel, all CUs, node-major): one wave owns one
//    64-node word of the shard (lane = node) and scores a group of KSG_PG
//    window pods against ONE snapshot of the node state. The pod-side work of
//    the predicates (nodeSelector pairs, host ports, GCE PDs, ServiceAffinity,
//    LabelsPresence, HostName) collapses into one 64-bit fit word per (pod,
//    word), built by lane j for pod j; the node state (capacity, requested
//    totals) is loaded once per wave and reused for every pod of the group.
//    Per (pod, word) it stores the word's best score and the bitmap of nodes at
//    that score; the wave that owns word 0 also writes each pod's 192-byte
//    resolver record (KsgWinSum).
//  phase B: walks the window in order and reproduces the sequential result.
//    M0 = max over the words of the best scores, T0 = nodes at M0. For a
//    "clean" pod — one whose service scalars (ServiceSpreading maxCount,
//    ServiceAffinity peer) no earlier pod of the window changed — a commit can
//    only make the committed node WORSE (requested totals grow: LeastRequested
//    falls and PodFitsResources can flip to false; host ports / PDs only get
//    added; service counts grow under a fixed maxCount; extensions: extended
//    resources only get taken), and every other node is untouched. So the
//    sequential max is still M0 unless all of T0 was made worse, and the
//    sequential tie set is T0 minus the nodes committed earlier in the window
//    (set C, "slots") whose re-evaluated score dropped. Phase B re-checks only
//    T0 ∩ C, draws the Int63 the reference draws (generic_scheduler.go:94),
//    selects the ix-th tie in descending name order, commits into the slot,
//    and continues. A pod that is not clean, or whose whole T0 dropped, ends
//    the window; the next window (a new snapshot) starts at that pod. Results
//    are bit-identical to the one-pod-at-a-time path (tests/test_gpu_parity.py
//    compares both with the oracle).
//    Resolvers, each one workgroup of 512 threads (committer, checkers,
//    x-checker, producers pipelined over the window's pods):
//      ksg_win_plain_kernel (ksg_plain.hip) — every configuration without
//        ServiceAntiAffinity; reads the per-pod T0 images ksg_win_t0_kernel
//        builds between the two phases;
//      ksg_win_resolve2_kernel (this file) — ServiceAntiAffinity with the
//        per-domain re-rank (one anti priority, one rank, <= 31 label values);
//      ksg_win_resolve_kernel (this file, LDS slots) — the other
//        ServiceAntiAffinity configurations.
//
// ServiceAntiAffinity scores a node by its domain's count of the pod's service
// pods over the pod's FILTERED nodes: phase A runs a count pass first; a pod
// whose service had commits earlier in the window is re-ranked per domain
// (resolve2), or (LDS-slot resolver) ends the window.
#include "ksg_device.h"
#include "ksg_resolver.h"

#include <algorithm>

#include "ksg_score.h"

// ---------------------------------------------------------------------------
// phase A as its own launch (ksg_score.h has the per-wave body)
// ---------------------------------------------------------------------------
template <int MODE, int KSG_PG, bool EXT = false>
__global__ __launch_bounds__(KSG_SC_NT) KSG_PA_ATTR void ksg_win_score_kernel(KsgDev d, const ksg_pod* __restrict__ batch,
                                                                 const uint32_t* __restrict__ ids,
                                                                 const KsgWinRun* __restrict__ run, uint32_t wcap,
                                                                 KsgWinSum* __restrict__ sums,
                                                                 uint64_t* __restrict__ wbits,
                                                                 int32_t* __restrict__ wmax, uint32_t ostride,
                                                                 int32_t* __restrict__ dcnt,
                                                                 uint64_t* __restrict__ wfit,
                                                                 int32_t* __restrict__ dmb,
                                                                 uint64_t* __restrict__ wbz, uint32_t dz,
                                                                 const ksg_pod_ext* __restrict__ exts,
                                                                 int32_t* __restrict__ tmax,
                                                                 uint64_t* __restrict__ psoft,
                                                                 int32_t* __restrict__ thist) {
  // XCD-aware order (a 1-D grid padded to a multiple of 8): the hardware deals
  // workgroups round-robin to the 8 XCDs (linear id mod 8), so XCD k takes the
  // k-th contiguous eighth of the (word group, pod group) pairs, pod group
  // fastest: the node state of a word group is fetched into one XCD's L2 for all
  // the window's pod groups instead of into every XCD's
  const uint32_t gx = (d.nwords + KSG_SC_NT / 64 - 1) / (KSG_SC_NT / 64), gy = (wcap + KSG_PG - 1) / KSG_PG;
  const uint32_t per = gridDim.x >> 3, lin = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  if (lin >= max(gx, 1u) * gy) return;  // (padding; wave-uniform, no barrier in this kernel)
  const uint32_t bx = lin / gy, by = lin - bx * gy;
  const uint32_t w = __builtin_amdgcn_readfirstlane(bx * (KSG_SC_NT / 64) + (threadIdx.x >> 6));
  // this window = pods [pos, pos + n_pods) of the batch (set by the previous resolver)
  const uint32_t pos = run->pos, n_batch = run->n;
  if (run->halt || pos >= n_batch) return;
  win_score_wave<MODE, KSG_PG, EXT, false>(d, batch, ids, pos, n_batch, wcap, w, by * KSG_PG, sums, wbits, wmax,
                                           ostride, dcnt, wfit, dmb, wbz, dz, exts, tmax, psoft, thist, nullptr);
}

// ---------------------------------------------------------------------------
// phase B
// ---------------------------------------------------------------------------
// One workgroup of 8 waves in four roles, pipelined over the window's pods
// (wave 0 committer, wave 1 scribe, waves 2..3 checkers, waves 4..7 producers):
//
//  PRODUCERS stage pod j into ring entry j mod KSG_RING: its
//    record, its T0 bitmap (nodes at the snapshot max M0, from phase A's
//    per-word maxima), k0 = |T0|, its tie-break draw r (the splitmix64 output
//    at the pod's draw index = the number of earlier window pods that draw:
//    those that neither error nor find no fit), r mod (k0 - d) for d = 0..63
//    dropped ties, and the PREDICTED node: the (r mod k0)-th tie of T0 from
//    the top, the answer whenever no tie dropped, with its snapshot state
//    (capacity, requested totals, 10/capacity) and the pod's service counts
//    on it and service scalars.
//  CHECKERS re-check pod i against the nodes committed earlier
//    in the window ("slots", set C): checker c owns slots 64c..64c+63, one per
//    lane. A slot is a candidate when its node is in T0 (one LDS read); a
//    candidate drops when the window's deltas pushed its score below M0
//    (resources, host ports / PDs, LeastRequested, ServiceSpreading). Dropped
//    nodes are scattered into an LDS bitmap. Pod i is checked as soon as the
//    COMMITTER has selected pod i-1's node, against every slot except the one
//    pod i-1 is committing into.
//  COMMITTER (wave 0) walks the window in order: for pod i it takes the
//    checkers' drops, re-checks the one slot pod i-1 just committed into,
//    selects the ix-th live tie in descending name order (the staged
//    prediction when nothing dropped), publishes the choice — which releases
//    the checkers onto pod i+1 — and then commits into the slot.
//
//  SCRIBE (wave 1) writes each order the committer issues into the slot arrays
//    (AssumePod's delta, the pod's keys and service entries, the services'
//    snapshot counts), sets the service flags and first peers in commit order,
//    counts each service's window commits (re-rank), and frees the pod's ring
//    entry.
//
// So the checkers' scan of pod i+1 overlaps the commit of pod i, and the
// sequential chain per pod is select + commit + one slot's re-check. Slot
// state lives in LDS (structure of arrays by slot, at most KSG_MAX_SLOTS).
//
// Hand-offs (LDS; polls are acquire loads, posts release stores after the data
// they cover; VERDICT r3 "bring the anti-affinity resolvers up to ksg_plain.hip's
// standard"):
//
//   flag / data              writer      reader               pod index      ordered by
//   r_hdr[e].ready + entry   producer j  checkers, committer, j              ready = j+1 release after the entry
//    (record, T0, fit, r mod,            scribe
//    services, B words)
//   draw_count               producer j  producer j+1         j              draw_next = j+1 release after it
//   consumed                 scribe      producers            i              consumed = i+1 release once order i
//                                                                            is written (entry i mod KSG_RING free)
//   xs_slot, xs_nslots       committer   checkers             i (pod i+1     sel_seq = i+1 release after them
//                                                             skips xs_slot)
//   L_drop[i & 1], chk_cnt,  checker c   committer            i              chk_seq[c] = i+1 release after the
//    chk_stop, L_dca                                                         drop bits (atomicOr), counts, rows
//   L_ord[i & 1] (WinOrder)  committer   scribe               i              order_seq = i+1 release after a
//                                                                            wavefront fence (lds_fence)
//   slot arrays, L_flag,     scribe      checkers, committer  orders <= i    scribe_done = i+1 release after the
//    L_peer, n_peer, L_nsv                                                   writes; checkers of pod i+2 wait for
//                                                                            scribe_done >= i+1, the committer
//                                                                            (wait_scribe) before it reads a slot
//   stop                     committer   all                  —              release; every other wave exits
//
// Every wait has a spin limit (the committer's and the checkers' end the
// window with KSG_STOP_HANG; the host fails the batch). KSG_DEBUG bits 16..19
// add a fixed delay per pod to the committer, scribe, checkers or producers
// (tests/test_gpu_fuzz.py runs each skew once against the oracle).
// The node state in HBM stays the pristine snapshot while the window
// resolves; the window's deltas are written back once, at the end.
// ANTI: ServiceAntiAffinity is on (its checks are compiled only into these
// instantiations: they cost the others scalar registers on the chain)
template <int P, bool STAMP, bool ANTI>
__global__ __launch_bounds__(win_res_nt(P)) void ksg_win_resolve_kernel(KsgDev d, uint32_t wcap, KsgWinRun* run,
                                                                    const KsgWinSum* __restrict__ sums,
                                                                    const KsgWinXchg x, uint64_t* rng_io,
                                                                    int32_t* __restrict__ out_batch) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t pos = run->pos, n_batch = run->n;
  if (run->halt || pos >= n_batch) return;  // the chain is done (uniform, before any barrier)
  const uint32_t n_pods = min(wcap, n_batch - pos);
  int32_t* __restrict__ out = out_batch + pos;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nflag = (d.n_services + 31) / 32;
  const uint32_t nwords = d.nwords;
  constexpr uint32_t KSG_RING = win_ring(P);
  constexpr uint32_t KSG_RES_NT = win_res_nt(P);
  // re-rank: a pod whose service had commits earlier in the window is ranked
  // again per domain row (committer) instead of ending the window
  const bool rr = ANTI && x.rr != 0;
  const uint32_t dz = rr ? x.dz : 0u;
  if constexpr (ANTI) {  // this window's score pass has read the domain counts: zero them for the next
    // (with the re-rank the producers stage them: the committer zeroes them at the end)
    if (!rr)
      for (uint32_t t = tid; t < x.dcnt_n; t += KSG_RES_NT) x.dcnt[t] = 0;
  }
  constexpr bool anti_on = ANTI;  // (the host passes fit bitmaps, x.fit_off != 0, exactly then)
  const WinLdsOff o = win_lds_offsets(P, nflag, wcap, anti_on, dz, d.n_services);
  uint64_t* const r_b = reinterpret_cast<uint64_t*>(smem + o.r_b);   // [ring][P*64] best-per-row words
  int32_t* const r_mb = reinterpret_cast<int32_t*>(smem + o.r_mb);   // [ring][KSG_RR_MAXZ] best per row
  int32_t* const r_dc = reinterpret_cast<int32_t*>(smem + o.r_dc);   // [ring][KSG_RR_MAXZ] domain counts
  uint64_t* const L_zm = reinterpret_cast<uint64_t*>(smem + o.zm);   // [dz][P*64] nodes of each row
  uint32_t* const L_nsv = reinterpret_cast<uint32_t*>(smem + o.nsv); // window commits per service
  int32_t* const L_dca = reinterpret_cast<int32_t*>(smem + o.dca);   // [chk][parity][KSG_RR_MAXZ]
  WinCtl* ctl = reinterpret_cast<WinCtl*>(smem + o.ctl);
  RingHdr* r_hdr = reinterpret_cast<RingHdr*>(smem + o.r_hdr);
  uint64_t* r_t0 = reinterpret_cast<uint64_t*>(smem + o.r_t0);
  uint32_t* r_rec = reinterpret_cast<uint32_t*>(smem + o.r_rec);
  uint32_t* r_mod = reinterpret_cast<uint32_t*>(smem + o.r_mod);
  RingSvc* r_svc = reinterpret_cast<RingSvc*>(smem + o.r_svc);
  uint64_t* r_fit = reinterpret_cast<uint64_t*>(smem + o.r_fit);
  // pod j's fit-at-the-snapshot word w: its ring copy, or past 64k nodes (win2_fg) phase A's row
  // (the rank that scored word w wrote it at its block of the exchanged buffer)
  auto fit_word = [&](uint32_t e, uint32_t j, uint32_t w) -> uint64_t {
    if constexpr (win2_fg(P)) {
      uint32_t g = 0;
      for (uint32_t r = 1; r < x.world; ++r)
        if (w >= x.wlo[r] && x.nw[r] > 0) g = r;
      const uint32_t iw = w - x.wlo[g];
      return (w < nwords && iw < x.nw[g])
                 ? gld(reinterpret_cast<const uint64_t*>(x.buf + (size_t)g * x.blk + (size_t)iw * 8 + x.fit_off +
                                                         (size_t)j * x.ostride * 8))
                 : 0ULL;
    } else {
      return r_fit[(size_t)e * P * 64 + w];
    }
  };
  const WinSlots S{reinterpret_cast<SlotMeta*>(smem + o.s_meta), reinterpret_cast<I64x2*>(smem + o.s_cap),
                   reinterpret_cast<I64x2*>(smem + o.s_snp),     reinterpret_cast<I64x2*>(smem + o.s_dl),
                   reinterpret_cast<F64x2*>(smem + o.s_inv),     reinterpret_cast<uint32_t*>(smem + o.keys),
                   reinterpret_cast<uint32_t*>(smem + o.svcs),   reinterpret_cast<int32_t*>(smem + o.scnt)};
  uint64_t* const L_drop = reinterpret_cast<uint64_t*>(smem + o.drop);  // [2][P*64] by pod parity
  const bool spread_on = d.w_spread != 0;
  const bool aff_on = (d.preds & KSG_PRED_SERVICEAFFINITY) && d.n_aff > 0;
  const bool res_on = (d.preds & KSG_PRED_PODFITSRESOURCES) != 0;
  const bool ports_on = (d.preds & KSG_PRED_PODFITSPORTS) != 0;
  const bool disk_on = (d.preds & KSG_PRED_NODISKCONFLICT) != 0;
  // KSG_DEBUG bits 16..19: a fixed delay per pod in one role (committer, scribe, checkers,
  // producers): another interleaving of the hand-offs than the natural one (tests/test_gpu_fuzz.py)
  const uint32_t skew = STAMP ? ((uint32_t)d.dbg >> 16) & 15u : 0u;  // (debug instantiation only)

  for (uint32_t t = tid; t < KSG_RING; t += KSG_RES_NT) r_hdr[t].ready = 0;
  if (tid == 0) {
    *ctl = WinCtl{};
    ctl->xs_slot = KSG_NO_SLOT;
  }
  if (wave == 0) {
    uint32_t* flag = reinterpret_cast<uint32_t*>(smem + o.flag);
    uint32_t* peerset = reinterpret_cast<uint32_t*>(smem + o.peerset);
    for (uint32_t w = lane; w < nflag; w += 64) {
      flag[w] = 0;
      peerset[w] = 0;
    }
  }
  for (uint32_t w = tid; w < 2 * P * 64u; w += KSG_RES_NT) L_drop[w] = 0;
  if (rr) {
    for (uint32_t t = tid; t < dz * P * 64; t += KSG_RES_NT) {
      const uint32_t row = t / (P * 64), w = t % (P * 64);
      L_zm[t] = w < nwords ? x.zmap[(size_t)row * d.nw + d.wlo + w] : 0ULL;
    }
    for (uint32_t t = tid; t < d.n_services; t += KSG_RES_NT) L_nsv[t] = 0;
  }
  __syncthreads();
  const uint64_t rng0 = *rng_io;

  // =========================================================================
  // producers
  // =========================================================================
  if (wave >= KSG_RES_P0) {
    const uint32_t* recs = reinterpret_cast<const uint32_t*>(sums);
    // this lane's words lane*P + q: byte offsets of the rank block and row phase
    // A wrote them at (~0u = no such word)
    uint32_t wb_at[P], wm_at[P];
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const uint32_t wq = lane * P + q;
      uint32_t g = 0;
      for (uint32_t r = 1; r < x.world; ++r)
        if (wq >= x.wlo[r] && x.nw[r] > 0) g = r;
      const uint32_t i = wq - x.wlo[g];
      const bool ok = wq < nwords && i < x.nw[g];
      const uint32_t base = (uint32_t)(g * x.blk);
      wb_at[q] = ok ? base + i * 8 : ~0u;
      wm_at[q] = ok ? base + x.wcap * x.ostride * 8 + i * 4 : ~0u;
      // (the fit bitmaps sit at wb_at + fit_off)
    }
    const uint32_t row_b = x.ostride * 8, row_m = x.ostride * 4;
    // KSG_DEBUG & 8: producer sections (slot wait, loads, draw wait, rest) into dbgbuf[12..15]
    uint64_t pt_last = 0, pt_acc = 0;
    auto pstamp = [&](uint32_t k) {
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        pt_acc += lane == k ? t_now - pt_last : 0ULL;
        pt_last = t_now;
      }
    };
    auto pflush = [&]() {
      if constexpr (STAMP)
        if (d.dbgbuf && lane >= 12 && lane < 16) atomicAdd(d.dbgbuf + lane, (int32_t)(pt_acc / 64));
    };
    if constexpr (STAMP) pt_last = __builtin_amdgcn_s_memtime();
    for (uint32_t j = wave - KSG_RES_P0; j < n_pods; j += KSG_RES_NPW) {
      const uint32_t e = j % KSG_RING;
      for (uint32_t spin = 0;; ++spin) {  // ring entry free: the resolver is done with pod j - KSG_RING
        if (ld_acq(&ctl->stop) || spin > KSG_SPIN_LIMIT) {
          pflush();
          return;
        }
        if (ld_acq(&ctl->consumed) + KSG_RING > j) break;
        __builtin_amdgcn_s_sleep(1);
      }
      pstamp(12);
      if (skew & 8u) __builtin_amdgcn_s_sleep(8);
      const uint32_t rec = lane < KSG_WIN_SUM_DWORDS ? recs[(size_t)j * KSG_WIN_SUM_DWORDS + lane] : 0u;
      uint64_t t0[P];
      int32_t mw[P];
      int32_t lm = KSG_S32_NONE;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        t0[q] = wb_at[q] != ~0u ? *reinterpret_cast<const uint64_t*>(x.buf + wb_at[q] + j * row_b) : 0ULL;
        mw[q] = wm_at[q] != ~0u ? *reinterpret_cast<const int32_t*>(x.buf + wm_at[q] + j * row_m) : KSG_S32_NONE;
        lm = mw[q] > lm ? mw[q] : lm;
      }
      const int32_t m0 = wave_total_max(lm);
      uint32_t cnt = 0;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        t0[q] = (m0 != KSG_S32_NONE && mw[q] == m0) ? t0[q] : 0ULL;
        cnt += __popcll(t0[q]);
      }
      const uint32_t incl = dpp_scan_add(cnt);
      const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      const bool drawable = __builtin_amdgcn_readlane(rec, WS_ERR) == 0 && m0 != KSG_S32_NONE;

      pstamp(13);
      // draw index = draws of the window pods before j
      for (uint32_t spin = 0;; ++spin) {
        if (ld_acq(&ctl->stop) || spin > KSG_SPIN_LIMIT) {
          pflush();
          return;
        }
        if (ld_acq(&ctl->draw_next) == j) break;
        __builtin_amdgcn_s_sleep(1);
      }
      pstamp(14);
      const uint32_t idx = __builtin_amdgcn_readfirstlane(ctl->draw_count);
      if (lane == 0) {
        ctl->draw_count = idx + (drawable ? 1u : 0u);
        st_rel(&ctl->draw_next, j + 1);
      }
      const uint64_t r = ksg_rng_draw(d.draws, rng0 + (uint64_t)idx * ksg_rng_step(d.draws));  // rand.Int() (generic_scheduler.go:94)

      uint32_t mv = 0;
      if (drawable && lane < k0) mv = umod64_32(r, k0 - lane);

      // predicted node: the (r mod k0)-th tie from the top (nothing dropped)
      int32_t pred = -1;
      int64_t pv = 0;  // lanes 0..3: cap_c, cap_m, used_c, used_m of pred
      double pinv = 0.0;
      const uint32_t n_svcs = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NSS) >> 16;
      const uint32_t nk = ((uint32_t)__builtin_amdgcn_readlane(rec, WS_NPP) & 0xffff) +
                          ((uint32_t)__builtin_amdgcn_readlane(rec, WS_NPP) >> 16);
      const uint32_t n_sel = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NSS) & 0xffff;
      const bool inl = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NINL) <= KSG_WIN_INLINE &&
                       n_svcs <= KSG_SLOT_SVCS;
      // the pod's services are record dwords WS_IDS + nk + n_sel + t (all lanes shuffle)
      const uint32_t t_sv = lane < n_svcs ? lane : 0u;
      const uint32_t my_sv = (uint32_t)__shfl((int)rec, (int)min(WS_IDS + nk + n_sel + t_sv, 63u), 64);
      int32_t s_cnt = 0, s_max = 0, s_peer = 0;
      if (drawable) {
        const uint32_t ix0 = __builtin_amdgcn_readfirstlane(mv);  // lane 0: r mod k0
        pred = (int32_t)select_in_lanes<P>(t0, cnt, incl, k0 - 1 - ix0, lane);
        const uint32_t pn = d.lo + (uint32_t)pred;
        if (lane == 0) pv = d.cap_cpu[pn];
        else if (lane == 1) pv = d.cap_mem[pn];
        else if (lane == 2) pv = d.used_cpu[pn];
        else if (lane == 3) pv = d.used_mem[pn];
        if (inl && lane < n_svcs) {
          s_cnt = d.svc_cnt[(size_t)my_sv * d.n_nodes + pn];
          s_max = d.svc_max[my_sv];
          s_peer = d.svc_peer[my_sv];
        }
        pinv = lr_inv10(pv);
      }

      // publish the entry
      r_mod[e * 64 + lane] = mv;
      if (lane < KSG_WIN_SUM_DWORDS) r_rec[e * KSG_WIN_SUM_DWORDS + lane] = rec;
#pragma unroll
      for (int q = 0; q < P; ++q) r_t0[(size_t)e * P * 64 + lane * P + q] = t0[q];
      if (anti_on) {
        if constexpr (!win2_fg(P))
#pragma unroll
          for (int q = 0; q < P; ++q)
            r_fit[(size_t)e * P * 64 + lane * P + q] =
                wb_at[q] != ~0u ? *reinterpret_cast<const uint64_t*>(x.buf + wb_at[q] + x.fit_off + j * row_b) : 0ULL;
        if (rr) {  // the re-rank's inputs: best-per-row words, best per row, domain counts
#pragma unroll
          for (int q = 0; q < P; ++q)
            r_b[(size_t)e * P * 64 + lane * P + q] =
                wb_at[q] != ~0u ? *reinterpret_cast<const uint64_t*>(x.buf + wb_at[q] + x.b_off + j * row_b) : 0ULL;
          if (lane < dz) {
            r_mb[e * KSG_RR_MAXZ + lane] = x.dmb[(size_t)j * dz + lane];
            r_dc[e * KSG_RR_MAXZ + lane] =
                lane + 1 < dz ? x.dcnt[(size_t)j * d.n_domains_total + d.anti_dom_off[0] + lane] : 0;
          }
        }
      }
      if (inl && lane < n_svcs) {
        r_svc[e].cnt[lane] = s_cnt;
        r_svc[e].max[lane] = s_max;
        r_svc[e].peer[lane] = s_peer;
      }
      if (lane < 4) (&r_hdr[e].cap_c)[lane] = pv;
      if (lane < 2) (&r_hdr[e].inv_c)[lane] = pinv;
      if (lane == 0) {
        r_hdr[e].m0 = m0;
        r_hdr[e].k0 = k0;
        r_hdr[e].r = r;
        r_hdr[e].drawable = drawable;
        r_hdr[e].pred = pred;
        st_rel(&r_hdr[e].ready, j + 1);
      }
      pstamp(15);
    }
    pflush();
    return;
  }

  // =========================================================================
  // checkers (waves KSG_RES_C0 ..): slot 64c + lane of checker c
  // =========================================================================
  if (wave >= KSG_RES_C0) {
    __builtin_amdgcn_s_setprio(2);
    const uint32_t c = wave - KSG_RES_C0;
    const uint32_t sl = c * 64 + lane;
    for (uint32_t i = 0; i < n_pods; ++i) {
      const uint32_t e = i % KSG_RING, par = i & 1;
      // pod i is staged, the committer has chosen pod i-1's node (slot xs,
      // skipped here), and the scribe has written every commit before pod i-1.
      // While this checker works on pod i the committer cannot pass pod i-1:
      // it waits for this checker before selecting pod i.
      for (uint32_t spin = 0;; ++spin) {
        if (ld_acq(&ctl->stop) || spin > 16 * KSG_SPIN_LIMIT) return;
        if (ld_acq(&r_hdr[e].ready) == i + 1 && ld_acq(&ctl->sel_seq) >= i && ld_acq(&ctl->scribe_done) + 1 >= i)
          break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (skew & 4u) __builtin_amdgcn_s_sleep(8);
      const uint32_t xs = ctl->xs_slot, ns = ctl->xs_nslots;
      const uint32_t rec = lane < KSG_WIN_SUM_DWORDS ? r_rec[e * KSG_WIN_SUM_DWORDS + lane] : 0u;
      const int32_t m0 = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].m0);
      uint32_t cnt = 0, astop = 0;
      int32_t dadd = 0;  // (re-rank) this lane's domain row: window commits of the pod's service it counts
      if (!__builtin_amdgcn_readlane(rec, WS_ERR) && m0 != KSG_S32_NONE && c * 64 < ns) {
        const PodView pv = pod_view(rec);
        const uint64_t* t0e = r_t0 + (size_t)e * P * 64;
        bool drop = false, moved = false, t0_drop = false;
        uint32_t ks = 0, zr = ~0u;
        if (sl < ns && sl != xs) {
          const uint32_t nd = S.meta[sl].node;
          const bool in_t0 = (t0e[nd >> 6] >> (nd & 63)) & 1ULL;
          // (re-rank: every node at its domain row's best is a candidate, T0 among them)
          const bool in_b = rr ? ((r_b[(size_t)e * P * 64 + (nd >> 6)] >> (nd & 63)) & 1ULL) != 0 : in_t0;
          if (in_b) {
            drop = slot_drops(d, S, sl, pv, rec, res_on, ports_on, disk_on, spread_on);
            if (drop)
              atomicOr(reinterpret_cast<unsigned long long*>(L_drop + (size_t)par * P * 64 + (nd >> 6)),
                       1ULL << (nd & 63));
            t0_drop = drop && in_t0;
          }
          const bool fit_snap = anti_on && pv.s >= 0 && ((fit_word(e, i, nd >> 6) >> (nd & 63)) & 1ULL);
          bool fits_now = false;
          if (fit_snap) {
            fits_now = slot_fits_now(S, sl, pv, rec, res_on, ports_on, disk_on);
            if (!fits_now) moved = anti_counts_move(d, nd, pv.s);
          }
          if (rr && fits_now && ((S.meta[sl].smask >> (pv.s & 31)) & 1u)) {
            // the window's commits of the pod's service on this node count in its domain
            const uint32_t* sv = S.svcs + (size_t)sl * KSG_SLOT_SVCS;
            for (uint32_t a = 0; a < S.meta[sl].ns; ++a) ks += sv[a] == (uint32_t)pv.s;
            for (uint32_t r = 0; r + 1 < dz; ++r)
              if ((L_zm[(size_t)r * P * 64 + (nd >> 6)] >> (nd & 63)) & 1ULL) zr = r;
          }
        }
        cnt = __popcll(__ballot(t0_drop));
        astop = __ballot(moved) != 0;
        if (rr) {
          uint64_t pm = __ballot(ks != 0 && zr != ~0u);
          while (pm) {
            const int b = (int)__builtin_ctzll(pm);
            pm &= pm - 1;
            const uint32_t zz = (uint32_t)__builtin_amdgcn_readlane((int)zr, b);
            const int32_t kk = __builtin_amdgcn_readlane((int)ks, b);
            if (lane == zz) dadd += kk;
          }
        }
      }
      if (rr && lane < dz) L_dca[(c * 2 + par) * KSG_RR_MAXZ + lane] = dadd;
      if (lane == 0) {
        ctl->chk_cnt[c][par] = cnt;
        ctl->chk_stop[c][par] = astop;
        st_rel(&ctl->chk_seq[c], i + 1);
      }
    }
    return;
  }

  uint32_t* const L_peer = reinterpret_cast<uint32_t*>(smem + o.peer);
  int32_t* const L_out = reinterpret_cast<int32_t*>(smem + o.out);
  uint32_t* const L_flag = reinterpret_cast<uint32_t*>(smem + o.flag);
  uint32_t* const L_peerset = reinterpret_cast<uint32_t*>(smem + o.peerset);
  WinOrder* const L_ord = reinterpret_cast<WinOrder*>(smem + o.ord);  // [2] by pod parity

  // =========================================================================
  // scribe (wave 1): applies each commit to the LDS slot state, in order
  // =========================================================================
  if (wave == 1) {
    __builtin_amdgcn_s_setprio(2);
    uint32_t n_peer = 0;
    for (uint32_t i = 0;; ++i) {
      bool have = false;
      // (no spin limit: the committer's own waits are bounded and it always
      // raises stop, after its last order)
      for (;;) {
        if (ld_acq(&ctl->order_seq) >= i + 1) {
          have = true;
          break;
        }
        if (ld_acq(&ctl->stop) && ld_acq(&ctl->order_seq) <= i) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (!have) break;
      if (skew & 2u) __builtin_amdgcn_s_sleep(8);
      const WinOrder& od = L_ord[i & 1];
      const uint32_t kind = __builtin_amdgcn_readfirstlane(od.kind);
      const int32_t outv = __builtin_amdgcn_readfirstlane(od.out);
      if (kind == 1) {
        const uint32_t slot = __builtin_amdgcn_readfirstlane(od.slot);
        const uint32_t woff = __builtin_amdgcn_readfirstlane(od.node);
        const uint32_t e = __builtin_amdgcn_readfirstlane(od.e);
        const bool in_c = __builtin_amdgcn_readfirstlane(od.in_c) != 0;
        const bool is_pred = __builtin_amdgcn_readfirstlane(od.is_pred) != 0;
        const uint32_t wn = d.lo + woff;
        // the pod, from its ring entry (released to the producers only below)
        const uint32_t rec = lane < KSG_WIN_SUM_DWORDS ? r_rec[e * KSG_WIN_SUM_DWORDS + lane] : 0u;
        const PodView pv = pod_view(rec);
        const uint32_t nss = __builtin_amdgcn_readlane(rec, WS_NSS);
        const uint32_t n_sel = nss & 0xffff, n_svcs = nss >> 16, nk = pv.nk;
        uint32_t base_nk = 0, base_ns = 0, om = 0;
        if (in_c) {
          base_nk = __builtin_amdgcn_readfirstlane(S.meta[slot].nk);
          base_ns = __builtin_amdgcn_readfirstlane(S.meta[slot].ns);
          om = __builtin_amdgcn_readfirstlane(S.meta[slot].smask);
        }
        // new slot: the node's snapshot (staged for the predicted node, else from HBM)
        if (!in_c && lane < 6) {
          uint64_t v;
          if (is_pred) {
            v = reinterpret_cast<const uint64_t*>(&r_hdr[e].cap_c)[lane];
          } else {
            const uint64_t* src = lane == 0   ? reinterpret_cast<const uint64_t*>(d.cap_cpu)
                                  : lane == 1 ? reinterpret_cast<const uint64_t*>(d.cap_mem)
                                  : lane == 2 ? reinterpret_cast<const uint64_t*>(d.used_cpu)
                                  : lane == 3 ? reinterpret_cast<const uint64_t*>(d.used_mem)
                                  : lane == 4 ? reinterpret_cast<const uint64_t*>(d.inv10_cpu)
                                              : reinterpret_cast<const uint64_t*>(d.inv10_mem);
            v = gld(src + wn);
          }
          uint64_t* dst = lane < 2   ? reinterpret_cast<uint64_t*>(&S.cap[slot]) + lane
                          : lane < 4 ? reinterpret_cast<uint64_t*>(&S.snp[slot]) + (lane - 2)
                                     : reinterpret_cast<uint64_t*>(&S.inv[slot]) + (lane & 1);
          *dst = v;
        }
        // the pod's keys and service entries, appended to the slot's lists
        const uint32_t my_key = (uint32_t)__shfl((int)rec, (int)(WS_IDS + (lane < nk ? lane : 0u)), 64);
        if (lane < nk) S.keys[(size_t)slot * KSG_SLOT_KEYS + base_nk + lane] = my_key;
        const bool sv_lane = lane < n_svcs;
        const uint32_t my_sv = (uint32_t)__shfl((int)rec, (int)min(WS_IDS + nk + n_sel + (sv_lane ? lane : 0u), 63u), 64);
        uint32_t new_mask = 0;
        if (n_svcs) {
          int32_t cnt = 0, mx = 0, peer = 0;
          uint32_t before = 0;
          bool changed = false;
          if (sv_lane) {
            cnt = is_pred ? r_svc[e].cnt[lane] : gld(d.svc_cnt + (size_t)my_sv * d.n_nodes + wn);
            mx = r_svc[e].max[lane];
            peer = r_svc[e].peer[lane];
            // in-window commits of this service on this node before this one
            const uint32_t* sl = S.svcs + (size_t)slot * KSG_SLOT_SVCS;
            for (uint32_t b = 0; b < base_ns; ++b) before += sl[b] == my_sv;
            changed = aff_on && peer == -1 && !((L_peerset[my_sv >> 5] >> (my_sv & 31)) & 1u);
            // ServiceAntiAffinity divides by the service's pod count: any commit changes it
            // (the re-rank takes that: later pods of the service are ranked again)
            changed |= anti_on && !rr;
            if (rr) atomicAdd(&L_nsv[my_sv], 1u);
          }
          // first commit of a service with no peer yet: record the peer (in order)
          uint64_t pm = __ballot(sv_lane && peer == -1);
          while (pm) {
            const uint32_t b = __builtin_ctzll(pm);
            pm &= pm - 1;
            const uint32_t fsv = (uint32_t)__builtin_amdgcn_readlane((int)my_sv, (int)b);
            const bool fresh = !((L_peerset[fsv >> 5] >> (fsv & 31)) & 1u);
            if (fresh) {
              if (lane == 0) {
                L_peerset[fsv >> 5] |= 1u << (fsv & 31);
                L_peer[2 * n_peer] = fsv;
                L_peer[2 * n_peer + 1] = wn;
              }
              ++n_peer;
              lds_fence();
            }
          }
          new_mask = wave_or_u32(sv_lane ? (1u << (my_sv & 31)) : 0u);
          if (sv_lane) {
            if (spread_on && cnt + (int32_t)before + 1 > mx) changed = true;  // maxCount rises
            S.svcs[(size_t)slot * KSG_SLOT_SVCS + base_ns + lane] = my_sv;
            S.scnt[(size_t)slot * KSG_SLOT_SVCS + base_ns + lane] = cnt;
            if (changed) atomicOr(&L_flag[my_sv >> 5], 1u << (my_sv & 31));
          }
        }
        lds_fence();
        if (lane == 0) {
          const I64x2 ov = in_c ? S.dl[slot] : I64x2{0, 0};
          S.dl[slot] = I64x2{(int64_t)((uint64_t)ov.c + (uint64_t)pv.req_c), (int64_t)((uint64_t)ov.m + (uint64_t)pv.req_m)};
          S.meta[slot] = SlotMeta{woff, base_nk + nk, base_ns + n_svcs, om | new_mask};
        }
      }
      if (lane == 0) {
        L_out[i] = outv;
        ctl->n_peer = n_peer;
        st_rel(&ctl->scribe_done, i + 1);
        st_rel(&ctl->consumed, i + 1);  // the pod's ring entry is free
      }
    }
    return;
  }

  // =========================================================================
  // committer (wave 0)
  // =========================================================================
  __builtin_amdgcn_s_setprio(3);
  uint32_t resolved = n_pods, reason = 0, n_slots = 0, n_draws = 0;
  uint32_t cn0 = ~0u, cn1 = ~0u;  // nodes of slots lane and 64 + lane (the committer's copy)
  // The slot the previous pod committed into, as it is after that commit, in
  // registers: the next pod re-checks it here (the checkers skip it) without
  // waiting for the scribe. Lists: lane t holds key t, service entry t.
  bool ls_valid = false;
  uint32_t ls_slot = KSG_NO_SLOT, ls_node = 0, ls_nk = 0, ls_ns = 0, ls_mask = 0;
  int64_t ls_cap_c = 0, ls_cap_m = 0, ls_snp_c = 0, ls_snp_m = 0, ls_dl_c = 0, ls_dl_m = 0;
  double ls_inv_c = 0.0, ls_inv_m = 0.0;
  uint32_t ls_key = 0, ls_sv = 0;
  int32_t ls_scnt = 0;
  uint32_t prev_nsv = 0, prev_sv = 0;  // the previous pod's services (lane t < prev_nsv)
  uint32_t ls_cnt_stale = 0;          // n > 0: ls_scnt misses the counts order n-1 loads

  auto wait_scribe = [&](uint32_t n) -> bool {  // the scribe has written orders [0, n)
    if (ld_acq(&ctl->scribe_done) >= n) return true;
    __builtin_amdgcn_s_setprio(0);  // (see the ring wait below)
    bool ok = true;
    for (uint32_t spin = 0; ld_acq(&ctl->scribe_done) < n; ++spin)
      if (spin > 16 * KSG_SPIN_LIMIT) {
        ok = false;
        break;
      }
    __builtin_amdgcn_s_setprio(3);
    return ok;
  };
  auto issue = [&](uint32_t i) {  // publish order i (written by the lanes before)
    lds_fence();
    if (lane == 0) st_rel(&ctl->order_seq, i + 1);
  };

  // KSG_DEBUG & 8: per-section s_memtime; lane k accumulates section k in a
  // VGPR (no scalar registers taken from the chain)
  uint64_t t_last = 0, t_acc = 0;
#define KSG_STAMP(k)                                         \
  if constexpr (STAMP) {                                     \
    const uint64_t t_now = __builtin_amdgcn_s_memtime();     \
    t_acc += lane == (uint32_t)(k) ? t_now - t_last : 0ULL;  \
    t_last = t_now;                                          \
  }
#define KSG_COUNT(k, v)                                    \
  if constexpr (STAMP) {                                   \
    t_acc += lane == (uint32_t)(k) ? (uint64_t)(v) : 0ULL; \
  }
  if constexpr (STAMP) t_last = __builtin_amdgcn_s_memtime();

  bool hung = false;
  for (uint32_t i = 0; i < n_pods; ++i) {
    const uint32_t e = i % KSG_RING, par = i & 1;
    if (ld_acq(&r_hdr[e].ready) != i + 1) {
      // waiting on a producer, one of which shares this SIMD: drop the issue
      // priority while spinning so it is not starved
      __builtin_amdgcn_s_setprio(0);
      for (uint32_t spin = 0; ld_acq(&r_hdr[e].ready) != i + 1; ++spin) {
        if (spin > 16 * KSG_SPIN_LIMIT) {
          hung = true;
          break;
        }
      }
      __builtin_amdgcn_s_setprio(3);
    }
    if (hung) {
      resolved = i;
      reason = KSG_STOP_HANG;
      break;
    }
    if constexpr (STAMP) {  // ring wait of the window's first 4 pods (10) vs the rest (11)
      const uint64_t t_now = __builtin_amdgcn_s_memtime();
      t_acc += lane == (i < 4 ? 10u : 11u) ? t_now - t_last : 0ULL;
    }
    KSG_STAMP(0)
    if (skew & 1u) __builtin_amdgcn_s_sleep(8);
    // ---- head
    const uint32_t rec = lane < KSG_WIN_SUM_DWORDS ? r_rec[e * KSG_WIN_SUM_DWORDS + lane] : 0u;
    const int32_t m0 = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].m0);
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(r_hdr[e].k0);
    const int32_t s = (int32_t)__builtin_amdgcn_readlane(rec, WS_SVC);
    uint32_t mv_n = 0;  // (re-rank) earlier window commits of the pod's service
    if (s >= 0 && (spread_on || aff_on || anti_on)) {
      // the flags of every earlier commit that may concern this pod's service
      const bool prev_has = __ballot(lane < prev_nsv && prev_sv == (uint32_t)s) != 0;
      if (!wait_scribe(prev_has ? i : (i ? i - 1 : 0))) {
        resolved = i;
        reason = KSG_STOP_HANG;
        break;
      }
      if ((L_flag[s >> 5] >> (s & 31)) & 1u) {
        resolved = i;  // a service scalar this pod reads changed in the window
        reason = KSG_STOP_SERVICE;
        break;
      }
      if (rr) mv_n = __builtin_amdgcn_readfirstlane(L_nsv[s]);
    }
    const bool moved = mv_n != 0;
    // (the order buffer of parity i was last used by order i-2)
    if (!wait_scribe(i >= 1 ? i - 1 : 0)) {
      resolved = i;
      reason = KSG_STOP_HANG;
      break;
    }
    WinOrder& od = L_ord[par];
    if (__builtin_amdgcn_readlane(rec, WS_ERR) || m0 == KSG_S32_NONE) {
      // ServiceAffinity peer error / nothing fit at the snapshot (commits only
      // remove fits): no draw, no commit. The checkers skip this pod too.
      if (lane == 0) {
        od.kind = 0;
        od.out = __builtin_amdgcn_readlane(rec, WS_ERR) ? KSG_OUT_ERROR : KSG_OUT_NOFIT;
        ctl->xs_slot = KSG_NO_SLOT;
        ctl->xs_nslots = n_slots;
        st_rel(&ctl->sel_seq, i + 1);
      }
      issue(i);
      prev_nsv = 0;
      ls_valid = false;  // (the next pod re-checks nothing; the checkers cover every slot)
      continue;
    }
    const PodView pv = pod_view(rec);
    const uint32_t nss = __builtin_amdgcn_readlane(rec, WS_NSS);
    const uint32_t n_sel = nss & 0xffff, n_svcs = nss >> 16, nk = pv.nk;
    if (__builtin_amdgcn_readlane(rec, WS_NINL) > KSG_WIN_INLINE || nk > KSG_SLOT_KEYS ||
        n_svcs > KSG_SLOT_SVCS) {
      // lists longer than the record / a slot: the exact per-pod kernel takes it
      resolved = i;
      reason = i == 0 ? KSG_STOP_OVERSIZE : KSG_STOP_SLOT;
      break;
    }
    KSG_STAMP(1)
    // ---- the slot the previous pod just committed into: re-check it here
    const uint64_t* t0e = r_t0 + (size_t)e * P * 64;
    bool a_drop = false;
    const bool a_in_t0 = ls_valid && ((t0e[ls_node >> 6] >> (ls_node & 63)) & 1ULL);
    // (re-rank: a node at its domain row's best may be a tie once the pod is ranked again)
    const bool a_in_b = ls_valid && rr && ((r_b[(size_t)e * P * 64 + (ls_node >> 6)] >> (ls_node & 63)) & 1ULL);
    if (a_in_t0 || a_in_b) {
      const int64_t now_c = (int64_t)((uint64_t)ls_snp_c + (uint64_t)ls_dl_c);
      const int64_t now_m = (int64_t)((uint64_t)ls_snp_m + (uint64_t)ls_dl_m);
      if (res_on && !pv.zero_req) {  // PodFitsResources
        const bool fc = ls_cap_c == 0 || ls_cap_c - now_c >= pv.req_c;
        const bool fm = ls_cap_m == 0 || ls_cap_m - now_m >= pv.req_m;
        a_drop = !(fc && fm);
      }
      if (nk && !a_drop && ls_nk) {  // PodFitsPorts / NoDiskConflict
        bool hit = false;
        if (lane < ls_nk) {
          if (ports_on)
            for (uint32_t b = 0; b < pv.n_ports; ++b) hit |= (uint32_t)__builtin_amdgcn_readlane(rec, WS_IDS + b) == ls_key;
          if (disk_on)
            for (uint32_t b = 0; b < pv.n_pds; ++b)
              hit |= (uint32_t)__builtin_amdgcn_readlane(rec, WS_IDS + pv.n_ports + b) == ls_key;
        }
        a_drop = __ballot(hit) != 0;
      }
      if (!a_drop && d.w_lr) {  // LeastRequested
        const int32_t lr_now = lr_win(now_c + pv.req_c, ls_cap_c, ls_inv_c) + lr_win(now_m + pv.req_m, ls_cap_m, ls_inv_m);
        const int32_t lr_snap =
            lr_win(ls_snp_c + pv.req_c, ls_cap_c, ls_inv_c) + lr_win(ls_snp_m + pv.req_m, ls_cap_m, ls_inv_m);
        a_drop = (lr_now >> 1) != (lr_snap >> 1);
      }
      if (!a_drop && spread_on && pv.s >= 0 && ((ls_mask >> (pv.s & 31)) & 1u)) {  // ServiceSpreading
        if (ls_cnt_stale) {  // the scribe loaded the counts of the last commit: take them from LDS
          if (!wait_scribe(ls_cnt_stale)) {
            resolved = i;
            reason = KSG_STOP_HANG;
            break;
          }
          ls_scnt = lane < ls_ns ? S.scnt[(size_t)ls_slot * KSG_SLOT_SVCS + lane] : 0;
          ls_cnt_stale = 0;
        }
        const uint64_t mm = __ballot(lane < ls_ns && ls_sv == (uint32_t)pv.s);
        if (mm) {
          const int32_t delta = (int32_t)__popcll(mm);
          const int32_t snapc = __builtin_amdgcn_readlane(ls_scnt, (int)__builtin_ctzll(mm));
          a_drop = frac10_i32(pv.smax - snapc - delta, pv.smax) != frac10_i32(pv.smax - snapc, pv.smax);
        }
      }
      a_drop = __builtin_amdgcn_readfirstlane((int)a_drop) != 0;
    }
    const uint32_t a_node = ls_node;
    KSG_STAMP(2)
    // ---- the checkers' drops for this pod (every slot but the last one)
    for (uint32_t spin = 0;; ++spin) {
      bool done = true;
#pragma unroll
      for (int c = 0; c < KSG_RES_NCHK; ++c) done = done && ld_acq(&ctl->chk_seq[c]) >= i + 1;
      if (done) break;
      if (spin > 16 * KSG_SPIN_LIMIT) {
        hung = true;
        break;
      }
    }
    if (hung) {
      resolved = i;
      reason = KSG_STOP_HANG;
      break;
    }
    uint32_t chk_drops = 0, chk_stop = 0;
#pragma unroll
    for (int c = 0; c < KSG_RES_NCHK; ++c) {
      chk_drops += __builtin_amdgcn_readfirstlane(ctl->chk_cnt[c][par]);
      chk_stop |= __builtin_amdgcn_readfirstlane(ctl->chk_stop[c][par]);
    }
    bool ls_counts = false;  // (re-rank) the last slot's node is still among the pod's filtered nodes
    if (anti_on && pv.s >= 0 && !chk_stop && ls_valid &&
        ((fit_word(e, i, ls_node >> 6) >> (ls_node & 63)) & 1ULL)) {
      // the last slot, from the register copy: does the pod still fit it?
      const int64_t now_c = (int64_t)((uint64_t)ls_snp_c + (uint64_t)ls_dl_c);
      const int64_t now_m = (int64_t)((uint64_t)ls_snp_m + (uint64_t)ls_dl_m);
      bool fit = true;
      if (res_on && !pv.zero_req)
        fit = (ls_cap_c == 0 || ls_cap_c - now_c >= pv.req_c) && (ls_cap_m == 0 || ls_cap_m - now_m >= pv.req_m);
      if (fit && nk && ls_nk) {
        bool hit = false;
        if (lane < ls_nk) {
          if (ports_on)
            for (uint32_t b = 0; b < pv.n_ports; ++b) hit |= (uint32_t)__builtin_amdgcn_readlane(rec, WS_IDS + b) == ls_key;
          if (disk_on)
            for (uint32_t b = 0; b < pv.n_pds; ++b)
              hit |= (uint32_t)__builtin_amdgcn_readlane(rec, WS_IDS + pv.n_ports + b) == ls_key;
        }
        fit = __ballot(hit) == 0;
      }
      if (!fit && anti_counts_move(d, ls_node, pv.s)) chk_stop = 1;
      ls_counts = fit;
    }
    if (chk_stop) {
      resolved = i;  // the pod's anti-affinity domain counts changed in the window
      reason = KSG_STOP_SERVICE;
      break;
    }
    KSG_STAMP(3)
    // ---- selection: k live ties, ix-th in descending rank = (k-1-ix)-th ascending
    const uint32_t dropped = chk_drops + ((a_drop && a_in_t0) ? 1u : 0u);
    if (!moved && dropped >= k0) {
      resolved = i;  // every snapshot tie got worse: needs a fresh snapshot
      reason = KSG_STOP_EXHAUSTED;
      break;
    }
    const uint32_t k = k0 - dropped;
    uint32_t woff;
    if (moved) {
      // ---- re-rank (calculateAntiAffinityPriority, spreading.go:104-168): the
      // service's pod count n and the pod's per-domain counts over its filtered
      // nodes moved with the window's commits of the service. A node's score is
      // its score without the anti term (unchanged unless the node was committed
      // in the window: those are the checkers' drops) plus its domain row's
      // term, so the best is among each row's best nodes at the snapshot (B) and
      // the sequential tie set is B minus drops, in the rows whose best + term
      // is the maximum. A row whose every B node dropped ends the window if its
      // snapshot best + term could still reach that maximum.
      KSG_COUNT(9, 64)
      uint64_t* dw = L_drop + (size_t)par * P * 64;
      const int32_t nn = (int32_t)__builtin_amdgcn_readlane(rec, WS_STOT) + (int32_t)mv_n;
      int32_t ls_add = 0;
      uint32_t ls_row = ~0u;
      if (ls_counts) {  // the last slot's commits of the service (the checkers skip that slot)
        const uint32_t kls = (uint32_t)__popcll(__ballot(lane < ls_ns && ls_sv == (uint32_t)s));
        if (kls) {
          const uint64_t zb = __ballot(lane + 1 < dz &&
                                       ((L_zm[(size_t)lane * P * 64 + (ls_node >> 6)] >> (ls_node & 63)) & 1ULL));
          if (zb) {
            ls_row = (uint32_t)__builtin_ctzll(zb);
            ls_add = (int32_t)kls;
          }
        }
      }
      int32_t cz = 0, mbz = KSG_S32_NONE;
      if (lane < dz) {
        cz = r_dc[e * KSG_RR_MAXZ + lane] + L_dca[par * KSG_RR_MAXZ + lane] +
             L_dca[(2 + par) * KSG_RR_MAXZ + lane] + (lane == ls_row ? ls_add : 0);
        mbz = r_mb[e * KSG_RR_MAXZ + lane];
      }
      // unlabelled nodes (row dz-1) score 0 (spreading.go:164-166)
      const int64_t aa = lane + 1 < dz ? (int64_t)d.w_anti[0] * frac10_f32((int64_t)nn - cz, nn) : 0;
      uint64_t lw[P];
#pragma unroll
      for (int q = 0; q < P; ++q) {
        lw[q] = r_b[(size_t)e * P * 64 + lane * P + q] & ~dw[lane * P + q];
        if (a_drop && lane * P + q == (a_node >> 6)) lw[q] &= ~(1ULL << (a_node & 63));
      }
      uint32_t livez = 0;
      for (uint32_t r = 0; r < dz; ++r) {
        uint32_t c1 = 0;
#pragma unroll
        for (int q = 0; q < P; ++q) c1 += __popcll(lw[q] & L_zm[(size_t)r * P * 64 + lane * P + q]);
        const uint32_t tr = wave_total_add(c1);
        if (lane == r) livez = tr;
      }
      const int32_t val = (lane < dz && mbz != KSG_S32_NONE) ? (int32_t)((int64_t)mbz + aa) : KSG_S32_NONE;
      const int32_t mlive = wave_total_max(livez > 0 ? val : KSG_S32_NONE);
      if (mlive == KSG_S32_NONE || __ballot(lane < dz && livez == 0 && mbz != KSG_S32_NONE && val > mlive)) {
        resolved = i;  // the best row's best nodes all got worse: needs a fresh snapshot
        reason = KSG_STOP_EXHAUSTED;
        break;
      }
      const bool zs = lane < dz && livez > 0 && val == mlive;
      const uint64_t zsel = __ballot(zs);
      const uint32_t k2 = wave_total_add(zs ? livez : 0u);
      const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r_hdr[e].r >> 32)) << 32) |
                         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r_hdr[e].r);
      const uint32_t ix = umod64_32(r, k2);
      uint64_t sw[P];
      uint32_t cl = 0;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        uint64_t m = 0;
        for (uint64_t zz = zsel; zz; zz &= zz - 1)
          m |= L_zm[(size_t)__builtin_ctzll(zz) * P * 64 + lane * P + q];
        sw[q] = lw[q] & m;
        cl += __popcll(sw[q]);
      }
      const uint32_t incl = dpp_scan_add(cl);
      woff = select_in_lanes<P>(sw, cl, incl, k2 - 1 - ix, lane);
    } else if (dropped == 0) {
      woff = (uint32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].pred);  // staged by the producer
    } else {
      KSG_COUNT(7, 64)
      uint32_t ix;
      if (dropped < 64 && !(d.dbg & 32)) {  // KSG_DEBUG & 32: always the direct modulo
        ix = __builtin_amdgcn_readfirstlane(r_mod[e * 64 + dropped]);
      } else {
        // (readfirstlane returns int: widen through uint32_t, no sign extension)
        const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r_hdr[e].r >> 32)) << 32) |
                           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r_hdr[e].r);
        ix = umod64_32(r, k);
      }
      // live ties: T0 minus the checkers' drops (lane l owns words l*P + q and
      // clears them for the pod two ahead) minus the re-checked slot's node
      uint64_t* dw = L_drop + (size_t)par * P * 64;
      uint64_t live[P];
#pragma unroll
      for (int q = 0; q < P; ++q) {
        live[q] = t0e[lane * P + q];
        if (chk_drops) {
          live[q] &= ~dw[lane * P + q];
          dw[lane * P + q] = 0;
        }
        if (a_drop && lane * P + q == (a_node >> 6)) live[q] &= ~(1ULL << (a_node & 63));
      }
      uint32_t cl = 0;
#pragma unroll
      for (int q = 0; q < P; ++q) cl += __popcll(live[q]);
      const uint32_t incl = dpp_scan_add(cl);
      woff = select_in_lanes<P>(live, cl, incl, k - 1 - ix, lane);
    }
    if (rr) {  // (re-rank: drops outside T0 are scattered too) clear them for the pod two ahead
#pragma unroll
      for (int q = 0; q < P; ++q) L_drop[(size_t)par * P * 64 + lane * P + q] = 0;
    }
    const uint32_t wn = d.lo + woff;
    KSG_STAMP(4)

    // ---- AssumePod: the slot and its state after this commit (registers); the
    // scribe applies the commit to the LDS slot state from the order
    const bool is_pred = (int32_t)woff == (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].pred);
    const uint64_t hit0 = __ballot(cn0 == woff);
    const uint64_t hit1 = __ballot(cn1 == woff);
    const bool in_c = (hit0 | hit1) != 0;
    uint32_t slot;
    bool cnt_wait = false;  // the register copy's counts of this pod's services are still loading
    if (in_c) {
      slot = hit0 ? (uint32_t)__builtin_ctzll(hit0) : 64u + (uint32_t)__builtin_ctzll(hit1);
      if (!(ls_valid && slot == ls_slot)) {
        // an older slot: its LDS state is final once the scribe is past order i-2
        if (!wait_scribe(i >= 1 ? i - 1 : 0)) {
          resolved = i;
          reason = KSG_STOP_HANG;
          break;
        }
        const I64x2 cp = S.cap[slot], sp = S.snp[slot], dl = S.dl[slot];
        const F64x2 iv = S.inv[slot];
        const SlotMeta me = S.meta[slot];
        ls_cap_c = cp.c; ls_cap_m = cp.m; ls_snp_c = sp.c; ls_snp_m = sp.m; ls_dl_c = dl.c; ls_dl_m = dl.m;
        ls_inv_c = iv.c; ls_inv_m = iv.m;
        ls_nk = me.nk; ls_ns = me.ns; ls_mask = me.smask;
        ls_key = lane < ls_nk ? S.keys[(size_t)slot * KSG_SLOT_KEYS + lane] : 0u;
        ls_sv = lane < ls_ns ? S.svcs[(size_t)slot * KSG_SLOT_SVCS + lane] : 0u;
        ls_scnt = lane < ls_ns ? S.scnt[(size_t)slot * KSG_SLOT_SVCS + lane] : 0;
      }
      if (ls_nk + nk > KSG_SLOT_KEYS || ls_ns + n_svcs > KSG_SLOT_SVCS) {
        resolved = i;  // this pod is redone (with the same draw) in the next window
        reason = KSG_STOP_SLOT;
        break;
      }
    } else {
      if (n_slots == KSG_MAX_SLOTS) {
        resolved = i;
        reason = KSG_STOP_SLOT;
        break;
      }
      slot = n_slots++;
      if (lane == (slot & 63)) {
        if (slot < 64) cn0 = woff;
        else cn1 = woff;
      }
    }
    // the choice is made: the checkers move on to pod i+1 (every slot but this
    // one), the scribe to the order
    if (lane == 0) {
      ctl->xs_slot = slot;
      ctl->xs_nslots = n_slots;
      st_rel(&ctl->sel_seq, i + 1);
      od.kind = 1;
      od.slot = slot;
      od.node = woff;
      od.out = (int32_t)wn;
      od.e = e;
      od.in_c = in_c;
      od.is_pred = is_pred;
    }
    issue(i);
    if (!in_c) {
      // snapshot of the node: staged by the producer when it is the predicted
      // node, else loaded here (L2-warm); the window's lists start empty
      if (is_pred) {
        ls_cap_c = r_hdr[e].cap_c; ls_cap_m = r_hdr[e].cap_m;
        ls_snp_c = r_hdr[e].used_c; ls_snp_m = r_hdr[e].used_m;
        ls_inv_c = r_hdr[e].inv_c; ls_inv_m = r_hdr[e].inv_m;
      } else {
        KSG_COUNT(8, 64)
        ls_cap_c = gld(d.cap_cpu + wn); ls_cap_m = gld(d.cap_mem + wn);
        ls_snp_c = gld(d.used_cpu + wn); ls_snp_m = gld(d.used_mem + wn);
        ls_inv_c = gld(d.inv10_cpu + wn); ls_inv_m = gld(d.inv10_mem + wn);
      }
      ls_dl_c = 0;
      ls_dl_m = 0;
      ls_nk = ls_ns = ls_mask = 0;
      ls_key = ls_sv = 0;
      ls_scnt = 0;
    }
    // this pod's keys and service entries, appended at lanes [ls_nk, +nk), [ls_ns, +n_svcs)
    const uint32_t base_nk = ls_nk, base_ns = ls_ns;
    const uint32_t tk = lane - base_nk, ts = lane - base_ns;
    const bool key_lane = lane >= base_nk && tk < nk, sv_lane = lane >= base_ns && ts < n_svcs;
    const uint32_t new_key = (uint32_t)__shfl((int)rec, (int)(WS_IDS + (key_lane ? tk : 0u)), 64);
    const uint32_t new_sv = (uint32_t)__shfl((int)rec, (int)min(WS_IDS + nk + n_sel + (sv_lane ? ts : 0u), 63u), 64);
    if (key_lane) ls_key = new_key;
    if (sv_lane) {
      ls_sv = new_sv;
      if (is_pred) ls_scnt = r_svc[e].cnt[ts];
      else cnt_wait = true;  // (the scribe loads it; read back from LDS if a re-check needs it)
    }
    ls_nk = base_nk + nk;
    ls_ns = base_ns + n_svcs;
    if (n_svcs) ls_mask |= wave_or_u32(sv_lane ? (1u << (new_sv & 31)) : 0u);
    ls_dl_c = (int64_t)((uint64_t)ls_dl_c + (uint64_t)pv.req_c);
    ls_dl_m = (int64_t)((uint64_t)ls_dl_m + (uint64_t)pv.req_m);
    ls_slot = slot;
    ls_node = woff;
    ls_valid = true;
    ls_cnt_stale = __builtin_amdgcn_readfirstlane((int)cnt_wait) != 0 ? i + 1 : 0u;
    prev_nsv = n_svcs;
    prev_sv = (uint32_t)__shfl((int)rec, (int)min(WS_IDS + nk + n_sel + (lane < n_svcs ? lane : 0u), 63u), 64);
    ++n_draws;
    KSG_STAMP(5)
  }
  // every other wave finishes: the scribe drains the orders issued (one per pod < resolved)
  if (lane == 0) st_rel(&ctl->stop, 1u);
  const bool drained = wait_scribe(resolved);
  if (!drained) reason = KSG_STOP_HANG;
  if (rr) {  // the producers staged this window's domain counts and row bests: reset them for the next
    for (uint32_t t = lane; t < x.dcnt_n; t += 64) x.dcnt[t] = 0;
    for (uint32_t t = lane; t < wcap * dz; t += 64) x.dmb[t] = KSG_S32_NONE;
    for (uint32_t t = lane; t < wcap * dz; t += 64) x.dmb[(size_t)wcap * dz + t] = 0;  // (B counts per row)
  }
  if constexpr (STAMP) {
    if (d.dbgbuf && lane < 16) atomicAdd(d.dbgbuf + lane, (int32_t)(t_acc / 64));
  }
#undef KSG_STAMP
#undef KSG_COUNT
  const uint32_t n_peer = __builtin_amdgcn_readfirstlane(ctl->n_peer);

  // ---- write the window's deltas back to HBM (the next snapshot) -------------
  for (uint32_t t = lane; t < n_slots; t += 64) {
    const SlotMeta me = S.meta[t];
    const uint32_t n = d.lo + me.node;
    const I64x2 snp = S.snp[t], dl = S.dl[t];
    d.used_cpu[n] = (int64_t)((uint64_t)snp.c + (uint64_t)dl.c);
    d.used_mem[n] = (int64_t)((uint64_t)snp.m + (uint64_t)dl.m);
    const uint32_t* ks = S.keys + (size_t)t * KSG_SLOT_KEYS;
    for (uint32_t a = 0; a < me.nk; ++a)
      __hip_atomic_fetch_or(d.keymap + (size_t)ks[a] * d.nw + (n >> 6), 1ULL << (n & 63), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t* sv = S.svcs + (size_t)t * KSG_SLOT_SVCS;
    const int32_t* sc = S.scnt + (size_t)t * KSG_SLOT_SVCS;
    for (uint32_t a = 0; a < me.ns; ++a) {
      const uint32_t sa = sv[a];
      bool first = true;
      int32_t count = 0;
      for (uint32_t b = 0; b < me.ns; ++b) {
        if (sv[b] == sa) {
          if (b < a) first = false;
          ++count;
        }
      }
      __hip_atomic_fetch_add(d.svc_total + sa, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (first) {
        const int32_t fin = sc[a] + count;
        d.svc_cnt[(size_t)sa * d.n_nodes + n] = fin;
        if (fin > 0)
          __hip_atomic_fetch_or(d.svc_bits + (size_t)sa * d.nw + (n >> 6), 1ULL << (n & 63), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(d.svc_max + sa, fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  for (uint32_t t = lane; t < n_peer; t += 64) {
    const uint32_t sv = L_peer[2 * t];
    int32_t expect = -1;
    __hip_atomic_compare_exchange_strong(d.svc_peer + sv, &expect, (int32_t)L_peer[2 * t + 1], __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (uint32_t t = lane; t < resolved; t += 64) out[t] = L_out[t];
  if (lane == 0) {
    *rng_io = rng0 + (uint64_t)n_draws * ksg_rng_step(d.draws);
    if (reason == KSG_STOP_HANG) {
      run->halt = KSG_HALT_HANG;
    } else if (reason == KSG_STOP_OVERSIZE) {
      run->halt = KSG_HALT_OVERSIZE;  // pod pos: the host runs the exact per-pod path, then resumes
    } else if (resolved == 0 || resolved > n_pods) {
      run->halt = KSG_HALT_BADCOUNT;
    } else {
      run->pos = pos + resolved;
      run->windows += 1;
      if (reason >= 1 && reason <= 3) run->stops[reason] += 1;
    }
  }
}

// ---------------------------------------------------------------------------
// phase B, register-slot resolver (every configuration without
// ServiceAntiAffinity; that one keeps the resolver above)
// ---------------------------------------------------------------------------
// The window's committed nodes ("slots", at most 128) are owned by two checker
// waves, one slot per lane: the node's capacity, snapshot and window delta of
// the requested totals and 10/capacity live in the owner lane's registers; the
// conflict keys and service entries the window added live in an LDS table by
// slot (keys and service ids written by the committer at the commit, the
// services' snapshot counts by the owner checker).
//  CHECKERS run a pod ahead of the committer: for pod i they apply commit i-2
//    (a new slot takes the node's snapshot from the producer's staging when it
//    is the predicted node, else from L2; the service flags and first peers
//    later pods stop on are set here) and test pod i against every slot as of
//    commits <= i-2.
//  COMMITTER (wave 0) re-checks only the slot commit i-1 went into (its window
//    delta in registers, its lists from the table, the node's snapshot loaded at
//    the top of the iteration), adds the checkers' drops (a commit can only
//    make a node worse, so drops as of i-2 stay drops), selects the ix-th live
//    tie (the staged prediction when nothing dropped), writes the pod's lists
//    into the table and publishes the commit record.
//  PRODUCERS stage pods ahead into the ring. The draw index of pod j is the
//    number of drawable pods before j, read from two LDS bitmaps every producer
//    fills as soon as it knows its pod's max score (no producer-to-producer
//    hand-off chain).
// one per window pod; the first 16 bytes are the commit record (one 16-byte store),
// then the pod's answer and its drawn node (written apart)
struct alignas(16) WinCommit {
  uint32_t kind;   // 0: no commit (error / no fit), 1: commit
  uint32_t slot;
  uint32_t node;   // shard offset of the node
  uint32_t flags;  // bit 0: a new slot, bit 1: the node is the producer's predicted node,
                   // bits 8..15: the pod's service count
  int32_t out;     // the pod's answer
  uint32_t xn;     // node drawn (~0u: no commit), for the x-checker
  uint32_t pad[2];
};
struct alignas(16) WinCtl2 {
  uint32_t stop;      // the committer is done: pods [0, resolved) are decided
  uint32_t resolved;
  uint32_t sel_seq;   // commit records published for pods [0, sel_seq)
  uint32_t n_peer;    // first service peers recorded in the window (L_peer entries)
  uint32_t chk_seq[KSG_RES_NCHK];     // pods checker c is done with
  uint32_t chk_cnt[KSG_RES_NCHK][2];  // checker c's drops for the pod of parity p
  // (no ServiceAntiAffinity) checker c's dropping slots for the pod of parity p
  // (lane l: slot 64c + l; its drop's ascending T0 position is in L_dpos)
  uint32_t chk_msk[KSG_RES_NCHK][2][2];
  uint32_t fin[KSG_RES_NCHK];         // checker c applied every commit and wrote its slots back
  uint32_t hang;                      // a wait exceeded its spin limit (a bug)
  uint32_t xseq;                      // pods the x-checker is done with
  uint32_t xres[2];                   // its verdict for the pod of parity p: bit 0 x drops, bit 1 flag
  // pods whose drawn node is posted in L_xn (~0u: no commit), posted right after
  // the draw so the x-checker's work overlaps the rest of the commit
  uint32_t xn_seq, xn_pad;
  uint32_t fin_x;                     // the x-checker applied every commit's flags and first peers
  uint32_t pad[1];
  uint32_t t_x, t_n;                  // KSG_DEBUG & 8: clock at the xres / xn posts
  // ServiceAntiAffinity (re-rank): checker c found a slot the pod fitted at the
  // snapshot, no longer fits, labelled and holding pods of its service (the
  // domain counts moved: the window ends); the x-checker's correction of the
  // domain count of commit i-1's node's row (row ~0u: none), by pod parity
  uint32_t chk_stop[KSG_RES_NCHK][2];
  uint32_t xdz[2];
  int32_t xdc[2];
  uint32_t xrw[2];  // domain row of commit i-1's node (its drop's row)
  // window commits of the pod's service up to commit i-2, read by the x-checker
  // before it applies commit i-1's (the committer adds commit i-1 itself)
  uint32_t xnsv[2];
};

struct WinLdsOff2 {
  // r_lp: per ring entry and lane, the T0 bits in lanes below / up to it
  // (exclusive, inclusive prefix); r_wp: per ring entry and word, the T0 bits
  // in the lane's words below it (u16); dpos: the checkers' drop positions in
  // T0 by pod parity and slot (no ServiceAntiAffinity: the sparse select)
  uint32_t r_lp, r_wp, dpos;
  uint32_t ctl, r_hdr, r_t0, r_rec, r_mod, r_svc;
  uint32_t cm, peer, flag, peerset, drop, pub, drw, clist;
  // ServiceAntiAffinity re-rank (dz > 0; see the LDS-slot resolver's WinLdsOff)
  uint32_t r_fit, r_b, r_mb, r_dc, zm, nsv, dca, r_kz, ddr;
  uint32_t total;
};


// (rr: the re-rank's arrays; -1: iff dz > 0; the kernel passes a constant)
__host__ __device__ inline WinLdsOff2 win2_lds_offsets(uint32_t P, uint32_t nflag, uint32_t W, uint32_t dz = 0,
                                                       uint32_t nsvc = 0, int rr_ = -1) {
  WinLdsOff2 o;
  const uint32_t R = win2_ring(P, dz != 0);
  uint32_t at = 0;
  o.ctl = at;     at += win_al16(sizeof(WinCtl2));
  o.r_hdr = at;   at += win_al16((size_t)R * sizeof(RingHdr));
  o.r_t0 = at;    at += win_al16((size_t)R * P * 64 * 8);
  o.r_rec = at;   at += win_al16((size_t)R * KSG_WIN_SUM_DWORDS * 4);
  o.r_mod = at;   at += win_al16((size_t)R * 64 * 4);
  o.r_svc = at;   at += win_al16((size_t)R * sizeof(RingSvc));
  // fixed sizes first (given P and whether the re-rank runs): their offsets are
  // compile-time constants in the kernel, not registers the roles' loops keep
  const bool rr = rr_ < 0 ? dz != 0 : rr_ != 0;
  o.clist = at;   at += win_al16((size_t)KSG_MAX_SLOTS * KSG_CL_W * 4);
  o.drop = at;    at += rr ? win_al16((size_t)2 * P * 64 * 8) : 0u;  // (the re-rank's drop bitmap)
  // (P > 16: the fit and B bitmaps are read from phase A's output instead, win2_fg)
  o.r_fit = at;   at += rr && !win2_fg(P) ? win_al16((size_t)R * P * 64 * 8) : 0u;
  o.r_b = at;     at += rr && !win2_fg(P) ? win_al16((size_t)R * P * 64 * 8) : 0u;
  o.r_mb = at;    at += rr ? win_al16((size_t)R * KSG_RR_MAXZ * 4) : 0u;
  o.r_dc = at;    at += rr ? win_al16((size_t)R * KSG_RR_MAXZ * 4) : 0u;
  o.dca = at;     at += rr ? win_al16((size_t)KSG_RES_NCHK * 2 * KSG_RR_MAXZ * 4) : 0u;
  o.r_kz = at;    at += rr ? win_al16((size_t)R * KSG_RR_MAXZ * 4) : 0u;
  o.ddr = at;     at += rr ? win_al16((size_t)KSG_RES_NCHK * 2 * KSG_RR_MAXZ * 4) : 0u;
  o.r_lp = at;    at += rr ? 0u : win_al16((size_t)R * 64 * 8);
  o.r_wp = at;    at += rr ? 0u : win_al16((size_t)R * P * 64 * 2);
  o.dpos = at;    at += rr ? 0u : win_al16((size_t)2 * KSG_MAX_SLOTS * 4);
  o.cm = at;      at += win_al16((size_t)W * sizeof(WinCommit));
  o.peer = at;    at += win_al16((size_t)W * 2 * 4);
  o.pub = at;     at += win_al16((size_t)((W + 31) / 32) * 4);
  o.drw = at;     at += win_al16((size_t)((W + 31) / 32) * 4);
  o.flag = at;    at += win_al16((size_t)nflag * 4);
  o.peerset = at; at += win_al16((size_t)nflag * 4);
  o.zm = at;      at += win2_zg(P) ? 0u : win_al16((size_t)dz * P * 64 * 8);  // (P > 8: from HBM, win2_zg)
  o.nsv = at;     at += rr ? win_al16((size_t)nsvc * 4) : 0u;
  o.total = at;
  return o;
}


// ANTI: ServiceAntiAffinity with the re-rank (x.rr; the LDS-slot resolver above
// takes every other anti-affinity configuration)
//
// Hand-offs (LDS; every poll is relaxed loads then one LDS-only acquire fence,
// every post a workgroup-scope release store after the data it covers):
//
//   flag / data              writer      reader              pod index        ordered by
//   r_hdr[e].ready + entry   producer j  all but producers   j                ready = j+1 release after the entry
//    (record, T0, fit, B,                                                     (lane prefixes r_lp / r_wp too)
//    row bests / counts)
//   L_pub / L_drw bits       producer j  producers > j       j                L_drw before L_pub (atomicOr, in order)
//   L_cm[i].xn               committer   x-checker           i (checks i+1)   xn_seq = i+1 release after it
//   L_cm[i] record, .out,    committer   checkers (apply i   i                sel_seq = i+1 release after them
//    slot row keys / ids                 at pod i+2)
//   slot row counts          checker     checkers,           commits <= i-2   chk_seq release (the x-checker
//                            (apply)     x-checker                            reads rows of commits it replayed)
//   chk_seq[c], chk_cnt,     checker c   committer,          i                chk_seq[c] = i+1 release after the
//    chk_msk, L_dpos,                    producers                            masks, counts, positions and the
//    chk_stop, L_dca, L_ddr                                                   anti-affinity row sums
//   xres, xdz, xdc, xrw,     x-checker   committer           i                xseq = i+1 release after them
//    xnsv [i & 1]
//   L_flag, L_peer,          x-checker   committer           commits <= i-2   program order in the x-checker,
//    L_peerset, n_peer,                  (reads at pod i)                     xseq >= i+1 acquired by the committer
//    L_nsv
//   stop, resolved           committer   all                 —                stop = 1 release after resolved
//   fin[c], fin_x            checkers,   committer           —                release after the write-back /
//                            x-checker                                        the last first peers
//
// Ring entry e = j mod RING is rewritten for pod j once the checkers are done
// with pod j-RING+2 and the x-checker with pod j-RING+1. Every wait has a spin
// limit; a timed-out wait sets ctl->hang and the host fails the batch. KSG_DEBUG
// bits 16..19 add a fixed delay per pod to the committer, x-checker, checkers or
// producers (tests/test_gpu_fuzz.py runs each skew once against the oracle).
template <int P, bool STAMP, bool ANTI>
__global__ __launch_bounds__(512) void ksg_win_resolve2_kernel(KsgDev d, uint32_t wcap, KsgWinRun* run,
                                                               const KsgWinSum* __restrict__ sums,
                                                               const KsgWinXchg x, uint64_t* rng_io,
                                                               int32_t* __restrict__ out_batch) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t pos = run->pos, n_batch = run->n;
  if (run->halt || pos >= n_batch) return;  // the chain is done (uniform, before any barrier)
  const uint32_t n_pods = min(wcap, n_batch - pos);
  int32_t* __restrict__ out = out_batch + pos;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nflag = (d.n_services + 31) / 32;
  const uint32_t nwords = d.nwords;
  constexpr uint32_t RING = win2_ring(P, ANTI);
  constexpr uint32_t NT = 512;
  constexpr uint32_t NPW = NT / 64 - KSG_RES_P0;  // producer waves
  constexpr uint32_t DW = KSG_WIN_SUM_DWORDS;
  const uint32_t dz = ANTI ? x.dz : 0u;
  const WinLdsOff2 o = win2_lds_offsets(P, nflag, wcap, dz, d.n_services, ANTI ? 1 : 0);
  uint64_t* const r_fit = reinterpret_cast<uint64_t*>(smem + o.r_fit);  // [ring][P*64] fit at the snapshot
  uint64_t* const r_b = reinterpret_cast<uint64_t*>(smem + o.r_b);      // [ring][P*64] best-per-row nodes
  int32_t* const r_mb = reinterpret_cast<int32_t*>(smem + o.r_mb);      // [ring][KSG_RR_MAXZ] best per row
  int32_t* const r_dc = reinterpret_cast<int32_t*>(smem + o.r_dc);      // [ring][KSG_RR_MAXZ] domain counts
  uint64_t* const L_zm = reinterpret_cast<uint64_t*>(smem + o.zm);      // [dz][P*64] nodes of each row
  uint32_t* const L_nsv = reinterpret_cast<uint32_t*>(smem + o.nsv);    // window commits per service
  int32_t* const L_dca = reinterpret_cast<int32_t*>(smem + o.dca);      // [chk][parity][KSG_RR_MAXZ]
  int32_t* const r_kz = reinterpret_cast<int32_t*>(smem + o.r_kz);      // [ring][KSG_RR_MAXZ] B nodes per row
  int32_t* const L_ddr = reinterpret_cast<int32_t*>(smem + o.ddr);      // [chk][parity][KSG_RR_MAXZ] B drops per row
  WinCtl2* ctl = reinterpret_cast<WinCtl2*>(smem + o.ctl);
  RingHdr* r_hdr = reinterpret_cast<RingHdr*>(smem + o.r_hdr);
  uint64_t* r_t0 = reinterpret_cast<uint64_t*>(smem + o.r_t0);
  uint32_t* r_rec = reinterpret_cast<uint32_t*>(smem + o.r_rec);
  uint32_t* r_mod = reinterpret_cast<uint32_t*>(smem + o.r_mod);
  RingSvc* r_svc = reinterpret_cast<RingSvc*>(smem + o.r_svc);
  // per window pod: commit record, answer and drawn node (the drawn node one entry per pod: the
  // committer runs ahead of the x-checker through pods that make no commit, so a single mailbox
  // would be overwritten before the x-checker reads commit p's node)
  WinCommit* L_cm = reinterpret_cast<WinCommit*>(smem + o.cm);
  uint32_t* L_peer = reinterpret_cast<uint32_t*>(smem + o.peer);
  uint32_t* L_flag = reinterpret_cast<uint32_t*>(smem + o.flag);
  uint32_t* L_peerset = reinterpret_cast<uint32_t*>(smem + o.peerset);
  uint64_t* L_drop = reinterpret_cast<uint64_t*>(smem + o.drop);  // [2][P*64] by pod parity
  uint32_t* L_pub = reinterpret_cast<uint32_t*>(smem + o.pub);    // pods whose drawable bit is known
  uint32_t* L_drw = reinterpret_cast<uint32_t*>(smem + o.drw);    // drawable pods
  uint32_t* L_cl = reinterpret_cast<uint32_t*>(smem + o.clist);   // [slot][KSG_CL_W]
  uint32_t* r_lp = reinterpret_cast<uint32_t*>(smem + o.r_lp);    // [ring][64][2] lane prefix (excl, incl)
  uint16_t* r_wp = reinterpret_cast<uint16_t*>(smem + o.r_wp);    // [ring][P*64] prefix within the lane
  uint32_t* L_dpos = reinterpret_cast<uint32_t*>(smem + o.dpos);  // [2][KSG_MAX_SLOTS] drop positions
  const bool spread_on = d.w_spread != 0;
  const bool aff_on = (d.preds & KSG_PRED_SERVICEAFFINITY) && d.n_aff > 0;
  const bool res_on = (d.preds & KSG_PRED_PODFITSRESOURCES) != 0;
  const bool ports_on = (d.preds & KSG_PRED_PODFITSPORTS) != 0;
  const bool disk_on = (d.preds & KSG_PRED_NODISKCONFLICT) != 0;
  const uint32_t nbits = (wcap + 31) / 32;
  // KSG_DEBUG bits 16..19: a fixed delay per pod in one role (committer, x-checker, checkers,
  // producers): another interleaving of the hand-offs than the natural one (tests/test_gpu_fuzz.py)
  // (the debug instantiation only: the production one keeps no debug switch in a register)
  const uint32_t skew = STAMP ? ((uint32_t)d.dbg >> 16) & 15u : 0u;
  // (P > 8 / P > 16, win2_zg / win2_fg) the domain rows' node bitmaps and the pod's fit / B bitmaps
  // from HBM: word w of domain row r (x.zmap), word w of window pod j's phase-A row at byte offset
  // off (x.fit_off, x.b_off; the re-rank runs on one rank, so word w sits at w * 8); words past
  // the shard read 0, as their LDS copies do
  constexpr bool ZG = ANTI && win2_zg(P), FG = ANTI && win2_fg(P);
  auto zm_word = [&](uint32_t r, uint32_t w) -> uint64_t {
    if constexpr (ZG) return w < nwords ? gld(x.zmap + (size_t)r * d.nw + d.wlo + w) : 0ULL;
    else return L_zm[(size_t)r * P * 64 + w];
  };
  auto pa_word = [&](uint32_t off, uint32_t j, uint32_t w) -> uint64_t {
    return w < nwords ? gld(reinterpret_cast<const uint64_t*>(x.buf + off + (size_t)j * x.ostride * 8 + (size_t)w * 8))
                      : 0ULL;
  };

  for (uint32_t t = tid; t < RING; t += NT) r_hdr[t].ready = 0;
  if (tid == 0) *ctl = WinCtl2{};
  for (uint32_t w = tid; w < nflag; w += NT) {
    L_flag[w] = 0;
    L_peerset[w] = 0;
  }
  for (uint32_t w = tid; w < nbits; w += NT) {
    L_pub[w] = 0;
    L_drw[w] = 0;
  }
  if constexpr (ANTI)
    for (uint32_t w = tid; w < 2 * P * 64u; w += NT) L_drop[w] = 0;
  if constexpr (ANTI) {
    if constexpr (!ZG)
      for (uint32_t t = tid; t < dz * P * 64; t += NT) {
        const uint32_t row = t / (P * 64), w = t % (P * 64);
        L_zm[t] = w < nwords ? x.zmap[(size_t)row * d.nw + d.wlo + w] : 0ULL;
      }
    for (uint32_t t = tid; t < d.n_services; t += NT) L_nsv[t] = 0;
  }
  __syncthreads();
  const uint64_t rng0 = *rng_io;

  // =========================================================================
  // producers
  // =========================================================================
  if (wave >= KSG_RES_P0) {
    const uint32_t* recs = reinterpret_cast<const uint32_t*>(sums);
    uint32_t wb_at[P], wm_at[P];
#pragma unroll
    for (int q = 0; q < P; ++q) {
      // lane l holds words l*P + q (ServiceAntiAffinity: the LDS-slot layout its
      // re-rank walks), else q*64 + l (coalesced loads, bank-conflict-free LDS)
      const uint32_t wq = ANTI ? lane * P + q : q * 64 + lane;
      uint32_t g = 0;
      for (uint32_t r = 1; r < x.world; ++r)
        if (wq >= x.wlo[r] && x.nw[r] > 0) g = r;
      const uint32_t i = wq - x.wlo[g];
      const bool ok = wq < nwords && i < x.nw[g];
      const uint32_t base = (uint32_t)(g * x.blk);
      wb_at[q] = ok ? base + i * 8 : ~0u;
      wm_at[q] = ok ? base + x.wcap * x.ostride * 8 + i * 4 : ~0u;
    }
    const uint32_t row_b = x.ostride * 8, row_m = x.ostride * 4;
    uint64_t p_last = 0, p_acc = 0;  // KSG_DEBUG & 8: lanes 24..27 ring wait, loads, draw wait, the rest
    auto pstamp = [&](uint32_t k) {
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        p_acc += lane == k ? t_now - p_last : 0ULL;
        p_last = t_now;
      }
    };
    if constexpr (STAMP) p_last = __builtin_amdgcn_s_memtime();
    for (uint32_t j = wave - KSG_RES_P0; j < n_pods; j += NPW) {
      const uint32_t e = j % RING;
      // ring entry free: the checkers applied the commit of pod j - RING (while
      // checking pod j - RING + 2), so neither they nor the committer need it
      for (uint32_t spin = 0;; ++spin) {
        if (ld_acq(&ctl->stop)) return;
        if (spin > KSG_SPIN_LIMIT) {
          ctl->hang = 1;
          return;
        }
        uint32_t done = ld_acq(&ctl->xseq);  // (the x-checker of pod i reads pod i-1's entry until it is done)
#pragma unroll
        for (int c = 0; c < KSG_RES_NCHK; ++c) done = min(done, ld_acq(&ctl->chk_seq[c]));
        if (j < RING || done + RING >= j + 3) break;
        __builtin_amdgcn_s_sleep(1);
      }
      pstamp(24);
      if (skew & 8u) __builtin_amdgcn_s_sleep(8);
      const uint32_t rec = lane < DW ? recs[(size_t)j * DW + lane] : 0u;
      uint64_t t0[P];
      int32_t mw[P];
      int32_t lm = KSG_S32_NONE;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        t0[q] = wb_at[q] != ~0u ? *reinterpret_cast<const uint64_t*>(x.buf + wb_at[q] + j * row_b) : 0ULL;
        mw[q] = wm_at[q] != ~0u ? *reinterpret_cast<const int32_t*>(x.buf + wm_at[q] + j * row_m) : KSG_S32_NONE;
        lm = mw[q] > lm ? mw[q] : lm;
      }
      const int32_t m0 = wave_total_max(lm);
      const bool drawable = __builtin_amdgcn_readlane(rec, WS_ERR) == 0 && m0 != KSG_S32_NONE;
      const uint32_t wj = j >> 5, bj = 1u << (j & 31);
      if (lane == 0) {  // the drawable bit first, then "known" (readers read them in that order)
        if (drawable) atomicOr(&L_drw[wj], bj);
        atomicOr(&L_pub[wj], bj);
      }
      uint32_t cnt = 0;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        t0[q] = (m0 != KSG_S32_NONE && mw[q] == m0) ? t0[q] : 0ULL;
        cnt += __popcll(t0[q]);
      }
      uint32_t incl = 0, k0 = 0;
      // (q-major) per row q = words [64q, 64q + 64): the T0 bits below each lane's
      // word in the row (ex_q) and below the row (rowex[q], wave-uniform)
      uint32_t ex_q[P], rowex[P];
      if constexpr (ANTI) {
        incl = dpp_scan_add(cnt);
        k0 = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      } else {
#pragma unroll
        for (int q = 0; q < P; ++q) {
          const uint32_t c1 = (uint32_t)__popcll(t0[q]);
          const uint32_t in1 = dpp_scan_add(c1);
          ex_q[q] = in1 - c1;
          rowex[q] = k0;
          k0 += (uint32_t)__builtin_amdgcn_readlane((int)in1, 63);
        }
      }
      pstamp(25);
      // draw index = drawable pods before j (every one of them known)
      uint32_t idx = 0;
      for (uint32_t spin = 0;; ++spin) {
        if (ld_acq(&ctl->stop)) return;
        if (spin > KSG_SPIN_LIMIT) {
          ctl->hang = 1;
          return;
        }
        bool all = true;
        idx = 0;
        for (uint32_t w = 0; w <= wj; ++w) {
          const uint32_t mask = w < wj ? ~0u : bj - 1u;
          const uint32_t pub = __builtin_amdgcn_readfirstlane(ld_acq(&L_pub[w]));
          all = all && (pub & mask) == mask;
          idx += __popc(__builtin_amdgcn_readfirstlane(L_drw[w]) & mask);
        }
        if (all) break;
        __builtin_amdgcn_s_sleep(1);
      }
      pstamp(26);
      const uint64_t r = ksg_rng_draw(d.draws, rng0 + (uint64_t)idx * ksg_rng_step(d.draws));  // rand.Int() (generic_scheduler.go:94)
      uint32_t mv = 0;
      if (drawable && lane < k0) mv = umod64_32(r, k0 - lane);
      int32_t pred = -1;
      int64_t pv = 0;  // lanes 0..3: cap_c, cap_m, used_c, used_m of pred
      double pinv = 0.0;
      const uint32_t n_svcs = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NSS) >> 16;
      const uint32_t nk = ((uint32_t)__builtin_amdgcn_readlane(rec, WS_NPP) & 0xffff) +
                          ((uint32_t)__builtin_amdgcn_readlane(rec, WS_NPP) >> 16);
      const uint32_t n_sel = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NSS) & 0xffff;
      const bool inl = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NINL) <= KSG_WIN_INLINE && n_svcs <= KSG_SLOT_SVCS;
      const uint32_t t_sv = lane < n_svcs ? lane : 0u;
      const uint32_t my_sv = (uint32_t)__shfl((int)rec, (int)min(WS_IDS + nk + n_sel + t_sv, 63u), 64);
      int32_t s_cnt = 0, s_max = 0, s_peer = 0;
      if (drawable) {
        const uint32_t ix0 = __builtin_amdgcn_readfirstlane(mv);  // lane 0: r mod k0
        if constexpr (ANTI) pred = (int32_t)select_in_lanes<P>(t0, cnt, incl, k0 - 1 - ix0, lane);
        else pred = (int32_t)select_qmajor<P>(t0, ex_q, rowex, k0 - 1 - ix0, lane);
        const uint32_t pn = d.lo + (uint32_t)pred;
        if (lane == 0) pv = d.cap_cpu[pn];
        else if (lane == 1) pv = d.cap_mem[pn];
        else if (lane == 2) pv = d.used_cpu[pn];
        else if (lane == 3) pv = d.used_mem[pn];
        if (inl && lane < n_svcs) {
          s_cnt = d.svc_cnt[(size_t)my_sv * d.n_nodes + pn];
          s_max = d.svc_max[my_sv];
          s_peer = d.svc_peer[my_sv];
        }
        pinv = lr_inv10(pv);
      }
      r_mod[e * 64 + lane] = mv;
      if (lane < DW) r_rec[e * DW + lane] = rec;
      if constexpr (ANTI) {
#pragma unroll
        for (int q = 0; q < P; ++q) r_t0[(size_t)e * P * 64 + lane * P + q] = t0[q];
      } else {
        // T0 by word, and the sparse select's prefix counts: T0 bits below each
        // row (r_lp[q] = {below, up to the row's end}) and below each word within
        // its row (r_wp, u16), so the ascending position of node n in T0 is
        // r_lp[n >> 12] + r_wp[n >> 6] + the bits below n in its word
        uint32_t lpe = 0, lpi = 0;
#pragma unroll
        for (int q = 0; q < P; ++q) {
          r_t0[(size_t)e * P * 64 + q * 64 + lane] = t0[q];
          r_wp[(size_t)e * P * 64 + q * 64 + lane] = (uint16_t)ex_q[q];
          if (lane == (uint32_t)q) {
            lpe = rowex[q];
            lpi = q + 1 < P ? rowex[q + 1 < P ? q + 1 : q] : k0;
          }
        }
        if (lane < P) {
          r_lp[(e * 64 + lane) * 2] = lpe;
          r_lp[(e * 64 + lane) * 2 + 1] = lpi;
        }
      }
      if constexpr (ANTI) {  // fit at the snapshot, best-per-row nodes, row bests, domain counts
        uint64_t bw[P];
#pragma unroll
        for (int q = 0; q < P; ++q) {
          bw[q] = wb_at[q] != ~0u ? *reinterpret_cast<const uint64_t*>(x.buf + wb_at[q] + x.b_off + j * row_b) : 0ULL;
          if constexpr (!FG) {
            r_fit[(size_t)e * P * 64 + lane * P + q] =
                wb_at[q] != ~0u ? *reinterpret_cast<const uint64_t*>(x.buf + wb_at[q] + x.fit_off + j * row_b) : 0ULL;
            r_b[(size_t)e * P * 64 + lane * P + q] = bw[q];
          }
        }
        // B nodes per domain row (the committer's re-rank subtracts the drops): counted here over
        // the LDS row bitmaps, past 32k nodes by phase A (win2_zg)
        int32_t kz = 0;
        if constexpr (ZG) {
          if (lane < dz) kz = x.dmb[(size_t)wcap * dz + (size_t)j * dz + lane];
        } else {
          for (uint32_t rw = 0; rw < dz; ++rw) {
            uint32_t c1 = 0;
#pragma unroll
            for (int q = 0; q < P; ++q) c1 += __popcll(bw[q] & L_zm[(size_t)rw * P * 64 + lane * P + q]);
            const uint32_t tr = wave_total_add(c1);
            if (lane == rw) kz = (int32_t)tr;
          }
        }
        if (lane < dz) r_kz[e * KSG_RR_MAXZ + lane] = kz;
        if (lane < dz) {
          r_mb[e * KSG_RR_MAXZ + lane] = x.dmb[(size_t)j * dz + lane];
          r_dc[e * KSG_RR_MAXZ + lane] =
              lane + 1 < dz ? x.dcnt[(size_t)j * d.n_domains_total + d.anti_dom_off[0] + lane] : 0;
        }
      }
      if (inl && lane < n_svcs) {
        r_svc[e].cnt[lane] = s_cnt;
        r_svc[e].max[lane] = s_max;
        r_svc[e].peer[lane] = s_peer;
      }
      if (lane < 4) (&r_hdr[e].cap_c)[lane] = pv;
      if (lane < 2) (&r_hdr[e].inv_c)[lane] = pinv;
      if (lane == 0) {
        r_hdr[e].m0 = m0;
        r_hdr[e].k0 = k0;
        r_hdr[e].r = r;
        r_hdr[e].drawable = drawable;
        r_hdr[e].pred = pred;
        st_rel(&r_hdr[e].ready, j + 1);
      }
      pstamp(27);
    }
    if constexpr (STAMP) {
      if (d.dbgbuf && lane >= 24 && lane < 28) atomicAdd(d.dbgbuf + lane, (int32_t)(p_acc / 64));
    }
    return;
  }

  // =========================================================================
  // checkers (waves KSG_RES_C0 ..): lane l of checker c owns slot 64c + l
  // =========================================================================
  if (wave >= KSG_RES_C0) {
    __builtin_amdgcn_s_setprio(2);
    const uint32_t c = wave - KSG_RES_C0;
    const uint32_t my_slot = c * 64 + lane;
    const uint32_t* my_cl = L_cl + (size_t)my_slot * KSG_CL_W;
    RegSlot S;
    S.node = ~0u;
    S.cap_c = S.cap_m = S.snp_c = S.snp_m = S.dl_c = S.dl_m = 0;
    S.inv_c = S.inv_m = 0.0;
    S.nk = S.ns = S.smask = 0;
    S.row = ~0u;
    // AssumePod of pod p (plugin/pkg/scheduler/scheduler.go:115-118) into the
    // owner lane's slot: requested totals, list lengths; the services' snapshot
    // counts into the table (the x-checker applies the service flags, in commit
    // order)
    auto apply = [&](uint32_t p) {
      // (the commit record's 16 bytes and the pod's record in one round of LDS reads)
      const uint4 cmv = *reinterpret_cast<const uint4*>(&L_cm[p]);
      const uint32_t ep = p % RING;
      const uint32_t prec_l = r_rec[ep * DW + min(lane, DW - 1)];
      const uint32_t kind = __builtin_amdgcn_readfirstlane(cmv.x);
      const uint32_t slot = __builtin_amdgcn_readfirstlane(cmv.y);
      if (kind != 1 || (slot >> 6) != c) return;
      const uint32_t woff = __builtin_amdgcn_readfirstlane(cmv.z);
      const uint32_t fl = __builtin_amdgcn_readfirstlane(cmv.w);
      const bool fresh = (fl & 1u) != 0, is_pred = (fl & 2u) != 0;
      const uint32_t ol = slot & 63, wn = d.lo + woff;
      const uint32_t prec = lane < DW ? prec_l : 0u;
      const PodView ppv = pod_view(prec);
      const uint32_t nss = __builtin_amdgcn_readlane(prec, WS_NSS);
      const uint32_t n_sel = nss & 0xffff, n_svcs = nss >> 16, nk = ppv.nk;
      const uint32_t base_nk = fresh ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)S.nk, (int)ol);
      const uint32_t base_ns = fresh ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)S.ns, (int)ol);
      // the new slot's snapshot: staged for the predicted node, else from L2
      if (fresh && lane == ol) {
        if (is_pred) {
          S.cap_c = r_hdr[ep].cap_c;
          S.cap_m = r_hdr[ep].cap_m;
          S.snp_c = r_hdr[ep].used_c;
          S.snp_m = r_hdr[ep].used_m;
          S.inv_c = r_hdr[ep].inv_c;
          S.inv_m = r_hdr[ep].inv_m;
        } else {
          S.cap_c = gld(d.cap_cpu + wn);
          S.cap_m = gld(d.cap_mem + wn);
          S.snp_c = gld(d.used_cpu + wn);
          S.snp_m = gld(d.used_mem + wn);
          S.inv_c = gld(d.inv10_cpu + wn);
          S.inv_m = gld(d.inv10_mem + wn);
        }
        S.node = woff;
        S.dl_c = S.dl_m = 0;
        S.smask = 0;
        if constexpr (ANTI) {
          const int32_t dm = gld(d.anti_domain + wn);  // (first anti priority: the re-rank's domain rows)
          S.row = dm >= 0 ? (uint32_t)dm : ~0u;
        }
      }
      uint32_t new_mask = 0;
      if (n_svcs) {
        // the pod's services (lane t < n_svcs): snapshot count on the node, max, peer
        const bool sv_lane = lane < n_svcs;
        const uint32_t my_sv =
            (uint32_t)__shfl((int)prec, (int)min(WS_IDS + nk + n_sel + (sv_lane ? lane : 0u), 63u), 64);
        int32_t cnt = 0;
        if (sv_lane) cnt = is_pred ? r_svc[ep].cnt[lane] : gld(d.svc_cnt + (size_t)my_sv * d.n_nodes + wn);
        if (sv_lane) L_cl[(size_t)slot * KSG_CL_W + KSG_CL_SC + base_ns + lane] = (uint32_t)cnt;
        new_mask = wave_or_u32(sv_lane ? (1u << (my_sv & 31)) : 0u);
      }
      if (lane == ol) {
        S.dl_c = (int64_t)((uint64_t)S.dl_c + (uint64_t)ppv.req_c);
        S.dl_m = (int64_t)((uint64_t)S.dl_m + (uint64_t)ppv.req_m);
        S.nk = base_nk + nk;
        S.ns = base_ns + n_svcs;
        S.smask |= new_mask;
      }
    };

    uint64_t t_last = 0, t_acc = 0;
    auto cstamp = [&](uint32_t k) {
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        t_acc += lane == k ? t_now - t_last : 0ULL;
        t_last = t_now;
      }
    };
    if constexpr (STAMP) t_last = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0;; ++i) {
      const uint32_t e = i % RING, par = i & 1;
      bool stopped = false;
      // pod i is checked against the slots as of commits <= i-2 (the committer
      // re-checks the slot of commit i-1 itself): it starts once commit i-2 is
      // published, a whole pod before the committer needs its drops
      for (uint32_t spin = 0;; ++spin) {
        const uint32_t ss = ld_rlx(&ctl->sel_seq), rd = ld_rlx(&r_hdr[e].ready), st = ld_rlx(&ctl->stop);
        if (i < n_pods && ss + 1 >= i && rd == i + 1) break;
        if (st) {
          stopped = true;
          break;
        }
        if (spin > 16 * KSG_SPIN_LIMIT) {
          ctl->hang = 1;
          stopped = true;
          break;
        }
        __builtin_amdgcn_s_sleep(2);  // (off the chain: leave the LDS to the committer and the x-checker)
      }
      acq_lds();
      cstamp(c == 0 ? 16 : 19);
      if (!stopped && (skew & 4u)) __builtin_amdgcn_s_sleep(8);
      if (stopped) {
        // pods [0, resolved) are decided: apply the commits this checker has not
        // (the committer runs ahead of the checkers over pods that do not commit)
        const uint32_t R = __builtin_amdgcn_readfirstlane(ctl->resolved);
        for (uint32_t q = i >= 2 ? i - 2 : 0; q < R; ++q) apply(q);
        break;
      }
      if (i >= 2) apply(i - 2);
      cstamp(c == 0 ? 17 : 20);
      const uint32_t rec = lane < DW ? r_rec[e * DW + lane] : 0u;
      const int32_t m0 = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].m0);
      uint32_t cntd = 0;
      uint64_t dmsk = 0;
      if constexpr (ANTI) {
        // the pod against this lane's slot as of commits <= i-2: a drop among the
        // nodes at their domain row's best (B; T0 drops counted for the fast
        // path), the domain-count stop, and the window's commits of the pod's
        // service the slot adds to its row's count while the pod still fits it
        bool drop = false, t0d = false, astop = false;
        uint32_t ks = 0;
        cstamp(c == 0 ? 22 : 40);  // (checker 0: the pod's record; lane 40 is dropped)
        if (!__builtin_amdgcn_readlane(rec, WS_ERR) && m0 != KSG_S32_NONE && S.node != ~0u) {
          const PodView pv = pod_view(rec);
          const uint32_t wd = S.node >> 6;
          const uint64_t nb = 1ULL << (S.node & 63);
          SlotRow R;  // the slot's lists, in registers (in flight with the slot's T0 / B / fit words)
          R.load(my_cl);
          const bool in_t0 = (r_t0[(size_t)e * P * 64 + wd] & nb) != 0;
          const bool in_b = ((FG ? pa_word(x.b_off, i, wd) : r_b[(size_t)e * P * 64 + wd]) & nb) != 0;
          const bool fsnap = pv.s >= 0 && ((FG ? pa_word(x.fit_off, i, wd) : r_fit[(size_t)e * P * 64 + wd]) & nb) != 0;
          if (in_b || fsnap) {
            const int64_t now_c = (int64_t)((uint64_t)S.snp_c + (uint64_t)S.dl_c);
            const int64_t now_m = (int64_t)((uint64_t)S.snp_m + (uint64_t)S.dl_m);
            bool nofit = false;
            if (res_on && !pv.zero_req)  // PodFitsResources (predicates.go:127-145)
              nofit = !((S.cap_c == 0 || S.cap_c - now_c >= pv.req_c) && (S.cap_m == 0 || S.cap_m - now_m >= pv.req_m));
            if (!nofit && pv.nk && S.nk)  // PodFitsPorts / NoDiskConflict vs the window's keys
              nofit |= R.key_hit(S.nk, rec, pv.nk, pv.n_ports, ports_on, disk_on);
            if (in_b) {
              drop = nofit;
              if (!drop && d.w_lr) {  // LeastRequested (priorities.go:43-76)
                // (branch-free terms: the four interleave)
                const int32_t lr_now =
                    lr_win_nb(now_c + pv.req_c, S.cap_c, S.inv_c) + lr_win_nb(now_m + pv.req_m, S.cap_m, S.inv_m);
                const int32_t lr_snap =
                    lr_win_nb(S.snp_c + pv.req_c, S.cap_c, S.inv_c) + lr_win_nb(S.snp_m + pv.req_m, S.cap_m, S.inv_m);
                drop = (lr_now >> 1) != (lr_snap >> 1);
              }
              if (!drop && spread_on && pv.s >= 0 && ((S.smask >> (pv.s & 31)) & 1u)) {
                int32_t delta = 0, snapc = 0;  // ServiceSpreading (spreading.go:72-86) under an unchanged maxCount
                R.svc(S.ns, (uint32_t)pv.s, snapc, delta);
                if (delta)
                  drop = frac10_i32(pv.smax - snapc - delta, pv.smax) !=
                         frac10_i32(pv.smax - snapc, pv.smax);
              }
              if (drop)
                atomicOr(reinterpret_cast<unsigned long long*>(L_drop + (size_t)par * P * 64 + wd), nb);
              t0d = drop && in_t0;
            }
            if (fsnap) {
              if (nofit) {
                astop = anti_counts_move(d, S.node, pv.s);
              } else if ((S.smask >> (pv.s & 31)) & 1u) {
                int32_t sc_ = 0, kn_ = 0;
                R.svc(S.ns, (uint32_t)pv.s, sc_, kn_);
                ks = (uint32_t)kn_;
              }
            }
          }
        }
        cstamp(c == 0 ? 23 : 40);  // (checker 0: the slot's check)
        cntd = __popcll(__ballot(t0d));
        // per domain row: the B drops (unlabelled nodes: row dz-1) and the window commits of the
        // pod's service on slots it still fits, summed by LDS atomics after the rows are zeroed
        // (one wave's LDS operations run in issue order)
        int32_t* const ddr = L_ddr + (c * 2 + par) * KSG_RR_MAXZ;
        int32_t* const dca = L_dca + (c * 2 + par) * KSG_RR_MAXZ;
        if (lane < dz) {
          ddr[lane] = 0;
          dca[lane] = 0;
        }
        if (drop) atomicAdd(&ddr[S.row != ~0u ? S.row : dz - 1], 1);
        if (ks != 0 && S.row != ~0u) atomicAdd(&dca[S.row], (int32_t)ks);
        const uint32_t ast = __ballot(astop) != 0;
        if (lane == 0) ctl->chk_stop[c][par] = ast;
      } else if (!__builtin_amdgcn_readlane(rec, WS_ERR) && m0 != KSG_S32_NONE) {
        const PodView pv = pod_view(rec);
        bool drop = false;
        uint32_t dpos = 0;
        if (S.node != ~0u) {
          const uint64_t* t0e = r_t0 + (size_t)e * P * 64;
          const uint32_t wd = S.node >> 6;
          const uint64_t tw = t0e[wd];
          SlotRow R;  // the slot's lists, in registers (in flight with the T0 word)
          R.load(my_cl);
          // the node's ascending position in T0 (used only if it drops)
          dpos = r_lp[(e * 64 + (wd >> 6)) * 2] + r_wp[(size_t)e * P * 64 + wd] +
                 (uint32_t)__popcll(tw & ((1ULL << (S.node & 63)) - 1ULL));
          if ((tw >> (S.node & 63)) & 1ULL) {
            // does the slot (a snapshot tie of the pod) score below M0 now?
            const int64_t now_c = (int64_t)((uint64_t)S.snp_c + (uint64_t)S.dl_c);
            const int64_t now_m = (int64_t)((uint64_t)S.snp_m + (uint64_t)S.dl_m);
            if (res_on && !pv.zero_req)  // PodFitsResources (predicates.go:127-145)
              drop = !((S.cap_c == 0 || S.cap_c - now_c >= pv.req_c) && (S.cap_m == 0 || S.cap_m - now_m >= pv.req_m));
            if (d.w_lr) {  // LeastRequested (priorities.go:43-76) can only fall as requested grows
              const int32_t lr_now = lr_win(now_c + pv.req_c, S.cap_c, S.inv_c) + lr_win(now_m + pv.req_m, S.cap_m, S.inv_m);
              const int32_t lr_snap =
                  lr_win(S.snp_c + pv.req_c, S.cap_c, S.inv_c) + lr_win(S.snp_m + pv.req_m, S.cap_m, S.inv_m);
              drop |= (lr_now >> 1) != (lr_snap >> 1);
            }
            if (!drop && pv.nk && S.nk)  // PodFitsPorts / NoDiskConflict vs the window's keys
              drop |= R.key_hit(S.nk, rec, pv.nk, pv.n_ports, ports_on, disk_on);
            if (!drop && spread_on && pv.s >= 0 && ((S.smask >> (pv.s & 31)) & 1u)) {
              // ServiceSpreading (spreading.go:72-86) under an unchanged maxCount
              int32_t delta = 0, snapc = 0;
              R.svc(S.ns, (uint32_t)pv.s, snapc, delta);
              if (delta)
                drop = frac10_i32(pv.smax - snapc - delta, pv.smax) !=
                       frac10_i32(pv.smax - snapc, pv.smax);
            }
          }
        }
        if (drop) L_dpos[par * KSG_MAX_SLOTS + my_slot] = dpos;
        dmsk = __ballot(drop);
        cntd = __popcll(dmsk);
      }
      if (lane == 0) {
        ctl->chk_cnt[c][par] = cntd;
        if constexpr (!ANTI) {
          ctl->chk_msk[c][par][0] = (uint32_t)dmsk;
          ctl->chk_msk[c][par][1] = (uint32_t)(dmsk >> 32);
        }
        st_post(&ctl->chk_seq[c], i + 1);
      }
      cstamp(c == 0 ? 18 : 21);
    }
    // write the window's deltas of this checker's slots back to HBM (the next snapshot)
    if (S.node != ~0u) {
      const uint32_t n = d.lo + S.node;
      d.used_cpu[n] = (int64_t)((uint64_t)S.snp_c + (uint64_t)S.dl_c);
      d.used_mem[n] = (int64_t)((uint64_t)S.snp_m + (uint64_t)S.dl_m);
      for (uint32_t a = 0; a < S.nk; ++a)
        __hip_atomic_fetch_or(d.keymap + (size_t)my_cl[KSG_CL_KEY + a] * d.nw + (n >> 6), 1ULL << (n & 63),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (uint32_t a = 0; a < S.ns; ++a) {
        const uint32_t sa = my_cl[KSG_CL_SV + a];
        bool first = true;
        int32_t count = 0;
        for (uint32_t b = 0; b < S.ns; ++b) {
          if (my_cl[KSG_CL_SV + b] == sa) {
            if (b < a) first = false;
            ++count;
          }
        }
        __hip_atomic_fetch_add(d.svc_total + sa, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (first) {
          const int32_t fin = (int32_t)my_cl[KSG_CL_SC + a] + count;
          d.svc_cnt[(size_t)sa * d.n_nodes + n] = fin;
          if (fin > 0)
            __hip_atomic_fetch_or(d.svc_bits + (size_t)sa * d.nw + (n >> 6), 1ULL << (n & 63), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_max(d.svc_max + sa, fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    if constexpr (STAMP) {
      if (d.dbgbuf && lane >= 16 && lane < 24) atomicAdd(d.dbgbuf + lane, (int32_t)(t_acc / 64));
    }
    drain_stores();
    if (lane == 0) st_rel(&ctl->fin[c], 1u);
    return;
  }
  // =========================================================================
  // x-checker (wave 1): pod i against the slot commit i-1 went into, as of that
  // commit (the checkers' view lags a pod), while the committer finishes commit
  // i-1 and reads pod i; also whether commit i-1 raised the pod's service's
  // maxCount or gave it its first peer. The x-checker follows the slots itself
  // (the same in-order bookkeeping as the committer's: node, list lengths and
  // delta per slot in registers), so it needs only the drawn node from the
  // committer; commit i-1's lists come from pod i-1's ring record, earlier
  // commits' from the table row.
  // =========================================================================
  if (wave == 1) {
    __builtin_amdgcn_s_setprio(2);
    // lane L < 4 evaluates one LeastRequested term: resource L & 1 (cpu, memory),
    // at the slot's requested total now (L < 2) or at the snapshot (L >= 2)
    const uint32_t rl = lane & 1;
    const int64_t* const cap_src = rl ? d.cap_mem : d.cap_cpu;
    const int64_t* const use_src = rl ? d.used_mem : d.used_cpu;
    const double* const inv_src = rl ? d.inv10_mem : d.inv10_cpu;
    uint32_t xcn0 = ~0u, xcn1 = ~0u, xsk0 = 0, xsk1 = 0, xss0 = 0, xss1 = 0, xn_slots = 0;
    int64_t xdc0 = 0, xdm0 = 0, xdc1 = 0, xdm1 = 0;
    // commit q (node) into its slot, the committer's bookkeeping replayed: the
    // slot, its list lengths before q, its delta after q, pod q's record
    bool x_in_c = false;  // the last replayed commit went into an existing slot
    auto replay = [&](uint32_t node, uint32_t prec, uint32_t& slot, uint32_t& bnk, uint32_t& bns, uint64_t& dlc,
                      uint64_t& dlm) {
      const PodView ppv = pod_view(prec);
      const uint32_t p_svcs = (uint32_t)__builtin_amdgcn_readlane(prec, WS_NSS) >> 16;
      const uint64_t hit0 = __ballot(xcn0 == node), hit1 = __ballot(xcn1 == node);
      const bool in_c = (hit0 | hit1) != 0;
      x_in_c = in_c;
      bnk = bns = 0;
      dlc = dlm = 0;
      if (in_c) {
        slot = hit0 ? (uint32_t)__builtin_ctzll(hit0) : 64u + (uint32_t)__builtin_ctzll(hit1);
        const uint32_t sl = slot & 63;
        bnk = (uint32_t)__builtin_amdgcn_readlane((int)(slot < 64 ? xsk0 : xsk1), (int)sl);
        bns = (uint32_t)__builtin_amdgcn_readlane((int)(slot < 64 ? xss0 : xss1), (int)sl);
        dlc = readlane64((uint64_t)(slot < 64 ? xdc0 : xdc1), (int)sl);
        dlm = readlane64((uint64_t)(slot < 64 ? xdm0 : xdm1), (int)sl);
      } else {
        slot = xn_slots < KSG_MAX_SLOTS ? xn_slots++ : 0u;  // (a full table stops the committer)
      }
      dlc += (uint64_t)ppv.req_c;
      dlm += (uint64_t)ppv.req_m;
      if (lane == (slot & 63)) {
        if (slot >= 64) {
          if (!in_c) xcn1 = node;
          xsk1 = bnk + ppv.nk;
          xss1 = bns + p_svcs;
          xdc1 = (int64_t)dlc;
          xdm1 = (int64_t)dlm;
        } else {
          if (!in_c) xcn0 = node;
          xsk0 = bnk + ppv.nk;
          xss0 = bns + p_svcs;
          xdc0 = (int64_t)dlc;
          xdm0 = (int64_t)dlm;
        }
      }
    };
    // the service flags later pods stop on (maxCount rises, first peer) and the
    // first peers of commit q, in commit order (one wave: L_peer, n_peer and
    // L_peerset have a single writer)
    auto flags = [&](uint32_t q, uint32_t node, uint32_t slot, uint32_t bns, uint32_t prec) {
      const uint32_t nss = __builtin_amdgcn_readlane(prec, WS_NSS), npp = __builtin_amdgcn_readlane(prec, WS_NPP);
      const uint32_t n_svcs = nss >> 16, n_sel = nss & 0xffff, pnk = (npp & 0xffff) + (npp >> 16);
      if (!n_svcs) return;
      const uint32_t wn = d.lo + node, eq = q % RING;
      const bool sv_lane = lane < n_svcs;
      const uint32_t my_sv =
          (uint32_t)__shfl((int)prec, (int)min(WS_IDS + pnk + n_sel + (sv_lane ? lane : 0u), 63u), 64);
      if constexpr (ANTI) {  // (re-rank) the service's window commits: its pod count n moved
        if (sv_lane) atomicAdd(&L_nsv[my_sv], 1u);
      }
      int32_t mx = 0, peer = 0, cnt = 0;
      if (sv_lane) {
        cnt = gld(d.svc_cnt + (size_t)my_sv * d.n_nodes + wn);
        mx = r_svc[eq].max[lane];
        peer = r_svc[eq].peer[lane];
      }
      // earlier window commits of each service on this node (table lanes KSG_CL_SV..)
      const uint32_t ent = lane - KSG_CL_SV < bns ? L_cl[(size_t)slot * KSG_CL_W + lane] : ~0u;
      uint32_t before = 0;
      for (uint32_t t = 0; t < n_svcs; ++t) {
        const uint32_t sv_t = (uint32_t)__builtin_amdgcn_readlane((int)my_sv, (int)t);
        const uint32_t b_t = (uint32_t)__popcll(__ballot(ent == sv_t));
        if (lane == t) before = b_t;
      }
      bool changed = sv_lane && aff_on && peer == -1 && !((L_peerset[my_sv >> 5] >> (my_sv & 31)) & 1u);
      uint64_t pm = __ballot(sv_lane && peer == -1);
      if (pm) {  // first commit of a service with no peer yet: its first peer
        uint32_t n_peer = __builtin_amdgcn_readfirstlane(ctl->n_peer);
        while (pm) {
          const uint32_t b = __builtin_ctzll(pm);
          pm &= pm - 1;
          const uint32_t fsv = (uint32_t)__builtin_amdgcn_readlane((int)my_sv, (int)b);
          if (!((L_peerset[fsv >> 5] >> (fsv & 31)) & 1u)) {
            if (lane == 0) {
              L_peerset[fsv >> 5] |= 1u << (fsv & 31);
              L_peer[2 * n_peer] = fsv;
              L_peer[2 * n_peer + 1] = wn;
            }
            ++n_peer;
            lds_fence();
          }
        }
        if (lane == 0) ctl->n_peer = n_peer;
      }
      if (sv_lane && spread_on && cnt + (int32_t)before + 1 > mx) changed = true;  // maxCount rises
      if (changed) atomicOr(&L_flag[my_sv >> 5], 1u << (my_sv & 31));
    };
    uint64_t x_last = 0, x_acc = 0;  // KSG_DEBUG & 8: lanes 28..30 wait, check, loads
    if constexpr (STAMP) x_last = __builtin_amdgcn_s_memtime();
    uint32_t i = 0;
    for (; i < n_pods; ++i) {
      const uint32_t e = i % RING, par = i & 1;
      bool stopped = false;
      for (uint32_t spin = 0;; ++spin) {  // pod i staged (long before pod i-1's node is drawn), or the end
        const uint32_t rd = ld_u(&r_hdr[e].ready), st = ld_u(&ctl->stop);
        if (rd == i + 1) break;
        if (st) {
          stopped = true;
          break;
        }
        if (spin > 16 * KSG_SPIN_LIMIT) {
          ctl->hang = 1;
          stopped = true;
          break;
        }
      }
      acq_lds();
      if (stopped) break;
      // pods i's and i-1's records ahead of the node
      const uint32_t rec = lane < DW ? r_rec[e * DW + lane] : 0u;
      const int32_t m0 = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].m0);
      const uint32_t prec = (i && lane < DW) ? r_rec[((i - 1) % RING) * DW + lane] : 0u;
      const PodView pv = pod_view(rec);
      const int32_t s = pv.s;
      for (uint32_t spin = 0;; ++spin) {  // pod i-1's node drawn, or the end
        const uint32_t xn = ld_u(&ctl->xn_seq), st = ld_u(&ctl->stop);
        if (xn >= i) break;
        if (st) {
          stopped = true;
          break;
        }
        if (spin > 16 * KSG_SPIN_LIMIT) {
          ctl->hang = 1;
          stopped = true;
          break;
        }
      }
      acq_lds();
      if (stopped) break;
      if (skew & 2u) __builtin_amdgcn_s_sleep(8);
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        x_acc += lane == 28 ? t_now - x_last : 0ULL;
        x_last = t_now;
        if (i) x_acc += lane == 31 ? (uint64_t)(uint32_t)((uint32_t)t_now - ctl->t_n) : 0ULL;
      }
      uint32_t res = 0;
      const uint32_t xnode = i ? __builtin_amdgcn_readfirstlane(L_cm[i - 1].xn) : ~0u;
      // the node's snapshot first (in flight over the bookkeeping below)
      const bool do_check = xnode != ~0u && !__builtin_amdgcn_readlane(rec, WS_ERR) && m0 != KSG_S32_NONE;
      const uint32_t xw = d.lo + (do_check ? xnode : 0u);
      int64_t capv = 0, usev = 0;
      double invv = 0.0;
      int32_t xcv = 0, xdm = -1;
      if (do_check) {
        capv = gld(cap_src + xw);
        usev = gld(use_src + xw);
        invv = gld(inv_src + xw);
        xcv = gld(d.svc_cnt + (size_t)(s >= 0 ? s : 0) * d.n_nodes + xw);
        if constexpr (ANTI) xdm = gld(d.anti_domain + xw);
      }
      uint32_t xst = 0, xrow = ~0u;  // (re-rank) domain-count stop; row of x and its count correction
      int32_t xcorr = 0;
      uint32_t xrw = 0;              // (re-rank) x's domain row (dz-1: unlabelled)
      // commit i-1 into its slot (the committer's bookkeeping, replayed)
      uint32_t xslot = 0, bnk = 0, bns = 0;
      uint64_t dlc = 0, dlm = 0;
      if (xnode != ~0u) replay(xnode, prec, xslot, bnk, bns, dlc, dlm);
      if (do_check) {
        // pod i-1's record: its keys and service ids follow the earlier commits' in the slot's lists
        const uint32_t pnpp = __builtin_amdgcn_readlane(prec, WS_NPP), pnss = __builtin_amdgcn_readlane(prec, WS_NSS);
        const uint32_t pnk = (pnpp & 0xffff) + (pnpp >> 16), pnsel = pnss & 0xffff, pns = pnss >> 16;
        const uint32_t xnk = bnk + pnk, xns = bns + pns;
        // lane t < 8: key t of the slot; lane 8 + u (u < 12): its service u
        const uint32_t kt = lane - KSG_CL_KEY, ut = lane - KSG_CL_SV;
        const bool from_row = (kt < KSG_SLOT_KEYS && kt < bnk) || (ut < KSG_SLOT_SVCS && ut < bns);
        const uint32_t src = kt < KSG_SLOT_KEYS ? WS_IDS + (kt - bnk) : WS_IDS + pnk + pnsel + (ut - bns);
        const uint32_t from_rec = (uint32_t)__shfl((int)prec, (int)min(src, 63u), 64);
        const uint32_t rowv = from_row ? L_cl[(size_t)xslot * KSG_CL_W + lane] : 0u;
        const uint32_t xcl = from_row ? rowv : from_rec;
        const uint32_t nk = pv.nk;
        const bool s_ent = s >= 0 && ut < xns && xcl == (uint32_t)s;
        const uint32_t x_cnt_s = (uint32_t)__popcll(__ballot(s_ent));
        const bool prev_has = __ballot(s_ent && ut >= bns) != 0;  // pod i-1 is a pod of service s
        if constexpr (STAMP) {
          const uint64_t t_now = __builtin_amdgcn_s_memtime();
          x_acc += lane == 30 ? t_now - x_last : 0ULL;
          x_last = t_now;
        }
        const int64_t reqv = rl ? pv.req_m : pv.req_c;
        const int64_t nowv = (int64_t)((uint64_t)usev + (rl ? dlm : dlc));  // requested total now
        bool xd = false, flag_x = false;
        if (res_on && !pv.zero_req)  // PodFitsResources: lanes 0 and 1
          xd = (__ballot(lane < 2 && !(capv == 0 || capv - nowv >= reqv)) & 3ULL) != 0;
        if (d.w_lr) {  // LeastRequested: one term per lane
          const int32_t lrv = lr_win((lane < 2 ? nowv : usev) + reqv, capv, invv);
          const int32_t lr_now = __builtin_amdgcn_readlane(lrv, 0) + __builtin_amdgcn_readlane(lrv, 1);
          const int32_t lr_snap = __builtin_amdgcn_readlane(lrv, 2) + __builtin_amdgcn_readlane(lrv, 3);
          xd |= (lr_now >> 1) != (lr_snap >> 1);
        }
        if (x_cnt_s) {
          const int32_t x_snapc = __builtin_amdgcn_readfirstlane(xcv);
          if (spread_on) {  // ServiceSpreading under an unchanged maxCount: lane 0 now, lane 1 the snapshot
            const int32_t fr = (int32_t)frac10_i32(pv.smax - x_snapc - (lane == 0 ? (int32_t)x_cnt_s : 0),
                                                   pv.smax);
            xd |= __builtin_amdgcn_readlane(fr, 0) != __builtin_amdgcn_readlane(fr, 1);
          }
          if (prev_has) {  // commit i-1, a pod of service s: maxCount rises / first peer
            flag_x = spread_on && x_snapc + (int32_t)x_cnt_s > pv.smax;
            if (aff_on && (int32_t)__builtin_amdgcn_readfirstlane(r_svc[e].peer[0]) == -1 &&
                !((L_peerset[s >> 5] >> (s & 31)) & 1u))
              flag_x = true;
          }
        }
        if (nk && xnk) {  // PodFitsPorts / NoDiskConflict: lane t holds key t
          bool hit = false;
          for (uint32_t b = 0; b < nk; ++b) {
            const bool on = b < pv.n_ports ? ports_on : disk_on;
            hit |= on && kt < xnk && xcl == (uint32_t)__builtin_amdgcn_readlane((int)rec, (int)(WS_IDS + b));
          }
          xd |= __ballot(hit) != 0;
        }
        if constexpr (ANTI) {
          xrw = xdm >= 0 ? (uint32_t)xdm : dz - 1;
          // x as of commit i-1 and as of i-2 (the checkers' view of it): does the
          // pod still fit it (PodFitsResources, host ports, PDs), and its
          // service's window commits there; the domain count of x's row moves by
          // the difference, or the window ends if the pod no longer fits a
          // labelled x that held pods of its service at the snapshot
          const uint64_t xfw = FG ? pa_word(x.fit_off, i, xnode >> 6) : r_fit[(size_t)e * P * 64 + (xnode >> 6)];
          if (s >= 0 && ((xfw >> (xnode & 63)) & 1ULL)) {
            const PodView qv = pod_view(prec);
            const int64_t befv = (int64_t)((uint64_t)nowv - (uint64_t)(rl ? qv.req_m : qv.req_c));
            bool fa = true, fb = true;
            if (res_on && !pv.zero_req) {
              fa = (__ballot(lane < 2 && !(capv == 0 || capv - nowv >= reqv)) & 3ULL) == 0;
              fb = (__ballot(lane < 2 && !(capv == 0 || capv - befv >= reqv)) & 3ULL) == 0;
            }
            if (nk && xnk) {
              bool ha = false, hb = false;
              for (uint32_t b = 0; b < nk; ++b) {
                const bool on = b < pv.n_ports ? ports_on : disk_on;
                const bool eq = on && xcl == (uint32_t)__builtin_amdgcn_readlane((int)rec, (int)(WS_IDS + b));
                ha |= eq && kt < xnk;
                hb |= eq && kt < bnk;
              }
              fa = fa && __ballot(ha) == 0;
              fb = fb && __ballot(hb) == 0;
            }
            const uint32_t kb = (uint32_t)__popcll(__ballot(s_ent && ut < bns));
            if (!fa && xdm >= 0 && xcv > 0) xst = 1;
            if (xdm >= 0) {
              xrow = (uint32_t)xdm;
              xcorr = (fa ? (int32_t)x_cnt_s : 0) - ((x_in_c && fb) ? (int32_t)kb : 0);
            }
          }
        }
        res = (xd ? 1u : 0u) | (flag_x ? 2u : 0u) | (xst ? 4u : 0u);
      }
      if (lane == 0) {
        if constexpr (ANTI) {
          ctl->xdz[par] = xrow;
          ctl->xdc[par] = xcorr;
          ctl->xrw[par] = xrw;
          ctl->xnsv[par] = s >= 0 ? L_nsv[s] : 0u;
        }
        ctl->xres[par] = res;
        if constexpr (STAMP) ctl->t_x = (uint32_t)__builtin_amdgcn_s_memtime();
        st_post(&ctl->xseq, i + 1);
      }
      // off the chain now: commit i-1's service flags and first peers (the
      // committer reads them for pod i+1 once this iteration is done)
      if (xnode != ~0u) flags(i - 1, xnode, xslot, bns, prec);
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        x_acc += lane == 29 ? t_now - x_last : 0ULL;
        x_last = t_now;
      }
    }
    // the committer is done: the commits from i-1 on were not replayed yet; their
    // first peers still count (the window's end writes them)
    for (uint32_t spin = 0; !ld_acq(&ctl->stop); ++spin) {
      if (spin > 16 * KSG_SPIN_LIMIT) {
        ctl->hang = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const uint32_t R = __builtin_amdgcn_readfirstlane(ctl->resolved);
    for (uint32_t q = i >= 1 ? i - 1 : 0; q < R; ++q) {
      if (__builtin_amdgcn_readfirstlane(L_cm[q].kind) != 1) continue;
      const uint32_t node = __builtin_amdgcn_readfirstlane(L_cm[q].node);
      const uint32_t prec = lane < DW ? r_rec[(q % RING) * DW + lane] : 0u;
      uint32_t slot, bnk, bns;
      uint64_t dlc, dlm;
      replay(node, prec, slot, bnk, bns, dlc, dlm);
      flags(q, node, slot, bns, prec);
    }
    if constexpr (STAMP) {
      if (d.dbgbuf && lane >= 28 && lane < 32) atomicAdd(d.dbgbuf + lane, (int32_t)(x_acc / 64));
    }
    if (lane == 0) st_rel(&ctl->fin_x, 1u);
    return;
  }
  if (wave != 0) return;

  // =========================================================================
  // committer (wave 0)
  // =========================================================================
  __builtin_amdgcn_s_setprio(3);
  uint32_t resolved = n_pods, reason = 0, n_slots = 0, n_draws = 0;
  uint32_t cn0 = ~0u, cn1 = ~0u;  // nodes of slots lane and 64 + lane
  uint32_t sk0 = 0, sk1 = 0;      // their key counts
  uint32_t ss0 = 0, ss1 = 0;      // their service entry counts
  int64_t dc0 = 0, dm0 = 0, dc1 = 0, dm1 = 0;  // their window deltas (current through the last commit)
  uint32_t xnode = 0;                    // node of the last commit (pod i-1)
  uint32_t xslot = 0;                    // and its slot
  bool have_x = false;
  uint32_t prev_sv = ~0u;                // (ServiceAntiAffinity) services of commit i-1, lane t < count
  uint64_t t_last = 0, t_acc = 0;
#define KSG_STAMP2(k)                                        \
  if constexpr (STAMP) {                                     \
    const uint64_t t_now = __builtin_amdgcn_s_memtime();     \
    t_acc += lane == (uint32_t)(k) ? t_now - t_last : 0ULL;  \
    t_last = t_now;                                          \
  }
#define KSG_COUNT2(k, v)                                   \
  if constexpr (STAMP) {                                   \
    t_acc += lane == (uint32_t)(k) ? (uint64_t)(v) : 0ULL; \
  }
  if constexpr (STAMP) t_last = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < n_pods; ++i) {
    const uint32_t e = i % RING, par = i & 1;
    // (relaxed polls, then one LDS-only acquire: an acquire load also waits for
    // the previous pod's stores in flight)
    if (ld_u(&r_hdr[e].ready) != i + 1) {
      __builtin_amdgcn_s_setprio(0);  // a producer shares this SIMD: do not starve it
      bool hung = false;
      for (uint32_t spin = 0; ld_u(&r_hdr[e].ready) != i + 1; ++spin)
        if (spin > 16 * KSG_SPIN_LIMIT || ld_u(&ctl->hang)) {
          hung = true;
          break;
        }
      __builtin_amdgcn_s_setprio(3);
      if (hung) {
        resolved = i;
        reason = KSG_STOP_HANG;
        break;
      }
    }
    acq_lds();
    if (skew & 1u) __builtin_amdgcn_s_sleep(8);
    if constexpr (STAMP) {  // ring wait of the window's first 4 pods (lane 10) vs the rest (lane 11)
      const uint64_t t_now = __builtin_amdgcn_s_memtime();
      t_acc += lane == (i < 4 ? 10u : 11u) ? t_now - t_last : 0ULL;
    }
    KSG_STAMP2(0)
    // ---- the staged pod: record, header, T0 words, r mod (k0 - d) (one round of LDS reads)
    const uint32_t rec = lane < DW ? r_rec[e * DW + lane] : 0u;
    const uint32_t rmod = r_mod[e * 64 + lane];
    const uint64_t* t0e = r_t0 + (size_t)e * P * 64;
    uint64_t t0w[P];
    uint32_t lp_ex = 0, lp_in = 0, xlp = 0, xwp = 0;
    uint64_t t0x = 0;
    if constexpr (ANTI) {
#pragma unroll
      for (int q = 0; q < P; ++q) t0w[q] = t0e[lane * P + q];
    } else {
      // the sparse select's row prefixes (lane q < P: row q), and where commit
      // i-1's node sits in T0
      if (lane < P) {
        lp_ex = r_lp[(e * 64 + lane) * 2];
        lp_in = r_lp[(e * 64 + lane) * 2 + 1];
      }
      if (have_x) {
        const uint32_t xw = xnode >> 6;
        t0x = t0e[xw];
        xwp = r_wp[(size_t)e * P * 64 + xw];
        xlp = r_lp[(e * 64 + (xw >> 6)) * 2];
      }
    }
    const int32_t m0 = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].m0);
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(r_hdr[e].k0);
    const int32_t pred = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].pred);
    if (__builtin_amdgcn_readlane(rec, WS_ERR) || m0 == KSG_S32_NONE) {
      // ServiceAffinity peer error / nothing fit at the snapshot (commits only
      // remove fits): no draw, no commit
      if (lane == 0) {
        L_cm[i].kind = 0;
        L_cm[i].out = __builtin_amdgcn_readlane(rec, WS_ERR) ? KSG_OUT_ERROR : KSG_OUT_NOFIT;
        L_cm[i].xn = ~0u;
        st_post(&ctl->xn_seq, i + 1);
        st_post(&ctl->sel_seq, i + 1);
      }
      have_x = false;  // pod i+1's checkers see every commit up to i-1
      prev_sv = ~0u;
      continue;
    }
    const PodView pv = pod_view(rec);
    const int32_t s = pv.s;
    const uint32_t nss = __builtin_amdgcn_readlane(rec, WS_NSS);
    const uint32_t n_sel = nss & 0xffff, n_svcs = nss >> 16, nk = pv.nk;
    if (__builtin_amdgcn_readlane(rec, WS_NINL) > KSG_WIN_INLINE || nk > KSG_SLOT_KEYS || n_svcs > KSG_SLOT_SVCS) {
      resolved = i;  // lists longer than the record / a slot: the exact per-pod kernel takes it
      reason = i == 0 ? KSG_STOP_OVERSIZE : KSG_STOP_SLOT;
      break;
    }
    KSG_STAMP2(1)
    // ---- the checkers' drops (slots as of commits <= i-2) and the x-checker's
    // verdict on the slot of commit i-1
    bool hung = false;
    for (uint32_t spin = 0;; ++spin) {
      const uint32_t xs = ld_rlx(&ctl->xseq), hg = ld_rlx(&ctl->hang);
      uint32_t cs = ld_rlx(&ctl->chk_seq[0]);
#pragma unroll
      for (int c = 1; c < KSG_RES_NCHK; ++c) cs = min(cs, ld_rlx(&ctl->chk_seq[c]));
      if (xs >= i + 1 && cs >= i + 1) break;
      if (spin > 16 * KSG_SPIN_LIMIT || hg) {
        hung = true;
        break;
      }
    }
    acq_lds();
    if (hung) {
      resolved = i;
      reason = KSG_STOP_HANG;
      break;
    }
    KSG_STAMP2(2)
    if constexpr (STAMP) t_acc += lane == 6 ? (uint64_t)(uint32_t)((uint32_t)t_last - ctl->t_x) : 0ULL;
    // one round of LDS reads: drop counts, verdict, the service flag word, the drop bitmap
    uint64_t* dw = L_drop + (size_t)par * P * 64;
    const uint32_t cc0 = ctl->chk_cnt[0][par], cc1 = ctl->chk_cnt[1][par];
    const uint32_t xr = ctl->xres[par];
    const uint32_t fw = s >= 0 ? L_flag[s >> 5] : 0u;
    uint64_t dww[P];
    uint64_t msk0 = 0, msk1 = 0;
    uint32_t dp0 = 0, dp1 = 0;
    if constexpr (ANTI) {
#pragma unroll
      for (int q = 0; q < P; ++q) dww[q] = dw[lane * P + q];
    } else {  // the checkers' dropping slots and the drops' positions in T0
      msk0 = ((uint64_t)__builtin_amdgcn_readfirstlane(ctl->chk_msk[0][par][1]) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane(ctl->chk_msk[0][par][0]);
      msk1 = ((uint64_t)__builtin_amdgcn_readfirstlane(ctl->chk_msk[1][par][1]) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane(ctl->chk_msk[1][par][0]);
      dp0 = L_dpos[par * KSG_MAX_SLOTS + lane];
      dp1 = L_dpos[par * KSG_MAX_SLOTS + 64 + lane];
    }
    const uint32_t xres = __builtin_amdgcn_readfirstlane(xr);
    if (s >= 0 && (spread_on || aff_on) && ((xres & 2u) || ((__builtin_amdgcn_readfirstlane(fw) >> (s & 31)) & 1u))) {
      resolved = i;  // a service scalar this pod reads changed in the window
      reason = KSG_STOP_SERVICE;
      break;
    }
    uint32_t mv_n = 0;  // (ServiceAntiAffinity) window commits of the pod's service before it
    if constexpr (ANTI) {
      if ((xres & 4u) || __builtin_amdgcn_readfirstlane(ctl->chk_stop[0][par] | ctl->chk_stop[1][par])) {
        resolved = i;  // the pod's domain counts moved: a fitted node holding its service's pods left its filter
        reason = KSG_STOP_SERVICE;
        break;
      }
      if (s >= 0)
        mv_n = __builtin_amdgcn_readfirstlane(ctl->xnsv[par]) + (__ballot(prev_sv == (uint32_t)s) != 0 ? 1u : 0u);
    }
    const bool moved = mv_n != 0;
    uint32_t dropped = __builtin_amdgcn_readfirstlane(cc0) + __builtin_amdgcn_readfirstlane(cc1);
    bool x_drop = false;
    if constexpr (!ANTI) {
      // x counts as a new drop iff it is a snapshot tie whose slot the checkers
      // kept (a new slot: they have not seen it)
      const bool x_kept = !(((xslot < 64 ? msk0 : msk1) >> (xslot & 63)) & 1ULL);
      x_drop = have_x && (xres & 1u) && ((t0x >> (xnode & 63)) & 1ULL) && x_kept;
    } else if (have_x && (xres & 1u)) {  // x counts as a new drop iff it was a snapshot tie the checkers kept
      const uint32_t xwd = xnode >> 6, xo = xwd / P, xq = xwd % P;
      uint64_t t0x = 0, dwx = 0;
#pragma unroll
      for (int q = 0; q < P; ++q)
        if ((uint32_t)q == xq) {
          t0x = readlane64(t0w[q], (int)xo);
          dwx = readlane64(dww[q], (int)xo);
        }
      const uint64_t xb = 1ULL << (xnode & 63);
      x_drop = (t0x & xb) && !(dwx & xb);
    }
    dropped += x_drop ? 1u : 0u;
    if (!moved && dropped >= k0) {
      resolved = i;  // every snapshot tie got worse: needs a fresh snapshot
      reason = KSG_STOP_EXHAUSTED;
      break;
    }
    // ---- selection: k live ties, ix-th in descending rank = (k-1-ix)-th ascending
    const uint32_t k = k0 - dropped;
    uint32_t woff;
    if (moved) {
      // ---- ServiceAntiAffinity re-rank (calculateAntiAffinityPriority,
      // spreading.go:104-168; the LDS-slot resolver has the same step): the
      // service's pod count and the pod's domain counts moved, so every domain
      // row's term is recomputed and the tie set is the live best-per-row nodes
      // of the rows whose best + term is the maximum
      KSG_COUNT2(9, 64)
      const uint64_t t_rr = STAMP ? __builtin_amdgcn_s_memtime() : 0ULL;
      const int32_t nn = (int32_t)__builtin_amdgcn_readlane(rec, WS_STOT) + (int32_t)mv_n;
      const uint32_t xz = __builtin_amdgcn_readfirstlane(ctl->xdz[par]);
      const int32_t xc = (int32_t)__builtin_amdgcn_readfirstlane(ctl->xdc[par]);
      int32_t cz = 0, mbz = KSG_S32_NONE;
      if (lane < dz) {
        cz = r_dc[e * KSG_RR_MAXZ + lane] + L_dca[par * KSG_RR_MAXZ + lane] + L_dca[(2 + par) * KSG_RR_MAXZ + lane] +
             (lane == xz ? xc : 0);
        mbz = r_mb[e * KSG_RR_MAXZ + lane];
      }
      // unlabelled nodes (row dz-1) score 0 (spreading.go:164-166)
      const int64_t aa = lane + 1 < dz ? (int64_t)d.w_anti[0] * frac10_f32((int64_t)nn - cz, nn) : 0;
      uint64_t lw[P];
#pragma unroll
      for (int q = 0; q < P; ++q)
        lw[q] = (FG ? pa_word(x.b_off, i, lane * P + q) : r_b[(size_t)e * P * 64 + lane * P + q]) & ~dww[q];
      // live B nodes per row: the producer's count minus the checkers' drops
      // minus x if it is a B node the checkers kept and the x-checker dropped
      bool x_new = false;
      if (have_x && (xres & 1u)) {
        const uint32_t xwd = xnode >> 6, xo = xwd / P, xq = xwd % P;
        uint64_t lx = 0;
#pragma unroll
        for (int q = 0; q < P; ++q)
          if ((uint32_t)q == xq) lx = readlane64(lw[q], (int)xo);
        x_new = (lx >> (xnode & 63)) & 1ULL;
        if (lane == xo) {
#pragma unroll
          for (int q = 0; q < P; ++q)
            if ((uint32_t)q == xq) lw[q] &= ~(1ULL << (xnode & 63));
        }
      }
      const uint32_t xrwv = __builtin_amdgcn_readfirstlane(ctl->xrw[par]);
      uint32_t livez = 0;
      if (lane < dz)
        livez = (uint32_t)(r_kz[e * KSG_RR_MAXZ + lane] - L_ddr[par * KSG_RR_MAXZ + lane] -
                           L_ddr[(2 + par) * KSG_RR_MAXZ + lane] - ((x_new && lane == xrwv) ? 1 : 0));
      const int32_t val = (lane < dz && mbz != KSG_S32_NONE) ? (int32_t)((int64_t)mbz + aa) : KSG_S32_NONE;
      const int32_t mlive = wave_total_max(livez > 0 ? val : KSG_S32_NONE);
      if (mlive == KSG_S32_NONE || __ballot(lane < dz && livez == 0 && mbz != KSG_S32_NONE && val > mlive)) {
        resolved = i;  // the best row's best nodes all got worse: needs a fresh snapshot
        reason = KSG_STOP_EXHAUSTED;
        break;
      }
      const bool zs = lane < dz && livez > 0 && val == mlive;
      const uint64_t zsel = __ballot(zs);
      const uint32_t k2 = wave_total_add(zs ? livez : 0u);
      const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r_hdr[e].r >> 32)) << 32) |
                         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r_hdr[e].r);
      const uint32_t ix = umod64_32(r, k2);
      uint64_t sw[P];
      uint32_t cl = 0;
      if constexpr (ZG) {  // the selected rows' nodes from HBM: one round of loads per row, then live B
#pragma unroll
        for (int q = 0; q < P; ++q) sw[q] = 0;
        for (uint64_t zz = zsel; zz; zz &= zz - 1) {
          const uint32_t zr = (uint32_t)__builtin_ctzll(zz);
          uint64_t zw[P];
#pragma unroll
          for (int q = 0; q < P; ++q) zw[q] = zm_word(zr, lane * P + q);
#pragma unroll
          for (int q = 0; q < P; ++q) sw[q] |= zw[q];
        }
#pragma unroll
        for (int q = 0; q < P; ++q) {
          sw[q] &= lw[q];
          cl += __popcll(sw[q]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < P; ++q) {
          uint64_t m = 0;
          for (uint64_t zz = zsel; zz; zz &= zz - 1) m |= L_zm[(size_t)__builtin_ctzll(zz) * P * 64 + lane * P + q];
          sw[q] = lw[q] & m;
          cl += __popcll(sw[q]);
        }
      }
      const uint32_t incl = dpp_scan_add(cl);
      woff = select_in_lanes<P>(sw, cl, incl, k2 - 1 - ix, lane);
      KSG_COUNT2(12, __builtin_amdgcn_s_memtime() - t_rr)  // (the re-rank's cycles)
    } else if (dropped == 0) {
      woff = (uint32_t)pred;  // staged by the producer
    } else if constexpr (!ANTI) {
      // ---- sparse select: the live ties are T0 minus the drops, whose
      // ascending T0 positions are known (the checkers' and x's). The (k-1-ix)-th
      // live tie ascending is T0's tp-th, tp the least fixed point of
      // tp = t + #(drops at positions <= tp); then its lane (lane prefixes), its
      // word (the owner lane's word prefixes) and its bit (mbcnt rank)
      KSG_COUNT2(7, 64)
      uint32_t ix;
      if (dropped < 64) {
        ix = (uint32_t)__builtin_amdgcn_readlane((int)rmod, (int)dropped);
      } else {
        const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r_hdr[e].r >> 32)) << 32) |
                           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r_hdr[e].r);
        ix = umod64_32(r, k);
      }
      const uint32_t t = k - 1 - ix;
      const uint32_t d0 = ((msk0 >> lane) & 1ULL) ? dp0 : ~0u;
      const uint32_t d1 = ((msk1 >> lane) & 1ULL) ? dp1 : ~0u;
      const uint32_t xpos = x_drop ? xlp + xwp + (uint32_t)__popcll(t0x & ((1ULL << (xnode & 63)) - 1ULL)) : ~0u;
      uint32_t tp = t;
      for (;;) {
        const uint32_t cnt = (uint32_t)__popcll(__ballot(d0 <= tp)) + (uint32_t)__popcll(__ballot(d1 <= tp)) +
                             (xpos <= tp ? 1u : 0u);
        if (t + cnt == tp) break;
        tp = t + cnt;
      }
      const uint32_t qs = (uint32_t)__builtin_ctzll(__ballot(lane < P && lp_ex <= tp && tp < lp_in));
      const uint32_t loc = tp - (uint32_t)__builtin_amdgcn_readlane((int)lp_ex, (int)qs);
      const uint64_t w = t0e[qs * 64 + lane];
      const uint32_t wpq = r_wp[(size_t)e * P * 64 + qs * 64 + lane];
      const uint32_t ls = (uint32_t)__builtin_ctzll(__ballot(wpq <= loc && loc < wpq + (uint32_t)__popcll(w)));
      const uint64_t ws = readlane64(w, (int)ls);
      const uint32_t lw = loc - (uint32_t)__builtin_amdgcn_readlane((int)wpq, (int)ls);
      const uint32_t rank =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(ws >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ws, 0u));
      const uint32_t bsel = (uint32_t)__builtin_ctzll(__ballot(((ws >> lane) & 1ULL) && rank == lw));
      woff = (qs * 64 + ls) * 64 + bsel;
    } else {
      KSG_COUNT2(7, 64)
      uint32_t ix;
      if (dropped < 64) {
        ix = (uint32_t)__builtin_amdgcn_readlane((int)rmod, (int)dropped);
      } else {
        const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r_hdr[e].r >> 32)) << 32) |
                           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r_hdr[e].r);
        ix = umod64_32(r, k);
      }
      uint64_t live[P];
#pragma unroll
      for (int q = 0; q < P; ++q) {
        live[q] = t0w[q] & ~dww[q];
        if (dww[q]) dw[lane * P + q] = 0;  // (cleared for the pod two ahead)
        if (x_drop && lane * P + q == (xnode >> 6)) live[q] &= ~(1ULL << (xnode & 63));
      }
      uint32_t cl = 0;
#pragma unroll
      for (int q = 0; q < P; ++q) cl += __popcll(live[q]);
      const uint32_t incl = dpp_scan_add(cl);
      woff = select_in_lanes<P>(live, cl, incl, k - 1 - ix, lane);
    }
    if constexpr (ANTI) {  // (drops outside T0 are scattered too) clear them for the pod two ahead
#pragma unroll
      for (int q = 0; q < P; ++q)
        if (dww[q]) dw[lane * P + q] = 0;
    }
    if (lane == 0) {  // the x-checker loads the node's snapshot meanwhile
      L_cm[i].xn = woff;
      if constexpr (STAMP) ctl->t_n = (uint32_t)__builtin_amdgcn_s_memtime();
      st_post(&ctl->xn_seq, i + 1);
    }
    KSG_STAMP2(3)
    // ---- AssumePod's slot
    const uint64_t hit0 = __ballot(cn0 == woff);
    const uint64_t hit1 = __ballot(cn1 == woff);
    const bool in_c = (hit0 | hit1) != 0;
    uint32_t slot, base_nk = 0, base_ns = 0;
    int64_t base_dc = 0, base_dm = 0;
    if (in_c) {
      slot = hit0 ? (uint32_t)__builtin_ctzll(hit0) : 64u + (uint32_t)__builtin_ctzll(hit1);
      const uint32_t sl = slot & 63;
      base_nk = (uint32_t)__builtin_amdgcn_readlane((int)(slot < 64 ? sk0 : sk1), (int)sl);
      base_ns = (uint32_t)__builtin_amdgcn_readlane((int)(slot < 64 ? ss0 : ss1), (int)sl);
      if (base_nk + nk > KSG_SLOT_KEYS || base_ns + n_svcs > KSG_SLOT_SVCS) {
        resolved = i;  // this pod is redone (with the same draw) in the next window
        reason = KSG_STOP_SLOT;
        break;
      }
      base_dc = (int64_t)readlane64((uint64_t)(slot < 64 ? dc0 : dc1), (int)sl);
      base_dm = (int64_t)readlane64((uint64_t)(slot < 64 ? dm0 : dm1), (int)sl);
    } else {
      if (n_slots == KSG_MAX_SLOTS) {
        resolved = i;
        reason = KSG_STOP_SLOT;
        break;
      }
      slot = n_slots++;
    }
    const int64_t new_dc = (int64_t)((uint64_t)base_dc + (uint64_t)pv.req_c);
    const int64_t new_dm = (int64_t)((uint64_t)base_dm + (uint64_t)pv.req_m);
    KSG_STAMP2(4)
    // the slot's table row: the pod's keys and service ids (record lane L holds
    // dword L, so each list entry is stored by the lane that holds it)
    {
      uint32_t* row = L_cl + (size_t)slot * KSG_CL_W;
      const uint32_t kt = lane - WS_IDS, st = lane - (WS_IDS + nk + n_sel);
      if (kt < nk) row[KSG_CL_KEY + base_nk + kt] = rec;
      if (st < n_svcs) row[KSG_CL_SV + base_ns + st] = rec;
    }
    if (lane == 0) {
      // (the record's 16 bytes only: the drawn node next to it is the x-checker's)
      *reinterpret_cast<uint4*>(&L_cm[i]) =
          uint4{1u, slot, woff, (in_c ? 0u : 1u) | ((int32_t)woff == pred ? 2u : 0u) | (n_svcs << 8)};
      L_cm[i].out = (int32_t)(d.lo + woff);
      st_post(&ctl->sel_seq, i + 1);  // the checkers and the x-checker move on
    }
    if ((int32_t)woff != pred) KSG_COUNT2(8, 64)
    if (lane == (slot & 63)) {  // this wave's counts and deltas of the slot
      if (slot >= 64) {
        if (!in_c) cn1 = woff;
        dc1 = new_dc;
        dm1 = new_dm;
        sk1 = base_nk + nk;
        ss1 = base_ns + n_svcs;
      } else {
        if (!in_c) cn0 = woff;
        dc0 = new_dc;
        dm0 = new_dm;
        sk0 = base_nk + nk;
        ss0 = base_ns + n_svcs;
      }
    }
    have_x = true;
    xnode = woff;
    xslot = slot;
    if constexpr (ANTI) {
      const uint32_t sv_t = (uint32_t)__shfl((int)rec, (int)min(WS_IDS + nk + n_sel + (lane < n_svcs ? lane : 0u), 63u), 64);
      prev_sv = lane < n_svcs ? sv_t : ~0u;
    }
    ++n_draws;
    KSG_STAMP2(5)
  }
  if (lane == 0) {
    ctl->resolved = resolved;
    st_rel(&ctl->stop, 1u);
  }
  // the checkers apply the last commits and write their slots back; the
  // x-checker records the last first peers
  bool drained = false;
  for (uint32_t spin = 0; spin <= 16 * KSG_SPIN_LIMIT; ++spin) {
    bool done = ld_acq(&ctl->fin_x) != 0;
#pragma unroll
    for (int c = 0; c < KSG_RES_NCHK; ++c) done = done && ld_acq(&ctl->fin[c]) != 0;
    if (done) {
      drained = true;
      break;
    }
  }
  if (!drained || ld_acq(&ctl->hang)) reason = KSG_STOP_HANG;
  if constexpr (ANTI) {  // the producers staged this window's domain counts and row bests: reset them for the next
    for (uint32_t t = lane; t < x.dcnt_n; t += 64) x.dcnt[t] = 0;
    for (uint32_t t = lane; t < wcap * dz; t += 64) x.dmb[t] = KSG_S32_NONE;
    for (uint32_t t = lane; t < wcap * dz; t += 64) x.dmb[(size_t)wcap * dz + t] = 0;  // (B counts per row)
  }
  if constexpr (STAMP) {
    if (d.dbgbuf && lane < 16) atomicAdd(d.dbgbuf + lane, (int32_t)(t_acc / 64));
  }
#undef KSG_STAMP2
#undef KSG_COUNT2
  const uint32_t n_peer = __builtin_amdgcn_readfirstlane(ctl->n_peer);
  for (uint32_t t = lane; t < n_peer; t += 64) {
    const uint32_t sv = L_peer[2 * t];
    int32_t expect = -1;
    __hip_atomic_compare_exchange_strong(d.svc_peer + sv, &expect, (int32_t)L_peer[2 * t + 1], __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (uint32_t t = lane; t < resolved; t += 64) out[t] = L_cm[t].out;
  if (lane == 0) {
    *rng_io = rng0 + (uint64_t)n_draws * ksg_rng_step(d.draws);
    if (reason == KSG_STOP_HANG) {
      run->halt = KSG_HALT_HANG;
    } else if (reason == KSG_STOP_OVERSIZE) {
      run->halt = KSG_HALT_OVERSIZE;  // pod pos: the host runs the exact per-pod path, then resumes
    } else if (resolved == 0 || resolved > n_pods) {
      run->halt = KSG_HALT_BADCOUNT;
    } else {
      run->pos = pos + resolved;
      run->windows += 1;
      if (reason >= 1 && reason <= 3) run->stops[reason] += 1;
    }
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
// the plain resolver (every configuration without ServiceAntiAffinity, ksg_plain.hip)
uint32_t ksg_win_plain_lds(const KsgDev& d, uint32_t wcap);
hipError_t ksg_launch_win_plain(const KsgDev& d, uint32_t P, uint32_t wcap, KsgWinRun* run, const KsgWinSum* sums,
                                const KsgWinXchg& x, uint64_t* rng, int32_t* out, hipStream_t st);

static uint32_t win_P(const KsgDev& d) {
  const uint32_t P = (d.nwords + 63) / 64;
  return P <= 1 ? 1 : P <= 2 ? 2 : P <= 4 ? 4 : P <= 8 ? 8 : P <= 16 ? 16 : P <= 32 ? 32 : 0;
}

static const size_t kWinLdsBudget = 156 * 1024;

hipError_t ksg_launch_win_eval(const KsgDev& d, int mode, const ksg_pod* batch, const uint32_t* ids,
                               const KsgWinRun* run, uint32_t wcap, KsgWinSum* sums, uint64_t* wbits, int32_t* wmax,
                               uint32_t ostride, int32_t* dcnt, uint64_t* wfit, int32_t* dmb, uint64_t* wbz,
                               uint32_t dz, hipStream_t st, const ksg_pod_ext* exts, int32_t* tmax,
                               uint64_t* psoft, int32_t* thist) {
  const uint32_t gx = std::max<uint32_t>(1, (d.nwords + KSG_SC_NT / 64 - 1) / (KSG_SC_NT / 64));
  const bool small = d.nwords < KSG_PG_WORDS;
  const uint32_t pg = small ? KSG_PG_SMALL : KSG_PG_LARGE;
  // one dimension, a multiple of 8 workgroups (the kernel's XCD-aware order)
  const dim3 grid((gx * ((wcap + pg - 1) / pg) + 7) & ~7u);
#define KSG_EVAL_LAUNCH(M, G)                                                                                    \
  hipLaunchKernelGGL((ksg_win_score_kernel<M, G>), grid, dim3(KSG_SC_NT), 0, st, d, batch, ids, run, wcap, sums, \
                     wbits, wmax, ostride, dcnt, wfit, dmb, wbz, dz, nullptr, nullptr, nullptr, nullptr)
#define KSG_EVAL_LAUNCH_X(M, G)                                                                              \
  hipLaunchKernelGGL((ksg_win_score_kernel<M, G, true>), grid, dim3(KSG_SC_NT), 0, st, d, batch, ids, \
                     run, wcap, sums, wbits, wmax, ostride, dcnt, wfit, dmb, wbz, dz, exts, tmax, psoft, thist)
  if (exts && mode == KSG_WIN_TMAX) {  // extensions: the TaintToleration count pass
    if (small) KSG_EVAL_LAUNCH_X(KSG_WIN_TMAX, KSG_PG_SMALL);
    else KSG_EVAL_LAUNCH_X(KSG_WIN_TMAX, KSG_PG_LARGE);
  } else if (exts && mode == KSG_WIN_COUNT) {  // ServiceAntiAffinity with the extension filters (round 6:
    // taints only, no extension scores, no extended-resource requests in the batch; use_window)
    if (small) KSG_EVAL_LAUNCH_X(KSG_WIN_COUNT, KSG_PG_SMALL);
    else KSG_EVAL_LAUNCH_X(KSG_WIN_COUNT, KSG_PG_LARGE);
  } else if (exts && mode == KSG_WIN_ANTI) {
    if (small) KSG_EVAL_LAUNCH_X(KSG_WIN_ANTI, KSG_PG_SMALL);
    else KSG_EVAL_LAUNCH_X(KSG_WIN_ANTI, KSG_PG_LARGE);
  } else if (exts) {  // extensions, plain mode
    if (small) KSG_EVAL_LAUNCH_X(KSG_WIN_PLAIN, KSG_PG_SMALL);
    else KSG_EVAL_LAUNCH_X(KSG_WIN_PLAIN, KSG_PG_LARGE);
  } else if (mode == KSG_WIN_COUNT) {
    if (small) KSG_EVAL_LAUNCH(KSG_WIN_COUNT, KSG_PG_SMALL);
    else KSG_EVAL_LAUNCH(KSG_WIN_COUNT, KSG_PG_LARGE);
  } else if (mode == KSG_WIN_ANTI) {
    if (small) KSG_EVAL_LAUNCH(KSG_WIN_ANTI, KSG_PG_SMALL);
    else KSG_EVAL_LAUNCH(KSG_WIN_ANTI, KSG_PG_LARGE);
  } else {
    if (small) KSG_EVAL_LAUNCH(KSG_WIN_PLAIN, KSG_PG_SMALL);
    else KSG_EVAL_LAUNCH(KSG_WIN_PLAIN, KSG_PG_LARGE);
  }
#undef KSG_EVAL_LAUNCH
#undef KSG_EVAL_LAUNCH_X
  return hipGetLastError();
}

// largest window the resolver's LDS holds for this shard
uint32_t ksg_win_max_window(const KsgDev& d) {
  const uint32_t P = win_P(d);
  if (P == 0) return 0;
  const uint32_t nflag = (d.n_services + 31) / 32;
  const bool anti = d.n_anti > 0 && d.n_domains_total > 0;
  // the LDS-slot resolver with the re-rank (KSG_DEBUG & 4096, a comparison path): up to 32k nodes
  if (anti && P > 8 && d.rr_dz && (d.dbg & 4096)) return 0;
  uint32_t lo = 0, hi = 4096;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) / 2;
    const uint32_t need = (anti && d.rr_dz && !(d.dbg & 4096))
                              ? win2_lds_offsets(P, nflag, mid, d.rr_dz, d.n_services).total
                          : anti ? win_lds_offsets(P, nflag, mid, d.n_anti > 0, d.rr_dz, d.n_services).total
                                 : ksg_win_plain_lds(d, mid);
    if (need <= kWinLdsBudget) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <int PP, bool ST, bool AN>
static hipError_t win_resolve_launch(const KsgDev& d, uint32_t wcap, size_t lds, KsgWinRun* run,
                                     const KsgWinSum* sums, const KsgWinXchg& x, uint64_t* rng, int32_t* out,
                                     hipStream_t st) {
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(ksg_win_resolve_kernel<PP, ST, AN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();  // do not leave a sticky error behind
    once = true;
  }
  hipLaunchKernelGGL((ksg_win_resolve_kernel<PP, ST, AN>), dim3(1), dim3(win_res_nt(PP)), lds, st, d, wcap, run, sums, x,
                     rng, out);
  return hipGetLastError();
}

template <int PP, bool ST, bool AN>
static hipError_t win_resolve2_launch(const KsgDev& d, uint32_t wcap, size_t lds, KsgWinRun* run,
                                      const KsgWinSum* sums, const KsgWinXchg& x, uint64_t* rng, int32_t* out,
                                      hipStream_t st) {
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(ksg_win_resolve2_kernel<PP, ST, AN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
    once = true;
  }
  hipLaunchKernelGGL((ksg_win_resolve2_kernel<PP, ST, AN>), dim3(1), dim3(512), lds, st, d, wcap, run, sums, x, rng,
                     out);
  return hipGetLastError();
}

hipError_t ksg_launch_win_resolve(const KsgDev& d, uint32_t wcap, KsgWinRun* run, const KsgWinSum* sums,
                                  const KsgWinXchg& x, uint64_t* rng, int32_t* out, hipStream_t st) {
  const uint32_t P = win_P(d);
  if (x.fit_off == 0)  // no ServiceAntiAffinity: the plain resolver (ksg_plain.hip)
    return ksg_launch_win_plain(d, P, wcap, run, sums, x, rng, out, st);
  if (x.fit_off != 0 && x.rr && !(d.dbg & 4096)) {
    // ServiceAntiAffinity with the re-rank: the register-slot resolver
    // (KSG_DEBUG & 4096: the LDS-slot resolver instead, for comparison)
    const size_t lds2 = win2_lds_offsets(P, (d.n_services + 31) / 32, wcap, x.dz, d.n_services, 1).total;
    // the debug instantiation: stamps (KSG_DEBUG & 8) or skews (bits 16..19)
    const bool stamp2 = (d.dbg & 8) != 0 || ((uint32_t)d.dbg & 0x000f0000u) != 0;
#define KSG_RES2A_CASE(PP)                                                                        \
  if (P == PP)                                                                                    \
    return stamp2 ? win_resolve2_launch<PP, true, true>(d, wcap, lds2, run, sums, x, rng, out, st) \
                  : win_resolve2_launch<PP, false, true>(d, wcap, lds2, run, sums, x, rng, out, st);
    KSG_RES2A_CASE(1)
    KSG_RES2A_CASE(2)
    KSG_RES2A_CASE(4)
    KSG_RES2A_CASE(8)
    KSG_RES2A_CASE(16)
    KSG_RES2A_CASE(32)
#undef KSG_RES2A_CASE
    return hipErrorInvalidValue;
  }
  const size_t lds =
      win_lds_offsets(P, (d.n_services + 31) / 32, wcap, x.fit_off != 0, x.rr ? x.dz : 0u, d.n_services).total;
  // the debug instantiation: stamps (KSG_DEBUG & 8) or skews (bits 16..19)
  const bool stamp = (d.dbg & 8) != 0 || ((uint32_t)d.dbg & KSG_DBG_SKEW_MASK) != 0;
  const bool anti = x.fit_off != 0;
#define KSG_RES_CASE(PP, AN)                                                                          \
  if (P == PP && anti == AN)                                                                          \
    return stamp ? win_resolve_launch<PP, true, AN>(d, wcap, lds, run, sums, x, rng, out, st)         \
                 : win_resolve_launch<PP, false, AN>(d, wcap, lds, run, sums, x, rng, out, st);
  KSG_RES_CASE(1, true)
  KSG_RES_CASE(2, true)
  KSG_RES_CASE(4, true)
  KSG_RES_CASE(8, true)
  KSG_RES_CASE(16, true)
  KSG_RES_CASE(32, true)
#undef KSG_RES_CASE
  return hipErrorInvalidValue;
}
