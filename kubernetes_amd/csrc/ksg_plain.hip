// ksg_plain.hip — phase B of the window path (the in-order resolver) for every
// configuration without ServiceAntiAffinity; ksg_window.hip has phase A and the
// anti-affinity resolvers.
//
// Phase A scored the window's W pods against one snapshot: per (pod, 64-node
// word) the word's best score and the bitmap of nodes at it. For pod i, M0 is
// its best score and T0 the nodes at M0 (k0 of them). A commit can only make
// its node worse for a later pod of the window whose service scalars it did not
// change (requested totals grow, keys and service entries are only added), so
// the reference's sequential answer (generic_scheduler.go:54-96) is the
// ix-th node, from the top, of T0 minus the committed nodes ("slots") whose
// score for pod i fell below M0 ("drops"), ix = Int63() mod (k0 - drops).
//
// One workgroup of 12 waves (8 above 16k nodes), pipelined over the window's pods:
//  PRODUCERS (waves 5..) stage pod j into ring entry j mod RING: its record,
//    T0 by word with its prefix counts (T0 bits below each 64-word row and
//    below each word inside its row: the ascending position of any node in T0
//    is two LDS reads away), its draw r (splitmix64 at the pod's draw index =
//    the drawable pods before it) and r mod (k0 - d) for d < 64, and six
//    CANDIDATES: the nodes the draw lands on when 0, 1 or 2 ties drop (the
//    (k0-1-r mod k0)-th tie ascending; the (k0-2-r mod (k0-1))-th and the next;
//    the (k0-3-r mod (k0-2))-th and the two next), with their snapshots
//    (capacity, requested totals, 10 / capacity) and the pod's service counts
//    on them.
//  CHECKERS (waves 2, 3; lane l of checker c owns slot 64c + l, its state in
//    registers) check pod i once commit i-2 is published: apply commit i-2 to
//    its slot (a new slot's snapshot from the candidate staging, else from L2),
//    then test pod i against every slot in T0 as of commits <= i-2, and post
//    the dropping slots (a 64-bit mask per checker) and each drop's position in
//    T0.
//  X-CHECKER (wave 1) re-checks pod i against the node x of commit i-1 as of
//    that commit (the checkers' view lags a commit): x's window delta and lists
//    from its own replay of the committer's slot bookkeeping (node -> slot, list
//    lengths, delta; the lists in its own rows L_xr), x's snapshot from the
//    candidate staging. Round 5: before x is drawn it computes pod i's verdict
//    on each of pod i-1's six staged candidates as of commit i-1 landing there
//    (lane-parallel, off the chain), so for a candidate x (the usual case) it
//    posts "x drops" / "commit i-1 raised a service scalar of the pod" as soon
//    as x arrives; a non-candidate x (and the extended-resource build) is
//    checked on arrival as before.
//  FLAGGER (wave 4) applies each commit's service flags in commit order from
//    the committer's published records (a ServiceSpreading maxCount rise or a
//    ServiceAffinity first peer ends the window at the next pod of that
//    service; the window's first peers are recorded for the write-back); round 4
//    had the x-checker do this after each post, which kept it busy while the
//    next node was being drawn.
//  COMMITTER (wave 0) walks the window in order. Per pod i: the ring entry; the
//    checkers' drops and the x-checker's verdict; the select: the staged
//    prediction when nothing dropped, else T0's tp-th node ascending, tp the
//    least fixed point of tp = (k-1-ix) + #(drop positions <= tp), found
//    through the row and word prefixes (no walk over the node words: the chain
//    does not grow with the node count); the drawn node and its candidate
//    index to the x-checker; the slot; the pod's keys and service ids into the
//    slot's table row; the commit record.
//
// Hand-offs (LDS; every poll is relaxed loads then one LDS-only acquire
// fence, every post a workgroup-scope release store after the data it covers):
//
//   flag / data            writer      reader              pod index        ordered by
//   r_hdr[e].ready         producer j  all but producers   j                ready = j+1 release after the entry
//   L_pub / L_drw bits     producer j  producers > j       j                L_drw before L_pub (atomicOr, in order)
//   L_cm[i].xn             committer   x-checker           i (checks i+1)   xn_seq = i+1 release after it
//   L_cm[i] record, .out,  committer   checkers (apply i   i                sel_seq = i+1 release after them
//    slot row keys / ids               at pod i+2)
//   slot row counts        checker     checkers, x-checker commits <= i-2   chk_seq release (x-checker reads
//                          (apply)                                          rows of commits it replayed: lists
//                                                                           only; counts from the staging / L2)
//   chk_seq[c], chk_msk,   checker c   committer, producers i               chk_seq[c] = i+1 release after
//    chk_cnt, L_dpos                                                        the mask, count, positions
//   xres[i & 1]            x-checker   committer           i                xseq = i+1 release after xres
//   L_xr rows              x-checker   x-checker           commits <= i-1   program order (one wave)
//   L_flag, L_peer,        flagger     committer           commits <= i-2   fseq = q+1 release after commit q's,
//    L_peerset, n_peer                 (reads at pod i)                     fseq >= i-1 acquired by the committer
//   L_peerset              flagger     x-checker (flag of  commits <= i-2   none: a stale bit only matters when
//                                      commit i-1)                          commit i-2 set it, and then L_flag
//                                                                           stops pod i anyway
//   stop, resolved         committer   all                 —                stop = 1 release after resolved
//   fin[c], fin_x, fin_f   checkers,   committer           —                release after the write-back /
//                          x-checker, flagger                               the last first peers
//
// Ring entry e = j mod RING is rewritten for pod j once the checkers are done
// with pod j-RING+2 (they apply commit j-RING while checking it), the
// x-checker with pod j-RING+1 (it reads pod j-RING's record, candidates and
// staged counts) and the flagger with commit j-RING (its record and staged
// counts). The committer reads an entry only for its own pod. Every
// wait has a spin limit; a timed-out wait sets ctl->hang and the host fails
// the batch.
#include "ksg_resolver.h"
#include "ksg_score.h"

#define KSG_NCAND 6     // candidate nodes staged per pod (0, 1 or 2 drops)
#define KSG_CSV_MAX 10  // services of a pod whose counts on the candidates are staged (6 x 10 lanes)
#define KSG_NO_CAND 7u  // commit flags: the drawn node is no candidate
// staged snapshot fields per candidate: capacity, requested totals, 10 / capacity (cpu, memory),
// (extension scores) the node's static score and taint mask, (extended resources) the
// headroom of kinds 0, 1 and of kinds 2, 3 (two int32 each)
#define KSG_CSNAP 10
// the x-checker's copy of each slot's lists (keys [0, 8), services [8, 20)), written by its own
// replay of the commits: it reads them ahead of the committer's table rows being published
#define KSG_XR_W 20
// poll pacing of the roles off the chain (s_sleep units of 64 cycles): every LDS request a
// poller issues queues with the committer's (one LDS per CU for the workgroup's 12 waves)
#ifndef KSG_PL_PROD_SLEEP
#define KSG_PL_PROD_SLEEP 1  // producers waiting for a free ring entry (8 and 32 measured no faster)
#endif
#ifndef KSG_PL_CHK_SLEEP
#define KSG_PL_CHK_SLEEP 2   // the checkers waiting for the commit they apply (0 measured the same)
#endif
#ifndef KSG_PL_XN_SLEEP
#define KSG_PL_XN_SLEEP 0    // the x-checker waiting for the drawn node (1, 2 measured no faster)
#endif
// waves of the resolver workgroup: 0 committer, 1 x-checker, 2..3 checkers, 4 flagger (service
// flags and first peers in commit order), 5.. producers: 12 waves (7 producers), 8 at P = 32,
// where a producer's T0 copy needs the registers of two waves per SIMD
__host__ __device__ constexpr uint32_t pl_nt(int P) { return P >= 32 ? 512u : 768u; }
#define KSG_PL_FW KSG_RES_P0
#define KSG_PL_P0 (KSG_PL_FW + 1)
// the resolver's ring holds the d1 bitmaps up to P = 4 (16,384 nodes)
__host__ __device__ constexpr bool pl_d1(uint32_t P) { return P <= 4; }

// one per window pod; the first 16 bytes are the commit record (stored as one
// 16-byte write), then the pod's answer and its drawn node (written apart)
struct alignas(16) PlCommit {
  uint32_t kind;   // 0: no commit (error / no fit), 1: commit
  uint32_t slot;
  uint32_t node;   // shard offset of the node
  uint32_t flags;  // bit 0: a new slot; bits 1..3: candidate index (KSG_NO_CAND: none);
                   // bits 8..15: the pod's service count; 16..23: the slot's service
                   // entries before the commit; 24..31: its conflict keys before it
  int32_t out;     // the pod's answer (shard offset + lo, or KSG_OUT_*)
  uint32_t xn;     // node drawn | its candidate index << 28 (~0u: no commit), for the x-checker
  uint32_t pad[2];
};
struct alignas(16) PlCtl {
  uint32_t stop;      // the committer is done: pods [0, resolved) are decided
  uint32_t resolved;
  uint32_t sel_seq;   // commit records published for pods [0, sel_seq)
  uint32_t n_peer;    // first service peers recorded in the window (L_peer entries)
  uint32_t chk_seq[KSG_RES_NCHK];        // pods checker c is done with
  uint32_t chk_cnt[KSG_RES_NCHK][2];     // checker c's drops for the pod of parity p
  uint32_t chk_msk[KSG_RES_NCHK][2][2];  // ... and its dropping slots (lane l: slot 64c + l)
  uint32_t fin[KSG_RES_NCHK];            // checker c applied every commit and wrote its slots back
  uint32_t hang;                         // a wait exceeded its spin limit (a bug)
  uint32_t bad;                          // a producer found the T0 prefixes inconsistent (a bug)
  uint32_t xseq;                         // pods the x-checker is done with
  uint32_t xres[2];                      // its verdict for the pod of parity p: bit 0 x drops, bit 1 flag
  uint32_t xn_seq;                       // pods whose drawn node is posted in L_cm[].xn
  uint32_t fin_x;                        // the x-checker is done
  uint32_t t_x, t_n;                     // KSG_DEBUG & 8: clock at the xres / xn posts
  uint32_t fseq;                         // commits the flagger applied the service flags of
  uint32_t fin_f;                        // the flagger applied every commit's flags and first peers
  // (extension scores) checker c's slots for the pod of parity p whose score ROSE above M0
  // (L_sig: the score) and non-T0 slots that JOINED T0 (L_dpos: their T0 position), and a
  // normalisation stop (a slot the pod fitted at its TaintToleration max no longer fits)
  uint32_t chk_rmsk[KSG_RES_NCHK][2][2];
  uint32_t chk_jmsk[KSG_RES_NCHK][2][2];
  uint32_t chk_nmsk[KSG_RES_NCHK][2][2];  // slots the pod fitted at its TaintToleration max that stopped fitting
  int32_t xsig[2];                       // (extension scores) x's score when it rose (xres bit 2)
};
struct PlLdsOff {
  uint32_t ctl, r_hdr, r_t0, r_wp, r_lp, r_rec, r_mod, r_svc, r_cand, r_csnap, r_csv, r_d1;  // ring
  uint32_t clist, xrow, dpos, sig, cm, peer, pub, drw, flag, peerset;                  // window
  uint32_t total;
};

__host__ __device__ inline PlLdsOff plain_lds_offsets(uint32_t P, uint32_t nflag, uint32_t W) {
  PlLdsOff o;
  const uint32_t R = win2_ring(P, false);
  uint32_t at = 0;
  o.ctl = at;     at += win_al16(sizeof(PlCtl));
  o.r_hdr = at;   at += win_al16((size_t)R * sizeof(RingHdr));
  o.r_t0 = at;    at += win_al16((size_t)R * P * 64 * 8);       // T0 by word
  o.r_wp = at;    at += win_al16((size_t)R * P * 64 * 2);       // T0 bits below the word in its row (u16)
  o.r_lp = at;    at += win_al16((size_t)R * 32 * 8);           // per row: T0 bits below it, up to its end
  o.r_rec = at;   at += win_al16((size_t)R * KSG_WIN_SUM_DWORDS * 4);
  o.r_mod = at;   at += win_al16((size_t)R * 64 * 4);           // r mod (k0 - d)
  o.r_svc = at;   at += win_al16((size_t)R * sizeof(RingSvc));  // the pod's services' max / peer
  o.r_cand = at;  at += win_al16((size_t)R * 8 * 4);            // candidate nodes (~0u: none)
  o.r_csnap = at; at += win_al16((size_t)R * KSG_NCAND * KSG_CSNAP * 8);  // [cand][cap c, m, used c, m, inv c, m, sst, taints]
  o.r_csv = at;   at += win_al16((size_t)R * KSG_NCAND * KSG_SLOT_SVCS * 4);  // [cand][service t] counts
  o.r_d1 = at;    at += pl_d1(P) ? win_al16((size_t)R * P * 64 * 8) : 0u;   // single-commit drop bitmaps
  // fixed sizes first: every offset up to the commit records is a compile-time
  // constant for a given P (an LDS immediate, not a register the roles' loops keep)
  o.clist = at;   at += win_al16((size_t)KSG_MAX_SLOTS * KSG_CL_W * 4);
  o.xrow = at;    at += win_al16((size_t)KSG_MAX_SLOTS * KSG_XR_W * 4);  // the x-checker's own slot lists
  o.dpos = at;    at += win_al16((size_t)2 * KSG_MAX_SLOTS * 4);
  o.sig = at;     at += win_al16((size_t)2 * KSG_MAX_SLOTS * 4);    // (extension scores) risen slots' scores
  o.cm = at;      at += win_al16((size_t)W * sizeof(PlCommit));
  o.peer = at;    at += win_al16((size_t)W * 2 * 4);
  o.pub = at;     at += win_al16((size_t)((W + 31) / 32) * 4);
  o.drw = at;     at += win_al16((size_t)((W + 31) / 32) * 4);
  o.flag = at;    at += win_al16((size_t)nflag * 4);
  o.peerset = at; at += win_al16((size_t)nflag * 4);
  o.total = at;
  return o;
}

// ---------------------------------------------------------------------------
// T0 images: per window pod, T0 by word and its prefix counts, built in parallel
// (one workgroup per pod) between phase A and the resolver, so a producer only
// copies the image into its ring entry
// ---------------------------------------------------------------------------
// image of one pod at img + pod * stride: t0 uint64[P*64] (word q*64 + l), wp
// uint16[P*64] (T0 bits below the word in its row), lp uint32[32][2] (per row:
// T0 bits below it, up to its end), hdr int32 {m0, k0}, and (KsgWinXchg.d1) d1
// uint64[P*64]: the pod's single-commit drop bitmap by word
__host__ __device__ constexpr uint32_t t0img_wp(uint32_t P) { return P * 64 * 8; }
__host__ __device__ constexpr uint32_t t0img_lp(uint32_t P) { return P * 64 * 10; }
__host__ __device__ constexpr uint32_t t0img_hdr(uint32_t P) { return P * 64 * 10 + 256; }
__host__ __device__ constexpr uint32_t t0img_d1(uint32_t P) { return (P * 64 * 10 + 256 + 16 + 15) & ~15u; }
__host__ __device__ constexpr uint32_t t0img_stride(uint32_t P) { return (t0img_d1(P) + P * 64 * 8 + 255) & ~255u; }

// byte offsets of word w's best-score bitmap and best score in the (gathered)
// phase-A blocks (KsgWinXchg), ~0u: no such word
__device__ __forceinline__ void xchg_word_at(const KsgWinXchg& x, uint32_t nwords, uint32_t w, uint32_t& b_at,
                                             uint32_t& m_at) {
  uint32_t g = 0;
  for (uint32_t r = 1; r < x.world; ++r)
    if (w >= x.wlo[r] && x.nw[r] > 0) g = r;
  const uint32_t i = w - x.wlo[g];
  const bool ok = w < nwords && i < x.nw[g];
  const uint32_t base = (uint32_t)(g * x.blk);
  b_at = ok ? base + i * 8 : ~0u;
  m_at = ok ? base + x.wcap * x.ostride * 8 + i * 4 : ~0u;
}

// (extension scores) pod i's fit word w (phase A's fit bitmaps at efit_off): in the
// block of the rank that owns word w once the blocks are all-gathered (sharded)
__device__ __forceinline__ const uint64_t* efit_word(const KsgWinXchg& x, uint32_t i, uint32_t w) {
  uint32_t g = 0;
  for (uint32_t r = 1; r < x.world; ++r)
    if (w >= x.wlo[r] && x.nw[r] > 0) g = r;
  return reinterpret_cast<const uint64_t*>(x.buf + (size_t)g * x.blk + x.efit_off) + (size_t)i * x.ostride + (w - x.wlo[g]);
}

// does the pod of resolver record `prec` (lane L holds dword L) list service s among its
// services (the record's ids after its keys and nodeSelector pairs)? (wave-uniform)
__device__ __forceinline__ bool pod_has_service(uint32_t prec, int32_t s) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint32_t npp = __builtin_amdgcn_readlane(prec, WS_NPP), nss = __builtin_amdgcn_readlane(prec, WS_NSS);
  const uint32_t at = WS_IDS + (npp & 0xffff) + (npp >> 16) + (nss & 0xffff);
  return s >= 0 && __ballot(lane - at < (nss >> 16) && lane < KSG_WIN_SUM_DWORDS && prec == (uint32_t)s) != 0;
}

template <int P>
__global__ __launch_bounds__(256) void ksg_win_t0_kernel(uint32_t nwords, uint32_t wcap, const KsgWinRun* run,
                                                         const KsgWinXchg x) {
  __shared__ int32_t s_max[4];
  __shared__ uint32_t s_tot[32];
  const uint32_t pos = run->pos, n_batch = run->n;
  if (run->halt || pos >= n_batch) return;
  const uint32_t j = blockIdx.x;
  if (j >= min(wcap, n_batch - pos)) return;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t RPW = (P + 3) / 4;  // rows per wave
  uint64_t t0[RPW];
  int32_t mw[RPW];
  int32_t lm = KSG_S32_NONE;
#pragma unroll
  for (uint32_t k = 0; k < RPW; ++k) {
    const uint32_t q = wave + 4 * k;
    uint32_t b_at = ~0u, m_at = ~0u;
    if (q < P) xchg_word_at(x, nwords, q * 64 + lane, b_at, m_at);
    t0[k] = b_at != ~0u ? *reinterpret_cast<const uint64_t*>(x.buf + b_at + (size_t)j * x.ostride * 8) : 0ULL;
    mw[k] = m_at != ~0u ? *reinterpret_cast<const int32_t*>(x.buf + m_at + (size_t)j * x.ostride * 4) : KSG_S32_NONE;
    lm = mw[k] > lm ? mw[k] : lm;
  }
  lm = wave_total_max(lm);
  if (lane == 0) s_max[wave] = lm;
  __syncthreads();
  const int32_t m0 = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
  uint8_t* im = x.img + (size_t)j * x.img_stride;
  uint64_t* it0 = reinterpret_cast<uint64_t*>(im);
  uint16_t* iwp = reinterpret_cast<uint16_t*>(im + t0img_wp(P));
  if (pl_d1(P) && x.d1) {  // (the single-commit drop bitmap: copied as it is)
    uint64_t* id1 = reinterpret_cast<uint64_t*>(im + t0img_d1(P));
#pragma unroll
    for (uint32_t k = 0; k < RPW; ++k) {
      const uint32_t q = wave + 4 * k;
      if (q >= P) break;  // (wave-uniform)
      uint32_t b_at = ~0u, m_at = ~0u;
      xchg_word_at(x, nwords, q * 64 + lane, b_at, m_at);
      id1[q * 64 + lane] = b_at != ~0u ? *reinterpret_cast<const uint64_t*>(x.buf + b_at + x.d1_off + (size_t)j * x.ostride * 8) : 0ULL;
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < RPW; ++k) {
    const uint32_t q = wave + 4 * k;
    if (q >= P) break;  // (wave-uniform)
    const uint64_t w = (m0 != KSG_S32_NONE && mw[k] == m0) ? t0[k] : 0ULL;
    const uint32_t c1 = (uint32_t)__popcll(w);
    const uint32_t in1 = dpp_scan_add(c1);
    it0[q * 64 + lane] = w;
    iwp[q * 64 + lane] = (uint16_t)(in1 - c1);
    if (lane == 63) s_tot[q] = in1;
  }
  __syncthreads();
  if (wave == 0) {  // row prefixes, k0, m0
    const uint32_t tot = lane < P ? s_tot[lane] : 0u;
    const uint32_t in1 = dpp_scan_add(tot);
    // (the cross-lane read stays outside the lane-0 branch: inside it, only
    // lane 0 would be active for the scan the compiler may sink there)
    const int32_t k0 = __builtin_amdgcn_readlane((int)in1, 63);
    uint32_t* ilp = reinterpret_cast<uint32_t*>(im + t0img_lp(P));
    if (lane < P) {
      ilp[lane * 2] = in1 - tot;
      ilp[lane * 2 + 1] = in1;
    }
    if (lane == 0) {
      int32_t* ih = reinterpret_cast<int32_t*>(im + t0img_hdr(P));
      ih[0] = m0;
      ih[1] = k0;
    }
  }
}

// XS: extended resources re-checked on the slots (extensions; a separate
// instantiation: their per-slot state would cost every other configuration
// registers on the chain)
// ---------------------------------------------------------------------------
// the fused launch's scoring blocks (KsgFused, ksg_internal.h)
// ---------------------------------------------------------------------------
// pods per phase-A wave in the fused launch: 4 up to 512 words per shard (P <= 8), 8 above
__host__ __device__ constexpr int pl_pg(int P) { return P <= 8 ? 4 : 8; }

// Blocks 1.. of the fused launch: every (pod group, word group) task of the window, pod group
// major, so the resolver's first pods are scored first. Word groups are split into 8 contiguous
// ranges, one per block % 8 (the hardware deals blocks round-robin to the 8 XCDs: a word group's
// node state is fetched into one XCD's L2 for every pod group; speed only, nothing depends on the
// placement). One wave = one 64-node word x pl_pg(P) pods (ksg_score.h); its outputs are stored
// write-through, every wave drains them, and after the block's barrier one lane adds 1 to the
// group's counter shard (MI355X_MICROARCH.md, visibility: sc1 stores + vmcnt(0) + an agent
// atomic, read with sc1 loads).
// one scoring task (KSG_FUSED_NOINLINE, an A/B build: a separate function, so its registers do
// not add to the resolver's pressure in the same kernel, at the price of a call frame in scratch)
#ifdef KSG_FUSED_NOINLINE
#define KSG_FUSED_TASK_ATTR __attribute__((noinline))
#else
#define KSG_FUSED_TASK_ATTR __forceinline__
#endif
template <int PG>
__device__ KSG_FUSED_TASK_ATTR void fused_score_task(const KsgDev& d, const KsgFused& f, uint32_t pos,
                                                           uint32_t n_batch, uint32_t wcap, uint32_t w, uint32_t p0,
                                                           KsgWinSum* sums, uint64_t* wbits, int32_t* wmax,
                                                           uint32_t ostride, uint64_t* wd1, uint32_t* rec_lds) {
  win_score_wave<KSG_WIN_PLAIN, PG, false, true>(d, f.batch, f.ids, pos, n_batch, wcap, w, p0, sums, wbits, wmax,
                                                 ostride, nullptr, wd1, nullptr, nullptr, 0u, nullptr, nullptr,
                                                 nullptr, nullptr, rec_lds);
}

// arrivals that complete pod group g's counter: group 0 is scored one pod per task (the
// resolver's first pod waits for it: a quarter of a task's scoring time), the others a group per task
__host__ __device__ constexpr uint32_t fused_group_arrivals(uint32_t g, uint32_t nwg, uint32_t pg) {
  return g == 0 ? nwg * pg : nwg;
}

template <int P, bool STAMP>
__device__ __forceinline__ void fused_score_blocks(const KsgDev& d, uint32_t wcap, const KsgWinRun* run,
                                                   const KsgWinSum* sums_c, const KsgWinXchg& x, const KsgFused& f,
                                                   char* smem) {
  // (KSG_DEBUG & 8: the first task's timeline in 10-ns ticks from block 0's start, dbgbuf[55])
  const uint32_t t_b0 = STAMP ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
  constexpr uint32_t NWV = pl_nt(P) / 64;
  constexpr int PGF = pl_pg(P);
  const uint32_t pos = run->pos, n_batch = run->n;
  if (run->halt || pos >= n_batch) return;
  const uint32_t n_pods = min(wcap, n_batch - pos);
  const uint32_t ngrp = (n_pods + PGF - 1) / PGF;
  const uint32_t nwg = (d.nwords + NWV - 1) / NWV;
  const uint32_t b = blockIdx.x, xs = b & 7u;
  const uint32_t nbx = (gridDim.x - xs + 7u) / 8u - (xs == 0 ? 1u : 0u);  // (block 0 resolves)
  const uint32_t ix = (b >> 3) - (xs == 0 ? 1u : 0u);
  const uint32_t wg0 = nwg * xs / 8u, nwx = nwg * (xs + 1u) / 8u - wg0;
  const uint32_t wave = threadIdx.x >> 6;
  uint32_t* rec_lds = reinterpret_cast<uint32_t*>(smem) + wave * PGF * KSG_WIN_SUM_DWORDS;
  KsgWinSum* sums = const_cast<KsgWinSum*>(sums_c);
  uint64_t* wbits = reinterpret_cast<uint64_t*>(const_cast<uint8_t*>(x.buf));
  int32_t* wmax = reinterpret_cast<int32_t*>(const_cast<uint8_t*>(x.buf) + (size_t)x.wcap * x.ostride * 8);
  uint64_t* wd1 = x.d1 ? reinterpret_cast<uint64_t*>(const_cast<uint8_t*>(x.buf) + x.d1_off) : nullptr;
  // tasks of this XCD's word groups: group 0 as PGF one-pod tasks per word group first, then
  // groups 1.. a group per task
  const uint32_t nsplit = nwx * (uint32_t)PGF;
  for (uint32_t t = ix; t < nsplit + nwx * (ngrp - 1u); t += nbx) {
    const bool one = t < nsplit;
    const uint32_t sp = t / nwx;                        // (one: the pod; else the group - 1 past them)
    const uint32_t u = one ? t : t - nsplit;
    const uint32_t g = one ? 0u : 1u + (u / nwx);
    const uint32_t wgp = wg0 + (u - (one ? sp : g - 1u) * nwx);
    const uint32_t w = __builtin_amdgcn_readfirstlane(wgp * NWV + wave);
    const uint32_t t_k0 = STAMP ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
    if (one)
      fused_score_task<1>(d, f, pos, n_batch, wcap, w, sp, sums, wbits, wmax, x.ostride, wd1, rec_lds);
    else
      fused_score_task<PGF>(d, f, pos, n_batch, wcap, w, g * PGF, sums, wbits, wmax, x.ostride, wd1, rec_lds);
    const uint32_t t_k1 = STAMP ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
    drain_stores();  // (every storing wave: its write-through stores have landed)
    __syncthreads();
    const uint32_t t_k2 = STAMP ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(f.cnt + ((size_t)f.set * f.ngroups + g) * 8u + xs, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (STAMP) {
        // the first task (group 0, word group 0): block start, task start, scored (wave 0), drained
        // and barrier, counter added, each from block 0's start (dbgbuf[55], written by block 0)
        if (t == ix && g == 0 && wgp == 0 && d.dbgbuf) {
          const uint32_t t_k3 = (uint32_t)__builtin_amdgcn_s_memrealtime();
          const uint32_t base = (uint32_t)__hip_atomic_load(d.dbgbuf + 55, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          atomicAdd(d.dbgbuf + 56, (int32_t)(t_b0 - base));
          atomicAdd(d.dbgbuf + 57, (int32_t)(t_k0 - base));
          atomicAdd(d.dbgbuf + 58, (int32_t)(t_k1 - base));
          atomicAdd(d.dbgbuf + 59, (int32_t)(t_k2 - base));
          atomicAdd(d.dbgbuf + 60, (int32_t)(t_k3 - base));
          atomicAdd(d.dbgbuf + 61, 1);
        }
      }
    }
  }
}

// has pod group g of the fused launch been scored (all word groups, summed over the 8 shards)?
// (wave-uniform; sc1 loads of the counters)
template <int P>
__device__ __forceinline__ bool fused_group_done(const KsgFused& f, uint32_t g, uint32_t nwg) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint32_t v = lane < 8 ? ld_mut(f.cnt + ((size_t)f.set * f.ngroups + g) * 8u + lane) : 0u;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += (uint32_t)__builtin_amdgcn_readlane((int)v, k);
  return s >= fused_group_arrivals(g, nwg, (uint32_t)pl_pg(P));
}

// the resolver's body; two kernels below: the plain launch (no fused-launch argument at all, so
// its code and register allocation are the resolver's alone) and the fused window launch
template <int P, bool STAMP, bool XS, bool FUSED>
__device__ __forceinline__ void win_plain_body(const KsgDev d, uint32_t wcap, KsgWinRun* run,
                                               const KsgWinSum* __restrict__ sums, const KsgWinXchg x,
                                               uint64_t* rng_io, int32_t* __restrict__ out_batch, const KsgFused f) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t t_blk0 = 0;  // (KSG_DEBUG & 8, fused: block 0's start, the base of the scoring blocks' stamps)
  if constexpr (FUSED) {
    if (blockIdx.x != 0) {
      fused_score_blocks<P, STAMP>(d, wcap, run, sums, x, f, smem);
      return;
    }
    if constexpr (STAMP) t_blk0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
  }
  // (the fused launch: the window's outcome goes into the next launch's slot)
  KsgWinRun* const run_out = FUSED ? f.run_out : run;
  const uint32_t pos = run->pos, n_batch = run->n;
  if (run->halt || pos >= n_batch) {  // the chain is done (uniform, before any barrier)
    if (FUSED && threadIdx.x == 0) *run_out = *run;
    return;
  }
  // (a mailbox in dbgbuf[55] while the window runs: the committer clears it at the window's end)
  if (FUSED && STAMP && threadIdx.x == 0 && d.dbgbuf)
    __hip_atomic_store(d.dbgbuf + 55, (int32_t)t_blk0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t n_pods = min(wcap, n_batch - pos);
  int32_t* __restrict__ out = out_batch + pos;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nflag = (d.n_services + 31) / 32;
  constexpr uint32_t RING = win2_ring(P, false);
  constexpr uint32_t NT = pl_nt(P);
  constexpr uint32_t NPW = NT / 64 - KSG_PL_P0;  // producer waves
  const uint32_t f_nwg = FUSED ? (d.nwords + NT / 64 - 1) / (NT / 64) : 0u;  // (fused: word groups per pod group)
  constexpr uint32_t DW = KSG_WIN_SUM_DWORDS;
  const PlLdsOff o = plain_lds_offsets(P, nflag, wcap);
  PlCtl* ctl = reinterpret_cast<PlCtl*>(smem + o.ctl);
  RingHdr* r_hdr = reinterpret_cast<RingHdr*>(smem + o.r_hdr);
  uint64_t* r_t0 = reinterpret_cast<uint64_t*>(smem + o.r_t0);
  uint64_t* r_d1 = reinterpret_cast<uint64_t*>(smem + o.r_d1);  // (pl_d1(P): single-commit drop bitmaps)
  uint16_t* r_wp = reinterpret_cast<uint16_t*>(smem + o.r_wp);
  uint32_t* r_lp = reinterpret_cast<uint32_t*>(smem + o.r_lp);
  uint32_t* r_rec = reinterpret_cast<uint32_t*>(smem + o.r_rec);
  uint32_t* r_mod = reinterpret_cast<uint32_t*>(smem + o.r_mod);
  RingSvc* r_svc = reinterpret_cast<RingSvc*>(smem + o.r_svc);
  uint32_t* r_cand = reinterpret_cast<uint32_t*>(smem + o.r_cand);
  uint64_t* r_csnap = reinterpret_cast<uint64_t*>(smem + o.r_csnap);
  int32_t* r_csv = reinterpret_cast<int32_t*>(smem + o.r_csv);
  // per window pod: commit record, answer and drawn node (the drawn node one entry per pod: the
  // committer runs ahead of the x-checker through pods that make no commit, so a single mailbox
  // would be overwritten before it is read)
  PlCommit* L_cm = reinterpret_cast<PlCommit*>(smem + o.cm);
  uint32_t* L_peer = reinterpret_cast<uint32_t*>(smem + o.peer);
  uint32_t* L_flag = reinterpret_cast<uint32_t*>(smem + o.flag);
  uint32_t* L_peerset = reinterpret_cast<uint32_t*>(smem + o.peerset);
  uint32_t* L_pub = reinterpret_cast<uint32_t*>(smem + o.pub);  // pods whose drawable bit is known
  uint32_t* L_drw = reinterpret_cast<uint32_t*>(smem + o.drw);  // drawable pods
  uint32_t* L_cl = reinterpret_cast<uint32_t*>(smem + o.clist);  // [slot][KSG_CL_W]
  uint32_t* L_xr = reinterpret_cast<uint32_t*>(smem + o.xrow);   // [slot][KSG_XR_W] (the x-checker's)
  uint32_t* L_dpos = reinterpret_cast<uint32_t*>(smem + o.dpos);  // [parity][slot] drop positions in T0
  int32_t* L_sig = reinterpret_cast<int32_t*>(smem + o.sig);       // [parity][slot] (extension scores) risen scores
  const bool spread_on = d.w_spread != 0;
  const bool aff_on = (d.preds & KSG_PRED_SERVICEAFFINITY) && d.n_aff > 0;
  const bool res_on = (d.preds & KSG_PRED_PODFITSRESOURCES) != 0;
  const bool ports_on = (d.preds & KSG_PRED_PODFITSPORTS) != 0;
  const bool disk_on = (d.preds & KSG_PRED_NODISKCONFLICT) != 0;
  // (extensions) extended resources: re-checked on the slots like cpu / memory
  const bool xs_on = XS && (d.ext_filters & KSG_EXT_SCALAR) && d.n_scalar > 0;
  // (extensions) TaintToleration / BalancedAllocation: the slots are re-scored (risers and
  // joiners, see the committer)
  const bool esc = XS && x.esc != 0;
  const uint32_t nbits = (wcap + 31) / 32;
  // KSG_DEBUG bits 16..19: a fixed delay per pod in one wave role (committer,
  // x-checker, checkers, producers) to test the hand-offs under another
  // interleaving than the natural one (tests/test_gpu_fuzz.py)
  const uint32_t skew = STAMP ? ((uint32_t)d.dbg >> 16) & 15u : 0u;  // (debug instantiation only)
  // KSG_DEBUG bits 24..27: TIMING EXPERIMENTS ONLY (decisions are wrong): 1 the x-checker posts
  // "no drop" as soon as the node arrives, 2 the checkers post "no drops" without checking, 4 the
  // committer takes the staged prediction, 8 the committer does not wait for the verdicts
  const uint32_t xpt = STAMP ? ((uint32_t)d.dbg >> 24) & 15u : 0u;  // (debug instantiation only)

  for (uint32_t t = tid; t < RING; t += NT) r_hdr[t].ready = 0;
  if (tid == 0) *ctl = PlCtl{};
  if constexpr (FUSED)  // the next launch's counters (launch k - 1, their last user, has ended)
    for (uint32_t t = tid; t < f.ngroups * 8u; t += NT) st_mut(f.cnt + (size_t)(f.set ^ 1u) * f.ngroups * 8u + t, 0u);
  for (uint32_t w = tid; w < nflag; w += NT) {
    L_flag[w] = 0;
    L_peerset[w] = 0;
  }
  for (uint32_t w = tid; w < nbits; w += NT) {
    L_pub[w] = 0;
    L_drw[w] = 0;
  }
  __syncthreads();
  const uint64_t rng0 = *rng_io;

  // =========================================================================
  // producers
  // =========================================================================
  if (wave >= KSG_PL_P0) {
    const uint32_t* recs = reinterpret_cast<const uint32_t*>(sums);
    uint64_t p_last = 0, p_acc = 0;  // KSG_DEBUG & 8: lanes 24..27 ring wait, loads, draw wait, the rest
    auto pstamp = [&](uint32_t k) {
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        p_acc += lane == k ? t_now - p_last : 0ULL;
        p_last = t_now;
      }
    };
    if constexpr (STAMP) p_last = __builtin_amdgcn_s_memtime();
    // (KSG_DEBUG & 8, fused: 10-ns ticks from the block's start to pod 0's group scored and on to
    // its ring entry staged, summed over windows into dbgbuf[52..54])
    const uint64_t f_t0 = (STAMP && FUSED) ? __builtin_amdgcn_s_memrealtime() : 0ULL;
    uint64_t f_tg = 0;
    for (uint32_t j = wave - KSG_PL_P0; j < n_pods; j += NPW) {
      const uint32_t e = j % RING;
      // ring entry free: the checkers applied commit j - RING (while checking
      // pod j - RING + 2); the x-checker of pod j - RING + 1 read its record; the
      // flagger applied commit j - RING's flags
      for (uint32_t spin = 0;; ++spin) {
        if (ld_acq(&ctl->stop)) return;
        if (spin > KSG_SPIN_LIMIT) {
          ctl->hang = 1;
          return;
        }
        uint32_t done = min(ld_acq(&ctl->xseq), ld_acq(&ctl->fseq) + 2u);
#pragma unroll
        for (int c = 0; c < KSG_RES_NCHK; ++c) done = min(done, ld_acq(&ctl->chk_seq[c]));
        if (j < RING || done + RING >= j + 3) break;
        __builtin_amdgcn_s_sleep(KSG_PL_PROD_SLEEP);  // (far ahead of the committer: poll the LDS rarely)
      }
      pstamp(24);
      if (skew & 8u) __builtin_amdgcn_s_sleep(8);
      uint32_t rec, lpv, k0;
      int32_t m0;
      if constexpr (FUSED) {
        // pod j's group scored by the worker blocks (and pod j-1's: its record is read below)
        const uint32_t g = j / (uint32_t)pl_pg(P);
        const uint32_t g_lo = (j > 0 && j % (uint32_t)pl_pg(P) == 0) ? g - 1u : g;
        for (uint32_t spin = 0;; ++spin) {
          if (ld_acq(&ctl->stop)) return;
          if (spin > KSG_SPIN_LIMIT) {
            ctl->hang = 1;
            return;
          }
          if (fused_group_done<P>(f, g, f_nwg) && (g_lo == g || fused_group_done<P>(f, g_lo, f_nwg))) break;
          __builtin_amdgcn_s_sleep(1);
        }
        rec = lane < DW ? ld_mut(recs + (size_t)j * DW + lane) : 0u;
        // pod j's T0 image, built here from phase A's per-word results (sc1 loads of the worker
        // blocks' write-through stores): m0 = the best word maximum, T0 = the words' bitmaps at
        // m0, their in-row prefixes, the row prefixes (lane 2q: T0 bits below row q, 2q + 1:
        // through it) and k0; the single-commit drop bitmaps copied as they are
        const int32_t* pm = reinterpret_cast<const int32_t*>(x.buf + (size_t)x.wcap * x.ostride * 8) + (size_t)j * x.ostride;
        const uint64_t* pb = reinterpret_cast<const uint64_t*>(x.buf) + (size_t)j * x.ostride;
        const uint64_t* pd = reinterpret_cast<const uint64_t*>(x.buf + x.d1_off) + (size_t)j * x.ostride;
        int32_t mw[P];
        int32_t lm = KSG_S32_NONE;
        // up to 8 rows (P <= 8) the bitmaps are loaded with the maxima, one round of loads
        constexpr bool ONE = P <= 8;
        uint64_t b1[ONE ? P : 1];
#pragma unroll
        for (uint32_t q = 0; q < P; ++q) {
          const uint32_t wq = q * 64 + lane;
          mw[q] = wq < d.nwords ? ld_mut(pm + wq) : KSG_S32_NONE;
          if constexpr (ONE) b1[q] = wq < d.nwords ? ld_mut(pb + wq) : 0ULL;
          lm = mw[q] > lm ? mw[q] : lm;
        }
        m0 = wave_total_max(lm);
        if constexpr (STAMP) {
          if (j == 0) f_tg = __builtin_amdgcn_s_memrealtime();
        }
        uint64_t* f_t0 = r_t0 + (size_t)e * P * 64;
        uint16_t* f_wp = r_wp + (size_t)e * P * 64;
        uint64_t* f_d1 = r_d1 + (size_t)e * P * 64;
        const bool cp_d1 = pl_d1(P) && x.d1 != 0;
        constexpr uint32_t QC = P < 8 ? P : 8;  // rows whose loads are in flight together
        uint32_t below = 0;
        lpv = 0;
#pragma unroll
        for (uint32_t q0 = 0; q0 < P; q0 += QC) {
          uint64_t bw[QC], dw[QC];
#pragma unroll
          for (uint32_t k = 0; k < QC; ++k) {
            const uint32_t wq = (q0 + k) * 64 + lane;
            if constexpr (ONE) bw[k] = (m0 != KSG_S32_NONE && mw[q0 + k] == m0) ? b1[q0 + k] : 0ULL;
            else bw[k] = (m0 != KSG_S32_NONE && wq < d.nwords && mw[q0 + k] == m0) ? ld_mut(pb + wq) : 0ULL;
            dw[k] = (cp_d1 && wq < d.nwords) ? ld_mut(pd + wq) : 0ULL;
          }
#pragma unroll
          for (uint32_t k = 0; k < QC; ++k) {
            const uint32_t q = q0 + k;
            const uint32_t c1 = (uint32_t)__popcll(bw[k]);
            const uint32_t in1 = dpp_scan_add(c1);
            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)in1, 63);
            f_t0[q * 64 + lane] = bw[k];
            f_wp[q * 64 + lane] = (uint16_t)(in1 - c1);
            if (cp_d1) f_d1[q * 64 + lane] = dw[k];
            if (lane == 2 * q) lpv = below;
            if (lane == 2 * q + 1) lpv = below + tot;
            below += tot;
          }
        }
        k0 = below;
      } else {
      rec = lane < DW ? recs[(size_t)j * DW + lane] : 0u;
      // the pod's T0 image into the ring entry: 16-byte loads, all in flight,
      // then the LDS stores (T0 words, in-row prefixes, row prefixes, m0 / k0)
      const uint8_t* im = x.img + (size_t)j * x.img_stride;
      constexpr uint32_t NT0 = P * 64 * 8 / 16, NWP = P * 64 * 2 / 16;  // 16-byte chunks
      constexpr uint32_t ND1 = pl_d1(P) ? P * 64 * 8 / 16 : 0;             // (the d1 bitmap's, after them)
      constexpr uint32_t NC = (NT0 + NWP + ND1 + 63) / 64;
      const uint32_t nch = NT0 + NWP + (x.d1 ? ND1 : 0u);
      uint4 ch[NC];
#pragma unroll
      for (uint32_t k = 0; k < NC; ++k) {
        const uint32_t t = k * 64 + lane;
        const uint8_t* src = t < NT0 + NWP ? im + (size_t)t * 16 : im + t0img_d1(P) + (size_t)(t - NT0 - NWP) * 16;
        ch[k] = t < nch ? *reinterpret_cast<const uint4*>(src) : uint4{0, 0, 0, 0};
      }
      lpv = lane < 2 * P ? *reinterpret_cast<const uint32_t*>(im + t0img_lp(P) + lane * 4) : 0u;
      m0 = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int32_t*>(im + t0img_hdr(P)));
      k0 = (uint32_t)__builtin_amdgcn_readfirstlane(*reinterpret_cast<const int32_t*>(im + t0img_hdr(P) + 4));
      uint4* e_t0 = reinterpret_cast<uint4*>(r_t0 + (size_t)e * P * 64);
      uint4* e_wp = reinterpret_cast<uint4*>(r_wp + (size_t)e * P * 64);
      uint4* e_d1 = reinterpret_cast<uint4*>(r_d1 + (size_t)e * P * 64);
#pragma unroll
      for (uint32_t k = 0; k < NC; ++k) {
        const uint32_t t = k * 64 + lane;
        if (t < NT0) e_t0[t] = ch[k];
        else if (t < NT0 + NWP) e_wp[t - NT0] = ch[k];
        else if (t < nch) e_d1[t - NT0 - NWP] = ch[k];
      }
      }
      const bool drawable = __builtin_amdgcn_readlane(rec, WS_ERR) == 0 && m0 != KSG_S32_NONE;
      const uint32_t wj = j >> 5, bj = 1u << (j & 31);
      if (lane == 0) {  // the drawable bit first, then "known" (readers read them in that order)
        if (drawable) atomicOr(&L_drw[wj], bj);
        atomicOr(&L_pub[wj], bj);
      }
      if (lane < 2 * P) r_lp[e * 64 + lane] = lpv;
      // (the entry is read back below through other pointer types: no
      // reordering of those loads above these stores)
      asm volatile("" ::: "memory");
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
      const uint32_t n_svcs = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NSS) >> 16;
      const uint32_t nk = ((uint32_t)__builtin_amdgcn_readlane(rec, WS_NPP) & 0xffff) +
                          ((uint32_t)__builtin_amdgcn_readlane(rec, WS_NPP) >> 16);
      const uint32_t n_sel = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NSS) & 0xffff;
      const bool inl = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NINL) <= KSG_WIN_INLINE && n_svcs <= KSG_SLOT_SVCS;
      // the candidates: ascending T0 positions k0-1-ix0; k0-2-ix1 (+1); k0-3-ix2
      // (+1, +2), found like the committer's select (row prefixes, then the row's
      // word prefixes, then the bit); lane c < 6 holds candidate c
      // (shuffles with every lane active: a disabled source lane reads as 0)
      const uint32_t lpe_ = (uint32_t)__shfl((int)lpv, (int)((2 * lane) & 63), 64);
      const uint32_t lpi_ = (uint32_t)__shfl((int)lpv, (int)((2 * lane + 1) & 63), 64);
      const uint32_t lp_ex = lane < P ? lpe_ : 0u, lp_in = lane < P ? lpi_ : 0u;
      const uint64_t* t0e = r_t0 + (size_t)e * P * 64;
      uint32_t cand_l = ~0u, cand0 = ~0u;
      if (drawable) {
#pragma unroll
        for (int c = 0; c < KSG_NCAND; ++c) {
          const uint32_t dd = c == 0 ? 0u : c < 3 ? 1u : 2u;
          const uint32_t off = c == 0 ? 0u : c < 3 ? (uint32_t)c - 1 : (uint32_t)c - 3;
          if (k0 > dd) {
            const uint32_t ixd = (uint32_t)__builtin_amdgcn_readlane((int)mv, (int)dd);
            const uint32_t tp = k0 - 1 - dd - ixd + off;
            const uint32_t qs = (uint32_t)__builtin_ctzll(__ballot(lane < P && lp_ex <= tp && tp < lp_in));
            const uint32_t loc = tp - (uint32_t)__builtin_amdgcn_readlane((int)lp_ex, (int)qs);
            const uint64_t w = t0e[qs * 64 + lane];
            const uint32_t wpq = r_wp[(size_t)e * P * 64 + qs * 64 + lane];
            const uint32_t ls = (uint32_t)__builtin_ctzll(__ballot(wpq <= loc && loc < wpq + (uint32_t)__popcll(w)));
            const uint64_t ws = readlane64(w, (int)ls);
            const uint32_t lw = loc - (uint32_t)__builtin_amdgcn_readlane((int)wpq, (int)ls);
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(ws >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ws, 0u));
            uint32_t node = (qs * 64 + ls) * 64 + (uint32_t)__builtin_ctzll(__ballot(((ws >> lane) & 1ULL) && rank == lw));
            if (qs >= P || ls >= 64 || node >= d.hi - d.lo) {  // (inconsistent prefixes: a bug; the host fails the batch)
              if ((d.dbg & 32) && lane == 0) {  // what the producer saw (ksg_debug_counters)
                int32_t* g = d.dbgbuf;
                g[0] = (int32_t)j; g[1] = (int32_t)c; g[2] = (int32_t)k0; g[3] = (int32_t)tp; g[4] = (int32_t)qs;
                g[5] = (int32_t)ls; g[6] = (int32_t)loc; g[7] = (int32_t)__builtin_amdgcn_readlane((int)lp_ex, 0);
                g[8] = (int32_t)__builtin_amdgcn_readlane((int)lp_in, 0); g[9] = m0; g[10] = (int32_t)ixd;
                g[11] = (int32_t)__builtin_amdgcn_readlane((int)wpq, 0);
                g[12] = (int32_t)__builtin_amdgcn_readlane((int)__popcll(w), 0);
                g[13] = (int32_t)__builtin_amdgcn_readlane((int)wpq, 7);
                g[14] = (int32_t)__builtin_amdgcn_readlane((int)__popcll(w), 7);
                g[15] = (int32_t)lpv; g[16] = (int32_t)__builtin_amdgcn_readlane((int)lpv, 1);
                g[17] = (int32_t)e; g[18] = (int32_t)node;
              }
              node = ~0u;
              ctl->bad = 1;
              ctl->hang = 1;  // (the other roles stop waiting)
            }
            if (lane == (uint32_t)c) cand_l = node;
            if (c == 0) cand0 = node;
          }
        }
      }
      // their snapshots (lane L < 60: candidate L / 10, field L % 10; the static score and the
      // taints only with extension scores, the extended resources' headroom only with those) and the pod's service counts on them (lane
      // L < 6 n_svcs: candidate L / n_svcs, service L % n_svcs), all loads in flight together
      const bool csv_on = inl && n_svcs > 0 && n_svcs <= KSG_CSV_MAX;
      const uint32_t cL = lane / KSG_CSNAP, fL = lane % KSG_CSNAP;
      const uint32_t cn_ = (uint32_t)__shfl((int)cand_l, (int)(cL < KSG_NCAND ? cL : 0u), 64);
      const uint32_t cn = lane < KSG_CSNAP * KSG_NCAND ? cn_ : ~0u;
      uint64_t snap = 0;
      if (cn != ~0u) {
        const uint32_t pn = d.lo + cn;
        const int64_t* src = fL == 0 ? d.cap_cpu : fL == 1 ? d.cap_mem : fL == 2 ? d.used_cpu : d.used_mem;
        if (fL < 4)
          snap = (uint64_t)gld(src + pn);
        else if (fL < 6)
          snap = (uint64_t)gld(reinterpret_cast<const int64_t*>(fL == 4 ? d.inv10_cpu : d.inv10_mem) + pn);
        else if (esc && fL == 6)
          snap = d.has_static_score ? (uint64_t)gld(d.static_score + pn) : 0ULL;
        else if (esc && fL == 7)
          snap = d.ntaint ? gld(d.ntaint + pn) : 0ULL;
        else if (xs_on && fL >= 8) {
          const uint32_t r0 = (fL - 8) * 2;
          int32_t h0 = 0, h1 = 0;
          if (r0 < d.n_scalar)
            h0 = xhead(gld(d.scalar_cap + (size_t)r0 * d.n_nodes + pn), gld(d.scalar_used + (size_t)r0 * d.n_nodes + pn));
          if (r0 + 1 < d.n_scalar)
            h1 = xhead(gld(d.scalar_cap + (size_t)(r0 + 1) * d.n_nodes + pn),
                       gld(d.scalar_used + (size_t)(r0 + 1) * d.n_nodes + pn));
          snap = (uint64_t)(uint32_t)h0 | ((uint64_t)(uint32_t)h1 << 32);
        }
      }
      const uint32_t cS = csv_on ? lane / n_svcs : KSG_NCAND, tS = csv_on ? lane % n_svcs : 0u;
      const uint32_t sv_s = (uint32_t)__shfl((int)rec, (int)min(WS_IDS + nk + n_sel + tS, 63u), 64);
      const uint32_t cns_ = (uint32_t)__shfl((int)cand_l, (int)(cS < KSG_NCAND ? cS : 0u), 64);
      const uint32_t cns = cS < KSG_NCAND ? cns_ : ~0u;
      int32_t scv = 0;
      if (cns != ~0u) scv = gld(d.svc_cnt + (size_t)sv_s * d.n_nodes + d.lo + cns);
      // the pod's services' max and first peer (the flagger's service flags)
      const uint32_t t_sv = lane < n_svcs ? lane : 0u;
      const uint32_t my_sv = (uint32_t)__shfl((int)rec, (int)min(WS_IDS + nk + n_sel + t_sv, 63u), 64);
      int32_t s_max = 0, s_peer = 0;
      if (drawable && inl && lane < n_svcs) {
        s_max = gld(d.svc_max + my_sv);
        s_peer = gld(d.svc_peer + my_sv);
      }
      r_mod[e * 64 + lane] = mv;
      if (lane < DW) r_rec[e * DW + lane] = rec;
      if (lane < KSG_NCAND) r_cand[e * 8 + lane] = cand_l;
      if (lane < KSG_CSNAP * KSG_NCAND) r_csnap[(e * KSG_NCAND + cL) * KSG_CSNAP + fL] = snap;
      if (cS < KSG_NCAND) r_csv[(e * KSG_NCAND + cS) * KSG_SLOT_SVCS + tS] = scv;
      if (inl && lane < n_svcs) {
        r_svc[e].max[lane] = s_max;
        r_svc[e].peer[lane] = s_peer;
      }
      uint64_t e_ps = 0;
      int32_t e_tm = 0, e_tc = 0;
      if (esc) {  // (extension scores) the pod's soft-taint mask, TaintToleration max and its node count
        e_ps = x.psoft[j];
        e_tm = x.tmax ? x.tmax[j] : 0;
        e_tc = (x.thist && e_tm > 0) ? x.thist[(size_t)j * KSG_TBINS + e_tm] : 0;
      }
      // the committer's pod scalars (RingHdr::ps / pfl)
      const int32_t h_s = __builtin_amdgcn_readlane(rec, WS_SVC);
      const bool h_over = (uint32_t)__builtin_amdgcn_readlane(rec, WS_NINL) > KSG_WIN_INLINE || nk > KSG_SLOT_KEYS ||
                          n_svcs > KSG_SLOT_SVCS;
      // (pod j-1 of pod j's service: read only where the committer takes the d1 bitmap)
      const bool h_d1 = !XS && pl_d1(P) && x.d1 != 0 && j > 0;
      const uint32_t h_prv = (h_d1 && lane < DW) ? (FUSED ? ld_mut(recs + (size_t)(j - 1) * DW + lane)
                                                          : recs[(size_t)(j - 1) * DW + lane])
                                                 : 0u;
      const bool h_prev_s = h_d1 && pod_has_service(h_prv, h_s);
      const uint32_t h_pfl = (drawable ? 0u : 1u) | (h_prev_s ? 2u : 0u) | (h_over ? 4u : 0u) | (min(nk, 255u) << 8) |
                             (min(n_svcs, 255u) << 16) | (min(n_sel, 255u) << 24);
      if (lane == 0) {
        r_hdr[e].ps = h_s;
        r_hdr[e].pfl = h_pfl;
        r_hdr[e].psoft = e_ps;
        r_hdr[e].tmax = e_tm;
        r_hdr[e].tcnt = e_tc;
        r_hdr[e].m0 = m0;
        r_hdr[e].k0 = k0;
        r_hdr[e].r = r;
        r_hdr[e].drawable = drawable;
        r_hdr[e].pred = (int32_t)cand0;
        r_hdr[e].pad = csv_on ? 1u : 0u;  // the candidates' service counts are staged
        st_rel(&r_hdr[e].ready, j + 1);
      }
      if constexpr (STAMP && FUSED) {
        if (j == 0 && lane == 0 && d.dbgbuf) {
          const uint64_t t_r = __builtin_amdgcn_s_memrealtime();
          atomicAdd(d.dbgbuf + 52, (int32_t)(f_tg - f_t0));
          atomicAdd(d.dbgbuf + 53, (int32_t)(t_r - f_tg));
          atomicAdd(d.dbgbuf + 54, 1);
        }
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
  if (wave >= KSG_RES_C0 && wave < KSG_RES_C0 + KSG_RES_NCHK) {
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
    S.xk = 0;
    S.sst = 0;
    S.ntm = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) S.xh[r] = S.xdl[r] = 0;
    // AssumePod of pod p (plugin/pkg/scheduler/scheduler.go:115-118) into the
    // owner lane's slot: requested totals, list lengths (the committer wrote the
    // lists into the table row) and the services' snapshot counts
    // (cmv: commit p's record, prec_v: pod p's record lane, both read by the caller)
    auto apply_v = [&](uint32_t p, uint4 cmv, uint32_t prec_v) {
      const uint32_t kind = __builtin_amdgcn_readfirstlane(cmv.x);
      const uint32_t slot = __builtin_amdgcn_readfirstlane(cmv.y);
      if (kind != 1 || (slot >> 6) != c) return;
      const uint32_t woff = __builtin_amdgcn_readfirstlane(cmv.z);
      const uint32_t fl = __builtin_amdgcn_readfirstlane(cmv.w);
      const bool fresh = (fl & 1u) != 0;
      const uint32_t cidx = (fl >> 1) & 7u, n_svcs = (fl >> 8) & 0xffu, bns = (fl >> 16) & 0xffu, bnk = fl >> 24;
      const uint32_t ol = slot & 63, ep = p % RING, wn = d.lo + woff;
      const uint32_t prec = lane < DW ? prec_v : 0u;
      const PodView ppv = pod_view(prec);
      if (fresh && lane == ol) {  // the new slot's snapshot: staged for a candidate, else from L2
        if (cidx < KSG_NCAND) {
          const uint64_t* cs = r_csnap + (ep * KSG_NCAND + cidx) * KSG_CSNAP;
          S.cap_c = (int64_t)cs[0];
          S.cap_m = (int64_t)cs[1];
          S.snp_c = (int64_t)cs[2];
          S.snp_m = (int64_t)cs[3];
          S.inv_c = __longlong_as_double((long long)cs[4]);
          S.inv_m = __longlong_as_double((long long)cs[5]);
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
        S.xk = 0;
        const uint64_t* cs = r_csnap + (ep * KSG_NCAND + (cidx < KSG_NCAND ? cidx : 0u)) * KSG_CSNAP;
        if (esc) {  // (extension scores) the node's static score and taints: staged for a candidate
          S.sst = cidx < KSG_NCAND ? (int32_t)cs[6] : d.has_static_score ? (int32_t)gld(d.static_score + wn) : 0;
          S.ntm = cidx < KSG_NCAND ? cs[7] : d.ntaint ? gld(d.ntaint + wn) : 0ULL;
        }
        if (xs_on)  // (extensions) the node's extended resource headroom at the snapshot (staged likewise)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            S.xdl[r] = 0;
            S.xh[r] = cidx < KSG_NCAND ? (int32_t)(uint32_t)(cs[8 + (r >> 1)] >> (32 * (r & 1)))
                      : (uint32_t)r < d.n_scalar ? xhead(gld(d.scalar_cap + (size_t)r * d.n_nodes + wn),
                                                         gld(d.scalar_used + (size_t)r * d.n_nodes + wn))
                                                 : 0;
          }
      }
      uint32_t new_mask = 0;
      if (n_svcs) {
        // the pod's services' snapshot counts on the node into the table row:
        // staged for a candidate, else from L2
        const bool sv_lane = lane < n_svcs;
        const uint32_t sv = sv_lane ? L_cl[(size_t)slot * KSG_CL_W + KSG_CL_SV + bns + lane] : 0u;
        const bool staged = cidx < KSG_NCAND && r_hdr[ep].pad != 0;
        int32_t cnt = 0;
        if (sv_lane)
          cnt = staged ? r_csv[(ep * KSG_NCAND + cidx) * KSG_SLOT_SVCS + lane] : gld(d.svc_cnt + (size_t)sv * d.n_nodes + wn);
        if (sv_lane) L_cl[(size_t)slot * KSG_CL_W + KSG_CL_SC + bns + lane] = (uint32_t)cnt;
        new_mask = wave_or_u32(sv_lane ? (1u << (sv & 31)) : 0u);
      }
      if (lane == ol) {
        S.dl_c = (int64_t)((uint64_t)S.dl_c + (uint64_t)ppv.req_c);
        S.dl_m = (int64_t)((uint64_t)S.dl_m + (uint64_t)ppv.req_m);
        S.nk = bnk + ppv.nk;
        S.ns = bns + n_svcs;
        S.smask |= new_mask;
        if (XS) {
          S.xk |= ppv.xm;
#pragma unroll
          for (int r = 0; r < 4; ++r) S.xdl[r] += (int32_t)__builtin_amdgcn_readlane(prec, WS_XREQ + r);
        }
      }
    };
    auto apply = [&](uint32_t p) {
      apply_v(p, *reinterpret_cast<const uint4*>(&L_cm[p]), r_rec[(p % RING) * DW + min(lane, DW - 1)]);
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
      // re-checks the node of commit i-1 itself): it starts once commit i-2 is
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
        if (KSG_PL_CHK_SLEEP) __builtin_amdgcn_s_sleep(KSG_PL_CHK_SLEEP);
      }
      acq_lds();
      cstamp(c == 0 ? 16 : 19);
      if (stopped) {
        // pods [0, resolved) are decided: apply the commits this checker has not
        // (the committer runs ahead of the checkers over pods that do not commit)
        const uint32_t R = __builtin_amdgcn_readfirstlane(ctl->resolved);
        for (uint32_t q = i >= 2 ? i - 2 : 0; q < R; ++q) apply(q);
        break;
      }
      if (skew & 4u) __builtin_amdgcn_s_sleep(8);
      if (xpt & 2u) {
        if (lane == 0) {
          ctl->chk_cnt[c][par] = 0;
          ctl->chk_msk[c][par][0] = ctl->chk_msk[c][par][1] = 0;
          st_post(&ctl->chk_seq[c], i + 1);
        }
        continue;
      }
      if (i >= 2) apply(i - 2);
      cstamp(c == 0 ? 17 : 20);
      const uint32_t rec = lane < DW ? r_rec[e * DW + lane] : 0u;
      const int32_t m0 = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].m0);
      // (extension scores) the slot's fit word and service count at the snapshot for this pod,
      // in flight over the check (read only for a node outside T0 whose score may rise)
      uint64_t e_fw = 0;
      int32_t e_cs = 0;
      if (esc && S.node != ~0u) {
        e_fw = gld(efit_word(x, i, S.node >> 6));
        const int32_t ps = (int32_t)__builtin_amdgcn_readfirstlane(r_rec[e * DW + WS_SVC]);
        if (spread_on && ps >= 0) e_cs = gld(d.svc_cnt + (size_t)ps * d.n_nodes + d.lo + S.node);
      }
      bool drop = false;
      uint32_t dpos = 0;
      uint32_t est = 0;  // (extension scores) 2: rose above M0 (esig), 4: joined T0, 8: normalisation stop
      int32_t esig = 0;
      if (!__builtin_amdgcn_readlane(rec, WS_ERR) && m0 != KSG_S32_NONE && S.node != ~0u) {
        const PodView pv = pod_view(rec);
        const uint32_t wd = S.node >> 6;
        const uint64_t tw = r_t0[(size_t)e * P * 64 + wd];
        SlotRow R;  // the slot's lists (as of the commits applied), in flight with the T0 word
        R.load(my_cl);
        // the node's ascending position in T0 (used if it drops; for a node outside
        // T0, the T0 nodes below it: where it joins)
        dpos = r_lp[e * 64 + (wd >> 6) * 2] + r_wp[(size_t)e * P * 64 + wd] +
               (uint32_t)__popcll(tw & ((1ULL << (S.node & 63)) - 1ULL));
        cstamp(c == 0 ? 22 : 40);  // (KSG_DEBUG & 8, checker 0: the check's loads; lane 40 is dropped)
        if (esc) {
          // (extension scores) the slot's whole score for pod i now (es_snap_score's sum at the
          // window's totals), against M0, the score every T0 node had at the snapshot: T0 nodes
          // drop (unfit / below M0) or rise above it; nodes outside T0 that the pod fitted at the
          // snapshot (so below M0 then) can reach M0 (join T0) or pass it (BalancedAllocation
          // rises). No snapshot terms: now - M0 is es_delta's sum for a T0 node
          const bool in_t0 = (tw >> (S.node & 63)) & 1ULL;
          const int64_t now_c = (int64_t)((uint64_t)S.snp_c + (uint64_t)S.dl_c);
          const int64_t now_m = (int64_t)((uint64_t)S.snp_m + (uint64_t)S.dl_m);
          bool unfit = false;
          if (res_on && !pv.zero_req)  // PodFitsResources (predicates.go:127-145)
            unfit = !((S.cap_c == 0 || S.cap_c - now_c >= pv.req_c) && (S.cap_m == 0 || S.cap_m - now_m >= pv.req_m));
          if (S.xk & pv.xm)  // extended resources
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int32_t q = (int32_t)__builtin_amdgcn_readlane(rec, WS_XREQ + r);
              unfit |= q > 0 && S.xh[r] - S.xdl[r] < q;
            }
          if (!unfit && pv.nk && S.nk)  // PodFitsPorts / NoDiskConflict vs the window's keys
            unfit |= R.key_hit(S.nk, rec, pv.nk, pv.n_ports, ports_on, disk_on);
          // ServiceSpreading: the window's entries of the pod's service here (maxCount fixed)
          int32_t snapc = 0, sdel = 0;
          if (spread_on && pv.s >= 0 && ((S.smask >> (pv.s & 31)) & 1u)) R.svc(S.ns, (uint32_t)pv.s, snapc, sdel);
          cstamp(c == 0 ? 14 : 40);  // (checker 0, extension scores: fit and the window's service entries)
          const bool sp = spread_on && pv.s >= 0 && pv.smax > 0;
          const uint64_t psoft = r_hdr[e].psoft;
          const int32_t tmx = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].tmax);
          const int32_t soft = __popcll(S.ntm & psoft);
          const bool at_max = d.w_taint != 0 && tmx > 0 && soft == tmx;
          // two independent LeastRequested terms (branch-free, so they interleave), the
          // BalancedAllocation term, then the service count (its load the last to be waited for)
          const int64_t tcn = (int64_t)((uint64_t)now_c + (uint64_t)pv.req_c), tmn = (int64_t)((uint64_t)now_m + (uint64_t)pv.req_m);
          int32_t now = S.sst;  // (int32: every window-path score sum stays below 2^30, use_window)
          if (d.w_lr) now += (int32_t)d.w_lr * ((lr_win_nb(tcn, S.cap_c, S.inv_c) + lr_win_nb(tmn, S.cap_m, S.inv_m)) >> 1);
          if (d.w_bal) now += d.w_bal * (int32_t)balanced_score(tcn, S.cap_c, tmn, S.cap_m);
          if (d.w_taint) now += d.w_taint * (d.ntaint ? taint_score_i32(soft, tmx) : 10);
          if (d.w_spread) now += (int32_t)d.w_spread * (sp ? frac10_i32(pv.smax - (sdel ? snapc : e_cs) - sdel, pv.smax) : 10);
          cstamp(c == 0 ? 15 : 40);  // (... the score)
          if (in_t0) {
            if (unfit) {
              drop = true;
              if (at_max) est |= 8u;  // (one fewer filtered node at the normalisation max)
            } else if (now < m0) {
              drop = true;
            } else if (now > m0) {
              est |= 2u;
              esig = (int32_t)now;
            }
          } else if (unfit ? at_max : now >= m0) {
            if ((e_fw >> (S.node & 63)) & 1ULL) {  // fitted at the snapshot
              if (unfit) {
                est |= 8u;  // (an unfit node off the max changes nothing)
              } else if (now > m0) {
                est |= 2u;
                esig = (int32_t)now;
              } else {
                est |= 4u;
              }
            }
          }
          cstamp(c == 0 ? 9 : 40);  // (... the verdict)
        } else if ((tw >> (S.node & 63)) & 1ULL) {
          // does the slot (a snapshot tie of the pod) score below M0 now?
          const int64_t now_c = (int64_t)((uint64_t)S.snp_c + (uint64_t)S.dl_c);
          const int64_t now_m = (int64_t)((uint64_t)S.snp_m + (uint64_t)S.dl_m);
          if (res_on && !pv.zero_req)  // PodFitsResources (predicates.go:127-145)
            drop = !((S.cap_c == 0 || S.cap_c - now_c >= pv.req_c) && (S.cap_m == 0 || S.cap_m - now_m >= pv.req_m));
          if (XS && (S.xk & pv.xm))  // (extensions) extended resources: allocatable >= used + request
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int32_t q = (int32_t)__builtin_amdgcn_readlane(rec, WS_XREQ + r);
              drop |= q > 0 && S.xh[r] - S.xdl[r] < q;
            }
          if (d.w_lr) {  // LeastRequested (priorities.go:43-76) can only fall as requested grows
            const int32_t lr_now =
                lr_win_nb(now_c + pv.req_c, S.cap_c, S.inv_c) + lr_win_nb(now_m + pv.req_m, S.cap_m, S.inv_m);
            const int32_t lr_snap =
                lr_win_nb(S.snp_c + pv.req_c, S.cap_c, S.inv_c) + lr_win_nb(S.snp_m + pv.req_m, S.cap_m, S.inv_m);
            drop |= (lr_now >> 1) != (lr_snap >> 1);
          }
          cstamp(c == 0 ? 23 : 40);  // (checker 0: resources and LeastRequested)
          if (!drop && pv.nk && S.nk)  // PodFitsPorts / NoDiskConflict vs the window's keys
            drop |= R.key_hit(S.nk, rec, pv.nk, pv.n_ports, ports_on, disk_on);
          if (!drop && spread_on && pv.s >= 0 && ((S.smask >> (pv.s & 31)) & 1u)) {
            // ServiceSpreading (spreading.go:72-86) under an unchanged maxCount
            int32_t delta = 0, snapc = 0;
            R.svc(S.ns, (uint32_t)pv.s, snapc, delta);
            if (delta)
              drop = frac10_i32(pv.smax - snapc - delta, pv.smax) != frac10_i32(pv.smax - snapc, pv.smax);
          }
        }
      }
      if (drop || (est & 4u)) L_dpos[par * KSG_MAX_SLOTS + my_slot] = dpos;
      if (est & 2u) L_sig[par * KSG_MAX_SLOTS + my_slot] = esig;
      const uint64_t dmsk = __ballot(drop);
      if (esc) {
        const uint64_t rm = __ballot((est & 2u) != 0), jm = __ballot((est & 4u) != 0), nm = __ballot((est & 8u) != 0);
        if (lane == 0) {
          ctl->chk_rmsk[c][par][0] = (uint32_t)rm;
          ctl->chk_rmsk[c][par][1] = (uint32_t)(rm >> 32);
          ctl->chk_jmsk[c][par][0] = (uint32_t)jm;
          ctl->chk_jmsk[c][par][1] = (uint32_t)(jm >> 32);
          ctl->chk_nmsk[c][par][0] = (uint32_t)nm;
          ctl->chk_nmsk[c][par][1] = (uint32_t)(nm >> 32);
        }
      }
      if (lane == 0) {
        ctl->chk_cnt[c][par] = (uint32_t)__popcll(dmsk);
        ctl->chk_msk[c][par][0] = (uint32_t)dmsk;
        ctl->chk_msk[c][par][1] = (uint32_t)(dmsk >> 32);
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
      if (d.dbgbuf && ((lane >= 16 && lane < 24) || lane == 9 || lane == 14 || lane == 15))
        atomicAdd(d.dbgbuf + lane, (int32_t)(t_acc / 64));
    }
    drain_stores();
    if (lane == 0) st_rel(&ctl->fin[c], 1u);
    return;
  }

  // =========================================================================
  // commit q's service flags (a ServiceSpreading maxCount rise: its snapshot count
  // on the node plus the window's entries there above the snapshot max; a
  // ServiceAffinity first peer) end the window at the next pod of that service; the
  // window's first peer of a service is the earliest commit's node. One wave (the
  // flagger), in commit order, from the committer's published commit records.
  // =========================================================================
  auto flags = [&](uint32_t q, uint32_t node, uint32_t cidx, uint32_t slot, uint32_t bns, uint32_t prec) {
    const uint32_t nss = __builtin_amdgcn_readlane(prec, WS_NSS), npp = __builtin_amdgcn_readlane(prec, WS_NPP);
    const uint32_t n_svcs = nss >> 16, n_sel = nss & 0xffff, pnk = (npp & 0xffff) + (npp >> 16);
    if (!n_svcs) return;
    const uint32_t wn = d.lo + node, eq = q % RING;
    const bool sv_lane = lane < n_svcs;
    const uint32_t my_sv =
        (uint32_t)__shfl((int)prec, (int)min(WS_IDS + pnk + n_sel + (sv_lane ? lane : 0u), 63u), 64);
    const bool staged = cidx < KSG_NCAND && r_hdr[eq].pad != 0;
    int32_t mx = 0, peer = 0, cnt = 0;
    if (sv_lane) {
      cnt = staged ? r_csv[(eq * KSG_NCAND + cidx) * KSG_SLOT_SVCS + lane] : gld(d.svc_cnt + (size_t)my_sv * d.n_nodes + wn);
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
  if (wave == KSG_PL_FW) {
    // commit q's record (kind, slot, node, flags) is published with sel_seq > q; the ring
    // entry of pod q stays until fseq > q (the producers wait for it)
    auto flag_commit = [&](uint32_t q) {
      const uint4 cmv = *reinterpret_cast<const uint4*>(&L_cm[q]);
      if (__builtin_amdgcn_readfirstlane(cmv.x) != 1) return;
      const uint32_t slot = __builtin_amdgcn_readfirstlane(cmv.y), node = __builtin_amdgcn_readfirstlane(cmv.z);
      const uint32_t fl = __builtin_amdgcn_readfirstlane(cmv.w);
      const uint32_t prec = lane < DW ? r_rec[(q % RING) * DW + lane] : 0u;
      flags(q, node, (fl >> 1) & 7u, slot, (fl >> 16) & 0xffu, prec);
    };
    uint64_t f_last = 0, f_acc = 0;  // KSG_DEBUG & 8: lanes 39 wait, 40 flags
    auto fstamp = [&](uint32_t k) {
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        f_acc += lane == k ? t_now - f_last : 0ULL;
        f_last = t_now;
      }
    };
    if constexpr (STAMP) f_last = __builtin_amdgcn_s_memtime();
    uint32_t q = 0;
    for (;; ++q) {
      bool stopped = false;
      for (uint32_t spin = 0;; ++spin) {
        const uint32_t ss = ld_u(&ctl->sel_seq), st = ld_u(&ctl->stop);
        if (ss > q) break;
        if (st) {
          stopped = true;
          break;
        }
        if (spin > 16 * KSG_SPIN_LIMIT) {
          ctl->hang = 1;
          stopped = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      acq_lds();
      if (stopped) break;
      if (skew & 2u) __builtin_amdgcn_s_sleep(8);
      fstamp(39);
      flag_commit(q);
      if (lane == 0) st_post(&ctl->fseq, q + 1);
      fstamp(40);
    }
    // the committer is done: pods [0, resolved) are decided; the first peers of the
    // commits not applied yet still count (the window's end writes them)
    const uint32_t R = __builtin_amdgcn_readfirstlane(ctl->resolved);
    for (; q < R; ++q) flag_commit(q);
    if constexpr (STAMP) {
      if (d.dbgbuf && lane >= 39 && lane < 41) atomicAdd(d.dbgbuf + lane, (int32_t)(f_acc / 64));
    }
    if (lane == 0) st_rel(&ctl->fin_f, 1u);
    return;
  }

  // =========================================================================
  // x-checker (wave 1): pod i against commit i-1's node x as of that commit
  // (the checkers' view lags a commit). Without extended resources (XS) the
  // verdicts on each of pod i-1's staged candidates are computed BEFORE x is
  // drawn (x is usually one of them) and the one for x is posted as soon as x
  // arrives; otherwise, or for a non-candidate x, x is checked on arrival.
  // =========================================================================
  if (wave == 1) {
    __builtin_amdgcn_s_setprio(2);
    // lane L < 4 evaluates one LeastRequested term: resource L & 1 (cpu, memory),
    // at the node's requested total now (L < 2) or at the snapshot (L >= 2)
    const uint32_t rl = lane & 1;
    // the committer's slot bookkeeping, replayed: lane l holds slots l and 64 + l
    // (node, list lengths, window delta after the commits replayed so far); the
    // slots' lists go into this wave's own rows (L_xr)
    uint32_t xcn0 = ~0u, xcn1 = ~0u, xsk0 = 0, xsk1 = 0, xss0 = 0, xss1 = 0, xn_slots = 0;
    uint32_t xsx0 = 0, xsx1 = 0;  // (extensions) extended resource kinds the window took on the slot
    int32_t xsd0[4] = {0, 0, 0, 0}, xsd1[4] = {0, 0, 0, 0};  // ... and its requests of each kind
    int64_t xdc0 = 0, xdm0 = 0, xdc1 = 0, xdm1 = 0;
    // KSG_DEBUG & 8: lanes 28 wait for the node, 29 post + replay, 31 node hand-off, 32 / 33
    // the check / extension scores, 34 ring wait; 41 / 42 (x 64) commits answered from the
    // d1 bitmap by the committer / checked here
    uint64_t x_last = 0, x_acc = 0;
    auto xstamp = [&](uint32_t k) {
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        x_acc += lane == k ? t_now - x_last : 0ULL;
        x_last = t_now;
      }
    };
    auto replay = [&](uint32_t node, uint32_t prec, uint32_t& slot, uint32_t& bnk, uint32_t& bns, uint64_t& dlc,
                      uint64_t& dlm, uint32_t& xk, int32_t (&xd)[4]) {
      const PodView ppv = pod_view(prec);
      const uint32_t p_nss = (uint32_t)__builtin_amdgcn_readlane(prec, WS_NSS);
      const uint32_t p_svcs = p_nss >> 16, p_sel = p_nss & 0xffff;
      const uint64_t hit0 = __ballot(xcn0 == node), hit1 = __ballot(xcn1 == node);
      const bool in_c = (hit0 | hit1) != 0;
      bnk = bns = 0;
      dlc = dlm = 0;
      xk = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) xd[r] = 0;
      if (in_c) {
        slot = hit0 ? (uint32_t)__builtin_ctzll(hit0) : 64u + (uint32_t)__builtin_ctzll(hit1);
        const uint32_t sl = slot & 63;
        bnk = (uint32_t)__builtin_amdgcn_readlane((int)(slot < 64 ? xsk0 : xsk1), (int)sl);
        bns = (uint32_t)__builtin_amdgcn_readlane((int)(slot < 64 ? xss0 : xss1), (int)sl);
        if (XS) xk = (uint32_t)__builtin_amdgcn_readlane((int)(slot < 64 ? xsx0 : xsx1), (int)sl);
        if (xs_on)
#pragma unroll
          for (int r = 0; r < 4; ++r) xd[r] = __builtin_amdgcn_readlane(slot < 64 ? xsd0[r] : xsd1[r], (int)sl);
        dlc = readlane64((uint64_t)(slot < 64 ? xdc0 : xdc1), (int)sl);
        dlm = readlane64((uint64_t)(slot < 64 ? xdm0 : xdm1), (int)sl);
      } else {
        slot = xn_slots < KSG_MAX_SLOTS ? xn_slots++ : 0u;  // (a full table stops the committer)
      }
      // the pod's keys and service ids into this wave's row (record lane L holds dword L)
      {
        uint32_t* row = L_xr + (size_t)slot * KSG_XR_W;
        const uint32_t kt = lane - WS_IDS, st_ = lane - (WS_IDS + ppv.nk + p_sel);
        if (kt < ppv.nk && bnk + kt < KSG_SLOT_KEYS) row[bnk + kt] = prec;
        if (st_ < p_svcs && bns + st_ < KSG_SLOT_SVCS) row[KSG_SLOT_KEYS + bns + st_] = prec;
      }
      dlc += (uint64_t)ppv.req_c;
      dlm += (uint64_t)ppv.req_m;
      if (XS) {
        xk |= ppv.xm;
#pragma unroll
        for (int r = 0; r < 4; ++r) xd[r] += (int32_t)__builtin_amdgcn_readlane(prec, WS_XREQ + r);
      }
      if (lane == (slot & 63)) {
        if (slot >= 64) {
          if (!in_c) xcn1 = node;
          xsk1 = bnk + ppv.nk;
          xss1 = bns + p_svcs;
          xsx1 = xk;
#pragma unroll
          for (int r = 0; r < 4; ++r) xsd1[r] = xd[r];
          xdc1 = (int64_t)dlc;
          xdm1 = (int64_t)dlm;
        } else {
          if (!in_c) xcn0 = node;
          xsk0 = bnk + ppv.nk;
          xss0 = bns + p_svcs;
          xsx0 = xk;
#pragma unroll
          for (int r = 0; r < 4; ++r) xsd0[r] = xd[r];
          xdc0 = (int64_t)dlc;
          xdm0 = (int64_t)dlm;
        }
      }
    };
    if constexpr (STAMP) x_last = __builtin_amdgcn_s_memtime();
    uint32_t i = 0;
    for (; i < n_pods; ++i) {
      const uint32_t e = i % RING, par = i & 1, ep = (i + RING - 1) % RING;
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
        __builtin_amdgcn_s_sleep(1);
      }
      acq_lds();
      if (stopped) break;
      xstamp(34);
      // pods i's and i-1's records ahead of the node
      const uint32_t rec = lane < DW ? r_rec[e * DW + lane] : 0u;
      const int32_t m0 = (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].m0);
      const int32_t peer0 = __builtin_amdgcn_readfirstlane(r_svc[e].peer[0]);
      // (extension scores) the pod's PreferNoSchedule taints and TaintToleration max, ahead of the node
      const uint64_t x_psoft = esc ? r_hdr[e].psoft : 0ULL;
      const int32_t x_tmx = esc ? (int32_t)__builtin_amdgcn_readfirstlane(r_hdr[e].tmax) : 0;
      const uint32_t prec = (i && lane < DW) ? r_rec[ep * DW + lane] : 0u;
      const bool p_staged = i && r_hdr[ep].pad != 0;
      const PodView pv = pod_view(rec);
      const int32_t s = pv.s;
      const bool chk_pod = !__builtin_amdgcn_readlane(rec, WS_ERR) && m0 != KSG_S32_NONE;
      // (extension scores) pod i's fit word, the node taints, static score and service count of
      // each of pod i-1's staged candidates (lane c), in flight while the node is drawn: the
      // drawn node is usually one of them, and its re-score then reads no L2 on the chain
      uint64_t c_fw = 0, c_ntm = 0;
      int32_t c_sst = 0, c_cs = 0;
      const uint32_t c_node = (esc && i > 0 && lane < KSG_NCAND) ? r_cand[ep * 8 + lane] : ~0u;
      if (c_node != ~0u) {
        c_fw = gld(efit_word(x, i, c_node >> 6));
        const uint64_t* cs = r_csnap + (ep * KSG_NCAND + lane) * KSG_CSNAP;  // (staged by the producer)
        c_ntm = cs[7];
        c_sst = (int32_t)cs[6];
        c_cs = (spread_on && s >= 0) ? gld(d.svc_cnt + (size_t)s * d.n_nodes + d.lo + c_node) : 0;
      }
      // pod i-1's drawn node: its post and the node, read in one round (one wave's LDS reads
      // complete in issue order: the round that sees the post has read the node too)
      uint32_t xv = ~0u;
      for (uint32_t spin = 0;; ++spin) {
        const uint32_t xn = ld_rlx(&ctl->xn_seq), st = ld_rlx(&ctl->stop);
        asm volatile("" ::: "memory");  // (the node read stays behind the post's)
        const uint32_t xvr = L_cm[i ? i - 1 : 0].xn;
        asm volatile("" ::"v"(xvr));
        if (__builtin_amdgcn_readfirstlane(xn) >= i) {
          xv = i ? (uint32_t)__builtin_amdgcn_readfirstlane(xvr) : ~0u;
          break;
        }
        if (__builtin_amdgcn_readfirstlane(st)) {
          stopped = true;
          break;
        }
        if (spin > 16 * KSG_SPIN_LIMIT) {
          ctl->hang = 1;
          stopped = true;
          break;
        }
        if (KSG_PL_XN_SLEEP) __builtin_amdgcn_s_sleep(KSG_PL_XN_SLEEP);
      }
      acq_lds();
      if (stopped) break;
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        x_acc += lane == 28 ? t_now - x_last : 0ULL;
        x_last = t_now;
        if (i) x_acc += lane == 31 ? (uint64_t)(uint32_t)((uint32_t)t_now - ctl->t_n) : 0ULL;
      }
      if (skew & 2u) __builtin_amdgcn_s_sleep(8);
      if ((xpt & 1u) && lane == 0) {
        ctl->xres[par] = 0;
        st_post(&ctl->xseq, i + 1);
      }
      const uint32_t xnode = xv == ~0u ? ~0u : xv & 0x0fffffffu, xcid = xv == ~0u ? KSG_NO_CAND : xv >> 28;
      uint32_t xslot = 0, bnk = 0, bns = 0, xkinds = 0;
      int32_t xdl[4];
      uint64_t dlc = 0, dlm = 0;
      if (!XS && pl_d1(P) && x.d1 && xnode != ~0u && i > 0 && chk_pod) {  // (the committer's x_fast, alike)
        // a fresh x (no slot before commit i-1) under a pod i-1 of another service: phase A's
        // single-commit drop bitmap answers for x, and the committer reads it itself (x_fast);
        // only the replay is left here (off the chain)
        const bool fresh = (__ballot(xcn0 == xnode) | __ballot(xcn1 == xnode)) == 0;
        if (fresh && !pod_has_service(prec, s)) {
          if (lane == 0) st_post(&ctl->xseq, i + 1);  // (no verdict: the committer does not read it)
          replay(xnode, prec, xslot, bnk, bns, dlc, dlm, xkinds, xdl);
          if constexpr (STAMP) {
            const uint64_t t_now = __builtin_amdgcn_s_memtime();
            x_acc += lane == 29 ? t_now - x_last : 0ULL;
            x_last = t_now;
            x_acc += lane == 41 ? 64ULL : 0ULL;  // (pods whose x the committer answered)
          }
          continue;
        }
      }
      if constexpr (STAMP) x_acc += (lane == 42 && xnode != ~0u && chk_pod) ? 64ULL : 0ULL;  // (x checked on arrival)
      uint32_t res = 0;
      const bool do_check = xnode != ~0u && chk_pod;
      const uint32_t xw = d.lo + (do_check ? xnode : 0u);
      // x's snapshot: staged for a candidate (LDS), else from L2 (in flight over
      // the bookkeeping below)
      int64_t capv = 0, usev = 0;
      double invv = 0.0;
      // (extensions) lane r < 4: x's headroom of extended resource r at the snapshot
      const bool xk_chk = do_check && xs_on && pv.xm != 0;
      int32_t xhv = 0;
      if (xk_chk && lane < d.n_scalar)  // (staged with a candidate's snapshot)
        xhv = xcid < KSG_NCAND
                  ? (int32_t)(uint32_t)(r_csnap[(ep * KSG_NCAND + xcid) * KSG_CSNAP + 8 + (lane >> 1)] >> (32 * (lane & 1)))
                  : xhead(gld(d.scalar_cap + (size_t)lane * d.n_nodes + xw), gld(d.scalar_used + (size_t)lane * d.n_nodes + xw));
      if (do_check) {
        if (xcid < KSG_NCAND) {
          const uint64_t* cs = r_csnap + (ep * KSG_NCAND + xcid) * KSG_CSNAP;
          capv = (int64_t)cs[rl];
          usev = (int64_t)cs[2 + rl];
          invv = __longlong_as_double((long long)cs[4 + rl]);
        } else {
          capv = gld((rl ? d.cap_mem : d.cap_cpu) + xw);
          usev = gld((rl ? d.used_mem : d.used_cpu) + xw);
          invv = gld((rl ? d.inv10_mem : d.inv10_cpu) + xw);
        }
      }
      // (extension scores) a non-candidate x's service count at the snapshot (the checkers write
      // theirs back at the window's end), taints, static score and fit word (a candidate's were
      // staged / read before the node: no load is waited for on the chain then): in flight over
      // the replay and the check
      const int32_t n_cs = (esc && do_check && s >= 0 && xcid >= KSG_NCAND) ? gld(d.svc_cnt + (size_t)s * d.n_nodes + xw) : 0;
      const uint64_t x_t0w = (esc && do_check) ? r_t0[(size_t)e * P * 64 + (xnode >> 6)] : 0ULL;  // (x's T0 word)
      uint64_t n_fw = 0, n_ntm = 0;
      int32_t n_sst = 0;
      if (esc && do_check && xcid >= KSG_NCAND) {
        n_ntm = d.ntaint ? gld(d.ntaint + xw) : 0ULL;
        n_fw = gld(efit_word(x, i, xnode >> 6));
        n_sst = d.has_static_score ? (int32_t)gld(d.static_score + xw) : 0;
      }
      // commit i-1 into its slot (the committer's bookkeeping, replayed). A fresh x (its first
      // commit in the window, no slot yet) is checked from pod i-1's own record -- the slot holds
      // exactly that pod -- and replayed after the verdict is posted, off the committer's chain
      const bool x_new = xnode != ~0u && (__ballot(xcn0 == xnode) | __ballot(xcn1 == xnode)) == 0;
      uint32_t fx_cl = ~0u;  // (fresh x) the row the replay would write: pod i-1's keys, then its services
      if (x_new) {
        const PodView xpv = pod_view(prec);
        const uint32_t xnss = __builtin_amdgcn_readlane(prec, WS_NSS);
        const uint32_t psel = xnss & 0xffff, psv = xnss >> 16;
        const uint32_t src = lane < KSG_SLOT_KEYS ? WS_IDS + lane : WS_IDS + xpv.nk + psel + (lane - KSG_SLOT_KEYS);
        const uint32_t v = (uint32_t)__shfl((int)prec, (int)min(src, 63u), 64);
        fx_cl = (lane < KSG_SLOT_KEYS ? lane < xpv.nk : (lane < KSG_XR_W && lane - KSG_SLOT_KEYS < psv)) ? v : ~0u;
        bnk = bns = 0;
        dlc = (uint64_t)xpv.req_c;
        dlm = (uint64_t)xpv.req_m;
        xkinds = XS ? xpv.xm : 0u;
#pragma unroll
        for (int r = 0; r < 4; ++r) xdl[r] = XS ? (int32_t)__builtin_amdgcn_readlane(prec, WS_XREQ + r) : 0;
      } else if (xnode != ~0u) {
        replay(xnode, prec, xslot, bnk, bns, dlc, dlm, xkinds, xdl);
      }
      if (do_check) {
        // the slot's lists with commit i-1's entries: this wave's row (just written by the replay)
        const uint32_t pnpp = __builtin_amdgcn_readlane(prec, WS_NPP), pnss = __builtin_amdgcn_readlane(prec, WS_NSS);
        const uint32_t pnk = (pnpp & 0xffff) + (pnpp >> 16), pns = pnss >> 16;
        const uint32_t xnk = bnk + pnk, xns = bns + pns;
        // lane t < 8: key t of the slot; lane 8 + u (u < 12): its service u
        const uint32_t kt = lane - KSG_CL_KEY, ut = lane - KSG_CL_SV;
        const uint32_t xcl = x_new ? fx_cl : lane < KSG_XR_W ? L_xr[(size_t)xslot * KSG_XR_W + lane] : ~0u;
        const uint32_t nk = pv.nk;
        const bool s_ent = s >= 0 && ut < KSG_SLOT_SVCS && ut < xns && xcl == (uint32_t)s;
        const uint64_t ents = __ballot(s_ent);
        const uint32_t x_cnt_s = (uint32_t)__popcll(ents);
        const uint64_t prev_ents = __ballot(s_ent && ut >= bns);  // commit i-1's entries of service s
        const int64_t reqv = rl ? pv.req_m : pv.req_c;
        const int64_t nowv = (int64_t)((uint64_t)usev + (rl ? dlm : dlc));  // requested total now
        bool xd = false, flag_x = false;
        bool xu = false;  // x no longer fits the pod (resources, keys, extended resources)
        int32_t x_snapc = 0;
        if (res_on && !pv.zero_req)  // PodFitsResources: lanes 0 and 1
          xu = xd = (__ballot(lane < 2 && !(capv == 0 || capv - nowv >= reqv)) & 3ULL) != 0;
        if (d.w_lr && !esc) {  // LeastRequested: one term per lane (extension scores: below)
          const int32_t lrv = lr_win((lane < 2 ? nowv : usev) + reqv, capv, invv);
          const int32_t lr_now = __builtin_amdgcn_readlane(lrv, 0) + __builtin_amdgcn_readlane(lrv, 1);
          const int32_t lr_snap = __builtin_amdgcn_readlane(lrv, 2) + __builtin_amdgcn_readlane(lrv, 3);
          xd |= (lr_now >> 1) != (lr_snap >> 1);
        }
        if (x_cnt_s) {
          // s's snapshot count on x: staged with pod i-1's services when pod i-1 is
          // a pod of s, else from L2 (the checkers may not have written it yet)
          if (prev_ents && p_staged && xcid < KSG_NCAND)
            x_snapc = r_csv[(ep * KSG_NCAND + xcid) * KSG_SLOT_SVCS + (uint32_t)__builtin_ctzll(prev_ents) - KSG_CL_SV - bns];
          else
            x_snapc = !esc ? gld(d.svc_cnt + (size_t)s * d.n_nodes + xw)
                      : xcid < KSG_NCAND ? __builtin_amdgcn_readlane(c_cs, (int)xcid) : n_cs;
          x_snapc = __builtin_amdgcn_readfirstlane(x_snapc);
          if (spread_on && !esc) {  // ServiceSpreading under an unchanged maxCount: lane 0 now, lane 1 the snapshot
            const int32_t fr = (int32_t)frac10_i32(pv.smax - x_snapc - (lane == 0 ? (int32_t)x_cnt_s : 0),
                                                   pv.smax);
            xd |= __builtin_amdgcn_readlane(fr, 0) != __builtin_amdgcn_readlane(fr, 1);
          }
          if (prev_ents) {  // commit i-1, a pod of service s: maxCount rises / first peer
            flag_x = spread_on && x_snapc + (int32_t)x_cnt_s > pv.smax;
            if (aff_on && peer0 == -1 && !((L_peerset[s >> 5] >> (s & 31)) & 1u)) flag_x = true;
          }
        }
        if (nk && xnk) {  // PodFitsPorts / NoDiskConflict: lane t holds key t
          bool hit = false;
          for (uint32_t b = 0; b < nk; ++b) {
            const bool on = b < pv.n_ports ? ports_on : disk_on;
            hit |= on && kt < KSG_SLOT_KEYS && kt < xnk && xcl == (uint32_t)__builtin_amdgcn_readlane((int)rec, (int)(WS_IDS + b));
          }
          const bool kh = __ballot(hit) != 0;
          xd |= kh;
          xu |= kh;
        }
        if (xk_chk && (xkinds & pv.xm)) {  // (extensions) extended resources, lane r: kind r
          const int32_t q = __shfl((int)rec, (int)(WS_XREQ + (lane & 3)), 64);  // (a per-lane source: not readlane)
          const int32_t dl = (lane & 3) == 0 ? xdl[0] : (lane & 3) == 1 ? xdl[1] : (lane & 3) == 2 ? xdl[2] : xdl[3];
          const bool xh = (__ballot(lane < 4 && q > 0 && xhv - dl < q) & 15ULL) != 0;
          xd |= xh;
          xu |= xh;
        }
        res = (xd ? 1u : 0u) | (flag_x ? 2u : 0u);
        if constexpr (STAMP) {  // (lane 32: the check before the extension scores)
          const uint64_t t_now = __builtin_amdgcn_s_memtime();
          x_acc += lane == 32 ? t_now - x_last : 0ULL;
          x_last = t_now;
        }
        if (esc) {
          // (extension scores) x re-scored as the checkers do a slot: bit 0 drop (a T0 node unfit
          // or below M0), 4 rose above M0 (xsig), 8 joined T0, 16 normalisation stop
          const bool in_t0 = (x_t0w >> (xnode & 63)) & 1ULL;
          const int64_t capc = (int64_t)readlane64((uint64_t)capv, 0), capm = (int64_t)readlane64((uint64_t)capv, 1);
          const int64_t usec = (int64_t)readlane64((uint64_t)usev, 0), usem = (int64_t)readlane64((uint64_t)usev, 1);
          const double invc = __longlong_as_double((long long)readlane64((uint64_t)__double_as_longlong(invv), 0));
          const double invm = __longlong_as_double((long long)readlane64((uint64_t)__double_as_longlong(invv), 1));
          const int64_t nowc = (int64_t)((uint64_t)usec + dlc), nowm = (int64_t)((uint64_t)usem + dlm);
          const bool sp = spread_on && s >= 0 && pv.smax > 0;
          const int32_t fr_snap = (sp && x_cnt_s) ? frac10_i32(pv.smax - x_snapc, pv.smax) : 0;
          const int32_t fr_now = (sp && x_cnt_s) ? frac10_i32(pv.smax - x_snapc - (int32_t)x_cnt_s, pv.smax) : 0;
          // es_delta / es_snap_score lane-parallel (this wave's chain is the pod's): lanes 0..3 the
          // LeastRequested terms (cpu / memory, now / at the snapshot), lanes 0 / 1 BalancedAllocation
          // now / at the snapshot, one pass each instead of six calls one after another
          const int64_t tcn = (int64_t)((uint64_t)nowc + (uint64_t)pv.req_c), tmn = (int64_t)((uint64_t)nowm + (uint64_t)pv.req_m);
          const int64_t tcs = (int64_t)((uint64_t)usec + (uint64_t)pv.req_c), tms = (int64_t)((uint64_t)usem + (uint64_t)pv.req_m);
          const bool l_cpu = (lane & 1) == 0, l_now = lane < 2;
          const int32_t lrv = d.w_lr ? lr_win_nb(l_now ? (l_cpu ? tcn : tmn) : (l_cpu ? tcs : tms), l_cpu ? capc : capm,
                                                 l_cpu ? invc : invm)
                                     : 0;
          const int32_t bav = d.w_bal ? (int32_t)balanced_score(lane == 0 ? tcn : tcs, capc, lane == 0 ? tmn : tms, capm) : 0;
          const int32_t lr_n = (__builtin_amdgcn_readlane(lrv, 0) + __builtin_amdgcn_readlane(lrv, 1)) >> 1;
          const int32_t lr_s = (__builtin_amdgcn_readlane(lrv, 2) + __builtin_amdgcn_readlane(lrv, 3)) >> 1;
          const int32_t ba_n = __builtin_amdgcn_readlane(bav, 0), ba_s = __builtin_amdgcn_readlane(bav, 1);
          int32_t dl = 0;  // (es_delta's sum, term for term; int32: window-path scores stay below 2^30)
          if (d.w_lr) dl += (int32_t)d.w_lr * (lr_n - lr_s);
          if (d.w_spread) dl += (int32_t)d.w_spread * (fr_now - fr_snap);
          if (d.w_bal) dl += d.w_bal * (ba_n - ba_s);
          const uint64_t psoft = x_psoft;
          const int32_t tmx = x_tmx;
          // x's taints, static score, fit word and service count: prefetched for a candidate
          const bool cand_x = xcid < KSG_NCAND;
          const uint64_t xntm = cand_x ? readlane64(c_ntm, (int)xcid) : n_ntm;
          const int32_t soft = __popcll(xntm & psoft);
          const bool at_max = d.w_taint != 0 && tmx > 0 && soft == tmx;
          uint32_t es = 0;
          int32_t sig = 0;
          bool edrop = false;
          if (in_t0) {
            if (xu) {
              edrop = true;
              if (at_max) es |= 16u;
            } else if (dl < 0) {
              edrop = true;
            } else if (dl > 0) {
              es |= 4u;
              sig = m0 + dl;
            }
          } else if (dl > 0 || (xu && at_max)) {
            const uint64_t fw = cand_x ? readlane64(c_fw, (int)xcid) : n_fw;
            if ((fw >> (xnode & 63)) & 1ULL) {  // fitted at the snapshot
              if (xu) {
                if (at_max) es |= 16u;  // (an unfit node off the max changes nothing)
              } else {
                const int32_t cs = x_cnt_s ? x_snapc
                                           : !sp ? 0
                                           : cand_x ? __builtin_amdgcn_readlane(c_cs, (int)xcid) : n_cs;
                const int32_t frs = sp ? frac10_i32(pv.smax - cs, pv.smax) : 10;
                const int32_t xsst = cand_x ? __builtin_amdgcn_readlane(c_sst, (int)xcid) : n_sst;
                int32_t now = xsst;  // (es_snap_score's sum from the terms above, then the change)
                if (d.w_lr) now += (int32_t)d.w_lr * lr_s;
                if (d.w_spread) now += (int32_t)d.w_spread * frs;
                if (d.w_bal) now += d.w_bal * ba_s;
                if (d.w_taint) now += d.w_taint * (d.ntaint ? taint_score_i32(soft, tmx) : 10);
                now += dl;
                if (now > m0) {
                  es |= 4u;
                  sig = (int32_t)now;
                } else if (now == m0) {
                  es |= 8u;
                }
              }
            }
          }
          res = (edrop ? 1u : 0u) | (flag_x ? 2u : 0u) | es;
          if constexpr (STAMP) {  // (lane 33: the extension scores)
            const uint64_t t_now = __builtin_amdgcn_s_memtime();
            x_acc += lane == 33 ? t_now - x_last : 0ULL;
            x_last = t_now;
          }
          if (lane == 0) ctl->xsig[par] = sig;
        }
      }
      if (lane == 0 && !(xpt & 1u)) {
        ctl->xres[par] = res;
        if constexpr (STAMP) ctl->t_x = (uint32_t)__builtin_amdgcn_s_memtime();
        st_post(&ctl->xseq, i + 1);
      }
      if (x_new) replay(xnode, prec, xslot, bnk, bns, dlc, dlm, xkinds, xdl);  // (after the post)
      if constexpr (STAMP) {
        const uint64_t t_now = __builtin_amdgcn_s_memtime();
        x_acc += lane == 29 ? t_now - x_last : 0ULL;
        x_last = t_now;
      }
    }
    if constexpr (STAMP) {
      if (d.dbgbuf && ((lane >= 28 && lane < 35) || lane == 41 || lane == 42)) atomicAdd(d.dbgbuf + lane, (int32_t)(x_acc / 64));
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
  bool have_x = false;                   // commit i-1's node x (and its slot)
  uint32_t xnode = 0, xslot = 0;
  // x took a new slot at commit i-1 (its first commit in the window): with phase A's single-commit drop bitmaps (d1) this wave answers "does x drop for
  // pod i" itself when pod i-1 is of another service than pod i (x_fast below)
  bool x_fresh = false;
  const bool d1_on = !XS && pl_d1(P) && x.d1 != 0;
  uint64_t t_last = 0, t_acc = 0;
#define KSG_STAMPP(k)                                        \
  if constexpr (STAMP) {                                     \
    const uint64_t t_now = __builtin_amdgcn_s_memtime();     \
    t_acc += lane == (uint32_t)(k) ? t_now - t_last : 0ULL;  \
    t_last = t_now;                                          \
  }
#define KSG_COUNTP(k, v)                                   \
  if constexpr (STAMP) {                                   \
    t_acc += lane == (uint32_t)(k) ? (uint64_t)(v) : 0ULL; \
  }
  if constexpr (STAMP) t_last = __builtin_amdgcn_s_memtime();
  // the staged pod's entry: record, header, r mod (k0 - d), the row prefixes (lane
  // q < P), the candidates (lane c < 6), where x sits in T0 -- one round of LDS reads,
  // issued right behind the read of the entry's ready word (LDS runs one wave's reads in
  // issue order, so what they return is the staged entry whenever that ready read says
  // so; a compiler barrier keeps them behind it)
  struct Head {
    uint32_t rec, rmod, lp_ex, lp_in, cand, xlp, xwp, k0, pred, ps, pfl;
    uint64_t t0x, d1x;
  };
  const uint32_t zv = opaque_v(0u);
  auto head_reads = [&](uint32_t e) -> Head {
    // (every lane reads, at a clamped index: no exec-mask branch between the reads; the
    // lanes past each array are masked once the reads are back)
    Head h;
    h.rec = r_rec[e * DW + min(lane, DW - 1)];
    h.rmod = r_mod[e * 64 + lane];
    h.lp_ex = r_lp[e * 64 + min(lane, (uint32_t)P - 1) * 2];
    h.lp_in = r_lp[e * 64 + min(lane, (uint32_t)P - 1) * 2 + 1];
    h.cand = r_cand[e * 8 + min(lane, (uint32_t)KSG_NCAND - 1)];
    // (read whether or not there is an x: no branch between the reads, the word is
    // masked once they are back)
    // (uniform words, read at an index offset by zv, a zero the compiler cannot see: it keeps
    // them in VGPRs until their use instead of moving each to an SGPR right behind its read,
    // which would wait for the read there, splitting this round in two)
    const uint32_t xw = (have_x ? xnode >> 6 : 0u) + zv;
    h.t0x = r_t0[(size_t)e * P * 64 + xw];
    h.d1x = pl_d1(P) ? r_d1[(size_t)e * P * 64 + xw] : 0ULL;
    h.xlp = r_lp[e * 64 + (xw >> 6) * 2];
    h.xwp = r_wp[(size_t)e * P * 64 + xw];
    h.k0 = r_hdr[e + zv].k0;
    h.pred = (uint32_t)r_hdr[e + zv].pred;
    h.ps = (uint32_t)r_hdr[e + zv].ps;
    h.pfl = r_hdr[e + zv].pfl;
    __builtin_amdgcn_sched_barrier(0);  // (every read issued before any of them is used)
    return h;
  };
  for (uint32_t i = 0; i < n_pods; ++i) {
    const uint32_t e = i % RING, par = i & 1;
    const uint32_t rd0 = ld_rlx(&r_hdr[e].ready);
    asm volatile("" ::: "memory");  // (the entry's reads stay behind the ready read)
    Head h = head_reads(e);
    if (KSG_UNLIKELY(__builtin_amdgcn_readfirstlane(rd0) != i + 1)) {
      KSG_COUNTP(43, 64)  // (pods whose entry was not staged yet when the head round read it)
      const uint64_t tw0 = STAMP ? __builtin_amdgcn_s_memtime() : 0ULL;
      __builtin_amdgcn_s_setprio(0);  // a producer shares this SIMD: do not starve it
      bool hung = false;
      for (uint32_t spin = 0; ld_u(&r_hdr[e].ready) != i + 1; ++spin)
        if (spin > 16 * KSG_SPIN_LIMIT || ld_u(&ctl->hang)) {
          hung = true;
          break;
        }
      __builtin_amdgcn_s_setprio(3);
      if (KSG_UNLIKELY(hung)) {
        resolved = i;
        reason = KSG_STOP_HANG;
        break;
      }
      acq_lds();
      h = head_reads(e);  // (the staged entry, read after the wait)
      KSG_COUNTP(44, __builtin_amdgcn_s_memtime() - tw0)  // (the wait for it)
    }
    if constexpr (STAMP) {  // ring wait of the window's first 4 pods (lane 10) vs the rest (lane 11)
      const uint64_t t_now = __builtin_amdgcn_s_memtime();
      t_acc += lane == (i < 4 ? 10u : 11u) ? t_now - t_last : 0ULL;
    }
    KSG_STAMPP(0)
    if (skew & 1u) __builtin_amdgcn_s_sleep(8);
    const uint32_t rec = lane < DW ? h.rec : 0u, rmod = h.rmod;
    const uint32_t lp_ex = lane < P ? h.lp_ex : 0u, lp_in = lane < P ? h.lp_in : 0u;
    const uint32_t cand = lane < KSG_NCAND ? h.cand : ~0u;
    const uint32_t xpos0 = have_x ? __builtin_amdgcn_readfirstlane(h.xlp + h.xwp) : 0u;
    const uint64_t* t0e = r_t0 + (size_t)e * P * 64;
    const uint64_t t0x = have_x ? readlane64(h.t0x, 0) : 0ULL;
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(h.k0);
    const int32_t pred = (int32_t)__builtin_amdgcn_readfirstlane(h.pred);
    const uint32_t pfl = __builtin_amdgcn_readfirstlane(h.pfl);
    KSG_STAMPP(13)  // (the head's LDS reads; lane 1: the rest of the head)
    if (KSG_UNLIKELY(pfl & 1u)) {
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
      continue;
    }
    const PodView pv = pod_view(rec);
    const int32_t s = (int32_t)__builtin_amdgcn_readfirstlane(h.ps);  // (staged: RingHdr::ps / pfl)
    const uint32_t n_sel = pfl >> 24, n_svcs = (pfl >> 16) & 0xffu, nk = (pfl >> 8) & 0xffu;
    // x's verdict from phase A's bitmap: x fresh (its state is the snapshot plus pod i-1) and
    // pod i-1 of another service (x's service entries cannot move pod i's spreading term or
    // raise its service's scalars); the x-checker only replays such a commit
    const bool x_fast = d1_on && have_x && x_fresh && !(pfl & 2u);
    if (KSG_UNLIKELY(pfl & 4u)) {
      resolved = i;  // lists longer than the record / a slot: the exact per-pod kernel takes it
      reason = i == 0 ? KSG_STOP_OVERSIZE : KSG_STOP_SLOT;
      break;
    }
    KSG_STAMPP(1)
    // ---- the checkers' drops (slots as of commits <= i-2) and the x-checker's
    // verdict on commit i-1's node
    // the verdicts (drop counts and masks, the drops' positions, the x-checker's verdict, the
    // service flag word) are read in every poll round, right behind the sequence words
    // (LDS runs one wave's reads in issue order, so the round that finds both sequence words
    // posted has read the posted verdicts too: no second round of reads after the wait)
    struct Verd {
      uint32_t cc0, cc1, xres, fw, m0l, m0h, m1l, m1h, dp0, dp1, esw;
    };
    // (extension scores) lane w < 12: word w of the checkers' risen / joined / normalisation-stop
    // masks (checker w/2 & 1, half w & 1), lane 12 the pod's TaintToleration max count: one read
    const uint32_t* esp = lane < 4    ? &ctl->chk_rmsk[lane >> 1][par][lane & 1]
                          : lane < 8  ? &ctl->chk_jmsk[(lane - 4) >> 1][par][lane & 1]
                          : lane < 12 ? &ctl->chk_nmsk[(lane - 8) >> 1][par][lane & 1]
                                      : reinterpret_cast<const uint32_t*>(&r_hdr[e].tcnt);
    auto verdict_reads = [&]() -> Verd {
      Verd v;
      v.cc0 = ctl->chk_cnt[0][par];
      v.cc1 = ctl->chk_cnt[1][par];
      v.xres = ctl->xres[par];
      v.fw = L_flag[(s >= 0 ? (uint32_t)s : 0u) >> 5];
      v.m0l = ctl->chk_msk[0][par][0];
      v.m0h = ctl->chk_msk[0][par][1];
      v.m1l = ctl->chk_msk[1][par][0];
      v.m1h = ctl->chk_msk[1][par][1];
      v.dp0 = L_dpos[par * KSG_MAX_SLOTS + lane];
      v.dp1 = L_dpos[par * KSG_MAX_SLOTS + 64 + lane];
      v.esw = esc ? *esp : 0u;
      return v;
    };
    bool hung = false;
    Verd vd;
    for (uint32_t spin = 0;; ++spin) {
      const uint32_t xs = ld_rlx(&ctl->xseq), hg = ld_rlx(&ctl->hang), fs = ld_rlx(&ctl->fseq);
      uint32_t cs = ld_rlx(&ctl->chk_seq[0]);
#pragma unroll
      for (int c = 1; c < KSG_RES_NCHK; ++c) cs = min(cs, ld_rlx(&ctl->chk_seq[c]));
      asm volatile("" ::: "memory");  // (the verdict reads stay behind the sequence reads)
      vd = verdict_reads();
      // (and in this round: the values are inputs here, so the reads are not moved past the loop)
      asm volatile("" ::"v"(vd.cc0), "v"(vd.cc1), "v"(vd.xres), "v"(vd.fw), "v"(vd.m0l), "v"(vd.m0h), "v"(vd.m1l),
                   "v"(vd.m1h), "v"(vd.dp0), "v"(vd.dp1), "v"(vd.esw));
      // (the flagger applied the flags of commits <= i-2: fseq >= i-1; the x-checker's verdict
      // covers commit i-1's)
      if ((cs >= i + 1 && (x_fast || xs >= i + 1) && fs + 1 >= i) || (xpt & 8u)) break;
      if (KSG_UNLIKELY(spin > 16 * KSG_SPIN_LIMIT || hg)) {
        hung = true;
        break;
      }
    }
    if (KSG_UNLIKELY(hung)) {
      resolved = i;
      reason = KSG_STOP_HANG;
      break;
    }
    KSG_STAMPP(2)
    if constexpr (STAMP) t_acc += lane == 6 ? (uint64_t)(uint32_t)((uint32_t)t_last - ctl->t_x) : 0ULL;
    const uint32_t cc0 = vd.cc0, cc1 = vd.cc1, fw = vd.fw;
    const uint32_t xres = x_fast ? (uint32_t)((readlane64(h.d1x, 0) >> (xnode & 63)) & 1ULL) : __builtin_amdgcn_readfirstlane(vd.xres);
    uint64_t msk0 = ((uint64_t)__builtin_amdgcn_readfirstlane(vd.m0h) << 32) | (uint32_t)__builtin_amdgcn_readfirstlane(vd.m0l);
    uint64_t msk1 = ((uint64_t)__builtin_amdgcn_readfirstlane(vd.m1h) << 32) | (uint32_t)__builtin_amdgcn_readfirstlane(vd.m1l);
    const uint32_t dp0 = vd.dp0, dp1 = vd.dp1;
    acq_lds();  // (the ES masks, signs and the drop positions read below: after the wait)
    if (KSG_UNLIKELY(s >= 0 && (spread_on || aff_on) && ((xres & 2u) || ((__builtin_amdgcn_readfirstlane(fw) >> (s & 31)) & 1u)))) {
      resolved = i;  // a service scalar this pod reads changed in the window
      reason = KSG_STOP_SERVICE;
      break;
    }

    // x counts as a new drop iff it is a snapshot tie whose slot the checkers
    // kept (a new slot: they have not seen it)
    const bool x_kept = !(((xslot < 64 ? msk0 : msk1) >> (xslot & 63)) & 1ULL);
    bool x_drop = have_x && (xres & 1u) && ((t0x >> (xnode & 63)) & 1ULL) && x_kept;
    uint32_t dropped = (xpt & 4u) ? 0u : __builtin_amdgcn_readfirstlane(cc0) + __builtin_amdgcn_readfirstlane(cc1) + (x_drop ? 1u : 0u);
    KSG_STAMPP(12)  // (the verdicts' LDS reads; lane 3: the select and the node post)
    // (extension scores) risen slots (a score above M0: the ties are among them) and joined
    // ones (non-T0 nodes now at M0: the ties are T0 minus the drops plus them); x's verdict
    // replaces the checkers' for its slot (a BalancedAllocation score moves both ways)
    uint64_t rm0 = 0, rm1 = 0, jm0 = 0, jm1 = 0;
    uint32_t xpos = 0;
    if (esc) {
      const uint64_t xb0 = (have_x && xslot < 64) ? 1ULL << (xslot & 63) : 0ULL;
      const uint64_t xb1 = (have_x && xslot >= 64) ? 1ULL << (xslot & 63) : 0ULL;
      auto esw64 = [&](int w) -> uint64_t {  // (the poll round's words w, w + 1)
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)vd.esw, w + 1) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)vd.esw, w);
      };
      rm0 = esw64(0) & ~xb0;
      rm1 = esw64(2) & ~xb1;
      jm0 = esw64(4) & ~xb0;
      jm1 = esw64(6) & ~xb1;
      msk0 &= ~xb0;
      msk1 &= ~xb1;
      // the TaintToleration max falls once every filtered node at it stopped fitting: the
      // checkers' such slots (x's by the x-checker) against the count pass's node count
      const uint64_t nm0 = esw64(8) & ~xb0;
      const uint64_t nm1 = esw64(10) & ~xb1;
      const uint32_t gone = (uint32_t)__popcll(nm0) + (uint32_t)__popcll(nm1) + ((have_x && (xres & 16u)) ? 1u : 0u);
      const int32_t tcnt = __builtin_amdgcn_readlane((int)vd.esw, 12);
      if (gone && (int32_t)gone >= tcnt) {
        resolved = i;  // every filtered node at the pod's TaintToleration max stopped fitting
        reason = KSG_STOP_SERVICE;
        break;
      }
      x_drop = have_x && (xres & 1u);
      if (have_x && (xres & 4u)) (xslot < 64 ? rm0 : rm1) |= 1ULL << (xslot & 63);
      if (have_x && (xres & 8u)) (xslot < 64 ? jm0 : jm1) |= 1ULL << (xslot & 63);
      xpos = xpos0 + (uint32_t)__popcll(t0x & ((1ULL << (xnode & 63)) - 1ULL));
      dropped = (uint32_t)__popcll(msk0) + (uint32_t)__popcll(msk1) + (x_drop ? 1u : 0u);
    }
    const uint32_t n_add = (uint32_t)__popcll(jm0) + (uint32_t)__popcll(jm1);
    if (KSG_UNLIKELY(dropped >= k0 && n_add == 0 && (rm0 | rm1) == 0)) {
      resolved = i;  // every snapshot tie got worse: needs a fresh snapshot
      reason = KSG_STOP_EXHAUSTED;
      break;
    }
    // T0's tp-th node ascending: its row (row prefixes, lane q < P), its word (the
    // row's word prefixes) and its bit (mbcnt rank)
    auto t0_node = [&](uint32_t tp) -> uint32_t {
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
      return (qs * 64 + ls) * 64 + bsel;
    };
    // the least fixed point tp = t + #(drop positions <= tp): the t-th node of T0 minus the drops
    auto t0_minus_drops = [&](uint32_t t) -> uint32_t {
      const uint32_t d0 = ((msk0 >> lane) & 1ULL) ? dp0 : ~0u;
      const uint32_t d1 = ((msk1 >> lane) & 1ULL) ? dp1 : ~0u;
      const uint32_t xp = x_drop ? (esc ? xpos : xpos0 + (uint32_t)__popcll(t0x & ((1ULL << (xnode & 63)) - 1ULL))) : ~0u;
      uint32_t tp = t;
      for (;;) {
        const uint32_t cnt = (uint32_t)__popcll(__ballot(d0 <= tp)) + (uint32_t)__popcll(__ballot(d1 <= tp)) +
                             (xp <= tp ? 1u : 0u);
        if (t + cnt == tp) break;
        tp = t + cnt;
      }
      return tp;
    };
    auto r_draw = [&]() -> uint64_t {  // the pod's Int63 draw (staged)
      return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r_hdr[e].r >> 32)) << 32) |
             (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r_hdr[e].r);
    };
    // ---- selection: k live ties, the ix-th in descending rank = the (k-1-ix)-th ascending
    const uint32_t k = k0 - dropped;
    uint32_t woff;
    if (esc && (rm0 | rm1) != 0) {
      // risers: M* = their best score, the ties the risers at it, ix-th from the top by rank
      const int32_t sg0 = L_sig[par * KSG_MAX_SLOTS + lane], sg1 = L_sig[par * KSG_MAX_SLOTS + 64 + lane];
      const int32_t xsg = (int32_t)__builtin_amdgcn_readfirstlane(ctl->xsig[par]);
      const bool x_in0 = have_x && (xres & 4u) && xslot < 64 && lane == (xslot & 63);
      const bool x_in1 = have_x && (xres & 4u) && xslot >= 64 && lane == (xslot & 63);
      const int32_t v0 = ((rm0 >> lane) & 1ULL) ? (x_in0 ? xsg : sg0) : KSG_S32_NONE;
      const int32_t v1 = ((rm1 >> lane) & 1ULL) ? (x_in1 ? xsg : sg1) : KSG_S32_NONE;
      const int32_t ms = wave_total_max(max(v0, v1));
      uint64_t tm0 = __ballot(((rm0 >> lane) & 1ULL) && v0 == ms), tm1 = __ballot(((rm1 >> lane) & 1ULL) && v1 == ms);
      const uint32_t ks = (uint32_t)__popcll(tm0) + (uint32_t)__popcll(tm1);
      uint32_t ix = umod64_32(r_draw(), ks);
      int32_t top = -1;
      for (;;) {  // the ix-th tie from the top (HostPriorityList: score desc, host desc)
        const int32_t c0 = ((tm0 >> lane) & 1ULL) ? (int32_t)cn0 : -1, c1 = ((tm1 >> lane) & 1ULL) ? (int32_t)cn1 : -1;
        top = wave_total_max(max(c0, c1));
        if (ix == 0) break;
        --ix;
        tm0 &= ~__ballot(cn0 == (uint32_t)top);
        tm1 &= ~__ballot(cn1 == (uint32_t)top);
      }
      woff = (uint32_t)top;
    } else if (esc && n_add != 0) {
      // joiners: the ties are T0 minus the drops plus the joined nodes (each between the
      // T0 nodes around its rank: ap = the T0 nodes below it)
      const bool x_j0 = have_x && (xres & 8u) && xslot < 64 && lane == (xslot & 63);
      const bool x_j1 = have_x && (xres & 8u) && xslot >= 64 && lane == (xslot & 63);
      const uint32_t ap0 = ((jm0 >> lane) & 1ULL) ? (x_j0 ? xpos : dp0) : ~0u;
      const uint32_t ap1 = ((jm1 >> lane) & 1ULL) ? (x_j1 ? xpos : dp1) : ~0u;
      const uint32_t d0 = ((msk0 >> lane) & 1ULL) ? dp0 : ~0u, d1 = ((msk1 >> lane) & 1ULL) ? dp1 : ~0u;
      const uint32_t xdp = x_drop ? xpos : ~0u;
      const uint32_t kk = k0 - dropped + n_add;
      const uint32_t t = kk - 1 - umod64_32(r_draw(), kk);
      woff = ~0u;
      // a joined node with exactly t ties below it
      for (uint64_t mm = jm0, mh = jm1; (mm | mh) && woff == ~0u;) {
        const bool lo = mm != 0;
        const uint32_t l = (uint32_t)__builtin_ctzll(lo ? mm : mh);
        if (lo) mm &= mm - 1;
        else mh &= mh - 1;
        const uint32_t pa = (uint32_t)__builtin_amdgcn_readlane((int)(lo ? ap0 : ap1), (int)l);
        const uint32_t na = (uint32_t)__builtin_amdgcn_readlane((int)(lo ? cn0 : cn1), (int)l);
        const uint32_t bd = (uint32_t)__popcll(__ballot(d0 < pa)) + (uint32_t)__popcll(__ballot(d1 < pa)) +
                            (xdp < pa ? 1u : 0u);
        const uint32_t ba = (uint32_t)__popcll(__ballot(ap0 != ~0u && (ap0 < pa || (ap0 == pa && cn0 < na)))) +
                            (uint32_t)__popcll(__ballot(ap1 != ~0u && (ap1 < pa || (ap1 == pa && cn1 < na))));
        if (pa - bd + ba == t) woff = na;
      }
      // else a T0 node: with j joined nodes below it, the (t - j)-th of T0 minus the drops
      for (uint32_t j = 0; woff == ~0u && j <= n_add && j <= t; ++j) {
        const uint32_t tp = t0_minus_drops(t - j);
        if (tp >= k0) continue;
        const uint32_t ca = (uint32_t)__popcll(__ballot(ap0 != ~0u && ap0 <= tp)) +
                            (uint32_t)__popcll(__ballot(ap1 != ~0u && ap1 <= tp));
        if (ca == j) woff = t0_node(tp);
      }
    } else if (dropped == 0) {
      woff = (uint32_t)pred;  // staged by the producer
    } else if (dropped <= 2) {
      // one or two drops: the node is one of the producer's candidates for that
      // count (positions t, t+1 [, t+2] ascending, t = k - 1 - ix); which one
      // follows from the drop positions, no walk over T0
      KSG_COUNTP(7, 64)
      uint32_t pa = ~0u, pb = ~0u;  // the drop positions, ascending
      for (uint64_t mm = msk0; mm; mm &= mm - 1) {
        const uint32_t p = (uint32_t)__builtin_amdgcn_readlane((int)dp0, (int)__builtin_ctzll(mm));
        if (p < pa) { pb = pa; pa = p; } else if (p < pb) { pb = p; }
      }
      for (uint64_t mm = msk1; mm; mm &= mm - 1) {
        const uint32_t p = (uint32_t)__builtin_amdgcn_readlane((int)dp1, (int)__builtin_ctzll(mm));
        if (p < pa) { pb = pa; pa = p; } else if (p < pb) { pb = p; }
      }
      if (x_drop) {
        const uint32_t p = xpos0 + (uint32_t)__popcll(t0x & ((1ULL << (xnode & 63)) - 1ULL));
        if (p < pa) { pb = pa; pa = p; } else if (p < pb) { pb = p; }
      }
      const uint32_t ix = (uint32_t)__builtin_amdgcn_readlane((int)rmod, (int)dropped);
      const uint32_t t = k - 1 - ix;
      uint32_t tp = t;
      if (pa <= tp) ++tp;
      if (pb <= tp) ++tp;  // (pb > pa: the least fixed point of tp = t + #(drops <= tp))
      // candidates: 1 + (tp - t) for one drop, 3 + (tp - t) for two
      woff = (uint32_t)__builtin_amdgcn_readlane((int)cand, (int)((dropped == 1 ? 1u : 3u) + (tp - t)));
    } else {
      // T0's tp-th node ascending, tp the least fixed point of
      // tp = t + #(drop positions <= tp): its row (row prefixes, lane q < P),
      // its word (the row's word prefixes) and its bit (mbcnt rank)
      KSG_COUNTP(7, 64)
      uint32_t ix;
      if (dropped < 64) {
        ix = (uint32_t)__builtin_amdgcn_readlane((int)rmod, (int)dropped);
      } else {
        ix = umod64_32(r_draw(), k);
      }
      woff = t0_node(t0_minus_drops(k - 1 - ix));
    }
    if (KSG_UNLIKELY(woff >= d.hi - d.lo)) {  // (never: inconsistent prefixes or drop positions; the host fails the batch)
      resolved = i;
      reason = KSG_STOP_BAD;
      break;
    }
    const uint64_t cm = __ballot(cand == woff);
    const uint32_t cidx = cm ? (uint32_t)__builtin_ctzll(cm) : KSG_NO_CAND;
    if (lane == 0) {  // the x-checker takes the node's snapshot meanwhile
      L_cm[i].xn = woff | (cidx << 28);
      if constexpr (STAMP) ctl->t_n = (uint32_t)__builtin_amdgcn_s_memtime();
      st_post(&ctl->xn_seq, i + 1);
    }
    KSG_STAMPP(3)
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
      if (KSG_UNLIKELY(base_nk + nk > KSG_SLOT_KEYS || base_ns + n_svcs > KSG_SLOT_SVCS)) {
        resolved = i;  // this pod is redone (with the same draw) in the next window
        reason = KSG_STOP_SLOT;
        break;
      }
      base_dc = (int64_t)readlane64((uint64_t)(slot < 64 ? dc0 : dc1), (int)sl);
      base_dm = (int64_t)readlane64((uint64_t)(slot < 64 ? dm0 : dm1), (int)sl);
    } else {
      if (KSG_UNLIKELY(n_slots == KSG_MAX_SLOTS)) {
        resolved = i;
        reason = KSG_STOP_SLOT;
        break;
      }
      slot = n_slots++;
    }
    const int64_t new_dc = (int64_t)((uint64_t)base_dc + (uint64_t)pv.req_c);
    const int64_t new_dm = (int64_t)((uint64_t)base_dm + (uint64_t)pv.req_m);
    const uint32_t wn = d.lo + woff;
    KSG_STAMPP(4)
    // the slot's table row: the pod's keys and service ids (record lane L holds
    // dword L, so each list entry is stored by the lane that holds it)
    {
      uint32_t* row = L_cl + (size_t)slot * KSG_CL_W;
      const uint32_t kt = lane - WS_IDS, st_ = lane - (WS_IDS + nk + n_sel);
      if (kt < nk) row[KSG_CL_KEY + base_nk + kt] = rec;
      if (st_ < n_svcs) row[KSG_CL_SV + base_ns + st_] = rec;
    }
    if (lane == 0) {
      // (the record's 16 bytes only: the drawn node next to it is the x-checker's)
      *reinterpret_cast<uint4*>(&L_cm[i]) =
          uint4{1u, slot, woff, (in_c ? 0u : 1u) | (cidx << 1) | (n_svcs << 8) | (base_ns << 16) | (base_nk << 24)};
      L_cm[i].out = (int32_t)wn;
      st_post(&ctl->sel_seq, i + 1);  // the checkers move on
    }
    if ((int32_t)woff != pred) KSG_COUNTP(8, 64)
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
    x_fresh = !in_c;
    ++n_draws;
    KSG_STAMPP(5)
  }
  if (lane == 0) {
    ctl->resolved = resolved;
    st_rel(&ctl->stop, 1u);
  }
  // the checkers apply the last commits and write their slots back; the
  // x-checker records the last first peers
  bool drained = false;
  for (uint32_t spin = 0; spin <= 16 * KSG_SPIN_LIMIT; ++spin) {
    bool done = ld_acq(&ctl->fin_x) != 0 && ld_acq(&ctl->fin_f) != 0;
#pragma unroll
    for (int c = 0; c < KSG_RES_NCHK; ++c) done = done && ld_acq(&ctl->fin[c]) != 0;
    if (done) {
      drained = true;
      break;
    }
  }
  if (ld_acq(&ctl->bad)) reason = KSG_STOP_BAD;
  else if (!drained || ld_acq(&ctl->hang)) reason = KSG_STOP_HANG;
  if constexpr (STAMP) {
    if (d.dbgbuf && (lane < 16 || lane == 43 || lane == 44)) atomicAdd(d.dbgbuf + lane, (int32_t)(t_acc / 64));
  }
#undef KSG_STAMPP
#undef KSG_COUNTP
  const uint32_t n_peer = __builtin_amdgcn_readfirstlane(ctl->n_peer);
  for (uint32_t t = lane; t < n_peer; t += 64) {
    const uint32_t sv = L_peer[2 * t];
    int32_t expect = -1;
    __hip_atomic_compare_exchange_strong(d.svc_peer + sv, &expect, (int32_t)L_peer[2 * t + 1], __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (uint32_t t = lane; t < resolved; t += 64) out[t] = L_cm[t].out;
  if (esc && x.tmax) {  // (extension scores) the TaintToleration maxima and histograms start at 0 for the next window
    for (uint32_t t = lane; t < wcap; t += 64) x.tmax[t] = 0;
    for (uint32_t t = lane; t < n_pods * KSG_TBINS; t += 64) x.thist[t] = 0;
  }
  if (XS) {
    // (extensions) the window's extended resource requests into the node state
    // (the checkers wrote cpu / memory back; these live in no slot)
    for (uint32_t t = lane; t < resolved; t += 64) {
      if (L_cm[t].kind != 1) continue;
      const ksg_pod_ext& pe = x.exts[pos + t];
      const uint32_t wn = d.lo + L_cm[t].node;
      for (uint32_t r = 0; r < d.n_scalar; ++r)
        if (pe.scalar[r] != 0)
          __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(d.scalar_used + (size_t)r * d.n_nodes + wn),
                                 (uint64_t)pe.scalar[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    drain_stores();
  }
  if (lane == 0) {
    *rng_io = rng0 + (uint64_t)n_draws * ksg_rng_step(d.draws);
    if constexpr (STAMP && FUSED)  // (the scoring blocks' stamp base, a mailbox, not a counter)
      if (d.dbgbuf) __hip_atomic_store(d.dbgbuf + 55, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    KsgWinRun r = *run;
    if (reason == KSG_STOP_HANG) {
      r.halt = KSG_HALT_HANG;
    } else if (reason == KSG_STOP_BAD) {
      r.halt = KSG_HALT_BAD;
    } else if (reason == KSG_STOP_OVERSIZE) {
      r.halt = KSG_HALT_OVERSIZE;  // pod pos: the host runs the exact per-pod path, then resumes
    } else if (resolved == 0 || resolved > n_pods) {
      r.halt = KSG_HALT_BADCOUNT;
    } else {
      r.pos = pos + resolved;
      r.windows += 1;
      // (constant indices: a dynamic one puts r in scratch, and the compiler then budgets the
      // whole kernel's registers for a higher occupancy it never gets: config 5 -4 %)
      r.stops[1] += reason == 1 ? 1u : 0u;
      r.stops[2] += reason == 2 ? 1u : 0u;
      r.stops[3] += reason == 3 ? 1u : 0u;
    }
    *run_out = r;
  }
}

template <int P, bool STAMP, bool XS>
__global__ __launch_bounds__(pl_nt(P)) void ksg_win_plain_kernel(KsgDev d, uint32_t wcap, KsgWinRun* run,
                                                            const KsgWinSum* __restrict__ sums, const KsgWinXchg x,
                                                            uint64_t* rng_io, int32_t* __restrict__ out_batch) {
  win_plain_body<P, STAMP, XS, false>(d, wcap, run, sums, x, rng_io, out_batch, KsgFused{});
}

template <int P, bool STAMP>
__global__ __launch_bounds__(pl_nt(P)) void ksg_win_fused_kernel(KsgDev d, uint32_t wcap, KsgWinRun* run,
                                                            const KsgWinSum* __restrict__ sums, const KsgWinXchg x,
                                                            uint64_t* rng_io, int32_t* __restrict__ out_batch,
                                                            const KsgFused f) {
  win_plain_body<P, STAMP, false, true>(d, wcap, run, sums, x, rng_io, out_batch, f);
}

// ---------------------------------------------------------------------------
// host launcher
// ---------------------------------------------------------------------------
// The plain resolver past 512 words per shard (P = 16, 32: config 5's 100,000 nodes) and the
// extension (XS) resolvers are instantiated in their own translation unit, ksg_plain_large.hip,
// which includes this file with KSG_PLAIN_LARGE_TU and is compiled with the max-ILP machine
// scheduler: its default schedule
// holds the P = 32 production resolver to 137 VGPRs (3 waves per SIMD, an occupancy the LDS never
// allows) and measured 3.5 % slower at config 5 than with 181 (same box, profiles/r6_ab_trees.json
// ab5); the fused and small-shard kernels keep the default schedule (config 2: -1 % under max-ILP).
template <int PP, bool ST, bool XS, bool FU = false>
static hipError_t win_plain_launch_x(const KsgDev& d, uint32_t wcap, size_t lds, KsgWinRun* run,
                                     const KsgWinSum* sums, const KsgWinXchg& x, uint64_t* rng, int32_t* out,
                                     hipStream_t st, const KsgFused& f = KsgFused{}, uint32_t grid = 1) {
  // (each branch names only its own kernel: a kernel template instantiated in both translation
  // units would be registered twice, with two schedules)
  const void* fn;
  if constexpr (FU) fn = reinterpret_cast<const void*>(ksg_win_fused_kernel<PP, ST>);
  else fn = reinterpret_cast<const void*>(ksg_win_plain_kernel<PP, ST, XS>);
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();  // do not leave a sticky error behind
    once = true;
  }
  if constexpr (FU)
    hipLaunchKernelGGL((ksg_win_fused_kernel<PP, ST>), dim3(grid), dim3(pl_nt(PP)), lds, st, d, wcap, run, sums, x,
                       rng, out, f);
  else
    hipLaunchKernelGGL((ksg_win_plain_kernel<PP, ST, XS>), dim3(grid), dim3(pl_nt(PP)), lds, st, d, wcap, run, sums,
                       x, rng, out);
  return hipGetLastError();
}

// (extensions) extended resources / extension scores re-checked on the slots: the XS instantiation
static bool plain_xs(const KsgDev& d, const KsgWinXchg& x) {
  return x.exts != nullptr && (((d.ext_filters & KSG_EXT_SCALAR) && d.n_scalar > 0) || x.esc);
}

// the debug instantiation: KSG_DEBUG & 8 (per-section s_memtime stamps), bits 16..19 (skews) or
// 24..27 (timing switches); the production one keeps no debug switch in a register. Bits 22 / 23
// (the runtime's request-corruption hook for the resident server's rejection test) and every
// other bit keep the production resolver: a fault-injection switch never changes which resolver
// build runs
static bool plain_stamp(const KsgDev& d) { return (d.dbg & 8) != 0 || ((uint32_t)d.dbg & KSG_DBG_RESOLVER_MASK) != 0; }

#define KSG_PLAIN_CASE(PP, XS)                                                                              \
  if (P == PP)                                                                                              \
    return plain_stamp(d) ? win_plain_launch_x<PP, true, XS>(d, wcap, lds, run, sums, x, rng, out, st)    \
                          : win_plain_launch_x<PP, false, XS>(d, wcap, lds, run, sums, x, rng, out, st);

// the max-ILP translation unit's share: P = 16, 32, and the extension (XS) resolvers at every P
// (config 2 + every extension: 230k -> 235k pods/s under max-ILP, same box, profiles/r6_ab_trees.json ab7)
hipError_t ksg_launch_win_plain_ilp(const KsgDev& d, uint32_t P, uint32_t wcap, size_t lds, KsgWinRun* run,
                                    const KsgWinSum* sums, const KsgWinXchg& x, uint64_t* rng, int32_t* out,
                                    hipStream_t st)
#ifdef KSG_PLAIN_LARGE_TU
{
  if (plain_xs(d, x)) {
    KSG_PLAIN_CASE(1, true)
    KSG_PLAIN_CASE(2, true)
    KSG_PLAIN_CASE(4, true)
    KSG_PLAIN_CASE(8, true)
    KSG_PLAIN_CASE(16, true)
    KSG_PLAIN_CASE(32, true)
  } else {
    KSG_PLAIN_CASE(16, false)
    KSG_PLAIN_CASE(32, false)
  }
  return hipErrorInvalidValue;
}
#else
    ;  // (ksg_plain_large.hip)

static uint32_t plain_P(const KsgDev& d);
uint32_t ksg_win_plain_lds(const KsgDev& d, uint32_t wcap) {
  return plain_lds_offsets(plain_P(d), (d.n_services + 31) / 32, wcap).total;
}

static uint32_t plain_P(const KsgDev& d) {
  const uint32_t P = (d.nwords + 63) / 64;
  return P <= 1 ? 1 : P <= 2 ? 2 : P <= 4 ? 4 : P <= 8 ? 8 : P <= 16 ? 16 : 32;
}

uint32_t ksg_win_t0_stride(const KsgDev& d) { return t0img_stride(plain_P(d)); }

// the window's T0 images (x.img), after phase A (and its all-gather)
hipError_t ksg_launch_win_t0(const KsgDev& d, uint32_t wcap, const KsgWinRun* run, const KsgWinXchg& x,
                             hipStream_t st) {
  const uint32_t P = plain_P(d);
#define KSG_T0_CASE(PP) \
  if (P == PP) hipLaunchKernelGGL((ksg_win_t0_kernel<PP>), dim3(wcap), dim3(256), 0, st, d.nwords, wcap, run, x);
  KSG_T0_CASE(1)
  KSG_T0_CASE(2)
  KSG_T0_CASE(4)
  KSG_T0_CASE(8)
  KSG_T0_CASE(16)
  KSG_T0_CASE(32)
#undef KSG_T0_CASE
  return hipGetLastError();
}

hipError_t ksg_launch_win_plain(const KsgDev& d, uint32_t P, uint32_t wcap, KsgWinRun* run, const KsgWinSum* sums,
                                const KsgWinXchg& x, uint64_t* rng, int32_t* out, hipStream_t st) {
  const size_t lds = plain_lds_offsets(P, (d.n_services + 31) / 32, wcap).total;
  if (P >= 16 || plain_xs(d, x)) return ksg_launch_win_plain_ilp(d, P, wcap, lds, run, sums, x, rng, out, st);
  KSG_PLAIN_CASE(1, false)
  KSG_PLAIN_CASE(2, false)
  KSG_PLAIN_CASE(4, false)
  KSG_PLAIN_CASE(8, false)
  return hipErrorInvalidValue;
}

// the fused window launch (KsgFused): block 0 resolves, blocks 1 .. grid-1 score the window
// (no ServiceAntiAffinity, no extensions, one rank); run = this launch's slot
bool ksg_win_fused_ok(const KsgDev& d) { return plain_P(d) >= 1 && d.nwords > 0; }

uint32_t ksg_win_fused_groups(const KsgDev& d, uint32_t wcap) {
  const uint32_t pg = (uint32_t)pl_pg((int)plain_P(d));
  return (wcap + pg - 1) / pg;
}

hipError_t ksg_launch_win_fused(const KsgDev& d, uint32_t wcap, KsgWinRun* run, const KsgWinSum* sums,
                                const KsgWinXchg& x, uint64_t* rng, int32_t* out, const KsgFused& f, uint32_t grid,
                                hipStream_t st) {
  const uint32_t P = plain_P(d);
  // (the scoring blocks stage their pods' records in LDS: waves x pods x 192 B)
  const size_t lds = std::max<size_t>(plain_lds_offsets(P, (d.n_services + 31) / 32, wcap).total,
                                      (size_t)(pl_nt(P) / 64) * pl_pg((int)P) * sizeof(KsgWinSum));
  const bool stamp = plain_stamp(d);
#define KSG_FUSED_CASE(PP)                                                                                  \
  if (P == PP)                                                                                              \
    return stamp ? win_plain_launch_x<PP, true, false, true>(d, wcap, lds, run, sums, x, rng, out, st, f, grid) \
                 : win_plain_launch_x<PP, false, false, true>(d, wcap, lds, run, sums, x, rng, out, st, f, grid);
  KSG_FUSED_CASE(1)
  KSG_FUSED_CASE(2)
  KSG_FUSED_CASE(4)
  KSG_FUSED_CASE(8)
  KSG_FUSED_CASE(16)
  KSG_FUSED_CASE(32)
#undef KSG_FUSED_CASE
  return hipErrorInvalidValue;
}
#endif  // KSG_PLAIN_LARGE_TU
#undef KSG_PLAIN_CASE
