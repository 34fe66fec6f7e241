// ksg_exact.h — the exact one-pod-at-a-time building blocks shared by the
// persistent batch kernel, the single-pod scan (ksg_kernels.hip) and the
// resident drop-in server (ksg_serve.hip): one workgroup of KSG_NT threads,
// thread t owns nodes lo + j*KSG_NT + t (j < R), per-node scores in LDS (or HBM
// scratch past KSG_R_LDS), the block max + tie ballots, and the ix-th tie.
#pragma once
#include <hip/hip_runtime.h>
#include "ksg_internal.h"

#include "ksg_device.h"

// Combined-score type SC: int32 while every |score| stays below
// KSG_SCORE_BOUND; int64 wrapping like Go's int otherwise (KsgDev.wide: weights
// the reference accepts up to int64, generic_scheduler.go:145-159).
template <typename SC>
struct ScoreT;
template <>
struct ScoreT<int32_t> {
  static constexpr int32_t none = KSG_S32_NONE;
  static constexpr int r_lds = KSG_R_LDS;  // nodes per thread whose scores fit the LDS
  static __device__ __forceinline__ int32_t wave_max(int32_t v) { return wave_max_i32(v); }
  static __device__ __forceinline__ int32_t add(int32_t a, int64_t b) { return a + (int32_t)b; }
};
template <>
struct ScoreT<int64_t> {
  static constexpr int64_t none = KSG_SCORE_NONE;
  static constexpr int r_lds = KSG_R_LDS / 2;
  static __device__ __forceinline__ int64_t wave_max(int64_t v) { return wave_max_i64(v); }
  static __device__ __forceinline__ int64_t add(int64_t a, int64_t b) { return wsum(a, b); }
};

// Filter + score every node of the shard into s_score; returns this thread's max.
// With ANTI the ServiceAntiAffinity term is added after the domain counts are
// complete (one extra barrier).
// UNR: unroll the node loop by up to 4 (the loads of 4 nodes in flight
// together) without the register-cached totals
template <int R, bool ANTI, bool REG, typename SC, bool UNR = REG>
__device__ __forceinline__ SC scan_pod(const KsgDev& d, const PodCtx& c, uint32_t tid, uint32_t wave,
                                       uint64_t bit, SC* s_score, int32_t* s_dcount,
                                       const int32_t* dglobal, const int64_t* rcapc, const int64_t* rcapm,
                                       const int64_t* rusedc, const int64_t* rusedm,
                                       uint8_t* fail_out, int32_t* s_tmax = nullptr) {
  using T = ScoreT<SC>;
  const bool need_cnt = (d.w_spread != 0 || ANTI) && c.svc >= 0;
  // extension TaintTolerationPriority: normalised by the max over the filtered
  // nodes, so it is added in a second pass like the anti-affinity term
  // (s_tmax: zeroed by the caller before the barrier that precedes this scan)
  const bool tt = d.w_taint != 0 && c.ext != nullptr && s_tmax != nullptr && !d.equal_fallback;
  int32_t tmax = 0;
  SC m = T::none;
  // register-cached node state needs compile-time j; otherwise keep the loop rolled
  constexpr int kUnroll = REG ? R : UNR ? (R < 4 ? R : 4) : 1;
#pragma unroll kUnroll
  for (int j = 0; j < R; ++j) {
    const uint32_t n = d.lo + j * KSG_NT + tid;
    const uint32_t wi = (d.lo >> 6) + j * KSG_NWAVE + wave;
    SC sc = T::none;
    if (n < d.hi) {
      int64_t capc, capm, usedc, usedm;
      if constexpr (REG) {
        capc = rcapc[j]; capm = rcapm[j]; usedc = rusedc[j]; usedm = rusedm[j];
      } else {
        capc = d.cap_cpu[n]; capm = d.cap_mem[n];
        usedc = ld_mut(d.used_cpu + n); usedm = ld_mut(d.used_mem + n);
      }
      const int32_t cnt = need_cnt ? ld_mut(d.svc_cnt + (size_t)c.svc * d.n_nodes + n) : 0;
      const int f = node_fail(d, c, n, wi, bit, capc, capm, usedc, usedm);
      if (fail_out) fail_out[n - d.lo] = (uint8_t)f;
      if (f == KSG_FAIL_NONE) {
        sc = (SC)node_score(d, c, n, capc, capm, usedc, usedm, cnt);
        if (tt) tmax = max(tmax, soft_taints(d, c, wi, bit));
        if (ANTI && s_dcount && cnt != 0) {
          for (uint32_t a = 0; a < d.n_anti; ++a) {
            const int32_t dom = d.anti_domain[(size_t)a * d.n_nodes + n];
            if (dom >= 0) atomicAdd(&s_dcount[d.anti_dom_off[a] + dom], cnt);
          }
        }
      }
    }
    s_score[j * KSG_NT + tid] = sc;
    if (!ANTI && !tt) m = sc > m ? sc : m;
  }
  if (ANTI || tt) {
    if (tt) {
      tmax = wave_max_i32(tmax);
      if ((tid & 63) == 0) atomicMax(s_tmax, tmax);
    }
    __syncthreads();
    const int32_t* dc = dglobal ? dglobal : s_dcount;
    // (sharded: the all-reduced max over every shard's filtered nodes, after the domain counts)
    const int32_t tm = tt ? (dglobal ? dglobal[d.n_domains_total] : *s_tmax) : 0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      SC v = s_score[j * KSG_NT + tid];
      if (v != T::none && !d.equal_fallback) {
        if (ANTI) v = T::add(v, anti_term(d, c, d.lo + j * KSG_NT + tid, dc));
        if (tt) {
          const uint32_t wi = (d.lo >> 6) + j * KSG_NWAVE + wave;
          v = T::add(v, (int64_t)d.w_taint * taint_score(soft_taints(d, c, wi, bit), tm));
        }
        s_score[j * KSG_NT + tid] = v;
      }
      m = v > m ? v : m;
    }
  }
  return m;
}

// Block max of the per-thread maxima, then tie ballots into s_tie and the tie count.
template <int R, typename SC>
__device__ __forceinline__ void reduce_ties(const KsgDev& d, SC m, uint32_t tid, uint32_t lane, uint32_t wave,
                                            const SC* s_score, SC* s_wmax, uint32_t* s_wcnt,
                                            uint64_t* s_tie, SC& M, uint64_t& k) {
  using T = ScoreT<SC>;
  m = T::wave_max(m);
  if (lane == 0) s_wmax[wave] = m;
  __syncthreads();
  M = s_wmax[0];
#pragma unroll
  for (int w = 1; w < KSG_NWAVE; ++w) M = s_wmax[w] > M ? s_wmax[w] : M;
  if (d.empty_priorities) M = T::none;  // all weights 0: empty HostPriorityList
  uint32_t wc = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint64_t b = __ballot(M != T::none && s_score[j * KSG_NT + tid] == M);
    if (lane == 0) s_tie[j * KSG_NWAVE + wave] = b;
    wc += __popcll(b);
  }
  if (lane == 0) s_wcnt[wave] = wc;
  __syncthreads();
  k = 0;
#pragma unroll
  for (int w = 0; w < KSG_NWAVE; ++w) k += s_wcnt[w];
}

// wave 0: rank of the target-th (ascending) set bit over nwords tie words
__device__ __forceinline__ int32_t select_tie(const uint64_t* words, uint32_t nwords, uint64_t target,
                                              uint32_t lane, uint32_t base_node) {
  uint64_t acc = 0;
  for (uint32_t base = 0; base < nwords; base += 64) {
    const uint32_t widx = base + lane;
    const uint64_t w = widx < nwords ? words[widx] : 0ULL;
    const uint32_t cnt = __popcll(w);
    const uint32_t incl = wave_incl_scan_u32(cnt, lane);
    const uint32_t tot = __shfl(incl, 63, 64);
    if (target < acc + tot) {
      const uint32_t excl = incl - cnt;
      int32_t cand = -1;
      if (acc + excl <= target && target < acc + incl)
        cand = (int32_t)(base_node + widx * 64 + select_bit(w, (uint32_t)(target - acc - excl)));
      const uint64_t own = __ballot(cand >= 0);
      return __shfl(cand, (int)__builtin_ctzll(own), 64);
    }
    acc += tot;
  }
  return -1;
}
