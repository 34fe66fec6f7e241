// ksg_kernels.hip — CDNA4 (gfx950) kernels for the kube-scheduler Filter/Score pass.
//
// Reference algorithm (smarterclayton/kubernetes v0.13.0-dev, /root/reference):
//   genericScheduler.Schedule        pkg/scheduler/generic_scheduler.go:54-80
//   findNodesThatFit                 pkg/scheduler/generic_scheduler.go:100-128
//   prioritizeNodes                  pkg/scheduler/generic_scheduler.go:136-165
//   selectHost/getBestHosts          pkg/scheduler/generic_scheduler.go:84-96,167-177
//   predicates                       pkg/scheduler/predicates.go:52-350
//   LeastRequestedPriority           pkg/scheduler/priorities.go:27-91
//   ServiceSpread / AntiAffinity     pkg/scheduler/spreading.go:37-168
//   AssumePod (commit)               plugin/pkg/scheduler/scheduler.go:115-118
//
// Design: one workgroup of 1024 threads (16 waves) scans the node
// shard for a pod; node n = lo + j*1024 + tid, so every wave covers 64 consecutive
// node ranks per step j and each bitmap (ports/PDs in use, label pairs, static
// fit) is read as ONE uint64 word per wave. Filter results become wave ballots
// (the tie words), the argmax is a wave DPP max + 16-entry LDS max, and the
// reference's random tie pick "ix-th host in descending name order" is a popcount
// prefix scan over the tie words. The persistent batch kernel then commits the
// winner (AssumePod's delta) in HBM and moves on to the next pod without
// returning to the host. No MFMA: the pass is integer compare/bit work.
#include <hip/hip_runtime.h>
#include "ksg_internal.h"

#define LR_FAST_CAP (0x7fffffffffffffffLL / 16)

// ---- memory helpers -------------------------------------------------------
// Mutable state (used, keymap, svc_*) is written by the committing lane and
// re-read by every wave for the next pod: load/store it at agent scope (L1
// bypass, L2 coherent) so no stale vector-L1 or scalar-cache copy is read.
template <typename T>
__device__ __forceinline__ T ld_mut(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_mut(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- Go-exact arithmetic ----------------------------------------------------
__device__ __forceinline__ int64_t go_div64(int64_t a, int64_t b) {
  if (b == -1) return (int64_t)(0ULL - (uint64_t)a);  // Go wraps MinInt64/-1
  return a / b;                                       // truncation toward zero
}

// calculateScore (priorities.go:27-37):
//   cap==0 -> 0; requested>cap -> 0; else int(((cap-requested)*10)/cap)
// with Go's wrapping int64 multiply. Fast path: 0 <= x=cap-req <= cap <= 2^59,
// q = floor(10x/cap) in [0,10] found by an exact 4-step binary search on
// t*cap <= 10x (no divide instruction sequence, no overflow).
__device__ __forceinline__ int64_t lr_calc(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  const uint64_t x = (uint64_t)capacity - (uint64_t)requested;
  if (capacity > 0 && capacity <= LR_FAST_CAP && requested >= 0) {
    const int64_t y = (int64_t)(x * 10ULL);
    int64_t q = 0;
#pragma unroll
    for (int b = 8; b >= 1; b >>= 1) {
      const int64_t t = q + b;
      if (t <= 10 && t * capacity <= y) q = t;
    }
    return q;
  }
  return go_div64((int64_t)(x * 10ULL), capacity);
}

// int(10 * (float32(num) / float32(den))) with IEEE f32 divide and multiply,
// no contraction (spreading.go:79-83, 156-160).
__device__ __forceinline__ int64_t frac10_f32(int64_t num, int64_t den) {
  const float q = __fdiv_rn((float)num, (float)den);
  const float s = __fmul_rn(10.0f, q);
  return (int64_t)s;
}

__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int64_t o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(v, off, 64);
    if (lane >= (uint32_t)off) v += o;
  }
  return v;
}

// position of the m-th (0-based) set bit of w, ascending
__device__ __forceinline__ uint32_t select_bit(uint64_t w, uint32_t m) {
  uint32_t pos = 0;
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) {
    const uint64_t lowmask = (sh == 64) ? ~0ULL : ((1ULL << sh) - 1);
    const uint32_t c = __popcll(w & lowmask);
    if (m >= c) {
      m -= c;
      w >>= sh;
      pos += sh;
    }
  }
  return pos;
}

// ---- per-pod context (wave-uniform) --------------------------------------
struct PodCtx {
  int64_t req_cpu, req_mem;
  int32_t zero_req;
  int32_t host;
  int32_t svc;
  int32_t spread_max;
  int32_t svc_total;
  int32_t error;
  uint32_t n_ports, n_pds, n_sel;
  const uint32_t* ports;
  const uint32_t* pds;
  const uint32_t* sel;
  int32_t req_aff[KSG_MAX_AFF];
};

__device__ __forceinline__ void pod_resolve(const KsgDev& d, const ksg_pod& p, const uint32_t* ids,
                                            PodCtx& c) {
  c.req_cpu = p.milli_cpu;
  c.req_mem = p.memory;
  c.zero_req = (p.milli_cpu == 0 && p.memory == 0);  // predicates.go:129-132
  c.host = p.host;
  c.svc = p.service;
  c.ports = ids + p.ports_off;
  c.n_ports = p.n_ports;
  c.pds = ids + p.pds_off;
  c.n_pds = p.n_pds;
  c.sel = ids + p.sel_off;
  c.n_sel = p.n_sel;
  c.error = 0;
  c.spread_max = 0;
  c.svc_total = 0;
  int32_t peer = -1;
  if (c.svc >= 0) {
    c.spread_max = ld_mut(d.svc_max + c.svc);
    c.svc_total = ld_mut(d.svc_total + c.svc);
    peer = ld_mut(d.svc_peer + c.svc);
  }
  // ServiceAffinity (predicates.go:257-324): labels the pod's nodeSelector does
  // not give come from the node of the first service peer.
  for (uint32_t j = 0; j < KSG_MAX_AFF; ++j) c.req_aff[j] = -1;
  if (d.preds & KSG_PRED_SERVICEAFFINITY) {
    bool all_given = true;
    for (uint32_t j = 0; j < d.n_aff; ++j) {
      c.req_aff[j] = p.aff_pair[j];
      if (p.aff_pair[j] < 0) all_given = false;
    }
    if (!all_given && peer != -1) {
      if (peer == -2) {
        c.error = 1;  // GetNodeInfo of the peer's host fails (predicates.go:293-296)
      } else {
        for (uint32_t j = 0; j < d.n_aff; ++j)
          if (c.req_aff[j] < 0) c.req_aff[j] = d.aff_pair[(size_t)j * d.n_nodes + peer];
      }
    }
  }
}

// Filter: first failing predicate (fixed order) or 0. wi/bit locate node n in
// the bitmaps; wi is wave-uniform.
__device__ __forceinline__ int node_fail(const KsgDev& d, const PodCtx& c, uint32_t n, uint32_t wi,
                                         uint64_t bit, int64_t capc, int64_t capm, int64_t usedc,
                                         int64_t usedm) {
  const uint32_t P = d.preds;
  if ((P & KSG_PRED_HOSTNAME) && c.host != -1 && (int32_t)n != c.host) return KSG_FAIL_HOSTNAME;
  if (d.has_static_fit && !(d.static_fit[wi] & bit)) return KSG_FAIL_LABELSPRESENCE;
  if (P & KSG_PRED_MATCHNODESELECTOR) {
    for (uint32_t i = 0; i < c.n_sel; ++i)
      if (!(d.pairmap[(size_t)c.sel[i] * d.nw + wi] & bit)) return KSG_FAIL_MATCHNODESELECTOR;
  }
  if (P & KSG_PRED_NODISKCONFLICT) {
    for (uint32_t i = 0; i < c.n_pds; ++i)
      if (ld_mut(d.keymap + (size_t)c.pds[i] * d.nw + wi) & bit) return KSG_FAIL_NODISKCONFLICT;
  }
  if (P & KSG_PRED_PODFITSPORTS) {
    for (uint32_t i = 0; i < c.n_ports; ++i)
      if (ld_mut(d.keymap + (size_t)c.ports[i] * d.nw + wi) & bit) return KSG_FAIL_PODFITSPORTS;
  }
  if ((P & KSG_PRED_PODFITSRESOURCES) && !c.zero_req) {
    // CheckPodsExceedingCapacity (predicates.go:104-124) over existing+pod, in
    // closed form: every pod fits greedily iff cap==0 || cap - sum(existing) >= req.
    const bool fc = capc == 0 || (int64_t)((uint64_t)capc - (uint64_t)usedc) >= c.req_cpu;
    const bool fm = capm == 0 || (int64_t)((uint64_t)capm - (uint64_t)usedm) >= c.req_mem;
    if (!(fc && fm)) return KSG_FAIL_PODFITSRESOURCES;
  }
  if (P & KSG_PRED_SERVICEAFFINITY) {
    for (uint32_t j = 0; j < d.n_aff; ++j)
      if (c.req_aff[j] >= 0 && !(d.pairmap[(size_t)c.req_aff[j] * d.nw + wi] & bit))
        return KSG_FAIL_SERVICEAFFINITY;
  }
  return KSG_FAIL_NONE;
}

// Priorities without ServiceAntiAffinity (added after the domain counts).
__device__ __forceinline__ int64_t node_score(const KsgDev& d, const PodCtx& c, uint32_t n,
                                              int64_t capc, int64_t capm, int64_t usedc,
                                              int64_t usedm, int32_t cnt) {
  if (d.equal_fallback) return 1;  // EqualPriority (generic_scheduler.go:141-143,180-195)
  int64_t s = 0;
  if (d.has_static_score) s += d.static_score[n];
  if (d.w_lr) {  // calculateOccupancy (priorities.go:43-76): all pods on node + this pod
    const int64_t tc = (int64_t)((uint64_t)usedc + (uint64_t)c.req_cpu);
    const int64_t tm = (int64_t)((uint64_t)usedm + (uint64_t)c.req_mem);
    s += (int64_t)d.w_lr * ((lr_calc(tc, capc) + lr_calc(tm, capm)) / 2);
  }
  if (d.w_spread) {  // CalculateSpreadPriority (spreading.go:72-86)
    const int64_t sc = c.spread_max > 0 ? frac10_f32((int64_t)c.spread_max - cnt, c.spread_max) : 10;
    s += (int64_t)d.w_spread * sc;
  }
  return s;
}

__device__ __forceinline__ int64_t anti_term(const KsgDev& d, const PodCtx& c, uint32_t n,
                                             const int32_t* dcount) {
  int64_t s = 0;
  for (uint32_t a = 0; a < d.n_anti; ++a) {
    const int32_t dom = d.anti_domain[(size_t)a * d.n_nodes + n];
    int64_t sc = 0;  // unlabeled nodes score 0 (spreading.go:164-166)
    if (dom >= 0) {
      const int64_t tot = c.svc_total;
      sc = tot > 0 ? frac10_f32(tot - dcount[d.anti_dom_off[a] + dom], tot) : 10;
    }
    s += (int64_t)d.w_anti[a] * sc;
  }
  return s;
}

// AssumePod delta (plugin/pkg/scheduler/scheduler.go:115-118 -> modeler.go:77-79):
// the pod now counts on node w for resources, ports, PDs and service counts.
__device__ void commit_pod(const KsgDev& d, const ksg_pod& p, const uint32_t* ids, uint32_t w) {
  st_mut(d.used_cpu + w, (int64_t)((uint64_t)ld_mut(d.used_cpu + w) + (uint64_t)p.milli_cpu));
  st_mut(d.used_mem + w, (int64_t)((uint64_t)ld_mut(d.used_mem + w) + (uint64_t)p.memory));
  const uint64_t bit = 1ULL << (w & 63);
  const size_t wi = w >> 6;
  for (uint32_t i = 0; i < p.n_ports; ++i) {
    uint64_t* a = d.keymap + (size_t)ids[p.ports_off + i] * d.nw + wi;
    st_mut(a, ld_mut(a) | bit);
  }
  for (uint32_t i = 0; i < p.n_pds; ++i) {
    uint64_t* a = d.keymap + (size_t)ids[p.pds_off + i] * d.nw + wi;
    st_mut(a, ld_mut(a) | bit);
  }
  for (uint32_t i = 0; i < p.n_svcs; ++i) {
    const uint32_t s = ids[p.svcs_off + i];
    int32_t* ca = d.svc_cnt + (size_t)s * d.n_nodes + w;
    const int32_t cnt = ld_mut(ca) + 1;
    st_mut(ca, cnt);
    if (cnt > ld_mut(d.svc_max + s)) st_mut(d.svc_max + s, cnt);
    st_mut(d.svc_total + s, ld_mut(d.svc_total + s) + 1);
    if (ld_mut(d.svc_peer + s) == -1) st_mut(d.svc_peer + s, (int32_t)w);
  }
}

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ============================================================================
// Persistent batch kernel (single GPU): schedules pods[0..n) in order. One
// workgroup of 1024 threads; thread t owns nodes lo + j*1024 + t (j < R). With
// REG, capacity and requested totals live in registers for the whole batch
// (only the winner's owner lane updates them), so the per-pod scan reads only
// the per-pod service counts and one bitmap word per wave per key from memory.
// ============================================================================
template <int R, bool ANTI, bool REG>
__global__ __launch_bounds__(KSG_NT) void ksg_batch_kernel(KsgDev d, const ksg_pod* __restrict__ pods,
                                                          const uint32_t* __restrict__ ids,
                                                          uint32_t n_pods, uint64_t* rng_io,
                                                          int32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int32_t* s_dcount = reinterpret_cast<int32_t*>(smem);
  __shared__ uint64_t s_tie[R * KSG_NWAVE];
  __shared__ int64_t s_wmax[KSG_NWAVE];
  __shared__ uint32_t s_wcnt[KSG_NWAVE];
  __shared__ int32_t s_winner;

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t bit = 1ULL << lane;
  uint64_t rng = *rng_io;

  int64_t rcapc[REG ? R : 1], rcapm[REG ? R : 1], rusedc[REG ? R : 1], rusedm[REG ? R : 1];
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
  const bool need_cnt = d.w_spread != 0 || ANTI;

  for (uint32_t i = 0; i < n_pods; ++i) {
    const ksg_pod& p = pods[i];
    PodCtx c;
    pod_resolve(d, p, ids, c);
    if (c.error) {
      if (tid == 0) out[i] = KSG_OUT_ERROR;
      continue;  // uniform; no barrier-protected LDS was touched for this pod
    }
    if (ANTI) {
      for (uint32_t k = tid; k < d.n_domains_total; k += KSG_NT) s_dcount[k] = 0;
      __syncthreads();
    }
    int64_t sc[R];
    bool fit[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t n = d.lo + j * KSG_NT + tid;
      const uint32_t wi = (d.lo >> 6) + j * KSG_NWAVE + wave;
      const bool valid = n < d.hi;
      int64_t capc, capm, usedc, usedm;
      if constexpr (REG) {
        capc = rcapc[j]; capm = rcapm[j]; usedc = rusedc[j]; usedm = rusedm[j];
      } else {
        capc = valid ? d.cap_cpu[n] : 0;
        capm = valid ? d.cap_mem[n] : 0;
        usedc = valid ? ld_mut(d.used_cpu + n) : 0;
        usedm = valid ? ld_mut(d.used_mem + n) : 0;
      }
      int32_t cnt = 0;
      if (need_cnt && c.svc >= 0 && valid) cnt = ld_mut(d.svc_cnt + (size_t)c.svc * d.n_nodes + n);
      const int f = valid ? node_fail(d, c, n, wi, bit, capc, capm, usedc, usedm) : -1;
      fit[j] = (f == KSG_FAIL_NONE);
      sc[j] = fit[j] ? node_score(d, c, n, capc, capm, usedc, usedm, cnt) : KSG_SCORE_NONE;
      if (ANTI && fit[j] && cnt != 0) {
        for (uint32_t a = 0; a < d.n_anti; ++a) {
          const int32_t dom = d.anti_domain[(size_t)a * d.n_nodes + n];
          if (dom >= 0) atomicAdd(&s_dcount[d.anti_dom_off[a] + dom], cnt);
        }
      }
    }
    if (ANTI) {
      __syncthreads();
      if (!d.equal_fallback) {
#pragma unroll
        for (int j = 0; j < R; ++j)
          if (fit[j]) sc[j] += anti_term(d, c, d.lo + j * KSG_NT + tid, s_dcount);
      }
    }
    int64_t m = KSG_SCORE_NONE;
#pragma unroll
    for (int j = 0; j < R; ++j) m = sc[j] > m ? sc[j] : m;
    m = wave_max_i64(m);
    if (lane == 0) s_wmax[wave] = m;
    __syncthreads();
    int64_t M = s_wmax[0];
#pragma unroll
    for (int w = 1; w < KSG_NWAVE; ++w) M = s_wmax[w] > M ? s_wmax[w] : M;
    uint32_t wc = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint64_t b = __ballot(fit[j] && sc[j] == M);
      if (lane == 0) s_tie[j * KSG_NWAVE + wave] = b;
      wc += __popcll(b);
    }
    if (lane == 0) s_wcnt[wave] = wc;
    __syncthreads();
    uint64_t k = 0;
#pragma unroll
    for (int w = 0; w < KSG_NWAVE; ++w) k += s_wcnt[w];
    if (M == KSG_SCORE_NONE || k == 0 || d.empty_priorities) {
      if (tid == 0) out[i] = KSG_OUT_NOFIT;  // *FitError: no rand draw
      __syncthreads();
      continue;
    }
    const uint64_t r = ksg_splitmix_next(&rng) >> 1;  // rand.Int() (generic_scheduler.go:94)
    const uint64_t target = k - 1 - (r % k);           // ix-th in descending rank order
    if (wave == 0) {
      uint64_t acc = 0;
      for (uint32_t base = 0; base < (uint32_t)(R * KSG_NWAVE); base += 64) {
        const uint32_t widx = base + lane;
        const uint64_t w = widx < (uint32_t)(R * KSG_NWAVE) ? s_tie[widx] : 0ULL;
        const uint32_t cnt = __popcll(w);
        const uint32_t incl = wave_incl_scan_u32(cnt, lane);
        const uint32_t tot = __shfl(incl, 63, 64);
        if (target < acc + tot) {
          const uint32_t excl = incl - cnt;
          if (acc + excl <= target && target < acc + incl)
            s_winner = (int32_t)(d.lo + widx * 64 + select_bit(w, (uint32_t)(target - acc - excl)));
          break;
        }
        acc += tot;
      }
    }
    __syncthreads();
    const uint32_t win = (uint32_t)s_winner;
    if (tid == 0) {
      commit_pod(d, p, ids, win);
      out[i] = (int32_t)win;
      drain_stores();
    }
    if constexpr (REG) {
      const uint32_t off = win - d.lo;
      const uint32_t jw = off / KSG_NT, tw = off % KSG_NT;
#pragma unroll
      for (int j = 0; j < R; ++j)
        if ((uint32_t)j == jw && tid == tw) {
          rusedc[j] = (int64_t)((uint64_t)rusedc[j] + (uint64_t)p.milli_cpu);
          rusedm[j] = (int64_t)((uint64_t)rusedm[j] + (uint64_t)p.memory);
        }
    }
    __syncthreads();
  }
  if (tid == 0) *rng_io = rng;
}

// ============================================================================
// Single-pod scan (begin / evaluate / sharded steps). Writes, per mode:
//   EVAL : fail code and combined score of every node of the shard
//   BEGIN: the exchange record {max score, tie count, error, tie words}
// phase 0: complete pass; phase 1: only ServiceAntiAffinity domain counts
// (partial over this shard, written to dpart); phase 2: complete pass with
// all-reduced domain counts read from dglobal.
// ============================================================================
template <int R, bool ANTI>
__global__ __launch_bounds__(KSG_NT) void ksg_scan_kernel(KsgDev d, const ksg_pod* __restrict__ pods,
                                                         const uint32_t* __restrict__ ids, int mode,
                                                         int phase, uint8_t* __restrict__ fail_out,
                                                         int64_t* __restrict__ score_out,
                                                         uint8_t* __restrict__ record,
                                                         int32_t* __restrict__ dpart,
                                                         const int32_t* __restrict__ dglobal) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int32_t* s_dcount = reinterpret_cast<int32_t*>(smem);
  __shared__ int64_t s_wmax[KSG_NWAVE];
  __shared__ uint32_t s_wcnt[KSG_NWAVE];

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t bit = 1ULL << lane;
  const ksg_pod& p = pods[0];
  PodCtx c;
  pod_resolve(d, p, ids, c);
  KsgRecordHdr* hdr = reinterpret_cast<KsgRecordHdr*>(record);
  uint64_t* words = reinterpret_cast<uint64_t*>(record + sizeof(KsgRecordHdr));
  if (c.error) {
    if (mode == KSG_MODE_BEGIN && phase != 1 && tid == 0) {
      hdr->max_score = KSG_SCORE_NONE;
      hdr->tie_count = 0;
      hdr->error = 1;
    }
    if (phase == 1)
      for (uint32_t k = tid; k < d.n_domains_total; k += KSG_NT) dpart[k] = 0;
    return;
  }
  const bool use_lds_dcount = ANTI && phase != 2;
  if (use_lds_dcount) {
    for (uint32_t k = tid; k < d.n_domains_total; k += KSG_NT) s_dcount[k] = 0;
    __syncthreads();
  }
  const bool need_cnt = d.w_spread != 0 || ANTI;
  int64_t sc[R];
  bool fit[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t n = d.lo + j * KSG_NT + tid;
    const uint32_t wi = (d.lo >> 6) + j * KSG_NWAVE + wave;
    const bool valid = n < d.hi;
    const int64_t capc = valid ? d.cap_cpu[n] : 0;
    const int64_t capm = valid ? d.cap_mem[n] : 0;
    const int64_t usedc = valid ? ld_mut(d.used_cpu + n) : 0;
    const int64_t usedm = valid ? ld_mut(d.used_mem + n) : 0;
    int32_t cnt = 0;
    if (need_cnt && c.svc >= 0 && valid) cnt = ld_mut(d.svc_cnt + (size_t)c.svc * d.n_nodes + n);
    const int f = valid ? node_fail(d, c, n, wi, bit, capc, capm, usedc, usedm) : -1;
    fit[j] = (f == KSG_FAIL_NONE);
    sc[j] = fit[j] ? node_score(d, c, n, capc, capm, usedc, usedm, cnt) : KSG_SCORE_NONE;
    if (use_lds_dcount && fit[j] && cnt != 0) {
      for (uint32_t a = 0; a < d.n_anti; ++a) {
        const int32_t dom = d.anti_domain[(size_t)a * d.n_nodes + n];
        if (dom >= 0) atomicAdd(&s_dcount[d.anti_dom_off[a] + dom], cnt);
      }
    }
    if (valid && fail_out && phase != 1) fail_out[n - d.lo] = (uint8_t)f;
  }
  if (ANTI) {
    __syncthreads();
    if (phase == 1) {
      for (uint32_t k = tid; k < d.n_domains_total; k += KSG_NT) dpart[k] = s_dcount[k];
      return;
    }
    const int32_t* dc = phase == 2 ? dglobal : s_dcount;
    if (!d.equal_fallback) {
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (fit[j]) sc[j] += anti_term(d, c, d.lo + j * KSG_NT + tid, dc);
    }
  }
  if (mode == KSG_MODE_EVAL) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t n = d.lo + j * KSG_NT + tid;
      if (n < d.hi) score_out[n - d.lo] = sc[j];
    }
    return;
  }
  int64_t m = KSG_SCORE_NONE;
#pragma unroll
  for (int j = 0; j < R; ++j) m = sc[j] > m ? sc[j] : m;
  m = wave_max_i64(m);
  if (lane == 0) s_wmax[wave] = m;
  __syncthreads();
  int64_t M = s_wmax[0];
#pragma unroll
  for (int w = 1; w < KSG_NWAVE; ++w) M = s_wmax[w] > M ? s_wmax[w] : M;
  uint32_t wc = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint64_t b = __ballot(fit[j] && sc[j] == M);
    const uint32_t widx = j * KSG_NWAVE + wave;
    if (lane == 0 && widx < d.nwords) words[widx] = b;
    wc += __popcll(b);
  }
  if (lane == 0) s_wcnt[wave] = wc;
  __syncthreads();
  if (tid == 0) {
    uint64_t k = 0;
    for (int w = 0; w < KSG_NWAVE; ++w) k += s_wcnt[w];
    hdr->max_score = M;
    hdr->tie_count = (M == KSG_SCORE_NONE) ? 0 : k;
    hdr->error = 0;
  }
}

// ============================================================================
// Decide + commit (one wave): from the all-gathered per-shard records, find the
// global max score and tie count, draw ix (or take the caller's tie_index), walk
// shards in descending rank order to the owner of the ix-th tie, select its
// node and commit it to this rank's replica of the node state.
// ============================================================================
// mode: 0 = summarize only (write {M, k, error} to summary), 1 = draw ix from the
// device splitmix64 stream and commit, 2 = commit the caller's tie_index.
__global__ __launch_bounds__(64) void ksg_decide_kernel(KsgDev d, const ksg_pod* __restrict__ pods,
                                                       const uint32_t* __restrict__ ids,
                                                       const uint8_t* __restrict__ records,
                                                       uint32_t rec_bytes, uint32_t world,
                                                       const uint32_t* __restrict__ shard_wlo,
                                                       int mode, uint64_t tie_index,
                                                       uint64_t* rng_io, int32_t* out,
                                                       uint32_t out_idx, int64_t* summary) {
  __shared__ int32_t s_winner;
  const uint32_t lane = threadIdx.x;
  if (lane == 0) s_winner = -1;
  int64_t M = KSG_SCORE_NONE;
  int err = 0;
  for (uint32_t g = 0; g < world; ++g) {
    const KsgRecordHdr* h = reinterpret_cast<const KsgRecordHdr*>(records + (size_t)g * rec_bytes);
    if (h->error) err = 1;
    if (h->tie_count > 0 && h->max_score > M) M = h->max_score;
  }
  uint64_t k = 0;
  for (uint32_t g = 0; g < world; ++g) {
    const KsgRecordHdr* h = reinterpret_cast<const KsgRecordHdr*>(records + (size_t)g * rec_bytes);
    if (h->tie_count > 0 && h->max_score == M) k += h->tie_count;
  }
  if (d.empty_priorities) k = 0;  // all priority weights 0: empty HostPriorityList
  if (mode == 0) {
    if (lane == 0) {
      summary[0] = M;
      summary[1] = (int64_t)k;
      summary[2] = err;
    }
    return;
  }
  if (err) {
    if (lane == 0) out[out_idx] = KSG_OUT_ERROR;
    return;
  }
  if (k == 0) {
    if (lane == 0) out[out_idx] = KSG_OUT_NOFIT;  // no rand draw on FitError
    return;
  }
  uint64_t ix;
  if (mode == 1) {
    uint64_t rng = *rng_io;
    ix = (ksg_splitmix_next(&rng) >> 1) % k;
    __syncthreads();
    if (lane == 0) *rng_io = rng;
  } else {
    ix = tie_index % k;
  }
  // descending rank order: highest shard first (generic_scheduler.go:88-95)
  int32_t owner = -1;
  uint64_t lix = 0, kg = 0;
  for (int32_t g = (int32_t)world - 1; g >= 0; --g) {
    const KsgRecordHdr* h = reinterpret_cast<const KsgRecordHdr*>(records + (size_t)g * rec_bytes);
    if (h->tie_count > 0 && h->max_score == M) {
      if (ix < h->tie_count) {
        owner = g;
        lix = ix;
        kg = h->tie_count;
        break;
      }
      ix -= h->tie_count;
    }
  }
  if (owner < 0) {
    if (lane == 0) out[out_idx] = KSG_OUT_ERROR;
    return;
  }
  const uint8_t* rec = records + (size_t)owner * rec_bytes;
  const uint64_t* words = reinterpret_cast<const uint64_t*>(rec + sizeof(KsgRecordHdr));
  const uint32_t nwords = (rec_bytes - (uint32_t)sizeof(KsgRecordHdr)) / 8;
  const uint64_t target = kg - 1 - lix;
  uint64_t acc = 0;
  for (uint32_t base = 0; base < nwords; base += 64) {
    const uint32_t widx = base + lane;
    const uint64_t w = widx < nwords ? words[widx] : 0ULL;
    const uint32_t cnt = __popcll(w);
    const uint32_t incl = wave_incl_scan_u32(cnt, lane);
    const uint32_t tot = __shfl(incl, 63, 64);
    if (target < acc + tot) {
      const uint32_t excl = incl - cnt;
      if (acc + excl <= target && target < acc + incl)
        s_winner = (int32_t)((shard_wlo[owner] + widx) * 64 + select_bit(w, (uint32_t)(target - acc - excl)));
      break;
    }
    acc += tot;
  }
  __syncthreads();
  if (lane == 0) {
    const int32_t win = s_winner;
    if (win < 0) {
      out[out_idx] = KSG_OUT_ERROR;
    } else {
      commit_pod(d, pods[0], ids, (uint32_t)win);
      out[out_idx] = win;
    }
  }
}

// ============================================================================
// Static per-node tables (once per ksg_set_cluster): LabelsPresence fit bitmap
// (predicates.go:215-229), EqualPriority + LabelPreference static score
// (generic_scheduler.go:180-195, priorities.go:109-134), anti-affinity domain
// and ServiceAffinity pair per node. One thread per node.
// ============================================================================

__device__ __forceinline__ bool node_has_key(const uint32_t* pairs, uint32_t np,
                                             const uint32_t* pair_keys, uint32_t key) {
  for (uint32_t i = 0; i < np; ++i)
    if (pair_keys[pairs[i]] == key) return true;
  return false;
}

__global__ void ksg_static_kernel(KsgStaticCfg sc, uint32_t n_nodes, const ksg_node* __restrict__ nodes,
                                  const uint32_t* __restrict__ node_pairs,
                                  const uint32_t* __restrict__ pair_keys,
                                  const int32_t* __restrict__ dom_of_pair,  // [n_anti][n_pairs]
                                  uint32_t n_pairs, uint32_t nw, uint64_t* static_fit,
                                  int32_t* static_score, int32_t* anti_domain, int32_t* aff_pair) {
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  bool fits = true;
  int32_t score = 0;
  if (n < n_nodes) {
    const uint32_t* pairs = node_pairs + nodes[n].label_off;
    const uint32_t np = nodes[n].n_labels;
    for (uint32_t q = 0; q < sc.n_presence; ++q) {
      for (uint32_t i = 0; i < sc.presence_n_keys[q]; ++i) {
        const bool exists = node_has_key(pairs, np, pair_keys, sc.presence_keys[q][i]);
        if ((exists && !sc.presence_flag[q]) || (!exists && sc.presence_flag[q])) fits = false;
      }
    }
    score = sc.w_equal;  // EqualPriority: 1 * weight
    for (uint32_t q = 0; q < sc.n_pref; ++q) {
      const bool exists = node_has_key(pairs, np, pair_keys, sc.pref_key[q]);
      const bool ok = (exists && sc.pref_presence[q]) || (!exists && !sc.pref_presence[q]);
      score += sc.w_pref[q] * (ok ? 10 : 0);
    }
    static_score[n] = score;
    for (uint32_t a = 0; a < sc.n_anti; ++a) {
      int32_t dom = -1;
      for (uint32_t i = 0; i < np; ++i) {
        const int32_t x = dom_of_pair[(size_t)a * n_pairs + pairs[i]];
        if (x >= 0) dom = x;
      }
      anti_domain[(size_t)a * n_nodes + n] = dom;
    }
    for (uint32_t j = 0; j < sc.n_aff; ++j) {
      int32_t pr = -1;
      for (uint32_t i = 0; i < np; ++i)
        if (pair_keys[pairs[i]] == sc.aff_key[j]) pr = (int32_t)pairs[i];
      aff_pair[(size_t)j * n_nodes + n] = pr;
    }
  }
  const uint64_t b = __ballot(n < n_nodes && fits);
  if ((threadIdx.x & 63) == 0 && (n >> 6) < nw) static_fit[n >> 6] = b;
}

// label pair bitmaps: pairmap[p][n/64] |= bit for every (node, pair)
__global__ void ksg_pairmap_kernel(uint32_t n_nodes, const ksg_node* __restrict__ nodes,
                                   const uint32_t* __restrict__ node_pairs, uint32_t nw,
                                   unsigned long long* pairmap) {
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes) return;
  const uint32_t* pairs = node_pairs + nodes[n].label_off;
  for (uint32_t i = 0; i < nodes[n].n_labels; ++i)
    atomicOr(pairmap + (size_t)pairs[i] * nw + (n >> 6), 1ULL << (n & 63));
}

// host-mirror deltas (add/remove pod outside a batch)
// op: 0 store32, 1 store64, 2 or64, 3 andnot64. Patches are applied in order
// by one thread so that several patches to one word compose.
__global__ void ksg_patch_kernel(const KsgPatch* __restrict__ patches, uint32_t n) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (uint32_t i = 0; i < n; ++i) {
    const KsgPatch pt = patches[i];
    switch (pt.width) {
      case 0: *reinterpret_cast<uint32_t*>(pt.addr) = (uint32_t)pt.value; break;
      case 1: *reinterpret_cast<uint64_t*>(pt.addr) = pt.value; break;
      case 2: *reinterpret_cast<uint64_t*>(pt.addr) |= pt.value; break;
      case 3: *reinterpret_cast<uint64_t*>(pt.addr) &= ~pt.value; break;
    }
  }
}

// ---- launch wrappers (called from ksg_runtime.cpp) ------------------------
template <int R, bool ANTI, bool REG>
static hipError_t launch_batch_t(const KsgDev& d, const ksg_pod* pods, const uint32_t* ids,
                                 uint32_t n, uint64_t* rng, int32_t* out, size_t lds,
                                 hipStream_t st) {
  hipLaunchKernelGGL((ksg_batch_kernel<R, ANTI, REG>), dim3(1), dim3(KSG_NT), lds, st, d, pods, ids, n,
                     rng, out);
  return hipGetLastError();
}

template <bool ANTI>
static hipError_t launch_batch_a(int R, const KsgDev& d, const ksg_pod* pods, const uint32_t* ids,
                                 uint32_t n, uint64_t* rng, int32_t* out, size_t lds,
                                 hipStream_t st) {
  switch (R) {
    case 1: return launch_batch_t<1, ANTI, true>(d, pods, ids, n, rng, out, lds, st);
    case 2: return launch_batch_t<2, ANTI, true>(d, pods, ids, n, rng, out, lds, st);
    case 4: return launch_batch_t<4, ANTI, true>(d, pods, ids, n, rng, out, lds, st);
    case 8: return launch_batch_t<8, ANTI, true>(d, pods, ids, n, rng, out, lds, st);
    case 16: return launch_batch_t<16, ANTI, false>(d, pods, ids, n, rng, out, lds, st);
    case 32: return launch_batch_t<32, ANTI, false>(d, pods, ids, n, rng, out, lds, st);
  }
  return hipErrorInvalidValue;
}

template <bool ANTI>
static hipError_t launch_scan_a(int R, const KsgDev& d, const ksg_pod* pods, const uint32_t* ids,
                                int mode, int phase, uint8_t* fail_out, int64_t* score_out,
                                uint8_t* record, int32_t* dpart, const int32_t* dglobal, size_t lds,
                                hipStream_t st) {
#define KSG_SCAN_CASE(RR)                                                                           \
  case RR:                                                                                          \
    hipLaunchKernelGGL((ksg_scan_kernel<RR, ANTI>), dim3(1), dim3(KSG_NT), lds, st, d, pods, ids, mode, \
                       phase, fail_out, score_out, record, dpart, dglobal);                         \
    return hipGetLastError();
  switch (R) {
    KSG_SCAN_CASE(1)
    KSG_SCAN_CASE(2)
    KSG_SCAN_CASE(4)
    KSG_SCAN_CASE(8)
    KSG_SCAN_CASE(16)
    KSG_SCAN_CASE(32)
  }
#undef KSG_SCAN_CASE
  return hipErrorInvalidValue;
}

hipError_t ksg_launch_batch(int R, bool anti, const KsgDev& d, const ksg_pod* pods,
                            const uint32_t* ids, uint32_t n, uint64_t* rng, int32_t* out,
                            size_t lds, hipStream_t st) {
  return anti ? launch_batch_a<true>(R, d, pods, ids, n, rng, out, lds, st)
              : launch_batch_a<false>(R, d, pods, ids, n, rng, out, lds, st);
}

hipError_t ksg_launch_scan(int R, bool anti, const KsgDev& d, const ksg_pod* pods,
                           const uint32_t* ids, int mode, int phase, uint8_t* fail_out,
                           int64_t* score_out, uint8_t* record, int32_t* dpart,
                           const int32_t* dglobal, size_t lds, hipStream_t st) {
  return anti ? launch_scan_a<true>(R, d, pods, ids, mode, phase, fail_out, score_out, record, dpart,
                                    dglobal, lds, st)
              : launch_scan_a<false>(R, d, pods, ids, mode, phase, fail_out, score_out, record, dpart,
                                     dglobal, lds, st);
}

hipError_t ksg_launch_decide(const KsgDev& d, const ksg_pod* pods, const uint32_t* ids,
                             const uint8_t* records, uint32_t rec_bytes, uint32_t world,
                             const uint32_t* shard_wlo, int mode, uint64_t tie_index,
                             uint64_t* rng, int32_t* out, uint32_t out_idx, int64_t* summary,
                             hipStream_t st) {
  hipLaunchKernelGGL(ksg_decide_kernel, dim3(1), dim3(64), 0, st, d, pods, ids, records, rec_bytes,
                     world, shard_wlo, mode, tie_index, rng, out, out_idx, summary);
  return hipGetLastError();
}

hipError_t ksg_launch_static(const KsgStaticCfg& sc, uint32_t n_nodes, const ksg_node* nodes,
                             const uint32_t* node_pairs, const uint32_t* pair_keys,
                             const int32_t* dom_of_pair, uint32_t n_pairs, uint32_t nw,
                             uint64_t* static_fit, int32_t* static_score, int32_t* anti_domain,
                             int32_t* aff_pair, unsigned long long* pairmap, hipStream_t st) {
  const uint32_t blocks = (n_nodes + 255) / 256;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(ksg_pairmap_kernel, dim3(blocks), dim3(256), 0, st, n_nodes, nodes, node_pairs,
                     nw, pairmap);
  hipLaunchKernelGGL(ksg_static_kernel, dim3(blocks), dim3(256), 0, st, sc, n_nodes, nodes, node_pairs,
                     pair_keys, dom_of_pair, n_pairs, nw, static_fit, static_score, anti_domain,
                     aff_pair);
  return hipGetLastError();
}

hipError_t ksg_launch_patch(const KsgPatch* patches, uint32_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(ksg_patch_kernel, dim3(1), dim3(64), 0, st, patches, n);
  return hipGetLastError();
}
