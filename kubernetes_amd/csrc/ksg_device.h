// ksg_device.h — device-side building blocks shared by the CDNA4 kernels:
// Go-exact arithmetic, the per-node filter (predicates) and score (priorities)
// of the reference, wave reductions, and the AssumePod commit.
#pragma once
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
// Load of mutable state: coherent (agent scope) when other waves commit
// concurrently (exact path), plain when the reader is the only writer or the
// state is read-only for the kernel's lifetime (window path).
template <bool COH, typename T>
__device__ __forceinline__ T ld_st(const T* p) {
  if constexpr (COH) return ld_mut(p);
  else return *p;
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

// calculateScore for the window path, whose host guard (use_window) holds
// 0 <= cap <= 2^49 and 0 <= requested < 2^50: q = 10u/cap (u = cap - requested)
// through a per-node f64 reciprocal inv10 = 10.0/cap. |q - 10u/cap| <= ~2.2e-15,
// so trunc(q) can differ from the exact floor only when q lies within that of
// an integer; every q within 1e-9 of an integer takes the exact integer fix-up
// (10u < 2^53, (q+1)*cap < 2^53: no overflow), so the result equals lr_calc.
__device__ __forceinline__ int32_t lr_win(int64_t requested, int64_t cap, double inv10) {
  if (requested > cap || cap == 0) return 0;  // priorities.go:29-35
  const int64_t u = cap - requested;
  const double q = (double)u * inv10;
  int32_t qi = (int32_t)q;
  const double fr = q - (double)qi;
  if (fr < 1e-9 || fr > 1.0 - 1e-9) {
    const uint64_t y = (uint64_t)u * 10ULL;
    if ((uint64_t)(qi + 1) * (uint64_t)cap <= y) qi += 1;
    else if ((uint64_t)qi * (uint64_t)cap > y) qi -= 1;
  }
  return qi;
}
__device__ __forceinline__ double lr_inv10(int64_t cap) { return cap > 0 ? 10.0 / (double)cap : 0.0; }
// lr_win without the branch: the integer check runs every time (it changes nothing where q is
// far from an integer, so the result is lr_win's), and independent calls interleave -- for the
// latency-bound resolvers; phase A (VALU-bound, the check rarely needed) keeps the branch
__device__ __forceinline__ int32_t lr_win_nb(int64_t requested, int64_t cap, double inv10) {
  const bool zero = requested > cap || cap == 0;
  const int64_t u = cap - requested;
  int32_t qi = (int32_t)((double)u * inv10);
  const uint64_t y = (uint64_t)u * 10ULL;
  const bool up = (uint64_t)(qi + 1) * (uint64_t)cap <= y;
  const bool dn = !up && (uint64_t)qi * (uint64_t)cap > y;
  qi += up ? 1 : dn ? -1 : 0;
  return zero ? 0 : qi;
}

// int(10 * (float32(num) / float32(den))) with IEEE f32 divide and multiply,
// no contraction (spreading.go:79-83, 156-160).
__device__ __forceinline__ int64_t frac10_f32(int64_t num, int64_t den) {
  const float q = __fdiv_rn((float)num, (float)den);
  const float s = __fmul_rn(10.0f, q);
  return (int64_t)s;
}

// the same for operands that fit int32 (counts and their maxima): (float)int32 rounds
// the integer exactly as (float)int64 does, at a fraction of the conversion's cost
__device__ __forceinline__ int32_t frac10_i32(int32_t num, int32_t den) {
  const float q = __fdiv_rn((float)num, (float)den);
  const float s = __fmul_rn(10.0f, q);
  return (int32_t)s;
}

// Go's int arithmetic wraps (two's complement); so do these
__host__ __device__ __forceinline__ int64_t wsum(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__host__ __device__ __forceinline__ int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int64_t o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int32_t o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
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

// ---- DPP wave scans (GFX9 row_shr + row_bcast; no LDS round trip) ----------
// Inclusive prefix over the 64 lanes; lane 63 holds the wave total. Lanes whose
// DPP source falls outside the row (or whose row is masked) receive `old`,
// the identity of the operator.
#define KSG_DPP(old, v, ctrl, rmask) __builtin_amdgcn_update_dpp((old), (v), (ctrl), (rmask), 0xf, false)

__device__ __forceinline__ uint32_t dpp_scan_add(uint32_t v) {
  int x = (int)v;
  x += KSG_DPP(0, x, 0x111, 0xf);  // row_shr:1
  x += KSG_DPP(0, x, 0x112, 0xf);  // row_shr:2
  x += KSG_DPP(0, x, 0x114, 0xf);  // row_shr:4
  x += KSG_DPP(0, x, 0x118, 0xf);  // row_shr:8
  x += KSG_DPP(0, x, 0x142, 0xa);  // row_bcast:15 -> rows 1, 3
  x += KSG_DPP(0, x, 0x143, 0xc);  // row_bcast:31 -> rows 2, 3
  return (uint32_t)x;
}

__device__ __forceinline__ int32_t dpp_scan_max(int32_t x) {
  const int lo = (int)0x80000000;
  x = max(x, KSG_DPP(lo, x, 0x111, 0xf));
  x = max(x, KSG_DPP(lo, x, 0x112, 0xf));
  x = max(x, KSG_DPP(lo, x, 0x114, 0xf));
  x = max(x, KSG_DPP(lo, x, 0x118, 0xf));
  x = max(x, KSG_DPP(lo, x, 0x142, 0xa));
  x = max(x, KSG_DPP(lo, x, 0x143, 0xc));
  return x;
}

__device__ __forceinline__ uint32_t dpp_scan_or(uint32_t v) {
  int x = (int)v;
  x |= KSG_DPP(0, x, 0x111, 0xf);
  x |= KSG_DPP(0, x, 0x112, 0xf);
  x |= KSG_DPP(0, x, 0x114, 0xf);
  x |= KSG_DPP(0, x, 0x118, 0xf);
  x |= KSG_DPP(0, x, 0x142, 0xa);
  x |= KSG_DPP(0, x, 0x143, 0xc);
  return (uint32_t)x;
}

// wave-uniform results of the scans
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)dpp_scan_or(v), 63);
}
__device__ __forceinline__ uint32_t wave_total_add(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)dpp_scan_add(v), 63);
}
__device__ __forceinline__ int32_t wave_total_max(int32_t v) {
  return __builtin_amdgcn_readlane(dpp_scan_max(v), 63);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane)) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane) << 32);
}

// register copy the compiler cannot see through: the s_waitcnt for a pending
// load into `x` lands here, not at a later use
__device__ __forceinline__ uint32_t opaque_v(uint32_t x) {
  uint32_t y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}
__device__ __forceinline__ uint64_t opaque_v64(uint64_t x) {
  return ((uint64_t)opaque_v((uint32_t)(x >> 32)) << 32) | opaque_v((uint32_t)x);
}

// r % k for r < 2^64, 0 < k < 2^32, without the 64-bit division routine:
// hi % k in 32 bits, then (rem * 2^32 + lo) / k through one f64 divide whose
// quotient is off by at most one (x < k * 2^32 <= 2^64, 53-bit mantissa), fixed
// with exact integer arithmetic.
__device__ __forceinline__ uint32_t umod64_32(uint64_t r, uint32_t k) {
  const uint32_t hi = (uint32_t)(r >> 32), lo = (uint32_t)r;
  const uint64_t x = ((uint64_t)(hi % k) << 32) | lo;
  uint64_t q = (uint64_t)((double)x / (double)k);
  if (q > 0) q -= 1;  // never overshoot: x - q*k >= 0
  uint64_t rem = x - q * (uint64_t)k;
  while (rem >= k) rem -= k;  // at most 3 steps
  return (uint32_t)rem;
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
  const ksg_pod_ext* ext;  // extensions (nullptr: none); its taint lists index ids
  const uint32_t* ids;
};

// SelectorFromSet's trap per ServiceAffinity predicate (predicates.go:311-315,
// labels.go:60-61, selector.go:654-668): a predicate whose affinity map holds
// an invalid (key, value) builds the empty selector and fits every node, so
// its labels are only required through the predicates that stayed valid.
// req_aff[j] < 0 afterwards means "no requirement on label j".
__device__ __forceinline__ void aff_apply_trap(const KsgDev& d, int32_t (&req_aff)[KSG_MAX_AFF]) {
  uint32_t bad = 0;
#pragma unroll
  for (uint32_t j = 0; j < KSG_MAX_AFF; ++j)
    if (j < d.n_aff && req_aff[j] == KSG_AFF_INVALID) bad |= 1u << j;
  if (!bad) return;
  uint32_t active = 0;
  for (uint32_t g = 0; g < d.n_aff_groups; ++g)
    if (!(d.aff_group_mask[g] & bad)) active |= d.aff_group_mask[g];
#pragma unroll
  for (uint32_t j = 0; j < KSG_MAX_AFF; ++j)
    if (!((active >> j) & 1u)) req_aff[j] = -1;
}

template <bool COH = true>
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
  c.ext = nullptr;
  c.ids = ids;
  int32_t peer = -1;
  if (c.svc >= 0) {
    c.spread_max = ld_st<COH>(d.svc_max + c.svc);
    c.svc_total = ld_st<COH>(d.svc_total + c.svc);
    peer = ld_st<COH>(d.svc_peer + c.svc);
  }
  // ServiceAffinity (predicates.go:257-324): labels the pod's nodeSelector does
  // not give come from the node of the first service peer.
  // (loops over KSG_MAX_AFF are fully unrolled so req_aff stays in registers)
#pragma unroll
  for (uint32_t j = 0; j < KSG_MAX_AFF; ++j) c.req_aff[j] = -1;
  if (d.preds & KSG_PRED_SERVICEAFFINITY) {
    bool all_given = true;
#pragma unroll
    for (uint32_t j = 0; j < KSG_MAX_AFF; ++j) {
      if (j < d.n_aff) {
        c.req_aff[j] = p.aff_pair[j];
        if (p.aff_pair[j] == -1) all_given = false;  // (KSG_AFF_INVALID: given, invalid)
      }
    }
    if (!all_given && peer != -1) {
      if (peer == -2) {
        c.error = 1;  // GetNodeInfo of the peer's host fails (predicates.go:293-296)
      } else {
#pragma unroll
        for (uint32_t j = 0; j < KSG_MAX_AFF; ++j)
          if (j < d.n_aff && c.req_aff[j] == -1) c.req_aff[j] = d.aff_pair[(size_t)j * d.n_nodes + peer];
      }
    }
    aff_apply_trap(d, c.req_aff);
  }
}

// Filter: first failing predicate (fixed order) or 0. wi/bit locate node n in
// the bitmaps; wi is wave-uniform for the scan kernels. `L` yields the pod's
// list entries: L.port(i), L.pd(i), L.sel(i).
template <bool COH, typename L>
__device__ __forceinline__ int node_fail_l(const KsgDev& d, const PodCtx& c, const L& lists, uint32_t n,
                                           uint32_t wi, uint64_t bit, int64_t capc, int64_t capm,
                                           int64_t usedc, int64_t usedm) {
  const uint32_t P = d.preds;
  if ((P & KSG_PRED_HOSTNAME) && c.host != -1 && (int32_t)n != c.host) return KSG_FAIL_HOSTNAME;
  if (d.has_static_fit && !(d.static_fit[wi] & bit)) return KSG_FAIL_LABELSPRESENCE;
  if (P & KSG_PRED_MATCHNODESELECTOR) {  // PodMatchesNodeLabels (predicates.go:161-167)
    for (uint32_t i = 0; i < c.n_sel; ++i)
      if (!(d.pairmap[(size_t)lists.sel(i) * d.nw + wi] & bit)) return KSG_FAIL_MATCHNODESELECTOR;
  }
  if (P & KSG_PRED_NODISKCONFLICT) {  // NoDiskConflict (predicates.go:73-83)
    for (uint32_t i = 0; i < c.n_pds; ++i)
      if (ld_st<COH>(d.keymap + (size_t)lists.pd(i) * d.nw + wi) & bit) return KSG_FAIL_NODISKCONFLICT;
  }
  if (P & KSG_PRED_PODFITSPORTS) {  // PodFitsPorts (predicates.go:326-338)
    for (uint32_t i = 0; i < c.n_ports; ++i)
      if (ld_st<COH>(d.keymap + (size_t)lists.port(i) * d.nw + wi) & bit) return KSG_FAIL_PODFITSPORTS;
  }
  if ((P & KSG_PRED_PODFITSRESOURCES) && !c.zero_req) {
    // CheckPodsExceedingCapacity (predicates.go:104-124) over existing+pod, in
    // closed form: every pod fits greedily iff cap==0 || cap - sum(existing) >= req.
    const bool fc = capc == 0 || (int64_t)((uint64_t)capc - (uint64_t)usedc) >= c.req_cpu;
    const bool fm = capm == 0 || (int64_t)((uint64_t)capm - (uint64_t)usedm) >= c.req_mem;
    if (!(fc && fm)) return KSG_FAIL_PODFITSRESOURCES;
  }
  if (P & KSG_PRED_SERVICEAFFINITY) {
#pragma unroll
    for (uint32_t j = 0; j < KSG_MAX_AFF; ++j)
      if (j < d.n_aff && c.req_aff[j] >= 0 && !(d.pairmap[(size_t)c.req_aff[j] * d.nw + wi] & bit))
        return KSG_FAIL_SERVICEAFFINITY;
  }
  if (d.ext_filters && c.ext) {  // extensions (include/kschedgpu.h; parity unpinned)
    if (d.ext_filters & KSG_EXT_TAINTS)  // PodToleratesNodeTaints: an untolerated NoSchedule/NoExecute taint
      for (uint32_t i = 0; i < c.ext->n_hard; ++i)
        if (d.taintmap[(size_t)c.ids[c.ext->hard_off + i] * d.nw + wi] & bit) return KSG_FAIL_TAINTS;
    if (d.ext_filters & KSG_EXT_SCALAR)  // PodFitsResources' ScalarResources: allocatable < used + request
      for (uint32_t r = 0; r < d.n_scalar; ++r) {
        const int64_t req = c.ext->scalar[r];
        if (req > 0) {
          const int64_t cap = d.scalar_cap[(size_t)r * d.n_nodes + n];
          const int64_t used = ld_st<COH>(d.scalar_used + (size_t)r * d.n_nodes + n);
          if (cap < (int64_t)((uint64_t)used + (uint64_t)req)) return KSG_FAIL_SCALAR;
        }
      }
  }
  return KSG_FAIL_NONE;
}

// BalancedResourceAllocation (kube-scheduler v1.10 balanced_resource_allocation.go,
// not in this reference; parity unpinned) over the same requested totals as
// LeastRequested, float64 op for op: fraction = requested / capacity (1 when
// capacity is 0); 0 if either fraction >= 1, else int((1 - |fc - fm|) * 10).
__device__ __forceinline__ int64_t balanced_score(int64_t tc, int64_t capc, int64_t tm, int64_t capm) {
  const double fc = capc == 0 ? 1.0 : __ddiv_rn((double)tc, (double)capc);
  const double fm = capm == 0 ? 1.0 : __ddiv_rn((double)tm, (double)capm);
  if (fc >= 1.0 || fm >= 1.0) return 0;
  return (int64_t)__dmul_rn(__dsub_rn(1.0, fabs(__dsub_rn(fc, fm))), 10.0);
}

// TaintTolerationPriority's map (v1.10 taint_toleration.go): the node's
// PreferNoSchedule taints the pod does not tolerate
__device__ __forceinline__ int32_t soft_taints(const KsgDev& d, const PodCtx& c, uint32_t wi, uint64_t bit) {
  int32_t k = 0;
  for (uint32_t i = 0; i < c.ext->n_soft; ++i) k += (d.taintmap[(size_t)c.ids[c.ext->soft_off + i] * d.nw + wi] & bit) != 0;
  return k;
}
// ... and its reduce, NormalizeReduce(10, reverse=true): 10 - 10 * count / max
// over the filtered nodes (every node 10 when the max is 0)
__device__ __forceinline__ int64_t taint_score(int32_t cnt, int32_t mx) {
  return mx == 0 ? 10 : 10 - (10 * (int64_t)cnt) / mx;
}
// the same in 32 bits (counts of a node's taints, at most 64): a 32-bit divide instead of
// the 64-bit one's long expansion, for the resolvers' per-pod chain
__device__ __forceinline__ int32_t taint_score_i32(int32_t cnt, int32_t mx) {
  return mx == 0 ? 10 : 10 - (10 * cnt) / mx;
}

struct PtrLists {
  const uint32_t* ports_;
  const uint32_t* pds_;
  const uint32_t* sel_;
  __device__ __forceinline__ uint32_t port(uint32_t i) const { return ports_[i]; }
  __device__ __forceinline__ uint32_t pd(uint32_t i) const { return pds_[i]; }
  __device__ __forceinline__ uint32_t sel(uint32_t i) const { return sel_[i]; }
};

template <bool COH = true>
__device__ __forceinline__ int node_fail(const KsgDev& d, const PodCtx& c, uint32_t n, uint32_t wi,
                                         uint64_t bit, int64_t capc, int64_t capm, int64_t usedc,
                                         int64_t usedm) {
  const PtrLists L{c.ports, c.pds, c.sel};
  return node_fail_l<COH>(d, c, L, n, wi, bit, capc, capm, usedc, usedm);
}

// Priorities without ServiceAntiAffinity (added after the domain counts).
__device__ __forceinline__ int64_t node_score(const KsgDev& d, const PodCtx& c, uint32_t n,
                                              int64_t capc, int64_t capm, int64_t usedc,
                                              int64_t usedm, int32_t cnt) {
  if (d.equal_fallback) return 1;  // EqualPriority (generic_scheduler.go:141-143,180-195)
  // combinedScores[host] += score * weight (generic_scheduler.go:145-159), Go int: wrapping
  int64_t s = 0;
  if (d.has_static_score) s = d.static_score[n];
  if (d.w_lr) {  // calculateOccupancy (priorities.go:43-76): all pods on node + this pod
    const int64_t tc = (int64_t)((uint64_t)usedc + (uint64_t)c.req_cpu);
    const int64_t tm = (int64_t)((uint64_t)usedm + (uint64_t)c.req_mem);
    s = wsum(s, wmul(d.w_lr, (lr_calc(tc, capc) + lr_calc(tm, capm)) / 2));
  }
  if (d.w_spread) {  // CalculateSpreadPriority (spreading.go:72-86)
    const int64_t sc = c.spread_max > 0 ? frac10_f32((int64_t)c.spread_max - cnt, c.spread_max) : 10;
    s = wsum(s, wmul(d.w_spread, sc));
  }
  if (d.w_bal) {  // extension: BalancedResourceAllocation
    const int64_t tc = (int64_t)((uint64_t)usedc + (uint64_t)c.req_cpu);
    const int64_t tm = (int64_t)((uint64_t)usedm + (uint64_t)c.req_mem);
    s = wsum(s, wmul(d.w_bal, balanced_score(tc, capc, tm, capm)));
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
    s = wsum(s, wmul(d.w_anti[a], sc));
  }
  return s;
}

// AssumePod delta (plugin/pkg/scheduler/scheduler.go:115-118 -> modeler.go:77-79):
// the pod now counts on node w for resources, ports, PDs and service counts.
// Executed by one whole wave: each lane issues one independent agent-scope
// atomic (no return except the per-service count), so the commit costs one
// memory round trip instead of a serial chain. Caller drains with vmcnt(0).
__device__ __forceinline__ void commit_pod_wave(const KsgDev& d, const ksg_pod& p, const uint32_t* ids,
                                                uint32_t w, uint32_t lane, const ksg_pod_ext* ext = nullptr) {
  const uint32_t nk = p.n_ports + p.n_pds;
  if (lane == 0) {
    __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(d.used_cpu + w), (uint64_t)p.milli_cpu,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (lane == 1) {
    __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(d.used_mem + w), (uint64_t)p.memory,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (ext && lane - 2 < d.n_scalar && ext->scalar[lane - 2]) {  // extended resources
    __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(d.scalar_used + (size_t)(lane - 2) * d.n_nodes + w),
                           (uint64_t)ext->scalar[lane - 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint64_t bit = 1ULL << (w & 63);
  const size_t wi = w >> 6;
  for (uint32_t i = lane; i < nk; i += 64) {
    const uint32_t key = i < p.n_ports ? ids[p.ports_off + i] : ids[p.pds_off + (i - p.n_ports)];
    __hip_atomic_fetch_or(d.keymap + (size_t)key * d.nw + wi, bit, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
  }
  for (uint32_t i = lane; i < p.n_svcs; i += 64) {
    const uint32_t s = ids[p.svcs_off + i];
    const int32_t old = __hip_atomic_fetch_add(d.svc_cnt + (size_t)s * d.n_nodes + w, 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_or(d.svc_bits + (size_t)s * d.nw + wi, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(d.svc_max + s, old + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(d.svc_total + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int32_t expect = -1;
    __hip_atomic_compare_exchange_strong(d.svc_peer + s, &expect, (int32_t)w, __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

