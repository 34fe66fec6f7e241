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

#include "ksg_device.h"
#include "ksg_exact.h"
#include "ksg_shard.h"

// ============================================================================
// Exact per-pod path. One workgroup of 1024 threads (16 waves); thread t owns
// nodes lo + j*1024 + t (j < R). Per-node int32 scores live in LDS (R*4 KiB),
// so the only per-node registers are the optional cached capacity/requested
// totals (REG, R <= 4). The filter+score of node n is evaluated once per pod.
// ============================================================================

template <int R, bool ANTI, bool REG, typename SC>
__global__ __launch_bounds__(KSG_NT) void ksg_batch_kernel(KsgDev d, const ksg_pod* __restrict__ pods,
                                                          const uint32_t* __restrict__ ids,
                                                          uint32_t n_pods, uint64_t* rng_io,
                                                          int32_t* __restrict__ out,
                                                          const ksg_pod_ext* __restrict__ exts) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // per-node scores: LDS up to KSG_R_LDS nodes per thread, else HBM scratch
  // (each thread only ever reads back its own entries)
  using T = ScoreT<SC>;
  SC* s_score = R > T::r_lds ? reinterpret_cast<SC*>(d.score_scratch) : reinterpret_cast<SC*>(smem);
  int32_t* s_dcount = R > T::r_lds ? reinterpret_cast<int32_t*>(smem) : reinterpret_cast<int32_t*>(s_score + R * KSG_NT);
  int32_t* s_tmax = s_dcount + d.n_domains_total;  // (extension TaintTolerationPriority's max)
  __shared__ uint64_t s_tie[R * KSG_NWAVE];
  __shared__ SC s_wmax[KSG_NWAVE];
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

  for (uint32_t i = 0; i < n_pods; ++i) {
    const ksg_pod& p = pods[i];
    PodCtx c;
    pod_resolve(d, p, ids, c);
    if (exts) c.ext = exts + i;
    if (c.error) {
      if (tid == 0) out[i] = KSG_OUT_ERROR;
      continue;  // uniform; no LDS touched for this pod
    }
    if (ANTI || exts) {
      for (uint32_t k = tid; k < d.n_domains_total; k += KSG_NT) s_dcount[k] = 0;
      if (tid == 0) *s_tmax = 0;
      __syncthreads();
    }
    const SC m = scan_pod<R, ANTI, REG, SC>(d, c, tid, wave, bit, s_score, s_dcount, nullptr, rcapc, rcapm,
                                            rusedc, rusedm, nullptr, exts ? s_tmax : nullptr);
    SC M;
    uint64_t k;
    reduce_ties<R, SC>(d, m, tid, lane, wave, s_score, s_wmax, s_wcnt, s_tie, M, k);
    if (M == T::none || k == 0) {
      if (tid == 0) out[i] = KSG_OUT_NOFIT;  // *FitError: no rand draw
      __syncthreads();
      continue;
    }
    const uint64_t r = ksg_rng_draw(d.draws, rng);  // rand.Int() (generic_scheduler.go:94)
    rng += ksg_rng_step(d.draws);
    const uint64_t target = k - 1 - (r % k);           // ix-th host in descending name order
    if (wave == 0) {
      const int32_t win = select_tie(s_tie, R * KSG_NWAVE, target, lane, d.lo);
      commit_pod_wave(d, p, ids, (uint32_t)win, lane, exts ? exts + i : nullptr);
      if (lane == 0) {
        s_winner = win;
        out[i] = win;
      }
      drain_stores();
    }
    __syncthreads();
    if constexpr (REG) {
      const uint32_t off = (uint32_t)s_winner - d.lo;
      const uint32_t jw = off / KSG_NT, tw = off % KSG_NT;
#pragma unroll
      for (int j = 0; j < R; ++j)
        if ((uint32_t)j == jw && tid == tw) {
          rusedc[j] = (int64_t)((uint64_t)rusedc[j] + (uint64_t)p.milli_cpu);
          rusedm[j] = (int64_t)((uint64_t)rusedm[j] + (uint64_t)p.memory);
        }
    }
  }
  if (tid == 0) *rng_io = rng;
}

// ============================================================================
// Single-pod scan (begin / evaluate / sharded steps). Writes, per mode:
//   EVAL : fail code and combined score of every node of the shard
//   BEGIN: the exchange record {max score, tie count, error, tie words}
// phase 0: complete pass; phase 1: only the terms normalised over every shard's
// filtered nodes, partial over this shard: ServiceAntiAffinity's domain counts
// (dpart[0, n_domains_total)) and the extension TaintTolerationPriority's max soft
// count (dpart[n_domains_total]); phase 2: complete pass with the all-reduced
// ones read from dglobal (sum of the counts, max of the max).
// ============================================================================
template <int R, bool ANTI, typename SC>
__global__ __launch_bounds__(KSG_NT) void ksg_scan_kernel(KsgDev d, const ksg_pod* __restrict__ pods,
                                                         const uint32_t* __restrict__ ids, int mode,
                                                         int phase, uint8_t* __restrict__ fail_out,
                                                         int64_t* __restrict__ score_out,
                                                         uint8_t* __restrict__ record,
                                                         int32_t* __restrict__ dpart,
                                                         const int32_t* __restrict__ dglobal,
                                                         const ksg_pod_ext* __restrict__ ext) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // per-node scores: LDS up to KSG_R_LDS nodes per thread, else HBM scratch
  // (each thread only ever reads back its own entries)
  using T = ScoreT<SC>;
  SC* s_score = R > T::r_lds ? reinterpret_cast<SC*>(d.score_scratch) : reinterpret_cast<SC*>(smem);
  int32_t* s_dcount = R > T::r_lds ? reinterpret_cast<int32_t*>(smem) : reinterpret_cast<int32_t*>(s_score + R * KSG_NT);
  int32_t* s_tmax = s_dcount + d.n_domains_total;  // (extension TaintTolerationPriority's max)
  __shared__ uint64_t s_tie[R * KSG_NWAVE];
  __shared__ SC s_wmax[KSG_NWAVE];
  __shared__ uint32_t s_wcnt[KSG_NWAVE];

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t bit = 1ULL << lane;
  const ksg_pod& p = pods[0];
  PodCtx c;
  pod_resolve(d, p, ids, c);
  c.ext = ext;
  KsgRecordHdr* hdr = reinterpret_cast<KsgRecordHdr*>(record);
  uint64_t* words = reinterpret_cast<uint64_t*>(record + sizeof(KsgRecordHdr));
  if (c.error) {
    if (mode == KSG_MODE_BEGIN && phase != 1 && tid == 0) {
      hdr->max_score = KSG_SCORE_NONE;
      hdr->tie_count = 0;
      hdr->error = 1;
    }
    if (phase == 1)
      for (uint32_t k = tid; k <= d.n_domains_total; k += KSG_NT) dpart[k] = 0;
    return;
  }
  const bool lds_dcount = ANTI && phase != 2;
  if (lds_dcount || ext || phase == 1) {
    if (lds_dcount)
      for (uint32_t k = tid; k < d.n_domains_total; k += KSG_NT) s_dcount[k] = 0;
    if (tid == 0) *s_tmax = 0;
    __syncthreads();
  }
  if (phase == 1) {
    // the normalised terms' inputs only (the sharded all-reduce needs them before any score)
    scan_pod<R, false, false, SC>(d, c, tid, wave, bit, s_score, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                  nullptr);
    const bool need = ANTI && c.svc >= 0;
    const bool tt = d.w_taint != 0 && ext != nullptr && !d.equal_fallback;
    int32_t tmax = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t n = d.lo + j * KSG_NT + tid;
      const bool fit = n < d.hi && s_score[j * KSG_NT + tid] != T::none;
      if (need && fit) {
        const int32_t cnt = ld_mut(d.svc_cnt + (size_t)c.svc * d.n_nodes + n);
        if (cnt)
          for (uint32_t a = 0; a < d.n_anti; ++a) {
            const int32_t dom = d.anti_domain[(size_t)a * d.n_nodes + n];
            if (dom >= 0) atomicAdd(&s_dcount[d.anti_dom_off[a] + dom], cnt);
          }
      }
      if (tt && fit) tmax = max(tmax, soft_taints(d, c, (d.lo >> 6) + j * KSG_NWAVE + wave, bit));
    }
    if (tt) {
      tmax = wave_max_i32(tmax);
      if (lane == 0) atomicMax(s_tmax, tmax);
    }
    __syncthreads();
    for (uint32_t k = tid; k < d.n_domains_total; k += KSG_NT) dpart[k] = ANTI ? s_dcount[k] : 0;
    if (tid == 0) dpart[d.n_domains_total] = tt ? *s_tmax : 0;
    return;
  }
  const SC m = scan_pod<R, ANTI, false, SC>(d, c, tid, wave, bit, s_score, lds_dcount ? s_dcount : nullptr,
                                            phase == 2 ? dglobal : nullptr, nullptr, nullptr, nullptr, nullptr,
                                            fail_out, ext ? s_tmax : nullptr);
  if (mode == KSG_MODE_EVAL) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t n = d.lo + j * KSG_NT + tid;
      if (n < d.hi) {
        const SC v = s_score[j * KSG_NT + tid];
        score_out[n - d.lo] = v == T::none ? KSG_SCORE_NONE : (int64_t)v;
      }
    }
    return;
  }
  SC M;
  uint64_t k;
  reduce_ties<R, SC>(d, m, tid, lane, wave, s_score, s_wmax, s_wcnt, s_tie, M, k);
  for (uint32_t w = tid; w < d.nwords; w += KSG_NT) words[w] = s_tie[w];
  if (tid == 0) {
    hdr->max_score = M == T::none ? KSG_SCORE_NONE : (int64_t)M;
    hdr->tie_count = M == T::none ? 0 : k;
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
                                                       uint32_t out_idx, int64_t* summary,
                                                       const ksg_pod_ext* ext) {
  const uint32_t lane = threadIdx.x;
  const KsgMerged mg = ksg_merge_summary(records, rec_bytes, world, d.empty_priorities);
  const int64_t M = mg.max_score;
  const uint64_t k = mg.tie_count;
  if (mode == 0) {
    if (lane == 0) {
      summary[0] = M;
      summary[1] = (int64_t)k;
      summary[2] = mg.error;
    }
    return;
  }
  if (mg.error) {
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
    ix = ksg_rng_draw(d.draws, rng) % k;
    rng += ksg_rng_step(d.draws);
    if (lane == 0) *rng_io = rng;
  } else {
    ix = tie_index % k;
  }
  // descending rank order: highest shard first (generic_scheduler.go:88-95)
  uint64_t lix = 0, kg = 0;
  const int32_t owner = ksg_merge_owner(records, rec_bytes, world, M, ix, &lix, &kg);
  if (owner < 0) {
    if (lane == 0) out[out_idx] = KSG_OUT_ERROR;
    return;
  }
  const uint8_t* rec = records + (size_t)owner * rec_bytes;
  const uint64_t* words = reinterpret_cast<const uint64_t*>(rec + sizeof(KsgRecordHdr));
  const uint32_t nwords = (rec_bytes - (uint32_t)sizeof(KsgRecordHdr)) / 8;
  const int32_t win = select_tie(words, nwords, kg - 1 - lix, lane, shard_wlo[owner] * 64);
  if (win < 0) {
    if (lane == 0) out[out_idx] = KSG_OUT_ERROR;
    return;
  }
  commit_pod_wave(d, pods[0], ids, (uint32_t)win, lane, ext);
  if (lane == 0) out[out_idx] = win;
}

// ============================================================================
// Static per-node tables (once per ksg_set_cluster): LabelsPresence fit bitmap
// (predicates.go:215-229), EqualPriority + LabelPreference static score
// (generic_scheduler.go:180-195, priorities.go:109-134), anti-affinity domain
// and ServiceAffinity pair per node. One thread per node.
// ============================================================================

// pair_keys[p] carries KSG_PAIR_INVALID for pairs SelectorFromSet rejects
__device__ __forceinline__ uint32_t pair_key_of(const uint32_t* pair_keys, uint32_t p) {
  return pair_keys[p] & ~KSG_PAIR_INVALID;
}

__device__ __forceinline__ bool node_has_key(const uint32_t* pairs, uint32_t np,
                                             const uint32_t* pair_keys, uint32_t key) {
  for (uint32_t i = 0; i < np; ++i)
    if (pair_key_of(pair_keys, pairs[i]) == key) return true;
  return false;
}

__global__ void ksg_static_kernel(KsgStaticCfg sc, uint32_t n_nodes, const ksg_node* __restrict__ nodes,
                                  const uint32_t* __restrict__ node_pairs,
                                  const uint32_t* __restrict__ pair_keys,
                                  const int32_t* __restrict__ dom_of_pair,  // [n_anti][n_pairs]
                                  uint32_t n_pairs, uint32_t nw, uint64_t* static_fit,
                                  int64_t* static_score, int32_t* anti_domain, int32_t* aff_pair) {
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  bool fits = true;
  int64_t score = 0;
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
      score = wsum(score, wmul(sc.w_pref[q], ok ? 10 : 0));
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
        if (pair_key_of(pair_keys, pairs[i]) == sc.aff_key[j])
          pr = (pair_keys[pairs[i]] & KSG_PAIR_INVALID) ? KSG_AFF_INVALID : (int32_t)pairs[i];
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

// ServiceAntiAffinity re-rank (ksg_window.hip): zmap[row][n/64] |= bit, row =
// the node's domain of the first anti priority, d0 for unlabelled nodes
__global__ void ksg_zonemap_kernel(uint32_t n_nodes, const int32_t* __restrict__ anti_domain, uint32_t d0,
                                   uint32_t nw, unsigned long long* zmap) {
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes) return;
  const int32_t z = anti_domain[n];
  const uint32_t row = z >= 0 ? (uint32_t)z : d0;
  atomicOr(zmap + (size_t)row * nw + (n >> 6), 1ULL << (n & 63));
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
// dynamic LDS = R*1024 scores + the anti-affinity domain counts
template <typename SC>
static size_t lds_bytes(int R, const KsgDev& d) {
  return (R > ScoreT<SC>::r_lds ? 0 : (size_t)R * KSG_NT * sizeof(SC)) + (size_t)d.n_domains_total * sizeof(int32_t) +
         16;  // + TaintTolerationPriority's max (extension)
}

template <typename K>
static void allow_big_lds(K kernel) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024 - 8 * 1024);
  (void)hipGetLastError();  // do not leave a sticky error behind
}

template <int R, bool ANTI, bool REG>
static hipError_t launch_batch_t(const KsgDev& d, const ksg_pod* pods, const uint32_t* ids, uint32_t n,
                                 uint64_t* rng, int32_t* out, const ksg_pod_ext* ext, hipStream_t st) {
  if (d.wide) {
    static bool once64 = (allow_big_lds(ksg_batch_kernel<R, ANTI, REG, int64_t>), true);
    (void)once64;
    hipLaunchKernelGGL((ksg_batch_kernel<R, ANTI, REG, int64_t>), dim3(1), dim3(KSG_NT), lds_bytes<int64_t>(R, d), st,
                       d, pods, ids, n, rng, out, ext);
    return hipGetLastError();
  }
  static bool once = (allow_big_lds(ksg_batch_kernel<R, ANTI, REG, int32_t>), true);
  (void)once;
  hipLaunchKernelGGL((ksg_batch_kernel<R, ANTI, REG, int32_t>), dim3(1), dim3(KSG_NT), lds_bytes<int32_t>(R, d), st, d,
                     pods, ids, n, rng, out, ext);
  return hipGetLastError();
}

template <bool ANTI>
static hipError_t launch_batch_a(int R, const KsgDev& d, const ksg_pod* pods, const uint32_t* ids, uint32_t n,
                                 uint64_t* rng, int32_t* out, const ksg_pod_ext* ext, hipStream_t st) {
  switch (R) {
    case 1: return launch_batch_t<1, ANTI, true>(d, pods, ids, n, rng, out, ext, st);
    case 2: return launch_batch_t<2, ANTI, true>(d, pods, ids, n, rng, out, ext, st);
    case 4: return launch_batch_t<4, ANTI, true>(d, pods, ids, n, rng, out, ext, st);
    case 8: return launch_batch_t<8, ANTI, false>(d, pods, ids, n, rng, out, ext, st);
    case 16: return launch_batch_t<16, ANTI, false>(d, pods, ids, n, rng, out, ext, st);
    case 32: return launch_batch_t<32, ANTI, false>(d, pods, ids, n, rng, out, ext, st);
    case 64: return launch_batch_t<64, ANTI, false>(d, pods, ids, n, rng, out, ext, st);
    case 128: return launch_batch_t<128, ANTI, false>(d, pods, ids, n, rng, out, ext, st);
  }
  return hipErrorInvalidValue;
}

template <int R, bool ANTI>
static hipError_t launch_scan_t(const KsgDev& d, const ksg_pod* pods, const uint32_t* ids, int mode, int phase,
                                uint8_t* fail_out, int64_t* score_out, uint8_t* record, int32_t* dpart,
                                const int32_t* dglobal, const ksg_pod_ext* ext, hipStream_t st) {
  if (d.wide) {
    static bool once64 = (allow_big_lds(ksg_scan_kernel<R, ANTI, int64_t>), true);
    (void)once64;
    hipLaunchKernelGGL((ksg_scan_kernel<R, ANTI, int64_t>), dim3(1), dim3(KSG_NT), lds_bytes<int64_t>(R, d), st, d,
                       pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext);
    return hipGetLastError();
  }
  static bool once = (allow_big_lds(ksg_scan_kernel<R, ANTI, int32_t>), true);
  (void)once;
  hipLaunchKernelGGL((ksg_scan_kernel<R, ANTI, int32_t>), dim3(1), dim3(KSG_NT), lds_bytes<int32_t>(R, d), st, d, pods,
                     ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext);
  return hipGetLastError();
}

template <bool ANTI>
static hipError_t launch_scan_a(int R, const KsgDev& d, const ksg_pod* pods, const uint32_t* ids, int mode,
                                int phase, uint8_t* fail_out, int64_t* score_out, uint8_t* record, int32_t* dpart,
                                const int32_t* dglobal, const ksg_pod_ext* ext, hipStream_t st) {
  switch (R) {
    case 1: return launch_scan_t<1, ANTI>(d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st);
    case 2: return launch_scan_t<2, ANTI>(d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st);
    case 4: return launch_scan_t<4, ANTI>(d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st);
    case 8: return launch_scan_t<8, ANTI>(d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st);
    case 16: return launch_scan_t<16, ANTI>(d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st);
    case 32: return launch_scan_t<32, ANTI>(d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st);
    case 64: return launch_scan_t<64, ANTI>(d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st);
    case 128: return launch_scan_t<128, ANTI>(d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st);
  }
  return hipErrorInvalidValue;
}

hipError_t ksg_launch_batch(int R, bool anti, const KsgDev& d, const ksg_pod* pods, const uint32_t* ids,
                            uint32_t n, uint64_t* rng, int32_t* out, hipStream_t st, const ksg_pod_ext* ext) {
  return anti ? launch_batch_a<true>(R, d, pods, ids, n, rng, out, ext, st)
              : launch_batch_a<false>(R, d, pods, ids, n, rng, out, ext, st);
}

hipError_t ksg_launch_scan(int R, bool anti, const KsgDev& d, const ksg_pod* pods, const uint32_t* ids, int mode,
                           int phase, uint8_t* fail_out, int64_t* score_out, uint8_t* record, int32_t* dpart,
                           const int32_t* dglobal, hipStream_t st, const ksg_pod_ext* ext) {
  return anti ? launch_scan_a<true>(R, d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext, st)
              : launch_scan_a<false>(R, d, pods, ids, mode, phase, fail_out, score_out, record, dpart, dglobal, ext,
                                     st);
}

hipError_t ksg_launch_decide(const KsgDev& d, const ksg_pod* pods, const uint32_t* ids,
                             const uint8_t* records, uint32_t rec_bytes, uint32_t world,
                             const uint32_t* shard_wlo, int mode, uint64_t tie_index,
                             uint64_t* rng, int32_t* out, uint32_t out_idx, int64_t* summary,
                             hipStream_t st, const ksg_pod_ext* ext) {
  hipLaunchKernelGGL(ksg_decide_kernel, dim3(1), dim3(64), 0, st, d, pods, ids, records, rec_bytes,
                     world, shard_wlo, mode, tie_index, rng, out, out_idx, summary, ext);
  return hipGetLastError();
}

hipError_t ksg_launch_static(const KsgStaticCfg& sc, uint32_t n_nodes, const ksg_node* nodes,
                             const uint32_t* node_pairs, const uint32_t* pair_keys,
                             const int32_t* dom_of_pair, uint32_t n_pairs, uint32_t nw,
                             uint64_t* static_fit, int64_t* static_score, int32_t* anti_domain,
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

// ksg_add_static_config: one slot pass of LabelsPresence / LabelPreference terms past the
// config's slots, evaluated from the node labels into scratch (fit words, scores), then folded
hipError_t ksg_launch_static_terms(const KsgStaticCfg& sc, uint32_t n_nodes, const ksg_node* nodes,
                                   const uint32_t* node_pairs, const uint32_t* pair_keys, uint32_t n_pairs, uint32_t nw,
                                   uint64_t* fit, int64_t* score, hipStream_t st) {
  const uint32_t blocks = (n_nodes + 255) / 256;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(ksg_static_kernel, dim3(blocks), dim3(256), 0, st, sc, n_nodes, nodes, node_pairs, pair_keys,
                     nullptr, n_pairs, nw, fit, score, nullptr, nullptr);
  return hipGetLastError();
}

// ksg_set_static_terms: the caller's static node terms folded into the
// config's (LabelsPresence predicates: AND of the fit words; LabelPreference
// priorities: Go-int sum of the scores). own_fit / own_score: 0 when the config
// set none (the arrays hold no terms yet: assign instead).
__global__ void ksg_static_fold_kernel(uint64_t* static_fit, int64_t* static_score, const uint64_t* xfit,
                                       const int64_t* xscore, uint32_t nw, uint32_t n, int own_fit, int own_score) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (xfit && t < nw) static_fit[t] = own_fit ? (static_fit[t] & xfit[t]) : xfit[t];
  if (xscore && t < n)
    static_score[t] = own_score ? (int64_t)((uint64_t)static_score[t] + (uint64_t)xscore[t]) : xscore[t];
}

hipError_t ksg_launch_static_fold(uint64_t* static_fit, int64_t* static_score, const uint64_t* xfit,
                                  const int64_t* xscore, uint32_t nw, uint32_t n, int own_fit, int own_score,
                                  hipStream_t st) {
  const uint32_t blocks = ((nw > n ? nw : n) + 255) / 256;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(ksg_static_fold_kernel, dim3(blocks), dim3(256), 0, st, static_fit, static_score, xfit, xscore,
                     nw, n, own_fit, own_score);
  return hipGetLastError();
}

hipError_t ksg_launch_zonemap(uint32_t n_nodes, const int32_t* anti_domain, uint32_t d0, uint32_t nw,
                              uint64_t* zmap, hipStream_t st) {
  const uint32_t blocks = (n_nodes + 255) / 256;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(ksg_zonemap_kernel, dim3(blocks), dim3(256), 0, st, n_nodes, anti_domain, d0, nw,
                     reinterpret_cast<unsigned long long*>(zmap));
  return hipGetLastError();
}

hipError_t ksg_launch_patch(const KsgPatch* patches, uint32_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(ksg_patch_kernel, dim3(1), dim3(64), 0, st, patches, n);
  return hipGetLastError();
}
