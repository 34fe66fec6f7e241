// ksg_admit.hip — the kubelet's admission re-check of its own pods with the
// scheduler's predicates (pkg/kubelet/kubelet.go:1716-1771, handleNotFittingPods):
//
//   checkNodeSelectorMatching -> scheduler.PodMatchesNodeLabels   predicates.go:161-167
//   checkCapacityExceeded     -> scheduler.CheckPodsExceedingCapacity over the
//                                pods in creation order          predicates.go:104-124
//
// Many nodes' admission sets are checked in one launch: one lane per set walks
// the set's pods in the caller's order (the greedy capacity pass accumulates
// only the pods that fit, so it is sequential within a set and parallel across
// sets). Node label pairs and pod nodeSelector pairs are interned ids, as in
// the scheduling path; SelectorFromSet's invalid-selector trap is resolved by
// the host ingest (n_sel == 0: matches every node).
#include <hip/hip_runtime.h>

#include "ksg_internal.h"

#define KSG_ADMIT_NT 64

__global__ __launch_bounds__(KSG_ADMIT_NT) void ksg_admit_kernel(const ksg_admission_set* __restrict__ sets,
                                                                uint32_t n_sets, const ksg_pod* __restrict__ pods,
                                                                const uint32_t* __restrict__ ids,
                                                                const uint32_t* __restrict__ pairs, int mode,
                                                                uint8_t* __restrict__ out) {
  const uint32_t s = blockIdx.x * KSG_ADMIT_NT + threadIdx.x;
  if (s >= n_sets) return;
  const ksg_admission_set set = sets[s];
  const bool match_on = (mode & KSG_ADMIT_MODE_SELECTOR) != 0;
  const bool cap_on = (mode & KSG_ADMIT_MODE_CAPACITY) != 0;
  // CheckPodsExceedingCapacity: totals from the capacity, requested sums of the
  // pods that fit so far; Go int64 arithmetic wraps (done in uint64)
  const int64_t total_c = set.cap_milli_cpu, total_m = set.cap_memory;
  int64_t req_c = 0, req_m = 0;
  for (uint32_t i = set.pod_off; i < set.pod_off + set.n_pods; ++i) {
    const ksg_pod p = pods[i];
    uint8_t code = KSG_ADMIT_OK;
    if (match_on) {  // PodMatchesNodeLabels: every nodeSelector pair on the node
      for (uint32_t k = 0; k < p.n_sel && code == KSG_ADMIT_OK; ++k) {
        const uint32_t want = ids[p.sel_off + k];
        bool found = false;
        for (uint32_t l = 0; l < set.n_labels; ++l) found |= want != 0 && pairs[set.label_off + l] == want;
        if (!found) code = KSG_ADMIT_NODESELECTOR;
      }
    }
    if (cap_on && code == KSG_ADMIT_OK) {
      const bool fits_c = total_c == 0 || (int64_t)((uint64_t)total_c - (uint64_t)req_c) >= p.milli_cpu;
      const bool fits_m = total_m == 0 || (int64_t)((uint64_t)total_m - (uint64_t)req_m) >= p.memory;
      if (fits_c && fits_m) {
        req_c = (int64_t)((uint64_t)req_c + (uint64_t)p.milli_cpu);
        req_m = (int64_t)((uint64_t)req_m + (uint64_t)p.memory);
      } else {
        code = KSG_ADMIT_CAPACITY;
      }
    }
    out[i] = code;
  }
}

hipError_t ksg_launch_admit(const ksg_admission_set* sets, uint32_t n_sets, const ksg_pod* pods,
                            const uint32_t* ids, const uint32_t* pairs, int mode, uint8_t* out, hipStream_t st) {
  if (n_sets == 0) return hipSuccess;
  hipLaunchKernelGGL(ksg_admit_kernel, dim3((n_sets + KSG_ADMIT_NT - 1) / KSG_ADMIT_NT), dim3(KSG_ADMIT_NT), 0, st,
                     sets, n_sets, pods, ids, pairs, mode, out);
  return hipGetLastError();
}
