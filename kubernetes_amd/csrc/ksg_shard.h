// ksg_shard.h — node sharding and the cross-shard winner rule, shared by the
// device decide kernel (ksg_kernels.hip), the runtime (ksg_runtime.cpp) and the
// host entry points ksg_shard_range / ksg_merge_records (include/kschedgpu.h).
//
// Shards are contiguous runs of 64-node words in name-rank order, so walking
// shards from the highest rank down visits ties in the reference's order
// (score desc, host desc; generic_scheduler.go:84-95, types.go:42-47).
#pragma once
#include "ksg_internal.h"

// words [a, b) of shard `rank` out of `world` over nw words
static inline KSG_HD void ksg_shard_words(uint32_t nw, uint32_t rank, uint32_t world, uint32_t* a, uint32_t* b) {
  *a = (uint32_t)((uint64_t)rank * nw / world);
  *b = (uint32_t)((uint64_t)(rank + 1) * nw / world);
}

static inline KSG_HD const KsgRecordHdr* ksg_rec(const uint8_t* records, uint32_t rec_bytes, uint32_t g) {
  return reinterpret_cast<const KsgRecordHdr*>(records + (size_t)g * rec_bytes);
}

// global best score M, tie count k (= sum of shard counts at M) and error flag
struct KsgMerged {
  int64_t max_score;
  uint64_t tie_count;
  int32_t error;
};

static inline KSG_HD KsgMerged ksg_merge_summary(const uint8_t* records, uint32_t rec_bytes, uint32_t world,
                                                 int32_t empty_priorities) {
  KsgMerged m{KSG_SCORE_NONE, 0, 0};
  for (uint32_t g = 0; g < world; ++g) {
    const KsgRecordHdr* h = ksg_rec(records, rec_bytes, g);
    if (h->error) m.error = 1;
    if (h->tie_count > 0 && h->max_score > m.max_score) m.max_score = h->max_score;
  }
  for (uint32_t g = 0; g < world; ++g) {
    const KsgRecordHdr* h = ksg_rec(records, rec_bytes, g);
    if (h->tie_count > 0 && h->max_score == m.max_score) m.tie_count += h->tie_count;
  }
  if (empty_priorities) m.tie_count = 0;  // all weights 0: empty HostPriorityList -> FitError
  return m;
}

// owner shard of global tie ix (0 = highest-ranked tie); *lix = index of that
// tie inside the owner, counted from the owner's highest rank. -1 if none.
static inline KSG_HD int32_t ksg_merge_owner(const uint8_t* records, uint32_t rec_bytes, uint32_t world,
                                             int64_t max_score, uint64_t ix, uint64_t* lix, uint64_t* kg) {
  for (int32_t g = (int32_t)world - 1; g >= 0; --g) {
    const KsgRecordHdr* h = ksg_rec(records, rec_bytes, (uint32_t)g);
    if (h->tie_count > 0 && h->max_score == max_score) {
      if (ix < h->tie_count) {
        *lix = ix;
        *kg = h->tie_count;
        return g;
      }
      ix -= h->tie_count;
    }
  }
  return -1;
}
