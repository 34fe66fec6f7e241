// ksg_plain_large.hip — the plain window resolver's large-shard instantiations (P = 16, 32 words
// per lane: shards past 512 64-node words, BASELINE config 5) and its extension (XS) instantiations
// at every P, in a translation unit of their own,
// compiled with the max-ILP machine scheduler (__graft_entry__.build: -mllvm
// -amdgpu-sched-strategy=max-ilp). Everything else about them is ksg_plain.hip; see its host
// launcher section for why and for the measurement.
#define KSG_PLAIN_LARGE_TU 1
#include "ksg_plain.hip"
