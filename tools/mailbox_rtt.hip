// Host <-> resident-kernel mailbox round trip over host-mapped pinned memory
// (measurement tool for the drop-in per-pod server, not product code).
// Host writes seq i (and a payload of `pay` bytes, each 64-B line tagged with i);
// one resident workgroup polls with system-scope loads, reads the payload,
// answers with i; the host spins on the answer. Prints p50/p90/p99 in us.
// build: hipcc --offload-arch=gfx950 -O3 tools/mailbox_rtt.hip -o tools/bin/mailbox_rtt
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct alignas(64) Req { uint32_t seq; uint32_t pad[15]; };
struct alignas(64) Resp { uint32_t seq; uint32_t val; uint32_t pad[14]; };

__device__ __forceinline__ uint32_t sys_ld(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// mode 0: poll seq only; mode 1: poll seq, then read the payload lines (second round trip);
// mode 2: every poll reads seq + payload in one go (one load per lane), accepted when every
// line's tag equals the seq
__global__ __launch_bounds__(64) void rtt_kernel(Req* req, uint32_t* pay, uint32_t pay_dw, Resp* resp, uint32_t n,
                                                 int mode, uint32_t* hang) {
  const uint32_t lane = threadIdx.x;
  const uint64_t t_start = wall_clock64();
  const uint64_t limit = 100ull * 1000 * 1000 * 20;  // 20 s at 100 MHz
  for (uint32_t i = 1; i <= n; ++i) {
    uint32_t sum = 0;
    if (mode == 2) {
      for (;;) {
        uint32_t v = lane < pay_dw ? sys_ld(pay + lane) : i;
        // tag dword: the last dword of each 64-B line (16 dwords)
        const bool tag_lane = (lane & 15) == 15 || lane + 1 == pay_dw;
        const bool ok = __all(!(lane < pay_dw && tag_lane) || v == i);
        if (ok) { sum = v; break; }
        if (wall_clock64() - t_start > limit) { if (lane == 0) *hang = 1; return; }
      }
    } else {
      for (;;) {
        const uint32_t s = sys_ld(&req->seq);
        if (s == i) break;
        if (wall_clock64() - t_start > limit) { if (lane == 0) *hang = 1; return; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (mode == 1 && lane < pay_dw) sum = sys_ld(pay + lane);
    }
    sum = __reduce_add_sync(~0ull, sum);
    if (lane == 0) {
      sys_st(&resp->val, sum);
      __hip_atomic_store(&resp->seq, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const uint32_t pay_dw = argc > 2 ? (uint32_t)atoi(argv[2]) : 64;
  const uint32_t n = argc > 3 ? (uint32_t)atoi(argv[3]) : 20000;
  Req* req; Resp* resp; uint32_t* pay; uint32_t* hang;
  hipHostMalloc((void**)&req, sizeof(Req), hipHostMallocCoherent | hipHostMallocMapped);
  hipHostMalloc((void**)&resp, sizeof(Resp), hipHostMallocCoherent | hipHostMallocMapped);
  hipHostMalloc((void**)&pay, 4096, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostMalloc((void**)&hang, 64, hipHostMallocCoherent | hipHostMallocMapped);
  req->seq = 0; resp->seq = 0; *hang = 0;
  for (uint32_t k = 0; k < 1024; ++k) pay[k] = 0;
  Req* dreq; Resp* dresp; uint32_t* dpay; uint32_t* dhang;
  hipHostGetDevicePointer((void**)&dreq, req, 0);
  hipHostGetDevicePointer((void**)&dresp, resp, 0);
  hipHostGetDevicePointer((void**)&dpay, pay, 0);
  hipHostGetDevicePointer((void**)&dhang, hang, 0);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipLaunchKernelGGL(rtt_kernel, dim3(1), dim3(64), 0, st, dreq, dpay, pay_dw, dresp, n, mode, dhang);
  std::vector<double> us;
  us.reserve(n);
  volatile uint32_t* vreq = &req->seq;
  volatile uint32_t* vresp = &resp->seq;
  volatile uint32_t* vpay = pay;
  bool bad = false;
  for (uint32_t i = 1; i <= n && !bad; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0; k < pay_dw; ++k) vpay[k] = (mode == 2 && ((k & 15) == 15 || k + 1 == pay_dw)) ? i : k;
    __atomic_store_n(vreq, i, __ATOMIC_RELEASE);
    while (__atomic_load_n(vresp, __ATOMIC_ACQUIRE) != i) {
      if (*hang) { bad = true; break; }
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 5.0) { bad = true; break; }
    }
    const auto t1 = std::chrono::steady_clock::now();
    us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  if (bad) {
    // let the kernel drain: answer nothing more; it exits at its own limit
    fprintf(stderr, "round trip stalled\n");
  }
  hipStreamSynchronize(st);
  std::sort(us.begin() + std::min<size_t>(us.size(), 100), us.end());
  std::vector<double> s(us.begin() + std::min<size_t>(us.size(), 100), us.end());
  auto q = [&](double f) { return s.empty() ? -1.0 : s[(size_t)(f * (s.size() - 1))]; };
  printf("{\"mode\": %d, \"payload_dwords\": %u, \"n\": %zu, \"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f, \"min_us\": %.2f}\n",
         mode, pay_dw, s.size(), q(0.5), q(0.9), q(0.99), q(0.0));
  return bad ? 1 : 0;
}
