// Dev probe (round 6): can the host write a tick's descriptor and payload
// straight into device memory (fine-grained / uncached VRAM reached through
// the PCIe BAR), so a resident kernel polls and reads locally instead of
// pulling both over PCIe?  Steps, each in a child process (a host-side fault
// on an unmapped pointer ends only the child): allocate with
// hipExtMallocWithFlags(flag), write and read it from the host, then time
// per-tick round trips of a one-block resident kernel that polls a sequence
// word in that memory, sums the 1500-byte payload the host copied next to
// it, and stores the result + sequence into page-locked host memory — against
// the same kernel with mailbox and payload in page-locked host memory (the
// shipped tick server's layout).  One JSON line per variant.
//   hipcc --offload-arch=gfx950 -O3 vram_mailbox.hip -o vram_mailbox
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      std::exit(3);                                                           \
    }                                                                         \
  } while (0)

struct Box {
  uint64_t seq;      // host: the job's number (written after the payload)
  uint64_t quit;
  uint64_t pad[14];
};
constexpr uint32_t kMaxPay = 24576;
struct Res {
  uint64_t seq;  // device: the last job done
  uint64_t sum;
};

__global__ void k_server(Box* box, const uint8_t* payload, Res* res, uint32_t len) {
  const uint32_t lane = threadIdx.x;
  uint64_t expect = 1;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    uint64_t s = 0, q = 0;
    if (lane == 0) {
      do {
        s = __hip_atomic_load(&box->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        q = __hip_atomic_load(&box->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 300000000ull) q = 1;  // 3 s backstop
      } while (s < expect && !q);
    }
    q = __shfl(q, 0);
    if (q) break;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    // 16 lanes x up to 8 dwordx4 (k_tick's shape), byte sum
    uint32_t acc = 0;
    for (uint32_t o = lane * 16; o < len; o += 64 * 16) {
      uint4 v = *reinterpret_cast<const uint4*>(payload + o);
      acc += v.x + v.y + v.z + v.w;
    }
    for (int d = 32; d > 0; d >>= 1) acc += __shfl_down(acc, d);
    if (lane == 0) {
      res->sum = acc;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(&res->seq, expect, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    ++expect;
  }
}

int run(const char* name, int box_vram, int pay_vram, uint32_t plen) {
  // box_vram / pay_vram: 0 page-locked host memory (the shipped layout), 1
  // uncached VRAM the host writes through the BAR
  Box* box = nullptr;
  uint8_t* payload = nullptr;
  if (box_vram)
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&box), sizeof(Box), hipDeviceMallocUncached));
  else
    CK(hipHostMalloc(reinterpret_cast<void**>(&box), sizeof(Box), hipHostMallocCoherent));
  if (pay_vram)
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&payload), kMaxPay, hipDeviceMallocUncached));
  else
    CK(hipHostMalloc(reinterpret_cast<void**>(&payload), kMaxPay, hipHostMallocCoherent));
  Res* res = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&res), sizeof(Res), hipHostMallocCoherent));
  std::memset(res, 0, sizeof(Res));
  // the host touches the box directly (a fault here ends this child)
  volatile uint64_t* hs = &box->seq;
  *hs = 0;
  box->quit = 0;
  std::fprintf(stderr, "%s: host write ok, read back %llu\n", name, (unsigned long long)*hs);
  static uint8_t src[kMaxPay];
  for (uint32_t i = 0; i < plen; ++i) src[i] = uint8_t(i * 7 + 3);
  uint32_t w0 = 0;
  std::memcpy(&w0, src, 4);
  uint32_t want = 0;
  for (uint32_t i = 0; i < plen; i += 4) {
    uint32_t w = 0;
    std::memcpy(&w, src + i, 4);
    want += w;
  }
  std::memset(payload, 0, kMaxPay);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(k_server, dim3(1), dim3(64), 0, st, box, payload, res, (plen + 15) & ~15u);
  CK(hipGetLastError());
  std::vector<double> ts, tc;
  bool ok = true;
  for (uint64_t k = 1; k <= 3000; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(src, &k, 4);  // a different payload every job: a stale read shows in the sum
    std::memcpy(payload, src, plen);
    __builtin_ia32_sfence();  // the payload lands before the sequence word
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const double cus = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    __atomic_store_n(&box->seq, k, __ATOMIC_RELEASE);
    // a store to BAR-mapped VRAM can sit in the CPU's write-combining buffer
    // until something flushes it: without this fence the first runs saw
    // 1 s timeouts and a 10 ms p99 (profiles/r6_probe_vram_mailbox*.jsonl)
    __builtin_ia32_sfence();
    while (__atomic_load_n(&res->seq, __ATOMIC_ACQUIRE) < k) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {  // the job never arrived
        __atomic_store_n(&box->quit, 1, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(st);
        std::printf("{\"layout\": \"%s\", \"timeout_at_job\": %llu}\n", name, (unsigned long long)k);
        return 4;
      }
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (k > 100) {
      ts.push_back(us);
      tc.push_back(cus);
    }
    if (uint32_t(res->sum) != want - w0 + uint32_t(k)) ok = false;
  }
  __atomic_store_n(&box->quit, 1, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(st));
  std::sort(ts.begin(), ts.end());
  std::sort(tc.begin(), tc.end());
  std::printf("{\"layout\": \"%s\", \"bytes\": %u, \"p10_us\": %.2f, \"p50_us\": %.2f, \"p90_us\": %.2f, "
              "\"p99_us\": %.2f, \"copy_p50_us\": %.2f, \"copy_p90_us\": %.2f, \"sum_ok\": %s}\n",
              name, plen, ts[ts.size() / 10], ts[ts.size() / 2], ts[ts.size() * 9 / 10], ts[ts.size() * 99 / 100],
              tc[tc.size() / 2], tc[tc.size() * 9 / 10], ok ? "true" : "false");
  std::fflush(stdout);
  return ok ? 0 : 2;
}

int main() {
  const char* names[] = {"box_host_payload_host", "box_vram_payload_host", "box_vram_payload_vram"};
  const int bv[] = {0, 1, 1}, pv[] = {0, 0, 1};
  int rc_all = 0;
  for (int rep = 0; rep < 2; ++rep)
    for (uint32_t plen : {1500u, 24000u})
      for (int w = 0; w < 3; ++w) {
        std::fflush(stdout);
        const pid_t pid = fork();  // before any HIP call in this process
        if (pid == 0) _exit(run(names[w], bv[w], pv[w], plen));
        int st = 0;
        waitpid(pid, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st)) {
          std::printf("{\"layout\": \"%s\", \"bytes\": %u, \"child_status\": %d}\n", names[w], plen, st);
          rc_all = 1;
        }
      }
  return rc_all;
}
