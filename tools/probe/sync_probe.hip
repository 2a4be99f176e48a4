// sync_probe.hip — dev tool: how a host thread learns that one small launch
// has finished.  Per-tick host batches (icsum_host.cpp's zero-copy path) cost
// one launch plus one wait; the wait, not the kernel, is most of it.  One
// IPv4 VERIFY launch over n MTU datagrams in HBM with its outputs written
// straight into coherent page-locked host memory, then:
//   sync      hipStreamSynchronize
//   evsync    hipEventRecord + hipEventSynchronize
//   evquery   hipEventRecord + spin on hipEventQuery
//   flagk     a one-thread kernel behind it on the stream stores a ticket
//             into page-locked memory; the host spins on that word
//   wvalue    hipStreamWriteValue64 of the ticket behind it; host spins
//   lastblk   the kernel itself: every block adds to a device counter after
//             its stores; the last one releases and stores the ticket
// Outputs are checked against the sync variant's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 sync_probe.hip -o sync_probe
#include "../../tcpip_network_protocol_stack_amd/csrc/kernels/icsum_kernels.hip"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

namespace icsum {
namespace {

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_flag(uint64_t* flag, uint64_t t) {
  __hip_atomic_store(flag, t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// k_ipv4_tcp<16, 8, true, 3> whose last block to finish stores the ticket
__global__ __launch_bounds__(kBlock) void k_ipv4_last(uint8_t* __restrict__ dg, uint64_t stride, uint64_t dlen,
                                                      uint64_t n, uint16_t* __restrict__ ip_ck,
                                                      uint16_t* __restrict__ tcp_ck, uint8_t* __restrict__ status,
                                                      const uint8_t* __restrict__ zpad, uint32_t* counter,
                                                      uint64_t* flag, uint64_t t) {
  ipv4_body<16, 8, true, 3>(dg, nullptr, stride, dlen, n, 1, ip_ck, tcp_ck, status, zpad, blockIdx.x, gridDim.x);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == gridDim.x) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag, t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[size_t(p * (v.size() - 1))];
}

using clk = std::chrono::steady_clock;
double us_since(clk::time_point a) { return std::chrono::duration<double, std::micro>(clk::now() - a).count(); }

void spin(volatile uint64_t* flag, uint64_t t) {
  const auto a = clk::now();
  while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < t)
    if (us_since(a) > 2e6) {
      fprintf(stderr, "flag %llu not seen\n", (unsigned long long)t);
      exit(3);
    }
}

void run() {
  constexpr uint64_t kMaxN = 4096, kL = 1500;
  uint8_t* d_dg;
  CK(hipMalloc(&d_dg, kMaxN * kL));
  CK(launch_fill_bytes(d_dg, kMaxN * kL, 0x10710002ull, 0, nullptr));
  CK(launch_ipv4_tcp_headers(d_dg, kL, kL, kMaxN, 0x10710002ull, 0, nullptr));
  void* zero;
  CK(hipMalloc(&zero, 256));
  CK(hipMemset(zero, 0, 256));
  uint8_t *h_ref, *h_out;
  CK(hipHostMalloc(reinterpret_cast<void**>(&h_ref), kMaxN * 5, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(reinterpret_cast<void**>(&h_out), kMaxN * 5, hipHostMallocCoherent | hipHostMallocMapped));
  uint64_t* flag;
  CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 256, hipHostMallocCoherent | hipHostMallocMapped));
  *flag = 0;
  uint32_t* counter;
  CK(hipMalloc(&counter, 256));
  CK(hipMemset(counter, 0, 256));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const Geometry geo{16, 8, true, 3};
  uint64_t ticket = 0;
  {  // host-side costs of one call: pointer query, launch issue
    std::vector<double> pq, li;
    for (int i = 0; i < 2000; ++i) {
      hipPointerAttribute_t a{};
      auto t0 = clk::now();
      CK(hipPointerGetAttributes(&a, h_out));
      pq.push_back(us_since(t0));
      const SegSpec sp{d_dg, nullptr, kL, kL, 1, zero};
      uint16_t* ip = reinterpret_cast<uint16_t*>(h_out);
      t0 = clk::now();
      CK(launch_ipv4_tcp(sp, 1, ip, ip + 1, h_out + 4, geo, 0, st));
      li.push_back(us_since(t0));
      CK(hipStreamSynchronize(st));
    }
    printf("{\"host_cost\": true, \"pointer_query_p50_us\": %.3f, \"launch_issue_p50_us\": %.3f}\n", pct(pq, 0.5),
           pct(li, 0.5));
  }
  const char* names[] = {"sync", "evsync", "evquery", "flagk", "wvalue", "lastblk"};
  for (uint64_t n : {1ull, 16ull, 256ull, 4096ull}) {
    const SegSpec sp{d_dg, nullptr, kL, kL, n, zero};
    for (int r = 0; r < 5; ++r)
      for (int var = 0; var < 6; ++var) {
        uint8_t* ob = var == 0 ? h_ref : h_out;
        uint16_t* ip = reinterpret_cast<uint16_t*>(ob);
        uint16_t* tcp = ip + n;
        uint8_t* status = reinterpret_cast<uint8_t*>(tcp + n);
        std::vector<double> v;
        int mism = 0;
        for (int i = 0; i < 400; ++i) {
          memset(ob, 0x5A, n * 5);
          const uint64_t t = ++ticket;
          const auto a = clk::now();
          if (var == 5) {
            const uint32_t blocks = uint32_t((n + 15) / 16);
            hipLaunchKernelGGL(k_ipv4_last, dim3(blocks), dim3(kBlock), 0, st, d_dg, kL, kL, n, ip, tcp, status,
                               static_cast<const uint8_t*>(zero), counter, flag, t);
          } else {
            CK(launch_ipv4_tcp(sp, 1, ip, tcp, status, geo, 0, st));
          }
          switch (var) {
            case 0: CK(hipStreamSynchronize(st)); break;
            case 1: CK(hipEventRecord(ev, st)); CK(hipEventSynchronize(ev)); break;
            case 2:
              CK(hipEventRecord(ev, st));
              while (hipEventQuery(ev) == hipErrorNotReady) {
              }
              break;
            case 3: hipLaunchKernelGGL(k_flag, dim3(1), dim3(1), 0, st, flag, t); spin(flag, t); break;
            case 4: CK(hipStreamWriteValue64(st, flag, t, 0)); spin(flag, t); break;
            case 5: spin(flag, t); break;
          }
          if (i >= 20) v.push_back(us_since(a));
          if (var && memcmp(ob, h_ref, n * 5)) ++mism;
        }
        CK(hipStreamSynchronize(st));
        printf("{\"variant\": \"%s\", \"n\": %llu, \"round\": %d, \"p10_us\": %.2f, \"p50_us\": %.2f, "
               "\"p90_us\": %.2f, \"mismatch\": %d}\n",
               names[var], (unsigned long long)n, r, pct(v, 0.1), pct(v, 0.5), pct(v, 0.9), mism);
        fflush(stdout);
      }
  }
}

}  // namespace
}  // namespace icsum

int main() {
  icsum::run();
  return 0;
}
