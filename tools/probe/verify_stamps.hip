// Dev probe (round 5): the stack receive tick as ONE call.
// Builds the kernel file with -DICSUM_STAMPS (diagnostic build: every block of
// k_ipv4_twoclass stores s_memrealtime — 100 MHz — at its start and end, and
// its HW_ID) and runs VERIFY on the stack tick's receive shape (256 Ki
// datagrams, half 40-byte ACKs, half 1500-byte segments, packed offsets; the
// launch the default dispatch takes: 16 datagrams per wave) alone — each call
// after a synchronize, HIP events around it — and back to back.  For the last
// alone call it prints the block timeline: kernel span (first start to last
// end; span_b2b_us: the same for the last back-to-back call), when the first and the last block started, and when 50 / 90 / 99 /
// 100 % of the blocks (and of the datagram bytes) had finished.
//   hipcc --offload-arch=gfx950 -O3 -DICSUM_STAMPS -I../../include \
//     -I../../tcpip_network_protocol_stack_amd/csrc/kernels verify_stamps.hip -o verify_stamps
#include "../../tcpip_network_protocol_stack_amd/csrc/kernels/icsum_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                    \
  do {                                                           \
    hipError_t e = (x);                                          \
    if (e != hipSuccess) {                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                              \
    }                                                            \
  } while (0)

__global__ void k_empty(uint32_t* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] = 1;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (1u << 18);
  std::mt19937_64 rng(11);
  std::vector<uint64_t> off(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) off[i + 1] = off[i] + ((rng() & 1) ? 40 : 1500);
  std::vector<uint8_t> h(off[n] + 64, 0x5a);
  for (uint64_t i = 0; i < n; ++i) {  // IPv4 / TCP fields where the kernel looks (verdicts need not pass)
    const uint64_t s = off[i], L = off[i + 1] - s;
    h[s] = 0x45;
    h[s + 2] = uint8_t(L >> 8);
    h[s + 3] = uint8_t(L);
    h[s + 9] = 6;
    h[s + 32] = 0x50;
  }
  void* zero;
  uint8_t *d, *st;
  uint64_t* doff;
  uint16_t *ip, *tcp;
  CK(hipMalloc(&zero, 64));
  CK(hipMemset(zero, 0, 64));
  CK(hipMalloc(&d, h.size()));
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&doff, (n + 1) * 8));
  CK(hipMemcpy(doff, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&ip, n * 2));
  CK(hipMalloc(&tcp, n * 2));
  CK(hipMalloc(&st, n));
  icsum::SegSpec sp{d, doff, 0, 0, n, zero};
  auto launch = [&]() { CK(icsum::launch_ipv4_twoclass(sp, 1, ip, tcp, st, 16, 0, nullptr)); };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 200; ++i) launch();
  CK(hipDeviceSynchronize());
  std::vector<float> alone, b2b;
  for (int i = 0; i < 50; ++i) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, nullptr));
    launch();
    CK(hipEventRecord(e1, nullptr));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    alone.push_back(ms * 1000.f);
  }
  static uint64_t stamps[1u << 16][3];
  const uint64_t blocks = (n + 63) / 64;
  CK(hipMemcpyFromSymbol(stamps, HIP_SYMBOL(icsum::g_block_stamps), sizeof(stamps)));
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, nullptr));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipEventRecord(e1, nullptr));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    b2b.push_back(ms * 1000.f / 20.f);
  }
  // the last back-to-back call's blocks: its span by the waves' own clock
  static uint64_t stamps_b2b[1u << 16][3];
  CK(hipMemcpyFromSymbol(stamps_b2b, HIP_SYMBOL(icsum::g_block_stamps), sizeof(stamps_b2b)));
  // the fixed cost of one launch from an idle stream, HIP events around it:
  // an empty kernel of one block and of the VERIFY launch's 4096 blocks
  std::vector<float> empty1, emptyN;
  for (int i = 0; i < 50; ++i)
    for (int which = 0; which < 2; ++which) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, nullptr));
      hipLaunchKernelGGL(k_empty, dim3(which ? uint32_t((n + 63) / 64) : 1u), dim3(256), 0, nullptr, nullptr);
      CK(hipEventRecord(e1, nullptr));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      (which ? emptyN : empty1).push_back(ms * 1000.f);
    }
  std::sort(empty1.begin(), empty1.end());
  std::sort(emptyN.begin(), emptyN.end());
  std::sort(alone.begin(), alone.end());
  std::sort(b2b.begin(), b2b.end());
  uint64_t t0 = ~0ull, t1 = 0, lastStart = 0;
  std::vector<uint64_t> ends, starts, dur;
  std::vector<double> endw;
  for (uint64_t b = 0; b < blocks; ++b) {
    t0 = std::min(t0, stamps[b][0]);
    t1 = std::max(t1, stamps[b][1]);
    lastStart = std::max(lastStart, stamps[b][0]);
  }
  for (uint64_t b = 0; b < blocks; ++b) {
    starts.push_back(stamps[b][0] - t0);
    ends.push_back(stamps[b][1] - t0);
    dur.push_back(stamps[b][1] - stamps[b][0]);
  }
  std::sort(starts.begin(), starts.end());
  std::sort(ends.begin(), ends.end());
  std::sort(dur.begin(), dur.end());
  uint64_t u0 = ~0ull, u1 = 0;
  for (uint64_t b = 0; b < blocks; ++b) {
    u0 = std::min(u0, stamps_b2b[b][0]);
    u1 = std::max(u1, stamps_b2b[b][1]);
  }
  auto q = [&](const std::vector<uint64_t>& v, double f) { return 0.01 * double(v[size_t(f * (v.size() - 1))]); };
  const double bytes = double(off[n]);
  std::printf("{\"n\": %llu, \"blocks\": %llu, \"bytes\": %.0f, \"alone_us_p50\": %.2f, \"b2b_us\": %.2f, "
              "\"span_us\": %.2f, \"span_b2b_us\": %.2f, \"start_us\": {\"p50\": %.2f, \"p90\": %.2f, \"last\": %.2f}, "
              "\"end_us\": {\"first\": %.2f, \"p50\": %.2f, \"p90\": %.2f, \"p99\": %.2f, \"last\": %.2f}, "
              "\"block_us\": {\"p10\": %.2f, \"p50\": %.2f, \"p90\": %.2f, \"max\": %.2f}, \"frac_alone\": %.4f, "
              "\"frac_span\": %.4f, \"empty_launch_us\": {\"one_block\": %.2f, \"same_grid\": %.2f}}\n",
              (unsigned long long)n, (unsigned long long)blocks, bytes, alone[alone.size() / 2], b2b[2],
              0.01 * double(t1 - t0), 0.01 * double(u1 - u0), q(starts, 0.5), q(starts, 0.9), q(starts, 1.0), q(ends, 0.0), q(ends, 0.5),
              q(ends, 0.9), q(ends, 0.99), q(ends, 1.0), q(dur, 0.1), q(dur, 0.5), q(dur, 0.9), q(dur, 1.0),
              bytes / (alone[alone.size() / 2] * 1e3) / 8000.0, bytes / (0.01 * double(t1 - t0) * 1e3) / 8000.0,
              empty1[empty1.size() / 2], emptyN[emptyN.size() / 2]);
  return 0;
}
