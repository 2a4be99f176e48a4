// Dev probe (round 5): what k_span's window pass costs.  Built twice from the
// kernel file: as shipped, and with -DICSUM_SPAN_PROBE_STREAM_ONLY (every
// window only loaded and written to LDS; results wrong, time only).  Times the
// checksum span launch on the transmit mix (256 Ki segments of 40..1040 B)
// and on 1 M x 770 B offsets at S = 8, 16, 32, 63 segments per span, back to
// back (HIP events around 20 launches, median of 5).
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

int main() {
  void* zero;
  CK(hipMalloc(&zero, 64));
  CK(hipMemset(zero, 0, 64));
  std::mt19937_64 rng(3);
#ifdef ICSUM_SPAN_PROBE_STREAM_ONLY
  const char* build = "stream_only";
#else
  const char* build = "shipped";
#endif
  for (int shape = 0; shape < 2; ++shape)
  for (uint32_t S : {8u, 16u, 32u, 63u}) {
    const uint64_t n = shape == 0 ? (1u << 18) : (1u << 20);
    std::vector<uint64_t> off(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) off[i + 1] = off[i] + (shape == 0 ? 40 + rng() % 1001 : 770);
    uint8_t* d[2];
    uint64_t* doff[2];
    uint16_t* dout;
    for (int r = 0; r < 2; ++r) {
      CK(hipMalloc(&d[r], off[n] + 64));
      CK(hipMemset(d[r], 0x5a, off[n] + 64));
      CK(hipMalloc(&doff[r], (n + 1) * 8));
      CK(hipMemcpy(doff[r], off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    }
    CK(hipMalloc(&dout, n * 2));
    auto launch = [&](int i) {
      icsum::SegSpec sp{d[i & 1], doff[i & 1], 0, 0, n, zero};
      CK(icsum::launch_tile_checksum(sp, nullptr, nullptr, dout, 0, S, nullptr));
    };
    for (int i = 0; i < 50; ++i) launch(i);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, nullptr));
      for (int i = 0; i < 20; ++i) launch(i);
      CK(hipEventRecord(e1, nullptr));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1000.f / 20.f);
    }
    std::sort(ts.begin(), ts.end());
    std::printf("{\"build\": \"%s\", \"shape\": \"%s\", \"S\": %u, \"bytes\": %llu, \"us\": %.2f, \"frac\": %.4f}\n",
                build, shape == 0 ? "tx256k" : "u770_1m", S, (unsigned long long)off[n], ts[2],
                off[n] / (ts[2] * 1e3) / 8000.0);
    for (int r = 0; r < 2; ++r) {
      CK(hipFree(d[r]));
      CK(hipFree(doff[r]));
    }
    CK(hipFree(dout));
  }
  return 0;
}
