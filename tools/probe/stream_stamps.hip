// Dev probe (round 5): where k_stream's waves spend their cycles.  Builds the
// kernel file itself with -DICSUM_STAMPS (a diagnostic build: every wave adds
// up s_memtime deltas — working on tiles, waiting at the tile barrier,
// finishing the last tile — into g_stream_stamps) and runs the checksum tile
// launch on 1 M x 770 B and on 256 Ki segments of 40..1040 B, printing per
// role (stream waves, metadata wave) the mean cycles per block of each bucket
// and the launch's HIP-event time.
//   hipcc --offload-arch=gfx950 -O3 -DICSUM_STAMPS -I../../include \
//     -I../../tcpip_network_protocol_stack_amd/csrc/kernels stream_stamps.hip -o stream_stamps
#include "../../tcpip_network_protocol_stack_amd/csrc/kernels/icsum_kernels.hip"

#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

int main() {
  void* zero;
  CK(hipMalloc(&zero, 64));
  CK(hipMemset(zero, 0, 64));
  std::mt19937_64 rng(7);
  for (int shape = 0; shape < 2; ++shape) {
    const uint64_t n = shape == 0 ? (1u << 20) : (1u << 18);
    std::vector<uint64_t> off(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) off[i + 1] = off[i] + (shape == 0 ? 770 : 40 + rng() % 1001);
    uint8_t* d;
    uint64_t* doff;
    uint16_t* dout;
    CK(hipMalloc(&d, off[n] + 64));
    CK(hipMemset(d, 0x5a, off[n] + 64));
    CK(hipMalloc(&doff, (n + 1) * 8));
    CK(hipMemcpy(doff, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&dout, n * 2));
    for (uint32_t T : {128u, 256u}) {
      icsum::SegSpec sp{d, doff, 0, 0, n, zero};
      for (int i = 0; i < 10; ++i)
        CK(icsum::launch_tile_checksum(sp, nullptr, nullptr, dout, 0, T, 0, nullptr, true));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, nullptr));
      CK(icsum::launch_tile_checksum(sp, nullptr, nullptr, dout, 0, T, 0, nullptr, true));
      CK(hipEventRecord(e1, nullptr));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      static uint64_t st[4096][5][4];
      CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(icsum::g_stream_stamps), sizeof(st)));
      const uint64_t tiles = (n + T - 1) / T, blocks = tiles < 1024 ? tiles : 1024;
      double acc[2][4] = {};
      for (uint64_t b = 0; b < blocks; ++b)
        for (int w = 0; w < 5; ++w)
          for (int k = 0; k < 4; ++k) acc[w == 4][k] += double(st[b][w][k]) / (w == 4 ? 1.0 : 4.0);
      std::printf("{\"shape\": \"%s\", \"T\": %u, \"blocks\": %llu, \"us\": %.2f, "
                  "\"stream_work\": %.0f, \"stream_barrier\": %.0f, \"stream_last\": %.0f, \"tiles_per_block\": %.2f, "
                  "\"meta_work\": %.0f, \"meta_barrier\": %.0f, \"meta_last\": %.0f}\n",
                  shape == 0 ? "u770_1m" : "tx256k", T, (unsigned long long)blocks, ms * 1000.0,
                  acc[0][0] / blocks, acc[0][1] / blocks, acc[0][2] / blocks, acc[0][3] / blocks, acc[1][0] / blocks,
                  acc[1][1] / blocks, acc[1][2] / blocks);
      std::fflush(stdout);
    }
    CK(hipFree(d));
    CK(hipFree(doff));
    CK(hipFree(dout));
  }
  return 0;
}
