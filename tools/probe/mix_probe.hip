// mix_probe.hip — dev tool: the two-class IPv4 launch (k_ipv4_twoclass) on a
// received ACK/MTU mix, against variants of its shape.  One call over 1 M
// datagrams (40-byte ACKs and 1500-byte segments, valid headers) runs ≈ 14 %
// slower than the same datagrams repacked by class and verified in two calls
// (tools/ab_mix_split.py).  Variants (all VERIFY, outputs compared with the
// shipped kernel's):
//   ship     k_ipv4_twoclass<32> as shipped (78 VGPRs: 6 waves per SIMD)
//   u6       long class 16 lanes x 6 loads in flight (fewer VGPRs)
//   occ8     the shipped body under __launch_bounds__(256, 8): 8 waves per SIMD
//   u6occ8   both
//   spw16    16 datagrams per wave
// Launches are timed interleaved (20 launches x 7 rounds, HIP events).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 mix_probe.hip -o mix_probe
#include "../../tcpip_network_protocol_stack_amd/csrc/kernels/icsum_kernels.hip"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <random>
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

template <int SPW, int LU>
__device__ __forceinline__ void twoclass_body(uint8_t* __restrict__ dg, const uint64_t* __restrict__ offsets,
                                              uint64_t n, int mode, uint16_t* __restrict__ ip_ck,
                                              uint16_t* __restrict__ tcp_ck, uint8_t* __restrict__ status,
                                              const uint8_t* __restrict__ zpad) {
  __shared__ uint64_t lst[kBlock / 64][64][2];
  __shared__ uint32_t lseg[kBlock / 64][64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t* const zlast = reinterpret_cast<const uint32_t*>(zpad) + 7;
  const uint64_t seg = (uint64_t(blockIdx.x) * (kBlock / 64) + wv) * SPW + (lane < SPW ? lane : 0u);
  const bool valid = seg < n && lane < SPW;
  uint64_t s, e;
  seg_bounds(offsets, 0, 0, seg < n ? seg : n - 1, s, e);
  if (!valid) e = s;
  const bool is_short = e - s <= 64;
  const uint64_t lmask = __ballot(valid && !is_short);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(lmask >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(lmask), 0u));
  if (valid && !is_short) {
    lst[wv][rank][0] = s;
    lst[wv][rank][1] = e;
    lseg[wv][rank] = uint32_t(seg);
  }
  ipv4_item<1, 4, false, 0>(dg, s, is_short ? e : s, seg, valid && is_short, 0u, mode, ip_ck, tcp_ck, status, zpad,
                            zlast);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t nlong = uint32_t(__builtin_popcountll(lmask));
  const uint32_t g = lane >> 4, gl = lane & 15u;
  for (uint32_t r0 = 0; r0 < nlong; r0 += 4) {
    const uint32_t k = r0 + g;
    const bool mine = k < nlong;
    const uint32_t kc = mine ? k : 0u;
    const uint64_t ls = lst[wv][kc][0], le = mine ? lst[wv][kc][1] : ls;
    ipv4_item<16, LU, true, 3>(dg, ls, le, lseg[wv][kc], mine, gl, mode, ip_ck, tcp_ck, status, zpad, zlast);
  }
}

template <int SPW, int LU>
__global__ __launch_bounds__(kBlock) void k_mix(uint8_t* dg, const uint64_t* offsets, uint64_t n, int mode,
                                                uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status,
                                                const uint8_t* zpad) {
  twoclass_body<SPW, LU>(dg, offsets, n, mode, ip_ck, tcp_ck, status, zpad);
}

template <int SPW, int LU>
__global__ __launch_bounds__(kBlock, 8) void k_mix_occ8(uint8_t* dg, const uint64_t* offsets, uint64_t n, int mode,
                                                        uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status,
                                                        const uint8_t* zpad) {
  twoclass_body<SPW, LU>(dg, offsets, n, mode, ip_ck, tcp_ck, status, zpad);
}

void run() {
  constexpr uint64_t kN = 1 << 20;
  std::mt19937_64 rng(11);
  std::vector<uint64_t> off(kN + 1, 0);
  for (uint64_t i = 0; i < kN; ++i) off[i + 1] = off[i] + ((rng() & 1) ? 40 : 1500);
  const uint64_t bytes = off[kN];
  std::vector<uint8_t> h(bytes + 16);
  for (auto& b : h) b = uint8_t(rng());
  for (uint64_t i = 0; i < kN; ++i) {
    uint8_t* p = h.data() + off[i];
    const uint64_t L = off[i + 1] - off[i];
    p[0] = 0x45, p[1] = 0, p[2] = uint8_t(L >> 8), p[3] = uint8_t(L), p[6] = 0x40, p[7] = 0, p[8] = 64, p[9] = 6;
    p[32] = 0x50;
  }
  uint8_t* d;
  uint64_t* doff;
  void* zero;
  CK(hipMalloc(&d, h.size()));
  CK(hipMalloc(&doff, off.size() * 8));
  CK(hipMalloc(&zero, 256));
  CK(hipMemset(zero, 0, 256));
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(doff, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  const SegSpec sp{d, doff, 0, 0, kN, zero};
  uint16_t *ip, *tcp;
  uint8_t *st, *ref;
  CK(hipMalloc(&ip, kN * 2));
  CK(hipMalloc(&tcp, kN * 2));
  CK(hipMalloc(&st, kN));
  CK(hipMalloc(&ref, kN * 5));
  CK(launch_ipv4_tcp(sp, 2, ip, tcp, st, Geometry{16, 8, true, 3}, 0, nullptr));  // valid checksums
  const uint8_t* z = static_cast<const uint8_t*>(zero);
  struct V {
    const char* name;
    std::function<void()> f;
  };
  auto grid = [](int spw) { return dim3(uint32_t((kN + uint64_t(4 * spw) - 1) / uint64_t(4 * spw))); };
  std::vector<V> vs = {
      {"ship", [&] { CK(launch_ipv4_twoclass(sp, 1, ip, tcp, st, nullptr)); }},
      {"u6", [&] { hipLaunchKernelGGL((k_mix<32, 6>), grid(32), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"occ8", [&] { hipLaunchKernelGGL((k_mix_occ8<32, 8>), grid(32), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"u6occ8", [&] { hipLaunchKernelGGL((k_mix_occ8<32, 6>), grid(32), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"spw16", [&] { hipLaunchKernelGGL((k_mix<16, 8>), grid(16), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
  };
  std::vector<uint8_t> want(kN * 5), got(kN * 5);
  vs[0].f();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(want.data(), ip, kN * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(want.data() + kN * 2, tcp, kN * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(want.data() + kN * 4, st, kN, hipMemcpyDeviceToHost));
  size_t accept = 0;
  for (uint64_t i = 0; i < kN; ++i) accept += want[kN * 4 + i] == 0x0F;
  std::vector<std::vector<float>> t(vs.size());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (size_t v = 0; v < vs.size(); ++v) {  // correctness + warm-up
    CK(hipMemset(ip, 0x5A, kN * 2));
    CK(hipMemset(tcp, 0x5A, kN * 2));
    CK(hipMemset(st, 0x5A, kN));
    for (int i = 0; i < 30; ++i) vs[v].f();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), ip, kN * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(got.data() + kN * 2, tcp, kN * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(got.data() + kN * 4, st, kN, hipMemcpyDeviceToHost));
    if (got != want) {
      fprintf(stderr, "variant %s differs\n", vs[v].name);
      exit(2);
    }
  }
  for (int r = 0; r < 7; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      for (int i = 0; i < 5; ++i) vs[v].f();
      CK(hipEventRecord(a, nullptr));
      for (int i = 0; i < 20; ++i) vs[v].f();
      CK(hipEventRecord(b, nullptr));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      t[v].push_back(ms * 1e3f / 20);
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("{\"variant\": \"%s\", \"us_median\": %.2f, \"us_min\": %.2f, \"bytes\": %llu, \"accepted\": %zu}\n",
           vs[v].name, t[v][t[v].size() / 2], t[v][0], (unsigned long long)bytes, accept);
  }
}

}  // namespace
}  // namespace icsum

int main() {
  icsum::run();
  return 0;
}
