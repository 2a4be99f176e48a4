// csum_mix_probe.hip — dev tool: the plain checksum's two-class launch
// (k_checksum_twoclass) on the bimodal receive mix (2 M segments of 40-43 or
// 1460-1463 bytes, packed offsets, pseudo-header inits: bench_configs'
// "bimodal" row) against a block-list version (the shape that moved the
// fused IPv4 kernel, DESIGN.md §4 "Block lists"): the block's short segments
// on wave 0, one per lane, its long ones claimed four at a time by every wave
// from an LDS counter.  Outputs compared with the shipped kernel's; launches
// timed interleaved (20 x 7, HIP events).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 csum_mix_probe.hip -o csum_mix_probe
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

template <int SPW>
__global__ __launch_bounds__(kBlock) void k_blk(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                const uint32_t* __restrict__ init, const u32x4* __restrict__ zero16,
                                                uint16_t* __restrict__ out, uint64_t n) {
  constexpr uint32_t kPer = (kBlock / 64) * SPW;
  __shared__ uint64_t lst[kPer][2], sst[kPer][2];
  __shared__ uint32_t lseg[kPer], sseg[kPer];
  __shared__ uint32_t cnt[3];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t seg = (uint64_t(blockIdx.x) * (kBlock / 64) + wv) * SPW + (lane < SPW ? lane : 0u);
  const bool valid = seg < n && lane < SPW;
  const uint64_t c = seg < n ? seg : n - 1;
  const uint64_t s = off[c], e = valid ? off[c + 1] : s;
  const uint64_t a0 = s & ~uint64_t(15);
  const uint32_t nch = uint32_t(((e > s ? e - a0 : 0) + 15) >> 4);
  const bool is_short = nch <= 4;
  const uint64_t lmask = __ballot(valid && !is_short), smask = __ballot(valid && is_short);
  uint32_t lbase = 0, sbase = 0;
  if (lane == 0) {
    lbase = atomicAdd(&cnt[0], uint32_t(__builtin_popcountll(lmask)));
    sbase = atomicAdd(&cnt[1], uint32_t(__builtin_popcountll(smask)));
  }
  lbase = __builtin_amdgcn_readfirstlane(lbase);
  sbase = __builtin_amdgcn_readfirstlane(sbase);
  const uint32_t lr = __builtin_amdgcn_mbcnt_hi(uint32_t(lmask >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(lmask), 0u));
  const uint32_t sr = __builtin_amdgcn_mbcnt_hi(uint32_t(smask >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(smask), 0u));
  if (valid && !is_short) {
    lst[lbase + lr][0] = s;
    lst[lbase + lr][1] = e;
    lseg[lbase + lr] = uint32_t(seg);
  }
  if (valid && is_short) {
    sst[sbase + sr][0] = s;
    sst[sbase + sr][1] = e;
    sseg[sbase + sr] = uint32_t(seg);
  }
  __syncthreads();
  const uint32_t nlong = cnt[0], nshort = cnt[1];
  if (wv == 0)
    for (uint32_t r0 = 0; r0 < nshort; r0 += 64) {  // uniform
      const uint32_t k = r0 + lane;
      const bool mine = k < nshort;
      const uint32_t kc = mine ? k : 0u;
      const uint64_t ss = sst[kc][0], se = mine ? sst[kc][1] : ss;
      const uint64_t b0 = ss & ~uint64_t(15), span = se > ss ? se - b0 : 0;
      const uint32_t nc = uint32_t((span + 15) >> 4);
      const u32x4* p = reinterpret_cast<const u32x4*>(bytes + b0);
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(nc ? p + (uint32_t(u) < nc ? uint32_t(u) : nc - 1) : zero16);
      const uint32_t i0 = init[sseg[kc]];
      uint32_t ev = 0, od = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t at = uint64_t(u) << 4;
        const uint32_t lo = u == 0 ? uint32_t(ss) & 15u : 0u;
        const uint32_t hi = at >= span ? 0u : (span - at >= 16 ? 16u : uint32_t(span - at));
        acc_chunk(v[u] & byte_range_mask(lo, hi), ev, od);
      }
      if (mine) out[sseg[kc]] = fold_value(i0 + combine_roles(ev, od, uint32_t(ss) & 1u));
    }
  const uint32_t g = lane >> 4, gl = lane & 15u;
  for (;;) {
    uint32_t r0 = 0;
    if (lane == 0) r0 = atomicAdd(&cnt[2], 4u);
    r0 = __builtin_amdgcn_readfirstlane(r0);
    if (r0 >= nlong) break;
    const uint32_t k = r0 + g;
    const bool mine = k < nlong;
    const uint32_t kc = mine ? k : 0u;
    const uint64_t ls = mine ? lst[kc][0] : 0, le = mine ? lst[kc][1] : 0;
    const uint32_t lsg = lseg[kc];
    const uint32_t i0 = init[lsg];
    uint32_t ev = 0, od = 0;
    range_sums_line_primed<16, 8, true>(bytes, ls, le, gl, ev, od);
    const uint32_t tot = group_sum<16>(combine_roles(ev, od, uint32_t(ls) & 1u));
    if (mine && gl == 15) out[lsg] = fold_value(i0 + tot);
  }
}

void run() {
  constexpr uint64_t kN = 2 << 20;
  std::mt19937_64 rng(0x10710006);
  std::vector<uint64_t> off(kN + 1, 0);
  for (uint64_t i = 0; i < kN; ++i) off[i + 1] = off[i] + ((rng() & 1) ? 40 : 1460) + (rng() & 3);
  std::vector<uint8_t> h(off[kN] + 16);
  for (auto& b : h) b = uint8_t(rng());
  std::vector<uint32_t> hi(kN);
  for (auto& x : hi) x = uint32_t(rng() % 400000);
  uint8_t* d;
  uint64_t* doff;
  uint32_t* init;
  void* zero;
  uint16_t* out;
  CK(hipMalloc(&d, h.size()));
  CK(hipMalloc(&doff, off.size() * 8));
  CK(hipMalloc(&init, kN * 4));
  CK(hipMalloc(&zero, 256));
  CK(hipMalloc(&out, kN * 2));
  CK(hipMemset(zero, 0, 256));
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(doff, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(init, hi.data(), kN * 4, hipMemcpyHostToDevice));
  const SegSpec sp{d, doff, 0, 0, kN, zero};
  const u32x4* z = static_cast<const u32x4*>(zero);
  auto grid = [](int spw) { return dim3(uint32_t((kN + uint64_t(4 * spw) - 1) / uint64_t(4 * spw))); };
  struct V {
    const char* name;
    std::function<void()> f;
  };
  std::vector<V> vs = {
      {"ship16", [&] { CK(launch_checksum_twoclass(sp, init, nullptr, out, 0, 16, nullptr)); }},
      {"ship32", [&] { CK(launch_checksum_twoclass(sp, init, nullptr, out, 0, 32, nullptr)); }},
      {"blk16", [&] { hipLaunchKernelGGL(k_blk<16>, grid(16), dim3(kBlock), 0, nullptr, d, doff, init, z, out, kN); }},
      {"blk32", [&] { hipLaunchKernelGGL(k_blk<32>, grid(32), dim3(kBlock), 0, nullptr, d, doff, init, z, out, kN); }},
      {"blk64", [&] { hipLaunchKernelGGL(k_blk<64>, grid(64), dim3(kBlock), 0, nullptr, d, doff, init, z, out, kN); }},
  };
  std::vector<uint16_t> want(kN), got(kN);
  vs[0].f();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(want.data(), out, kN * 2, hipMemcpyDeviceToHost));
  for (size_t v = 0; v < vs.size(); ++v) {
    CK(hipMemset(out, 0x5A, kN * 2));
    for (int i = 0; i < 30; ++i) vs[v].f();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), out, kN * 2, hipMemcpyDeviceToHost));
    if (got != want) {
      fprintf(stderr, "variant %s differs\n", vs[v].name);
      exit(2);
    }
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<std::vector<float>> t(vs.size());
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
    printf("{\"variant\": \"%s\", \"us_median\": %.2f, \"us_min\": %.2f, \"bytes\": %llu}\n", vs[v].name,
           t[v][t[v].size() / 2], t[v][0], (unsigned long long)off[kN]);
  }
}

}  // namespace
}  // namespace icsum

int main() {
  icsum::run();
  return 0;
}
