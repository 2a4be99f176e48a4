// mixed_probe.hip — dev tool: BASELINE config 4 (1 M segments, log-uniform
// 64 B - 64 KiB, packed offsets, pseudo-header inits) under its shipped single
// launch (k_checksum<64,8,nt,line grid>: one wave per segment, the whole-batch
// plan) against a block-list launch in the style of the two-class kernels:
// the block reads 4 x SPW segment bounds into a medium (<= T bytes, 16 lanes
// each, 4 per claim) and a long list (64 lanes each, 1 per claim) in LDS and
// every wave claims medium groups, then long segments, from LDS counters —
// so the segments of a few hundred bytes stop taking a wave each.  Outputs
// compared with the shipped kernel's; launches timed interleaved.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 mixed_probe.hip -o mixed_probe
#include "../../tcpip_network_protocol_stack_amd/csrc/kernels/icsum_kernels.hip"

#include <math.h>
#include <stdio.h>

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

template <int SPW, uint32_t T>
__global__ __launch_bounds__(kBlock) void k_blk(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                const uint32_t* __restrict__ init, uint16_t* __restrict__ out,
                                                uint64_t n) {
  constexpr uint32_t kPer = (kBlock / 64) * SPW;
  __shared__ uint64_t mst[kPer][2], lst[kPer][2];
  __shared__ uint32_t mseg[kPer], lseg[kPer];
  __shared__ uint32_t cnt[4];  // medium, long, medium claimed, long claimed
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t seg = (uint64_t(blockIdx.x) * (kBlock / 64) + wv) * SPW + (lane < SPW ? lane : 0u);
  const bool valid = seg < n && lane < SPW;
  const uint64_t c = seg < n ? seg : n - 1;
  const uint64_t s = off[c], e = valid ? off[c + 1] : s;
  const bool med = e - s <= T;
  const uint64_t mmask = __ballot(valid && med), lmask = __ballot(valid && !med);
  uint32_t mb = 0, lb = 0;
  if (lane == 0) {
    mb = atomicAdd(&cnt[0], uint32_t(__builtin_popcountll(mmask)));
    lb = atomicAdd(&cnt[1], uint32_t(__builtin_popcountll(lmask)));
  }
  mb = __builtin_amdgcn_readfirstlane(mb);
  lb = __builtin_amdgcn_readfirstlane(lb);
  const uint32_t mr = __builtin_amdgcn_mbcnt_hi(uint32_t(mmask >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(mmask), 0u));
  const uint32_t lr = __builtin_amdgcn_mbcnt_hi(uint32_t(lmask >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(lmask), 0u));
  if (valid && med) {
    mst[mb + mr][0] = s;
    mst[mb + mr][1] = e;
    mseg[mb + mr] = uint32_t(seg);
  }
  if (valid && !med) {
    lst[lb + lr][0] = s;
    lst[lb + lr][1] = e;
    lseg[lb + lr] = uint32_t(seg);
  }
  __syncthreads();
  const uint32_t nmed = cnt[0], nlong = cnt[1];
  const uint32_t g = lane >> 4, gl = lane & 15u;
  for (;;) {  // medium segments, 4 per claim, 16 lanes each
    uint32_t r0 = 0;
    if (lane == 0) r0 = atomicAdd(&cnt[2], 4u);
    r0 = __builtin_amdgcn_readfirstlane(r0);
    if (r0 >= nmed) break;
    const uint32_t k = r0 + g;
    const bool mine = k < nmed;
    const uint32_t kc = mine ? k : 0u;
    const uint64_t ms = mine ? mst[kc][0] : 0, me = mine ? mst[kc][1] : 0;
    const uint32_t sg = mseg[kc];
    const uint32_t i0 = init[sg];
    uint32_t ev = 0, od = 0;
    range_sums_line_primed<16, 8, true>(bytes, ms, me, gl, ev, od);
    const uint32_t tot = group_sum<16>(combine_roles(ev, od, uint32_t(ms) & 1u));
    if (mine && gl == 15) out[sg] = fold_value(i0 + tot);
  }
  for (;;) {  // long segments, one per claim, 64 lanes
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(&cnt[3], 1u);
    k = __builtin_amdgcn_readfirstlane(k);
    if (k >= nlong) break;
    const uint64_t ls = lst[k][0], le = lst[k][1];
    const uint32_t sg = lseg[k];
    const uint32_t i0 = init[sg];
    uint32_t ev = 0, od = 0;
    range_sums_line_primed<64, 8, true>(bytes, ls, le, lane, ev, od);
    const uint32_t tot = group_sum<64>(combine_roles(ev, od, uint32_t(ls) & 1u));
    if (lane == 63) out[sg] = fold_value(i0 + tot);
  }
}

void run() {
  constexpr uint64_t kN = 1 << 20;
  std::mt19937_64 rng(0x10710004);
  std::vector<uint64_t> off(kN + 1, 0);
  for (uint64_t i = 0; i < kN; ++i) {
    const double u = double(rng() >> 11) * 0x1.0p-53;
    uint64_t L = uint64_t(floor(exp(log(64.0) + u * (log(65537.0) - log(64.0)))));
    L = std::min<uint64_t>(std::max<uint64_t>(L, 64), 65536);
    off[i + 1] = off[i] + L;
  }
  const uint64_t bytes = off[kN];
  uint8_t* d;
  uint64_t* doff;
  uint32_t* init;
  uint16_t* out;
  void* zero;
  CK(hipMalloc(&d, bytes + 64));
  CK(hipMalloc(&doff, off.size() * 8));
  CK(hipMalloc(&init, kN * 4));
  CK(hipMalloc(&out, kN * 2));
  CK(hipMalloc(&zero, 256));
  CK(hipMemset(zero, 0, 256));
  CK(launch_fill_bytes(d, bytes + 64, 0x10710004ull, 0, nullptr));
  CK(launch_fill_bytes(reinterpret_cast<uint8_t*>(init), kN * 4, 0x1234ull, 0, nullptr));
  CK(hipMemcpy(doff, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  const SegSpec sp{d, doff, 0, 0, kN, zero};
  auto grid = [](int spw) { return dim3(uint32_t((kN + uint64_t(4 * spw) - 1) / uint64_t(4 * spw))); };
  struct V {
    const char* name;
    std::function<void()> f;
  };
  std::vector<V> vs = {
      {"ship64", [&] { CK(launch_checksum(sp, init, nullptr, out, 0, Geometry{64, 8, true, 3, 1}, 0, nullptr)); }},
      {"blk16_1k", [&] { hipLaunchKernelGGL((k_blk<16, 1024>), grid(16), dim3(kBlock), 0, nullptr, d, doff, init, out, kN); }},
      {"blk16_2k", [&] { hipLaunchKernelGGL((k_blk<16, 2048>), grid(16), dim3(kBlock), 0, nullptr, d, doff, init, out, kN); }},
      {"blk32_2k", [&] { hipLaunchKernelGGL((k_blk<32, 2048>), grid(32), dim3(kBlock), 0, nullptr, d, doff, init, out, kN); }},
      {"blk16_4k", [&] { hipLaunchKernelGGL((k_blk<16, 4096>), grid(16), dim3(kBlock), 0, nullptr, d, doff, init, out, kN); }},
  };
  std::vector<uint16_t> want(kN), got(kN);
  vs[0].f();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(want.data(), out, kN * 2, hipMemcpyDeviceToHost));
  for (size_t v = 0; v < vs.size(); ++v) {
    CK(hipMemset(out, 0x5A, kN * 2));
    for (int i = 0; i < 3; ++i) vs[v].f();
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
      vs[v].f();
      CK(hipEventRecord(a, nullptr));
      for (int i = 0; i < 5; ++i) vs[v].f();
      CK(hipEventRecord(b, nullptr));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      t[v].push_back(ms * 1e3f / 5);
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("{\"variant\": \"%s\", \"us_median\": %.2f, \"us_min\": %.2f, \"bytes\": %llu, \"frac\": %.4f}\n",
           vs[v].name, t[v][t[v].size() / 2], t[v][0], (unsigned long long)bytes,
           double(bytes) / (t[v][t[v].size() / 2] * 1e-6) / 8e12);
  }
}

}  // namespace
}  // namespace icsum

int main() {
  icsum::run();
  return 0;
}
