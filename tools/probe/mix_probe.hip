// mix_probe.hip — dev tool: the two-class IPv4 launch on a received ACK/MTU
// mix (1 M datagrams, 40-byte ACKs and 1500-byte segments, valid headers;
// the ACK shares on the command line), against shapes around it.  VERIFY,
// outputs compared with the library kernel's, launches timed interleaved
// (20 launches x 7 rounds, HIP events).
//   ship     launch_ipv4_twoclass (since round 3 the block-list kernel, 16
//            datagrams per wave; before that the per-wave one, = spw16's body
//            at 32 per wave)
//   spw16    the round-2 per-wave kernel at 16 datagrams per wave: the wave
//            verifies its short datagrams, then its long ones 4 at a time
//   blk*     block lists: wave 0 verifies the block's short datagrams, every
//            wave claims groups of 4 long ones from an LDS counter (* =
//            datagrams per wave in the bounds pass)
//   blkq*    one LDS queue of short passes and long groups claimed by every wave
// (round 3, first runs: long class 16 x 6 and 8 waves / SIMD by launch
// bounds were slower than the per-wave kernel and are gone from the list)
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

// block lists: the block's 4 x SPW datagrams go to one long and one short
// list in LDS; wave 0 verifies the short ones (one lane each, 64 per pass),
// every wave claims groups of 4 long ones (16 lanes each) from an LDS counter
// — wave 0 joining once its short passes are done
template <int SPW>
__global__ __launch_bounds__(kBlock) void k_mix_blk(uint8_t* __restrict__ dg, const uint64_t* __restrict__ offsets,
                                                    uint64_t n, int mode, uint16_t* __restrict__ ip_ck,
                                                    uint16_t* __restrict__ tcp_ck, uint8_t* __restrict__ status,
                                                    const uint8_t* __restrict__ zpad) {
  constexpr uint32_t kPer = (kBlock / 64) * SPW;
  __shared__ uint64_t lst[kPer][2];
  __shared__ uint32_t lseg[kPer];
  __shared__ uint64_t sst[kPer][2];
  __shared__ uint32_t sseg[kPer];
  __shared__ uint32_t cnt[3];  // long, short, long claimed
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t* const zlast = reinterpret_cast<const uint32_t*>(zpad) + 7;
  if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t seg = (uint64_t(blockIdx.x) * (kBlock / 64) + wv) * SPW + (lane < SPW ? lane : 0u);
  const bool valid = seg < n && lane < SPW;
  uint64_t s, e;
  seg_bounds(offsets, 0, 0, seg < n ? seg : n - 1, s, e);
  if (!valid) e = s;
  const bool is_short = e - s <= 64;
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
      ipv4_item<1, 4, false, 0>(dg, ss, se, sseg[kc], mine, 0u, mode, ip_ck, tcp_ck, status, zpad, zlast);
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
    const uint64_t ls = lst[kc][0], le = mine ? lst[kc][1] : ls;
    ipv4_item<16, 8, true, 3>(dg, ls, le, lseg[kc], mine, gl, mode, ip_ck, tcp_ck, status, zpad, zlast);
  }
}

// one LDS work queue per block: short passes (64 short datagrams, one lane
// each) first, then groups of 4 long datagrams (16 lanes each); every wave
// claims the next item until the queue is empty
template <int SPW>
__global__ __launch_bounds__(kBlock) void k_mix_blkq(uint8_t* __restrict__ dg, const uint64_t* __restrict__ offsets,
                                                     uint64_t n, int mode, uint16_t* __restrict__ ip_ck,
                                                     uint16_t* __restrict__ tcp_ck, uint8_t* __restrict__ status,
                                                     const uint8_t* __restrict__ zpad) {
  constexpr uint32_t kPer = (kBlock / 64) * SPW;
  __shared__ uint64_t lst[kPer][2];
  __shared__ uint32_t lseg[kPer];
  __shared__ uint64_t sst[kPer][2];
  __shared__ uint32_t sseg[kPer];
  __shared__ uint32_t cnt[3];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t* const zlast = reinterpret_cast<const uint32_t*>(zpad) + 7;
  if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t seg = (uint64_t(blockIdx.x) * (kBlock / 64) + wv) * SPW + (lane < SPW ? lane : 0u);
  const bool valid = seg < n && lane < SPW;
  uint64_t s, e;
  seg_bounds(offsets, 0, 0, seg < n ? seg : n - 1, s, e);
  if (!valid) e = s;
  const bool is_short = e - s <= 64;
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
  const uint32_t spass = (nshort + 63) / 64, items = spass + (nlong + 3) / 4;
  const uint32_t g = lane >> 4, gl = lane & 15u;
  for (;;) {
    uint32_t it = 0;
    if (lane == 0) it = atomicAdd(&cnt[2], 1u);
    it = __builtin_amdgcn_readfirstlane(it);
    if (it >= items) break;
    if (it < spass) {
      const uint32_t k = it * 64 + lane;
      const bool mine = k < nshort;
      const uint32_t kc = mine ? k : 0u;
      const uint64_t ss = sst[kc][0], se = mine ? sst[kc][1] : ss;
      ipv4_item<1, 4, false, 0>(dg, ss, se, sseg[kc], mine, 0u, mode, ip_ck, tcp_ck, status, zpad, zlast);
    } else {
      const uint32_t k = (it - spass) * 4 + g;
      const bool mine = k < nlong;
      const uint32_t kc = mine ? k : 0u;
      const uint64_t ls = lst[kc][0], le = mine ? lst[kc][1] : ls;
      ipv4_item<16, 8, true, 3>(dg, ls, le, lseg[kc], mine, gl, mode, ip_ck, tcp_ck, status, zpad, zlast);
    }
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

void run(double ack) {
  constexpr uint64_t kN = 1 << 20;
  std::mt19937_64 rng(11);
  std::vector<uint64_t> off(kN + 1, 0);
  for (uint64_t i = 0; i < kN; ++i) off[i + 1] = off[i] + (double(rng() >> 11) * 0x1.0p-53 < ack ? 40 : 1500);
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
      {"ship", [&] { CK(launch_ipv4_twoclass(sp, 1, ip, tcp, st, 16, nullptr)); }},
      {"spw16", [&] { hipLaunchKernelGGL((k_mix<16, 8>), grid(16), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"blk32", [&] { hipLaunchKernelGGL((k_mix_blk<32>), grid(32), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"blk16", [&] { hipLaunchKernelGGL((k_mix_blk<16>), grid(16), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"blkq16", [&] { hipLaunchKernelGGL((k_mix_blkq<16>), grid(16), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"blkq24", [&] { hipLaunchKernelGGL((k_mix_blkq<24>), grid(24), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"blkq32", [&] { hipLaunchKernelGGL((k_mix_blkq<32>), grid(32), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
      {"blk24", [&] { hipLaunchKernelGGL((k_mix_blk<24>), grid(24), dim3(kBlock), 0, nullptr, d, doff, kN, 1, ip, tcp, st, z); }},
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
    printf("{\"ack_share\": %.2f, \"variant\": \"%s\", \"us_median\": %.2f, \"us_min\": %.2f, \"bytes\": %llu, "
           "\"accepted\": %zu}\n",
           ack, vs[v].name, t[v][t[v].size() / 2], t[v][0], (unsigned long long)bytes, accept);
  }
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  for (void* p : {static_cast<void*>(d), static_cast<void*>(doff), zero, static_cast<void*>(ip),
                  static_cast<void*>(tcp), static_cast<void*>(st), static_cast<void*>(ref)})
    CK(hipFree(p));
}

}  // namespace
}  // namespace icsum

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) icsum::run(atof(argv[i]));
  if (argc < 2) icsum::run(0.5);
  return 0;
}
