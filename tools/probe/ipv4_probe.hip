// ipv4_probe.hip — dev tool: where the fused IPv4/TCP kernel's time goes on
// BASELINE config 2 (64 Ki x 1500 B datagrams, 6 rotated copies so launches
// read HBM).  Compiles the engine's kernel file into this translation unit and
// times, interleaved in one process:
//   engine   icsum::launch_ipv4_tcp COMPUTE (the shipped path)
//   plain    icsum::launch_checksum over the same datagrams (no header work)
//   v<F>     a copy of k_ipv4_tcp's COMPUTE path with parts switched off by
//            the bits of F: 1 no IPv4 header loads, 2 no TCP field loads,
//            4 no output stores, 8 16-byte grid (mode 0) instead of mode 3,
//            16 hardware block order, 32 boundary chunks non-temporal too;
//            and PATCH-store shapes P (1 two 2-byte
//            field stores, 2 the same write-through (sc1), 3 non-temporal,
//            4 the two aligned 16-byte chunks holding the fields, 5 those
//            non-temporal, 6 the aligned 64-byte blocks; 7 the whole 128-byte
//            line holding the IPv4 header, one 16-byte store per lane of
//            lanes 0-7, 8 the same non-temporal; junk values; 9 (round 3) the
//            64 bytes from the 32-byte sector holding the IPv4 checksum field,
//            which hold both fields, loaded by the group's 16 lanes (one
//            dword each), the two fields spliced in and all 64 bytes stored
//            back: two WHOLE sectors written with the real bytes, no masked
//            partial-sector write; checked equal to the engine's PATCH)
//   split    v0, then a second launch that scatters the two fields from the
//            contiguous ip_ck / tcp_ck arrays into the datagrams (split_nt:
//            non-temporal stores; scatter: that launch alone)
//   flat     16 lanes x 8 non-temporal dwordx4 per datagram, nothing else
// The buffers hold random bytes: constant data (memset) runs at a higher
// clock and reads as several us faster (MI355X_MICROARCH.md, DVFS).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../tcpip_network_protocol_stack_amd/csrc/kernels \
//         -I../../include ipv4_probe.hip -o ipv4_probe
#include "../../tcpip_network_protocol_stack_amd/csrc/kernels/icsum_kernels.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
#include <vector>

namespace icsum {
namespace {

// range_sums_line_primed with the boundary chunks non-temporal too (F & 32):
// no line of the datagram is kept in L2 by the checksum pass
template <int LPS, int UNROLL>
__device__ __forceinline__ void line_primed_all_nt(const uint8_t* __restrict__ base, uint64_t s, uint64_t e,
                                                   uint32_t lane, uint32_t& ev, uint32_t& od) {
  const uint64_t a0 = s & ~uint64_t(127);
  const uint64_t span = e > s ? e - a0 : 0;
  const uint32_t nch = uint32_t((span + 15) >> 4);
  const uint32_t cs = uint32_t(s - a0) >> 4;
  const uint32_t lastc = nch ? nch - 1 : 0u;
  const u32x4* __restrict__ p = reinterpret_cast<const u32x4*>(base + a0);
  const uint32_t tail = nch ? uint32_t(span - (uint64_t(lastc) << 4)) : 0u;
  u32x4 bnd = {0u, 0u, 0u, 0u};
  uint32_t blo = 0, bhi = 0;
  if (nch) {
    const bool is_tail = lane == 1 && lastc != cs;
    bnd = load16<true>(p + (is_tail ? lastc : cs));
    blo = is_tail ? 0u : (uint32_t(s) & 15u);
    bhi = (is_tail || lastc == cs) ? tail : 16u;
    if (lane >= 2 || (lane == 1 && lastc == cs)) bhi = 0u;
  }
  for (uint32_t c = lane; c < nch; c += uint32_t(LPS * UNROLL)) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t cc = c + uint32_t(u * LPS);
      v[u] = load16<true>(p + (cc < lastc ? cc : lastc));
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t cc = c + uint32_t(u * LPS);
      const uint32_t keep = (cc > cs && cc < lastc) ? ~0u : 0u;
      acc_chunk(v[u] & keep, ev, od);
    }
  }
  acc_chunk(bnd & byte_range_mask(blo, bhi), ev, od);
}

template <int P>
__device__ __forceinline__ void patch_store(uint8_t* dg, uint64_t s, uint64_t t0, uint32_t ipc, uint32_t tcv) {
  uint8_t* f[2] = {dg + s + 10, dg + t0 + 16};
  const uint32_t v[2] = {ipc, tcv};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    uint16_t* q = reinterpret_cast<uint16_t*>(f[k]);
    const uint16_t w = uint16_t(v[k]);
    if (P == 1) *q = w;
    if (P == 2) __hip_atomic_store(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (P == 3) __builtin_nontemporal_store(w, q);
    if (P == 4 || P == 5 || P == 6) {
      constexpr uint64_t kB = P == 6 ? 64 : 16;
      u32x4* c = reinterpret_cast<u32x4*>(reinterpret_cast<uintptr_t>(f[k]) & ~uintptr_t(kB - 1));
#pragma unroll
      for (uint64_t j = 0; j < kB / 16; ++j) {
        const u32x4 x = {v[k], v[k] + 1, v[k] + 2, v[k] + 3};
        if (P == 5)
          __builtin_nontemporal_store(x, c + j);
        else
          c[j] = x;
      }
    }
  }
}

template <int F, int P = 0>
__global__ __launch_bounds__(kBlock) void k_v(uint8_t* __restrict__ dg, uint64_t stride, uint64_t dlen, uint64_t n,
                                              uint16_t* __restrict__ ip_ck, uint16_t* __restrict__ tcp_ck,
                                              uint8_t* __restrict__ status, uint32_t remap) {
  constexpr int LPS = 16, UNROLL = 8, MODE = (F & 8) ? 0 : 3;
  constexpr uint32_t kGroups = kBlock / LPS;
  const uint32_t lane = threadIdx.x & (LPS - 1);
  const uint64_t seg = uint64_t(block_order((F & 16) ? 0u : remap)) * kGroups + threadIdx.x / LPS;
  const bool valid = seg < n;
  uint64_t s = 0, e = 0;
  if (valid) seg_bounds(nullptr, stride, dlen, seg, s, e);
  const bool hdr = valid && e - s >= 20;
  const uint64_t t0 = hdr ? s + 20 : e;
  Hdr h = {};
  uint32_t tf0 = 0, tf1 = 0;
  if (!(F & 1) && hdr) h = load_hdr(dg + s, last_dword(dg + e));
  if (!(F & 2) && hdr && e - t0 >= 18) load_tcp_fields(dg + t0, last_dword(dg + e), tf0, tf1);
  uint32_t ev = 0, od = 0;
  if (F & 32)
    line_primed_all_nt<LPS, UNROLL>(dg, t0, e, lane, ev, od);
  else
    seg_sums<LPS, UNROLL, true, MODE>(dg, t0, e, lane, ev, od);
  const uint32_t tot = group_sum<LPS>(combine_roles(ev, od, uint32_t(t0) & 1u));
  if ((P == 7 || P == 8) && valid && lane < 8) {  // whole head line, junk
    u32x4* c = reinterpret_cast<u32x4*>(dg + (s & ~uint64_t(127))) + lane;
    const u32x4 x = {tot, tot + 1, tot + 2, tot + 3};
    if (P == 8)
      __builtin_nontemporal_store(x, c);
    else
      *c = x;
  }
  if (P == 9) {  // whole sectors with the fields spliced in (hlen 5 datagrams of >= 64 bytes)
    const uint16_t ipc = fold_value(ipv4_header_sum(h));
    // tcp_segment.cpp:143: the checksum field (TCP bytes 16, 17) counts as 0
    const uint16_t tcv = fold_value(ipv4_pseudo(h) + tot - ((tf1 & 0xffu) << 8) - ((tf1 >> 8) & 0xffu));
    const uint64_t S0 = (s + 10) & ~uint64_t(31);
    uint32_t* q = reinterpret_cast<uint32_t*>(dg + S0) + lane;  // 16 lanes: bytes [S0, S0 + 64)
    uint32_t w = valid ? *q : 0u;
    const uint64_t at = S0 + 4 * lane;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint64_t x = at + b;
      uint32_t v = (w >> (8 * b)) & 0xffu;
      if (x == s + 10) v = ipc >> 8;
      if (x == s + 11) v = ipc & 0xffu;
      if (x == t0 + 16) v = tcv >> 8;
      if (x == t0 + 17) v = tcv & 0xffu;
      w = (w & ~(0xffu << (8 * b))) | (v << (8 * b));
    }
    if (valid) *q = w;
  }
  if (valid && lane == LPS - 1) {
    const uint16_t ipc = fold_value(ipv4_header_sum(h));
    uint32_t sum = ipv4_pseudo(h) + tot - (tf1 & 0xffffu);
    const uint16_t tcv = fold_value(sum);
    const uint8_t st = uint8_t(((tf0 & 0xffu) >> 4) | (h.byte(9) == 6 ? 8 : 0));
    if (P && P < 7) patch_store<P>(dg, s, t0, ipc, tcv);
    (void)0;
    if (F & 4) {
      if (ipc == 0x1234u && tcv == 0x5678u && st == 9) status[0] = 1;  // keep the work, drop the stores
    } else {
      ip_ck[seg] = ipc;
      tcp_ck[seg] = tcv;
      status[seg] = st;
    }
  }
}

template <bool NTS>
__global__ __launch_bounds__(256) void k_scatter(uint8_t* __restrict__ dg, uint64_t stride, uint64_t n,
                                                 const uint16_t* __restrict__ ip_ck,
                                                 const uint16_t* __restrict__ tcp_ck) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  uint16_t* a = reinterpret_cast<uint16_t*>(dg + i * stride + 10);
  uint16_t* b = reinterpret_cast<uint16_t*>(dg + i * stride + 36);
  const uint16_t x = __builtin_bswap16(ip_ck[i]), y = __builtin_bswap16(tcp_ck[i]);
  if (NTS) {
    __builtin_nontemporal_store(x, a);
    __builtin_nontemporal_store(y, b);
  } else {
    *a = x;
    *b = y;
  }
}

__global__ __launch_bounds__(256) void k_flat(const uint8_t* __restrict__ d, uint64_t n, uint16_t* __restrict__ out) {
  const uint64_t g = (uint64_t(blockIdx.x) * 256 + threadIdx.x) / 16;
  const uint32_t lane = threadIdx.x % 16;
  if (g >= n) return;
  const uint64_t s = g * 1500, a0 = s & ~uint64_t(15), e = s + 1500;
  const uint32_t nch = uint32_t((e - a0 + 15) >> 4);
  const u32x4* p = reinterpret_cast<const u32x4*>(d + a0);
  uint32_t ev = 0, od = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint32_t c = lane + u * 16;
    acc_chunk(__builtin_nontemporal_load(p + (c < nch ? c : nch - 1)), ev, od);
  }
  const uint32_t t = group_sum<16>(ev * 256u + od);
  if (lane == 15) out[g] = fold_value(t);
}

}  // namespace
}  // namespace icsum

using namespace icsum;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr int kCopies = 6;
constexpr uint64_t kN = 1 << 16, kL = 1500;

struct Bufs {
  uint8_t* d[kCopies];
  uint16_t *ip, *tcp;
  uint8_t* st;
  void* zero;
};

template <class Launch>
int timeit(const char* name, Launch fn, hipEvent_t a, hipEvent_t b, float* acc) {
  const int reps = 60;
  CK(hipEventRecord(a, nullptr));
  for (int r = 0; r < reps; ++r) fn(r % kCopies);
  CK(hipEventRecord(b, nullptr));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  *acc = ms * 1e3f / reps;
  (void)name;
  return 0;
}

int main() {
  Bufs B;
  for (int c = 0; c < kCopies; ++c) {
    CK(hipMalloc(&B.d[c], kN * kL + 64));
    CK(launch_fill_bytes(B.d[c], kN * kL, 0x10710002, c * kN * kL, nullptr));
    CK(launch_ipv4_tcp_headers(B.d[c], kL, kL, kN, 0x10710002, c * kN, nullptr));
  }
  CK(hipMalloc(&B.ip, kN * 2));
  CK(hipMalloc(&B.tcp, kN * 2));
  CK(hipMalloc(&B.st, kN));
  CK(hipMalloc(&B.zero, 16));
  CK(hipMemset(B.zero, 0, 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint32_t blocks = uint32_t(kN * 16 / 256);
  const Geometry g = pick_geometry(kL);

  struct V {
    const char* name;
    std::function<void(int)> fn;
  };
  auto spec = [&](int c) { return SegSpec{B.d[c], nullptr, kL, kL, kN, B.zero}; };
  std::vector<V> vs;
  vs.push_back({"engine", [&](int c) { (void)launch_ipv4_tcp(spec(c), 0, B.ip, B.tcp, B.st, g, 0, nullptr); }});
  vs.push_back({"plain", [&](int c) { (void)launch_checksum(spec(c), nullptr, nullptr, B.ip, 0, g, 0, nullptr); }});
#define VAR(F)                                                                                            \
  vs.push_back({"v" #F, [&](int c) {                                                                      \
                  hipLaunchKernelGGL(k_v<F>, dim3(blocks), dim3(256), 0, nullptr, B.d[c], kL, kL, kN, B.ip, \
                                     B.tcp, B.st, 10u);                                                   \
                }});
  VAR(0) VAR(1) VAR(3) VAR(4)
#undef VAR
  vs.push_back({"engine_patch", [&](int c) { (void)launch_ipv4_tcp(spec(c), 2, B.ip, B.tcp, B.st, g, 0, nullptr); }});
#define PVAR(P)                                                                                           \
  vs.push_back({"p" #P, [&](int c) {                                                                      \
                  hipLaunchKernelGGL((k_v<0, P>), dim3(blocks), dim3(256), 0, nullptr, B.d[c], kL, kL, kN, B.ip, \
                                     B.tcp, B.st, 10u);                                                   \
                }});
  PVAR(1) PVAR(2) PVAR(3) PVAR(4) PVAR(5) PVAR(6) PVAR(7) PVAR(8) PVAR(9)
#undef PVAR
  const uint32_t sblocks = uint32_t(kN / 256);
  vs.push_back({"split", [&](int c) {
                  hipLaunchKernelGGL((k_v<0, 0>), dim3(blocks), dim3(256), 0, nullptr, B.d[c], kL, kL, kN, B.ip, B.tcp,
                                     B.st, 10u);
                  hipLaunchKernelGGL(k_scatter<false>, dim3(sblocks), dim3(256), 0, nullptr, B.d[c], kL, kN, B.ip, B.tcp);
                }});
  vs.push_back({"split_nt", [&](int c) {
                  hipLaunchKernelGGL((k_v<0, 0>), dim3(blocks), dim3(256), 0, nullptr, B.d[c], kL, kL, kN, B.ip, B.tcp,
                                     B.st, 10u);
                  hipLaunchKernelGGL(k_scatter<true>, dim3(sblocks), dim3(256), 0, nullptr, B.d[c], kL, kN, B.ip, B.tcp);
                }});
  vs.push_back({"v32", [&](int c) {
                  hipLaunchKernelGGL((k_v<32, 0>), dim3(blocks), dim3(256), 0, nullptr, B.d[c], kL, kL, kN, B.ip, B.tcp,
                                     B.st, 10u);
                }});
  vs.push_back({"p1_v32", [&](int c) {
                  hipLaunchKernelGGL((k_v<32, 1>), dim3(blocks), dim3(256), 0, nullptr, B.d[c], kL, kL, kN, B.ip, B.tcp,
                                     B.st, 10u);
                }});
  vs.push_back({"split_v32", [&](int c) {
                  hipLaunchKernelGGL((k_v<32, 0>), dim3(blocks), dim3(256), 0, nullptr, B.d[c], kL, kL, kN, B.ip, B.tcp,
                                     B.st, 10u);
                  hipLaunchKernelGGL(k_scatter<false>, dim3(sblocks), dim3(256), 0, nullptr, B.d[c], kL, kN, B.ip, B.tcp);
                }});
  vs.push_back({"scatter", [&](int c) {
                  hipLaunchKernelGGL(k_scatter<false>, dim3(sblocks), dim3(256), 0, nullptr, B.d[c], kL, kN, B.ip, B.tcp);
                }});
  vs.push_back({"flat", [&](int c) {
                  hipLaunchKernelGGL(k_flat, dim3(blocks), dim3(256), 0, nullptr, B.d[c], kN, B.ip);
                }});

  {  // p9 (whole sectors, real bytes) writes exactly the engine PATCH's bytes
    uint8_t *x = nullptr, *y = nullptr;
    CK(hipMalloc(&x, kN * kL + 64));
    CK(hipMalloc(&y, kN * kL + 64));
    CK(hipMemcpy(x, B.d[0], kN * kL + 64, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(y, B.d[0], kN * kL + 64, hipMemcpyDeviceToDevice));
    CK(launch_ipv4_tcp(SegSpec{x, nullptr, kL, kL, kN, B.zero}, 2, B.ip, B.tcp, B.st, g, 0, nullptr));
    hipLaunchKernelGGL((k_v<0, 9>), dim3(blocks), dim3(256), 0, nullptr, y, kL, kL, kN, B.ip, B.tcp, B.st, 10u);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> hx(kN * kL), hy(kN * kL);
    CK(hipMemcpy(hx.data(), x, kN * kL, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hy.data(), y, kN * kL, hipMemcpyDeviceToHost));
    printf("{\"p9_equals_engine_patch\": %s}\n", hx == hy ? "true" : "false");
    CK(hipFree(x));
    CK(hipFree(y));
  }
  for (int r = 0; r < 4000; ++r) vs[0].fn(r % kCopies);  // settle clocks
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> t(vs.size());
  for (int round = 0; round < 7; ++round) {
    for (size_t k = 0; k < vs.size(); ++k) {
      const size_t i = round % 2 ? vs.size() - 1 - k : k;
      float us = 0;
      if (timeit(vs[i].name, vs[i].fn, a, b, &us)) return 1;
      t[i].push_back(us);
    }
  }
  for (size_t i = 0; i < vs.size(); ++i) {
    std::sort(t[i].begin(), t[i].end());
    printf("{\"variant\": \"%s\", \"med_us\": %.2f, \"min_us\": %.2f}\n", vs[i].name, t[i][t[i].size() / 2], t[i][0]);
  }
  CK(hipGetLastError());
  return 0;
}
