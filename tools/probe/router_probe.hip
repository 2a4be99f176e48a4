// router_probe.hip — dev tool: the router TTL batch (k_router_ttl,
// src/router/router.cpp:43-50) on 1 M x 1500 B datagrams, 6 rotated copies,
// variants timed interleaved in one process.  The memory-side counters show
// ~1.9 128-byte read requests per datagram where the header needs ~1.16
// lines: the six dword loads of one lane per datagram are six wave
// instructions, each touching 64 different lines.  Variants:
//   engine  the shipped kernel (one lane per datagram, six dword loads)
//   c4      four lanes per datagram: lane j loads dwords j (and j+4 for j<2),
//           the group assembles the header with DPP (two instructions touch
//           16 lines each)
//   c2      two lanes per datagram, three dwords each
//   rd      reads only (one lane per datagram, no store) — the read floor
//   sec     round 3: four lanes per datagram load the 64-byte window from the
//           32-byte sector holding the header start (16 B each), and the
//           sectors holding the rewritten bytes 4..11 are stored WHOLE (two
//           16-byte stores per sector, the new fields spliced into the bytes
//           just loaded) instead of one masked 8-byte store: no partial-sector
//           write reaches the memory side (dword-aligned headers, stride >= 64,
//           so no other datagram's bytes share those sectors)
//   rdsec   the same 64-byte window loads, no store
//   rt*     the shipped two-lane structure with a 4-byte store of bytes 8..11
//           (w4) and / or 20-byte reads of aligned headers (r20), see k_rt
// Every variant forwards (ttl--, checksum recomputed) the same datagrams, so
// the copies start at ttl 255 and each is forwarded at most 240 times.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include router_probe.hip -o router_probe
#include "../../tcpip_network_protocol_stack_amd/csrc/kernels/icsum_kernels.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
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

constexpr uint64_t kN = 1 << 20, kL = 1500;
constexpr int kCopies = 6;

// ttl := 255 on every datagram, then PATCH recomputes both checksums
__global__ void k_ttl255(uint8_t* dg, uint64_t n, uint64_t stride) {
  ICS_GRID_STRIDE(i, n) dg[i * stride + 8] = 255;
}

// forward the datagram whose (aligned) header dwords are d[0..5]
__device__ __forceinline__ uint8_t forward(uint8_t* p, const uint32_t* d, uint32_t sh) {
  Hdr h;
#pragma unroll
  for (int k = 0; k < 5; ++k) h.w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
  const uint32_t ver = h.byte(0) >> 4, hlen = h.byte(0) & 0x0fu, ttl = h.byte(8);
  if (!(ver == 4 && hlen >= 5 && fold_value(ipv4_header_sum(h)) == h.be16(10) && ttl > 1)) return 0;
  h.w[2] = (h.w[2] & ~0xffu) | (ttl - 1);
  const uint32_t c = fold_value(ipv4_header_sum(h));
  if ((reinterpret_cast<uintptr_t>(p) & 3u) == 0) {
    const uint32_t w1 = h.w[1] & ~0x00800000u;
    const uint32_t w2 = (h.w[2] & 0x0000ffffu) | ((c >> 8) << 16) | ((c & 0xffu) << 24);
    uint32_t* q = reinterpret_cast<uint32_t*>(p + 4);
    q[0] = w1;
    q[1] = w2;
  } else {
    p[6] = uint8_t(h.byte(6) & 0x7fu);
    p[8] = uint8_t(ttl - 1);
    store_be16(p + 10, c);
  }
  return 1;
}

// LPS lanes per datagram; lane j loads dwords j, j+LPS, ... of the 6
template <int LPS, bool STORE>
__global__ __launch_bounds__(kBlock) void k_coop(uint8_t* __restrict__ dg, uint64_t stride, uint64_t n,
                                                 uint8_t* __restrict__ status) {
  constexpr uint32_t kG = kBlock / LPS;
  const uint32_t lane = threadIdx.x & (LPS - 1);
  for (uint64_t i = uint64_t(blockIdx.x) * kG + threadIdx.x / LPS; i - threadIdx.x / LPS < n;
       i += uint64_t(gridDim.x) * kG) {
    const bool valid = i < n;
    const uint64_t s = (valid ? i : n - 1) * stride;
    uint8_t* p = dg + s;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
    const uint32_t* last = last_dword(p + stride);
    uint32_t mine[(6 + LPS - 1) / LPS];
#pragma unroll
    for (int k = 0; k < (6 + LPS - 1) / LPS; ++k) {
      const uint32_t idx = lane + uint32_t(k * LPS);
      const uint32_t* a = q + (idx < 6 ? idx : 5);
      mine[k] = *(a < last ? a : last);
    }
    uint32_t d[6];
#pragma unroll
    for (int w = 0; w < 6; ++w) {  // dword w lives in lane w % LPS, slot w / LPS
      const int src = int(threadIdx.x & 63u & ~uint32_t(LPS - 1)) + (w % LPS);
      d[w] = LPS == 1 ? mine[w] : uint32_t(__shfl(int(mine[w / LPS]), src, 64));
    }
    if (valid && lane == 0) {
      if (STORE) {
        status[i] = forward(p, d, sh);
      } else {
        Hdr h;
#pragma unroll
        for (int k = 0; k < 5; ++k) h.w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        status[i] = uint8_t(fold_value(ipv4_header_sum(h)) == h.be16(10));
      }
    }
  }
}

// dword k (0..15) of the 64-byte window held 4 per lane by the group's lanes
__device__ __forceinline__ uint32_t win_dword(const u32x4& v, uint32_t k, uint32_t base_lane) {
  const uint32_t e = k & 3u;
  const uint32_t mine = e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;  // every lane picks element k & 3
  return uint32_t(__shfl(int(mine), int(base_lane + (k >> 2)), 64));
}

template <bool STORE>
__global__ __launch_bounds__(kBlock) void k_sec(uint8_t* __restrict__ dg, uint64_t stride, uint64_t n,
                                                uint8_t* __restrict__ status) {
  constexpr uint32_t kG = kBlock / 4;
  const uint32_t lane = threadIdx.x & 3u, base_lane = threadIdx.x & 63u & ~3u;
  for (uint64_t i = uint64_t(blockIdx.x) * kG + threadIdx.x / 4; i - threadIdx.x / 4 < n;
       i += uint64_t(gridDim.x) * kG) {
    const bool valid = i < n;
    const uint64_t s = (valid ? i : n - 1) * stride;
    const uint64_t B = s & ~uint64_t(31);
    u32x4* w = reinterpret_cast<u32x4*>(dg + B) + lane;
    u32x4 v = *w;
    const uint32_t k0 = uint32_t(s - B) >> 2;  // header dword 0 in the window (s dword-aligned)
    uint32_t d[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) d[k] = win_dword(v, k0 + uint32_t(k), base_lane);
    Hdr h;
#pragma unroll
    for (int k = 0; k < 5; ++k) h.w[k] = d[k];
    const uint32_t ver = h.byte(0) >> 4, hlen = h.byte(0) & 0x0fu, ttl = h.byte(8);
    const bool fwd = valid && ver == 4 && hlen >= 5 && fold_value(ipv4_header_sum(h)) == h.be16(10) && ttl > 1;
    if (!STORE) {
      if (valid && lane == 0) status[i] = uint8_t(fold_value(ipv4_header_sum(h)) == h.be16(10));
      continue;
    }
    h.w[2] = (h.w[2] & ~0xffu) | (ttl - 1);
    const uint32_t c = fold_value(ipv4_header_sum(h));
    const uint32_t w1 = h.w[1] & ~0x00800000u;
    const uint32_t w2 = (h.w[2] & 0x0000ffffu) | ((c >> 8) << 16) | ((c & 0xffu) << 24);
    // window dwords k0+1, k0+2 take w1, w2; this lane holds dwords 4 lane .. 4 lane + 3
    const uint32_t a = k0 + 1;
    u32x4 o = v;
    o.x = (4 * lane + 0 == a) ? w1 : (4 * lane + 0 == a + 1) ? w2 : o.x;
    o.y = (4 * lane + 1 == a) ? w1 : (4 * lane + 1 == a + 1) ? w2 : o.y;
    o.z = (4 * lane + 2 == a) ? w1 : (4 * lane + 2 == a + 1) ? w2 : o.z;
    o.w = (4 * lane + 3 == a) ? w1 : (4 * lane + 3 == a + 1) ? w2 : o.w;
    // sectors touched: the ones holding window bytes 4 k0 + 4 .. 4 k0 + 11
    const uint32_t sec_lo = (4 * k0 + 4) >> 5, sec_hi = (4 * k0 + 11) >> 5, my_sec = lane >> 1;
    if (fwd && my_sec >= sec_lo && my_sec <= sec_hi) *w = o;
    if (valid && lane == 0) status[i] = fwd ? 1 : 0;
  }
}

// round 3 (later): the shipped kernel's two lanes per datagram, with
//   W4      for a dword-aligned header whose reserved flag bit is clear (the
//           flags byte then re-serializes to itself), ONE aligned 4-byte store
//           of bytes 8..11 (ttl - 1, protocol, checksum) instead of the 8-byte
//           store of bytes 4..11: it never straddles a 32-byte sector
//   READ20  lane 1's third dword (header bytes 20..23, only needed to realign
//           an unaligned header) re-reads dword 4 when the header is aligned
template <bool READ20, bool W4>
__global__ __launch_bounds__(kBlock) void k_rt(uint8_t* __restrict__ dg, uint64_t stride, uint64_t n,
                                               uint8_t* __restrict__ status, const uint32_t* __restrict__ zpad) {
  constexpr uint32_t kG = kBlock / 2;
  const uint32_t lane = threadIdx.x & 1u;
  const uint64_t step = uint64_t(gridDim.x) * kG;
  for (uint64_t g0 = uint64_t(blockIdx.x) * kG; g0 < n; g0 += step) {
    const uint64_t i = g0 + threadIdx.x / 2;
    const bool valid = i < n;
    uint64_t s, e;
    seg_bounds(nullptr, stride, stride, valid ? i : n - 1, s, e);
    const bool hdr = valid && e - s >= 20;
    uint8_t* p = dg + s;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
    const uint32_t* q = hdr ? reinterpret_cast<const uint32_t*>(p - sh) : zpad;
    const uint32_t* last = hdr ? last_dword(dg + e) : zpad + 7;
    uint32_t mine[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      uint32_t idx = lane + 2u * k;
      if (READ20 && k == 2 && sh == 0) idx = 4;
      const uint32_t* a = q + idx;
      mine[k] = *(a < last ? a : last);
    }
    const int pair = int(threadIdx.x & 63u & ~1u);
    uint32_t d[6];
#pragma unroll
    for (int w = 0; w < 6; ++w) d[w] = uint32_t(__shfl(int(mine[w / 2]), pair + (w & 1), 64));
    if (valid && lane == 0) {
      uint8_t st = 0;
      if (hdr) {
        Hdr h;
#pragma unroll
        for (int k = 0; k < 5; ++k) h.w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        const uint32_t ver = h.byte(0) >> 4, hlen = h.byte(0) & 0x0fu, ttl = h.byte(8);
        if (ver == 4 && hlen >= 5 && fold_value(ipv4_header_sum(h)) == h.be16(10) && ttl > 1) {
          h.w[2] = (h.w[2] & ~0xffu) | (ttl - 1);
          const uint32_t c = fold_value(ipv4_header_sum(h));
          const uint32_t w2 = (h.w[2] & 0x0000ffffu) | ((c >> 8) << 16) | ((c & 0xffu) << 24);
          if (W4 && sh == 0 && (h.byte(6) & 0x80u) == 0) {
            *reinterpret_cast<uint32_t*>(p + 8) = w2;
          } else if (sh == 0) {
            uint32_t* o = reinterpret_cast<uint32_t*>(p + 4);
            o[0] = h.w[1] & ~0x00800000u;
            o[1] = w2;
          } else {
            p[6] = uint8_t(h.byte(6) & 0x7fu);
            p[8] = uint8_t(ttl - 1);
            store_be16(p + 10, c);
          }
          st = 1;
        }
      }
      status[i] = st;
    }
  }
}

}  // namespace
}  // namespace icsum

using namespace icsum;

int main() {
  std::vector<uint8_t*> d(kCopies);
  uint8_t *st = nullptr, *zero = nullptr;
  for (int c = 0; c < kCopies; ++c) {
    CK(hipMalloc(&d[c], kN * kL + 64));
    CK(launch_fill_bytes(d[c], kN * kL, 0x10710003, c * kN * kL, nullptr));
    CK(launch_ipv4_tcp_headers(d[c], kL, kL, kN, 0x10710003, c * kN, nullptr));
    hipLaunchKernelGGL(k_ttl255, dim3(4096), dim3(256), 0, nullptr, d[c], kN, kL);
  }
  CK(hipMalloc(&st, kN));
  CK(hipMalloc(&zero, 64));
  CK(hipMemset(zero, 0, 64));
  for (int c = 0; c < kCopies; ++c) {
    const SegSpec sp{d[c], nullptr, kL, kL, kN, zero};
    CK(launch_ipv4_tcp(sp, 2, nullptr, nullptr, nullptr, pick_geometry(kL), 0, nullptr));
  }
  CK(hipDeviceSynchronize());
  struct V {
    const char* name;
    std::function<void(int)> fn;
  };
  std::vector<V> vs;
  vs.push_back({"engine", [&](int c) {
                  const SegSpec sp{d[c], nullptr, kL, kL, kN, zero};
                  CK(launch_router_ttl(sp, st, nullptr));
                }});
  vs.push_back({"c1", [&](int c) { hipLaunchKernelGGL((k_coop<1, true>), dim3(4096), dim3(256), 0, nullptr, d[c], kL, kN, st); }});
  vs.push_back({"c2", [&](int c) { hipLaunchKernelGGL((k_coop<2, true>), dim3(8192), dim3(256), 0, nullptr, d[c], kL, kN, st); }});
  vs.push_back({"c4", [&](int c) { hipLaunchKernelGGL((k_coop<4, true>), dim3(16384), dim3(256), 0, nullptr, d[c], kL, kN, st); }});
  vs.push_back({"c8", [&](int c) { hipLaunchKernelGGL((k_coop<8, true>), dim3(32768), dim3(256), 0, nullptr, d[c], kL, kN, st); }});
  vs.push_back({"rd1", [&](int c) { hipLaunchKernelGGL((k_coop<1, false>), dim3(4096), dim3(256), 0, nullptr, d[c], kL, kN, st); }});
  vs.push_back({"rd4", [&](int c) { hipLaunchKernelGGL((k_coop<4, false>), dim3(16384), dim3(256), 0, nullptr, d[c], kL, kN, st); }});
  vs.push_back({"sec", [&](int c) { hipLaunchKernelGGL((k_sec<true>), dim3(16384), dim3(256), 0, nullptr, d[c], kL, kN, st); }});
  vs.push_back({"rdsec", [&](int c) { hipLaunchKernelGGL((k_sec<false>), dim3(16384), dim3(256), 0, nullptr, d[c], kL, kN, st); }});
  const uint32_t rt_blocks = uint32_t(std::min<uint64_t>((kN * 2 + kBlock - 1) / kBlock, 65536));
  vs.push_back({"rt", [&](int c) { hipLaunchKernelGGL((k_rt<false, false>), dim3(rt_blocks), dim3(kBlock), 0, nullptr, d[c], kL, kN, st, reinterpret_cast<const uint32_t*>(zero)); }});
  vs.push_back({"rt_w4", [&](int c) { hipLaunchKernelGGL((k_rt<false, true>), dim3(rt_blocks), dim3(kBlock), 0, nullptr, d[c], kL, kN, st, reinterpret_cast<const uint32_t*>(zero)); }});
  vs.push_back({"rt_r20", [&](int c) { hipLaunchKernelGGL((k_rt<true, false>), dim3(rt_blocks), dim3(kBlock), 0, nullptr, d[c], kL, kN, st, reinterpret_cast<const uint32_t*>(zero)); }});
  vs.push_back({"rt_w4_r20", [&](int c) { hipLaunchKernelGGL((k_rt<true, true>), dim3(rt_blocks), dim3(kBlock), 0, nullptr, d[c], kL, kN, st, reinterpret_cast<const uint32_t*>(zero)); }});
  {  // the whole-sector variant writes exactly the engine's bytes
    uint8_t *x = nullptr, *y = nullptr;
    CK(hipMalloc(&x, kN * kL + 64));
    CK(hipMalloc(&y, kN * kL + 64));
    CK(hipMemcpy(x, d[0], kN * kL + 64, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(y, d[0], kN * kL + 64, hipMemcpyDeviceToDevice));
    const SegSpec sp{x, nullptr, kL, kL, kN, zero};
    CK(launch_router_ttl(sp, st, nullptr));
    hipLaunchKernelGGL((k_sec<true>), dim3(16384), dim3(256), 0, nullptr, y, kL, kN, st);
    CK(hipDeviceSynchronize());
    {  // and the 4-byte-store / 20-byte-read variant, on a third copy
      uint8_t* z = nullptr;
      CK(hipMalloc(&z, kN * kL + 64));
      CK(hipMemcpy(z, d[0], kN * kL + 64, hipMemcpyDeviceToDevice));
      const uint32_t rb = uint32_t(std::min<uint64_t>((kN * 2 + kBlock - 1) / kBlock, 65536));
      hipLaunchKernelGGL((k_rt<true, true>), dim3(rb), dim3(kBlock), 0, nullptr, z, kL, kN, st,
                         reinterpret_cast<const uint32_t*>(zero));
      CK(hipDeviceSynchronize());
      std::vector<uint8_t> hx(kN * kL), hz(kN * kL);
      CK(hipMemcpy(hx.data(), x, kN * kL, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hz.data(), z, kN * kL, hipMemcpyDeviceToHost));
      printf("{\"rt_w4_r20_equals_engine\": %s}\n", hx == hz ? "true" : "false");
      CK(hipFree(z));
    }
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> hx(kN * kL), hy(kN * kL);
    CK(hipMemcpy(hx.data(), x, kN * kL, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hy.data(), y, kN * kL, hipMemcpyDeviceToHost));
    printf("{\"sec_equals_engine\": %s}\n", hx == hy ? "true" : "false");
    CK(hipFree(x));
    CK(hipFree(y));
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // settle on reads (no forwarding) for ~150 ms
  for (int k = 0; k < 400; ++k) hipLaunchKernelGGL((k_coop<4, false>), dim3(16384), dim3(256), 0, nullptr, d[k % kCopies], kL, kN, st);
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> t(vs.size());
  for (int r = 0; r < 12; ++r) {
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(hipEventRecord(a, nullptr));
      for (int k = 0; k < 12; ++k) vs[v].fn(k % kCopies);
      CK(hipEventRecord(b, nullptr));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      t[v].push_back(ms * 1e3f / 12);
    }
  }
  std::vector<uint8_t> h(kN);
  CK(hipMemcpy(h.data(), st, kN, hipMemcpyDeviceToHost));
  size_t ok = 0;
  for (auto x : h) ok += x;
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("{\"variant\": \"%s\", \"med_us\": %.2f, \"min_us\": %.2f}\n", vs[v].name, t[v][t[v].size() / 2], t[v][0]);
  }
  printf("{\"last_status_ok\": %zu}\n", ok);
  return 0;
}
