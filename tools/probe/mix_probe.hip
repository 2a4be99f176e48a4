// mix_probe.hip — dev tool: where the fused two-class VERIFY launch
// (k_ipv4_twoclass) spends its time over the plain two-class checksum of the
// same bytes, on the stack tick's receive shape (half 40-byte ACKs, half
// 1500-byte datagrams, valid headers, packed offsets; 256 Ki and 1 M
// datagrams).  Variants of the same block-list body, timed interleaved
// (20 launches x 7 rounds, HIP events):
//   ship   launch_ipv4_twoclass (the library's launch)
//   full   this file's copy of its body (equal outputs are checked)
//   nores  header loads and the stream, no verdict (the sum is stored)
//   nohdr  the stream alone (no header loads, no verdict)
//   st3    as nores, with the three output stores of the verdict (ip, tcp, status)
//   lds    the full verdict, its outputs staged in LDS and written by the
//          block as three coalesced rows at the end (equal outputs checked)
//   csum   launch_checksum_twoclass over the same datagrams
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 mix_probe.hip -o mix_probe
#include "../../tcpip_network_protocol_stack_amd/csrc/kernels/icsum_kernels.hip"

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

// one datagram per LPS lanes: header loads (HDR), the TCP-part stream, the
// verdict (RES) or just the group's sum into tcp_ck
template <int LPS, int UNROLL, bool NT, int MODE, bool HDR, bool RES, bool ST3 = false>
__device__ __forceinline__ void item(uint8_t* dg, uint64_t s, uint64_t e, uint64_t seg, bool valid, uint32_t lane,
                                     uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status, const uint8_t* zpad,
                                     const uint32_t* zlast) {
  if constexpr (HDR && RES) {
    ipv4_item<LPS, UNROLL, NT, MODE>(dg, s, e, seg, valid, lane, 1, ip_ck, tcp_ck, status, zpad, zlast);
  } else {
    const bool hdr = e - s >= 20;
    const uint64_t t0 = hdr ? s + 20 : e;
    const uint32_t* last = hdr ? last_dword(dg + e) : zlast;
    const bool tcpf = hdr && e - t0 >= 18;
    Hdr h{};
    uint32_t tf0 = 0, tf1 = 0;
    GroupHdr gh{};
    if constexpr (HDR) {
      if constexpr (LPS >= 16)
        gh = group_hdr_load<LPS>(hdr ? dg + s : zpad, last, tcpf ? dg + t0 : zpad, tcpf ? last : zlast);
      else {
        h = load_hdr(hdr ? dg + s : zpad, last);
        load_tcp_fields(tcpf ? dg + t0 : zpad, tcpf ? last : zlast, tf0, tf1);
      }
    }
    uint32_t ev = 0, od = 0;
    seg_sums<LPS, UNROLL, NT, MODE>(dg, t0, e, lane, ev, od);
    if constexpr (HDR && LPS >= 16) group_hdr_take<LPS>(gh, h, tf0, tf1);
    const uint32_t tot = group_sum<LPS>(combine_roles(ev, od, uint32_t(t0) & 1u));
    if (valid && lane == LPS - 1) {
      tcp_ck[seg] = uint16_t(tot + h.w[0] + h.w[4] + tf0 + tf1);
      if (ST3) {
        ip_ck[seg] = uint16_t(h.w[1] + tot);
        status[seg] = uint8_t(tf0 ^ h.w[2]);
      }
    }
  }
}

template <bool HDR, bool RES, bool ST3 = false, bool LDSOUT = false>
__global__ __launch_bounds__(kBlock) void k_var(uint8_t* dg, const uint64_t* offsets, uint64_t n, uint16_t* ip_ck,
                                                uint16_t* tcp_ck, uint8_t* status, const uint8_t* zpad) {
  constexpr uint32_t SPW = 16, kPer = (kBlock / 64) * SPW;
  __shared__ uint64_t lst[kPer][2], sst[kPer][2];
  __shared__ uint32_t lseg[kPer], sseg[kPer];
  __shared__ uint32_t cnt[3];
  __shared__ uint16_t o_ip[kPer], o_tcp[kPer];
  __shared__ uint8_t o_st[kPer];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t b0 = uint64_t(blockIdx.x) * kPer;  // the block's datagrams [b0, b0 + kPer): the staged rows
  // LDSOUT: the verdict's outputs go to the block's LDS rows (index - b0), written out coalesced at the end
  uint16_t* const ipo = LDSOUT ? o_ip : ip_ck;
  uint16_t* const tco = LDSOUT ? o_tcp : tcp_ck;
  uint8_t* const sto = LDSOUT ? o_st : status;
  const uint64_t ob = LDSOUT ? b0 : 0;
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
    for (uint32_t r0 = 0; r0 < nshort; r0 += 64) {
      const uint32_t k = r0 + lane;
      const bool mine = k < nshort;
      const uint32_t kc = mine ? k : 0u;
      const uint64_t ss = sst[kc][0], se = mine ? sst[kc][1] : ss;
      item<1, 4, false, 0, HDR, RES, ST3>(dg, ss, se, sseg[kc] - ob, mine, 0u, ipo, tco, sto, zpad, zlast);
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
    item<16, 8, true, 3, HDR, RES, ST3>(dg, ls, le, lseg[kc] - ob, mine, gl, ipo, tco, sto, zpad, zlast);
  }
  if constexpr (LDSOUT) {
    __syncthreads();
    const uint64_t i = b0 + threadIdx.x;
    if (threadIdx.x < kPer && i < n) {
      ip_ck[i] = o_ip[threadIdx.x];
      tcp_ck[i] = o_tcp[threadIdx.x];
      status[i] = o_st[threadIdx.x];
    }
  }
}

void run(uint64_t n) {
  std::mt19937_64 rng(11);
  std::vector<uint64_t> off(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) off[i + 1] = off[i] + ((rng() >> 11) & 1 ? 40 : 1500);
  const uint64_t bytes = off[n];
  std::vector<uint8_t> h(bytes + 16);
  for (auto& b : h) b = uint8_t(rng());
  for (uint64_t i = 0; i < n; ++i) {
    uint8_t* p = h.data() + off[i];
    const uint64_t L = off[i + 1] - off[i];
    p[0] = 0x45, p[1] = 0, p[2] = uint8_t(L >> 8), p[3] = uint8_t(L), p[6] = 0x40, p[7] = 0, p[8] = 64, p[9] = 6;
    p[32] = 0x50;
  }
  uint8_t *d, *d2;
  uint64_t* doff;
  void* zero;
  CK(hipMalloc(&d, h.size()));
  CK(hipMalloc(&d2, h.size()));  // a second copy: consecutive launches do not find the bytes in the MALL
  CK(hipMalloc(&doff, off.size() * 8));
  CK(hipMalloc(&zero, 256));
  CK(hipMemset(zero, 0, 256));
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(doff, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  uint16_t *ip, *tcp;
  uint8_t* st;
  CK(hipMalloc(&ip, n * 2));
  CK(hipMalloc(&tcp, n * 2));
  CK(hipMalloc(&st, n));
  const SegSpec sp0{d, doff, 0, 0, n, zero}, sp1{d2, doff, 0, 0, n, zero};
  CK(launch_ipv4_tcp(sp0, 2, ip, tcp, st, Geometry{16, 8, true, 3}, 0, nullptr));  // valid checksums
  CK(hipMemcpy(d2, d, h.size(), hipMemcpyDeviceToDevice));
  const uint8_t* z = static_cast<const uint8_t*>(zero);
  const dim3 grid(uint32_t((n + 63) / 64));
  int rot = 0;
  auto buf = [&] { return (rot++ & 1) ? d2 : d; };
  auto spec = [&] { return (rot++ & 1) ? sp1 : sp0; };
  struct V {
    const char* name;
    std::function<void()> f;
  };
  std::vector<V> vs = {
      {"ship", [&] { CK(launch_ipv4_twoclass(spec(), 1, ip, tcp, st, 16, 0, nullptr, 0)); }},
      {"full", [&] { hipLaunchKernelGGL((k_var<true, true>), grid, dim3(kBlock), 0, nullptr, buf(), doff, n, ip, tcp, st, z); }},
      {"nores", [&] { hipLaunchKernelGGL((k_var<true, false>), grid, dim3(kBlock), 0, nullptr, buf(), doff, n, ip, tcp, st, z); }},
      {"nohdr", [&] { hipLaunchKernelGGL((k_var<false, false>), grid, dim3(kBlock), 0, nullptr, buf(), doff, n, ip, tcp, st, z); }},
      {"csum", [&] { CK(launch_checksum_twoclass(spec(), nullptr, nullptr, tcp, 0, 16, 0, nullptr, 0)); }},
      {"st3", [&] { hipLaunchKernelGGL((k_var<true, false, true>), grid, dim3(kBlock), 0, nullptr, buf(), doff, n, ip, tcp, st, z); }},
      {"lds", [&] { hipLaunchKernelGGL((k_var<true, true, false, true>), grid, dim3(kBlock), 0, nullptr, buf(), doff, n, ip, tcp, st, z); }},
  };
  std::vector<uint8_t> want(n * 5), got(n * 5);
  auto fetch = [&](std::vector<uint8_t>& v) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(v.data(), ip, n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(v.data() + n * 2, tcp, n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(v.data() + n * 4, st, n, hipMemcpyDeviceToHost));
  };
  vs[0].f();
  fetch(want);
  CK(hipMemset(ip, 0x5A, n * 2));
  CK(hipMemset(tcp, 0x5A, n * 2));
  CK(hipMemset(st, 0x5A, n));
  for (size_t v : {size_t(1), vs.size() - 1}) {  // full, lds
    CK(hipMemset(ip, 0x5A, n * 2));
    CK(hipMemset(tcp, 0x5A, n * 2));
    CK(hipMemset(st, 0x5A, n));
    vs[v].f();
    fetch(got);
    if (got != want) {
      fprintf(stderr, "%s differs from ship\n", vs[v].name);
      exit(2);
    }
  }
  std::vector<std::vector<float>> t(vs.size());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
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
    printf("{\"n\": %llu, \"variant\": \"%s\", \"us_median\": %.2f, \"us_min\": %.2f, \"bytes\": %llu, "
           "\"frac\": %.4f}\n",
           (unsigned long long)n, vs[v].name, t[v][t[v].size() / 2], t[v][0], (unsigned long long)bytes,
           double(bytes) / (t[v][t[v].size() / 2] * 1e-6) / 8e12);
  }
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  for (void* p : {static_cast<void*>(d), static_cast<void*>(d2), static_cast<void*>(doff), zero,
                  static_cast<void*>(ip), static_cast<void*>(tcp), static_cast<void*>(st)})
    CK(hipFree(p));
}

}  // namespace
}  // namespace icsum

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) icsum::run(strtoull(argv[i], nullptr, 10));
  if (argc < 2) {
    icsum::run(1u << 18);
    icsum::run(1u << 20);
  }
  return 0;
}
