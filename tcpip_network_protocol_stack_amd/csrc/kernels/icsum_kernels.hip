// icsum_kernels.hip — HIP kernels of the Internet-checksum engine, CDNA4 (gfx950).
//
// Every kernel is a memory-bound integer fold: HBM-read roofline, no MFMA.
//   k_checksum    a1-a4  InternetChecksum{init}.add(seg).value()  (checksum.h:17-41)
//                        or the unfolded sum_ for add() chains (checksum.h:44-59)
//   k_ipv4_tcp    a7/a8/a10/a11/a13 fused per raw datagram: header checksum,
//                        pseudo-header, TCP compute/verify, optional in-place patch
//                        (ipv4_header.cpp:9-123, tcp_segment.cpp:9-118, tcp_over_ip.cpp:69-88)
//   k_router_ttl  router.cpp:43-50 ttl-- + header recompute in place
// plus the synthetic-workload generators of icsum_workload.h.
//
// Work mapping: a group of LPS lanes (4..64, aligned inside the 64-lane wave)
// owns one segment; each lane streams 16-byte chunks with non-temporal
// dwordx4 loads (UNROLL in flight per step), accumulates with v_dot4_u32_u8,
// and the group reduces with cross-lane shuffles.  Segments are independent,
// so there is no inter-workgroup communication and no XCD dependence.
#include <hip/hip_runtime.h>

#include "icsum_device.h"
#include "icsum_launch.h"

namespace icsum {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ void seg_bounds(const uint64_t* __restrict__ offsets, uint64_t stride,
                                           uint64_t seg_len, uint64_t i, uint64_t& s,
                                           uint64_t& e) {
  if (offsets) {
    s = offsets[i];
    e = offsets[i + 1];
  } else {
    s = i * stride;
    e = s + seg_len;
  }
}

// ------------------------------------------------------------ a1-a4 -------
template <int LPS, int UNROLL, int OUT>
__global__ __launch_bounds__(kBlock) void k_checksum(const uint8_t* __restrict__ bytes,
                                                     const uint64_t* __restrict__ offsets,
                                                     uint64_t stride, uint64_t seg_len,
                                                     const uint32_t* __restrict__ init,
                                                     const uint8_t* __restrict__ odd,
                                                     void* __restrict__ out, uint64_t n) {
  constexpr uint32_t kGroups = kBlock / LPS;
  const uint32_t lane = threadIdx.x & (LPS - 1);
  const uint64_t step = uint64_t(gridDim.x) * kGroups;
  // the loop bound is uniform per block, so every lane reaches the shuffles
  for (uint64_t g0 = uint64_t(blockIdx.x) * kGroups; g0 < n; g0 += step) {
    const uint64_t seg = g0 + threadIdx.x / LPS;
    const bool valid = seg < n;
    uint64_t s = 0, e = 0;
    uint32_t flip = 0;
    if (valid) {
      seg_bounds(offsets, stride, seg_len, seg, s, e);
      if (odd) flip = odd[seg] & 1u;
    }
    const uint32_t part = range_partial<LPS, UNROLL>(bytes, s, e, lane, flip);
    const uint32_t tot = group_sum<LPS>(part);
    if (valid && lane == 0) {
      const uint32_t sum = (init ? init[seg] : 0u) + tot;
      if (OUT == 0)
        static_cast<uint16_t*>(out)[seg] = fold_value(sum);
      else
        static_cast<uint32_t*>(out)[seg] = sum;
    }
  }
}

__global__ void k_fold(const uint32_t* __restrict__ sum, uint16_t* __restrict__ out, uint64_t n) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = fold_value(sum[i]);
}

// ---------------------------------------------- IPv4 header fields ------
// The first 20 wire bytes of a datagram as 5 little-endian dwords relative to
// its (possibly unaligned) start: 6 aligned dword loads + alignbyte.  The
// sixth dword may extend <= 3 bytes past a 20-byte datagram inside the same
// aligned dword, never into another page.
struct Hdr {
  uint32_t w[5];
  __device__ __forceinline__ uint32_t byte(int k) const { return (w[k >> 2] >> (8 * (k & 3))) & 0xffu; }
  __device__ __forceinline__ uint32_t be16(int k) const { return (byte(k) << 8) | byte(k + 1); }
};

__device__ __forceinline__ Hdr load_hdr(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t sh = uint32_t(a & 3u);
  uint32_t d[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) d[k] = q[k];
  Hdr h;
#pragma unroll
  for (int k = 0; k < 5; ++k) h.w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
  return h;
}

// IPv4Header::compute_checksum (ipv4_header.cpp:113-123): the 20 serialized
// bytes equal the wire bytes with cksum = 0 and the reserved flag bit (0x8000
// of the flags word, wire byte 6 bit 7) dropped (serialize, :78); options are
// never part of the sum.
__device__ __forceinline__ uint32_t ipv4_header_sum(const Hdr& h) {
  uint32_t e = 0, o = 0;
  acc_dword(h.w[0], e, o);
  acc_dword(h.w[1] & ~0x00800000u, e, o);
  acc_dword(h.w[2] & 0x0000ffffu, e, o);
  acc_dword(h.w[3], e, o);
  acc_dword(h.w[4], e, o);
  return e * 256u + o;
}

// IPv4Header::pseudo_checksum (ipv4_header.cpp:103-110); payload_length()
// wraps mod 2^16 (:89-92).
__device__ __forceinline__ uint32_t ipv4_pseudo(const Hdr& h) {
  const uint32_t hlen = h.byte(0) & 0x0fu;
  const uint32_t len = h.be16(2);
  const uint32_t src = bswap32(h.w[3]);
  const uint32_t dst = bswap32(h.w[4]);
  const uint32_t plen = (len - 4u * hlen) & 0xffffu;
  return (src >> 16) + (src & 0xffffu) + (dst >> 16) + (dst & 0xffffu) + h.byte(9) + plen;
}

// --------------------------------------------- fused IPv4 + TCP ----------
template <int LPS, int UNROLL>
__global__ __launch_bounds__(kBlock) void k_ipv4_tcp(uint8_t* __restrict__ dg,
                                                     const uint64_t* __restrict__ offsets,
                                                     uint64_t stride, uint64_t dlen, uint64_t n,
                                                     int mode, uint16_t* __restrict__ ip_ck,
                                                     uint16_t* __restrict__ tcp_ck,
                                                     uint8_t* __restrict__ status) {
  constexpr uint32_t kGroups = kBlock / LPS;
  const uint32_t lane = threadIdx.x & (LPS - 1);
  const uint64_t step = uint64_t(gridDim.x) * kGroups;
  for (uint64_t g0 = uint64_t(blockIdx.x) * kGroups; g0 < n; g0 += step) {
    const uint64_t seg = g0 + threadIdx.x / LPS;
    const bool valid = seg < n;
    uint64_t s = 0, e = 0;
    if (valid) seg_bounds(offsets, stride, dlen, seg, s, e);
    const bool hdr = valid && e - s >= 20;
    Hdr h = {};
    uint64_t t0 = e;  // TCP part: [t0, e)
    if (hdr) {
      h = load_hdr(dg + s);
      uint64_t off = 4u * (h.byte(0) & 0x0fu);  // options skipped (ipv4_header.cpp:50)
      if (off < 20) off = 20;
      if (off > e - s) off = e - s;
      t0 = s + off;
    }
    const uint32_t part = range_partial<LPS, UNROLL>(dg, hdr ? t0 : 0, hdr ? e : 0, lane, 0u);
    const uint32_t tot = group_sum<LPS>(part);
    if (valid && lane == 0) {
      uint16_t ipc = 0, tcv = 0;
      uint8_t st = 0;
      if (hdr) {
        const uint32_t ver = h.byte(0) >> 4, hlen = h.byte(0) & 0x0fu;
        const bool hdr_ok = ver == 4 && hlen >= 5;  // ipv4_header.cpp:32-41
        ipc = fold_value(ipv4_header_sum(h));
        const uint32_t pseudo = ipv4_pseudo(h);
        const uint64_t rem = e - t0;
        if (h.byte(9) == 6) st |= 0x08;  // proto TCP
        if (rem >= 20 && (dg[t0 + 12] >> 4) >= 5) st |= 0x04;  // tcp_segment.cpp:25-65
        if (mode == 1) {
          tcv = fold_value(pseudo + tot);  // tcp_segment.cpp:11-18
          if (hdr_ok && ipc == h.be16(10)) st |= 0x01;  // ipv4_header.cpp:53-58
          if (tcv == 0) st |= 0x02;
        } else {
          // tcp_segment.cpp:143: the checksum field counts as 0
          uint32_t sum = pseudo + tot;
          if (rem > 16) sum -= uint32_t(dg[t0 + 16]) << 8;
          if (rem > 17) sum -= uint32_t(dg[t0 + 17]);
          tcv = fold_value(sum);
          if (hdr_ok) st |= 0x01;
          if (rem >= 18) st |= 0x02;
          if (mode == 2) {
            dg[s + 10] = uint8_t(ipc >> 8);
            dg[s + 11] = uint8_t(ipc);
            if (rem >= 18) {
              dg[t0 + 16] = uint8_t(tcv >> 8);
              dg[t0 + 17] = uint8_t(tcv);
            }
          }
        }
      }
      if (ip_ck) ip_ck[seg] = ipc;
      if (tcp_ck) tcp_ck[seg] = tcv;
      if (status) status[seg] = st;
    }
  }
}

// --------------------------------------------------- router batch -------
__global__ __launch_bounds__(kBlock) void k_router_ttl(uint8_t* __restrict__ dg,
                                                       const uint64_t* __restrict__ offsets,
                                                       uint64_t stride, uint64_t dlen, uint64_t n,
                                                       uint8_t* __restrict__ status) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s, e;
  seg_bounds(offsets, stride, dlen, i, s, e);
  uint8_t st = 0;
  if (e - s >= 20) {
    Hdr h = load_hdr(dg + s);
    const uint32_t ver = h.byte(0) >> 4, hlen = h.byte(0) & 0x0fu, ttl = h.byte(8);
    // NetworkInterface::recv_frame parse (network_interface.cpp:51) then
    // Router::route: ttl <= 1 dropped, else ttl-- and compute_checksum()
    if (ver == 4 && hlen >= 5 && fold_value(ipv4_header_sum(h)) == h.be16(10) && ttl > 1) {
      h.w[2] = (h.w[2] & ~0xffu) | (ttl - 1);
      const uint16_t c = fold_value(ipv4_header_sum(h));
      dg[s + 6] = uint8_t(h.byte(6) & 0x7fu);  // re-serialized flags word
      dg[s + 8] = uint8_t(ttl - 1);
      dg[s + 10] = uint8_t(c >> 8);
      dg[s + 11] = uint8_t(c);
      st = 1;
    }
  }
  status[i] = st;
}

// ------------------------------------------------- workload spec ---------
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t sm64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t spec_word(uint64_t seed, uint64_t c) {
  return sm64(seed + (c + 1) * kGolden);
}

// Fast path: pos0 % 8 == 0 and d 16-byte aligned -> 16 bytes per thread.
__global__ void k_fill16(u32x4* __restrict__ d, uint64_t nvec, uint64_t seed, uint64_t w0) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const uint64_t a = spec_word(seed, w0 + 2 * i), b = spec_word(seed, w0 + 2 * i + 1);
  d[i] = u32x4{uint32_t(a), uint32_t(a >> 32), uint32_t(b), uint32_t(b >> 32)};
}

__global__ void k_fill1(uint8_t* __restrict__ d, uint64_t n, uint64_t seed, uint64_t pos0) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t p = pos0 + j;
  d[j] = uint8_t(spec_word(seed, p >> 3) >> (8 * (p & 7)));
}

__device__ __forceinline__ void spec_addrs(uint64_t seed, uint64_t i, uint32_t& src, uint32_t& dst) {
  const uint64_t m = spec_word(seed ^ 0xA5A5A5A5A5A5A5A5ull, i);
  src = 0x0A000000u | uint32_t(m & 0xFFFFFFu);
  dst = 0x0A000000u | uint32_t((m >> 24) & 0xFFFFFFu);
}

__global__ void k_pseudo_inits(uint32_t* __restrict__ init, const uint64_t* __restrict__ offsets,
                               uint64_t seg_len, uint64_t n, uint64_t seed, uint64_t index0) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t L = offsets ? offsets[i + 1] - offsets[i] : seg_len;
  uint32_t s, d;
  spec_addrs(seed, index0 + i, s, d);
  init[i] = (s >> 16) + (s & 0xffffu) + (d >> 16) + (d & 0xffffu) + 6u + uint32_t(L & 0xffffu);
}

__global__ void k_ipv4_tcp_headers(uint8_t* __restrict__ dg, uint64_t stride, uint64_t dlen,
                                   uint64_t n, uint64_t seed, uint64_t index0) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* d = dg + i * stride;
  const uint64_t id = index0 + i;
  uint32_t s, t;
  spec_addrs(seed, id, s, t);
  d[0] = 0x45;
  d[1] = 0;
  d[2] = uint8_t(dlen >> 8);
  d[3] = uint8_t(dlen);
  d[4] = uint8_t(id >> 8);
  d[5] = uint8_t(id);
  d[6] = 0x40;
  d[7] = 0;
  d[8] = 64;
  d[9] = 6;
  for (int k = 0; k < 4; ++k) {
    d[12 + k] = uint8_t(s >> (24 - 8 * k));
    d[16 + k] = uint8_t(t >> (24 - 8 * k));
  }
  if (dlen >= 40) {
    d[32] = 0x50;
    d[33] = 0x10;
    d[38] = 0;
    d[39] = 0;
  }
}

inline uint32_t blocks_for(uint64_t groups, uint32_t groups_per_block, uint32_t max_blocks) {
  uint64_t b = (groups + groups_per_block - 1) / groups_per_block;
  if (b == 0) b = 1;
  const uint64_t cap = max_blocks ? max_blocks : 0x7fffffffull;
  return uint32_t(b < cap ? b : cap);
}

template <int LPS, int UNROLL>
hipError_t launch_checksum_t(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                             int out_kind, uint32_t max_blocks, hipStream_t st) {
  const uint32_t blocks = blocks_for(sp.n, kBlock / LPS, max_blocks);
  if (out_kind == 0)
    hipLaunchKernelGGL((k_checksum<LPS, UNROLL, 0>), dim3(blocks), dim3(kBlock), 0, st, sp.bytes,
                       sp.offsets, sp.stride, sp.seg_len, init, odd, out, sp.n);
  else
    hipLaunchKernelGGL((k_checksum<LPS, UNROLL, 1>), dim3(blocks), dim3(kBlock), 0, st, sp.bytes,
                       sp.offsets, sp.stride, sp.seg_len, init, odd, out, sp.n);
  return hipGetLastError();
}

template <int LPS, int UNROLL>
hipError_t launch_ipv4_t(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck,
                         uint8_t* status, uint32_t max_blocks, hipStream_t st) {
  const uint32_t blocks = blocks_for(sp.n, kBlock / LPS, max_blocks);
  hipLaunchKernelGGL((k_ipv4_tcp<LPS, UNROLL>), dim3(blocks), dim3(kBlock), 0, st,
                     const_cast<uint8_t*>(sp.bytes), sp.offsets, sp.stride, sp.seg_len, sp.n, mode,
                     ip_ck, tcp_ck, status);
  return hipGetLastError();
}

}  // namespace

// geometry table: (LPS, UNROLL) pairs that are instantiated
Geometry pick_geometry(uint64_t avg_len) {
  const uint64_t chunks = avg_len / 16 + 2;
  if (chunks <= 8) return {4, 2};
  if (chunks <= 32) return {8, 4};
  if (chunks <= 64) return {16, 4};
  if (chunks <= 96) return {32, 3};
  if (chunks <= 128) return {32, 4};
  return {64, 4};
}

#define ICS_GEOMETRIES(X) X(4, 2) X(8, 4) X(16, 4) X(32, 3) X(32, 4) X(64, 4) X(64, 8)

hipError_t launch_checksum(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                           int out_kind, Geometry g, uint32_t max_blocks, hipStream_t st) {
#define ICS_CASE(L, U) \
  if (g.lps == L && g.unroll == U) return launch_checksum_t<L, U>(sp, init, odd, out, out_kind, max_blocks, st);
  ICS_GEOMETRIES(ICS_CASE)
#undef ICS_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_ipv4_tcp(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck,
                           uint8_t* status, Geometry g, uint32_t max_blocks, hipStream_t st) {
#define ICS_CASE(L, U) \
  if (g.lps == L && g.unroll == U) return launch_ipv4_t<L, U>(sp, mode, ip_ck, tcp_ck, status, max_blocks, st);
  ICS_GEOMETRIES(ICS_CASE)
#undef ICS_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_fold(const uint32_t* sum, uint16_t* out, uint64_t n, hipStream_t st) {
  const uint32_t blocks = uint32_t((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_fold, dim3(blocks ? blocks : 1), dim3(kBlock), 0, st, sum, out, n);
  return hipGetLastError();
}

hipError_t launch_router_ttl(const SegSpec& sp, uint8_t* status, hipStream_t st) {
  const uint32_t blocks = uint32_t((sp.n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_router_ttl, dim3(blocks ? blocks : 1), dim3(kBlock), 0, st,
                     const_cast<uint8_t*>(sp.bytes), sp.offsets, sp.stride, sp.seg_len, sp.n, status);
  return hipGetLastError();
}

hipError_t launch_fill_bytes(uint8_t* d, uint64_t nbytes, uint64_t seed, uint64_t pos0,
                             hipStream_t st) {
  if (nbytes == 0) return hipSuccess;
  if ((pos0 & 7) == 0 && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    const uint64_t nvec = nbytes / 16;
    if (nvec) {
      const uint64_t blocks = (nvec + kBlock - 1) / kBlock;
      hipLaunchKernelGGL(k_fill16, dim3(uint32_t(blocks)), dim3(kBlock), 0, st,
                         reinterpret_cast<u32x4*>(d), nvec, seed, pos0 >> 3);
    }
    const uint64_t done = nvec * 16, rest = nbytes - done;
    if (rest)
      hipLaunchKernelGGL(k_fill1, dim3(1), dim3(kBlock), 0, st, d + done, rest, seed, pos0 + done);
  } else {
    const uint64_t blocks = (nbytes + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_fill1, dim3(uint32_t(blocks)), dim3(kBlock), 0, st, d, nbytes, seed, pos0);
  }
  return hipGetLastError();
}

hipError_t launch_pseudo_inits(uint32_t* init, const uint64_t* offsets, uint64_t seg_len,
                               uint64_t n, uint64_t seed, uint64_t index0, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pseudo_inits, dim3(uint32_t((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                     init, offsets, seg_len, n, seed, index0);
  return hipGetLastError();
}

hipError_t launch_ipv4_tcp_headers(uint8_t* d, uint64_t stride, uint64_t dgram_len, uint64_t n,
                                   uint64_t seed, uint64_t index0, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ipv4_tcp_headers, dim3(uint32_t((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     st, d, stride, dgram_len, n, seed, index0);
  return hipGetLastError();
}

}  // namespace icsum
