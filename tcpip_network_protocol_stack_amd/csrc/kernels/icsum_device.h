// icsum_device.h — device building blocks of the checksum engine (gfx950).
//
// The reference sums one byte at a time with a parity flag
// (util/tools/checksum.h:20-28): sum_ += parity ? b : b << 8.  Over a segment
// that is S = s0 + 256*E + O (mod 2^32) where E / O are the sums of the bytes at
// even / odd positions relative to the segment start.  uint32 addition is
// associative, so any split of the bytes over lanes, waves or launches
// reproduces sum_ exactly, wrap above 131074 bytes of 0xFF included.
//
// Per 16-byte chunk a lane does one dwordx4 load and eight v_dot4_u32_u8:
// udot4(w, 0x00010001) adds the two bytes of a little-endian dword that sit at
// even addresses, udot4(w, 0x01000100) the two at odd addresses.  Roles are
// taken from the absolute address and swapped once at the end when the
// segment starts at an odd address.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace icsum {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kEvenBytes = 0x00010001u;  // bytes 0 and 2 of a dword
constexpr uint32_t kOddBytes = 0x01000100u;   // bytes 1 and 3 of a dword

__device__ __forceinline__ void acc_dword(uint32_t w, uint32_t& e, uint32_t& o) {
  e = __builtin_amdgcn_udot4(w, kEvenBytes, e, false);
  o = __builtin_amdgcn_udot4(w, kOddBytes, o, false);
}

__device__ __forceinline__ void acc_chunk(u32x4 v, uint32_t& e, uint32_t& o) {
  acc_dword(v.x, e, o);
  acc_dword(v.y, e, o);
  acc_dword(v.z, e, o);
  acc_dword(v.w, e, o);
}

// Mask keeping bytes [lo, hi) of a 16-byte chunk (0 <= lo <= 16, 0 <= hi <= 16).
__device__ __forceinline__ u32x4 byte_range_mask(uint32_t lo, uint32_t hi) {
  // keep-from-lo: 128-bit ~0 << 8*lo ; keep-below-hi: (1 << 8*hi) - 1
  const uint64_t all = ~0ull;
  const uint64_t f0 = lo >= 8 ? 0ull : all << (8 * lo);
  const uint64_t f1 = lo >= 16 ? 0ull : (lo >= 8 ? all << (8 * (lo - 8)) : all);
  const uint64_t b0 = hi >= 8 ? all : ((1ull << (8 * hi)) - 1);
  const uint64_t b1 = hi >= 16 ? all : (hi <= 8 ? 0ull : ((1ull << (8 * (hi - 8))) - 1));
  const uint64_t m0 = f0 & b0, m1 = f1 & b1;
  u32x4 m;
  m.x = uint32_t(m0);
  m.y = uint32_t(m0 >> 32);
  m.z = uint32_t(m1);
  m.w = uint32_t(m1 >> 32);
  return m;
}

// checksum.h:31-41 — two end-around folds always reach <= 0xFFFF for a uint32.
__device__ __forceinline__ uint16_t fold_value(uint32_t s) {
  uint32_t r = (s >> 16) + (s & 0xffffu);
  r = (r >> 16) + (r & 0xffffu);
  return uint16_t(~r);
}

// This lane's share of the running sum over bytes [s, e) of `base`, with byte
// roles relative to s, XOR `flip` (1 = the first byte is a low byte, i.e. the
// reference's parity_ was already odd).  A group of LPS lanes covers the
// 16-byte-aligned chunks that overlap [s, e); bytes outside [s, e) inside
// those chunks are read and masked off (they share a 16-byte block, hence a
// page, with bytes of the segment).
template <int LPS, int UNROLL>
__device__ __forceinline__ uint32_t range_partial(const uint8_t* __restrict__ base, uint64_t s,
                                                  uint64_t e, uint32_t lane, uint32_t flip) {
  uint32_t ev = 0, od = 0;
  if (e > s) {
    const uint64_t a0 = s & ~uint64_t(15);
    const uint64_t span = e - a0;  // bytes from the first chunk start to the end
    const uint32_t nch = uint32_t((span + 15) >> 4);
    const uint32_t lo0 = uint32_t(s - a0);
    const u32x4* __restrict__ p = reinterpret_cast<const u32x4*>(base + a0);
    for (uint32_t c = lane; c < nch; c += uint32_t(LPS * UNROLL)) {
      u32x4 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const uint32_t cc = c + uint32_t(u * LPS);
        v[u] = cc < nch ? __builtin_nontemporal_load(p + cc) : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const uint32_t cc = c + uint32_t(u * LPS);
        const uint64_t at = uint64_t(cc) << 4;
        const uint32_t lo = cc == 0 ? lo0 : 0u;
        const uint32_t hi = at >= span ? 0u : (span - at >= 16 ? 16u : uint32_t(span - at));
        acc_chunk(v[u] & byte_range_mask(lo, hi), ev, od);
      }
    }
  }
  // absolute even addresses are high bytes iff the segment starts even
  if (((uint32_t(s) & 1u) ^ flip) != 0u) {
    const uint32_t t = ev;
    ev = od;
    od = t;
  }
  return ev * 256u + od;
}

// Sum over the LPS lanes of an aligned lane group (all 64 lanes must execute).
template <int LPS>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
#pragma unroll
  for (int o = LPS / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

}  // namespace icsum
