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

// ---- bounds-checked build (libicsum_debug.so, -DICSUM_BOUNDS_CHECK) --------
// SURVEY §5's device bounds-check variant.  Every 16-byte payload load is
// checked against its segment's envelope (the aligned blocks that hold the
// segment's bytes: the documented read set), every
// offsets pair for e >= s, and every IPv4 header dword against the
// datagram's last dword.  A violation sets a bit in a device word (vector
// atomics) with the first offending address; the C-ABI synchronises after
// each call, reads it and returns ICS_ERR_INVALID.  The release build
// compiles all of it away.
#ifdef ICSUM_BOUNDS_CHECK
struct BoundsState {
  unsigned int flags;  // ICS_BOUNDS_* bits
  unsigned int pad;
  unsigned long long addr;  // first offending address (or segment index for an offsets fault)
};
extern __device__ BoundsState g_icsum_bounds;
constexpr unsigned kBoundsLoad = 1u, kBoundsOffsets = 2u, kBoundsHeader = 4u;
__device__ __forceinline__ void bounds_fail(unsigned bit, unsigned long long what) {
  if (atomicOr(&g_icsum_bounds.flags, bit) == 0u) atomicExch(&g_icsum_bounds.addr, what);
}
__device__ __forceinline__ void bounds_check16(const void* p, const uint8_t* lo, const uint8_t* hi) {
  const uint8_t* q = static_cast<const uint8_t*>(p);
  if (q < lo || q + 16 > hi) bounds_fail(kBoundsLoad, reinterpret_cast<unsigned long long>(p));
}
#define ICS_CHECK16(p, lo, hi) ::icsum::bounds_check16((p), (lo), (hi))
#else
#define ICS_CHECK16(p, lo, hi) ((void)0)
#endif

// ---- byte bases at any address -------------------------------------------
// The reference sums bytes at any address (InternetChecksum::add takes any
// string_view, checksum.h:20-28; a receive arena of Ethernet frames holds its
// IPv4 datagrams 14 bytes in, network_interface.cpp:51).  Every kernel works
// in the frame of the 16-byte-aligned address at or below its byte base: it
// moves the base down by frame_shift(base) and adds the shift to every
// segment bound, so chunk loads, 128-byte lines and byte roles are absolute
// and a boundary load never leaves the 16-byte block — hence the page — that
// holds a byte of the batch.  (Pointer arithmetic, not an integer mask: the
// base stays a global pointer.)
__device__ __forceinline__ uint32_t frame_shift(const void* p) {
  return uint32_t(reinterpret_cast<uintptr_t>(p) & 15u);
}

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

template <bool NT>
__device__ __forceinline__ u32x4 load16(const u32x4* __restrict__ p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

// Even/odd byte sums of this lane's share of bytes [s, e) of `base`, roles by
// ABSOLUTE address (even address -> `ev`).  The range is cut into the 16-byte
// aligned chunks that overlap it: chunk 0 and chunk nch-1 are the only ones
// that can be partial.  A group of LPS lanes streams the interior chunks
// 1..nch-2 unmasked — lane l takes l+1, l+1+LPS, ... with UNROLL loads issued
// back to back per step and no branches (slots past the end re-load the last
// interior chunk and are zeroed) — then one masked slot handles the two
// boundary chunks (lane 0: chunk 0, lane 1: chunk nch-1; LPS == 1 does both).
// Bytes outside [s, e) inside a boundary chunk are read and discarded: they
// share a 16-byte block, hence a page, with bytes of the segment.
template <int LPS, int UNROLL, bool NT>
__device__ __forceinline__ void range_sums(const uint8_t* __restrict__ base, uint64_t s, uint64_t e,
                                           uint32_t lane, uint32_t& ev, uint32_t& od) {
  const uint64_t a0 = s & ~uint64_t(15);
  const uint64_t span = e > a0 ? e - a0 : 0;  // bytes from the first chunk start to the end
  const uint32_t nch = uint32_t((span + 15) >> 4);
  const u32x4* __restrict__ p = reinterpret_cast<const u32x4*>(base + a0);
  [[maybe_unused]] const uint8_t* env_lo = base + a0;
  [[maybe_unused]] const uint8_t* env_hi = base + ((e + 15) & ~uint64_t(15));
  // boundary chunks 0 and nch-1 are loaded FIRST so that their latency
  // overlaps the interior stream: lane 0 -> chunk 0, lane 1 -> chunk nch-1
  // (when distinct), other lanes re-load chunk 0 and mask it to nothing.
  const uint32_t lo0 = uint32_t(s - a0);
  const uint32_t tail = nch ? uint32_t(span - (uint64_t(nch - 1) << 4)) : 0u;  // valid bytes of the last chunk
  const uint32_t lastc = nch ? nch - 1 : 0u;
  u32x4 bh = {0u, 0u, 0u, 0u}, bt = {0u, 0u, 0u, 0u};
  uint32_t blo = 0, bhi = 0;
  if (LPS == 1) {
    if (nch) {
      ICS_CHECK16(p, env_lo, env_hi);
      ICS_CHECK16(p + lastc, env_lo, env_hi);
      bh = load16<NT>(p);
      bt = load16<NT>(p + lastc);
    }
  } else if (nch) {
    const bool is_tail = lane == 1 && nch >= 2;
    ICS_CHECK16(p + (is_tail ? lastc : 0u), env_lo, env_hi);
    bh = load16<NT>(p + (is_tail ? lastc : 0u));
    blo = is_tail ? 0u : lo0;
    bhi = (is_tail || nch == 1) ? tail : 16u;
    if (lane >= 2 || (lane == 1 && nch < 2)) bhi = 0u;  // empty mask
  }
  // interior chunks [1, nch-1), unmasked
  const uint32_t last_in = nch >= 2 ? nch - 2 : 0;  // last interior chunk index (if nch >= 3)
  for (uint32_t c = lane + 1; c + 1 < nch; c += uint32_t(LPS * UNROLL)) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t cc = c + uint32_t(u * LPS);
      ICS_CHECK16(p + (cc <= last_in ? cc : last_in), env_lo, env_hi);
      v[u] = load16<NT>(p + (cc <= last_in ? cc : last_in));
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t cc = c + uint32_t(u * LPS);
      const uint32_t keep = cc <= last_in ? ~0u : 0u;
      acc_chunk(v[u] & keep, ev, od);
    }
  }
  if (LPS == 1) {
    if (nch) {
      acc_chunk(bh & byte_range_mask(lo0, nch == 1 ? tail : 16u), ev, od);
      if (nch >= 2) acc_chunk(bt & byte_range_mask(0u, tail), ev, od);
    }
  } else {
    acc_chunk(bh & byte_range_mask(blo, bhi), ev, od);
  }
}

// Line-anchored grid with the two boundary chunks loaded FIRST, with the
// default (cache-allocating) policy, by lanes 0 (head) and 1 (tail) of the
// group; the slot loop then streams only the interior chunks non-temporally
// and unmasked (a keep mask per slot, no per-slot copies).  The boundary lines
// are the ones a neighbouring segment also touches: kept in L2 they are read
// from HBM once.
template <int LPS, int UNROLL, bool NT>
__device__ __forceinline__ void range_sums_line_primed(const uint8_t* __restrict__ base, uint64_t s,
                                                       uint64_t e, uint32_t lane, uint32_t& ev,
                                                       uint32_t& od) {
  const uint64_t a0 = s & ~uint64_t(127);
  const uint64_t span = e > s ? e - a0 : 0;
  const uint32_t nch = uint32_t((span + 15) >> 4);
  const uint32_t cs = uint32_t(s - a0) >> 4;  // head chunk (0..7)
  const uint32_t lastc = nch ? nch - 1 : 0u;  // tail chunk
  const u32x4* __restrict__ p = reinterpret_cast<const u32x4*>(base + a0);
  [[maybe_unused]] const uint8_t* env_lo = base + a0;
  [[maybe_unused]] const uint8_t* env_hi = base + ((e + 15) & ~uint64_t(15));
  const uint32_t tail = nch ? uint32_t(span - (uint64_t(lastc) << 4)) : 0u;
  u32x4 bnd = {0u, 0u, 0u, 0u};
  uint32_t blo = 0, bhi = 0;
  if (nch) {
    const bool is_tail = (LPS == 1 ? false : lane == 1) && lastc != cs;
    ICS_CHECK16(p + (is_tail ? lastc : cs), env_lo, env_hi);
    bnd = load16<false>(p + (is_tail ? lastc : cs));
    blo = is_tail ? 0u : (uint32_t(s) & 15u);
    bhi = (is_tail || lastc == cs) ? tail : 16u;
    if (LPS > 1 && (lane >= 2 || (lane == 1 && lastc == cs))) bhi = 0u;
  }
  u32x4 bt = {0u, 0u, 0u, 0u};
  if (LPS == 1 && nch && lastc != cs) {
    ICS_CHECK16(p + lastc, env_lo, env_hi);
    bt = load16<false>(p + lastc);
  }
  for (uint32_t c = lane; c < nch; c += uint32_t(LPS * UNROLL)) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t cc = c + uint32_t(u * LPS);
      ICS_CHECK16(p + (cc < lastc ? cc : lastc), env_lo, env_hi);
      v[u] = load16<NT>(p + (cc < lastc ? cc : lastc));
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t cc = c + uint32_t(u * LPS);
      const uint32_t keep = (cc > cs && cc < lastc) ? ~0u : 0u;
      acc_chunk(v[u] & keep, ev, od);
    }
  }
  acc_chunk(bnd & byte_range_mask(blo, bhi), ev, od);
  if (LPS == 1) acc_chunk(bt & byte_range_mask(0u, tail), ev, od);
}

// Fully masked variant on the 16-byte grid: slot u of lane l is chunk
// l + u*LPS of [s & ~15, e), every slot masked to [s, e).  One load per
// useful chunk with no separate boundary instruction: the cheapest shape for
// segments of a few chunks (64 B = 4 lanes x 1 load, one 1 KiB wave
// instruction per 16 segments), at ~20 more VALU per slot.
template <int LPS, int UNROLL, bool NT>
__device__ __forceinline__ void range_sums_masked(const uint8_t* __restrict__ base, uint64_t s,
                                                  uint64_t e, uint32_t lane, uint32_t& ev,
                                                  uint32_t& od) {
  const uint64_t a0 = s & ~uint64_t(15);
  const uint64_t span = e > s ? e - a0 : 0;
  const uint32_t nch = uint32_t((span + 15) >> 4);
  const uint32_t lo0 = uint32_t(s - a0);
  const u32x4* __restrict__ p = reinterpret_cast<const u32x4*>(base + a0);
  [[maybe_unused]] const uint8_t* env_lo = base + a0;
  [[maybe_unused]] const uint8_t* env_hi = base + ((e + 15) & ~uint64_t(15));
  for (uint32_t c = lane; c < nch; c += uint32_t(LPS * UNROLL)) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t cc = c + uint32_t(u * LPS);
      ICS_CHECK16(p + (cc < nch ? cc : nch - 1), env_lo, env_hi);
      v[u] = load16<NT>(p + (cc < nch ? cc : nch - 1));
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

// Chunk-grid modes (Geometry::mode): 0 = 16-byte grid, interior unmasked +
// boundary instruction (the fused kernel's one-lane shape); 2 = 16-byte grid,
// all masked (4- and 8-lane shapes); 3 = 128-byte-line grid, slot u of a group
// covering chunks [u*LPS, (u+1)*LPS) from the line that holds the start, with
// default-policy boundary loads issued first (every longer segment).  Mode 1
// (the line grid without the primed boundary loads) was superseded by 3.
template <int LPS, int UNROLL, bool NT, int MODE>
__device__ __forceinline__ void seg_sums(const uint8_t* __restrict__ base, uint64_t s, uint64_t e,
                                         uint32_t lane, uint32_t& ev, uint32_t& od) {
  static_assert(MODE == 0 || MODE == 2 || MODE == 3, "chunk-grid mode");
  if (MODE == 3)
    range_sums_line_primed<LPS, UNROLL, NT>(base, s, e, lane, ev, od);
  else if (MODE == 2)
    range_sums_masked<LPS, UNROLL, NT>(base, s, e, lane, ev, od);
  else
    range_sums<LPS, UNROLL, NT>(base, s, e, lane, ev, od);
}

// Sum over each aligned group of LPS lanes with DPP (no LDS round trips):
// quad_perm xor1/xor2, row_half_mirror, row_mirror, then row_bcast15 /
// row_bcast31 for 32/64-lane groups.  The complete sum lands in the group's
// last lane (LPS-1); for LPS <= 16 every lane of the group holds it.  All 64
// lanes must execute this.
template <int LPS>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
  if (LPS >= 2) x += __builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  if (LPS >= 4) x += __builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  if (LPS >= 8) x += __builtin_amdgcn_update_dpp(0u, x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if (LPS >= 16) x += __builtin_amdgcn_update_dpp(0u, x, 0x140, 0xF, 0xF, false); // row_mirror
  if (LPS >= 32) x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false); // row_bcast:15
  if (LPS >= 64) x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false); // row_bcast:31
  return x;
}

// S contribution of a range from its absolute even/odd sums: the byte at the
// range start is a high byte unless (start address parity XOR carried parity).
__device__ __forceinline__ uint32_t combine_roles(uint32_t ev, uint32_t od, uint32_t swap) {
  return swap ? od * 256u + ev : ev * 256u + od;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

}  // namespace icsum
