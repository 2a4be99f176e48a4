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

#include <algorithm>
#include <type_traits>

#include "icsum_device.h"
#include "icsum_launch.h"

namespace icsum {

#ifdef ICSUM_BOUNDS_CHECK
__device__ BoundsState g_icsum_bounds;
#endif

namespace {

constexpr int kBlock = 256;

// segment i's bounds in the kernel's frame (sh = frame_shift of the batch's
// byte base, icsum_device.h)
__device__ __forceinline__ void seg_bounds(const uint64_t* __restrict__ offsets, uint64_t stride,
                                           uint64_t seg_len, uint64_t i, uint64_t& s,
                                           uint64_t& e, uint32_t sh) {
  if (offsets) {
    s = offsets[i];
    e = offsets[i + 1];
#ifdef ICSUM_BOUNDS_CHECK
    if (e < s) bounds_fail(kBoundsOffsets, i);  // offsets must be monotone
#endif
  } else {
    s = i * stride;
    e = s + seg_len;
  }
  s += sh;
  e += sh;
}

// ------------------------------------------------------- length binning ---
// Bin of a segment by its 16-byte chunk count; the boundaries are those of
// pick_geometry, so bin b runs with the geometry pick_geometry gives a batch
// of such segments.
constexpr uint64_t kBinMaxChunks[kBins - 1] = {9, 56, 120, 256};
constexpr int kBinPerThread = 8;  // segments per thread per tile
constexpr int kBinTile = kBlock * kBinPerThread;
constexpr int kBinField = 12;  // bits per bin in a packed count

__device__ __forceinline__ int bin_of(uint64_t len) {
  const uint64_t m = (len + 15) >> 4;
  int b = 0;
#pragma unroll
  for (int k = 0; k < kBins - 1; ++k) b += m > kBinMaxChunks[k];
  return b;
}

// Packed per-bin counts: kBins fields of 12 bits in a uint64 (a tile holds
// 2048 segments, so no field overflows and adding packed words never carries
// across fields).
__device__ __forceinline__ uint32_t field(uint64_t p, int b) {
  return uint32_t(p >> (kBinField * b)) & ((1u << kBinField) - 1);
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t u = __shfl_up(v, d, 64);
    if (lane >= uint32_t(d)) v += u;
  }
  return v;
}

// exclusive block scan of packed counts; returns the block total in `total`
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t& total) {
  __shared__ uint64_t wsum[kBlock / 64];
  const uint64_t inc = wave_incl_scan(v);
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) wsum[w] = inc;
  __syncthreads();
  uint64_t before = 0;
  total = 0;
#pragma unroll
  for (uint32_t k = 0; k < kBlock / 64; ++k) {
    before += k < w ? wsum[k] : 0;
    total += wsum[k];
  }
  __syncthreads();  // wsum is reused by the next tile
  return before + inc - v;
}

// Dispatch plan of a binned batch, decided on the device (k_bin_plan, one
// block after the stats pass) from
// the bin sizes the binning pass recorded, with no host round trip:
//   kPlanWhole  the last bin's launch takes every segment with its own
//               (64- or 32-lane) geometry; the other launches exit at once
//   kPlanSplit  every bin runs from its list with its own geometry
//   kPlanWhole16 the last bin's launch takes every segment with 16-lane
//               groups in its first n/16 blocks (the rest exit at once)
//   kPlanWholeSmall the last bin's launch takes every segment through the
//               small-segment body (or one lane per segment for ACK-sized means)
// The choice is the cheapest plan under kPlanCost (below): every estimate is
// in ns, a sum over the bins of max(bytes / rate, segments * per-segment
// cost) plus the dispatch of the last bin's idle waves.
// Measured under each forced plan (git 7692616:tools/ab_lastbin.py --var ICSUM_BIN_PLAN,
// profiles/r1_ab_plans.jsonl), µs whole / split / whole16: config 4
// 1429 / 1622 / 1682, 2 M bimodal 40+1460 B 525 / 473 / 364, 2 M x 4-6 KiB
// 1515 / 1589 / 1593, 1 M x 1460 B 520 / 429 / 296, 1 M x 40 B 451 / 168 / 205.
struct PlanCostTable {
  // rates in GB/s (= bytes per ns), per-segment costs in ns x 100; sources in profiles/
  uint32_t whole_rate;            // whole: 64-lane groups over a long mix; config 4 whole 1429 us = 7.2 TB/s (r1_ab_plans)
  uint32_t whole_seg_c;           // whole: ns x 100 per segment floor; 1 M x 40 B whole 451 us (r1_ab_plans)
  uint32_t split_fixed_ns;        // split: the scatter pass and the bins 0-3 launch, 26 us fixed (git 7692616:tools/ab_bins.py, r1_ab_bins)
  uint32_t empty_wave_ps;         // every plan: an idle wave of the last bin's launch, 0.053 ns (git 7692616:tools/probe/dispatch_probe.hip)
  uint32_t split_rate_bins;       // split: bins 0-3 from their lists, 5.0 TB/s (r1_ab_bins)
  uint32_t split_rate_last;       // split: last bin, segments no longer contiguous, 6.4 TB/s (r1_ab_bins)
  uint32_t split_seg_c;           // split: ns x 100 per listed segment (r1_ab_bins: 1 M x 40 B split 168 us)
  uint32_t w16_rate[kBins];       // whole16 per bin: 7.0 TB/s to 1920 B, 6.5 to 4 KiB, 5.0 above (16 lanes loop; r1_ab_plans)
  uint32_t w16_seg_c;             // whole16: ns x 100 per segment (1 M x 1460 B whole16 296 us)
  uint32_t small_rate[kBins];     // wholeS per bin: 5.0 TB/s for bin 0, 0.8 for longer (4 lanes loop; r1_ab_plans small)
  uint32_t small_seg_c[kBins];    // wholeS: ns x 100 per segment, 0.02 bin 0 / 0.5 longer (1 M x 40-43 B small 140 us)
};
constexpr PlanCostTable kPlanCost = {7100, 45, 26000, 53, 5000, 6400, 10,
                                     {7000, 7000, 7000, 6500, 5000}, 16,
                                     {5000, 800, 800, 800, 800}, {2, 50, 50, 50, 50}};
constexpr uint32_t kPlanWhole = 0, kPlanSplit = 1, kPlanWhole16 = 2, kPlanWholeSmall = 3;
static_assert(kPlanWhole == kPlanWholeBatch && kPlanSplit == kPlanSplitBins && kPlanWhole16 == kPlanWholeBatch16 &&
              kPlanWholeSmall == kPlanWholeBatchSmall, "plan ids shared with the host's plan cache");

__global__ __launch_bounds__(kBlock) void k_bin_plan(uint32_t* __restrict__ meta, const uint32_t* __restrict__ cnt_part,
                                                     const uint64_t* __restrict__ by_part, uint32_t parts, uint64_t n,
                                                     int force, uint32_t last_lps, uint64_t* __restrict__ plan_out,
                                                     uint32_t gen) {
  // totals per bin from the stats pass's per-block partials (parts <= kBlock:
  // one partial per thread, all loads in flight together)
  __shared__ uint32_t wc[kBlock / 64][kBins];
  __shared__ uint64_t wb[kBlock / 64][kBins];
  const uint32_t w = threadIdx.x >> 6;
  const bool mine = threadIdx.x < parts;
  uint32_t cs[kBins];
  uint64_t vs[kBins];
#pragma unroll
  for (int k = 0; k < kBins; ++k) {
    cs[k] = mine ? cnt_part[k * parts + threadIdx.x] : 0;
    vs[k] = mine ? by_part[k * parts + threadIdx.x] : 0;
  }
#pragma unroll
  for (int k = 0; k < kBins; ++k) {
    uint32_t c = cs[k];
    uint64_t v = vs[k];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      c += __shfl_xor(c, d, 64);
      v += __shfl_xor(v, d, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      wc[w][k] = c;
      wb[w][k] = v;
    }
  }
  // the scatter pass's cursors start at 0 (zeroed here, in stream order before
  // it, instead of by a separate memset launch: one dispatch less per batch)
  if (threadIdx.x < kBins) meta[kBinMetaCursor + threadIdx.x] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t waves = n * last_lps / 64;  // the last bin's launch
    const PlanCostTable& C = kPlanCost;
    uint64_t total = 0, short_n = 0, long_bytes = 0;
    uint64_t t_split = C.split_fixed_ns + waves * C.empty_wave_ps / 1000;
    uint64_t t16 = (waves - n / 4) * C.empty_wave_ps / 1000;        // whole16 uses the first n/16 blocks
    uint64_t t_small = (waves - n / 32) * C.empty_wave_ps / 1000;   // wholeS the first n/128
#pragma unroll
    for (int k = 0; k < kBins; ++k) {
      uint32_t c = 0;
      uint64_t v = 0;
#pragma unroll
      for (uint32_t q = 0; q < kBlock / 64; ++q) {
        c += wc[q][k];
        v += wb[q][k];
      }
      meta[kBinMetaCount + k] = c;
      if (k == 0) short_n = c;
      if (k >= 3) long_bytes += v;  // segments > 1920 bytes
      total += v;
      const uint64_t tb = v / (k == kBins - 1 ? C.split_rate_last : C.split_rate_bins), tn = uint64_t(c) * C.split_seg_c / 100;
      t_split += tb > tn ? tb : tn;
      const uint64_t sb = v / C.w16_rate[k], sn = uint64_t(c) * C.w16_seg_c / 100;
      t16 += sb > sn ? sb : sn;
      const uint64_t mb = v / C.small_rate[k], mn = uint64_t(c) * C.small_seg_c[k] / 100;
      t_small += mb > mn ? mb : mn;
    }
    const uint64_t tb = total / C.whole_rate, tn = n * C.whole_seg_c / 100, t_whole = tb > tn ? tb : tn;
    uint32_t plan = kPlanWhole;
    if (force >= 0) {
      plan = uint32_t(force);
    } else {
      uint64_t best = t_whole;
      if (t_split < best) best = t_split, plan = kPlanSplit;
      if (t16 < best) best = t16, plan = kPlanWhole16;
      if (t_small < best) plan = kPlanWholeSmall;
    }
    meta[kBinMetaPlan] = plan;
    const uint64_t avg = n ? total / n : 0;
    meta[kBinMetaAvgLen] = uint32_t(avg < 0xFFFFFFFFull ? avg : 0xFFFFFFFFull);
    // the host's plan cache (icsum_dispatch.cpp), one 8-byte store to page-locked
    // host memory: the plan (bits 0-3), the share of bin-0 (<= 144-byte)
    // segments in sixteenths (bits 4-7), the batch size (bits 8-39), the
    // share of bytes in segments over 1920 bytes in sixteenths (bits 40-43)
    // the mean segment length in bytes, capped at 4095 (bits 44-55), and the
    // generation of the cache slot that asked for it (bits 56-63)
    const uint64_t short16 = n ? short_n * 16 / n : 0, long16 = total ? long_bytes * 16 / total : 0;
    if (plan_out)
      *plan_out = plan | ((short16 < 15 ? short16 : 15) << 4) | ((n & 0xFFFFFFFFull) << 8) |
                  ((long16 < 15 ? long16 : 15) << 40) | ((avg < 4095 ? avg : 4095) << 44) |
                  (uint64_t(gen & 0xffu) << 56);
  }
}

// Where a launch finds its segments: fixed stride, packed offsets, or a
// length bin written by k_bin_segments (entries {start lo, start hi, length,
// segment index}; capacity n, so any index < n is a safe read).
struct SegSrc {
  const uint64_t* offsets;
  uint64_t stride, seg_len;
  const u32x4* list;     // bin launch: this bin's entries
  const uint32_t* meta;  // bin launch: the binning pass's sizes and plan
  int bin;
  uint32_t shift = 0;    // frame_shift of the byte base, set by the kernel (rebase)
};

// the kernel's frame of its byte base (icsum_device.h): bytes moved down to
// the 16-byte-aligned address, the shift recorded for src_decode
template <typename T>
__device__ __forceinline__ T* rebase(T* bytes, SegSrc& src) {
  src.shift = frame_shift(bytes);
  return bytes - src.shift;
}

// A launch's work, resolved once at kernel start: the bin's list (split plan)
// or, for the last bin's launch under the whole-batch plan, every segment by
// index.  Items are walked by a grid stride; the last bin's launch has one
// lane group per segment of the batch (no stride), bins 0..3 a capped grid.
struct Work {
  uint64_t items;
  const u32x4* list;  // null: segment i = item i
};

__device__ __forceinline__ Work resolve(const SegSrc& src, uint64_t n) {
  if (!src.list) return Work{n, nullptr};
  // selects, not branches, keep every path explicit
  const uint32_t plan = src.meta[kBinMetaPlan];
  const bool split = plan == kPlanSplit;
  const bool last = src.bin == kBins - 1;
  Work w;
  w.items = split ? uint64_t(src.meta[kBinMetaCount + src.bin]) : (last && plan == kPlanWhole ? n : 0);
  w.list = split ? src.list : nullptr;
  return w;
}

constexpr uint32_t kLongEntry = 0xFFFFFFFFu;  // entry length: >= 4 GiB, re-read the offsets

// Raw metadata of one work item (loads from clamped indices, so they are
// unconditional and never wait at a join).
struct ItemMeta {
  u32x4 ent;     // list entry
  uint64_t a, b;  // offsets[i], offsets[i + 1]
};

__device__ __forceinline__ ItemMeta src_fetch(const SegSrc& src, const Work& w, uint64_t gi, uint64_t n) {
  ItemMeta m{};
  const uint64_t c = gi < n ? gi : n - 1;  // list capacity n, offsets n + 1
  if (w.list) {
    m.ent = w.list[c];
  } else if (src.offsets) {
    m.a = src.offsets[c];
    m.b = src.offsets[c + 1];
  }
  return m;
}

// segment number, start and end of work item gi; an item past the end
// (gi >= items) gets seg = s = e = 0
__device__ __forceinline__ void src_decode(const SegSrc& src, const Work& w, uint64_t gi, const ItemMeta& m,
                                           uint64_t& seg, uint64_t& s, uint64_t& e) {
  seg = s = e = 0;
  if (gi >= w.items) return;
  if (w.list) {
    seg = m.ent.w;
    if (m.ent.z != kLongEntry) {
      s = uint64_t(m.ent.x) | (uint64_t(m.ent.y) << 32);
      e = s + m.ent.z;
    } else {
      seg_bounds(src.offsets, 0, 0, seg, s, e, 0u);
    }
  } else {
    seg = gi;
    if (src.offsets) {
      s = m.a;
      e = m.b;
#ifdef ICSUM_BOUNDS_CHECK
      if (e < s) bounds_fail(kBoundsOffsets, gi);  // offsets must be monotone
#endif
    } else {
      s = gi * src.stride;
      e = s + src.seg_len;
    }
  }
  s += src.shift;  // the kernel's frame (rebase)
  e += src.shift;
}

__device__ __forceinline__ void src_locate(const SegSrc& src, const Work& w, uint64_t gi, uint64_t n,
                                           uint64_t& seg, uint64_t& s, uint64_t& e) {
  src_decode(src, w, gi, src_fetch(src, w, gi, n), seg, s, e);
}

// ------------------------------------------------------------ a1-a4 -------
// `init` / `odd` are never null here: an absent array is replaced by a
// 16-byte zero buffer read with index step 0 (init_step / odd_step).
// (block blk of nblk: a kernel of its own, or one bin's share of k_checksum_bins)
template <int LPS, int UNROLL, bool NT, int MODE, int OUT>
__device__ __forceinline__ void checksum_body(const uint8_t* __restrict__ bytes, const SegSrc& src,
                                              const uint32_t* __restrict__ init, uint32_t init_step,
                                              const uint8_t* __restrict__ odd, uint32_t odd_step,
                                              void* __restrict__ out, uint64_t n, uint32_t blk, uint32_t nblk) {
  constexpr uint32_t kGroups = kBlock / LPS;
  const uint32_t lane = threadIdx.x & (LPS - 1);
  const Work w = resolve(src, n);
  auto item = [&](uint64_t gi, const ItemMeta& m) {
    uint64_t seg, s, e;
    src_decode(src, w, gi, m, seg, s, e);
    const bool valid = gi < w.items;
    // per-segment metadata is requested together with the byte stream, so a
    // wave waits on memory once (the leader lane folds it in at the end)
    // (unconditional loads from a clamped index: a load under a divergent
    // branch would make the compiler wait for it at the join)
    const bool leader = valid && lane == LPS - 1;
    const uint64_t cseg = seg;  // 0 for idle lanes (n >= 1)
    const uint32_t i0 = init[cseg * init_step];
    // a high byte at the start unless the start is odd XOR parity_ was already odd
    const uint32_t swap = (uint32_t(s) ^ uint32_t(odd[cseg * odd_step])) & 1u;
    uint32_t ev = 0, od = 0;
    seg_sums<LPS, UNROLL, NT, MODE>(bytes, s, e, lane, ev, od);
    const uint32_t tot = group_sum<LPS>(combine_roles(ev, od, swap));
    if (leader) {
      const uint32_t sum = i0 + tot;
      if (OUT == 0)
        static_cast<uint16_t*>(out)[seg] = fold_value(sum);
      else
        static_cast<uint32_t*>(out)[seg] = sum;
    }
  };
  // the pass bound is uniform per block, so every lane reaches the DPP sums
  for (uint64_t g0 = uint64_t(blk) * kGroups; g0 < w.items; g0 += uint64_t(nblk) * kGroups) {
    const uint64_t gi = g0 + threadIdx.x / LPS;
    item(gi, src_fetch(src, w, gi, n));
  }
}

// XCD-aware block order.  Blocks b and b + 8 are observed to share an XCD
// (MI355X_MICROARCH.md §Workgroup dispatch: blocks are dealt round-robin over
// the 8 XCDs), so the hardware order gives every XCD every 8th block — each
// XCD's L2 and address translation see 8 disjoint pieces per run of blocks.
// Remapped, XCD label x = b % 8 takes runs of c consecutive logical blocks
// (c = min(run, grid / 8), powers of two): each XCD streams contiguous memory, neighbouring
// segments (whose shared boundary lines mode 3 keeps in L2) sit on one XCD,
// and the 8 runs still form one front of 8c blocks.  Blocks past the last
// whole 8c window keep their order (a bijection for any grid).  Measured,
// interleaved in one process on 5 boxes (profiles/r1_ab_xcd.jsonl):
//   NS 1 M x 1500 B     213.3 -> 208.5 us   (FETCH 1.5855 -> 1.5771 GB)
//   1 M x 9000 B       1307.0 -> 1255.5 us
//   8 M x 9000 B      10524.9 -> 10087.9 us
// (c = grid / 8, i.e. eight contiguous eighths, lost 1.8 % on the 75 GB batch).
// c is a power of two (run_log2 caps it), so the mapping is shifts and masks:
// short-lived blocks (small segments) pay a few scalar instructions, not an
// emulated integer division per block.
__device__ __forceinline__ uint32_t block_order(uint32_t run_log2) {
  const uint32_t nblk = gridDim.x, b = blockIdx.x;
  if (run_log2 == 0 || nblk < 16) return b;
  const uint32_t fl = 31u - uint32_t(__builtin_clz(nblk >> 3));  // floor(log2(nblk / 8))
  const uint32_t lc = fl < run_log2 ? fl : run_log2;              // c = 2^lc
  const uint32_t full = (nblk >> (lc + 3)) << (lc + 3);           // whole 8c windows
  if (b >= full) return b;
  const uint32_t k = b >> 3, x = b & 7u;
  return ((k >> lc) << (lc + 3)) + (x << lc) + (k & ((1u << lc) - 1u));
}

// End of a launch that completes a zero-copy host call (Done): every wave
// first waits for its own outstanding memory operations (s_waitcnt 0: on
// gfx9 stores count in vmcnt, so its result stores have left the CU — made
// explicit rather than relying on the barrier's workgroup-scope release to
// emit that wait), then the block's barrier orders them before lane 0, whose
// system-scope release (cumulative: one L2 write-back per block, not per
// wave) puts them where the host reads them before it takes a ticket; the
// block with the last ticket resets the ticket word and releases the
// completion value into the host word.  A one-block launch (a tick of up to
// 16 MTU datagrams) skips the ticket and releases the word at once: the
// agent-scope atomic behind the system-scope release cost 1.7-1.9 us of a
// 9-13 us call (profiles/r5_tick_latency_single_block_ab.jsonl).  A no-op
// (one uniform branch) for every device-path launch.  Every thread of the
// block must reach it: kernels call their body first.
__device__ __forceinline__ void signal_done(const Done& d) {
  if (d.flag == nullptr) return;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    if (gridDim.x == 1) {  // the only block (a tick of a few datagrams): no ticket to draw
      __hip_atomic_store(d.flag, d.value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    const uint32_t t = __hip_atomic_fetch_add(d.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(d.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(d.flag, d.value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <int LPS, int UNROLL, int SEGS, int OUT>
__device__ __forceinline__ void checksum_small_body(const uint8_t* __restrict__ bytes, const SegSrc& src,
                                                    const uint32_t* __restrict__ init, uint32_t init_step,
                                                    const uint8_t* __restrict__ odd, uint32_t odd_step,
                                                    const u32x4* __restrict__ zero16, void* __restrict__ out,
                                                    uint64_t n, uint32_t blk, uint32_t nblk);  // below

template <int OUT>
__device__ __forceinline__ void checksum_tiny_body(const uint8_t* __restrict__ bytes, const SegSrc& src,
                                                   const uint32_t* __restrict__ init, uint32_t init_step,
                                                   const uint8_t* __restrict__ odd, uint32_t odd_step,
                                                   const u32x4* __restrict__ zero16, void* __restrict__ out,
                                                   uint64_t n, uint32_t blk, uint32_t nblk);  // below

template <int LPS, int UNROLL, bool NT, int MODE, int OUT>
__device__ __forceinline__ void checksum_entry(const uint8_t* __restrict__ bytes, const SegSrc& src,
                                               const uint32_t* __restrict__ init, uint32_t init_step,
                                               const uint8_t* __restrict__ odd, uint32_t odd_step,
                                               void* __restrict__ out, uint64_t n, uint32_t remap,
                                               const u32x4* __restrict__ zero16) {
  const uint32_t blk = block_order(remap);
  if constexpr (MODE == 3 && NT && UNROLL == 8 && (LPS == 32 || LPS == 64)) {
    // the last bin's launch under kPlanWhole16: every segment of the batch,
    // 16-lane groups in the first n/16 (logical) blocks, the rest exit
    if (src.list && src.bin == kBins - 1 && src.meta[kBinMetaPlan] == kPlanWhole16) {
      constexpr uint32_t kG16 = kBlock / 16;
      const uint64_t need = (n + kG16 - 1) / kG16;
      const uint32_t nblk16 = uint32_t(need < gridDim.x ? need : gridDim.x);
      if (blk >= nblk16) return;
      SegSrc whole = src;
      whole.list = nullptr;  // resolve(): every segment by index
      checksum_body<16, 8, true, 3, OUT>(bytes, whole, init, init_step, odd, odd_step, out, n, blk, nblk16);
      return;
    }
    // ... under kPlanWholeSmall: ACK-sized segments (mean <= kTinyMaxAvg
    // bytes) one per lane in the first n/256 (logical) blocks, otherwise the
    // small-segment body (4 lanes, 2 segments per group in flight) in the
    // first n/128
    if (src.list && src.bin == kBins - 1 && src.meta[kBinMetaPlan] == kPlanWholeSmall &&
        src.meta[kBinMetaAvgLen] <= kTinyMaxAvg) {
      const uint64_t need = (n + kBlock - 1) / kBlock;
      const uint32_t nblks = uint32_t(need < gridDim.x ? need : gridDim.x);
      if (blk >= nblks) return;
      SegSrc whole = src;
      whole.list = nullptr;
      checksum_tiny_body<OUT>(bytes, whole, init, init_step, odd, odd_step, zero16, out, n, blk, nblks);
      return;
    }
    if (src.list && src.bin == kBins - 1 && src.meta[kBinMetaPlan] == kPlanWholeSmall) {
      constexpr uint32_t kPerBlock = (kBlock / 4) * 2;
      const uint64_t need = (n + kPerBlock - 1) / kPerBlock;
      const uint32_t nblks = uint32_t(need < gridDim.x ? need : gridDim.x);
      if (blk >= nblks) return;
      SegSrc whole = src;
      whole.list = nullptr;
      checksum_small_body<4, 2, 2, OUT>(bytes, whole, init, init_step, odd, odd_step, zero16, out, n, blk, nblks);
      return;
    }
  }
  // a bin launch whose bin is empty (the last bin under the split plan) is
  // dispatch-bound — ~0.05 ns per wave whatever the block shape (measured,
  // git 7692616:tools/probe/dispatch_probe.hip) — so its waves leave before anything else
  if (src.list && resolve(src, n).items == 0) return;
  checksum_body<LPS, UNROLL, NT, MODE, OUT>(bytes, src, init, init_step, odd, odd_step, out, n, blk,
                                            gridDim.x);
}

template <int LPS, int UNROLL, bool NT, int MODE, int OUT>
__global__ __launch_bounds__(kBlock) void k_checksum(const uint8_t* __restrict__ bytes, SegSrc src,
                                                     const uint32_t* __restrict__ init,
                                                     uint32_t init_step,
                                                     const uint8_t* __restrict__ odd,
                                                     uint32_t odd_step,
                                                     void* __restrict__ out, uint64_t n, uint32_t remap,
                                                     const u32x4* __restrict__ zero16, Done done) {
  bytes = rebase(bytes, src);
  checksum_entry<LPS, UNROLL, NT, MODE, OUT>(bytes, src, init, init_step, odd, odd_step, out, n, remap, zero16);
  signal_done(done);
}

// Small segments (a few 16-byte chunks): a lane group owns SEGS segments per
// pass and issues the first LPS*UNROLL chunk loads of ALL of them before any
// is consumed, so a wave keeps SEGS times the bytes in flight of the
// one-segment kernel (small segments are latency-bound, not VALU-bound).
// Instruction k of a wave covers 64/LPS consecutive segments, i.e. one
// contiguous 1 KiB run for 64-byte segments.  Every slot is masked to its
// segment (range_sums_masked semantics); a segment longer than LPS*UNROLL
// chunks finishes in a loop.  Absent per-segment arrays: zero16 + step 0.
template <int LPS, int UNROLL, int SEGS, int OUT>
__device__ __forceinline__ void checksum_small_body(const uint8_t* __restrict__ bytes, const SegSrc& src,
                                                    const uint32_t* __restrict__ init, uint32_t init_step,
                                                    const uint8_t* __restrict__ odd, uint32_t odd_step,
                                                    const u32x4* __restrict__ zero16, void* __restrict__ out,
                                                    uint64_t n, uint32_t blk, uint32_t nblk) {
  constexpr uint32_t kGroups = kBlock / LPS;
  constexpr uint32_t kSlots = LPS * UNROLL;
  const uint32_t lane = threadIdx.x & (LPS - 1);
  const uint32_t group = threadIdx.x / LPS;
  const Work w = resolve(src, n);  // never a whole-batch run (the last bin is not small)
  for (uint64_t g0 = uint64_t(blk) * kGroups * SEGS; g0 < w.items; g0 += uint64_t(nblk) * kGroups * SEGS) {
    uint64_t s[SEGS], span[SEGS], segk[SEGS];
    bool validk[SEGS];
    uint32_t nch[SEGS], i0[SEGS], swap[SEGS];
    u32x4 v[SEGS][UNROLL];
#pragma unroll
    for (int k = 0; k < SEGS; ++k) {
      const uint64_t gi = g0 + uint64_t(k) * kGroups + group;
      validk[k] = gi < w.items;
      uint64_t e;
      src_locate(src, w, gi, n, segk[k], s[k], e);
      const uint64_t a0 = s[k] & ~uint64_t(15);
      span[k] = e > s[k] ? e - a0 : 0;
      nch[k] = uint32_t((span[k] + 15) >> 4);
      const uint64_t cseg = segk[k];  // 0 for idle lanes (n >= 1)
      i0[k] = init[cseg * init_step];
      swap[k] = (uint32_t(s[k]) ^ uint32_t(odd[cseg * odd_step])) & 1u;
      const u32x4* p = reinterpret_cast<const u32x4*>(bytes + a0);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const uint32_t cc = lane + uint32_t(u * LPS);
        // unconditional load from a valid address (empty segment -> zero16)
        const u32x4* q = nch[k] ? p + (cc < nch[k] ? cc : nch[k] - 1) : zero16;
        if (nch[k]) ICS_CHECK16(q, bytes + a0, bytes + a0 + (uint64_t(nch[k]) << 4));
        v[k][u] = __builtin_nontemporal_load(q);
      }
    }
#pragma unroll
    for (int k = 0; k < SEGS; ++k) {
      uint32_t ev = 0, od = 0;
      const uint32_t lo0 = uint32_t(s[k]) & 15u;
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const uint32_t cc = lane + uint32_t(u * LPS);
        const uint64_t at = uint64_t(cc) << 4;
        const uint32_t lo = cc == 0 ? lo0 : 0u;
        const uint32_t hi = at >= span[k] ? 0u : (span[k] - at >= 16 ? 16u : uint32_t(span[k] - at));
        acc_chunk(v[k][u] & byte_range_mask(lo, hi), ev, od);
      }
      if (nch[k] > kSlots) {  // long segment: the rest, masked (rare in this kernel's range)
        const u32x4* p = reinterpret_cast<const u32x4*>(bytes + (s[k] & ~uint64_t(15)));
        for (uint32_t cc = lane + kSlots; cc < nch[k]; cc += LPS) {
          const uint64_t at = uint64_t(cc) << 4;
          const uint32_t hi = span[k] - at >= 16 ? 16u : uint32_t(span[k] - at);
          ICS_CHECK16(p + cc, reinterpret_cast<const uint8_t*>(p),
                      reinterpret_cast<const uint8_t*>(p) + (uint64_t(nch[k]) << 4));
          acc_chunk(__builtin_nontemporal_load(p + cc) & byte_range_mask(0u, hi), ev, od);
        }
      }
      const uint32_t tot = group_sum<LPS>(combine_roles(ev, od, swap[k]));
      const uint64_t seg = segk[k];
      if (validk[k] && lane == LPS - 1) {
        const uint32_t sum = i0[k] + tot;
        if (OUT == 0)
          static_cast<uint16_t*>(out)[seg] = fold_value(sum);
        else
          static_cast<uint32_t*>(out)[seg] = sum;
      }
    }
  }
}

template <int LPS, int UNROLL, int SEGS, int OUT>
__global__ __launch_bounds__(kBlock) void k_checksum_small(const uint8_t* __restrict__ bytes, SegSrc src,
                                                           const uint32_t* __restrict__ init,
                                                           uint32_t init_step,
                                                           const uint8_t* __restrict__ odd,
                                                           uint32_t odd_step,
                                                           const u32x4* __restrict__ zero16,
                                                           void* __restrict__ out, uint64_t n, Done done) {
  bytes = rebase(bytes, src);
  checksum_small_body<LPS, UNROLL, SEGS, OUT>(bytes, src, init, init_step, odd, odd_step, zero16, out, n,
                                              blockIdx.x, gridDim.x);
  signal_done(done);
}

// Tiny segments (ACK-sized TCP segments, <= 4 chunks): ONE lane per segment.
// The wave's offsets load is one coalesced 512-byte read, each lane then
// issues its segment's (up to) four 16-byte loads at once — neighbouring
// lanes' segments share lines, so the loads keep the default cache policy
// and a line a neighbour also reads comes from L2 — and masks them to the
// segment.  A longer segment finishes its remaining chunks in a loop (rare
// in this kernel's range: the plans send it batches of short segments).
// Absent per-segment arrays: zero16 + step 0.
template <int OUT>
__device__ __forceinline__ void checksum_tiny_body(const uint8_t* __restrict__ bytes, const SegSrc& src,
                                                   const uint32_t* __restrict__ init, uint32_t init_step,
                                                   const uint8_t* __restrict__ odd, uint32_t odd_step,
                                                   const u32x4* __restrict__ zero16, void* __restrict__ out,
                                                   uint64_t n, uint32_t blk, uint32_t nblk) {
  constexpr int kSlots = 4;
  const Work w = resolve(src, n);
  for (uint64_t g0 = uint64_t(blk) * kBlock; g0 < w.items; g0 += uint64_t(nblk) * kBlock) {
    const uint64_t gi = g0 + threadIdx.x;
    uint64_t seg, s, e;
    src_locate(src, w, gi, n, seg, s, e);
    const uint64_t a0 = s & ~uint64_t(15);
    const uint64_t span = e > s ? e - a0 : 0;
    const uint32_t nch = uint32_t((span + 15) >> 4);
    const u32x4* __restrict__ p = reinterpret_cast<const u32x4*>(bytes + a0);
    u32x4 v[kSlots];
#pragma unroll
    for (int u = 0; u < kSlots; ++u) {
      // unconditional load from a valid address (empty segment -> zero16)
      const u32x4* q = nch ? p + (uint32_t(u) < nch ? uint32_t(u) : nch - 1) : zero16;
      if (nch) ICS_CHECK16(q, bytes + a0, bytes + a0 + (uint64_t(nch) << 4));
      v[u] = *q;
    }
    const uint32_t i0 = init[seg * init_step];
    const uint32_t swap = (uint32_t(s) ^ uint32_t(odd[seg * odd_step])) & 1u;
    uint32_t ev = 0, od = 0;
#pragma unroll
    for (int u = 0; u < kSlots; ++u) {
      const uint64_t at = uint64_t(u) << 4;
      const uint32_t lo = u == 0 ? uint32_t(s) & 15u : 0u;
      const uint32_t hi = at >= span ? 0u : (span - at >= 16 ? 16u : uint32_t(span - at));
      acc_chunk(v[u] & byte_range_mask(lo, hi), ev, od);
    }
    for (uint32_t c = kSlots; c < nch; ++c) {  // longer segments
      const uint64_t at = uint64_t(c) << 4;
      const uint32_t hi = span - at >= 16 ? 16u : uint32_t(span - at);
      ICS_CHECK16(p + c, bytes + a0, bytes + a0 + (uint64_t(nch) << 4));
      acc_chunk(p[c] & byte_range_mask(0u, hi), ev, od);
    }
    if (gi < w.items) {
      const uint32_t sum = i0 + combine_roles(ev, od, swap);
      if (OUT == 0)
        static_cast<uint16_t*>(out)[seg] = fold_value(sum);
      else
        static_cast<uint32_t*>(out)[seg] = sum;
    }
  }
}

template <int OUT>
__global__ __launch_bounds__(kBlock) void k_checksum_tiny(const uint8_t* __restrict__ bytes, SegSrc src,
                                                          const uint32_t* __restrict__ init, uint32_t init_step,
                                                          const uint8_t* __restrict__ odd, uint32_t odd_step,
                                                          const u32x4* __restrict__ zero16, void* __restrict__ out,
                                                          uint64_t n, Done done) {
  bytes = rebase(bytes, src);
  checksum_tiny_body<OUT>(bytes, src, init, init_step, odd, odd_step, zero16, out, n, blockIdx.x, gridDim.x);
  signal_done(done);
}

// Two-class launch for receive mixes (ACKs among MTU segments), no binning
// pass: block b takes segments [4 SPW b, 4 SPW b + 4 SPW); wave w reads the
// bounds of SPW of them and appends each to the block's short (<= 4 chunks)
// or long list in LDS.  Wave 0 then finishes the short ones one per lane (64
// per pass, as k_checksum_tiny does), while every wave — wave 0 once its
// short passes are done — claims the long ones 64 / LONG_LPS at a time from
// an LDS counter (LONG_LPS lanes each, the line grid, unroll 8).  The fused
// IPv4 launch's block lists (k_ipv4_twoclass); 2 M x 40 / 1460 B 230.8 ->
// 224.8 us against the per-wave version (git 7692616:tools/probe/csum_mix_probe.hip).
template <int LONG_LPS, int SPW, int OUT>
__global__ __launch_bounds__(kBlock) void k_checksum_twoclass(const uint8_t* __restrict__ bytes, SegSrc src,
                                                              const uint32_t* __restrict__ init, uint32_t init_step,
                                                              const uint8_t* __restrict__ odd, uint32_t odd_step,
                                                              const u32x4* __restrict__ zero16,
                                                              void* __restrict__ out, uint64_t n, uint32_t remap) {
  constexpr uint32_t kPer = (kBlock / 64) * SPW;
  __shared__ uint64_t lst[kPer][2], sst[kPer][2];  // the block's long / short segments' {start, end}
  __shared__ uint32_t lseg[kPer], sseg[kPer];
  __shared__ uint32_t cnt[3];  // long, short, long claimed
  __shared__ uint32_t o_sum[kPer];  // the block's sums, written out as one coalesced row at the end
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  bytes = rebase(bytes, src);
  if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
  __syncthreads();
  const Work w{n, nullptr};
  const uint64_t bb = uint64_t(block_order(remap)) * kPer;  // the block's segments [bb, bb + kPer) (no list)
  const uint64_t gi = bb + wv * SPW + (lane < SPW ? lane : 0u);
  uint64_t seg, s, e;
  src_locate(src, w, gi, n, seg, s, e);
  const bool valid = gi < n && lane < SPW;
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
  auto store = [&](uint64_t sg, uint32_t sum) { o_sum[sg - bb] = sum; };
  if (wv == 0)
    for (uint32_t r0 = 0; r0 < nshort; r0 += 64) {  // uniform
      const uint32_t k = r0 + lane;
      const bool mine = k < nshort;
      const uint32_t kc = mine ? k : 0u;
      const uint64_t ss = sst[kc][0], se = mine ? sst[kc][1] : ss;
      const uint64_t sg = sseg[kc];
      const uint64_t b0 = ss & ~uint64_t(15), span = se > ss ? se - b0 : 0;
      const uint32_t nc = uint32_t((span + 15) >> 4);
      const u32x4* __restrict__ p = reinterpret_cast<const u32x4*>(bytes + b0);
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // an empty slot loads the zero block
        const u32x4* q = nc ? p + (uint32_t(u) < nc ? uint32_t(u) : nc - 1) : zero16;
        if (nc) ICS_CHECK16(q, bytes + b0, bytes + b0 + (uint64_t(nc) << 4));
        v[u] = *q;
      }
      const uint32_t i0 = init[sg * init_step];
      const uint32_t sw = (uint32_t(ss) ^ uint32_t(odd[sg * odd_step])) & 1u;
      uint32_t ev = 0, od = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t at = uint64_t(u) << 4;
        const uint32_t lo = u == 0 ? uint32_t(ss) & 15u : 0u;
        const uint32_t hi = at >= span ? 0u : (span - at >= 16 ? 16u : uint32_t(span - at));
        acc_chunk(v[u] & byte_range_mask(lo, hi), ev, od);
      }
      if (mine) store(sg, i0 + combine_roles(ev, od, sw));
    }
  constexpr uint32_t kGroups = 64 / LONG_LPS;
  const uint32_t g = lane / LONG_LPS, gl = lane & (LONG_LPS - 1);
  for (;;) {
    uint32_t r0 = 0;
    if (lane == 0) r0 = atomicAdd(&cnt[2], kGroups);
    r0 = __builtin_amdgcn_readfirstlane(r0);
    if (r0 >= nlong) break;  // uniform
    const uint32_t k = r0 + g;
    const bool mine = k < nlong;
    const uint32_t kc = mine ? k : 0u;
    const uint64_t ls = mine ? lst[kc][0] : 0, le = mine ? lst[kc][1] : 0;
    const uint64_t lsg = lseg[kc];
    const uint32_t i0 = init[lsg * init_step];
    const uint32_t sw = (uint32_t(ls) ^ uint32_t(odd[lsg * odd_step])) & 1u;
    uint32_t ev = 0, od = 0;
    // 7 loads per lane: an MSS segment's line-grid span (<= 100 chunks) in one
    // pass of 112 chunks, fewer clamped slot loads than 8 (2 M bimodal
    // 226.6 -> 221.1 us, profiles/r4_ab_csum_twoclass_unroll7.jsonl)
    range_sums_line_primed<LONG_LPS, 7, true>(bytes, ls, le, gl, ev, od);
    const uint32_t tot = group_sum<LONG_LPS>(combine_roles(ev, od, sw));
    if (mine && gl == LONG_LPS - 1) store(lsg, i0 + tot);
  }
  __syncthreads();
  const uint64_t i = bb + threadIdx.x;  // every segment of the block was summed: its row is complete
  if (threadIdx.x < kPer && i < n) {
    if (OUT == 0)
      static_cast<uint16_t*>(out)[i] = fold_value(o_sum[threadIdx.x]);
    else
      static_cast<uint32_t*>(out)[i] = o_sum[threadIdx.x];
  }
}

// Dense fixed-stride batches of short segments (stride == seg_len == 16*LPS,
// 16-byte aligned base — config 3's 1 M x 64 B TCP segments): the batch is one
// flat array of 16-byte chunks, every chunk belongs whole to one segment, so
// a wave instruction reads 1 KiB contiguous and no slot needs a mask, an
// address clamp or a boundary case.  Lane group g of wave w owns segments
// (w*SEGS + k)*kSegsPerWave + g, k < SEGS: all SEGS loads (plus the init
// words) are issued before the first is consumed.  Every start is even (the
// base is aligned, the stride a multiple of 16), so byte roles never swap.
// Measured floor for 64 MiB + 4 MiB inits + 2 MiB outputs on MI355X:
// ≈12.4 us (git 7692616:tools/probe/small_probe.hip).
// (block blk of the launch; init_step 0 reads one shared zero word)
template <int LPS, int SEGS, bool INIT, int OUT>
__device__ __forceinline__ void checksum_dense_body(const u32x4* __restrict__ chunks, const uint32_t* __restrict__ init,
                                                    uint32_t init_step, void* __restrict__ out, uint64_t n,
                                                    uint32_t blk) {
  constexpr uint32_t kSegsPerWave = 64 / LPS;
  const uint32_t lane64 = threadIdx.x & 63u, lane = threadIdx.x & (LPS - 1), group = lane64 / LPS;
  const uint64_t wave = (uint64_t(blk) * kBlock + threadIdx.x) >> 6;
  const uint64_t seg0 = wave * SEGS * kSegsPerWave + group;
  const uint64_t nch = n * LPS;
  u32x4 v[SEGS];
  uint32_t i0[SEGS];
#pragma unroll
  for (int k = 0; k < SEGS; ++k) {
    const uint64_t seg = seg0 + uint64_t(k) * kSegsPerWave;
    const uint64_t c = seg * LPS + lane;
    ICS_CHECK16(chunks + (c < nch ? c : nch - 1), reinterpret_cast<const uint8_t*>(chunks),
                reinterpret_cast<const uint8_t*>(chunks + nch));
    v[k] = __builtin_nontemporal_load(chunks + (c < nch ? c : nch - 1));
    i0[k] = INIT ? init[(seg < n ? seg : n - 1) * init_step] : 0u;
  }
#pragma unroll
  for (int k = 0; k < SEGS; ++k) {
    uint32_t ev = 0, od = 0;
    acc_chunk(v[k], ev, od);
    const uint32_t tot = group_sum<LPS>(ev * 256u + od);
    const uint64_t seg = seg0 + uint64_t(k) * kSegsPerWave;
    if (seg < n && lane == LPS - 1) {
      const uint32_t sum = i0[k] + tot;
      if (OUT == 0)
        static_cast<uint16_t*>(out)[seg] = fold_value(sum);
      else
        static_cast<uint32_t*>(out)[seg] = sum;
    }
  }
}

template <int LPS, int SEGS, bool INIT, int OUT>
__global__ __launch_bounds__(kBlock) void k_checksum_dense(const u32x4* __restrict__ chunks,
                                                           const uint32_t* __restrict__ init,
                                                           void* __restrict__ out, uint64_t n) {
  checksum_dense_body<LPS, SEGS, INIT, OUT>(chunks, init, 1u, out, n, blockIdx.x);
}

// Bins 0..kBins-2 of a binned batch in ONE launch: nblk blocks per bin, each
// bin with its own geometry (kBinGeometry; blocks of bin b = [b*nblk,
// (b+1)*nblk)).  One launch instead of four: no drain between bins, and one
// launch to skip under the whole-batch plan.
template <int OUT>
__global__ __launch_bounds__(kBlock) void k_checksum_bins(const uint8_t* __restrict__ bytes, SegSrc src,
                                                          const uint32_t* __restrict__ init, uint32_t init_step,
                                                          const uint8_t* __restrict__ odd, uint32_t odd_step,
                                                          const u32x4* __restrict__ zero16,
                                                          void* __restrict__ out, uint64_t n, uint32_t nblk) {
  const uint32_t b = blockIdx.x / nblk, blk = blockIdx.x - b * nblk;
  bytes = rebase(bytes, src);
  SegSrc bs = src;
  bs.list = src.list + uint64_t(b) * n;
  bs.bin = int(b);
  switch (b) {
    case 0:
      checksum_small_body<4, 2, 2, OUT>(bytes, bs, init, init_step, odd, odd_step, zero16, out, n, blk, nblk);
      break;
    case 1:
      checksum_body<16, 4, true, 3, OUT>(bytes, bs, init, init_step, odd, odd_step, out, n, blk, nblk);
      break;
    case 2:
      checksum_body<16, 8, true, 3, OUT>(bytes, bs, init, init_step, odd, odd_step, out, n, blk, nblk);
      break;
    default:
      checksum_body<32, 4, true, 3, OUT>(bytes, bs, init, init_step, odd, odd_step, out, n, blk, nblk);
      break;
  }
}

// HSA dispatch packets carry the grid size in work-items as a uint32, so
// element-wise kernels use a capped grid and stride over the rest.
#define ICS_GRID_STRIDE(i, n) \
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < (n); i += uint64_t(gridDim.x) * blockDim.x)

__global__ void k_fold(const uint32_t* __restrict__ sum, uint16_t* __restrict__ out, uint64_t n) {
  ICS_GRID_STRIDE(i, n) out[i] = fold_value(sum[i]);
}

// ---------------------------------------------- IPv4 header fields ------
// The first 20 wire bytes of a datagram as 5 little-endian dwords relative to
// its (possibly unaligned) start: 6 aligned dword loads + alignbyte.
struct Hdr {
  uint32_t w[5];
  __device__ __forceinline__ uint32_t byte(int k) const { return (w[k >> 2] >> (8 * (k & 3))) & 0xffu; }
  __device__ __forceinline__ uint32_t be16(int k) const { return (byte(k) << 8) | byte(k + 1); }
};

// The aligned dword holding the byte before `end`: the last dword a load for
// a range ending at `end` (exclusive) may touch.
__device__ __forceinline__ const uint32_t* last_dword(const uint8_t* end) {
  const uint8_t* b = end - 1;
  return reinterpret_cast<const uint32_t*>(b - (reinterpret_cast<uintptr_t>(b) & 3u));
}

// Header of the datagram at p (>= 20 bytes; `last` = last_dword of its end).
// Address arithmetic stays on the global pointer p (an integer-to-pointer
// cast would turn these into flat loads, which count in both vmcnt and
// lgkmcnt and are waited for before the byte stream is issued), and every
// load is unconditional: the sixth dword, which reaches up to 3 bytes past
// byte 19 when the start is aligned, is clamped to `last`, so nothing past
// the datagram's final dword is read.
__device__ __forceinline__ Hdr load_hdr(const uint8_t* p, const uint32_t* last) {
  const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
  uint32_t d[6];
#ifdef ICSUM_BOUNDS_CHECK
  if (q + 4 > last) bounds_fail(kBoundsHeader, reinterpret_cast<unsigned long long>(q + 4));
#endif
#pragma unroll
  for (int k = 0; k < 5; ++k) d[k] = q[k];
  d[5] = *(q + 5 < last ? q + 5 : last);
  Hdr h;
#pragma unroll
  for (int k = 0; k < 5; ++k) h.w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
  return h;
}

// big-endian 16-bit field store: one short store when 2-byte aligned.  The
// default write-back policy: write-through (sc1), non-temporal and wider
// (16-byte, 64-byte, whole-line) stores of the same fields all measured the
// same or slower (PATCH).
__device__ __forceinline__ void store_be16(uint8_t* p, uint32_t v) {
  if ((reinterpret_cast<uintptr_t>(p) & 1u) == 0) {
    *reinterpret_cast<uint16_t*>(p) = uint16_t(((v & 0xffu) << 8) | ((v >> 8) & 0xffu));
  } else {
    p[0] = uint8_t(v >> 8);
    p[1] = uint8_t(v);
  }
}

// TCP header bytes 12..19 of a segment starting at t (>= 18 bytes present;
// `last` = last_dword of its end): tf0 = bytes 12..15, tf1 = bytes 16..19
// (bytes 18, 19 only meaningful when present).  Unconditional global loads;
// the third dword (needed only when byte 12 sits at offset 3 of its dword) is
// clamped to `last`.
__device__ __forceinline__ void load_tcp_fields(const uint8_t* t, const uint32_t* last, uint32_t& tf0,
                                                uint32_t& tf1) {
  const uint8_t* p = t + 12;
  const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
#ifdef ICSUM_BOUNDS_CHECK
  if (q + 1 > last) bounds_fail(kBoundsHeader, reinterpret_cast<unsigned long long>(q + 1));
#endif
  const uint32_t d0 = q[0], d1 = q[1];
  const uint32_t d2 = *(q + 2 < last ? q + 2 : last);
  tf0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  tf1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
}

// The same dwords unaligned (the stashed form, VRec): the six aligned dwords
// holding header bytes 0..19 at p and the three holding TCP bytes 12..19 at
// t, with their byte shifts.
__device__ __forceinline__ void load_hdr_raw(const uint8_t* p, const uint32_t* last, uint32_t* d, uint32_t& sh) {
  sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
#ifdef ICSUM_BOUNDS_CHECK
  if (q + 4 > last) bounds_fail(kBoundsHeader, reinterpret_cast<unsigned long long>(q + 4));
#endif
#pragma unroll
  for (int k = 0; k < 5; ++k) d[k] = q[k];
  d[5] = *(q + 5 < last ? q + 5 : last);
}

__device__ __forceinline__ uint32_t tcp_shift(const uint8_t* t) {
  return uint32_t(reinterpret_cast<uintptr_t>(t + 12) & 3u);
}

// dword k (0..2) of the TCP-field window of the segment at t (the third
// clamped to `last`)
__device__ __forceinline__ uint32_t load_tcp_raw(const uint8_t* t, const uint32_t* last, uint32_t k) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(t + 12 - tcp_shift(t));
#ifdef ICSUM_BOUNDS_CHECK
  if (q + 1 > last) bounds_fail(kBoundsHeader, reinterpret_cast<unsigned long long>(q + 1));
#endif
  return *(q + k < last ? q + k : last);
}

// The header dwords and the TCP fields with ONE load instruction for a lane
// group of >= 16 lanes: lane k (< 9) of the group loads header dword k (k <
// 6: the aligned window at p, the sixth clamped to `last`) or TCP-field dword
// k - 6 (the window at t + 12, the third clamped to `tlast`), the other lanes
// repeat lane 0's address.  group_hdr_take, called after the byte stream has
// been summed (loads return in order, so waiting for the stream covers this
// load too), hands every lane the nine dwords from the group's lanes —
// row_newbcast DPP for 16-lane groups (one DPP row), readlane for 64,
// ds_bpermute for 32 — and aligns them: the values of load_hdr +
// load_tcp_fields, which take 9 load instructions per lane.
struct GroupHdr {
  uint32_t v, sh, tsh;
};

template <int LPS>
__device__ __forceinline__ GroupHdr group_hdr_load(const uint8_t* p, const uint32_t* last, const uint8_t* t,
                                                   const uint32_t* tlast) {
  static_assert(LPS >= 16, "nine dwords need nine lanes of the group");
  const uint32_t k = threadIdx.x & (LPS - 1);
  GroupHdr g;
  g.sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p - g.sh);
  const uint8_t* tp = t + 12;
  g.tsh = uint32_t(reinterpret_cast<uintptr_t>(tp) & 3u);
  const uint32_t* tq = reinterpret_cast<const uint32_t*>(tp - g.tsh);
#ifdef ICSUM_BOUNDS_CHECK
  if (k == 0 && q + 4 > last) bounds_fail(kBoundsHeader, reinterpret_cast<unsigned long long>(q + 4));
  if (k == 0 && tq + 1 > tlast) bounds_fail(kBoundsHeader, reinterpret_cast<unsigned long long>(tq + 1));
#endif
  const uint32_t* a = q;
  if (k < 5) a = q + k;
  else if (k == 5) a = q + 5 < last ? q + 5 : last;
  else if (k < 8) a = tq + (k - 6);
  else if (k == 8) a = tq + 2 < tlast ? tq + 2 : tlast;
  g.v = *a;
  return g;
}

template <int LPS>
__device__ __forceinline__ void group_hdr_take(const GroupHdr& g, Hdr& h, uint32_t& tf0, uint32_t& tf1) {
  uint32_t d[9];
  if constexpr (LPS == 16) {
#define ICS_NEWBCAST(j) d[j] = __builtin_amdgcn_update_dpp(0u, g.v, 0x150 + (j), 0xF, 0xF, false);  // row_newbcast:j
    ICS_NEWBCAST(0) ICS_NEWBCAST(1) ICS_NEWBCAST(2) ICS_NEWBCAST(3) ICS_NEWBCAST(4)
    ICS_NEWBCAST(5) ICS_NEWBCAST(6) ICS_NEWBCAST(7) ICS_NEWBCAST(8)
#undef ICS_NEWBCAST
  } else {
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      if (LPS == 64)
        d[j] = __builtin_amdgcn_readlane(g.v, j);
      else
        d[j] = uint32_t(__shfl(int(g.v), int((threadIdx.x & 63u & ~(LPS - 1u)) + j), 64));
    }
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) h.w[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], g.sh);
  tf0 = __builtin_amdgcn_alignbyte(d[7], d[6], g.tsh);
  tf1 = __builtin_amdgcn_alignbyte(d[8], d[7], g.tsh);
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

// The per-datagram results of the fused kernels from its header fields, the
// TCP bytes 12..19 (tf0 / tf1, read at t0 + 12), tot = the sum of the TCP
// part [t0, e) with roles relative to t0 and its length rem = e - t0 (b16:
// the TCP part's byte 16 when rem == 17, the checksum field's only byte
// there; COMPUTE / PATCH only): IPv4Header::compute_checksum and the parse
// checks (ipv4_header.cpp:9-59, 113-123), pseudo_checksum (:103-110),
// TCPSegment::parse's verify (tcp_segment.cpp:11-18) or compute_checksum with
// the checksum field counted as 0 (:109-118), and the status bits of
// include/icsum.h.  hdr false (a datagram under 20 bytes): zeros.
struct Verdict {
  uint32_t ipc, tcv, st;
};
__device__ __forceinline__ Verdict ipv4_verdict(bool hdr, const Hdr& h, uint32_t tf0, uint32_t tf1, uint32_t tot,
                                                uint64_t rem, uint32_t b16, int mode) {
  Verdict v{0, 0, 0};
  if (hdr) {
    const uint32_t ver = h.byte(0) >> 4, hlen = h.byte(0) & 0x0fu;
    const bool hdr_ok = ver == 4 && hlen >= 5;  // ipv4_header.cpp:32-41
    v.ipc = fold_value(ipv4_header_sum(h));
    const uint32_t pseudo = ipv4_pseudo(h);
    if (h.byte(9) == 6) v.st |= 0x08;  // proto TCP
    if (rem >= 20 && ((tf0 & 0xffu) >> 4) >= 5) v.st |= 0x04;  // tcp_segment.cpp:25-65
    if (mode == 1) {
      v.tcv = fold_value(pseudo + tot);  // tcp_segment.cpp:11-18
      if (hdr_ok && v.ipc == h.be16(10)) v.st |= 0x01;  // ipv4_header.cpp:53-58
      if (v.tcv == 0) v.st |= 0x02;
    } else {
      // tcp_segment.cpp:143: the checksum field counts as 0
      uint32_t sum = pseudo + tot;
      if (rem > 16) sum -= (rem >= 18 ? tf1 & 0xffu : b16) << 8;
      if (rem > 17) sum -= (tf1 >> 8) & 0xffu;
      v.tcv = fold_value(sum);
      if (hdr_ok) v.st |= 0x01;
      if (rem >= 18) v.st |= 0x02;
    }
  }
  return v;
}

// ipv4_verdict in the claim, PATCH's two big-endian stores and the outputs
__device__ __forceinline__ void ipv4_result(uint8_t* __restrict__ dg, uint64_t s, uint64_t e, uint64_t t0, bool hdr,
                                            const Hdr& h, uint32_t tf0, uint32_t tf1, uint32_t tot, int mode,
                                            uint64_t seg, uint16_t* __restrict__ ip_ck, uint16_t* __restrict__ tcp_ck,
                                            uint8_t* __restrict__ status) {
  const uint64_t rem = e - t0;
  const uint32_t b16 = (hdr && mode != 1 && rem == 17) ? uint32_t(dg[t0 + 16]) : 0u;
  const Verdict v = ipv4_verdict(hdr, h, tf0, tf1, tot, rem, b16, mode);
  if (hdr && mode == 2) {
    store_be16(dg + s + 10, v.ipc);
    if (rem >= 18) store_be16(dg + t0 + 16, v.tcv);
  }
  if (ip_ck) ip_ck[seg] = uint16_t(v.ipc);
  if (tcp_ck) tcp_ck[seg] = uint16_t(v.tcv);
  if (status) status[seg] = uint8_t(v.st);
}

#ifdef ICSUM_STAMPS
// diagnostic build only (tools/probe/verify_stamps.hip): per block of
// k_ipv4_twoclass, s_memrealtime (100 MHz) at its start and end, and HW_ID
__device__ uint64_t g_block_stamps[1u << 16][3];
#endif

// What ipv4_result needs, kept per datagram by k_ipv4_twoclass COMPUTE /
// VERIFY, which computes the block's verdicts at its end one datagram per
// lane instead of in one lane of each group per claim: the nine dwords as
// loaded (d[0..5]: the header window, shift sh; d[6..8]: the TCP-field window,
// shift tsh; lane k < 9 of a 16-lane group writes d[k] — no broadcast, no
// alignment in the claim), the TCP part's sum and the rest packed in meta:
// hdr | sh << 2 | tsh << 4 | b16 << 8 | min(rem, 0xffff) << 16 (rem = e - t0;
// the verdict only compares it with 16..20).  44 bytes: an odd dword stride,
// conflict-free rows at the end.
struct VRec {
  uint32_t d[9], tot, meta;
};

__device__ __forceinline__ uint32_t vrec_meta(bool hdr, uint32_t sh, uint32_t tsh, uint32_t b16, uint64_t rem) {
  return uint32_t(hdr) | (sh << 2) | (tsh << 4) | (b16 << 8) | (uint32_t(rem < 0xffffu ? rem : 0xffffu) << 16);
}

__device__ __forceinline__ Verdict vrec_verdict(const VRec& r, int mode) {
  const uint32_t sh = (r.meta >> 2) & 3u, tsh = (r.meta >> 4) & 3u;
  Hdr h;
#pragma unroll
  for (int j = 0; j < 5; ++j) h.w[j] = __builtin_amdgcn_alignbyte(r.d[j + 1], r.d[j], sh);
  const uint32_t tf0 = __builtin_amdgcn_alignbyte(r.d[7], r.d[6], tsh);
  const uint32_t tf1 = __builtin_amdgcn_alignbyte(r.d[8], r.d[7], tsh);
  return ipv4_verdict((r.meta & 1u) != 0, h, tf0, tf1, r.tot, r.meta >> 16, (r.meta >> 8) & 0xffu, mode);
}

// --------------------------------------------- fused IPv4 + TCP ----------
// One datagram [s, e) per group of LPS lanes (every lane of the wave calls it:
// group sums and the wave-uniform re-sum below); `valid` false: an idle group.
// STASH: the datagram's VRec goes to stash[seg] instead of its results to
// the output rows (COMPUTE / VERIFY only).
template <int LPS, int UNROLL, bool NT, int MODE, bool STASH = false>
__device__ __forceinline__ void ipv4_item(uint8_t* __restrict__ dg, uint64_t s, uint64_t e, uint64_t seg, bool valid,
                                          uint32_t lane, int mode, uint16_t* __restrict__ ip_ck,
                                          uint16_t* __restrict__ tcp_ck, uint8_t* __restrict__ status,
                                          const uint8_t* __restrict__ zpad, const uint32_t* zlast,
                                          VRec* stash = nullptr) {
  const bool hdr = e - s >= 20;
  // Speculate the usual header length (hlen = 5): the IPv4 header dwords,
  // the TCP fields the verdict needs (data offset, checksum) and the TCP
  // byte stream are all requested before any of them returns; every lane
  // loads the header (same addresses per group, one request per wave
  // instruction), from the 32-byte zero pad when the datagram is too short.
  // A datagram with options (rare) redoes its stream below.
  uint64_t t0 = hdr ? s + 20 : e;  // TCP part: [t0, e)
  const uint32_t* last = hdr ? last_dword(dg + e) : zlast;
  Hdr h;
  uint32_t tf0 = 0, tf1 = 0;  // TCP bytes 12..15 and 16..19 (little-endian)
  const bool tcpf = hdr && e - t0 >= 18;
  GroupHdr gh{};
  [[maybe_unused]] uint32_t raw[9], sh = 0;  // STASH, one lane per datagram
  if constexpr (LPS >= 16) {
    gh = group_hdr_load<LPS>(hdr ? dg + s : zpad, last, tcpf ? dg + t0 : zpad, tcpf ? last : zlast);
  } else if constexpr (STASH) {
    load_hdr_raw(hdr ? dg + s : zpad, last, raw, sh);
    gh.tsh = tcp_shift(tcpf ? dg + t0 : zpad);
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) raw[6 + k] = load_tcp_raw(tcpf ? dg + t0 : zpad, tcpf ? last : zlast, k);
  } else {
    h = load_hdr(hdr ? dg + s : zpad, last);
    load_tcp_fields(tcpf ? dg + t0 : zpad, tcpf ? last : zlast, tf0, tf1);
  }
  uint32_t ev = 0, od = 0;
  seg_sums<LPS, UNROLL, NT, MODE>(dg, t0, e, lane, ev, od);
  uint32_t b0;  // header byte 0 (version, hlen)
  if constexpr (STASH) {
    if constexpr (LPS >= 16) {
      sh = gh.sh;
      b0 = (__builtin_amdgcn_update_dpp(0u, gh.v, 0x150, 0xF, 0xF, false) >> (8 * sh)) & 0xffu;  // row_newbcast:0
    } else {
      b0 = (raw[0] >> (8 * sh)) & 0xffu;
    }
  } else {
    if constexpr (LPS >= 16) group_hdr_take<LPS>(gh, h, tf0, tf1);
    b0 = h.byte(0);
  }
  bool redo = false;
  if (hdr) {
    uint64_t off = 4u * (b0 & 0x0fu);  // options skipped (ipv4_header.cpp:50)
    if (off < 20) off = 20;
    if (off > e - s) off = e - s;
    redo = s + off != t0;
    t0 = s + off;
    if (redo) {
      const bool f = e - t0 >= 18;
      if constexpr (STASH) {
        gh.tsh = tcp_shift(dg + t0);
        if constexpr (LPS >= 16) {
          if (lane >= 6 && lane < 9) gh.v = f ? load_tcp_raw(dg + t0, last, lane - 6) : 0u;
        } else {
#pragma unroll
          for (uint32_t k = 0; k < 3; ++k) raw[6 + k] = f ? load_tcp_raw(dg + t0, last, k) : 0u;
        }
      } else {
        tf0 = tf1 = 0;
        if (f) load_tcp_fields(dg + t0, last, tf0, tf1);
      }
    }
  }
  if (__any(redo)) {  // wave-uniform
    // The stream summed [s + 20, e); the TCP part starts at t0 = s + 4 hlen
    // (or is empty when the header claims more than the datagram holds).
    // Byte roles are by absolute address and 4 hlen - 20 is even, so the
    // options' own even / odd sums (at most 40 bytes, a few masked chunks
    // per group) come off exactly — no second pass over the payload.
    uint32_t oe = 0, oo = 0;
    if (redo) range_sums_masked<LPS, 1, false>(dg, s + 20, t0, lane, oe, oo);
    ev -= oe;
    od -= oo;
  }
  const uint32_t tot = group_sum<LPS>(combine_roles(ev, od, uint32_t(t0) & 1u));
  if constexpr (STASH) {  // the verdict later, from stash[seg]
    if (valid) {
      VRec& r = stash[seg];
      if constexpr (LPS >= 16) {
        if (lane < 9) r.d[lane] = gh.v;
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) r.d[k] = raw[k];
      }
      if (lane == LPS - 1) {
        const uint64_t rem = e - t0;
        const uint32_t b16 = (hdr && mode != 1 && rem == 17) ? uint32_t(dg[t0 + 16]) : 0u;
        r.tot = tot;
        r.meta = vrec_meta(hdr, sh, gh.tsh, b16, rem);
      }
    }
  } else if (valid && lane == LPS - 1) {
    ipv4_result(dg, s, e, t0, hdr, h, tf0, tf1, tot, mode, seg, ip_ck, tcp_ck, status);
  }
}

// datagrams [blk * groups, ...) striding by nblk blocks (block blk of nblk:
// a kernel of its own, or one batch's share of a multi-batch launch)
template <int LPS, int UNROLL, bool NT, int MODE>
__device__ __forceinline__ void ipv4_body(uint8_t* __restrict__ dg, const uint64_t* __restrict__ offsets,
                                          uint64_t stride, uint64_t dlen, uint64_t n, int mode,
                                          uint16_t* __restrict__ ip_ck, uint16_t* __restrict__ tcp_ck,
                                          uint8_t* __restrict__ status, const uint8_t* __restrict__ zpad,
                                          uint32_t blk, uint32_t nblk) {
  constexpr uint32_t kGroups = kBlock / LPS;
  const uint32_t lane = threadIdx.x & (LPS - 1);
  const uint64_t step = uint64_t(nblk) * kGroups;
  const uint32_t* const zlast = reinterpret_cast<const uint32_t*>(zpad) + 7;  // zpad: 32 zero bytes
  const uint32_t bsh = frame_shift(dg);
  dg -= bsh;
  for (uint64_t g0 = uint64_t(blk) * kGroups; g0 < n; g0 += step) {
    const uint64_t seg = g0 + threadIdx.x / LPS;
    const bool valid = seg < n;
    // offsets from a clamped index, unconditionally (a load under a divergent
    // branch is waited for at the join, before the stream below is issued)
    uint64_t s, e;
    seg_bounds(offsets, stride, dlen, valid ? seg : n - 1, s, e, bsh);
    if (!valid) e = s;
    ipv4_item<LPS, UNROLL, NT, MODE>(dg, s, e, seg, valid, lane, mode, ip_ck, tcp_ck, status, zpad, zlast);
  }
}

template <int LPS, int UNROLL, bool NT, int MODE>
__global__ __launch_bounds__(kBlock) void k_ipv4_tcp(uint8_t* __restrict__ dg,
                                                     const uint64_t* __restrict__ offsets,
                                                     uint64_t stride, uint64_t dlen, uint64_t n,
                                                     int mode, uint16_t* __restrict__ ip_ck,
                                                     uint16_t* __restrict__ tcp_ck,
                                                     uint8_t* __restrict__ status, uint32_t remap,
                                                     const uint8_t* __restrict__ zpad, Done done) {
  ipv4_body<LPS, UNROLL, NT, MODE>(dg, offsets, stride, dlen, n, mode, ip_ck, tcp_ck, status, zpad,
                                   block_order(remap), gridDim.x);
  signal_done(done);
}

// Two-class launch for receive mixes (ACKs among MTU datagrams): block b
// takes datagrams [4 SPW b, 4 SPW b + 4 SPW), wave w reads the bounds of SPW
// of them and appends each to the block's short (<= 64 bytes) or long list
// in LDS.  Wave 0 then verifies the short ones one per lane, 64 per pass,
// while the other waves — and wave 0 once its short passes are done — claim
// the long ones four at a time (16 lanes each) from an LDS counter.  A wave
// that verified both classes in turn spent a whole memory round trip on its
// short phase for a fraction of a long round's bytes; with the classes
// split over the block's waves only one wave does (½-ACK
// VERIFY of 1 M datagrams 135.5 -> 129.1 us, ¼-ACK 189.7 -> 177.8 us).
template <int SPW, int MODE_OP>  // MODE_OP: the batch's mode as a constant (only its code is built)
__global__ __launch_bounds__(kBlock) void k_ipv4_twoclass(uint8_t* __restrict__ dg, const uint64_t* __restrict__ offsets,
                                                          uint64_t stride, uint64_t dlen, uint64_t n,
                                                          int /*mode: MODE_OP*/, uint16_t* __restrict__ ip_ck,
                                                          uint16_t* __restrict__ tcp_ck, uint8_t* __restrict__ status,
                                                          const uint8_t* __restrict__ zpad, uint32_t remap) {
  constexpr uint32_t kPer = (kBlock / 64) * SPW;
  __shared__ uint64_t lst[kPer][2], sst[kPer][2];  // the block's long / short datagrams' {start, end}
  __shared__ uint32_t lseg[kPer], sseg[kPer];       // ... and their index within the block
  __shared__ uint32_t cnt[3];  // long, short, long claimed
  // COMPUTE / VERIFY: each datagram's header and TCP-field dwords as loaded
  // and its sum land in the block's records (VRec), and the block computes the
  // verdicts at its end, one datagram per lane, and writes them as three
  // coalesced rows: no header broadcast, alignment or verdict in the claims,
  // no 1-2-byte stores in claim order (stack VERIFY of 256 Ki datagrams
  // 36.22 -> 35.72 us back to back; profiles/r4_ab_twoclass_block_verdicts.jsonl).
  // PATCH stages the outputs only (its stores into the datagrams stay in the
  // claim).
  constexpr bool kStash = MODE_OP != 2;
  __shared__ VRec recs[kStash ? kPer : 1];
  __shared__ uint16_t o_ip[kStash ? 1 : kPer], o_tcp[kStash ? 1 : kPer];
  __shared__ uint8_t o_st[kStash ? 1 : kPer];
  VRec* const stash = kStash ? recs : nullptr;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t* const zlast = reinterpret_cast<const uint32_t*>(zpad) + 7;
#ifdef ICSUM_STAMPS
  const uint64_t stamp0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t b0 = uint64_t(block_order(remap)) * kPer;  // the block's datagrams [b0, b0 + kPer)
  const uint64_t seg = b0 + wv * SPW + (lane < SPW ? lane : 0u);
  const bool valid = seg < n && lane < SPW;
  const uint32_t bsh = frame_shift(dg);
  dg -= bsh;
  uint64_t s, e;
  seg_bounds(offsets, stride, dlen, seg < n ? seg : n - 1, s, e, bsh);
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
    lseg[lbase + lr] = uint32_t(seg - b0);
  }
  if (valid && is_short) {
    sst[sbase + sr][0] = s;
    sst[sbase + sr][1] = e;
    sseg[sbase + sr] = uint32_t(seg - b0);
  }
  __syncthreads();
  const uint32_t nlong = cnt[0], nshort = cnt[1];
  if (wv == 0)
    for (uint32_t r0 = 0; r0 < nshort; r0 += 64) {  // uniform
      const uint32_t k = r0 + lane;
      const bool mine = k < nshort;
      const uint32_t kc = mine ? k : 0u;
      const uint64_t ss = sst[kc][0], se = mine ? sst[kc][1] : ss;
      ipv4_item<1, 4, false, 0, kStash>(dg, ss, se, sseg[kc], mine, 0u, MODE_OP, o_ip, o_tcp, o_st, zpad, zlast, stash);
    }
  const uint32_t g = lane >> 4, gl = lane & 15u;
  for (;;) {
    uint32_t r0 = 0;
    if (lane == 0) r0 = atomicAdd(&cnt[2], 4u);
    r0 = __builtin_amdgcn_readfirstlane(r0);
    if (r0 >= nlong) break;  // uniform
    const uint32_t k = r0 + g;
    const bool mine = k < nlong;
    const uint32_t kc = mine ? k : 0u;
    const uint64_t ls = lst[kc][0], le = mine ? lst[kc][1] : ls;
    // 7 loads per lane: a 1500-byte datagram's line-grid span (<= 101 chunks)
    // in one pass of 112 chunks, 70 VGPRs, 7 waves / SIMD (8 loads: 76 VGPRs,
    // 6 waves; stack VERIFY 35.46 -> 34.18 us, r4_ab_twoclass_unroll7.jsonl)
    ipv4_item<16, 7, true, 3, kStash>(dg, ls, le, lseg[kc], mine, gl, MODE_OP, o_ip, o_tcp, o_st, zpad, zlast, stash);
  }
  __syncthreads();
  const uint64_t i = b0 + threadIdx.x;  // every datagram of the block was summed: its row is complete
  if (threadIdx.x < kPer && i < n) {
    uint32_t ipc, tcv, st;
    if constexpr (kStash) {
      const Verdict v = vrec_verdict(recs[threadIdx.x], MODE_OP);
      ipc = v.ipc, tcv = v.tcv, st = v.st;
    } else {
      ipc = o_ip[threadIdx.x], tcv = o_tcp[threadIdx.x], st = o_st[threadIdx.x];
    }
    if (ip_ck) ip_ck[i] = uint16_t(ipc);
    if (tcp_ck) tcp_ck[i] = uint16_t(tcv);
    if (status) status[i] = uint8_t(st);
  }
#ifdef ICSUM_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < (1u << 16)) {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    g_block_stamps[blockIdx.x][0] = stamp0;
    g_block_stamps[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
    g_block_stamps[blockIdx.x][2] = hw;
  }
#endif
}

// ------------------------------------------------- multi-batch launches ---
// The table of a multi-batch launch, by value in the kernel arguments (the
// block offsets are scanned with scalar loads; a batch's fields are loaded
// from the kernel-argument segment at its index — no scratch copy).
template <typename D>
struct BvTable {
  D b[kMaxBatchv];
  uint32_t block0[kMaxBatchv];  // first block of batch j (ascending; block0[0] = 0)
  uint32_t nblk[kMaxBatchv];
  uint32_t k;
};

// the batch that owns (logical) block blk: block0 is ascending and padded
// with 0xFFFFFFFF past the last batch, so the batch index is the number of
// entries 1..15 at or below blk — one scalar compare per entry, a bitmask and
// s_bcnt1 (the uniform index keeps the descriptor load a scalar load)
template <typename D>
__device__ __forceinline__ uint32_t bv_find(const BvTable<D>& t, uint32_t blk) {
  uint32_t mask = 0;
#pragma unroll
  for (uint32_t q = 1; q < uint32_t(kMaxBatchv); ++q) mask |= blk >= t.block0[q] ? (1u << q) : 0u;
  return __builtin_amdgcn_readfirstlane(uint32_t(__builtin_popcount(mask)));
}

template <int CLS>
__global__ __launch_bounds__(kBlock) void k_checksum_batchv(BvTable<BvSeg> t, const u32x4* __restrict__ zero16,
                                                            uint32_t remap) {
  const uint32_t blk = block_order(remap);  // XCD runs over the whole grid, batches in turn
  const uint32_t j = bv_find(t, blk);
  const BvSeg& b = t.b[j];
  const uint32_t lb = blk - t.block0[j], nb = t.nblk[j];
  const uint32_t* ip = b.init ? b.init : reinterpret_cast<const uint32_t*>(zero16);
  const uint32_t is = b.init ? 1u : 0u;
  const uint8_t* op = reinterpret_cast<const uint8_t*>(zero16);
  SegSrc src{b.offsets, b.stride, b.seg_len, nullptr, nullptr, -1};
  const uint8_t* const bytes = rebase(b.bytes, src);  // the dense class is chosen for aligned bases only
  if constexpr (CLS == kBvDense64)
    checksum_dense_body<4, 4, true, 0>(reinterpret_cast<const u32x4*>(b.bytes), ip, is, b.out, b.n, lb);
  else if constexpr (CLS == kBvTiny)
    checksum_tiny_body<0>(bytes, src, ip, is, op, 0u, zero16, b.out, b.n, lb, nb);
  else if constexpr (CLS == kBvSmall)
    checksum_small_body<4, 2, 2, 0>(bytes, src, ip, is, op, 0u, zero16, b.out, b.n, lb, nb);
  else if constexpr (CLS == kBvLine16)
    checksum_body<16, 8, true, 3, 0>(bytes, src, ip, is, op, 0u, b.out, b.n, lb, nb);
  else
    checksum_body<64, 8, true, 3, 0>(bytes, src, ip, is, op, 0u, b.out, b.n, lb, nb);
}

template <int CLS>
__global__ __launch_bounds__(kBlock) void k_ipv4_batchv(BvTable<BvDgram> t, int mode,
                                                        const uint8_t* __restrict__ zpad, uint32_t remap) {
  const uint32_t blk = block_order(remap);
  const uint32_t j = bv_find(t, blk);
  const BvDgram& b = t.b[j];
  const uint32_t lb = blk - t.block0[j], nb = t.nblk[j];
  if constexpr (CLS == kBvLane1)
    ipv4_body<1, 4, false, 0>(b.dgrams, b.offsets, b.stride, b.dlen, b.n, mode, b.ip_ck, b.tcp_ck, b.status, zpad,
                              lb, nb);
  else if constexpr (CLS == kBvLine16)
    ipv4_body<16, 8, true, 3>(b.dgrams, b.offsets, b.stride, b.dlen, b.n, mode, b.ip_ck, b.tcp_ck, b.status, zpad,
                              lb, nb);
  else
    ipv4_body<64, 8, true, 3>(b.dgrams, b.offsets, b.stride, b.dlen, b.n, mode, b.ip_ck, b.tcp_ck, b.status, zpad,
                              lb, nb);
}

// ------------------------------------------------- per-tick host calls ----
// A zero-copy host call of at most kTickSegs segments with offsets (a TUN or
// socket loop's tick, INTEGRATION.md §4 "Per-tick host batches"): one block,
// a 16-lane group per segment, the n + 1 offsets in the kernel arguments.  The
// grid-wide kernels read them from the caller's page-locked offsets, a
// dependent PCIe round trip ahead of the first payload load (1.3-1.6 us of a
// 10-13 us call, profiles/r5_tick_latency.jsonl); here the first loads are
// the payload bytes.  OP 0: checksum (u16 value), 1: the fused IPv4/TCP item.
template <int OP>
__global__ __launch_bounds__(kBlock) void k_tick(uint8_t* __restrict__ bytes, TickOffsets t, uint32_t n,
                                                 const uint32_t* __restrict__ init, uint32_t init_step,
                                                 uint16_t* __restrict__ out, int mode, uint16_t* __restrict__ ip_ck,
                                                 uint16_t* __restrict__ tcp_ck, uint8_t* __restrict__ status,
                                                 const uint8_t* __restrict__ zpad, Done done) {
  const uint32_t g = threadIdx.x >> 4, lane = threadIdx.x & 15u;
  const uint32_t bsh = frame_shift(bytes);
  bytes -= bsh;
  // the wave's four groups' five bounds by scalar loads at a wave-uniform
  // index, in the kernel's first batch of argument loads (nothing they
  // depend on is loaded: the array is zero past n, an idle group's segment
  // is empty), then each group picks its pair
  const uint32_t w4 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 4u;
  uint64_t o[5];
#pragma unroll
  for (uint32_t k = 0; k < 5; ++k) o[k] = t.o[w4 + k];
  const uint32_t q = g & 3u;
  uint64_t s = o[0], e = o[1];
#pragma unroll
  for (uint32_t k = 1; k < 4; ++k)
    if (q == k) s = o[k], e = o[k + 1];
  const bool valid = g < n;
  s += bsh;
  e = valid ? e + bsh : s;
  const uint32_t gi = valid ? g : 0u;
  if constexpr (OP == 0) {
    const uint32_t i0 = init[gi * init_step];
    uint32_t ev = 0, od = 0;
    seg_sums<16, 8, true, 3>(bytes, s, e, lane, ev, od);
    const uint32_t tot = group_sum<16>(combine_roles(ev, od, uint32_t(s) & 1u));
    if (valid && lane == 15) out[g] = fold_value(i0 + tot);
  } else {
    const uint32_t* const zlast = reinterpret_cast<const uint32_t*>(zpad) + 7;
    ipv4_item<16, 8, true, 3>(bytes, s, e, g, valid, lane, mode, ip_ck, tcp_ck, status, zpad, zlast);
  }
  signal_done(done);
}

// ------------------------------------------- device-side wrap (f2) -------
// TCPOverIPv4Adapter::wrap_tcp_in_ip (tcp_over_ip.cpp:69-88) for a batch:
// datagram i = [40 header bytes][payload], the payload already in place (laid
// once at its final offset by the caller).  One pass per datagram sums the
// payload; the lanes of its group then write the serialized IPv4 header
// (ipv4_header.cpp:62-86: ver 4, hlen 5, tos 0, len, id, DF, ttl, proto 6,
// checksum, src, dst) and TCP header (tcp_segment.cpp:76-106: ports, seqno,
// ackno, data offset 5, flags, window, checksum, urgent 0) with both
// checksums: TCPSegment::compute_checksum seeded with the pseudo sum (len =
// 40 + payload, uint16 like the reference's field), then
// IPv4Header::compute_checksum.  hdr_out != nullptr: the 40 bytes go to
// hdr_out[40 i ..] instead of in place (the host-memory path copies only them
// back).  Datagrams shorter than 40 bytes are left as they are.
template <int LPS, int UNROLL, bool NT, int MODE, bool SUMS>
__global__ __launch_bounds__(kBlock) void k_tcp_wrap(uint8_t* __restrict__ dg,
                                                     const uint64_t* __restrict__ offsets,
                                                     uint64_t stride, uint64_t dlen, uint64_t n,
                                                     const TcpMsg* __restrict__ msgs,
                                                     uint32_t* __restrict__ hdr_out,
                                                     uint16_t* __restrict__ ip_ck,
                                                     uint16_t* __restrict__ tcp_ck, uint32_t remap,
                                                     int payload_only, uint32_t* __restrict__ sums, Done done) {
  constexpr uint32_t kGroups = kBlock / LPS;
  const uint32_t lane = threadIdx.x & (LPS - 1);
  const uint64_t step = uint64_t(gridDim.x) * kGroups;
  const uint32_t bsh = frame_shift(dg);
  dg -= bsh;
  for (uint64_t g0 = uint64_t(block_order(remap)) * kGroups; g0 < n; g0 += step) {
    const uint64_t seg = g0 + threadIdx.x / LPS;
    const bool valid = seg < n;
    const uint64_t idx = valid ? seg : n - 1;  // clamped index: every load unconditional
    uint64_t s, e;
    seg_bounds(offsets, stride, dlen, idx, s, e, bsh);
    if (!valid) e = s;
    // payload_only: segment i is the payload alone, its headers go to hdr_out
    const bool ok = valid && (payload_only || e - s >= 40);
    TcpMsg m{};
    if (!SUMS) m = msgs[idx];  // same address across the group: one request per wave instruction
    const uint64_t p0 = ok ? (payload_only ? s : s + 40) : e;  // payload [p0, e)
    uint32_t ev = 0, od = 0;
    seg_sums<LPS, UNROLL, NT, MODE>(dg, p0, e, lane, ev, od);
    uint32_t tot = group_sum<LPS>(combine_roles(ev, od, uint32_t(p0) & 1u));
    if (SUMS) {  // pass 1 of the two-pass wrap: the payload sums only (k_tcp_hdr writes the headers)
      if (valid && lane == LPS - 1) sums[seg] = tot;
      continue;
    }
    if (LPS > 16) tot = __shfl(tot, int((threadIdx.x & 63u) | (LPS - 1)) & 63, 64);  // to every lane of the group
    // both checksums (16-bit big-endian words of the serialized headers)
    const uint32_t len = uint32_t(e - p0 + 40) & 0xffffu;  // IPv4Header::len is uint16
    const uint32_t ttl_proto = (uint32_t(m.ttl) << 8) | 6u;  // big-endian word 4 of the IPv4 header
    const uint32_t addr = (m.src >> 16) + (m.src & 0xffffu) + (m.dst >> 16) + (m.dst & 0xffffu);
    const uint32_t ipc = fold_value(0x4500u + len + m.id + 0x4000u + ttl_proto + addr);
    const uint32_t pseudo = addr + 6u + ((len - 20u) & 0xffffu);  // ipv4_header.cpp:103-110
    const uint32_t thdr = uint32_t(m.sport) + m.dport + (m.seqno >> 16) + (m.seqno & 0xffffu) + (m.ackno >> 16) +
                          (m.ackno & 0xffffu) + (0x5000u | m.flags) + m.window;
    const uint32_t tcv = fold_value(pseudo + thdr + tot);
    // the 10 header dwords over the group's lanes (groups of 4 or 8 lanes
    // write two or three each)
    auto be16 = [](uint32_t v) { return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu); };
    uint8_t* h = dg + s;
    const bool aligned = (reinterpret_cast<uintptr_t>(h) & 3u) == 0;
    for (uint32_t k = lane; ok && k < 10; k += LPS) {
      uint32_t w;  // dword k of the 40 wire bytes, little-endian
      switch (k) {
        case 0: w = 0x45u | (be16(len) << 16); break;
        case 1: w = be16(m.id) | (0x40u << 16); break;
        case 2: w = uint32_t(m.ttl) | (6u << 8) | (be16(ipc) << 16); break;  // ttl, proto, checksum
        case 3: w = bswap32(m.src); break;
        case 4: w = bswap32(m.dst); break;
        case 5: w = be16(m.sport) | (be16(m.dport) << 16); break;
        case 6: w = bswap32(m.seqno); break;
        case 7: w = bswap32(m.ackno); break;
        case 8: w = 0x50u | (uint32_t(m.flags) << 8) | (be16(m.window) << 16); break;
        default: w = be16(tcv); break;  // checksum, urgent pointer 0
      }
      if (hdr_out)
        hdr_out[seg * 10 + k] = w;
      else if (aligned)
        reinterpret_cast<uint32_t*>(h)[k] = w;
      else {
#pragma unroll
        for (int b = 0; b < 4; ++b) h[4 * k + b] = uint8_t(w >> (8 * b));
      }
    }
    if (valid && lane == 0) {
      if (ip_ck) ip_ck[seg] = ok ? uint16_t(ipc) : uint16_t(0);
      if (tcp_ck) tcp_ck[seg] = ok ? uint16_t(tcv) : uint16_t(0);
    }
  }
  signal_done(done);
}

// The 40 wire bytes wrap_tcp_in_ip puts in front of a payload of plen bytes
// whose sum (roles relative to the payload start) is tot, from the message
// record (ics_tcp_msg as dwords: a = src, dst, seqno, ackno; r4 = sport |
// dport << 16; r5 = window | flags << 16 | ttl << 24; r6 = id): the IPv4
// header (ipv4_header.cpp:62-86) and TCP header (tcp_segment.cpp:76-106) as
// 10 little-endian dwords into w, with both checksums —
// TCPSegment::compute_checksum seeded with the pseudo sum, then
// IPv4Header::compute_checksum (tcp_over_ip.cpp:83-84) — also into ipc / tcv.
__device__ __forceinline__ void wrap_header(const u32x4& a, uint32_t r4, uint32_t r5, uint32_t r6, uint64_t plen,
                                            uint32_t tot, uint32_t* w, uint32_t& ipc, uint32_t& tcv) {
  auto be16 = [](uint32_t v) { return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu); };
  const uint32_t sport = r4 & 0xffffu, dport = r4 >> 16, window = r5 & 0xffffu;
  const uint32_t flags = (r5 >> 16) & 0xffu, ttl = r5 >> 24;
  const uint32_t len = uint32_t(plen + 40) & 0xffffu;  // IPv4Header::len is uint16
  const uint32_t addr = (a.x >> 16) + (a.x & 0xffffu) + (a.y >> 16) + (a.y & 0xffffu);
  ipc = fold_value(0x4500u + len + r6 + 0x4000u + ((ttl << 8) | 6u) + addr);
  const uint32_t pseudo = addr + 6u + ((len - 20u) & 0xffffu);  // ipv4_header.cpp:103-110
  const uint32_t thdr = sport + dport + (a.z >> 16) + (a.z & 0xffffu) + (a.w >> 16) + (a.w & 0xffffu) +
                        (0x5000u | flags) + window;
  tcv = fold_value(pseudo + thdr + tot);
  w[0] = 0x45u | (be16(len) << 16);
  w[1] = be16(r6) | (0x40u << 16);                     // id, DF
  w[2] = ttl | (6u << 8) | (be16(ipc) << 16);          // ttl, proto, checksum
  w[3] = bswap32(a.x);
  w[4] = bswap32(a.y);
  w[5] = be16(sport) | (be16(dport) << 16);
  w[6] = bswap32(a.z);
  w[7] = bswap32(a.w);
  w[8] = 0x50u | (flags << 8) | (be16(window) << 16);  // data offset 5, flags, window
  w[9] = be16(tcv);                                    // checksum, urgent pointer 0
}

// Pass 2 of the device wrap when the headers go to an array of their own and
// the batch is large (in place, and for short batches, the one-pass k_tcp_wrap
// above is faster): the headers of 64 datagrams per wave from their 28-byte
// records and the payload sums pass 1 left in `sums`.  Lane d builds datagram
// d's 10 dwords and both checksums (the same arithmetic as k_tcp_wrap); LDS
// turns them around so each store instruction writes 64 consecutive header
// dwords — 256 contiguous bytes of hdr_out, or the headers of 6-7
// neighbouring datagrams in place.  Header stores inside the payload stream
// cost ≈40 ps per datagram apart and ≈85 ps in place
// (profiles/r2_ab_wrap_variant.jsonl); here the apart ones are a
// 14 us launch of their own per 1 M datagrams.
__global__ __launch_bounds__(kBlock) void k_tcp_hdr(uint8_t* __restrict__ dg,
                                                    const uint64_t* __restrict__ offsets, uint64_t stride,
                                                    uint64_t dlen, uint64_t n, const TcpMsg* __restrict__ msgs,
                                                    const uint32_t* __restrict__ sums,
                                                    uint32_t* __restrict__ hdr_out, uint16_t* __restrict__ ip_ck,
                                                    uint16_t* __restrict__ tcp_ck, int payload_only, Done done) {
  __shared__ uint32_t stage[kBlock / 64][64 * 10];  // 10 KiB: each wave's 640 header dwords
  const uint32_t lane64 = threadIdx.x & 63u;
  uint32_t* const sw = stage[threadIdx.x >> 6];
  const uint32_t bsh = frame_shift(dg);
  dg -= bsh;
  for (uint64_t b0 = uint64_t(blockIdx.x) * kBlock; b0 < n; b0 += uint64_t(gridDim.x) * kBlock) {
    const uint64_t base = b0 + (threadIdx.x & ~63u);  // the wave's first datagram
    if (base >= n) continue;                          // wave-uniform
    const uint64_t i = base + lane64;
    const bool valid = i < n;
    const uint64_t idx = valid ? i : n - 1;
    uint64_t s, e;
    seg_bounds(offsets, stride, dlen, idx, s, e, bsh);
    const bool ok = valid && (payload_only || e - s >= 40);
    // the record as dwordx4 + dwordx3 (ics_tcp_msg: src, dst, seqno, ackno;
    // sport | dport << 16; window | flags << 16 | ttl << 24; id)
    const uint32_t* r = reinterpret_cast<const uint32_t*>(msgs + idx);
    u32x4 a;
    __builtin_memcpy(&a, r, 16);
    const uint32_t r4 = r[4], r5 = r[5], r6 = r[6] & 0xffffu;
    const uint32_t tot = sums[idx];
    const uint64_t p0 = payload_only ? s : s + 40;
    uint32_t ipc, tcv;
    wrap_header(a, r4, r5, r6, e - p0, tot, sw + lane64 * 10, ipc, tcv);
    if (valid) {
      if (ip_ck) ip_ck[i] = ok ? uint16_t(ipc) : uint16_t(0);
      if (tcp_ck) tcp_ck[i] = ok ? uint16_t(tcv) : uint16_t(0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // store j: the wave's header dword t = 64 j + lane64 = dword t % 10 of datagram t / 10
    const int s_lo = int(uint32_t(s)), s_hi = int(uint32_t(s >> 32)), ok_i = int(ok);
#pragma unroll
    for (uint32_t j = 0; j < 10; ++j) {
      const uint32_t t = j * 64 + lane64, d = t / 10, k = t - d * 10;
      const uint32_t w = sw[t];
      const bool dok = __shfl(ok_i, int(d), 64) != 0;
      if (hdr_out) {
        if (dok) hdr_out[base * 10 + t] = w;
      } else {
        const uint64_t ds = (uint64_t(uint32_t(__shfl(s_hi, int(d), 64))) << 32) | uint32_t(__shfl(s_lo, int(d), 64));
        uint8_t* h = dg + ds + 4 * k;
        if (dok) {
          if ((reinterpret_cast<uintptr_t>(h) & 3u) == 0)
            *reinterpret_cast<uint32_t*>(h) = w;
          else {
#pragma unroll
            for (int b = 0; b < 4; ++b) h[b] = uint8_t(w >> (8 * b));
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next step rewrites sw
  }
  signal_done(done);
}

// ---------------------------------------------- resident tick server -----
// A one-block kernel that stays resident between ticks and takes each tick's
// job from a mailbox in coherent page-locked host memory (TickMailbox,
// icsum_launch.h) instead of being launched per tick: a tick then pays no
// launch (the ~3-5 us from the doorbell to the first wave), only the
// mailbox poll and the payload's PCIe reads.  Every descriptor word carries
// the job's sequence number in its high half, so one poll (wave 0: lane k
// reads word k, lane 63 the quit word) that finds the expected number in
// every word the job uses has read a complete descriptor, whatever order the
// host's stores landed in.  The job runs as k_tick's body (16-lane group per
// segment, starts / lengths from the descriptor), its results go to the
// job's page-locked result area, and `done` takes the sequence number with a
// system-scope release.  The server exits on the quit word, after idle_us
// without a job, or after kSrvMaxLife of 100 MHz ticks (the host relaunches
// it when a job finds it gone): every wave reaches an exit.
// Several blocks (ics_ctx::srv_blocks): block b serves mailbox b, with its
// own sequence numbers; a tick of n > 16 segments is split over mailboxes
// 0 .. ceil(n / 16) - 1 (w[kSrvPart]: the sub-job's first segment and the
// tick's n place its results), and every tick has a part in mailbox 0.  Block
// 0 alone decides to leave (quit word, idle, lifetime) and says so in its
// `state`; blocks b > 0 poll that word in place of the quit word and leave
// once they see it, so the grid leaves as a whole and the host relaunches
// only a grid that has fully left (no two blocks ever serve one mailbox).
constexpr uint64_t kSrvMaxLife = 100000000ull;  // 1 s of s_memrealtime

__global__ __launch_bounds__(kBlock) void k_tick_server(uint64_t* words, TickMailbox* mbs,
                                                        const uint8_t* __restrict__ zpad, uint32_t idle_us,
                                                        uint32_t pollers) {
  __shared__ uint32_t s_desc[64];
  __shared__ uint32_t s_cmd;  // 0 none yet, 1 a job, 2 exit
  TickMailbox* const mb = mbs + blockIdx.x;
  const uint64_t* const mw = words + kSrvWords * blockIdx.x;  // this block's descriptor words
  const bool lead = blockIdx.x == 0;
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t g = threadIdx.x >> 4, gl = threadIdx.x & 15u;
  const uint32_t* const zlast = reinterpret_cast<const uint32_t*>(zpad) + 7;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t_job = t0;
  // the oldest job of this mailbox not done (the grid before this one has
  // left: its last `done` store is final)
  uint32_t expect = uint32_t(__hip_atomic_load(&mb->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) + 1u;
  // lane 63's poll word: the quit word (block 0) or block 0's exit word
  const uint64_t* const w63 = lead ? &words[kSrvQuit] : &words[kSrvExit];
  if (threadIdx.x == 0) s_cmd = 0u;
  __syncthreads();
  for (;;) {
    // waves 0 .. pollers - 1 poll, each on its own, started a fraction of a
    // PCIe round trip apart: a job posted at a random moment is seen by the
    // next poll to start, sooner with more pollers.  The first to see the
    // job, the quit word or the idle limit claims s_cmd (a job claimed
    // first wins over another wave's idle verdict); the rest stop polling.
    if (wv < pollers) {
      for (uint32_t k = 0; k < wv; ++k) __builtin_amdgcn_s_sleep(14);  // ~0.4 us each
      while (__hip_atomic_load(&s_cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
        const uint64_t word =
            __hip_atomic_load(lane == kSrvQuit ? w63 : &mw[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t pay = uint32_t(word), seq = uint32_t(word >> 32);
        const uint32_t w0 = __builtin_amdgcn_readlane(pay, 0), s0 = __builtin_amdgcn_readlane(seq, 0);
        const uint32_t nj = (w0 >> 8) & 0xffu, nw = kSrvHead + 2u * nj;  // the words this job uses
        const bool inits = (w0 >> 16) & 1u;
        const bool used = lane < nw || lane == kSrvPart || (inits && lane >= kSrvInit && lane < kSrvInit + nj);
        const bool fresh = !used || seq == expect;
        const bool job = s0 == expect && __all(fresh);
        const uint64_t q = __builtin_amdgcn_readlane(uint32_t(word | (word >> 32)), kSrvQuit);
        const bool quit = q != 0;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        // blocks b > 0 leave with block 0 (their lifetime bound only a backstop)
        const bool idle = lead ? now - t_job > uint64_t(idle_us) * 100u || now - t0 > kSrvMaxLife
                               : now - t0 > 2 * kSrvMaxLife;
        if (job && !quit) s_desc[lane] = pay;  // (another poller may store the same words)
        if (job || quit || idle) {
          if (lane == 0) {
            uint32_t none = 0u;
            __hip_atomic_compare_exchange_strong(&s_cmd, &none, quit ? 2u : job ? 1u : 2u, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
    const uint32_t cmd = s_cmd;
    if (cmd == 2u) break;  // uniform
    // a resident kernel gets no launch-time cache invalidation: without this
    // system-scope acquire its loads of the reused staging slots would hit
    // the previous job's lines still held in L1 / L2
    // (the L2 holds such lines: without it, or with the CU's L1 alone
    // invalidated, the tests read the previous job's bytes;
    // profiles/r6_tick_server_inv.jsonl)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    // the job: checksum (op 0) or the fused IPv4 item (op 1, mode), n <= 16
    // segments at [bytes + s_j, + len_j), results into the page-locked area
    const uint32_t w0 = s_desc[0], op = w0 & 0xfu, mode = (w0 >> 4) & 0xfu, n = (w0 >> 8) & 0xffu;
    // the sub-job's segments are the tick's [first, first + n) of nt
    const uint32_t first = s_desc[kSrvPart] & 0xffu, nt = (s_desc[kSrvPart] >> 8) & 0xffu;
    uint8_t* bytes = reinterpret_cast<uint8_t*>(uint64_t(s_desc[1]) | (uint64_t(s_desc[2]) << 32));
    const uint32_t* init = reinterpret_cast<const uint32_t*>(uint64_t(s_desc[3]) | (uint64_t(s_desc[4]) << 32));
    uint8_t* res = reinterpret_cast<uint8_t*>(uint64_t(s_desc[5]) | (uint64_t(s_desc[6]) << 32));
    const uint32_t bsh = frame_shift(bytes);
    bytes -= bsh;
    const bool valid = g < n;
    const uint32_t gi = valid ? g : 0u;
    const uint64_t s = uint64_t(s_desc[kSrvHead + 2u * gi]) + bsh;
    const uint64_t e = valid ? s + s_desc[kSrvHead + 2u * gi + 1u] : s;
    // per-segment words (inits, message records) requested with the stream,
    // unconditionally (a load under a branch is waited for at its join,
    // ahead of the stream: one more PCIe round trip)
    const uint32_t* const iw = init ? init : reinterpret_cast<const uint32_t*>(zpad);
    if (op == 0u) {
      const uint32_t i0 = (w0 >> 16) & 1u ? s_desc[kSrvInit + gi] : 0u;
      uint32_t ev = 0, od = 0;
      seg_sums<16, 8, true, 3>(bytes, s, e, gl, ev, od);
      const uint32_t tot = group_sum<16>(combine_roles(ev, od, uint32_t(s) & 1u));
      if (valid && gl == 15) reinterpret_cast<uint16_t*>(res)[first + g] = uint16_t(fold_value(i0 + tot));
    } else if (op == 2u) {
      // wrap_tcp_in_ip (tcp_over_ip.cpp:69-88) as k_tcp_wrap with its headers
      // to an array: the payload after 40 bytes of header room (mode 0) or
      // the segment alone (mode 1); the record (ics_tcp_msg) at `init`
      const bool ok = valid && (mode == 1u || e - s >= 40);
      const uint64_t p0 = ok ? (mode == 1u ? s : s + 40) : e;
      const uint32_t* rec = iw + 7u * (first + gi);  // 28-byte records
      uint32_t r[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) r[k] = rec[k];
      uint32_t ev = 0, od = 0;
      seg_sums<16, 8, true, 3>(bytes, p0, e, gl, ev, od);
      const uint32_t tot = __shfl(group_sum<16>(combine_roles(ev, od, uint32_t(p0) & 1u)),
                                  int((threadIdx.x & 63u) | 15u), 64);  // to every lane of the group
      const u32x4 a{r[0], r[1], r[2], r[3]};
      uint32_t w[10], ipc, tcv;
      wrap_header(a, r[4], r[5], r[6] & 0xffffu, e - p0, tot, w, ipc, tcv);
      uint32_t wk = w[0];
#pragma unroll
      for (uint32_t k = 1; k < 10; ++k) wk = gl == k ? w[k] : wk;
      if (ok && gl < 10) reinterpret_cast<uint32_t*>(res)[10u * (first + g) + gl] = wk;
    } else {
      uint16_t* ip = reinterpret_cast<uint16_t*>(res);
      ipv4_item<16, 8, true, 3>(bytes, s, e, g, valid, gl, int(mode), ip + first, ip + nt + first,
                                res + 4u * nt + first, zpad, zlast);
    }
    // results out before `done` (signal_done's order): every wave's stores
    // retired, the block's barrier, one system-scope release
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(&mb->done, uint64_t(expect), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    ++expect;
    t_job = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) s_cmd = 0u;  // every wave read it at the barrier before the done store
    __syncthreads();  // s_desc / s_cmd are rewritten by the next poll
  }
  if (threadIdx.x == 0) {
    if (lead) __hip_atomic_store(&words[kSrvExit], uint64_t(1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&mb->state, uint64_t(kSrvExited), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// --------------------------------------------------- router batch -------
// Two lanes per datagram: lane 0 loads header dwords 0, 2, 4 and lane 1
// dwords 1, 3, 5, so each wave instruction touches 32 header lines with two
// neighbouring dwords each instead of 64 lines with one (one lane loading all
// six dwords: six instructions of 64 lines; the memory side then saw ~1.9
// 128-byte read requests per datagram for ~1.16 lines of header).  Measured
// (git 7692616:tools/probe/router_probe.hip, profiles/r2_router_probe.jsonl): 1 M x 1500 B
// 59.8 -> 57.3 us; the read-only floor of the same headers is 35-41 us, the
// rest is the scattered 8-byte write-back of every forwarded header.
__global__ __launch_bounds__(kBlock) void k_router_ttl(uint8_t* __restrict__ dg,
                                                       const uint64_t* __restrict__ offsets,
                                                       uint64_t stride, uint64_t dlen, uint64_t n,
                                                       uint8_t* __restrict__ status,
                                                       const uint32_t* __restrict__ zpad) {
  constexpr uint32_t kG = kBlock / 2;
  const uint32_t lane = threadIdx.x & 1u;
  const uint64_t step = uint64_t(gridDim.x) * kG;
  const uint32_t bsh = frame_shift(dg);
  dg -= bsh;
  // the loop bound is uniform per block (group base index), so both lanes of
  // every pair reach the shuffles together
  for (uint64_t g0 = uint64_t(blockIdx.x) * kG; g0 < n; g0 += step) {
    const uint64_t i = g0 + threadIdx.x / 2;
    const bool valid = i < n;
    uint64_t s, e;
    seg_bounds(offsets, stride, dlen, valid ? i : n - 1, s, e, bsh);
    const bool hdr = valid && e - s >= 20;
    uint8_t* p = dg + s;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
    // a datagram too short for a header (or an idle pair) reads the zero pad
    const uint32_t* q = hdr ? reinterpret_cast<const uint32_t*>(p - sh) : zpad;
    const uint32_t* last = hdr ? last_dword(dg + e) : zpad + 7;
    uint32_t mine[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t* a = q + (lane + 2u * k);
#ifdef ICSUM_BOUNDS_CHECK
      if (hdr && k < 2 && a > last) bounds_fail(kBoundsHeader, reinterpret_cast<unsigned long long>(a));
#endif
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
        // NetworkInterface::recv_frame parse (network_interface.cpp:51) then
        // Router::route: ttl <= 1 dropped, else ttl-- and compute_checksum()
        if (ver == 4 && hlen >= 5 && fold_value(ipv4_header_sum(h)) == h.be16(10) && ttl > 1) {
          h.w[2] = (h.w[2] & ~0xffu) | (ttl - 1);
          const uint32_t c = fold_value(ipv4_header_sum(h));
          if (sh == 0) {
            // dword-aligned header (every fixed stride that is a multiple of 4):
            // wire bytes 4..11 rewritten by ONE 8-byte store instead of three
            // narrow ones — id and fragment offset as read, the flags byte
            // re-serialized (reserved bit dropped), ttl - 1, protocol, checksum
            const uint32_t w1 = h.w[1] & ~0x00800000u;
            const uint32_t w2 = (h.w[2] & 0x0000ffffu) | ((c >> 8) << 16) | ((c & 0xffu) << 24);
            uint32_t* o = reinterpret_cast<uint32_t*>(p + 4);  // 4-byte aligned: merged to one dwordx2 store
            o[0] = w1;
            o[1] = w2;
          } else {
            p[6] = uint8_t(h.byte(6) & 0x7fu);  // re-serialized flags word
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

// Router batch with the forwarded headers apart.  Router::route decrements
// the ttl, recomputes the header checksum and hands send_datagram the
// datagram (router.cpp:39-66), which serialize() turns into two pieces: the
// 20 serialized header bytes (ipv4_header.cpp:62-86: options never written,
// the reserved flag bit dropped) and the payload after the parsed header
// (4 hlen bytes in, ipv4_header.cpp:50).  Here the payloads stay where they
// are (read-only batch) and the forwarded headers go to one coalesced array,
// 20 bytes per datagram: a forwarded datagram's header there is byte for
// byte what the in-place k_router_ttl leaves in its first 20 bytes; a
// dropped or unparseable one gets 20 zero bytes.  Headers are read as in
// k_router_ttl (two lanes per datagram, three dwords each); each wave stages
// its 32 headers in LDS and stores them as 160 consecutive dwords.
__global__ __launch_bounds__(kBlock) void k_router_hdrs(const uint8_t* __restrict__ dg,
                                                        const uint64_t* __restrict__ offsets, uint64_t stride,
                                                        uint64_t dlen, uint64_t n, uint32_t* __restrict__ hdr_out,
                                                        uint8_t* __restrict__ status,
                                                        const uint32_t* __restrict__ zpad) {
  constexpr uint32_t kG = kBlock / 2, kPerWave = 32;
  __shared__ uint32_t stage[kBlock / 64][kPerWave * 5];
  const uint32_t lane = threadIdx.x & 1u, lane64 = threadIdx.x & 63u;
  uint32_t* const sw = stage[threadIdx.x >> 6];
  const uint64_t step = uint64_t(gridDim.x) * kG;
  const uint32_t bsh = frame_shift(dg);
  dg -= bsh;
  for (uint64_t g0 = uint64_t(blockIdx.x) * kG; g0 < n; g0 += step) {  // uniform per block
    const uint64_t i = g0 + threadIdx.x / 2;
    const bool valid = i < n;
    uint64_t s, e;
    seg_bounds(offsets, stride, dlen, valid ? i : n - 1, s, e, bsh);
    const bool hdr = valid && e - s >= 20;
    const uint8_t* p = dg + s;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
    const uint32_t* q = hdr ? reinterpret_cast<const uint32_t*>(p - sh) : zpad;
    const uint32_t* last = hdr ? last_dword(dg + e) : zpad + 7;
    uint32_t mine[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t* a = q + (lane + 2u * k);
#ifdef ICSUM_BOUNDS_CHECK
      if (hdr && k < 2 && a > last) bounds_fail(kBoundsHeader, reinterpret_cast<unsigned long long>(a));
#endif
      mine[k] = *(a < last ? a : last);
    }
    const int pair = int(lane64 & ~1u);
    uint32_t d[6];
#pragma unroll
    for (int w = 0; w < 6; ++w) d[w] = uint32_t(__shfl(int(mine[w / 2]), pair + (w & 1), 64));
    Hdr h;
#pragma unroll
    for (int k = 0; k < 5; ++k) h.w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
    const uint32_t ver = h.byte(0) >> 4, hlen = h.byte(0) & 0x0fu, ttl = h.byte(8);
    // NetworkInterface::recv_frame parse (network_interface.cpp:51), then
    // Router::route: ttl <= 1 dropped, else ttl-- and compute_checksum()
    const bool fwd = hdr && ver == 4 && hlen >= 5 && fold_value(ipv4_header_sum(h)) == h.be16(10) && ttl > 1;
    h.w[2] = (h.w[2] & ~0xffu) | ((ttl - 1) & 0xffu);
    const uint32_t c = fold_value(ipv4_header_sum(h));
    uint32_t o[5];
    o[0] = h.w[0];
    o[1] = h.w[1] & ~0x00800000u;  // the flags word re-serialized: reserved bit dropped
    o[2] = (h.w[2] & 0x0000ffffu) | ((c >> 8) << 16) | ((c & 0xffu) << 24);
    o[3] = h.w[3];
    o[4] = h.w[4];
    const uint32_t slot = (lane64 >> 1) * 5;
    for (uint32_t k = lane; k < 5; k += 2) sw[slot + k] = fwd ? o[k] : 0u;
    if (valid && lane == 0) status[i] = fwd ? 1 : 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the wave's datagrams [wbase, wbase + 32): 160 consecutive dwords of the array
    const uint64_t wbase = g0 + (threadIdx.x >> 6) * kPerWave;
    const uint64_t cnt = wbase < n ? (n - wbase < kPerWave ? n - wbase : kPerWave) : 0;
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
      const uint32_t t = j * 64u + lane64;
      if (t < cnt * 5) hdr_out[wbase * 5 + t] = sw[t];
    }
    __builtin_amdgcn_wave_barrier();  // the next pass rewrites sw
  }
}

// ------------------------------------------ tile launches (offsets) -------
// An offsets batch is one packed byte stream: segment i = [off[i], off[i+1]).
// The tile launch streams it by position, whatever the segment lengths: no
// lane idles on an ACK-sized segment and no lane group waits on an MTU-sized
// one (the per-segment launches above map one segment to a lane group).
// Segment i's sums over [lo_i, hi_i) are F(hi_i) - F(lo_i), F(x) the sums of
// the stream's bytes below x: exact in uint32 (addition mod 2^32), roles by
// address parity.
//   checksum  lo = start                        (checksum.h:20-41)
//   IPv4/TCP  lo = start + 4 hlen (TCP part)    (ipv4_header.cpp:50, tcp_segment.cpp:11-18)
//   wrap      lo = start + 40 (the payload)     (tcp_over_ip.cpp:69-88)
//   wrap, headers apart: lo = start (segments are payloads), the headers go
//             to an array of their own, 40 contiguous bytes per segment
// k_span below runs it; round 4's k_tile (a block per T segments, each wave
// streaming a quarter of the tile, the points sorted in LDS) is gone since
// round 5 (git c581ecc; profiles/r5k_ab_span_ops.jsonl).
constexpr uint32_t kWinChunks = 256;          // one wave window: 4 KiB, four loads per lane
constexpr int kTileSum = 0, kTileIpv4 = 1, kTileWrap = 2, kTileWrapApart = 3;

// LDS slot of chunk r of a window (16-byte slots): r ^ ((r >> 4) & 3).  The
// window is written as loaded (lane l: chunks 64 u + l, eight contiguous
// lanes per ds_write_b128 group: still conflict-free) and read back four
// consecutive chunks per lane (lane L: 4 L .. 4 L + 3); without the swizzle
// every ds_read_b128 lane group (16 lanes, banks (a / 4) mod 64) of that
// read hits only 4 distinct 16-byte bank groups — 4-way conflicts
// (SQ_LDS_BANK_CONFLICT 15 M cycles per 1 M x 770 B launch,
// profiles/r5_pmc_stream.jsonl); with it each group's 16 lanes cover all 16.
__device__ __forceinline__ uint32_t win_slot(uint32_t r) { return r ^ ((r >> 4) & 3u); }

// inclusive prefix sum over the 64 lanes of a wave: row shifts 1, 2, 4, 8,
// then row 0's total into row 1 and row 2's into row 3, then rows 0-1's into
// rows 2-3
__device__ __forceinline__ uint32_t wave_prefix_incl(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

struct TileArgs {
  // checksum: per-segment initial sums and parities (zero16 + step 0 when absent), u16 or u32 out
  const uint32_t* init;
  const uint8_t* odd;
  uint32_t init_step, odd_step;
  void* out;
  // IPv4 / TCP: mode and the three outputs (each nullable)
  int mode;
  uint16_t* ip_ck;
  uint16_t* tcp_ck;
  uint8_t* status;
  // wrap: the message records; headers apart: the 40-byte headers' array
  const TcpMsg* msgs;
  uint32_t* hdr_out;
};

// ---------------------------------------- wave spans (round 5) -------------
// k_span: every wave on its own.  Wave w owns segments [S w, S w + S) of an
// offsets batch (S <= 63: the dispatch sizes spans from the batch's mean
// length) and streams their bytes [off[i0] & ~15, off[i0 + m]) as
// one range in 4 KiB windows: three register sets, each reloaded as soon as
// its window is in LDS (three windows in flight while one is summed), the
// window written to swizzled LDS slots as loaded and read back four chunks
// per lane, one wave scan per role.  Lane p holds point A = off[i0 + p]
// (p <= m <= S) in registers for the whole span: the window holding it sets
// the lane's F (prefix + masked chunk) — no point lists, loops or LDS buffers
// — and segment t's sums up to its end are F(t + 1), lane t + 1's value one
// shuffle away.  The lo = start operations (checksum; headers-apart wrap)
// take segment t's sums as F(t + 1) - F(t); the others give lane t a second
// point B = lo_t (IPv4: start + 4 IHL, the header's first dword fetched
// before the stream; in-place wrap: start + 40) and take F(t + 1) - F(B).
// No block barrier and no block-level state: a block is four independent
// waves, and the hardware dispatcher balances them over the chip the way it
// does one-shot waves (a persistent or one-tile-per-block grid leaves the
// chip's last waves unbalanced: static tiles 72 %, one-shot waves 82 % of
// 8 TB/s streaming the same 141 MB, profiles/r5_probe_grab.jsonl).
// Every F of a span comes from the wave's single copy of each window, so
// bytes of a neighbouring span's segments that share a boundary chunk (and
// that span's in-place stores into them) cancel out of every difference.
// Per-segment words the outputs need are fetched after the stream (the
// checksum's two ride along it): fewer registers across the window loop.
constexpr uint32_t kSpanSegs = 63;  // most segments per wave: 64 points, one per lane

__device__ __forceinline__ uint64_t shfl_down64(uint64_t v) {
  return uint64_t(uint32_t(__shfl_down(uint32_t(v), 1))) | (uint64_t(uint32_t(__shfl_down(uint32_t(v >> 32), 1))) << 32);
}

// The outputs of a span of m segments [i0, i0 + m) once every lane holds
// F of its point A (fe, fo: the sums of the span's bytes below x) and of its
// point B (ge, go: below lo): segment t = lane t's sums are F(A_{t+1}) -
// F(B_t).  Checksum: init0 / odd0 are the segment's init and parity words.
// Wraps: `stage` is 10 * 64 dwords of the wave's LDS (free once the stream is
// summed).  Every lane of the wave calls it.
template <int OP, int OUT>
__device__ __forceinline__ void span_outputs(uint8_t* __restrict__ bytes, const TileArgs& a, uint32_t lane,
                                             bool valid, uint64_t i, uint64_t i0, uint32_t m, uint64_t x,
                                             uint64_t e, uint64_t lo, bool hdr, uint32_t fe, uint32_t fo,
                                             uint32_t ge, uint32_t go, uint32_t init0, uint32_t odd0,
                                             uint32_t* __restrict__ stage) {
  // segment t's sums up to its end: lane t + 1's F (every lane shuffles,
  // outside the branches below: a shuffle from a lane a branch disables
  // reads nothing defined)
  const uint32_t he = __shfl_down(fe, 1), ho = __shfl_down(fo, 1);
  const uint32_t se = he - ge, so = ho - go;  // sums of [lo, e), roles by address
  if constexpr (OP == kTileSum) {
    if (valid) {
      const uint32_t sum = init0 + combine_roles(se, so, (uint32_t(x) ^ odd0) & 1u);
      if (OUT == 0)
        static_cast<uint16_t*>(a.out)[i] = fold_value(sum);
      else
        static_cast<uint32_t*>(a.out)[i] = sum;
    }
  } else if constexpr (OP == kTileIpv4) {
    // the header and the TCP fields at the real start of the TCP part (after
    // the stream: no window load waits behind them)
    if (valid) {
      const uint32_t* last = last_dword(bytes + e);
      Hdr h{};
      uint32_t tf0 = 0, tf1 = 0;
      if (hdr) {
        h = load_hdr(bytes + x, last);
        if (e - lo >= 18) load_tcp_fields(bytes + lo, last, tf0, tf1);
      }
      ipv4_result(bytes, x, e, lo, hdr, h, tf0, tf1, combine_roles(se, so, uint32_t(lo) & 1u), a.mode, i, a.ip_ck,
                  a.tcp_ck, a.status);
    }
  } else {
    // the message record, then the header into the wave's (now idle) window
    // slots: 10 dwords per segment, the span's m headers contiguous
    const uint32_t* rec = reinterpret_cast<const uint32_t*>(a.msgs + i);
    uint32_t w[7];
#pragma unroll
    for (uint32_t k = 0; k < 7; ++k) w[k] = rec[k];
    const bool ok = valid && (OP == kTileWrapApart || e - x >= 40);
    if (valid) {
      uint32_t ipc = 0, tcv = 0;
      wrap_header(u32x4{w[0], w[1], w[2], w[3]}, w[4], w[5], w[6] & 0xffffu, e - lo,
                  combine_roles(se, so, uint32_t(lo) & 1u), stage + lane * 10u, ipc, tcv);
      if (a.ip_ck) a.ip_ck[i] = ok ? uint16_t(ipc) : uint16_t(0);
      if (a.tcp_ck) a.tcp_ck[i] = ok ? uint16_t(tcv) : uint16_t(0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (OP == kTileWrapApart) {
      // the span's 10 m header dwords are one contiguous run of hdr_out:
      // coalesced 256-byte stores instead of 40-byte strides per lane
      uint32_t* const dst = a.hdr_out + i0 * 10;
#pragma unroll
      for (uint32_t j = 0; j < 10; ++j) {
        const uint32_t q = j * 64u + lane;
        if (q < m * 10u) dst[q] = stage[q];
      }
    } else {
      // in place: dword q of the span = dword q % 10 of segment q / 10
      // (neighbouring lanes, neighbouring bytes); its start and whether it
      // holds a header come from lane q / 10 (every lane shuffles)
      const uint32_t okw = ok ? 1u : 0u;
#pragma unroll 2
      for (uint32_t j = 0; j < 10; ++j) {
        const uint32_t q = j * 64u + lane, d = q / 10u, k = q - d * 10u;
        const uint32_t src = d < 64u ? d : 63u;
        const uint64_t ds = uint64_t(uint32_t(__shfl(uint32_t(x), int(src)))) |
                            (uint64_t(uint32_t(__shfl(uint32_t(x >> 32), int(src)))) << 32);
        const uint32_t dok = uint32_t(__shfl(okw, int(src)));
        if (d < m && dok) {
          const uint32_t v = stage[q];
          uint8_t* q8 = bytes + ds + 4u * k;
          if ((reinterpret_cast<uintptr_t>(q8) & 3u) == 0) {
            *reinterpret_cast<uint32_t*>(q8) = v;
          } else {
#pragma unroll
            for (int b = 0; b < 4; ++b) q8[b] = uint8_t(v >> (8 * b));
          }
        }
      }
    }
  }
}

template <int OP, int OUT, bool STRIDE>
__global__ __launch_bounds__(kBlock) void k_span(uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                 uint64_t n, uint32_t S, TileArgs a, uint32_t remap,
                                                 const u32x4* __restrict__ zero16) {
  constexpr bool TWO = OP == kTileIpv4 || OP == kTileWrap;  // a second point per lane: lo_t
  constexpr uint32_t kWaves = kBlock / 64;
  __shared__ uint32_t s_pre[kWaves][kWinChunks][2];
  __shared__ u32x4 s_raw[kWaves][kWinChunks];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nspans = (n + S - 1) / S;
  const uint32_t bsh = frame_shift(bytes);  // the kernel's frame (icsum_device.h): points and windows absolute
  bytes -= bsh;
  // one span per wave; STRIDE (batches of more spans than 2^24 blocks hold):
  // grid-stride beyond the grid.  Wave-uniform, no block barrier anywhere.
  auto span_body = [&](uint64_t span) {
  const uint64_t i0 = span * S;
  const uint32_t m = uint32_t(n - i0 < S ? n - i0 : S);
  const bool valid = lane < m;
  const uint64_t i = i0 + (valid ? lane : 0u);  // lanes >= m: a harmless copy of segment 0
  // point A (one load per lane) and, for the checksum, the per-segment words —
  // in flight before the first window is requested
  const uint64_t x = off[i0 + (lane <= m ? lane : m)] + bsh;
  uint32_t w[2] = {0u, 0u};  // checksum: the segment's init and parity
  if constexpr (OP == kTileSum) {
    w[0] = a.init[i * a.init_step];
    w[1] = a.odd[i * a.odd_step];
  }
  // the span's byte range: two scalar loads at wave-uniform indices (the
  // stream's addresses wait for the scalar cache, not for the vector load)
  const uint64_t first = off[i0] + bsh, tend = off[i0 + m] + bsh;
  // segment t = [x, e): e is lane t + 1's point (taken by every lane).  IPv4
  // takes it before the stream, for the header's first dword (the IHL); the
  // other operations after the stream is requested
  uint64_t e = 0;
  bool hdr = false;
  uint32_t d0 = 0, d0sh = 0;  // the dword holding header byte 0 and that byte's place in it
  if constexpr (OP == kTileIpv4) {
    e = shfl_down64(x);
    hdr = valid && e - x >= 20;
    const uint8_t* hp = hdr ? bytes + x : reinterpret_cast<const uint8_t*>(zero16);
    d0sh = uint32_t(reinterpret_cast<uintptr_t>(hp) & 3u);
    d0 = *reinterpret_cast<const uint32_t*>(hp - d0sh);
  }
  // the windows start on the 128-byte line (of `bytes`) holding the first
  // byte, so each 1 KiB load instruction covers 8 whole lines, not 9 partial
  // ones; the chunks below `first` enter every F of the span alike and cancel
  const uint64_t a0c = (first >> 7) << 3;
  const uint64_t nch = tend > (a0c << 4) ? ((tend + 15) >> 4) - a0c : 0;
  const uint64_t nw = (nch + kWinChunks - 1) / kWinChunks;
  // three register sets per wave, each reloaded as soon as its window is in
  // LDS: up to three windows in flight (two sets at 6 waves / SIMD, and three
  // forced to 5 waves / SIMD by spilling, measured equal or slower:
  // profiles/r5y_ab_span_sets_waves.jsonl)
  constexpr uint32_t kSets = 3;
  const uint64_t nwin3 = nw ? (nw + kSets - 1) / kSets * kSets : kSets;  // whole rounds of the sets
  const uint32_t voff = lane * 16u;
  auto load_win = [&](uint64_t k, u32x4 (&v)[4]) {
    const uint64_t c0 = k * kWinChunks;
    const uint64_t left = nch > c0 ? nch - c0 : 0;
    const uint32_t len = uint32_t(left < kWinChunks ? left : kWinChunks);
    const u32x4* pw = reinterpret_cast<const u32x4*>(bytes) + a0c + (len ? c0 : 0);
#ifdef ICSUM_BOUNDS_CHECK
    if (len) {
      const uint8_t* lo8 = bytes + (a0c << 4);
      ICS_CHECK16(pw, lo8, lo8 + (nch << 4));
      ICS_CHECK16(pw + len - 1, lo8, lo8 + (nch << 4));
    }
#endif
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4*>(pw), 0, int(len * 16u), 0x00020000);
#pragma unroll
    for (int u = 0; u < 4; ++u)  // aux 2: non-temporal
      v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, u * 1024, 2));
  };
  u32x4 b0[4], b1[4], b2[4];
  // in this order: the loop consumes b0 first, and vmcnt retires loads in issue order
  load_win(0, b0);
  __builtin_amdgcn_sched_barrier(0);
  load_win(1, b1);
  __builtin_amdgcn_sched_barrier(0);
  load_win(2, b2);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (OP != kTileIpv4) e = shfl_down64(x);
#ifdef ICSUM_BOUNDS_CHECK
  if (valid && e < x) bounds_fail(kBoundsOffsets, i);
#endif
  // point B, once the windows are out: IPv4 past the header (options skipped,
  // ipv4_header.cpp:50), the in-place wrap past the 40 header bytes it rewrites
  auto point_b = [&](uint64_t e_) {
    uint64_t lo_ = x;
    if constexpr (OP == kTileIpv4) {
      uint64_t o = 4u * ((d0 >> (8u * d0sh)) & 0x0fu);  // the byte in the frame of the load
      if (o < 20) o = 20;
      if (hdr && o > e_ - x) o = e_ - x;
      lo_ = hdr ? x + o : e_;
    } else if constexpr (OP == kTileWrap) {
      lo_ = valid && e_ - x >= 40 ? x + 40 : e_;
    }
    return lo_;
  };
  const uint64_t lo = point_b(e);
  // the lane's points: chunk (span-relative, 32 bits) and byte; lanes past m
  // hold no A, lanes >= m no B
  const uint32_t pc = lane <= m ? uint32_t((x >> 4) - a0c) : ~0u;
  const uint32_t pb = uint32_t(x) & 15u;
  const uint32_t qc = TWO && valid ? uint32_t((lo >> 4) - a0c) : ~0u;
  const uint32_t qb = uint32_t(lo) & 15u;
  uint32_t ce = 0, co = 0;  // the span's sums so far
  uint32_t fe = 0, fo = 0;  // F of point A (set by the window holding it)
  uint32_t ge = 0, go = 0;  // F of point B
  // F at a point inside window [c0, c1): its chunk's prefix + the chunk's bytes below it
  auto point_F = [&](uint32_t c, uint32_t b, uint64_t c0, uint32_t& fe_, uint32_t& fo_) {
    const uint32_t k2 = uint32_t(c - c0);
    fe_ = s_pre[wv][k2][0];
    fo_ = s_pre[wv][k2][1];
    acc_chunk(s_raw[wv][win_slot(k2)] & byte_range_mask(0u, b), fe_, fo_);
  };
  auto window = [&](uint64_t k, u32x4 (&v)[4]) {
    const uint64_t c0 = k * kWinChunks;
    const bool live = c0 < nch;  // uniform; else a padding window
    if (live) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s_raw[wv][win_slot(uint32_t(u) * 64u + lane)] = v[u];
    }
    load_win(k + kSets, v);  // the registers are free: window k + kSets goes out now (one load site)
    if (!live) return;
#ifdef ICSUM_SPAN_PROBE_STREAM_ONLY
    // diagnostic build only (tools/probe/span_probe.hip): the loads, the LDS
    // writes and one read back per lane, no scan, prefix or points (results
    // wrong, time only)
    {
      const u32x4 r = s_raw[wv][win_slot(4u * lane)];
      ce += r.x ^ r.y ^ r.z ^ r.w;
      __builtin_amdgcn_wave_barrier();
      return;
    }
#endif
    const uint64_t c1 = nch - c0 < kWinChunks ? nch : c0 + kWinChunks;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t pe[4], po[4], te = 0, to = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t ev = 0, od = 0;
      acc_chunk(s_raw[wv][win_slot(4u * lane + uint32_t(j))], ev, od);
      pe[j] = te;
      po[j] = to;
      te += ev;
      to += od;
    }
    const uint32_t ie = wave_prefix_incl(te), io = wave_prefix_incl(to);
    const uint32_t xe = ce + ie - te, xo = co + io - to;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s_pre[wv][4u * lane + uint32_t(j)][0] = xe + pe[j];
      s_pre[wv][4u * lane + uint32_t(j)][1] = xo + po[j];
    }
    ce += __builtin_amdgcn_readlane(ie, 63);
    co += __builtin_amdgcn_readlane(io, 63);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (pc >= c0 && pc < c1) point_F(pc, pb, c0, fe, fo);  // (~0u: no point, past any window)
    if constexpr (TWO) {
      if (qc >= c0 && qc < c1) point_F(qc, qb, c0, ge, go);
    }
    __builtin_amdgcn_wave_barrier();  // the next window rewrites s_pre / s_raw
  };
  // wave-uniform; nwin3 >= kSets, so a do-while: no zero-trip test for the
  // compiler to sink the first three windows' loads behind
  uint64_t k = 0;
  do {
    window(k, b0);
    window(k + 1, b1);
    window(k + 2, b2);
    k += kSets;
  } while (k < nwin3);
  // a point at the aligned end of the last chunk: every byte is below it
  if (lane <= m && pc >= nch) {
    fe = ce;
    fo = co;
  }
  if constexpr (TWO) {
    if (valid && qc >= nch) {
      ge = ce;
      go = co;
    }
  } else {
    ge = fe;
    go = fo;
  }
  span_outputs<OP, OUT>(bytes, a, lane, valid, i, i0, m, x, e, lo, hdr, fe, fo, ge, go, w[0], w[1],
                        reinterpret_cast<uint32_t*>(&s_raw[wv][0]));
  __builtin_amdgcn_wave_barrier();  // the next span rewrites s_pre / s_raw
  };
  const uint64_t span0 = uint64_t(block_order(remap)) * kWaves + wv;
  if constexpr (STRIDE) {
    for (uint64_t span = span0; span < nspans; span += uint64_t(gridDim.x) * kWaves) span_body(span);
  } else if (span0 < nspans) {
    span_body(span0);
  }
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
  ICS_GRID_STRIDE(i, nvec) {
  const uint64_t a = spec_word(seed, w0 + 2 * i), b = spec_word(seed, w0 + 2 * i + 1);
  d[i] = u32x4{uint32_t(a), uint32_t(a >> 32), uint32_t(b), uint32_t(b >> 32)};
  }
}

__global__ void k_fill1(uint8_t* __restrict__ d, uint64_t n, uint64_t seed, uint64_t pos0) {
  ICS_GRID_STRIDE(j, n) {
    const uint64_t p = pos0 + j;
    d[j] = uint8_t(spec_word(seed, p >> 3) >> (8 * (p & 7)));
  }
}

__device__ __forceinline__ void spec_addrs(uint64_t seed, uint64_t i, uint32_t& src, uint32_t& dst) {
  const uint64_t m = spec_word(seed ^ 0xA5A5A5A5A5A5A5A5ull, i);
  src = 0x0A000000u | uint32_t(m & 0xFFFFFFu);
  dst = 0x0A000000u | uint32_t((m >> 24) & 0xFFFFFFu);
}

__global__ void k_pseudo_inits(uint32_t* __restrict__ init, const uint64_t* __restrict__ offsets,
                               uint64_t seg_len, uint64_t n, uint64_t seed, uint64_t index0) {
  ICS_GRID_STRIDE(i, n) {
  const uint64_t L = offsets ? offsets[i + 1] - offsets[i] : seg_len;
  uint32_t s, d;
  spec_addrs(seed, index0 + i, s, d);
  init[i] = (s >> 16) + (s & 0xffffu) + (d >> 16) + (d & 0xffffu) + 6u + uint32_t(L & 0xffffu);
  }
}

__global__ void k_ipv4_tcp_headers(uint8_t* __restrict__ dg, uint64_t stride, uint64_t dlen,
                                   uint64_t n, uint64_t seed, uint64_t index0) {
  ICS_GRID_STRIDE(i, n) {
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
}


// Pass 1: segments and bytes per bin, one partial per block (no same-address
// atomics: they serialise at a few ns each; no last-block reduction: its
// device-wide fence writes back L2 in every block); k_bin_plan adds them up.
__global__ __launch_bounds__(kBlock) void k_bin_stats(const uint64_t* __restrict__ off, uint64_t n,
                                                      uint32_t* __restrict__ cnt_part,
                                                      uint64_t* __restrict__ by_part) {
  uint32_t cnt[kBins] = {};
  uint64_t by[kBins] = {};
  // tiles of kBinTile segments; a thread's kBinPerThread offset pairs are all
  // requested before any is used
  for (uint64_t t0 = uint64_t(blockIdx.x) * kBinTile; t0 < n; t0 += uint64_t(gridDim.x) * kBinTile) {
    uint64_t a[kBinPerThread], z[kBinPerThread];
#pragma unroll
    for (int j = 0; j < kBinPerThread; ++j) {
      const uint64_t i = t0 + uint64_t(j) * kBlock + threadIdx.x;
      const uint64_t c = i < n ? i : n - 1;
      a[j] = off[c];
      z[j] = off[c + 1];
    }
#pragma unroll
    for (int j = 0; j < kBinPerThread; ++j) {
      const bool in = t0 + uint64_t(j) * kBlock + threadIdx.x < n;
      const uint64_t len = z[j] - a[j];
      const int b = bin_of(len);
#pragma unroll
      for (int k = 0; k < kBins; ++k) {
        cnt[k] += in && b == k;
        by[k] += in && b == k ? len : 0;
      }
    }
  }
  __shared__ uint32_t wc[kBlock / 64][kBins];
  __shared__ uint64_t wb[kBlock / 64][kBins];
  const uint32_t w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kBins; ++k) {
    uint32_t c = cnt[k];
    uint64_t v = by[k];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      c += __shfl_xor(c, d, 64);
      v += __shfl_xor(v, d, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      wc[w][k] = c;
      wb[w][k] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < kBins) {
    uint32_t c = 0;
    uint64_t v = 0;
#pragma unroll
    for (uint32_t q = 0; q < kBlock / 64; ++q) {
      c += wc[q][threadIdx.x];
      v += wb[q][threadIdx.x];
    }
    cnt_part[threadIdx.x * gridDim.x + blockIdx.x] = c;
    by_part[threadIdx.x * gridDim.x + blockIdx.x] = v;
  }
}

// Pass 3 (split plan only): every tile reserves its slice of each bin with
// one atomic per bin (bin b's list holds its entries at list + b * n).
__global__ __launch_bounds__(kBlock) void k_bin_scatter(const uint64_t* __restrict__ off, uint64_t n,
                                                        uint32_t* __restrict__ meta,
                                                        u32x4* __restrict__ list) {
  if (meta[kBinMetaPlan] != kPlanSplit) return;  // whole-batch plans: no lists
  __shared__ uint32_t resv[kBins];
  for (uint64_t t0 = uint64_t(blockIdx.x) * kBinTile; t0 < n; t0 += uint64_t(gridDim.x) * kBinTile) {
    uint64_t s[kBinPerThread], len[kBinPerThread];
    int bin[kBinPerThread];
    uint64_t mine = 0;
#pragma unroll
    for (int j = 0; j < kBinPerThread; ++j) {
      const uint64_t i = t0 + uint64_t(j) * kBlock + threadIdx.x;
      bin[j] = -1;
      if (i < n) {
        s[j] = off[i];
        len[j] = off[i + 1] - s[j];
        bin[j] = bin_of(len[j]);
        mine += uint64_t(1) << (kBinField * bin[j]);
      }
    }
    uint64_t total;
    uint64_t excl = block_excl_scan(mine, total);
    if (threadIdx.x < kBins) {
      const uint32_t c = field(total, threadIdx.x);
      resv[threadIdx.x] = c ? atomicAdd(&meta[kBinMetaCursor + threadIdx.x], c) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kBinPerThread; ++j) {
      if (bin[j] < 0) continue;
      const int b = bin[j];
      const uint64_t pos = uint64_t(b) * n + resv[b] + field(excl, b);
      excl += uint64_t(1) << (kBinField * b);
      const uint64_t i = t0 + uint64_t(j) * kBlock + threadIdx.x;
      const uint32_t l = len[j] < kLongEntry ? uint32_t(len[j]) : kLongEntry;
      list[pos] = u32x4{uint32_t(s[j]), uint32_t(s[j] >> 32), l, uint32_t(i)};
    }
    __syncthreads();  // resv is reused by the next tile
  }
}

// The most 256-thread blocks one dispatch holds: HSA packets carry the grid
// in work-items as a uint32, so 2^24 blocks would be one work-item too many.
// The two-class launches (one block per 64 or 128 segments) refuse batches
// past it with hipErrorInvalidValue, and the dispatch falls back to a
// grid-stride launch (8-lane groups / the fused kernel).
constexpr uint64_t kMaxGridBlocks = (uint64_t(1) << 24) - 1;
constexpr uint64_t twoclass_blocks(uint64_t n, uint64_t spw) {  // 4 waves x spw segments per block
  return (n + (kBlock / 64) * spw - 1) / ((kBlock / 64) * spw);
}
static_assert(uint64_t(kBlock) * kMaxGridBlocks <= 0xFFFFFFFFull, "grid work-items fit a uint32");
// the boundary ADVICE r3 found: n in (2^31 - 128, 2^31] at 32 per wave (or
// (2^30 - 64, 2^30] at 16) needs 2^24 blocks and must be refused
static_assert(twoclass_blocks((uint64_t(1) << 31) - 127, 32) > kMaxGridBlocks &&
                  twoclass_blocks((uint64_t(1) << 31) - 128, 32) == kMaxGridBlocks &&
                  twoclass_blocks((uint64_t(1) << 30) - 63, 16) > kMaxGridBlocks &&
                  twoclass_blocks((uint64_t(1) << 30) - 64, 16) == kMaxGridBlocks,
              "two-class grids: the largest batches that still fit");

// element-wise grid: at most 64K blocks (16M work-items), grid-stride beyond
inline uint32_t ew_blocks(uint64_t n) {
  const uint64_t b = (n + kBlock - 1) / kBlock;
  return uint32_t(b == 0 ? 1 : (b < 65536 ? b : 65536));
}

inline uint32_t blocks_for(uint64_t groups, uint32_t groups_per_block, uint32_t max_blocks) {
  uint64_t b = (groups + groups_per_block - 1) / groups_per_block;
  if (b == 0) b = 1;
  // cap keeps blocks * 256 work-items far below the uint32 AQL grid limit;
  // the kernels grid-stride over the remaining segments
  const uint64_t cap = max_blocks ? max_blocks : (uint64_t(1) << 22);
  return uint32_t(b < cap ? b : cap);
}

uint32_t g_xcd_remap = 10;  // log2 of the XCD run length of block_order (1024 blocks); 0: hardware order

inline SegSrc src_of(const SegSpec& sp) {
  return SegSrc{sp.offsets, sp.stride, sp.seg_len, static_cast<const u32x4*>(sp.list), sp.meta, sp.bin};
}

template <int LPS, int UNROLL, bool NT, int MODE>
hipError_t launch_checksum_t(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                             int out_kind, uint32_t max_blocks, hipStream_t st) {
  const uint32_t blocks = blocks_for(sp.n, kBlock / LPS, max_blocks);
  const uint32_t* ip = init ? init : static_cast<const uint32_t*>(sp.zero16);
  const uint8_t* op = odd ? odd : static_cast<const uint8_t*>(sp.zero16);
  const uint32_t is = init ? 1u : 0u, os = odd ? 1u : 0u;
  if (out_kind == 0)
    hipLaunchKernelGGL((k_checksum<LPS, UNROLL, NT, MODE, 0>), dim3(blocks), dim3(kBlock), 0, st, sp.bytes,
                       src_of(sp), ip, is, op, os, out, sp.n, g_xcd_remap, static_cast<const u32x4*>(sp.zero16), sp.done);
  else
    hipLaunchKernelGGL((k_checksum<LPS, UNROLL, NT, MODE, 1>), dim3(blocks), dim3(kBlock), 0, st, sp.bytes,
                       src_of(sp), ip, is, op, os, out, sp.n, g_xcd_remap, static_cast<const u32x4*>(sp.zero16), sp.done);
  return hipGetLastError();
}

template <int LPS, int UNROLL, int SEGS>
hipError_t launch_checksum_small_t(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                                   int out_kind, uint32_t max_blocks, hipStream_t st) {
  const uint32_t blocks = blocks_for((sp.n + SEGS - 1) / SEGS, kBlock / LPS, max_blocks);
  const uint32_t* ip = init ? init : static_cast<const uint32_t*>(sp.zero16);
  const uint8_t* op = odd ? odd : static_cast<const uint8_t*>(sp.zero16);
  const uint32_t is = init ? 1u : 0u, os = odd ? 1u : 0u;
  const u32x4* z = static_cast<const u32x4*>(sp.zero16);
  if (out_kind == 0)
    hipLaunchKernelGGL((k_checksum_small<LPS, UNROLL, SEGS, 0>), dim3(blocks), dim3(kBlock), 0, st, sp.bytes,
                       src_of(sp), ip, is, op, os, z, out, sp.n, sp.done);
  else
    hipLaunchKernelGGL((k_checksum_small<LPS, UNROLL, SEGS, 1>), dim3(blocks), dim3(kBlock), 0, st, sp.bytes,
                       src_of(sp), ip, is, op, os, z, out, sp.n, sp.done);
  return hipGetLastError();
}

template <int LONG_LPS, int SPW>
hipError_t launch_twoclass_t(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out, int out_kind,
                             uint32_t remap, uint32_t lds_pad, hipStream_t st) {
  const uint64_t blocks = twoclass_blocks(sp.n, SPW);
  if (blocks == 0 || blocks > kMaxGridBlocks) return hipErrorInvalidValue;
  const uint32_t* ip = init ? init : static_cast<const uint32_t*>(sp.zero16);
  const uint8_t* op = odd ? odd : static_cast<const uint8_t*>(sp.zero16);
  const uint32_t is = init ? 1u : 0u, os = odd ? 1u : 0u;
  const u32x4* z = static_cast<const u32x4*>(sp.zero16);
  if (out_kind == 0)
    hipLaunchKernelGGL((k_checksum_twoclass<LONG_LPS, SPW, 0>), dim3(uint32_t(blocks)), dim3(kBlock), lds_pad, st,
                       sp.bytes, src_of(sp), ip, is, op, os, z, out, sp.n, remap);
  else
    hipLaunchKernelGGL((k_checksum_twoclass<LONG_LPS, SPW, 1>), dim3(uint32_t(blocks)), dim3(kBlock), lds_pad, st,
                       sp.bytes, src_of(sp), ip, is, op, os, z, out, sp.n, remap);
  return hipGetLastError();
}

hipError_t launch_checksum_tiny_t(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                                  int out_kind, uint32_t max_blocks, hipStream_t st) {
  const uint32_t blocks = blocks_for(sp.n, kBlock, max_blocks);
  const uint32_t* ip = init ? init : static_cast<const uint32_t*>(sp.zero16);
  const uint8_t* op = odd ? odd : static_cast<const uint8_t*>(sp.zero16);
  const uint32_t is = init ? 1u : 0u, os = odd ? 1u : 0u;
  const u32x4* z = static_cast<const u32x4*>(sp.zero16);
  if (out_kind == 0)
    hipLaunchKernelGGL(k_checksum_tiny<0>, dim3(blocks), dim3(kBlock), 0, st, sp.bytes, src_of(sp), ip, is, op, os,
                       z, out, sp.n, sp.done);
  else
    hipLaunchKernelGGL(k_checksum_tiny<1>, dim3(blocks), dim3(kBlock), 0, st, sp.bytes, src_of(sp), ip, is, op, os,
                       z, out, sp.n, sp.done);
  return hipGetLastError();
}

template <int LPS, int SEGS>
hipError_t launch_dense_t(const SegSpec& sp, const uint32_t* init, void* out, int out_kind, hipStream_t st) {
  const uint64_t segs_per_block = uint64_t(kBlock / LPS) * SEGS;
  const uint64_t blocks = (sp.n + segs_per_block - 1) / segs_per_block;
  if (blocks == 0 || blocks > (uint64_t(1) << 22)) return hipErrorInvalidValue;
  const u32x4* c = reinterpret_cast<const u32x4*>(sp.bytes);
#define ICS_DENSE(I, O) \
  hipLaunchKernelGGL((k_checksum_dense<LPS, SEGS, I, O>), dim3(uint32_t(blocks)), dim3(kBlock), 0, st, c, init, out, sp.n)
  if (init && out_kind == 0) ICS_DENSE(true, 0);
  else if (init) ICS_DENSE(true, 1);
  else if (out_kind == 0) ICS_DENSE(false, 0);
  else ICS_DENSE(false, 1);
#undef ICS_DENSE
  return hipGetLastError();
}

template <int LPS, int UNROLL, bool NT, int MODE>
hipError_t launch_ipv4_t(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck,
                         uint8_t* status, uint32_t max_blocks, hipStream_t st) {
  const uint32_t blocks = blocks_for(sp.n, kBlock / LPS, max_blocks);
  hipLaunchKernelGGL((k_ipv4_tcp<LPS, UNROLL, NT, MODE>), dim3(blocks), dim3(kBlock), 0, st,
                     const_cast<uint8_t*>(sp.bytes), sp.offsets, sp.stride, sp.seg_len, sp.n, mode,
                     ip_ck, tcp_ck, status, g_xcd_remap, static_cast<const uint8_t*>(sp.zero16), sp.done);
  return hipGetLastError();
}

template <int LPS, int UNROLL, bool NT, int MODE>
hipError_t launch_wrap_t(const SegSpec& sp, const TcpMsg* msgs, uint32_t* hdr_out, uint16_t* ip_ck,
                         uint16_t* tcp_ck, bool payload_only, uint32_t* sums, uint32_t max_blocks, hipStream_t st) {
  const uint32_t blocks = blocks_for(sp.n, kBlock / LPS, max_blocks);
  if (sums)
    hipLaunchKernelGGL((k_tcp_wrap<LPS, UNROLL, NT, MODE, true>), dim3(blocks), dim3(kBlock), 0, st,
                       const_cast<uint8_t*>(sp.bytes), sp.offsets, sp.stride, sp.seg_len, sp.n, msgs, hdr_out,
                       ip_ck, tcp_ck, g_xcd_remap, int(payload_only), sums, Done{});  // k_tcp_hdr completes
  else
    hipLaunchKernelGGL((k_tcp_wrap<LPS, UNROLL, NT, MODE, false>), dim3(blocks), dim3(kBlock), 0, st,
                       const_cast<uint8_t*>(sp.bytes), sp.offsets, sp.stride, sp.seg_len, sp.n, msgs, hdr_out,
                       ip_ck, tcp_ck, g_xcd_remap, int(payload_only), sums, sp.done);
  return hipGetLastError();
}

// k_span: one wave per S segments, four independent waves per block
template <int OP, int OUT>
hipError_t launch_span_t(const SegSpec& sp, const TileArgs& a, uint32_t S, hipStream_t st, uint32_t max_blocks) {
  if (!sp.offsets || sp.list || sp.n == 0 || S == 0 || S > kSpanSegs) return hipErrorInvalidValue;
  const uint64_t waves = (sp.n + S - 1) / S;
  const uint64_t blocks = (waves + kBlock / 64 - 1) / (kBlock / 64);
  const uint64_t cap = max_blocks && max_blocks < kMaxGridBlocks ? max_blocks : kMaxGridBlocks;
  uint8_t* const bytes = const_cast<uint8_t*>(sp.bytes);
  const u32x4* const z = static_cast<const u32x4*>(sp.zero16);
  if (blocks > cap)  // more spans than one grid: grid-stride
    hipLaunchKernelGGL((k_span<OP, OUT, true>), dim3(uint32_t(cap)), dim3(kBlock), 0, st, bytes,
                       sp.offsets, sp.n, S, a, g_xcd_remap, z);
  else
    hipLaunchKernelGGL((k_span<OP, OUT, false>), dim3(uint32_t(blocks)), dim3(kBlock), 0, st, bytes, sp.offsets,
                       sp.n, S, a, g_xcd_remap, z);
  return hipGetLastError();
}

}  // namespace

// Geometry choice from the (average) segment length, measured on MI355X
// (git 7692616:tools/sweep_geometry.py; profiles/r1_sweep_geometry.jsonl,
// r1_sweep_line_grid.jsonl, r1_sweep_small.jsonl).  Small segments
// (<= ~270 B): k_checksum_small with about one load slot per 16-byte chunk
// and 2 segments per lane group in flight (64 B = 4 lanes x 1 load x 2).
// From ~270 bytes up: the 128-byte-line grid with default-policy boundary
// loads first (mode 3, range_sums_line_primed; profiles/r1_sweep_primed.jsonl)
// with slots >= chunks + 8 so one step covers a segment (1500 B -> 16 lanes x
// 8 loads), and 64 x 8 (8 KiB per wave step) looping for long segments.
// Interior chunks stream non-temporally (read once).
//
// Round 2 (git 7692616:tools/sweep_geometry.py, profiles/r2_sweep_mtu.jsonl,
// r2_sweep_mid.jsonl; 1 M segments, GB/s of the best vs the round-1 pick):
// slots close above the chunks a line-anchored segment spans win — 1000 B
// (16,5) 7569 vs (16,8) 6577, 1040 B (16,5) 7526 vs 6394, 1200 B (16,6) 7571
// vs 7133, 2000 B (16,4) 7477 vs (32,4) 7107, 2500 B (32,8) 7486 vs 7359,
// 3000 B (32,8) 7416 vs 7294, 4096 B (64,8) 7561 vs 7324; 600/800 B keep
// (16,4), 1460/1500 B (16,8).
Geometry pick_geometry(uint64_t avg_len) {
  const uint64_t m = (avg_len + 15) / 16;  // 16-byte chunks of the payload
  if (avg_len <= kTinyMaxAvg) return {1, 4, false, kModeTiny, 1};  // one lane per segment (ACK-sized)
  if (m <= 5) return {4, 1, true, 2, 2};   // small-segment kernel, 2 segments per group in flight
  if (m <= 9) return {4, 2, true, 2, 2};
  if (m <= 17) return {8, 2, true, 2, 2};
  if (m <= 56) return {16, 4, true, 3, 1};
  if (m <= 69) return {16, 5, true, 3, 1};
  if (m <= 82) return {16, 6, true, 3, 1};
  if (m <= 120) return {16, 8, true, 3, 1};
  if (m <= 140) return {16, 4, true, 3, 1};
  if (m <= 220) return {32, 8, true, 3, 1};
  return {64, 8, true, 3, 1};
}

// every instantiated (LPS, UNROLL, NT, MODE) of k_checksum, k_ipv4_tcp and
// k_tcp_wrap: exactly the shapes the dispatch can reach — pick_geometry's line
// grids, the last bin's 32/64-lane launch, the fused kernel's 4/8-lane shapes of
// short datagrams (ipv4_geometry), its one-lane shape for ACK-sized datagrams
// (mode 0, default-policy loads) and the 8-lane groups of ACK + MTU mixes
#define ICS_GEOMETRIES(X)                                                                     \
  X(1, 4, false, 0) X(4, 1, true, 2) X(4, 2, true, 2) X(8, 2, true, 2) X(8, 8, true, 3)      \
  X(16, 4, true, 3) X(16, 5, true, 3) X(16, 6, true, 3) X(16, 7, true, 3) X(16, 8, true, 3) \
  X(32, 8, true, 3) X(64, 8, true, 3)

// small-segment kernel instantiations (LPS, UNROLL, SEGS); Geometry::segs > 1
#define ICS_SMALL_GEOMETRIES(X) X(4, 1, 2) X(4, 2, 2) X(8, 2, 2)

hipError_t launch_checksum(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                           int out_kind, Geometry g, uint32_t max_blocks, hipStream_t st) {
  if (g.mode == kModeTiny) return launch_checksum_tiny_t(sp, init, odd, out, out_kind, max_blocks, st);
  if (g.segs > 1) {
#define ICS_SMALL(L, U, K)                                                            \
  if (g.lps == L && g.unroll == U && g.segs == K)                                     \
    return launch_checksum_small_t<L, U, K>(sp, init, odd, out, out_kind, max_blocks, st);
    ICS_SMALL_GEOMETRIES(ICS_SMALL)
#undef ICS_SMALL
    return hipErrorInvalidValue;
  }
#define ICS_CASE(L, U, T, A)                                      \
  if (g.lps == L && g.unroll == U && g.nt == T && g.mode == A)                \
    return launch_checksum_t<L, U, T, A>(sp, init, odd, out, out_kind, max_blocks, st);
  ICS_GEOMETRIES(ICS_CASE)
#undef ICS_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_checksum_twoclass(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                                    int out_kind, int spw, uint32_t remap, hipStream_t st, uint32_t lds_pad) {
  if (sp.list) return hipErrorInvalidValue;
  if (spw == 32) return launch_twoclass_t<16, 32>(sp, init, odd, out, out_kind, remap, lds_pad, st);
  if (spw == 16) return launch_twoclass_t<16, 16>(sp, init, odd, out, out_kind, remap, lds_pad, st);
  if (spw == 8) return launch_twoclass_t<16, 8>(sp, init, odd, out, out_kind, remap, lds_pad, st);
  return hipErrorInvalidValue;
}

bool dense_supported(const SegSpec& sp) {
  if (sp.offsets || sp.n == 0 || sp.stride != sp.seg_len) return false;
  if ((reinterpret_cast<uintptr_t>(sp.bytes) & 15) != 0) return false;
  return sp.seg_len == 32 || sp.seg_len == 64 || sp.seg_len == 128;
}

hipError_t launch_checksum_dense(const SegSpec& sp, const uint32_t* init, void* out, int out_kind, int segs,
                                 hipStream_t st) {
  if (!dense_supported(sp)) return hipErrorInvalidValue;
  const int lps = int(sp.seg_len / 16);
#define ICS_DENSE_CASE(L, K) \
  if (lps == L && segs == K) return launch_dense_t<L, K>(sp, init, out, out_kind, st);
  ICS_DENSE_CASE(2, 2) ICS_DENSE_CASE(2, 4) ICS_DENSE_CASE(2, 8)
  ICS_DENSE_CASE(4, 1) ICS_DENSE_CASE(4, 2) ICS_DENSE_CASE(4, 4) ICS_DENSE_CASE(4, 8)
  ICS_DENSE_CASE(8, 1) ICS_DENSE_CASE(8, 2) ICS_DENSE_CASE(8, 4)
#undef ICS_DENSE_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_bin_segments(const uint64_t* offsets, uint64_t n, void* list, uint32_t* meta, int force_plan,
                               uint32_t last_lps, uint64_t* plan_out, uint32_t gen, hipStream_t st) {
  if (!offsets || n == 0 || n > 0xFFFFFFFFull) return hipErrorInvalidValue;
  uint32_t* cnt_part = meta + kBinMetaWords;
  uint64_t* by_part = reinterpret_cast<uint64_t*>(cnt_part + kBins * kBinStatBlocks);
  const uint64_t tiles = (n + kBinTile - 1) / kBinTile;
  const uint32_t parts = uint32_t(tiles < kBinStatBlocks ? tiles : kBinStatBlocks);
  hipLaunchKernelGGL(k_bin_stats, dim3(parts), dim3(kBlock), 0, st, offsets, n, cnt_part, by_part);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(k_bin_plan, dim3(1), dim3(kBlock), 0, st, meta, cnt_part, by_part, parts, n, force_plan,
                     last_lps, plan_out, gen);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(k_bin_scatter, dim3(uint32_t(tiles < 2048 ? tiles : 2048)), dim3(kBlock), 0, st,
                     offsets, n, meta, static_cast<u32x4*>(list));
  return hipGetLastError();
}

hipError_t launch_bin_plan(const uint64_t* offsets, uint64_t n, uint32_t* meta, uint32_t last_lps,
                           uint64_t* plan_out, uint32_t gen, hipStream_t st) {
  if (!offsets || n == 0 || n > 0xFFFFFFFFull) return hipErrorInvalidValue;
  uint32_t* cnt_part = meta + kBinMetaWords;
  uint64_t* by_part = reinterpret_cast<uint64_t*>(cnt_part + kBins * kBinStatBlocks);
  const uint64_t tiles = (n + kBinTile - 1) / kBinTile;
  const uint32_t parts = uint32_t(tiles < kBinStatBlocks ? tiles : kBinStatBlocks);
  hipLaunchKernelGGL(k_bin_stats, dim3(parts), dim3(kBlock), 0, st, offsets, n, cnt_part, by_part);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(k_bin_plan, dim3(1), dim3(kBlock), 0, st, meta, cnt_part, by_part, parts, n, -1, last_lps,
                     plan_out, gen);
  return hipGetLastError();
}

// geometries k_checksum_bins hard-codes for bins 0..kBins-2
constexpr Geometry kBinGeometry[kBins - 1] = {{4, 2, true, 2, 2}, {16, 4, true, 3, 1}, {16, 8, true, 3, 1},
                                              {32, 4, true, 3, 1}};

hipError_t launch_checksum_bins(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                                int out_kind, uint32_t blocks_per_bin, hipStream_t st) {
  for (int b = 0; b < kBins - 1; ++b) {  // the table must agree with bin_geometry
    const Geometry g = bin_geometry(b), h = kBinGeometry[b];
    if (g.lps != h.lps || g.unroll != h.unroll || g.nt != h.nt || g.mode != h.mode || g.segs != h.segs)
      return hipErrorInvalidValue;
  }
  if (!sp.list || blocks_per_bin == 0) return hipErrorInvalidValue;
  if (blocks_per_bin > (1u << 20)) blocks_per_bin = 1u << 20;  // grid work-items stay < 2^32
  const uint32_t* ip = init ? init : static_cast<const uint32_t*>(sp.zero16);
  const uint8_t* op = odd ? odd : static_cast<const uint8_t*>(sp.zero16);
  const uint32_t is = init ? 1u : 0u, os = odd ? 1u : 0u;
  const u32x4* z = static_cast<const u32x4*>(sp.zero16);
  const dim3 grid(blocks_per_bin * (kBins - 1));
  if (out_kind == 0)
    hipLaunchKernelGGL(k_checksum_bins<0>, grid, dim3(kBlock), 0, st, sp.bytes, src_of(sp), ip, is, op, os, z,
                       out, sp.n, blocks_per_bin);
  else
    hipLaunchKernelGGL(k_checksum_bins<1>, grid, dim3(kBlock), 0, st, sp.bytes, src_of(sp), ip, is, op, os, z,
                       out, sp.n, blocks_per_bin);
  return hipGetLastError();
}

void set_xcd_remap(uint32_t run_log2) { g_xcd_remap = run_log2 < 31 ? run_log2 : 31; }

bool bounds_checked_build() {
#ifdef ICSUM_BOUNDS_CHECK
  return true;
#else
  return false;
#endif
}

hipError_t bounds_take(hipStream_t st, uint32_t* flags, uint64_t* what) {
  *flags = 0;
  *what = 0;
#ifdef ICSUM_BOUNDS_CHECK
  BoundsState b{};
  if (hipError_t e = hipStreamSynchronize(st)) return e;
  if (hipError_t e = hipMemcpyFromSymbol(&b, HIP_SYMBOL(g_icsum_bounds), sizeof b)) return e;
  if (b.flags) {
    const BoundsState z{};
    if (hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_icsum_bounds), &z, sizeof z)) return e;
  }
  *flags = b.flags;
  *what = b.addr;
#else
  (void)st;
#endif
  return hipSuccess;
}

Geometry bin_geometry(int bin) {
  // bins 0..kBins-2: the geometries k_checksum_bins hard-codes (kBinGeometry,
  // chosen by the round-1 binning A/B); the last bin: a long segment
  return bin < kBins - 1 ? kBinGeometry[bin] : pick_geometry(uint64_t(1) << 16);
}

SegSpec bin_spec(const SegSpec& whole, const void* list, const uint32_t* meta, int bin) {
  SegSpec sp = whole;
  sp.list = static_cast<const u32x4*>(list) + uint64_t(bin) * whole.n;
  sp.meta = meta;
  sp.bin = bin;
  return sp;
}

hipError_t launch_ipv4_tcp(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck,
                           uint8_t* status, Geometry g, uint32_t max_blocks, hipStream_t st) {
#define ICS_CASE(L, U, T, A)                                      \
  if (g.lps == L && g.unroll == U && g.nt == T && g.mode == A)                \
    return launch_ipv4_t<L, U, T, A>(sp, mode, ip_ck, tcp_ck, status, max_blocks, st);
  ICS_GEOMETRIES(ICS_CASE)
#undef ICS_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_ipv4_twoclass(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status,
                                int spw, uint32_t remap, hipStream_t st, uint32_t lds_pad) {
  if (spw != 8 && spw != 16 && spw != 32) return hipErrorInvalidValue;
  const uint64_t blocks = twoclass_blocks(sp.n, uint64_t(spw));
  if (sp.list || blocks == 0 || blocks > kMaxGridBlocks) return hipErrorInvalidValue;
  uint8_t* const dg = const_cast<uint8_t*>(sp.bytes);
  const uint8_t* const z = static_cast<const uint8_t*>(sp.zero16);
  if (mode < 0 || mode > 2) return hipErrorInvalidValue;
#define ICS_TWO(W, M)                                                                                        \
  hipLaunchKernelGGL((k_ipv4_twoclass<W, M>), dim3(uint32_t(blocks)), dim3(kBlock), lds_pad, st, dg, sp.offsets, \
                     sp.stride, sp.seg_len, sp.n, mode, ip_ck, tcp_ck, status, z, remap)
#define ICS_TWO_M(W) \
  if (mode == 0) ICS_TWO(W, 0); else if (mode == 1) ICS_TWO(W, 1); else ICS_TWO(W, 2)
  if (spw == 8) { ICS_TWO_M(8); }
  else if (spw == 16) { ICS_TWO_M(16); }
  else { ICS_TWO_M(32); }
#undef ICS_TWO_M
#undef ICS_TWO
  return hipGetLastError();
}

hipError_t launch_tcp_wrap(const SegSpec& sp, const TcpMsg* msgs, uint32_t* hdr_out, uint16_t* ip_ck,
                           uint16_t* tcp_ck, bool payload_only, uint32_t* sums, Geometry g, uint32_t max_blocks,
                           hipStream_t st) {
  if (sp.n == 0) return hipSuccess;
  if (payload_only && !hdr_out) return hipErrorInvalidValue;
  hipError_t e = hipErrorInvalidValue;
#define ICS_CASE(L, U, T, A)                                                                         \
  if (e == hipErrorInvalidValue && g.lps == L && g.unroll == U && g.nt == T && g.mode == A)        \
    e = launch_wrap_t<L, U, T, A>(sp, msgs, hdr_out, ip_ck, tcp_ck, payload_only, sums, max_blocks, st);
  ICS_GEOMETRIES(ICS_CASE)
#undef ICS_CASE
  if (e != hipSuccess || !sums) return e;
  return launch_tcp_hdr(sp, msgs, sums, hdr_out, ip_ck, tcp_ck, payload_only, st);
}

hipError_t launch_tcp_hdr(const SegSpec& sp, const TcpMsg* msgs, const uint32_t* sums, uint32_t* hdr_out,
                          uint16_t* ip_ck, uint16_t* tcp_ck, bool payload_only, hipStream_t st) {
  if (sp.n == 0) return hipSuccess;
  const uint64_t blocks = (sp.n + kBlock - 1) / kBlock;  // one datagram per lane
  hipLaunchKernelGGL(k_tcp_hdr, dim3(uint32_t(blocks < (uint64_t(1) << 22) ? blocks : (uint64_t(1) << 22))),
                     dim3(kBlock), 0, st, const_cast<uint8_t*>(sp.bytes), sp.offsets, sp.stride, sp.seg_len, sp.n,
                     msgs, sums, hdr_out, ip_ck, tcp_ck, int(payload_only), sp.done);
  return hipGetLastError();
}

hipError_t launch_tick(const uint8_t* bytes, const uint64_t* offsets, uint32_t n, int op, const uint32_t* init,
                       uint16_t* out, int mode, uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status,
                       const void* zero16, const Done& done, hipStream_t st) {
  if (n == 0 || n > kTickSegs || !bytes || !offsets) return hipErrorInvalidValue;
  TickOffsets t{};
  for (uint32_t j = 0; j <= n; ++j) t.o[j] = offsets[j];
  uint8_t* const b = const_cast<uint8_t*>(bytes);
  const uint32_t* ip = init ? init : static_cast<const uint32_t*>(zero16);
  const uint8_t* z = static_cast<const uint8_t*>(zero16);
  if (op == 0)
    hipLaunchKernelGGL(k_tick<0>, dim3(1), dim3(kBlock), 0, st, b, t, n, ip, init ? 1u : 0u, out, 0, nullptr, nullptr,
                       nullptr, z, done);
  else if (mode >= 0 && mode <= 2)
    hipLaunchKernelGGL(k_tick<1>, dim3(1), dim3(kBlock), 0, st, b, t, n, ip, 0u, nullptr, mode, ip_ck, tcp_ck, status,
                       z, done);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_tick_server(uint64_t* words, TickMailbox* mbs, uint32_t blocks, const void* zero16,
                              uint32_t idle_us, uint32_t pollers, hipStream_t st) {
  if (pollers < 1 || pollers > kBlock / 64 || blocks < 1 || blocks > kSrvBlocksMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_tick_server, dim3(blocks), dim3(kBlock), 0, st, words, mbs,
                     static_cast<const uint8_t*>(zero16), idle_us, pollers);
  return hipGetLastError();
}

hipError_t launch_tile_checksum(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out, int out_kind,
                                uint32_t S, hipStream_t st, uint32_t max_blocks) {
  TileArgs a{};
  a.init = init ? init : static_cast<const uint32_t*>(sp.zero16);
  a.odd = odd ? odd : static_cast<const uint8_t*>(sp.zero16);
  a.init_step = init ? 1u : 0u;
  a.odd_step = odd ? 1u : 0u;
  a.out = out;
  return out_kind == 0 ? launch_span_t<kTileSum, 0>(sp, a, S, st, max_blocks)
                       : launch_span_t<kTileSum, 1>(sp, a, S, st, max_blocks);
}

hipError_t launch_tile_ipv4(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status,
                            uint32_t S, hipStream_t st, uint32_t max_blocks) {
  TileArgs a{};
  a.mode = mode;
  a.ip_ck = ip_ck;
  a.tcp_ck = tcp_ck;
  a.status = status;
  return launch_span_t<kTileIpv4, 0>(sp, a, S, st, max_blocks);
}

hipError_t launch_tile_wrap(const SegSpec& sp, const TcpMsg* msgs, uint32_t* hdr_out, uint16_t* ip_ck,
                            uint16_t* tcp_ck, uint32_t S, hipStream_t st, uint32_t max_blocks) {
  TileArgs a{};
  a.msgs = msgs;
  a.hdr_out = hdr_out;
  a.ip_ck = ip_ck;
  a.tcp_ck = tcp_ck;
  return hdr_out ? launch_span_t<kTileWrapApart, 0>(sp, a, S, st, max_blocks)
                 : launch_span_t<kTileWrap, 0>(sp, a, S, st, max_blocks);
}

uint64_t batchv_blocks(int cls, uint64_t n) {
  // segments per block: dense 64 groups x 4 in flight, tiny 256 lanes,
  // small 64 groups x 2 in flight, line grids kBlock / lanes per segment
  const uint64_t per = cls == kBvDense64 || cls == kBvTiny || cls == kBvLane1 ? 256 : cls == kBvSmall ? 128
                       : cls == kBvLine16 ? 16 : 4;
  return (n + per - 1) / per;
}

namespace {
template <typename D>
bool bv_table(const D* b, int k, int cls, BvTable<D>& t, uint64_t& blocks) {
  if (k < 1 || k > kMaxBatchv) return false;
  t = {};
  t.k = uint32_t(k);
  blocks = 0;
  for (int j = k; j < kMaxBatchv; ++j) t.block0[j] = 0xFFFFFFFFu;  // no batch: never at or below a block
  for (int j = 0; j < k; ++j) {
    t.b[j] = b[j];
    const uint64_t nb = batchv_blocks(cls, b[j].n);
    if (nb == 0) return false;
    t.block0[j] = uint32_t(blocks);
    t.nblk[j] = uint32_t(nb);
    blocks += nb;
  }
  return blocks < (uint64_t(1) << 24);
}
}  // namespace

hipError_t launch_checksum_batchv(const BvSeg* b, int k, int cls, const void* zero16, hipStream_t st) {
  BvTable<BvSeg> t;
  uint64_t blocks = 0;
  if (!bv_table(b, k, cls, t, blocks)) return hipErrorInvalidValue;
  const u32x4* z = static_cast<const u32x4*>(zero16);
  const dim3 grid{uint32_t(blocks), 1, 1};
  switch (cls) {
    case kBvDense64: hipLaunchKernelGGL(k_checksum_batchv<kBvDense64>, grid, dim3(kBlock), 0, st, t, z, g_xcd_remap); break;
    case kBvTiny: hipLaunchKernelGGL(k_checksum_batchv<kBvTiny>, grid, dim3(kBlock), 0, st, t, z, g_xcd_remap); break;
    case kBvSmall: hipLaunchKernelGGL(k_checksum_batchv<kBvSmall>, grid, dim3(kBlock), 0, st, t, z, g_xcd_remap); break;
    case kBvLine16: hipLaunchKernelGGL(k_checksum_batchv<kBvLine16>, grid, dim3(kBlock), 0, st, t, z, g_xcd_remap); break;
    case kBvLine64: hipLaunchKernelGGL(k_checksum_batchv<kBvLine64>, grid, dim3(kBlock), 0, st, t, z, g_xcd_remap); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_ipv4_batchv(const BvDgram* b, int k, int cls, int mode, const void* zero16, hipStream_t st) {
  BvTable<BvDgram> t;
  uint64_t blocks = 0;
  if (!bv_table(b, k, cls, t, blocks)) return hipErrorInvalidValue;
  const uint8_t* z = static_cast<const uint8_t*>(zero16);
  const dim3 grid{uint32_t(blocks), 1, 1};
  switch (cls) {
    case kBvLane1: hipLaunchKernelGGL(k_ipv4_batchv<kBvLane1>, grid, dim3(kBlock), 0, st, t, mode, z, g_xcd_remap); break;
    case kBvLine16: hipLaunchKernelGGL(k_ipv4_batchv<kBvLine16>, grid, dim3(kBlock), 0, st, t, mode, z, g_xcd_remap); break;
    case kBvLine64: hipLaunchKernelGGL(k_ipv4_batchv<kBvLine64>, grid, dim3(kBlock), 0, st, t, mode, z, g_xcd_remap); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

bool geometry_supported(Geometry g) {
  if (g.mode == kModeTiny) return g.lps == 1 && g.segs == 1;
  if (g.segs > 1) {
#define ICS_SMALL(L, U, K) \
  if (g.lps == L && g.unroll == U && g.segs == K) return true;
    ICS_SMALL_GEOMETRIES(ICS_SMALL)
#undef ICS_SMALL
    return false;
  }
#define ICS_CASE(L, U, T, A) \
  if (g.lps == L && g.unroll == U && g.nt == T && g.mode == A) return true;
  ICS_GEOMETRIES(ICS_CASE)
#undef ICS_CASE
  return false;
}

hipError_t launch_fold(const uint32_t* sum, uint16_t* out, uint64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_fold, dim3(ew_blocks(n)), dim3(kBlock), 0, st, sum, out, n);
  return hipGetLastError();
}

hipError_t launch_router_hdrs(const SegSpec& sp, uint32_t* hdr_out, uint8_t* status, hipStream_t st) {
  hipLaunchKernelGGL(k_router_hdrs, dim3(ew_blocks(sp.n * 2)), dim3(kBlock), 0, st, sp.bytes, sp.offsets, sp.stride,
                     sp.seg_len, sp.n, hdr_out, status, static_cast<const uint32_t*>(sp.zero16));
  return hipGetLastError();
}

hipError_t launch_router_ttl(const SegSpec& sp, uint8_t* status, hipStream_t st) {
  hipLaunchKernelGGL(k_router_ttl, dim3(ew_blocks(sp.n * 2)), dim3(kBlock), 0, st,
                     const_cast<uint8_t*>(sp.bytes), sp.offsets, sp.stride, sp.seg_len, sp.n, status,
                     static_cast<const uint32_t*>(sp.zero16));
  return hipGetLastError();
}

hipError_t launch_fill_bytes(uint8_t* d, uint64_t nbytes, uint64_t seed, uint64_t pos0,
                             hipStream_t st) {
  if (nbytes == 0) return hipSuccess;
  if ((pos0 & 7) == 0 && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    const uint64_t nvec = nbytes / 16;
    if (nvec) {
      hipLaunchKernelGGL(k_fill16, dim3(ew_blocks(nvec)), dim3(kBlock), 0, st,
                         reinterpret_cast<u32x4*>(d), nvec, seed, pos0 >> 3);
    }
    const uint64_t done = nvec * 16, rest = nbytes - done;
    if (rest)
      hipLaunchKernelGGL(k_fill1, dim3(1), dim3(kBlock), 0, st, d + done, rest, seed, pos0 + done);
  } else {
    hipLaunchKernelGGL(k_fill1, dim3(ew_blocks(nbytes)), dim3(kBlock), 0, st, d, nbytes, seed, pos0);
  }
  return hipGetLastError();
}

hipError_t launch_pseudo_inits(uint32_t* init, const uint64_t* offsets, uint64_t seg_len,
                               uint64_t n, uint64_t seed, uint64_t index0, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pseudo_inits, dim3(ew_blocks(n)), dim3(kBlock), 0, st,
                     init, offsets, seg_len, n, seed, index0);
  return hipGetLastError();
}

hipError_t launch_ipv4_tcp_headers(uint8_t* d, uint64_t stride, uint64_t dgram_len, uint64_t n,
                                   uint64_t seed, uint64_t index0, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ipv4_tcp_headers, dim3(ew_blocks(n)), dim3(kBlock), 0,
                     st, d, stride, dgram_len, n, seed, index0);
  return hipGetLastError();
}

}  // namespace icsum
