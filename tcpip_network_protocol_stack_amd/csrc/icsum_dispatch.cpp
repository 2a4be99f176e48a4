// icsum_dispatch.cpp — device-buffer dispatch behind the C-ABI (icsum_api.cpp):
// which kernel and geometry runs a batch, the plan cache that remembers the
// device's view of an offsets batch's length mix, the binned launches, the
// device wrap's one- or two-pass choice and the multi-batch grouping.  All
// arithmetic happens in the HIP kernels (kernels/icsum_kernels.hip).
#include <algorithm>
#include <string>
#include <vector>

#include "icsum_ctx.h"

namespace icsum::detail {

static_assert(icsum::kBvDense64 == ICS_BV_DENSE64 && icsum::kBvTiny == ICS_BV_TINY && icsum::kBvSmall == ICS_BV_SMALL &&
                  icsum::kBvLine16 == ICS_BV_LINE16 && icsum::kBvLine64 == ICS_BV_LINE64 &&
                  icsum::kBvLane1 == ICS_BV_LANE1,
              "multi-batch shapes are reported as ICS_BV_*");

// Segments per k_span wave: the forced value; with the cached plan's mean
// length (capped at 4095 by the plan), about ics_ctx::kSpanBytes of segments
// per span, 1..63 (a wave streams its span alone: spans of long segments
// leave the chip a few long-lived waves); without one, 63.  Measured
// (tools/ab_stream.py; profiles/r5n_ab_span_size.jsonl,
// r5o_ab_span_size_fine.jsonl; us back to back, S = 4 / 16 / 32 / 63): 1 M
// x 40..1040 B checksum 236.3 / 89.9 / 83.9 / 91.2, VERIFY 315.7 / 122.3 /
// 111.6 / 122.2; 1 M x 770 B checksum 250.4 / 129.1 / 118.4 / 123.1;
// 128 Ki of config 4's 64 B..64 KiB mix VERIFY 191.5 / 209.3 / 221.1 /
// 265.9 — flat from about 16 to 40 KiB per span.
uint32_t span_segs_for(const ics_ctx* ctx, uint32_t avg) {
  if (ctx->span_segs) return ctx->span_segs;
  if (avg == 0) return 63;
  return uint32_t(std::clamp<uint64_t>(ics_ctx::kSpanBytes / avg, 1, 63));
}

bool wrap_two_pass(const ics_ctx* ctx, bool headers_apart, uint64_t n) {
  return ctx->wrap_passes == 2 || (ctx->wrap_passes == 0 && headers_apart && n >= ics_ctx::kWrapTwoPassMin);
}

icsum::Geometry geometry_for(const ics_ctx* ctx, uint64_t avg_len) {
  icsum::Geometry g = icsum::pick_geometry(avg_len);
  if (ctx->force_lps) g = {ctx->force_lps, ctx->force_unroll ? ctx->force_unroll : g.unroll, g.nt, g.mode, 1};
  if (ctx->force_mode >= 0) g.mode = ctx->force_mode;
  if (ctx->force_segs > 0) g.segs = ctx->force_segs;
  if (!icsum::geometry_supported(g)) g.nt = !g.nt;  // a forced shape exists with one load policy
  if (!icsum::geometry_supported(g)) g = icsum::pick_geometry(avg_len);
  return g;
}

// the fused IPv4 kernel has no small-segment (multi-segment) variant: use the
// one-segment kernel of the same lane shape
icsum::Geometry ipv4_geometry(icsum::Geometry g) {
  g.segs = 1;
  if (g.mode == icsum::kModeTiny) g = {4, 1, true, 2, 1};  // the tiny kernel is checksum-only
  if (!icsum::geometry_supported(g)) g = {16, 8, true, 3, 1};
  return g;
}

// Fixed-length datagrams of at most 1664 bytes on the 16 x 8 line grid: 7
// loads per lane still cover the span (<= 111 chunks with the line's head) in
// one pass, and the fused kernel drops from 82 to 76 VGPRs (5 -> 6 waves /
// SIMD): config 2 COMPUTE / PATCH / VERIFY 16.88 / 20.88 / 16.73 -> 16.74 /
// 20.68 / 16.58 us (profiles/r4_ab_ipv4_unroll7.jsonl).  The plain checksum
// keeps 8 (already 8 waves; 1 M x 1500 B 209.2 vs 211.2 us at 7).
icsum::Geometry ipv4_fixed_geometry(const ics_ctx* ctx, icsum::Geometry g, uint64_t len) {
  const bool forced = ctx->force_lps || ctx->force_unroll || ctx->force_mode >= 0 || ctx->force_segs;
  if (!forced && g.lps == 16 && g.unroll == 8 && g.mode == 3 && len > 0 && len <= 1664) g.unroll = 7;
  return g;
}

namespace {

// average segment length for the geometry choice without reading d_offsets
uint64_t avg_len_hint(const uint64_t* offsets, uint64_t seg_len) {
  return offsets ? 65536 : seg_len;  // unknown mix: the long-segment geometry
}

bool forced_geometry(const ics_ctx* ctx) {
  return ctx->force_lps || ctx->force_unroll || ctx->force_mode >= 0 || ctx->force_segs;
}

// diagnostics: the last call's main launch (ics_dispatch_info)
void note(ics_ctx* ctx, int kernel, icsum::Geometry g = {0, 0, true, 0, 1}, int plan = -1) {
  ctx->last_kernel.store(kernel, std::memory_order_relaxed);
  ctx->last_lps.store(g.lps, std::memory_order_relaxed);
  ctx->last_unroll.store(g.unroll, std::memory_order_relaxed);
  ctx->last_plan.store(plan, std::memory_order_relaxed);
}

int kernel_of(icsum::Geometry g) {
  return g.mode == icsum::kModeTiny ? ICS_K_TINY : g.segs > 1 ? ICS_K_SMALL : ICS_K_CHECKSUM;
}

// a1-a4 on device buffers.  An offsets batch of unknown length mix is split
// into length bins on the device (two passes over the offsets), and every bin
// runs with the geometry that suits its lengths; the bin lists live in
// stream-ordered scratch, so concurrent calls on different streams are safe.
//
// The plan cache (ics_ctx::plan_slot): a lookup finds the slot keyed by this
// batch's (offsets pointer, n) and trusts its word only when the word carries
// the slot's generation — i.e. it was written by a plan kernel this key's
// miss (or refresh) queued, and has landed.  any_plan = false accepts only
// the whole-batch plans.  The mix receives the shares k_bin_plan reported, in
// sixteenths: segments of <= 144 bytes, and bytes in segments over 1920
// bytes.  A miss (re)keys the least recently used slot; *want_plan asks the
// caller to queue the plan kernels (into *plan_dst, with *plan_gen) behind its
// launch: on a miss, on every kPlanRefresh-th hit, and every kPlanRefresh-th
// lookup of a key whose plan has not landed yet.
struct PlanMix {
  uint32_t short16 = 0, long16 = 0, avg = 0;  // avg: mean segment length, bytes (capped at 4095)
};
struct PlanReq {
  bool want = false;
  uint64_t* dst = nullptr;  // device view of the slot's word
  uint32_t gen = 0;
};
bool plan_lookup(ics_ctx* ctx, const icsum::SegSpec& sp, bool any_plan, uint32_t* plan, PlanReq* req,
                 PlanMix* mix = nullptr) {
  *req = {};
  if (!ctx->plan_host) return false;
  std::lock_guard<std::mutex> lock(ctx->plan_mu);
  int k = -1, lru = 0;
  for (int i = 0; i < ics_ctx::kPlanSlots; ++i) {
    const ics_ctx::PlanSlot& ps = ctx->plan_slot[i];
    if (ps.key == sp.offsets && ps.n == sp.n && ps.gen) k = i;
    if (ps.used < ctx->plan_slot[lru].used) lru = i;
  }
  if (k >= 0) {
    ics_ctx::PlanSlot& ps = ctx->plan_slot[k];
    ps.used = ++ctx->plan_clock;
    const uint64_t v = __atomic_load_n(ctx->plan_host + k, __ATOMIC_ACQUIRE);
    const uint32_t p = uint32_t(v & 0xfu);
    const bool landed = (v >> 56) == ps.gen && ((v >> 8) & 0xFFFFFFFFull) == (sp.n & 0xFFFFFFFFull);
    const bool whole = p == icsum::kPlanWholeBatch || p == icsum::kPlanWholeBatch16 || p == icsum::kPlanWholeBatchSmall;
    const bool again = ++ps.hits % ics_ctx::kPlanRefresh == 0;
    *req = {again, ctx->plan_host_dev + k, ps.gen};
    if (landed && (whole || any_plan)) {
      if (mix) *mix = {uint32_t(v >> 4) & 0xfu, uint32_t(v >> 40) & 0xfu, uint32_t(v >> 44) & 0xfffu};
      *plan = p;
      ctx->n_hits.fetch_add(1, std::memory_order_relaxed);
      return true;
    }
    ctx->n_misses.fetch_add(1, std::memory_order_relaxed);
    return false;
  }
  ics_ctx::PlanSlot& ps = ctx->plan_slot[lru];
  ctx->plan_gen = ctx->plan_gen % 254 + 1;  // 1..254: never the 0xFF of an unwritten word
  ps = {sp.offsets, sp.n, ctx->plan_gen, 0, ++ctx->plan_clock};
  __atomic_store_n(ctx->plan_host + lru, ~uint64_t(0), __ATOMIC_RELEASE);
  *req = {true, ctx->plan_host_dev + lru, ps.gen};
  ctx->n_misses.fetch_add(1, std::memory_order_relaxed);
  return false;
}

// stats + plan kernels only (no lists) behind a launch: the plan for the next
// call with the same offsets lands in the slot plan_lookup named
int replan(ics_ctx* ctx, const icsum::SegSpec& sp, uint32_t lps, const PlanReq& req, hipStream_t st) {
  if (!req.want) return ICS_OK;
  Scratch meta(ctx, (icsum::kBinMetaBytesTotal + 255) & ~size_t(255), st);
  ICS_HIP(meta.error());
  ICS_HIP(icsum::launch_bin_plan(sp.offsets, sp.n, static_cast<uint32_t*>(meta.get()), lps, req.dst, req.gen, st));
  ctx->n_replans.fetch_add(1, std::memory_order_relaxed);
  return ICS_OK;
}

// a batch of many short segments with (almost) no bytes in long ones: from
// kShortMix16 sixteenths of <= 144-byte segments and under 1/16 of the bytes
// in segments over 1920 bytes, one launch beats the binned launches and
// 16-lane groups — first 8-lane groups (1 M datagrams, 50 % / 75 % 40-byte
// ACKs + 1500 B: 139.5 / 107.4 us vs 146.0 / 125.6 us AUTO;
// profiles/r2_csum_mix_sweep.jsonl), now the two-class launch (launch_mix)
bool short_mix(const PlanMix& m) { return m.short16 >= ics_ctx::kShortMix16 && m.long16 == 0; }

// The tile launch (k_span) for an offsets batch whose device-reported mix
// favours it: from kTileMin segments, a mean length of at most kTileMaxAvg
// bytes (variable lengths leave per-segment lane groups idle), or — for the
// wraps, which have no length binning — a sixteenth or more of the bytes in
// segments over 1920 bytes; the fused IPv4 kernel on every mix but the
// short-heavy ones (ipv4_device).  Short-heavy mixes keep the two-class
// launches (checked first by the callers), MTU-sized means the 16-lane line
// grid.  tools/ab_stream.py, profiles/r5l_ab_span_vs_per_segment.jsonl,
// r5m_ab_c4.jsonl, r5p_ab_span_thresholds.jsonl (us back to back,
// per-segment vs span): checksum 40..1040 B 256 Ki / 1 M 35.7 / 27.0 and
// 286.7 / 89.3, 770 B 1 M 153.0 / 122.8, MTU 1 M 212.2 / 236.8, 64 Ki 11.1 /
// 11.3; VERIFY 40..1040 B 64 Ki / 1 M 16.1 / 11.9 and 204.9 / 123.5, MTU
// 256 Ki / 1 M 70.4 / 61.3 and 264.6 / 237.6, 128 Ki of config 4's mix
// 233.5 / 192.3; headers-apart wrap 40..1040 B 64 Ki / 1 M 11.7 / 9.8 and
// 137.4 / 103.4, MTU 1 M 244.8 / 265.2; in-place wrap 40..1040 B 1 M 156.9 /
// 156.3, 770 B 1 M 193.2 / 207.2, config 4's mix 265.6 / 230.6.
// The plain checksum keeps the per-segment launches up to kTileMinChecksum
// (64 Ki 40..1040 B: 11.1 us per segment vs 11.3 us span above); VERIFY and
// the headers-apart wrap already win at 64 Ki (16.1 / 11.9, 11.7 / 9.8 us).
bool tile_wins(const ics_ctx* ctx, const PlanMix& m, uint64_t n, bool fused) {
  if (ctx->tile == 0 || n < (fused ? ics_ctx::kTileMin : ics_ctx::kTileMinChecksum)) return false;
  return m.avg <= ics_ctx::kTileMaxAvg || (fused && m.long16 >= 4);
}

// a short-heavy mix's single launch: the two-class launch (ACK-sized segments
// one per lane, the rest 16 lanes each; block lists since round 3), 32
// segments per wave from 3/4 short segments up and 16 below (round 2, the
// per-wave version: fewer long segments per wave, shorter-lived waves).  2 M x 40 / 1460 B: 8-lane groups 279.5, two-class 64 / 32 / 16 per
// wave 255.7 / 234.9 / 231.1 us; raw-datagram mixes (git 7692616:tools/ab_ipv4_mix.py
// plain rows, 64 / 32 / 16): 7/8 ACKs 43.5 / 42.2 / 54.5, 3/4 74.8 / 68.5 /
// 74.5, 1/2 132.4 / 122.5 / 119.0, 7/16 145.0 / 139.3 / 131.9 us
// (profiles/r2_twoclass_spw*.jsonl).  Batches past the two-class grid's
// limit run 8-lane groups.
hipError_t launch_mix(ics_ctx* ctx, const icsum::SegSpec& sp, const uint32_t* d_init, const uint8_t* d_odd,
                      void* d_out, int out_kind, const PlanMix& mix, hipStream_t st) {
  const int spw = mix.short16 >= 12 ? 32 : 16;
  const hipError_t e = icsum::launch_checksum_twoclass(sp, d_init, d_odd, d_out, out_kind, spw, ctx->twoclass_remap, st, ctx->twoclass_lds);
  if (e != hipErrorInvalidValue) {
    note(ctx, ICS_K_TWOCLASS, {16, spw, true, 3, 1});
    return e;
  }
  note(ctx, ICS_K_CHECKSUM, {8, 8, true, 3, 1});
  return icsum::launch_checksum(sp, d_init, d_odd, d_out, out_kind, icsum::Geometry{8, 8, true, 3, 1}, 0, st);
}

// the small-segment plan's single launch: one lane per segment for ACK-sized
// means (icsum::kTinyMaxAvg), else 4-lane groups with 2 segments in flight
icsum::Geometry small_plan_geometry(const PlanMix& m) {
  return m.avg <= icsum::kTinyMaxAvg ? icsum::Geometry{1, 4, false, icsum::kModeTiny, 1}
                                     : icsum::Geometry{4, 2, true, 2, 2};
}

}  // namespace

int checksum_device(ics_ctx* ctx, const icsum::SegSpec& sp, const uint32_t* d_init, const uint8_t* d_odd,
                    void* d_out, int out_kind, hipStream_t st) {
  if (sp.offsets && ctx->twoclass) {  // test hook: the two-class launch on every offsets batch
    ICS_HIP(icsum::launch_checksum_twoclass(sp, d_init, d_odd, d_out, out_kind, ctx->twoclass, ctx->twoclass_remap, st, ctx->twoclass_lds));
    note(ctx, ICS_K_TWOCLASS, {16, ctx->twoclass, true, 3, 1});
    return ICS_OK;
  }
  if (sp.offsets && ctx->tile == 1) {  // test hook: the tile launch on every offsets batch
    const uint32_t S = span_segs_for(ctx, 0);
    ICS_HIP(icsum::launch_tile_checksum(sp, d_init, d_odd, d_out, out_kind, S, st, ctx->span_blocks));
    note(ctx, ICS_K_TILE, {int(S), ICS_TILE_CHECKSUM, true, 0, 1});
    return ICS_OK;
  }
  const bool binned = sp.offsets && sp.n <= 0xFFFFFFFFull &&
                      (ctx->bin == 1 || (ctx->bin < 0 && sp.n >= ctx->bin_min && !forced_geometry(ctx)));
  const bool plannable = ctx->bin < 0 && ctx->bin_plan < 0 && ctx->plan_host && sp.n <= 0xFFFFFFFFull;
  if (!binned && sp.offsets && plannable && !forced_geometry(ctx) && sp.n >= ics_ctx::kSmallPlanMin) {
    // an offsets batch below the binning threshold: one launch, its geometry
    // from the plan the device reported for this batch last time (16-lane
    // groups for MTU-sized mixes, the small-segment body for short ones);
    // on a miss the unknown-mix geometry, and the plan kernels run behind
    // the launch for the next call (git 7692616:tools/ab_small_offsets.py)
    uint32_t plan = 0;
    PlanMix mix;
    PlanReq req;
    const bool hit = plan_lookup(ctx, sp, true, &plan, &req, &mix);
    icsum::Geometry g = geometry_for(ctx, avg_len_hint(sp.offsets, sp.seg_len));
    if (hit && plan == icsum::kPlanWholeBatch16) g = {16, 8, true, 3, 1};
    if (hit && plan == icsum::kPlanWholeBatchSmall) g = small_plan_geometry(mix);
    if (hit && plan != icsum::kPlanWholeBatchSmall && short_mix(mix)) {
      ICS_HIP(launch_mix(ctx, sp, d_init, d_odd, d_out, out_kind, mix, st));
    } else {
      ICS_HIP(icsum::launch_checksum(sp, d_init, d_odd, d_out, out_kind, g, 0, st));
      note(ctx, kernel_of(g), g, hit ? int(plan) : -1);
    }
    return replan(ctx, sp, 64, req, st);
  }
  if (!binned) {
    // dense fixed-stride batch of short segments (config 3): the flat-array kernel
    if (!d_odd && ctx->dense_segs > 0 && !forced_geometry(ctx) && icsum::dense_supported(sp)) {
      const hipError_t e = icsum::launch_checksum_dense(sp, d_init, d_out, out_kind, ctx->dense_segs, st);
      if (e != hipErrorInvalidValue) {
        ICS_HIP(e);
        note(ctx, ICS_K_DENSE, {int(sp.seg_len / 16), ctx->dense_segs, true, 0, 1});
        return ICS_OK;
      }
    }
    const icsum::Geometry g = geometry_for(ctx, avg_len_hint(sp.offsets, sp.seg_len));
    ICS_HIP(icsum::launch_checksum(sp, d_init, d_odd, d_out, out_kind, g, 0, st));
    note(ctx, kernel_of(g), g);
    return ICS_OK;
  }
  // the whole-batch plan's launch geometry: one lane group per segment of the
  // batch; above 1 M segments 32-lane groups halve the waves an empty last bin
  // costs to dispatch
  icsum::Geometry g_last = icsum::bin_geometry(icsum::kBins - 1);
  const uint32_t lps = ctx->last_bin_lps ? ctx->last_bin_lps : (sp.n > (uint64_t(1) << 20) ? 32u : 64u);
  if (lps == 32) g_last = {32, 8, true, 3, 1};
  PlanReq req;
  if (plannable) {
    uint32_t hit_plan = 0;
    PlanMix mix;
    const bool hit = plan_lookup(ctx, sp, true, &hit_plan, &req, &mix);
    const bool mix8 = hit && hit_plan != icsum::kPlanWholeBatchSmall && short_mix(mix);
    if (hit && !mix8 && hit_plan != icsum::kPlanWholeBatchSmall && tile_wins(ctx, mix, sp.n, false)) {
      const uint32_t S = span_segs_for(ctx, mix.avg);
      ICS_HIP(icsum::launch_tile_checksum(sp, d_init, d_odd, d_out, out_kind, S, st, ctx->span_blocks));
      note(ctx, ICS_K_TILE, {int(S), ICS_TILE_CHECKSUM, true, 0, 1}, int(hit_plan));
      return replan(ctx, sp, lps, req, st);
    }
    if (hit && (hit_plan != icsum::kPlanSplitBins || mix8)) {
      // the whole-batch plan the device chose for this batch last time, as
      // its single launch: the last bin's geometry (whole), 16-lane groups
      // (whole16) or the small-segment body (wholeS) over every segment; a
      // short-heavy mix with no long segments (received traffic: ACKs + MTU
      // data) runs the two-class launch whatever the plan (launch_mix)
      const icsum::Geometry g_hit = hit_plan == icsum::kPlanWholeBatch16      ? icsum::Geometry{16, 8, true, 3, 1}
                                    : hit_plan == icsum::kPlanWholeBatchSmall ? small_plan_geometry(mix)
                                                                              : g_last;
      if (mix8) {
        ICS_HIP(launch_mix(ctx, sp, d_init, d_odd, d_out, out_kind, mix, st));
      } else {
        ICS_HIP(icsum::launch_checksum(sp, d_init, d_odd, d_out, out_kind, g_hit,
                                       hit_plan == icsum::kPlanWholeBatch ? ctx->last_bin_blocks : 0, st));
        note(ctx, kernel_of(g_hit), g_hit, int(hit_plan));
      }
      // re-plan behind it: a batch whose mix changed under the same pointer
      // and size is re-binned from the next call on
      return replan(ctx, sp, lps, req, st);
    }
  }
  const size_t meta_bytes = (icsum::kBinMetaBytesTotal + 255) & ~size_t(255);
  Scratch ws(ctx, meta_bytes + sp.n * 16 * icsum::kBins, st);
  ICS_HIP(ws.error());
  uint32_t* meta = static_cast<uint32_t*>(ws.get());
  void* list = static_cast<uint8_t*>(ws.get()) + meta_bytes;
  // the binning passes; the plan kernel also reports into the plan cache's
  // slot when this call's lookup asked for a plan
  hipError_t e = icsum::launch_bin_segments(sp.offsets, sp.n, list, meta, ctx->bin_plan, lps,
                                            req.want ? req.dst : nullptr, req.gen, st);
  // bins 0..3: one launch, a capped grid striding over each bin; the last
  // bin: one lane group per segment of the batch (it takes the whole batch
  // under the whole-batch plans)
  if (e == hipSuccess)
    e = icsum::launch_checksum_bins(icsum::bin_spec(sp, list, meta, 0), d_init, d_odd, d_out, out_kind,
                                    ctx->bin_blocks, st);
  if (e == hipSuccess)
    e = icsum::launch_checksum(icsum::bin_spec(sp, list, meta, icsum::kBins - 1), d_init, d_odd, d_out, out_kind,
                               g_last, ctx->last_bin_blocks, st);
  ICS_HIP(e);
  if (req.want) ctx->n_replans.fetch_add(1, std::memory_order_relaxed);
  note(ctx, ICS_K_BINNED, g_last, ctx->bin_plan);
  return ICS_OK;
}

int ipv4_device(ics_ctx* ctx, const icsum::SegSpec& sp, int mode, uint16_t* d_ip_ck, uint16_t* d_tcp_ck,
                uint8_t* d_status, hipStream_t st) {
  const uint64_t* d_offsets = sp.offsets;
  const uint64_t n = sp.n;
  // an offsets batch of raw datagrams gives no length hint; datagrams are at
  // most 64 KiB and mostly MTU-sized, and the 16-lane line grid is the best
  // measured geometry for both 1500- and 9000-byte datagrams (64 Ki x 1500 B:
  // 18.3 us vs 48.8 us with the 64-lane default; git 7692616:tools/ab_ipv4_offsets.py)
  // ACK-sized datagrams (a fixed length <= kTinyMaxAvg, or a cached plan
  // whose mean is) run one lane per datagram with default-policy loads
  // (neighbours share lines): 1 M x 40 B VERIFY 30.3 -> 10.6 us (git 7692616:tools/ab_ipv4_mix.py, AB_LANE1)
  const icsum::Geometry lane1{1, 4, false, 0, 1};
  const icsum::Geometry base = geometry_for(ctx, d_offsets ? 1500 : sp.seg_len);
  icsum::Geometry g = base.mode == icsum::kModeTiny ? lane1 : ipv4_geometry(base);
  if (!d_offsets) g = ipv4_fixed_geometry(ctx, g, sp.seg_len);
  // a receive batch of mostly short datagrams (pure ACKs: 40 bytes) leaves
  // most of a 16-lane group idle: from 16 Ki datagrams up the geometry
  // follows the plan the device reported for the same offsets buffer last
  // time (4-lane groups when it was the small-segment plan, 8-lane groups
  // from 5/16 of <= 144-byte datagrams, 16 x 4 below that), the plan
  // kernels running behind the first and every 64th launch (DESIGN.md §4,
  // git 7692616:tools/ab_ipv4_mix.py, profiles/r2_ipv4_mix_sweep.jsonl)
  bool two = false, tile = false;
  uint32_t span_avg = 0;  // the cached plan's mean length (span_segs_for)
  int spw = 16;
  PlanReq req;
  int plan_used = -1;
  if (d_offsets && !forced_geometry(ctx) && !ctx->twoclass && n >= ics_ctx::kSmallPlanMin && n <= 0xFFFFFFFFull) {
    uint32_t plan = 0;
    PlanMix mix;
    const bool hit = plan_lookup(ctx, sp, true, &plan, &req, &mix);
    if (hit && plan == icsum::kPlanWholeBatchSmall && mix.avg <= icsum::kTinyMaxAvg)
      g = lane1;
    else if (hit && plan == icsum::kPlanWholeBatchSmall)
      g = ipv4_geometry({4, 2, true, 2, 1});
    else if (hit && mix.short16 >= ics_ctx::kIpv4ShortMix16 && mix.long16 == 0)
      g = ipv4_geometry({8, 8, true, 3, 1});  // ACK + MTU mixes past the two-class grid's limit
    else if (hit)
      g = ipv4_geometry({16, 4, true, 3, 1});  // MTU + a few ACKs: shorter unroll, 1-4 % (1 M datagrams)
    // the two-class launch (block lists, ics_ctx::kIpv4TwoClass16 for the
    // crossover against 16 x 4 groups; round 2's per-wave version beat the
    // 8-lane groups from 5/16 ACKs up, git 7692616:tools/ab_ipv4_mix.py)
    two = hit && plan != icsum::kPlanWholeBatchSmall && mix.short16 >= ics_ctx::kIpv4TwoClass16 && mix.long16 == 0;
    // ACK-heavy mixes: 128 datagrams per block, so the block's one short
    // pass carries more of them (3/4 ACKs 78.4 -> 75.4 us, mix_probe blk32)
    spw = mix.short16 >= ics_ctx::kIpv4TwoClassWide16 ? 32 : 16;
    plan_used = hit ? int(plan) : -1;
    tile = hit && !two && plan != icsum::kPlanWholeBatchSmall && ctx->tile != 0 && n >= ics_ctx::kTileMin;
    span_avg = hit ? mix.avg : 0u;
  }
  if (d_offsets && ctx->twoclass) {  // test hook
    two = true;
    spw = ctx->twoclass;
  }
  if (d_offsets && (ctx->tile == 1 || tile)) {  // the test hook, or the cached mix favours the tile launch
    const uint32_t S = span_segs_for(ctx, span_avg);
    ICS_HIP(icsum::launch_tile_ipv4(sp, mode, d_ip_ck, d_tcp_ck, d_status, S, st, ctx->span_blocks));
    note(ctx, ICS_K_TILE, {int(S), ICS_TILE_IPV4, true, 0, 1}, plan_used);
    return replan(ctx, sp, 64, req, st);
  }
  hipError_t le = hipErrorInvalidValue;
  if (two) {
    le = icsum::launch_ipv4_twoclass(sp, mode, d_ip_ck, d_tcp_ck, d_status, spw, ctx->twoclass_remap, st, ctx->twoclass_lds);
    if (le != hipErrorInvalidValue) note(ctx, ICS_K_IPV4_TWOCLASS, {16, spw, true, 3, 1}, plan_used);
  }
  if (le == hipErrorInvalidValue) {
    le = icsum::launch_ipv4_tcp(sp, mode, d_ip_ck, d_tcp_ck, d_status, g, 0, st);
    note(ctx, ICS_K_IPV4, g, plan_used);
  }
  ICS_HIP(le);
  if (int rc = replan(ctx, sp, 64, req, st)) return rc;
  return ICS_OK;
}

namespace {
// The device wrap: two passes (payload sums into n words of scratch, then the
// header launch) or one (ics_ctx::wrap_passes)
hipError_t device_wrap(ics_ctx* ctx, const icsum::SegSpec& sp, const ics_tcp_msg* msgs, uint32_t* hdr_out,
                       uint16_t* ip_ck, uint16_t* tcp_ck, bool payload_only, icsum::Geometry g, int plan,
                       hipStream_t st) {
  const icsum::TcpMsg* m = reinterpret_cast<const icsum::TcpMsg*>(msgs);
  if (!wrap_two_pass(ctx, hdr_out != nullptr, sp.n)) {
    note(ctx, ICS_K_WRAP, g, plan);
    return icsum::launch_tcp_wrap(sp, m, hdr_out, ip_ck, tcp_ck, payload_only, nullptr, g, 0, st);
  }
  Scratch sums(ctx, sp.n * 4, st);
  if (sums.error() != hipSuccess) return sums.error();
  note(ctx, ICS_K_WRAP_2PASS, g, plan);
  return icsum::launch_tcp_wrap(sp, m, hdr_out, ip_ck, tcp_ck, payload_only, static_cast<uint32_t*>(sums.get()), g,
                                0, st);
}

// The device wrap's geometry: one lane per datagram for ACK-sized batches (a
// fixed length, or a cached small plan with a mean <= kTinyMaxAvg: 1 M pure
// ACKs in place 78.3 -> 36.6 us, 40-56 B 119.0 -> 47.4 us,
// git 7692616:tools/ab_wrap_ack.py), else the fused kernel's geometry for the length
// hint.  The plan kernels run behind the launch as plan_lookup asks (the
// wrap's transmit buffer keeps its own cache slot: a stack's receive-side
// verify in between does not evict it).
icsum::Geometry wrap_geometry(ics_ctx* ctx, const icsum::SegSpec& sp, uint64_t hint, PlanReq* req, int* plan_used,
                              PlanMix* mix_out) {
  const icsum::Geometry lane1{1, 4, false, 0, 1};
  const icsum::Geometry base = geometry_for(ctx, sp.offsets ? hint : sp.seg_len);
  icsum::Geometry g = base.mode == icsum::kModeTiny ? lane1 : ipv4_geometry(base);
  *req = {};
  *plan_used = -1;
  if (sp.offsets && !forced_geometry(ctx) && sp.n >= ics_ctx::kSmallPlanMin && sp.n <= 0xFFFFFFFFull) {
    uint32_t plan = 0;
    PlanMix mix;
    const bool hit = plan_lookup(ctx, sp, true, &plan, req, &mix);
    if (hit && plan == icsum::kPlanWholeBatchSmall && mix.avg <= icsum::kTinyMaxAvg) g = lane1;
    if (hit) {
      *plan_used = int(plan);
      *mix_out = mix;
    }
  }
  return g;
}
}  // namespace

int wrap_device(ics_ctx* ctx, const icsum::SegSpec& sp, const ics_tcp_msg* d_msgs, uint32_t* hdr_out,
                uint16_t* d_ip_ck, uint16_t* d_tcp_ck, bool payload_only, uint64_t hint, hipStream_t st) {
  PlanReq req;
  int plan = -1;
  PlanMix mix;
  const icsum::Geometry g = wrap_geometry(ctx, sp, hint, &req, &plan, &mix);
  // the tile launch: the test hook; headers apart when the cached mix favours
  // it; in place only for long-segment mixes (its header stores cost the
  // same scattered write per datagram either way, and the per-segment wrap
  // is faster on short ones: 40..1040 B, 256 Ki: 40.3 / 44.7 us; config-4 mix
  // 499.3 / 464.2 us, git 7692616:tools/ab_dispatch.py).  Headers apart, the receive-side
  // mix of empty and MTU payloads tiles too (256 Ki / 1 M: 48.8 / 40.5 and
  // 169.3 / 150.8 us), payloads nearly all empty (pure ACKs) do not (1 M:
  // 24.2 / 41.0 us; profiles/r4_ab_dispatch_tile.jsonl)
  const bool tile_pick = plan >= 0 && plan != int(icsum::kPlanWholeBatchSmall) &&
                         (payload_only ? mix.short16 < ics_ctx::kTileApartShort16 && tile_wins(ctx, mix, sp.n, true)
                                       : !short_mix(mix) && ctx->tile != 0 && sp.n >= ics_ctx::kTileMin &&
                                             mix.long16 >= 4);
  if (sp.offsets && (ctx->tile == 1 || tile_pick)) {  // the wrap (in place or headers apart) as a tile launch
    const uint32_t S = span_segs_for(ctx, plan >= 0 ? mix.avg : 0u);
    ICS_HIP(icsum::launch_tile_wrap(sp, reinterpret_cast<const icsum::TcpMsg*>(d_msgs), hdr_out, d_ip_ck, d_tcp_ck,
                                    S, st, ctx->span_blocks));
    note(ctx, ICS_K_TILE, {int(S), hdr_out ? ICS_TILE_WRAP_APART : ICS_TILE_WRAP, true, 0, 1}, plan);
    return replan(ctx, sp, 64, req, st);
  }
  ICS_HIP(device_wrap(ctx, sp, d_msgs, hdr_out, d_ip_ck, d_tcp_ck, payload_only, g, plan, st));
  return replan(ctx, sp, 64, req, st);
}

int router_device(ics_ctx* ctx, const icsum::SegSpec& sp, uint32_t* d_hdrs, uint8_t* d_status, hipStream_t st) {
  if (d_hdrs) {
    ICS_HIP(icsum::launch_router_hdrs(sp, d_hdrs, d_status, st));
    note(ctx, ICS_K_ROUTER_HDRS);
  } else {
    ICS_HIP(icsum::launch_router_ttl(sp, d_status, st));
    note(ctx, ICS_K_ROUTER);
  }
  return ICS_OK;
}

namespace {
// Group the batches of a multi-batch call by kernel shape and issue one
// launch per group of up to kMaxBatchv (whose grids together stay below the
// dispatch's work-item limit); a batch too large for that runs alone through
// the single-batch path.
template <typename D, typename ClassFn, typename LaunchFn, typename AloneFn>
int run_batchv(ics_ctx* ctx, const D* b, uint32_t k, ClassFn cls_of, LaunchFn launch, AloneFn alone) {
  constexpr uint64_t kMaxBlocks = (uint64_t(1) << 24) - 1;
  std::vector<int> cls(k);
  for (uint32_t j = 0; j < k; ++j) cls[j] = b[j].n ? cls_of(b[j]) : -1;
  int last_cls = -1;
  for (int c = 0; c <= icsum::kBvLane1; ++c) {
    D group[icsum::kMaxBatchv];
    int m = 0;
    uint64_t blocks = 0;
    auto flush = [&]() -> int {
      if (m == 0) return ICS_OK;
      ICS_HIP(launch(group, m, c));
      last_cls = c;
      m = 0;
      blocks = 0;
      return ICS_OK;
    };
    for (uint32_t j = 0; j < k; ++j) {
      if (cls[j] != c) continue;
      const uint64_t nb = icsum::batchv_blocks(c, b[j].n);
      if (nb > kMaxBlocks / 4) {  // a large batch: a launch of its own, its usual path
        if (int rc = alone(b[j])) return rc;
        continue;
      }
      if (m == icsum::kMaxBatchv || blocks + nb > kMaxBlocks)
        if (int rc = flush()) return rc;
      group[m++] = b[j];
      blocks += nb;
    }
    if (int rc = flush()) return rc;
  }
  if (last_cls >= 0) note(ctx, ICS_K_BATCHV, {last_cls, int(k), true, 0, 1});
  return ICS_OK;
}
}  // namespace

int checksum_batchv_device(ics_ctx* ctx, const ics_seg_batch* batches, uint32_t k, hipStream_t st) {
  std::vector<icsum::BvSeg> b(k);
  for (uint32_t j = 0; j < k; ++j)
    b[j] = {static_cast<const uint8_t*>(batches[j].bytes), batches[j].offsets, batches[j].stride, batches[j].seg_len,
            batches[j].n, batches[j].init, batches[j].out, 0};
  auto cls_of = [&](const icsum::BvSeg& x) -> int {
    const icsum::SegSpec sp{x.bytes, x.offsets, x.stride, x.seg_len, x.n, ctx->d_zero};
    if (!x.offsets && x.seg_len == 64 && icsum::dense_supported(sp)) return icsum::kBvDense64;
    const icsum::Geometry g = icsum::pick_geometry(avg_len_hint(x.offsets, x.seg_len));
    if (g.mode == icsum::kModeTiny) return icsum::kBvTiny;
    if (g.segs > 1) return icsum::kBvSmall;
    return g.lps >= 32 ? icsum::kBvLine64 : icsum::kBvLine16;
  };
  auto launch = [&](const icsum::BvSeg* g, int m, int c) {
    return icsum::launch_checksum_batchv(g, m, c, ctx->d_zero, st);
  };
  auto alone = [&](const icsum::BvSeg& x) {
    const icsum::SegSpec sp{x.bytes, x.offsets, x.stride, x.seg_len, x.n, ctx->d_zero};
    return checksum_device(ctx, sp, x.init, nullptr, x.out, 0, st);
  };
  return run_batchv(ctx, b.data(), k, cls_of, launch, alone);
}

int ipv4_batchv_device(ics_ctx* ctx, const ics_dgram_batch* batches, uint32_t k, int mode, hipStream_t st) {
  std::vector<icsum::BvDgram> b(k);
  for (uint32_t j = 0; j < k; ++j)
    b[j] = {static_cast<uint8_t*>(batches[j].dgrams), batches[j].offsets, batches[j].stride, batches[j].dgram_len,
            batches[j].n, batches[j].ip_ck, batches[j].tcp_ck, batches[j].status};
  // the single call's unplanned choice: one lane per ACK-sized fixed-length
  // datagram, 64-lane groups past 3.5 KB, 16-lane line grids otherwise (and
  // for every offsets batch: mostly MTU-sized datagrams)
  auto cls_of = [&](const icsum::BvDgram& x) -> int {
    if (x.offsets) return icsum::kBvLine16;
    const icsum::Geometry g = icsum::pick_geometry(x.dlen);
    if (g.mode == icsum::kModeTiny) return icsum::kBvLane1;
    return g.lps >= 32 ? icsum::kBvLine64 : icsum::kBvLine16;
  };
  auto launch = [&](const icsum::BvDgram* g, int m, int c) {
    return icsum::launch_ipv4_batchv(g, m, c, mode, ctx->d_zero, st);
  };
  auto alone = [&](const icsum::BvDgram& x) {
    const icsum::SegSpec sp{x.dgrams, x.offsets, x.stride, x.dlen, x.n, ctx->d_zero};
    return ipv4_device(ctx, sp, mode, x.ip_ck, x.tcp_ck, x.status, st);
  };
  return run_batchv(ctx, b.data(), k, cls_of, launch, alone);
}

// ICSUM_FORCE (test hook): "key=value,key=value" forcing
// one kernel shape or dispatch decision so parity tests reach every
// instantiation.  An unknown key fails ics_create (a mistyped hook must not
// silently test the default path).
int apply_force(ics_ctx* ctx, const char* spec) {
  if (!spec || !*spec) return ICS_OK;
  std::string all(spec);
  size_t pos = 0;
  while (pos <= all.size()) {
    const size_t end = std::min(all.find(',', pos), all.size());
    const std::string item = all.substr(pos, end - pos);
    pos = end + 1;
    if (item.empty()) continue;
    const size_t eq = item.find('=');
    if (eq == std::string::npos) return fail(ICS_ERR_INVALID, "ICSUM_FORCE: '%s' is not key=value", item.c_str());
    const std::string k = item.substr(0, eq);
    char* tail = nullptr;
    const long long v = std::strtoll(item.c_str() + eq + 1, &tail, 0);
    if (!tail || *tail) return fail(ICS_ERR_INVALID, "ICSUM_FORCE: bad value in '%s'", item.c_str());
    if (k == "lps") ctx->force_lps = int(v);
    else if (k == "unroll") ctx->force_unroll = int(v);
    else if (k == "mode") ctx->force_mode = int(v);
    else if (k == "segs") ctx->force_segs = int(v);
    else if (k == "bin") ctx->bin = int(v);
    else if (k == "bin_min") ctx->bin_min = uint64_t(v);
    else if (k == "bin_plan") ctx->bin_plan = v >= 0 && v <= 3 ? int(v) : -1;
    else if (k == "bin_blocks") ctx->bin_blocks = uint32_t(std::max<long long>(v, 1));
    else if (k == "last_bin_lps") ctx->last_bin_lps = uint32_t(v);
    else if (k == "last_bin_blocks") ctx->last_bin_blocks = uint32_t(v);
    else if (k == "dense_segs") ctx->dense_segs = int(v);
    else if (k == "twoclass" && (v == 0 || v == 8 || v == 16 || v == 32)) ctx->twoclass = int(v);
    else if (k == "wrap_passes" && v >= 0 && v <= 2) ctx->wrap_passes = uint32_t(v);
    else if (k == "xcd_remap") icsum::set_xcd_remap(uint32_t(v));
    else if (k == "span_segs" && v >= 0 && v <= 63) ctx->span_segs = uint32_t(v);
    else if (k == "span_blocks" && v >= 0 && v <= 0xFFFFFF) ctx->span_blocks = uint32_t(v);
    else if (k == "tick_inline" && (v == 0 || v == 1)) ctx->tick_inline = int(v);
    else if (k == "slot_prio" && v >= -8 && v <= 8) ctx->slot_prio = int(v);
    else if (k == "tick_server" && v >= 0 && v <= 10000000) ctx->srv_idle_us = uint32_t(v);
    else if (k == "srv_pollers" && v >= 1 && v <= 4) ctx->srv_pollers = uint32_t(v);
    else if (k == "srv_blocks" && v >= 1 && v <= int64_t(icsum::kSrvBlocksMax)) ctx->srv_blocks = uint32_t(v);
    else if (k == "srv_vram" && (v == 0 || v == 1)) ctx->srv_vram = int(v);
    else if (k == "twoclass_remap" && v >= 0 && v <= 30) ctx->twoclass_remap = uint32_t(v);
    else if (k == "twoclass_lds" && v >= 0 && v <= 65536) ctx->twoclass_lds = uint32_t(v);
    else if (k == "zero_copy_max" && v >= 0) ctx->zero_copy_max = uint64_t(v);
    else if (k == "poison_ticket" && v > 0 && v <= 0xFFFFFFFFll) ctx->poison_ticket = uint32_t(v);
    else if (k == "tile" && v >= -1 && v <= 1) ctx->tile = int(v);
    else return fail(ICS_ERR_INVALID, "ICSUM_FORCE: unknown or out-of-range '%s'", item.c_str());
  }
  return ICS_OK;
}

}  // namespace icsum::detail
