// icsum_api.cpp — the C-ABI of libicsum.so (declared in include/icsum.h).
//
// Thin, exception-free layer: argument validation, device binding, error
// strings, geometry choice, and the host-memory (PCIe-inclusive) pipeline.
// All arithmetic happens in the HIP kernels (kernels/icsum_kernels.hip); there
// is no CPU fallback — without a usable GPU every call returns an error.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "icsum.h"
#include "icsum_workload.h"
#include "common/par_for.h"
#include "kernels/icsum_launch.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? ICS_ERR_NOMEM : ICS_ERR_HIP, "%s: %s (%d)", what,
              hipGetErrorString(e), int(e));
}

#define ICS_HIP(call)                                 \
  do {                                                \
    hipError_t e_ = (call);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #call); \
  } while (0)

uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = std::getenv(name);
  return v && *v ? uint32_t(std::strtoul(v, nullptr, 0)) : dflt;
}

}  // namespace

namespace icsum::detail {
// Device scratch kept across calls (hipMallocAsync + hipFreeAsync per call
// cost ≈5 us between the kernels).  A Scratch lease holds `mu` while the
// call enqueues its kernels, then records `ev` on its stream; a call on
// another stream first makes its stream wait for that event, and growing the
// buffer waits for it on the host.  It grows to the largest call's need and
// lives until ics_destroy; `zeroed` areas are cleared (stream-ordered) when
// they grow.
struct ScratchArea {
  explicit ScratchArea(bool zero = false) : zeroed(zero) {}
  std::mutex mu;
  void* buf = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  hipStream_t owner = nullptr;
  bool used = false;
  bool zeroed = false;
  void release() {
    if (buf) {
      if (used) (void)hipEventSynchronize(ev);
      (void)hipFree(buf);
      buf = nullptr;
    }
    if (ev) (void)hipEventDestroy(ev);
    ev = nullptr;
  }
};
}  // namespace icsum::detail

// One engine context per GPU.  Staging for the host-memory path is created
// on first use and guarded by `mu`.
struct ics_ctx {
  int device = 0;
  void* d_zero = nullptr;  // 64 zero bytes (icsum::SegSpec::zero16; the IPv4 kernel's header pad)
  // ---- test hooks (ICSUM_FORCE, read once at ics_create; parity tests only):
  // force one kernel shape or dispatch decision so every instantiation can be
  // pinned against the oracle.  None selects anything faster than the default.
  int force_lps = 0, force_unroll = 0, force_mode = -1, force_segs = 0;
  // length binning of offsets batches: -1 auto (n >= bin_min), 0 off, 1 always
  int bin = -1;
  uint64_t bin_min = uint64_t(1) << 16;
  uint32_t bin_blocks = 2048;    // grid of the bins 0-3 launch (their sizes are only known on the device)
  uint32_t last_bin_blocks = 0;  // grid cap of the last bin's launch (0: one lane group per segment)
  uint32_t last_bin_lps = 0;     // lanes per segment of the last bin's launch (0: auto, see checksum_device)
  int dense_segs = 4;            // k_checksum_dense segments per lane group in flight (0: off)
  int bin_plan = -1;  // -1: decided on the device per batch; forced: 0 whole, 1 split, 2 whole16, 3 wholeS
  int twoclass = 0;   // 0: auto; 16 / 32: every offsets batch through the two-class launch (that many per wave)
  // device wrap: 0 = two passes (payload sums, then a header launch) when
  // the headers go to an array of their own and the batch has at least
  // kWrapTwoPassMin datagrams, otherwise one pass (headers stored inside the
  // payload stream) — each the faster there (tools/ab_wrap_twopass.py,
  // DESIGN.md §6); 1 / 2 = always one / two (tests)
  static constexpr uint64_t kWrapTwoPassMin = uint64_t(1) << 18;
  uint32_t wrap_passes = 0;
  // ---- plan cache of the AUTO dispatch: the plan kernel (k_bin_plan)
  // reports its plan word into one of kPlanSlots page-locked host words, each
  // keyed by (offsets pointer, n) and stamped with the slot's generation, so
  // a word is only trusted for the batch whose miss asked for it.  A batch
  // whose key holds a whole-batch plan skips the binning passes (their 4
  // dispatches, ~25 us) and runs that plan's single launch; every
  // kPlanRefresh-th hit re-plans behind its launch, so a changed mix is
  // noticed within kPlanRefresh calls.  Several slots: a stack alternates its
  // transmit buffer (wrap) with its receive buffer (verify / unwrap), and
  // neither may evict the other's plan (LRU over the slots).
  static constexpr uint32_t kPlanRefresh = 16;
  static constexpr int kPlanSlots = 4;
  struct PlanSlot {
    const uint64_t* key = nullptr;
    uint64_t n = 0;
    uint32_t gen = 0;   // 1..254, in bits 56-63 of the slot's word
    uint32_t hits = 0;  // lookups since the slot was keyed
    uint64_t used = 0;  // LRU clock
  };
  PlanSlot plan_slot[kPlanSlots];
  uint64_t plan_clock = 0;
  uint32_t plan_gen = 0;
  // offsets batches from this many segments up (below the binning threshold)
  // take their single launch's geometry from the cached plan
  static constexpr uint64_t kSmallPlanMin = 16384;
  // ics_ipv4_tcp_batch: from this share of <= 144-byte datagrams (sixteenths,
  // the plan word's bits 4-7) an offsets batch runs 8-lane groups
  static constexpr uint32_t kIpv4ShortMix16 = 5;
  // ... and from this share up the two-class launch (k_ipv4_twoclass, 32
  // datagrams per wave), which beats the 8-lane groups from 5/16 ACKs up
  static constexpr uint32_t kIpv4TwoClass16 = 5;
  // the plain checksum's short-mix threshold (short_mix: the two-class
  // launch); raw-datagram ACK shares, AUTO vs two-class at 16 per wave
  // (tools/ab_ipv4_mix.py plain rows): 3/8 156.1 vs 144.1 us, 5/16 163.6 vs
  // 157.8, 1/4 169.6 vs 169.0, 3/16 178.3 vs 181.4
  static constexpr uint32_t kShortMix16 = 5;
  uint64_t* plan_host = nullptr;      // host view of the kPlanSlots words
  uint64_t* plan_host_dev = nullptr;  // the device's pointer to them
  std::mutex plan_mu;
  // diagnostics (ics_dispatch_info)
  std::atomic<uint64_t> n_hits{0}, n_misses{0}, n_replans{0};
  std::atomic<int32_t> last_kernel{0}, last_lps{0}, last_unroll{0}, last_plan{-1};
  // device scratch of the binned dispatch and the two-pass wrap (a binned
  // batch of n segments: 80 n bytes + 16 KiB; a two-pass wrap: 4 n)
  icsum::detail::ScratchArea scratch;
  std::mutex mu;
  // host path: nslots slots (2..kMaxSlots, ICSUM_HOST_SLOTS) of slot_bytes each
  // (ICSUM_HOST_SLOT_MB), each with pinned in/out staging, device buffers and a stream
  static constexpr int kMaxSlots = 4;
  static constexpr size_t kSlotSegs = size_t(1) << 20;
  int nslots = 3;  // 3 x 32 MiB: pageable 49.2 -> 51.4 GB/s over 2 x 64 MiB, pinned equal (tools/ab_host.py)
  size_t slot_bytes = size_t(32) << 20;
  bool staged = false;
  hipStream_t st[kMaxSlots] = {};
  hipEvent_t ev[kMaxSlots] = {};
  uint8_t* h_in[kMaxSlots] = {};
  uint8_t* d_in[kMaxSlots] = {};
  uint64_t* h_off[kMaxSlots] = {};
  uint64_t* d_off[kMaxSlots] = {};
  uint32_t* h_init[kMaxSlots] = {};
  uint32_t* d_init[kMaxSlots] = {};
  uint8_t* h_out[kMaxSlots] = {};   // u16 outputs or 5-byte ipv4 results
  uint8_t* d_out[kMaxSlots] = {};
  // wrap from host memory (allocated on first use): per slot up to
  // kWrapSlotSegs messages in, 40 header bytes per datagram back
  static constexpr size_t kWrapSlotSegs = size_t(1) << 18;
  bool wrap_staged = false;
  uint8_t* h_msg[kMaxSlots] = {};
  uint8_t* d_msg[kMaxSlots] = {};
  uint8_t* h_hdr[kMaxSlots] = {};
  uint8_t* d_hdr[kMaxSlots] = {};
  uint32_t* d_sums[kMaxSlots] = {};  // the two-pass wrap's payload sums
  // staging copies of pageable host batches: copy_threads ranges (the caller
  // and copy_threads - 1 kept workers, started on first use;
  // ICSUM_COPY_THREADS, default min(8, hardware threads))
  size_t copy_threads = 8;
  std::unique_ptr<icsum::detail::WorkerPool> copy_pool;
};

namespace {

int bind(ics_ctx* ctx) {
  if (!ctx) return fail(ICS_ERR_INVALID, "null context");
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != ctx->device) ICS_HIP(hipSetDevice(ctx->device));
  return ICS_OK;
}

bool wrap_two_pass(const ics_ctx* ctx, bool headers_apart, uint64_t n) {
  return ctx->wrap_passes == 2 || (ctx->wrap_passes == 0 && headers_apart && n >= ics_ctx::kWrapTwoPassMin);
}

// Scratch for the kernels one call enqueues on `st` (see ics_ctx::scratch).
class Scratch {
 public:
  Scratch(icsum::detail::ScratchArea& a, size_t bytes, hipStream_t st) : a_(a), lock_(a.mu), st_(st) {
    if (a.used && a.owner != st) err_ = hipStreamWaitEvent(st, a.ev, 0);
    if (err_ == hipSuccess && bytes > a.cap) {
      if (a.buf) {
        if (a.used) err_ = hipEventSynchronize(a.ev);
        if (err_ == hipSuccess) err_ = hipFree(a.buf);
        a.buf = nullptr;
        a.cap = 0;
      }
      const size_t cap = (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
      if (err_ == hipSuccess) err_ = hipMalloc(&a.buf, cap);
      if (err_ == hipSuccess && a.zeroed) err_ = hipMemsetAsync(a.buf, 0, cap, st);
      if (err_ == hipSuccess) a.cap = cap;
      else a.buf = nullptr;
    }
  }
  Scratch(ics_ctx* ctx, size_t bytes, hipStream_t st) : Scratch(ctx->scratch, bytes, st) {}
  ~Scratch() {
    if (err_ != hipSuccess) return;
    if (hipEventRecord(a_.ev, st_) == hipSuccess) {
      a_.owner = st_;
      a_.used = true;
    } else {  // cannot track this call's use: the next one waits for the device
      (void)hipDeviceSynchronize();
      a_.used = false;
    }
  }
  Scratch(const Scratch&) = delete;
  Scratch& operator=(const Scratch&) = delete;
  hipError_t error() const { return err_; }
  void* get() const { return a_.buf; }

 private:
  icsum::detail::ScratchArea& a_;
  std::lock_guard<std::mutex> lock_;
  hipStream_t st_;
  hipError_t err_ = hipSuccess;
};


// Bounds-checked build only: wait for the call's kernels and turn a device
// violation record into ICS_ERR_INVALID (the release build returns rc as is).
int bounds_verdict(hipStream_t st, int rc) {
  if (rc != ICS_OK || !icsum::bounds_checked_build()) return rc;
  uint32_t flags = 0;
  uint64_t what = 0;
  ICS_HIP(icsum::bounds_take(st, &flags, &what));
  if (flags)
    return fail(ICS_ERR_INVALID,
                "bounds check: %s%s%s (first: %s 0x%llx)", (flags & 1u) ? "load outside a segment's envelope " : "",
                (flags & 2u) ? "offsets not monotone " : "", (flags & 4u) ? "header load past a datagram " : "",
                (flags & 2u) && !(flags & 5u) ? "segment" : "address", (unsigned long long)what);
  return ICS_OK;
}

icsum::Geometry geometry_for(const ics_ctx* ctx, uint64_t avg_len) {
  icsum::Geometry g = icsum::pick_geometry(avg_len);
  if (ctx->force_lps) g = {ctx->force_lps, ctx->force_unroll ? ctx->force_unroll : g.unroll, g.nt, g.mode, 1};
  if (ctx->force_mode >= 0) g.mode = ctx->force_mode;
  if (ctx->force_segs > 0) g.segs = ctx->force_segs;
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

// a short-heavy mix's single launch: the two-class launch (ACK-sized segments
// one per lane, the rest 16 lanes each), 32 segments per wave from 3/4 short
// segments up and 16 below (fewer long segments per wave: shorter-lived
// waves).  2 M x 40 / 1460 B: 8-lane groups 279.5, two-class 64 / 32 / 16 per
// wave 255.7 / 234.9 / 231.1 us; raw-datagram mixes (tools/ab_ipv4_mix.py
// plain rows, 64 / 32 / 16): 7/8 ACKs 43.5 / 42.2 / 54.5, 3/4 74.8 / 68.5 /
// 74.5, 1/2 132.4 / 122.5 / 119.0, 7/16 145.0 / 139.3 / 131.9 us
// (profiles/r2_twoclass_spw*.jsonl).  Batches past the two-class grid's
// limit run 8-lane groups.
hipError_t launch_mix(ics_ctx* ctx, const icsum::SegSpec& sp, const uint32_t* d_init, const uint8_t* d_odd,
                      void* d_out, int out_kind, const PlanMix& mix, hipStream_t st) {
  const int spw = mix.short16 >= 12 ? 32 : 16;
  const hipError_t e = icsum::launch_checksum_twoclass(sp, d_init, d_odd, d_out, out_kind, spw, st);
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

int checksum_device(ics_ctx* ctx, const icsum::SegSpec& sp, const uint32_t* d_init, const uint8_t* d_odd,
                    void* d_out, int out_kind, hipStream_t st) {
  if (sp.offsets && ctx->twoclass) {  // test hook: the two-class launch on every offsets batch
    ICS_HIP(icsum::launch_checksum_twoclass(sp, d_init, d_odd, d_out, out_kind, ctx->twoclass, st));
    note(ctx, ICS_K_TWOCLASS, {16, ctx->twoclass, true, 3, 1});
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
    // the launch for the next call (tools/ab_small_offsets.py)
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

int ensure_staging(ics_ctx* ctx) {
  if (ctx->staged) return ICS_OK;
  for (int k = 0; k < ctx->nslots; ++k) {
    ICS_HIP(hipStreamCreateWithFlags(&ctx->st[k], hipStreamNonBlocking));
    ICS_HIP(hipEventCreateWithFlags(&ctx->ev[k], hipEventDisableTiming));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_in[k]), ctx->slot_bytes, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_in[k]), ctx->slot_bytes));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_off[k]), (ics_ctx::kSlotSegs + 1) * 8, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_off[k]), (ics_ctx::kSlotSegs + 1) * 8));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_init[k]), ics_ctx::kSlotSegs * 4, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_init[k]), ics_ctx::kSlotSegs * 4));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_out[k]), ics_ctx::kSlotSegs * 5, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_out[k]), ics_ctx::kSlotSegs * 5));
  }
  ctx->staged = true;
  return ICS_OK;
}

int ensure_wrap_staging(ics_ctx* ctx) {
  if (ctx->wrap_staged) return ICS_OK;
  for (int k = 0; k < ctx->nslots; ++k) {
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_msg[k]), ics_ctx::kWrapSlotSegs * sizeof(ics_tcp_msg), 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_msg[k]), ics_ctx::kWrapSlotSegs * sizeof(ics_tcp_msg)));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_hdr[k]), ics_ctx::kWrapSlotSegs * 40, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_hdr[k]), ics_ctx::kWrapSlotSegs * 40));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_sums[k]), ics_ctx::kWrapSlotSegs * 4));
  }
  ctx->wrap_staged = true;
  return ICS_OK;
}

void free_staging(ics_ctx* ctx) {
  for (int k = 0; k < ics_ctx::kMaxSlots; ++k) {
    if (ctx->st[k]) (void)hipStreamSynchronize(ctx->st[k]);
    if (ctx->h_in[k]) (void)hipHostFree(ctx->h_in[k]);
    if (ctx->d_in[k]) (void)hipFree(ctx->d_in[k]);
    if (ctx->h_off[k]) (void)hipHostFree(ctx->h_off[k]);
    if (ctx->d_off[k]) (void)hipFree(ctx->d_off[k]);
    if (ctx->h_init[k]) (void)hipHostFree(ctx->h_init[k]);
    if (ctx->d_init[k]) (void)hipFree(ctx->d_init[k]);
    if (ctx->h_out[k]) (void)hipHostFree(ctx->h_out[k]);
    if (ctx->d_out[k]) (void)hipFree(ctx->d_out[k]);
    if (ctx->h_msg[k]) (void)hipHostFree(ctx->h_msg[k]);
    if (ctx->d_msg[k]) (void)hipFree(ctx->d_msg[k]);
    if (ctx->h_hdr[k]) (void)hipHostFree(ctx->h_hdr[k]);
    if (ctx->d_hdr[k]) (void)hipFree(ctx->d_hdr[k]);
    if (ctx->d_sums[k]) (void)hipFree(ctx->d_sums[k]);
    if (ctx->ev[k]) (void)hipEventDestroy(ctx->ev[k]);
    if (ctx->st[k]) (void)hipStreamDestroy(ctx->st[k]);
  }
  ctx->staged = false;
  ctx->wrap_staged = false;
}

// One staged chunk of segments [i0, i1) covering bytes [b0, b1).  A segment
// longer than a staging slot goes through the slots as PIECES: chunks with
// piece = true, i1 = i0 + 1 and [b0, b1) a slot-sized part of that one
// segment (pos = the part's offset inside it).
struct Chunk {
  uint64_t i0, i1, b0, b1;
  bool piece = false, last = false;
  uint64_t pos = 0;
};

// Next chunk starting at segment i0 (whose first `pos` bytes were already
// staged as pieces) that fits the slot.
int next_chunk(const ics_ctx* ctx, const uint64_t* offsets, uint64_t stride, uint64_t seg_len, uint64_t n,
               uint64_t i0, uint64_t pos, bool allow_pieces, uint64_t cap_n, Chunk* c) {
  const uint64_t cap_b = ctx->slot_bytes;
  const uint64_t s0 = offsets ? offsets[i0] : i0 * stride;
  const uint64_t len0 = offsets ? offsets[i0 + 1] - s0 : seg_len;
  if (pos || len0 > cap_b) {  // segment i0 does not fit a slot: its next piece
    if (!allow_pieces)
      return fail(ICS_ERR_INVALID, "datagram %llu (%llu bytes) exceeds the %zu-byte staging slot",
                  (unsigned long long)i0, (unsigned long long)len0, ctx->slot_bytes);
    const uint64_t take = std::min<uint64_t>(cap_b, len0 - pos);
    *c = {i0, i0 + 1, s0 + pos, s0 + pos + take, true, pos + take == len0, pos};
    return ICS_OK;
  }
  if (!offsets) {
    const uint64_t per = std::max<uint64_t>(stride, seg_len);
    uint64_t k = per ? cap_b / per : cap_n;
    if (k == 0) k = 1;  // stride > slot but the segment itself fits
    k = std::min<uint64_t>({k, cap_n, n - i0});
    *c = {i0, i0 + k, i0 * stride, (i0 + k - 1) * stride + seg_len};
    return ICS_OK;
  }
  const uint64_t b0 = offsets[i0];
  uint64_t i1 = i0;
  while (i1 < n && i1 - i0 < cap_n && offsets[i1 + 1] - b0 <= cap_b) ++i1;
  *c = {i0, i1, b0, offsets[i1]};
  return ICS_OK;
}

// InternetChecksum::value() of a raw sum (util/tools/checksum.h:31-41)
uint16_t fold_value(uint32_t sum) {
  while (sum > 0xFFFFu) sum = (sum >> 16) + (sum & 0xFFFFu);
  return uint16_t(~sum & 0xFFFFu);
}

// A piece is summed on the device as sub-pieces of this many bytes (one lane
// group each, so a 32 MiB piece is 512 segments of work, not one long one);
// even, so every sub-piece starts with the piece's parity.
constexpr uint64_t kSubPiece = uint64_t(64) << 10;

// Is [p, p+bytes) page-locked host memory the DMA engines can read directly?
bool host_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory is not an error for us
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// memcpy split over the context's copy workers: a single core copies pageable
// memory into the pinned slots at ~10-20 GB/s, below what PCIe Gen5 x16 moves
void par_memcpy(ics_ctx* ctx, void* dst, const void* src, size_t n) {
  constexpr size_t kMinPerThread = size_t(4) << 20;
  const size_t t = std::min<size_t>(ctx->copy_threads, std::max<size_t>(1, n / kMinPerThread));
  if (t <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  if (!ctx->copy_pool) ctx->copy_pool = std::make_unique<icsum::detail::WorkerPool>(ctx->copy_threads - 1);
  ctx->copy_pool->run(n, t, [=](size_t a, size_t b) {
    std::memcpy(static_cast<char*>(dst) + a, static_cast<const char*>(src) + a, b - a);
  });
}

// fn(j0, j1) over [0, m) datagrams on the copy workers (host-side stores into
// the caller's batch at retire), serially below 16 Ki datagrams per range
template <typename Fn>
void host_ranges(ics_ctx* ctx, uint64_t m, Fn&& fn) {
  constexpr uint64_t kMinPerThread = 16384;
  const size_t t = std::min<size_t>(ctx->copy_threads, std::max<uint64_t>(1, m / kMinPerThread));
  if (t <= 1) {
    fn(size_t(0), size_t(m));
    return;
  }
  if (!ctx->copy_pool) ctx->copy_pool = std::make_unique<icsum::detail::WorkerPool>(ctx->copy_threads - 1);
  ctx->copy_pool->run(m, t, fn);
}

// ICS_MODE_PATCH's stores (k_ipv4_tcp, mode 2) applied on the host from a
// COMPUTE pass's results: for every datagram of >= 20 bytes the IPv4
// checksum goes to bytes 10..11; when >= 18 bytes follow the header
// (4 * hlen clamped to [20, len]) the TCP checksum goes to bytes 16..17 of
// the TCP header.  Both big-endian.  `res` = the slot's results: m ip u16,
// m tcp u16, m status bytes.
void host_patch_fields(uint8_t* bytes, const uint64_t* offsets, uint64_t stride, uint64_t dlen, const Chunk& c,
                       const uint8_t* res, uint64_t j0, uint64_t j1) {
  const uint64_t m = c.i1 - c.i0;
  const uint16_t* ip = reinterpret_cast<const uint16_t*>(res);
  const uint16_t* tcp = ip + m;
  for (uint64_t j = j0; j < j1; ++j) {
    const uint64_t i = c.i0 + j;
    const uint64_t s = offsets ? offsets[i] : i * stride;
    const uint64_t len = offsets ? offsets[i + 1] - s : dlen;
    if (len < 20) continue;
    uint8_t* d = bytes + s;
    d[10] = uint8_t(ip[j] >> 8);
    d[11] = uint8_t(ip[j]);
    uint64_t off = 4u * (d[0] & 0x0fu);
    if (off < 20) off = 20;
    if (off > len) off = len;
    if (len - off >= 18) {
      d[off + 16] = uint8_t(tcp[j] >> 8);
      d[off + 17] = uint8_t(tcp[j]);
    }
  }
}

// kind 0: checksum batch (u16 out); kind 1: ipv4_tcp batch (ip u16, tcp u16, status u8);
// kind 2: tcp wrap (40 header bytes per datagram back, written into h_bytes).
// The slots take turns, one stream each: while the GPU moves and sums chunk
// k, the host prepares chunk k+1.  Pinned user buffers are DMA'd directly (no
// host copy); pageable ones are staged through the pinned slots by par_memcpy.
int host_pipeline(ics_ctx* ctx, int kind, void* h_bytes, const uint64_t* h_offsets,
                  uint64_t stride, uint64_t seg_len, const uint32_t* h_init, uint64_t n, int mode,
                  uint16_t* out_a, uint16_t* out_b, uint8_t* out_c, const ics_tcp_msg* h_msgs = nullptr) {
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (int rc = ensure_staging(ctx)) return rc;
  if (kind == 2)
    if (int rc = ensure_wrap_staging(ctx)) return rc;
  const bool direct = host_pinned(h_bytes);
  Chunk pending[ics_ctx::kMaxSlots];
  bool busy[ics_ctx::kMaxSlots] = {};
  uint32_t piece_sum = 0;  // running sum of the long segment whose pieces are in flight
  auto retire = [&](int k) -> int {
    if (!busy[k]) return ICS_OK;
    ICS_HIP(hipEventSynchronize(ctx->ev[k]));
    const Chunk& c = pending[k];
    const uint64_t m = c.i1 - c.i0;
    if (c.piece) {
      // raw u32 sums of the piece's sub-pieces; uint32 addition is
      // associative, so sum_ of the whole segment = init + every part's sum
      // (each summed with its own start parity), wrap included
      const uint64_t parts = (c.b1 - c.b0 + kSubPiece - 1) / kSubPiece;
      const uint32_t* raw = reinterpret_cast<const uint32_t*>(ctx->h_out[k]);
      for (uint64_t j = 0; j < parts; ++j) piece_sum += raw[j];
      if (c.last) {
        out_a[c.i0] = fold_value((h_init ? h_init[c.i0] : 0u) + piece_sum);
        piece_sum = 0;
      }
    } else if (kind == 0) {
      std::memcpy(out_a + c.i0, ctx->h_out[k], m * 2);
    } else if (kind == 2 && mode == 1) {  // payload-only: headers to the caller's array
      std::memcpy(reinterpret_cast<uint8_t*>(out_c) + 40 * c.i0, ctx->h_hdr[k], m * 40);
    } else if (kind == 2) {  // 40 header bytes into each datagram of the caller's batch
      uint8_t* bytes = static_cast<uint8_t*>(h_bytes);
      host_ranges(ctx, m, [&](size_t j0, size_t j1) {
        for (uint64_t j = j0; j < j1; ++j) {
          const uint64_t i = c.i0 + j;
          const uint64_t s0 = h_offsets ? h_offsets[i] : i * stride;
          const uint64_t len = h_offsets ? h_offsets[i + 1] - s0 : seg_len;
          if (len >= 40) std::memcpy(bytes + s0, ctx->h_hdr[k] + 40 * j, 40);
        }
      });
    } else {
      if (out_a) std::memcpy(out_a + c.i0, ctx->h_out[k], m * 2);
      if (out_b) std::memcpy(out_b + c.i0, ctx->h_out[k] + m * 2, m * 2);
      if (out_c) std::memcpy(out_c + c.i0, ctx->h_out[k] + m * 4, m);
      if (mode == ICS_MODE_PATCH)  // scattered 2-byte stores into the caller's batch
        host_ranges(ctx, m, [&](size_t j0, size_t j1) {
          host_patch_fields(static_cast<uint8_t*>(h_bytes), h_offsets, stride, seg_len, c, ctx->h_out[k], j0, j1);
        });
    }
    busy[k] = false;
    return ICS_OK;
  };
  uint64_t i0 = 0, pos = 0;
  int slot = 0;
  while (i0 < n) {
    Chunk c;
    if (int rc = next_chunk(ctx, h_offsets, stride, seg_len, n, i0, pos, kind == 0,
                            kind == 2 ? ics_ctx::kWrapSlotSegs : ics_ctx::kSlotSegs, &c))
      return rc;
    if (int rc = retire(slot)) return rc;
    const uint64_t m = c.i1 - c.i0, nb = c.b1 - c.b0;
    uint8_t* src = static_cast<uint8_t*>(h_bytes) + c.b0;
    if (!direct) {
      par_memcpy(ctx, ctx->h_in[slot], src, nb);
      src = ctx->h_in[slot];
    }
    hipStream_t st = ctx->st[slot];
    ICS_HIP(hipMemcpyAsync(ctx->d_in[slot], src, nb, hipMemcpyHostToDevice, st));
    if (c.piece) {
      // ics_sum_batch over the piece's sub-pieces: raw sums, parity = the
      // piece's offset in its segment (checksum.h:24-26 carried across add()s)
      const uint64_t parts = (nb + kSubPiece - 1) / kSubPiece;
      for (uint64_t j = 0; j <= parts; ++j) ctx->h_off[slot][j] = std::min<uint64_t>(j * kSubPiece, nb);
      uint8_t* odd = reinterpret_cast<uint8_t*>(ctx->h_init[slot]);
      std::memset(odd, int(c.pos & 1), parts);
      ICS_HIP(hipMemcpyAsync(ctx->d_off[slot], ctx->h_off[slot], (parts + 1) * 8, hipMemcpyHostToDevice, st));
      ICS_HIP(hipMemcpyAsync(ctx->d_init[slot], odd, parts, hipMemcpyHostToDevice, st));
      const icsum::SegSpec sp{ctx->d_in[slot], ctx->d_off[slot], 0, 0, parts, ctx->d_zero};
      ICS_HIP(icsum::launch_checksum(sp, nullptr, reinterpret_cast<const uint8_t*>(ctx->d_init[slot]),
                                     ctx->d_out[slot], 1, geometry_for(ctx, kSubPiece), 0, st));
      ICS_HIP(hipMemcpyAsync(ctx->h_out[slot], ctx->d_out[slot], parts * 4, hipMemcpyDeviceToHost, st));
      ICS_HIP(hipEventRecord(ctx->ev[slot], st));
      pending[slot] = c;
      busy[slot] = true;
      if (c.last) {
        i0 = c.i1;
        pos = 0;
      } else {
        pos = c.pos + nb;
      }
      slot = (slot + 1) % ctx->nslots;
      continue;
    }
    const uint64_t* d_off = nullptr;
    if (h_offsets) {
      for (uint64_t j = 0; j <= m; ++j) ctx->h_off[slot][j] = h_offsets[c.i0 + j] - c.b0;
      ICS_HIP(hipMemcpyAsync(ctx->d_off[slot], ctx->h_off[slot], (m + 1) * 8, hipMemcpyHostToDevice, st));
      d_off = ctx->d_off[slot];
    }
    const icsum::SegSpec sp{ctx->d_in[slot], d_off, stride, seg_len, m, ctx->d_zero};
    const uint64_t avg = h_offsets ? nb / m : seg_len;
    const icsum::Geometry g = geometry_for(ctx, avg);
    if (kind == 2) {
      std::memcpy(ctx->h_msg[slot], h_msgs + c.i0, m * sizeof(ics_tcp_msg));
      ICS_HIP(hipMemcpyAsync(ctx->d_msg[slot], ctx->h_msg[slot], m * sizeof(ics_tcp_msg), hipMemcpyHostToDevice, st));
      ICS_HIP(icsum::launch_tcp_wrap(sp, reinterpret_cast<const icsum::TcpMsg*>(ctx->d_msg[slot]),
                                     reinterpret_cast<uint32_t*>(ctx->d_hdr[slot]), nullptr, nullptr, mode == 1,
                                     wrap_two_pass(ctx, true, m) ? ctx->d_sums[slot] : nullptr, ipv4_geometry(g),
                                     0, st));
      ICS_HIP(hipMemcpyAsync(ctx->h_hdr[slot], ctx->d_hdr[slot], m * 40, hipMemcpyDeviceToHost, st));
    } else if (kind == 0) {
      const uint32_t* d_init = nullptr;
      if (h_init) {
        std::memcpy(ctx->h_init[slot], h_init + c.i0, m * 4);
        ICS_HIP(hipMemcpyAsync(ctx->d_init[slot], ctx->h_init[slot], m * 4, hipMemcpyHostToDevice, st));
        d_init = ctx->d_init[slot];
      }
      ICS_HIP(icsum::launch_checksum(sp, d_init, nullptr, ctx->d_out[slot], 0, g, 0, st));
      ICS_HIP(hipMemcpyAsync(ctx->h_out[slot], ctx->d_out[slot], m * 2, hipMemcpyDeviceToHost, st));
    } else {
      uint16_t* a = reinterpret_cast<uint16_t*>(ctx->d_out[slot]);
      uint16_t* b = a + m;
      uint8_t* s = ctx->d_out[slot] + m * 4;
      // PATCH from host memory: the device computes (COMPUTE gives the very
      // values PATCH stores) and only the 5-byte results come back; the two
      // fields are written into the caller's bytes on the host at retire,
      // instead of copying every patched byte back over PCIe
      const int dev_mode = mode == ICS_MODE_PATCH ? ICS_MODE_COMPUTE : mode;
      ICS_HIP(icsum::launch_ipv4_tcp(sp, dev_mode, a, b, s, ipv4_geometry(g), 0, st));
      ICS_HIP(hipMemcpyAsync(ctx->h_out[slot], ctx->d_out[slot], m * 5, hipMemcpyDeviceToHost, st));
    }
    ICS_HIP(hipEventRecord(ctx->ev[slot], st));
    pending[slot] = c;
    busy[slot] = true;
    i0 = c.i1;
    slot = (slot + 1) % ctx->nslots;
  }
  for (int k = 0; k < ctx->nslots; ++k)  // oldest first
    if (int rc = retire((slot + k) % ctx->nslots)) return rc;
  return bounds_verdict(ctx->st[0], ICS_OK);
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
    else if (k == "twoclass" && (v == 0 || v == 16 || v == 32)) ctx->twoclass = int(v);
    else if (k == "wrap_passes" && v >= 0 && v <= 2) ctx->wrap_passes = uint32_t(v);
    else if (k == "xcd_remap") icsum::set_xcd_remap(uint32_t(v));
    else return fail(ICS_ERR_INVALID, "ICSUM_FORCE: unknown or out-of-range '%s'", item.c_str());
  }
  return ICS_OK;
}

}  // namespace

extern "C" {

const char* ics_version(void) {
  return icsum::bounds_checked_build() ? "icsum 0.2.0 (gfx950, bounds-checked debug build)" : "icsum 0.2.0 (gfx950)";
}
int ics_abi_version(void) { return ICS_ABI_VERSION; }
const char* ics_last_error(void) { return g_err.c_str(); }

int ics_device_count(int* count) {
  if (!count) return fail(ICS_ERR_INVALID, "null count");
  *count = 0;
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e == hipErrorNoDevice || (e == hipSuccess && c == 0)) return ICS_OK;
  ICS_HIP(e);
  *count = c;
  return ICS_OK;
}

int ics_create(int device, ics_ctx** out) {
  if (!out) return fail(ICS_ERR_INVALID, "null output pointer");
  *out = nullptr;
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess || c == 0) return fail(ICS_ERR_NODEVICE, "no GPU available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= c) return fail(ICS_ERR_NODEVICE, "device %d out of range [0,%d)", device, c);
  ICS_HIP(hipSetDevice(device));
  ics_ctx* ctx = new (std::nothrow) ics_ctx();
  if (!ctx) return fail(ICS_ERR_NOMEM, "context allocation failed");
  ctx->device = device;
  if (int rc = apply_force(ctx, std::getenv("ICSUM_FORCE"))) {
    delete ctx;
    return rc;
  }
  if (hipMalloc(&ctx->d_zero, 64) != hipSuccess || hipMemset(ctx->d_zero, 0, 64) != hipSuccess) {
    delete ctx;
    return fail(ICS_ERR_NOMEM, "device allocation failed");
  }
  {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    ctx->copy_threads = std::max<size_t>(1, env_u32("ICSUM_COPY_THREADS", std::min(8u, hw)));
  }
  if (hipEventCreateWithFlags(&ctx->scratch.ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipFree(ctx->d_zero);
    delete ctx;
    return fail(ICS_ERR_HIP, "event creation failed");
  }
  {  // the plan cache's words; coherent: the plan kernel's store reaches host memory without a flush
    void* p = nullptr;
    if (hipHostMalloc(&p, 8 * ics_ctx::kPlanSlots, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess) {
      ctx->plan_host = static_cast<uint64_t*>(p);
      for (int k = 0; k < ics_ctx::kPlanSlots; ++k) ctx->plan_host[k] = ~uint64_t(0);
      void* dp = nullptr;
      if (hipHostGetDevicePointer(&dp, p, 0) == hipSuccess) {
        ctx->plan_host_dev = static_cast<uint64_t*>(dp);
      } else {
        (void)hipHostFree(p);
        ctx->plan_host = nullptr;
      }
    }
    (void)hipGetLastError();
  }
  ctx->nslots = int(std::min<uint32_t>(std::max<uint32_t>(env_u32("ICSUM_HOST_SLOTS", 3), 2), ics_ctx::kMaxSlots));
  ctx->slot_bytes = size_t(std::max<uint32_t>(env_u32("ICSUM_HOST_SLOT_MB", 32), 1)) << 20;
  *out = ctx;
  return ICS_OK;
}

int ics_destroy(ics_ctx* ctx) {
  if (!ctx) return ICS_OK;
  if (bind(ctx) == ICS_OK) {
    free_staging(ctx);
    if (ctx->d_zero) (void)hipFree(ctx->d_zero);
    if (ctx->plan_host) (void)hipHostFree(ctx->plan_host);
    ctx->scratch.release();
  }
  delete ctx;
  return ICS_OK;
}

int ics_dispatch_info(const ics_ctx* ctx, ics_dispatch_info_t* info) {
  if (!ctx || !info) return fail(ICS_ERR_INVALID, "null argument");
  info->plan_hits = ctx->n_hits.load(std::memory_order_relaxed);
  info->plan_misses = ctx->n_misses.load(std::memory_order_relaxed);
  info->plan_requests = ctx->n_replans.load(std::memory_order_relaxed);
  info->last_kernel = ctx->last_kernel.load(std::memory_order_relaxed);
  info->last_lps = ctx->last_lps.load(std::memory_order_relaxed);
  info->last_unroll = ctx->last_unroll.load(std::memory_order_relaxed);
  info->last_plan = ctx->last_plan.load(std::memory_order_relaxed);
  return ICS_OK;
}

int ics_device_of(const ics_ctx* ctx, int* device) {
  if (!ctx || !device) return fail(ICS_ERR_INVALID, "null argument");
  *device = ctx->device;
  return ICS_OK;
}

int ics_checksum_batch(ics_ctx* ctx, const void* d_bytes, const uint64_t* d_offsets, uint64_t stride,
                       uint64_t seg_len, const uint32_t* d_init, uint16_t* d_out, uint64_t n,
                       void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_bytes || !d_out) return fail(ICS_ERR_INVALID, "null device buffer");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_bytes), d_offsets, stride, seg_len, n, ctx->d_zero};
  return bounds_verdict(static_cast<hipStream_t>(stream),
                        checksum_device(ctx, sp, d_init, nullptr, d_out, 0, static_cast<hipStream_t>(stream)));
}

int ics_sum_batch(ics_ctx* ctx, const void* d_bytes, const uint64_t* d_offsets, uint64_t stride,
                  uint64_t seg_len, const uint32_t* d_init, const uint8_t* d_odd, uint32_t* d_sum,
                  uint64_t n, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_bytes || !d_sum) return fail(ICS_ERR_INVALID, "null device buffer");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_bytes), d_offsets, stride, seg_len, n, ctx->d_zero};
  return bounds_verdict(static_cast<hipStream_t>(stream),
                        checksum_device(ctx, sp, d_init, d_odd, d_sum, 1, static_cast<hipStream_t>(stream)));
}

int ics_set_binning(ics_ctx* ctx, int mode) {
  if (!ctx) return fail(ICS_ERR_INVALID, "null context");
  if (mode < ICS_BINNING_AUTO || mode > ICS_BINNING_BINNED) return fail(ICS_ERR_INVALID, "bad binning mode %d", mode);
  ctx->bin = mode;
  return ICS_OK;
}

int ics_fold_batch(ics_ctx* ctx, const uint32_t* d_sum, uint16_t* d_out, uint64_t n, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_sum || !d_out) return fail(ICS_ERR_INVALID, "null device buffer");
  ICS_HIP(icsum::launch_fold(d_sum, d_out, n, static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int ics_ipv4_tcp_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets, uint64_t stride,
                       uint64_t dgram_len, uint64_t n, int mode, uint16_t* d_ip_ck,
                       uint16_t* d_tcp_ck, uint8_t* d_status, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (mode < ICS_MODE_COMPUTE || mode > ICS_MODE_PATCH) return fail(ICS_ERR_INVALID, "bad mode %d", mode);
  if (n == 0) return ICS_OK;
  if (!d_dgrams) return fail(ICS_ERR_INVALID, "null datagram buffer");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_dgrams), d_offsets, stride, dgram_len, n, ctx->d_zero};
  // an offsets batch of raw datagrams gives no length hint; datagrams are at
  // most 64 KiB and mostly MTU-sized, and the 16-lane line grid is the best
  // measured geometry for both 1500- and 9000-byte datagrams (64 Ki x 1500 B:
  // 18.3 us vs 48.8 us with the 64-lane default; tools/ab_ipv4_offsets.py)
  // ACK-sized datagrams (a fixed length <= kTinyMaxAvg, or a cached plan
  // whose mean is) run one lane per datagram with default-policy loads
  // (neighbours share lines): 1 M x 40 B VERIFY 30.3 -> 10.6 us (tools/ab_ipv4_mix.py, AB_LANE1)
  const icsum::Geometry lane1{1, 4, false, 0, 1};
  const icsum::Geometry base = geometry_for(ctx, d_offsets ? 1500 : dgram_len);
  icsum::Geometry g = base.mode == icsum::kModeTiny ? lane1 : ipv4_geometry(base);
  hipStream_t st = static_cast<hipStream_t>(stream);
  // a receive batch of mostly short datagrams (pure ACKs: 40 bytes) leaves
  // most of a 16-lane group idle: from 16 Ki datagrams up the geometry
  // follows the plan the device reported for the same offsets buffer last
  // time (4-lane groups when it was the small-segment plan, 8-lane groups
  // from 5/16 of <= 144-byte datagrams, 16 x 4 below that), the plan
  // kernels running behind the first and every 16th launch (DESIGN.md §4,
  // tools/ab_ipv4_mix.py, profiles/r2_ipv4_mix_sweep.jsonl)
  bool two = false;
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
    // the two-class launch, 32 datagrams per wave.  1 M datagrams VERIFY,
    // 8-lane groups vs two-class at 64 / 32 / 16 per wave (tools/ab_ipv4_mix.py):
    // 3/4 ACKs 127.3 vs 85.3 / 83.7 / 98.9 us, 1/2 157.9 vs 154.0 / 139.8 /
    // 149.7, 7/16 166.0 vs 169.7 / 153.8 / 164.3, 5/16 183.1 vs 201.0 / 181.1 / 185.5
    two = hit && plan != icsum::kPlanWholeBatchSmall && mix.short16 >= ics_ctx::kIpv4TwoClass16 && mix.long16 == 0;
    plan_used = hit ? int(plan) : -1;
  }
  if (d_offsets && ctx->twoclass) two = true;  // test hook
  hipError_t le = hipErrorInvalidValue;
  if (two) {
    le = icsum::launch_ipv4_twoclass(sp, mode, d_ip_ck, d_tcp_ck, d_status, st);
    if (le != hipErrorInvalidValue) note(ctx, ICS_K_IPV4_TWOCLASS, {16, 32, true, 3, 1}, plan_used);
  }
  if (le == hipErrorInvalidValue) {
    le = icsum::launch_ipv4_tcp(sp, mode, d_ip_ck, d_tcp_ck, d_status, g, 0, st);
    note(ctx, ICS_K_IPV4, g, plan_used);
  }
  ICS_HIP(le);
  if (int rc = replan(ctx, sp, 64, req, st)) return rc;
  return bounds_verdict(st, ICS_OK);
}

}  // extern "C"

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
// tools/ab_wrap_ack.py), else the fused kernel's geometry for the length
// hint.  The plan kernels run behind the launch as plan_lookup asks (the
// wrap's transmit buffer keeps its own cache slot: a stack's receive-side
// verify in between does not evict it).
icsum::Geometry wrap_geometry(ics_ctx* ctx, const icsum::SegSpec& sp, uint64_t hint, PlanReq* req, int* plan_used) {
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
    if (hit) *plan_used = int(plan);
  }
  return g;
}
}  // namespace

extern "C" {

int ics_tcp_wrap_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets, uint64_t stride,
                       uint64_t dgram_len, uint64_t n, const ics_tcp_msg* d_msgs, uint16_t* d_ip_ck,
                       uint16_t* d_tcp_ck, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_dgrams || !d_msgs) return fail(ICS_ERR_INVALID, "null device buffer");
  if (reinterpret_cast<uintptr_t>(d_msgs) & 3u) return fail(ICS_ERR_INVALID, "message records not 4-byte aligned");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_dgrams), d_offsets, stride, dgram_len, n, ctx->d_zero};
  // the stack's segments are <= 1000 B of payload (TCPConfig::MAX_PAYLOAD_SIZE): the
  // 16-lane line grid of MTU-sized datagrams unless a fixed length says otherwise
  PlanReq req;
  int plan = -1;
  const icsum::Geometry g = wrap_geometry(ctx, sp, 1040, &req, &plan);
  hipStream_t st = static_cast<hipStream_t>(stream);
  ICS_HIP(device_wrap(ctx, sp, d_msgs, nullptr, d_ip_ck, d_tcp_ck, false, g, plan, st));
  if (int rc = replan(ctx, sp, 64, req, st)) return rc;
  return bounds_verdict(st, ICS_OK);
}

int ics_tcp_wrap_headers(ics_ctx* ctx, const void* d_payloads, const uint64_t* d_offsets, uint64_t stride,
                         uint64_t payload_len, uint64_t n, const ics_tcp_msg* d_msgs, void* d_hdrs,
                         uint16_t* d_ip_ck, uint16_t* d_tcp_ck, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_payloads || !d_msgs || !d_hdrs) return fail(ICS_ERR_INVALID, "null device buffer");
  if (reinterpret_cast<uintptr_t>(d_msgs) & 3u) return fail(ICS_ERR_INVALID, "message records not 4-byte aligned");
  if (reinterpret_cast<uintptr_t>(d_hdrs) & 3u) return fail(ICS_ERR_INVALID, "header array not 4-byte aligned");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_payloads), d_offsets, stride, payload_len, n, ctx->d_zero};
  PlanReq req;
  int plan = -1;
  const icsum::Geometry g = wrap_geometry(ctx, sp, 1000, &req, &plan);
  hipStream_t st = static_cast<hipStream_t>(stream);
  ICS_HIP(device_wrap(ctx, sp, d_msgs, static_cast<uint32_t*>(d_hdrs), d_ip_ck, d_tcp_ck, true, g, plan, st));
  if (int rc = replan(ctx, sp, 64, req, st)) return rc;
  return bounds_verdict(st, ICS_OK);
}

}  // extern "C"

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

extern "C" {

int ics_checksum_batchv(ics_ctx* ctx, const ics_seg_batch* batches, uint32_t k, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (k == 0) return ICS_OK;
  if (!batches) return fail(ICS_ERR_INVALID, "null batch array");
  for (uint32_t j = 0; j < k; ++j)
    if (batches[j].n && (!batches[j].bytes || !batches[j].out))
      return fail(ICS_ERR_INVALID, "batch %u: null device buffer", j);
  hipStream_t st = static_cast<hipStream_t>(stream);
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
  return bounds_verdict(st, run_batchv(ctx, b.data(), k, cls_of, launch, alone));
}

int ics_ipv4_tcp_batchv(ics_ctx* ctx, const ics_dgram_batch* batches, uint32_t k, int mode, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (mode < ICS_MODE_COMPUTE || mode > ICS_MODE_PATCH) return fail(ICS_ERR_INVALID, "bad mode %d", mode);
  if (k == 0) return ICS_OK;
  if (!batches) return fail(ICS_ERR_INVALID, "null batch array");
  for (uint32_t j = 0; j < k; ++j)
    if (batches[j].n && !batches[j].dgrams) return fail(ICS_ERR_INVALID, "batch %u: null datagram buffer", j);
  hipStream_t st = static_cast<hipStream_t>(stream);
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
    return ics_ipv4_tcp_batch(ctx, x.dgrams, x.offsets, x.stride, x.dlen, x.n, mode, x.ip_ck, x.tcp_ck, x.status,
                              stream);
  };
  return bounds_verdict(st, run_batchv(ctx, b.data(), k, cls_of, launch, alone));
}

int ics_tcp_wrap_headers_host(ics_ctx* ctx, const void* h_payloads, const uint64_t* h_offsets, uint64_t stride,
                              uint64_t payload_len, uint64_t n, const ics_tcp_msg* h_msgs, void* h_hdrs) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!h_payloads || !h_msgs || !h_hdrs) return fail(ICS_ERR_INVALID, "null host buffer");
  return host_pipeline(ctx, 2, const_cast<void*>(h_payloads), h_offsets, stride, payload_len, nullptr, n, 1,
                       nullptr, nullptr, static_cast<uint8_t*>(h_hdrs), h_msgs);
}

int ics_tcp_wrap_batch_host(ics_ctx* ctx, void* h_dgrams, const uint64_t* h_offsets, uint64_t stride,
                            uint64_t dgram_len, uint64_t n, const ics_tcp_msg* h_msgs) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!h_dgrams || !h_msgs) return fail(ICS_ERR_INVALID, "null host buffer");
  return host_pipeline(ctx, 2, h_dgrams, h_offsets, stride, dgram_len, nullptr, n, 0, nullptr, nullptr, nullptr,
                       h_msgs);
}

int ics_router_ttl_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets, uint64_t stride,
                         uint64_t dgram_len, uint64_t n, uint8_t* d_status, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_dgrams || !d_status) return fail(ICS_ERR_INVALID, "null device buffer");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_dgrams), d_offsets, stride, dgram_len, n, ctx->d_zero};
  ICS_HIP(icsum::launch_router_ttl(sp, d_status, static_cast<hipStream_t>(stream)));
  note(ctx, ICS_K_ROUTER);
  return bounds_verdict(static_cast<hipStream_t>(stream), ICS_OK);
}

int ics_checksum_batch_host(ics_ctx* ctx, const void* h_bytes, const uint64_t* h_offsets,
                            uint64_t stride, uint64_t seg_len, const uint32_t* h_init,
                            uint16_t* h_out, uint64_t n) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!h_bytes || !h_out) return fail(ICS_ERR_INVALID, "null host buffer");
  return host_pipeline(ctx, 0, const_cast<void*>(h_bytes), h_offsets, stride, seg_len, h_init, n, 0,
                       h_out, nullptr, nullptr);
}

int ics_ipv4_tcp_batch_host(ics_ctx* ctx, void* h_dgrams, const uint64_t* h_offsets, uint64_t stride,
                            uint64_t dgram_len, uint64_t n, int mode, uint16_t* h_ip_ck,
                            uint16_t* h_tcp_ck, uint8_t* h_status) {
  if (int rc = bind(ctx)) return rc;
  if (mode < ICS_MODE_COMPUTE || mode > ICS_MODE_PATCH) return fail(ICS_ERR_INVALID, "bad mode %d", mode);
  if (n == 0) return ICS_OK;
  if (!h_dgrams) return fail(ICS_ERR_INVALID, "null host buffer");
  return host_pipeline(ctx, 1, h_dgrams, h_offsets, stride, dgram_len, nullptr, n, mode, h_ip_ck,
                       h_tcp_ck, h_status);
}

int ics_malloc(ics_ctx* ctx, void** d_ptr, size_t bytes) {
  if (int rc = bind(ctx)) return rc;
  if (!d_ptr) return fail(ICS_ERR_INVALID, "null output pointer");
  ICS_HIP(hipMalloc(d_ptr, bytes ? bytes : 1));
  return ICS_OK;
}

int ics_free(ics_ctx* ctx, void* d_ptr) {
  if (int rc = bind(ctx)) return rc;
  if (d_ptr) ICS_HIP(hipFree(d_ptr));
  return ICS_OK;
}

int ics_host_alloc(ics_ctx* ctx, void** h_ptr, size_t bytes) {
  if (int rc = bind(ctx)) return rc;
  if (!h_ptr) return fail(ICS_ERR_INVALID, "null output pointer");
  ICS_HIP(hipHostMalloc(h_ptr, bytes ? bytes : 1, 0));
  return ICS_OK;
}

int ics_host_free(ics_ctx* ctx, void* h_ptr) {
  if (int rc = bind(ctx)) return rc;
  if (h_ptr) ICS_HIP(hipHostFree(h_ptr));
  return ICS_OK;
}

int ics_memcpy_htod(ics_ctx* ctx, void* d_dst, const void* h_src, size_t bytes, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (!bytes) return ICS_OK;
  ICS_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int ics_memcpy_dtoh(ics_ctx* ctx, void* h_dst, const void* d_src, size_t bytes, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (!bytes) return ICS_OK;
  ICS_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int ics_stream_synchronize(ics_ctx* ctx, void* stream) {
  if (int rc = bind(ctx)) return rc;
  ICS_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

// ---- synthetic workloads (icsum_workload.h) -----------------------------

int icsw_fill_bytes(ics_ctx* ctx, void* d_bytes, uint64_t nbytes, uint64_t seed, uint64_t pos0,
                    void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (nbytes && !d_bytes) return fail(ICS_ERR_INVALID, "null device buffer");
  ICS_HIP(icsum::launch_fill_bytes(static_cast<uint8_t*>(d_bytes), nbytes, seed, pos0,
                                   static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int icsw_pseudo_inits(ics_ctx* ctx, uint32_t* d_init, const uint64_t* d_offsets, uint64_t seg_len,
                      uint64_t n, uint64_t seed, uint64_t index0, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n && !d_init) return fail(ICS_ERR_INVALID, "null device buffer");
  ICS_HIP(icsum::launch_pseudo_inits(d_init, d_offsets, seg_len, n, seed, index0,
                                     static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int icsw_ipv4_tcp_headers(ics_ctx* ctx, void* d_dgrams, uint64_t stride, uint64_t dgram_len,
                          uint64_t n, uint64_t seed, uint64_t index0, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n && !d_dgrams) return fail(ICS_ERR_INVALID, "null device buffer");
  if (dgram_len < 20) return fail(ICS_ERR_INVALID, "datagram length %llu < 20", (unsigned long long)dgram_len);
  ICS_HIP(icsum::launch_ipv4_tcp_headers(static_cast<uint8_t*>(d_dgrams), stride, dgram_len, n, seed,
                                         index0, static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t icsw_mixed_len(uint64_t seed, uint64_t i) {
  const uint64_t m = mix64((seed ^ 0x3C3C3C3C3C3C3C3Cull) + (i + 1) * 0x9E3779B97F4A7C15ull);
  const unsigned e = 6u + unsigned(m % 10u);
  return (1ull << e) + ((m >> 8) & ((1ull << e) - 1));
}

int icsw_mixed_offsets(uint64_t* h_offsets, uint64_t n, uint64_t seed) {
  if (!h_offsets) return fail(ICS_ERR_INVALID, "null offsets");
  h_offsets[0] = 0;
  for (uint64_t i = 0; i < n; ++i) h_offsets[i + 1] = h_offsets[i] + icsw_mixed_len(seed, i);
  return ICS_OK;
}

}  // extern "C"
