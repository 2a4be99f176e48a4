// icsum_ctx.h — internal to libicsum.so: the engine context (struct ics_ctx,
// opaque in include/icsum.h) and what the three translation units behind the
// C-ABI share:
//   icsum_api.cpp       argument validation, device binding, error strings, the extern "C" entry points
//   icsum_dispatch.cpp  device-buffer dispatch: geometry choice, the plan cache, binning, multi-batch grouping
//   icsum_host.cpp      the host-memory (PCIe-inclusive) pipeline and its staging slots
// Not installed, not part of the ABI.
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <mutex>

#include "icsum.h"
#include "common/par_for.h"
#include "kernels/icsum_launch.h"

namespace icsum::detail {

// Error reporting (ics_last_error): set the calling thread's message, return code.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_fail(hipError_t e, const char* what);

#define ICS_HIP(call)                                                 \
  do {                                                                \
    hipError_t e_ = (call);                                           \
    if (e_ != hipSuccess) return ::icsum::detail::hip_fail(e_, #call); \
  } while (0)

inline uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = std::getenv(name);
  return v && *v ? uint32_t(std::strtoul(v, nullptr, 0)) : dflt;
}

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
  // tile launches of offsets batches (k_span): -1 auto, 0 never, 1 every
  // offsets batch (checksum, fused IPv4, wraps); span_segs: segments per
  // wave (0: span_segs_for)
  int tile = -1;
  uint32_t span_segs = 0;
  uint32_t span_blocks = 0;  // test hook: grid cap of the tile launch (0: none), reaches its grid-stride form
  int slot_prio = 0;    // staging-slot stream priority (ICSUM_FORCE slot_prio; 0: default stream creation)
  int tick_inline = 1;  // zero-copy ticks of <= kTickSegs offsets segments through k_tick (ICSUM_FORCE tick_inline=0: off)
  static constexpr uint64_t kSpanBytes = 20 << 10;  // segment bytes per span (span_segs_for)
  static constexpr uint64_t kTileMin = uint64_t(1) << 16;  // tile launches from this many segments (AUTO)
  static constexpr uint64_t kTileMinChecksum = uint64_t(1) << 17;  // ... of the plain checksum (tile_wins)
  static constexpr uint32_t kTileMaxAvg = 1024;            // ... and up to this mean length (tile_wins)
  static constexpr uint32_t kTileApartShort16 = 12;       // headers-apart wrap: below 12/16 empty-ish payloads
  uint32_t twoclass_remap = 0;  // block_order run length (log2) of the two-class launches; 0: hardware order
  uint32_t twoclass_lds = 0;    // dynamic LDS bytes per two-class block (residency cap; ICSUM_FORCE twoclass_lds)
  // device wrap: 0 = two passes (payload sums, then a header launch) when
  // the headers go to an array of their own and the batch has at least
  // kWrapTwoPassMin datagrams, otherwise one pass (headers stored inside the
  // payload stream) — each the faster there (git 7692616:tools/ab_wrap_twopass.py,
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
  // noticed within kPlanRefresh calls (64: the stats + plan kernels cost
  // ≈ 9.5 us behind a 256 Ki-datagram call, 0.6 us per call at every 16th,
  // profiles/r4_stack_kernel_stats.csv).  Several slots: a stack alternates its
  // transmit buffer (wrap) with its receive buffer (verify / unwrap), and
  // neither may evict the other's plan (LRU over the slots).
  static constexpr uint32_t kPlanRefresh = 64;
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
  // ... and from this share up the two-class launch (k_ipv4_twoclass, block
  // lists, 16 datagrams per wave in the bounds pass), which beats 16 x 4
  // groups from 3/16 ACKs up (1 M datagrams VERIFY, git 7692616:tools/ab_mix_split.py,
  // profiles/r3_mix_twoclass_ab.jsonl: 1/8 200.2 vs 198.5 us, 3/16 187.3 vs
  // 191.4, 1/4 176.0 vs 185.4, 5/16 164.3 vs 184.2)
  static constexpr uint32_t kIpv4TwoClass16 = 3;
  // ... with 32 datagrams per wave (128 per block) from this share up
  static constexpr uint32_t kIpv4TwoClassWide16 = 11;
  // the plain checksum's short-mix threshold (short_mix: the two-class
  // launch); raw-datagram ACK shares, AUTO vs two-class at 16 per wave
  // (round 2, git 7692616:tools/ab_ipv4_mix.py plain rows): 3/8 156.1 vs 144.1 us, 5/16
  // 163.6 vs 157.8, 1/4 169.6 vs 169.0, 3/16 178.3 vs 181.4; with the block
  // lists (round 3, git 7692616:tools/ab_plain_mix_threshold.py,
  // profiles/r3_plain_mix_threshold.jsonl): 1/4 169.0 vs 166.1, 3/16 177.3
  // vs 178.9, 1/8 186.8 vs 190.8
  static constexpr uint32_t kShortMix16 = 4;
  uint64_t* plan_host = nullptr;      // host view of the kPlanSlots words
  uint64_t* plan_host_dev = nullptr;  // the device's pointer to them
  std::mutex plan_mu;
  // diagnostics (ics_dispatch_info)
  std::atomic<uint64_t> n_hits{0}, n_misses{0}, n_replans{0};
  std::atomic<uint64_t> n_host_zc{0}, n_host_dma{0};  // host pipeline: zero-copy calls, DMA'd chunks
  std::atomic<int32_t> last_kernel{0}, last_lps{0}, last_unroll{0}, last_plan{-1};
  // device scratch of the binned dispatch and the two-pass wrap (a binned
  // batch of n segments: 80 n bytes + 16 KiB; a two-pass wrap: 4 n)
  icsum::detail::ScratchArea scratch;
  std::mutex mu;
  // host path: nslots slots (2..kMaxSlots, ICSUM_HOST_SLOTS) of slot_bytes each
  // (ICSUM_HOST_SLOT_MB), each with pinned in/out staging, device buffers and a stream
  static constexpr int kMaxSlots = 4;
  static constexpr size_t kSlotSegs = size_t(1) << 20;
  int nslots = 3;  // 3 x 32 MiB: pageable 49.2 -> 51.4 GB/s over 2 x 64 MiB, pinned equal (git 7692616:tools/ab_host.py)
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
  // a host-memory batch of at most this many bytes that fits one slot is not
  // copied to the device: the kernel reads it (and its offsets, inits or
  // messages) straight from page-locked memory over PCIe and writes its
  // results straight into the pinned result area — one launch and one
  // synchronisation per call instead of DMA copies on either side, which is
  // what a per-tick TUN / socket batch pays for ("Per-tick host
  // batches"); ICSUM_FORCE zero_copy_max=0 turns it off (tests)
  uint64_t zero_copy_max = uint64_t(2) << 20;
  // ... and it ends in a completion word the launch's last block stores
  // (icsum::Done, a block-count ticket in d_ticket), which the caller spins
  // on: ~3.7 us less than waiting for the stream's completion signal
  // (git 7692616:tools/probe/sync_probe.hip), and no second launch behind the kernel
  uint64_t* h_flag = nullptr;  // kMaxSlots words, 64 bytes apart, coherent page-locked
  uint64_t flag_ticket = 0;
  uint32_t* d_ticket = nullptr;  // kMaxSlots block-count tickets, 64 bytes apart (icsum::Done)
  // test hook (ICSUM_FORCE poison_ticket=V): slot 0's ticket is set to V once
  // staging exists, so a test can drive the recovery in wait_flag
  uint32_t poison_ticket = 0;
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
  // resident tick server (ics_set_tick_server; icsum_host.cpp): zero-copy
  // ticks of <= kTickSegs x srv_blocks segments go to a kernel that stays
  // resident between ticks and takes them from mailboxes in coherent
  // page-locked memory — no launch per tick.  srv_idle_us 0: off.
  uint32_t srv_idle_us = 0;
  uint32_t srv_blocks = 4;  // resident blocks, one mailbox each (ics_set_tick_server_blocks; ICSUM_FORCE srv_blocks)
  uint32_t srv_grid = 0;    // the blocks of the grid launched last
  icsum::TickMailbox* h_mb = nullptr;  // kSrvBlocksMax done / state words (page-locked)
  // kSrvBlocksMax x kSrvWords descriptor words: page-locked, or with srv_vram
  // uncached device memory the host writes through the PCIe BAR (then each
  // tick's bytes are copied into d_srv_stage too: the server reads nothing
  // over PCIe; ICSUM_FORCE srv_vram)
  uint64_t* srv_words = nullptr;
  int srv_vram = 0;
  bool srv_words_vram = false;
  static constexpr size_t kSrvStageBytes = size_t(256) << 10;  // per slot: a tick's bytes + records
  uint8_t* d_srv_stage[kMaxSlots] = {};
  hipStream_t st_srv = nullptr;
  uint32_t srv_seq[icsum::kSrvBlocksMax] = {};  // the last job posted to each mailbox
  bool srv_launched = false;  // a server was launched (its `state` words say whether it still runs)
  uint64_t n_srv_jobs = 0, n_srv_launches = 0;
  uint32_t srv_pollers = 1;  // waves polling the mailbox, staggered (ICSUM_FORCE srv_pollers, 1..4)
};

namespace icsum::detail {

// Make ctx's device current on the calling thread (ICS_ERR_INVALID for null).
int bind(ics_ctx* ctx);

// Bounds-checked build only: wait for the call's kernels and turn a device
// violation record into ICS_ERR_INVALID (the release build returns rc as is).
int bounds_verdict(hipStream_t st, int rc);

// Scratch for the kernels one call enqueues on `st` (see ics_ctx::scratch).
class Scratch {
 public:
  Scratch(ScratchArea& a, size_t bytes, hipStream_t st) : a_(a), lock_(a.mu), st_(st) {
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
  ScratchArea& a_;
  std::lock_guard<std::mutex> lock_;
  hipStream_t st_;
  hipError_t err_ = hipSuccess;
};

// ---- icsum_dispatch.cpp: device-buffer calls, arguments already validated.
// Each enqueues on `st` and returns ICS_OK or an error code (no bounds verdict).

// ICSUM_FORCE: parse "key=value,..." into ctx's test hooks.
int apply_force(ics_ctx* ctx, const char* spec);
// The geometry of a batch whose mean length is avg_len (test hooks applied).
icsum::Geometry geometry_for(const ics_ctx* ctx, uint64_t avg_len);
// The fused IPv4 kernels' variant of a checksum geometry.
icsum::Geometry ipv4_geometry(icsum::Geometry g);
icsum::Geometry ipv4_fixed_geometry(const ics_ctx* ctx, icsum::Geometry g, uint64_t len);
// Does the device wrap use two passes for this call?
bool wrap_two_pass(const ics_ctx* ctx, bool headers_apart, uint64_t n);
// a1-a4: checksum (out_kind 0: folded u16) or raw sums (1: u32) of a batch.
int checksum_device(ics_ctx* ctx, const icsum::SegSpec& sp, const uint32_t* d_init, const uint8_t* d_odd,
                    void* d_out, int out_kind, hipStream_t st);
// b1-b4: the fused IPv4 header + TCP checksum kernel (mode COMPUTE / VERIFY / PATCH).
int ipv4_device(ics_ctx* ctx, const icsum::SegSpec& sp, int mode, uint16_t* d_ip_ck, uint16_t* d_tcp_ck,
                uint8_t* d_status, hipStream_t st);
// c1: TCP wrap in place (hdr_out null) or into a header array (payload_only);
// hint = the mean length an offsets batch is assumed to have before its plan lands.
int wrap_device(ics_ctx* ctx, const icsum::SegSpec& sp, const ics_tcp_msg* d_msgs, uint32_t* hdr_out,
                uint16_t* d_ip_ck, uint16_t* d_tcp_ck, bool payload_only, uint64_t hint, hipStream_t st);
// c2: the router's TTL decrement + header checksum recompute, in place
// (d_hdrs null) or with the forwarded headers to d_hdrs (20 bytes each).
int router_device(ics_ctx* ctx, const icsum::SegSpec& sp, uint32_t* d_hdrs, uint8_t* d_status, hipStream_t st);
// Multi-batch calls: batches grouped by kernel shape, one launch per group.
int checksum_batchv_device(ics_ctx* ctx, const ics_seg_batch* batches, uint32_t k, hipStream_t st);
int ipv4_batchv_device(ics_ctx* ctx, const ics_dgram_batch* batches, uint32_t k, int mode, hipStream_t st);

// ---- icsum_host.cpp: the host-memory pipeline.
// kind 0: checksum batch (u16 out); kind 1: ipv4_tcp batch (ip u16, tcp u16, status u8);
// kind 2: tcp wrap (40 header bytes per datagram back, written into h_bytes, or
// into out_c for mode 1 = payload-only).  Returns with every result in place.
int host_pipeline(ics_ctx* ctx, int kind, void* h_bytes, const uint64_t* h_offsets, uint64_t stride,
                  uint64_t seg_len, const uint32_t* h_init, uint64_t n, int mode, uint16_t* out_a, uint16_t* out_b,
                  uint8_t* out_c, const ics_tcp_msg* h_msgs = nullptr);
// Release the pipeline's staging slots (ics_destroy).
void free_staging(ics_ctx* ctx);
// the resident tick server: quit word, wait for the kernel to leave (ICS_OK when none runs)
int server_stop(ics_ctx* ctx);

}  // namespace icsum::detail
