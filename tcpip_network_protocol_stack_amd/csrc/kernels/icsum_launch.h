// icsum_launch.h — internal launcher interface between the C-ABI layer
// (icsum_api.cpp, icsum_dispatch.cpp, icsum_host.cpp) and the HIP kernels (icsum_kernels.hip).  Not installed.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace icsum {

// Lane-group geometry of one launch: LPS lanes share a segment, each lane
// keeps UNROLL 16-byte loads in flight per step.
struct Geometry {
  int lps;
  int unroll;
  bool nt;   // non-temporal loads
  int mode;  // chunk grid: 0 16-byte + boundary slot, 2 16-byte all masked, 3 128-byte line, primed boundaries
  int segs = 1;  // > 1: small-segment kernel, SEGS segments per lane group in flight
};

// Geometry::mode of the tiny-segment kernel (k_checksum_tiny: one lane per
// segment, up to four 16-byte loads in flight; {1, 4, false, kModeTiny, 1})
constexpr int kModeTiny = 4;
// batches of at most this mean segment length run one lane per segment:
// 1 M x 40-43 B offsets 21.9 -> 11.4 us, fixed 40 / 52 B 15.8 -> 13.2 us;
// 64-144 B segments are faster 4 lanes each (git 7692616:tools/ab_tiny.py)
constexpr uint32_t kTinyMaxAvg = 56;

// Pick a geometry from the (average) segment length in bytes.
Geometry pick_geometry(uint64_t avg_len);
bool geometry_supported(Geometry g);

// In-kernel completion of a zero-copy host call: every block makes its
// results visible at system scope and takes a ticket; the block that takes
// the last one resets the ticket word and stores `value` into the host word
// `flag` with a system-scope release (the host spins on it).  flag == nullptr:
// nothing (every device-path launch).  Honoured by the kernels the host path
// launches: checksum (tiny, small, per-group), the fused IPv4 kernel, the
// one-pass wrap and the two-pass wrap's header pass.
struct Done {
  uint32_t* ticket = nullptr;  // device word, 0 between launches
  uint64_t* flag = nullptr;    // coherent page-locked host word
  uint64_t value = 0;
};

struct SegSpec {
  const uint8_t* bytes;
  const uint64_t* offsets;  // n+1 or nullptr
  uint64_t stride;
  uint64_t seg_len;
  uint64_t n;
  const void* zero16;  // 64 zero bytes in device memory (stand-in for absent arrays, header pad)
  // length-binned launch (bin_spec): bin `bin`'s list (16-byte entries, see
  // launch_bin_segments) and the binning pass's meta words; n stays the batch
  // size (the list's capacity)
  const void* list = nullptr;
  const uint32_t* meta = nullptr;
  int bin = -1;
  Done done{};  // see Done
};

// Length binning of an offsets batch (mixed segment sizes): every segment
// goes to the bin whose geometry suits its length, and each bin is run with
// its own geometry, reading its work list on the device.
//   list  kBins * n entries of 16 bytes ({start lo, start hi, length,
//         segment}; length 0xFFFFFFFF = re-read the offsets): bin b's
//         entries at list + b * n, in no particular order
//   meta  kBinMetaBytesTotal bytes: bin sizes at kBinMetaCount, the plan at
//         kBinMetaPlan, scatter cursors, then the stats pass's partials
// Passes: bin statistics, a one-block plan kernel and, under the split plan
// only, the scatter into the lists; needs n < 2^32.  The plan kernel zeroes the scatter cursors.  The plan
// (k_bin_plan) decides on the device whether the batch runs split into bins
// or whole with the long-segment geometry (then the last bin's launch, one
// lane group per segment of the batch, takes every segment).
constexpr int kBins = 5;
constexpr int kBinMetaCount = 0;
constexpr int kBinMetaCursor = 20;  // scatter pass: entries placed per bin
constexpr int kBinMetaPlan = 28;    // 0: whole batch, 1: split into bins, 2: whole batch in 16-lane groups,
                                    // 3: whole batch through the small-segment body (or, for a mean
                                    // segment length <= kTinyMaxAvg, the tiny-segment body)
constexpr int kBinMetaAvgLen = 29;  // mean segment length in bytes (plan kernel)
constexpr int kBinMetaWords = 32;
constexpr uint32_t kBinStatBlocks = 256;  // stats pass partials follow meta (<= 256: one per plan thread)
// bytes of meta + the stats pass's partials (the lists follow, 16-byte aligned)
constexpr size_t kBinMetaBytesTotal = kBinMetaWords * 4 + kBins * kBinStatBlocks * 12;
// force_plan: -1 the device plan decides, 0 whole batch, 1 split, 2 whole
// batch in 16-lane groups, 3 whole batch through the small-segment body (tests); last_lps: lanes per segment of the last
// bin's launch (its wave count enters the plan's cost model)
// plan_out (nullable, device-visible page-locked host memory): the plan
// kernel stores its plan word there for the host's plan cache (k_bin_plan:
// plan bits 0-3, <= 144-byte segments in sixteenths 4-7, n 8-39, bytes in
// segments over 1920 bytes in sixteenths 40-43, mean length 44-55, `gen`
// 56-63: the cache slot's generation, so the host trusts only the word its
// own request produced)
hipError_t launch_bin_segments(const uint64_t* offsets, uint64_t n, void* list, uint32_t* meta, int force_plan,
                               uint32_t last_lps, uint64_t* plan_out, uint32_t gen, hipStream_t st);
// k_bin_plan's plans: the whole-batch ones and the split plan
constexpr uint32_t kPlanWholeBatch = 0, kPlanSplitBins = 1, kPlanWholeBatch16 = 2, kPlanWholeBatchSmall = 3;
// the stats + plan passes alone (no bin lists): a re-plan for the plan cache
hipError_t launch_bin_plan(const uint64_t* offsets, uint64_t n, uint32_t* meta, uint32_t last_lps,
                           uint64_t* plan_out, uint32_t gen, hipStream_t st);
Geometry bin_geometry(int bin);
// bins 0..kBins-2 in one launch (sp = bin_spec(whole, list, meta, 0)),
// blocks_per_bin blocks striding over each bin
hipError_t launch_checksum_bins(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                                int out_kind, uint32_t blocks_per_bin, hipStream_t st);
// bin b's launch spec
SegSpec bin_spec(const SegSpec& whole, const void* list, const uint32_t* meta, int bin);

// out_kind 0: u16 value(), 1: u32 raw sum
hipError_t launch_checksum(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                           int out_kind, Geometry g, uint32_t max_blocks, hipStream_t st);
// Two-class launch (k_checksum_twoclass, block lists): each block's short
// segments (<= 4 chunks) one per lane on one wave, its long ones 16 lanes
// each claimed by every wave; spw (16 or 32) segments per wave in the
// bounds pass
// (remap: block_order's log2 XCD run length, 0 = hardware order)
hipError_t launch_checksum_twoclass(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                                    int out_kind, int spw, uint32_t remap, hipStream_t st, uint32_t lds_pad = 0);
// Dense fixed-stride batches (stride == seg_len in {32, 64, 128}, 16-byte
// aligned bytes, no parity array): k_checksum_dense, SEGS segments per lane
// group in flight (segs in {1, 2, 4, 8}; not every (seg_len, segs) pair exists)
bool dense_supported(const SegSpec& sp);
hipError_t launch_checksum_dense(const SegSpec& sp, const uint32_t* init, void* out, int out_kind, int segs,
                                 hipStream_t st);

// ---- several batches in one launch (ics_checksum_batchv / ics_ipv4_tcp_batchv)
// Up to kMaxBatchv batches of one kernel shape (BvClass) share a launch: the
// grid is the concatenation of each batch's own grid, the table travels in the
// kernel arguments (no copy), and every block finds its batch by a scan of
// the table's block offsets.  One ramp and one drain for all of them instead
// of one per batch ("Short batches").
constexpr int kMaxBatchv = 16;
struct BvSeg {  // one ics_checksum_batch call's arguments (u16 outputs); 64 bytes
  const uint8_t* bytes;
  const uint64_t* offsets;
  uint64_t stride, seg_len, n;
  const uint32_t* init;
  uint16_t* out;
  uint64_t pad;  // a power-of-two stride: the indexed descriptor address is a shift
};
struct BvDgram {  // one ics_ipv4_tcp_batch call's arguments; 64 bytes
  uint8_t* dgrams;
  const uint64_t* offsets;
  uint64_t stride, dlen, n;
  uint16_t* ip_ck;
  uint16_t* tcp_ck;
  uint8_t* status;
};
static_assert(sizeof(BvSeg) == 64 && sizeof(BvDgram) == 64, "multi-batch descriptors: 64-byte stride");
// the kernel shapes a multi-batch launch can take: the dense kernel (fixed
// stride == length == 64 B, aligned), one lane per segment (ACK-sized fixed
// lengths), 4-lane groups with two segments in flight (short fixed lengths),
// the 16- and 64-lane line grids (MTU-sized / long or unknown mixes), and the
// fused kernel's one lane per ACK-sized datagram
// (the ICS_BV_* values ics_dispatch_info reports)
enum BvClass : int { kBvDense64 = 0, kBvTiny = 1, kBvSmall = 2, kBvLine16 = 3, kBvLine64 = 4, kBvLane1 = 5 };
// blocks one batch of n segments takes in a launch of class cls
uint64_t batchv_blocks(int cls, uint64_t n);
// k batches (1 <= k <= kMaxBatchv) of one class; the caller keeps the sum of
// their batchv_blocks below 2^24 (the dispatch's work-item limit)
hipError_t launch_checksum_batchv(const BvSeg* b, int k, int cls, const void* zero16, hipStream_t st);
hipError_t launch_ipv4_batchv(const BvDgram* b, int k, int cls, int mode, const void* zero16, hipStream_t st);

// XCD-aware block order of k_checksum / k_ipv4_tcp launches (process-wide)
void set_xcd_remap(uint32_t run_log2);
hipError_t launch_fold(const uint32_t* sum, uint16_t* out, uint64_t n, hipStream_t st);
hipError_t launch_ipv4_tcp(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck,
                           uint8_t* status, Geometry g, uint32_t max_blocks, hipStream_t st);
// fused IPv4 + TCP for receive mixes: each block's datagrams of <= 64 bytes
// one per lane on one wave, the rest 16 lanes each claimed by every wave
// (k_ipv4_twoclass); spw (16 or 32) datagrams per wave in the bounds pass,
// i.e. 64 or 128 per block; lds_pad: bytes of dynamic LDS per block on top
// of the kernel's own (caps the blocks resident per CU; 0 in the default
// dispatch, ICSUM_FORCE twoclass_lds)
hipError_t launch_ipv4_twoclass(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status,
                                int spw, uint32_t remap, hipStream_t st, uint32_t lds_pad = 0);
hipError_t launch_router_ttl(const SegSpec& sp, uint8_t* status, hipStream_t st);
// the router step with the forwarded 20-byte headers to hdr_out (coalesced),
// the datagrams read only (k_router_hdrs)
hipError_t launch_router_hdrs(const SegSpec& sp, uint32_t* hdr_out, uint8_t* status, hipStream_t st);

// Tile launches of offsets batches (k_span): one wave per S (1..63)
// consecutive segments, the span's bytes streamed whole in 4 KiB windows
// whatever the lengths.  Checksum (out_kind as launch_checksum), the fused IPv4/TCP kernel
// (mode as launch_ipv4_tcp) and the in-place wrap (as launch_tcp_wrap in place).
// max_blocks (test hook ICSUM_FORCE span_blocks; 0: none): a grid of more
// blocks runs the grid-stride instantiation with that many, as batches of
// more spans than 2^24 blocks hold do.
hipError_t launch_tile_checksum(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out, int out_kind,
                                uint32_t S, hipStream_t st, uint32_t max_blocks = 0);
hipError_t launch_tile_ipv4(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status,
                            uint32_t S, hipStream_t st, uint32_t max_blocks = 0);

// Per-tick zero-copy host calls (k_tick): at most kTickSegs segments of an
// offsets batch in one block, the n + 1 offsets (relative to `bytes`) copied
// into the kernel arguments; op 0 checksum (u16 out, init nullable), op 1 the
// fused IPv4/TCP kernel (mode, the three outputs nullable).  `done` as the
// zero-copy launches take it.
constexpr uint32_t kTickSegs = 16;
struct TickOffsets {
  uint64_t o[kTickSegs + 1];
};
hipError_t launch_tick(const uint8_t* bytes, const uint64_t* offsets, uint32_t n, int op, const uint32_t* init,
                       uint16_t* out, int mode, uint16_t* ip_ck, uint16_t* tcp_ck, uint8_t* status,
                       const void* zero16, const Done& done, hipStream_t st);

// Resident tick server (k_tick_server): 1..kSrvBlocksMax blocks that stay
// resident, block b taking per-tick jobs from mailbox b of an array in
// coherent page-locked host memory (a tick of n segments: sub-jobs of <= 16
// in mailboxes 0 .. ceil(n / 16) - 1, each with its own sequence numbers).
// Descriptor word k = payload (low 32 bits) | job sequence number (high 32):
//   w[0] = op (0 checksum, 1 fused IPv4, 2 wrap) | mode << 4 | n << 8
//          (the sub-job's n <= kTickSegs) | inits in the descriptor << 16
//   w[kSrvPart] = the sub-job's first segment in the tick | the tick's n << 8
//          (results: value first + j of the tick's result arrays)
//   w[1], w[2] = the bytes' (device-visible) address, low / high half
//   w[3], w[4] = the wrap's message records (op 2)
//   w[5], w[6] = the result area: u16 x n values (op 0) or u16 ip, u16 tcp,
//                u8 status x n (op 1)
//   w[kSrvHead + 2 j], w[kSrvHead + 2 j + 1] = segment j's start (relative to
//                the bytes) and length
//   w[kSrvInit + j] = segment j's init (op 0 with w[0] bit 16 set: the inits
//                travel in the descriptor, not as a PCIe read of their own)
// Mailbox b = 64 descriptor words at words + 64 b (page-locked host memory,
// or with srv_vram uncached device memory the host writes through the BAR)
// and a TickMailbox in page-locked memory.  Mailbox 0's w[kSrvQuit] != 0:
// exit; block 0 sets w[kSrvExit] when it leaves and blocks b > 0 leave on
// seeing it.  Block b writes mailbox b's `done` (the last finished sequence
// number) and, when it exits, `state` = kSrvExited.
constexpr uint32_t kSrvHead = 7, kSrvInit = kSrvHead + 2 * kTickSegs, kSrvPart = kSrvInit + kTickSegs,
                   kSrvExit = 62, kSrvQuit = 63;
constexpr uint32_t kSrvBlocksMax = 8;  // ticks of up to 128 segments
constexpr uint32_t kSrvWords = 64;     // descriptor words per mailbox
constexpr uint64_t kSrvRunning = 1, kSrvExited = 2;
struct alignas(128) TickMailbox {
  uint64_t done;
  uint64_t state;
  uint64_t pad[14];
};
static_assert(kSrvPart < kSrvExit, "the descriptor fits below the exit and quit words");
hipError_t launch_tick_server(uint64_t* words, TickMailbox* mbs, uint32_t blocks, const void* zero16,
                              uint32_t idle_us, uint32_t pollers, hipStream_t st);

// Fields of one TCP message for the device-side wrap; layout of ics_tcp_msg
// (include/icsum.h), 28 bytes.
struct TcpMsg {
  uint32_t src, dst, seqno, ackno;
  uint16_t sport, dport, window;
  uint8_t flags, ttl;
  uint16_t id, reserved;
};
static_assert(sizeof(TcpMsg) == 28, "ics_tcp_msg layout");
// wrap_tcp_in_ip for a batch: headers + both checksums written in place, or
// to hdr_out (40 bytes per datagram) when it is not null; payload_only:
// segment i is the payload alone (no header room), hdr_out required.
// sums != nullptr (n words of scratch): two passes, the payload sums
// (k_tcp_wrap, pass-1 mode) then the headers (k_tcp_hdr); nullptr: the
// one-pass k_tcp_wrap
hipError_t launch_tcp_wrap(const SegSpec& sp, const TcpMsg* msgs, uint32_t* hdr_out, uint16_t* ip_ck,
                           uint16_t* tcp_ck, bool payload_only, uint32_t* sums, Geometry g, uint32_t max_blocks,
                           hipStream_t st);
// the wrap as a tile launch: in place (hdr_out null) or, with hdr_out, the
// payload-only batch of ics_tcp_wrap_headers with its headers to hdr_out
hipError_t launch_tile_wrap(const SegSpec& sp, const TcpMsg* msgs, uint32_t* hdr_out, uint16_t* ip_ck,
                            uint16_t* tcp_ck, uint32_t S, hipStream_t st, uint32_t max_blocks = 0);
// pass 2 of the two-pass wrap alone (k_tcp_hdr): headers from the records and
// the payload sums pass 1 left in `sums` (roles from each payload's start)
hipError_t launch_tcp_hdr(const SegSpec& sp, const TcpMsg* msgs, const uint32_t* sums, uint32_t* hdr_out,
                          uint16_t* ip_ck, uint16_t* tcp_ck, bool payload_only, hipStream_t st);

// bounds-checked build (libicsum_debug.so): synchronise `st` and take (read
// and clear) the device's violation record; flags 0 = clean.  No-op returning
// flags 0 in the release build.
bool bounds_checked_build();
hipError_t bounds_take(hipStream_t st, uint32_t* flags, uint64_t* what);

// synthetic workloads (icsum_workload.h)
hipError_t launch_fill_bytes(uint8_t* d, uint64_t nbytes, uint64_t seed, uint64_t pos0,
                             hipStream_t st);
hipError_t launch_pseudo_inits(uint32_t* init, const uint64_t* offsets, uint64_t seg_len,
                               uint64_t n, uint64_t seed, uint64_t index0, hipStream_t st);
hipError_t launch_ipv4_tcp_headers(uint8_t* d, uint64_t stride, uint64_t dgram_len, uint64_t n,
                                   uint64_t seed, uint64_t index0, hipStream_t st);

}  // namespace icsum
