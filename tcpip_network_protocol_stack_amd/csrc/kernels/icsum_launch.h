// icsum_launch.h — internal launcher interface between the C-ABI layer
// (icsum_api.cpp) and the HIP kernels (icsum_kernels.hip).  Not installed.
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
  int mode;  // chunk grid: 0 16-byte + boundary slot, 1 128-byte line, 2 16-byte all masked
  int segs = 1;  // > 1: small-segment kernel, SEGS segments per lane group in flight
};

// Pick a geometry from the (average) segment length in bytes.
Geometry pick_geometry(uint64_t avg_len);
bool geometry_supported(Geometry g);

struct SegSpec {
  const uint8_t* bytes;
  const uint64_t* offsets;  // n+1 or nullptr
  uint64_t stride;
  uint64_t seg_len;
  uint64_t n;
  const void* zero16;  // 16 zero bytes in device memory (stand-in for absent arrays)
  // length-binned launch: work items come from a bin list (16-byte entries,
  // see launch_bin_segments) of *count entries starting at entry *base;
  // n stays the batch size (an upper bound of *count)
  const void* list = nullptr;
  const uint32_t* count = nullptr;
  const uint32_t* base = nullptr;
};

// Length binning of an offsets batch (mixed segment sizes): every segment
// goes to the bin whose geometry suits its length, and each bin is run with
// its own geometry, reading its work list on the device.
//   list  n entries of 16 bytes ({start lo, start hi, length, segment};
//         length 0xFFFFFFFF = re-read the offsets), bins stored back to back
//   meta  kBinMetaWords uint32: [0, kBins) bin sizes, [8, 8 + kBins) cursors,
//         [16, 16 + kBins) bin bases (written by the scatter pass)
// Needs n < 2^32.  The launcher zeroes meta itself.
constexpr int kBins = 5;
constexpr int kBinMetaWords = 32;
hipError_t launch_bin_segments(const uint64_t* offsets, uint64_t n, void* list, uint32_t* meta,
                               hipStream_t st);
Geometry bin_geometry(int bin);
// bin b's launch spec: list = bin's entries, count = its size
SegSpec bin_spec(const SegSpec& whole, const void* list, const uint32_t* meta, int bin);

// out_kind 0: u16 value(), 1: u32 raw sum
hipError_t launch_checksum(const SegSpec& sp, const uint32_t* init, const uint8_t* odd, void* out,
                           int out_kind, Geometry g, uint32_t max_blocks, hipStream_t st);
hipError_t launch_fold(const uint32_t* sum, uint16_t* out, uint64_t n, hipStream_t st);
hipError_t launch_ipv4_tcp(const SegSpec& sp, int mode, uint16_t* ip_ck, uint16_t* tcp_ck,
                           uint8_t* status, Geometry g, uint32_t max_blocks, hipStream_t st);
hipError_t launch_router_ttl(const SegSpec& sp, uint8_t* status, hipStream_t st);

// synthetic workloads (icsum_workload.h)
hipError_t launch_fill_bytes(uint8_t* d, uint64_t nbytes, uint64_t seed, uint64_t pos0,
                             hipStream_t st);
hipError_t launch_pseudo_inits(uint32_t* init, const uint64_t* offsets, uint64_t seg_len,
                               uint64_t n, uint64_t seed, uint64_t index0, hipStream_t st);
hipError_t launch_ipv4_tcp_headers(uint8_t* d, uint64_t stride, uint64_t dgram_len, uint64_t n,
                                   uint64_t seed, uint64_t index0, hipStream_t st);

}  // namespace icsum
