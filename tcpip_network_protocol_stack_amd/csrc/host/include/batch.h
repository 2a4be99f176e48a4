// batch.h — batch entry points of the drop-in types, backed by the MI355X
// engine (libicsum.so, include/icsum.h).  These are the calls a busy stack
// makes instead of one compute_checksum()/parse() per object:
//
//   checksum()            InternetChecksum{init_i}.add(seg_i).value()     checksum.h:17-41
//   compute_checksums()   TCPSegment::compute_checksum(pseudo) per pair    tcp_segment.cpp:109-118
//                         IPv4Header::compute_checksum() per header        ipv4_header.cpp:113-123
//   verify_raw()          IPv4Header::parse + TCPSegment::parse checks     ipv4_header.cpp:9-59, tcp_segment.cpp:11-65
//   wrap()                TCPOverIPv4Adapter::wrap_tcp_in_ip per message   tcp_over_ip.cpp:69-88
//                         (headers + both checksums serialized on the GPU;
//                         payloads copied once, into the DMA arena)
//   unwrap()/unwrap_raw() TCPOverIPv4Adapter::unwrap_tcp_in_ip per datagram tcp_over_ip.cpp:10-67
//
// Results are bit-identical to the per-object calls.  All checksum arithmetic
// runs on the GPU; a BatchEngine cannot be constructed without one (there is
// no silent CPU fallback).  One engine per thread, or guard it externally.
#ifndef ICSUM_HOST_BATCH_H
#define ICSUM_HOST_BATCH_H

#include <cstdint>
#include <memory>
#include <optional>
#include <span>
#include <string>
#include <string_view>
#include <vector>

#include "icsum.h"
#include "ipv4_datagram.h"
#include "ipv4_header.h"
#include "tcp_over_ip.h"
#include "tcp_segment.h"

namespace icsum {

namespace detail {
class WorkerPool;  // par_for.h
}

// The fields wrap_tcp_in_ip puts on the wire for `msg` from an adapter with
// configuration `cfg` (tcp_over_ip.cpp:71-80, tcp_segment.cpp:76-106): the
// record the device-side wrap (ics_tcp_wrap_batch) serializes.
ics_tcp_msg wrap_fields(const FdAdapterConfig& cfg, const TCPMessage& msg);

class BatchEngine
{
  public:
    explicit BatchEngine(int device = 0);  // throws std::runtime_error without a usable GPU
    ~BatchEngine();
    BatchEngine(const BatchEngine&) = delete;
    BatchEngine& operator=(const BatchEngine&) = delete;

    std::vector<uint16_t> checksum(std::span<const std::string_view> segs, std::span<const uint32_t> init = {});
    void compute_checksums(std::span<TCPSegment> segs, std::span<const IPv4Header> hdrs);
    void compute_checksums(std::span<IPv4Header> hdrs);
    // ICS_ST_* status bits per raw wire datagram (ICS_ST_ACCEPT = all parse checks pass)
    std::vector<uint8_t> verify_raw(std::span<const std::string_view> wires);
    std::vector<InternetDatagram> wrap(TCPOverIPv4Adapter& adapter, std::span<const TCPMessage> msgs);
    // the same, consuming the messages: each payload string is moved into its
    // datagram after the one copy into the arena
    std::vector<InternetDatagram> wrap(TCPOverIPv4Adapter& adapter, std::vector<TCPMessage>&& msgs);
    std::vector<std::optional<TCPMessage>> unwrap(TCPOverIPv4Adapter& adapter,
                                                  std::span<const InternetDatagram> dgrams);
    std::vector<std::optional<TCPMessage>> unwrap_raw(TCPOverIPv4Adapter& adapter,
                                                      std::span<const std::string_view> wires);

    // the same operations on an already packed batch (bytes + n+1 offsets),
    // e.g. a DatagramBatch arena in page-locked memory: no packing copy
    std::vector<uint8_t> verify_packed(const uint8_t* bytes, const uint64_t* offsets, size_t n);
    void patch_packed(uint8_t* bytes, const uint64_t* offsets, size_t n);  // compute + store both checksums
    // device-side wrap of a packed batch: datagram i = [40 B room][payload i],
    // headers + both checksums written into `bytes` (ics_tcp_wrap_batch_host)
    void wrap_packed(uint8_t* bytes, const uint64_t* offsets, const ics_tcp_msg* msgs, size_t n);
    std::vector<std::optional<TCPMessage>> unwrap_packed(TCPOverIPv4Adapter& adapter, const uint8_t* bytes,
                                                         const uint64_t* offsets, size_t n);

    // the resident tick server (ics_set_tick_server): a per-tick loop's calls
    // of <= 16 x blocks datagrams without a kernel launch each; 0 turns it
    // off; blocks 1..8 (ics_set_tick_server_blocks, default 4)
    void set_tick_server(uint32_t idle_us);
    void set_tick_server_blocks(uint32_t blocks);

    // page-locked host memory from the engine's device runtime
    void* host_alloc(size_t bytes);
    void host_free(void* p);

    int device() const { return device_; }

  private:
    template <typename Msgs, typename Take>
    std::vector<InternetDatagram> wrap_impl(const TCPOverIPv4Adapter& adapter, Msgs& msgs, Take take_payload);
    uint8_t* scratch(size_t bytes);  // page-locked arena reused across calls
    template <typename Fn>
    void ranges(size_t n, Fn&& fn);  // fn(i0, i1) over [0, n) on up to 8 of the engine's threads
    template <typename Len, typename Put>
    std::vector<uint64_t> pack(size_t n, Len len, Put put);  // n items into scratch(), offsets back

    ics_ctx* ctx_ = nullptr;
    int device_ = 0;
    uint8_t* scratch_ = nullptr;
    size_t scratch_cap_ = 0;
    std::unique_ptr<detail::WorkerPool> pool_{};  // ranges()' workers, started on first use
};

}  // namespace icsum

#endif
