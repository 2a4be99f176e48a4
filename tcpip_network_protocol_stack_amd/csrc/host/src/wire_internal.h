// wire_internal.h — not installed.  Pieces of the per-object codec that the
// batch engine (batch.cpp) shares, so a batch applies exactly the rules the
// per-object calls do; the GPU only takes over the checksum arithmetic.
#pragma once

#include <cstdint>
#include <optional>
#include <string_view>

#include "tcp_over_ip.h"

namespace icsum::detail {

// tcp_segment.cpp:25-65: header fields, flags, data offset, payload (the
// half of TCPSegment::parse after its checksum check)
void parse_tcp_fields(Parser& parser, TCPSegment& seg);
// the same over one contiguous buffer (the segment's bytes): false where the
// Parser would have flagged an error (fewer than 20 bytes, data offset < 5);
// the payload is copied once
bool parse_tcp_fields(std::string_view bytes, TCPSegment& seg);
uint32_t raw_of(const Wrap32& w);
// the 20 header bytes TCPSegment::serialize emits first (tcp_segment.cpp:76-106)
void tcp_header_bytes(const TCPSegment& seg, char* b);

// tcp_over_ip.cpp:14-29 — before any TCP byte is looked at: a connected
// adapter only takes datagrams from its peer to itself, and only TCP
bool ip_gate(const FdAdapterBase& adapter, const IPv4Header& h);

// tcp_over_ip.cpp:39-64 — after a clean parse: destination port, the
// listen -> connected transition on a SYN without RST (which rewrites the
// adapter's endpoints), then the source port
std::optional<TCPMessage> tcp_gate(FdAdapterBase& adapter, const IPv4Header& h, const TCPSegment& seg);
// the same, moving the message (and its payload) out of `seg` when it passes
std::optional<TCPMessage> tcp_gate(FdAdapterBase& adapter, const IPv4Header& h, TCPSegment&& seg);

// tcp_over_ip.cpp:71-80 — the ports, addresses and total length wrap sets
// before either checksum is computed (checksum fields are left at 0)
void stamp_outgoing(const FdAdapterConfig& cfg, const TCPMessage& msg, IPv4Header& h, TCPSegment& seg);

}  // namespace icsum::detail
