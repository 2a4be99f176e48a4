// tcp_over_ip.cpp — TCPOverIPv4Adapter on the host, one datagram at a time
// (reference util/tcp_over_ip/tcp_over_ip.cpp:10-88).
//
// The adapter's admission rules are written once, as the three steps in
// wire_internal.h, and used both here and by icsum::BatchEngine: the batch
// path differs only in where the checksum arithmetic runs.
#include "tcp_over_ip.h"

#include "wire_internal.h"

namespace icsum::detail {

bool ip_gate(const FdAdapterBase& adapter, const IPv4Header& h)
{
    // a listening adapter bound to "0" accepts any destination and learns the
    // peer from the first SYN (tcp_gate); a connected one is pinned to it
    if (!adapter.listening()) {
        const FdAdapterConfig& cfg = adapter.config();
        if (h.dst != cfg.source.ipv4_numeric()) return false;
        if (h.src != cfg.destination.ipv4_numeric()) return false;
    }
    return h.proto == IPv4Header::PROTO_TCP;
}

namespace {
bool tcp_gate_ok(FdAdapterBase& adapter, const IPv4Header& h, const TCPSegment& seg)
{
    const uint16_t local_port = adapter.config().source.port();
    if (seg.udinfo.dst_port != local_port) return false;
    if (adapter.listening()) {
        const TCPSenderMessage& s = seg.message.sender;
        if (!s.SYN || s.RST) return false;  // only a clean SYN opens the connection
        FdAdapterConfig& cfg = adapter.config_mut();
        cfg.source = Address{Address::from_ipv4_numeric(h.dst).ip(), local_port};
        cfg.destination = Address{Address::from_ipv4_numeric(h.src).ip(), seg.udinfo.src_port};
        adapter.set_listening(false);
    }
    return seg.udinfo.src_port == adapter.config().destination.port();
}
}  // namespace

std::optional<TCPMessage> tcp_gate(FdAdapterBase& adapter, const IPv4Header& h, const TCPSegment& seg)
{
    if (!tcp_gate_ok(adapter, h, seg)) return std::nullopt;
    return seg.message;
}

std::optional<TCPMessage> tcp_gate(FdAdapterBase& adapter, const IPv4Header& h, TCPSegment&& seg)
{
    if (!tcp_gate_ok(adapter, h, seg)) return std::nullopt;
    return std::move(seg.message);
}

void stamp_outgoing(const FdAdapterConfig& cfg, const TCPMessage& msg, IPv4Header& h, TCPSegment& seg)
{
    seg.message = msg;
    seg.udinfo = UserDatagramInfo{cfg.source.port(), cfg.destination.port(), 0};
    h.src = cfg.source.ipv4_numeric();
    h.dst = cfg.destination.ipv4_numeric();
    constexpr size_t kTcpHeaderBytes = 20;  // serialize() never writes TCP options
    h.len = static_cast<uint16_t>(4U * h.hlen + kTcpHeaderBytes + msg.sender.payload.size());
}

}  // namespace icsum::detail

std::optional<TCPMessage> TCPOverIPv4Adapter::unwrap_tcp_in_ip(const InternetDatagram& ip_dgram)
{
    const IPv4Header& h = ip_dgram.header;
    if (!icsum::detail::ip_gate(*this, h)) return std::nullopt;
    TCPSegment seg;
    // checksum over pseudo header + every payload byte, then the fields
    if (!parse(seg, ip_dgram.payload, h.pseudo_checksum())) return std::nullopt;
    return icsum::detail::tcp_gate(*this, h, seg);
}

InternetDatagram TCPOverIPv4Adapter::wrap_tcp_in_ip(const TCPMessage& msg)
{
    InternetDatagram out;
    TCPSegment seg;
    icsum::detail::stamp_outgoing(config(), msg, out.header, seg);
    // TCP first: its pseudo sum reads len, which the IPv4 checksum then covers
    seg.compute_checksum(out.header.pseudo_checksum());
    out.header.compute_checksum();
    out.payload = serialize(seg);
    return out;
}
