// tcp_over_ip.cpp — drop-in TCPOverIPv4Adapter (reference: util/tcp_over_ip/tcp_over_ip.cpp:10-88).
#include "tcp_over_ip.h"

#include "ipv4_header.h"
#include "parser.h"

std::optional<TCPMessage> TCPOverIPv4Adapter::unwrap_tcp_in_ip(const InternetDatagram& ip_dgram)
{
    // address filters (binding to "0" accepts any destination when listening)
    if (!listening() && ip_dgram.header.dst != config().source.ipv4_numeric()) return {};
    if (!listening() && ip_dgram.header.src != config().destination.ipv4_numeric()) return {};
    if (ip_dgram.header.proto != IPv4Header::PROTO_TCP) return {};
    TCPSegment seg;
    if (!parse(seg, ip_dgram.payload, ip_dgram.header.pseudo_checksum())) return {};  // checksum + header
    if (seg.udinfo.dst_port != config().source.port()) return {};
    if (listening()) {
        if (!seg.message.sender.SYN || seg.message.sender.RST) return {};
        config_mutable().source = Address{Address::from_ipv4_numeric(ip_dgram.header.dst).ip(), config().source.port()};
        config_mutable().destination = Address{Address::from_ipv4_numeric(ip_dgram.header.src).ip(), seg.udinfo.src_port};
        set_listening(false);
    }
    if (seg.udinfo.src_port != config().destination.port()) return {};
    return seg.message;
}

InternetDatagram TCPOverIPv4Adapter::wrap_tcp_in_ip(const TCPMessage& msg)
{
    TCPSegment seg{.message = msg, .udinfo = {}};
    seg.udinfo.src_port = config().source.port();
    seg.udinfo.dst_port = config().destination.port();
    InternetDatagram ip_dgram;
    ip_dgram.header.src = config().source.ipv4_numeric();
    ip_dgram.header.dst = config().destination.ipv4_numeric();
    ip_dgram.header.len = static_cast<uint16_t>(ip_dgram.header.hlen * 4 + 20 + seg.message.sender.payload.size());
    seg.compute_checksum(ip_dgram.header.pseudo_checksum());
    ip_dgram.header.compute_checksum();
    ip_dgram.payload = serialize(seg);
    return ip_dgram;
}
