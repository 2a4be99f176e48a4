// tcp_segment.cpp — drop-in TCPSegment (reference: util/tcp_segment/tcp_segment.cpp:9-118).
// parse() first verifies InternetChecksum{pseudo} over ALL remaining bytes
// (value() != 0 -> error) and only then reads fields; serialize() always
// writes a 20-byte header (data offset 5, no options); compute_checksum()
// sums that header with cksum = 0 plus the payload, seeded with the pseudo sum.
#include "tcp_segment.h"

#include <algorithm>

#include "checksum.h"
#include "wire_internal.h"

namespace {
constexpr uint8_t kMinDataOffset = 5;  // 32-bit words

struct WrapRaw : Wrap32
{
    explicit WrapRaw(const Wrap32& w) : Wrap32(w) {}
    uint32_t raw() const { return raw_value_; }
};

uint8_t flags_of(const TCPMessage& m)
{
    return static_cast<uint8_t>((m.receiver.ackno.has_value() ? 0x10U : 0U) |
                                (m.sender.RST || m.receiver.RST ? 0x04U : 0U) | (m.sender.SYN ? 0x02U : 0U) |
                                (m.sender.FIN ? 0x01U : 0U));
}

// the 20 header bytes serialize() emits
void header_bytes(const TCPSegment& s, char* b)
{
    auto put16 = [&](int at, uint16_t v) {
        b[at] = static_cast<char>(v >> 8);
        b[at + 1] = static_cast<char>(v);
    };
    auto put32 = [&](int at, uint32_t v) {
        put16(at, static_cast<uint16_t>(v >> 16));
        put16(at + 2, static_cast<uint16_t>(v));
    };
    put16(0, s.udinfo.src_port);
    put16(2, s.udinfo.dst_port);
    put32(4, WrapRaw{s.message.sender.seqno}.raw());
    put32(8, WrapRaw{s.message.receiver.ackno.value_or(Wrap32{0})}.raw());
    b[12] = static_cast<char>(kMinDataOffset << 4);
    b[13] = static_cast<char>(flags_of(s.message));
    put16(14, s.message.receiver.window_size);
    put16(16, s.udinfo.cksum);
    put16(18, 0);  // urgent pointer
}
}  // namespace

namespace icsum::detail {
uint32_t raw_of(const Wrap32& w) { return WrapRaw{w}.raw(); }

void tcp_header_bytes(const TCPSegment& seg, char* b) { header_bytes(seg, b); }

void parse_tcp_fields(Parser& parser, TCPSegment& seg)
{
    uint32_t raw32 = 0;
    uint16_t urgent = 0;
    uint8_t octet = 0;
    parser.integer(seg.udinfo.src_port);
    parser.integer(seg.udinfo.dst_port);
    parser.integer(raw32);
    seg.message.sender.seqno = Wrap32{raw32};
    parser.integer(raw32);
    seg.message.receiver.ackno = Wrap32{raw32};
    parser.integer(octet);
    const uint8_t data_offset = octet >> 4;
    parser.integer(octet);
    if (!(octet & 0x10)) seg.message.receiver.ackno.reset();
    seg.message.sender.RST = seg.message.receiver.RST = (octet & 0x04) != 0;
    seg.message.sender.SYN = (octet & 0x02) != 0;
    seg.message.sender.FIN = (octet & 0x01) != 0;
    parser.integer(seg.message.receiver.window_size);
    parser.integer(seg.udinfo.cksum);
    parser.integer(urgent);
    if (data_offset < kMinDataOffset) {
        parser.set_error();
        parser.remove_prefix(~size_t{0});  // the reference's negative skip swallows the rest
    } else {
        parser.remove_prefix(static_cast<size_t>(data_offset - kMinDataOffset) * 4);  // options
    }
    parser.all_remaining(seg.message.sender.payload);
}
bool parse_tcp_fields(std::string_view b, TCPSegment& seg)
{
    if (b.size() < 20) return false;
    auto u8 = [&](size_t k) { return static_cast<uint8_t>(b[k]); };
    auto be16 = [&](size_t k) { return static_cast<uint16_t>((u8(k) << 8) | u8(k + 1)); };
    auto be32 = [&](size_t k) { return (static_cast<uint32_t>(be16(k)) << 16) | be16(k + 2); };
    seg.udinfo.src_port = be16(0);
    seg.udinfo.dst_port = be16(2);
    seg.message.sender.seqno = Wrap32{be32(4)};
    seg.message.receiver.ackno = Wrap32{be32(8)};
    const uint8_t data_offset = u8(12) >> 4;
    const uint8_t flags = u8(13);
    if (!(flags & 0x10)) seg.message.receiver.ackno.reset();
    seg.message.sender.RST = seg.message.receiver.RST = (flags & 0x04) != 0;
    seg.message.sender.SYN = (flags & 0x02) != 0;
    seg.message.sender.FIN = (flags & 0x01) != 0;
    seg.message.receiver.window_size = be16(14);
    seg.udinfo.cksum = be16(16);
    if (data_offset < kMinDataOffset) return false;
    // options past the end: the Parser's skip stops at the end without an
    // error, and the payload is empty (parser.h remove_prefix)
    const size_t hdr = std::min(static_cast<size_t>(data_offset) * 4, b.size());
    seg.message.sender.payload.assign(b.data() + hdr, b.size() - hdr);
    return true;
}
}  // namespace icsum::detail

void TCPSegment::parse(Parser& parser, uint32_t datagram_layer_pseudo_checksum)
{
    InternetChecksum check{datagram_layer_pseudo_checksum};
    check.add(parser.buffer());
    if (check.value()) {
        parser.set_error();
        return;
    }
    icsum::detail::parse_tcp_fields(parser, *this);
}

void TCPSegment::serialize(Serializer& serializer) const
{
    char b[20];
    header_bytes(*this, b);
    for (char c : b) serializer.integer(static_cast<uint8_t>(c));
    serializer.buffer(message.sender.payload);
}

void TCPSegment::compute_checksum(uint32_t datagram_layer_pseudo_checksum)
{
    udinfo.cksum = 0;
    char b[20];
    header_bytes(*this, b);
    InternetChecksum check{datagram_layer_pseudo_checksum};
    check.add(std::string_view{b, 20});  // even length: the payload starts on a high byte
    check.add(std::string_view{message.sender.payload});
    udinfo.cksum = check.value();
}
