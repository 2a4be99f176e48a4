// ipv4_header.cpp — drop-in IPv4Header (reference: util/ipv4_header/ipv4_header.cpp:9-123).
// Reference quirks kept on purpose (they decide which datagrams the stack
// accepts): the reserved flag bit 0x8000 is dropped when serializing, the
// checksum covers the 20 serialized bytes only (never options), and parse()
// compares the recomputed value with the wire value (a wire 0xFFFF is
// rejected where the computation yields 0x0000).
#include "ipv4_header.h"

#include <arpa/inet.h>

#include <sstream>
#include <stdexcept>

#include "checksum.h"

namespace {
void put16(char* p, uint16_t v)
{
    p[0] = static_cast<char>(v >> 8);
    p[1] = static_cast<char>(v);
}
void put32(char* p, uint32_t v)
{
    put16(p, static_cast<uint16_t>(v >> 16));
    put16(p + 2, static_cast<uint16_t>(v));
}
}  // namespace

void IPv4Header::parse(Parser& parser)
{
    uint8_t first = 0;
    parser.integer(first);
    ver = first >> 4;
    hlen = first & 0x0f;
    parser.integer(tos);
    parser.integer(len);
    parser.integer(id);
    uint16_t fo = 0;
    parser.integer(fo);
    df = (fo & 0x4000) != 0;
    mf = (fo & 0x2000) != 0;
    offset = fo & 0x1fff;
    parser.integer(ttl);
    parser.integer(proto);
    parser.integer(cksum);
    parser.integer(src);
    parser.integer(dst);
    if (ver != 4 || hlen < 5) parser.set_error();
    if (parser.has_error()) return;
    parser.remove_prefix(static_cast<uint64_t>(hlen) * 4 - LENGTH);  // options are skipped
    const uint16_t given = cksum;
    compute_checksum();
    if (cksum != given) parser.set_error();
}

void IPv4Header::serialize(Serializer& serializer) const
{
    if (ver != 4) throw std::runtime_error("wrong IP version");
    serializer.integer(static_cast<uint8_t>((static_cast<uint32_t>(ver) << 4) | (hlen & 0xfU)));
    serializer.integer(tos);
    serializer.integer(len);
    serializer.integer(id);
    serializer.integer(static_cast<uint16_t>((df ? 0x4000U : 0U) | (mf ? 0x2000U : 0U) | (offset & 0x1fffU)));
    serializer.integer(ttl);
    serializer.integer(proto);
    serializer.integer(cksum);
    serializer.integer(src);
    serializer.integer(dst);
}

uint16_t IPv4Header::payload_length() const { return static_cast<uint16_t>(len - 4 * hlen); }

uint32_t IPv4Header::pseudo_checksum() const
{
    uint32_t p = (src >> 16) + static_cast<uint16_t>(src);
    p += (dst >> 16) + static_cast<uint16_t>(dst);
    p += proto;
    p += payload_length();
    return p;
}

void IPv4Header::compute_checksum()
{
    // the 20 bytes serialize() would emit, with cksum = 0, summed in place
    if (ver != 4) throw std::runtime_error("wrong IP version");
    char b[LENGTH];
    b[0] = static_cast<char>((static_cast<uint32_t>(ver) << 4) | (hlen & 0xfU));
    b[1] = static_cast<char>(tos);
    put16(b + 2, len);
    put16(b + 4, id);
    put16(b + 6, static_cast<uint16_t>((df ? 0x4000U : 0U) | (mf ? 0x2000U : 0U) | (offset & 0x1fffU)));
    b[8] = static_cast<char>(ttl);
    b[9] = static_cast<char>(proto);
    put16(b + 10, 0);
    put32(b + 12, src);
    put32(b + 16, dst);
    InternetChecksum c;
    c.add(std::string_view{b, LENGTH});
    cksum = c.value();
}

std::string IPv4Header::to_string() const
{
    in_addr s{}, d{};
    s.s_addr = htonl(src);
    d.s_addr = htonl(dst);
    char sb[INET_ADDRSTRLEN] = {}, db[INET_ADDRSTRLEN] = {};
    inet_ntop(AF_INET, &s, sb, sizeof sb);
    inet_ntop(AF_INET, &d, db, sizeof db);
    std::ostringstream ss;
    ss << "IPv" << +ver << " len=" << +len << " protocol=" << +proto << " ttl=" << +ttl << " src=" << sb
       << " dst=" << db;
    return ss.str();
}
