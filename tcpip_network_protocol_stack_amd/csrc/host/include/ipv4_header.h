// ipv4_header.h — drop-in IPv4Header (reference: util/ipv4_header/ipv4_header.h:10-70).
// Same fields, defaults and methods; parse() verifies the header checksum with
// the reference's exact rules (see ipv4_header.cpp).
#ifndef IPV4_HEADER_H  // the reference header's guard
#define IPV4_HEADER_H

#include <cstddef>
#include <cstdint>
#include <string>

#include "parser.h"

struct IPv4Header
{
    static constexpr size_t LENGTH = 20;
    static constexpr uint8_t DEFAULT_TTL = 128;
    static constexpr uint8_t PROTO_TCP = 6;

    static constexpr uint64_t serialized_length() { return LENGTH; }

    uint8_t ver = 4;
    uint8_t hlen = LENGTH / 4;
    uint8_t tos = 0;
    uint16_t len = 0;
    uint16_t id = 0;
    bool df = true;
    bool mf = false;
    uint16_t offset = 0;
    uint8_t ttl = DEFAULT_TTL;
    uint8_t proto = PROTO_TCP;
    uint16_t cksum = 0;
    uint32_t src = 0;  // host order
    uint32_t dst = 0;  // host order

    uint16_t payload_length() const;
    uint32_t pseudo_checksum() const;
    void compute_checksum();
    std::string to_string() const;
    void parse(Parser& parser);
    void serialize(Serializer& serializer) const;
};

#endif
