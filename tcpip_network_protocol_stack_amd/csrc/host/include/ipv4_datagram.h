// ipv4_datagram.h — reference: util/tools/ipv4_datagram.h:10-34
#ifndef ICSUM_HOST_IPV4_DATAGRAM_H
#define ICSUM_HOST_IPV4_DATAGRAM_H

#include <string>
#include <vector>

#include "ipv4_header.h"
#include "parser.h"

struct IPv4Datagram
{
    IPv4Header header{};
    std::vector<std::string> payload{};

    void parse(Parser& parser)
    {
        header.parse(parser);
        parser.all_remaining(payload);
    }

    void serialize(Serializer& serializer) const
    {
        header.serialize(serializer);
        for (const auto& x : payload) serializer.buffer(x);
    }
};

using InternetDatagram = IPv4Datagram;

#endif
