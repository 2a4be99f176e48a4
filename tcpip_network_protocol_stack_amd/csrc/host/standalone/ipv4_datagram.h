// ipv4_datagram.h — standalone stand-in for util/tools/ipv4_datagram.h:10-34
// (see udinfo.h in this directory for when it is used): a header plus its
// payload pieces, kept as the Parser hands them over.
#ifndef IPV4_DATAGRAM_H
#define IPV4_DATAGRAM_H

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
        serializer.buffer(payload);
    }
};

using InternetDatagram = IPv4Datagram;

#endif
