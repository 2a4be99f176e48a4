// tcp_segment.h — drop-in TCPMessage / TCPSegment (reference: util/tcp_segment/tcp_segment.h:10-30)
#ifndef ICSUM_HOST_TCP_SEGMENT_H
#define ICSUM_HOST_TCP_SEGMENT_H

#include <cstdint>

#include "parser.h"
#include "tcp_receiver_message.h"
#include "tcp_sender_message.h"
#include "udinfo.h"

struct TCPMessage
{
    TCPSenderMessage sender{};
    TCPReceiverMessage receiver{};
};

struct TCPSegment
{
    TCPMessage message{};
    UserDatagramInfo udinfo{};

    void parse(Parser& parser, uint32_t datagram_layer_pseudo_checksum);
    void serialize(Serializer& serializer) const;
    void compute_checksum(uint32_t datagram_layer_pseudo_checksum);
};

#endif
