// tcp_segment.h — drop-in TCPSegment / TCPMessage (reference:
// util/tcp_segment/tcp_segment.h:10-30).  Same names, members and methods;
// parse() checks InternetChecksum{pseudo} over ALL bytes it is handed before it
// reads a field, compute_checksum() stores exactly what the engine's COMPUTE
// mode produces (src/tcp_segment.cpp).  The message types come from the
// reference's own util/tools headers when integrated.
//
// Byte map of one TCP-in-IPv4 datagram as the device kernels see it
// (k_ipv4_tcp, csrc/kernels/icsum_kernels.hip), with the member that owns
// each field:
//
//   IPv4 [0,20)   IPv4Header                     (ipv4_header.h)
//   TCP  [0,2)    UserDatagramInfo::src_port
//        [2,4)    UserDatagramInfo::dst_port
//        [4,8)    TCPSenderMessage::seqno        raw Wrap32
//        [8,12)   TCPReceiverMessage::ackno      0 when absent
//        [12]     data offset << 4               always 5 when serialized
//        [13]     flags  ACK 0x10  RST 0x04  SYN 0x02  FIN 0x01
//        [14,16)  TCPReceiverMessage::window_size
//        [16,18)  UserDatagramInfo::cksum        the engine's tcp_ck output
//        [18,20)  urgent pointer                 always 0
//        [20,..)  TCPSenderMessage::payload
#ifndef TCP_SEGMENT_H  // the reference header's guard: either one defines TCPSegment
#define TCP_SEGMENT_H

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
