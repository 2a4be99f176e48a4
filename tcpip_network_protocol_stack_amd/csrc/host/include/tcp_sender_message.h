// tcp_sender_message.h — reference: util/tools/tcp_sender_message.h:25-40
#ifndef ICSUM_HOST_TCP_SENDER_MESSAGE_H
#define ICSUM_HOST_TCP_SENDER_MESSAGE_H

#include <cstddef>
#include <string>

#include "wrapping_integers.h"

struct TCPSenderMessage
{
    Wrap32 seqno{0};
    bool SYN{};
    std::string payload{};
    bool FIN{};
    bool RST{};

    size_t sequence_length() const { return SYN + payload.size() + FIN; }
};

#endif
