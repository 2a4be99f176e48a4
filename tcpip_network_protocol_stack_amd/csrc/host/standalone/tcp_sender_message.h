// tcp_sender_message.h — standalone stand-in for util/tools/tcp_sender_message.h:25-40
// (see udinfo.h in this directory for when it is used).  Member order is the
// reference's: src/tcp_sender builds these by aggregate initialisation.
#ifndef TCP_SENDER_MESSAGE_H
#define TCP_SENDER_MESSAGE_H

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

    // SYN and FIN each occupy one sequence number
    size_t sequence_length() const { return static_cast<size_t>(SYN) + payload.size() + static_cast<size_t>(FIN); }
};

#endif
