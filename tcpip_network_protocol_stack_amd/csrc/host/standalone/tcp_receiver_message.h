// tcp_receiver_message.h — standalone stand-in for util/tools/tcp_receiver_message.h:22-27
// (see udinfo.h in this directory for when it is used).
#ifndef TCP_RECEIVER_MESSAGE_H
#define TCP_RECEIVER_MESSAGE_H

#include <cstdint>
#include <optional>

#include "wrapping_integers.h"

struct TCPReceiverMessage
{
    std::optional<Wrap32> ackno{};
    uint16_t window_size{};
    bool RST{};
};

#endif
