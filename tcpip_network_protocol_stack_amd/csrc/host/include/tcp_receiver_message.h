// tcp_receiver_message.h — reference: util/tools/tcp_receiver_message.h:22-27
#ifndef ICSUM_HOST_TCP_RECEIVER_MESSAGE_H
#define ICSUM_HOST_TCP_RECEIVER_MESSAGE_H

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
