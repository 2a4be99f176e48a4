// tcp_config.h — standalone stand-in for util/tools/tcp_config.h:11-42 (see
// udinfo.h in this directory for when it is used).  src/tcp_sender reads
// MAX_PAYLOAD_SIZE and the capacities; the values are the reference's.
#ifndef TCP_CONFIG_H
#define TCP_CONFIG_H

#include <cstddef>
#include <cstdint>

#include "address.h"
#include "wrapping_integers.h"

class TCPConfig
{
  public:
    static constexpr size_t DEFAULT_CAPACITY = 64000;
    static constexpr size_t MAX_PAYLOAD_SIZE = 1000;
    static constexpr uint16_t TIMEOUT_DFLT = 1000;
    static constexpr unsigned MAX_RETX_ATTEMPTS = 8;

    uint16_t rt_timeout = TIMEOUT_DFLT;
    size_t recv_capacity = DEFAULT_CAPACITY;
    size_t send_capacity = DEFAULT_CAPACITY;
    Wrap32 isn{137};
};

// the two endpoints the adapter filters on; the loss rates are read by the
// reference's LossyFdAdapter, which is not part of the standalone build
class FdAdapterConfig
{
  public:
    Address source{"0", 0};
    Address destination{"0", 0};
    uint16_t loss_rate_dn = 0;
    uint16_t loss_rate_up = 0;
};

#endif
