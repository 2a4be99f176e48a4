// tcp_over_ip.h: include-name forwarder.  The stack #includes "tcp_over_ip.h" (reference
// util/tcp_over_ip/tcp_over_ip.h); the declarations live in icsum_wire.h.
#pragma once
#include "icsum_wire.h"
