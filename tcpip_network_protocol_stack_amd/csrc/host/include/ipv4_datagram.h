// ipv4_datagram.h: include-name forwarder.  The stack #includes "ipv4_datagram.h" (reference
// util/tools/ipv4_datagram.h); the declarations live in icsum_wire.h.
#pragma once
#include "icsum_wire.h"
