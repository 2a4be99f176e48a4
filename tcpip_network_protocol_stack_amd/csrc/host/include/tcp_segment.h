// tcp_segment.h: include-name forwarder.  The stack #includes "tcp_segment.h" (reference
// util/tcp_segment/tcp_segment.h); the declarations live in icsum_wire.h.
#pragma once
#include "icsum_wire.h"
