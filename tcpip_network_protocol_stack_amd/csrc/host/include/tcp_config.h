// tcp_config.h: include-name forwarder.  The stack #includes "tcp_config.h" (reference
// util/tools/tcp_config.h); the declarations live in icsum_wire.h.
#pragma once
#include "icsum_wire.h"
