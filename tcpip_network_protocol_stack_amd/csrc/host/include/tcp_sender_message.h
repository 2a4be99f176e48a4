// tcp_sender_message.h: include-name forwarder.  The stack #includes "tcp_sender_message.h" (reference
// util/tools/tcp_sender_message.h); the declarations live in icsum_wire.h.
#pragma once
#include "icsum_wire.h"
