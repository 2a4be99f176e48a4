// fd_adapter.h: include-name forwarder.  The stack #includes "fd_adapter.h" (reference
// util/tools/fd_adapter.h); the declarations live in icsum_wire.h.
#pragma once
#include "icsum_wire.h"
