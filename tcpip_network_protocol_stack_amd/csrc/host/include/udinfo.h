// udinfo.h: include-name forwarder.  The stack #includes "udinfo.h" (reference
// util/tools/udinfo.h); the declarations live in icsum_wire.h.
#pragma once
#include "icsum_wire.h"
