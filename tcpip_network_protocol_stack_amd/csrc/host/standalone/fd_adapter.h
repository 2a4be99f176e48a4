// fd_adapter.h — standalone stand-in for util/tools/fd_adapter.h:13-38 (see
// udinfo.h in this directory for when it is used): the adapter's state, i.e.
// the endpoint configuration and the listen flag.  The reference's header
// also pulls in its file-descriptor, socket and lossy-adapter runtime; with
// the reference tree present that header is used unchanged.
#ifndef FD_ADAPTER_H
#define FD_ADAPTER_H

#include <cstddef>

#include "tcp_config.h"
#include "tcp_segment.h"

class FdAdapterBase
{
    FdAdapterConfig endpoints_{};
    bool listen_ = false;

  protected:
    FdAdapterConfig& config_mutable() { return endpoints_; }

  public:
    void set_listening(const bool l) { listen_ = l; }
    bool listening() const { return listen_; }
    const FdAdapterConfig& config() const { return endpoints_; }
    FdAdapterConfig& config_mut() { return endpoints_; }
    void tick(const size_t /*ms_since_last_tick*/) {}
};

#endif
