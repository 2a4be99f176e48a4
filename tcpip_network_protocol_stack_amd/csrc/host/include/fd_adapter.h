// fd_adapter.h — adapter configuration base (reference: util/tools/fd_adapter.h:13-38,
// util/tools/tcp_config.h:30-42) without the fd / lossy-adapter runtime, which
// is out of this engine's scope.
#ifndef ICSUM_HOST_FD_ADAPTER_H
#define ICSUM_HOST_FD_ADAPTER_H

#include <cstddef>
#include <cstdint>

#include "tcp_config.h"

class FdAdapterBase
{
  private:
    FdAdapterConfig _cfg{};
    bool _listen = false;

  protected:
    FdAdapterConfig& config_mutable() { return _cfg; }

  public:
    void set_listening(const bool l) { _listen = l; }
    bool listening() const { return _listen; }
    const FdAdapterConfig& config() const { return _cfg; }
    FdAdapterConfig& config_mut() { return _cfg; }
    void tick(const size_t unused [[maybe_unused]]) {}
};

#endif
