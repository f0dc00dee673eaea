// Host utilities with the reference's spellings (include/mscclpp/utils.hpp, src/core/utils.cc:13-22).
// getHostName is the reference's (the host name up to the first `delim`, at most maxlen - 1
// characters); the InfiniBand queries answer for a build whose only transport is CudaIpc over xGMI:
// no IB devices, and naming one is an InvalidUsage error.  Fabric memory handles are an NVLink
// feature: not available.
#pragma once

#include <unistd.h>

#include <functional>
#include <string>

#include "mscclpp_amd/core.hpp"

namespace mscclpp_amd {

namespace detail {
// boost::hash_combine (utils.hpp:14-21)
template <typename T>
inline void hashCombine(std::size_t& seed, const T& value) {
  std::hash<T> hasher;
  seed ^= hasher(value) + 0x9e3779b9 + (seed << 6) + (seed >> 2);
}
}  // namespace detail

inline std::string getHostName(int maxlen, const char delim) {
  std::string hostname(maxlen + 1, '\0');
  if (gethostname(&hostname[0], maxlen) != 0) throw Error("gethostname failed", ErrorCode::SystemError);
  int i = 0;
  while (hostname[i] != delim && hostname[i] != '\0' && i < maxlen - 1) ++i;
  return hostname.substr(0, i);
}

inline int getIBDeviceCount() { return 0; }
inline std::string getIBDeviceName(Transport) {
  throw Error("no InfiniBand transport on this build (CudaIpc over xGMI only)", ErrorCode::InvalidUsage);
}
inline Transport getIBTransportByDeviceName(const std::string& name) {
  throw Error("no InfiniBand device " + name + " on this build (CudaIpc over xGMI only)", ErrorCode::InvalidUsage);
}
inline bool isFabricMemHandleAvailable() { return false; }

}  // namespace mscclpp_amd
