// <mscclpp/proxy.hpp> on this library: Proxy / ProxyHandlerResult.
// A caller written against the reference's include/mscclpp/proxy.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/proxy.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_PROXY_HPP_
#define MSCCLPP_AMD_FWD_PROXY_HPP_

#include "mscclpp_amd/proxy.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_PROXY_HPP_
