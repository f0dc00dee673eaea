// <mscclpp/port_channel.hpp> on this library: ProxyService / PortChannel / BasePortChannel.
// A caller written against the reference's include/mscclpp/port_channel.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/port_channel.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_PORT_CHANNEL_HPP_
#define MSCCLPP_AMD_FWD_PORT_CHANNEL_HPP_

#include "mscclpp_amd/port_channel.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_PORT_CHANNEL_HPP_
