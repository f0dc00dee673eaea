// <mscclpp/fifo.hpp> on this library: Fifo (host side).
// A caller written against the reference's include/mscclpp/fifo.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/fifo.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_FIFO_HPP_
#define MSCCLPP_AMD_FWD_FIFO_HPP_

#include "mscclpp_amd/fifo.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_FIFO_HPP_
