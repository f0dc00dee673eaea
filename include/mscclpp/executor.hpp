// <mscclpp/executor.hpp> on this library: Executor / ExecutionPlan / PacketType.
// A caller written against the reference's include/mscclpp/executor.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/algorithm.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_EXECUTOR_HPP_
#define MSCCLPP_AMD_FWD_EXECUTOR_HPP_

#include "mscclpp_amd/algorithm.hpp"  // the C++ ExecutionPlan / Executor (the C ABI is executor.h)
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_EXECUTOR_HPP_
