// <mscclpp/algorithm.hpp> on this library: Algorithm / AlgorithmBuilder / NativeAlgorithm / AlgorithmCollection.
// A caller written against the reference's include/mscclpp/algorithm.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/algorithm.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_ALGORITHM_HPP_
#define MSCCLPP_AMD_FWD_ALGORITHM_HPP_

#include "mscclpp_amd/algorithm.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_ALGORITHM_HPP_
