// <mscclpp/ext/collectives/algorithm_collection_builder.hpp> on this library: collective::AlgorithmCollectionBuilder.
// A caller written against the reference's include/mscclpp/ext/collectives/algorithm_collection_builder.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/algorithm.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_EXT_COLLECTIVES_ALGORITHM_COLLECTION_BUILDER_HPP_
#define MSCCLPP_AMD_FWD_EXT_COLLECTIVES_ALGORITHM_COLLECTION_BUILDER_HPP_

#include "mscclpp_amd/algorithm.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_EXT_COLLECTIVES_ALGORITHM_COLLECTION_BUILDER_HPP_
