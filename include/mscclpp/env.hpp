// <mscclpp/env.hpp> on this library (include/mscclpp_amd/env.hpp).
// A caller written against the reference's include/mscclpp/env.hpp compiles unchanged with
// `-I include`; namespace mscclpp names the declarations through a using-directive
// (include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_ENV_HPP_
#define MSCCLPP_AMD_FWD_ENV_HPP_

#include "mscclpp_amd/env.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_ENV_HPP_
