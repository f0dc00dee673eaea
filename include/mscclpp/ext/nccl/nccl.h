/* <mscclpp/ext/nccl/nccl.h> on this library: the NCCL drop-in API (ncclAllReduce, ncclCommInitRank,
 * ...) with the reference's signatures and enum values, declared in mscclpp_amd/nccl.h (C). */
#ifndef MSCCLPP_AMD_FWD_EXT_NCCL_NCCL_H_
#define MSCCLPP_AMD_FWD_EXT_NCCL_NCCL_H_

#include "mscclpp_amd/nccl.h"

#endif /* MSCCLPP_AMD_FWD_EXT_NCCL_NCCL_H_ */
