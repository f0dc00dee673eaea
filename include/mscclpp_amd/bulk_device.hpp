// Hopper bulk-copy (TMA) helpers of the reference (include/mscclpp/bulk_device.hpp): available there
// only for CUDA on sm_90 and later (:16-20), so on gfx950 -- as in the reference's own HIP build --
// MSCCLPP_BULK_AVAILABLE is 0 and BulkBarrier keeps only its 8-byte storage (so host code sizing
// shared memory with it gets the reference's size, :137-141); code guarded by the macro compiles
// and takes its other branch.  (Bulk moves here are the buffer-descriptor dwordx4 kernels.)
#pragma once

#include <cstdint>

#define MSCCLPP_BULK_AVAILABLE 0

namespace mscclpp_amd {

struct BulkBarrier {
 private:
  [[maybe_unused]] alignas(8) uint64_t mbar_;
};
static_assert(sizeof(BulkBarrier) == 8, "the reference's BulkBarrier is one 8-byte mbarrier word");

}  // namespace mscclpp_amd
