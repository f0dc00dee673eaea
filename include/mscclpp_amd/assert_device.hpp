// MSCCLPP_ASSERT_DEVICE with the reference's spelling (include/mscclpp/assert_device.hpp:13-38): a
// no-op unless DEBUG_BUILD is defined, as in the reference.  With DEBUG_BUILD a failed condition is
// printed (thread, block, message) and execution continues: a device trap would take the whole
// GPU's queue down, so this build never traps.
#pragma once

#include <hip/hip_runtime.h>

#if !defined(DEBUG_BUILD)
#define MSCCLPP_ASSERT_DEVICE(__cond, __msg)
#else
#define MSCCLPP_ASSERT_DEVICE(__cond, __msg)                                                       \
  do {                                                                                             \
    if (!(__cond))                                                                                 \
      printf("MSCCLPP_ASSERT_DEVICE failed (block %d thread %d): %s\n", (int)blockIdx.x,          \
             (int)threadIdx.x, __msg);                                                             \
  } while (0)
#endif
