// POLL_MAYBE_JAILBREAK / OR_POLL_MAYBE_JAILBREAK with the reference's spelling
// (include/mscclpp/poll_device.hpp:12-33): spin while the condition holds.  The reference bounds the
// spin only in debug builds, by a spin count and a device assert; in release builds it spins
// forever.  Here every build bounds it by wall clock (kDefaultSpinTicks, 20 s, device.hpp) and then
// stops waiting -- the caller's next step sees the state it polled for missing, and no wave is left
// spinning on the GPU.  The spin-count argument is accepted and, as in a release build, unused.
#pragma once

#include "mscclpp_amd/device.hpp"

#define POLL_MAYBE_JAILBREAK(__cond, __max_spin_cnt)                     \
  do {                                                                   \
    (void)(__max_spin_cnt);                                              \
    ::mscclpp_amd::SpinGuard __poll_guard(::mscclpp_amd::kDefaultSpinTicks); \
    while (__cond) {                                                     \
      if (__poll_guard.expired()) break;                                 \
    }                                                                    \
  } while (0)

// as above; __cond1 is checked first (cheaper), and the spin ends when either is false
#define OR_POLL_MAYBE_JAILBREAK(__cond1, __cond2, __max_spin_cnt)        \
  do {                                                                   \
    (void)(__max_spin_cnt);                                              \
    ::mscclpp_amd::SpinGuard __poll_guard(::mscclpp_amd::kDefaultSpinTicks); \
    while ((__cond1) && (__cond2)) {                                     \
      if (__poll_guard.expired()) break;                                 \
    }                                                                    \
  } while (0)
