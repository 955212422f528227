// Shared by the persistent recurrences' translation units: lstm_persist.hip (the forward
// recurrences and the co-resident launch machinery) and lstm_bptt.hip (the persistent BPTT),
// which are compiled with different machine-scheduler strategies (Makefile).
// Internal: not part of the C ABI.
#pragma once
#include "kernels.h"

// Each translation unit numbers its own give-ups (a __device__ counter per code object); the tag
// keeps the BPTT's numbers apart from the forward recurrences' (persist_guard compares the pinned
// failure word for change, so two give-ups must never write the same number).
#ifndef AVC_GIVEUP_TAG
#define AVC_GIVEUP_TAG 0u
#endif

namespace avc {

typedef __attribute__((address_space(1))) unsigned gu32;
constexpr unsigned kSpinLimit = 1u << 21;
// Counter region layout: line 0 = the launch ticket (u64), line 1 = the give-up word (epoch of
// the last launch that gave up), then the counters.
constexpr int kRegionHeaderWords = 2 * 32;

// the co-resident launch machinery (lstm_persist.hip) for the other translation unit
int persist_region_t(avc_context* ctx, int kind, int T, int ngrp, int ncb, int nwg, size_t counter_words,
                     hipStream_t s, unsigned** out);
bool persist_inject_take();  // a failure injection is pending: consume it (avc_debug_persist_inject)
// the BPTT translation unit's give-up count (avc_lstm_persist_status sums both units)
unsigned bptt_giveup_count();
#ifdef AVC_STAMPS
int bptt_set_stamps(void* buf);
#endif

namespace {

__device__ unsigned g_persist_giveups = 0;  // sticky count of timed-out launches (host-read), per unit

// One wave, every lane: leave a spin?  The give-up word is read every 64 passes; past the limit
// the launch gives up (the first wave to do so reports it, as wait_ge_ctl).  spins is uniform.
__device__ bool spin_give_up_ctl(unsigned spins, unsigned* tmo, unsigned* fail_host, unsigned spin_limit, unsigned E,
                                 int lane) {
  if ((spins & 63) == 63 && __hip_atomic_load((gu32*)tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == E)
    return true;
  if (spins < spin_limit) return false;
  if (lane == 0) {
    const unsigned old = __hip_atomic_fetch_max((gu32*)tmo, E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old != E) {
      const unsigned nf = (atomicAdd(&g_persist_giveups, 1u) + 1u) | AVC_GIVEUP_TAG;
      if (fail_host) __hip_atomic_store(fail_host, nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  return true;
}
// One lane waits until *p reaches target (wrap-safe; relaxed agent-scope polls).  false = gave
// up, or another workgroup of this launch (epoch E) did: the give-up word is checked every 64
// polls.  The first workgroup to give up reports the launch to the host.
__device__ bool wait_ge_ctl(unsigned* p, unsigned target, unsigned* tmo, unsigned* fail_host, unsigned spin_limit,
                            unsigned E) {
  gu32* gp = (gu32*)(p);
  gu32* gt = (gu32*)(tmo);
  for (unsigned spins = 0;; ++spins) {
    if ((int)(__hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) >= 0) return true;
    if ((spins & 63) == 63 && __hip_atomic_load(gt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == E)
      return false;
    if (spins >= spin_limit) {
      const unsigned old = __hip_atomic_fetch_max(gt, E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old != E) {  // first to give up in this launch: a device-wide unique failure number
        const unsigned n = (atomicAdd(&g_persist_giveups, 1u) + 1u) | AVC_GIVEUP_TAG;
        if (fail_host)
          __hip_atomic_store(fail_host, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

}  // namespace
}  // namespace avc
