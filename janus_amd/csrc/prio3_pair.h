// prio3_pair.h -- lane-pair pieces shared by the two-work-items-per-report kernels:
// k_xof_pair (prio3_xof_pair.hip, long shares) and k_prep_hp (prio3_prep_pair.hip, the fused
// Histogram prepare for groups too small to fill the chip with one lane per report).
// The even lane of a pair squeezes the measurement share, the odd lane absorbs the same bytes
// into the joint-rand-part sponge, taking them from its partner by DPP.
#pragma once
#include <hip/hip_runtime.h>

#include "prio3_device.h"
#include "prio3_common.h"

// the even partner's value (lane & ~1): DPP quad_perm [0,0,2,2]
DEV uint32_t from_even(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xA0, 0xF, 0xF, false);
}
// the odd partner's value (lane | 1): DPP quad_perm [1,1,3,3]
DEV uint32_t from_odd(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xF5, 0xF, 0xF, false);
}


// Block b of the share phase after the even lane squeezed it: the odd lane XORs block b of the
// joint-rand-part message into its state.  Message word j is a 16-bit funnel shift of two
// squeezed words (the 42-byte prefix is 10.5 words): words 0..9 come from the previous block's
// tail (or the prefix, FIRST), word 10 straddles, words 11..41 come from this block -- streamed
// word by word from the even lane (DPP), so no block-sized array is live.  LAST: padding.
template <bool FIRST, bool LAST>
DEV void absorb_share_block(KState& st, uint32_t h, bool hasW, uint32_t (&tail)[11],
                            const uint32_t (&pre)[11], uint32_t rem) {
  auto pad = [&](int j, uint32_t x) {
    if (LAST) {
      const uint32_t lo = 4 * j;
      const uint32_t mask = (lo + 4 <= rem) ? 0xffffffffu
                                            : (lo >= rem ? 0u : ((1u << (8 * (rem - lo))) - 1u));
      x &= mask;
      if ((uint32_t)j == (rem >> 2)) x ^= 1u << (8 * (rem & 3));
      if (j == 41) x ^= 0x80000000u;
    }
    return x;
  };
#pragma unroll
  for (int j = 0; j < 10; j++) {
    const uint32_t x = FIRST ? pre[j] : __builtin_amdgcn_alignbit(tail[j + 1], tail[j], 16);
    kxor_word(st, j, h ? pad(j, x) : 0u);
  }
  uint32_t prev = hasW ? from_even(kword(st, 0)) : 0u;
  {
    const uint32_t x = FIRST ? ((pre[10] & 0xffffu) | (prev << 16))
                             : __builtin_amdgcn_alignbit(prev, tail[10], 16);
    kxor_word(st, 10, h ? pad(10, x) : 0u);
  }
#pragma unroll
  for (int j = 11; j < 42; j++) {
    // lane 0's word j - 10 is read before lane 0's own XOR of word j (a no-op on the even lane)
    const uint32_t cur = hasW ? from_even(kword(st, j - 10)) : 0u;
    kxor_word(st, j, h ? pad(j, __builtin_amdgcn_alignbit(cur, prev, 16)) : 0u);
    prev = cur;
  }
  // the next block's words 0..10 need this block's words 31..41 (uniform branch: DPP converged)
  if (hasW) {
    tail[0] = prev;
#pragma unroll
    for (int t = 1; t < 11; t++) tail[t] = from_even(kword(st, 31 + t));
  }
}
