// prio3_engine.hip -- MI355X (gfx950) batched Prio3 helper prepare+aggregate engine and its
// C ABI (include/janus_prio3.h).
//
// Pipeline for one device call over n reports (one work-item = one report; SoA scratch
// [element][report] so that every wave-wide load/store is 64 x 16 B contiguous):
//   k_xof      helper XOF work: query randomness, measurement-share expansion fused with
//              the joint-randomness-part absorb (one Keccak state squeezes while a second
//              absorbs the same bytes, 16-bit funnel shifted), proofs-share expansion,
//              corrected joint-rand seed and joint randomness.  Any rejection-sampling hit
//              flags the report.                 [prio Prio3::prepare_init, VDAF-08 7.2.2]
//   k_xof_slow general byte-level sponge with rejection sampling, run only for flagged
//              reports (probability ~2^-59 per Field128 element, ~2^-32 per Field64 one).
//   k_query    FLP query (wire polynomials evaluated at t with the Lagrange basis obtained
//              from one size-P DFT of t-powers, gadget polynomial at the P-th roots from one
//              folded size-P DFT), decode+add the leader verifier share, decide, prepare
//              message, joint-rand check, truncate.  [prio FlpGeneric::query/decide,
//              Prio3::prepare_shares_to_prepare_message, prepare_next]
//   k_mask/k_acc_partial/k_acc_final  masked, segmented mod-p reduction of the output
//              shares into per-batch aggregate shares [aggregation_job_writer.rs:591-695].
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/janus_hpke.h"
#include "../../include/janus_prio3.h"
#include "prio3_device.h"

#include "prio3_common.h"
#include "prio3_query_sum.h"
#include "prio3_runtime.h"
#include "sha256_device.h"
#include "sha256_host.h"

#ifndef XOFD_OCC
#define XOFD_OCC 3
#endif
template <class F>
__device__ __forceinline__ void xof_body(const DevParams& p, const InPtrs& in, const Scratch& sc,
                                         const uint32_t r) {
  // r: this lane's report
  if (r >= p.n) return;
  constexpr uint32_t ES = F::ES;
  uint32_t flag = p.force_slow;
  uint32_t nonce[4], km[4], kp[4], kb[4] = {0, 0, 0, 0};
  load16(in.nonces + 16 * (size_t)r, nonce);
  const uint8_t* hs = in.helper + (size_t)r * p.helper_share_len;
  load16(hs, km);
  load16(hs + 16, kp);
  const bool JR = p.jr_len > 0;
  if (JR) load16(hs + 32, kb);

  // 1. query randomness: XOF(vk, dst(5), [PROOFS] || nonce), qr_len elements (<= 10)
  {
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[5]);
    {
      uint32_t vk[4];
      load_vk(p, in, r, vk);
      msg_bytes16(m, 9, vk);
    }
    msg_byte(m, 25, 1);
    msg_bytes16(m, 26, nonce);
    msg_absorb_final(s, m, 42);
    uint32_t q0 = 0, q1 = 0;
    squeeze_block<F>(p, s, 0, p.qr_len, q0, q1, sc.qr, r, flag);
  }

  // 2. measurement share XOF(k_meas, dst(1), [1]) fused with the joint-rand part
  //    XOF(k_blind, dst(7), [1] || nonce || enc(meas)).
  KState ms;
  kzero(ms);
  {
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[1]);
    msg_bytes16(m, 9, km);
    msg_byte(m, 25, 1);
    msg_absorb_final(ms, m, 26);
  }
  const uint32_t M = p.meas_len;
  const uint32_t mbytes = M * ES;
  const uint32_t K = (mbytes + 167) / 168;
  const uint32_t L = 42 + mbytes;
  const uint32_t B = L / 168, rem = L % 168;
  KState js;
  uint32_t pre[11], tail[11];
  uint32_t part[4] = {0, 0, 0, 0};
  if (JR) {
    kzero(js);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[7]);
    msg_bytes16(m, 9, kb);
    msg_byte(m, 25, 1);
    msg_bytes16(m, 26, nonce);
#pragma unroll
    for (int j = 0; j < 11; j++) pre[j] = m.w[j];
  }
#pragma unroll
  for (int j = 0; j < 11; j++) tail[j] = 0;
  uint32_t pend0 = 0, pend1 = 0;
  const uint32_t nb = JR ? B + 1 : K;
  for (uint32_t b = 0; b < nb; b++) {
    const bool hasW = b < K;
    if (hasW) squeeze_block<F>(p, ms, b, M, pend0, pend1, sc.meas, r, flag);
    if (JR && b < B) {  // full block: each message word goes straight into the state
      const uint32_t w0 = hasW ? kword(ms, 0) : 0u;
#pragma unroll
      for (int j = 0; j < 10; j++)
        kxor_word(js, j, b == 0 ? pre[j] : __builtin_amdgcn_alignbit(tail[j + 1], tail[j], 16));
      kxor_word(js, 10, b == 0 ? ((pre[10] & 0xffffu) | (w0 << 16))
                               : __builtin_amdgcn_alignbit(w0, tail[10], 16));
#pragma unroll
      for (int j = 11; j < 42; j++)
        kxor_word(js, j, hasW ? __builtin_amdgcn_alignbit(kword(ms, j - 10), kword(ms, j - 11), 16)
                              : 0u);
      keccak_p12(js);
    } else if (JR) {
      uint32_t x[42];
#pragma unroll
      for (int j = 0; j < 10; j++)
        x[j] = b == 0 ? pre[j] : __builtin_amdgcn_alignbit(tail[j + 1], tail[j], 16);
      uint32_t w0 = hasW ? kword(ms, 0) : 0u;
      x[10] = b == 0 ? ((pre[10] & 0xffffu) | (w0 << 16))
                     : __builtin_amdgcn_alignbit(w0, tail[10], 16);
#pragma unroll
      for (int j = 11; j < 42; j++)
        x[j] = hasW ? __builtin_amdgcn_alignbit(kword(ms, j - 10), kword(ms, j - 11), 16) : 0u;
      {
#pragma unroll
        for (int j = 0; j < 42; j++) {
          const uint32_t lo = 4 * j;
          uint32_t mask = (lo + 4 <= rem) ? 0xffffffffu
                                          : (lo >= rem ? 0u : ((1u << (8 * (rem - lo))) - 1u));
          x[j] &= mask;
          if ((uint32_t)j == (rem >> 2)) x[j] ^= 1u << (8 * (rem & 3));
        }
        x[41] ^= 0x80000000u;
#pragma unroll
        for (int j = 0; j < 42; j++) kxor_word(js, j, x[j]);
        keccak_p12(js);
        part[0] = kword(js, 0);
        part[1] = kword(js, 1);
        part[2] = kword(js, 2);
        part[3] = kword(js, 3);
      }
    }
    if (hasW) {
#pragma unroll
      for (int t = 0; t < 11; t++) tail[t] = kword(ms, 31 + t);
    }
    if (b + 1 < K) keccak_p12(ms);
  }

  // 3. proofs share XOF(k_proofs, dst(2), [PROOFS, 1])
  {
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[2]);
    msg_bytes16(m, 9, kp);
    msg_byte(m, 25, 1);
    msg_byte(m, 26, 1);
    msg_absorb_final(s, m, 27);
    const uint32_t PL = p.proof_len;
    const uint32_t Kp = (PL * ES + 167) / 168;
    uint32_t q0 = 0, q1 = 0;
    for (uint32_t b = 0; b < Kp; b++) {
      squeeze_block<F>(p, s, b, PL, q0, q1, sc.proofs, r, flag);
      if (b + 1 < Kp) keccak_p12(s);
    }
  }

  // 4. corrected joint-rand seed and joint randomness
  if (JR) {
    uint32_t pub0[4];
    load16(in.pub + (size_t)r * p.public_share_len, pub0);
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[6]);
    msg_bytes16(m, 25, pub0);
    msg_bytes16(m, 41, part);
    msg_absorb_final(s, m, 57);
    uint32_t cor[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
    KState t;
    kzero(t);
    Msg m2;
    msg_zero(m2);
    msg_dst(m2, p.dst[3]);
    msg_bytes16(m2, 9, cor);
    msg_byte(m2, 25, 1);
    msg_absorb_final(t, m2, 26);
    uint32_t q0 = 0, q1 = 0;
    squeeze_block<F>(p, t, 0, p.jr_len, q0, q1, sc.jr, r, flag);
    sc.part[r] = make_uint4(part[0], part[1], part[2], part[3]);
    sc.corrected[r] = make_uint4(cor[0], cor[1], cor[2], cor[3]);
  }
  sc.flag[r] = (uint8_t)flag;
}
template <class F>
__global__ __launch_bounds__(256, XOFD_OCC) void k_xof(DevParams p, InPtrs in, Scratch sc) {
  xof_body<F>(p, in, sc, blockIdx.x * blockDim.x + threadIdx.x);
}


// ------------------------------------------------------------------------------------
// k_xofd: k_xof_a + k_jrpart in one pass with two live Keccak states -- each squeezed
// measurement-share block is absorbed into the joint-rand-part sponge while still in
// registers (no 4 KiB re-read), the two permutation streams give each wave 2x the ILP.
// Field128 joint-randomness instances with at least three joint-rand blocks; peeled first and
// last blocks keep the steady-state loop free of the prefix / padding code.
// ------------------------------------------------------------------------------------
// FUSE: the optimistic per-segment aggregate of the fused path (see k_jrpart<true>) is taken
// here, from the squeezed elements while they are in registers; a wave in which any report got
// flagged for the slow path is un-fused at the end (its partials are ignored, its reports go
// through the fix-up list with their corrected shares).
// TR: the measurement share is also truncated into sc.out on the fly (DevParams::trunc_xof).
// PULL (executor groups): the lane's leader prep share is copied from the mapped host staging
// (in.leader_src) into in.leader in 16-byte pieces spread over the share loop -- each load issued
// before the iteration's two permutations and stored after them, so the PCIe latency hides under
// the Keccak work and the transfer runs at the XOF's pace -- plus its segment id and accept byte.
template <bool FUSE, bool TR = false, bool PULL = false>
__device__ __forceinline__ void xofd_body(const DevParams& p, const InPtrs& in, const Scratch& sc,
                                          const uint32_t r) {  // r & 63 == this lane
  typedef Fp128 F;
  const uint32_t lane = threadIdx.x & 63u;
  bool fuse = false, oor = false, haspad = false;
  uint32_t s0 = 0;
  if constexpr (FUSE) {
    const bool valid = r < p.n;
    const uint32_t sg = valid ? (sc.seg ? sc.seg[r] : 0u) : 0xffffffffu;
    // A segment id >= n_segments puts the report in no aggregate.  Such lanes (the executor's
    // pad columns between jobs, excluded reports) are masked out of the wave partials, so they
    // do not keep the wave's other 63 reports from fusing; k_agg_fix knows them (oor_masked).
    const uint64_t inr = __ballot(valid && sg < p.nseg);
    s0 = inr ? (uint32_t)__shfl((int)sg, __ffsll((long long)inr) - 1) : 0xffffffffu;
    oor = valid && sg >= p.nseg;
    fuse = inr != 0 && __all(valid && (sg == s0 || sg >= p.nseg));
    haspad = __any(oor);
    if (lane == 0 && (r - lane) < p.n && !fuse) sc.wseg[r >> 6] = 0xffffffffu;
  }
  if (r >= p.n) return;
  uint32_t flag = p.force_slow;
  uint32_t nonce[4], km[4], kb[4];
  load16(in.nonces + 16 * (size_t)r, nonce);
  const uint8_t* hs = in.helper + (size_t)r * p.helper_share_len;
  load16(hs, km);
  load16(hs + 32, kb);
  {  // query randomness
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[5]);
    {
      uint32_t vk[4];
      load_vk(p, in, r, vk);
      msg_bytes16(m, 9, vk);
    }
    msg_byte(m, 25, 1);
    msg_bytes16(m, 26, nonce);
    msg_absorb_final(s, m, 42);
    if (p.qr_len == 1) {  // wave-uniform
      uint32_t w[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
      put_elem<F>(p, sc.qr, 0, r, w, flag);
    } else {  // FPVec: one query point per gadget
      uint32_t q0 = 0, q1 = 0;
      squeeze_block<F>(p, s, 0, p.qr_len, q0, q1, sc.qr, r, flag);
    }
  }
  const uint32_t M = p.meas_len, K = (M * 16 + 167) / 168;
  const uint32_t L = 42 + M * 16, B = L / 168, rem = L % 168;  // B >= 2 (checked on the host)
  KState ms, js;
  kzero(ms);
  kzero(js);
  {
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[1]);
    msg_bytes16(m, 9, km);
    msg_byte(m, 25, 1);
    msg_absorb_final(ms, m, 26);
  }
  uint32_t pend0 = 0, pend1 = 0;
  TruncSink ts(p, sc.out, r);
  const int Mi = (int)M;
  // wave totals of share elements e0, e0+1 (zero outside [0, M)), slot lane of lanes 0..15
  auto fused_pair = [&](int e0, f128 a, f128 b2) __attribute__((always_inline)) {
    if (e0 >= Mi) return;  // wave-uniform
    if (haspad && oor) {   // wave-uniform test; the masked lanes add nothing
      a = zero128();
      b2 = zero128();
    }
    const uint32_t tot = wave_halfsum2(a, b2, lane);  // slot lane >> 2 on each lane of a quad
    const int e = e0 + (int)(lane >> 5);
    if ((lane & 3u) == 0 && e < Mi)
      sc.wpart[((size_t)(r >> 6) * M + (uint32_t)e) * 8u + ((lane >> 2) & 7u)] = tot;
  };
  // the elements squeezed from share block b (state ms, pend = carried half element)
  auto fuse_block = [&](uint32_t b, uint32_t q0, uint32_t q1) __attribute__((always_inline)) {
    const int e0 = 21 * (int)(b >> 1);
    const f128 z = zero128();
    if ((b & 1) == 0) {
#pragma unroll
      for (int t = 0; t < 10; t += 2)
        fused_pair(e0 + t, mk128(kword(ms, 4 * t), kword(ms, 4 * t + 1), kword(ms, 4 * t + 2),
                                 kword(ms, 4 * t + 3)),
                   mk128(kword(ms, 4 * t + 4), kword(ms, 4 * t + 5), kword(ms, 4 * t + 6),
                         kword(ms, 4 * t + 7)));
    } else {
      fused_pair(e0 + 10, mk128(q0, q1, kword(ms, 0), kword(ms, 1)),
                 mk128(kword(ms, 2), kword(ms, 3), kword(ms, 4), kword(ms, 5)));
#pragma unroll
      for (int t = 1; t < 10; t += 2)
        fused_pair(e0 + 11 + t,
                   mk128(kword(ms, 2 + 4 * t), kword(ms, 3 + 4 * t), kword(ms, 4 + 4 * t),
                         kword(ms, 5 + 4 * t)),
                   t + 1 < 10 ? mk128(kword(ms, 6 + 4 * t), kword(ms, 7 + 4 * t),
                                      kword(ms, 8 + 4 * t), kword(ms, 9 + 4 * t))
                              : z);
    }
  };
  // Joint-rand block b holds the last 42 bytes of share block b-1 (words 0..10, a 16-bit funnel
  // shift) and the first 126 bytes of share block b (words 10..41).  The first part is XORed into
  // js as soon as js has been permuted for block b-1 and before ms moves on, so no share words
  // are carried across a permutation (the 11-word tail buffer spilled at 168 VGPRs).
  auto wmask = [&](int j) __attribute__((always_inline)) {  // bytes of word j below rem
    const uint32_t lo = 4u * (uint32_t)j;
    return (lo + 4 <= rem) ? 0xffffffffu : (lo >= rem ? 0u : ((1u << (8 * (rem - lo))) - 1u));
  };
  auto carry_tail = [&](bool last) __attribute__((always_inline)) {  // last: block B is next
#pragma unroll
    for (int j = 0; j < 10; j++) {
      uint32_t x = __builtin_amdgcn_alignbit(kword(ms, 32 + j), kword(ms, 31 + j), 16);
      if (last) x &= wmask(j);
      kxor_word(js, j, x);
    }
    uint32_t x = kword(ms, 41) >> 16;
    if (last) x &= wmask(10);
    kxor_word(js, 10, x);
  };
  // block 0: prefix (42 bytes) + the first 126 bytes of the share
  {
    if (FUSE && fuse) fuse_block(0, 0, 0);
    squeeze_meas<TR>(p, ms, 0, M, pend0, pend1, sc.meas, r, flag, ts);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[7]);
    msg_bytes16(m, 9, kb);
    msg_byte(m, 25, 1);
    msg_bytes16(m, 26, nonce);
#pragma unroll
    for (int j = 0; j < 10; j++) kxor_word(js, j, m.w[j]);
    kxor_word(js, 10, (m.w[10] & 0xffffu) | (kword(ms, 0) << 16));
#pragma unroll
    for (int j = 11; j < 42; j++)
      kxor_word(js, j, __builtin_amdgcn_alignbit(kword(ms, j - 10), kword(ms, j - 11), 16));
    keccak_p12(js);
    carry_tail(B == 1);
    keccak_p12(ms);
  }
  if constexpr (PULL) {
    if (in.seg_dst) in.seg_dst[r] = in.seg_src[r];
    if (in.accept_dst) in.accept_dst[r] = in.accept_src[r];
  }
  // PULL: the wave's 64 leader shares are one contiguous run of 64 Q 16-byte pieces; iteration b
  // copies rows [Q (b-1) / (B-1), Q b / (B-1)) (1 or 2) of 64 pieces, lane l taking piece
  // 64 row + l, so every load instruction reads 1 KiB of consecutive host bytes (one 16-byte
  // piece per report per lane made the PCIe reads scattered: 18.5 GB/s, profiles/r03/r03o)
  const uint32_t Q = PULL ? p.prep_share_len / 16 : 0u;
  const size_t wbase = PULL ? (size_t)(r - lane) * (p.prep_share_len / 16) + lane : 0;
  const uint4* lsrc = PULL ? (const uint4*)in.leader_src + wbase : nullptr;
  uint4* ldst = PULL ? (uint4*)in.leader + wbase : nullptr;
  // full joint-rand blocks 1 .. B-1 (B <= K, so share block b exists for every b < B)
#pragma unroll 1
  for (uint32_t b = 1; b < B; b++) {
    uint4 pc0, pc1;
    uint32_t q0 = 0, q1 = 0;
    if constexpr (PULL) {
      q0 = Q * (b - 1) / (B - 1);
      q1 = Q * b / (B - 1);
      if (q0 < q1) pc0 = lsrc[64 * (size_t)q0];
      if (q0 + 1 < q1) pc1 = lsrc[64 * (size_t)(q0 + 1)];
    }
    if (FUSE && fuse) fuse_block(b, pend0, pend1);
    squeeze_meas<TR>(p, ms, b, M, pend0, pend1, sc.meas, r, flag, ts);
    kxor_word(js, 10, kword(ms, 0) << 16);
#pragma unroll
    for (int j = 11; j < 42; j++)
      kxor_word(js, j, __builtin_amdgcn_alignbit(kword(ms, j - 10), kword(ms, j - 11), 16));
    keccak_p12(js);
    carry_tail(b + 1 == B);
    if (b + 1 < K) keccak_p12(ms);
    if constexpr (PULL) {
      if (q0 < q1) ldst[64 * (size_t)q0] = pc0;
      if (q0 + 1 < q1) ldst[64 * (size_t)(q0 + 1)] = pc1;
    }
  }
  // final joint-rand block B: remaining share bytes, padding
  uint32_t part[4];
  {
    const bool hasW = B < K;
    if (FUSE && fuse && hasW) fuse_block(B, pend0, pend1);
    if (hasW) squeeze_meas<TR>(p, ms, B, M, pend0, pend1, sc.meas, r, flag, ts);
#pragma unroll
    for (int j = 0; j < 42; j++) {
      uint32_t x = 0;
      if (j == 10) x = hasW ? kword(ms, 0) << 16 : 0u;
      else if (j > 10)
        x = hasW ? __builtin_amdgcn_alignbit(kword(ms, j - 10), kword(ms, j - 11), 16) : 0u;
      x &= wmask(j);
      if ((uint32_t)j == (rem >> 2)) x ^= 1u << (8 * (rem & 3));
      if (j == 41) x ^= 0x80000000u;
      kxor_word(js, j, x);
    }
    keccak_p12(js);
    part[0] = kword(js, 0);
    part[1] = kword(js, 1);
    part[2] = kword(js, 2);
    part[3] = kword(js, 3);
  }
  {  // proofs share
    uint32_t kp[4];  // loaded here: it was live across the share loop
    load16(hs + 16, kp);
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[2]);
    msg_bytes16(m, 9, kp);
    msg_byte(m, 25, 1);
    msg_byte(m, 26, 1);
    msg_absorb_final(s, m, 27);
    const uint32_t PL = p.proof_len, Kp = (PL * 16 + 167) / 168;
    uint32_t q0 = 0, q1 = 0;
    for (uint32_t b = 0; b < Kp; b++) {
      squeeze_block<F>(p, s, b, PL, q0, q1, sc.proofs, r, flag);
      if (b + 1 < Kp) keccak_p12(s);
    }
  }
  {  // corrected seed, joint randomness
    uint32_t pub0[4];
    load16(in.pub + (size_t)r * p.public_share_len, pub0);
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[6]);
    msg_bytes16(m, 25, pub0);
    msg_bytes16(m, 41, part);
    msg_absorb_final(s, m, 57);
    uint32_t cor[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
    KState t;
    kzero(t);
    Msg m2;
    msg_zero(m2);
    msg_dst(m2, p.dst[3]);
    msg_bytes16(m2, 9, cor);
    msg_byte(m2, 25, 1);
    msg_absorb_final(t, m2, 26);
    uint32_t q0 = 0, q1 = 0;
    squeeze_block<F>(p, t, 0, p.jr_len, q0, q1, sc.jr, r, flag);
    sc.part[r] = make_uint4(part[0], part[1], part[2], part[3]);
    sc.corrected[r] = make_uint4(cor[0], cor[1], cor[2], cor[3]);
  }
  sc.flag[r] = (uint8_t)flag;
  if constexpr (FUSE) {
    if (fuse) {  // all 64 lanes are live here
      const bool anyflag = __any(flag != 0);
      if (lane == 0) sc.wseg[r >> 6] = anyflag ? 0xffffffffu : s0;
    }
  }
}
template <bool FUSE, bool TR = false>
__global__ __launch_bounds__(256, XOFD_OCC) void k_xofd(DevParams p, InPtrs in, Scratch sc) {
  xofd_body<FUSE, TR>(p, in, sc, blockIdx.x * blockDim.x + threadIdx.x);
}

// Zero-fills up to 4 ranges in one launch (4-byte aligned lengths and pointers: 16-byte stores
// for the aligned body, 4-byte stores at the ends)
struct ZeroRanges {
  uint8_t* dst[4];
  size_t bytes[4];
};
__global__ __launch_bounds__(256) void k_zero(ZeroRanges z) {
  const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint8_t* d = z.dst[k];
    const size_t n = z.bytes[k];
    if (!d || !n) continue;
    const size_t head = std::min(n, (size_t)((16 - ((uintptr_t)d & 15)) & 15));
    const size_t n16 = (n - head) / 16;
    for (size_t i = tid; i < n16; i += nth) ((uint4*)(d + head))[i] = make_uint4(0, 0, 0, 0);
    for (size_t i = tid * 4; i < head; i += nth * 4) *(uint32_t*)(d + i) = 0u;
    for (size_t i = head + 16 * n16 + tid * 4; i < n; i += nth * 4) *(uint32_t*)(d + i) = 0u;
  }
}

// Copies by the shader cores between device memory and mapped pinned memory (up to 4 ranges,
// 16-byte aligned; 16-byte accesses, the byte tails by lane).  Host -> device, this reads PCIe at
// ~55 GB/s where the SDMA copy of the same staging ran at ~32 GB/s beside the XOF's own host
// reads (profiles/r03/r03l trace); device -> host, one launch returns a group's four outputs
// where four SDMA copies each paid their own setup.
struct PullRanges {
  const uint8_t* src[4];
  uint8_t* dst[4];
  size_t bytes[4];
};
DEV void pull_body(const PullRanges& pr, size_t tid, size_t nth) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const size_t n16 = pr.bytes[k] / 16;
    const uint4* s16 = (const uint4*)pr.src[k];
    uint4* d16 = (uint4*)pr.dst[k];
    for (size_t i = tid; i < n16; i += nth) d16[i] = s16[i];
    const size_t t = 16 * n16 + tid;
    if (t < pr.bytes[k] && tid < 16) pr.dst[k][t] = pr.src[k][t];
  }
}
__global__ __launch_bounds__(256) void k_pull(PullRanges pr) {
  pull_body(pr, (size_t)blockIdx.x * blockDim.x + threadIdx.x, (size_t)gridDim.x * blockDim.x);
}


// ------------------------------------------------------------------------------------
// Split XOF path (one Keccak state live per kernel, for occupancy):
//   k_xof_a   query randomness, measurement share and proofs share squeezed to scratch
//   k_jrpart  joint-rand part absorbed from the measurement share in scratch, corrected
//             seed, joint randomness.  The 42-byte prefix leaves every message word a 16-bit
//             funnel shift of two share words whose element/word offsets are compile-time
//             constants relative to 21*(b/2) (b = block index), so each 168-byte block is 11-12
//             coalesced 16-byte loads + 42 v_alignbit.
// ------------------------------------------------------------------------------------
template <class F>
#ifndef XOF_OCC
#define XOF_OCC 4
#endif
#ifndef JR_OCC
#define JR_OCC 4
#endif
__global__ __launch_bounds__(256, XOF_OCC) void k_xof_a(DevParams p, InPtrs in, Scratch sc) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  constexpr uint32_t ES = F::ES;
  uint32_t flag = p.force_slow;
  uint32_t nonce[4], km[4], kp[4];
  load16(in.nonces + 16 * (size_t)r, nonce);
  const uint8_t* hs = in.helper + (size_t)r * p.helper_share_len;
  load16(hs, km);
  load16(hs + 16, kp);
  {
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[5]);
    {
      uint32_t vk[4];
      load_vk(p, in, r, vk);
      msg_bytes16(m, 9, vk);
    }
    msg_byte(m, 25, 1);
    msg_bytes16(m, 26, nonce);
    msg_absorb_final(s, m, 42);
    uint32_t w[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
    put_elem<F>(p, sc.qr, 0, r, w, flag);
  }
  {
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[1]);
    msg_bytes16(m, 9, km);
    msg_byte(m, 25, 1);
    msg_absorb_final(s, m, 26);
    const uint32_t M = p.meas_len, K = (M * ES + 167) / 168;
    uint32_t q0 = 0, q1 = 0;
    for (uint32_t b = 0; b < K; b++) {
      squeeze_block<F>(p, s, b, M, q0, q1, sc.meas, r, flag);
      if (b + 1 < K) keccak_p12(s);
    }
  }
  {
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[2]);
    msg_bytes16(m, 9, kp);
    msg_byte(m, 25, 1);
    msg_byte(m, 26, 1);
    msg_absorb_final(s, m, 27);
    const uint32_t PL = p.proof_len, Kp = (PL * ES + 167) / 168;
    uint32_t q0 = 0, q1 = 0;
    for (uint32_t b = 0; b < Kp; b++) {
      squeeze_block<F>(p, s, b, PL, q0, q1, sc.proofs, r, flag);
      if (b + 1 < Kp) keccak_p12(s);
    }
  }
  sc.flag[r] = (uint8_t)flag;
}

// Field128 only (every joint-randomness Prio3 instance uses Field128).
// FUSE: the measurement share streams through here anyway, so the (optimistic) per-segment
// aggregate is accumulated on the way: every element of the share is summed over the wave's 64
// reports by wave_halfsum2 and the wave's half-limb partials go to sc.wpart.  Only waves whose
// 64 reports are all present and in one segment are fused (sc.wseg records which); the rest,
// and every report the verdict or the host mask excludes, are fixed up in aggregate_finish.
// LEADER: agg_id 0 -- the blind is the last 16 bytes of the explicit leader input share
// (in.helper then points at the leader input shares), the binder byte is 0, and the corrected
// seed is derive_seed(own part || public part 1) (leader part first).
template <bool FUSE, bool LEADER = false>
__global__ __launch_bounds__(256, JR_OCC) void k_jrpart(DevParams p, InPtrs in, Scratch sc) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  bool fuse = false;
  if constexpr (FUSE) {
    const bool valid = r < p.n;
    const uint32_t sg = valid ? (sc.seg ? sc.seg[r] : 0u) : 0xffffffffu;
    const uint32_t s0 = (uint32_t)__shfl((int)sg, 0);
    // a report flagged for the rejection-sampling slow path gets its share rewritten later:
    // its wave is left to the fix-up pass
    const bool flagged = valid && sc.flag[r];
    fuse = __all(valid && sg == s0 && sg < p.nseg && !flagged);
    if (lane == 0 && (r - lane) < p.n) sc.wseg[r >> 6] = fuse ? s0 : 0xffffffffu;
  }
  if (r >= p.n) return;
  const size_t ld = p.ld;
  const int M = (int)p.meas_len;
  uint32_t nonce[4], kb[4];
  load16(in.nonces + 16 * (size_t)r, nonce);
  if constexpr (LEADER)
    load16(in.helper + (size_t)r * p.leader_share_len + (size_t)(p.meas_len + p.proof_len) * 16, kb);
  else
    load16(in.helper + (size_t)r * p.helper_share_len + 32, kb);
  uint32_t pre[11];
  {
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[7]);
    msg_bytes16(m, 9, kb);
    msg_byte(m, 25, LEADER ? 0 : 1);
    msg_bytes16(m, 26, nonce);
#pragma unroll
    for (int j = 0; j < 11; j++) pre[j] = m.w[j];
  }
  const uint4* meas = (const uint4*)sc.meas;
  auto ldel = [&](int e) -> uint4 {
    const bool ok = e >= 0 && e < M;
    uint4 v = meas[(size_t)(ok ? e : 0) * ld + r];
    return ok ? v : make_uint4(0, 0, 0, 0);
  };
  auto wsel = [](const uint4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; };
  // wave totals of elements e0, e0+1 (zero outside [0, M)); lanes 0..15 store slot lane
  auto fused_pair = [&](int e0, const uint4& a, const uint4& b) {
    if (e0 + 1 < 0 || e0 >= M) return;  // wave-uniform
    const uint32_t tot = wave_halfsum2(mk128(a.x, a.y, a.z, a.w), mk128(b.x, b.y, b.z, b.w), lane);
    const int e = e0 + (int)(lane >> 5);  // slot lane >> 2 on each lane of a quad
    if ((lane & 3u) == 0 && e >= 0 && e < M)
      sc.wpart[((size_t)(r >> 6) * (uint32_t)M + (uint32_t)e) * 8u + ((lane >> 2) & 7u)] = tot;
  };
  const uint32_t L = 42 + (uint32_t)M * 16;
  const uint32_t B = L / 168, rem = L % 168;
  KState s;
  kzero(s);
  for (uint32_t b = 0; b <= B; b++) {
    uint32_t x[42];
    const int q21 = 21 * (int)(b >> 1);
    if ((b & 1) == 0) {
      // u = 84q + j - 11: element 21q + floor((j-11)/4), word (j-11) mod 4; window 21q-3..21q+7
      uint4 E[11];
#pragma unroll
      for (int t = 0; t < 11; t++) E[t] = ldel(q21 - 3 + t);
      if (FUSE && fuse) {  // this window accounts for elements q21-2 .. q21+7 (E[1..10])
#pragma unroll
        for (int t = 1; t < 11; t += 2) fused_pair(q21 - 3 + t, E[t], E[t + 1]);
      }
#pragma unroll
      for (int j = 0; j < 42; j++) {
        const int u0 = j - 11 + 12, u1 = j - 10 + 12;  // +12 keeps the offsets non-negative
        const uint32_t w0 = wsel(E[u0 >> 2], u0 & 3), w1 = wsel(E[u1 >> 2], u1 & 3);
        x[j] = __builtin_amdgcn_alignbit(w1, w0, 16);
      }
      if (b == 0) {
#pragma unroll
        for (int j = 0; j < 10; j++) x[j] = pre[j];
        x[10] = (pre[10] & 0xffffu) | (wsel(E[3], 0) << 16);
      }
    } else {
      // u = 84q + 31 + j: element 21q + 7 + floor((j+3)/4), word (j+3) mod 4; window 21q+7..21q+18
      uint4 E[12];
#pragma unroll
      for (int t = 0; t < 12; t++) E[t] = ldel(q21 + 7 + t);
      if (FUSE && fuse) {  // elements q21+8 .. q21+18 (E[1..11])
#pragma unroll
        for (int t = 1; t < 12; t += 2)
          fused_pair(q21 + 7 + t, E[t], t + 1 < 12 ? E[t + 1] : make_uint4(0, 0, 0, 0));
      }
#pragma unroll
      for (int j = 0; j < 42; j++) {
        const int u0 = j + 3, u1 = j + 4;
        const uint32_t w0 = wsel(E[u0 >> 2], u0 & 3), w1 = wsel(E[u1 >> 2], u1 & 3);
        x[j] = __builtin_amdgcn_alignbit(w1, w0, 16);
      }
    }
    if (b == B) {
#pragma unroll
      for (int j = 0; j < 42; j++) {
        const uint32_t lo = 4 * j;
        uint32_t mask = (lo + 4 <= rem) ? 0xffffffffu
                                        : (lo >= rem ? 0u : ((1u << (8 * (rem - lo))) - 1u));
        x[j] &= mask;
        if ((uint32_t)j == (rem >> 2)) x[j] ^= 1u << (8 * (rem & 3));
      }
      x[41] ^= 0x80000000u;
    }
#pragma unroll
    for (int j = 0; j < 42; j++) kxor_word(s, j, x[j]);
    keccak_p12(s);
  }
  uint32_t part[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
  uint32_t flag = sc.flag[r];
  uint32_t pub0[4];
  load16(in.pub + (size_t)r * p.public_share_len + (LEADER ? 16 : 0), pub0);
  KState c;
  kzero(c);
  {
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[6]);
    msg_bytes16(m, 25, LEADER ? part : pub0);
    msg_bytes16(m, 41, LEADER ? pub0 : part);
    msg_absorb_final(c, m, 57);
  }
  uint32_t cor[4] = {kword(c, 0), kword(c, 1), kword(c, 2), kword(c, 3)};
  {
    KState t;
    kzero(t);
    Msg m2;
    msg_zero(m2);
    msg_dst(m2, p.dst[3]);
    msg_bytes16(m2, 9, cor);
    msg_byte(m2, 25, 1);
    msg_absorb_final(t, m2, 26);
    uint32_t q0 = 0, q1 = 0;
    squeeze_block<Fp128>(p, t, 0, p.jr_len, q0, q1, sc.jr, r, flag);
  }
  sc.part[r] = make_uint4(part[0], part[1], part[2], part[3]);
  sc.corrected[r] = make_uint4(cor[0], cor[1], cor[2], cor[3]);
  sc.flag[r] = (uint8_t)flag;
}


// ------------------------------------------------------------------------------------
// k_leader_unpack: the leader's explicit input share (AoS, leader_input_share_len bytes per
// report) into the SoA measurement / proofs scratch with the canonical-encoding check, plus the
// query randomness (1 permutation) -- the leader analogue of k_xof_a.
// ------------------------------------------------------------------------------------
// wpart / wseg (non-null: the device leader's fused accumulate, leader_fuse_acc): while a chunk
// sits in LDS, thread (element tid / 8, half-limb tid % 8) also sums that 16-bit half-limb over
// the block's 64 reports -- the wave partials k_agg_waves reads (the layout of wave_halfsum2's)
// -- and the block's wave is marked fused for segment 0 when all 64 reports are present and
// canonical.
__global__ __launch_bounds__(256) void k_leader_unpack(DevParams p, InPtrs in, Scratch sc,
                                                       uint8_t* status, uint32_t* wpart,
                                                       uint32_t* wseg) {
  // block = 64 reports; the explicit shares are transposed through LDS in chunks of 32
  // elements (rows read 512 B contiguous per report, columns written 1 KiB contiguous per
  // element) -- per-lane row streaming of the 5.6 KiB rows ran at a fraction of HBM speed.
  typedef Fp128 F;
  constexpr int RB = 64, CE = 32;
  __shared__ uint4 tile[RB][CE + 1];
  __shared__ uint32_t bad[RB];
  const uint32_t tid = threadIdx.x, r0 = blockIdx.x * RB;
  const size_t ld = p.ld;
  const uint32_t M = p.meas_len, PL = p.proof_len, E = M + PL;
  const uint32_t nrep = min((uint32_t)RB, p.n - r0);
  if (tid < RB) bad[tid] = 0;
  for (uint32_t c0 = 0; c0 < E; c0 += CE) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RB * CE / 256; i++) {
      const uint32_t idx = tid + 256 * i, rr = idx / CE, e = c0 + idx % CE;
      if (rr < nrep && e < E) {
        const uint4 v =
            ((const uint4*)(in.helper + (size_t)(r0 + rr) * p.leader_share_len))[e];
        if (!F::lt_p(mk128(v.x, v.y, v.z, v.w))) atomicOr(&bad[rr], 1u);
        tile[rr][idx % CE] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RB * CE / 256; i++) {
      const uint32_t idx = tid + 256 * i, rr = idx % RB, el = idx / RB, e = c0 + el;
      if (rr < nrep && e < E) {
        if (e < M)
          ((uint4*)sc.meas)[(size_t)e * ld + r0 + rr] = tile[rr][el];
        else
          ((uint4*)sc.proofs)[(size_t)(e - M) * ld + r0 + rr] = tile[rr][el];
      }
    }
    if (wpart && nrep == RB && c0 < M) {  // uniform
      const uint32_t el = tid >> 3, h = tid & 7u, e = c0 + el;
      if (e < M) {
        uint32_t sum = 0;
#pragma unroll 8
        for (uint32_t rr = 0; rr < RB; rr++) {
          const uint32_t* w = (const uint32_t*)&tile[rr][el];
          sum += (w[h >> 1] >> ((h & 1u) * 16u)) & 0xffffu;
        }
        wpart[((size_t)blockIdx.x * M + e) * 8u + h] = sum;
      }
    }
  }
  __syncthreads();
  if (tid >= nrep) return;
  const uint32_t r = r0 + tid;
  uint32_t flag = p.force_slow;
  uint32_t nonce[4];
  load16(in.nonces + 16 * (size_t)r, nonce);
  KState s;
  kzero(s);
  Msg m;
  msg_zero(m);
  msg_dst(m, p.dst[5]);
  {
    uint32_t vk[4];
    load_vk(p, in, r, vk);  // coalesced groups of several tasks: the report's own key
    msg_bytes16(m, 9, vk);
  }
  msg_byte(m, 25, 1);
  msg_bytes16(m, 26, nonce);
  msg_absorb_final(s, m, 42);
  uint32_t w[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
  put_elem<F>(p, sc.qr, 0, r, w, flag);
  if (p.qr_len > 1) {  // FPVec: one query point per gadget, from the same squeeze block
    uint32_t w1[4] = {kword(s, 4), kword(s, 5), kword(s, 6), kword(s, 7)};
    put_elem<F>(p, sc.qr, 1, r, w1, flag);
  }
  sc.flag[r] = (uint8_t)flag;
  status[r] = bad[tid] ? PRIO3_STATUS_INPUT_SHARE_DECODE : PRIO3_STATUS_FINISHED;
  if (wseg) {
    const bool fuse = nrep == RB && __all(!bad[tid]);  // nrep == RB: all 64 lanes are here
    if (tid == 0) wseg[blockIdx.x] = fuse ? 0u : 0xffffffffu;
  }
}

// ------------------------------------------------------------------------------------
// k_leader_jr: k_leader_unpack + k_jrpart<false, true> in one launch.  Each lane absorbs its
// own report's measurement share into the joint-rand sponge straight from the AoS input (the
// 11-12 16-byte loads of a sponge block run back to back over the same 176-192 bytes of the
// row), checks the encodings and writes the SoA measurement / proofs scratch the query reads;
// the share is read from HBM once instead of twice.  Then the joint-rand part, corrected seed,
// joint randomness (k_jrpart) and the query randomness (k_leader_unpack).  wpart / wseg as
// k_leader_unpack's (the device leader's fused accumulate): the wave totals of each element by
// wave_halfsum2, the wave marked fused when all 64 reports are present and canonical.
// Interleaved on one box (profiles/r05/leader_jr/): 173.4-173.9 against 165.4-166.5 M reports/s
// for the two kernels (k_leader_jr 3.76 ms against 2.32 + 1.70 ms per 1 Mi).  Staging each
// sponge block's 64 x 11-12 elements through LDS with coalesced row segments instead (one wave
// per block, 12 KiB, 3 waves per SIMD) took 4.12 ms.
// ------------------------------------------------------------------------------------
DEV void leader_jr_body(const DevParams& p, const InPtrs& in, const Scratch& sc,
                        uint8_t* status, uint32_t* wpart, uint32_t* wseg, const uint32_t r) {
  typedef Fp128 F;
  const uint32_t lane = threadIdx.x & 63u;
  const bool acc = wpart != nullptr && __all(r < p.n);  // wave-uniform
  if (r >= p.n) return;
  const size_t ld = p.ld;
  const int M = (int)p.meas_len;
  const uint32_t PL = p.proof_len;
  const uint4* row = (const uint4*)(in.helper + (size_t)r * p.leader_share_len);
  // the executor's SoA staging (InPtrs::lin_ld): element e of report r at cell e * lin_ld + r
  const uint4* soa = (const uint4*)in.helper + r;
  const size_t sld = in.lin_ld;
  auto rel = [&](int e) -> uint4 { return sld ? soa[(size_t)e * sld] : row[e]; };
  uint32_t bad = 0;
  uint32_t nonce[4], kb[4];
  load16(in.nonces + 16 * (size_t)r, nonce);
  {
    const uint4 k = rel(M + (int)PL);
    kb[0] = k.x;
    kb[1] = k.y;
    kb[2] = k.z;
    kb[3] = k.w;
  }
  uint32_t pre[11];
  {
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[7]);
    msg_bytes16(m, 9, kb);
    msg_byte(m, 25, 0);
    msg_bytes16(m, 26, nonce);
#pragma unroll
    for (int j = 0; j < 11; j++) pre[j] = m.w[j];
  }
  uint4* meas = (uint4*)sc.meas;
  auto ldel = [&](int e) -> uint4 {
    const bool ok = e >= 0 && e < M;
    const uint4 v = rel(ok ? e : 0);
    return ok ? v : make_uint4(0, 0, 0, 0);
  };
  // element e (owned by this window): canonical check and the SoA copy
  auto own = [&](int e, const uint4& v) {
    if (e < 0 || e >= M) return;
    if (!F::lt_p(mk128(v.x, v.y, v.z, v.w))) bad = 1;
    meas[(size_t)e * ld + r] = v;
  };
  auto wsel = [](const uint4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; };
  // wave totals of elements e0, e0 + 1 (the second only if below lim)
  auto acc_pair = [&](int e0, const uint4& a, const uint4& b, int lim) {
    if (e0 + 1 < 0 || e0 >= M) return;  // wave-uniform
    const uint32_t tot = wave_halfsum2(mk128(a.x, a.y, a.z, a.w), mk128(b.x, b.y, b.z, b.w), lane);
    const int e = e0 + (int)(lane >> 5);
    if ((lane & 3u) == 0 && e >= 0 && e < M && e < lim)
      wpart[((size_t)(r >> 6) * (uint32_t)M + (uint32_t)e) * 8u + ((lane >> 2) & 7u)] = tot;
  };
  const uint32_t L = 42 + (uint32_t)M * 16;
  const uint32_t B = L / 168, rem = L % 168;
  KState s;
  kzero(s);
  for (uint32_t b = 0; b <= B; b++) {
    uint32_t x[42];
    const int q21 = 21 * (int)(b >> 1);
    if ((b & 1) == 0) {
      // window q21-3 .. q21+7; this block owns q21-2 .. q21+7 (E[1..10])
      uint4 E[11];
#pragma unroll
      for (int t = 0; t < 11; t++) E[t] = ldel(q21 - 3 + t);
#pragma unroll
      for (int t = 1; t < 11; t++) own(q21 - 3 + t, E[t]);
      if (acc) {
#pragma unroll
        for (int t = 1; t < 11; t += 2) acc_pair(q21 - 3 + t, E[t], E[t + 1], q21 + 8);
      }
#pragma unroll
      for (int j = 0; j < 42; j++) {
        const int u0 = j - 11 + 12, u1 = j - 10 + 12;
        const uint32_t w0 = wsel(E[u0 >> 2], u0 & 3), w1 = wsel(E[u1 >> 2], u1 & 3);
        x[j] = __builtin_amdgcn_alignbit(w1, w0, 16);
      }
      if (b == 0) {
#pragma unroll
        for (int j = 0; j < 10; j++) x[j] = pre[j];
        x[10] = (pre[10] & 0xffffu) | (wsel(E[3], 0) << 16);
      }
    } else {
      // window q21+7 .. q21+18; this block owns q21+8 .. q21+18 (E[1..11])
      uint4 E[12];
#pragma unroll
      for (int t = 0; t < 12; t++) E[t] = ldel(q21 + 7 + t);
#pragma unroll
      for (int t = 1; t < 12; t++) own(q21 + 7 + t, E[t]);
      if (acc) {
#pragma unroll
        for (int t = 1; t < 12; t += 2)
          acc_pair(q21 + 7 + t, E[t], t + 1 < 12 ? E[t + 1] : make_uint4(0, 0, 0, 0), q21 + 19);
      }
#pragma unroll
      for (int j = 0; j < 42; j++) {
        const int u0 = j + 3, u1 = j + 4;
        const uint32_t w0 = wsel(E[u0 >> 2], u0 & 3), w1 = wsel(E[u1 >> 2], u1 & 3);
        x[j] = __builtin_amdgcn_alignbit(w1, w0, 16);
      }
    }
    if (b == B) {
#pragma unroll
      for (int j = 0; j < 42; j++) {
        const uint32_t lo = 4 * j;
        uint32_t mask = (lo + 4 <= rem) ? 0xffffffffu
                                        : (lo >= rem ? 0u : ((1u << (8 * (rem - lo))) - 1u));
        x[j] &= mask;
        if ((uint32_t)j == (rem >> 2)) x[j] ^= 1u << (8 * (rem & 3));
      }
      x[41] ^= 0x80000000u;
    }
#pragma unroll
    for (int j = 0; j < 42; j++) kxor_word(s, j, x[j]);
    keccak_p12(s);
  }
  {  // the proofs share: canonical check and SoA copy
    uint4* proofs = (uint4*)sc.proofs;
    for (uint32_t e = 0; e < PL; e++) {
      const uint4 v = rel(M + (int)e);
      if (!F::lt_p(mk128(v.x, v.y, v.z, v.w))) bad = 1;
      proofs[(size_t)e * ld + r] = v;
    }
  }
  uint32_t flag = p.force_slow;
  {  // query randomness (k_leader_unpack)
    KState q;
    kzero(q);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[5]);
    {
      uint32_t vk[4];
      load_vk(p, in, r, vk);
      msg_bytes16(m, 9, vk);
    }
    msg_byte(m, 25, 1);
    msg_bytes16(m, 26, nonce);
    msg_absorb_final(q, m, 42);
    uint32_t w[4] = {kword(q, 0), kword(q, 1), kword(q, 2), kword(q, 3)};
    put_elem<F>(p, sc.qr, 0, r, w, flag);
  }
  uint32_t part[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
  uint32_t pub0[4];
  load16(in.pub + (size_t)r * p.public_share_len + 16, pub0);
  KState c;
  kzero(c);
  {
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[6]);
    msg_bytes16(m, 25, part);
    msg_bytes16(m, 41, pub0);
    msg_absorb_final(c, m, 57);
  }
  uint32_t cor[4] = {kword(c, 0), kword(c, 1), kword(c, 2), kword(c, 3)};
  {
    KState t;
    kzero(t);
    Msg m2;
    msg_zero(m2);
    msg_dst(m2, p.dst[3]);
    msg_bytes16(m2, 9, cor);
    msg_byte(m2, 25, 1);
    msg_absorb_final(t, m2, 26);
    uint32_t q0 = 0, q1 = 0;
    squeeze_block<Fp128>(p, t, 0, p.jr_len, q0, q1, sc.jr, r, flag);
  }
  sc.part[r] = make_uint4(part[0], part[1], part[2], part[3]);
  sc.corrected[r] = make_uint4(cor[0], cor[1], cor[2], cor[3]);
  sc.flag[r] = (uint8_t)flag;
  status[r] = bad ? PRIO3_STATUS_INPUT_SHARE_DECODE : PRIO3_STATUS_FINISHED;
  if (wseg) {
    const bool fuse = acc && __all(!bad);
    if (lane == 0) wseg[r >> 6] = fuse ? 0u : 0xffffffffu;
  }
}
__global__ __launch_bounds__(256, JR_OCC) void k_leader_jr(DevParams p, InPtrs in, Scratch sc,
                                                         uint8_t* status, uint32_t* wpart,
                                                         uint32_t* wseg) {
  leader_jr_body(p, in, sc, status, wpart, wseg, blockIdx.x * blockDim.x + threadIdx.x);
}

// Leader slow path: reports whose query or joint-rand expansion hit a rejection-sampling
// event (flagged by k_leader_unpack / k_jrpart) get both redone by the byte-level sponge.
__global__ __launch_bounds__(64) void k_leader_slowfix(DevParams p, InPtrs in, Scratch sc) {
  typedef Fp128 F;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n || !sc.flag[r]) return;
  uint32_t nonce[4];
  load16(in.nonces + 16 * (size_t)r, nonce);
  uint8_t b[17];
  b[0] = 1;
  for (int i = 0; i < 16; i++) b[1 + i] = (uint8_t)(nonce[i >> 2] >> (8 * (i & 3)));
  uint32_t vk[4];
  load_vk(p, in, r, vk);
  bx_expand<F>(p.dst[5], vk, b, 17, p.qr_len, sc.qr, p.ld, r);
  const uint4 c = sc.corrected[r];
  const uint32_t cor[4] = {c.x, c.y, c.z, c.w};
  bx_expand<F>(p.dst[3], cor, b, 1, p.jr_len, sc.jr, p.ld, r);
}

// ------------------------------------------------------------------------------------
// k_xof_slow: general byte-level sponge with rejection sampling (flagged reports only)
// ------------------------------------------------------------------------------------
// (byte-level sponge helpers BX / bx_* live in prio3_common.h)
// The sponges run one at a time (one Keccak state live): the joint-rand-part sponge absorbs the
// measurement share from the scratch rows this lane has just written, instead of beside the
template <class F, int SITE = 0>
__device__ __noinline__ void xof_slow_one(const DevParams& p, const InPtrs& in, const Scratch& sc,
                                          uint32_t r) {
  uint32_t nonce[4];
  load16(in.nonces + 16 * (size_t)r, nonce);
  const uint8_t* hs = in.helper + (size_t)r * p.helper_share_len;
  const bool JR = p.jr_len > 0;
  uint32_t w[4];
  {  // query rand
    BX x;
    uint32_t vk[4];
    load_vk(p, in, r, vk);
    bx_init(x, p.dst[5], vk);
    bx_absorb(x, 1);
    bx_absorb_w(x, nonce, 16);
    bx_finalize(x);
    for (uint32_t i = 0; i < p.qr_len; i++) {
      bx_next_elem<F>(x, w);
      F::store(sc.qr, (size_t)i * p.ld + r, F::from_words(w));
    }
  }
  {  // measurement share
    BX x;
    uint32_t km[4];
    load16(hs, km);
    bx_init(x, p.dst[1], km);
    bx_absorb(x, 1);
    bx_finalize(x);
    if constexpr (F::ES == 16) {
      TruncSink ts(p, sc.out, r);
      for (uint32_t i = 0; i < p.meas_len; i++) {
        bx_next_elem<F>(x, w);
        F::store(sc.meas, (size_t)i * p.ld + r, F::from_words(w));
        if (p.trunc_xof) ts.put(mk128(w[0], w[1], w[2], w[3]));
      }
    } else {
      for (uint32_t i = 0; i < p.meas_len; i++) {
        bx_next_elem<F>(x, w);
        F::store(sc.meas, (size_t)i * p.ld + r, F::from_words(w));
      }
    }
  }
  uint32_t part[4] = {0, 0, 0, 0};
  if (JR) {  // joint-rand part over the encoded share, read back from this lane's rows
    BX y;
    uint32_t kb[4];
    load16(hs + 32, kb);
    bx_init(y, p.dst[7], kb);
    bx_absorb(y, 1);
    bx_absorb_w(y, nonce, 16);
    for (uint32_t i = 0; i < p.meas_len; i++) {
      const typename F::T v = F::load(sc.meas, (size_t)i * p.ld + r);
      if constexpr (F::ES == 16) {
        w[0] = v.w[0], w[1] = v.w[1], w[2] = v.w[2], w[3] = v.w[3];
      } else {
        w[0] = (uint32_t)v, w[1] = (uint32_t)(v >> 32);
      }
      bx_absorb_w(y, w, F::ES);
    }
    bx_finalize(y);
    for (int k = 0; k < 4; k++) {
      uint32_t v = 0;
      for (int b = 0; b < 4; b++) v |= (uint32_t)bx_squeeze(y) << (8 * b);
      part[k] = v;
    }
  }
  {  // proofs
    BX x;
    uint32_t kp[4];
    load16(hs + 16, kp);
    bx_init(x, p.dst[2], kp);
    bx_absorb(x, 1);
    bx_absorb(x, 1);
    bx_finalize(x);
    for (uint32_t i = 0; i < p.proof_len; i++) {
      bx_next_elem<F>(x, w);
      F::store(sc.proofs, (size_t)i * p.ld + r, F::from_words(w));
    }
  }
  if (JR) {
    uint32_t cor[4];
    {
      BX x;
      uint32_t pub0[4], zero[4] = {0, 0, 0, 0};
      load16(in.pub + (size_t)r * p.public_share_len, pub0);
      bx_init(x, p.dst[6], zero);
      bx_absorb_w(x, pub0, 16);
      bx_absorb_w(x, part, 16);
      bx_finalize(x);
      for (int k = 0; k < 4; k++) {
        uint32_t v = 0;
        for (int b = 0; b < 4; b++) v |= (uint32_t)bx_squeeze(x) << (8 * b);
        cor[k] = v;
      }
    }
    BX y;
    bx_init(y, p.dst[3], cor);
    bx_absorb(y, 1);
    bx_finalize(y);
    for (uint32_t i = 0; i < p.jr_len; i++) {
      bx_next_elem<F>(y, w);
      F::store(sc.jr, (size_t)i * p.ld + r, F::from_words(w));
    }
    sc.part[r] = make_uint4(part[0], part[1], part[2], part[3]);
    sc.corrected[r] = make_uint4(cor[0], cor[1], cor[2], cor[3]);
  }
  sc.flag[r] = p.slow_defer ? 2u : 0u;
}

// The slow path's launch: each lane scans the flags of 16 reports with one 16-byte load and
// re-runs the byte-level XOF only for flagged ones (a rejection has probability ~2^-59 per
// Field128 element, so in practice every lane exits after its one load; the old one-lane-per-
// report grid of 64-thread blocks cost a mean 15 us per launch).
template <class F, int RPL = 16>
__global__ __launch_bounds__(64) void k_xof_slow(DevParams p, InPtrs in, Scratch sc) {
  const uint32_t r0 = (blockIdx.x * blockDim.x + threadIdx.x) * RPL;
  if (r0 >= p.n) return;
  const uint8_t* fl = sc.flag + r0;
  uint32_t any = 0;
  if (RPL == 16 && r0 + 16 <= p.n && ((uintptr_t)fl & 15) == 0) {
    const uint4 v = *(const uint4*)fl;
    any = v.x | v.y | v.z | v.w;
  } else {
    for (uint32_t i = 0; i < RPL && r0 + i < p.n; i++) any |= fl[i];
  }
  if (!any) return;
  for (uint32_t i = 0; i < RPL && r0 + i < p.n; i++)
    if (fl[i]) xof_slow_one<F>(p, in, sc, r0 + i);
}

// launch geometry of k_xof_slow: 16 reports per lane, one wave per block (a one-wave block
// needs one SIMD with room for it, not four on one CU, beside the other streams' kernels)
static inline uint32_t slow_blocks(uint32_t n) { return (n + 1023) / 1024; }
// the deferred slow path's redo launches (k_slow_redo*): REDO_RPL reports scanned per lane, so a
// run without flagged reports costs few waves
constexpr uint32_t REDO_RPL = 64;
static inline uint32_t redo_blocks(uint32_t n) {
  return (n + 64 * REDO_RPL - 1) / (64 * REDO_RPL);
}
// any flag among reports [r0, r0 + REDO_RPL) of the run
__device__ __forceinline__ bool redo_any(const DevParams& p, const Scratch& sc, uint32_t r0) {
  const uint8_t* fl = sc.flag + r0;
  uint32_t any = 0;
  if (r0 + REDO_RPL <= p.n && ((uintptr_t)fl & 15) == 0) {
#pragma unroll
    for (uint32_t k = 0; k < REDO_RPL / 16; k++) {
      const uint4 v = ((const uint4*)fl)[k];
      any |= v.x | v.y | v.z | v.w;
    }
  } else {
    for (uint32_t i = 0; i < REDO_RPL && r0 + i < p.n; i++) any |= fl[i];
  }
  return any != 0;
}
template <class F>
static void launch_xof_slow(const prio3_engine* e, const DevParams& p, const InPtrs& in,
                            const Scratch& sc, hipStream_t st);

// ------------------------------------------------------------------------------------
// k_query: FLP query + decide + prepare message + prepare_next + truncate
// ------------------------------------------------------------------------------------
template <class F>
__device__ __forceinline__ void query_body(const DevParams& p, const InPtrs& in, const Scratch& sc,
                                           const OutPtrs& out, const uint32_t r) {
  typedef typename F::T T;
  // r: this lane's report; slow_defer / redo (DevParams) as in query_h_body
  if (r >= p.n) return;
  if (p.redo) {
    if (sc.flag[r] != 2) return;
  } else if (p.slow_defer && sc.flag[r]) {
    return;
  }
  const size_t ld = p.ld;
  const uint32_t A = p.arity;
  uint8_t status = PRIO3_STATUS_FINISHED;
  const T t = ldf<F>(sc.qr, 0, ld, r);
  T v, pt;
  if (!flp_query_lane<F>(p, sc.meas, sc.proofs, sc.jr, t, sc.Lbuf, sc.PVbuf, sc.acc, r, v, pt))
    status = PRIO3_STATUS_PREP_INIT;
  // combine with the leader's verifier share and decide
  const uint8_t* lps = in.leader + (size_t)r * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    T x = F::load(lps, e);
    if (!F::lt_p(x)) decode_ok = false;
    return x;
  };
  const T V0 = F::add(lv(0), v);
  T G = F::zero();
  if (p.kind == PRIO3_COUNT) {
    T a = F::add(lv(1), F::load(sc.acc, 0 * ld + r));
    T b = F::add(lv(2), F::load(sc.acc, 1 * ld + r));
    G = F::mul(a, b);
  } else if (p.kind == PRIO3_SUM) {
    T a = F::add(lv(1), F::load(sc.acc, r));
    G = F::sub(F::mul(a, a), a);
  } else {
    for (uint32_t j = 0; j < p.chunk; j++) {
      T a = F::add(lv(1 + 2 * j), F::load(sc.acc, (size_t)(2 * j) * ld + r));
      T b = F::add(lv(2 + 2 * j), F::load(sc.acc, (size_t)(2 * j + 1) * ld + r));
      G = F::add(G, F::mul(a, b));
    }
  }
  const T PT = F::add(lv(A + 1), pt);
  if (status == PRIO3_STATUS_FINISHED) {
    if (!decode_ok)
      status = PRIO3_STATUS_PREP_SHARE_DECODE;
    else if (!F::is_zero(V0) || !F::eq(G, PT))
      status = PRIO3_STATUS_PREP_MSG;
  }
  uint32_t msg[4] = {0, 0, 0, 0};
  if (p.jr_len > 0) {
    uint32_t lpart[4], hpart[4];
    load16(lps + (size_t)p.verifier_len * F::ES, lpart);
    uint4 hp = sc.part[r];
    hpart[0] = hp.x;
    hpart[1] = hp.y;
    hpart[2] = hp.z;
    hpart[3] = hp.w;
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[6]);
    msg_bytes16(m, 25, lpart);
    msg_bytes16(m, 41, hpart);
    msg_absorb_final(s, m, 57);
    uint4 cor = sc.corrected[r];
    msg[0] = kword(s, 0);
    msg[1] = kword(s, 1);
    msg[2] = kword(s, 2);
    msg[3] = kword(s, 3);
    if (status == PRIO3_STATUS_FINISHED &&
        (msg[0] != cor.x || msg[1] != cor.y || msg[2] != cor.z || msg[3] != cor.w))
      status = PRIO3_STATUS_PREP_NEXT;
    if (status != PRIO3_STATUS_FINISHED) msg[0] = msg[1] = msg[2] = msg[3] = 0;
    ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
  }
  out.status[r] = status;
  // truncate (Count/Histogram: identity, read straight from the meas scratch)
  if (p.kind == PRIO3_SUM) {
    T acc = F::zero(), pw = F::one();
    for (uint32_t i = 0; i < p.meas_len; i++) {
      acc = F::add(acc, F::mul(pw, ldf<F>(sc.meas, i, ld, r)));
      pw = F::add(pw, pw);
    }
    F::store(sc.out, r, acc);
  } else if (p.kind == PRIO3_SUMVEC) {
    for (uint32_t e = 0; e < p.out_len; e++) {
      T acc = F::zero(), pw = F::one();
      for (uint32_t b = 0; b < p.bits; b++) {
        acc = F::add(acc, F::mul(pw, ldf<F>(sc.meas, e * p.bits + b, ld, r)));
        pw = F::add(pw, pw);
      }
      F::store(sc.out, (size_t)e * ld + r, acc);
    }
  }
}
template <class F>
__global__ __launch_bounds__(256) void k_query(DevParams p, InPtrs in, Scratch sc, OutPtrs out) {
  query_body<F>(p, in, sc, out, blockIdx.x * blockDim.x + threadIdx.x);
}

// k_prep_gen<F>: the generic XOF and query of one report on one lane in one launch (Prio3Count,
// C1), the slow path deferred to the run's redo launch, as k_prep_h.  (Taking the byte-level
// sponge inline for a flagged report instead -- a noinline call in the kernel -- doubled the
// kernel, 37.6 -> 73.6 us per 100k, r05ai; the 13 us redo launch stays.)
template <class F>
__global__ __launch_bounds__(256) void k_prep_gen(DevParams p, InPtrs in, Scratch sc, OutPtrs out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  xof_body<F>(p, in, sc, r);
  query_body<F>(p, in, sc, out, r);
}

// k_slow_redo_gen<F>: k_prep_gen's deferred slow path in one launch (as k_slow_redo): each lane
// scans the flags of REDO_RPL reports and, for a flagged one, re-runs its XOF on the
// byte-level sponge (flag := 2) and then its query (p.redo = 1)
template <class F>
__global__ __launch_bounds__(64) void k_slow_redo_gen(DevParams p, InPtrs in, Scratch sc,
                                                      OutPtrs out) {
  const uint32_t r0 = (blockIdx.x * blockDim.x + threadIdx.x) * REDO_RPL;
  if (r0 >= p.n || !redo_any(p, sc, r0)) return;
  const uint8_t* fl = sc.flag + r0;
  for (uint32_t i = 0; i < REDO_RPL && r0 + i < p.n; i++)
    if (fl[i]) {
      xof_slow_one<F>(p, in, sc, r0 + i);
      query_body<F>(p, in, sc, out, r0 + i);
    }
}

// ------------------------------------------------------------------------------------
// k_query_ps: FLP query + decide for the ParallelSum(Mul, C) circuits (Histogram, SumVec).
//
// Wire 2j of gadget call k carries r^(Ck+j+1) m_(Ck+j), wire 2j+1 carries m_(Ck+j) - 1/2, so
// with beta_k = L_(k+1)(t) r^(Ck):
//   f_2j(t)   = seed_2j L_0 + r^(j+1) sum_k beta_k m_(Ck+j)
//   f_2j+1(t) = seed_2j+1 L_0 + sum_k L_(k+1) m_(Ck+j) - (1/2) sum_k L_(k+1)
// The 2C wire accumulators are swept GS wires-pairs at a time in registers (each measurement
// element is read exactly once from HBM), two Field128 multiplies per element.
// ------------------------------------------------------------------------------------
template <int GS>
__global__ __launch_bounds__(256) void k_query_ps(DevParams p, InPtrs in, Scratch sc,
                                                  OutPtrs out) {
  typedef Fp128 F;
  typedef f128 T;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  const size_t ld = p.ld;
  const uint32_t P = p.P, A = p.arity, C = p.chunk, M = p.meas_len, K = p.calls;
  uint8_t status = PRIO3_STATUS_FINISHED;
  const T t = ldf<F>(sc.qr, 0, ld, r);
  {
    T tp = t;
    for (uint32_t l = 0; l < p.logP; l++) tp = F::mul(tp, tp);
    if (F::eq(tp, F::one())) status = PRIO3_STATUS_PREP_INIT;
  }
  // Lagrange basis at t (one size-P DFT of t^e/P) and gadget polynomial at the P-th roots
  {
    T pw = FC<F>::invP(p);
    for (uint32_t e = 0; e < P; e++) {
      F::store(sc.Lbuf, (size_t)bitrev(e, p.logP) * ld + r, pw);
      pw = F::mul(pw, t);
    }
    dft_lane<F>(p, sc.Lbuf, r, P, p.logP);
    for (uint32_t e = 0; e < P; e++) {
      T q = ldf<F>(sc.proofs, A + e, ld, r);
      if (e + P < p.glen) q = F::add(q, ldf<F>(sc.proofs, A + e + P, ld, r));
      F::store(sc.PVbuf, (size_t)bitrev(e, p.logP) * ld + r, q);
    }
    dft_lane<F>(p, sc.PVbuf, r, P, p.logP);
  }
  auto Lc = [&](uint32_t c) { return ldf<F>(sc.Lbuf, (P - c) & (P - 1), ld, r); };
  T pt = F::zero();
  for (uint32_t e = p.glen; e-- > 0;) pt = F::add(F::mul(pt, t), ldf<F>(sc.proofs, A + e, ld, r));
  // beta_k, sum of L_(k+1), sum of p(alpha^(k+1))
  const T r0 = ldf<F>(sc.jr, 0, ld, r);
  T rC = F::one();
  for (uint32_t j = 0; j < C; j++) rC = F::mul(rC, r0);
  T sumL = F::zero(), range = F::zero();
  {
    T rk = F::one();
    for (uint32_t k = 0; k < K; k++) {
      const T L = Lc(k + 1);
      sumL = F::add(sumL, L);
      range = F::add(range, ldf<F>(sc.PVbuf, k + 1, ld, r));
      F::store(sc.beta, (size_t)k * ld + r, F::mul(L, rk));
      rk = F::mul(rk, rC);
    }
  }
  const T L0 = Lc(0);
  const T half = FC<F>::half(p);
  const T halfL = F::mul(half, sumL);
  const uint8_t* lps = in.leader + (size_t)r * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    T x = F::load(lps, e);
    if (!F::lt_p(x)) decode_ok = false;
    return x;
  };
  T S = F::zero(), G = F::zero(), rj = r0;
  const T Z = F::zero();
  for (uint32_t jg = 0; jg < C; jg += GS) {
    T Aa[GS], Bb[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) Aa[q] = Bb[q] = Z;
    // software-pipelined as in k_query_fp: call k+1's loads are in flight during call k's
    // products; invalid slots load element 0 and are zeroed at use
    auto ldm = [&](uint32_t k, int q) {
      const uint32_t i = k * C + jg + (uint32_t)q;
      return ldf<F>(sc.meas, (jg + q < C && i < M) ? i : 0, ld, r);
    };
    T be_n = ldf<F>(sc.beta, 0, ld, r), L_n = Lc(1), mn[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) mn[q] = ldm(0, q);
#pragma unroll 1
    for (uint32_t k = 0; k < K; k++) {
      const T be = be_n, L = L_n;
      T mc[GS];
#pragma unroll
      for (int q = 0; q < GS; q++) mc[q] = mn[q];
      const uint32_t kn = k + 1 < K ? k + 1 : k;
      be_n = ldf<F>(sc.beta, kn, ld, r);
      L_n = Lc(kn + 1);
#pragma unroll
      for (int q = 0; q < GS; q++) mn[q] = ldm(kn, q);
      const uint32_t base = k * C + jg;
#pragma unroll
      for (int q = 0; q < GS; q++) {
        const bool valid = (jg + q < C) && (base + q < M);
        const T m = F::sel(valid, mc[q], Z);
        Aa[q] = F::add(Aa[q], F::mul(be, m));
        Bb[q] = F::add(Bb[q], F::mul(L, m));
        S = F::add(S, m);
      }
    }
#pragma unroll
    for (int q = 0; q < GS; q++) {
      const uint32_t j = jg + q;
      const bool valid = j < C;
      const uint32_t jj = valid ? j : 0;
      const T f0 = F::add(F::mul(ldf<F>(sc.proofs, 2 * jj, ld, r), L0), F::mul(rj, Aa[q]));
      const T f1 = F::sub(F::add(F::mul(ldf<F>(sc.proofs, 2 * jj + 1, ld, r), L0), Bb[q]), halfL);
      const T prod = F::mul(F::add(lv(1 + 2 * jj), f0), F::add(lv(2 + 2 * jj), f1));
      G = F::add(G, F::sel(valid, prod, Z));
      rj = F::sel(valid, F::mul(rj, r0), rj);
    }
  }
  T v;
  if (p.kind == PRIO3_SUMVEC) {
    v = range;
  } else {
    const T r1 = ldf<F>(sc.jr, 1, ld, r);
    v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), F::sub(S, half)));
  }
  const T V0 = F::add(lv(0), v);
  const T PT = F::add(lv(A + 1), pt);
  if (status == PRIO3_STATUS_FINISHED) {
    if (!decode_ok)
      status = PRIO3_STATUS_PREP_SHARE_DECODE;
    else if (!F::is_zero(V0) || !F::eq(G, PT))
      status = PRIO3_STATUS_PREP_MSG;
  }
  uint32_t lpart[4], hpart[4];
  load16(lps + (size_t)p.verifier_len * F::ES, lpart);
  {
    uint4 hp = sc.part[r];
    hpart[0] = hp.x;
    hpart[1] = hp.y;
    hpart[2] = hp.z;
    hpart[3] = hp.w;
  }
  KState s;
  kzero(s);
  Msg mm;
  msg_zero(mm);
  msg_dst(mm, p.dst[6]);
  msg_bytes16(mm, 25, lpart);
  msg_bytes16(mm, 41, hpart);
  msg_absorb_final(s, mm, 57);
  uint4 cor = sc.corrected[r];
  uint32_t msg[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
  if (status == PRIO3_STATUS_FINISHED &&
      (msg[0] != cor.x || msg[1] != cor.y || msg[2] != cor.z || msg[3] != cor.w))
    status = PRIO3_STATUS_PREP_NEXT;
  if (status != PRIO3_STATUS_FINISHED) msg[0] = msg[1] = msg[2] = msg[3] = 0;
  ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
  out.status[r] = status;
  if (p.kind == PRIO3_SUMVEC) {
    for (uint32_t e = 0; e < p.out_len; e++) {
      T acc = F::zero(), pw = F::one();
      for (uint32_t b = 0; b < p.bits; b++) {
        acc = F::add(acc, F::mul(pw, ldf<F>(sc.meas, e * p.bits + b, ld, r)));
        pw = F::add(pw, pw);
      }
      F::store(sc.out, (size_t)e * ld + r, acc);
    }
  }
}

// ------------------------------------------------------------------------------------
// k_query_h<GS, PP>: k_query_ps specialised for a compile-time wire-polynomial length
// PP <= 32 (Prio3Histogram(256,16) has PP = 32).  The Lagrange basis comes from an
// in-register PP-point DFT of (t^e / P) -- no scratch round trips -- and the circuit only
// needs sum_c p(alpha^c) = sum_e coef_e * sigma_(e mod P) (sigma precomputed on the host),
// so the gadget polynomial is never evaluated on the roots.  The measurement loads of the
// next gadget call are issued before the current call's arithmetic (register double buffer).
// ------------------------------------------------------------------------------------
// LEADER = 1: the leader's prepare_init (agg_id 0) on the same data flow -- the wire values
// f_j(t), v and p(t) are written as the leader prepare share (out.prep_msgs is the prepare
// share buffer, stride prep_share_len) instead of being decided against a peer's share.
// QH_BLOCK_HORNER: p(t) in blocks of eight lazy MACs (below); 0 = the plain Horner chain (A/B)
#ifndef QH_BLOCK_HORNER
#define QH_BLOCK_HORNER 1
#endif
template <int GS, int PP, int LEADER = 0>
__device__ __forceinline__ void query_h_body(const DevParams& p, const InPtrs& in, const Scratch& sc,
                                             const OutPtrs& out, const uint32_t r) {
  typedef Fp128 F;
  typedef f128 T;
  constexpr int LOGP = PP <= 2 ? 1 : PP <= 4 ? 2 : PP <= 8 ? 3 : PP <= 16 ? 4 : 5;
  if (r >= p.n) return;
  // slow_defer: a report the XOF flagged (a rejected sample) is skipped here; after the whole
  // run, k_xof_slow re-runs its XOF (flag := 2) and this kernel runs again with p.redo = 1 for
  // exactly those reports -- no k_xof_slow launch between the XOF and the query of each chunk
  if constexpr (!LEADER) {
    if (p.redo) {
      if (sc.flag[r] != 2) return;
    } else if (p.slow_defer && sc.flag[r]) {
      return;
    }
  } else {
    // the fused leader kernel (k_leader_prep) defers a flagged report; k_leader_slowfix redoes
    // its randomness and this query runs again for exactly those reports (p.redo)
    if (p.redo) {
      if (!sc.flag[r]) return;
    } else if (p.slow_defer && sc.flag[r]) {
      return;
    }
  }
  const size_t ld = p.ld;
  const uint32_t A = p.arity, C = p.chunk, M = p.meas_len, K = p.calls;
  uint8_t status = LEADER ? out.status[r] : PRIO3_STATUS_FINISHED;  // leader: unpack verdict
  uint8_t* lout = LEADER ? out.prep_msgs + (size_t)r * p.prep_share_len : nullptr;
  const T t = ldf<F>(sc.qr, 0, ld, r);
  T L0, sumL = F::zero();
  // u_e = t^e / P.  PP <= 16: one in-register DFT.  PP == 32: decimation in frequency,
  // X[2k] = DFT16(u_e + u_(e+16)), X[2k+1] = DFT16((u_e - u_(e+16)) w32^e), each a geometric
  // sequence, so only 16 values (64 VGPRs) are live at a time.
  auto store_L = [&](int idx, const T& val) {  // X[idx] = L_c with c = (P - idx) mod P
    const uint32_t c = (uint32_t)((PP - idx) & (PP - 1));
    if (c == 0) {
      L0 = val;
    } else if (c <= K) {
      F::store(sc.Lbuf, (size_t)c * ld + r, val);
      sumL = F::add(sumL, val);
    }
  };
  if constexpr (PP <= 16) {
    T x[PP];
    T pw = FC<F>::invP(p);
#pragma unroll
    for (int e = 0; e < PP; e++) {
      x[__builtin_bitreverse32(e) >> (32 - LOGP)] = pw;
      pw = F::mul(pw, t);
    }
    if (F::eq(pw, FC<F>::invP(p))) status = PRIO3_STATUS_PREP_INIT;  // t^P == 1
    dft_reg<PP, LOGP>(p, x, 1);
#pragma unroll
    for (int k = 0; k < PP; k++) store_L(k, x[k]);
  } else {
    static_assert(PP == 32, "PP must be <= 32");
    // Four phases of an 8-point DFT: X[4k + ph] = DFT8(y^ph)[k] with y^ph_n = (G_ph / P)(t w^ph)^n,
    // w = w32 and G_ph = sum_(i<4) (t^8 w4^ph)^i, so only 8 values (32 VGPRs) are live at a time
    // (two 16-point phases held 64 and spilled at 168 VGPRs).
    T t8 = t;
#pragma unroll
    for (int i = 0; i < 3; i++) t8 = F::mul(t8, t8);
    const T t16 = F::mul(t8, t8);
    const T t32 = F::mul(t16, t16);
    if (F::eq(t32, F::one())) status = PRIO3_STATUS_PREP_INIT;
    const T ip = FC<F>::invP(p);
    const T a = F::add(F::one(), t16), b = F::sub(F::one(), t16);
    const T c = F::mul(t8, a), wd = F::mul(F::mul(t8, b), F::from_words(p.tw128[8]));  // w4 = w32^8
#pragma unroll
    for (int ph = 0; ph < 4; ph++) {
      const T g = ph == 0 ? F::add(a, c) : ph == 1 ? F::add(b, wd) : ph == 2 ? F::sub(a, c)
                                                                              : F::sub(b, wd);
      T x[8];
      T pw = F::mul(ip, g);
      const T ratio = ph == 0 ? t : F::mul(t, F::from_words(p.tw128[ph]));
#pragma unroll
      for (int e = 0; e < 8; e++) {
        x[__builtin_bitreverse32(e) >> 29] = pw;
        if (e + 1 < 8) pw = F::mul(pw, ratio);
      }
      dft_reg<8, 3>(p, x, 4);
#pragma unroll
      for (int k = 0; k < 8; k++) store_L(4 * k + ph, x[k]);
    }
  }
  // p(t) and range = sum_c p(alpha^c) = sum_e coef_e sigma_(e mod P); the range sum is a lazily
  // reduced dot product with the (uniform) sigma.
  T pt = F::zero(), range;
#if QH_BLOCK_HORNER
  // p(t) = sum_q (t^8)^q S_q, S_q = sum_(i<8) coef_(8q+i) t^i: 63 lazy MACs against t^0..t^7
  // (6 multiplies), one reduction per block of eight and a Horner step in t^8 per block -- 13
  // full multiplies + 8 reductions instead of 63 multiplies (r05)
  {
    constexpr int GLEN = 2 * (PP - 1) + 1, NB = (GLEN + 7) / 8;
    T pw[8];
    pw[0] = F::one();
    pw[1] = t;
#pragma unroll
    for (int i = 2; i < 8; i++) pw[i] = F::mul(pw[i - 1], t);
    const T t8b = F::mul(pw[7], t);
    mac128 R;
    mac_zero(R);
    auto ldc = [&](int e) { return ldf<F>(sc.proofs, A + (e < GLEN ? e : 0), ld, r); };
    T cb[8];
#pragma unroll
    for (int i = 0; i < 8; i++) cb[i] = ldc(8 * (NB - 1) + i);
#pragma unroll 1
    for (int q = NB - 1; q >= 0; q--) {
      T cn[8];
      const int qn = q > 0 ? q - 1 : 0;
#pragma unroll
      for (int i = 0; i < 8; i++) cn[i] = ldc(8 * qn + i);  // the next block's, one block ahead
      mac128 S;
      mac_zero(S);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int e = 8 * q + i;
        if (e < GLEN) {  // uniform
          mac_add(S, cb[i], pw[i]);
          mac_add(R, cb[i], F::from_words(p.sigma128[e & (PP - 1)]));
        }
        cb[i] = cn[i];
      }
      const T sq = mac_reduce_f(S);
      pt = q == NB - 1 ? sq : F::add(F::mul(pt, t8b), sq);
    }
    range = mac_reduce_f(R);
  }
#else
  {
    mac128 R;
    mac_zero(R);
    // glen = 2 (PP - 1) + 1 for the degree-2 ParallelSum(Mul) gadget; the coefficients are
    // loaded HD ahead (one exposed load latency per coefficient otherwise).
    constexpr int GLEN = 2 * (PP - 1) + 1, HD = 4;
    auto ldc = [&](int q) {  // coefficient e = GLEN-1-q (clamped; unused past the end)
      const int e = GLEN - 1 - q;
      return ldf<F>(sc.proofs, A + (e >= 0 ? e : 0), ld, r);
    };
    T cb[HD];
#pragma unroll
    for (int q = 0; q < HD; q++) cb[q] = ldc(q);
#pragma unroll 1
    for (int q0 = 0; q0 < GLEN; q0 += HD) {
      T cn[HD];
#pragma unroll
      for (int q = 0; q < HD; q++) cn[q] = ldc(q0 + HD + q);
#pragma unroll
      for (int q = 0; q < HD; q++) {
        const int e = GLEN - 1 - (q0 + q);
        if (e >= 0) {
          pt = F::add(F::mul(pt, t), cb[q]);
          mac_add(R, cb[q], F::from_words(p.sigma128[e & (PP - 1)]));
        }
        cb[q] = cn[q];
      }
    }
    range = mac_reduce_f(R);
  }
#endif
  const T r0 = ldf<F>(sc.jr, 0, ld, r);
  {
    // r0^C by square-and-multiply over the (uniform) bits of C
    T rC = F::one(), sq = r0;
    for (uint32_t e = C; e; e >>= 1) {
      if (e & 1) rC = F::mul(rC, sq);
      if (e > 1) sq = F::mul(sq, sq);
    }
    // beta_k = L_(k+1) r^(Ck), eight L values loaded at a time
    T rk = F::one();
    for (uint32_t k0 = 0; k0 < K; k0 += 8) {
      T lb[8];
#pragma unroll
      for (int q = 0; q < 8; q++) lb[q] = ldf<F>(sc.Lbuf, k0 + q < K ? k0 + q + 1 : 1, ld, r);
#pragma unroll
      for (int q = 0; q < 8; q++) {
        if (k0 + q < K) {
          F::store(sc.beta, (size_t)(k0 + q) * ld + r, F::mul(lb[q], rk));
          rk = F::mul(rk, rC);
        }
      }
    }
  }
  const T half = FC<F>::half(p);
  const T halfL = F::mul(half, sumL);
  const uint8_t* lps = in.leader + (size_t)r * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    T x = F::load(lps, e);
    if (!F::lt_p(x)) decode_ok = false;
    return x;
  };
  sum128 Ssum;
  sum_zero(Ssum);
  T G = F::zero(), rj = r0;
  for (uint32_t jg = 0; jg < C; jg += GS) {
    mac128 Aa[GS], Bb[GS];
    T mc[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) {
      mac_zero(Aa[q]);
      mac_zero(Bb[q]);
    }
    // One dwordx4 load per element from a clamped (always in-bounds) address; padding
    // elements are zeroed with a wave-uniform mask (a select on the loaded value made the
    // compiler split the load into four branch-guarded dword loads).
    auto fetch = [&](uint32_t k, T* dst) {
#pragma unroll
      for (int q = 0; q < GS; q++) {
        const uint32_t i = k * C + jg + q;
        const bool valid = (k < K) && (jg + q < C) && (i < M);
        const uint32_t msk = valid ? 0xffffffffu : 0u;
        const uint4 v = ((const uint4*)sc.meas)[(size_t)(valid ? i : 0) * ld + r];
        dst[q] = mk128(v.x & msk, v.y & msk, v.z & msk, v.w & msk);
      }
    };
    fetch(0, mc);
    // The per-call coefficients beta_k, L_(k+1) of the next call are loaded together with its
    // measurement elements, one iteration ahead (they come from L2/MALL, and loading them at
    // their use left the waves parked on s_waitcnt).
    T be = ldf<F>(sc.beta, 0, ld, r), Lk = ldf<F>(sc.Lbuf, 1, ld, r);
#pragma unroll 1
    for (uint32_t k = 0; k < K; k++) {
      T mn[GS];
      fetch(k + 1, mn);
      const uint32_t kn = k + 1 < K ? k + 1 : k;
      const T be_n = ldf<F>(sc.beta, kn, ld, r), L_n = ldf<F>(sc.Lbuf, kn + 1, ld, r);
#pragma unroll
      for (int q = 0; q < GS; q++) {
        mac_add(Aa[q], be, mc[q]);
        mac_add(Bb[q], Lk, mc[q]);
        sum_add(Ssum, mc[q]);
      }
#pragma unroll
      for (int q = 0; q < GS; q++) mc[q] = mn[q];
      be = be_n;
      Lk = L_n;
    }
    // Wire values at t, lazily reduced: f1 = seed_(2j+1) L0 + B_j - L/2 folds the seed term into
    // B's accumulator, f0 = seed_2j L0 + r^(j+1) A_j is one two-product MAC, and the gadget
    // products of the group are summed in one MAC before a single reduction.
    mac128 Gq;
    mac_zero(Gq);
#pragma unroll
    for (int q = 0; q < GS; q++) {
      const uint32_t j = jg + q;
      if (j < C) {  // wave-uniform
        mac_add(Bb[q], ldf<F>(sc.proofs, 2 * j + 1, ld, r), L0);
        const T f1 = F::sub(mac_reduce_f(Bb[q]), halfL);
        const T Aq = mac_reduce_f(Aa[q]);
        mac128 F0;
        mac_zero(F0);
        mac_add(F0, ldf<F>(sc.proofs, 2 * j, ld, r), L0);
        mac_add(F0, rj, Aq);
        const T f0 = mac_reduce_f(F0);
        if constexpr (LEADER) {
          F::store(lout, 1 + 2 * j, f0);
          F::store(lout, 2 + 2 * j, f1);
        } else {
          mac_add(Gq, F::add(lv(1 + 2 * j), f0), F::add(lv(2 + 2 * j), f1));
        }
        rj = F::mul(rj, r0);
      }
    }
    if constexpr (!LEADER) G = F::add(G, mac_reduce_f(Gq));
  }
  const T S = sum_reduce(Ssum);
  T v;
  if (p.kind == PRIO3_SUMVEC) {
    v = range;
  } else {
    const T r1 = ldf<F>(sc.jr, 1, ld, r);
    v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), F::sub(S, half)));
  }
  if constexpr (LEADER) {
    F::store(lout, 0, v);
    F::store(lout, A + 1, pt);
    *(uint4*)(lout + (size_t)p.verifier_len * F::ES) = sc.part[r];
    out.status[r] = status;
  } else {
  const T V0 = F::add(lv(0), v);
  const T PT = F::add(lv(A + 1), pt);
  if (status == PRIO3_STATUS_FINISHED) {
    if (!decode_ok)
      status = PRIO3_STATUS_PREP_SHARE_DECODE;
    else if (!F::is_zero(V0) || !F::eq(G, PT))
      status = PRIO3_STATUS_PREP_MSG;
  }
  uint32_t lpart[4], msg[4];
  load16(lps + (size_t)p.verifier_len * F::ES, lpart);
  if (!prep_msg_check(p, in, sc, r, lpart, msg) && status == PRIO3_STATUS_FINISHED)
    status = PRIO3_STATUS_PREP_NEXT;
  if (status != PRIO3_STATUS_FINISHED) msg[0] = msg[1] = msg[2] = msg[3] = 0;
  ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
  out.status[r] = status;
  }
  if (p.kind == PRIO3_SUMVEC) {
    for (uint32_t e = 0; e < p.out_len; e++) {
      T acc = F::zero(), pw = F::one();
      for (uint32_t b = 0; b < p.bits; b++) {
        acc = F::add(acc, F::mul(pw, ldf<F>(sc.meas, e * p.bits + b, ld, r)));
        pw = F::add(pw, pw);
      }
      F::store(sc.out, (size_t)e * ld + r, acc);
    }
  }
}
template <int GS, int PP, int LEADER = 0>
__global__ __launch_bounds__(256, 3) void k_query_h(DevParams p, InPtrs in, Scratch sc,
                                                  OutPtrs out) {
  query_h_body<GS, PP, LEADER>(p, in, sc, out, blockIdx.x * blockDim.x + threadIdx.x);
}

// k_prep_h<FUSE>: the whole helper prepare of Prio3Histogram with P = 32 in one launch -- the
// dual-state XOF (xofd_body) and then the query (query_h_body; flagged reports deferred to the
// run's redo pass, slow_defer) of the same 64 reports on the same wave.  Both phases fit 3 waves per SIMD, and the waves of a
// SIMD drift apart, so one wave's memory-bound query runs beside other waves' issue-bound Keccak
// without a kernel boundary, a second stream or the k_xof_slow launch between them.  The query
// reads the scratch rows its own lane has just written.
template <bool FUSE, bool PULL = false>
__global__ __launch_bounds__(256, 3) void k_prep_h(DevParams p, InPtrs in, Scratch sc,
                                                   OutPtrs out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  xofd_body<FUSE, false, PULL>(p, in, sc, r);
  // two wires per sweep: 3 and 4 spill inside the wire loop
  query_h_body<2, 32>(p, in, sc, out, r);
}

// k_leader_prep<PP>: the leader's prepare_init of Prio3Histogram / SumVec in one launch, as
// k_prep_h is the helper's: leader_jr_body (the explicit share streamed once into the joint-rand
// sponge and the SoA scratch) and then query_h_body<2, PP, 1> on the scratch rows the same lane
// has just written, so one wave's memory-bound share streaming runs beside other waves' query.
// Flagged reports are deferred to k_leader_slowfix + a k_query_h redo launch.
template <int PP>
__global__ __launch_bounds__(256, 3) void k_leader_prep(DevParams p, InPtrs in, Scratch sc,
                                                        OutPtrs out, uint32_t* wpart,
                                                        uint32_t* wseg) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  leader_jr_body(p, in, sc, out.status, wpart, wseg, r);
  query_h_body<2, PP, 1>(p, in, sc, out, r);
}

// k_prep_sum<NPH>: the same for Prio3Sum (P = 16 NPH): the dual-state XOF and k_query_sum's body
// (prio3_query_sum.h) on the same wave, flagged reports deferred to the run's redo launch
template <int NPH>
__global__ __launch_bounds__(256, 3) void k_prep_sum(DevParams p, InPtrs in, Scratch sc,
                                                     OutPtrs out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  xofd_body<false, false>(p, in, sc, r);
  qsum::query_sum_body<NPH, 0>(p, in, sc, out, r);
}




// ------------------------------------------------------------------------------------
// Accumulate: masked segmented mod-p reduction of output shares
// ------------------------------------------------------------------------------------
// Per-report inclusion: a report counts in its segment if its status is FINISHED, the host mask
// is non-zero and its segment id is < n_segments.  A segment id past n_segments excludes the
// report from every aggregate and count, on every path (fused: k_agg_fix; metadata: k_meta).

// Segmented partial sums in one pass over the output shares.  grid: x = output element, y =
// report chunk, z = group of SG segments; each thread keeps SG running sums (one per segment of
// its group) and the block reduces them through LDS into partial[chunk][segment][element]
// (counts into pcount[chunk][segment] from the element-0 blocks).
// Inclusion is decided inline (status, segment id, accept mask; no separate code pass), so the
// accumulate is one launch plus k_acc_fin.
template <class F, int SG>
__global__ __launch_bounds__(256) void k_acc_seg(uint32_t n, size_t ld, uint32_t chunk,
                                                 uint32_t out_len, uint32_t nseg, const void* src,
                                                 const uint8_t* status, const uint32_t* seg,
                                                 const uint8_t* accept, void* partial,
                                                 uint64_t* pcount) {
  typedef typename F::T T;
  __shared__ T red[256];
  __shared__ uint32_t cred[256];
  const uint32_t e = blockIdx.x, c = blockIdx.y, s0 = blockIdx.z * SG;
  const uint32_t lo = c * chunk, hi = min(n, lo + chunk);
  T acc[SG];
  uint32_t cnt[SG];
#pragma unroll
  for (int q = 0; q < SG; q++) {
    acc[q] = F::zero();
    cnt[q] = 0;
  }
  for (uint32_t r = lo + threadIdx.x; r < hi; r += 256) {
    const uint32_t sr = seg ? seg[r] : 0u;
    const bool ok = status[r] == PRIO3_STATUS_FINISHED && sr < nseg && (!accept || accept[r]);
    const uint32_t k = (ok ? sr : 0xffffffffu) - s0;  // ~0 (excluded) wraps past SG
    if (k < (uint32_t)SG) {
      const T x = F::load(src, (size_t)e * ld + r);
#pragma unroll
      for (int q = 0; q < SG; q++)
        if ((uint32_t)q == k) {
          acc[q] = F::add(acc[q], x);
          cnt[q]++;
        }
    }
  }
#pragma unroll
  for (int q = 0; q < SG; q++) {
    if (s0 + q >= nseg) break;  // uniform
    red[threadIdx.x] = acc[q];
    cred[threadIdx.x] = cnt[q];
    __syncthreads();
    for (uint32_t st = 128; st > 0; st >>= 1) {
      if (threadIdx.x < st) {
        red[threadIdx.x] = F::add(red[threadIdx.x], red[threadIdx.x + st]);
        cred[threadIdx.x] += cred[threadIdx.x + st];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      F::store(partial, ((size_t)c * nseg + s0 + q) * out_len + e, red[0]);
      if (e == 0) pcount[(size_t)c * nseg + s0 + q] = cred[0];
    }
    __syncthreads();
  }
}

// grid (ceil(out_len / 256), nseg): per segment and element, the sum over the chunk partials
template <class F>
__global__ void k_acc_fin(uint32_t nchunks, uint32_t out_len, uint32_t nseg, const void* partial,
                          const uint64_t* pcount, uint8_t* agg, uint64_t* count) {
  typedef typename F::T T;
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x, s = blockIdx.y;
  if (e < out_len) {
    T acc = F::zero();
    for (uint32_t c = 0; c < nchunks; c++)
      acc = F::add(acc, F::load(partial, ((size_t)c * nseg + s) * out_len + e));
    F::store(agg, (size_t)s * out_len + e, acc);
  }
  if (e == 0) {
    uint64_t t = 0;
    for (uint32_t c = 0; c < nchunks; c++) t += pcount[(size_t)c * nseg + s];
    count[s] = t;
  }
}


// k_acc_fin for the short outputs (Count, Sum: 2048-report chunks, so hundreds of partials per
// element): grid (out_len, nseg), the block's threads stride over the chunks and reduce in LDS
template <class F>
__global__ __launch_bounds__(256) void k_acc_fin_blk(uint32_t nchunks, uint32_t out_len,
                                                     uint32_t nseg, const void* partial,
                                                     const uint64_t* pcount, uint8_t* agg,
                                                     uint64_t* count) {
  typedef typename F::T T;
  __shared__ T red[256];
  __shared__ uint64_t cred[256];
  const uint32_t e = blockIdx.x, s = blockIdx.y;
  T acc = F::zero();
  uint64_t t = 0;
  for (uint32_t c = threadIdx.x; c < nchunks; c += 256) {
    acc = F::add(acc, F::load(partial, ((size_t)c * nseg + s) * out_len + e));
    if (e == 0) t += pcount[(size_t)c * nseg + s];
  }
  red[threadIdx.x] = acc;
  cred[threadIdx.x] = t;
  __syncthreads();
  for (uint32_t st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      red[threadIdx.x] = F::add(red[threadIdx.x], red[threadIdx.x + st]);
      cred[threadIdx.x] += cred[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    F::store(agg, (size_t)s * out_len + e, red[0]);
    if (e == 0) count[s] = cred[0];
  }
}// Accumulate of many small batches in one launch (the accumulate executor: concurrent
// prio3_accumulate calls of Janus's aggregation jobs).  grid: x = output element, y = job; the
// block sums its element over the job's reports (inclusion as k_acc_seg) into up to 8 segments at
// a time and writes the job's aggregate share element and, from element 0, its counts.
template <class F>
__global__ __launch_bounds__(256) void k_acc_multi(const AccDesc* descs, uint8_t* base) {
  typedef typename F::T T;
  __shared__ T red[256];
  __shared__ uint32_t cred[256];
  const AccDesc d = descs[blockIdx.y];
  const uint32_t e = blockIdx.x;
  if (e >= d.out_len) return;  // uniform per block
  const uint32_t* seg = (d.flags & 1) ? (const uint32_t*)(base + d.seg_off) : nullptr;
  const uint8_t* acc = (d.flags & 2) ? base + d.acc_off : nullptr;
  for (uint32_t s0 = 0; s0 < d.nseg; s0 += 8) {
    T a[8];
    uint32_t c[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      a[q] = F::zero();
      c[q] = 0;
    }
    for (uint32_t r = threadIdx.x; r < d.n; r += 256) {
      const uint32_t s = seg ? seg[r] : 0u;
      const bool inc = d.status[r] == PRIO3_STATUS_FINISHED && s < d.nseg && (!acc || acc[r]);
      const uint32_t k = s - s0;
      if (inc && k < 8u) {
        const T x = F::load(d.src, (size_t)e * d.ld + r);
#pragma unroll
        for (int q = 0; q < 8; q++)
          if ((uint32_t)q == k) {
            a[q] = F::add(a[q], x);
            c[q]++;
          }
      }
    }
    const uint32_t ns = min(8u, d.nseg - s0);
    for (uint32_t q = 0; q < ns; q++) {
      T v = F::zero();
      uint32_t cv = 0;
#pragma unroll
      for (int q2 = 0; q2 < 8; q2++)
        if ((uint32_t)q2 == q) {
          v = a[q2];
          cv = c[q2];
        }
      red[threadIdx.x] = v;
      cred[threadIdx.x] = cv;
      __syncthreads();
      for (uint32_t st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) {
          red[threadIdx.x] = F::add(red[threadIdx.x], red[threadIdx.x + st]);
          cred[threadIdx.x] += cred[threadIdx.x + st];
        }
        __syncthreads();
      }
      if (threadIdx.x == 0) {
        F::store(base + d.agg_off, (size_t)(s0 + q) * d.out_len + e, red[0]);
        if (e == 0) ((uint64_t*)(base + d.cnt_off))[s0 + q] = cred[0];
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------------
// Fused accumulate, second half: combine the per-wave half-limb partials per segment,
// then fix up exclusions / non-fused reports and reduce mod p.
// ------------------------------------------------------------------------------------
// Level 1: grid (ceil(M*8/1024), chunks of WCH waves): thread = 4 consecutive slots (element,
// half), read as one 16-byte load per wave (4x the bytes in flight of a slot per thread: the
// 1-slot version moved the 134 MB of a 1 Mi batch's wave partials at 1.8 TB/s).  A chunk whose
// fused waves all carry one segment writes 64-bit chunk partials (cseg[chunk] = its segment); a
// chunk mixing segments adds each run with a 64-bit atomic into agg64 directly (cseg = ~0, as
// for a chunk with no fused wave).
constexpr uint32_t WCH = 32;
__global__ __launch_bounds__(256) void k_agg_waves(uint32_t nwaves, uint32_t M,
                                                   const uint32_t* wpart, const uint32_t* wseg,
                                                   unsigned long long* cpart, uint32_t* cseg,
                                                   unsigned long long* agg64) {
  static_assert(WCH <= 64, "one chunk's wave segments are read by one wave");
  const uint32_t slot = 4 * (blockIdx.x * blockDim.x + threadIdx.x), c = blockIdx.y;
  const uint32_t w0 = c * WCH, w1 = min(nwaves, w0 + WCH), lane = threadIdx.x & 63u;
  // the chunk's wave segments in one load per lane (not a dependent scalar load per wave):
  // bit i of `fused` = wave w0 + i was fused; s0 = the first fused wave's segment
  const uint32_t my = w0 + lane < w1 ? wseg[w0 + lane] : 0xffffffffu;
  const uint64_t fused = __ballot(my != 0xffffffffu);
  const uint32_t s0 = fused ? (uint32_t)__shfl((int)my, __ffsll((long long)fused) - 1) : 0xffffffffu;
  const bool mixed = __any(my != 0xffffffffu && my != s0);
  if (slot == 0 && blockIdx.x == 0) cseg[c] = mixed ? 0xffffffffu : s0;
  if (s0 == 0xffffffffu) return;  // wave-uniform: no fused wave in the chunk
  // Lanes past the last slot (M * 8 is a multiple of 4, not of 256) stay alive through the mixed
  // path's readlane of `my` below: their loads are clamped to slot 0 and their atomics masked.
  const bool act = slot < M * 8;
  const uint32_t ls = act ? slot : 0u;
  const size_t row = (size_t)M * 8;
  if (!mixed) {
    if (!act) return;
    // all WCH loads independent and unconditional (clamped to the last wave, masked by bit)
    unsigned long long a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
    for (uint32_t i = 0; i < WCH; i++) {
      const uint32_t w = min(w0 + i, w1 - 1);
      const uint4 v = *(const uint4*)(wpart + (size_t)w * row + slot);
      const uint32_t m = 0u - (uint32_t)((fused >> i) & 1u);
      a0 += v.x & m, a1 += v.y & m, a2 += v.z & m, a3 += v.w & m;
    }
    unsigned long long* o = cpart + (size_t)c * row + slot;
    o[0] = a0, o[1] = a1, o[2] = a2, o[3] = a3;
    return;
  }
  // segment runs inside the chunk (e.g. the executor's jobs of a few waves each): the loads in
  // batches of 8 waves, unconditional (clamped, masked), the run boundaries read from `my` by
  // shuffle (wave-uniform), one 64-bit atomic per run and slot
  unsigned long long a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  uint32_t cur = 0xffffffffu;
  auto flush = [&]() {
    if (cur == 0xffffffffu || !act) return;
    unsigned long long* o = agg64 + (size_t)cur * row + slot;
    if (a0) atomicAdd(o, a0);
    if (a1) atomicAdd(o + 1, a1);
    if (a2) atomicAdd(o + 2, a2);
    if (a3) atomicAdd(o + 3, a3);
  };
#pragma unroll 1
  for (uint32_t b = 0; b < WCH; b += 8) {
    uint4 v[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; j++)
      v[j] = *(const uint4*)(wpart + (size_t)min(w0 + b + j, w1 - 1) * row + ls);
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) {
      // every lane of the wave is still active here (no early return above), so reading lane
      // b + j of `my` is well defined; ~0 = absent or unfused
      const uint32_t sg = (uint32_t)__builtin_amdgcn_readlane((int)my, (int)(b + j));
      if (sg == 0xffffffffu) continue;
      if (sg != cur) {
        flush();
        cur = sg;
        a0 = a1 = a2 = a3 = 0;
      }
      a0 += v[j].x, a1 += v[j].y, a2 += v[j].z, a3 += v[j].w;
    }
  }
  flush();
}

// Counts the reports the aggregate must contain (status FINISHED and accepted by the host
// mask) per segment and lists every report whose fused inclusion differs (entry = r, or
// r | 0x80000000 when it must be subtracted).  A block covers FIX_R consecutive reports and
// keeps its counts in a small LDS table keyed by segment, flushed with one atomic per entry.
// per: reports per block (4096 for large runs; 512 for the executor's 20-60k-report groups,
// whose 4096-report blocks left most of the chip idle)
constexpr uint32_t FIX_T = 64;
static uint32_t fix_per(uint32_t n) { return n >= (1u << 18) ? 4096u : 512u; }
// oor_masked: the fused kernel masked lanes with an out-of-range segment id out of its wave
// partials (xofd_body); they are then not part of a fused wave's sum.  0: the wave partials
// include them (the fused leader unpack), so they are subtracted like any excluded report.
__global__ __launch_bounds__(256) void k_agg_fix(uint32_t n, const uint8_t* status,
                                                 const uint32_t* seg, const uint8_t* accept,
                                                 const uint32_t* wseg, uint32_t* fix,
                                                 uint32_t fix_cap, uint32_t nseg,
                                                 unsigned long long* counts, uint32_t oor_masked,
                                                 uint32_t per, uint32_t wshift) {
  __shared__ uint32_t tseg[FIX_T];
  __shared__ unsigned int tcnt[FIX_T];
  if (threadIdx.x < FIX_T) {
    tseg[threadIdx.x] = 0xffffffffu;
    tcnt[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint32_t lo = blockIdx.x * per, hi = min(n, lo + per);
  for (uint32_t base = lo; base < hi; base += 256) {
    const uint32_t r = base + threadIdx.x;
    const bool valid = r < hi;
    const uint32_t sg = valid ? (seg ? seg[r] : 0u) : 0xffffffffu;
    // out-of-range segment ids are excluded everywhere (as k_mask and k_meta do)
    const bool inc = valid && sg < nseg && status[r] == PRIO3_STATUS_FINISHED &&
                     (!accept || accept[r]);
    const bool fused = valid && wseg[r >> wshift] != 0xffffffffu && (!oor_masked || sg < nseg);
    const uint32_t s0 = (uint32_t)__shfl((int)sg, 0);
    const bool uni = __all(!valid || sg == s0);
    const unsigned long long b = __ballot(inc);
    auto add = [&](uint32_t s, unsigned int k) {
      const uint32_t h = s % FIX_T;
      const uint32_t old = atomicCAS(&tseg[h], 0xffffffffu, s);
      if (old == 0xffffffffu || old == s) atomicAdd(&tcnt[h], k);
      else atomicAdd(&counts[s], (unsigned long long)k);  // table collision
    };
    if (uni) {
      if ((threadIdx.x & 63u) == 0 && b) add(s0, (unsigned int)__popcll(b));
    } else if (inc) {
      add(sg, 1u);
    }
    if (valid && fused != inc) {
      const uint32_t i = atomicAdd(&fix[0], 1u);
      if (i < fix_cap) fix[1 + i] = r | (inc ? 0u : 0x80000000u);
    }
  }
  __syncthreads();
  if (threadIdx.x < FIX_T && tseg[threadIdx.x] != 0xffffffffu && tcnt[threadIdx.x])
    atomicAdd(&counts[tseg[threadIdx.x]], (unsigned long long)tcnt[threadIdx.x]);
}

DEV f128 fold_halves_impl(const unsigned long long (&Hs)[8]);
DEV f128 fold_halves(const unsigned long long (&Hs)[8]) { return fold_halves_impl(Hs); }

// One block per (segment, element): thread (half h = tid & 7, lane cl = tid >> 3) sums the chunk
// partials of its segment for chunks cl, cl+32, ...; then the fix-up list is applied by all
// 256 threads (lazily reduced signed sums), reduced through LDS, and thread 0 folds the
// half-limb totals X = sum_h H_h 2^(16h) (H_h < 2^48) mod p.
__global__ __launch_bounds__(256) void k_agg_final(uint32_t M, size_t ld,
                                                   const unsigned long long* agg64,
                                                   uint32_t nchunks,
                                                   const unsigned long long* cpart,
                                                   const uint32_t* cseg, const uint32_t* fix,
                                                   const uint32_t* seg, const void* meas,
                                                   uint8_t* agg) {
  const uint32_t idx = blockIdx.x, s = idx / M, e = idx % M;
  const uint32_t tid = threadIdx.x, h = tid & 7u, cl = tid >> 3;
  __shared__ unsigned long long red[256];
  __shared__ f128 fadd[256], fsub[256];
  unsigned long long acc = 0;
  for (uint32_t c = cl; c < nchunks; c += 32)
    if (cseg[c] == s) acc += cpart[((size_t)c * M + e) * 8 + h];
  red[tid] = acc;
  // fix-up entries, strided over the block
  f128 ad = zero128(), sb = zero128();
  const uint32_t nfix = fix[0];
  for (uint32_t i = tid; i < nfix; i += 256) {
    const uint32_t ent = fix[1 + i], r = ent & 0x7fffffffu;
    if ((seg ? seg[r] : 0u) != s) continue;
    const f128 x = Fp128::load(meas, (size_t)e * ld + r);
    if (ent & 0x80000000u) sb = add128(sb, x);
    else ad = add128(ad, x);
  }
  fadd[tid] = ad;
  fsub[tid] = sb;
  __syncthreads();
  for (uint32_t st = 128; st >= 8; st >>= 1) {
    if (tid < st) red[tid] += red[tid + st];
    __syncthreads();
  }
  for (uint32_t st = 128; st >= 1; st >>= 1) {
    if (tid < st) {
      fadd[tid] = add128(fadd[tid], fadd[tid + st]);
      fsub[tid] = add128(fsub[tid], fsub[tid + st]);
    }
    __syncthreads();
  }
  if (tid != 0) return;
  unsigned long long Hs[8];
  for (int hh = 0; hh < 8; hh++) Hs[hh] = red[hh] + agg64[(size_t)idx * 8 + hh];
  Fp128::store(agg, idx, sub128(add128(fold_halves(Hs), fadd[0]), fsub[0]));
}

// Runs with few chunks and many segments (the executor's groups: one segment per job, 2-8 waves
// each): one block per (segment, 32 elements), thread (element tid / 8, half h = tid % 8), so a
// block does not reduce 256 threads through LDS for one element; the fix-up list (empty when
// every wave fused) is split over the 8 halves and summed by shuffles.
__global__ __launch_bounds__(256) void k_agg_final_s(uint32_t M, size_t ld,
                                                     const unsigned long long* agg64,
                                                     uint32_t nchunks,
                                                     const unsigned long long* cpart,
                                                     const uint32_t* cseg, const uint32_t* fix,
                                                     const uint32_t* seg, const void* meas,
                                                     uint8_t* agg) {
  const uint32_t s = blockIdx.y, tid = threadIdx.x, h = tid & 7u, lane = tid & 63u;
  const uint32_t e = blockIdx.x * 32u + (tid >> 3);
  const bool live = e < M;
  const uint32_t ec = live ? e : 0u;
  unsigned long long H = agg64[((size_t)s * M + ec) * 8 + h];
  for (uint32_t c = 0; c < nchunks; c++)
    if (cseg[c] == s) H += cpart[((size_t)c * M + ec) * 8 + h];
  f128 ad = zero128(), sb = zero128();
  const uint32_t nfix = fix[0];
  for (uint32_t i = h; i < nfix; i += 8) {
    const uint32_t ent = fix[1 + i], r = ent & 0x7fffffffu;
    if ((seg ? seg[r] : 0u) != s) continue;
    const f128 x = Fp128::load(meas, (size_t)ec * ld + r);
    if (ent & 0x80000000u) sb = add128(sb, x);
    else ad = add128(ad, x);
  }
  if (nfix) {  // block-uniform
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
      f128 xa, xs;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        xa.w[k] = (uint32_t)__shfl_xor((int)ad.w[k], m);
        xs.w[k] = (uint32_t)__shfl_xor((int)sb.w[k], m);
      }
      ad = add128(ad, xa);
      sb = add128(sb, xs);
    }
  }
  unsigned long long Hs[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int src = (int)((lane & ~7u) + (uint32_t)k);
    Hs[k] = ((unsigned long long)(uint32_t)__shfl((int)(uint32_t)(H >> 32), src) << 32) |
            (uint32_t)__shfl((int)(uint32_t)H, src);
  }
  if (h != 0 || !live) return;
  Fp128::store(agg, (size_t)s * M + e, sub128(add128(fold_halves(Hs), ad), sb));
}

// X = sum_h H_h 2^(16h) (H_h < 2^48) mod p
DEV f128 fold_halves_impl(const unsigned long long (&Hs)[8]) {
  uint32_t w[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int hh = 0; hh < 8; hh++) {
    const unsigned long long H = Hs[hh];
    const int sh = 16 * hh, wi = sh >> 5, bi = sh & 31;
    const unsigned long long lo = bi ? (H << 16) & 0xffffffffull : H & 0xffffffffull;
    const unsigned long long mid = bi ? (H >> 16) & 0xffffffffull : H >> 32;
    const unsigned long long hi = bi ? H >> 48 : 0ull;
    unsigned long long c = (unsigned long long)w[wi] + lo;
    w[wi] = (uint32_t)c;
    c = (unsigned long long)w[wi + 1] + mid + (c >> 32);
    w[wi + 1] = (uint32_t)c;
    c = (unsigned long long)w[wi + 2] + hi + (c >> 32);
    w[wi + 2] = (uint32_t)c;
    for (int k = wi + 3; k < 9 && (c >> 32); k++) {
      c = (unsigned long long)w[k] + (c >> 32);
      w[k] = (uint32_t)c;
    }
  }
  return red288(w, w[8]);
}

// sum of k partial aggregates (multi-GPU combine)
template <class F>
__global__ void k_combine(uint32_t k, uint32_t len, uint32_t n_segments, const uint8_t* in,
                          const uint64_t* cin, uint8_t* out, uint64_t* cout) {
  typedef typename F::T T;
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < len) {
    T acc = F::zero();
    for (uint32_t i = 0; i < k; i++) acc = F::add(acc, F::load(in, (size_t)i * len + e));
    F::store(out, e, acc);
  }
  if (e < n_segments) {
    uint64_t s = 0;
    for (uint32_t i = 0; i < k; i++) s += cin[(size_t)i * n_segments + e];
    cout[e] = s;
  }
}

// ------------------------------------------------------------------------------------
// Batch metadata of the per-segment BatchAggregation: besides the
// aggregate share and the count, every finished report XORs SHA-256(report_id) into the
// segment's ReportIdChecksum (core/src/report_id.rs:18-42, called from
// aggregation_job_writer.rs:650-656) and every report aggregation of the segment widens its
// client-timestamp interval (Interval::from_time + merge, core/src/time.rs:294-317; merged for
// failed reports too, aggregation_job_writer.rs:643-647).
// One report per lane: one SHA-256 compression of the padded 16-byte ID, then a block-level
// XOR / min / max reduction when a tile's 1024 reports share a segment (the common case:
// contiguous batches) and per-report atomics on the segment otherwise.
// ------------------------------------------------------------------------------------
// SHA-256 of the 16 bytes id[0..3] (little-endian words as loaded); the digest is returned as
// 8 little-endian words of its byte string (so a byte-wise XOR is a word-wise XOR).
DEV void sha256_id16(const uint32_t id[4], uint32_t out[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = __builtin_bswap32(id[i]);
  w[4] = 0x80000000u;
#pragma unroll
  for (int i = 5; i < 15; i++) w[i] = 0;
  w[15] = 128;  // message length in bits
  uint32_t st[8];
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = sha256d::IV[i];
  sha256d::compress(st, w);
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = __builtin_bswap32(st[i]);
}

// checksums[s][8 words] = 0, intervals[s] = (UINT64_MAX, 0) as a (min start, max end) pair
__global__ void k_meta_init(uint32_t n_segments, uint32_t* ck, unsigned long long* iv) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_segments) return;
  if (ck)
    for (int i = 0; i < 8; i++) ck[8 * s + i] = 0;
  if (iv) {
    iv[2 * s] = ~0ull;
    iv[2 * s + 1] = 0;
  }
}

// Grid-stride over tiles of 1024 reports (16 waves): a tile whose reports share one segment is
// reduced in the block and folded into the block's running (segment, XOR, min, max) registers,
// which go out with one atomic per word when the segment changes and at the end -- so a 1 Mi
// batch of one segment issues ~5 k atomics on the segment's 10 words instead of ~41 k from
// 256-report blocks, whose serialisation on those addresses had set the kernel's time (112 us).
constexpr uint32_t META_T = 1024, META_W = META_T / 64, META_BLOCKS = 512;
__global__ __launch_bounds__(1024) void k_meta(uint32_t n, const uint8_t* ids, const uint64_t* times,
                                             const uint8_t* status, const uint8_t* mask,
                                             const uint32_t* seg, uint32_t n_segments, uint32_t* ck,
                                             unsigned long long* iv) {
  __shared__ uint32_t s_seg0;
  __shared__ uint32_t s_ck[META_W][8];
  __shared__ unsigned long long s_lo[META_W], s_hi[META_W];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  // the block's running partial (block-uniform `cur`; word tid on threads 0..7, the interval on
  // thread 8)
  uint32_t cur = 0xffffffffu, acc_x = 0;
  unsigned long long acc_lo = ~0ull, acc_hi = 0;
  auto flush = [&]() {
    if (cur != 0xffffffffu) {
      if (ck && tid < 8 && acc_x) atomicXor(ck + 8 * cur + tid, acc_x);
      if (iv && tid == 8 && acc_hi) {
        atomicMin(iv + 2 * cur, acc_lo);
        atomicMax(iv + 2 * cur + 1, acc_hi);
      }
    }
    acc_x = 0;
    acc_lo = ~0ull;
    acc_hi = 0;
  };
  for (uint32_t base = blockIdx.x * META_T; base < n; base += gridDim.x * META_T) {
    const uint32_t r = base + tid;
    const bool valid = r < n;
    const uint32_t sg = valid ? (seg ? seg[r] : 0u) : 0xffffffffu;
    const bool in_range = valid && sg < n_segments;
    const bool inc = in_range && status[r] == PRIO3_STATUS_FINISHED && (!mask || mask[r]);
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ck && inc) {
      uint32_t id[4];
      load16(ids + 16 * (size_t)r, id);
      sha256_id16(id, h);
    }
    unsigned long long lo = ~0ull, hi = 0;
    if (times && in_range) {
      lo = times[r];
      hi = lo + 1;  // Interval::from_time: [t, t + 1)
    }
    if (tid == 0) s_seg0 = sg;  // thread 0 of a tile is always a valid report
    __syncthreads();
    const bool uniform = __syncthreads_and(!valid || sg == s_seg0) && s_seg0 < n_segments;
    if (uniform) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
        for (int i = 0; i < 8; i++) h[i] ^= (uint32_t)__shfl_xor((int)h[i], off);
        const unsigned long long l2 = __shfl_xor(lo, off), h2 = __shfl_xor(hi, off);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
      }
      if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) s_ck[wv][i] = h[i];
        s_lo[wv] = lo;
        s_hi[wv] = hi;
      }
      __syncthreads();
      if (s_seg0 != cur) {  // block-uniform
        flush();
        cur = s_seg0;
      }
      if (tid < 8) {
        uint32_t x = 0;
        for (uint32_t q = 0; q < META_W; q++) x ^= s_ck[q][tid];
        acc_x ^= x;
      }
      if (tid == 8) {
        for (uint32_t q = 0; q < META_W; q++) {
          acc_lo = s_lo[q] < acc_lo ? s_lo[q] : acc_lo;
          acc_hi = s_hi[q] > acc_hi ? s_hi[q] : acc_hi;
        }
      }
    } else {
      if (ck && inc)
#pragma unroll
        for (int i = 0; i < 8; i++) atomicXor(ck + 8 * sg + i, h[i]);
      if (iv && times && in_range) {
        atomicMin(iv + 2 * sg, lo);
        atomicMax(iv + 2 * sg + 1, hi);
      }
    }
    __syncthreads();  // s_seg0 / s_ck of this tile are read before the next tile writes them
  }
  flush();
}

// multi-GPU combine of k per-rank metadata: checksums XOR, intervals Interval::merge
// (an empty (.., 0) interval is the identity, core/src/time.rs:294-307)
__global__ void k_combine_meta(uint32_t k, uint32_t n_segments, const uint32_t* ck_in,
                               const unsigned long long* iv_in, uint32_t* ck_out,
                               unsigned long long* iv_out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_segments * 8) return;
  const uint32_t s = t >> 3, w = t & 7u;
  if (ck_in && ck_out) {
    uint32_t x = 0;
    for (uint32_t i = 0; i < k; i++) x ^= ck_in[((size_t)i * n_segments + s) * 8 + w];
    ck_out[(size_t)s * 8 + w] = x;
  }
  if (iv_in && iv_out && w == 0) {
    unsigned long long lo = ~0ull, hi = 0;
    for (uint32_t i = 0; i < k; i++) {
      const unsigned long long a = iv_in[((size_t)i * n_segments + s) * 2];
      const unsigned long long d = iv_in[((size_t)i * n_segments + s) * 2 + 1];
      if (d == 0) continue;
      lo = a < lo ? a : lo;
      hi = a + d > hi ? a + d : hi;
    }
    iv_out[2 * s] = hi ? lo : 0;
    iv_out[2 * s + 1] = hi ? hi - lo : 0;
  }
}

// (min start, max end) -> (start, duration); a segment with no report -> Interval::EMPTY (0, 0)
__global__ void k_meta_final(uint32_t n_segments, unsigned long long* iv) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_segments) return;
  const unsigned long long lo = iv[2 * s], hi = iv[2 * s + 1];
  iv[2 * s] = hi ? lo : 0;
  iv[2 * s + 1] = hi ? hi - lo : 0;
}


// ------------------------------------------------------------------------------------
// Field self-test (parity of the hand-scheduled Field128 blocks against Python bigints)
// ------------------------------------------------------------------------------------
// op 0: mul128 (compiler code), 1: mul128_asm, 2: add128, 3: sub128,
// op 4: sum_{i<16} a_(16x+i) b_(16x+i) via mac_add + mac_reduce (compiler code),
// op 5: the same with mac_reduce_asm.   a, b, out: [n][16 B] (ops 4/5: a, b [16 n][16 B]).
__global__ void k_selftest_f128(int op, uint32_t n, const uint4* a, const uint4* b, uint4* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  auto ld = [](const uint4* p, size_t k) {
    const uint4 v = p[k];
    return mk128(v.x, v.y, v.z, v.w);
  };
  f128 z;
  if (op == 0) z = mul128(ld(a, i), ld(b, i));
  else if (op == 1) z = mul128_asm(ld(a, i), ld(b, i));
  else if (op == 2) z = add128(ld(a, i), ld(b, i));
  else if (op == 3) z = sub128(ld(a, i), ld(b, i));
  else {
    mac128 m;
    mac_zero(m);
    for (int k = 0; k < 16; k++) mac_add(m, ld(a, (size_t)i * 16 + k), ld(b, (size_t)i * 16 + k));
    z = op == 4 ? mac_reduce(m) : mac_reduce_asm(m);
  }
  out[i] = make_uint4(z.w[0], z.w[1], z.w[2], z.w[3]);
}

// ====================================================================================
// Host side
// ====================================================================================


// ====================================================================================
// Host side
// ====================================================================================

// A batch handle: one job's column range of a (possibly coalesced, shared) device run.  Every
// handle owns its reference, so concurrent jobs of one engine never see each other's output
// shares or verdicts (the run's slab stays out of the pool until the last handle is freed).
// Handles must be freed before their engine is destroyed.
struct prio3_batch {
  prio3_engine* e;
  Run* run;  // nullptr for an empty batch
  uint32_t c0, n;
};

static uint32_t next_pow2(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

// prio flp/gadgets.rs optimal_chunk_length: over calls = 2^k - 1, the chunk length minimising
// the ParallelSum proof length 2 * chunk + 2 * ((1 + calls).next_power_of_two() - 1) + 1
// (first minimum from the largest k, as min_by_key over the reversed range keeps)
static uint32_t optimal_chunk_length(uint32_t m) {
  if (m <= 1) return 1;
  uint32_t max_log2 = 0;
  while ((1u << max_log2) < m) max_log2++;
  max_log2 += 1;
  uint64_t best = UINT64_MAX;
  uint32_t best_chunk = 1;
  for (uint32_t l = max_log2; l >= 1; l--) {
    const uint64_t calls = (1ull << l) - 1, chunk = (m + calls - 1) / calls;
    const uint64_t cost = 2 * chunk + 2 * ((1ull << l) - 1) + 1;  // next_pow2(1 + calls) = 2^l
    if (cost < best) {
      best = cost;
      best_chunk = (uint32_t)chunk;
    }
  }
  return best_chunk;
}

static int fill_sizes(const prio3_params* pp, prio3_sizes_t* s, DevParams* dp) {
  if (!pp) return PRIO3_EINVAL;
  uint32_t proofs = pp->num_proofs ? pp->num_proofs : 1;
  const bool mp = pp->kind == PRIO3_SUMVEC_F64_MP;
  if (mp ? (proofs < 2 || proofs > 8) : proofs != 1) return mp ? PRIO3_EINVAL : PRIO3_EUNSUPPORTED;
  DevParams d;
  memset(&d, 0, sizeof d);
  d.kind = pp->kind;
  d.bits = pp->bits;
  d.length = pp->length;
  d.chunk = pp->chunk_length;
  uint32_t algo;
  switch (pp->kind) {
    case PRIO3_COUNT:
      algo = 0;
      d.es = 8;
      d.meas_len = 1;
      d.out_len = 1;
      d.jr_len = 0;
      d.arity = 2;
      d.calls = 1;
      break;
    case PRIO3_SUM:
      if (pp->bits == 0 || pp->bits > 64) return PRIO3_EINVAL;
      algo = 1;
      d.es = 16;
      d.meas_len = pp->bits;
      d.out_len = 1;
      d.jr_len = 1;
      d.arity = 1;
      d.calls = pp->bits;
      break;
    case PRIO3_SUMVEC:
      if (pp->bits == 0 || pp->bits > 64 || pp->length == 0 || pp->chunk_length == 0)
        return PRIO3_EINVAL;
      algo = 2;
      d.es = 16;
      d.meas_len = pp->bits * pp->length;
      d.out_len = pp->length;
      d.jr_len = 1;
      d.arity = 2 * pp->chunk_length;
      d.calls = (d.meas_len + pp->chunk_length - 1) / pp->chunk_length;
      break;
    case PRIO3_SUMVEC_F64_MP:  // SumVec<Field64, ParallelSum<Mul>> (vdaf.rs:173-195)
      if (pp->bits == 0 || pp->bits > 64 || pp->length == 0 || pp->chunk_length == 0)
        return PRIO3_EINVAL;
      algo = 0xFFFF1003u;  // ALGORITHM_ID_PRIO3_SUM_VEC_FIELD64_MULTIPROOF_HMACSHA256_AES128
      d.es = 8;
      d.meas_len = pp->bits * pp->length;
      d.out_len = pp->length;
      d.jr_len = 1;
      d.arity = 2 * pp->chunk_length;
      d.calls = (d.meas_len + pp->chunk_length - 1) / pp->chunk_length;
      break;
    case PRIO3_FPVEC_BOUNDED_L2:  // Prio3FixedPointBoundedL2VecSum (vdaf.rs:292-335)
      if ((pp->bits != 16 && pp->bits != 32) || pp->length == 0 || pp->length > (1u << 22))
        return PRIO3_EINVAL;
      algo = 0xFFFF0000u;
      d.es = 16;
      d.meas_len = pp->bits * pp->length + 2 * pp->bits - 2;
      d.out_len = pp->length;
      d.jr_len = 2;
      d.qr_len = 2;
      d.chunk = optimal_chunk_length(d.meas_len);
      d.arity = 2 * d.chunk;
      d.calls = (d.meas_len + d.chunk - 1) / d.chunk;
      d.chunk1 = optimal_chunk_length(pp->length);
      d.calls1 = (pp->length + d.chunk1 - 1) / d.chunk1;
      break;
    case PRIO3_HISTOGRAM:
      if (pp->length == 0 || pp->chunk_length == 0) return PRIO3_EINVAL;
      algo = 3;
      d.es = 16;
      d.meas_len = pp->length;
      d.out_len = pp->length;
      d.jr_len = 2;
      d.arity = 2 * pp->chunk_length;
      d.calls = (pp->length + pp->chunk_length - 1) / pp->chunk_length;
      break;
    default:
      return PRIO3_EINVAL;
  }
  d.P = next_pow2(1 + d.calls);
  d.logP = 0;
  while ((1u << d.logP) < d.P) d.logP++;
  if (d.logP > MAX_ROOTS) return PRIO3_EUNSUPPORTED;
  d.glen = 2 * (d.P - 1) + 1;
  d.proof_len = d.arity + d.glen;
  d.verifier_len = d.arity + 2;
  if (!d.qr_len) d.qr_len = 1;
  if (d.kind == PRIO3_FPVEC_BOUNDED_L2) {  // second gadget: seeds1 || coeffs1 follow
    d.P1 = next_pow2(1 + d.calls1);
    while ((1u << d.logP1) < d.P1) d.logP1++;
    if (d.logP1 > MAX_ROOTS) return PRIO3_EUNSUPPORTED;
    d.glen1 = 2 * (d.P1 - 1) + 1;
    d.proof_len += d.chunk1 + d.glen1;
    d.verifier_len = 1 + d.arity + 1 + d.chunk1 + 1;
  }
  const uint32_t S = mp ? 32 : 16;  // seed size
  d.helper_share_len = d.jr_len ? 3 * S : 2 * S;
  d.public_share_len = d.jr_len ? 2 * S : 0;
  d.prep_share_len = d.verifier_len * proofs * d.es + (d.jr_len ? S : 0);
  d.leader_share_len = (d.meas_len + d.proof_len * proofs) * d.es + (d.jr_len ? S : 0);
  for (uint32_t u = 1; u <= 7; u++) {
    uint8_t b[8] = {8, 0, (uint8_t)(algo >> 24), (uint8_t)(algo >> 16), (uint8_t)(algo >> 8),
                    (uint8_t)algo, 0, (uint8_t)u};
    memcpy(d.dst[u], b, 8);
  }
  // roots and constants
  {
    u128 g128 = 0;
    for (const char* c = "145091266659756586618791329697897684742"; *c; c++)
      g128 = g128 * 10 + (u128)(*c - '0');
    uint64_t g64 = 1753635133440165772ULL;
    for (int l = 0; l <= MAX_ROOTS; l++) {
      u128 r = g128;
      for (int i = 0; i < 66 - l; i++) r = hmul(r, r, HP128);
      for (int k = 0; k < 4; k++) d.roots128[l][k] = (uint32_t)(r >> (32 * k));
      u128 r64 = g64;
      for (int i = 0; i < 32 - l; i++) r64 = hmul(r64, r64, HP64);
      d.roots64[l] = (uint64_t)r64;
    }
    u128 ip = hpow(d.P, HP128 - 2, HP128), h = hpow(2, HP128 - 2, HP128);
    for (int k = 0; k < 4; k++) {
      d.invP128[k] = (uint32_t)(ip >> (32 * k));
      d.half128[k] = (uint32_t)(h >> (32 * k));
    }
    d.invP64 = (uint64_t)hpow(d.P, HP64 - 2, HP64);
    if (d.kind == PRIO3_FPVEC_BOUNDED_L2) {
      const u128 ip1 = hpow(d.P1, HP128 - 2, HP128);
      // entries * 2^(2n-2) / num_shares (2): < 2^22 * 2^62 / 2 < p
      const u128 nc = ((u128)d.out_len << (2 * d.bits - 2)) >> 1;
      const u128 tn = (u128)1 << d.bits;
      for (int k = 0; k < 4; k++) {
        d.invP1_128[k] = (uint32_t)(ip1 >> (32 * k));
        d.normc128[k] = (uint32_t)(nc >> (32 * k));
        d.twon128[k] = (uint32_t)(tn >> (32 * k));
      }
    }
    if (d.P <= 32) {
      u128 alpha = 0;
      for (int k = 0; k < 4; k++) alpha |= (u128)d.roots128[d.logP][k] << (32 * k);
      for (uint32_t e2 = 0; e2 < d.P; e2++) {
        u128 ae = hpow(alpha, e2, HP128), s = 0, x = 1;
        for (uint32_t cc = 1; cc <= d.calls; cc++) {
          x = hmul(x, ae, HP128);
          s += x;
          if (s < x || s >= HP128) s -= HP128;
        }
        for (int k = 0; k < 4; k++) d.sigma128[e2][k] = (uint32_t)(s >> (32 * k));
      }
      for (uint32_t i = 0; i < d.P / 2; i++) {
        u128 w = hpow(alpha, i, HP128);
        for (int k = 0; k < 4; k++) d.tw128[i][k] = (uint32_t)(w >> (32 * k));
      }
    } else if (d.P == 64 || d.P == 128) {  // k_query_w's four-step DFT
      u128 alpha = 0;
      for (int k = 0; k < 4; k++) alpha |= (u128)d.roots128[d.logP][k] << (32 * k);
      const u128 aq = hpow(alpha, 8, HP128);  // alpha_(P/8)
      for (uint32_t i = 0; i < d.P / 16; i++) {
        const u128 w = hpow(aq, i, HP128);
        for (int k = 0; k < 4; k++) d.tw128[i][k] = (uint32_t)(w >> (32 * k));
      }
      for (uint32_t i = 0; i < 8; i++) {
        const u128 w = hpow(alpha, i, HP128);
        for (int k = 0; k < 4; k++) d.tw128[8 + i][k] = (uint32_t)(w >> (32 * k));
      }
    }
    if (d.P >= 16 && d.P <= 128) {  // k_query_sum's twiddles
      u128 alpha = 0;
      for (int k = 0; k < 4; k++) alpha |= (u128)d.roots128[d.logP][k] << (32 * k);
      const u128 w16 = hpow(alpha, d.P / 16, HP128), a16 = hpow(alpha, 16, HP128);
      for (uint32_t i = 0; i < 8; i++) {
        const u128 v[3] = {hpow(w16, i, HP128), hpow(alpha, i, HP128), hpow(a16, i, HP128)};
        for (int t = 0; t < 3; t++)
          for (int k = 0; k < 4; k++) d.tws[8 * t + i][k] = (uint32_t)(v[t] >> (32 * k));
      }
    }
    d.half64 = (uint64_t)hpow(2, HP64 - 2, HP64);
  }
  if (s) {
    s->field_bytes = d.es;
    s->meas_len = d.meas_len;
    s->out_len = d.out_len;
    s->proof_len = d.proof_len;
    s->verifier_len = d.verifier_len;
    s->joint_rand_len = d.jr_len;
    s->nonce_len = 16;
    s->public_share_len = d.public_share_len;
    s->helper_share_len = d.helper_share_len;
    s->prep_share_len = d.prep_share_len;
    s->prep_msg_len = d.jr_len ? S : 0;
    s->agg_share_len = d.out_len * d.es;
    s->leader_input_share_len = d.leader_share_len;
  }
  d.proof_len *= proofs;  // scratch holds every proof (prio3_sizes_t reports one)
  if (dp) *dp = d;
  return PRIO3_OK;
}

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t _e = (x);                                                            \
    if (_e != hipSuccess) {                                                         \
      fprintf(stderr, "janus_prio3: HIP error %s at %s:%d\n", hipGetErrorString(_e), \
              __FILE__, __LINE__);                                                  \
      return PRIO3_EDEVICE;                                                         \
    }                                                                               \
  } while (0)


// ---- per-kernel timing (option "timing"): HIP events on the launch stream ----
struct Pending {
  prio3_engine* e;
  size_t idx;
  hipEvent_t a, b;
};
static std::vector<Pending>& pending() {
  static thread_local std::vector<Pending> v;
  return v;
}
static size_t time_slot(prio3_engine* e, const char* name) {
  std::lock_guard<std::mutex> lk(e->tmu);
  for (size_t i = 0; i < e->times.size(); i++)
    if (e->times[i].name == name) return i;
  e->times.push_back(KTime{name, 0, 0});
  return e->times.size() - 1;
}
// timing 2: launches are counted only (no events: the host-buffer executor's launch path stays
// as in production, bench.py --role jobs)
static void count_launch(prio3_engine* e, const char* name) {
  const size_t i = time_slot(e, name);
  std::lock_guard<std::mutex> lk(e->tmu);
  e->times[i].launches += 1;
}
#define TIMED(e, st, name, launch)                                   \
  do {                                                               \
    hipEvent_t _a = nullptr, _b = nullptr;                           \
    const bool _t = (e)->timing == 1 && hipEventCreate(&_a) == hipSuccess && \
                    hipEventCreate(&_b) == hipSuccess;               \
    if (_t) (void)hipEventRecord(_a, st);                            \
    launch;                                                          \
    HIPCHK(hipGetLastError());                                       \
    if (_t) {                                                        \
      (void)hipEventRecord(_b, st);                                  \
      pending().push_back(Pending{(e), time_slot(e, name), _a, _b}); \
    } else if ((e)->timing == 2) {                                   \
      count_launch((e), name);                                       \
    }                                                                \
  } while (0)

// folds this thread's finished timing events of engine e into e->times.  wait = false (the
// executor's group finish): events still pending -- those of the group issued ahead behind the
// finishing one -- are left for a later call instead of blocking the launcher on them
static void collect_times(prio3_engine* e, bool wait = true) {
  auto& v = pending();
  std::vector<Pending> keep;
  for (auto& pd : v) {
    if (pd.e != e || (!wait && hipEventQuery(pd.b) == hipErrorNotReady)) {
      keep.push_back(pd);
      continue;
    }
    float ms = 0;
    (void)hipEventSynchronize(pd.b);
    (void)hipEventElapsedTime(&ms, pd.a, pd.b);
    {
      std::lock_guard<std::mutex> lk(e->tmu);
      e->times[pd.idx].ms += ms;
      e->times[pd.idx].launches += 1;
    }
    (void)hipEventDestroy(pd.a);
    (void)hipEventDestroy(pd.b);
  }
  v.swap(keep);
}

// ---- runs: the device state of one prepare call, carved from one pooled slab ----
enum : unsigned {
  RUN_SCRATCH = 1,  // SoA prepare scratch
  RUN_IO = 2,       // device copies of host inputs / outputs (host-buffer entry points)
  RUN_VK = 4,       // per-report verify-key slots + key table (coalesced launches)
  RUN_LINPUT = 8,   // leader input shares (host-buffer leader entry point)
  RUN_FUSED = 16,   // fused-accumulate partials (prio3_device_prepare_aggregate, Histogram)
  RUN_AGG_IO = 32,  // group segment ids, accept bytes, aggregate shares + counts (executor)
  RUN_HPKE = 64,    // open statuses + plaintext scratch of a sealed-input group (executor)
};

// FPVec per-report scratch bytes of one sub-batch column: every buffer indexed [row][column]
// with the sub-batch leading dimension ld (meas, proofs, jr, qr, part, corrected, flag, L, PV,
// beta); the output shares have one column per report of the batch (ld_out).
static size_t fp_column_bytes(const DevParams& d) {
  const size_t es = d.es;
  return es * ((size_t)d.meas_len + d.proof_len + d.jr_len + d.qr_len + 2 * ((size_t)d.P + d.P1) +
               d.calls) +
         16 + 16 + 1;
}

// FPVec sub-batch width: the per-report scratch (2.6 MB at 10^4 entries) of a whole batch does
// not fit, so the batch runs in equal sub-batches of ld columns.  Auto budget: free HBM plus the
// pool's idle slabs, minus the batch's output shares and a fixed reserve for the runtime
// (private segments, queues, the caller's allocator) -- the r01u hipErrorIllegalAddress came
// with a budget of 85% of free HBM and did not recur with an explicit reserve.
// The kernels are latency-bound per lane, so the widest sub-batch wins.
// FPVec sub-batch sizes for n reports in scratch of cap columns: nsub equal sub-batches (columns
// rounded to 256), except that under the eight-lane query (k_query_fpw, two waves per SIMD, eight
// reports per wave) the first nsub - 1 are rounded down to whole query rounds -- n_cu x 4 SIMDs x
// 2 waves x 8 reports (16,384 on MI355X) -- when the last still fits the scratch (option
// fp_round).  The query's waves all take the same time, so a sub-batch of 3.05 rounds takes 4:
// 2 x 50,000 run 8 rounds, 49,152 + 50,848 run 7, while the XOF of either size keeps at most two
// waves per SIMD.
static void fp_sub_sizes(const prio3_engine* e, uint32_t n, uint32_t cap, bool wide,
                         uint32_t& nsub, uint32_t& sub) {
  nsub = (n + cap - 1) / cap;
  sub = std::min(cap, (((n + nsub - 1) / nsub) + 255) & ~255u);
  if (wide && e->fp_round && nsub > 1) {
    const uint32_t Q = (uint32_t)e->n_cu * 4u * 2u * 8u;
    const uint32_t s2 = sub / Q * Q;
    if (s2 > 0 && n - (nsub - 1) * s2 <= cap) sub = s2;
  }
}

static uint32_t fp_sub_ld(const prio3_engine* e, const DevParams& d, uint32_t ld_out,
                          size_t other_bytes) {
  const size_t per = fp_column_bytes(d);
  int64_t budget = e->fp_sub_bytes;
  if (budget <= 0) {
    size_t fr = 0, tot = 0, idle = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
      (void)hipGetLastError();
      fr = tot = 0;
    }
    (void)ws_pool_bytes(e->device, &idle);
    const int64_t outb = (int64_t)(d.es * d.out_len * (size_t)ld_out + 64 * (size_t)ld_out);
    const int64_t reserve = std::max<int64_t>((int64_t)8 << 30, (int64_t)(0.10 * (double)tot));
    budget = (int64_t)(fr + idle) - outb - reserve - (int64_t)other_bytes;
  }
  uint64_t cols = (uint64_t)std::max<int64_t>(budget, 1) / per;
  cols = std::max<uint64_t>(256, cols & ~255ull);
  return (uint32_t)std::min<uint64_t>(ld_out, cols);
}

static bool own_out(const DevParams& d) {  // the output share is not the measurement share
  return d.kind == PRIO3_SUM || d.kind == PRIO3_SUMVEC || d.kind == PRIO3_SUMVEC_F64_MP ||
         d.kind == PRIO3_FPVEC_BOUNDED_L2;
}

constexpr uint32_t WCH_HOST = 32;  // waves per fused-partial chunk (k_agg_waves WCH)

template <class F>
static void launch_xof_slow(const prio3_engine* e, const DevParams& p, const InPtrs& in,
                            const Scratch& sc, hipStream_t st) {
  (void)e;
  k_xof_slow<F><<<slow_blocks(p.n), 64, 0, st>>>(p, in, sc);
}

// Lays the run's buffers out from `base` (nullptr: sizes only), 256-byte aligned.
static size_t run_carve(Run* R, unsigned flags, uint32_t n_keys, uint8_t* base) {
  const DevParams& d = R->dp;
  const size_t es = d.es, ld = d.ld, ldo = d.ld_out, n = R->n ? R->n : 1;
  size_t off = 0;
  auto take = [&](auto** ptr, size_t bytes) {
    *ptr = base ? (std::remove_pointer_t<decltype(ptr)>)(base + off) : nullptr;
    off += (bytes + 255) & ~(size_t)255;
  };
  if (flags & RUN_SCRATCH) {
    const bool fp = d.kind == PRIO3_FPVEC_BOUNDED_L2;
    take(&R->sc.meas, es * d.meas_len * ld);
    take(&R->sc.proofs, es * d.proof_len * ld);
    take(&R->sc.jr, es * (d.jr_len ? d.jr_len : 1) * ld);
    take(&R->sc.qr, es * d.qr_len * ld);
    take(&R->sc.part, 16 * ld);
    take(&R->sc.corrected, 16 * ld);
    take(&R->sc.flag, ld);
    take(&R->sc.Lbuf, es * ((size_t)d.P + d.P1) * ld);
    take(&R->sc.PVbuf, es * ((size_t)d.P + d.P1) * ld);
    take(&R->sc.acc, fp ? 16 : es * d.arity * ld);
    take(&R->sc.out, own_out(d) ? es * d.out_len * ldo : 16);
    take(&R->sc.beta, es * d.calls * ld);
    // FPVec runs in sub-batches of ld columns: the leader's corrected seeds of every report
    // outlive their sub-batch's scratch (prepare_next reads them)
    if (fp) take(&R->corr_all, 16 * n);
  }
  if (flags & RUN_IO) {
    const size_t ml = R->e->sz.prep_msg_len ? R->e->sz.prep_msg_len : 16;
    take(&R->nonces, 16 * n);
    take(&R->pub, (size_t)(d.public_share_len ? d.public_share_len : 16) * n);
    take(&R->helper, (size_t)d.helper_share_len * n);
    take(&R->leader, (size_t)d.prep_share_len * n);
    take(&R->msgs, ml * n);
    take(&R->status, n);
  }
  if (flags & RUN_LINPUT) take(&R->linput, (size_t)d.leader_share_len * n);
  if (flags & RUN_VK) {
    take(&R->vk_slot, 2 * n);
    take(&R->vk_tab, 16 * (size_t)(n_keys ? n_keys : 1));
  }
  if (flags & RUN_AGG_IO) {
    const size_t S = R->nseg ? R->nseg : 1;
    take(&R->gseg, 4 * n);
    take(&R->gaccept, n);
    take(&R->gagg, (size_t)d.out_len * es * S);
    take(&R->gcnt, 8 * S);
  }
  if (flags & RUN_HPKE) {
    take(&R->hstatus, n);
    take(&R->hpt, (size_t)R->hpke_stride * n);
  }
  if (flags & RUN_FUSED) {
    // sized for 32-report waves (k_prep_hp); the one-lane kernels use the first half
    const size_t waves = (n + 31) / 32, M = d.meas_len, chunks = (waves + WCH_HOST - 1) / WCH_HOST;
    take(&R->wpart, waves * M * 8 * sizeof(uint32_t));
    take(&R->wseg, waves * sizeof(uint32_t));
    take(&R->cpart, chunks * M * 8 * 8);
    take(&R->cseg, chunks * sizeof(uint32_t));
    take(&R->agg64, (size_t)(R->nseg ? R->nseg : 1) * M * 8 * 8);
    take(&R->fix, (n + 1) * sizeof(uint32_t));
  }
  return off;
}

static Run* run_create(prio3_engine* e, uint32_t n, unsigned flags, uint32_t nseg,
                       uint32_t n_keys, hipStream_t st, int* rc, uint32_t hpke_stride = 0) {
  Run* R = new Run();
  R->e = e;
  R->hpke_stride = hpke_stride;
  R->device = e->device;
  R->n = n;
  R->nseg = nseg;
  R->dp = e->dp;
  R->dp.n = n;
  R->dp.nseg = nseg ? nseg : 1;
  const uint32_t ld_out = ((n ? n : 1) + 63) & ~63u;
  R->dp.ld_out = ld_out;
  R->dp.ld = ld_out;
  if ((flags & RUN_SCRATCH) && e->dp.kind == PRIO3_FPVEC_BOUNDED_L2) {
    // the rest of the run (I/O copies, the leader's explicit input shares: 2.6 MB per report at
    // 10^4 entries) comes out of the same budget as the scratch sub-batch
    const size_t other = run_carve(R, flags & ~RUN_SCRATCH, n_keys, nullptr);
    R->dp.ld = fp_sub_ld(e, e->dp, ld_out, other);
  }
  const size_t bytes = run_carve(R, flags, n_keys, nullptr);
  R->slab = ws_acquire(e->device, bytes, st, rc);
  if (!R->slab) {
    delete R;
    return nullptr;
  }
  run_carve(R, flags, n_keys, R->slab->base);
  R->keep = e->keep_scratch != 0;
  R->fix_cap = (size_t)n + 1;
  R->last = st;
  return R;
}

// drops one reference; the last one returns the slab to the pool, ordered after `st` (or the
// stream of the run's latest work)
static void run_release(Run* R, hipStream_t st, bool use_st) {
  if (!R) return;
  if (R->refs.fetch_sub(1) != 1) return;
  ws_release(R->slab, use_st ? st : R->last, R->keep);
  delete R;
}

// ---- one-pass segmented accumulate over columns [c0, c0 + n) of a run ----
// d_status[n] (the run's verdicts for those columns), d_seg[n] (nullable: segment 0), d_accept[n]
// (nullable: all accepted); d_agg[nseg][out_len * es], d_counts[nseg].
static int run_accumulate(prio3_engine* e, Run* R, uint32_t c0, uint32_t n,
                          const uint8_t* d_status, const uint32_t* d_seg, const uint8_t* d_accept,
                          uint32_t nseg, uint8_t* d_agg, uint64_t* d_counts, hipStream_t st) {
  const DevParams& d = R->dp;
  const size_t es = d.es, agg_len = (size_t)d.out_len * es;
  if (n == 0) {
    HIPCHK(hipMemsetAsync(d_agg, 0, agg_len * nseg, st));
    HIPCHK(hipMemsetAsync(d_counts, 0, 8 * (size_t)nseg, st));
    return PRIO3_OK;
  }
  // reports per k_acc_seg block: 8192, or 2048 for the short outputs (Count, Sum) whose grid
  // would otherwise be a few blocks wide
  const bool short_out = d.out_len <= 4;
  const uint32_t chunk = short_out ? 2048 : 8192, nchunks = (n + chunk - 1) / chunk;
  const size_t part_b = ((size_t)nchunks * nseg * agg_len + 255) & ~(size_t)255;
  int rc = PRIO3_OK;
  Slab* tmp = ws_acquire(R->device, part_b + 8 * (size_t)nchunks * nseg, st, &rc);
  if (!tmp) return rc;
  void* partial = tmp->base;
  uint64_t* pcount = (uint64_t*)(tmp->base + part_b);
  const uint8_t* src = (const uint8_t*)(own_out(d) ? R->sc.out : R->sc.meas) + es * c0;
  const size_t ld = d.ld_out;  // output shares: one column per report of the run
  auto body = [&]() -> int {
    const int SG = nseg == 1 ? 1 : nseg <= 4 ? 4 : 8;
    dim3 grid(d.out_len, nchunks, (nseg + SG - 1) / SG);
    dim3 gfin((d.out_len + 255) / 256, nseg);
    if (es == 16) {
      if (SG == 1)
        TIMED(e, st, "k_acc_seg", (k_acc_seg<Fp128, 1><<<grid, 256, 0, st>>>(n, ld, chunk, d.out_len, nseg, src, d_status, d_seg, d_accept, partial, pcount)));
      else if (SG == 4)
        TIMED(e, st, "k_acc_seg", (k_acc_seg<Fp128, 4><<<grid, 256, 0, st>>>(n, ld, chunk, d.out_len, nseg, src, d_status, d_seg, d_accept, partial, pcount)));
      else
        TIMED(e, st, "k_acc_seg", (k_acc_seg<Fp128, 8><<<grid, 256, 0, st>>>(n, ld, chunk, d.out_len, nseg, src, d_status, d_seg, d_accept, partial, pcount)));
      if (short_out)
        TIMED(e, st, "k_acc_fin", (k_acc_fin_blk<Fp128><<<dim3(d.out_len, nseg), 256, 0, st>>>(nchunks, d.out_len, nseg, partial, pcount, d_agg, d_counts)));
      else
        TIMED(e, st, "k_acc_fin", (k_acc_fin<Fp128><<<gfin, 256, 0, st>>>(nchunks, d.out_len, nseg, partial, pcount, d_agg, d_counts)));
    } else {
      if (SG == 1)
        TIMED(e, st, "k_acc_seg", (k_acc_seg<Fp64, 1><<<grid, 256, 0, st>>>(n, ld, chunk, d.out_len, nseg, src, d_status, d_seg, d_accept, partial, pcount)));
      else if (SG == 4)
        TIMED(e, st, "k_acc_seg", (k_acc_seg<Fp64, 4><<<grid, 256, 0, st>>>(n, ld, chunk, d.out_len, nseg, src, d_status, d_seg, d_accept, partial, pcount)));
      else
        TIMED(e, st, "k_acc_seg", (k_acc_seg<Fp64, 8><<<grid, 256, 0, st>>>(n, ld, chunk, d.out_len, nseg, src, d_status, d_seg, d_accept, partial, pcount)));
      if (short_out)
        TIMED(e, st, "k_acc_fin", (k_acc_fin_blk<Fp64><<<dim3(d.out_len, nseg), 256, 0, st>>>(nchunks, d.out_len, nseg, partial, pcount, d_agg, d_counts)));
      else
        TIMED(e, st, "k_acc_fin", (k_acc_fin<Fp64><<<gfin, 256, 0, st>>>(nchunks, d.out_len, nseg, partial, pcount, d_agg, d_counts)));
    }
    return PRIO3_OK;
  };
  rc = body();
  ws_release(tmp, st);
  R->last = st;
  return rc;
}

// columns [c0, c0 + n) of the run's output shares to host, per report (n x out_len x es)
static int run_output_shares(Run* R, uint32_t c0, uint32_t n, uint8_t* out, hipStream_t st) {
  const DevParams& d = R->dp;
  const size_t es = d.es;
  if (n == 0) return PRIO3_OK;
  const uint8_t* src = (const uint8_t*)(own_out(d) ? R->sc.out : R->sc.meas) + es * c0;
  std::vector<uint8_t> soa((size_t)d.out_len * n * es);
  HIPCHK(hipMemcpy2DAsync(soa.data(), n * es, src, (size_t)d.ld_out * es, n * es, d.out_len,
                          hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  for (uint32_t r = 0; r < n; r++)
    for (uint32_t i = 0; i < d.out_len; i++)
      memcpy(out + ((size_t)r * d.out_len + i) * es, soa.data() + ((size_t)i * n + r) * es, es);
  return PRIO3_OK;
}

// a pooled stream for one blocking host-buffer call
struct PooledStream {
  int device;
  hipStream_t s;
  explicit PooledStream(int dev) : device(dev), s(ws_stream_get(dev)) {}
  ~PooledStream() { ws_stream_put(device, s); }
};


// The fused accumulate applies where the output share is the measurement share (Histogram;
// truncate is the identity) and the joint-rand kernel streams that share.
static bool fusable(const prio3_engine* e) {
  return e->fuse_acc && e->dp.kind == PRIO3_HISTOGRAM && e->dp.jr_len &&
         (42 + e->dp.meas_len * 16) / 168 >= 2;
}

// side streams + their join events and the fork event, created once per engine
static int ensure_side_streams(prio3_engine* e) {
  while (e->side.size() < 2) {
    hipStream_t s2;
    hipEvent_t j;
    HIPCHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
    e->side.push_back(s2);
    e->side_ev.push_back(j);
  }
  if (!e->fork_ev) HIPCHK(hipEventCreateWithFlags(&e->fork_ev, hipEventDisableTiming));
  return PRIO3_OK;
}

// The helper chain of this instance is the fused k_prep_h (dual-state XOF + k_query_h<2, 32>
// in one launch; the conditions under which launch_prepare would launch exactly those two).
static bool prep_fused_takes(const prio3_engine* e, const DevParams& dp, bool fuse) {
  if (e->force_generic) return false;
  const bool ps = dp.kind == PRIO3_HISTOGRAM || dp.kind == PRIO3_SUMVEC;
  const bool dual = dp.es == 16 && dp.jr_len && (42 + dp.meas_len * 16) / 168 >= 2;
  if (dp.kind == PRIO3_SUM) return dual && !fuse && query_sum_takes(dp);  // k_prep_sum
  return ps && dual && dp.P == 32;                                         // k_prep_h
}

// which query family deferred the slow path of its flagged reports (launch_slow_redo redoes them)
enum : int { DEFER_NONE = 0, DEFER_QH = 1, DEFER_SUM = 2, DEFER_GEN64 = 3 };
// *deferred: set when a query kernel of this chain skipped flagged reports (slow_defer); the
// caller then ends the run with launch_slow_redo
// in.leader_src (executor groups, pulls_in_xof): the leader prep shares are still in the mapped
// host staging and the fused k_prep_h<.., PULL> copies them lane by lane during its XOF.
// pair: Histogram on lane pairs (k_prep_hp, prio3_prep_pair.hip) instead of k_prep_h
static int launch_prepare(prio3_engine* e, const DevParams& base, uint32_t c0, uint32_t n,
                          InPtrs in, OutPtrs out, Scratch sc, hipStream_t st, bool fuse,
                          int* deferred, bool pair = false) {
  DevParams dp = base;
  dp.n = n;
  dp.force_slow = (uint32_t)e->force_slow;
  dp.slow_defer = 0;
  dp.redo = 0;
  const size_t es = dp.es;
  in.nonces += 16 * (size_t)c0;
  if (in.pub) in.pub += (size_t)dp.public_share_len * c0;
  in.helper += (size_t)dp.helper_share_len * c0;
  in.leader += (size_t)dp.prep_share_len * c0;
  if (in.vk_slot) in.vk_slot += c0;
  out.prep_msgs += (size_t)(dp.kind == PRIO3_SUMVEC_F64_MP ? 32 : 16) * c0;
  out.status += c0;
  void** soa[] = {&sc.meas, &sc.proofs, &sc.jr, &sc.qr, &sc.Lbuf, &sc.PVbuf, &sc.acc, &sc.out,
                  &sc.beta};
  for (auto q : soa)
    if (*q) *q = (uint8_t*)*q + es * c0;
  sc.part += c0;
  sc.corrected += c0;
  sc.flag += c0;
  if (sc.seg) sc.seg += c0;
  if (sc.wseg) sc.wseg += c0 / 64;
  if (sc.wpart) sc.wpart += (size_t)(c0 / 64) * dp.meas_len * 8;
  const uint32_t blocks = (n + 255) / 256;
  if (dp.kind == PRIO3_SUMVEC_F64_MP) {
    int rc = PRIO3_OK;
    TIMED(e, st, "k_mp64_prepare", (rc = launch_mp64(e, n, dp.ld, in, out, sc, st)));
    return rc;
  }
  if (dp.kind == PRIO3_FPVEC_BOUNDED_L2) {
    // Sub-batches of dp.ld reports through the per-report scratch (the whole batch's meas
    // shares would not fit: 2.56 MB per report at 10^4 entries); output shares keep one
    // column per report of the batch (ld_out), so accumulate runs once over all of them.
    // Equal sub-batches, cut at whole query rounds (fp_sub_sizes): per-lane latency, not lane
    // count, sets a launch's duration.
    uint32_t nsub, sub;
    const bool qwide = !e->force_generic && fpvec_query_wide_takes(dp);
    fp_sub_sizes(e, n, dp.ld, qwide, nsub, sub);
    for (uint32_t si = 0; si < nsub; si++) {
      const uint32_t s0 = si * sub;
      DevParams q = dp;
      q.n = si + 1 < nsub ? sub : n - s0;
      InPtrs qi = in;
      qi.nonces += 16 * (size_t)s0;
      qi.pub += (size_t)dp.public_share_len * s0;
      qi.helper += (size_t)dp.helper_share_len * s0;
      qi.leader += (size_t)dp.prep_share_len * s0;
      if (qi.vk_slot) qi.vk_slot += s0;
      OutPtrs qo = out;
      qo.prep_msgs += 16 * (size_t)s0;
      qo.status += s0;
      Scratch qs = sc;
      qs.out = (uint8_t*)sc.out + es * s0;
      const uint32_t qb = (q.n + 255) / 256;
      // the lane-pair XOF (k_xof_pair, the entries decoded as the share is squeezed), else the
      // dual-state k_xofd; both decode the entries (the output share) on the fly
      const bool dual = (42 + dp.meas_len * 16) / 168 >= 2;
      q.trunc_xof = dual ? 1u : 0u;
      bool paired = false;
      if (dual) TIMED(e, st, "k_xof_pair", (paired = launch_xof_pair(q, qi, qs, st)));
      if (!paired && dual)
        TIMED(e, st, "k_xofd", (k_xofd<false, true><<<qb, 256, 0, st>>>(q, qi, qs)));
      else if (!paired)
        TIMED(e, st, "k_xof", (k_xof<Fp128><<<qb, 256, 0, st>>>(q, qi, qs)));
      TIMED(e, st, "k_xof_slow", launch_xof_slow<Fp128>(e, q, qi, qs, st));
      if (qwide)
        TIMED(e, st, "k_query_fpw", launch_fpvec_query(q, qi, qs, qo, st, true, false));
      else
        TIMED(e, st, "k_query_fp", launch_fpvec_query(q, qi, qs, qo, st, false, false));
    }
    return PRIO3_OK;
  }
  if (dp.es == 16) {
    const bool ps = dp.kind == PRIO3_HISTOGRAM || dp.kind == PRIO3_SUMVEC;
    // P = 64 / 128 on eight lanes per report (k_query_w)
    const bool wide = ps && !e->force_generic && dp.P != 32 && query_wide_takes(dp);
    const bool dual = dp.jr_len && (42 + dp.meas_len * 16) / 168 >= 2;
    // SumVec under k_query_w: the truncation rides on the XOF's squeeze (the query then reads
    // the share once)
    dp.trunc_xof = dp.kind == PRIO3_SUMVEC && wide && dual && !fuse ? 1u : 0u;
    // XOF + query in one launch: Prio3Sum (k_prep_sum) and Histogram / SumVec with P = 32
    // (k_prep_h); the slow path of both is deferred to the run's redo launch
    if (prep_fused_takes(e, dp, fuse)) {
      dp.slow_defer = 1u;
      if (dp.kind == PRIO3_SUM) {
        if (deferred) *deferred = DEFER_SUM;
        switch (dp.P) {
          case 16: TIMED(e, st, "k_prep_sum", (k_prep_sum<1><<<blocks, 256, 0, st>>>(dp, in, sc, out))); break;
          case 32: TIMED(e, st, "k_prep_sum", (k_prep_sum<2><<<blocks, 256, 0, st>>>(dp, in, sc, out))); break;
          case 64: TIMED(e, st, "k_prep_sum", (k_prep_sum<4><<<blocks, 256, 0, st>>>(dp, in, sc, out))); break;
          default: TIMED(e, st, "k_prep_sum", (k_prep_sum<8><<<blocks, 256, 0, st>>>(dp, in, sc, out))); break;
        }
      } else {
        if (deferred) *deferred = DEFER_QH;
        const bool pl = in.leader_src != nullptr;
        bool paired = false;
        if (pair)
          TIMED(e, st, "k_prep_hp", (paired = launch_prep_pair(dp, in, sc, out, st, fuse, pl)));
        if (paired) {
        } else if (fuse && pl)
          TIMED(e, st, "k_prep_h", (k_prep_h<true, true><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
        else if (fuse)
          TIMED(e, st, "k_prep_h", (k_prep_h<true><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
        else if (pl)
          TIMED(e, st, "k_prep_h", (k_prep_h<false, true><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
        else
          TIMED(e, st, "k_prep_h", (k_prep_h<false><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
      }
      return PRIO3_OK;
    }
    // two kernels: the XOF (dual-state k_xofd when the share spans >= 2 joint-rand blocks, else
    // k_xof_a + k_jrpart), then the query
    if (dual) {
      if (fuse)
        TIMED(e, st, "k_xofd", (k_xofd<true><<<blocks, 256, 0, st>>>(dp, in, sc)));
      else if (dp.trunc_xof)
        TIMED(e, st, "k_xofd", (k_xofd<false, true><<<blocks, 256, 0, st>>>(dp, in, sc)));
      else
        TIMED(e, st, "k_xofd", (k_xofd<false><<<blocks, 256, 0, st>>>(dp, in, sc)));
    } else {
      TIMED(e, st, "k_xof_a", (k_xof_a<Fp128><<<blocks, 256, 0, st>>>(dp, in, sc)));
      TIMED(e, st, "k_jrpart", (k_jrpart<false><<<blocks, 256, 0, st>>>(dp, in, sc)));
    }
    // k_query_h defers flagged reports to the run's redo pass (slow_defer); the other queries
    // read the shares the k_xof_slow launch rewrote
    const bool qh_path =
        ps && !e->force_generic && !wide && (dp.P == 32 || dp.P == 16 || dp.P == 8);
    dp.slow_defer = qh_path ? 1u : 0u;
    if (qh_path && deferred) *deferred = DEFER_QH;
    if (!qh_path) TIMED(e, st, "k_xof_slow", launch_xof_slow<Fp128>(e, dp, in, sc, st));
    bool done = false;
    if (wide) TIMED(e, st, "k_query_w", (done = launch_query_wide(dp, in, sc, out, st)));
    if (done) {
    } else if (qh_path && dp.P == 32)
      TIMED(e, st, "k_query_h", (k_query_h<2, 32><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
    else if (qh_path && dp.P == 16)
      TIMED(e, st, "k_query_h", (k_query_h<2, 16><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
    else if (qh_path && dp.P == 8)
      TIMED(e, st, "k_query_h", (k_query_h<2, 8><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
    else if (ps)
      TIMED(e, st, "k_query_ps", (k_query_ps<4><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
    else {
      bool qs = false;
      if (!e->force_generic && query_sum_takes(dp))
        TIMED(e, st, "k_query_sum", (qs = launch_query_sum(dp, in, sc, out, st)));
      if (!qs) TIMED(e, st, "k_query", (k_query<Fp128><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
    }
  } else {  // Field64 (Prio3Count): XOF + query in one launch, the slow path deferred
    dp.slow_defer = 1u;
    if (deferred) *deferred = DEFER_GEN64;
    TIMED(e, st, "k_prep_gen", (k_prep_gen<Fp64><<<blocks, 256, 0, st>>>(dp, in, sc, out)));
  }
  return PRIO3_OK;
}



// The deferred slow path of a run whose k_query_h launches skipped the reports the XOF flagged
// (slow_defer): one k_slow_redo launch over the whole run redoes their XOF (marking them 2) and
// then their query (redo = 1), lane by lane.  One launch per run instead of one k_xof_slow
// launch between the XOF and the query of every chunk, where its one-wave blocks waited behind
// the other stream's kernels (~0.2 ms per chunk in the r02 trace).
// k_slow_redo<PP>: both halves in one launch -- each lane scans the flags of REDO_RPL reports
// (16-byte loads) and, for a flagged report, re-runs its XOF (flag := 2) and then its query on
// the same lane.
template <int PP>
__global__ __launch_bounds__(64) void k_slow_redo(DevParams p, InPtrs in, Scratch sc, OutPtrs out) {
  const uint32_t r0 = (blockIdx.x * blockDim.x + threadIdx.x) * REDO_RPL;
  if (r0 >= p.n || !redo_any(p, sc, r0)) return;
  const uint8_t* fl = sc.flag + r0;
  for (uint32_t i = 0; i < REDO_RPL && r0 + i < p.n; i++)
    if (fl[i]) {
      xof_slow_one<Fp128>(p, in, sc, r0 + i);
      query_h_body<2, PP>(p, in, sc, out, r0 + i);
    }
}

template <int NPH>
__global__ __launch_bounds__(64) void k_slow_redo_sum(DevParams p, InPtrs in, Scratch sc,
                                                      OutPtrs out) {
  const uint32_t r0 = (blockIdx.x * blockDim.x + threadIdx.x) * REDO_RPL;
  if (r0 >= p.n || !redo_any(p, sc, r0)) return;
  const uint8_t* fl = sc.flag + r0;
  for (uint32_t i = 0; i < REDO_RPL && r0 + i < p.n; i++)
    if (fl[i]) {
      xof_slow_one<Fp128>(p, in, sc, r0 + i);
      qsum::query_sum_body<NPH, 0>(p, in, sc, out, r0 + i);
    }
}

static int launch_slow_redo(prio3_engine* e, const DevParams& base, uint32_t n, InPtrs in,
                            OutPtrs out, Scratch sc, hipStream_t st, int family) {
  DevParams dp = base;
  dp.n = n;
  dp.force_slow = (uint32_t)e->force_slow;
  dp.trunc_xof = 0;
  dp.slow_defer = 1;
  dp.redo = 1;
  const uint32_t g = redo_blocks(n);
  if (family == DEFER_GEN64) {  // k_prep_gen<Fp64>: XOF redo, then the generic query
    TIMED(e, st, "k_slow_redo", (k_slow_redo_gen<Fp64><<<g, 64, 0, st>>>(dp, in, sc, out)));
  } else if (family == DEFER_SUM) {
    switch (dp.P) {
      case 16: TIMED(e, st, "k_slow_redo", (k_slow_redo_sum<1><<<g, 64, 0, st>>>(dp, in, sc, out))); break;
      case 32: TIMED(e, st, "k_slow_redo", (k_slow_redo_sum<2><<<g, 64, 0, st>>>(dp, in, sc, out))); break;
      case 64: TIMED(e, st, "k_slow_redo", (k_slow_redo_sum<4><<<g, 64, 0, st>>>(dp, in, sc, out))); break;
      default: TIMED(e, st, "k_slow_redo", (k_slow_redo_sum<8><<<g, 64, 0, st>>>(dp, in, sc, out))); break;
    }
  } else if (dp.P == 32)
    TIMED(e, st, "k_slow_redo", (k_slow_redo<32><<<g, 64, 0, st>>>(dp, in, sc, out)));
  else if (dp.P == 16)
    TIMED(e, st, "k_slow_redo", (k_slow_redo<16><<<g, 64, 0, st>>>(dp, in, sc, out)));
  else
    TIMED(e, st, "k_slow_redo", (k_slow_redo<8><<<g, 64, 0, st>>>(dp, in, sc, out)));
  return PRIO3_OK;
}

// The kernel chain over the whole run.  Option "chunks" > 1 (auto: one chunk per 128Ki reports,
// measured best on MI355X at 1Mi reports: 8 chunks +4-5% over 1; 16: slower): the batch is cut
// into column ranges whose chains alternate over the engine's two side streams (joined to `st`
// before and after), so one chunk's memory-bound query overlaps the next chunk's VALU-bound
// Keccak.  Side streams are per engine: callers that may overlap (the executor's concurrent
// groups) pass allow_chunks = false.
// The chains whose XOF can pull the leader prep shares (the fused k_prep_h: the query reads them
// only after the same lane's XOF); the share is copied in 16-byte pieces over the share loop.
// Every wave must be whole (the executor pads its groups to 64 columns for these instances).
static bool pulls_in_xof(const prio3_engine* e, const DevParams& dp, bool fuse, uint32_t n) {
  const uint32_t B = (42 + dp.meas_len * 16) / 168;  // share-loop iterations: B - 1
  return prep_fused_takes(e, dp, fuse) && dp.kind != PRIO3_SUM && dp.prep_share_len % 16 == 0 &&
         B >= 2 && dp.prep_share_len / 16 <= 2 * (B - 1) && n % 64 == 0;
}

// Histogram (P = 32) runs of at most pair_max reports on lane pairs (k_prep_hp)
static bool pair_takes(const prio3_engine* e, const DevParams& base, uint32_t n, bool fuse,
                       bool pulling) {
  if (e->pair_max <= 0 || n == 0 || n > (uint32_t)e->pair_max || !prep_fused_takes(e, base, fuse))
    return false;
  DevParams d = base;
  d.n = n;
  return prep_pair_takes(d, pulling);
}

// pull (nullable; executor groups): copies the leader prep shares (and the fix-up inputs) from
// the mapped host staging into the run -- inside the fused XOF + query launch where the chain is
// k_prep_h (pulls_in_xof), else by one copy launch ahead of the chain.
static int prepare_run(prio3_engine* e, Run* R, InPtrs in, OutPtrs out, hipStream_t st, bool fuse,
                       bool allow_chunks, const PullRanges* pull = nullptr) {
  const uint32_t n = R->n;
  if (pull && pulls_in_xof(e, R->dp, fuse, n)) {
    in.leader_src = pull->src[0];
    in.seg_src = (const uint32_t*)pull->src[1];
    in.seg_dst = (uint32_t*)pull->dst[1];
    in.accept_src = pull->src[2];
    in.accept_dst = pull->dst[2];
    allow_chunks = false;
  } else if (pull) {
    k_pull<<<256, 256, 0, st>>>(*pull);
    HIPCHK(hipGetLastError());
  }
  Scratch sc = R->sc;
  sc.seg = R->seg;
  sc.wpart = R->wpart;
  sc.wseg = R->wseg;
  R->last = st;
  // small Histogram runs (the executor's groups) on lane pairs: twice the waves, half the work each
  const bool pair = pair_takes(e, R->dp, n, fuse, in.leader_src != nullptr);
  R->wshift = pair ? 5u : 6u;
  // auto: one chunk per 128Ki reports on the two-kernel chain; one launch for the fused k_prep_h
  // (A/B on MI355X, 1 Mi reports: 169.9 M/s at 1 chunk vs 163.2 M/s at 8) and for the one-kernel
  // multiproof prepare (1 M reports: 93.1-93.3 M/s at 1 chunk vs 89.0-91.5 at 8, r04e2)
  const uint32_t K = e->chunks > 0 ? (uint32_t)e->chunks
                     : (prep_fused_takes(e, R->dp, fuse) || R->dp.kind == PRIO3_SUMVEC_F64_MP)
                         ? 1u
                         : std::max(1u, (n + (1u << 16)) >> 17);
  const uint32_t csz = ((n + K - 1) / K + 255) & ~255u;
  int deferred = DEFER_NONE;
  if (pair || !allow_chunks || K == 1 || n <= csz || R->dp.kind == PRIO3_FPVEC_BOUNDED_L2) {
    const int rc = launch_prepare(e, R->dp, 0, n, in, out, sc, st, fuse, &deferred, pair);
    if (rc == PRIO3_OK && deferred)
      return launch_slow_redo(e, R->dp, n, in, out, sc, st, deferred);
    return rc;
  }
  int rc = ensure_side_streams(e);
  if (rc) return rc;
  HIPCHK(hipEventRecord(e->fork_ev, st));
  for (auto s2 : e->side) HIPCHK(hipStreamWaitEvent(s2, e->fork_ev, 0));
  uint32_t c = 0;
  for (uint32_t c0 = 0; c0 < n; c0 += csz, c++) {
    rc = launch_prepare(e, R->dp, c0, std::min(csz, n - c0), in, out, sc, e->side[c % 2], fuse,
                        &deferred);
    if (rc) return rc;
  }
  for (size_t i = 0; i < e->side.size(); i++) {
    HIPCHK(hipEventRecord(e->side_ev[i], e->side[i]));
    HIPCHK(hipStreamWaitEvent(st, e->side_ev[i], 0));
  }
  if (deferred) return launch_slow_redo(e, R->dp, n, in, out, sc, st, deferred);
  return PRIO3_OK;
}

// the leader's prepare_init (agg_id 0) over the run
extern "C" int launch_leader_init(const DevParams& dp, const uint8_t* d_nonces, const uint8_t* d_pub,
                                  const uint8_t* d_lshares, const Scratch& sc,
                                  uint8_t* d_prep_shares, uint8_t* d_status, hipStream_t st,
                                  const uint16_t* vk_slot, const uint4* vk_tab);
extern "C" int launch_leader_next(const DevParams& dp, const uint8_t* d_prep_msgs, const Scratch& sc,
                       uint8_t* d_status, hipStream_t st);

// FPVec leader (agg_id 0): sub-batches of the run's ld columns, each through the helper's
// kernels in their leader role -- k_leader_unpack (explicit share -> SoA, canonical check, both
// query points), k_jrpart<false, true> (the leader's joint-rand part over its 2.56 MB share,
// corrected seed, joint randomness), k_leader_slowfix, k_query_fpw<GS, LEADER> (verifier share,
// the decoded entries as output shares) -- and the corrected seeds saved for prepare_next.
static int leader_init_fpvec(prio3_engine* e, Run* R, const uint8_t* d_nonces,
                             const uint8_t* d_pub, const uint8_t* d_lin, uint8_t* d_prep_shares,
                             uint8_t* d_status, hipStream_t st) {
  DevParams dp = R->dp;
  dp.force_slow = (uint32_t)e->force_slow;
  dp.trunc_xof = 0;
  if (!fpvec_query_wide_takes(dp) || !R->corr_all) return PRIO3_EUNSUPPORTED;
  const uint32_t n = R->n, cap = dp.ld;
  uint32_t nsub, sub;
  fp_sub_sizes(e, n, cap, true, nsub, sub);
  const size_t es = dp.es;
  for (uint32_t si = 0; si < nsub; si++) {
    const uint32_t s0 = si * sub;
    DevParams q = dp;
    q.n = si + 1 < nsub ? sub : n - s0;
    InPtrs qi{d_nonces + 16 * (size_t)s0,
              d_pub ? d_pub + (size_t)dp.public_share_len * s0 : nullptr,
              d_lin + (size_t)dp.leader_share_len * s0, nullptr};
    OutPtrs qo{d_prep_shares + (size_t)dp.prep_share_len * s0, d_status + s0};
    Scratch qs = R->sc;
    qs.out = (uint8_t*)R->sc.out + es * s0;
    const uint32_t blocks = (q.n + 255) / 256, blocks64 = (q.n + 63) / 64;
    TIMED(e, st, "k_leader_unpack",
          (k_leader_unpack<<<(q.n + 63) / 64, 256, 0, st>>>(q, qi, qs, qo.status, nullptr, nullptr)));
    TIMED(e, st, "k_jrpart", (k_jrpart<false, true><<<blocks, 256, 0, st>>>(q, qi, qs)));
    TIMED(e, st, "k_leader_slowfix", (k_leader_slowfix<<<blocks64, 64, 0, st>>>(q, qi, qs)));
    TIMED(e, st, "k_query_fpw", launch_fpvec_query(q, qi, qs, qo, st, true, true));
    HIPCHK(hipMemcpyAsync(R->corr_all + s0, qs.corrected, 16 * (size_t)q.n,
                          hipMemcpyDeviceToDevice, st));
  }
  return PRIO3_OK;
}

#ifndef LEADER_FUSED
#define LEADER_FUSED 1  // k_leader_prep (k_leader_jr + the query in one launch); 0: two kernels (A/B)
#endif
// vk_slot / vk_tab (nullable): per-report verify keys of a coalesced group of several tasks
// The instances whose leader prepare_init is one k_leader_prep launch (the only leader kernel that
// reads the leader input shares from SoA staging, InPtrs::lin_ld)
static bool leader_prep_takes(const prio3_engine* e) {
  const DevParams& dp = e->dp;
  return LEADER_FUSED && e->leader_fast && (dp.kind == PRIO3_HISTOGRAM || dp.kind == PRIO3_SUMVEC) &&
         dp.jr_len && (dp.P == 32 || dp.P == 16 || dp.P == 8) &&
         dp.leader_share_len == 16 * (dp.meas_len + dp.proof_len + 1);
}

static int leader_init_run(prio3_engine* e, Run* R, const uint8_t* d_nonces,
                           const uint8_t* d_public_shares, const uint8_t* d_leader_input_shares,
                           uint8_t* d_prep_shares, uint8_t* d_status, hipStream_t st,
                           const uint16_t* vk_slot = nullptr, const uint4* vk_tab = nullptr,
                           uint32_t lin_ld = 0) {
  DevParams dp = R->dp;
  dp.force_slow = (uint32_t)e->force_slow;
  const uint32_t n = R->n;
  R->last = st;
  if (dp.kind == PRIO3_FPVEC_BOUNDED_L2)
    return leader_init_fpvec(e, R, d_nonces, d_public_shares, d_leader_input_shares,
                             d_prep_shares, d_status, st);
  if (dp.kind == PRIO3_SUMVEC_F64_MP) {
    int rc = PRIO3_OK;
    TIMED(e, st, "k_mp64_prepare",
          (rc = launch_mp64_leader(e, n, dp.ld, InPtrs{d_nonces, d_public_shares,
                                                       d_leader_input_shares, nullptr},
                                   OutPtrs{d_prep_shares, d_status}, R->sc, st)));
    return rc;
  }
  const bool ps = dp.kind == PRIO3_HISTOGRAM || dp.kind == PRIO3_SUMVEC;
  if (ps && dp.jr_len && (dp.P == 32 || dp.P == 16 || dp.P == 8) && e->leader_fast) {
    // the helper kernels in their leader role
    InPtrs in{d_nonces, d_public_shares, d_leader_input_shares, nullptr};
    in.vk_slot = vk_slot;
    in.vk_tab = vk_tab;
    in.lin_ld = LEADER_FUSED ? lin_ld : 0u;
    OutPtrs out{d_prep_shares, d_status};
    const uint32_t blocks = (n + 255) / 256, blocks64 = (n + 63) / 64;
    // R->lfused: the wave partials of the share for segment 0, fixed up at accumulate
    uint32_t* wp = R->lfused ? R->wpart : nullptr;
    uint32_t* wsg = R->lfused ? R->wseg : nullptr;
    if (LEADER_FUSED) {  // one launch; flagged reports redone after k_leader_slowfix
      DevParams d1 = dp;
      d1.slow_defer = 1;
      if (dp.P == 32)
        TIMED(e, st, "k_leader_prep",
              (k_leader_prep<32><<<blocks, 256, 0, st>>>(d1, in, R->sc, out, wp, wsg)));
      else if (dp.P == 16)
        TIMED(e, st, "k_leader_prep",
              (k_leader_prep<16><<<blocks, 256, 0, st>>>(d1, in, R->sc, out, wp, wsg)));
      else
        TIMED(e, st, "k_leader_prep",
              (k_leader_prep<8><<<blocks, 256, 0, st>>>(d1, in, R->sc, out, wp, wsg)));
      dp.redo = 1;
    } else {
      TIMED(e, st, "k_leader_jr",
            (k_leader_jr<<<blocks, 256, 0, st>>>(dp, in, R->sc, d_status, wp, wsg)));
    }
    TIMED(e, st, "k_leader_slowfix",
          (k_leader_slowfix<<<blocks64, 64, 0, st>>>(dp, in, R->sc)));
    if (dp.P == 32)
      TIMED(e, st, "k_query_h", (k_query_h<2, 32, 1><<<blocks, 256, 0, st>>>(dp, in, R->sc, out)));
    else if (dp.P == 16)
      TIMED(e, st, "k_query_h", (k_query_h<2, 16, 1><<<blocks, 256, 0, st>>>(dp, in, R->sc, out)));
    else
      TIMED(e, st, "k_query_h", (k_query_h<2, 8, 1><<<blocks, 256, 0, st>>>(dp, in, R->sc, out)));
    return PRIO3_OK;
  }
  if (dp.kind == PRIO3_SUM && e->leader_fast && query_sum_takes(dp)) {
    // Prio3Sum: the same unpack / joint-rand kernels, then k_query_sum in its leader role
    InPtrs in{d_nonces, d_public_shares, d_leader_input_shares, nullptr};
    in.vk_slot = vk_slot;
    in.vk_tab = vk_tab;
    OutPtrs out{d_prep_shares, d_status};
    const uint32_t blocks = (n + 255) / 256, blocks64 = (n + 63) / 64;
    // (k_leader_jr's per-lane row streaming loses here: the short share leaves little Keccak
    // to hide the 1.6 KB rows' uncoalesced reads -- 2.63 against 1.30 + 0.46 ms per 1.25 M)
    TIMED(e, st, "k_leader_unpack",
          (k_leader_unpack<<<(n + 63) / 64, 256, 0, st>>>(dp, in, R->sc, d_status, nullptr,
                                                         nullptr)));
    TIMED(e, st, "k_jrpart", (k_jrpart<false, true><<<blocks, 256, 0, st>>>(dp, in, R->sc)));
    TIMED(e, st, "k_leader_slowfix",
          (k_leader_slowfix<<<blocks64, 64, 0, st>>>(dp, in, R->sc)));
    bool ok = false;
    TIMED(e, st, "k_query_sum", (ok = launch_query_sum(dp, in, R->sc, out, st, true)));
    return ok ? PRIO3_OK : PRIO3_EDEVICE;
  }
  int rc2 = PRIO3_OK;
  TIMED(e, st, "k_leader_init",
        rc2 = launch_leader_init(dp, d_nonces, d_public_shares, d_leader_input_shares, R->sc,
                                 d_prep_shares, d_status, st, vk_slot, vk_tab));
  return rc2;
}

// ---- executor hooks (prio3_runtime.h) ----
int engine_device(const prio3_engine* e) { return e->device; }
int engine_exec_id(const prio3_engine* e) { return e->device * EXEC_LANES + e->lane; }

// Host-buffer jobs of a multi-GPU engine go whole to the member whose executor holds the fewest
// reports (all engines' jobs counted: tasks of one instance share the executors), equally loaded
// members taken round-robin.  No collective: each job's outputs come back from the GPU that ran
// it, and Janus merges the per-job aggregations at collection
// (/root/reference/aggregator/src/aggregator/aggregation_job_writer.rs:510 writes a random `ord`
// shard per job; aggregate_share.rs:55-96 sums the shards).
static prio3_engine* place(prio3_engine* e, uint32_t n) {
  prio3_engine* best = e;
  const size_t k = e->members.size();
  if (k > 1) {
    const uint32_t s0 = e->rr.fetch_add(1, std::memory_order_relaxed);
    uint64_t bl = UINT64_MAX;
    for (size_t i = 0; i < k; i++) {
      prio3_engine* m = e->members[(s0 + i) % k];
      const uint64_t l = exec_load(engine_exec_id(m));
      if (l < bl) {
        bl = l;
        best = m;
      }
    }
  }
  best->placed_jobs.fetch_add(1, std::memory_order_relaxed);
  best->placed_reports.fetch_add(n, std::memory_order_relaxed);
  return best;
}

void engine_vk(const prio3_engine* e, uint8_t out[16]) { memcpy(out, e->dp.vk, 16); }

static uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

// aggregating jobs start at a wave boundary where the XOF fuses the accumulate (their waves then
// hold one job's reports and fuse; the pad columns carry an out-of-range segment id)
uint32_t engine_job_align(const prio3_engine* e) { return fusable(e) ? 64u : 1u; }

uint64_t engine_group_key(const prio3_engine* e) {
  uint64_t h = 1469598103934665603ull;
  h = fnv(h, &e->params, sizeof e->params);
  h = fnv(h, &e->device, sizeof e->device);
  // every option that changes what a launch computes or records (an A/B set on one
  // engine must not silently run with the lead engine's options)
  const int opts[] = {e->force_slow, e->chunks, e->fuse_acc,           e->leader_fast,
                      e->leader_fuse_acc, e->fp_round, e->experimental_fpvec, e->force_generic,
                      e->timing, e->pair_max};
  h = fnv(h, opts, sizeof opts);
  h = fnv(h, &e->fp_sub_bytes, sizeof e->fp_sub_bytes);
  // XofHmacSha256Aes128 keys enter the kernels as HMAC midstates: one engine per launch; an
  // engine with coalescing off gets a key of its own for every call
  if (e->dp.kind == PRIO3_SUMVEC_F64_MP || !e->coalesce) {
    static std::atomic<uint64_t> solo{0};
    const uint64_t u[2] = {(uint64_t)(uintptr_t)e, e->coalesce ? 0 : ++solo};
    h = fnv(h, u, sizeof u);
  }
  return h;
}

uint64_t exec_job_key(const ExecJob* j) {
  uint64_t h = engine_group_key(j->e);
  if (j->opener) {  // sealed-input jobs: one keypair and ciphertext shape per launch
    const uint64_t u[4] = {0x5345414C4544ull, hpke_opener_key(j->opener), j->ct_stride,
                           (uint64_t)j->require_taskprov};
    h = fnv(h, u, sizeof u);
  }
  return h;
}

void engine_io_layout(const prio3_engine* e, uint32_t cap, IoLayout* L, const ExecJob* job) {
  const DevParams& d = e->dp;
  const bool sealed = job && job->opener;
  L->len[0] = 16;
  L->len[1] = d.public_share_len;
  L->len[2] = sealed ? 0 : d.helper_share_len;  // sealed: opened into the run on the device
  L->len[3] = d.prep_share_len;
  size_t off = 0;
  for (int f = 0; f < 4; f++) {
    L->off[f] = off;
    off += (L->len[f] * cap + 15) & ~(size_t)15;
  }
  L->slot_off = off;
  off += (2 * (size_t)cap + 15) & ~(size_t)15;
  L->tab_off = off;
  off += 16 * (size_t)exec_max_keys();
  L->msg_len = e->sz.prep_msg_len;
  L->msg_off = off;
  off += L->msg_len * cap;
  L->status_off = off;
  off += cap;
  // aggregating jobs (prio3_helper_prepare_aggregate_batch): group segment ids, accept bytes,
  // and up to max_seg aggregate shares (at most 16 MiB of them) + counts
  off = (off + 15) & ~(size_t)15;
  L->seg_off = off;
  off += (4 * (size_t)cap + 15) & ~(size_t)15;
  L->accept_off = off;
  off += (cap + 15) & ~(size_t)15;
  L->agg_len = (size_t)d.out_len * d.es;
  L->max_seg = (uint32_t)std::max<size_t>(1, std::min<size_t>(EXEC_MAX_SEGS,
                                                                ((size_t)16 << 20) / L->agg_len));
  L->agg_off = off;
  off += (L->agg_len * L->max_seg + 15) & ~(size_t)15;
  L->cnt_off = off;
  off += 8 * (size_t)L->max_seg;
  L->nenc = L->ct_stride = 0;
  if (sealed) {  // the ciphertexts and their AAD fields (report IDs and public shares above)
    auto up = [](size_t x) { return (x + 15) & ~(size_t)15; };
    L->nenc = (uint32_t)hpke_opener_nenc(job->opener);
    L->ct_stride = job->ct_stride;
    off = up(off);
    L->enc_off = off;
    off += up((size_t)L->nenc * cap);
    L->ct_off = off;
    off += up((size_t)L->ct_stride * cap);
    L->ctlen_off = off;
    off += up(4 * (size_t)cap);
    L->time_off = off;
    off += up(8 * (size_t)cap);
    L->tslot_off = off;
    off += up(2 * (size_t)cap);
    L->ttab_off = off;
    off += 32 * (size_t)HPKE_MAX_TASKS;
  }
  L->bytes = off;
}

static int fused_finish(prio3_engine* e, Run* R, const uint8_t* d_status, const uint32_t* seg,
                        const uint32_t* fix_seg, const uint8_t* d_accept_mask, uint32_t S,
                        uint8_t* d_agg_shares, uint64_t* d_counts, hipStream_t st);

#ifndef SEALED_EARLY_NEXT  // A/B builds: 0 = a sealed group's next group waits for its prepare
#define SEALED_EARLY_NEXT 1
#endif
// the group's "prepared" event (engine_group_prepared), recorded on its stream now
static void record_prep(GroupRun* gr, hipStream_t st) {
  if (hipEventCreateWithFlags(&gr->prep, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(gr->prep, st) != hipSuccess) {
    (void)hipGetLastError();
    if (gr->prep) (void)hipEventDestroy(gr->prep);
    gr->prep = nullptr;
  }
}

// Sealed-input groups: a report the open rejected (HPKE status 4 or 8) gets status 0x80 | that
// PrepareError, whatever its prepare computed on the zeroed share -- so the accumulate, which
// counts status 0 only, leaves it out, and the caller sees the error Janus records first.
__global__ __launch_bounds__(256) void k_hpke_merge(uint32_t n, const uint8_t* hs, uint8_t* status) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n && hs[i]) status[i] = (uint8_t)(0x80u | hs[i]);
}

// Group launch (host pull, the r03 form).  The kernels read each report's nonce, public share,
// helper share and verify-key slot straight from the pinned staging (mapped), and each lane of the
// fused XOF + query launch copies its own leader prep share, segment id and accept byte into the
// run during its XOF (xofd_body PULL), so the transfer runs under that group's own Keccak work at
// the rate the lanes pull (~35 GB/s, profiles/r04).  One pinned-staging H2D copy per field ahead
// of the prepare, without the overlap (the r02 form), left transfer and prepare in series
// (profiles/r03/r03e_jobs128_*.json: 21.5 M reports/s); SDMA copies of each group issued under the
// previous group's compute (r04 option group_dma) measured 19.5-30.8 against 32-40 M/s for the
// pull and were removed in r05.
int engine_group_issue(prio3_engine* lead, const GroupView& g, GroupRun* gr, bool own_queue) {
  *gr = GroupRun();
  gr->lead = lead;
  gr->jobs = g.jobs;
  DeviceGuard dg_(lead->device);
  HIPCHK(dg_.rc);
  hipStream_t st = own_queue ? ws_exec_stream_get(lead->device) : ws_stream_get(lead->device);
  if (!st) return PRIO3_EDEVICE;
  const bool mp = lead->dp.kind == PRIO3_SUMVEC_F64_MP;
  // aggregating jobs: the group's reports are accumulated per job segment in this launch (the
  // wave partials of the XOF where the instance fuses; waves that straddle two jobs and the
  // excluded reports go through the fix-up list)
  const bool agg = g.nseg > 0;
  const bool fuse = agg && fusable(lead);
  IoLayout L;
  if (g.L)
    L = *g.L;
  else
    engine_io_layout(lead, g.cap, &L);
  const bool sealed = L.ct_stride > 0 && g.opener;
  int rc = PRIO3_OK;
  Run* R = run_create(lead, g.n,
                      RUN_SCRATCH | RUN_IO | (agg ? (unsigned)RUN_AGG_IO : 0u) |
                          (fuse ? (unsigned)RUN_FUSED : 0u) | (sealed ? (unsigned)RUN_HPKE : 0u),
                      agg ? g.nseg : 0, g.n_keys, st, &rc, sealed ? L.ct_stride : 0);
  if (!R) {
    ws_exec_stream_put(lead->device, st);
    return rc;
  }
  auto fail = [&](int code) {
    (void)hipStreamSynchronize(st);
    run_release(R, st, true);
    if (gr->prep) (void)hipEventDestroy(gr->prep);
    *gr = GroupRun();
    ws_exec_stream_put(lead->device, st);
    return code;
  };
  const uint8_t* hd = g.stg_dev;
  InPtrs in{hd + L.off[0], L.len[1] ? hd + L.off[1] : nullptr, hd + L.off[2], R->leader};
  if (sealed) {
    // the helper's loop body from its first line (aggregator.rs:1847-1990): each report's input
    // share opened, decoded and checked into the run's helper-share buffer, which the prepare
    // below reads from HBM -- the plaintexts never cross PCIe
    HpkeGroupArgs a{};
    a.n = g.n;
    a.ct_stride = L.ct_stride;
    a.share_len = lead->dp.helper_share_len;
    a.pub_len = (uint32_t)L.len[1];
    a.require_taskprov = g.require_taskprov;
    a.enc = hd + L.enc_off;
    a.ct = hd + L.ct_off;
    a.ct_len = (const uint32_t*)(hd + L.ctlen_off);
    a.ids = hd + L.off[0];
    a.times = (const uint64_t*)(hd + L.time_off);
    a.pubs = L.len[1] ? hd + L.off[1] : nullptr;
    a.task_slot = (const uint16_t*)(hd + L.tslot_off);
    a.task_tab = (const uint32_t*)(hd + L.ttab_off);
    a.pt = R->hpt;
    a.shares = R->helper;
    a.status = R->hstatus;
    if (hpke_open_group_launch(g.opener, a, st) != PRIO3_OK) return fail(PRIO3_EDEVICE);
    in.helper = R->helper;
    // the executor may issue the next group as soon as this one's open is done: a group's open
    // (one X25519 ladder per lane, ~1 wave per SIMD on half the SIMDs at 31k reports) then runs
    // beside this group's prepare instead of after it
    if (SEALED_EARLY_NEXT) record_prep(gr, st);
  }
  if (!mp) {  // the slots and the key table are read from the staging by the XOF
    in.vk_slot = (const uint16_t*)(hd + L.slot_off);
    in.vk_tab = (const uint4*)(hd + L.tab_off);
  }
  if (agg) R->seg = (const uint32_t*)(hd + L.seg_off);  // the fused XOF's segment check
  // the leader prep shares (and the segment ids / accept bytes of the fix-up pass)
  PullRanges pr{};
  pr.src[0] = hd + L.off[3];
  pr.dst[0] = R->leader;
  pr.bytes[0] = L.len[3] * g.n;
  if (agg) {
    pr.src[1] = hd + L.seg_off;
    pr.dst[1] = (uint8_t*)R->gseg;
    pr.bytes[1] = 4 * (size_t)g.n;
    pr.src[2] = hd + L.accept_off;
    pr.dst[2] = R->gaccept;
    pr.bytes[2] = g.n;
  }
  OutPtrs out{R->msgs, R->status};
  rc = prepare_run(lead, R, in, out, st, fuse, false, &pr);
  if (agg) R->seg = R->gseg;
  if (rc) return fail(rc);
  if (sealed) {  // the open's rejections take precedence (aggregator.rs:1850-1990 before :2020)
    k_hpke_merge<<<(g.n + 255) / 256, 256, 0, st>>>(g.n, R->hstatus, R->status);
    if (hipGetLastError() != hipSuccess) return fail(PRIO3_EDEVICE);
  }
  // the executor may issue its next group once this group's prepare kernels are done
  if (!gr->prep) record_prep(gr, st);
  if (agg) {
    rc = fuse ? fused_finish(lead, R, R->status, R->gseg, R->gseg, R->gaccept, g.nseg, R->gagg,
                             (uint64_t*)R->gcnt, st)
              : run_accumulate(lead, R, 0, g.n, R->status, R->gseg, R->gaccept, g.nseg, R->gagg,
                               (uint64_t*)R->gcnt, st);
    if (rc) return fail(rc);
  }
  {  // the outputs go back by one copy launch writing the mapped staging
    uint8_t* sd = g.stg_dev;
    PullRanges o{};
    o.src[0] = R->status;
    o.dst[0] = sd + L.status_off;
    o.bytes[0] = g.n;
    if (L.msg_len) {
      o.src[1] = R->msgs;
      o.dst[1] = sd + L.msg_off;
      o.bytes[1] = L.msg_len * g.n;
    }
    if (agg) {
      o.src[2] = R->gagg;
      o.dst[2] = sd + L.agg_off;
      o.bytes[2] = L.agg_len * g.nseg;
      o.src[3] = (const uint8_t*)R->gcnt;
      o.dst[3] = sd + L.cnt_off;
      o.bytes[3] = 8 * (size_t)g.nseg;
    }
    const size_t tot = o.bytes[0] + o.bytes[1] + o.bytes[2] + o.bytes[3];
    const unsigned blocks = (unsigned)std::min<size_t>(256, (tot / 16 + 255) / 256 + 1);
    k_pull<<<blocks, 256, 0, st>>>(o);
    if (hipGetLastError() != hipSuccess) return fail(PRIO3_EDEVICE);
  }
  gr->st = st;
  gr->R = R;
  return PRIO3_OK;
}

// (declared above engine_group_issue)
// the launcher polls these instead of sleeping in hipStreamSynchronize: the group's jobs are woken
// as soon as their outputs land (the blocking wait added ~0.1 ms per group)
bool engine_group_prepared(const GroupRun& gr) {
  return gr.prep && hipEventQuery(gr.prep) == hipSuccess;
}
bool engine_group_done(const GroupRun& gr) { return hipStreamQuery(gr.st) != hipErrorNotReady; }

int engine_group_finish(GroupRun* gr, Run** run_out) {
  *run_out = nullptr;
  hipError_t q = hipStreamQuery(gr->st);
  if (q == hipErrorNotReady) q = hipStreamSynchronize(gr->st);
  if (gr->prep) (void)hipEventDestroy(gr->prep);
  gr->prep = nullptr;
  const int dev = gr->lead->device;
  if (q != hipSuccess) {
    (void)hipGetLastError();
    run_release(gr->R, gr->st, true);
    ws_exec_stream_put(dev, gr->st);
    return PRIO3_EDEVICE;
  }
  if (gr->lead->timing) collect_times(gr->lead, false);
  gr->R->refs.store(gr->jobs);
  *run_out = gr->R;
  ws_exec_stream_put(dev, gr->st);
  return PRIO3_OK;
}


// ---- accumulate-executor hooks (prio3_runtime.h) ----
uint32_t engine_acc_key(const AccJob* j) { return j->run->dp.es; }

size_t engine_acc_out_bytes(const AccJob* j) {
  const size_t agg = (size_t)j->run->dp.out_len * j->run->dp.es * j->nseg;
  return ((agg + 7) & ~(size_t)7) + 8 * (size_t)j->nseg;
}

void engine_acc_stage(AccJob* j, uint8_t* stg, const AccLayout& L) {
  const Run* R = j->run;
  const DevParams& d = R->dp;
  AccDesc& D = ((AccDesc*)(stg + L.desc_off))[j->slot];
  D.src = (const uint8_t*)(own_out(d) ? R->sc.out : R->sc.meas) + (size_t)d.es * j->c0;
  D.status = R->status + j->c0;
  D.ld = d.ld_out;
  D.n = j->n;
  D.nseg = j->nseg;
  D.out_len = d.out_len;
  D.flags = (j->seg ? 1u : 0u) | (j->accept ? 2u : 0u);
  D.seg_off = L.seg_off + 4 * (size_t)j->rep_off;
  D.acc_off = L.acc_off + j->rep_off;
  D.agg_off = L.out_off + j->out_off;
  const size_t agg = (size_t)d.out_len * d.es * j->nseg;
  D.cnt_off = D.agg_off + ((agg + 7) & ~(size_t)7);
  if (j->seg) memcpy(stg + D.seg_off, j->seg, 4 * (size_t)j->n);
  if (j->accept) memcpy(stg + D.acc_off, j->accept, j->n);
}

void engine_acc_unstage(AccJob* j, const uint8_t* stg, const AccLayout& L) {
  const DevParams& d = j->run->dp;
  const AccDesc& D = ((const AccDesc*)(stg + L.desc_off))[j->slot];
  memcpy(j->agg_out, stg + D.agg_off, (size_t)d.out_len * d.es * j->nseg);
  memcpy(j->counts_out, stg + D.cnt_off, 8 * (size_t)j->nseg);
}

int engine_acc_group(int device, int es, uint8_t* stg, const AccLayout& L, uint32_t n_jobs,
                     size_t out_bytes) {
  DeviceGuard dg_(device);
  HIPCHK(dg_.rc);
  PooledStream ps(device);
  hipStream_t st = ps.s;
  if (!st) return PRIO3_EDEVICE;
  int rc = PRIO3_OK;
  Slab* sl = ws_acquire(device, L.bytes, st, &rc);
  if (!sl) return rc;
  const AccDesc* D = (const AccDesc*)(stg + L.desc_off);
  uint32_t reps = 0, max_len = 0;
  for (uint32_t i = 0; i < n_jobs; i++) {
    reps = std::max(reps, (uint32_t)((D[i].acc_off - L.acc_off) + D[i].n));
    max_len = std::max(max_len, D[i].out_len);
  }
  uint8_t* b = sl->base;
  if (hipMemcpyAsync(b + L.desc_off, stg + L.desc_off, sizeof(AccDesc) * n_jobs,
                     hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(b + L.seg_off, stg + L.seg_off, 4 * (size_t)reps, hipMemcpyHostToDevice,
                     st) != hipSuccess ||
      hipMemcpyAsync(b + L.acc_off, stg + L.acc_off, reps, hipMemcpyHostToDevice, st) !=
          hipSuccess)
    rc = PRIO3_EDEVICE;
  if (rc == PRIO3_OK) {
    dim3 grid(max_len, n_jobs);
    if (es == 16)
      k_acc_multi<Fp128><<<grid, 256, 0, st>>>((const AccDesc*)(b + L.desc_off), b);
    else
      k_acc_multi<Fp64><<<grid, 256, 0, st>>>((const AccDesc*)(b + L.desc_off), b);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(stg + L.out_off, b + L.out_off, out_bytes, hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      rc = PRIO3_EDEVICE;
  }
  ws_release(sl, st);
  return rc;
}

// ---- leader-executor hooks (prio3_runtime.h) ----
// The leader groups take the TurboSHAKE instances; FPVec (sub-batched runs) and the multiproof
// instance (HMAC midstates per engine) keep one run per call.
static bool leader_coalescable(const prio3_engine* e) {
  return e->coalesce && e->dp.kind != PRIO3_FPVEC_BOUNDED_L2 && e->dp.kind != PRIO3_SUMVEC_F64_MP;
}

void engine_leader_layout(const prio3_engine* e, uint32_t cap, LeaderLayout* L) {
  const DevParams& d = e->dp;
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  L->len[0] = 16;
  L->len[1] = d.public_share_len;
  L->len[2] = d.leader_share_len;
  size_t off = 0;
  for (int f = 0; f < 3; f++) {
    L->off[f] = off;
    off += up(L->len[f] * cap);
  }
  L->slot_off = off;
  off += up(2 * (size_t)cap);
  L->tab_off = off;
  off += up(16 * (size_t)exec_max_keys());
  L->ps_len = d.prep_share_len;
  L->ps_off = off;
  off += up(L->ps_len * cap);
  L->status_off = off;
  off += up(cap);
  L->bytes = off;
  L->cap = cap;
  // The executor's leader groups stage the input shares as plain rows, one DMA copies them into
  // the run, and the next group is issued as soon as that copy is done, so its copy runs under this
  // group's kernels.  Interleaved on one box (r06ai): 9.24 / 8.57 / 8.76 M reports/s against
  // 6.97 / 7.31 / 7.58 for the transposed staging read in-kernel (r06), whose
  // host-side transpose (~870 us of CPU per 500-report job) ran the process into the box's 16-CPU
  // quota.  JANUS_LEADER_SOA=1 (A/B): the transposed form.
  static const bool soa = [] {
    const char* v = getenv("JANUS_LEADER_SOA");
    return v && atoi(v) != 0;
  }();
  L->lin_soa = leader_prep_takes(e) && soa;
}

// A leader group: the explicit input shares (5.6 KB per Histogram(256) report) go to the run by
// one DMA, the kernels read the nonces, public shares and verify-key slots from the mapped
// staging, and one copy launch writes the prepare shares and statuses back into it.
#ifndef LEADER_OUT_DMA  // A/B builds: 0 = the prepare shares back by the k_pull copy kernel
#define LEADER_OUT_DMA 1
#endif
int engine_leader_issue(prio3_engine* lead, const LeaderLayout& L, uint8_t* stg, uint8_t* stg_dev,
                        uint32_t n, uint32_t n_keys, int jobs, GroupRun* gr, bool own_queue) {
  (void)n_keys;
  *gr = GroupRun();
  gr->lead = lead;
  gr->jobs = jobs;
  DeviceGuard dg_(lead->device);
  HIPCHK(dg_.rc);
  hipStream_t st = own_queue ? ws_exec_stream_get(lead->device) : ws_stream_get(lead->device);
  if (!st) return PRIO3_EDEVICE;
  int rc = PRIO3_OK;
  Run* R = run_create(lead, n, RUN_SCRATCH | RUN_IO | RUN_LINPUT, 0, 0, st, &rc);
  if (!R) {
    ws_exec_stream_put(lead->device, st);
    return rc;
  }
  auto fail = [&](int code) {
    (void)hipStreamSynchronize(st);
    run_release(R, st, true);
    if (gr->prep) (void)hipEventDestroy(gr->prep);
    *gr = GroupRun();
    ws_exec_stream_put(lead->device, st);
    return code;
  };
  // The input shares (5.6 KB per Histogram(256) report) go to the run by one DMA, and the kernels
  // read AoS rows from HBM.  r05 issued the next group only after this group's kernels, so copy
  // and kernels ran in series; now the group's 'prepared' event follows the copy (below).  With
  // lin_soa (A/B) k_leader_prep reads the transposed staging itself instead, each wave load one
  // 1 KiB PCIe read, and the other leader kernels read AoS rows from the run.
  if (!L.lin_soa &&
      hipMemcpyAsync(R->linput, stg_dev + L.off[2], L.len[2] * n, hipMemcpyDefault, st) !=
          hipSuccess)
    return fail(PRIO3_EDEVICE);
  // the DMA form: the executor may issue its next group once this group's shares are in HBM, so
  // the next group's copy runs under this group's kernels (as a sealed group's next goes after
  // its open)
  if (!L.lin_soa) record_prep(gr, st);
  rc = leader_init_run(lead, R, stg_dev + L.off[0], L.len[1] ? stg_dev + L.off[1] : nullptr,
                       L.lin_soa ? stg_dev + L.off[2] : R->linput, R->leader, R->status, st,
                       (const uint16_t*)(stg_dev + L.slot_off), (const uint4*)(stg_dev + L.tab_off),
                       L.lin_soa ? L.cap : 0u);
  if (rc) return fail(rc);
  if (!gr->prep) record_prep(gr, st);
  // the prepare shares (560 B per Histogram(256) report, 17 MB per 31k group) go back by the
  // copy engine: written by k_pull into the mapped staging they took 0.88 ms per group (~20 GB/s,
  // r06c kernel trace); the statuses by the copy kernel
  PullRanges o{};
  o.src[0] = R->status;
  o.dst[0] = stg_dev + L.status_off;
  o.bytes[0] = n;
  if (LEADER_OUT_DMA) {
    if (hipMemcpyAsync(stg + L.ps_off, R->leader, L.ps_len * n, hipMemcpyDeviceToHost, st) !=
        hipSuccess)
      return fail(PRIO3_EDEVICE);
  } else {
    o.src[1] = R->leader;
    o.dst[1] = stg_dev + L.ps_off;
    o.bytes[1] = L.ps_len * n;
  }
  const size_t tot = o.bytes[0] + o.bytes[1];
  k_pull<<<(unsigned)std::min<size_t>(256, (tot / 16 + 255) / 256 + 1), 256, 0, st>>>(o);
  if (hipGetLastError() != hipSuccess) return fail(PRIO3_EDEVICE);
  gr->st = st;
  gr->R = R;
  return PRIO3_OK;
}

uint32_t engine_lnext_key(const LNextJob* j) { return j->run->dp.es; }

void engine_lnext_stage(LNextJob* j, uint8_t* stg, const LNextLayout& L) {
  const Run* R = j->run;
  const DevParams& d = R->dp;
  const size_t es = d.es;
  LNextDesc& D = ((LNextDesc*)(stg + L.desc_off))[j->slot];
  D.corrected = R->sc.corrected + j->c0;
  D.meas = (const uint8_t*)R->sc.meas + es * j->c0;
  D.out = own_out(d) ? (uint8_t*)R->sc.out + es * j->c0 : nullptr;
  D.dstatus = R->status + j->c0;
  D.ld = d.ld;
  D.n = j->n;
  D.rep_off = j->rep_off;
  D.kind = d.kind;
  D.bits = d.bits;
  D.out_len = d.out_len;
  D.jr = d.jr_len ? 1u : 0u;
  if (D.jr && j->msgs) memcpy(stg + L.msg_off + 16 * (size_t)j->rep_off, j->msgs, 16 * (size_t)j->n);
  memcpy(stg + L.status_off + j->rep_off, j->status, j->n);
  if (j->nseg) {  // its accumulate descriptor (offsets from the accumulate area's base)
    const AccLayout& A = L.acc;
    uint8_t* base = stg + L.acc_base;
    AccDesc& X = ((AccDesc*)(base + A.desc_off))[j->acc_slot];
    X.src = (const uint8_t*)(own_out(d) ? R->sc.out : R->sc.meas) + es * j->c0;
    X.status = R->status + j->c0;  // the device verdicts, after the check of the same launch
    X.ld = d.ld_out;
    X.n = j->n;
    X.nseg = j->nseg;
    X.out_len = d.out_len;
    X.flags = (j->seg ? 1u : 0u) | (j->accept ? 2u : 0u);
    X.seg_off = A.seg_off + 4 * (size_t)j->rep_off;
    X.acc_off = A.acc_off + j->rep_off;
    X.agg_off = A.out_off + j->out_off;
    const size_t agg = (size_t)d.out_len * es * j->nseg;
    X.cnt_off = X.agg_off + ((agg + 7) & ~(size_t)7);
    if (j->seg) memcpy(base + X.seg_off, j->seg, 4 * (size_t)j->n);
    if (j->accept) memcpy(base + X.acc_off, j->accept, j->n);
  }
}

size_t engine_lnext_out_bytes(const LNextJob* j) {
  if (!j->nseg) return 0;
  const size_t agg = (size_t)j->run->dp.out_len * j->run->dp.es * j->nseg;
  return ((agg + 7) & ~(size_t)7) + 8 * (size_t)j->nseg;
}

void engine_lnext_unstage(LNextJob* j, const uint8_t* stg, const LNextLayout& L) {
  memcpy(j->status, stg + L.status_off + j->rep_off, j->n);
  if (!j->nseg) return;
  const DevParams& d = j->run->dp;
  const uint8_t* base = stg + L.acc_base;
  const AccDesc& X = ((const AccDesc*)(base + L.acc.desc_off))[j->acc_slot];
  memcpy(j->agg_out, base + X.agg_off, (size_t)d.out_len * d.es * j->nseg);
  memcpy(j->counts_out, base + X.cnt_off, 8 * (size_t)j->nseg);
}

extern "C" int launch_leader_next_multi(uint32_t es, const LNextDesc* d_desc, const uint8_t* d_msgs,
                                        uint8_t* d_status, uint32_t n_jobs, uint32_t max_n,
                                        hipStream_t st);

int engine_lnext_issue(int device, uint32_t es, uint8_t* stg, uint8_t* stg_dev,
                       const LNextLayout& L, uint32_t n_jobs, uint32_t max_n, uint32_t n_acc,
                       size_t out_bytes, hipStream_t* st_out, Slab** slab_out, bool own_queue) {
  *st_out = nullptr;
  *slab_out = nullptr;
  DeviceGuard dg_(device);
  HIPCHK(dg_.rc);
  hipStream_t st = own_queue ? ws_exec_stream_get(device) : ws_stream_get(device);
  if (!st) return PRIO3_EDEVICE;
  int rc = launch_leader_next_multi(es, (const LNextDesc*)(stg_dev + L.desc_off),
                                    stg_dev + L.msg_off, stg_dev + L.status_off, n_jobs, max_n, st);
  Slab* sl = nullptr;
  if (rc == PRIO3_OK && n_acc) {
    // the aggregating jobs' accumulate (leader_continued's output shares merged by the writer,
    // aggregation_job_writer.rs:591-695) on the same stream: descriptors, segment ids and accept
    // bytes into a device area, k_acc_multi, the aggregate shares and counts back into the staging
    const AccLayout& A = L.acc;
    uint8_t* host = stg + L.acc_base;  // the accumulate area as the host sees it
    const AccDesc* D = (const AccDesc*)(host + A.desc_off);
    uint32_t reps = 0, max_len = 0;
    for (uint32_t i = 0; i < n_acc; i++) {
      reps = std::max(reps, (uint32_t)((D[i].acc_off - A.acc_off) + D[i].n));
      max_len = std::max(max_len, D[i].out_len);
    }
    sl = ws_acquire(device, A.bytes, st, &rc);
    if (sl) {
      uint8_t* b = sl->base;
      if (hipMemcpyAsync(b + A.desc_off, host + A.desc_off, sizeof(AccDesc) * n_acc,
                         hipMemcpyHostToDevice, st) != hipSuccess ||
          hipMemcpyAsync(b + A.seg_off, host + A.seg_off, 4 * (size_t)reps, hipMemcpyHostToDevice,
                         st) != hipSuccess ||
          hipMemcpyAsync(b + A.acc_off, host + A.acc_off, reps, hipMemcpyHostToDevice, st) !=
              hipSuccess) {
        rc = PRIO3_EDEVICE;
      } else {
        dim3 grid(max_len, n_acc);
        if (es == 16)
          k_acc_multi<Fp128><<<grid, 256, 0, st>>>((const AccDesc*)(b + A.desc_off), b);
        else
          k_acc_multi<Fp64><<<grid, 256, 0, st>>>((const AccDesc*)(b + A.desc_off), b);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(host + A.out_off, b + A.out_off, out_bytes, hipMemcpyDeviceToHost,
                           st) != hipSuccess)
          rc = PRIO3_EDEVICE;
      }
    }
  }
  if (rc != PRIO3_OK) {
    (void)hipStreamSynchronize(st);
    if (sl) ws_release(sl, st);
    ws_exec_stream_put(device, st);
    return rc;
  }
  *st_out = st;
  *slab_out = sl;
  return PRIO3_OK;
}

extern "C" {

// A blocking host-to-device copy on a pooled non-blocking stream: a synchronous hipMemcpy runs on
// the legacy null stream, which waits for every blocking stream of the device -- the executor's
// CU-masked group streams are such streams -- so an engine created while another
// task's groups run would wait for them.
static int upload_blocking(int device, void* dst, const void* src, size_t bytes) {
  hipStream_t st = ws_stream_get(device);
  if (!st) return PRIO3_EDEVICE;
  const bool ok = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
                  hipStreamSynchronize(st) == hipSuccess;
  ws_stream_put(device, st);
  if (!ok) (void)hipGetLastError();
  return ok ? PRIO3_OK : PRIO3_EDEVICE;
}

int prio3_sizes(const prio3_params* params, prio3_sizes_t* out) {
  return fill_sizes(params, out, nullptr);
}

int prio3_engine_create_ex(const prio3_params* params, const uint8_t* verify_key,
                           size_t verify_key_len, int device, prio3_engine** out) {
  if (!params || !verify_key || !out) return PRIO3_EINVAL;
  const bool mp = params->kind == PRIO3_SUMVEC_F64_MP;
  if (verify_key_len != (mp ? 32u : 16u)) return PRIO3_EINVAL;
  prio3_engine* e = new prio3_engine();
  int rc = fill_sizes(params, &e->sz, &e->dp);
  if (rc) {
    delete e;
    return rc;
  }
  e->params = *params;
  if (!mp) memcpy(e->dp.vk, verify_key, 16);
  e->device = device;
  if (hipDeviceGetAttribute(&e->n_cu, hipDeviceAttributeMultiprocessorCount, device) !=
          hipSuccess ||
      e->n_cu <= 0)
    e->n_cu = 256;
  hipStream_t probe = nullptr;  // a GPU must be present: the product path has no CPU fallback
  DeviceGuard dg_(device);
  if (dg_.rc != hipSuccess ||
      hipStreamCreateWithFlags(&probe, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    delete e;
    return PRIO3_EDEVICE;
  }
  ws_stream_put(device, probe);  // the first member of the GPU's stream pool
  ws_warm(device);               // the rest of it, before any job runs
  const bool fpv = e->dp.kind == PRIO3_FPVEC_BOUNDED_L2;
  if (((e->dp.kind == PRIO3_HISTOGRAM || e->dp.kind == PRIO3_SUMVEC) &&
       (e->dp.P == 32 || e->dp.P == 64 || e->dp.P == 128)) ||
      (fpv && e->dp.logP <= 10 && e->dp.logP1 <= 10)) {
    // k_query_w / k_query_fpw: sigma_e = sum_(c=1..calls) alpha_P^(ce), e < P -- the weights of
    // sum_c p(alpha^c) over the polynomial's coefficients (FPVec: gadget 0's table, then gadget
    // 1's)
    const DevParams& d = e->dp;
    std::vector<uint4> sig;
    auto table = [&](uint32_t logP, uint32_t calls) {
      u128 alpha = 0;
      for (int k = 0; k < 4; k++) alpha |= (u128)d.roots128[logP][k] << (32 * k);
      for (uint32_t e2 = 0; e2 < (1u << logP); e2++) {
        const u128 ae = hpow(alpha, e2, HP128);
        u128 s = 0, x = 1;
        for (uint32_t c = 1; c <= calls; c++) {
          x = hmul(x, ae, HP128);
          s += x;
          if (s < x || s >= HP128) s -= HP128;
        }
        sig.push_back(make_uint4((uint32_t)s, (uint32_t)(s >> 32), (uint32_t)(s >> 64),
                                 (uint32_t)(s >> 96)));
      }
    };
    table(d.logP, d.calls);
    if (fpv) table(d.logP1, d.calls1);
    if (hipMalloc((void**)&e->d_sigma128, sizeof(uint4) * sig.size()) != hipSuccess ||
        upload_blocking(device, e->d_sigma128, sig.data(), sizeof(uint4) * sig.size()) !=
            PRIO3_OK) {
      delete e;
      return PRIO3_EDEVICE;
    }
    e->dp.sigma_dev = e->d_sigma128;
  }
  if (mp) {  // prio3_mp64.hip constants
    const DevParams& d = e->dp;
    Mp64Params& m = e->mp;
    m.meas_len = d.meas_len;
    m.out_len = d.out_len;
    m.bits = params->bits;
    m.chunk = params->chunk_length;
    m.calls = d.calls;
    m.P = d.P;
    m.logP = d.logP;
    m.glen = d.glen;
    m.np = params->num_proofs;
    m.proof_len = d.proof_len / m.np;
    m.arity = d.arity;
    m.vlen = d.verifier_len;
    memcpy(m.dst, d.dst, sizeof m.dst);
    hmac_midstates_host(verify_key, 32, m.vk_ist, m.vk_ost);
    static const uint8_t zero32[32] = {0};
    hmac_midstates_host(zero32, 32, m.z_ist, m.z_ost);
    const u128 alpha = d.roots64[d.logP];
    m.alpha = (uint64_t)alpha;
    m.alpha_inv = (uint64_t)hpow(alpha, d.P - 1, HP64);
    m.invP = d.invP64;
    m.half = d.half64;
    std::vector<uint64_t> sig(d.P);
    for (uint32_t e2 = 0; e2 < d.P; e2++) {
      const u128 ae = hpow(alpha, e2, HP64);
      u128 sum = 0, x = 1;
      for (uint32_t c = 1; c <= d.calls; c++) {
        x = hmul(x, ae, HP64);
        sum = (sum + x) % HP64;
      }
      sig[e2] = (uint64_t)sum;
    }
    if (hipMalloc((void**)&e->d_sigma64, 8 * (size_t)d.P) != hipSuccess ||
        upload_blocking(device, e->d_sigma64, sig.data(), 8 * (size_t)d.P) != PRIO3_OK) {
      delete e;
      return PRIO3_EDEVICE;
    }
    m.sigma = e->d_sigma64;
  }
  *out = e;
  return PRIO3_OK;
}

int prio3_engine_create(const prio3_params* params, const uint8_t verify_key[16], int device,
                        prio3_engine** out) {
  return prio3_engine_create_ex(params, verify_key, 16, device, out);
}

int prio3_engine_create_devices(const prio3_params* params, const uint8_t* verify_key,
                                size_t verify_key_len, const int* devices, uint32_t n_devices,
                                prio3_engine** out) {
  if (!out || !devices || n_devices == 0 || n_devices > (uint32_t)EXEC_LANES * 64)
    return PRIO3_EINVAL;
  *out = nullptr;
  std::vector<prio3_engine*> ms;
  for (uint32_t i = 0; i < n_devices; i++) {
    // the lane of a GPU named again: its own executor (a one-GPU rehearsal of the placement)
    int lane = 0;
    for (uint32_t j = 0; j < i; j++) lane += devices[j] == devices[i];
    prio3_engine* m = nullptr;
    const int rc = lane < EXEC_LANES
                       ? prio3_engine_create_ex(params, verify_key, verify_key_len, devices[i], &m)
                       : PRIO3_EINVAL;
    if (rc != PRIO3_OK) {
      for (auto x : ms) prio3_engine_destroy(x);
      return rc;
    }
    m->lane = lane;
    ms.push_back(m);
  }
  prio3_engine* e = ms[0];
  if (ms.size() > 1) {
    e->members = ms;
    for (size_t i = 1; i < ms.size(); i++) ms[i]->owner = e;
  }
  *out = e;
  return PRIO3_OK;
}

int prio3_engine_create_mask(const prio3_params* params, const uint8_t* verify_key,
                             size_t verify_key_len, int device_mask, prio3_engine** out) {
  std::vector<int> devs;
  for (int d = 0; d < 31; d++)
    if (device_mask & (1 << d)) devs.push_back(d);
  if (device_mask <= 0 || devs.empty()) return PRIO3_EINVAL;
  return prio3_engine_create_devices(params, verify_key, verify_key_len, devs.data(),
                                     (uint32_t)devs.size(), out);
}

int prio3_engine_members(const prio3_engine* e, prio3_member_info* out, uint32_t cap) {
  if (!e) return PRIO3_EINVAL;
  const uint32_t k = e->members.empty() ? 1u : (uint32_t)e->members.size();
  for (uint32_t i = 0; i < k && i < cap && out; i++) {
    const prio3_engine* m = e->members.empty() ? e : e->members[i];
    prio3_member_info& x = out[i];
    x.device = m->device;
    x.lane = (uint32_t)m->lane;
    x.jobs = m->placed_jobs.load();
    x.reports = m->placed_reports.load();
    ExecStats st;
    if (exec_stats(EXEC_PREP, engine_exec_id(m), &st) != PRIO3_OK) st = ExecStats();
    x.exec_jobs = st.jobs;
    x.exec_groups = st.groups;
  }
  return (int)k;
}

int prio3_executor_stats_get(const prio3_engine* e, uint32_t member, int kind,
                             prio3_executor_stats* out) {
  if (!e || !out || kind < 0 || kind >= EXEC_KINDS) return PRIO3_EINVAL;
  const size_t k = e->members.empty() ? 1 : e->members.size();
  if (member >= k) return PRIO3_EINVAL;
  const prio3_engine* m = e->members.empty() ? e : e->members[member];
  const bool per_gpu = kind == EXEC_ACC || kind == EXEC_LNEXT;
  ExecStats st;
  const int rc = exec_stats(kind, per_gpu ? m->device * EXEC_LANES : engine_exec_id(m), &st);
  if (rc != PRIO3_OK) return rc;
  out->jobs = st.jobs;
  out->reports = st.reports;
  out->groups = st.groups;
  out->active_jobs = st.active_jobs;
  out->active_reports = st.active_reports;
  return PRIO3_OK;
}

int prio3_executor_control(prio3_engine* e, int which, const char* key, int64_t value) {
  if (!e || !key || which < -1 || which >= EXEC_KINDS) return PRIO3_EINVAL;
  const size_t k = e->members.empty() ? 1 : e->members.size();
  for (size_t i = 0; i < k; i++) {
    const prio3_engine* m = e->members.empty() ? e : e->members[i];
    for (int kind : {(int)EXEC_PREP, (int)EXEC_ACC, (int)EXEC_LEADER, (int)EXEC_LNEXT}) {
      if (which >= 0 && kind != which) continue;
      // the accumulate and prepare_next executors are one per GPU (lane 0)
      const bool per_gpu = kind == EXEC_ACC || kind == EXEC_LNEXT;
      const int id = per_gpu ? m->device * EXEC_LANES : engine_exec_id(m);
      const int rc = exec_control(kind, id, key, value);
      if (rc != PRIO3_OK) return rc;
    }
  }
  return PRIO3_OK;
}

void prio3_engine_destroy(prio3_engine* e) {
  if (!e) return;
  for (size_t i = 1; i < e->members.size(); i++) prio3_engine_destroy(e->members[i]);
  e->members.clear();
  DeviceGuard dg_(e->device);
  (void)hipDeviceSynchronize();
  {
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->cur) run_release(e->cur, nullptr, true);
    e->cur = nullptr;
  }
  collect_times(e);
  if (e->d_sigma64) (void)hipFree(e->d_sigma64);
  if (e->d_sigma128) (void)hipFree(e->d_sigma128);
  for (auto s2 : e->side) (void)hipStreamDestroy(s2);
  for (auto j : e->side_ev) (void)hipEventDestroy(j);
  if (e->fork_ev) (void)hipEventDestroy(e->fork_ev);
  delete e;
}

int prio3_engine_set_option(prio3_engine* e, const char* key, int64_t value) {
  if (!e || !key) return PRIO3_EINVAL;
  for (size_t i = 1; i < e->members.size(); i++) {  // a multi-GPU engine: every member alike
    const int rc = prio3_engine_set_option(e->members[i], key, value);
    if (rc != PRIO3_OK) return rc;
  }
  struct {
    const char* name;
    int* field;
  } ints[] = {{"force_slow_path", &e->force_slow}, {"chunks", &e->chunks},
              {"leader_fast", &e->leader_fast},    {"fuse_acc", &e->fuse_acc},
              {"fp_round", &e->fp_round},          {"timing", &e->timing},
              {"coalesce", &e->coalesce},          {"experimental_fpvec", &e->experimental_fpvec},
              {"leader_fuse_acc", &e->leader_fuse_acc},
              {"force_generic_query", &e->force_generic}, {"pair_max", &e->pair_max},
              {"keep_scratch", &e->keep_scratch}};
  for (auto& o : ints)
    if (!strcmp(key, o.name)) {
      *o.field = (int)value;
      return PRIO3_OK;
    }
  if (!strcmp(key, "fp_sub_bytes")) {  // FPVec scratch budget per sub-batch (0 = auto)
    if (value < 0) return PRIO3_EINVAL;
    e->fp_sub_bytes = value;
    return PRIO3_OK;
  }
  return PRIO3_EINVAL;
}

// ---- device-resident entry points ----
// A device-resident prepare replaces the engine's current run: the previous one is released
// (stream-ordered, so its slab can be reused by this very call) and this one stays until the
// next device-resident prepare -- "output shares remain until the next prio3_device_prepare".
static Run* device_run(prio3_engine* e, uint32_t n, unsigned flags, uint32_t nseg,
                       hipStream_t st, int* rc) {
  if (e->cur) run_release(e->cur, st, true);
  e->cur = run_create(e, n, flags, nseg, 0, st, rc);
  return e->cur;
}

int prio3_device_prepare(prio3_engine* e, uint32_t n, const uint8_t* d_nonces,
                         const uint8_t* d_public_shares, const uint8_t* d_helper_shares,
                         const uint8_t* d_leader_prep_shares, uint8_t* d_prep_msgs,
                         uint8_t* d_status, void* stream) {
  TraceSpan span_("VDAF preparation");
  if (!e) return PRIO3_EINVAL;
  if (e->dp.kind == PRIO3_FPVEC_BOUNDED_L2 && !e->experimental_fpvec)
    return PRIO3_EUNSUPPORTED;  // unpinned reconstruction: explicit opt-in only
  if (n == 0) return PRIO3_OK;
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  int rc = PRIO3_OK;
  Run* R = device_run(e, n, RUN_SCRATCH, 0, st, &rc);
  if (!R) return rc;
  InPtrs in{d_nonces, d_public_shares, d_helper_shares, d_leader_prep_shares};
  return prepare_run(e, R, in, OutPtrs{d_prep_msgs, d_status}, st, false, true);
}

// The aggregate from the run's wave partials: k_agg_waves (chunk partials), k_agg_fix (counts
// and the reports whose fused inclusion differs from their verdict), k_agg_final.  seg: the
// inclusion segment ids; fix_seg: the segment each fix-up entry applies to (nullptr: 0 -- the
// leader's partials are all summed for segment 0, so with one segment every fix-up, an
// out-of-range id included, is a correction of segment 0).
static int fused_finish(prio3_engine* e, Run* R, const uint8_t* d_status, const uint32_t* seg,
                        const uint32_t* fix_seg, const uint8_t* d_accept_mask, uint32_t S,
                        uint8_t* d_agg_shares, uint64_t* d_counts, hipStream_t st) {
  const uint32_t n = R->n, M = R->dp.meas_len, ws = R->wshift;
  const uint32_t nwaves = (n + (1u << ws) - 1) >> ws;
  {  // one zeroing launch for the three accumulators (three memsets were ~15 us per group, r03ag)
    ZeroRanges z{};
    z.dst[0] = (uint8_t*)R->agg64;
    z.bytes[0] = (size_t)S * M * 8 * 8;
    z.dst[1] = (uint8_t*)R->fix;
    z.bytes[1] = sizeof(uint32_t);
    z.dst[2] = (uint8_t*)d_counts;
    z.bytes[2] = 8 * (size_t)S;
    TIMED(e, st, "k_zero", (k_zero<<<std::min<uint32_t>(256, (uint32_t)((z.bytes[0] / 16 + 255) / 256) + 1), 256, 0, st>>>(z)));
  }
  const uint32_t nchunks = (nwaves + WCH - 1) / WCH;
  dim3 g1((M * 8 / 4 + 255) / 256, nchunks);  // 4 slots per thread (k_agg_waves)
  TIMED(e, st, "k_agg_waves",
        (k_agg_waves<<<g1, 256, 0, st>>>(nwaves, M, R->wpart, R->wseg, R->cpart, R->cseg,
                                         R->agg64)));
  TIMED(e, st, "k_agg_fix",
        (k_agg_fix<<<(n + fix_per(n) - 1) / fix_per(n), 256, 0, st>>>(
            n, d_status, seg, d_accept_mask, R->wseg, R->fix, (uint32_t)(R->fix_cap - 1), S,
            (unsigned long long*)d_counts, fix_seg ? 1u : 0u, fix_per(n), ws)));
  if (nchunks <= 64 && S > 1)
    TIMED(e, st, "k_agg_final",
          (k_agg_final_s<<<dim3((M + 31) / 32, S), 256, 0, st>>>(
              M, R->dp.ld, R->agg64, nchunks, R->cpart, R->cseg, R->fix, fix_seg, R->sc.meas,
              d_agg_shares)));
  else
    TIMED(e, st, "k_agg_final",
          (k_agg_final<<<S * M, 256, 0, st>>>(M, R->dp.ld, R->agg64, nchunks, R->cpart, R->cseg,
                                               R->fix, fix_seg, R->sc.meas, d_agg_shares)));
  return PRIO3_OK;
}

// Device leader init with the accumulate fused into k_leader_jr (option leader_fuse_acc):
// Histogram on the helper kernels' leader role, whose output share is the measurement share
// that k_leader_jr streams through anyway.
static bool leader_fuse_takes(const prio3_engine* e) {
  const DevParams& d = e->dp;
  return e->leader_fuse_acc && e->leader_fast && d.jr_len && d.kind == PRIO3_HISTOGRAM &&
         (d.P == 32 || d.P == 16 || d.P == 8) && !own_out(d) && d.es == 16;
}

int prio3_device_prepare_aggregate(prio3_engine* e, uint32_t n, const uint8_t* d_nonces,
                                   const uint8_t* d_public_shares, const uint8_t* d_helper_shares,
                                   const uint8_t* d_leader_prep_shares,
                                   const uint32_t* d_segment_ids, uint32_t n_segments,
                                   uint8_t* d_prep_msgs, uint8_t* d_status, void* stream) {
  TraceSpan span_("VDAF preparation + batch aggregation");
  if (!e || n_segments == 0) return PRIO3_EINVAL;
  if (e->dp.kind == PRIO3_FPVEC_BOUNDED_L2 && !e->experimental_fpvec)
    return PRIO3_EUNSUPPORTED;  // unpinned reconstruction: explicit opt-in only
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  const bool fuse = n > 0 && fusable(e);
  int rc = PRIO3_OK;
  Run* R = device_run(e, n, RUN_SCRATCH | (fuse ? (unsigned)RUN_FUSED : 0u), n_segments, st, &rc);
  if (!R) return rc;
  R->seg = d_segment_ids;
  R->aggregate = true;
  if (n == 0) return PRIO3_OK;
  InPtrs in{d_nonces, d_public_shares, d_helper_shares, d_leader_prep_shares};
  rc = prepare_run(e, R, in, OutPtrs{d_prep_msgs, d_status}, st, fuse, true);
  if (rc == PRIO3_OK) R->fused = fuse;
  return rc;
}

int prio3_device_aggregate_finish(prio3_engine* e, const uint8_t* d_status,
                                  const uint8_t* d_accept_mask, uint8_t* d_agg_shares,
                                  uint64_t* d_counts, void* stream) {
  TraceSpan span_("batch aggregation");
  if (!e) return PRIO3_EINVAL;
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  Run* R = e->cur;
  if (!R || !R->aggregate) return PRIO3_EINVAL;  // finish follows prio3_device_prepare_aggregate
  R->last = st;
  if (!R->fused)  // not fusable (or an empty batch): the one-pass segmented reduction
    return run_accumulate(e, R, 0, R->n, d_status, R->seg, d_accept_mask, R->nseg, d_agg_shares,
                          d_counts, st);
  return fused_finish(e, R, d_status, R->seg, R->seg, d_accept_mask, R->nseg, d_agg_shares,
                      d_counts, st);
}

int prio3_device_accumulate(prio3_engine* e, uint32_t n, const uint8_t* d_status,
                            const uint32_t* d_segment_ids, const uint8_t* d_accept_mask,
                            uint32_t n_segments, uint8_t* d_agg_shares, uint64_t* d_counts,
                            void* stream) {
  TraceSpan span_("batch aggregation");
  if (!e || n_segments == 0) return PRIO3_EINVAL;
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  const size_t agg_len = (size_t)e->dp.out_len * e->dp.es;
  if (n == 0) {
    HIPCHK(hipMemsetAsync(d_agg_shares, 0, agg_len * n_segments, st));
    HIPCHK(hipMemsetAsync(d_counts, 0, 8 * (size_t)n_segments, st));
    return PRIO3_OK;
  }
  Run* R = e->cur;
  if (!R || n > R->n) return PRIO3_EINVAL;
  if (R->lfused && n == R->n && n_segments == 1) {
    R->last = st;
    return fused_finish(e, R, d_status, d_segment_ids, nullptr, d_accept_mask, 1, d_agg_shares,
                        d_counts, st);
  }
  return run_accumulate(e, R, 0, n, d_status, d_segment_ids, d_accept_mask, n_segments,
                        d_agg_shares, d_counts, st);
}

int prio3_device_combine(prio3_engine* e, uint32_t k, uint32_t n_segments, const uint8_t* d_in,
                         const uint64_t* d_counts_in, uint8_t* d_out, uint64_t* d_counts_out,
                         void* stream) {
  TraceSpan span_("aggregate share combine");
  if (!e || k == 0 || n_segments == 0) return PRIO3_EINVAL;
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  const DevParams& d = e->dp;
  uint32_t len = d.out_len * n_segments;
  uint32_t threads = len > n_segments ? len : n_segments;
  if (d.es == 16)
    TIMED(e, st, "k_combine",
          (k_combine<Fp128><<<(threads + 255) / 256, 256, 0, st>>>(k, len, n_segments, d_in,
                                                                  d_counts_in, d_out,
                                                                  d_counts_out)));
  else
    TIMED(e, st, "k_combine",
          (k_combine<Fp64><<<(threads + 255) / 256, 256, 0, st>>>(k, len, n_segments, d_in,
                                                                 d_counts_in, d_out,
                                                                 d_counts_out)));
  return PRIO3_OK;
}

int prio3_device_batch_metadata(prio3_engine* e, uint32_t n, const uint8_t* d_report_ids,
                                const uint64_t* d_times, const uint8_t* d_status,
                                const uint8_t* d_accept_mask, const uint32_t* d_segment_ids,
                                uint32_t n_segments, uint8_t* d_checksums, uint64_t* d_intervals,
                                void* stream) {
  TraceSpan span_("batch aggregation metadata");
  if (!e || n_segments == 0 || (n && (!d_status || (d_checksums && !d_report_ids))))
    return PRIO3_EINVAL;
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  uint32_t* ck = (uint32_t*)d_checksums;
  unsigned long long* iv = (unsigned long long*)d_intervals;
  const uint32_t sb = (n_segments + 255) / 256;
  TIMED(e, st, "k_meta_init", (k_meta_init<<<sb, 256, 0, st>>>(n_segments, ck, iv)));
  if (n)
    TIMED(e, st, "k_meta",
          (k_meta<<<std::min((n + META_T - 1) / META_T, META_BLOCKS), META_T, 0, st>>>(
              n, d_report_ids, d_times, d_status,
                                                   d_accept_mask, d_segment_ids, n_segments, ck,
                                                   d_times ? iv : nullptr)));
  if (iv) TIMED(e, st, "k_meta_final", (k_meta_final<<<sb, 256, 0, st>>>(n_segments, iv)));
  return PRIO3_OK;
}

int prio3_device_combine_metadata(prio3_engine* e, uint32_t k, uint32_t n_segments,
                                  const uint8_t* d_checksums_in, const uint64_t* d_intervals_in,
                                  uint8_t* d_checksums_out, uint64_t* d_intervals_out,
                                  void* stream) {
  if (!e || k == 0 || n_segments == 0) return PRIO3_EINVAL;
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  TIMED(e, st, "k_combine_meta",
        (k_combine_meta<<<(n_segments * 8 + 255) / 256, 256, 0, st>>>(
            k, n_segments, (const uint32_t*)d_checksums_in,
            (const unsigned long long*)d_intervals_in, (uint32_t*)d_checksums_out,
            (unsigned long long*)d_intervals_out)));
  return PRIO3_OK;
}

int prio3_batch_metadata(prio3_engine* e, uint32_t n, const uint8_t* report_ids,
                         const uint64_t* times, const uint8_t* status, const uint8_t* accept_mask,
                         const uint32_t* segment_ids, uint32_t n_segments, uint8_t* checksums_out,
                         uint64_t* intervals_out) {
  if (!e || n_segments == 0 || (n && (!status || !report_ids))) return PRIO3_EINVAL;
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  PooledStream ps(e->device);
  hipStream_t st = ps.s;
  if (!st) return PRIO3_EDEVICE;
  const size_t N = n ? n : 1, S = n_segments;
  const size_t al = 256;
  auto up = [&](size_t b) { return (b + al - 1) / al * al; };
  const size_t o_ids = 0, o_st = o_ids + up(16 * N), o_t = o_st + up(N), o_mask = o_t + up(8 * N),
               o_seg = o_mask + up(N), o_ck = o_seg + up(4 * N), o_iv = o_ck + up(32 * S),
               total = o_iv + up(16 * S);
  int rc = PRIO3_OK;
  Slab* sl = ws_acquire(e->device, total, st, &rc);
  if (!sl) return rc;
  uint8_t* b = sl->base;
  auto h2d = [&](size_t off, const void* src, size_t bytes) {
    return !src || !bytes ||
           hipMemcpyAsync(b + off, src, bytes, hipMemcpyHostToDevice, st) == hipSuccess;
  };
  if (!h2d(o_ids, report_ids, 16 * (size_t)n) || !h2d(o_st, status, n) ||
      !h2d(o_t, times, 8 * (size_t)n) || !h2d(o_mask, accept_mask, n) ||
      !h2d(o_seg, segment_ids, 4 * (size_t)n))
    rc = PRIO3_EDEVICE;
  if (rc == PRIO3_OK)
    rc = prio3_device_batch_metadata(
        e, n, b + o_ids, times ? (const uint64_t*)(b + o_t) : nullptr, b + o_st,
        accept_mask ? b + o_mask : nullptr, segment_ids ? (const uint32_t*)(b + o_seg) : nullptr,
        n_segments, checksums_out ? b + o_ck : nullptr,
        intervals_out ? (uint64_t*)(b + o_iv) : nullptr, st);
  if (rc == PRIO3_OK &&
      ((checksums_out && hipMemcpyAsync(checksums_out, b + o_ck, 32 * S, hipMemcpyDeviceToHost,
                                        st) != hipSuccess) ||
       (intervals_out && hipMemcpyAsync(intervals_out, b + o_iv, 16 * S, hipMemcpyDeviceToHost,
                                        st) != hipSuccess) ||
       hipStreamSynchronize(st) != hipSuccess))
    rc = PRIO3_EDEVICE;
  if (e->timing) collect_times(e);
  ws_release(sl, st);
  return rc;
}

int prio3_device_output_shares(prio3_engine* e, uint32_t n, uint8_t* out) {
  if (!e || !out) return PRIO3_EINVAL;
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  Run* R = e->cur;
  if (!R || n > R->n) return PRIO3_EINVAL;
  HIPCHK(hipDeviceSynchronize());  // the run's work may sit on any caller stream
  PooledStream ps(e->device);
  if (!ps.s) return PRIO3_EDEVICE;
  return run_output_shares(R, 0, n, out, ps.s);
}

// ---- host-buffer entry points (what the Rust FFI calls from inside rayon::spawn) ----
// (e: the member the job was placed on)
static int helper_prepare_batch(prio3_engine* e, uint32_t n, const uint8_t* nonces,
                                const uint8_t* public_shares, const uint8_t* helper_shares,
                                const uint8_t* leader_prep_shares, uint8_t* prep_msgs_out,
                                uint8_t* status_out, prio3_batch** batch_out, bool placed) {
  if (!e || (n && (!nonces || !helper_shares || !leader_prep_shares || !status_out)))
    return PRIO3_EINVAL;
  if (e->dp.kind == PRIO3_FPVEC_BOUNDED_L2 && !e->experimental_fpvec)
    return PRIO3_EUNSUPPORTED;  // unpinned reconstruction: explicit opt-in only
  const DevParams& d = e->dp;
  if (n && d.jr_len && (!public_shares || !prep_msgs_out)) return PRIO3_EINVAL;
  if (n && !placed) e = place(e, n);
  if (n == 0) {
    if (batch_out) *batch_out = new prio3_batch{e, nullptr, 0, 0};
    return PRIO3_OK;
  }
  ExecJob job;
  job.e = e;
  job.n = n;
  job.nonces = nonces;
  job.pub = d.jr_len ? public_shares : nullptr;
  job.helper = helper_shares;
  job.leader = leader_prep_shares;
  job.msgs_out = prep_msgs_out;
  job.status_out = status_out;
  const int rc = exec_submit(&job);
  if (rc) return rc;
  if (batch_out)
    *batch_out = new prio3_batch{e, job.run, job.c0, n};
  else
    run_release(job.run, nullptr, false);
  return PRIO3_OK;
}

int prio3_helper_prepare_batch(prio3_engine* e, uint32_t n, const uint8_t* nonces,
                               const uint8_t* public_shares, const uint8_t* helper_shares,
                               const uint8_t* leader_prep_shares, uint8_t* prep_msgs_out,
                               uint8_t* status_out, prio3_batch** batch_out) {
  TraceSpan span_("handle_aggregate_init_generic threadpool task");
  return helper_prepare_batch(e, n, nonces, public_shares, helper_shares, leader_prep_shares,
                              prep_msgs_out, status_out, batch_out, false);
}

int prio3_helper_prepare_aggregate_batch(prio3_engine* e, uint32_t n, const uint8_t* nonces,
                                         const uint8_t* public_shares,
                                         const uint8_t* helper_shares,
                                         const uint8_t* leader_prep_shares,
                                         const uint32_t* segment_ids, const uint8_t* accept_mask,
                                         uint32_t n_segments, uint8_t* prep_msgs_out,
                                         uint8_t* status_out, uint8_t* agg_shares_out,
                                         uint64_t* counts_out) {
  TraceSpan span_("handle_aggregate_init_generic threadpool task");
  if (!e || n_segments == 0 || !agg_shares_out || !counts_out ||
      (n && (!nonces || !helper_shares || !leader_prep_shares || !status_out)))
    return PRIO3_EINVAL;
  if (e->dp.kind == PRIO3_FPVEC_BOUNDED_L2 && !e->experimental_fpvec)
    return PRIO3_EUNSUPPORTED;  // unpinned reconstruction: explicit opt-in only
  const DevParams& d = e->dp;
  if (n && d.jr_len && (!public_shares || !prep_msgs_out)) return PRIO3_EINVAL;
  if (n) e = place(e, n);
  const size_t agg_len = (size_t)d.out_len * d.es;
  IoLayout L1;
  engine_io_layout(e, 1, &L1);
  if (n == 0 || !e->coalesce || n_segments > L1.max_seg) {
    // not coalescable (or empty): the two calls, as the caller would make them
    prio3_batch* b = nullptr;
    int rc = helper_prepare_batch(e, n, nonces, public_shares, helper_shares,
                                  leader_prep_shares, prep_msgs_out, status_out, &b, true);
    if (rc == PRIO3_OK) rc = prio3_accumulate(b, segment_ids, accept_mask, n_segments,
                                              agg_shares_out, counts_out);
    prio3_batch_free(b);
    if (rc == PRIO3_OK && n == 0) {
      memset(agg_shares_out, 0, agg_len * n_segments);
      memset(counts_out, 0, 8 * (size_t)n_segments);
    }
    return rc;
  }
  ExecJob job;
  job.e = e;
  job.n = n;
  job.nonces = nonces;
  job.pub = d.jr_len ? public_shares : nullptr;
  job.helper = helper_shares;
  job.leader = leader_prep_shares;
  job.msgs_out = prep_msgs_out;
  job.status_out = status_out;
  job.seg = segment_ids;
  job.accept = accept_mask;
  job.nseg = n_segments;
  job.agg_out = agg_shares_out;
  job.counts_out = counts_out;
  const int rc = exec_submit(&job);
  if (rc) return rc;
  run_release(job.run, nullptr, false);  // no batch handle: the output shares are not kept
  return PRIO3_OK;
}

// The helper's whole per-report loop body over one job, from the sealed input shares
// (VdafOps::handle_aggregate_init_generic, /root/reference/aggregator/src/aggregator.rs:1794-2096:
// HPKE open :1847-1890, PlaintextInputShare decode and extension checks :1893-1983,
// helper_initialized + evaluate :2020-2042, then the writer's merge).  One job of the executor: the
// group's launch opens every report's input share into HBM, prepares the reports from there and
// accumulates them per segment; only statuses, prepare messages, aggregate shares and counts come
// back.  A group too wide for its segments takes the same steps as two host calls.
int prio3_helper_aggregate_init_batch(
    prio3_engine* e, janus_hpke_opener* opener, uint32_t n, const uint8_t task_id[32],
    int require_taskprov, const uint8_t* report_ids, const uint64_t* times,
    const uint8_t* public_shares, const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
    uint32_t ct_stride, const uint8_t* leader_prep_shares, const uint32_t* segment_ids,
    const uint8_t* accept_mask, uint32_t n_segments, uint8_t* prep_msgs_out, uint8_t* status_out,
    uint8_t* agg_shares_out, uint64_t* counts_out) {
  TraceSpan span_("handle_aggregate_init_generic threadpool task");
  if (!e || !opener || !task_id || n_segments == 0 || !agg_shares_out || !counts_out ||
      ct_stride == 0 || ct_stride % 16 != 0 ||
      (n && (!report_ids || !times || !enc || !ct || !ct_len || !leader_prep_shares ||
             !status_out)))
    return PRIO3_EINVAL;
  if (e->dp.kind == PRIO3_FPVEC_BOUNDED_L2 && !e->experimental_fpvec)
    return PRIO3_EUNSUPPORTED;  // unpinned reconstruction: explicit opt-in only
  const DevParams& d = e->dp;
  // the open kernel's AAD takes public shares of 0 or 32 bytes (every TurboSHAKE instance)
  if (d.public_share_len != 0 && d.public_share_len != 32) return PRIO3_EUNSUPPORTED;
  if (n && d.jr_len && (!public_shares || !prep_msgs_out)) return PRIO3_EINVAL;
  const size_t agg_len = (size_t)d.out_len * d.es;
  if (n == 0) {
    memset(agg_shares_out, 0, agg_len * n_segments);
    memset(counts_out, 0, 8 * (size_t)n_segments);
    return PRIO3_OK;
  }
  e = place(e, n);
  IoLayout L1;
  engine_io_layout(e, 1, &L1);
  if (n_segments > L1.max_seg) {  // the open, then the prepare + aggregate of what it opened
    std::vector<uint8_t> shares((size_t)d.helper_share_len * n), hs(n), acc(n);
    int rc = janus_hpke_open_input_shares(opener, n, task_id, enc, ct, ct_len, ct_stride,
                                          report_ids, times, d.jr_len ? public_shares : nullptr,
                                          d.public_share_len, d.helper_share_len,
                                          require_taskprov, shares.data(), hs.data());
    if (rc) return rc == JANUS_HPKE_EDEVICE ? PRIO3_EDEVICE : PRIO3_EINVAL;
    for (uint32_t i = 0; i < n; i++) acc[i] = (!accept_mask || accept_mask[i]) && hs[i] == 0;
    rc = prio3_helper_prepare_aggregate_batch(e, n, report_ids, public_shares, shares.data(),
                                              leader_prep_shares, segment_ids, acc.data(),
                                              n_segments, prep_msgs_out, status_out,
                                              agg_shares_out, counts_out);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++)
      if (hs[i]) status_out[i] = (uint8_t)(0x80u | hs[i]);
    return PRIO3_OK;
  }
  ExecJob job;
  job.e = e;
  job.n = n;
  job.nonces = report_ids;
  job.pub = d.jr_len ? public_shares : nullptr;
  job.helper = nullptr;
  job.leader = leader_prep_shares;
  job.msgs_out = prep_msgs_out;
  job.status_out = status_out;
  job.seg = segment_ids;
  job.accept = accept_mask;
  job.nseg = n_segments;
  job.agg_out = agg_shares_out;
  job.counts_out = counts_out;
  job.opener = opener;
  job.task_id = task_id;
  job.times = times;
  job.enc = enc;
  job.ct = ct;
  job.ct_len = ct_len;
  job.ct_stride = ct_stride;
  job.require_taskprov = require_taskprov ? 1 : 0;
  const int rc = exec_submit(&job);
  if (rc) return rc;
  run_release(job.run, nullptr, false);
  return PRIO3_OK;
}

int prio3_accumulate(prio3_batch* b, const uint32_t* segment_ids, const uint8_t* accept_mask,
                     uint32_t n_segments, uint8_t* agg_shares_out, uint64_t* counts_out) {
  TraceSpan span_("batch aggregation");
  if (!b || !agg_shares_out || !counts_out || n_segments == 0) return PRIO3_EINVAL;
  prio3_engine* e = b->e;
  const size_t agg_len = (size_t)e->dp.out_len * e->dp.es, S = n_segments;
  if (!b->run || b->n == 0) {
    memset(agg_shares_out, 0, agg_len * S);
    memset(counts_out, 0, 8 * S);
    return PRIO3_OK;
  }
  Run* R = b->run;
  const uint32_t n = b->n;
  if (n <= (1u << 14) && e->coalesce) {  // a job-sized batch: coalesced with concurrent ones
    AccJob job;
    job.device = e->device;
    job.run = R;
    job.c0 = b->c0;
    job.n = n;
    job.seg = segment_ids;
    job.accept = accept_mask;
    job.nseg = n_segments;
    job.agg_out = agg_shares_out;
    job.counts_out = counts_out;
    if (engine_acc_out_bytes(&job) <= ((size_t)16 << 20)) return exec_accumulate(&job);
  }
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  PooledStream ps(e->device);
  hipStream_t st = ps.s;
  if (!st) return PRIO3_EDEVICE;
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_seg = 0, o_acc = up(4 * (size_t)n), o_agg = o_acc + up(n),
               o_cnt = o_agg + up(agg_len * S), total = o_cnt + up(8 * S);
  int rc = PRIO3_OK;
  Slab* sl = ws_acquire(e->device, total, st, &rc);
  if (!sl) return rc;
  uint8_t* base = sl->base;
  if ((segment_ids && hipMemcpyAsync(base + o_seg, segment_ids, 4 * (size_t)n,
                                     hipMemcpyHostToDevice, st) != hipSuccess) ||
      (accept_mask &&
       hipMemcpyAsync(base + o_acc, accept_mask, n, hipMemcpyHostToDevice, st) != hipSuccess))
    rc = PRIO3_EDEVICE;
  if (rc == PRIO3_OK)
    rc = run_accumulate(e, R, b->c0, n, R->status + b->c0,
                        segment_ids ? (const uint32_t*)(base + o_seg) : nullptr,
                        accept_mask ? base + o_acc : nullptr, n_segments, base + o_agg,
                        (uint64_t*)(base + o_cnt), st);
  if (rc == PRIO3_OK &&
      (hipMemcpyAsync(agg_shares_out, base + o_agg, agg_len * S, hipMemcpyDeviceToHost, st) !=
           hipSuccess ||
       hipMemcpyAsync(counts_out, base + o_cnt, 8 * S, hipMemcpyDeviceToHost, st) !=
           hipSuccess ||
       hipStreamSynchronize(st) != hipSuccess))
    rc = PRIO3_EDEVICE;
  if (e->timing) collect_times(e);
  ws_release(sl, st);
  return rc;
}

int prio3_debug_output_shares(prio3_batch* b, uint8_t* out) {
  if (!b || !out) return PRIO3_EINVAL;
  if (!b->run) return PRIO3_OK;
  DeviceGuard dg_(b->e->device);
  HIPCHK(dg_.rc);
  PooledStream ps(b->e->device);
  if (!ps.s) return PRIO3_EDEVICE;
  return run_output_shares(b->run, b->c0, b->n, out, ps.s);
}

void prio3_batch_free(prio3_batch* b) {
  if (!b) return;
  if (b->run) run_release(b->run, nullptr, false);
  delete b;
}

int prio3_engine_timing(prio3_engine* e, char* names, size_t cap_names, double* ms,
                        uint64_t* launches, int cap) {
  if (!e) return PRIO3_EINVAL;
  // a multi-GPU engine: its members' times, summed per kernel name
  std::vector<KTime> sum;
  const size_t nm = e->members.empty() ? 1 : e->members.size();
  for (size_t i = 0; i < nm; i++) {
    prio3_engine* m = e->members.empty() ? e : e->members[i];
    DeviceGuard dg_(m->device);
    collect_times(m);
    std::lock_guard<std::mutex> lk(m->tmu);
    for (auto& t : m->times) {
      size_t j = 0;
      while (j < sum.size() && sum[j].name != t.name) j++;
      if (j == sum.size()) sum.push_back(KTime{t.name, 0, 0});
      sum[j].ms += t.ms;
      sum[j].launches += t.launches;
    }
  }
  std::string all;
  int k = 0;
  for (auto& t : sum) {
    if (k < cap) {
      if (ms) ms[k] = t.ms;
      if (launches) launches[k] = t.launches;
    }
    if (!all.empty()) all += ",";
    all += t.name;
    k++;
  }
  if (names && cap_names) {
    strncpy(names, all.c_str(), cap_names - 1);
    names[cap_names - 1] = 0;
  }
  return k;
}

void prio3_engine_timing_reset(prio3_engine* e) {
  if (!e) return;
  for (size_t i = 1; i < e->members.size(); i++) prio3_engine_timing_reset(e->members[i]);
  collect_times(e);
  std::lock_guard<std::mutex> lk(e->tmu);
  for (auto& t : e->times) {
    t.ms = 0;
    t.launches = 0;
  }
}

// ---- leader side ----
int prio3_device_leader_prepare_init(prio3_engine* e, uint32_t n, const uint8_t* d_nonces,
                                     const uint8_t* d_public_shares,
                                     const uint8_t* d_leader_input_shares, uint8_t* d_prep_shares,
                                     uint8_t* d_status, void* stream) {
  TraceSpan span_("leader VDAF preparation");
  if (e && e->dp.kind == PRIO3_FPVEC_BOUNDED_L2 && !e->experimental_fpvec)
    return PRIO3_EUNSUPPORTED;  // FPVec: explicit opt-in
  if (!e) return PRIO3_EINVAL;
  if (n == 0) return PRIO3_OK;
  if (!d_nonces || !d_leader_input_shares || !d_prep_shares || !d_status ||
      (e->dp.jr_len && !d_public_shares))
    return PRIO3_EINVAL;
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  hipStream_t st = (hipStream_t)stream;
  int rc = PRIO3_OK;
  const bool lfuse = leader_fuse_takes(e);
  Run* R = device_run(e, n, RUN_SCRATCH | (lfuse ? (unsigned)RUN_FUSED : 0u), lfuse ? 1u : 0u, st,
                      &rc);
  if (!R) return rc;
  R->lfused = lfuse;
  return leader_init_run(e, R, d_nonces, d_public_shares, d_leader_input_shares, d_prep_shares,
                         d_status, st);
}

int prio3_device_leader_prepare_next(prio3_engine* e, uint32_t n, const uint8_t* d_prep_msgs,
                                     uint8_t* d_status, void* stream) {
  TraceSpan span_("leader VDAF preparation");
  if (e && e->dp.kind == PRIO3_FPVEC_BOUNDED_L2 && !e->experimental_fpvec)
    return PRIO3_EUNSUPPORTED;  // FPVec: explicit opt-in
  if (!e) return PRIO3_EINVAL;
  if (n == 0) return PRIO3_OK;
  if (!d_status || (e->dp.jr_len && !d_prep_msgs)) return PRIO3_EINVAL;
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  Run* R = e->cur;
  if (!R || n > R->n) return PRIO3_EINVAL;
  DevParams dp = R->dp;
  dp.n = n;
  hipStream_t st = (hipStream_t)stream;
  R->last = st;
  Scratch sc = R->sc;
  if (R->corr_all) sc.corrected = R->corr_all;  // FPVec: seeds of every sub-batch
  int rc2 = PRIO3_OK;
  if (dp.kind == PRIO3_SUMVEC_F64_MP)
    TIMED(e, st, "k_leader_next", rc2 = launch_mp64_leader_next(n, d_prep_msgs, sc, d_status, st));
  else
    TIMED(e, st, "k_leader_next", rc2 = launch_leader_next(dp, d_prep_msgs, sc, d_status, st));
  return rc2;
}

int prio3_leader_prepare_init_batch(prio3_engine* e, uint32_t n, const uint8_t* nonces,
                                    const uint8_t* public_shares,
                                    const uint8_t* leader_input_shares, uint8_t* prep_shares_out,
                                    uint8_t* status_out, prio3_batch** batch_out) {
  TraceSpan span_("leader VDAF preparation");
  if (e && e->dp.kind == PRIO3_FPVEC_BOUNDED_L2 && !e->experimental_fpvec)
    return PRIO3_EUNSUPPORTED;  // FPVec: explicit opt-in
  if (!e || (n && (!nonces || !leader_input_shares || !prep_shares_out || !status_out)))
    return PRIO3_EINVAL;
  const DevParams& d = e->dp;
  if (n && d.jr_len && !public_shares) return PRIO3_EINVAL;
  if (n == 0) {
    if (batch_out) *batch_out = new prio3_batch{e, nullptr, 0, 0};
    return PRIO3_OK;
  }
  e = place(e, n);
  if (leader_coalescable(e)) {  // concurrent jobs (of any task of the instance): one launch
    LeaderJob job{};
    job.e = e;
    job.n = n;
    job.nonces = nonces;
    job.pub = d.jr_len ? public_shares : nullptr;
    job.linput = leader_input_shares;
    job.prep_out = prep_shares_out;
    job.status_out = status_out;
    const int rc = exec_leader(&job);
    if (rc) return rc;
    if (batch_out)
      *batch_out = new prio3_batch{e, job.run, job.c0, n};
    else
      run_release(job.run, nullptr, false);
    return PRIO3_OK;
  }
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  PooledStream ps(e->device);
  hipStream_t st = ps.s;
  if (!st) return PRIO3_EDEVICE;
  int rc = PRIO3_OK;
  Run* R = run_create(e, n, RUN_SCRATCH | RUN_IO | RUN_LINPUT, 0, 0, st, &rc);
  if (!R) return rc;
  if (hipMemcpyAsync(R->nonces, nonces, 16 * (size_t)n, hipMemcpyHostToDevice, st) != hipSuccess ||
      (d.jr_len && hipMemcpyAsync(R->pub, public_shares, (size_t)d.public_share_len * n,
                                  hipMemcpyHostToDevice, st) != hipSuccess) ||
      hipMemcpyAsync(R->linput, leader_input_shares, (size_t)d.leader_share_len * n,
                     hipMemcpyHostToDevice, st) != hipSuccess)
    rc = PRIO3_EDEVICE;
  if (rc == PRIO3_OK)
    rc = leader_init_run(e, R, R->nonces, d.jr_len ? R->pub : nullptr, R->linput, R->leader,
                         R->status, st);
  if (rc == PRIO3_OK &&
      (hipMemcpyAsync(status_out, R->status, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
       hipMemcpyAsync(prep_shares_out, R->leader, (size_t)d.prep_share_len * n,
                      hipMemcpyDeviceToHost, st) != hipSuccess ||
       hipStreamSynchronize(st) != hipSuccess))
    rc = PRIO3_EDEVICE;
  if (e->timing) collect_times(e);
  if (rc != PRIO3_OK) {
    run_release(R, st, true);
    return rc;
  }
  if (batch_out)
    *batch_out = new prio3_batch{e, R, 0, n};
  else
    run_release(R, st, true);
  return PRIO3_OK;
}

int prio3_leader_prepare_next_batch(prio3_batch* b, const uint8_t* prep_msgs,
                                    uint8_t* status_inout) {
  TraceSpan span_("leader VDAF preparation");
  if (!b || !status_inout) return PRIO3_EINVAL;
  prio3_engine* e = b->e;
  const uint32_t n = b->n;
  const DevParams& d = e->dp;
  if (n == 0 || !b->run) return PRIO3_OK;
  if (d.jr_len && !prep_msgs) return PRIO3_EINVAL;
  Run* R = b->run;
  if (!R->msgs || !R->linput) return PRIO3_EINVAL;  // a leader batch
  const uint32_t c0 = b->c0;
  if (leader_coalescable(e) && n <= LNEXT_MAX_REPS) {
    // concurrent jobs' prepare_next (of any runs of this GPU) in one launch
    LNextJob job;
    job.device = e->device;
    job.run = R;
    job.c0 = c0;
    job.n = n;
    job.msgs = d.jr_len ? prep_msgs : nullptr;
    job.status = status_inout;
    return exec_leader_next(&job);
  }
  DeviceGuard dg_(e->device);
  HIPCHK(dg_.rc);
  PooledStream ps(e->device);
  hipStream_t st = ps.s;
  if (!st) return PRIO3_EDEVICE;
  if (d.jr_len)
    HIPCHK(hipMemcpyAsync(R->msgs + 16 * (size_t)c0, prep_msgs, (size_t)e->sz.prep_msg_len * n,
                          hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(R->status + c0, status_inout, n, hipMemcpyHostToDevice, st));
  DevParams dp = R->dp;
  dp.n = n;
  R->last = st;
  Scratch sc = R->sc;
  if (R->corr_all) sc.corrected = R->corr_all;  // FPVec: seeds of every sub-batch
  if (c0) {  // the batch's columns of a shared run (FPVec and multiproof runs are whole: c0 = 0)
    sc.corrected += c0;
    sc.meas = (uint8_t*)sc.meas + (size_t)dp.es * c0;
    sc.out = (uint8_t*)sc.out + (size_t)dp.es * c0;
  }
  int rc2 = PRIO3_OK;
  if (dp.kind == PRIO3_SUMVEC_F64_MP)
    TIMED(e, st, "k_leader_next", rc2 = launch_mp64_leader_next(n, R->msgs, sc, R->status, st));
  else
    TIMED(e, st, "k_leader_next",
          rc2 = launch_leader_next(dp, R->msgs + 16 * (size_t)c0, sc, R->status + c0, st));
  if (rc2) return rc2;
  HIPCHK(hipMemcpyAsync(status_inout, R->status + c0, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (e->timing) collect_times(e);
  return PRIO3_OK;
}

// leader_continued on the helper's messages and the writer's merge of the job's output shares
// (/root/reference/aggregator/src/aggregator/aggregation_job_driver.rs:677-691, then
// aggregation_job_writer.rs:591-695) in one launch of the prepare_next executor: the check of
// each report, then the per-segment sum of the reports it kept, for many jobs at once.
int prio3_leader_prepare_next_aggregate_batch(prio3_batch* b, const uint8_t* prep_msgs,
                                              uint8_t* status_inout, const uint32_t* segment_ids,
                                              const uint8_t* accept_mask, uint32_t n_segments,
                                              uint8_t* agg_shares_out, uint64_t* counts_out) {
  TraceSpan span_("leader VDAF preparation");
  if (!b || !status_inout || n_segments == 0 || !agg_shares_out || !counts_out)
    return PRIO3_EINVAL;
  prio3_engine* e = b->e;
  const uint32_t n = b->n;
  const DevParams& d = e->dp;
  Run* R = b->run;
  const bool one = R && n && leader_coalescable(e) && n <= LNEXT_MAX_REPS && R->msgs &&
                   R->linput;
  LNextJob job;
  job.device = e->device;
  job.run = R;
  job.nseg = n_segments;
  if (one && engine_lnext_out_bytes(&job) <= LNEXT_MAX_OUT) {
    if (d.jr_len && !prep_msgs) return PRIO3_EINVAL;
    job.c0 = b->c0;
    job.n = n;
    job.msgs = d.jr_len ? prep_msgs : nullptr;
    job.status = status_inout;
    job.seg = segment_ids;
    job.accept = accept_mask;
    job.agg_out = agg_shares_out;
    job.counts_out = counts_out;
    return exec_leader_next(&job);
  }
  int rc = prio3_leader_prepare_next_batch(b, prep_msgs, status_inout);
  if (rc == PRIO3_OK)
    rc = prio3_accumulate(b, segment_ids, accept_mask, n_segments, agg_shares_out, counts_out);
  return rc;
}

int prio3_trace_enabled(void) { return trace_enabled() ? 1 : 0; }

int prio3_selftest_field(int op, uint32_t n, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  if (op < 0 || op > 5) return PRIO3_EINVAL;
  if (n == 0) return PRIO3_OK;
  const size_t m = (op >= 4 ? 16 : 1) * (size_t)n * 16;
  void *da = nullptr, *db = nullptr, *dout = nullptr;
  int rc = PRIO3_OK;
  if (hipMalloc(&da, m) != hipSuccess || hipMalloc(&db, m) != hipSuccess ||
      hipMalloc(&dout, (size_t)n * 16) != hipSuccess ||
      hipMemcpy(da, a, m, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(db, b, m, hipMemcpyHostToDevice) != hipSuccess) {
    rc = PRIO3_EDEVICE;
  } else {
    k_selftest_f128<<<(n + 255) / 256, 256>>>(op, n, (const uint4*)da, (const uint4*)db, (uint4*)dout);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpy(out, dout, (size_t)n * 16, hipMemcpyDeviceToHost) != hipSuccess)
      rc = PRIO3_EDEVICE;
  }
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  return rc;
}

}  // extern "C"
