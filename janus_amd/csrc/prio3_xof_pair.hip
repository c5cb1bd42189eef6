// prio3_xof_pair.hip -- the helper XOF half of Prio3::prepare_init for LONG measurement shares
// (Prio3SumVec 8x1000: 8,000 elements; FixedPointBoundedL2VecSum 10^4 entries: 160,030), two
// work-items per report (MI355X, gfx950).
//
// prio 0.16.2 prepare_init (agg_id 1), SURVEY.md A.5.1-A.5.4: query randomness, the
// measurement share XOF(k_meas, dst(1), [1]), the joint-rand part XOF(k_blind, dst(7),
// [1] || nonce || enc(meas)) over the same bytes, the proofs share, the corrected joint-rand seed
// and the joint randomness.  Call site: helper_initialized, aggregator.rs:2020-2042.
//
// The one-lane kernel (k_xofd) keeps both sponges of the share phase in one lane's VGPRs (the
// squeeze of the share and the absorb of its bytes, ~760 permutations each for SumVec 8x1000)
// and interleaves them for ILP.  At the per-GPU batch sizes of these configs (125k and 100k
// reports: 2 and 0.8 waves per SIMD) that kernel is latency-bound: one lane walks ~1,500
// (SumVec) or ~30,500 (FPVec) permutations in sequence.  Here the two sponges live in the two
// lanes of a pair, in lockstep:
//   even lane  query header -> squeeze the share block b, store its elements, then the proofs
//   odd lane   query randomness -> absorb block b of [1] || nonce || enc(meas) (the 42-byte
//              prefix leaves every message word a 16-bit funnel shift of two squeezed words,
//              which arrive from the even lane by DPP quad_perm [0,0,2,2]) -> joint-rand part,
//              corrected seed, joint randomness
// so a report's share phase takes one permutation time per block instead of two, with one
// Keccak state per lane (fewer VGPRs: more waves per SIMD) and twice the work-items.
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"
#include "prio3_pair.h"

namespace {

typedef Fp128 F;

// TR: the even lane also truncates the share into sc.out as it squeezes (DevParams::trunc_xof)
template <bool TR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TR ? 4 : 5, TR ? 4 : 5))) void k_xof_pair(
    DevParams p, InPtrs in, Scratch sc) {
  const uint32_t tid = threadIdx.x, h = tid & 1u;
  const uint32_t r = blockIdx.x * 128 + (tid >> 1);
  const bool live = r < p.n;
  const uint32_t rr = live ? r : p.n - 1;  // a dead pair computes on a valid report, stores nothing
  uint32_t flag = p.force_slow;
  uint32_t nonce[4], km[4], kp[4], kb[4];
  load16(in.nonces + 16 * (size_t)rr, nonce);
  const uint8_t* hs = in.helper + (size_t)rr * p.helper_share_len;
  load16(hs, km);
  load16(hs + 16, kp);
  load16(hs + 32, kb);
  KState st;
  kzero(st);
  // 1. even: the share XOF header XOF(k_meas, dst(1), [1]); odd: the query-randomness message
  //    XOF(vk, dst(5), [PROOFS] || nonce) -- one absorb + permutation, per-lane message words
  {
    Msg a, q;
    msg_zero(a);
    msg_dst(a, p.dst[1]);
    msg_bytes16(a, 9, km);
    msg_byte(a, 25, 1);
    msg_byte(a, 26, 0x01);
    a.w[41] ^= 0x80000000u;
    uint32_t vk[4];
    load_vk(p, in, rr, vk);
    msg_zero(q);
    msg_dst(q, p.dst[5]);
    msg_bytes16(q, 9, vk);
    msg_byte(q, 25, 1);
    msg_bytes16(q, 26, nonce);
    msg_byte(q, 42, 0x01);
    q.w[41] ^= 0x80000000u;
#pragma unroll
    for (int i = 0; i < 42; i++) kxor_word(st, i, h ? q.w[i] : a.w[i]);
    keccak_p12(st);
  }
  if (h && live) {  // query randomness (qr_len <= 2 elements, block 0)
    uint32_t q0 = 0, q1 = 0;
    squeeze_block<F>(p, st, 0, p.qr_len, q0, q1, sc.qr, rr, flag);
  }
  // the odd lane restarts its state for the joint-rand part; its first 42 message bytes are
  // [len(dst)] || dst(7) || k_blind || [1] || nonce
  {
    const uint32_t keep = h ? 0u : 0xffffffffu;
#pragma unroll
    for (int i = 0; i < 25; i++) {
      st.lo[i] &= keep;
      st.hi[i] &= keep;
    }
  }
  uint32_t pre[11];
  {
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[7]);
    msg_bytes16(m, 9, kb);
    msg_byte(m, 25, 1);
    msg_bytes16(m, 26, nonce);
#pragma unroll
    for (int j = 0; j < 11; j++) pre[j] = m.w[j];
  }
  // 2. the share phase: block b of the squeeze (even) is block b of the absorb (odd)
  const uint32_t M = p.meas_len, K = (M * 16 + 167) / 168;
  const uint32_t Lb = 42 + M * 16, B = Lb / 168, rem = Lb % 168;  // absorb blocks 0..B
  uint32_t tail[11];
#pragma unroll
  for (int t = 0; t < 11; t++) tail[t] = 0;
  uint32_t pend0 = 0, pend1 = 0;
  TruncSink ts(p, sc.out, rr);
  // block 0 (prefix), full blocks 1 .. B-1, the padded last block B (B >= 2: see the launcher)
  if (h == 0 && live) squeeze_meas<TR>(p, st, 0, M, pend0, pend1, sc.meas, rr, flag, ts);
  absorb_share_block<true, false>(st, h, true, tail, pre, rem);
  keccak_p12(st);
#pragma unroll 1
  for (uint32_t b = 1; b < B; b++) {
    const bool hasW = b < K;  // uniform
    if (hasW && h == 0 && live) squeeze_meas<TR>(p, st, b, M, pend0, pend1, sc.meas, rr, flag, ts);
    absorb_share_block<false, false>(st, h, hasW, tail, pre, rem);
    keccak_p12(st);  // even: next squeeze block; odd: absorb
  }
  {
    const bool hasW = B < K;
    if (hasW && h == 0 && live) squeeze_meas<TR>(p, st, B, M, pend0, pend1, sc.meas, rr, flag, ts);
    absorb_share_block<false, true>(st, h, hasW, tail, pre, rem);
    keccak_p12(st);
  }
  uint32_t part[4] = {kword(st, 0), kword(st, 1), kword(st, 2), kword(st, 3)};
  // 3. even: the proofs share XOF(k_proofs, dst(2), [PROOFS, 1]); odd: corrected seed and
  //    joint randomness
  if (h == 0) {
    kzero(st);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[2]);
    msg_bytes16(m, 9, kp);
    msg_byte(m, 25, 1);
    msg_byte(m, 26, 1);
    msg_absorb_final(st, m, 27);
    const uint32_t PL = p.proof_len, Kp = (PL * 16 + 167) / 168;
    uint32_t q0 = 0, q1 = 0;
    for (uint32_t b = 0; b < Kp; b++) {
      if (live) squeeze_block<F>(p, st, b, PL, q0, q1, sc.proofs, rr, flag);
      if (b + 1 < Kp) keccak_p12(st);
    }
  } else {
    uint32_t pub0[4];
    load16(in.pub + (size_t)rr * p.public_share_len, pub0);
    kzero(st);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[6]);
    msg_bytes16(m, 25, pub0);
    msg_bytes16(m, 41, part);
    msg_absorb_final(st, m, 57);
    uint32_t cor[4] = {kword(st, 0), kword(st, 1), kword(st, 2), kword(st, 3)};
    kzero(st);
    Msg m2;
    msg_zero(m2);
    msg_dst(m2, p.dst[3]);
    msg_bytes16(m2, 9, cor);
    msg_byte(m2, 25, 1);
    msg_absorb_final(st, m2, 26);
    uint32_t q0 = 0, q1 = 0;
    if (live) {
      squeeze_block<F>(p, st, 0, p.jr_len, q0, q1, sc.jr, rr, flag);
      sc.part[rr] = make_uint4(part[0], part[1], part[2], part[3]);
      sc.corrected[rr] = make_uint4(cor[0], cor[1], cor[2], cor[3]);
    }
  }
  flag |= from_odd(flag);  // any rejection-sampling event of either lane flags the report
  if (h == 0 && live) sc.flag[rr] = (uint8_t)flag;
}

}  // namespace

// long-share joint-randomness instances (SumVec / FPVec): true if launched
bool launch_xof_pair(const DevParams& p, InPtrs in, Scratch sc, hipStream_t st) {
  if (p.es != 16 || !p.jr_len || (42 + p.meas_len * 16) / 168 < 2) return false;
  if (p.trunc_xof)
    k_xof_pair<true><<<(p.n + 127) / 128, 256, 0, st>>>(p, in, sc);
  else
    k_xof_pair<false><<<(p.n + 127) / 128, 256, 0, st>>>(p, in, sc);
  return true;
}
