// prio3_mp64.hip -- helper prepare of Prio3SumVecField64MultiproofHmacSha256Aes128 on MI355X
// (SURVEY 8(f) row 4): SumVec<Field64, ParallelSum<Mul>> with XofHmacSha256Aes128, 32-byte
// seeds, num_proofs >= 2 (/root/reference/core/src/vdaf.rs:173-195; the Daphne-interop VDAF).
//
// XofHmacSha256Aes128 (prio 0.16 vdaf/xof.rs, restated; parity with prio UNPINNED, see
// DESIGN.md): HMAC-SHA256 keyed by the 32-byte seed over len(dst) || dst || binder; the 32-byte
// tag is an AES-128 key and IV of a CTR keystream with a 64-bit big-endian counter in the IV's
// low half (Ctr64BE<Aes128>).  Field64 elements are 8-byte LE chunks, rejected if >= p.
//
// One report per lane (k_mp64_prepare), everything in one launch: measurement and proofs
// shares expanded to SoA scratch (one inlined keystream loop with the round keys in registers
// and a bank-replicated T-table, expand_soa_inl), the joint-rand part HMAC streamed over the encoded
// measurement share as a 32-bit-word stream (the 26-byte prefix leaves every word a 16-bit
// funnel shift of two elements), corrected seed, joint and query randomness, then per proof
// the FLP query (Lagrange basis at t by one batch inversion over the P roots, wire sums, p(t) by
// Horner, the call sum through sigma), decide against the leader's verifier share, the prepare
// message, the joint-rand check and the truncated output share.
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"
#include "sha256_device.h"
#include "aes_device.h"
#include "prio3_mp64_xof.h"

namespace {

typedef Fp64 F;
typedef uint64_t T;

DEV T sqn64(T x, int n) {
  for (int i = 0; i < n; i++) x = mul64f(x, x);
  return x;
}
// x^(p-2), p - 2 = (2^32 - 2) 2^32 + (2^32 - 1): u = x^(2^32 - 2) = (x^(2^31 - 1))^2 by an
// addition chain (31 squarings, 8 multiplies), then u^(2^32) u x -- 63 squarings and 9 multiplies
// instead of the 64 + 62 of square-and-multiply
DEV T inv64(T x) {
  const T t2 = mul64f(sqn64(x, 1), x);      // 2^2 - 1
  const T t3 = mul64f(sqn64(t2, 1), x);     // 2^3 - 1
  const T t6 = mul64f(sqn64(t3, 3), t3);    // 2^6 - 1
  const T t12 = mul64f(sqn64(t6, 6), t6);   // 2^12 - 1
  const T t15 = mul64f(sqn64(t12, 3), t3);  // 2^15 - 1
  const T t16 = mul64f(sqn64(t15, 1), x);   // 2^16 - 1
  const T t31 = mul64f(sqn64(t16, 15), t15);  // 2^31 - 1
  const T u = sqn64(t31, 1);                // 2^32 - 2
  return mul64f(sqn64(u, 32), mul64f(u, x));  // (2^32 - 2) 2^32 + 2^32 - 1
}

}  // namespace

// LEADER = 1: the leader's prepare_init (agg_id 0, aggregation_job_driver.rs:397-415) on its
// explicit input share (in.helper = the leader input shares: enc(meas) || enc(proofs) ||
// k_blind): the shares are decoded (non-canonical -> INPUT_SHARE_DECODE) instead of expanded,
// the verifier share || joint-rand part is written to out.prep_msgs (stride prep_share_len), and
// the corrected seed is kept for prepare_next (words 0-3 in sc.corrected, 4-7 in sc.part).
// 4 waves per SIMD (120 VGPRs, a few more spilled bytes in the short XOF calls; 37 KiB of LDS per
// block still fits four blocks per CU): 100.9-101.2 against 96.8-97.0 M reports/s at the
// default's 132 VGPRs / 3 waves (r04p, interleaved)
template <int LEADER>
__global__ __launch_bounds__(256, 4) void k_mp64_prepare(Mp64Params P, uint32_t n, size_t ld,
                                                      InPtrs in, Scratch sc, OutPtrs out,
                                                      uint32_t force_slow) {
  __shared__ AesT A;
  __shared__ AesR AR;  // bank-replicated T0 for the two share expansions (expand_soa_inl)
  aes_tables_init(A);
  if (!LEADER) aesr_init(AR);
  __syncthreads();
  const AesRLane AL = aesr_lane(AR);
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  (void)force_slow;
  uint64_t* meas = (uint64_t*)sc.meas;
  uint64_t* proofs = (uint64_t*)sc.proofs;
  uint64_t* Lb = (uint64_t*)sc.Lbuf;
  uint8_t status = PRIO3_STATUS_FINISHED;
  uint32_t nonce[4], kmeas[8], kproofs[8], kblind[8], pub0[8];
  const uint32_t M = P.meas_len, np = P.np, PL = P.proof_len;
  const size_t lshare_len = (size_t)(M + PL * np) * 8 + 32;
  {
    const uint4 v = *(const uint4*)(in.nonces + 16 * (size_t)r);
    nonce[0] = v.x, nonce[1] = v.y, nonce[2] = v.z, nonce[3] = v.w;
    // helper: k_meas || k_proofs || k_blind and the leader's part (public share bytes 0..31);
    // leader: k_blind at the end of its explicit share and the helper's part (bytes 32..63)
    const uint4* hs = (const uint4*)(in.helper + (LEADER ? lshare_len : 96) * (size_t)r);
    const uint4* kb = LEADER ? (const uint4*)((const uint8_t*)hs + lshare_len - 32) : hs + 4;
    const uint4* ps = (const uint4*)(in.pub + 64 * (size_t)r) + (LEADER ? 2 : 0);
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint4 c = kb[i], d = ps[i];
      if (!LEADER) {
        const uint4 a = hs[i], b = hs[2 + i];
        kmeas[4 * i] = a.x, kmeas[4 * i + 1] = a.y, kmeas[4 * i + 2] = a.z,
        kmeas[4 * i + 3] = a.w;
        kproofs[4 * i] = b.x, kproofs[4 * i + 1] = b.y, kproofs[4 * i + 2] = b.z,
        kproofs[4 * i + 3] = b.w;
      }
      kblind[4 * i] = c.x, kblind[4 * i + 1] = c.y, kblind[4 * i + 2] = c.z,
      kblind[4 * i + 3] = c.w;
      pub0[4 * i] = d.x, pub0[4 * i + 1] = d.y, pub0[4 * i + 2] = d.z, pub0[4 * i + 3] = d.w;
    }
  }
  uint32_t rej = 0;
  if (LEADER) {  // the explicit shares into SoA scratch, canonical encodings only
    const uint64_t* ls = (const uint64_t*)(in.helper + lshare_len * (size_t)r);
    bool ok = true;
    for (uint32_t e = 0; e < M; e++) {
      const uint64_t x = ls[e];
      ok = ok && x < P64;
      meas[(size_t)e * ld + r] = x;
    }
    for (uint32_t e = 0; e < PL * np; e++) {
      const uint64_t x = ls[M + e];
      ok = ok && x < P64;
      proofs[(size_t)e * ld + r] = x;
    }
    if (!ok) status = PRIO3_STATUS_INPUT_SHARE_DECODE;
  }
  // 1. measurement share: XOF(k_meas, dst(1), [1]); 2. proofs share: XOF(k_proofs, dst(2),
  //    [np, 1]) -- one loop, so the unrolled keystream (expand_soa_inl) is inlined once
  if (!LEADER) {
#pragma nounroll
    for (int sh = 0; sh < 2; sh++) {
      Msg32<16> m;
      mz(m);
      msg_dst(m, P, 1 + sh);
      mbyte(m, 9, sh ? np : 1);
      if (sh) mbyte(m, 10, 1);
      uint32_t seed[8], tag[8];
#pragma unroll
      for (int i = 0; i < 8; i++) seed[i] = sh ? kproofs[i] : kmeas[i];
      xof_tag(seed, m, 10 + sh, tag);
      rej += expand_soa_inl(AL, tag, sh ? proofs : meas, ld, r, sh ? PL * np : M);
    }
  }
  // 3. joint-rand part: XOF(k_blind, dst(7), [1] || nonce || enc(meas)) -> 32 bytes
  uint32_t part[8];
  {
    HmacKey k;
    hmac_key_ni(kblind, k.ist, k.ost);
    Msg32<8> pm;  // the 26-byte prefix, big-endian words 0..6 (+2 bytes of word 6 free)
    mz(pm);
    msg_dst(pm, P, 7);
    mbyte(pm, 9, LEADER ? 0 : 1);
    mwords_le(pm, 10, nonce, 4);
    const uint32_t L = 26 + 8 * M;
    const uint32_t nblk = (L + 9 + 63) / 64;
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = k.ist[i];
    jr_inner_inl(st, pm.w, meas, ld, r, M, L, nblk);
    uint32_t o[16] = {st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], 0x80000000u,
                      0, 0, 0, 0, 0, 0, (64 + 32) * 8};
    uint32_t tag[8];
#pragma unroll
    for (int i = 0; i < 8; i++) tag[i] = k.ost[i];
    compress_ni(tag, o);
    Stream s;
    stream_init(A, s, tag);
    derive32(A, s, part);
  }
  // 4. corrected seed: XOF(0^32, dst(6), leader part || helper part) -> 32 bytes (the other
  //    party's part from the public share)
  uint32_t corrected[8];
  {
    Msg32<32> m;
    mz(m);
    msg_dst(m, P, 6);
    mwords_le(m, 9, LEADER ? part : pub0, 8);
    mwords_le(m, 41, LEADER ? pub0 : part, 8);
    uint32_t tag[8];
    hmac_ni(P.z_ist, P.z_ost, m.w, 73, tag);
    Stream s;
    stream_init(A, s, tag);
    derive32(A, s, corrected);
  }
  // 5. joint randomness XOF(corrected, dst(3), [np]) and query randomness
  //    XOF(vk, dst(5), [np] || nonce), one element per proof
  constexpr int MAXP = 8;
  T jr[MAXP], qr[MAXP];
  {
    Msg32<16> m;
    mz(m);
    msg_dst(m, P, 3);
    mbyte(m, 9, np);
    uint32_t tag[8];
    xof_tag(corrected, m, 10, tag);
    Stream s;
    stream_init(A, s, tag);
    expand_regs<MAXP>(A, s, jr, np);
  }
  {
    Msg32<16> m;
    mz(m);
    msg_dst(m, P, 5);
    mbyte(m, 9, np);
    mwords_le(m, 10, nonce, 4);
    uint32_t tag[8];
    hmac_ni(P.vk_ist, P.vk_ost, m.w, 26, tag);
    Stream s;
    stream_init(A, s, tag);
    expand_regs<MAXP>(A, s, qr, np);
  }
  // 6. FLP query per proof + decide against the leader's verifier share
  const uint8_t* lps = LEADER ? nullptr : in.leader + (size_t)(P.vlen * np * 8 + 32) * r;
  uint8_t* lout = LEADER ? out.prep_msgs + (size_t)(P.vlen * np * 8 + 32) * r : nullptr;
  bool decode_ok = true, decide_ok = true;
  const T half = P.half;
  const uint32_t C = P.chunk, K = P.calls, PP = P.P;
  for (uint32_t k = 0; k < np; k++) {
    const T t = qr[k < MAXP ? k : 0], rr = jr[k < MAXP ? k : 0];
    // Lagrange basis at t over the P-th roots: L_i = (t^P - 1)/P * alpha^i / (t - alpha^i)
    T tp = t;
    for (uint32_t i = 0; i < P.logP; i++) tp = F::mul(tp, tp);
    if (tp == 1) status = PRIO3_STATUS_PREP_INIT;
    const T cst = F::mul(F::sub(tp, 1), P.invP);
    T pre = 1, ai = 1;
    for (uint32_t i = 0; i < PP; i++) {  // prefix products of d_i = t - alpha^i
      pre = F::mul(pre, F::sub(t, ai));
      Lb[(size_t)i * ld + r] = pre;
      ai = F::mul(ai, P.alpha);
    }
    T inv = inv64(pre);
    T aback = P.alpha_inv;  // alpha^i, i = P-1 .. 0 (alpha^(P-1) = alpha^-1)
    for (uint32_t i = PP; i-- > 0;) {
      const T di = F::sub(t, aback);
      const T inv_i = i ? F::mul(inv, Lb[(size_t)(i - 1) * ld + r]) : inv;
      inv = F::mul(inv, di);
      Lb[(size_t)i * ld + r] = F::mul(F::mul(cst, aback), inv_i);
      aback = F::mul(aback, P.alpha_inv);
    }
    const T L0 = Lb[r];
    const uint64_t* pf = proofs + (size_t)k * PL * ld;
    // wire sums at t; r^(idx+1) on the even wires, (m - 1/2) on the odd ones (zero-padded
    // measurement elements count as 0, VDAF-08 SumVec.eval).  With rC = r^C, call kk of column
    // jj weighs m_(kk C + jj) by r^(jj+1) rC^kk L_(kk+1) on the even wire and by L_(kk+1) on the
    // odd one, so per column f0 = r^(jj+1) sum_kk m G_kk and f1 = sum_kk m L_(kk+1) - (1/2) SL
    // with G_kk = rC^kk L_(kk+1) (kept in sc.beta) and SL = sum_kk L_(kk+1): two products per
    // call instead of four
    T rC = 1;
    for (uint32_t i = 0; i < C; i++) rC = F::mul(rC, rr);
    uint64_t* Gb = (uint64_t*)sc.beta;
    T hSL = 0;
    {
      T g = 1;
      for (uint32_t kk = 0; kk < K; kk++) {
        const T Lk = Lb[(size_t)(kk + 1) * ld + r];
        Gb[(size_t)kk * ld + r] = F::mul(g, Lk);
        hSL = F::add(hSL, Lk);
        g = F::mul(g, rC);
      }
      hSL = F::mul(hSL, half);
    }
    T G = 0, rj = rr;
    const uint8_t* lv = LEADER ? nullptr : lps + (size_t)k * P.vlen * 8;
    T* vo = LEADER ? (T*)(lout + (size_t)k * P.vlen * 8) : nullptr;
    auto lvf = [&](uint32_t e) {
      const T x = *(const T*)(lv + 8 * e);
      if (x >= P64) decode_ok = false;
      return x;
    };
    for (uint32_t jj = 0; jj < C; jj++) {
      mac64 a0, a1;  // lazily reduced sums of the call products (one fold per column)
      mac64_zero(a0);
      mac64_zero(a1);
      for (uint32_t kk = 0; kk < K; kk++) {
        const uint32_t idx = kk * C + jj;
        if (idx >= M) break;  // zero-padded elements add nothing to s0 / s1
        const T m = ld64(meas, ld, idx, r);
        mac64_add(a0, m, Gb[(size_t)kk * ld + r]);
        mac64_add(a1, m, Lb[(size_t)(kk + 1) * ld + r]);
      }
      const T s0 = mac64_reduce(a0), s1 = mac64_reduce(a1);
      const T f0 = F::add(F::mul(ld64(pf, ld, 2 * jj, r), L0), F::mul(rj, s0));
      const T f1 = F::sub(F::add(F::mul(ld64(pf, ld, 2 * jj + 1, r), L0), s1), hSL);
      if (LEADER) {
        vo[1 + 2 * jj] = f0;
        vo[2 + 2 * jj] = f1;
      } else {
        G = F::add(G, F::mul(F::add(f0, lvf(1 + 2 * jj)), F::add(f1, lvf(2 + 2 * jj))));
      }
      rj = F::mul(rj, rr);
    }
    // p(t) by Horner; v = sum_calls p(alpha^(c+1)) = sum_e coef_e sigma_(e mod P)
    T pt = 0;
    mac64 va;
    mac64_zero(va);
    for (uint32_t q = 0; q < P.glen; q++) {
      const uint32_t e = P.glen - 1 - q;
      const T c = ld64(pf, ld, P.arity + e, r);
      pt = F::add(F::mul(pt, t), c);
      mac64_add(va, c, P.sigma[e & (PP - 1)]);
    }
    const T v = mac64_reduce(va);
    if (LEADER) {
      vo[0] = v;
      vo[P.arity + 1] = pt;
    } else {
      const T V0 = F::add(lvf(0), v), PT = F::add(lvf(P.arity + 1), pt);
      if (V0 != 0 || G != PT) decide_ok = false;
    }
  }
  if (LEADER) {  // joint-rand part after the verifiers; corrected seed kept for prepare_next
    uint4* po = (uint4*)(lout + (size_t)P.vlen * np * 8);
    po[0] = make_uint4(part[0], part[1], part[2], part[3]);
    po[1] = make_uint4(part[4], part[5], part[6], part[7]);
    sc.corrected[r] = make_uint4(corrected[0], corrected[1], corrected[2], corrected[3]);
    sc.part[r] = make_uint4(corrected[4], corrected[5], corrected[6], corrected[7]);
    out.status[r] = status;
  } else {
  // 7. prepare message XOF(0^32, dst(6), leader part || helper part), joint-rand check
  uint32_t lpart[8];
  {
    const uint4* lp = (const uint4*)(lps + (size_t)P.vlen * np * 8);
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint4 a = lp[i];
      lpart[4 * i] = a.x, lpart[4 * i + 1] = a.y, lpart[4 * i + 2] = a.z, lpart[4 * i + 3] = a.w;
    }
  }
  uint32_t msg[8];
  {
    Msg32<32> m;
    mz(m);
    msg_dst(m, P, 6);
    mwords_le(m, 9, lpart, 8);
    mwords_le(m, 41, part, 8);
    uint32_t tag[8];
    hmac_ni(P.z_ist, P.z_ost, m.w, 73, tag);
    Stream s;
    stream_init(A, s, tag);
    derive32(A, s, msg);
  }
  if (status == PRIO3_STATUS_FINISHED) {
    if (!decode_ok)
      status = PRIO3_STATUS_PREP_SHARE_DECODE;
    else if (!decide_ok)
      status = PRIO3_STATUS_PREP_MSG;
    else {
      uint32_t diff = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) diff |= msg[i] ^ corrected[i];
      if (diff) status = PRIO3_STATUS_PREP_NEXT;
    }
  }
  (void)rej;  // a rejected sample only moves the stream on; no slow path needed here
  uint4* mo = (uint4*)(out.prep_msgs + 32 * (size_t)r);
  const bool fin = status == PRIO3_STATUS_FINISHED;
  mo[0] = fin ? make_uint4(msg[0], msg[1], msg[2], msg[3]) : make_uint4(0, 0, 0, 0);
  mo[1] = fin ? make_uint4(msg[4], msg[5], msg[6], msg[7]) : make_uint4(0, 0, 0, 0);
  out.status[r] = status;
  }
  // 8. output share: SumVec truncate (bit recomposition)
  uint64_t* o = (uint64_t*)sc.out;
  for (uint32_t e = 0; e < P.out_len; e++) {
    T acc;
    if (P.bits <= 31) {  // sum of m_b 2^b as two 64-bit columns (no carries: < 2^63), one fold
      uint64_t c0 = 0, c1 = 0;
      for (uint32_t b = 0; b < P.bits; b++) {
        const T m = ld64(meas, ld, e * P.bits + b, r);
        c0 += (uint64_t)(uint32_t)m * (1u << b);
        c1 += (uint64_t)(uint32_t)(m >> 32) * (1u << b);
      }
      const uint64_t s1 = (c0 >> 32) + (uint32_t)c1;
      acc = red128_64((s1 << 32) | (uint32_t)c0, (s1 >> 32) + (c1 >> 32));
    } else {
      T pw = 1;
      acc = 0;
      for (uint32_t b = 0; b < P.bits; b++) {
        acc = F::add(acc, F::mul(pw, ld64(meas, ld, e * P.bits + b, r)));
        pw = F::add(pw, pw);
      }
    }
    o[(size_t)e * ld + r] = acc;
  }
}

int launch_mp64(prio3_engine* e, uint32_t n, uint32_t ld, InPtrs in, OutPtrs out, Scratch sc,
                hipStream_t st) {
  k_mp64_prepare<0><<<(n + 255) / 256, 256, 0, st>>>(e->mp, n, ld, in, sc, out,
                                                     (uint32_t)e->force_slow);
  return hipGetLastError() == hipSuccess ? PRIO3_OK : PRIO3_EDEVICE;
}

// leader prepare_init (in.helper = the leader input shares, out.prep_msgs = prep shares)
int launch_mp64_leader(prio3_engine* e, uint32_t n, uint32_t ld, InPtrs in, OutPtrs out,
                       Scratch sc, hipStream_t st) {
  k_mp64_prepare<1><<<(n + 255) / 256, 256, 0, st>>>(e->mp, n, ld, in, sc, out,
                                                     (uint32_t)e->force_slow);
  return hipGetLastError() == hipSuccess ? PRIO3_OK : PRIO3_EDEVICE;
}

// leader prepare_next: the helper's 32-byte prepare message must equal the corrected seed
// (else VdafPrepareNext); the output share was written by the init kernel
__global__ __launch_bounds__(256) void k_mp64_leader_next(uint32_t n, const uint8_t* prep_msgs,
                                                          Scratch sc, uint8_t* status) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n || status[r] != PRIO3_STATUS_FINISHED) return;
  const uint4* m = (const uint4*)(prep_msgs + 32 * (size_t)r);
  const uint4 a = m[0], b = m[1], c = sc.corrected[r], d = sc.part[r];
  const uint32_t diff = (a.x ^ c.x) | (a.y ^ c.y) | (a.z ^ c.z) | (a.w ^ c.w) | (b.x ^ d.x) |
                        (b.y ^ d.y) | (b.z ^ d.z) | (b.w ^ d.w);
  if (diff) status[r] = PRIO3_STATUS_PREP_NEXT;
}

int launch_mp64_leader_next(uint32_t n, const uint8_t* d_prep_msgs, Scratch sc, uint8_t* d_status,
                            hipStream_t st) {
  k_mp64_leader_next<<<(n + 255) / 256, 256, 0, st>>>(n, d_prep_msgs, sc, d_status);
  return hipGetLastError() == hipSuccess ? PRIO3_OK : PRIO3_EDEVICE;
}
