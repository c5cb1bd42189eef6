// prio3_query_sum.h -- the Prio3Sum helper/leader query body (k_query_sum, prio3_query_sum.hip),
// shared with the fused XOF + query kernel of prio3_engine.hip (k_prep_sum).  See
// prio3_query_sum.hip for the algorithm.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"

namespace qsum {


typedef Fp128 F;
typedef f128 T;

DEV T tw(const DevParams& p, int i) { return F::from_words(p.tws[i]); }

// in-register radix-2 DFT16, input in bit-reversed order, output natural; w16^j = p.tws[j]
DEV void dft16(const DevParams& p, T (&x)[16]) {
#pragma unroll
  for (int l = 1; l <= 4; l++) {
    const int half = 1 << (l - 1);
#pragma unroll
    for (int i = 0; i < half; i++) {
      const T w = tw(p, i * (16 >> l));
#pragma unroll
      for (int j = i; j < 16; j += 2 * half) {
        const T u = x[j];
        const T v = (i == 0) ? x[j + half] : F::mul(w, x[j + half]);
        x[j] = F::add(u, v);
        x[j + half] = F::sub(u, v);
      }
    }
  }
}

// x[bitrev(n)] = s q^n, n < 16
DEV void geo16(T (&x)[16], T s, const T& q) {
#pragma unroll
  for (int n = 0; n < 16; n++) {
    x[__builtin_bitreverse32(n) >> 28] = s;
    if (n < 15) s = F::mul(s, q);
  }
}

// LEADER = 1: the leader's prepare_init (agg_id 0) on the same data flow (after k_leader_unpack
// and the leader k_jrpart): the verifier share [v, f(t), p(t)] and the joint-rand part go to
// out.prep_msgs (stride prep_share_len) instead of being decided against a peer's share;
// out.status holds the unpack verdict on entry.
// slow_defer / redo (DevParams): as query_h_body -- a flagged report is skipped here and redone
// by the run's k_slow_redo launch (prio3_engine.hip)
template <int NPH, int LEADER = 0>
__device__ __forceinline__ void query_sum_body(const DevParams& p, const InPtrs& in,
                                               const Scratch& sc, const OutPtrs& out,
                                               const uint32_t r) {
  constexpr uint32_t P = 16 * NPH;
  if (r >= p.n) return;
  if constexpr (!LEADER) {
    if (p.redo) {
      if (sc.flag[r] != 2) return;
    } else if (p.slow_defer && sc.flag[r]) {
      return;
    }
  }
  const size_t ld = p.ld;
  const uint32_t K = p.calls, GL = p.glen;
  const T one = F::one(), Z = F::zero();
  uint8_t status = LEADER ? out.status[r] : PRIO3_STATUS_FINISHED;
  const T t = ldf<F>(sc.qr, 0, ld, r);
  T t16 = F::mul(t, t);
  t16 = F::mul(t16, t16);
  t16 = F::mul(t16, t16);
  t16 = F::mul(t16, t16);
  {
    T tP = t16;
#pragma unroll
    for (uint32_t q = 1; q < NPH; q <<= 1) tP = F::mul(tP, tP);
    if (F::eq(tP, one)) status = PRIO3_STATUS_PREP_INIT;  // t is a P-th root of unity
  }
  const T r0 = ldf<F>(sc.jr, 0, ld, r);
  T r16 = F::mul(r0, r0);
  r16 = F::mul(r16, r16);
  r16 = F::mul(r16, r16);
  r16 = F::mul(r16, r16);
  const T invP = FC<F>::invP(p);
  // s(n): K = 16 a + b; s(0) = sum_(i=1..a) g^i, s(1..b) = sum_(i=0..a) g^i,
  // s(b+1..15) = sum_(i=0..a-1) g^i
  const uint32_t a = K >> 4, b = K & 15u;
  T L0 = Z, v = Z, f = Z;  // f: sum_c L_c m_(c-1), reduced once per phase
#pragma unroll 1
  for (uint32_t ph = 0; ph < NPH; ph++) {
    const T aph = tw(p, 8 + (int)ph), a16 = tw(p, 16 + (int)ph);
    T x[16];
    // ---- Lagrange phase: X[NPH k + ph] = L_c, c = (P - NPH k - ph) mod P
    {
      const T h = F::mul(t16, a16);
      T G = one;
      for (uint32_t i = 1; i < NPH; i++) G = F::add(F::mul(G, h), one);
      geo16(x, F::mul(G, invP), F::mul(t, aph));
      dft16(p, x);
      mac128 Fw;
      mac_zero(Fw);
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t c = (P - NPH * (uint32_t)k - ph) & (P - 1);
        if (c == 0) {
          L0 = x[k];
        } else if (c <= K) {  // uniform
          mac_add(Fw, x[k], ldf<F>(sc.meas, c - 1, ld, r));
        }
      }
      f = F::add(f, mac_reduce_f(Fw));
    }
    // ---- validity phase: W_(NPH k + ph) = DFT16_k((r alpha^ph)^n s(n))
    {
      const T g = F::mul(r16, a16);
      T Sa = Z, ga = one;  // sum_(i<a) g^i, g^a
      for (uint32_t i = 0; i < a; i++) {
        Sa = F::add(Sa, ga);
        ga = F::mul(ga, g);
      }
      const T Sa1 = F::add(Sa, ga);     // sum_(i<=a) g^i
      const T s0 = F::sub(Sa1, one);    // sum_(i=1..a) g^i
      geo16(x, one, F::mul(r0, aph));
      if (b != 0) {  // uniform: per-element weights s(n), n >= 1
#pragma unroll
        for (int n = 1; n < 16; n++) {
          const int bn = __builtin_bitreverse32(n) >> 28;
          x[bn] = F::mul(x[bn], (uint32_t)n <= b ? Sa1 : Sa);
        }
        x[0] = s0;
      }
      dft16(p, x);
      mac128 Vp;
      mac_zero(Vp);
      sum128 Qs;
      sum_zero(Qs);
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t e = NPH * (uint32_t)k + ph;
        T q = ldf<F>(sc.proofs, 1 + e, ld, r);
        if (e + P < GL) q = F::add(q, ldf<F>(sc.proofs, 1 + e + P, ld, r));  // uniform
        mac_add(Vp, q, x[k]);
        sum_add(Qs, q);
      }
      T vp = mac_reduce_f(Vp);
      if (b == 0) {  // s(n >= 1) = Sa applied once; n = 0 contributes (s0 - Sa) * sum_k q_k
        vp = F::add(F::mul(vp, Sa), F::mul(F::sub(s0, Sa), sum_reduce(Qs)));
      }
      v = F::add(v, vp);
    }
  }
  f = F::add(f, F::mul(L0, ldf<F>(sc.proofs, 0, ld, r)));
  // p(t) = sum_j (t^16)^j sum_(n<16) coef_(16 j + n) t^n: the inner sums as lazy MACs against
  // t^0..t^15, Horner in t^16 over the GL / 16 blocks (GL = 2P - 1: 2 NPH blocks)
  T pt = Z;
  {
    T pw[16];
    pw[0] = one;
#pragma unroll
    for (int n = 1; n < 16; n++) pw[n] = F::mul(pw[n - 1], t);
#pragma unroll 1
    for (uint32_t j = 2 * NPH; j-- > 0;) {
      mac128 S;
      mac_zero(S);
#pragma unroll
      for (int n = 0; n < 16; n++) {
        const uint32_t e = 16 * j + (uint32_t)n;
        if (e < GL) mac_add(S, ldf<F>(sc.proofs, 1 + e, ld, r), pw[n]);  // uniform
      }
      pt = F::add(F::mul(pt, t16), mac_reduce_f(S));
    }
  }
  if constexpr (LEADER) {
    uint8_t* lout = out.prep_msgs + (size_t)r * p.prep_share_len;
    F::store(lout, 0, v);
    F::store(lout, 1, f);
    F::store(lout, 2, pt);
    *(uint4*)(lout + (size_t)p.verifier_len * F::ES) = sc.part[r];
    out.status[r] = status;
  } else {
  // decide against the leader's verifier share [v, f(t), p(t)]
  const uint8_t* lps = in.leader + (size_t)r * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    const T x = F::load(lps, e);
    if (!F::lt_p(x)) decode_ok = false;
    return x;
  };
  const T V0 = F::add(lv(0), v);
  const T fa = F::add(lv(1), f);
  const T G = F::sub(F::mul(fa, fa), fa);
  const T PT = F::add(lv(2), pt);
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
  // truncate: sum_b 2^b m_b
  if (K <= 32) {  // shift-and-add over 160 bits (< 2^160 for at most 32 steps)
    sum128 acc;
    sum_zero(acc);
    for (uint32_t i = K; i-- > 0;) {
      const T m = ldf<F>(sc.meas, i, ld, r);
      acc.w[4] = __builtin_amdgcn_alignbit(acc.w[4], acc.w[3], 31);
      acc.w[3] = __builtin_amdgcn_alignbit(acc.w[3], acc.w[2], 31);
      acc.w[2] = __builtin_amdgcn_alignbit(acc.w[2], acc.w[1], 31);
      acc.w[1] = __builtin_amdgcn_alignbit(acc.w[1], acc.w[0], 31);
      acc.w[0] <<= 1;
      sum_add(acc, m);
    }
    F::store(sc.out, r, sum_reduce(acc));
  } else {
    T acc = Z, pw = one;
    for (uint32_t i = 0; i < K; i++) {
      acc = F::add(acc, F::mul(pw, ldf<F>(sc.meas, i, ld, r)));
      pw = F::add(pw, pw);
    }
    F::store(sc.out, r, acc);
  }
}

}  // namespace qsum
