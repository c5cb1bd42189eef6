// prio3_query_wide.h -- the eight-lanes-per-report ParallelSum(Mul) query body (k_query_w,
// prio3_query_wide.hip), shared with the fused XOF + query kernel of prio3_engine.hip
// (k_prep_w).  See prio3_query_wide.hip for the algorithm.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"

namespace qwide {


typedef Fp128 F;
typedef f128 T;

DEV T shfl_xor128(const T& x, int m) {
  return mk128((uint32_t)__shfl_xor((int)x.w[0], m), (uint32_t)__shfl_xor((int)x.w[1], m),
               (uint32_t)__shfl_xor((int)x.w[2], m), (uint32_t)__shfl_xor((int)x.w[3], m));
}
DEV T shfl128(const T& x, int src) {
  return mk128((uint32_t)__shfl((int)x.w[0], src), (uint32_t)__shfl((int)x.w[1], src),
               (uint32_t)__shfl((int)x.w[2], src), (uint32_t)__shfl((int)x.w[3], src));
}
// sum over the 8 lanes of a report (every lane gets the total)
DEV T group_sum(T x) {
  x = F::add(x, shfl_xor128(x, 1));
  x = F::add(x, shfl_xor128(x, 2));
  return F::add(x, shfl_xor128(x, 4));
}
// a^l for a lane-dependent l < 8, from a, a^2, a^4 (no dynamic register indexing)
DEV T lane_pow(const T& a1, const T& a2, const T& a4, uint32_t l) {
  const T one = F::one();
  const T x = F::sel(l & 1u, a1, one);
  return F::mul(F::mul(x, F::sel(l & 2u, a2, one)), F::sel(l & 4u, a4, one));
}
// a <- 2a + m over a 160-bit accumulator (no reduction; < 2^160 for at most 32 steps)
DEV void horner2(sum128& a, const T& m) {
  a.w[4] = __builtin_amdgcn_alignbit(a.w[4], a.w[3], 31);
  a.w[3] = __builtin_amdgcn_alignbit(a.w[3], a.w[2], 31);
  a.w[2] = __builtin_amdgcn_alignbit(a.w[2], a.w[1], 31);
  a.w[1] = __builtin_amdgcn_alignbit(a.w[1], a.w[0], 31);
  a.w[0] <<= 1;
  sum_add(a, m);
}
DEV T ldm(const void* base, uint32_t row, bool valid, size_t ld, uint32_t r) {
  // one dwordx4 load from a clamped (always in-bounds) row, zeroed by mask when invalid
  const uint32_t msk = valid ? 0xffffffffu : 0u;
  const uint4 v = ((const uint4*)base)[(size_t)(valid ? row : 0u) * ld + r];
  return mk128(v.x & msk, v.y & msk, v.z & msk, v.w & msk);
}

// r: the report, l: this lane's place in the report's group of 8 consecutive lanes of the wave.
// slow_defer / redo (DevParams): as query_h_body -- a group whose report the XOF flagged leaves
// here (all 8 lanes: the flag is the report's) and is redone by the run's redo launch.
template <int PQ, int LOGQ, int GS>
__device__ __forceinline__ void query_w_body(const DevParams& p, const InPtrs& in,
                                             const Scratch& sc, const OutPtrs& out,
                                             const uint32_t r, const uint32_t l) {
  constexpr uint32_t P = 8 * PQ;
  // the 8 lanes of a report stay together for the group sums; a group past n computes on report
  // n - 1 and stores nothing
  const bool live = r < p.n;
  const uint32_t rr = live ? r : p.n - 1;
  if (live) {
    if (p.redo) {
      if (sc.flag[r] != 2) return;
    } else if (p.slow_defer && sc.flag[r]) {
      return;
    }
  } else if (p.redo) {
    return;
  }
  const size_t ld = p.ld;
  const uint32_t A = p.arity, C = p.chunk, M = p.meas_len, K = p.calls;
  const T one = F::one(), Z = F::zero();
  uint8_t status = PRIO3_STATUS_FINISHED;
  // ---- Lagrange basis (four-step DFT, see the header)
  T x[PQ];
  {
    const T t = ldf<F>(sc.qr, 0, ld, rr);
    T tq = F::mul(t, t);
    tq = F::mul(tq, tq);
#pragma unroll
    for (int i = 2; i < LOGQ; i++) tq = F::mul(tq, tq);  // t^PQ
    T tP = tq;
#pragma unroll
    for (int i = 0; i < 3; i++) tP = F::mul(tP, tP);
    if (F::eq(tP, one)) status = PRIO3_STATUS_PREP_INIT;  // t is a P-th root of unity
    // P = 64 / 128: tw128[k] = alpha_PQ^k (k < PQ/2), tw128[8 + i] = alpha_P^i (i < 8), so
    // alpha_8 = alpha_PQ^(PQ/8).  P = 32: tw128[i] = alpha_32^i (i < 16), alpha_8 = tw128[4].
    constexpr int I8 = PQ == 4 ? 4 : PQ / 8, I4 = PQ == 4 ? 8 : PQ / 4;
    constexpr int IP = PQ == 4 ? 0 : 8;  // alpha_P^i at tw128[IP + i]
    const T w8l = lane_pow(F::from_words(p.tw128[I8]), F::from_words(p.tw128[I4]),
                           F::sub(Z, one), l);
    const T wl = lane_pow(F::from_words(p.tw128[IP + 1]), F::from_words(p.tw128[IP + 2]),
                          F::from_words(p.tw128[IP + 4]), l);
    const T z = F::mul(tq, w8l);
    T g = F::add(z, one);
#pragma unroll
    for (int i = 0; i < 6; i++) g = F::add(F::mul(g, z), one);
    T y = F::mul(g, FC<F>::invP(p));
    const T ratio = F::mul(t, wl);
#pragma unroll
    for (int n2 = 0; n2 < PQ; n2++) {
      x[__builtin_bitreverse32(n2) >> (32 - LOGQ)] = y;
      if (n2 + 1 < PQ) y = F::mul(y, ratio);
    }
    dft_reg<PQ, LOGQ>(p, x, PQ == 4 ? 8 : 1);  // P = 32: alpha_4^i = alpha_32^(8i)
  }
  // x[m] = L_c, c = (P - 8m - l) mod P.  L_0 is lane 0's x[0].
  const T L0 = shfl128(x[0], (int)(threadIdx.x & 56u));
  // ---- beta_(c-1) = L_c rho^(c-1), rho = r0^C; L_c and beta to scratch, sum of L_1..L_K
  const T r0 = ldf<F>(sc.jr, 0, ld, rr);
  T sumL;
  {
    T rho = one, sq = r0;
    for (uint32_t e = C; e; e >>= 1) {
      if (e & 1) rho = F::mul(rho, sq);
      if (e > 1) sq = F::mul(sq, sq);
    }
    const T rho2 = F::mul(rho, rho), rho4 = F::mul(rho2, rho2), rho8 = F::mul(rho4, rho4);
    // this lane's smallest c >= 1 is 8 - l (l > 0) or 8 (l = 0): rho^(7 - l)
    T rk = lane_pow(rho, rho2, rho4, 7u - l);
    sum128 sl;
    sum_zero(sl);
#pragma unroll
    for (int mm = PQ - 1; mm >= 0; mm--) {
      const uint32_t c = (P - 8u * (uint32_t)mm - l) & (P - 1);
      if (c != 0) {
        if (c <= K) {
          sum_add(sl, x[mm]);
          if (live) {
            F::store(sc.Lbuf, (size_t)c * ld + r, x[mm]);
            F::store(sc.beta, (size_t)(c - 1) * ld + r, F::mul(x[mm], rk));
          }
        }
        if (mm > 0) rk = F::mul(rk, rho8);
      }
    }
    sumL = group_sum(sum_reduce(sl));
  }
  const T half = FC<F>::half(p);
  const T halfL = F::mul(half, sumL);
  // ---- the wire sweeps: lane l owns columns j = (s GS + q) 8 + l of sweep s
  const uint8_t* lps = in.leader + (size_t)rr * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    const T v = F::load(lps, e);
    if (!F::lt_p(v)) decode_ok = false;
    return v;
  };
  // the group reads rows other lanes just wrote: their stores must have reached L2
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sum128 Ssum;
  sum_zero(Ssum);
  T Gsum = Z;  // gadget outputs of this lane's columns
  const T r02 = F::mul(r0, r0), r04 = F::mul(r02, r02), r08 = F::mul(r04, r04);
  T rj = F::mul(r0, lane_pow(r0, r02, r04, l));  // r0^(j+1) for j = l
  const uint32_t NSW = (C + 8 * GS - 1) / (8 * GS);
  for (uint32_t s = 0; s < NSW; s++) {
    mac128 Aa[GS], Bb[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) {
      mac_zero(Aa[q]);
      mac_zero(Bb[q]);
    }
    auto fetch = [&](uint32_t k, T* dst) {
#pragma unroll
      for (int q = 0; q < GS; q++) {
        const uint32_t j = (s * GS + (uint32_t)q) * 8u + l, i = k * C + j;
        dst[q] = ldm(sc.meas, i, k < K && j < C && i < M, ld, rr);
      }
    };
    T mc[GS];
    fetch(0, mc);
    T be = ldf<F>(sc.beta, 0, ld, rr), Lk = ldf<F>(sc.Lbuf, 1, ld, rr);
#pragma unroll 1
    for (uint32_t k = 0; k < K; k++) {
      T mn[GS];
      fetch(k + 1, mn);
      const uint32_t kn = k + 1 < K ? k + 1 : k;
      const T be_n = ldf<F>(sc.beta, kn, ld, rr), L_n = ldf<F>(sc.Lbuf, kn + 1, ld, rr);
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
    // f_2j(t) = seed_2j L0 + r^(j+1) A_j, f_2j+1(t) = seed_2j+1 L0 + B_j - L/2; gadget products
    // of this lane's columns summed lazily
#pragma unroll
    for (int q = 0; q < GS; q++) {
      const uint32_t j = (s * GS + (uint32_t)q) * 8u + l;
      if (j < C) {
        // compiler-scheduled reductions here: the asm ones pin v40-v68 while the other columns'
        // accumulators are live
        mac_add(Bb[q], ldf<F>(sc.proofs, 2 * j + 1, ld, rr), L0);
        const T f1 = F::sub(mac_reduce(Bb[q]), halfL);
        const T Aq = mac_reduce(Aa[q]);
        mac128 F0;
        mac_zero(F0);
        mac_add(F0, ldf<F>(sc.proofs, 2 * j, ld, rr), L0);
        mac_add(F0, rj, Aq);
        const T f0 = mac_reduce(F0);
        Gsum = F::add(Gsum, mul128(F::add(lv(1 + 2 * j), f0), F::add(lv(2 + 2 * j), f1)));
      }
      rj = F::mul(rj, r08);
    }
  }
  // ---- (after the sweeps, fewer live registers there) p(t) and range = sum_(c=1..K) p(alpha^c) = sum_e coef_e sigma_(e mod P); lane l takes
  // the coefficients e = 8q + l: p(t) = sum_l t^l sum_q coef_(8q+l) (t^8)^q
  T pt, range;
  {
    const uint32_t GL = p.glen, NQ = (GL + 7) / 8;
    const T t = ldf<F>(sc.qr, 0, ld, rr);
    const T t2 = F::mul(t, t), t4 = F::mul(t2, t2), t8 = F::mul(t4, t4);
    const uint4* sig = p.sigma_dev;
    mac128 R;
    mac_zero(R);
    T acc = Z;
    constexpr int HD = 8;
    for (uint32_t q0 = 0; q0 < NQ; q0 += HD) {  // q descending: q = NQ - 1 - (q0 + h)
      T cf[HD], sg[HD];
#pragma unroll
      for (int h = 0; h < HD; h++) {
        const int q = (int)NQ - 1 - (int)(q0 + h);
        const uint32_t e = 8u * (uint32_t)(q < 0 ? 0 : q) + l;
        const bool valid = q >= 0 && e < GL;
        cf[h] = ldm(sc.proofs, A + e, valid, ld, rr);
        const uint4 s = sig[e & (P - 1)];
        sg[h] = mk128(s.x, s.y, s.z, s.w);
      }
#pragma unroll
      for (int h = 0; h < HD; h++) {
        if (q0 + h < NQ) {  // uniform
          acc = F::add(F::mul(acc, t8), cf[h]);
          mac_add(R, cf[h], sg[h]);
        }
      }
    }
    pt = group_sum(F::mul(acc, lane_pow(t, t2, t4, l)));
    range = group_sum(mac_reduce_f(R));
  }
  const T G = group_sum(Gsum);
  const T S = group_sum(sum_reduce(Ssum));
  T v;
  if (p.kind == PRIO3_SUMVEC) {
    v = range;
  } else {
    const T r1 = ldf<F>(sc.jr, 1, ld, rr);
    v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), F::sub(S, half)));
  }
  const T V0 = F::add(lv(0), v);
  const T PT = F::add(lv(A + 1), pt);
  int bad = decode_ok ? 0 : 1;
  bad |= __shfl_xor(bad, 1);
  bad |= __shfl_xor(bad, 2);
  bad |= __shfl_xor(bad, 4);
  if (l == 0 && live) {
    if (status == PRIO3_STATUS_FINISHED) {
      if (bad)
        status = PRIO3_STATUS_PREP_SHARE_DECODE;
      else if (!F::is_zero(V0) || !F::eq(G, PT))
        status = PRIO3_STATUS_PREP_MSG;
    }
    // prepare message: joint-rand seed of (leader part, helper part), checked against the
    // corrected seed (prepare_next)
    uint32_t lpart[4], msg[4];
    load16(lps + (size_t)p.verifier_len * F::ES, lpart);
    if (!prep_msg_check(p, in, sc, r, lpart, msg) && status == PRIO3_STATUS_FINISHED)
      status = PRIO3_STATUS_PREP_NEXT;
    if (status != PRIO3_STATUS_FINISHED) msg[0] = msg[1] = msg[2] = msg[3] = 0;
    ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
    out.status[r] = status;
  }
  // ---- truncate (SumVec): entry e = sum_b 2^b m_(e bits + b), entries e = l mod 8 per lane
  if (p.kind == PRIO3_SUMVEC && live && !p.trunc_xof) {
    const uint32_t nb = p.bits;  // <= 32 (launcher)
    for (uint32_t e = l; e < p.out_len; e += 8) {
      sum128 a;
      sum_zero(a);
      for (uint32_t hi = nb; hi > 0;) {
        const uint32_t cnt = hi < 8 ? hi : 8;
        T m[8];
#pragma unroll
        for (int b = 0; b < 8; b++)
          m[b] = ldm(sc.meas, e * nb + hi - 1 - (uint32_t)b, (uint32_t)b < cnt, ld, r);
#pragma unroll
        for (int b = 0; b < 8; b++)
          if ((uint32_t)b < cnt) horner2(a, m[b]);
        hi -= cnt;
      }
      F::store(sc.out, (size_t)e * ld + r, sum_reduce(a));
    }
  }
}

}  // namespace qwide
