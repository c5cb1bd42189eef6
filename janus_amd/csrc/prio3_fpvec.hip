// prio3_fpvec.hip -- helper FLP query + decide + prepare message + prepare_next + truncate for
// Prio3FixedPointBoundedL2VecSum (Janus VdafInstance::Prio3FixedPointBoundedL2VecSum,
// /root/reference/core/src/vdaf.rs:292-335; config C5 of BASELINE.json), MI355X (gfx950).
//
// The XOF half of prepare_init (measurement / proofs share expansion, joint-rand part over the
// 2.56 MB measurement share, corrected seed, joint randomness, two query-randomness elements)
// is the engine's dual-state k_xofd (k_xof with split_xof=0); this file is the two-gadget
// query that follows it.  The
// circuit is the reconstruction fixed in oracle/fpvec_py.py:
//   gadget 0 = ParallelSum(Mul, C0): range checks of every bit (SumVec's construction, r0);
//   gadget 1 = ParallelSum(PolyEval(y^2 - 2^n y), C1) over the decoded entries y_e;
//   v = r1 * range + r1^2 * (sum gadget-1 outputs + entries 2^(2n-2)/2 - claimed norm).
// One report per lane, SoA scratch [element][report] (sub-batch leading dimension p.ld);
// output shares (the decoded entries) go to sc.out with leading dimension p.ld_out.
//
// Per report (10^4 entries, n = 16): the measurement share (160,030 elements) is read twice --
// once by the gadget-0 sweep (2 Field128 multiplies per element) and once by the entry decode
// of the gadget-1 sweep (doublings only) -- and 10^4 output elements are written.
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"
#include "prio3_wide.h"

namespace {

typedef Fp128 F;
typedef f128 T;

// Lagrange basis on the P-th roots at t (scaled DFT of t^e / P, reversed as in k_query_ps) into
// rows [0, P) of L, and the gadget polynomial's values at the P-th roots into rows [0, P) of PV.
DEV void basis_and_roots(const DevParams& p, uint8_t* L, uint8_t* PV, const void* proofs,
                         uint32_t coeff_off, uint32_t glen, uint32_t P, uint32_t logP, T invP,
                         T t, uint32_t r) {
  const size_t ld = p.ld;
  T pw = invP;
  for (uint32_t e = 0; e < P; e++) {
    F::store(L, (size_t)bitrev(e, logP) * ld + r, pw);
    pw = F::mul(pw, t);
  }
  dft_lane<F>(p, L, r, P, logP);
  for (uint32_t e = 0; e < P; e++) {
    T q = ldf<F>(proofs, coeff_off + e, ld, r);
    for (uint32_t e2 = e + P; e2 < glen; e2 += P) q = F::add(q, ldf<F>(proofs, coeff_off + e2, ld, r));
    F::store(PV, (size_t)bitrev(e, logP) * ld + r, q);
  }
  dft_lane<F>(p, PV, r, P, logP);
}

DEV T horner(const void* proofs, uint32_t off, uint32_t len, T t, size_t ld, uint32_t r) {
  T acc = F::zero();
  for (uint32_t e = len; e-- > 0;) acc = F::add(F::mul(acc, t), ldf<F>(proofs, off + e, ld, r));
  return acc;
}

DEV bool root_of_unity(T t, uint32_t logP) {
  for (uint32_t l = 0; l < logP; l++) t = F::mul(t, t);
  return F::eq(t, F::one());
}

// y = sum_b 2^b m[base + b] (Field128::decode_bitvector), Horner from the top bit
DEV T decode_bits(const void* meas, uint32_t base, uint32_t nbits, size_t ld, uint32_t r) {
  T y = F::zero();
  for (uint32_t b = nbits; b-- > 0;) y = F::add(F::add(y, y), ldf<F>(meas, base + b, ld, r));
  return y;
}

// the same for nbits a multiple of 16: each 16-bit group's loads are issued together (the
// generic loop waits out one HBM latency per bit: 16 x 10^4 serialized misses per report)
DEV T decode_bits16(const void* meas, uint32_t base, uint32_t nbits, size_t ld, uint32_t r) {
  T y = F::zero();
  for (uint32_t hi = nbits; hi > 0; hi -= 16) {
    T m[16];
#pragma unroll
    for (int b = 0; b < 16; b++) m[b] = ldf<F>(meas, base + hi - 16 + b, ld, r);
#pragma unroll
    for (int b = 15; b >= 0; b--) y = F::add(F::add(y, y), m[b]);
  }
  return y;
}

template <int GS>
__global__ __launch_bounds__(256) void k_query_fp(DevParams p, InPtrs in, Scratch sc, OutPtrs out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  const size_t ld = p.ld;
  const uint32_t P0 = p.P, A0 = p.arity, C0 = p.chunk, M = p.meas_len, K0 = p.calls;
  const uint32_t P1 = p.P1, C1 = p.chunk1, K1 = p.calls1, E = p.out_len, nb = p.bits;
  const uint32_t off1 = A0 + p.glen;  // proof: seeds0 | coeffs0 | seeds1 | coeffs1
  DCHECK(r < p.ld && off1 + C1 + p.glen1 <= p.proof_len && K0 * C0 >= M && K1 * C1 >= E);
  DCHECK(p.ld_out >= p.n && nb * E + 2 * nb - 2 == M);
  uint8_t status = PRIO3_STATUS_FINISHED;
  const T t0 = ldf<F>(sc.qr, 0, ld, r), t1 = ldf<F>(sc.qr, 1, ld, r);
  if (root_of_unity(t0, p.logP) || root_of_unity(t1, p.logP1)) status = PRIO3_STATUS_PREP_INIT;
  uint8_t* L = (uint8_t*)sc.Lbuf;
  uint8_t* PV = (uint8_t*)sc.PVbuf;
  uint8_t* L1 = L + (size_t)F::ES * P0 * ld;
  uint8_t* PV1 = PV + (size_t)F::ES * P0 * ld;
  basis_and_roots(p, L, PV, sc.proofs, A0, p.glen, P0, p.logP, FC<F>::invP(p), t0, r);
  basis_and_roots(p, L1, PV1, sc.proofs, off1 + C1, p.glen1, P1, p.logP1,
                  F::from_words(p.invP1_128), t1, r);
  auto Lc0 = [&](uint32_t c) { return ldf<F>(L, (P0 - c) & (P0 - 1), ld, r); };
  auto Lc1 = [&](uint32_t c) { return ldf<F>(L1, (P1 - c) & (P1 - 1), ld, r); };
  const T p0t = horner(sc.proofs, A0, p.glen, t0, ld, r);
  const T p1t = horner(sc.proofs, off1 + C1, p.glen1, t1, ld, r);

  // gadget 0: range checks (k_query_ps's sweep): beta_k = L_(k+1)(t0) r0^(C0 k)
  const T r0 = ldf<F>(sc.jr, 0, ld, r), r1 = ldf<F>(sc.jr, 1, ld, r);
  T rC = F::one();
  for (uint32_t j = 0; j < C0; j++) rC = F::mul(rC, r0);
  T sumL = F::zero(), range = F::zero(), normg = F::zero();
  {
    T rk = F::one();
    for (uint32_t k = 0; k < K0; k++) {
      const T Lk = Lc0(k + 1);
      sumL = F::add(sumL, Lk);
      range = F::add(range, ldf<F>(PV, k + 1, ld, r));
      F::store(sc.beta, (size_t)k * ld + r, F::mul(Lk, rk));
      rk = F::mul(rk, rC);
    }
    for (uint32_t k = 0; k < K1; k++) normg = F::add(normg, ldf<F>(PV1, k + 1, ld, r));
  }
  const T L00 = Lc0(0), L10 = Lc1(0);
  const T halfL = F::mul(FC<F>::half(p), sumL);
  const uint8_t* lps = in.leader + (size_t)r * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    T x = F::load(lps, e);
    if (!F::lt_p(x)) decode_ok = false;
    return x;
  };
  const T Z = F::zero();
  T G0 = F::zero(), rj = r0;
  for (uint32_t jg = 0; jg < C0; jg += GS) {
    T Aa[GS], Bb[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) Aa[q] = Bb[q] = Z;
    // software-pipelined: call k+1's beta, L and meas loads are in flight while call k's
    // products run (a lone wave per SIMD has nothing else to hide the HBM latency with);
    // invalid slots load element 0 and are zeroed at use, so no select waits on a load early
    auto ldm = [&](uint32_t k, int q) {
      const uint32_t i = k * C0 + jg + (uint32_t)q;
      return ldf<F>(sc.meas, (jg + q < C0 && i < M) ? i : 0, ld, r);
    };
    T be_n = ldf<F>(sc.beta, 0, ld, r), Lk_n = Lc0(1), mn[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) mn[q] = ldm(0, q);
#pragma unroll 1
    for (uint32_t k = 0; k < K0; k++) {
      const T be = be_n, Lk = Lk_n;
      T mc[GS];
#pragma unroll
      for (int q = 0; q < GS; q++) mc[q] = mn[q];
      const uint32_t kn = k + 1 < K0 ? k + 1 : k;  // the last pass reloads its own call
      be_n = ldf<F>(sc.beta, kn, ld, r);
      Lk_n = Lc0(kn + 1);
#pragma unroll
      for (int q = 0; q < GS; q++) mn[q] = ldm(kn, q);
      const uint32_t base = k * C0 + jg;
#pragma unroll
      for (int q = 0; q < GS; q++) {
        const bool valid = (jg + q < C0) && (base + q < M);
        const T m = F::sel(valid, mc[q], Z);
        Aa[q] = F::add(Aa[q], F::mul(be, m));
        Bb[q] = F::add(Bb[q], F::mul(Lk, m));
      }
    }
#pragma unroll
    for (int q = 0; q < GS; q++) {
      const uint32_t j = jg + q;
      const bool valid = j < C0;
      const uint32_t jj = valid ? j : 0;
      const T f0 = F::add(F::mul(ldf<F>(sc.proofs, 2 * jj, ld, r), L00), F::mul(rj, Aa[q]));
      const T f1 = F::sub(F::add(F::mul(ldf<F>(sc.proofs, 2 * jj + 1, ld, r), L00), Bb[q]), halfL);
      const T prod = F::mul(F::add(lv(1 + 2 * jj), f0), F::add(lv(2 + 2 * jj), f1));
      G0 = F::add(G0, F::sel(valid, prod, Z));
      rj = F::sel(valid, F::mul(rj, r0), rj);
    }
  }

  // gadget 1: wires are the decoded entries y_(k C1 + j) (zero padded); each entry is decoded
  // once here and written as the output share (truncate)
  const T twon = F::from_words(p.twon128);
  T G1 = F::zero();
  for (uint32_t jg = 0; jg < C1; jg += GS) {
    T Ac[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) Ac[q] = Z;
#pragma unroll 1
    for (uint32_t k = 0; k < K1; k++) {
      const T Lk = Lc1(k + 1);
#pragma unroll
      for (int q = 0; q < GS; q++) {
        const uint32_t idx = k * C1 + jg + q;
        if (jg + q < C1 && idx < E) {
          T y;
          if (p.trunc_xof) {  // decoded by the XOF kernel as it squeezed the share
            y = F::load(sc.out, (size_t)idx * p.ld_out + r);
          } else {
            y = decode_bits16(sc.meas, nb * idx, nb, ld, r);  // nb is 16 or 32
            DCHECK(nb * idx + nb <= M);
            F::store(sc.out, (size_t)idx * p.ld_out + r, y);
          }
          Ac[q] = F::add(Ac[q], F::mul(Lk, y));
        }
      }
    }
#pragma unroll
    for (int q = 0; q < GS; q++) {
      const uint32_t j = jg + q;
      const bool valid = j < C1;
      const uint32_t jj = valid ? j : 0;
      const T f = F::add(F::mul(ldf<F>(sc.proofs, off1 + jj, ld, r), L10), Ac[q]);
      const T a = F::add(lv(2 + A0 + jj), f);
      const T qa = F::sub(F::mul(a, a), F::mul(twon, a));
      G1 = F::add(G1, F::sel(valid, qa, Z));
    }
  }
  const T claimed = decode_bits(sc.meas, nb * E, 2 * nb - 2, ld, r);
  const T normd = F::sub(F::add(normg, F::from_words(p.normc128)), claimed);
  const T v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), normd));

  const T V0 = F::add(lv(0), v);
  const T PT0 = F::add(lv(1 + A0), p0t);
  const T PT1 = F::add(lv(2 + A0 + C1), p1t);
  if (status == PRIO3_STATUS_FINISHED) {
    if (!decode_ok)
      status = PRIO3_STATUS_PREP_SHARE_DECODE;
    else if (!F::is_zero(V0) || !F::eq(G0, PT0) || !F::eq(G1, PT1))
      status = PRIO3_STATUS_PREP_MSG;
  }
  // prepare message = joint-rand seed of (leader part, helper part); prepare_next checks it
  // against the corrected seed
  uint32_t lpart[4], hpart[4];
  load16(lps + (size_t)p.verifier_len * F::ES, lpart);
  {
    const uint4 hp = sc.part[r];
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
  const uint4 cor = sc.corrected[r];
  uint32_t msg[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
  if (status == PRIO3_STATUS_FINISHED &&
      (msg[0] != cor.x || msg[1] != cor.y || msg[2] != cor.z || msg[3] != cor.w))
    status = PRIO3_STATUS_PREP_NEXT;
  if (status != PRIO3_STATUS_FINISHED) msg[0] = msg[1] = msg[2] = msg[3] = 0;
  ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
  out.status[r] = status;
}

// ------------------------------------------------------------------------------------
// k_query_fpw<GS>: the same query and decide with EIGHT lanes per report (k_query_w's layout,
// prio3_query_wide.hip).  At 10^4 entries a sub-batch holds ~50k reports: one lane per report
// is 0.76 waves per SIMD and every product a fully reduced Field128 multiply (r02l: 85 ms per
// 50k).  Here:
//   * both Lagrange bases (P0 = 512, P1 = 128) by the group's four-step DFT on the geometric
//     input t^e / P (wide::lagrange_group), no HBM round trips per butterfly;
//   * range = sum_e coef0_e sigma0_(e mod P0), the norm sum = sum_e coef1_e sigma1_(e mod P1)
//     (sigma tables on the device), so neither gadget polynomial is evaluated on the roots;
//   * gadget-0 wire sums as lazily reduced MACs, the C0 columns dealt over the 8 lanes, GS per
//     lane and sweep (beta_k, L_(k+1) loads shared by the group);
//   * gadget-1 wires from the entries the XOF decoded (trunc_xof) or decoded here.
// ------------------------------------------------------------------------------------
// LEADER = 1: the leader's prepare_init (agg_id 0) on the same data flow -- the verifier share
// [v, f0 wires, p0(t0), f1 wires, p1(t1)] || joint-rand part goes to out.prep_msgs (stride
// prep_share_len) instead of being decided against a peer's share; out.status holds the unpack
// verdict on entry; the entries (output share) are decoded here (trunc_xof = 0).
template <int GS, int LEADER = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_query_fpw(
    DevParams p, InPtrs in, Scratch sc, OutPtrs out) {
  using namespace wide;
  constexpr int GS1 = 4;
  const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
  const uint32_t l = tid & 7u, r = tid >> 3;
  const bool live = r < p.n;
  const uint32_t rr = live ? r : p.n - 1;  // a group past n computes on report n - 1, stores nothing
  const size_t ld = p.ld;
  const uint32_t P0 = p.P, A0 = p.arity, C0 = p.chunk, M = p.meas_len, K0 = p.calls;
  const uint32_t P1 = p.P1, C1 = p.chunk1, K1 = p.calls1, E = p.out_len, nb = p.bits;
  const uint32_t off1 = A0 + p.glen;  // proof: seeds0 | coeffs0 | seeds1 | coeffs1
  DCHECK(rr < p.ld && off1 + C1 + p.glen1 <= p.proof_len && K0 * C0 >= M && K1 * C1 >= E);
  DCHECK(p.ld_out >= p.n && nb * E + 2 * nb - 2 == M);
  const T one = F::one(), Z = F::zero();
  uint8_t status = PRIO3_STATUS_FINISHED;
  if (LEADER && live) status = out.status[r];
  uint8_t* lout = LEADER ? out.prep_msgs + (size_t)rr * p.prep_share_len : nullptr;
  uint8_t* L = (uint8_t*)sc.Lbuf;                   // rows [0, P0): L_c(t0)
  uint8_t* L1 = L + (size_t)F::ES * P0 * ld;        // rows [0, P1): L_c(t1)
  // ---- Lagrange bases: L_c for c = 1..K to scratch rows c, L_0 and the sum of L0_1..L0_K0
  T L00 = Z, L10 = Z, halfL;
  {
    const T t0 = ldf<F>(sc.qr, 0, ld, rr), t1 = ldf<F>(sc.qr, 1, ld, rr);
    if (F::eq(sqr_n(t0, (int)p.logP), one) || F::eq(sqr_n(t1, (int)p.logP1), one))
      status = PRIO3_STATUS_PREP_INIT;
    sum128 sl;
    sum_zero(sl);
    lagrange_group(p, p.logP, FC<F>::invP(p), t0, l, [&](uint32_t i, const T& v) {
      const uint32_t c = (P0 - i) & (P0 - 1);
      if (c == 0) {
        L00 = v;
      } else if (c <= K0) {
        sum_add(sl, v);
        if (live) F::store(L, (size_t)c * ld + r, v);
      }
    });
    lagrange_group(p, p.logP1, F::from_words(p.invP1_128), t1, l, [&](uint32_t i, const T& v) {
      const uint32_t c = (P1 - i) & (P1 - 1);
      if (c == 0)
        L10 = v;
      else if (c <= K1 && live)
        F::store(L1, (size_t)c * ld + r, v);
    });
    L00 = group_sum(L00);  // one lane holds it, the others zero
    L10 = group_sum(L10);
    halfL = F::mul(FC<F>::half(p), group_sum(sum_reduce(sl)));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the group reads rows other lanes wrote
  // ---- beta_k = L0_(k+1) rho^k, rho = r0^C0; lane l takes calls [l per, (l + 1) per)
  const T r0 = ldf<F>(sc.jr, 0, ld, rr);
  {
    T rho = one, sq = r0;
    for (uint32_t e = C0; e; e >>= 1) {
      if (e & 1) rho = F::mul(rho, sq);
      if (e > 1) sq = F::mul(sq, sq);
    }
    const uint32_t per = (K0 + 7) / 8, k0 = l * per, k1 = min(K0, k0 + per);
    T rk = one;  // rho^k0: square-and-multiply over the lane's own exponent
    sq = rho;
    for (uint32_t e = k0, hi = (K0 + 7) / 8 * 7; hi; hi >>= 1, e >>= 1) {
      rk = F::sel(e & 1u, F::mul(rk, sq), rk);
      sq = F::mul(sq, sq);
    }
    for (uint32_t k = k0; k < k1; k++) {
      const T Lk = ldf<F>(L, k + 1, ld, rr);
      if (live) F::store(sc.beta, (size_t)k * ld + r, F::mul(Lk, rk));
      rk = F::mul(rk, rho);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint8_t* lps = in.leader + (size_t)rr * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    const T v = F::load(lps, e);
    if (!F::lt_p(v)) decode_ok = false;
    return v;
  };
  // ---- gadget 0: lane l owns columns j = (s GS + q) 8 + l
  T G0 = Z;
  {
    const T r02 = F::mul(r0, r0), r04 = F::mul(r02, r02), r08 = F::mul(r04, r04);
    T rj = F::mul(r0, lane_pow(r0, r02, r04, l));  // r0^(j+1)
    const uint32_t NSW = (C0 + 8 * GS - 1) / (8 * GS);
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
          const uint32_t j = (s * GS + (uint32_t)q) * 8u + l, i = k * C0 + j;
          dst[q] = ldm(sc.meas, i, k < K0 && j < C0 && i < M, ld, rr);
        }
      };
      T mc[GS];
      fetch(0, mc);
      T be = ldf<F>(sc.beta, 0, ld, rr), Lk = ldf<F>(L, 1, ld, rr);
#pragma unroll 1
      for (uint32_t k = 0; k < K0; k++) {
        T mn[GS];
        fetch(k + 1, mn);
        const uint32_t kn = k + 1 < K0 ? k + 1 : k;
        const T be_n = ldf<F>(sc.beta, kn, ld, rr), L_n = ldf<F>(L, kn + 1, ld, rr);
#pragma unroll
        for (int q = 0; q < GS; q++) {
          mac_add(Aa[q], be, mc[q]);
          mac_add(Bb[q], Lk, mc[q]);
        }
#pragma unroll
        for (int q = 0; q < GS; q++) mc[q] = mn[q];
        be = be_n;
        Lk = L_n;
      }
#pragma unroll
      for (int q = 0; q < GS; q++) {
        const uint32_t j = (s * GS + (uint32_t)q) * 8u + l;
        if (j < C0) {
          mac_add(Bb[q], ldf<F>(sc.proofs, 2 * j + 1, ld, rr), L00);
          const T f1 = F::sub(mac_reduce(Bb[q]), halfL);
          const T Aq = mac_reduce(Aa[q]);
          mac128 F0;
          mac_zero(F0);
          mac_add(F0, ldf<F>(sc.proofs, 2 * j, ld, rr), L00);
          mac_add(F0, rj, Aq);
          const T f0 = mac_reduce(F0);
          if constexpr (LEADER) {
            if (live) {
              F::store(lout, 1 + 2 * j, f0);
              F::store(lout, 2 + 2 * j, f1);
            }
          } else {
            G0 = F::add(G0, mul128(F::add(lv(1 + 2 * j), f0), F::add(lv(2 + 2 * j), f1)));
          }
        }
        rj = F::mul(rj, r08);
      }
    }
  }
  // ---- gadget 1: wires are the entries y_(k C1 + j); lane l owns columns j = (s GS1 + q) 8 + l
  T G1 = Z;
  {
    const T twon = F::from_words(p.twon128);
    const uint32_t NSW = (C1 + 8 * GS1 - 1) / (8 * GS1);
    for (uint32_t s = 0; s < NSW; s++) {
      mac128 Ac[GS1];
#pragma unroll
      for (int q = 0; q < GS1; q++) mac_zero(Ac[q]);
#pragma unroll 1
      for (uint32_t k = 0; k < K1; k++) {
        const T Lk = ldf<F>(L1, k + 1, ld, rr);
#pragma unroll
        for (int q = 0; q < GS1; q++) {
          const uint32_t j = (s * GS1 + (uint32_t)q) * 8u + l, idx = k * C1 + j;
          const bool valid = j < C1 && idx < E;
          T y;
          if (p.trunc_xof) {  // decoded by the XOF kernel as it squeezed the share
            y = ldm(sc.out, idx, valid, p.ld_out, rr);
          } else {
            sum128 a;
            sum_zero(a);
            T m[16];
            for (uint32_t hi = nb; hi > 0; hi -= 16) {  // nb is 16 or 32
#pragma unroll
              for (int b = 0; b < 16; b++)
                m[b] = ldm(sc.meas, nb * idx + hi - 1 - (uint32_t)b, valid, ld, rr);
#pragma unroll
              for (int b = 0; b < 16; b++) horner2(a, m[b]);
            }
            y = sum_reduce(a);
            if (valid && live) F::store(sc.out, (size_t)idx * p.ld_out + r, y);
          }
          mac_add(Ac[q], Lk, y);
        }
      }
#pragma unroll
      for (int q = 0; q < GS1; q++) {
        const uint32_t j = (s * GS1 + (uint32_t)q) * 8u + l;
        if (j < C1) {
          mac_add(Ac[q], ldf<F>(sc.proofs, off1 + j, ld, rr), L10);
          if constexpr (LEADER) {
            if (live) F::store(lout, 2 + A0 + j, mac_reduce(Ac[q]));
          } else {
            const T a = F::add(lv(2 + A0 + j), mac_reduce(Ac[q]));
            G1 = F::add(G1, F::sub(mul128(a, a), mul128(twon, a)));
          }
        }
      }
    }
  }
  // ---- p0(t0), range = sum_e coef0_e sigma0_(e mod P0); p1(t1), norm sum likewise
  auto poly_group = [&](uint32_t coff, uint32_t glen, uint32_t P, const uint4* sig, const T& t,
                        T& pt, T& rs) {
    const uint32_t NQ = (glen + 7) / 8;
    const T t2 = F::mul(t, t), t4 = F::mul(t2, t2), t8 = F::mul(t4, t4);
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
        cf[h] = ldm(sc.proofs, coff + e, q >= 0 && e < glen, ld, rr);
        const uint4 v = sig[e & (P - 1)];
        sg[h] = mk128(v.x, v.y, v.z, v.w);
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
    rs = group_sum(mac_reduce(R));
  };
  T p0t, range, p1t, normg;
  poly_group(A0, p.glen, P0, p.sigma_dev, ldf<F>(sc.qr, 0, ld, rr), p0t, range);
  poly_group(off1 + C1, p.glen1, P1, p.sigma_dev + P0, ldf<F>(sc.qr, 1, ld, rr), p1t, normg);
  G0 = group_sum(G0);
  G1 = group_sum(G1);
  // claimed norm: the last 2 nb - 2 share elements as bits (every lane, broadcast loads)
  T claimed = Z;
  for (uint32_t b = 2 * nb - 2; b-- > 0;)
    claimed = F::add(F::add(claimed, claimed), ldf<F>(sc.meas, nb * E + b, ld, rr));
  const T r1 = ldf<F>(sc.jr, 1, ld, rr);
  const T normd = F::sub(F::add(normg, F::from_words(p.normc128)), claimed);
  const T v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), normd));
  if constexpr (LEADER) {
    if (l == 0 && live) {
      F::store(lout, 0, v);
      F::store(lout, 1 + A0, p0t);
      F::store(lout, 2 + A0 + C1, p1t);
      *(uint4*)(lout + (size_t)p.verifier_len * F::ES) = sc.part[r];
      out.status[r] = status;
    }
    return;
  }
  const T V0 = F::add(lv(0), v);
  const T PT0 = F::add(lv(1 + A0), p0t);
  const T PT1 = F::add(lv(2 + A0 + C1), p1t);
  const int bad = group_or(decode_ok ? 0 : 1);
  if (l == 0 && live) {
    if (status == PRIO3_STATUS_FINISHED) {
      if (bad)
        status = PRIO3_STATUS_PREP_SHARE_DECODE;
      else if (!F::is_zero(V0) || !F::eq(G0, PT0) || !F::eq(G1, PT1))
        status = PRIO3_STATUS_PREP_MSG;
    }
    uint32_t lpart[4], hpart[4];
    load16(lps + (size_t)p.verifier_len * F::ES, lpart);
    const uint4 hp = sc.part[r];
    hpart[0] = hp.x;
    hpart[1] = hp.y;
    hpart[2] = hp.z;
    hpart[3] = hp.w;
    KState ks;
    kzero(ks);
    Msg mm;
    msg_zero(mm);
    msg_dst(mm, p.dst[6]);
    msg_bytes16(mm, 25, lpart);
    msg_bytes16(mm, 41, hpart);
    msg_absorb_final(ks, mm, 57);
    const uint4 cor = sc.corrected[r];
    uint32_t msg[4] = {kword(ks, 0), kword(ks, 1), kword(ks, 2), kword(ks, 3)};
    if (status == PRIO3_STATUS_FINISHED &&
        (msg[0] != cor.x || msg[1] != cor.y || msg[2] != cor.z || msg[3] != cor.w))
      status = PRIO3_STATUS_PREP_NEXT;
    if (status != PRIO3_STATUS_FINISHED) msg[0] = msg[1] = msg[2] = msg[3] = 0;
    ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
    out.status[r] = status;
  }
}

}  // namespace

// the eight-lane query applies: both domains within the four-step split (P <= 1024), the sigma
// tables present, entries of 16 or 32 bits
bool fpvec_query_wide_takes(const DevParams& p) {
  return p.sigma_dev && p.logP <= 10 && p.logP1 <= 10 && (p.bits == 16 || p.bits == 32) &&
         p.glen == 2 * p.P - 1 && p.arity == 2 * p.chunk;
}

// The eight-lane k_query_fpw (three gadget-0 columns per lane and sweep: 268 K/s against 261 K/s
// at two and 240 K/s at four, r02m), helper or leader role; the one-lane k_query_fp (eight chunk
// columns per pass) where the eight-lane kernel does not apply.
void launch_fpvec_query(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st,
                        bool wide, bool leader) {
  if (wide) {
    const uint32_t b = (p.n + 31) / 32;
    if (leader)
      k_query_fpw<3, 1><<<b, 256, 0, st>>>(p, in, sc, out);
    else
      k_query_fpw<3><<<b, 256, 0, st>>>(p, in, sc, out);
    return;
  }
  k_query_fp<8><<<(p.n + 255) / 256, 256, 0, st>>>(p, in, sc, out);
}
