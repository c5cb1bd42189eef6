// prio3_query_pair.hip -- the helper FLP query + decide + prepare message + prepare_next of the
// ParallelSum(Mul) circuits (Prio3Histogram, Prio3SumVec) with a gadget-polynomial domain of
// PP = 16 or 32 points, two work-items per report (MI355X, gfx950).
//
// prio 0.16.2 FlpGeneric::query / decide, Prio3::prepare_shares_to_prepare_message and
// prepare_next (the call site is helper_initialized + evaluate,
// /root/reference/aggregator/src/aggregator.rs:2020-2042).
//
// Per report the circuit is two K x C matrix-vector products over the measurement share M
// (K gadget calls, chunk C):  A_j = sum_k beta_k M[k][j],  B_j = sum_k L_(k+1) M[k][j]
// (beta_k = L_(k+1)(t) r^(C k)), followed by one gadget product per wire pair j.  The
// one-lane-per-report kernel (k_query_h) cannot hold both coefficient vectors and the
// accumulators in VGPRs, so it re-reads beta/L from scratch on each of its C/GS column sweeps --
// about half of its HBM traffic (12.6 KB/report against a 6.3 KB algorithmic floor).
//
// Here the two lanes of a pair share one report:
//   * prologue split by lane: each lane evaluates one half of the decimation-in-frequency split
//     of the PP-point Lagrange DFT (the even- or odd-indexed basis values), one parity class of
//     the gadget-polynomial coefficients for Horner (p(t) = E(t^2) + t O(t^2)) and the
//     sigma-weighted range sum, and beta_k for the rows whose L_(k+1) it owns;
//   * beta_k and L_(k+1) go to LDS once ([row][report] in the block, 2 K x 16 B per report) --
//     the coefficient re-reads of every sweep become LDS reads, never HBM;
//   * the column sweeps are split between the lanes (lane h owns the column groups
//     jg = 2 GS s + h GS), so every measurement element is loaded from HBM exactly once and every
//     wire pair is finalised by exactly one lane;
//   * partial sums (p(t), range, sum of the share, gadget sum) are joined with one DPP
//     quad_perm [1,0,3,2] exchange each; both lanes then run decide and the 1-permutation
//     prepare-message XOF, and the even lane writes the verdict.
// Block: 128 work-items = 64 reports, 2 K x 1 KiB of LDS (32 KiB at K = 16: 5 blocks per CU).
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"

namespace {

typedef Fp128 F;
typedef f128 T;

constexpr uint32_t RPB = 64;  // reports per block (two lanes each)

// value of the partner lane (lane ^ 1): DPP quad_perm [1,0,3,2]
DEV uint32_t xor1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
DEV T xor1(const T& a) { return mk128(xor1(a.w[0]), xor1(a.w[1]), xor1(a.w[2]), xor1(a.w[3])); }
// a + (partner's a): the same value on both lanes of the pair
DEV T pair_sum(const T& a) { return F::add(a, xor1(a)); }

template <int PP, int GS>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_query_pair(DevParams p, InPtrs in, Scratch sc,
                                                       OutPtrs out) {
  constexpr int HALF = PP / 2;
  constexpr int LOGH = HALF == 16 ? 4 : 3;
  static_assert(PP == 16 || PP == 32, "PP must be 16 or 32");
  extern __shared__ uint4 lds[];  // beta rows [0, K), then L rows [K, 2K); [row][RPB]
  const uint32_t tid = threadIdx.x, h = tid & 1u, rl = tid >> 1;
  const uint32_t r = blockIdx.x * RPB + rl;
  const bool live = r < p.n;
  const uint32_t rr = live ? r : p.n - 1;  // a dead pair computes on a valid column, stores nothing
  const size_t ld = p.ld;
  const uint32_t A = p.arity, C = p.chunk, M = p.meas_len, K = p.calls;
  DCHECK(K <= (uint32_t)PP - 1 && p.P == (uint32_t)PP && rr < ld);
  auto lds_beta = [&](uint32_t k) -> uint4& { return lds[(size_t)k * RPB + rl]; };
  auto lds_L = [&](uint32_t k) -> uint4& { return lds[(size_t)(K + k) * RPB + rl]; };
  auto put = [](uint4& d, const T& v) { d = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]); };
  auto get = [](const uint4& v) { return mk128(v.x, v.y, v.z, v.w); };

  uint8_t status = PRIO3_STATUS_FINISHED;
  const T t = ldf<F>(sc.qr, 0, ld, rr);
  const T r0 = ldf<F>(sc.jr, 0, ld, rr);
  // rho = r0^C by square-and-multiply over the (uniform) bits of C
  T rho = F::one();
  {
    T sq = r0;
    for (uint32_t e = C; e; e >>= 1) {
      if (e & 1) rho = F::mul(rho, sq);
      if (e > 1) sq = F::mul(sq, sq);
    }
  }
  // ---- Lagrange basis, this lane's half of the DIF split ----
  // u_e = t^e / P; X[2k] = DFT_HALF((u_e + u_(e+HALF))), X[2k+1] = DFT_HALF((u_e - u_(e+HALF)) w^e),
  // each a geometric sequence; L_c = X[(P - c) mod P].
  T L0 = F::zero(), sumL = F::zero();
  {
    T tH = t;
#pragma unroll
    for (int i = 0; i < LOGH; i++) tH = F::mul(tH, tH);
    if (F::eq(F::mul(tH, tH), F::one())) status = PRIO3_STATUS_PREP_INIT;  // t^P == 1
    const T ip = FC<F>::invP(p);
    T pw = F::mul(ip, h ? F::sub(F::one(), tH) : F::add(F::one(), tH));
    const T ratio = h ? F::mul(t, F::from_words(p.tw128[1])) : t;
    T x[HALF];
#pragma unroll
    for (int e = 0; e < HALF; e++) {
      x[__builtin_bitreverse32(e) >> (32 - LOGH)] = pw;
      pw = F::mul(pw, ratio);
    }
    dft_reg<HALF, LOGH>(p, x, 2);
    // rows in ascending c = k + 1: idx = 2 kk + h, c = (P - idx) mod P rises by 2 as kk falls;
    // the lowest c of this lane is 2 - h, so beta's power starts at rho^(1 - h), step rho^2
    const T rho2 = F::mul(rho, rho);
    T rp = h ? F::one() : rho;
#pragma unroll
    for (int kk = HALF - 1; kk >= 0; kk--) {
      const uint32_t c = (uint32_t)(PP - 2 * kk - (int)h) & (PP - 1);
      if (c == 0) {
        L0 = x[kk];
      } else {
        if (c <= K) {
          put(lds_L(c - 1), x[kk]);
          put(lds_beta(c - 1), F::mul(x[kk], rp));
          sumL = F::add(sumL, x[kk]);
        }
        rp = F::mul(rp, rho2);
      }
    }
  }
  {  // L_0 lives on the even lane (DPP outside any lane-divergent branch)
    const T L0x = xor1(L0);
    L0 = h ? L0x : L0;
  }
  sumL = pair_sum(sumL);
  // ---- p(t) and the range sum = sum_e coef_e sigma_(e mod P), coefficients split by parity ----
  T pt, range;
  {
    constexpr int GLEN = 2 * (PP - 1) + 1;
    const T t2 = F::mul(t, t);
    mac128 R;
    mac_zero(R);
    T q = F::zero();
    auto ldc = [&](int m) {  // coefficient 2m + h, zero past the end
      const int e = 2 * m + (int)h;
      const bool ok = e < GLEN;
      const uint4 v = ((const uint4*)sc.proofs)[(size_t)(A + (ok ? e : 0)) * ld + rr];
      const uint32_t mk = ok ? 0xffffffffu : 0u;
      return mk128(v.x & mk, v.y & mk, v.z & mk, v.w & mk);
    };
    constexpr int HD = 4;
    T cb[HD];
#pragma unroll
    for (int i = 0; i < HD; i++) cb[i] = ldc(PP - 1 - i);
#pragma unroll
    for (int m0 = PP - 1; m0 >= 0; m0 -= HD) {
      T cn[HD];
#pragma unroll
      for (int i = 0; i < HD; i++) cn[i] = m0 - HD - i >= 0 ? ldc(m0 - HD - i) : F::zero();
#pragma unroll
      for (int i = 0; i < HD; i++) {
        const int m = m0 - i;
        if (m >= 0) {
          q = F::add(F::mul(q, t2), cb[i]);
          const T s_even = F::from_words(p.sigma128[(2 * m) & (PP - 1)]);
          const T s_odd = F::from_words(p.sigma128[(2 * m + 1) & (PP - 1)]);
          mac_add(R, cb[i], h ? s_odd : s_even);
        }
        cb[i] = cn[i];
      }
    }
    const T qt = F::mul(q, t);
    pt = pair_sum(h ? qt : q);
    range = pair_sum(mac_reduce_f(R));
  }
  __syncthreads();  // beta / L rows of every report of the block are in LDS

  const T half = FC<F>::half(p);
  const T halfL = F::mul(half, sumL);
  const uint8_t* lps = in.leader + (size_t)rr * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    const T x = F::load(lps, e);
    if (!F::lt_p(x)) decode_ok = false;
    return x;
  };
  sum128 Ssum;
  sum_zero(Ssum);
  T G = F::zero();
  const T Z = F::zero();
  // r0^(j+1) for this lane's first column (jg = h GS), then r0 per column and r0^GS per skip
  T r0GS = F::one();
#pragma unroll
  for (int i = 0; i < GS; i++) r0GS = F::mul(r0GS, r0);
  T rj = h ? F::mul(r0GS, r0) : r0;
  const size_t rowb = ld * 16;  // bytes per scratch row
  const uint8_t* mbase = (const uint8_t*)sc.meas + (size_t)rr * 16;
  auto ld4 = [](const uint8_t* a) {
    const uint4 v = *(const uint4*)a;
    return mk128(v.x, v.y, v.z, v.w);
  };
  for (uint32_t jg2 = 0; jg2 < C; jg2 += 2 * GS) {
    const uint32_t jg = jg2 + h * GS;
    mac128 Aa[GS], Bb[GS];
    bool cv[GS];
    const uint8_t* colp[GS];  // this lane's column q of row 0
#pragma unroll
    for (int q = 0; q < GS; q++) {
      mac_zero(Aa[q]);
      mac_zero(Bb[q]);
      cv[q] = jg + q < C;
      // an invalid column (past C) reads a valid element (clamped below M) into accumulators
      // that are never used
      colp[q] = mbase + (size_t)min(jg + q, M - 1) * rowb;
    }
    // the last call's row first (its padding past M masked), so its latency hides behind the
    // sweep; rows 0 .. K-2 are then streamed one call ahead without any per-row masking
    T ml[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) {
      const uint32_t i = (K - 1) * C + jg + q;
      const bool ok = cv[q] && i < M;
      const T x = ld4(mbase + (size_t)(ok ? i : 0) * rowb);
      ml[q] = F::sel(ok, x, Z);
    }
    const size_t callb = (size_t)C * rowb;  // bytes per call (C rows)
    // rows k <= K-2 of an invalid column may run past M for small C: clamp the call offset
    const size_t lastb = (size_t)(K >= 2 ? K - 2 : 0) * callb;
    T mc[GS];
    if (K >= 2) {
#pragma unroll
      for (int q = 0; q < GS; q++) mc[q] = cv[q] ? ld4(colp[q]) : Z;
    }
    uint4 beN = lds_beta(0), LN = lds_L(0);
#pragma unroll 1
    for (uint32_t k = 0; k + 1 < K; k++) {
      const size_t nb = min((size_t)(k + 1) * callb, lastb);
      T mn[GS];
#pragma unroll
      for (int q = 0; q < GS; q++) mn[q] = ld4(colp[q] + nb);
      const T be = get(beN), Lk = get(LN);
      beN = lds_beta(k + 1);
      LN = lds_L(k + 1);
#pragma unroll
      for (int q = 0; q < GS; q++) {
        mac_add(Aa[q], be, mc[q]);
        mac_add(Bb[q], Lk, mc[q]);
        sum_add(Ssum, F::sel(cv[q], mc[q], Z));
      }
#pragma unroll
      for (int q = 0; q < GS; q++) mc[q] = mn[q];
    }
    {  // call K-1
      const T be = get(beN), Lk = get(LN);
#pragma unroll
      for (int q = 0; q < GS; q++) {
        mac_add(Aa[q], be, ml[q]);
        mac_add(Bb[q], Lk, ml[q]);
        sum_add(Ssum, ml[q]);
      }
    }
    // wire values at t: f1 = seed_(2j+1) L0 + B_j - L/2, f0 = seed_2j L0 + r^(j+1) A_j; the
    // gadget products of the group are summed in one MAC before a single reduction
    mac128 Gq;
    mac_zero(Gq);
#pragma unroll
    for (int q = 0; q < GS; q++) {
      const uint32_t j = jg + q;
      const bool vj = j < C;  // lane-varying when C is not a multiple of 2 GS
      const uint32_t jj = vj ? j : 0;
      mac_add(Bb[q], ldf<F>(sc.proofs, 2 * jj + 1, ld, rr), L0);
      const T f1 = F::sub(mac_reduce_f(Bb[q]), halfL);
      const T Aq = mac_reduce_f(Aa[q]);
      mac128 F0;
      mac_zero(F0);
      mac_add(F0, ldf<F>(sc.proofs, 2 * jj, ld, rr), L0);
      mac_add(F0, rj, Aq);
      const T f0 = mac_reduce_f(F0);
      const T a0 = F::add(lv(1 + 2 * jj), f0), a1 = F::add(lv(2 + 2 * jj), f1);
      mac_add(Gq, F::sel(vj, a0, Z), a1);
      rj = F::mul(rj, r0);
    }
    G = F::add(G, mac_reduce_f(Gq));
    rj = F::mul(rj, r0GS);  // skip the partner lane's column group
  }
  G = pair_sum(G);
  const T S = pair_sum(sum_reduce(Ssum));
  T v;
  if (p.kind == PRIO3_SUMVEC) {
    v = range;
  } else {
    const T r1 = ldf<F>(sc.jr, 1, ld, rr);
    v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), F::sub(S, half)));
  }
  decode_ok = decode_ok && xor1((uint32_t)decode_ok);
  const T V0 = F::add(lv(0), v);
  const T PT = F::add(lv(A + 1), pt);
  if (status == PRIO3_STATUS_FINISHED) {
    if (!decode_ok)
      status = PRIO3_STATUS_PREP_SHARE_DECODE;
    else if (!F::is_zero(V0) || !F::eq(G, PT))
      status = PRIO3_STATUS_PREP_MSG;
  }
  // prepare message = the joint-rand seed of (leader part, helper part); prepare_next checks it
  // against the helper's corrected seed
  uint32_t lpart[4], hpart[4];
  load16(lps + (size_t)p.verifier_len * F::ES, lpart);
  {
    const uint4 hp = sc.part[rr];
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
  const uint4 cor = sc.corrected[rr];
  uint32_t msg[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
  if (status == PRIO3_STATUS_FINISHED &&
      (msg[0] != cor.x || msg[1] != cor.y || msg[2] != cor.z || msg[3] != cor.w))
    status = PRIO3_STATUS_PREP_NEXT;
  if (status != PRIO3_STATUS_FINISHED) msg[0] = msg[1] = msg[2] = msg[3] = 0;
  if (live && h == 0) {
    ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
    out.status[r] = status;
  }
  // SumVec truncate: output entry e = sum_b 2^b m[e bits + b], entries split over the pair
  if (p.kind == PRIO3_SUMVEC && live) {
    for (uint32_t e = h; e < p.out_len; e += 2) {
      T acc = F::zero(), pw = F::one();
      for (uint32_t b = 0; b < p.bits; b++) {
        acc = F::add(acc, F::mul(pw, ldf<F>(sc.meas, e * p.bits + b, ld, r)));
        pw = F::add(pw, pw);
      }
      F::store(sc.out, (size_t)e * p.ld_out + r, acc);
    }
  }
}

}  // namespace

// P = 16 / 32 ParallelSum(Mul) helper query on lane pairs; returns false if the instance is not
// one this kernel takes (the caller then launches k_query_h)
bool launch_query_pair(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st) {
  if ((p.kind != PRIO3_HISTOGRAM && p.kind != PRIO3_SUMVEC) || p.es != 16 || p.jr_len == 0)
    return false;
  if ((p.P != 32 && p.P != 16) || p.calls > p.P - 1) return false;
  const uint32_t blocks = (p.n + RPB - 1) / RPB;
  const size_t lds_bytes = (size_t)2 * p.calls * RPB * 16;
  if (p.P == 32)
    k_query_pair<32, 2><<<blocks, 2 * RPB, lds_bytes, st>>>(p, in, sc, out);
  else
    k_query_pair<16, 2><<<blocks, 2 * RPB, lds_bytes, st>>>(p, in, sc, out);
  return true;
}
