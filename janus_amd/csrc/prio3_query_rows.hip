// prio3_query_rows.hip -- the helper FLP query + decide + prepare message + prepare_next of
// Prio3Histogram with 16 gadget calls (P = 32; Histogram(256, 16) is the headline config C2), on
// two work-items per report that split the gadget calls (rows of the measurement share) between
// them (MI355X, gfx950).
//
// prio 0.16.2 FlpGeneric::query / decide, Prio3::prepare_shares_to_prepare_message and
// prepare_next (the call site is helper_initialized + evaluate,
// /root/reference/aggregator/src/aggregator.rs:2020-2042).
//
// Per report the circuit is two K x C matrix-vector products over the measurement share M
// (K = 16 gadget calls, chunk C):  A_j = sum_k beta_k M[k][j],  B_j = sum_k L_(k+1) M[k][j]
// with beta_k = L_(k+1)(t) rho^k, rho = r^C, then one gadget product per wire pair j.  One lane
// cannot keep both 16-element coefficient vectors and the accumulators in VGPRs, so k_query_h
// re-reads beta / L from scratch on each of its 8 column sweeps: 12.6 KB of HBM traffic per
// report against 6.3 KB of share, proof and prep-share bytes.  Here:
//   * The decimation-in-frequency split of the 32-point Lagrange DFT hands lane h of the pair the
//     basis values L_c with c = h (mod 2) -- exactly the L_(k+1) of the rows k = 1 - h (mod 2).
//     So each lane computes one 16-point half (no exchange), owns 8 rows, and keeps its 8 L and
//     8 beta in VGPRs for the whole sweep: the coefficients never touch memory.
//   * Column pairs (2i, 2i+1): each lane first accumulates the partner's column over its own rows,
//     the pair swaps these unreduced lazy accumulators (DPP quad_perm [1,0,3,2]), and each lane
//     continues its own column 2i + h from the partner's partial over its rows, then finalises
//     it.  Every share element is loaded once; two accumulator pairs are never live together.
//   * p(t) = E(t^2) + t O(t^2) and the sigma-weighted range sum split the gadget-polynomial
//     coefficients by parity; S, G, p(t) and the range are joined with one exchange each; both
//     lanes run decide and the prepare-message XOF, the even lane writes the verdict.
//   * The column-pair sweep is software-pipelined by half: the own column of pair i+1 is loaded
//     while the partner column of pair i is multiplied, and vice versa.
// 2 waves per SIMD (a lane holds 64 VGPRs of coefficients, 42 of accumulators, 64 of loads).
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"

namespace {

typedef Fp128 F;
typedef f128 T;

// value of the partner lane (lane ^ 1): DPP quad_perm [1,0,3,2]
DEV uint32_t xor1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
DEV uint64_t xor1(uint64_t v) {
  return (uint64_t)xor1((uint32_t)v) | ((uint64_t)xor1((uint32_t)(v >> 32)) << 32);
}
DEV T xor1(const T& a) { return mk128(xor1(a.w[0]), xor1(a.w[1]), xor1(a.w[2]), xor1(a.w[3])); }
// a + (partner's a): the same value on both lanes of the pair
DEV T pair_sum(const T& a) { return F::add(a, xor1(a)); }

// the partner lane's lazy accumulator (21 DPP moves)
DEV mac128 xor1(const mac128& a) {
  mac128 b;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    b.c[k] = xor1(a.c[k]);
    b.h[k] = xor1(a.h[k]);
  }
  return b;
}

constexpr int K = 16;    // gadget calls (rows)
constexpr int KH = 8;    // rows per lane
constexpr int PP = 32;   // gadget-polynomial domain
constexpr int GLEN = 2 * (PP - 1) + 1;

template <int C>
__global__ __launch_bounds__(256, 2) void k_query_rows(DevParams p, InPtrs in, Scratch sc,
                                                       OutPtrs out) {
  static_assert(C % 2 == 0 && C >= 2, "column pairs");
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (r >= p.n) return;  // both lanes of a pair leave together (DPP stays inside live pairs)
  const size_t ld = p.ld;
  const uint32_t A = p.arity, M = p.meas_len;
  DCHECK(p.calls == (uint32_t)K && p.chunk == (uint32_t)C && p.P == (uint32_t)PP && r < ld);
  uint8_t status = PRIO3_STATUS_FINISHED;
  const T t = ldf<F>(sc.qr, 0, ld, r);

  // ---- Lagrange basis: lane h evaluates X[2kk + h] = DFT16 of the h-th DIF half of
  // u_e = t^e / P; L_c = X[(32 - c) mod 32].  Row k = 2q + 1 - h uses L_(k+1) = x[15 - q].
  T Lr[KH], be[KH], L0, sumL;
  {
    T t16 = t;
#pragma unroll
    for (int i = 0; i < 4; i++) t16 = F::mul(t16, t16);
    if (F::eq(F::mul(t16, t16), F::one())) status = PRIO3_STATUS_PREP_INIT;  // t^P == 1
    const T ip = FC<F>::invP(p);
    T pw = F::mul(ip, h ? F::sub(F::one(), t16) : F::add(F::one(), t16));
    const T ratio = h ? F::mul(t, F::from_words(p.tw128[1])) : t;
    T x[16];
#pragma unroll
    for (int e = 0; e < 16; e++) {
      x[__builtin_bitreverse32(e) >> 28] = pw;
      if (e < 15) pw = F::mul(pw, ratio);
    }
    dft_reg<16, 4>(p, x, 2);
    const T L0x = xor1(x[0]);  // L_0 = X[0] lives on the even lane
    L0 = h ? L0x : x[0];
    T s = x[15];
#pragma unroll
    for (int q = 0; q < KH; q++) {
      Lr[q] = x[15 - q];
      if (q) s = F::add(s, Lr[q]);
    }
    sumL = pair_sum(s);
  }

  // ---- beta_k = L_(k+1) rho^k for this lane's rows k = 2q + 1 - h
  const T r0 = ldf<F>(sc.jr, 0, ld, r);
  {
    T rho = F::one(), sq = r0;  // rho = r0^C by square-and-multiply (C compile-time)
#pragma unroll
    for (int e = C; e; e >>= 1) {
      if (e & 1) rho = F::mul(rho, sq);
      if (e > 1) sq = F::mul(sq, sq);
    }
    const T rho2 = F::mul(rho, rho);
    T rp = h ? F::one() : rho;
#pragma unroll
    for (int q = 0; q < KH; q++) {
      be[q] = F::mul(Lr[q], rp);
      if (q + 1 < KH) rp = F::mul(rp, rho2);
    }
  }

  const T half = FC<F>::half(p);
  const T halfL = F::mul(half, sumL);
  const uint8_t* lps = in.leader + (size_t)r * p.prep_share_len;
  bool decode_ok = true;
  auto lv = [&](uint32_t e) {
    const T x = F::load(lps, e);
    if (!F::lt_p(x)) decode_ok = false;
    return x;
  };

  // ---- column-pair sweep.  Element i = k C + j; lane h, row q (k = 2q + 1 - h):
  // own column 2i + h at k C + 2i + h, the partner's column 2i + 1 - h.
  const size_t rowb = ld * 16;  // bytes per scratch row
  const uint8_t* mbase = (const uint8_t*)sc.meas + (size_t)r * 16;
  const uint32_t off_own = (1u - h) * C + h, off_snd = (1u - h) * (C + 1);
  auto ld_col = [&](uint32_t i0, T (&dst)[KH]) {  // rows of this lane, column offset i0
#pragma unroll
    for (int q = 0; q < KH; q++) {
      const uint32_t i = i0 + 2u * C * q;
      const bool ok = i < M;
      const uint4 v = *(const uint4*)(mbase + (size_t)(ok ? i : 0) * rowb);
      const uint32_t mk = ok ? 0xffffffffu : 0u;
      dst[q] = mk128(v.x & mk, v.y & mk, v.z & mk, v.w & mk);
    }
  };
  T mo[KH], ms[KH];
  ld_col(off_own, mo);
  ld_col(off_snd, ms);
  sum128 Ssum;
  sum_zero(Ssum);
  T G = F::zero();
  const T r02 = F::mul(r0, r0);
  T rj = h ? r02 : r0;  // r0^(j+1) for this lane's column j = 2i + h
#pragma unroll 1
  for (uint32_t i = 0; i < C / 2; i++) {
    // the partner's column over this lane's rows first; the pair then swaps these partials, so
    // each lane's own-column accumulators start from the partner's rows (two live at a time)
    mac128 Ao, Bo;
    {
      mac128 As, Bs;
      mac_zero(As);
      mac_zero(Bs);
#pragma unroll
      for (int q = 0; q < KH; q++) {
        mac_add(As, be[q], ms[q]);
        mac_add(Bs, Lr[q], ms[q]);
        sum_add(Ssum, ms[q]);
      }
      if (i + 1 < C / 2) ld_col(off_snd + 2 * (i + 1), ms);  // wave-uniform
      Ao = xor1(As);
      Bo = xor1(Bs);
    }
#pragma unroll
    for (int q = 0; q < KH; q++) {
      mac_add(Ao, be[q], mo[q]);
      mac_add(Bo, Lr[q], mo[q]);
      sum_add(Ssum, mo[q]);
    }
    // wire values of column j at t: f1 = seed_(2j+1) L0 + B_j - L/2, f0 = seed_2j L0 + r^(j+1) A_j
    const uint32_t j = 2 * i + h;
    mac_add(Bo, ldf<F>(sc.proofs, 2 * j + 1, ld, r), L0);
    const T f1 = F::sub(mac_reduce_f(Bo), halfL);
    const T Aq = mac_reduce_f(Ao);
    mac128 F0;
    mac_zero(F0);
    mac_add(F0, ldf<F>(sc.proofs, 2 * j, ld, r), L0);
    mac_add(F0, rj, Aq);
    const T f0 = mac_reduce_f(F0);
    G = F::add(G, F::mul(F::add(lv(1 + 2 * j), f0), F::add(lv(2 + 2 * j), f1)));
    rj = F::mul(rj, r02);
    // the own column of pair i+1 flies during the partner-column MACs of pair i+1
    if (i + 1 < C / 2) ld_col(off_own + 2 * (i + 1), mo);
  }
  G = pair_sum(G);
  // ---- (after the sweep, so none of it is live there) p(t) and range = sum_e coef_e sigma_(e mod P), coefficients split by parity:
  // lane h takes e = 2m + h, p(t) = E(t^2) + t O(t^2)
  T pt, range;
  {
    const T t2 = F::mul(t, t);
    mac128 R;
    mac_zero(R);
    T q = F::zero();
    auto ldc = [&](int m) {  // coefficient 2m + h, zero past the end
      const int e = 2 * m + (int)h;
      const bool ok = e < GLEN;
      const uint4 v = ((const uint4*)sc.proofs)[(size_t)(A + (ok ? e : 0)) * ld + r];
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

  const T S = pair_sum(sum_reduce(Ssum));
  const T r1 = ldf<F>(sc.jr, 1, ld, r);
  const T v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), F::sub(S, half)));
  const T V0 = F::add(lv(0), v);
  const T PT = F::add(lv(A + 1), pt);
  decode_ok = decode_ok && xor1((uint32_t)decode_ok);
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
  if (h == 0) {
    ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
    out.status[r] = status;
  }
}

}  // namespace

// Prio3Histogram helper query with K = 16 calls and chunk 16 on row-split lane pairs; returns
// false if the instance is not one this kernel takes (the caller then launches k_query_h)
bool query_rows_takes(const DevParams& p) {
  return p.kind == PRIO3_HISTOGRAM && p.es == 16 && p.jr_len >= 2 && p.P == PP &&
         p.calls == (uint32_t)K && p.chunk == 16 && p.meas_len <= K * 16u;
}

bool launch_query_rows(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st) {
  if (!query_rows_takes(p)) return false;
  if (p.n == 0) return true;
  const uint32_t blocks = (uint32_t)(((uint64_t)p.n * 2 + 255) / 256);
  k_query_rows<16><<<blocks, 256, 0, st>>>(p, in, sc, out);
  return true;
}
