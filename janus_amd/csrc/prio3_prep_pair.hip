// prio3_prep_pair.hip -- k_prep_hp: the whole helper prepare (+ the fused accumulate) of
// Prio3Histogram with P = 32 on TWO work-items per report, for executor groups too small to fill
// the chip with one lane per report (MI355X, gfx950).
//
// prio 0.16.2 Prio3::prepare_init (agg_id 1), prepare_shares_to_prepare_message and prepare_next
// (VDAF-08 A.5.1-A.6, A.9) -- Janus's helper_initialized(..).evaluate(..)
// per report, aggregator.rs:2020-2042 -- with the output shares summed into the job's
// aggregation as AggregationJobWriter does (aggregation_job_writer.rs:591-695).
//
// Why: Janus hands the engine 100-500-report jobs (aggregation_job_creator.rs:63-64); the
// executor coalesces concurrent jobs, but 128 callers keep only ~64k reports in flight, so a
// group is ~31k reports: 485 waves of the one-lane k_prep_h on 1,024 SIMDs, each SIMD with one
// wave at most that issues at about half the SIMD's rate.  Here each report
// has a lane pair, so the group has twice the waves and each wave half the work:
//   XOF    even lane: query-randomness header -> squeeze the measurement share (stored, and summed
//          into the wave partials while in registers), then the proofs share;
//          odd lane: query randomness -> absorb the same share bytes into the joint-rand-part
//          sponge (words from the partner by DPP, as k_xof_pair) -> corrected seed, joint rand
//   query  the 4 Lagrange phases, the 63 proof coefficients (Horner + the range dot), the 16
//          beta_k and the 16 wires are split between the two lanes (same instruction stream,
//          lane-dependent data); the partial G, S, sum_L, p(t) and range meet by one DPP swap
// A wave holds 32 reports: wave partials and wave segments are indexed by r >> 5
// (DevParams-independent; fused_finish passes wshift = 5 to k_agg_fix for these runs).
// Flagged reports (rejection sampling) are deferred to the run's k_slow_redo, as k_prep_h's.
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"
#include "prio3_pair.h"

namespace {

typedef Fp128 F;
typedef f128 T;

// the partner's value (lane ^ 1): DPP quad_perm [1,0,3,2]
DEV uint32_t pair_x(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
DEV T pair_x(const T& a) { return mk128(pair_x(a.w[0]), pair_x(a.w[1]), pair_x(a.w[2]), pair_x(a.w[3])); }
DEV T sel(bool c, const T& a, const T& b) { return F::sel(c, a, b); }

// ---- the query of one report on its lane pair (h = 0 even, 1 odd); both lanes active --------
// The one-lane form is query_h_body<2, 32> (prio3_engine.hip); this splits its work in halves.
// PAIR_GS: wires per sweep of the wire loop (each sweep re-reads the 16 beta_k and L_k); 2 keeps
// four lazy 128-bit MAC accumulators (21 VGPRs each) live.  PAIR_DIRECT_BETA: the beta_k are
// formed and stored as the Lagrange phases produce their L values (r^C taken first), instead of
// keeping this lane's eight L values in registers through the Horner / range pass.
#ifndef PAIR_GS
#define PAIR_GS 2
#endif
#ifndef PAIR_DIRECT_BETA
#define PAIR_DIRECT_BETA 0
#endif
DEV void query_pair(const DevParams& p, const InPtrs& in, const Scratch& sc, const OutPtrs& out,
                    const uint32_t r, const uint32_t h) {
  constexpr int PP = 32, GLEN = 2 * (PP - 1) + 1, GS = PAIR_GS;
  const size_t ld = p.ld;
  const uint32_t A = p.arity, C = p.chunk, M = p.meas_len, K = p.calls;
  uint8_t status = PRIO3_STATUS_FINISHED;
  const T t = ldf<F>(sc.qr, 0, ld, r);
  // 1. Lagrange basis: X[4k + ph] = DFT8(y^ph)[k], y^ph_n = (G_ph / P)(t w32^ph)^n; lane h
  //    takes phases 2h, 2h + 1.  X[idx] = L_c, c = (32 - idx) mod 32.
  T t8 = t;
#pragma unroll
  for (int i = 0; i < 3; i++) t8 = F::mul(t8, t8);
  const T t16 = F::mul(t8, t8);
  const T t32 = F::mul(t16, t16);
  if (F::eq(t32, F::one())) status = PRIO3_STATUS_PREP_INIT;
  const T ip = FC<F>::invP(p);
  const T a = F::add(F::one(), t16), b = F::sub(F::one(), t16);
  const T c = F::mul(t8, a), wd = F::mul(F::mul(t8, b), F::from_words(p.tw128[8]));  // w4 = w32^8
  T L0 = F::zero(), sumL = F::zero();
  const T r0 = ldf<F>(sc.jr, 0, ld, r);
#if PAIR_DIRECT_BETA
  // r^C, r^(2C), r^(4C): beta_k = L_(k+1) r^(C k) leaves each phase straight to scratch
  T rC = F::one();
  {
    T sq = r0;
    for (uint32_t e = C; e; e >>= 1) {
      if (e & 1) rC = F::mul(rC, sq);
      if (e > 1) sq = F::mul(sq, sq);
    }
  }
  const T rC2 = F::mul(rC, rC), rC4 = F::mul(rC2, rC2);
#else
  // the betas this lane can form from its own L values: k with (31 - k) & 3 in {2h, 2h + 1}
  T Lmine[8];
#endif
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const T g = i == 0 ? sel(h, F::sub(a, c), F::add(a, c)) : sel(h, F::sub(b, wd), F::add(b, wd));
    const T tw = sel(h, F::from_words(p.tw128[2 + i]), F::from_words(p.tw128[i]));
    const T ratio = F::mul(t, tw);
    T x[8];
    T pw = F::mul(ip, g);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      x[__builtin_bitreverse32(e) >> 29] = pw;
      if (e + 1 < 8) pw = F::mul(pw, ratio);
    }
    dft_reg<8, 3>(p, x, 4);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      // idx = 4k + 2h + i; c = (32 - idx) & 31 (lane-dependent)
      const uint32_t idx = 4u * k + 2u * h + (uint32_t)i, cc = (32u - idx) & 31u;
      if (cc == 0) {
        L0 = x[k];
      } else if (cc <= K) {
        F::store(sc.Lbuf, (size_t)cc * ld + r, x[k]);
        sumL = F::add(sumL, x[k]);
      }
#if !PAIR_DIRECT_BETA
      // c = k' + 1 for beta_k' (k' = 31 - idx): this lane owns the betas of its L values
      if (k >= 4) Lmine[2 * (k - 4) + i] = x[k];  // idx >= 16: c <= 16
#endif
    }
#if PAIR_DIRECT_BETA
    // beta_k' for idx = 4 kx + 2h + i >= 16 (kx = 7 .. 4): k' = 31 - idx = 3 - 2h - i + 4 (7 - kx),
    // r^(C k') from r^(C (3 - 2h - i)) by r^(4C) steps
    T rk = i == 0 ? sel(h, rC, F::mul(rC2, rC)) : sel(h, F::one(), rC2);
#pragma unroll
    for (int kx = 7; kx >= 4; kx--) {
      const uint32_t k = 31u - (4u * kx + 2u * h + (uint32_t)i);
      if (k < K) F::store(sc.beta, (size_t)k * ld + r, F::mul(x[kx], rk));
      if (kx > 4) rk = F::mul(rk, rC4);
    }
#endif
  }
  L0 = sel(h, pair_x(L0), L0);  // c = 0 is idx 0: the even lane's phase 0
  sumL = F::add(sumL, pair_x(sumL));
  // 2. p(t) by Horner and the range sum = sum_e coef_e sigma_(e mod P) over the GLEN = 63
  //    coefficients: even lane e = 63 .. 32 (c_63 = 0 past the end), odd lane e = 31 .. 0, so
  //    p(t) = hi t^32 + lo
  T pt = F::zero(), range;
  {
    mac128 R;
    mac_zero(R);
    const int base = h ? 31 : 63;
    constexpr int HD = 4;
    auto ldc = [&](int q) {  // coefficient e = base - q, zero below this lane's range
      const int e = base - q;
      const bool ok = q < 32 && e < GLEN && (h ? e >= 0 : e >= 32);
      const T v = ldf<F>(sc.proofs, A + (ok ? (uint32_t)e : 0u), ld, r);
      return ok ? v : F::zero();
    };
    T cb[HD];
#pragma unroll
    for (int q = 0; q < HD; q++) cb[q] = ldc(q);
#pragma unroll 1
    for (int q0 = 0; q0 < 32; q0 += HD) {
      T cn[HD];
#pragma unroll
      for (int q = 0; q < HD; q++) cn[q] = ldc(q0 + HD + q);
#pragma unroll
      for (int q = 0; q < HD; q++) {
        const int e = base - (q0 + q);
        pt = F::add(F::mul(pt, t), cb[q]);
        // sigma index e mod 32 (a zero coefficient contributes nothing)
        mac_add(R, cb[q], F::from_words(p.sigma128[(e & 31)]));
        cb[q] = cn[q];
      }
    }
    range = mac_reduce_f(R);
    range = F::add(range, pair_x(range));
    const T other = pair_x(pt);
    const T hi = sel(h, other, pt), lo = sel(h, pt, other);
    pt = F::add(F::mul(hi, t32), lo);
  }
#if !PAIR_DIRECT_BETA
  // 3. beta_k = L_(k+1) r^(C k): this lane's eight k (k & 3 = 3 - (2h + i)), from its registers
  T rC = F::one();
  {
    T sq = r0;
    for (uint32_t e = C; e; e >>= 1) {
      if (e & 1) rC = F::mul(rC, sq);
      if (e > 1) sq = F::mul(sq, sq);
    }
    const T rC2 = F::mul(rC, rC), rC4 = F::mul(rC2, rC2);
    // k = 4 m + 3 - 2h - i for idx = 4 k_x + 2h + i (k_x = 4 + m' ...): enumerate this lane's
    // (k_x >= 4, i) pairs: idx = 4 kx + 2h + i, k = 31 - idx
    T rk0 = sel(h, F::one(), rC2);  // r^(C k) at k = 2 - 2h (k of kx = 7, i = 1)
#pragma unroll
    for (int kx = 7; kx >= 4; kx--) {
#pragma unroll
      for (int i = 1; i >= 0; i--) {
        // k = 31 - (4 kx + 2h + i): kx = 7 gives k = 3 - 2h - i, each kx step down adds 4
        const uint32_t k = 31u - (4u * kx + 2u * h + (uint32_t)i);
        const T rk = i == 1 ? rk0 : F::mul(rk0, rC);
        if (k < K) F::store(sc.beta, (size_t)k * ld + r, F::mul(Lmine[2 * (kx - 4) + i], rk));
      }
      rk0 = F::mul(rk0, rC4);
    }
  }
#endif
  // the wire loop reads every beta_k and L_(k+1): the partner's stores must have landed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // 4. the wires: lane h owns j in [8h, 8h + 8): four sweeps of two wires
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
  T G = F::zero();
  T rj = r0;  // r0^(j + 1) at this lane's first wire
  {
    const T r2 = F::mul(r0, r0), r4 = F::mul(r2, r2), r8 = F::mul(r4, r4);
    rj = sel(h, F::mul(r8, r0), r0);
  }
  const uint32_t jlo = 8u * h, jhi = jlo + 8u < C ? jlo + 8u : C;
  for (uint32_t jg = jlo; jg < jlo + 8u; jg += GS) {  // same trip count on both lanes
    mac128 Aa[GS], Bb[GS];
    T mc[GS];
#pragma unroll
    for (int q = 0; q < GS; q++) {
      mac_zero(Aa[q]);
      mac_zero(Bb[q]);
    }
    auto fetch = [&](uint32_t k, T* dst) {
#pragma unroll
      for (int q = 0; q < GS; q++) {
        const uint32_t i = k * C + jg + q;
        const bool valid = (k < K) && (jg + q < jhi) && (i < M);
        const uint32_t msk = valid ? 0xffffffffu : 0u;
        const uint4 v = ((const uint4*)sc.meas)[(size_t)(valid ? i : 0) * ld + r];
        dst[q] = mk128(v.x & msk, v.y & msk, v.z & msk, v.w & msk);
      }
    };
    fetch(0, mc);
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
    mac128 Gq;
    mac_zero(Gq);
#pragma unroll
    for (int q = 0; q < GS; q++) {
      const uint32_t j = jg + q;
      const bool wj = j < jhi;  // lane-dependent only when C is not 16
      const uint32_t jj = wj ? j : 0u;  // wire 0 always exists: in-bounds loads
      mac_add(Bb[q], ldf<F>(sc.proofs, 2 * jj + 1, ld, r), L0);
      const T f1 = F::sub(mac_reduce_f(Bb[q]), halfL);
      const T Aq = mac_reduce_f(Aa[q]);
      mac128 F0;
      mac_zero(F0);
      mac_add(F0, ldf<F>(sc.proofs, 2 * jj, ld, r), L0);
      mac_add(F0, rj, Aq);
      const T f0 = mac_reduce_f(F0);
      T u = F::zero(), w = F::zero();
      if (wj) {  // only this lane's wires are checked and summed (no cross-lane work inside)
        u = F::add(lv(1 + 2 * jj), f0);
        w = F::add(lv(2 + 2 * jj), f1);
      }
      mac_add(Gq, u, w);
      rj = F::mul(rj, r0);
    }
    G = F::add(G, mac_reduce_f(Gq));
  }
  // 5. the pair's halves meet: G, S, the decode verdict; then decide and the prepare message
  G = F::add(G, pair_x(G));
  T S = sum_reduce(Ssum);
  S = F::add(S, pair_x(S));
  decode_ok = decode_ok && pair_x((uint32_t)decode_ok) != 0u;
  const T r1 = ldf<F>(sc.jr, 1, ld, r);
  const T v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), F::sub(S, half)));
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
  if (h == 0) {
    ((uint4*)out.prep_msgs)[r] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
    out.status[r] = status;
  }
}

// ---- the kernel: XOF (k_xof_pair's lane split, plus the fused accumulate and the leader-share
//      pull of the executor groups), then query_pair on the same lanes ------------------------
// PAIR_OCC: waves per SIMD the compiler must fit (0: its own choice, 188 VGPRs = 2 waves)
#ifndef PAIR_OCC
#define PAIR_OCC 0
#endif
template <bool FUSE, bool PULL>
__global__ __launch_bounds__(256, PAIR_OCC) void k_prep_hp(DevParams p, InPtrs in, Scratch sc,
                                                           OutPtrs out) {
  const uint32_t tid = threadIdx.x, h = tid & 1u, lane = tid & 63u;
  const uint32_t r = blockIdx.x * 128 + (tid >> 1);
  const bool live = r < p.n;
  const uint32_t rr = live ? r : p.n - 1;  // a dead pair computes on a valid report, stores nothing
  // fused accumulate: a wave (32 reports) is fused when all its reports are live and every one
  // with an in-range segment id has the same one (lanes with ids >= nseg are masked out)
  bool fuse = false, oor = false, haspad = false;
  uint32_t s0 = 0;
  if constexpr (FUSE) {
    const uint32_t sg = live ? (sc.seg ? sc.seg[r] : 0u) : 0xffffffffu;
    const uint64_t inr = __ballot(live && sg < p.nseg);
    s0 = inr ? (uint32_t)__shfl((int)sg, __ffsll((long long)inr) - 1) : 0xffffffffu;
    oor = live && sg >= p.nseg;
    fuse = inr != 0 && __all(live && (sg == s0 || sg >= p.nseg));
    haspad = __any(oor);
    if (lane == 0 && (r - (lane >> 1)) < p.n && !fuse) sc.wseg[r >> 5] = 0xffffffffu;
  }
  uint32_t flag = p.force_slow;
  uint32_t nonce[4], km[4], kb[4];
  load16(in.nonces + 16 * (size_t)rr, nonce);
  const uint8_t* hs = in.helper + (size_t)rr * p.helper_share_len;
  load16(hs, km);
  load16(hs + 32, kb);
  KState st;
  kzero(st);
  // 1. even: the share XOF header XOF(k_meas, dst(1), [1]); odd: the query-randomness message
  //    XOF(vk, dst(5), [PROOFS] || nonce)
  {
    Msg ma, q;
    msg_zero(ma);
    msg_dst(ma, p.dst[1]);
    msg_bytes16(ma, 9, km);
    msg_byte(ma, 25, 1);
    msg_byte(ma, 26, 0x01);
    ma.w[41] ^= 0x80000000u;
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
    for (int i = 0; i < 42; i++) kxor_word(st, i, h ? q.w[i] : ma.w[i]);
    keccak_p12(st);
  }
  if (h && live) {  // query randomness (one element, block 0)
    uint32_t w[4] = {kword(st, 0), kword(st, 1), kword(st, 2), kword(st, 3)};
    put_elem<F>(p, sc.qr, 0, rr, w, flag);
  }
  {  // the odd lane restarts its state for the joint-rand part
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
  const uint32_t M = p.meas_len, K = (M * 16 + 167) / 168;
  const uint32_t Lb = 42 + M * 16, B = Lb / 168, rem = Lb % 168;  // absorb blocks 0..B
  const int Mi = (int)M;
  // wave totals of share elements e0, e0 + 1 (the even lanes' words; odd and masked lanes add
  // nothing): slot lane >> 2 on each lane of a quad
  auto fused_pair = [&](int e0, f128 x0, f128 x1) __attribute__((always_inline)) {
    if (e0 >= Mi) return;  // wave-uniform
    if (h || (haspad && oor)) {
      x0 = zero128();
      x1 = zero128();
    }
    const uint32_t tot = wave_halfsum2(x0, x1, lane);
    const int e = e0 + (int)(lane >> 5);
    if ((lane & 3u) == 0 && e < Mi)
      sc.wpart[((size_t)(r >> 5) * M + (uint32_t)e) * 8u + ((lane >> 2) & 7u)] = tot;
  };
  auto fuse_block = [&](uint32_t b, uint32_t q0, uint32_t q1) __attribute__((always_inline)) {
    const int e0 = 21 * (int)(b >> 1);
    const f128 z = zero128();
    if ((b & 1) == 0) {
#pragma unroll
      for (int t = 0; t < 10; t += 2)
        fused_pair(e0 + t, mk128(kword(st, 4 * t), kword(st, 4 * t + 1), kword(st, 4 * t + 2),
                                 kword(st, 4 * t + 3)),
                   mk128(kword(st, 4 * t + 4), kword(st, 4 * t + 5), kword(st, 4 * t + 6),
                         kword(st, 4 * t + 7)));
    } else {
      fused_pair(e0 + 10, mk128(q0, q1, kword(st, 0), kword(st, 1)),
                 mk128(kword(st, 2), kword(st, 3), kword(st, 4), kword(st, 5)));
#pragma unroll
      for (int t = 1; t < 10; t += 2)
        fused_pair(e0 + 11 + t,
                   mk128(kword(st, 2 + 4 * t), kword(st, 3 + 4 * t), kword(st, 4 + 4 * t),
                         kword(st, 5 + 4 * t)),
                   t + 1 < 10 ? mk128(kword(st, 6 + 4 * t), kword(st, 7 + 4 * t),
                                      kword(st, 8 + 4 * t), kword(st, 9 + 4 * t))
                              : z);
    }
  };
  // PULL: the wave's 32 leader shares are one contiguous run of 32 Q 16-byte pieces, NR rows of
  // 64 (the last one partial); iteration b of the share loop copies rows [NR (b-1) / (B-1),
  // NR b / (B-1)) (1 or 2), lane l taking piece 64 row + l: each load reads 1 KiB of host bytes
  const uint32_t Q = PULL ? p.prep_share_len / 16 : 0u, NR = (32 * Q + 63) / 64;
  const size_t wbase = PULL ? (size_t)(r - (lane >> 1)) * Q + lane : 0;
  const uint4* lsrc = PULL ? (const uint4*)in.leader_src + wbase : nullptr;
  uint4* ldst = PULL ? (uint4*)in.leader + wbase : nullptr;
  if constexpr (PULL) {
    if (h == 0 && live) {
      if (in.seg_dst) in.seg_dst[r] = in.seg_src[r];
      if (in.accept_dst) in.accept_dst[r] = in.accept_src[r];
    }
  }
  // 2. the share phase: block b of the squeeze (even) is block b of the absorb (odd)
  uint32_t tail[11];
#pragma unroll
  for (int t = 0; t < 11; t++) tail[t] = 0;
  uint32_t pend0 = 0, pend1 = 0;
  TruncSink ts(p, sc.out, rr);
  if (FUSE && fuse) fuse_block(0, 0, 0);
  if (h == 0 && live) squeeze_meas<false>(p, st, 0, M, pend0, pend1, sc.meas, rr, flag, ts);
  absorb_share_block<true, false>(st, h, true, tail, pre, rem);
  keccak_p12(st);
#pragma unroll 1
  for (uint32_t b = 1; b < B; b++) {
    const bool hasW = b < K;  // uniform
    uint4 pc0, pc1;
    uint32_t q0 = 0, q1 = 0;
    bool v0 = false, v1 = false;
    if constexpr (PULL) {
      q0 = NR * (b - 1) / (B - 1);
      q1 = NR * b / (B - 1);
      // whole waves are live or dead (n % 32 == 0 with the pull): a dead wave past the group
      // must not copy, its pieces lie past both the staging run and the device leader array
      v0 = live && q0 < q1 && 64 * q0 + lane < 32 * Q;
      v1 = live && q0 + 1 < q1 && 64 * (q0 + 1) + lane < 32 * Q;
      if (v0) pc0 = lsrc[64 * (size_t)q0];
      if (v1) pc1 = lsrc[64 * (size_t)(q0 + 1)];
    }
    if (FUSE && fuse && hasW) fuse_block(b, pend0, pend1);
    if (hasW && h == 0 && live) squeeze_meas<false>(p, st, b, M, pend0, pend1, sc.meas, rr, flag, ts);
    absorb_share_block<false, false>(st, h, hasW, tail, pre, rem);
    keccak_p12(st);  // even: next squeeze block; odd: absorb
    if constexpr (PULL) {
      if (v0) ldst[64 * (size_t)q0] = pc0;
      if (v1) ldst[64 * (size_t)(q0 + 1)] = pc1;
    }
  }
  {
    const bool hasW = B < K;
    if (FUSE && fuse && hasW) fuse_block(B, pend0, pend1);
    if (hasW && h == 0 && live) squeeze_meas<false>(p, st, B, M, pend0, pend1, sc.meas, rr, flag, ts);
    absorb_share_block<false, true>(st, h, hasW, tail, pre, rem);
    keccak_p12(st);
  }
  uint32_t part[4] = {kword(st, 0), kword(st, 1), kword(st, 2), kword(st, 3)};
  // 3. even: the proofs share XOF(k_proofs, dst(2), [PROOFS, 1]); odd: corrected seed and
  //    joint randomness
  if (h == 0) {
    uint32_t kp[4];
    load16(hs + 16, kp);
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
  flag |= pair_x(flag);  // any rejection-sampling event of either lane flags the report
  if (h == 0 && live) sc.flag[rr] = (uint8_t)flag;
  if constexpr (FUSE) {
    if (fuse) {  // all 64 lanes are live here
      const bool anyflag = __any(flag != 0);
      if (lane == 0) sc.wseg[r >> 5] = anyflag ? 0xffffffffu : s0;
    }
  }
  // the query reads rows this wave's lanes (and the partner) just wrote
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (live && !flag) query_pair(p, in, sc, out, r, h);  // flagged: deferred to k_slow_redo
}

}  // namespace

bool prep_pair_takes(const DevParams& p, bool pull);
void launch_prep_pair_k(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st,
                        bool fuse, bool pull);
// Prio3Histogram (P = 32) on lane pairs: true if launched.  fuse: the fused accumulate into
// sc.wpart / sc.wseg with 32-report waves; pull: in.leader_src etc. set (executor groups).
bool launch_prep_pair(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st,
                      bool fuse, bool pull) {
  return prep_pair_takes(p, pull) ? (launch_prep_pair_k(p, in, sc, out, st, fuse, pull), true)
                                 : false;
}
// the instances the pair query covers: Histogram with P = 32, at most 16 calls and a chunk of at
// most 16 (the wires split 8 / 8); pull: whole 32-report waves and at most two 1 KiB rows of
// leader-share pieces per share-loop iteration
bool prep_pair_takes(const DevParams& p, bool pull) {
  const uint32_t B = (42 + p.meas_len * 16) / 168;
  if (p.es != 16 || p.kind != PRIO3_HISTOGRAM || p.P != 32 || !p.jr_len || B < 2 ||
      p.calls > 16 || p.chunk > 16 || p.arity != 2 * p.chunk)
    return false;
  if (pull && (p.prep_share_len % 16 != 0 || p.n % 32 != 0 ||
               (32 * (p.prep_share_len / 16) + 63) / 64 > 2 * (B - 1)))
    return false;
  return true;
}
void launch_prep_pair_k(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st,
                        bool fuse, bool pull) {
  const uint32_t blocks = (p.n + 127) / 128;
  if (fuse && pull)
    k_prep_hp<true, true><<<blocks, 256, 0, st>>>(p, in, sc, out);
  else if (fuse)
    k_prep_hp<true, false><<<blocks, 256, 0, st>>>(p, in, sc, out);
  else if (pull)
    k_prep_hp<false, true><<<blocks, 256, 0, st>>>(p, in, sc, out);
  else
    k_prep_hp<false, false><<<blocks, 256, 0, st>>>(p, in, sc, out);
}
