// prio3_client.hip -- leader-side preparation (k_leader_init / k_leader_next, below) and the
// on-device synthetic report generator: the client's Prio3 shard
// (VDAF-08 7.2.1, prio Prio3::shard) followed by the leader's prepare_init (agg_id 0), so
// that benchmarks and full-size tests get honest, distinct reports at HBM speed without a
// CPU in the loop.  Report i is derived from (seed, i) exactly like the oracle's
// orc_gen_reports: stream = TurboSHAKE128("janus-amd-gen" || seed || i, D=1) gives the
// nonce (16 B), the shard randomness (5 or 3 seeds) and the measurement (8 B per entry).
//
// Prover path per lane: record the validity circuit's wire values (num_shares = 1), turn each
// wire into coefficients with a size-P inverse DFT, evaluate on the 2P-th roots with a
// size-2P DFT, apply the gadget pointwise, inverse-DFT back: the gadget polynomial
// (prio FlpGeneric::prove, ProveShimGadget).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "prio3_common.h"
#include "prio3_runtime.h"
#include "prio3_mp64_xof.h"

struct GenScratch {
  void *meas, *hm, *lm, *wires, *evals, *g, *tmp, *proof, *hp, *prand, *jr, *qr, *L, *PV, *acc;
};
struct GenOut {
  uint8_t *nonces, *pub, *helper, *leader_ps, *leader_out, *leader_in;
  uint64_t* meas;
  uint8_t* flags;
};

// XOF(seed, dst, binder).expand_into_vec(n) into an SoA column set (no rejection: flagged)
template <class F>
DEV void expand_to(const DevParams& p, const uint32_t* dst2, const uint32_t* seed,
                   const uint8_t* binder, int blen, uint32_t n, void* base, uint32_t r,
                   uint32_t& flag) {
  KState s;
  kzero(s);
  Msg m;
  msg_zero(m);
  msg_dst(m, dst2);
  msg_bytes16(m, 9, seed);
  for (int i = 0; i < blen; i++) msg_byte(m, 25 + i, binder[i]);
  msg_absorb_final(s, m, 25 + blen);
  const uint32_t K = (n * F::ES + 167) / 168;
  uint32_t q0 = 0, q1 = 0;
  for (uint32_t b = 0; b < K; b++) {
    squeeze_block<F>(p, s, b, n, q0, q1, base, r, flag);
    if (b + 1 < K) keccak_p12(s);
  }
}

// joint_rand_part = XOF(blind, dst(7), [agg_id] || nonce || enc(share)) -> 16 bytes; Sw(u) is
// word u of the encoded share (0 past its end), asked for in increasing u.
template <class Get>
DEV void jr_part_words(const DevParams& p, const uint32_t* blind, uint32_t agg_id,
                       const uint32_t* nonce, uint32_t share_bytes, Get&& Sw, uint32_t* part) {
  Msg pm;
  msg_zero(pm);
  msg_dst(pm, p.dst[7]);
  msg_bytes16(pm, 9, blind);
  msg_byte(pm, 25, agg_id);
  msg_bytes16(pm, 26, nonce);
  const uint32_t L = 42 + share_bytes;
  const uint32_t B = L / 168, rem = L % 168;
  KState s;
  kzero(s);
  uint32_t prev = 0;  // word u - 1 of the share (the 16-bit funnel shift's low half)
  for (uint32_t b = 0; b <= B; b++) {
    uint32_t x[42];
#pragma unroll
    for (int j = 0; j < 42; j++) {
      uint32_t v;
      if (b == 0 && j < 10) {
        v = pm.w[j];
      } else if (b == 0 && j == 10) {
        prev = Sw(0);
        v = (pm.w[10] & 0xffffu) | (prev << 16);
      } else {
        const uint32_t u = 42 * b + j - 11;
        const uint32_t nx = Sw(u + 1);
        v = __builtin_amdgcn_alignbit(nx, prev, 16);
        prev = nx;
      }
      if (b == B) {
        const uint32_t lo = 4 * j;
        uint32_t mask = (lo + 4 <= rem) ? 0xffffffffu
                                        : (lo >= rem ? 0u : ((1u << (8 * (rem - lo))) - 1u));
        v &= mask;
        if ((uint32_t)j == (rem >> 2)) v ^= 1u << (8 * (rem & 3));
        if (j == 41) v ^= 0x80000000u;
      }
      x[j] = v;
    }
#pragma unroll
    for (int j = 0; j < 42; j++) kxor_word(s, j, x[j]);
    keccak_p12(s);
  }
  for (int k = 0; k < 4; k++) part[k] = kword(s, k);
}

// the same with the share read back from an SoA scratch column set
template <class F>
DEV void jr_part_scratch(const DevParams& p, const uint32_t* blind, uint32_t agg_id,
                         const uint32_t* nonce, const void* src, uint32_t r, uint32_t* part) {
  constexpr uint32_t WPE = F::ES / 4;  // words per element
  const uint32_t nwords = p.meas_len * WPE;
  jr_part_words(p, blind, agg_id, nonce, p.meas_len * F::ES, [&](uint32_t u) -> uint32_t {
    if (u >= nwords) return 0u;
    const uint32_t e = u / WPE, k = u % WPE;
    return ((const uint32_t*)src)[((size_t)e * p.ld + r) * WPE + k];
  }, part);
}

template <class F>
DEV void seed_of(const DevParams& p, uint32_t usage, const uint32_t* seed16, const uint32_t* a,
                 const uint32_t* b, uint32_t* out) {  // derive_seed(seed, dst(usage), a || b)
  KState s;
  kzero(s);
  Msg m;
  msg_zero(m);
  msg_dst(m, p.dst[usage]);
  msg_bytes16(m, 9, seed16);
  msg_bytes16(m, 25, a);
  msg_bytes16(m, 41, b);
  msg_absorb_final(s, m, 57);
  for (int k = 0; k < 4; k++) out[k] = kword(s, k);
}

// out[c] = IDFT_n(in)[c] (natural order in and out; tmp is scratch)
template <class F>
DEV void idft_lane(const DevParams& p, const void* in, uint32_t in_len, void* out, uint32_t n,
                   uint32_t logn, uint32_t r, typename F::T n_inv) {
  typedef typename F::T T;
  const size_t ld = p.ld;
  for (uint32_t e = 0; e < n; e++)
    F::store(out, (size_t)bitrev(e, logn) * ld + r,
             e < in_len ? F::load(in, (size_t)e * ld + r) : F::zero());
  dft_lane<F>(p, out, r, n, logn);
  // out[c] <- out[(n - c) % n] / n
  F::store(out, r, F::mul(F::load(out, r), n_inv));
  F::store(out, (size_t)(n / 2) * ld + r, F::mul(F::load(out, (size_t)(n / 2) * ld + r), n_inv));
  for (uint32_t c = 1; c < n / 2; c++) {
    T a = F::load(out, (size_t)c * ld + r), b = F::load(out, (size_t)(n - c) * ld + r);
    F::store(out, (size_t)c * ld + r, F::mul(b, n_inv));
    F::store(out, (size_t)(n - c) * ld + r, F::mul(a, n_inv));
  }
}

template <class F>
DEV typename F::T gadget_eval_lane(const DevParams& p, const void* ev, uint32_t k, uint32_t n2,
                                   uint32_t r) {
  typedef typename F::T T;
  const size_t ld = p.ld;
  auto E = [&](uint32_t w) { return F::load(ev, ((size_t)w * n2 + k) * ld + r); };
  if (p.kind == PRIO3_COUNT) return F::mul(E(0), E(1));
  if (p.kind == PRIO3_SUM) {
    T x = E(0);
    return F::sub(F::mul(x, x), x);
  }
  T s = F::zero();
  for (uint32_t j = 0; j < p.chunk; j++) s = F::add(s, F::mul(E(2 * j), E(2 * j + 1)));
  return s;
}

// FlpGeneric::prove (VDAF-08 7.3.3.1, num_shares = 1) of the single-gadget circuits -- Count,
// Sum, and the ParallelSum(Mul) range check of SumVec / Histogram -- on one lane: the wire values
// of every gadget call recorded (seed = prand[w] at point 0), each wire polynomial evaluated on
// the 2P-th roots (size-P inverse DFT, size-2P DFT), the gadget applied pointwise and the gadget
// polynomial's coefficients back by a size-2P inverse DFT.  meas / prand / jr / proof: SoA
// column sets (the first jr element is the circuit's joint randomness); proof = prand || coeffs.
template <class F>
DEV void prove_lane(const DevParams& p, const GenScratch& gs, const void* meas, const void* prand,
                    const void* jr, void* proof, uint32_t r, typename F::T invP,
                    typename F::T inv2P) {
  typedef typename F::T T;
  const size_t ld = p.ld;
  const uint32_t M = p.meas_len, A = p.arity, P = p.P, P2 = 2 * P;
  for (uint32_t w = 0; w < A; w++) {
    F::store(gs.wires, ((size_t)w * P) * ld + r, F::load(prand, (size_t)w * ld + r));
    for (uint32_t c = 1; c < P; c++) F::store(gs.wires, ((size_t)w * P + c) * ld + r, F::zero());
  }
  auto wset = [&](uint32_t w, uint32_t c, const T& x) {
    F::store(gs.wires, ((size_t)w * P + c) * ld + r, x);
  };
  if (p.kind == PRIO3_COUNT) {
    T m = F::load(meas, r);
    wset(0, 1, m);
    wset(1, 1, m);
  } else if (p.kind == PRIO3_SUM) {
    for (uint32_t i = 0; i < M; i++) wset(0, i + 1, F::load(meas, (size_t)i * ld + r));
  } else {
    const T r0 = F::load(jr, r);
    T rp = r0;
    for (uint32_t k = 0; k < p.calls; k++)
      for (uint32_t j = 0; j < p.chunk; j++) {
        const uint32_t i = k * p.chunk + j;
        const T m = i < M ? F::load(meas, (size_t)i * ld + r) : F::zero();
        wset(2 * j, k + 1, F::mul(rp, m));
        wset(2 * j + 1, k + 1, F::sub(m, F::one()));
        rp = F::mul(rp, r0);
      }
  }
  // ---- wire polys -> evaluations on the 2P-th roots ----
  for (uint32_t w = 0; w < A; w++) {
    void* wcol = (uint8_t*)gs.wires + (size_t)w * P * ld * F::ES;
    idft_lane<F>(p, wcol, P, gs.tmp, P, p.logP, r, invP);  // coefficients in tmp[0..P)
    void* ecol = (uint8_t*)gs.evals + (size_t)w * P2 * ld * F::ES;
    for (uint32_t e = 0; e < P2; e++)
      F::store(ecol, (size_t)bitrev(e, p.logP + 1) * ld + r,
               e < P ? F::load(gs.tmp, (size_t)e * ld + r) : F::zero());
    dft_lane<F>(p, ecol, r, P2, p.logP + 1);
  }
  for (uint32_t k = 0; k < P2; k++)
    F::store(gs.g, (size_t)k * ld + r, gadget_eval_lane<F>(p, gs.evals, k, P2, r));
  idft_lane<F>(p, gs.g, P2, gs.tmp, P2, p.logP + 1, r, inv2P);  // gadget poly coefficients
  // proof = prove_rand || coeffs[0..glen)
  for (uint32_t w = 0; w < A; w++)
    F::store(proof, (size_t)w * ld + r, F::load(prand, (size_t)w * ld + r));
  for (uint32_t e = 0; e < p.glen; e++)
    F::store(proof, (size_t)(A + e) * ld + r, F::load(gs.tmp, (size_t)e * ld + r));
}

template <class F>
__global__ __launch_bounds__(64) void k_gen(DevParams p, uint64_t seed, uint64_t first,
                                            GenScratch gs, GenOut go, typename F::T invP,
                                            typename F::T inv2P) {
  typedef typename F::T T;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  const size_t ld = p.ld;
  const uint64_t idx = first + r;
  const uint32_t M = p.meas_len, A = p.arity, PL = p.proof_len;
  const bool JR = p.jr_len > 0;
  const uint32_t mstride = p.kind == PRIO3_SUMVEC ? p.length : 1;
  uint32_t flag = 0;
  // ---- per-report stream: nonce || rand || measurement bytes ----
  KState st;
  kzero(st);
  {
    Msg m;
    msg_zero(m);
    const char tag[13] = {'j', 'a', 'n', 'u', 's', '-', 'a', 'm', 'd', '-', 'g', 'e', 'n'};
    for (int i = 0; i < 13; i++) msg_byte(m, i, (uint8_t)tag[i]);
    for (int i = 0; i < 8; i++) msg_byte(m, 13 + i, (uint32_t)(seed >> (8 * i)));
    for (int i = 0; i < 8; i++) msg_byte(m, 21 + i, (uint32_t)(idx >> (8 * i)));
    msg_absorb_final(st, m, 29);
  }
  uint32_t nonce[4], k_hm[4], k_hp[4], k_hb[4] = {0, 0, 0, 0}, k_lb[4] = {0, 0, 0, 0}, k_pr[4];
  for (int k = 0; k < 4; k++) {
    nonce[k] = kword(st, k);
    k_hm[k] = kword(st, 4 + k);
    k_hp[k] = kword(st, 8 + k);
  }
  if (JR) {
    for (int k = 0; k < 4; k++) {
      k_hb[k] = kword(st, 12 + k);
      k_lb[k] = kword(st, 16 + k);
      k_pr[k] = kword(st, 20 + k);
    }
  } else {
    for (int k = 0; k < 4; k++) k_pr[k] = kword(st, 12 + k);
  }
  // measurement bytes start at stream byte 96 (word 24); 168-byte blocks
  uint32_t blk = 0;
  auto stream_word = [&](uint32_t wi) -> uint32_t {  // wi: absolute word index, non-decreasing
    while (wi >= 42 * (blk + 1)) {
      keccak_p12(st);
      blk++;
    }
    uint32_t w = wi - 42 * blk;
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 42; q++)
      if ((uint32_t)q == w) v = kword(st, q);
    return v;
  };
  // encode measurement into gs.meas and record it
  for (uint32_t e = 0; e < M; e++) F::store(gs.meas, (size_t)e * ld + r, F::zero());
  for (uint32_t e = 0; e < mstride; e++) {
    uint64_t v = (uint64_t)stream_word(24 + 2 * e) | ((uint64_t)stream_word(25 + 2 * e) << 32);
    switch (p.kind) {
      case PRIO3_COUNT:
        v &= 1;
        break;
      case PRIO3_SUM:
      case PRIO3_SUMVEC:
        if (p.bits < 64) v &= (1ull << p.bits) - 1;
        break;
      default:
        v %= p.length;
        break;
    }
    if (go.meas) go.meas[(size_t)r * mstride + e] = v;
    if (p.kind == PRIO3_HISTOGRAM) {
      F::store(gs.meas, (size_t)v * ld + r, F::one());
    } else if (p.kind == PRIO3_COUNT) {
      F::store(gs.meas, r, F::from_u32((uint32_t)v));
    } else {
      for (uint32_t b = 0; b < p.bits; b++)
        F::store(gs.meas, (size_t)(e * p.bits + b) * ld + r, F::from_u32((uint32_t)((v >> b) & 1)));
    }
  }
  // ---- shard ----
  const uint8_t b_hm[1] = {1};
  expand_to<F>(p, p.dst[1], k_hm, b_hm, 1, M, gs.hm, r, flag);
  for (uint32_t e = 0; e < M; e++)
    F::store(gs.lm, (size_t)e * ld + r,
             F::sub(F::load(gs.meas, (size_t)e * ld + r), F::load(gs.hm, (size_t)e * ld + r)));
  uint32_t part0[4] = {0, 0, 0, 0}, part1[4] = {0, 0, 0, 0}, jseed[4];
  if (JR) {
    jr_part_scratch<F>(p, k_hb, 1, nonce, gs.hm, r, part1);
    jr_part_scratch<F>(p, k_lb, 0, nonce, gs.lm, r, part0);
    const uint32_t zero[4] = {0, 0, 0, 0};
    seed_of<F>(p, 6, zero, part0, part1, jseed);
    const uint8_t b1[1] = {1};
    expand_to<F>(p, p.dst[3], jseed, b1, 1, p.jr_len, gs.jr, r, flag);
  }
  {
    const uint8_t b1[1] = {1};
    expand_to<F>(p, p.dst[4], k_pr, b1, 1, A, gs.prand, r, flag);
  }
  prove_lane<F>(p, gs, gs.meas, gs.prand, gs.jr, gs.proof, r, invP, inv2P);
  // leader proofs share = proof - helper proofs share
  {
    const uint8_t b2[2] = {1, 1};
    expand_to<F>(p, p.dst[2], k_hp, b2, 2, PL, gs.hp, r, flag);
    for (uint32_t e = 0; e < PL; e++)
      F::store(gs.hp, (size_t)e * ld + r,
               F::sub(F::load(gs.proof, (size_t)e * ld + r), F::load(gs.hp, (size_t)e * ld + r)));
  }
  // ---- leader prepare_init (agg_id 0): query on (lm, leader proofs share) ----
  {
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[5]);
    msg_bytes16(m, 9, p.vk);
    msg_byte(m, 25, 1);
    msg_bytes16(m, 26, nonce);
    msg_absorb_final(s, m, 42);
    uint32_t w[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
    put_elem<F>(p, gs.qr, 0, r, w, flag);
  }
  const T t = F::load(gs.qr, r);
  T v, pt;
  if (!flp_query_lane<F>(p, gs.lm, gs.hp, gs.jr, t, gs.L, gs.PV, gs.acc, r, v, pt)) flag = 1;
  uint8_t* lps = go.leader_ps + (size_t)r * p.prep_share_len;
  F::store(lps, 0, v);
  for (uint32_t w = 0; w < A; w++) F::store(lps, 1 + w, F::load(gs.acc, (size_t)w * ld + r));
  F::store(lps, A + 1, pt);
  if (JR) *(uint4*)(lps + (size_t)p.verifier_len * F::ES) = make_uint4(part0[0], part0[1], part0[2], part0[3]);
  // leader input share = enc(meas share) || enc(proofs share) [|| k_blind]
  if (go.leader_in) {
    uint8_t* li = go.leader_in + (size_t)r * p.leader_share_len;
    for (uint32_t e = 0; e < M; e++) F::store(li, e, F::load(gs.lm, (size_t)e * ld + r));
    for (uint32_t e = 0; e < PL; e++)
      F::store(li + (size_t)M * F::ES, e, F::load(gs.hp, (size_t)e * ld + r));
    if (JR) *(uint4*)(li + (size_t)(M + PL) * F::ES) = make_uint4(k_lb[0], k_lb[1], k_lb[2], k_lb[3]);
  }
  // ---- public outputs ----
  *(uint4*)(go.nonces + 16 * (size_t)r) = make_uint4(nonce[0], nonce[1], nonce[2], nonce[3]);
  uint8_t* hs = go.helper + (size_t)r * p.helper_share_len;
  *(uint4*)hs = make_uint4(k_hm[0], k_hm[1], k_hm[2], k_hm[3]);
  *(uint4*)(hs + 16) = make_uint4(k_hp[0], k_hp[1], k_hp[2], k_hp[3]);
  if (JR) {
    *(uint4*)(hs + 32) = make_uint4(k_hb[0], k_hb[1], k_hb[2], k_hb[3]);
    uint8_t* pb = go.pub + (size_t)r * p.public_share_len;
    *(uint4*)pb = make_uint4(part0[0], part0[1], part0[2], part0[3]);
    *(uint4*)(pb + 16) = make_uint4(part1[0], part1[1], part1[2], part1[3]);
  }
  // leader output share = truncate(leader meas share)
  if (go.leader_out) {
    uint8_t* lo = go.leader_out + (size_t)r * p.out_len * F::ES;
    if (p.kind == PRIO3_SUM || p.kind == PRIO3_SUMVEC) {
      const uint32_t outs = p.kind == PRIO3_SUM ? 1 : p.out_len;
      for (uint32_t e = 0; e < outs; e++) {
        T acc = F::zero(), pw = F::one();
        for (uint32_t b = 0; b < p.bits; b++) {
          acc = F::add(acc, F::mul(pw, F::load(gs.lm, (size_t)(e * p.bits + b) * ld + r)));
          pw = F::add(pw, pw);
        }
        F::store(lo, e, acc);
      }
    } else {
      for (uint32_t e = 0; e < M; e++) F::store(lo, e, F::load(gs.lm, (size_t)e * ld + r));
    }
  }
  if (go.flags) go.flags[r] = (uint8_t)flag;
}

// ====================================================================================
// Prio3FixedPointBoundedL2VecSum client.  Report i of (seed, i): the stream
// TurboSHAKE128("janus-amd-gen" || seed || i, D = 1) as for the other kinds gives the nonce and
// the five seeds (helper measurement, helper proofs, helper blind, leader blind, prove rand);
// entry e is the signed byte at stream offset 96 + e shifted right by gsh (the host picks the
// smallest gsh with length * 2^(14 - 2 gsh) < 2^(2 bits - 2), so the claimed squared norm always
// fits: |x| <= 2^(7 - gsh) / 2^(bits - 1)).  oracle/fpvec_py.py gen_report is the same in Python.
// Three launches per chunk: k_fg_shares (lane per report: entries, the measurement share, both
// joint-rand parts, joint and prove randomness), k_fg_prove (one 256-thread workgroup per report:
// both gadget polynomials by NTTs in LDS) and k_fg_finish (lane per report: the leader's proofs
// share); then the engine's own device leader prepare_init on the explicit leader shares.
// ====================================================================================
struct FgBufs {
  int16_t* X;        // [m][length] entries
  uint64_t* norm;    // [m] claimed squared norm (sum of X^2)
  uint8_t* lin;      // [m][leader_share_len] leader input shares being built
  void* jr;          // SoA [2][ld] joint randomness
  void* pr;          // SoA [arity + chunk1][ld] prove randomness
  uint8_t* proof;    // [m][proof_len] 16-byte elements
  uint32_t gsh;
};
// Field128 tables of one gadget's NTTs (host-computed, device memory): w[i] = omega_P^i (i < P),
// tw[m] = psi^m / P and ipsi[m] = psi^-m (m < P) for psi a primitive 2P-th root
struct FgGadget {
  const f128 *w, *tw, *ipsi;
  f128 c2P;  // 1 / (2P)
};

// the report's stream word wi, 168-byte blocks; wi never below the current block's first word
struct GenStream {
  KState st;
  uint32_t blk = 0;
  DEV uint32_t word(uint32_t wi) {
    while (wi >= 42 * (blk + 1)) {
      keccak_p12(st);
      blk++;
    }
    const uint32_t w = wi - 42 * blk;
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 42; q++)
      if ((uint32_t)q == w) v = kword(st, q);
    return v;
  }
};

DEV void gen_stream_init(KState& st, uint64_t seed, uint64_t idx) {
  kzero(st);
  Msg m;
  msg_zero(m);
  const char tag[13] = {'j', 'a', 'n', 'u', 's', '-', 'a', 'm', 'd', '-', 'g', 'e', 'n'};
  for (int i = 0; i < 13; i++) msg_byte(m, i, (uint8_t)tag[i]);
  for (int i = 0; i < 8; i++) msg_byte(m, 13 + i, (uint32_t)(seed >> (8 * i)));
  for (int i = 0; i < 8; i++) msg_byte(m, 21 + i, (uint32_t)(idx >> (8 * i)));
  msg_absorb_final(st, m, 29);
}

// measurement bit i of the encoding (entry bits y_e = X_e + 2^(bits-1), little-endian, then the
// claimed norm's 2 bits - 2 bits); cur / ce cache the current entry
DEV uint32_t fg_mbit(const DevParams& p, const int16_t* X, uint64_t N, uint32_t i) {
  const uint32_t nb = p.bits, nl = nb * p.length;
  if (i >= nl) return (uint32_t)(N >> (i - nl)) & 1u;
  const uint32_t y = (uint32_t)(int32_t)X[i / nb] + (1u << (nb - 1));
  return (y >> (i % nb)) & 1u;
}

__global__ __launch_bounds__(64) void k_fg_shares(DevParams p, uint64_t seed, uint64_t first,
                                                  GenOut go, FgBufs fb) {
  typedef Fp128 F;
  typedef f128 T;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  const uint32_t M = p.meas_len, Ln = p.length, nb = p.bits;
  uint32_t flag = 0;
  GenStream gst;
  gen_stream_init(gst.st, seed, first + r);
  uint32_t nonce[4], k_hm[4], k_hp[4], k_hb[4], k_lb[4], k_pr[4];
  for (int k = 0; k < 4; k++) {
    nonce[k] = kword(gst.st, k);
    k_hm[k] = kword(gst.st, 4 + k);
    k_hp[k] = kword(gst.st, 8 + k);
    k_hb[k] = kword(gst.st, 12 + k);
    k_lb[k] = kword(gst.st, 16 + k);
    k_pr[k] = kword(gst.st, 20 + k);
  }
  // entries: signed bytes from stream offset 96
  int16_t* X = fb.X + (size_t)r * Ln;
  uint64_t N = 0;
  for (uint32_t e = 0; e < Ln; e++) {
    const uint32_t B = 96 + e;
    const int32_t v = (int32_t)(int8_t)(gst.word(B >> 2) >> (8 * (B & 3))) >> fb.gsh;
    X[e] = (int16_t)v;
    N += (uint64_t)((int64_t)v * v);
    if (go.meas) go.meas[(size_t)r * Ln + e] = (uint64_t)(int64_t)v;
  }
  fb.norm[r] = N;
  // helper measurement share hm = XOF(k_hm, dst(1), [1]) and the leader's lm = meas - hm,
  // written encoded into the leader input share; the leader output share (the decoded entries
  // of lm) on the way
  uint8_t* lin = fb.lin + (size_t)r * p.leader_share_len;
  {
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[1]);
    msg_bytes16(m, 9, k_hm);
    msg_byte(m, 25, 1);
    msg_absorb_final(s, m, 26);
    const uint32_t K = (M * 16 + 167) / 168;
    uint32_t q0 = 0, q1 = 0;
    T acc = F::zero(), pw = F::one();
    for (uint32_t b = 0; b < K; b++) {
      squeeze_block_with<F>(s, b, M, q0, q1, [&](uint32_t i, const uint32_t* w) {
        const T h = F::from_words(w);
        if (!F::lt_p(h)) flag = 1;
        const T l = F::sub(F::from_u32(fg_mbit(p, X, N, i)), h);
        F::store(lin, i, l);
        if (i < nb * Ln) {
          const uint32_t bt = i % nb;
          if (bt == 0) {
            acc = F::zero();
            pw = F::one();
          }
          acc = F::add(acc, F::mul(l, pw));
          pw = F::add(pw, pw);
          if (bt == nb - 1 && go.leader_out) F::store(go.leader_out + (size_t)r * Ln * 16, i / nb, acc);
        }
      });
      if (b + 1 < K) keccak_p12(s);
    }
  }
  // joint-rand parts: the helper's over enc(hm) (the hm stream squeezed again word by word),
  // the leader's over enc(lm) (read back from the leader share)
  uint32_t part0[4], part1[4], jseed[4];
  {
    GenStream hs;
    kzero(hs.st);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[1]);
    msg_bytes16(m, 9, k_hm);
    msg_byte(m, 25, 1);
    msg_absorb_final(hs.st, m, 26);
    const uint32_t nw = M * 4;
    jr_part_words(p, k_hb, 1, nonce, M * 16, [&](uint32_t u) -> uint32_t {
      return u < nw ? hs.word(u) : 0u;
    }, part1);
    const uint32_t* lw = (const uint32_t*)lin;
    jr_part_words(p, k_lb, 0, nonce, M * 16, [&](uint32_t u) -> uint32_t {
      return u < nw ? lw[u] : 0u;
    }, part0);
  }
  const uint32_t zero[4] = {0, 0, 0, 0};
  seed_of<F>(p, 6, zero, part0, part1, jseed);
  const uint8_t b1[1] = {1};
  expand_to<F>(p, p.dst[3], jseed, b1, 1, p.jr_len, fb.jr, r, flag);
  expand_to<F>(p, p.dst[4], k_pr, b1, 1, p.arity + p.chunk1, fb.pr, r, flag);
  // public outputs; the leader share's blind goes after its proofs share (k_fg_finish)
  *(uint4*)(go.nonces + 16 * (size_t)r) = make_uint4(nonce[0], nonce[1], nonce[2], nonce[3]);
  uint8_t* hsh = go.helper + (size_t)r * p.helper_share_len;
  *(uint4*)hsh = make_uint4(k_hm[0], k_hm[1], k_hm[2], k_hm[3]);
  *(uint4*)(hsh + 16) = make_uint4(k_hp[0], k_hp[1], k_hp[2], k_hp[3]);
  *(uint4*)(hsh + 32) = make_uint4(k_hb[0], k_hb[1], k_hb[2], k_hb[3]);
  uint8_t* pb = go.pub + (size_t)r * p.public_share_len;
  *(uint4*)pb = make_uint4(part0[0], part0[1], part0[2], part0[3]);
  *(uint4*)(pb + 16) = make_uint4(part1[0], part1[1], part1[2], part1[3]);
  *(uint4*)(lin + (size_t)(M + p.proof_len) * 16) = make_uint4(k_lb[0], k_lb[1], k_lb[2], k_lb[3]);
  if (go.flags) go.flags[r] = (uint8_t)flag;
}

// In-place transforms of the two LDS vectors V0, V1 of P elements by the 256 threads.
// DIF with omega^-1: natural order in, P x the inverse DFT out in bit-reversed order.
DEV void fg_dif_inv(f128* V0, f128* V1, uint32_t P, const f128* w, uint32_t t) {
  typedef Fp128 F;
  for (uint32_t len = P >> 1; len >= 1; len >>= 1) {
    for (uint32_t bf = t; bf < (P >> 1); bf += 256) {
      const uint32_t j = bf % len, i0 = (bf / len) * 2 * len + j, i1 = i0 + len;
      const uint32_t e = j * (P / (2 * len));
      const f128 tw = w[e ? P - e : 0];
      f128 u = V0[i0], v = V0[i1];
      V0[i0] = F::add(u, v);
      V0[i1] = F::mul(F::sub(u, v), tw);
      u = V1[i0];
      v = V1[i1];
      V1[i0] = F::add(u, v);
      V1[i1] = F::mul(F::sub(u, v), tw);
    }
    __syncthreads();
  }
}
// DIT with omega: bit-reversed order in, the DFT out in natural order
DEV void fg_dit_fwd(f128* V0, f128* V1, uint32_t P, const f128* w, uint32_t t) {
  typedef Fp128 F;
  for (uint32_t len = 1; len < P; len <<= 1) {
    for (uint32_t bf = t; bf < (P >> 1); bf += 256) {
      const uint32_t j = bf % len, i0 = (bf / len) * 2 * len + j, i1 = i0 + len;
      const f128 tw = w[j * (P / (2 * len))];
      f128 u = V0[i0], v = F::mul(V0[i1], tw);
      V0[i0] = F::add(u, v);
      V0[i1] = F::sub(u, v);
      u = V1[i0];
      v = F::mul(V1[i1], tw);
      V1[i0] = F::add(u, v);
      V1[i1] = F::sub(u, v);
    }
    __syncthreads();
  }
}

// One gadget's polynomial, FlpGeneric::prove (VDAF-08 7.3.3.1) on P-point wire polynomials:
// G(psi^(2k)) = the gadget of the wire values at omega^k (computed directly), G(psi^(2k+1)) =
// the gadget of the wires' coset evaluations DFT(psi^m c_m) with c = IDFT(wire values); then the
// 2P - 1 coefficients g_m = (e_m + psi^-m o_m) / 2, g_(m+P) = (e_m - psi^-m o_m) / 2 from
// e = IDFT(even values), o = IDFT(odd values).  val(j, k, a, b) fills wire pair j at point k
// (gadget 1 takes its wires two at a time, j and j + 1); gad(acc, a, b) adds the gadget term of
// one point.  PPT = points per thread (P <= 256 PPT).
template <int PPT, class Val, class Gad>
DEV void fg_gadget(uint32_t P, uint32_t logP, uint32_t npairs, const FgGadget& G, f128* V0,
                   f128* V1, uint32_t t, Val&& val, Gad&& gad, f128* coef_out, uint32_t glen) {
  typedef Fp128 F;
  mac128 PE[PPT], PO[PPT];
#pragma unroll
  for (int q = 0; q < PPT; q++) {
    mac_zero(PE[q]);
    mac_zero(PO[q]);
  }
  for (uint32_t j = 0; j < npairs; j++) {
#pragma unroll
    for (int q = 0; q < PPT; q++) {
      const uint32_t k = t + 256 * q;
      if (k < P) {
        f128 a, b;
        val(j, k, q, a, b);
        V0[k] = a;
        V1[k] = b;
        gad(PE[q], a, b);
      }
    }
    __syncthreads();
    fg_dif_inv(V0, V1, P, G.w, t);
    for (uint32_t s = t; s < P; s += 256) {  // coset twist psi^m / P of coefficient m
      const f128 tw = G.tw[bitrev(s, logP)];
      V0[s] = F::mul(V0[s], tw);
      V1[s] = F::mul(V1[s], tw);
    }
    __syncthreads();
    fg_dit_fwd(V0, V1, P, G.w, t);
#pragma unroll
    for (int q = 0; q < PPT; q++) {
      const uint32_t k = t + 256 * q;
      if (k < P) gad(PO[q], V0[k], V1[k]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < PPT; q++) {
    const uint32_t k = t + 256 * q;
    if (k < P) {
      V0[k] = mac_reduce_f(PE[q]);
      V1[k] = mac_reduce_f(PO[q]);
    }
  }
  __syncthreads();
  fg_dif_inv(V0, V1, P, G.w, t);
  for (uint32_t m = t; m < P; m += 256) {
    const f128 e = V0[bitrev(m, logP)], o = F::mul(V1[bitrev(m, logP)], G.ipsi[m]);
    coef_out[m] = F::mul(F::add(e, o), G.c2P);
    if (m + P < glen) coef_out[m + P] = F::mul(F::sub(e, o), G.c2P);
  }
  __syncthreads();
}

template <int PPT>
__global__ __launch_bounds__(256) void k_fg_prove(DevParams p, FgBufs fb, FgGadget G0,
                                                  FgGadget G1, f128 twon) {
  typedef Fp128 F;
  typedef f128 T;
  extern __shared__ f128 lds[];
  const uint32_t r = blockIdx.x, t = threadIdx.x;
  const uint32_t Pm = p.P > p.P1 ? p.P : p.P1;
  f128* V0 = lds;
  f128* V1 = lds + Pm;
  const size_t ld = p.ld;
  const uint32_t M = p.meas_len, Ln = p.length, nb = p.bits;
  const uint32_t C0 = p.chunk, K0 = p.calls, A0 = p.arity, C1 = p.chunk1, K1 = p.calls1;
  const int16_t* X = fb.X + (size_t)r * Ln;
  const uint64_t N = fb.norm[r];
  f128* proof = (f128*)(fb.proof + (size_t)r * p.proof_len * 16);
  auto prv = [&](uint32_t w) { return F::load(fb.pr, (size_t)w * ld + r); };
  const T r0 = F::load(fb.jr, r);
  const T neg1 = F::sub(F::zero(), F::one());
  // gadget 0: ParallelSum(Mul, C0) over the range-check wires; rp[q] = r0^(c C0 + j + 1) for
  // call c = k - 1 of this thread's point k (valid(): the power advances per element)
  T rp[PPT];
  {
    T rc = F::one(), sq = r0;
    for (uint32_t e = C0; e; e >>= 1) {
      if (e & 1) rc = F::mul(rc, sq);
      if (e > 1) sq = F::mul(sq, sq);
    }
#pragma unroll
    for (int q = 0; q < PPT; q++) {
      const uint32_t k = t + 256 * q;
      T x = r0, b = rc;
      for (uint32_t e = k ? k - 1 : 0; e; e >>= 1) {
        if (e & 1) x = F::mul(x, b);
        if (e > 1) b = F::mul(b, b);
      }
      rp[q] = x;
    }
  }
  for (uint32_t w = t; w < A0; w += 256) proof[w] = prv(w);
  fg_gadget<PPT>(
      p.P, p.logP, C0, G0, V0, V1, t,
      [&](uint32_t j, uint32_t k, int q, T& a, T& b) {
        if (k == 0) {
          a = prv(2 * j);
          b = prv(2 * j + 1);
        } else if (k <= K0) {
          const uint32_t i = (k - 1) * C0 + j;
          const uint32_t mi = i < M ? fg_mbit(p, X, N, i) : 0u;
          a = mi ? rp[q] : F::zero();
          b = mi ? F::zero() : neg1;
          rp[q] = F::mul(rp[q], r0);
        } else {
          a = F::zero();
          b = F::zero();
        }
      },
      [&](mac128& acc, const T& a, const T& b) { mac_add(acc, a, b); }, proof + A0, p.glen);
  // gadget 1: ParallelSum(PolyEval(y^2 - 2^n y), C1) over the decoded entries, two wires
  // (j, j + 1) per pass; a missing wire is zero and adds q(0) = 0
  const uint32_t o1 = A0 + p.glen;
  for (uint32_t w = t; w < C1; w += 256) proof[o1 + w] = prv(A0 + w);
  const uint32_t half = 1u << (nb - 1);
  auto wire1 = [&](uint32_t j, uint32_t k) -> T {
    if (j >= C1) return F::zero();
    if (k == 0) return prv(A0 + j);
    if (k > K1) return F::zero();
    const uint32_t idx = (k - 1) * C1 + j;
    return idx < Ln ? F::from_u32((uint32_t)(int32_t)X[idx] + half) : F::zero();
  };
  fg_gadget<PPT>(
      p.P1, p.logP1, (C1 + 1) / 2, G1, V0, V1, t,
      [&](uint32_t j, uint32_t k, int, T& a, T& b) {
        a = wire1(2 * j, k);
        b = wire1(2 * j + 1, k);
      },
      [&](mac128& acc, const T& a, const T& b) {
        mac_add(acc, a, F::sub(a, twon));
        mac_add(acc, b, F::sub(b, twon));
      },
      proof + o1 + C1, p.glen1);
}

// the leader's proofs share = proof - XOF(k_hp, dst(2), [1, 1]), after lm in the leader share
__global__ __launch_bounds__(64) void k_fg_finish(DevParams p, GenOut go, FgBufs fb) {
  typedef Fp128 F;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  uint32_t flag = go.flags ? go.flags[r] : 0u;
  uint32_t k_hp[4];
  load16(go.helper + (size_t)r * p.helper_share_len + 16, k_hp);
  const uint8_t* prf = fb.proof + (size_t)r * p.proof_len * 16;
  uint8_t* lp = fb.lin + (size_t)r * p.leader_share_len + (size_t)p.meas_len * 16;
  KState s;
  kzero(s);
  Msg m;
  msg_zero(m);
  msg_dst(m, p.dst[2]);
  msg_bytes16(m, 9, k_hp);
  msg_byte(m, 25, 1);
  msg_byte(m, 26, 1);
  msg_absorb_final(s, m, 27);
  const uint32_t PL = p.proof_len, K = (PL * 16 + 167) / 168;
  uint32_t q0 = 0, q1 = 0;
  for (uint32_t b = 0; b < K; b++) {
    squeeze_block_with<F>(s, b, PL, q0, q1, [&](uint32_t i, const uint32_t* w) {
      const f128 h = F::from_words(w);
      if (!F::lt_p(h)) flag = 1;
      F::store(lp, i, F::sub(F::load(prf, i), h));
    });
    if (b + 1 < K) keccak_p12(s);
  }
  if (go.flags) go.flags[r] = (uint8_t)flag;
}

// ====================================================================================
// Prio3SumVecField64MultiproofHmacSha256Aes128 client: the same seeded
// stream, 32-byte seeds (nonce at bytes 0..15, then helper measurement, helper proofs, helper
// blind, leader blind and prove-rand seeds, 32 bytes each, entries 8 bytes each from byte 176,
// masked to `bits`), the shares and num_proofs proofs of the SumVec circuit over Field64 with
// XofHmacSha256Aes128 (prio3_mp64_xof.h), one report per lane; then the engine's device leader
// prepare_init on the leader input shares.  oracle/prio3_py.py is the same in Python
// (tests/test_mp64_client.py).
// ====================================================================================
// joint_rand_part = XOF(k_blind, dst(7), [agg_id] || nonce || enc(share)) -> 32 bytes
DEV void mp_jr_part(const AesT& A, const Mp64Params& P, const uint32_t kblind[8], uint32_t agg_id,
                    const uint32_t nonce[4], const uint64_t* share, size_t ld, uint32_t r,
                    uint32_t part[8]) {
  HmacKey k;
  hmac_key_ni(kblind, k.ist, k.ost);
  Msg32<8> pm;
  mz(pm);
  msg_dst(pm, P, 7);
  mbyte(pm, 9, agg_id);
  mwords_le(pm, 10, nonce, 4);
  const uint32_t M = P.meas_len, L = 26 + 8 * M, nblk = (L + 9 + 63) / 64;
  uint32_t st[8];
  for (int i = 0; i < 8; i++) st[i] = k.ist[i];
  for (uint32_t b = 0; b < nblk; b++) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = jr_word(16 * b + i, pm.w, share, ld, r, M, L, 16 * nblk);
    compress_ni(st, w);
  }
  uint32_t o[16] = {st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], 0x80000000u,
                    0, 0, 0, 0, 0, 0, (64 + 32) * 8};
  uint32_t tag[8];
  for (int i = 0; i < 8; i++) tag[i] = k.ost[i];
  compress_ni(tag, o);
  Stream s;
  stream_init(A, s, tag);
  derive32(A, s, part);
}

// XOF(seed, dst(usage), binder) -> n elements into SoA rows of base (rejection sampling)
DEV void mp_expand(const AesT& A, const Mp64Params& P, const uint32_t seed[8], int usage,
                   const uint8_t* binder, int blen, uint64_t* base, size_t ld, uint32_t r,
                   uint32_t n) {
  Msg32<16> m;
  mz(m);
  msg_dst(m, P, usage);
  for (int i = 0; i < blen; i++) mbyte(m, 9 + i, binder[i]);
  uint32_t tag[8];
  xof_tag(seed, m, 9 + blen, tag);
  Stream s;
  stream_init(A, s, tag);
  (void)expand_soa(A, s, base, ld, r, n);
}

__global__ __launch_bounds__(64) void k_gen_mp64(DevParams p, Mp64Params P, uint64_t seed,
                                                 uint64_t first, GenScratch gs, GenOut go,
                                                 uint8_t* lin, uint64_t invP, uint64_t inv2P) {
  __shared__ AesT A;
  aes_tables_init(A);
  __syncthreads();
  typedef Fp64 F;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  const size_t ld = p.ld;
  // DevParams::proof_len counts every proof here; Mp64Params::proof_len is one proof's
  const uint32_t M = p.meas_len, np = P.np, Ar = p.arity, PL = P.proof_len, Ln = p.length;
  GenStream gst;
  gen_stream_init(gst.st, seed, first + r);
  uint32_t nonce[4], k_hm[8], k_hp[8], k_hb[8], k_lb[8], k_pr[8];
  // stream words in increasing order (GenStream moves forward only; words 42, 43 of the last
  // seed are in the second block)
  for (int k = 0; k < 4; k++) nonce[k] = gst.word(k);
  for (int k = 0; k < 8; k++) k_hm[k] = gst.word(4 + k);
  for (int k = 0; k < 8; k++) k_hp[k] = gst.word(12 + k);
  for (int k = 0; k < 8; k++) k_hb[k] = gst.word(20 + k);
  for (int k = 0; k < 8; k++) k_lb[k] = gst.word(28 + k);
  for (int k = 0; k < 8; k++) k_pr[k] = gst.word(36 + k);
  uint64_t* meas = (uint64_t*)gs.meas;
  const uint64_t mask = p.bits < 64 ? (1ull << p.bits) - 1 : ~0ull;
  for (uint32_t e = 0; e < Ln; e++) {
    uint64_t v = (uint64_t)gst.word(44 + 2 * e);
    v |= (uint64_t)gst.word(45 + 2 * e) << 32;
    v &= mask;
    if (go.meas) go.meas[(size_t)r * Ln + e] = v;
    for (uint32_t b = 0; b < p.bits; b++) meas[(size_t)(e * p.bits + b) * ld + r] = (v >> b) & 1;
  }
  // shares and joint-rand parts
  uint64_t* hm = (uint64_t*)gs.hm;
  uint64_t* lm = (uint64_t*)gs.lm;
  const uint8_t b1[1] = {1};
  mp_expand(A, P, k_hm, 1, b1, 1, hm, ld, r, M);
  for (uint32_t i = 0; i < M; i++)
    lm[(size_t)i * ld + r] = F::sub(meas[(size_t)i * ld + r], hm[(size_t)i * ld + r]);
  uint32_t part0[8], part1[8], jseed[8];
  mp_jr_part(A, P, k_hb, 1, nonce, hm, ld, r, part1);
  mp_jr_part(A, P, k_lb, 0, nonce, lm, ld, r, part0);
  {
    Msg32<32> m;
    mz(m);
    msg_dst(m, P, 6);
    mwords_le(m, 9, part0, 8);
    mwords_le(m, 41, part1, 8);
    uint32_t tag[8];
    hmac_ni(P.z_ist, P.z_ost, m.w, 73, tag);
    Stream s;
    stream_init(A, s, tag);
    derive32(A, s, jseed);
  }
  const uint8_t bnp[2] = {(uint8_t)np, 1};
  mp_expand(A, P, jseed, 3, bnp, 1, (uint64_t*)gs.jr, ld, r, np);           // one per proof
  mp_expand(A, P, k_pr, 4, bnp, 1, (uint64_t*)gs.prand, ld, r, Ar * np);
  // the num_proofs proofs (proof k: prove rand rows k A .., joint rand row k)
  for (uint32_t k = 0; k < np; k++)
    prove_lane<F>(p, gs, gs.meas, (const uint64_t*)gs.prand + (size_t)k * Ar * ld,
                  (const uint64_t*)gs.jr + (size_t)k * ld, (uint64_t*)gs.proof + (size_t)k * PL * ld,
                  r, invP, inv2P);
  // leader input share = enc(lm) || enc(proofs - helper proofs share) || k_blind
  uint64_t* hp = (uint64_t*)gs.hp;
  mp_expand(A, P, k_hp, 2, bnp, 2, hp, ld, r, PL * np);
  uint64_t* li = (uint64_t*)(lin + (size_t)r * p.leader_share_len);
  for (uint32_t i = 0; i < M; i++) li[i] = lm[(size_t)i * ld + r];
  const uint64_t* prf = (const uint64_t*)gs.proof;
  for (uint32_t i = 0; i < PL * np; i++)
    li[M + i] = F::sub(prf[(size_t)i * ld + r], hp[(size_t)i * ld + r]);
  uint32_t* lt = (uint32_t*)(li + M + PL * np);
  for (int k = 0; k < 8; k++) lt[k] = k_lb[k];
  // public outputs
  *(uint4*)(go.nonces + 16 * (size_t)r) = make_uint4(nonce[0], nonce[1], nonce[2], nonce[3]);
  uint32_t* hs = (uint32_t*)(go.helper + (size_t)r * p.helper_share_len);
  uint32_t* pb = (uint32_t*)(go.pub + (size_t)r * p.public_share_len);
  for (int k = 0; k < 8; k++) {
    hs[k] = k_hm[k];
    hs[8 + k] = k_hp[k];
    hs[16 + k] = k_hb[k];
    pb[k] = part0[k];
    pb[8 + k] = part1[k];
  }
  if (go.leader_out) {  // truncate(lm): entry e = sum_b 2^b lm[e bits + b]
    uint64_t* lo = (uint64_t*)(go.leader_out + (size_t)r * p.out_len * 8);
    for (uint32_t e = 0; e < p.out_len; e++) {
      uint64_t acc = 0, pw = 1;
      for (uint32_t b = 0; b < p.bits; b++) {
        acc = F::add(acc, F::mul(pw, lm[(size_t)(e * p.bits + b) * ld + r]));
        pw = F::add(pw, pw);
      }
      lo[e] = acc;
    }
  }
  if (go.flags) go.flags[r] = 0;
}

// ====================================================================================
// Host ABI
// ====================================================================================
#define GCHK(x)                                                                       \
  do {                                                                                \
    hipError_t _e = (x);                                                              \
    if (_e != hipSuccess) {                                                           \
      fprintf(stderr, "janus_prio3: HIP error %s at %s:%d\n", hipGetErrorString(_e),  \
              __FILE__, __LINE__);                                                    \
      rc = PRIO3_EDEVICE;                                                             \
      goto done;                                                                      \
    }                                                                                 \
  } while (0)


// ------------------------------------------------------------------------------------
// Leader-side preparation: prio Prio3::prepare_init with agg_id 0 on the
// explicit leader input share, as Janus's leader calls it through
// PingPongTopology::leader_initialized (aggregation_job_driver.rs:397-415), and prepare_next on
// the helper's prepare message (leader_continued, aggregation_job_driver.rs:677-691).
// One report per lane with the generic lane helpers (the leader's own input share is in
// HBM, so the share XOF of the helper path does not exist here).
// ------------------------------------------------------------------------------------
template <class F>
__global__ __launch_bounds__(64) void k_leader_init(DevParams p, const uint8_t* nonces,
                                                    const uint8_t* pub, const uint8_t* lshares,
                                                    Scratch sc, uint8_t* prep_shares,
                                                    uint8_t* status, InPtrs keys) {
  typedef typename F::T T;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  const size_t ld = p.ld;
  const uint32_t M = p.meas_len, PL = p.proof_len, A = p.arity;
  const bool JR = p.jr_len > 0;
  uint8_t st = PRIO3_STATUS_FINISHED;
  uint32_t flag = p.force_slow;
  // decode the explicit shares into SoA scratch (canonical elements only)
  const uint8_t* ls = lshares + (size_t)r * p.leader_share_len;
  bool ok = true;
  for (uint32_t e = 0; e < M; e++) {
    const T x = F::load(ls, e);
    ok = ok && F::lt_p(x);
    F::store(sc.meas, (size_t)e * ld + r, x);
  }
  for (uint32_t e = 0; e < PL; e++) {
    const T x = F::load(ls + (size_t)M * F::ES, e);
    ok = ok && F::lt_p(x);
    F::store(sc.proofs, (size_t)e * ld + r, x);
  }
  if (!ok) st = PRIO3_STATUS_INPUT_SHARE_DECODE;
  uint32_t nonce[4];
  load16(nonces + 16 * (size_t)r, nonce);
  // query randomness
  {
    const uint8_t b1[1] = {1};
    uint32_t vk[4];
    load_vk(p, keys, r, vk);  // coalesced groups of several tasks: the report's own key
    KState s;
    kzero(s);
    Msg m;
    msg_zero(m);
    msg_dst(m, p.dst[5]);
    msg_bytes16(m, 9, vk);
    msg_byte(m, 25, b1[0]);
    msg_bytes16(m, 26, nonce);
    msg_absorb_final(s, m, 42);
    uint32_t w[4] = {kword(s, 0), kword(s, 1), kword(s, 2), kword(s, 3)};
    put_elem<F>(p, sc.qr, 0, r, w, flag);
  }
  uint32_t part0[4] = {0, 0, 0, 0};
  if (JR) {
    uint32_t kb[4], part1[4], cor[4];
    load16(ls + (size_t)(M + PL) * F::ES, kb);
    jr_part_scratch<F>(p, kb, 0, nonce, sc.meas, r, part0);
    load16(pub + (size_t)r * p.public_share_len + 16, part1);
    const uint32_t zero[4] = {0, 0, 0, 0};
    seed_of<F>(p, 6, zero, part0, part1, cor);
    const uint8_t b1[1] = {1};
    expand_to<F>(p, p.dst[3], cor, b1, 1, p.jr_len, sc.jr, r, flag);
    sc.corrected[r] = make_uint4(cor[0], cor[1], cor[2], cor[3]);
  }
  if (flag) {  // a rejection-sampling event: redo the expansions with the byte-level sponge
    uint32_t vk[4];
    load_vk(p, keys, r, vk);
    uint8_t b[17];
    b[0] = 1;
    for (int i = 0; i < 16; i++) b[1 + i] = (uint8_t)(nonce[i >> 2] >> (8 * (i & 3)));
    bx_expand<F>(p.dst[5], vk, b, 17, 1, sc.qr, ld, r);
    if (JR) {
      const uint4 c = sc.corrected[r];
      const uint32_t cor[4] = {c.x, c.y, c.z, c.w};
      bx_expand<F>(p.dst[3], cor, b, 1, p.jr_len, sc.jr, ld, r);
    }
  }
  const T t = F::load(sc.qr, r);
  T v, pt;
  if (!flp_query_lane<F>(p, sc.meas, sc.proofs, sc.jr, t, sc.Lbuf, sc.PVbuf, sc.acc, r, v, pt) &&
      st == PRIO3_STATUS_FINISHED)
    st = PRIO3_STATUS_PREP_INIT;
  uint8_t* ps = prep_shares + (size_t)r * p.prep_share_len;
  F::store(ps, 0, v);
  for (uint32_t w = 0; w < A; w++) F::store(ps, 1 + w, F::load(sc.acc, (size_t)w * ld + r));
  F::store(ps, A + 1, pt);
  if (JR) *(uint4*)(ps + (size_t)p.verifier_len * F::ES) = make_uint4(part0[0], part0[1], part0[2], part0[3]);
  sc.flag[r] = (uint8_t)flag;
  status[r] = st;
}

// prepare_next: the helper's prepare message must equal the leader's corrected joint-rand
// seed (else VdafPrepareNext); the output share is truncate(meas share).
template <class F>
__global__ __launch_bounds__(256) void k_leader_next(DevParams p, const uint8_t* prep_msgs,
                                                     Scratch sc, uint8_t* status) {
  typedef typename F::T T;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  const size_t ld = p.ld;
  uint8_t st = status[r];
  if (st == PRIO3_STATUS_FINISHED && p.jr_len) {
    uint32_t m[4];
    load16(prep_msgs + 16 * (size_t)r, m);
    const uint4 c = sc.corrected[r];
    if (m[0] != c.x || m[1] != c.y || m[2] != c.z || m[3] != c.w) st = PRIO3_STATUS_PREP_NEXT;
  }
  status[r] = st;
  if (p.kind == PRIO3_SUM || p.kind == PRIO3_SUMVEC) {
    const uint32_t outs = p.kind == PRIO3_SUM ? 1 : p.out_len;
    for (uint32_t e = 0; e < outs; e++) {
      T acc = F::zero(), pw = F::one();
      for (uint32_t b = 0; b < p.bits; b++) {
        acc = F::add(acc, F::mul(pw, F::load(sc.meas, (size_t)(e * p.bits + b) * ld + r)));
        pw = F::add(pw, pw);
      }
      F::store(sc.out, (size_t)e * ld + r, acc);
    }
  }
}

// prepare_next of many jobs' leader batches (of different runs) in one launch: block row y is
// job y (its descriptor, prepare messages and statuses in the executor's mapped staging); the
// verdict goes back to the staging and to the run's device statuses (which prio3_accumulate
// reads).  Same per-report work as k_leader_next.
template <class F>
__global__ __launch_bounds__(256) void k_leader_next_multi(const LNextDesc* descs,
                                                           const uint8_t* msgs, uint8_t* status) {
  typedef typename F::T T;
  __shared__ LNextDesc D;
  if (threadIdx.x == 0) D = descs[blockIdx.y];
  __syncthreads();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= D.n) return;
  const size_t g = (size_t)D.rep_off + r, ld = D.ld;
  uint8_t st = status[g];
  if (st == PRIO3_STATUS_FINISHED && D.jr) {
    uint32_t m[4];
    load16(msgs + 16 * g, m);
    const uint4 c = D.corrected[r];
    if (m[0] != c.x || m[1] != c.y || m[2] != c.z || m[3] != c.w) st = PRIO3_STATUS_PREP_NEXT;
  }
  status[g] = st;
  D.dstatus[r] = st;
  if (D.kind == PRIO3_SUM || D.kind == PRIO3_SUMVEC) {
    const uint32_t outs = D.kind == PRIO3_SUM ? 1 : D.out_len;
    for (uint32_t e = 0; e < outs; e++) {
      T acc = F::zero(), pw = F::one();
      for (uint32_t b = 0; b < D.bits; b++) {
        acc = F::add(acc, F::mul(pw, F::load(D.meas, (size_t)(e * D.bits + b) * ld + r)));
        pw = F::add(pw, pw);
      }
      F::store(D.out, (size_t)e * ld + r, acc);
    }
  }
}

extern "C" int launch_leader_next_multi(uint32_t es, const LNextDesc* d_desc, const uint8_t* d_msgs,
                                        uint8_t* d_status, uint32_t n_jobs, uint32_t max_n,
                                        hipStream_t st) {
  const dim3 grid((max_n + 255) / 256, n_jobs);
  if (es == 16)
    k_leader_next_multi<Fp128><<<grid, 256, 0, st>>>(d_desc, d_msgs, d_status);
  else
    k_leader_next_multi<Fp64><<<grid, 256, 0, st>>>(d_desc, d_msgs, d_status);
  return hipGetLastError() == hipSuccess ? PRIO3_OK : PRIO3_EDEVICE;
}

// a leader prepare_init that did not finish marks the generated report unusable
__global__ void k_fg_status(const uint8_t* status, uint8_t* flags, uint32_t n) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n && status[r] != PRIO3_STATUS_FINISHED) flags[r] |= 2;
}

extern "C" int launch_leader_init(const DevParams& dp, const uint8_t* d_nonces, const uint8_t* d_pub,
                       const uint8_t* d_lshares, const Scratch& sc, uint8_t* d_prep_shares,
                       uint8_t* d_status, hipStream_t st, const uint16_t* vk_slot,
                       const uint4* vk_tab) {
  const uint32_t blocks = (dp.n + 63) / 64;
  InPtrs keys{};
  keys.vk_slot = vk_slot;
  keys.vk_tab = vk_tab;
  if (dp.es == 16)
    k_leader_init<Fp128><<<blocks, 64, 0, st>>>(dp, d_nonces, d_pub, d_lshares, sc,
                                                d_prep_shares, d_status, keys);
  else
    k_leader_init<Fp64><<<blocks, 64, 0, st>>>(dp, d_nonces, d_pub, d_lshares, sc,
                                               d_prep_shares, d_status, keys);
  return hipGetLastError() == hipSuccess ? PRIO3_OK : PRIO3_EDEVICE;
}

extern "C" int launch_leader_next(const DevParams& dp, const uint8_t* d_prep_msgs, const Scratch& sc,
                       uint8_t* d_status, hipStream_t st) {
  const uint32_t blocks = (dp.n + 255) / 256;
  if (dp.es == 16)
    k_leader_next<Fp128><<<blocks, 256, 0, st>>>(dp, d_prep_msgs, sc, d_status);
  else
    k_leader_next<Fp64><<<blocks, 256, 0, st>>>(dp, d_prep_msgs, sc, d_status);
  return hipGetLastError() == hipSuccess ? PRIO3_OK : PRIO3_EDEVICE;
}

static f128 h128x(u128 x) {
  f128 r;
  for (int k = 0; k < 4; k++) r.w[k] = (uint32_t)(x >> (32 * k));
  return r;
}
static f128 h128(const uint32_t* w) {
  f128 r;
  for (int k = 0; k < 4; k++) r.w[k] = w[k];
  return r;
}

// FPVec generator (k_fg_*): chunks of reports through the three kernels, then the engine's device
// leader prepare_init on the chunk's leader input shares (so e->mu is not held here: that entry
// point takes it).  Needs the engine's experimental_fpvec opt-in like every FPVec entry point.
static int gen_fpvec(prio3_engine* e, uint32_t n, uint64_t seed, uint64_t first_index,
                     uint8_t* d_nonces, uint8_t* d_pub, uint8_t* d_helper, uint8_t* d_lps,
                     uint64_t* d_meas, uint8_t* d_lout, uint8_t* d_flags, uint8_t* d_lin,
                     hipStream_t st) {
  DevParams p = e->dp;
  if (!d_pub) return PRIO3_EINVAL;
  const uint32_t Pm = std::max(p.P, p.P1);
  if (Pm > 1024 || p.logP + 1 > MAX_ROOTS || p.logP1 + 1 > MAX_ROOTS) return PRIO3_EUNSUPPORTED;
  DeviceGuard dg_(e->device);
  if (dg_.rc != hipSuccess) return PRIO3_EDEVICE;
  // entries are signed bytes >> gsh, |X| <= 2^(7 - gsh): the claimed norm must stay below
  // 2^(2 bits - 2) (FixedPointBoundedL2VecSum's bound, ||x|| < 1)
  uint32_t gsh = 0;
  while (gsh < 7 && std::ldexp((double)p.length, 14 - 2 * (int)gsh) >= std::ldexp(1.0, 2 * (int)p.bits - 2))
    gsh++;
  // NTT tables of both gadgets (one device buffer)
  auto word4 = [](u128 x, uint32_t* w) {
    for (int k = 0; k < 4; k++) w[k] = (uint32_t)(x >> (32 * k));
  };
  auto rootof = [&](uint32_t l) {
    u128 x = 0;
    for (int k = 0; k < 4; k++) x |= (u128)p.roots128[l][k] << (32 * k);
    return x;
  };
  std::vector<uint32_t> tab;
  struct Off { size_t w, tw, ipsi; u128 c2P; } offs[2];
  for (int g = 0; g < 2; g++) {
    const uint32_t P = g ? p.P1 : p.P, lg = g ? p.logP1 : p.logP;
    const u128 om = rootof(lg), psi = rootof(lg + 1), ipsi = hpow(psi, HP128 - 2, HP128);
    const u128 iP = hpow(P, HP128 - 2, HP128);
    offs[g].c2P = hpow(2 * (u128)P, HP128 - 2, HP128);
    uint32_t w4[4];
    offs[g].w = tab.size() / 4;
    u128 x = 1;
    for (uint32_t i = 0; i < P; i++, x = hmul(x, om, HP128)) {
      word4(x, w4);
      tab.insert(tab.end(), w4, w4 + 4);
    }
    offs[g].tw = tab.size() / 4;
    x = iP;
    for (uint32_t i = 0; i < P; i++, x = hmul(x, psi, HP128)) {
      word4(x, w4);
      tab.insert(tab.end(), w4, w4 + 4);
    }
    offs[g].ipsi = tab.size() / 4;
    x = 1;
    for (uint32_t i = 0; i < P; i++, x = hmul(x, ipsi, HP128)) {
      word4(x, w4);
      tab.insert(tab.end(), w4, w4 + 4);
    }
  }
  // chunk: at most 40 % of free HBM for the per-report buffers (the leader prepare's own
  // sub-batched scratch takes what is left)
  const size_t A = p.arity + p.chunk1;
  const size_t per = 2 * (size_t)p.length + 8 + p.leader_share_len + 16 * (size_t)p.jr_len +
                     16 * A + 16 * (size_t)p.proof_len + 1 + 64;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return PRIO3_EDEVICE;
  size_t chunk = std::min<size_t>({(size_t)n, (size_t)16384, std::max<size_t>(64, (size_t)(0.4 * (double)fr) / per)});
  chunk = (chunk + 63) & ~(size_t)63;
  std::vector<void*> bufs;
  int rc = PRIO3_OK;
  auto alloc = [&](size_t bytes) -> void* {
    void* b = nullptr;
    if (hipMalloc(&b, std::max<size_t>(bytes, 256)) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    bufs.push_back(b);
    return b;
  };
  FgBufs fb;
  fb.gsh = gsh;
  fb.X = (int16_t*)alloc(2 * (size_t)p.length * chunk);
  fb.norm = (uint64_t*)alloc(8 * chunk);
  fb.lin = (uint8_t*)alloc((size_t)p.leader_share_len * chunk);
  fb.jr = alloc(16 * (size_t)p.jr_len * chunk);
  fb.pr = alloc(16 * A * chunk);
  fb.proof = (uint8_t*)alloc(16 * (size_t)p.proof_len * chunk);
  uint8_t* stat = (uint8_t*)alloc(chunk);
  f128* dtab = (f128*)alloc(4 * tab.size());
  if (!fb.X || !fb.norm || !fb.lin || !fb.jr || !fb.pr || !fb.proof || !stat || !dtab) {
    rc = PRIO3_EDEVICE;  // out of device memory
  } else if (hipMemcpyAsync(dtab, tab.data(), 4 * tab.size(), hipMemcpyHostToDevice, st) !=
             hipSuccess) {
    rc = PRIO3_EDEVICE;
  }
  FgGadget G[2];
  for (int g = 0; g < 2 && rc == PRIO3_OK; g++) {
    G[g].w = dtab + offs[g].w;
    G[g].tw = dtab + offs[g].tw;
    G[g].ipsi = dtab + offs[g].ipsi;
    G[g].c2P = h128x(offs[g].c2P);
  }
  const f128 twon = h128x((u128)1 << p.bits);
  const uint32_t ppt = (Pm + 255) / 256;
  const size_t lds = 2 * (size_t)Pm * 16;
  for (uint64_t off = 0; off < n && rc == PRIO3_OK; off += chunk) {
    const uint32_t m = (uint32_t)std::min<uint64_t>(chunk, n - off);
    DevParams q = p;
    q.n = m;
    q.ld = (uint32_t)chunk;
    GenOut go{};
    go.nonces = d_nonces + 16 * off;
    go.pub = d_pub + (size_t)p.public_share_len * off;
    go.helper = d_helper + (size_t)p.helper_share_len * off;
    go.leader_out = d_lout ? d_lout + (size_t)p.out_len * 16 * off : nullptr;
    go.meas = d_meas ? d_meas + (size_t)p.length * off : nullptr;
    go.flags = d_flags ? d_flags + off : nullptr;
    k_fg_shares<<<(m + 63) / 64, 64, 0, st>>>(q, seed, first_index + off, go, fb);
    if (ppt == 1)
      k_fg_prove<1><<<m, 256, lds, st>>>(q, fb, G[0], G[1], twon);
    else if (ppt == 2)
      k_fg_prove<2><<<m, 256, lds, st>>>(q, fb, G[0], G[1], twon);
    else
      k_fg_prove<4><<<m, 256, lds, st>>>(q, fb, G[0], G[1], twon);
    k_fg_finish<<<(m + 63) / 64, 64, 0, st>>>(q, go, fb);
    if (hipGetLastError() != hipSuccess) {
      rc = PRIO3_EDEVICE;
      break;
    }
    rc = prio3_device_leader_prepare_init(e, m, go.nonces, go.pub, fb.lin,
                                          d_lps + (size_t)p.prep_share_len * off, stat, st);
    if (rc != PRIO3_OK) break;
    if (d_flags) k_fg_status<<<(m + 255) / 256, 256, 0, st>>>(stat, d_flags + off, m);
    if (d_lin && hipMemcpyAsync(d_lin + (size_t)p.leader_share_len * off, fb.lin,
                                (size_t)p.leader_share_len * m, hipMemcpyDeviceToDevice,
                                st) != hipSuccess)
      rc = PRIO3_EDEVICE;
  }
  if (hipStreamSynchronize(st) != hipSuccess && rc == PRIO3_OK) rc = PRIO3_EDEVICE;
  for (auto b : bufs) (void)hipFree(b);
  return rc;
}

// multiproof generator: chunks through k_gen_mp64, then the device leader prepare_init
static int gen_mp64(prio3_engine* e, uint32_t n, uint64_t seed, uint64_t first_index,
                    uint8_t* d_nonces, uint8_t* d_pub, uint8_t* d_helper, uint8_t* d_lps,
                    uint64_t* d_meas, uint8_t* d_lout, uint8_t* d_flags, uint8_t* d_lin,
                    hipStream_t st) {
  DevParams p = e->dp;
  const Mp64Params& P = e->mp;
  if (!d_pub) return PRIO3_EINVAL;
  DeviceGuard dg_(e->device);
  if (dg_.rc != hipSuccess) return PRIO3_EDEVICE;
  const uint32_t A = p.arity, np = P.np, PP = p.P;
  const size_t chunk = std::min<size_t>(((size_t)n + 63) & ~(size_t)63, 65536);
  std::vector<void*> bufs;
  int rc = PRIO3_OK;
  auto alloc = [&](size_t bytes) -> void* {
    void* b = nullptr;
    if (hipMalloc(&b, std::max<size_t>(bytes, 256)) != hipSuccess) {
      (void)hipGetLastError();
      rc = PRIO3_EDEVICE;
      return nullptr;
    }
    bufs.push_back(b);
    return b;
  };
  GenScratch gs{};
  const size_t es = 8;
  gs.meas = alloc(es * p.meas_len * chunk);
  gs.hm = alloc(es * p.meas_len * chunk);
  gs.lm = alloc(es * p.meas_len * chunk);
  gs.wires = alloc(es * A * PP * chunk);
  gs.evals = alloc(es * A * 2 * PP * chunk);
  gs.g = alloc(es * 2 * PP * chunk);
  gs.tmp = alloc(es * 2 * PP * chunk);
  gs.proof = alloc(es * (size_t)P.proof_len * np * chunk);
  gs.hp = alloc(es * (size_t)P.proof_len * np * chunk);
  gs.prand = alloc(es * A * np * chunk);
  gs.jr = alloc(es * np * chunk);
  uint8_t* lin = (uint8_t*)alloc((size_t)p.leader_share_len * chunk);
  uint8_t* stat = (uint8_t*)alloc(chunk);
  const uint64_t invP = (uint64_t)hpow(PP, HP64 - 2, HP64), inv2P = (uint64_t)hpow(2 * PP, HP64 - 2, HP64);
  for (uint64_t off = 0; off < n && rc == PRIO3_OK; off += chunk) {
    const uint32_t m = (uint32_t)std::min<uint64_t>(chunk, n - off);
    DevParams q = p;
    q.n = m;
    q.ld = (uint32_t)chunk;
    GenOut go{};
    go.nonces = d_nonces + 16 * off;
    go.pub = d_pub + (size_t)p.public_share_len * off;
    go.helper = d_helper + (size_t)p.helper_share_len * off;
    go.leader_out = d_lout ? d_lout + (size_t)p.out_len * 8 * off : nullptr;
    go.meas = d_meas ? d_meas + (size_t)p.length * off : nullptr;
    go.flags = d_flags ? d_flags + off : nullptr;
    k_gen_mp64<<<(m + 63) / 64, 64, 0, st>>>(q, P, seed, first_index + off, gs, go, lin, invP,
                                              inv2P);
    if (hipGetLastError() != hipSuccess) {
      rc = PRIO3_EDEVICE;
      break;
    }
    rc = prio3_device_leader_prepare_init(e, m, go.nonces, go.pub, lin,
                                          d_lps + (size_t)p.prep_share_len * off, stat, st);
    if (rc != PRIO3_OK) break;
    if (d_flags) k_fg_status<<<(m + 255) / 256, 256, 0, st>>>(stat, d_flags + off, m);
    if (d_lin && hipMemcpyAsync(d_lin + (size_t)p.leader_share_len * off, lin,
                                (size_t)p.leader_share_len * m, hipMemcpyDeviceToDevice,
                                st) != hipSuccess)
      rc = PRIO3_EDEVICE;
  }
  if (hipStreamSynchronize(st) != hipSuccess && rc == PRIO3_OK) rc = PRIO3_EDEVICE;
  for (auto b : bufs) (void)hipFree(b);
  return rc;
}

extern "C" int prio3_client_generate_device(prio3_engine* e, uint32_t n, uint64_t seed,
                                            uint64_t first_index, uint8_t* d_nonces,
                                            uint8_t* d_public_shares, uint8_t* d_helper_shares,
                                            uint8_t* d_leader_prep_shares,
                                            uint64_t* d_measurements,
                                            uint8_t* d_leader_out_shares, uint8_t* d_flags,
                                            uint8_t* d_leader_input_shares, void* stream) {
  if (!e || !d_nonces || !d_helper_shares || !d_leader_prep_shares) return PRIO3_EINVAL;
  if (n == 0) return PRIO3_OK;
  if (e->dp.kind == PRIO3_SUMVEC_F64_MP)
    return gen_mp64(e, n, seed, first_index, d_nonces, d_public_shares, d_helper_shares,
                    d_leader_prep_shares, d_measurements, d_leader_out_shares, d_flags,
                    d_leader_input_shares, (hipStream_t)stream);
  if (e->dp.kind == PRIO3_FPVEC_BOUNDED_L2)
    return gen_fpvec(e, n, seed, first_index, d_nonces, d_public_shares, d_helper_shares,
                     d_leader_prep_shares, d_measurements, d_leader_out_shares, d_flags,
                     d_leader_input_shares, (hipStream_t)stream);
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg_(e->device);
  if (dg_.rc != hipSuccess) return PRIO3_EDEVICE;
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  DevParams p = e->dp;
  const size_t es = p.es;
  const uint32_t A = p.arity, P = p.P;
  // per-report scratch elements
  const size_t per = 3 * (size_t)p.meas_len + (size_t)A * P + (size_t)A * 2 * P + 4 * (size_t)P +
                     2 * (size_t)p.proof_len + A + p.jr_len + 1 + 2 * P + A;
  size_t chunk = ((size_t)2 << 30) / (per * es);  // <= 2 GiB of scratch
  if (chunk > 65536) chunk = 65536;
  chunk = chunk < 64 ? 64 : (chunk & ~(size_t)63);
  std::vector<void*> bufs;
  int rc = PRIO3_OK;
  GenScratch gs;
  void** slots[] = {&gs.meas, &gs.hm, &gs.lm, &gs.wires, &gs.evals, &gs.g, &gs.tmp, &gs.proof,
                    &gs.hp, &gs.prand, &gs.jr, &gs.qr, &gs.L, &gs.PV, &gs.acc};
  size_t counts[] = {p.meas_len, p.meas_len, p.meas_len, (size_t)A * P, (size_t)A * 2 * P,
                     2 * (size_t)P, 2 * (size_t)P, p.proof_len, p.proof_len, A,
                     p.jr_len ? p.jr_len : 1, 1, P, P, A};
  for (size_t i = 0; i < sizeof(counts) / sizeof(counts[0]); i++) {
    void* b = nullptr;
    GCHK(hipMalloc(&b, counts[i] * chunk * es));
    bufs.push_back(b);
    *slots[i] = b;
  }
  {
    u128 ip = hpow(p.P, HP128 - 2, HP128), i2 = hpow(2 * p.P, HP128 - 2, HP128);
    uint32_t w1[4], w2[4];
    for (int k = 0; k < 4; k++) {
      w1[k] = (uint32_t)(ip >> (32 * k));
      w2[k] = (uint32_t)(i2 >> (32 * k));
    }
    uint64_t ip64 = (uint64_t)hpow(p.P, HP64 - 2, HP64), i264 = (uint64_t)hpow(2 * p.P, HP64 - 2, HP64);
    const uint32_t mstride = p.kind == PRIO3_SUMVEC ? p.length : 1;
    for (uint64_t off = 0; off < n; off += chunk) {
      const uint32_t m = (uint32_t)std::min<uint64_t>(chunk, n - off);
      p.n = m;
      p.ld = (uint32_t)chunk;
      GenOut go;
      go.nonces = d_nonces + 16 * off;
      go.pub = d_public_shares ? d_public_shares + p.public_share_len * off : nullptr;
      go.helper = d_helper_shares + p.helper_share_len * off;
      go.leader_ps = d_leader_prep_shares + p.prep_share_len * off;
      go.leader_out = d_leader_out_shares ? d_leader_out_shares + (size_t)p.out_len * es * off : nullptr;
      go.meas = d_measurements ? d_measurements + (size_t)mstride * off : nullptr;
      go.flags = d_flags ? d_flags + off : nullptr;
      go.leader_in = d_leader_input_shares ? d_leader_input_shares + (size_t)p.leader_share_len * off
                                           : nullptr;
      if (es == 16)
        k_gen<Fp128><<<(m + 63) / 64, 64, 0, st>>>(p, seed, first_index + off, gs, go, h128(w1),
                                                   h128(w2));
      else
        k_gen<Fp64><<<(m + 63) / 64, 64, 0, st>>>(p, seed, first_index + off, gs, go, ip64, i264);
      GCHK(hipGetLastError());
    }
  }
  GCHK(hipStreamSynchronize(st));
done:
  for (auto b : bufs) (void)hipFree(b);
  return rc;
}
