// prio3_common.h -- kernel-side structures and per-lane building blocks shared by the
// helper engine (prio3_engine.hip) and the synthetic client (prio3_client.hip).
#pragma once
#include <atomic>
#include <mutex>
#include <string>
#include <vector>
#include "../../include/janus_prio3.h"
#include "prio3_device.h"

#define MAX_ROOTS 20

// Debug build (make -C janus_amd DEVICE_CHECKS=1 -> libjanus_prio3_dbg.so): device-side bounds
// assertions on the SoA scratch indexing (column < leading dimension, row < rows of the buffer)
// that print the failing condition and trap.  Compiled out of the product library.
#ifdef JANUS_DEVICE_CHECKS
#define DCHECK(c)                                                                        \
  do {                                                                                   \
    if (!(c)) {                                                                          \
      printf("janus device check failed: %s (%s:%d) block %u thread %u\n", #c, __FILE__, \
             __LINE__, (unsigned)blockIdx.x, (unsigned)threadIdx.x);                     \
      __builtin_trap();                                                                  \
    }                                                                                    \
  } while (0)
#else
#define DCHECK(c) ((void)0)
#endif

struct DevParams {
  uint32_t kind, es, meas_len, out_len, jr_len, arity, calls, P, logP, glen, proof_len,
      verifier_len, chunk, bits, length, prep_share_len, helper_share_len, public_share_len,
      leader_share_len;
  uint32_t n, ld, force_slow;
  uint32_t nseg;  // fused accumulate: segment ids >= nseg are excluded from every aggregate
  // query-randomness elements per proof (2 for the two-gadget FPVec circuit, else 1) and the
  // leading dimension of the output-share scratch (FPVec runs the other scratch in sub-batches
  // of ld columns; out keeps one column per report of the batch)
  uint32_t qr_len, ld_out;
  // FPVec gadget 1 (ParallelSum(PolyEval(y^2 - 2^n y), chunk1)): calls, domain, poly length;
  // gadget 0 uses chunk / arity / calls / P / logP / glen.  invP1 = 1/P1, normc = entries *
  // 2^(2n-2) / 2 (the norm's constant term, one share of it), twon = 2^n.
  uint32_t chunk1, calls1, P1, logP1, glen1;
  uint32_t invP1_128[4], normc128[4], twon128[4];
  uint32_t vk[4];
  uint32_t dst[8][2];
  uint32_t roots128[MAX_ROOTS + 1][4];
  uint64_t roots64[MAX_ROOTS + 1];
  uint32_t invP128[4], half128[4];
  // P <= 32 only: sigma_e = sum_{c=1..calls} alpha^(ce) and twiddles alpha_P^i (i < P/2).
  // P = 64 / 128 (k_query_w): tw128[k] = alpha_(P/8)^k (k < P/16), tw128[8 + i] = alpha_P^i
  // (i < 8), and the sigma table of P entries in device memory (engine-owned; null if absent)
  uint32_t sigma128[32][4];
  uint32_t tw128[16][4];
  uint64_t invP64, half64;
  const uint4* sigma_dev;
  // 1: the helper XOF kernel also truncates the measurement share into the output-share
  // scratch (TruncSink); the query kernel then leaves sc.out alone
  uint32_t trunc_xof;
  // 1: the query kernel skips reports the XOF flagged for the rejection-sampling slow path; the
  // run ends with one k_xof_slow launch (which marks the redone reports 2) and a redo launch of
  // the query (redo = 1) over exactly those reports, instead of a k_xof_slow launch per chunk
  // between the XOF and the query
  uint32_t slow_defer, redo;
  // Prio3Sum query (k_query_sum, P = 16 NPH): tws[j] = w16^j (j < 8), tws[8 + i] = alpha_P^i
  // (i < 8), tws[16 + i] = alpha_P^(16 i) (i < 8)
  uint32_t tws[24][4];
};

struct InPtrs {
  const uint8_t* nonces;
  const uint8_t* pub;
  const uint8_t* helper;
  const uint8_t* leader;
  // coalesced launches of several tasks: per-report verify-key slot into vk_tab (nullable: the
  // engine's own key, DevParams::vk)
  const uint16_t* vk_slot = nullptr;
  const uint4* vk_tab = nullptr;
  // executor groups (xofd_body<.., PULL>): the lane's leader prep share is copied from here (the
  // mapped host staging) into `leader` during its XOF, and its segment id / accept byte from
  // seg_src / accept_src into seg_dst / accept_dst (nullable)
  const uint8_t* leader_src = nullptr;
  const uint32_t* seg_src = nullptr;
  uint32_t* seg_dst = nullptr;
  const uint8_t* accept_src = nullptr;
  uint8_t* accept_dst = nullptr;
  // leader executor groups (k_leader_prep): the leader input shares are read by the kernel
  // straight from the mapped staging, transposed there by the job threads into [element][lin_ld]
  // 16-byte cells, so each load of a wave is 64 consecutive cells (one 1 KiB PCIe read) -- 0:
  // AoS rows of leader_share_len bytes (device memory)
  uint32_t lin_ld = 0;
};

// the verify key of report r (query randomness: XOF(vk, dst(5), [PROOFS] || nonce))
DEV void load_vk(const DevParams& p, const InPtrs& in, uint32_t r, uint32_t vk[4]) {
  if (in.vk_slot) {
    const uint4 v = in.vk_tab[in.vk_slot[r]];
    vk[0] = v.x;
    vk[1] = v.y;
    vk[2] = v.z;
    vk[3] = v.w;
  } else {
    vk[0] = p.vk[0];
    vk[1] = p.vk[1];
    vk[2] = p.vk[2];
    vk[3] = p.vk[3];
  }
}

struct Scratch {
  void* meas;
  void* proofs;
  void* jr;
  void* qr;
  uint4* part;
  uint4* corrected;
  uint8_t* flag;
  void* Lbuf;
  void* PVbuf;
  void* acc;
  void* out;
  void* beta;
  // fused accumulate (prio3_device_prepare_aggregate): per-report segment ids (nullable),
  // per-wave half-limb partial sums [wave][meas_len][8] and per-wave segment (~0 = not fused)
  const uint32_t* seg;
  uint32_t* wpart;
  uint32_t* wseg;
};

struct OutPtrs {
  uint8_t* prep_msgs;
  uint8_t* status;
};

template <class F>
struct FC;  // per-field constants from DevParams
template <>
struct FC<Fp128> {
  static DEV f128 root(const DevParams& p, int l) { return Fp128::from_words(p.roots128[l]); }
  static DEV f128 invP(const DevParams& p) { return Fp128::from_words(p.invP128); }
  static DEV f128 half(const DevParams& p) { return Fp128::from_words(p.half128); }
};
template <>
struct FC<Fp64> {
  static DEV uint64_t root(const DevParams& p, int l) { return p.roots64[l]; }
  static DEV uint64_t invP(const DevParams& p) { return p.invP64; }
  static DEV uint64_t half(const DevParams& p) { return p.half64; }
};

DEV void load16(const uint8_t* p, uint32_t* w) {
  uint4 v = *(const uint4*)p;
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
}

// The helper's prepare message and its prepare_next check (prio Prio3:
// prepare_shares_to_prepare_message hashes the two joint-rand parts of the prep shares into the
// joint-rand seed; prepare_next requires it to equal the corrected seed, which the XOF kernel
// derived from the leader part of the public share and the helper's own part).  The message is
// re-hashed as prio does.  Returns true if the check passes; msg gets the message.
DEV bool prep_msg_check(const DevParams& p, const InPtrs& in, const Scratch& sc, uint32_t r,
                        const uint32_t lpart[4], uint32_t msg[4]) {
  const uint4 cor = sc.corrected[r];
  uint32_t hpart[4];
  {
    const uint4 hp = sc.part[r];
    hpart[0] = hp.x, hpart[1] = hp.y, hpart[2] = hp.z, hpart[3] = hp.w;
  }
  KState s;
  kzero(s);
  Msg mm;
  msg_zero(mm);
  msg_dst(mm, p.dst[6]);
  msg_bytes16(mm, 25, lpart);
  msg_bytes16(mm, 41, hpart);
  msg_absorb_final(s, mm, 57);
  msg[0] = kword(s, 0), msg[1] = kword(s, 1), msg[2] = kword(s, 2), msg[3] = kword(s, 3);
  return msg[0] == cor.x && msg[1] == cor.y && msg[2] == cor.z && msg[3] == cor.w;
}

// ------------------------------------------------------------------------------------
// Byte-level sponge with rejection sampling (the slow path for flagged reports)
// ------------------------------------------------------------------------------------
struct BX {
  KState s;
  uint8_t buf[168];
  uint32_t pos;
};
DEV void bx_xor_block(BX& x) {
#pragma unroll
  for (int w = 0; w < 42; w++) {
    uint32_t v = (uint32_t)x.buf[4 * w] | ((uint32_t)x.buf[4 * w + 1] << 8) |
                 ((uint32_t)x.buf[4 * w + 2] << 16) | ((uint32_t)x.buf[4 * w + 3] << 24);
    kxor_word(x.s, w, v);
  }
  keccak_p12(x.s);
}
DEV void bx_fill(BX& x) {
#pragma unroll
  for (int w = 0; w < 42; w++) {
    uint32_t v = kword(x.s, w);
    x.buf[4 * w] = v;
    x.buf[4 * w + 1] = v >> 8;
    x.buf[4 * w + 2] = v >> 16;
    x.buf[4 * w + 3] = v >> 24;
  }
  x.pos = 0;
}
DEV void bx_absorb(BX& x, uint8_t b) {
  x.buf[x.pos++] = b;
  if (x.pos == 168) {
    bx_xor_block(x);
    x.pos = 0;
  }
}
DEV void bx_absorb_w(BX& x, const uint32_t* w, int nbytes) {
  for (int i = 0; i < nbytes; i++) bx_absorb(x, (uint8_t)(w[i >> 2] >> (8 * (i & 3))));
}
DEV void bx_init(BX& x, const uint32_t* dst2, const uint32_t* seed) {
  kzero(x.s);
  x.pos = 0;
  bx_absorb(x, 8);
  bx_absorb_w(x, dst2, 8);
  bx_absorb_w(x, seed, 16);
}
DEV void bx_finalize(BX& x) {
  for (uint32_t i = x.pos; i < 168; i++) x.buf[i] = 0;
  x.buf[x.pos] ^= 0x01;
  x.buf[167] ^= 0x80;
  bx_xor_block(x);
  bx_fill(x);
}
DEV uint8_t bx_squeeze(BX& x) {
  if (x.pos == 168) {
    keccak_p12(x.s);
    bx_fill(x);
  }
  return x.buf[x.pos++];
}
// next accepted element (rejection sampling); writes ES/4 words
template <class F>
DEV void bx_next_elem(BX& x, uint32_t* w) {
  for (;;) {
    for (int k = 0; k < F::ES / 4; k++) {
      uint32_t v = 0;
      for (int b = 0; b < 4; b++) v |= (uint32_t)bx_squeeze(x) << (8 * b);
      w[k] = v;
    }
    if (F::lt_p(F::from_words(w))) return;
  }
}

// XOF(seed, dst, binder).expand_into_vec(n) with rejection sampling, into SoA columns
template <class F>
DEV void bx_expand(const uint32_t* dst2, const uint32_t* seed, const uint8_t* binder, int blen,
                   uint32_t n, void* base, size_t ld, uint32_t r) {
  BX x;
  bx_init(x, dst2, seed);
  for (int i = 0; i < blen; i++) bx_absorb(x, binder[i]);
  bx_finalize(x);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t w[4];
    bx_next_elem<F>(x, w);
    F::store(base, (size_t)i * ld + r, F::from_words(w));
  }
}

// ------------------------------------------------------------------------------------
// k_xof: fast path (no rejection)
// ------------------------------------------------------------------------------------
template <class F>
DEV void put_elem(const DevParams& p, void* base, uint32_t idx, uint32_t r, const uint32_t* w,
                  uint32_t& flag) {
  typename F::T x = F::from_words(w);
  if (!F::lt_p(x)) flag = 1;
  DCHECK(r < p.ld);
  F::store(base, (size_t)idx * p.ld + r, x);
}

// Elements contained in squeeze block b of an XOF stream (no rejection), handed to put(idx, w)
// in index order.
template <class F, class Put>
DEV void squeeze_block_with(const KState& s, uint32_t b, uint32_t n_elems, uint32_t& pend0,
                            uint32_t& pend1, Put&& put) {
  if constexpr (F::ES == 16) {
    uint32_t e0 = 21 * (b >> 1);
    if ((b & 1) == 0) {
#pragma unroll
      for (int t = 0; t < 10; t++) {
        uint32_t w[4] = {kword(s, 4 * t), kword(s, 4 * t + 1), kword(s, 4 * t + 2),
                         kword(s, 4 * t + 3)};
        if (e0 + t < n_elems) put(e0 + t, w);
      }
      pend0 = kword(s, 40);
      pend1 = kword(s, 41);
    } else {
      {
        uint32_t w[4] = {pend0, pend1, kword(s, 0), kword(s, 1)};
        if (e0 + 10 < n_elems) put(e0 + 10, w);
      }
#pragma unroll
      for (int t = 0; t < 10; t++) {
        uint32_t w[4] = {kword(s, 2 + 4 * t), kword(s, 3 + 4 * t), kword(s, 4 + 4 * t),
                         kword(s, 5 + 4 * t)};
        if (e0 + 11 + t < n_elems) put(e0 + 11 + t, w);
      }
    }
  } else {
    uint32_t e0 = 21 * b;
#pragma unroll
    for (int t = 0; t < 21; t++) {
      uint32_t w[2] = {kword(s, 2 * t), kword(s, 2 * t + 1)};
      if (e0 + t < n_elems) put(e0 + t, w);
    }
  }
}

// Elements of squeeze block b stored to SoA column r of base (rejections flagged)
template <class F>
DEV void squeeze_block(const DevParams& p, const KState& s, uint32_t b, uint32_t n_elems,
                       uint32_t& pend0, uint32_t& pend1, void* base, uint32_t r,
                       uint32_t& flag) {
  squeeze_block_with<F>(s, b, n_elems, pend0, pend1, [&](uint32_t i, const uint32_t* w) {
    put_elem<F>(p, base, i, r, w, flag);
  });
}

// a += m << s over a 160-bit accumulator, s < 32 (wave-uniform)
DEV void shl_add160(sum128& a, const f128& m, uint32_t s) {
  uint32_t w0 = m.w[0], w1 = m.w[1], w2 = m.w[2], w3 = m.w[3], w4 = 0;
  if (s) {
    const uint32_t rs = 32 - s;
    w4 = m.w[3] >> rs;
    w3 = __builtin_amdgcn_alignbit(m.w[3], m.w[2], rs);
    w2 = __builtin_amdgcn_alignbit(m.w[2], m.w[1], rs);
    w1 = __builtin_amdgcn_alignbit(m.w[1], m.w[0], rs);
    w0 = m.w[0] << s;
  }
  uint32_t c;
  a.w[0] = addc(a.w[0], w0, 0, &c);
  a.w[1] = addc(a.w[1], w1, c, &c);
  a.w[2] = addc(a.w[2], w2, c, &c);
  a.w[3] = addc(a.w[3], w3, c, &c);
  a.w[4] = a.w[4] + w4 + c;
}

// On-the-fly truncation of a Field128 measurement-share stream (SumVec truncate, FPVec entry
// decode): entry e = sum_(b < nb) 2^b m_(e nb + b), accumulated over 160 bits as the elements
// are squeezed and stored to out[e] (leading dimension ld_out), so the query kernel does not
// re-read the share for it.  nb <= 32; elements arrive in index order from 0; elements past
// the n_ent entries (FPVec's claimed-norm bits) are not entries.  DevParams::trunc_xof.
struct TruncSink {
  void* out;
  size_t ld_out;
  uint32_t r, nb, n_ent, e, bit;
  sum128 acc;
  DEV TruncSink(const DevParams& p, void* o, uint32_t rr)
      : out(o), ld_out(p.ld_out), r(rr), nb(p.bits), n_ent(p.out_len), e(0), bit(0) {
    sum_zero(acc);
  }
  DEV void put(const f128& m) {
    if (e >= n_ent) return;  // wave-uniform
    shl_add160(acc, m, bit);
    if (++bit == nb) {
      Fp128::store(out, (size_t)e * ld_out + r, sum_reduce(acc));
      sum_zero(acc);
      bit = 0;
      e++;
    }
  }
};

// squeeze_block for the measurement share with the truncation sink (TR) or without
template <bool TR>
DEV void squeeze_meas(const DevParams& p, const KState& s, uint32_t b, uint32_t n_elems,
                      uint32_t& pend0, uint32_t& pend1, void* base, uint32_t r, uint32_t& flag,
                      TruncSink& ts) {
  squeeze_block_with<Fp128>(s, b, n_elems, pend0, pend1, [&](uint32_t i, const uint32_t* w) {
    put_elem<Fp128>(p, base, i, r, w, flag);
    if constexpr (TR) ts.put(mk128(w[0], w[1], w[2], w[3]));
  });
}


DEV uint32_t bitrev(uint32_t x, uint32_t d) { return __builtin_bitreverse32(x) >> (32 - d); }

// In-place radix-2 DIT DFT of one lane's n-element SoA column (input in bit-reversed
// order), twiddles from the field's principal 2^l-th roots -- the same butterfly order as
// prio fft.rs discrete_fourier_transform.
template <class F>
DEV void dft_lane(const DevParams& p, void* buf, uint32_t r, uint32_t n, uint32_t logn) {
  typedef typename F::T T;
  const size_t ld = p.ld;
  DCHECK(r < ld);
  for (uint32_t l = 1; l <= logn; l++) {
    const uint32_t half = 1u << (l - 1);
    const T wl = FC<F>::root(p, l);
    T w = F::one();
    for (uint32_t i = 0; i < half; i++) {
      for (uint32_t j = i; j < n; j += 2 * half) {
        T u = F::load(buf, (size_t)j * ld + r);
        T v = F::mul(w, F::load(buf, (size_t)(j + half) * ld + r));
        F::store(buf, (size_t)j * ld + r, F::add(u, v));
        F::store(buf, (size_t)(j + half) * ld + r, F::sub(u, v));
      }
      w = F::mul(w, wl);
    }
  }
}

template <class F>
DEV typename F::T ldf(const void* base, uint32_t e, size_t ld, uint32_t r) {
  DCHECK(r < ld);
  return F::load(base, (size_t)e * ld + r);
}


// In-register radix-2 DFT of N (<= 16) Field128 values given in bit-reversed order; twiddle
// w_N^i = p.tw128[i * stride * (32 / 2 / (N/2)) ...] is taken from the P-th root table.
template <int N, int LOGN>
DEV void dft_reg(const DevParams& p, f128 (&x)[N], int stride) {
  typedef Fp128 F;
#pragma unroll
  for (int l = 1; l <= LOGN; l++) {
    const int half = 1 << (l - 1);
#pragma unroll
    for (int i = 0; i < half; i++) {
      // w_(2^l)^i = w_(N*stride)^(i * stride * N / 2^l)
      const f128 w = F::from_words(p.tw128[i * stride * (N >> l)]);
#pragma unroll
      for (int j = i; j < N; j += 2 * half) {
        const f128 u = x[j];
        const f128 v = (i == 0) ? x[j + half] : F::mul(w, x[j + half]);
        x[j] = F::add(u, v);
        x[j + half] = F::sub(u, v);
      }
    }
  }
}

// FlpGeneric::query for one report (one lane), num_shares = 2.  Writes the wire-polynomial
// values at t into acc[0..arity) and returns v (circuit output share) and pt = p(t).
// Returns false if t is a P-th root of unity (prio FlpError -> VdafPrepareInit).
template <class F>
DEV bool flp_query_lane(const DevParams& p, const void* meas, const void* proofs, const void* jr,
                        typename F::T t, void* Lbuf, void* PVbuf, void* acc, uint32_t r,
                        typename F::T& v, typename F::T& pt) {
  typedef typename F::T T;
  const size_t ld = p.ld;
  const uint32_t P = p.P, A = p.arity;
  T tp = t;
  for (uint32_t l = 0; l < p.logP; l++) tp = F::mul(tp, tp);
  const bool t_ok = !F::eq(tp, F::one());
  // Lagrange basis at t: L_c = (1/P) sum_e t^e alpha^(-ce) = DFT(t^e / P)[(P - c) mod P]
  {
    T pw = FC<F>::invP(p);
    for (uint32_t e = 0; e < P; e++) {
      F::store(Lbuf, (size_t)bitrev(e, p.logP) * ld + r, pw);
      pw = F::mul(pw, t);
    }
    dft_lane<F>(p, Lbuf, r, p.P, p.logP);
  }
  // gadget polynomial at the P-th roots: fold coefficients mod x^P - 1, DFT
  for (uint32_t e = 0; e < P; e++) {
    T q = ldf<F>(proofs, A + e, ld, r);
    if (e + P < p.glen) q = F::add(q, ldf<F>(proofs, A + e + P, ld, r));
    F::store(PVbuf, (size_t)bitrev(e, p.logP) * ld + r, q);
  }
  dft_lane<F>(p, PVbuf, r, p.P, p.logP);
  // p(t)
  pt = F::zero();
  for (uint32_t e = p.glen; e-- > 0;) pt = F::add(F::mul(pt, t), ldf<F>(proofs, A + e, ld, r));
  auto Lc = [&](uint32_t c) { return ldf<F>(Lbuf, (P - c) & (P - 1), ld, r); };
  // wire accumulators start from the proof's wire seeds
  {
    const T L0 = Lc(0);
    for (uint32_t w = 0; w < A; w++)
      F::store(acc, (size_t)w * ld + r, F::mul(ldf<F>(proofs, w, ld, r), L0));
  }
  auto acc_add = [&](uint32_t w, const T& v) {
    size_t idx = (size_t)w * ld + r;
    F::store(acc, idx, F::add(F::load(acc, idx), v));
  };
  v = F::zero();
  if (p.kind == PRIO3_COUNT) {
    const T m = ldf<F>(meas, 0, ld, r);
    const T x = F::mul(m, Lc(1));
    acc_add(0, x);
    acc_add(1, x);
    v = F::sub(ldf<F>(PVbuf, 1, ld, r), m);
  } else if (p.kind == PRIO3_SUM) {
    const T r0 = ldf<F>(jr, 0, ld, r);
    T rp = r0;
    for (uint32_t i = 0; i < p.meas_len; i++) {
      acc_add(0, F::mul(ldf<F>(meas, i, ld, r), Lc(i + 1)));
      v = F::add(v, F::mul(rp, ldf<F>(PVbuf, i + 1, ld, r)));
      rp = F::mul(rp, r0);
    }
  } else {
    const T r0 = ldf<F>(jr, 0, ld, r);
    const T half = FC<F>::half(p);
    T rp = r0, range = F::zero(), sum = F::zero();
    for (uint32_t k = 0; k < p.calls; k++) {
      const T L = Lc(k + 1);
      for (uint32_t j = 0; j < p.chunk; j++) {
        const uint32_t i = k * p.chunk + j;
        const T m = i < p.meas_len ? ldf<F>(meas, i, ld, r) : F::zero();
        acc_add(2 * j, F::mul(F::mul(rp, m), L));
        acc_add(2 * j + 1, F::mul(F::sub(m, half), L));
        rp = F::mul(rp, r0);
        sum = F::add(sum, m);
      }
      range = F::add(range, ldf<F>(PVbuf, k + 1, ld, r));
    }
    if (p.kind == PRIO3_SUMVEC) {
      v = range;
    } else {
      const T r1 = ldf<F>(jr, 1, ld, r);
      v = F::add(F::mul(r1, range), F::mul(F::mul(r1, r1), F::sub(sum, half)));
    }
  }
  return t_ok;
}

// host-side field helpers (parameter setup only)
namespace {

typedef unsigned __int128 u128;
const u128 HP128 = (((u128)0xffffffffffffffe4ULL) << 64) | 1;
const uint64_t HP64 = 0xffffffff00000001ULL;

u128 hmul(u128 a, u128 b, u128 p) {  // slow but simple: double-and-add
  u128 r = 0;
  a %= p;
  while (b) {
    if (b & 1) {
      r += a;
      if (r < a || r >= p) r -= p;
    }
    u128 a2 = a + a;
    if (a2 < a || a2 >= p) a2 -= p;
    a = a2;
    b >>= 1;
  }
  return r;
}
u128 hpow(u128 a, u128 e, u128 p) {
  u128 r = 1;
  while (e) {
    if (e & 1) r = hmul(r, a, p);
    a = hmul(a, a, p);
    e >>= 1;
  }
  return r;
}

}  // namespace

// ------------------------------------------------------------------------------------
// Host-side engine object (shared by both translation units)
// ------------------------------------------------------------------------------------
struct KTime {
  std::string name;
  double ms = 0;
  uint64_t launches = 0;
};

// PRIO3_SUMVEC_F64_MP (prio3_mp64.hip): Field64 SumVec, XofHmacSha256Aes128, multiproof
struct Mp64Params {
  uint32_t meas_len, out_len, bits, chunk, calls, P, logP, glen, proof_len /* one proof */,
      arity, vlen, np;
  uint32_t dst[8][2];          // dst(usage) bytes, LE words
  uint32_t vk_ist[8], vk_ost[8];    // HMAC midstates of the verify key (query randomness)
  uint32_t z_ist[8], z_ost[8];      // HMAC midstates of the all-zero seed (joint-rand seeds)
  uint64_t alpha, alpha_inv, invP, half;
  const uint64_t* sigma;       // device [P]: sum_{k=1..calls} alpha^(k e)
};

struct prio3_engine;
// prio3_query_sum.hip: true if launched (Prio3Sum with 16 <= P <= 128)
bool query_sum_takes(const DevParams& p);
bool launch_query_sum(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st,
                      bool leader = false);
int launch_mp64(prio3_engine* e, uint32_t n, uint32_t ld, InPtrs in, OutPtrs out, Scratch sc,
                hipStream_t st);
int launch_mp64_leader(prio3_engine* e, uint32_t n, uint32_t ld, InPtrs in, OutPtrs out,
                       Scratch sc, hipStream_t st);
int launch_mp64_leader_next(uint32_t n, const uint8_t* d_prep_msgs, Scratch sc, uint8_t* d_status,
                            hipStream_t st);
// long-share helper XOF on lane pairs (prio3_xof_pair.hip); false if the instance is not one it takes
bool launch_xof_pair(const DevParams& p, InPtrs in, Scratch sc, hipStream_t st);
// prio3_prep_pair.hip: Histogram (P = 32) prepare on lane pairs (k_prep_hp); true if launched
bool prep_pair_takes(const DevParams& p, bool pull);
bool launch_prep_pair(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st,
                      bool fuse, bool pull);
// P = 64 / 128 ParallelSum(Mul) helper query, eight lanes per report (prio3_query_wide.hip);
// false if the instance is not one it takes
bool launch_query_wide(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st);
bool query_wide_takes(const DevParams& p);
// FPVec FLP query + decide + prepare message + truncate for p.n reports (prio3_fpvec.hip)
// wide: the eight-lane kernel k_query_fpw (fpvec_query_wide_takes); leader: its agg_id-0 role
void launch_fpvec_query(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st,
                        bool wide, bool leader);
bool fpvec_query_wide_takes(const DevParams& p);

struct Slab;
// The device state of one prepare call (helper or leader) over n reports: the SoA scratch, the
// device copies of host-buffer inputs/outputs and the fused-accumulate state, carved out of one
// slab of the GPU's shared scratch pool (prio3_runtime.h).  Reference-counted: every batch handle
// of the call holds one reference (host entry points), the engine holds one for its latest
// device-resident call; the slab returns to the pool when the last reference goes.
struct Run {
  prio3_engine* e = nullptr;  // engine whose instance / options planned it
  Slab* slab = nullptr;
  int device = 0;
  DevParams dp;    // instance parameters with n, ld, ld_out of this run
  uint32_t n = 0;  // reports (columns)
  Scratch sc{};
  uint8_t *nonces = nullptr, *pub = nullptr, *helper = nullptr, *leader = nullptr,
          *linput = nullptr, *msgs = nullptr, *status = nullptr;
  uint16_t* vk_slot = nullptr;
  uint4* vk_tab = nullptr;
  // fused accumulate (prio3_device_prepare_aggregate)
  uint32_t *wpart = nullptr, *wseg = nullptr, *cseg = nullptr, *fix = nullptr;
  uint4* corr_all = nullptr;  // FPVec: corrected joint-rand seeds of all n reports (leader)
  unsigned long long *cpart = nullptr, *agg64 = nullptr;
  size_t fix_cap = 0;
  bool fused = false;
  bool aggregate = false;  // made by prio3_device_prepare_aggregate (finish may follow)
  bool lfused = false;     // leader init summed the wave partials (segment 0; leader_fuse_acc)
  // reports per wave of the fused partials: 2^6 (one lane per report), 2^5 (k_prep_hp's pairs)
  uint32_t wshift = 6;
  uint32_t nseg = 0;
  const uint32_t* seg = nullptr;
  // executor groups with aggregating jobs (RUN_AGG_IO): group segment ids, accept bytes, the
  // per-segment aggregate shares and counts
  uint32_t* gseg = nullptr;
  uint8_t *gaccept = nullptr, *gagg = nullptr, *gcnt = nullptr;
  std::atomic<int> refs{1};
  hipStream_t last = nullptr;  // stream of the latest work on the run (its release point)
  bool keep = false;  // the engine's keep_scratch: the slab stays in the pool above its budget
  // sealed-input groups (RUN_HPKE): the open's status per report and its plaintext scratch
  uint32_t hpke_stride = 0;
  uint8_t *hstatus = nullptr, *hpt = nullptr;
};

struct prio3_engine {
  prio3_params params;
  prio3_sizes_t sz;
  DevParams dp;
  int device;
  Run* cur = nullptr;  // the latest device-resident prepare (its output shares stay here)
  int fuse_acc = 1;
  int leader_fast = 1;
  int leader_fuse_acc = 1;  // option: device leader init accumulates wave partials (k_jrpart<true>)
  int chunks = 0;            // option: prepare in this many stream-overlapped chunks (0 = auto)
  int64_t fp_sub_bytes = 0;  // option: FPVec per-sub-batch scratch budget (bytes; 0 = auto)
  int coalesce = 1;          // option: host-buffer prepare through the coalescing executor
  // option: PRIO3_FPVEC_BOUNDED_L2 prepares only after this explicit opt-in -- its circuit is a
  // reconstruction (prio's fixedpoint_l2.rs is not in the reference; parity with prio unpinned)
  int experimental_fpvec = 0;
  std::vector<hipStream_t> side;  // side streams for chunked prepare
  std::vector<hipEvent_t> side_ev;
  hipEvent_t fork_ev = nullptr;
  int force_slow = 0;     // test hook: every report through the rejection-sampling slow path
  int force_generic = 0;  // test hook: the one-lane fallback queries (k_query_ps, k_query,
                          // k_query_fp) that take the shapes the specialised kernels do not
  int n_cu = 256;    // compute units of the engine's GPU
  int fp_round = 1;  // FPVec sub-batches rounded to whole query rounds (fp_sub_sizes)
  // option: Histogram (P = 32) prepares of at most this many reports run on lane pairs
  // (k_prep_hp; 0 = never): below ~3 waves per SIMD the one-lane k_prep_h leaves SIMDs idle
  int pair_max = 196608;
  int timing = 0;
  // option: a released run's slab stays in the GPU's pool even above the pool's budget (a
  // device-resident caller running FPVec batches back to back; default: the budget applies)
  int keep_scratch = 0;
  Mp64Params mp{};  // PRIO3_SUMVEC_F64_MP only
  uint64_t* d_sigma64 = nullptr;
  uint4* d_sigma128 = nullptr;  // k_query_w's sigma table (DevParams::sigma_dev)
  std::vector<KTime> times;
  std::vector<hipEvent_t> ev_pool;
  std::mutex tmu;  // timing bookkeeping (launches may come from several executor threads)
  std::mutex mu;   // device-resident calls, `cur`, side streams
  // ---- one engine over several GPUs (prio3_engine_create_devices / _mask) ----
  // lane: this engine's executor on its GPU (0 unless a device list names the GPU again)
  int lane = 0;
  // members[0] is the engine itself; the others are engines of the same instance and verify key
  // on the other listed GPUs (owned by it).  Host-buffer jobs go to the least-loaded member;
  // device-resident calls act on members[0].
  std::vector<prio3_engine*> members;
  prio3_engine* owner = nullptr;   // the engine whose member this is (nullptr: itself)
  std::atomic<uint32_t> rr{0};     // round-robin start among equally loaded members
  std::atomic<uint64_t> placed_jobs{0}, placed_reports{0};  // host-buffer jobs placed here
};

