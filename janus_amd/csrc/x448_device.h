// x448_device.h -- X448 (RFC 7748 section 5) for DHKEM(X448, HKDF-SHA512) (RFC 9180 7.1, KEM
// 0x0021, messages/src/lib.rs:770-784 HpkeKemId::X448HkdfSha512), one report per work-item.
//
// GF(p), p = 2^448 - 2^224 - 1 (the "Goldilocks" prime): 16 limbs of 28 bits in 32-bit words
// (unsaturated, so a product's 16 x 16 limb products accumulate per column in 64 bits with no
// carry chains: v_mad_u64_u32 each).  Operands of a product have limbs < 2^29, so a column of
// at most 16 products (+ the previous column's carry) stays < 2^63.  The 896-bit product folds
// with 2^448 = 2^224 + 1 (mod p).
// The scalar is the server's private key, the same in every lane: the ladder's swaps are
// wave-uniform branches (no key-dependent divergence; every lane runs the same stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace x448 {

constexpr uint32_t M28 = 0x0fffffffu;

struct fe {
  uint32_t v[16];
};

DEV fe set(uint32_t x) {
  fe r;
#pragma unroll
  for (int i = 0; i < 16; i++) r.v[i] = i ? 0u : x;
  return r;
}

// limbs -> [0, 2^28) each, except limbs 0 and 8, which take the fold of the carry out of 2^448
// (2^448 = 2^224 + 1) and may exceed 2^28 by that carry (< 2^29 in every use here)
DEV void carry(uint32_t v[16]) {
#pragma unroll
  for (int i = 0; i < 15; i++) {
    v[i + 1] += v[i] >> 28;
    v[i] &= M28;
  }
  const uint32_t t = v[15] >> 28;
  v[15] &= M28;
  v[0] += t;
  v[8] += t;
}

DEV fe add(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 16; i++) r.v[i] = a.v[i] + b.v[i];
  carry(r.v);
  return r;
}

// a - b + 2p (2p's limbs: 2^29 - 2, limb 8: 2^29 - 4), then carried
DEV fe sub(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 16; i++) r.v[i] = a.v[i] + (i == 8 ? 0x1ffffffcu : 0x1ffffffeu) - b.v[i];
  carry(r.v);
  return r;
}


// Product scanning (r05): each column accumulates in one 64-bit register (one v_mad_u64_u32 per
// limb product with the running sum as its addend), is carried into the next column at once and
// leaves one 28-bit limb, so the 2^448 = 2^224 + 1 fold runs on 32-bit limbs instead of 64-bit
// columns: 4,049 instructions per ladder step against 4,481 with 64-bit column sums, 18.0
// against 16.6 M input shares/s (profiles/r05/x448/).
// value = L + 2^448 (H + 2^448 top) (28-bit limbs): H 2^448 = H (1 + 2^224), its limbs 8..15
// wrapping once more; top 2^896 = 3 2^224 + 2 (mod p)
DEV fe fold_ps(const uint32_t lo[16], const uint32_t hi[16], uint32_t top) {
  uint32_t r[16];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = lo[k] + hi[k] + hi[k + 8] + (k == 0 ? 2 * top : 0);
#pragma unroll
  for (int k = 8; k < 16; k++) r[k] = lo[k] + 2 * hi[k] + hi[k - 8] + (k == 8 ? 3 * top : 0);
  fe o;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    r[k + 1] += r[k] >> 28;
    o.v[k] = r[k] & M28;
  }
  const uint32_t t = r[15] >> 28;
  o.v[15] = r[15] & M28;
  o.v[0] += t;  // limbs 0 and 8 may exceed 2^28 by t (< 2^29, as carry() leaves them)
  o.v[8] += t;
  return o;
}
DEV fe mul_ps(const fe& a, const fe& b) {
  uint32_t lo[16], hi[16];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 31; k++) {
#pragma unroll
    for (int i = (k < 16 ? 0 : k - 15); i <= (k < 16 ? k : 15); i++)
      acc += (uint64_t)a.v[i] * b.v[k - i];
    (k < 16 ? lo[k] : hi[k - 16]) = (uint32_t)acc & M28;
    acc >>= 28;
  }
  hi[15] = (uint32_t)acc & M28;
  return fold_ps(lo, hi, (uint32_t)(acc >> 28));
}
DEV fe sqr_ps(const fe& a) {
  uint32_t lo[16], hi[16], d[16];
#pragma unroll
  for (int i = 0; i < 16; i++) d[i] = 2 * a.v[i];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 31; k++) {
#pragma unroll
    for (int i = (k < 16 ? 0 : k - 15); 2 * i < k; i++) acc += (uint64_t)d[i] * a.v[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.v[k / 2] * a.v[k / 2];
    (k < 16 ? lo[k] : hi[k - 16]) = (uint32_t)acc & M28;
    acc >>= 28;
  }
  hi[15] = (uint32_t)acc & M28;
  return fold_ps(lo, hi, (uint32_t)(acc >> 28));
}

DEV fe mul(const fe& a, const fe& b) { return mul_ps(a, b); }

// 136 products: the off-diagonal ones once, against the doubled limb
DEV fe sqr(const fe& a) { return sqr_ps(a); }

DEV fe mul_small(const fe& a, uint32_t k) {  // k < 2^16
  uint64_t r[16];
#pragma unroll
  for (int i = 0; i < 16; i++) r[i] = (uint64_t)a.v[i] * k;
#pragma unroll
  for (int i = 0; i < 15; i++) {
    r[i + 1] += r[i] >> 28;
    r[i] &= M28;
  }
  const uint64_t t = r[15] >> 28;
  r[15] &= M28;
  r[0] += t;
  r[8] += t;
  fe o;
#pragma unroll
  for (int i = 0; i < 16; i++) o.v[i] = (uint32_t)r[i];
  carry(o.v);
  return o;
}

DEV fe sqr_n(fe x, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) x = sqr(x);
  return x;
}

// a^(p - 2), p - 2 = [223 ones][0][222 ones][0][1] (MSB first); x_k = a^(2^k - 1)
DEV fe inv(const fe& a) {
  const fe x2 = mul(sqr(a), a);
  const fe x3 = mul(sqr(x2), a);
  const fe x6 = mul(sqr_n(x3, 3), x3);
  const fe x12 = mul(sqr_n(x6, 6), x6);
  const fe x24 = mul(sqr_n(x12, 12), x12);
  const fe x48 = mul(sqr_n(x24, 24), x24);
  const fe x96 = mul(sqr_n(x48, 48), x48);
  const fe x192 = mul(sqr_n(x96, 96), x96);
  const fe x216 = mul(sqr_n(x192, 24), x24);
  const fe x222 = mul(sqr_n(x216, 6), x6);
  const fe x223 = mul(sqr(x222), a);
  fe t = sqr(x223);             // [223 ones][0]
  t = mul(sqr_n(t, 222), x222);  // [222 ones]
  return mul(sqr_n(t, 2), a);   // [0][1]
}

// canonical representative in [0, p)
DEV fe freeze(const fe& a) {
  fe r = a;
  // after the second pass the value is < 2^448 (a carry out of 2^448 leaves a small value), after
  // the third every limb is < 2^28 as well
  carry(r.v);
  carry(r.v);
  carry(r.v);
  uint32_t d[16];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int32_t x = (int32_t)r.v[i] - (int32_t)(i == 8 ? 0x0ffffffeu : M28) + br;
    d[i] = (uint32_t)x & M28;
    br = x >> 28;  // 0 or -1
  }
  const bool ge = br == 0;
#pragma unroll
  for (int i = 0; i < 16; i++) r.v[i] = ge ? d[i] : r.v[i];
  return r;
}

// 56 little-endian bytes (as 14 LE words) -> limbs (any value < 2^448: RFC 7748 accepts
// non-canonical u-coordinates and reduces them)
DEV fe from_words(const uint32_t w[14]) {
  fe r;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int bit = 28 * k, q = bit >> 5, o = bit & 31;
    uint32_t x = w[q] >> o;
    if (o > 4 && q + 1 < 14) x |= w[q + 1] << (32 - o);
    r.v[k] = x & M28;
  }
  return r;
}
DEV void to_words(const fe& a, uint32_t w[14]) {
  const fe f = freeze(a);
#pragma unroll
  for (int q = 0; q < 14; q++) w[q] = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int bit = 28 * k, q = bit >> 5, o = bit & 31;
    w[q] |= f.v[k] << o;
    if (o > 4 && q + 1 < 14) w[q + 1] |= f.v[k] >> (32 - o);
  }
}

// X448(k, u) (RFC 7748 section 5): k = the clamped scalar as 14 LE words (wave-uniform), u the
// peer's u-coordinate as 14 LE words; the result u-coordinate as 14 LE words
__device__ __noinline__ void ladder(const uint32_t* k, const uint32_t u_w[14], uint32_t out[14]) {
  const fe x1 = from_words(u_w);
  fe x2 = set(1), z2 = set(0), x3 = x1, z3 = set(1);
  bool swap = false;
#pragma unroll 1
  for (int t = 447; t >= 0; t--) {
    const bool kt = (k[t >> 5] >> (t & 31)) & 1u;  // wave-uniform
    if (swap != kt) {
      const fe tx = x2, tz = z2;
      x2 = x3, z2 = z3, x3 = tx, z3 = tz;
    }
    swap = kt;
    const fe A = add(x2, z2), AA = sqr(A), B = sub(x2, z2), BB = sqr(B), E = sub(AA, BB);
    const fe C = add(x3, z3), D = sub(x3, z3), DA = mul(D, A), CB = mul(C, B);
    x3 = sqr(add(DA, CB));
    z3 = mul(x1, sqr(sub(DA, CB)));
    x2 = mul(AA, BB);
    z2 = mul(E, add(AA, mul_small(E, 39081)));
  }
  if (swap) {
    x2 = x3;
    z2 = z3;
  }
  to_words(mul(x2, inv(z2)), out);
}

}  // namespace x448
