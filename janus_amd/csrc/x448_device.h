// x448_device.h -- X448 (RFC 7748 section 5) for DHKEM(X448, HKDF-SHA512) (RFC 9180 7.1, KEM
// 0x0021, messages/src/lib.rs:770-784 HpkeKemId::X448HkdfSha512), one report per work-item.
//
// GF(p), p = 2^448 - 2^224 - 1 (the "Goldilocks" prime): 16 limbs of 28 bits in 32-bit words
// (unsaturated, so a product's 16 x 16 limb products accumulate per column in 64 bits with no
// carry chains: v_mad_u64_u32 each).  Operands of a product have limbs < 2^29, so a column of
// at most 16 products stays < 2^62.  The 896-bit product folds with 2^448 = 2^224 + 1 (mod p).
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

// the 31 column sums c of a product (each < 2^62) -> reduced limbs
DEV fe reduce(uint64_t c[32]) {
  c[31] = 0;
#pragma unroll
  for (int k = 0; k < 31; k++) {
    c[k + 1] += c[k] >> 28;
    c[k] &= M28;
  }
  // X = L + H 2^448 = L + H + H 2^224, whose H[8..15] 2^448 part folds once more:
  // r_k = l_k + h_k + h_(k+8) (k < 8), l_k + 2 h_k + h_(k-8) (k >= 8); h_15 = c[31] is < 2^35
  uint64_t r[16];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = c[k] + c[16 + k] + c[24 + k];
#pragma unroll
  for (int k = 8; k < 16; k++) r[k] = c[k] + 2 * c[16 + k] + c[8 + k];
#pragma unroll
  for (int k = 0; k < 15; k++) {
    r[k + 1] += r[k] >> 28;
    r[k] &= M28;
  }
  const uint64_t t = r[15] >> 28;
  r[15] &= M28;
  r[0] += t;
  r[8] += t;
  fe o;
#pragma unroll
  for (int k = 0; k < 16; k++) o.v[k] = (uint32_t)r[k];
  // t < 2^9: limbs 0 and 8 stay < 2^28 + 2^9; one more pass keeps product inputs < 2^29
  carry(o.v);
  return o;
}

DEV fe mul(const fe& a, const fe& b) {
  uint64_t c[32];
#pragma unroll
  for (int k = 0; k < 32; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 16; i++)
#pragma unroll
    for (int j = 0; j < 16; j++) c[i + j] += (uint64_t)a.v[i] * b.v[j];
  return reduce(c);
}

// 136 products: the off-diagonal ones once, against the doubled limb
DEV fe sqr(const fe& a) {
  uint64_t c[32];
  uint32_t d[16];
#pragma unroll
  for (int k = 0; k < 32; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) d[i] = 2 * a.v[i];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    c[2 * i] += (uint64_t)a.v[i] * a.v[i];
#pragma unroll
    for (int j = i + 1; j < 16; j++) c[i + j] += (uint64_t)d[i] * a.v[j];
  }
  return reduce(c);
}

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
