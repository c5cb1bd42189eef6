// p521_device.h -- GF(2^521 - 1) for DHKEM(P-521, HKDF-SHA512) (RFC 9180 7.1, KEM 0x0012,
// messages/src/lib.rs:770-784 HpkeKemId::P521HkdfSha512), one report per work-item.
//
// 18 limbs of 29 bits in 32-bit words (limb 17 holds bits 493..520), unsaturated: a product's
// 18 x 18 limb products accumulate per column in 64 bits (v_mad_u64_u32 each) with no carry
// chains.  Product operands have limbs < 2^29 + 2^6, so a column of 18 products is < 2^62.2.
// The 1044-bit product is carried into 29-bit limbs and folded with 2^522 = 2 (mod p); the
// carry out of bit 521 folds into limb 0 (2^521 = 1).  The curve arithmetic (a = -3 Jacobian
// formulas, fixed signed window over the server key) is ecdh_a3.h's, shared with nothing else
// (P-256 keeps its generated-asm field, p256_device.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace p521 {

constexpr uint32_t M29 = 0x1fffffffu, M28 = 0x0fffffffu;
constexpr int NL = 18;

struct fp {
  uint32_t v[NL];
};

// limbs 0..16 -> [0, 2^29), limb 17 -> [0, 2^28); the carry out of bit 521 is added to limb 0,
// which may then exceed 2^29 by it (< 2^6 in every use here)
DEV void carry(uint32_t v[NL]) {
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    v[i + 1] += v[i] >> 29;
    v[i] &= M29;
  }
  const uint32_t t = v[NL - 1] >> 28;
  v[NL - 1] &= M28;
  v[0] += t;
}

DEV fp add(const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] + b.v[i];
  carry(r.v);
  return r;
}

// a - b + 2p (2p's limbs: 2^30 - 2, limb 17: 2^29 - 2), then carried
DEV fp sub(const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] + (i == NL - 1 ? 0x1ffffffeu : 0x3ffffffeu) - b.v[i];
  carry(r.v);
  return r;
}

DEV fp neg(const fp& a) {
  fp z;
#pragma unroll
  for (int i = 0; i < NL; i++) z.v[i] = 0;
  return sub(z, a);
}

// column sums c[0..34] (each < 2^62.2) -> reduced limbs
DEV fp reduce(uint64_t c[2 * NL]) {
  c[2 * NL - 1] = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
    c[k + 1] += c[k] >> 29;
    c[k] &= M29;
  }
  // limb k + 18 sits at 2^(29 k + 522) = 2 * 2^(29 k) (mod p)
  uint64_t r[NL];
#pragma unroll
  for (int k = 0; k < NL; k++) r[k] = c[k] + 2 * c[k + NL];
#pragma unroll
  for (int k = 0; k < NL - 1; k++) {
    r[k + 1] += r[k] >> 29;
    r[k] &= M29;
  }
  const uint64_t t = r[NL - 1] >> 28;
  r[NL - 1] &= M28;
  r[0] += t;
  fp o;
#pragma unroll
  for (int k = 0; k < NL; k++) o.v[k] = (uint32_t)r[k];
  carry(o.v);
  return o;
}

// Product scanning: column k of the 1044-bit product is accumulated in one 64-bit register
// (each limb product one v_mad_u64_u32 with the running sum as its addend), carried into the
// next column at once, and leaves one 29-bit limb: 36 limbs + 2 64-bit registers live instead of
// 35 64-bit columns, so the product can be inlined into the curve formulas (ecdh_a3.h's dbl4).
// The high limbs fold with 2^522 = 2 (mod p).
DEV fp fold(const uint32_t lo[NL], const uint32_t hi[NL], uint32_t top) {
  // value = lo + 2^522 (hi + 2^522 top), limbs 29 bits; 2^522 = 2 (mod p)
  fp o;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    const uint32_t x = lo[k] + 2 * hi[k] + (k == 0 ? 4 * top : 0) + c;  // < 2^31
    c = x >> (k == NL - 1 ? 28 : 29);
    o.v[k] = x & (k == NL - 1 ? M28 : M29);
  }
  o.v[0] += c;  // 2^521 = 1
  return o;
}
DEV fp mul_i(const fp& a, const fp& b) {
  uint32_t lo[NL], hi[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int i = (k < NL ? 0 : k - NL + 1); i <= (k < NL ? k : NL - 1); i++)
      acc += (uint64_t)a.v[i] * b.v[k - i];
    (k < NL ? lo[k] : hi[k - NL]) = (uint32_t)acc & M29;
    acc >>= 29;
  }
  hi[NL - 1] = (uint32_t)acc & M29;
  return fold(lo, hi, (uint32_t)(acc >> 29));
}
DEV fp sqr_i(const fp& a) {
  uint32_t lo[NL], hi[NL], d[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) d[i] = 2 * a.v[i];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int i = (k < NL ? 0 : k - NL + 1); 2 * i < k; i++) acc += (uint64_t)d[i] * a.v[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.v[k / 2] * a.v[k / 2];
    (k < NL ? lo[k] : hi[k - NL]) = (uint32_t)acc & M29;
    acc >>= 29;
  }
  hi[NL - 1] = (uint32_t)acc & M29;
  return fold(lo, hi, (uint32_t)(acc >> 29));
}

// out of line for the mixed additions, the table and the inversions (one copy each); the
// doublings, 3/4 of the multiplies, inline them (dbl4)
__device__ __noinline__ fp mul(const fp& a, const fp& b) { return mul_i(a, b); }
__device__ __noinline__ fp sqr(const fp& a) { return sqr_i(a); }

DEV fp mul_small(const fp& a, uint32_t k) {  // k <= 8
  uint64_t r[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) r[i] = (uint64_t)a.v[i] * k;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    r[i + 1] += r[i] >> 29;
    r[i] &= M29;
  }
  const uint64_t t = r[NL - 1] >> 28;
  r[NL - 1] &= M28;
  r[0] += t;
  fp o;
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = (uint32_t)r[i];
  carry(o.v);
  return o;
}

// x^(2^n): one out-of-line call around a loop of inlined squarings (the inversions' 520)
__device__ __noinline__ void sqr_n_ool(fp& x, int n) {
  fp y = x;
#pragma unroll 1
  for (int i = 0; i < n; i++) y = sqr_i(y);
  x = y;
}
DEV fp sqr_n(fp x, int n) {
  sqr_n_ool(x, n);
  return x;
}

// a^(p - 2), p - 2 = [519 ones][0][1] (MSB first); x_k = a^(2^k - 1)
DEV fp inv(const fp& a) {
  const fp x2 = mul(sqr(a), a);
  const fp x3 = mul(sqr(x2), a);
  const fp x4 = mul(sqr_n(x2, 2), x2);
  const fp x7 = mul(sqr_n(x4, 3), x3);
  const fp x8 = mul(sqr_n(x4, 4), x4);
  const fp x16 = mul(sqr_n(x8, 8), x8);
  const fp x32 = mul(sqr_n(x16, 16), x16);
  const fp x64 = mul(sqr_n(x32, 32), x32);
  const fp x128 = mul(sqr_n(x64, 64), x64);
  const fp x256 = mul(sqr_n(x128, 128), x128);
  const fp x512 = mul(sqr_n(x256, 256), x256);
  const fp x519 = mul(sqr_n(x512, 7), x7);
  return mul(sqr_n(x519, 2), a);
}

// canonical representative in [0, p)
DEV fp freeze(const fp& a) {
  fp r = a;
  carry(r.v);
  carry(r.v);
  carry(r.v);  // every limb in range, the value < 2^521
  // the only value in [p, 2^521) is p itself (all limbs at their maximum)
  uint32_t all = r.v[NL - 1] ^ M28;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) all |= r.v[i] ^ M29;
  if (all == 0) {
#pragma unroll
    for (int i = 0; i < NL; i++) r.v[i] = 0;
  }
  return r;
}
DEV bool is_zero(const fp& a) {
  const fp x = freeze(a);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) d |= x.v[i];
  return d == 0;
}
DEV bool eq(const fp& a, const fp& b) {
  const fp x = freeze(a), y = freeze(b);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) d |= x.v[i] ^ y.v[i];
  return d == 0;
}

// 66 big-endian bytes -> limbs; false unless the value is < p (a canonical coordinate, SEC 1
// 2.3.4 / RFC 9180 7.1.1)
DEV bool from_be(const uint8_t* b, fp& out) {
#pragma unroll
  for (int k = 0; k < NL; k++) {
    uint32_t x = 0;
    // bits 29k .. 29k + 28 live in bytes 65 - (29k + 28) / 8 .. 65 - 29k / 8
#pragma unroll
    for (int j = (29 * k) / 8; j <= (29 * k + 28) / 8 && j < 66; j++) {
      const int sh = 8 * j - 29 * k;  // byte j (from the LSB end) starts at this bit of the limb
      const uint32_t byte = b[65 - j];
      x |= sh >= 0 ? byte << sh : byte >> (-sh);
    }
    out.v[k] = x & (k == NL - 1 ? 0x1fffffffu : M29);
  }
  // canonical: bits >= 521 zero (byte 0 <= 1, limb 17 below 2^28) and not p itself
  bool ok = b[0] <= 1 && out.v[NL - 1] <= M28;
  uint32_t all = out.v[NL - 1] ^ M28;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) all |= out.v[i] ^ M29;
  return ok && all != 0;
}

// canonical value -> 66 big-endian bytes
DEV void to_be(const fp& a, uint8_t out[66]) {
  const fp f = freeze(a);
#pragma unroll
  for (int j = 0; j < 66; j++) {
    uint32_t byte = 0;
    const int bit = 8 * j;  // byte j from the LSB end holds bits 8j .. 8j + 7
#pragma unroll
    for (int k = bit / 29; k <= (bit + 7) / 29 && k < NL; k++) {
      const int sh = bit - 29 * k;
      byte |= sh >= 0 ? f.v[k] >> sh : f.v[k] << (-sh);
    }
    out[65 - j] = (uint8_t)byte;
  }
}

// the curve constant b (SEC 2 2.6.1) in 29-bit limbs
constexpr fp kB = {{0x0b503f00u, 0x1a28fea3u, 0x0b0d3c7bu, 0x07bf107au, 0x1bf07357u, 0x005e9dd8u,
                    0x0dec594bu, 0x0a3d8fd2u, 0x01561939u, 0x0c77884fu, 0x0e2d2264u, 0x13662be7u,
                    0x0da725b9u, 0x02a07751u, 0x088682dau, 0x1343f253u, 0x19618e1cu, 0x028ca9f5u}};

// the field as ecdh_a3.h reads it
struct Field {
  typedef fp T;
  static constexpr int kBytes = 66;
  DEV static T add(const T& a, const T& b) { return p521::add(a, b); }
  DEV static T sub(const T& a, const T& b) { return p521::sub(a, b); }
  DEV static T mul(const T& a, const T& b) { return p521::mul(a, b); }
  DEV static T sqr(const T& a) { return p521::sqr(a); }
  DEV static T mul_small(const T& a, uint32_t k) { return p521::mul_small(a, k); }
  DEV static T neg(const T& a) { return p521::neg(a); }
  DEV static T inv(const T& a) { return p521::inv(a); }
  DEV static bool is_zero(const T& a) { return p521::is_zero(a); }
  DEV static bool eq(const T& a, const T& b) { return p521::eq(a, b); }
  DEV static bool from_be(const uint8_t* b, T& out) { return p521::from_be(b, out); }
  DEV static void to_be(const T& a, uint8_t* out) { p521::to_be(a, out); }
  DEV static T one() {
    T r;
#pragma unroll
    for (int i = 0; i < NL; i++) r.v[i] = i ? 0u : 1u;
    return r;
  }
  DEV static T b() { return kB; }
};
// the same field with the products inlined (ecdh_a3.h's dbl4)
struct FieldInl : Field {
  DEV static T mul(const T& a, const T& b) { return p521::mul_i(a, b); }
  DEV static T sqr(const T& a) { return p521::sqr_i(a); }
};

}  // namespace p521
