// p384_device.h -- GF(p384), p = 2^384 - 2^128 - 2^96 + 2^32 - 1, for DHKEM(P-384, HKDF-SHA384)
// (RFC 9180 7.1, KEM 0x0011, messages/src/lib.rs:770-784 HpkeKemId::P384HkdfSha384), one
// report per work-item.
//
// 12 saturated 32-bit limbs in Montgomery form (R = 2^384): every value is kept in [0, p).  The
// product is product-scanning Montgomery multiplication (each limb product one v_mad_u64_u32 and
// one carry count; -p^-1 = 1 mod 2^32, so the reduction multiplier is the column's low word).  An element is 12 VGPRs, so the
// out-of-line multiply takes both operands and returns its result in argument registers (no
// scratch, unlike P-521's 18-limb elements).  The curve arithmetic is ecdh_a3.h's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace p384 {

constexpr int NL = 12;

struct fp {
  uint32_t v[NL];
};

// p, R mod p, R^2 mod p and b R mod p (b: SEC 2 2.5.1), little-endian words
constexpr uint32_t kP[NL] = {0xffffffffu, 0x00000000u, 0x00000000u, 0xffffffffu,
                             0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                             0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
constexpr fp kOne = {{0x00000001u, 0xffffffffu, 0xffffffffu, 0x00000000u, 0x00000001u, 0, 0, 0,
                      0, 0, 0, 0}};
constexpr fp kR2 = {{0x00000001u, 0xfffffffeu, 0x00000000u, 0x00000002u, 0x00000000u,
                     0xfffffffeu, 0x00000000u, 0x00000002u, 0x00000001u, 0, 0, 0}};
constexpr fp kBR = {{0x9d412dccu, 0x08118871u, 0x7a4c32ecu, 0xf729add8u, 0x1920022eu,
                     0x77f2209bu, 0x94938ae2u, 0xe3374beeu, 0x1f022094u, 0xb62b21f4u,
                     0x604fbff9u, 0xcd08114bu}};

// s (NL words) + carry-out c -> s mod p, given s + c 2^384 < 2p.  The carry chains are
// __builtin_addc / __builtin_subc (one v_add_co / v_addc / v_sub_co / v_subb each; int64
// arithmetic here compiled to 64-bit adds and moves, 155 instructions per add).
DEV fp cond_sub(const uint32_t s[NL], uint32_t c) {
  uint32_t t[NL], br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) t[i] = __builtin_subc(s[i], kP[i], br, &br);
  // s - p borrowed past the carry-out: keep s
  const bool keep_s = br > c;
  fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = keep_s ? s[i] : t[i];
  return r;
}

DEV fp add(const fp& a, const fp& b) {
  uint32_t s[NL], c = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) s[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  return cond_sub(s, c);
}

DEV fp sub(const fp& a, const fp& b) {
  uint32_t d[NL], br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) d[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  // borrow: add p back
  const uint32_t m = 0u - br;
  fp r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = __builtin_addc(d[i], kP[i] & m, c, &c);
  return r;
}

DEV fp neg(const fp& a) {
  fp z;
#pragma unroll
  for (int i = 0; i < NL; i++) z.v[i] = 0;
  return sub(z, a);
}

// a b R^-1 mod p (a, b < p) by product scanning (the FIPS form of Montgomery multiplication):
// column k accumulates a_i b_(k-i) and m_i p_(k-i) in a 96-bit register (acc + h 2^64); each
// limb product is one v_mad_u64_u32 into acc with its carry-out counted by one v_addc into h, no
// moves.  m_k = the column's low word (-p^-1 = 1 mod 2^32); p's two zero words are skipped.
// 660 instructions; LLVM's CIOS from C built every term from a v_mad_u64_u32, a 64-bit add and
// two moves (1,209): 5.12 against 6.44 M input shares/s (profiles/r05/p384/).
DEV void mac_ps(uint64_t& acc, uint32_t& h, uint32_t a, uint32_t b) {
  uint64_t c;  // the carry-out lane mask (an SGPR pair: no VCC between the statements)
  asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, 0, %2, %1"
               : "+v"(acc), "=&s"(c), "+v"(h)
               : "v"(a), "v"(b));
}
DEV fp mul_i(const fp& a, const fp& b) {
  uint64_t acc = 0;
  uint32_t h = 0, m[NL], r[NL + 1];
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int i = (k < NL ? 0 : k - NL + 1); i <= (k < NL ? k : NL - 1); i++) {
      mac_ps(acc, h, a.v[i], b.v[k - i]);
      if (i < k && kP[k - i] != 0) mac_ps(acc, h, m[i], kP[k - i]);
    }
    if (k < NL) {
      m[k] = (uint32_t)acc;
      mac_ps(acc, h, m[k], kP[0]);  // the column's low word becomes 0
    } else {
      r[k - NL] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)h << 32);
    h = 0;
  }
  r[NL - 1] = (uint32_t)acc;
  r[NL] = (uint32_t)(acc >> 32);
  return cond_sub(r, r[NL]);  // < 2p
}

// Out of line, with both operands and the result in registers: an element is 12 VGPRs, but a
// second struct argument is passed by reference through scratch, so the operands cross the call
// as 8 + 4-word vectors.
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
DEV u32x8 lo8(const fp& a) {
  return u32x8{a.v[0], a.v[1], a.v[2], a.v[3], a.v[4], a.v[5], a.v[6], a.v[7]};
}
DEV u32x4 hi4(const fp& a) { return u32x4{a.v[8], a.v[9], a.v[10], a.v[11]}; }
DEV fp join(u32x8 l, u32x4 h) {
  return fp{{l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7], h[0], h[1], h[2], h[3]}};
}
__device__ __noinline__ fp mul_v(u32x8 al, u32x4 ah, u32x8 bl, u32x4 bh) {
  return mul_i(join(al, ah), join(bl, bh));
}
__device__ __noinline__ fp sqr_v(u32x8 al, u32x4 ah) {
  const fp a = join(al, ah);
  return mul_i(a, a);
}
DEV fp mul(const fp& a, const fp& b) { return mul_v(lo8(a), hi4(a), lo8(b), hi4(b)); }
DEV fp sqr(const fp& a) { return sqr_v(lo8(a), hi4(a)); }

DEV fp mul_small(const fp& a, uint32_t k) {  // k in {3, 4, 8} (ecdh_a3.h) or any small k
  fp r = a;
  bool first = true;
  fp acc;
#pragma unroll 1
  for (uint32_t kk = k; kk; kk >>= 1) {
    if (kk & 1u) {
      acc = first ? r : add(acc, r);
      first = false;
    }
    if (kk > 1) r = add(r, r);
  }
  return acc;
}

DEV fp sqr_n(fp x, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) x = sqr(x);
  return x;
}

// a^(p - 2): p - 2 = [255 ones][0][32 ones][64 zeros][30 ones][0][1] (MSB first);
// x_k = a^(2^k - 1)
DEV fp inv(const fp& a) {
  const fp x2 = mul(sqr(a), a);
  const fp x3 = mul(sqr(x2), a);
  const fp x6 = mul(sqr_n(x3, 3), x3);
  const fp x12 = mul(sqr_n(x6, 6), x6);
  const fp x15 = mul(sqr_n(x12, 3), x3);
  const fp x30 = mul(sqr_n(x15, 15), x15);
  const fp x32 = mul(sqr_n(x30, 2), x2);
  const fp x60 = mul(sqr_n(x30, 30), x30);
  const fp x120 = mul(sqr_n(x60, 60), x60);
  const fp x240 = mul(sqr_n(x120, 120), x120);
  const fp x255 = mul(sqr_n(x240, 15), x15);
  fp t = mul(sqr_n(x255, 33), x32);  // [255 ones][0][32 ones]
  t = mul(sqr_n(t, 94), x30);         // [64 zeros][30 ones]
  return mul(sqr_n(t, 2), a);         // [0][1]
}

DEV bool is_zero(const fp& a) {
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) d |= a.v[i];
  return d == 0;
}
DEV bool eq(const fp& a, const fp& b) {
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) d |= a.v[i] ^ b.v[i];
  return d == 0;
}

// 48 big-endian bytes -> Montgomery form; false unless the value is < p (SEC 1 2.3.4)
DEV bool from_be(const uint8_t* b, fp& out) {
  fp x;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    const uint8_t* q = b + 4 * (NL - 1 - k);
    x.v[k] = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  }
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) br = ((int64_t)x.v[i] - kP[i] + br) >> 32;
  out = mul_i(x, kR2);
  return br != 0;  // x - p borrowed: x < p
}

// Montgomery form -> 48 big-endian bytes of the canonical value
DEV void to_be(const fp& a, uint8_t out[48]) {
  fp one;
#pragma unroll
  for (int i = 0; i < NL; i++) one.v[i] = i ? 0u : 1u;
  const fp x = mul_i(a, one);
#pragma unroll
  for (int k = 0; k < NL; k++) {
    uint8_t* q = out + 4 * (NL - 1 - k);
    q[0] = (uint8_t)(x.v[k] >> 24), q[1] = (uint8_t)(x.v[k] >> 16), q[2] = (uint8_t)(x.v[k] >> 8),
    q[3] = (uint8_t)x.v[k];
  }
}

// the field as ecdh_a3.h reads it
struct Field {
  typedef fp T;
  static constexpr int kBytes = 48;
  DEV static T add(const T& a, const T& b) { return p384::add(a, b); }
  DEV static T sub(const T& a, const T& b) { return p384::sub(a, b); }
  DEV static T mul(const T& a, const T& b) { return p384::mul(a, b); }
  DEV static T sqr(const T& a) { return p384::sqr(a); }
  DEV static T mul_small(const T& a, uint32_t k) { return p384::mul_small(a, k); }
  DEV static T neg(const T& a) { return p384::neg(a); }
  DEV static T inv(const T& a) { return p384::inv(a); }
  DEV static bool is_zero(const T& a) { return p384::is_zero(a); }
  DEV static bool eq(const T& a, const T& b) { return p384::eq(a, b); }
  DEV static bool from_be(const uint8_t* b, T& out) { return p384::from_be(b, out); }
  DEV static void to_be(const T& a, uint8_t* out) { p384::to_be(a, out); }
  DEV static T one() { return kOne; }
  DEV static T b() { return kBR; }
};

}  // namespace p384
