// p256_device.h -- NIST P-256 (FIPS 186-4 D.1.2.3, SEC 2) ECDH for DHKEM(P-256, HKDF-SHA256)
// (RFC 9180 7.1), one report per work-item on MI355X (gfx950).  Used by the HPKE opener
// (hpke.hip, KEM 0x0010).
//
// GF(p), p = 2^256 - 2^224 + 2^192 + 2^96 - 1: 8 little-endian 32-bit limbs, values loosely
// reduced in [0, 2^256).  A product is the 16-word schoolbook (v_mad_u64_u32) folded by the
// NIST fast reduction (FIPS 186-4 D.2.3: s1 + 2 s2 + 2 s3 + s4 + s5 - s6 - s7 - s8 - s9) in
// signed 64-bit word sums, whose carry out of 2^256 folds back as 2^256 = 2^224 - 2^192 - 2^96 + 1
// (mod p); three carry passes always leave [0, 2^256).
// The scalar is the server's private key, the same in every lane: a fixed signed window (w = 4)
// over its host-side recoding, so every key runs the same instruction stream (see ecdh).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif
#ifndef P256_ASM
#define P256_ASM 1  // 1: the generated single-asm-statement products (p256_asm.h)
#endif
namespace p256 {

struct fp {
  uint32_t v[8];
};

#if P256_ASM
#include "p256_asm.h"  // p256_mul / sqr / add / sub / mul_small (generated: tools/gen_p256_asm.py)
#endif

// carry-propagate signed word sums t[0..7] (each |t| < 2^40) into [0, 2^256), folding the
// carry out of 2^256 twice (the second carry is in {-1, 0, 1}, the third always 0)
DEV fp fold(int64_t t[8]) {
#pragma unroll
  for (int pass = 0; pass < 3; pass++) {
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      t[i] += c;
      c = t[i] >> 32;  // arithmetic shift: floor division
      t[i] &= 0xffffffffll;
    }
    if (pass < 2) {
      t[0] += c;
      t[3] -= c;
      t[6] -= c;
      t[7] += c;
    }
  }
  fp r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = (uint32_t)t[i];
  return r;
}

#if P256_ASM
DEV fp add(const fp& a, const fp& b) { return p256_add(a, b); }
DEV fp sub(const fp& a, const fp& b) { return p256_sub(a, b); }
DEV fp mul_small(const fp& a, uint32_t k) { return p256_mul_small(a, k); }  // k <= 8
DEV fp mul(const fp& a, const fp& b) { return p256_mul(a, b); }
DEV fp sqr(const fp& a) { return p256_sqr(a); }
#else
DEV fp add(const fp& a, const fp& b) {
  int64_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = (int64_t)a.v[i] + b.v[i];
  return fold(t);
}
DEV fp sub(const fp& a, const fp& b) {
  int64_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = (int64_t)a.v[i] - b.v[i];
  return fold(t);
}
DEV fp mul_small(const fp& a, uint32_t k) {  // k <= 8
  int64_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = (int64_t)a.v[i] * k;
  return fold(t);
}

// NIST fast reduction of a 512-bit product c[0..15] (FIPS 186-4 D.2.3 as signed word sums)
DEV fp reduce(const uint32_t c[16]) {
  typedef int64_t s;
  int64_t t[8];
  t[0] = (s)c[0] + c[8] + c[9] - (s)c[11] - c[12] - c[13] - c[14];
  t[1] = (s)c[1] + c[9] + c[10] - (s)c[12] - c[13] - c[14] - c[15];
  t[2] = (s)c[2] + c[10] + c[11] - (s)c[13] - c[14] - c[15];
  t[3] = (s)c[3] + 2 * (s)c[11] + 2 * (s)c[12] + c[13] - (s)c[15] - c[8] - c[9];
  t[4] = (s)c[4] + 2 * (s)c[12] + 2 * (s)c[13] + c[14] - (s)c[9] - c[10];
  t[5] = (s)c[5] + 2 * (s)c[13] + 2 * (s)c[14] + c[15] - (s)c[10] - c[11];
  t[6] = (s)c[6] + 3 * (s)c[14] + 2 * (s)c[15] + c[13] - (s)c[8] - c[9];
  t[7] = (s)c[7] + 3 * (s)c[15] + c[8] - (s)c[10] - c[11] - c[12] - c[13];
  return fold(t);
}

__device__ __noinline__ fp mul(const fp& a, const fp& b) {
  uint32_t c[16];
#pragma unroll
  for (int i = 0; i < 16; i++) c[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t x = (uint64_t)a.v[i] * b.v[j] + c[i + j] + carry;
      c[i + j] = (uint32_t)x;
      carry = x >> 32;
    }
    c[i + 8] = (uint32_t)carry;
  }
  return reduce(c);
}
__device__ __noinline__ fp sqr(const fp& a) { return mul(a, a); }
#endif  // P256_ASM

// canonical representative in [0, p)
DEV fp freeze(const fp& a) {
  constexpr uint32_t P[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 1u, 0xffffffffu};
  fp d;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int64_t x = (int64_t)a.v[i] - P[i] + br;
    d.v[i] = (uint32_t)x;
    br = x >> 32;  // 0 or -1
  }
  const bool ge = br == 0;  // a >= p
  fp r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = ge ? d.v[i] : a.v[i];
  return r;
}
DEV bool eq(const fp& a, const fp& b) {
  const fp x = freeze(a), y = freeze(b);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d |= x.v[i] ^ y.v[i];
  return d == 0;
}
DEV bool is_zero(const fp& a) {
  const fp x = freeze(a);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d |= x.v[i];
  return d == 0;
}

// a^(p - 2) by an addition chain: p - 2 = [32 ones][31 zeros][1][96 zeros][94 ones][0][1]
// (MSB first); x_k = a^(2^k - 1).  255 squarings + 12 multiplies (the bit loop took 128).
DEV fp sqr_n(fp x, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) x = sqr(x);
  return x;
}
DEV fp inv(const fp& a) {
  const fp x2 = mul(sqr(a), a);
  const fp x3 = mul(sqr(x2), a);
  const fp x6 = mul(sqr_n(x3, 3), x3);
  const fp x12 = mul(sqr_n(x6, 6), x6);
  const fp x15 = mul(sqr_n(x12, 3), x3);
  const fp x30 = mul(sqr_n(x15, 15), x15);
  const fp x32 = mul(sqr_n(x30, 2), x2);
  fp t = mul(sqr_n(x32, 32), a);   // [32 ones][31 zeros][1]
  t = sqr_n(t, 96);                // [96 zeros]
  t = mul(sqr_n(t, 32), x32);      // [32 ones]
  t = mul(sqr_n(t, 32), x32);      // [32 ones]
  t = mul(sqr_n(t, 30), x30);      // [30 ones]
  return mul(sqr_n(t, 2), a);      // [0][1]
}

// 32 big-endian bytes -> limbs; false if the value is >= p (a non-canonical coordinate)
DEV bool from_be(const uint8_t* b, fp& out) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = b + 4 * (7 - i);
    out.v[i] = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  }
  const fp f = freeze(out);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d |= f.v[i] ^ out.v[i];
  return d == 0;
}

struct jac {
  fp X, Y, Z;
};

// dbl-2001-b (a = -3): delta = Z^2, gamma = Y^2, beta = X gamma, alpha = 3 (X - delta)(X + delta);
// Z3 = 2 Y Z (one multiply and one add instead of (Y + Z)^2 - gamma - delta: 284 instructions
// against 314 with the generated field routines) and 8 beta = 4 beta + 4 beta
DEV jac dbl(const jac& P) {
  const fp delta = sqr(P.Z), gamma = sqr(P.Y), beta = mul(P.X, gamma);
  const fp alpha = mul_small(mul(sub(P.X, delta), add(P.X, delta)), 3);
  const fp b4 = mul_small(beta, 4);
  jac R;
  R.X = sub(sqr(alpha), add(b4, b4));
  const fp yz = mul(P.Y, P.Z);
  R.Z = add(yz, yz);
  R.Y = sub(mul(alpha, sub(b4, R.X)), mul_small(sqr(gamma), 8));
  return R;
}

// madd-2007-bl: P (Jacobian) + (x2, y2) (affine), P != +-(x2, y2), P not at infinity; doublings
// as additions and Z3 = 2 Z1 H (as in dbl)
DEV jac madd(const jac& P, const fp& x2, const fp& y2) {
  const fp Z1Z1 = sqr(P.Z);
  const fp U2 = mul(x2, Z1Z1), S2 = mul(y2, mul(P.Z, Z1Z1));
  const fp H = sub(U2, P.X), HH = sqr(H);
  const fp I = mul_small(HH, 4), J = mul(H, I);
  const fp s = sub(S2, P.Y), rr = add(s, s), V = mul(P.X, I);
  jac R;
  R.X = sub(sub(sqr(rr), J), add(V, V));
  const fp yj = mul(P.Y, J);
  R.Y = sub(mul(rr, sub(V, R.X)), add(yj, yj));
  const fp zh = mul(P.Z, H);
  R.Z = add(zh, zh);
  return R;
}

DEV fp neg(const fp& a) { return sub(fp{{0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}}, a); }

// Digits of the regular signed window recoding (w = 4) of the private key, computed on the host
// (hpke.hip p256_recode): k' = sk if sk is odd, else n - sk (x(k'P) = x(-sk P) = x(sk P)), and
// k' = sum_i d_i 16^i with every d_i odd in [-15, 15], d_63 odd in [1, 15].
constexpr int kDigits = 64;

// DH(sk, pkE) for an uncompressed SEC1 point enc = 0x04 || X || Y (65 bytes): validates the
// point (prefix, canonical coordinates, y^2 = x^3 - 3x + b) and writes the shared x-coordinate
// as 8 big-endian words (its 32-byte encoding, RFC 9180 7.1.1).
// Fixed window over the recoded key: a table of P, 3P, .., 15P (affine, one shared inversion by
// Montgomery's trick), then 63 x (four doublings + one mixed addition of +-table[|d|]): 252
// doublings and 63 additions, where w = 3 took 255 and 85 (r03: -4.5 % of the kernel's
// instructions for 23 more operations in the table).  The digits are the same in every lane
// (one server key), so every key runs the same instruction stream and the table is read at a
// wave-uniform index from the lane's private memory (64 bytes per window).
// The additions never meet the doubling case R = +-T except, for k' in {n - 2, n - 6, .., n - 30},
// at the last window (16 k_1 = k' - d_0 = d_0 mod n); there madd returns Z = 0 and the doubled R,
// computed beside it for every key, is the sum.
DEV bool ecdh(const int8_t* dig, const uint8_t* enc, uint32_t dh_be[8]) {
  constexpr fp B = {{0x27d2604bu, 0x3bce3c3eu, 0xcc53b0f6u, 0x651d06b0u, 0x769886bcu, 0xb3ebbd55u,
                     0xaa3a93e7u, 0x5ac635d8u}};
  constexpr fp ONE = {{1u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}};
  fp x, y;
  bool ok = enc[0] == 0x04;
  ok = from_be(enc + 1, x) && ok;
  ok = from_be(enc + 33, y) && ok;
  const fp rhs = add(sub(mul(sqr(x), x), mul_small(x, 3)), B);
  ok = ok && eq(sqr(y), rhs);
  // odd multiples (2i+1)P, i = 1..7, in Jacobian coordinates: 6 doublings and 7 mixed additions
  //   3P = 2P + P, 5P = 4P + P, 7P = 8P - P, 9P = 8P + P, 11P = 12P - P, 13P = 12P + P,
  //   15P = 16P - P, with 4P = 2(2P), 8P = 2(4P), 12P = 2(2(3P)), 16P = 2(8P).
  // tab / zz / pz are indexed by runtime values below, so they live in the lane's private memory
  // and the points leave registers as soon as they are made.
  fp tab[8][2];  // affine (x, y) of (2i+1)P; Jacobian X, Y until the inversion
  fp zz[8], pz[8];  // Z of (2i+1)P; prefix products Z_1 .. Z_i
  tab[0][0] = x;
  tab[0][1] = y;
  {
    const fp ny = neg(y);
    auto put = [&](int k, const jac& T) {
      tab[k][0] = T.X;
      tab[k][1] = T.Y;
      zz[k] = T.Z;
    };
    const jac P2 = dbl(jac{x, y, ONE});
    const jac P3 = madd(P2, x, y);
    put(1, P3);
    const jac P12 = dbl(dbl(P3));
    put(5, madd(P12, x, ny));  // 11P
    put(6, madd(P12, x, y));   // 13P
    const jac P4 = dbl(P2);
    put(2, madd(P4, x, y));    // 5P
    const jac P8 = dbl(P4);
    put(3, madd(P8, x, ny));   // 7P
    put(4, madd(P8, x, y));    // 9P
    put(7, madd(dbl(P8), x, ny));  // 15P
  }
  {  // Montgomery's trick: one inversion for the seven Z
    fp acc = zz[1];
    pz[1] = acc;
#pragma unroll 1
    for (int k = 2; k < 8; k++) {
      acc = mul(acc, zz[k]);
      pz[k] = acc;
    }
    fp ia = inv(acc);  // 1 / (Z_1 .. Z_k) for the k of the next step
#pragma unroll 1
    for (int k = 7; k >= 1; k--) {
      fp zi = ia;  // 1 / Z_k
      if (k > 1) {  // wave-uniform
        zi = mul(ia, pz[k - 1]);
        ia = mul(ia, zz[k]);
      }
      const fp zi2 = sqr(zi);
      tab[k][0] = mul(tab[k][0], zi2);
      tab[k][1] = mul(tab[k][1], mul(zi2, zi));
    }
  }
  auto pick = [&](int d, fp& tx, fp& ty) {
    const int a = (d < 0 ? -d : d) >> 1;
    tx = tab[a][0];
    ty = tab[a][1];
    const fp ny = neg(ty);
    if (d < 0) ty = ny;
  };
  jac R;
  pick(dig[kDigits - 1], R.X, R.Y);
  R.Z = ONE;
  // one doubling and one addition in the loop body (the inlined asm field operations make each
  // ~3k instructions; four unrolled doublings would not fit the instruction cache)
#pragma unroll 1
  for (int i = kDigits - 2; i >= 1; i--) {
#pragma unroll 1
    for (int j = 0; j < 4; j++) R = dbl(R);
    fp tx, ty;
    pick(dig[i], tx, ty);
    R = madd(R, tx, ty);
  }
#pragma unroll 1
  for (int j = 0; j < 4; j++) R = dbl(R);
  {
    fp tx, ty;
    pick(dig[0], tx, ty);
    const jac D = dbl(R);
    const jac S = madd(R, tx, ty);
    R = is_zero(S.Z) ? D : S;
  }
  ok = ok && !is_zero(R.Z);
  const fp zi = inv(R.Z);
  const fp ax = freeze(mul(R.X, sqr(zi)));
#pragma unroll
  for (int i = 0; i < 8; i++) dh_be[i] = ax.v[7 - i];
  return ok;
}

}  // namespace p256
