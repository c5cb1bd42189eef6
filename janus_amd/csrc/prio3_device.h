// prio3_device.h -- gfx950 device arithmetic for the batched Prio3 engine.
//
//  * Field128 (p = 2^128 - 28*2^64 + 1) and Field64 (p = 2^64 - 2^32 + 1) modular arithmetic
//    on 32-bit VALU limbs (v_mad_u64_u32 products, add/sub carry chains, special-form
//    reduction; no Montgomery form, so encodings are the canonical LE bytes prio puts on
//    the wire [prio field.rs FieldElement::encode]).
//  * Keccak-p[1600,12] (TurboSHAKE128 core, RFC 9861) with the 25 lanes held as 50 VGPRs
//    per work-item (lo/hi halves), v_bitop3_b32 three-input XORs and v_alignbit_b32 rotates.
//
// No MFMA anywhere: nothing on this path is a dense contraction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

// -------------------------------------------------------------------------------------
// Field128
// -------------------------------------------------------------------------------------
struct f128 {
  uint32_t w[4];
};

DEV f128 mk128(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  f128 r;
  r.w[0] = a;
  r.w[1] = b;
  r.w[2] = c;
  r.w[3] = d;
  return r;
}
DEV f128 zero128() { return mk128(0, 0, 0, 0); }
// element-wise select (a struct-valued ?: can be lowered through private memory)
DEV f128 sel128(bool c, const f128& a, const f128& b) {
  return mk128(c ? a.w[0] : b.w[0], c ? a.w[1] : b.w[1], c ? a.w[2] : b.w[2], c ? a.w[3] : b.w[3]);
}
DEV f128 one128() { return mk128(1, 0, 0, 0); }
DEV bool is_zero128(const f128& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0; }
DEV bool eq128(const f128& a, const f128& b) {
  return ((a.w[0] ^ b.w[0]) | (a.w[1] ^ b.w[1]) | (a.w[2] ^ b.w[2]) | (a.w[3] ^ b.w[3])) == 0;
}

#define P128_0 1u
#define P128_1 0u
#define P128_2 0xffffffe4u
#define P128_3 0xffffffffu

DEV uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  return __builtin_addc(a, b, cin, cout);
}
DEV uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  return __builtin_subc(a, b, bin, bout);
}

// x >= p ?
DEV bool ge_p128(const f128& x) {
  uint32_t b0, b1, b2, b3;
  subb(x.w[0], P128_0, 0, &b0);
  subb(x.w[1], P128_1, b0, &b1);
  subb(x.w[2], P128_2, b1, &b2);
  subb(x.w[3], P128_3, b2, &b3);
  return b3 == 0;
}

// Reduce a value known to be < 2^128 into [0, p).
DEV f128 canon128(const f128& x) {
  uint32_t b0, b1, b2, b3;
  f128 d;
  d.w[0] = subb(x.w[0], P128_0, 0, &b0);
  d.w[1] = subb(x.w[1], P128_1, b0, &b1);
  d.w[2] = subb(x.w[2], P128_2, b1, &b2);
  d.w[3] = subb(x.w[3], P128_3, b2, &b3);
  return sel128(b3 != 0, x, d);
}

DEV f128 add128(const f128& a, const f128& b) {
  uint32_t c0, c1, c2, c3, b0, b1, b2, b3;
  f128 s, d;
  s.w[0] = addc(a.w[0], b.w[0], 0, &c0);
  s.w[1] = addc(a.w[1], b.w[1], c0, &c1);
  s.w[2] = addc(a.w[2], b.w[2], c1, &c2);
  s.w[3] = addc(a.w[3], b.w[3], c2, &c3);
  d.w[0] = subb(s.w[0], P128_0, 0, &b0);
  d.w[1] = subb(s.w[1], P128_1, b0, &b1);
  d.w[2] = subb(s.w[2], P128_2, b1, &b2);
  d.w[3] = subb(s.w[3], P128_3, b2, &b3);
  bool use_d = c3 | (b3 ^ 1u);
  return sel128(use_d, d, s);
}

DEV f128 sub128(const f128& a, const f128& b) {
  uint32_t b0, b1, b2, b3, c0, c1, c2, c3;
  f128 d;
  d.w[0] = subb(a.w[0], b.w[0], 0, &b0);
  d.w[1] = subb(a.w[1], b.w[1], b0, &b1);
  d.w[2] = subb(a.w[2], b.w[2], b1, &b2);
  d.w[3] = subb(a.w[3], b.w[3], b2, &b3);
  uint32_t m = 0u - b3;  // all-ones if borrow
  d.w[0] = addc(d.w[0], P128_0 & m, 0, &c0);
  d.w[1] = addc(d.w[1], P128_1 & m, c0, &c1);
  d.w[2] = addc(d.w[2], P128_2 & m, c1, &c2);
  d.w[3] = addc(d.w[3], P128_3 & m, c2, &c3);
  return d;
}

DEV f128 neg128(const f128& a) { return sub128(zero128(), a); }

// a*b mod p.  Product by schoolbook v_mad_u64_u32; reduction uses
//   2^128 == 28*2^64 - 1,  2^192 == 783*2^64 - 28  (mod p).
DEV f128 mul128(const f128& a, const f128& b) {
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint64_t t = (uint64_t)a.w[i] * b.w[j] + (uint64_t)r[i + j] + carry;
      r[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    r[i + 4] = (uint32_t)carry;
  }
  // X = x3*2^192 + x2*2^128 + x1*2^64 + x0  (x_k = 64-bit words)
  // S = x1 + 28*x2 + 783*x3 = s1*2^64 + (s_1:s_0)
  uint64_t t0 = (uint64_t)r[2] + (uint64_t)r[4] * 28u + (uint64_t)r[6] * 783u;
  uint32_t s_0 = (uint32_t)t0;
  uint64_t t1 = (uint64_t)r[3] + (uint64_t)r[5] * 28u + (uint64_t)r[7] * 783u + (t0 >> 32);
  uint32_t s_1 = (uint32_t)t1;
  uint32_t s1 = (uint32_t)(t1 >> 32);  // < 2^11
  // u = (s_1:s_0) + 28*s1, carry c into 2^128
  uint64_t u = ((uint64_t)s_1 << 32 | s_0) + (uint64_t)s1 * 28u;
  uint32_t c = u < (uint64_t)s1 * 28u ? 1u : 0u;
  // N = x2 + 28*x3 + s1  (< 2^70)
  uint64_t n0 = (uint64_t)r[4] + (uint64_t)r[6] * 28u + s1;
  uint64_t n1 = (uint64_t)r[5] + (uint64_t)r[7] * 28u + (n0 >> 32);
  // A = x0 + u*2^64 + c*(28*2^64 - 1)
  uint32_t m = 0u - c, c0, c1, c2, c3;
  f128 A;
  A.w[0] = addc(r[0], m, 0, &c0);
  A.w[1] = addc(r[1], m, c0, &c1);
  A.w[2] = addc((uint32_t)u, 27u & m, c1, &c2);
  A.w[3] = addc((uint32_t)(u >> 32), 0, c2, &c3);
  m = 0u - c3;  // second fold (cannot overflow again)
  A.w[0] = addc(A.w[0], m, 0, &c0);
  A.w[1] = addc(A.w[1], m, c0, &c1);
  A.w[2] = addc(A.w[2], 27u & m, c1, &c2);
  A.w[3] = addc(A.w[3], 0, c2, &c3);
  // A - N
  uint32_t b0, b1, b2, b3;
  A.w[0] = subb(A.w[0], (uint32_t)n0, 0, &b0);
  A.w[1] = subb(A.w[1], (uint32_t)n1, b0, &b1);
  A.w[2] = subb(A.w[2], (uint32_t)(n1 >> 32), b1, &b2);
  A.w[3] = subb(A.w[3], 0, b2, &b3);
  m = 0u - b3;
  A.w[0] = addc(A.w[0], P128_0 & m, 0, &c0);
  A.w[1] = addc(A.w[1], P128_1 & m, c0, &c1);
  A.w[2] = addc(A.w[2], P128_2 & m, c1, &c2);
  A.w[3] = addc(A.w[3], P128_3 & m, c2, &c3);
  return canon128(A);
}

// -------------------------------------------------------------------------------------
// Lazily reduced multiply-accumulate: sum of Field128 products kept as 7 product-scanning
// columns (column k = c[k] + h[k]*2^64, weight 2^(32k)); each 32x32 limb product is ONE
// v_mad_u64_u32 (carry-out to VCC) plus ONE v_addc into the column's top word -- no per-product
// modular reduction.  Up to 2^31 products fit; mac_reduce() folds the result once.
// -------------------------------------------------------------------------------------
struct mac128 {
  uint64_t c[7];
  uint32_t h[7];
};
DEV void mac_zero(mac128& a) {
#pragma unroll
  for (int k = 0; k < 7; k++) {
    a.c[k] = 0;
    a.h[k] = 0;
  }
}
// One asm statement for all 16 limb products: the compiler's hazard recogniser treats every
// inline-asm boundary that writes VCC conservatively and pads it with s_nop, so splitting the
// products into 16 statements cost ~1 s_nop per product (seen in the gfx950 assembly).
DEV void mac_add(mac128& a, const f128& x, const f128& y) {
  asm(
      "v_mad_u64_u32 %0, vcc, %14, %18, %0\n\t"
      "v_addc_co_u32 %7, vcc, 0, %7, vcc\n\t"
      "v_mad_u64_u32 %1, vcc, %14, %19, %1\n\t"
      "v_addc_co_u32 %8, vcc, 0, %8, vcc\n\t"
      "v_mad_u64_u32 %2, vcc, %14, %20, %2\n\t"
      "v_addc_co_u32 %9, vcc, 0, %9, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %14, %21, %3\n\t"
      "v_addc_co_u32 %10, vcc, 0, %10, vcc\n\t"
      "v_mad_u64_u32 %1, vcc, %15, %18, %1\n\t"
      "v_addc_co_u32 %8, vcc, 0, %8, vcc\n\t"
      "v_mad_u64_u32 %2, vcc, %15, %19, %2\n\t"
      "v_addc_co_u32 %9, vcc, 0, %9, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %15, %20, %3\n\t"
      "v_addc_co_u32 %10, vcc, 0, %10, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %15, %21, %4\n\t"
      "v_addc_co_u32 %11, vcc, 0, %11, vcc\n\t"
      "v_mad_u64_u32 %2, vcc, %16, %18, %2\n\t"
      "v_addc_co_u32 %9, vcc, 0, %9, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %16, %19, %3\n\t"
      "v_addc_co_u32 %10, vcc, 0, %10, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %16, %20, %4\n\t"
      "v_addc_co_u32 %11, vcc, 0, %11, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %16, %21, %5\n\t"
      "v_addc_co_u32 %12, vcc, 0, %12, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %17, %18, %3\n\t"
      "v_addc_co_u32 %10, vcc, 0, %10, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %17, %19, %4\n\t"
      "v_addc_co_u32 %11, vcc, 0, %11, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %17, %20, %5\n\t"
      "v_addc_co_u32 %12, vcc, 0, %12, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %17, %21, %6\n\t"
      "v_addc_co_u32 %13, vcc, 0, %13, vcc\n\t"
      : "+v"(a.c[0]), "+v"(a.c[1]), "+v"(a.c[2]), "+v"(a.c[3]), "+v"(a.c[4]), "+v"(a.c[5]),
        "+v"(a.c[6]), "+v"(a.h[0]), "+v"(a.h[1]), "+v"(a.h[2]), "+v"(a.h[3]), "+v"(a.h[4]),
        "+v"(a.h[5]), "+v"(a.h[6])
      : "v"(x.w[0]), "v"(x.w[1]), "v"(x.w[2]), "v"(x.w[3]), "v"(y.w[0]), "v"(y.w[1]),
        "v"(y.w[2]), "v"(y.w[3])
      : "vcc");
}
// 2^128 mod p and 2^256 mod p
DEV f128 mac_reduce(const mac128& a) {
  // normalise columns into 10 words: word n = lo32(c_n) + hi32(c_(n-1)) + h_(n-2) + carry
  uint32_t w[10];
  uint64_t carry = 0;
#pragma unroll
  for (int n = 0; n < 10; n++) {
    uint64_t s = carry;
    if (n < 7) s += (uint32_t)a.c[n];
    if (n >= 1 && n - 1 < 7) s += (uint32_t)(a.c[n - 1] >> 32);
    if (n >= 2 && n - 2 < 7) s += a.h[n - 2];
    w[n] = (uint32_t)s;
    carry = s >> 32;
  }
  // X = L + H*2^128 + T*2^256,  2^128 = 28*2^64 - 1,  2^256 = (2^128)^2 (mod p)
  const f128 L = canon128(mk128(w[0], w[1], w[2], w[3]));
  const f128 H = mk128(w[4], w[5], w[6], w[7]);
  const f128 T = mk128(w[8], w[9], 0, 0);
  const f128 c128 = mk128(0xffffffffu, 0xffffffffu, 27u, 0u);
  const f128 c256 = mul128(c128, c128);
  return add128(add128(L, mul128(canon128(H), c128)), mul128(T, c256));
}
// lazily reduced sum of Field128 values (128-bit sum + 32-bit carry word)
struct sum128 {
  uint32_t w[5];
};
DEV void sum_zero(sum128& s) {
#pragma unroll
  for (int k = 0; k < 5; k++) s.w[k] = 0;
}
DEV void sum_add(sum128& s, const f128& x) {
  uint32_t c0, c1, c2, c3;
  s.w[0] = addc(s.w[0], x.w[0], 0, &c0);
  s.w[1] = addc(s.w[1], x.w[1], c0, &c1);
  s.w[2] = addc(s.w[2], x.w[2], c1, &c2);
  s.w[3] = addc(s.w[3], x.w[3], c2, &c3);
  s.w[4] += c3;
}
DEV f128 sum_reduce(const sum128& s) {
  const f128 c128 = mk128(0xffffffffu, 0xffffffffu, 27u, 0u);
  return add128(canon128(mk128(s.w[0], s.w[1], s.w[2], s.w[3])),
                mul128(mk128(s.w[4], 0, 0, 0), c128));
}

// -------------------------------------------------------------------------------------
// Field64 (Goldilocks)
// -------------------------------------------------------------------------------------
#define P64 0xffffffff00000001ull
DEV uint64_t add64f(uint64_t a, uint64_t b) {
  uint64_t s = a + b;
  uint64_t d = s - P64;
  bool ovf = s < a;
  return (ovf || s >= P64) ? d : s;
}
DEV uint64_t sub64f(uint64_t a, uint64_t b) {
  uint64_t d = a - b;
  return a < b ? d + P64 : d;
}
DEV uint64_t mul64f(uint64_t a, uint64_t b) {
  uint64_t lo = a * b, hi = __umul64hi(a, b);
  uint64_t hh = hi >> 32, hl = hi & 0xffffffffull;
  uint64_t t0 = lo - hh;
  if (lo < hh) t0 -= 0xffffffffull;
  uint64_t t1 = hl * 0xffffffffull;
  uint64_t r = t0 + t1;
  if (r < t0) r += 0xffffffffull;
  if (r >= P64) r -= P64;
  return r;
}

// -------------------------------------------------------------------------------------
// Generic field traits so kernels can be templated on the field.
// -------------------------------------------------------------------------------------
struct Fp128 {
  typedef f128 T;
  static constexpr int ES = 16;
  static DEV T zero() { return zero128(); }
  static DEV T one() { return one128(); }
  static DEV T add(const T& a, const T& b) { return add128(a, b); }
  static DEV T sub(const T& a, const T& b) { return sub128(a, b); }
  static DEV T mul(const T& a, const T& b) { return mul128(a, b); }
  static DEV bool eq(const T& a, const T& b) { return eq128(a, b); }
  static DEV bool is_zero(const T& a) { return is_zero128(a); }
  static DEV bool lt_p(const T& a) { return !ge_p128(a); }
  static DEV T sel(bool c, const T& a, const T& b) { return sel128(c, a, b); }
  static DEV T from_words(const uint32_t* w) { return mk128(w[0], w[1], w[2], w[3]); }
  static DEV T from_u32(uint32_t x) { return mk128(x, 0, 0, 0); }
  static DEV T load(const void* base, size_t idx) {
    uint4 v = ((const uint4*)base)[idx];
    return mk128(v.x, v.y, v.z, v.w);
  }
  static DEV void store(void* base, size_t idx, const T& a) {
    ((uint4*)base)[idx] = make_uint4(a.w[0], a.w[1], a.w[2], a.w[3]);
  }
};

struct Fp64 {
  typedef uint64_t T;
  static constexpr int ES = 8;
  static DEV T zero() { return 0; }
  static DEV T one() { return 1; }
  static DEV T add(T a, T b) { return add64f(a, b); }
  static DEV T sub(T a, T b) { return sub64f(a, b); }
  static DEV T mul(T a, T b) { return mul64f(a, b); }
  static DEV bool eq(T a, T b) { return a == b; }
  static DEV bool is_zero(T a) { return a == 0; }
  static DEV bool lt_p(T a) { return a < P64; }
  static DEV T sel(bool c, T a, T b) { return c ? a : b; }
  static DEV T from_words(const uint32_t* w) { return (uint64_t)w[1] << 32 | w[0]; }
  static DEV T from_u32(uint32_t x) { return x; }
  static DEV T load(const void* base, size_t idx) { return ((const uint64_t*)base)[idx]; }
  static DEV void store(void* base, size_t idx, T a) { ((uint64_t*)base)[idx] = a; }
};

template <class F>
DEV typename F::T fpow(typename F::T a, uint32_t e) {
  typename F::T r = F::one();
  while (e) {
    if (e & 1) r = F::mul(r, a);
    a = F::mul(a, a);
    e >>= 1;
  }
  return r;
}

// -------------------------------------------------------------------------------------
// Keccak-p[1600, 12] on registers.  Lane i = (lo[i], hi[i]); state word w (0..49) is
// (w & 1 ? hi : lo)[w >> 1], i.e. little-endian byte order of the sponge.
// -------------------------------------------------------------------------------------
__constant__ static const uint32_t KRC_LO[12] = {0x8000808Bu, 0x0000008Bu, 0x00008089u, 0x00008003u,
                                          0x00008002u, 0x00000080u, 0x0000800Au, 0x8000000Au,
                                          0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
__constant__ static const uint32_t KRC_HI[12] = {0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u,
                                          0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u,
                                          0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};

DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// rotate-left of the 64-bit lane (lo, hi) by N (compile-time).
template <int N>
DEV void rotl64(uint32_t& lo, uint32_t& hi) {
  if constexpr (N == 0) {
    return;
  } else if constexpr (N == 32) {
    uint32_t t = lo;
    lo = hi;
    hi = t;
  } else if constexpr (N < 32) {
    uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - N);
    uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - N);
    lo = nlo;
    hi = nhi;
  } else {
    uint32_t nlo = __builtin_amdgcn_alignbit(hi, lo, 64 - N);
    uint32_t nhi = __builtin_amdgcn_alignbit(lo, hi, 64 - N);
    lo = nlo;
    hi = nhi;
  }
}

struct KState {
  uint32_t lo[25], hi[25];
};

DEV void kzero(KState& s) {
#pragma unroll
  for (int i = 0; i < 25; i++) s.lo[i] = s.hi[i] = 0;
}

DEV uint32_t kword(const KState& s, int w) { return (w & 1) ? s.hi[w >> 1] : s.lo[w >> 1]; }
DEV void kxor_word(KState& s, int w, uint32_t v) {
  if (w & 1)
    s.hi[w >> 1] ^= v;
  else
    s.lo[w >> 1] ^= v;
}

#define KROT_XY(x, y) KROT_TABLE[(x) + 5 * (y)]

template <int X, int Y>
struct Rho {
  static constexpr int table[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                    25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
  static constexpr int value = table[X + 5 * Y];
};

template <int X, int Y>
DEV void rho_pi_one(const KState& a, uint32_t (&blo)[25], uint32_t (&bhi)[25]) {
  uint32_t lo = a.lo[X + 5 * Y], hi = a.hi[X + 5 * Y];
  rotl64<Rho<X, Y>::value>(lo, hi);
  constexpr int dst = Y + 5 * ((2 * X + 3 * Y) % 5);
  blo[dst] = lo;
  bhi[dst] = hi;
}

template <int I>
DEV void rho_pi_all(const KState& a, uint32_t (&blo)[25], uint32_t (&bhi)[25]) {
  if constexpr (I < 25) {
    rho_pi_one<I % 5, I / 5>(a, blo, bhi);
    rho_pi_all<I + 1>(a, blo, bhi);
  }
}

DEV void keccak_round(KState& a, uint32_t rc_lo, uint32_t rc_hi) {
  uint32_t clo[5], chi[5];
#pragma unroll
  for (int x = 0; x < 5; x++) {
    clo[x] = xor3(xor3(a.lo[x], a.lo[x + 5], a.lo[x + 10]), a.lo[x + 15], a.lo[x + 20]);
    chi[x] = xor3(xor3(a.hi[x], a.hi[x + 5], a.hi[x + 10]), a.hi[x + 15], a.hi[x + 20]);
  }
  // theta: A[x,y] ^= C[x-1] ^ rot1(C[x+1]) as one v_bitop3 xor3 per half-lane
  uint32_t rlo[5], rhi[5];
#pragma unroll
  for (int x = 0; x < 5; x++) {
    rlo[x] = __builtin_amdgcn_alignbit(clo[x], chi[x], 31);
    rhi[x] = __builtin_amdgcn_alignbit(chi[x], clo[x], 31);
  }
#pragma unroll
  for (int x = 0; x < 5; x++) {
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      a.lo[x + y] = xor3(a.lo[x + y], clo[(x + 4) % 5], rlo[(x + 1) % 5]);
      a.hi[x + y] = xor3(a.hi[x + y], chi[(x + 4) % 5], rhi[(x + 1) % 5]);
    }
  }
  uint32_t blo[25], bhi[25];
  rho_pi_all<0>(a, blo, bhi);
#pragma unroll
  for (int y = 0; y < 25; y += 5) {
#pragma unroll
    for (int x = 0; x < 5; x++) {
      a.lo[y + x] = blo[y + x] ^ (~blo[y + (x + 1) % 5] & blo[y + (x + 2) % 5]);
      a.hi[y + x] = bhi[y + x] ^ (~bhi[y + (x + 1) % 5] & bhi[y + (x + 2) % 5]);
    }
  }
  a.lo[0] ^= rc_lo;
  a.hi[0] ^= rc_hi;
}

DEV void keccak_p12(KState& a) {
#pragma unroll 2
  for (int r = 0; r < 12; r++) keccak_round(a, KRC_LO[r], KRC_HI[r]);
}

// -------------------------------------------------------------------------------------
// Small-message XOF helpers.  A message of at most 167 bytes is assembled into the 42
// rate words with compile-time byte positions, then padded (TurboSHAKE D=0x01) and
// permuted once.
// -------------------------------------------------------------------------------------
struct Msg {
  uint32_t w[42];
};
DEV void msg_zero(Msg& m) {
#pragma unroll
  for (int i = 0; i < 42; i++) m.w[i] = 0;
}
DEV void msg_byte(Msg& m, int pos, uint32_t b) { m.w[pos >> 2] |= (b & 0xffu) << (8 * (pos & 3)); }
// 16 bytes given as 4 LE words, at byte position pos
DEV void msg_bytes16(Msg& m, int pos, const uint32_t* s) {
#pragma unroll
  for (int b = 0; b < 16; b++) msg_byte(m, pos + b, s[b >> 2] >> (8 * (b & 3)));
}
// [len(dst)=8] || dst(8 bytes: 2 words)  -> 9 bytes at position 0
DEV void msg_dst(Msg& m, const uint32_t* dst2) {
  msg_byte(m, 0, 8);
#pragma unroll
  for (int b = 0; b < 8; b++) msg_byte(m, 1 + b, dst2[b >> 2] >> (8 * (b & 3)));
}
// absorb a single padded block of `len` message bytes and permute
DEV void msg_absorb_final(KState& s, Msg& m, int len) {
  msg_byte(m, len, 0x01);
  m.w[41] ^= 0x80000000u;
#pragma unroll
  for (int i = 0; i < 42; i++) kxor_word(s, i, m.w[i]);
  keccak_p12(s);
}
