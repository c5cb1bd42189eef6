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
// 1: Field128 multiply and MAC reduction use the hand-scheduled asm blocks below.
#ifndef F128_ASM
#define F128_ASM 1
#endif

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

// Reduce X = r[0..7] + t * 2^256 (32-bit words; t < 2^32) mod p.  With 64-bit digits x_i:
//   2^128 == 28*2^64 - 1,  2^192 == 783*2^64 - 28,  2^256 == 21896*2^64 - 783  (mod p), so
//   X == (x0 - x2 - 28 x3 - 783 t) + 2^64 (x1 + 28 x2 + 783 x3 + 21896 t).
DEV f128 red288(const uint32_t* r, uint32_t t) {
  // S = x1 + 28*x2 + 783*x3 + 21896*t = s1*2^64 + (s_1:s_0)
  uint64_t t0 = (uint64_t)r[2] + (uint64_t)r[4] * 28u + (uint64_t)r[6] * 783u + (uint64_t)t * 21896u;
  uint32_t s_0 = (uint32_t)t0;
  uint64_t t1 = (uint64_t)r[3] + (uint64_t)r[5] * 28u + (uint64_t)r[7] * 783u + (t0 >> 32);
  uint32_t s_1 = (uint32_t)t1;
  uint32_t s1 = (uint32_t)(t1 >> 32);  // < 2^11
  // u = (s_1:s_0) + 28*s1, carry c into 2^128
  uint64_t u = ((uint64_t)s_1 << 32 | s_0) + (uint64_t)s1 * 28u;
  uint32_t c = u < (uint64_t)s1 * 28u ? 1u : 0u;
  // N = x2 + 28*x3 + 783*t + s1  (< 2^70)
  uint64_t n0 = (uint64_t)r[4] + (uint64_t)r[6] * 28u + (uint64_t)t * 783u + s1;
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

// a*b mod p.  Product by schoolbook v_mad_u64_u32, then red288.
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
  return red288(r, 0);
}


// ---- hand-scheduled Field128 multiply / MAC reduction (gfx950 asm) ----------------------
// The compiler pads every VCC/SGPR-carry chain it emits on gfx94x/gfx950 with s_nop (about one
// per two VALU in mul128); these blocks are written as single asm statements whose VCC carry
// chains are back to back.  Scratch lives in fixed registers v40-v68 (declared clobbered);
// w0..w8 of the 288-bit value to reduce sit in v60-v68 so that every 64-bit operand
// (x0 = v[60:61], x1 = v[62:63], x2 = v[64:65], x3 = v[66:67]) is an even-aligned pair.
// Word-level model with every carry bound checked: tools/red288_model.py.
#define F128_RED288_ASM                                                              \
  /* S = x1 + 28 x2 + 783 x3 + 21896 t  ->  Y = v[40:41] (low 64), S2 = v44 */     \
  "s_movk_i32 %[k783], 0x30f\n\t"                                                   \
  "s_movk_i32 %[k21896], 0x5588\n\t"                                                \
  "v_mad_u64_u32 v[40:41], vcc, v64, 28, v[62:63]\n\t"                              \
  "v_cndmask_b32_e64 v44, 0, 1, vcc\n\t"                                            \
  "v_mad_u64_u32 v[40:41], vcc, v66, %[k783], v[40:41]\n\t"                         \
  "v_addc_co_u32_e32 v44, vcc, 0, v44, vcc\n\t"                                     \
  "v_mad_u64_u32 v[40:41], vcc, v68, %[k21896], v[40:41]\n\t"                       \
  "v_addc_co_u32_e32 v44, vcc, 0, v44, vcc\n\t"                                     \
  "v_mad_u64_u32 v[42:43], vcc, v65, 28, 0\n\t"                                     \
  "v_mad_u64_u32 v[42:43], vcc, v67, %[k783], v[42:43]\n\t"                         \
  "v_add_co_u32_e32 v41, vcc, v41, v42\n\t"                                         \
  "v_addc_co_u32_e32 v44, vcc, v43, v44, vcc\n\t"                                   \
  /* N = x2 + 28 x3 + 783 t + S2  ->  Nn = v[46:47], N2 = v45 */                   \
  "v_mad_u64_u32 v[46:47], vcc, v66, 28, v[64:65]\n\t"                              \
  "v_cndmask_b32_e64 v45, 0, 1, vcc\n\t"                                            \
  "v_mad_u64_u32 v[46:47], vcc, v68, %[k783], v[46:47]\n\t"                         \
  "v_addc_co_u32_e32 v45, vcc, 0, v45, vcc\n\t"                                     \
  "v_mad_u64_u32 v[46:47], vcc, v44, 1, v[46:47]\n\t"                               \
  "v_addc_co_u32_e32 v45, vcc, 0, v45, vcc\n\t"                                     \
  "v_mad_u64_u32 v[42:43], vcc, v67, 28, 0\n\t"                                     \
  "v_add_co_u32_e32 v47, vcc, v47, v42\n\t"                                         \
  "v_addc_co_u32_e32 v45, vcc, v43, v45, vcc\n\t"                                   \
  /* U = Y + 28 S2 (carry c), A = (w0, w1, U) + c (28 2^64 - 1), folded twice */   \
  "v_mad_u64_u32 v[40:41], vcc, v44, 28, v[40:41]\n\t"                              \
  "v_cndmask_b32_e64 v48, 0, -1, vcc\n\t"                                           \
  "v_add_co_u32_e32 v60, vcc, v60, v48\n\t"                                         \
  "v_addc_co_u32_e32 v61, vcc, v61, v48, vcc\n\t"                                   \
  "v_and_b32_e32 v49, 27, v48\n\t"                                                  \
  "v_addc_co_u32_e32 v40, vcc, v40, v49, vcc\n\t"                                   \
  "v_addc_co_u32_e32 v41, vcc, 0, v41, vcc\n\t"                                     \
  "v_cndmask_b32_e64 v48, 0, -1, vcc\n\t"                                           \
  "v_add_co_u32_e32 v60, vcc, v60, v48\n\t"                                         \
  "v_addc_co_u32_e32 v61, vcc, v61, v48, vcc\n\t"                                   \
  "v_and_b32_e32 v49, 27, v48\n\t"                                                  \
  "v_addc_co_u32_e32 v40, vcc, v40, v49, vcc\n\t"                                   \
  "v_addc_co_u32_e32 v41, vcc, 0, v41, vcc\n\t"                                     \
  /* A - N, + p on borrow */                                                        \
  "v_sub_co_u32_e32 v60, vcc, v60, v46\n\t"                                         \
  "v_subb_co_u32_e32 v61, vcc, v61, v47, vcc\n\t"                                   \
  "v_subb_co_u32_e32 v40, vcc, v40, v45, vcc\n\t"                                   \
  "v_subbrev_co_u32_e32 v41, vcc, 0, v41, vcc\n\t"                                  \
  "v_cndmask_b32_e64 v48, 0, -1, vcc\n\t"                                           \
  "v_and_b32_e32 v49, 1, v48\n\t"                                                   \
  "v_add_co_u32_e32 v60, vcc, v60, v49\n\t"                                         \
  "v_addc_co_u32_e32 v61, vcc, 0, v61, vcc\n\t"                                     \
  "v_and_b32_e32 v49, 0xffffffe4, v48\n\t"                                          \
  "v_addc_co_u32_e32 v40, vcc, v40, v49, vcc\n\t"                                   \
  "v_addc_co_u32_e32 v41, vcc, v41, v48, vcc\n\t"                                   \
  /* canonical: A >= p  <=>  A + (2^128 - p) carries; 2^128 - p = (-1, -1, 27, 0) */ \
  "v_add_co_u32_e32 v62, vcc, -1, v60\n\t"                                          \
  "v_addc_co_u32_e32 v63, vcc, -1, v61, vcc\n\t"                                    \
  "v_addc_co_u32_e32 v64, vcc, 27, v40, vcc\n\t"                                    \
  "v_addc_co_u32_e32 v65, vcc, 0, v41, vcc\n\t"                                     \
  "v_cndmask_b32_e32 %[r0], v60, v62, vcc\n\t"                                      \
  "v_cndmask_b32_e32 %[r1], v61, v63, vcc\n\t"                                      \
  "v_cndmask_b32_e32 %[r2], v40, v64, vcc\n\t"                                      \
  "v_cndmask_b32_e32 %[r3], v41, v65, vcc\n\t"

// reduction scratch: v40-v49 and w0..w8 = v60-v68
#define F128_RED_CLOBBERS                                                                \
  "vcc", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v60", "v61", \
      "v62", "v63", "v64", "v65", "v66", "v67", "v68"
// mul128_asm additionally holds the product columns in v40-v53 and h1..h5 in v54-v58
#define F128_MUL_CLOBBERS                                                                 \
  F128_RED_CLOBBERS, "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58"

// a*b mod p: 16 v_mad_u64_u32 into even/odd product columns c_k = v[40+2k : 41+2k] with
// overflow words h1..h5 = v54..v58 (first overflow of a column by v_cndmask), column
// normalisation into w0..w8 = v60..v68, then the shared reduction.
DEV f128 mul128_asm(const f128& a, const f128& b) {
  f128 r;
  uint32_t k783, k21896;
  asm volatile(
      "v_mad_u64_u32 v[40:41], vcc, %[a0], %[b0], 0\n\t"
      "v_mad_u64_u32 v[42:43], vcc, %[a0], %[b1], 0\n\t"
      "v_mad_u64_u32 v[42:43], vcc, %[a1], %[b0], v[42:43]\n\t"
      "v_cndmask_b32_e64 v54, 0, 1, vcc\n\t"
      "v_mad_u64_u32 v[44:45], vcc, %[a0], %[b2], 0\n\t"
      "v_mad_u64_u32 v[44:45], vcc, %[a1], %[b1], v[44:45]\n\t"
      "v_cndmask_b32_e64 v55, 0, 1, vcc\n\t"
      "v_mad_u64_u32 v[44:45], vcc, %[a2], %[b0], v[44:45]\n\t"
      "v_addc_co_u32_e32 v55, vcc, 0, v55, vcc\n\t"
      "v_mad_u64_u32 v[46:47], vcc, %[a0], %[b3], 0\n\t"
      "v_mad_u64_u32 v[46:47], vcc, %[a1], %[b2], v[46:47]\n\t"
      "v_cndmask_b32_e64 v56, 0, 1, vcc\n\t"
      "v_mad_u64_u32 v[46:47], vcc, %[a2], %[b1], v[46:47]\n\t"
      "v_addc_co_u32_e32 v56, vcc, 0, v56, vcc\n\t"
      "v_mad_u64_u32 v[46:47], vcc, %[a3], %[b0], v[46:47]\n\t"
      "v_addc_co_u32_e32 v56, vcc, 0, v56, vcc\n\t"
      "v_mad_u64_u32 v[48:49], vcc, %[a1], %[b3], 0\n\t"
      "v_mad_u64_u32 v[48:49], vcc, %[a2], %[b2], v[48:49]\n\t"
      "v_cndmask_b32_e64 v57, 0, 1, vcc\n\t"
      "v_mad_u64_u32 v[48:49], vcc, %[a3], %[b1], v[48:49]\n\t"
      "v_addc_co_u32_e32 v57, vcc, 0, v57, vcc\n\t"
      "v_mad_u64_u32 v[50:51], vcc, %[a2], %[b3], 0\n\t"
      "v_mad_u64_u32 v[50:51], vcc, %[a3], %[b2], v[50:51]\n\t"
      "v_cndmask_b32_e64 v58, 0, 1, vcc\n\t"
      "v_mad_u64_u32 v[52:53], vcc, %[a3], %[b3], 0\n\t"
      /* X = E + O + H: E = c0 c2 c4 c6 (words 0-7), O = c1 c3 c5 (words 1-6), h_k at word k+2 */
      "v_mov_b32_e32 v60, v40\n\t"
      "v_add_co_u32_e32 v61, vcc, v41, v42\n\t"
      "v_addc_co_u32_e32 v62, vcc, v44, v43, vcc\n\t"
      "v_addc_co_u32_e32 v63, vcc, v45, v46, vcc\n\t"
      "v_addc_co_u32_e32 v64, vcc, v48, v47, vcc\n\t"
      "v_addc_co_u32_e32 v65, vcc, v49, v50, vcc\n\t"
      "v_addc_co_u32_e32 v66, vcc, v52, v51, vcc\n\t"
      "v_addc_co_u32_e32 v67, vcc, 0, v53, vcc\n\t"
      "v_add_co_u32_e32 v63, vcc, v63, v54\n\t"
      "v_addc_co_u32_e32 v64, vcc, v64, v55, vcc\n\t"
      "v_addc_co_u32_e32 v65, vcc, v65, v56, vcc\n\t"
      "v_addc_co_u32_e32 v66, vcc, v66, v57, vcc\n\t"
      "v_addc_co_u32_e32 v67, vcc, v67, v58, vcc\n\t"
      "v_mov_b32_e32 v68, 0\n\t"
      F128_RED288_ASM
      : [r0] "=&v"(r.w[0]), [r1] "=&v"(r.w[1]), [r2] "=&v"(r.w[2]), [r3] "=&v"(r.w[3]),
        [k783] "=&s"(k783), [k21896] "=&s"(k21896)
      : [a0] "v"(a.w[0]), [a1] "v"(a.w[1]), [a2] "v"(a.w[2]), [a3] "v"(a.w[3]),
        [b0] "v"(b.w[0]), [b1] "v"(b.w[1]), [b2] "v"(b.w[2]), [b3] "v"(b.w[3])
      : F128_MUL_CLOBBERS);
  return r;
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
// Column normalisation (X = E + O + H: even columns, odd columns, overflow words -- each a
// plain concatenation) into 9 words, then one red288.  Valid for < 2^31 accumulated products.
DEV f128 mac_reduce(const mac128& a) {
  uint32_t w[9], cy;
  w[0] = (uint32_t)a.c[0];
  w[1] = addc((uint32_t)(a.c[0] >> 32), (uint32_t)a.c[1], 0, &cy);
  w[2] = addc((uint32_t)a.c[2], (uint32_t)(a.c[1] >> 32), cy, &cy);
  w[3] = addc((uint32_t)(a.c[2] >> 32), (uint32_t)a.c[3], cy, &cy);
  w[4] = addc((uint32_t)a.c[4], (uint32_t)(a.c[3] >> 32), cy, &cy);
  w[5] = addc((uint32_t)(a.c[4] >> 32), (uint32_t)a.c[5], cy, &cy);
  w[6] = addc((uint32_t)a.c[6], (uint32_t)(a.c[5] >> 32), cy, &cy);
  w[7] = addc((uint32_t)(a.c[6] >> 32), 0, cy, &cy);
  w[8] = cy;
  w[2] = addc(w[2], a.h[0], 0, &cy);
  w[3] = addc(w[3], a.h[1], cy, &cy);
  w[4] = addc(w[4], a.h[2], cy, &cy);
  w[5] = addc(w[5], a.h[3], cy, &cy);
  w[6] = addc(w[6], a.h[4], cy, &cy);
  w[7] = addc(w[7], a.h[5], cy, &cy);
  w[8] = w[8] + a.h[6] + cy;
  return red288(w, w[8]);
}

// mac_reduce in asm: X = E + O + H over the accumulator columns, then the shared reduction.
DEV f128 mac_reduce_asm(const mac128& a) {
  f128 r;
  uint32_t k783, k21896;
  asm volatile(
      "v_mov_b32_e32 v60, %[c0l]\n\t"
      "v_add_co_u32_e32 v61, vcc, %[c0h], %[c1l]\n\t"
      "v_addc_co_u32_e32 v62, vcc, %[c2l], %[c1h], vcc\n\t"
      "v_addc_co_u32_e32 v63, vcc, %[c2h], %[c3l], vcc\n\t"
      "v_addc_co_u32_e32 v64, vcc, %[c4l], %[c3h], vcc\n\t"
      "v_addc_co_u32_e32 v65, vcc, %[c4h], %[c5l], vcc\n\t"
      "v_addc_co_u32_e32 v66, vcc, %[c6l], %[c5h], vcc\n\t"
      "v_addc_co_u32_e32 v67, vcc, 0, %[c6h], vcc\n\t"
      "v_cndmask_b32_e64 v68, 0, 1, vcc\n\t"
      "v_add_co_u32_e32 v62, vcc, v62, %[h0]\n\t"
      "v_addc_co_u32_e32 v63, vcc, v63, %[h1], vcc\n\t"
      "v_addc_co_u32_e32 v64, vcc, v64, %[h2], vcc\n\t"
      "v_addc_co_u32_e32 v65, vcc, v65, %[h3], vcc\n\t"
      "v_addc_co_u32_e32 v66, vcc, v66, %[h4], vcc\n\t"
      "v_addc_co_u32_e32 v67, vcc, v67, %[h5], vcc\n\t"
      "v_addc_co_u32_e32 v68, vcc, v68, %[h6], vcc\n\t"
      F128_RED288_ASM
      : [r0] "=&v"(r.w[0]), [r1] "=&v"(r.w[1]), [r2] "=&v"(r.w[2]), [r3] "=&v"(r.w[3]),
        [k783] "=&s"(k783), [k21896] "=&s"(k21896)
      : [c0l] "v"((uint32_t)a.c[0]), [c0h] "v"((uint32_t)(a.c[0] >> 32)),
        [c1l] "v"((uint32_t)a.c[1]), [c1h] "v"((uint32_t)(a.c[1] >> 32)),
        [c2l] "v"((uint32_t)a.c[2]), [c2h] "v"((uint32_t)(a.c[2] >> 32)),
        [c3l] "v"((uint32_t)a.c[3]), [c3h] "v"((uint32_t)(a.c[3] >> 32)),
        [c4l] "v"((uint32_t)a.c[4]), [c4h] "v"((uint32_t)(a.c[4] >> 32)),
        [c5l] "v"((uint32_t)a.c[5]), [c5h] "v"((uint32_t)(a.c[5] >> 32)),
        [c6l] "v"((uint32_t)a.c[6]), [c6h] "v"((uint32_t)(a.c[6] >> 32)), [h0] "v"(a.h[0]),
        [h1] "v"(a.h[1]), [h2] "v"(a.h[2]), [h3] "v"(a.h[3]), [h4] "v"(a.h[4]), [h5] "v"(a.h[5]),
        [h6] "v"(a.h[6])
      : F128_RED_CLOBBERS);
  return r;
}

#if F128_ASM
DEV f128 mac_reduce_f(const mac128& a) { return mac_reduce_asm(a); }
#else
DEV f128 mac_reduce_f(const mac128& a) { return mac_reduce(a); }
#endif

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
// (hi:lo) mod p, canonical: 2^64 = 2^32 - 1 and 2^96 = -1 (mod p), so with hi = x3:x2 the value
// is lo + x2 (2^32 - 1) - x3.
DEV uint64_t red128_64(uint64_t lo, uint64_t hi) {
  const uint32_t x2 = (uint32_t)hi, x3 = (uint32_t)(hi >> 32);
  uint64_t t0 = lo - x3;
  if (lo < x3) t0 -= 0xffffffffull;  // borrow: -2^64 = -(2^32 - 1)
  const uint64_t t1 = ((uint64_t)x2 << 32) - x2;
  uint64_t r = t0 + t1;
  if (r < t1) r += 0xffffffffull;  // carry: 2^64 = 2^32 - 1
  if (r >= P64) r -= P64;
  return r;
}
// The 128-bit product as four v_mad_u64_u32 (each partial sum fits 64 bits), then red128_64.
DEV uint64_t mul64f(uint64_t a, uint64_t b) {
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b,
                 b1 = (uint32_t)(b >> 32);
  const uint64_t p00 = (uint64_t)a0 * b0;
  const uint64_t p01 = (uint64_t)a0 * b1 + (p00 >> 32);
  const uint64_t p10 = (uint64_t)a1 * b0 + (uint32_t)p01;
  const uint64_t hi = (uint64_t)a1 * b1 + (p01 >> 32) + (p10 >> 32);  // <= 2^64 - 1
  return red128_64((p10 << 32) | (uint32_t)p00, hi);
}

// Lazily reduced Field64 multiply-accumulate: column k (weight 2^(32k)) = c_k + h_k 2^64; each
// 32x32 limb product is one v_mad_u64_u32 with its carry-out counted by one v_addc (as
// mac_add for Field128).  Up to 2^31 products; mac64_reduce folds once.
struct mac64 {
  uint64_t c0, c1, c2;
  uint32_t h0, h1, h2;
};
DEV void mac64_zero(mac64& a) {
  a.c0 = a.c1 = a.c2 = 0;
  a.h0 = a.h1 = a.h2 = 0;
}
DEV void mac64_add(mac64& a, uint64_t x, uint64_t y) {
  asm("v_mad_u64_u32 %0, vcc, %6, %8, %0\n\t"
      "v_addc_co_u32 %3, vcc, 0, %3, vcc\n\t"
      "v_mad_u64_u32 %1, vcc, %6, %9, %1\n\t"
      "v_addc_co_u32 %4, vcc, 0, %4, vcc\n\t"
      "v_mad_u64_u32 %1, vcc, %7, %8, %1\n\t"
      "v_addc_co_u32 %4, vcc, 0, %4, vcc\n\t"
      "v_mad_u64_u32 %2, vcc, %7, %9, %2\n\t"
      "v_addc_co_u32 %5, vcc, 0, %5, vcc"
      : "+v"(a.c0), "+v"(a.c1), "+v"(a.c2), "+v"(a.h0), "+v"(a.h1), "+v"(a.h2)
      : "v"((uint32_t)x), "v"((uint32_t)(x >> 32)), "v"((uint32_t)y), "v"((uint32_t)(y >> 32))
      : "vcc");
}
// value = c0 + c1 2^32 + (c2 + h0) 2^64 + h1 2^96 + h2 2^128 as 32-bit words w0..w4, then
// w0..w3 by red128_64 and w4 2^128 = -w4 2^32 (mod p)
DEV uint64_t mac64_reduce(const mac64& a) {
  const uint64_t s1 = (a.c0 >> 32) + (uint32_t)a.c1;
  const uint64_t s2 = (s1 >> 32) + (a.c1 >> 32) + (uint32_t)a.c2 + a.h0;
  const uint64_t s3 = (s2 >> 32) + (a.c2 >> 32) + a.h1;
  const uint32_t w4 = (uint32_t)(s3 >> 32) + a.h2;
  const uint64_t r = red128_64((s1 << 32) | (uint32_t)a.c0, (s3 << 32) | (uint32_t)s2);
  return sub64f(r, (uint64_t)w4 << 32);
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
#if F128_ASM
  static DEV T mul(const T& a, const T& b) { return mul128_asm(a, b); }
#else
  static DEV T mul(const T& a, const T& b) { return mul128(a, b); }
#endif
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

#ifndef KECCAK_UNROLL
#define KECCAK_UNROLL 2
#endif
DEV void keccak_p12(KState& a) {
#pragma unroll KECCAK_UNROLL
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

// -------------------------------------------------------------------------------------
// Cross-lane aggregation for the fused accumulate: the 64 lanes' copies of two Field128
// elements, split into 16-bit half-limbs (16 values per lane, slot s = element s >> 3,
// half-limb s & 7), are reduce-scattered over the wave:
//   - across the wave halves with v_permlane32_swap (8 swaps + 8 adds: lanes 0-31 keep slots
//     0-7, lanes 32-63 slots 8-15) and across row pairs with v_permlane16_swap (4 + 4), so the
//     two cross-row stages need no lane-select masks and no LDS (they were ds_swizzle and
//     ds_bpermute after the in-row stages, r03);
//   - inside each row of 16 by two DPP butterfly stages (row_mirror = xor 15, row_half_mirror
//     = xor 7: keep the half selected by lane bit 3 / 2, add the partner's matching half);
//   - the four lanes of a quad, which then hold the same slot, summed by two DPP adds.
// Lane l returns the wave total of slot l >> 2 (element (l >> 5) & 1, half-limb (l >> 2) & 7,
// weight 2^(16 ((l >> 2) & 7))); each total is < 2^22.
// -------------------------------------------------------------------------------------
template <int N, int CTRL, int BIT>
DEV void halfsum_stage(uint32_t (&v)[16], uint32_t lane) {
  const bool sel = (lane >> BIT) & 1;
#pragma unroll
  for (int i = 0; i < N / 2; i++) {
    const uint32_t lo = v[i], hi = v[i + N / 2];
    const uint32_t send = sel ? lo : hi, keep = sel ? hi : lo;
    v[i] = keep + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, CTRL, 0xf, 0xf, false);
  }
}
DEV uint32_t wave_halfsum2(const f128& x0, const f128& x1, uint32_t lane) {
  uint32_t v[16];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    v[2 * w] = x0.w[w] & 0xffffu;
    v[2 * w + 1] = x0.w[w] >> 16;
    v[8 + 2 * w] = x1.w[w] & 0xffffu;
    v[8 + 2 * w + 1] = x1.w[w] >> 16;
  }
  // lanes 32-63 of v[i] <-> lanes 0-31 of v[i + 8]: the sum is slot i on lanes 0-31, i + 8 above
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const auto r = __builtin_amdgcn_permlane32_swap(v[i], v[i + 8], false, false);
    v[i] = r[0] + r[1];
  }
  // odd rows of v[i] <-> even rows of v[i + 4]: slot i + 4 (lane bit 4) + 8 (lane bit 5)
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const auto r = __builtin_amdgcn_permlane16_swap(v[i], v[i + 4], false, false);
    v[i] = r[0] + r[1];
  }
  halfsum_stage<4, 0x140, 3>(v, lane);  // row_mirror: slot bit 1 = lane bit 3
  halfsum_stage<2, 0x141, 2>(v, lane);  // row_half_mirror: slot bit 0 = lane bit 2
  uint32_t x = v[0];
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);  // quad xor 1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);  // quad xor 2
  return x;
}
