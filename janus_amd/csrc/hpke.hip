// hpke.hip -- batched HPKE open of DAP input shares on MI355X (gfx950), SURVEY 8(f) row 2.
//
// One report per lane, the whole RFC 9180 base-mode open in one kernel:
//   X25519 (RFC 7748 Montgomery ladder, GF(2^255-19) in 8 x 32-bit limbs: column-MAC products
//   with v_mad_u64_u32 + carry-out words, like the Field128 MAC of prio3_device.h) or P-256
//   ECDH (p256_device.h: validated uncompressed point, NIST fast reduction, Jacobian ladder)
//   -> DHKEM ExtractAndExpand and the key schedule (HMAC-SHA256, 19 compressions)
//   -> AES-128-GCM / AES-256-GCM (T-tables in LDS, bitwise GHASH) or ChaCha20Poly1305
//   (RFC 8439: ARX keystream, Poly1305 in 26-bit limbs) -> for DAP input shares the
//   PlaintextInputShare decode and checks of aggregator.rs:1893-1990.
// The server scalar is the same for every lane: its bits are wave-uniform (SGPR) and the
// ladder's conditional swaps are v_cndmask on an SGPR mask, so every report runs the same
// instruction stream (no key-dependent branch).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/janus_hpke.h"
#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "sha256_device.h"
#include "aes_device.h"
#include "p256_device.h"
#include "p521_device.h"
#include "p384_device.h"
#include "ecdh_a3.h"
#include "x448_device.h"
#include "sha512_device.h"
#include "sha256_host.h"
#include "prio3_runtime.h"

// -------------------------------------------------------------------------------------
// GF(2^255 - 19), values in [0, 2^256) (loosely reduced), 8 little-endian 32-bit limbs
// -------------------------------------------------------------------------------------
struct fe {
  uint32_t v[8];
};

DEV fe fe_set(uint32_t x) {
  fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = i ? 0u : x;
  return r;
}

#ifndef FE_ASM
#define FE_ASM 1  // 1: the generated single-asm-statement field routines (fe25519_asm.h)
#endif
#if FE_ASM
#include "fe25519_asm.h"
#else
// r = lo + 38 * c (c small), folded twice so the result is < 2^256
DEV void fe_fold(uint32_t r[8], uint32_t c) {
  uint32_t cy;
  r[0] = addc(r[0], c * 38u, 0, &cy);
#pragma unroll
  for (int i = 1; i < 8; i++) r[i] = addc(r[i], 0, cy, &cy);
  r[0] = addc(r[0], cy * 38u, 0, &cy);  // second carry leaves r < 76: no further carry
}

DEV fe fe_add(const fe& a, const fe& b) {
  fe r;
  uint32_t cy;
  r.v[0] = addc(a.v[0], b.v[0], 0, &cy);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc(a.v[i], b.v[i], cy, &cy);
  fe_fold(r.v, cy);
  return r;
}

// a - b: a wrap adds 2^256 = 38 (mod p), compensated by subtracting 38 (twice at most)
DEV fe fe_sub(const fe& a, const fe& b) {
  fe r;
  uint32_t bw;
  r.v[0] = subb(a.v[0], b.v[0], 0, &bw);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = subb(a.v[i], b.v[i], bw, &bw);
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    r.v[0] = subb(r.v[0], bw * 38u, 0, &bw);
#pragma unroll
    for (int i = 1; i < 8; i++) r.v[i] = subb(r.v[i], 0, bw, &bw);
  }
  return r;
}

// X = sum_k c[k] 2^(32k) + sum_k h[k] 2^(32(k+2)) -> 16 words, then reduce (2^256 = 38)
DEV fe fe_reduce512(const uint32_t w[16]) {
  fe r;
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = (uint64_t)w[8 + i] * 38u + w[i] + cy;
    r.v[i] = (uint32_t)t;
    cy = (uint32_t)(t >> 32);
  }
  fe_fold(r.v, cy);
  return r;
}

DEV void fe_normalize(const uint64_t c[15], const uint32_t h[14], uint32_t w[16]) {
  uint32_t cy;
#pragma unroll
  for (int k = 0; k < 15; k += 2) {  // even columns: a plain concatenation
    w[k] = (uint32_t)c[k];
    w[k + 1] = (uint32_t)(c[k] >> 32);
  }
  // + odd columns: c[k] (k odd) at words k, k+1
  w[1] = addc(w[1], (uint32_t)c[1], 0, &cy);
  w[2] = addc(w[2], (uint32_t)(c[1] >> 32), cy, &cy);
#pragma unroll
  for (int k = 3; k < 14; k += 2) {
    w[k] = addc(w[k], (uint32_t)c[k], cy, &cy);
    w[k + 1] = addc(w[k + 1], (uint32_t)(c[k] >> 32), cy, &cy);
  }
  w[15] = addc(w[15], 0, cy, &cy);
  // + overflow words: h[k] at word k + 2
  w[3] = addc(w[3], h[1], 0, &cy);
#pragma unroll
  for (int k = 2; k < 14; k++) w[k + 2] = addc(w[k + 2], h[k], cy, &cy);
}

DEV fe fe_mul(const fe& a, const fe& b) {
  uint64_t c[15];
  uint32_t h[14];
#pragma unroll
  for (int k = 0; k < 15; k++) c[k] = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) h[k] = 0;
  asm(
            "v_mad_u64_u32 %0, vcc, %28, %36, %0\n\t"
      "v_mad_u64_u32 %1, vcc, %28, %37, %1\n\t"
      "v_addc_co_u32 %15, vcc, 0, %15, vcc\n\t"
      "v_mad_u64_u32 %2, vcc, %28, %38, %2\n\t"
      "v_addc_co_u32 %16, vcc, 0, %16, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %28, %39, %3\n\t"
      "v_addc_co_u32 %17, vcc, 0, %17, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %28, %40, %4\n\t"
      "v_addc_co_u32 %18, vcc, 0, %18, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %28, %41, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %28, %42, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %28, %43, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %1, vcc, %29, %36, %1\n\t"
      "v_addc_co_u32 %15, vcc, 0, %15, vcc\n\t"
      "v_mad_u64_u32 %2, vcc, %29, %37, %2\n\t"
      "v_addc_co_u32 %16, vcc, 0, %16, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %29, %38, %3\n\t"
      "v_addc_co_u32 %17, vcc, 0, %17, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %29, %39, %4\n\t"
      "v_addc_co_u32 %18, vcc, 0, %18, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %29, %40, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %29, %41, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %29, %42, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %29, %43, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %2, vcc, %30, %36, %2\n\t"
      "v_addc_co_u32 %16, vcc, 0, %16, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %30, %37, %3\n\t"
      "v_addc_co_u32 %17, vcc, 0, %17, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %30, %38, %4\n\t"
      "v_addc_co_u32 %18, vcc, 0, %18, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %30, %39, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %30, %40, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %30, %41, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %30, %42, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %30, %43, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %31, %36, %3\n\t"
      "v_addc_co_u32 %17, vcc, 0, %17, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %31, %37, %4\n\t"
      "v_addc_co_u32 %18, vcc, 0, %18, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %31, %38, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %31, %39, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %31, %40, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %31, %41, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %31, %42, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %10, vcc, %31, %43, %10\n\t"
      "v_addc_co_u32 %24, vcc, 0, %24, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %32, %36, %4\n\t"
      "v_addc_co_u32 %18, vcc, 0, %18, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %32, %37, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %32, %38, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %32, %39, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %32, %40, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %32, %41, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %10, vcc, %32, %42, %10\n\t"
      "v_addc_co_u32 %24, vcc, 0, %24, vcc\n\t"
      "v_mad_u64_u32 %11, vcc, %32, %43, %11\n\t"
      "v_addc_co_u32 %25, vcc, 0, %25, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %33, %36, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %33, %37, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %33, %38, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %33, %39, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %33, %40, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %10, vcc, %33, %41, %10\n\t"
      "v_addc_co_u32 %24, vcc, 0, %24, vcc\n\t"
      "v_mad_u64_u32 %11, vcc, %33, %42, %11\n\t"
      "v_addc_co_u32 %25, vcc, 0, %25, vcc\n\t"
      "v_mad_u64_u32 %12, vcc, %33, %43, %12\n\t"
      "v_addc_co_u32 %26, vcc, 0, %26, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %34, %36, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %34, %37, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %34, %38, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %34, %39, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %10, vcc, %34, %40, %10\n\t"
      "v_addc_co_u32 %24, vcc, 0, %24, vcc\n\t"
      "v_mad_u64_u32 %11, vcc, %34, %41, %11\n\t"
      "v_addc_co_u32 %25, vcc, 0, %25, vcc\n\t"
      "v_mad_u64_u32 %12, vcc, %34, %42, %12\n\t"
      "v_addc_co_u32 %26, vcc, 0, %26, vcc\n\t"
      "v_mad_u64_u32 %13, vcc, %34, %43, %13\n\t"
      "v_addc_co_u32 %27, vcc, 0, %27, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %35, %36, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %35, %37, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %35, %38, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %10, vcc, %35, %39, %10\n\t"
      "v_addc_co_u32 %24, vcc, 0, %24, vcc\n\t"
      "v_mad_u64_u32 %11, vcc, %35, %40, %11\n\t"
      "v_addc_co_u32 %25, vcc, 0, %25, vcc\n\t"
      "v_mad_u64_u32 %12, vcc, %35, %41, %12\n\t"
      "v_addc_co_u32 %26, vcc, 0, %26, vcc\n\t"
      "v_mad_u64_u32 %13, vcc, %35, %42, %13\n\t"
      "v_addc_co_u32 %27, vcc, 0, %27, vcc\n\t"
      "v_mad_u64_u32 %14, vcc, %35, %43, %14\n\t"
      : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]),
        "+v"(c[7]), "+v"(c[8]), "+v"(c[9]), "+v"(c[10]), "+v"(c[11]), "+v"(c[12]), "+v"(c[13]),
        "+v"(c[14]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]), "+v"(h[5]), "+v"(h[6]),
        "+v"(h[7]), "+v"(h[8]), "+v"(h[9]), "+v"(h[10]), "+v"(h[11]), "+v"(h[12]), "+v"(h[13])
      : "v"(a.v[0]), "v"(a.v[1]), "v"(a.v[2]), "v"(a.v[3]), "v"(a.v[4]), "v"(a.v[5]),
        "v"(a.v[6]), "v"(a.v[7]), "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]),
        "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]), "v"(b.v[7])
      : "vcc");
  uint32_t w[16];
  fe_normalize(c, h, w);
  return fe_reduce512(w);
}

DEV fe fe_sqr(const fe& a) {
  uint64_t c[15];
  uint32_t h[14];
#pragma unroll
  for (int k = 0; k < 15; k++) c[k] = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) h[k] = 0;
  asm(
            "v_mad_u64_u32 %1, vcc, %28, %29, %1\n\t"
      "v_addc_co_u32 %15, vcc, 0, %15, vcc\n\t"
      "v_mad_u64_u32 %2, vcc, %28, %30, %2\n\t"
      "v_addc_co_u32 %16, vcc, 0, %16, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %28, %31, %3\n\t"
      "v_addc_co_u32 %17, vcc, 0, %17, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %28, %32, %4\n\t"
      "v_addc_co_u32 %18, vcc, 0, %18, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %28, %33, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %28, %34, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %28, %35, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %3, vcc, %29, %30, %3\n\t"
      "v_addc_co_u32 %17, vcc, 0, %17, vcc\n\t"
      "v_mad_u64_u32 %4, vcc, %29, %31, %4\n\t"
      "v_addc_co_u32 %18, vcc, 0, %18, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %29, %32, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %29, %33, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %29, %34, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %29, %35, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %5, vcc, %30, %31, %5\n\t"
      "v_addc_co_u32 %19, vcc, 0, %19, vcc\n\t"
      "v_mad_u64_u32 %6, vcc, %30, %32, %6\n\t"
      "v_addc_co_u32 %20, vcc, 0, %20, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %30, %33, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %30, %34, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %30, %35, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %7, vcc, %31, %32, %7\n\t"
      "v_addc_co_u32 %21, vcc, 0, %21, vcc\n\t"
      "v_mad_u64_u32 %8, vcc, %31, %33, %8\n\t"
      "v_addc_co_u32 %22, vcc, 0, %22, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %31, %34, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %10, vcc, %31, %35, %10\n\t"
      "v_addc_co_u32 %24, vcc, 0, %24, vcc\n\t"
      "v_mad_u64_u32 %9, vcc, %32, %33, %9\n\t"
      "v_addc_co_u32 %23, vcc, 0, %23, vcc\n\t"
      "v_mad_u64_u32 %10, vcc, %32, %34, %10\n\t"
      "v_addc_co_u32 %24, vcc, 0, %24, vcc\n\t"
      "v_mad_u64_u32 %11, vcc, %32, %35, %11\n\t"
      "v_addc_co_u32 %25, vcc, 0, %25, vcc\n\t"
      "v_mad_u64_u32 %11, vcc, %33, %34, %11\n\t"
      "v_addc_co_u32 %25, vcc, 0, %25, vcc\n\t"
      "v_mad_u64_u32 %12, vcc, %33, %35, %12\n\t"
      "v_addc_co_u32 %26, vcc, 0, %26, vcc\n\t"
      "v_mad_u64_u32 %13, vcc, %34, %35, %13\n\t"
      "v_addc_co_u32 %27, vcc, 0, %27, vcc\n\t"

      : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]),
        "+v"(c[7]), "+v"(c[8]), "+v"(c[9]), "+v"(c[10]), "+v"(c[11]), "+v"(c[12]), "+v"(c[13]),
        "+v"(c[14]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]), "+v"(h[5]), "+v"(h[6]),
        "+v"(h[7]), "+v"(h[8]), "+v"(h[9]), "+v"(h[10]), "+v"(h[11]), "+v"(h[12]), "+v"(h[13])
      : "v"(a.v[0]), "v"(a.v[1]), "v"(a.v[2]), "v"(a.v[3]), "v"(a.v[4]), "v"(a.v[5]),
        "v"(a.v[6]), "v"(a.v[7])
      : "vcc");
  uint32_t w[16], d[16];
  fe_normalize(c, h, w);  // off-diagonal sum S
  // 2S (S < 2^511) + D, D = sum a_i^2 2^(64 i) (non-overlapping 64-bit products)
#pragma unroll
  for (int i = 15; i > 0; i--) w[i] = __builtin_amdgcn_alignbit(w[i], w[i - 1], 31);
  w[0] <<= 1;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t q = (uint64_t)a.v[i] * a.v[i];
    d[2 * i] = (uint32_t)q;
    d[2 * i + 1] = (uint32_t)(q >> 32);
  }
  uint32_t cy;
  w[0] = addc(w[0], d[0], 0, &cy);
#pragma unroll
  for (int i = 1; i < 16; i++) w[i] = addc(w[i], d[i], cy, &cy);
  return fe_reduce512(w);
}

DEV fe fe_mul121665(const fe& a) {
  fe r;
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = (uint64_t)a.v[i] * 121665u + cy;
    r.v[i] = (uint32_t)t;
    cy = (uint32_t)(t >> 32);
  }
  fe_fold(r.v, cy);
  return r;
}

#endif

DEV fe fe_sqr_n(fe a, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) a = fe_sqr(a);
  return a;
}

// z^(p - 2) (the ref10 addition chain: 254 squarings, 11 multiplications)
DEV fe fe_inv(const fe& z) {
  const fe z2 = fe_sqr(z);
  const fe z9 = fe_mul(fe_sqr_n(z2, 2), z);
  const fe z11 = fe_mul(z9, z2);
  const fe z5_0 = fe_mul(fe_sqr(z11), z9);
  const fe z10_0 = fe_mul(fe_sqr_n(z5_0, 5), z5_0);
  const fe z20_0 = fe_mul(fe_sqr_n(z10_0, 10), z10_0);
  const fe z40_0 = fe_mul(fe_sqr_n(z20_0, 20), z20_0);
  const fe z50_0 = fe_mul(fe_sqr_n(z40_0, 10), z10_0);
  const fe z100_0 = fe_mul(fe_sqr_n(z50_0, 50), z50_0);
  const fe z200_0 = fe_mul(fe_sqr_n(z100_0, 100), z100_0);
  const fe z250_0 = fe_mul(fe_sqr_n(z200_0, 50), z50_0);
  return fe_mul(fe_sqr_n(z250_0, 5), z11);
}

// canonical representative in [0, p): at most two subtractions of p (values < 2^256 = 2p + 38)
DEV fe fe_freeze(fe a) {
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    fe t;
    uint32_t bw;
    t.v[0] = subb(a.v[0], 0xffffffedu, 0, &bw);
#pragma unroll
    for (int i = 1; i < 7; i++) t.v[i] = subb(a.v[i], 0xffffffffu, bw, &bw);
    t.v[7] = subb(a.v[7], 0x7fffffffu, bw, &bw);
#pragma unroll
    for (int i = 0; i < 8; i++) a.v[i] = bw ? a.v[i] : t.v[i];
  }
  return a;
}

DEV void fe_cswap(bool swap, fe& a, fe& b) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t x = a.v[i], y = b.v[i];
    a.v[i] = swap ? y : x;
    b.v[i] = swap ? x : y;
  }
}

// X25519(k, u) (RFC 7748 section 5); k = the clamped scalar (LE words, wave-uniform)
DEV fe x25519_ladder(const uint32_t* k, const fe& u) {
  const fe x1 = u;
  fe x2 = fe_set(1), z2 = fe_set(0), x3 = u, z3 = fe_set(1);
  bool swap = false;
#pragma unroll 1
  for (int t = 254; t >= 0; t--) {
    const bool kt = (k[t >> 5] >> (t & 31)) & 1u;
    swap ^= kt;
    fe_cswap(swap, x2, x3);
    fe_cswap(swap, z2, z3);
    swap = kt;
    const fe A = fe_add(x2, z2), B = fe_sub(x2, z2);
    const fe AA = fe_sqr(A), BB = fe_sqr(B);
    const fe E = fe_sub(AA, BB);
    const fe C = fe_add(x3, z3), D = fe_sub(x3, z3);
    const fe DA = fe_mul(D, A), CB = fe_mul(C, B);
    x3 = fe_sqr(fe_add(DA, CB));
    z3 = fe_mul(x1, fe_sqr(fe_sub(DA, CB)));
    x2 = fe_mul(AA, BB);
    z2 = fe_mul(E, fe_add(AA, fe_mul121665(E)));
  }
  fe_cswap(swap, x2, x3);
  fe_cswap(swap, z2, z3);
  return fe_freeze(fe_mul(x2, fe_inv(z2)));
}

// The same ladder on a lane pair (both lanes hold the whole state; `odd` = the pair's second lane):
// per step each lane runs one square and one product of the first stage (lane 0: AA = A^2,
// DA = D A; lane 1: BB = B^2, CB = C B), they swap them by DPP, then three products of the
// second stage (lane 0: x2 = AA BB, z2 = E (AA + a24 E); lane 1: x3 = (DA + CB)^2,
// t = (DA - CB)^2, z3 = x1 t) and swap again -- 1S + 4M per lane instead of 4S + 5M, so a small
// group's open (one wave per SIMD, each lane's ladder a long dependent chain) runs on twice the
// waves with a shorter chain per lane.  Both lanes end with the same result.
DEV uint32_t pair_swap(uint32_t x) {  // the value of the other lane of the pair (quad_perm 1,0,3,2)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
}
DEV fe fe_pair_swap(const fe& a) {
  fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = pair_swap(a.v[i]);
  return r;
}
DEV fe fe_sel(bool c, const fe& a, const fe& b) {  // c ? a : b
  fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}
DEV fe x25519_ladder_pair(const uint32_t* k, const fe& u, const bool odd) {
  const fe x1 = u;
  fe x2 = fe_set(1), z2 = fe_set(0), x3 = u, z3 = fe_set(1);
  bool swap = false;
#pragma unroll 1
  for (int t = 254; t >= 0; t--) {
    const bool kt = (k[t >> 5] >> (t & 31)) & 1u;
    swap ^= kt;
    fe_cswap(swap, x2, x3);
    fe_cswap(swap, z2, z3);
    swap = kt;
    // stage 1: lane 0 (A, D), lane 1 (B, C); every choice is a select -- no branch, so the two
    // lanes run one instruction stream
    const fe A = fe_add(x2, z2), B = fe_sub(x2, z2), C = fe_add(x3, z3), D = fe_sub(x3, z3);
    const fe X = fe_sel(odd, B, A), Y = fe_sel(odd, C, D);
    const fe s1 = fe_sqr(X), m1 = fe_mul(Y, X);
    const fe s1o = fe_pair_swap(s1), m1o = fe_pair_swap(m1);
    const fe AA = fe_sel(odd, s1o, s1), BB = fe_sel(odd, s1, s1o);
    const fe DA = fe_sel(odd, m1o, m1), CB = fe_sel(odd, m1, m1o);
    // stage 2
    const fe E = fe_sub(AA, BB);
    const fe sp = fe_add(DA, CB), sm = fe_sub(DA, CB);
    const fe G = fe_add(AA, fe_mul121665(E));
    const fe r1 = fe_mul(fe_sel(odd, sp, AA), fe_sel(odd, sp, BB));  // x3 | x2
    const fe r2 = fe_mul(fe_sel(odd, sm, E), fe_sel(odd, sm, G));    // t  | z2
    const fe r3 = fe_mul(x1, r2);                                    // z3 | -
    const fe r1o = fe_pair_swap(r1), r2o = fe_pair_swap(r2), r3o = fe_pair_swap(r3);
    x2 = fe_sel(odd, r1o, r1);
    z2 = fe_sel(odd, r2o, r2);
    x3 = fe_sel(odd, r1, r1o);
    z3 = fe_sel(odd, r3, r3o);
  }
  fe_cswap(swap, x2, x3);
  fe_cswap(swap, z2, z3);
  return fe_freeze(fe_mul(x2, fe_inv(z2)));
}

// GHASH step (SP 800-38D Algorithm 1): y = (y ^ x) * H in GF(2^128), big-endian words
DEV void ghash_block(uint32_t y[4], const uint32_t x[4], const uint32_t H[4]) {
  uint32_t X[4] = {y[0] ^ x[0], y[1] ^ x[1], y[2] ^ x[2], y[3] ^ x[3]};
  uint32_t Z[4] = {0, 0, 0, 0}, V[4] = {H[0], H[1], H[2], H[3]};
#pragma unroll
  for (int wi = 0; wi < 4; wi++) {
#pragma unroll 8
    for (int bit = 31; bit >= 0; bit--) {
      const uint32_t m = 0u - ((X[wi] >> bit) & 1u);
      Z[0] ^= V[0] & m;
      Z[1] ^= V[1] & m;
      Z[2] ^= V[2] & m;
      Z[3] ^= V[3] & m;
      const uint32_t lsb = 0u - (V[3] & 1u);
      V[3] = __builtin_amdgcn_alignbit(V[2], V[3], 1);
      V[2] = __builtin_amdgcn_alignbit(V[1], V[2], 1);
      V[1] = __builtin_amdgcn_alignbit(V[0], V[1], 1);
      V[0] = (V[0] >> 1) ^ (0xe1000000u & lsb);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; i++) y[i] = Z[i];
}

// -------------------------------------------------------------------------------------
// ChaCha20 (RFC 8439 2.3) and Poly1305 (2.5) for the ChaCha20Poly1305 AEAD (2.8)
// -------------------------------------------------------------------------------------
DEV uint32_t rotl32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
#define CHACHA_QR(a, b, c, d)                  \
  a += b, d ^= a, d = rotl32(d, 16);           \
  c += d, b ^= c, b = rotl32(b, 12);           \
  a += b, d ^= a, d = rotl32(d, 8);            \
  c += d, b ^= c, b = rotl32(b, 7)

// one 64-byte keystream block as 16 little-endian words
DEV void chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3],
                        uint32_t out[16]) {
  uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1],
                    key[2],      key[3],      key[4],      key[5],      key[6], key[7],
                    counter,     nonce[0],    nonce[1],    nonce[2]};
#pragma unroll
  for (int i = 0; i < 10; i++) {
    CHACHA_QR(x[0], x[4], x[8], x[12]);
    CHACHA_QR(x[1], x[5], x[9], x[13]);
    CHACHA_QR(x[2], x[6], x[10], x[14]);
    CHACHA_QR(x[3], x[7], x[11], x[15]);
    CHACHA_QR(x[0], x[5], x[10], x[15]);
    CHACHA_QR(x[1], x[6], x[11], x[12]);
    CHACHA_QR(x[2], x[7], x[8], x[13]);
    CHACHA_QR(x[3], x[4], x[9], x[14]);
  }
  const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1],
                          key[2],      key[3],      key[4],      key[5],      key[6], key[7],
                          counter,     nonce[0],    nonce[1],    nonce[2]};
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

// Poly1305 over 16-byte blocks with the 2^128 pad bit (the AEAD's zero-padded data): h and r in
// five 26-bit limbs, 32 x 32 -> 64-bit products (v_mad_u64_u32)
struct Poly1305 {
  uint32_t r0, r1, r2, r3, r4, h0, h1, h2, h3, h4, pad[4];
};
DEV void poly_init(Poly1305& P, const uint32_t otk[8]) {  // one-time key: r || s, LE words
  P.r0 = otk[0] & 0x3ffffffu;
  P.r1 = ((otk[0] >> 26) | (otk[1] << 6)) & 0x3ffff03u;
  P.r2 = ((otk[1] >> 20) | (otk[2] << 12)) & 0x3ffc0ffu;
  P.r3 = ((otk[2] >> 14) | (otk[3] << 18)) & 0x3f03fffu;
  P.r4 = (otk[3] >> 8) & 0x00fffffu;
  P.h0 = P.h1 = P.h2 = P.h3 = P.h4 = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) P.pad[i] = otk[4 + i];
}
DEV void poly_block(Poly1305& P, const uint32_t m[4]) {  // m: 16 bytes as LE words
  constexpr uint32_t M26 = 0x3ffffffu;
  P.h0 += m[0] & M26;
  P.h1 += ((m[0] >> 26) | (m[1] << 6)) & M26;
  P.h2 += ((m[1] >> 20) | (m[2] << 12)) & M26;
  P.h3 += ((m[2] >> 14) | (m[3] << 18)) & M26;
  P.h4 += (m[3] >> 8) | (1u << 24);
  const uint32_t s1 = P.r1 * 5, s2 = P.r2 * 5, s3 = P.r3 * 5, s4 = P.r4 * 5;
  typedef uint64_t u64;
  u64 d0 = (u64)P.h0 * P.r0 + (u64)P.h1 * s4 + (u64)P.h2 * s3 + (u64)P.h3 * s2 + (u64)P.h4 * s1;
  u64 d1 = (u64)P.h0 * P.r1 + (u64)P.h1 * P.r0 + (u64)P.h2 * s4 + (u64)P.h3 * s3 + (u64)P.h4 * s2;
  u64 d2 = (u64)P.h0 * P.r2 + (u64)P.h1 * P.r1 + (u64)P.h2 * P.r0 + (u64)P.h3 * s4 + (u64)P.h4 * s3;
  u64 d3 = (u64)P.h0 * P.r3 + (u64)P.h1 * P.r2 + (u64)P.h2 * P.r1 + (u64)P.h3 * P.r0 + (u64)P.h4 * s4;
  u64 d4 = (u64)P.h0 * P.r4 + (u64)P.h1 * P.r3 + (u64)P.h2 * P.r2 + (u64)P.h3 * P.r1 + (u64)P.h4 * P.r0;
  uint32_t c = (uint32_t)(d0 >> 26);
  P.h0 = (uint32_t)d0 & M26;
  d1 += c, c = (uint32_t)(d1 >> 26), P.h1 = (uint32_t)d1 & M26;
  d2 += c, c = (uint32_t)(d2 >> 26), P.h2 = (uint32_t)d2 & M26;
  d3 += c, c = (uint32_t)(d3 >> 26), P.h3 = (uint32_t)d3 & M26;
  d4 += c, c = (uint32_t)(d4 >> 26), P.h4 = (uint32_t)d4 & M26;
  P.h0 += c * 5, c = P.h0 >> 26, P.h0 &= M26;
  P.h1 += c;
}
// tag = (h mod 2^130 - 5) + s mod 2^128, LE words
DEV void poly_finish(Poly1305& P, uint32_t tag[4]) {
  constexpr uint32_t M26 = 0x3ffffffu;
  uint32_t h0 = P.h0, h1 = P.h1, h2 = P.h2, h3 = P.h3, h4 = P.h4, c;
  c = h1 >> 26, h1 &= M26, h2 += c;
  c = h2 >> 26, h2 &= M26, h3 += c;
  c = h3 >> 26, h3 &= M26, h4 += c;
  c = h4 >> 26, h4 &= M26, h0 += c * 5;
  c = h0 >> 26, h0 &= M26, h1 += c;
  uint32_t g0 = h0 + 5;  // h - p = h + 5 - 2^130
  c = g0 >> 26, g0 &= M26;
  uint32_t g1 = h1 + c;
  c = g1 >> 26, g1 &= M26;
  uint32_t g2 = h2 + c;
  c = g2 >> 26, g2 &= M26;
  uint32_t g3 = h3 + c;
  c = g3 >> 26, g3 &= M26;
  const uint32_t g4 = h4 + c - (1u << 26);
  const uint32_t keep_g = (g4 >> 31) - 1u;  // all ones when h >= p
  h0 = (h0 & ~keep_g) | (g0 & keep_g);
  h1 = (h1 & ~keep_g) | (g1 & keep_g);
  h2 = (h2 & ~keep_g) | (g2 & keep_g);
  h3 = (h3 & ~keep_g) | (g3 & keep_g);
  h4 = (h4 & ~keep_g) | (g4 & keep_g);
  const uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14),
                 w3 = (h3 >> 18) | (h4 << 8);
  uint64_t f = (uint64_t)w0 + P.pad[0];
  tag[0] = (uint32_t)f;
  f = (uint64_t)w1 + P.pad[1] + (f >> 32);
  tag[1] = (uint32_t)f;
  f = (uint64_t)w2 + P.pad[2] + (f >> 32);
  tag[2] = (uint32_t)f;
  f = (uint64_t)w3 + P.pad[3] + (f >> 32);
  tag[3] = (uint32_t)f;
}

// -------------------------------------------------------------------------------------
// Kernel
// -------------------------------------------------------------------------------------
struct HpkeParams {
  uint32_t sk[8];        // clamped X25519 scalar, LE words
  uint32_t pk[8];        // pkRm bytes, LE-packed words
  uint32_t ksc[17];      // key_schedule_context (65 bytes) as BE words, zero padded (KDF 0x0001)
  uint32_t task[8];      // task ID (input-share AAD), BE words
  uint32_t ipad0[8], opad0[8];  // HMAC-SHA256 midstates of the empty key
  uint32_t aead;                // AEAD id (1, 2, 3), wave-uniform
  uint32_t kem;                 // KEM id (0x20 X25519, 0x10 P-256, 0x21 X448, 0x12 P-521)
  uint32_t kdf;                 // key-schedule KDF id (1 HKDF-SHA256, 2 -SHA384, 3 -SHA512)
  uint8_t pk65[68];             // P-256: pkRm, the 65-byte uncompressed point (kem_context)
  int8_t p256_dig[88];          // P-256: signed window digits of the private key (p256_recode)
  uint64_t ksc64[17];           // key_schedule_context (97 / 129 bytes) as BE 64-bit words (KDF 2, 3)
  uint64_t ipad0_64[8], opad0_64[8];  // HMAC-SHA512 midstates of the empty key (X448, P-521 KEMs)
  uint32_t sk448[14];           // X448: clamped scalar, LE words
  uint8_t pkraw[136];           // X448 / P-521: pkRm bytes (56 / 133)
  int8_t p521_dig[136];         // P-521: signed window digits of the private key (recode_w4)
  int8_t p384_dig[96];          // P-384: the same (recode_w4, 96 digits)
  uint64_t ipad0_384[8], opad0_384[8];  // HMAC-SHA384 midstates of the empty key (P-384 KEM)
};

// KEM constants (RFC 9180 7.1): Nenc (= Npk) and Nsecret, i.e. the Nh of the KEM's own KDF
template <int KEM>
struct KemC {
  static constexpr int NENC =
      KEM == 0x20 ? 32 : KEM == 0x10 ? 65 : KEM == 0x21 ? 56 : KEM == 0x11 ? 97 : 133;
  static constexpr int NSS_W =  // shared secret (the KEM KDF's Nh), 32-bit words
      (KEM == 0x20 || KEM == 0x10) ? 8 : KEM == 0x11 ? 12 : 16;
};
constexpr int P521_DIGITS = 131;  // w = 4 digits of a 521-bit key (130 windows + the top digit)
constexpr int P384_DIGITS = 96;   // 95 windows of a 384-bit key + the top digit

struct OpenArgs {
  uint32_t n, ct_stride, aad_stride, share_len;
  int require_taskprov;
  const uint8_t *enc, *ct, *aad, *ids, *pubs;
  const uint32_t *ct_len, *aad_len;
  const uint64_t* times;
  uint8_t *pt, *shares, *status;
  // coalesced groups of several tasks (the executor): per-report slot into task_tab[slot][8]
  // (BE words, like HpkeParams::task); nullable: HpkeParams::task
  const uint16_t* task_slot;
  const uint32_t* task_tab;
};

// word i of report r's task ID (input-share AAD), BE
DEV uint32_t task_word(const HpkeParams& P, const OpenArgs& a, uint32_t r, int i) {
  return a.task_slot ? a.task_tab[8 * (size_t)a.task_slot[r] + i] : P.task[i];
}

DEV void load16(const uint8_t* p, uint32_t* w) {
  const uint4 v = *(const uint4*)p;
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
}

DEV void load_words(const uint8_t* p, uint32_t* w, int n16) {
#pragma unroll
  for (int i = 0; i < n16; i++) load16(p + 16 * i, w + 4 * i);
}

// suite_id = "HPKE" || kem || kdf || aead at byte pos of a SHA-256 / SHA-512 message
template <class M>
DEV void msuite(M& m, int pos, uint32_t kem, uint32_t kdf, uint32_t aead) {
  mstr(m, pos, "HPKE");
  mbyte(m, pos + 4, 0x00);
  mbyte(m, pos + 5, kem);
  mbyte(m, pos + 6, 0x00);
  mbyte(m, pos + 7, kdf);
  mbyte(m, pos + 8, 0x00);
  mbyte(m, pos + 9, aead);
}

// RFC 9180 5.1 KeySchedule(mode_base) with HKDF-SHA256 (KDF 0x0001): shared secret (NSS 32-bit
// BE words) -> AEAD key (BE words) and base_nonce (3 BE words).  key_schedule_context is
// constant per opener (P.ksc, host-computed).
template <int NSS>
__device__ __noinline__ void key_schedule_sha256(const HpkeParams& P, uint32_t kem, const uint32_t* ss,
                             uint32_t keyw[8], uint32_t noncew[3]) {
  const uint32_t AEAD = P.aead, NK = AEAD == 1 ? 16 : 32;
  uint32_t secret[8];
  {  // secret = LabeledExtract(shared_secret, "secret", "")
    Msg32<16> m;
    mz(m);
    mstr(m, 0, "HPKE-v1");
    msuite(m, 7, kem, 1, AEAD);
    mstr(m, 17, "secret");
    HmacKey k;
    hmac_keyw<NSS>(k, ss);
    hmac(k, m, 23, secret);
  }
  // key / base_nonce = LabeledExpand(secret, "key" | "base_nonce", ksc, Nk | 12)
  HmacKey k;
  hmac_key32(k, secret);
  Msg32<32> m;
  mz(m);
  mbyte(m, 0, 0);
  mbyte(m, 1, NK);
  mstr(m, 2, "HPKE-v1");
  msuite(m, 9, kem, 1, AEAD);
  mstr(m, 19, "key");
  mwords_be(m, 22, P.ksc, 17);  // 65 bytes + 3 zero padding bytes
  mbyte(m, 87, 0x01);
  hmac(k, m, 88, keyw);
  Msg32<32> n2;
  mz(n2);
  mbyte(n2, 0, 0);
  mbyte(n2, 1, 12);
  mstr(n2, 2, "HPKE-v1");
  msuite(n2, 9, kem, 1, AEAD);
  mstr(n2, 19, "base_nonce");
  mwords_be(n2, 29, P.ksc, 17);
  mbyte(n2, 94, 0x01);
  uint32_t nw[8];
  hmac(k, n2, 95, nw);
  noncew[0] = nw[0], noncew[1] = nw[1], noncew[2] = nw[2];
}

// The same with HKDF-SHA384 (S384, KDF 0x0002) or HKDF-SHA512 (KDF 0x0003): Nh = 48 / 64, so
// key_schedule_context is 97 / 129 bytes (P.ksc64) and the expand messages take two blocks.
template <int NSS, bool S384>
__device__ __noinline__ void key_schedule_sha512(const HpkeParams& P, uint32_t kem, const uint32_t* ss,
                             uint32_t keyw[8], uint32_t noncew[3]) {
  constexpr int NH = S384 ? 48 : 64, KSC = 1 + 2 * NH;
  constexpr uint32_t KDF = S384 ? 2 : 3;
  const uint32_t AEAD = P.aead, NK = AEAD == 1 ? 16 : 32;
  uint64_t secret[8];
  {  // secret = LabeledExtract(shared_secret, "secret", "")
    uint64_t key[NSS / 2];
#pragma unroll
    for (int i = 0; i < NSS / 2; i++) key[i] = (uint64_t)ss[2 * i] << 32 | ss[2 * i + 1];
    HmacKey64 k;
    hmac64_key(k, key, NSS / 2, S384);
    Msg64<16> m;
    mz(m);
    mstr(m, 0, "HPKE-v1");
    msuite(m, 7, kem, KDF, AEAD);
    mstr(m, 17, "secret");
    hmac64(k, m, 23, secret);
  }
  HmacKey64 k;
  hmac64_key(k, secret, NH / 8, S384);
  uint64_t o[8];
  {  // key = LabeledExpand(secret, "key", ksc, Nk)
    Msg64<32> m;
    mz(m);
    mbyte(m, 0, 0);
    mbyte(m, 1, NK);
    mstr(m, 2, "HPKE-v1");
    msuite(m, 9, kem, KDF, AEAD);
    mstr(m, 19, "key");
    mwords64(m, 22, P.ksc64, 17);  // KSC bytes + zero padding
    mbyte(m, 22 + KSC, 0x01);
    hmac64(k, m, 23 + KSC, o);
#pragma unroll
    for (int i = 0; i < 4; i++) keyw[2 * i] = (uint32_t)(o[i] >> 32), keyw[2 * i + 1] = (uint32_t)o[i];
  }
  {  // base_nonce = LabeledExpand(secret, "base_nonce", ksc, 12)
    Msg64<32> m;
    mz(m);
    mbyte(m, 0, 0);
    mbyte(m, 1, 12);
    mstr(m, 2, "HPKE-v1");
    msuite(m, 9, kem, KDF, AEAD);
    mstr(m, 19, "base_nonce");
    mwords64(m, 29, P.ksc64, 17);
    mbyte(m, 29 + KSC, 0x01);
    hmac64(k, m, 30 + KSC, o);
    noncew[0] = (uint32_t)(o[0] >> 32), noncew[1] = (uint32_t)o[0], noncew[2] = (uint32_t)(o[1] >> 32);
  }
}

// DHKEM ExtractAndExpand with HKDF-SHA512 (the X448 and P-521 KEMs) or HKDF-SHA384 (S384: the
// P-384 KEM): dh (NDH bytes, a byte accessor) and kem_context = enc || pkRm (NENC bytes each)
// -> shared_secret (Nh = 64 / 48 bytes: 16 / 12 BE words)
template <int KEM, int NDH, bool S384 = false, class DhByte, class EncByte>
DEV void eae_sha512(const HpkeParams& P, DhByte dh, EncByte enc, uint32_t* ss) {
  constexpr int NENC = KemC<KEM>::NENC, NHW = S384 ? 6 : 8;  // Nh in 64-bit words
  uint64_t prk[8];
  {  // eae_prk = LabeledExtract("", "eae_prk", dh)
    HmacKey64 k0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      k0.ist[i] = S384 ? P.ipad0_384[i] : P.ipad0_64[i];
      k0.ost[i] = S384 ? P.opad0_384[i] : P.opad0_64[i];
    }
    k0.out_words = NHW;
    Msg64<(19 + NDH + 17 + 127) / 128 * 16> m;
    mz(m);
    mstr(m, 0, "HPKE-v1");
    mstr(m, 7, "KEM");
    mbyte(m, 10, 0x00);
    mbyte(m, 11, KEM);
    mstr(m, 12, "eae_prk");
#pragma unroll
    for (int i = 0; i < NDH; i++) mbyte(m, 19 + i, dh(i));
    hmac64(k0, m, 19 + NDH, prk);
  }
  // shared_secret = LabeledExpand(eae_prk, "shared_secret", enc || pkRm, Nh)
  HmacKey64 k;
  hmac64_key(k, prk, NHW, S384);
  constexpr int LEN = 27 + 2 * NENC + 1;
  Msg64<(LEN + 17 + 127) / 128 * 16> m;
  mz(m);
  mbyte(m, 0, 0);
  mbyte(m, 1, 8 * NHW);
  mstr(m, 2, "HPKE-v1");
  mstr(m, 9, "KEM");
  mbyte(m, 12, 0x00);
  mbyte(m, 13, KEM);
  mstr(m, 14, "shared_secret");
#pragma unroll
  for (int i = 0; i < NENC; i++) mbyte(m, 27 + i, enc(i));
#pragma unroll
  for (int i = 0; i < NENC; i++) mbyte(m, 27 + NENC + i, P.pkraw[i]);
  mbyte(m, LEN - 1, 0x01);
  uint64_t o[8];
  hmac64(k, m, LEN, o);
#pragma unroll
  for (int i = 0; i < NHW; i++) ss[2 * i] = (uint32_t)(o[i] >> 32), ss[2 * i + 1] = (uint32_t)o[i];
}

// the P-521 ECDH, out of line (one copy for the three kernel instances of the KEM)
__device__ __noinline__ bool p521_dh(const int8_t* dig, const uint8_t* enc, uint8_t* dh) {
  return ecdh_a3::ecdh<p521::Field, P521_DIGITS, p521::FieldInl>(dig, enc, dh);
}
// the P-384 ECDH, out of line (its field products are out-of-line calls with register operands)
__device__ __noinline__ bool p384_dh(const int8_t* dig, const uint8_t* enc, uint8_t* dh) {
  return ecdh_a3::ecdh<p384::Field, P384_DIGITS>(dig, enc, dh);
}

// MODE 0: explicit AAD, plaintext out.  MODE 1: DAP helper input share with PUB bytes of
// public share (InputShareAad built here), decoded helper share out.
// AEAD (P.aead): 1 AES-128-GCM, 2 AES-256-GCM, 3 ChaCha20Poly1305 (RFC 9180 7.3 ids).
// KEM: 0x20 DHKEM(X25519, HKDF-SHA256) (enc: 32 bytes), 0x10 DHKEM(P-256, HKDF-SHA256) (enc: the
// 65-byte uncompressed point), 0x21 DHKEM(X448, HKDF-SHA512) (56 bytes), 0x12 DHKEM(P-521,
// HKDF-SHA512) (133 bytes), 0x11 DHKEM(P-384, HKDF-SHA384) (97 bytes).  The key-schedule KDF (P.kdf: HKDF-SHA256 / -384 / -512) and the AEAD
// are kernel arguments (wave-uniform): one instance per (MODE, PUB, KEM).
// (amdgpu_waves_per_eu(2), which caps the P-384 instance's 354 VGPRs + AGPRs at 256: 5.15 against
// 5.16 M/s, X25519 / P-521 unchanged -- not kept)
#ifndef HPKE_WAVES  // A/B builds: e.g. -DHPKE_WAVES='__attribute__((amdgpu_waves_per_eu(3, 3)))'
#define HPKE_WAVES
#endif
template <int MODE, int PUB, int KEM, bool PAIR = false>
__global__ __launch_bounds__(256) HPKE_WAVES void k_hpke_open(HpkeParams P, OpenArgs a) {
  static_assert(KEM == 0x20 || KEM == 0x10 || KEM == 0x21 || KEM == 0x12 || KEM == 0x11, "KEM id");
  static_assert(!PAIR || KEM == 0x20, "the lane-pair ladder is X25519's");
  const uint32_t AEAD = P.aead;
  __shared__ AesT T;
  aes_tables_init(T);
  __syncthreads();
  // PAIR: two lanes per report; they differ only inside the ladder and write the same bytes
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t r = PAIR ? gid >> 1 : gid;
  if (r >= a.n) return;
  // ---- DHKEM Decap (RFC 9180 4.1): dh, then ExtractAndExpand(dh, enc || pkRm) -------------
  constexpr int NSS = KemC<KEM>::NSS_W;
  uint32_t ss[NSS], keyw[8], noncew[3];
  bool ok;
  if constexpr (KEM == 0x20 || KEM == 0x10) {
  uint32_t prk[8];
  HmacKey k0;  // the empty-key HMAC midstates (eae_prk extraction)
#pragma unroll
  for (int i = 0; i < 8; i++) {
    k0.ist[i] = P.ipad0[i];
    k0.ost[i] = P.opad0[i];
  }
  if constexpr (KEM == 0x20) {
    uint32_t encw[8];
    load_words(a.enc + 32 * (size_t)r, encw, 2);
    fe u;
#pragma unroll
    for (int i = 0; i < 8; i++) u.v[i] = encw[i];
    u.v[7] &= 0x7fffffffu;  // decodeUCoordinate masks bit 255
    const fe dh = PAIR ? x25519_ladder_pair(P.sk, u, (threadIdx.x & 1u) != 0) : x25519_ladder(P.sk, u);
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) nz |= dh.v[i];
    ok = nz != 0;  // all-zero shared secret: DeserializeError / ValidationError
    {  // eae_prk = LabeledExtract("", "eae_prk", dh)
      Msg32<16> m;
      mz(m);
      mstr(m, 0, "HPKE-v1");
      mstr(m, 7, "KEM");
      mbyte(m, 10, 0x00);
      mbyte(m, 11, 0x20);
      mstr(m, 12, "eae_prk");
      mwords_le(m, 19, dh.v, 8);
      hmac(k0, m, 51, prk);
    }
    {  // shared_secret = LabeledExpand(eae_prk, "shared_secret", enc || pkRm, 32)
      Msg32<32> m;
      mz(m);
      mbyte(m, 0, 0);
      mbyte(m, 1, 32);
      mstr(m, 2, "HPKE-v1");
      mstr(m, 9, "KEM");
      mbyte(m, 12, 0x00);
      mbyte(m, 13, 0x20);
      mstr(m, 14, "shared_secret");
      mwords_le(m, 27, encw, 8);
      mwords_le(m, 59, P.pk, 8);
      mbyte(m, 91, 0x01);
      HmacKey k;
      hmac_key32(k, prk);
      hmac(k, m, 92, ss);
    }
  } else {
    const uint8_t* ep = a.enc + 65 * (size_t)r;
    uint32_t dh[8];  // x-coordinate, big-endian words
    ok = p256::ecdh(P.p256_dig, ep, dh);
    {  // eae_prk = LabeledExtract("", "eae_prk", dh)
      Msg32<16> m;
      mz(m);
      mstr(m, 0, "HPKE-v1");
      mstr(m, 7, "KEM");
      mbyte(m, 10, 0x00);
      mbyte(m, 11, 0x10);
      mstr(m, 12, "eae_prk");
      mwords_be(m, 19, dh, 8);
      hmac(k0, m, 51, prk);
    }
    {  // shared_secret = LabeledExpand(eae_prk, "shared_secret", enc || pkRm (130 B), 32)
      Msg32<48> m;
      mz(m);
      mbyte(m, 0, 0);
      mbyte(m, 1, 32);
      mstr(m, 2, "HPKE-v1");
      mstr(m, 9, "KEM");
      mbyte(m, 12, 0x00);
      mbyte(m, 13, 0x10);
      mstr(m, 14, "shared_secret");
      for (int i = 0; i < 65; i++) mbyte(m, 27 + i, ep[i]);
#pragma unroll
      for (int i = 0; i < 65; i++) mbyte(m, 92 + i, P.pk65[i]);
      mbyte(m, 157, 0x01);
      HmacKey k;
      hmac_key32(k, prk);
      hmac(k, m, 158, ss);
    }
  }
  } else if constexpr (KEM == 0x21) {
    // X448 (RFC 7748): enc is the 56-byte u-coordinate; rows are 8-byte aligned
    uint32_t encw[14], dh[14];
    const uint2* ep = (const uint2*)(a.enc + 56 * (size_t)r);
#pragma unroll
    for (int i = 0; i < 7; i++) {
      const uint2 v = ep[i];
      encw[2 * i] = v.x, encw[2 * i + 1] = v.y;
    }
    x448::ladder(P.sk448, encw, dh);
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) nz |= dh[i];
    ok = nz != 0;  // all-zero shared secret: ValidationError
    auto byte_of = [](const uint32_t* w) {
      return [w](int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xffu; };
    };
    eae_sha512<KEM, 56>(P, byte_of(dh), byte_of(encw), ss);
  } else if constexpr (KEM == 0x11) {
    // P-384 (SEC 1): enc is the 97-byte uncompressed point; the KEM's KDF is HKDF-SHA384
    const uint8_t* ep = a.enc + 97 * (size_t)r;
    uint8_t dh[48];
    ok = p384_dh(P.p384_dig, ep, dh);
    eae_sha512<KEM, 48, true>(P, [&](int i) { return (uint32_t)dh[i]; },
                              [&](int i) { return (uint32_t)ep[i]; }, ss);
  } else {
    // P-521 (SEC 1): enc is the 133-byte uncompressed point
    const uint8_t* ep = a.enc + 133 * (size_t)r;
    uint8_t dh[66];
    ok = p521_dh(P.p521_dig, ep, dh);
    eae_sha512<KEM, 66>(P, [&](int i) { return (uint32_t)dh[i]; },
                        [&](int i) { return (uint32_t)ep[i]; }, ss);
  }
  // ---- KeySchedule(mode_base) with the suite's KDF -----------------------------------------
  if (P.kdf == 1)
    key_schedule_sha256<NSS>(P, KEM, ss, keyw, noncew);
  else if (P.kdf == 2)
    key_schedule_sha512<NSS, true>(P, KEM, ss, keyw, noncew);
  else
    key_schedule_sha512<NSS, false>(P, KEM, ss, keyw, noncew);
  uint32_t aad_len, pt_len;
  uint8_t* pp;
  auto gcm_open = [&](auto nr_tag) {  // NR = 10 (AES-128-GCM) or 14 (AES-256-GCM)
    constexpr int NR = decltype(nr_tag)::value;
  // ---- AES-GCM open (AEAD 1, 2), sequence number 0 (nonce = base_nonce) --------------
  uint32_t kcol[8], rk[4 * (NR + 1)];
#pragma unroll
  for (int i = 0; i < 8; i++) kcol[i] = __builtin_bswap32(keyw[i]);
  if constexpr (NR == 10)
    aes128_expand(T, kcol, rk);
  else
    aes256_expand(T, kcol, rk);
  uint32_t H[4];
  {
    const uint32_t z[4] = {0, 0, 0, 0};
    uint32_t hc[4];
    aes_encrypt<NR>(T, rk, z, hc);
#pragma unroll
    for (int i = 0; i < 4; i++) H[i] = __builtin_bswap32(hc[i]);
  }
  uint32_t y[4] = {0, 0, 0, 0};
  if constexpr (MODE == 1) {
    // InputShareAad: task_id (32) || report_id (16) || time (u64 BE) || u32 BE len || public
    constexpr int AW = (60 + PUB + 3) / 4;
    uint32_t aw[((AW + 3) / 4) * 4];
#pragma unroll
    for (int i = 0; i < ((AW + 3) / 4) * 4; i++) aw[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) aw[i] = task_word(P, a, r, i);
    uint32_t idw[4];
    load16(a.ids + 16 * (size_t)r, idw);
#pragma unroll
    for (int i = 0; i < 4; i++) aw[8 + i] = __builtin_bswap32(idw[i]);
    const uint64_t tm = a.times[r];
    aw[12] = (uint32_t)(tm >> 32);
    aw[13] = (uint32_t)tm;
    aw[14] = PUB;
    if constexpr (PUB > 0) {
      uint32_t pw[PUB / 4];
#pragma unroll
      for (int i = 0; i < PUB / 16; i++) load16(a.pubs + (size_t)PUB * r + 16 * i, pw + 4 * i);
#pragma unroll
      for (int i = 0; i < PUB / 4; i++) aw[15 + i] = __builtin_bswap32(pw[i]);
    }
    aad_len = 60 + PUB;
#pragma unroll
    for (int b = 0; b < (AW + 3) / 4; b++) ghash_block(y, aw + 4 * b, H);
  } else {
    // a per-report length past the row stride would authenticate the next rows (or read past
    // the buffer): such a report fails to open, and only its own row is read
    const uint32_t al = a.aad_len[r];
    ok = ok && al <= a.aad_stride;
    aad_len = al <= a.aad_stride ? al : a.aad_stride;
    const uint8_t* ap = a.aad + (size_t)a.aad_stride * r;
    for (uint32_t off = 0; off < aad_len; off += 16) {
      uint32_t xw[4];
      load16(ap + off, xw);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t lo = off + 4 * i;  // bytes past the end are zero
        const uint32_t keep = lo + 4 <= aad_len ? 0xffffffffu
                              : lo >= aad_len  ? 0u
                                               : (1u << (8 * (aad_len - lo))) - 1u;
        xw[i] = __builtin_bswap32(xw[i] & keep);
      }
      ghash_block(y, xw, H);
    }
  }
  const uint32_t ct_len = a.ct_len[r];
  const bool len_ok = ct_len >= 16 && ct_len <= a.ct_stride;
  ok = ok && len_ok;
  pt_len = len_ok ? ct_len - 16 : 0;
  const uint8_t* cp = a.ct + (size_t)a.ct_stride * r;
  pp = a.pt + (size_t)a.ct_stride * r;
  uint32_t ctr[4];
#pragma unroll
  for (int i = 0; i < 3; i++) ctr[i] = __builtin_bswap32(noncew[i]);
  for (uint32_t off = 0, blk = 2; off < pt_len; off += 16, blk++) {
    uint32_t cw[4], ks[4];
    load16(cp + off, cw);
    ctr[3] = __builtin_bswap32(blk);
    aes_encrypt<NR>(T, rk, ctr, ks);
    uint32_t xw[4], pw[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t lo = off + 4 * i;
      const uint32_t keep = lo + 4 <= pt_len ? 0xffffffffu
                            : lo >= pt_len  ? 0u
                                            : (1u << (8 * (pt_len - lo))) - 1u;
      xw[i] = __builtin_bswap32(cw[i] & keep);
      pw[i] = (cw[i] ^ ks[i]) & keep;
    }
    ghash_block(y, xw, H);
    *(uint4*)(pp + off) = make_uint4(pw[0], pw[1], pw[2], pw[3]);
  }
  {  // lengths block, tag
    const uint32_t lw[4] = {0, aad_len * 8, 0, pt_len * 8};
    ghash_block(y, lw, H);
    ctr[3] = __builtin_bswap32(1u);
    uint32_t ek[4];
    aes_encrypt<NR>(T, rk, ctr, ek);
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t t = __builtin_bswap32(y[i]) ^ ek[i];  // expected tag, LE-packed bytes
      uint32_t got = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) got |= (uint32_t)cp[pt_len + 4 * i + j] << (8 * j);
      diff |= t ^ got;
    }
    ok = ok && diff == 0;
  }
  };
  if (AEAD == 3) {
  // ---- ChaCha20Poly1305 open (AEAD 3, RFC 8439 2.8), sequence number 0 -------------------
  uint32_t ckey[8], cnon[3];
#pragma unroll
  for (int i = 0; i < 8; i++) ckey[i] = __builtin_bswap32(keyw[i]);  // key bytes as LE words
#pragma unroll
  for (int i = 0; i < 3; i++) cnon[i] = __builtin_bswap32(noncew[i]);
  Poly1305 mac;
  {
    uint32_t b0[16];
    chacha20_block(ckey, 0, cnon, b0);  // Poly1305 one-time key = first 32 bytes of block 0
    poly_init(mac, b0);
  }
  if constexpr (MODE == 1) {
    // InputShareAad (as the GCM path builds it), zero padded to 16 bytes, as LE words
    constexpr int AW = (60 + PUB + 3) / 4;
    uint32_t aw[((AW + 3) / 4) * 4];
#pragma unroll
    for (int i = 0; i < ((AW + 3) / 4) * 4; i++) aw[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) aw[i] = __builtin_bswap32(task_word(P, a, r, i));
    uint32_t idw[4];
    load16(a.ids + 16 * (size_t)r, idw);
#pragma unroll
    for (int i = 0; i < 4; i++) aw[8 + i] = idw[i];
    const uint64_t tm = a.times[r];
    aw[12] = __builtin_bswap32((uint32_t)(tm >> 32));
    aw[13] = __builtin_bswap32((uint32_t)tm);
    aw[14] = __builtin_bswap32((uint32_t)PUB);
    if constexpr (PUB > 0) {
      uint32_t pw[PUB / 4];
#pragma unroll
      for (int i = 0; i < PUB / 16; i++) load16(a.pubs + (size_t)PUB * r + 16 * i, pw + 4 * i);
#pragma unroll
      for (int i = 0; i < PUB / 4; i++) aw[15 + i] = pw[i];
    }
    aad_len = 60 + PUB;
#pragma unroll
    for (int b = 0; b < (AW + 3) / 4; b++) poly_block(mac, aw + 4 * b);
  } else {
    // a per-report length past the row stride would authenticate the next rows (or read past
    // the buffer): such a report fails to open, and only its own row is read
    const uint32_t al = a.aad_len[r];
    ok = ok && al <= a.aad_stride;
    aad_len = al <= a.aad_stride ? al : a.aad_stride;
    const uint8_t* ap = a.aad + (size_t)a.aad_stride * r;
    for (uint32_t off = 0; off < aad_len; off += 16) {
      uint32_t xw[4];
      load16(ap + off, xw);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t lo = off + 4 * i;  // bytes past the end are zero
        const uint32_t keep = lo + 4 <= aad_len ? 0xffffffffu
                              : lo >= aad_len  ? 0u
                                               : (1u << (8 * (aad_len - lo))) - 1u;
        xw[i] &= keep;
      }
      poly_block(mac, xw);
    }
  }
  const uint32_t ct_len = a.ct_len[r];
  const bool len_ok = ct_len >= 16 && ct_len <= a.ct_stride;
  ok = ok && len_ok;
  pt_len = len_ok ? ct_len - 16 : 0;
  const uint8_t* cp = a.ct + (size_t)a.ct_stride * r;
  pp = a.pt + (size_t)a.ct_stride * r;
  for (uint32_t off0 = 0, blk = 1; off0 < pt_len; off0 += 64, blk++) {
    uint32_t ks[16];
    chacha20_block(ckey, blk, cnon, ks);
#pragma unroll
    for (int c4 = 0; c4 < 4; c4++) {
      const uint32_t off = off0 + 16 * c4;
      if (off >= pt_len) break;
      uint32_t cw[4], xw[4], pw[4];
      load16(cp + off, cw);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t lo = off + 4 * i;
        const uint32_t keep = lo + 4 <= pt_len ? 0xffffffffu
                              : lo >= pt_len  ? 0u
                                              : (1u << (8 * (pt_len - lo))) - 1u;
        xw[i] = cw[i] & keep;
        pw[i] = (cw[i] ^ ks[4 * c4 + i]) & keep;
      }
      poly_block(mac, xw);
      *(uint4*)(pp + off) = make_uint4(pw[0], pw[1], pw[2], pw[3]);
    }
  }
  {  // le64(aad_len) || le64(ct_len), tag
    const uint32_t lw[4] = {aad_len, 0, pt_len, 0};
    poly_block(mac, lw);
    uint32_t tag[4];
    poly_finish(mac, tag);
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      uint32_t got = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) got |= (uint32_t)cp[pt_len + 4 * i + j] << (8 * j);
      diff |= tag[i] ^ got;
    }
    ok = ok && diff == 0;
  }
  } else if (AEAD == 2) {
    gcm_open(std::integral_constant<int, 14>{});
  } else {
    gcm_open(std::integral_constant<int, 10>{});
  }
  if constexpr (MODE == 0) {
    a.status[r] = ok ? JANUS_HPKE_OK : JANUS_HPKE_DECRYPT_ERROR;
  } else {
    // PlaintextInputShare::get_decoded + extension checks + helper share length
    // (aggregator.rs:1893-1990): extensions (u16-prefixed list of {u16 type, u16-prefixed
    // data}), payload (u32-prefixed) -- exact total length.
    uint8_t st = ok ? JANUS_HPKE_OK : JANUS_HPKE_DECRYPT_ERROR;
    uint32_t pay = 0;
    if (ok) {
      bool good = pt_len >= 2;
      const uint32_t el = good ? ((uint32_t)pp[0] << 8 | pp[1]) : 0u;
      good = good && 2 + el <= pt_len;
      uint32_t q = 2;
      bool taskprov_seen = false, taskprov_ok = false, tbd_seen = false;
      while (good && q < 2 + el) {
        if (q + 4 > 2 + el) {
          good = false;
          break;
        }
        const uint32_t ty = (uint32_t)pp[q] << 8 | pp[q + 1];
        const uint32_t dl = (uint32_t)pp[q + 2] << 8 | pp[q + 3];
        if (q + 4 + dl > 2 + el || (ty != 0 && ty != 0xFF00u)) {
          good = false;
          break;
        }
        // ExtensionType has two values, so a duplicate is a second Tbd or Taskprov
        if (ty == 0) {
          good = good && !tbd_seen;
          tbd_seen = true;
        } else {
          good = good && !taskprov_seen;
          taskprov_seen = true;
          taskprov_ok = dl == 0;
        }
        q += 4 + dl;
      }
      q = 2 + el;
      good = good && q + 4 <= pt_len;
      const uint32_t pl = good ? ((uint32_t)pp[q] << 24 | (uint32_t)pp[q + 1] << 16 |
                                  (uint32_t)pp[q + 2] << 8 | pp[q + 3])
                               : 0u;
      good = good && q + 4 + pl == pt_len;
      good = good && (a.require_taskprov ? taskprov_ok : !taskprov_seen);
      good = good && pl == a.share_len;
      st = good ? JANUS_HPKE_OK : JANUS_HPKE_INVALID_MESSAGE;
      pay = q + 4;
    }
    uint8_t* so = a.shares + (size_t)a.share_len * r;
    for (uint32_t i = 0; i < a.share_len; i++) so[i] = st == JANUS_HPKE_OK ? pp[pay + i] : 0;
    a.status[r] = st;
  }
}

// -------------------------------------------------------------------------------------
// Host side
// -------------------------------------------------------------------------------------
namespace {

void sha256_host(const std::vector<uint8_t>& msg, uint8_t out[32]) {
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  std::vector<uint8_t> m = msg;
  const uint64_t bits = (uint64_t)msg.size() * 8;
  m.push_back(0x80);
  while (m.size() % 64 != 56) m.push_back(0);
  for (int i = 7; i >= 0; i--) m.push_back((uint8_t)(bits >> (8 * i)));
  for (size_t o = 0; o < m.size(); o += 64) sha256_compress_host(st, m.data() + o);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(st[i] >> (24 - 8 * j));
}

void hmac_host(const uint8_t* key, size_t klen, const std::vector<uint8_t>& msg, uint8_t out[32]) {
  uint8_t k[64] = {0};
  memcpy(k, key, klen);  // klen <= 64 here
  std::vector<uint8_t> in(64), outer(64);
  for (int i = 0; i < 64; i++) in[i] = k[i] ^ 0x36, outer[i] = k[i] ^ 0x5c;
  in.insert(in.end(), msg.begin(), msg.end());
  uint8_t ih[32];
  sha256_host(in, ih);
  outer.insert(outer.end(), ih, ih + 32);
  sha256_host(outer, out);
}

// SHA-512 / SHA-384 and their HMAC on the host (key_schedule_context of KDFs 0x0002 / 0x0003)
void sha512_host(const std::vector<uint8_t>& msg, bool s384, uint8_t* out) {
  uint64_t st[8];
  for (int i = 0; i < 8; i++) st[i] = s384 ? sha512d::IV384[i] : sha512d::IV512[i];
  std::vector<uint8_t> m = msg;
  const uint64_t bits = (uint64_t)msg.size() * 8;
  m.push_back(0x80);
  while (m.size() % 128 != 112) m.push_back(0);
  for (int i = 0; i < 8; i++) m.push_back(0);
  for (int i = 7; i >= 0; i--) m.push_back((uint8_t)(bits >> (8 * i)));
  for (size_t o = 0; o < m.size(); o += 128) {
    uint64_t w[16];
    for (int i = 0; i < 16; i++) {
      w[i] = 0;
      for (int j = 0; j < 8; j++) w[i] = w[i] << 8 | m[o + 8 * i + j];
    }
    sha512d::compress(st, w);
  }
  for (int i = 0; i < (s384 ? 6 : 8); i++)
    for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(st[i] >> (56 - 8 * j));
}
void hmac512_host(const uint8_t* key, size_t klen, const std::vector<uint8_t>& msg, bool s384,
                  uint8_t* out) {
  uint8_t k[128] = {0};
  memcpy(k, key, klen);  // klen <= 128 here
  std::vector<uint8_t> in(128), outer(128);
  for (int i = 0; i < 128; i++) in[i] = k[i] ^ 0x36, outer[i] = k[i] ^ 0x5c;
  in.insert(in.end(), msg.begin(), msg.end());
  uint8_t ih[64];
  sha512_host(in, s384, ih);
  outer.insert(outer.end(), ih, ih + (s384 ? 48 : 64));
  sha512_host(outer, s384, out);
}

std::vector<uint8_t> cat(std::initializer_list<std::vector<uint8_t>> parts) {
  std::vector<uint8_t> r;
  for (auto& p : parts) r.insert(r.end(), p.begin(), p.end());
  return r;
}
std::vector<uint8_t> bytes(const char* s) { return std::vector<uint8_t>(s, s + strlen(s)); }

// suite_id = "HPKE" || kem_id || kdf_id || aead_id (RFC 9180 5.1)
std::vector<uint8_t> hpke_suite(uint16_t kem, uint16_t kdf, uint16_t aead) {
  return {'H', 'P', 'K', 'E', (uint8_t)(kem >> 8), (uint8_t)kem, (uint8_t)(kdf >> 8), (uint8_t)kdf,
          (uint8_t)(aead >> 8), (uint8_t)aead};
}
// P-521 group order n (SEC 2), big-endian
const uint8_t kP521N[66] = {
    0x01, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xff, 0xff, 0xff, 0xff, 0xff, 0xfa, 0x51, 0x86, 0x87, 0x83, 0xbf, 0x2f, 0x96, 0x6b,
    0x7f, 0xcc, 0x01, 0x48, 0xf7, 0x09, 0xa5, 0xd0, 0x3b, 0xb5, 0xc9, 0xb8, 0x89, 0x9c,
    0x47, 0xae, 0xbb, 0x6f, 0xb7, 0x1e, 0x91, 0x38, 0x64, 0x09};
// 1 <= sk < n for a big-endian scalar of the group order's length
bool scalar_in_range(const uint8_t* sk, const uint8_t* n, size_t len) {
  bool zero = true, below = false, decided = false;
  for (size_t i = 0; i < len; i++) {
    zero = zero && sk[i] == 0;
    if (!decided && sk[i] != n[i]) below = sk[i] < n[i], decided = true;
  }
  return !zero && below;
}
// KEM sizes (RFC 9180 7.1): private key, Nenc (= Npk); 0 = not a KEM this opener implements
size_t kem_nsk(uint16_t kem) {
  return kem == 0x20 || kem == 0x10 ? 32 : kem == 0x21 ? 56 : kem == 0x12 ? 66 : kem == 0x11 ? 48 : 0;
}
size_t kem_nenc(uint16_t kem) {
  return kem == 0x20 ? 32 : kem == 0x10 ? 65 : kem == 0x21 ? 56 : kem == 0x12 ? 133 : kem == 0x11 ? 97 : 0;
}
// P-384 group order n (SEC 2 2.5.1), big-endian
const uint8_t kP384N[48] = {
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xc7, 0x63, 0x4d, 0x81, 0xf4, 0x37, 0x2d, 0xdf,
    0x58, 0x1a, 0x0d, 0xb2, 0x48, 0xb0, 0xa7, 0x7a, 0xec, 0xec, 0x19, 0x6a, 0xcc, 0xc5, 0x29, 0x73};
// P-256 group order n (SEC 2), big-endian
const uint8_t kP256N[32] = {0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x00, 0xff, 0xff, 0xff,
                            0xff, 0xff, 0xff, 0xff, 0xff, 0xbc, 0xe6, 0xfa, 0xad, 0xa7, 0x17,
                            0x9e, 0x84, 0xf3, 0xb9, 0xca, 0xc2, 0xfc, 0x63, 0x25, 0x51};

uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

}  // namespace

// Regular signed window recoding (w = 4) of a P-256 private key for p256::ecdh: k' = sk when sk
// is odd, else n - sk (same x-coordinate of k'P), then 63 digits d = (k' mod 32) - 16 (odd, in
// [-15, 15]) with k' <- (k' - d) / 16, which stays odd, and the remaining odd k' < 16 on top.
static void p256_recode(const uint32_t sk[8], int8_t dig[88]) {
  uint32_t k[8];
  memcpy(k, sk, sizeof(k));
  if (!(k[0] & 1u)) {
    int64_t br = 0;
    for (int i = 0; i < 8; i++) {
      const uint32_t ni = be32(kP256N + 4 * (7 - i));
      const int64_t t = (int64_t)ni - k[i] + br;
      k[i] = (uint32_t)t;
      br = t >> 32;
    }
  }
  for (int i = 0; i < p256::kDigits - 1; i++) {
    const int d = (int)(k[0] & 31u) - 16;
    dig[i] = (int8_t)d;
    int64_t c = -(int64_t)d;  // k -= d
    for (int j = 0; j < 8; j++) {
      const int64_t t = (int64_t)k[j] + c;
      k[j] = (uint32_t)t;
      c = t >> 32;
    }
    for (int j = 0; j < 8; j++) k[j] = k[j] >> 4 | (j < 7 ? k[j + 1] << 28 : 0u);
  }
  dig[p256::kDigits - 1] = (int8_t)k[0];
  for (int i = p256::kDigits; i < 88; i++) dig[i] = 0;
}

// The same recoding for a key of nw little-endian words against the group order n (nw words):
// ndig - 1 digits of four bits, then the odd top digit (P-521: 131 digits for 521 bits).
static void recode_w4(const uint32_t* sk, const uint32_t* n, int nw, int ndig, int8_t* dig) {
  std::vector<uint32_t> k(sk, sk + nw);
  if (!(k[0] & 1u)) {
    int64_t br = 0;
    for (int i = 0; i < nw; i++) {
      const int64_t t = (int64_t)n[i] - k[i] + br;
      k[i] = (uint32_t)t;
      br = t >> 32;
    }
  }
  for (int i = 0; i < ndig - 1; i++) {
    const int d = (int)(k[0] & 31u) - 16;
    dig[i] = (int8_t)d;
    int64_t c = -(int64_t)d;
    for (int j = 0; j < nw; j++) {
      const int64_t t = (int64_t)k[j] + c;
      k[j] = (uint32_t)t;
      c = t >> 32;
    }
    for (int j = 0; j < nw; j++) k[j] = k[j] >> 4 | (j < nw - 1 ? k[j + 1] << 28 : 0u);
  }
  dig[ndig - 1] = (int8_t)k[0];
}

// X25519 opens of at most this many reports run the ladder on lane pairs (x25519_ladder_pair).
// Interleaved (r06h, HPKE jobs lines, every job checked): at 16 threads (groups of ~3-7k
// reports) 6.50 / 6.54 / 6.64 against 6.37 / 6.11 / 6.43 M/s one lane per report; at 128 threads
// (~30k) the pair loses (19.2 / 21.3 / 19.0 against 21.0 / 24.7 / 24.3 M/s; the helper init line
// 16.2-18.0 against 18.0-19.4) -- its second lane repeats the key schedule and the AEAD, and at two
// waves per SIMD the one-lane ladder's chains already overlap.  A/B builds: 0 = never.
#ifndef JANUS_HPKE_PAIR_MAX
#define JANUS_HPKE_PAIR_MAX 8192
#endif
struct janus_hpke_opener {
  int device = 0;
  int coalesce = 1;  // host-buffer opens through the executor (janus_hpke_executor_control)
  int pair_max = JANUS_HPKE_PAIR_MAX;  // lane-pair ladder for opens of at most this many reports
  hipStream_t stream = nullptr;
  HpkeParams P;
  uint8_t* d_pt = nullptr;
  size_t pt_cap = 0;
  std::mutex mu;
  int timing = 0;
  double ms = 0;
  uint32_t launches = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
};

#define HCHK(x)                                                                       \
  do {                                                                                \
    hipError_t _e = (x);                                                              \
    if (_e != hipSuccess) {                                                           \
      fprintf(stderr, "janus_hpke: HIP error %s at %s:%d\n", hipGetErrorString(_e),   \
              __FILE__, __LINE__);                                                    \
      return JANUS_HPKE_EDEVICE;                                                      \
    }                                                                                 \
  } while (0)

extern "C" {

int janus_hpke_opener_create(uint16_t kem_id, uint16_t kdf_id, uint16_t aead_id,
                             const uint8_t* private_key, size_t private_key_len,
                             const uint8_t* public_key, size_t public_key_len,
                             const uint8_t* info, size_t info_len, int device,
                             janus_hpke_opener** out) {
  if (!out || !private_key || !public_key || (info_len && !info)) return JANUS_HPKE_EINVAL;
  *out = nullptr;
  if (!kem_nsk(kem_id) || kdf_id < JANUS_HPKE_KDF_HKDF_SHA256 ||
      kdf_id > JANUS_HPKE_KDF_HKDF_SHA512 ||
      (aead_id != JANUS_HPKE_AEAD_AES_128_GCM && aead_id != JANUS_HPKE_AEAD_AES_256_GCM &&
       aead_id != JANUS_HPKE_AEAD_CHACHA20_POLY1305))
    return JANUS_HPKE_EUNSUPPORTED;
  if (private_key_len != kem_nsk(kem_id) || public_key_len != kem_nenc(kem_id))
    return JANUS_HPKE_EINVAL;
  // DeserializePrivateKey (RFC 9180 7.1.2): the NIST curves need 1 <= sk < n; pkRm uncompressed
  if (kem_id == JANUS_HPKE_KEM_P256_HKDF_SHA256 &&
      (!scalar_in_range(private_key, kP256N, 32) || public_key[0] != 0x04))
    return JANUS_HPKE_EINVAL;
  if (kem_id == JANUS_HPKE_KEM_P521_HKDF_SHA512 &&
      (!scalar_in_range(private_key, kP521N, 66) || public_key[0] != 0x04))
    return JANUS_HPKE_EINVAL;
  if (kem_id == JANUS_HPKE_KEM_P384_HKDF_SHA384 &&
      (!scalar_in_range(private_key, kP384N, 48) || public_key[0] != 0x04))
    return JANUS_HPKE_EINVAL;
  auto* o = new janus_hpke_opener();
  o->device = device;
  memset(&o->P, 0, sizeof(o->P));
  o->P.kem = kem_id;
  o->P.kdf = kdf_id;
  o->P.aead = aead_id;
  if (kem_id == JANUS_HPKE_KEM_X25519_HKDF_SHA256) {
    uint8_t k[32];
    memcpy(k, private_key, 32);
    k[0] &= 248;  // decodeScalar25519 (RFC 7748 section 5)
    k[31] &= 127;
    k[31] |= 64;
    for (int i = 0; i < 8; i++) o->P.sk[i] = le32(k + 4 * i), o->P.pk[i] = le32(public_key + 4 * i);
  } else if (kem_id == JANUS_HPKE_KEM_P256_HKDF_SHA256) {
    for (int i = 0; i < 8; i++) o->P.sk[i] = be32(private_key + 4 * (7 - i));  // LE limbs
    memcpy(o->P.pk65, public_key, 65);
    p256_recode(o->P.sk, o->P.p256_dig);
  } else if (kem_id == JANUS_HPKE_KEM_X448_HKDF_SHA512) {
    uint8_t k[56];
    memcpy(k, private_key, 56);
    k[0] &= 252;  // decodeScalar448 (RFC 7748 section 5)
    k[55] |= 128;
    for (int i = 0; i < 14; i++) o->P.sk448[i] = le32(k + 4 * i);
    memcpy(o->P.pkraw, public_key, 56);
  } else if (kem_id == JANUS_HPKE_KEM_P384_HKDF_SHA384) {  // 12 LE words, recoded against n
    uint32_t kw[12], nw[12];
    for (int i = 0; i < 12; i++)
      kw[i] = be32(private_key + 4 * (11 - i)), nw[i] = be32(kP384N + 4 * (11 - i));
    recode_w4(kw, nw, 12, P384_DIGITS, o->P.p384_dig);
    memcpy(o->P.pkraw, public_key, 97);
  } else {  // P-521: the 66-byte big-endian scalar as 17 LE words, recoded against n
    uint8_t kb[68] = {0}, nb[68] = {0};
    memcpy(kb + 2, private_key, 66);
    memcpy(nb + 2, kP521N, 66);
    uint32_t kw[17], nw[17];
    for (int i = 0; i < 17; i++) kw[i] = be32(kb + 4 * (16 - i)), nw[i] = be32(nb + 4 * (16 - i));
    recode_w4(kw, nw, 17, P521_DIGITS, o->P.p521_dig);
    memcpy(o->P.pkraw, public_key, 133);
  }
  // key_schedule_context = mode_base || LabeledExtract("", "psk_id_hash", "") ||
  //                        LabeledExtract("", "info_hash", info)        (RFC 9180 5.1)
  std::vector<uint8_t> inf(info, info + info_len);
  const std::vector<uint8_t> suite = hpke_suite(kem_id, kdf_id, aead_id);
  const std::vector<uint8_t> psk_msg = cat({bytes("HPKE-v1"), suite, bytes("psk_id_hash")}),
                             info_msg = cat({bytes("HPKE-v1"), suite, bytes("info_hash"), inf});
  if (kdf_id == JANUS_HPKE_KDF_HKDF_SHA256) {
    uint8_t ksc[68] = {0};
    hmac_host(nullptr, 0, psk_msg, ksc + 1);
    hmac_host(nullptr, 0, info_msg, ksc + 33);
    for (int i = 0; i < 17; i++) o->P.ksc[i] = be32(ksc + 4 * i);
  } else {
    const bool s384 = kdf_id == JANUS_HPKE_KDF_HKDF_SHA384;
    const size_t nh = s384 ? 48 : 64;
    uint8_t ksc[136] = {0};
    hmac512_host(nullptr, 0, psk_msg, s384, ksc + 1);
    hmac512_host(nullptr, 0, info_msg, s384, ksc + 1 + nh);
    for (int i = 0; i < 17; i++) {
      uint64_t w = 0;
      for (int j = 0; j < 8; j++) w = w << 8 | ksc[8 * i + j];
      o->P.ksc64[i] = w;
    }
  }
  // HMAC midstates of the empty key: SHA-256 (eae_prk of the X25519 / P-256 KEMs) and SHA-512
  // (eae_prk of the X448 / P-521 KEMs, whose KDF is HKDF-SHA512 whatever the key schedule's)
  uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint8_t b36[64], b5c[64];
  memset(b36, 0x36, 64);
  memset(b5c, 0x5c, 64);
  memcpy(o->P.ipad0, iv, 32);
  memcpy(o->P.opad0, iv, 32);
  sha256_compress_host(o->P.ipad0, b36);
  sha256_compress_host(o->P.opad0, b5c);
  {
    HmacKey64 k0;
    hmac64_key(k0, nullptr, 0, false);
    memcpy(o->P.ipad0_64, k0.ist, 64);
    memcpy(o->P.opad0_64, k0.ost, 64);
    hmac64_key(k0, nullptr, 0, true);  // HKDF-SHA384 (eae_prk of the P-384 KEM)
    memcpy(o->P.ipad0_384, k0.ist, 64);
    memcpy(o->P.opad0_384, k0.ost, 64);
  }
  DeviceGuard dg_(device);
  if (dg_.rc != hipSuccess ||
      hipStreamCreateWithFlags(&o->stream, hipStreamNonBlocking) != hipSuccess) {
    delete o;
    return JANUS_HPKE_EDEVICE;
  }
  ws_warm(device);  // the GPU's pooled streams, before any job runs
  *out = o;
  return JANUS_HPKE_SUCCESS;
}

void janus_hpke_opener_destroy(janus_hpke_opener* o) {
  if (!o) return;
  DeviceGuard dg_(o->device);
  (void)hipStreamSynchronize(o->stream);
  if (o->d_pt) (void)hipFree(o->d_pt);
  for (auto& e : o->pending) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  (void)hipStreamDestroy(o->stream);
  delete o;
}

int janus_hpke_set_timing(janus_hpke_opener* o, int on) {
  if (!o) return JANUS_HPKE_EINVAL;
  std::lock_guard<std::mutex> lk(o->mu);
  o->timing = on;
  o->ms = 0;
  o->launches = 0;
  return JANUS_HPKE_SUCCESS;
}

int janus_hpke_timing(janus_hpke_opener* o, double* ms_total, uint32_t* launches) {
  if (!o) return JANUS_HPKE_EINVAL;
  std::lock_guard<std::mutex> lk(o->mu);
  for (auto& e : o->pending) {
    float ms = 0;
    HCHK(hipEventSynchronize(e.second));
    HCHK(hipEventElapsedTime(&ms, e.first, e.second));
    o->ms += ms;
    o->launches++;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  o->pending.clear();
  if (ms_total) *ms_total = o->ms;
  if (launches) *launches = o->launches;
  return JANUS_HPKE_SUCCESS;
}

}  // extern "C"

static int launch_open(janus_hpke_opener* o, int mode, int pub, const OpenArgs& a,
                       hipStream_t st) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (o->timing) {
    HCHK(hipEventCreate(&e0));
    HCHK(hipEventCreate(&e1));
    HCHK(hipEventRecord(e0, st));
  }
  const uint32_t blocks = (a.n + 255) / 256;
#define JANUS_HPKE_LAUNCH(KE)                                    \
  if (mode == 0)                                                 \
    k_hpke_open<0, 0, KE><<<blocks, 256, 0, st>>>(o->P, a);      \
  else if (pub == 32)                                            \
    k_hpke_open<1, 32, KE><<<blocks, 256, 0, st>>>(o->P, a);     \
  else                                                           \
    k_hpke_open<1, 0, KE><<<blocks, 256, 0, st>>>(o->P, a);
  // small X25519 batches (the executors' groups) on lane pairs: below ~2 waves per SIMD the
  // one-lane open leaves SIMDs idle and each lane's ladder is a long dependent chain
  const bool pair = o->P.kem == JANUS_HPKE_KEM_X25519_HKDF_SHA256 && mode == 1 &&
                    a.n <= (uint32_t)o->pair_max;
  if (pair) {
    const uint32_t b2 = (2 * a.n + 255) / 256;
    if (pub == 32)
      k_hpke_open<1, 32, 0x20, true><<<b2, 256, 0, st>>>(o->P, a);
    else
      k_hpke_open<1, 0, 0x20, true><<<b2, 256, 0, st>>>(o->P, a);
  } else if (o->P.kem == JANUS_HPKE_KEM_P256_HKDF_SHA256) {
    JANUS_HPKE_LAUNCH(0x10)
  } else if (o->P.kem == JANUS_HPKE_KEM_X448_HKDF_SHA512) {
    JANUS_HPKE_LAUNCH(0x21)
  } else if (o->P.kem == JANUS_HPKE_KEM_P521_HKDF_SHA512) {
    JANUS_HPKE_LAUNCH(0x12)
  } else if (o->P.kem == JANUS_HPKE_KEM_P384_HKDF_SHA384) {
    JANUS_HPKE_LAUNCH(0x11)
  } else {
    JANUS_HPKE_LAUNCH(0x20)
  }
#undef JANUS_HPKE_LAUNCH
  HCHK(hipGetLastError());
  if (o->timing) {
    HCHK(hipEventRecord(e1, st));
    o->pending.push_back({e0, e1});
  }
  return JANUS_HPKE_SUCCESS;
}

static int ensure_pt(janus_hpke_opener* o, size_t bytes) {
  if (bytes <= o->pt_cap) return JANUS_HPKE_SUCCESS;
  if (o->d_pt) HCHK(hipFree(o->d_pt));
  o->d_pt = nullptr;
  HCHK(hipMalloc((void**)&o->d_pt, bytes));
  o->pt_cap = bytes;
  return JANUS_HPKE_SUCCESS;
}

// ---- executor hooks (prio3_runtime.h) ----
int hpke_opener_device(const janus_hpke_opener* o) { return o->device; }
size_t hpke_opener_nenc(const janus_hpke_opener* o) { return kem_nenc((uint16_t)o->P.kem); }
uint64_t hpke_opener_key(const janus_hpke_opener* o) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
  mix((uint64_t)(uintptr_t)o);
  mix((uint64_t)o->timing);
  mix((uint64_t)o->pair_max);
  return h;
}

// the open of a sealed-input prepare group (engine_group_issue), on the group's stream
int hpke_open_group_launch(janus_hpke_opener* o, const HpkeGroupArgs& g, hipStream_t st) {
  OpenArgs a{};
  a.n = g.n;
  a.ct_stride = g.ct_stride;
  a.share_len = g.share_len;
  a.require_taskprov = g.require_taskprov;
  a.enc = g.enc;
  a.ct = g.ct;
  a.ct_len = g.ct_len;
  a.ids = g.ids;
  a.times = g.times;
  a.pubs = g.pubs;
  a.pt = g.pt;
  a.shares = g.shares;
  a.status = g.status;
  a.task_slot = g.task_slot;
  a.task_tab = g.task_tab;
  std::lock_guard<std::mutex> lk(o->mu);  // o->P and the timing list
  return launch_open(o, 1, (int)g.pub_len, a, st) == JANUS_HPKE_SUCCESS ? PRIO3_OK : PRIO3_EDEVICE;
}

uint64_t hpke_group_key(const HpkeJob* j) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
  mix((uint64_t)(uintptr_t)j->o);
  mix((uint64_t)j->o->pair_max);
  mix(j->ct_stride);
  mix(j->pub_len);
  mix(j->share_len);
  mix((uint64_t)j->require_taskprov);
  mix((uint64_t)j->o->timing);
  return h;
}

void hpke_layout(const HpkeJob* j, uint32_t cap, HpkeLayout* L) {
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  L->nenc = (uint32_t)kem_nenc((uint16_t)j->o->P.kem);
  size_t off = 0;
  L->off_enc = off;
  off += up((size_t)L->nenc * cap);
  L->off_ct = off;
  off += up((size_t)j->ct_stride * cap);
  L->off_len = off;
  off += up(4 * (size_t)cap);
  L->off_ids = off;
  off += up(16 * (size_t)cap);
  L->off_times = off;
  off += up(8 * (size_t)cap);
  L->off_pub = off;
  off += up((size_t)j->pub_len * cap);
  L->slot_off = off;
  off += up(2 * (size_t)cap);
  L->tab_off = off;
  off += up(32 * (size_t)HPKE_MAX_TASKS);
  L->shares_off = off;
  off += up((size_t)j->share_len * cap + 1);
  L->status_off = off;
  off += up(cap);
  L->pt_off = off;
  off += up((size_t)j->ct_stride * cap);
  L->bytes = off;
}

// The group's per-field inputs to a device mirror (pinned-memory DMA), the open kernel (its AAD
// task IDs from the group's table), the helper shares and statuses back into the staging.
int hpke_group_issue(const HpkeJob& pj, const HpkeLayout& L, const uint8_t* stg, uint8_t* out,
                     uint32_t n, hipStream_t* st_out, Slab** slab_out, bool own_queue) {
  janus_hpke_opener* o = pj.o;
  *st_out = nullptr;
  *slab_out = nullptr;
  DeviceGuard dg_(o->device);
  HCHK(dg_.rc);
  hipStream_t st = own_queue ? ws_exec_stream_get(o->device) : ws_stream_get(o->device);
  if (!st) return JANUS_HPKE_EDEVICE;
  int rc = JANUS_HPKE_SUCCESS;
  Slab* sl = ws_acquire(o->device, L.bytes, st, &rc);
  if (!sl) {
    ws_exec_stream_put(o->device, st);
    return rc;
  }
  uint8_t* b = sl->base;
  const struct {
    size_t off, bytes;
  } f[] = {{L.off_enc, (size_t)L.nenc * n},    {L.off_ct, (size_t)pj.ct_stride * n},
           {L.off_len, 4 * (size_t)n},         {L.off_ids, 16 * (size_t)n},
           {L.off_times, 8 * (size_t)n},       {L.off_pub, (size_t)pj.pub_len * n},
           {L.slot_off, 2 * (size_t)n},        {L.tab_off, 32 * (size_t)HPKE_MAX_TASKS}};
  for (auto& x : f)
    if (rc == JANUS_HPKE_SUCCESS && x.bytes &&
        hipMemcpyAsync(b + x.off, stg + x.off, x.bytes, hipMemcpyHostToDevice, st) != hipSuccess)
      rc = JANUS_HPKE_EDEVICE;
  if (rc == JANUS_HPKE_SUCCESS) {
    OpenArgs a{};
    a.n = n;
    a.ct_stride = pj.ct_stride;
    a.share_len = pj.share_len;
    a.require_taskprov = pj.require_taskprov;
    a.enc = b + L.off_enc;
    a.ct = b + L.off_ct;
    a.ct_len = (const uint32_t*)(b + L.off_len);
    a.ids = b + L.off_ids;
    a.times = (const uint64_t*)(b + L.off_times);
    a.pubs = pj.pub_len ? b + L.off_pub : nullptr;
    a.pt = b + L.pt_off;
    a.shares = b + L.shares_off;
    a.status = b + L.status_off;
    a.task_slot = (const uint16_t*)(b + L.slot_off);
    a.task_tab = (const uint32_t*)(b + L.tab_off);
    std::lock_guard<std::mutex> lk(o->mu);  // o->P and the timing list
    rc = launch_open(o, 1, (int)pj.pub_len, a, st);
  }
  if (rc == JANUS_HPKE_SUCCESS &&
      (hipMemcpyAsync(out + L.shares_off, b + L.shares_off, (size_t)pj.share_len * n,
                      hipMemcpyDeviceToHost, st) != hipSuccess ||
       hipMemcpyAsync(out + L.status_off, b + L.status_off, n, hipMemcpyDeviceToHost, st) !=
           hipSuccess))
    rc = JANUS_HPKE_EDEVICE;
  if (rc != JANUS_HPKE_SUCCESS) {
    (void)hipStreamSynchronize(st);
    ws_release(sl, st);
    ws_exec_stream_put(o->device, st);
    return rc;
  }
  *st_out = st;
  *slab_out = sl;
  return JANUS_HPKE_SUCCESS;
}

extern "C" {

int janus_hpke_open_input_shares_device(janus_hpke_opener* o, uint32_t n,
                                        const uint8_t task_id[32], const uint8_t* d_enc,
                                        const uint8_t* d_ct, const uint32_t* d_ct_len,
                                        uint32_t ct_stride, const uint8_t* d_report_ids,
                                        const uint64_t* d_times, const uint8_t* d_public_shares,
                                        uint32_t public_share_len, uint32_t helper_share_len,
                                        int require_taskprov, uint8_t* d_helper_shares,
                                        uint8_t* d_status, void* stream) {
  if (!o || !task_id) return JANUS_HPKE_EINVAL;
  if (n == 0) return JANUS_HPKE_SUCCESS;
  if (!d_enc || !d_ct || !d_ct_len || !d_report_ids || !d_times || !d_helper_shares ||
      !d_status || ct_stride == 0 || ct_stride % 16 != 0 ||
      (public_share_len != 0 && public_share_len != 32) || (public_share_len && !d_public_shares))
    return JANUS_HPKE_EINVAL;
  std::lock_guard<std::mutex> lk(o->mu);
  DeviceGuard dg_(o->device);
  HCHK(dg_.rc);
  int rc = ensure_pt(o, (size_t)n * ct_stride);
  if (rc) return rc;
  for (int i = 0; i < 8; i++) o->P.task[i] = be32(task_id + 4 * i);
  OpenArgs a{};
  a.n = n;
  a.ct_stride = ct_stride;
  a.share_len = helper_share_len;
  a.require_taskprov = require_taskprov;
  a.enc = d_enc;
  a.ct = d_ct;
  a.ct_len = d_ct_len;
  a.ids = d_report_ids;
  a.times = d_times;
  a.pubs = d_public_shares;
  a.pt = o->d_pt;
  a.shares = d_helper_shares;
  a.status = d_status;
  return launch_open(o, 1, (int)public_share_len, a, (hipStream_t)stream);
}

int janus_hpke_open_device(janus_hpke_opener* o, uint32_t n, const uint8_t* d_enc,
                           const uint8_t* d_ct, const uint32_t* d_ct_len, uint32_t ct_stride,
                           const uint8_t* d_aad, const uint32_t* d_aad_len, uint32_t aad_stride,
                           uint8_t* d_pt, uint8_t* d_status, void* stream) {
  if (!o) return JANUS_HPKE_EINVAL;
  if (n == 0) return JANUS_HPKE_SUCCESS;
  if (!d_enc || !d_ct || !d_ct_len || !d_pt || !d_status || ct_stride == 0 ||
      ct_stride % 16 != 0 || aad_stride % 16 != 0 || (aad_stride && (!d_aad || !d_aad_len)))
    return JANUS_HPKE_EINVAL;
  std::lock_guard<std::mutex> lk(o->mu);
  DeviceGuard dg_(o->device);
  HCHK(dg_.rc);
  OpenArgs a{};
  a.n = n;
  a.ct_stride = ct_stride;
  a.aad_stride = aad_stride;
  a.enc = d_enc;
  a.ct = d_ct;
  a.ct_len = d_ct_len;
  a.aad = d_aad;
  a.aad_len = d_aad_len;
  a.pt = d_pt;
  a.status = d_status;
  return launch_open(o, 0, 0, a, (hipStream_t)stream);
}

}  // extern "C"

namespace {
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
int up(DevBuf& b, const void* h, size_t bytes, hipStream_t st) {
  if (!h || !bytes) return JANUS_HPKE_SUCCESS;
  HCHK(hipMalloc(&b.p, bytes));
  HCHK(hipMemcpyAsync(b.p, h, bytes, hipMemcpyHostToDevice, st));
  return JANUS_HPKE_SUCCESS;
}
}  // namespace

// Test-only (janus_hpke_selftest_p256): one GF(p256) operation of p256_device.h per element.
__global__ __launch_bounds__(256) void k_selftest_p256(int op, uint32_t n, const uint32_t* a,
                                                       const uint32_t* b, uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  p256::fp x, y, r;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    x.v[k] = a[8 * (size_t)i + k];
    y.v[k] = b[8 * (size_t)i + k];
  }
  switch (op) {
    case 0: r = p256::mul(x, y); break;
    case 1: r = p256::sqr(x); break;
    case 2: r = p256::add(x, y); break;
    case 3: r = p256::sub(x, y); break;
    case 4: r = p256::mul_small(x, 3); break;
    case 5: r = p256::mul_small(x, 8); break;
    default: r = p256::inv(x); break;
  }
#pragma unroll
  for (int k = 0; k < 8; k++) out[8 * (size_t)i + k] = r.v[k];
}

// Test-only (janus_hpke_selftest_field): one operation of the X448 (field 1) or P-521 (field 2)
// field code per element; operands and results as canonical little-endian 32-bit words (14 / 17)
__device__ p521::fp p521_from_words(const uint32_t* w) {
  p521::fp r;
#pragma unroll
  for (int k = 0; k < p521::NL; k++) {
    const int bit = 29 * k, q = bit >> 5, o = bit & 31;
    uint32_t x = w[q] >> o;
    if (o > 3 && q + 1 < 17) x |= w[q + 1] << (32 - o);
    r.v[k] = x & (k == p521::NL - 1 ? p521::M28 : p521::M29);
  }
  return r;
}
__device__ void p521_to_words(const p521::fp& a, uint32_t* w) {
  const p521::fp f = p521::freeze(a);
#pragma unroll
  for (int q = 0; q < 17; q++) w[q] = 0;
#pragma unroll
  for (int k = 0; k < p521::NL; k++) {
    const int bit = 29 * k, q = bit >> 5, o = bit & 31;
    w[q] |= f.v[k] << o;
    if (o > 3 && q + 1 < 17) w[q + 1] |= f.v[k] >> (32 - o);
  }
}
__global__ __launch_bounds__(256) void k_selftest_field(int field, int op, uint32_t n,
                                                        const uint32_t* a, const uint32_t* b,
                                                        uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (field == 1) {
    uint32_t wa[14], wb[14], wr[14];
#pragma unroll
    for (int k = 0; k < 14; k++) wa[k] = a[14 * (size_t)i + k], wb[k] = b[14 * (size_t)i + k];
    const x448::fe x = x448::from_words(wa), y = x448::from_words(wb);
    x448::fe r;
    switch (op) {
      case 0: r = x448::mul(x, y); break;
      case 1: r = x448::sqr(x); break;
      case 2: r = x448::add(x, y); break;
      case 3: r = x448::sub(x, y); break;
      case 4: r = x448::mul_small(x, 39081); break;
      default: r = x448::inv(x); break;
    }
    x448::to_words(r, wr);
#pragma unroll
    for (int k = 0; k < 14; k++) out[14 * (size_t)i + k] = wr[k];
  } else if (field == 3) {  // P-384: operands below 2^384, into / out of Montgomery form
    p384::fp x, y, r;
#pragma unroll
    for (int k = 0; k < 12; k++) x.v[k] = a[12 * (size_t)i + k], y.v[k] = b[12 * (size_t)i + k];
    x = p384::mul_i(x, p384::kR2);
    y = p384::mul_i(y, p384::kR2);
    switch (op) {
      case 0: r = p384::mul(x, y); break;
      case 1: r = p384::sqr(x); break;
      case 2: r = p384::add(x, y); break;
      case 3: r = p384::sub(x, y); break;
      case 4: r = p384::mul_small(x, 8); break;
      default: r = p384::inv(x); break;
    }
    p384::fp one;
#pragma unroll
    for (int k = 0; k < 12; k++) one.v[k] = k ? 0u : 1u;
    r = p384::mul_i(r, one);
#pragma unroll
    for (int k = 0; k < 12; k++) out[12 * (size_t)i + k] = r.v[k];
  } else {
    uint32_t wa[17], wb[17], wr[17];
#pragma unroll
    for (int k = 0; k < 17; k++) wa[k] = a[17 * (size_t)i + k], wb[k] = b[17 * (size_t)i + k];
    const p521::fp x = p521_from_words(wa), y = p521_from_words(wb);
    p521::fp r;
    switch (op) {
      case 0: r = p521::mul(x, y); break;
      case 1: r = p521::sqr(x); break;
      case 2: r = p521::add(x, y); break;
      case 3: r = p521::sub(x, y); break;
      case 4: r = p521::mul_small(x, 8); break;
      default: r = p521::inv(x); break;
    }
    p521_to_words(r, wr);
#pragma unroll
    for (int k = 0; k < 17; k++) out[17 * (size_t)i + k] = wr[k];
  }
}

extern "C" {

int janus_hpke_selftest_field(int field, int op, uint32_t n, const uint32_t* a, const uint32_t* b,
                              uint32_t* out) {
  if (field < 1 || field > 3 || op < 0 || op > 5) return JANUS_HPKE_EINVAL;
  if (n == 0) return JANUS_HPKE_OK;
  const size_t m = (size_t)n * (field == 1 ? 14 : field == 3 ? 12 : 17) * 4;
  void *da = nullptr, *db = nullptr, *dout = nullptr;
  int rc = JANUS_HPKE_OK;
  if (hipMalloc(&da, m) != hipSuccess || hipMalloc(&db, m) != hipSuccess ||
      hipMalloc(&dout, m) != hipSuccess || hipMemcpy(da, a, m, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(db, b, m, hipMemcpyHostToDevice) != hipSuccess) {
    rc = JANUS_HPKE_EDEVICE;
  } else {
    k_selftest_field<<<(n + 255) / 256, 256>>>(field, op, n, (const uint32_t*)da,
                                               (const uint32_t*)db, (uint32_t*)dout);
    if (hipGetLastError() != hipSuccess || hipMemcpy(out, dout, m, hipMemcpyDeviceToHost) != hipSuccess)
      rc = JANUS_HPKE_EDEVICE;
  }
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  return rc;
}

int janus_hpke_open_input_shares(janus_hpke_opener* o, uint32_t n, const uint8_t task_id[32],
                                 const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
                                 uint32_t ct_stride, const uint8_t* report_ids,
                                 const uint64_t* times, const uint8_t* public_shares,
                                 uint32_t public_share_len, uint32_t helper_share_len,
                                 int require_taskprov, uint8_t* helper_shares, uint8_t* status) {
  if (!o || !task_id) return JANUS_HPKE_EINVAL;
  if (n == 0) return JANUS_HPKE_SUCCESS;
  if (!enc || !ct || !ct_len || !report_ids || !times || !helper_shares || !status ||
      ct_stride == 0 || ct_stride % 16 != 0 || (public_share_len != 0 && public_share_len != 32) ||
      (public_share_len && !public_shares))
    return JANUS_HPKE_EINVAL;
  if (o->coalesce) {  // concurrent jobs of every task on this keypair: one launch (exec_hpke)
    HpkeJob j;
    j.o = o;
    j.n = n;
    j.task_id = task_id;
    j.enc = enc;
    j.ct = ct;
    j.ct_len = ct_len;
    j.ct_stride = ct_stride;
    j.ids = report_ids;
    j.times = times;
    j.pubs = public_shares;
    j.pub_len = public_share_len;
    j.share_len = helper_share_len;
    j.require_taskprov = require_taskprov;
    j.shares_out = helper_shares;
    j.status_out = status;
    return exec_hpke(&j);
  }
  DeviceGuard dg_(o->device);
  HCHK(dg_.rc);
  DevBuf de, dc, dl, di, dt, dp, ds, dst;
  int rc;
  const size_t nenc = kem_nenc((uint16_t)o->P.kem);
  if ((rc = up(de, enc, nenc * n, o->stream)) || (rc = up(dc, ct, (size_t)ct_stride * n, o->stream)) ||
      (rc = up(dl, ct_len, 4 * (size_t)n, o->stream)) ||
      (rc = up(di, report_ids, 16 * (size_t)n, o->stream)) ||
      (rc = up(dt, times, 8 * (size_t)n, o->stream)) ||
      (rc = up(dp, public_shares, (size_t)public_share_len * n, o->stream)))
    return rc;
  HCHK(hipMalloc(&ds.p, (size_t)helper_share_len * n + 1));
  HCHK(hipMalloc(&dst.p, n));
  rc = janus_hpke_open_input_shares_device(
      o, n, task_id, (const uint8_t*)de.p, (const uint8_t*)dc.p, (const uint32_t*)dl.p, ct_stride,
      (const uint8_t*)di.p, (const uint64_t*)dt.p, (const uint8_t*)dp.p, public_share_len,
      helper_share_len, require_taskprov, (uint8_t*)ds.p, (uint8_t*)dst.p, o->stream);
  if (rc) return rc;
  HCHK(hipMemcpyAsync(helper_shares, ds.p, (size_t)helper_share_len * n, hipMemcpyDeviceToHost,
                      o->stream));
  HCHK(hipMemcpyAsync(status, dst.p, n, hipMemcpyDeviceToHost, o->stream));
  HCHK(hipStreamSynchronize(o->stream));
  return JANUS_HPKE_SUCCESS;
}

int janus_hpke_executor_stats_get(const janus_hpke_opener* o, janus_hpke_executor_stats* out) {
  if (!o || !out) return JANUS_HPKE_EINVAL;
  ExecStats st;
  const int rc = exec_stats(EXEC_HPKE, o->device * EXEC_LANES, &st);
  if (rc) return rc;
  out->jobs = st.jobs;
  out->reports = st.reports;
  out->groups = st.groups;
  out->active_jobs = st.active_jobs;
  out->active_reports = st.active_reports;
  return JANUS_HPKE_SUCCESS;
}

int janus_hpke_executor_control(janus_hpke_opener* o, const char* key, int64_t value) {
  if (!o || !key) return JANUS_HPKE_EINVAL;
  if (!strcmp(key, "coalesce")) {
    o->coalesce = value != 0;
    return JANUS_HPKE_SUCCESS;
  }
  if (!strcmp(key, "pair_max")) {  // X25519 opens of at most this many reports on lane pairs
    if (value < 0) return JANUS_HPKE_EINVAL;
    std::lock_guard<std::mutex> lk(o->mu);
    o->pair_max = (int)std::min<int64_t>(value, INT32_MAX);
    return JANUS_HPKE_SUCCESS;
  }
  return exec_control(EXEC_HPKE, o->device * EXEC_LANES, key, value);
}

int janus_hpke_selftest_p256(int op, uint32_t n, const uint32_t* a, const uint32_t* b,
                             uint32_t* out) {
  if (op < 0 || op > 6) return JANUS_HPKE_EINVAL;
  if (n == 0) return JANUS_HPKE_OK;
  const size_t m = (size_t)n * 32;
  void *da = nullptr, *db = nullptr, *dout = nullptr;
  int rc = JANUS_HPKE_OK;
  if (hipMalloc(&da, m) != hipSuccess || hipMalloc(&db, m) != hipSuccess ||
      hipMalloc(&dout, m) != hipSuccess || hipMemcpy(da, a, m, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(db, b, m, hipMemcpyHostToDevice) != hipSuccess) {
    rc = JANUS_HPKE_EDEVICE;
  } else {
    k_selftest_p256<<<(n + 255) / 256, 256>>>(op, n, (const uint32_t*)da, (const uint32_t*)db,
                                              (uint32_t*)dout);
    if (hipGetLastError() != hipSuccess || hipMemcpy(out, dout, m, hipMemcpyDeviceToHost) != hipSuccess)
      rc = JANUS_HPKE_EDEVICE;
  }
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  return rc;
}

int janus_hpke_open(janus_hpke_opener* o, uint32_t n, const uint8_t* enc, const uint8_t* ct,
                    const uint32_t* ct_len, uint32_t ct_stride, const uint8_t* aad,
                    const uint32_t* aad_len, uint32_t aad_stride, uint8_t* pt, uint8_t* status) {
  if (!o) return JANUS_HPKE_EINVAL;
  if (n == 0) return JANUS_HPKE_SUCCESS;
  DeviceGuard dg_(o->device);
  HCHK(dg_.rc);
  DevBuf de, dc, dl, da, dal, dpt, dst;
  int rc;
  const size_t nenc = kem_nenc((uint16_t)o->P.kem);
  if ((rc = up(de, enc, nenc * n, o->stream)) || (rc = up(dc, ct, (size_t)ct_stride * n, o->stream)) ||
      (rc = up(dl, ct_len, 4 * (size_t)n, o->stream)) ||
      (rc = up(da, aad, (size_t)aad_stride * n, o->stream)) ||
      (rc = up(dal, aad_len, aad_stride ? 4 * (size_t)n : 0, o->stream)))
    return rc;
  HCHK(hipMalloc(&dpt.p, (size_t)ct_stride * n));
  HCHK(hipMalloc(&dst.p, n));
  rc = janus_hpke_open_device(o, n, (const uint8_t*)de.p, (const uint8_t*)dc.p,
                              (const uint32_t*)dl.p, ct_stride, (const uint8_t*)da.p,
                              (const uint32_t*)dal.p, aad_stride, (uint8_t*)dpt.p,
                              (uint8_t*)dst.p, o->stream);
  if (rc) return rc;
  HCHK(hipMemcpyAsync(pt, dpt.p, (size_t)ct_stride * n, hipMemcpyDeviceToHost, o->stream));
  HCHK(hipMemcpyAsync(status, dst.p, n, hipMemcpyDeviceToHost, o->stream));
  HCHK(hipStreamSynchronize(o->stream));
  return JANUS_HPKE_SUCCESS;
}

}  // extern "C"
