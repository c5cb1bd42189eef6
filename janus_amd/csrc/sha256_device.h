// sha256_device.h -- SHA-256 compression (FIPS 180-4) for one message block per work-item.
// Used for ReportIdChecksum (prio3_engine.hip, k_meta) and for HMAC/HKDF-SHA256 of the HPKE
// key schedule (hpke.hip).  Fully unrolled: the round constants become instruction literals.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace sha256d {

DEV uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
// Three-input logic as one full-rate v_bitop3_b32 (truth table over src0 = 0xF0, src1 = 0xCC,
// src2 = 0xAA): LLVM emits two v_xor for a ^ b ^ c and v_xor + v_and + v_bitop3 for Maj.
DEV uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
DEV uint32_t maj(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8); }
DEV uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA); }

constexpr uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                            0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

// st <- compress(st, w): w[16] are the block's big-endian words (consumed as schedule space).
DEV void compress(uint32_t st[8], uint32_t w[16]) {
  constexpr uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
      0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
      0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
      0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
      0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
      0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
      0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
      0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
      0xc67178f2u};
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
#pragma unroll
  for (int t = 0; t < 64; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {  // rolling 16-word schedule
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = x3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = x3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      wt = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
    }
    const uint32_t S1 = x3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t t1 = h + S1 + ch(e, f, g) + K[t] + wt;
    const uint32_t S0 = x3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t mj = maj(a, b, c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

}  // namespace sha256d

// -------------------------------------------------------------------------------------
// SHA-256 message buffers (big-endian words) and HMAC
// -------------------------------------------------------------------------------------
template <int NW>
struct Msg32 {
  uint32_t w[NW];
};
template <int NW>
DEV void mz(Msg32<NW>& m) {
#pragma unroll
  for (int i = 0; i < NW; i++) m.w[i] = 0;
}
template <int NW>
DEV void mbyte(Msg32<NW>& m, int pos, uint32_t b) {
  m.w[pos >> 2] |= (b & 0xffu) << (24 - 8 * (pos & 3));
}
template <int NW, int N>
DEV void mstr(Msg32<NW>& m, int pos, const char (&s)[N]) {  // N - 1 bytes (no terminator)
#pragma unroll
  for (int i = 0; i < N - 1; i++) mbyte(m, pos + i, (uint8_t)s[i]);
}
// nbytes (multiple of 4) of big-endian words d at byte position pos
template <int NW>
DEV void mwords_be(Msg32<NW>& m, int pos, const uint32_t* d, int nwords) {
  const int q = pos >> 2, o = pos & 3;
  if (o == 0) {
#pragma unroll
    for (int i = 0; i < nwords; i++) m.w[q + i] |= d[i];
  } else {
#pragma unroll
    for (int i = 0; i < nwords; i++) {
      m.w[q + i] |= d[i] >> (8 * o);
      m.w[q + i + 1] |= d[i] << (32 - 8 * o);
    }
  }
}
// little-endian packed bytes (as loaded from memory) at byte position pos
template <int NW>
DEV void mwords_le(Msg32<NW>& m, int pos, const uint32_t* d, int nwords) {
  uint32_t be[16];
#pragma unroll
  for (int i = 0; i < nwords; i++) be[i] = __builtin_bswap32(d[i]);
  mwords_be(m, pos, be, nwords);
}
// SHA-256 over the len message bytes of m after `prefix` bytes already compressed into st
template <int NW>
DEV void sha_final(uint32_t st[8], Msg32<NW>& m, int len, int prefix) {
  mbyte(m, len, 0x80);
  const int nblk = (len + 9 + 63) / 64;
  m.w[nblk * 16 - 1] = (uint32_t)((prefix + len) * 8);
#pragma unroll
  for (int b = 0; b < nblk; b++) {
    uint32_t blk[16];
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = m.w[16 * b + i];
    sha256d::compress(st, blk);
  }
}

struct HmacKey {
  uint32_t ist[8], ost[8];
};
// HMAC key of 4 NW bytes (NW <= 16 big-endian words): the ipad / opad midstates
template <int NW>
DEV void hmac_keyw(HmacKey& k, const uint32_t* key) {
  static_assert(NW <= 16, "HMAC-SHA256 keys up to the 64-byte block");
  uint32_t bi[16], bo[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t x = i < NW ? key[i] : 0u;
    bi[i] = x ^ 0x36363636u;
    bo[i] = x ^ 0x5c5c5c5cu;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) k.ist[i] = k.ost[i] = sha256d::IV[i];
  sha256d::compress(k.ist, bi);
  sha256d::compress(k.ost, bo);
}
DEV void hmac_key32(HmacKey& k, const uint32_t key[8]) { hmac_keyw<8>(k, key); }
template <int NW>
DEV void hmac(const HmacKey& k, Msg32<NW>& m, int len, uint32_t out[8]) {
  uint32_t st[8];
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = k.ist[i];
  sha_final(st, m, len, 64);
  Msg32<16> o;
  mz(o);
#pragma unroll
  for (int i = 0; i < 8; i++) o.w[i] = st[i];
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = k.ost[i];
  sha_final(out, o, 32, 64);
}
