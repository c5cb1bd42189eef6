// sha512_device.h -- SHA-512 / SHA-384 compression (FIPS 180-4 6.4, 6.5), HMAC and the byte
// message builder, for the HKDF-SHA512 / HKDF-SHA384 of the HPKE opener (hpke.hip): the KEM
// KDF of DHKEM(X448, HKDF-SHA512) and DHKEM(P-521, HKDF-SHA512), and the key-schedule KDFs 0x0002
// / 0x0003 of RFC 9180 7.2 (messages/src/lib.rs:809-815, HpkeKdfId).
// The same code runs on the host (opener creation: key_schedule_context, empty-key midstates).
// 64-bit words are pairs of 32-bit VGPRs on gfx950; rotations are two v_alignbit each.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef HD
#define HD __host__ __device__ __forceinline__
#endif

namespace sha512d {

// Rotations and shifts on the device as v_alignbit_b32 on the 32-bit halves (LLVM otherwise
// builds them from 64-bit shifts and ORs)
HD uint64_t rotr(uint64_t x, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n < 32)
    return (uint64_t)__builtin_amdgcn_alignbit(lo, hi, n) << 32 | __builtin_amdgcn_alignbit(hi, lo, n);
  return (uint64_t)__builtin_amdgcn_alignbit(hi, lo, n - 32) << 32 |
         __builtin_amdgcn_alignbit(lo, hi, n - 32);
#else
  return (x >> n) | (x << (64 - n));
#endif
}
HD uint64_t shr(uint64_t x, uint32_t n) {  // n < 32
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return (uint64_t)(hi >> n) << 32 | __builtin_amdgcn_alignbit(hi, lo, n);
#else
  return x >> n;
#endif
}
// Three-input logic on both 32-bit halves as v_bitop3_b32 (full rate) on the device; LLVM emits
// two v_xor per half for a ^ b ^ c and v_xor + v_and + v_bitop3 for Maj.
template <uint32_t TT>
HD uint64_t bop3(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, TT);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32),
                                                  (uint32_t)(c >> 32), TT);
  return (uint64_t)hi << 32 | lo;
#else
  uint64_t r = 0;  // the truth table bit by bit (src0 = 0xF0, src1 = 0xCC, src2 = 0xAA)
  for (int i = 0; i < 8; i++)
    if ((TT >> i) & 1) {
      r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    }
  return r;
#endif
}

// IVs: SHA-512 (FIPS 180-4 5.3.5) and SHA-384 (5.3.4)
constexpr uint64_t IV512[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                               0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                               0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
constexpr uint64_t IV384[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull,
                               0x152fecd8f70e5939ull, 0x67332667ffc00b31ull, 0x8eb44a8768581511ull,
                               0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};

// st <- compress(st, w): w[16] the block's big-endian 64-bit words (consumed as schedule space).
// Out of line on the device: one copy per kernel (a compression is ~3.5 k instructions and the
// key schedules call it a dozen times; inlined, hpke.hip took minutes to compile).
__host__ __device__ __noinline__ void compress(uint64_t st[8], uint64_t w[16]) {
  constexpr uint64_t K[80] = {
      0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
      0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
      0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
      0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
      0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
      0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
      0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
      0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
      0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
      0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
      0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
      0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
      0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
      0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
      0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
      0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
      0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
      0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
      0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
      0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
#pragma unroll
  for (int t = 0; t < 80; t++) {
    uint64_t wt;
    if (t < 16) {
      wt = w[t];
    } else {  // rolling 16-word schedule
      const uint64_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint64_t s0 = bop3<0x96>(rotr(w15, 1), rotr(w15, 8), shr(w15, 7));
      const uint64_t s1 = bop3<0x96>(rotr(w2, 19), rotr(w2, 61), shr(w2, 6));
      wt = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
    }
    const uint64_t S1 = bop3<0x96>(rotr(e, 14), rotr(e, 18), rotr(e, 41));
    const uint64_t ch = bop3<0xCA>(e, f, g);
    const uint64_t t1 = h + S1 + ch + K[t] + wt;
    const uint64_t S0 = bop3<0x96>(rotr(a, 28), rotr(a, 34), rotr(a, 39));
    const uint64_t mj = bop3<0xE8>(a, b, c);
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

}  // namespace sha512d

// -------------------------------------------------------------------------------------
// Byte messages as big-endian 64-bit words (positions known at compile time: registers)
// -------------------------------------------------------------------------------------
template <int NW>
struct Msg64 {
  uint64_t w[NW];
};
template <int NW>
HD void mz(Msg64<NW>& m) {
#pragma unroll
  for (int i = 0; i < NW; i++) m.w[i] = 0;
}
template <int NW>
HD void mbyte(Msg64<NW>& m, int pos, uint32_t b) {
  m.w[pos >> 3] |= (uint64_t)(b & 0xffu) << (56 - 8 * (pos & 7));
}
template <int NW, int N>
HD void mstr(Msg64<NW>& m, int pos, const char (&s)[N]) {  // N - 1 bytes (no terminator)
#pragma unroll
  for (int i = 0; i < N - 1; i++) mbyte(m, pos + i, (uint8_t)s[i]);
}
// nbytes bytes of b at byte position pos
template <int NW>
HD void mbytes(Msg64<NW>& m, int pos, const uint8_t* b, int nbytes) {
#pragma unroll
  for (int i = 0; i < nbytes; i++) mbyte(m, pos + i, b[i]);
}
// nw big-endian 64-bit words at byte position pos
template <int NW>
HD void mwords64(Msg64<NW>& m, int pos, const uint64_t* d, int nw) {
  const int q = pos >> 3, o = pos & 7;
  if (o == 0) {
#pragma unroll
    for (int i = 0; i < nw; i++) m.w[q + i] |= d[i];
  } else {
#pragma unroll
    for (int i = 0; i < nw; i++) {
      m.w[q + i] |= d[i] >> (8 * o);
      m.w[q + i + 1] |= d[i] << (64 - 8 * o);
    }
  }
}
// SHA-512 over the len message bytes of m after `prefix` bytes already compressed into st
template <int NW>
HD void sha512_final(uint64_t st[8], Msg64<NW>& m, int len, int prefix) {
  mbyte(m, len, 0x80);
  const int nblk = (len + 17 + 127) / 128;
  m.w[nblk * 16 - 1] = (uint64_t)(prefix + len) * 8;
#pragma unroll
  for (int b = 0; b < nblk; b++) {
    uint64_t blk[16];
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = m.w[16 * b + i];
    sha512d::compress(st, blk);
  }
}

// HMAC-SHA512 / HMAC-SHA384 (RFC 2104, block 128 bytes): the ipad / opad midstates of the key
struct HmacKey64 {
  uint64_t ist[8], ost[8];
  int out_words;  // 8 (SHA-512) or 6 (SHA-384)
};
// key of kw big-endian 64-bit words (kw <= 16); sha384 selects the IV and the 48-byte output
HD void hmac64_key(HmacKey64& k, const uint64_t* key, int kw, bool sha384) {
  uint64_t bi[16], bo[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint64_t x = i < kw ? key[i] : 0ull;
    bi[i] = x ^ 0x3636363636363636ull;
    bo[i] = x ^ 0x5c5c5c5c5c5c5c5cull;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) k.ist[i] = k.ost[i] = sha384 ? sha512d::IV384[i] : sha512d::IV512[i];
  sha512d::compress(k.ist, bi);
  sha512d::compress(k.ost, bo);
  k.out_words = sha384 ? 6 : 8;
}
// out[0 .. out_words) = HMAC(k, m[0 .. len))
template <int NW>
HD void hmac64(const HmacKey64& k, Msg64<NW>& m, int len, uint64_t out[8]) {
  uint64_t st[8];
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = k.ist[i];
  sha512_final(st, m, len, 128);
  Msg64<16> o;
  mz(o);
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (i < k.out_words) o.w[i] = st[i];
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = k.ost[i];
  sha512_final(out, o, 8 * k.out_words, 128);
  if (k.out_words == 6) out[6] = out[7] = 0;
}
