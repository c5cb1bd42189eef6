// prio3_mp64_xof.h -- XofHmacSha256Aes128 building blocks on the device (prio 0.16
// vdaf/xof.rs, restated; parity with prio UNPINNED): HMAC-SHA256 keyed by a
// 32-byte seed over len(dst) || dst || binder; the 32-byte tag is the AES-128 key and IV of a CTR
// keystream with a 64-bit big-endian counter in the IV's low half (Ctr64BE<Aes128>); Field64
// elements are 8-byte LE chunks, rejected if >= p.  Shared by the multiproof VDAF's prepare
// (prio3_mp64.hip) and its device client (prio3_client.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/janus_prio3.h"
#include "prio3_device.h"
#include "prio3_common.h"
#include "sha256_device.h"
#include "aes_device.h"

namespace {

// The SHA-256 / AES / HMAC building blocks of the short XOF instances are out-of-line calls
// (inlined ~40 times they would not fit the register file; their arrays pass through the scratch
// stack).  The two long ones -- the share expansions and the joint-rand part's hash over the
// measurement share, ~95 % of the blocks -- are inlined once each (expand_soa_inl, jr_inner_inl).
#define NI __device__ __attribute__((noinline))

NI void compress_ni(uint32_t st[8], uint32_t w[16]) { sha256d::compress(st, w); }
NI void aes_enc_ni(const AesT& A, const uint32_t rk[44], const uint32_t in[4], uint32_t out[4]) {
  aes128_encrypt(A, rk, in, out);
}
NI void aes_expand_ni(const AesT& A, const uint32_t key[4], uint32_t rk[44]) {
  aes128_expand(A, key, rk);
}
// HMAC-SHA256 with given ipad / opad midstates over the len bytes of m (len <= 119)
NI void hmac_ni(const uint32_t ist[8], const uint32_t ost[8], const uint32_t* mw, int len,
                uint32_t tag[8]) {
  uint32_t st[8], w[16];
  for (int i = 0; i < 8; i++) st[i] = ist[i];
  const int nblk = (len + 9 + 63) / 64;
  for (int b = 0; b < nblk; b++) {
    for (int i = 0; i < 16; i++) {
      const int t = 16 * b + i;
      uint32_t x = t < (len + 3) / 4 ? mw[t] : 0u;
      if (t == len / 4) {  // the 0x80 padding byte (message bytes past len are zero)
        x |= 0x80u << (24 - 8 * (len & 3));
      }
      if (b == nblk - 1 && i == 15) x = (uint32_t)((64 + len) * 8);
      w[i] = x;
    }
    compress_ni(st, w);
  }
  uint32_t o[16] = {st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], 0x80000000u,
                    0, 0, 0, 0, 0, 0, (64 + 32) * 8};
  for (int i = 0; i < 8; i++) tag[i] = ost[i];
  compress_ni(tag, o);
}
// HMAC midstates of a 32-byte key (LE words as loaded)
NI void hmac_key_ni(const uint32_t key_le[8], uint32_t ist[8], uint32_t ost[8]) {
  uint32_t bi[16], bo[16];
  for (int i = 0; i < 16; i++) {
    const uint32_t x = i < 8 ? __builtin_bswap32(key_le[i]) : 0u;
    bi[i] = x ^ 0x36363636u;
    bo[i] = x ^ 0x5c5c5c5cu;
  }
  for (int i = 0; i < 8; i++) ist[i] = ost[i] = sha256d::IV[i];
  compress_ni(ist, bi);
  compress_ni(ost, bo);
}

// ---- XofHmacSha256Aes128 seed stream ---------------------------------------------------
struct Stream {
  uint32_t rk[44];
  uint32_t iv0, iv1;  // AES input columns 0, 1 (IV bytes 0..7)
  uint64_t ctr;       // IV bytes 8..15 as a big-endian integer, + blocks consumed
};

// tag (big-endian words of the HMAC output) -> AES key / IV
DEV void stream_init(const AesT& A, Stream& s, const uint32_t tag[8]) {
  uint32_t key[4];
#pragma unroll
  for (int i = 0; i < 4; i++) key[i] = __builtin_bswap32(tag[i]);
  aes_expand_ni(A, key, s.rk);
  s.iv0 = __builtin_bswap32(tag[4]);
  s.iv1 = __builtin_bswap32(tag[5]);
  s.ctr = ((uint64_t)tag[6] << 32) | tag[7];
}
// next 16 keystream bytes as 4 little-endian words
DEV void stream_block(const AesT& A, Stream& s, uint32_t out[4]) {
  const uint32_t in[4] = {s.iv0, s.iv1, __builtin_bswap32((uint32_t)(s.ctr >> 32)),
                          __builtin_bswap32((uint32_t)s.ctr)};
  aes_enc_ni(A, s.rk, in, out);
  s.ctr++;
}

// HMAC-SHA256 tag of `seed` (LE words of its 32 bytes) over [len(dst)] || dst || binder,
// binder given as m (bytes from position 9), total message length len
template <int NW>
DEV void xof_tag(const uint32_t seed_le[8], Msg32<NW>& m, int len, uint32_t tag[8]) {
  uint32_t ist[8], ost[8];
  hmac_key_ni(seed_le, ist, ost);
  hmac_ni(ist, ost, m.w, len, tag);
}

template <int NW>
DEV void msg_dst(Msg32<NW>& m, const Mp64Params& P, int usage) {
  mbyte(m, 0, 8);
  uint32_t d[2] = {__builtin_bswap32(P.dst[usage][0]), __builtin_bswap32(P.dst[usage][1])};
  mwords_be(m, 1, d, 2);
}

// n Field64 elements from the stream into SoA scratch base[e * ld + r] (rejection sampling)
DEV uint32_t expand_soa(const AesT& A, Stream& s, uint64_t* base, size_t ld, uint32_t r,
                        uint32_t n) {
  uint32_t k = 0, rej = 0;
  while (k < n) {
    uint32_t w[4];
    stream_block(A, s, w);
    const uint64_t c0 = ((uint64_t)w[1] << 32) | w[0], c1 = ((uint64_t)w[3] << 32) | w[2];
    if (c0 < P64) {
      base[(size_t)k * ld + r] = c0;
      k++;
    } else {
      rej++;
    }
    if (k < n) {
      if (c1 < P64) {
        base[(size_t)k * ld + r] = c1;
        k++;
      } else {
        rej++;
      }
    }
  }
  return rej;
}

// expand_soa at one inlined call site of the prepare kernel: the key schedule and the
// encryptions unrolled, so the 44 round-key words stay in registers (the out-of-line
// aes_enc_ni takes them from the scratch stack, 176 B per block).  Same stream, same rejection.
DEV void aes_expand_any(const AesT& A, const uint32_t key[4], uint32_t rk[44]) {
  aes128_expand(A, key, rk);
}
DEV void aes_expand_any(const AesRLane& A, const uint32_t key[4], uint32_t rk[44]) {
  aesr128_expand(A, key, rk);
}
DEV void aes_encrypt_any(const AesT& A, const uint32_t rk[44], const uint32_t in[4],
                         uint32_t out[4]) {
  aes128_encrypt(A, rk, in, out);
}
DEV void aes_encrypt_any(const AesRLane& A, const uint32_t rk[44], const uint32_t in[4],
                         uint32_t out[4]) {
  aesr128_encrypt(A, rk, in, out);
}

template <class TB>
DEV uint32_t expand_soa_inl(const TB& A, const uint32_t tag[8], uint64_t* base, size_t ld,
                            uint32_t r, uint32_t n) {
  uint32_t key[4], rk[44];
#pragma unroll
  for (int i = 0; i < 4; i++) key[i] = __builtin_bswap32(tag[i]);
  aes_expand_any(A, key, rk);
  const uint32_t iv0 = __builtin_bswap32(tag[4]), iv1 = __builtin_bswap32(tag[5]);
  uint64_t ctr = ((uint64_t)tag[6] << 32) | tag[7];
  uint32_t k = 0, rej = 0;
  while (k < n) {
    const uint32_t in[4] = {iv0, iv1, __builtin_bswap32((uint32_t)(ctr >> 32)),
                            __builtin_bswap32((uint32_t)ctr)};
    uint32_t w[4];
    aes_encrypt_any(A, rk, in, w);
    ctr++;
    const uint64_t c0 = ((uint64_t)w[1] << 32) | w[0], c1 = ((uint64_t)w[3] << 32) | w[2];
    if (c0 < P64) {
      base[(size_t)k * ld + r] = c0;
      k++;
    } else {
      rej++;
    }
    if (k < n) {
      if (c1 < P64) {
        base[(size_t)k * ld + r] = c1;
        k++;
      } else {
        rej++;
      }
    }
  }
  return rej;
}

// first 32 bytes of the stream (derive_seed) as LE words
DEV void derive32(const AesT& A, Stream& s, uint32_t out[8]) {
  stream_block(A, s, out);
  stream_block(A, s, out + 4);
}

// n field elements from the stream into registers (n small: jr / qr)
template <int N>
DEV void expand_regs(const AesT& A, Stream& s, uint64_t* out, uint32_t n) {
  uint32_t k = 0;
  while (k < n) {
    uint32_t w[4];
    stream_block(A, s, w);
    const uint64_t c[2] = {((uint64_t)w[1] << 32) | w[0], ((uint64_t)w[3] << 32) | w[2]};
#pragma unroll
    for (int h = 0; h < 2; h++)
      if (k < n && c[h] < P64) {
#pragma unroll
        for (int q = 0; q < N; q++)
          if ((uint32_t)q == k) out[q] = c[h];
        k++;
      }
  }
}

DEV uint64_t ld64(const uint64_t* base, size_t ld, uint32_t e, uint32_t r) {
  return base[(size_t)e * ld + r];
}

// the joint-rand part message after the key: [8] || dst(7) || [1] || nonce || enc(meas), as
// big-endian word t (bytes 4t..4t+3), with SHA-256 padding for total message length L
// (L = 26 + 8M, L mod 4 = 2) and the HMAC prefix of 64 bytes in the length field
NI uint32_t jr_word(uint32_t t, const uint32_t pre[7], const uint64_t* meas, size_t ld,
                     uint32_t r, uint32_t M, uint32_t L, uint32_t nblk_words) {
  const uint32_t lw = L >> 2;  // the word holding the last 2 data bytes and 0x80
  if (t + 1 == nblk_words) return (uint32_t)((64ull + L) * 8);  // length (low word)
  if (t + 2 == nblk_words) return (uint32_t)(((64ull + L) * 8) >> 32);
  if (t > lw) return 0;
  auto elem = [&](uint32_t e) -> uint64_t { return e < M ? ld64(meas, ld, e, r) : 0ull; };
  uint32_t le;
  if (t < 6) return pre[t];
  if (t == 6) {  // prefix bytes 24, 25 + element 0 bytes 0, 1
    const uint64_t v = elem(0);
    le = (pre[6] & 0xffff0000u) | (__builtin_bswap32((uint32_t)v) >> 16);
    if (t == lw) le = (le & 0xffff0000u) | 0x8000u;
    return le;
  }
  const uint32_t d = 4 * t - 26;  // data byte index, = 2 or 6 (mod 8)
  const uint32_t e = d >> 3;
  const uint64_t v = elem(e);
  uint32_t w;
  if ((d & 7) == 2) {
    w = __builtin_amdgcn_alignbit((uint32_t)(v >> 32), (uint32_t)v, 16);  // bytes 2..5
  } else {
    const uint64_t v2 = elem(e + 1);
    w = __builtin_amdgcn_alignbit((uint32_t)v2, (uint32_t)(v >> 32), 16);  // 6, 7, 0', 1'
  }
  uint32_t be = __builtin_bswap32(w);
  if (t == lw) be = (be & 0xffff0000u) | 0x8000u;  // 2 data bytes, then 0x80
  return be;
}

// The joint-rand part's HMAC inner hash (st = the key's ipad midstate on entry) over the
// message jr_word describes, with the compression inlined at this one site.  Block b's data
// bytes 64b - 26 .. 64b + 37 lie in elements 8b - 4 .. 8b + 4: the nine are loaded once, and
// word i of the block is a 16-bit funnel shift of element 8b - 4 + (floor((4i - 26) / 8) + 4)
// (odd i: its bytes 2..5) or of it and the next (even i: bytes 6, 7, 0', 1').  The first block
// (the prefix) and the tail blocks (0x80, zero fill, length) take jr_word's cases.
DEV void jr_inner_inl(uint32_t st[8], const uint32_t pre[7], const uint64_t* meas, size_t ld,
                      uint32_t r, uint32_t M, uint32_t L, uint32_t nblk) {
  const uint32_t lw = L >> 2, nw = 16 * nblk;
#pragma nounroll
  for (uint32_t b = 0; b < nblk; b++) {
    uint64_t v[9];
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const int e = (int)(8 * b) - 4 + j;
      v[j] = (e >= 0 && (uint32_t)e < M) ? ld64(meas, ld, (uint32_t)e, r) : 0ull;
    }
    const bool interior = b > 0 && 16 * b + 15 < lw;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int rel = ((4 * i - 26) >> 3) + 4;  // arithmetic shift: floor
      const uint64_t x = v[rel];
      uint32_t dw;
      if (i & 1) {
        dw = __builtin_amdgcn_alignbit((uint32_t)(x >> 32), (uint32_t)x, 16);
      } else {
        dw = __builtin_amdgcn_alignbit((uint32_t)v[rel + 1], (uint32_t)(x >> 32), 16);
      }
      uint32_t be = __builtin_bswap32(dw);
      if (!interior) {
        const uint32_t t = 16 * b + i;
        if (t + 1 == nw) {
          be = (uint32_t)((64ull + L) * 8);
        } else if (t + 2 == nw) {
          be = (uint32_t)(((64ull + L) * 8) >> 32);
        } else if (t > lw) {
          be = 0;
        } else if (t < 6) {
          be = pre[t];
        } else if (t == 6) {
          be = (pre[6] & 0xffff0000u) | (be & 0xffffu);
        } else if (t == lw) {
          be = (be & 0xffff0000u) | 0x8000u;
        }
      }
      w[i] = be;
    }
    sha256d::compress(st, w);
  }
}

}  // namespace
