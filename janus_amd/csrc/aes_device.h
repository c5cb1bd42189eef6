// aes_device.h -- AES-128 / AES-256 encryption (FIPS 197) for one block per work-item,
// little-endian packed column words, T-tables in LDS (filled by the workgroup at kernel start).
// Used by the HPKE opener (AES-128-GCM and AES-256-GCM, hpke.hip) and by XofHmacSha256Aes128
// (AES-128-CTR seed streams, prio3_mp64.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

// -------------------------------------------------------------------------------------
// AES-128 (FIPS 197) with little-endian packed column words and LDS T-tables
// -------------------------------------------------------------------------------------
static __constant__ uint8_t c_sbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76,
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0,
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75,
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84,
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8,
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2,
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb,
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79,
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a,
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e,
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

struct AesT {
  uint32_t t[5][256];  // T0..T3 (MixColumns of the S-box output, row-rotated), T4 = S * 0x01010101
};

DEV void aes_tables_init(AesT& T) {
  for (uint32_t x = threadIdx.x; x < 256; x += blockDim.x) {
    const uint32_t s = c_sbox[x];
    const uint32_t s2 = ((s << 1) ^ ((s >> 7) * 0x1bu)) & 0xffu, s3 = s2 ^ s;
    const uint32_t t0 = s2 | (s << 8) | (s << 16) | (s3 << 24);
    T.t[0][x] = t0;
    T.t[1][x] = __builtin_amdgcn_alignbit(t0, t0, 24);  // rotl 8
    T.t[2][x] = __builtin_amdgcn_alignbit(t0, t0, 16);
    T.t[3][x] = __builtin_amdgcn_alignbit(t0, t0, 8);
    T.t[4][x] = s * 0x01010101u;
  }
}

// Byte offset 4 (byte K of w) into a 1 KiB table as a full-rate shift and one v_bitop3_b32 AND
// (LLVM otherwise forms v_bfe_u32 + v_lshl_add_u32, both half rate); an inlined table's LDS
// address folds into the ds_read offset field.
template <int K>
DEV uint32_t boff(uint32_t w) {
  const uint32_t sh = K == 0 ? w << 2 : w >> (8 * K - 2);
  return __builtin_amdgcn_bitop3_b32(sh, 0x3FCu, 0u, 0xC0);
}
template <int K>
DEV uint32_t tlook(const uint32_t* tab, uint32_t w) {
  return *(const uint32_t*)((const char*)tab + boff<K>(w));
}
DEV uint32_t b0(uint32_t x) { return x & 0xffu; }
DEV uint32_t b1(uint32_t x) { return (x >> 8) & 0xffu; }
DEV uint32_t b2(uint32_t x) { return (x >> 16) & 0xffu; }
DEV uint32_t b3(uint32_t x) { return x >> 24; }

DEV uint32_t sub_word(const AesT& T, uint32_t x) {
  return (T.t[4][b0(x)] & 0xffu) | (T.t[4][b1(x)] & 0xff00u) | (T.t[4][b2(x)] & 0xff0000u) |
         (T.t[4][b3(x)] & 0xff000000u);
}

DEV void aes128_expand(const AesT& T, const uint32_t key[4], uint32_t rk[44]) {
  constexpr uint8_t RC[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
#pragma unroll
  for (int i = 0; i < 4; i++) rk[i] = key[i];
#pragma unroll
  for (int i = 4; i < 44; i++) {
    uint32_t t = rk[i - 1];
    if ((i & 3) == 0) t = sub_word(T, __builtin_amdgcn_alignbit(t, t, 8)) ^ RC[i / 4 - 1];
    rk[i] = rk[i - 4] ^ t;
  }
}

// AES-256 key expansion (FIPS 197 5.2, Nk = 8): 60 round-key words
DEV void aes256_expand(const AesT& T, const uint32_t key[8], uint32_t rk[60]) {
  constexpr uint8_t RC[7] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40};
#pragma unroll
  for (int i = 0; i < 8; i++) rk[i] = key[i];
#pragma unroll
  for (int i = 8; i < 60; i++) {
    uint32_t t = rk[i - 1];
    if ((i & 7) == 0)
      t = sub_word(T, __builtin_amdgcn_alignbit(t, t, 8)) ^ RC[i / 8 - 1];
    else if ((i & 7) == 4)
      t = sub_word(T, t);
    rk[i] = rk[i - 8] ^ t;
  }
}

// NR rounds (10: AES-128, 14: AES-256) over the 4 (NR + 1) round-key words rk
template <int NR>
DEV void aes_encrypt(const AesT& T, const uint32_t* rk, const uint32_t in[4], uint32_t out[4]) {
  uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
  for (int r = 1; r < NR; r++) {
    // five-way XORs as two v_bitop3_b32 (LLVM emits four v_xor)
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
      return __builtin_amdgcn_bitop3_b32(
          __builtin_amdgcn_bitop3_b32(tlook<0>(T.t[0], a), tlook<1>(T.t[1], b),
                                      tlook<2>(T.t[2], c), 0x96),
          tlook<3>(T.t[3], d), k, 0x96);
    };
    const uint32_t t0 = col(s0, s1, s2, s3, rk[4 * r]);
    const uint32_t t1 = col(s1, s2, s3, s0, rk[4 * r + 1]);
    const uint32_t t2 = col(s2, s3, s0, s1, rk[4 * r + 2]);
    const uint32_t t3 = col(s3, s0, s1, s2, rk[4 * r + 3]);
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  out[0] = ((T.t[4][b0(s0)] & 0xffu) | (T.t[4][b1(s1)] & 0xff00u) | (T.t[4][b2(s2)] & 0xff0000u) |
            (T.t[4][b3(s3)] & 0xff000000u)) ^ rk[4 * NR];
  out[1] = ((T.t[4][b0(s1)] & 0xffu) | (T.t[4][b1(s2)] & 0xff00u) | (T.t[4][b2(s3)] & 0xff0000u) |
            (T.t[4][b3(s0)] & 0xff000000u)) ^ rk[4 * NR + 1];
  out[2] = ((T.t[4][b0(s2)] & 0xffu) | (T.t[4][b1(s3)] & 0xff00u) | (T.t[4][b2(s0)] & 0xff0000u) |
            (T.t[4][b3(s1)] & 0xff000000u)) ^ rk[4 * NR + 2];
  out[3] = ((T.t[4][b0(s3)] & 0xffu) | (T.t[4][b1(s0)] & 0xff00u) | (T.t[4][b2(s1)] & 0xff0000u) |
            (T.t[4][b3(s2)] & 0xff000000u)) ^ rk[4 * NR + 3];
}

DEV void aes128_encrypt(const AesT& T, const uint32_t rk[44], const uint32_t in[4],
                        uint32_t out[4]) {
  aes_encrypt<10>(T, rk, in, out);
}

// -------------------------------------------------------------------------------------
// The same cipher on a bank-replicated T0 (32 KiB of LDS): entry x of copy c at word 32x + c,
// and lane l reads copy l mod 32, so each 32-lane group of a ds_read_b32 touches 32 distinct
// banks whatever the indices (with 4 KiB tables the 32 random indices of a group collide on a
// bank 3-4 deep).  T1..T3 are T0 rotated (v_alignbit); the S-box is byte 1 of T0.
// -------------------------------------------------------------------------------------
struct AesR {
  uint32_t t[256 * 32];
};

DEV void aesr_init(AesR& T) {
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) {
    const uint32_t s = c_sbox[i >> 5];
    const uint32_t s2 = ((s << 1) ^ ((s >> 7) * 0x1bu)) & 0xffu, s3 = s2 ^ s;
    T.t[i] = s2 | (s << 8) | (s << 16) | (s3 << 24);
  }
}

// Entry x of this lane's copy is at byte offset 128 x + 4 (lane mod 32) from T.t.  The round
// forms that offset for byte k of a state word as one shift and one v_bitop3_b32
// ((w >> (8k - 7)) & 0x7F80 | 4 (lane mod 32), both full rate); the table's own LDS address is
// a constant the compiler folds into the ds_read offset field.
struct AesRLane {
  const char* base;  // (const char*)T.t
  uint32_t lane4;    // 4 (lane mod 32)
  DEV uint32_t t0(uint32_t x) const { return *(const uint32_t*)(base + (x << 7) + lane4); }
  DEV uint32_t at(uint32_t off) const { return *(const uint32_t*)(base + off); }
  template <int K>
  DEV uint32_t off(uint32_t w) const {
    const uint32_t sh = K == 0 ? w << 7 : w >> (8 * K - 7);
    return __builtin_amdgcn_bitop3_b32(sh, 0x7F80u, lane4, 0xEA);  // (a & b) | c
  }
};

DEV AesRLane aesr_lane(const AesR& T) {
  return AesRLane{(const char*)T.t, (threadIdx.x & 31u) << 2};
}
DEV uint32_t aes_x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

DEV uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
DEV uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
DEV uint32_t rotl24(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 8); }

// S-box bytes of x's four bytes, in place
DEV uint32_t aesr_sub_word(const AesRLane& L, uint32_t x) {
  return ((L.t0(b0(x)) >> 8) & 0xffu) | (L.t0(b1(x)) & 0xff00u) | (L.t0(b2(x)) & 0xff0000u) |
         ((L.t0(b3(x)) << 8) & 0xff000000u);
}

DEV void aesr128_expand(const AesRLane& L, const uint32_t key[4], uint32_t rk[44]) {
  constexpr uint8_t RC[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
#pragma unroll
  for (int i = 0; i < 4; i++) rk[i] = key[i];
#pragma unroll
  for (int i = 4; i < 44; i++) {
    uint32_t t = rk[i - 1];
    if ((i & 3) == 0) t = aesr_sub_word(L, __builtin_amdgcn_alignbit(t, t, 8)) ^ RC[i / 4 - 1];
    rk[i] = rk[i - 4] ^ t;
  }
}

DEV void aesr128_encrypt(const AesRLane& L, const uint32_t rk[44], const uint32_t in[4],
                         uint32_t out[4]) {
  uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
  for (int r = 1; r < 10; r++) {
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
      return aes_x3(aes_x3(L.at(L.off<0>(a)), rotl8(L.at(L.off<1>(b))), rotl16(L.at(L.off<2>(c)))),
                    rotl24(L.at(L.off<3>(d))), k);
    };
    const uint32_t t0 = col(s0, s1, s2, s3, rk[4 * r]);
    const uint32_t t1 = col(s1, s2, s3, s0, rk[4 * r + 1]);
    const uint32_t t2 = col(s2, s3, s0, s1, rk[4 * r + 2]);
    const uint32_t t3 = col(s3, s0, s1, s2, rk[4 * r + 3]);
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  const uint32_t x[4] = {s0, s1, s2, s3};
#pragma unroll
  for (int c = 0; c < 4; c++)
    out[c] = (((L.t0(b0(x[c])) >> 8) & 0xffu) | (L.t0(b1(x[(c + 1) & 3])) & 0xff00u) |
              (L.t0(b2(x[(c + 2) & 3])) & 0xff0000u) |
              ((L.t0(b3(x[(c + 3) & 3])) << 8) & 0xff000000u)) ^ rk[40 + c];
}

