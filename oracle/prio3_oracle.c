/*
 * prio3_oracle.c -- CPU restatement of prio 0.16.2 Prio3 (VDAF draft-08) for the
 * Janus helper preparation path.  TEST INFRASTRUCTURE ONLY: used by tests/, by
 * __graft_entry__.smoke() as the checker and by bench.py's cpu_baseline leg.
 * Parity with prio bytes is UNPINNED (see prio3_oracle.h); pinned sub-results are
 * listed there and in DESIGN.md.
 *
 * Section references "[VDAF-08 §x]" are to draft-irtf-cfrg-vdaf-08; "[prio]" marks
 * an implementation detail of prio 0.16.2 that is mirrored for cost fidelity
 * (e.g. DFT-based wire interpolation in FlpGeneric::query, the measurement-share
 * re-expansion in Prio3::prepare_next).
 */
#include "prio3_oracle.h"

#include <openssl/evp.h>
#include <malloc.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------------------ */
/* Keccak-p[1600, n_r] and TurboSHAKE128 (RFC 9861)                                     */
/* ------------------------------------------------------------------------------------ */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL,
    0x8000000080008000ULL, 0x000000000000808BULL, 0x0000000080000001ULL,
    0x8000000080008081ULL, 0x8000000000008009ULL, 0x000000000000008AULL,
    0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL,
    0x8000000000008003ULL, 0x8000000000008002ULL, 0x8000000000000080ULL,
    0x000000000000800AULL, 0x800000008000000AULL, 0x8000000080008081ULL,
    0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

static inline uint64_t rol64(uint64_t x, int n) {
  return (x << (n & 63)) | (x >> ((64 - n) & 63));
}

/* Lane-complementing-free reference-style loop, fully unrolled by the compiler
 * (pi lane walk + rho offsets from the Keccak reference). */
static const int PI_LANE[24] = {10, 7,  11, 17, 18, 3, 5,  16, 8,  21, 24, 4,
                                15, 23, 19, 13, 12, 2, 20, 14, 22, 9,  6,  1};
static const int RHO_OFF[24] = {1,  3,  6,  10, 15, 21, 28, 36, 45, 55, 2,  14,
                                27, 41, 56, 8,  25, 43, 62, 18, 39, 61, 20, 44};

void orc_keccak_p1600(uint64_t st[25], int rounds) {
  uint64_t bc[5], t;
  for (int ir = 24 - rounds; ir < 24; ir++) {
#pragma GCC unroll 5
    for (int i = 0; i < 5; i++) bc[i] = st[i] ^ st[i + 5] ^ st[i + 10] ^ st[i + 15] ^ st[i + 20];
#pragma GCC unroll 5
    for (int i = 0; i < 5; i++) {
      t = bc[(i + 4) % 5] ^ rol64(bc[(i + 1) % 5], 1);
#pragma GCC unroll 5
      for (int j = 0; j < 25; j += 5) st[j + i] ^= t;
    }
    t = st[1];
#pragma GCC unroll 24
    for (int i = 0; i < 24; i++) {
      int j = PI_LANE[i];
      bc[0] = st[j];
      st[j] = rol64(t, RHO_OFF[i]);
      t = bc[0];
    }
#pragma GCC unroll 5
    for (int j = 0; j < 25; j += 5) {
#pragma GCC unroll 5
      for (int i = 0; i < 5; i++) bc[i] = st[j + i];
#pragma GCC unroll 5
      for (int i = 0; i < 5; i++) st[j + i] ^= (~bc[(i + 1) % 5]) & bc[(i + 2) % 5];
    }
    st[0] ^= KRC[ir];
  }
}

#define TS_RATE 168
typedef struct {
  uint64_t s[25];
  uint32_t pos;
  int rounds;
} sponge;

static void sp_init(sponge* t, int rounds) {
  memset(t->s, 0, sizeof t->s);
  t->pos = 0;
  t->rounds = rounds;
}
static inline uint8_t* sp_bytes(sponge* t) { return (uint8_t*)t->s; } /* little-endian host */
/* Absorb and squeeze a block's worth of bytes at a time (the rate region is XORed / copied as one
 * run), as the sha3 crate's sponge does, not byte by byte. */
static void sp_absorb(sponge* t, const uint8_t* d, size_t n) {
  uint8_t* b = sp_bytes(t);
  while (n) {
    size_t k = TS_RATE - t->pos;
    if (k > n) k = n;
    for (size_t i = 0; i < k; i++) b[t->pos + i] ^= d[i];
    t->pos += (uint32_t)k;
    d += k;
    n -= k;
    if (t->pos == TS_RATE) {
      orc_keccak_p1600(t->s, t->rounds);
      t->pos = 0;
    }
  }
}
static void sp_finalize(sponge* t, uint8_t domain) {
  uint8_t* b = sp_bytes(t);
  b[t->pos] ^= domain;
  b[TS_RATE - 1] ^= 0x80;
  orc_keccak_p1600(t->s, t->rounds);
  t->pos = 0;
}
static void sp_squeeze(sponge* t, uint8_t* out, size_t n) {
  const uint8_t* b = sp_bytes(t);
  while (n) {
    if (t->pos == TS_RATE) {
      orc_keccak_p1600(t->s, t->rounds);
      t->pos = 0;
    }
    size_t k = TS_RATE - t->pos;
    if (k > n) k = n;
    memcpy(out, b + t->pos, k);
    t->pos += (uint32_t)k;
    out += k;
    n -= k;
  }
}

void orc_turboshake128(const uint8_t* msg, size_t len, uint8_t domain, uint8_t* out,
                       size_t out_len) {
  sponge t;
  sp_init(&t, 12);
  sp_absorb(&t, msg, len);
  sp_finalize(&t, domain);
  sp_squeeze(&t, out, out_len);
}
void orc_shake128(const uint8_t* msg, size_t len, uint8_t* out, size_t out_len) {
  sponge t;
  sp_init(&t, 24);
  sp_absorb(&t, msg, len);
  sp_finalize(&t, 0x1F);
  sp_squeeze(&t, out, out_len);
}

/* XofTurboShake128(seed, dst, binder) = TurboSHAKE128(len(dst) || dst || seed || binder, D=1)
 * [VDAF-08 §6.2.1; prio vdaf/xof.rs XofTurboShake128::init], and XofHmacSha256Aes128 (prio 0.16,
 * SEED_SIZE 32; restated in oracle/prio3_py.py): tag = HMAC-SHA256(seed, len(dst) || dst ||
 * binder), then an AES-128 keystream, key tag[0:16], IV tag[16:32] with a 64-bit big-endian
 * counter in its low half (Ctr64BE). */
typedef struct {
  int hm;
  sponge sp;
  EVP_MD_CTX* md;
  uint8_t okey[64];
  EVP_CIPHER_CTX* aes;
  uint8_t iv[16], ks[16];
  uint64_t ctr;
  uint32_t kpos;
} xof_t;
static void xf_init(xof_t* x, int hm, const uint8_t* seed, size_t seed_len, const uint8_t* dst,
                    size_t dst_len) {
  const uint8_t l = (uint8_t)dst_len;
  x->hm = hm;
  x->md = NULL;
  x->aes = NULL;
  if (!hm) {
    sp_init(&x->sp, 12);
    sp_absorb(&x->sp, &l, 1);
    sp_absorb(&x->sp, dst, dst_len);
    sp_absorb(&x->sp, seed, seed_len);
    return;
  }
  uint8_t ikey[64];
  memset(ikey, 0x36, 64);
  memset(x->okey, 0x5c, 64);
  for (size_t i = 0; i < seed_len; i++) {  /* seed_len <= 64: the key is used as is */
    ikey[i] ^= seed[i];
    x->okey[i] ^= seed[i];
  }
  x->md = EVP_MD_CTX_new();
  EVP_DigestInit_ex(x->md, EVP_sha256(), NULL);
  EVP_DigestUpdate(x->md, ikey, 64);
  EVP_DigestUpdate(x->md, &l, 1);
  EVP_DigestUpdate(x->md, dst, dst_len);
}
static void xf_absorb(xof_t* x, const uint8_t* d, size_t n) {
  if (x->hm)
    EVP_DigestUpdate(x->md, d, n);
  else
    sp_absorb(&x->sp, d, n);
}
static void xf_finalize(xof_t* x) {
  if (!x->hm) {
    sp_finalize(&x->sp, 1);
    return;
  }
  uint8_t inner[32], tag[32];
  unsigned int len = 0;
  EVP_DigestFinal_ex(x->md, inner, &len);
  EVP_DigestInit_ex(x->md, EVP_sha256(), NULL);
  EVP_DigestUpdate(x->md, x->okey, 64);
  EVP_DigestUpdate(x->md, inner, 32);
  EVP_DigestFinal_ex(x->md, tag, &len);
  x->aes = EVP_CIPHER_CTX_new();
  EVP_EncryptInit_ex(x->aes, EVP_aes_128_ecb(), NULL, tag, NULL);
  EVP_CIPHER_CTX_set_padding(x->aes, 0);
  memcpy(x->iv, tag + 16, 16);
  x->ctr = 0;
  for (int i = 0; i < 8; i++) x->ctr = x->ctr << 8 | x->iv[8 + i];
  x->kpos = 16;
}
static void xf_squeeze(xof_t* x, uint8_t* out, size_t n) {
  if (!x->hm) {
    sp_squeeze(&x->sp, out, n);
    return;
  }
  while (n--) {
    if (x->kpos == 16) {
      uint8_t blk[16];
      int l = 0;
      memcpy(blk, x->iv, 8);
      for (int i = 0; i < 8; i++) blk[8 + i] = (uint8_t)(x->ctr >> (56 - 8 * i));
      x->ctr++;
      EVP_EncryptUpdate(x->aes, x->ks, &l, blk, 16);
      x->kpos = 0;
    }
    *out++ = x->ks[x->kpos++];
  }
}
static void xf_free(xof_t* x) {
  if (x->md) EVP_MD_CTX_free(x->md);
  if (x->aes) EVP_CIPHER_CTX_free(x->aes);
  x->md = NULL;
  x->aes = NULL;
}

/* ------------------------------------------------------------------------------------ */
/* Fields [VDAF-08 §6.1.2]: Field64 p = 2^64 - 2^32 + 1, Field128 p = 2^128 - 28*2^64 + 1  */
/* Elements are canonical integers in [0, p) held in a u128 for both fields.             */
/* ------------------------------------------------------------------------------------ */
typedef u128 fe;
#define P64 0xffffffff00000001ULL
static const u128 P128 = (((u128)0xffffffffffffffe4ULL) << 64) | 1;
static const u128 C1_128 = (((u128)27) << 64) | 0xffffffffffffffffULL; /* 2^128 mod p = 28*2^64-1 */

typedef struct {
  int is128;
  u128 p;
} fld;

static inline fe f_add(const fld* F, fe a, fe b) {
  if (F->is128) {
    u128 s = a + b;
    if (s < a || s >= P128) s -= P128;
    return s;
  }
  u128 s = a + b;
  return s >= P64 ? s - P64 : s;
}
static inline fe f_sub(const fld* F, fe a, fe b) {
  if (a >= b) return a - b;
  return a + (F->p - b);
}
static inline fe f_neg(const fld* F, fe a) { return a ? F->p - a : 0; }

static inline uint64_t f64_reduce128(u128 x) {
  uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
  uint64_t hh = hi >> 32, hl = hi & 0xffffffffULL;
  uint64_t t0 = lo - hh;
  if (lo < hh) t0 -= 0xffffffffULL;
  uint64_t t1 = hl * 0xffffffffULL;
  uint64_t r = t0 + t1;
  if (r < t0) r += 0xffffffffULL;
  if (r >= P64) r -= P64;
  return r;
}

static inline u128 f128_mul(u128 a, u128 b) {
  uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64);
  uint64_t b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  u128 p00 = (u128)a0 * b0, p01 = (u128)a0 * b1, p10 = (u128)a1 * b0, p11 = (u128)a1 * b1;
  u128 mid = p01 + p10;
  uint64_t cmid = mid < p01;
  u128 lo = p00 + (mid << 64);
  uint64_t clo = lo < p00;
  u128 hi = p11 + (mid >> 64) + ((u128)cmid << 64) + clo;
  /* X = hi*2^128 + lo;  2^128 = 28*2^64 - 1,  2^192 = 783*2^64 - 28  (mod p) */
  uint64_t h0 = (uint64_t)hi, h1 = (uint64_t)(hi >> 64);
  u128 T = (u128)h0 * 28 + (u128)h1 * 783;
  uint64_t tlo = (uint64_t)T, t2 = (uint64_t)(T >> 64);
  u128 U = (u128)tlo + (u128)t2 * 28;
  int carry = (int)(U >> 64);
  u128 acc = lo, add = U << 64;
  acc += add;
  if (acc < add) carry++;
  u128 sub = (u128)h0 + (u128)h1 * 28 + t2;
  if (acc < sub) carry--;
  acc -= sub;
  while (carry > 0) {
    u128 c = (u128)(unsigned)carry * C1_128;
    carry = 0;
    acc += c;
    if (acc < c) carry = 1;
  }
  while (carry < 0) {
    carry++;
    if (acc < C1_128) carry--;
    acc -= C1_128;
  }
  while (acc >= P128) acc -= P128;
  return acc;
}

static inline fe f_mul(const fld* F, fe a, fe b) {
  if (F->is128) return f128_mul(a, b);
  return f64_reduce128((u128)(uint64_t)a * (uint64_t)b);
}
static fe f_pow(const fld* F, fe a, u128 e) {
  fe r = 1;
  while (e) {
    if (e & 1) r = f_mul(F, r, a);
    a = f_mul(F, a, a);
    e >>= 1;
  }
  return r;
}
static fe f_inv(const fld* F, fe a) { return f_pow(F, a, F->p - 2); }
static fe f_from_u64(const fld* F, uint64_t x) { return F->is128 ? (fe)x : (fe)(x % P64); }

/* Generator of the 2^num_roots subgroup [prio fp.rs FP64/FP128 `g`; VDAF-08 §6.1.2]. */
/* roots[l] = g^(2^(num_roots - l)), the principal 2^l-th root (prio FieldParameters::roots). */
#define MAX_ROOTS 20
static fe ROOTS64[MAX_ROOTS + 1], ROOTS128[MAX_ROOTS + 1];
static pthread_once_t roots_once = PTHREAD_ONCE_INIT;
static void roots_init(void) {
  fld F64 = {0, (u128)P64}, F128 = {1, 0};
  F128.p = P128;
  fe g128 = 0;
  for (const char* c = "145091266659756586618791329697897684742"; *c; c++)
    g128 = g128 * 10 + (u128)(*c - '0');
  fe g64 = 1753635133440165772ULL;
  for (int l = 0; l <= MAX_ROOTS; l++) {
    fe r = g128;
    for (int i = 0; i < 66 - l; i++) r = f_mul(&F128, r, r);
    ROOTS128[l] = r;
    r = g64;
    for (int i = 0; i < 32 - l; i++) r = f_mul(&F64, r, r);
    ROOTS64[l] = r;
  }
}
static fe f_root(const fld* F, int l) {
  pthread_once(&roots_once, roots_init);
  return F->is128 ? ROOTS128[l] : ROOTS64[l];
}

static void enc_fe(const fld* F, fe x, uint8_t* out) {
  int n = F->is128 ? 16 : 8;
  for (int i = 0; i < n; i++) out[i] = (uint8_t)(x >> (8 * i));
}
static int dec_fe(const fld* F, const uint8_t* in, fe* x) {
  int n = F->is128 ? 16 : 8;
  u128 v = 0;
  for (int i = n - 1; i >= 0; i--) v = (v << 8) | in[i];
  if (v >= F->p) return -1;
  *x = v;
  return 0;
}

/* Xof.expand_into_vec with rejection sampling [VDAF-08 §6.2; prio Prng::get]. */
static void xof_expand(const fld* F, xof_t* t, fe* out, uint32_t n) {
  int es = F->is128 ? 16 : 8;
  uint8_t buf[16];
  for (uint32_t i = 0; i < n;) {
    xf_squeeze(t, buf, es);
    u128 v = 0;
    for (int k = es - 1; k >= 0; k--) v = (v << 8) | buf[k];
    if (v < F->p) out[i++] = v;
  }
}

/* ------------------------------------------------------------------------------------ */
/* Polynomials / DFT -- mirrors prio fft.rs discrete_fourier_transform (bit-reversed      */
/* input, iterative butterflies with roots(l)), discrete_fourier_transform_inv_finish     */
/* and polynomial.rs poly_eval.                                                           */
/* ------------------------------------------------------------------------------------ */
static uint32_t log2u(uint32_t n) {
  uint32_t d = 0;
  while ((1u << d) < n) d++;
  return d;
}
static uint32_t bitrev(uint32_t d, uint32_t x) {
  uint32_t y = 0;
  for (uint32_t i = 0; i < d; i++) {
    y = (y << 1) | (x & 1);
    x >>= 1;
  }
  return y;
}
static void dft(const fld* F, fe* outp, const fe* inp, uint32_t inp_len, uint32_t size) {
  uint32_t d = log2u(size);
  for (uint32_t i = 0; i < size; i++) {
    uint32_t j = bitrev(d, i);
    outp[i] = j < inp_len ? inp[j] : 0;
  }
  for (uint32_t l = 1; l <= d; l++) {
    fe w = 1, r = f_root(F, (int)l);
    uint32_t y = 1u << (l - 1), chunk = (size / y) >> 1;
    for (uint32_t i = 0; i < y; i++) {
      for (uint32_t j = 0; j < chunk; j++) {
        uint32_t x = j << l;
        fe u = outp[i + x], v = f_mul(F, w, outp[i + x + y]);
        outp[i + x] = f_add(F, u, v);
        outp[i + x + y] = f_sub(F, u, v);
      }
      w = f_mul(F, w, r);
    }
  }
}
static void dft_inv_finish(const fld* F, fe* outp, uint32_t size, fe size_inv) {
  outp[0] = f_mul(F, outp[0], size_inv);
  outp[size >> 1] = f_mul(F, outp[size >> 1], size_inv);
  for (uint32_t i = 1; i < (size >> 1); i++) {
    fe tmp = f_mul(F, outp[i], size_inv);
    outp[i] = f_mul(F, outp[size - i], size_inv);
    outp[size - i] = tmp;
  }
}
static fe poly_eval(const fld* F, const fe* poly, uint32_t len, fe x) {
  fe r = 0;
  for (uint32_t i = len; i-- > 0;) r = f_add(F, f_mul(F, r, x), poly[i]);
  return r;
}

/* ------------------------------------------------------------------------------------ */
/* Parameters [VDAF-08 §7.4 (Prio3Count/Sum/SumVec/Histogram); core/src/vdaf.rs:198-300] */
/* ------------------------------------------------------------------------------------ */
static uint32_t next_pow2(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

/* prio flp/gadgets.rs optimal_chunk_length (restated as in oracle/fpvec_py.py): the chunk length
 * minimising 2 chunk + 2 ((1 + calls).next_power_of_two() - 1) + 1 over calls = 2^k - 1, the
 * first minimum from the largest k down */
static uint32_t optimal_chunk_length(uint32_t meas_len) {
  if (meas_len <= 1) return 1;
  uint32_t max_log2 = log2u(next_pow2(meas_len)) + 1, best_cost = 0, best = 1;
  for (uint32_t l2 = max_log2; l2 >= 1; l2--) {
    const uint32_t calls = (1u << l2) - 1, chunk = (meas_len + calls - 1) / calls;
    const uint32_t cost = 2 * chunk + 2 * (next_pow2(1 + calls) - 1) + 1;
    if (l2 == max_log2 || cost < best_cost) {
      best_cost = cost;
      best = chunk;
    }
  }
  return best;
}

int orc_params_init(orc_params* p, int type, uint32_t bits, uint32_t length,
                    uint32_t chunk_length, uint32_t num_proofs) {
  memset(p, 0, sizeof *p);
  p->type = type;
  p->bits = bits;
  p->length = length;
  p->chunk_length = chunk_length;
  p->num_proofs = num_proofs ? num_proofs : 1;
  if (p->num_proofs > 255) return -1;
  p->seed_size = 16;
  p->qr_len = 1;
  p->degree = 2;
  switch (type) {
    case ORC_COUNT: /* Prio3::new_count(2): Count<Field64>, Mul gadget, 1 call */
      p->algorithm_id = 0;
      p->field_bits = 64;
      p->meas_len = 1;
      p->out_len = 1;
      p->jr_len = 0;
      p->arity = 2;
      p->calls = 1;
      break;
    case ORC_SUM: /* Prio3::new_sum(2, bits): Sum<Field128>, PolyEval(x^2-x) x bits */
      if (bits == 0 || bits > 64) return -1;
      p->algorithm_id = 1;
      p->field_bits = 128;
      p->meas_len = bits;
      p->out_len = 1;
      p->jr_len = 1;
      p->arity = 1;
      p->calls = bits;
      break;
    case ORC_SUMVEC: /* SumVec<Field128, ParallelSum<Mul>> */
      if (bits == 0 || bits > 64 || length == 0 || chunk_length == 0) return -1;
      p->algorithm_id = 2;
      p->field_bits = 128;
      p->meas_len = bits * length;
      p->out_len = length;
      p->jr_len = 1;
      p->arity = 2 * chunk_length;
      p->calls = (p->meas_len + chunk_length - 1) / chunk_length;
      break;
    case ORC_HISTOGRAM: /* Histogram<Field128, ParallelSum<Mul>> */
      if (length == 0 || chunk_length == 0) return -1;
      p->algorithm_id = 3;
      p->field_bits = 128;
      p->meas_len = length;
      p->out_len = length;
      p->jr_len = 2;
      p->arity = 2 * chunk_length;
      p->calls = (length + chunk_length - 1) / chunk_length;
      break;
    case ORC_SUMVEC_F64_MP: /* SumVec<Field64, ParallelSum<Mul>>, XofHmacSha256Aes128,
                               algorithm id 0xFFFF1003 (core/src/vdaf.rs:20, 173-195) */
      if (bits == 0 || bits > 64 || length == 0 || chunk_length == 0 || p->num_proofs < 2)
        return -1;
      p->algorithm_id = 0xFFFF1003u;
      p->field_bits = 64;
      p->meas_len = bits * length;
      p->out_len = length;
      p->jr_len = 1;
      p->arity = 2 * chunk_length;
      p->calls = (p->meas_len + chunk_length - 1) / chunk_length;
      p->seed_size = 32;
      p->xof_hm = 1;
      break;
    case ORC_FPVEC: /* FixedPointBoundedL2VecSum (reconstruction, oracle/fpvec_py.py) */
      if ((bits != 16 && bits != 32) || length == 0 || p->num_proofs != 1) return -1;
      p->algorithm_id = 0xFFFF0000u;
      p->field_bits = 128;
      p->meas_len = bits * length + 2 * bits - 2;
      p->out_len = length;
      p->jr_len = 2;
      p->qr_len = 2;
      p->chunk_length = optimal_chunk_length(p->meas_len);
      p->arity = 2 * p->chunk_length;
      p->calls = (p->meas_len + p->chunk_length - 1) / p->chunk_length;
      p->fp_C1 = optimal_chunk_length(length);
      p->fp_K1 = (length + p->fp_C1 - 1) / p->fp_C1;
      p->fp_P1 = next_pow2(1 + p->fp_K1);
      break;
    default:
      return -1;
  }
  p->es = p->field_bits / 8;
  p->prove_rand_len = p->arity;
  p->wire_len = next_pow2(1 + p->calls);
  p->proof_len = p->arity + p->degree * (p->wire_len - 1) + 1;
  p->verifier_len = 1 + p->arity + 1;
  if (type == ORC_FPVEC) {  /* proof = seeds0 | coeffs0 | seeds1 | coeffs1 */
    p->prove_rand_len = p->arity + p->fp_C1;
    p->proof_len += p->fp_C1 + 2 * (p->fp_P1 - 1) + 1;
    p->verifier_len += p->fp_C1 + 1;
  }
  const uint32_t S = p->seed_size;
  if (p->jr_len * p->num_proofs > 64 || p->qr_len * p->num_proofs > 64) return -1;
  p->helper_share_len = S * (p->jr_len ? 3 : 2);
  p->public_share_len = p->jr_len ? 2 * S : 0;
  p->leader_share_len =
      (p->meas_len + p->proof_len * p->num_proofs) * p->es + (p->jr_len ? S : 0);
  p->prep_share_len = p->verifier_len * p->num_proofs * p->es + (p->jr_len ? S : 0);
  p->prep_msg_len = p->jr_len ? S : 0;
  p->out_share_bytes = p->out_len * p->es;
  return 0;
}

static fld mkfld(const orc_params* p) {
  fld F;
  F.is128 = p->field_bits == 128;
  F.p = F.is128 ? P128 : (u128)P64;
  return F;
}

/* format_dst(algo_class=0, algo, usage) [VDAF-08 §7.2.1 / prio Prio3::domain_separation_tag] */
static void mkdst(const orc_params* p, uint16_t usage, uint8_t dst[8]) {
  dst[0] = 8; /* VERSION */
  dst[1] = 0; /* algorithm class: VDAF */
  dst[2] = (uint8_t)(p->algorithm_id >> 24);
  dst[3] = (uint8_t)(p->algorithm_id >> 16);
  dst[4] = (uint8_t)(p->algorithm_id >> 8);
  dst[5] = (uint8_t)(p->algorithm_id);
  dst[6] = (uint8_t)(usage >> 8);
  dst[7] = (uint8_t)usage;
}
enum {
  U_MEAS_SHARE = 1,
  U_PROOF_SHARE = 2,
  U_JOINT_RANDOMNESS = 3,
  U_PROVE_RANDOMNESS = 4,
  U_QUERY_RANDOMNESS = 5,
  U_JOINT_RAND_SEED = 6,
  U_JOINT_RAND_PART = 7
};

static void xof_for(const orc_params* p, xof_t* t, const uint8_t* seed, uint16_t usage) {
  uint8_t dst[8];
  mkdst(p, usage, dst);
  xf_init(t, (int)p->xof_hm, seed, p->seed_size, dst, 8);
}

/* ------------------------------------------------------------------------------------ */
/* FLP (FlpBBCGGI19, [VDAF-08 §7.3]; prio flp.rs FlpGeneric) with shim gadgets           */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  const fld* F;
  const orc_params* p;
  int prove; /* 1: ProveShimGadget (evaluate inner), 0: QueryShimGadget */
  uint32_t ct;
  fe* f_vals;  /* arity x wire_len (row = wire), zero-padded */
  fe* p_vals;  /* query: gadget polynomial at the 2P-th roots */
  uint32_t step;
} shim;

static fe gadget_eval(const fld* F, const orc_params* p, const fe* x) {
  switch (p->type) {
    case ORC_COUNT:
      return f_mul(F, x[0], x[1]); /* Mul */
    case ORC_SUM:
      return f_sub(F, f_mul(F, x[0], x[0]), x[0]); /* PolyEval([0,-1,1]) */
    default: {                                     /* ParallelSum(Mul, chunk) */
      fe s = 0;
      for (uint32_t j = 0; j < p->chunk_length; j++)
        s = f_add(F, s, f_mul(F, x[2 * j], x[2 * j + 1]));
      return s;
    }
  }
}

static fe shim_call(shim* s, const fe* x) {
  const orc_params* p = s->p;
  for (uint32_t w = 0; w < p->arity; w++) s->f_vals[w * p->wire_len + s->ct] = x[w];
  fe y = s->prove ? gadget_eval(s->F, p, x) : s->p_vals[s->ct * s->step];
  s->ct++;
  return y;
}

/* parallel_sum_range_checks [prio flp/types.rs; VDAF-08 §7.4.3/7.4.4 valid()] */
static fe range_checks(shim* s, const fe* in, uint32_t n, fe r, fe shares_inv, fe* args) {
  const fld* F = s->F;
  uint32_t c = s->p->chunk_length;
  fe out = 0, rp = r;
  for (uint32_t base = 0; base < n; base += c) {
    for (uint32_t j = 0; j < c; j++) {
      uint32_t i = base + j;
      fe m = i < n ? in[i] : 0; /* padding: measurement element 0 */
      args[2 * j] = f_mul(F, rp, m);
      args[2 * j + 1] = f_sub(F, m, shares_inv);
      rp = f_mul(F, rp, r);
    }
    out = f_add(F, out, shim_call(s, args));
  }
  return out;
}

static fe valid(shim* s, const fe* in, const fe* jr, uint32_t num_shares) {
  const fld* F = s->F;
  const orc_params* p = s->p;
  fe shares_inv = f_inv(F, f_from_u64(F, num_shares));
  switch (p->type) {
    case ORC_COUNT: { /* Count::valid: g(m, m) - m */
      fe x[2] = {in[0], in[0]};
      return f_sub(F, shim_call(s, x), in[0]);
    }
    case ORC_SUM: { /* Sum::valid: sum_i r^(i+1) * g(m_i) */
      fe out = 0, r = jr[0];
      for (uint32_t i = 0; i < p->meas_len; i++) {
        out = f_add(F, out, f_mul(F, r, shim_call(s, &in[i])));
        r = f_mul(F, r, jr[0]);
      }
      return out;
    }
    case ORC_SUMVEC:
    case ORC_SUMVEC_F64_MP: {
      fe* args = (fe*)malloc(sizeof(fe) * p->arity);
      fe out = range_checks(s, in, p->meas_len, jr[0], shares_inv, args);
      free(args);
      return out;
    }
    case ORC_HISTOGRAM: {
      fe* args = (fe*)malloc(sizeof(fe) * p->arity);
      fe rc = range_checks(s, in, p->meas_len, jr[0], shares_inv, args);
      free(args);
      fe sc = f_neg(F, shares_inv);
      for (uint32_t i = 0; i < p->meas_len; i++) sc = f_add(F, sc, in[i]);
      return f_add(F, f_mul(F, jr[1], rc), f_mul(F, f_mul(F, jr[1], jr[1]), sc));
    }
  }
  return 0;
}

/* FlpGeneric::query -> verifier (verifier_len elements). Returns -1 if t is a P-th root. */
static int flp_query(const fld* F, const orc_params* p, const fe* meas, const fe* proof,
                     const fe* qr, const fe* jr, fe* verifier) {
  uint32_t P = p->wire_len, size = next_pow2(P * p->degree);
  fe t = qr[0];
  if (f_pow(F, t, P) == 1) return -1;
  uint32_t glen = p->degree * (P - 1) + 1;
  shim s;
  s.F = F;
  s.p = p;
  s.prove = 0;
  s.ct = 1;
  s.f_vals = (fe*)calloc((size_t)p->arity * P, sizeof(fe));
  s.p_vals = (fe*)malloc(sizeof(fe) * size);
  s.step = size / P;
  dft(F, s.p_vals, proof + p->arity, glen, size);
  fe p_at_r = poly_eval(F, proof + p->arity, glen, t);
  for (uint32_t w = 0; w < p->arity; w++) s.f_vals[w * P] = proof[w];
  verifier[0] = valid(&s, meas, jr, 2);
  fe* f = (fe*)malloc(sizeof(fe) * P);
  fe m_inv = f_inv(F, P);
  for (uint32_t w = 0; w < p->arity; w++) {
    dft(F, f, s.f_vals + (size_t)w * P, 1 + p->calls, P);
    dft_inv_finish(F, f, P, m_inv);
    verifier[1 + w] = poly_eval(F, f, P, t);
  }
  verifier[1 + p->arity] = p_at_r;
  free(f);
  free(s.f_vals);
  free(s.p_vals);
  return 0;
}

/* FlpGeneric::decide */
static int flp_decide(const fld* F, const orc_params* p, const fe* v) {
  if (v[0] != 0) return 0;
  return gadget_eval(F, p, v + 1) == v[1 + p->arity];
}

/* FixedPointBoundedL2VecSum query (oracle/fpvec_py.py FpVecType.query, the two-gadget FLP):
 * verifier = [v, f0(t0) (A0 wires), p0(t0), f1(t1) (C1 wires), p1(t1)]. */
static int fpvec_query(const fld* F, const orc_params* p, const fe* meas, const fe* proof,
                       const fe* qr, const fe* jr, fe* ver) {
  const uint32_t A0 = p->arity, C0 = p->chunk_length, K0 = p->calls, P0 = p->wire_len;
  const uint32_t C1 = p->fp_C1, K1 = p->fp_K1, P1 = p->fp_P1, n = p->bits, E = p->length;
  const uint32_t G0 = 2 * (P0 - 1) + 1, G1 = 2 * (P1 - 1) + 1, M = p->meas_len;
  const fe *s0 = proof, *c0 = s0 + A0, *s1 = c0 + G0, *c1 = s1 + C1;
  const fe t0 = qr[0], t1 = qr[1];
  if (f_pow(F, t0, P0) == 1 || f_pow(F, t1, P1) == 1) return -1;
  /* gadget polynomials at the P-th roots: coefficients folded mod x^P - 1, one DFT */
  fe* fold = (fe*)calloc(P0 > P1 ? P0 : P1, sizeof(fe));
  fe* pr0 = (fe*)malloc(sizeof(fe) * P0);
  fe* pr1 = (fe*)malloc(sizeof(fe) * P1);
  for (uint32_t i = 0; i < G0; i++) fold[i % P0] = f_add(F, fold[i % P0], c0[i]);
  dft(F, pr0, fold, P0, P0);
  memset(fold, 0, sizeof(fe) * (P0 > P1 ? P0 : P1));
  for (uint32_t i = 0; i < G1; i++) fold[i % P1] = f_add(F, fold[i % P1], c1[i]);
  dft(F, pr1, fold, P1, P1);
  /* Lagrange basis at t: L_c(t) = alpha^c (t^P - 1) / (P (t - alpha^c)), c = 0..K, with one
   * field inversion per gadget (batch inversion of the t - alpha^c) */
  const uint32_t KM = K0 > K1 ? K0 : K1;
  fe* L0 = (fe*)malloc(sizeof(fe) * (KM + 1) * 3);
  fe *Lg = L0, *pre = L0 + (KM + 1), *den = L0 + 2 * (KM + 1);
  fe* Lb1 = (fe*)malloc(sizeof(fe) * (K1 + 1));
  for (int g = 0; g < 2; g++) {
    const uint32_t P = g ? P1 : P0, K = g ? K1 : K0;
    const fe t = g ? t1 : t0;
    fe* L = g ? Lb1 : Lg;
    const fe num = f_mul(F, f_sub(F, f_pow(F, t, P), 1), f_inv(F, P)), a = f_root(F, (int)log2u(P));
    fe ac = 1, acc = 1;
    for (uint32_t c = 0; c <= K; c++) {
      den[c] = f_sub(F, t, ac);
      pre[c] = acc;  /* product of den[0..c-1] */
      acc = f_mul(F, acc, den[c]);
      L[c] = ac;
      ac = f_mul(F, ac, a);
    }
    fe inv = f_inv(F, acc);  /* 1 / prod den */
    for (uint32_t c = K + 1; c-- > 0;) {
      const fe ic = f_mul(F, inv, pre[c]);  /* 1 / den[c] */
      inv = f_mul(F, inv, den[c]);
      L[c] = f_mul(F, f_mul(F, L[c], ic), num);
    }
  }
  /* valid() with each gadget call's wire values folded straight into the wire polynomials at t
   * (f_w(t) = sum_c L_c(t) w[c], row c = 0 the proof's seeds): gadget 0's wires 2j, 2j+1 carry
   * r^(i+1) m_i and m_i - 1/2 (i = k C0 + j, m = 0 past the share), gadget 1's wire j the
   * decoded entry k C1 + j (0 past the last) */
  fe* out0 = ver + 1;
  fe* out1 = ver + 2 + A0;
  for (uint32_t w = 0; w < A0; w++) out0[w] = f_mul(F, Lg[0], s0[w]);
  for (uint32_t w = 0; w < C1; w++) out1[w] = f_mul(F, Lb1[0], s1[w]);
  const fe sinv = f_inv(F, 2);
  fe rng = 0, rp = jr[0];
  for (uint32_t k = 0; k < K0; k++) {
    const fe Lk = Lg[k + 1];
    for (uint32_t j = 0; j < C0; j++) {
      const uint32_t i = k * C0 + j;
      const fe m = i < M ? meas[i] : 0;
      out0[2 * j] = f_add(F, out0[2 * j], f_mul(F, Lk, f_mul(F, rp, m)));
      out0[2 * j + 1] = f_add(F, out0[2 * j + 1], f_mul(F, Lk, f_sub(F, m, sinv)));
      rp = f_mul(F, rp, jr[0]);
    }
    rng = f_add(F, rng, pr0[k + 1]);
  }
  fe norm = 0;
  for (uint32_t k = 0; k < K1; k++) {
    for (uint32_t j = 0; j < C1; j++) {
      const uint32_t e = k * C1 + j;
      fe y = 0;
      if (e < E)
        for (uint32_t b = n; b-- > 0;) y = f_add(F, f_add(F, y, y), meas[n * e + b]);
      out1[j] = f_add(F, out1[j], f_mul(F, Lb1[k + 1], y));
    }
    norm = f_add(F, norm, pr1[k + 1]);
  }
  norm = f_add(F, norm, f_mul(F, f_mul(F, (fe)E, (fe)1 << (2 * n - 2)), sinv));
  fe claimed = 0;
  for (uint32_t b = 2 * n - 2; b-- > 0;) claimed = f_add(F, f_add(F, claimed, claimed), meas[n * E + b]);
  ver[0] = f_add(F, f_mul(F, jr[1], rng),
                 f_mul(F, f_mul(F, jr[1], jr[1]), f_sub(F, norm, claimed)));
  free(L0);
  free(Lb1);
  ver[1 + A0] = poly_eval(F, c0, G0, t0);
  ver[2 + A0 + C1] = poly_eval(F, c1, G1, t1);
  free(fold);
  free(pr0);
  free(pr1);
  return 0;
}

static int fpvec_decide(const fld* F, const orc_params* p, const fe* v) {
  if (v[0] != 0) return 0;
  const uint32_t A0 = p->arity, C1 = p->fp_C1;
  fe g0 = 0, g1 = 0;
  for (uint32_t j = 0; j < p->chunk_length; j++)
    g0 = f_add(F, g0, f_mul(F, v[1 + 2 * j], v[2 + 2 * j]));
  const fe twon = (fe)1 << p->bits;
  for (uint32_t j = 0; j < C1; j++) {
    const fe y = v[2 + A0 + j];
    g1 = f_add(F, g1, f_sub(F, f_mul(F, y, y), f_mul(F, twon, y)));
  }
  return g0 == v[1 + A0] && g1 == v[2 + A0 + C1];
}

/* FlpGeneric::prove (client side; used only to synthesise honest reports). */
static void flp_prove(const fld* F, const orc_params* p, const fe* meas, const fe* prove_rand,
                      const fe* jr, fe* proof) {
  uint32_t P = p->wire_len, size = next_pow2(P * p->degree);
  uint32_t glen = p->degree * (P - 1) + 1;
  shim s;
  s.F = F;
  s.p = p;
  s.prove = 1;
  s.ct = 1;
  s.f_vals = (fe*)calloc((size_t)p->arity * P, sizeof(fe));
  s.p_vals = NULL;
  s.step = 0;
  for (uint32_t w = 0; w < p->arity; w++) s.f_vals[w * P] = prove_rand[w];
  (void)valid(&s, meas, jr, 1);
  fe m_inv = f_inv(F, P), size_inv = f_inv(F, size);
  fe* coef = (fe*)malloc(sizeof(fe) * P);
  fe* evals = (fe*)malloc(sizeof(fe) * (size_t)p->arity * size);
  for (uint32_t w = 0; w < p->arity; w++) {
    dft(F, coef, s.f_vals + (size_t)w * P, 1 + p->calls, P);
    dft_inv_finish(F, coef, P, m_inv);
    proof[w] = s.f_vals[(size_t)w * P];
    dft(F, evals + (size_t)w * size, coef, P, size); /* wire poly at 2P-th roots */
  }
  fe* g = (fe*)malloc(sizeof(fe) * size);
  fe* x = (fe*)malloc(sizeof(fe) * p->arity);
  for (uint32_t k = 0; k < size; k++) {
    for (uint32_t w = 0; w < p->arity; w++) x[w] = evals[(size_t)w * size + k];
    g[k] = gadget_eval(F, p, x);
  }
  fe* gc = (fe*)malloc(sizeof(fe) * size);
  dft(F, gc, g, size, size);
  dft_inv_finish(F, gc, size, size_inv);
  for (uint32_t k = 0; k < glen; k++) proof[p->arity + k] = gc[k];
  free(coef);
  free(evals);
  free(g);
  free(x);
  free(gc);
  free(s.f_vals);
}

/* ------------------------------------------------------------------------------------ */
/* Prio3 [VDAF-08 §7.2]                                                                  */
/* ------------------------------------------------------------------------------------ */
static void expand_seed(const orc_params* p, const fld* F, const uint8_t* seed, uint16_t usage,
                        const uint8_t* binder, size_t blen, fe* out, uint32_t n) {
  xof_t t;
  xof_for(p, &t, seed, usage);
  xf_absorb(&t, binder, blen);
  xf_finalize(&t);
  xof_expand(F, &t, out, n);
  xf_free(&t);
}
static void derive_seed(const orc_params* p, const uint8_t* seed, uint16_t usage,
                        const uint8_t* binder, size_t blen, uint8_t* out) {
  xof_t t;
  xof_for(p, &t, seed, usage);
  xf_absorb(&t, binder, blen);
  xf_finalize(&t);
  xf_squeeze(&t, out, p->seed_size);
  xf_free(&t);
}
static void helper_meas_share(const orc_params* p, const fld* F, const uint8_t* k, uint8_t agg,
                              fe* out) {
  expand_seed(p, F, k, U_MEAS_SHARE, &agg, 1, out, p->meas_len);
}
static void helper_proofs_share(const orc_params* p, const fld* F, const uint8_t* k,
                                uint8_t agg, fe* out) {
  uint8_t b[2] = {(uint8_t)p->num_proofs, agg};
  expand_seed(p, F, k, U_PROOF_SHARE, b, 2, out, p->proof_len * p->num_proofs);
}
static void joint_rand_part(const orc_params* p, const fld* F, const uint8_t* blind, uint8_t agg,
                            const uint8_t nonce[16], const fe* meas, uint8_t* out) {
  xof_t t;
  xof_for(p, &t, blind, U_JOINT_RAND_PART);
  xf_absorb(&t, &agg, 1);
  xf_absorb(&t, nonce, 16);
  uint8_t buf[16 * 64];
  uint32_t nb = 0;
  for (uint32_t i = 0; i < p->meas_len; i++) {  /* absorbed 64 elements at a time */
    enc_fe(F, meas[i], buf + nb * p->es);
    if (++nb == 64) {
      xf_absorb(&t, buf, nb * p->es);
      nb = 0;
    }
  }
  xf_absorb(&t, buf, nb * p->es);
  xf_finalize(&t);
  xf_squeeze(&t, out, p->seed_size);
  xf_free(&t);
}
static void joint_rand_seed(const orc_params* p, const uint8_t* part0, const uint8_t* part1,
                            uint8_t* out) {
  static const uint8_t zero[32] = {0};
  uint8_t b[64];
  const uint32_t S = p->seed_size;
  memcpy(b, part0, S);
  memcpy(b + S, part1, S);
  derive_seed(p, zero, U_JOINT_RAND_SEED, b, 2 * S, out);
}
static void joint_rands(const orc_params* p, const fld* F, const uint8_t* seed, fe* out) {
  uint8_t b = (uint8_t)p->num_proofs;
  expand_seed(p, F, seed, U_JOINT_RANDOMNESS, &b, 1, out, p->jr_len * p->num_proofs);
}
static void query_rands(const orc_params* p, const fld* F, const uint8_t* vk,
                        const uint8_t nonce[16], fe* out) {
  uint8_t b[17];
  b[0] = (uint8_t)p->num_proofs;
  memcpy(b + 1, nonce, 16);
  expand_seed(p, F, vk, U_QUERY_RANDOMNESS, b, 17, out, p->qr_len * p->num_proofs);
}

static int encode_measurement(const orc_params* p, const fld* F, const uint64_t* m, fe* out) {
  switch (p->type) {
    case ORC_COUNT:
      if (m[0] > 1) return -1;
      out[0] = m[0];
      return 0;
    case ORC_SUM:
      if (p->bits < 64 && (m[0] >> p->bits)) return -1;
      for (uint32_t i = 0; i < p->bits; i++) out[i] = (m[0] >> i) & 1;
      return 0;
    case ORC_SUMVEC:
      for (uint32_t e = 0; e < p->length; e++) {
        if (p->bits < 64 && (m[e] >> p->bits)) return -1;
        for (uint32_t b = 0; b < p->bits; b++) out[e * p->bits + b] = (m[e] >> b) & 1;
      }
      return 0;
    case ORC_HISTOGRAM:
      if (m[0] >= p->length) return -1;
      for (uint32_t i = 0; i < p->length; i++) out[i] = i == m[0];
      return 0;
  }
  (void)F;
  return -1;
}

static void truncate_share(const orc_params* p, const fld* F, const fe* meas, fe* out) {
  switch (p->type) {
    case ORC_COUNT:
    case ORC_HISTOGRAM:
      memcpy(out, meas, sizeof(fe) * p->meas_len);
      return;
    case ORC_SUM: {
      fe acc = 0, pw = 1;
      for (uint32_t i = 0; i < p->bits; i++) {
        acc = f_add(F, acc, f_mul(F, pw, meas[i]));
        pw = f_add(F, pw, pw);
      }
      out[0] = acc;
      return;
    }
    case ORC_SUMVEC:
    case ORC_SUMVEC_F64_MP:
    case ORC_FPVEC: /* FPVec: the decoded entries (the claimed-norm bits are not output) */
      for (uint32_t e = 0; e < p->length; e++) {
        fe acc = 0, pw = 1;
        for (uint32_t b = 0; b < p->bits; b++) {
          acc = f_add(F, acc, f_mul(F, pw, meas[e * p->bits + b]));
          pw = f_add(F, pw, pw);
        }
        out[e] = acc;
      }
      return;
  }
}

int orc_shard(const orc_params* p, const uint64_t* meas, const uint8_t nonce[16],
              const uint8_t* rand, uint8_t* public_share, uint8_t* leader_share,
              uint8_t* helper_share) {
  if (p->seed_size != 16 || p->type == ORC_FPVEC) return -1; /* client side: TurboSHAKE types */
  fld F = mkfld(p);
  uint32_t np = p->num_proofs;
  fe* enc = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* hm = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* lm = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* proofs = (fe*)malloc(sizeof(fe) * p->proof_len * np);
  fe* hp = (fe*)malloc(sizeof(fe) * p->proof_len * np);
  fe* prove_rand = (fe*)malloc(sizeof(fe) * p->prove_rand_len * np);
  fe jr[64];
  int rc = encode_measurement(p, &F, meas, enc);
  if (rc) goto out;
  const uint8_t* k_hmeas = rand;
  const uint8_t* k_hproof = rand + 16;
  const uint8_t* k_hblind = p->jr_len ? rand + 32 : NULL;
  const uint8_t* k_lblind = p->jr_len ? rand + 48 : NULL;
  const uint8_t* k_prove = p->jr_len ? rand + 64 : rand + 32;
  helper_meas_share(p, &F, k_hmeas, 1, hm);
  for (uint32_t i = 0; i < p->meas_len; i++) lm[i] = f_sub(&F, enc[i], hm[i]);
  if (p->jr_len) {
    uint8_t part0[16], part1[16], seed[16];
    joint_rand_part(p, &F, k_hblind, 1, nonce, hm, part1);
    joint_rand_part(p, &F, k_lblind, 0, nonce, lm, part0);
    memcpy(public_share, part0, 16);
    memcpy(public_share + 16, part1, 16);
    joint_rand_seed(p, part0, part1, seed);
    joint_rands(p, &F, seed, jr);
  }
  {
    uint8_t b = (uint8_t)np;
    expand_seed(p, &F, k_prove, U_PROVE_RANDOMNESS, &b, 1, prove_rand, p->prove_rand_len * np);
  }
  for (uint32_t k = 0; k < np; k++)
    flp_prove(&F, p, enc, prove_rand + k * p->prove_rand_len, jr + k * p->jr_len,
              proofs + k * p->proof_len);
  helper_proofs_share(p, &F, k_hproof, 1, hp);
  for (uint32_t i = 0; i < p->proof_len * np; i++) proofs[i] = f_sub(&F, proofs[i], hp[i]);
  /* leader share: enc(meas) || enc(proofs) || [blind] */
  uint8_t* o = leader_share;
  for (uint32_t i = 0; i < p->meas_len; i++, o += p->es) enc_fe(&F, lm[i], o);
  for (uint32_t i = 0; i < p->proof_len * np; i++, o += p->es) enc_fe(&F, proofs[i], o);
  if (p->jr_len) memcpy(o, k_lblind, 16);
  memcpy(helper_share, k_hmeas, 16);
  memcpy(helper_share + 16, k_hproof, 16);
  if (p->jr_len) memcpy(helper_share + 32, k_hblind, 16);
out:
  free(enc);
  free(hm);
  free(lm);
  free(proofs);
  free(hp);
  free(prove_rand);
  return rc;
}

/* Core of prepare_init; optionally exports intermediates. */
static int prepare_init_core(const orc_params* p, const fld* F, const uint8_t* vk, int agg_id,
                             const uint8_t nonce[16], const uint8_t* public_share,
                             const uint8_t* input_share, fe* meas, fe* proofs, uint8_t* part,
                             uint8_t* corrected, fe* jr, fe* qr, fe* verifiers) {
  const uint32_t S = p->seed_size;
  uint32_t np = p->num_proofs;
  if (agg_id == 0) {
    const uint8_t* in = input_share;
    for (uint32_t i = 0; i < p->meas_len; i++, in += p->es)
      if (dec_fe(F, in, &meas[i])) return ORC_ERR_PREP_INIT;
    for (uint32_t i = 0; i < p->proof_len * np; i++, in += p->es)
      if (dec_fe(F, in, &proofs[i])) return ORC_ERR_PREP_INIT;
  } else {
    helper_meas_share(p, F, input_share, (uint8_t)agg_id, meas);
    helper_proofs_share(p, F, input_share + S, (uint8_t)agg_id, proofs);
  }
  if (p->jr_len) {
    const uint8_t* blind = agg_id == 0
                               ? input_share + (p->meas_len + p->proof_len * np) * p->es
                               : input_share + 2 * S;
    joint_rand_part(p, F, blind, (uint8_t)agg_id, nonce, meas, part);
    if (agg_id == 0)
      joint_rand_seed(p, part, public_share + S, corrected);
    else
      joint_rand_seed(p, public_share, part, corrected);
    joint_rands(p, F, corrected, jr);
  }
  query_rands(p, F, vk, nonce, qr);
  for (uint32_t k = 0; k < np; k++)
    if ((p->type == ORC_FPVEC ? fpvec_query : flp_query)(
            F, p, meas, proofs + k * p->proof_len, qr + k * p->qr_len, jr + k * p->jr_len,
            verifiers + k * p->verifier_len))
      return ORC_ERR_PREP_INIT;
  return ORC_OK;
}

int orc_prepare_init(const orc_params* p, const uint8_t* vk, int agg_id,
                     const uint8_t nonce[16], const uint8_t* public_share,
                     const uint8_t* input_share, uint8_t* state_out, uint8_t* prep_share_out) {
  fld F = mkfld(p);
  uint32_t np = p->num_proofs;
  fe* meas = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* proofs = (fe*)malloc(sizeof(fe) * p->proof_len * np);
  fe* ver = (fe*)malloc(sizeof(fe) * p->verifier_len * np);
  fe jr[64], qr[64];
  uint8_t part[32], corrected[32];
  int rc = prepare_init_core(p, &F, vk, agg_id, nonce, public_share, input_share, meas, proofs,
                             part, corrected, jr, qr, ver);
  if (rc == ORC_OK) {
    uint8_t* o = state_out;
    for (uint32_t i = 0; i < p->meas_len; i++, o += p->es) enc_fe(&F, meas[i], o);
    if (p->jr_len) memcpy(o, corrected, p->seed_size);
    o = prep_share_out;
    for (uint32_t i = 0; i < p->verifier_len * np; i++, o += p->es) enc_fe(&F, ver[i], o);
    if (p->jr_len) memcpy(o, part, p->seed_size);
  }
  free(meas);
  free(proofs);
  free(ver);
  return rc;
}

int orc_helper_trace(const orc_params* p, const uint8_t* vk, const uint8_t nonce[16],
                     const uint8_t* public_share, const uint8_t* helper_share,
                     uint8_t* meas_out, uint8_t* proofs_out, uint8_t* part_out,
                     uint8_t* corrected_out, uint8_t* jr_out, uint8_t* qr_out,
                     uint8_t* verifier_out) {
  fld F = mkfld(p);
  uint32_t np = p->num_proofs;
  fe* meas = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* proofs = (fe*)malloc(sizeof(fe) * p->proof_len * np);
  fe* ver = (fe*)malloc(sizeof(fe) * p->verifier_len * np);
  fe jr[64] = {0}, qr[64] = {0};
  uint8_t part[32] = {0}, corrected[32] = {0};
  int rc = prepare_init_core(p, &F, vk, 1, nonce, public_share, helper_share, meas, proofs, part,
                             corrected, jr, qr, ver);
  for (uint32_t i = 0; i < p->meas_len; i++) enc_fe(&F, meas[i], meas_out + i * p->es);
  for (uint32_t i = 0; i < p->proof_len * np; i++) enc_fe(&F, proofs[i], proofs_out + i * p->es);
  memcpy(part_out, part, p->seed_size);
  memcpy(corrected_out, corrected, p->seed_size);
  for (uint32_t i = 0; i < p->jr_len * np; i++) enc_fe(&F, jr[i], jr_out + i * p->es);
  for (uint32_t i = 0; i < p->qr_len * np; i++) enc_fe(&F, qr[i], qr_out + i * p->es);
  if (rc == ORC_OK)
    for (uint32_t i = 0; i < p->verifier_len * np; i++)
      enc_fe(&F, ver[i], verifier_out + i * p->es);
  free(meas);
  free(proofs);
  free(ver);
  return rc;
}

/* prepare_shares_to_prepare_message: shares = [leader, helper]. */
static int prep_msg_core(const orc_params* p, const fld* F, const uint8_t* lps, const uint8_t* hps,
                         uint8_t* msg) {
  uint32_t nv = p->verifier_len * p->num_proofs;
  fe* v = (fe*)malloc(sizeof(fe) * nv);
  int rc = ORC_OK;
  for (uint32_t i = 0; i < nv; i++) {
    fe a, b;
    if (dec_fe(F, lps + i * p->es, &a) || dec_fe(F, hps + i * p->es, &b)) {
      rc = ORC_ERR_PREP_SHARE_DECODE;
      goto out;
    }
    v[i] = f_add(F, a, b);
  }
  for (uint32_t k = 0; k < p->num_proofs; k++)
    if (!(p->type == ORC_FPVEC ? fpvec_decide : flp_decide)(F, p, v + k * p->verifier_len)) {
      rc = ORC_ERR_DECIDE;
      goto out;
    }
  if (p->jr_len) joint_rand_seed(p, lps + nv * p->es, hps + nv * p->es, msg);
out:
  free(v);
  return rc;
}

int orc_prep_shares_to_prep_msg(const orc_params* p, const uint8_t* leader_prep_share,
                                const uint8_t* helper_prep_share, uint8_t* prep_msg_out) {
  fld F = mkfld(p);
  return prep_msg_core(p, &F, leader_prep_share, helper_prep_share, prep_msg_out);
}

int orc_prepare_next(const orc_params* p, const uint8_t* state, const uint8_t* prep_msg,
                     uint8_t* out_share_out) {
  fld F = mkfld(p);
  if (p->jr_len && memcmp(state + p->meas_len * p->es, prep_msg, p->seed_size) != 0)
    return ORC_ERR_PREP_NEXT;
  fe* meas = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* out = (fe*)malloc(sizeof(fe) * p->out_len);
  for (uint32_t i = 0; i < p->meas_len; i++) dec_fe(&F, state + i * p->es, &meas[i]);
  truncate_share(p, &F, meas, out);
  for (uint32_t i = 0; i < p->out_len; i++) enc_fe(&F, out[i], out_share_out + i * p->es);
  free(meas);
  free(out);
  return ORC_OK;
}

void orc_agg_merge(const orc_params* p, uint8_t* acc, const uint8_t* other) {
  fld F = mkfld(p);
  for (uint32_t i = 0; i < p->out_len; i++) {
    fe a = 0, b = 0;
    dec_fe(&F, acc + i * p->es, &a);
    dec_fe(&F, other + i * p->es, &b);
    enc_fe(&F, f_add(&F, a, b), acc + i * p->es);
  }
}

/* ------------------------------------------------------------------------------------ */
/* Batched helper path with Janus's job structure (CPU baseline + batch oracle).         */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  const orc_params* p;
  const uint8_t* vk;
  uint32_t n;
  const uint8_t *nonces, *publics, *helpers, *leader_ps;
  const uint32_t* seg;
  const uint8_t* accept;
  uint32_t n_segments;
  uint8_t* msgs;
  uint8_t* status;
  int job_size;
  atomic_uint next_job;
  pthread_mutex_t mu;
  fe* agg;          /* n_segments x out_len */
  uint64_t* count;
} batch_ctx;

static void* batch_worker(void* arg) {
  batch_ctx* c = (batch_ctx*)arg;
  const orc_params* p = c->p;
  fld F = mkfld(p);
  uint32_t np = p->num_proofs;
  fe* meas = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* proofs = (fe*)malloc(sizeof(fe) * p->proof_len * np);
  fe* ver = (fe*)malloc(sizeof(fe) * p->verifier_len * np);
  fe* out = (fe*)malloc(sizeof(fe) * p->out_len);
  uint8_t* hps = (uint8_t*)malloc(p->prep_share_len);
  fe* lagg = (fe*)calloc((size_t)c->n_segments * p->out_len, sizeof(fe));
  uint64_t* lcnt = (uint64_t*)calloc(c->n_segments, sizeof(uint64_t));
  fe jr[64], qr[64];
  uint8_t part[32], corrected[32], msg[32];
  const uint32_t S = p->seed_size;
  for (;;) {
    uint32_t job = atomic_fetch_add(&c->next_job, 1);
    uint64_t lo = (uint64_t)job * c->job_size;
    if (lo >= c->n) break;
    uint64_t hi = lo + c->job_size;
    if (hi > c->n) hi = c->n;
    for (uint64_t i = lo; i < hi; i++) {
      const uint8_t* pub = c->publics ? c->publics + i * p->public_share_len : NULL;
      int rc = prepare_init_core(p, &F, c->vk, 1, c->nonces + i * 16, pub,
                                 c->helpers + i * p->helper_share_len, meas, proofs, part,
                                 corrected, jr, qr, ver);
      if (rc == ORC_OK) {
        uint8_t* o = hps;
        for (uint32_t k = 0; k < p->verifier_len * np; k++, o += p->es) enc_fe(&F, ver[k], o);
        if (p->jr_len) memcpy(o, part, S);
        rc = prep_msg_core(p, &F, c->leader_ps + i * p->prep_share_len, hps, msg);
      }
      if (rc == ORC_OK && p->jr_len && memcmp(corrected, msg, S) != 0) rc = ORC_ERR_PREP_NEXT;
      c->status[i] = (uint8_t)rc;
      if (p->prep_msg_len) {
        if (rc == ORC_OK)
          memcpy(c->msgs + i * S, msg, S);
        else
          memset(c->msgs + i * S, 0, S);
      }
      if (rc != ORC_OK || (c->accept && !c->accept[i])) continue;
      /* prepare_next re-derives the helper measurement share from its seed [prio]. */
      helper_meas_share(p, &F, c->helpers + i * p->helper_share_len, 1, meas);
      truncate_share(p, &F, meas, out);
      uint32_t s = c->seg ? c->seg[i] : 0;
      if (s >= c->n_segments) continue;
      fe* a = lagg + (size_t)s * p->out_len;
      for (uint32_t k = 0; k < p->out_len; k++) a[k] = f_add(&F, a[k], out[k]);
      lcnt[s]++;
    }
  }
  pthread_mutex_lock(&c->mu);
  for (size_t k = 0; k < (size_t)c->n_segments * p->out_len; k++)
    c->agg[k] = f_add(&F, c->agg[k], lagg[k]);
  for (uint32_t s = 0; s < c->n_segments; s++) c->count[s] += lcnt[s];
  pthread_mutex_unlock(&c->mu);
  free(meas);
  free(proofs);
  free(ver);
  free(out);
  free(hps);
  free(lagg);
  free(lcnt);
  return NULL;
}

/* The per-report buffers of the long instances (FPVec: a 2.56 MB measurement share and its
 * encoding) come from the heap arenas and are reused, not mmap'ed and unmapped per report: with
 * several worker threads each munmap's TLB shootdown stalls every thread (8 threads ran 4.4x
 * slower per report than one). */
static pthread_once_t malloc_once = PTHREAD_ONCE_INIT;
static void malloc_setup(void) {
  mallopt(M_MMAP_THRESHOLD, 256 << 20);
  mallopt(M_TRIM_THRESHOLD, 1 << 30);
}

int orc_helper_batch(const orc_params* p, const uint8_t* vk, uint32_t n,
                     const uint8_t* nonces, const uint8_t* public_shares,
                     const uint8_t* helper_shares, const uint8_t* leader_prep_shares,
                     const uint32_t* segment_ids, const uint8_t* accept_mask,
                     uint32_t n_segments, uint8_t* prep_msgs_out, uint8_t* status_out,
                     uint8_t* agg_out, uint64_t* count_out, int n_threads, int job_size) {
  pthread_once(&malloc_once, malloc_setup);
  if (n_threads < 1) n_threads = 1;
  if (job_size < 1) job_size = 500;
  if (n_segments < 1) n_segments = 1;
  batch_ctx c;
  c.p = p;
  c.vk = vk;
  c.n = n;
  c.nonces = nonces;
  c.publics = public_shares;
  c.helpers = helper_shares;
  c.leader_ps = leader_prep_shares;
  c.seg = segment_ids;
  c.accept = accept_mask;
  c.n_segments = n_segments;
  c.msgs = prep_msgs_out;
  c.status = status_out;
  c.job_size = job_size;
  atomic_init(&c.next_job, 0);
  pthread_mutex_init(&c.mu, NULL);
  c.agg = (fe*)calloc((size_t)n_segments * p->out_len, sizeof(fe));
  c.count = count_out;
  memset(count_out, 0, sizeof(uint64_t) * n_segments);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
  for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, batch_worker, &c);
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  fld F = mkfld(p);
  for (size_t k = 0; k < (size_t)n_segments * p->out_len; k++)
    enc_fe(&F, c.agg[k], agg_out + k * p->es);
  free(th);
  free(c.agg);
  pthread_mutex_destroy(&c.mu);
  return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Batched leader path (CPU baseline of bench.py --role leader): per report prepare_init   */
/* with agg_id 0 on the explicit share (aggregation_job_driver.rs:397-415), prepare_next   */
/* on the helper's prepare message (:700-760: corrected-seed check), then the output share */
/* merged per segment, in jobs of job_size on n_threads workers.                          */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  const orc_params* p;
  const uint8_t* vk;
  uint32_t n;
  const uint8_t *nonces, *publics, *leaders, *msgs;
  uint8_t *prep_out, *status;
  const uint32_t* seg;  /* segment of each report (NULL: all segment 0) */
  uint32_t n_segments;
  int job_size;
  atomic_uint next_job;
  pthread_mutex_t mu;
  fe* agg;          /* [n_segments][out_len] */
  uint64_t* count;  /* [n_segments] */
} leader_ctx;

/* adds a worker's partial of segment s into the batch's (under the mutex) and clears it */
static void leader_flush(leader_ctx* c, const fld* F, uint32_t s, fe* lagg, uint64_t* lcnt) {
  const orc_params* p = c->p;
  if (*lcnt == 0) return;
  pthread_mutex_lock(&c->mu);
  for (uint32_t k = 0; k < p->out_len; k++) {
    fe* g = c->agg + (size_t)s * p->out_len + k;
    *g = f_add(F, *g, lagg[k]);
    lagg[k] = 0;
  }
  c->count[s] += *lcnt;
  pthread_mutex_unlock(&c->mu);
  *lcnt = 0;
}

static void* leader_worker(void* arg) {
  leader_ctx* c = (leader_ctx*)arg;
  const orc_params* p = c->p;
  fld F = mkfld(p);
  const uint32_t np = p->num_proofs, S = p->seed_size;
  fe* meas = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* proofs = (fe*)malloc(sizeof(fe) * p->proof_len * np);
  fe* ver = (fe*)malloc(sizeof(fe) * p->verifier_len * np);
  fe* out = (fe*)malloc(sizeof(fe) * p->out_len);
  fe* lagg = (fe*)calloc(p->out_len, sizeof(fe));
  uint64_t lcnt = 0;
  uint32_t lseg = 0;  /* the segment lagg / lcnt belong to */
  fe jr[64], qr[64];
  uint8_t part[32], corrected[32];
  for (;;) {
    uint32_t job = atomic_fetch_add(&c->next_job, 1);
    uint64_t lo = (uint64_t)job * c->job_size;
    if (lo >= c->n) break;
    uint64_t hi = lo + c->job_size;
    if (hi > c->n) hi = c->n;
    for (uint64_t i = lo; i < hi; i++) {
      const uint32_t sg = c->seg ? c->seg[i] : 0;
      const uint8_t* pub = c->publics ? c->publics + i * p->public_share_len : NULL;
      uint8_t* o = c->prep_out + i * p->prep_share_len;
      int rc = prepare_init_core(p, &F, c->vk, 0, c->nonces + i * 16, pub,
                                 c->leaders + i * p->leader_share_len, meas, proofs, part,
                                 corrected, jr, qr, ver);
      if (rc == ORC_OK) {
        for (uint32_t k = 0; k < p->verifier_len * np; k++, o += p->es) enc_fe(&F, ver[k], o);
        if (p->jr_len) memcpy(o, part, S);
        if (p->jr_len && c->msgs && memcmp(corrected, c->msgs + i * S, S) != 0)
          rc = ORC_ERR_PREP_NEXT;
      } else {
        memset(o, 0, p->prep_share_len);
      }
      c->status[i] = (uint8_t)rc;
      if (rc != ORC_OK || sg >= c->n_segments) continue;
      if (sg != lseg) {
        leader_flush(c, &F, lseg, lagg, &lcnt);
        lseg = sg;
      }
      truncate_share(p, &F, meas, out);
      for (uint32_t k = 0; k < p->out_len; k++) lagg[k] = f_add(&F, lagg[k], out[k]);
      lcnt++;
    }
  }
  leader_flush(c, &F, lseg, lagg, &lcnt);
  free(meas);
  free(proofs);
  free(ver);
  free(out);
  free(lagg);
  return NULL;
}

int orc_leader_batch(const orc_params* p, const uint8_t* vk, uint32_t n, const uint8_t* nonces,
                     const uint8_t* public_shares, const uint8_t* leader_shares,
                     const uint8_t* prep_msgs, uint8_t* prep_shares_out, uint8_t* status_out,
                     uint8_t* agg_out, uint64_t* count_out, int n_threads, int job_size) {
  return orc_leader_batch_seg(p, vk, n, nonces, public_shares, leader_shares, prep_msgs, NULL, 1,
                              prep_shares_out, status_out, agg_out, count_out, n_threads,
                              job_size);
}

int orc_leader_batch_seg(const orc_params* p, const uint8_t* vk, uint32_t n,
                         const uint8_t* nonces, const uint8_t* public_shares,
                         const uint8_t* leader_shares, const uint8_t* prep_msgs,
                         const uint32_t* segment_ids, uint32_t n_segments,
                         uint8_t* prep_shares_out, uint8_t* status_out, uint8_t* agg_out,
                         uint64_t* count_out, int n_threads, int job_size) {
  if (n_threads < 1) n_threads = 1;
  if (job_size < 1) job_size = 500;
  if (n_segments < 1) n_segments = 1;
  leader_ctx c;
  c.seg = segment_ids;
  c.n_segments = n_segments;
  c.p = p;
  c.vk = vk;
  c.n = n;
  c.nonces = nonces;
  c.publics = public_shares;
  c.leaders = leader_shares;
  c.msgs = prep_msgs;
  c.prep_out = prep_shares_out;
  c.status = status_out;
  c.job_size = job_size;
  atomic_init(&c.next_job, 0);
  pthread_mutex_init(&c.mu, NULL);
  c.agg = (fe*)calloc((size_t)n_segments * p->out_len, sizeof(fe));
  c.count = count_out;
  memset(count_out, 0, 8 * (size_t)n_segments);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
  for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, leader_worker, &c);
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  fld F = mkfld(p);
  for (size_t k = 0; k < (size_t)n_segments * p->out_len; k++)
    enc_fe(&F, c.agg[k], agg_out + k * p->es);
  free(th);
  free(c.agg);
  pthread_mutex_destroy(&c.mu);
  return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Deterministic synthetic report generator (client shard + leader prepare_init), for   */
/* tests only.  Per report i: stream = TurboSHAKE128("janus-amd-gen" || seed || i, D=1).  */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  const orc_params* p;
  const uint8_t* vk;
  uint32_t n;
  uint64_t seed;
  uint8_t *nonces, *publics, *helpers, *leader_ps, *leader_out;
  uint64_t* meas;
  atomic_uint next;
} gen_ctx;

static void* gen_worker(void* arg) {
  gen_ctx* g = (gen_ctx*)arg;
  const orc_params* p = g->p;
  fld F = mkfld(p);
  uint32_t mstride = p->type == ORC_SUMVEC ? p->length : 1;
  uint8_t* ls = (uint8_t*)malloc(p->leader_share_len);
  uint8_t* st = (uint8_t*)malloc(p->meas_len * p->es + 16);
  uint8_t* ps = (uint8_t*)malloc(p->prep_share_len);
  uint64_t* m = (uint64_t*)malloc(sizeof(uint64_t) * mstride);
  fe* lm = (fe*)malloc(sizeof(fe) * p->meas_len);
  fe* lo = (fe*)malloc(sizeof(fe) * p->out_len);
  size_t slen = 16 + 80 + 8 * (size_t)mstride;
  uint8_t* stream = (uint8_t*)malloc(slen);
  uint8_t pub[32];
  for (;;) {
    uint32_t i = atomic_fetch_add(&g->next, 1);
    if (i >= g->n) break;
    uint8_t in[29];
    memcpy(in, "janus-amd-gen", 13);
    for (int k = 0; k < 8; k++) in[13 + k] = (uint8_t)(g->seed >> (8 * k));
    for (int k = 0; k < 8; k++) in[21 + k] = (uint8_t)((uint64_t)i >> (8 * k));
    orc_turboshake128(in, sizeof in, 0x01, stream, slen);
    for (uint32_t e = 0; e < mstride; e++) {
      uint64_t v = 0;
      for (int k = 0; k < 8; k++) v |= (uint64_t)stream[96 + 8 * e + k] << (8 * k);
      switch (p->type) {
        case ORC_COUNT: v &= 1; break;
        case ORC_SUM:
        case ORC_SUMVEC: if (p->bits < 64) v &= ((uint64_t)1 << p->bits) - 1; break;
        case ORC_HISTOGRAM: v %= p->length; break;
      }
      m[e] = v;
    }
    const uint8_t* nonce = stream;
    orc_shard(p, m, nonce, stream + 16, pub, ls, g->helpers + (size_t)i * p->helper_share_len);
    orc_prepare_init(p, g->vk, 0, nonce, pub, ls, st, ps);
    memcpy(g->nonces + (size_t)i * 16, nonce, 16);
    if (p->public_share_len) memcpy(g->publics + (size_t)i * p->public_share_len, pub, 32);
    memcpy(g->leader_ps + (size_t)i * p->prep_share_len, ps, p->prep_share_len);
    if (g->meas) memcpy(g->meas + (size_t)i * mstride, m, sizeof(uint64_t) * mstride);
    if (g->leader_out) {
      for (uint32_t k = 0; k < p->meas_len; k++) dec_fe(&F, st + k * p->es, &lm[k]);
      truncate_share(p, &F, lm, lo);
      for (uint32_t k = 0; k < p->out_len; k++)
        enc_fe(&F, lo[k], g->leader_out + ((size_t)i * p->out_len + k) * p->es);
    }
  }
  free(ls);
  free(st);
  free(ps);
  free(m);
  free(lm);
  free(lo);
  free(stream);
  return NULL;
}

int orc_gen_reports(const orc_params* p, const uint8_t vk[16], uint32_t n, uint64_t seed,
                    int n_threads, uint8_t* nonces, uint8_t* publics, uint8_t* helpers,
                    uint8_t* leader_ps, uint64_t* meas_out, uint8_t* leader_out_shares) {
  if (p->type == ORC_FPVEC || p->seed_size != 16) return -1;  /* helper side only */
  gen_ctx g;
  g.p = p;
  g.vk = vk;
  g.n = n;
  g.seed = seed;
  g.nonces = nonces;
  g.publics = publics;
  g.helpers = helpers;
  g.leader_ps = leader_ps;
  g.leader_out = leader_out_shares;
  g.meas = meas_out;
  atomic_init(&g.next, 0);
  if (n_threads < 1) n_threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
  for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, gen_worker, &g);
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  free(th);
  return 0;
}

/* Single-core cost of the two primitives the CPU baseline's per-report time is made of (bench.py
 * reports the op-count estimate beside the measured time): one Keccak-p[1600, 12] permutation
 * and one Field128 multiply, in ns. */
void orc_prim_bench(double* ns_perm, double* ns_mul) {
  struct timespec a, b;
  uint64_t st[25] = {1, 2, 3};
  const int NP = 200000, NM = 4000000;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int i = 0; i < NP; i++) orc_keccak_p1600(st, 12);
  clock_gettime(CLOCK_MONOTONIC, &b);
  *ns_perm = ((b.tv_sec - a.tv_sec) * 1e9 + (b.tv_nsec - a.tv_nsec)) / NP;
  volatile u128 sink;
  u128 x = ((u128)st[0] << 64 | st[1]) % P128, y = ((u128)st[2] << 64 | st[3]) % P128;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int i = 0; i < NM; i++) x = f128_mul(x, y);  /* a dependent chain, like Horner / MACs */
  clock_gettime(CLOCK_MONOTONIC, &b);
  sink = x;
  (void)sink;
  *ns_mul = ((b.tv_sec - a.tv_sec) * 1e9 + (b.tv_nsec - a.tv_nsec)) / NM;
}
