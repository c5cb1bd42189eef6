/*
 * hpke_oracle.c -- CPU restatement of the helper's input-share decryption.
 * TEST INFRASTRUCTURE ONLY: the checker for tests/ and bench.py's cpu_baseline leg.
 *
 * HPKE base mode (RFC 9180 §5.1, §5.2) with DHKEM(X25519, HKDF-SHA256) (§4.1, §7.1),
 * HKDF-SHA256 and AES-128-GCM -- the suite Janus generates by default -- or any other suite of
 * KEM {X25519, P-256, X448, P-521, P-384} x KDF {HKDF-SHA256, -SHA384, -SHA512} x AEAD {AES-128-GCM,
 * AES-256-GCM, ChaCha20Poly1305} (pinned by the 24 RFC 9180 base-mode vectors of
 * core/src/test-vectors.json; the HKDF-SHA384 suites have none there and rest on OpenSSL)
 * (/root/reference/core/src/hpke.rs:260-280, generate_test_hpke_config_and_private_key), whose
 * Rust implementation (hpke-dispatch -> hpke crate) is not in /root/reference.  The RFC 9180
 * composition (labels, suite ids, key schedule) is restated here over OpenSSL 3.0 primitives
 * (X25519, HMAC-SHA256, AES-128-GCM); it is pinned by the RFC 9180 test vector that Janus's
 * own test reads (core/src/test-vectors.json, mode 0 / kem 0x20 / kdf 1 / aead 1,
 * hpke.rs:480-560).
 *
 * The Janus layer around hpke::open follows aggregator.rs:1796-1990: application info
 * "dap-09 input share" || Role::Client || Role::Helper (hpke.rs:55-85), AAD = InputShareAad
 * { task_id, ReportMetadata { report_id, time }, public_share } (messages/src/lib.rs:1825-1872),
 * then PlaintextInputShare::get_decoded (lib.rs:1301-1350), the duplicate-extension and
 * taskprov-extension checks, and the exact-length helper input share decode.
 */
#define OPENSSL_SUPPRESS_DEPRECATED
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdh.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/obj_mac.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { HPKE_OK = 0, HPKE_DECRYPT_ERROR = 4, HPKE_INVALID_MESSAGE = 8 };

/* KEMs (RFC 9180 7.1): 0x0020 DHKEM(X25519, HKDF-SHA256), 0x0010 DHKEM(P-256, HKDF-SHA256),
 * 0x0021 DHKEM(X448, HKDF-SHA512), 0x0012 DHKEM(P-521, HKDF-SHA512), 0x0011 DHKEM(P-384,
 * HKDF-SHA384) (messages/src/lib.rs:770-784; P-384 has no RFC 9180 vector: OpenSSL is its pin);
 * Nsk, Nenc (= Npk, the NIST curves' uncompressed points), Ndh, and the KEM's own KDF. */
typedef struct {
  uint16_t id;
  size_t nsk, nenc, ndh;
  int kdf; /* 1 HKDF-SHA256, 2 HKDF-SHA384, 3 HKDF-SHA512 */
} Kem;
static const Kem KEMS[] = {{0x20, 32, 32, 32, 1}, {0x10, 32, 65, 32, 1},
                           {0x21, 56, 56, 56, 3}, {0x12, 66, 133, 66, 3},
                           {0x11, 48, 97, 48, 2}};
static const Kem* kem_of(uint16_t kem) {
  for (size_t i = 0; i < sizeof(KEMS) / sizeof(KEMS[0]); i++)
    if (KEMS[i].id == kem) return &KEMS[i];
  return NULL;
}
static size_t kem_nenc(uint16_t kem) { return kem_of(kem) ? kem_of(kem)->nenc : 0; }
/* KDFs (RFC 9180 7.2, lib.rs:809-815): 1 HKDF-SHA256, 2 HKDF-SHA384, 3 HKDF-SHA512 */
static const EVP_MD* kdf_md(int kdf) {
  return kdf == 1 ? EVP_sha256() : kdf == 2 ? EVP_sha384() : kdf == 3 ? EVP_sha512() : NULL;
}
static size_t kdf_nh(int kdf) { return kdf == 1 ? 32 : kdf == 2 ? 48 : 64; }

static void kem_suite(uint16_t kem, uint8_t s[5]) {
  s[0] = 'K', s[1] = 'E', s[2] = 'M', s[3] = (uint8_t)(kem >> 8), s[4] = (uint8_t)kem;
}
/* suite_id = "HPKE" || kem || kdf || aead (RFC 9180 5.1); aead 1 AES-128-GCM, 2 AES-256-GCM,
 * 3 ChaCha20Poly1305 (messages/src/lib.rs:844-853) */
static void hpke_suite(uint16_t kem, uint16_t kdf, uint16_t aead, uint8_t s[10]) {
  s[0] = 'H', s[1] = 'P', s[2] = 'K', s[3] = 'E';
  s[4] = (uint8_t)(kem >> 8), s[5] = (uint8_t)kem, s[6] = (uint8_t)(kdf >> 8), s[7] = (uint8_t)kdf;
  s[8] = (uint8_t)(aead >> 8);
  s[9] = (uint8_t)aead;
}
static size_t aead_nk(uint16_t aead) { return aead == 1 ? 16 : 32; }

static void hmac_md(int kdf, const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen,
                    uint8_t* out) {
  unsigned int ol = 64;
  static const uint8_t zero = 0;
  HMAC(kdf_md(kdf), klen ? key : &zero, (int)klen, msg, mlen, out, &ol);
}

/* LabeledExtract(salt, label, ikm) = HKDF-Extract(salt, "HPKE-v1" || suite_id || label || ikm) */
static void labeled_extract(int kdf, const uint8_t* suite, size_t slen, const uint8_t* salt,
                            size_t saltlen, const char* label, const uint8_t* ikm, size_t ikmlen,
                            uint8_t* out) {
  uint8_t buf[512];
  size_t l = 0, ll = strlen(label);
  memcpy(buf + l, "HPKE-v1", 7), l += 7;
  memcpy(buf + l, suite, slen), l += slen;
  memcpy(buf + l, label, ll), l += ll;
  memcpy(buf + l, ikm, ikmlen), l += ikmlen;
  hmac_md(kdf, salt, saltlen, buf, l, out);
}

/* LabeledExpand(prk, label, info, L <= Nh) = HKDF-Expand(prk, I2OSP(L, 2) || "HPKE-v1" ||
 * suite_id || label || info, L): one HMAC block T(1) = HMAC(prk, labeled_info || 0x01) */
static void labeled_expand(int kdf, const uint8_t* suite, size_t slen, const uint8_t* prk,
                           const char* label, const uint8_t* info, size_t infolen, size_t L,
                           uint8_t* out) {
  uint8_t buf[512], t[64];
  size_t l = 0, ll = strlen(label);
  buf[l++] = (uint8_t)(L >> 8);
  buf[l++] = (uint8_t)L;
  memcpy(buf + l, "HPKE-v1", 7), l += 7;
  memcpy(buf + l, suite, slen), l += slen;
  memcpy(buf + l, label, ll), l += ll;
  memcpy(buf + l, info, infolen), l += infolen;
  buf[l++] = 0x01;
  hmac_md(kdf, prk, kdf_nh(kdf), buf, l, t);
  memcpy(out, t, L);
}

/* X25519 / X448 (RFC 7748) through OpenSSL's raw keys */
static int xdh(int type, size_t len, const uint8_t* sk, const uint8_t* pk, uint8_t* out) {
  EVP_PKEY* k = EVP_PKEY_new_raw_private_key(type, NULL, sk, len);
  EVP_PKEY* p = EVP_PKEY_new_raw_public_key(type, NULL, pk, len);
  EVP_PKEY_CTX* c = k ? EVP_PKEY_CTX_new(k, NULL) : NULL;
  size_t ol = len;
  int ok = c && p && EVP_PKEY_derive_init(c) == 1 && EVP_PKEY_derive_set_peer(c, p) == 1 &&
           EVP_PKEY_derive(c, out, &ol) == 1 && ol == len;
  EVP_PKEY_CTX_free(c);
  EVP_PKEY_free(k);
  EVP_PKEY_free(p);
  return ok ? 0 : -1;
}
static int xdh_public(int type, size_t len, const uint8_t* sk, uint8_t* pk) {
  EVP_PKEY* k = EVP_PKEY_new_raw_private_key(type, NULL, sk, len);
  size_t ol = len;
  int ok = k && EVP_PKEY_get_raw_public_key(k, pk, &ol) == 1 && ol == len;
  EVP_PKEY_free(k);
  return ok ? 0 : -1;
}

/* NIST-curve ECDH (SEC 1): the x-coordinate of sk * pk, pk an uncompressed point (validated) */
static int ec_dh(int nid, size_t n, const uint8_t* sk, const uint8_t* pk, uint8_t* out) {
  EC_KEY* k = EC_KEY_new_by_curve_name(nid);
  const EC_GROUP* g = k ? EC_KEY_get0_group(k) : NULL;
  BIGNUM* d = BN_bin2bn(sk, (int)n, NULL);
  EC_POINT* q = g ? EC_POINT_new(g) : NULL;
  int ok = k && d && q && EC_KEY_set_private_key(k, d) == 1 &&
           EC_POINT_oct2point(g, q, pk, 2 * n + 1, NULL) == 1 &&
           EC_POINT_is_on_curve(g, q, NULL) == 1 && ECDH_compute_key(out, n, q, k, NULL) == (int)n;
  EC_POINT_free(q);
  BN_free(d);
  EC_KEY_free(k);
  return ok ? 0 : -1;
}
static int ec_public(int nid, size_t n, const uint8_t* sk, uint8_t* pk) {
  EC_KEY* k = EC_KEY_new_by_curve_name(nid);
  const EC_GROUP* g = k ? EC_KEY_get0_group(k) : NULL;
  BIGNUM* d = BN_bin2bn(sk, (int)n, NULL);
  EC_POINT* q = g ? EC_POINT_new(g) : NULL;
  int ok = k && d && q && EC_POINT_mul(g, q, d, NULL, NULL, NULL) == 1 &&
           EC_POINT_point2oct(g, q, POINT_CONVERSION_UNCOMPRESSED, pk, 2 * n + 1, NULL) == 2 * n + 1;
  EC_POINT_free(q);
  BN_free(d);
  EC_KEY_free(k);
  return ok ? 0 : -1;
}

static int kem_dh(uint16_t kem, const uint8_t* sk, const uint8_t* pk, uint8_t* out) {
  switch (kem) {
    case 0x20: return xdh(EVP_PKEY_X25519, 32, sk, pk, out);
    case 0x21: return xdh(EVP_PKEY_X448, 56, sk, pk, out);
    case 0x10: return ec_dh(NID_X9_62_prime256v1, 32, sk, pk, out);
    case 0x12: return ec_dh(NID_secp521r1, 66, sk, pk, out);
    case 0x11: return ec_dh(NID_secp384r1, 48, sk, pk, out);
  }
  return -1;
}
/* SerializePublicKey(DerivePublicKey(sk)) for any of the KEMs */
int hpke_kem_public(uint16_t kem, const uint8_t* sk, uint8_t* pk) {
  switch (kem) {
    case 0x20: return xdh_public(EVP_PKEY_X25519, 32, sk, pk);
    case 0x21: return xdh_public(EVP_PKEY_X448, 56, sk, pk);
    case 0x10: return ec_public(NID_X9_62_prime256v1, 32, sk, pk);
    case 0x12: return ec_public(NID_secp521r1, 66, sk, pk);
    case 0x11: return ec_public(NID_secp384r1, 48, sk, pk);
  }
  return -1;
}
int hpke_p256_public(const uint8_t sk[32], uint8_t pk[65]) { return hpke_kem_public(0x10, sk, pk); }
int hpke_x25519_public(const uint8_t sk[32], uint8_t pk[32]) { return hpke_kem_public(0x20, sk, pk); }

/* KeySchedule(mode_base, shared_secret, info) -> key (Nk), base_nonce (12)  [RFC 9180 §5.1] */
static void key_schedule(uint16_t kem, int kdf, uint16_t aead, const uint8_t* ss, size_t nss,
                         const uint8_t* info, size_t infolen, uint8_t key[32], uint8_t nonce[12]) {
  uint8_t ksc[129], secret[64], su[10];
  const size_t nh = kdf_nh(kdf);
  hpke_suite(kem, (uint16_t)kdf, aead, su);
  ksc[0] = 0x00; /* mode_base */
  labeled_extract(kdf, su, 10, NULL, 0, "psk_id_hash", NULL, 0, ksc + 1);
  labeled_extract(kdf, su, 10, NULL, 0, "info_hash", info, infolen, ksc + 1 + nh);
  labeled_extract(kdf, su, 10, ss, nss, "secret", NULL, 0, secret);
  labeled_expand(kdf, su, 10, secret, "key", ksc, 1 + 2 * nh, aead_nk(aead), key);
  labeled_expand(kdf, su, 10, secret, "base_nonce", ksc, 1 + 2 * nh, 12, nonce);
}

/* ExtractAndExpand(dh, enc || pkRm) with the KEM's KDF -> shared_secret (Nsecret = its Nh) */
static void extract_and_expand(const Kem* K, const uint8_t* dh, const uint8_t* enc,
                               const uint8_t* pkR, uint8_t* ss) {
  uint8_t prk[64], kc[266], ks[5];
  kem_suite(K->id, ks);
  labeled_extract(K->kdf, ks, 5, NULL, 0, "eae_prk", dh, K->ndh, prk);
  memcpy(kc, enc, K->nenc);
  memcpy(kc + K->nenc, pkR, K->nenc);
  labeled_expand(K->kdf, ks, 5, prk, "shared_secret", kc, 2 * K->nenc, kdf_nh(K->kdf), ss);
}

/* Decap (§4.1): dh = DH(skR, enc); shared_secret = ExtractAndExpand(dh, enc || pkRm) */
static int decap(const Kem* K, const uint8_t* enc, const uint8_t* skR, const uint8_t* pkR,
                 uint8_t* ss) {
  uint8_t dh[66];
  static const uint8_t zero[66];
  if (kem_dh(K->id, skR, enc, dh)) return -1;
  /* X25519 / X448 all-zero output: ValidationError */
  if ((K->id == 0x20 || K->id == 0x21) && !memcmp(dh, zero, K->ndh)) return -1;
  extract_and_expand(K, dh, enc, pkR, ss);
  return 0;
}

/* the AEAD of the suite through OpenSSL's EVP AEAD interface (16-byte tag, 12-byte nonce) */
static int aead_crypt(uint16_t aead, int decrypt, const uint8_t* key, const uint8_t nonce[12],
                      const uint8_t* aad, size_t aadlen, const uint8_t* in, size_t inlen,
                      uint8_t* out, uint8_t tag[16]) {
  const EVP_CIPHER* ci = aead == 1   ? EVP_aes_128_gcm()
                         : aead == 2 ? EVP_aes_256_gcm()
                         : aead == 3 ? EVP_chacha20_poly1305()
                                     : NULL;
  if (!ci) return -1;
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  int l = 0;
  int ok = c && EVP_CipherInit_ex(c, ci, NULL, NULL, NULL, !decrypt) == 1 &&
                  EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL) == 1 &&
                  EVP_CipherInit_ex(c, NULL, NULL, key, nonce, !decrypt) == 1;
  if (ok && aadlen) ok = EVP_CipherUpdate(c, NULL, &l, aad, (int)aadlen) == 1;
  l = 0;
  if (ok && inlen) ok = EVP_CipherUpdate(c, out, &l, in, (int)inlen) == 1;
  if (ok && decrypt) ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, tag) == 1;
  int fl = 0;
  if (ok) ok = EVP_CipherFinal_ex(c, out + l, &fl) == 1;
  if (ok && !decrypt) ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1;
  EVP_CIPHER_CTX_free(c);
  return ok ? 0 : -1;
}

/* base-mode single-shot open (sequence number 0) of any suite; the plaintext length or -1 */
int hpke_open_suite(uint16_t kem, uint16_t kdf, uint16_t aead, const uint8_t* skR,
                    const uint8_t* pkR, const uint8_t* enc, const uint8_t* info, size_t infolen,
                    const uint8_t* aad, size_t aadlen, const uint8_t* ct, size_t ctlen,
                    uint8_t* pt) {
  uint8_t ss[64], key[32], nonce[12], tag[16];
  const Kem* K = kem_of(kem);
  if (!K || !kdf_md(kdf) || ctlen < 16 || decap(K, enc, skR, pkR, ss)) return -1;
  key_schedule(kem, kdf, aead, ss, kdf_nh(K->kdf), info, infolen, key, nonce);
  memcpy(tag, ct + ctlen - 16, 16);
  if (aead_crypt(aead, 1, key, nonce, aad, aadlen, ct, ctlen - 16, pt, tag)) return -1;
  return (int)(ctlen - 16);
}
int hpke_open_kem(uint16_t kem, uint16_t aead, const uint8_t skR[32], const uint8_t* pkR,
                  const uint8_t* enc, const uint8_t* info, size_t infolen, const uint8_t* aad,
                  size_t aadlen, const uint8_t* ct, size_t ctlen, uint8_t* pt) {
  return hpke_open_suite(kem, 1, aead, skR, pkR, enc, info, infolen, aad, aadlen, ct, ctlen, pt);
}
int hpke_open_ex(uint16_t aead, const uint8_t skR[32], const uint8_t pkR[32],
                 const uint8_t enc[32], const uint8_t* info, size_t infolen, const uint8_t* aad,
                 size_t aadlen, const uint8_t* ct, size_t ctlen, uint8_t* pt) {
  return hpke_open_kem(0x20, aead, skR, pkR, enc, info, infolen, aad, aadlen, ct, ctlen, pt);
}
int hpke_open(const uint8_t skR[32], const uint8_t pkR[32], const uint8_t enc[32],
              const uint8_t* info, size_t infolen, const uint8_t* aad, size_t aadlen,
              const uint8_t* ct, size_t ctlen, uint8_t* pt) {
  return hpke_open_ex(1, skR, pkR, enc, info, infolen, aad, aadlen, ct, ctlen, pt);
}

/* base-mode seal with the ephemeral key skE (Encap with a given ephemeral key, as the RFC 9180
 * test vectors do); writes enc[Nenc] and ct[ptlen + 16] */
int hpke_seal_suite(uint16_t kem, uint16_t kdf, uint16_t aead, const uint8_t* pkR,
                    const uint8_t* skE, const uint8_t* info, size_t infolen, const uint8_t* aad,
                    size_t aadlen, const uint8_t* pt, size_t ptlen, uint8_t* enc, uint8_t* ct) {
  uint8_t dh[66], ss[64], key[32], nonce[12];
  const Kem* K = kem_of(kem);
  if (!K || !kdf_md(kdf) || hpke_kem_public(kem, skE, enc) || kem_dh(kem, skE, pkR, dh)) return -1;
  extract_and_expand(K, dh, enc, pkR, ss);
  key_schedule(kem, kdf, aead, ss, kdf_nh(K->kdf), info, infolen, key, nonce);
  return aead_crypt(aead, 0, key, nonce, aad, aadlen, pt, ptlen, ct, ct + ptlen);
}
int hpke_seal_kem(uint16_t kem, uint16_t aead, const uint8_t* pkR, const uint8_t skE[32],
                  const uint8_t* info, size_t infolen, const uint8_t* aad, size_t aadlen,
                  const uint8_t* pt, size_t ptlen, uint8_t* enc, uint8_t* ct) {
  return hpke_seal_suite(kem, 1, aead, pkR, skE, info, infolen, aad, aadlen, pt, ptlen, enc, ct);
}
int hpke_seal_ex(uint16_t aead, const uint8_t pkR[32], const uint8_t skE[32],
                 const uint8_t* info, size_t infolen, const uint8_t* aad, size_t aadlen,
                 const uint8_t* pt, size_t ptlen, uint8_t enc[32], uint8_t* ct) {
  return hpke_seal_kem(0x20, aead, pkR, skE, info, infolen, aad, aadlen, pt, ptlen, enc, ct);
}
int hpke_seal(const uint8_t pkR[32], const uint8_t skE[32], const uint8_t* info, size_t infolen,
              const uint8_t* aad, size_t aadlen, const uint8_t* pt, size_t ptlen, uint8_t enc[32],
              uint8_t* ct) {
  return hpke_seal_ex(1, pkR, skE, info, infolen, aad, aadlen, pt, ptlen, enc, ct);
}

/* ---- Janus helper layer ------------------------------------------------------------ */

/* PlaintextInputShare::get_decoded + extension checks + helper input share length
 * (aggregator.rs:1893-1990).  Returns HPKE_OK and copies the payload, or HPKE_INVALID_MESSAGE. */
static int decode_plaintext(const uint8_t* pt, size_t len, uint32_t share_len,
                            int require_taskprov, uint8_t* share_out) {
  if (len < 2) return HPKE_INVALID_MESSAGE;
  size_t el = ((size_t)pt[0] << 8) | pt[1], p = 2;
  if (p + el > len) return HPKE_INVALID_MESSAGE;
  uint16_t seen[64];
  int ns = 0, taskprov_ok = 0, taskprov_seen = 0;
  size_t q = p;
  while (q < p + el) {
    if (q + 4 > p + el) return HPKE_INVALID_MESSAGE;
    uint16_t ty = (uint16_t)((pt[q] << 8) | pt[q + 1]);
    size_t dl = ((size_t)pt[q + 2] << 8) | pt[q + 3];
    if (q + 4 + dl > p + el) return HPKE_INVALID_MESSAGE;
    if (ty != 0 && ty != 0xFF00) return HPKE_INVALID_MESSAGE; /* ExtensionType::try_from */
    for (int i = 0; i < ns; i++)
      if (seen[i] == ty) return HPKE_INVALID_MESSAGE; /* duplicate extension */
    if (ns < 64) seen[ns++] = ty;
    if (ty == 0xFF00) { /* ExtensionType::Taskprov */
      taskprov_seen = 1;
      taskprov_ok = dl == 0;
    }
    q += 4 + dl;
  }
  p += el;
  if (p + 4 > len) return HPKE_INVALID_MESSAGE;
  size_t pl = ((size_t)pt[p] << 24) | ((size_t)pt[p + 1] << 16) | ((size_t)pt[p + 2] << 8) | pt[p + 3];
  p += 4;
  if (p + pl != len) return HPKE_INVALID_MESSAGE; /* trailing or missing bytes */
  if (require_taskprov ? !taskprov_ok : taskprov_seen) return HPKE_INVALID_MESSAGE;
  if (pl != share_len) return HPKE_INVALID_MESSAGE;  /* Prio3 helper share: fixed seeds */
  memcpy(share_out, pt + p, pl);
  return HPKE_OK;
}

/* InputShareAad { task_id, ReportMetadata { report_id, time (u64 BE) }, public_share (u32
 * length-prefixed) } (messages/src/lib.rs:1825-1872, 1257-1300) */
size_t hpke_input_share_aad(const uint8_t task_id[32], const uint8_t report_id[16], uint64_t time,
                            const uint8_t* pub, uint32_t publen, uint8_t* out) {
  size_t l = 0;
  memcpy(out, task_id, 32), l += 32;
  memcpy(out + l, report_id, 16), l += 16;
  for (int i = 7; i >= 0; i--) out[l++] = (uint8_t)(time >> (8 * i));
  out[l++] = (uint8_t)(publen >> 24), out[l++] = (uint8_t)(publen >> 16);
  out[l++] = (uint8_t)(publen >> 8), out[l++] = (uint8_t)publen;
  if (publen) memcpy(out + l, pub, publen), l += publen;
  return l;
}

typedef struct {
  const uint8_t *skR, *pkR, *task_id, *enc, *ct, *report_ids, *pubs;
  const uint32_t* ct_len;
  const uint64_t* times;
  uint32_t n, ct_stride, publen, share_len;
  int require_taskprov;
  uint8_t *shares, *status;
  uint32_t lo, hi;
  uint16_t aead, kem, kdf;
} Job;

static const uint8_t INFO[20] = {'d', 'a', 'p', '-', '0', '9', ' ', 'i', 'n', 'p',
                                 'u', 't', ' ', 's', 'h', 'a', 'r', 'e', 1, 3};

static void* run(void* arg) {
  Job* j = (Job*)arg;
  uint8_t aad[256], pt[4096];
  for (uint32_t r = j->lo; r < j->hi; r++) {
    size_t al = hpke_input_share_aad(j->task_id, j->report_ids + 16 * (size_t)r, j->times[r],
                                     j->pubs ? j->pubs + (size_t)j->publen * r : NULL, j->publen,
                                     aad);
    uint32_t cl = j->ct_len[r];
    int ptl = cl <= sizeof(pt) + 16
                  ? hpke_open_suite(j->kem, j->kdf, j->aead, j->skR, j->pkR,
                                    j->enc + kem_nenc(j->kem) * (size_t)r, INFO, sizeof(INFO), aad,
                                    al, j->ct + (size_t)j->ct_stride * r, cl, pt)
                  : -1;
    uint8_t* so = j->shares + (size_t)j->share_len * r;
    memset(so, 0, j->share_len);
    j->status[r] = ptl < 0 ? HPKE_DECRYPT_ERROR
                           : (uint8_t)decode_plaintext(pt, (size_t)ptl, j->share_len,
                                                       j->require_taskprov, so);
    if (j->status[r]) memset(so, 0, j->share_len);
  }
  return NULL;
}

/* Batched helper input-share open: status[r] = 0 (helper share written), 4 (HpkeDecryptError)
 * or 8 (InvalidMessage), the PrepareError codes of messages/src/lib.rs. */
int hpke_open_input_shares_suite(uint16_t kem, uint16_t kdf, uint16_t aead, const uint8_t* skR,
                                 const uint8_t* pkR, const uint8_t task_id[32], uint32_t n,
                                 const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
                                 uint32_t ct_stride, const uint8_t* report_ids,
                                 const uint64_t* times, const uint8_t* pubs, uint32_t publen,
                                 uint32_t share_len, int require_taskprov, uint8_t* shares,
                                 uint8_t* status, int n_threads);
int hpke_open_input_shares_suite(uint16_t kem, uint16_t kdf, uint16_t aead, const uint8_t* skR,
                                 const uint8_t* pkR, const uint8_t task_id[32], uint32_t n,
                                 const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
                                 uint32_t ct_stride, const uint8_t* report_ids,
                                 const uint64_t* times, const uint8_t* pubs, uint32_t publen,
                                 uint32_t share_len, int require_taskprov, uint8_t* shares,
                                 uint8_t* status, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  pthread_t th[256];
  Job jobs[256];
  if (n_threads > 256) n_threads = 256;
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (Job){skR, pkR, task_id, enc, ct, report_ids, pubs, ct_len, times, n, ct_stride,
                    publen, share_len, require_taskprov, shares, status,
                    (uint32_t)((uint64_t)n * t / n_threads),
                    (uint32_t)((uint64_t)n * (t + 1) / n_threads), aead, kem, kdf};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  return 0;
}
int hpke_open_input_shares_kem(uint16_t kem, uint16_t aead, const uint8_t skR[32],
                               const uint8_t* pkR, const uint8_t task_id[32], uint32_t n,
                               const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
                               uint32_t ct_stride, const uint8_t* report_ids,
                               const uint64_t* times, const uint8_t* pubs, uint32_t publen,
                               uint32_t share_len, int require_taskprov, uint8_t* shares,
                               uint8_t* status, int n_threads);
int hpke_open_input_shares_kem(uint16_t kem, uint16_t aead, const uint8_t skR[32],
                               const uint8_t* pkR, const uint8_t task_id[32], uint32_t n,
                               const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
                               uint32_t ct_stride, const uint8_t* report_ids,
                               const uint64_t* times, const uint8_t* pubs, uint32_t publen,
                               uint32_t share_len, int require_taskprov, uint8_t* shares,
                               uint8_t* status, int n_threads) {
  return hpke_open_input_shares_suite(kem, 1, aead, skR, pkR, task_id, n, enc, ct, ct_len,
                                      ct_stride, report_ids, times, pubs, publen, share_len,
                                      require_taskprov, shares, status, n_threads);
}
int hpke_open_input_shares_ex(uint16_t aead, const uint8_t skR[32], const uint8_t pkR[32],
                              const uint8_t task_id[32], uint32_t n, const uint8_t* enc,
                              const uint8_t* ct, const uint32_t* ct_len, uint32_t ct_stride,
                              const uint8_t* report_ids, const uint64_t* times,
                              const uint8_t* pubs, uint32_t publen, uint32_t share_len,
                              int require_taskprov, uint8_t* shares, uint8_t* status,
                              int n_threads) {
  return hpke_open_input_shares_kem(0x20, aead, skR, pkR, task_id, n, enc, ct, ct_len, ct_stride,
                                    report_ids, times, pubs, publen, share_len, require_taskprov,
                                    shares, status, n_threads);
}
int hpke_open_input_shares(const uint8_t skR[32], const uint8_t pkR[32], const uint8_t task_id[32],
                           uint32_t n, const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
                           uint32_t ct_stride, const uint8_t* report_ids, const uint64_t* times,
                           const uint8_t* pubs, uint32_t publen, uint32_t share_len,
                           int require_taskprov, uint8_t* shares, uint8_t* status, int n_threads) {
  return hpke_open_input_shares_ex(1, skR, pkR, task_id, n, enc, ct, ct_len, ct_stride,
                                   report_ids, times, pubs, publen, share_len, require_taskprov,
                                   shares, status, n_threads);
}

/* ---- synthetic batch generation (bench / large tests): the client side of the same layer,
 * seeded per report (every byte = SHA-256(seed || r || purpose) stream), multithreaded ----- */
#include <openssl/sha.h>

typedef struct {
  const uint8_t *pkR, *task_id;
  uint64_t seed;
  uint32_t share_len, publen, stride, lo, hi;
  int taskprov;
  uint8_t *enc, *ct, *ids, *pubs, *shares;
  uint32_t* ct_len;
  uint64_t* times;
  uint16_t aead, kem, kdf;
} GenJob;

static void prf(uint64_t seed, uint32_t r, uint8_t purpose, uint8_t* out, size_t len) {
  uint8_t in[13], h[32];
  memcpy(in, &seed, 8);
  memcpy(in + 8, &r, 4);
  in[12] = purpose;
  for (size_t o = 0; o < len; o += 32) {
    in[12] = (uint8_t)(purpose + 16 * (o / 32));
    SHA256(in, 13, h);
    memcpy(out + o, h, len - o < 32 ? len - o : 32);
  }
}

static void* gen_run(void* arg) {
  GenJob* j = (GenJob*)arg;
  uint8_t pt[4096], aad[256], skE[66];
  const Kem* K = kem_of(j->kem);
  for (uint32_t r = j->lo; r < j->hi; r++) {
    uint8_t* id = j->ids + 16 * (size_t)r;
    uint8_t* share = j->shares + (size_t)j->share_len * r;
    uint8_t* pub = j->publen ? j->pubs + (size_t)j->publen * r : NULL;
    prf(j->seed, r, 1, id, 16);
    prf(j->seed, r, 2, share, j->share_len);
    if (pub) prf(j->seed, r, 3, pub, j->publen);
    prf(j->seed, r, 4, skE, K->nsk);
    uint8_t t8[8];
    prf(j->seed, r, 5, t8, 8);
    j->times[r] = 1700000000ull + (t8[0] | (uint32_t)t8[1] << 8) % 3600u;
    size_t l = 0;
    if (j->taskprov) {
      pt[l++] = 0, pt[l++] = 4;             /* extensions: 4 bytes */
      pt[l++] = 0xFF, pt[l++] = 0x00, pt[l++] = 0, pt[l++] = 0; /* Taskprov, empty */
    } else {
      pt[l++] = 0, pt[l++] = 0;
    }
    pt[l++] = (uint8_t)(j->share_len >> 24), pt[l++] = (uint8_t)(j->share_len >> 16);
    pt[l++] = (uint8_t)(j->share_len >> 8), pt[l++] = (uint8_t)j->share_len;
    memcpy(pt + l, share, j->share_len), l += j->share_len;
    size_t al = hpke_input_share_aad(j->task_id, id, j->times[r], pub, j->publen, aad);
    uint8_t* ct = j->ct + (size_t)j->stride * r;
    memset(ct, 0, j->stride);
    if (j->kem == 0x10) skE[0] &= 0x7f; /* a P-256 scalar below the group order */
    if (j->kem == 0x12) skE[0] = 0;     /* a P-521 scalar below the group order */
    if (j->kem == 0x11) skE[0] &= 0x7f; /* a P-384 scalar below the group order */
    hpke_seal_suite(j->kem, j->kdf, j->aead, j->pkR, skE, INFO, sizeof(INFO), aad, al, pt, l,
                    j->enc + kem_nenc(j->kem) * (size_t)r, ct);
    j->ct_len[r] = (uint32_t)(l + 16);
  }
  return NULL;
}

int hpke_make_input_shares_suite(uint16_t kem, uint16_t kdf, uint16_t aead, const uint8_t* pkR,
                                 const uint8_t task_id[32], uint32_t n, uint64_t seed,
                                 uint32_t share_len, uint32_t publen, int taskprov,
                                 uint32_t stride, uint8_t* enc, uint8_t* ct, uint32_t* ct_len,
                                 uint8_t* ids, uint64_t* times, uint8_t* pubs, uint8_t* shares,
                                 int n_threads) {
  if ((taskprov ? 10u : 6u) + share_len + 16 > stride || !kem_of(kem)) return -1;
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  GenJob jobs[256];
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (GenJob){pkR, task_id, seed, share_len, publen, stride,
                       (uint32_t)((uint64_t)n * t / n_threads),
                       (uint32_t)((uint64_t)n * (t + 1) / n_threads), taskprov, enc, ct, ids, pubs,
                       shares, ct_len, times, aead, kem, kdf};
    pthread_create(&th[t], NULL, gen_run, &jobs[t]);
  }
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  return 0;
}
int hpke_make_input_shares_kem(uint16_t kem, uint16_t aead, const uint8_t* pkR,
                               const uint8_t task_id[32], uint32_t n, uint64_t seed,
                               uint32_t share_len, uint32_t publen, int taskprov, uint32_t stride,
                               uint8_t* enc, uint8_t* ct, uint32_t* ct_len, uint8_t* ids,
                               uint64_t* times, uint8_t* pubs, uint8_t* shares, int n_threads) {
  return hpke_make_input_shares_suite(kem, 1, aead, pkR, task_id, n, seed, share_len, publen,
                                      taskprov, stride, enc, ct, ct_len, ids, times, pubs, shares,
                                      n_threads);
}
int hpke_make_input_shares_ex(uint16_t aead, const uint8_t pkR[32], const uint8_t task_id[32],
                              uint32_t n, uint64_t seed, uint32_t share_len, uint32_t publen,
                              int taskprov, uint32_t stride, uint8_t* enc, uint8_t* ct,
                              uint32_t* ct_len, uint8_t* ids, uint64_t* times, uint8_t* pubs,
                              uint8_t* shares, int n_threads) {
  return hpke_make_input_shares_kem(0x20, aead, pkR, task_id, n, seed, share_len, publen,
                                    taskprov, stride, enc, ct, ct_len, ids, times, pubs, shares,
                                    n_threads);
}
int hpke_make_input_shares(const uint8_t pkR[32], const uint8_t task_id[32], uint32_t n,
                           uint64_t seed, uint32_t share_len, uint32_t publen, int taskprov,
                           uint32_t stride, uint8_t* enc, uint8_t* ct, uint32_t* ct_len,
                           uint8_t* ids, uint64_t* times, uint8_t* pubs, uint8_t* shares,
                           int n_threads) {
  return hpke_make_input_shares_kem(0x20, 1, pkR, task_id, n, seed, share_len, publen, taskprov,
                                    stride, enc, ct, ct_len, ids, times, pubs, shares, n_threads);
}

/* Seal given helper input shares (bench data for the request->response pipeline): enc[n][32],
 * ct[n][stride], ct_len[n]; the ephemeral key of report r is prf(seed, r). */
typedef struct {
  const uint8_t *pkR, *task_id, *ids, *pubs, *shares;
  const uint64_t* times;
  uint64_t seed;
  uint32_t share_len, publen, stride, lo, hi;
  uint8_t *enc, *ct;
  uint32_t* ct_len;
} SealJob;

static void* seal_run(void* arg) {
  SealJob* j = (SealJob*)arg;
  uint8_t pt[4096], aad[256], skE[32];
  for (uint32_t r = j->lo; r < j->hi; r++) {
    size_t l = 0;
    pt[l++] = 0, pt[l++] = 0;
    pt[l++] = (uint8_t)(j->share_len >> 24), pt[l++] = (uint8_t)(j->share_len >> 16);
    pt[l++] = (uint8_t)(j->share_len >> 8), pt[l++] = (uint8_t)j->share_len;
    memcpy(pt + l, j->shares + (size_t)j->share_len * r, j->share_len), l += j->share_len;
    size_t al = hpke_input_share_aad(j->task_id, j->ids + 16 * (size_t)r, j->times[r],
                                     j->publen ? j->pubs + (size_t)j->publen * r : NULL, j->publen,
                                     aad);
    prf(j->seed, r, 4, skE, 32);
    uint8_t* ct = j->ct + (size_t)j->stride * r;
    memset(ct, 0, j->stride);
    hpke_seal(j->pkR, skE, INFO, sizeof(INFO), aad, al, pt, l, j->enc + 32 * (size_t)r, ct);
    j->ct_len[r] = (uint32_t)(l + 16);
  }
  return NULL;
}

int hpke_seal_input_shares(const uint8_t pkR[32], const uint8_t task_id[32], uint32_t n,
                           uint64_t seed, const uint8_t* ids, const uint64_t* times,
                           const uint8_t* pubs, uint32_t publen, const uint8_t* shares,
                           uint32_t share_len, uint32_t stride, uint8_t* enc, uint8_t* ct,
                           uint32_t* ct_len, int n_threads) {
  if (6u + share_len + 16 > stride) return -1;
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  SealJob jobs[256];
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (SealJob){pkR, task_id, ids, pubs, shares, times, seed, share_len, publen, stride,
                        (uint32_t)((uint64_t)n * t / n_threads),
                        (uint32_t)((uint64_t)n * (t + 1) / n_threads), enc, ct, ct_len};
    pthread_create(&th[t], NULL, seal_run, &jobs[t]);
  }
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  return 0;
}

/* AES-128 in CTR mode with a 64-bit big-endian counter in the low half of the IV (the
 * `ctr::Ctr64BE<Aes128>` of prio's SeedStreamAes128, restated): keystream block i =
 * AES(key, iv[0..8] || BE64(iv[8..16] + i)).  For XofHmacSha256Aes128 (oracle/prio3_py.py). */
int aes128_ctr64_keystream(const uint8_t key[16], const uint8_t iv[16], uint8_t* out,
                           size_t len) {
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  if (!c || EVP_EncryptInit_ex(c, EVP_aes_128_ecb(), NULL, key, NULL) != 1) return -1;
  EVP_CIPHER_CTX_set_padding(c, 0);
  uint64_t lo = 0;
  for (int i = 0; i < 8; i++) lo = lo << 8 | iv[8 + i];
  uint8_t blk[16], ks[16];
  for (size_t o = 0; o < len; o += 16) {
    memcpy(blk, iv, 8);
    const uint64_t ctr = lo + o / 16;
    for (int i = 0; i < 8; i++) blk[8 + i] = (uint8_t)(ctr >> (56 - 8 * i));
    int l = 0;
    if (EVP_EncryptUpdate(c, ks, &l, blk, 16) != 1 || l != 16) {
      EVP_CIPHER_CTX_free(c);
      return -1;
    }
    memcpy(out + o, ks, len - o < 16 ? len - o : 16);
  }
  EVP_CIPHER_CTX_free(c);
  return 0;
}
