/*
 * janus_hpke.h -- C ABI of the batched HPKE opener for DAP input shares on MI355X (gfx950)
 * (SURVEY.md 8(f) row 2).
 *
 * It replaces, for a whole aggregation-job batch in one device call, the per-report decryption
 * in the helper's VdafOps::handle_aggregate_init_generic loop
 * (/root/reference/aggregator/src/aggregator.rs:1796-1990): hpke::open(keypair,
 * HpkeApplicationInfo(InputShare, Client, Helper), encrypted_input_share, InputShareAad)
 * (/root/reference/core/src/hpke.rs:186-203), PlaintextInputShare::get_decoded, the
 * duplicate / taskprov extension checks and the helper input share decode -- writing the decoded
 * helper input shares straight into the layout prio3_device_prepare[_aggregate] reads.
 *
 * Suites: mode_base with any KEM x KDF x AEAD of messages/src/lib.rs:770-853:
 *   KEM  DHKEM(X25519, HKDF-SHA256) 0x0020, DHKEM(P-256, HKDF-SHA256) 0x0010 -- the two Janus's
 *        hpke crate implements (core/src/hpke.rs:414-466, 520-525) -- and DHKEM(X448,
 *        HKDF-SHA512) 0x0021, DHKEM(P-521, HKDF-SHA512) 0x0012 (pinned by the RFC 9180 vectors
 *        of core/src/test-vectors.json, which Janus's own test skips), and DHKEM(P-384,
 *        HKDF-SHA384) 0x0011 (no RFC 9180 vector: pinned to the OpenSSL-composed oracle only);
 *   KDF  HKDF-SHA256 0x0001, HKDF-SHA384 0x0002, HKDF-SHA512 0x0003 (the key schedule's);
 *   AEAD AES-128-GCM 0x0001 (X25519 + AES-128-GCM is the configuration Janus generates by
 *        default, hpke.rs:260-300), AES-256-GCM 0x0002, ChaCha20Poly1305 0x0003.
 * Key and enc sizes follow the KEM (RFC 9180 7.1): private key 32 / 32 / 56 / 66 / 48 bytes (the
 * NIST curves' a big-endian scalar, 1 <= sk < n), public key = enc[n][Nenc] with Nenc 32 / 65 /
 * 56 / 133 / 97 (the NIST curves' uncompressed SEC1 points).
 *
 * Conventions as in janus_prio3.h: plain pointers and sizes, caller-owned buffers, device
 * pointers (d_*) stream-ordered on a hipStream_t (NULL = the null stream), per-report failures
 * reported in status, never aborting the batch.
 */
#ifndef JANUS_HPKE_H
#define JANUS_HPKE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  JANUS_HPKE_KEM_X25519_HKDF_SHA256 = 0x0020,
  JANUS_HPKE_KEM_P256_HKDF_SHA256 = 0x0010,
  JANUS_HPKE_KEM_X448_HKDF_SHA512 = 0x0021,
  JANUS_HPKE_KEM_P521_HKDF_SHA512 = 0x0012,
  JANUS_HPKE_KEM_P384_HKDF_SHA384 = 0x0011,
  JANUS_HPKE_KDF_HKDF_SHA256 = 0x0001,
  JANUS_HPKE_KDF_HKDF_SHA384 = 0x0002,
  JANUS_HPKE_KDF_HKDF_SHA512 = 0x0003,
  JANUS_HPKE_AEAD_AES_128_GCM = 0x0001,
  JANUS_HPKE_AEAD_AES_256_GCM = 0x0002,
  JANUS_HPKE_AEAD_CHACHA20_POLY1305 = 0x0003,
};

/* Per-report status: the DAP PrepareError code Janus records for the report
 * (messages/src/lib.rs PrepareError; aggregator.rs:1880-1990). */
enum {
  JANUS_HPKE_OK = 0,
  JANUS_HPKE_DECRYPT_ERROR = 4,    /* PrepareError::HpkeDecryptError */
  JANUS_HPKE_INVALID_MESSAGE = 8,  /* PrepareError::InvalidMessage (plaintext decode, extensions,
                                      input share length) */
};

/* Whole-call return codes (same values as janus_prio3.h). */
enum {
  JANUS_HPKE_SUCCESS = 0,
  JANUS_HPKE_EINVAL = -1,
  JANUS_HPKE_EDEVICE = -2,
  JANUS_HPKE_EUNSUPPORTED = -3,
};

typedef struct janus_hpke_opener janus_hpke_opener;

/* One opener per (HPKE keypair, application info), bound to one GPU: Janus's HpkeKeypair
 * (hpke.rs:283-305) -- private_key is the KEM's SerializePrivateKey, public_key its pkRm -- and
 * HpkeApplicationInfo (hpke.rs:70-85; for helper input shares
 * "dap-09 input share" || 0x01 || 0x03). */
int janus_hpke_opener_create(uint16_t kem_id, uint16_t kdf_id, uint16_t aead_id,
                             const uint8_t* private_key, size_t private_key_len,
                             const uint8_t* public_key, size_t public_key_len,
                             const uint8_t* info, size_t info_len, int device,
                             janus_hpke_opener** out);
void janus_hpke_opener_destroy(janus_hpke_opener* opener);

/* Helper input shares of one task.  Per report r:
 *   d_enc[r][Nenc]                    HpkeCiphertext.encapsulated_key (Nenc of the KEM, above)
 *   d_ct[r][ct_stride], d_ct_len[r]   HpkeCiphertext.payload (ciphertext || 16-byte tag)
 *   d_report_ids[r][16], d_times[r]   ReportMetadata (report ID, time in seconds)
 *   d_public_shares[r][public_share_len]
 * The AAD is InputShareAad { task_id, metadata, public_share } (messages/src/lib.rs:1825-1872),
 * built on the device.  Output: d_helper_shares[r][helper_share_len] (zeroed unless status OK)
 * and d_status[r].  require_taskprov: the task is a taskprov task (aggregator.rs:1925-1958). */
int janus_hpke_open_input_shares_device(janus_hpke_opener* opener, uint32_t n,
                                        const uint8_t task_id[32], const uint8_t* d_enc,
                                        const uint8_t* d_ct, const uint32_t* d_ct_len,
                                        uint32_t ct_stride, const uint8_t* d_report_ids,
                                        const uint64_t* d_times, const uint8_t* d_public_shares,
                                        uint32_t public_share_len, uint32_t helper_share_len,
                                        int require_taskprov, uint8_t* d_helper_shares,
                                        uint8_t* d_status, void* stream);
/* Host-buffer form (blocking).  Concurrent calls -- the helper opens each job's reports on the
 * job's own rayon worker (/root/reference/aggregator/src/aggregator.rs:1847-1890) -- are coalesced
 * by the GPU's HPKE executor into shared launches: every opener's jobs with the same ct_stride,
 * share lengths and taskprov flag, whatever their task IDs (each report carries its task's slot in
 * the group's task-ID table for the AAD). */
int janus_hpke_open_input_shares(janus_hpke_opener* opener, uint32_t n, const uint8_t task_id[32],
                                 const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
                                 uint32_t ct_stride, const uint8_t* report_ids,
                                 const uint64_t* times, const uint8_t* public_shares,
                                 uint32_t public_share_len, uint32_t helper_share_len,
                                 int require_taskprov, uint8_t* helper_shares, uint8_t* status);

/* Generic single-shot open (sequence number 0) with explicit AAD: d_aad[r][aad_stride],
 * d_aad_len[r]; plaintext to d_pt[r][ct_stride] (length d_ct_len[r] - 16), status OK or
 * DECRYPT_ERROR.  Host-buffer form below. */
int janus_hpke_open_device(janus_hpke_opener* opener, uint32_t n, const uint8_t* d_enc,
                           const uint8_t* d_ct, const uint32_t* d_ct_len, uint32_t ct_stride,
                           const uint8_t* d_aad, const uint32_t* d_aad_len, uint32_t aad_stride,
                           uint8_t* d_pt, uint8_t* d_status, void* stream);
int janus_hpke_open(janus_hpke_opener* opener, uint32_t n, const uint8_t* enc, const uint8_t* ct,
                    const uint32_t* ct_len, uint32_t ct_stride, const uint8_t* aad,
                    const uint32_t* aad_len, uint32_t aad_stride, uint8_t* pt, uint8_t* status);

/* The GPU's HPKE executor (shared by every opener on the GPU): counters, and control -- "hold"
 * 1/0 (tests queue jobs behind it; expires by itself after 30 s, or after N ms for hold = N > 1),
 * "heavy" N (as prio3_executor_control; 0 = this executor's default, which never leaves the
 * light-load pipeline: concurrent groups win for the latency-bound open), and two options of this
 * opener: "coalesce" 0/1 (its host-buffer opens launch alone / through the executor, the
 * default), "pair_max" N (X25519 opens of at most N reports run the ladder on lane pairs, default
 * 8192; 0 = never). */
typedef struct {
  uint64_t jobs, reports, groups, active_jobs, active_reports;
} janus_hpke_executor_stats;
int janus_hpke_executor_stats_get(const janus_hpke_opener* opener, janus_hpke_executor_stats* out);
int janus_hpke_executor_control(janus_hpke_opener* opener, const char* key, int64_t value);

/* Per-kernel HIP-event timing of the opener's launches (as prio3_engine_timing). */
int janus_hpke_set_timing(janus_hpke_opener* opener, int on);
int janus_hpke_timing(janus_hpke_opener* opener, double* ms_total, uint32_t* launches);

/* Test-only: one GF(p256) operation of the P-256 KEM's device field code over n host operand
 * pairs (8 x 32-bit LE limbs each, loosely reduced in [0, 2^256)) -- op 0 a*b, 1 a^2, 2 a+b,
 * 3 a-b, 4 3a, 5 8a, 6 a^(p-2); results loosely reduced.  Pins the generated asm
 * (tools/gen_p256_asm.py) against Python integers. */
int janus_hpke_selftest_p256(int op, uint32_t n, const uint32_t* a, const uint32_t* b,
                             uint32_t* out);
/* Test-only: the same for GF(2^448 - 2^224 - 1) (field 1, the X448 KEM; 14 words),
 * GF(2^521 - 1) (field 2, the P-521 KEM; 17 words) and GF(p384) (field 3, the P-384 KEM; 12
 * words, Montgomery form inside), operands canonical LE words below 2^448 / 2^521 / 2^384 --
 * op 0 a*b, 1 a^2, 2 a+b, 3 a-b, 4 a*39081 (X448) or 8a (P-521, P-384), 5 a^(p-2); results
 * canonical (fully reduced). */
int janus_hpke_selftest_field(int field, int op, uint32_t n, const uint32_t* a, const uint32_t* b,
                              uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif
