/*
 * prio3_oracle.h -- CPU restatement of the Prio3 helper/leader preparation path
 * (TEST INFRASTRUCTURE: the parity checker and the CPU baseline; never shipped, never
 * linked into janus_amd).
 *
 * What this restates
 *   prio 0.16.2 (pinned at /root/reference/Cargo.toml:76, Cargo.lock:3656-3685), which
 *   implements draft-irtf-cfrg-vdaf-08 Prio3 + FlpBBCGGI19 + XofTurboShake128.  The crate
 *   source is NOT present in this container, so the restatement
 *   follows the VDAF-08 specification, cross-checked against the prio call sites Janus
 *   makes: aggregator/src/aggregator.rs:2022-2031 (helper_initialized + evaluate),
 *   aggregator/src/aggregator/aggregation_job_writer.rs:591-695 (accumulate),
 *   aggregator_core/src/datastore/models.rs:1318-1372 (AggregateShare::merge),
 *   core/src/vdaf.rs:198-300 (which Prio3 instance each VdafInstance maps to).
 *
 * Parity status: prio byte-parity is UNPINNED (no prio vectors exist in the reference and
 * the crate cannot be built here).  Pinned: Keccak-p[1600] vs hashlib.shake_128, the
 * RFC 9861 TurboSHAKE128 KAT, field moduli/generators, ping-pong framing bytes
 * (messages/src/tests/aggregation.rs:96-268) and end-to-end unshard == plaintext sum
 * (integration_tests/tests/integration/common.rs:332-554).  An independently written
 * pure-Python restatement (oracle/prio3_py.py) must agree with this file bit-for-bit.
 */
#ifndef PRIO3_ORACLE_H
#define PRIO3_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_COUNT = 0, ORC_SUM = 1, ORC_SUMVEC = 2, ORC_HISTOGRAM = 3, ORC_FPVEC = 4,
       ORC_SUMVEC_F64_MP = 5 };

/* Per-report status codes; identical to include/janus_prio3.h (PRIO3_STATUS_*). */
enum {
  ORC_OK = 0,
  ORC_ERR_PREP_INIT = 1,      /* PingPongError::VdafPrepareInit */
  ORC_ERR_PREP_SHARE_DECODE = 2, /* PingPongError::CodecPrepShare */
  ORC_ERR_DECIDE = 3,         /* PingPongError::VdafPrepareSharesToPrepareMessage */
  ORC_ERR_PREP_NEXT = 4,      /* PingPongError::VdafPrepareNext (joint rand mismatch) */
};

typedef struct {
  int type;
  uint32_t bits, length, chunk_length;
  uint32_t num_proofs;
  uint32_t algorithm_id;
  /* derived */
  uint32_t field_bits;     /* 64 or 128 */
  uint32_t es;             /* encoded element size in bytes */
  uint32_t meas_len, out_len, jr_len, qr_len, prove_rand_len;
  uint32_t arity, degree, calls, wire_len; /* wire_len = P = next_pow2(1+calls) */
  uint32_t proof_len, verifier_len;
  uint32_t helper_share_len, public_share_len, leader_share_len;
  uint32_t prep_share_len, prep_msg_len, out_share_bytes;
  /* ORC_FPVEC (Prio3FixedPointBoundedL2VecSum, the reconstruction fixed in oracle/fpvec_py.py;
   * helper side only: shard / gen_reports return -1): gadget 0 uses chunk_length / arity /
   * calls / wire_len; gadget 1 = ParallelSum(PolyEval(y^2 - 2^n y), fp_C1) over the entries. */
  uint32_t fp_C1, fp_K1, fp_P1;
  /* XOF: seed size (16: XofTurboShake128; 32: XofHmacSha256Aes128, ORC_SUMVEC_F64_MP =
   * Prio3SumVecField64MultiproofHmacSha256Aes128, core/src/vdaf.rs:173-195, helper side only) */
  uint32_t seed_size, xof_hm;
} orc_params;

int orc_params_init(orc_params* p, int type, uint32_t bits, uint32_t length,
                    uint32_t chunk_length, uint32_t num_proofs);

/* Keccak / TurboSHAKE primitives (exported for KAT tests). */
void orc_keccak_p1600(uint64_t s[25], int rounds);
void orc_turboshake128(const uint8_t* msg, size_t len, uint8_t domain, uint8_t* out,
                       size_t out_len);
void orc_shake128(const uint8_t* msg, size_t len, uint8_t* out, size_t out_len);

/* Client: shard one measurement.  meas: Count {0/1}; Sum {value}; SumVec {length values};
 * Histogram {bucket}.  rand: SEEDS*16 bytes (5 seeds with joint randomness, 3 without). */
int orc_shard(const orc_params* p, const uint64_t* meas, const uint8_t nonce[16],
              const uint8_t* rand, uint8_t* public_share, uint8_t* leader_share,
              uint8_t* helper_share);

/* prepare_init for agg_id 0 (leader, explicit share) or 1 (helper, seeds).
 * state_out: meas share (meas_len*es bytes) || corrected joint-rand seed (16, if JR).
 * prep_share_out: prep_share_len bytes. */
int orc_prepare_init(const orc_params* p, const uint8_t* vk, int agg_id,
                     const uint8_t nonce[16], const uint8_t* public_share,
                     const uint8_t* input_share, uint8_t* state_out, uint8_t* prep_share_out);

int orc_prep_shares_to_prep_msg(const orc_params* p, const uint8_t* leader_prep_share,
                                const uint8_t* helper_prep_share, uint8_t* prep_msg_out);

/* out_share_out: out_len*es bytes. */
int orc_prepare_next(const orc_params* p, const uint8_t* state, const uint8_t* prep_msg,
                     uint8_t* out_share_out);

/* Intermediate values of the helper's prepare_init, for golden fixtures. */
int orc_helper_trace(const orc_params* p, const uint8_t* vk, const uint8_t nonce[16],
                     const uint8_t* public_share, const uint8_t* helper_share,
                     uint8_t* meas_out, uint8_t* proofs_out, uint8_t* part_out,
                     uint8_t* corrected_out, uint8_t* jr_out, uint8_t* qr_out,
                     uint8_t* verifier_out);

/* Batched helper prepare+aggregate with Janus's structure: reports are cut into jobs of
 * job_size, each job is processed serially on one of n_threads worker threads
 * (aggregator.rs:1794-2096 inside rayon::spawn 2100-2123), and finished output shares are
 * merged per segment (aggregation_job_writer.rs:591-695).  The leader prep share is the
 * raw prep_share bytes (ping-pong framing is removed by the caller).
 * agg_out: n_segments * out_len * es bytes; count_out: n_segments. */
int orc_helper_batch(const orc_params* p, const uint8_t* vk, uint32_t n,
                     const uint8_t* nonces, const uint8_t* public_shares,
                     const uint8_t* helper_shares, const uint8_t* leader_prep_shares,
                     const uint32_t* segment_ids, const uint8_t* accept_mask,
                     uint32_t n_segments, uint8_t* prep_msgs_out, uint8_t* status_out,
                     uint8_t* agg_out, uint64_t* count_out, int n_threads, int job_size);

/* Batched leader prepare_init (agg_id 0) + prepare_next (prep_msgs: the helper's prepare
 * messages, seed_size bytes each, nullable without joint randomness) + aggregate, one
 * segment.  Status: 0 finished, ORC_ERR_PREP_INIT (non-canonical share element) or
 * ORC_ERR_PREP_NEXT.  prep_shares_out: n x prep_share_len (zero on init failure). */
int orc_leader_batch(const orc_params* p, const uint8_t* vk, uint32_t n, const uint8_t* nonces,
                     const uint8_t* public_shares, const uint8_t* leader_shares,
                     const uint8_t* prep_msgs, uint8_t* prep_shares_out, uint8_t* status_out,
                     uint8_t* agg_out, uint64_t* count_out, int n_threads, int job_size);
/* orc_leader_batch with per-report segment ids (NULL: segment 0; ids >= n_segments are
 * prepared but aggregated nowhere): agg_out[n_segments][out_len * es], count_out[n_segments]. */
int orc_leader_batch_seg(const orc_params* p, const uint8_t* vk, uint32_t n,
                         const uint8_t* nonces, const uint8_t* public_shares,
                         const uint8_t* leader_shares, const uint8_t* prep_msgs,
                         const uint32_t* segment_ids, uint32_t n_segments,
                         uint8_t* prep_shares_out, uint8_t* status_out, uint8_t* agg_out,
                         uint64_t* count_out, int n_threads, int job_size);

/* Deterministic synthetic reports (client shard + leader prepare_init), multithreaded.
 * meas_out: n x (SumVec: length, else 1) u64; leader_out_shares: n x out_len*es (nullable). */
int orc_gen_reports(const orc_params* p, const uint8_t vk[16], uint32_t n, uint64_t seed,
                    int n_threads, uint8_t* nonces, uint8_t* publics, uint8_t* helpers,
                    uint8_t* leader_ps, uint64_t* meas_out, uint8_t* leader_out_shares);

/* Mod-p element-wise sum of agg shares (AggregateShare::merge). */
void orc_agg_merge(const orc_params* p, uint8_t* acc, const uint8_t* other);

/* ns per Keccak-p[1600, 12] permutation and per Field128 multiply on one core */
void orc_prim_bench(double* ns_perm, double* ns_mul);

#ifdef __cplusplus
}
#endif
#endif
