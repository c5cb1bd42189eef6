/*
 * janus_prio3.h -- C ABI of the MI355X (gfx950) batched Prio3 helper prepare+aggregate
 * engine.  This is the drop-in boundary a Janus FFI crate binds.
 *
 * It replaces, for a whole aggregation-job batch in one device call:
 *   - the VDAF part of the helper's per-report loop in
 *     VdafOps::handle_aggregate_init_generic, /root/reference/aggregator/src/aggregator.rs:2020-2042
 *     (prio `helper_initialized(verify_key, agg_param, nonce, public_share, input_share,
 *      inbound)` followed by `PingPongTransition::evaluate`, i.e. prio 0.16.2 Prio3
 *      prepare_init(agg_id=1) -> decode leader PrepareShare ->
 *      prepare_shares_to_prepare_message([leader, helper]) -> prepare_next);
 *   - the per-report accumulate in AggregationJobWriter::
 *     update_batch_aggregations_from_report_aggregations,
 *     /root/reference/aggregator/src/aggregator/aggregation_job_writer.rs:591-695
 *     (BatchAggregation::merged_with -> AggregateShare::merge,
 *      /root/reference/aggregator_core/src/datastore/models.rs:1318-1372).
 * The instance it is created for corresponds to one arm of `vdaf_dispatch!`
 * (/root/reference/core/src/vdaf.rs:198-300): Prio3Count, Prio3Sum{bits},
 * Prio3SumVec{bits,length,chunk_length}, Prio3Histogram{length,chunk_length}.
 *
 * Conventions: plain pointers and sizes, caller-owned buffers, no callbacks.  All
 * per-report byte strings are fixed-length for a given instance (see prio3_sizes).
 * A per-report failure never aborts the batch; it is reported in status_out.
 */
#ifndef JANUS_PRIO3_H
#define JANUS_PRIO3_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* VDAF kinds (VdafInstance variants, core/src/vdaf.rs:65-108). */
enum {
  PRIO3_COUNT = 0,     /* Prio3::new_count(2)                         (vdaf.rs:201-208) */
  PRIO3_SUM = 1,       /* Prio3::new_sum(2, bits)                     (vdaf.rs:210-217) */
  PRIO3_SUMVEC = 2,    /* Prio3::new_sum_vec_multithreaded(2, ...)    (vdaf.rs:219-235) */
  PRIO3_HISTOGRAM = 3, /* Prio3::new_histogram(2, length, chunk)      (vdaf.rs:257-266) */
  /* Prio3SumVecField64MultiproofHmacSha256Aes128 (vdaf.rs:173-195, algorithm 0xFFFF1003):
   * SumVec<Field64, ParallelSum<Mul>> with XofHmacSha256Aes128, 32-byte seeds and verify key,
   * num_proofs >= 2.  Created with prio3_engine_create_ex (32-byte verify key); helper role. */
  PRIO3_SUMVEC_F64_MP = 4,
  /* Prio3FixedPointBoundedL2VecSum<FixedI16<U15> | FixedI32<U31>> (vdaf.rs:26-31, 292-335,
   * algorithm 0xFFFF0000): bits = 16 or 32 (the BitSize), length = entries; chunk_length is
   * ignored (both gadgets use optimal_chunk_length, as prio does).  Helper role.  The circuit
   * is reconstructed (prio's fixedpoint_l2.rs is not in the reference): DESIGN.md section 10. */
  PRIO3_FPVEC_BOUNDED_L2 = 5,
};

/* Per-report status; each maps 1:1 to the PingPongError variant prio returns and to the
 * metric label Janus records in handle_ping_pong_error
 * (/root/reference/aggregator/src/aggregator/error.rs:365-428). */
enum {
  PRIO3_STATUS_FINISHED = 0,          /* PingPongState::Finished + PingPongMessage::Finish */
  PRIO3_STATUS_PREP_INIT = 1,         /* VdafPrepareInit -> "prepare_init_failure" */
  PRIO3_STATUS_PREP_SHARE_DECODE = 2, /* CodecPrepShare -> "leader_prep_share_decode_failure" */
  PRIO3_STATUS_PREP_MSG = 3,          /* VdafPrepareSharesToPrepareMessage (decide failed) */
  PRIO3_STATUS_PREP_NEXT = 4,         /* VdafPrepareNext (joint randomness mismatch) */
  PRIO3_STATUS_PEER_MISMATCH = 5,     /* PeerMessageMismatch (set by the host framing layer) */
  PRIO3_STATUS_INPUT_SHARE_DECODE = 6, /* leader: input share not canonical -> PrepareError::
                                          InvalidMessage (aggregation_job_driver.rs:397-415) */
};

/* Merged per-report status of prio3_helper_aggregate_init_batch for a report the helper rejects
 * before its VDAF runs: 0x80 | the DAP PrepareError Janus records (messages/src/lib.rs
 * PrepareError; aggregator.rs:1847-1983), which takes precedence over any VDAF status. */
enum {
  PRIO3_STATUS_HPKE_DECRYPT = 0x84,     /* PrepareError::HpkeDecryptError (open / AAD failed) */
  PRIO3_STATUS_INVALID_MESSAGE = 0x88,  /* PrepareError::InvalidMessage (PlaintextInputShare,
                                           extensions, helper input share length) */
};

/* Whole-call return codes. */
enum {
  PRIO3_OK = 0,
  PRIO3_EINVAL = -1,   /* bad parameters / sizes */
  PRIO3_EDEVICE = -2,  /* HIP error (device lost, OOM): caller falls back to its CPU path */
  PRIO3_EUNSUPPORTED = -3,
};

typedef struct {
  uint32_t kind;         /* PRIO3_* */
  uint32_t bits;         /* Sum, SumVec; FPVec bit size (16 or 32) */
  uint32_t length;       /* SumVec, Histogram, FPVec entries */
  uint32_t chunk_length; /* SumVec, Histogram */
  uint32_t num_proofs;   /* 1 for every standard Prio3 instance */
} prio3_params;

typedef struct {
  uint32_t field_bytes;       /* 8 (Field64) or 16 (Field128) */
  uint32_t meas_len, out_len, proof_len, verifier_len, joint_rand_len;
  uint32_t nonce_len;         /* 16 (report ID) */
  uint32_t public_share_len;  /* 2 seeds with joint randomness (32 B; 64 B for 32-byte seeds) */
  uint32_t helper_share_len;  /* 3 seeds with joint randomness, else 2 (16- or 32-byte seeds) */
  uint32_t prep_share_len;    /* leader PrepareShare bytes (verifiers || jr part) */
  uint32_t prep_msg_len;      /* one seed with joint randomness (16 or 32 B), else 0 */
  uint32_t agg_share_len;     /* out_len * field_bytes */
  uint32_t leader_input_share_len; /* enc(meas share) || enc(proofs share) [|| k_blind] */
} prio3_sizes_t;

typedef struct prio3_engine prio3_engine;
typedef struct prio3_batch prio3_batch;

int prio3_sizes(const prio3_params* params, prio3_sizes_t* out);

/* Created where Janus builds VdafOps for a task (aggregator.rs:880-988): one engine per
 * (VDAF instance, verify key), bound to one GPU. */
int prio3_engine_create(const prio3_params* params, const uint8_t verify_key[16], int device,
                        prio3_engine** out);
/* As prio3_engine_create with a verify key of verify_key_len bytes: 16 for the TurboSHAKE
 * instances, 32 for PRIO3_SUMVEC_F64_MP (VERIFY_KEY_LENGTH_HMACSHA256_AES128, vdaf.rs). */
int prio3_engine_create_ex(const prio3_params* params, const uint8_t* verify_key,
                           size_t verify_key_len, int device, prio3_engine** out);
void prio3_engine_destroy(prio3_engine* engine);

/* One engine over several GPUs of the node: the `device_mask` form of SURVEY.md 8(b)'s
 * prio3_engine_create.  A Janus helper process that owns the node's GPUs creates each task's
 * engine over all of them (bit d = GPU d).  Host-buffer jobs (prio3_helper_prepare_batch,
 * prio3_helper_prepare_aggregate_batch, prio3_leader_prepare_init_batch) go whole to the GPU
 * whose executor holds the fewest reports -- the jobs of every engine of the same VDAF instance
 * counted, equally loaded GPUs taken in turn -- and are coalesced there with the other engines'
 * concurrent jobs.  No collective: a job's outputs (prepare messages, statuses, aggregate shares,
 * batch handle) come back whole from the GPU that ran it, and Janus already merges per-job
 * aggregations at collection (aggregation_job_writer.rs:510 writes a random `ord` shard per job;
 * aggregate_share.rs:55-96 sums them).  Device-resident entry points act on the lowest GPU of the
 * mask.  Options set on the engine apply to every GPU's part. */
int prio3_engine_create_mask(const prio3_params* params, const uint8_t* verify_key,
                             size_t verify_key_len, int device_mask, prio3_engine** out);
/* The same over an explicit device list; a GPU named k times gets k executors of its own (lanes
 * 0..k-1, at most 8), which lets a one-GPU box rehearse the placement (tests). */
int prio3_engine_create_devices(const prio3_params* params, const uint8_t* verify_key,
                                size_t verify_key_len, const int* devices, uint32_t n_devices,
                                prio3_engine** out);
typedef struct {
  int32_t device;        /* the member's GPU */
  uint32_t lane;         /* its executor on that GPU (0 unless the device list repeats the GPU) */
  uint64_t jobs;         /* host-buffer jobs this engine placed on the member */
  uint64_t reports;      /* their reports */
  uint64_t exec_jobs;    /* jobs the member's helper executor took (every engine sharing it) */
  uint64_t exec_groups;  /* group launches of that executor */
} prio3_member_info;
/* Fills out[0 .. min(cap, members)) and returns the member count (1 for a one-GPU engine). */
int prio3_engine_members(const prio3_engine* engine, prio3_member_info* out, uint32_t cap);
/* Counters of one executor a member's jobs use (shared with every engine of the same instance on
 * that GPU): kind 0 helper prepare, 1 accumulate, 2 leader prepare_init, 3 leader prepare_next. */
typedef struct {
  uint64_t jobs, reports;  /* submitted since the process started */
  uint64_t groups;         /* launches */
  uint64_t active_jobs, active_reports;  /* inside the executor now */
} prio3_executor_stats;
int prio3_executor_stats_get(const prio3_engine* engine, uint32_t member, int kind,
                             prio3_executor_stats* out);
/* Executor control on the executors of `kind` (as above; -1: every kind) that the engine's jobs
 * use (shared with the other engines of the same GPUs): "hold" = 1 -- launch nothing until
 * "hold" = 0 (tests queue jobs behind it to pin coalescing); "heavy" = N -- reports inside the
 * executor at which it switches from its light-load pipeline to the heavy-load launcher
 * (0: the default 32768; 1: always the heavy-load one). */
int prio3_executor_control(prio3_engine* engine, int kind, const char* key, int64_t value);

/* ---- Host-buffer entry points (what the Rust FFI calls from inside rayon::spawn) ---- */

/* Prepares n reports.  Inputs are packed per report:
 *   nonces[n][16]  (report IDs), public_shares[n][public_share_len],
 *   helper_shares[n][helper_share_len], leader_prep_shares[n][prep_share_len]
 *   (the prep_share of each PingPongMessage::Initialize, framing already removed).
 * Outputs: prep_msgs_out[n][prep_msg_len] (the Finish message payload) and status_out[n].
 * The output shares stay on the device inside *batch_out until prio3_accumulate.
 * Thread-safe: concurrent calls (from any engines of the same VDAF instance on the same GPU,
 * whatever their verify keys) are coalesced by the GPU's executor into shared launches.
 * Each batch owns the device state of its own call: batches of one engine may be accumulated
 * in any order, also after later prepares (free each with prio3_batch_free).
 * PRIO3_FPVEC_BOUNDED_L2 returns PRIO3_EUNSUPPORTED unless option "experimental_fpvec" is 1
 * (its circuit is a reconstruction; parity with prio unpinned). */
int prio3_helper_prepare_batch(prio3_engine* engine, uint32_t n, const uint8_t* nonces,
                               const uint8_t* public_shares, const uint8_t* helper_shares,
                               const uint8_t* leader_prep_shares, uint8_t* prep_msgs_out,
                               uint8_t* status_out, prio3_batch** batch_out);

/* Accumulates the finished reports whose accept_mask byte is non-zero (NULL = all) into
 * per-segment aggregate shares (segment = batch identifier, query_type.rs:72-82).  A segment id
 * >= n_segments excludes the report from every aggregate and count (all accumulate paths).
 * segment_ids (NULL = all segment 0) and accept_mask, when given, must each hold exactly n
 * entries (n = the batch's report count); n_segments >= 1.
 * agg_shares_out[n_segments][agg_share_len] (LE field elements, mod-p sums), counts_out. */
int prio3_accumulate(prio3_batch* batch, const uint32_t* segment_ids, const uint8_t* accept_mask,
                     uint32_t n_segments, uint8_t* agg_shares_out, uint64_t* counts_out);

/* prio3_helper_prepare_batch followed by prio3_accumulate of the same reports, in ONE coalesced
 * launch: the job's reports are accumulated into its n_segments aggregations in the group
 * launch that prepares them (no batch handle, no second round trip through the executor).
 * For callers whose accept mask is known before preparation (the host-side exclusions of the
 * aggregation job writer, aggregation_job_writer.rs:591-695); the output shares are not kept.
 * Same arguments and results as the two calls. */
int prio3_helper_prepare_aggregate_batch(prio3_engine* engine, uint32_t n, const uint8_t* nonces,
                                         const uint8_t* public_shares,
                                         const uint8_t* helper_shares,
                                         const uint8_t* leader_prep_shares,
                                         const uint32_t* segment_ids, const uint8_t* accept_mask,
                                         uint32_t n_segments, uint8_t* prep_msgs_out,
                                         uint8_t* status_out, uint8_t* agg_shares_out,
                                         uint64_t* counts_out);

/* The helper's whole per-report loop body for one aggregation job, from the sealed input shares
 * (VdafOps::handle_aggregate_init_generic, /root/reference/aggregator/src/aggregator.rs:1794-2096):
 * hpke::open of each report's encrypted input share (:1847-1890, the opener of janus_hpke.h, AAD
 * InputShareAad{task_id, metadata, public_share}), PlaintextInputShare decode and the extension
 * checks (:1893-1983; require_taskprov as in janus_hpke_open_input_shares), then
 * helper_initialized + evaluate (:2020-2042) and the accumulate of prio3_helper_prepare_aggregate_
 * batch -- in ONE coalesced group launch: concurrent jobs of every task of the instance that open
 * with the same keypair, ciphertext stride and taskprov flag share it, and the decrypted helper
 * shares never leave the GPU.  Inputs per report: report_ids[n][16] (the VDAF nonces), times[n]
 * (seconds), public_shares[n][public_share_len], enc[n][Nenc], ct[n][ct_stride] with ct_len[n],
 * leader_prep_shares[n][prep_share_len]; segment_ids / accept_mask / n_segments as in
 * prio3_accumulate.  status_out[n]: PRIO3_STATUS_* of the report's VDAF, or
 * PRIO3_STATUS_HPKE_DECRYPT / PRIO3_STATUS_INVALID_MESSAGE when the open rejected it (such a
 * report is never counted).  Instances whose public share is neither 0 nor 32 bytes
 * (PRIO3_SUMVEC_F64_MP) return PRIO3_EUNSUPPORTED.  The opener may be bound to any GPU: the open
 * runs on the GPU the job is placed on. */
struct janus_hpke_opener;
int prio3_helper_aggregate_init_batch(
    prio3_engine* engine, struct janus_hpke_opener* opener, uint32_t n,
    const uint8_t task_id[32], int require_taskprov, const uint8_t* report_ids,
    const uint64_t* times, const uint8_t* public_shares, const uint8_t* enc, const uint8_t* ct,
    const uint32_t* ct_len, uint32_t ct_stride, const uint8_t* leader_prep_shares,
    const uint32_t* segment_ids, const uint8_t* accept_mask, uint32_t n_segments,
    uint8_t* prep_msgs_out, uint8_t* status_out, uint8_t* agg_shares_out, uint64_t* counts_out);

/* Parity-only: copies the n output shares (n x agg_share_len). */
int prio3_debug_output_shares(prio3_batch* batch, uint8_t* out);
void prio3_batch_free(prio3_batch* batch);

/* ---- Device-resident entry points (buffers already in HBM; stream-ordered) ---- */
/* d_* are device pointers with the same packed layouts; stream is a hipStream_t, ordered like
 * any HIP call on it (NULL = the null stream, as in HIP itself -- so a caller whose inputs were
 * produced on the null stream needs no extra synchronisation).  The output shares of the
 * latest device-resident prepare of an engine stay on the device (its "current run") until the
 * next device-resident prepare of that engine replaces it; the accumulate / finish / output-share
 * calls act on that run. */
int prio3_device_prepare(prio3_engine* engine, uint32_t n, const uint8_t* d_nonces,
                         const uint8_t* d_public_shares, const uint8_t* d_helper_shares,
                         const uint8_t* d_leader_prep_shares, uint8_t* d_prep_msgs,
                         uint8_t* d_status, void* stream);
int prio3_device_accumulate(prio3_engine* engine, uint32_t n, const uint8_t* d_status,
                            const uint32_t* d_segment_ids, const uint8_t* d_accept_mask,
                            uint32_t n_segments, uint8_t* d_agg_shares, uint64_t* d_counts,
                            void* stream);
/* Prepare + aggregate in one pass.  Same as prio3_device_prepare, and additionally the output
 * shares of the batch are summed per segment (d_segment_ids[n], NULL = all in segment 0;
 * segment = batch identifier) while the measurement shares stream through the device
 * (Histogram: fused into the joint-randomness kernel; other instances: deferred to the
 * finish call).  prio3_device_aggregate_finish then applies the verdicts in d_status and
 * the host's accept mask (reports Janus drops after preparation -- replays, collected
 * batches: aggregation_job_writer.rs:540-588) and writes d_agg_shares[n_segments][agg_len]
 * and d_counts[n_segments].  Equivalent to prio3_device_prepare + prio3_device_accumulate. */
int prio3_device_prepare_aggregate(prio3_engine* engine, uint32_t n, const uint8_t* d_nonces,
                                   const uint8_t* d_public_shares, const uint8_t* d_helper_shares,
                                   const uint8_t* d_leader_prep_shares,
                                   const uint32_t* d_segment_ids, uint32_t n_segments,
                                   uint8_t* d_prep_msgs, uint8_t* d_status, void* stream);
int prio3_device_aggregate_finish(prio3_engine* engine, const uint8_t* d_status,
                                  const uint8_t* d_accept_mask, uint8_t* d_agg_shares,
                                  uint64_t* d_counts, void* stream);
/* The rest of the per-segment BatchAggregation update (aggregation_job_writer.rs:637-690,
 * models.rs:1318-1372), for the same batch and verdicts:
 *   d_checksums[n_segments][32]  ReportIdChecksum = XOR of SHA-256(report_id) over the reports
 *                                counted in d_counts (status FINISHED and accept mask non-zero;
 *                                core/src/report_id.rs:18-42);
 *   d_intervals[n_segments][2]   client-timestamp interval (start, duration) in seconds over
 *                                every report of the segment, failed ones included
 *                                (Interval::from_time + merge, core/src/time.rs:294-317);
 *                                (0, 0) = Interval::EMPTY for a segment without reports.
 * d_report_ids[n][16] are the report IDs (the VDAF nonces), d_times[n] the report timestamps
 * (NULL: intervals not computed).  Either output may be NULL.  Both are overwritten; merging
 * them into the batch aggregation already stored (XOR / Interval::merge) is the caller's. */
int prio3_device_batch_metadata(prio3_engine* engine, uint32_t n, const uint8_t* d_report_ids,
                                const uint64_t* d_times, const uint8_t* d_status,
                                const uint8_t* d_accept_mask, const uint32_t* d_segment_ids,
                                uint32_t n_segments, uint8_t* d_checksums, uint64_t* d_intervals,
                                void* stream);
/* Multi-GPU combine of k ranks' metadata after an all-gather: d_checksums_in[k][n_segments][32]
 * XORed, d_intervals_in[k][n_segments][2] merged (Interval::merge, empty = identity). */
int prio3_device_combine_metadata(prio3_engine* engine, uint32_t k, uint32_t n_segments,
                                  const uint8_t* d_checksums_in, const uint64_t* d_intervals_in,
                                  uint8_t* d_checksums_out, uint64_t* d_intervals_out,
                                  void* stream);
/* Host-buffer form of prio3_device_batch_metadata (blocking). */
int prio3_batch_metadata(prio3_engine* engine, uint32_t n, const uint8_t* report_ids,
                         const uint64_t* times, const uint8_t* status, const uint8_t* accept_mask,
                         const uint32_t* segment_ids, uint32_t n_segments, uint8_t* checksums_out,
                         uint64_t* intervals_out);
/* Copies the output shares of the last device prepare (n x agg_share_len) to host. */
int prio3_device_output_shares(prio3_engine* engine, uint32_t n, uint8_t* out);

/* Mod-p element-wise sum of k partial aggregate shares (the multi-GPU combine after an
 * RCCL all-gather; RCCL's integer sum is mod 2^64, not mod p).  d_in[k][n_segments*agg_len],
 * d_counts_in[k][n_segments] -> d_out[n_segments*agg_len], d_counts_out[n_segments]. */
int prio3_device_combine(prio3_engine* engine, uint32_t k, uint32_t n_segments,
                         const uint8_t* d_in, const uint64_t* d_counts_in, uint8_t* d_out,
                         uint64_t* d_counts_out, void* stream);

/* ---- Leader side ---- */
/* The leader's half of the same VDAF on the same engine: prio Prio3::prepare_init with
 * agg_id 0 on the explicit leader input shares (what PingPongTopology::leader_initialized
 * runs for each report in AggregationJobDriver::step_aggregation_job_aggregate_init,
 * /root/reference/aggregator/src/aggregator/aggregation_job_driver.rs:397-415), producing the
 * leader prepare shares that go into PingPongMessage::Initialize; then prepare_next on the
 * helper's prepare messages (leader_continued in process_response_from_helper, :677-691):
 * status becomes PREP_NEXT when the message is not the leader's joint-rand seed, and the
 * output shares stay on the device for prio3_accumulate / prio3_device_accumulate.
 * leader_input_shares[n][leader_input_share_len]; prep_shares_out[n][prep_share_len]. */
int prio3_leader_prepare_init_batch(prio3_engine* engine, uint32_t n, const uint8_t* nonces,
                                    const uint8_t* public_shares,
                                    const uint8_t* leader_input_shares, uint8_t* prep_shares_out,
                                    uint8_t* status_out, prio3_batch** batch_out);
int prio3_leader_prepare_next_batch(prio3_batch* batch, const uint8_t* prep_msgs,
                                    uint8_t* status_inout);
/* prio3_leader_prepare_next_batch followed by prio3_accumulate of the same batch, in ONE launch of
 * the GPU's prepare_next executor (concurrent jobs' checks and merges together): for a leader that
 * knows the job's batch identifiers and accept mask when the helper's response arrives
 * (process_response_from_helper, aggregation_job_driver.rs:629-691, then the writer's merge,
 * aggregation_job_writer.rs:591-695).  Same arguments and results as the two calls; the batch
 * keeps its output shares (it may be accumulated again) until prio3_batch_free. */
int prio3_leader_prepare_next_aggregate_batch(prio3_batch* batch, const uint8_t* prep_msgs,
                                              uint8_t* status_inout, const uint32_t* segment_ids,
                                              const uint8_t* accept_mask, uint32_t n_segments,
                                              uint8_t* agg_shares_out, uint64_t* counts_out);
int prio3_device_leader_prepare_init(prio3_engine* engine, uint32_t n, const uint8_t* d_nonces,
                                     const uint8_t* d_public_shares,
                                     const uint8_t* d_leader_input_shares, uint8_t* d_prep_shares,
                                     uint8_t* d_status, void* stream);
int prio3_device_leader_prepare_next(prio3_engine* engine, uint32_t n, const uint8_t* d_prep_msgs,
                                     uint8_t* d_status, void* stream);
/* The device leader's output shares are summed by prio3_device_accumulate.  For Histogram the
 * sum is started inside prio3_device_leader_prepare_init (wave partials while the explicit
 * shares are unpacked; option leader_fuse_acc, default 1): an accumulate over the whole batch
 * with n_segments == 1 finishes from them (the verdicts, the accept mask and out-of-range
 * segment ids are applied as corrections), any other accumulate reads the output shares. */

/* ---- Synthetic client (benchmarks and tests) ---- */
/* Generates n honest reports on the device: the client's shard (prio Prio3::shard,
 * client/src/lib.rs:339-341) and the leader's prepare_init (agg_id 0,
 * aggregation_job_driver.rs:397-415), for the engine's instance and verify key.  Report i is
 * derived from (seed, first_index + i) exactly like the oracle's generator.
 * d_measurements: n x (SumVec: length, else 1) u64 (nullable); d_leader_out_shares:
 * n x agg_share_len (nullable); d_flags: n bytes, non-zero if a rejection-sampling event made
 * the report unusable (nullable); d_leader_input_shares: n x leader_input_share_len, the
 * leader's input shares for the leader-side entry points (nullable). */
int prio3_client_generate_device(prio3_engine* engine, uint32_t n, uint64_t seed,
                                 uint64_t first_index, uint8_t* d_nonces,
                                 uint8_t* d_public_shares, uint8_t* d_helper_shares,
                                 uint8_t* d_leader_prep_shares, uint64_t* d_measurements,
                                 uint8_t* d_leader_out_shares, uint8_t* d_flags,
                                 uint8_t* d_leader_input_shares, void* stream);

/* Frees the idle scratch slabs the device's pool keeps for later calls (up to 1/8 of HBM, shared
 * by every engine on the GPU; a run an engine or a batch handle still references stays).  For a
 * process that hands the GPU's memory to something else between batches. */
int prio3_device_trim(int device);

/* ---- Test / measurement knobs ---- */
/* force_slow_path=1 routes every report through the general rejection-sampling kernel;
 * leader_fuse_acc=0 turns off the fused device-leader accumulate (A/B); pair_max=N runs
 * Histogram(P = 32) prepares of at most N reports on lane pairs (0: never); the other keys are
 * the launch variants prio3_engine.hip's prio3_engine_set_option lists. */
int prio3_engine_set_option(prio3_engine* engine, const char* key, int64_t value);
/* Per-kernel device time (ms) accumulated since the last reset, measured with HIP events
 * on the launch stream when option "timing" is 1 (2: launches counted, no events or times).
 * names: comma-separated kernel names. */
int prio3_engine_timing(prio3_engine* engine, char* names, size_t names_cap, double* ms,
                        uint64_t* launches, int cap);
void prio3_engine_timing_reset(prio3_engine* engine);
/* 1 if the entry points emit roctx ranges (environment JANUS_ROCTX=1 when the library was first
 * used and a roctx library loadable): "handle_aggregate_init_generic threadpool task" around
 * prio3_helper_prepare_batch, "VDAF preparation" around the device prepares, "batch aggregation"
 * around the accumulates -- the spans of aggregator.rs:1786-1790, 2021. */
int prio3_trace_enabled(void);

/* Test-only: runs one Field128 primitive of the device library over n host-supplied operand
 * pairs (16-byte LE elements) -- op 0/1: a*b (compiler / hand-scheduled), 2: a+b, 3: a-b,
 * 4/5: sum of 16 products per output through the lazily reduced MAC (a, b hold 16 n elements).
 * Lets tests pin the hand-written asm arithmetic against Python integers directly. */
int prio3_selftest_field(int op, uint32_t n, const uint8_t* a, const uint8_t* b, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
