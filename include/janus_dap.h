/*
 * janus_dap.h -- C ABI of the DAP wire-format <-> SoA marshaling around the device calls
 * (SURVEY.md 8(f) row 3), MI355X (gfx950).
 *
 * Helper side of an aggregation job, DAP-09 encodings of /root/reference/messages/src/lib.rs:
 *   AggregationJobInitializeReq (lib.rs:2362-2400) = u32-prefixed aggregation parameter,
 *     PartialBatchSelector (query type byte, + 32-byte BatchId for FixedSize),
 *     u32-prefixed list of PrepareInit (lib.rs:2021-2070):
 *       ReportShare { ReportMetadata { report_id[16], time u64 }, u32-prefixed public share,
 *                     HpkeCiphertext { config_id u8, u16-prefixed enc, u32-prefixed payload } }
 *       u32-prefixed PingPongMessage (type u8, u32-prefixed prep_share for Initialize)
 *   AggregationJobResp (lib.rs:2535-2550) = u32-prefixed list of PrepareResp { report_id,
 *     PrepareStepResult: 0 Continue { u32-prefixed PingPongMessage } | 1 Finished |
 *     2 Reject(PrepareError u8) }  (lib.rs:2130-2190)
 *
 * These replace Janus's per-report decode (`AggregationJobInitializeReq::get_decoded`,
 * aggregator.rs:1720-1790) and the response assembly (aggregator.rs:2044-2096, 2140-2170):
 * the request body is unpacked on the device straight into the SoA buffers
 * janus_hpke_open_input_shares_device and prio3_device_prepare_aggregate read, and the response
 * body is encoded on the device from their outputs.
 *
 * Unpack is speculative: when every PrepareInit of the body has the byte length of the first
 * one (one VDAF, one HPKE suite, same extensions -- the normal case) the device parses all of
 * them in parallel and validates each; any record that does not fit is reported and the caller
 * uses the host parser (janus_dap_agg_init_unpack_host) for the body.
 */
#ifndef JANUS_DAP_H
#define JANUS_DAP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { JANUS_DAP_QUERY_TIME_INTERVAL = 1, JANUS_DAP_QUERY_FIXED_SIZE = 2 };

/* Per-report message status written by unpack (prio3 status codes, janus_prio3.h): 0 = the
 * message is PingPongMessage::Initialize with a prep_share of the expected length;
 * 2 = CodecPrepShare (wrong prep_share length); 5 = PeerMessageMismatch (Continue / Finish);
 * 6 = the public share has another length than layout->public_share_len -- it does not decode:
 * PrepareError::InvalidMessage (aggregator.rs:1985-1999), after any HPKE error of the report.
 * A PingPongMessage that does not decode (unknown type, bad framing) rejects the whole request,
 * as Janus's request decode does.  janus_dap_agg_init_scan_ex takes the lengths the task
 * expects (VDAF public share, KEM Nenc, VDAF prep share), so a malformed first record fails
 * alone; janus_dap_agg_init_scan takes them from the first record. */

typedef struct {
  /* filled by janus_dap_agg_init_scan */
  uint32_t n;                   /* number of PrepareInits (valid after unpack_host; for the
                                   device path n = list bytes / record_len) */
  uint8_t query_type;           /* JANUS_DAP_QUERY_* */
  uint8_t batch_id[32];         /* FixedSize only */
  uint64_t agg_param_off, agg_param_len;
  uint64_t list_off, list_len;  /* byte range of the PrepareInit list */
  uint32_t record_len;          /* byte length of the first PrepareInit */
  uint32_t public_share_len;    /* expected (scan_ex) or of the first record */
  uint32_t enc_len, payload_len, message_len, prep_share_len;  /* enc / prep share: as
                                   public_share_len; payload, message: of the first record */
  int uniform;                  /* list_len is a multiple of record_len */
} janus_dap_agg_init_layout;

/* Parses the header and the first PrepareInit of an AggregationJobInitializeReq body (host
 * memory; O(1)).  Returns 0, or -1 if the header does not decode. */
int janus_dap_agg_init_scan(const uint8_t* body, size_t len, janus_dap_agg_init_layout* out);

/* As janus_dap_agg_init_scan, with the lengths every record must have: the VDAF's public share
 * length, the HPKE KEM's Nenc and the VDAF's leader prep share length (JANUS_DAP_LEN_ANY: the
 * first record's).  The layout carries the expected lengths; if the first record differs from
 * them, layout->uniform is 0 and the caller unpacks on the host, where each record with another
 * public share / prep share length gets msg_status 6 / 2 and another enc length ct_len 0 (HPKE
 * decrypt error) -- the reference fails only that report (aggregator.rs:1967-1999). */
#define JANUS_DAP_LEN_ANY 0xFFFFFFFFu
int janus_dap_agg_init_scan_ex(const uint8_t* body, size_t len, uint32_t public_share_len,
                               uint32_t enc_len, uint32_t prep_share_len,
                               janus_dap_agg_init_layout* out);

/* Device unpack of a body whose records all have layout->record_len bytes (layout->uniform).
 * d_body is the request body in device memory.  Outputs (device, n = list_len / record_len):
 *   d_report_ids[n][16], d_times[n] (seconds), d_public_shares[n][public_share_len],
 *   d_config_ids[n], d_enc[n][enc_len], d_ct[n][ct_stride] + d_ct_len[n] (the HPKE payload),
 *   d_prep_shares[n][prep_share_len] (leader prep share), d_msg_status[n].
 * ct_stride must be >= payload_len and a multiple of 16.  *d_mismatch (device u32, zeroed here)
 * counts the records that do not have the first record's shape; when it is non-zero the outputs
 * are incomplete and the caller must use janus_dap_agg_init_unpack_host. */
int janus_dap_agg_init_unpack_device(const janus_dap_agg_init_layout* layout, const uint8_t* d_body,
                                     uint8_t* d_report_ids, uint64_t* d_times,
                                     uint8_t* d_public_shares, uint8_t* d_config_ids,
                                     uint8_t* d_enc, uint8_t* d_ct, uint32_t* d_ct_len,
                                     uint32_t ct_stride, uint8_t* d_prep_shares,
                                     uint8_t* d_msg_status, uint32_t* d_mismatch, void* stream);

/* Host (sequential) unpack of any well-formed body into host SoA buffers sized for `cap`
 * records: prep shares / public shares of another length than the first record's get
 * msg_status 2 / 6 (the public share row is zero-filled);
 * payloads longer than ct_stride give ct_len 0 (HPKE decrypt error).  Returns the number of
 * records, or -1 if the body does not decode (the whole request is rejected, as Janus does). */
int64_t janus_dap_agg_init_unpack_host(const uint8_t* body, size_t len,
                                       const janus_dap_agg_init_layout* layout, uint32_t cap,
                                       uint8_t* report_ids, uint64_t* times,
                                       uint8_t* public_shares, uint8_t* config_ids, uint8_t* enc,
                                       uint8_t* ct, uint32_t* ct_len, uint32_t ct_stride,
                                       uint8_t* prep_shares, uint8_t* msg_status);

/* AggregationJobResp for the helper's init step.  Per report the PrepareStepResult is
 *   prepare_error[r] != 0xFF  -> Reject(prepare_error[r])       (HPKE / decode / host checks)
 *   else prio3_status[r] == 0 -> Continue { PingPongMessage::Finish { prep_msg[r] } }
 *   else                      -> Reject(VdafPrepError = 5)        (handle_ping_pong_error)
 * Device form: d_out must hold janus_dap_agg_job_resp_max_len(n, prep_msg_len) bytes;
 * *d_out_len (device u64) receives the encoded length.  d_scratch: 4 * (n / 256 + 2) bytes. */
size_t janus_dap_agg_job_resp_max_len(uint32_t n, uint32_t prep_msg_len);
int janus_dap_agg_job_resp_encode_device(uint32_t n, const uint8_t* d_report_ids,
                                         const uint8_t* d_prepare_error,
                                         const uint8_t* d_prio3_status, const uint8_t* d_prep_msgs,
                                         uint32_t prep_msg_len, uint8_t* d_out,
                                         uint64_t* d_out_len, uint32_t* d_scratch, void* stream);
int64_t janus_dap_agg_job_resp_encode_host(uint32_t n, const uint8_t* report_ids,
                                           const uint8_t* prepare_error,
                                           const uint8_t* prio3_status, const uint8_t* prep_msgs,
                                           uint32_t prep_msg_len, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
