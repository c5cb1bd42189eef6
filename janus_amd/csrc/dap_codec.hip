// dap_codec.hip -- DAP-09 wire format <-> SoA marshaling for the helper's aggregation-job init
// on MI355X (gfx950); SURVEY 8(f) row 3.  See include/janus_dap.h for the encodings.
//
//  k_unpack_check / k_unpack_gather
//                 the speculative uniform layout (every PrepareInit has the first one's
//                 length): one lane per record validates its length and type fields; then one
//                 lane per OUTPUT DWORD gathers the byte fields (report ID, public share, enc,
//                 payload, leader prep share) into the SoA buffers the HPKE opener and the
//                 prio3 engine read -- coalesced reads of the body and coalesced writes.
//  k_resp_count / k_resp_scan / k_resp_write
//                 AggregationJobResp: per-block counts of the two PrepareResp sizes, an
//                 exclusive scan of the block totals, then each lane writes its record at its
//                 byte offset (block-local prefix via __syncthreads_count-style LDS scan).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "../../include/janus_dap.h"

#define DEV __device__ __forceinline__

namespace {

// big-endian reads at an arbitrary byte offset of a device buffer (dword-aligned loads)
DEV uint32_t ld_be32(const uint8_t* base, uint64_t off) {
  const uint64_t a = off & ~3ull;
  const uint32_t sh = (uint32_t)(off & 3u);
  const uint32_t lo = *(const uint32_t*)(base + a);
  const uint32_t hi = sh ? *(const uint32_t*)(base + a + 4) : 0u;
  const uint32_t le = sh ? __builtin_amdgcn_alignbit(hi, lo, 8 * sh) : lo;
  return __builtin_bswap32(le);
}
DEV uint32_t ld_u8(const uint8_t* base, uint64_t off) { return base[off]; }
DEV uint32_t ld_be16(const uint8_t* base, uint64_t off) {
  return (ld_u8(base, off) << 8) | ld_u8(base, off + 1);
}
// little-endian word (memory order) at an arbitrary byte offset
DEV uint32_t ld_le32(const uint8_t* base, uint64_t off) {
  const uint64_t a = off & ~3ull;
  const uint32_t sh = (uint32_t)(off & 3u);
  const uint32_t lo = *(const uint32_t*)(base + a);
  if (!sh) return lo;
  const uint32_t hi = *(const uint32_t*)(base + a + 4);
  return __builtin_amdgcn_alignbit(hi, lo, 8 * sh);
}
struct UnpackArgs {
  const uint8_t* body;
  uint64_t list_off;
  uint32_t n, rec, psl, enc_len, pay_len, msg_len, ps_len;
  uint8_t *cfg, *msg_status;
  uint64_t* times;
  uint32_t *ct_len, *mismatch;
};

// The body buffer must be readable up to a dword past its end (the host pads the copy).
// k_unpack_check: one lane per record, only the length / type fields (a few scattered loads):
// validates the record against the first record's shape and writes the small per-report
// outputs (time, config id, payload length, message status).
__global__ __launch_bounds__(256) void k_unpack_check(UnpackArgs a) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  const uint8_t* b = a.body;
  uint64_t o = a.list_off + (uint64_t)r * a.rec;
  const uint64_t end = o + a.rec;
  const uint64_t o_time = o + 16;
  o += 24;
  const uint32_t psl = ld_be32(b, o);
  o += 4 + (uint64_t)psl;
  bool ok = psl == a.psl && o + 3 <= end;
  const uint32_t cfg = ok ? ld_u8(b, o) : 0u;
  const uint32_t encl = ok ? ld_be16(b, o + 1) : 0u;
  o += 3 + (uint64_t)encl;
  ok = ok && encl == a.enc_len && o + 4 <= end;
  const uint32_t payl = ok ? ld_be32(b, o) : 0u;
  o += 4 + (uint64_t)payl;
  ok = ok && payl == a.pay_len && o + 4 <= end;
  const uint32_t msgl = ok ? ld_be32(b, o) : 0u;
  const uint64_t o_msg = o + 4;
  ok = ok && msgl == a.msg_len && o_msg + msgl == end;
  if (!ok) {
    atomicAdd(a.mismatch, 1u);
    a.msg_status[r] = 2;
    return;
  }
  // PingPongMessage: Initialize { u32-prefixed prep_share } expected (ping_pong.rs framing,
  // messages/src/tests/aggregation.rs:201-209)
  const uint32_t ty = ld_u8(b, o_msg);
  const uint32_t psl2 = msgl >= 5 ? ld_be32(b, o_msg + 1) : 0xffffffffu;
  // a message that does not decode rejects the whole request: leave it to the host parser
  bool wf = msgl >= 5 && ty <= 2;
  if (wf && ty != 1) wf = (uint64_t)msgl == 5 + (uint64_t)psl2;
  if (wf && ty == 1)
    wf = 9 + (uint64_t)psl2 <= msgl &&
         (uint64_t)msgl == 9 + (uint64_t)psl2 + ld_be32(b, o_msg + 5 + psl2);
  if (!wf) {
    atomicAdd(a.mismatch, 1u);
    a.msg_status[r] = 2;
    return;
  }
  uint8_t st = 0;
  if (ty != 0)
    st = 5;  // PeerMessageMismatch
  else if (psl2 != a.ps_len)
    st = 2;  // CodecPrepShare
  a.msg_status[r] = st;
  a.times[r] = ((uint64_t)ld_be32(b, o_time) << 32) | ld_be32(b, o_time + 4);
  a.cfg[r] = (uint8_t)cfg;
  a.ct_len[r] = a.pay_len;
}

// k_unpack_gather: the byte fields, one output dword per lane (grid.y = field): adjacent lanes
// read adjacent source bytes of the uniform records and write adjacent output dwords, so both
// sides are coalesced.  Output rows are `row` bytes, the field is `len` bytes at `off` within
// each record; bytes past `len` in a row are zeroed.  Rows that are not a multiple of 4 bytes
// (no Prio3 / X25519 field has one, but the ABI allows it) take a bytewise branch.
struct GatherField {
  uint8_t* dst;
  uint32_t row, len, off;
};
struct GatherArgs {
  const uint8_t* body;
  uint64_t list_off;
  uint32_t n, rec;
  GatherField f[5];
};
__global__ __launch_bounds__(256) void k_unpack_gather(GatherArgs g) {
  const GatherField F = g.f[blockIdx.y];
  if (!F.dst) return;
  const uint64_t total = (uint64_t)g.n * F.row;  // output bytes
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * i >= total) return;
  if ((F.row & 3u) == 0) {
    const uint32_t wpr = F.row >> 2;
    const uint32_t r = (uint32_t)(i / wpr), b = 4 * (uint32_t)(i - (uint64_t)r * wpr);
    uint32_t v = 0;
    if (b < F.len) {
      v = ld_le32(g.body, g.list_off + (uint64_t)r * g.rec + F.off + b);
      if (b + 4 > F.len) v &= (1u << (8 * (F.len - b))) - 1u;
    }
    ((uint32_t*)F.dst)[i] = v;
    return;
  }
  for (uint32_t k = 0; k < 4; k++) {
    const uint64_t j = 4 * i + k;
    if (j >= total) break;
    const uint32_t r = (uint32_t)(j / F.row), c = (uint32_t)(j - (uint64_t)r * F.row);
    F.dst[j] = c < F.len ? g.body[g.list_off + (uint64_t)r * g.rec + F.off + c] : 0;
  }
}

// ---- AggregationJobResp ----------------------------------------------------------------
// record sizes: Continue{Finish{prep_msg}} = 16 + 1 + 4 + 1 + 4 + pml; Reject = 16 + 1 + 1
DEV bool resp_ok(const uint8_t* pe, const uint8_t* st, uint32_t r) {
  return pe[r] == 0xFF && st[r] == 0;
}

__global__ __launch_bounds__(256) void k_resp_count(uint32_t n, const uint8_t* pe,
                                                    const uint8_t* st, uint32_t* blk) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const int ok = r < n && resp_ok(pe, st, r);
  const int c = __syncthreads_count(ok);
  if (threadIdx.x == 0) blk[blockIdx.x] = (uint32_t)c;
}

// exclusive scan of the per-block ok counts (one block of 1024 threads, sequential chunks)
__global__ __launch_bounds__(1024) void k_resp_scan(uint32_t nb, uint32_t* blk, uint32_t n,
                                                    uint32_t pml, uint64_t* out_len,
                                                    uint8_t* out) {
  __shared__ uint32_t s[1024];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nb; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < nb ? blk[i] : 0u;
    s[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
      const uint32_t t = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < nb) blk[i] = carry + s[threadIdx.x] - v;  // exclusive
    __syncthreads();
    if (threadIdx.x == 1023) carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const uint64_t n_ok = carry;
    const uint64_t body = n_ok * (26ull + pml) + ((uint64_t)n - n_ok) * 18ull;
    *out_len = 4 + body;
    out[0] = (uint8_t)(body >> 24);  // u32-prefixed PrepareResp list
    out[1] = (uint8_t)(body >> 16);
    out[2] = (uint8_t)(body >> 8);
    out[3] = (uint8_t)body;
  }
}

__global__ __launch_bounds__(256) void k_resp_write(uint32_t n, const uint8_t* ids,
                                                    const uint8_t* pe, const uint8_t* st,
                                                    const uint8_t* pm, uint32_t pml,
                                                    const uint32_t* blk, uint8_t* out) {
  __shared__ uint32_t s[256];
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t ok = (r < n && resp_ok(pe, st, r)) ? 1u : 0u;
  s[threadIdx.x] = ok;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    const uint32_t t = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  if (r >= n) return;
  const uint64_t oks_before = (uint64_t)blk[blockIdx.x] + s[threadIdx.x] - ok;
  const uint64_t before = r;  // records before r
  uint64_t o = 4 + oks_before * (26ull + pml) + (before - oks_before) * 18ull;
  for (int i = 0; i < 16; i++) out[o + i] = ids[16 * (size_t)r + i];
  o += 16;
  if (ok) {
    const uint32_t ml = 5 + pml;  // PingPongMessage::Finish { prep_msg }
    out[o] = 0;                   // PrepareStepResult::Continue
    out[o + 1] = (uint8_t)(ml >> 24);
    out[o + 2] = (uint8_t)(ml >> 16);
    out[o + 3] = (uint8_t)(ml >> 8);
    out[o + 4] = (uint8_t)ml;
    out[o + 5] = 2;  // PingPongMessage type Finish
    out[o + 6] = (uint8_t)(pml >> 24);
    out[o + 7] = (uint8_t)(pml >> 16);
    out[o + 8] = (uint8_t)(pml >> 8);
    out[o + 9] = (uint8_t)pml;
    for (uint32_t i = 0; i < pml; i++) out[o + 10 + i] = pm[(size_t)pml * r + i];
  } else {
    out[o] = 2;  // PrepareStepResult::Reject
    out[o + 1] = pe[r] != 0xFF ? pe[r] : 5;  // PrepareError (VdafPrepError for prio3 failures)
  }
}

// ---- host helpers -----------------------------------------------------------------------
struct Cur {
  const uint8_t* p;
  size_t len, o;
  bool ok = true;
  bool need(size_t k) {
    if (!ok || o + k > len) ok = false;
    return ok;
  }
  uint32_t u8() { return need(1) ? p[o++] : 0; }
  uint32_t u16() {
    if (!need(2)) return 0;
    const uint32_t v = (uint32_t)p[o] << 8 | p[o + 1];
    o += 2;
    return v;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    const uint32_t v = (uint32_t)p[o] << 24 | (uint32_t)p[o + 1] << 16 | (uint32_t)p[o + 2] << 8 |
                       p[o + 3];
    o += 4;
    return v;
  }
  uint64_t u64() {
    const uint64_t hi = u32();
    return hi << 32 | u32();
  }
};

struct RecShape {
  uint64_t o_id, o_pub, o_enc, o_pay, o_msg;
  uint32_t psl, cfg, enc_len, pay_len, msg_len;
  uint64_t time, end;
};

uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

// PingPongMessage framing (ping_pong.rs; messages/src/tests/aggregation.rs:201-268):
// 0 Initialize { prep_share<u32> }, 1 Continue { prep_msg<u32>, prep_share<u32> },
// 2 Finish { prep_msg<u32> }; the message must use every byte of its u32-prefixed field
bool pingpong_wellformed(const uint8_t* m, uint64_t len) {
  if (len < 5) return false;
  const uint64_t a = be32(m + 1);
  switch (m[0]) {
    case 0:
    case 2:
      return len == 5 + a;
    case 1:
      return 9 + a <= len && len == 9 + a + be32(m + 5 + a);
    default:
      return false;
  }
}

bool parse_record(Cur& c, RecShape& s) {
  s.o_id = c.o;
  c.need(16);
  c.o += 16;
  s.time = c.u64();
  s.psl = c.u32();
  s.o_pub = c.o;
  if (!c.need(s.psl)) return false;
  c.o += s.psl;
  s.cfg = c.u8();
  s.enc_len = c.u16();
  s.o_enc = c.o;
  if (!c.need(s.enc_len)) return false;
  c.o += s.enc_len;
  s.pay_len = c.u32();
  s.o_pay = c.o;
  if (!c.need(s.pay_len)) return false;
  c.o += s.pay_len;
  s.msg_len = c.u32();
  s.o_msg = c.o;
  if (!c.need(s.msg_len)) return false;
  c.o += s.msg_len;
  s.end = c.o;
  return c.ok;
}

}  // namespace

#define DCHK(x)                                                                       \
  do {                                                                                \
    hipError_t _e = (x);                                                              \
    if (_e != hipSuccess) {                                                           \
      fprintf(stderr, "janus_dap: HIP error %s at %s:%d\n", hipGetErrorString(_e),    \
              __FILE__, __LINE__);                                                    \
      return -2;                                                                      \
    }                                                                                 \
  } while (0)

extern "C" {

int janus_dap_agg_init_scan(const uint8_t* body, size_t len, janus_dap_agg_init_layout* L) {
  if (!body || !L) return -1;
  memset(L, 0, sizeof(*L));
  Cur c{body, len, 0};
  L->agg_param_len = c.u32();
  L->agg_param_off = c.o;
  if (!c.need(L->agg_param_len)) return -1;
  c.o += L->agg_param_len;
  L->query_type = (uint8_t)c.u8();
  if (L->query_type == JANUS_DAP_QUERY_FIXED_SIZE) {
    if (!c.need(32)) return -1;
    memcpy(L->batch_id, body + c.o, 32);
    c.o += 32;
  } else if (L->query_type != JANUS_DAP_QUERY_TIME_INTERVAL) {
    return -1;
  }
  L->list_len = c.u32();
  L->list_off = c.o;
  if (!c.ok || L->list_off + L->list_len != len) return -1;  // trailing bytes: decode error
  if (L->list_len == 0) {
    L->uniform = 1;
    return 0;
  }
  RecShape s;
  Cur r{body, L->list_off + L->list_len, L->list_off};
  if (!parse_record(r, s)) return -1;
  L->record_len = (uint32_t)(s.end - L->list_off);
  L->public_share_len = s.psl;
  L->enc_len = s.enc_len;
  L->payload_len = s.pay_len;
  L->message_len = s.msg_len;
  L->prep_share_len = (s.msg_len >= 5 && body[s.o_msg] == 0) ? s.msg_len - 5 : 0;
  L->uniform = L->list_len % L->record_len == 0;
  L->n = L->uniform ? (uint32_t)(L->list_len / L->record_len) : 0;
  return 0;
}

int janus_dap_agg_init_scan_ex(const uint8_t* body, size_t len, uint32_t public_share_len,
                               uint32_t enc_len, uint32_t prep_share_len,
                               janus_dap_agg_init_layout* L) {
  const int rc = janus_dap_agg_init_scan(body, len, L);
  if (rc || L->list_len == 0) return rc;
  // the task's expected lengths, not the first record's: a record whose public share, enc or
  // prep share has another length fails alone, and a body whose first record is off
  // is unpacked on the host, where every record is checked against these
  const bool fits = (public_share_len == JANUS_DAP_LEN_ANY || L->public_share_len == public_share_len) &&
                    (enc_len == JANUS_DAP_LEN_ANY || L->enc_len == enc_len) &&
                    (prep_share_len == JANUS_DAP_LEN_ANY || L->prep_share_len == prep_share_len);
  if (public_share_len != JANUS_DAP_LEN_ANY) L->public_share_len = public_share_len;
  if (enc_len != JANUS_DAP_LEN_ANY) L->enc_len = enc_len;
  if (prep_share_len != JANUS_DAP_LEN_ANY) L->prep_share_len = prep_share_len;
  if (!fits) {
    L->uniform = 0;
    L->n = 0;
  }
  return 0;
}

int janus_dap_agg_init_unpack_device(const janus_dap_agg_init_layout* L, const uint8_t* d_body,
                                     uint8_t* d_report_ids, uint64_t* d_times,
                                     uint8_t* d_public_shares, uint8_t* d_config_ids,
                                     uint8_t* d_enc, uint8_t* d_ct, uint32_t* d_ct_len,
                                     uint32_t ct_stride, uint8_t* d_prep_shares,
                                     uint8_t* d_msg_status, uint32_t* d_mismatch, void* stream) {
  if (!L || !d_mismatch || !L->uniform) return -1;
  hipStream_t st = (hipStream_t)stream;
  DCHK(hipMemsetAsync(d_mismatch, 0, 4, st));
  if (L->n == 0) return 0;
  if (!d_body || !d_report_ids || !d_times || !d_config_ids || !d_enc || !d_ct || !d_ct_len ||
      !d_prep_shares || !d_msg_status || (L->public_share_len && !d_public_shares) ||
      ct_stride < L->payload_len || ct_stride % 16)
    return -1;
  UnpackArgs a{};
  a.body = d_body;
  a.list_off = L->list_off;
  a.n = L->n;
  a.rec = L->record_len;
  a.psl = L->public_share_len;
  a.enc_len = L->enc_len;
  a.pay_len = L->payload_len;
  a.msg_len = L->message_len;
  a.ps_len = L->prep_share_len;
  a.cfg = d_config_ids;
  a.msg_status = d_msg_status;
  a.times = d_times;
  a.ct_len = d_ct_len;
  a.mismatch = d_mismatch;
  k_unpack_check<<<(L->n + 255) / 256, 256, 0, st>>>(a);
  DCHK(hipGetLastError());
  // field offsets within a record of the first record's shape
  const uint32_t o_pub = 28, o_enc = o_pub + L->public_share_len + 3,
                 o_pay = o_enc + L->enc_len + 4, o_ps = o_pay + L->payload_len + 4 + 5;
  GatherArgs g{};
  g.body = d_body;
  g.list_off = L->list_off;
  g.n = L->n;
  g.rec = L->record_len;
  g.f[0] = GatherField{d_report_ids, 16, 16, 0};
  g.f[1] = GatherField{L->public_share_len ? d_public_shares : nullptr, L->public_share_len,
                       L->public_share_len, o_pub};
  g.f[2] = GatherField{d_enc, L->enc_len, L->enc_len, o_enc};
  g.f[3] = GatherField{d_ct, ct_stride, L->payload_len, o_pay};
  g.f[4] = GatherField{L->prep_share_len ? d_prep_shares : nullptr, L->prep_share_len,
                       L->prep_share_len, o_ps};
  uint64_t maxw = 0;
  for (auto& f : g.f)
    if (f.dst && ((uint64_t)L->n * f.row + 3) / 4 > maxw) maxw = ((uint64_t)L->n * f.row + 3) / 4;
  const uint64_t blocks = (maxw + 255) / 256;
  k_unpack_gather<<<dim3((uint32_t)blocks, 5), 256, 0, st>>>(g);
  DCHK(hipGetLastError());
  return 0;
}

int64_t janus_dap_agg_init_unpack_host(const uint8_t* body, size_t len,
                                       const janus_dap_agg_init_layout* L, uint32_t cap,
                                       uint8_t* report_ids, uint64_t* times,
                                       uint8_t* public_shares, uint8_t* config_ids, uint8_t* enc,
                                       uint8_t* ct, uint32_t* ct_len, uint32_t ct_stride,
                                       uint8_t* prep_shares, uint8_t* msg_status) {
  if (!body || !L) return -1;
  Cur c{body, (size_t)(L->list_off + L->list_len), (size_t)L->list_off};
  uint32_t r = 0;
  while (c.o < c.len) {
    RecShape s;
    if (!parse_record(c, s)) return -1;
    if (r >= cap) return -1;
    memcpy(report_ids + 16 * (size_t)r, body + s.o_id, 16);
    times[r] = s.time;
    if (L->public_share_len) {
      uint8_t* pd = public_shares + (size_t)L->public_share_len * r;
      if (s.psl == L->public_share_len)
        memcpy(pd, body + s.o_pub, s.psl);
      else
        memset(pd, 0, L->public_share_len);
    }
    config_ids[r] = (uint8_t)s.cfg;
    uint8_t* ed = enc + (size_t)L->enc_len * r;
    if (s.enc_len == L->enc_len)
      memcpy(ed, body + s.o_enc, s.enc_len);
    else
      memset(ed, 0, L->enc_len);
    uint8_t* cd = ct + (size_t)ct_stride * r;
    memset(cd, 0, ct_stride);
    if (s.pay_len <= ct_stride && s.enc_len == L->enc_len) {
      memcpy(cd, body + s.o_pay, s.pay_len);
      ct_len[r] = s.pay_len;
    } else {
      ct_len[r] = 0;  // HPKE decrypt error for this report
    }
    // the PingPongMessage is decoded with the request: a malformed one rejects the request
    if (!pingpong_wellformed(body + s.o_msg, s.msg_len)) return -1;
    const uint32_t ty = body[s.o_msg];
    const uint32_t psl2 = be32(body + s.o_msg + 1);
    uint8_t stt = 0;
    if (s.psl != L->public_share_len)
      stt = 6;  // public share does not decode: InvalidMessage (aggregator.rs:1985-1999)
    else if (ty != 0)
      stt = 5;  // PeerMessageMismatch: Continue / Finish where Initialize is due
    else if (psl2 != L->prep_share_len)
      stt = 2;  // CodecPrepShare
    msg_status[r] = stt;
    uint8_t* pd = prep_shares + (size_t)L->prep_share_len * r;
    if (stt == 0)
      memcpy(pd, body + s.o_msg + 5, L->prep_share_len);
    else
      memset(pd, 0, L->prep_share_len);
    r++;
  }
  return r;
}

size_t janus_dap_agg_job_resp_max_len(uint32_t n, uint32_t pml) {
  return 4 + (size_t)n * (26 + pml > 18 ? 26 + pml : 18) + 8;
}

int janus_dap_agg_job_resp_encode_device(uint32_t n, const uint8_t* d_report_ids,
                                         const uint8_t* d_prepare_error,
                                         const uint8_t* d_prio3_status, const uint8_t* d_prep_msgs,
                                         uint32_t pml, uint8_t* d_out, uint64_t* d_out_len,
                                         uint32_t* d_scratch, void* stream) {
  if (!d_out || !d_out_len || !d_scratch || (n && (!d_report_ids || !d_prepare_error ||
                                                   !d_prio3_status || (pml && !d_prep_msgs))))
    return -1;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t nb = (n + 255) / 256;
  if (n) {
    k_resp_count<<<nb, 256, 0, st>>>(n, d_prepare_error, d_prio3_status, d_scratch);
    DCHK(hipGetLastError());
  }
  k_resp_scan<<<1, 1024, 0, st>>>(nb, d_scratch, n, pml, d_out_len, d_out);
  DCHK(hipGetLastError());
  if (n) {
    k_resp_write<<<nb, 256, 0, st>>>(n, d_report_ids, d_prepare_error, d_prio3_status,
                                     d_prep_msgs, pml, d_scratch, d_out);
    DCHK(hipGetLastError());
  }
  return 0;
}

int64_t janus_dap_agg_job_resp_encode_host(uint32_t n, const uint8_t* ids, const uint8_t* pe,
                                           const uint8_t* st, const uint8_t* pm, uint32_t pml,
                                           uint8_t* out) {
  if (!out) return -1;
  size_t o = 4;
  for (uint32_t r = 0; r < n; r++) {
    memcpy(out + o, ids + 16 * (size_t)r, 16);
    o += 16;
    if (pe[r] == 0xFF && st[r] == 0) {
      const uint32_t ml = 5 + pml;
      const uint8_t hdr[10] = {0, (uint8_t)(ml >> 24), (uint8_t)(ml >> 16), (uint8_t)(ml >> 8),
                               (uint8_t)ml, 2, (uint8_t)(pml >> 24), (uint8_t)(pml >> 16),
                               (uint8_t)(pml >> 8), (uint8_t)pml};
      memcpy(out + o, hdr, 10);
      if (pml) memcpy(out + o + 10, pm + (size_t)pml * r, pml);
      o += 10 + pml;
    } else {
      out[o] = 2;
      out[o + 1] = pe[r] != 0xFF ? pe[r] : 5;
      o += 2;
    }
  }
  const size_t body = o - 4;
  out[0] = (uint8_t)(body >> 24);
  out[1] = (uint8_t)(body >> 16);
  out[2] = (uint8_t)(body >> 8);
  out[3] = (uint8_t)body;
  return (int64_t)o;
}

}  // extern "C"
