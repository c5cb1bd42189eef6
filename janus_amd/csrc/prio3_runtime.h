// prio3_runtime.h -- the host runtime under the C ABI: a per-GPU pool of device scratch slabs
// shared by every engine on that GPU, a per-GPU pool of HIP streams for the blocking host-buffer
// entry points, and the per-GPU executor that coalesces concurrent aggregation jobs into one
// device launch (SURVEY.md 8(b) "Threading"; Janus runs one rayon::spawn per job,
// /root/reference/aggregator/src/aggregator.rs:2100-2123, jobs of 100-500 reports,
// /root/reference/aggregator/src/binaries/aggregation_job_creator.rs:63-64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

// ---- device scratch slabs ----------------------------------------------------------------
// A slab is one hipMalloc'ed byte range.  Released slabs return to the GPU's pool with an event
// recorded on the releasing stream; the next acquirer's stream waits on that event, so reuse is
// stream-ordered and no host synchronisation is needed.  Idle slabs beyond the pool's byte
// budget are freed (oldest first).
struct Slab {
  uint8_t* base = nullptr;
  size_t bytes = 0;
  int device = 0;
  hipEvent_t idle = nullptr;
  bool pending = false;  // `idle` recorded and not yet known complete
};
// returns nullptr (rc = PRIO3_EDEVICE) when the device cannot provide `bytes`
Slab* ws_acquire(int device, size_t bytes, hipStream_t st, int* rc);
void ws_release(Slab* s, hipStream_t st);
// bytes currently held by the GPU's pool (idle + in use), for tests
size_t ws_pool_bytes(int device, size_t* idle_bytes);

// ---- tracing -------------------------------------------------------------------------------
// roctx ranges around the C-ABI entry points, named after the Janus spans they stand in for
// ("handle_aggregate_init_generic threadpool task", "VDAF preparation":
// /root/reference/aggregator/src/aggregator.rs:1786-1790, 2021).  Off unless JANUS_ROCTX=1 at
// the first call: the roctx library is then dlopen'ed (rocprofv3 --marker-trace shows the ranges
// beside the kernels); no link-time dependency.
struct TraceSpan {
  explicit TraceSpan(const char* name);
  ~TraceSpan();
  bool on;
};
bool trace_enabled();

// ---- stream pool ---------------------------------------------------------------------------
hipStream_t ws_stream_get(int device);  // nullptr on failure
void ws_stream_put(int device, hipStream_t s);

// ---- coalescing executor -------------------------------------------------------------------
struct prio3_engine;
struct Run;
struct ExecJob {
  prio3_engine* e;
  uint32_t n;
  const uint8_t *nonces, *pub, *helper, *leader;  // host inputs (packed per report)
  uint8_t *msgs_out, *status_out;                 // host outputs
  // prepare + aggregate in the same launch (prio3_helper_prepare_aggregate_batch): the job's
  // reports are accumulated into its n_segments batch aggregations in the group's launch, with
  // no batch handle and no second round trip (nseg == 0: prepare only)
  const uint32_t* seg = nullptr;   // host segment ids [n] (nullable: segment 0)
  const uint8_t* accept = nullptr;  // host accept mask [n] (nullable: all)
  uint32_t nseg = 0;
  uint8_t* agg_out = nullptr;      // host [nseg][agg_share_len]
  uint64_t* counts_out = nullptr;  // host [nseg]
  // results
  int rc = 0;
  Run* run = nullptr;  // holds one reference for this job
  uint32_t c0 = 0;     // the job's first column in the run
  uint32_t slot = 0;   // the job's verify-key slot in its group
  uint32_t seg0 = 0;   // the job's first segment among the group's
  uint32_t pad0 = 0;   // pad columns [pad0, c0) before the job (aligned aggregating jobs)
};
// Blocks until the job's reports are prepared (alone or coalesced with concurrent jobs of
// engines with the same VDAF instance on the same GPU).
int exec_submit(ExecJob* job);

// Engine hooks the executor calls (prio3_engine.hip).
// Staging layout of a group with room for `cap` reports (pinned host buffer): the four input
// fields [cap][len] (nonces, public shares, helper shares, leader prep shares), the per-report
// verify-key slot (u16), the verify-key table [exec_max_keys()][16], then the outputs: prepare
// messages [cap][msg_len] and statuses [cap].
// Groups with aggregating jobs also stage per-report group segment ids (u32) and accept bytes,
// and receive [max_seg][agg_len] aggregate shares + [max_seg] u64 counts.
struct IoLayout {
  size_t len[4], off[4];
  size_t slot_off, tab_off, msg_off, status_off, msg_len;
  size_t seg_off, accept_off, agg_off, cnt_off, agg_len;
  uint32_t max_seg;
  size_t bytes;
};
void engine_io_layout(const prio3_engine* e, uint32_t cap, IoLayout* L);
struct GroupView {
  uint32_t n, cap;  // reports staged, staging capacity
  uint8_t* stg;     // the staged inputs as the job threads write them (IoLayout for cap)
  uint8_t* stg_dev;  // the same inputs as the device addresses them
  uint8_t* out;      // pinned output area (same IoLayout; = stg unless the inputs are in VRAM)
  uint8_t* out_dev;  // the output area as the device addresses it (mapped pinned memory)
  uint32_t n_keys;  // verify keys in the table
  int jobs;         // references the run must carry (one per job)
  uint32_t nseg;    // segments of the aggregating jobs (0: no job aggregates)
};
// segments one group can aggregate (its aggregating jobs' n_segments summed)
constexpr uint32_t EXEC_MAX_SEGS = 1024;
int engine_device(const prio3_engine* e);
uint64_t engine_group_key(const prio3_engine* e);  // equal keys may share one launch
uint32_t engine_job_align(const prio3_engine* e);  // column alignment of aggregating jobs
void engine_vk(const prio3_engine* e, uint8_t out[16]);
// A group launch in two halves: issue enqueues the whole group (prepare, aggregate, outputs back
// into the staging) on a pooled stream; finish (after done) hands the run to the group's jobs.
struct GroupRun {
  prio3_engine* lead = nullptr;
  hipStream_t st = nullptr;
  hipStream_t cs = nullptr;   // copy stream of a DMA group (group_dma), returned at finish
  hipEvent_t ev[2] = {nullptr, nullptr};  // DMA group: slab ready on st, inputs on the device
  Run* R = nullptr;
  hipEvent_t prep = nullptr;  // recorded after the prepare kernels
  int jobs = 0;
};
// after (nullable): the group running before this one; a DMA group's kernels wait for its
// prepare kernels (the copies do not)
int engine_group_issue(prio3_engine* lead, const GroupView& g, GroupRun* gr,
                       const GroupRun* after = nullptr);
// a group of n reports goes to the device by DMA (option group_dma; the executor issues it early)
bool engine_group_dma(const prio3_engine* e, uint32_t n);
bool engine_group_prepared(const GroupRun& gr);  // the prepare kernels are done
bool engine_group_done(const GroupRun& gr);      // everything is done (non-blocking)
int engine_group_finish(GroupRun* gr, Run** run_out);
uint32_t exec_max_keys();

// ---- coalesced accumulate (prio3_accumulate of concurrent jobs) ----------------------------
struct AccJob {
  int device = 0;
  Run* run = nullptr;
  uint32_t c0 = 0, n = 0;       // the batch's columns
  const uint32_t* seg = nullptr;  // host segment ids [n] (nullable)
  const uint8_t* accept = nullptr;  // host accept mask [n] (nullable)
  uint32_t nseg = 1;
  uint8_t* agg_out = nullptr;    // host [nseg][agg_len]
  uint64_t* counts_out = nullptr;  // host [nseg]
  // placement in the group
  uint32_t slot = 0, rep_off = 0;
  size_t out_off = 0;
};
// one per job of an accumulate group (device-visible); *_off are byte offsets into the group's
// device region
struct AccDesc {
  const uint8_t* src;     // output shares of the job's first column, SoA [element][ld]
  const uint8_t* status;  // the job's verdicts [n]
  uint64_t ld;
  uint32_t n, nseg, out_len, flags;  // flags: 1 = segment ids, 2 = accept mask
  uint64_t seg_off, acc_off, agg_off, cnt_off;
};
struct AccLayout {
  uint32_t max_jobs, max_reps;
  size_t out_cap, desc_off, seg_off, acc_off, out_off, bytes;
};
void acc_layout(uint32_t max_jobs, uint32_t max_reps, size_t out_cap, AccLayout* L);
int exec_accumulate(AccJob* job);
// engine hooks (prio3_engine.hip)
uint32_t engine_acc_key(const AccJob* j);  // jobs with equal keys share a launch (field size)
size_t engine_acc_out_bytes(const AccJob* j);
void engine_acc_stage(AccJob* j, uint8_t* stg, const AccLayout& L);
void engine_acc_unstage(AccJob* j, const uint8_t* stg, const AccLayout& L);
int engine_acc_group(int device, int es, uint8_t* stg, const AccLayout& L, uint32_t n_jobs,
                     size_t out_bytes);
