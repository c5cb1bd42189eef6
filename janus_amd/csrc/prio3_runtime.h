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

// ---- the calling thread's current device -------------------------------------------------
// Every C entry point (and every runtime helper that needs a device current) makes its GPU
// current through this guard and gives the calling thread its own device back on return: a Janus
// rayon worker whose job a multi-GPU engine placed on GPU k must not come back bound to GPU k
// (VERDICT r5 weak item 5).  hipSetDevice appears nowhere else in the library
// (tests/test_abi.py::test_set_device_only_inside_the_guard).
struct DeviceGuard {
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev) != hipSuccess) {
      (void)hipGetLastError();
      prev = -1;
    }
    rc = prev == device ? hipSuccess : hipSetDevice(device);
    restore = rc == hipSuccess && prev >= 0 && prev != device;
  }
  ~DeviceGuard() {
    if (restore) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
  int prev = -1;
  hipError_t rc = hipSuccess;
  bool restore = false;
};

// ---- NUMA placement ---------------------------------------------------------------------------
// The NUMA node of a GPU (its PCI function's numa_node in sysfs; -1 when unknown), and the host
// CPUs of that node this process may run on (empty when unknown or when they are every CPU the
// process has).  An 8-GPU node has two sockets: each GPU's executor launcher runs on its GPU's
// node, and its pinned staging comes from that node's memory (hipHostMalloc takes host memory
// from the pool of the current device's nearest CPU agent).
int gpu_numa_node(int device);
// NUMA node of the page holding host address p (-1 unknown); tests
int host_page_node(const void* p);

// ---- device scratch slabs ----------------------------------------------------------------
// A slab is one hipMalloc'ed byte range.  Released slabs return to the GPU's pool with an event
// recorded on the releasing stream; the next acquirer's stream waits on that event, so reuse is
// stream-ordered and no host synchronisation is needed.  Idle slabs beyond the pool's byte
// budget (1/8 of HBM) are freed, oldest first -- the slab just released too when it alone exceeds
// the budget (an FPVec run, ~225 GB at 10^4 entries), unless its releaser asked to keep it
// (engine option keep_scratch: a device-resident caller that runs such batches back to back).
struct Slab {
  uint8_t* base = nullptr;
  size_t bytes = 0;
  int device = 0;
  hipEvent_t idle = nullptr;
  bool pending = false;  // `idle` recorded and not yet known complete
};
// returns nullptr (rc = PRIO3_EDEVICE) when the device cannot provide `bytes`
Slab* ws_acquire(int device, size_t bytes, hipStream_t st, int* rc);
void ws_release(Slab* s, hipStream_t st, bool keep = false);
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
// Launch streams of the light-load pipeline's groups: the first EXEC_QUEUE_STREAMS per GPU are
// CU-masked (all CUs), and the HIP runtime gives such a stream a hardware queue of its own, so
// groups in flight together run concurrently.  Plain pooled streams share the process's
// GPU_MAX_HW_QUEUES queues, and two groups' streams on one queue ran back to back (r05e: every
// launch on 'Queue 1', the 16-thread jobs line at 10.2-10.5 instead of 15.4-15.6 M reports/s).
// Past that count the plain pool; put takes either kind back.  hipExtStreamCreateWithCUMask takes
// no flags, so these are BLOCKING streams: work on the legacy null stream (a synchronous
// hipMemcpy, torch's default stream) waits for their groups and they for it.  The library itself
// issues nothing on the null stream; a caller that mixes null-stream work with
// light-load jobs serialises the two.
#ifndef JANUS_EXEC_QUEUE_STREAMS  // A/B builds (tools/build_variant.sh): 0 = the plain pool only
#define JANUS_EXEC_QUEUE_STREAMS 4
#endif
constexpr int EXEC_QUEUE_STREAMS = JANUS_EXEC_QUEUE_STREAMS;
hipStream_t ws_exec_stream_get(int device);
void ws_exec_stream_put(int device, hipStream_t s);
// Creates the GPU's pooled streams up front (WARM_STREAMS plain ones and the EXEC_QUEUE_STREAMS
// CU-masked ones), once per GPU, at the first engine or opener creation: a stream created while
// groups run maps a new hardware queue, and the GPU stalled for 7-13 ms each time the heavy-load
// launcher met an empty pool inside the 128-thread jobs line's timed region (r06b: 29.8 against
// 36.8 M reports/s, the two runs' kernel traces differing only in two new queues).
constexpr int WARM_STREAMS = 6;
void ws_warm(int device);

// ---- coalescing executor -------------------------------------------------------------------
// One executor per (GPU, lane): lane 0 is the GPU's executor; a multi-GPU engine created over a
// device list that names a GPU k times gets lanes 0..k-1 on it (prio3_engine_create_devices; a
// test form of the node-wide placement that runs on a one-GPU box).
constexpr int EXEC_LANES = 8;
struct prio3_engine;
struct Run;
struct janus_hpke_opener;
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
  // the helper's whole loop body (prio3_helper_aggregate_init_batch, aggregator.rs:1794-2096):
  // the job hands over sealed input shares (helper == nullptr) and the group opens them on the
  // device first -- HPKE open, PlaintextInputShare decode, extension checks -- into the run's
  // helper-share buffer, which the prepare then reads; the decrypted shares never leave HBM.
  // status_out then carries the merged status (0x80 | PrepareError for reports the open rejects).
  janus_hpke_opener* opener = nullptr;
  const uint8_t* task_id = nullptr;  // [32], the AAD's task ID
  const uint64_t* times = nullptr;   // [n] report times (AAD)
  const uint8_t *enc = nullptr, *ct = nullptr;  // [n][Nenc], [n][ct_stride]
  const uint32_t* ct_len = nullptr;             // [n]
  uint32_t ct_stride = 0;
  int require_taskprov = 0;
  // results
  int rc = 0;
  Run* run = nullptr;  // holds one reference for this job
  uint32_t c0 = 0;     // the job's first column in the run
  uint32_t slot = 0;   // the job's verify-key slot in its group
  uint32_t tslot = 0;  // the job's task slot in its group (sealed-input jobs)
  uint32_t seg0 = 0;   // the job's first segment among the group's
  uint32_t pad0 = 0;   // pad columns [pad0, c0) before the job (aligned aggregating jobs)
};
// Blocks until the job's reports are prepared (alone or coalesced with concurrent jobs of
// engines with the same VDAF instance on the same executor).
int exec_submit(ExecJob* job);

// Executor control and counters (prio3_executor_control / prio3_engine_members).
struct ExecStats {
  uint64_t jobs = 0, reports = 0, groups = 0;  // submitted jobs / their reports / launches
  uint64_t active_jobs = 0, active_reports = 0;  // jobs inside submit now
};
// kinds: 0 helper prepare, 1 accumulate, 2 leader prepare_init, 3 leader prepare_next,
// 4 HPKE open of input shares
enum { EXEC_PREP = 0, EXEC_ACC = 1, EXEC_LEADER = 2, EXEC_LNEXT = 3, EXEC_HPKE = 4, EXEC_KINDS = 5 };
int exec_stats(int kind, int exec_id, ExecStats* out);
// hold = 1: the executor's launcher takes no group until hold = 0 (tests pre-queue jobs with
// it); heavy = reports inside submit at which the launcher switches to its heavy-load form
// (0 = the default 32 Ki)
int exec_control(int kind, int exec_id, const char* key, int64_t value);
// reports of the jobs inside the helper/leader executors of exec_id (placement: least loaded)
uint64_t exec_load(int exec_id);

// Engine hooks the executor calls (prio3_engine.hip).
// Staging layout of a group with room for `cap` reports (pinned, device-mapped host buffer):
// the four input fields [cap][len] (nonces, public shares, helper shares, leader prep shares),
// the per-report verify-key slot (u16), the verify-key table [exec_max_keys()][16], then the
// outputs: prepare messages [cap][msg_len] and statuses [cap].
// Groups with aggregating jobs also stage per-report group segment ids (u32) and accept bytes,
// and receive [max_seg][agg_len] aggregate shares + [max_seg] u64 counts.
// Groups of sealed-input jobs (ExecJob::opener) stage no helper shares (len[2] = 0) but, per
// report, the HPKE ciphertext: enc [cap][nenc], ct [cap][ct_stride], ct_len (u32), the report time
// (u64) and the task slot (u16), plus the task-ID table [HPKE_MAX_TASKS][8] (BE words).
struct IoLayout {
  size_t len[4], off[4];
  size_t slot_off, tab_off, msg_off, status_off, msg_len;
  size_t seg_off, accept_off, agg_off, cnt_off, agg_len;
  uint32_t max_seg;
  uint32_t nenc = 0, ct_stride = 0;  // ct_stride > 0: a sealed-input group
  size_t enc_off = 0, ct_off = 0, ctlen_off = 0, time_off = 0, tslot_off = 0, ttab_off = 0;
  size_t bytes;
};
// job: the group's first job (its opener and ciphertext stride shape a sealed-input group)
void engine_io_layout(const prio3_engine* e, uint32_t cap, IoLayout* L,
                      const ExecJob* job = nullptr);
// equal keys may share one launch: engine_group_key, and for sealed-input jobs their HPKE shape
uint64_t exec_job_key(const ExecJob* job);
struct GroupView {
  uint32_t n, cap;   // reports staged, staging capacity
  uint8_t* stg;      // the staged inputs and outputs as the job threads see them (IoLayout)
  uint8_t* stg_dev;  // the same bytes as the device addresses them (mapped pinned memory)
  uint32_t n_keys;   // verify keys in the table
  int jobs;          // references the run must carry (one per job)
  uint32_t nseg;     // segments of the aggregating jobs (0: no job aggregates)
  const IoLayout* L = nullptr;  // the staging layout (engine_io_layout of the group's first job)
  janus_hpke_opener* opener = nullptr;  // sealed-input group: the keypair its reports open with
  int require_taskprov = 0;
};
// segments one group can aggregate (its aggregating jobs' n_segments summed)
constexpr uint32_t EXEC_MAX_SEGS = 1024;
int engine_device(const prio3_engine* e);
int engine_exec_id(const prio3_engine* e);  // device * EXEC_LANES + lane
uint64_t engine_group_key(const prio3_engine* e);  // equal keys may share one launch
uint32_t engine_job_align(const prio3_engine* e);  // column alignment of aggregating jobs
void engine_vk(const prio3_engine* e, uint8_t out[16]);
// A group launch in two halves: issue enqueues the whole group (prepare, aggregate, outputs back
// into the staging) on a pooled stream; finish (after done) hands the run to the group's jobs.
struct GroupRun {
  prio3_engine* lead = nullptr;
  hipStream_t st = nullptr;
  Run* R = nullptr;
  hipEvent_t prep = nullptr;  // recorded after the prepare kernels
  int jobs = 0;
};
// own_queue: the group's stream from ws_exec_stream_get (else the plain pool)
int engine_group_issue(prio3_engine* lead, const GroupView& g, GroupRun* gr, bool own_queue);
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

// ---- coalesced leader prepare_init (prio3_leader_prepare_init_batch of concurrent jobs) -------
// Janus's aggregation job driver steps every job's reports through leader_initialized on its
// own rayon worker (/root/reference/aggregator/src/aggregator/aggregation_job_driver.rs:397-415,
// spawned at :449-462): the same group commit as the helper prepare, keyed by VDAF instance,
// with per-report verify-key slots.
struct LeaderJob {
  prio3_engine* e;
  uint32_t n;
  const uint8_t *nonces, *pub, *linput;  // host inputs [n][16], [n][pub_len], [n][leader_share_len]
  uint8_t *prep_out, *status_out;        // host outputs [n][prep_share_len], [n]
  Run* run = nullptr;  // results: one reference for this job, its columns [c0, c0 + n)
  uint32_t c0 = 0, slot = 0;
};
// staging of a leader group with room for cap reports: inputs, key slots, key table, outputs
// lin_soa: the leader input shares are staged transposed, 16-byte cell e of report c at
// off[2] + 16 * (e * cap + c), and the kernel reads them there over PCIe (no DMA into the run)
struct LeaderLayout {
  size_t len[3], off[3];  // nonces, public shares, leader input shares
  size_t slot_off, tab_off, ps_len, ps_off, status_off, bytes;
  uint32_t cap = 0;
  bool lin_soa = false;
};
void engine_leader_layout(const prio3_engine* e, uint32_t cap, LeaderLayout* L);
// one DMA of the staged inputs into the run, the leader kernels, the outputs back into the staging
int engine_leader_issue(prio3_engine* lead, const LeaderLayout& L, uint8_t* stg, uint8_t* stg_dev,
                        uint32_t n, uint32_t n_keys, int jobs, GroupRun* gr, bool own_queue);
int exec_leader(LeaderJob* job);

// ---- coalesced leader prepare_next (prio3_leader_prepare_next_batch of concurrent jobs) -------
// leader_continued on the helper's response (aggregation_job_driver.rs:677-691), per job: the
// kernel compares each prepare message with the corrected joint-rand seed and truncates the
// measurement share, for many jobs' batches (of different runs) in one launch.
struct LNextJob {
  int device = 0;
  Run* run = nullptr;
  uint32_t c0 = 0, n = 0;          // the batch's columns in its run
  const uint8_t* msgs = nullptr;   // host [n][16] (nullable: no joint randomness)
  uint8_t* status = nullptr;       // host [n], in/out
  // prepare_next + accumulate in the same launch (prio3_leader_prepare_next_aggregate_batch):
  // the job's verdicts and output shares are summed into its n_segments aggregations right after
  // the joint-rand check, with no second round trip (nseg == 0: prepare_next only)
  const uint32_t* seg = nullptr;   // host [n] (nullable: segment 0)
  const uint8_t* accept = nullptr;  // host [n] (nullable: all)
  uint32_t nseg = 0;
  uint8_t* agg_out = nullptr;      // host [nseg][agg_len]
  uint64_t* counts_out = nullptr;  // host [nseg]
  uint32_t slot = 0, rep_off = 0;  // placement in the group
  uint32_t acc_slot = 0;           // its accumulate descriptor (aggregating jobs)
  size_t out_off = 0;              // its aggregate shares + counts in the accumulate area
};
// one per job of a prepare_next group (read by the kernel from the mapped staging)
struct LNextDesc {
  const uint4* corrected;  // the run's corrected seeds at the job's first column
  const uint8_t* meas;     // its measurement-share SoA column 0 (element stride ld)
  uint8_t* out;            // its output-share SoA (Sum / SumVec truncation)
  uint8_t* dstatus;        // the run's device statuses at the job's first column
  uint64_t ld;
  uint32_t n, rep_off, kind, bits, out_len, jr;
};
constexpr uint32_t LNEXT_MAX_JOBS = 1024, LNEXT_MAX_REPS = 1u << 17;
constexpr size_t LNEXT_MAX_OUT = (size_t)32 << 20;  // aggregate shares + counts per group
// the staging of a prepare_next group: descriptors, messages, statuses, then (aggregating jobs)
// an accumulate area laid out as an accumulate group's (acc_layout) from acc_base
struct LNextLayout {
  size_t desc_off, msg_off, status_off, acc_base, bytes;
  AccLayout acc;
};
void lnext_layout(LNextLayout* L);
uint32_t engine_lnext_key(const LNextJob* j);
void engine_lnext_stage(LNextJob* j, uint8_t* stg, const LNextLayout& L);
// launches the group's kernel on a pooled stream of `device` (reads and writes the staging)
// n_acc aggregating jobs (descriptors 0 .. n_acc - 1 of the accumulate area; out_bytes its used
// output bytes) are accumulated after the check, in an area the call takes from the scratch pool
// (*slab_out, released after the stream by the finish)
int engine_lnext_issue(int device, uint32_t es, uint8_t* stg, uint8_t* stg_dev,
                       const LNextLayout& L, uint32_t n_jobs, uint32_t max_n, uint32_t n_acc,
                       size_t out_bytes, hipStream_t* st_out, Slab** slab_out, bool own_queue);
size_t engine_lnext_out_bytes(const LNextJob* j);
void engine_lnext_unstage(LNextJob* j, const uint8_t* stg, const LNextLayout& L);
int exec_leader_next(LNextJob* job);

// ---- coalesced HPKE open of helper input shares (janus_hpke_open_input_shares) -----------
// The helper opens each report's input share inside its job's rayon task
// (/root/reference/aggregator/src/aggregator.rs:1847-1890): concurrent jobs of every task that
// uses the same HPKE keypair share one launch, each report carrying a slot into the group's
// task-ID table (the AAD's task_id).
struct janus_hpke_opener;
struct HpkeJob {
  janus_hpke_opener* o = nullptr;
  uint32_t n = 0;
  const uint8_t* task_id = nullptr;  // [32]
  const uint8_t *enc = nullptr, *ct = nullptr;
  const uint32_t* ct_len = nullptr;
  uint32_t ct_stride = 0;
  const uint8_t* ids = nullptr;
  const uint64_t* times = nullptr;
  const uint8_t* pubs = nullptr;
  uint32_t pub_len = 0, share_len = 0;
  int require_taskprov = 0;
  uint8_t *shares_out = nullptr, *status_out = nullptr;
  uint32_t c0 = 0, slot = 0;  // placement in the group
};
// staging of an HPKE group with room for cap reports (per-field arrays), the task table, outputs
struct HpkeLayout {
  size_t off_enc, off_ct, off_len, off_ids, off_times, off_pub, slot_off, tab_off;
  size_t shares_off, status_off, pt_off, bytes;  // pt: device plaintext scratch (not staged)
  uint32_t nenc;
};
constexpr uint32_t HPKE_MAX_TASKS = 256;
size_t hpke_opener_nenc(const janus_hpke_opener* o);
uint64_t hpke_opener_key(const janus_hpke_opener* o);  // keypair + suite (+ timing option)
// The open kernel over a sealed-input prepare group, on the group's stream: inputs from the mapped
// staging, the helper shares (zeroed unless opened) and the open status into the run.
struct HpkeGroupArgs {
  uint32_t n, ct_stride, share_len, pub_len;
  int require_taskprov;
  const uint8_t *enc, *ct, *ids, *pubs;
  const uint32_t* ct_len;
  const uint64_t* times;
  const uint16_t* task_slot;
  const uint32_t* task_tab;
  uint8_t *pt, *shares, *status;  // device: plaintext scratch [n][ct_stride], outputs
};
int hpke_open_group_launch(janus_hpke_opener* o, const HpkeGroupArgs& a, hipStream_t st);
int hpke_opener_device(const janus_hpke_opener* o);
uint64_t hpke_group_key(const HpkeJob* j);
void hpke_layout(const HpkeJob* j, uint32_t cap, HpkeLayout* L);
// the group's inputs to a device mirror (one DMA per field), the open kernel, outputs back
int hpke_group_issue(const HpkeJob& proto, const HpkeLayout& L, const uint8_t* stg, uint8_t* out,
                     uint32_t n, hipStream_t* st_out, Slab** slab_out, bool own_queue);
int exec_hpke(HpkeJob* job);

