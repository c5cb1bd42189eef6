// prio3_runtime.hip -- host runtime: per-GPU scratch slab pool, stream pool and the coalescing
// executor of the blocking host-buffer entry point (see prio3_runtime.h).
//
// Executor.  Janus prepares every aggregation job inside its own rayon::spawn
// (/root/reference/aggregator/src/aggregator.rs:2100-2123), so with C worker threads up to C
// jobs of 100-500 reports (binaries/aggregation_job_creator.rs:63-64) call
// prio3_helper_prepare_batch at once, possibly for different tasks (verify keys) of the same VDAF
// instance.  One 500-report device launch is latency-bound, so concurrent jobs are merged:
//   * a job reserves columns in the open group of its key (VDAF instance + options), copies its
//     inputs into that group's pinned staging itself (the copies run in parallel on the callers'
//     threads) and registers its verify key in the group's key table (one slot per report);
//   * a group is launched by one of its callers as soon as a launch slot is free (at most
//     `max_inflight` groups are in flight per GPU) and all of its writers are done -- so an idle
//     GPU takes a lone job at once, and under load jobs pile into the next group while the
//     previous one runs (adaptive batching, no timer);
//   * the launch is one H2D copy of the staged inputs, the prepare kernels over all columns, one
//     D2H copy of prepare messages + statuses; every caller then copies its own outputs back and
//     gets a batch handle that references its column range of the shared device run.
#include "prio3_runtime.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/janus_prio3.h"

namespace {

constexpr int MAX_DEVICES = 64;

// ---- slabs ----------------------------------------------------------------------------------
struct Pool {
  std::mutex mu;
  std::deque<Slab*> idle;  // oldest first
  size_t idle_bytes = 0, total_bytes = 0;
  size_t budget = 0;  // idle bytes kept; 0 = not yet initialised
};
Pool g_pools[MAX_DEVICES];

size_t round_slab(size_t b) {
  const size_t g = (size_t)2 << 20;  // 2 MiB
  return (b + g - 1) / g * g;
}

void free_slab(Slab* s) {
  if (s->idle) {
    (void)hipEventSynchronize(s->idle);
    (void)hipEventDestroy(s->idle);
  }
  (void)hipFree(s->base);
  delete s;
}

// frees idle slabs (oldest first) until at most `keep` idle bytes remain; caller holds p.mu
void trim_locked(Pool& p, size_t keep) {
  while (!p.idle.empty() && p.idle_bytes > keep) {
    Slab* s = p.idle.front();
    p.idle.pop_front();
    p.idle_bytes -= s->bytes;
    p.total_bytes -= s->bytes;
    free_slab(s);
  }
}

// ---- streams --------------------------------------------------------------------------------
struct StreamPool {
  std::mutex mu;
  std::vector<hipStream_t> free;
};
StreamPool g_streams[MAX_DEVICES];

}  // namespace

Slab* ws_acquire(int device, size_t bytes, hipStream_t st, int* rc) {
  if (device < 0 || device >= MAX_DEVICES) {
    *rc = PRIO3_EINVAL;
    return nullptr;
  }
  Pool& p = g_pools[device];
  if (bytes == 0) bytes = 256;
  {
    std::lock_guard<std::mutex> lk(p.mu);
    if (!p.budget) {
      size_t fr = 0, tot = 0;
      p.budget = hipMemGetInfo(&fr, &tot) == hipSuccess ? tot / 8 : ((size_t)8 << 30);
    }
    // best fit among idle slabs, at most 4x the request (a huge idle slab is not pinned down by
    // a small request)
    auto best = p.idle.end();
    for (auto it = p.idle.begin(); it != p.idle.end(); ++it)
      if ((*it)->bytes >= bytes && (*it)->bytes <= 4 * bytes + ((size_t)8 << 20) &&
          (best == p.idle.end() || (*it)->bytes < (*best)->bytes))
        best = it;
    if (best != p.idle.end()) {
      Slab* s = *best;
      p.idle.erase(best);
      p.idle_bytes -= s->bytes;
      if (s->pending && hipStreamWaitEvent(st, s->idle, 0) != hipSuccess) {
        *rc = PRIO3_EDEVICE;
        p.idle.push_back(s);
        p.idle_bytes += s->bytes;
        return nullptr;
      }
      *rc = PRIO3_OK;
      return s;
    }
  }
  const size_t want = round_slab(bytes);
  Slab* s = new Slab();
  s->device = device;
  s->bytes = want;
  hipError_t err = hipMalloc((void**)&s->base, want);
  if (err != hipSuccess) {  // make room: free every idle slab and try once more
    (void)hipGetLastError();
    {
      std::lock_guard<std::mutex> lk(p.mu);
      trim_locked(p, 0);
    }
    err = hipMalloc((void**)&s->base, want);
  }
  if (err != hipSuccess) {
    (void)hipGetLastError();
    fprintf(stderr, "janus_prio3: scratch slab of %zu bytes unavailable (%s)\n", want,
            hipGetErrorString(err));
    delete s;
    *rc = PRIO3_EDEVICE;
    return nullptr;
  }
  if (hipEventCreateWithFlags(&s->idle, hipEventDisableTiming) != hipSuccess) {
    (void)hipFree(s->base);
    delete s;
    *rc = PRIO3_EDEVICE;
    return nullptr;
  }
  {
    std::lock_guard<std::mutex> lk(p.mu);
    p.total_bytes += want;
  }
  *rc = PRIO3_OK;
  return s;
}

void ws_release(Slab* s, hipStream_t st) {
  if (!s) return;
  Pool& p = g_pools[s->device];
  s->pending = hipEventRecord(s->idle, st) == hipSuccess;
  if (!s->pending) (void)hipStreamSynchronize(st);
  std::lock_guard<std::mutex> lk(p.mu);
  p.idle.push_back(s);
  p.idle_bytes += s->bytes;
  trim_locked(p, p.budget);
}

size_t ws_pool_bytes(int device, size_t* idle_bytes) {
  if (device < 0 || device >= MAX_DEVICES) return 0;
  Pool& p = g_pools[device];
  std::lock_guard<std::mutex> lk(p.mu);
  if (idle_bytes) *idle_bytes = p.idle_bytes;
  return p.total_bytes;
}

hipStream_t ws_stream_get(int device) {
  if (device < 0 || device >= MAX_DEVICES) return nullptr;
  StreamPool& sp = g_streams[device];
  {
    std::lock_guard<std::mutex> lk(sp.mu);
    if (!sp.free.empty()) {
      hipStream_t s = sp.free.back();
      sp.free.pop_back();
      return s;
    }
  }
  hipStream_t s = nullptr;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    return nullptr;
  return s;
}

void ws_stream_put(int device, hipStream_t s) {
  if (!s) return;
  StreamPool& sp = g_streams[device];
  std::lock_guard<std::mutex> lk(sp.mu);
  sp.free.push_back(s);
}

// ---- executor -------------------------------------------------------------------------------
namespace {

struct Staging {
  uint8_t* p = nullptr;
  size_t bytes = 0;
};

struct Group {
  uint64_t key = 0;
  prio3_engine* lead = nullptr;
  std::vector<ExecJob*> jobs;
  std::vector<const prio3_engine*> keys;  // verify-key table, slot = index
  uint32_t n = 0, cap = 0;
  size_t per_in = 0, per_out = 0;  // bytes per report (inputs incl. slot, outputs)
  int writers = 0, readers = 0;
  bool closed = false, flushing = false, done = false;
  int rc = PRIO3_OK;
  Staging stg;
  size_t in_bytes = 0, out_bytes = 0, slot_off = 0, tab_off = 0;
  Run* run = nullptr;
};

struct Executor {
  std::mutex mu;
  std::condition_variable cv;
  std::map<uint64_t, Group*> open;
  std::vector<Staging> staging;  // idle pinned buffers
  int inflight = 0;
};
Executor g_exec[MAX_DEVICES];

int max_inflight() {
  static const int v = [] {
    const char* s = getenv("JANUS_PRIO3_MAX_INFLIGHT");
    const int x = s ? atoi(s) : 2;
    return x < 1 ? 1 : x;
  }();
  return v;
}
uint32_t max_group_reports() {
  static const uint32_t v = [] {
    const char* s = getenv("JANUS_PRIO3_GROUP_REPORTS");
    const long x = s ? atol(s) : (1L << 17);
    return (uint32_t)std::max(1L, x);
  }();
  return v;
}
constexpr size_t STAGING_TARGET = (size_t)96 << 20;  // pinned bytes per group (grows to fit)

Staging staging_get(Executor& X, size_t bytes) {  // caller holds X.mu
  for (size_t i = 0; i < X.staging.size(); i++)
    if (X.staging[i].bytes >= bytes) {
      Staging s = X.staging[i];
      X.staging.erase(X.staging.begin() + (long)i);
      return s;
    }
  Staging s;
  s.bytes = std::max(bytes, STAGING_TARGET);
  if (hipHostMalloc((void**)&s.p, s.bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    s.p = nullptr;
    s.bytes = 0;
  }
  return s;
}

void staging_put(Executor& X, Staging s) {  // caller holds X.mu
  if (!s.p) return;
  X.staging.push_back(s);
  if (X.staging.size() > 8) {  // keep a few
    (void)hipHostFree(X.staging.front().p);
    X.staging.erase(X.staging.begin());
  }
}

}  // namespace

uint32_t exec_max_keys() { return 256; }

int exec_submit(ExecJob* job) {
  prio3_engine* e = job->e;
  const int device = engine_device(e);
  if (device < 0 || device >= MAX_DEVICES) return PRIO3_EINVAL;
  Executor& X = g_exec[device];
  const uint64_t key = engine_group_key(e);
  std::unique_lock<std::mutex> lk(X.mu);
  Group* g = nullptr;
  uint32_t slot = 0;
  for (;;) {
    auto it = X.open.find(key);
    g = it == X.open.end() ? nullptr : it->second;
    if (g) {
      uint32_t s = 0;
      while (s < g->keys.size() && g->keys[s] != e) s++;
      const bool key_ok = s < g->keys.size() || g->keys.size() < exec_max_keys();
      if (key_ok && g->n + job->n <= g->cap) {
        if (s == g->keys.size()) g->keys.push_back(e);
        slot = s;
        break;
      }
      g->closed = true;  // full: launch it as is, open another
      X.open.erase(it);
      X.cv.notify_all();
      continue;
    }
    g = new Group();
    g->key = key;
    g->lead = e;
    IoLayout l1, l2;
    engine_io_layout(e, 1, &l1);
    engine_io_layout(e, 2, &l2);
    const size_t per = l2.bytes - l1.bytes + 1;
    const uint32_t cap_b = (uint32_t)std::max<size_t>(1, STAGING_TARGET / per);
    g->cap = std::max(job->n, std::min(max_group_reports(), cap_b));
    IoLayout L;
    engine_io_layout(e, g->cap, &L);
    g->stg = staging_get(X, L.bytes);
    if (!g->stg.p) {
      delete g;
      return PRIO3_EDEVICE;
    }
    g->keys.push_back(e);
    slot = 0;
    X.open[key] = g;
    break;
  }
  job->c0 = g->n;
  g->n += job->n;
  g->jobs.push_back(job);
  g->writers++;
  g->readers++;
  const uint32_t cap = g->cap;
  lk.unlock();

  // ---- stage this job's inputs (parallel across the callers' threads) ----
  IoLayout L;
  engine_io_layout(e, cap, &L);
  {
    const uint8_t* src[4] = {job->nonces, job->pub, job->helper, job->leader};
    for (int f = 0; f < 4; f++)
      if (L.len[f] && src[f])
        memcpy(g->stg.p + L.off[f] + L.len[f] * job->c0, src[f], L.len[f] * job->n);
    uint16_t* slots = (uint16_t*)(g->stg.p + L.slot_off) + job->c0;
    for (uint32_t i = 0; i < job->n; i++) slots[i] = (uint16_t)slot;
    engine_vk(e, g->stg.p + L.tab_off + 16 * (size_t)slot);
  }

  lk.lock();
  g->writers--;
  X.cv.notify_all();
  while (!g->done) {
    if (!g->flushing && (g->closed || X.inflight < max_inflight())) {
      g->flushing = true;
      if (!g->closed) {
        g->closed = true;
        auto it = X.open.find(key);
        if (it != X.open.end() && it->second == g) X.open.erase(it);
      }
      while (g->writers > 0) X.cv.wait(lk);
      while (X.inflight >= max_inflight()) X.cv.wait(lk);
      X.inflight++;
      GroupView v;
      v.n = g->n;
      v.cap = g->cap;
      v.stg = g->stg.p;
      v.n_keys = (uint32_t)g->keys.size();
      v.jobs = (int)g->jobs.size();
      lk.unlock();
      Run* run = nullptr;
      const int rc = engine_run_group(g->lead, v, &run);
      lk.lock();
      X.inflight--;
      g->rc = rc;
      g->run = run;
      g->done = true;
      X.cv.notify_all();
    } else {
      X.cv.wait(lk);
    }
  }
  const int rc = g->rc;
  Run* run = g->run;
  lk.unlock();

  // ---- copy this job's outputs back ----
  if (rc == PRIO3_OK) {
    if (L.msg_len && job->msgs_out)
      memcpy(job->msgs_out, g->stg.p + L.msg_off + L.msg_len * job->c0, L.msg_len * job->n);
    if (job->status_out) memcpy(job->status_out, g->stg.p + L.status_off + job->c0, job->n);
    job->run = run;  // one reference per job (engine_run_group sets refs = jobs)
  }
  lk.lock();
  if (--g->readers == 0) {
    staging_put(X, g->stg);
    delete g;
  }
  return rc;
}
