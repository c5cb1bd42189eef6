// prio3_runtime.hip -- host runtime: per-GPU scratch slab pool, stream pool and the coalescing
// executor of the blocking host-buffer entry point (see prio3_runtime.h).
//
// Executor.  Janus prepares every aggregation job inside its own rayon::spawn
// (/root/reference/aggregator/src/aggregator.rs:2100-2123), so with C worker threads up to C
// jobs of 100-500 reports (binaries/aggregation_job_creator.rs:63-64) call
// prio3_helper_prepare_batch at once, possibly for different tasks (verify keys) of the same VDAF
// instance.  One 500-report device launch is latency-bound, so concurrent jobs are merged:
//   * a job reserves columns in the open group of its key (VDAF instance + options), copies its
//     inputs into that group's pinned, device-mapped staging itself (the copies run in parallel on
//     the callers' threads) and registers its verify key in the group's key table (one slot per
//     report);
//   * the executor's launcher thread takes a group as soon as the GPU can take it and all of its
//     writers are done -- so an idle GPU takes a lone job at once, and under load jobs pile into
//     the next group while the previous one runs (adaptive batching, no timer);
//   * the launch's kernels read the staged inputs over PCIe and write the outputs back into the
//     staging; every caller then copies its own outputs out and gets a batch handle that
//     references its column range of the shared device run.
#include "prio3_runtime.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/janus_prio3.h"
#include <dlfcn.h>
#include <emmintrin.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>

namespace {

constexpr int MAX_DEVICES = 64;

// ---- NUMA ---------------------------------------------------------------------------------
// the CPUs listed in a sysfs cpulist ("0-15,64-79")
std::vector<int> parse_cpulist(const char* path) {
  std::vector<int> cpus;
  FILE* f = fopen(path, "r");
  if (!f) return cpus;
  char buf[4096];
  const size_t m = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[m] = 0;
  for (char* q = buf; *q;) {
    char* e = nullptr;
    const long a = strtol(q, &e, 10);
    if (e == q) break;
    long b = a;
    if (*e == '-') {
      q = e + 1;
      b = strtol(q, &e, 10);
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; c++) cpus.push_back((int)c);
    q = e;
    while (*q == ',' || *q == '\n' || *q == ' ') q++;
  }
  return cpus;
}

// pins the calling thread to the CPUs of `device`'s NUMA node that the process may use (no-op
// when the node is unknown, or when those are all the CPUs it has -- e.g. a one-socket box)
void pin_to_gpu_node(int device) {
  const int node = gpu_numa_node(device);
  if (node < 0) return;
  char path[96];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  const std::vector<int> cpus = parse_cpulist(path);
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (cpus.empty() || sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
  for (int c : cpus)
    if (CPU_ISSET(c, &allowed)) CPU_SET(c, &want);
  if (CPU_COUNT(&want) == 0 || CPU_EQUAL(&want, &allowed)) return;
  (void)pthread_setaffinity_np(pthread_self(), sizeof want, &want);
}

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

// frees idle slabs (oldest first) until at most `keep` idle bytes remain, never `spare` (a slab
// its releaser asked to keep: a device-resident caller that re-acquires it on its next call -- an
// FPVec run is ~225 GB, and re-allocating it per step cost C5 40 % in r02j); caller holds p.mu.
// Without a spare the slab just released is the newest, so it goes only when it alone exceeds
// the budget (r05 kept it whatever its size: ~225 GB stayed reserved after one C5 batch).
void trim_locked(Pool& p, size_t keep, const Slab* spare = nullptr) {
  while (!p.idle.empty() && p.idle_bytes > keep && p.idle.front() != spare) {
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

int gpu_numa_node(int device) {
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  int node = -1;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, device) == hipSuccess) {
    for (char* c = bus; *c; c++) *c = (char)tolower((unsigned char)*c);
    char path[160];
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    if (FILE* f = fopen(path, "r")) {
      if (fscanf(f, "%d", &node) != 1) node = -1;
      fclose(f);
    }
  } else {
    (void)hipGetLastError();
  }
  cache[device] = node;
  return node;
}

int host_page_node(const void* p) {
  int node = -1;
  // get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR): the node of the page at p
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0UL, p, 3UL) != 0) return -1;
  return node;
}

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

void ws_release(Slab* s, hipStream_t st, bool keep) {
  if (!s) return;
  Pool& p = g_pools[s->device];
  s->pending = hipEventRecord(s->idle, st) == hipSuccess;
  if (!s->pending) (void)hipStreamSynchronize(st);
  std::lock_guard<std::mutex> lk(p.mu);
  p.idle.push_back(s);
  p.idle_bytes += s->bytes;
  trim_locked(p, p.budget, keep ? s : nullptr);
}

size_t ws_pool_bytes(int device, size_t* idle_bytes) {
  if (device < 0 || device >= MAX_DEVICES) return 0;
  Pool& p = g_pools[device];
  std::lock_guard<std::mutex> lk(p.mu);
  if (idle_bytes) *idle_bytes = p.idle_bytes;
  return p.total_bytes;
}

// frees every idle scratch slab of the device's pool (the C ABI's prio3_device_trim)
extern "C" int prio3_device_trim(int device) {
  if (device < 0 || device >= MAX_DEVICES) return PRIO3_EINVAL;
  Pool& p = g_pools[device];
  std::lock_guard<std::mutex> lk(p.mu);
  trim_locked(p, 0);
  return PRIO3_OK;
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
  DeviceGuard dg(device);
  if (dg.rc != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    return nullptr;
  return s;
}

void ws_stream_put(int device, hipStream_t s) {
  if (!s) return;
  StreamPool& sp = g_streams[device];
  std::lock_guard<std::mutex> lk(sp.mu);
  sp.free.push_back(s);
}

namespace {
struct QueuePool {
  std::mutex mu;
  std::vector<hipStream_t> own, free;  // the CU-masked streams made so far / idle ones
};
QueuePool g_queues[MAX_DEVICES];
// the idle CU-masked streams are destroyed at exit before the HIP runtime's own teardown (an exit
// handler registered after the runtime's runs first): under rocprofv3 a process that left them
// to the runtime crashed in __cxa_finalize (r05f).  A stream a launcher still holds (a group in
// flight at exit) is left to the runtime: the launcher may still query or synchronize it (ADVICE
// r5), and `closing` keeps it from being returned to a pool that is being torn down.
std::atomic<bool> g_queues_closing{false};
void destroy_queues() {
  g_queues_closing = true;
  for (int d = 0; d < MAX_DEVICES; d++) {
    QueuePool& qp = g_queues[d];
    std::lock_guard<std::mutex> lk(qp.mu);
    if (qp.free.empty()) continue;
    DeviceGuard dg(d);
    for (hipStream_t s : qp.free) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
      qp.own.erase(std::find(qp.own.begin(), qp.own.end(), s));
    }
    qp.free.clear();
  }
}
}  // namespace

hipStream_t ws_exec_stream_get(int device) {
  if (device < 0 || device >= MAX_DEVICES) return nullptr;
  QueuePool& qp = g_queues[device];
  {
    std::lock_guard<std::mutex> lk(qp.mu);
    if (!qp.free.empty()) {
      hipStream_t s = qp.free.back();
      qp.free.pop_back();
      return s;
    }
    if ((int)qp.own.size() < EXEC_QUEUE_STREAMS) {
      int cus = 0;
      hipStream_t s = nullptr;
      DeviceGuard dg(device);
      if (dg.rc == hipSuccess &&
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) ==
              hipSuccess &&
          cus > 0) {
        std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xffffffffu);
        if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
        if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
          static const int reg = std::atexit(destroy_queues);
          (void)reg;
          qp.own.push_back(s);
          return s;
        }
      }
      (void)hipGetLastError();
    }
  }
  return ws_stream_get(device);
}

void ws_exec_stream_put(int device, hipStream_t s) {
  if (!s) return;
  QueuePool& qp = g_queues[device];
  {
    std::lock_guard<std::mutex> lk(qp.mu);
    if (std::find(qp.own.begin(), qp.own.end(), s) != qp.own.end()) {
      if (!g_queues_closing) qp.free.push_back(s);
      return;
    }
  }
  ws_stream_put(device, s);
}

void ws_warm(int device) {
  if (device < 0 || device >= MAX_DEVICES) return;
  static std::once_flag once[MAX_DEVICES];
  std::call_once(once[device], [device] {
    hipStream_t s[WARM_STREAMS > EXEC_QUEUE_STREAMS ? WARM_STREAMS : EXEC_QUEUE_STREAMS] = {};
    for (int i = 0; i < WARM_STREAMS; i++) s[i] = ws_stream_get(device);
    for (int i = 0; i < WARM_STREAMS; i++) ws_stream_put(device, s[i]);
    for (int i = 0; i < EXEC_QUEUE_STREAMS; i++) s[i] = ws_exec_stream_get(device);
    for (int i = 0; i < EXEC_QUEUE_STREAMS; i++) ws_exec_stream_put(device, s[i]);
  });
}

// ---- executors -----------------------------------------------------------------------------
// A generic group-commit executor, one per (GPU, lane, work kind).  Callers reserve room in the
// open group of their key and stage their inputs themselves (in parallel); the executor's one
// launcher thread takes the oldest ready group -- or, when idle, the oldest open one -- waits for
// its writers, launches it and wakes exactly that group's callers.  An idle GPU therefore runs a
// lone job at once, and under load jobs pile into the next group while the launcher is busy.
namespace {

struct Staging {
  uint8_t* p = nullptr;    // inputs and outputs, as the job threads see them (pinned host memory)
  uint8_t* dev = nullptr;  // the same bytes as the device addresses them (kernels read per-report
                           // inputs straight from here and write outputs back: engine_group_issue)
  size_t bytes = 0;
  void* map = nullptr;  // huge-page staging: the mapping (hipHostRegister'ed at p) and its length
  size_t map_bytes = 0;
};

void staging_free(Staging& s) {
  if (s.map) {
    (void)hipHostUnregister(s.p);
    munmap(s.map, s.map_bytes);
  } else if (s.p) {
    (void)hipHostFree(s.p);
  }
  s = Staging();
}

constexpr size_t STAGING_TARGET = (size_t)96 << 20;  // pinned bytes per group (grows to fit)
// a leader group stages 5.7 KB per Histogram(256) report: 96 MB caps it at ~16k reports, half the
// helper's groups at the same load (A/B builds: JANUS_LEADER_STAGING_MB)
#ifndef JANUS_LEADER_STAGING_MB
#define JANUS_LEADER_STAGING_MB 96
#endif
constexpr size_t LEADER_STAGING_TARGET = (size_t)JANUS_LEADER_STAGING_MB << 20;

struct StagingPool {
  std::mutex mu;
  std::vector<Staging> idle;
  bool refilling = false;  // a spare is being allocated off the caller's path
};
StagingPool* g_staging = new StagingPool[MAX_DEVICES];  // never destroyed (see Exec)

// JANUS_STAGING_HUGE=0 (A/B): the staging from hipHostMalloc (4 KB pages) instead
bool staging_huge() {
  static const bool v = [] {
    const char* e = getenv("JANUS_STAGING_HUGE");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

// Pinned staging on 2 MB pages: an anonymous mapping on 2 MB boundaries with MADV_HUGEPAGE, bound
// to the GPU's NUMA node, faulted in, then registered with the GPU (mapped).  The leader's staging
// writes each report's 5.6 KB share transposed into [cell][report] form, one 16-byte cell into
// each of 352 rows ~1.5 MB apart: on 4 KB pages every cell is a TLB miss.  On the GPU box 16
// threads transposed 97 GB/s into 2 MB pages against 50 GB/s into 4 KB ones, and copied 113
// against 85 GB/s (tools/ubench_staging.cpp, profiles/r06/jobs/r06aa/).
Staging staging_alloc_huge(int dev, size_t bytes) {
  constexpr size_t H = (size_t)2 << 20;
  Staging s;
  s.bytes = (std::max(bytes, STAGING_TARGET) + H - 1) & ~(H - 1);
  s.map_bytes = s.bytes + H;
  void* m = mmap(nullptr, s.map_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return Staging();
  s.map = m;
  s.p = (uint8_t*)(((uintptr_t)m + H - 1) & ~(uintptr_t)(H - 1));
  (void)madvise(s.p, s.bytes, MADV_HUGEPAGE);
  // not inherited by a child (a subprocess started after the engine): a copy-on-write share of
  // the registered pages would make the driver re-validate the mapping when this process writes
  (void)madvise(s.p, s.bytes, MADV_DONTFORK);
  const int node = gpu_numa_node(dev);
  if (node >= 0 && node < 64) {  // MPOL_PREFERRED: the GPU's node first, any node if it is full
    const unsigned long mask = 1UL << node;
    (void)syscall(SYS_mbind, s.p, s.bytes, 1 /* MPOL_PREFERRED */, &mask, 64UL, 0U);
  }
  memset(s.p, 0, s.bytes);
  DeviceGuard dg(dev);
  const bool ok = dg.rc == hipSuccess &&
                  hipHostRegister(s.p, s.bytes, hipHostRegisterMapped) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    munmap(s.map, s.map_bytes);
    return Staging();
  }
  if (hipHostGetDevicePointer((void**)&s.dev, s.p, 0) != hipSuccess) {
    (void)hipGetLastError();
    staging_free(s);
  }
  return s;
}

Staging staging_alloc(int dev, size_t bytes) {
  if (staging_huge()) {
    Staging h = staging_alloc_huge(dev, bytes);
    if (h.p) return h;
  }
  Staging s;
  s.bytes = std::max(bytes, STAGING_TARGET);
  // pinned host memory of the GPU's own NUMA node: hipHostMalloc takes it from the pool of the
  // current device's nearest CPU agent (tests/test_gpu_executor.py::test_staging_on_gpu_numa_node)
  DeviceGuard dg(dev);
  const bool ok = dg.rc == hipSuccess &&
                  hipHostMalloc((void**)&s.p, s.bytes, hipHostMallocMapped) == hipSuccess &&
                  hipHostGetDevicePointer((void**)&s.dev, s.p, 0) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    staging_free(s);
  }
  return s;
}

// Takes an idle staging of at least `bytes`, or allocates one.  The executor calls this with its
// lock held when it opens a group, and a 96 MB hipHostMalloc takes ~13 ms: every job of the GPU
// then waited for it (r06q: a 12.8 ms gap in the 128-thread line, 36.0 -> 28.8 M reports/s).  So
// whenever the pool runs dry a spare of the same size is allocated on a thread of its own, and the
// next group finds it ready.
Staging staging_get(int dev, size_t bytes) {
  Staging s;
  size_t refill = 0;
  {
    std::lock_guard<std::mutex> lk(g_staging[dev].mu);
    auto& v = g_staging[dev].idle;
    for (size_t i = 0; i < v.size(); i++)
      if (v[i].bytes >= bytes) {
        s = v[i];
        v.erase(v.begin() + (long)i);
        break;
      }
    if (v.empty() && !g_staging[dev].refilling && !g_queues_closing) {
      g_staging[dev].refilling = true;
      refill = std::max(bytes, STAGING_TARGET);
    }
  }
  if (refill) {
    // a process that exits right after a job waits for a spare still being allocated (at most
    // 2 s), before the HIP runtime's own teardown (an exit handler registered after the runtime's
    // runs first)
    static std::once_flag once;
    std::call_once(once, [] {
      std::atexit([] {
        for (int i = 0; i < 2000; i++) {
          bool busy = false;
          for (int d = 0; d < MAX_DEVICES; d++) {
            std::lock_guard<std::mutex> lk(g_staging[d].mu);
            busy |= g_staging[d].refilling;
          }
          if (!busy) return;
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
      });
    });
    std::thread([dev, refill] {
      pin_to_gpu_node(dev);
      Staging r = g_queues_closing ? Staging() : staging_alloc(dev, refill);
      std::lock_guard<std::mutex> lk(g_staging[dev].mu);
      if (r.p) g_staging[dev].idle.push_back(r);
      g_staging[dev].refilling = false;
    }).detach();
  }
  return s.p ? s : staging_alloc(dev, bytes);
}

void staging_put(int dev, Staging s) {
  if (!s.p) return;
  std::lock_guard<std::mutex> lk(g_staging[dev].mu);
  auto& v = g_staging[dev].idle;
  v.push_back(s);
  if (v.size() > 8) {  // keep a few
    staging_free(v.front());
    v.erase(v.begin());
  }
}

constexpr uint32_t MAX_GROUP_REPORTS = 1u << 17;  // reports per prepare group
// an executor "hold" (tests queue jobs behind it) expires by itself: a caller that fails between
// hold = 1 and hold = 0 must not stall every engine sharing the executor forever
constexpr int64_t HOLD_MAX_MS = 30000;
// reports inside submit at which the launcher leaves its light-load pipeline (the box's 16 rayon
// threads keep ~8 Ki in flight, 128 threads ~64 Ki)
constexpr uint64_t HEAVY_DEFAULT = 32768;
// the heavy-load launcher's streams: 0 the plain pool (r05i), 1 the light pipeline's CU-masked
// streams, whose hardware queues are already active when the load crosses HEAVY_DEFAULT (the
// first heavy groups on idle plain queues stalled 7-20 ms, r06b / r06c kernel traces; interleaved
// r06d: 35.5 / 35.7 / 36.2 against 34.5 / 35.7 / 33.6 M reports/s at 128 threads)
#ifndef JANUS_HEAVY_OWN_QUEUE
#define JANUS_HEAVY_OWN_QUEUE 1
#endif
constexpr bool HEAVY_OWN_QUEUE = JANUS_HEAVY_OWN_QUEUE != 0;
// JANUS_COHORT_CAP=0 (A/B): no cap on a heavy-load group's share of the jobs (Exec::cohort_full)
bool cohort_cap() {
  static const bool v = [] {
    const char* s = getenv("JANUS_COHORT_CAP");
    return !(s && atoi(s) == 0);
  }();
  return v;
}

// JANUS_EXEC_TRACE=<path>: one line per launched group (microseconds: created, taken by the
// launcher, writers done, launch returned; jobs; reports), for tuning the executor
// (profiles/r03/r03t .. r03ab)
FILE* exec_trace() {
  static FILE* f = [] {
    const char* p = getenv("JANUS_EXEC_TRACE");
    return p ? fopen(p, "w") : (FILE*)nullptr;
  }();
  return f;
}
double exec_us(std::chrono::steady_clock::time_point t) {
  static const auto t0 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t - t0).count();
}
double ns_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t).count();
}

// JANUS_HOST_CPU=1: the job threads' CPU time in staging and unstaging per executor kind, printed
// to stderr at exit (where the jobs lines' host CPU goes)
bool host_cpu_on() {
  static const bool v = getenv("JANUS_HOST_CPU") != nullptr;
  return v;
}
double host_cpu_ns() {
  if (!host_cpu_on()) return 0;
  timespec t;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
  return t.tv_sec * 1e9 + t.tv_nsec;
}
std::atomic<uint64_t> g_host_cpu[8][3];  // per kind: stage ns, unstage ns, jobs
void host_cpu_add(int kind, double stage_ns, double unstage_ns) {
  static std::once_flag once;
  std::call_once(once, [] {
    std::atexit([] {
      static const char* names[] = {"prepare", "accumulate", "leader", "leader_next", "hpke"};
      for (int k = 0; k < 5; k++)
        if (const uint64_t n = g_host_cpu[k][2])
          fprintf(stderr, "janus host cpu: %s jobs %lu stage %.3f s unstage %.3f s (%.1f / %.1f us per job)\n",
                  names[k], (unsigned long)n, g_host_cpu[k][0] / 1e9, g_host_cpu[k][1] / 1e9,
                  g_host_cpu[k][0] / 1e3 / n, g_host_cpu[k][1] / 1e3 / n);
    });
  });
  g_host_cpu[kind][0] += (uint64_t)stage_ns;
  g_host_cpu[kind][1] += (uint64_t)unstage_ns;
  g_host_cpu[kind][2] += 1;
}

template <class P>
struct Exec {
  struct Group {
    uint64_t key = 0;
    typename P::State st;
    Staging stg;
    int writers = 0, readers = 0;
    bool closed = false, done = false;
    int rc = PRIO3_OK;
    std::chrono::steady_clock::time_point created, t_take, t_staged;
    int njobs = 0;
    std::condition_variable cv;
  };
  int device = 0, id = 0;
  std::mutex mu;
  std::condition_variable cv;  // the launcher
  std::map<uint64_t, Group*> open;
  std::deque<Group*> order;  // groups not yet taken by the launcher, oldest first
  bool started = false;
  // under mu:
  bool hold = false;  // exec_control "hold": take no group until hold_until at the latest
  std::chrono::steady_clock::time_point hold_until;
  uint64_t heavy_at = P::heavy_default();  // exec_control "heavy"
  ExecStats stats;

  bool holding() const { return hold && std::chrono::steady_clock::now() < hold_until; }
  // the launcher's wait for work (caller holds mu): a hold wakes it when it expires
  void wait_work(std::unique_lock<std::mutex>& lk) {
    if (hold)
      cv.wait_until(lk, hold_until);
    else
      cv.wait(lk);
  }

  void finish_locked(Group* g, int rc) {
    g->rc = rc;
    g->done = true;
    g->cv.notify_all();
  }
  bool takeable() const { return !order.empty() && !holding(); }
  // the oldest group, closed to later jobs, once its writers are done (caller holds mu)
  Group* take_locked(std::unique_lock<std::mutex>& lk) {
    Group* g = order.front();
    order.pop_front();
    if (!g->closed) {  // take an open group: no later job joins it
      g->closed = true;
      auto it = open.find(g->key);
      if (it != open.end() && it->second == g) open.erase(it);
    }
    g->t_take = std::chrono::steady_clock::now();
    while (g->writers > 0) g->cv.wait(lk);
    g->t_staged = std::chrono::steady_clock::now();
    return g;
  }
  // issues g with mu released; on failure its callers are woken with the error (returns false)
  // own_queue: the group's kernels on a hardware queue of their own (ws_exec_stream_get) -- the
  // light-load pipeline, whose groups are meant to run concurrently, and since r06 the heavy-load
  // launcher too (HEAVY_OWN_QUEUE; r05 had put it on the plain stream pool, r05i: 38.5-39.8 M/s
  // at 128 threads against 30.2-36.0 with dedicated queues, interleaved)
  bool issue_unlocked(std::unique_lock<std::mutex>& lk, Group* g, typename P::Handle* h,
                      bool own_queue) {
    lk.unlock();
    const int rc = P::issue(device, g->st, g->stg, h, own_queue);
    lk.lock();
    if (rc != PRIO3_OK) {
      finish_locked(g, rc);
      return false;
    }
    stats.groups++;
    return true;
  }
  void trace(const Group* g) {
    if (FILE* f = exec_trace())
      fprintf(f, "%.1f %.1f %.1f %.1f %d %u\n", exec_us(g->created), exec_us(g->t_take),
              exec_us(g->t_staged), exec_us(std::chrono::steady_clock::now()), g->njobs,
              P::reports(g->st));
  }

  // Light load vs heavy load (reports of the jobs inside submit): launcher_pipe() below
  // heavy_at, launcher() from there; launcher() hands back only below a third of it (between two
  // cohorts the callers of the finished group leave submit for a moment, and a handover there
  // cost the 128-thread line 10 %, r04z6).
  bool light() const { return stats.active_reports < heavy_at; }
  // Heavy load runs two cohorts of callers in turn: while one group runs, the callers it released
  // last fill the next.  Their sizes are whatever the start-up or a late caller made them, and they
  // persist: 41 / 87 jobs of the 128-thread line ran at 33.5 M reports/s, 58 / 68 at 37.6 (r06r).
  // A group open under heavy load takes at most about half the jobs inside submit, so a cohort
  // that is too big spills into the next group, which the other cohort then joins.
  bool cohort_full(const Group* g) const {
    return cohort_cap() && !light() && 2 * (uint64_t)g->njobs >= stats.active_jobs + 4;
  }
  bool lighter() const { return stats.active_reports < heavy_at / 3; }

  // Heavy load: one group on the GPU at a time.  While it runs, the launcher polls it; once its
  // prepare kernels are done, the next group -- by then holding the callers released by the
  // group before, all staged -- is issued behind it on its own stream, so the GPU does not idle
  // while this group's completion is noticed and the next launch is set up (r03y trace: 124 us
  // between groups).  The launcher must notice a group's 'prepared' event within microseconds,
  // but spinning through the whole ~0.7 ms group kept a core busy beside the staging writers
  // (ADVICE r3): it learns the prepare time per report from groups it watched complete while
  // spinning, and sleeps through the first 70 % of each later group (per group key: instances
  // of very different cost share the executor).  A sleep that overshoots (the group was already
  // prepared at the first poll) tells only an upper bound, so it shrinks the estimate instead of
  // feeding it (r04a: feeding it made the estimate hold itself up, 5.4 M reports/s).  `preds` is
  // the launcher thread's own table.  Returns (with nothing in flight) when the load turns light.
  struct Pred {
    double ns_per_report = 0;
    int seen = 0;
  };
  void launcher(std::map<uint64_t, Pred>& preds) {
    std::unique_lock<std::mutex> lk(mu);
    Group* cur = nullptr;
    typename P::Handle hc{};
    auto t0 = std::chrono::steady_clock::now();  // when cur could start
    for (;;) {
      if (!cur) {
        if (lighter()) return;
        while (!takeable()) wait_work(lk);
        Group* g = take_locked(lk);
        t0 = std::chrono::steady_clock::now();
        if (!issue_unlocked(lk, g, &hc, HEAVY_OWN_QUEUE)) continue;
        cur = g;
      }
      lk.unlock();
      Group* nxt = nullptr;
      typename P::Handle hn{};
      bool looked = false;
      auto tn = t0;  // when nxt was issued
      auto tp = t0;  // when cur was seen prepared (nxt's kernels start then)
      const uint32_t nrep = P::reports(cur->st);
      Pred& pr = preds[cur->key];
      bool just_slept = false;
      {  // sleep to 70 % of the predicted prepare time, less the timer slack (~60 us), <= 2 ms
        const double ns = std::min(2e6, 0.7 * pr.ns_per_report * nrep - 60e3 - ns_since(t0));
        if (pr.seen >= 2 && ns > 20e3) {
          std::this_thread::sleep_for(std::chrono::nanoseconds((int64_t)ns));
          just_slept = true;
        }
      }
      while (!P::done(hc)) {
        if (!looked && P::prepared(hc)) {
          looked = true;
          tp = std::chrono::steady_clock::now();
          const double x = nrep ? ns_since(t0) / nrep : 0;
          if (just_slept) {
            pr.ns_per_report *= 0.8;  // overslept: the elapsed time is only an upper bound
          } else {
            pr.ns_per_report = pr.seen ? std::min(x, 0.8 * pr.ns_per_report + 0.2 * x) : x;
            pr.seen++;
          }
          lk.lock();
          if (takeable() && order.front()->writers == 0 && !lighter()) {
            nxt = take_locked(lk);
            tn = std::chrono::steady_clock::now();
            if (!issue_unlocked(lk, nxt, &hn, HEAVY_OWN_QUEUE)) nxt = nullptr;
          }
          lk.unlock();
        }
        just_slept = false;
        std::this_thread::yield();
      }
      const int rc = P::finish(&hc);
      trace(cur);
      lk.lock();
      finish_locked(cur, rc);
      cur = nullptr;
      if (nxt) {
        cur = nxt;
        hc = hn;
        t0 = std::max(tn, tp);  // its prepare time counts from when its kernels could start
      }
    }
  }

  // Light load (the box's 16 rayon threads make groups of a few jobs, each a latency-bound kernel
  // at well under a wave per SIMD): up to four groups whose kernels run concurrently (no group
  // waits for another's prepare), each issued as soon as it is staged and holds >= 2 Ki reports
  // (smaller ones wait for an empty pipeline), any finished group completed at once: 10-15 M
  // reports/s at 16 threads against 5.6-7.6 M/s for launcher() on the same boxes (r04z).  Under
  // heavy load (the 128-thread line) launcher()'s two-cohort rhythm stays ahead (38.6-39.6 M/s
  // against 28-35 M/s for this pipeline, r04z2-4).  The pipeline yields between polls (a sleep's
  // timer slack would be a fifth of a small group's time).
  void launcher_pipe() {
    struct Slot {
      Group* g;
      typename P::Handle h;
    };
    std::deque<Slot> q;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      if (q.empty() && !light()) return;  // heavy load: launcher() from here
      while (takeable()) {
        Group* g = order.front();
        if (!q.empty()) {
          // heavy load: let the pipeline drain (one bubble) and hand over to launcher()
          if (g->writers > 0 || !light() || q.size() >= 4) break;
          if (P::reports(g->st) < 2048u) break;  // a small group waits for a drained pipeline
        }
        take_locked(lk);
        Slot sl{g, typename P::Handle{}};
        if (issue_unlocked(lk, g, &sl.h, true)) q.push_back(sl);
      }
      if (q.empty()) {
        while (!takeable() && light()) wait_work(lk);
        continue;
      }
      lk.unlock();
      bool any = false;
      for (size_t i = 0; i < q.size();) {
        if (P::done(q[i].h)) {
          Slot sl = q[i];
          q.erase(q.begin() + (long)i);
          const int rc = P::finish(&sl.h);
          trace(sl.g);
          std::lock_guard<std::mutex> lg(mu);
          finish_locked(sl.g, rc);
          any = true;
        } else {
          i++;
        }
      }
      if (!any) std::this_thread::yield();
      lk.lock();
    }
  }

  int submit(typename P::Job* job) {
    std::unique_lock<std::mutex> lk(mu);
    stats.jobs++;
    stats.reports += job->n;
    stats.active_jobs++;
    stats.active_reports += job->n;
    struct Done {  // runs with mu held: every return below holds lk
      ExecStats& s;
      uint32_t n;
      ~Done() {
        s.active_jobs--;
        s.active_reports -= n;
      }
    } done_{stats, job->n};
    if (!started) {  // one launcher thread per executor (never joined: see g_exec)
      started = true;
      std::thread([this] {
        pin_to_gpu_node(device);  // the launcher runs on its GPU's NUMA node
        std::map<uint64_t, Pred> preds;
        for (;;) {  // launcher() under heavy load, launcher_pipe() under light load
          launcher(preds);
          launcher_pipe();
        }
      }).detach();
    }
    // the load may have crossed heavy_at: a launcher waiting in light mode re-checks
    cv.notify_one();
    const uint64_t key = P::key(job);
    Group* g = nullptr;
    for (;;) {
      auto it = open.find(key);
      g = it == open.end() ? nullptr : it->second;
      if (g && !cohort_full(g) && P::reserve(g->st, job)) break;
      if (g) {  // full: it stays queued for the launcher as it is
        g->closed = true;
        open.erase(it);
      }
      g = new Group();
      g->key = key;
      size_t bytes = 0;
      if (!P::create(g->st, job, &bytes)) {
        delete g;
        return PRIO3_EINVAL;
      }
      g->stg = staging_get(device, bytes);
      if (!g->stg.p) {
        delete g;
        return PRIO3_EDEVICE;
      }
      g->created = std::chrono::steady_clock::now();
      open[key] = g;
      order.push_back(g);
      cv.notify_one();
      if (!P::reserve(g->st, job)) return PRIO3_EINVAL;  // cannot happen: sized for the job
      break;
    }
    g->writers++;
    g->readers++;
    g->njobs++;
    lk.unlock();
    const double c0 = host_cpu_ns();
    P::stage(g->st, g->stg, job);
    const double c1 = host_cpu_ns();
    lk.lock();
    if (--g->writers == 0) g->cv.notify_all();
    while (!g->done) g->cv.wait(lk);
    const int rc = g->rc;
    lk.unlock();
    const double c2 = host_cpu_ns();
    if (rc == PRIO3_OK) P::unstage(g->st, g->stg, job);
    if (host_cpu_on()) host_cpu_add(P::kind, c1 - c0, host_cpu_ns() - c2);
    lk.lock();
    if (--g->readers == 0) {
      staging_put(device, g->stg);
      delete g;
    }
    return rc;
  }

  int control(const char* key, int64_t value) {
    std::lock_guard<std::mutex> lk(mu);
    if (!strcmp(key, "hold")) {  // 1: at most HOLD_MAX_MS; v > 1: at most v ms
      hold = value != 0;
      hold_until = std::chrono::steady_clock::now() +
                   std::chrono::milliseconds(value > 1 ? value : HOLD_MAX_MS);
    } else if (!strcmp(key, "heavy")) {
      heavy_at = value > 0 ? (uint64_t)value : P::heavy_default();
    } else {
      return PRIO3_EINVAL;
    }
    cv.notify_all();
    return PRIO3_OK;
  }
  ExecStats get_stats() {
    std::lock_guard<std::mutex> lk(mu);
    return stats;
  }
};

// Copies into the pinned staging with non-temporal stores: the kernels read the staging over
// PCIe moments later, and lines left dirty in the writer's cache turn those reads into snoops
// of that cache (r03x: 34.5-36.8 M reports/s on the jobs line against 30.2-35.7 before, within
// the run-to-run spread).
void stream_copy(uint8_t* dst, const uint8_t* src, size_t n) {
  const size_t head = std::min(n, (size_t)((16 - ((uintptr_t)dst & 15)) & 15));
  memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128((const __m128i*)(src + i));
    const __m128i b = _mm_loadu_si128((const __m128i*)(src + i + 16));
    const __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32));
    const __m128i d = _mm_loadu_si128((const __m128i*)(src + i + 48));
    _mm_stream_si128((__m128i*)(dst + i), a);
    _mm_stream_si128((__m128i*)(dst + i + 16), b);
    _mm_stream_si128((__m128i*)(dst + i + 32), c);
    _mm_stream_si128((__m128i*)(dst + i + 48), d);
  }
  memcpy(dst + i, src + i, n - i);
  _mm_sfence();
}

// Rows of `cells` 16-byte cells (n reports from src) into the columns [c0, c0 + n) of a
// [cell][cap] staging array, with non-temporal stores: eight reports at a time, so each cell's
// stores fill two whole 64-byte lines and the eight source rows stream through the cache once.
void stream_transpose16(uint8_t* dst, size_t cap, size_t c0, const uint8_t* src, uint32_t n,
                        uint32_t cells) {
  const size_t row = 16 * (size_t)cells;
  for (uint32_t r0 = 0; r0 < n; r0 += 8) {
    const uint32_t k = std::min(8u, n - r0);
    const uint8_t* s0 = src + row * r0;
    for (uint32_t e = 0; e < cells; e++) {
      __m128i* d = (__m128i*)(dst + 16 * (e * cap + c0 + r0));
      for (uint32_t i = 0; i < k; i++)
        _mm_stream_si128(d + i, _mm_loadu_si128((const __m128i*)(s0 + row * i + 16 * (size_t)e)));
    }
  }
  _mm_sfence();
}

// ---- prepare groups ----
struct PrepPolicy {
  static constexpr int kind = 0;
  typedef ExecJob Job;
  static uint64_t heavy_default() { return HEAVY_DEFAULT; }
  struct State {
    prio3_engine* lead = nullptr;
    std::vector<const prio3_engine*> keys;  // verify-key table, slot = index
    std::vector<std::array<uint8_t, 32>> tasks;  // sealed-input groups: task-ID table, slot = index
    janus_hpke_opener* opener = nullptr;
    int require_taskprov = 0;
    uint32_t n = 0, cap = 0, jobs = 0, nseg = 0, align = 1;
    IoLayout L;
    Run* run = nullptr;
  };
  static uint64_t key(Job* j) { return exec_job_key(j); }
  static uint32_t reports(const State& s) { return s.n; }
  static bool create(State& s, Job* j, size_t* bytes) {
    s.lead = j->e;
    s.opener = j->opener;
    s.require_taskprov = j->require_taskprov;
    IoLayout l1, l2;
    engine_io_layout(j->e, 1, &l1, j);
    engine_io_layout(j->e, 2, &l2, j);
    const size_t per = l2.bytes - l1.bytes + 1;
    const uint32_t cap_b = (uint32_t)std::max<size_t>(1, STAGING_TARGET / per);
    s.align = engine_job_align(j->e);
    s.cap = std::max(j->n, std::min(MAX_GROUP_REPORTS, cap_b));
    s.cap = (s.cap + 63) & ~63u;  // room for the tail pad of a wave-aligned group
    engine_io_layout(j->e, s.cap, &s.L, j);
    *bytes = s.L.bytes;
    return true;
  }
  static bool reserve(State& s, Job* j) {
    uint32_t k = 0;
    while (k < s.keys.size() && s.keys[k] != j->e) k++;
    if (k == s.keys.size() && s.keys.size() >= exec_max_keys()) return false;
    uint32_t t = 0;
    if (j->opener) {
      while (t < s.tasks.size() && memcmp(s.tasks[t].data(), j->task_id, 32)) t++;
      if (t == s.tasks.size() && s.tasks.size() >= HPKE_MAX_TASKS) return false;
    }
    const uint32_t al = j->nseg ? s.align : 1u;
    const uint32_t c0 = (s.n + al - 1) / al * al;
    if (c0 + j->n > s.cap || ((c0 + j->n + 63) & ~63u) > s.cap ||
        s.nseg + j->nseg > s.L.max_seg)
      return false;
    if (k == s.keys.size()) s.keys.push_back(j->e);
    if (j->opener && t == s.tasks.size()) {
      std::array<uint8_t, 32> id;
      memcpy(id.data(), j->task_id, 32);
      s.tasks.push_back(id);
    }
    j->tslot = t;
    j->pad0 = s.n;
    j->c0 = c0;
    j->slot = k;
    j->seg0 = s.nseg;
    s.n = c0 + j->n;
    s.nseg += j->nseg;
    s.jobs++;
    return true;
  }
  // pad columns [a, b): verify-key slot 0, an out-of-range segment id, not accepted (their
  // prepare runs on whatever bytes the staging holds and is never returned)
  // (sealed-input groups: ciphertext length 0, which the open rejects at once, and task slot 0)
  static void pad(const IoLayout& L, Staging& g, uint32_t a, uint32_t b) {
    if (a >= b) return;
    memset(g.p + L.slot_off + 2 * (size_t)a, 0, 2 * (size_t)(b - a));
    memset(g.p + L.seg_off + 4 * (size_t)a, 0xff, 4 * (size_t)(b - a));
    memset(g.p + L.accept_off + a, 0, b - a);
    if (L.ct_stride) {
      memset(g.p + L.ctlen_off + 4 * (size_t)a, 0, 4 * (size_t)(b - a));
      memset(g.p + L.tslot_off + 2 * (size_t)a, 0, 2 * (size_t)(b - a));
    }
  }
  static void stage(State& s, Staging& g, Job* j) {
    const IoLayout& L = s.L;
    pad(L, g, j->pad0, j->c0);
    const uint8_t* src[4] = {j->nonces, j->pub, j->helper, j->leader};
    for (int f = 0; f < 4; f++)
      if (L.len[f] && src[f]) stream_copy(g.p + L.off[f] + L.len[f] * j->c0, src[f], L.len[f] * j->n);
    uint16_t* slots = (uint16_t*)(g.p + L.slot_off) + j->c0;
    for (uint32_t i = 0; i < j->n; i++) slots[i] = (uint16_t)j->slot;
    engine_vk(j->e, g.p + L.tab_off + 16 * (size_t)j->slot);
    if (L.ct_stride) {  // the sealed input shares and their AAD fields
      const size_t c0 = j->c0, n = j->n;
      stream_copy(g.p + L.enc_off + (size_t)L.nenc * c0, j->enc, (size_t)L.nenc * n);
      stream_copy(g.p + L.ct_off + (size_t)L.ct_stride * c0, j->ct, (size_t)L.ct_stride * n);
      memcpy(g.p + L.ctlen_off + 4 * c0, j->ct_len, 4 * n);
      memcpy(g.p + L.time_off + 8 * c0, j->times, 8 * n);
      uint16_t* ts = (uint16_t*)(g.p + L.tslot_off) + c0;
      for (uint32_t i = 0; i < j->n; i++) ts[i] = (uint16_t)j->tslot;
      uint32_t* tab = (uint32_t*)(g.p + L.ttab_off) + 8 * (size_t)j->tslot;
      for (int i = 0; i < 8; i++) {  // BE words, as the open kernel's AAD takes them
        const uint8_t* b = j->task_id + 4 * i;
        tab[i] = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
      }
    }
    // group segment ids: the job's own ids shifted to its segment range (an id >= its n_segments
    // stays out of every aggregate: 0xFFFFFFFF); a prepare-only job's reports are out
    uint32_t* sg = (uint32_t*)(g.p + L.seg_off) + j->c0;
    uint8_t* ac = g.p + L.accept_off + j->c0;
    if (j->nseg == 0) {
      for (uint32_t i = 0; i < j->n; i++) sg[i] = 0xFFFFFFFFu;
      memset(ac, 0, j->n);
    } else {
      for (uint32_t i = 0; i < j->n; i++) {
        const uint32_t x = j->seg ? j->seg[i] : 0u;
        sg[i] = x < j->nseg ? j->seg0 + x : 0xFFFFFFFFu;
      }
      if (j->accept)
        memcpy(ac, j->accept, j->n);
      else
        memset(ac, 1, j->n);
    }
  }
  struct Handle {
    GroupRun gr;
    State* s = nullptr;
  };
  static int issue(int device, State& s, Staging& g, Handle* h, bool own_queue) {
    (void)device;
    GroupView v;
    if (s.align > 1) {  // whole waves: the group's tail padded like the gaps
      const uint32_t n1 = (s.n + s.align - 1) / s.align * s.align;
      pad(s.L, g, s.n, n1);
      s.n = n1;
    }
    v.n = s.n;
    v.cap = s.cap;
    v.stg = g.p;
    v.stg_dev = g.dev;
    v.n_keys = (uint32_t)s.keys.size();
    v.jobs = (int)s.jobs;
    v.nseg = s.nseg;
    v.L = &s.L;
    v.opener = s.opener;
    v.require_taskprov = s.require_taskprov;
    h->s = &s;
    return engine_group_issue(s.lead, v, &h->gr, own_queue);
  }
  static bool prepared(const Handle& h) { return engine_group_prepared(h.gr); }
  static bool done(const Handle& h) { return engine_group_done(h.gr); }
  static int finish(Handle* h) { return engine_group_finish(&h->gr, &h->s->run); }
  static void unstage(State& s, Staging& g, Job* j) {
    const IoLayout& L = s.L;
    if (L.msg_len && j->msgs_out)
      memcpy(j->msgs_out, g.p + L.msg_off + L.msg_len * j->c0, L.msg_len * j->n);
    if (j->status_out) memcpy(j->status_out, g.p + L.status_off + j->c0, j->n);
    if (j->nseg) {
      memcpy(j->agg_out, g.p + L.agg_off + L.agg_len * j->seg0, L.agg_len * j->nseg);
      memcpy(j->counts_out, g.p + L.cnt_off + 8 * (size_t)j->seg0, 8 * (size_t)j->nseg);
    }
    j->run = s.run;  // one reference per job (engine_group_finish sets refs = jobs)
  }
};

// ---- accumulate groups ----
struct AccPolicy {
  static constexpr int kind = 1;
  typedef AccJob Job;
  static uint64_t heavy_default() { return HEAVY_DEFAULT; }
  static constexpr uint32_t MAX_JOBS = 1024, MAX_REPS = 1u << 17;
  static constexpr size_t MAX_OUT = (size_t)32 << 20;
  struct State {
    AccLayout L;
    uint32_t jobs = 0, reps = 0;
    size_t out = 0;
    int es = 16;
  };
  static uint64_t key(Job* j) { return (uint64_t)engine_acc_key(j); }
  static uint32_t reports(const State& s) { return s.reps; }
  static bool create(State& s, Job* j, size_t* bytes) {
    s.es = (int)engine_acc_key(j);
    const uint32_t reps = std::max(MAX_REPS, j->n);
    const size_t out = std::max(MAX_OUT, engine_acc_out_bytes(j));
    acc_layout(MAX_JOBS, reps, out, &s.L);
    *bytes = s.L.bytes;
    return true;
  }
  static bool reserve(State& s, Job* j) {
    const size_t ob = engine_acc_out_bytes(j);
    if (s.jobs + 1 > s.L.max_jobs || s.reps + j->n > s.L.max_reps || s.out + ob > s.L.out_cap)
      return false;
    j->slot = s.jobs++;
    j->rep_off = s.reps;
    j->out_off = s.out;
    s.reps += j->n;
    s.out += ob;
    return true;
  }
  static void stage(State& s, Staging& g, Job* j) { engine_acc_stage(j, g.p, s.L); }
  struct Handle {};  // the accumulate group runs to completion inside issue
  static int issue(int device, State& s, Staging& g, Handle*, bool) {
    return engine_acc_group(device, s.es, g.p, s.L, s.jobs, s.out);
  }
  static bool prepared(const Handle&) { return true; }
  static bool done(const Handle&) { return true; }
  static int finish(Handle*) { return PRIO3_OK; }
  static void unstage(State& s, Staging& g, Job* j) { engine_acc_unstage(j, g.p, s.L); }
};

// ---- leader prepare_init groups ----
struct LeaderPolicy {
  static constexpr int kind = 2;
  typedef LeaderJob Job;
  static uint64_t heavy_default() { return HEAVY_DEFAULT; }
  struct State {
    prio3_engine* lead = nullptr;
    std::vector<const prio3_engine*> keys;  // verify-key table, slot = index
    uint32_t n = 0, cap = 0, jobs = 0;
    LeaderLayout L;
    Run* run = nullptr;
  };
  // a different key space from the helper's groups: the executors are separate
  static uint64_t key(Job* j) { return engine_group_key(j->e); }
  static uint32_t reports(const State& s) { return s.n; }
  static bool create(State& s, Job* j, size_t* bytes) {
    s.lead = j->e;
    LeaderLayout l1, l2;
    engine_leader_layout(j->e, 1, &l1);
    engine_leader_layout(j->e, 2, &l2);
    const size_t per = l2.bytes - l1.bytes + 1;
    const uint32_t cap_b = (uint32_t)std::max<size_t>(1, LEADER_STAGING_TARGET / per);
    s.cap = std::max(j->n, std::min(MAX_GROUP_REPORTS, cap_b));
    engine_leader_layout(j->e, s.cap, &s.L);
    *bytes = s.L.bytes;
    return true;
  }
  static bool reserve(State& s, Job* j) {
    uint32_t k = 0;
    while (k < s.keys.size() && s.keys[k] != j->e) k++;
    if (k == s.keys.size() && s.keys.size() >= exec_max_keys()) return false;
    if (s.n + j->n > s.cap) return false;
    if (k == s.keys.size()) s.keys.push_back(j->e);
    j->c0 = s.n;
    j->slot = k;
    s.n += j->n;
    s.jobs++;
    return true;
  }
  static void stage(State& s, Staging& g, Job* j) {
    const LeaderLayout& L = s.L;
    const uint8_t* src[3] = {j->nonces, j->pub, j->linput};
    for (int f = 0; f < 3; f++) {
      if (!L.len[f] || !src[f]) continue;
      if (f == 2 && L.lin_soa)
        stream_transpose16(g.p + L.off[2], L.cap, j->c0, src[2], j->n, (uint32_t)(L.len[2] / 16));
      else
        stream_copy(g.p + L.off[f] + L.len[f] * j->c0, src[f], L.len[f] * j->n);
    }
    uint16_t* slots = (uint16_t*)(g.p + L.slot_off) + j->c0;
    for (uint32_t i = 0; i < j->n; i++) slots[i] = (uint16_t)j->slot;
    engine_vk(j->e, g.p + L.tab_off + 16 * (size_t)j->slot);
  }
  struct Handle {
    GroupRun gr;
    State* s = nullptr;
  };
  static int issue(int, State& s, Staging& g, Handle* h, bool own_queue) {
    h->s = &s;
    return engine_leader_issue(s.lead, s.L, g.p, g.dev, s.n, (uint32_t)s.keys.size(),
                               (int)s.jobs, &h->gr, own_queue);
  }
  static bool prepared(const Handle& h) { return engine_group_prepared(h.gr); }
  static bool done(const Handle& h) { return engine_group_done(h.gr); }
  static int finish(Handle* h) { return engine_group_finish(&h->gr, &h->s->run); }
  static void unstage(State& s, Staging& g, Job* j) {
    const LeaderLayout& L = s.L;
    memcpy(j->prep_out, g.p + L.ps_off + L.ps_len * j->c0, L.ps_len * j->n);
    memcpy(j->status_out, g.p + L.status_off + j->c0, j->n);
    j->run = s.run;  // one reference per job
  }
};

// ---- leader prepare_next groups ----
struct LNextPolicy {
  static constexpr int kind = 3;
  typedef LNextJob Job;
  static uint64_t heavy_default() { return HEAVY_DEFAULT; }
  struct State {
    LNextLayout L;
    uint32_t jobs = 0, reps = 0, max_n = 0, es = 16;
    uint32_t acc_jobs = 0;  // aggregating jobs (next + accumulate)
    size_t out = 0;
  };
  struct Handle {
    int device = 0;
    hipStream_t st = nullptr;
    Slab* slab = nullptr;  // the accumulate area on the device (aggregating jobs)
  };
  static uint64_t key(Job* j) { return engine_lnext_key(j); }
  static uint32_t reports(const State& s) { return s.reps; }
  static bool create(State& s, Job* j, size_t* bytes) {
    if (j->n > LNEXT_MAX_REPS || engine_lnext_out_bytes(j) > LNEXT_MAX_OUT) return false;
    s.es = engine_lnext_key(j);
    lnext_layout(&s.L);
    *bytes = s.L.bytes;
    return true;
  }
  static bool reserve(State& s, Job* j) {
    const size_t ob = engine_lnext_out_bytes(j);
    if (s.jobs + 1 > LNEXT_MAX_JOBS || s.reps + j->n > LNEXT_MAX_REPS ||
        s.out + ob > LNEXT_MAX_OUT)
      return false;
    j->slot = s.jobs++;
    j->rep_off = s.reps;
    s.reps += j->n;
    s.max_n = std::max(s.max_n, j->n);
    if (j->nseg) {
      j->acc_slot = s.acc_jobs++;
      j->out_off = s.out;
      s.out += ob;
    }
    return true;
  }
  static void stage(State& s, Staging& g, Job* j) { engine_lnext_stage(j, g.p, s.L); }
  static int issue(int device, State& s, Staging& g, Handle* h, bool own_queue) {
    h->device = device;
    return engine_lnext_issue(device, s.es, g.p, g.dev, s.L, s.jobs, s.max_n, s.acc_jobs, s.out,
                              &h->st, &h->slab, own_queue);
  }
  static bool prepared(const Handle& h) { return done(h); }
  static bool done(const Handle& h) { return hipStreamQuery(h.st) != hipErrorNotReady; }
  static int finish(Handle* h) {
    const hipError_t q = hipStreamSynchronize(h->st);
    if (h->slab) ws_release(h->slab, h->st);
    ws_exec_stream_put(h->device, h->st);
    return q == hipSuccess ? PRIO3_OK : PRIO3_EDEVICE;
  }
  static void unstage(State& s, Staging& g, Job* j) { engine_lnext_unstage(j, g.p, s.L); }
};

// ---- HPKE open groups ----
struct HpkePolicy {
  static constexpr int kind = 4;
  typedef HpkeJob Job;
  // never the heavy-load launcher: one wave's HPKE open is a long dependent chain, so a group
  // takes about as long at 31k reports as at 62k, and the light-load pipeline's concurrent groups
  // win (r05o, 128 threads: 20.6-23.4 against 13.8-13.9 M reports/s interleaved; the prepare and
  // leader executors lose the other way, 19.4-21.4 against 34.3-40.0 and 4.0-4.8 against 5.9-6.8)
  static uint64_t heavy_default() { return UINT64_MAX / 4; }
  struct State {
    HpkeJob proto;  // the group's opener and per-task constants (stride, share lengths)
    std::vector<std::array<uint8_t, 32>> tasks;  // task-ID table, slot = index
    uint32_t n = 0, cap = 0;
    HpkeLayout L;
  };
  struct Handle {
    int device = 0;
    hipStream_t st = nullptr;
    Slab* slab = nullptr;
  };
  static uint64_t key(Job* j) { return hpke_group_key(j); }
  static uint32_t reports(const State& s) { return s.n; }
  static bool create(State& s, Job* j, size_t* bytes) {
    s.proto = *j;
    HpkeLayout l1, l2;
    hpke_layout(j, 1, &l1);
    hpke_layout(j, 2, &l2);
    const size_t per = l2.pt_off - l1.pt_off + 1;
    const uint32_t cap_b = (uint32_t)std::max<size_t>(1, STAGING_TARGET / per);
    s.cap = std::max(j->n, std::min(MAX_GROUP_REPORTS, cap_b));
    hpke_layout(j, s.cap, &s.L);
    *bytes = s.L.pt_off;  // the staging holds everything but the device plaintext scratch
    return true;
  }
  static bool reserve(State& s, Job* j) {
    uint32_t k = 0;
    while (k < s.tasks.size() && memcmp(s.tasks[k].data(), j->task_id, 32)) k++;
    if (k == s.tasks.size() && s.tasks.size() >= HPKE_MAX_TASKS) return false;
    if (s.n + j->n > s.cap) return false;
    if (k == s.tasks.size()) {
      std::array<uint8_t, 32> t;
      memcpy(t.data(), j->task_id, 32);
      s.tasks.push_back(t);
    }
    j->c0 = s.n;
    j->slot = k;
    s.n += j->n;
    return true;
  }
  static void stage(State& s, Staging& g, Job* j) {
    const HpkeLayout& L = s.L;
    const size_t c0 = j->c0, n = j->n;
    stream_copy(g.p + L.off_enc + L.nenc * c0, j->enc, L.nenc * n);
    stream_copy(g.p + L.off_ct + (size_t)j->ct_stride * c0, j->ct, (size_t)j->ct_stride * n);
    memcpy(g.p + L.off_len + 4 * c0, j->ct_len, 4 * n);
    memcpy(g.p + L.off_ids + 16 * c0, j->ids, 16 * n);
    memcpy(g.p + L.off_times + 8 * c0, j->times, 8 * n);
    if (j->pub_len) memcpy(g.p + L.off_pub + (size_t)j->pub_len * c0, j->pubs, (size_t)j->pub_len * n);
    uint16_t* slots = (uint16_t*)(g.p + L.slot_off) + c0;
    for (uint32_t i = 0; i < j->n; i++) slots[i] = (uint16_t)j->slot;
    uint32_t* tab = (uint32_t*)(g.p + L.tab_off) + 8 * (size_t)j->slot;
    for (int i = 0; i < 8; i++) {  // BE words, as the kernel's AAD takes them
      const uint8_t* b = j->task_id + 4 * i;
      tab[i] = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
    }
  }
  static int issue(int device, State& s, Staging& g, Handle* h, bool own_queue) {
    h->device = device;
    return hpke_group_issue(s.proto, s.L, g.p, g.p, s.n, &h->st, &h->slab, own_queue);
  }
  static bool prepared(const Handle& h) { return done(h); }
  static bool done(const Handle& h) { return hipStreamQuery(h.st) != hipErrorNotReady; }
  static int finish(Handle* h) {
    const hipError_t q = hipStreamSynchronize(h->st);
    ws_release(h->slab, h->st);
    ws_exec_stream_put(h->device, h->st);
    return q == hipSuccess ? PRIO3_OK : PRIO3_EDEVICE;
  }
  static void unstage(State& s, Staging& g, Job* j) {
    const HpkeLayout& L = s.L;
    memcpy(j->shares_out, g.p + L.shares_off + (size_t)j->share_len * j->c0,
           (size_t)j->share_len * j->n);
    memcpy(j->status_out, g.p + L.status_off + j->c0, j->n);
  }
};

constexpr int N_EXEC = MAX_DEVICES * EXEC_LANES;

template <class P>
Exec<P>* make_execs() {  // never destroyed: launcher threads may wait on them at exit
  auto* x = new Exec<P>[N_EXEC];
  for (int i = 0; i < N_EXEC; i++) {
    x[i].id = i;
    x[i].device = i / EXEC_LANES;
  }
  return x;
}
Exec<PrepPolicy>* g_prep = make_execs<PrepPolicy>();
Exec<AccPolicy>* g_acc = make_execs<AccPolicy>();
Exec<LeaderPolicy>* g_lead = make_execs<LeaderPolicy>();
Exec<LNextPolicy>* g_lnext = make_execs<LNextPolicy>();
Exec<HpkePolicy>* g_hpke = make_execs<HpkePolicy>();

bool exec_id_ok(int id) { return id >= 0 && id < N_EXEC; }

}  // namespace

uint32_t exec_max_keys() { return 256; }

void acc_layout(uint32_t max_jobs, uint32_t max_reps, size_t out_cap, AccLayout* L) {
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  L->max_jobs = max_jobs;
  L->max_reps = max_reps;
  L->out_cap = out_cap;
  L->desc_off = 0;
  L->seg_off = up(sizeof(AccDesc) * (size_t)max_jobs);
  L->acc_off = L->seg_off + up(4 * (size_t)max_reps);
  L->out_off = L->acc_off + up((size_t)max_reps);
  L->bytes = L->out_off + up(out_cap);
}

int exec_submit(ExecJob* job) {
  const int id = engine_exec_id(job->e);
  if (!exec_id_ok(id)) return PRIO3_EINVAL;
  return g_prep[id].submit(job);
}

int exec_accumulate(AccJob* job) {
  if (job->device < 0 || job->device >= MAX_DEVICES) return PRIO3_EINVAL;
  return g_acc[job->device * EXEC_LANES].submit(job);
}

int exec_leader(LeaderJob* job) {
  const int id = engine_exec_id(job->e);
  if (!exec_id_ok(id)) return PRIO3_EINVAL;
  return g_lead[id].submit(job);
}

int exec_hpke(HpkeJob* job) {
  const int d = hpke_opener_device(job->o);
  if (d < 0 || d >= MAX_DEVICES) return PRIO3_EINVAL;
  return g_hpke[d * EXEC_LANES].submit(job);
}

int exec_leader_next(LNextJob* job) {
  if (job->device < 0 || job->device >= MAX_DEVICES) return PRIO3_EINVAL;
  return g_lnext[job->device * EXEC_LANES].submit(job);
}

void lnext_layout(LNextLayout* L) {
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  L->desc_off = 0;
  L->msg_off = up(sizeof(LNextDesc) * (size_t)LNEXT_MAX_JOBS);
  L->status_off = L->msg_off + up(16 * (size_t)LNEXT_MAX_REPS);
  L->acc_base = L->status_off + up((size_t)LNEXT_MAX_REPS);
  acc_layout(LNEXT_MAX_JOBS, LNEXT_MAX_REPS, LNEXT_MAX_OUT, &L->acc);
  L->bytes = L->acc_base + L->acc.bytes;
}

int exec_stats(int kind, int id, ExecStats* out) {
  if (!exec_id_ok(id) || !out) return PRIO3_EINVAL;
  switch (kind) {
    case EXEC_PREP: *out = g_prep[id].get_stats(); return PRIO3_OK;
    case EXEC_ACC: *out = g_acc[id].get_stats(); return PRIO3_OK;
    case EXEC_LEADER: *out = g_lead[id].get_stats(); return PRIO3_OK;
    case EXEC_LNEXT: *out = g_lnext[id].get_stats(); return PRIO3_OK;
    case EXEC_HPKE: *out = g_hpke[id].get_stats(); return PRIO3_OK;
    default: return PRIO3_EINVAL;
  }
}

int exec_control(int kind, int id, const char* key, int64_t value) {
  if (!exec_id_ok(id) || !key) return PRIO3_EINVAL;
  switch (kind) {
    case EXEC_PREP: return g_prep[id].control(key, value);
    case EXEC_ACC: return g_acc[id].control(key, value);
    case EXEC_LEADER: return g_lead[id].control(key, value);
    case EXEC_LNEXT: return g_lnext[id].control(key, value);
    case EXEC_HPKE: return g_hpke[id].control(key, value);
    default: return PRIO3_EINVAL;
  }
}

uint64_t exec_load(int id) {
  if (!exec_id_ok(id)) return 0;
  return g_prep[id].get_stats().active_reports + g_lead[id].get_stats().active_reports;
}

// ---- tracing -------------------------------------------------------------------------------
namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  bool on = false;
  Roctx() {
    const char* v = getenv("JANUS_ROCTX");
    if (!v || strcmp(v, "1") != 0) return;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                            "libroctx64.so.4", "libroctx64.so"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
      pop = (int (*)())dlsym(h, "roctxRangePop");
      if (push && pop) {
        on = true;
        return;
      }
    }
  }
};
Roctx& roctx() {
  static Roctx r;
  return r;
}
}  // namespace

TraceSpan::TraceSpan(const char* name) : on(roctx().on) {
  if (on) roctx().push(name);
}
TraceSpan::~TraceSpan() {
  if (on) roctx().pop();
}
bool trace_enabled() { return roctx().on; }
