// jobs_driver.cpp -- measurement harness for the production call shape (bench.py --role jobs):
// C host threads, each playing one Janus rayon worker that runs whole aggregation jobs
// (/root/reference/aggregator/src/aggregator.rs:2100-2123) of `job_size` reports
// (binaries/aggregation_job_creator.rs:63-64, default 100-500), calling the C ABI exactly as the
// FFI crate of INTEGRATION.md would: prio3_helper_prepare_batch (host buffers, PCIe included),
// then prio3_accumulate into the job's batch aggregation, then prio3_batch_free.  The leader and
// HPKE forms do the same for the leader's prepare_init / prepare_next
// (aggregation_job_driver.rs:397-415, 677-691, spawned per job at :449-462) and the helper's
// input-share open (aggregator.rs:1847-1890).
// Not part of the engine: a separate library (libjanus_jobs.so) that links libjanus_prio3.so.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/janus_hpke.h"
#include "../../include/janus_prio3.h"

namespace {
// A persistent pool, as Janus's rayon pool is (aggregator/src/binary_utils.rs:514-518): its
// threads are created by the first call that needs them (the lines' warmup run) and parked on a
// condition variable between calls, so a timed call neither creates threads nor pays each new
// thread's first HIP calls.  r06 timed 128 fresh threads per call: their creation added 4-9 ms to
// a ~55 ms region (r06o), and spinning while parked burnt CPU quota (r06v).
struct Pool {
  std::mutex mu;
  std::condition_variable cv, done;
  std::function<void()> work;
  uint64_t gen = 0;
  int threads = 0, want = 0, active = 0;
};
Pool& pool() {
  static Pool* p = new Pool();  // never destroyed: its threads stay parked until exit
  return *p;
}

// `threads` workers taking jobs 0..jobs-1 in order; returns elapsed seconds (< 0: a call failed)
template <class F>
double run_pool(int threads, int jobs, F job) {
  Pool& P = pool();
  std::atomic<int> next{0}, failed{0};
  std::unique_lock<std::mutex> lk(P.mu);
  while (P.threads < threads) {
    const int idx = P.threads++;
    std::thread([&P, idx] {
      uint64_t seen = 0;
      std::unique_lock<std::mutex> l(P.mu);
      for (;;) {
        P.cv.wait(l, [&] { return P.gen != seen; });
        seen = P.gen;
        if (idx >= P.want) continue;
        const std::function<void()> w = P.work;
        l.unlock();
        w();
        l.lock();
        if (--P.active == 0) P.done.notify_all();
      }
    }).detach();
  }
  P.work = [&] {
    for (;;) {
      const int j = next.fetch_add(1);
      if (j >= jobs) return;
      if (!job(j)) failed = 1;
    }
  };
  P.want = threads;
  P.active = threads;
  P.gen++;
  const auto t0 = std::chrono::steady_clock::now();
  P.cv.notify_all();
  P.done.wait(lk, [&] { return P.active == 0; });
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  P.work = nullptr;
  return failed ? -1.0 : dt;
}
}  // namespace

extern "C" {

// engines[n_engines] (tasks of one VDAF instance, sizes *szp); one report pool per engine (its
// own verify key): nonces[n_engines * pool][16], pub[..][psl], helper[..][hsl], lps[..][L].  Job j
// runs on engine t = j % n_engines over `job_size` consecutive reports of pool t starting at
// ((j / n_engines) * job_size) % (pool - job_size + 1).  status_out[jobs * job_size],
// counts_out[jobs] and agg_out[jobs][agg_len] receive every job's verdicts, count and aggregate
// share.  combined = 0: prio3_helper_prepare_batch + prio3_accumulate + prio3_batch_free per job
// (two round trips through the executor); 1: prio3_helper_prepare_aggregate_batch (one).
// Returns elapsed seconds (< 0: a call failed).
double janus_jobs_run(prio3_engine** engines, int n_engines, const prio3_sizes_t* szp,
                      int threads, int jobs, int job_size,
                      uint32_t pool, const uint8_t* nonces, const uint8_t* pub,
                      const uint8_t* helper, const uint8_t* lps, uint8_t* status_out,
                      uint64_t* counts_out, uint8_t* agg_out, int combined) {
  const prio3_sizes_t sz = *szp;  // the instance's sizes (prio3_sizes; all engines share it)
  const uint32_t span = pool - (uint32_t)job_size + 1;
  return run_pool(threads, jobs, [&](int j) {
    thread_local std::vector<uint8_t> msgs;
    msgs.resize((size_t)job_size * (sz.prep_msg_len ? sz.prep_msg_len : 1));
    const uint32_t t = (uint32_t)(j % n_engines);
    const uint32_t r0 = t * pool + (uint32_t)(((uint64_t)(j / n_engines) * job_size) % span);
    const uint8_t* jp = sz.public_share_len ? pub + (size_t)sz.public_share_len * r0 : nullptr;
    uint8_t* agg = agg_out + (size_t)sz.agg_share_len * j;
    uint64_t cnt = 0;
    int rc;
    if (combined) {
      rc = prio3_helper_prepare_aggregate_batch(
          engines[t], (uint32_t)job_size, nonces + 16 * (size_t)r0, jp,
          helper + (size_t)sz.helper_share_len * r0, lps + (size_t)sz.prep_share_len * r0,
          nullptr, nullptr, 1, msgs.data(), status_out + (size_t)j * job_size, agg, &cnt);
    } else {
      prio3_batch* b = nullptr;
      rc = prio3_helper_prepare_batch(
          engines[t], (uint32_t)job_size, nonces + 16 * (size_t)r0, jp,
          helper + (size_t)sz.helper_share_len * r0, lps + (size_t)sz.prep_share_len * r0,
          msgs.data(), status_out + (size_t)j * job_size, &b);
      if (rc == PRIO3_OK) rc = prio3_accumulate(b, nullptr, nullptr, 1, agg, &cnt);
      if (b) prio3_batch_free(b);
    }
    counts_out[j] = cnt;
    return rc == PRIO3_OK;
  });
}


// The leader's side of the same jobs: per job prio3_leader_prepare_init_batch on the explicit
// leader input shares lin[..][leader_input_share_len], prio3_leader_prepare_next_batch on the
// helper's prepare messages msgs[..][prep_msg_len], prio3_accumulate, prio3_batch_free.  Job j's
// reports are chosen as in janus_jobs_run; ps_out[jobs * job_size][prep_share_len].
// combined = 1: prio3_leader_prepare_next_aggregate_batch instead of the last two calls.
double janus_jobs_run_leader(prio3_engine** engines, int n_engines, const prio3_sizes_t* szp,
                             int threads, int jobs, int job_size, uint32_t pool,
                             const uint8_t* nonces, const uint8_t* pub, const uint8_t* lin,
                             const uint8_t* msgs, uint8_t* ps_out, uint8_t* status_out,
                             uint64_t* counts_out, uint8_t* agg_out, int combined) {
  const prio3_sizes_t sz = *szp;
  const uint32_t span = pool - (uint32_t)job_size + 1;
  return run_pool(threads, jobs, [&](int j) {
    const uint32_t t = (uint32_t)(j % n_engines);
    const uint32_t r0 = t * pool + (uint32_t)(((uint64_t)(j / n_engines) * job_size) % span);
    const size_t o = (size_t)j * job_size;
    prio3_batch* b = nullptr;
    int rc = prio3_leader_prepare_init_batch(
        engines[t], (uint32_t)job_size, nonces + 16 * (size_t)r0,
        sz.public_share_len ? pub + (size_t)sz.public_share_len * r0 : nullptr,
        lin + (size_t)sz.leader_input_share_len * r0, ps_out + (size_t)sz.prep_share_len * o,
        status_out + o, &b);
    const uint8_t* m = sz.prep_msg_len ? msgs + (size_t)sz.prep_msg_len * r0 : nullptr;
    uint8_t* agg = agg_out + (size_t)sz.agg_share_len * j;
    uint64_t cnt = 0;
    if (rc == PRIO3_OK && combined) {
      rc = prio3_leader_prepare_next_aggregate_batch(b, m, status_out + o, nullptr, nullptr, 1,
                                                     agg, &cnt);
    } else if (rc == PRIO3_OK) {
      rc = prio3_leader_prepare_next_batch(b, m, status_out + o);
      if (rc == PRIO3_OK) rc = prio3_accumulate(b, nullptr, nullptr, 1, agg, &cnt);
    }
    prio3_batch_free(b);
    counts_out[j] = cnt;
    return rc == PRIO3_OK;
  });
}

// The helper's input-share open per job: janus_hpke_open_input_shares over job j's reports of
// task t = j % n_tasks (task_ids[t][32]; per-task report pools as above, per-report rows of
// nenc / ct_stride / 4 / 16 / 8 / pub_len bytes).  shares_out[jobs * job_size][share_len].
double janus_jobs_run_hpke(janus_hpke_opener* op, int n_tasks, const uint8_t* task_ids,
                           int threads, int jobs, int job_size, uint32_t pool, uint32_t nenc,
                           const uint8_t* enc, const uint8_t* ct, const uint32_t* ct_len,
                           uint32_t ct_stride, const uint8_t* ids, const uint64_t* times,
                           const uint8_t* pubs, uint32_t pub_len, uint32_t share_len,
                           uint8_t* shares_out, uint8_t* status_out) {
  const uint32_t span = pool - (uint32_t)job_size + 1;
  return run_pool(threads, jobs, [&](int j) {
    const uint32_t t = (uint32_t)(j % n_tasks);
    const size_t r0 = t * (size_t)pool + (((uint64_t)(j / n_tasks) * job_size) % span);
    const size_t o = (size_t)j * job_size;
    return janus_hpke_open_input_shares(
               op, (uint32_t)job_size, task_ids + 32 * (size_t)t, enc + nenc * r0,
               ct + (size_t)ct_stride * r0, ct_len + r0, ct_stride, ids + 16 * r0, times + r0,
               pub_len ? pubs + pub_len * r0 : nullptr, pub_len, share_len,
               0, shares_out + (size_t)share_len * o, status_out + o) == JANUS_HPKE_SUCCESS;
  });
}

// The helper's whole loop body per job from the sealed input shares (aggregator.rs:1794-2096):
// job j of task t = j % n_engines over the same report windows as janus_jobs_run, whose input
// shares were sealed to `opener`'s keypair under task_ids[t][32] (enc[..][nenc], ct[..][ct_stride],
// ct_len, times).  one_call = 1: prio3_helper_aggregate_init_batch (the open, prepare and
// accumulate in one coalesced launch); 0: the two-call composition a caller of r05's ABI makes --
// janus_hpke_open_input_shares into host buffers, then prio3_helper_prepare_aggregate_batch with
// the open's rejections masked out and their statuses merged (0x80 | PrepareError).
double janus_jobs_run_init(prio3_engine** engines, int n_engines, const prio3_sizes_t* szp,
                           janus_hpke_opener* opener, const uint8_t* task_ids, int threads,
                           int jobs, int job_size, uint32_t pool, const uint8_t* nonces,
                           const uint8_t* pub, const uint64_t* times, const uint8_t* enc,
                           uint32_t nenc, const uint8_t* ct, const uint32_t* ct_len,
                           uint32_t ct_stride, const uint8_t* lps, uint8_t* status_out,
                           uint64_t* counts_out, uint8_t* agg_out, int one_call) {
  const prio3_sizes_t sz = *szp;
  const uint32_t span = pool - (uint32_t)job_size + 1;
  return run_pool(threads, jobs, [&](int j) {
    thread_local std::vector<uint8_t> msgs, shares, hs, acc;
    msgs.resize((size_t)job_size * (sz.prep_msg_len ? sz.prep_msg_len : 1));
    const uint32_t t = (uint32_t)(j % n_engines);
    const size_t r0 = t * (size_t)pool + (((uint64_t)(j / n_engines) * job_size) % span);
    const size_t o = (size_t)j * job_size;
    const uint8_t* jp = sz.public_share_len ? pub + (size_t)sz.public_share_len * r0 : nullptr;
    uint8_t* st = status_out + o;
    uint8_t* agg = agg_out + (size_t)sz.agg_share_len * j;
    uint64_t cnt = 0;
    int rc;
    if (one_call) {
      rc = prio3_helper_aggregate_init_batch(
          engines[t], opener, (uint32_t)job_size, task_ids + 32 * (size_t)t, 0,
          nonces + 16 * r0, times + r0, jp, enc + (size_t)nenc * r0,
          ct + (size_t)ct_stride * r0, ct_len + r0, ct_stride, lps + (size_t)sz.prep_share_len * r0,
          nullptr, nullptr, 1, msgs.data(), st, agg, &cnt);
    } else {
      shares.resize((size_t)job_size * sz.helper_share_len);
      hs.resize(job_size);
      acc.resize(job_size);
      rc = janus_hpke_open_input_shares(
          opener, (uint32_t)job_size, task_ids + 32 * (size_t)t, enc + (size_t)nenc * r0,
          ct + (size_t)ct_stride * r0, ct_len + r0, ct_stride, nonces + 16 * r0, times + r0, jp,
          sz.public_share_len, sz.helper_share_len, 0, shares.data(), hs.data());
      if (rc == 0) {
        for (int i = 0; i < job_size; i++) acc[i] = hs[i] == 0;
        rc = prio3_helper_prepare_aggregate_batch(
            engines[t], (uint32_t)job_size, nonces + 16 * r0, jp, shares.data(),
            lps + (size_t)sz.prep_share_len * r0, nullptr, acc.data(), 1, msgs.data(), st, agg,
            &cnt);
        for (int i = 0; i < job_size; i++)
          if (hs[i]) st[i] = (uint8_t)(0x80u | hs[i]);
      }
    }
    counts_out[j] = cnt;
    return rc == 0;
  });
}

}  // extern "C"
