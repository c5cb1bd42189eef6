// jobs_driver.cpp -- measurement harness for the production call shape (bench.py --role jobs):
// C host threads, each playing one Janus rayon worker that runs whole aggregation jobs
// (/root/reference/aggregator/src/aggregator.rs:2100-2123) of `job_size` reports
// (binaries/aggregation_job_creator.rs:63-64, default 100-500), calling the C ABI exactly as the
// FFI crate of INTEGRATION.md would: prio3_helper_prepare_batch (host buffers, PCIe included),
// then prio3_accumulate into the job's batch aggregation, then prio3_batch_free.
// Not part of the engine: a separate library (libjanus_jobs.so) that links libjanus_prio3.so.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/janus_prio3.h"

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
  std::atomic<int> next{0};
  std::atomic<int> failed{0};
  const uint32_t span = pool - (uint32_t)job_size + 1;
  auto worker = [&]() {
    std::vector<uint8_t> msgs((size_t)job_size * (sz.prep_msg_len ? sz.prep_msg_len : 1));
    for (;;) {
      const int j = next.fetch_add(1);
      if (j >= jobs) return;
      const uint32_t t = (uint32_t)(j % n_engines);
      const uint32_t r0 =
          t * pool + (uint32_t)(((uint64_t)(j / n_engines) * job_size) % span);
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
      if (rc != PRIO3_OK) failed = 1;
      counts_out[j] = cnt;
    }
  };
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int i = 0; i < threads; i++) th.emplace_back(worker);
  for (auto& t : th) t.join();
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return failed ? -1.0 : dt;
}

}  // extern "C"
