"""Benchmark: helper-side Prio3Histogram(length=256, chunk_length=16) prepare+aggregate on
MI355X (BASELINE.json metric; configs[1]: 1M reports per GPU).

One step = one device call over the whole resident batch: k_xof -> k_xof_slow (flagged
reports only) -> k_query (FLP query, decide, prepare message, joint-rand check) -> masked
segmented mod-p accumulate into the aggregate share; with N>1 ranks the per-GPU partial
aggregate shares are RCCL-all-gathered over xGMI and summed mod p on every rank (RCCL's
integer sum is mod 2^64, not mod p).  Reports are distinct, honest, seed-derived and
generated on the device before timing (inputs resident in HBM when the timed region starts).

Usage: python bench.py [--gpus N --steps K --warmup W]  (N>1 via torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from janus_amd import prio3 as J  # noqa: E402
import roofline_model as RM  # noqa: E402

METRIC = "reports prepared+aggregated/sec (helper, Prio3Histogram len=256) at 1/2/4/8 GPUs"
VK = bytes.fromhex("4a414e55532d414d442d42454e434821")

# --- roofline inputs.  Per kernel, profiles/kernel_counts.json (written by
# tools/summarize_profiles.py from the committed rocprofv3 passes) holds the dynamic VALU
# instructions per report (SQ_INSTS_VALU / SQ_WAVES, one report per lane) and its PMC HBM bytes
# per launch (plus the static half-rate fraction of its hot loop, tools/isa_mix.py, for reference).
COUNTS_PATH = os.path.join(ROOT, "profiles", "kernel_counts.json")
# per-report HBM bytes each kernel must move at minimum (algorithmic; Histogram(256,16))
KERNEL_BYTES = {"k_xof_a": 16 + 16 + 16 + 256 * 16 + 95 * 16,  # nonce, k_meas, k_proofs in; shares out
                "k_jrpart": 16 + 16 + 32 + 256 * 16 + 2 * 16 + 16,
                "k_xofd": 16 + 48 + 32 + 256 * 16 + 95 * 16 + 16 + 16 + 3 * 16,  # + jr/qr/part out
                "k_query_h": 256 * 16 + 95 * 16 + 560 + 2 * 16 + 16 + 16 + 17,
                "k_query_rows": 256 * 16 + 95 * 16 + 560 + 2 * 16 + 16 + 16 + 17,
                "k_acc_partial": 256 * 16 + 1}
# the fused XOF + query kernel moves both kernels' bytes (the share still round-trips through HBM)
KERNEL_BYTES["k_prep_h"] = KERNEL_BYTES["k_xofd"] + KERNEL_BYTES["k_query_h"]
# --- algorithmic VALU denominator ("The roofline denominator").  A frozen
# table of gfx950 lane-instruction costs of the cheapest sequences known for each primitive,
# times the algorithm's primitive counts per report.  No kernel can issue fewer instructions for
# the same algorithm with these primitives, and no kernel can issue faster than the 78.6 T peak,
# so model_instr x reports/s / 78.6 T is a roofline fraction <= 1; measured SQ_INSTS_VALU per
# report / model_instr is the instruction-bloat ratio reported beside it.
PRIM = dict(
    keccak_round=190,  # 20 bitop3 (theta C) + 10 alignbit + 10 xor (theta D) + 50 xor (theta
                       # apply) + 48 alignbit (rho; no lane rotates by a multiple of 32) +
                       # 50 bitop3 (chi) + 2 (iota), 32-bit halves of the 64-bit lanes
    f128_mul=90,       # 16 v_mad_u64_u32 schoolbook + carries, 2^128 = 28*2^64 - 1 fold (asm)
    f128_mac=32,       # lazily reduced multiply-accumulate: 16 v_mad_u64_u32 + 16 carries
    f128_reduce=67,    # lazy 288-bit accumulator -> canonical (asm)
    f128_add=13,       # 4-limb add, conditional subtract of p
    f128_sum_add=5,    # lazy sum of field elements (carry word)
    lt_p=4,            # canonical-encoding check of one decoded / squeezed element
    sha256_compress=1440,  # 64 rounds x 15 (bitop3 Ch/Maj, alignbit rotates, add3) + 48 x 10
)


def valu_model(kernel: str, length=256, chunk=16) -> float:
    """Minimum lane-instructions per report of a Prio3Histogram(length, chunk) kernel."""
    P = 1
    calls = -(-length // chunk)
    while P < calls + 1:
        P *= 2
    glen = 2 * (P - 1) + 1
    perm = 12 * PRIM["keccak_round"]
    if kernel in ("k_xofd", "k_xof"):
        meas_blocks = -(-(16 * length) // 168)
        jr_blocks = (42 + 16 * length) // 168 + 1
        proof_len = 2 * chunk + glen
        proofs_blocks = -(-(16 * proof_len) // 168)
        perms = 1 + meas_blocks + jr_blocks + proofs_blocks + 1 + 1
        squeezed = length + proof_len + 2 + 1
        return perms * perm + squeezed * PRIM["lt_p"] + jr_blocks * 42  # + funnel shifts
    if kernel in ("k_query_h", "k_query_pair", "k_query_rows"):
        # Lagrange basis at t: four 8-point DFTs of geometric sequences (P = 32; radix 2, 12
        # butterflies each, 5 with a non-trivial twiddle): t^8/t^16/t^32, the four phase sums G_ph
        # (3 muls), the start values and ratios, 4 x 7 sequence steps, 4 x 5 twiddle products
        nph, pts = 4, P // 4
        bfly = (pts // 2) * 3
        twid = 5
        muls = 5 + 3 + nph + (nph - 1) + nph * (pts - 1) + nph * twid
        adds = nph * 2 * bfly + 6 + calls
        muls += (glen - 1) + chunk.bit_length() + 2 * calls  # Horner, r^C, beta
        macs = (glen - 1) + 2 * length + 4 * chunk            # range, A/B sums, finalize
        reduces = 1 + 3 * chunk + chunk // 2                 # range, A/B/f0 per wire, gadget groups
        muls += chunk + 1 + 3 + 2                             # r^(j+1), L/2, v, sum fold
        adds += (glen - 1) + 3 * chunk + 6
        return (muls * PRIM["f128_mul"] + macs * PRIM["f128_mac"] +
                reduces * PRIM["f128_reduce"] + adds * PRIM["f128_add"] +
                length * PRIM["f128_sum_add"] + (2 * chunk + 2) * PRIM["lt_p"] + perm)
    if kernel == "k_prep_h":  # dual-state XOF + P = 32 query in one launch
        return valu_model("k_xofd", length, chunk) + valu_model("k_query_h", length, chunk)
    if kernel == "k_meta":
        return PRIM["sha256_compress"]
    return 0.0


# Peak: the guide's vector issue rate (MI355X_MICROARCH.md: 157.3 TFLOPS FP32 vector = 256 CU x
# 4 SIMD x 32 lanes/clk x 2.4 GHz = 78.6 T lane-instructions/s); measured full-rate issue on
# this chip is 64.5 T (profiles/r01_ubench_valu_gfx950.txt), reported beside it.
PEAK_VALU_NOMINAL = 256 * 4 * 32 * 2.4e9  # 78.6e12 lane-instr/s
MEASURED_ISSUE_T = 64.5
PEAK_HBM = 8.0e12


ISSUED_PATH = os.path.join(ROOT, "profiles", "issued_per_report.json")


def model_roofline(line: str, model: dict, n: int, steps: int, elapsed: float,
                   note: str = "") -> dict:
    """Roofline of a whole step from roofline_model: achieved = the frozen
    minimum-instruction model per report x reports/s; peak = the guide's 78.6 T VALU issue rate.
    issued_over_model: PMC SQ_INSTS_VALU x 64 per report of the same step (committed table
    profiles/issued_per_report.json, tools/pmc_issued.py) over the model."""
    peak_T = PEAK_VALU_NOMINAL / 1e12
    ach = model["total"] * n * steps / elapsed / 1e12
    r = dict(bound="valu", achieved=ach, peak=peak_T,
             unit="T lane-instr/s (achieved = roofline_model.py minimum-instruction model x "
                  "reports/s over the whole step; peak = guide vector rate)",
             frac=ach / peak_T, frac_of_measured_issue=ach / MEASURED_ISSUE_T,
             model_instr_per_report=model["total"],
             model_parts={k: v for k, v in model.items() if k != "total"}, traffic=None)
    if note:
        r["note"] = note
    issued = json.load(open(ISSUED_PATH)) if os.path.exists(ISSUED_PATH) else {}
    if line in issued:
        r["issued_instr_per_report"] = issued[line]["issued_instr_per_report"]
        r["issued_over_model"] = issued[line]["issued_instr_per_report"] / model["total"]
        r["issued_source"] = issued[line]["source"]
    return r


def cpu_threads() -> int:
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(env))) if env else aff


def cpu_baseline(eng, data, n_gpu_sample: int, target_s: float = 10.0):
    """The oracle (CPU restatement of prio 0.16.2, Janus job structure) timed on this host on a
    bounded sample of the same (GPU-generated) reports; also cross-checks the GPU results."""
    from oracle.oracle import Oracle, build
    build()
    o = Oracle("histogram", length=256, chunk_length=16)
    th = cpu_threads()
    host = {k: data[k][:n_gpu_sample].cpu().numpy() for k in
            ("nonces", "public_shares", "helper_shares", "leader_prep_shares")}

    def run(m):
        t0 = time.perf_counter()
        r = o.helper_batch(VK, host["nonces"][:m], host["public_shares"][:m],
                           host["helper_shares"][:m], host["leader_prep_shares"][:m],
                           n_threads=th, job_size=500)
        return time.perf_counter() - t0, r

    probe = min(n_gpu_sample, 500 * th)
    dt, _ = run(probe)
    m = int(min(n_gpu_sample, max(probe, probe * target_s / max(dt, 1e-6))))
    dt, (msgs, status, agg, cnt) = run(m)
    return dict(value=m / dt, unit="reports/s", cores=th, kind="port",
                sample=f"{m} of the benchmark's GPU-generated reports, jobs of 500 reports, "
                       f"one job per worker thread (aggregator.rs:1794,2100), {dt:.1f}s wall",
                seconds=dt, n=m), (msgs, status, agg, cnt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reports", type=int, default=1 << 20, help="reports per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--role", choices=["helper", "leader", "hpke", "pipeline", "mp64", "fpvec", "config",
                                       "jobs"],
                    default="helper",
                    help="helper (the BASELINE metric), the leader side (SURVEY 8(f) row 1) or "
                         "the batched HPKE open of helper input shares (8(f) row 2)")
    ap.add_argument("--vdaf", choices=["count", "sumvec", "sum32"], default="sumvec",
                    help="--role config: C1 Prio3Count (100k), C3 Prio3SumVec 8x1000 chunk 63 "
                         "(1M/8 per GPU), C4 Prio3Sum 32 (10M/8 per GPU)")
    ap.add_argument("--hpke-aead", type=int, choices=[1, 2, 3], default=1,
                    help="--role hpke: AEAD id (1 AES-128-GCM, 2 AES-256-GCM, 3 ChaCha20Poly1305)")
    ap.add_argument("--hpke-kem", choices=["x25519", "p256", "x448", "p521", "p384"], default="x25519",
                    help="--role hpke: DHKEM(X25519, HKDF-SHA256), DHKEM(P-256, HKDF-SHA256), "
                         "DHKEM(X448, HKDF-SHA512) or DHKEM(P-521, HKDF-SHA512); the key "
                         "schedule's KDF follows the KEM's (RFC 9180 suites of the reference's "
                         "test vectors)")
    ap.add_argument("--leader-vdaf", choices=["hist", "sum32"], default="hist",
                    help="--role leader: Prio3Histogram(256,16) at 1Mi (default) or Prio3Sum(32) "
                         "at C4's 1.25M per GPU")
    ap.add_argument("--threads", type=int, default=128,
                    help="--role jobs: host worker threads (Janus's rayon pool)")
    ap.add_argument("--job-size", type=int, default=500,
                    help="--role jobs: reports per aggregation job (aggregation_job_creator.rs:63-64)")
    ap.add_argument("--jobs-call", choices=["combined", "two"], default="combined",
                    help="--role jobs: prio3_helper_prepare_aggregate_batch per job (one round "
                         "trip) or prio3_helper_prepare_batch + prio3_accumulate (two); the "
                         "leader: prio3_leader_prepare_next_aggregate_batch after the init, or "
                         "prio3_leader_prepare_next_batch + prio3_accumulate")
    ap.add_argument("--tasks", type=int, default=4,
                    help="--role jobs: tasks (verify keys) of the VDAF instance the jobs rotate over")
    ap.add_argument("--jobs-role", choices=["helper", "leader", "hpke", "init"], default="helper",
                    help="--role jobs: the helper's prepare + aggregate per job (default), the "
                         "leader's prepare_init + prepare_next + aggregate per job, the "
                         "helper's HPKE open of each job's input shares, or the helper's whole "
                         "loop body from sealed input shares in one call (init; with the two-call "
                         "composition measured beside it)")
    ap.add_argument("--exec-heavy", type=int, default=0,
                    help="--role jobs: the executors' light/heavy switch in reports inside them "
                         "(prio3_executor_control / janus_hpke_executor_control \"heavy\"; 0: the "
                         "default 32768), for A/B runs")
    ap.add_argument("--devices", default=None,
                    help="--role jobs: the engines' GPUs as a comma (or +) list (prio3_engine_create_"
                         "devices; a GPU named twice gets two executors); default: every visible "
                         "GPU as one device mask (prio3_engine_create_mask)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N>1: nccl (RCCL over xGMI, the measured path) or gloo with the combine's "
                         "all-gather staged through host memory (lets N ranks share one GPU in a "
                         "test; never a measurement)")
    ap.add_argument("--check-combined", action="store_true",
                    help="N>1: rank 0 regenerates every rank's shard and checks the combined "
                         "aggregate, count, checksum and interval against the CPU restatement")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option key=value (e.g. chunks=3, force_generic_query=1), for A/B runs")
    ap.add_argument("--no-secondary", action="store_true",
                    help="helper role, N=1: skip the secondary lines (C1/C3/C4 configs and a short "
                         "jobs line) that the default run adds as extra keys")
    ap.add_argument("--secondary-cpu-seconds", type=float, default=1.5,
                    help="CPU restatement sample size (seconds) for each secondary config line")
    args = ap.parse_args()
    if os.environ.get("JANUS_BENCH_STACKDUMP"):  # tests: every thread's stack after N s, to stderr
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["JANUS_BENCH_STACKDUMP"]), exit=False)
    if args.role == "leader":
        return leader_main(args)
    if args.role == "hpke":
        return hpke_main(args)
    if args.role == "pipeline":
        return pipeline_main(args)
    if args.role == "mp64":
        return mp64_main(args)
    if args.role == "fpvec":
        return fpvec_main(args)
    if args.role == "config":
        return config_main(args)
    if args.role == "jobs":
        return jobs_main(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 and args.dist_backend == "gloo":
        # ranks may outnumber GPUs here (a one-GPU test of this step): device = local rank mod count
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n = args.reports

    eng = J.HelperEngine(J.Prio3Histogram(256, 16), VK, device=local)
    sz = eng.sz
    chunks_opt = 0  # engine default: auto
    for kv in args.opt:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
        if k == "chunks":
            chunks_opt = int(v)
    data = eng.generate_reports_device(n, seed=0x4A414E5553000001, first_index=rank * n,
                                       with_checks=True)
    torch.cuda.synchronize()
    flags = int(data["flags"].sum().item())
    prep_msgs = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    agg = torch.zeros((1, sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    # report timestamps (seconds) inside one hour-long batch interval, seeded
    def times_of(r):
        g = torch.Generator(device=dev).manual_seed(0x4A414E55 + r)
        return 1_700_000_000 + torch.randint(0, 3600, (n,), generator=g, device=dev,
                                             dtype=torch.int64)
    report_times = times_of(rank)
    cks = torch.zeros((1, 32), dtype=torch.uint8, device=dev)
    ivs = torch.zeros((1, 2), dtype=torch.int64, device=dev)
    combiner = None
    if world > 1:
        from janus_amd.dist import AggregateCombiner
        cur = lambda: torch.cuda.current_stream().cuda_stream
        combiner = AggregateCombiner(
            dist, agg, cnt,
            lambda k, ga, gc, oa, oc: eng.combine_device(k, 1, ga, gc, oa, oc, stream=cur()),
            cks, ivs,
            lambda k, gk, gi, ok, oi: eng.combine_metadata_device(k, 1, gk, gi, ok, oi,
                                                                  stream=cur()),
            stage_device="cpu" if args.dist_backend == "gloo" else None)

    def step():
        # SURVEY 8(a) a3-a11 + a14: prepare, decide, prepare message, and the per-segment batch
        # aggregation update (aggregate share, count, report-ID checksum, client interval)
        s = torch.cuda.current_stream().cuda_stream
        eng.prepare_aggregate_device(data["nonces"], data["public_shares"], data["helper_shares"],
                                     data["leader_prep_shares"], seg, 1, prep_msgs, status,
                                     stream=s)
        eng.aggregate_finish_device(status, None, agg, cnt, stream=s)
        eng.batch_metadata_device(data["nonces"], report_times, status, None, seg, 1, cks, ivs, stream=s)
        if combiner is not None:
            combiner(agg, cnt, cks, ivs)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.set_option("timing", 1)
    eng.timing_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_times = eng.timing()
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # Roofline pass (after the timed region): whole-batch launches (option chunks=1, which the
    # fused k_prep_h default already uses; the two-kernel chain would cut a 1Mi batch into 8
    # stream-overlapped chunks, where a launch's duration includes its neighbour's share of the
    # CU), a few steps on the same stream and data.
    eng.set_option("chunks", 1)
    eng.timing_reset()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    times = eng.timing()
    eng.set_option("timing", 0)
    eng.set_option("chunks", chunks_opt)

    ok = int((status == 0).sum().item())
    final_cnt = int((combiner.out_cnt if combiner is not None else cnt)[0].item())
    value = world * n * args.steps / elapsed

    # roofline of the dominant kernel, from the live HIP-event times on the launch stream:
    # achieved = the frozen gfx950 VALU model (valu_model) x reports / duration;
    # the measured instructions per report (PMC SQ_INSTS_VALU / SQ_WAVES, profiles/) give the
    # issued rate and the bloat ratio beside it
    per_kernel = {k: dict(ms_total=v[0], launches=v[1], ms_avg=v[0] / max(v[1], 1))
                  for k, v in times.items()}
    counts = json.load(open(COUNTS_PATH)) if os.path.exists(COUNTS_PATH) else dict(kernels={})
    kc = counts["kernels"]
    peak_T = PEAK_VALU_NOMINAL / 1e12
    for k, v in per_kernel.items():
        m = valu_model(k)
        if m:
            v["model_instr_per_report"] = m
            v["model_T"] = m * n / (v["ms_avg"] / 1e3) / 1e12
            v["frac"] = v["model_T"] / peak_T
        if k in kc and "valu_instr_per_item" in kc[k]:
            v["issued_instr_per_report"] = kc[k]["valu_instr_per_item"]
            v["issued_T"] = kc[k]["valu_instr_per_item"] * n / (v["ms_avg"] / 1e3) / 1e12
            if m:
                v["issued_over_model"] = kc[k]["valu_instr_per_item"] / m
        if k in kc and "bytes" in kc[k]:
            v["hbm_pmc_TBps"] = kc[k]["bytes"] / (v["ms_avg"] / 1e3) / 1e12
            v["hbm_frac"] = v["hbm_pmc_TBps"] * 1e12 / PEAK_HBM
        if k in KERNEL_BYTES:
            v["hbm_algorithmic_GBps"] = KERNEL_BYTES[k] * n / (v["ms_avg"] / 1e3) / 1e9
    dom = max((k for k in per_kernel if "model_T" in per_kernel[k]),
              key=lambda k: per_kernel[k]["ms_total"])
    d = per_kernel[dom]
    step_model = sum(valu_model(k) for k in per_kernel if valu_model(k))
    roofline = dict(bound="valu", achieved=d["model_T"], peak=peak_T,
                    unit="T lane-instr/s (32-bit VALU; achieved = frozen gfx950 minimum-"
                         "instruction model x reports / kernel time; peak = guide vector rate)",
                    frac=d["frac"], traffic=kc.get(dom, {}).get("bytes"),
                    traffic_source=f"{kc.get(dom, {}).get('source', counts.get('source'))} "
                                   "(PMC FETCH_SIZE*2+WRITE_SIZE, bytes/launch)",
                    kernel=dom, ms_avg=d["ms_avg"],
                    model_instr_per_report=d["model_instr_per_report"],
                    issued_instr_per_report=d.get("issued_instr_per_report"),
                    issued_over_model=d.get("issued_over_model"),
                    issued_frac=(d["issued_T"] / peak_T) if "issued_T" in d else None,
                    frac_of_measured_issue=d["model_T"] / MEASURED_ISSUE_T,
                    hbm_algorithmic_GBps=d.get("hbm_algorithmic_GBps"), hbm_peak_GBps=PEAK_HBM / 1e9,
                    step=dict(model_instr_per_report=step_model,
                              achieved=step_model * n * args.steps / elapsed / 1e12,
                              frac=step_model * n * args.steps / elapsed / 1e12 / peak_T,
                              note="whole timed step (all kernels), per GPU"))
    qk = next((k for k in ("k_query_rows", "k_query_h", "k_query_pair") if k in per_kernel), None)
    qh = per_kernel.get(qk) if qk else None
    if qh and "hbm_frac" in qh:
        roofline["query_hbm"] = dict(kernel=qk,
                                     achieved_TBps=qh["hbm_pmc_TBps"], peak_TBps=PEAK_HBM / 1e12,
                                     frac=qh["hbm_frac"])

    out = dict(metric=METRIC, value=value, unit="reports/s", n_gpus=world, steps=args.steps,
               warmup=args.warmup, ms_per_step=elapsed / args.steps * 1e3,
               higher_is_better=True, scaling="weak", vs_baseline=None,
               dtype="u32 limbs (Field128 mod-p integer arithmetic)",
               data="synthetic: distinct honest reports generated on-device from a seed "
                    "(client shard + leader prepare_init); verify key fixed",
               config=dict(workload="Prio3Histogram length=256 chunk_length=16 helper "
                                    "prepare_init+prepare_shares_to_prepare_message+prepare_next"
                                    "+aggregate, 1 segment",
                           reports_per_gpu=n, global_batch=world * n,
                           parallelism=f"dp{world} (report shards; RCCL all-gather + mod-p combine)"),
               roofline=roofline, kernels=per_kernel,
               kernels_timed_region={k: dict(ms_total=v[0], launches=v[1]) for k, v in step_times.items()},
               checks=dict(finished=ok, generator_flags=flags, agg_count=final_cnt))
    if world > 1:
        out["dist_backend"] = args.dist_backend
        if args.dist_backend == "gloo":
            out["note"] = "gloo: all-gather staged through host memory (a correctness run, not RCCL)"
    if world > 1 and args.check_combined and rank == 0:
        out["checks"]["combined_matches_oracle"] = check_combined(eng, args, world, n, times_of,
                                                                  combiner)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, (msgs, cst, cagg, ccnt) = cpu_baseline(eng, data, min(n, 1 << 20), args.cpu_seconds)
        m = cb.pop("n")
        gm = prep_msgs[:m].cpu().numpy()
        gs = status[:m].cpu().numpy()
        # the GPU aggregate share and count of the same sample: the last step's device run
        # finished again with an accept mask selecting its first m reports
        accept = torch.zeros(n, dtype=torch.uint8, device=dev)
        accept[:m] = 1
        agg_s = torch.zeros_like(agg)
        cnt_s = torch.zeros_like(cnt)
        eng.aggregate_finish_device(status, accept, agg_s, cnt_s)
        torch.cuda.synchronize()
        out["checks"]["cpu_gpu_parity_on_sample"] = bool(
            np.array_equal(gs, cst) and np.array_equal(gm, msgs) and
            np.array_equal(agg_s.cpu().numpy().reshape(-1), np.asarray(cagg).reshape(-1)) and
            int(cnt_s[0].item()) == int(np.asarray(ccnt).reshape(-1)[0]))
        out["checks"]["cpu_gpu_parity_covers"] = (f"statuses, prepare messages, aggregate share "
                                                  f"and count of {m} reports")
        from oracle.oracle import batch_metadata
        eck, eiv = batch_metadata(data["nonces"].cpu().numpy(), report_times.cpu().numpy(),
                                  status.cpu().numpy(), None, None, 1)
        out["checks"]["batch_metadata_parity"] = bool(
            np.array_equal(cks.cpu().numpy(), eck) and
            np.array_equal(ivs.cpu().numpy().view(np.uint64), eiv))
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu"] = value / cb["value"]
    if rank == 0 and world == 1 and not args.no_secondary:
        del data, prep_msgs, status, seg, report_times
        eng.close()
        torch.cuda.empty_cache()
        out.update(secondary_lines(args))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def _summary(d: dict) -> dict:
    """The fields of a secondary line the default bench keeps (the full line is what --role
    config / --role jobs print)."""
    rf = d.get("roofline") or {}
    cb = d.get("cpu_baseline") or {}
    ck = d.get("checks") or {}
    return dict(metric=d["metric"], value=d["value"], unit=d["unit"], ms_per_step=d["ms_per_step"],
                steps=d.get("steps"), config=d.get("config"),
                roofline=dict(bound=rf.get("bound"), kernel=rf.get("kernel"), frac=rf.get("frac"),
                              achieved=rf.get("achieved"), peak=rf.get("peak"), unit=rf.get("unit")),
                checks=ck, cpu_baseline=dict(value=cb.get("value"), unit=cb.get("unit"),
                                             cores=cb.get("cores"), sample=cb.get("sample"))
                if cb else None)


def secondary_lines(args) -> dict:
    """the other BASELINE.json configs on this GPU (C1 Count 100k, C3
    SumVec 8x1000 and C4 Sum(32) at one GPU's 1/8 shard), each with its roofline frac and the
    GPU-vs-restatement parity of a bounded CPU sample, and a short host-buffer jobs line
    (4194 jobs x 500 reports at 128 threads and 2048 jobs at 16 threads, every job checked).  Extra keys of the headline line;
    its `value` stays the C2 helper rate."""
    out = {}
    t0 = time.perf_counter()
    for key, vdaf, steps in (("secondary_c1_count", "count", 20),
                             ("secondary_c3_sumvec", "sumvec", 5),
                             ("secondary_c4_sum32", "sum32", 10)):
        try:
            out[key] = _summary(config_line(vdaf, CONFIGS[vdaf][2], steps, 2,
                                            args.secondary_cpu_seconds))
        except Exception as ex:  # a secondary line never hides the headline
            out[key] = dict(error=f"{type(ex).__name__}: {ex}")
        torch.cuda.empty_cache()
    # the jobs lines at jobs_main's default size (2 Mi reports at 128 threads): with 2048 jobs the
    # timed region was ~40 ms and read 27-33 M/s against 38-40 M/s for the same launcher; the
    # leader and HPKE jobs lines at 1 Mi reports
    cs = args.secondary_cpu_seconds
    for key, fn in (("secondary_jobs", lambda: jobs_line(128, 500, (1 << 21) // 500, 4,
                                                         cpu_seconds=cs)),
                    ("secondary_jobs_16t", lambda: jobs_line(16, 500, 2048, 4, cpu_seconds=cs)),
                    # (the leader line at 2 Mi reports too: at 1 Mi its 66 groups are a third
                    # ramp, r06ae: 5.7 against 5.8-7.5 M/s at 2 Mi)
                    ("secondary_jobs_leader", lambda: leader_jobs_line(128, 500, (1 << 21) // 500,
                                                                       4, cpu_seconds=cs)),
                    ("secondary_jobs_hpke", lambda: hpke_jobs_line(128, 500, 2048, 4,
                                                                   cpu_seconds=cs)),
                    # the whole loop body from sealed input shares in one call,
                    # with the two-call composition measured beside it in the same run
                    # (at jobs_main's 2 Mi reports like secondary_jobs: with 1 Mi the ~80 ms timed
                    # region is mostly the ramp from the light-load pipeline, r06f: 12.4 M/s)
                    ("secondary_jobs_init", lambda: init_jobs_line(128, 500, (1 << 21) // 500, 4,
                                                                   cpu_seconds=cs)),
                    ("secondary_jobs_init_16t", lambda: init_jobs_line(16, 500, 1024, 4,
                                                                       cpu_seconds=cs))):
        try:
            j = fn()
            out[key] = dict(metric=j["metric"], value=j["value"], unit=j["unit"],
                            ms_per_step=j["ms_per_step"], config=j["config"],
                            coalescing=j["coalescing"], placement=j.get("placement"),
                            host=j.get("host"),
                            two_call=j.get("two_call"),
                            roofline={k: j["roofline"][k] for k in ("bound", "achieved", "peak",
                                                                    "unit", "frac")},
                            checks=j["checks"], cpu_baseline=j["cpu_baseline"])
        except Exception as ex:
            out[key] = dict(error=f"{type(ex).__name__}: {ex}")
        torch.cuda.empty_cache()
    out["secondary_seconds"] = time.perf_counter() - t0
    return out


def check_combined(eng, args, world, n, times_of, combiner) -> bool:
    """Rank 0, N>1: every rank's shard regenerated here (same seed and report indices), the CPU
    restatement's helper batch over all world x n reports, and the combined aggregate share,
    count, ReportIdChecksum and interval compared with it (aggregate_share.rs:55-96)."""
    from oracle.oracle import Oracle, batch_metadata
    o = Oracle("histogram", length=256, chunk_length=16)
    cols = {k: [] for k in ("nonces", "public_shares", "helper_shares", "leader_prep_shares")}
    times = []
    for r in range(world):
        d = eng.generate_reports_device(n, seed=0x4A414E5553000001, first_index=r * n)
        for k in cols:
            cols[k].append(d[k].cpu().numpy())
        times.append(times_of(r).cpu().numpy())
    host = {k: np.concatenate(v) for k, v in cols.items()}
    _, st, agg, cnt = o.helper_batch(VK, host["nonces"], host["public_shares"],
                                     host["helper_shares"], host["leader_prep_shares"],
                                     n_threads=cpu_threads(), job_size=500)
    ck, iv = batch_metadata(host["nonces"], np.concatenate(times), st, None,
                            None, 1)
    torch.cuda.synchronize()
    return bool(
        np.array_equal(combiner.out_agg.cpu().numpy().reshape(-1), np.asarray(agg).reshape(-1)) and
        int(combiner.out_cnt[0].item()) == int(np.asarray(cnt).reshape(-1)[0]) and
        np.array_equal(combiner.out_checksums.cpu().numpy(), ck) and
        np.array_equal(combiner.out_intervals.cpu().numpy().view(np.uint64), iv))


def _cpu_waves(fn, cores: int, js: int, avail: int, min_s: float = 2.0):
    """a jobs line's CPU baseline on WHOLE waves -- fn(m) runs the restatement
    over the first m reports as jobs of js, one job per worker thread (binary_utils.rs:514-518,
    aggregator.rs:2100), so m is a multiple of cores x js -- repeated until at least min_s of wall
    time.  A sample of 19.2 jobs on 16 threads had timed a full wave plus a wave with 13 threads idle
    (100 K/s against the headline's 166.6 K/s for the same work).  Returns (reports/s, sample)."""
    w = cores * js
    m = avail // w * w if avail >= w else avail
    fn(min(m, w))  # warm: the oracle library, page cache, thread pool
    reps, tot = 0, 0.0
    while tot < min_s:
        t0 = time.perf_counter()
        fn(m)
        tot += time.perf_counter() - t0
        reps += 1
    waves = m / w
    return reps * m / tot, (f"{reps} x {m} reports = {reps * waves:.0f} whole waves of {cores} "
                            f"jobs of {js} on {cores} threads, {tot:.1f}s")


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def jobs_main(args):
    """The production call shape: `--threads` host threads, each a Janus rayon
    worker running whole aggregation jobs of `--job-size` reports (aggregator.rs:2100-2123;
    aggregation_job_creator.rs:63-64) through the HOST-BUFFER C ABI -- prio3_helper_prepare_batch
    (PCIe H2D of the job's shares, prepare, D2H of messages + statuses) then prio3_accumulate
    and prio3_batch_free -- on `--tasks` engines (verify keys) of Prio3Histogram(256,16).
    Concurrent jobs are coalesced by the engine's executor.  The harness is native
    (janus_amd/libjanus_jobs.so, C++ threads), so Python is not on the timed path.  Reported
    against the PCIe H2D roof and next to the CPU restatement's single-core latency."""
    n_jobs = max(args.tasks, (args.reports if args.reports != 1 << 20 else 1 << 21) // args.job_size)
    devices = None if args.devices is None else [int(x) for x in args.devices.replace("+", ",").split(",")]
    if args.jobs_role == "leader":
        out = leader_jobs_line(args.threads, args.job_size, n_jobs, args.tasks, devices,
                               not args.no_cpu_baseline, args.cpu_seconds, args.exec_heavy,
                               combined=args.jobs_call == "combined")
    elif args.jobs_role == "hpke":
        out = hpke_jobs_line(args.threads, args.job_size, n_jobs, args.tasks,
                             not args.no_cpu_baseline, args.cpu_seconds, args.exec_heavy)
    elif args.jobs_role == "init":
        out = init_jobs_line(args.threads, args.job_size, n_jobs, args.tasks,
                             not args.no_cpu_baseline, args.cpu_seconds, args.exec_heavy)
    else:
        out = jobs_line(args.threads, args.job_size, n_jobs, args.tasks, args.opt,
                        args.jobs_call == "combined", not args.no_cpu_baseline,
                        devices=devices, cpu_seconds=args.cpu_seconds, heavy=args.exec_heavy)
    print(json.dumps(out), flush=True)


def _job_engines(vdaf, vks, devices):
    """One engine per task over the node's GPUs: `devices` (a list, prio3_engine_create_devices)
    or every visible GPU as a device mask (prio3_engine_create_mask)."""
    if devices is not None:
        return [J.HelperEngine(vdaf, vk, devices=devices) for vk in vks], devices
    mask = (1 << max(torch.cuda.device_count(), 1)) - 1
    return ([J.HelperEngine(vdaf, vk, device_mask=mask) for vk in vks],
            [d for d in range(32) if mask >> d & 1])


def _placement(engines, before=None):
    """Jobs / reports each member GPU (lane) took over all the line's engines."""
    tot = None
    for e in engines:
        ms = e.members()
        if tot is None:
            tot = [dict(device=m["device"], lane=m["lane"], jobs=0, reports=0) for m in ms]
        for t, m in zip(tot, ms):
            t["jobs"] += m["jobs"]
            t["reports"] += m["reports"]
    if before:
        for t, b in zip(tot, before):
            t["jobs"] -= b["jobs"]
            t["reports"] -= b["reports"]
    return tot


def _host_timed(fn):
    """fn()'s elapsed seconds (as fn returns them) and the host side of it: CPU seconds of this
    process over the call, and how often / how long the container's CPU quota (cgroup v2
    cpu.stat) throttled it meanwhile -- on the GPU box a 16-CPU quota throttles the whole process
    for up to the rest of a 100 ms period, which shows up as a 12-30 ms stall of a jobs line."""
    import resource

    def cg():
        try:
            d = dict(ln.split() for ln in open("/sys/fs/cgroup/cpu.stat"))
            return int(d["nr_throttled"]), int(d["throttled_usec"])
        except (OSError, KeyError, ValueError):
            return None

    r0, g0 = resource.getrusage(resource.RUSAGE_SELF), cg()
    dt = fn()
    r1, g1 = resource.getrusage(resource.RUSAGE_SELF), cg()
    c = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    host = dict(cpu_seconds=c, sys_seconds=r1.ru_stime - r0.ru_stime,
                cpus_busy=c / dt if dt > 0 else None,
                ctx_switches=(r1.ru_nvcsw - r0.ru_nvcsw) + (r1.ru_nivcsw - r0.ru_nivcsw))
    if g0 and g1:
        host.update(cgroup_throttled=g1[0] - g0[0], cgroup_throttled_ms=(g1[1] - g0[1]) / 1e3)
    return dt, host


def _warm(*arrays):
    """Writes the jobs lines' output arrays once before the clock: np.zeros maps zero pages lazily,
    so the first job to write each 4 KB page took a fault inside the timed region (the leader
    line's 1.2 GB of prepare shares: 1.1-1.9 s of system time per run, which pushed the process
    over the GPU box's 16-CPU quota), where a Janus worker writes into buffers its allocator has
    long mapped."""
    for a in arrays:
        a.fill(0)


def _job_windows(t, n_jobs, K, js, pool):
    """The report indices (into the concatenated per-task pools) of task t's jobs, and the job
    numbers, as the native drivers choose them (jobs_driver.cpp)."""
    jl = list(range(t, n_jobs, K))
    r0s = [t * pool + ((j // K) * js) % (pool - js + 1) for j in jl]
    return jl, np.concatenate([np.arange(r, r + js) for r in r0s])


def jobs_line(T, js, n_jobs, K, opts=(), combined=True, with_cpu=True, check_tasks=None,
              devices=None, cpu_seconds=10.0, heavy=0):
    """jobs_main's measurement (see there); check_tasks: check the jobs of only the first
    check_tasks tasks against the restatement (None: all).  The engines span `devices` (or
    every visible GPU): each job runs whole on the least-loaded one."""
    import ctypes as C
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n_jobs = max(K, n_jobs)
    pool = 1 << 16
    vks = [bytes([0x51 + t]) * 16 for t in range(K)]
    engines, devs = _job_engines(J.Prio3Histogram(256, 16), vks, devices)
    engines[0].executor_control("heavy", heavy)  # the executors are process-wide: 0 resets
    for kv in opts:
        k, v = kv.split("=")
        for e in engines:
            e.set_option(k, int(v))
    sz = engines[0].sz
    parts = [e.generate_reports_device(pool, seed=0x4A414E5553000003 + t)
             for t, e in enumerate(engines)]
    torch.cuda.synchronize()
    host = {k: np.ascontiguousarray(np.concatenate([p[k].cpu().numpy() for p in parts]))
            for k in ("nonces", "public_shares", "helper_shares", "leader_prep_shares")}
    lib = C.CDLL(os.path.join(ROOT, "janus_amd", "libjanus_jobs.so"))
    lib.janus_jobs_run.restype = C.c_double
    vp = C.c_void_p
    lib.janus_jobs_run.argtypes = [C.POINTER(vp), C.c_int, vp, C.c_int, C.c_int, C.c_int,
                                   C.c_uint32, vp, vp, vp, vp, vp, vp, vp, C.c_int]
    eng_arr = (vp * K)(*[e.handle.value for e in engines])
    status = np.zeros(n_jobs * js, np.uint8)
    counts = np.zeros(n_jobs, np.uint64)
    agg = np.zeros((n_jobs, sz.agg_share_len), np.uint8)
    _warm(status, counts, agg)
    P = lambda a: a.ctypes.data_as(vp)

    def run(jobs):
        status[:] = 0xFF
        return lib.janus_jobs_run(eng_arr, K, C.cast(C.pointer(sz), vp), T, jobs, js, pool,
                                  P(host["nonces"]), P(host["public_shares"]),
                                  P(host["helper_shares"]), P(host["leader_prep_shares"]),
                                  P(status), P(counts), P(agg), int(combined))

    run(max(K, min(n_jobs, 8 * T)))  # warmup: pools, pinned staging, streams
    for e in engines:  # launches counted, no timing events on the production launch path
        e.set_option("timing", 2)
        e.timing_reset()
    pl0 = _placement(engines)
    dt, host_side = _host_timed(lambda: run(n_jobs))
    placement = _placement(engines, pl0)
    if dt < 0:
        raise RuntimeError("janus_jobs_run: a C-ABI call failed")
    # the prepare launches: the fused XOF + query (k_prep_h, or k_prep_hp on lane pairs for small
    # groups) or, on the two-kernel chain, k_xofd
    launches = sum(e.timing().get(k, (0, 0))[1] for e in engines
                   for k in ("k_prep_h", "k_prep_hp", "k_xofd"))
    value = n_jobs * js / dt
    # every job against the restatement: per task, the jobs' report windows concatenated with
    # segment id = the job, so each segment of the oracle's batch is one job's aggregate
    from oracle.oracle import Oracle
    o = Oracle("histogram", length=256, chunk_length=16)
    t_chk = time.perf_counter()
    jobs_ok = True
    statuses_ok = True
    for t in range(K if check_tasks is None else min(K, check_tasks)):
        jl, idx = _job_windows(t, n_jobs, K, js, pool)
        seg = np.repeat(np.arange(len(jl), dtype=np.uint32), js)
        _, rst, ragg, rcnt = o.helper_batch(
            vks[t], host["nonces"][idx], host["public_shares"][idx], host["helper_shares"][idx],
            host["leader_prep_shares"][idx], segment_ids=seg, n_segments=len(jl),
            n_threads=cpu_threads())
        jobs_ok &= bool(np.array_equal(agg[jl], ragg) and
                        np.array_equal(counts[jl], rcnt.astype(np.uint64)))
        statuses_ok &= bool(np.array_equal(status.reshape(n_jobs, js)[jl], rst.reshape(-1, js)))
    t_chk = time.perf_counter() - t_chk
    # the CPU reference path on this host: the restatement at the same job structure on all
    # cores, and its single-core per-report latency
    cores = cpu_threads()
    cpu = None
    if with_cpu:
        def cpu_run(m):  # task 0's pool (its own verify key)
            o.helper_batch(vks[0], host["nonces"][:m], host["public_shares"][:m],
                           host["helper_shares"][:m], host["leader_prep_shares"][:m],
                           n_threads=cores, job_size=js)
        rate, sample = _cpu_waves(cpu_run, cores, js, pool, max(2.0, cpu_seconds))
        m1 = 2000
        t0 = time.perf_counter()
        o.helper_batch(vks[0], host["nonces"][:m1], host["public_shares"][:m1],
                       host["helper_shares"][:m1], host["leader_prep_shares"][:m1],
                       n_threads=1, job_size=js)
        dt1 = time.perf_counter() - t0
        cpu = dict(value=rate, unit="reports/s", cores=cores, kind="port", sample=sample,
                   single_core_us_per_report=dt1 / m1 * 1e6, cpu_model=cpu_model())
    per_report_h2d = 16 + sz.public_share_len + sz.helper_share_len + sz.prep_share_len
    return dict(metric="reports prepared+aggregated/sec through the host-buffer C ABI "
                      "(helper, Prio3Histogram len=256, concurrent aggregation jobs)",
               value=value, unit="reports/s", n_gpus=1, steps=1, warmup=1,
               ms_per_step=dt * 1e3, higher_is_better=True, scaling="weak", vs_baseline=None,
               dtype="u32 limbs (Field128 mod-p integer arithmetic)",
               data=f"synthetic: {K} x {pool} on-device client reports copied to host memory",
               config=dict(workload="Prio3Histogram length=256 chunk_length=16 helper prepare + "
                                    "accumulate per aggregation job, host buffers (PCIe included)",
                           job_size=js, jobs=n_jobs, threads=T, tasks=K, devices=devs),
               placement=placement,
               pcie=dict(h2d_bytes_per_report=per_report_h2d,
                         h2d_GBps=value * per_report_h2d / 1e9,
                         roof_reports_per_s=63e9 / per_report_h2d,
                         roof_note="PCIe Gen5 x16 ~63 GB/s (MI355X_MICROARCH.md)"),
               roofline=dict(bound="pcie", achieved=value * per_report_h2d / 1e9, peak=63.0,
                             unit="GB/s host->device (the report bytes each job hands over)",
                             frac=value * per_report_h2d / 63e9,
                             frac_of_measured_link=value * per_report_h2d / 57e9,
                             note="measured link: 55-57 GB/s for 16-64 MB pinned copies and kernel "
                                  "reads of mapped host memory (tools/ubench_h2d.hip, "
                                  "profiles/r03/r03i_h2d.txt)", traffic=None),
               host=host_side,
               coalescing=dict(launches=launches, jobs=n_jobs,
                               mean_reports_per_launch=n_jobs * js / max(launches, 1)),
               call=("prio3_helper_prepare_aggregate_batch (one coalesced launch per group)"
                     if combined else "prio3_helper_prepare_batch + prio3_accumulate"),
               checks=dict(all_finished=bool((status == 0).all()),
                           counts_ok=bool((counts == js).all()),
                           every_job_matches_cpu=jobs_ok, statuses_match_cpu=statuses_ok,
                           jobs_checked=sum(len(range(t, n_jobs, K)) for t in
                                            range(K if check_tasks is None else min(K, check_tasks))),
                           check_seconds=t_chk),
               cpu_baseline=cpu,
               speedup_vs_cpu=(value / cpu["value"]) if cpu else None)


def leader_jobs_line(T, js, n_jobs, K, devices=None, with_cpu=True, cpu_seconds=10.0, heavy=0,
                     combined=True):
    """the leader's production call shape.  T host threads, each a worker of
    Janus's aggregation job driver stepping whole jobs (aggregation_job_driver.rs:397-415,
    677-691, one spawn per job at :449-462): prio3_leader_prepare_init_batch on the job's explicit
    leader input shares, prio3_leader_prepare_next_batch on the helper's prepare messages,
    prio3_accumulate, prio3_batch_free -- host buffers, PCIe included, coalesced by the leader
    executors.  Every job's prepare shares, statuses, aggregate and count are checked against
    the restatement's leader path (orc_leader_batch_seg)."""
    import ctypes as C
    torch.cuda.set_device(0)
    n_jobs = max(K, n_jobs)
    pool = 1 << 15
    vks = [bytes([0x61 + t]) * 16 for t in range(K)]
    engines, devs = _job_engines(J.Prio3Histogram(256, 16), vks, devices)
    engines[0].executor_control("heavy", heavy)
    sz = engines[0].sz
    cols = {k: [] for k in ("nonces", "public_shares", "leader_input_shares", "msgs")}
    for t, e in enumerate(engines):
        p = e.generate_reports_device(pool, seed=0x4A414E5553000005 + t, with_leader_inputs=True)
        msgs = torch.empty((pool, sz.prep_msg_len), dtype=torch.uint8, device=p["nonces"].device)
        st = torch.empty(pool, dtype=torch.uint8, device=p["nonces"].device)
        # the helper's prepare messages: the engine's own device helper prepare of the pool
        e.prepare_device(p["nonces"], p["public_shares"], p["helper_shares"],
                         p["leader_prep_shares"], msgs, st)
        torch.cuda.synchronize()
        assert int((st != 0).sum().item()) == 0
        for k in ("nonces", "public_shares", "leader_input_shares"):
            cols[k].append(p[k].cpu().numpy())
        cols["msgs"].append(msgs.cpu().numpy())
        del p, msgs, st
    host = {k: np.ascontiguousarray(np.concatenate(v)) for k, v in cols.items()}
    lib = C.CDLL(os.path.join(ROOT, "janus_amd", "libjanus_jobs.so"))
    lib.janus_jobs_run_leader.restype = C.c_double
    vp = C.c_void_p
    lib.janus_jobs_run_leader.argtypes = [C.POINTER(vp), C.c_int, vp, C.c_int, C.c_int, C.c_int,
                                          C.c_uint32, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int]
    eng_arr = (vp * K)(*[e.handle.value for e in engines])
    ps = np.zeros((n_jobs * js, sz.prep_share_len), np.uint8)
    status = np.zeros(n_jobs * js, np.uint8)
    counts = np.zeros(n_jobs, np.uint64)
    agg = np.zeros((n_jobs, sz.agg_share_len), np.uint8)
    _warm(ps, status, counts, agg)
    P = lambda a: a.ctypes.data_as(vp)

    def run(jobs):
        status[:] = 0xFF
        return lib.janus_jobs_run_leader(eng_arr, K, C.cast(C.pointer(sz), vp), T, jobs, js, pool,
                                         P(host["nonces"]), P(host["public_shares"]),
                                         P(host["leader_input_shares"]), P(host["msgs"]), P(ps),
                                         P(status), P(counts), P(agg), int(combined))

    run(max(K, min(n_jobs, 8 * T)))  # warmup
    g0 = [engines[0].executor_stats(k)["groups"] for k in (J.EXEC_LEADER_INIT,
                                                          J.EXEC_LEADER_NEXT)]
    pl0 = _placement(engines)
    dt, host_side = _host_timed(lambda: run(n_jobs))
    if dt < 0:
        raise RuntimeError("janus_jobs_run_leader: a C-ABI call failed")
    placement = _placement(engines, pl0)
    g1 = [engines[0].executor_stats(k)["groups"] for k in (J.EXEC_LEADER_INIT,
                                                          J.EXEC_LEADER_NEXT)]
    value = n_jobs * js / dt
    from oracle.oracle import Oracle
    o = Oracle("histogram", length=256, chunk_length=16)
    t_chk = time.perf_counter()
    jobs_ok = statuses_ok = ps_ok = True
    for t in range(K):
        jl, idx = _job_windows(t, n_jobs, K, js, pool)
        seg = np.repeat(np.arange(len(jl), dtype=np.uint32), js)
        rps, rst, ragg, rcnt = o.leader_batch(
            vks[t], host["nonces"][idx], host["public_shares"][idx],
            host["leader_input_shares"][idx], host["msgs"][idx], n_threads=cpu_threads(),
            job_size=js, segment_ids=seg, n_segments=len(jl))
        rows = np.concatenate([np.arange(j * js, (j + 1) * js) for j in jl])
        ps_ok &= bool(np.array_equal(ps[rows], rps))
        statuses_ok &= bool(np.array_equal(status[rows], rst))
        jobs_ok &= bool(np.array_equal(agg[jl], ragg) and
                        np.array_equal(counts[jl], rcnt.astype(np.uint64)))
    t_chk = time.perf_counter() - t_chk
    cores = cpu_threads()
    cpu = None
    if with_cpu:
        def cpu_run(m):
            o.leader_batch(vks[0], host["nonces"][:m], host["public_shares"][:m],
                           host["leader_input_shares"][:m], host["msgs"][:m], n_threads=cores,
                           job_size=js)
        rate, sample = _cpu_waves(cpu_run, cores, js, pool, max(2.0, cpu_seconds))
        cpu = dict(value=rate, unit="reports/s", cores=cores, kind="port",
                   sample="the restatement's leader path (prepare_init agg_id 0 + prepare_next + "
                          "aggregate): " + sample, cpu_model=cpu_model())
    h2d = 16 + sz.public_share_len + sz.leader_input_share_len + sz.prep_msg_len
    return dict(metric="leader reports prepared (init + next) + aggregated/sec through the "
                       "host-buffer C ABI (Prio3Histogram len=256, concurrent aggregation jobs)",
                value=value, unit="reports/s", n_gpus=len(set(devs)), steps=1, warmup=1,
                ms_per_step=dt * 1e3, higher_is_better=True, scaling="weak", vs_baseline=None,
                dtype="u32 limbs (Field128 mod-p integer arithmetic)",
                data=f"synthetic: {K} x {pool} on-device client reports (leader input shares) "
                     "and the helper's prepare messages, copied to host memory",
                config=dict(workload="Prio3Histogram length=256 chunk_length=16 leader "
                                     "prepare_init + prepare_next + accumulate per aggregation "
                                     "job, host buffers (PCIe included)",
                            job_size=js, jobs=n_jobs, threads=T, tasks=K, devices=devs),
                placement=placement,
                roofline=dict(bound="pcie", achieved=value * h2d / 1e9, peak=63.0,
                              unit="GB/s host->device (leader input share, nonce, public share, "
                                   "prepare message per report)",
                              frac=value * h2d / 63e9, h2d_bytes_per_report=h2d, traffic=None),
                host=host_side,
               coalescing=dict(init_launches=g1[0] - g0[0], next_launches=g1[1] - g0[1],
                                jobs=n_jobs),
                call=("prio3_leader_prepare_init_batch + prio3_leader_prepare_next_aggregate_batch"
                      if combined else "prio3_leader_prepare_init_batch + "
                      "prio3_leader_prepare_next_batch + prio3_accumulate"),
                checks=dict(all_finished=bool((status == 0).all()),
                            counts_ok=bool((counts == js).all()), prep_shares_match_cpu=ps_ok,
                            statuses_match_cpu=statuses_ok, every_job_matches_cpu=jobs_ok,
                            jobs_checked=n_jobs, check_seconds=t_chk),
                cpu_baseline=cpu, speedup_vs_cpu=(value / cpu["value"]) if cpu else None)


def hpke_jobs_line(T, js, n_jobs, K, with_cpu=True, cpu_seconds=10.0, heavy=0):
    """the helper's input-share open at the production call shape -- T host
    threads each opening whole jobs' input shares (aggregator.rs:1847-1890) through
    janus_hpke_open_input_shares (host buffers, PCIe included), K tasks (their own AAD task IDs)
    under one X25519 keypair, coalesced by the GPU's HPKE executor.  Every job's helper shares and
    statuses are checked against the restatement (OpenSSL)."""
    import ctypes as C
    from janus_amd import hpke as G
    from oracle import hpke as H
    torch.cuda.set_device(0)
    n_jobs = max(K, n_jobs)
    pool = 1 << 15
    rng = np.random.default_rng(0x4A414E55)
    skR = H.kem_private(rng)
    parts = [H.make_batch_fast(pool, 48, 32, seed=0x4A41 + t, skR=skR, n_threads=cpu_threads())
             for t in range(K)]
    host = {k: np.ascontiguousarray(np.concatenate([p[k] for p in parts]))
            for k in ("enc", "ct", "ct_len", "report_ids", "times", "pubs")}
    task_ids = np.frombuffer(b"".join(p["task_id"] for p in parts), np.uint8).copy()
    stride = host["ct"].shape[1]
    op = G.HpkeOpener(skR, H.kem_public(skR), device=0)
    op.executor_control("heavy", heavy)
    lib = C.CDLL(os.path.join(ROOT, "janus_amd", "libjanus_jobs.so"))
    lib.janus_jobs_run_hpke.restype = C.c_double
    vp, u32 = C.c_void_p, C.c_uint32
    lib.janus_jobs_run_hpke.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, u32, u32, vp,
                                        vp, vp, u32, vp, vp, vp, u32, u32, vp, vp]
    shares = np.zeros((n_jobs * js, 48), np.uint8)
    status = np.zeros(n_jobs * js, np.uint8)
    _warm(shares, status)
    P = lambda a: a.ctypes.data_as(vp)

    def run(jobs):
        status[:] = 0xFF
        return lib.janus_jobs_run_hpke(op.handle, K, P(task_ids), T, jobs, js, pool, 32,
                                       P(host["enc"]), P(host["ct"]), P(host["ct_len"]), stride,
                                       P(host["report_ids"]), P(host["times"]), P(host["pubs"]),
                                       32, 48, P(shares), P(status))

    run(max(K, min(n_jobs, 8 * T)))  # warmup
    g0 = op.executor_stats()["groups"]
    dt, host_side = _host_timed(lambda: run(n_jobs))
    if dt < 0:
        raise RuntimeError("janus_jobs_run_hpke: a C-ABI call failed")
    launches = op.executor_stats()["groups"] - g0
    value = n_jobs * js / dt
    t_chk = time.perf_counter()
    ok = True
    for t in range(K):
        d = parts[t]
        rsh, rst = H.open_input_shares(skR, d["pkR"], d["task_id"], d["enc"], d["ct"],
                                       d["ct_len"], d["report_ids"], d["times"], d["pubs"], 48,
                                       n_threads=cpu_threads())
        jl, idx = _job_windows(t, n_jobs, K, js, pool)
        rows = np.concatenate([np.arange(j * js, (j + 1) * js) for j in jl])
        ok &= bool(np.array_equal(shares[rows], rsh[idx - t * pool]) and
                   np.array_equal(status[rows], rst[idx - t * pool]))
    t_chk = time.perf_counter() - t_chk
    cores = cpu_threads()
    cpu = None
    if with_cpu:
        d = parts[0]

        def cpu_run(m):
            H.open_input_shares(skR, d["pkR"], d["task_id"], d["enc"][:m], d["ct"][:m],
                                d["ct_len"][:m], d["report_ids"][:m], d["times"][:m],
                                d["pubs"][:m], 48, n_threads=cores)
        rate, sample = _cpu_waves(cpu_run, cores, js, pool, max(2.0, cpu_seconds))
        cpu = dict(value=rate, unit="reports/s", cores=cores, kind="port",
                   sample="sealed input shares, OpenSSL 3.0 X25519 / HKDF-SHA256 / AES-128-GCM: "
                          + sample, cpu_model=cpu_model())
    h2d = 32 + stride + 4 + 16 + 8 + 32
    roofline = model_roofline("hpke_x25519_aead1", RM.hpke_model("x25519", 1), n_jobs * js, 1, dt)
    roofline["pcie"] = dict(h2d_bytes_per_report=h2d, frac=value * h2d / 63e9)
    return dict(metric="helper input shares HPKE-opened+decoded/sec through the host-buffer C ABI "
                       "(X25519-HKDF-SHA256, AES-128-GCM, concurrent aggregation jobs)",
                value=value, unit="reports/s", n_gpus=1, steps=1, warmup=1, ms_per_step=dt * 1e3,
                higher_is_better=True, scaling="weak", vs_baseline=None,
                dtype="u32 limbs (GF(2^255 - 19), GF(2^128), bytes)",
                data=f"synthetic: {K} tasks x {pool} input shares sealed by the oracle (OpenSSL, "
                     "seeded), host memory",
                config=dict(workload="DAP helper input share open per aggregation job: X25519 "
                                     "decap + HPKE key schedule + AES-128-GCM + PlaintextInputShare "
                                     "decode, Prio3Histogram(256,16) shares, host buffers",
                            job_size=js, jobs=n_jobs, threads=T, tasks=K),
                roofline=roofline, host=host_side,
                coalescing=dict(launches=launches, jobs=n_jobs),
                checks=dict(all_opened=bool((status == 0).all()), every_job_matches_cpu=ok,
                            jobs_checked=n_jobs, check_seconds=t_chk),
                cpu_baseline=cpu, speedup_vs_cpu=(value / cpu["value"]) if cpu else None)


def init_jobs_line(T, js, n_jobs, K, with_cpu=True, cpu_seconds=10.0, heavy=0, two_call=True):
    """the helper's whole loop body at the production call shape -- T host
    threads, each running whole aggregation jobs from the SEALED input shares
    (VdafOps::handle_aggregate_init_generic, aggregator.rs:1794-2096) through
    prio3_helper_aggregate_init_batch: HPKE open, decode, prepare and accumulate in one coalesced
    launch per group, the decrypted shares kept in HBM.  K tasks (verify keys and task IDs) of
    Prio3Histogram(256,16) under one X25519 keypair.  Beside it, in the same run, the two-call
    composition (janus_hpke_open_input_shares, then prio3_helper_prepare_aggregate_batch).  Every
    job's statuses, aggregate and count are checked against OpenSSL + the restatement."""
    import ctypes as C
    from janus_amd import hpke as G
    from oracle import hpke as H
    from oracle.oracle import Oracle
    torch.cuda.set_device(0)
    n_jobs = max(K, n_jobs)
    pool = 1 << 15
    rng = np.random.default_rng(0x4A414E56)
    vks = [bytes([0x81 + t]) * 16 for t in range(K)]
    tasks = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(K)]
    skR = H.kem_private(rng)
    pkR = H.kem_public(skR)
    engines, devs = _job_engines(J.Prio3Histogram(256, 16), vks, None)
    engines[0].executor_control("heavy", heavy)
    sz = engines[0].sz
    cores = cpu_threads()
    cols = {k: [] for k in ("nonces", "public_shares", "helper_shares", "leader_prep_shares",
                            "times", "enc", "ct", "ct_len")}
    stride = None
    for t, e in enumerate(engines):
        p = e.generate_reports_device(pool, seed=0x4A414E5553000007 + t)
        torch.cuda.synchronize()
        h = {k: p[k].cpu().numpy() for k in ("nonces", "public_shares", "helper_shares",
                                              "leader_prep_shares")}
        del p
        times = (1_700_000_000 + rng.integers(0, 3600, pool)).astype(np.uint64)
        enc, ct, cl, stride = H.seal_input_shares(pkR, tasks[t], h["nonces"], times,
                                                  h["public_shares"], h["helper_shares"],
                                                  seed=0x5EA1 + t, n_threads=cores)
        for k, v in dict(h, times=times, enc=enc, ct=ct, ct_len=cl).items():
            cols[k].append(v)
    host = {k: np.ascontiguousarray(np.concatenate(v)) for k, v in cols.items()}
    task_arr = np.frombuffer(b"".join(tasks), np.uint8).copy()
    op = G.HpkeOpener(skR, pkR, device=0)
    lib = C.CDLL(os.path.join(ROOT, "janus_amd", "libjanus_jobs.so"))
    lib.janus_jobs_run_init.restype = C.c_double
    vp, u32 = C.c_void_p, C.c_uint32
    lib.janus_jobs_run_init.argtypes = [C.POINTER(vp), C.c_int, vp, vp, vp, C.c_int, C.c_int,
                                        C.c_int, u32, vp, vp, vp, vp, u32, vp, vp, u32, vp, vp, vp,
                                        vp, C.c_int]
    eng_arr = (vp * K)(*[e.handle.value for e in engines])
    status = np.zeros(n_jobs * js, np.uint8)
    counts = np.zeros(n_jobs, np.uint64)
    agg = np.zeros((n_jobs, sz.agg_share_len), np.uint8)
    _warm(status, counts, agg)
    P = lambda a: a.ctypes.data_as(vp)

    def run(jobs, one_call):
        status[:] = 0xFF
        counts[:] = 0
        return lib.janus_jobs_run_init(eng_arr, K, C.cast(C.pointer(sz), vp), op.handle,
                                       P(task_arr), T, jobs, js, pool, P(host["nonces"]),
                                       P(host["public_shares"]), P(host["times"]), P(host["enc"]),
                                       32, P(host["ct"]), P(host["ct_len"]), stride,
                                       P(host["leader_prep_shares"]), P(status), P(counts), P(agg),
                                       int(one_call))

    # the reference the jobs are checked against: OpenSSL opens each task's pool, the restatement
    # prepares + aggregates every job's window of it
    o = Oracle("histogram", length=256, chunk_length=16)
    opened = []
    for t in range(K):
        sl = slice(t * pool, (t + 1) * pool)
        sh, hs = H.open_input_shares(skR, pkR, tasks[t], host["enc"][sl], host["ct"][sl],
                                     host["ct_len"][sl], host["nonces"][sl], host["times"][sl],
                                     host["public_shares"][sl], sz.helper_share_len,
                                     n_threads=cores)
        assert (hs == 0).all()
        opened.append(sh)

    def check():
        ok_jobs = ok_st = True
        for t in range(K):
            jl, idx = _job_windows(t, n_jobs, K, js, pool)
            seg = np.repeat(np.arange(len(jl), dtype=np.uint32), js)
            _, rst, ragg, rcnt = o.helper_batch(
                vks[t], host["nonces"][idx], host["public_shares"][idx], opened[t][idx - t * pool],
                host["leader_prep_shares"][idx], segment_ids=seg, n_segments=len(jl),
                n_threads=cores)
            ok_jobs &= bool(np.array_equal(agg[jl], ragg) and
                            np.array_equal(counts[jl], rcnt.astype(np.uint64)))
            ok_st &= bool(np.array_equal(status.reshape(n_jobs, js)[jl], rst.reshape(-1, js)))
        return ok_jobs, ok_st

    run(max(K, min(n_jobs, 8 * T)), True)  # warmup: pools, pinned staging, streams
    g0 = engines[0].executor_stats(J.EXEC_PREPARE)["groups"]
    dt, host_side = _host_timed(lambda: run(n_jobs, True))
    if dt < 0:
        raise RuntimeError("janus_jobs_run_init: a C-ABI call failed")
    launches = engines[0].executor_stats(J.EXEC_PREPARE)["groups"] - g0
    value = n_jobs * js / dt
    t_chk = time.perf_counter()
    jobs_ok, st_ok = check()
    all_fin = bool((status == 0).all())
    cnt_ok = bool((counts == js).all())
    t_chk = time.perf_counter() - t_chk
    two = None
    if two_call:
        run(max(K, min(n_jobs, 8 * T)), False)
        dt2 = run(n_jobs, False)
        if dt2 < 0:
            raise RuntimeError("janus_jobs_run_init (two calls): a C-ABI call failed")
        j2, s2 = check()
        two = dict(value=n_jobs * js / dt2, ms=dt2 * 1e3, every_job_matches_cpu=j2,
                   statuses_match_cpu=s2,
                   call="janus_hpke_open_input_shares + prio3_helper_prepare_aggregate_batch")
    cpu = None
    if with_cpu:
        def cpu_run(m):  # the helper's CPU loop body: OpenSSL open, then the restatement
            sh, _ = H.open_input_shares(skR, pkR, tasks[0], host["enc"][:m], host["ct"][:m],
                                        host["ct_len"][:m], host["nonces"][:m], host["times"][:m],
                                        host["public_shares"][:m], sz.helper_share_len,
                                        n_threads=cores)
            o.helper_batch(vks[0], host["nonces"][:m], host["public_shares"][:m], sh,
                           host["leader_prep_shares"][:m], n_threads=cores, job_size=js)
        rate, sample = _cpu_waves(cpu_run, cores, js, pool, max(2.0, cpu_seconds))
        cpu = dict(value=rate, unit="reports/s", cores=cores, kind="port",
                   sample="OpenSSL 3.0 HPKE open + the restatement's helper prepare + aggregate: "
                          + sample, cpu_model=cpu_model())
    h2d = 16 + sz.public_share_len + 8 + 32 + stride + 4 + sz.prep_share_len
    return dict(metric="reports opened+prepared+aggregated/sec through the host-buffer C ABI "
                       "(helper aggregate-init loop body from sealed input shares, Prio3Histogram "
                       "len=256, X25519/AES-128-GCM, concurrent aggregation jobs)",
                value=value, unit="reports/s", n_gpus=len(set(devs)), steps=1, warmup=1,
                ms_per_step=dt * 1e3, higher_is_better=True, scaling="weak", vs_baseline=None,
                dtype="u32 limbs (Field128 mod-p, GF(2^255 - 19), GF(2^128), bytes)",
                data=f"synthetic: {K} tasks x {pool} on-device client reports, helper input "
                     "shares sealed by the oracle (OpenSSL, seeded), host memory",
                config=dict(workload="VdafOps::handle_aggregate_init_generic loop body per "
                                     "aggregation job: HPKE open + PlaintextInputShare decode + "
                                     "Prio3Histogram(256,16) helper prepare + accumulate, host "
                                     "buffers (PCIe included)",
                            job_size=js, jobs=n_jobs, threads=T, tasks=K, devices=devs),
                roofline=dict(bound="pcie", achieved=value * h2d / 1e9, peak=63.0,
                              unit="GB/s host->device (report ID, time, public share, HPKE "
                                   "ciphertext, leader prep share per report)",
                              frac=value * h2d / 63e9, h2d_bytes_per_report=h2d, traffic=None),
                host=host_side,
               coalescing=dict(launches=launches, jobs=n_jobs,
                                mean_reports_per_launch=n_jobs * js / max(launches, 1)),
                call="prio3_helper_aggregate_init_batch (one coalesced launch per group)",
                two_call=two,
                checks=dict(all_finished=all_fin, counts_ok=cnt_ok,
                            every_job_matches_cpu=jobs_ok, statuses_match_cpu=st_ok,
                            jobs_checked=n_jobs, check_seconds=t_chk),
                cpu_baseline=cpu, speedup_vs_cpu=(value / cpu["value"]) if cpu else None)


def leader_main(args):
    """Leader-side line (not the BASELINE metric): one step = leader prepare_init (agg_id 0) on
    the explicit input shares + prepare_next on the helper's prepare messages + accumulate,
    for a Histogram(256,16) batch (or Prio3Sum(32) at C4's per-GPU share with
    --leader-vdaf sum32).  The prepare messages are the helper engine's own output on the same
    reports, computed once before timing."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    hist = args.leader_vdaf == "hist"
    n = args.reports if (hist or args.reports != 1 << 20) else 10_000_000 // 8
    eng = J.HelperEngine(J.Prio3Histogram(256, 16) if hist else J.Prio3Sum(32), VK, device=0)
    for kv in args.opt:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    sz = eng.sz
    data = eng.generate_reports_device(n, seed=0x4A414E5553000002, with_checks=True,
                                       with_leader_inputs=True)
    u8 = dict(dtype=torch.uint8, device=dev)
    msgs = torch.empty((n, 16), **u8)
    status = torch.empty(n, **u8)
    eng.prepare_device(data["nonces"], data["public_shares"], data["helper_shares"],
                       data["leader_prep_shares"], msgs, status)
    torch.cuda.synchronize()
    helper_ok = int((status == 0).sum().item())
    prep = torch.empty((n, sz.prep_share_len), **u8)
    lstatus = torch.empty(n, **u8)
    agg = torch.zeros((1, sz.agg_share_len), **u8)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)

    def step():
        eng.leader_prepare_init_device(data["nonces"], data["public_shares"],
                                       data["leader_input_shares"], prep, lstatus)
        eng.leader_prepare_next_device(n, msgs, lstatus)
        eng.accumulate_device(n, lstatus, None, None, 1, agg, cnt)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.set_option("timing", 1)
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    times = eng.timing()
    per_kernel = {k: dict(ms_total=v[0], launches=v[1], ms_avg=v[0] / max(v[1], 1))
                  for k, v in times.items()}
    same = bool(torch.equal(prep, data["leader_prep_shares"]))
    name = "Prio3Histogram len=256" if hist else "Prio3Sum bits=32"
    out = dict(metric=f"reports prepared+aggregated/sec (leader, {name})",
               value=n * args.steps / elapsed, unit="reports/s", n_gpus=1, steps=args.steps,
               warmup=args.warmup, ms_per_step=elapsed / args.steps * 1e3,
               higher_is_better=True, scaling="weak", vs_baseline=None,
               dtype="u32 limbs (Field128 mod-p integer arithmetic)",
               data="synthetic: on-device client reports (leader input shares explicit)",
               config=dict(workload=("Prio3Histogram length=256 chunk_length=16" if hist else
                                     "Prio3Sum bits=32") + " leader prepare_init+prepare_next+"
                                    "aggregate", reports_per_gpu=n),
               kernels=per_kernel,
               roofline=model_roofline(f"leader_{args.leader_vdaf}", RM.leader_model(
                   RM.instance("histogram", sz, length=256, chunk=16) if hist else
                   RM.instance("sum", sz, bits=32)), n, args.steps, elapsed),
               checks=dict(helper_finished=helper_ok,
                           leader_finished=int((lstatus == 0).sum().item()),
                           leader_prep_shares_equal_generator=same, agg_count=int(cnt[0].item())),
               cpu_baseline=None)
    if not args.no_cpu_baseline:
        # the C restatement's leader path (orc_leader_batch: prepare_init agg_id 0 +
        # prepare_next + aggregate in Janus-sized jobs) on a bounded sample of the same reports
        from oracle.oracle import Oracle, build
        build()
        o = (Oracle("histogram", length=256, chunk_length=16) if hist else
             Oracle("sum", bits=32))
        th = cpu_threads()
        host = [t.cpu().numpy() for t in (data["nonces"], data["public_shares"],
                                          data["leader_input_shares"], msgs)]

        def crun(m):
            t1 = time.perf_counter()
            r = o.leader_batch(VK, *(h[:m] for h in host), n_threads=th, job_size=500)
            return time.perf_counter() - t1, r

        probe = min(n, 500 * th)
        dt, _ = crun(probe)
        m = int(min(n, max(probe, probe * args.cpu_seconds / max(dt, 1e-6))))
        dt, (cps, cst, cagg, ccnt) = crun(m)
        out["cpu_baseline"] = dict(value=m / dt, unit="reports/s", cores=th, kind="port",
                                   sample=f"{m} of the same reports through the C restatement's "
                                          f"leader path (oracle/prio3_oracle.c orc_leader_batch), "
                                          f"jobs of 500, {th} threads, {dt:.1f}s wall")
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
        agg_s = torch.zeros_like(agg)
        cnt_s = torch.zeros_like(cnt)
        eng.accumulate_device(m, lstatus[:m], None, None, 1, agg_s, cnt_s)
        torch.cuda.synchronize()
        out["checks"]["cpu_gpu_parity_on_sample"] = bool(
            np.array_equal(lstatus[:m].cpu().numpy(), cst) and
            np.array_equal(prep[:m].cpu().numpy(), cps) and
            np.array_equal(agg_s.cpu().numpy(), cagg) and int(cnt_s[0].item()) == int(ccnt[0]))
    print(json.dumps(out), flush=True)


def hpke_main(args):
    """Batched HPKE open line (not the BASELINE metric): one step = decrypt +
    PlaintextInputShare decode of n helper input shares of Prio3Histogram(256,16) (48-byte
    helper shares, 32-byte public shares) with DHKEM(X25519, HKDF-SHA256)/AES-128-GCM -- the
    per-report hpke::open of aggregator.rs:1796-1990.  Inputs are sealed on the host by the
    oracle (OpenSSL, seeded) and resident in HBM before timing."""
    from janus_amd import hpke as G
    from oracle import hpke as H
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = args.reports
    uniq = min(n, 1 << 18)
    t0 = time.perf_counter()
    aead = args.hpke_aead
    aead_name = {1: "AES-128-GCM", 2: "AES-256-GCM", 3: "ChaCha20Poly1305"}[aead]
    kem = dict(x25519=H.KEM_X25519, p256=H.KEM_P256, x448=H.KEM_X448, p521=H.KEM_P521,
               p384=H.KEM_P384)[args.hpke_kem]
    kem_name = dict(x25519="X25519", p256="P256", x448="X448", p521="P521",
                    p384="P384")[args.hpke_kem]
    # each KEM with its own KDF in the key schedule too (the suites of the RFC 9180 vectors)
    kdf = {"x448": H.KDF_SHA512, "p521": H.KDF_SHA512, "p384": H.KDF_SHA384}.get(args.hpke_kem,
                                                                             H.KDF_SHA256)
    kdf_name = {H.KDF_SHA256: "HKDF-SHA256", H.KDF_SHA384: "HKDF-SHA384",
                H.KDF_SHA512: "HKDF-SHA512"}[kdf]
    d = H.make_batch_fast(uniq, 48, 32, seed=0x4A414E55, n_threads=cpu_threads(), aead=aead,
                          kem=kem, kdf=kdf)
    gen_s = time.perf_counter() - t0
    reps = -(-n // uniq)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(np.concatenate([a] * reps)[:n])).to(dev)
    enc, ct, ct_len = T(d["enc"]), T(d["ct"]), T(d["ct_len"].view(np.int32))
    ids, times, pubs = T(d["report_ids"]), T(d["times"].view(np.int64)), T(d["pubs"])
    shares = torch.empty((n, 48), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    op = G.HpkeOpener(d["skR"], d["pkR"], device=0, aead_id=aead, kem_id=kem, kdf_id=kdf)

    def step():
        op.open_input_shares_device(d["task_id"], enc, ct, ct_len, ids, times, pubs, shares,
                                    status, stream=torch.cuda.current_stream().cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    op.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms_total, launches = op.timing()
    op.set_timing(False)
    value = n * args.steps / elapsed
    ms_avg = ms_total / max(launches, 1)
    roofline = model_roofline(f"hpke_{args.hpke_kem}_aead{aead}",
                              RM.hpke_model(args.hpke_kem, aead), n, args.steps, elapsed)
    roofline.update(kernel="k_hpke_open", ms_avg=ms_avg)
    ok = int((status == 0).sum().item())
    out = dict(metric=f"helper input shares HPKE-opened+decoded/sec ({kem_name}-{kdf_name}, "
                      f"{aead_name})", value=value, unit="reports/s", n_gpus=1, steps=args.steps,
               warmup=args.warmup, ms_per_step=elapsed / args.steps * 1e3, higher_is_better=True,
               scaling="weak", vs_baseline=None, dtype="u32 limbs (the KEM field, GF(2^128), bytes)",
               data=f"synthetic: {uniq} distinct sealed input shares (oracle/OpenSSL, seeded) "
                    f"tiled x{reps}; generation {gen_s:.1f}s, not timed",
               config=dict(workload=f"DAP helper input share open: {kem_name} decap + HPKE key "
                                    f"schedule + {aead_name} + PlaintextInputShare decode, "
                                    "Prio3Histogram(256,16) shares", reports=n),
               roofline=roofline, kernel_ms_avg=ms_avg, checks=dict(opened=ok))
    if not args.no_cpu_baseline:
        th = cpu_threads()
        m = min(uniq, max(4096, int(16000 * th * args.cpu_seconds / 10)))
        t0 = time.perf_counter()
        csh, cst = H.open_input_shares(d["skR"], d["pkR"], d["task_id"], d["enc"][:m],
                                       d["ct"][:m], d["ct_len"][:m], d["report_ids"][:m],
                                       d["times"][:m], d["pubs"][:m], 48, n_threads=th,
                                       aead=aead, kem=kem, kdf=kdf)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = dict(value=m / dt, unit="reports/s", cores=th, kind="port",
                                   sample=f"{m} of the sealed input shares, OpenSSL 3.0 {kem_name} / "
                                          f"{kdf_name} / {aead_name}, {th} threads, {dt:.1f}s")
        out["speedup_vs_cpu"] = value / (m / dt)
        out["checks"]["cpu_gpu_parity_on_sample"] = bool(
            np.array_equal(shares[:m].cpu().numpy(), csh) and
            np.array_equal(status[:m].cpu().numpy(), cst))
    print(json.dumps(out), flush=True)


def pipeline_main(args):
    """Whole helper aggregation-job init on the device, request bytes to response bytes (not
    the BASELINE metric): janus_dap unpack of the AggregationJobInitializeReq body -> HPKE open
    of the helper input shares -> prio3 prepare + aggregate + batch metadata -> AggregationJobResp
    encode.  The request body (Prio3Histogram(256,16), X25519/AES-128-GCM, 738 B per report)
    is resident in HBM before timing; aggregator.rs:1720-2096 per report in Janus."""
    from janus_amd import dap as DJ
    from janus_amd import hpke as G
    from oracle import hpke as H
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = args.reports
    th = cpu_threads()
    eng = J.HelperEngine(J.Prio3Histogram(256, 16), VK, device=0)
    t0 = time.perf_counter()
    d = eng.generate_reports_device(n, seed=0x4A414E5553000002)
    host = {k: d[k].cpu().numpy() for k in ("nonces", "public_shares", "helper_shares",
                                             "leader_prep_shares")}
    rng = np.random.default_rng(7)
    skR = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    pkR = H.x25519_public(skR)
    task = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    times = (1_700_000_000 + rng.integers(0, 3600, n)).astype(np.uint64)
    enc, ct, ct_len, _ = H.seal_input_shares(pkR, task, host["nonces"], times,
                                             host["public_shares"], host["helper_shares"],
                                             seed=11, n_threads=th)
    pl = int(ct_len[0])
    L = host["leader_prep_shares"].shape[1]
    rec = 16 + 8 + 4 + 32 + 1 + 2 + 32 + 4 + pl + 4 + 1 + 4 + L
    R = np.zeros((n, rec), np.uint8)
    be = lambda v, w: np.array([v], dtype=f">u{w}").view(np.uint8)
    o = 0
    for part in (host["nonces"], times.astype(">u8").view(np.uint8).reshape(n, 8),
                 np.tile(be(32, 4), (n, 1)), host["public_shares"], np.full((n, 1), 1, np.uint8),
                 np.tile(be(32, 2), (n, 1)), enc, np.tile(be(pl, 4), (n, 1)), ct[:, :pl],
                 np.tile(be(5 + L, 4), (n, 1)), np.zeros((n, 1), np.uint8),
                 np.tile(be(L, 4), (n, 1)), host["leader_prep_shares"]):
        R[:, o:o + part.shape[1]] = part
        o += part.shape[1]
    body = (be(0, 4).tobytes() + b"\x01" + be(n * rec, 4).tobytes() + R.tobytes())
    gen_s = time.perf_counter() - t0
    # the task's expected lengths (VDAF public share, X25519 Nenc, leader prep share): every record
    # is checked against them, as the handler knows them from the task
    lay = DJ.scan(body, public_share_len=32, enc_len=32, prep_share_len=L)
    assert lay.uniform and lay.n == n
    d_body = torch.zeros(len(body) + 8, dtype=torch.uint8, device=dev)
    d_body[:len(body)] = torch.frombuffer(bytearray(body), dtype=torch.uint8).to(dev)
    stride = DJ.ct_stride_for(lay)
    op = G.HpkeOpener(skR, pkR, device=0)
    shares = torch.empty((n, 48), dtype=torch.uint8, device=dev)
    hs = torch.empty(n, dtype=torch.uint8, device=dev)
    msgs = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    agg = torch.zeros((1, eng.sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    cks = torch.zeros((1, 32), dtype=torch.uint8, device=dev)
    ivs = torch.zeros((1, 2), dtype=torch.int64, device=dev)
    res = {}

    def step():
        s = torch.cuda.current_stream().cuda_stream
        u, mism = DJ.unpack_device(lay, d_body, stride, stream=s)
        op.open_input_shares_device(task, u["enc"], u["ct"], u["ct_len"], u["report_ids"],
                                    u["times"], u["public_shares"], shares, hs, stream=s)
        eng.prepare_aggregate_device(u["report_ids"], u["public_shares"], shares,
                                     u["prep_shares"], seg, 1, msgs, st, stream=s)
        accept = ((hs == 0) & (u["msg_status"] == 0)).to(torch.uint8)
        eng.aggregate_finish_device(st, accept, agg, cnt, stream=s)
        st_all = st | u["msg_status"]
        eng.batch_metadata_device(u["report_ids"], u["times"], st_all, accept, seg, 1, cks, ivs,
                                  stream=s)
        pe = DJ.prepare_error(hs, u["msg_status"])
        res["out"], res["len"] = DJ.encode_resp_device(u["report_ids"], pe, st_all, msgs, 16,
                                                       stream=s)
        res["mism"] = mism

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    value = n * args.steps / elapsed
    resp_len = int(res["len"][0])
    ok = int((st == 0).sum().item())
    out = dict(metric="helper aggregation-job init reports/sec, request bytes to response bytes "
                      "(DAP unpack + HPKE open + Prio3Histogram(256,16) prepare/aggregate + "
                      "response encode)", value=value, unit="reports/s", n_gpus=1,
               steps=args.steps, warmup=args.warmup, ms_per_step=elapsed / args.steps * 1e3,
               higher_is_better=True, scaling="weak", vs_baseline=None,
               dtype="u32 limbs / bytes",
               data=f"synthetic: {n} distinct reports (device client + oracle HPKE seal), one "
                    f"{len(body) / 1e6:.0f} MB request body resident in HBM; generation "
                    f"{gen_s:.1f}s, not timed",
               config=dict(workload="DAP-09 AggregationJobInitializeReq -> AggregationJobResp, "
                                    "helper, Prio3Histogram(256,16), X25519-HKDF-SHA256/"
                                    "AES-128-GCM", reports=n, request_bytes=len(body)),
               roofline=model_roofline("pipeline", _pipeline_model(eng.sz), n, args.steps, elapsed),
               checks=dict(finished=ok, unpack_mismatch=int(res["mism"][0]),
                           response_bytes=resp_len,
                           response_len_expected=4 + ok * 42 + (n - ok) * 18))
    if not args.no_cpu_baseline:
        from oracle.oracle import Oracle
        m = min(n, max(2048, int(4000 * th * args.cpu_seconds / 10)))
        t0 = time.perf_counter()
        csh, cst = H.open_input_shares(skR, pkR, task, enc[:m], ct[:m], ct_len[:m],
                                       host["nonces"][:m], times[:m], host["public_shares"][:m],
                                       48, n_threads=th)
        t1 = time.perf_counter()
        o_ = Oracle("histogram", length=256, chunk_length=16)
        cm, cs, _, _ = o_.helper_batch(VK, host["nonces"][:m], host["public_shares"][:m], csh,
                                       host["leader_prep_shares"][:m], n_threads=th,
                                       job_size=500)
        t2 = time.perf_counter()
        out["cpu_baseline"] = dict(value=m / (t2 - t0), unit="reports/s", cores=th, kind="port",
                                   sample=f"{m} reports: OpenSSL HPKE open ({t1 - t0:.1f}s) then "
                                          f"the C Prio3 restatement in 500-report jobs "
                                          f"({t2 - t1:.1f}s), {th} threads; DAP codec excluded")
        out["speedup_vs_cpu"] = value / out["cpu_baseline"]["value"]
        out["checks"]["cpu_gpu_parity_on_sample"] = bool(
            np.array_equal(st[:m].cpu().numpy(), cs) and
            np.array_equal(msgs[:m].cpu().numpy(), cm))
    print(json.dumps(out), flush=True)


def _pipeline_model(sz) -> dict:
    """HPKE open (X25519, AES-128-GCM) + the Histogram(256,16) helper step + the ReportIdChecksum
    (one SHA-256 compression per report id); the DAP codec is byte movement (HBM), not VALU."""
    h = RM.hpke_model("x25519", 1)
    p = RM.helper_model(RM.instance("histogram", sz, length=256, chunk=16))
    parts = dict(hpke=h["total"], prepare=p["total"], checksum=RM.PRIM["sha256_compress"])
    return dict(parts, total=sum(parts.values()))


def mp64_main(args):
    """Prio3SumVecField64MultiproofHmacSha256Aes128 helper prepare+aggregate line (not the
    BASELINE metric) at the reference's own end-to-end configuration
    (proofs 2, bits 16, length 15, chunk 16: integration_tests janus.rs:387-392).  Reports are
    distinct and generated on the device by the engine's client (prio3_client_generate_device,
    pinned to oracle/prio3_py.py gen_report_mp64 by tests/test_mp64_client.py).  cpu_baseline: the compiled C restatement
    (oracle/prio3_oracle.c ORC_SUMVEC_F64_MP, OpenSSL SHA-256 / AES-128) in 500-report jobs on
    every host thread, on a bounded sample of the same reports, cross-checking the GPU there."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    cfg = (2, 16, 15, 16)
    vk = bytes(range(0x40, 0x60))
    n = args.reports
    eng = J.HelperEngine(J.Prio3SumVecField64MultiproofHmacSha256Aes128(*cfg), vk, device=0)
    for kv in args.opt:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    t0 = time.perf_counter()
    gen = eng.generate_reports_device(n, seed=0x4A414E5553000008, with_checks=True)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    nonces, pub, helper, lps = (gen["nonces"], gen["public_shares"], gen["helper_shares"],
                                gen["leader_prep_shares"])
    gen_flags = int(gen["flags"].sum().item())
    msgs = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    agg = torch.zeros((1, eng.sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)

    def step():
        s = torch.cuda.current_stream().cuda_stream
        eng.prepare_aggregate_device(nonces, pub, helper, lps, seg, 1, msgs, status, stream=s)
        eng.aggregate_finish_device(status, None, agg, cnt, stream=s)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.set_option("timing", 1)
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    times = eng.timing()
    eng.set_option("timing", 0)
    value = n * args.steps / elapsed
    out = dict(metric="reports prepared+aggregated/sec (helper, Prio3SumVecField64Multiproof"
                      "HmacSha256Aes128 proofs=2 bits=16 length=15 chunk=16)", value=value,
               unit="reports/s", n_gpus=1, steps=args.steps, warmup=args.warmup,
               ms_per_step=elapsed / args.steps * 1e3, higher_is_better=True, scaling="weak",
               vs_baseline=None, dtype="u64 (Field64), bytes",
               data=f"synthetic: {n} distinct reports from the device client (seeded); "
                    f"generation {gen_s:.1f}s, not timed",
               config=dict(workload="Prio3SumVecField64MultiproofHmacSha256Aes128 helper "
                                    "prepare+aggregate", proofs=2, bits=16, length=15,
                           chunk_length=16, reports=n),
               kernels={k: dict(ms_total=v[0], launches=v[1], ms_avg=v[0] / max(v[1], 1))
                        for k, v in times.items()},
               roofline=model_roofline("mp64", RM.mp64_model(eng.sz, cfg[1], cfg[2], cfg[3], cfg[0]),
                                       n, args.steps, elapsed),
               checks=dict(finished=int((status == 0).sum().item()), agg_count=int(cnt[0]),
                           generator_flags=gen_flags),
               cpu_baseline=None)
    if not args.no_cpu_baseline:
        from oracle.oracle import Oracle, build
        build()
        o = Oracle("sumvec_f64_mp", bits=cfg[1], length=cfg[2], chunk_length=cfg[3],
                   num_proofs=cfg[0])
        th = cpu_threads()
        mh = min(n, 1 << 20)
        host = [t[:mh].cpu().numpy() for t in (nonces, pub, helper, lps)]

        def crun(m):
            t1 = time.perf_counter()
            r = o.helper_batch(vk, *(h[:m] for h in host), n_threads=th, job_size=500)
            return time.perf_counter() - t1, r

        probe = min(mh, 500 * th)
        dt, _ = crun(probe)
        m = int(min(mh, max(probe, probe * args.cpu_seconds / max(dt, 1e-6))))
        dt, (cm, cs, cagg, ccnt) = crun(m)
        out["cpu_baseline"] = dict(value=m / dt, unit="reports/s", cores=th, kind="port",
                                   sample=f"{m} of the same reports through the C restatement "
                                          f"(oracle/prio3_oracle.c ORC_SUMVEC_F64_MP), jobs of "
                                          f"500, {th} threads, {dt:.1f}s wall")
        out["speedup_vs_cpu"] = value / out["cpu_baseline"]["value"]
        accept = torch.zeros(n, dtype=torch.uint8, device=dev)
        accept[:m] = 1
        agg_s = torch.zeros_like(agg)
        cnt_s = torch.zeros_like(cnt)
        eng.aggregate_finish_device(status, accept, agg_s, cnt_s)
        torch.cuda.synchronize()
        out["checks"]["cpu_gpu_parity_on_sample"] = bool(
            np.array_equal(status[:m].cpu().numpy(), cs) and
            np.array_equal(msgs[:m].cpu().numpy(), cm) and
            np.array_equal(agg_s.cpu().numpy(), cagg) and int(cnt_s[0].item()) == int(ccnt[0]))
    print(json.dumps(out), flush=True)

def fpvec_main(args):
    """Prio3FixedPointBoundedL2VecSum(length=10000, BitSize16) helper prepare+aggregate line
    (BASELINE.json configs[4], C5: 100k reports; not the headline metric).  Inputs are --reports
    (default here 100k) distinct honest reports from the engine's device client
    (prio3_client_generate_device: entries, shares, the two-gadget proof and the leader's
    prepare_init on the GPU, pinned to oracle/fpvec_py.py gen_report by
    tests/test_fpvec_client.py), resident in HBM.  One step = prepare (the XOF and query kernels
    per scratch sub-batch) + masked mod-p accumulate of the 10000-entry output shares.
    cpu_baseline: the compiled C restatement (oracle/prio3_oracle.c ORC_FPVEC) on a bounded
    sample of the same reports, every host thread; it also cross-checks the GPU on the sample."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    vk = bytes(range(0x70, 0x80))
    n = args.reports if args.reports != 1 << 20 else 100_000
    eng = J.HelperEngine(J.Prio3FixedPointBoundedL2VecSum(10000, 16), vk, device=0,
                         allow_unpinned=True)
    # a device-resident caller running ~225 GB FPVec batches back to back keeps the released run
    # in the pool (keep_scratch; by default a slab above the pool's 1/8-of-HBM budget is freed on
    # release): re-allocating it every step cost C5 40 % in r02j
    eng.set_option("keep_scratch", 1)
    for kv in args.opt:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    t0 = time.perf_counter()
    gen = eng.generate_reports_device(n, seed=0x4A414E5553000007, with_checks=True)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    nonces, pub, helper, lps = (gen["nonces"], gen["public_shares"], gen["helper_shares"],
                                gen["leader_prep_shares"])
    gen_flags = int(gen["flags"].sum().item())
    msgs = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    agg = torch.zeros((1, eng.sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)

    def step():
        s = torch.cuda.current_stream().cuda_stream
        eng.prepare_device(nonces, pub, helper, lps, msgs, status, stream=s)
        eng.accumulate_device(n, status, seg, None, 1, agg, cnt, stream=s)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.set_option("timing", 1)
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    times = eng.timing()
    eng.set_option("timing", 0)
    # check: the step's aggregate plus the leader's (the generator's leader output shares,
    # summed by the combine kernel in two levels) unshards to the sum of all n entry vectors
    P128 = (1 << 128) - 28 * (1 << 64) + 1
    k1 = next(k for k in (1000, 500, 100, 10, 1) if n % k == 0)
    part = torch.zeros((n // k1, eng.sz.agg_share_len), dtype=torch.uint8, device=dev)
    pc = torch.zeros(n // k1, dtype=torch.int64, device=dev)
    eng.combine_device(k1, n // k1, gen["leader_out_shares"],
                       torch.zeros(n, dtype=torch.int64, device=dev), part, pc)
    lagg = torch.zeros_like(agg)
    eng.combine_device(n // k1, 1, part, pc, lagg, torch.zeros_like(cnt))
    esum = gen["measurements"].sum(dim=0).cpu().tolist()
    del part, gen["leader_out_shares"]
    a, la = agg.cpu().numpy()[0].tobytes(), lagg.cpu().numpy()[0].tobytes()
    dec = lambda b, e: int.from_bytes(b[16 * e:16 * e + 16], "little")
    ok_unshard = all((dec(a, e) + dec(la, e)) % P128 == esum[e] + n * (1 << 15)
                     for e in range(10000))
    cpu = None
    if not args.no_cpu_baseline:
        # the compiled C restatement (oracle/prio3_oracle.c ORC_FPVEC, pinned to the Python one
        # and to the fixtures by tests/test_fpvec.py) in 500-report jobs on every host thread,
        # on a bounded sample of the same reports; cross-checks the GPU on that sample
        from oracle.oracle import Oracle, build
        build()
        o = Oracle("fpvec", bits=16, length=10000)
        th = cpu_threads()
        mh = min(n, 8192)
        hostd = dict(nonce=nonces[:mh].cpu().numpy(), pub=pub[:mh].cpu().numpy(),
                     helper=helper[:mh].cpu().numpy(), lps=lps[:mh].cpu().numpy())

        # Janus's jobs hold up to 500 reports; a bounded sample of a few thousand 20-50 ms
        # reports must still give every worker thread jobs, so the jobs here are m / threads
        # reports (r02's 500-report jobs put a sub-500 sample on ONE thread)
        def crun(m, threads=th):
            js = max(1, min(500, m // threads))
            t1 = time.perf_counter()
            r = o.helper_batch(vk, hostd["nonce"][:m], hostd["pub"][:m], hostd["helper"][:m],
                               hostd["lps"][:m], n_threads=threads, job_size=js)
            return time.perf_counter() - t1, r

        dt1, _ = crun(4, 1)  # single core, per report
        probe = min(n, 2 * th)
        dt, _ = crun(probe)
        m = int(min(mh, max(probe, probe * args.cpu_seconds / max(dt, 1e-6))))
        dt, (cm, cs, cagg, ccnt) = crun(m)
        # op count of one report on one core: the Keccak-p[1600,12] permutations (share
        # expansion, the joint-rand part over the encoded share, prio's re-expansion in
        # prepare_next, proofs, seeds) and the Field128 multiplies of the query (3 per gadget-0
        # element, 1 per gadget-1 entry), priced at this host's measured single-core rates
        from oracle.oracle import prim_bench
        ns_perm, ns_mul = prim_bench()
        M = o.meas_len
        perms = 2 * -(-16 * M // 168) + (42 + 16 * M) // 168 + 1 + -(-16 * o.proof_len // 168) + 4
        muls = 3 * o.calls * (o.arity // 2) + o.fp_K1 * o.fp_C1
        model_ms = (perms * ns_perm + muls * ns_mul) / 1e6
        cpu = dict(value=m / dt, unit="reports/s", cores=th, kind="port",
                   sample=f"{m} of the device-generated reports through the C restatement "
                          f"(oracle/prio3_oracle.c, ORC_FPVEC), {th} threads, jobs of "
                          f"{max(1, min(500, m // th))}, {dt:.1f}s wall",
                   single_core_ms_per_report=dt1 / 4 * 1e3,
                   op_count=dict(keccak_p12_perms=perms, f128_muls=muls, ns_per_perm=ns_perm,
                                 ns_per_f128_mul=ns_mul, model_ms_per_report=model_ms,
                                 note="perms x ns + muls x ns on one core; the rest of the "
                                      "measured single-core time is the element decode / "
                                      "encode passes over the 2.56 MB measurement share"),
                   cpu_model=cpu_model())
        accept = torch.zeros(n, dtype=torch.uint8, device=dev)
        accept[:m] = 1
        agg_s = torch.zeros_like(agg)
        cnt_s = torch.zeros_like(cnt)
        eng.accumulate_device(n, status, seg, accept, 1, agg_s, cnt_s)
        torch.cuda.synchronize()
        cpu_parity = bool(np.array_equal(status[:m].cpu().numpy(), cs) and
                          np.array_equal(msgs[:m].cpu().numpy(), cm) and
                          np.array_equal(agg_s.cpu().numpy(), cagg) and
                          int(cnt_s[0].item()) == int(ccnt[0]))
    kern = {k: dict(ms_total=v[0], launches=v[1], ms_avg=v[0] / max(v[1], 1))
            for k, v in times.items()}
    value = n * args.steps / elapsed
    out = dict(metric="reports prepared+aggregated/sec (helper, Prio3FixedPointBoundedL2VecSum "
                      "length=10000)", value=value, unit="reports/s", n_gpus=1, steps=args.steps,
               warmup=args.warmup, ms_per_step=elapsed / args.steps * 1e3, higher_is_better=True,
               scaling="weak", vs_baseline=None, dtype="u32 limbs (Field128 mod-p integer arithmetic)",
               data=f"synthetic: {n} distinct honest reports from the device client (seeded; "
                    f"generation {gen_s:.1f}s, not timed)",
               config=dict(workload="Prio3FixedPointBoundedL2VecSum length=10000 BitSize16 helper "
                                    "prepare+aggregate (configs[4], C5)", length=10000, bits=16,
                           reports=n),
               kernels=kern,
               roofline=model_roofline("fpvec", RM.helper_model(RM.instance(
                   "fpvec", eng.sz, bits=16, length=10000)), n, args.steps, elapsed),
               checks=dict(finished=int((status == 0).sum().item()), agg_count=int(cnt[0]),
                           generator_flags=gen_flags, unshard_equals_entry_sum=bool(ok_unshard),
                           cpu_gpu_parity_on_sample=cpu_parity if cpu else None),
               cpu_baseline=cpu,
               speedup_vs_cpu=(value / cpu["value"]) if cpu else None)
    print(json.dumps(out), flush=True)


CONFIGS = {  # BASELINE.json configs[0], [2], [3]: (engine vdaf, oracle kwargs, reports per GPU)
    "count": (lambda: J.Prio3Count(), dict(kind="count"), 100_000),
    "sumvec": (lambda: J.Prio3SumVec(8, 1000, 63), dict(kind="sumvec", bits=8, length=1000,
                                                         chunk_length=63), 1_000_000 // 8),
    "sum32": (lambda: J.Prio3Sum(32), dict(kind="sum", bits=32), 10_000_000 // 8),
}


def config_main(args):
    """Helper prepare+aggregate lines for the other BASELINE.json configs on one MI355X
    (C1 Count 100k; C3 SumVec(8, 1000, chunk 63) and C4 Sum(32) at one GPU's 1/8 shard of
    their 8-GPU totals).  Same step as the headline (prio3_device_prepare_aggregate +
    aggregate_finish over resident device-generated reports); cpu_baseline = the C
    restatement on a bounded sample of the same reports, Janus job structure."""
    n = args.reports if args.reports != 1 << 20 else CONFIGS[args.vdaf][2]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "gloo":
            local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    out = config_line(args.vdaf, n, args.steps, args.warmup, args.cpu_seconds, args.opt,
                      not args.no_cpu_baseline and rank == 0, dist=dist, local=local,
                      gloo=args.dist_backend == "gloo")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def _leader_sum(eng, shares, n, dev):
    """Mod-p sum of n leader output shares on the device: the combine kernel in two levels
    (k1 rows of k2 "segments", then the k2 partial sums), so no work-item loops over millions
    of rows."""
    sz = eng.sz
    k1 = next(k for k in (1000, 512, 500, 100, 64, 10, 8, 1) if n % k == 0)
    k2 = n // k1
    part = torch.zeros((k2, sz.agg_share_len), dtype=torch.uint8, device=dev)
    pcnt = torch.zeros(k2, dtype=torch.int64, device=dev)
    eng.combine_device(k1, k2, shares, torch.zeros(n, dtype=torch.int64, device=dev), part, pcnt)
    lagg = torch.zeros((1, sz.agg_share_len), dtype=torch.uint8, device=dev)
    lcnt = torch.zeros(1, dtype=torch.int64, device=dev)
    eng.combine_device(k2, 1, part, pcnt, lagg, lcnt)
    return lagg


def config_line(vdaf, n, steps, warmup, cpu_seconds, opts=(), with_cpu=True, dist=None, local=0,
                gloo=False):
    """One config's helper step on this GPU (n reports); with `dist` (N ranks, one shard of n
    reports each, report indices rank*n + i) the step ends in the AggregateCombiner as the
    headline's does, elapsed is the max over ranks and value counts every rank's reports.
    Checks: every honest report finishes; unshard -- the (combined) helper aggregate plus the
    leader aggregate summed from the on-device client's leader output shares equals the plain
    sum of all measurements (integration_tests/tests/integration/common.rs:332-554,
    aggregate_share.rs:55-96); and on rank 0 the restatement's statuses, prepare messages,
    aggregate share and count over a bounded sample of its shard."""
    from oracle.oracle import Oracle, build
    mk, okw, _ = CONFIGS[vdaf]
    world = dist.get_world_size() if dist else 1
    rank = dist.get_rank() if dist else 0
    dev = torch.device("cuda", local)
    torch.cuda.set_device(local)
    eng = J.HelperEngine(mk(), VK, device=local)
    for kv in opts:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    sz = eng.sz
    d = eng.generate_reports_device(n, seed=0x4A414E5553000001, first_index=rank * n,
                                    with_checks=True)
    torch.cuda.synchronize()
    flags = int(d["flags"].sum().item())
    msgs = torch.empty((n, max(sz.prep_msg_len, 1)), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    agg = torch.zeros((1, sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    pub = d["public_shares"] if sz.public_share_len else None
    cur = lambda: torch.cuda.current_stream().cuda_stream
    combiner = lcombiner = None
    if dist:
        from janus_amd.dist import AggregateCombiner
        comb = lambda k, ga, gc, oa, oc: eng.combine_device(k, 1, ga, gc, oa, oc, stream=cur())
        combiner = AggregateCombiner(dist, agg, cnt, comb, stage_device="cpu" if gloo else None)
        lcombiner = AggregateCombiner(dist, agg, cnt, comb, stage_device="cpu" if gloo else None)

    def step():
        s = cur()
        eng.prepare_aggregate_device(d["nonces"], pub, d["helper_shares"],
                                     d["leader_prep_shares"], seg, 1, msgs, status, stream=s)
        eng.aggregate_finish_device(status, None, agg, cnt, stream=s)
        if combiner is not None:
            combiner(agg, cnt)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # the timed steps run without the per-kernel HIP events (two event records per launch add
    # host work to C1's 0.1 ms, four-launch step); the kernel table comes from a separate pass
    # over the same steps afterwards, as the headline's roofline pass
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_option("timing", 1)
    eng.timing_reset()
    for _ in range(steps):  # same step count: launches per step stay launches / steps
        step()
    torch.cuda.synchronize()
    times = eng.timing()
    eng.set_option("timing", 0)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * n * steps / elapsed

    # unshard: helper (combined) + leader (combined) aggregate == sum of every measurement
    lagg = _leader_sum(eng, d["leader_out_shares"], n, dev)
    msum = d["measurements"].sum(dim=0)
    if dist:
        lagg, _ = lcombiner(lagg, torch.full_like(cnt, n))
        msum = msum.cpu() if gloo else msum
        dist.all_reduce(msum)
        hagg, hcnt = combiner.out_agg, combiner.out_cnt
    else:
        hagg, hcnt = agg, cnt
    torch.cuda.synchronize()
    es = 8 if okw["kind"] == "count" else 16
    P = 2**64 - 2**32 + 1 if es == 8 else 2**128 - 28 * 2**64 + 1
    hb = hagg.cpu().numpy().reshape(-1, es)
    lb = lagg.cpu().numpy().reshape(-1, es)
    ms = [int(x) for x in msum.cpu().numpy().reshape(-1)]
    unshard = len(ms) == hb.shape[0] and all(
        (int.from_bytes(hb[e].tobytes(), "little") + int.from_bytes(lb[e].tobytes(), "little"))
        % P == ms[e] for e in range(len(ms)))
    total_cnt = int(hcnt[0].item())
    del lagg, msum

    cpu, parity, m = None, None, 0
    if with_cpu:
        build()
        o = Oracle(**okw)
        th = cpu_threads()
        host = {k: d[k].cpu().numpy() for k in
                ("nonces", "public_shares", "helper_shares", "leader_prep_shares")}

        def run(m):
            t1 = time.perf_counter()
            r = o.helper_batch(VK, host["nonces"][:m], host["public_shares"][:m],
                               host["helper_shares"][:m], host["leader_prep_shares"][:m],
                               n_threads=th, job_size=500)
            return time.perf_counter() - t1, r

        probe = min(n, 500 * th)
        dt, _ = run(probe)
        m = int(min(n, max(probe, probe * cpu_seconds / max(dt, 1e-6))))
        dt, (cm, cs, ca, cc) = run(m)
        # the GPU aggregate share and count of the same sample: the last step's statuses
        # finished again with an accept mask selecting the first m reports
        accept = torch.zeros(n, dtype=torch.uint8, device=dev)
        accept[:m] = 1
        agg_s = torch.zeros_like(agg)
        cnt_s = torch.zeros_like(cnt)
        eng.aggregate_finish_device(status, accept, agg_s, cnt_s)
        torch.cuda.synchronize()
        parity = bool(np.array_equal(status[:m].cpu().numpy(), cs) and
                      np.array_equal(msgs[:m, :cm.shape[1]].cpu().numpy(), cm) and
                      np.array_equal(agg_s.cpu().numpy().reshape(-1), np.asarray(ca).reshape(-1))
                      and int(cnt_s[0].item()) == int(np.asarray(cc).reshape(-1)[0]))
        cpu = dict(value=m / dt, unit="reports/s", cores=th, kind="port",
                   sample=f"{m} of the benchmark's GPU-generated reports, jobs of 500 reports, "
                          f"one job per worker thread (aggregator.rs:1794,2100), {dt:.1f}s wall")
    out = dict(metric=f"reports prepared+aggregated/sec (helper, {vdaf})", value=value,
               unit="reports/s", n_gpus=world, steps=steps, warmup=warmup,
               ms_per_step=elapsed / steps * 1e3, higher_is_better=True, scaling="weak",
               vs_baseline=None, dtype="u32 limbs (mod-p integer arithmetic)",
               data="synthetic: distinct honest reports generated on-device from a seed",
               config=dict(workload=f"{vdaf} helper prepare+aggregate, 1 segment",
                           reports=n, reports_per_rank=n, global_batch=world * n,
                           **{k: v for k, v in okw.items() if k != "kind"}),
               kernels={k: dict(ms_total=v[0], launches=v[1], ms_avg=v[0] / max(v[1], 1))
                        for k, v in times.items()},
               roofline=model_roofline(f"config_{vdaf}", RM.helper_model(RM.instance(
                   okw["kind"], sz, bits=okw.get("bits", 0), length=okw.get("length", 0),
                   chunk=okw.get("chunk_length", 0))), n, steps, elapsed),
               checks=dict(finished=int((status == 0).sum().item()), agg_count=total_cnt,
                           all_counted=total_cnt == world * n, generator_flags=flags,
                           unshard_equals_measurement_sum=unshard,
                           cpu_gpu_parity_on_sample=parity,
                           cpu_gpu_parity_covers=(f"statuses, prepare messages, aggregate share "
                                                  f"and count of rank 0's first {m} reports")
                           if with_cpu else None),
               cpu_baseline=cpu, speedup_vs_cpu=(value / cpu["value"]) if cpu else None)
    if dist:
        out["dist_backend"] = "gloo" if gloo else "nccl"
        out["config"]["parallelism"] = f"dp{world} (report shards; all-gather + mod-p combine)"
        if gloo:
            out["note"] = ("gloo, ranks sharing the box's GPUs: a correctness run of the sharded "
                           "step (all-gather staged through host memory), unmeasured on "
                           "hardware -- the RCCL scaling curve is the driver's")
    return out


if __name__ == "__main__":
    main()
