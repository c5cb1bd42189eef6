"""Generates tests/golden/prio3_*.json: seeded helper-side transcripts (inputs + every
intermediate value + outputs), produced by the pure-Python restatement
(oracle/prio3_py.py) and asserted equal to the C restatement (oracle/prio3_oracle.c)
before writing.  These pin GPU-vs-CPU parity; they do NOT pin prio itself (no prio
vectors exist in the reference; see DESIGN.md "Oracle").

Usage: python tests/golden/gen_golden.py
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import prio3_py as py  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

CASES = {
    "count": dict(kind="count"),
    "sum_8": dict(kind="sum", bits=8),
    "sumvec_3x5_c4": dict(kind="sumvec", bits=3, length=5, chunk_length=4),
    "histogram_10_c3": dict(kind="histogram", length=10, chunk_length=3),
    "histogram_256_c16": dict(kind="histogram", length=256, chunk_length=16),
}
N_REPORTS = {"histogram_256_c16": 3}


def measurement(rnd, cfg):
    k = cfg["kind"]
    if k == "count":
        return rnd.randrange(2)
    if k == "sum":
        return rnd.randrange(2 ** cfg["bits"])
    if k == "sumvec":
        return [rnd.randrange(2 ** cfg["bits"]) for _ in range(cfg["length"])]
    return rnd.randrange(cfg["length"])


def main():
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name, cfg in CASES.items():
        rnd = random.Random("janus-amd-golden-" + name)
        kw = {k: v for k, v in cfg.items() if k != "kind"}
        t = py.Prio3Type(cfg["kind"], **kw)
        vdaf = py.Prio3(t)
        o = Oracle(**cfg)
        F = t.F
        vk = bytes(rnd.randrange(256) for _ in range(16))
        reports = []
        helper_outs = []
        for i in range(N_REPORTS.get(name, 6)):
            m = measurement(rnd, cfg)
            nonce = bytes(rnd.randrange(256) for _ in range(16))
            rand = bytes(rnd.randrange(256) for _ in range(o.rand_size))
            pub, ls, hs = vdaf.shard(m, nonce, rand)
            assert (pub, ls, hs) == o.shard(m, nonce, rand)
            lstate, lps, _ = vdaf.prepare_init(vk, 0, nonce, pub, ls)
            hstate, hps, tr = vdaf.prepare_init(vk, 1, nonce, pub, hs)
            rc, ctr = o.helper_trace(vk, nonce, pub, hs)
            assert rc == 0
            enc = lambda xs: b"".join(F.enc(x) for x in xs)
            assert ctr["meas"] == enc(tr["meas"]) and ctr["proofs"] == enc(tr["proofs"])
            assert ctr["verifiers"] == enc(tr["verifiers"]) and ctr["jr"] == enc(tr["jr"])
            assert ctr["part"] == tr["part"] and ctr["corrected"] == tr["corrected"]
            assert ctr["qr"] == enc(tr["qr"])
            msg = vdaf.prep_shares_to_prep_msg(lps, hps)
            out = vdaf.prepare_next(hstate, msg)
            helper_outs.append(out)
            reports.append(dict(
                measurement=m, nonce=nonce.hex(), public_share=pub.hex(),
                helper_share=hs.hex(), leader_share=ls.hex(), leader_prep_share=lps.hex(),
                helper_meas_share=enc(tr["meas"]).hex(), helper_proofs_share=enc(tr["proofs"]).hex(),
                joint_rand_part=tr["part"].hex(), corrected_joint_rand_seed=tr["corrected"].hex(),
                joint_rands=enc(tr["jr"]).hex(), query_rands=enc(tr["qr"]).hex(),
                helper_verifier=enc(tr["verifiers"]).hex(), helper_prep_share=hps.hex(),
                prep_msg=msg.hex(), helper_output_share=enc(out).hex(), status=0))
        agg = vdaf.aggregate(helper_outs)
        # negative cases: tampered copies of report 0 with their expected status
        neg = []
        r0 = reports[0]
        lps0 = bytearray(bytes.fromhex(r0["leader_prep_share"]))
        bad = bytearray(lps0)
        bad[F.es] ^= 1
        neg.append(dict(base=0, field="leader_prep_share", value=bytes(bad).hex(), status=3))
        bad = bytearray(lps0)
        bad[:F.es] = b"\xff" * F.es
        neg.append(dict(base=0, field="leader_prep_share", value=bytes(bad).hex(), status=2))
        if t.jr_len:
            bad = bytearray(lps0)
            bad[-1] ^= 0x80
            neg.append(dict(base=0, field="leader_prep_share", value=bytes(bad).hex(), status=4))
            pub0 = bytearray(bytes.fromhex(r0["public_share"]))
            pub0[0] ^= 1
            neg.append(dict(base=0, field="public_share", value=bytes(pub0).hex(), status=4))
        # expected statuses come from the restatement itself (which check fires first is
        # data-dependent, e.g. a wrong public share usually fails decide before prepare_next)
        for ng in neg:
            r = dict(r0)
            r[ng["field"]] = ng["value"]
            hx = bytes.fromhex
            try:
                hst, hps2, _ = vdaf.prepare_init(vk, 1, hx(r["nonce"]), hx(r["public_share"]),
                                                  hx(r["helper_share"]))
                try:
                    m2 = vdaf.prep_shares_to_prep_msg(hx(r["leader_prep_share"]), hps2)
                except ValueError as e:
                    ng["status"] = 2 if "range" in str(e) else 3
                    continue
                try:
                    vdaf.prepare_next(hst, m2)
                    ng["status"] = 0
                except ValueError:
                    ng["status"] = 4
            except ValueError:
                ng["status"] = 1
        doc = dict(
            description="Seeded Prio3 helper transcripts (VDAF-08 restatement of prio 0.16.2; "
                        "parity with prio bytes unpinned). Generated by tests/golden/gen_golden.py.",
            vdaf=cfg, verify_key=vk.hex(), reports=reports,
            helper_aggregate_share=b"".join(F.enc(x) for x in agg).hex(), negative=neg)
        with open(os.path.join(out_dir, f"prio3_{name}.json"), "w") as f:
            json.dump(doc, f, indent=1)
        print("wrote", name, len(reports))


if __name__ == "__main__":
    main()
