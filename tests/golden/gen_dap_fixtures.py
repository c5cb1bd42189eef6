"""Extracts the DAP-09 wire-format fixtures the reference's own codec tests hold
(/root/reference/messages/src/tests/aggregation.rs: roundtrip_aggregation_job_initialize_req,
roundtrip_prepare_resp, roundtrip_aggregation_job_resp) as hex byte strings -- data only: the
concatenated hex literals of each roundtrip_encoding(..) call.  Run in the build container;
writes tests/golden/dap_fixtures.json."""
import json
import os
import re

SRC = "/root/reference/messages/src/tests/aggregation.rs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dap_fixtures.json")


def calls(src, fn):
    start = src.index(f"fn {fn}()")
    end = src.find("#[test]", start)
    body = src[start:end if end > 0 else len(src)]
    parts = body.split("roundtrip_encoding(")[1:]
    out = []
    for p in parts:
        p = re.sub(r'Vec::from\("[^"]*"\)', "", p)  # field values, not encodings
        lits = re.findall(r'"([0-9A-Fa-f]*)"', p)
        out.append("".join(lits).lower())
    return out


def main():
    src = open(SRC).read()
    fx = {
        "agg_init_req_time_interval": calls(src, "roundtrip_aggregation_job_initialize_req")[0],
        "agg_init_req_fixed_size": calls(src, "roundtrip_aggregation_job_initialize_req")[1],
        "prepare_resps": calls(src, "roundtrip_prepare_resp")[0],
        "agg_job_resp": calls(src, "roundtrip_aggregation_job_resp")[0],
        "source": "messages/src/tests/aggregation.rs (reference codec roundtrip fixtures)",
    }
    json.dump(fx, open(OUT, "w"), indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
