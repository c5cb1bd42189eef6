"""Static VALU instruction mix of the engine's kernels, from the gfx950 assembly.

Usage: python tools/isa_mix.py [--asm FILE] [--kernel SUBSTR]
  (without --asm the engine is compiled with `hipcc --cuda-device-only -S` into /tmp)

For every kernel it prints the VALU instructions of the whole kernel and of each loop (a
`=>This Inner Loop Header` label up to the last branch back to it), split by issue class.
The issue cost per class (SIMD cycles per wave64 instruction) comes from the measured
throughput at 8 waves/SIMD in profiles/*ubench_valu*.txt: full-rate instructions (bitop3,
xor, add_u32, mov, cndmask, ...) issue every 2 cycles, half-rate ones (carry adds, 64-bit
integer ops, 32-bit multiplies, alignbit, perm, 3-operand shifts) every 4.
The mix-weighted VALU ceiling of a loop is  PEAK_FULL * 2 / (2 f_full + 4 f_half)
lane-instructions/s.  bench.py uses it as roofline.peak for the dominant kernel.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Measured on MI355X (tools/ubench_valu.hip, 8 waves/SIMD): ~64.5 T lane-instr/s for full-rate
# ops, ~37 T for half-rate.  Everything not matched below is treated as full rate.
HALF_RATE = re.compile(
    r"^v_(alignbit|mad_u64_u32|mad_i64_i32|lshl_add_u64|mul_lo_u32|mul_hi_u32|perm_b32|"
    r"lshl_or_b32|add_co_u32|addc_co_u32|sub_co_u32|subb_co_u32|subrev_co_u32|subbrev_co_u32|"
    r"cmp_\w+_u64|cmp_\w+_i64|mov_b64|lshlrev_b64|lshrrev_b64|add_u64|sub_u64|add3_u32|"
    r"lshl_add_u32|add_lshl_u32|xad_u32|mad_u32_u24|mad_u32_u16)")
PEAK_FULL_T = 64.5
PEAK_HALF_T = 37.0


def asm_path(source: str = "prio3_engine.hip"):
    out = f"/tmp/{source.replace('.hip', '')}_gfx950.s"
    src = os.path.join(ROOT, "janus_amd", "csrc", source)
    deps = [src] + [os.path.join(ROOT, "janus_amd", "csrc", h) for h in
                    ("prio3_device.h", "prio3_common.h", "sha256_device.h")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "--cuda-device-only", "-S", "-o", out, src], check=True)
    return out


def split_kernels(lines):
    kern, cur = {}, None
    for ln in lines:
        m = re.match(r"^(_Z\w+):\s*;\s*@", ln)
        if m:
            cur = m.group(1)
            kern[cur] = []
            continue
        if cur and ln.startswith(".Lfunc_end"):
            cur = None
        if cur:
            kern[cur].append(ln)
    return kern


def mix(body):
    c = Counter()
    for ln in body:
        s = ln.strip()
        if not s.startswith("v_"):
            continue
        op = s.split()[0]
        c["half" if HALF_RATE.match(op) else "full"] += 1
    return c


def loops(body):
    """(header, [lines]) per innermost loop, from LLVM's block comments: the header block
    (`=>This Inner Loop Header`) plus every block tagged `in Loop: Header=<it>`."""
    blocks, cur, hdr = {}, None, None
    for ln in body:
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            hdr = None
            h = re.search(r"Header=(BB\w+)", ln)
            if "Loop Header" in ln:
                hdr = m.group(1).lstrip(".L")
            elif h:
                hdr = h.group(1)
            cur = hdr
            if cur:
                blocks.setdefault(cur, [])
        elif cur:
            blocks[cur].append(ln)
    return sorted(blocks.items(), key=lambda kv: -len(kv[1]))


def ceiling(c):
    n = c["full"] + c["half"]
    if not n:
        return PEAK_FULL_T
    cyc = 2 * c["full"] + 4 * c["half"]
    return PEAK_FULL_T * 2 * n / cyc


def demangle(k):
    m = re.match(r"_Z\d+(\w+?)(I.*E)?v?\d", k)
    n = re.match(r"_Z(\d+)", k)
    return k[len(n.group(0)):len(n.group(0)) + int(n.group(1))] if n else k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--source", default="prio3_engine.hip")
    a = ap.parse_args()
    lines = open(a.asm or asm_path(a.source)).read().splitlines()
    for k, body in split_kernels(lines).items():
        if a.kernel not in k:
            continue
        c = mix(body)
        print(f"{k}\n  whole kernel: full {c['full']:6d} half {c['half']:6d} "
              f"half-frac {c['half'] / max(1, c['full'] + c['half']):.3f} "
              f"ceiling {ceiling(c):.1f} T")
        for lab, lb in loops(body):
            lc = mix(lb)
            if lc["full"] + lc["half"] < 50:
                continue
            print(f"  loop {lab:10s}: full {lc['full']:6d} half {lc['half']:6d} "
                  f"half-frac {lc['half'] / max(1, lc['full'] + lc['half']):.3f} "
                  f"ceiling {ceiling(lc):.1f} T")


if __name__ == "__main__":
    main()
