"""The Rust side of the drop-in boundary, derived from include/*.h.

  python tools/ffi_rs.py            prints the `janus_prio3_sys` declarations
  python tools/ffi_rs.py --check    exits 1 if INTEGRATION.md's block drifted from the headers
  python tools/ffi_rs.py --write    rewrites that block from the headers (after a header change)

parse_header() reads the C prototypes, typedef'd structs and enum constants of a header;
rust_type() maps a C parameter type to the Rust FFI type the crate must declare (pointers keep
their constness, arrays decay to pointers, opaque handles stay opaque); parse_rust() reads an
`extern "C"` / `#[repr(C)]` block back.  tests/test_ffi_decls.py compares the two: every function
of every header by name, arity and per-parameter Rust type, every struct field, every constant.
"""
from __future__ import annotations

import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("janus_prio3.h", "janus_hpke.h",
                                                       "janus_dap.h")]
INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")

SCALARS = {"uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64",
           "int8_t": "i8", "int16_t": "i16", "int32_t": "i32", "int64_t": "i64", "int": "c_int",
           "size_t": "usize", "char": "c_char", "double": "f64", "float": "f32", "void": "c_void"}
OPAQUE = ("prio3_engine", "prio3_batch", "janus_hpke_opener")


def _strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def rust_type(ctype: str) -> str:
    """C type of a parameter / return / field (array suffix already removed) -> Rust type."""
    t = ctype.replace("struct ", "").strip()
    const = t.startswith("const ")
    if const:
        t = t[len("const "):].strip()
    stars = t.count("*")
    base = t.replace("*", "").strip()
    if base.endswith(" const"):  # `T* const` never appears in these headers
        raise ValueError(ctype)
    r = SCALARS.get(base, base)
    if stars == 0:
        return "()" if r == "c_void" else r
    out = r
    for i in range(stars):
        # the innermost pointer carries the declared constness; outer ones are mutable
        out = ("*const " if (const and i == 0) else "*mut ") + out
    return out


def _split_params(s: str):
    s = s.strip()
    if s in ("", "void"):
        return []
    return [p.strip() for p in s.split(",")]


def _param(p: str):
    """'const uint8_t verify_key[16]' -> ('verify_key', '*const u8')"""
    m = re.match(r"^(.*?)([A-Za-z_]\w*)\s*(\[[^\]]*\])?$", p.strip())
    ctype, name, arr = m.group(1).strip(), m.group(2), m.group(3)
    if arr:
        ctype += "*"
    return name, rust_type(ctype)


def parse_header(path: str) -> dict:
    src = _strip_comments(open(path).read())
    funcs = {}
    for m in re.finditer(r"(?:^|\n)\s*((?:const\s+)?[A-Za-z_][\w\s]*?\**)\s*\b([a-z_][a-z0-9_]*)\s*"
                         r"\(([^;{}]*?)\)\s*;", src):
        ret, name, params = m.group(1).strip(), m.group(2), m.group(3)
        if ret.startswith(("typedef", "return")) or name in ("defined",):
            continue
        funcs[name] = dict(ret=rust_type(ret), params=[_param(p) for p in _split_params(params)])
    structs = {}
    for m in re.finditer(r"typedef\s+struct\s*\{(.*?)\}\s*(\w+)\s*;", src, re.S):
        fields = []
        for decl in m.group(1).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            tm = re.match(r"^((?:const\s+)?[\w]+\s*\**)\s*(.*)$", decl)
            ctype, names = tm.group(1).strip(), tm.group(2)
            for nm in names.split(","):
                nm = nm.strip()
                am = re.match(r"^(\w+)\s*\[(\d+)\]$", nm)
                if am:
                    fields.append((am.group(1), f"[{rust_type(ctype)}; {am.group(2)}]"))
                else:
                    fields.append((nm, rust_type(ctype)))
        structs[m.group(2)] = fields
    consts = {}
    for m in re.finditer(r"enum\s*\{(.*?)\}\s*;", src, re.S):
        for item in m.group(1).split(","):
            item = item.strip()
            if "=" in item:
                k, v = (x.strip() for x in item.split("=", 1))
                consts[k] = int(v, 0)
    for m in re.finditer(r"#define\s+(JANUS_\w+|PRIO3_\w+)\s+(0x[0-9A-Fa-f]+|\d+)u?\b", src):
        consts[m.group(1)] = int(m.group(2), 0)
    return dict(funcs=funcs, structs=structs, consts=consts)


def parse_headers(paths=HEADERS) -> dict:
    out = dict(funcs={}, structs={}, consts={}, order=[])
    for p in paths:
        h = parse_header(p)
        for k in ("funcs", "structs", "consts"):
            out[k].update(h[k])
        out["order"].append((os.path.basename(p), h))
    return out


def gen_rust(paths=HEADERS) -> str:
    lines = ["#![allow(non_camel_case_types)]",
             "use std::os::raw::{c_char, c_int, c_void};", ""]
    lines += [f"#[repr(C)] pub struct {o} {{ _p: [u8; 0] }}" for o in OPAQUE]
    for hname, h in parse_headers(paths)["order"]:
        lines += ["", f"// ---- include/{hname} ----"]
        for k, v in h["consts"].items():
            lines.append(f"pub const {k}: i64 = {v:#x};" if v > 9 else f"pub const {k}: i64 = {v};")
        for sname, fields in h["structs"].items():
            lines.append("#[repr(C)] #[derive(Clone, Copy)]")
            lines.append(f"pub struct {sname} {{")
            lines += [f"    pub {n}: {t}," for n, t in fields]
            lines.append("}")
        lines.append('extern "C" {')
        for name, f in h["funcs"].items():
            ps = ", ".join(f"{n}: {t}" for n, t in f["params"])
            ret = "" if f["ret"] == "()" else f" -> {f['ret']}"
            decl = f"    pub fn {name}({ps}){ret};"
            if len(decl) <= 100:
                lines.append(decl)
            else:  # one parameter per line
                lines.append(f"    pub fn {name}(")
                lines += [f"        {n}: {t}," for n, t in f["params"]]
                lines.append(f"    ){ret};")
        lines.append("}")
    return "\n".join(lines) + "\n"


def parse_rust(text: str) -> dict:
    """The functions, structs and constants of a generated / hand-written Rust block."""
    funcs, structs, consts = {}, {}, {}
    body = re.sub(r"//[^\n]*", " ", text)
    for m in re.finditer(r"pub\s+fn\s+(\w+)\s*\((.*?)\)\s*(?:->\s*([^;{]+?))?\s*;", body, re.S):
        params = []
        for p in [x.strip() for x in m.group(2).split(",") if x.strip()]:
            n, t = p.split(":", 1)
            params.append((n.strip(), " ".join(t.split())))
        funcs[m.group(1)] = dict(ret=" ".join((m.group(3) or "()").split()), params=params)
    for m in re.finditer(r"pub\s+struct\s+(\w+)\s*\{(.*?)\}", body, re.S):
        if "_p: [u8; 0]" in m.group(2):
            continue
        fields = []
        for f in [x.strip() for x in m.group(2).split(",") if x.strip()]:
            n, t = f.replace("pub ", "", 1).split(":", 1)
            fields.append((n.strip(), " ".join(t.split())))
        structs[m.group(1)] = fields
    for m in re.finditer(r"pub\s+const\s+(\w+)\s*:\s*\w+\s*=\s*(-?0x[0-9a-fA-F]+|-?\d+)\s*;", body):
        consts[m.group(1)] = int(m.group(2), 0)
    return dict(funcs=funcs, structs=structs, consts=consts)


def integration_block(path=INTEGRATION) -> str:
    """The ```rust block of INTEGRATION.md that follows the marker line `src/lib.rs`."""
    src = open(path).read()
    m = re.search(r"`src/lib\.rs`[^\n]*\n+```rust\n(.*?)```", src, re.S)
    if not m:
        raise ValueError("INTEGRATION.md has no src/lib.rs rust block")
    return m.group(1)


def diff(c: dict, r: dict) -> list:
    """Every way the Rust declarations r differ from the headers c (empty: in sync)."""
    out = []
    for name, f in c["funcs"].items():
        g = r["funcs"].get(name)
        if g is None:
            out.append(f"missing fn {name}")
            continue
        if len(g["params"]) != len(f["params"]):
            out.append(f"{name}: arity {len(g['params'])} != {len(f['params'])}")
            continue
        for i, ((_, ct), (_, rt)) in enumerate(zip(f["params"], g["params"])):
            if ct != rt:
                out.append(f"{name}: parameter {i} is {rt}, header says {ct}")
        if g["ret"] != f["ret"]:
            out.append(f"{name}: returns {g['ret']}, header says {f['ret']}")
    for name in r["funcs"]:
        if name not in c["funcs"]:
            out.append(f"fn {name} is not in the headers")
    for name, fields in c["structs"].items():
        if r["structs"].get(name) != fields:
            out.append(f"struct {name} differs")
    for name, v in c["consts"].items():
        if r["consts"].get(name) != v:
            out.append(f"const {name} differs")
    return out


def write_integration(path=INTEGRATION) -> None:
    """Replaces INTEGRATION.md's src/lib.rs block with gen_rust()."""
    src = open(path).read()
    m = re.search(r"(`src/lib\.rs`[^\n]*\n+```rust\n)(.*?)(```)", src, re.S)
    open(path, "w").write(src[:m.start(2)] + gen_rust() + src[m.end(2):])


if __name__ == "__main__":
    if "--write" in sys.argv:
        write_integration()
        sys.argv.append("--check")
    if "--check" in sys.argv:
        d = diff(parse_headers(), parse_rust(integration_block()))
        print("\n".join(d) if d else "INTEGRATION.md src/lib.rs matches include/*.h")
        sys.exit(1 if d else 0)
    sys.stdout.write(gen_rust())
