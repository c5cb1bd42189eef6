"""Generates janus_amd/csrc/p256_asm.h: the GF(p256) field operations of the HPKE opener's
P-256 ECDH (p256_device.h), each ONE inline-asm statement, inlined at every use.

p = 2^256 - 2^224 + 2^192 + 2^96 - 1; values are 8 little-endian 32-bit limbs, loosely reduced in
[0, 2^256); C = 2^256 - p = 2^224 - 2^192 - 2^96 + 1 (words [1, 0, 0, -1, -1, -1, -2, 0]).

  p256_mul / p256_sqr  the 512-bit product (tools/gen_fe25519_asm.py's column-MAC and
                       normalisation emitters and its scratch layout v40-v82), then the NIST fast
                       reduction (FIPS 186-4 D.2.3, s1 + 2 s2 + 2 s3 + s4 + s5 - s6 - s7 - s8 - s9)
                       as ten add / subtract chains over the 16 product words, started from 5p (so
                       the running top word t never goes negative), then t * C added as one
                       non-negative 8-word value and its carry folded as C once more;
  p256_add / p256_sub  one 8-word carry (borrow) chain, then the carry (borrow) folded twice as
                       +C (-C): a loose result never needs a third;
  p256_mul_small       a x k for a small constant k (8 v_mad_u64_u32), the top word folded as in
                       the reduction.

Written in C (r02zm), each product was an out-of-line call with its operands through the stack,
and every add / subtract folded three times in signed 64-bit words.

Usage: python tools/gen_p256_asm.py > janus_amd/csrc/p256_asm.h
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_fe25519_asm import CLOB, c_pair, normalise, products, t_hi, t_lo, t_pair, w  # noqa: E402

P = 2**256 - 2**224 + 2**192 + 2**96 - 1
C = 2**256 - P
K5 = (5 * P) % 2**256          # 5p = 4 * 2^256 + K5
assert 5 * P == 4 * 2**256 + K5
CW = [(C >> (32 * i)) & 0xFFFFFFFF for i in range(8)]
assert CW == [1, 0, 0, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFE, 0]
OUT = [f"%{i}" for i in range(8)]
# reduction temporaries: odd-column registers of the product scratch, free after normalise
TT, TU, TM, TW = "v42", "v43", "v46", "v47"


def lit(x):
    """an operand for a 32-bit constant (inline constants where the ISA has them)"""
    if x <= 64:
        return str(x)
    if x >= 0xFFFFFFF0:
        return str(x - 2**32)
    return hex(x)


def chain(sign, words, top):
    """OUT (+|-)= the 8-word term `words` (entries: a register name or None for zero), the carry
    (borrow) into `top`"""
    i0 = next(i for i, x in enumerate(words) if x is not None)
    op0, opc, opz = (("v_add_co_u32", "v_addc_co_u32", "v_addc_co_u32 {o}, vcc, 0, {o}, vcc")
                     if sign > 0 else
                     ("v_sub_co_u32", "v_subb_co_u32", "v_subbrev_co_u32 {o}, vcc, 0, {o}, vcc"))
    out = [f"{op0} {OUT[i0]}, vcc, {OUT[i0]}, {words[i0]}"]
    for i in range(i0 + 1, 8):
        out.append(opz.format(o=OUT[i]) if words[i] is None else
                   f"{opc} {OUT[i]}, vcc, {OUT[i]}, {words[i]}, vcc")
    if top is not None:
        out.append(opz.format(o=top))
    return out


def fold_top(top):
    """OUT + top * 2^256 (0 <= top < 2^31) -> [0, 2^256).  top * C < 2^228 as one non-negative
    8-word addend: [t, 0, 0, -t, m, m, -t-1, t-1] (m = ~0 if t else 0; the -t words borrow from
    their neighbours), so one chain; its carry u in {0, 1} is folded as u * C once more."""
    T, U, M, A, W6, W7 = top, TU, TM, TW, "v50", "v51"
    out = [f"v_cmp_ne_u32 vcc, 0, {T}",
           f"v_cndmask_b32_e64 {M}, 0, -1, vcc",
           f"v_sub_u32 {A}, 0, {T}",
           f"v_add_u32 {W6}, -1, {A}",
           f"v_and_b32 {W6}, {M}, {W6}",
           f"v_add_u32 {W7}, -1, {T}",
           f"v_and_b32 {W7}, {M}, {W7}"]
    out += chain(+1, [T, None, None, A, M, M, W6, W7], None)
    out.append(f"v_cndmask_b32_e64 {U}, 0, 1, vcc")
    out.append(f"v_sub_u32 {M}, 0, {U}")
    out.append(f"v_and_b32 {A}, {lit(0xFFFFFFFE)}, {M}")
    out += chain(+1, [U, None, None, M, M, M, A, None], None)
    return out


def nist_reduce():
    """w(0..15) (normalised product) -> OUT, FIPS 186-4 D.2.3 from 5p"""
    c = [w(t) for t in range(16)]
    Z = None
    out = [f"v_add_co_u32 {OUT[0]}, vcc, {lit(K5 & 0xFFFFFFFF)}, {c[0]}"]
    for i in range(1, 8):
        out.append(f"v_addc_co_u32 {OUT[i]}, vcc, {lit((K5 >> (32 * i)) & 0xFFFFFFFF)}, {c[i]}, vcc")
    out.append(f"v_cndmask_b32_e64 {TT}, 4, 5, vcc")
    terms = [  # (sign, little-endian words) of s2 .. s9
        (+1, [Z, Z, Z, c[11], c[12], c[13], c[14], c[15]]),
        (+1, [Z, Z, Z, c[11], c[12], c[13], c[14], c[15]]),
        (+1, [Z, Z, Z, c[12], c[13], c[14], c[15], Z]),
        (+1, [Z, Z, Z, c[12], c[13], c[14], c[15], Z]),
        (+1, [c[8], c[9], c[10], Z, Z, Z, c[14], c[15]]),
        (+1, [c[9], c[10], c[11], c[13], c[14], c[15], c[13], c[8]]),
        (-1, [c[11], c[12], c[13], Z, Z, Z, c[8], c[10]]),
        (-1, [c[12], c[13], c[14], c[15], Z, Z, c[9], c[11]]),
        (-1, [c[13], c[14], c[15], c[8], c[9], c[10], Z, c[12]]),
        (-1, [c[14], c[15], Z, c[9], c[10], c[11], Z, c[13]]),
    ]
    for sign, words in terms:
        out += chain(sign, words, TT)
    out += fold_top(TT)
    return out


def emit(name, args, body, ins, temps=0, clob=True):
    """temps: extra "=&v" outputs %8.. (compiler-allocated scratch) instead of the fixed layout"""
    code = "\n".join(f'      "{ln}\\n\\t"' for ln in body)
    tdecl = f"  uint32_t t[{temps}];\n" if temps else ""
    touts = "".join(f', "=&v"(t[{i}])' for i in range(temps))
    return f"""DEV fp {name}({args}) {{
  fp r;
{tdecl}  asm volatile(
{code}
      : {", ".join(f'"=&v"(r.v[{i}])' for i in range(8))}{touts}
      : {ins}
      : "vcc"{", " + CLOB if clob else ""});
  return r;
}}
"""


def ins8(x):
    return ", ".join(f'"v"({x}.v[{i}])' for i in range(8))


def gen_mul():
    A = lambda i: f"%{8 + i}"
    B = lambda j: f"%{16 + j}"
    body, seen, hov = products([(i, j) for i in range(8) for j in range(8)], A, B)
    body += normalise(hov)
    body += nist_reduce()
    return emit("p256_mul", "const fp& a, const fp& b", body, ins8("a") + ", " + ins8("b"))


def gen_sqr():
    A = lambda i: f"%{8 + i}"
    body = [f"v_mov_b64 {c_pair(0)}, 0", f"v_mov_b64 {c_pair(14)}, 0"]
    pb, seen, hov = products([(i, j) for i in range(8) for j in range(i + 1, 8)], A, A)
    body += pb
    body += normalise(hov)
    for t in range(15, 0, -1):  # 2 S
        body.append(f"v_alignbit_b32 {w(t)}, {w(t)}, {w(t - 1)}, 31")
    body.append(f"v_lshlrev_b32 {w(0)}, 1, {w(0)}")
    for i in range(8):  # + sum a_i^2 2^(64 i)
        body.append(f"v_mad_u64_u32 {t_pair(i)}, vcc, {A(i)}, {A(i)}, 0")
    body.append(f"v_add_co_u32 {w(0)}, vcc, {w(0)}, {t_lo(0)}")
    for t in range(1, 16):
        src = t_lo(t // 2) if t % 2 == 0 else t_hi(t // 2)
        body.append(f"v_addc_co_u32 {w(t)}, vcc, {w(t)}, {src}, vcc")
    body += nist_reduce()
    return emit("p256_sqr", "const fp& a", body, ins8("a"))


def _addsub(name, sign):
    """a (+|-) b: one chain, then the carry (borrow) folded as (+|-)C twice; scratch in four
    compiler-allocated registers (no fixed-layout clobbers for this short op)"""
    tu, tm, tw = "%8", "%9", "%10"
    A = [f"%{11 + i}" for i in range(8)]
    B = [f"%{19 + i}" for i in range(8)]
    first, rest = (("v_add_co_u32", "v_addc_co_u32") if sign > 0 else
                   ("v_sub_co_u32", "v_subb_co_u32"))
    body = [f"{first} %0, vcc, {A[0]}, {B[0]}"]
    body += [f"{rest} %{i}, vcc, {A[i]}, {B[i]}, vcc" for i in range(1, 8)]
    body.append(f"v_cndmask_b32_e64 {tu}, 0, 1, vcc")
    for k in range(2):  # the second carry (borrow) is rare but possible for loose inputs
        body.append(f"v_sub_u32 {tm}, 0, {tu}")
        body.append(f"v_and_b32 {tw}, {lit(0xFFFFFFFE)}, {tm}")
        body += chain(sign, [tu, None, None, tm, tm, tm, tw, None], None)
        if k == 0:
            body.append(f"v_cndmask_b32_e64 {tu}, 0, 1, vcc")
    return emit(name, "const fp& a, const fp& b", body, ins8("a") + ", " + ins8("b"), temps=3,
                clob=False)


def gen_add():
    return _addsub("p256_add", +1)


def gen_sub():
    return _addsub("p256_sub", -1)


def gen_mul_small():
    A = [f"%{8 + i}" for i in range(8)]
    K = "%16"
    body = [f"v_mad_u64_u32 {t_pair(i)}, vcc, {A[i]}, {K}, 0" for i in range(8)]
    body.append(f"v_mov_b32 %0, {t_lo(0)}")
    body.append(f"v_add_co_u32 %1, vcc, {t_lo(1)}, {t_hi(0)}")
    for i in range(2, 8):
        body.append(f"v_addc_co_u32 %{i}, vcc, {t_lo(i)}, {t_hi(i - 1)}, vcc")
    body.append(f"v_addc_co_u32 {TT}, vcc, 0, {t_hi(7)}, vcc")
    body += fold_top(TT)
    return emit("p256_mul_small", "const fp& a, uint32_t k", body, ins8("a") + ', "s"(k)')


HEADER = """// p256_asm.h -- GENERATED by tools/gen_p256_asm.py (see its docstring); do not edit.
// GF(p256) multiply / square / add / subtract / small multiple, 8 x 32-bit limbs loosely
// reduced in [0, 2^256), one inline-asm statement each (p256_device.h).
#pragma once
"""

if __name__ == "__main__":
    print(HEADER)
    for g in (gen_mul, gen_sqr, gen_add, gen_sub, gen_mul_small):
        print(g())
