"""Generates janus_amd/csrc/fe25519_asm.h: GF(2^255 - 19) multiply / square / add / subtract /
multiply-by-121665 for the HPKE opener's X25519 ladder, each ONE inline-asm statement.

Why asm: written in C, every carry chain of these routines is a VCC chain that the compiler
pads with s_nop on gfx950 (~570 per ladder step), and the column accumulators of the products
were zero-initialised with ~450 v_mov per step.  Here the first product of a column writes it
(v_mad_u64_u32 ..., 0), the first carry of a column creates its overflow word (v_cndmask), and
the scratch lives in fixed registers v40-v82, so the 32-bit halves of the 64-bit columns can be
addressed directly in the normalisation (no sub-register syntax exists for asm operands).

Layout of the scratch: column c_k (64-bit) at v[40+2k : 41+2k] (k = 0..14), overflow word h_k
at v(69+k) (k = 1..13).  After normalisation, 512-bit word w_t sits in the even columns'
registers: w_(2m) = v(40+4m), w_(2m+1) = v(41+4m); the odd columns' registers and h_1, h_2 are
then free for the reduction products T_i = 38 * w_(8+i) at v[42+4i : 43+4i] (i < 7) and v[70:71].
Values are loosely reduced: inputs and outputs in [0, 2^256), 2^256 = 38 (mod p).

Usage: python tools/gen_fe25519_asm.py > janus_amd/csrc/fe25519_asm.h
"""

CLOB = ", ".join(f'"v{r}"' for r in range(40, 83))


def c_lo(k):
    return f"v{40 + 2 * k}"


def c_hi(k):
    return f"v{41 + 2 * k}"


def c_pair(k):
    return f"v[{40 + 2 * k}:{41 + 2 * k}]"


def h(k):
    return f"v{69 + k}"


def w(t):
    m, odd = divmod(t, 2)
    return f"v{40 + 4 * m + odd}"


def t_pair(i):
    return f"v[{42 + 4 * i}:{43 + 4 * i}]" if i < 7 else "v[70:71]"


def t_lo(i):
    return f"v{42 + 4 * i}" if i < 7 else "v70"


def t_hi(i):
    return f"v{43 + 4 * i}" if i < 7 else "v71"


def products(pairs, A, B):
    """column MAC of the products A[i] * B[j] for (i, j) in pairs; returns (code, set of k with
    an overflow word)"""
    out, seen, hov = [], set(), set()
    for i, j in pairs:
        k = i + j
        if k not in seen:
            out.append(f"v_mad_u64_u32 {c_pair(k)}, vcc, {A(i)}, {B(j)}, 0")
            seen.add(k)
        else:
            out.append(f"v_mad_u64_u32 {c_pair(k)}, vcc, {A(i)}, {B(j)}, {c_pair(k)}")
            if k not in hov:
                out.append(f"v_cndmask_b32_e64 {h(k)}, 0, 1, vcc")
                hov.add(k)
            else:
                out.append(f"v_addc_co_u32 {h(k)}, vcc, 0, {h(k)}, vcc")
    return out, seen, hov


def normalise(hov):
    """w = E + O + H in place (E: even columns, O: odd columns at +32 bits, H: h_k at word k+2)"""
    out = [f"v_add_co_u32 {w(1)}, vcc, {w(1)}, {c_lo(1)}"]
    for t in range(2, 15):
        src = c_hi(t - 1) if t % 2 == 0 else c_lo(t)
        out.append(f"v_addc_co_u32 {w(t)}, vcc, {w(t)}, {src}, vcc")
    out.append(f"v_addc_co_u32 {w(15)}, vcc, 0, {w(15)}, vcc")
    ks = sorted(hov)
    first = True
    for t in range(3, 16):
        k = t - 2
        if first:
            if k in hov:
                out.append(f"v_add_co_u32 {w(t)}, vcc, {w(t)}, {h(k)}")
                first = False
            continue
        if k in hov:
            out.append(f"v_addc_co_u32 {w(t)}, vcc, {w(t)}, {h(k)}, vcc")
        else:
            out.append(f"v_addc_co_u32 {w(t)}, vcc, 0, {w(t)}, vcc")
    return out


def reduce_to(outs):
    """r = w_lo + 38 w_hi, folded twice; outs = the 8 output operand names"""
    out = [f"v_mad_u64_u32 {t_pair(i)}, vcc, {w(8 + i)}, 38, 0" for i in range(8)]
    out.append(f"v_add_co_u32 {outs[0]}, vcc, {w(0)}, {t_lo(0)}")
    for i in range(1, 8):
        out.append(f"v_addc_co_u32 {outs[i]}, vcc, {w(i)}, {t_lo(i)}, vcc")
    out.append(f"v_addc_co_u32 {t_lo(7)}, vcc, 0, {t_hi(7)}, vcc")  # top
    out.append(f"v_add_co_u32 {outs[1]}, vcc, {outs[1]}, {t_hi(0)}")
    for i in range(2, 8):
        out.append(f"v_addc_co_u32 {outs[i]}, vcc, {outs[i]}, {t_hi(i - 1)}, vcc")
    out.append(f"v_addc_co_u32 {t_lo(7)}, vcc, 0, {t_lo(7)}, vcc")
    out += fold(outs, t_lo(7), mul38=True)
    return out


def fold(outs, top, mul38):
    """outs += 38 * top (top small), then the second carry (<= 1) folded into outs[0]"""
    out = []
    if mul38:
        out.append(f"v_mul_u32_u24 {top}, 38, {top}")
    out.append(f"v_add_co_u32 {outs[0]}, vcc, {outs[0]}, {top}")
    for i in range(1, 8):
        out.append(f"v_addc_co_u32 {outs[i]}, vcc, 0, {outs[i]}, vcc")
    out.append(f"v_cndmask_b32_e64 {top}, 0, 38, vcc")
    out.append(f"v_add_u32 {outs[0]}, {outs[0]}, {top}")
    return out


def emit(name, body, outs, ins, clob=True, extra_out=""):
    code = "\n".join(f'      "{ln}\\n\\t"' for ln in body)
    return f"""DEV fe {name}({ins[0]}) {{
  fe r;
  asm volatile(
{code}
      : {", ".join(f'"=&v"(r.v[{i}])' for i in range(8))}{extra_out}
      : {ins[1]}
      : "vcc"{", " + CLOB if clob else ""});
  return r;
}}
"""


OUT = [f"%{i}" for i in range(8)]


def gen_mul():
    A = lambda i: f"%{8 + i}"
    B = lambda j: f"%{16 + j}"
    body, seen, hov = products([(i, j) for i in range(8) for j in range(8)], A, B)
    body += normalise(hov)
    body += reduce_to(OUT)
    ins = ", ".join(f'"v"(a.v[{i}])' for i in range(8)) + ", " + \
        ", ".join(f'"v"(b.v[{i}])' for i in range(8))
    return emit("fe_mul", body, OUT, ("const fe& a, const fe& b", ins))


def gen_sqr():
    A = lambda i: f"%{8 + i}"
    body = [f"v_mov_b64 {c_pair(0)}, 0", f"v_mov_b64 {c_pair(14)}, 0"]
    pb, seen, hov = products([(i, j) for i in range(8) for j in range(i + 1, 8)], A, A)
    body += pb
    body += normalise(hov)
    # 2S
    for t in range(15, 0, -1):
        body.append(f"v_alignbit_b32 {w(t)}, {w(t)}, {w(t - 1)}, 31")
    body.append(f"v_lshlrev_b32 {w(0)}, 1, {w(0)}")
    # + D = sum a_i^2 2^(64 i): into the T registers, then one 16-word chain
    for i in range(8):
        body.append(f"v_mad_u64_u32 {t_pair(i)}, vcc, {A(i)}, {A(i)}, 0")
    body.append(f"v_add_co_u32 {w(0)}, vcc, {w(0)}, {t_lo(0)}")
    for t in range(1, 16):
        src = t_lo(t // 2) if t % 2 == 0 else t_hi(t // 2)
        body.append(f"v_addc_co_u32 {w(t)}, vcc, {w(t)}, {src}, vcc")
    body += reduce_to(OUT)
    ins = ", ".join(f'"v"(a.v[{i}])' for i in range(8))
    return emit("fe_sqr", body, OUT, ("const fe& a", ins))


def gen_add():
    A = [f"%{8 + i}" for i in range(8)]
    B = [f"%{16 + i}" for i in range(8)]
    body = [f"v_add_co_u32 %0, vcc, {A[0]}, {B[0]}"]
    body += [f"v_addc_co_u32 %{i}, vcc, {A[i]}, {B[i]}, vcc" for i in range(1, 8)]
    body.append("v_cndmask_b32_e64 %24, 0, 38, vcc")
    body += fold(OUT, "%24", mul38=False)
    ins = ", ".join(f'"v"(a.v[{i}])' for i in range(8)) + ", " + \
        ", ".join(f'"v"(b.v[{i}])' for i in range(8))
    code = "\n".join(f'      "{ln}\\n\\t"' for ln in body)
    return f"""DEV fe fe_add(const fe& a, const fe& b) {{
  fe r;
  uint32_t t;
  asm volatile(
{code}
      : {", ".join(f'"=&v"(r.v[{i}])' for i in range(8))}
      : {ins}, "v"(0u)
      : "vcc");
  (void)t;
  return r;
}}
""".replace('"v"(0u)', '"v"(0u)')


def gen_sub():
    A = [f"%{9 + i}" for i in range(8)]
    B = [f"%{17 + i}" for i in range(8)]
    T = "%8"
    body = [f"v_sub_co_u32 %0, vcc, {A[0]}, {B[0]}"]
    body += [f"v_subb_co_u32 %{i}, vcc, {A[i]}, {B[i]}, vcc" for i in range(1, 8)]
    body.append(f"v_cndmask_b32_e64 {T}, 0, 38, vcc")
    body.append(f"v_sub_co_u32 %0, vcc, %0, {T}")
    body += [f"v_subbrev_co_u32 %{i}, vcc, 0, %{i}, vcc" for i in range(1, 8)]
    body.append(f"v_cndmask_b32_e64 {T}, 0, 38, vcc")
    body.append(f"v_sub_u32 %0, %0, {T}")
    ins = ", ".join(f'"v"(a.v[{i}])' for i in range(8)) + ", " + \
        ", ".join(f'"v"(b.v[{i}])' for i in range(8))
    code = "\n".join(f'      "{ln}\\n\\t"' for ln in body)
    return f"""DEV fe fe_sub(const fe& a, const fe& b) {{
  fe r;
  uint32_t t;
  asm volatile(
{code}
      : {", ".join(f'"=&v"(r.v[{i}])' for i in range(8))}, "=&v"(t)
      : {ins}
      : "vcc");
  return r;
}}
"""


def gen_add2():
    A = [f"%{9 + i}" for i in range(8)]
    B = [f"%{17 + i}" for i in range(8)]
    T = "%8"
    body = [f"v_add_co_u32 %0, vcc, {A[0]}, {B[0]}"]
    body += [f"v_addc_co_u32 %{i}, vcc, {A[i]}, {B[i]}, vcc" for i in range(1, 8)]
    body.append(f"v_cndmask_b32_e64 {T}, 0, 38, vcc")
    body += fold(OUT, T, mul38=False)
    ins = ", ".join(f'"v"(a.v[{i}])' for i in range(8)) + ", " + \
        ", ".join(f'"v"(b.v[{i}])' for i in range(8))
    code = "\n".join(f'      "{ln}\\n\\t"' for ln in body)
    return f"""DEV fe fe_add(const fe& a, const fe& b) {{
  fe r;
  uint32_t t;
  asm volatile(
{code}
      : {", ".join(f'"=&v"(r.v[{i}])' for i in range(8))}, "=&v"(t)
      : {ins}
      : "vcc");
  return r;
}}
"""


def gen_mul_small():
    A = [f"%{10 + i}" for i in range(8)]
    K, T = "%9", "%8"
    body = [f"s_mov_b32 {K}, 121665"]
    for i in range(8):
        body.append(f"v_mad_u64_u32 {t_pair(i)}, vcc, {A[i]}, {K}, 0")
    body.append(f"v_mov_b32 %0, {t_lo(0)}")
    body.append(f"v_add_co_u32 %1, vcc, {t_lo(1)}, {t_hi(0)}")
    for i in range(2, 8):
        body.append(f"v_addc_co_u32 %{i}, vcc, {t_lo(i)}, {t_hi(i - 1)}, vcc")
    body.append(f"v_addc_co_u32 {T}, vcc, 0, {t_hi(7)}, vcc")
    body += fold(OUT, T, mul38=True)
    ins = ", ".join(f'"v"(a.v[{i}])' for i in range(8))
    code = "\n".join(f'      "{ln}\\n\\t"' for ln in body)
    return f"""DEV fe fe_mul121665(const fe& a) {{
  fe r;
  uint32_t t, k;
  asm volatile(
{code}
      : {", ".join(f'"=&v"(r.v[{i}])' for i in range(8))}, "=&v"(t), "=&s"(k)
      : {ins}
      : "vcc", {CLOB});
  return r;
}}
"""


HEADER = """// fe25519_asm.h -- GENERATED by tools/gen_fe25519_asm.py (see its docstring); do not edit.
// GF(2^255 - 19) in 8 x 32-bit limbs, loosely reduced in [0, 2^256), for hpke.hip.
#pragma once
"""

if __name__ == "__main__":
    print(HEADER)
    print(gen_mul())
    print(gen_sqr())
    print(gen_add2())
    print(gen_sub())
    print(gen_mul_small())
