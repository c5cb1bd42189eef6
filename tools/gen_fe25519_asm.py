"""Emits the inline-asm column MAC blocks of janus_amd/csrc/hpke.hip (fe_mul / fe_sqr of
GF(2^255 - 19) in 8 x 32-bit limbs): every partial product a_i * b_j goes into the 64-bit column
c[i + j] with v_mad_u64_u32, and the column's carry-out into its overflow word h[i + j]
(v_addc_co_u32) -- one asm statement, so the compiler's VCC hazard padding never splits it.
Operands: %0..%14 c[0..14] (u64), %15..%27 h[1..13], then the inputs."""


def block(pairs, n_in):
    lines = []
    for i, j in pairs:
        k = i + j
        a = 28 + i
        b = 28 + (8 + j if n_in == 16 else j)
        lines.append(f'"v_mad_u64_u32 %{k}, vcc, %{a}, %{b}, %{k}\\n\\t"')
        if 1 <= k <= 13:
            lines.append(f'"v_addc_co_u32 %{14 + k}, vcc, 0, %{14 + k}, vcc\\n\\t"')
    return "\n      ".join(lines)


mul_pairs = [(i, j) for i in range(8) for j in range(8)]
sqr_pairs = [(i, j) for i in range(8) for j in range(i + 1, 8)]
print("// fe_mul products\n      " + block(mul_pairs, 16))
print("// fe_sqr off-diagonal products\n      " + block(sqr_pairs, 8))
