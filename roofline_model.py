"""Algorithmic VALU models behind every bench.py line's roofline.

Each model is a frozen count of gfx950 lane-instructions per report (one report per lane), built
from the cheapest instruction sequence known for each primitive (PRIM) times the number of times
the algorithm needs it.  So `model x reports/s / 78.6 T` is a roofline fraction that instruction
bloat cannot raise: a kernel that issued fewer instructions would have to use a cheaper sequence
than any written down here.  The PMC-measured issued instructions per report (SQ_INSTS_VALU x 64 /
reports, profiles/) are printed beside each model as `issued_over_model`.

Primitive counts follow the algorithms the reference runs (prio 0.16.2 / VDAF-08 Prio3, RFC 9180
HPKE); the structure of every count is written next to it.  This file is measurement code: the
product path never imports it.
"""
from __future__ import annotations

import math

# lane-instructions per primitive (gfx950)
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
    # Field64 (Goldilocks, p = 2^64 - 2^32 + 1) as two 32-bit limbs
    f64_mul=16,        # 4 v_mad_u64_u32 + carries (128-bit product) + 2^64 = 2^32 - 1 fold
    f64_mac=8,         # 4 v_mad_u64_u32 + 4 carry adds into a 3-word accumulator
    f64_reduce=12,     # 3-word accumulator -> canonical
    f64_add=6,         # 64-bit add + conditional subtract of p
    f64_sum_add=3,
    sha256_compress=1440,  # 64 rounds x 15 (bitop3 Ch/Maj, alignbit rotates, add3) + 48 x 10
    # HPKE (fe25519 counts are the generated asm routines of janus_amd/csrc/fe25519_asm.h,
    # tools/gen_fe25519_asm.py: one statement each, no moves or hazard pads)
    fe25519_mul=177, fe25519_sqr=147, fe25519_add=19, fe25519_sub=19, fe25519_mul_small=29,
    # GF(p256): 64 (36 for squares) v_mad_u64_u32 + as many carries, the column normalisation
    # (~30) and the NIST fast reduction as nine 8-word add/sub chains (~90)
    p256_mul=250, p256_sqr=200, p256_add=24,
    # GF(2^448 - 2^224 - 1) in 16 x 28-bit limbs (x448_device.h): 256 (136 for squares)
    # v_mad_u64_u32 into 64-bit columns, the 31-column carry (~95) and the 2^448 = 2^224 + 1 fold
    fe448_mul=380, fe448_sqr=260, fe448_add=34, fe448_mul_small=50,
    # GF(2^521 - 1) in 18 x 29-bit limbs (p521_device.h): 324 (171 + 18 doublings for squares)
    # v_mad_u64_u32, the 35-column carry (~105), the 2^522 = 2 fold and a limb carry (~90)
    p521_mul=520, p521_sqr=385, p521_add=72,
    # GF(p384) Montgomery (CIOS) in 12 saturated words: 144 + 130 v_mad_u64_u32 (the reduction
    # skips p's two zero words) + one carry add each, the conditional subtract (~36); squares
    # run as products.  An add / sub is a 12-word carry chain + the conditional correction
    p384_mul=600, p384_add=48,
    sha512_compress=4000,  # 80 rounds x ~33 (64-bit words on 32-bit halves) + 64 x ~22 schedule
    aes_round=36,      # T-table round: 16 byte extracts + 16 XORs + 4 key XORs (lookups are LDS)
    ghash_block=320,   # 4-bit table (Shoup) GF(2^128) multiply: 32 nibble steps x ~10
    chacha_block=960,  # 20 rounds x 4 quarter rounds x 12 (add, xor, v_alignbit rotate)
    poly1305_block=60,  # 5 x 26-bit limbs: 25 v_mad_u64_u32 + carries
)
PERM = 12 * PRIM["keccak_round"]  # Keccak-p[1600, 12] (TurboSHAKE128)
RATE = 168


def blocks(nbytes: int) -> int:
    """Keccak permutations to absorb a short message and squeeze nbytes (first block free)."""
    return max(1, -(-nbytes // RATE))


def next_pow2(x: int) -> int:
    p = 1
    while p < x:
        p *= 2
    return p


def optimal_chunk_length(meas_len: int) -> int:
    """prio flp/gadgets.rs optimal_chunk_length (as oracle/fpvec_py.py restates it)."""
    if meas_len <= 1:
        return 1
    best = None
    for log2 in range(next_pow2(meas_len).bit_length(), 0, -1):
        calls = (1 << log2) - 1
        chunk = -(-meas_len // calls)
        cost = 2 * chunk + 2 * (next_pow2(1 + calls) - 1) + 1
        if best is None or cost < best[0]:
            best = (cost, chunk)
    return best[1]


def lagrange(P: int):
    """(muls, adds) for the P Lagrange basis values at t: P/8 phases of an 8-point DFT of a
    geometric sequence (P = 32 is k_query_h's four phases): t powers, the phase sums and start
    values, 7 sequence steps and 5 non-trivial twiddles per 8 points, 24 butterfly add/subs."""
    ph = max(1, P // 8)
    pts = P // ph
    tw = {8: 5, 4: 1, 2: 0, 1: 0}[pts]
    lg = int(math.log2(pts)) if pts > 1 else 0
    muls = int(math.log2(max(P, 2))) + 3 + ph + (ph - 1) + ph * (pts - 1) + ph * tw
    return muls, ph * pts * lg + 6


class Field:
    def __init__(self, es: int):
        self.es = es
        k = "f128" if es == 16 else "f64"
        self.mul, self.mac = PRIM[k + "_mul"], PRIM[k + "_mac"]
        self.reduce, self.add = PRIM[k + "_reduce"], PRIM[k + "_add"]
        self.sum_add = PRIM[k + "_sum_add"]


def _ps_mul_query(F: Field, meas: int, chunk: int, lead: bool):
    """FLP query of a ParallelSum(Mul, chunk) range circuit over `meas` elements (Histogram,
    SumVec, FPVec gadget 0; VDAF-08 A.5.5 / prio flp.rs query): Lagrange basis at t, the two
    wire sums A (weighted by beta_k = L_(k+1) r^(Ck)) and B per element as lazy MACs, the seeds,
    p(t) by Horner and the range sum through sigma (sum_c p(alpha^c)), the gadget at t."""
    calls = -(-meas // chunk)
    P = next_pow2(calls + 1)
    glen = 2 * (P - 1) + 1
    lm, la = lagrange(P)
    muls = lm + (glen - 1) + chunk.bit_length() + 2 * calls + chunk + 1 + 3 + 2
    macs = (glen - 1) + 2 * meas + 4 * chunk
    reduces = 1 + 3 * chunk + chunk // 2
    adds = la + calls + (glen - 1) + 3 * chunk + 6
    ops = muls * F.mul + macs * F.mac + reduces * F.reduce + adds * F.add + meas * F.sum_add
    verifier = 2 * chunk + 2
    return ops + (0 if lead else verifier * PRIM["lt_p"])


def instance(kind: str, sz, bits=0, length=0, chunk=0) -> dict:
    """The FLP / XOF structure of a Prio3 instance (sizes sz = prio3_sizes)."""
    return dict(kind=kind, es=sz.field_bytes, meas=sz.meas_len, proof=sz.proof_len,
                jr=sz.joint_rand_len, out=sz.out_len, verifier=sz.verifier_len,
                bits=bits, length=length, chunk=chunk)


def _xof_helper(I: dict) -> int:
    """Helper prepare_init XOF work: query randomness, measurement share, proofs share, and with
    joint randomness the joint-rand part (42-byte prefix + the share, funnel-shifted words), the
    corrected seed and the joint randomness; one canonical check per squeezed element."""
    es, jr = I["es"], I["jr"] > 0
    qr = 2 if I["kind"] == "fpvec" else 1
    perms = blocks(qr * es) + blocks(I["meas"] * es) + blocks(I["proof"] * es)
    jr_blocks = (42 + I["meas"] * es) // RATE + 1 if jr else 0
    if jr:
        perms += jr_blocks + 1 + blocks(I["jr"] * es)
    squeezed = I["meas"] + I["proof"] + I["jr"] + qr
    return perms * PERM + squeezed * PRIM["lt_p"] + jr_blocks * 42


def _query(I: dict, lead: bool = False) -> int:
    """FLP query + decide (helper) or verifier share (leader) of one report."""
    F = Field(I["es"])
    kind = I["kind"]
    if kind in ("histogram", "sumvec"):
        q = _ps_mul_query(F, I["meas"], I["chunk"], lead)
        if kind == "sumvec":
            q += I["meas"] * F.sum_add  # truncate: sum_b 2^b m_b per entry
    elif kind == "sum":
        # PolyEval(x^2 - x) on one wire, K = bits calls: f(t) (K + 1 MACs), the validity weights
        # W = DFT of r^c (a second geometric DFT) dotted with the folded proof polynomial, p(t)
        calls = I["meas"]
        P = next_pow2(calls + 1)
        glen = 2 * (P - 1) + 1
        lm, la = lagrange(P)
        q = ((2 * lm + glen + 4) * F.mul + (calls + 1 + P) * F.mac + 3 * F.reduce +
             (2 * la + glen + 4) * F.add + calls * F.sum_add + I["verifier"] * PRIM["lt_p"])
    elif kind == "count":
        # Mul(m, m) - m, one call, P = 2: both wire values, p(t) (3 coefficients), v
        q = 12 * F.mul + 8 * F.add + I["verifier"] * PRIM["lt_p"]
    elif kind == "fpvec":
        E = I["length"]
        n_bits = I["bits"]
        c0 = optimal_chunk_length(I["meas"])
        c1 = optimal_chunk_length(E)
        q = _ps_mul_query(F, I["meas"], c0, lead)
        # gadget 1: ParallelSum(PolyEval(y^2 - 2^n y), c1) over the decoded entries (decode:
        # n shift-adds per entry): Lagrange at t1, one wire MAC per entry, p1(t1), sigma sum
        k1 = -(-E // c1)
        P1 = next_pow2(k1 + 1)
        g1 = 2 * (P1 - 1) + 1
        lm, la = lagrange(P1)
        q += ((lm + g1 + 2 * k1 + 4) * F.mul + (E + 2 * g1) * F.mac + (c1 + 3) * F.reduce +
              (la + g1 + c1) * F.add + E * n_bits * F.sum_add)
    else:
        raise ValueError(kind)
    if I["jr"] and not lead:
        q += PERM  # the prepare message (joint-rand seed of both parts)
    return q


def helper_model(I: dict) -> dict:
    """Minimum lane-instructions per report of the helper step: prepare_init + decide +
    prepare message + prepare_next check + accumulate (one lazy add per output element)."""
    F = Field(I["es"])
    xof, query = _xof_helper(I), _query(I)
    acc = I["out"] * F.sum_add
    return dict(xof=xof, query=query, accumulate=acc, total=xof + query + acc)


def leader_model(I: dict) -> dict:
    """Leader prepare_init (agg_id 0) on the explicit input share: canonical check of every
    share element, query randomness, joint-rand part over the share, corrected seed, joint
    randomness, the query writing the verifier share; prepare_next compares the helper's
    message with the corrected seed; accumulate."""
    F = Field(I["es"])
    es = I["es"]
    jr_blocks = (42 + I["meas"] * es) // RATE + 1 if I["jr"] else 0
    perms = blocks(es * (2 if I["kind"] == "fpvec" else 1)) + jr_blocks + \
        ((1 + blocks(I["jr"] * es)) if I["jr"] else 0)
    checks = (I["meas"] + I["proof"]) * PRIM["lt_p"]
    xof = perms * PERM + checks + jr_blocks * 42
    query = _query(I, lead=True)
    acc = I["out"] * F.sum_add
    return dict(xof=xof, query=query, accumulate=acc, total=xof + query + acc)


def hpke_model(kem: str, aead: int, pt_len: int = 48 + 8 + 32 + 16, aad_len: int = 32 + 16 + 8 + 4 + 32) -> dict:
    """One DAP input-share open: the KEM's DH, DHKEM ExtractAndExpand + the RFC 9180 key schedule
    (19 SHA-256 compressions with the HMAC midstates of constant keys precomputed), and the AEAD
    over the plaintext (PlaintextInputShare) and AAD (InputShareAad)."""
    if kem == "x25519":
        step = (5 * PRIM["fe25519_mul"] + 4 * PRIM["fe25519_sqr"] + PRIM["fe25519_mul_small"] +
                4 * PRIM["fe25519_add"] + 4 * PRIM["fe25519_sub"] + 64)  # RFC 7748 + 2 cswaps
        inv = 254 * PRIM["fe25519_sqr"] + 11 * PRIM["fe25519_mul"]
        dh = 255 * step + inv + PRIM["fe25519_mul"] + 24
        compress = 19
    elif kem == "x448":
        # RFC 7748 ladder over 448 bits + the p - 2 inversion; HKDF-SHA512 (kem_context 112 B)
        step = (5 * PRIM["fe448_mul"] + 4 * PRIM["fe448_sqr"] + PRIM["fe448_mul_small"] +
                8 * PRIM["fe448_add"] + 64)
        dh = 448 * step + 446 * PRIM["fe448_sqr"] + 14 * PRIM["fe448_mul"] + 40
        compress = 21
    elif kem == "p384":
        M, S, A = PRIM["p384_mul"], PRIM["p384_mul"], PRIM["p384_add"]
        # ecdh_a3.h as for P-521 (Montgomery products, squares as products), 96 digits
        dbl = 4 * M + 4 * S + 13 * A
        madd = 8 * M + 3 * S + 12 * A
        inv = 385 * S + 15 * M                 # p - 2 addition chain (p384_device.h inv)
        check = 3 * M + 2 * S + 4 * A
        table = 5 * dbl + 7 * madd + inv + 39 * M + 7 * S
        dh = check + table + 94 * (4 * dbl + madd) + 5 * dbl + madd + inv + M + S + 2 * M
        compress = 23  # HKDF-SHA384: kem_context = enc || pkR is 194 bytes
    elif kem == "p521":
        M, S, A = PRIM["p521_mul"], PRIM["p521_sqr"], PRIM["p521_add"]
        # ecdh_a3.h, counted from its code (the r4 model charged a 12M + 4S
        # general addition where the code runs the 8M + 3S mixed one): a = -3 Jacobian
        # doublings (dbl-2001-b), mixed additions (madd-2007-bl), the odd multiples P..15P by 5
        # doublings and 7 mixed additions made affine by Montgomery's trick, a fixed signed w = 4
        # window over the 131 host-recoded digits, affine output
        dbl = 4 * M + 4 * S + 13 * A           # three small multiples counted as two adds each
        madd = 8 * M + 3 * S + 12 * A
        inv = 520 * S + 13 * M                 # p - 2 addition chain
        check = 3 * M + 2 * S + 4 * A          # y^2 = x^3 - 3x + b
        table = 5 * dbl + 7 * madd + inv + 39 * M + 7 * S
        dh = check + table + 129 * (4 * dbl + madd) + 5 * dbl + madd + inv + M + S
        compress = 23  # kem_context = enc || pkR is 266 bytes
    else:
        M, S, A = PRIM["p256_mul"], PRIM["p256_sqr"], PRIM["p256_add"]
        # the w = 4 window of p256_device.h (r03; a small multiple counted as two adds)
        dbl = 4 * M + 4 * S + 13 * A           # dbl-2001-b (a = -3), Z3 = 2 Y Z
        madd = 8 * M + 3 * S + 12 * A          # madd-2007-bl, Z3 = 2 Z1 H
        inv = 255 * S + 12 * M                 # p - 2 addition chain
        # 3P .. 15P: 6 doublings, 7 mixed additions, then affine by Montgomery's trick
        table = 6 * dbl + 7 * madd + inv + 39 * M + 7 * S + A
        check = 3 * M + 2 * S + 4 * A          # y^2 = x^3 - 3x + b
        # 63 windows of 4 doublings + 1 addition (the last one also doubles, for the R = T case)
        dh = check + table + 63 * (4 * dbl + madd) + dbl + inv + M + S
        compress = 21  # kem_context = enc || pkR is 130 bytes (three-block HMAC message)
    ct_blocks = -(-pt_len // 16)
    if aead == 3:
        aead_ops = (ct_blocks // 4 + 2) * PRIM["chacha_block"] + \
            (ct_blocks + -(-aad_len // 16) + 1) * PRIM["poly1305_block"]
    else:
        rounds = 10 if aead == 1 else 14
        aead_ops = (ct_blocks + 2) * rounds * PRIM["aes_round"] + rounds * 20 + \
            (ct_blocks + -(-aad_len // 16) + 1) * PRIM["ghash_block"]
    kdf = compress * PRIM["sha512_compress" if kem in ("x448", "p521", "p384") else "sha256_compress"]
    return dict(dh=dh, kdf=kdf, aead=aead_ops, total=dh + kdf + aead_ops)


def mp64_model(sz, bits: int, length: int, chunk: int, proofs: int) -> dict:
    """Prio3SumVecField64MultiproofHmacSha256Aes128 helper step (Janus vdaf.rs:173-195): every
    XOF is HMAC-SHA256 (seed-keyed; the inner/outer midstates of the 32-byte seed cost 2
    compressions) over dst || binder, then an AES-128 CTR keystream (key schedule + one block
    per 16 bytes).  Per report: the measurement share, `proofs` proofs shares, query and joint
    randomness, the joint-rand part (HMAC over the encoded share), the corrected seed; then one
    ParallelSum(Mul) FLP query per proof over Field64, decide, prepare message, truncate."""
    F = Field(8)
    meas, proof = sz.meas_len, sz.proof_len // proofs
    aes = lambda nbytes: 10 * PRIM["aes_round"] * -(-nbytes // 16) + 200
    hmac = lambda msg_bytes: (2 + 2 + -(-(msg_bytes + 9) // 64)) * PRIM["sha256_compress"]
    xof = (hmac(16) + aes(meas * 8) + hmac(16) + aes(proofs * proof * 8) +
           hmac(8 + meas * 8) + hmac(64) + hmac(16) + aes(proofs * 2 * 8) +
           hmac(16) + aes(proofs * 8) + meas + proofs * proof) * 1
    query = proofs * (_ps_mul_query(F, meas, chunk, False) - (2 * chunk + 2) * PRIM["lt_p"]) + \
        proofs * (2 * chunk + 2) * PRIM["lt_p"] + hmac(64) + meas * F.sum_add
    acc = sz.out_len * F.sum_add
    return dict(xof=xof, query=query, accumulate=acc, total=xof + query + acc)
