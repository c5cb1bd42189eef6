"""Prio3FixedPointBoundedL2VecSum restated in pure Python -- TEST INFRASTRUCTURE ONLY.

Janus instance: `VdafInstance::Prio3FixedPointBoundedL2VecSum { bitsize, dp_strategy, length }`
dispatched to prio's `Prio3FixedPointBoundedL2VecSumMultithreaded<FixedI16<U15>>` /
`<FixedI32<U31>>` (/root/reference/core/src/vdaf.rs:26-31, 292-335).  The type lives in prio
0.16.2 `flp/types/fixedpoint_l2.rs`, which is NOT in this container; SURVEY.md A.10/A.11(3)
records the circuit as approximate.  This file fixes one self-consistent reading of it and the
GPU path is pinned to THIS restatement (prio-byte parity UNPINNED, circuit reconstructed):

  * n = bits per entry (16 or 32); an entry x in [-1, 1) with raw signed value X (x = X/2^(n-1))
    is encoded as y = X + 2^(n-1) in [0, 2^n), as n little-endian bits;
  * the claimed squared norm N = sum_i (y_i - 2^(n-1))^2 = 2^(2n-2) ||x||^2 < 2^(2n-2) follows
    as 2n-2 little-endian bits; MEAS_LEN = n * entries + 2n - 2, OUTPUT_LEN = entries;
  * gadget 0 = ParallelSum(Mul, C0) range-checks every bit (the SumVec construction,
    `parallel_sum_range_checks` with joint randomness r0);
  * gadget 1 = ParallelSum(PolyEval(q), C1), q(y) = y^2 - 2^n y, over the decoded entries
    (chunks zero-padded, q(0) = 0); the computed norm is sum of gadget-1 outputs
    + entries * 2^(2n-2) / num_shares;
  * valid = r1 * range + r1^2 * (computed norm - claimed norm), JOINT_RAND_LEN 2;
  * C0 = optimal_chunk_length(MEAS_LEN), C1 = optimal_chunk_length(entries) (prio
    flp/gadgets.rs `optimal_chunk_length`, restated below);
  * FLP with two gadgets (VDAF-08 FlpBBCGGI19): proof = seeds0 || coeffs0 || seeds1 ||
    coeffs1, QUERY_RAND_LEN 2 (one t per gadget), verifier = [v, f0(t0).., p0(t0), f1(t1)..,
    p1(t1)]; decide checks v = 0 and G_i(f_i(t_i)) = p_i(t_i) for both gadgets;
  * truncate = the decoded entries y_i (the aggregate of c reports decodes to
    sum_i (agg_i - c 2^(n-1)) / 2^(n-1)).
Differential-privacy noise (dp_strategy) is added to aggregate shares at collection time, not in
prepare, and is out of scope here.  Algorithm id 0xFFFF0000.
"""
from __future__ import annotations

from oracle.prio3_py import Field128, Xof, next_pow2


def optimal_chunk_length(meas_len: int) -> int:
    """prio flp/gadgets.rs optimal_chunk_length: the chunk length minimising
    2 * chunk + 2 * ((1 + calls).next_power_of_two() - 1) + 1 over calls = 2^k - 1."""
    if meas_len <= 1:
        return 1
    best = None
    max_log2 = (next_pow2(meas_len).bit_length() - 1) + 1
    for log2 in range(max_log2, 0, -1):
        calls = (1 << log2) - 1
        chunk = -(-meas_len // calls)
        cost = 2 * chunk + 2 * (next_pow2(1 + calls) - 1) + 1
        if best is None or cost < best[0]:  # min_by_key keeps the first minimum
            best = (cost, chunk)
    return best[1]


def _ntt(F, a: list[int], inverse: bool = False) -> list[int]:
    """Evaluations of the polynomial a at alpha^i (alpha a primitive len(a)-th root), or the
    inverse map (values -> coefficients)."""
    n = len(a)
    p = F.p
    w = F.root(n)
    if inverse:
        w = F.inv(w)
    a = list(a)
    j = 0
    for i in range(1, n):  # bit-reversal permutation
        bit = n >> 1
        while j & bit:
            j ^= bit
            bit >>= 1
        j |= bit
        if i < j:
            a[i], a[j] = a[j], a[i]
    m = 2
    while m <= n:
        wm = pow(w, n // m, p)
        for s in range(0, n, m):
            ww = 1
            for k in range(m // 2):
                u, v = a[s + k], a[s + k + m // 2] * ww % p
                a[s + k] = (u + v) % p
                a[s + k + m // 2] = (u - v) % p
                ww = ww * wm % p
        m <<= 1
    if inverse:
        ninv = F.inv(n)
        a = [x * ninv % p for x in a]
    return a


class FpVecType:
    """Drop-in for prio3_py.Prio3Type in prio3_py.Prio3 (two gadgets)."""

    kind = "fpvec"

    def __init__(self, length: int, bits: int = 16):
        if bits not in (16, 32):
            raise ValueError("bitsize must be 16 or 32 (core/src/vdaf.rs:26-31)")
        self.F = Field128
        self.algo_id = 0xFFFF0000
        self.seed_size = 16
        self.xof = Xof
        self.num_proofs = 1
        self.bits = bits
        self.length = length
        self.bits_for_norm = 2 * bits - 2
        self.meas_len = bits * length + self.bits_for_norm
        self.out_len = length
        self.jr_len = 2
        self.qr_len = 2
        self.C0 = optimal_chunk_length(self.meas_len)
        self.K0 = -(-self.meas_len // self.C0)
        self.C1 = optimal_chunk_length(length)
        self.K1 = -(-length // self.C1)
        self.P0 = next_pow2(1 + self.K0)
        self.P1 = next_pow2(1 + self.K1)
        self.A0, self.A1 = 2 * self.C0, self.C1
        self.glen0, self.glen1 = 2 * (self.P0 - 1) + 1, 2 * (self.P1 - 1) + 1
        self.arity = self.A0 + self.A1  # prove-randomness length
        self.proof_len = self.A0 + self.glen0 + self.A1 + self.glen1
        self.verifier_len = 1 + self.A0 + 1 + self.A1 + 1

    # --- circuit ---
    def _q(self, y: int) -> int:
        return (y * y - (y << self.bits)) % self.F.p

    def gadget0(self, x):
        return sum(x[2 * j] * x[2 * j + 1] for j in range(self.C0)) % self.F.p

    def gadget1(self, x):
        return sum(self._q(v) for v in x) % self.F.p

    def valid(self, call0, call1, meas, jr, num_shares):
        F, n = self.F, self.bits
        sinv = F.inv(num_shares)
        rng, rp = 0, jr[0]
        for k in range(self.K0):
            inputs = []
            for j in range(self.C0):
                i = k * self.C0 + j
                m = meas[i] if i < self.meas_len else 0  # padding: [0, -1/num_shares]
                inputs += [rp * m % F.p, (m - sinv) % F.p]
                rp = rp * jr[0] % F.p
            rng = (rng + call0(inputs)) % F.p
        ys = [sum(meas[n * e + b] << b for b in range(n)) % F.p for e in range(self.length)]
        norm = 0
        for k in range(self.K1):
            chunk = ys[k * self.C1:(k + 1) * self.C1]
            norm = (norm + call1(chunk + [0] * (self.C1 - len(chunk)))) % F.p
        norm = (norm + self.length * (1 << (2 * n - 2)) * sinv) % F.p
        base = n * self.length
        claimed = sum(meas[base + b] << b for b in range(self.bits_for_norm)) % F.p
        return (jr[1] * rng + jr[1] * jr[1] % F.p * (norm - claimed)) % F.p

    def encode(self, xs: list[int]) -> list[int]:
        """xs: raw signed fixed-point values X_i (x_i = X_i / 2^(n-1))."""
        n = self.bits
        assert len(xs) == self.length
        half = 1 << (n - 1)
        out = []
        for X in xs:
            assert -half <= X < half
            y = X + half
            out += [(y >> b) & 1 for b in range(n)]
        norm = sum(X * X for X in xs)
        if norm >= 1 << self.bits_for_norm:
            raise ValueError("L2 norm of the vector must be < 1")
        out += [(norm >> b) & 1 for b in range(self.bits_for_norm)]
        return out

    def truncate(self, meas):
        n = self.bits
        return [sum(meas[n * e + b] << b for b in range(n)) % self.F.p for e in range(self.length)]

    def decode_agg(self, agg):
        return list(agg)

    def decode_result(self, agg, num_measurements: int) -> list[float]:
        half = 1 << (self.bits - 1)
        return [((a - num_measurements * half) % self.F.p if a >= num_measurements * half else
                 a - num_measurements * half) / half for a in agg]

    # --- FLP (two gadgets) ---
    def prove(self, meas, prove_rand, jr):
        F = self.F
        w0 = [[prove_rand[w]] for w in range(self.A0)]
        w1 = [[prove_rand[self.A0 + w]] for w in range(self.A1)]

        def call0(x):
            for w in range(self.A0):
                w0[w].append(x[w])
            return self.gadget0(x)

        def call1(x):
            for w in range(self.A1):
                w1[w].append(x[w])
            return self.gadget1(x)

        self.valid(call0, call1, meas, jr, 1)
        out = []
        for wires, P, glen, g in ((w0, self.P0, self.glen0, 0), (w1, self.P1, self.glen1, 1)):
            # wire polynomial evaluations on the 2P-th roots (degree < P)
            ev = []
            for vals in wires:
                coef = _ntt(F, vals + [0] * (P - len(vals)), inverse=True)
                ev.append(_ntt(F, coef + [0] * P))
            if g == 0:
                pv = [sum(ev[2 * j][i] * ev[2 * j + 1][i] for j in range(self.C0)) % F.p
                      for i in range(2 * P)]
            else:
                pv = [sum(self._q(ev[j][i]) for j in range(self.C1)) % F.p for i in range(2 * P)]
            coeffs = _ntt(F, pv, inverse=True)
            assert all(c == 0 for c in coeffs[glen:])
            out += [wires[w][0] for w in range(len(wires))] + coeffs[:glen]
        return out

    def _split_proof(self, proof):
        a = 0
        s0 = proof[a:a + self.A0]; a += self.A0
        c0 = proof[a:a + self.glen0]; a += self.glen0
        s1 = proof[a:a + self.A1]; a += self.A1
        c1 = proof[a:a + self.glen1]
        return s0, c0, s1, c1

    def query(self, meas, proof, qr, jr, num_shares=2):
        F = self.F
        p = F.p
        s0, c0, s1, c1 = self._split_proof(proof)
        t0, t1 = qr[0], qr[1]
        if pow(t0, self.P0, p) == 1 or pow(t1, self.P1, p) == 1:
            raise ValueError("query randomness is a root of unity")

        def at_roots(coeffs, P):  # p(alpha_P^k), k < P
            fold = [0] * P
            for i, c in enumerate(coeffs):
                fold[i % P] = (fold[i % P] + c) % p
            return _ntt(F, fold)

        pr0, pr1 = at_roots(c0, self.P0), at_roots(c1, self.P1)
        w0 = [[s0[w]] for w in range(self.A0)]
        w1 = [[s1[w]] for w in range(self.A1)]
        ct = [1, 1]

        def call0(x):
            for w in range(self.A0):
                w0[w].append(x[w])
            ct[0] += 1
            return pr0[ct[0] - 1]

        def call1(x):
            for w in range(self.A1):
                w1[w].append(x[w])
            ct[1] += 1
            return pr1[ct[1] - 1]

        v = self.valid(call0, call1, meas, jr, num_shares)

        def lagrange_basis(P, t, m):  # L_c(t), c < m, on the P-th roots
            a = F.root(P)
            num = (pow(t, P, p) - 1) * F.inv(P) % p
            out, ac = [], 1
            for _ in range(m):
                out.append(ac * F.inv((t - ac) % p) % p * num % p)
                ac = ac * a % p
            return out

        L0 = lagrange_basis(self.P0, t0, self.K0 + 1)
        L1 = lagrange_basis(self.P1, t1, self.K1 + 1)
        f0 = [sum(a * b for a, b in zip(L0, w)) % p for w in w0]
        f1 = [sum(a * b for a, b in zip(L1, w)) % p for w in w1]

        def horner(c, t):
            acc = 0
            for x in reversed(c):
                acc = (acc * t + x) % p
            return acc

        return [v] + f0 + [horner(c0, t0)] + f1 + [horner(c1, t1)]

    def decide(self, verifier) -> bool:
        if verifier[0] != 0:
            return False
        f0 = verifier[1:1 + self.A0]
        p0 = verifier[1 + self.A0]
        f1 = verifier[2 + self.A0:2 + self.A0 + self.A1]
        p1 = verifier[2 + self.A0 + self.A1]
        return self.gadget0(f0) == p0 and self.gadget1(f1) == p1


def gen_gsh(length: int, bits: int) -> int:
    """The generator's entry shift: entries are signed bytes >> gsh, so |X| <= 2^(7 - gsh); the
    smallest gsh with length * 2^(14 - 2 gsh) < 2^(2 bits - 2) keeps the squared norm in range."""
    s = 0
    while s < 7 and length * 2 ** (14 - 2 * s) >= 2 ** (2 * bits - 2):
        s += 1
    return s


def gen_report(vk: bytes, length: int, bits: int, seed: int, idx: int) -> dict:
    """Report idx of the synthetic client's seeded stream, as the device generator derives it
    (janus_amd/csrc/prio3_client.hip k_fg_*): stream = TurboSHAKE128("janus-amd-gen" || seed ||
    idx, D = 1) gives the nonce (16 bytes), the five shard seeds (80 bytes: helper measurement,
    helper proofs, helper blind, leader blind, prove randomness) and one signed byte per entry
    (>> gen_gsh) from offset 96; then Prio3 shard and the leader's prepare_init (agg_id 0).
    Pure Python: seconds per report at length 100, about a minute at 10000."""
    from oracle.prio3_py import Prio3, turboshake128
    typ = FpVecType(length, bits)
    P = Prio3(typ)
    msg = b"janus-amd-gen" + seed.to_bytes(8, "little") + idx.to_bytes(8, "little")
    stream = turboshake128(msg, 1, 96 + length)
    nonce, rand = stream[:16], stream[16:96]
    sh = gen_gsh(length, bits)
    X = [((b - 256) if b >= 128 else b) >> sh for b in stream[96:96 + length]]
    public, leader, helper = P.shard(X, nonce, rand)
    _, lps, trace = P.prepare_init(vk, 0, nonce, public, leader)
    out = typ.truncate(trace["meas"])
    return dict(nonce=nonce, public=public, helper=helper, leader=leader, lps=lps, X=X,
                leader_out=b"".join(P.F.enc(x) for x in out))
