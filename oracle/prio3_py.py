"""Independent pure-Python restatement of Prio3 (VDAF draft-08, as implemented by
prio 0.16.2) -- TEST INFRASTRUCTURE ONLY (small cases; cross-checks oracle/prio3_oracle.c
and generates tests/golden/ fixtures).

It is written independently of the C restatement and deliberately uses different
algorithms where the result is algorithm-independent:
  * wire polynomials are evaluated with the barycentric Lagrange formula instead of
    prio's inverse DFT + Horner (prio flp.rs FlpGeneric::query);
  * the gadget polynomial's values at the roots of unity are evaluated point-by-point
    (Horner) instead of a size-2P DFT;
  * the prover multiplies polynomials in coefficient form.
Agreement between the two restatements therefore checks the algebra, not a shared
implementation.  Byte parity with the prio crate itself is UNPINNED (the crate is not
available in this container; see DESIGN.md "Oracle").

Reference call sites this mirrors: aggregator/src/aggregator.rs:2022-2031
(helper_initialized + evaluate), aggregator/src/aggregator/aggregation_job_writer.rs:591-695
(accumulate), core/src/vdaf.rs:198-300 (instances).
"""
from __future__ import annotations

from dataclasses import dataclass, field as dc_field

# ------------------------------------------------------------------------------------
# Keccak-p[1600, n_r] / TurboSHAKE128 (RFC 9861)
# ------------------------------------------------------------------------------------
_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_M64 = (1 << 64) - 1


def _rotations():
    # rho offsets generated from the spec recurrence (not a table): (x,y) walk
    rot = [[0] * 5 for _ in range(5)]
    x, y = 1, 0
    for t in range(24):
        rot[x][y] = ((t + 1) * (t + 2) // 2) % 64
        x, y = y, (2 * x + 3 * y) % 5
    return rot


_ROT = _rotations()


def keccak_p(lanes: list[list[int]], rounds: int) -> None:
    """In-place Keccak-p[1600, rounds] on lanes[x][y] (uses the LAST `rounds` constants)."""
    A = lanes
    for rc in _RC[24 - rounds:]:
        C = [A[x][0] ^ A[x][1] ^ A[x][2] ^ A[x][3] ^ A[x][4] for x in range(5)]
        D = [C[(x - 1) % 5] ^ (((C[(x + 1) % 5] << 1) | (C[(x + 1) % 5] >> 63)) & _M64)
             for x in range(5)]
        B = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                v = A[x][y] ^ D[x]
                r = _ROT[x][y]
                B[y][(2 * x + 3 * y) % 5] = ((v << r) | (v >> (64 - r))) & _M64 if r else v
        for x in range(5):
            for y in range(5):
                A[x][y] = B[x][y] ^ ((~B[(x + 1) % 5][y]) & B[(x + 2) % 5][y])
        A[0][0] ^= rc


class Sponge:
    RATE = 168

    def __init__(self, rounds: int = 12):
        self.rounds = rounds
        self.buf = bytearray()
        self.out = bytearray()
        self.lanes = [[0] * 5 for _ in range(5)]
        self.done = False

    def _xor_block(self, block: bytes):
        for i in range(self.RATE // 8):
            x, y = i % 5, i // 5
            self.lanes[x][y] ^= int.from_bytes(block[8 * i:8 * i + 8], "little")
        keccak_p(self.lanes, self.rounds)

    def update(self, data: bytes):
        assert not self.done
        self.buf += data
        while len(self.buf) >= self.RATE:
            self._xor_block(bytes(self.buf[:self.RATE]))
            del self.buf[:self.RATE]

    def finalize(self, domain: int):
        block = bytearray(self.buf) + bytes(self.RATE - len(self.buf))
        block[len(self.buf)] ^= domain
        block[self.RATE - 1] ^= 0x80
        self._xor_block(bytes(block))
        self.buf = bytearray()
        self.done = True

    def _state_bytes(self) -> bytes:
        return b"".join(self.lanes[i % 5][i // 5].to_bytes(8, "little")
                        for i in range(self.RATE // 8))

    def read(self, n: int) -> bytes:
        assert self.done
        while len(self.out) < n:
            if not hasattr(self, "_started"):
                self._started = True
            else:
                keccak_p(self.lanes, self.rounds)
            self.out += self._state_bytes()
        r = bytes(self.out[:n])
        del self.out[:n]
        return r


def turboshake128(msg: bytes, domain: int, n: int) -> bytes:
    s = Sponge(12)
    s.update(msg)
    s.finalize(domain)
    return s.read(n)


def shake128_24(msg: bytes, n: int) -> bytes:
    s = Sponge(24)
    s.update(msg)
    s.finalize(0x1F)
    return s.read(n)


# ------------------------------------------------------------------------------------
# Fields
# ------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Field:
    p: int
    es: int
    gen: int
    gen_order_log2: int

    def root(self, n: int) -> int:
        assert n & (n - 1) == 0
        return pow(self.gen, (1 << self.gen_order_log2) // n, self.p)

    def inv(self, a: int) -> int:
        return pow(a, self.p - 2, self.p)

    def enc(self, x: int) -> bytes:
        return x.to_bytes(self.es, "little")

    def dec(self, b: bytes) -> int:
        v = int.from_bytes(b, "little")
        if v >= self.p:
            raise ValueError("field element out of range")
        return v


Field64 = Field(2**64 - 2**32 + 1, 8, 1753635133440165772, 32)
Field128 = Field(2**128 - 28 * 2**64 + 1, 16, 145091266659756586618791329697897684742, 66)


# ------------------------------------------------------------------------------------
# XofTurboShake128
# ------------------------------------------------------------------------------------
class Xof:
    def __init__(self, seed: bytes, dst: bytes, binder: bytes):
        assert len(seed) == 16
        self.s = Sponge(12)
        self.s.update(bytes([len(dst)]) + dst + seed + binder)
        self.s.finalize(1)

    def next(self, n: int) -> bytes:
        return self.s.read(n)

    def next_vec(self, F: Field, n: int) -> list[int]:
        out = []
        while len(out) < n:
            v = int.from_bytes(self.next(F.es), "little")
            if v < F.p:
                out.append(v)
        return out


class XofHmacSha256Aes128:
    """prio 0.16 XofHmacSha256Aes128 (SEED_SIZE 32), restated: HMAC-SHA256 keyed by the seed
    over len(dst) || dst || binder; the 32-byte tag is split into an AES-128 key and IV for a
    CTR keystream with a 64-bit big-endian counter (`Ctr64BE<Aes128>`, SeedStreamAes128).  The
    janus custom VDAF using it: core/src/vdaf.rs:173-195.  Parity with prio UNPINNED."""

    def __init__(self, seed: bytes, dst: bytes, binder: bytes):
        import hashlib
        import hmac
        assert len(seed) == 32
        tag = hmac.new(seed, bytes([len(dst)]) + dst + binder, hashlib.sha256).digest()
        self.key, self.iv, self.pos, self.buf = tag[:16], tag[16:], 0, b""

    def next(self, n: int) -> bytes:
        from oracle.hpke import aes128_ctr64_keystream
        need = self.pos + n
        if len(self.buf) < need:
            self.buf = aes128_ctr64_keystream(self.key, self.iv, -(-max(need, 2 * len(self.buf), 64) // 16) * 16)
        out = self.buf[self.pos:need]
        self.pos = need
        return out

    next_vec = Xof.next_vec


def derive_seed(seed: bytes, dst: bytes, binder: bytes, xof=Xof) -> bytes:
    return xof(seed, dst, binder).next(len(seed))


def expand_into_vec(F: Field, seed: bytes, dst: bytes, binder: bytes, n: int,
                    xof=Xof) -> list[int]:
    return xof(seed, dst, binder).next_vec(F, n)


# ------------------------------------------------------------------------------------
# Polynomial helpers (coefficient lists, ascending)
# ------------------------------------------------------------------------------------
def poly_eval(F: Field, c: list[int], x: int) -> int:
    r = 0
    for a in reversed(c):
        r = (r * x + a) % F.p
    return r


def poly_mul(F: Field, a: list[int], b: list[int]) -> list[int]:
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                out[i + j] = (out[i + j] + x * y) % F.p
    return out


def poly_add(F: Field, a: list[int], b: list[int]) -> list[int]:
    n = max(len(a), len(b))
    return [((a[i] if i < len(a) else 0) + (b[i] if i < len(b) else 0)) % F.p for i in range(n)]


def interp_roots(F: Field, vals: list[int], P: int) -> list[int]:
    """Coefficients of the degree<P polynomial through (alpha^i, vals[i]) (vals zero-padded)."""
    a = F.root(P)
    ainv = F.inv(a)
    pinv = F.inv(P)
    v = vals + [0] * (P - len(vals))
    return [pinv * sum(v[i] * pow(ainv, i * e, F.p) for i in range(P)) % F.p for e in range(P)]


def lagrange_at(F: Field, vals: list[int], P: int, t: int) -> int:
    """Barycentric evaluation at t of the interpolant through (alpha^i, vals[i])."""
    a = F.root(P)
    num = (pow(t, P, F.p) - 1) * F.inv(P) % F.p
    acc = 0
    for i, w in enumerate(vals):
        if w:
            ai = pow(a, i, F.p)
            acc += w * ai % F.p * F.inv((t - ai) % F.p)
    return acc * num % F.p


# ------------------------------------------------------------------------------------
# Gadgets and validity circuits [VDAF-08 §7.3-7.4]
# ------------------------------------------------------------------------------------
def next_pow2(n: int) -> int:
    p = 1
    while p < n:
        p <<= 1
    return p


@dataclass
class Prio3Type:
    kind: str  # "count" | "sum" | "sumvec" | "histogram" | "sumvec_f64_mp"
    bits: int = 0
    length: int = 0
    chunk_length: int = 0
    num_proofs: int = 1
    F: Field = dc_field(init=False)
    algo_id: int = dc_field(init=False)
    seed_size: int = dc_field(init=False)
    xof: object = dc_field(init=False)

    def __post_init__(self):
        # sumvec_f64_mp: Prio3SumVecField64MultiproofHmacSha256Aes128 (core/src/vdaf.rs:173-195:
        # SumVec<Field64, ParallelSum<Mul>>, XofHmacSha256Aes128, SEED_SIZE 32, algorithm id
        # 0xFFFF1003 (vdaf.rs:20), num_proofs >= 2)
        self.algo_id = {"count": 0, "sum": 1, "sumvec": 2, "histogram": 3,
                        "sumvec_f64_mp": 0xFFFF1003}[self.kind]
        self.F = Field64 if self.kind in ("count", "sumvec_f64_mp") else Field128
        self.seed_size = 32 if self.kind == "sumvec_f64_mp" else 16
        self.xof = XofHmacSha256Aes128 if self.kind == "sumvec_f64_mp" else Xof
        if self.kind == "sumvec_f64_mp":
            if self.num_proofs < 2:
                raise ValueError("Must use at least two proofs with Field64")
            self.kind = "sumvec"  # the circuit is SumVec's

    # --- shapes ---
    @property
    def meas_len(self):
        return {"count": 1, "sum": self.bits, "sumvec": self.bits * self.length,
                "histogram": self.length}[self.kind]

    @property
    def out_len(self):
        return {"count": 1, "sum": 1, "sumvec": self.length, "histogram": self.length}[self.kind]

    @property
    def jr_len(self):
        return {"count": 0, "sum": 1, "sumvec": 1, "histogram": 2}[self.kind]

    @property
    def arity(self):
        return {"count": 2, "sum": 1}.get(self.kind, 2 * self.chunk_length)

    @property
    def calls(self):
        if self.kind == "count":
            return 1
        if self.kind == "sum":
            return self.bits
        return -(-self.meas_len // self.chunk_length)

    @property
    def P(self):
        return next_pow2(1 + self.calls)

    @property
    def proof_len(self):
        return self.arity + 2 * (self.P - 1) + 1

    @property
    def verifier_len(self):
        return self.arity + 2

    def gadget(self, x: list[int]) -> int:
        F = self.F
        if self.kind == "count":
            return x[0] * x[1] % F.p
        if self.kind == "sum":
            return (x[0] * x[0] - x[0]) % F.p
        return sum(x[2 * j] * x[2 * j + 1] for j in range(self.chunk_length)) % F.p

    def gadget_poly(self, f: list[list[int]]) -> list[int]:
        F = self.F
        if self.kind == "count":
            return poly_mul(F, f[0], f[1])
        if self.kind == "sum":
            sq = poly_mul(F, f[0], f[0])
            return poly_add(F, sq, [(-c) % F.p for c in f[0]])
        acc = [0]
        for j in range(self.chunk_length):
            acc = poly_add(F, acc, poly_mul(F, f[2 * j], f[2 * j + 1]))
        return acc

    def valid(self, call, meas: list[int], jr: list[int], num_shares: int) -> int:
        F = self.F
        sinv = F.inv(num_shares)
        if self.kind == "count":
            return (call([meas[0], meas[0]]) - meas[0]) % F.p
        if self.kind == "sum":
            out, r = 0, jr[0]
            for b in meas:
                out = (out + r * call([b])) % F.p
                r = r * jr[0] % F.p
            return out

        def range_check(r):
            out, rp = 0, r
            for k in range(self.calls):
                inputs = []
                for j in range(self.chunk_length):
                    i = k * self.chunk_length + j
                    m = meas[i] if i < len(meas) else 0
                    inputs += [rp * m % F.p, (m - sinv) % F.p]
                    rp = rp * r % F.p
                out = (out + call(inputs)) % F.p
            return out

        if self.kind == "sumvec":
            return range_check(jr[0])
        rc = range_check(jr[0])
        sc = (sum(meas) - sinv) % F.p
        return (jr[1] * rc + jr[1] * jr[1] % F.p * sc) % F.p

    def encode(self, m) -> list[int]:
        if self.kind == "count":
            assert m in (0, 1)
            return [m]
        if self.kind == "sum":
            assert 0 <= m < 2**self.bits
            return [(m >> i) & 1 for i in range(self.bits)]
        if self.kind == "sumvec":
            assert len(m) == self.length
            return [(v >> b) & 1 for v in m for b in range(self.bits)]
        assert 0 <= m < self.length
        return [int(i == m) for i in range(self.length)]

    def truncate(self, meas: list[int]) -> list[int]:
        F = self.F
        if self.kind in ("count", "histogram"):
            return list(meas)
        if self.kind == "sum":
            return [sum(b << i for i, b in enumerate(meas)) % F.p]
        return [sum(meas[e * self.bits + b] << b for b in range(self.bits)) % F.p
                for e in range(self.length)]

    def decode_agg(self, agg: list[int]):
        if self.kind in ("count", "sum"):
            return agg[0]
        return list(agg)

    # --- FLP ---
    def prove(self, meas, prove_rand, jr) -> list[int]:
        F = self.F
        P = self.P
        wires = [[prove_rand[w]] for w in range(self.arity)]

        def call(x):
            for w in range(self.arity):
                wires[w].append(x[w])
            return self.gadget(x)

        self.valid(call, meas, jr, 1)
        f = [interp_roots(F, wires[w], P) for w in range(self.arity)]
        g = self.gadget_poly(f)
        glen = 2 * (P - 1) + 1
        g = g + [0] * (glen - len(g))
        assert all(c == 0 for c in g[glen:])
        return list(prove_rand[:self.arity]) + g[:glen]

    def query(self, meas, proof, qr, jr, num_shares=2) -> list[int]:
        F = self.F
        P = self.P
        t = qr[0]
        if pow(t, P, F.p) == 1:
            raise ValueError("query randomness is a root of unity")
        coeffs = proof[self.arity:]
        a = F.root(P)
        wires = [[proof[w]] for w in range(self.arity)]
        ct = [1]

        def call(x):
            for w in range(self.arity):
                wires[w].append(x[w])
            y = poly_eval(F, coeffs, pow(a, ct[0], F.p))
            ct[0] += 1
            return y

        v = self.valid(call, meas, jr, num_shares)
        return [v] + [lagrange_at(F, wires[w], P, t) for w in range(self.arity)] + \
            [poly_eval(F, coeffs, t)]

    def decide(self, verifier) -> bool:
        if verifier[0] != 0:
            return False
        return self.gadget(verifier[1:1 + self.arity]) == verifier[1 + self.arity]


# ------------------------------------------------------------------------------------
# Prio3 [VDAF-08 §7.2]
# ------------------------------------------------------------------------------------
USAGE = dict(meas=1, proof=2, jr=3, prove=4, query=5, jr_seed=6, jr_part=7)


class Prio3:
    def __init__(self, typ: Prio3Type):
        self.t = typ
        self.F = typ.F

    def dst(self, usage: str) -> bytes:
        return bytes([8, 0]) + self.t.algo_id.to_bytes(4, "big") + USAGE[usage].to_bytes(2, "big")

    @property
    def np(self):
        return self.t.num_proofs

    @property
    def S(self):
        return self.t.seed_size

    def helper_meas(self, agg_id, k):
        return expand_into_vec(self.F, k, self.dst("meas"), bytes([agg_id]), self.t.meas_len,
                               self.t.xof)

    def helper_proofs(self, agg_id, k):
        return expand_into_vec(self.F, k, self.dst("proof"), bytes([self.np, agg_id]),
                               self.t.proof_len * self.np, self.t.xof)

    def jr_part(self, agg_id, blind, meas, nonce):
        return derive_seed(blind, self.dst("jr_part"),
                           bytes([agg_id]) + nonce + b"".join(self.F.enc(x) for x in meas),
                           self.t.xof)

    def jr_seed(self, parts):
        return derive_seed(bytes(self.S), self.dst("jr_seed"), b"".join(parts), self.t.xof)

    def joint_rands(self, seed):
        return expand_into_vec(self.F, seed, self.dst("jr"), bytes([self.np]),
                               self.t.jr_len * self.np, self.t.xof)

    def query_rands(self, vk, nonce):
        return expand_into_vec(self.F, vk, self.dst("query"), bytes([self.np]) + nonce,
                               getattr(self.t, "qr_len", 1) * self.np, self.t.xof)

    def shard(self, measurement, nonce: bytes, rand: bytes):
        t, F = self.t, self.F
        S = self.S
        seeds = [rand[i:i + S] for i in range(0, len(rand), S)]
        meas = t.encode(measurement)
        k_hm, k_hp = seeds[0], seeds[1]
        if t.jr_len:
            k_hb, k_lb, k_prove = seeds[2], seeds[3], seeds[4]
        else:
            k_prove = seeds[2]
        hm = self.helper_meas(1, k_hm)
        lm = [(a - b) % F.p for a, b in zip(meas, hm)]
        jr = []
        public = b""
        if t.jr_len:
            parts = [self.jr_part(0, k_lb, lm, nonce), self.jr_part(1, k_hb, hm, nonce)]
            public = parts[0] + parts[1]
            jr = self.joint_rands(self.jr_seed(parts))
        prove_rands = expand_into_vec(F, k_prove, self.dst("prove"), bytes([self.np]),
                                      t.arity * self.np, t.xof)
        proofs = []
        for k in range(self.np):
            proofs += t.prove(meas, prove_rands[k * t.arity:(k + 1) * t.arity],
                              jr[k * t.jr_len:(k + 1) * t.jr_len])
        hp = self.helper_proofs(1, k_hp)
        lp = [(a - b) % F.p for a, b in zip(proofs, hp)]
        leader = b"".join(F.enc(x) for x in lm + lp) + (k_lb if t.jr_len else b"")
        helper = k_hm + k_hp + (k_hb if t.jr_len else b"")
        return public, leader, helper

    def prepare_init(self, vk, agg_id, nonce, public, share):
        """Returns (state, prep_share_bytes, trace) with state = (meas, corrected_seed)."""
        t, F = self.t, self.F
        if agg_id == 0:
            es = F.es
            vals = [F.dec(share[i * es:(i + 1) * es])
                    for i in range(t.meas_len + t.proof_len * self.np)]
            meas, proofs = vals[:t.meas_len], vals[t.meas_len:]
            blind = share[(t.meas_len + t.proof_len * self.np) * es:]
        else:
            S = self.S
            meas = self.helper_meas(agg_id, share[:S])
            proofs = self.helper_proofs(agg_id, share[S:2 * S])
            blind = share[2 * S:3 * S]
        jr, part, corrected = [], b"", b""
        if t.jr_len:
            part = self.jr_part(agg_id, blind, meas, nonce)
            parts = [public[0:self.S], public[self.S:2 * self.S]]
            parts[agg_id] = part
            corrected = self.jr_seed(parts)
            jr = self.joint_rands(corrected)
        qr = self.query_rands(vk, nonce)
        ql = getattr(t, "qr_len", 1)
        verifiers = []
        for k in range(self.np):
            verifiers += t.query(meas, proofs[k * t.proof_len:(k + 1) * t.proof_len],
                                 qr[k * ql:(k + 1) * ql], jr[k * t.jr_len:(k + 1) * t.jr_len])
        ps = b"".join(F.enc(x) for x in verifiers) + part
        trace = dict(meas=meas, proofs=proofs, part=part, corrected=corrected, jr=jr, qr=qr,
                     verifiers=verifiers)
        return (meas, corrected), ps, trace

    def prep_shares_to_prep_msg(self, leader_ps: bytes, helper_ps: bytes) -> bytes:
        t, F = self.t, self.F
        nv = t.verifier_len * self.np
        es = F.es
        lv = [F.dec(leader_ps[i * es:(i + 1) * es]) for i in range(nv)]
        hv = [F.dec(helper_ps[i * es:(i + 1) * es]) for i in range(nv)]
        v = [(a + b) % F.p for a, b in zip(lv, hv)]
        for k in range(self.np):
            if not t.decide(v[k * t.verifier_len:(k + 1) * t.verifier_len]):
                raise ValueError("decide failed")
        if t.jr_len:
            S = self.S
            return self.jr_seed([leader_ps[nv * es:nv * es + S], helper_ps[nv * es:nv * es + S]])
        return b""

    def prepare_next(self, state, msg: bytes) -> list[int]:
        meas, corrected = state
        if self.t.jr_len and corrected != msg:
            raise ValueError("joint randomness mismatch")
        return self.t.truncate(meas)

    def aggregate(self, out_shares) -> list[int]:
        acc = [0] * self.t.out_len
        for s in out_shares:
            acc = [(a + b) % self.F.p for a, b in zip(acc, s)]
        return acc

    def unshard(self, agg_shares) -> object:
        return self.t.decode_agg(self.aggregate(agg_shares))


def gen_report_mp64(vk: bytes, bits: int, length: int, chunk: int, proofs: int, seed: int,
                    idx: int) -> dict:
    """Report idx of the synthetic client's seeded stream for the Field64 multiproof VDAF, as the
    device generator derives it (janus_amd/csrc/prio3_client.hip k_gen_mp64): stream =
    TurboSHAKE128("janus-amd-gen" || seed || idx, D = 1) gives the nonce (16 bytes), the five
    32-byte shard seeds (helper measurement, helper proofs, helper blind, leader blind, prove
    randomness) and one 8-byte little-endian entry per element from byte 176, masked to `bits`;
    then shard and the leader's prepare_init (agg_id 0).  TEST INFRASTRUCTURE ONLY."""
    typ = Prio3Type("sumvec_f64_mp", bits=bits, length=length, chunk_length=chunk,
                    num_proofs=proofs)
    P = Prio3(typ)
    msg = b"janus-amd-gen" + seed.to_bytes(8, "little") + idx.to_bytes(8, "little")
    stream = turboshake128(msg, 1, 176 + 8 * length)
    nonce, rand = stream[:16], stream[16:176]
    m = [int.from_bytes(stream[176 + 8 * e:184 + 8 * e], "little") & ((1 << bits) - 1)
         for e in range(length)]
    public, leader, helper = P.shard(m, nonce, rand)
    _, lps, trace = P.prepare_init(vk, 0, nonce, public, leader)
    out = typ.truncate(trace["meas"])
    return dict(nonce=nonce, public=public, helper=helper, leader=leader, lps=lps, m=m,
                leader_out=b"".join(P.F.enc(x) for x in out))
