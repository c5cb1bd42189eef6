# Word-level model of the planned asm mul128 / red288 (checks every carry bound).
import random
P = 2**128 - 28*2**64 + 1
M32, M64 = 2**32-1, 2**64-1
def mad(a, b, c):  # v_mad_u64_u32: returns (64-bit result, carry)
    assert 0 <= a <= M32 and 0 <= b <= M32 and 0 <= c <= M64
    s = a*b + c
    return s & M64, s >> 64
def product_cols(a, b):
    v = [0]*10
    aw = [(a >> (32*i)) & M32 for i in range(4)]
    bw = [(b >> (32*i)) & M32 for i in range(4)]
    def pair(k): return v[k] | (v[k+1] << 32)
    def setpair(k, x): v[k] = x & M32; v[k+1] = x >> 32
    cols = [[(0,0)], [(0,1),(1,0)], [(0,2),(1,1),(2,0)], [(0,3),(1,2),(2,1),(3,0)], [(1,3),(2,2),(3,1)], [(2,3),(3,2)], [(3,3)]]
    for k, prods in enumerate(cols):
        for n, (i, j) in enumerate(prods):
            r, c = mad(aw[i], bw[j], pair(k))
            setpair(k, r)
            if k == 0 or (k == 1 and n == 0):
                assert c == 0
            else:
                v[k+2] = (v[k+2] + c)  # v_addc_co_u32 v[k+2], vcc, 0, v[k+2], vcc
                assert v[k+2] <= M32
    return v[:9]
def red288(w):
    t = w[8]
    X = sum(w[i] << (32*i) for i in range(8)) + (t << 256)
    x1 = w[2] | (w[3] << 32); x2 = w[4] | (w[5] << 32)
    # S = x1 + 28 x2 + 783 x3 + 21896 t
    Y, c1 = mad(w[4], 28, x1)
    Y, c2 = mad(w[6], 783, Y)
    Y, c3 = mad(t, 21896, Y)
    Z, cz = mad(w[5], 28, 0); assert cz == 0
    Z, cz = mad(w[7], 783, Z); assert cz == 0 and Z < 2**43
    yh = (Y >> 32) + (Z & M32); c4 = yh >> 32; Y = (Y & M32) | ((yh & M32) << 32)
    S2 = (Z >> 32) + c1 + c2 + c3 + c4
    assert S2 < 2**11
    S = Y + (S2 << 64)
    assert S == x1 + 28*x2 + 783*(w[6] | (w[7] << 32)) + 21896*t
    # N = x2 + 28 x3 + 783 t + s1
    Nn, n1 = mad(w[6], 28, x2)
    Nn, n2 = mad(t, 783, Nn)
    Nn, n3 = mad(S2, 1, Nn)
    Zn, cz = mad(w[7], 28, 0); assert cz == 0
    nh = (Nn >> 32) + (Zn & M32); n4 = nh >> 32; Nn = (Nn & M32) | ((nh & M32) << 32)
    N2 = (Zn >> 32) + n1 + n2 + n3 + n4
    assert N2 < 2**7
    N = Nn + (N2 << 64)
    # U = s_lo + 28 s1
    U, c = mad(S2, 28, Y)
    # A = x0 + U 2^64 + c (28 2^64 - 1)
    x0 = w[0] | (w[1] << 32)
    A = x0 + (U << 64)
    assert A < 2**128
    if c:
        A += 28*2**64 - 1
        if A >= 2**128:
            A -= 2**128; A += 28*2**64 - 1; assert A < 2**128
    # A - N (+p on borrow)
    A -= N
    if A < 0:
        A += P; assert A >= 0
    if A >= P:
        A -= P
    assert A == X % P, (A, X % P)
    return A
random.seed(1)
edge = [0, 1, P-1, P-2, 2**128-1, 2**127, 28*2**64, 2**64-1, 2**96]
for _ in range(200000):
    a = random.choice(edge) if random.random() < 0.1 else random.randrange(2**128)
    b = random.choice(edge) if random.random() < 0.1 else random.randrange(2**128)
    w = product_cols(a, b)
    assert sum(w[i] << (32*i) for i in range(9)) == a*b
    assert red288(w) == (a*b) % P
# MAC-sum inputs (t up to 2^31)
for _ in range(100000):
    X = random.randrange(2**287) if random.random() < .5 else random.randrange(2**262)
    w = [(X >> (32*i)) & M32 for i in range(9)]
    red288(w)
for X in [2**287-1, 2**256-1, 0, P, 2**256, (2**256-1)*17]:
    w = [(X >> (32*i)) & M32 for i in range(9)]; red288(w)
print("model ok")
