"""Integer models of the device's 29-bit-limb arithmetic (fr29.hpp) at the
operand bounds the kernels rely on: the FIPS product with full-word quotient
digits (every 64-bit column sum must stay below 2^64, the asm drops the MAD
carry-out), the top-limb reduction f29_reduce and the LDS-table reduction
f29_reduce_qt (biased 32-bit limb sums).  CPU only; the kernels themselves
are checked bit for bit by the GPU parity suites, which random data cannot
drive to these extremes.

Bounds exercised:
  * radix-4 DIF group (k_ntt.hip dif4): (u0 + 32r - u1) * w with u0 carry-free
    (limbs < 2^30) -- column sums < 2^63.74;
  * f29_reduce / f29_reduce_qt on limb-wise sums with limbs up to 3 * 2^30 - 8
    and values < 64 r (the NTT's sub16 of a sub16 reaches 2.42 * 2^30; the
    Poseidon2 partial rounds' lazy s1 2^31)."""
import random

import pytest

P29 = [0x1, 0x108C0000, 0x42, 0x14EDFDA0, 0x1B00159A, 0x68F2E1B, 0x155982D1, 0xBD34594, 0x12AB65]
R = sum(p << (29 * i) for i, p in enumerate(P29))
MASK = (1 << 29) - 1
M32, M64 = (1 << 32) - 1, (1 << 64) - 1
C29 = [0x1FFFFE49, 0x1077FFFF, 0x1FFF8E31, 0x10D0103F, 0xDDB0965, 0x7071C5C, 0x18DA2E10, 0x486F3A3, 0xEC090, 0]
L32 = [0x20000020, 0x317FFFFF, 0x2000084F, 0x3DBFB3FF, 0x2002B353, 0x31E5C37A, 0x2B305A25, 0x3A68B294, 0x2556CAA]
L16 = [0x20000010, 0x28BFFFFF, 0x20000427, 0x2EDFD9FF, 0x300159A9, 0x28F2E1BC, 0x35982D12, 0x3D345949, 0x12AB654]


def val(l):
    return sum(x << (29 * i) for i, x in enumerate(l))


def limbs(v):
    return [(v >> (29 * i)) & MASK for i in range(8)] + [v >> 232]


def f29_mul(a, b):
    """f29_mul_c (fr29.hpp:81) with every 64-bit column sum checked; returns
    (output limbs, worst column sum)."""
    m = [0] * 9
    o = [0] * 9
    acc, worst = C29[0], 0
    for k in range(9):
        for j in range(k):
            acc += a[j] * b[k - j] + m[j] * P29[k - j]
        acc += a[k] * b[0]
        worst = max(worst, acc)
        assert acc <= M64, f"column {k} overflows"
        m[k] = ~acc & M32
        acc = (acc >> 32) * 8 + 7 + C29[k + 1]
    for k in range(9, 17):
        for j in range(k - 8, 9):
            acc += a[j] * b[k - j] + m[j] * P29[k - j]
        worst = max(worst, acc)
        assert acc <= M64, f"column {k} overflows"
        o[k - 9] = acc & MASK
        acc >>= 29
    o[8] = acc & M32
    return o, worst


def f29_reduce(a):
    """fr29.hpp:170, signed carries"""
    q = ((a[8] * 0xDB651D12) >> 52) & M32
    o, c = [0] * 9, 0
    for i in range(8):
        s = a[i] - q * P29[i] + c
        o[i] = s & MASK
        c = s >> 29  # arithmetic
    o[8] = (a[8] - q * P29[8] + c) & M32
    return o


def qtab(q):
    Q = limbs(q * R)
    return [((1 << 30) - Q[0]) & M32] + [((1 << 30) - 2 - Q[i]) & M32 for i in range(1, 8)] + [(-2 - Q[8]) & M32]


def f29_reduce_qt(a):
    """fr29.hpp:221: 32-bit biased limb sums, carries by logical shifts"""
    q = (((a[8] * 0xDB651D12) >> 32) & M32) >> 20
    assert q < 64
    T = qtab(q)
    o, k = [0] * 9, 0
    for i in range(8):
        s = a[i] + T[i] + k
        assert s <= M32, f"limb {i} sum leaves 32 bits"
        o[i] = s & MASK
        k = s >> 29
    o[8] = (a[8] + T[8] + k) & M32
    return o


def check_reduced(o, v):
    assert all(x <= MASK for x in o[:8])
    assert val(o) % R == v % R and val(o) < 2 * R


def test_product_columns_dif4_lazy_u0():
    # a = u0 + 32r - u1 with u0 carry-free (limbs < 2^30), u1 normalised; b a
    # canonical twiddle: the worst limbs everywhere (the value bound caps a[8])
    a = [(1 << 30) - 2 + L32[i] for i in range(8)] + [(49 * R) >> 232]
    b = [MASK] * 8 + [R >> 232]
    o, worst = f29_mul(a, b)
    assert worst < 1 << 64 and worst.bit_length() == 64  # 2^63.74: the margin is real but thin
    assert all(x <= MASK for x in o[:8])
    rng = random.Random(5)
    for _ in range(300):
        u0 = [rng.randrange(1 << 30) for _ in range(8)] + [rng.randrange((16 * R) >> 232)]
        u1v = rng.randrange(16 * R)
        u1 = limbs(u1v)
        aa = [u0[i] + L32[i] - u1[i] for i in range(9)]
        assert all(0 <= x < 1 << 31 for x in aa[:8])
        w = rng.randrange(R)
        o, worst = f29_mul(aa, limbs(w))
        assert worst < 1 << 64
        assert val(o) % R == val(aa) * w * pow(2, -261, R) % R


@pytest.mark.parametrize("red", [f29_reduce, f29_reduce_qt])
def test_reductions_on_lazy_limbs(red):
    rng = random.Random(11)
    for top in (1 << 30, 1 << 31, int(2.42 * (1 << 30)), 3 * (1 << 30) - 8):
        for _ in range(200):
            v = rng.randrange(63 * R)
            lo = limbs(v)
            # move value from higher limbs into lower ones (carry-free form), limbs < top
            a = lo[:]
            for i in range(8, 0, -1):
                while a[i] > 0 and a[i - 1] + (1 << 29) < top and rng.random() < 0.9:
                    a[i] -= 1
                    a[i - 1] += 1 << 29
            assert val(a) == v and max(a[:8]) < top
            check_reduced(red(a), v)
        # extreme: every low limb at the cap, the top limb as large as the value bound allows
        a = [top - 1] * 8
        a.append(max(0, (63 * R - val(a + [0])) >> 232))
        check_reduced(red(a), val(a))


def test_sub16_of_sub16_limbs():
    # dit4's v3 = reduce(sub16(u1, q3)) with u1 = sub16(v0, p1): limbs < 2.42 2^30
    a = [MASK + L16[i] for i in range(8)]
    b = [x + L16[i] for i, x in enumerate(a)]
    assert max(b) < int(2.42 * (1 << 30)) < 3 * (1 << 30) - 8


@pytest.mark.parametrize("red", [f29_reduce, f29_reduce_qt])
def test_trivial_end_groups(red):
    """the radix-4 groups at the trivial end of a transform skip the w_4^0
    product (k_ntt.hip dif4 / dit4 with triv): dif4 reduces sub16(v0, v2) +- u3
    unreduced, dit4 reduces u0 + 32r - norm(v2 + v3); worst limbs, values at
    the bounds the comments state"""
    rng = random.Random(17)
    for _ in range(300):
        v0, v2 = rng.randrange(int(8.3 * R)), rng.randrange(int(8.3 * R))
        u3 = rng.randrange(int(8.06 * R))
        # dif4: u2 = v0 + 16r - v2 limb-wise, normalised operands
        u2 = [a + L16[i] - b for i, (a, b) in enumerate(zip(limbs(v0), limbs(v2)))]
        s = [a + b for a, b in zip(u2, limbs(u3))]
        d = [a + L16[i] - b for i, (a, b) in enumerate(zip(u2, limbs(u3)))]
        assert max(s[:8]) < 1 << 31 and max(d[:8]) < int(2.42 * (1 << 30))
        assert val(s) < 64 * R and val(d) < 64 * R
        check_reduced(red(s), v0 - v2 + u3)
        check_reduced(red(d), v0 - v2 - u3)
        # dit4: u0 = v0 + v1 carry-free (limbs < 2^30), u2 = v2 + v3 normalised
        v1, v3 = rng.randrange(int(8.3 * R)), rng.randrange(int(8.3 * R))
        u0 = [a + b for a, b in zip(limbs(v0), limbs(v1))]
        u2v = v2 + v3
        e = [a + L32[i] - b for i, (a, b) in enumerate(zip(u0, limbs(u2v)))]
        assert min(e) >= 0 and max(e[:8]) < 1 << 31 and val(e) < 64 * R
        check_reduced(red(e), v0 + v1 - u2v)
    # extremes: every operand limb at its cap
    a = [MASK + L16[i] + MASK for i in range(8)]
    assert max(a) < 1 << 31
    b = [(1 << 30) - 2 + L32[i] for i in range(8)]
    assert max(b) < 1 << 31
