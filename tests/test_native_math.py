"""CPU: the device math headers (csrc/*.h) compiled for the host by g++ (test-only library
tests/native/libedc_hostcheck.so) agree with the oracle -- checks the radix-2^29 lazy-bound
arithmetic, ZIP215 decode, SHA-512, scalar mod l and ChaCha20 logic without a GPU."""
import ctypes
import hashlib
import os
import random
import subprocess

import pytest

from conftest import ROOT

NATIVE = os.path.join(ROOT, "tests", "native")
CSRC = os.path.join(ROOT, "ed25519-consensus_amd", "csrc")


@pytest.fixture(scope="module")
def hc():
    so = os.path.join(NATIVE, "libedc_hostcheck.so")
    src = os.path.join(NATIVE, "hostcheck.cpp")
    deps = [src] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if not os.path.exists(so) or any(os.path.getmtime(d) > os.path.getmtime(so) for d in deps):
        subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-Wno-unknown-pragmas",
                               "-I", CSRC, "-o", so, src])
    return ctypes.CDLL(so)


def b32(x):
    return (x % (1 << 256)).to_bytes(32, "little")


def test_field_ops(hc, oracle):
    P = oracle.P
    rnd = random.Random(7)
    out = ctypes.create_string_buffer(64)
    edge = [0, 1, P - 1, P, P + 1, 2**255 - 1, 2**255 - 20, 2**254, 19]
    vals = edge + [rnd.getrandbits(255) for _ in range(400)]
    for i, a in enumerate(vals):
        c = vals[(i * 7 + 3) % len(vals)]
        for op, exp in [(0, a * c), (1, a * a), (2, a + c), (3, a - c), (6, -a)]:
            hc.hc_fe_op(op, b32(a), b32(c), out)
            assert int.from_bytes(out.raw[:32], "little") == exp % P, (op, a, c)
    for a in vals[:40]:
        hc.hc_fe_op(5, b32(a), b32(0), out)
        assert int.from_bytes(out.raw[:32], "little") == pow(a, (P - 5) // 8, P)
        if a % P:
            hc.hc_fe_op(4, b32(a), b32(0), out)
            assert int.from_bytes(out.raw[:32], "little") == pow(a, P - 2, P)


def test_lazy_bound_chains(hc, oracle):
    P = oracle.P
    rnd = random.Random(11)
    out = ctypes.create_string_buffer(32)
    for _ in range(50):
        x, y = rnd.getrandbits(255), rnd.getrandbits(255)
        hc.hc_fe_chain(b32(x), b32(y), 64, out)
        for _ in range(64):
            s = (x + y) * (y + x)
            t = s - (x + x)
            x, y = y, (t - y) ** 2 % P
        assert int.from_bytes(out.raw, "little") == y % P


def test_mul_at_input_bound(hc, oracle):
    """fe_mul / fe_sqr on limbs at and near the mul-input bound (every limb up to twice the
    reduced bound: a lazy sum of two reduced elements): the value mod p, and reduced outputs
    (limbs < 2^29 + 2^19)."""
    P = oracle.P
    rnd = random.Random(29)
    top = 2 * ((1 << 29) + (1 << 19)) - 1
    LimbsT = ctypes.c_uint32 * 9
    out = ctypes.create_string_buffer(32)
    lim = LimbsT()
    cases = [[top] * 9, [top] * 8 + [0], [0] * 8 + [top], [(1 << 29) - 1] * 9]
    cases += [[rnd.randrange(top + 1) for _ in range(9)] for _ in range(300)]
    cases += [[top - rnd.randrange(1 << 12) for _ in range(9)] for _ in range(100)]
    for i, a in enumerate(cases):
        b = cases[(i * 5 + 1) % len(cases)]
        va = sum(x << (29 * k) for k, x in enumerate(a))
        vb = sum(x << (29 * k) for k, x in enumerate(b))
        for op, exp in [(0, va * vb), (1, va * va)]:
            hc.hc_fe_limbs(op, LimbsT(*a), LimbsT(*b), out, lim)
            assert int.from_bytes(out.raw, "little") == exp % P, (op, a, b)
            assert max(lim) < (1 << 29) + (1 << 19), (op, list(lim))


def test_mul_lazy_sub_operand_at_bound(hc, oracle):
    """The asymmetric fe_mul bound the point formulas rely on (fe25519.h fe_sub_lazy): one
    operand a lazy difference at its largest (D = 2Z at its lazy maximum minus 0, limbs up to
    2^31.61), the other reduced at its largest (limbs 2^29 + 2^19 - 1): exact mod p, reduced out."""
    P = oracle.P
    rnd = random.Random(31)
    LimbsT = ctypes.c_uint32 * 9
    red = (1 << 29) + (1 << 19) - 1
    dmax = 2 * red
    out = ctypes.create_string_buffer(32)
    lim, lz = LimbsT(), LimbsT()
    cases = [([dmax] * 9, [0] * 9), ([dmax] * 9, [red] * 9)]
    cases += [([rnd.randrange(dmax + 1) for _ in range(9)], [rnd.randrange(red + 1) for _ in range(9)])
              for _ in range(200)]
    val = lambda x: sum(v << (29 * k) for k, v in enumerate(x))
    for a, b in cases:
        hc.hc_fe_sub_lazy(LimbsT(*a), LimbsT(*b), lz)
        assert val(list(lz)) % P == (val(a) - val(b)) % P
        assert max(lz) < 2**31.61
        for partner in ([red] * 9, [rnd.randrange(red + 1) for _ in range(9)]):
            for x, y in ((list(lz), partner), (partner, list(lz))):
                hc.hc_fe_limbs(0, LimbsT(*x), LimbsT(*y), out, lim)
                assert int.from_bytes(out.raw, "little") == val(x) * val(y) % P
                assert max(lim) < (1 << 29) + (1 << 19)


def test_signed_mixed_addition(hc, oracle):
    """ge_madd_sgn (the bucket accumulation's addition, lazy carries) for both signs, on affine and
    projective accumulators, against the oracle."""
    from conftest import golden
    valid = [bytes.fromhex(c["enc"]) for c in golden("decode.json")["cases"] if c["ok"]]
    out = ctypes.create_string_buffer(32)
    rnd = random.Random(13)
    for _ in range(80):
        e1, e2 = rnd.choice(valid), rnd.choice(valid)
        P1, P2 = oracle.decompress(e1), oracle.decompress(e2)
        for pre in (0, 3):
            A = P1
            for _ in range(pre):
                A = oracle.double(A)
            for neg in (0, 1):
                assert hc.hc_point_madd_sgn(e1, e2, neg, pre, out)
                exp = oracle.add(A, oracle.neg(P2) if neg else P2)
                assert out.raw == oracle.compress(exp)


def test_decompress_and_point_ops(hc, oracle):
    from conftest import golden
    out = ctypes.create_string_buffer(64)
    valid = []
    for c in golden("decode.json")["cases"]:
        e = bytes.fromhex(c["enc"])
        ok = hc.hc_decompress(e, out)
        assert bool(ok) == c["ok"], c["enc"]
        if ok:
            assert out.raw[:32].hex() == c["x"] and out.raw[32:].hex() == c["y"]
            valid.append(e)
    bufs = [ctypes.create_string_buffer(32) for _ in range(4)]
    rnd = random.Random(3)
    for _ in range(60):
        e1, e2 = rnd.choice(valid), rnd.choice(valid)
        assert hc.hc_point_ops(e1, e2, *bufs)
        P1, P2 = oracle.decompress(e1), oracle.decompress(e2)
        assert bufs[0].raw == oracle.compress(oracle.add(P1, P2))
        assert bufs[1].raw == oracle.compress(oracle.double(P1))
        assert bufs[2].raw == oracle.compress(oracle.add(P1, P2))
        assert bufs[3].raw == oracle.compress(oracle.mul_by_cofactor(P1))


def test_sha512_challenge_scalars_chacha(hc, oracle):
    rnd = random.Random(5)
    out = ctypes.create_string_buffer(64)
    for ml in [0, 1, 47, 48, 63, 64, 111, 112, 127, 128, 175, 176, 300, 1024]:
        R, A, M = rnd.randbytes(32), rnd.randbytes(32), rnd.randbytes(ml)
        hc.hc_sha512(R, A, M, ctypes.c_uint64(ml), out)
        assert out.raw == hashlib.sha512(R + A + M).digest()
        hc.hc_sha512(R, None, M, ctypes.c_uint64(ml), out)
        assert out.raw == hashlib.sha512(R + M).digest()
        hc.hc_challenge(R, A, M, ctypes.c_uint64(ml), out)
        assert int.from_bytes(out.raw[:32], "little") == oracle.challenge(R, A, M)
    L = oracle.L
    for i in range(500):
        x = rnd.getrandbits(512) if i % 4 else (1 << 512) - 1 - rnd.getrandbits(40)
        hc.hc_sc_reduce_wide(x.to_bytes(64, "little"), out)
        assert int.from_bytes(out.raw[:32], "little") == x % L
        a, c = rnd.randrange(L), rnd.randrange(L)
        for op, exp in [(0, a * c), (1, a + c), (2, a - c), (3, (a % (1 << 128)) * c)]:
            hc.hc_sc_op(op, b32(a), b32(c), out)
            assert int.from_bytes(out.raw[:32], "little") == exp % L
    # the folds' boundaries: multiples of l and their neighbours, 2^252 / 2^260 / 2^385 edges,
    # all-ones, single bits (each fold's sign and carry cases)
    edges = [0, 1, L - 1, L, L + 1, 2 * L - 1, 2 * L, 2**252 - 1, 2**252, 2**253, 2**260 - 1,
             2**385, 2**512 - 1, 2**511, ((2**512 - 1) // L) * L, ((2**512 - 1) // L) * L - 1]
    edges += [1 << b for b in range(0, 512, 7)] + [(1 << b) - 1 for b in range(1, 513, 13)]
    edges += [k * L + d for k in [1, 3, 2**130, 2**259] for d in [-1, 0, 1]]
    edges += [(h << 252) + rnd.getrandbits(rnd.randrange(1, 200)) for h in range(1, 300)]   # third fold < 0
    for x in edges:
        hc.hc_sc_reduce_wide(x.to_bytes(64, "little"), out)
        assert int.from_bytes(out.raw[:32], "little") == x % L, hex(x)
    for v in [0, L - 1, L, L + 1, 2**255, 2**256 - 1]:
        assert hc.hc_sc_is_canonical(b32(v)) == (v < L)
    for key in [bytes(32), bytes([0x33]) * 32]:
        for ctr in [0, 1, 7, 2**32 + 1]:
            hc.hc_chacha_block(key, ctypes.c_uint64(ctr), out)
            assert out.raw == oracle.chacha20_block(key, ctr)


def test_fe_is_zero_lazy_limbs(hc):
    """fe_is_zero's short form (one fold, compare with 0 and p) on every multiple of p that the
    lazy limb bound (< 2^30.41 per limb) can hold, in normalized and carry-shifted limb forms, and
    on random non-zero neighbours."""
    P = 2**255 - 19
    bound = int(2**30.41)
    rnd = random.Random(11)

    def limbs(v):
        return [(v >> (29 * i)) & ((1 << 29) - 1) if i < 8 else v >> 232 for i in range(9)]

    def call(ls):
        assert all(0 <= x < bound for x in ls)
        return hc.hc_fe_is_zero_limbs((ctypes.c_uint32 * 9)(*ls))

    checked = 0
    for k in range(0, 2**262 // P):
        base = limbs(k * P)
        if base[8] >= bound:
            break
        forms = [base]
        for _ in range(6):                    # move 2^29 down from limb i+1 into limb i
            f = list(forms[-1])
            i = rnd.randrange(8)
            if f[i + 1] > 0 and f[i] + (1 << 29) < bound:
                f[i + 1] -= 1
                f[i] += 1 << 29
            forms.append(f)
        for f in forms:
            assert call(f) == 1, (k, f)
            g = list(f)
            g[rnd.randrange(9)] ^= 1 << rnd.randrange(20)
            v = sum(x << (29 * i) for i, x in enumerate(g))
            if all(x < bound for x in g):
                assert call(g) == (1 if v % P == 0 else 0)
            checked += 1
    assert checked > 50
    for _ in range(2000):
        ls = [rnd.randrange(bound) for _ in range(9)]
        v = sum(x << (29 * i) for i, x in enumerate(ls))
        assert call(ls) == (1 if v % P == 0 else 0)
