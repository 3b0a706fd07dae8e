"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer over the host-side code.

tests/native/sanitize_main.cpp links the device math headers (through tests/native/hostcheck.cpp,
the same csrc/*.h the kernels use) and the oracle's C restatement (oracle/edc_oracle.c) into ONE
executable built with -fsanitize=address,undefined -fno-sanitize-recover=all. It runs as a child
process fed by stdin (no sanitizer runtime is preloaded into Python), over the golden fixtures and
random inputs; any sanitizer report aborts it, and every result must match the Python oracle /
the fixtures. GPU code is not covered (GPU sanitizers are unavailable on this pool)."""
import hashlib
import os
import random
import shutil
import subprocess

import pytest

from conftest import ROOT, golden

CSRC = os.path.join(ROOT, "ed25519-consensus_amd", "csrc")
NATIVE = os.path.join(ROOT, "tests", "native")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.fixture(scope="module")
def san(tmp_path_factory):
    if not shutil.which("gcc") or not shutil.which("g++"):
        pytest.skip("no host compiler")
    d = tmp_path_factory.mktemp("san")
    obj, exe = str(d / "oracle.o"), str(d / "san")
    subprocess.check_call(["gcc", *SAN, "-std=c11", "-pthread", "-c", os.path.join(ROOT, "oracle", "edc_oracle.c"),
                           "-o", obj])
    subprocess.check_call(["g++", *SAN, "-std=c++17", "-Wno-unknown-pragmas", "-I", CSRC,
                           os.path.join(NATIVE, "hostcheck.cpp"), os.path.join(NATIVE, "sanitize_main.cpp"), obj,
                           "-o", exe, "-lpthread"])

    def run(lines):
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
                   UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
        p = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, env=env,
                           timeout=600)
        assert p.returncode == 0 and "Sanitizer" not in p.stderr, p.stderr[-4000:]
        out = p.stdout.splitlines()
        assert len(out) == len(lines)
        return out
    return run


def h(b):
    return b.hex() if b else "-"


def b32(x):
    return (x % (1 << 256)).to_bytes(32, "little")


def test_sanitized_field_scalar_hash_chacha(san, oracle):
    P, L = oracle.P, oracle.L
    rnd = random.Random(17)
    vals = [0, 1, P - 1, P, P + 1, 2**255 - 1, 2**255 - 20, 19] + [rnd.getrandbits(255) for _ in range(120)]
    lines, exp = [], []
    for i, a in enumerate(vals):
        c = vals[(5 * i + 1) % len(vals)]
        for op, e in [(0, a * c), (1, a * a), (2, a + c), (3, a - c), (6, -a)]:
            lines.append(f"fe {op} {b32(a).hex()} {b32(c).hex()}")
            exp.append(b32(e % P).hex())
    for a in vals[:12]:
        lines.append(f"fe 5 {b32(a).hex()} {b32(0).hex()}")
        exp.append(b32(pow(a, (P - 5) // 8, P)).hex())
    for ml in [0, 1, 47, 48, 111, 112, 127, 128, 175, 176, 1024]:
        R, A, M = rnd.randbytes(32), rnd.randbytes(32), rnd.randbytes(ml)
        lines.append(f"sha {R.hex()} {A.hex()} {h(M)}")
        exp.append(hashlib.sha512(R + A + M).hexdigest())
        lines.append(f"chal {R.hex()} {A.hex()} {h(M)}")
        exp.append(b32(oracle.challenge(R, A, M)).hex())
    for _ in range(100):
        x = rnd.getrandbits(512)
        lines.append(f"scw {x.to_bytes(64, 'little').hex()}")
        exp.append(b32(x % L).hex())
        a, c = rnd.randrange(L), rnd.randrange(L)
        for op, e in [(0, a * c), (1, a + c), (2, a - c), (3, (a % (1 << 128)) * c)]:
            lines.append(f"sco {op} {b32(a).hex()} {b32(c).hex()}")
            exp.append(b32(e % L).hex())
    for v in [0, L - 1, L, L + 1, 2**255, 2**256 - 1]:
        lines.append(f"canon {b32(v).hex()}")
        exp.append("1" if v < L else "0")
    for key in [bytes(32), bytes([0x33]) * 32]:
        for ctr in [0, 1, 2**32 + 1]:
            lines.append(f"chacha {key.hex()} {ctr}")
            exp.append(oracle.chacha20_block(key, ctr).hex())
    assert san(lines) == exp


def test_sanitized_decode_and_point_ops(san, oracle):
    cases = golden("decode.json")["cases"]
    out = san([f"dec {c['enc']}" for c in cases])
    valid = []
    for c, o in zip(cases, out):
        ok, xy = o.split()
        assert bool(int(ok)) == c["ok"], c["enc"]
        if c["ok"]:
            assert xy == c["x"] + c["y"]
            valid.append(bytes.fromhex(c["enc"]))
    rnd = random.Random(4)
    pairs = [(rnd.choice(valid), rnd.choice(valid)) for _ in range(30)]
    for (e1, e2), o in zip(pairs, san([f"pt {a.hex()} {b.hex()}" for a, b in pairs])):
        ok, r = o.split()
        P1, P2 = oracle.decompress(e1), oracle.decompress(e2)
        s = oracle.compress(oracle.add(P1, P2)).hex()
        assert ok == "1" and r == s + oracle.compress(oracle.double(P1)).hex() + s + \
            oracle.compress(oracle.mul_by_cofactor(P1)).hex()


def test_sanitized_c_oracle_batches_and_single(san):
    lines, exp = [], []
    for b in golden("batches.json")["batches"]:
        it = [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]
        offs = [0]
        for _, _, m in it:
            offs.append(offs[-1] + len(m))
        arena = b"".join(m for _, _, m in it)
        lines.append(f"obv {b['z_seed']} {h(b''.join(v for v, _, _ in it))} {h(b''.join(s for _, s, _ in it))} "
                     f"{h(arena)} {','.join(map(str, offs))}")
        exp.append((b["expect_code"], b["expect_check8"]))
        for (v, s, m), e in zip(it, b["expect_single"]):
            lines.append(f"ov {v.hex()} {s.hex()} {h(m)}")
            exp.append(e)
    fx = golden("zip215_small_order.json")
    for c in fx["cases"]:
        lines.append(f"ov {c['vk']} {c['sig']} {fx['msg']}")
        exp.append(c["expect_single"])
    for o, e in zip(san(lines), exp):
        if isinstance(e, tuple):
            rc, ev, c8 = o.split()
            assert int(rc) == e[0]
            assert (c8 if ev == "1" else None) == e[1]
        else:
            assert int(o) == e
