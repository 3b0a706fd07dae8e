"""GPU: the persistent validator-key cache (include/edc.h edc_keycache_*, keycache.h) and batched key
ingestion (edc_vk_validate = VerificationKey::try_from, src/verification_key.rs:160-175).

The cache must not change a single verdict: with keys registered, batch verdicts and the compressed
[8]*check equal the C oracle's (dalek algorithm, no cache) bit-exactly, and per-item verdicts equal
Item::verify_single's (src/batch.rs:104-107) for every item -- including the ZIP215 small-order /
non-canonical keys of tests/small_order.rs:12-77 and an undecodable key registered in the cache
(MalformedPublicKey per item, a failed batch)."""
import random

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

L_ORDER = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def oracle_c():
    import os
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c as oc
    return oc


@pytest.fixture()
def cached(engine):
    yield engine
    engine.keycache_clear()


def test_vk_validate_matches_golden_decode(engine, edc):
    cases = golden("decode.json")["cases"]
    encs = [bytes.fromhex(c["enc"]) for c in cases]
    assert engine.vk_validate(encs) == [0 if c["ok"] else 2 for c in cases]
    fx = golden("zip215_small_order.json")
    vks = [bytes.fromhex(c["vk"]) for c in fx["cases"]]
    assert engine.vk_validate(vks) == [0] * len(vks)          # every corpus key decodes (ZIP215)
    assert engine.vk_validate([]) == []
    got = edc.VerificationKey.try_from_many(encs, engine=engine)
    for c, g in zip(cases, got):
        assert isinstance(g, edc.VerificationKey) == c["ok"]
        assert isinstance(g, edc.MalformedPublicKey) == (not c["ok"])


def test_keycache_load_dedupes_and_flags(cached):
    cases = golden("decode.json")["cases"]
    encs = [bytes.fromhex(c["enc"]) for c in cases]
    keys = encs + encs[:5]                                      # duplicates map to one entry
    u, ok = cached.keycache_load(keys)
    assert u == len(set(encs)) == cached.keycache_size()
    assert ok == [c["ok"] for c in cases] + [c["ok"] for c in cases[:5]]
    cached.keycache_clear()
    assert cached.keycache_size() == 0


@pytest.mark.parametrize("n,m,register,bad", [(8192, 150, "all", None), (8192, 150, "all", 4321),
                                              (8192, 150, "half", 17), (4096, 4096, "all", None),
                                              (2048, 2048, "half", 100), (8192, 1, "all", None)])
def test_keycache_batch_matches_oracle(cached, oracle_c, n, m, register, bad):
    rnd = random.Random(n * 7 + m)
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(120) for _ in range(n)]
    vks, sigs = cached.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
    if bad is not None:
        msgs[bad] = msgs[bad][:-1] + bytes([msgs[bad][-1] ^ 1])
    zseed = rnd.randbytes(32)
    items = list(zip(vks, sigs, msgs))
    exp_code, exp_c8 = oracle_c.batch_verify(items, zseed)
    plain = cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    distinct = list(dict.fromkeys(vks))
    reg = distinct if register == "all" else distinct[::2]
    u, ok = cached.keycache_load(reg + [rnd.randbytes(32) for _ in range(3)])   # plus unrelated keys
    assert u == len(reg) + 3 and all(ok[:len(reg)])
    got = cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    assert got == plain == (exp_code, exp_c8)
    assert exp_code == (0 if bad is None else 1)
    each = cached.verify_each(vks[:512], sigs[:512], msgs[:512])
    assert each == [1 if (bad is not None and i == bad) else 0 for i in range(512)]


def test_keycache_undecodable_key_fails_batch(cached):
    rnd = random.Random(5)
    n, m = 4096, 8
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(40) for _ in range(n)]
    vks, sigs = cached.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
    bad_key = bytes.fromhex([c for c in golden("decode.json")["cases"] if not c["ok"]][0]["enc"])
    vks = list(vks)
    vks[9] = bad_key
    zseed = rnd.randbytes(32)
    plain = cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    u, ok = cached.keycache_load(list(dict.fromkeys(vks)))
    assert ok.count(False) == 1
    assert cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True) == plain
    assert plain[0] == 1
    each = cached.verify_each(vks[:16], sigs[:16], msgs[:16])
    assert each == [2 if i == 9 else 0 for i in range(16)]


def test_keycache_corpus_fallback(cached):
    """configs[3] shape with every key registered: the small-order corpus keys, the validators and
    an undecodable key; per-item (comb path) and grouped fallback verdicts == verify_single's."""
    torch = pytest.importorskip("torch")
    import ctypes
    dev = torch.device("cuda:0")
    n, keys = 1 << 14, 150
    rnd = random.Random(99)
    seeds = [rnd.randbytes(32) for _ in range(keys)]
    msgs = [rnd.randbytes(64) for _ in range(n)]
    vks, sigs = cached.sign(seeds, msgs, seed_index=[i % keys for i in range(n)])
    expect = [0] * n
    fx = golden("zip215_small_order.json")
    pos = rnd.sample(range(n), len(fx["cases"]) + 4)
    for p, c in zip(pos, fx["cases"]):
        vks[p], sigs[p], msgs[p] = bytes.fromhex(c["vk"]), bytes.fromhex(c["sig"]), bytes.fromhex(fx["msg"])
        expect[p] = c["expect_single"]
    p_bad, p_A, p_R, p_s = pos[-4:]
    msgs[p_bad] = msgs[p_bad][:-1] + bytes([msgs[p_bad][-1] ^ 1])
    expect[p_bad] = 1
    dec = [c for c in golden("decode.json")["cases"] if not c["ok"]]
    vks[p_A] = bytes.fromhex(dec[0]["enc"])
    expect[p_A] = 2
    sigs[p_R] = bytes.fromhex(dec[1]["enc"]) + sigs[p_R][32:]
    expect[p_R] = 1
    s = int.from_bytes(sigs[p_s][32:], "little") + L_ORDER
    sigs[p_s] = sigs[p_s][:32] + s.to_bytes(32, "little")
    expect[p_s] = 1
    # per-item verdicts without the cache, then with every key registered
    assert cached.verify_each(vks, sigs, msgs) == expect
    u, ok = cached.keycache_load(vks)
    assert u == len(set(vks)) and ok.count(False) == 1
    assert cached.verify_each(vks, sigs, msgs) == expect
    offs = [0]
    for mm in msgs:
        offs.append(offs[-1] + len(mm))

    def _dev(b):
        return torch.tensor(list(b) or [0], dtype=torch.uint8, device=dev)
    d_vk, d_sig, d_msg = _dev(b"".join(vks)), _dev(b"".join(sigs)), _dev(b"".join(msgs))
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    zseed = rnd.randbytes(32)
    verdicts = ctypes.create_string_buffer(n)
    nbad = cached.lib.edc_find_invalid_device(cached.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                              d_off.data_ptr(), zseed, 1024, verdicts)
    assert list(verdicts.raw) == expect and nbad == 4
