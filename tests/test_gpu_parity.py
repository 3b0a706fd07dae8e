"""GPU parity: the HIP path through the C ABI vs the committed golden fixtures (oracle outputs)
and vs the oracle on seeded inputs. Bit-exact: verdicts, per-item error codes, challenge
scalars, decoded coordinates and the compressed [8]*check point."""
import hashlib
import random

import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _items(b):
    return [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]


def test_decompress_matches_fixture(engine):
    cases = golden("decode.json")["cases"]
    res = engine.decompress([bytes.fromhex(c["enc"]) for c in cases])
    for c, (ok, x, y) in zip(cases, res):
        assert ok == c["ok"], c["enc"]
        if ok:
            assert x.hex() == c["x"] and y.hex() == c["y"], c["enc"]


def test_challenge_matches_fixture(engine):
    for b in golden("batches.json")["batches"]:
        it = _items(b)
        if not it:
            continue
        ks = engine.challenge([v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it])
        assert [k.hex() for k in ks] == b["k"], b["name"]


@pytest.mark.parametrize("b", golden("batches.json")["batches"], ids=lambda b: b["name"])
def test_batch_fixture(engine, b):
    it = _items(b)
    code, check8 = engine.batch_verify([v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it],
                                       z_seed=bytes.fromhex(b["z_seed"]), want_check8=True)
    assert code == b["expect_code"]
    if b["expect_check8"] is not None:
        assert check8.hex() == b["expect_check8"]
    else:
        assert check8 == bytes(32)
    singles = engine.verify_each([v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it])
    assert singles == b["expect_single"]
    pre = engine.verify_prehashed_each([v for v, _, _ in it], [s for _, s, _ in it],
                                       [bytes.fromhex(k) for k in b["k"]])
    assert pre == b["expect_single"]


def test_explicit_z_equals_seeded_z(engine, oracle):
    b = [x for x in golden("batches.json")["batches"] if x["name"] == "two_bad_of_300"][0]
    it = _items(b)
    seed = bytes.fromhex(b["z_seed"])
    z = b"".join(zz.to_bytes(16, "little") for zz in oracle.z_values(seed, len(it)))
    code, check8 = engine.batch_verify([v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it],
                                       z=z, want_check8=True)
    assert code == b["expect_code"] and check8.hex() == b["expect_check8"]


def test_zip215_corpus_single_and_batch(engine, edc):
    fx = golden("zip215_small_order.json")
    msg = bytes.fromhex(fx["msg"])
    vks = [bytes.fromhex(c["vk"]) for c in fx["cases"]]
    sigs = [bytes.fromhex(c["sig"]) for c in fx["cases"]]
    assert engine.verify_each(vks, sigs, [msg] * len(vks)) == [c["expect_single"] for c in fx["cases"]]
    for vk, sig, c in zip(vks, sigs, fx["cases"]):
        code, check8 = engine.batch_verify([vk], [sig], [msg], z_seed=bytes([0x33]) * 32, want_check8=True)
        assert code == c["expect_batch1"] == 0
        assert check8 == bytes([1]) + bytes(31)
    # the reference test body, through the mirrored API (tests/small_order.rs:88-104); try_from
    # keeps each decoded key in the engine's cache, dropped again at the end
    try:
        for vk, sig in list(zip(vks, sigs))[::13]:
            single_ok = True
            try:
                edc.VerificationKey.try_from(vk, engine).verify(sig, msg)
            except edc.Error:
                single_ok = False
            bv = edc.batch.Verifier(engine)
            bv.queue((vk, sig, msg))
            try:
                bv.verify(bytes(32))
                batch_ok = True
            except edc.InvalidSignature:
                batch_ok = False
            assert single_ok == batch_ok
    finally:
        engine.keycache_clear()


def test_rfc8032_via_api(engine, edc):
    try:
        for v in golden("rfc8032.json")["vectors"]:
            sk, pk, sig, msg = (bytes.fromhex(v[k]) for k in ("sk", "pk", "sig", "msg"))
            vk = edc.VerificationKey.try_from(pk, engine)
            assert vk.cached
            vk.verify(sig, msg)
            key = edc.SigningKey(sk, engine)
            assert key.sign(msg).to_bytes() == sig
            assert key.verification_key_bytes().to_bytes() == pk
    finally:
        engine.keycache_clear()


def test_reference_batch_tests_via_api(engine, edc):
    # tests/batch.rs:5-44 with GPU-signed data
    rnd = random.Random(99)
    keys = [edc.SigningKey(rnd.randbytes(32), engine) for _ in range(32)]
    bv = edc.batch.Verifier(engine)
    for k in keys:
        bv.queue((k.verification_key_bytes(), k.sign(b"BatchVerifyTest"), b"BatchVerifyTest"))
    bv.verify(rnd.randbytes(32))
    bv = edc.batch.Verifier(engine)
    items = []
    for i, k in enumerate(keys):
        sig = k.sign(b"BatchVerifyTest" if i != 10 else b"badmsg")
        item = edc.batch.Item(k.verification_key_bytes(), sig, b"BatchVerifyTest")
        items.append(item)
        bv.queue(item)
    with pytest.raises(edc.InvalidSignature):
        bv.verify(rnd.randbytes(32))
    for i, item in enumerate(items):
        if i != 10:
            item.verify_single(engine)
        else:
            with pytest.raises(edc.InvalidSignature):
                item.verify_single(engine)
    assert [i for i, c in enumerate(edc.batch.Item.verify_single_many(items, engine)) if c] == [10]


def test_sign_matches_oracle(engine, oracle):
    rnd = random.Random(1234)
    seeds = [rnd.randbytes(32) for _ in range(24)]
    msgs = [rnd.randbytes(rnd.randrange(0, 300)) for _ in range(24)]
    vks, sigs = engine.sign(seeds, msgs)
    for s, m, vk, sig in zip(seeds, msgs, vks, sigs):
        assert vk == oracle.public_key(s)
        assert sig == oracle.sign(s, m)


def test_random_batches_against_oracle(engine, oracle):
    """Seeded batches with random corruption, sizes up to ~400, repeated and distinct keys."""
    rnd = random.Random(2024)
    for trial in range(6):
        n = rnd.choice([3, 17, 64, 150, 257, 400])
        nkeys = rnd.choice([1, 2, 5, n])
        seeds = [rnd.randbytes(32) for _ in range(nkeys)]
        msgs = [rnd.randbytes(rnd.randrange(0, 200)) for _ in range(n)]
        vks, sigs = engine.sign(seeds, msgs, seed_index=[i % nkeys for i in range(n)])
        vks, sigs = list(vks), list(sigs)
        if trial % 2:
            j = rnd.randrange(n)
            sigs[j] = sigs[j][:40] + bytes([sigs[j][40] ^ 4]) + sigs[j][41:]
        zseed = rnd.randbytes(32)
        items = list(zip(vks, sigs, msgs))
        exp_code, exp_check8 = oracle.batch_verify_seeded(items, zseed)
        code, check8 = engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
        assert code == exp_code
        assert check8 == (exp_check8 if exp_check8 is not None else bytes(32))


def test_shard_partials_combine_bit_exact(engine, edc):
    """Multi-GPU math on one GPU: shards with global z offsets -> partial points -> combine
    equals the unsharded verdict and [8]*check byte for byte."""
    import ctypes
    b = [x for x in golden("batches.json")["batches"] if x["name"] == "mixed_corpus_one_bad"][0]
    it = _items(b)
    seed = bytes.fromhex(b["z_seed"])
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")

    def to_dev(buf):
        return torch.tensor(list(buf) or [0], dtype=torch.uint8, device=dev)

    for nshards in (1, 2, 3, 5):
        bounds = [len(it) * s // nshards for s in range(nshards + 1)]
        partials, bad_any = [], 0
        for s in range(nshards):
            sub = it[bounds[s]:bounds[s + 1]]
            vk = to_dev(b"".join(v for v, _, _ in sub))
            sg = to_dev(b"".join(x for _, x, _ in sub))
            ms = to_dev(b"".join(m for _, _, m in sub))
            offs = [0]
            for _, _, m in sub:
                offs.append(offs[-1] + len(m))
            off = torch.tensor(offs, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            part = ctypes.create_string_buffer(128)
            bad = ctypes.c_int(0)
            rc = engine.lib.edc_batch_partial_device(engine.ctx, len(sub), vk.data_ptr(), sg.data_ptr(),
                                                     ms.data_ptr(), off.data_ptr(), seed, bounds[s], None,
                                                     part, ctypes.byref(bad))
            assert rc == 0
            partials.append(part.raw)
            bad_any |= bad.value
        code, check8 = engine.combine_partials(partials, bad_any)
        assert code == b["expect_code"] and check8.hex() == b["expect_check8"], nshards


def test_large_batch_properties(engine):
    """2^16 distinct keys (BASELINE configs[1]): valid batch -> Ok and identity; one flipped
    message byte -> Err, and the fallback pinpoints exactly that item."""
    import os as _os
    rnd = random.Random(77)
    n = 1 << 16
    seeds = [hashlib.sha256(i.to_bytes(4, "little")).digest() for i in range(n)]
    msgs = [rnd.randbytes(32) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs)
    code, check8 = engine.batch_verify(vks, sigs, msgs, z_seed=_os.urandom(32), want_check8=True)
    assert code == 0 and check8 == bytes([1]) + bytes(31)
    bad = 40000
    msgs2 = list(msgs)
    msgs2[bad] = msgs2[bad][:-1] + bytes([msgs2[bad][-1] ^ 1])
    code, _ = engine.batch_verify(vks, sigs, msgs2, z_seed=_os.urandom(32))
    assert code == 1
    v = engine.verify_each(vks, sigs, msgs2)
    assert [i for i, c in enumerate(v) if c] == [bad]


def test_async_submit_wait_two_in_flight(engine, edc):
    """edc_batch_submit_device / edc_batch_wait: two batches in flight on separate slots give the
    same verdicts and [8]*check as the synchronous path."""
    import ctypes
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    bs = {x["name"]: x for x in golden("batches.json")["batches"]}
    jobs = []
    for name in ["two_bad_of_300", "repeated_keys_varlen", "mixed_corpus_one_bad", "c1_1024_distinct"]:
        b = bs[name]
        it = _items(b)
        vk = torch.tensor(list(b"".join(v for v, _, _ in it)), dtype=torch.uint8, device=dev)
        sg = torch.tensor(list(b"".join(s for _, s, _ in it)), dtype=torch.uint8, device=dev)
        ms = torch.tensor(list(b"".join(m for _, _, m in it)) or [0], dtype=torch.uint8, device=dev)
        offs = [0]
        for _, _, m in it:
            offs.append(offs[-1] + len(m))
        off = torch.tensor(offs, dtype=torch.int64, device=dev)
        jobs.append((b, len(it), vk, sg, ms, off))
    torch.cuda.synchronize()
    lib = engine.lib
    tickets = []
    results = []
    for b, n, vk, sg, ms, off in jobs:
        if len(tickets) == 2:
            t0, b0 = tickets.pop(0)
            c8 = ctypes.create_string_buffer(32)
            results.append((b0, lib.edc_batch_wait(engine.ctx, t0, c8, None, None), c8.raw))
        t = lib.edc_batch_submit_device(engine.ctx, n, vk.data_ptr(), sg.data_ptr(), ms.data_ptr(), off.data_ptr(),
                                        bytes.fromhex(b["z_seed"]), 0, None, 1)
        assert t >= 0
        tickets.append((t, b))
    while tickets:
        t0, b0 = tickets.pop(0)
        c8 = ctypes.create_string_buffer(32)
        results.append((b0, lib.edc_batch_wait(engine.ctx, t0, c8, None, None), c8.raw))
    assert len(results) == 4
    for b, code, c8 in results:
        assert code == b["expect_code"], b["name"]
        assert c8.hex() == b["expect_check8"], b["name"]


def test_host_submit_wait_in_flight(engine):
    """edc_batch_submit (host buffers staged per slot, copies overlapping the batches in flight):
    every golden batch, four at a time, gives the fixture's verdict and [8]*check."""
    bs = golden("batches.json")["batches"]
    pending, results = [], []
    for b in bs + bs:                                   # two passes: every slot is reused
        if len(pending) == 4:
            t0, b0 = pending.pop(0)
            results.append((b0, engine.batch_wait(t0, want_check8=True)))
        it = _items(b)
        t = engine.batch_submit([v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it],
                                bytes.fromhex(b["z_seed"]), want_check8=True)
        pending.append((t, b))
    while pending:
        t0, b0 = pending.pop(0)
        results.append((b0, engine.batch_wait(t0, want_check8=True)))
    assert len(results) == 2 * len(bs)
    for b, (code, c8) in results:
        assert code == b["expect_code"], b["name"]
        assert c8 == (bytes.fromhex(b["expect_check8"]) if b["expect_check8"] is not None else bytes(32)), b["name"]


def test_host_submit_offsets_not_zero_based(engine):
    """msg_off[0] != 0 (a caller's arena slice): offsets are rebased on the host, same verdict."""
    import ctypes
    b = [x for x in golden("batches.json")["batches"] if x["name"] == "repeated_keys_varlen"][0]
    it = _items(b)
    prefix = b"\xAA" * 7
    arena = prefix + b"".join(m for _, _, m in it)
    offs = (ctypes.c_uint64 * (len(it) + 1))()
    offs[0] = len(prefix)
    for i, (_, _, m) in enumerate(it):
        offs[i + 1] = offs[i] + len(m)
    c8 = ctypes.create_string_buffer(32)
    vks, sigs = b"".join(v for v, _, _ in it), b"".join(s for _, s, _ in it)
    t = engine.lib.edc_batch_submit(engine.ctx, len(it), vks, sigs, arena, offs, bytes.fromhex(b["z_seed"]), 0, 1)
    assert t >= 0
    assert engine.lib.edc_batch_wait(engine.ctx, t, c8, None, None) == b["expect_code"]
    assert c8.raw.hex() == b["expect_check8"]


@pytest.mark.parametrize("name", ["repeated_keys_varlen", "undecodable_A", "zip215_corpus_batch", "two_bad_of_300",
                                  "mixed_corpus_one_bad", "c1_1024_distinct"])
def test_host_submit_indexed_equals_fixture(engine, name):
    """edc_batch_submit_indexed: keys as positions in the registered list (registered in reverse
    first-occurrence order with a duplicate, so list position != cache index); same verdict and
    [8]*check as the fixture; an index past the list is an argument error."""
    from conftest import load_pkg
    b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
    it = _items(b)
    distinct = list(dict.fromkeys(v for v, _, _ in it))[::-1]
    reg = [distinct[0]] + distinct                       # position 0 duplicates position 1
    pos = {}
    for i, k in enumerate(reg):
        pos.setdefault(k, i)
    engine.keycache_load(reg)
    try:
        idx = [pos[v] for v, _, _ in it]
        if idx:
            idx[0] = 1 if idx[0] == 0 else idx[0]            # either position of the duplicated key
        t = engine.batch_submit_indexed(idx, [s for _, s, _ in it], [m for _, _, m in it],
                                        bytes.fromhex(b["z_seed"]), want_check8=True)
        code, c8 = engine.batch_wait(t, want_check8=True)
        assert code == b["expect_code"]
        assert c8 == (bytes.fromhex(b["expect_check8"]) if b["expect_check8"] is not None else bytes(32))
        with pytest.raises(load_pkg().EngineError):
            engine.batch_submit_indexed([len(reg)] + idx[1:], [s for _, s, _ in it], [m for _, _, m in it],
                                        bytes.fromhex(b["z_seed"]))
    finally:
        engine.keycache_clear()


def _dev_batch(torch, it, dev):
    vk = torch.tensor(list(b"".join(v for v, _, _ in it)) or [0], dtype=torch.uint8, device=dev)
    sg = torch.tensor(list(b"".join(s for _, s, _ in it)) or [0], dtype=torch.uint8, device=dev)
    mg = torch.tensor(list(b"".join(m for _, _, m in it)) or [0], dtype=torch.uint8, device=dev)
    offs = [0]
    for _, _, m in it:
        offs.append(offs[-1] + len(m))
    return vk, sg, mg, torch.tensor(offs, dtype=torch.int64, device=dev)


@pytest.mark.parametrize("b", golden("batches.json")["batches"], ids=lambda b: b["name"])
@pytest.mark.parametrize("shape", [(32, 10), (128, 9), (1024, 8)])
def test_batch_then_fallback_fixture(engine, b, shape):
    """edc_batch_verify_fallback_device (batch, then the one-pass grouped fallback and the quad
    per-item kernel on the failing ranges) returns the fixture's batch code, [8]*check and, for a
    failed batch, exactly Item::verify_single's code for every item."""
    torch = pytest.importorskip("torch")
    import ctypes
    it = _items(b)
    n = len(it)
    dev = torch.device("cuda:0")
    vk, sg, mg, off = _dev_batch(torch, it, dev)
    torch.cuda.synchronize()
    lib = engine.lib
    assert lib.edc_set_fallback_shape(engine.ctx, *shape) == 0
    try:
        v = ctypes.create_string_buffer(max(n, 1))
        cnt = ctypes.c_int(-1)
        c8 = ctypes.create_string_buffer(32)
        rc = lib.edc_batch_verify_fallback_device(engine.ctx, n, vk.data_ptr(), sg.data_ptr(), mg.data_ptr(),
                                                  off.data_ptr(), bytes.fromhex(b["z_seed"]), v, ctypes.byref(cnt), c8)
    finally:
        lib.edc_set_fallback_shape(engine.ctx, 128, 9)
    assert rc == b["expect_code"]
    if b["expect_check8"] is not None:
        assert c8.raw.hex() == b["expect_check8"]
    exp = b["expect_single"] if rc else [0] * n
    assert list(v.raw[:n]) == exp
    assert cnt.value == (sum(1 for e in exp if e) if rc else 0)
