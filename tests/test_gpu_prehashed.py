"""GPU: batch verification of prehashed items -- the reference's batch::Item is {vk_bytes, sig, k}
(src/batch.rs:76-80); k is computed once at Item::from (:82-94) and Verifier::verify (:149-217)
never sees the message. edc_batch_verify_prehashed / _device / edc_batch_submit_prehashed /
_device / edc_batch_verify_prehashed_fallback take that k instead of the message arena.

Checked bit-exactly: every golden batch with the fixture's own `k` field (tests/golden/batches.json)
against expect_code / expect_check8 / expect_single, through each entry; configs[2] at 2^20 (k from
the GPU's own SHA-512) against the message path, valid and with one corrupted signature; a k >= l is
a runtime error, never a verdict. Also: the synchronous slot's two-stream decode (slot 0) against a
pipelined slot (one stream) on batches that fail in the decode or the s check."""
import ctypes
import sys

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

IDENTITY = bytes([1]) + bytes(31)
IDENTITY_PARTIAL = bytes(32) + IDENTITY + IDENTITY + bytes(32)    # canonical X | Y | Z | T
L_ORDER = 2**252 + 27742317777372353535851937790883648493
BATCHES = golden("batches.json")["batches"]


def _items(b):
    return ([bytes.fromhex(v) for v, _, _ in b["items"]], [bytes.fromhex(s) for _, s, _ in b["items"]],
            [bytes.fromhex(m) for _, _, m in b["items"]], [bytes.fromhex(k) for k in b["k"]])


def _check(b, code, check8):
    assert code == b["expect_code"], b["name"]
    if b["expect_check8"] is not None:
        assert check8.hex() == b["expect_check8"], b["name"]
    else:
        assert check8 == bytes(32), b["name"]


@pytest.mark.parametrize("b", BATCHES, ids=lambda b: b["name"])
def test_golden_prehashed_host(engine, b):
    vks, sigs, _, ks = _items(b)
    zseed = bytes.fromhex(b["z_seed"])
    _check(b, *engine.batch_verify_prehashed(vks, sigs, ks, z_seed=zseed, want_check8=True))
    t = engine.batch_submit_prehashed(vks, sigs, ks, zseed, want_check8=True)
    _check(b, *engine.batch_wait(t, want_check8=True))
    code, verdicts, nbad, check8 = engine.batch_verify_prehashed_fallback(vks, sigs, ks, zseed)
    _check(b, code, check8)
    assert verdicts == (b["expect_single"] if code else [0] * len(vks))
    assert nbad == sum(1 for v in b["expect_single"] if v)


@pytest.mark.parametrize("b", BATCHES, ids=lambda b: b["name"])
def test_golden_prehashed_device(engine, b):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    vks, sigs, _, ks = _items(b)
    n = len(vks)
    d = {name: torch.tensor(list(b"".join(x)) or [0], dtype=torch.uint8, device=dev)
         for name, x in (("vk", vks), ("sig", sigs), ("k", ks))}
    torch.cuda.synchronize()
    lib = engine.lib
    zseed = bytes.fromhex(b["z_seed"])
    c8 = ctypes.create_string_buffer(32)
    code = lib.edc_batch_verify_prehashed_device(engine.ctx, n, d["vk"].data_ptr(), d["sig"].data_ptr(),
                                                 d["k"].data_ptr(), zseed, 0, None, c8)
    _check(b, code, c8.raw)
    t = lib.edc_batch_submit_prehashed_device(engine.ctx, n, d["vk"].data_ptr(), d["sig"].data_ptr(),
                                              d["k"].data_ptr(), zseed, 0, None, 1)
    assert t >= 0
    c8 = ctypes.create_string_buffer(32)
    _check(b, lib.edc_batch_wait(engine.ctx, t, c8, None, None), c8.raw)
    v = ctypes.create_string_buffer(max(n, 1))
    cnt = ctypes.c_int(0)
    c8 = ctypes.create_string_buffer(32)
    code = lib.edc_batch_verify_prehashed_fallback_device(engine.ctx, n, d["vk"].data_ptr(), d["sig"].data_ptr(),
                                                          d["k"].data_ptr(), zseed, v, ctypes.byref(cnt), c8)
    _check(b, code, c8.raw)
    assert list(v.raw[:n]) == (b["expect_single"] if code else [0] * n)


def test_explicit_z_prehashed(engine, oracle):
    b = [x for x in BATCHES if x["name"] == "two_bad_of_300"][0]
    vks, sigs, _, ks = _items(b)
    z = b"".join(zz.to_bytes(16, "little") for zz in oracle.z_values(bytes.fromhex(b["z_seed"]), len(vks)))
    _check(b, *engine.batch_verify_prehashed(vks, sigs, ks, z=z, want_check8=True))


def test_verifier_mirror_prehashed_items(engine, edc):
    """The mirrored Verifier over Items built as the reference stores them ({vk_bytes, sig, k}, no
    message), over message Items, and over a mix: same verdict and [8]*check as the fixture."""
    for name in ("two_bad_of_300", "repeated_keys_varlen", "undecodable_A"):
        b = [x for x in BATCHES if x["name"] == name][0]
        vks, sigs, msgs, ks = _items(b)
        seed = bytes.fromhex(b["z_seed"])
        for mode in ("prehashed", "message", "mixed"):
            v = edc.batch.Verifier(engine)
            for i, (vk, s, m, k) in enumerate(zip(vks, sigs, msgs, ks)):
                if mode == "prehashed" or (mode == "mixed" and i % 2):
                    v.queue(edc.batch.Item.prehashed(vk, s, k))
                else:
                    v.queue(edc.batch.Item(vk, s, m))
            _check(b, *v.verify_detailed(seed))


def test_noncanonical_k_is_an_error(engine, edc):
    b = [x for x in BATCHES if x["name"] == "batch_verify_32"][0]
    vks, sigs, _, ks = _items(b)
    k_bad = list(ks)
    k_bad[5] = (int.from_bytes(ks[5], "little") + L_ORDER).to_bytes(32, "little")   # same scalar mod l, >= l
    with pytest.raises(edc.EngineError, match="canonical"):
        engine.batch_verify_prehashed(vks, sigs, k_bad, z_seed=bytes(32))
    with pytest.raises(edc.EngineError, match="canonical"):
        engine.batch_wait(engine.batch_submit_prehashed(vks, sigs, k_bad, bytes(32)))
    # per-item path: checked on the host before any launch, including k = 2^256 - 1,
    # whose top radix-16 digit would index past the per-item tables
    with pytest.raises(edc.EngineError, match="canonical"):
        engine.verify_prehashed_each(vks, sigs, k_bad)
    with pytest.raises(edc.EngineError, match="canonical"):
        engine.verify_prehashed_each(vks[:1], sigs[:1], [b"\xff" * 32])
    with pytest.raises(ValueError, match="canonical"):
        edc.batch.Item.prehashed(vks[0], sigs[0], b"\xff" * 32)
    # the context stays usable
    _check(b, *engine.batch_verify_prehashed(vks, sigs, ks, z_seed=bytes.fromhex(b["z_seed"]), want_check8=True))
    assert engine.verify_prehashed_each(vks, sigs, ks) == b["expect_single"]


def test_misaligned_device_pointer_is_an_error(engine):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    b = [x for x in BATCHES if x["name"] == "batch_verify_32"][0]
    vks, sigs, _, ks = _items(b)
    buf = torch.zeros(64 + 32 * len(ks), dtype=torch.uint8, device=dev)
    buf[4:4 + 32 * len(ks)] = torch.tensor(list(b"".join(ks)), dtype=torch.uint8, device=dev)
    d_vk = torch.tensor(list(b"".join(vks)), dtype=torch.uint8, device=dev)
    d_sig = torch.tensor(list(b"".join(sigs)), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    rc = engine.lib.edc_batch_verify_prehashed_device(engine.ctx, len(ks), d_vk.data_ptr(), d_sig.data_ptr(),
                                                      buf.data_ptr() + 4, bytes(32), 0, None, None)
    assert rc == -2
    assert b"aligned" in engine.lib.edc_last_error(engine.ctx)


def _host_k(engine, vk, sig, msg, off):
    """k of every item from the GPU's SHA-512 through the host-buffer edc_challenge."""
    n = vk.numel() // 32
    hv, hs = vk.cpu().numpy().tobytes(), sig.cpu().numpy().tobytes()
    o = off.cpu()
    hm = msg.cpu().numpy().tobytes()
    offs = (ctypes.c_uint64 * (n + 1)).from_buffer_copy(o.numpy().astype("uint64").tobytes())
    out = ctypes.create_string_buffer(32 * n)
    assert engine.lib.edc_challenge(engine.ctx, n, hv, hs, hm, offs, out) == 0
    return out.raw


def test_config2_prehashed_equals_message_path(engine):
    """configs[2] at full size (2^20 votes from 150 validators, 120-byte messages): the prehashed
    device and host paths give the message path's verdict and [8]*check, valid and with one
    corrupted signature (a non-identity check point)."""
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    n, keys, mlen = bench.CONFIGS["c3"][:3]
    pkg = sys.modules["ed25519_consensus_amd"]
    vk, sig, msg, off = bench.make_workload(pkg, engine, torch, dev, n, keys, mlen, 0)
    torch.cuda.synchronize()
    lib = engine.lib
    zseed = bytes([0x6D]) * 32
    for corrupt in (False, True):
        if corrupt:
            sig[64 * 654321 + 50] ^= 0x04
            torch.cuda.synchronize()
        kb = _host_k(engine, vk, sig, msg, off)
        d_k = torch.frombuffer(bytearray(kb), dtype=torch.uint8).to(dev)
        torch.cuda.synchronize()
        c8_msg, c8_pre, c8_sub = (ctypes.create_string_buffer(32) for _ in range(3))
        code_msg = lib.edc_batch_verify_device(engine.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                               off.data_ptr(), zseed, 0, None, c8_msg)
        code_pre = lib.edc_batch_verify_prehashed_device(engine.ctx, n, vk.data_ptr(), sig.data_ptr(), d_k.data_ptr(),
                                                         zseed, 0, None, c8_pre)
        t = lib.edc_batch_submit_prehashed(engine.ctx, n, vk.cpu().numpy().tobytes(), sig.cpu().numpy().tobytes(), kb,
                                           zseed, 0, 1)
        assert t >= 0
        code_sub = lib.edc_batch_wait(engine.ctx, t, c8_sub, None, None)
        assert code_msg == code_pre == code_sub == (1 if corrupt else 0)
        assert c8_msg.raw == c8_pre.raw == c8_sub.raw
        assert (c8_msg.raw == IDENTITY) != corrupt
    del vk, sig, msg, off
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kind", ["bad_R", "bad_s", "bad_A", "wrong_msg", "valid"])
def test_dual_stream_slot0_equals_pipelined_slot(engine, kind):
    """Slot 0 (synchronous calls) decodes on a second stream beside SHA-512 / coefficients /
    binning; the pipelined slots run everything on one stream. On both: the same verdict and bad
    flag; for batches whose points all decode (a wrong message, valid) the same partial point
    ([8]*P compared, partials being projective); a batch rejected by its bad flag (undecodable R or
    key, s >= l) reports the identity as its partial on every slot, byte for byte (the MSM sum of
    an off-curve point would depend on the addition order; SURVEY §5: identical results across
    runs); slot 0's grouped fallback agrees with the per-item kernel."""
    torch = pytest.importorskip("torch")
    import random
    dev = torch.device("cuda:0")
    rnd = random.Random(kind)
    n, keys = 5000, 40
    seeds = [rnd.randbytes(32) for _ in range(keys)]
    msgs = [rnd.randbytes(48) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % keys for i in range(n)])
    vks, sigs = list(vks), list(sigs)
    dec_bad = [c for c in golden("decode.json")["cases"] if not c["ok"]]
    for p in rnd.sample(range(n), 3):
        if kind == "bad_R":
            sigs[p] = bytes.fromhex(dec_bad[1]["enc"]) + sigs[p][32:]
        elif kind == "bad_s":
            s = int.from_bytes(sigs[p][32:], "little") + L_ORDER
            sigs[p] = sigs[p][:32] + s.to_bytes(32, "little")
        elif kind == "bad_A":
            vks[p] = bytes.fromhex(dec_bad[0]["enc"])
        elif kind == "wrong_msg":
            msgs[p] = msgs[p][:-1] + bytes([msgs[p][-1] ^ 1])
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    t8 = lambda b: torch.tensor(list(b), dtype=torch.uint8, device=dev)
    d_vk, d_sig, d_msg = t8(b"".join(vks)), t8(b"".join(sigs)), t8(b"".join(msgs))
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    lib = engine.lib
    zseed = rnd.randbytes(32)
    p0, f0 = ctypes.create_string_buffer(128), ctypes.c_int(0)
    assert lib.edc_batch_partial_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                        d_off.data_ptr(), zseed, 0, None, p0, ctypes.byref(f0)) == 0
    bad_flag = 1 if kind in ("bad_R", "bad_s", "bad_A") else 0
    verdict = 0 if kind == "valid" else 1
    assert f0.value == bad_flag
    assert lib.edc_set_slots(engine.ctx, 16) == 0            # tickets 0, 1, 2, 3 -> slots 0, 1, 2, 3
    tickets = []
    for _ in range(4):          # four batches in flight at once: slot 0 (two streams) and slots 1-3 (one)
        t = lib.edc_batch_submit_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                        d_off.data_ptr(), zseed, 0, None, 0)
        assert t >= 0
        tickets.append(t)
    assert tickets == [0, 1, 2, 3]
    # partials are projective (X:Y:Z:T in the order the MSM summed): compare [8]*P compressed
    ref = engine.combine_partials([p0.raw], False)
    if bad_flag:
        assert p0.raw == IDENTITY_PARTIAL
    if kind == "valid":
        assert ref == (0, IDENTITY)
    elif kind == "wrong_msg":
        assert ref[0] == 1 and ref[1] != IDENTITY
    for t in tickets:
        p1, f1 = ctypes.create_string_buffer(128), ctypes.c_int(0)
        assert lib.edc_batch_wait(engine.ctx, t, None, p1, ctypes.byref(f1)) == verdict
        assert f1.value == bad_flag
        if bad_flag:
            assert p1.raw == p0.raw
        else:
            assert engine.combine_partials([p1.raw], False) == ref
    v = ctypes.create_string_buffer(n)
    cnt = ctypes.c_int(0)
    assert lib.edc_batch_verify_fallback_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                                d_off.data_ptr(), zseed, v, ctypes.byref(cnt), None) == verdict
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    assert lib.edc_verify_each_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                      d_off.data_ptr(), d_v.data_ptr()) == 0
    single = bytes(d_v.cpu().tolist())
    assert v.raw == single and cnt.value == sum(1 for x in single if x)


@pytest.mark.parametrize("b", [b for b in BATCHES if b["items"]], ids=lambda b: b["name"])
def test_golden_prehashed_indexed(engine, edc, b):
    """edc_batch_submit_prehashed_indexed: keys as positions in the registered list (100 B per item
    over PCIe) give the fixture's verdict and check8."""
    vks, sigs, _, ks = _items(b)
    zseed = bytes.fromhex(b["z_seed"])
    distinct = list(dict.fromkeys(vks))
    pos = {v: i for i, v in enumerate(distinct)}
    try:
        engine.keycache_load(distinct)
        t = engine.batch_submit_prehashed_indexed([pos[v] for v in vks], sigs, ks, zseed, want_check8=True)
        _check(b, *engine.batch_wait(t, want_check8=True))
        with pytest.raises(edc.EngineError, match="registered"):
            engine.batch_submit_prehashed_indexed([len(distinct)] + [0] * (len(vks) - 1), sigs, ks, zseed)
    finally:
        engine.keycache_clear()
