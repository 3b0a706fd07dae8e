"""GPU: edge cases of the round-2 entry points -- the fused batch + fallback call, the one-pass
grouped fallback, the multi-device context and the tuning knobs: empty and one-item batches,
every item invalid, many invalid items spread over all ranges (distinct keys: one key term per
signature), the forced grouping-overflow path under the fallback, more devices than items, and
argument errors. Per-item codes are checked against the per-item kernel (Item::verify_single,
reference src/batch.rs:104-107) and, where they are constructed, against the construction."""
import ctypes
import random

import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _dev(torch, b, dev):
    return torch.tensor(list(b) or [0], dtype=torch.uint8, device=dev)


def _upload(torch, vks, sigs, msgs, dev):
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    return (_dev(torch, b"".join(vks), dev), _dev(torch, b"".join(sigs), dev), _dev(torch, b"".join(msgs), dev),
            torch.tensor(offs, dtype=torch.int64, device=dev))


def _fused(engine, n, d, zseed):
    v = ctypes.create_string_buffer(max(n, 1))
    cnt = ctypes.c_int(-1)
    rc = engine.lib.edc_batch_verify_fallback_device(engine.ctx, n, d[0].data_ptr(), d[1].data_ptr(),
                                                     d[2].data_ptr(), d[3].data_ptr(), zseed, v, ctypes.byref(cnt),
                                                     None)
    return rc, list(v.raw[:n]), cnt.value


def _each(engine, torch, n, d, dev):
    out = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
    assert engine.lib.edc_verify_each_device(engine.ctx, n, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                             d[3].data_ptr(), out.data_ptr()) == 0
    return out[:n].cpu().tolist()


def test_fused_fallback_empty_and_single(engine):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    d = _upload(torch, [], [], [], dev)
    assert _fused(engine, 0, d, bytes(32)) == (0, [], 0)
    vks, sigs = engine.sign([bytes([9]) * 32], [b"one"])
    d = _upload(torch, vks, sigs, [b"one"], dev)
    assert _fused(engine, 1, d, bytes([1]) * 32) == (0, [0], 0)
    d = _upload(torch, vks, sigs, [b"onf"], dev)
    assert _fused(engine, 1, d, bytes([1]) * 32) == (1, [1], 1)
    bad_key = bytes.fromhex([c for c in golden("decode.json")["cases"] if not c["ok"]][0]["enc"])
    d = _upload(torch, [bad_key], sigs, [b"one"], dev)
    assert _fused(engine, 1, d, bytes([1]) * 32) == (1, [2], 1)


@pytest.mark.parametrize("keys", [37, 0])
def test_every_item_invalid(engine, keys):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    rnd = random.Random(keys + 1)
    n = 5000
    m = keys or n
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(40) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
    msgs = [x[:-1] + bytes([x[-1] ^ 0x80]) for x in msgs]     # every signature over another message
    d = _upload(torch, vks, sigs, msgs, dev)
    torch.cuda.synchronize()
    rc, got, cnt = _fused(engine, n, d, rnd.randbytes(32))
    assert rc == 1 and cnt == n and got == [1] * n
    v = ctypes.create_string_buffer(n)
    assert engine.lib.edc_find_invalid_device(engine.ctx, n, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                              d[3].data_ptr(), rnd.randbytes(32), 0, v) == n


@pytest.mark.parametrize("mode", [0, 2, 3])
def test_many_invalid_spread_over_ranges(engine, mode):
    """70 invalid items of several kinds at random positions of a 40,000-item batch with distinct keys
    (one key term per signature once auto grouping has seen distinct keys), under each grouping
    mode including the forced overflow path: fallback codes == per-item kernel codes."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    rnd = random.Random(300 + mode)
    n = 40000
    seeds = [rnd.randbytes(32) for _ in range(n)]
    msgs = [rnd.randbytes(rnd.randrange(0, 200)) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs)
    vks, sigs = list(vks), list(sigs)
    dec_bad = [bytes.fromhex(c["enc"]) for c in golden("decode.json")["cases"] if not c["ok"]]
    expect = {}
    for j, p in enumerate(rnd.sample(range(n), 70)):
        kind = j % 4
        if kind == 0:
            msgs[p] = msgs[p] + b"x"
            expect[p] = 1
        elif kind == 1:
            vks[p] = dec_bad[j % len(dec_bad)]
            expect[p] = 2
        elif kind == 2:
            sigs[p] = dec_bad[(j + 1) % len(dec_bad)] + sigs[p][32:]
            expect[p] = 1
        else:
            s = int.from_bytes(sigs[p][32:], "little") + 2**252 + 27742317777372353535851937790883648493
            sigs[p] = sigs[p][:32] + s.to_bytes(32, "little")
            expect[p] = 1
    d = _upload(torch, vks, sigs, msgs, dev)
    torch.cuda.synchronize()
    engine.set_key_grouping(mode)
    try:
        for _ in range(2):                                   # the second run sees the grouping hint
            rc, got, cnt = _fused(engine, n, d, rnd.randbytes(32))
            assert rc == 1 and cnt == len(expect)
            assert {i: c for i, c in enumerate(got) if c} == expect
    finally:
        engine.set_key_grouping(0)
    assert {i: c for i, c in enumerate(_each(engine, torch, n, d, dev)) if c} == expect


def test_multi_more_devices_than_items_and_bad_args(edc, engine):
    lib = engine.lib
    assert not lib.edc_create_multi((ctypes.c_int * 1)(99), 1)           # no such device
    assert not lib.edc_create_multi((ctypes.c_int * 1)(0), 0)
    m = edc.MultiEngine([0, 0, 0, 0, 0])
    try:
        vks, sigs = engine.sign([bytes([3]) * 32, bytes([4]) * 32], [b"a", b"b"])
        assert m.batch_verify(vks, sigs, [b"a", b"b"], bytes([2]) * 32)[0] == 0
        code, v, cnt, _ = m.batch_verify_fallback(vks, sigs, [b"a", b"c"], bytes([2]) * 32)
        assert (code, v, cnt) == (1, [0, 1], 1)
        assert m.batch_verify([], [], [], bytes(32))[0] == 0
    finally:
        m.close()
    assert lib.edc_set_msm_shape(engine.ctx, 17, 0) < 0
    assert lib.edc_set_msm_shape(engine.ctx, 12, 65) < 0
    assert lib.edc_set_fallback_shape(engine.ctx, 0, 10) < 0
    assert lib.edc_set_key_grouping(engine.ctx, 4) < 0


def test_device_chacha_two_block_known_answer(engine):
    """The device ChaCha20 (z stream, synthetic data) against the published zero-key blocks 0 and
    1 of the original 64-bit-counter layout (rand_chacha's ChaCha20Rng), and a block past 2^32
    against the oracle (the counter's high word)."""
    torch = pytest.importorskip("torch")
    import os
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ed25519_ref as oracle
    from test_oracle_golden import CHACHA20_ZERO_KEY_BLOCKS_0_1
    dev = torch.device("cuda:0")
    out = torch.zeros(128, dtype=torch.uint8, device=dev)
    assert engine.lib.edc_chacha_fill_device(engine.ctx, bytes(32), 0, 2, out.data_ptr()) == 0
    assert bytes(out.cpu().tolist()).hex() == CHACHA20_ZERO_KEY_BLOCKS_0_1
    key = bytes(range(32))
    blk = (1 << 32) + 5
    assert engine.lib.edc_chacha_fill_device(engine.ctx, key, blk, 2, out.data_ptr()) == 0
    assert bytes(out.cpu().tolist()) == oracle.chacha20_keystream(key, 128, blk)


def test_timing_report_and_accum_counts(edc):
    """edc_set_timing / edc_last_timings / edc_last_msm_accum (the bench's phase times and the
    accumulation's own roofline): an error before any timed batch, then the phase names, positive
    durations, and a digit-entry count within what the plan can add (at most one entry per term
    and window: 2n + 1 terms over at most 29 windows for a small distinct-key batch)."""
    import ctypes
    eng = edc.Engine(0)
    try:
        lib = eng.lib
        ms, ent = ctypes.c_float(0), ctypes.c_uint64(0)
        assert lib.edc_last_msm_accum(eng.ctx, ctypes.byref(ms), ctypes.byref(ent)) < 0
        rnd = __import__("random").Random(5)
        n = 64
        seeds = [rnd.randbytes(32) for _ in range(n)]
        msgs = [rnd.randbytes(40) for _ in range(n)]
        vks, sigs = eng.sign(seeds, msgs)
        lib.edc_set_timing(eng.ctx, 1)
        code, _ = eng.batch_verify(vks, sigs, msgs, z_seed=bytes(32))
        assert code == 0
        names = [lib.edc_timing_name(i).decode() for i in range(7)]
        assert "decompress_R" in names and "challenge_sha512" in names
        buf = (ctypes.c_float * 7)()
        assert lib.edc_last_timings(eng.ctx, buf, 7) == 7 and all(x >= 0 for x in buf)
        assert lib.edc_last_msm_accum(eng.ctx, ctypes.byref(ms), ctypes.byref(ent)) == 0
        assert ms.value > 0
        assert ent.value > 0 and ent.value <= (n + n + 1) * 29
    finally:
        eng.close()
