"""GPU: BASELINE configs[3] shape -- the ZIP215 small-order corpus (tests/small_order.rs:12-77) mixed
into a large batch of votes together with invalid items of every kind. The batch must fail;
the grouped fallback (edc_find_invalid_device, bisection on partial check points) must return,
for EVERY item, exactly the verdict of Item::verify_single (src/batch.rs:104-107) as computed one
by one by the per-signature kernel (edc_verify_each_device): the corpus items valid, the bad
signature InvalidSignature, an undecodable key MalformedPublicKey, an undecodable R and a
non-canonical s InvalidSignature. Per-item codes of the corpus and of the hand-made invalid
items are pinned by the golden fixtures / by construction."""
import random

import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

L_ORDER = 2**252 + 27742317777372353535851937790883648493


def _dev(torch, b, dev):
    return torch.tensor(list(b) or [0], dtype=torch.uint8, device=dev)


@pytest.mark.parametrize("n,keys", [(1 << 16, 150), (40000, 40000)])
def test_corpus_mixed_batch_grouped_fallback(engine, n, keys):
    torch = pytest.importorskip("torch")
    import ctypes
    dev = torch.device("cuda:0")
    rnd = random.Random(n + keys)
    seeds = [rnd.randbytes(32) for _ in range(keys)]
    msgs = [rnd.randbytes(64) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % keys for i in range(n)])
    vks, sigs = list(vks), list(sigs)
    expect = [0] * n
    # the 196 corpus cases at seeded positions (all valid under ZIP215)
    fx = golden("zip215_small_order.json")
    pos = rnd.sample(range(n), len(fx["cases"]) + 4)
    for p, c in zip(pos, fx["cases"]):
        vks[p], sigs[p], msgs[p] = bytes.fromhex(c["vk"]), bytes.fromhex(c["sig"]), bytes.fromhex(fx["msg"])
        expect[p] = c["expect_single"]
    p_bad, p_A, p_R, p_s = pos[-4:]
    msgs[p_bad] = msgs[p_bad][:-1] + bytes([msgs[p_bad][-1] ^ 1])          # signed another message
    expect[p_bad] = 1
    dec = [c for c in golden("decode.json")["cases"] if not c["ok"]]
    vks[p_A] = bytes.fromhex(dec[0]["enc"])                                  # key not on the curve
    expect[p_A] = 2
    sigs[p_R] = bytes.fromhex(dec[1]["enc"]) + sigs[p_R][32:]               # R not on the curve
    expect[p_R] = 1
    s = int.from_bytes(sigs[p_s][32:], "little") + L_ORDER                  # s + l: same point, s >= l
    sigs[p_s] = sigs[p_s][:32] + s.to_bytes(32, "little")
    expect[p_s] = 1

    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    d_vk, d_sig, d_msg = _dev(torch, b"".join(vks), dev), _dev(torch, b"".join(sigs), dev), _dev(torch, b"".join(msgs), dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    zseed = rnd.randbytes(32)
    lib = engine.lib
    rc = lib.edc_batch_verify_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                     d_off.data_ptr(), zseed, 0, None, None)
    assert rc == 1
    verdicts = ctypes.create_string_buffer(n)
    nbad = lib.edc_find_invalid_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                       d_off.data_ptr(), zseed, 4096, verdicts)
    got = list(verdicts.raw)
    d_ver = torch.zeros(n, dtype=torch.uint8, device=dev)
    assert lib.edc_verify_each_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                      d_off.data_ptr(), d_ver.data_ptr()) == 0
    each = d_ver.cpu().tolist()
    assert each == expect
    assert got == expect
    assert nbad == 4
    # batch + fallback in one call (reuses the failed batch's k, points and grouping)
    v2 = ctypes.create_string_buffer(n)
    cnt = ctypes.c_int(-1)
    rc = lib.edc_batch_verify_fallback_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                              d_off.data_ptr(), zseed, v2, ctypes.byref(cnt), None)
    assert rc == 1 and cnt.value == 4 and list(v2.raw) == expect
    # and the valid remainder (bad items removed) verifies as one batch
    keep = [i for i in range(n) if expect[i] == 0]
    code, c8 = engine.batch_verify([vks[i] for i in keep], [sigs[i] for i in keep], [msgs[i] for i in keep],
                                   z_seed=zseed, want_check8=True)
    assert code == 0 and c8 == bytes([1]) + bytes(31)


def test_sharded_fallback_on_one_gpu(engine):
    """sharded.find_invalid_sharded with 4 shards on one GPU: each shard's partial
    (edc_batch_partial_device at its global z offset) alone decides whether the shard holds an
    invalid item; only failing shards run edc_find_invalid_device on their slice; the gathered
    global indices and codes equal Item::verify_single's."""
    torch = pytest.importorskip("torch")
    import ctypes
    from importlib import import_module
    sharded = import_module("ed25519_consensus_amd.sharded")
    dev = torch.device("cuda:0")
    rnd = random.Random(2024)
    n, keys, world = 20000, 50, 4
    seeds = [rnd.randbytes(32) for _ in range(keys)]
    msgs = [rnd.randbytes(rnd.randrange(0, 300)) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % keys for i in range(n)])
    expect = {}
    for p in (123, 5001, 5002):                                   # shards 0 and 1; 2 and 3 clean
        msgs[p] = msgs[p] + b"!"
        expect[p] = 1
    dec = [c for c in golden("decode.json")["cases"] if not c["ok"]]
    vks[19999] = bytes.fromhex(dec[0]["enc"])                     # shard 3: undecodable key
    expect[19999] = 2
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    d_vk, d_sig, d_msg = _dev(torch, b"".join(vks), dev), _dev(torch, b"".join(sigs), dev), _dev(torch, b"".join(msgs), dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    zseed = rnd.randbytes(32)
    lib = engine.lib
    found = []
    bounds = sharded.shard_bounds(n, world)
    for rank, (lo, hi) in enumerate(bounds):
        m = hi - lo
        args = (d_vk.data_ptr() + 32 * lo, d_sig.data_ptr() + 64 * lo, d_msg.data_ptr(), d_off.data_ptr() + 8 * lo)

        def shard_ok():
            part = ctypes.create_string_buffer(128)
            bad = ctypes.c_int(0)
            assert lib.edc_batch_partial_device(engine.ctx, m, *args, zseed, lo, None, part, ctypes.byref(bad)) == 0
            return engine.combine_partials([part.raw], bad.value, want_check8=False)[0] == 0

        def find():
            v = ctypes.create_string_buffer(m)
            assert lib.edc_find_invalid_device(engine.ctx, m, *args, zseed, 1024, v) >= 0
            return [(i, c) for i, c in enumerate(v.raw) if c]

        found.append(sharded.find_invalid_sharded(shard_ok, find, lambda obj: [obj], 0, 1, lo))
    assert sorted(x for f in found for x in f) == sorted(expect.items())
    assert found[2] == []
