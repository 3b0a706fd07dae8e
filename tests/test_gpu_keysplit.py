"""GPU: split coefficients with the validator-key cache (include/edc.h edc_set_key_split,
edc_common.h msm_num_points_split). Each 253-bit B / key coefficient is evaluated as
lo + 2^128 hi on the point and on its cached [2^128] multiple; the MSM (src/batch.rs:205-210) is the
same group element, so the verdict and the compressed [8]*check must equal the unsplit evaluation's
and the C oracle's bit for bit -- for grouped, per-signature and overflowed key grouping, small and
large batches, valid and corrupted ones, and for batches holding keys missing from the cache (the
device doubles those 128 times; the host stops splitting until a batch finds every key again).
Randomized shapes (test_random_split_vs_oracle): 4 cases by default, EDC_SPLIT_SOAK=<k> for a soak."""
import os
import random

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


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
    engine.set_key_split(0)
    engine.set_key_grouping(0)


def _batch(engine, rnd, n, m, msg_len=64):
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(msg_len) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
    return list(vks), list(sigs), msgs


@pytest.mark.parametrize("n,m,grouping,bad", [(1 << 14, 150, 0, None), (1 << 14, 150, 0, 777), (150, 150, 0, None),
                                              (150, 150, 0, 3), (4096, 4096, 2, None), (4096, 64, 3, 4000),
                                              (64, 1, 0, None)])
def test_split_matches_unsplit_and_oracle(cached, oracle_c, n, m, grouping, bad):
    rnd = random.Random(n * 31 + m + grouping)
    vks, sigs, msgs = _batch(cached, rnd, n, m)
    if bad is not None:
        msgs[bad] = msgs[bad][:-1] + bytes([msgs[bad][-1] ^ 1])
    zseed = rnd.randbytes(32)
    exp = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    assert exp[0] == (0 if bad is None else 1)
    cached.set_key_grouping(grouping)
    u, ok = cached.keycache_load(list(dict.fromkeys(vks)))
    assert all(ok)
    split = cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    cached.set_key_split(1)
    unsplit = cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    assert split == unsplit == exp


def test_split_with_uncached_keys_sequence(cached, oracle_c):
    """all cached (split) -> one unregistered key (split, doubled on the device) -> all cached
    again (unsplit, the previous batch missed a key) -> all cached (split again): every verdict
    and [8]*check equals the oracle's."""
    rnd = random.Random(2024)
    n, m = 8192, 150
    vks, sigs, msgs = _batch(cached, rnd, n, m)
    reg = list(dict.fromkeys(vks))
    cached.keycache_load(reg[1:])                       # key 0 (items 0, 150, 300, ...) unregistered
    other = [i for i in range(n) if i % m != 0]
    cached_only = ([vks[i] for i in other], [sigs[i] for i in other], [msgs[i] for i in other])
    stranger = _batch(cached, rnd, 3, 1)
    mixed = (cached_only[0][:4000] + stranger[0], cached_only[1][:4000] + stranger[1],
             cached_only[2][:4000] + stranger[2])
    for step, (v, s, mm) in enumerate([cached_only, mixed, cached_only, cached_only, mixed]):
        zseed = bytes([step + 1]) * 32
        exp = oracle_c.batch_verify(list(zip(v, s, mm)), zseed)
        assert exp[0] == 0
        assert cached.batch_verify(v, s, mm, z_seed=zseed, want_check8=True) == exp, step
    # a corrupted signature next to an unregistered key
    v, s, mm = mixed
    mm = list(mm)
    mm[10] = mm[10][:-1] + bytes([mm[10][-1] ^ 1])
    zseed = bytes([9]) * 32
    exp = oracle_c.batch_verify(list(zip(v, s, mm)), zseed)
    assert exp[0] == 1
    assert cached.batch_verify(v, s, mm, z_seed=zseed, want_check8=True) == exp


def test_split_in_flight_batches(cached, oracle_c):
    """submit/wait with several batches in flight on the split plan (device-resident inputs)."""
    torch = pytest.importorskip("torch")
    import ctypes
    dev = torch.device("cuda:0")
    rnd = random.Random(77)
    n, m = 1 << 13, 100
    vks, sigs, msgs = _batch(cached, rnd, n, m, msg_len=120)
    cached.keycache_load(list(dict.fromkeys(vks)))
    d_vk = torch.tensor(list(b"".join(vks)), dtype=torch.uint8, device=dev)
    d_sig = torch.tensor(list(b"".join(sigs)), dtype=torch.uint8, device=dev)
    d_msg = torch.tensor(list(b"".join(msgs)), dtype=torch.uint8, device=dev)
    d_off = torch.arange(0, n + 1, dtype=torch.int64, device=dev) * 120
    torch.cuda.synchronize()
    lib = cached.lib
    tickets, expect = [], []
    for b in range(6):
        zseed = bytes([0x40 + b]) * 32
        t = lib.edc_batch_submit_device(cached.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                        d_off.data_ptr(), zseed, 0, None, 1)
        assert t >= 0
        tickets.append(t)
        expect.append(oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed))
    for t, exp in zip(tickets, expect):
        c8 = ctypes.create_string_buffer(32)
        rc = lib.edc_batch_wait(cached.ctx, t, c8, None, None)
        assert (rc, c8.raw) == exp


@pytest.mark.parametrize("register", ["all", "validators"])
def test_split_batch_then_grouped_fallback(cached, register):
    """configs[3] shape on the split plan: the corpus, a forged signature, an undecodable key,
    R and s; batch + grouped fallback in one call (which reuses the split batch's points and
    sums) gives Item::verify_single's code for every item, twice in a row."""
    torch = pytest.importorskip("torch")
    import ctypes
    from conftest import golden
    dev = torch.device("cuda:0")
    L_ORDER = 2**252 + 27742317777372353535851937790883648493
    rnd = random.Random(31337)
    n, keys = 1 << 14, 150
    vks, sigs, msgs = _batch(cached, rnd, n, keys)
    validators = list(dict.fromkeys(vks))
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
    cached.keycache_load(list(dict.fromkeys(vks)) if register == "all" else validators)
    offs = [0]
    for mm in msgs:
        offs.append(offs[-1] + len(mm))

    def _dev(b):
        return torch.tensor(list(b) or [0], dtype=torch.uint8, device=dev)
    d_vk, d_sig, d_msg = _dev(b"".join(vks)), _dev(b"".join(sigs)), _dev(b"".join(msgs))
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    for rep in range(2):
        v = ctypes.create_string_buffer(n)
        cnt = ctypes.c_int(-1)
        rc = cached.lib.edc_batch_verify_fallback_device(cached.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(),
                                                         d_msg.data_ptr(), d_off.data_ptr(), bytes([rep + 3]) * 32,
                                                         v, ctypes.byref(cnt), None)
        assert rc == 1 and cnt.value == 4 and list(v.raw) == expect, rep


SPLIT_SOAK = int(os.environ.get("EDC_SPLIT_SOAK", "0"))


@pytest.mark.parametrize("case", range(SPLIT_SOAK or 4))
def test_random_split_vs_oracle(cached, oracle_c, case):
    """random n, key count, grouping mode, window shape and message length; all keys cached, or a
    random part of them (the device doubles the missing ones 128 times); then the same batch
    unsplit. Verdict and [8]*check equal the C oracle's each time."""
    rnd = random.Random(8080 + case)
    n = rnd.choice([rnd.randrange(1, 400), rnd.randrange(400, 6000), rnd.randrange(6000, 30000)])
    m = rnd.choice([1, rnd.randrange(1, 300), max(1, n // rnd.choice([1, 3, 40]))])
    grouping = rnd.choice([0, 0, 1, 2, 3])
    bits, parts = rnd.choice([(0, 0), (0, 0), (12, 1), (16, 1), (11, 4), (14, 2)])
    vks, sigs, msgs = _batch(cached, rnd, n, m, msg_len=rnd.randrange(1, 200))
    bad = rnd.choice([None, rnd.randrange(n)])
    if bad is not None:
        msgs[bad] = msgs[bad][:-1] + bytes([msgs[bad][-1] ^ 1])
    zseed = rnd.randbytes(32)
    exp = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    keys = list(dict.fromkeys(vks))
    if rnd.random() < 0.4 and len(keys) > 1:
        keys = rnd.sample(keys, rnd.randrange(1, len(keys)))
    cached.set_key_grouping(grouping)
    cached.set_msm_shape(bits, parts)
    tag = (case, n, m, grouping, bits, parts, bad, len(keys))
    try:
        _, ok = cached.keycache_load(keys)
        assert all(ok)
        for _ in range(2):       # the second run plans from the first one's key counts
            assert cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True) == exp, tag
        cached.set_key_split(1)
        assert cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True) == exp, tag
    finally:
        cached.set_msm_shape(0, 0)
