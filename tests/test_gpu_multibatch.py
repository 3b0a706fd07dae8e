"""GPU: several consecutive batches in ONE launch sequence (edc_batch_submit_multi_device /
edc_batch_wait_multi). Batch b of nb (items [b n_per, (b+1) n_per) of one input, z drawn at global
indices z_base + b n_per + i) must give exactly what edc_batch_verify_device / _partial_device of
that batch alone gives: verdict, bad flag, compressed [8]*check (reference src/batch.rs:149-217,
once per batch); failing batches are also pinned to the C oracle. Covered: grouped keys (votes),
distinct keys (one key term per signature, by the host's choice and by the device's key-count
cap), the forced grouping overflow, undecodable R / non-canonical s / undecodable key in one
batch only, prehashed k, and full size (8 x 2^17 votes = 2^20). Each comparison runs in three
modes: union first (the default: the launch is verified as one batch and rerun batch by batch only
when that fails), batch by batch (edc_set_multi_union(0)), and union first with the per-batch
partials asked for (which reruns it batch by batch)."""
import ctypes
import os
import random
import sys

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

IDENTITY = bytes([1]) + bytes(31)
L_ORDER = 2**252 + 27742317777372353535851937790883648493


def _oc():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    return oracle_c


def _make(engine, torch, nb, n_per, keys, seed, spoil=()):
    """nb * n_per items signed by `keys` validators (0 = distinct); spoil: list of (index, kind)."""
    dev = torch.device("cuda:0")
    rnd = random.Random(seed)
    n = nb * n_per
    nk = keys or n
    seeds = [rnd.randbytes(32) for _ in range(nk)]
    msgs = [rnd.randbytes(rnd.randrange(0, 200)) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % nk for i in range(n)])
    vks, sigs = list(vks), list(sigs)
    dec_bad = [c for c in golden("decode.json")["cases"] if not c["ok"]]
    for i, kind in spoil:
        if kind == "msg":
            msgs[i] = msgs[i] + b"!"
        elif kind == "R":
            sigs[i] = bytes.fromhex(dec_bad[1]["enc"]) + sigs[i][32:]
        elif kind == "s":
            s = int.from_bytes(sigs[i][32:], "little") + L_ORDER
            sigs[i] = sigs[i][:32] + s.to_bytes(32, "little")
        elif kind == "A":
            vks[i] = bytes.fromhex(dec_bad[0]["enc"])
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    t8 = lambda b: torch.tensor(list(b) or [0], dtype=torch.uint8, device=dev)
    d = {"vk": t8(b"".join(vks)), "sig": t8(b"".join(sigs)), "msg": t8(b"".join(msgs)),
         "off": torch.tensor(offs, dtype=torch.int64, device=dev)}
    torch.cuda.synchronize()
    return vks, sigs, msgs, offs, d


def _single(engine, d, b, n_per, offs, zseed, z_base, torch):
    """batch b alone through the one-batch device entry: (code, check8, partial, bad)."""
    lo, hi = b * n_per, (b + 1) * n_per
    o = (d["off"][lo:hi + 1] - offs[lo]).contiguous()
    c8 = ctypes.create_string_buffer(32)
    code = engine.lib.edc_batch_verify_device(engine.ctx, n_per, d["vk"].data_ptr() + 32 * lo,
                                              d["sig"].data_ptr() + 64 * lo, d["msg"].data_ptr() + offs[lo],
                                              o.data_ptr(), zseed, z_base + lo, None, c8)
    part, bad = ctypes.create_string_buffer(128), ctypes.c_int(0)
    assert engine.lib.edc_batch_partial_device(engine.ctx, n_per, d["vk"].data_ptr() + 32 * lo,
                                               d["sig"].data_ptr() + 64 * lo, d["msg"].data_ptr() + offs[lo],
                                               o.data_ptr(), zseed, z_base + lo, None, part, ctypes.byref(bad)) == 0
    return code, c8.raw, part.raw, bad.value


def _multi(engine, d, nb, n_per, zseed, z_base, d_k=None, want_partials=False):
    t = engine.batch_submit_multi_device(nb, n_per, d["vk"].data_ptr(), d["sig"].data_ptr(),
                                         d["msg"].data_ptr() if d_k is None else None,
                                         d["off"].data_ptr() if d_k is None else None, zseed, z_base,
                                         d_k=d_k, want_check8=True)
    return engine.batch_wait_multi(t, nb, want_partials=want_partials)


@pytest.fixture(params=["union", "exact", "partials"])
def mode(request, engine):
    """union: union-first launches (default); exact: edc_set_multi_union(0); partials: union-first
    with the per-batch partials asked for at the wait (which reruns the launch batch by batch)."""
    engine.set_multi_union(request.param != "exact")
    yield request.param
    engine.set_multi_union(True)


def _check_against_single(engine, torch, d, nb, n_per, offs, zseed, z_base, res):
    code, verdicts, c8s, parts, bads = res
    for b in range(nb):
        sc, sc8, spart, sbad = _single(engine, d, b, n_per, offs, zseed, z_base, torch)
        assert verdicts[b] == sc, b
        assert bads[b] == sbad, b
        assert c8s[b] == sc8, b
        if not sbad and parts is not None:       # partials are projective: compare [8]*P of the two
            assert engine.combine_partials([parts[b]], 0) == engine.combine_partials([spart], 0), b
    assert code == (1 if any(verdicts) else 0)


@pytest.mark.parametrize("keys,grouping", [(20, 0), (0, 2), (0, 1), (20, 3)],
                         ids=["votes", "distinct_per_sig", "distinct_grouped_over_cap", "forced_overflow"])
def test_multi_equals_single_batches(engine, mode, keys, grouping):
    torch = pytest.importorskip("torch")
    nb, n_per = 4, 2048 if grouping != 1 else 4096          # 16,384 distinct keys > the 4,096 cap
    spoil = [(1 * n_per + 77, "msg"), (2 * n_per + 5, "R"), (3 * n_per + 1000, "s")]
    vks, sigs, msgs, offs, d = _make(engine, torch, nb, n_per, keys, seed=keys * 7 + grouping, spoil=spoil)
    engine.set_key_grouping(grouping)
    try:
        for z_base in (0, 12345):
            zseed = bytes([0x4D + z_base % 7]) * 32
            res = _multi(engine, d, nb, n_per, zseed, z_base, want_partials=mode == "partials")
            assert res[1] == [0, 1, 1, 1]
            assert res[4] == [0, 0, 1, 1]
            assert res[2][0] == IDENTITY
            _check_against_single(engine, torch, d, nb, n_per, offs, zseed, z_base, res)
    finally:
        engine.set_key_grouping(0)


def test_multi_failing_batch_vs_oracle(engine):
    """The non-identity check point of a failing batch inside a multi launch equals the C oracle's
    for that batch alone at its global z offset (reference src/batch.rs:205-216)."""
    torch = pytest.importorskip("torch")
    oc = _oc()
    nb, n_per = 3, 2048
    vks, sigs, msgs, offs, d = _make(engine, torch, nb, n_per, 16, seed=5, spoil=[(n_per + 9, "msg")])
    zseed = bytes([0x61]) * 32
    code, verdicts, c8s, _, _ = _multi(engine, d, nb, n_per, zseed, 0)
    assert verdicts == [0, 1, 0]
    lo, hi = n_per, 2 * n_per
    o = [x - offs[lo] for x in offs[lo:hi + 1]]
    oc_code, oc_c8, _ = oc.batch_verify_parallel(b"".join(vks[lo:hi]), b"".join(sigs[lo:hi]), b"".join(msgs[lo:hi]), o,
                                                 zseed, parts=4, z_base=lo)
    assert (oc_code, oc_c8) == (1, c8s[1])


def test_multi_undecodable_key_in_one_batch(engine, mode):
    torch = pytest.importorskip("torch")
    nb, n_per = 2, 2048
    vks, sigs, msgs, offs, d = _make(engine, torch, nb, n_per, 10, seed=9, spoil=[(n_per + 3, "A")])
    zseed = bytes([0x19]) * 32
    res = _multi(engine, d, nb, n_per, zseed, 0, want_partials=mode == "partials")
    assert res[1] == [0, 1] and res[4] == [0, 1]
    _check_against_single(engine, torch, d, nb, n_per, offs, zseed, 0, res)


def test_multi_union_first_counts(engine):
    """A valid launch passes as one union (no rerun, identity check8 for every batch); a launch
    with one failing batch is rerun batch by batch and reports that batch alone; asking for the
    partials reruns a valid launch too; with the union off nothing is counted."""
    torch = pytest.importorskip("torch")
    nb, n_per = 4, 2048
    vks, sigs, msgs, offs, d = _make(engine, torch, nb, n_per, 24, seed=77)
    zseed = bytes([0x5C]) * 32
    engine.set_multi_union(True)
    h0, r0 = engine.multi_union_stats()
    res = _multi(engine, d, nb, n_per, zseed, 0)
    assert res[0] == 0 and res[1] == [0] * nb and res[2] == [IDENTITY] * nb and res[4] == [0] * nb
    assert engine.multi_union_stats() == (h0 + 1, r0)
    _check_against_single(engine, torch, d, nb, n_per, offs, zseed, 0, res)
    res = _multi(engine, d, nb, n_per, zseed, 0, want_partials=True)
    assert engine.multi_union_stats() == (h0 + 1, r0 + 1)
    _check_against_single(engine, torch, d, nb, n_per, offs, zseed, 0, res)
    d["sig"][64 * (2 * n_per + 9) + 40] ^= 0x10
    torch.cuda.synchronize()
    res = _multi(engine, d, nb, n_per, zseed, 0)
    assert res[1] == [0, 0, 1, 0] and res[2][2] != IDENTITY
    assert engine.multi_union_stats() == (h0 + 1, r0 + 2)
    _check_against_single(engine, torch, d, nb, n_per, offs, zseed, 0, res)
    engine.set_multi_union(False)
    try:
        res = _multi(engine, d, nb, n_per, zseed, 0)
        assert res[1] == [0, 0, 1, 0]
        assert engine.multi_union_stats() == (h0 + 1, r0 + 2)
    finally:
        engine.set_multi_union(True)


def test_multi_prehashed(engine):
    torch = pytest.importorskip("torch")
    nb, n_per = 4, 2048
    vks, sigs, msgs, offs, d = _make(engine, torch, nb, n_per, 12, seed=21, spoil=[(2 * n_per + 44, "msg")])
    ks = engine.challenge(vks, sigs, msgs)
    d_k = torch.tensor(list(b"".join(ks)), dtype=torch.uint8, device=torch.device("cuda:0"))
    torch.cuda.synchronize()
    zseed = bytes([0x2E]) * 32
    ref = _multi(engine, d, nb, n_per, zseed, 0)
    pre = _multi(engine, d, nb, n_per, zseed, 0, d_k=d_k.data_ptr())
    assert pre[1] == ref[1] == [0, 0, 1, 0]
    assert pre[2] == ref[2]


def test_multi_full_size_votes_2_20(engine):
    """8 x 2^17 votes from 150 validators (2^20 items, the strong-scaling shard shape of configs[2]
    over 8 GPUs, 8 consecutive blocks at once): valid -> every batch Ok with the identity; one
    corrupted signature -> only its batch fails, with the check point of that batch alone."""
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    nb, n_per = 8, 1 << 17
    pkg = sys.modules["ed25519_consensus_amd"]
    vk, sig, msg, off = bench.make_workload(pkg, engine, torch, dev, nb * n_per, 150, 120, 0)
    torch.cuda.synchronize()
    d = {"vk": vk, "sig": sig, "msg": msg, "off": off}
    zseed = bytes([0x3A]) * 32
    for _ in range(2):                          # grouped, then with the few-keys plan
        code, verdicts, c8s, _, _ = _multi(engine, d, nb, n_per, zseed, 0)
        assert code == 0 and verdicts == [0] * nb and c8s == [IDENTITY] * nb
    sig[64 * (5 * n_per + 4242) + 40] ^= 0x02
    torch.cuda.synchronize()
    res = _multi(engine, d, nb, n_per, zseed, 0)
    assert res[1] == [0] * 5 + [1] + [0] * 2
    offs = [120 * i for i in range(nb * n_per + 1)]   # fixed 120-byte messages
    sc, sc8, _, _ = _single(engine, d, 5, n_per, offs, zseed, 0, torch)
    assert sc == 1 and sc8 == res[2][5]
    # and the C oracle on that batch alone at its global z offset (all host threads)
    oc = _oc()
    lo, hi = 5 * n_per, 6 * n_per
    hv = vk[32 * lo:32 * hi].cpu().numpy().tobytes()
    hs = sig[64 * lo:64 * hi].cpu().numpy().tobytes()
    hm = msg[120 * lo:120 * hi].cpu().numpy().tobytes()
    code, c8, secs = oc.batch_verify_parallel(hv, hs, hm, [120 * i for i in range(n_per + 1)], zseed, z_base=lo)
    print(f"\n[multibatch-oracle] 2^17 batch at z offset {lo}: oracle {secs:.2f} s, check8 {c8.hex()}")
    assert (code, c8) == (1, res[2][5])


def test_multi_argument_errors(engine, edc):
    torch = pytest.importorskip("torch")
    vks, sigs, msgs, offs, d = _make(engine, torch, 2, 2048, 4, seed=1)
    lib = engine.lib
    for nb, n_per in ((2, 1000), (17, 2048), (0, 2048)):
        t = lib.edc_batch_submit_multi_device(engine.ctx, nb, n_per, d["vk"].data_ptr(), d["sig"].data_ptr(),
                                              d["msg"].data_ptr(), d["off"].data_ptr(), None, bytes(32), 0, 0)
        assert t == -2
    t = engine.batch_submit_multi_device(2, 2048, d["vk"].data_ptr(), d["sig"].data_ptr(), d["msg"].data_ptr(),
                                         d["off"].data_ptr(), bytes(32))
    with pytest.raises(edc.EngineError):
        engine.batch_wait(t)                      # a multi ticket needs edc_batch_wait_multi
    with pytest.raises(edc.EngineError):
        engine.batch_wait_multi(t, 3)             # wrong batch count
    assert engine.batch_wait_multi(t, 2)[1] == [0, 0]


def test_multi_union_with_key_cache(engine):
    """Union-first launches on a context whose key cache holds the validators (the union then runs
    with split coefficients): the same per-batch results as single batches, valid and failing."""
    torch = pytest.importorskip("torch")
    nb, n_per = 4, 2048
    vks, sigs, msgs, offs, d = _make(engine, torch, nb, n_per, 30, seed=313, spoil=[(3 * n_per + 17, "msg")])
    zseed = bytes([0x7E]) * 32
    engine.set_multi_union(True)
    try:
        engine.keycache_load(list(dict.fromkeys(vks)))
        for _ in range(2):                            # the second launch plans split coefficients
            res = _multi(engine, d, nb, n_per, zseed, 0)
            assert res[1] == [0, 0, 0, 1]
            _check_against_single(engine, torch, d, nb, n_per, offs, zseed, 0, res)
        valid = _make(engine, torch, nb, n_per, 30, seed=313)[4]
        for _ in range(2):
            res = _multi(engine, valid, nb, n_per, zseed, 0)
            assert res[0] == 0 and res[2] == [IDENTITY] * nb
    finally:
        engine.keycache_clear()
