"""GPU: the in-process multi-device C ABI (include/edc.h edc_create_multi, the drop-in for one
batch::Verifier::verify over all of a node's GPUs; reference src/batch.rs:149-217), rehearsed on
the one-GPU box with the same device listed several times (one context each). For every golden
batch and device list: verdict and compressed [8]*check equal the fixture (the single-device
result) bit-exactly, and the sharded fallback gives Item::verify_single's code for every item.
At configs[2]/[3] scale: a valid 2^20-vote batch is Ok with [8]*check = identity, and with the
ZIP215 corpus + one bad signature mixed in exactly the bad item is flagged."""
import json
import os
import sys

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

IDENTITY = bytes([1]) + bytes(31)


def _items(b):
    return [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]


@pytest.fixture(scope="module", params=[[0], [0, 0], [0, 0, 0], [0, 0, 0, 0]], ids=lambda d: f"dev{len(d)}")
def multi(edc, engine, request):
    m = edc.MultiEngine(request.param)
    yield m
    m.close()


@pytest.mark.parametrize("b", golden("batches.json")["batches"], ids=lambda b: b["name"])
def test_multi_batch_fixture(multi, b):
    it = _items(b)
    vks, sigs, msgs = [v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it]
    zs = bytes.fromhex(b["z_seed"])
    code, c8 = multi.batch_verify(vks, sigs, msgs, zs, want_check8=True)
    assert code == b["expect_code"]
    if b["expect_check8"] is not None:
        assert c8.hex() == b["expect_check8"]
    code, verdicts, cnt, c8 = multi.batch_verify_fallback(vks, sigs, msgs, zs)
    assert code == b["expect_code"]
    exp = b["expect_single"] if code else [0] * len(it)
    assert verdicts == exp and cnt == sum(1 for e in exp if e)


def test_multi_config3_scale(multi, engine):
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    n = 1 << 20
    fx = golden("zip215_small_order.json")
    pkg = sys.modules["ed25519_consensus_amd"]
    vk, sig, msg, off, expect, _ = bench.make_c4_workload(pkg, engine, torch, dev, n, 150, 120, fx["cases"],
                                                          bytes.fromhex(fx["msg"]))
    hv, hs, hm, ho = vk[:32 * n].cpu().numpy().tobytes(), sig[:64 * n].cpu().numpy().tobytes(), \
        msg.cpu().numpy().tobytes(), off.cpu().tolist()
    vks = [hv[32 * i:32 * i + 32] for i in range(n)]
    sigs = [hs[64 * i:64 * i + 64] for i in range(n)]
    msgs = [hm[ho[i]:ho[i + 1]] for i in range(n)]
    zs = bytes([0x33]) * 32
    code, verdicts, cnt, c8 = multi.batch_verify_fallback(vks, sigs, msgs, zs)
    assert code == 1 and cnt == len(expect)
    assert {i: v for i, v in enumerate(verdicts) if v} == expect
    bad = next(iter(expect))
    keep = [i for i in range(n) if i != bad]
    code, c8 = multi.batch_verify([vks[i] for i in keep], [sigs[i] for i in keep], [msgs[i] for i in keep], zs,
                                  want_check8=True)
    assert code == 0 and c8 == IDENTITY


@pytest.mark.parametrize("b", golden("batches.json")["batches"], ids=lambda b: b["name"])
def test_multi_submit_fixture(multi, b):
    """Pipelined multi-device form (edc_multi_submit / edc_multi_wait: shard partials copied
    device to device and combined on the first device): every golden batch, submitted twice and
    in flight together, gives the fixture's verdict and [8]*check."""
    it = _items(b)
    vks, sigs, msgs = [v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it]
    zs = bytes.fromhex(b["z_seed"])
    t1 = multi.batch_submit(vks, sigs, msgs, zs, want_check8=True)
    t2 = multi.batch_submit(vks, sigs, msgs, zs, want_check8=True)
    for t in (t1, t2):
        code, c8 = multi.batch_wait(t, want_check8=True)
        assert code == b["expect_code"]
        if b["expect_check8"] is not None:
            assert c8.hex() == b["expect_check8"]


def test_multi_routes_and_ring(multi, edc):
    """Every shard of a device list that repeats GPU 0 is routed locally; the multi ticket ring is
    the shard contexts' share of the GPU's 16 slots (16 / contexts): that many batches can be in
    flight, one more is refused cleanly (no shard slot is left half-submitted), and all verify."""
    G = len(multi.devices)
    assert [multi.route(i) for i in range(G)] == [0] * G
    b = [x for x in golden("batches.json")["batches"] if x["name"] == "batch_verify_one_bad"][0]
    it = _items(b)
    vks, sigs, msgs = [v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it]
    zs = bytes.fromhex(b["z_seed"])
    ring = 16 // G
    ts = [multi.batch_submit(vks, sigs, msgs, zs, want_check8=True) for _ in range(ring)]
    with pytest.raises(edc.EngineError, match="in flight"):
        multi.batch_submit(vks, sigs, msgs, zs)
    for t in ts:
        code, c8 = multi.batch_wait(t, want_check8=True)
        assert code == 1 and c8.hex() == b["expect_check8"]


@pytest.mark.parametrize("b", golden("batches.json")["batches"], ids=lambda b: b["name"])
def test_multi_submit_staged_route(multi, b):
    """The route a shard takes when its device has no peer access to the first device (forced):
    each shard's result block goes through its slot's pinned host mirror and a host-to-device copy
    on the combine stream. Every golden batch, twice in flight: the fixture's verdict and [8]*check."""
    multi.force_staged(True)
    try:
        assert all(multi.route(i) == 2 for i in range(len(multi.devices)))
        it = _items(b)
        vks, sigs, msgs = [v for v, _, _ in it], [s for _, s, _ in it], [m for _, _, m in it]
        zs = bytes.fromhex(b["z_seed"])
        t1 = multi.batch_submit(vks, sigs, msgs, zs, want_check8=True)
        t2 = multi.batch_submit(vks, sigs, msgs, zs, want_check8=True)
        for t in (t1, t2):
            code, c8 = multi.batch_wait(t, want_check8=True)
            assert code == b["expect_code"]
            if b["expect_check8"] is not None:
                assert c8.hex() == b["expect_check8"]
    finally:
        multi.force_staged(False)
    assert multi.route(0) == 0


def test_multi_submit_device_config3(multi, engine):
    """Device-resident pipelined form (edc_multi_submit_device) on configs[3] at 2^20: per-device
    slices of one batch (the ZIP215 corpus + one bad signature among 2^20 votes) -> Err, and the
    same batch without the bad item -> Ok with the identity, several batches in flight."""
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    n = 1 << 20
    fx = golden("zip215_small_order.json")
    pkg = sys.modules["ed25519_consensus_amd"]
    vk, sig, msg, off, expect, _ = bench.make_c4_workload(pkg, engine, torch, dev, n, 150, 120, fx["cases"],
                                                          bytes.fromhex(fx["msg"]))
    G = len(multi.devices)

    def shards(vk, sig, msg, off, n):
        out = []
        for g in range(G):
            lo, hi = n * g // G, n * (g + 1) // G
            o = (off[lo:hi + 1] - off[lo]).contiguous()
            keep.append(o)
            out.append((hi - lo, vk.data_ptr() + 32 * lo, sig.data_ptr() + 64 * lo,
                        msg.data_ptr() + int(off[lo].item()), o.data_ptr()))
        return out

    keep = []
    zs = bytes([0x33]) * 32
    t_bad = multi.batch_submit_device(shards(vk, sig, msg, off, n), zs, want_check8=True)
    # the batch without every item whose verify_single fails (re-packed on the device)
    idx = torch.tensor([i for i in range(n) if i not in expect], dtype=torch.int64, device=dev)
    vk2 = vk.view(-1, 32)[:n][idx].reshape(-1).contiguous()
    sig2 = sig.view(-1, 64)[:n][idx].reshape(-1).contiguous()
    lens = (off[1:] - off[:-1])[idx]
    off2 = torch.zeros(len(idx) + 1, dtype=torch.int64, device=dev)
    off2[1:] = torch.cumsum(lens, 0)
    cols = torch.arange(int(lens.max().item()), device=dev)[None, :]
    starts = off[:-1][idx]
    msg2 = torch.cat([msg[(starts[:, None] + cols)[cols < lens[:, None]]], torch.zeros(1, dtype=torch.uint8, device=dev)])
    n2 = len(idx)
    # two batches in flight per context at most (contexts sharing one GPU split its slots)
    sh2 = shards(vk2, sig2, msg2, off2, n2)
    t_ok = [multi.batch_submit_device(sh2, zs, want_check8=True)]
    code, _ = multi.batch_wait(t_bad, want_check8=True)
    assert code == 1
    t_ok.append(multi.batch_submit_device(sh2, zs, want_check8=True))
    for t in t_ok:
        code, c8 = multi.batch_wait(t, want_check8=True)
        assert code == 0 and c8 == IDENTITY
    # single-device reference of the same cleaned batch: same verdict
    rc = engine.lib.edc_batch_verify_device(engine.ctx, n2, vk2.data_ptr(), sig2.data_ptr(), msg2.data_ptr(),
                                            off2.data_ptr(), zs, 0, None, None)
    assert rc == 0

