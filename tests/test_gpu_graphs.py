"""GPU: graph replays of pipelined submissions (edc_set_graphs; edc_api.hip "Graph replays").
Each slot captures its batch's launch sequence once and replays it while the shape stays the
same; the values that change per batch (key-hash salt, z seed, z base) travel in the slot's
parameter block. The same submissions with graphs off are the reference: verdict, bad flag,
check8 byte for byte and the partial as a point (reference src/batch.rs:149-217 once per batch;
the partial is the batch's check point, the identity when the bad flag is set).

Each sequence runs on three slots (slot 0, the synchronous calls' two-stream slot, always launches
directly), so the other two replay: the same inputs under new z seeds and z
bases (the parameter block), a copy of the inputs at other addresses and a shorter n (new
captures), a wrong signature and an undecodable R (rejections), and back. Shapes: vote batches
(150 validators, grouped keys), distinct keys (per-signature key terms once the context has seen
them), prehashed entries, and vote batches under the key cache (split coefficients)."""
import ctypes
import sys

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

UNDECODABLE = next(bytes.fromhex(c["enc"]) for c in golden("decode.json")["cases"] if not c["ok"])
SEEDS = [bytes([0x33]) * 32, bytes(range(32)), bytes([0xA5]) * 32]


@pytest.fixture(scope="module")
def env(edc):
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    return torch, bench, edc


def _workload(env, eng, n, keys, mlen):
    torch, bench, edc = env
    out = bench.make_workload(sys.modules["ed25519_consensus_amd"], eng, torch, torch.device("cuda:0"), n, keys, mlen, 0)
    torch.cuda.synchronize()
    return out


def _prehash(eng, vk, sig, msg, off, n):
    torch = sys.modules["torch"]
    o = (ctypes.c_uint64 * (n + 1)).from_buffer_copy((off[:n + 1] - off[0]).cpu().numpy().astype("uint64").tobytes())
    kb = ctypes.create_string_buffer(32 * n)
    eng._check(eng.lib.edc_challenge(eng.ctx, n, vk[:32 * n].cpu().numpy().tobytes(), sig[:64 * n].cpu().numpy().tobytes(),
                                     msg[int(off[0]):int(off[n])].cpu().numpy().tobytes() or b"\0", o, kb))
    return torch.frombuffer(bytearray(kb.raw), dtype=torch.uint8).to("cuda:0")


def _sequence(env, eng, n, keys, mlen, prehashed):
    """(n, vk, sig, msg, off, k, seed, zbase) submissions, all on the same engine"""
    torch = env[0]
    vk, sig, msg, off = _workload(env, eng, n, keys, mlen)
    k = _prehash(eng, vk, sig, msg, off, n) if prehashed else None
    vk2, sig2, msg2, off2 = vk.clone(), sig.clone(), msg.clone(), off.clone()   # other addresses
    k2 = k.clone() if k is not None else None
    bad_sig = sig.clone()                     # wrong signature: s of item 7 changed
    bad_sig[64 * 7 + 40] ^= 1
    bad_r = sig.clone()                       # undecodable R of item n - 2: the bad flag
    bad_r[64 * (n - 2):64 * (n - 2) + 32] = torch.tensor(list(UNDECODABLE), dtype=torch.uint8, device=sig.device)
    torch.cuda.synchronize()
    subs = []
    for i in range(6):                        # replays with new z seeds / bases
        subs.append((n, vk, sig, msg, off, k, SEEDS[i % 3], [0, 0, 12345, (1 << 40) + 3, 1, 77][i]))
    subs.append((n, vk2, sig2, msg2, off2, k2, SEEDS[0], 0))      # new capture (pointers)
    subs.append((n, vk, bad_sig, msg, off, k, SEEDS[1], 7))
    subs.append((n, vk, bad_sig, msg, off, k, SEEDS[2], 7))
    subs.append((n, vk, bad_r, msg, off, k, SEEDS[0], 0))
    subs.append((n - 2048, vk, sig, msg, off, k, SEEDS[0], 0))   # new capture (n)
    subs.append((n - 2048, vk, sig, msg, off, k, SEEDS[1], 99))
    subs.append((n, vk, sig, msg, off, k, SEEDS[2], 5))
    subs.append((n, vk, sig, msg, off, k, SEEDS[0], 0))
    subs.append((n, vk, sig, msg, off, k, SEEDS[1], 3))
    return subs, (vk, sig, msg, off, k, vk2, sig2, msg2, off2, k2, bad_sig, bad_r)


P = 2**255 - 19


def _same(a, b):
    """(rc, check8, partial, bad) of two runs: verdict, bad flag and check8 (a compressed, hence
    normalized, point) byte for byte; the partial is a projective X | Y | Z | T record whose scaling
    depends on the MSM plan the context's adaptive choices picked, so it is compared as a point"""
    if (a[0], a[1], a[3]) != (b[0], b[1], b[3]):
        return False
    x1, y1, z1, _ = (int.from_bytes(a[2][32 * i:32 * i + 32], "little") for i in range(4))
    x2, y2, z2, _ = (int.from_bytes(b[2][32 * i:32 * i + 32], "little") for i in range(4))
    return (x1 * z2 - x2 * z1) % P == 0 and (y1 * z2 - y2 * z1) % P == 0 and z1 % P and z2 % P


def _run(eng, subs, graphs, inflight=3, tickets=None):
    lib = eng.lib
    eng.set_graphs(graphs)
    out, pend = [], []

    def wait():
        t = pend.pop(0)
        c8 = ctypes.create_string_buffer(32)
        part = ctypes.create_string_buffer(128)
        bad = ctypes.c_int(0)
        rc = lib.edc_batch_wait(eng.ctx, t, c8, part, ctypes.byref(bad))
        assert rc >= 0, eng.lib.edc_last_error(eng.ctx)
        out.append((rc, c8.raw, part.raw, bad.value))

    for (n, vk, sig, msg, off, k, seed, zbase) in subs:
        if len(pend) >= inflight:
            wait()
        if k is None:
            t = lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                            seed, zbase, None, 1)
        else:
            t = lib.edc_batch_submit_prehashed_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), k.data_ptr(), seed,
                                                      zbase, None, 1)
        assert t >= 0, eng.lib.edc_last_error(eng.ctx)
        pend.append(t)
        if tickets is not None:
            tickets.append(t)
    while pend:
        wait()
    return out


@pytest.mark.parametrize("n,keys,mlen,prehashed,keycache", [
    (1 << 17, 150, 120, False, False),
    (8192 + 5, 0, 32, False, False),
    (1 << 17, 150, 120, True, False),
    (65536, 150, 120, False, True),
])
def test_graph_replays_equal_direct_launches(env, n, keys, mlen, prehashed, keycache):
    torch, bench, edc = env
    eng = edc.Engine(0)
    try:
        # three slots: slot 0 (the synchronous calls' two-stream slot) launches directly, slots 1
        # and 2 capture and replay
        eng._check(eng.lib.edc_set_slots(eng.ctx, 3))
        subs, keep = _sequence(env, eng, n, keys, mlen, prehashed)
        if keycache:
            vk = keep[0]
            kb = bytes(vk[:32 * keys].cpu().tolist())
            eng.keycache_load([kb[32 * i:32 * i + 32] for i in range(keys)])
        ref = _run(eng, subs, False)
        c0, r0 = eng.graph_stats()
        assert (c0, r0) == (0, 0)
        tickets = []
        got = _run(eng, subs, True, tickets=tickets)
        c1, r1 = eng.graph_stats()
        graphed = sum(1 for t in tickets if t % 3 != 0)
        assert c1 + r1 == graphed and r1 >= 2, (c1, r1, graphed)
        for i, (a, b) in enumerate(zip(ref, got)):
            assert _same(a, b), f"submission {i}: graphs off {a[0], a[3]} vs on {b[0], b[3]}"
        verdicts = [a[0] for a in ref]
        assert verdicts[:7] == [0] * 7 and verdicts[7:10] == [1, 1, 1] and verdicts[10:] == [0] * 5
        assert [a[3] for a in ref][9] == 1                # undecodable R: the bad flag
        # and once more with graphs on: graphs captured in the last run replay where the shapes meet
        again = _run(eng, subs, True)
        assert all(_same(a, b) for a, b in zip(again, got))
        c2, r2 = eng.graph_stats()
        assert r2 - r1 >= 2
    finally:
        eng.close()


def test_graph_replays_survive_slot_reallocation(env):
    """A larger batch reallocates a slot's buffers, which drops its graph: the next batch of the
    old shape is captured again against the new buffers (a stale replay would read freed memory)."""
    torch, bench, edc = env
    eng = edc.Engine(0)
    try:
        eng._check(eng.lib.edc_set_slots(eng.ctx, 2))
        eng.set_graphs(True)
        small = _workload(env, eng, 4096, 150, 120)
        big = _workload(env, eng, 1 << 16, 150, 120)
        # two slots alternate (slot 0 direct, slot 1 graphed): slot 1 captures and replays the small
        # shape, gets the large batch (reallocation, graph dropped), then captures the small again
        subs = [(4096,) + tuple(small) + (None, SEEDS[0], 0)] * 5 + [(1 << 16,) + tuple(big) + (None, SEEDS[0], 0)] + \
               [(4096,) + tuple(small) + (None, SEEDS[1], 3)] * 5
        got = _run(eng, subs, True, inflight=1)
        ref = _run(eng, subs, False, inflight=1)
        assert all(_same(a, b) for a, b in zip(got, ref))
        assert all(r[0] == 0 for r in got)
        assert eng.graph_stats() == (3, 2)
    finally:
        eng.close()
