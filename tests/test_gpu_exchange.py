"""GPU: the multi-rank exchange of bench.py (sharded.ExchangeRing) and its device-side combine
(edc_combine_records_device). Records are the 129-byte exchange format (canonical partial point
+ bad byte) in device memory; the combine is enqueued on the caller's stream behind the
collective. Checked against edc_combine_partials (host buffers) and the golden fixtures' verdicts
and [8]*check (tests/golden/batches.json), with 1-5 shards at global z offsets (reference
src/batch.rs:189-216: the batch equation is linear in the items)."""
import ctypes
import os
import socket

import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

BATCHES = [b for b in golden("batches.json")["batches"] if b["items"]]


def _partials(engine, torch, b, nshards):
    dev = torch.device("cuda:0")
    items = b["items"]
    zseed = bytes.fromhex(b["z_seed"])
    recs = []
    for s in range(nshards):
        lo, hi = len(items) * s // nshards, len(items) * (s + 1) // nshards
        mine = items[lo:hi]
        vk = torch.tensor(list(b"".join(bytes.fromhex(v) for v, _, _ in mine)) or [0], dtype=torch.uint8, device=dev)
        sg = torch.tensor(list(b"".join(bytes.fromhex(x) for _, x, _ in mine)) or [0], dtype=torch.uint8, device=dev)
        msgs = [bytes.fromhex(m) for _, _, m in mine]
        mm = torch.tensor(list(b"".join(msgs)) or [0], dtype=torch.uint8, device=dev)
        offs = [0]
        for m in msgs:
            offs.append(offs[-1] + len(m))
        off = torch.tensor(offs, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        part = ctypes.create_string_buffer(128)
        bad = ctypes.c_int(0)
        assert engine.lib.edc_batch_partial_device(engine.ctx, len(mine), vk.data_ptr(), sg.data_ptr(), mm.data_ptr(),
                                                   off.data_ptr(), zseed, lo, None, part, ctypes.byref(bad)) == 0
        recs.append(part.raw + bytes([1 if bad.value else 0]))
    return recs


@pytest.mark.parametrize("b", BATCHES, ids=lambda b: b["name"])
def test_combine_records_device(engine, b):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    for nshards in (1, 3, 5):
        recs = _partials(engine, torch, b, nshards)
        d_rec = torch.tensor(list(b"".join(recs)), dtype=torch.uint8, device=dev)
        d_out = torch.zeros(256, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream()
        engine.combine_records_device(st.cuda_stream, nshards, d_rec.data_ptr(), 129, d_out.data_ptr())
        st.synchronize()
        blk = bytes(d_out.cpu().tolist())
        verdict, bad = int.from_bytes(blk[:4], "little"), int.from_bytes(blk[4:8], "little")
        host = engine.combine_partials([r[:128] for r in recs], any(r[128] for r in recs))
        assert (1 if verdict else 0) == host[0] == b["expect_code"], b["name"]
        assert bad == (1 if any(r[128] for r in recs) else 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("group", [1, 3])
def test_exchange_ring_rccl_single_rank(engine, group):
    """ExchangeRing over a one-rank RCCL group with the device combine: several exchanges in
    flight (one record or `group` records per all-gather), completed in order, each giving its
    batch's fixture verdict."""
    torch = pytest.importorskip("torch")
    import torch.distributed as dist
    from conftest import load_pkg
    load_pkg()
    from importlib import import_module
    sharded = import_module("ed25519_consensus_amd.sharded")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        dev = torch.device("cuda:0")
        ring = sharded.ExchangeRing(dist, dev, depth=3, device_combine=engine, group=group)
        assert ring.combines
        stream = [BATCHES[i % len(BATCHES)] for i in range(2 * len(BATCHES))]
        recs = {id(b): _partials(engine, torch, b, 1)[0] for b in BATCHES}
        got = []
        for b in stream:
            ring.post(recs[id(b)])
            while len(ring) > 2:
                got.append(ring.pop())
        while len(ring):
            got.append(ring.pop())
        assert [1 if g else 0 for g in got] == [b["expect_code"] for b in stream]
    finally:
        dist.destroy_process_group()


def test_combine_records_device_arguments(engine):
    """Argument errors are errors, never a verdict: a stride below the 129-byte record, more than
    4,096 records, a missing or misaligned output."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    d = torch.zeros(4096, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    lib, ctx = engine.lib, engine.ctx
    rec, out = d.data_ptr(), d.data_ptr() + 2048
    assert lib.edc_combine_records_device(ctx, ctypes.c_void_p(st), 1, ctypes.c_void_p(rec), 128, ctypes.c_void_p(out)) < 0
    assert lib.edc_combine_records_device(ctx, ctypes.c_void_p(st), 4097, ctypes.c_void_p(rec), 129, ctypes.c_void_p(out)) < 0
    assert lib.edc_combine_records_device(ctx, ctypes.c_void_p(st), 1, ctypes.c_void_p(rec), 129, None) < 0
    assert lib.edc_combine_records_device(ctx, ctypes.c_void_p(st), 1, None, 129, ctypes.c_void_p(out)) < 0
    assert lib.edc_combine_records_device(ctx, ctypes.c_void_p(st), 1, ctypes.c_void_p(rec), 129,
                                          ctypes.c_void_p(out + 4)) < 0
    torch.cuda.synchronize()
