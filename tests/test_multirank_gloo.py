"""CPU, world_size 2 / 4 / 8 over gloo: the multi-GPU orchestration of bench.py / sharded.py --
contiguous queue slices, global z offsets, a 129-byte all-gather per rank and the combine --
reproduces the unsharded verdict and [8]*check, one batch at a time and as bench.py's pipelined
stream (asynchronous exchange ring, several batches and all-gathers in flight). The per-rank partial is computed by the C
oracle here (no GPU); on MI355X the same driver calls edc_batch_partial_device and RCCL."""
import json
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

from conftest import ROOT, golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, out_path):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_c
    from conftest import load_pkg
    load_pkg()
    from importlib import import_module
    sharded = import_module("ed25519_consensus_amd.sharded")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
    items = [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]
    seed = bytes.fromhex(b["z_seed"])
    lo, hi = sharded.shard_bounds(len(items), world)[rank]

    def partial(zbase):
        part, bad = oracle_c.shard_partial_affine(items[lo:hi], seed, zbase)
        return part + bytes(64), bad          # pad the 64-byte affine record to 128

    allgather = sharded.torch_allgather_fn(dist, torch.device("cpu"))   # bench.py's gloo all-gather

    def combine(parts, bad_any):
        code, c8 = oracle_c.combine_affine([p[:64] for p in parts])
        return (1 if bad_any else code), (None if bad_any else c8)

    code, c8 = sharded.verify_sharded(partial, combine, allgather, rank, world, lo)
    with open(out_path + f".{rank}", "w") as f:
        json.dump({"code": code, "check8": c8.hex() if c8 else None}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("mixed_corpus_one_bad", 2), ("repeated_keys_varlen", 2), ("undecodable_R", 2),
                                        ("mixed_corpus_one_bad", 4), ("repeated_keys_varlen", 8)])
def test_two_rank_sharded_verify(tmp_path, name, world):
    """world_size 2 (and 4 / 8 ranks, the driver's scaling shapes) over gloo."""
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _free_port(), name, out), nprocs=world, join=True,
                       start_method="spawn")
    b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
    for r in range(world):
        res = json.load(open(out + f".{r}"))
        assert res["code"] == b["expect_code"]
        assert res["check8"] == b["expect_check8"]


STREAM = ["mixed_corpus_one_bad", "repeated_keys_varlen", "undecodable_R", "batch_verify_32", "two_bad_of_300",
          "repeated_keys_varlen", "mixed_corpus_one_bad"]


def _stream_worker(rank, world, port, inflight, lag, group, out_path):
    """bench.py's multi-rank loop (sharded.run_sharded_stream + ExchangeRing over gloo): a stream of
    golden batches, `inflight` submitted ahead, `lag` all-gathers in flight; the oracle computes
    each rank's partial where the GPU runs edc_batch_wait(partial)."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_c
    from conftest import load_pkg
    load_pkg()
    from importlib import import_module
    sharded = import_module("ed25519_consensus_amd.sharded")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gold = {x["name"]: x for x in golden("batches.json")["batches"]}
    submitted, log = [], []

    def submit():
        j = len(submitted)
        submitted.append(j)
        log.append(("submit", j))
        return j

    def wait(j):
        b = gold[STREAM[j]]
        items = [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]
        lo, hi = sharded.shard_bounds(len(items), world)[rank]
        part, bad = oracle_c.shard_partial_affine(items[lo:hi], bytes.fromhex(b["z_seed"]), lo)
        log.append(("wait", j))
        return part + bytes(64), bad

    def combine(parts, bad_any):
        code, _ = oracle_c.combine_affine([p[:64] for p in parts])
        return 1 if bad_any else code

    ring = sharded.ExchangeRing(dist, torch.device("cpu"), depth=lag, group=group)
    codes = sharded.run_sharded_stream(len(STREAM), inflight, submit, wait, combine, ring, lag)
    with open(out_path + f".{rank}", "w") as f:
        json.dump({"codes": codes, "log": log}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,inflight,lag,group", [(2, 1, 1, 1), (4, 3, 2, 1), (8, 4, 3, 1), (4, 3, 5, 2),
                                                     (8, 4, 8, 3)])
def test_stream_loop_in_order(tmp_path, world, inflight, lag, group):
    """The multi-rank loop of bench.py at 2 / 4 / 8 ranks with several batches and exchanges in
    flight, one record or a group of records per all-gather (partial groups flushed when the
    oldest verdict is needed): every rank gets every batch's unsharded verdict, in batch order; a
    batch is submitted up to `inflight` ahead of its collection (the refill precedes the
    exchange)."""
    out = str(tmp_path / "stream")
    mp.start_processes(_stream_worker, args=(world, _free_port(), inflight, lag, group, out), nprocs=world, join=True,
                       start_method="spawn")
    gold = {x["name"]: x for x in golden("batches.json")["batches"]}
    expect = [gold[nm]["expect_code"] for nm in STREAM]
    for r in range(world):
        res = json.load(open(out + f".{r}"))
        assert res["codes"] == expect
        first_wait = [i for i, (op, _) in enumerate(res["log"]) if op == "wait"][0]
        assert [j for op, j in res["log"][:first_wait] if op == "submit"] == list(range(inflight))


def _fallback_worker(rank, world, port, name, out_path):
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_c
    from conftest import load_pkg
    load_pkg()
    from importlib import import_module
    sharded = import_module("ed25519_consensus_amd.sharded")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
    items = [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]
    seed = bytes.fromhex(b["z_seed"])
    lo, hi = sharded.shard_bounds(len(items), world)[rank]

    def shard_ok():
        part, bad = oracle_c.shard_partial_affine(items[lo:hi], seed, lo)
        code, _ = oracle_c.combine_affine([part])
        return not bad and code == 0

    def find():   # the GPU runs edc_find_invalid_device here; the oracle verifies item by item
        return [(i, c) for i, c in enumerate(oracle_c.verify(*it) for it in items[lo:hi]) if c]

    res = sharded.find_invalid_sharded(shard_ok, find, sharded.torch_allgather_obj_fn(dist), rank, world, lo)
    with open(out_path + f".{rank}", "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["two_bad_of_300", "mixed_corpus_one_bad", "batch_verify_32"])
def test_two_rank_sharded_fallback(tmp_path, name):
    world = 2
    out = str(tmp_path / "fb")
    mp.start_processes(_fallback_worker, args=(world, _free_port(), name, out), nprocs=world, join=True,
                       start_method="spawn")
    b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
    expect = [[i, c] for i, c in enumerate(b["expect_single"]) if c]
    for r in range(world):
        assert json.load(open(out + f".{r}")) == expect



def test_exchange_ring_pop_without_post():
    """ExchangeRing.pop with nothing posted is a usage error, not a hang or a bogus record (a
    single-rank gloo group on the CPU)."""
    import torch
    import torch.distributed as dist
    import importlib
    from conftest import load_pkg
    load_pkg()
    sharded = importlib.import_module("ed25519_consensus_amd.sharded")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        ring = sharded.ExchangeRing(dist, torch.device("cpu"), depth=2, group=2)
        with pytest.raises(RuntimeError):
            ring.pop()
        ring.post(bytes(range(129)))
        assert ring.pop() == [bytes(range(129))]
        assert len(ring) == 0
    finally:
        dist.destroy_process_group()


def test_exchange_ring_warm_uses_every_buffer():
    """ExchangeRing.warm (bench.py, before timing): one group through every staging buffer at once
    -- a single post / pop would reuse one buffer (LIFO free list) and leave the others' first
    collective inside the timed region -- then an empty ring that exchanges records as before."""
    import torch
    import torch.distributed as dist
    import importlib
    from conftest import load_pkg
    load_pkg()
    sharded = importlib.import_module("ed25519_consensus_amd.sharded")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        ring = sharded.ExchangeRing(dist, torch.device("cpu"), depth=8, group=4)
        in_flight, send = [], ring._send

        def spy():
            send()
            in_flight.append(len(ring.sent))
        ring._send = spy
        ring.warm()
        assert max(in_flight) == len(ring.bufs) == 4
        assert len(ring) == 0 and sorted(ring.free) == list(range(len(ring.bufs)))
        recs = [bytes([i]) * 129 for i in range(6)]
        for r in recs:
            ring.post(r)
        assert [ring.pop() for _ in recs] == [[r] for r in recs]
    finally:
        dist.destroy_process_group()
