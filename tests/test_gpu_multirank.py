"""GPU, world_size 2 over gloo (both ranks on cuda:0): the one-process-per-GPU path of bench.py /
sharded.py end to end on the device -- each rank computes its contiguous slice's partial point with
edc_batch_partial_device (z drawn at global queue indices), the ranks all-gather the 129-byte
records and every rank combines them with edc_combine_partials. The verdict and [8]*check must
equal the unsharded reference values: the golden batches' (tests/golden/batches.json) and the C
oracle's for a larger random batch with one forged signature. The CPU twin
(tests/test_multirank_gloo.py) uses oracle partials; RCCL replaces gloo on a multi-GPU node."""
import json
import os
import random
import socket
import sys

import pytest
import torch.multiprocessing as mp

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _items(name):
    if name.startswith("random"):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conftest import load_pkg
        pkg = load_pkg()
        eng = pkg.Engine(0)
        rnd = random.Random(4242)
        n, m = 5000, 40
        seeds = [rnd.randbytes(32) for _ in range(m)]
        msgs = [rnd.randbytes(rnd.randrange(0, 300)) for _ in range(n)]
        vks, sigs = eng.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
        eng.close()
        msgs[3777] = msgs[3777] + b"x"
        return list(zip(vks, sigs, msgs)), bytes([0x5A]) * 32
    b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
    items = [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]
    return items, bytes.fromhex(b["z_seed"])


def _worker(rank, world, port, name, out_path):
    import ctypes
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_pkg
    pkg = load_pkg()
    from importlib import import_module
    sharded = import_module("ed25519_consensus_amd.sharded")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    items, seed = _items(name)
    lo, hi = sharded.shard_bounds(len(items), world)[rank]
    mine = items[lo:hi]
    dev = torch.device("cuda:0")
    eng = pkg.Engine(0)

    def _dev(b):
        return torch.tensor(list(b) or [0], dtype=torch.uint8, device=dev)
    offs = [0]
    for it in mine:
        offs.append(offs[-1] + len(it[2]))
    d_vk, d_sig = _dev(b"".join(it[0] for it in mine)), _dev(b"".join(it[1] for it in mine))
    d_msg = _dev(b"".join(it[2] for it in mine))
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    def partial(zbase):
        part = ctypes.create_string_buffer(128)
        bad = ctypes.c_int(0)
        eng._check(eng.lib.edc_batch_partial_device(eng.ctx, len(mine), d_vk.data_ptr(), d_sig.data_ptr(),
                                                    d_msg.data_ptr(), d_off.data_ptr(), seed, zbase, None, part,
                                                    ctypes.byref(bad)))
        return part.raw, bad.value

    def allgather(rec):
        t = torch.tensor(list(rec), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return [bytes(o.tolist()) for o in out]

    def combine(parts, bad_any):       # an early reject has no check point (oracle contract: None)
        code, c8 = eng.combine_partials(parts, bad_any)
        return code, (None if bad_any else c8)

    code, c8 = sharded.verify_sharded(partial, combine, allgather, rank, world, lo)
    with open(out_path + f".{rank}", "w") as f:
        json.dump({"code": code, "check8": c8.hex() if c8 else None}, f)
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["mixed_corpus_one_bad", "repeated_keys_varlen", "undecodable_R", "random_5000"])
def test_two_rank_device_partials(tmp_path, name):
    world = 2
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _free_port(), name, out), nprocs=world, join=True,
                       start_method="spawn")
    if name.startswith("random"):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_c
        items, seed = _items(name)
        exp_code, exp_c8 = oracle_c.batch_verify(items, seed)
        assert exp_code == 1 and exp_c8 is not None
        exp_c8 = exp_c8.hex()
    else:
        b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
        exp_code, exp_c8 = b["expect_code"], b["expect_check8"]
    for r in range(world):
        res = json.load(open(out + f".{r}"))
        assert res["code"] == exp_code
        assert res["check8"] == exp_c8
