"""CPU: the oracle's C restatement (oracle/edc_oracle.c, dalek u64-backend algorithm) agrees
with the golden fixtures and the Python oracle; it is the checker for sizes Python cannot
reach and the bench's cpu_baseline."""
import os
import random
import sys

import pytest

from conftest import ROOT, golden

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_c  # noqa: E402


def _items(b):
    return [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]


@pytest.mark.parametrize("b", golden("batches.json")["batches"], ids=lambda b: b["name"])
def test_c_oracle_batches(b):
    it = _items(b)
    code, check8 = oracle_c.batch_verify(it, bytes.fromhex(b["z_seed"]))
    assert code == b["expect_code"]
    assert (check8.hex() if check8 else None) == b["expect_check8"]
    assert [oracle_c.verify(*x) for x in it] == b["expect_single"]


def test_c_oracle_corpus_and_rfc():
    fx = golden("zip215_small_order.json")
    msg = bytes.fromhex(fx["msg"])
    for c in fx["cases"]:
        assert oracle_c.verify(bytes.fromhex(c["vk"]), bytes.fromhex(c["sig"]), msg) == 0
    for v in golden("rfc8032.json")["vectors"]:
        assert oracle_c.verify(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"])) == 0


def test_c_oracle_random_vs_python(oracle):
    rnd = random.Random(8)
    seeds = [rnd.randbytes(32) for _ in range(5)]
    items = []
    for i in range(40):
        m = rnd.randbytes(rnd.randrange(0, 150))
        s = seeds[i % 5]
        items.append((oracle.public_key(s), oracle.sign(s, m), m))
    items[13] = (items[13][0], items[13][1], items[13][2] + b"x")
    for zs in (bytes(32), rnd.randbytes(32)):
        assert oracle_c.batch_verify(items, zs) == oracle.batch_verify_seeded(items, zs)


@pytest.mark.parametrize("name", ["two_bad_of_300", "repeated_keys_varlen", "undecodable_R", "c1_1024_distinct"])
def test_c_oracle_parallel_ranges(name):
    """The full-size checker (oracle_c.batch_verify_parallel: contiguous ranges at global z indices
    on host threads, partials summed) equals the fixture for any range count."""
    b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
    it = _items(b)
    offs = [0]
    for _, _, m in it:
        offs.append(offs[-1] + len(m))
    for parts in (1, 3, 8):
        code, c8, _ = oracle_c.batch_verify_parallel(b"".join(v for v, _, _ in it), b"".join(s for _, s, _ in it),
                                                     b"".join(m for _, _, m in it), offs, bytes.fromhex(b["z_seed"]),
                                                     parts=parts)
        assert code == b["expect_code"]
        assert (c8.hex() if c8 else None) == b["expect_check8"]


def test_c_oracle_shard_partials_combine():
    b = [x for x in golden("batches.json")["batches"] if x["name"] == "mixed_corpus_one_bad"][0]
    it = _items(b)
    seed = bytes.fromhex(b["z_seed"])
    for g in (1, 2, 4):
        bounds = [len(it) * r // g for r in range(g + 1)]
        parts = [oracle_c.shard_partial_affine(it[bounds[r]:bounds[r + 1]], seed, bounds[r])[0] for r in range(g)]
        code, c8 = oracle_c.combine_affine(parts)
        assert code == b["expect_code"] and c8.hex() == b["expect_check8"]
