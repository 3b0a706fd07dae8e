"""GPU: randomized sharded verification in one process -- the arithmetic of the multi-GPU path
(sharded.py) without the collective. A random batch is cut into G = 1..8 contiguous
shards (sharded.shard_bounds); each shard's partial point comes from edc_batch_partial_device with
z drawn at its global queue indices (z_base = the shard's first index), and the G records are
combined on the device (Engine.combine_partials). Verdict and [8]*check must equal the C oracle's
for the whole, unsharded batch (src/batch.rs:149-217: the shards' partials sum to its check point),
for valid batches, a wrong message (non-identity check) and early rejects (undecodable R, s >= l:
no check point). 4 cases by default, EDC_SHARD_SOAK=<k> for a soak run."""
import ctypes
import os
import random
import sys

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

L_BYTES = (2**252 + 27742317777372353535851937790883648493).to_bytes(32, "little")
BAD_ENC = [bytes.fromhex(c["enc"]) for c in golden("decode.json")["cases"] if not c["ok"]]
SOAK = int(os.environ.get("EDC_SHARD_SOAK", "0"))


@pytest.fixture(scope="module")
def oc():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    return oracle_c


@pytest.mark.parametrize("case", range(SOAK or 4))
def test_random_shards_equal_oracle(engine, oc, case):
    torch = pytest.importorskip("torch")
    from importlib import import_module
    sharded = import_module("ed25519_consensus_amd.sharded")
    rnd = random.Random(6060 + case)
    n = rnd.choice([rnd.randrange(1, 64), rnd.randrange(64, 3000), rnd.randrange(3000, 20000)])
    m = rnd.choice([1, rnd.randrange(1, 200), n])
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(rnd.randrange(0, 300)) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[rnd.randrange(m) for _ in range(n)])
    vks, sigs = list(vks), list(sigs)
    kind = rnd.choice(["none", "none", "wrong_msg", "bad_r", "s_ge_l"])
    i = rnd.randrange(n)
    if kind == "wrong_msg":
        msgs[i] = msgs[i] + b"x"
    elif kind == "bad_r":
        sigs[i] = rnd.choice(BAD_ENC) + sigs[i][32:]
    elif kind == "s_ge_l":
        sigs[i] = sigs[i][:32] + L_BYTES
    zseed = rnd.randbytes(32)
    exp_code, exp_c8 = oc.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    assert exp_code == (0 if kind == "none" else 1)

    dev = torch.device("cuda:0")
    world = rnd.randrange(1, 9)
    parts, bad_any = [], 0
    for lo, hi in sharded.shard_bounds(n, world):
        mine = list(range(lo, hi))

        def _dev(b):
            return torch.tensor(list(b) or [0], dtype=torch.uint8, device=dev)
        offs = [0]
        for j in mine:
            offs.append(offs[-1] + len(msgs[j]))
        d_vk, d_sig = _dev(b"".join(vks[j] for j in mine)), _dev(b"".join(sigs[j] for j in mine))
        d_msg = _dev(b"".join(msgs[j] for j in mine))
        d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        part = ctypes.create_string_buffer(128)
        bad = ctypes.c_int(0)
        engine._check(engine.lib.edc_batch_partial_device(engine.ctx, len(mine), d_vk.data_ptr(), d_sig.data_ptr(),
                                                          d_msg.data_ptr(), d_off.data_ptr(), zseed, lo, None, part,
                                                          ctypes.byref(bad)))
        parts.append(part.raw)
        bad_any |= bad.value
    code, c8 = engine.combine_partials(parts, bad_any)
    tag = (case, n, m, kind, world)
    assert code == exp_code, tag
    assert bool(bad_any) == (exp_c8 is None), tag          # early rejects have no check point
    if exp_c8 is not None:
        assert c8 == exp_c8, tag
