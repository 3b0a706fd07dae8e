"""GPU: key-grouping policy (include/edc.h edc_set_key_grouping). The reference coalesces signatures by
raw key bytes (src/batch.rs:114-137); keeping one A_i term per signature instead (coefficient
z_i k_i) is the same group element, so the verdict and the compressed [8]*check must equal the C
oracle's (which groups, like the reference) bit-exactly in every mode -- for repeated keys,
distinct keys, the ZIP215 corpus, undecodable keys and non-identity check points."""
import random

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle_c():
    import os
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c as oc
    return oc


@pytest.fixture()
def grouping(engine):
    yield engine
    engine.set_key_grouping(0)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("n,m,bad", [(8192, 150, None), (8192, 150, 4000), (4096, 4096, None), (5000, 5000, 17),
                                     (6000, 3000, None), (300, 7, 5)])
def test_grouping_modes_match_oracle(grouping, oracle_c, mode, n, m, bad):
    rnd = random.Random(n + 31 * m)
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(rnd.randrange(0, 200)) for _ in range(n)]
    vks, sigs = grouping.sign(seeds, msgs, seed_index=[rnd.randrange(m) for _ in range(n)])
    if bad is not None:
        sigs[bad] = sigs[bad][:40] + bytes([sigs[bad][40] ^ 4]) + sigs[bad][41:]
    zseed = rnd.randbytes(32)
    exp = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    grouping.set_key_grouping(mode)
    assert grouping.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True) == exp
    assert exp[0] == (0 if bad is None else 1)


def test_auto_mode_switches_and_agrees(grouping, oracle_c):
    """auto: a distinct-key batch is grouped first, the next ones are not (every 8th regroups);
    a repeated-key batch afterwards is still exact. Results never depend on the choice."""
    rnd = random.Random(7)
    n = 4096
    seeds = [rnd.randbytes(32) for _ in range(n)]
    msgs = [rnd.randbytes(32) for _ in range(n)]
    vks, sigs = grouping.sign(seeds, msgs)
    zseed = rnd.randbytes(32)
    exp = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    grouping.set_key_grouping(0)
    for _ in range(10):
        assert grouping.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True) == exp
    vks2, sigs2 = grouping.sign(seeds[:3], msgs, seed_index=[i % 3 for i in range(n)])
    exp2 = oracle_c.batch_verify(list(zip(vks2, sigs2, msgs)), zseed)
    for _ in range(3):
        assert grouping.batch_verify(vks2, sigs2, msgs, z_seed=zseed, want_check8=True) == exp2


def test_ungrouped_corpus_and_bad_key(grouping):
    """ZIP215 corpus (small-order / non-canonical A and R) and an undecodable key, keys ungrouped."""
    fx = golden("zip215_small_order.json")
    rnd = random.Random(11)
    n = 4096
    seeds = [rnd.randbytes(32) for _ in range(64)]
    msgs = [rnd.randbytes(48) for _ in range(n)]
    vks, sigs = grouping.sign(seeds, msgs, seed_index=[i % 64 for i in range(n)])
    pos = rnd.sample(range(n), len(fx["cases"]))
    for p, c in zip(pos, fx["cases"]):
        vks[p], sigs[p], msgs[p] = bytes.fromhex(c["vk"]), bytes.fromhex(c["sig"]), bytes.fromhex(fx["msg"])
    zseed = rnd.randbytes(32)
    grouping.set_key_grouping(1)
    g = grouping.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    grouping.set_key_grouping(2)
    u = grouping.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    assert g == u and g[0] == 0
    bad_key = bytes.fromhex([c for c in golden("decode.json")["cases"] if not c["ok"]][0]["enc"])
    vks[pos[0] ^ 1 if pos[0] ^ 1 not in pos else 0] = bad_key
    assert grouping.batch_verify(vks, sigs, msgs, z_seed=zseed)[0] == 1
    grouping.set_key_grouping(1)
    assert grouping.batch_verify(vks, sigs, msgs, z_seed=zseed)[0] == 1
