"""GPU parity of every MSM plan (edc_common.h MsmPlan, edc_api.hip make_plan / batch_plan) against
the C oracle (dalek algorithm: Straus below 190 terms, Pippenger w = 6/7/8 above): verdict and the
compressed [8]*check, bit-exact, for valid batches and for batches whose check point is NOT the
identity (one bad item).

Plans covered: window widths 9..16 (14 and 15 are the auto widths from 2^17) and the size-chosen default, one batch split into 1..16
parts (summed per window); 8-bit high windows for the B / key
coefficients (chosen when the previous grouped batch on the context had few distinct keys) and
full-width windows otherwise; grouped keys, one key term per signature, and the on-device overflow
path of key grouping (set_key_grouping(3): grouping abandoned mid-batch, as adversarial keys would
cause). Each batch is verified twice, so the second run uses the plan hinted by the first.
Randomized shapes (test_random_plans_match_oracle): n, key count, window width, parts, message
length and the bad item drawn per case, 6 cases by default, EDC_PLAN_SOAK=<k> for a soak run."""
import os
import random

import pytest

from conftest import ROOT  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle_c():
    import os
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c as oc
    return oc


def _batch(engine, n, m, bad, msg_len=120, seed=0):
    rnd = random.Random(n * 1000 + m + seed)
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(msg_len) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
    msgs = list(msgs)
    if bad is not None:
        msgs[bad] = msgs[bad][:-1] + bytes([msgs[bad][-1] ^ 1])
    return vks, sigs, msgs, rnd.randbytes(32)


@pytest.mark.parametrize("n,m,bad", [(4096, 256, None), (4096, 256, 77), (4096, 257, 5), (8192, 5, 8000),
                                     (8192, 1, None), (8192, 150, 3), (6000, 6000, 17)])
@pytest.mark.parametrize("bits,parts", [(0, 0), (9, 1), (12, 3), (13, 0), (14, 1), (15, 1), (16, 1), (16, 2), (11, 16)])
def test_plans_match_oracle(engine, oracle_c, n, m, bad, bits, parts):
    vks, sigs, msgs, zseed = _batch(engine, n, m, bad)
    exp_code, exp_c8 = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    assert exp_code == (0 if bad is None else 1)
    engine.set_msm_shape(bits, parts)
    try:
        for _ in range(2):
            code, c8 = engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
            assert code == exp_code
            assert c8 == exp_c8
    finally:
        engine.set_msm_shape(0, 0)


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("m,bad", [(150, None), (150, 9), (5000, 4321)])
def test_grouping_modes_and_overflow_path(engine, oracle_c, mode, m, bad):
    n = 5000
    vks, sigs, msgs, zseed = _batch(engine, n, m, bad, seed=mode)
    exp_code, exp_c8 = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    engine.set_key_grouping(mode)
    try:
        code, c8 = engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    finally:
        engine.set_key_grouping(0)
    assert (code, c8) == (exp_code, exp_c8)


@pytest.mark.parametrize("stage", [0, 512])
@pytest.mark.parametrize("n,m,bad", [(4096, 256, 77), (8192, 150, None), (6000, 6000, 17)])
@pytest.mark.parametrize("bits,parts", [(0, 0), (16, 1), (11, 16)])
def test_scatter_direct_path_matches_oracle(engine, oracle_c, stage, n, m, bad, bits, parts):
    """The binning scatter's direct-store path (workgroups whose digits overflow the LDS stage:
    at the default 16k-entry stage only very large bin counts take it) and a small stage that
    splits workgroups between both paths, against the C oracle (that path was only
    covered by bench.py's valid-batch assert)."""
    vks, sigs, msgs, zseed = _batch(engine, n, m, bad, seed=stage + 7)
    exp_code, exp_c8 = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    engine.lib.edc_debug_set_scatter_stage(stage)
    engine.set_msm_shape(bits, parts)
    try:
        for _ in range(2):
            assert engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True) == (exp_code, exp_c8)
    finally:
        engine.set_msm_shape(0, 0)
        engine.lib.edc_debug_set_scatter_stage(16384)


PLAN_SOAK = int(os.environ.get("EDC_PLAN_SOAK", "0"))


@pytest.mark.parametrize("case", range(PLAN_SOAK or 6))
def test_random_plans_match_oracle(engine, oracle_c, case):
    """bins from a few entries (E < 256: several accumulation lanes share a start, the lane-major
    index mapping's edge) to thousands, any window width the API accepts and 0..16 parts"""
    rnd = random.Random(31337 + case)
    n = rnd.choice([rnd.randrange(1, 300), rnd.randrange(300, 5000), rnd.randrange(5000, 20000)])
    m = rnd.choice([1, rnd.randrange(1, 200), max(1, n // rnd.choice([1, 2, 7, 50]))])
    bits = rnd.choice([0, 9, 10, 11, 12, 13, 14, 15, 16])
    parts = rnd.choice([0, 1, 2, 3, 4, 8, 16])
    bad = rnd.choice([None, rnd.randrange(n)])
    vks, sigs, msgs, zseed = _batch(engine, n, m, bad, msg_len=rnd.randrange(0 if bad is None else 1, 300),
                                        seed=case)
    exp_code, exp_c8 = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    engine.set_msm_shape(bits, parts)
    try:
        for _ in range(2):
            got = engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
            assert got == (exp_code, exp_c8), (case, n, m, bits, parts, bad)
    finally:
        engine.set_msm_shape(0, 0)
