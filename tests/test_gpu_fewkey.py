"""GPU parity of the few-key MSM mode (edc_common.h: n >= 4096 and 16 m <= n, every full-width
coefficient split over P and [2^128]P, 8 windows only) against the C oracle (dalek algorithm,
unsplit coefficients): verdict and the compressed [8]*check, bit-exact, for valid batches and
for batches whose check point is NOT the identity (one bad item), on both sides of the mode
boundary."""
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


@pytest.mark.parametrize("n,m,bad", [(4096, 256, None), (4096, 256, 77), (4096, 257, 5), (8192, 5, 8000),
                                     (8192, 1, None), (8192, 150, 3)])
def test_few_key_mode_matches_oracle(engine, oracle_c, n, m, bad):
    rnd = random.Random(n * 1000 + m)
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(120) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
    msgs = list(msgs)
    if bad is not None:
        msgs[bad] = msgs[bad][:-1] + bytes([msgs[bad][-1] ^ 1])
    zseed = rnd.randbytes(32)
    items = list(zip(vks, sigs, msgs))
    exp_code, exp_c8 = oracle_c.batch_verify(items, zseed)
    code, c8 = engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    assert code == exp_code == (0 if bad is None else 1)
    assert c8 == exp_c8
