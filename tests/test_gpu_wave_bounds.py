"""GPU: batch sizes around the 64-lane wave boundary. k_decompress decodes R_i on lanes [0, n) and
the distinct keys from the next wave boundary on (edc_prep.hip launch_decompress; one wave per
workgroup below 16k lanes), and the Horner / window combine run in the distributed quad layout
(ge_quad.h quad_pt). For n in {1, 2, 63, 64, 65, 127, 128, 129, 191, 200}, with distinct keys, one
key, and keys half cached (split coefficients on, so the uncached keys take the doubled-on-device
path), the verdict and the compressed [8]*check equal the C oracle's (reference batch::Verifier,
src/batch.rs:149-217), for a valid batch and for one with a corrupted signature at the last item."""
import random

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 63, 64, 65, 127, 128, 129, 191, 200]


@pytest.fixture(scope="module")
def oracle_c():
    import os
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c as oc
    return oc


@pytest.fixture()
def eng(engine):
    yield engine
    engine.keycache_clear()
    engine.set_key_split(0)


def _batch(engine, rnd, n, m):
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(rnd.randrange(0, 90)) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
    return list(vks), list(sigs), msgs


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("keys", ["distinct", "one", "half_cached"])
def test_sizes_around_wave_boundary(eng, oracle_c, n, keys):
    rnd = random.Random(n * 7 + len(keys))
    m = 1 if keys == "one" else n
    vks, sigs, msgs = _batch(eng, rnd, n, m)
    if keys == "half_cached":
        reg = list(dict.fromkeys(vks))
        u, ok = eng.keycache_load(reg[: (len(reg) + 1) // 2])
        assert all(ok)
    for bad in (None, n - 1):
        mm = list(msgs)
        if bad is not None:
            mm[bad] = mm[bad] + b"\x01"
        zseed = bytes([n & 0xFF, len(keys), 0 if bad is None else 1]) + bytes(29)
        exp = oracle_c.batch_verify(list(zip(vks, sigs, mm)), zseed)
        assert exp[0] == (0 if bad is None else 1)
        got = eng.batch_verify(vks, sigs, mm, z_seed=zseed, want_check8=True)
        assert got == exp, (n, keys, bad)
