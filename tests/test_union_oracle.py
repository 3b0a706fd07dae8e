"""CPU: the fact union-first multi-batch launches rely on (include/edc.h, edc_set_multi_union), on
the C oracle. Consecutive batches with z drawn at global queue indices: the union's check point
is the sum of the batches' check points, so the union passes exactly when the sum's [8]-multiple
is the identity, and with one failing batch the union fails (src/batch.rs:149-217 evaluated on
the concatenation). Checked over pairs of the golden batches that the oracle evaluates."""
import os
import sys

import pytest

from conftest import ROOT, golden

BATCHES = [b for b in golden("batches.json")["batches"] if b["items"]]


@pytest.fixture(scope="module")
def oc():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    return oracle_c


def _items(b):
    return [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]


@pytest.mark.parametrize("i", range(len(BATCHES)))
def test_union_is_sum_of_batches(oc, i):
    a, b = BATCHES[i], BATCHES[(i + 1) % len(BATCHES)]
    ia, ib = _items(a), _items(b)
    seed = bytes.fromhex(a["z_seed"])
    pa, bad_a = oc.shard_partial_affine(ia, seed, 0)
    pb, bad_b = oc.shard_partial_affine(ib, seed, len(ia))
    code_u, c8_u = oc.batch_verify(ia + ib, seed)                      # the union as one batch
    if bad_a or bad_b:                                                 # rejected before the MSM
        assert code_u == 1
        return
    code_sum, c8_sum = oc.combine_affine([pa, pb])
    assert (code_u, c8_u) == (code_sum, c8_sum)
    ca, _ = oc.combine_affine([pa])
    cb, _ = oc.combine_affine([pb])
    # union passes <=> both pass (no cancellation between independent random-z batches)
    assert (code_u == 0) == (ca == 0 and cb == 0)
