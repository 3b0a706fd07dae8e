"""GPU: the decode's key lanes are sized from the previous grouped batch's key count (k_decompress
loops over the keys when a batch has more than its lanes). A context that has just verified vote
batches (150 keys: 4,096 key lanes) then verifies grouped batches with 16k and 40k distinct keys
(more keys than lanes): verdict and [8]*check equal a fresh context's (one lane per possible
key), valid and with one wrong signature. Reference: src/batch.rs:182-185 (every distinct key is
decoded once)."""
import ctypes
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _gen(edc, torch, eng, n, keys, base):
    sys.path.insert(0, ROOT)
    import bench
    vk, sig, msg, off = bench.make_workload(sys.modules["ed25519_consensus_amd"], eng, torch, torch.device("cuda:0"),
                                            n, keys, 32, base)
    torch.cuda.synchronize()
    return vk, sig, msg, off


def _verify(eng, n, vk, sig, msg, off, zseed):
    c8 = ctypes.create_string_buffer(32)
    code = eng.lib.edc_batch_verify_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                           zseed, 0, None, c8)
    return code, c8.raw


@pytest.mark.parametrize("n", [16384, 40960])
def test_more_keys_than_hinted_lanes(edc, n):
    torch = pytest.importorskip("torch")
    warm, fresh = edc.Engine(0), edc.Engine(0)
    try:
        warm.set_key_grouping(1)             # always group: the distinct-key batch stays grouped
        fresh.set_key_grouping(1)
        votes = _gen(edc, torch, warm, 8192, 150, 0)
        assert _verify(warm, 8192, *votes, bytes([3]) * 32)[0] == 0        # hint: ~150 keys
        vk, sig, msg, off = _gen(edc, torch, warm, n, 0, 1 << 20)         # n distinct keys
        zseed = bytes([0x61]) * 32
        for corrupt in (False, True):
            if corrupt:
                msg[32 * (n - 7)] ^= 1
                torch.cuda.synchronize()
            got = _verify(warm, n, vk, sig, msg, off, zseed)
            want = _verify(fresh, n, vk, sig, msg, off, zseed)
            assert got == want
            assert got[0] == (1 if corrupt else 0)
            if corrupt:
                assert got[1] not in (bytes(32), bytes([1]) + bytes(31))
    finally:
        warm.close()
        fresh.close()
