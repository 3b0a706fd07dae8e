"""GPU: BASELINE configs[3] at its stated size -- 2^20 consensus votes from 150 validators
(120-byte messages), the 196-case ZIP215 small-order corpus (reference tests/small_order.rs:12-77)
at seeded positions and ONE signature made over another message (tests/batch.rs:27-31).

The reference flow (tests/batch.rs:18-44): the batch fails, then Item::verify_single on every item
(src/batch.rs:104-107) flags exactly the bad one. Here:
  * edc_batch_verify_device  -> InvalidSignature
  * edc_verify_each_device (the per-item kernel) and edc_find_invalid_device (the grouped fallback)
    return, for EVERY item, the code Item::verify_single gives: the corpus cases Ok (ZIP215, pinned
    by the golden fixture's expect_single), the bad item InvalidSignature, all others Ok
  * the valid remainder (bad item removed, corpus kept) verifies as one batch, [8]*check = identity.
Size-independent properties at full size; the per-item expectations come from the fixture and the
construction, not from running the oracle on 2^20 items."""
import ctypes
import os
import sys

import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IDENTITY = bytes([1]) + bytes(31)


def test_config3_corpus_and_bad_sig_in_2_20_votes(engine):
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    n, keys, msg_len = 1 << 20, 150, 120
    fx = golden("zip215_small_order.json")
    pkg = sys.modules["ed25519_consensus_amd"]
    vk, sig, msg, off, expect, cpos = bench.make_c4_workload(pkg, engine, torch, dev, n, keys, msg_len, fx["cases"],
                                                             bytes.fromhex(fx["msg"]))
    torch.cuda.synchronize()
    assert len(expect) == 1 and len(cpos) == 196      # every corpus case is valid under ZIP215
    lib = engine.lib
    zseed = bytes([0x33]) * 32
    args = (vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr())
    c8 = ctypes.create_string_buffer(32)
    assert lib.edc_batch_verify_device(engine.ctx, n, *args, zseed, 0, None, c8) == 1
    assert c8.raw != IDENTITY

    d_ver = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    assert lib.edc_verify_each_device(engine.ctx, n, *args, d_ver.data_ptr()) == 0
    each = d_ver.cpu()
    got_each = {int(i): int(each[i]) for i in torch.nonzero(each).flatten().tolist()}
    assert got_each == expect

    verdicts = ctypes.create_string_buffer(n)
    nbad = lib.edc_find_invalid_device(engine.ctx, n, *args, zseed, 1 << 16, verdicts)
    assert nbad == 1
    raw = verdicts.raw
    got_group = {i: raw[i] for i in expect}
    assert got_group == expect and raw.count(0) == n - 1

    # batch + fallback in one call (the failed batch's k, points and grouping reused)
    v2 = ctypes.create_string_buffer(n)
    cnt = ctypes.c_int(-1)
    assert lib.edc_batch_verify_fallback_device(engine.ctx, n, *args, zseed, v2, ctypes.byref(cnt), None) == 1
    assert cnt.value == 1 and {i: v2.raw[i] for i in expect} == expect and v2.raw.count(0) == n - 1

    # the valid remainder, corpus included, is one valid batch
    keep = torch.ones(n, dtype=torch.bool, device=dev)
    keep[list(expect)] = False
    idx = torch.nonzero(keep).flatten()
    m = idx.numel()
    vk2 = vk.view(-1, 32)[:n][idx].contiguous()
    sig2 = sig.view(-1, 64)[:n][idx].contiguous()
    lens = (off[1:] - off[:-1])[idx]
    starts = off[:-1][idx]
    off2 = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    off2[1:] = torch.cumsum(lens, 0)
    pos_in_item = torch.arange(int(off2[-1].item()), device=dev) - torch.repeat_interleave(off2[:-1], lens)
    msg2 = torch.cat([msg[torch.repeat_interleave(starts, lens) + pos_in_item],
                      torch.zeros(1, dtype=torch.uint8, device=dev)])
    torch.cuda.synchronize()
    assert lib.edc_batch_verify_device(engine.ctx, m, vk2.data_ptr(), sig2.data_ptr(), msg2.data_ptr(),
                                       off2.data_ptr(), zseed, 0, None, c8) == 0
    assert c8.raw == IDENTITY
    del vk, sig, msg, off, vk2, sig2, msg2
    torch.cuda.empty_cache()
