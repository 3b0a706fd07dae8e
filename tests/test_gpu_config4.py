"""GPU: BASELINE configs[4] at its own per-GPU shape -- 2^21 signatures with distinct keys and
uniform 0..1024-byte messages (1-9 SHA-512 blocks per challenge), the slice one of 8 GPUs gets of
the 2^24 batch, generated exactly as `bench.py --config c5` times it.

Size-independent properties (the oracle is not run at this size; the same shape at 5-6k items is
bit-exact against the C oracle in test_gpu_multiblock.py):
- a valid batch is Ok with [8]*check = identity (reference tests/batch.rs:18-26);
- one item whose message was altered after signing makes the batch fail with a non-identity
  check point, and the grouped fallback localizes exactly that item (InvalidSignature), as the
  caller's Item::verify_single loop (tests/batch.rs:37-43) would;
- 8 contiguous shards at global z offsets (edc_batch_partial_device, each with its own message
  arena slice) recombine through edc_combine_partials to the unsharded [8]*check, valid and
  invalid (the multi-GPU reduction of configs[4]).
test_config4_whole_2_24_one_batch runs the WHOLE configs[4] workload -- 2^24 distinct-key
signatures with 0..1024-byte messages -- as ONE batch on one GPU (it fits the 288 GB): valid
batch Ok with the identity, one altered message fails it and is localized exactly; host times
are printed (-s) for profiles/."""
import ctypes
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

IDENTITY = bytes([1]) + bytes(31)


def test_config4_shape_2_21(engine):
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    n_items, keys, msg_len = bench.CONFIGS["c5"][:3]
    assert (n_items, keys, msg_len) == (1 << 21, 0, -1)
    pkg = sys.modules["ed25519_consensus_amd"]
    vk, sig, msg, off = bench.make_workload(pkg, engine, torch, dev, n_items, keys, msg_len, 0)
    torch.cuda.synchronize()
    lens = (off[1:] - off[:-1])
    assert int(lens.min()) == 0 and int(lens.max()) == 1024          # the whole 0..1024 range occurs
    lib = engine.lib
    zseed = bytes([0x3C]) * 32
    c8 = ctypes.create_string_buffer(32)

    def verify():
        return lib.edc_batch_verify_device(engine.ctx, n_items, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                           off.data_ptr(), zseed, 0, None, c8)

    def sharded(nshards=8):
        parts, bad_any, offs = [], 0, []
        for s in range(nshards):
            lo, hi = n_items * s // nshards, n_items * (s + 1) // nshards
            o = (off[lo:hi + 1] - off[lo]).contiguous()
            offs.append(o)
            part = ctypes.create_string_buffer(128)
            flag = ctypes.c_int(0)
            rc = lib.edc_batch_partial_device(engine.ctx, hi - lo, vk.data_ptr() + 32 * lo, sig.data_ptr() + 64 * lo,
                                              msg.data_ptr() + int(off[lo].item()), o.data_ptr(), zseed, lo, None,
                                              part, ctypes.byref(flag))
            assert rc == 0
            parts.append(part.raw)
            bad_any |= flag.value
        return engine.combine_partials(parts, bad_any)

    assert verify() == 0 and c8.raw == IDENTITY
    assert sharded() == (0, IDENTITY)

    bad = 1_234_567
    assert int(lens[bad]) > 0
    msg[int(off[bad].item())] ^= 0x01                                # signed over a different message
    torch.cuda.synchronize()
    assert verify() == 1 and c8.raw != IDENTITY
    whole = c8.raw
    assert sharded() == (1, whole)

    verdicts = ctypes.create_string_buffer(n_items)
    nbad = lib.edc_find_invalid_device(engine.ctx, n_items, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                       off.data_ptr(), zseed, 1 << 16, verdicts)
    assert nbad == 1
    raw = verdicts.raw
    assert raw[bad] == 1 and raw.count(0) == n_items - 1
    del vk, sig, msg, off
    torch.cuda.empty_cache()


def test_config4_whole_2_24_one_batch(engine):
    torch = pytest.importorskip("torch")
    import time
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    n = 1 << 24
    pkg = sys.modules["ed25519_consensus_amd"]
    t0 = time.perf_counter()
    vk, sig, msg, off = bench.make_workload(pkg, engine, torch, dev, n, 0, -1, 0)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    lens = off[1:] - off[:-1]
    assert int(lens.min()) == 0 and int(lens.max()) == 1024
    lib = engine.lib
    zseed = bytes([0x3E]) * 32
    c8 = ctypes.create_string_buffer(32)

    def verify():
        t = time.perf_counter()
        rc = lib.edc_batch_verify_device(engine.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                         off.data_ptr(), zseed, 0, None, c8)
        return rc, time.perf_counter() - t

    rc1, t1 = verify()
    assert rc1 == 0 and c8.raw == IDENTITY                           # grouped (first batch)
    rc2, t2 = verify()
    assert rc2 == 0 and c8.raw == IDENTITY                           # per-signature key terms
    bad = 9_876_543
    assert int(lens[bad]) > 0
    msg[int(off[bad].item()) + int(lens[bad].item()) - 1] ^= 0x40   # signed over another message
    torch.cuda.synchronize()
    rc3, t3 = verify()
    assert rc3 == 1 and c8.raw != IDENTITY
    verdicts = ctypes.create_string_buffer(n)
    t = time.perf_counter()
    nbad = lib.edc_find_invalid_device(engine.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                       off.data_ptr(), zseed, 1 << 16, verdicts)
    t_fb = time.perf_counter() - t
    assert nbad == 1
    raw = verdicts.raw
    assert raw[bad] == 1 and raw.count(0) == n - 1
    print(f"\n[configs4-whole] n=2^24 msgs {int(off[-1].item()) / 2**30:.2f} GiB: gen {t_gen:.2f} s, "
          f"batches {t1 * 1e3:.1f} / {t2 * 1e3:.1f} / {t3 * 1e3:.1f} ms, fallback {t_fb * 1e3:.1f} ms")
    del vk, sig, msg, off, lens
    torch.cuda.empty_cache()
