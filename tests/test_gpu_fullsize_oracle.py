"""GPU vs the C oracle at FULL size: the non-identity [8]*check of a failing configs[2] batch (2^20
votes from 150 validators, 120-byte messages) and of a failing configs[4] shard (2^21 distinct keys,
0..1024-byte messages), byte for byte. Below 8,192 items every plan is compared with the oracle in
test_gpu_plans.py; here the full-size plans are: 16-bit windows, automatic sub-bins, the few-keys
plan with its overlapped top-run Horner (k_msm_window2, the second vote batch on a context), the
per-signature key layout of distinct-key batches (their second batch), bins near the top of the
plan range.

The oracle (oracle/edc_oracle.c, the dalek u64 restatement pinned to the reference's vectors) runs
the same batch as contiguous ranges at global z indices on every host thread
(oracle_c.batch_verify_parallel; the equation is linear, reference src/batch.rs:189-216), and the
range partials are summed. The host time is printed (-s) for profiles/."""
import ctypes
import os
import sys
import time

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

IDENTITY = bytes([1]) + bytes(31)


def _oracle_c():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    return oracle_c


def _host(vk, sig, msg, off):
    n = vk.numel() // 32
    o = off.cpu().numpy().astype("uint64")
    offs = (ctypes.c_uint64 * (n + 1)).from_buffer_copy(o.tobytes())
    return vk[:32 * n].cpu().numpy().tobytes(), sig[:64 * n].cpu().numpy().tobytes(), \
        msg.cpu().numpy().tobytes(), offs


def _run(edc, torch, config, corrupt):
    sys.path.insert(0, ROOT)
    import bench
    oc = _oracle_c()
    dev = torch.device("cuda:0")
    n, keys, mlen = bench.CONFIGS[config][:3]
    eng = edc.Engine(0)          # fresh context: first batch dense plan / grouped, second the adaptive one
    try:
        vk, sig, msg, off = bench.make_workload(sys.modules["ed25519_consensus_amd"], eng, torch, dev, n, keys, mlen, 0)
        torch.cuda.synchronize()
        corrupt(vk, sig, msg, off)
        torch.cuda.synchronize()
        zseed = bytes([0x7E]) * 32
        gpu = []
        for _ in range(2):
            c8 = ctypes.create_string_buffer(32)
            code = eng.lib.edc_batch_verify_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                                   off.data_ptr(), zseed, 0, None, c8)
            gpu.append((code, c8.raw))
        hv, hs, hm, ho = _host(vk, sig, msg, off)
        code, c8, secs = oc.batch_verify_parallel(hv, hs, hm, ho, zseed)
        print(f"\n[fullsize-oracle] {config} n={n}: oracle {secs:.2f} s on {oc.host_threads()} host threads; "
              f"gpu {gpu[0][0]} / {gpu[1][0]}, oracle {code}, check8 {c8.hex() if c8 else None}")
        return gpu, (code, c8)
    finally:
        eng.close()


def test_config2_failing_batch_vs_oracle(edc):
    torch = pytest.importorskip("torch")

    def corrupt(vk, sig, msg, off):
        sig[64 * 777_777 + 40] ^= 0x01        # s changed, still canonical: decodable, wrong equation

    gpu, (code, c8) = _run(edc, torch, "c3", corrupt)
    assert code == 1 and c8 is not None and c8 != IDENTITY
    assert gpu[0] == gpu[1] == (1, c8)


def test_config4_failing_shard_vs_oracle(edc):
    torch = pytest.importorskip("torch")

    def corrupt(vk, sig, msg, off):
        bad = 1_500_001
        o = int(off[bad].item())
        assert int(off[bad + 1].item()) > o
        msg[o] ^= 0x80                        # signed over a different message

    gpu, (code, c8) = _run(edc, torch, "c5", corrupt)
    assert code == 1 and c8 is not None and c8 != IDENTITY
    assert gpu[0] == gpu[1] == (1, c8)


def test_config2_valid_batch_vs_oracle(edc):
    """The same machinery on the valid batch: both sides give Ok with the identity (guards the
    checker itself: a broken range split would not sum to the identity)."""
    torch = pytest.importorskip("torch")
    gpu, (code, c8) = _run(edc, torch, "c3", lambda *a: None)
    assert (code, c8) == (0, IDENTITY)
    assert gpu[0] == gpu[1] == (0, IDENTITY)


def test_config1_failing_batch_vs_oracle(edc):
    """configs[1]: 2^16 signatures with distinct keys and 32-byte messages, one corrupted s: the
    non-identity [8]*check of both plans (grouped first batch, per-signature second) against the
    oracle."""
    torch = pytest.importorskip("torch")

    def corrupt(vk, sig, msg, off):
        sig[64 * 40_000 + 37] ^= 0x02         # s changed, still canonical

    gpu, (code, c8) = _run(edc, torch, "c2", corrupt)
    assert code == 1 and c8 is not None and c8 != IDENTITY
    assert gpu[0] == gpu[1] == (1, c8)


def test_config3_failing_batch_vs_oracle(edc):
    """configs[3]: 2^20 votes with the 196-case ZIP215 corpus (small-order and non-canonical A / R,
    reference tests/small_order.rs:12-77) at seeded positions and one signature over another
    message: the failing batch's non-identity [8]*check against the oracle, byte for byte (the
    corpus points are torsion points, so this pins their MSM terms at full size too)."""
    torch = pytest.importorskip("torch")
    from conftest import golden
    sys.path.insert(0, ROOT)
    import bench
    oc = _oracle_c()
    dev = torch.device("cuda:0")
    fx = golden("zip215_small_order.json")
    eng = edc.Engine(0)
    try:
        vk, sig, msg, off, expect, cpos = bench.make_c4_workload(sys.modules["ed25519_consensus_amd"], eng, torch, dev,
                                                                 1 << 20, 150, 120, fx["cases"],
                                                                 bytes.fromhex(fx["msg"]))
        torch.cuda.synchronize()
        n = 1 << 20
        zseed = bytes([0x3D]) * 32
        gpu = []
        for _ in range(2):
            c8 = ctypes.create_string_buffer(32)
            code = eng.lib.edc_batch_verify_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                                   off.data_ptr(), zseed, 0, None, c8)
            gpu.append((code, c8.raw))
        hv, hs, hm, ho = _host(vk, sig, msg, off)
        code, c8, secs = oc.batch_verify_parallel(hv, hs, hm, ho, zseed)
        print(f"\n[fullsize-oracle] configs[3] n={n}: oracle {secs:.2f} s on {oc.host_threads()} host threads; "
              f"gpu {gpu[0][0]} / {gpu[1][0]}, oracle {code}, check8 {c8.hex() if c8 else None}")
        assert code == 1 and c8 is not None and c8 != IDENTITY
        assert gpu[0] == gpu[1] == (1, c8)
    finally:
        eng.close()
