"""GPU: the synchronous host-buffer calls -- edc_batch_verify, edc_batch_verify_z and
edc_batch_verify_prehashed, the calls the Rust shim makes for `Verifier::verify` (reference
src/batch.rs:149-217) -- from 2^16 items copy their inputs in pieces and start each piece's decode,
SHA-512 and coefficient pass as it lands (edc_api.hip `enqueue_host_chunked`). Checked against the
device-resident one-piece path (edc_batch_verify_device / edc_batch_verify_prehashed_device) on the
same inputs and z: verdict and [8]*check byte for byte, twice per engine (the first batch on a
context plans dense/grouped, the second adaptively: few-keys windows, per-signature key terms).

Cases: vote batches (150 validators) and distinct keys; ragged n (a partial last chunk) and n at
the 2^16 threshold; 0..1024-byte messages with offsets that do not start at 0; a wrong signature in
the last chunk (a non-identity check8); an undecodable R in the last chunk and an s = l in the first
(the bad flag: code 1, zero check8); caller-drawn z. Grouped batches accumulate each chunk's R
terms into the MSM buckets as the chunk lands and add the key / B terms at the end; key grouping
forced for distinct keys (70,001 key terms at the end) and the device's grouping overflow (one A_i
term per signature at the end, FLAG_OVF) are covered too."""
import ctypes
import os
import sys

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

L_BYTES = (2**252 + 27742317777372353535851937790883648493).to_bytes(32, "little")
UNDECODABLE = next(bytes.fromhex(c["enc"]) for c in golden("decode.json")["cases"] if not c["ok"])


@pytest.fixture(scope="module")
def env(edc):
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    return torch, bench, edc


def _workload(env, eng, n, keys, mlen):
    torch, bench, edc = env
    vk, sig, msg, off = bench.make_workload(sys.modules["ed25519_consensus_amd"], eng, torch, torch.device("cuda:0"),
                                            n, keys, mlen, 0)
    torch.cuda.synchronize()
    return vk, sig, msg, off


def _corrupt(kind, vk, sig, msg, off, n):
    torch = sys.modules["torch"]
    if kind == "wrong_sig":        # signed over another message (tests/batch.rs:27-31), last chunk
        i = n - 3
        o = int(off[i])
        if int(off[i + 1]) > o:
            msg[o] ^= 1
        else:
            sig[64 * i + 40] ^= 1
    elif kind == "bad_r_and_s":    # undecodable R (last chunk) and s = l (first chunk): the bad flag
        sig[64 * (n - 2):64 * (n - 2) + 32] = torch.tensor(list(UNDECODABLE), dtype=torch.uint8, device=sig.device)
        sig[64 * 5 + 32:64 * 5 + 64] = torch.tensor(list(L_BYTES), dtype=torch.uint8, device=sig.device)
    torch.cuda.synchronize()


def _host_copies(vk, sig, msg, off, n, shift):
    """pageable host buffers; the arena starts `shift` junk bytes in, so offsets do not start at 0"""
    hv = vk[:32 * n].cpu().numpy().tobytes()
    hs = sig[:64 * n].cpu().numpy().tobytes()
    o = off[:n + 1].cpu().numpy().astype("uint64")
    hm = bytes(range(shift)) + msg[int(o[0]):int(o[-1])].cpu().numpy().tobytes() + b"\0"
    o = o - o[0] + shift
    return hv, hs, hm, (ctypes.c_uint64 * (n + 1)).from_buffer_copy(o.tobytes())


CASES = [   # (n, validators (0 = distinct), message bytes (-1 = 0..1024), corruption, key grouping mode)
    (70001, 150, 120, "wrong_sig", 0),
    (65536, 0, 32, "wrong_sig", 0),
    (70001, 0, -1, "wrong_sig", 0),
    (98304 + 77, 150, 120, "bad_r_and_s", 0),
    (70001, 150, 120, "none", 0),
    (1 << 20, 150, 120, "wrong_sig", 0),
    (70001, 0, 32, "none", 1),          # always grouped: every distinct key a term at the end
    (70001, 150, 120, "wrong_sig", 3),  # grouping overflow on the device: per-signature A_i terms
    (70001, 150, 120, "none", 3),
]


@pytest.mark.parametrize("n,keys,mlen,kind,grouping", CASES, ids=lambda v: str(v))
def test_host_chunked_equals_device(env, n, keys, mlen, kind, grouping):
    torch, bench, edc = env
    eng = edc.Engine(0)
    try:
        eng.set_key_grouping(grouping)
        vk, sig, msg, off = _workload(env, eng, n, keys, mlen)
        _corrupt(kind, vk, sig, msg, off, n)
        hv, hs, hm, ho = _host_copies(vk, sig, msg, off, n, shift=5)
        lib = eng.lib
        zseed = bytes([0x5A]) * 32
        kb = ctypes.create_string_buffer(32 * n)
        eng._check(lib.edc_challenge(eng.ctx, n, hv, hs, hm, ho, kb))
        d_k = torch.frombuffer(bytearray(kb.raw), dtype=torch.uint8).to("cuda:0")
        z = bytes((7 * i + 3) & 0xFF for i in range(16 * n))
        d_z = torch.frombuffer(bytearray(z), dtype=torch.uint8).to("cuda:0")
        torch.cuda.synchronize()
        want = 0 if kind == "none" else 1
        for rep in range(2):
            c_dev, c_host = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
            r_dev = lib.edc_batch_verify_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                                off.data_ptr(), zseed, 0, None, c_dev)
            r_host = lib.edc_batch_verify(eng.ctx, n, hv, hs, hm, ho, zseed, c_host)
            assert (r_host, c_host.raw) == (r_dev, c_dev.raw) and r_dev == want, (rep, "messages")
            if kind == "bad_r_and_s":
                assert c_host.raw == bytes(32)
            elif kind == "wrong_sig":
                assert c_host.raw not in (bytes(32), bytes([1]) + bytes(31))

            c_dev, c_host = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
            r_dev = lib.edc_batch_verify_prehashed_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), d_k.data_ptr(),
                                                          zseed, 0, None, c_dev)
            r_host = lib.edc_batch_verify_prehashed(eng.ctx, n, hv, hs, kb.raw, zseed, None, c_host)
            assert (r_host, c_host.raw) == (r_dev, c_dev.raw) and r_dev == want, (rep, "prehashed")

            c_dev, c_host = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
            r_dev = lib.edc_batch_verify_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                                off.data_ptr(), None, 0, d_z.data_ptr(), c_dev)
            r_host = lib.edc_batch_verify_z(eng.ctx, n, hv, hs, hm, ho, z, c_host)
            assert (r_host, c_host.raw) == (r_dev, c_dev.raw) and r_dev == want, (rep, "caller z")
            c_host = ctypes.create_string_buffer(32)
            r_host = lib.edc_batch_verify_prehashed(eng.ctx, n, hv, hs, kb.raw, None, z, c_host)
            assert (r_host, c_host.raw) == (r_dev, c_dev.raw), (rep, "prehashed, caller z")
    finally:
        eng.close()


def test_host_chunked_small_and_empty(engine):
    """below the threshold (one piece) and the empty batch: unchanged behaviour"""
    lib = engine.lib
    c8 = ctypes.create_string_buffer(32)
    assert lib.edc_batch_verify_prehashed(engine.ctx, 0, b"\0", b"\0", b"\0", bytes(32), None, c8) == 0
    assert c8.raw == bytes([1]) + bytes(31)


HOST_SOAK = int(os.environ.get("EDC_HOSTCHUNK_SOAK", "0"))


@pytest.mark.parametrize("case", range(HOST_SOAK or 3))
def test_random_host_chunked_equals_device(env, case):
    """random n (chunk counts 1..7 plus the last chunk, ragged edges), validators or distinct keys,
    message lengths, corruption and key-grouping mode; EDC_HOSTCHUNK_SOAK=<k> for a soak run"""
    import random
    torch, bench, edc = env
    rnd = random.Random(4242 + case)
    n = rnd.randrange(1 << 16, 1 << 21 if case % 4 == 3 else 1 << 19)
    keys = rnd.choice([150, 0, rnd.randrange(1, 5000)])
    mlen = rnd.choice([-1, 0, 32, 120, rnd.randrange(1, 400)])
    kind = rnd.choice(["none", "wrong_sig", "bad_r_and_s"])
    grouping = rnd.choice([0, 0, 1, 3])
    eng = edc.Engine(0)
    try:
        eng.set_key_grouping(grouping)
        vk, sig, msg, off = _workload(env, eng, n, keys, mlen)
        if kind == "wrong_sig" and mlen == 0:
            kind = "bad_r_and_s"
        _corrupt(kind, vk, sig, msg, off, n)
        hv, hs, hm, ho = _host_copies(vk, sig, msg, off, n, shift=rnd.randrange(0, 40))
        lib = eng.lib
        zseed = rnd.randbytes(32)
        kb = ctypes.create_string_buffer(32 * n)
        eng._check(lib.edc_challenge(eng.ctx, n, hv, hs, hm, ho, kb))
        d_k = torch.frombuffer(bytearray(kb.raw), dtype=torch.uint8).to("cuda:0")
        torch.cuda.synchronize()
        want = 0 if kind == "none" else 1
        tag = (case, n, keys, mlen, kind, grouping)
        for rep in range(2):
            c_dev, c_host = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
            r_dev = lib.edc_batch_verify_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                                off.data_ptr(), zseed, 0, None, c_dev)
            r_host = lib.edc_batch_verify(eng.ctx, n, hv, hs, hm, ho, zseed, c_host)
            assert (r_host, c_host.raw) == (r_dev, c_dev.raw) and r_dev == want, (tag, rep, "messages")
            c_dev, c_host = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
            r_dev = lib.edc_batch_verify_prehashed_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), d_k.data_ptr(),
                                                          zseed, 0, None, c_dev)
            r_host = lib.edc_batch_verify_prehashed(eng.ctx, n, hv, hs, kb.raw, zseed, None, c_host)
            assert (r_host, c_host.raw) == (r_dev, c_dev.raw) and r_dev == want, (tag, rep, "prehashed")
    finally:
        eng.close()
