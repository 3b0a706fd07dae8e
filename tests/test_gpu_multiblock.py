"""GPU parity for BASELINE configs[4]'s message shape (uniform 0..1024-byte messages, 1-9 SHA-512
blocks per challenge) and configs[1]'s distinct keys, against the C oracle (dalek algorithm):
challenge scalars k = H(R||A||M) mod l for every item, batch verdict and the compressed [8]*check
bit-exact, with and without an invalid item; shards with global z offsets recombine to the same
point (the multi-GPU reduction of configs[4])."""
import ctypes
import hashlib
import os
import random
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

L_ORDER = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def oracle_c():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c as oc
    return oc


def _items(engine, n, seed):
    rnd = random.Random(seed)
    seeds = [rnd.randbytes(32) for _ in range(n)]
    msgs = [rnd.randbytes(rnd.randrange(0, 1025)) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs)
    return list(vks), list(sigs), msgs, rnd


def test_variable_length_challenges(engine):
    vks, sigs, msgs, _ = _items(engine, 3000, 11)
    ks = engine.challenge(vks, sigs, msgs)
    for vk, sig, m, k in zip(vks, sigs, msgs, ks):
        want = int.from_bytes(hashlib.sha512(sig[:32] + vk + m).digest(), "little") % L_ORDER
        assert int.from_bytes(k, "little") == want


@pytest.mark.parametrize("bad", [None, 1234])
def test_variable_length_batch_matches_oracle(engine, oracle_c, bad):
    vks, sigs, msgs, rnd = _items(engine, 6000, 12)
    if bad is not None:
        m = msgs[bad] or b"\0"
        msgs[bad] = bytes([m[0] ^ 1]) + m[1:]
    zseed = rnd.randbytes(32)
    items = list(zip(vks, sigs, msgs))
    exp_code, exp_c8 = oracle_c.batch_verify(items, zseed)
    code, c8 = engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    assert code == exp_code == (0 if bad is None else 1)
    assert c8 == exp_c8


def test_variable_length_shards_recombine(engine, oracle_c):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    vks, sigs, msgs, rnd = _items(engine, 5000, 13)
    msgs[77] = msgs[77] + b"x"                         # one invalid item: a non-identity check point
    zseed = rnd.randbytes(32)
    exp_code, exp_c8 = oracle_c.batch_verify(list(zip(vks, sigs, msgs)), zseed)
    assert exp_code == 1
    for nshards in (2, 4, 8):
        bounds = [len(vks) * s // nshards for s in range(nshards + 1)]
        parts, bad_any = [], 0
        for s in range(nshards):
            lo, hi = bounds[s], bounds[s + 1]
            offs = [0]
            for m in msgs[lo:hi]:
                offs.append(offs[-1] + len(m))
            d_vk = torch.tensor(list(b"".join(vks[lo:hi])), dtype=torch.uint8, device=dev)
            d_sig = torch.tensor(list(b"".join(sigs[lo:hi])), dtype=torch.uint8, device=dev)
            d_msg = torch.tensor(list(b"".join(msgs[lo:hi])) or [0], dtype=torch.uint8, device=dev)
            d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            part = ctypes.create_string_buffer(128)
            flag = ctypes.c_int(0)
            assert engine.lib.edc_batch_partial_device(engine.ctx, hi - lo, d_vk.data_ptr(), d_sig.data_ptr(),
                                                       d_msg.data_ptr(), d_off.data_ptr(), zseed, lo, None, part,
                                                       ctypes.byref(flag)) == 0
            parts.append(part.raw)
            bad_any |= flag.value
        code, c8 = engine.combine_partials(parts, bad_any)
        assert code == exp_code and c8 == exp_c8, nshards


def test_message_window_edges_every_alignment(engine):
    """The LDS-staged message windows of k_challenge at every padding boundary and every arena
    alignment: messages of 0..400 bytes (1 to 4 SHA-512 blocks: every position of the end marker
    and of the length words), the arena placed at byte offsets 0..15 of a device buffer and ending
    at the buffer's last byte. Each item is signed over its message, so the per-item path
    (edc_verify_each_device: SHA-512 on the device, then the single verification) accepts it only
    if k = H(R||A||M) was hashed exactly; the batch over the same arena is Ok with the identity."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    rnd = random.Random(401)
    lens = list(range(0, 401))
    msgs = [rnd.randbytes(n) for n in lens]
    seeds = [rnd.randbytes(32) for _ in range(8)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[i % 8 for i in range(len(msgs))])
    n = len(msgs)
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    arena = b"".join(msgs)
    d_vk = torch.tensor(list(b"".join(vks)), dtype=torch.uint8, device=dev)
    d_sig = torch.tensor(list(b"".join(sigs)), dtype=torch.uint8, device=dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    lib = engine.lib
    for shift in range(16):
        buf = torch.tensor(list(bytes([0xA5]) * shift + arena), dtype=torch.uint8, device=dev)  # arena ends at the last byte
        out = torch.zeros(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        assert lib.edc_verify_each_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), buf.data_ptr() + shift,
                                          d_off.data_ptr(), out.data_ptr()) == 0
        assert out.cpu().tolist() == [0] * n, shift
        c8 = ctypes.create_string_buffer(32)
        assert lib.edc_batch_verify_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), buf.data_ptr() + shift,
                                           d_off.data_ptr(), bytes(32), 0, None, c8) == 0, shift
        assert c8.raw == bytes([1]) + bytes(31)
    # and one altered byte in every message is caught item by item
    bad = bytearray(arena)
    for i in range(n):
        if lens[i]:
            bad[offs[i] + rnd.randrange(lens[i])] ^= 0x01
    buf = torch.tensor(list(bad), dtype=torch.uint8, device=dev)
    out = torch.zeros(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    assert lib.edc_verify_each_device(engine.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), buf.data_ptr(),
                                      d_off.data_ptr(), out.data_ptr()) == 0
    assert out.cpu().tolist() == [0] + [1] * (n - 1)
