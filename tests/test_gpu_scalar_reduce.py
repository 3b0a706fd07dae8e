"""GPU: the device build of the wide scalar reduction (sc25519.h sc_reduce_wide, Scalar::from_hash's
mod-l step, reference src/batch.rs:86-91) on chosen 512-bit inputs, through the test hook
edc_debug_sc_reduce_wide. SHA-512 digests never reach the folds' edge cases (the final add of l
needs a third fold that lands below zero, probability ~2^-120 per digest), so the challenge tests
cannot: here every fold boundary, the negative-remainder family and random values are compared with
Python's x mod l."""
import random

import pytest

pytestmark = pytest.mark.gpu

L = (1 << 252) + 27742317777372353535851937790883648493


def _vectors():
    r = random.Random(21)
    v = [0, 1, L - 1, L, L + 1, 2 * L - 1, 2 * L, 2**252 - 1, 2**252, 2**253, 2**260 - 1, 2**385, 2**511,
         2**512 - 1, ((2**512 - 1) // L) * L, ((2**512 - 1) // L) * L - 1]
    v += [1 << b for b in range(512)] + [(1 << b) - 1 for b in range(1, 513)]
    v += [k * L + d for k in [1, 3, 2**64, 2**130, 2**200, 2**259] for d in [-2, -1, 0, 1, 2]]
    v += [(h << 252) + r.getrandbits(r.randrange(1, 200)) for h in range(1, 600)]   # third fold below zero
    v += [r.getrandbits(512) for _ in range(20000)]
    v += [r.getrandbits(r.randrange(1, 513)) for _ in range(5000)]
    return [x % (1 << 512) for x in v]


def test_sc_reduce_wide_device(engine):
    torch = pytest.importorskip("torch")
    import ctypes
    xs = _vectors()
    n = len(xs)
    dev = torch.device("cuda:0")
    d_in = torch.frombuffer(bytearray(b"".join(x.to_bytes(64, "little") for x in xs)), dtype=torch.uint8).to(dev)
    d_out = torch.zeros(32 * n, dtype=torch.uint8, device=dev)
    rc = engine.lib.edc_debug_sc_reduce_wide(engine.ctx, n, ctypes.c_void_p(d_in.data_ptr()),
                                            ctypes.c_void_p(d_out.data_ptr()))
    assert rc == 0
    out = d_out.cpu().numpy().tobytes()
    bad = [i for i, x in enumerate(xs) if int.from_bytes(out[32 * i:32 * i + 32], "little") != x % L]
    assert not bad, [hex(xs[i]) for i in bad[:4]]


def test_sc_reduce_wide_device_arguments(engine):
    torch = pytest.importorskip("torch")
    import ctypes
    d = torch.zeros(256, dtype=torch.uint8, device=torch.device("cuda:0"))
    p = d.data_ptr()
    assert engine.lib.edc_debug_sc_reduce_wide(engine.ctx, 0, None, None) == 0
    assert engine.lib.edc_debug_sc_reduce_wide(engine.ctx, 1, ctypes.c_void_p(p + 4), ctypes.c_void_p(p + 128)) < 0
    assert engine.lib.edc_debug_sc_reduce_wide(engine.ctx, 1, None, ctypes.c_void_p(p)) < 0
