"""GPU: the synchronous host-buffer calls under their two environment switches, which the engine
reads once per process (so each runs in a child process of its own): EDC_HOST_COPY_THREADS=1 (the
k / message chunks copied by the calling thread after each signature chunk instead of by a second
copying thread) and EDC_HOST_CHUNKS=0 (no chunking: the one-piece copy, then the batch). Both must
give the device-resident path's verdict and [8]*check byte for byte (edc_batch_verify and
edc_batch_verify_prehashed against edc_batch_verify_device / _prehashed_device on the same inputs
and z seed), for a valid vote batch and one with a wrong signature in the last chunk. Reference:
src/batch.rs:149-217 (Verifier::verify over host-held items)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import ctypes, json, sys
sys.path.insert(0, ROOT)
import torch
import bench
pkg = bench.load_pkg()
eng = pkg.Engine(0)
dev = torch.device("cuda:0")
n = 70001
vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, 150, 120, 0)
torch.cuda.synchronize()
lib = eng.lib
zseed = bytes([0x5A]) * 32
out = []
for corrupt in (False, True):
    if corrupt:
        o = int(off[n - 3])
        msg[o] ^= 1
        torch.cuda.synchronize()
    hv = vk[:32 * n].cpu().numpy().tobytes()
    hs = sig[:64 * n].cpu().numpy().tobytes()
    o = off[:n + 1].cpu().numpy().astype("uint64")
    hm = msg[int(o[0]):int(o[-1])].cpu().numpy().tobytes() + b"\0"
    o = o - o[0]
    ho = (ctypes.c_uint64 * (n + 1)).from_buffer_copy(o.tobytes())
    kb = ctypes.create_string_buffer(32 * n)
    eng._check(lib.edc_challenge(eng.ctx, n, hv, hs, hm, ho, kb))
    d_k = torch.frombuffer(bytearray(kb.raw), dtype=torch.uint8).to(dev)
    torch.cuda.synchronize()
    row = {}
    for name, call in (
        ("dev", lambda c: lib.edc_batch_verify_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                                      off.data_ptr(), zseed, 0, None, c)),
        ("host", lambda c: lib.edc_batch_verify(eng.ctx, n, hv, hs, hm, ho, zseed, c)),
        ("dev_pre", lambda c: lib.edc_batch_verify_prehashed_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(),
                                                                    d_k.data_ptr(), zseed, 0, None, c)),
        ("host_pre", lambda c: lib.edc_batch_verify_prehashed(eng.ctx, n, hv, hs, kb.raw, zseed, None, c)),
    ):
        c8 = ctypes.create_string_buffer(32)
        rc = call(c8)
        row[name] = [rc, c8.raw.hex()]
    out.append(row)
eng.close()
print("RESULT " + json.dumps(out))
"""


@pytest.mark.parametrize("knob", [{"EDC_HOST_COPY_THREADS": "1"}, {"EDC_HOST_CHUNKS": "0"}],
                         ids=["one_copy_thread", "one_piece"])
def test_host_call_knobs_equal_device(edc, knob):
    env = dict(os.environ)
    env.update(knob)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + CHILD], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = next(l for l in r.stdout.splitlines() if l.startswith("RESULT "))
    rows = json.loads(line[len("RESULT "):])
    for want, row in zip((0, 1), rows):
        assert row["host"] == row["dev"] and row["dev"][0] == want, (knob, row)
        assert row["host_pre"] == row["dev_pre"] and row["dev_pre"][0] == want, (knob, row)
        assert row["dev"][1] == row["dev_pre"][1]          # same k, same z: same check point
        if want:
            assert row["dev"][1] not in ("00" * 32, "01" + "00" * 31)
