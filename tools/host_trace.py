"""Where a synchronous host-buffer call spends its time (edc_batch_verify_prehashed at 2^20 votes,
the Rust shim's `Verifier::verify`): raw H2D rates of pageable and pinned host memory for the same
134 MB, then a few calls, meant to run under
  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d <dir> -o ht -- python3 tools/host_trace.py
and read with tools/host_timeline.py (copies and kernels of the last call on one time axis).
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0)
    n, keys, mlen, _ = bench.CONFIGS["c3"]
    vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, keys, mlen, 0)
    torch.cuda.synchronize()
    hv = vk[:32 * n].cpu().numpy().tobytes()
    hs = sig[:64 * n].cpu().numpy().tobytes()
    ho = off[:n + 1].cpu().numpy().astype("uint64")
    hm = msg.cpu().numpy().tobytes()
    optr = ho.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    kb = ctypes.create_string_buffer(32 * n)
    eng._check(eng.lib.edc_challenge(eng.ctx, n, hv, hs, hm, optr, kb))
    hk = kb.raw
    # raw copy rates of the same bytes (torch's H2D of a pageable / pinned CPU tensor)
    blob = torch.frombuffer(bytearray(hv + hs + hk), dtype=torch.uint8)
    pinned = blob.pin_memory()
    for name, src in (("pageable", blob), ("pinned", pinned)):
        for _ in range(2):
            src.to(dev)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            src.to(dev, non_blocking=(name == "pinned"))
        torch.cuda.synchronize()
        el = (time.perf_counter() - t) / 5
        print(f"h2d {name}: {blob.numel() / 1e6:.1f} MB in {el * 1e3:.3f} ms = {blob.numel() / el / 1e9:.1f} GB/s",
              flush=True)
    lib = eng.lib
    zseed = bytes([0x33]) * 32
    for i in range(6):
        t = time.perf_counter()
        eng._check(lib.edc_batch_verify_prehashed(eng.ctx, n, hv, hs, hk, zseed, None, None))
        print(f"call {i}: {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
