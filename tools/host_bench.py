"""Host-resident (PCIe-inclusive) batch verification rate: `edc_batch_verify` with the inputs in
host memory, as a Rust caller would hand them over (src/batch.rs:149 `Verifier::verify`). Each
call uploads vk / sig / message arena / offsets to the context's staging buffers and runs the
batch synchronously. This is NOT bench.py's `value` (inputs resident in HBM); DESIGN.md quotes it
next to the device-resident rate.

  python tools/host_bench.py [--config c3] [--steps 10] [--inflight 4]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--inflight", type=int, default=4)
    args = ap.parse_args()
    n, keys, msg_len, desc = bench.CONFIGS[args.config]
    import torch
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0)
    vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, keys, msg_len, 0)
    torch.cuda.synchronize()
    zseed = bytes([0x33]) * 32
    lib = eng.lib
    # the streamed runs rotate over `inflight` slots; each slot's workspace and host-staging
    # buffers are allocated on its first use, so the warmup touches every slot before timing
    eng._check(lib.edc_set_slots(eng.ctx, args.inflight))
    eng._check(lib.edc_reserve(eng.ctx, n))
    args.warmup = max(args.warmup, args.inflight)
    out = {"config": desc, "n": n}
    for kind in ("pageable", "pinned"):
        pin = kind == "pinned"
        hv, hs, hm, ho = (t.cpu().pin_memory() if pin else t.cpu() for t in (vk, sig, msg, off))
        ptr = lambda t: ctypes.cast(ctypes.c_void_p(t.data_ptr()), ctypes.c_char_p)   # borrowed, not copied
        optr = ctypes.cast(ctypes.c_void_p(ho.data_ptr()), ctypes.POINTER(ctypes.c_uint64))

        def step():
            rc = lib.edc_batch_verify(eng.ctx, n, ptr(hv), ptr(hs), ptr(hm), optr, zseed, None)
            assert rc == 0, f"valid synthetic batch rejected: {rc} {eng.lib.edc_last_error(eng.ctx)}"

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        el = time.perf_counter() - t0
        nbytes = hv.numel() + hs.numel() + hm.numel() + ho.numel() * 8
        out[kind] = {"sigs_per_s": round(n * args.steps / el, 1), "ms_per_batch": round(el / args.steps * 1e3, 3),
                     "h2d_bytes_per_batch": nbytes, "bytes_per_sig": round(nbytes / n, 1)}

        # streaming: edc_batch_submit with 4 batches in flight, so batch i+1's PCIe copy runs
        # under the kernels of batches i, i-1, ...
        pending = []

        def wait_oldest():
            rc = lib.edc_batch_wait(eng.ctx, pending.pop(0), None, None, None)
            assert rc == 0, f"valid synthetic batch rejected: {rc} {eng.lib.edc_last_error(eng.ctx)}"

        def stream(k):
            for _ in range(k):
                if len(pending) >= args.inflight:
                    wait_oldest()
                t = lib.edc_batch_submit(eng.ctx, n, ptr(hv), ptr(hs), ptr(hm), optr, zseed, 0, 0)
                assert t >= 0, eng.lib.edc_last_error(eng.ctx)
                pending.append(t)
            while pending:
                wait_oldest()

        stream(args.warmup)
        t0 = time.perf_counter()
        stream(args.steps)
        el = time.perf_counter() - t0
        out[kind + "_streamed"] = {"sigs_per_s": round(n * args.steps / el, 1),
                                   "ms_per_batch": round(el / args.steps * 1e3, 3), "inflight": args.inflight}
    # prehashed items (the reference's Item {vk_bytes, sig, k}, src/batch.rs:76-80): k computed
    # once before timing (at Item::from), then 128 B per item cross PCIe and SHA-512 is skipped
    ho_all = off.cpu()
    offs = (ctypes.c_uint64 * (n + 1)).from_buffer_copy(ho_all.numpy().astype("uint64").tobytes())
    kbuf = ctypes.create_string_buffer(32 * n)
    hv0, hs0 = vk[:32 * n].cpu(), sig[:64 * n].cpu()
    eng._check(lib.edc_challenge(eng.ctx, n, hv0.numpy().tobytes(), hs0.numpy().tobytes(), msg.cpu().numpy().tobytes(),
                                 offs, kbuf))
    k_host = torch.frombuffer(bytearray(kbuf.raw), dtype=torch.uint8)
    for kind in ("pageable", "pinned"):
        pin = kind == "pinned"
        hv, hs, hk = (t.pin_memory() if pin else t for t in (hv0, hs0, k_host))
        ptr = lambda t: ctypes.cast(ctypes.c_void_p(t.data_ptr()), ctypes.c_char_p)

        def step_pre():
            rc = lib.edc_batch_verify_prehashed(eng.ctx, n, ptr(hv), ptr(hs), ptr(hk), zseed, None, None)
            assert rc == 0, f"valid prehashed batch rejected: {rc} {eng.lib.edc_last_error(eng.ctx)}"

        for _ in range(args.warmup):
            step_pre()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_pre()
        el = time.perf_counter() - t0
        nbytes = hv.numel() + hs.numel() + hk.numel()
        out[kind + "_prehashed"] = {"sigs_per_s": round(n * args.steps / el, 1),
                                    "ms_per_batch": round(el / args.steps * 1e3, 3), "bytes_per_sig": round(nbytes / n, 1)}
        pending = []

        def stream_pre(k):
            for _ in range(k):
                if len(pending) >= args.inflight:
                    rc = lib.edc_batch_wait(eng.ctx, pending.pop(0), None, None, None)
                    assert rc == 0, rc
                t = lib.edc_batch_submit_prehashed(eng.ctx, n, ptr(hv), ptr(hs), ptr(hk), zseed, 0, 0)
                assert t >= 0, eng.lib.edc_last_error(eng.ctx)
                pending.append(t)
            while pending:
                rc = lib.edc_batch_wait(eng.ctx, pending.pop(0), None, None, None)
                assert rc == 0, rc

        stream_pre(args.warmup)
        t0 = time.perf_counter()
        stream_pre(args.steps)
        el = time.perf_counter() - t0
        out[kind + "_streamed_prehashed"] = {"sigs_per_s": round(n * args.steps / el, 1),
                                             "ms_per_batch": round(el / args.steps * 1e3, 3),
                                             "bytes_per_sig": round(nbytes / n, 1), "inflight": args.inflight}
    # key-indexed streaming (edc_batch_submit_indexed): the validator set registered once, votes
    # carry a 4-byte validator index instead of the 32-byte key
    if keys > 0:
        kb = bytes(vk[:32 * keys].cpu().tolist())
        eng.keycache_load([kb[32 * i:32 * i + 32] for i in range(keys)])
        import numpy as np
        idx = torch.from_numpy((np.arange(n, dtype=np.int64) % keys).astype(np.uint32).view(np.int32))
        iptr = ctypes.cast(ctypes.c_void_p(idx.data_ptr()), ctypes.POINTER(ctypes.c_uint32))
        hs, hm, ho = sig.cpu(), msg.cpu(), off.cpu()
        ptr = lambda t: ctypes.cast(ctypes.c_void_p(t.data_ptr()), ctypes.c_char_p)
        optr = ctypes.cast(ctypes.c_void_p(ho.data_ptr()), ctypes.POINTER(ctypes.c_uint64))
        pending = []

        def stream_idx(k):
            for _ in range(k):
                if len(pending) >= args.inflight:
                    rc = lib.edc_batch_wait(eng.ctx, pending.pop(0), None, None, None)
                    assert rc == 0, rc
                t = lib.edc_batch_submit_indexed(eng.ctx, n, iptr, ptr(hs), ptr(hm), optr, zseed, 0, 0)
                assert t >= 0, eng.lib.edc_last_error(eng.ctx)
                pending.append(t)
            while pending:
                rc = lib.edc_batch_wait(eng.ctx, pending.pop(0), None, None, None)
                assert rc == 0, rc

        stream_idx(args.warmup)
        t0 = time.perf_counter()
        stream_idx(args.steps)
        el = time.perf_counter() - t0
        nbytes = 4 * n + hs.numel() + hm.numel() + ho.numel() * 8
        out["pageable_streamed_key_indexed"] = {"sigs_per_s": round(n * args.steps / el, 1),
                                                "ms_per_batch": round(el / args.steps * 1e3, 3),
                                                "bytes_per_sig": round(nbytes / n, 1), "inflight": args.inflight,
                                                "note": "keys registered once (edc_keycache_load) outside the timing"}
        # prehashed and key-indexed (edc_batch_submit_prehashed_indexed): 4 + 64 + 32 bytes per vote
        kptr = ptr(k_host)

        def stream_pidx(k):
            for _ in range(k):
                if len(pending) >= args.inflight:
                    rc = lib.edc_batch_wait(eng.ctx, pending.pop(0), None, None, None)
                    assert rc == 0, rc
                t = lib.edc_batch_submit_prehashed_indexed(eng.ctx, n, iptr, ptr(hs), kptr, zseed, 0, 0)
                assert t >= 0, eng.lib.edc_last_error(eng.ctx)
                pending.append(t)
            while pending:
                rc = lib.edc_batch_wait(eng.ctx, pending.pop(0), None, None, None)
                assert rc == 0, rc

        stream_pidx(args.warmup)
        t0 = time.perf_counter()
        stream_pidx(args.steps)
        el = time.perf_counter() - t0
        out["pageable_streamed_prehashed_key_indexed"] = {
            "sigs_per_s": round(n * args.steps / el, 1), "ms_per_batch": round(el / args.steps * 1e3, 3),
            "bytes_per_sig": round((4 * n + hs.numel() + k_host.numel()) / n, 1), "inflight": args.inflight,
            "note": "keys registered once (edc_keycache_load) outside the timing"}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
