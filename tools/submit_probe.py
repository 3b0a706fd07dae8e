"""Host-side cost of one batch submission: wall time of edc_batch_submit_device (the enqueue of
one batch's kernels on its slot stream) and of edc_batch_wait, beside the pipelined batch rate,
for several batch sizes. Tells whether small batches are bound by the host's launch rate.
Usage (GPU box): python tools/submit_probe.py [--sizes 65536,131072,1048576] [--inflight 8]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="65536,131072,1048576")
    ap.add_argument("--inflight", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--keys", type=int, default=150)
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0)
    lib = eng.lib
    zseed = bytes([0x33]) * 32
    for n in [int(x) for x in a.sizes.split(",")]:
        vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, a.keys, 120 if a.keys else 32, 0)
        torch.cuda.synchronize()
        eng._check(lib.edc_reserve(eng.ctx, n))
        pend, t_sub, t_wait = [], [], []

        def run(k, rec):
            for _ in range(k):
                if len(pend) >= a.inflight:
                    t0 = time.perf_counter()
                    eng._check(lib.edc_batch_wait(eng.ctx, pend.pop(0), None, None, None))
                    if rec:
                        t_wait.append(time.perf_counter() - t0)
                t0 = time.perf_counter()
                t = lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                                off.data_ptr(), zseed, 0, None, 0)
                if rec:
                    t_sub.append(time.perf_counter() - t0)
                if t < 0:
                    eng._check(t)
                pend.append(t)
            while pend:
                eng._check(lib.edc_batch_wait(eng.ctx, pend.pop(0), None, None, None))

        run(8, False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(a.steps, True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        t_sub.sort()
        t_wait.sort()
        print(json.dumps({"n": n, "inflight": a.inflight, "ms_per_batch": round(el / a.steps * 1e3, 4),
                          "sigs_per_s": round(n * a.steps / el, 1),
                          "submit_ms_median": round(t_sub[len(t_sub) // 2] * 1e3, 4),
                          "submit_ms_max": round(t_sub[-1] * 1e3, 4),
                          "wait_ms_median": round(t_wait[len(t_wait) // 2] * 1e3, 4) if t_wait else None}),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
