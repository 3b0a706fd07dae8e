"""How many in-flight batches does the GPU actually run at once? Submits K batches back to back
(no waits; each goes to its own slot stream / hardware queue), then waits for all of them, and
reports the wall time per burst and per batch for K = 1..8. If the chains overlapped freely, the
burst time would stay near one batch's latency until the VALU work saturates the chip; if only a
few hardware queues are serviced at once, it grows in steps of the queue count.
Usage (GPU box): python tools/burst_probe.py [--n 131072] [--keys 150] [--reps 5]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 17)
    ap.add_argument("--keys", type=int, default=150)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ks", default="1,2,3,4,5,6,8")
    ap.add_argument("--lib", default=None, help="A/B build of libedc.so (measurement only)")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0, lib_path=a.lib)
    lib = eng.lib
    zseed = bytes([0x33]) * 32
    n = a.n
    vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, a.keys, 120 if a.keys else 32, 0)
    torch.cuda.synchronize()
    eng._check(lib.edc_reserve(eng.ctx, n))

    def burst(k):
        t0 = time.perf_counter()
        ts = []
        for _ in range(k):
            t = lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                            zseed, 0, None, 0)
            eng._check(t)
            ts.append(t)
        t_sub = time.perf_counter() - t0
        for t in ts:
            assert eng._check(lib.edc_batch_wait(eng.ctx, t, None, None, None)) == 0
        return time.perf_counter() - t0, t_sub

    for _ in range(3):
        burst(8)
    for k in [int(x) for x in a.ks.split(",")]:
        res = sorted(burst(k) for _ in range(a.reps))
        wall, sub = res[len(res) // 2]
        print(json.dumps({"n": n, "keys": a.keys, "k": k, "burst_ms": round(wall * 1e3, 4),
                          "ms_per_batch": round(wall * 1e3 / k, 4), "submit_ms_total": round(sub * 1e3, 4)}),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
