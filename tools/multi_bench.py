"""Pipelined multi-device path (include/edc.h edc_multi_submit_device / edc_multi_wait) against
one context's pipelined rate, on the same box and workload (configs[2]: 2^20 votes from 150
validators, 120-byte messages). On a one-GPU box the device list repeats device 0 (K contexts on
one GPU): the numbers then show the cost of the multi-device machinery (shard submissions, device-
to-device partial copies, combine on the first device), not a scaling curve.
Usage (GPU box): python tools/multi_bench.py [--devices 0,0,0,0] [--n 1048576] [--steps 30] [--inflight 6]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="0,0,0,0")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--inflight", type=int, default=6)
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0)
    n = a.n
    vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, 150, 120, 0)
    torch.cuda.synchronize()
    zs = bytes([0x33]) * 32
    lib = eng.lib

    def pipelined(submit, wait, k):
        pend = []
        for _ in range(k):
            if len(pend) >= a.inflight:
                assert wait(pend.pop(0)) == 0
            pend.append(submit())
        while pend:
            assert wait(pend.pop(0)) == 0

    def timed(submit, wait):
        pipelined(submit, wait, a.warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipelined(submit, wait, a.steps)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    eng._check(lib.edc_reserve(eng.ctx, n))
    single = timed(lambda: eng._check(lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(),
                                                                 msg.data_ptr(), off.data_ptr(), zs, 0, None, 0)),
                   lambda t: eng._check(lib.edc_batch_wait(eng.ctx, t, None, None, None)))
    devices = [int(x) for x in a.devices.split(",")]
    G = len(devices)
    eng.close()                     # its slot streams (hardware queues) go before the multi contexts come
    m = pkg.MultiEngine(devices)
    offs, shards = [], []
    for g in range(G):
        lo, hi = n * g // G, n * (g + 1) // G
        o = (off[lo:hi + 1] - off[lo]).contiguous()
        offs.append(o)
        shards.append((hi - lo, vk.data_ptr() + 32 * lo, sig.data_ptr() + 64 * lo, msg.data_ptr() + int(off[lo].item()),
                       o.data_ptr()))
    for g in range(G):
        c = lib.edc_multi_context(m.m, g)
        assert lib.edc_reserve(c, n // G + 1) == 0
    multi = timed(lambda: m.batch_submit_device(shards, zs), lambda t: m.batch_wait(t)[0])
    m.close()
    print(json.dumps({"n": n, "devices": devices, "inflight": a.inflight, "steps": a.steps,
                      "single_ctx_ms_per_batch": round(single * 1e3, 4), "single_ctx_sigs_per_s": round(n / single, 1),
                      "multi_ms_per_batch": round(multi * 1e3, 4), "multi_sigs_per_s": round(n / multi, 1),
                      "multi_over_single": round(single / multi, 4)}), flush=True)


if __name__ == "__main__":
    main()
