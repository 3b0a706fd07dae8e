"""One batch at a time: the latency a node sees when it verifies one block and waits for the
verdict before the next (reference src/batch.rs:149-217, one `verify` call). Times the synchronous
device entry edc_batch_verify_device (slot 0: the decode runs on a second stream beside SHA-512 /
coefficients / binning) and one pipelined-slot batch (edc_batch_submit_device + edc_batch_wait)
for each workload, median over --reps calls after --warmup calls, inputs already in HBM.
  python tools/latency_probe.py [--reps 20] [--warmup 3] [--sizes c3,n17,c2]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

SHAPES = {"c3": (1 << 20, 150, 120), "n17": (1 << 17, 150, 120), "n18": (1 << 18, 150, 120),
          "c2": (1 << 16, 0, 32), "n1024": (1024, 150, 120), "n150": (150, 150, 120)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sizes", default="c3,n17,c2")
    ap.add_argument("--lib", default=None, help="A/B build of libedc.so (measurement only)")
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0, lib_path=a.lib)
    lib = eng.lib
    zseed = bytes([0x33]) * 32
    for name in a.sizes.split(","):
        n, keys, mlen = SHAPES[name]
        vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, keys, mlen, 0)
        torch.cuda.synchronize()
        args = (eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(), zseed, 0)

        def sync_call():
            rc = lib.edc_batch_verify_device(*args, None, None)
            assert rc == 0, rc

        def slot_call():
            t = lib.edc_batch_submit_device(*args, None, 0)
            eng._check(t)
            assert eng._check(lib.edc_batch_wait(eng.ctx, t, None, None, None)) == 0

        out = {"workload": name, "n": n, "validators": keys or "distinct", "msg_len": mlen}
        for label, fn in (("sync_ms", sync_call), ("slot_ms", slot_call)):
            # every slot's first batch allocates its workspace: the pipelined call rotates over all
            # 16 slots, so its warmup touches each of them
            for _ in range(a.warmup if fn is sync_call else a.warmup + 16):
                fn()
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                fn()
                ts.append((time.perf_counter() - t0) * 1e3)
            out[label] = round(statistics.median(ts), 4)
            out[label + "_min"] = round(min(ts), 4)
        out["sync_sigs_per_s"] = round(n / (out["sync_ms"] * 1e-3), 1)
        print(json.dumps(out), flush=True)
        del vk, sig, msg, off
    eng.close()


if __name__ == "__main__":
    main()
