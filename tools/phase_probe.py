"""Per-phase device times (HIP events, one batch at a time) of a library build on a BASELINE
config, WITHOUT checking verdicts: for cost probes of experimental builds that deliberately skip
work (never for results). python tools/phase_probe.py --lib PATH [--config c3] [--batches 8]"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--batches", type=int, default=8)
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0, lib_path=args.lib)
    n, keys, msg_len, _ = bench.CONFIGS[args.config]
    vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, keys, msg_len, 0)
    torch.cuda.synchronize()
    lib = eng.lib
    names = [lib.edc_timing_name(i).decode() for i in range(7)]
    lib.edc_set_timing(eng.ctx, 1)
    acc = {k: [] for k in names}
    buf = (ctypes.c_float * 7)()
    for b in range(args.batches):
        t = lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                        bytes([0x33]) * 32, 0, None, 0)
        eng._check(t)
        lib.edc_batch_wait(eng.ctx, t, None, None, None)
        lib.edc_last_timings(eng.ctx, buf, 7)
        if b >= 2:
            for i, k in enumerate(names):
                acc[k].append(buf[i])
    print(os.path.basename(args.lib), " ".join(f"{k}={statistics.median(v):.4f}" for k, v in acc.items()), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
