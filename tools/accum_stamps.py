"""Per-workgroup phase times of k_msm_accum_dma from the diagnostic build's shader-clock stamps
(csrc: make variant VARIANT=stamps VFLAGS=-DEDC_STAMPS -> libedc_stamps.so; results unchanged).
Runs a few batches of a BASELINE config one at a time, then reads the stamps of the last batch:
per bin, the counting sort, the accumulation rounds and the head resolution (stamps 0-3), plus
the kernel span and how many workgroups were resident at once.
  python tools/accum_stamps.py [--config c2] [--window-bits B] [--msm-parts P]"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--window-bits", type=int, default=0)
    ap.add_argument("--msm-parts", type=int, default=0)
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--n", type=int, default=0, help="override the config's batch size (e.g. 150: a small call)")
    ap.add_argument("--keys", type=int, default=-1, help="override the config's validator count (0 = distinct)")
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    lib_path = os.path.join(ROOT, "ed25519-consensus_amd", "csrc", "libedc_stamps.so")
    eng = pkg.Engine(0, lib_path=lib_path)
    n, keys, msg_len, desc = bench.CONFIGS[args.config]
    if args.n:
        n, desc = args.n, f"{desc}, n overridden to {args.n}"
    if args.keys >= 0:
        keys = args.keys
    vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, keys, msg_len, 0)
    torch.cuda.synchronize()
    lib = eng.lib
    eng._check(lib.edc_set_msm_shape(eng.ctx, args.window_bits, args.msm_parts))
    zseed = bytes([0x33]) * 32
    for _ in range(args.batches):
        t = lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                        zseed, 0, None, 0)
        eng._check(t)
        assert eng._check(lib.edc_batch_wait(eng.ctx, t, None, None, None)) == 0
    nb = 8192
    buf = (ctypes.c_uint64 * (nb * 8))()
    lib.edc_debug_acc_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.edc_debug_acc_stamps(buf, ctypes.sizeof(buf)) == 0
    rows = [tuple(buf[8 * b:8 * b + 8]) for b in range(nb)]
    # every bin of the last batch (same plan each batch, so its stamps overwrote the earlier ones);
    # s_memtime runs per XCD, so only differences within one workgroup are used; the span and the
    # residency come from s_memrealtime (100 MHz, chip-wide)
    rows = [r for r in rows if r[0] and r[3] >= r[0] and r[6] >= r[5]]
    r0 = min(r[5] for r in rows)
    rt = max(r[6] for r in rows) - r0
    live = [r for r in rows if r[7] > 0]
    clk_ghz = statistics.median([(r[3] - r[0]) / ((r[6] - r[5]) / 100e6) / 1e9 for r in live if r[6] > r[5]])

    def st(vals):
        vals = sorted(vals)
        return {"median": vals[len(vals) // 2], "p90": vals[int(len(vals) * 0.9)], "max": vals[-1]}

    # residency: workgroups running at the middle of the span
    mid = r0 + rt // 2
    resident = sum(1 for r in rows if r[5] <= mid <= r[6])
    out = {
        "config": args.config, "desc": desc, "bins": len(rows), "live_bins": len(live),
        "span_us": round(rt / 100.0, 1), "clock_ghz": round(clk_ghz, 3),
        "resident_at_mid": resident,
        "entries": st([r[7] for r in live]),
        "sort_cycles": st([r[1] - r[0] for r in live]),
        "accum_cycles": st([r[2] - r[1] for r in live]),
        "heads_cycles": st([r[3] - r[2] for r in live]),
        "total_cycles": st([r[3] - r[0] for r in live]),
        "accum_cycles_per_round": st([(r[2] - r[1]) / max(1, (r[7] + 255) // 256) for r in live]),
        "start_us": st([(r[5] - r0) / 100.0 for r in live]),
        "end_us": st([(r[6] - r0) / 100.0 for r in live]),
    }
    print(json.dumps(out, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
