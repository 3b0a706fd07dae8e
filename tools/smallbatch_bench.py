"""Small-batch regime, the shape of the reference's own criterion bench (benches/bench.rs:25-71):
n in {8, 16, ..., 64} with empty messages, "Unbatched verification", "Signatures with Distinct
Pubkeys" and "Signatures with the Same Pubkey" -- plus n = 150 (one consensus commit) and 1024
(configs[0]).

GPU: synchronous latency of one call through the C ABI (median of --reps), host buffers in and out:
  batch       edc_batch_verify (Verifier::queue x n + verify)
  batch_dev   edc_batch_verify_device (inputs already in HBM)
  unbatched   edc_verify_each (VerificationKey::try_from + verify per item)
CPU: the oracle's C restatement of the reference algorithm (oracle/edc_oracle.c) on ONE thread,
the same inputs, queue+verify (batched) or try_from+verify per item (unbatched) -- a port, not the
Rust reference (no toolchain here). Prints one JSON line per (n, kind) and a summary line with the
crossover: the smallest n at which the GPU batch call beats one CPU thread.
  python tools/smallbatch_bench.py [--reps 50]"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--sizes", default="8,16,24,32,40,48,56,64,150,1024")
    ap.add_argument("--lib", default=None, help="A/B build of libedc.so (measurement only)")
    ap.add_argument("--keycache", action="store_true",
                    help="register the batch's keys in the context's key cache first (a node's validator set)")
    args = ap.parse_args()
    import torch
    import bench
    import oracle_c  # CPU baseline leg only
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0, lib_path=args.lib)
    lib = eng.lib
    sizes = [int(x) for x in args.sizes.split(",")]
    nmax = max(sizes)
    distinct_seeds = [bytes([(i >> 8) & 255, i & 255]) * 16 for i in range(nmax)]
    out = []

    def med_ms(fn):
        fn()                                       # warm (workspace growth, first launch)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e3)
        return statistics.median(ts)

    for kind in ("distinct", "same"):
        msgs = [b""] * nmax
        if kind == "distinct":
            vks, sigs = eng.sign(distinct_seeds, msgs)
        else:
            vks, sigs = eng.sign([bytes([7]) * 32], msgs, seed_index=[0] * nmax)
        if args.keycache:
            eng.keycache_load(list(dict.fromkeys(vks)))
        for n in sizes:
            v, s, m = vks[:n], sigs[:n], msgs[:n]
            zs = bytes([0x33]) * 32
            assert eng.batch_verify(v, s, m, z_seed=zs)[0] == 0
            t_batch = med_ms(lambda: eng.batch_verify(v, s, m, z_seed=zs))
            d_vk = torch.tensor(list(b"".join(v)), dtype=torch.uint8, device=dev)
            d_sig = torch.tensor(list(b"".join(s)), dtype=torch.uint8, device=dev)
            d_msg = torch.zeros(1, dtype=torch.uint8, device=dev)
            d_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            t_dev = med_ms(lambda: eng._check(lib.edc_batch_verify_device(
                eng.ctx, n, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), zs, 0, None,
                None)))
            row = {"n": n, "keys": kind, "keycache": args.keycache, "gpu_batch_ms": round(t_batch, 4),
                   "gpu_batch_dev_ms": round(t_dev, 4),
                   "gpu_batch_sigs_per_s": round(n / t_batch * 1e3, 1),
                   "cpu1_batch": oracle_c.bench_small(v, s, m, True)}
            if kind == "distinct":
                assert eng.verify_each(v, s, m) == [0] * n
                t_each = med_ms(lambda: eng.verify_each(v, s, m))
                row["gpu_unbatched_ms"] = round(t_each, 4)
                row["cpu1_unbatched"] = oracle_c.bench_small(v, s, m, False)
            row["gpu_over_cpu1_batch"] = round(row["gpu_batch_sigs_per_s"] / row["cpu1_batch"]["sigs_per_s"], 3)
            out.append(row)
            print(json.dumps(row), flush=True)
    cross = {}
    for kind in ("distinct", "same"):
        win = [r["n"] for r in out if r["keys"] == kind and r["gpu_over_cpu1_batch"] >= 1.0]
        cross[kind] = min(win) if win else None
    print(json.dumps({"summary": "crossover: smallest n where one GPU batch call beats one CPU thread",
                      "crossover_n": cross}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
