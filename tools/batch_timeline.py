"""Device-side timeline of a pipelined bench run, without a profiler: the EDC_BATCH_STAMPS build
(`make -C ed25519-consensus_amd/csrc variant VARIANT=bstamps VFLAGS=-DEDC_BATCH_STAMPS`) stamps
each batch's phase starts with the GPU's 100 MHz realtime counter (edc_common.h BST_*), and this
script runs bench.py's timed loop (W warmup steps, then K timed steps with F batches in flight)
and prints, per batch, the host submit time and the device phase times, then how many batches sit
in each phase over the run (50 us bins), so that the fill and the drain of a short run are
visible. rocprofv3's kernel trace is not usable for this: its per-dispatch interception makes
the host ~0.35 ms per submission, slower than a 2^17 batch.
  python tools/batch_timeline.py --lib ed25519-consensus_amd/csrc/libedc_bstamps.so [--n 131072]
      [--steps 20] [--warmup 5] [--inflight 16] [--bin-us 50]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

PHASES = ["init", "coef", "count", "decode", "accum", "reduce", "final", "end"]
REC = 4 + len(PHASES)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--n", type=int, default=1 << 17)
    ap.add_argument("--keys", type=int, default=150)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--inflight", type=int, default=16)
    ap.add_argument("--bin-us", type=float, default=50.0)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0, lib_path=a.lib)
    lib = eng.lib
    lib.edc_debug_batch_stamps.restype = ctypes.c_int
    lib.edc_debug_batch_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    n = a.n
    vk, sig, msg, off = bench.make_workload(pkg, eng, torch, dev, n, a.keys, 120 if a.keys else 32, 0)
    torch.cuda.synchronize()
    eng._check(lib.edc_set_slots(eng.ctx, a.inflight))
    eng._check(lib.edc_reserve(eng.ctx, n))
    zseed = bytes([0x33]) * 32
    pend = []

    def run(k):
        for _ in range(k):
            if len(pend) >= a.inflight:
                eng._check(lib.edc_batch_wait(eng.ctx, pend.pop(0), None, None, None))
            t = lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                            zseed, 0, None, 0)
            eng._check(t)
            pend.append(t)
        while pend:
            eng._check(lib.edc_batch_wait(eng.ctx, pend.pop(0), None, None, None))

    for rep in range(a.reps):
        run(a.warmup)
        lib.edc_debug_batch_stamps(None, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(a.steps)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        buf = (ctypes.c_uint32 * (REC * a.steps))()
        cnt = lib.edc_debug_batch_stamps(buf, REC * a.steps)
        recs = [list(buf[REC * i:REC * (i + 1)]) for i in range(cnt)]
        g0 = min(r[4] for r in recs)
        h0 = min(r[2] for r in recs)
        # device stamps: 10 ns ticks (100 MHz), 32-bit wrap handled relative to the first init
        dv = [[((x - g0) & 0xFFFFFFFF) / 100.0 for x in r[4:]] for r in recs]
        hs = [((r[2] - h0) & 0xFFFFFFFF) for r in recs]
        hw = [((r[3] - h0) & 0xFFFFFFFF) for r in recs]
        span = max(d[-1] for d in dv)
        print(f"# rep {rep}: n={n} steps={a.steps} inflight={a.inflight}: host {el * 1e3:.3f} ms "
              f"({n * a.steps / el:.4e} sigs/s); device span first init -> last end {span / 1e3:.3f} ms")
        print("batch  submit_us  " + " ".join(f"{p:>8s}" for p in PHASES) + "  wait_ret_us")
        for i, (d, s, w) in enumerate(zip(dv, hs, hw)):
            print(f"{i:5d} {s:10d}  " + " ".join(f"{x:8.1f}" for x in d) + f"  {w:10d}")
        # batches per phase over time
        nb = int(span // a.bin_us) + 1
        names = ["pre", "decode", "accum", "reduce+win", "final"]
        bounds = [(0, 3), (3, 4), (4, 5), (5, 6), (6, 7)]
        occ = [[0.0] * nb for _ in names]
        for d in dv:
            for k, (lo, hi) in enumerate(bounds):
                s0, s1 = d[lo], d[hi]
                b = int(s0 // a.bin_us)
                while b < nb and b * a.bin_us < s1:
                    ov = min(s1, (b + 1) * a.bin_us) - max(s0, b * a.bin_us)
                    if ov > 0:
                        occ[k][b] += ov / a.bin_us
                    b += 1
        print(f"batches in each phase per {a.bin_us:.0f} us bin (time-weighted):")
        print("   t_us " + " ".join(f"{x:>10s}" for x in names))
        for b in range(nb):
            print(f"{b * a.bin_us:7.0f} " + " ".join(f"{occ[k][b]:10.2f}" for k in range(len(names))))
        # summary: phase totals and where the last decode / accumulation end
        tot = {p: sum(d[k + 1] - d[k] for d in dv) / len(dv) for k, p in enumerate(PHASES[:-1])}
        last_dec_end = max(d[4] for d in dv)
        first_dec = min(d[3] for d in dv)
        print(json.dumps({"rep": rep, "n": n, "steps": a.steps, "inflight": a.inflight, "host_ms": round(el * 1e3, 3),
                          "device_span_ms": round(span / 1e3, 3), "first_decode_us": round(first_dec, 1),
                          "last_decode_end_us": round(last_dec_end, 1),
                          "tail_after_last_decode_us": round(span - last_dec_end, 1),
                          "mean_phase_us": {k: round(v, 1) for k, v in tot.items()},
                          "submit_span_us": max(hs), "mean_latency_us": round(sum(d[-1] for d in dv) / len(dv) -
                                                                              sum(d[0] for d in dv) / len(dv), 1)}),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
