"""BASELINE configs[3] timing: a 2^20-vote batch (150 validators, 120-byte messages) with the 196
ZIP215 small-order corpus cases (tests/golden/zip215_small_order.json, message "Zcash") and one
signature made over another message mixed in at seeded positions (bench.make_c4_workload). Times,
device-resident:
  batch      the failing batch verification (edc_batch_verify_device)
  per_sig    the reference's fallback, Item::verify_single on every item (edc_verify_each_device)
  grouped    the grouped fallback (edc_find_invalid_device: batch prefix + range MSM + leaves)
  fused      batch + fallback in one call (edc_batch_verify_fallback_device), the fallback part
             reusing the failed batch's k, points and grouping
and checks that both fallbacks return exactly the expected per-item codes (the bad item
InvalidSignature, every corpus case and every other vote Ok). Prints one JSON line.
  python tools/fallback_bench.py [--n 1048576] [--leaf 65536] [--keycache]"""
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
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--keys", type=int, default=150)
    ap.add_argument("--msg-len", type=int, default=120)
    ap.add_argument("--leaf", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--keycache", action="store_true", help="also time with the validator keys in the key cache")
    ap.add_argument("--shapes", default="", help="sweep fallback shapes 'ranges:bits,...' (edc_set_fallback_shape)")
    ap.add_argument("--lib", default=None, help="A/B build of libedc.so (measurement only)")
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0, lib_path=args.lib)
    lib = eng.lib
    n = args.n
    with open(os.path.join(ROOT, "tests", "golden", "zip215_small_order.json")) as f:
        fx = json.load(f)
    vk, sig, msg, off, expect, cpos = bench.make_c4_workload(pkg, eng, torch, dev, n, args.keys, args.msg_len,
                                                             fx["cases"], bytes.fromhex(fx["msg"]))
    torch.cuda.synchronize()
    zseed = bytes([0x33]) * 32

    def timed(fn):
        best, r = None, None
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            best = dt if best is None else min(best, dt)
        return r, best

    a = (vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr())
    eng._check(lib.edc_reserve(eng.ctx, n))
    ver = torch.zeros(n, dtype=torch.uint8, device=dev)
    verdicts = ctypes.create_string_buffer(n)

    def run_all():
        rc, t_batch = timed(lambda: lib.edc_batch_verify_device(eng.ctx, n, *a, zseed, 0, None, None))
        assert rc == 1, rc
        rc, t_each = timed(lambda: lib.edc_verify_each_device(eng.ctx, n, *a, ver.data_ptr()))
        eng._check(rc)
        h = ver.cpu()
        flagged_each = {int(i): int(h[i]) for i in torch.nonzero(h).flatten().tolist()}
        nbad, t_group = timed(lambda: lib.edc_find_invalid_device(eng.ctx, n, *a, zseed, args.leaf, verdicts))
        eng._check(nbad)
        raw = verdicts.raw
        flagged_group = {i: raw[i] for i in range(n) if raw[i]}
        assert flagged_each == flagged_group == expect, (flagged_each, flagged_group, expect)
        cnt = ctypes.c_int(0)
        rc, t_fused = timed(lambda: lib.edc_batch_verify_fallback_device(eng.ctx, n, *a, zseed, verdicts,
                                                                         ctypes.byref(cnt), None))
        assert rc == 1 and cnt.value == len(expect)
        raw = verdicts.raw
        assert {i: raw[i] for i in range(n) if raw[i]} == expect
        return {"batch_ms": round(t_batch, 3), "per_sig_fallback_ms": round(t_each, 3),
                "grouped_fallback_ms": round(t_group, 3), "grouped_over_batch": round(t_group / t_batch, 3),
                "batch_plus_fallback_ms": round(t_fused, 3),
                "fallback_after_batch_ms": round(t_fused - t_batch, 3),
                "fallback_after_batch_over_batch": round((t_fused - t_batch) / t_batch, 3),
                "per_sig_sigs_per_s": round(n / t_each * 1e3, 1)}

    out = {"workload": "configs[3]: 2^20 votes / 150 validators / 120-B msgs + 196 ZIP215 corpus cases + 1 bad sig",
           "n": n, "validators": args.keys, "corpus_cases": len(cpos), "expected_invalid": expect,
           "leaf": args.leaf, "timing": "best of %d, device-resident, synchronous" % args.reps}
    out.update(run_all())
    for sh in [x for x in args.shapes.split(",") if x]:
        r, b = (int(v) for v in sh.split(":"))
        eng._check(lib.edc_set_fallback_shape(eng.ctx, r, b))
        out.setdefault("shapes", {})[sh] = run_all()
    if args.shapes:
        eng._check(lib.edc_set_fallback_shape(eng.ctx, 128, 9))
    if args.keycache and args.keys:
        keys = bytes(vk[:32 * args.keys].cpu().tolist())
        t0 = time.perf_counter()
        u, ok = eng.keycache_load([keys[32 * i:32 * i + 32] for i in range(args.keys)])
        out["keycache"] = {"keys": u, "load_ms": round((time.perf_counter() - t0) * 1e3, 3)}
        out["keycache"].update(run_all())
        eng.keycache_clear()
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
