"""Ed25519 batch verification throughput on MI355X (BASELINE.json metric).

Workload (BASELINE configs[2], the 2^20-signature config the metric is quoted on):
2^20 consensus votes per GPU from 150 validators (vote i signed by validator i mod 150),
120-byte messages (2 SHA-512 blocks), one batch equation per step. Inputs are synthetic
(ChaCha20 streams: keygen [0x11;32], messages [0x22;32], z [0x33;32]) and signed on the GPU,
resident in HBM before timing starts. A step = the full hot path: SHA-512 challenges, ZIP215
decompression, key grouping, ChaCha z + scalar coefficients, Pippenger MSM, [8]/identity.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n 1048576] [--keys 150] [--msg-len 120]
  multi-GPU: python bench.py --gpus N ... starts N ranks itself (torch.distributed.run as a child
  process, before anything touches the GPU); under an outer torch.distributed.run it is one rank.
  At N > 1 the headline is the metric's shape, strong scaling: every step is ONE batch of --n
  (2^20) signatures split over the N ranks; each rank reduces its contiguous shard to one partial
  point and the ranks all-gather the 129-byte records over RCCL and combine them. The weak shape
  (--n per rank) is reported beside it as `scaling_other_shape`.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

# algorithmic multiply work per unit (SURVEY.md 8(d) convention: M = 64, S = 40 v_mad_u64_u32)
ALG_MAD_M, ALG_MAD_S = 64, 40
DECOMP_S, DECOMP_M = 255, 22                     # ZIP215 decode + Niels conversion, per point
ALG_MAD_DECOMP = DECOMP_S * ALG_MAD_S + DECOMP_M * ALG_MAD_M
# whole-path algorithmic work per signature, frozen by SURVEY.md 8(d): decompression 255 S + 20 M
# = 11,480 per point, MSM 7 M = 448 per point-window at c = 16 (R terms 8 windows, A terms 16)
ALG_MAD_PER_SIG_REPEATED = 11480 + 8 * 448            # configs[2]/[3]: repeated validator keys, 15,064
ALG_MAD_PER_SIG_DISTINCT = 2 * 11480 + 24 * 448       # configs[1]/[4]: distinct keys, 33,712
# peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz, v_mad_u64_u32 at half lane rate (measured
# 35.0 T/s sustained by tools/microbench/valu_rates.hip, profiles/r01_valu_rates.txt)
PEAK_TMAD = 256 * 4 * 32 * 2.4e9 / 2 / 1e12
HBM_PEAK_GBS = 8000.0
# SHA-512 compression per block and lane: 80 x (7 x 64-bit + 20 x 32-bit) + 64 x (3 x 64-bit + 14 x 32-bit)
SHA_VALU_PER_BLOCK = 80 * 27 + 64 * 17
SHA_CYCLES_PER_BLOCK = 80 * (7 * 4.1 + 20 * 2.3) + 64 * (3 * 4.1 + 14 * 2.3)   # per wave, per SIMD
SHA_PEAK_BLOCKS = 1024 * 2.4e9 / SHA_CYCLES_PER_BLOCK * 64


def load_pkg():
    import importlib.util
    d = os.path.join(ROOT, "ed25519-consensus_amd")
    if "ed25519_consensus_amd" in sys.modules:
        return sys.modules["ed25519_consensus_amd"]
    spec = importlib.util.spec_from_file_location("ed25519_consensus_amd", os.path.join(d, "__init__.py"),
                                                  submodule_search_locations=[d])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ed25519_consensus_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def chacha_device(pkg, eng, torch, key, blk0, nblocks, dev):
    out = torch.empty(max(nblocks, 1) * 64, dtype=torch.uint8, device=dev)
    rc = eng.lib.edc_chacha_fill_device(eng.ctx, key, blk0, nblocks, ctypes.c_void_p(out.data_ptr()))
    eng._check(rc)
    return out


def make_workload(pkg, eng, torch, dev, n, keys, msg_len, global_base):
    """Signed synthetic items for global queue indices [global_base, global_base + n).
    keys > 0: item i is signed by validator i mod keys; keys == 0: every item has its own key.
    msg_len >= 0: fixed-length messages; msg_len < 0: lengths uniform in [0, 1024] (configs[4])."""
    if keys > 0:
        seeds = chacha_device(pkg, eng, torch, bytes([0x11]) * 32, 0, (keys * 32 + 63) // 64, dev)[: keys * 32]
        idx = ((torch.arange(global_base, global_base + n, dtype=torch.int64, device=dev)) % keys).to(torch.int32)
    else:                                            # distinct keys: seed of global item i
        assert global_base % 2 == 0
        seeds = chacha_device(pkg, eng, torch, bytes([0x11]) * 32, global_base // 2, (n + 1) // 2, dev)[: n * 32]
        idx = torch.arange(0, n, dtype=torch.int32, device=dev)
    if msg_len == 0:                                 # empty messages (the reference benches/bench.rs shape)
        msg = torch.zeros(1, dtype=torch.uint8, device=dev)
        off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    elif msg_len > 0:
        stride = (msg_len + 63) // 64 * 64
        blocks_per_msg = stride // 64
        raw = chacha_device(pkg, eng, torch, bytes([0x22]) * 32, global_base * blocks_per_msg, n * blocks_per_msg, dev)
        msg = raw.view(n, stride)[:, :msg_len].contiguous().view(-1) if n else raw[:1]
        off = torch.arange(0, n + 1, dtype=torch.int64, device=dev) * msg_len
    else:
        lens = chacha_device(pkg, eng, torch, bytes([0x55]) * 32, global_base // 32, (n + 31) // 32 + 1, dev)
        lens = lens.view(torch.int16)[: n].to(torch.int64).abs() % 1025
        off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        off[1:] = torch.cumsum(lens, 0)
        raw = chacha_device(pkg, eng, torch, bytes([0x22]) * 32, global_base * 16, n * 16, dev).view(n, 1024)
        cols = torch.arange(1024, device=dev)[None, :]
        chunk = 1 << 18                              # boolean masks stay below 2^31 elements
        msg = torch.cat([raw[c:c + chunk][cols < lens[c:c + chunk, None]] for c in range(0, n, chunk)] +
                        [torch.zeros(1, dtype=torch.uint8, device=dev)])
    vk = torch.empty(max(n, 1) * 32, dtype=torch.uint8, device=dev)
    sig = torch.empty(max(n, 1) * 64, dtype=torch.uint8, device=dev)
    rc = eng.lib.edc_sign_device(eng.ctx, n, ctypes.c_void_p(seeds.data_ptr()), ctypes.c_void_p(idx.data_ptr()),
                                 ctypes.c_void_p(msg.data_ptr()), ctypes.c_void_p(off.data_ptr()),
                                 ctypes.c_void_p(vk.data_ptr()), ctypes.c_void_p(sig.data_ptr()))
    eng._check(rc)
    return vk, sig, msg, off


def make_c4_workload(pkg, eng, torch, dev, n, keys, msg_len, cases, corpus_msg, pos_seed=bytes([0x44]) * 32):
    """BASELINE configs[3]: the configs[2]-style vote batch (make_workload) with the ZIP215 small-order
    corpus (reference tests/small_order.rs:12-77; `cases` = tests/golden/zip215_small_order.json) put
    at seeded positions (their message is `corpus_msg`, b"Zcash") and ONE bad signature: the item at
    another seeded position keeps its signature but its message is changed, i.e. it was signed over a
    different message (tests/batch.rs:27-31). Positions come from random.Random(pos_seed) (SURVEY
    8(d) seed [0x44;32]). Returns vk, sig, msg, off (device) and {index: expected verify_single code}
    for every item whose code is not Ok, plus the corpus positions."""
    import random
    vk, sig, msg, off = make_workload(pkg, eng, torch, dev, n, keys, msg_len, 0)
    rnd = random.Random(pos_seed)
    pos = rnd.sample(range(n), len(cases) + 1)
    cpos, bad = pos[:-1], pos[-1]
    pt = torch.tensor(cpos, dtype=torch.int64, device=dev)
    vk.view(-1, 32)[:n][pt] = torch.tensor([list(bytes.fromhex(c["vk"])) for c in cases], dtype=torch.uint8,
                                           device=dev)
    sig.view(-1, 64)[:n][pt] = torch.tensor([list(bytes.fromhex(c["sig"])) for c in cases], dtype=torch.uint8,
                                            device=dev)
    m2d = msg.view(n, msg_len)
    m2d[pt, :len(corpus_msg)] = torch.tensor(list(corpus_msg), dtype=torch.uint8, device=dev)
    m2d[bad, 0] ^= 1                               # the bad item: signed over another message
    lens = torch.full((n,), msg_len, dtype=torch.int64, device=dev)
    lens[pt] = len(corpus_msg)
    cols = torch.arange(msg_len, device=dev)[None, :]
    arena = torch.cat([m2d[cols < lens[:, None]], torch.zeros(1, dtype=torch.uint8, device=dev)])
    off2 = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    off2[1:] = torch.cumsum(lens, 0)
    expect = {p: c["expect_single"] for p, c in zip(cpos, cases) if c["expect_single"]}
    expect[bad] = 1
    return vk, sig, arena, off2, expect, cpos


def cpu_baseline(vk, sig, msg, off, n_sample, keys, msg_len):
    """Oracle C restatement (dalek u64-backend algorithm, oracle/edc_oracle.c) on the host
    cores: the first n_sample items of the SAME GPU-generated workload, one Verifier per
    thread over equal contiguous chunks, queue (SHA-512 + grouping) + verify timed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle_c
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "sigs/s", "cores": 0, "kind": "port", "sample": f"unavailable: {e}"}
    n_sample = min(n_sample, vk.numel() // 32)
    vkb = vk[: 32 * n_sample].cpu().numpy().tobytes()
    sgb = sig[: 64 * n_sample].cpu().numpy().tobytes()
    o = off[: n_sample + 1].cpu().tolist()
    mb = msg[: o[-1]].cpu().numpy().tobytes()
    data = ([vkb[32 * i:32 * i + 32] for i in range(n_sample)], [sgb[64 * i:64 * i + 64] for i in range(n_sample)],
            [mb[o[i]:o[i + 1]] for i in range(n_sample)])
    return oracle_c.baseline_c3(n_sample=n_sample, keys=keys, msg_len=msg_len, data=data)


def host_api_leg(eng, vk, sig, msg, off, n, zseed, reps=8):
    """The synchronous host-buffer calls the Rust shim makes (reference
    `Verifier::verify`, src/batch.rs:149): the same n items copied once into pageable host memory,
    then `edc_batch_verify_prehashed` (queued `Item {vk_bytes, sig, k}`, 128 B per item over PCIe,
    the shim's call) and `edc_batch_verify` (vk, sig and the message arena; SHA-512 on the GPU),
    each call timed from the host pointers to its verdict. PCIe-inclusive, after the timed region,
    never the headline `value`."""
    import numpy as np
    lib = eng.lib
    hv = vk[:32 * n].cpu().numpy().tobytes()
    hs = sig[:64 * n].cpu().numpy().tobytes()
    ho = (off[:n + 1] - off[0]).cpu().numpy().astype(np.uint64)
    hm = msg[int(off[0]):int(off[n])].cpu().numpy().tobytes() or b"\0"
    optr = ho.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    kb = ctypes.create_string_buffer(32 * max(n, 1))
    eng._check(lib.edc_challenge(eng.ctx, n, hv, hs, hm, optr, kb))
    hk = kb.raw
    out = {"n": n, "reps": reps, "memory": "pageable host buffers (bytes objects), copied by the call"}
    calls = {"prehashed": lambda: lib.edc_batch_verify_prehashed(eng.ctx, n, hv, hs, hk, zseed, None, None),
             "with_messages": lambda: lib.edc_batch_verify(eng.ctx, n, hv, hs, hm, optr, zseed, None)}
    for name, f in calls.items():
        for _ in range(2):
            eng._check(f())
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            rc = f()
            ts.append(time.perf_counter() - t)
            assert rc == 0, f"host-API {name}: valid batch rejected ({rc})"
        ts.sort()
        med = ts[len(ts) // 2]
        out[name] = {"ms_median": round(med * 1e3, 3), "ms_min": round(ts[0] * 1e3, 3),
                     "sigs_per_s": round(n / med, 1),
                     "h2d_bytes": len(hv) + len(hs) + (len(hk) if name == "prehashed" else len(hm) + ho.nbytes)}
    return out


def openssl_anchor(seconds=2, cores=1):
    """SURVEY.md 8(d) / BASELINE.md anchor: `openssl speed ed25519` verify/s on the host. OpenSSL
    verifies one signature at a time under RFC 8032 cofactorless rules (it rejects non-canonical
    encodings and small-order keys that ZIP215 accepts), so it is a CPU scale reference for the
    primitive, not a parity baseline. Runs the system binary; None when it is absent."""
    import re
    import shutil
    import subprocess
    exe = shutil.which("openssl")
    if exe is None:
        return None
    cmd = [exe, "speed", "-seconds", str(seconds)] + (["-multi", str(cores)] if cores > 1 else []) + ["ed25519"]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=20 * seconds + 30, cwd="/tmp").stdout
    except Exception as e:  # pragma: no cover
        return {"value": None, "sample": f"openssl speed failed: {e}"}
    m = re.search(r"Ed25519\)\s+\S+\s+\S+\s+([0-9.]+)\s+([0-9.]+)", out)
    if m is None:
        return {"value": None, "sample": "openssl speed output not parsed"}
    ver = out.strip().splitlines()[0] if out.strip() else "openssl"
    return {"value": float(m.group(2)), "unit": "verify/s", "cores": cores, "kind": "openssl speed ed25519",
            "rules": "RFC 8032 single verify (cofactorless, canonical encodings only), not ZIP215 batch",
            "sample": f"{' '.join(cmd[1:])} ({ver})"}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(argv, nranks, port):
    """The child command that runs `nranks` ranks of this script (one process per GPU, RCCL)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(argv, nranks, call=None):
    """`--gpus N` (N > 1) without an outer torch.distributed.run: start the N ranks as ONE child
    process before this process imports torch or touches HIP (no exec: the child is waited for).
    Rank 0 prints the JSON line straight to the inherited stdout; torch.distributed.run exits
    non-zero when any rank fails, and that code is returned."""
    import subprocess
    call = call or subprocess.call
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")    # dmabuf IPC only on this pool (RCCL)
    return call(rank_launch_cmd(argv, nranks, free_port()), env=env)


def default_inflight(n, small_depth):
    """Batches in flight for n signatures per GPU: 6 from 2^20 (6 and 7 alternate within the spread
    there), 7 for 2^19 shards (+1.5 % over 6 in 4 of 4 alternating pairs, profiles/r06/r06zn_*),
    small_depth below (16, on one rank and beside RCCL's and the exchange ring's queues)."""
    if n >= (1 << 20):
        return 6
    return 7 if n >= (1 << 19) else small_depth


def world_error(gpus, world, backend, local_world, ndev):
    """Why this rank must not run (None if it may): the process group must be exactly the --gpus
    ranks asked for, and with RCCL every local rank needs a GPU of its own (the gloo rehearsal
    shares the visible GPUs on purpose)."""
    if world != gpus:
        return f"--gpus {gpus} but the process group has {world} rank(s)"
    if backend != "gloo" and world > 1 and ndev < local_world:
        return f"{local_world} ranks on this node but only {ndev} GPU(s) visible"
    return None


CONFIGS = {   # BASELINE.json configs: (items per GPU, validators (0 = distinct keys), message bytes (-1 = 0..1024))
    "c2": (1 << 16, 0, 32, "configs[1]: 2^16 sigs, distinct keys, 32-byte msgs"),
    "c3": (1 << 20, 150, 120, "configs[2]: 2^20 votes/GPU from 150 validators, 120-byte msgs"),
    "c5": (1 << 21, 0, -1, "configs[4]: 2^21 sigs/GPU (2^24 over 8 GPUs), distinct keys, 0..1024-byte msgs"),
}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS),
                    help="workload; c3 (configs[2]) is the one BASELINE.json's metric is quoted on")
    ap.add_argument("--n", "--batch", dest="n", type=int, default=None,
                    help="signatures per GPU per step (default: the config's; --batch under torch.distributed.run, "
                         "whose own parser takes --n for an abbreviation of its options)")
    ap.add_argument("--keys", type=int, default=None, help="validators (0 = distinct keys; default: the config's)")
    ap.add_argument("--msg-len", type=int, default=None, help="message bytes (-1 = uniform 0..1024)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-api", action="store_true",
                    help="skip the host-buffer (PCIe-inclusive) synchronous calls reported after the timed region")
    ap.add_argument("--profile-steps", type=int, default=3, help="extra instrumented steps for per-phase timings")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight per GPU (submit/wait pipelining, <= the context's 16 slots); "
                         "0 = 6 from 2^20 signatures per GPU up, 7 from 2^19, 16 below (small shards need "
                         "more overlap; 12 in a multi-rank run)")
    ap.add_argument("--keycache", action="store_true",
                    help="register the validator keys in the context's key cache before timing (edc_keycache_load)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="strong (default at N > 1, the metric's whole-node 2^20 batch): the ranks split one batch "
                         "of --n signatures (n/N each); weak (N = 1): every rank verifies --n signatures of one "
                         "global batch")
    ap.add_argument("--window-bits", type=int, default=0, help="Pippenger window width (0 = chosen from the batch size)")
    ap.add_argument("--msm-parts", type=int, default=0, help="MSM parts per batch (0 = chosen from the batch size)")
    ap.add_argument("--bin-entries", type=int, default=0, help="target MSM entries per bin (0 = chosen from the batch size)")
    ap.add_argument("--multi", type=int, default=1,
                    help="verify this many consecutive batches of --n signatures per launch sequence "
                         "(edc_batch_submit_multi_device; each keeps its own verdict and z range)")
    ap.add_argument("--multi-exact", action="store_true",
                    help="with --multi: every launch batch by batch (edc_set_multi_union(0)) instead of the "
                         "default union first (one batch over all items, rerun batch by batch only on failure)")
    ap.add_argument("--prehashed", action="store_true",
                    help="time edc_batch_submit_prehashed_device: items carry their queue-time k (the reference's "
                         "Item {vk_bytes, sig, k}); SHA-512 is then outside the timed region (not the headline)")
    ap.add_argument("--scatter-stage", type=int, default=0,
                    help="measurement only: cap the binning scatter's LDS stage (entries; edc_debug_set_scatter_stage)")
    ap.add_argument("--exchange-lag", type=int, default=8,
                    help="multi-rank: batches whose exchange is in flight before the oldest verdict is completed")
    ap.add_argument("--exchange-group", type=int, default=4,
                    help="multi-rank: batches whose records leave in one all-gather (sharded.ExchangeRing)")
    ap.add_argument("--spinup-ms", type=float, default=100.0,
                    help="device set-up before the warmup steps: run this workload's batches for this many "
                         "milliseconds (rank-local), so that the timed steps meet the GPU at its sustained "
                         "rate and not on its way up from idle (0 = none; reported as `spinup` in the line)")
    ap.add_argument("--lib", default=None, help="tools/ab_variants.sh only: load this A/B build of libedc.so")
    args = ap.parse_args(argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(sys.argv[1:] if argv is None else argv, args.gpus)
    c_n, c_keys, c_len, c_desc = CONFIGS[args.config]
    args.n = c_n if args.n is None else args.n
    args.keys = c_keys if args.keys is None else args.keys
    args.msg_len = c_len if args.msg_len is None else args.msg_len

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.scaling is None:
        args.scaling = "strong" if world > 1 else "weak"
    # EDC_DIST_BACKEND=gloo: rehearsal of the multi-rank path with several ranks sharing the
    # visible GPUs (the all-gather then goes through host memory); the default is RCCL
    backend = os.environ.get("EDC_DIST_BACKEND", "nccl")
    import torch
    # counting devices does not initialise the GPU
    err = world_error(args.gpus, world, backend, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))),
                      torch.cuda.device_count())
    if err:
        print(f"bench.py rank {rank}: {err}", file=sys.stderr, flush=True)
        return 2
    dist = None
    if backend == "gloo":
        local = local % torch.cuda.device_count()
    # EDC_FORCE_DIST=1 (rehearsal only): run the multi-rank path -- process group, per-batch
    # all-gather of the 129-byte record, combine -- even for one rank, e.g. to exercise RCCL on a
    # one-GPU box; the numbers are not a scaling measurement
    force_dist = os.environ.get("EDC_FORCE_DIST") == "1"
    if world > 1 or force_dist:
        import datetime
        import torch.distributed as dist
        # RCCL's streams at high priority: the per-group collective must not queue behind the
        # in-flight batches' kernels for a free CU
        os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
        torch.cuda.set_device(local)
        # a rank that dies mid-run ends the others' collectives within this bound instead of the
        # backend's default (10-30 min)
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=120))
        if dist.get_world_size() != args.gpus:
            print(f"bench.py rank {rank}: --gpus {args.gpus} but the group formed with {dist.get_world_size()} "
                  "rank(s)", file=sys.stderr, flush=True)
            dist.destroy_process_group()
            return 2
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    torch.zeros(1, device=dev)                     # initialise torch's HIP runtime first

    pkg = load_pkg()
    eng = pkg.Engine(local, lib_path=args.lib)
    from importlib import import_module
    sharded = import_module("ed25519_consensus_amd.sharded")

    n = args.n // world if args.scaling == "strong" else args.n
    base = rank * n
    # ranks sharing one GPU (the gloo rehearsal) split its in-flight slots: past ~16 user queues
    # per GPU the hardware scheduler time-slices them ("One hardware queue per slot")
    sharing = max(1, -(-world // max(1, torch.cuda.device_count()))) if backend == "gloo" else 1
    slots = max(1, 16 // sharing)
    nmb = max(1, args.multi)                       # batches per launch sequence
    inflight_auto = args.inflight <= 0
    # small shards want 16 batches in flight, one hardware queue each. A multi-rank run adds the
    # exchange ring's stream and RCCL's own; it kept 12 for a while (past ~16 user queues the
    # scheduler time-slices them), but over 160 steps of 2^17 shards 16 beats 12 with the RCCL
    # loop too: 5.67-5.68e8 against 5.48-5.54e8 (profiles/r06/r06zz4_inflight_s160_n17.log)
    small_depth = 16
    if args.inflight <= 0:
        if nmb > 1:    # several batches per launch: 3 launches of >= 2^20 items in flight (tools/sweep_multi.sh;
            # union first measured 6.38e8 at 3 and 5.55e8 at 6 at 8 x 2^17, profiles/r04/r04w_union_inflight6_summary.log)
            args.inflight = 3 if n * nmb >= (1 << 19) else 4
        else:
            args.inflight = default_inflight(n, small_depth)
    args.inflight = min(args.inflight, slots)
    if nmb > 1:    # every slot's multi-batch workspace is allocated on its first launch: warm them all
        args.warmup = max(args.warmup, args.inflight + 1)
    # the context rotates over exactly `inflight` slots, so only that many slot streams (hardware
    # queues) exist beside RCCL's own in a multi-rank run; a build with fewer slots keeps its count
    if nmb > 1:
        eng.set_multi_union(not args.multi_exact)
    if args.scatter_stage:
        eng._check(eng.lib.edc_debug_set_scatter_stage(args.scatter_stage))
    if eng.lib.edc_set_slots(eng.ctx, args.inflight) < 0 and sharing > 1:
        raise RuntimeError("cannot split the GPU's slots between the ranks sharing it")
    t_gen = time.perf_counter()
    vk, sig, msg, off = make_workload(pkg, eng, torch, dev, n * nmb, args.keys, args.msg_len, base * nmb)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen
    zseed = bytes([0x33]) * 32
    lib = eng.lib
    check8 = ctypes.create_string_buffer(32)

    d_k = None
    if args.prehashed:     # Item::from's k, computed once before timing (src/batch.rs:82-94)
        nt = n * nmb
        o = (ctypes.c_uint64 * (nt + 1)).from_buffer_copy((off - off[0]).cpu().numpy().astype("uint64").tobytes())
        kb = ctypes.create_string_buffer(32 * max(nt, 1))
        eng._check(lib.edc_challenge(eng.ctx, nt, vk[:32 * nt].cpu().numpy().tobytes(),
                                     sig[:64 * nt].cpu().numpy().tobytes(), msg.cpu().numpy().tobytes(), o, kb))
        d_k = torch.frombuffer(bytearray(kb.raw), dtype=torch.uint8).to(dev)
        torch.cuda.synchronize()

    pending = []
    combine = (lambda p, b: eng.combine_partials(p, b, want_check8=False))
    # multi-rank: the 129-byte records travel through a ring of asynchronous all-gathers (RCCL on the
    # device, gloo on the host for the one-GPU rehearsals); up to --exchange-lag are in flight
    # (RCCL: the gathered records are combined on the device right behind the collective)
    ring = (sharded.ExchangeRing(dist, dev if backend != "gloo" else torch.device("cpu"), depth=args.exchange_lag,
                                 device_combine=eng if backend != "gloo" else None, group=args.exchange_group)
            if dist else None)
    xstat = {"post": 0.0, "pop": 0.0, "combine": 0.0}

    def timed_ring_op(f, name):
        def g(*a):
            t = time.perf_counter()
            r = f(*a)
            xstat[name] += time.perf_counter() - t
            return r
        return g

    def submit():
        if nmb > 1:
            t = lib.edc_batch_submit_multi_device(eng.ctx, nmb, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                                  off.data_ptr(), d_k.data_ptr() if d_k is not None else None, zseed,
                                                  base * nmb, 0)
        elif d_k is not None:
            t = lib.edc_batch_submit_prehashed_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), d_k.data_ptr(), zseed,
                                                      base, None, 0)
        else:
            t = lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                            zseed, base, None, 0)
        if t < 0:
            eng._check(t)
        pending.append(t)

    def wait_oldest():
        """Collect the oldest batch; returns a function that completes its verdict."""
        if nmb > 1:
            assert dist is None, "--multi runs on one process per node"
            v = (ctypes.c_int * nmb)()
            rc = eng._check(lib.edc_batch_wait_multi(eng.ctx, pending.pop(0), nmb, v, None, None, None))
            return lambda: rc
        rc = eng._check(lib.edc_batch_wait(eng.ctx, pending.pop(0), None, None, None))
        return lambda: rc

    tail = {"t_wait": 0.0, "split": None}    # multi-rank: where the timed region's tail goes

    def wait_partial(t):
        """multi-GPU: this rank's partial point of the global batch (and its reject flag)"""
        part = ctypes.create_string_buffer(128)
        bad = ctypes.c_int(0)
        eng._check(lib.edc_batch_wait(eng.ctx, t, None, part, ctypes.byref(bad)))
        tail["t_wait"] = time.perf_counter()
        return part.raw, bad.value

    def submit_ticket():
        submit()
        return pending.pop()

    def run_steps(k):
        """k full batch verifications; with --inflight F, batch i+F-1 is enqueued before batch i's
        verdict is collected (every verdict is still completed inside the loop). Multi-GPU
        (sharded.run_sharded_stream): the freed slot is refilled first, then the collected batch's
        partial point is posted to the asynchronous all-gather ring, and the exchange --exchange-lag
        batches back is completed and combined: no rank waits for a collective per batch."""
        if dist is not None:
            return sharded.run_sharded_stream(k, args.inflight, submit_ticket, wait_partial,
                                              timed_ring_op(lambda p, b: combine(p, b)[0], "combine"), ring,
                                              args.exchange_lag)
        codes = []
        for _ in range(k):
            done = wait_oldest() if len(pending) >= max(1, args.inflight) else None
            submit()
            if done is not None:
                codes.append(done())
        while pending:
            codes.append(wait_oldest()())
        return codes

    if args.keycache and args.keys > 0:           # a node's known validator set, registered once
        kb = bytes(vk[:32 * min(args.keys, n)].cpu().tolist())
        eng.keycache_load([kb[32 * i:32 * i + 32] for i in range(len(kb) // 32)])
    eng._check(lib.edc_set_msm_shape(eng.ctx, args.window_bits, args.msm_parts))
    eng._check(lib.edc_set_msm_bin_entries(eng.ctx, args.bin_entries))
    eng._check(lib.edc_reserve(eng.ctx, n))        # every in-flight slot's workspace, before any step
    if ring is not None:                          # communicator and per-buffer set-up stay out of the
        ring.warm()                               # timed region, even with --warmup 0
        ring.post, ring.pop = timed_ring_op(ring.post, "post"), timed_ring_op(ring.pop, "pop")

    def timed(k):
        """k steps between barriers + device syncs; the max over ranks"""
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        codes = run_steps(k)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist and tail["split"] is None:
            # after the last batch's partial: completing the exchanges still in flight, then the
            # closing device sync and barrier (fixed per timed region, not per batch)
            tail["split"] = {"exchange_drain": round((t1 - tail["t_wait"]) * 1e6, 1),
                             "sync": round((t2 - t1) * 1e6, 1), "barrier": round((t0 + el - t2) * 1e6, 1)}
        if dist:
            tt = torch.tensor([el], dtype=torch.float64, device=dev if backend != "gloo" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el, codes

    spin = {"ms": 0.0, "batches": 0}

    def spin_up(ms):
        """Device set-up before the warmup steps: batches of this workload, rank-local (no
        collectives, so ranks need not agree on a count), for `ms` milliseconds. From idle the GPU
        needs ~50 ms of load before it runs at its sustained rate: the first 20 timed steps after
        only the 5 warmup steps measured 6.70-6.71e8 (2^20) and 4.53-4.70e8 (2^17 shards), after a
        50-800 ms spin-up 6.96-7.07e8 and 5.1-5.4e8 (profiles/r06/r06zq_*, r06zr_*)."""
        if ms <= 0:
            return
        t_spin = time.perf_counter()
        while True:
            if len(pending) >= max(1, args.inflight):
                wait_oldest()()
            submit()
            spin["batches"] += 1
            if (time.perf_counter() - t_spin) * 1e3 >= ms:
                break
        while pending:
            wait_oldest()()
        spin["ms"] += round((time.perf_counter() - t_spin) * 1e3, 1)

    spin_up(args.spinup_ms)
    run_steps(args.warmup)
    for key in xstat:
        xstat[key] = 0.0
    elapsed, codes = timed(args.steps)
    exchange_us = {key: round(v / max(1, args.steps) * 1e6, 1) for key, v in xstat.items()}
    # diagnostic only (EDC_TIMED_REPEATS=r): the same timed region r - 1 more times right after
    # the first, reported beside it; `value` is always the first
    again = []
    for _ in range(int(os.environ.get("EDC_TIMED_REPEATS", "1")) - 1):
        el_r, codes_r = timed(args.steps)
        assert all(c == 0 for c in codes_r) or args.lib, f"valid synthetic batch rejected: {codes_r}"
        again.append(round(n * nmb * world * args.steps / el_r, 1))
    other = None
    if dist and nmb == 1 and not args.prehashed:
        # multi-rank: the other scaling shape beside the headline one, on the same ranks and data
        # (strong: the ranks split one --n batch; weak: every rank verifies --n of its own), so a
        # SCALE record carries both; items are a prefix of this rank's slice, z at global indices
        n_main, base_main, inflight_main = n, base, args.inflight
        n = args.n if args.scaling == "strong" else args.n // world
        base = rank * n
        if inflight_auto:              # the in-flight depth the default picks for this shard size
            args.inflight = min(default_inflight(n, small_depth), slots)
            eng._check(lib.edc_set_slots(eng.ctx, args.inflight))
        eng._check(lib.edc_reserve(eng.ctx, n))
        main_data = (vk, sig, msg, off)
        if n > n_main:      # the weak shape beside a strong headline: --n signatures of this rank's own
            vk, sig, msg, off = make_workload(pkg, eng, torch, dev, n, args.keys, args.msg_len, base)
            torch.cuda.synchronize()
        # as many signatures as the headline run (steps x n_main / n): a short run of small
        # batches is mostly the pipeline's fill and drain (16 batches in flight)
        k2 = max(args.steps, round(args.steps * n_main / max(1, n)))
        spin_up(args.spinup_ms)
        run_steps(max(2, args.warmup))
        el2, codes2 = timed(k2)
        other = {"scaling": "weak" if args.scaling == "strong" else "strong", "sigs_per_gpu": n,
                 "inflight": args.inflight, "steps": k2,
                 "value": round(n * world * k2 / el2, 1), "ms_per_step": round(el2 / k2 * 1e3, 3),
                 "verdict_ok": all(c == 0 for c in codes2)}
        vk, sig, msg, off = main_data
        n, base = n_main, base_main
        if args.inflight != inflight_main:
            args.inflight = inflight_main
            eng._check(lib.edc_set_slots(eng.ctx, args.inflight))
    verdict_ok = all(c == 0 for c in codes)
    # an A/B build (--lib, tools/ab_variants.sh) may be a timing probe that is wrong by design:
    # report its verdicts instead of stopping; the product library must verify the batch
    assert verdict_ok or args.lib, f"valid synthetic batch rejected: {codes}"

    # instrumented steps (outside the timed region): per-phase HIP-event timings on the
    # context stream, for the roofline of the dominant kernel
    lib.edc_set_timing(eng.ctx, 1)
    names = [lib.edc_timing_name(i).decode() for i in range(7)]
    acc = [0.0] * 7
    acc_ms, acc_entries = [], []      # k_msm_accum_dma alone (edc_last_msm_accum)
    for _ in range(max(1, args.profile_steps)):
        rc = lib.edc_batch_verify_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
                                         off.data_ptr(), zseed, base, None, None)
        eng._check(rc)
        buf = (ctypes.c_float * 7)()
        lib.edc_last_timings(eng.ctx, buf, 7)
        for i in range(7):
            acc[i] += buf[i] / max(1, args.profile_steps)
        if hasattr(lib, "edc_last_msm_accum"):
            a_ms, a_ent = ctypes.c_float(0), ctypes.c_uint64(0)
            if lib.edc_last_msm_accum(eng.ctx, ctypes.byref(a_ms), ctypes.byref(a_ent)) == 0:
                acc_ms.append(a_ms.value)
                acc_entries.append(a_ent.value)
    # the same in-flight loop once more with HIP events on (still outside the timed region): the
    # dominant kernel's duration while it shares the GPU with the other in-flight batches (this is
    # what a kernel trace of the default command averages; no collectives, every rank alike)
    i_dec = names.index("decompress_R")
    pipe_ms, pend = [], []

    def wait_timed():
        eng._check(lib.edc_batch_wait(eng.ctx, pend.pop(0), None, None, None))
        buf = (ctypes.c_float * 7)()
        lib.edc_last_timings(eng.ctx, buf, 7)
        pipe_ms.append(buf[i_dec])

    for _ in range(3 * max(4, args.inflight)):
        if len(pend) >= max(1, args.inflight):
            wait_timed()
        t = lib.edc_batch_submit_device(eng.ctx, n, vk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                        zseed, base, None, 0)
        eng._check(t)
        pend.append(t)
    while pend:
        wait_timed()
    lib.edc_set_timing(eng.ctx, 0)
    pipe_dec_ms = sum(pipe_ms[max(4, args.inflight):]) / max(1, len(pipe_ms) - max(4, args.inflight))
    phases = {names[i]: round(acc[i], 4) for i in range(7)}
    # SHA-512 blocks of the instrumented batch (R || A || M, 17 bytes of padding + length)
    lens = (off[1:n + 1] - off[:n]).to(torch.int64)
    sha_blocks = int(((64 + lens + 17 + 127) // 128).sum().item())

    if rank == 0:
        total = n * nmb * world * args.steps    # strong scaling: n * world == --n
        value = total / elapsed
        ms_per_step = elapsed / args.steps * 1e3
        dom_ms = phases["decompress_R"]
        units = n                      # one launch decodes the R_i of every signature
        achieved = units * ALG_MAD_DECOMP / (dom_ms * 1e-3) / 1e12
        traffic = None
        tpath = os.path.join(ROOT, "profiles", "traffic_k_decompress.json")
        if os.path.exists(tpath):
            try:
                t = json.load(open(tpath))
                if t.get("n") == n:
                    traffic = t.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        valu = None                    # rocprof VALU counters of the same kernel (profiles/valu_pmc.json)
        vpath = os.path.join(ROOT, "profiles", "valu_pmc.json")
        if os.path.exists(vpath):
            try:
                v = json.load(open(vpath))
                if v.get("n") == n:
                    kd = v["kernels"]["k_decompress"]
                    valu = {"valu_insts_per_launch": kd["valu_insts"], "mad_insts_per_launch": kd["int64_insts"],
                            "executed_mad_frac_of_peak": round(kd["int64_lane_ops_per_cycle_per_simd"] / 16.0, 3),
                            "valu_issue_frac": kd["valu_issue_frac"],
                            "source": "profiles/valu_pmc.json (SQ_INSTS_VALU, SQ_INSTS_VALU_INT64, GRBM_GUI_ACTIVE)"}
            except Exception:
                valu = None
        host_api = None
        if not args.no_host_api and world == 1 and nmb == 1 and hasattr(lib, "edc_batch_verify_prehashed"):
            host_api = host_api_leg(eng, vk, sig, msg, off, n, zseed)
        cpu = None
        if not args.no_cpu_baseline and world == 1:     # rank 0 at N=1 only
            cpu = cpu_baseline(vk, sig, msg, off, args.cpu_sample, args.keys, args.msg_len)
            if isinstance(cpu, dict):
                cpu["openssl_anchor"] = openssl_anchor()
        alg_sig = ALG_MAD_PER_SIG_REPEATED if args.keys > 0 else ALG_MAD_PER_SIG_DISTINCT
        line = {
            "metric": "Ed25519 batch-verified signatures/sec (whole node) at 2^20 sigs",
            "value": round(value, 1),
            "unit": "sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u32/u64 integer (GF(2^255-19), radix 2^29 limbs)",
            "data": "synthetic (ChaCha20-seeded keys/messages, signed on GPU)",
            "config": {"workload": c_desc,
                       "sigs_per_gpu": n, "validators": args.keys or "distinct", "msg_len": args.msg_len,
                       "inflight": args.inflight, "keycache": bool(args.keycache and args.keys > 0),
                       "prehashed": bool(args.prehashed), "batches_per_launch": nmb,
                       "multi_union_first": bool(nmb > 1 and not args.multi_exact),
                       "parallelism": f"shard{world}" if world > 1 else "single"},
            # the process group the ranks actually formed (None: one process, no collectives)
            "comm": ({"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                      "exchange_lag": args.exchange_lag, "exchange_group": args.exchange_group,
                      "exchange_us": exchange_us, "timed_tail_us": tail["split"],
                      "exchange_note": "host time per batch inside the timed loop: posting the all-gather, "
                                       "completing it (waits for the collective), combining the partials; timed_tail_us: the "
                                       "headline region's end after the last batch's partial"}
                     if dist else None),
            "scaling_other_shape": other,
            "timed_repeats": again or None,
            # device set-up before the warmup steps (--spinup-ms): batches of this workload, untimed
            "spinup": {"ms": spin["ms"], "batches": spin["batches"],
                       "note": "untimed batches of this workload before the warmup steps: from idle the GPU needs "
                               "~50 ms of load to reach its sustained rate (profiles/r06/r06zr_spinup_sweep.log)"},
            "roofline": {"bound": "valu_int", "kernel": "k_decompress (R_i)",
                         "achieved": round(achieved, 3), "peak": round(PEAK_TMAD, 2),
                         "unit": "T v_mad_u64_u32/s", "frac": round(achieved / PEAK_TMAD, 4),
                         "traffic": traffic, "pmc_valu": valu,
                         "alg_mad_per_unit": ALG_MAD_DECOMP, "units_per_launch": units,
                         "pipeline": {"alg_mad_per_sig": alg_sig,
                                      "achieved": round(value / world * alg_sig / 1e12, 3),
                                      "peak": round(PEAK_TMAD, 2), "unit": "T v_mad_u64_u32/s per GPU",
                                      "frac": round(value / world * alg_sig / 1e12 / PEAK_TMAD, 4),
                                      "basis": "whole hot path: sigs/s per GPU x SURVEY.md 8(d) ALG_MAD_PER_SIG "
                                               "(decompression + MSM additions) / peak"},
                         "avg_launch_ms": dom_ms,
                         "pipelined": {"avg_launch_ms": round(pipe_dec_ms, 4),
                                       "achieved": round(units * ALG_MAD_DECOMP / (pipe_dec_ms * 1e-3) / 1e12, 3),
                                       "note": "same kernel inside the in-flight loop: HIP events on its stream, "
                                               "so the duration includes waiting for CUs held by the other "
                                               "in-flight batches (rocprof's begin-to-end average of the "
                                               "pipelined run is shorter: profiles/r06/r06_kernel_stats_pipelined.csv)"},
                         "measured": f"HIP events on the slot stream around each launch, {max(1, args.profile_steps)} "
                                     "instrumented batches run one at a time after the timed region "
                                     "(rocprof cross-check: profiles/r06/r06_kernel_stats_inflight1.csv)"},
            # k_challenge against its own issue bound: per 128-byte block and lane, 80 rounds of 7
            # v_lshl_add_u64 + 20 32-bit VALU (12 v_alignbit, 8 v_bitop3) and 64 schedule steps of
            # 3 + 14 (ISA of the compression loop, tools: llvm-objdump of libedc.so), priced at the
            # measured issue costs (64-bit VOP3 4.1, 32-bit 2.3 cycles per wave-instruction per SIMD,
            # profiles/r01_valu_rates.txt) at the nominal 2.4 GHz over 1024 SIMDs x 64 lanes
            "roofline_sha512": {"kernel": "k_challenge", "blocks_per_launch": sha_blocks,
                                "avg_launch_ms": phases["challenge_sha512"],
                                "achieved_blocks_per_s": round(sha_blocks / (phases["challenge_sha512"] * 1e-3), 1),
                                "peak_blocks_per_s": round(SHA_PEAK_BLOCKS, 1),
                                "frac": round(sha_blocks / (phases["challenge_sha512"] * 1e-3) / SHA_PEAK_BLOCKS, 4),
                                "valu_per_block": SHA_VALU_PER_BLOCK, "bound": "valu issue (integer)"}
            if phases["challenge_sha512"] > 0 else None,
            # k_msm_accum_dma against the same mad roofline: one signed mixed addition per digit
            # entry, 7 M = 448 algorithmic v_mad_u64_u32; 7 x 99 = 693 executed in
            # radix 2^29. Duration: HIP events around the kernel in the instrumented batches.
            "roofline_msm_accum": ({"kernel": "k_msm_accum_dma", "additions_per_launch": acc_entries[-1],
                                    "avg_launch_ms": round(sum(acc_ms) / len(acc_ms), 4),
                                    "achieved": round(acc_entries[-1] * 448 / (sum(acc_ms) / len(acc_ms) * 1e-3) / 1e12, 3),
                                    "peak": round(PEAK_TMAD, 2), "unit": "T v_mad_u64_u32/s",
                                    "frac": round(acc_entries[-1] * 448 / (sum(acc_ms) / len(acc_ms) * 1e-3) / 1e12
                                                  / PEAK_TMAD, 4),
                                    "executed_mad_frac": round(acc_entries[-1] * 693 / (sum(acc_ms) / len(acc_ms) * 1e-3)
                                                               / 1e12 / PEAK_TMAD, 4),
                                    "alg_mad_per_addition": 448}
                                   if acc_ms and acc_ms[-1] > 0 else None),
            "hbm_view": ({"achieved_gbs": round(traffic / (dom_ms * 1e-3) / 1e9, 1), "peak_gbs": HBM_PEAK_GBS,
                          "frac": round(traffic / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)} if traffic else None),
            "phases_ms": phases,
            # one batch alone, start to verdict (sum of the phases of the instrumented batches)
            "batch_latency_ms": round(sum(phases.values()), 3),
            # the host-buffer synchronous calls of the Rust shim (PCIe included), NOT `value`
            "host_api": host_api,
            "cpu_baseline": cpu,
            "gen_s": round(t_gen, 2),
        }
        if args.lib:
            line["ab_lib"] = {"path": args.lib, "verdict_ok": verdict_ok}
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
