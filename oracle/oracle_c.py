"""ctypes wrapper of oracle/build/libedc_oracle.so (the C restatement; TEST INFRASTRUCTURE /
CPU BASELINE ONLY -- imported by tests/ and bench.py's cpu_baseline leg, never by the product)."""
import ctypes
import os
import subprocess
import time

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "libedc_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(HERE, "edc_oracle.c")
        if not os.path.exists(SO) or os.path.getmtime(src) > os.path.getmtime(SO):
            subprocess.check_call(["make", "-C", HERE], stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(SO)
        c_sz, c_p, u64p = ctypes.c_size_t, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)
        L.oc_batch_verify.argtypes = [c_sz, c_p, c_p, c_p, u64p, c_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.oc_batch_verify_range.argtypes = [c_sz, c_p, c_p, c_p, u64p, c_p, c_p, ctypes.c_uint64, ctypes.c_void_p,
                                            ctypes.c_void_p]
        L.oc_verify.argtypes = [c_p, c_p, c_p, c_sz]
        L.oc_combine_affine.argtypes = [c_sz, c_p, ctypes.c_void_p]
        L.oc_partials_parallel.argtypes = [c_sz, c_p, c_p, c_p, u64p, c_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oc_baseline.restype = ctypes.c_double
        L.oc_baseline.argtypes = [c_sz, c_p, c_p, c_p, u64p, ctypes.c_int, c_sz, ctypes.POINTER(ctypes.c_int)]
        for f in (L.oc_bench_batch, L.oc_bench_single):
            f.restype = ctypes.c_double
            f.argtypes = [c_sz, c_p, c_p, c_p, u64p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


def _arena(msgs):
    offs = (ctypes.c_uint64 * (len(msgs) + 1))()
    t = 0
    for i, m in enumerate(msgs):
        offs[i] = t
        t += len(m)
    offs[len(msgs)] = t
    return b"".join(msgs) or b"\0", offs


def batch_verify(items, z_seed):
    """(code, check8 or None) -- same contract as ed25519_ref.batch_verify_seeded."""
    vks = b"".join(v for v, _, _ in items) or b"\0"
    sigs = b"".join(s for _, s, _ in items) or b"\0"
    arena, offs = _arena([bytes(m) for _, _, m in items])
    c8 = ctypes.create_string_buffer(32)
    ev = ctypes.c_int(0)
    rc = lib().oc_batch_verify(len(items), vks, sigs, arena, offs, bytes(z_seed), c8, ctypes.byref(ev))
    return rc, (c8.raw if ev.value else None)


def shard_partial_affine(items, z_seed, z_base):
    """This shard's check point (affine x || y, 64 bytes) and its early-reject flag."""
    vks = b"".join(v for v, _, _ in items) or b"\0"
    sigs = b"".join(s for _, s, _ in items) or b"\0"
    arena, offs = _arena([bytes(m) for _, _, m in items])
    part = ctypes.create_string_buffer(64)
    c8 = ctypes.create_string_buffer(32)
    rc = lib().oc_batch_verify_range(len(items), vks, sigs, arena, offs, bytes(z_seed), None, z_base, c8, part)
    evaluated = c8.raw != bytes(32)
    return part.raw, (not evaluated)


def combine_affine(parts):
    c8 = ctypes.create_string_buffer(32)
    rc = lib().oc_combine_affine(len(parts), b"".join(parts) or b"\0", c8)
    return rc, c8.raw


def batch_verify_parallel(vk, sig, msg, offs, z_seed, parts=None, z_base=0):
    """Whole-batch (code, check8) of a LARGE batch given as flat byte strings (vk n*32, sig n*64,
    the message arena and n+1 offsets) on all host threads: contiguous ranges at global z indices,
    one oc_batch_verify_range each, partial points summed by oc_combine_affine. check8 is None when
    a range was rejected before its MSM (the batch then fails, as in the reference). Test checker
    for full-size GPU batches; also returns the host seconds."""
    n = len(vk) // 32
    parts = parts or host_threads()
    o = (ctypes.c_uint64 * (n + 1))(*offs) if not isinstance(offs, ctypes.Array) else offs
    buf = ctypes.create_string_buffer(64 * parts)
    rcs, ev = (ctypes.c_int * parts)(), (ctypes.c_int * parts)()
    t0 = time.perf_counter()
    rc = lib().oc_partials_parallel(n, vk or b"\0", sig or b"\0", msg or b"\0", o, bytes(z_seed), parts, z_base, buf,
                                    rcs, ev)
    assert rc == 0
    if not all(ev):
        return 1, None, time.perf_counter() - t0
    code, c8 = combine_affine([buf.raw[64 * g:64 * g + 64] for g in range(parts)])
    return code, c8, time.perf_counter() - t0


def verify(vk, sig, msg):
    return lib().oc_verify(vk, sig, bytes(msg) or b"\0", len(msg))


def host_threads():
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, n)


def baseline(vks, sigs, msgs, threads=None, chunk=0):
    """All-core CPU baseline: one Verifier per thread over equal contiguous chunks, timing
    queue (SHA-512 + grouping) + verify like reference benches/bench.rs:42-68."""
    threads = threads or host_threads()
    arena, offs = _arena(msgs)
    ok = ctypes.c_int(0)
    secs = lib().oc_baseline(len(vks), b"".join(vks), b"".join(sigs), arena, offs, threads, chunk, ctypes.byref(ok))
    return secs, bool(ok.value), threads


def baseline_c3(n_sample=8192, keys=150, msg_len=120, data=None, min_seconds=1.5, max_reps=16):
    """Bounded sample of the bench workload shape (C3: repeated validator keys). The sample is
    verified repeatedly until min_seconds of wall time (~20-30 CPU-seconds on 16 threads) have
    been timed; the rate is all verified signatures over all timed seconds."""
    if data is None:
        raise ValueError("pass data=(vks, sigs, msgs) sampled from the GPU-generated workload")
    vks, sigs, msgs = data
    threads = host_threads()
    total, reps, ok = 0.0, 0, True
    while reps < max_reps and (reps == 0 or total < min_seconds):
        secs, ok_r, threads = baseline(vks, sigs, msgs, threads=threads)
        total += secs
        reps += 1
        ok = ok and ok_r
    return {"value": round(reps * len(vks) / total, 1), "unit": "sigs/s", "cores": threads, "kind": "port",
            "ok": ok, "seconds": round(total, 3), "repeats": reps,
            "sample": f"{len(vks)} sigs of the same workload ("
                      f"{f'{keys} validators' if keys else 'distinct keys'}, "
                      f"{f'{msg_len}-byte' if msg_len >= 0 else '0..1024-byte'} msgs), "
                      f"one Verifier per thread over {threads} equal chunks, queue+verify timed, "
                      f"{reps} repeats ({round(total * threads, 1)} CPU-seconds)"}


def bench_small(vks, sigs, msgs, batched, min_seconds=0.3):
    """One-thread rate (sigs/s) of queue+verify of this batch (batched) or of per-item
    try_from+verify (unbatched), repeated until min_seconds -- reference benches/bench.rs:25-71."""
    arena, offs = _arena(msgs)
    f = lib().oc_bench_batch if batched else lib().oc_bench_single
    ok = ctypes.c_int(0)
    reps, secs = 1, 0.0
    while True:
        secs = f(len(vks), b"".join(vks), b"".join(sigs), arena, offs, reps, ctypes.byref(ok))
        if secs >= min_seconds or reps >= 1 << 20:
            break
        reps = max(reps * 2, int(reps * min_seconds / max(secs, 1e-6)))
    return {"sigs_per_s": round(reps * len(vks) / secs, 1), "reps": reps, "seconds": round(secs, 3),
            "ok": bool(ok.value)}
