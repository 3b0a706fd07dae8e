"""Multi-GPU batch verification: one process per GPU, one batch equation.

The batch equation is linear (reference src/batch.rs:150-172): with the z_i drawn from one
ChaCha20 stream at GLOBAL queue indices, shard g's part
    P_g = [-sum_{i in g} z_i s_i]B + sum_keys [sum_{i in g} z_i k_i]A + sum_{i in g} [z_i]R_i
satisfies check = sum_g P_g exactly. Each rank evaluates its contiguous slice of the queue on
its own GPU (edc_batch_partial_device) and the ranks exchange ONE 128-byte partial point each
(all-gather; RCCL over xGMI when the group backend is nccl); every rank then combines the
partials and applies [8] / identity (edc_combine_partials) -- bit-identical to the unsharded
verdict and [8]*check for any number of shards.
"""


def shard_bounds(n_total, world):
    """Contiguous queue slices [lo, hi) per rank."""
    return [(n_total * r // world, n_total * (r + 1) // world) for r in range(world)]


def verify_sharded(partial_fn, combine_fn, allgather_fn, rank, world, n_local_base):
    """Generic driver (also used by the gloo CPU tests with oracle callbacks).

    partial_fn(z_base) -> (partial_bytes_128, bad_flag) for this rank's slice
    allgather_fn(bytes_129) -> list of per-rank bytes_129 (rank order)
    combine_fn(list_of_partials, bad_any) -> (code, check8)
    """
    part, bad = partial_fn(n_local_base)
    rec = bytes(part) + bytes([1 if bad else 0])
    recs = allgather_fn(rec)
    assert len(recs) == world
    partials = [r[:128] for r in recs]
    bad_any = any(r[128] for r in recs)
    return combine_fn(partials, bad_any)


def torch_allgather_fn(dist, device):
    """all_gather of fixed 129-byte records over the default process group.

    On a GPU device every tensor op runs on a private non-blocking torch stream: the engine's
    slot streams are blocking streams (hipExtStreamCreateWithCUMask takes no flags), so any work
    on the legacy default stream would wait for -- and hold back -- every batch in flight. The
    staging buffers are pinned and reused so the copies stay asynchronous DMA on that stream."""
    import numpy as np
    import torch

    if device.type == "cpu":
        def fn_cpu(rec):
            world = dist.get_world_size()
            t = torch.frombuffer(bytearray(rec), dtype=torch.uint8)
            out = torch.empty(world * len(rec), dtype=torch.uint8)
            dist.all_gather_into_tensor(out, t)
            host = out.numpy().tobytes()
            return [host[i * len(rec):(i + 1) * len(rec)] for i in range(world)]
        return fn_cpu

    side = torch.cuda.Stream(device=device)
    bufs = {}

    def fn(rec):
        world = dist.get_world_size()
        n = len(rec)
        if n not in bufs:
            with torch.cuda.stream(side):
                bufs[n] = (torch.empty(n, dtype=torch.uint8, pin_memory=True),
                           torch.empty(world * n, dtype=torch.uint8, pin_memory=True),
                           torch.empty(n, dtype=torch.uint8, device=device),
                           torch.empty(world * n, dtype=torch.uint8, device=device))
        h_in, h_out, d_in, d_out = bufs[n]
        with torch.cuda.stream(side):
            h_in.numpy()[:] = np.frombuffer(rec, dtype=np.uint8)
            d_in.copy_(h_in, non_blocking=True)
            dist.all_gather_into_tensor(d_out, d_in)
            h_out.copy_(d_out, non_blocking=True)
            side.synchronize()
            host = h_out.numpy().tobytes()
        return [host[i * n:(i + 1) * n] for i in range(world)]

    return fn


def find_invalid_sharded(shard_ok_fn, find_fn, allgather_obj_fn, rank, world, lo):
    """Multi-GPU fallback after a failed global batch (the caller's verify_single loop
    of reference tests/batch.rs:37-43). Every shard's own partial satisfies [8]P_g == 0 when all of
    its items are valid, so only the ranks whose partial fails localize their invalid items
    (edc_find_invalid_device on the local slice, per-item codes == Item::verify_single). The
    (global queue index, code) pairs are all-gathered; every rank returns the same sorted list.

    shard_ok_fn() -> bool      this rank's partial alone verifies ([8]P_g == 0, nothing undecodable)
    find_fn() -> [(i, code)]   invalid items of the local slice, local indices, codes 1 / 2
    allgather_obj_fn(obj) -> list of per-rank objects (rank order)
    """
    local = [] if shard_ok_fn() else [(lo + i, c) for i, c in find_fn()]
    recs = allgather_obj_fn(local)
    assert len(recs) == world
    return sorted(x for r in recs for x in r)


def torch_allgather_obj_fn(dist):
    """all_gather_object over the default process group (small per-rank lists)."""
    def fn(obj):
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, obj)
        return [list(map(tuple, o)) for o in out]

    return fn

