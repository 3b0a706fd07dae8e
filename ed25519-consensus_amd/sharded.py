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


class ExchangeRing:
    """Pipelined exchange of one fixed-size record per rank and batch (the 129-byte partial +
    reject flag). post() queues a batch's record and returns at once; every `group` records leave
    in ONE all-gather (group x 129 bytes per rank), so the per-collective costs -- the host's
    launch of the copies, the collective and the combine, and the collective's wait for a free CU
    on a full device -- are paid once per group; pop() completes the OLDEST batch (sending a
    partial group first if it is still pending) and returns its per-rank records (rank order).
    Every rank runs the same post/pop sequence, so the collectives match on all ranks and the
    verdicts complete in queue order.

    On a GPU device (RCCL) the staging copies, the collective and the combine run on a private
    high-priority non-blocking torch stream: the host never waits for the collective inside
    post(), and the engine's slot streams (blocking streams, hipExtStreamCreateWithCUMask takes no
    flags) never wait behind it. Each group in flight owns its pinned host and device buffers,
    reused only after its last pop(). On the CPU (gloo) the collective is async_op=True and pop()
    waits for its work handle.

    device_combine (GPU only): an Engine. The combine of each batch's gathered records is then
    enqueued on the same side stream right behind the collective (edc_combine_records_device: sum,
    x8, identity test on the device, no host round trip of the records), and pop() returns the
    verdict code instead of the records (`combines` is True)."""

    def __init__(self, dist, device, rec_len=129, depth=4, device_combine=None, group=1):
        import torch
        self.dist, self.n, self.K = dist, rec_len, max(1, group)
        self.world = dist.get_world_size()
        self.gpu = device.type != "cpu"
        self.eng = device_combine if self.gpu else None
        self.combines = self.eng is not None
        self.pending = []                 # records of the group being filled
        self.sent = []                    # [buffer index, records in the group, handle, records popped]
        nbuf = (depth + self.K) // self.K + 1
        K, n, W = self.K, rec_len, self.world
        if self.gpu:
            self.side = torch.cuda.Stream(device=device, priority=-1)
            nres = 256 * K if self.combines else W * K * n      # result blocks / the records
            with torch.cuda.stream(self.side):
                self.bufs = [(torch.empty(K * n, dtype=torch.uint8, pin_memory=True),
                              torch.empty(nres, dtype=torch.uint8, pin_memory=True),
                              torch.empty(K * n, dtype=torch.uint8, device=device),
                              torch.empty(W * K * n, dtype=torch.uint8, device=device),
                              torch.empty(256 * K, dtype=torch.uint8, device=device))
                             for _ in range(nbuf)]
        else:
            self.bufs = [(torch.empty(K * n, dtype=torch.uint8), torch.empty(W * K * n, dtype=torch.uint8))
                         for _ in range(nbuf)]
        self.free = list(range(nbuf))

    def __len__(self):
        return len(self.pending) + sum(cnt - done for _, cnt, _, done in self.sent)

    def warm(self):
        """Set-up outside a timed region: one full group through EVERY staging buffer at once (the
        free list is LIFO, so a single post/pop would only ever touch one of them). The first
        collective on each buffer pays the backend's per-buffer set-up (RCCL), which otherwise lands
        in the first timed batches. Every rank must call it (it runs collectives); the records are
        zeros and their results are discarded."""
        assert not self.pending and not self.sent, "ExchangeRing.warm: exchanges in flight"
        for _ in range(len(self.bufs)):
            for _ in range(self.K):
                self.post(bytes(self.n))
        while len(self):
            self.pop()

    def post(self, rec):
        assert len(rec) == self.n
        self.pending.append(bytes(rec))
        if len(self.pending) == self.K:
            self._send()

    def _send(self):
        import numpy as np
        import torch
        if not self.free:
            raise RuntimeError("ExchangeRing: more exchanges in flight than its depth; pop() first")
        i = self.free.pop()
        cnt, K, n = len(self.pending), self.K, self.n
        blob = b"".join(self.pending) + bytes((K - cnt) * n)      # a partial group is padded
        self.pending = []
        if self.gpu:
            h_in, h_out, d_in, d_out, d_res = self.bufs[i]
            with torch.cuda.stream(self.side):
                h_in.numpy()[:] = np.frombuffer(blob, dtype=np.uint8)
                d_in.copy_(h_in, non_blocking=True)
                work = self.dist.all_gather_into_tensor(d_out, d_in, async_op=True)
                work.wait()              # the side stream waits for the collective; the host does not
                if self.combines:        # batch k of the group: rank r's record at r K n + k n
                    for k in range(cnt):
                        self.eng.combine_records_device(self.side.cuda_stream, self.world, d_out.data_ptr() + k * n,
                                                        K * n, d_res.data_ptr() + 256 * k)
                    h_out.copy_(d_res, non_blocking=True)
                else:
                    h_out.copy_(d_out, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.side)
            self.sent.append([i, cnt, ev, 0])
        else:
            t_in, t_out = self.bufs[i]
            t_in.numpy()[:] = np.frombuffer(blob, dtype=np.uint8)
            self.sent.append([i, cnt, self.dist.all_gather_into_tensor(t_out, t_in, async_op=True), 0])

    def pop(self):
        if not self.sent:
            if not self.pending:
                raise RuntimeError("ExchangeRing.pop: nothing posted")
            self._send()                 # the oldest batch is still in the group being filled
        g = self.sent[0]
        i, cnt, h, k = g
        if k == 0:
            if self.gpu:
                h.synchronize()
            else:
                h.wait()
        g[3] += 1
        if g[3] == cnt:
            self.sent.pop(0)
            self.free.append(i)
        host = self.bufs[i][1].numpy()
        if self.combines:                # the device's verdict word: 0 Ok, 1 reject
            return int.from_bytes(host[256 * k:256 * k + 4].tobytes(), "little")
        K, n = self.K, self.n
        return [host[r * K * n + k * n:r * K * n + (k + 1) * n].tobytes() for r in range(self.world)]


def run_sharded_stream(k, inflight, submit_fn, wait_fn, combine_fn, ring, lag):
    """bench.py's multi-rank loop: k consecutive batches of this rank's shard, `inflight` of them
    submitted ahead on the device and `lag` exchanges in flight. When the oldest batch is
    collected, the freed slot is refilled first (the device stays full), then the batch's record
    is posted to the ring, and exchanges older than `lag` are completed and combined. Returns the
    verdict codes in batch order.

    submit_fn() -> ticket                     enqueue the next batch of this rank's shard
    wait_fn(ticket) -> (partial_128, bad)     its partial point and early-reject flag
    combine_fn(partials, bad_any) -> code     [8]*sum == identity over the ranks' partials
    """
    pending, codes = [], []

    def finish():
        res = ring.pop()
        if getattr(ring, "combines", False):         # combined on the device behind the collective
            codes.append(res)
        else:
            codes.append(combine_fn([r[:128] for r in res], any(r[128] for r in res)))

    def post(res):
        part, bad = res
        ring.post(bytes(part) + bytes([1 if bad else 0]))
        while len(ring) > lag:
            finish()

    for _ in range(k):
        res = wait_fn(pending.pop(0)) if len(pending) >= max(1, inflight) else None
        pending.append(submit_fn())
        if res is not None:
            post(res)
    while pending:
        post(wait_fn(pending.pop(0)))
    while len(ring):
        finish()
    return codes


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

