"""Diagnostic: edc_batch_submit_multi_device against one-batch verifies on small valid inputs
(prints verdicts, bad flags, check8 per batch for several shapes and grouping modes)."""
import ctypes
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    pkg = bench.load_pkg()
    eng = pkg.Engine(0)
    lib = eng.lib
    for nb, n_per, keys, grouping in [(1, 2048, 20, 1), (1, 2048, 0, 2), (2, 2048, 20, 1), (2, 2048, 0, 2),
                                      (4, 2048, 20, 0), (2, 4096, 20, 1)]:
        n = nb * n_per
        rnd = random.Random(n + keys)
        nk = keys or n
        seeds = [rnd.randbytes(32) for _ in range(nk)]
        msgs = [rnd.randbytes(48) for _ in range(n)]
        vks, sigs = eng.sign(seeds, msgs, seed_index=[i % nk for i in range(n)])
        t8 = lambda b: torch.tensor(list(b), dtype=torch.uint8, device=dev)
        d_vk, d_sig, d_msg = t8(b"".join(vks)), t8(b"".join(sigs)), t8(b"".join(msgs))
        d_off = torch.arange(0, n + 1, dtype=torch.int64, device=dev) * 48
        torch.cuda.synchronize()
        eng.set_key_grouping(grouping)
        zseed = bytes([7]) * 32
        t = eng.batch_submit_multi_device(nb, n_per, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                          d_off.data_ptr(), zseed, 0, want_check8=True)
        code, verdicts, c8s, parts, bads = eng.batch_wait_multi(t, nb)
        singles = []
        for b in range(nb):
            lo = b * n_per
            c8 = ctypes.create_string_buffer(32)
            o = (d_off[lo:lo + n_per + 1] - 48 * lo).contiguous()
            rc = lib.edc_batch_verify_device(eng.ctx, n_per, d_vk.data_ptr() + 32 * lo, d_sig.data_ptr() + 64 * lo,
                                             d_msg.data_ptr() + 48 * lo, o.data_ptr(), zseed, lo, None, c8)
            singles.append((rc, c8.raw[:8].hex()))
        print(f"nb={nb} n_per={n_per} keys={keys} grouping={grouping}: multi code={code} verdicts={verdicts} "
              f"bad={bads} c8={[c[:8].hex() for c in c8s]} singles={singles}", flush=True)
        eng.set_key_grouping(0)
    eng.close()


if __name__ == "__main__":
    main()
