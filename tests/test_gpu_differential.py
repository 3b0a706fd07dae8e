"""GPU: seeded differential test against the C oracle (oracle/edc_oracle.c, the dalek u64 algorithm)
over many mixed batches. Each batch draws its items from: honest GPU-signed votes (a few validators
or distinct keys, random message lengths), the ZIP215 small-order / non-canonical corpus
(tests/golden/zip215_small_order.json: accepted by ZIP215 batch and single verification alike),
corrupted signatures and messages, s >= l, undecodable R and A encodings (tests/golden/decode.json),
and duplicated items. For every batch the GPU's verdict and [8]*check (src/batch.rs:149-217) and
every item's verify_single code (src/batch.rs:104-107, verification_key.rs:225-258) must equal the
oracle's, through the message path, the prehashed path and (for sizes that allow it) a union-first
multi launch of the batch split in two. EDC_DIFF_SEEDS=<k> runs k seeds of each test instead of the
default 8 / 3 (soak runs of the final tree: profiles/r06/r06z_differential_soak.log)."""
import os
import random
import sys

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

L_ORDER = 2**252 + 27742317777372353535851937790883648493
CORPUS = golden("zip215_small_order.json")
BAD_ENC = [bytes.fromhex(c["enc"]) for c in golden("decode.json")["cases"] if not c["ok"]]


@pytest.fixture(scope="module")
def oc():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    return oracle_c


def _batch(engine, rnd, n, hard=None):
    """Mixed items; "hard" batches also hold items rejected before the MSM (undecodable R / key,
    s >= l, a flipped R byte), "soft" ones only items whose rejection the MSM must find (a wrong
    message, a flipped low byte of s), so large failing batches compare a non-identity check8."""
    hard = rnd.random() < 0.35 if hard is None else hard
    nkeys = rnd.choice([1, 3, 17, n])
    seeds = [rnd.randbytes(32) for _ in range(nkeys)]
    msgs = [rnd.randbytes(rnd.choice([0, 1, 32, 111, 112, 120, 200, rnd.randrange(0, 400)])) for _ in range(n)]
    vks, sigs = engine.sign(seeds, msgs, seed_index=[rnd.randrange(nkeys) for _ in range(n)])
    vks, sigs = list(vks), list(sigs)
    cmsg = bytes.fromhex(CORPUS["msg"])
    for i in range(n):
        r = rnd.random()
        if r < 0.02:                                   # a ZIP215 corpus item (valid under ZIP215)
            c = rnd.choice(CORPUS["cases"])
            vks[i], sigs[i], msgs[i] = bytes.fromhex(c["vk"]), bytes.fromhex(c["sig"]), cmsg
        elif r < 0.025:                                # corrupted signature byte (R anywhere if hard)
            j = rnd.randrange(64) if hard else rnd.randrange(32, 62)
            sigs[i] = sigs[i][:j] + bytes([sigs[i][j] ^ (1 << rnd.randrange(8))]) + sigs[i][j + 1:]
        elif r < 0.03:                                 # corrupted message
            msgs[i] = msgs[i] + b"\x00"
        elif not hard:
            if r < 0.04 and i:                         # duplicate of an earlier item
                j = rnd.randrange(i)
                vks[i], sigs[i], msgs[i] = vks[j], sigs[j], msgs[j]
        elif r < 0.033:                                # s + l (non-canonical s)
            s = int.from_bytes(sigs[i][32:], "little") + L_ORDER
            if s < 2**256:
                sigs[i] = sigs[i][:32] + s.to_bytes(32, "little")
        elif r < 0.036:                                # undecodable R
            sigs[i] = rnd.choice(BAD_ENC) + sigs[i][32:]
        elif r < 0.039:                                # undecodable key
            vks[i] = rnd.choice(BAD_ENC)
        elif r < 0.05 and i:                           # duplicate of an earlier item
            j = rnd.randrange(i)
            vks[i], sigs[i], msgs[i] = vks[j], sigs[j], msgs[j]
    return vks, sigs, msgs


SOAK = int(os.environ.get("EDC_DIFF_SEEDS", "0"))


@pytest.mark.parametrize("seed", range(SOAK or 8))
def test_mixed_batches_vs_oracle(engine, oc, seed):
    rnd = random.Random(9000 + seed)
    codes = []
    for trial in range(12):
        n = rnd.choice([1, 2, 7, 64, 150, 511, 1024, 2048, 3000, 4096])
        vks, sigs, msgs = _batch(engine, rnd, n)
        zseed = rnd.randbytes(32)
        items = list(zip(vks, sigs, msgs))
        exp_code, exp_c8 = oc.batch_verify(items, zseed)
        code, c8 = engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
        tag = f"seed {seed} trial {trial} n {n}"
        assert code == exp_code, tag
        assert c8 == (exp_c8 if exp_c8 is not None else bytes(32)), tag
        codes.append((n, code, exp_c8 is not None))
        ks = engine.challenge(vks, sigs, msgs)
        pcode, pc8 = engine.batch_verify_prehashed(vks, sigs, ks, z_seed=zseed, want_check8=True)
        assert (pcode, pc8) == (code, c8), tag
        if trial % 3 == 0:                             # per-item codes on a subset of the batches
            exp_each = [oc.verify(v, s, m) for v, s, m in items]
            assert engine.verify_each(vks, sigs, msgs) == exp_each, tag
            assert engine.verify_prehashed_each(vks, sigs, ks) == exp_each, tag
    print(f"\n[differential] seed {seed}: (n, code, evaluated) {codes}")
    if not SOAK:   # the fixed seeds draw both outcomes; a soak seed may draw only failing batches
        assert any(c == 0 for _, c, _ in codes) and any(c == 1 for _, c, _ in codes)


@pytest.mark.parametrize("seed", range(SOAK or 3))
def test_mixed_multi_union_vs_oracle(engine, oc, seed):
    """The same mixtures as two consecutive batches of one union-first launch: each batch's
    verdict and check8 equal the oracle's for that batch at its global z offset."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    rnd = random.Random(7100 + seed)
    n_per = 2048
    for trial in range(3):
        vks, sigs, msgs = _batch(engine, rnd, 2 * n_per)
        zseed = rnd.randbytes(32)
        offs = [0]
        for m in msgs:
            offs.append(offs[-1] + len(m))
        t8 = lambda b: torch.tensor(list(b) or [0], dtype=torch.uint8, device=dev)
        d_vk, d_sig, d_msg = t8(b"".join(vks)), t8(b"".join(sigs)), t8(b"".join(msgs))
        d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        t = engine.batch_submit_multi_device(2, n_per, d_vk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                             d_off.data_ptr(), zseed, 0, want_check8=True)
        code, verdicts, c8s, _, _ = engine.batch_wait_multi(t, 2)
        for b in range(2):
            lo, hi = b * n_per, (b + 1) * n_per
            o = [x - offs[lo] for x in offs[lo:hi + 1]]
            ec, e8, _ = oc.batch_verify_parallel(b"".join(vks[lo:hi]), b"".join(sigs[lo:hi]),
                                                 b"".join(msgs[lo:hi]), o, zseed, parts=2, z_base=lo)
            assert verdicts[b] == ec, (seed, trial, b)
            assert c8s[b] == (e8 if e8 is not None else bytes(32)), (seed, trial, b)


@pytest.mark.parametrize("n", [16384, 131072])
def test_large_mixed_batch_vs_oracle(engine, oc, n):
    """One larger mixed batch (larger MSM plans: 12-15-bit windows, parts, sub-bins) against the
    threaded C oracle: verdict and [8]*check, message and prehashed paths."""
    rnd = random.Random(n)
    vks, sigs, msgs = _batch(engine, rnd, n, hard=False)
    zseed = rnd.randbytes(32)
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    ec, e8, secs = oc.batch_verify_parallel(b"".join(vks), b"".join(sigs), b"".join(msgs), offs, zseed)
    code, c8 = engine.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    print(f"\n[differential-large] n {n}: code {code}, evaluated {e8 is not None}, oracle {secs:.2f} s")
    assert code == ec
    assert c8 == (e8 if e8 is not None else bytes(32))
    ks = engine.challenge(vks, sigs, msgs)
    assert engine.batch_verify_prehashed(vks, sigs, ks, z_seed=zseed, want_check8=True) == (code, c8)
