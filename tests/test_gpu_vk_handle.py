"""GPU: per-object decoded keys. The reference's VerificationKey decodes A once at try_from and
keeps minus_A for every later verify (src/verification_key.rs:106-114, :160-175, :251). The mirror's
VerificationKey.try_from adds the key to the engine's cache (edc_keycache_add: grows the cache, the
cached keys keep their places), so later per-item verifies, batches and fallbacks find the decoded
point. None of this may change a verdict or a [8]*check: checked against the golden batches
(tests/golden/batches.json, the RFC 8032 vectors, the ZIP215 corpus) and against the same engine
without a cache; the growth path (capacity doubling over several additions) and the indexed-key
list of edc_keycache_load surviving an addition are covered too."""
import random

import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

BATCHES = golden("batches.json")["batches"]


@pytest.fixture()
def cached(engine):
    engine.keycache_clear()
    yield engine
    engine.keycache_clear()


def _items(b):
    return ([bytes.fromhex(v) for v, _, _ in b["items"]], [bytes.fromhex(s) for _, s, _ in b["items"]],
            [bytes.fromhex(m) for _, _, m in b["items"]])


def test_try_from_keeps_decoded_key(cached, edc):
    vectors = golden("rfc8032.json")["vectors"]
    seen = set()
    for v in vectors:
        pk, sig, msg = (bytes.fromhex(v[k]) for k in ("pk", "sig", "msg"))
        vk = edc.VerificationKey.try_from(pk, cached)
        seen.add(pk)
        assert vk.cached and cached.keycache_size() == len(seen)
        vk.verify(sig, msg)
        with pytest.raises(edc.InvalidSignature):
            vk.verify(sig, msg + b"!")
        again = edc.VerificationKey.try_from(pk, cached)          # already cached: no growth
        assert again.cached and cached.keycache_size() == len(seen)
    plain = edc.VerificationKey.try_from(bytes.fromhex(vectors[0]["pk"]), cached, keep_decoded=False)
    assert not plain.cached


def test_try_from_malformed_key(cached, edc):
    bad = [bytes.fromhex(c["enc"]) for c in golden("decode.json")["cases"] if not c["ok"]]
    for enc in bad[:4]:
        with pytest.raises(edc.MalformedPublicKey):
            edc.VerificationKey.try_from(enc, cached)
    got = edc.VerificationKey.try_from_many(bad[:4] + [bad[0]], cached, keep_decoded=True)
    assert all(isinstance(g, edc.MalformedPublicKey) for g in got)
    assert cached.keycache_size() == 0                  # malformed keys never enter the cache
    n0, ok = cached.keycache_add(bad[:4])
    assert n0 == 0 and not any(ok)


def test_zip215_corpus_with_decoded_keys(cached, edc):
    fx = golden("zip215_small_order.json")
    msg = bytes.fromhex(fx["msg"])
    vks = [bytes.fromhex(c["vk"]) for c in fx["cases"]]
    sigs = [bytes.fromhex(c["sig"]) for c in fx["cases"]]
    expect = [c["expect_single"] for c in fx["cases"]]
    assert cached.verify_each(vks, sigs, [msg] * len(vks)) == expect          # no cache
    handles = edc.VerificationKey.try_from_many(vks, cached, keep_decoded=True)
    assert all(h.cached for h in handles)
    assert cached.verify_each(vks, sigs, [msg] * len(vks)) == expect          # every key cached
    for h, sig, e in list(zip(handles, sigs, expect))[::7]:
        if e == 0:
            h.verify(sig, msg)
        else:
            with pytest.raises(edc.Error):
                h.verify(sig, msg)


@pytest.mark.parametrize("b", BATCHES, ids=lambda b: b["name"])
def test_golden_batches_after_incremental_add(cached, b):
    vks, sigs, msgs = _items(b)
    zseed = bytes.fromhex(b["z_seed"])
    distinct = list(dict.fromkeys(vks))
    half = len(distinct) // 2
    for part in (distinct[:half], distinct[half:]):                # two additions, second grows
        if part:
            cached.keycache_add(part)
        code, check8 = cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
        assert code == b["expect_code"], b["name"]
        if b["expect_check8"] is not None:
            assert check8.hex() == b["expect_check8"], b["name"]
    # keys that do not decode are not added (edc_keycache_add): the cache holds the decodable ones
    assert cached.keycache_size() == sum(1 for c in cached.vk_validate(distinct) if c == 0)
    assert cached.verify_each(vks, sigs, msgs) == b["expect_single"]


def test_growth_and_registered_list(cached):
    """300 keys added in uneven chunks (capacity 16 -> 512 over several reallocations) after a
    registered list of 10: the registered indices still address the same keys, every key is found,
    and a failing batch's [8]*check equals the one computed with no cache."""
    rnd = random.Random(2024)
    n, m = 4096, 310
    seeds = [rnd.randbytes(32) for _ in range(m)]
    msgs = [rnd.randbytes(rnd.randrange(0, 160)) for _ in range(n)]
    vks, sigs = cached.sign(seeds, msgs, seed_index=[i % m for i in range(n)])
    msgs[1234] = msgs[1234] + b"x"
    zseed = rnd.randbytes(32)
    ref = cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True)
    ref_each = cached.verify_each(vks, sigs, msgs)
    assert ref[0] == 1 and ref_each.count(1) == 1
    keys = list(dict.fromkeys(vks))
    assert len(keys) == m
    u, ok = cached.keycache_load(keys[:10])
    assert u == 10 and all(ok)
    sizes = []
    lo = 10
    for step in (3, 14, 40, 1, 90, 152):
        u, ok = cached.keycache_add(keys[lo:lo + step] + keys[:2])            # with duplicates
        assert all(ok)
        lo += step
        sizes.append(u)
    assert sizes == [13, 27, 67, 68, 158, 310] and cached.keycache_size() == m
    assert cached.batch_verify(vks, sigs, msgs, z_seed=zseed, want_check8=True) == ref
    assert cached.verify_each(vks, sigs, msgs) == ref_each
    # the indexed entry still maps position j of the loaded list to keys[j]
    idx = [i % 10 for i in range(n)]
    ivk = [keys[j] for j in idx]
    isig = [sigs[i] if vks[i] == ivk[i] else None for i in range(n)]
    sel = [i for i in range(n) if isig[i] is not None]
    t = cached.batch_submit_indexed([idx[i] for i in sel], [sigs[i] for i in sel], [msgs[i] for i in sel],
                                    zseed, want_check8=True)
    got = cached.batch_wait(t, want_check8=True)
    want = cached.batch_verify([vks[i] for i in sel], [sigs[i] for i in sel], [msgs[i] for i in sel],
                               z_seed=zseed, want_check8=True)
    assert got == want
