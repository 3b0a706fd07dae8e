"""CPU: pin the oracle against the reference's own vectors, then check the committed fixtures
are exactly the oracle's outputs (reference tests/rfc8032.rs, tests/small_order.rs,
tests/batch.rs, tests/util/mod.rs)."""
import ctypes
import ctypes.util
import hashlib
import os

import pytest

from conftest import golden


def test_rfc8032_vectors(oracle):
    # tests/rfc8032.rs:13-40: verify Ok, pk regenerated from sk, deterministic re-sign
    for v in golden("rfc8032.json")["vectors"]:
        sk, pk, sig, msg = (bytes.fromhex(v[k]) for k in ("sk", "pk", "sig", "msg"))
        assert oracle.verify(pk, sig, msg) == oracle.OK
        assert oracle.public_key(sk) == pk
        assert oracle.sign(sk, msg) == sig
        # the 64-byte expanded form (rfc8032.rs:82-124) is SHA-512(seed): same key material
        a, prefix = oracle.expand_seed(sk)
        assert hashlib.sha512(sk).digest()[32:] == prefix


def test_small_order_corpus_matches_reference_construction(oracle):
    fx = golden("zip215_small_order.json")
    encs = oracle.eight_torsion_encodings() + oracle.non_canonical_point_encodings()[:6]
    assert [e.hex() for e in encs] == fx["encodings"]
    assert len(fx["cases"]) == 196
    for c in fx["cases"]:
        assert c["valid_zip215"] is True


def test_small_order_corpus_all_valid_single_and_batch(oracle):
    # tests/small_order.rs:79-104: every case verifies, individual == batch
    z = bytes([0x33]) * 32
    for vk, sig in oracle.small_order_corpus():
        single = oracle.verify(vk, sig, b"Zcash")
        b, _ = oracle.batch_verify_seeded([(vk, sig, b"Zcash")], z)
        assert single == oracle.OK and b == oracle.OK


def test_non_canonical_encodings_facts(oracle):
    # tests/util/mod.rs:81-155; the comment says 25 but the construction yields 26
    nc = oracle.non_canonical_point_encodings()
    assert len(nc) == 26
    assert [oracle.point_order(oracle.decompress(e)) for e in nc[:6]] == ["1", "2", "4", "4", "1", "1"]


def test_excluded_encodings_decode(oracle):
    # tests/util/mod.rs:193-202 prints which libsodium-excluded encodings decode
    res = [oracle.decompress(e) is not None for e in oracle.EXCLUDED_POINT_ENCODINGS]
    assert res == [True, True, True, True, True, False, True, True, True, False, True]


def test_decode_fixture_is_oracle_output(oracle):
    for c in golden("decode.json")["cases"]:
        pt = oracle.decompress(bytes.fromhex(c["enc"]))
        assert (pt is not None) == c["ok"]
        if pt is not None:
            assert (pt[0] % oracle.P).to_bytes(32, "little").hex() == c["x"]
            assert (pt[1] % oracle.P).to_bytes(32, "little").hex() == c["y"]


def test_chacha_stream(oracle):
    fx = golden("chacha_z.json")
    # RFC 7539 2.3.2-style known answer: zero key, zero nonce, block 0
    assert oracle.chacha20_block(bytes(32), 0).hex().startswith("76b8e0ada0f13d90405d6ae55386bd28")
    assert fx["zero_key_block0"] == oracle.chacha20_block(bytes(32), 0).hex()
    seed = bytes.fromhex(fx["seed"])
    assert [z.to_bytes(16, "little").hex() for z in oracle.z_values(seed, 64)] == fx["z"]
    assert [z.to_bytes(16, "little").hex() for z in oracle.z_values(seed, 8, start=1001)] == fx["z_from_1001"]


def test_scalars_fixture(oracle):
    fx = golden("scalars.json")
    for c in fx["from_hash"]:
        assert oracle.scalar_from_hash(bytes.fromhex(c["digest"])).to_bytes(32, "little").hex() == c["k"]
    for c in fx["from_canonical_bytes"]:
        assert (oracle.scalar_from_canonical_bytes(bytes.fromhex(c["s"])) is not None) == c["canonical"]


@pytest.mark.parametrize("name", ["empty", "one_valid", "batch_verify_32", "batch_verify_one_bad",
                                  "noncanonical_s_eq_l", "undecodable_A", "wrong_key", "torsion_R",
                                  "twin_encodings", "repeated_keys_3"])
def test_batch_fixtures_reproduce(oracle, name):
    b = [x for x in golden("batches.json")["batches"] if x["name"] == name][0]
    items = [(bytes.fromhex(v), bytes.fromhex(s), bytes.fromhex(m)) for v, s, m in b["items"]]
    code, check8 = oracle.batch_verify_seeded(items, bytes.fromhex(b["z_seed"]))
    assert code == b["expect_code"]
    assert (check8.hex() if check8 else None) == b["expect_check8"]
    assert [oracle.verify(*it) for it in items] == b["expect_single"]


def test_batch_semantics_from_reference_tests():
    # tests/batch.rs:18-44: batch fails, verify_single pinpoints exactly index 10
    b = [x for x in golden("batches.json")["batches"] if x["name"] == "batch_verify_one_bad"][0]
    assert b["expect_code"] == 1
    assert [i for i, c in enumerate(b["expect_single"]) if c] == [10]
    # ZIP215: a batch is valid iff every item is valid (batch == single) on every fixture
    for x in golden("batches.json")["batches"]:
        assert (x["expect_code"] == 0) == all(c == 0 for c in x["expect_single"]), x["name"]


def _libsodium():
    for p in ["/opt/conda/lib/libsodium.so", ctypes.util.find_library("sodium")]:
        if p and os.path.exists(p):
            try:
                return ctypes.CDLL(p)
            except OSError:
                pass
    return None


def test_libsodium_cross_check_on_canonical_signatures(oracle):
    """Secondary (non-oracle) check: libsodium agrees on canonical, torsion-free signatures."""
    lib = _libsodium()
    if lib is None:
        pytest.skip("libsodium not present")
    assert lib.sodium_init() >= 0
    for i in range(8):
        seed = hashlib.sha256(b"sodium%d" % i).digest()
        msg = hashlib.sha256(b"m%d" % i).digest()[: i * 3]
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        assert lib.crypto_sign_seed_keypair(pk, sk, seed) == 0
        sig = ctypes.create_string_buffer(64)
        assert lib.crypto_sign_detached(sig, None, msg, ctypes.c_ulonglong(len(msg)), sk) == 0
        assert pk.raw == oracle.public_key(seed)
        assert sig.raw == oracle.sign(seed, msg)
        assert oracle.verify(pk.raw, sig.raw, msg) == oracle.OK
        bad = bytearray(sig.raw)
        bad[5] ^= 1
        assert lib.crypto_sign_verify_detached(bytes(bad), msg, ctypes.c_ulonglong(len(msg)), pk.raw) != 0
        assert oracle.verify(pk.raw, bytes(bad), msg) != oracle.OK
