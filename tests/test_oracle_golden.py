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


# Published known answer for the original ChaCha20 layout (64-bit block counter in words 12-13,
# 64-bit nonce in words 14-15 -- the layout of rand_chacha's ChaCha20Rng, which the reference's
# z draws use, src/batch.rs:64-68 via rand_core 0.6): key = 0, nonce = 0, blocks 0 and 1
# (draft-strombergson-chacha-test-vectors TC1, also rand_chacha's `test_chacha_true_values_a`
# as u32 words 0xade0b876, 0x903df1a0, ... / 0xbee7079f, 0x7a385155, ...). Block 1 pins the
# counter word the z stream advances, beyond the block-0 vector above.
CHACHA20_ZERO_KEY_BLOCKS_0_1 = (
    "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
    "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586"
    "9f07e7be5551387a98ba977c732d080dcb0f29a048e3656912c6533e32ee7aed"
    "29b721769ce64e43d57133b074d839d531ed1f28510afb45ace10a1f4b794d6f")


def test_chacha_two_block_known_answer(oracle):
    assert oracle.chacha20_keystream(bytes(32), 128).hex() == CHACHA20_ZERO_KEY_BLOCKS_0_1
    # z_i = u128 of keystream bytes [16 i, 16 i + 16) little-endian (rand 0.8 Standard for u128:
    # first next_u64 is the low half; BlockRng::next_u64 joins two u32 words low first)
    z = oracle.z_values(bytes(32), 8)
    ks = bytes.fromhex(CHACHA20_ZERO_KEY_BLOCKS_0_1)
    assert z == [int.from_bytes(ks[16 * i:16 * i + 16], "little") for i in range(8)]
    assert z[0] == 0x28bd8653e56a5d40903df1a0ade0b876


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
