"""CPU: the C-ABI library loads and exports every symbol include/edc.h declares; the host
mirror exposes the reference API surface. No compute calls (no GPU here)."""
import ctypes
import os
import re

from conftest import ROOT


def header_symbols():
    src = open(os.path.join(ROOT, "include", "edc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(edc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol(edc):
    lib = edc.load_library()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(lib, s), f"libedc.so does not export {s}"
    assert sorted(edc.ABI_SYMBOLS) == syms


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "ed25519-consensus_amd", "csrc", "libedc.so")
    blob = open(so, "rb").read()
    assert b"gfx950" in blob


def test_timing_names_without_gpu(edc):
    lib = edc.load_library()
    names = [lib.edc_timing_name(i).decode() for i in range(7)]
    assert set(names) == {"keys_group", "challenge_sha512", "decompress_R", "coef_chacha_scalar", "msm_bin",
                          "msm_bucket", "msm_window_final"} and names[-1] == "msm_window_final"
    assert lib.edc_timing_name(99) == b""


def test_reference_api_surface(edc):
    # names mirror ed25519_consensus: Error variants, Signature, VerificationKey(Bytes), batch
    for name in ["Signature", "VerificationKeyBytes", "VerificationKey", "SigningKey", "InvalidSignature",
                 "MalformedPublicKey", "InvalidSliceLength"]:
        assert hasattr(edc, name)
    assert hasattr(edc.batch, "Verifier") and hasattr(edc.batch, "Item")
    assert hasattr(edc.batch.Item, "verify_single")
    sig = edc.Signature(bytes(range(64)))
    assert sig.R_bytes == bytes(range(32)) and sig.to_bytes() == bytes(range(64))
    try:
        edc.Signature(bytes(63))
        raise AssertionError("expected InvalidSliceLength")
    except edc.InvalidSliceLength:
        pass
    try:
        edc.VerificationKeyBytes(bytes(33))
        raise AssertionError("expected InvalidSliceLength")
    except edc.InvalidSliceLength:
        pass
    a, b = edc.VerificationKeyBytes(bytes(32)), edc.VerificationKeyBytes(bytes(32))
    assert a == b and hash(a) == hash(b)


def test_no_gpu_means_loud_failure(edc):
    lib = edc.load_library()
    if lib.edc_device_count() > 0:
        return  # on a GPU box this check does not apply
    try:
        edc.Engine(0)
        raise AssertionError("Engine must refuse to run without a GPU")
    except edc.EngineError:
        pass


def test_prehashed_item_surface(edc):
    """batch.Item as the reference stores it ({vk_bytes, sig, k}, src/batch.rs:76-80): built from
    the message (k hashed later, in one launch) or from a canonical k alone; k >= l is a ValueError."""
    vk, sig = bytes(32), bytes(64)
    k = bytes(range(31)) + b"\x0f"                      # < l
    it = edc.batch.Item.prehashed(vk, sig, k)
    assert it.k == k and it._msg is None
    try:                                                # k >= l: never from Scalar::from_hash
        edc.batch.Item.prehashed(vk, sig, bytes(range(32)))
        raise AssertionError("expected ValueError")
    except ValueError:
        pass
    assert edc.batch.Item(vk, sig, b"m").k is None
    try:
        edc.batch.Item(vk, sig)
        raise AssertionError("expected ValueError")
    except ValueError:
        pass
    try:
        edc.batch.Item.prehashed(vk, sig, bytes(31))
        raise AssertionError("expected InvalidSliceLength")
    except edc.InvalidSliceLength:
        pass
    v = edc.batch.Verifier()
    v.queue(it)
    v.queue((vk, sig, b"x"))
    assert v.batch_size == 2
