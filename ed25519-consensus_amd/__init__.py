"""ed25519-consensus on MI355X -- Python host mirror of the reference's verification API.

The reference (informalsystems/ed25519-consensus 2.1.0) is Rust; no Rust toolchain exists in
this image, so the host side above the C ABI (include/edc.h, built as csrc/libedc.so) is this
module (the Rust binding a maintainer would add is in INTEGRATION.md). Names, argument meaning and error behaviour follow the
reference:

    reference                                   here
    ---------------------------------------     -------------------------------------------
    Error::{MalformedPublicKey, InvalidSignature, InvalidSliceLength}  (src/error.rs:7-20)
                                                 MalformedPublicKey / InvalidSignature /
                                                 InvalidSliceLength exceptions
    Signature (src/signature.rs)                 Signature
    VerificationKeyBytes (src/verification_key.rs:32-87)      VerificationKeyBytes
    VerificationKey::try_from / verify (:160-258)            VerificationKey
    batch::Item, Item::verify_single (src/batch.rs:75-107)   batch.Item
    batch::Verifier::{new, queue, verify} (:110-217)         batch.Verifier
    SigningKey (src/signing_key.rs; test-data source)        SigningKey

All arithmetic runs in hand-written gfx950 kernels. There is NO CPU fallback: importing works
without a GPU (so the ABI can be inspected), but any verification call raises if the HIP
library or a GPU is missing.
"""
import ctypes
import os
import secrets
import sys
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "csrc", "libedc.so")

EDC_OK = 0
EDC_INVALID_SIGNATURE = 1
EDC_MALFORMED_PUBLIC_KEY = 2

# every symbol include/edc.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = [
    "edc_device_count", "edc_create", "edc_destroy", "edc_last_error", "edc_batch_verify",
    "edc_batch_verify_z", "edc_batch_verify_device", "edc_batch_partial_device", "edc_combine_partials",
    "edc_batch_submit_device", "edc_batch_wait", "edc_verify_each", "edc_verify_each_device",
    "edc_find_invalid_device", "edc_verify_prehashed_each", "edc_challenge", "edc_decompress", "edc_sign",
    "edc_sign_device", "edc_chacha_fill_device", "edc_reserve", "edc_set_timing", "edc_last_timings", "edc_timing_name",
    "edc_synchronize", "edc_vk_validate", "edc_keycache_load", "edc_keycache_clear", "edc_keycache_size",
    "edc_keycache_add", "edc_set_multi_union", "edc_multi_union_stats", "edc_batch_submit_prehashed_indexed",
    "edc_last_msm_accum",
    "edc_set_key_grouping", "edc_set_key_split", "edc_batch_submit", "edc_batch_submit_indexed", "edc_batch_verify_fallback_device",
    "edc_set_msm_shape", "edc_set_msm_bin_entries", "edc_set_fallback_shape", "edc_create_multi", "edc_destroy_multi", "edc_multi_size",
    "edc_multi_context", "edc_multi_last_error", "edc_multi_batch_verify", "edc_multi_batch_verify_fallback",
    "edc_multi_submit", "edc_multi_submit_device", "edc_multi_wait", "edc_set_slots", "edc_debug_set_scatter_stage",
    "edc_batch_verify_prehashed", "edc_batch_verify_prehashed_device", "edc_batch_submit_prehashed",
    "edc_batch_submit_prehashed_device", "edc_batch_verify_prehashed_fallback",
    "edc_batch_verify_prehashed_fallback_device", "edc_multi_route", "edc_multi_debug_force_staged",
    "edc_batch_submit_multi_device", "edc_batch_wait_multi", "edc_combine_records_device", "edc_debug_sc_reduce_wide",
]


class Error(Exception):
    """ed25519_consensus::Error (reference src/error.rs:7-20)."""


class MalformedSecretKey(Error):
    pass


class MalformedPublicKey(Error):
    pass


class InvalidSignature(Error):
    pass


class InvalidSliceLength(Error):
    pass


class EngineError(RuntimeError):
    """HIP/runtime failure. Never interpreted as a verification verdict."""


_CODE_TO_ERR = {EDC_INVALID_SIGNATURE: InvalidSignature, EDC_MALFORMED_PUBLIC_KEY: MalformedPublicKey}

_lib = None
_lib_lock = threading.Lock()


def load_library(path=None):
    """Load csrc/libedc.so and declare argument types. Raises if it is missing."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        # an explicit path is a measurement hook for tools/ (A/B builds); the product loads LIB_PATH
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise EngineError(f"HIP extension not built: {p} (run __graft_entry__.build())")
        _share_torch_hip_runtime()
        lib = ctypes.CDLL(p)
        c_sz, c_u8p, c_u64p, c_vp = ctypes.c_size_t, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p
        lib.edc_device_count.restype = ctypes.c_int
        lib.edc_create.restype = c_vp
        lib.edc_create.argtypes = [ctypes.c_int]
        lib.edc_destroy.argtypes = [c_vp]
        lib.edc_last_error.restype = ctypes.c_char_p
        lib.edc_last_error.argtypes = [c_vp]
        lib.edc_batch_verify.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u64p, c_u8p, c_vp]
        lib.edc_batch_verify_z.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u64p, c_u8p, c_vp]
        lib.edc_batch_verify_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_u8p, ctypes.c_uint64, c_vp, c_vp]
        lib.edc_batch_partial_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_u8p, ctypes.c_uint64, c_vp,
                                                 c_vp, ctypes.POINTER(ctypes.c_int)]
        lib.edc_combine_partials.argtypes = [c_vp, c_sz, c_u8p, ctypes.c_int, c_vp]
        if hasattr(lib, "edc_combine_records_device"):      # absent from older A/B builds (--lib)
            lib.edc_combine_records_device.argtypes = [c_vp, c_vp, c_sz, c_vp, c_sz, c_vp]
        if hasattr(lib, "edc_debug_sc_reduce_wide"):
            lib.edc_debug_sc_reduce_wide.argtypes = [c_vp, c_sz, c_vp, c_vp]
        lib.edc_batch_submit_device.restype = ctypes.c_int64
        lib.edc_batch_submit_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_u8p, ctypes.c_uint64, c_vp,
                                                ctypes.c_int]
        lib.edc_batch_submit.restype = ctypes.c_int64
        lib.edc_batch_submit.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u64p, c_u8p, ctypes.c_uint64, ctypes.c_int]
        lib.edc_batch_submit_indexed.restype = ctypes.c_int64
        lib.edc_batch_submit_indexed.argtypes = [c_vp, c_sz, ctypes.POINTER(ctypes.c_uint32), c_u8p, c_u8p, c_u64p,
                                                 c_u8p, ctypes.c_uint64, ctypes.c_int]
        lib.edc_batch_wait.argtypes = [c_vp, ctypes.c_int64, c_vp, c_vp, ctypes.POINTER(ctypes.c_int)]
        if hasattr(lib, "edc_batch_verify_prehashed"):       # absent from older A/B builds (tools/)
            lib.edc_batch_verify_prehashed.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u8p, c_u8p, c_vp]
            lib.edc_batch_verify_prehashed_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_u8p, ctypes.c_uint64,
                                                              c_vp, c_vp]
            lib.edc_batch_submit_prehashed.restype = ctypes.c_int64
            lib.edc_batch_submit_prehashed.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u8p, ctypes.c_uint64,
                                                       ctypes.c_int]
            lib.edc_batch_submit_prehashed_device.restype = ctypes.c_int64
            lib.edc_batch_submit_prehashed_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_u8p, ctypes.c_uint64,
                                                              c_vp, ctypes.c_int]
            lib.edc_batch_verify_prehashed_fallback.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u8p, c_vp,
                                                                ctypes.POINTER(ctypes.c_int), c_vp]
            lib.edc_batch_verify_prehashed_fallback_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_u8p, c_vp,
                                                                       ctypes.POINTER(ctypes.c_int), c_vp]
        lib.edc_verify_each.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u64p, c_vp]
        lib.edc_verify_each_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_vp]
        lib.edc_find_invalid_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_u8p, c_sz, c_vp]
        lib.edc_batch_verify_fallback_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_u8p, c_vp,
                                                         ctypes.POINTER(ctypes.c_int), c_vp]
        lib.edc_set_msm_shape.argtypes = [c_vp, ctypes.c_int, ctypes.c_int]
        lib.edc_set_msm_bin_entries.argtypes = [c_vp, ctypes.c_int]
        if hasattr(lib, "edc_debug_set_scatter_stage"):      # absent from older A/B builds (tools/)
            lib.edc_debug_set_scatter_stage.argtypes = [ctypes.c_uint32]
        lib.edc_set_fallback_shape.argtypes = [c_vp, ctypes.c_int, ctypes.c_int]
        lib.edc_create_multi.restype = c_vp
        lib.edc_create_multi.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        lib.edc_destroy_multi.argtypes = [c_vp]
        lib.edc_multi_size.argtypes = [c_vp]
        lib.edc_multi_context.restype = c_vp
        lib.edc_multi_context.argtypes = [c_vp, ctypes.c_int]
        lib.edc_multi_last_error.restype = ctypes.c_char_p
        lib.edc_multi_last_error.argtypes = [c_vp]
        lib.edc_multi_batch_verify.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u64p, c_u8p, c_vp]
        lib.edc_multi_batch_verify_fallback.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u64p, c_u8p, c_vp,
                                                        ctypes.POINTER(ctypes.c_int), c_vp]
        lib.edc_multi_submit.restype = ctypes.c_int64
        lib.edc_multi_submit.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u64p, c_u8p, ctypes.c_int]
        lib.edc_multi_submit_device.restype = ctypes.c_int64
        lib.edc_multi_submit_device.argtypes = [c_vp, ctypes.POINTER(c_sz), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                                                ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_u8p, ctypes.c_int]
        lib.edc_multi_wait.argtypes = [c_vp, ctypes.c_int64, c_vp]
        if hasattr(lib, "edc_batch_submit_multi_device"):
            lib.edc_batch_submit_multi_device.restype = ctypes.c_int64
            lib.edc_batch_submit_multi_device.argtypes = [c_vp, c_sz, c_sz, c_vp, c_vp, c_vp, c_vp, c_vp, c_u8p,
                                                          ctypes.c_uint64, ctypes.c_int]
            lib.edc_batch_wait_multi.argtypes = [c_vp, ctypes.c_int64, c_sz, ctypes.POINTER(ctypes.c_int), c_vp, c_vp,
                                                 ctypes.POINTER(ctypes.c_int)]
        if hasattr(lib, "edc_multi_route"):
            lib.edc_multi_route.argtypes = [c_vp, ctypes.c_int]
            lib.edc_multi_debug_force_staged.argtypes = [c_vp, ctypes.c_int]
        lib.edc_set_slots.argtypes = [c_vp, ctypes.c_int]
        lib.edc_verify_prehashed_each.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_vp]
        lib.edc_challenge.argtypes = [c_vp, c_sz, c_u8p, c_u8p, c_u8p, c_u64p, c_vp]
        lib.edc_decompress.argtypes = [c_vp, c_sz, c_u8p, c_vp, c_vp]
        lib.edc_sign.argtypes = [c_vp, c_sz, c_u8p, c_sz, c_vp, c_u8p, c_u64p, c_vp, c_vp]
        lib.edc_sign_device.argtypes = [c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]
        lib.edc_chacha_fill_device.argtypes = [c_vp, c_u8p, ctypes.c_uint64, ctypes.c_uint64, c_vp]
        lib.edc_reserve.argtypes = [c_vp, c_sz]
        lib.edc_set_timing.argtypes = [c_vp, ctypes.c_int]
        lib.edc_last_timings.restype = ctypes.c_int
        lib.edc_last_timings.argtypes = [c_vp, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        lib.edc_timing_name.restype = ctypes.c_char_p
        lib.edc_timing_name.argtypes = [ctypes.c_int]
        lib.edc_synchronize.argtypes = [c_vp]
        lib.edc_vk_validate.argtypes = [c_vp, c_sz, c_u8p, c_vp]
        lib.edc_keycache_load.restype = ctypes.c_int64
        lib.edc_keycache_load.argtypes = [c_vp, c_sz, c_u8p, c_vp]
        if hasattr(lib, "edc_keycache_add"):                 # absent from older A/B builds (tools/)
            lib.edc_set_multi_union.restype = ctypes.c_int
            lib.edc_set_multi_union.argtypes = [c_vp, ctypes.c_int]
            lib.edc_multi_union_stats.restype = ctypes.c_int
            lib.edc_multi_union_stats.argtypes = [c_vp, ctypes.POINTER(ctypes.c_uint64),
                                                  ctypes.POINTER(ctypes.c_uint64)]
            lib.edc_keycache_add.restype = ctypes.c_int64
            lib.edc_keycache_add.argtypes = [c_vp, c_sz, c_u8p, c_vp]
            lib.edc_last_msm_accum.restype = ctypes.c_int
            lib.edc_last_msm_accum.argtypes = [c_vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint64)]
            lib.edc_batch_submit_prehashed_indexed.restype = ctypes.c_int64
            lib.edc_batch_submit_prehashed_indexed.argtypes = [c_vp, c_sz, ctypes.POINTER(ctypes.c_uint32), c_u8p,
                                                               c_u8p, c_u8p, ctypes.c_uint64, ctypes.c_int]
        lib.edc_keycache_clear.argtypes = [c_vp]
        lib.edc_keycache_size.restype = c_sz
        lib.edc_keycache_size.argtypes = [c_vp]
        lib.edc_set_key_grouping.argtypes = [c_vp, ctypes.c_int]
        lib.edc_set_key_split.argtypes = [c_vp, ctypes.c_int]
        if path is None:
            _lib = lib
        return lib


def _share_torch_hip_runtime():
    """PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7). If torch is in this
    process, pre-load exactly that file so libedc.so's DT_NEEDED libamdhip64.so.7 binds to the
    same HIP runtime instead of /opt/rocm's copy (two runtimes in one process cannot share the
    device). Without torch, the system ROCm runtime is used."""
    torch = sys.modules.get("torch")
    if torch is None:
        return
    cand = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if os.path.exists(cand):
        ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)


def _arena(msgs):
    """Flatten messages into (arena bytes, uint64 offsets[n+1])."""
    offs = (ctypes.c_uint64 * (len(msgs) + 1))()
    total = 0
    for i, m in enumerate(msgs):
        offs[i] = total
        total += len(m)
    offs[len(msgs)] = total
    return b"".join(bytes(m) for m in msgs) or b"\0", offs


class Engine:
    """One C-ABI context = one GPU = one HIP stream (include/edc.h)."""

    def __init__(self, device=None, lib_path=None):
        self.lib = load_library(lib_path)
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        cnt = self.lib.edc_device_count()
        if cnt <= 0:
            raise EngineError("no HIP device visible; the MI355X path has no CPU fallback")
        self.device = device
        self.ctx = self.lib.edc_create(device)
        if not self.ctx:
            raise EngineError(f"edc_create({device}) failed")
        self._lock = threading.Lock()
        self._kc_keys = set()          # host mirror of the key cache's key bytes (keycache_missing)
        self._host_inflight = {}        # ticket -> host buffers borrowed by edc_batch_submit

    def close(self):
        if self.ctx:
            self.lib.edc_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc < 0:
            raise EngineError(f"edc error {rc}: {self.lib.edc_last_error(self.ctx).decode()}")
        return rc

    # ---- bulk entry points (bytes in, verdicts out) ----
    def batch_verify(self, vks, sigs, msgs, z_seed=None, z=None, want_check8=False):
        n = len(vks)
        arena, offs = _arena(msgs)
        check8 = ctypes.create_string_buffer(32) if want_check8 else None
        with self._lock:
            if z is not None:
                rc = self.lib.edc_batch_verify_z(self.ctx, n, b"".join(vks) or b"\0", b"".join(sigs) or b"\0", arena,
                                                 offs, bytes(z) or b"\0", check8)
            else:
                rc = self.lib.edc_batch_verify(self.ctx, n, b"".join(vks) or b"\0", b"".join(sigs) or b"\0", arena,
                                               offs, bytes(z_seed), check8)
        self._check(rc)
        return rc, (check8.raw if check8 is not None else None)

    def batch_verify_prehashed(self, vks, sigs, ks, z_seed=None, z=None, want_check8=False):
        """Batch of prehashed items {vk_bytes, sig, k} (edc_batch_verify_prehashed): the reference's
        Verifier::verify over Items whose k was computed at Item::from (src/batch.rs:76-94)."""
        n = len(vks)
        check8 = ctypes.create_string_buffer(32) if want_check8 else None
        with self._lock:
            rc = self.lib.edc_batch_verify_prehashed(
                self.ctx, n, b"".join(vks) or b"\0", b"".join(sigs) or b"\0", b"".join(ks) or b"\0",
                bytes(z_seed) if z is None else None, (bytes(z) or b"\0") if z is not None else None, check8)
        self._check(rc)
        return rc, (check8.raw if check8 is not None else None)

    def batch_submit_prehashed(self, vks, sigs, ks, z_seed, z_base=0, want_check8=False):
        """Asynchronous prehashed batch from host buffers (edc_batch_submit_prehashed)."""
        n = len(vks)
        bufs = (b"".join(vks) or b"\0", b"".join(sigs) or b"\0", b"".join(ks) or b"\0", bytes(z_seed))
        with self._lock:
            t = self.lib.edc_batch_submit_prehashed(self.ctx, n, bufs[0], bufs[1], bufs[2], bufs[3], z_base,
                                                    1 if want_check8 else 0)
            if t < 0:
                self._check(t)
            self._host_inflight[t] = bufs
        return t

    def batch_submit_prehashed_indexed(self, key_idx, sigs, ks, z_seed, z_base=0, want_check8=False):
        """edc_batch_submit_prehashed with keys given as positions in the last keycache_load list
        (100 bytes per item over PCIe)."""
        n = len(sigs)
        idx = (ctypes.c_uint32 * max(n, 1))(*key_idx)
        bufs = (idx, b"".join(sigs) or b"\0", b"".join(ks) or b"\0", bytes(z_seed))
        with self._lock:
            t = self.lib.edc_batch_submit_prehashed_indexed(self.ctx, n, bufs[0], bufs[1], bufs[2], bufs[3], z_base,
                                                            1 if want_check8 else 0)
            if t < 0:
                self._check(t)
            self._host_inflight[t] = bufs
        return t

    def batch_verify_prehashed_fallback(self, vks, sigs, ks, z_seed):
        """(code, per-item Item::verify_single codes, number invalid, check8) of a prehashed batch."""
        n = len(vks)
        check8 = ctypes.create_string_buffer(32)
        v = ctypes.create_string_buffer(max(n, 1))
        cnt = ctypes.c_int(0)
        with self._lock:
            rc = self.lib.edc_batch_verify_prehashed_fallback(self.ctx, n, b"".join(vks) or b"\0",
                                                              b"".join(sigs) or b"\0", b"".join(ks) or b"\0",
                                                              bytes(z_seed), v, ctypes.byref(cnt), check8)
        self._check(rc)
        return rc, list(v.raw[:n]), cnt.value, check8.raw

    def batch_submit(self, vks, sigs, msgs, z_seed, z_base=0, want_check8=False):
        """Asynchronous host-buffer batch (edc_batch_submit): returns a ticket; the staged host
        buffers are kept alive here until batch_wait(ticket)."""
        n = len(vks)
        arena, offs = _arena(msgs)
        bufs = (b"".join(vks) or b"\0", b"".join(sigs) or b"\0", arena, offs, bytes(z_seed))
        with self._lock:
            t = self.lib.edc_batch_submit(self.ctx, n, bufs[0], bufs[1], bufs[2], bufs[3], bufs[4], z_base,
                                          1 if want_check8 else 0)
            if t < 0:
                self._check(t)
            self._host_inflight[t] = bufs
        return t

    def batch_submit_indexed(self, key_idx, sigs, msgs, z_seed, z_base=0, want_check8=False):
        """edc_batch_submit with keys given as positions in the last keycache_load list."""
        n = len(sigs)
        arena, offs = _arena(msgs)
        idx = (ctypes.c_uint32 * max(n, 1))(*key_idx)
        bufs = (idx, b"".join(sigs) or b"\0", arena, offs, bytes(z_seed))
        with self._lock:
            t = self.lib.edc_batch_submit_indexed(self.ctx, n, bufs[0], bufs[1], bufs[2], bufs[3], bufs[4], z_base,
                                                  1 if want_check8 else 0)
            if t < 0:
                self._check(t)
            self._host_inflight[t] = bufs
        return t

    def batch_submit_multi_device(self, nb, n_per, d_vk, d_sig, d_msg, d_off, z_seed, z_base=0, d_k=None,
                                  want_check8=False):
        """nb consecutive batches of n_per items in one launch sequence (edc_batch_submit_multi_device);
        device pointers as ints. Returns a ticket for batch_wait_multi."""
        with self._lock:
            t = self.lib.edc_batch_submit_multi_device(self.ctx, nb, n_per, d_vk, d_sig, d_msg, d_off, d_k,
                                                       bytes(z_seed), z_base, 1 if want_check8 else 0)
        self._check(t)
        return t

    def batch_wait_multi(self, ticket, nb, want_partials=False):
        """(code, [verdict per batch], [check8 per batch], [partial per batch] or None, [bad per batch]).
        Asking for the partials makes a union-first launch run batch by batch (edc_set_multi_union)."""
        v = (ctypes.c_int * nb)()
        bad = (ctypes.c_int * nb)()
        c8 = ctypes.create_string_buffer(32 * nb)
        parts = ctypes.create_string_buffer(128 * nb) if want_partials else None
        with self._lock:
            rc = self.lib.edc_batch_wait_multi(self.ctx, ticket, nb, v, c8, parts, bad)
        self._check(rc)
        return (rc, list(v), [c8.raw[32 * g:32 * g + 32] for g in range(nb)],
                [parts.raw[128 * g:128 * g + 128] for g in range(nb)] if want_partials else None, list(bad))

    def set_multi_union(self, on):
        """Multi-batch launches verify the union of their batches first (default on)."""
        self._check(self.lib.edc_set_multi_union(self.ctx, 1 if on else 0))

    def multi_union_stats(self):
        """(union-first launches that passed, launches rerun batch by batch) on this context."""
        a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._check(self.lib.edc_multi_union_stats(self.ctx, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def batch_wait(self, ticket, want_check8=False):
        """Verdict of a submitted batch: (code, check8 or None); the ticket's host buffers are released."""
        check8 = ctypes.create_string_buffer(32) if want_check8 else None
        with self._lock:
            rc = self.lib.edc_batch_wait(self.ctx, ticket, check8, None, None)
            self._host_inflight.pop(ticket, None)
        self._check(rc)
        return rc, (check8.raw if check8 is not None else None)

    def verify_each(self, vks, sigs, msgs):
        n = len(vks)
        arena, offs = _arena(msgs)
        out = ctypes.create_string_buffer(max(n, 1))
        with self._lock:
            self._check(self.lib.edc_verify_each(self.ctx, n, b"".join(vks) or b"\0", b"".join(sigs) or b"\0",
                                                 arena, offs, out))
        return list(out.raw[:n])

    def verify_prehashed_each(self, vks, sigs, ks):
        n = len(vks)
        out = ctypes.create_string_buffer(max(n, 1))
        with self._lock:
            self._check(self.lib.edc_verify_prehashed_each(self.ctx, n, b"".join(vks) or b"\0",
                                                           b"".join(sigs) or b"\0", b"".join(ks) or b"\0", out))
        return list(out.raw[:n])

    def challenge(self, vks, sigs, msgs):
        n = len(vks)
        arena, offs = _arena(msgs)
        out = ctypes.create_string_buffer(max(32 * n, 1))
        with self._lock:
            self._check(self.lib.edc_challenge(self.ctx, n, b"".join(vks) or b"\0", b"".join(sigs) or b"\0",
                                               arena, offs, out))
        return [out.raw[32 * i:32 * i + 32] for i in range(n)]

    def decompress(self, encs):
        n = len(encs)
        xy = ctypes.create_string_buffer(max(64 * n, 1))
        ok = ctypes.create_string_buffer(max(n, 1))
        with self._lock:
            self._check(self.lib.edc_decompress(self.ctx, n, b"".join(encs) or b"\0", xy, ok))
        return [(bool(ok.raw[i]), xy.raw[64 * i:64 * i + 32], xy.raw[64 * i + 32:64 * i + 64]) for i in range(n)]

    def vk_validate(self, encs):
        """VerificationKey::try_from for many keys (src/verification_key.rs:160-175): codes 0 / 2."""
        n = len(encs)
        out = ctypes.create_string_buffer(max(n, 1))
        with self._lock:
            self._check(self.lib.edc_vk_validate(self.ctx, n, b"".join(encs) or b"\0", out))
        return list(out.raw[:n])

    def keycache_load(self, encs):
        """Register validator keys (decoded once per context, comb tables kept on the GPU).
        Returns (number of distinct keys cached, per-key ok list)."""
        n = len(encs)
        ok = ctypes.create_string_buffer(max(n, 1))
        with self._lock:
            u = self._check(self.lib.edc_keycache_load(self.ctx, n, b"".join(encs) or b"\0", ok))
            self._kc_keys = set(bytes(e) for e in encs)      # load caches every distinct key
        return u, [bool(b) for b in ok.raw[:n]]

    def keycache_add(self, encs):
        """Add keys to the context's cache without replacing it (a VerificationKey's decoded point,
        kept for every later verify: src/verification_key.rs:106-114). Returns (number of distinct
        keys now cached, per-key ok list)."""
        n = len(encs)
        ok = ctypes.create_string_buffer(max(n, 1))
        with self._lock:
            u = self._check(self.lib.edc_keycache_add(self.ctx, n, b"".join(encs) or b"\0", ok))
            oks = [bool(b) for b in ok.raw[:n]]
            self._kc_keys.update(bytes(e) for e, o in zip(encs, oks) if o)   # add keeps decodable keys only
        return u, oks

    def keycache_missing(self, encs):
        """The distinct keys of encs that the context's key cache does not hold yet (host-side
        mirror of the cache's key set, no device call)."""
        return set(bytes(e) for e in encs) - self._kc_keys

    def set_key_grouping(self, mode):
        """0 auto (default), 1 always group keys, 2 never (one A term per signature), 3 test mode:
        grouping abandoned on the device (the adversarial-key overflow path)."""
        self._check(self.lib.edc_set_key_grouping(self.ctx, int(mode)))

    def set_key_split(self, mode):
        """0 auto (default): split B / key coefficients at bit 128 onto the key cache's [2^128]A
        while the cache covers the batches' keys; 1 never."""
        self._check(self.lib.edc_set_key_split(self.ctx, int(mode)))

    def set_msm_shape(self, bits=0, parts=0):
        """Pippenger window width (8..16) and parts (1..64); 0 = chosen from the batch size."""
        self._check(self.lib.edc_set_msm_shape(self.ctx, int(bits), int(parts)))

    def set_msm_bin_entries(self, entries=0):
        """Target MSM entries per bin (>= 256); 0 = chosen from the batch size."""
        self._check(self.lib.edc_set_msm_bin_entries(self.ctx, int(entries)))

    def keycache_clear(self):
        with self._lock:
            self._check(self.lib.edc_keycache_clear(self.ctx))
            self._kc_keys = set()

    def keycache_size(self):
        return int(self.lib.edc_keycache_size(self.ctx))

    def sign(self, seeds, msgs, seed_index=None):
        n = len(msgs)
        arena, offs = _arena(msgs)
        vk = ctypes.create_string_buffer(max(32 * n, 1))
        sig = ctypes.create_string_buffer(max(64 * n, 1))
        idx = None
        if seed_index is not None:
            idx = (ctypes.c_uint32 * n)(*seed_index)
        with self._lock:
            self._check(self.lib.edc_sign(self.ctx, n, b"".join(seeds), len(seeds), idx, arena, offs, vk, sig))
        return [vk.raw[32 * i:32 * i + 32] for i in range(n)], [sig.raw[64 * i:64 * i + 64] for i in range(n)]

    def combine_records_device(self, stream, g, d_records, stride, d_out):
        """Enqueue the combine of g gathered 129-byte exchange records (device memory) on `stream`
        (a raw HIP stream handle); the 256-byte result block lands in d_out (device)."""
        with self._lock:
            self._check(self.lib.edc_combine_records_device(self.ctx, ctypes.c_void_p(stream), g,
                                                            ctypes.c_void_p(d_records), stride, ctypes.c_void_p(d_out)))

    def combine_partials(self, partials, bad_any, want_check8=True):
        check8 = ctypes.create_string_buffer(32) if want_check8 else None
        with self._lock:
            rc = self._check(self.lib.edc_combine_partials(self.ctx, len(partials), b"".join(partials) or b"\0",
                                                           1 if bad_any else 0, check8))
        return rc, (check8.raw if check8 is not None else None)


class MultiEngine:
    """Several GPUs in one process (include/edc.h edc_create_multi): each batch is split into
    contiguous shards, one per listed device; partial points are combined on the first device.
    A device may be listed several times (several contexts on one GPU)."""

    def __init__(self, devices):
        self.lib = load_library()
        if self.lib.edc_device_count() <= 0:
            raise EngineError("no HIP device visible; the MI355X path has no CPU fallback")
        arr = (ctypes.c_int * len(devices))(*devices)
        self.m = self.lib.edc_create_multi(arr, len(devices))
        if not self.m:
            raise EngineError(f"edc_create_multi({list(devices)}) failed")
        self.devices = list(devices)
        self._lock = threading.Lock()
        self._inflight = {}

    def close(self):
        if self.m:
            self.lib.edc_destroy_multi(self.m)
            self.m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc < 0:
            raise EngineError(f"edc error {rc}: {self.lib.edc_multi_last_error(self.m).decode()}")
        return rc

    def batch_verify(self, vks, sigs, msgs, z_seed, want_check8=False):
        arena, offs = _arena(msgs)
        check8 = ctypes.create_string_buffer(32) if want_check8 else None
        with self._lock:
            rc = self.lib.edc_multi_batch_verify(self.m, len(vks), b"".join(vks) or b"\0", b"".join(sigs) or b"\0",
                                                 arena, offs, bytes(z_seed), check8)
        self._check(rc)
        return rc, (check8.raw if check8 is not None else None)

    def batch_submit(self, vks, sigs, msgs, z_seed, want_check8=False):
        """Pipelined multi-device batch (edc_multi_submit): returns a ticket; the host buffers are
        kept alive here until batch_wait(ticket)."""
        arena, offs = _arena(msgs)
        bufs = (b"".join(vks) or b"\0", b"".join(sigs) or b"\0", arena, offs, bytes(z_seed))
        with self._lock:
            t = self.lib.edc_multi_submit(self.m, len(vks), bufs[0], bufs[1], bufs[2], bufs[3], bufs[4],
                                          1 if want_check8 else 0)
            self._check(t)
            self._inflight[t] = bufs
        return t

    def batch_submit_device(self, shards, z_seed, want_check8=False):
        """edc_multi_submit_device: shards[g] = (n, d_vk, d_sig, d_msg, d_msg_off) as device pointers
        (ints) on device g; returns a ticket."""
        G = len(shards)
        n = (ctypes.c_size_t * G)(*[s[0] for s in shards])
        ptr = lambda k: (ctypes.c_void_p * G)(*[s[k] for s in shards])
        with self._lock:
            t = self.lib.edc_multi_submit_device(self.m, n, ptr(1), ptr(2), ptr(3), ptr(4), bytes(z_seed),
                                                 1 if want_check8 else 0)
            self._check(t)
        return t

    def batch_wait(self, ticket, want_check8=False):
        check8 = ctypes.create_string_buffer(32) if want_check8 else None
        with self._lock:
            rc = self.lib.edc_multi_wait(self.m, ticket, check8)
            self._inflight.pop(ticket, None)
        self._check(rc)
        return rc, (check8.raw if check8 is not None else None)

    def route(self, i):
        """How shard i's result block reaches the first device: 0 local, 1 peer (xGMI), 2 host-staged."""
        return self._check(self.lib.edc_multi_route(self.m, int(i)))

    def force_staged(self, on=True):
        """Test knob: route every shard's result block through pinned host memory (the no-peer path)."""
        with self._lock:
            self._check(self.lib.edc_multi_debug_force_staged(self.m, 1 if on else 0))

    def batch_verify_fallback(self, vks, sigs, msgs, z_seed):
        """(code, per-item verify_single codes, number invalid, check8)."""
        n = len(vks)
        arena, offs = _arena(msgs)
        check8 = ctypes.create_string_buffer(32)
        v = ctypes.create_string_buffer(max(n, 1))
        cnt = ctypes.c_int(0)
        with self._lock:
            rc = self.lib.edc_multi_batch_verify_fallback(self.m, n, b"".join(vks) or b"\0", b"".join(sigs) or b"\0",
                                                          arena, offs, bytes(z_seed), v, ctypes.byref(cnt), check8)
        self._check(rc)
        return rc, list(v.raw[:n]), cnt.value, check8.raw


_default_engine = None
_default_lock = threading.Lock()


def default_engine():
    global _default_engine
    with _default_lock:
        if _default_engine is None:
            _default_engine = Engine()
        return _default_engine


# ------------------------------------------------------------------ reference types
def _as_bytes(x, n):
    b = bytes(x)
    if len(b) != n:
        raise InvalidSliceLength()
    return b


_L = (1 << 252) + 27742317777372353535851937790883648493    # the group order l


def _canonical_k(k):
    """A prehashed challenge as the reference's Item holds it: Scalar::from_hash output, < l
    (src/batch.rs:82-94). Anything else is an argument error, never a verdict."""
    b = _as_bytes(k, 32)
    if int.from_bytes(b, "little") >= _L:
        raise ValueError("prehashed k is not a canonical scalar (must be < l)")
    return b


class Signature:
    """reference src/signature.rs:8-62: 64 bytes R || s, not validated at parse time."""

    __slots__ = ("R_bytes", "s_bytes")

    def __init__(self, data):
        b = _as_bytes(data, 64)
        self.R_bytes, self.s_bytes = b[:32], b[32:]

    def to_bytes(self):
        return self.R_bytes + self.s_bytes

    def __bytes__(self):
        return self.to_bytes()

    def __eq__(self, other):
        return isinstance(other, Signature) and self.to_bytes() == other.to_bytes()

    def __hash__(self):
        return hash(self.to_bytes())

    def __repr__(self):
        return f"Signature(R_bytes={self.R_bytes.hex()}, s_bytes={self.s_bytes.hex()})"


class VerificationKeyBytes:
    """reference src/verification_key.rs:32-87: raw 32 bytes; Hash/Eq on the bytes."""

    __slots__ = ("_b",)

    def __init__(self, data):
        if isinstance(data, (VerificationKeyBytes, VerificationKey)):
            data = data.to_bytes()
        self._b = _as_bytes(data, 32)

    def to_bytes(self):
        return self._b

    def as_bytes(self):
        return self._b

    def __bytes__(self):
        return self._b

    def __eq__(self, other):
        return isinstance(other, VerificationKeyBytes) and self._b == other._b

    def __lt__(self, other):
        return self._b < other._b

    def __hash__(self):
        return hash(self._b)

    def __repr__(self):
        return f"VerificationKeyBytes({self._b.hex()})"


class VerificationKey:
    """reference src/verification_key.rs:106-258. try_from decodes A on the GPU once and keeps it:
    the reference stores minus_A in the object (:111-114, :160-175); here the decoded point and its
    fixed-base table go into the engine's key cache (edc_keycache_add), where every later verify,
    batch or fallback of that engine finds them (`cached`). keep_decoded=False only validates;
    True always adds; None (the default) adds while the engine's cache holds fewer than
    AUTO_CACHE_KEYS keys, so keys parsed from untrusted input cannot grow device memory without
    bound. Keys that do not decode are never added (edc_keycache_add)."""

    AUTO_CACHE_KEYS = 1024          # 64 MB of comb tables
    # Cost of the default (keep_decoded=None): a call that adds new keys rebuilds the cache's hash
    # table, decodes the new keys' comb tables and synchronises every slot of the engine (it may
    # not run while batches are in flight; it then only validates). Ingesting keys that are
    # already cached adds nothing.

    __slots__ = ("A_bytes", "_engine", "cached")

    def __init__(self, vkb, engine, cached=False):
        self.A_bytes = vkb
        self._engine = engine
        self.cached = cached

    @classmethod
    def try_from(cls, data, engine=None, keep_decoded=None):
        r = cls.try_from_many([data], engine, keep_decoded)[0]
        if isinstance(r, MalformedPublicKey):
            raise r
        return r

    @classmethod
    def try_from_many(cls, keys, engine=None, keep_decoded=None):
        """Batched key ingestion: [VerificationKey or MalformedPublicKey()] per input, one launch
        (keep_decoded: also add the keys to the engine's key cache; None: while it stays under
        AUTO_CACHE_KEYS)."""
        vkbs = [k if isinstance(k, VerificationKeyBytes) else VerificationKeyBytes(k) for k in keys]
        eng = engine or default_engine()
        encs = [v.to_bytes() for v in vkbs]
        if keep_decoded is None:      # keys already cached cost nothing: only new ones count
            keep_decoded = eng.keycache_size() + len(eng.keycache_missing(encs)) <= cls.AUTO_CACHE_KEYS
        cached = False
        if keep_decoded and encs:
            try:
                _, oks = eng.keycache_add(encs)
                codes = [EDC_OK if o else EDC_MALFORMED_PUBLIC_KEY for o in oks]
                cached = True
            except EngineError:        # cache full, or batches in flight: validate only
                codes = eng.vk_validate(encs)
        else:
            codes = eng.vk_validate(encs)
        return [cls(v, eng, cached) if c == EDC_OK else MalformedPublicKey() for v, c in zip(vkbs, codes)]


    def to_bytes(self):
        return self.A_bytes.to_bytes()

    def verify(self, signature, msg):
        """VerificationKey::verify (src/verification_key.rs:225-233)."""
        sig = signature if isinstance(signature, Signature) else Signature(signature)
        code = self._engine.verify_each([self.to_bytes()], [sig.to_bytes()], [bytes(msg)])[0]
        if code != EDC_OK:
            raise _CODE_TO_ERR[code]()


class SigningKey:
    """reference src/signing_key.rs (test-data source): seed -> key; sign on the GPU."""

    __slots__ = ("seed", "_engine", "_vk")

    def __init__(self, seed=None, engine=None):
        self.seed = _as_bytes(seed, 32) if seed is not None else secrets.token_bytes(32)
        self._engine = engine or default_engine()
        self._vk = None

    @classmethod
    def new(cls, rng=None, engine=None):
        seed = rng.token_bytes(32) if hasattr(rng, "token_bytes") else secrets.token_bytes(32)
        return cls(seed, engine)

    def verification_key_bytes(self):
        if self._vk is None:
            vks, _ = self._engine.sign([self.seed], [b""])
            self._vk = VerificationKeyBytes(vks[0])
        return self._vk

    def sign(self, msg):
        vks, sigs = self._engine.sign([self.seed], [bytes(msg)])
        self._vk = VerificationKeyBytes(vks[0])
        return Signature(sigs[0])


class batch:  # namespace mirroring `ed25519_consensus::batch`
    class Item:
        """reference src/batch.rs:75-107. k = H(R||A||M) is computed at construction on the GPU
        (Item::from), so verify_single is decoupled from the message."""

        __slots__ = ("vk_bytes", "sig", "k", "_msg")

        def __init__(self, vk_bytes, sig, msg=None, k=None):
            self.vk_bytes = vk_bytes if isinstance(vk_bytes, VerificationKeyBytes) else VerificationKeyBytes(vk_bytes)
            self.sig = sig if isinstance(sig, Signature) else Signature(sig)
            if msg is None and k is None:
                raise ValueError("an Item needs its message or its challenge k")
            self._msg = bytes(msg) if msg is not None else None
            self.k = _canonical_k(k) if k is not None else None

        @classmethod
        def from_tuple(cls, tup):
            return cls(*tup)

        @classmethod
        def prehashed(cls, vk_bytes, sig, k):
            """The reference's Item as it is stored, {vk_bytes, sig, k} (src/batch.rs:76-80): k was
            computed at Item::from (e.g. by another process), the message is not needed again."""
            return cls(vk_bytes, sig, None, k)

        @staticmethod
        def hash_many(items, engine=None):
            """Item::from's k = H(R||A||M) mod l (src/batch.rs:82-94) for every item still without
            one, in ONE GPU launch."""
            eng = engine or default_engine()
            need = [it for it in items if it.k is None]
            if need:
                ks = eng.challenge([it.vk_bytes.to_bytes() for it in need], [it.sig.to_bytes() for it in need],
                                   [it._msg for it in need])
                for it, k in zip(need, ks):
                    it.k = k
            return items

        def verify_single(self, engine=None):
            eng = engine or default_engine()
            if self.k is None:
                self.k = eng.challenge([self.vk_bytes.to_bytes()], [self.sig.to_bytes()], [self._msg])[0]
            code = eng.verify_prehashed_each([self.vk_bytes.to_bytes()], [self.sig.to_bytes()], [self.k])[0]
            if code != EDC_OK:
                raise _CODE_TO_ERR[code]()

        @staticmethod
        def verify_single_many(items, engine=None):
            """Fallback for many items in ONE GPU launch; returns per-item verdict codes."""
            eng = engine or default_engine()
            batch.Item.hash_many(items, eng)
            return eng.verify_prehashed_each([it.vk_bytes.to_bytes() for it in items],
                                             [it.sig.to_bytes() for it in items], [it.k for it in items])

    class Verifier:
        """reference src/batch.rs:110-217. Items are kept in queue order; grouping by key
        bytes, hashing and the coalesced MSM run on the GPU inside verify()."""

        def __init__(self, engine=None):
            self._engine = engine
            self._vks, self._sigs, self._msgs, self._ks = [], [], [], []

        @classmethod
        def new(cls, engine=None):
            return cls(engine)

        @property
        def batch_size(self):
            return len(self._vks)

        def queue(self, item, sig=None, msg=None):
            if sig is not None:
                item = batch.Item(item, sig, msg)
            elif isinstance(item, tuple):
                item = batch.Item(*item)
            self._vks.append(item.vk_bytes.to_bytes())
            self._sigs.append(item.sig.to_bytes())
            self._msgs.append(item._msg)
            self._ks.append(item.k)

        def verify_detailed(self, rng=None):
            """Returns (code, check8): check8 = compressed [8]*check (None when rejected before
            the MSM). rng: a 32-byte ChaCha20 seed, an object with fill_bytes(n)/token_bytes(n),
            or None (fresh OS randomness). Items that carry their k (prehashed, as the reference's
            Item always does) go through edc_batch_verify_prehashed; otherwise SHA-512 runs on the
            GPU inside the batch."""
            eng = self._engine or default_engine()
            n = len(self._vks)
            if isinstance(rng, (bytes, bytearray)) and len(rng) == 32:
                zkw = {"z_seed": bytes(rng)}
            elif rng is None:
                zkw = {"z_seed": secrets.token_bytes(32)}
            else:   # gen_u128 per item in queue order (src/batch.rs:64-68)
                draw = rng.fill_bytes if hasattr(rng, "fill_bytes") else rng.token_bytes
                zkw = {"z": b"".join(bytes(draw(16)) for _ in range(n))}
            if any(m is None for m in self._msgs) or (n and all(k is not None for k in self._ks)):
                if any(k is None for k in self._ks):     # mixed queue: hash the rest in one launch
                    need = [i for i, k in enumerate(self._ks) if k is None]
                    ks = eng.challenge([self._vks[i] for i in need], [self._sigs[i] for i in need],
                                       [self._msgs[i] for i in need])
                    for i, k in zip(need, ks):
                        self._ks[i] = k
                return eng.batch_verify_prehashed(self._vks, self._sigs, self._ks, want_check8=True, **zkw)
            return eng.batch_verify(self._vks, self._sigs, self._msgs, want_check8=True, **zkw)

        def verify(self, rng=None):
            """Verifier::verify: returns None on success, raises InvalidSignature otherwise."""
            code, _ = self.verify_detailed(rng)
            if code != EDC_OK:
                raise InvalidSignature()
