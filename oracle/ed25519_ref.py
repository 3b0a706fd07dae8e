"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- pure-Python big-integer restatement of the
ed25519-consensus 2.1.0 verification path (`/root/reference`), used to generate and check
golden vectors. Never imported by the product path; only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may use anything under oracle/.

Pinning: this restatement is checked (tests/test_oracle_golden.py) against every vector the
reference's own tests hold for this path: the three RFC 8032 vectors of tests/rfc8032.rs:55-124
(verify, pk regeneration, deterministic re-sign) and the 196-case ZIP215 small-order corpus
that tests/small_order.rs:12-77 builds (all cases must verify, single == batch, :79-104).

The arithmetic lives in third-party crates that are NOT vendored under /root/reference
(Cargo.toml:14-21, no lockfile): curve25519-dalek-ng ^4.1 (u64_backend), sha2 ^0.9,
rand_core ^0.6. Their published algorithms are restated here:
  * FieldElement::from_bytes masks bit 255 and does NOT reduce (y >= p accepted);
  * CompressedEdwardsY::decompress = sqrt_ratio_i(y^2-1, d*y^2+1), fail if non-square,
    conditional negate of x by bit 255 (so x = 0 with the sign bit set is accepted);
  * Scalar::from_hash = 512-bit LE digest mod l; Scalar::from_canonical_bytes accepts iff
    the 256-bit LE integer is < l (which implies bit 255 clear);
  * vartime_multiscalar_mul / vartime_double_scalar_mul_basepoint are exact group
    operations: any algorithm returns the same group element (compared via compress()).
"""
import hashlib
import struct

# ---- curve constants (RFC 8032 / curve25519-dalek constants) ----
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)
BY = (4 * pow(5, P - 2, P)) % P

OK = 0
INVALID_SIGNATURE = 1
MALFORMED_PUBLIC_KEY = 2
ERROR_NAMES = {OK: "Ok", INVALID_SIGNATURE: "InvalidSignature",
               MALFORMED_PUBLIC_KEY: "MalformedPublicKey"}


def _is_negative(x):
    return (x % P) & 1


def sqrt_ratio_i(u, v):
    """dalek FieldElement::sqrt_ratio_i: returns (was_nonzero_square, nonnegative root)."""
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = (u * v3 % P) * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (-u) % P
    flipped_i = check == (-u) * SQRT_M1 % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    if _is_negative(r):
        r = (-r) % P
    return (correct or flipped), r


def decompress(b):
    """CompressedEdwardsY::decompress (ZIP215): returns extended (X, Y, Z, T) or None.
    Call sites: reference src/batch.rs:183-185, :190-192; src/verification_key.rs:166-168, :242-244."""
    assert len(b) == 32
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)   # masked, NOT reduced mod p
    yy = y * y % P
    u = (yy - 1) % P
    v = (D * yy + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    if not ok:
        return None
    if b[31] >> 7:
        x = (-x) % P
    y %= P
    return (x, y, 1, x * y % P)


def compress(pt):
    X, Y, Z, _ = pt
    zi = pow(Z, P - 2, P)
    x = X * zi % P
    y = Y * zi % P
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


IDENTITY = (0, 1, 1, 0)
B_POINT = decompress(BY.to_bytes(32, "little"))


def add(p1, p2):
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    a = (Y1 - X1) * (Y2 - X2) % P
    b = (Y1 + X1) * (Y2 + X2) % P
    c = 2 * D * T1 * T2 % P
    d = 2 * Z1 * Z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def neg(pt):
    X, Y, Z, T = pt
    return ((-X) % P, Y, Z, (-T) % P)


def double(pt):
    return add(pt, pt)


def scalar_mul(k, pt):
    acc = IDENTITY
    for bit in bin(k)[2:] if k > 0 else "":
        acc = double(acc)
        if bit == "1":
            acc = add(acc, pt)
    return acc


def is_identity(pt):
    X, Y, Z, _ = pt
    return X % P == 0 and (Y - Z) % P == 0


def mul_by_cofactor(pt):
    return double(double(double(pt)))


def multiscalar_mul(scalars, points):
    """Exact sum of [c_i]P_i (windowed Pippenger, w=4, unsigned digits).
    Any MSM algorithm yields the same group element as dalek's Straus/Pippenger."""
    if not points:
        return IDENTITY
    nbits = max((s.bit_length() for s in scalars), default=0)
    w = 4
    nwin = (nbits + w - 1) // w
    acc = IDENTITY
    for win in reversed(range(nwin)):
        for _ in range(w):
            acc = double(acc)
        buckets = [None] * (1 << w)
        for s, pt in zip(scalars, points):
            dgt = (s >> (win * w)) & ((1 << w) - 1)
            if dgt:
                buckets[dgt] = pt if buckets[dgt] is None else add(buckets[dgt], pt)
        run = IDENTITY
        tot = IDENTITY
        for dgt in range((1 << w) - 1, 0, -1):
            if buckets[dgt] is not None:
                run = add(run, buckets[dgt])
            tot = add(tot, run)
        acc = add(acc, tot)
    return acc


# ---- scalars ----
def scalar_from_hash(digest):
    """Scalar::from_hash: 64-byte digest as LE integer mod l (reference src/batch.rs:86-91)."""
    return int.from_bytes(digest, "little") % L


def scalar_from_canonical_bytes(b):
    """Scalar::from_canonical_bytes: Some(s) iff s < l (reference src/batch.rs:193)."""
    s = int.from_bytes(b, "little")
    if (b[31] >> 7) or s >= L:
        return None
    return s


def challenge(R_bytes, A_bytes, msg):
    """k = H(R || A || M) mod l over the RAW byte encodings (reference src/batch.rs:86-91)."""
    return scalar_from_hash(hashlib.sha512(bytes(R_bytes) + bytes(A_bytes) + bytes(msg)).digest())


# ---- ChaCha20 (rand_chacha::ChaCha20Rng keystream, nonce/stream 0, 64-bit counter) ----
def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF


def chacha20_block(key32, counter):
    c = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    k = list(struct.unpack("<8I", key32))
    st = c + k + [counter & 0xFFFFFFFF, counter >> 32, 0, 0]
    x = st[:]

    def qr(a, b, cc, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 16)
        x[cc] = (x[cc] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[cc], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 8)
        x[cc] = (x[cc] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[cc], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return struct.pack("<16I", *[(x[i] + st[i]) & 0xFFFFFFFF for i in range(16)])


def chacha20_keystream(key32, nbytes, start_block=0):
    out = bytearray()
    blk = start_block
    while len(out) < nbytes:
        out += chacha20_block(key32, blk)
        blk += 1
    return bytes(out[:nbytes])


def z_values(seed32, n, start=0):
    """z_j = u128::from_le_bytes(keystream[16j..16j+16]) -- gen_u128 (reference src/batch.rs:64-68)
    drawn in QUEUE order j (the reference draws in HashMap order)."""
    if n == 0:
        return []
    first_blk = start // 4
    ks = chacha20_keystream(seed32, 16 * (n + start - 4 * first_blk), first_blk)
    off = 16 * (start - 4 * first_blk)
    return [int.from_bytes(ks[off + 16 * j: off + 16 * j + 16], "little") for j in range(n)]


# ---- signing (test-data source only; reference src/signing_key.rs) ----
def expand_seed(seed32):
    h = hashlib.sha512(seed32).digest()
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little"), h[32:]


def public_key(seed32):
    a, _ = expand_seed(seed32)
    return compress(scalar_mul(a, B_POINT))


def sign(seed32, msg):
    a, prefix = expand_seed(seed32)
    A = compress(scalar_mul(a, B_POINT))
    r = scalar_from_hash(hashlib.sha512(prefix + bytes(msg)).digest())
    R = compress(scalar_mul(r, B_POINT))
    k = challenge(R, A, msg)
    s = (r + k * a) % L
    return R + s.to_bytes(32, "little")


# ---- verification (the oracle proper) ----
def verify_prehashed(A_bytes, sig, k):
    """VerificationKey::try_from + verify_prehashed (reference src/verification_key.rs:160-175,
    :237-258; Item::verify_single src/batch.rs:104-107). Returns an error code."""
    A = decompress(A_bytes)
    if A is None:
        return MALFORMED_PUBLIC_KEY
    s = scalar_from_canonical_bytes(sig[32:64])       # s checked BEFORE R
    if s is None:
        return INVALID_SIGNATURE
    R = decompress(sig[0:32])
    if R is None:
        return INVALID_SIGNATURE
    # R' = [k](-A) + [s]B ; check [8](R - R') == 0
    Rp = add(scalar_mul(k, neg(A)), scalar_mul(s, B_POINT))
    return OK if is_identity(mul_by_cofactor(add(R, neg(Rp)))) else INVALID_SIGNATURE


def verify(A_bytes, sig, msg):
    """VerificationKey::verify (reference src/verification_key.rs:225-233)."""
    return verify_prehashed(A_bytes, sig, challenge(sig[0:32], A_bytes, msg))


def batch_verify(items, z):
    """batch::Verifier::queue + verify (reference src/batch.rs:127-137, :149-217).

    items: list of (vk_bytes32, sig_bytes64, msg_bytes); z: list of 128-bit ints in queue order.
    Returns (code, check8) where check8 is the compressed [8]*check point (bytes) or None when
    the batch is rejected before the MSM (undecodable A/R or non-canonical s)."""
    assert len(z) == len(items)
    groups = {}                       # HashMap<VerificationKeyBytes, Vec<(k, sig, z)>>, keyed by RAW bytes
    for (vk, sig, msg), zi in zip(items, z):
        k = challenge(sig[0:32], vk, msg)
        groups.setdefault(bytes(vk), []).append((k, bytes(sig), zi))
    B_coeff = 0
    scalars, points = [], []
    for vk, sigs in groups.items():
        A = decompress(vk)
        if A is None:
            return INVALID_SIGNATURE, None
        A_coeff = 0
        for k, sig, zi in sigs:
            R = decompress(sig[0:32])
            if R is None:
                return INVALID_SIGNATURE, None
            s = scalar_from_canonical_bytes(sig[32:64])
            if s is None:
                return INVALID_SIGNATURE, None
            B_coeff = (B_coeff - zi * s) % L
            scalars.append(zi)
            points.append(R)
            A_coeff = (A_coeff + zi * k) % L
        scalars.append(A_coeff)
        points.append(A)
    scalars.append(B_coeff)
    points.append(B_POINT)
    check = multiscalar_mul(scalars, points)
    c8 = mul_by_cofactor(check)
    return (OK if is_identity(c8) else INVALID_SIGNATURE), compress(c8)


def batch_verify_seeded(items, seed32):
    return batch_verify(items, z_values(seed32, len(items)))


def identity_bytes():
    return compress(IDENTITY)


# ---- ZIP215 corpus (reference tests/util/mod.rs:66-155, tests/small_order.rs:12-77) ----
def eight_torsion_encodings():
    """Compressed [i]T for i = 0..7, T a generator of the 8-torsion (dalek EIGHT_TORSION order)."""
    # T: the order-8 point with positive-sign canonical encoding c7176a70...037a (dalek EIGHT_TORSION[1])
    t = decompress(bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"))
    out, acc = [], IDENTITY
    for _ in range(8):
        out.append(compress(acc))
        acc = add(acc, t)
    return out


def non_canonical_field_encodings():
    out = []
    for i in range(19):
        b = bytearray([0xFF] * 32)
        b[0] = 237 + i
        b[31] = 0x7F
        out.append(bytes(b))
    return out


def non_canonical_point_encodings():
    enc = [bytes([1] + [0] * 30 + [0x80]), bytes([0xEC] + [0xFF] * 31)]
    for x in non_canonical_field_encodings():
        if decompress(x) is not None:
            enc.append(x)
        x2 = bytearray(x)
        x2[31] |= 0x80
        if decompress(bytes(x2)) is not None:
            enc.append(bytes(x2))
    for e in enc:
        assert compress(decompress(e)) != e
    return enc


def small_order_corpus():
    encs = eight_torsion_encodings() + non_canonical_point_encodings()[:6]
    cases = []
    for A in encs:
        for R in encs:
            cases.append((A, R + bytes(32)))
    return cases


EXCLUDED_POINT_ENCODINGS = [bytes.fromhex(h) for h in [
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0100000000000000000000000000000000000000000000000000000000000000",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "13e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
    "b4176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "d9ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "daffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
]]


def point_order(pt):
    """reference tests/util/mod.rs:170-191 order(): '1','2','4','8','p','8p'."""
    if is_identity(mul_by_cofactor(pt)):
        p2 = double(pt)
        p4 = double(p2)
        if is_identity(pt):
            return "1"
        if is_identity(p2):
            return "2"
        if is_identity(p4):
            return "4"
        return "8"
    return "p" if is_identity(scalar_mul(L, pt)) else "8p"
