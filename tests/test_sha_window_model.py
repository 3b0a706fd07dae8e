"""CPU: a Python model of k_challenge's LDS-staged message windows (csrc/edc_prep.hip,
sha_stage / sha_staged_state): the 16 words of every SHA-512 block built exactly as the kernel
builds them (16-byte aligned DMA chunks, a zero line for chunks past the message or for a window
that starts at or past its end, the end marker fixed in the lane's column, words read from the
window at the byte slack) must equal the FIPS 180-4 padded R || A || M, for every message length
up to 3 blocks and every arena alignment. The GPU tests check the kernel itself
(test_gpu_multiblock.py)."""
import random


def padded(head, msg):
    m = head + msg
    L = len(m)
    return m + b"\x80" + b"\0" * ((112 - (L + 1) % 128) % 128) + (8 * L).to_bytes(16, "big")


def model_blocks(mem, mbase, mlen, head):
    total = 64 + mlen
    nblocks = (total + 17 + 127) // 128
    out = b""
    for blk in range(nblocks):
        w0 = blk * 128 - 64 if blk else 0
        wlen = 128 if blk else 64
        S = (mbase + w0) & ~15
        last = ((mbase + mlen - 1) & ~15) if mlen else 0
        inside = mlen > w0
        nch = 9 if blk else 5
        col = bytearray()
        for c in range(9):
            g = S + 16 * c
            if c < nch:
                col += mem[g:g + 16] if inside and g <= last else bytes(16)
            else:
                col += b"\xee" * 16                        # never staged in block 0
        q0b = (mbase + w0) & 15
        e_rel = mlen - w0
        if 0 <= e_rel < wlen:                              # the message ends in this window
            pos = q0b + e_rel
            di, sb = pos >> 2, pos & 3
            d = bytearray(col[4 * di:4 * di + 4])
            for k in range(sb, 4):
                d[k] = 0
            d[sb] = 0x80
            col[4 * di:4 * di + 4] = d
            for x in range(di + 1, (di | 3) + 1):
                col[4 * x:4 * x + 4] = bytes(4)
        words = [head[8 * t:8 * t + 8] for t in range(8)] if blk == 0 else []
        t0 = 0 if blk else 8
        for t in range(t0, 16):
            st = q0b + 8 * (t - t0)
            words.append(bytes(col[st:st + 8]))
        b = b"".join(words)
        if blk == nblocks - 1:
            b = b[:112] + bytes(8) + (total * 8).to_bytes(8, "big")
        out += b
    return out


def test_staged_windows_equal_fips_padding():
    rnd = random.Random(1)
    for shift in range(16):
        for mlen in range(0, 420):
            mem = bytearray(rnd.randbytes(2048))
            mbase = 512 + shift
            head = rnd.randbytes(64)
            assert model_blocks(mem, mbase, mlen, head) == padded(head, bytes(mem[mbase:mbase + mlen])), (shift, mlen)
