"""GPU parity: libhbam.so (HIP, gfx950) against the CPU oracle on the same inputs.
Bit-exact for every byte, index and key; identical exception class at the same record."""
import os
import zlib

import numpy as np
import pytest

from conftest import GOLDEN
from helpers import assert_same_split

pytestmark = pytest.mark.gpu

GOLDEN_FILES = ["small_pe.bam", "edge_htslib_empty.bam", "edge_uniform_long.bam",
                "edge_unsorted_l1.bam"]


def _load(name):
    return np.fromfile(os.path.join(GOLDEN, name), dtype=np.uint8)


def _whole(data):
    return (len(data) << 16) | 0xffff


# ---- K1/K2: scan + inflate -------------------------------------------------------------
@pytest.mark.parametrize("name", GOLDEN_FILES)
def test_scan_and_inflate_bit_exact(gpu_ctx, oracle_mod, name):
    data = _load(name)
    rc, blocks = gpu_ctx.scan_blocks(data)
    ref = oracle_mod.scan_blocks(data)
    assert rc == 0
    for k in ("coff", "clen", "isize", "crc"):
        assert np.array_equal(blocks[k], ref[k]), k
    rc, u, off, st = gpu_ctx.inflate(data, blocks, check_crc=True)
    assert rc == 0 and np.all(st == 0)
    want = b"".join(zlib.decompressobj(-15).decompress(bytes(data[int(c) + 18:int(c) + int(l) - 8]))
                    for c, l in zip(ref["coff"], ref["clen"]))
    assert u.tobytes() == want


def test_terminator_known_answer_on_device(gpu_ctx, oracle_mod):
    """The reference's bgzf-terminator.bin through the HIP path: the device block scan finds
    one 28-byte block of ISIZE 0 and CRC 0, the device inflate yields 0 bytes with status OK,
    and a BAM whose records are followed by terminators (one mid-file, one at the end) decodes
    to the same records as the oracle reads (an empty block ends nothing but a read() call)."""
    t = np.fromfile(os.path.join(GOLDEN, "bgzf-terminator.bin"), np.uint8)
    rc, b = gpu_ctx.scan_blocks(t)
    assert rc == 0
    assert list(b["coff"]) == [0] and list(b["clen"]) == [28] and list(b["isize"]) == [0]
    assert list(b["crc"]) == [0]
    rc, u, off, st = gpu_ctx.inflate(t, b, check_crc=True)
    assert rc == 0 and list(st) == [0] and int(off[-1]) == 0
    assert gpu_ctx.guess_bgzf_block_start(t, 0, len(t)) == oracle_mod.guess_bgzf_block_start(t, 0, len(t))
    data = _load("small_pe.bam")
    blocks = oracle_mod.scan_blocks(data)
    cut = int(blocks["coff"][len(blocks["coff"]) // 2])
    twice = np.concatenate([data[:cut], t, data[cut:], t])
    h = oracle_mod.read_header(twice)
    ref = oracle_mod.read_split(twice, h["first_voffset"], _whole(twice))
    got = gpu_ctx.decode_split(twice, h["first_voffset"], _whole(twice), n_ref=-1)
    assert got["rc"] == 0, got
    assert_same_split(got, ref)


def test_thousands_of_empty_blocks(gpu_ctx, oracle_mod, genbam):
    """An empty BGZF block after every data block (1329 of them, past the former 1024-entry
    event list): the whole-file read and every guessed split equal the oracle's (a read that
    meets an exhausted block followed by an empty one sees end-of-stream, htsjdk 1.131)."""
    m = np.asarray(genbam.generate(records=260000, seed=11, straddle=0, empty_every=1, odd_every=13))
    blocks = oracle_mod.scan_blocks(m)
    assert int(np.sum(blocks["isize"] == 0)) > 1024
    h = oracle_mod.read_header(m)
    ref = oracle_mod.read_split(m, h["first_voffset"], _whole(m))
    got = gpu_ctx.decode_split(m, h["first_voffset"], _whole(m), n_ref=h["n_ref"])
    assert got["rc"] == 0, got
    assert_same_split(got, ref)
    b, e = oracle_mod.file_splits(len(m), 1 << 20)
    want = oracle_mod.probabilistic_splits(m, b, e)
    n, vs, ve = gpu_ctx.probabilistic_splits(m, b, e)
    assert not isinstance(want, int) and n == len(want[0])
    assert np.array_equal(vs, want[0]) and np.array_equal(ve, want[1])
    for a, z in zip(vs, ve):
        ref = oracle_mod.read_split(m, int(a), int(z))
        got = gpu_ctx.decode_split(m, int(a), int(z), n_ref=h["n_ref"])
        assert got["rc"] == 0, got
        assert_same_split(got, ref)


@pytest.mark.parametrize("kw", [dict(payload=64, level=6), dict(payload=300, level=1, straddle=0),
                                dict(records=20000, empty_every=1, payload=200, level=9)])
def test_tiny_blocks_scan_and_decode(gpu_ctx, oracle_mod, genbam, kw):
    """BGZF blocks far below 1 KiB compressed (more than the block scan's 64 candidate slots per
    64 KiB chunk: the exact two-pass scan takes over): the block table, the whole-file read
    and every guessed split equal the oracle's."""
    kw = dict(kw)
    m = np.asarray(genbam.generate(records=kw.pop("records", 3000), seed=35, **kw))
    ref_b = oracle_mod.scan_blocks(m)
    assert len(ref_b["coff"]) > 64 * (len(m) // 65536 + 1)  # some chunk overflows
    rc, blocks = gpu_ctx.scan_blocks(m)
    assert rc == 0, gpu_ctx.last_error()
    for k in ("coff", "clen", "isize", "crc"):
        assert np.array_equal(blocks[k], ref_b[k]), k
    h = oracle_mod.read_header(m)
    ref = oracle_mod.read_split(m, h["first_voffset"], _whole(m))
    got = gpu_ctx.decode_split(m, h["first_voffset"], _whole(m), n_ref=-1)
    assert got["rc"] == 0, got
    assert_same_split(got, ref)
    b, e = oracle_mod.file_splits(len(m), 1 << 17)
    want = oracle_mod.probabilistic_splits(m, b, e)
    n, vs, ve = gpu_ctx.probabilistic_splits(m, b, e)
    assert not isinstance(want, int) and n == len(want[0])
    assert np.array_equal(vs, want[0]) and np.array_equal(ve, want[1])
    for a, z in zip(vs, ve):
        ref = oracle_mod.read_split(m, int(a), int(z))
        got = gpu_ctx.decode_split(m, int(a), int(z), n_ref=h["n_ref"])
        assert got["rc"] == 0, got
        assert_same_split(got, ref)


def _bgzf_block(payload, level=6):
    """One BGZF block (BSIZE/CRC/ISIZE as htsjdk writes them) holding `payload`."""
    import struct
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    body = c.compress(payload) + c.flush()
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + \
        struct.pack("<H", len(body) + 25)
    return hdr + body + struct.pack("<II", zlib.crc32(payload), len(payload))


@pytest.mark.parametrize("fname", ["guess_window_4197.bin", "guess_window_7433.bin"])
def test_inflate_every_output_misalignment(gpu_ctx, fname):
    """Blocks whose output starts at each of the 16 offsets of a 16-byte chunk, among them
    ISIZE % 16 != 0 blocks that end in a match (the LZ77 pass must resolve and write back
    the last bytes of a block that starts unaligned).  Windows of the config #3 file."""
    import struct
    w = np.fromfile(os.path.join(GOLDEN, fname), np.uint8).tobytes()
    blocks, p = [], w.find(b"\x1f\x8b\x08\x04")
    while p + 18 <= len(w) and w[p:p + 4] == b"\x1f\x8b\x08\x04":
        bs = struct.unpack("<H", w[p + 16:p + 18])[0] + 1
        if p + bs > len(w):
            break
        blocks.append((p, bs) + struct.unpack("<II", w[p + bs - 8:p + bs]))
        p += bs
    assert any(b[3] % 16 for b in blocks)
    want = {b[0]: zlib.decompressobj(-15).decompress(w[b[0] + 18:b[0] + b[1] - 8]) for b in blocks}
    for lead in range(16):
        data = w + _bgzf_block(bytes(range(65, 65 + lead))) if lead else w
        lst = ([(len(w), len(data) - len(w), zlib.crc32(bytes(range(65, 65 + lead))), lead)] if lead else []) + blocks
        B = {"coff": np.array([b[0] for b in lst], np.uint64), "clen": np.array([b[1] for b in lst], np.uint32),
             "crc": np.array([b[2] for b in lst], np.uint32), "isize": np.array([b[3] for b in lst], np.uint32)}
        rc, u, off, st = gpu_ctx.inflate(np.frombuffer(data, np.uint8), B, check_crc=True)
        assert rc == 0 and np.all(st == 0), (lead, st)
        for j, b in enumerate(lst[1 if lead else 0:], start=1 if lead else 0):
            assert u[int(off[j]):int(off[j + 1])].tobytes() == want[b[0]], (lead, j)


@pytest.mark.parametrize("mode", ["lane", "wave"])
def test_inflate_independent_of_launch_position(oracle_mod, genbam, monkeypatch, mode):
    """The r02 profiling-build failure depended on a block's position in the
    launch, not on its bytes: only waves that started in a slot an earlier wave of the launch
    had vacated decoded wrongly.  Here the same blocks (zlib levels 1/5/9, uniform and binned
    qualities, stored and fixed-Huffman blocks) are repeated until the launch holds ~2.7
    waves per slot of the whole chip (2 waves/SIMD x 4 SIMDs x 256 CUs) for the lane pass
    (k_inflate_tokens), and 350,000 one-block waves for the wave pass (k_inflate_wave, forced by
    HBAM_WAVE_MAX_BLOCKS), so most copies run in a reused slot; every copy must inflate
    CRC-clean on the device (status 0)."""
    import ctypes as C
    from hadoop_bam import _lib
    monkeypatch.setenv("HBAM_WAVE_MAX_BLOCKS", "1000000000" if mode == "wave" else "0")
    gpu_ctx = _lib.Context(0)
    parts = [np.asarray(genbam.generate(records=4000, seed=31, level=1)),
             np.asarray(genbam.generate(records=4000, seed=32, level=9, uniform_qual=1)),
             np.asarray(genbam.generate(records=1500, seed=33, level=0)),
             np.asarray(genbam.generate(records=1500, seed=34, payload=64, level=6))]
    base, coffs, clens, isz, crcs = 0, [], [], [], []
    for d in parts:
        b = oracle_mod.scan_blocks(d)  # the block list only (this test is about the inflate)
        if len(b["coff"]) > 100:  # the fixed-Huffman file: a sample of its 64-byte blocks
            b = {k: v[:100] for k, v in b.items()}
        coffs += [int(c) + base for c in b["coff"]]
        clens += list(b["clen"]); isz += list(b["isize"]); crcs += list(b["crc"])
        base += len(d)
    data = np.concatenate(parts)
    nuniq = len(coffs)
    n = -(-350_000 // nuniq) * nuniq  # ~2.7 x 131,072 resident lanes
    arr = (_lib.Block * n)()
    for i in range(n):
        j = i % nuniq
        arr[i].coff, arr[i].clen, arr[i].isize, arr[i].crc = coffs[j], int(clens[j]), int(isz[j]), int(crcs[j])
    off = np.zeros(n + 1, np.uint64)
    st = np.full(n, 99, np.int32)
    try:
        rc = gpu_ctx.L.hbam_inflate(gpu_ctx.h, C.c_void_p(data.ctypes.data), 0, len(data), arr, n, 1,
                                    None, 0, off.ctypes.data, st.ctypes.data)
        assert rc == 0, gpu_ctx.last_error()
        bad = np.nonzero(st != 0)[0]
        assert len(bad) == 0, (mode, len(bad), n, bad[:8], st[bad[:8]])
    finally:
        gpu_ctx.close()


@pytest.mark.parametrize("kw", [dict(level=0), dict(level=1), dict(level=9),
                                dict(uniform_qual=1, level=6), dict(payload=64, level=6),
                                dict(payload=300, level=1, straddle=0)])
def test_inflate_deflate_variants(gpu_ctx, oracle_mod, genbam, kw):
    """stored blocks (level 0), fixed-Huffman blocks (tiny payloads), all zlib levels."""
    data = np.asarray(genbam.generate(records=1500, seed=21, **kw))
    ref = oracle_mod.scan_blocks(data)
    rc, u, off, st = gpu_ctx.inflate(data, ref, check_crc=True)
    assert rc == 0 and np.all(st == 0)
    want = b"".join(zlib.decompressobj(-15).decompress(bytes(data[int(c) + 18:int(c) + int(l) - 8]))
                    for c, l in zip(ref["coff"], ref["clen"]))
    assert u.tobytes() == want


def test_inflate_corrupted_blocks_match_zlib_classes(gpu_ctx, oracle_mod):
    """Bit flips in compressed data: the device reports the same outcome as zlib (via the
    oracle's BlockGunzipper restatement): OK / short (SAMFormatException) / data error."""
    data = _load("small_pe.bam").copy()
    ref = oracle_mod.scan_blocks(data)
    rng = np.random.default_rng(17)
    nb = len(ref["coff"])
    for i in range(nb):
        c, l = int(ref["coff"][i]), int(ref["clen"][i])
        if l <= 40:
            continue
        for _ in range(3):
            p = c + 18 + int(rng.integers(0, l - 26))
            data[p] ^= np.uint8(1 << int(rng.integers(0, 8)))
    rc, u, off, st = gpu_ctx.inflate(data, ref, check_crc=True)
    assert rc == 0
    codes = {0: 0, oracle_mod.OR_EFORMAT: -3, oracle_mod.OR_EDATA: -7}
    for i in range(nb):
        c, l = int(ref["coff"][i]), int(ref["clen"][i])
        orc, out = oracle_mod.inflate_block(bytes(data[c:c + l]), check_crc=True)
        assert int(st[i]) == codes[orc], (i, int(st[i]), orc)
        if orc == 0:
            assert u[int(off[i]):int(off[i + 1])].tobytes() == out
    assert len(set(int(x) for x in st)) >= 2  # the corruption exercised error paths


@pytest.mark.parametrize("kw", [dict(seed=31), dict(seed=32, level=1), dict(seed=33, level=9),
                                dict(seed=34, uniform_qual=1, level=6), dict(seed=35, level=0),
                                dict(seed=36, payload=64, level=6)])
def test_huffman_wave_and_lane_passes_agree(oracle_mod, genbam, monkeypatch, kw):
    """The two Huffman passes (k_inflate_wave: a wave per block, used for calls of up to
    HBAM_WAVE_MAX_BLOCKS blocks; k_inflate_tokens: a lane per block, above) give the same bytes
    and statuses as zlib on the same blocks, corrupted ones included."""
    from hadoop_bam import _lib
    data = np.asarray(genbam.generate(records=6000, seed=kw["seed"],
                                      **{k: v for k, v in kw.items() if k != "seed"})).copy()
    ref = oracle_mod.scan_blocks(data)
    bad = data.copy()
    rng = np.random.default_rng(kw["seed"])
    for i in range(0, len(ref["coff"]), 3):  # every third block: a bit flip
        c, l = int(ref["coff"][i]), int(ref["clen"][i])
        if l > 40:
            p = c + 18 + int(rng.integers(0, l - 26))
            bad[p] ^= np.uint8(1 << int(rng.integers(0, 8)))
    got = {}
    for mode, limit in (("wave", "1000000000"), ("lane", "0")):
        monkeypatch.setenv("HBAM_WAVE_MAX_BLOCKS", limit)
        ctx = _lib.Context(0)
        try:
            got[mode] = [ctx.inflate(d, ref, check_crc=True) for d in (data, bad)]
        finally:
            ctx.close()
    for (rw, uw, ow, sw), (rl, ul, ol, sl) in zip(got["wave"], got["lane"]):
        assert rw == rl == 0
        assert np.array_equal(sw, sl)
        for i in range(len(ref["coff"])):
            if int(sw[i]) == 0:
                assert uw[int(ow[i]):int(ow[i + 1])].tobytes() == ul[int(ol[i]):int(ol[i + 1])].tobytes(), i
    rc, u, off, st = got["wave"][0]
    want = b"".join(zlib.decompressobj(-15).decompress(bytes(data[int(c) + 18:int(c) + int(l) - 8]))
                    for c, l in zip(ref["coff"], ref["clen"]))
    assert np.all(st == 0) and u.tobytes() == want


@pytest.mark.parametrize("slices", [2, 3, 7])
def test_sliced_inflate_pipeline(oracle_mod, monkeypatch, slices):
    """The Huffman / LZ77 passes cut into slices on two streams (HBAM_INFLATE_SLICES forces it
    on small files): a whole-file decode equals the oracle's."""
    from hadoop_bam import _lib
    monkeypatch.setenv("HBAM_INFLATE_SLICES", str(slices))
    ctx = _lib.Context(0)
    try:
        for name in ("small_pe.bam", "edge_uniform_long.bam"):
            data = _load(name)
            h = oracle_mod.read_header(data)
            ref = oracle_mod.read_split(data, h["first_voffset"], _whole(data))
            got = ctx.decode_split(data, h["first_voffset"], _whole(data), n_ref=-1)
            assert got["rc"] == 0, got
            assert_same_split(got, ref)
    finally:
        ctx.close()


# ---- K5-K8: record reader over splits -------------------------------------------------
@pytest.mark.parametrize("name", GOLDEN_FILES)
def test_decode_whole_file(gpu_ctx, oracle_mod, name):
    data = _load(name)
    h = oracle_mod.read_header(data)
    ref = oracle_mod.read_split(data, h["first_voffset"], _whole(data))
    got = gpu_ctx.decode_split(data, h["first_voffset"], _whole(data), n_ref=-1)
    assert got["rc"] == 0, got
    assert_same_split(got, ref)


@pytest.mark.parametrize("name,split_size", [("small_pe.bam", 256 << 10),
                                             ("small_pe.bam", 64 << 10),
                                             ("edge_uniform_long.bam", 128 << 10),
                                             ("edge_htslib_empty.bam", 100 << 10)])
def test_probabilistic_splits_and_split_reads(gpu_ctx, oracle_mod, name, split_size):
    data = _load(name)
    b, e = oracle_mod.file_splits(len(data), split_size)
    want = oracle_mod.probabilistic_splits(data, b, e)
    n, vs, ve = gpu_ctx.probabilistic_splits(data, b, e)
    if isinstance(want, int):
        assert n == want
        return
    assert n == len(want[0])
    assert np.array_equal(vs, want[0]) and np.array_equal(ve, want[1])
    h = oracle_mod.read_header(data)
    for a, z in zip(vs, ve):
        ref = oracle_mod.read_split(data, int(a), int(z))
        got = gpu_ctx.decode_split(data, int(a), int(z), n_ref=h["n_ref"])
        assert got["rc"] == 0, got
        assert_same_split(got, ref)


def test_guesses_random_offsets(gpu_ctx, oracle_mod):
    data = _load("small_pe.bam")
    h = oracle_mod.read_header(data)
    rng = np.random.default_rng(3)
    beg = np.sort(rng.integers(0, len(data), 300)).astype(np.int64)
    end = np.minimum(beg + rng.integers(1, 400000, 300), len(data)).astype(np.int64)
    rc, out, err = gpu_ctx.guess_batch(data, beg, end, h["n_ref"])
    assert rc == 0
    for i in range(len(beg)):
        g, e = oracle_mod.guess_bam_record_start(data, int(beg[i]), int(end[i]), h["n_ref"])
        assert (int(out[i]), int(err[i])) == (g, e), i


@pytest.mark.parametrize("level,k", [(0, 60), (1, 200)])
def test_guesses_window_exhaustion(gpu_ctx, oracle_mod, genbam, level, k):
    """Stored / barely compressed blocks: three block changes do not fit the 256 KiB guess
    window, so every candidate's record chain runs out of bytes and the guesser walks the
    record starts of the block one by one (BAMSplitGuesser.java:159-208) — the chain memo's
    case.  Every guess equals the oracle's."""
    data = np.asarray(genbam.generate(target_bytes=6 << 20, seed=11, level=level, threads=8))
    h = oracle_mod.read_header(data)
    rng = np.random.default_rng(5)
    beg = np.sort(rng.integers(0, len(data), k)).astype(np.int64)
    end = np.minimum(beg + (128 << 20), len(data)).astype(np.int64)
    rc, out, err = gpu_ctx.guess_batch(data, beg, end, h["n_ref"])
    assert rc == 0
    for i in range(len(beg)):
        g, e = oracle_mod.guess_bam_record_start(data, int(beg[i]), int(end[i]), h["n_ref"])
        assert (int(out[i]), int(err[i])) == (g, e), i


def _windows(ctx, data, beg, end, bgzf=False):
    """The guess windows (the bytes each guess reads), concatenated, and their offsets."""
    f = ctx.guess_bgzf_window_len if bgzf else ctx.guess_window_len
    wl = [f(len(data), int(b), int(e)) for b, e in zip(beg, end)]
    off = np.zeros(len(wl) + 1, np.uint64)
    off[1:] = np.cumsum(wl)
    parts = [data[int(b):int(b) + n] for b, n in zip(beg, wl) if n]
    return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), off


def _edge_offsets(n, rng, k):
    beg = list(rng.integers(0, n, k)) + [0, 0, 1, n - 30, n - 2, n - 1, n, 5, 100, 4096]
    end = [min(int(b) + int(rng.integers(1, 400000)), n) for b in beg[:k]] + \
        [n, 3, 2, n, n, n, n, 5, 99, 4096 + 262139 + 7]
    return np.array(beg, np.int64), np.array(end, np.int64)


def test_guess_windows_match_oracle(gpu_ctx, oracle_mod):
    """hbam_guess_windows over caller-gathered windows (host and device buffers) equals the
    oracle's guess over the whole file, incl. windows cut by EOF, empty windows (end <= beg,
    beg at EOF) and windows shorter than a BGZF header."""
    import torch
    data = _load("small_pe.bam")
    h = oracle_mod.read_header(data)
    beg, end = _edge_offsets(len(data), np.random.default_rng(13), 200)
    w, off = _windows(gpu_ctx, data, beg, end)
    assert int(off[-1]) < 200 * 262139 + 1
    want = [oracle_mod.guess_bam_record_start(data, int(b), int(e), h["n_ref"]) for b, e in zip(beg, end)]
    for src in (w, torch.from_numpy(w.copy()).cuda() if len(w) else w):
        rc, out, err = gpu_ctx.guess_windows(src, off, len(data), beg, end, h["n_ref"])
        assert rc == 0, gpu_ctx.last_error()
        assert [(int(a), int(b)) for a, b in zip(out, err)] == [(int(g), int(e)) for g, e in want]
    # the whole-file call from host memory stages only these windows and agrees
    rc, out2, err2 = gpu_ctx.guess_batch(data, beg, end, h["n_ref"])
    assert rc == 0 and np.array_equal(out2, out) and np.array_equal(err2, err)


def test_guess_windows_reject_wrong_window(gpu_ctx, oracle_mod):
    data = _load("small_pe.bam")
    h = oracle_mod.read_header(data)
    beg, end = np.array([1000, 90000], np.int64), np.array([500000, 95000], np.int64)
    w, off = _windows(gpu_ctx, data, beg, end)
    off[1] -= 1  # one byte short
    rc, _, _ = gpu_ctx.guess_windows(w[:-1], off, len(data), beg, end, h["n_ref"])
    assert rc == -11  # HBAM_EINVAL


@pytest.mark.parametrize("name,split_size", [("small_pe.bam", 256 << 10), ("small_pe.bam", 64 << 10),
                                             ("edge_uniform_long.bam", 128 << 10),
                                             ("edge_htslib_empty.bam", 100 << 10)])
def test_probabilistic_splits_windows(gpu_ctx, oracle_mod, name, split_size):
    """getSplits from the header prefix + the FileSplits' guess windows only."""
    data = _load(name)
    b, e = oracle_mod.file_splits(len(data), split_size)
    want = oracle_mod.probabilistic_splits(data, b, e)
    w, off = _windows(gpu_ctx, data, b.astype(np.int64), e.astype(np.int64))
    for hl in (1 << 20, 40):  # 40 bytes: too short for the header -> HBAM_ETRUNC
        n, vs, ve = gpu_ctx.probabilistic_splits_windows(data[:hl], w, off, len(data), b, e)
        if hl == 40:
            assert n == -2
            continue
        if isinstance(want, int):
            assert n == want
            continue
        assert n == len(want[0]) and np.array_equal(vs, want[0]) and np.array_equal(ve, want[1])


def test_bgzf_guesser_window(gpu_ctx, oracle_mod):
    data = _load("edge_uniform_long.bam")
    rng = np.random.default_rng(4)
    for beg in list(rng.integers(0, len(data) - 10, 30)) + [len(data) - 3, len(data)]:
        end = min(int(beg) + int(rng.integers(10, 200000)), len(data))
        wl = gpu_ctx.guess_bgzf_window_len(len(data), int(beg), end)
        got = gpu_ctx.guess_bgzf_window(data[int(beg):int(beg) + wl], len(data), int(beg), end)
        assert got == oracle_mod.guess_bgzf_block_start(data, int(beg), end)


def test_mirror_guessers_read_only_windows(oracle_mod, tmp_path):
    """The mirror's BAMSplitGuesser / getSplits read the header prefix and each guess window from
    the file, never the whole file."""
    from hadoop_bam import BAMInputFormat, BAMSplitGuesser, Configuration, compute_file_splits
    data = _load("small_pe.bam")
    big = tmp_path / "big.bam"
    big.write_bytes(bytes(data))
    reads = []

    class Counting:
        def __init__(self, f):
            self.f = f

        def seek(self, *a):
            return self.f.seek(*a)

        def read(self, n=-1):
            b = self.f.read(n)
            reads.append(len(b))
            return b

    with open(big, "rb") as f:
        g = BAMSplitGuesser(Counting(f))
        h = oracle_mod.read_header(data)
        for beg in (0, 70000, 1 << 20, len(data) - 50000):
            end = min(beg + (1 << 20), len(data))
            assert g.guessNextBAMRecordStart(beg, end) == \
                oracle_mod.guess_bam_record_start(data, beg, end, h["n_ref"])[0]
    assert max(reads) <= max(262139, 1 << 20) and sum(reads) < len(data) * 2
    fs = compute_file_splits(str(big), len(data), 256 << 10)
    got = BAMInputFormat().getSplits(fs, Configuration())
    b, e = oracle_mod.file_splits(len(data), 256 << 10)
    vs, ve = oracle_mod.probabilistic_splits(data, b, e)
    assert [(s.getStartVirtualOffset(), s.getEndVirtualOffset()) for s in got] == \
        [(int(x), int(y)) for x, y in zip(vs, ve)]


def test_bgzf_guesser(gpu_ctx, oracle_mod):
    data = _load("edge_uniform_long.bam")
    rng = np.random.default_rng(4)
    for beg in rng.integers(0, len(data) - 10, 40):
        end = min(int(beg) + int(rng.integers(10, 200000)), len(data))
        assert gpu_ctx.guess_bgzf_block_start(data, int(beg), end) == \
            oracle_mod.guess_bgzf_block_start(data, int(beg), end)


# ---- exception semantics --------------------------------------------------------------
def _mutations(data, oracle_mod):
    h = oracle_mod.read_header(data)
    blocks = oracle_mod.scan_blocks(data)
    out = {}
    out["truncated_mid_block"] = data[:int(blocks["coff"][40]) + 100]
    out["truncated_at_block"] = data[:int(blocks["coff"][40])]
    out["garbage_tail"] = np.concatenate([data[:int(blocks["coff"][30])],
                                          np.frombuffer(b"\x00garbage-bytes-here-xxxxxxxx", np.uint8)])
    bad = data.copy()
    c, l = int(blocks["coff"][25]), int(blocks["clen"][25])
    bad[c + 18 + l // 2] ^= 0xff
    out["corrupt_deflate"] = bad
    return h, out


def test_error_semantics_match_oracle(gpu_ctx, oracle_mod):
    data = _load("small_pe.bam")
    h, muts = _mutations(data, oracle_mod)
    for name, m in muts.items():
        m = np.ascontiguousarray(m)
        ref = oracle_mod.read_split(m, h["first_voffset"], _whole(m))
        got = gpu_ctx.decode_split(m, h["first_voffset"], _whole(m), n_ref=h["n_ref"])
        assert got["rc"] == 0, (name, got)
        assert_same_split(got, ref, pools=True), name


def test_bad_refid_raises_illegal_argument_at_record(gpu_ctx, oracle_mod, genbam):
    """A record whose refID is outside the dictionary: IllegalArgumentException at that
    record (BAMRecord ctor via BAMRecordCodec(header)); htslib packing keeps it in one block."""
    import zlib as z
    data = np.asarray(genbam.generate(records=800, seed=5, straddle=0, level=6))
    h = oracle_mod.read_header(data)
    blocks = oracle_mod.scan_blocks(data)
    i = 3
    c, l = int(blocks["coff"][i]), int(blocks["clen"][i])
    u = bytearray(z.decompressobj(-15).decompress(bytes(data[c + 18:c + l - 8])))
    # second record in the block: set refID = n_ref + 3
    bs = int.from_bytes(u[0:4], "little")
    p = 4 + bs
    u[p + 4:p + 8] = (h["n_ref"] + 3).to_bytes(4, "little")
    co = z.compressobj(6, z.DEFLATED, -15)
    cd = co.compress(bytes(u)) + co.flush()
    import struct
    blk = (b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" +
           struct.pack("<H", len(cd) + 25) + cd + struct.pack("<II", z.crc32(bytes(u)), len(u)))
    m = np.concatenate([data[:c], np.frombuffer(blk, np.uint8), data[c + l:]])
    ref = oracle_mod.read_split(m, h["first_voffset"], _whole(m))
    assert ref["status"] == oracle_mod.OR_EREFID
    got = gpu_ctx.decode_split(m, h["first_voffset"], _whole(m), n_ref=h["n_ref"])
    assert_same_split(got, ref)


# ---- the drop-in API ---------------------------------------------------------------------
def test_bam_input_format_record_reader(oracle_mod, tmp_path):
    """getSplits + createRecordReader + nextKeyValue through the mirror: every handed-out
    (key, value) equals the oracle's BAMRecordReader over the same FileVirtualSplits — the key,
    the value's wire bytes (SAMRecordWritable.write = BAMRecordCodec.encode of the untouched
    record), every getter (fixed fields, name, CIGAR, SEQ, QUAL) against an independent host
    decode of the oracle's record bytes, and the write/readFields round trip."""
    import io
    from hadoop_bam import BAMInputFormat, Configuration, SAMRecordWritable, compute_file_splits
    from hadoop_bam.formats import BAMRecordBytes
    path = os.path.join(GOLDEN, "small_pe.bam")
    data = _load("small_pe.bam")
    fmt = BAMInputFormat()
    fsplits = compute_file_splits(path, len(data), 512 << 10)
    for j, f in enumerate(fsplits):
        f.hosts = ["host%d" % j]
    splits = fmt.getSplits(fsplits, Configuration())
    # locations follow the FileSplit whose guess opened each virtual split (BAMInputFormat.java:202)
    starts = [f.getStart() for f in fsplits]
    for s in splits:
        owner = max(j for j, b in enumerate(starts) if b <= s.getStartVirtualOffset() >> 16)
        assert s.getLocations() == ["host%d" % owner]
    b, e = oracle_mod.file_splits(len(data), 512 << 10)
    vs, ve = oracle_mod.probabilistic_splits(data, b, e)
    assert [(s.getStartVirtualOffset(), s.getEndVirtualOffset()) for s in splits] == \
        [(int(x), int(y)) for x, y in zip(vs, ve)]
    getters = ("getReferenceIndex", "getAlignmentStart", "getFlags", "getReadUnmappedFlag",
               "getMappingQuality", "getMateReferenceIndex", "getMateAlignmentStart",
               "getInferredInsertSize", "getIndexingBin", "getReadName", "getCigarString",
               "getReadString", "getBaseQualities", "getReadBases", "getVariableBinaryRepresentation")
    n_total = 0
    for s, a, z in zip(splits, vs, ve):
        ref = oracle_mod.read_split(data, int(a), int(z))
        pay, off = oracle_mod.record_payloads(ref)
        rr = fmt.createRecordReader(s, Configuration())
        k = 0
        while rr.nextKeyValue():
            assert rr.getCurrentKey().get() == int(ref["key"][k])
            v = rr.getCurrentValue()
            want_bytes = bytes(pay[int(off[k]):int(off[k + 1])])
            rec = v.get()
            assert rec.toBAMBytes() == want_bytes, k
            want = BAMRecordBytes(want_bytes)
            for g in getters:
                assert getattr(rec, g)() == getattr(want, g)(), (k, g)
            buf = io.BytesIO()
            v.write(buf)
            back = SAMRecordWritable()
            back.readFields(io.BytesIO(buf.getvalue()))
            assert back.get().toBAMBytes() == want_bytes
            k += 1
        assert k == ref["n"]
        n_total += k
        rr.close()
    assert n_total > 10000


# ---- full-size properties --------------------------------------------------------------
def test_large_file_properties(gpu_ctx, genbam):
    """~400 MB compressed: record count equals the generator's, voffsets strictly increase,
    mapped keys are non-decreasing in a coordinate-sorted file, inflated length matches."""
    g = genbam.generate(target_bytes=400 << 20, seed=2, threads=16)
    n_expected = g.n_records
    data = np.asarray(g)
    h = gpu_ctx.parse_header(data)
    got = gpu_ctx.decode_split(data, h["first_voffset"], _whole(data), n_ref=h["n_ref"])
    assert got["rc"] == 0 and got["status"] == 0
    assert got["n"] == n_expected
    assert np.all(np.diff(got["voffset"].astype(np.uint64)) > 0)
    mapped = (got["flag"] & 4) == 0
    k = got["key"][mapped & (got["ref_id"] >= 0)]
    assert np.all(np.diff(k) >= 0)
    assert got["timing"]["ubuf_bytes"] > 2 * len(data)


# ---- SplittingBAMIndexer on the device ----------------------------------
@pytest.mark.parametrize("fname", ["small_pe.bam", "edge_uniform_long.bam", "edge_unsorted_l1.bam"])
@pytest.mark.parametrize("g", [1, 7, 1024, 4096])
def test_splitting_index_matches_oracle(gpu_ctx, oracle_mod, fname, g):
    data = _load(fname)
    want = oracle_mod.splitting_index(data, granularity=g)
    rc, got = gpu_ctx.splitting_index(data, g)
    assert rc == 0, gpu_ctx.last_error()
    assert np.array_equal(got, want)


# ---- LZ77 pass on hand-built token blocks (k_resolve) ----------------------------------------
def _tokens(tokens, isize):
    """(bytes, bitmap) of a token block: literals as ints, matches as (len, dist)."""
    io = bytearray(isize)
    bm = np.zeros((isize + 31) // 32, np.uint32)
    op = 0
    for t in tokens:
        if isinstance(t, int):
            io[op] = t
            op += 1
        else:
            n, d = t
            io[op:op + 3] = bytes([n - 3, (d - 1) & 0xff, (d - 1) >> 8])
            bm[op >> 5] |= np.uint32(1 << (op & 31))
            op += n
    assert op == isize
    return bytes(io), bm


def test_resolve_tokens_expands_matches(gpu_ctx):
    lits = list(b"ACGTTGCA")
    toks = lits + [(20, 8), (5, 1)] + list(b"xy") + [(258, 30)]
    isize = len(lits) + 20 + 5 + 2 + 258
    io, bm = _tokens(toks, isize)
    rc, st, out = gpu_ctx.resolve_tokens(io, bm)
    want = bytearray()
    for t in toks:
        if isinstance(t, int):
            want.append(t)
        else:
            n, d = t
            for _ in range(n):
                want.append(want[-d])
    assert rc == 0 and st == 0
    assert out == bytes(want)


@pytest.mark.parametrize("case", ["dist_before_block", "hole_past_end", "tail_before_block",
                                  "dist_over_32k"])
def test_resolve_forged_descriptor_is_an_error_not_a_hang(gpu_ctx, case):
    """A descriptor the Huffman pass could not have written (source before the block start, or
    a hole running past the block end) makes k_resolve refuse the block (HBAM_EDATA) instead of
    copying from outside it or spinning on a batch that never becomes ready."""
    isize = 4096
    toks = list(range(64)) + [(100, 50)] + [0] * (isize - 164)
    io, bm = _tokens(toks, isize)
    io = bytearray(io)
    tail = (0, 0)
    if case == "dist_before_block":
        io[64 + 1], io[64 + 2] = 0xff, 0x0f  # dist 4096 > p = 64
    elif case == "hole_past_end":
        p = isize - 10
        io[p:p + 3] = bytes([200, 0, 0])      # len 203 from p: runs past isize
        bm[p >> 5] |= np.uint32(1 << (p & 31))
    elif case == "dist_over_32k":  # inside the block, but farther than DEFLATE's 32768
        isize = 40000
        io, bm = _tokens(list(range(64)) * 560 + [(100, 33000)] + [0] * (isize - 35940), isize)
        io = bytearray(io)
    else:
        tail = (5 | 2 << 16 | 0x80000000, 9)  # 2 bytes at op 5 from dist 9 > 5
    rc, st, _ = gpu_ctx.resolve_tokens(bytes(io), bm, *tail)
    assert rc == 0
    assert st == -7  # HBAM_EDATA


# ---- config #4 shape: byte-range shards read through streamed windows ------------------------
class _CountingReader:
    """A positioned read over a byte array that records every byte range requested (the
    FSDataInputStream.read(long, byte[], int, int) a Java map task would hand in)."""

    def __init__(self, data):
        self.data = data
        self.ranges = []

    def __call__(self, off, n):
        self.ranges.append((off, n))
        return self.data[off:off + n].tobytes()

    def total(self):
        return sum(n for _, n in self.ranges)

    def overlaps(self):
        r = sorted(self.ranges)
        return sum(max(0, (a0 + n0) - a1) for (a0, n0), (a1, _) in zip(r, r[1:]))


def _stream_read(gpu_ctx, data, a, z, n_ref, window, reader=None):
    """hbam_split_open/next (or hbam_split_open_reader/next with `reader`) over one
    FileVirtualSplit -> (concatenated columns, n windows)."""
    if reader is not None:
        ws = list(gpu_ctx.split_stream_reader(reader, len(data), int(a), int(z), n_ref, window_bytes=window))
    else:
        ws = list(gpu_ctx.split_stream(data, int(a), int(z), n_ref, window_bytes=window))
    cat = {"n": sum(w["n"] for w in ws), "status": 0, "err_record": 0}
    base = 0
    for w in ws:
        if w["status"] != 0:
            cat["status"] = w["status"]
            cat["err_record"] = base + w["err_record"]
        base += w["n"]
    from helpers import FIELDS
    for k in FIELDS + ("layout_ok",):
        cat[k] = np.concatenate([w[k] for w in ws]) if ws else np.zeros(0)
    for k in ("names", "cigars", "seq", "qual", "aux"):
        cat[k] = np.concatenate([w[k] for w in ws]) if ws else np.zeros(0)
    cat["payload"] = b"".join(w["ubuf"].tobytes() for w in ws)
    return cat, len(ws)


@pytest.mark.parametrize("name", GOLDEN_FILES)
@pytest.mark.parametrize("P", [2, 3, 5])
@pytest.mark.parametrize("split_local", [False, True])
def test_sharded_split_windows_match_oracle(gpu_ctx, oracle_mod, name, P, split_local):
    """P byte-range FileSplits of one file, aligned by the guesser (addProbabilisticSplits),
    each read through 64 KiB streamed windows (EMORE continuation at every window end): every
    shard equals the oracle's BAMRecordReader for that FileVirtualSplit, record bytes included;
    without the duplicated boundary-block records the shards concatenate to the whole-file read.
    split_local: the same through hbam_split_open_reader (positioned reads of the split's bytes
    only, each byte requested once)."""
    data = _load(name)
    L = len(data)
    b = np.array([L * k // P for k in range(P)], np.uint64)
    e = np.array([L * (k + 1) // P for k in range(P)], np.uint64)
    want = oracle_mod.probabilistic_splits(data, b, e)
    n, vs, ve = gpu_ctx.probabilistic_splits(data, b, e)
    if isinstance(want, int):
        assert n == want
        return
    assert np.array_equal(vs, want[0]) and np.array_equal(ve, want[1])
    h = oracle_mod.read_header(data)
    shards, windows = [], 0
    for a, z in zip(vs, ve):
        ref = oracle_mod.read_split(data, int(a), int(z))
        rd = _CountingReader(data) if split_local else None
        got, nwin = _stream_read(gpu_ctx, data, a, z, h["n_ref"], 64 << 10, reader=rd)
        assert_same_split(got, ref)
        if rd is not None:
            # only [vStart's block, vEnd's block + 192 KiB), no byte twice (the windows' overlap
            # is re-used from the previous window's staging)
            assert rd.overlaps() == 0
            assert min(o for o, _ in rd.ranges) >= int(a) >> 16
            assert max(o + n for o, n in rd.ranges) <= min(L, (int(z) >> 16) + (3 << 16))
        assert got["payload"] == oracle_mod.record_payloads(ref)[0].tobytes()
        windows += nwin
        shards.append(got)
    assert windows > 2 * len(shards)  # the EMORE continuation ran at many window ends
    whole = oracle_mod.read_split(data, h["first_voffset"], _whole(data))
    wv = set(int(x) for x in whole["voffset"])
    if all(int(a) in wv for a in vs[1:]) and whole["status"] == 0:
        vo = list(shards[0]["voffset"])
        for sh in shards[1:]:
            cut = int(np.searchsorted(sh["voffset"], vo[-1], side="right")) if vo else 0
            vo.extend(sh["voffset"][cut:])
        assert np.array_equal(np.array(vo, np.uint64), whole["voffset"])


def test_split_local_reader_reads_the_split_not_the_file(gpu_ctx, oracle_mod):
    """A small FileVirtualSplit of a 24 MB file through hbam_split_open_reader: the records equal
    the oracle's, and the bytes requested stay within the split's compressed bytes plus one
    window plus 64 KiB (BAMRecordReader.java:128-143 seeks; HipBAMRecordReader no longer copies
    the whole file for a non-local file system)."""
    import genbam
    data = np.asarray(genbam.generate(target_bytes=24 << 20, seed=11))
    h = oracle_mod.read_header(data)
    L = len(data)
    for beg, size, window in ((L // 3, 1 << 20, 1 << 20), (L // 2, 4 << 20, 256 << 10), (L - (2 << 20), 2 << 20, 1 << 20)):
        end = min(L, beg + size)
        vs, ve = oracle_mod.probabilistic_splits(data, np.array([beg], np.uint64), np.array([end], np.uint64))
        a, z = int(vs[0]), int(ve[0])
        ref = oracle_mod.read_split(data, a, z)
        rd = _CountingReader(data)
        got, nwin = _stream_read(gpu_ctx, data, a, z, h["n_ref"], window, reader=rd)
        assert_same_split(got, ref)
        assert got["payload"] == oracle_mod.record_payloads(ref)[0].tobytes()
        split_bytes = (z >> 16) - (a >> 16)
        assert rd.overlaps() == 0
        assert rd.total() <= split_bytes + window + (64 << 10), (rd.total(), split_bytes)
        assert rd.total() < L // 4


@pytest.mark.parametrize("name", ["small_pe.bam", "edge_uniform_long.bam", "edge_unsorted_l1.bam"])
def test_records_to_host_is_what_the_reader_hands_out(gpu_ctx, oracle_mod, name):
    """hbam_records_to_host (the drop-in reader's copy, BAMRecordReader.java:172-188): per window,
    key, voffset, block_size and exactly the records' bytes (rec_off into them) — equal to the
    oracle's — and nothing else: 28 B per record + the record bytes cross to the host."""
    data = _load(name)
    h = oracle_mod.read_header(data)
    ref = oracle_mod.read_split(data, h["first_voffset"], _whole(data))
    pay, off = oracle_mod.record_payloads(ref)
    got_k, got_v, got_b, recs, d2h = [], [], [], [], 0
    for w in gpu_ctx.split_stream(data, h["first_voffset"], _whole(data), h["n_ref"], window_bytes=64 << 10,
                                  host="records"):
        n = w["n"]
        got_k.append(w["key"].copy())
        got_v.append(w["voffset"].copy())
        got_b.append(w["block_size"].copy())
        u = w["ubuf"]
        assert len(u) == int(np.sum(w["block_size"].astype(np.int64) + 4)), "ubuf holds only the records"
        for i in range(n):
            r = int(w["rec_off"][i])
            recs.append(u[r:r + 4 + int(w["block_size"][i])].tobytes())
        assert w["d2h_bytes"] == 28 * n + len(u)
        d2h += w["d2h_bytes"]
        last = w
    assert last["status"] == ref["status"]
    assert np.array_equal(np.concatenate(got_k), ref["key"])
    assert np.array_equal(np.concatenate(got_v), ref["voffset"])
    assert np.array_equal(np.concatenate(got_b), ref["block_size"])
    assert b"".join(recs) == pay.tobytes()
    assert d2h == 28 * ref["n"] + len(pay)
    if name == "small_pe.bam":  # 150 bp PE records: within 1.1 x the record bytes
        assert d2h <= 1.1 * len(pay)


def test_two_readers_interleaved_on_one_context(gpu_ctx, oracle_mod):
    """Two drop-in readers sharing one context (formats.context() hands every reader of a device
    the same one), stepped alternately: each window's host copy lives in its own stream's staging
    (hbam_split_records_to_host), so a window still in use is never overwritten — or freed — by
    the other reader's next window.  Both readers' records equal the oracle's."""
    a_data, b_data = _load("small_pe.bam"), _load("edge_uniform_long.bam")
    want = {}
    for tag, data in (("a", a_data), ("b", b_data)):
        h = oracle_mod.read_header(data)
        ref = oracle_mod.read_split(data, h["first_voffset"], _whole(data))
        want[tag] = (ref, oracle_mod.record_payloads(ref)[0].tobytes(), h)
    # b's windows grow (one window, then larger ones) so its staging is re-allocated mid-way
    gens = {tag: gpu_ctx.split_stream(data, want[tag][2]["first_voffset"], _whole(data), want[tag][2]["n_ref"],
                                      window_bytes=(48 << 10) if tag == "a" else (96 << 10), host="records")
            for tag, data in (("a", a_data), ("b", b_data))}
    got = {"a": [], "b": []}
    held = {}
    live = ["a", "b"]
    while live:
        for tag in list(live):
            if tag in held:  # a reader is done with its window before it asks for the next one
                w = held.pop(tag)
                got[tag].append((w["key"].copy(), w["ubuf"][:].tobytes()))
            w = next(gens[tag], None)  # (the stream closes, and frees its staging, at the end)
            if w is None:
                live.remove(tag)
                continue
            other = "b" if tag == "a" else "a"
            if other in held:  # the other reader's window, read AFTER this reader's new window
                ow = held.pop(other)
                got[other].append((ow["key"].copy(), ow["ubuf"][:].tobytes()))
            held[tag] = w
    for tag in ("a", "b"):
        ref, pay, _ = want[tag]
        assert np.array_equal(np.concatenate([k for k, _ in got[tag]]), ref["key"]), tag
        assert b"".join(u for _, u in got[tag]) == pay, tag
    assert len(got["a"]) > 3 and len(got["b"]) > 1


def test_records_to_host_refuses_permuted_columns(gpu_ctx):
    """hbam_records_to_host copies the byte range of a decoded split's records; columns whose
    records are not back to back in index order (a permutation) are refused with HBAM_EINVAL
    instead of copying the wrong range."""
    import ctypes as C
    import torch
    from hadoop_bam import _lib
    data = _load("small_pe.bam")
    d = torch.from_numpy(data).cuda()
    h = gpu_ctx.parse_header(d)
    rc, cols = gpu_ctx.decode_split_device(d, h["first_voffset"], _whole(data), h["n_ref"])
    assert rc == 0 and cols.n_records > 10
    out = _lib.Columns()
    assert gpu_ctx.L.hbam_records_to_host(gpu_ctx.h, C.byref(cols), C.byref(out)) == 0
    n = int(cols.n_records)
    ro = torch.empty(n, dtype=torch.int64, device="cuda")
    # records 3 and 5 swapped: the first and last stay, so only the contiguity check can see it
    perm = torch.arange(n, dtype=torch.int32, device="cuda")
    perm[3], perm[5] = 5, 3
    torch.cuda.synchronize()
    assert gpu_ctx.L.hbam_permute(gpu_ctx.h, C.cast(cols.rec_off, C.c_void_p), 8, C.c_void_p(perm.data_ptr()),
                                  n, C.c_void_p(ro.data_ptr())) == 0
    torch.cuda.synchronize()
    cols.rec_off = C.cast(C.c_void_p(ro.data_ptr()), type(cols.rec_off))
    assert gpu_ctx.L.hbam_records_to_host(gpu_ctx.h, C.byref(cols), C.byref(out)) == -11
    assert "not contiguous" in gpu_ctx.last_error()


def test_windowed_decode_comp_base(gpu_ctx, oracle_mod):
    """hbam_decode_split with comp_base != 0: a window [c, c+W) of the file decodes the same
    records as the whole buffer up to the window's EMORE, whose voffset[n] is the resume point."""
    data = _load("small_pe.bam")
    h = oracle_mod.read_header(data)
    ref = oracle_mod.read_split(data, h["first_voffset"], _whole(data))
    k = len(ref["voffset"]) // 3
    v0 = int(ref["voffset"][k])
    c = v0 >> 16
    win = data[c:c + (300 << 10)]
    got = gpu_ctx.decode_split(np.ascontiguousarray(win), v0, _whole(data), n_ref=h["n_ref"],
                               comp_base=c, file_len=len(data))
    assert got["rc"] == 0
    assert got["status"] == -12  # HBAM_EMORE
    m = got["n"]
    assert m > 100
    assert np.array_equal(got["voffset"], ref["voffset"][k:k + m])
    assert np.array_equal(got["key"], ref["key"][k:k + m])


def test_guesses_across_launch_batches(oracle_mod, monkeypatch):
    """More guesses than one launch holds (HBAM_GUESS_BATCH=64 for this context): the batch
    loop's later launches give the oracle's answers too."""
    from hadoop_bam import _lib
    monkeypatch.setenv("HBAM_GUESS_BATCH", "64")
    ctx = _lib.Context(0)
    data = _load("small_pe.bam")
    h = oracle_mod.read_header(data)
    rng = np.random.default_rng(8)
    beg = rng.integers(0, len(data), 200).astype(np.int64)
    end = np.minimum(beg + rng.integers(1, 300000, 200), len(data)).astype(np.int64)
    rc, out, err = ctx.guess_batch(data, beg, end, h["n_ref"])
    assert rc == 0
    for i in range(len(beg)):
        assert (int(out[i]), int(err[i])) == oracle_mod.guess_bam_record_start(
            data, int(beg[i]), int(end[i]), h["n_ref"]), i


@pytest.mark.parametrize("label,text_fn,refs_fn,ok", __import__("helpers").CRAFTED_HEADERS,
                         ids=[c[0] for c in __import__("helpers").CRAFTED_HEADERS])
def test_header_dictionary_checks_on_device(gpu_ctx, oracle_mod, label, text_fn, refs_fn, ok):
    """hbam_parse_header (device inflate, host parse) and every n_ref = -1 decode raise
    SAMFormatException (HBAM_EFORMAT) exactly where the oracle's restatement of [htsjdk]
    BAMFileReader.readHeader does (dictionary count / name / length mismatch, empty binary name,
    @SQ without LN or with a non-integer LN) and accept the same headers with the same fields."""
    from helpers import reheader_bam
    data = reheader_bam(_load("small_pe.bam"), text_fn, refs_fn)
    want = oracle_mod.read_header(data)
    got = gpu_ctx.parse_header(data)
    assert got == want, (label, got, want)
    if ok:
        ref = oracle_mod.read_split(data, want["first_voffset"], _whole(data))
        dec = gpu_ctx.decode_split(data, want["first_voffset"], _whole(data), n_ref=-1)
        assert dec["rc"] == 0, dec
        assert_same_split(dec, ref)
    else:
        assert got == -3
        dec = gpu_ctx.decode_split(data, 0, _whole(data), n_ref=-1)
        assert dec["rc"] == -3, (label, dec.get("rc"))
