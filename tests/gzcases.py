"""GZIP page cases for k_inflate: one-column INT64 PLAIN files (tests/pqwrite.py)
whose pages are gzip members built by tests/gzcraft.py or by zlib itself.

cases() -> [(name, expected, file_bytes)], expected in "ok" / "codec" /
"size": the outcome of the library's zlib call (pq_host.cpp gzip_inflate,
oracle/pqref.c) — checked against the oracle on the CPU
(tests/test_gzip_cases.py) and against the GPU by tests/test_gpu_inflate.py.
Test infrastructure only."""
import zlib

import numpy as np

import gzcraft as gc
import pqwrite

CODEC_GZIP = 2
INT64, PLAIN = 2, 0


def _pad8(b, fill=0x55):
    return b + bytes([fill]) * ((-len(b)) % 8)


def file_of(pages):
    """pages: [(body, member)] with len(body) % 8 == 0 -> file bytes (the
    header's uncompressed size is len(body), its stored size len(member))."""
    members = iter([m for _, m in pages])
    return pqwrite.write_column([(len(b) // 8, None, b) for b, _ in pages], ptype=INT64, encoding=PLAIN,
                                codec=CODEC_GZIP, compress=lambda _b: next(members))


def zgz(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8):
    c = zlib.compressobj(level, zlib.DEFLATED, 31, mem, strategy)
    return c.compress(data) + c.flush()


def _texty(rng, n):
    words = [bytes(rng.integers(97, 123, int(k)).astype(np.uint8)) for k in rng.integers(2, 9, 400)]
    out, i = bytearray(), 0
    while len(out) < n:
        out += words[int(rng.integers(0, len(words)))] + b" "
        i += 1
    return bytes(out[:n])


def data_sets(seed=71, n=1 << 16):
    rng = np.random.default_rng(seed)
    return {
        "random": rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
        "small_ints": rng.integers(0, 50, n // 8, dtype=np.int64).tobytes(),
        "runs": np.repeat(rng.integers(0, 4, n // 64, dtype=np.int64), 8).tobytes()[:n],
        "text": _texty(rng, n),
        "zeros": bytes(n),
    }


def crafted_valid():
    """(name, body, member) for valid hand-built members."""
    out = []
    # fixed block: literals, overlapping copies (dist 1, dist 3 < len), len 258
    toks = [("lit", b) for b in b"abcdefgh"] + [("copy", 20, 1), ("copy", 17, 3), ("copy", 258, 8), ("copy", 3, 30)]
    body = gc.run_tokens(toks)
    pad = (-len(body)) % 8
    toks += [("lit", 0x41)] * pad
    body = gc.run_tokens(toks)
    w = gc.BitWriter()
    gc.fixed_block(w, toks)
    out.append(("fixed_overlap", body, gc.member(w.getvalue(), body)))
    # distance 32768 (the whole window) and 32767 after 40000 literal bytes (stored) then fixed copies
    rng = np.random.default_rng(5)
    lit = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()
    w = gc.BitWriter()
    gc.stored_block(w, lit, final=False)
    toks = [("copy", 258, 32768), ("copy", 100, 32767), ("copy", 4, 24577), ("copy", 6, 4096)]
    body = gc.run_tokens(toks, prefix=lit)
    toks += [("lit", 7)] * ((-len(body)) % 8)
    body = gc.run_tokens(toks, prefix=lit)
    gc.fixed_block(w, toks)
    out.append(("window_32k", body, gc.member(w.getvalue(), body)))
    # dynamic block with 15-bit literal/length and distance codes (past both root tables)
    lit_lens = [0] * 286
    # lengths 1..14 once, 15 twice: complete; EOB, 'a'..'n', two length symbols on the long codes
    syms = [ord("a"), 256, ord("b"), ord("c"), 257, ord("d"), ord("e"), ord("f"), ord("g"), ord("h"), ord("i"),
            ord("j"), 265, ord("k"), ord("l"), 285]
    Ls = list(range(1, 15)) + [15, 15]
    for s, L in zip(syms, Ls):
        lit_lens[s] = L
    dist_lens = [0] * 30
    for s, L in zip([0, 3, 5, 9, 12, 14, 16, 20, 23, 24, 25, 26, 27, 28, 29, 1],
                    list(range(1, 15)) + [15, 15]):
        dist_lens[s] = L
    toks = [("lit", b) for b in b"abcdefghijkl"]
    toks += [("copy", 3, 1), ("copy", 11, 4), ("copy", 258, 8), ("copy", 3, 2), ("lit", ord("l")),
             ("copy", 258, 30), ("copy", 12, 70), ("copy", 258, 300)]
    toks += [("copy", 258, 1)] * 5 + [("copy", 3, 1100)] + [("copy", 258, 2)] * 15 + [("copy", 3, 4000)]
    toks += [("copy", 258, 4)] * 100
    toks += [("copy", 3, d) for d in (24577, 16385, 12289, 8193, 6145, 4097, 129)]
    body = gc.run_tokens(toks)
    toks += [("lit", ord("k"))] * ((-len(body)) % 8)
    body = gc.run_tokens(toks)
    w = gc.BitWriter()
    gc.dynamic_block(w, toks, lit_lens, dist_lens, rle=True)
    out.append(("dynamic_long_codes", body, gc.member(w.getvalue(), body)))
    # one distance code of 1 bit (incomplete, accepted); code lengths through repeat codes 16 / 17 / 18
    toks = [("lit", b) for b in b"xyzxyzxy"] + [("copy", 9, 1), ("copy", 7, 1)]
    body = gc.run_tokens(toks)
    w = gc.BitWriter()
    gc.dynamic_block(w, toks, gc.DYN_LIT, [1], rle=True)
    out.append(("one_bit_distance_code", body, gc.member(w.getvalue(), body)))
    # no distance codes at all (literals only): an empty distance code builds
    toks = [("lit", b) for b in b"literals only!!!"]
    body = gc.run_tokens(toks)
    w = gc.BitWriter()
    gc.dynamic_block(w, toks, gc.DYN_LIT, [0] * 30)
    out.append(("empty_distance_code", body, gc.member(w.getvalue(), body)))
    # header fields: FEXTRA, FNAME, FCOMMENT, FHCRC; trailing bytes after the member
    data = data_sets()["text"][:4096]
    raw = zlib.compress(data, 6)[2:-4]
    out.append(("header_fields", data, gc.member(raw, data, flags=2 | 4 | 8 | 16, extra=b"ex" * 100, name=b"page.bin",
                                                 comment=b"c" * 300)))
    out.append(("trailing_bytes", data, gc.member(raw, data) + b"\x1f\x8bjunk-after-member"))
    # empty members: a page with no values
    out.append(("empty", b"", zgz(b"")))
    w = gc.BitWriter()
    gc.stored_block(w, b"")
    out.append(("empty_stored", b"", gc.member(w.getvalue(), b"")))
    # several blocks of each kind in one member
    w = gc.BitWriter()
    d1 = bytes(range(256)) * 4
    gc.stored_block(w, d1, final=False)
    t2 = [("lit", 1), ("copy", 100, 1), ("copy", 200, 1000)]
    gc.fixed_block(w, t2, final=False)
    t3 = [("copy", 258, 777), ("lit", 9)]
    gc.dynamic_block(w, t3, gc.DYN_LIT, gc.DYN_DIST, final=False, rle=True)
    mid = gc.run_tokens(t2 + t3, prefix=d1)
    tail = b"\x00" * ((-len(mid)) % 8 or 8)
    gc.stored_block(w, tail, final=True)
    body = mid + tail
    out.append(("mixed_blocks", body, gc.member(w.getvalue(), body)))
    return out


def crafted_errors():
    """(name, expected, body, member) for members zlib rejects."""
    out = []
    data = _pad8(b"0123456789abcdef" * 8)
    good = zgz(data)
    raw = zlib.compress(data, 6)[2:-4]
    out.append(("bad_magic", "codec", data, b"\x1f\x8c" + good[2:]))
    out.append(("bad_method", "codec", data, good[:2] + b"\x07" + good[3:]))
    out.append(("reserved_flag", "codec", data, good[:3] + b"\x20" + good[4:]))
    out.append(("short_header", "size", data, good[:7]))
    out.append(("one_byte", "size", data, good[:1]))
    out.append(("no_bytes", "size", data, b""))
    out.append(("bad_header_crc", "codec", data, gc.member(raw, data, flags=2 | 8, name=b"x", hcrc=0x1234)))
    out.append(("unterminated_name", "size", data, gc.member(b"", data, flags=8, name=b"abc", trailer=False)[:-1]))
    out.append(("short_extra", "size", data, gc.member(b"", data, flags=4, extra=b"e" * 50, trailer=False)[:-10]))
    out.append(("bad_crc", "codec", data, gc.member(raw, data, crc=zlib.crc32(data) ^ 1)))
    out.append(("bad_isize", "codec", data, gc.member(raw, data, isize=len(data) + 1)))
    out.append(("no_isize", "size", data, gc.member(raw, data)[:-4]))
    out.append(("no_trailer", "size", data, gc.member(raw, data, trailer=False)))
    out.append(("bad_crc_no_isize", "codec", data, gc.member(raw, data, crc=1)[:-4]))
    out.append(("truncated_mid", "size", data, good[: len(good) // 2]))
    out.append(("output_longer", "size", data, zgz(data + b"12345678")))
    out.append(("output_shorter", "size", data, zgz(data[:-8])))
    # block type 3
    w = gc.BitWriter()
    w.bits(1, 1)
    w.bits(3, 2)
    out.append(("block_type_3", "codec", data, gc.member(w.getvalue(), data)))
    # stored LEN / NLEN disagree; stored bytes cut short
    w = gc.BitWriter()
    gc.stored_block(w, data, nlen=5)
    out.append(("stored_nlen", "codec", data, gc.member(w.getvalue(), data)))
    w = gc.BitWriter()
    gc.stored_block(w, data)
    out.append(("stored_short", "size", data, gc.member(w.getvalue()[:-9], data, trailer=False)))
    # fixed: literal/length symbols 286 / 287, distance symbols 30 / 31
    for s in (286, 287):
        w = gc.BitWriter()
        gc.fixed_block(w, [("lit", 65), ("sym", s)])
        out.append(("fixed_sym_%d" % s, "codec", data, gc.member(w.getvalue(), data)))
    for s in (30, 31):
        w = gc.BitWriter()
        gc.fixed_block(w, [("lit", 65), ("sym", 257), ("dsym", s)])
        out.append(("fixed_dist_%d" % s, "codec", data, gc.member(w.getvalue(), data)))
    # a distance beyond the output so far
    w = gc.BitWriter()
    gc.fixed_block(w, [("lit", 65), ("lit", 66), ("copy", 5, 3)])
    out.append(("too_far", "codec", data, gc.member(w.getvalue(), data)))
    # the output full, then a copy too far back: zlib stops for room first (Z_BUF_ERROR)
    w = gc.BitWriter()
    toks = [("lit", b) for b in data] + [("copy", 5, len(data) + 10)]
    gc.fixed_block(w, toks)
    out.append(("full_then_too_far", "size", data, gc.member(w.getvalue(), data)))
    w = gc.BitWriter()
    gc.fixed_block(w, [("lit", b) for b in data] + [("lit", 1)])
    out.append(("full_then_literal", "size", data, gc.member(w.getvalue(), data)))
    # dynamic header errors
    fl = gc.DYN_LIT
    w = gc.BitWriter()
    gc.dynamic_block(w, [], fl + [8], gc.DYN_DIST, hlit=287)
    out.append(("hlit_287", "codec", data, gc.member(w.getvalue(), data)))
    w = gc.BitWriter()
    gc.dynamic_block(w, [], fl, [5] * 31, hdist=31)
    out.append(("hdist_31", "codec", data, gc.member(w.getvalue(), data)))
    cl_incomplete = [4] * 15 + [0, 0, 0, 0]
    w = gc.BitWriter()
    gc.dynamic_block(w, [], fl, gc.DYN_DIST, cl_lens=cl_incomplete, cl_syms=[])
    out.append(("cl_incomplete", "codec", data, gc.member(w.getvalue(), data)))
    cl_over = [3] * 19
    w = gc.BitWriter()
    gc.dynamic_block(w, [], fl, gc.DYN_DIST, cl_lens=cl_over, cl_syms=[])
    out.append(("cl_oversubscribed", "codec", data, gc.member(w.getvalue(), data)))
    cl = [4] * 16 + [0, 0, 0]
    cl[16], cl[15] = 4, 0  # 16 takes 15's place: still 16 codes of 4 bits
    w = gc.BitWriter()
    gc.dynamic_block(w, [], fl, gc.DYN_DIST, cl_lens=cl, cl_syms=[(16, 0)], eob=False)
    out.append(("repeat_first", "codec", data, gc.member(w.getvalue(), data, trailer=False)))
    cl = [4] * 16 + [0, 0, 0]
    cl[18], cl[15] = 4, 0
    w = gc.BitWriter()
    gc.dynamic_block(w, [], fl, gc.DYN_DIST, cl_lens=cl, cl_syms=[(8, 0)] + [(18, 127)] * 3, eob=False)
    out.append(("repeat_past_end", "codec", data, gc.member(w.getvalue(), data, trailer=False)))
    no_eob = list(fl)
    no_eob[256] = 0
    no_eob[257] = 6  # keep the code complete-ish: it is rejected before that matters
    w = gc.BitWriter()
    gc.dynamic_block(w, [], no_eob, gc.DYN_DIST, eob=False)
    out.append(("missing_eob", "codec", data, gc.member(w.getvalue(), data, trailer=False)))
    over = list(fl)
    over[0] = 1
    w = gc.BitWriter()
    gc.dynamic_block(w, [], over, gc.DYN_DIST, eob=False)
    out.append(("lit_oversubscribed", "codec", data, gc.member(w.getvalue(), data, trailer=False)))
    inc = list(fl)
    inc[0] = 0
    w = gc.BitWriter()
    gc.dynamic_block(w, [], inc, gc.DYN_DIST, eob=False)
    out.append(("lit_incomplete", "codec", data, gc.member(w.getvalue(), data, trailer=False)))
    w = gc.BitWriter()
    gc.dynamic_block(w, [], fl, gc.DYN_DIST[:-1] + [0], eob=False)
    out.append(("dist_incomplete", "codec", data, gc.member(w.getvalue(), data, trailer=False)))
    # the unused half of a 1-bit distance code
    w = gc.BitWriter()
    gc.dynamic_block(w, [("lit", 65), ("sym", 257)], fl, [1], eob=False)
    w.bits(1, 1)  # distance code '1': unused
    out.append(("dist_unused_code", "codec", data, gc.member(w.getvalue(), data, trailer=False)))
    # an empty distance code and a length symbol; and the same with the input ending there
    w = gc.BitWriter()
    gc.dynamic_block(w, [("lit", 65), ("sym", 257)], fl, [0] * 30, eob=False)
    w.bits(0, 1)
    out.append(("dist_empty_code_used", "codec", data, gc.member(w.getvalue(), data, trailer=False)))
    return out


def cases():
    res = []
    for name, d in sorted(data_sets().items()):
        for level, strat, sname in ((0, zlib.Z_DEFAULT_STRATEGY, "l0"), (1, zlib.Z_DEFAULT_STRATEGY, "l1"),
                                    (6, zlib.Z_DEFAULT_STRATEGY, "l6"), (9, zlib.Z_DEFAULT_STRATEGY, "l9"),
                                    (6, zlib.Z_FIXED, "fixed"), (6, zlib.Z_HUFFMAN_ONLY, "huff"),
                                    (6, zlib.Z_RLE, "rle"), (6, zlib.Z_FILTERED, "filtered")):
            half = len(d) // 2
            res.append(("%s_%s" % (name, sname), "ok",
                        file_of([(d[:half], zgz(d[:half], level, strat)), (d[half:], zgz(d[half:], level, strat))])))
    for name, body, m in crafted_valid():
        res.append((name, "ok", file_of([(body, m)])))
    for name, exp, body, m in crafted_errors():
        ok = _pad8(b"ok page!" * 16)
        res.append((name, exp, file_of([(ok, zgz(ok)), (body, m)])))
    return res
