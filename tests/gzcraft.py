"""Hand-built gzip members (RFC 1952) around hand-built DEFLATE blocks
(RFC 1951) for the k_inflate parity tests: stored, fixed and dynamic blocks
from explicit token lists and explicit code lengths, so that the tests can
reach every check of zlib's inflate — long codes, incomplete and
over-subscribed codes, invalid symbols, distances too far back, bad header
fields, bad trailers — not only what zlib's own encoder emits.

Test infrastructure only (no product code imports it)."""
import struct
import zlib

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
CL_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
FIXED_LIT = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
FIXED_DIST = [5] * 32
# complete codes for dynamic blocks (the fixed lengths over 286 / 30 symbols
# are incomplete, which zlib rejects)
DYN_LIT = [8] * 144 + [9] * 112 + [7] * 26 + [8] * 4
DYN_DIST = [5] * 28 + [4] * 2


class BitWriter:
    """DEFLATE bit order: fields from the least significant bit, Huffman
    codes from their most significant bit (RFC 1951 3.1.1)."""

    def __init__(self):
        self.acc, self.n, self.out = 0, 0, bytearray()

    def bits(self, v, k):
        self.acc |= (v & ((1 << k) - 1)) << self.n
        self.n += k
        while self.n >= 8:
            self.out.append(self.acc & 255)
            self.acc >>= 8
            self.n -= 8

    def code(self, c, length):
        rev = 0
        for i in range(length):
            rev |= ((c >> i) & 1) << (length - 1 - i)
        self.bits(rev, length)

    def align(self):
        if self.n:
            self.bits(0, 8 - self.n)

    def getvalue(self):
        self.align()
        return bytes(self.out)


def canonical(lengths):
    """symbol -> (code, length) for the lengths' canonical code (3.2.2)."""
    mx = max(lengths) if lengths else 0
    count = [0] * (mx + 2)
    for L in lengths:
        if L:
            count[L] += 1
    nxt, code = [0] * (mx + 2), 0
    for b in range(1, mx + 1):
        code = (code + count[b - 1]) << 1
        nxt[b] = code
    out = {}
    for s, L in enumerate(lengths):
        if L:
            out[s] = (nxt[L], L)
            nxt[L] += 1
    return out


def _len_sym(n):
    for i in range(28, -1, -1):
        if LBASE[i] <= n and (i < 28 or n == 258):
            return 257 + i, n - LBASE[i], LEXT[i]
    raise ValueError(n)


def _dist_sym(d):
    for i in range(29, -1, -1):
        if DBASE[i] <= d:
            return i, d - DBASE[i], DEXT[i]
    raise ValueError(d)


def run_tokens(tokens, prefix=b""):
    """The bytes a token list produces (lit / copy tokens; raw symbols are
    not interpreted)."""
    out = bytearray(prefix)
    for t in tokens:
        if t[0] == "lit":
            out.append(t[1])
        elif t[0] == "copy":
            _, n, d = t
            for _ in range(n):
                out.append(out[-d])
    return bytes(out)


def emit(w, tokens, lit, dist):
    """Write tokens with the given codes: ("lit", byte), ("copy", len, dist),
    ("sym", lit/len symbol[, extra value]) and ("dsym", distance symbol[,
    extra]) as raw symbols (invalid ones included), ("eob",)."""
    for t in tokens:
        if t[0] == "lit":
            w.code(*lit[t[1]])
        elif t[0] == "copy":
            s, x, nx = _len_sym(t[1])
            w.code(*lit[s])
            w.bits(x, nx)
            ds, dx, dnx = _dist_sym(t[2])
            w.code(*dist[ds])
            w.bits(dx, dnx)
        elif t[0] == "sym":
            w.code(*lit[t[1]])
            if len(t) > 2:
                w.bits(t[2], LEXT[t[1] - 257] if 257 <= t[1] <= 285 else 0)
        elif t[0] == "dsym":
            w.code(*dist[t[1]])
            if len(t) > 2:
                w.bits(t[2], DEXT[t[1]] if t[1] < 30 else 0)
        elif t[0] == "eob":
            w.code(*lit[256])
        else:
            raise ValueError(t)


def fixed_block(w, tokens, final=True, eob=True):
    w.bits(1 if final else 0, 1)
    w.bits(1, 2)
    emit(w, tokens + ([("eob",)] if eob else []), canonical(FIXED_LIT), canonical(FIXED_DIST))


def stored_block(w, data, final=True, nlen=None):
    w.bits(1 if final else 0, 1)
    w.bits(0, 2)
    w.align()
    n = len(data)
    w.bits(n, 16)
    w.bits((n ^ 0xFFFF) if nlen is None else nlen, 16)
    for b in data:
        w.bits(b, 8)


# a complete code-length code over all 19 symbols: 0..12 at 4 bits, 13..18 at 5
RLE_CL = [4] * 13 + [5] * 6


def rle_lengths(lens):
    """Code lengths as code-length symbols with repeats (16: previous 3-6
    times, 17: 3-10 zeros, 18: 11-138 zeros): [(symbol, extra value)]."""
    out, i = [], 0
    while i < len(lens):
        L, j = lens[i], i
        while j < len(lens) and lens[j] == L:
            j += 1
        run = j - i
        if L == 0:
            while run >= 11:
                k = min(run, 138)
                out.append((18, k - 11))
                run -= k
            while run >= 3:
                k = min(run, 10)
                out.append((17, k - 3))
                run -= k
            out += [(0, 0)] * run
        else:
            out.append((L, 0))
            run -= 1
            while run >= 3:
                k = min(run, 6)
                out.append((16, k - 3))
                run -= k
            out += [(L, 0)] * run
        i = j
    return out


def dynamic_block(w, tokens, lit_lens, dist_lens, final=True, eob=True, hlit=None, hdist=None, cl_lens=None,
                  cl_syms=None, rle=False):
    """A dynamic block whose literal/length and distance code lengths are
    given.  The code-length code is 0..15 at 4 bits each (complete) unless
    `cl_lens` (19 lengths by symbol) is given; `cl_syms` overrides the list
    of code-length symbols written ((symbol, extra value) pairs); `rle`
    writes the lengths with repeat codes (RLE_CL)."""
    if rle:
        cl_lens, cl_syms = RLE_CL, rle_lengths(list(lit_lens) + list(dist_lens))
    w.bits(1 if final else 0, 1)
    w.bits(2, 2)
    nl = len(lit_lens) if hlit is None else hlit
    nd = len(dist_lens) if hdist is None else hdist
    w.bits(nl - 257, 5)
    w.bits(nd - 1, 5)
    cl = cl_lens if cl_lens is not None else [4] * 16 + [0, 0, 0]
    w.bits(19 - 4, 4)
    for s in CL_ORDER:
        w.bits(cl[s], 3)
    clc = canonical(cl)
    syms = cl_syms if cl_syms is not None else [(L, 0) for L in list(lit_lens) + list(dist_lens)]
    for s, x in syms:
        w.code(*clc[s])
        if s == 16:
            w.bits(x, 2)
        elif s == 17:
            w.bits(x, 3)
        elif s == 18:
            w.bits(x, 7)
    emit(w, tokens + ([("eob",)] if eob else []), canonical(lit_lens), canonical(dist_lens))


def member(deflate, data, flags=0, extra=b"", name=b"", comment=b"", hcrc=None, crc=None, isize=None,
           trailer=True, magic=b"\x1f\x8b", cm=8):
    """A gzip member around raw DEFLATE bytes; `data` is what they decode to
    (for the CRC-32 / ISIZE trailer, unless overridden)."""
    h = bytearray(magic + bytes([cm, flags]) + b"\x00\x00\x00\x00\x00\x03")
    if flags & 4:
        h += struct.pack("<H", len(extra)) + extra
    if flags & 8:
        h += name + b"\x00"
    if flags & 16:
        h += comment + b"\x00"
    if flags & 2:
        h += struct.pack("<H", (zlib.crc32(bytes(h)) & 0xFFFF) if hcrc is None else hcrc)
    out = bytes(h) + deflate
    if trailer:
        out += struct.pack("<II", zlib.crc32(data) if crc is None else crc,
                           (len(data) & 0xFFFFFFFF) if isize is None else isize)
    return out


def zlib_outcome(gz, size):
    """What the library's zlib call (pq_host.cpp gzip_inflate, oracle/pqref.c)
    returns for a member and the page's uncompressed size: (code, bytes)."""
    d = zlib.decompressobj(31)
    try:
        out = d.decompress(gz, size) if size > 0 else d.decompress(gz, 1)
    except zlib.error:
        return "codec", None
    if size == 0 and out:
        return "size", None
    if not d.eof:
        return "size", None  # input ended or the output limit was reached
    if len(out) != size:
        return "size", None
    return "ok", out
