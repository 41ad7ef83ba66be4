"""DELTA_BINARY_PACKED streams in any block / miniblock layout (test
infrastructure only).

`encode` lays a value sequence out the way the reference's decoder reads it
(deltabp_decoder.go:14-334), including layouts no conformant writer emits:
miniblocks whose value count is not a multiple of 8 (the reader takes 8
values a group and starts a miniblock only where the position is a multiple
of both 8 and the miniblock size, :121-136) and any number of miniblocks per
block (:52-112).  `read` is a model of that reader (values, the position it
leaves the stream at, or the error class) used to check the encoder and to
place the bytes that follow a length stream (DELTA_LENGTH_BYTE_ARRAY).
"""
import math


def uvar(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def zz(x, bits=64):
    return uvar(((x << 1) ^ (x >> (bits - 1))) & ((1 << bits) - 1))


def _pack(vals, w):
    acc, nb, out = 0, 0, bytearray()
    for v in vals:
        acc |= int(v) << nb
        nb += w
        while nb >= 8:
            out.append(acc & 0xFF)
            acc >>= 8
            nb -= 8
    assert nb == 0
    return bytes(out)


def encode(values, block_size, mb_count, bits=64, rng=None, total=None, pad_widths=True):
    """values: python ints (the decoded sequence); returns the stream bytes.
    Widths of miniblocks after the data are random when `rng` is given (the
    reference skips them at the width of the current one, D5)."""
    mask = (1 << bits) - 1
    n = len(values)
    total = n if total is None else total
    mbvc = block_size // mb_count
    L = mbvc * 8 // math.gcd(8, mbvc)  # values per miniblock as read (lcm(8, mbvc))
    first = values[0] if n else 0
    out = bytearray(uvar(block_size) + uvar(mb_count) + uvar(total) + zz(first, bits))
    # the reader consumes deltas 0 .. n-1 (one lookahead), in groups of 8
    ngroups = (n + 7) // 8 if n else 0
    npos = ngroups * 8
    deltas = [((values[j + 1] - values[j]) & mask) if j + 1 < n else None for j in range(npos)]
    nint = (npos + L - 1) // L if npos else 0
    nblocks = max(1, (nint + mb_count - 1) // mb_count)
    pos = 0
    last = None
    for blk in range(nblocks):
        ivs = range(blk * mb_count, min(nint, (blk + 1) * mb_count))
        real = [deltas[p] for k in ivs for p in range(k * L, min((k + 1) * L, npos)) if deltas[p] is not None]
        signed = [d - (1 << bits) if d >> (bits - 1) else d for d in real]
        md = min(signed) if signed else 0
        widths = []
        for k in range(blk * mb_count, (blk + 1) * mb_count):
            if k < nint:
                ds = [((deltas[p] - md) & mask) for p in range(k * L, min((k + 1) * L, npos)) if deltas[p] is not None]
                widths.append(max([d.bit_length() for d in ds] + [0]))
            else:
                widths.append(int(rng.integers(0, bits + 1)) if (rng is not None and pad_widths) else 0)
        out += zz(md, bits) + bytes(widths)
        for k in ivs:
            w = widths[k - blk * mb_count]
            for g in range(k * L, min((k + 1) * L, npos), 8):
                grp = [((deltas[p] - md) & mask) if deltas[p] is not None else 0 for p in range(g, g + 8)]
                out += _pack(grp, w)
            last = (k, w, blk, widths)
    return bytes(out)


def pad_tail(stream, reader_end):
    """Zero bytes up to the reader's end position (the padding it skips)."""
    return stream + b"\x00" * max(0, reader_end - len(stream))


class DeltaError(Exception):
    def __init__(self, kind):
        super().__init__(kind)
        self.kind = kind


def _unpack(buf, w, bits):
    acc = int.from_bytes(buf, "little")
    return [(acc >> (w * i)) & ((1 << w) - 1) for i in range(8)]


def read(buf, pos, count, bits=64):
    """The reference reader (init + `count` next() calls): returns (values,
    end position).  Raises DeltaError("EOF" | "DELTA" | "BITWIDTH")."""
    mask = (1 << bits) - 1

    def ruvar():
        nonlocal pos
        x = s = 0
        while True:
            if pos >= len(buf):
                raise DeltaError("EOF")
            b = buf[pos]
            pos += 1
            x |= (b & 0x7F) << s
            s += 7
            if b < 0x80:
                return x

    def rzz():
        u = ruvar()
        return (u >> 1) ^ -(u & 1)

    def full(k):
        nonlocal pos
        if pos + k > len(buf):
            raise DeltaError("EOF")
        b = buf[pos:pos + k]
        pos += k
        return b

    bs = ruvar()
    m = ruvar()
    if m <= 0 or bs % m:
        raise DeltaError("DELTA")
    mbvc = bs // m
    if mbvc == 0:
        raise DeltaError("DELTA")
    vc = ruvar()
    prev = rzz()
    st = {"md": 0, "widths": b"", "cur": 0}

    def header():
        st["md"] = rzz()
        st["widths"] = full(m)
        if any(w > bits for w in st["widths"]):
            raise DeltaError("BITWIDTH")
        st["cur"] = 0

    header()
    out = []
    position = 0
    w = 0
    mbpos = 0
    group = [0] * 8
    for _ in range(count):
        if position >= vc:
            raise DeltaError("EOF")
        if position % 8 == 0:
            if position % mbvc == 0:
                if st["cur"] >= m:
                    header()
                w = st["widths"][st["cur"]]
                mbpos = 0
                st["cur"] += 1
            group = _unpack(full(w), w, bits) if w else [0] * 8
            mbpos += w
            if position + 8 >= vc:
                sl = (mbvc // 8) * w - mbpos
                if sl < 0:
                    raise DeltaError("DELTA")
                pos = min(len(buf), pos + sl)
                for _i in range(st["cur"], m):
                    w2 = st["widths"][st["cur"]]
                    if w2:
                        pos = min(len(buf), pos + (mbvc // 8) * w2)
        out.append(prev)
        prev = (prev + group[position % 8] + st["md"]) & mask
        if prev >> (bits - 1):
            prev -= 1 << bits
        position += 1
    return out, pos
