"""A minimal Parquet writer for test fixtures (test infrastructure only).

Writes one row group of INT32 leaves from explicit def / rep level arrays and
dense values: V1 data pages, PLAIN values, RLE/bit-packed hybrid levels (one
bit-packed run), uncompressed.  It exists so that the reference's own Dremel
level vectors (tests/golden/kat_levels.json, from data_store_test.go) can be
fed to both decoders exactly as the reference's column store holds them; the
schema uses the raw repeated groups those tests build (no LIST wrapping
unless the test asks for it).  Thrift compact protocol, field ids from
parquet/parquet.thrift.
"""
import struct

T_BOOL_TRUE, T_BYTE, T_I32, T_I64, T_BINARY, T_LIST, T_STRUCT = 1, 3, 5, 6, 8, 9, 12


def _uvar(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _zz(x):
    return _uvar((x << 1) ^ (x >> 63))


class _S:
    """Compact-protocol struct builder: fields must be added in increasing id."""

    def __init__(self):
        self.b = bytearray()
        self.last = 0

    def _h(self, fid, t):
        d = fid - self.last
        assert 0 < d <= 15
        self.b.append((d << 4) | t)
        self.last = fid

    def i32(self, fid, v):
        self._h(fid, T_I32)
        self.b += _zz(v)
        return self

    def i64(self, fid, v):
        self._h(fid, T_I64)
        self.b += _zz(v)
        return self

    def str(self, fid, s):
        self._h(fid, T_BINARY)
        s = s.encode() if isinstance(s, str) else s
        self.b += _uvar(len(s)) + s
        return self

    def struct(self, fid, st):
        self._h(fid, T_STRUCT)
        self.b += st.done()
        return self

    def list(self, fid, etype, items):
        self._h(fid, T_LIST)
        n = len(items)
        self.b += bytes([(n << 4) | etype]) if n < 15 else bytes([0xF0 | etype]) + _uvar(n)
        for it in items:
            if etype == T_I32:
                self.b += _zz(it)
            elif etype == T_BINARY:
                s = it.encode()
                self.b += _uvar(len(s)) + s
            else:
                self.b += it.done()
        return self

    def done(self):
        return bytes(self.b) + b"\x00"


def bit_len(v):
    return int(v).bit_length()


def hybrid_bitpacked(vals, bw):
    """One bit-packed run (hybrid_decoder.go:133-141 reads it back), zero padded to 8."""
    n = len(vals)
    groups = (n + 7) // 8
    acc, nb, out = 0, 0, bytearray()
    for v in list(vals) + [0] * (groups * 8 - n):
        acc |= int(v) << nb
        nb += bw
        while nb >= 8:
            out.append(acc & 0xFF)
            acc >>= 8
            nb -= 8
    return _uvar((groups << 1) | 1) + bytes(out)


def write(schema, columns):
    """schema: [{"path", "repetition" (0 req / 1 opt / 2 rep), "kind": "group"|"int32"}]
    in depth-first order; columns: {leaf path: {"def", "rep", "values"}}.
    Returns the file bytes."""
    # tree
    children = {"": []}
    for e in schema:
        parent = e["path"].rsplit(".", 1)[0] if "." in e["path"] else ""
        children.setdefault(parent, []).append(e)
        children.setdefault(e["path"], [])
    elems = [_S().str(4, "schema").i32(5, len(children[""]))]
    leaves = []

    def walk(e, d, r):
        d += e["repetition"] != 0
        r += e["repetition"] == 2
        s = _S()
        if e["kind"] == "int32":
            s.i32(1, 1)
        s.i32(3, e["repetition"]).str(4, e["path"].rsplit(".", 1)[-1])
        if e["kind"] == "group":
            s.i32(5, len(children[e["path"]]))
        elems.append(s)
        if e["kind"] == "group":
            for c in children[e["path"]]:
                walk(c, d, r)
        else:
            leaves.append((e["path"], d, r))

    for e in children[""]:
        walk(e, 0, 0)
    out = bytearray(b"PAR1")
    chunks = []
    num_rows = None
    for path, maxd, maxr in leaves:
        c = columns[path]
        dl, rl, vals = c["def"], c["rep"], c["values"]
        n = len(dl)
        rows = sum(1 for x in rl if x == 0) if maxr else n
        num_rows = rows if num_rows is None else num_rows
        body = bytearray()
        if maxr > 0:
            s = hybrid_bitpacked(rl, bit_len(maxr))
            body += struct.pack("<I", len(s)) + s
        if maxd > 0:
            s = hybrid_bitpacked(dl, bit_len(maxd))
            body += struct.pack("<I", len(s)) + s
        body += struct.pack("<%di" % len(vals), *vals)
        dph = _S().i32(1, n).i32(2, 0).i32(3, 3).i32(4, 3)
        ph = _S().i32(1, 0).i32(2, len(body)).i32(3, len(body)).struct(5, dph).done()
        off = len(out)
        out += ph + body
        meta = (_S().i32(1, 1).list(2, T_I32, [0, 3]).list(3, T_BINARY, path.split(".")).i32(4, 0).i64(5, n)
                .i64(6, len(ph) + len(body)).i64(7, len(ph) + len(body)).i64(9, off))
        chunks.append(_S().i64(2, off).struct(3, meta))
    rg = _S().list(1, T_STRUCT, chunks).i64(2, len(out) - 4).i64(3, num_rows or 0)
    fmd = _S().i32(1, 1).list(2, T_STRUCT, elems).i64(3, num_rows or 0).list(4, T_STRUCT, [rg]).done()
    out += fmd + struct.pack("<i", len(fmd)) + b"PAR1"
    return bytes(out)


def write_column(pages, ptype=1, encoding=5, optional=False, type_length=0, dict_page=None, dict_count=0,
                 codec=0, compress=None):
    """One leaf `v` (parquet.Type `ptype`, REQUIRED or OPTIONAL), one row group,
    V1 data pages whose values sections are given as bytes:
    pages = [(num_values, def_levels or None, values_section_bytes)].  With
    `optional`, def levels go in front of each values section as one
    bit-packed hybrid run (bit width 1).  `codec` (parquet.CompressionCodec)
    names the chunk's codec and `compress(page_body) -> bytes` writes each data
    page's stored bytes (default: uncompressed).  Returns the file bytes."""
    elems = [_S().str(4, "schema").i32(5, 1)]
    leaf = _S().i32(1, ptype)
    if type_length:
        leaf.i32(2, type_length)
    leaf.i32(3, 1 if optional else 0).str(4, "v")
    elems.append(leaf)
    out = bytearray(b"PAR1")
    first = len(out)
    dict_off = None
    if dict_page is not None:
        dph = _S().i32(1, dict_count).i32(2, 0)
        ph = _S().i32(1, 2).i32(2, len(dict_page)).i32(3, len(dict_page)).struct(7, dph).done()
        dict_off = len(out)
        out += ph + dict_page
    data_off = len(out)
    n_total = 0
    for n, dl, body in pages:
        b = bytearray()
        if optional:
            s = hybrid_bitpacked(dl, 1)
            b += struct.pack("<I", len(s)) + s
        b += body
        dph = _S().i32(1, n).i32(2, encoding).i32(3, 3).i32(4, 3)
        stored = compress(bytes(b)) if compress else bytes(b)
        out += _S().i32(1, 0).i32(2, len(b)).i32(3, len(stored)).struct(5, dph).done() + stored
        n_total += n
    size = len(out) - first
    meta = (_S().i32(1, ptype).list(2, T_I32, [0, 3, encoding]).list(3, T_BINARY, ["v"]).i32(4, codec).i64(5, n_total)
            .i64(6, size).i64(7, size).i64(9, data_off))
    if dict_off is not None:
        meta.i64(11, dict_off)
    chunk = _S().i64(2, first).struct(3, meta)
    rg = _S().list(1, T_STRUCT, [chunk]).i64(2, size).i64(3, n_total)
    fmd = _S().i32(1, 1).list(2, T_STRUCT, elems).i64(3, n_total).list(4, T_STRUCT, [rg]).done()
    out += fmd + struct.pack("<i", len(fmd)) + b"PAR1"
    return bytes(out)


def write_row_groups(row_groups, ptype=1, encoding=8, optional=False, dict_offset_field=True):
    """One leaf `v` (parquet.Type `ptype`), several row groups, V1
    uncompressed pages: row_groups = [{"pages": [(num_values, def_levels or
    None, values_section_bytes)], "dict_page": bytes or None, "dict_count":
    n}].  Values sections are given as they are stored (for RLE_DICTIONARY:
    the bit-width byte and the hybrid key stream).  Without
    `dict_offset_field` the chunk metadata leaves dictionary_page_offset unset
    and data_page_offset points at the dictionary page (as some writers do).
    Returns the file bytes."""
    elems = [_S().str(4, "schema").i32(5, 1), _S().i32(1, ptype).i32(3, 1 if optional else 0).str(4, "v")]
    out = bytearray(b"PAR1")
    rgs = []
    total = 0
    for g in row_groups:
        first = len(out)
        dict_off = None
        if g.get("dict_page") is not None:
            dp = g["dict_page"]
            dph = _S().i32(1, g["dict_count"]).i32(2, 0)
            ph = _S().i32(1, 2).i32(2, len(dp)).i32(3, len(dp)).struct(7, dph).done()
            dict_off = len(out)
            out += ph + dp
        data_off = len(out)
        n_rg = 0
        for n, dl, body in g["pages"]:
            b = bytearray()
            if optional:
                s_ = hybrid_bitpacked(dl, 1)
                b += struct.pack("<I", len(s_)) + s_
            b += body
            dph = _S().i32(1, n).i32(2, encoding).i32(3, 3).i32(4, 3)
            out += _S().i32(1, 0).i32(2, len(b)).i32(3, len(b)).struct(5, dph).done() + b
            n_rg += n
        size = len(out) - first
        if dict_off is not None and not dict_offset_field:
            data_off, dict_off = dict_off, None
        meta = (_S().i32(1, ptype).list(2, T_I32, [0, 3, encoding]).list(3, T_BINARY, ["v"]).i32(4, 0).i64(5, n_rg)
                .i64(6, size).i64(7, size).i64(9, data_off))
        if dict_off is not None:
            meta.i64(11, dict_off)
        chunk = _S().i64(2, first).struct(3, meta)
        rgs.append(_S().list(1, T_STRUCT, [chunk]).i64(2, size).i64(3, n_rg))
        total += n_rg
    fmd = _S().i32(1, 1).list(2, T_STRUCT, elems).i64(3, total).list(4, T_STRUCT, rgs).done()
    out += fmd + struct.pack("<i", len(fmd)) + b"PAR1"
    return bytes(out)
