"""ctypes binding for the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
`cpu_baseline` leg of bench.py as the parity checker.  The product path
(parquet-go_amd/pqgpu.py -> libpqgpu.so) never imports this module.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

BUF_VALUES, BUF_VALIDITY, BUF_LIST_OFFSETS, BUF_LIST_VALIDITY, BUF_STR_OFFSETS, BUF_DEF, BUF_REP = range(7)
CNT_LEVELS, CNT_SLOTS, CNT_ROWS, CNT_NONNULL, CNT_STR_BYTES, CNT_PAGES, CNT_VALUE_WIDTH = range(7)


class Leaf(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 512), ("physical_type", ctypes.c_int32),
                ("type_length", ctypes.c_int32), ("max_def", ctypes.c_int32),
                ("max_rep", ctypes.c_int32), ("rep_def", ctypes.c_int32),
                ("converted_type", ctypes.c_int32), ("unsigned_int", ctypes.c_int32)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so not built (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
        L.pqref_open.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(vp), ctypes.c_char_p, sz]
        L.pqref_close.argtypes = [vp]
        L.pqref_num_row_groups.argtypes = [vp]
        L.pqref_rg_num_rows.argtypes = [vp, i32]
        L.pqref_rg_num_rows.restype = i64
        L.pqref_num_rows.argtypes = [vp]
        L.pqref_num_rows.restype = i64
        L.pqref_num_leaves.argtypes = [vp]
        L.pqref_leaf_info.argtypes = [vp, i32, ctypes.POINTER(Leaf)]
        L.pqref_decode.argtypes = [vp, i32, i32, i32, ctypes.POINTER(vp)]
        L.pqref_result_free.argtypes = [vp]
        L.pqref_result_status.argtypes = [vp]
        L.pqref_result_error.argtypes = [vp]
        L.pqref_result_error.restype = ctypes.c_char_p
        L.pqref_result_count.argtypes = [vp, i32]
        L.pqref_result_count.restype = i64
        L.pqref_result_buffer.argtypes = [vp, i32, ctypes.POINTER(sz)]
        L.pqref_result_buffer.restype = vp
        L.pqref_result_error_rg.argtypes = [vp]
        L.pqref_result_error_page.argtypes = [vp]
        L.pqref_snappy_decode.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        L.pqref_unpack8_32.argtypes = [ctypes.c_char_p, i32, ctypes.POINTER(ctypes.c_int32)]
        L.pqref_unpack8_64.argtypes = [ctypes.c_char_p, i32, ctypes.POINTER(ctypes.c_int64)]
        L.pqref_hybrid_decode.argtypes = [ctypes.c_char_p, sz, i32, ctypes.POINTER(ctypes.c_int32), i64]
        L.pqref_decode_quirks.argtypes = [vp, i32, i32, i32, ctypes.POINTER(vp)]
        _LIB = L
    return _LIB


class OracleError(Exception):
    def __init__(self, code, msg, rg=-1, page=-1):
        super().__init__(f"oracle error {code}: {msg} (rg={rg}, page={page})")
        self.code, self.rg, self.page = code, rg, page


class File:
    """An opened Parquet file (pqref_open)."""

    def __init__(self, data: bytes):
        self._data = bytes(data)
        self._h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(256)
        rc = lib().pqref_open(self._data, len(self._data), ctypes.byref(self._h), err, 256)
        if rc != 0:
            raise OracleError(rc, err.value.decode())

    def close(self):
        if self._h:
            lib().pqref_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_row_groups(self):
        return lib().pqref_num_row_groups(self._h)

    @property
    def num_rows(self):
        return lib().pqref_num_rows(self._h)

    def rg_num_rows(self, rg):
        return lib().pqref_rg_num_rows(self._h, rg)

    def leaves(self):
        out = []
        for i in range(lib().pqref_num_leaves(self._h)):
            L = Leaf()
            lib().pqref_leaf_info(self._h, i, ctypes.byref(L))
            out.append({"name": L.name.decode(errors="surrogateescape"), "physical_type": L.physical_type,
                        "type_length": L.type_length, "max_def": L.max_def, "max_rep": L.max_rep,
                        "rep_def": L.rep_def, "converted_type": L.converted_type,
                        "unsigned": L.unsigned_int})
        return out

    def decode(self, leaf, rg0=0, rg1=None):
        """Return dict of numpy arrays (Arrow-style layout) or raise OracleError."""
        if rg1 is None:
            rg1 = self.num_row_groups
        r = ctypes.c_void_p()
        L = lib()
        L.pqref_decode(self._h, leaf, rg0, rg1, ctypes.byref(r))
        try:
            st = L.pqref_result_status(r)
            if st != 0:
                raise OracleError(st, L.pqref_result_error(r).decode(),
                                  L.pqref_result_error_rg(r), L.pqref_result_error_page(r))
            out = {}
            for name, cid in (("levels", CNT_LEVELS), ("slots", CNT_SLOTS), ("rows", CNT_ROWS),
                              ("non_null", CNT_NONNULL), ("str_bytes", CNT_STR_BYTES),
                              ("pages", CNT_PAGES), ("value_width", CNT_VALUE_WIDTH)):
                out[name] = L.pqref_result_count(r, cid)
            for name, bid in (("values", BUF_VALUES), ("validity", BUF_VALIDITY),
                              ("list_offsets", BUF_LIST_OFFSETS), ("list_validity", BUF_LIST_VALIDITY),
                              ("str_offsets", BUF_STR_OFFSETS), ("def", BUF_DEF), ("rep", BUF_REP)):
                n = ctypes.c_size_t()
                p = L.pqref_result_buffer(r, bid, ctypes.byref(n))
                out[name] = np.frombuffer(ctypes.string_at(p, n.value), dtype=np.uint8).copy() if n.value else np.zeros(0, np.uint8)
            return out
        finally:
            L.pqref_result_free(r)


    def decode_quirks(self, leaf, rg0=0, rg1=None):
        """ref-quirks mode (documentation only): the
        values the reference's row reader returns for a fixed-width leaf —
        'values' (one per defined level, in level order) and 'valid' (bool per
        value: not nil) — with its column store's aliasing reproduced."""
        if rg1 is None:
            rg1 = self.num_row_groups
        r = ctypes.c_void_p()
        L = lib()
        L.pqref_decode_quirks(self._h, leaf, rg0, rg1, ctypes.byref(r))
        try:
            st = L.pqref_result_status(r)
            if st != 0:
                raise OracleError(st, L.pqref_result_error(r).decode(),
                                  L.pqref_result_error_rg(r), L.pqref_result_error_page(r))
            n = L.pqref_result_count(r, CNT_NONNULL)
            sz = ctypes.c_size_t()
            p = L.pqref_result_buffer(r, BUF_VALUES, ctypes.byref(sz))
            vals = np.frombuffer(ctypes.string_at(p, sz.value), np.uint8).copy() if sz.value else np.zeros(0, np.uint8)
            p = L.pqref_result_buffer(r, BUF_VALIDITY, ctypes.byref(sz))
            bits = np.frombuffer(ctypes.string_at(p, sz.value), np.uint8) if sz.value else np.zeros(0, np.uint8)
            valid = np.unpackbits(bits, bitorder="little")[:n].astype(bool)
            return {"values": vals, "valid": valid, "nonnull": n,
                    "levels": L.pqref_result_count(r, CNT_LEVELS)}
        finally:
            L.pqref_result_free(r)


def snappy_decode(src: bytes, cap: int):
    dst = ctypes.create_string_buffer(max(cap, 1))
    n = ctypes.c_size_t()
    rc = lib().pqref_snappy_decode(src, len(src), dst, cap, ctypes.byref(n))
    return rc, dst.raw[:min(n.value, cap)], n.value


def unpack8_32(data: bytes, width: int):
    out = (ctypes.c_int32 * 8)()
    lib().pqref_unpack8_32(data + b"\0" * 8, width, out)
    return list(out)


def unpack8_64(data: bytes, width: int):
    out = (ctypes.c_int64 * 8)()
    lib().pqref_unpack8_64(data + b"\0" * 8, width, out)
    return list(out)


def hybrid_decode(src: bytes, bw: int, count: int):
    out = (ctypes.c_int32 * max(count, 1))()
    rc = lib().pqref_hybrid_decode(src, len(src), bw, out, count)
    return rc, np.frombuffer(bytes(out), dtype=np.int32)[:count].copy()
