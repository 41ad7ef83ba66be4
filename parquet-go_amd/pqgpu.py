"""pqgpu — Python mirror of parquet-go's read surface over libpqgpu.so.

Names follow the reference (module github.com/fraugster/parquet-go):

    NewFileReader(source, *columns)      file_reader.go:27
    FileReader.RowGroupCount/NumRows/RowGroupNumRows/CurrentRowGroup/SkipRowGroup/PreLoad
                                         file_reader.go:60-134
    FileReader.Columns / GetColumnByName schema.go:960-983
    RegisterBlockCompressor(codec, fn)   compress.go:130-135
    GetRegisteredBlockCompressors()      compress.go:139-150
    DecompressBlock(codec, data, n)      compress.go:90-122

Decoding runs on the GPU through the C ABI (include/pqgpu.h); there is no CPU
fallback: every decode entry point raises if libpqgpu.so or a HIP device is
missing.  Results come back as Arrow-style numpy buffers (values spaced over
slots with nulls zeroed, LSB-first validity bitmaps, list offsets, string
offsets) instead of the reference's map[string]interface{} rows.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PQGPU_LIB selects another in-tree build of the same ABI (the guarded build
# libpqgpu_guard.so in tests/test_gpu_guard.py); default: libpqgpu.so
_LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ.get("PQGPU_LIB", "libpqgpu.so")))
_LIB = None
_LOCK = threading.Lock()

# status codes (include/pqgpu.h)
OK, ERR_ARG, ERR_FORMAT, ERR_THRIFT, ERR_SCHEMA, ERR_CODEC, ERR_ENCODING, ERR_SNAPPY, ERR_SIZE, ERR_PAGE, \
    ERR_EOF, ERR_RLE, ERR_DICT_INDEX, ERR_DELTA, ERR_BYTE_ARRAY, ERR_BITWIDTH, ERR_NO_DICT, ERR_DEVICE, \
    ERR_COUNT, ERR_UNSUPPORTED = range(20)
STATUS_NAMES = ["OK", "ARG", "FORMAT", "THRIFT", "SCHEMA", "CODEC", "ENCODING", "SNAPPY", "SIZE", "PAGE", "EOF",
                "RLE", "DICT_INDEX", "DELTA", "BYTE_ARRAY", "BITWIDTH", "NO_DICT", "DEVICE", "COUNT", "UNSUPPORTED"]

# parquet.CompressionCodec
CompressionCodec_UNCOMPRESSED, CompressionCodec_SNAPPY, CompressionCodec_GZIP, CompressionCodec_LZO, \
    CompressionCodec_BROTLI, CompressionCodec_LZ4, CompressionCodec_ZSTD = range(7)
# parquet.Type
Type_BOOLEAN, Type_INT32, Type_INT64, Type_INT96, Type_FLOAT, Type_DOUBLE, Type_BYTE_ARRAY, \
    Type_FIXED_LEN_BYTE_ARRAY = range(8)

# include/pqgpu.h PQGPU_ABI_VERSION this mirror's structs and signatures follow
ABI_VERSION = 2

BUF_VALUES, BUF_VALIDITY, BUF_LIST_OFFSETS, BUF_LIST_VALIDITY, BUF_STR_OFFSETS, BUF_DEF, BUF_REP = range(7)
BATCH_LEVELS = 1
BATCH_HOST_INFLATE = 2

# every symbol include/pqgpu.h declares (checked by tests/test_capi_symbols.py)
EXPORTS = [
    "pqg_abi_version", "pqg_device_count", "pqg_last_error", "pqg_ctx_create", "pqg_ctx_destroy", "pqg_ctx_stream",
    "pqg_register_block_compressor", "pqg_get_registered_codecs", "pqg_decompress_block",
    "pqg_file_open_path", "pqg_file_open_buffer", "pqg_file_close", "pqg_file_num_rows",
    "pqg_file_row_group_count", "pqg_file_row_group_num_rows", "pqg_file_row_group_byte_size",
    "pqg_file_row_group_cost", "pqg_batch_stream",
    "pqg_file_column_count", "pqg_file_column_info", "pqg_file_find_column", "pqg_file_select_columns",
    "pqg_file_last_error", "pqg_batch_create", "pqg_batch_decode", "pqg_batch_sync",
    "pqg_batch_error_location", "pqg_batch_row_groups", "pqg_batch_column", "pqg_batch_copy", "pqg_batch_column_nest", "pqg_batch_copy_nest", "pqg_batch_stats_get",
    "pqg_batch_kernel_times", "pqg_batch_set_timing", "pqg_batch_destroy",
    "pqg_stream_open", "pqg_stream_next", "pqg_stream_close", "pqg_file_open_many", "pqg_release_cache",
]


class PqgError(Exception):
    def __init__(self, code, msg="", location=None):
        name = STATUS_NAMES[code] if 0 <= code < len(STATUS_NAMES) else str(code)
        super().__init__("pqgpu %s (%d): %s" % (name, code, msg))
        self.code = code
        self.location = location


class ColumnInfo(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 512), ("physical_type", ctypes.c_int32), ("type_length", ctypes.c_int32),
                ("max_def", ctypes.c_int32), ("max_rep", ctypes.c_int32), ("rep_def", ctypes.c_int32),
                ("converted_type", ctypes.c_int32), ("unsigned_int", ctypes.c_int32),
                ("value_width", ctypes.c_int32)]

    def as_dict(self):
        return {f: (getattr(self, f).decode(errors="surrogateescape") if f == "name" else getattr(self, f)) for f, _ in self._fields_}


class ColumnView(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("validity", ctypes.c_void_p), ("list_offsets", ctypes.c_void_p),
                ("list_validity", ctypes.c_void_p), ("str_offsets", ctypes.c_void_p),
                ("def_levels", ctypes.c_void_p), ("rep_levels", ctypes.c_void_p), ("levels", ctypes.c_int64),
                ("slots", ctypes.c_int64), ("rows", ctypes.c_int64), ("str_bytes", ctypes.c_int64),
                ("non_null", ctypes.c_int64), ("value_width", ctypes.c_int32), ("leaf", ctypes.c_int32)]


class BatchStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("pages", "data_pages", "dict_pages", "snappy_pages",
                                              "host_inflated_pages", "input_bytes", "staged_bytes",
                                              "output_bytes", "h2d_bytes", "snappy_in_bytes", "dict_bytes")] + \
        [(n, ctypes.c_double) for n in ("create_plan_ms", "create_alloc_ms", "create_upload_ms", "create_tables_ms",
                                        "upload_gather_ms", "upload_wait_ms")] + \
        [(n, ctypes.c_int64) for n in ("gzip_device_pages", "gzip_in_bytes")]


DECOMPRESS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t,
                                 ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t))


def lib():
    """Load libpqgpu.so (built in-tree by __graft_entry__.build() / make)."""
    global _LIB
    with _LOCK:
        if _LIB is None:
            if not os.path.exists(_LIB_PATH):
                raise RuntimeError("%s is not built (run `make -C parquet-go_amd/csrc`)" % os.path.basename(_LIB_PATH))
            L = ctypes.CDLL(_LIB_PATH)
            vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
            P = ctypes.POINTER
            sig = {
                "pqg_abi_version": (i32, []), "pqg_device_count": (i32, []),
                "pqg_last_error": (i32, [vp, ctypes.c_char_p, sz]),
                "pqg_ctx_create": (i32, [i32, P(vp)]), "pqg_ctx_destroy": (None, [vp]),
                "pqg_ctx_stream": (vp, [vp]),
                "pqg_register_block_compressor": (i32, [i32, DECOMPRESS_FN, vp]),
                "pqg_get_registered_codecs": (i32, [P(ctypes.c_int), i32]),
                "pqg_decompress_block": (i32, [vp, i32, ctypes.c_char_p, sz, ctypes.c_char_p, sz, sz, P(sz)]),
                "pqg_file_open_path": (i32, [ctypes.c_char_p, P(vp)]),
                "pqg_file_open_buffer": (i32, [ctypes.c_char_p, sz, i32, P(vp)]),
                "pqg_file_close": (None, [vp]), "pqg_file_num_rows": (i64, [vp]),
                "pqg_file_row_group_count": (i32, [vp]), "pqg_file_row_group_num_rows": (i64, [vp, i32]),
                "pqg_file_row_group_byte_size": (i64, [vp, i32]),
                "pqg_file_row_group_cost": (ctypes.c_double, [vp, i32]),
                "pqg_batch_stream": (vp, [vp]),
                "pqg_file_column_count": (i32, [vp]), "pqg_file_column_info": (i32, [vp, i32, P(ColumnInfo)]),
                "pqg_file_find_column": (i32, [vp, ctypes.c_char_p]),
                "pqg_file_select_columns": (i32, [vp, P(ctypes.c_char_p), i32, P(ctypes.c_int), i32]),
                "pqg_file_last_error": (i32, [vp, ctypes.c_char_p, sz]),
                "pqg_batch_create": (i32, [vp, vp, i32, i32, P(ctypes.c_int), i32, i32, P(vp)]),
                "pqg_batch_decode": (i32, [vp]), "pqg_batch_sync": (i32, [vp]),
                "pqg_batch_error_location": (i32, [vp, P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_int)]),
                "pqg_batch_row_groups": (i32, [vp, P(ctypes.c_int), P(ctypes.c_int)]),
                "pqg_batch_column": (i32, [vp, i32, P(ColumnView)]),
                "pqg_batch_copy": (i32, [vp, i32, i32, vp, sz, P(sz)]),
                "pqg_batch_column_nest": (i32, [vp, i32, i32, P(vp), P(vp), P(ctypes.c_int64)]),
                "pqg_batch_copy_nest": (i32, [vp, i32, i32, i32, vp, sz, P(sz)]),
                "pqg_batch_stats_get": (i32, [vp, P(BatchStats), sz]),
                "pqg_batch_kernel_times": (i32, [vp, P(ctypes.c_char_p), P(ctypes.c_float), i32]),
                "pqg_batch_set_timing": (i32, [vp, i32]),
                "pqg_batch_destroy": (None, [vp]),
                "pqg_stream_open": (i32, [vp, vp, i32, i32, P(ctypes.c_int), i32, i32, i32, i32, P(vp)]),
                "pqg_stream_next": (i32, [vp, P(vp), P(ctypes.c_int)]),
                "pqg_stream_close": (None, [vp]),
                "pqg_file_open_many": (i32, [P(ctypes.c_char_p), i32, i32, P(vp), P(ctypes.c_int)]),
                "pqg_release_cache": (i32, [i32]),
            }
            for name, (res, args) in sig.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if L.pqg_abi_version() != ABI_VERSION:
                raise RuntimeError("%s has ABI version %d, this module follows %d (rebuild the library)"
                                   % (os.path.basename(_LIB_PATH), L.pqg_abi_version(), ABI_VERSION))
            _LIB = L
        return _LIB


def last_error():
    buf = ctypes.create_string_buffer(512)
    lib().pqg_last_error(None, buf, 512)
    return buf.value.decode(errors="replace")


def _check(rc, what=""):
    if rc != OK:
        raise PqgError(rc, (what + ": " if what else "") + last_error())


def device_count():
    return lib().pqg_device_count()


def release_cache(device=-1):
    """Free the idle device buffers the library keeps for reuse (pqg_release_cache)."""
    _check(lib().pqg_release_cache(int(device)), "pqg_release_cache")


class Context:
    """One per GPU (the C ABI's pqg_ctx)."""

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        _check(lib().pqg_ctx_create(device, ctypes.byref(self._h)), "pqg_ctx_create")
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().pqg_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}


def default_context(device=0):
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


# ---------------------------------------------------------------------------
# codec registry (compress.go)
# ---------------------------------------------------------------------------
_registered_callbacks = {}


def RegisterBlockCompressor(codec, decompress):
    """Register a host decompressor `decompress(bytes) -> bytes` for `codec`
    (compress.go:130).  `None` restores the built-in for UNCOMPRESSED/SNAPPY/GZIP."""
    if decompress is None:
        _check(lib().pqg_register_block_compressor(codec, DECOMPRESS_FN(), None))
        _registered_callbacks.pop(codec, None)
        return

    def _cb(user, src, n, dst, cap, out_len):
        try:
            out = decompress(ctypes.string_at(src, n))
        except Exception:
            return ERR_CODEC
        if len(out) > cap:
            out_len[0] = len(out)
            return ERR_SIZE
        ctypes.memmove(dst, out, len(out))
        out_len[0] = len(out)
        return OK

    cfn = DECOMPRESS_FN(_cb)
    _registered_callbacks[codec] = cfn  # keep alive
    _check(lib().pqg_register_block_compressor(codec, cfn, None))


def GetRegisteredBlockCompressors():
    n = lib().pqg_get_registered_codecs(None, 0)
    arr = (ctypes.c_int * max(n, 1))()
    lib().pqg_get_registered_codecs(arr, n)
    return sorted(arr[i] for i in range(n))


def DecompressBlock(codec, data, uncompressed_size, ctx=None):
    """decompressBlock + newBlockReader size check (compress.go:90-122)."""
    out = ctypes.create_string_buffer(max(uncompressed_size, 1))
    n = ctypes.c_size_t()
    c = ctx.handle if ctx is not None else (default_context().handle if codec == CompressionCodec_SNAPPY else None)
    _check(lib().pqg_decompress_block(c, codec, bytes(data), len(data), out, uncompressed_size,
                                      uncompressed_size, ctypes.byref(n)), "DecompressBlock")
    return out.raw[:n.value]


# ---------------------------------------------------------------------------
# file + batches
# ---------------------------------------------------------------------------
class Batch:
    """Every page of row groups [rg0, rg1) of the selected leaves, planned into
    one descriptor table, uploaded once; decode() reruns the GPU pipeline."""

    def __init__(self, reader, rg0, rg1, leaves, flags=0, ctx=None):
        self.reader = reader
        self.ctx = ctx or reader.ctx
        self.leaves = list(leaves)
        self._h = ctypes.c_void_p()
        arr = (ctypes.c_int * max(len(self.leaves), 1))(*self.leaves)
        _check(lib().pqg_batch_create(self.ctx.handle, reader.handle, rg0, rg1, arr, len(self.leaves), flags,
                                      ctypes.byref(self._h)), "pqg_batch_create")

    def decode(self):
        _check(lib().pqg_batch_decode(self._h), "pqg_batch_decode")

    def sync(self, raise_on_error=True):
        rc = lib().pqg_batch_sync(self._h)
        if rc != OK and raise_on_error:
            rg, leaf, page = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            lib().pqg_batch_error_location(self._h, ctypes.byref(rg), ctypes.byref(leaf), ctypes.byref(page))
            raise PqgError(rc, last_error(), (rg.value, leaf.value, page.value))
        return rc

    def view(self, i):
        v = ColumnView()
        _check(lib().pqg_batch_column(self._h, i, ctypes.byref(v)))
        return v

    def copy(self, i, buf):
        n = ctypes.c_size_t()
        _check(lib().pqg_batch_copy(self._h, i, buf, None, 0, ctypes.byref(n)))
        out = np.empty(n.value, np.uint8)
        if n.value:
            _check(lib().pqg_batch_copy(self._h, i, buf, out.ctypes.data, n.value, ctypes.byref(n)))
        return out

    def nest(self, i):
        """Selected column i with max_rep >= 2: the list structure
        (pqg_batch_column_nest) as host arrays — for each repetition level k
        = 1..max_rep {"offsets": int32[count + 1], "validity": uint8 bitmap,
        "count": lists}, then the leaf slots {"validity", "count"}."""
        out = []
        k = 1
        while True:
            cnt = ctypes.c_int64()
            rc = lib().pqg_batch_column_nest(self._h, i, k, None, None, ctypes.byref(cnt))
            if rc == 1 and k > 1:  # PQG_ERR_ARG: past the leaf slots
                break
            _check(rc, "pqg_batch_column_nest")
            lvl = {"count": cnt.value}
            for what, name in ((0, "offsets"), (1, "validity")):
                n = ctypes.c_size_t()
                _check(lib().pqg_batch_copy_nest(self._h, i, k, what, None, 0, ctypes.byref(n)))
                a = np.empty(n.value, np.uint8)
                if n.value:
                    _check(lib().pqg_batch_copy_nest(self._h, i, k, what, a.ctypes.data, n.value, ctypes.byref(n)))
                lvl[name] = a.view(np.int32) if what == 0 else a
            out.append(lvl)
            k += 1
        return out

    def column(self, i):
        """Host copy of selected column i in the canonical layout."""
        v = self.view(i)
        out = {"levels": v.levels, "slots": v.slots, "rows": v.rows, "str_bytes": v.str_bytes,
               "value_width": v.value_width, "leaf": v.leaf}
        for name, b in (("values", BUF_VALUES), ("validity", BUF_VALIDITY), ("list_offsets", BUF_LIST_OFFSETS),
                        ("list_validity", BUF_LIST_VALIDITY), ("str_offsets", BUF_STR_OFFSETS),
                        ("def", BUF_DEF), ("rep", BUF_REP)):
            out[name] = self.copy(i, b)
        return out

    def stats(self):
        s = BatchStats()
        _check(lib().pqg_batch_stats_get(self._h, ctypes.byref(s), ctypes.sizeof(s)))
        return {f: getattr(s, f) for f, _ in s._fields_}

    def set_timing(self, every):
        """Record the timing events on every `every`-th decode (0: never)."""
        _check(lib().pqg_batch_set_timing(self._h, int(every)), "pqg_batch_set_timing")

    def kernel_times(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        n = lib().pqg_batch_kernel_times(self._h, names, ms, 16)
        return {names[i].decode(): ms[i] for i in range(n)}

    def close(self):
        if self._h:
            lib().pqg_batch_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


STREAM_RAMP = 1 << 8  # pqg_stream_open: the first two slices a quarter / half of rgs_per_slice (pqgpu.h)


class _SliceBatch(Batch):
    """A slice handed out by a Stream: the stream owns (and frees) its handle."""

    def __init__(self, reader, handle, rg0, leaves, ctx):
        self.reader, self.ctx, self.leaves, self.rg0 = reader, ctx, list(leaves), rg0
        self._h = ctypes.c_void_p(handle)
        lo, hi = ctypes.c_int(), ctypes.c_int()
        _check(lib().pqg_batch_row_groups(self._h, ctypes.byref(lo), ctypes.byref(hi)), "pqg_batch_row_groups")
        self.rg1 = hi.value  # the slice is row groups [rg0, rg1)

    def close(self):
        self._h = ctypes.c_void_p()


class Stream:
    """Row groups [rg0, rg1) in slices of `rgs_per_slice`, pipelined: the next
    slice is planned and uploaded by a host worker while the current one
    decodes (pqg_stream_*; file_reader.go:101-116 row-group iteration).
    Iterating yields each slice's batch with its decode launched; a yielded
    batch is valid until the next one is requested."""

    def __init__(self, reader, rg0, rg1, leaves, rgs_per_slice=1, depth=2, flags=0, ctx=None):
        self.reader = reader
        self.ctx = ctx or reader.ctx
        self.leaves = list(leaves)
        self._h = ctypes.c_void_p()
        arr = (ctypes.c_int * max(len(self.leaves), 1))(*self.leaves)
        _check(lib().pqg_stream_open(self.ctx.handle, reader.handle, rg0, rg1, arr, len(self.leaves), flags,
                                     rgs_per_slice, depth, ctypes.byref(self._h)), "pqg_stream_open")

    def __iter__(self):
        return self

    def __next__(self):
        if not self._h:
            raise StopIteration
        b, rg = ctypes.c_void_p(), ctypes.c_int()
        _check(lib().pqg_stream_next(self._h, ctypes.byref(b), ctypes.byref(rg)), "pqg_stream_next")
        if not b.value:
            self.close()
            raise StopIteration
        return _SliceBatch(self.reader, b.value, rg.value, self.leaves, self.ctx)

    def close(self):
        if self._h:
            lib().pqg_stream_close(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FileReader:
    """NewFileReader(r, columns...) (file_reader.go:27) backed by the GPU decoder."""

    def __init__(self, source, *columns, ctx=None, device=0):
        self._h = ctypes.c_void_p()
        self._buf = None
        if isinstance(source, (bytes, bytearray, memoryview)):
            self._buf = bytes(source)
            _check(lib().pqg_file_open_buffer(self._buf, len(self._buf), 0, ctypes.byref(self._h)), "NewFileReader")
        else:
            _check(lib().pqg_file_open_path(os.fsencode(source), ctypes.byref(self._h)), "NewFileReader")
        self._ctx = ctx
        self._device = device
        self.selected = self._select(columns)
        self.row_group_position = 0

    @property
    def handle(self):
        return self._h

    @property
    def ctx(self):
        if self._ctx is None:
            self._ctx = default_context(self._device)
        return self._ctx

    def _select(self, names):
        n = lib().pqg_file_column_count(self._h)
        arr = (ctypes.c_int * max(n, 1))()
        cn = (ctypes.c_char_p * max(len(names), 1))(*[os.fsencode(x) for x in names])
        k = lib().pqg_file_select_columns(self._h, cn, len(names), arr, n)
        return [arr[i] for i in range(min(k, n))]

    # --- metadata accessors (file_reader.go:60-134) ---
    def RowGroupCount(self):
        return lib().pqg_file_row_group_count(self._h)

    def NumRows(self):
        return lib().pqg_file_num_rows(self._h)

    def RowGroupNumRows(self, rg=None):
        return lib().pqg_file_row_group_num_rows(self._h, self.row_group_position if rg is None else rg)

    def RowGroupByteSize(self, rg):
        """Σ total_uncompressed_size of the row group's chunks (the shard balancing weight)."""
        return lib().pqg_file_row_group_byte_size(self._h, rg)

    def RowGroupCost(self, rg):
        """Estimated GPU decode cost of row group rg (pqg_file_row_group_cost):
        the weight plan_row_group_shards balances for multi-GPU shards."""
        return lib().pqg_file_row_group_cost(self._h, rg)

    def CurrentRowGroup(self):
        return self.row_group_position

    def SkipRowGroup(self):
        self.row_group_position += 1

    def Columns(self):
        out = []
        for i in range(lib().pqg_file_column_count(self._h)):
            ci = ColumnInfo()
            lib().pqg_file_column_info(self._h, i, ctypes.byref(ci))
            out.append(ci.as_dict())
        return out

    def GetColumnByName(self, name):
        i = lib().pqg_file_find_column(self._h, os.fsencode(name))
        return None if i < 0 else self.Columns()[i]

    # --- decode ---
    def batch(self, rg0=0, rg1=None, leaves=None, flags=0):
        rg1 = self.RowGroupCount() if rg1 is None else rg1
        return Batch(self, rg0, rg1, self.selected if leaves is None else leaves, flags)

    def stream(self, rg0=0, rg1=None, rgs_per_slice=1, leaves=None, depth=2, flags=0):
        """Pipelined decode of row groups [rg0, rg1) slice by slice (Stream;
        flags | STREAM_RAMP: the first two slices smaller, each slice's range
        is its batch's rg0 / rg1)."""
        rg1 = self.RowGroupCount() if rg1 is None else rg1
        return Stream(self, rg0, rg1, self.selected if leaves is None else leaves, rgs_per_slice, depth, flags)

    def read_row_groups(self, rg0=0, rg1=None, leaves=None, levels=False):
        """Decode row groups [rg0, rg1) on the GPU; returns {flat_name: buffers}."""
        b = self.batch(rg0, rg1, leaves, BATCH_LEVELS if levels else 0)
        try:
            b.decode()
            b.sync()
            cols = self.Columns()
            return {cols[leaf]["name"]: b.column(i) for i, leaf in enumerate(b.leaves)}
        finally:
            b.close()

    def PreLoad(self):
        """Decode the current row group (file_reader.go:116)."""
        return self.read_row_groups(self.row_group_position, self.row_group_position + 1)

    def close(self):
        if self._h:
            lib().pqg_file_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def NewFileReader(source, *columns, **kw):
    return FileReader(source, *columns, **kw)


def OpenFiles(paths, *columns, threads=0, **kw):
    """FileReaders for many files, their footers parsed in parallel by the
    library (pqg_file_open_many).  Raises on the first file that fails."""
    n = len(paths)
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    hs = (ctypes.c_void_p * max(n, 1))()
    failed = ctypes.c_int(-1)
    rc = lib().pqg_file_open_many(arr, n, int(threads), hs, ctypes.byref(failed))
    if rc != OK:
        for i in range(n):
            if hs[i]:
                lib().pqg_file_close(hs[i])
        raise PqgError(rc, last_error())
    out = []
    for i in range(n):
        r = FileReader.__new__(FileReader)
        r._h = ctypes.c_void_p(hs[i])
        r._buf = None
        r._ctx = kw.get("ctx")
        r._device = kw.get("device", 0)
        r.selected = r._select(columns)
        r.row_group_position = 0
        out.append(r)
    return out


def plan_row_group_shards(sizes, world):
    """Contiguous row-group ranges [(rg0, rg1)] for `world` ranks, balanced by
    the weights `sizes` (one per row group: FileReader.RowGroupCost, the
    estimated decode cost, or byte sizes).  Row groups are independent
    (one dictionary per chunk, chunk_reader.go:221), so a shard needs nothing
    from its neighbours and the decode path has no collective."""
    n = len(sizes)
    total = float(sum(sizes))
    out, rg = [], 0
    acc = 0.0
    for r in range(world):
        rg0 = rg
        if r == world - 1:
            rg = n
        else:
            target = total * (r + 1) / world
            # at least one row group per rank while any remain for the ranks after
            while rg < n - (world - 1 - r) and (rg == rg0 or acc + sizes[rg] / 2.0 <= target):
                acc += sizes[rg]
                rg += 1
        out.append((rg0, rg))
    return out
