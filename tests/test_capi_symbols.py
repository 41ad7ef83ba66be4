"""CPU tests of the C ABI boundary: libpqgpu.so loads, exports every symbol
include/pqgpu.h declares, agrees with the oracle on error numbering, and its
host planner (footer / schema parse) agrees with the oracle.  No compute calls."""
import ctypes
import json
import os
import re
import subprocess

import pytest

import oracle
import pqgpu
from conftest import GOLDEN, ROOT, golden_bytes


def header_functions():
    src = open(os.path.join(ROOT, "include", "pqgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pqg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_exactly_the_exports():
    declared = header_functions()
    assert declared == sorted(pqgpu.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = pqgpu.lib()
    for name in header_functions():
        assert hasattr(L, name), name
    assert L.pqg_abi_version() == pqgpu.ABI_VERSION == 2


def test_status_numbering_matches_oracle():
    hdr = open(os.path.join(ROOT, "include", "pqgpu.h")).read()
    ora = open(os.path.join(ROOT, "oracle", "pqref.h")).read()
    a = dict((k, int(v)) for k, v in re.findall(r"PQG_ERR_([A-Z_]+) = (\d+)", hdr))
    b = dict((k, int(v)) for k, v in re.findall(r"PQR_ERR_([A-Z_]+) = (\d+)", ora))
    assert a == b and len(a) == 19
    assert [pqgpu.STATUS_NAMES[v] for v in sorted(a.values())] == [k if k != "DICT_INDEX" else "DICT_INDEX" for k, _ in sorted(a.items(), key=lambda kv: kv[1])]


def test_codec_registry_defaults_and_registration():
    assert pqgpu.GetRegisteredBlockCompressors()[:3] == [0, 1, 2]
    pqgpu.RegisterBlockCompressor(pqgpu.CompressionCodec_ZSTD, lambda b: b[::-1])
    try:
        assert pqgpu.CompressionCodec_ZSTD in pqgpu.GetRegisteredBlockCompressors()
        # host codecs need no GPU
        assert pqgpu.DecompressBlock(pqgpu.CompressionCodec_ZSTD, b"abc", 3) == b"cba"
        with pytest.raises(pqgpu.PqgError) as ei:
            pqgpu.DecompressBlock(pqgpu.CompressionCodec_ZSTD, b"abc", 4)
        assert ei.value.code == pqgpu.ERR_SIZE
    finally:
        pqgpu.RegisterBlockCompressor(pqgpu.CompressionCodec_ZSTD, None)
    assert pqgpu.CompressionCodec_ZSTD not in pqgpu.GetRegisteredBlockCompressors()
    assert pqgpu.DecompressBlock(pqgpu.CompressionCodec_UNCOMPRESSED, b"xyz", 3) == b"xyz"
    with pytest.raises(pqgpu.PqgError) as ei:
        pqgpu.DecompressBlock(pqgpu.CompressionCodec_LZ4, b"xyz", 3)
    assert ei.value.code == pqgpu.ERR_CODEC


def test_gzip_host_codec():
    import gzip
    data = os.urandom(1000) + b"a" * 5000
    assert pqgpu.DecompressBlock(pqgpu.CompressionCodec_GZIP, gzip.compress(data), len(data)) == data


@pytest.mark.parametrize("name", sorted(json.load(open(os.path.join(GOLDEN, "manifest.json")))))
def test_host_metadata_matches_oracle(name):
    data = golden_bytes(name + ".parquet")
    r = pqgpu.FileReader(data)
    o = oracle.File(data)
    assert r.RowGroupCount() == o.num_row_groups
    assert r.NumRows() == o.num_rows
    for rg in range(o.num_row_groups):
        assert r.RowGroupNumRows(rg) == o.rg_num_rows(rg)
    lo, lr = o.leaves(), r.Columns()
    assert len(lo) == len(lr)
    for a, b in zip(lo, lr):
        for k in ("name", "physical_type", "type_length", "max_def", "max_rep", "rep_def", "converted_type"):
            assert a[k] == b[k], (k, a, b)
        assert a["unsigned"] == b["unsigned_int"]


def test_column_selection_prefix():
    r = pqgpu.FileReader(golden_bytes("c4_list_str.parquet"), "l")
    assert r.selected == [0]
    r = pqgpu.FileReader(golden_bytes("c4_list_str.parquet"), "l.list.element", "s")
    assert r.selected == [0, 1]
    r = pqgpu.FileReader(golden_bytes("c4_list_str.parquet"), "l.lis")
    assert r.selected == []


@pytest.mark.parametrize("blob", [b"", b"PAR1", b"PAR1" + b"\0" * 8 + b"PAR1", b"PAR1\x05\x00\x00\x00\x15\x15PAR1",
                                  b"XXXX" + b"\0" * 20 + b"PAR1"])
def test_malformed_files_error_not_crash(blob):
    with pytest.raises(pqgpu.PqgError):
        pqgpu.FileReader(blob)


def test_open_many_footers_in_parallel(tmp_path):
    """pqg_file_open_many: every golden file's footer parsed by a thread pool
    agrees with the single-file open; a bad file reports its index."""
    names = sorted(json.load(open(os.path.join(GOLDEN, "manifest.json"))))[:12]
    paths = [os.path.join(GOLDEN, n + ".parquet") for n in names]
    readers = pqgpu.OpenFiles(paths, threads=4)
    for p, r in zip(paths, readers):
        one = pqgpu.FileReader(p)
        assert r.NumRows() == one.NumRows() and r.RowGroupCount() == one.RowGroupCount()
        assert r.Columns() == one.Columns()
        one.close()
        r.close()
    bad = tmp_path / "bad.parquet"
    bad.write_bytes(b"PAR1" + b"\0" * 20 + b"PAR1")
    with pytest.raises(pqgpu.PqgError):
        pqgpu.OpenFiles(paths[:2] + [str(bad)])


def _c_layout(tmp_path, structs):
    """sizeof / offsetof of each (struct, [fields]) as the C compiler lays them
    out from include/pqgpu.h (a probe compiled with gcc, the reference's cgo
    toolchain would see the same)."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pqgpu.h"', "int main(void) {"]
    for st, fields in structs:
        lines.append('printf("%s sizeof %%zu\\n", sizeof(%s));' % (st, st))
        for f in fields:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (st, f, st, f))
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                           "-o", str(exe)])
    out = {}
    for ln in subprocess.check_output([str(exe)]).decode().split("\n"):
        if ln:
            st, f, v = ln.split()
            out[(st, f)] = int(v)
    return out


@pytest.mark.parametrize("cname,pyname", [("pqg_batch_stats", "BatchStats"), ("pqg_column_view", "ColumnView"),
                                          ("pqg_column_info", "ColumnInfo")])
def test_struct_layout_matches_ctypes_mirror(tmp_path, cname, pyname):
    """The header's structs and pqgpu.py's ctypes mirrors agree field by field
    (offsets) and in size, so neither side reads or writes past the other."""
    cls = getattr(pqgpu, pyname)
    fields = [f for f, _ in cls._fields_]
    lay = _c_layout(tmp_path, [(cname, fields)])
    assert lay[(cname, "sizeof")] == ctypes.sizeof(cls)
    for f in fields:
        assert lay[(cname, f)] == getattr(cls, f).offset, (cname, f)


def test_stats_get_argument_contract():
    """pqg_batch_stats_get(b, out, size) (ABI 2): a null batch or a size short
    of the version-1 prefix (the eleven int64 counters) is PQG_ERR_ARG.  The
    prefix rule on a real batch: tests/test_gpu_parity.py
    test_stats_get_old_caller_size."""
    L = pqgpu.lib()
    s = pqgpu.BatchStats()
    assert L.pqg_batch_stats_get(None, ctypes.byref(s), ctypes.sizeof(s)) == pqgpu.ERR_ARG
    assert pqgpu.BatchStats.create_plan_ms.offset == 11 * 8
