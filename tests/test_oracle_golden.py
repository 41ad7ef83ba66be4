"""CPU tests: the oracle (oracle/pqref.c) against the reference's own KAT
tables and against the committed pyarrow golden fixtures."""
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, golden_bytes

KEYS = ("values", "validity", "list_offsets", "list_validity", "str_offsets")


def test_bitpack_kat_int32():
    kat = json.load(open(os.path.join(GOLDEN, "kat_bitpack.json")))
    assert len(kat["int32"]) > 100
    for v in kat["int32"]:
        got = oracle.unpack8_32(bytes.fromhex(v["data"]), v["width"])
        want = [int(np.int32(np.uint32(x & 0xffffffff))) for x in v["values"]]
        assert got == want, v


def test_bitpack_kat_int64():
    kat = json.load(open(os.path.join(GOLDEN, "kat_bitpack.json")))
    assert len(kat["int64"]) > 300
    for v in kat["int64"]:
        got = oracle.unpack8_64(bytes.fromhex(v["data"]), v["width"])
        want = [int(np.int64(np.uint64(x & 0xffffffffffffffff))) for x in v["values"]]
        assert got == want, v


def compare(out, exp, key, max_def):
    for k in KEYS:
        ek = "%s_%s" % (key, k)
        if ek not in exp:
            continue
        if k == "validity" and max_def == 0:
            continue
        want = exp[ek].view(np.uint8).ravel()
        assert np.array_equal(out[k], want), (key, k, out[k].size, want.size)


def fixture_cases():
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    for name, e in sorted(man.items()):
        for key, c in sorted(e["columns"].items()):
            yield name, e["file"], key, c


@pytest.mark.parametrize("name,file,key,col", list(fixture_cases()))
def test_oracle_matches_golden(name, file, key, col):
    f = oracle.File(golden_bytes(file))
    leaf = col["leaf"]
    if "error" in col:
        with pytest.raises(oracle.OracleError) as ei:
            f.decode(leaf)
        assert ei.value.code == col["error"], col["why"]
        return
    out = f.decode(leaf)
    exp = np.load(os.path.join(GOLDEN, name + ".npz"))
    compare(out, exp, key, f.leaves()[leaf]["max_def"])


def test_hybrid_edge_cases():
    # bit width 0: infinite zeros, reads nothing (hybrid_decoder.go:84-86)
    rc, v = oracle.hybrid_decode(b"", 0, 5)
    assert rc == 0 and list(v) == [0] * 5
    # RLE run of 3 x value 5 at bw 3, then EOF
    rc, v = oracle.hybrid_decode(bytes([3 << 1, 5]), 3, 3)
    assert rc == 0 and list(v) == [5, 5, 5]
    rc, _ = oracle.hybrid_decode(bytes([3 << 1, 5]), 3, 4)
    assert rc == oracle_status("EOF")
    # RLE value wider than bw -> error (hybrid_decoder.go:127-129)
    rc, _ = oracle.hybrid_decode(bytes([3 << 1, 9]), 3, 1)
    assert rc == oracle_status("RLE")
    # empty runs are errors (:154-161)
    assert oracle.hybrid_decode(bytes([0]), 3, 1)[0] == oracle_status("RLE")
    assert oracle.hybrid_decode(bytes([1]), 3, 1)[0] == oracle_status("RLE")
    # short bit-packed group is zero-filled (:133-141): 1 group, bw 8, only 3 bytes present
    rc, v = oracle.hybrid_decode(bytes([3, 7, 8, 9]), 8, 8)
    assert rc == 0 and list(v) == [7, 8, 9, 0, 0, 0, 0, 0]
    # a group starting past the end is EOF
    assert oracle.hybrid_decode(bytes([5, 1, 2, 3, 4, 5, 6, 7, 8]), 8, 9)[0] == oracle_status("EOF")


def oracle_status(name):
    names = ["OK", "ARG", "FORMAT", "THRIFT", "SCHEMA", "CODEC", "ENCODING", "SNAPPY", "SIZE", "PAGE", "EOF",
             "RLE", "DICT_INDEX", "DELTA", "BYTE_ARRAY", "BITWIDTH", "NO_DICT", "DEVICE", "COUNT", "UNSUPPORTED"]
    return names.index(name)


def test_snappy_oracle_roundtrip():
    # raw snappy blocks produced by pyarrow's snappy codec (independent encoder)
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(0)
    for n in (0, 1, 63, 64, 65, 1000, 70000):
        for kind in ("rand", "rep"):
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes() if kind == "rand" else \
                (b"abcdefgh12" * (n // 10 + 1))[:n]
            comp = pa.compress(data, codec="snappy", asbytes=True)
            rc, out, _ = oracle.snappy_decode(comp, n)
            assert rc == 0 and out == data
    # corrupt inputs: offset 0, offset beyond output, truncated literal
    assert oracle.snappy_decode(bytes([4, 0b01, 0]), 4)[0] == oracle_status("SNAPPY")
    assert oracle.snappy_decode(bytes([4, 0x0c, 1, 2, 3]), 4)[0] == oracle_status("SNAPPY")
