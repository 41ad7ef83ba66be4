"""GPU regression tests for the k_snappy deferred-literal fault found in round 1.

k_snappy keeps a table of long literals it defers to k_copy (one entry per
lane); a far copy whose source lies inside one reads the bytes from the
literal's payload in the input buffer, taking the payload address from that
table with v_readlane.  readlane returns an int: widened without a uint32_t
cast, a payload pointer whose low word had bit 31 set was sign-extended, and
the copy read a wrong address — only under some allocation layouts.  These
tests force the layout and run the bounds-checked build:

* PQG_DEBUG_INPUT_HIGH_WORD=1 places the batch input buffer where every
  payload address has bit 31 of its low word set;
* libpqgpu_guard.so (-DPQ_SNAP_GUARD) checks every data-dependent global
  access of k_snappy / k_copy and printf-reports instead of faulting.
"""
import io
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
import pqgpu
from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def deferred_literal_file():
    """A Snappy page that google snappy encodes as one >= 16 KiB literal (k_copy
    takes it) followed by copies whose sources lie inside that literal, more
    than the 4 KiB LDS history back (k_snappy's far-copy path)."""
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(61)
    r = rng.integers(-(1 << 62), 1 << 62, 2500, dtype=np.int64)  # 20000 incompressible bytes
    z = np.zeros(500, np.int64)  # a compressible run resets the encoder's skip, so the repeats below are found
    # google snappy: literal [0, 20696), then copies of 64 / 62 bytes from offsets 802 / 866 (23200 back)
    vals = np.concatenate([r, z, r[100:116], z[:40], r[1500:1540], z[:40], r[600:608], rng.integers(0, 3, 200)])
    t = pa.table({"v": pa.array(vals)}, schema=pa.schema([pa.field("v", pa.int64(), nullable=False)]))
    buf = io.BytesIO()
    pq.write_table(t, buf, compression="snappy", use_dictionary=False, row_group_size=len(vals))
    return buf.getvalue()


def _check(data, ctx):
    from test_gpu_parity import check_file
    check_file(data, ctx)


def test_deferred_literal_payload_high_low_word():
    """Far copies into a deferred literal with every payload address's low
    word >= 0x80000000: bit-exact against the oracle (the round-1 fault
    returned wrong bytes or faulted here)."""
    data = deferred_literal_file()
    os.environ["PQG_DEBUG_INPUT_HIGH_WORD"] = "1"
    try:
        _check(data, "deferred literal, high low word")
        # (c2_dict_bw12's last row group goes to k_expand_wg, whose records'
        # run-table pointers are widened from lane words: the run tables are
        # shifted to high-low-word addresses by the same knob)
        for name in ("c3_delta_v2", "c4_list_str", "plain_strings", "c2_dict_bw16", "c2_dict_bw12"):
            _check(open(os.path.join(GOLDEN, name + ".parquet"), "rb").read(), name + " high low word")
    finally:
        del os.environ["PQG_DEBUG_INPUT_HIGH_WORD"]
    _check(data, "deferred literal")


@pytest.mark.parametrize("family", ["k_dba", "k_plain_str", "k_sw"])
def test_string_kernels_high_low_word(family):
    """The high-low-word input layout (every page address's low word has bit
    31 set) through one file per string kernel family: k_dba (DELTA_BYTE_ARRAY
    values rebuilt in order), k_plain_str (flat required PLAIN string pages in
    items) and k_sw_regions / _link / _emit (the region-parallel length walk of
    >= 64 KiB PLAIN pages and string dictionaries).  Bit-exact against the
    oracle, as with the ordinary layout."""
    from test_gpu_parity import _pq_bytes, _plain_string_cases
    rng = np.random.default_rng(62)
    if family == "k_dba":
        files = [("delta_strings", open(os.path.join(GOLDEN, "delta_strings.parquet"), "rb").read())]
        pa = pytest.importorskip("pyarrow")
        words = ["prefix_%06d_%s" % (i // 3, "x" * int(k)) for i, k in enumerate(rng.integers(0, 40, 30000))]
        t = pa.table({"s": pa.array(words)})
        files.append(("dba generated", _pq_bytes(t, compression="snappy", use_dictionary=False,
                                                 column_encoding={"s": "DELTA_BYTE_ARRAY"})))
    else:
        cases = _plain_string_cases(rng)
        t = cases["text"]
        if family == "k_plain_str":  # flat required PLAIN pages, Snappy and not
            files = [("text %s" % c, _pq_bytes(t, compression=c, use_dictionary=False, data_page_size=1 << 20,
                                               row_group_size=40000)) for c in ("none", "snappy")]
        else:  # nullable long pages and a >= 64 KiB string dictionary: the region walk
            files = [("blob nullable", _pq_bytes(cases["blob_nullable"], compression="snappy", use_dictionary=False,
                                                 data_page_size=1 << 20, row_group_size=40000)),
                     ("text dictionary", _pq_bytes(t, compression="none", use_dictionary=True,
                                                   dictionary_pagesize_limit=1 << 30, data_page_size=1 << 20,
                                                   row_group_size=40000))]
    os.environ["PQG_DEBUG_INPUT_HIGH_WORD"] = "1"
    try:
        for name, data in files:
            _check(data, "%s %s high low word" % (family, name))
    finally:
        del os.environ["PQG_DEBUG_INPUT_HIGH_WORD"]


_GUARD_SCRIPT = r"""
import glob, os, sys
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "oracle")]
import pqgpu
assert os.path.basename(pqgpu._LIB_PATH) == "libpqgpu_guard.so", pqgpu._LIB_PATH
from test_gpu_parity import check_file
from test_gpu_guard import deferred_literal_file
files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.parquet")))
for f in files:
    check_file(open(f, "rb").read(), os.path.basename(f))
check_file(deferred_literal_file(), "deferred literal")
os.environ["PQG_DEBUG_INPUT_HIGH_WORD"] = "1"
check_file(deferred_literal_file(), "deferred literal, high low word")
print("GUARD_OK %d" % (len(files) + 2), flush=True)
"""


@pytest.mark.timeout(300)
def test_guard_build_golden_set():
    """The bounds-checked build (libpqgpu_guard.so, PQ_SNAP_GUARD) over every
    golden fixture and the deferred-literal file: parity holds and no guard
    fires (device printf lines SNAP_GUARD / PQ_CHK)."""
    lib = os.path.join(ROOT, "parquet-go_amd", "libpqgpu_guard.so")
    if not os.path.exists(lib):
        pytest.fail("libpqgpu_guard.so is not built (make -C parquet-go_amd/csrc)")
    env = dict(os.environ, PQGPU_LIB="libpqgpu_guard.so")
    p = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + _GUARD_SCRIPT], env=env, cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=280)
    out = p.stdout.decode(errors="replace")
    assert p.returncode == 0, out[-4000:]
    assert "GUARD_OK" in out, out[-4000:]
    assert "SNAP_GUARD" not in out and "PQ_CHK" not in out, out[-4000:]
