"""ref-quirks mode of the oracle (documentation only).

The parity contract is per page: levels and the first notNull
values of every page, decoded against the right dictionary.  The reference's
row reader returns something else on multi-page chunks; these tests pin the
oracle's model of it (oracle.File.decode_quirks) on hand-built files:
  D1  a page's null slots are appended to the column store, so a 2-page
      nullable chunk's second page is shifted by the first page's null count
      (chunk_reader.go:383-398, data_store.go:169-173, type_dict.go:114-121);
  D2  from the second row group on, the dictionary page decodes into the
      store's reused array and the first data page's append overwrites it
      (chunk_reader.go:234-235, page_dict.go:50-53, type_dict.go:74, :397).
CPU only."""
import struct

import numpy as np

import oracle
import pqwrite


def _i32(vals):
    return struct.pack("<%di" % len(vals), *vals)


def test_d1_two_page_nullable_chunk_row_shift():
    # page 1: 10 levels, 3 nulls; page 2: 10 levels, all defined (PLAIN INT32)
    d1 = [1, 0, 1, 1, 0, 1, 1, 0, 1, 1]
    v1 = [11, 12, 13, 14, 15, 16, 17]
    d2 = [1] * 10
    v2 = list(range(100, 110))
    data = pqwrite.write_column([(10, d1, _i32(v1)), (10, d2, _i32(v2))], ptype=1, encoding=0, optional=True)
    f = oracle.File(data)
    right = f.decode(0)
    dense = right["values"].view(np.int32)[np.unpackbits(right["validity"], bitorder="little")[:20].astype(bool)]
    assert list(dense) == v1 + v2  # the page-level contract (what the GPU returns)
    q = f.decode_quirks(0)
    assert q["nonnull"] == 17 and q["levels"] == 20
    got = q["values"].view(np.int32)
    # the store holds [v1 (7), nil x 3, v2 (10)]: the 17 defined levels take its
    # first 17 slots -> page 1's values, 3 nils, page 2 shifted by 3
    assert list(q["valid"]) == [True] * 7 + [False] * 3 + [True] * 7
    assert list(got[:7]) == v1
    assert list(got[10:]) == v2[:7]


def _dict_page(vals):
    return _i32(vals)


def _keys(keys, bw=2):
    # RLE_DICTIONARY values section: bit width byte + one bit-packed run
    return bytes([bw]) + pqwrite.hybrid_bitpacked(keys, bw)


def test_d2_dictionary_overwritten_from_second_row_group():
    k1 = [3, 2, 1, 0, 3, 3, 3, 3]
    k2 = [0, 1, 2, 3, 1, 0, 2, 1]
    rg = lambda dvals: {"dict_page": _dict_page(dvals), "dict_count": 4,
                        "pages": [(8, None, _keys(k1)), (8, None, _keys(k2))]}
    dict0, dict1 = [10, 20, 30, 40], [100, 200, 300, 400]
    data = pqwrite.write_row_groups([rg(dict0), rg(dict1)], ptype=1, encoding=8)
    f = oracle.File(data)
    assert f.num_row_groups == 2
    right = f.decode(0).copy()
    want = [dict0[k] for k in k1 + k2] + [dict1[k] for k in k1 + k2]
    assert list(right["values"].view(np.int32)) == want  # the page-level contract
    q = f.decode_quirks(0)
    got = list(q["values"].view(np.int32))
    assert q["valid"].all()
    # row group 0: a fresh store, the right dictionary
    assert got[:16] == want[:16]
    # row group 1: page 1 reads the right dictionary, then its append writes
    # its 8 values over the store's first slots, where the dictionary lives:
    # page 2 looks its keys up in page 1's values
    p1 = [dict1[k] for k in k1]
    assert got[16:24] == p1
    assert got[24:32] == [p1[k] for k in k2]
    assert got[24:32] != want[24:32]
    # one row group alone: no aliasing, the right values
    q1 = f.decode_quirks(0, 1, 2)
    assert list(q1["values"].view(np.int32)) == want[16:]


def test_quirks_equal_page_contract_without_nulls_or_reuse():
    data = pqwrite.write_column([(6, None, _i32([1, 2, 3, 4, 5, 6]))], ptype=1, encoding=0)
    f = oracle.File(data)
    q = f.decode_quirks(0)
    assert list(q["values"].view(np.int32)) == [1, 2, 3, 4, 5, 6] and q["valid"].all()
