"""Test-side restatement of the list structure of a column with max_rep >= 2
(what k_nest_count / k_nest_write build, pq_nest.hip; contract in
include/pqgpu.h pqg_batch_column_nest) from its rep / def levels, with
numpy: per level k the offsets and validity of the level-k lists, then the
leaf slots' validity.  `rdefs[k-1]` is the def level of the k-th repeated
ancestor (schema.go:800-806 increments).  Test infrastructure only."""
import numpy as np


def nest_from_levels(defs, reps, rdefs, max_def):
    d = np.asarray(defs, np.int64)
    r = np.asarray(reps, np.int64)
    R = len(rdefs)
    f = [r == 0] + [(r <= k) & (d >= rdefs[k - 1]) for k in range(1, R + 1)]
    out = []
    for k in range(1, R + 1):
        starts = np.nonzero(f[k - 1])[0]
        cum = np.concatenate([[0], np.cumsum(f[k])])
        offs = np.concatenate([cum[starts], [cum[-1]]]).astype(np.int32)
        valid = d[starts] >= rdefs[k - 1] - 1
        out.append({"offsets": offs, "validity": np.packbits(valid, bitorder="little"), "count": len(starts)})
    slots = np.nonzero(f[R])[0]
    out.append({"validity": np.packbits(d[slots] == max_def, bitorder="little"), "count": len(slots)})
    return out


def nest_from_arrow(arr, depth):
    """The same structure read off a pyarrow nested ListArray (depth list
    levels): offsets rebased to 0, validity bitmaps, leaf slots."""
    out = []
    a = arr
    for _ in range(depth):
        offs = np.asarray(a.offsets, np.int64)
        valid = np.asarray(a.is_valid())
        out.append({"offsets": (offs - offs[0]).astype(np.int32),
                    "validity": np.packbits(valid, bitorder="little"), "count": len(a)})
        a = a.values.slice(int(offs[0]), int(offs[-1] - offs[0]))
    out.append({"validity": np.packbits(np.asarray(a.is_valid()), bitorder="little"), "count": len(a)})
    return out


def nested_tables(rng, rows=3000):
    """(name, table, depth, rdefs, max_def) cases: nulls and empty lists at
    every level, optional and required outer lists, 2 and 3 levels."""
    import pyarrow as pa

    def lst(depth, leaf_type, null_p=0.1, empty_p=0.1):
        if depth == 0:
            v = int(rng.integers(-1000, 1000))
            return None if rng.random() < null_p else (v if leaf_type == "int" else str(v))
        u = rng.random()
        if u < null_p:
            return None
        if u < null_p + empty_p:
            return []
        return [lst(depth - 1, leaf_type, null_p, empty_p) for _ in range(int(rng.integers(1, 5)))]
    out = []
    t2 = pa.list_(pa.list_(pa.int64()))
    out.append(("list2_int64", pa.table({"a": pa.array([lst(2, "int") for _ in range(rows)], type=t2)}), 2, [2, 4], 5))
    rq = [lst(2, "int") for _ in range(rows)]
    rq = [x if x is not None else [] for x in rq]
    out.append(("list2_required_outer",
                pa.table({"a": pa.array(rq, type=t2)},
                         schema=pa.schema([pa.field("a", t2, nullable=False)])), 2, [1, 3], 4))
    t3 = pa.list_(pa.list_(pa.list_(pa.int32())))
    out.append(("list3_int32", pa.table({"a": pa.array([lst(3, "int", 0.15, 0.1) for _ in range(rows)], type=t3)}),
                3, [2, 4, 6], 7))
    ts = pa.list_(pa.list_(pa.string()))
    out.append(("list2_string", pa.table({"a": pa.array([lst(2, "str") for _ in range(rows)], type=ts)}), 2,
                [2, 4], 5))
    return out
