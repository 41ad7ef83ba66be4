"""Transcribe the reference's own test vectors for the read path into data
fixtures.  Run in the build container, where
/root/reference is readable; the GPU box only reads the committed outputs.

1. kat_levels.json — the Dremel level known-answer tests of
   /root/reference/data_store_test.go:18-477: for every test, the schema it
   builds (AddGroup / AddColumn / NewListColumn calls) and, per leaf column,
   the asserted MaxDefinitionLevel, MaxRepetitionLevel, the dense values
   (`values.assemble()`) and the def / rep level arrays (`toArray()`).
2. crash/*.bin + crash/index.json — the fuzz-crash regression inputs the
   reference feeds to readAllData (schema_test.go:366-381): malformed files
   that must produce an error, never a crash.
     chunk_reader_test.go:5, page_v1_test.go:5, deltabp_decoder_test.go:5,152,
     type_dict_test.go:30, type_bytearray_test.go:5, schema_test.go:140,219

Both are data (inputs and expected outputs), parsed from the Go sources; no
reference code is copied.
"""
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

GO_ESC = {"a": 7, "b": 8, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11, "\\": 92, "'": 39, '"': 34}


def go_string(src, i):
    """Parse the Go interpreted string literal starting at src[i] == '"'.
    Returns (bytes, index after the closing quote)."""
    assert src[i] == '"'
    i += 1
    out = bytearray()
    while True:
        c = src[i]
        if c == '"':
            return bytes(out), i + 1
        if c != "\\":
            out += c.encode("utf-8")  # Go source is UTF-8: the literal holds those bytes
            i += 1
            continue
        e = src[i + 1]
        if e in GO_ESC:
            out.append(GO_ESC[e])
            i += 2
        elif e == "x":
            out.append(int(src[i + 2:i + 4], 16))
            i += 4
        elif e in "01234567":
            out.append(int(src[i + 1:i + 4], 8))
            i += 4
        elif e == "u":
            out += chr(int(src[i + 2:i + 6], 16)).encode("utf-8")
            i += 6
        elif e == "U":
            out += chr(int(src[i + 2:i + 10], 16)).encode("utf-8")
            i += 10
        else:
            raise ValueError("bad escape \\%s at %d" % (e, i))


def byte_literal(src, start):
    """[]byte("..." + "..." ...) starting at `start` (index of '[]byte(')."""
    i = src.index("(", start) + 1
    out = b""
    while True:
        while src[i] in " \t\r\n+":
            i += 1
        if src[i] == ")":
            return out
        piece, i = go_string(src, i)
        out += piece


def line_of(src, idx):
    return src.count("\n", 0, idx) + 1


# ---------------------------------------------------------------------------
# 1. crash inputs
# ---------------------------------------------------------------------------
CRASH = [("chunk_reader_test.go", "TestFuzzCrashReadRowGroup"),
         ("page_v1_test.go", "TestDataPageReaderV1InitCrash"),
         ("deltabp_decoder_test.go", "TestFuzzCrashDeltaBitPackDecoder64DivByZero"),
         ("deltabp_decoder_test.go", "TestFuzzCrashDeltaBitPackDecoder64LenOutOfRange"),
         ("type_dict_test.go", "TestFuzzCrashDictDecoderDecodeValues"),
         ("type_bytearray_test.go", "TestFuzzCrashByteArrayPlainDecoderNext"),
         ("schema_test.go", "TestFuzzCrashReadGroupSchema2"),
         ("schema_test.go", "TestFuzzCrashReadGroupSchema")]


def make_crash():
    d = os.path.join(HERE, "crash")
    os.makedirs(d, exist_ok=True)
    index = []
    for fname, test in CRASH:
        src = open(os.path.join(REF, fname), encoding="utf-8").read()
        f0 = src.index("func %s(" % test)
        b0 = src.index("[]byte(", f0)
        data = byte_literal(src, b0)
        out = "%s.bin" % test
        with open(os.path.join(d, out), "wb") as f:
            f.write(data)
        index.append({"test": test, "source": "%s:%d" % (fname, line_of(src, f0)), "file": out, "bytes": len(data)})
        print("crash: %-48s %6d bytes" % (test, len(data)))
    with open(os.path.join(d, "index.json"), "w") as f:
        json.dump(index, f, indent=1)


# ---------------------------------------------------------------------------
# 2. Dremel level KATs
# ---------------------------------------------------------------------------
REP = {"REQUIRED": 0, "OPTIONAL": 1, "REPEATED": 2}


def _ints(s):
    return [int(x) for x in re.findall(r"-?\d+", s)]


def make_levels():
    path = os.path.join(REF, "data_store_test.go")
    src = open(path, encoding="utf-8").read()
    funcs = [(m.start(), m.group(1)) for m in re.finditer(r"^func (Test\w+)\(t \*testing\.T\) \{", src, re.M)]
    out = {}
    for k, (f0, name) in enumerate(funcs):
        body = src[f0:funcs[k + 1][0] if k + 1 < len(funcs) else len(src)]
        schema = []
        for m in re.finditer(r'AddGroup\("([\w.]+)", parquet\.FieldRepetitionType_(\w+)\)', body):
            schema.append({"path": m.group(1), "repetition": REP[m.group(2)], "kind": "group", "at": m.start()})
        for m in re.finditer(r'AddColumn\("([\w.]+)", NewDataColumn\(newIntStore\(\), parquet\.FieldRepetitionType_(\w+)\)\)',
                             body):
            schema.append({"path": m.group(1), "repetition": REP[m.group(2)], "kind": "int32", "at": m.start()})
        lm = re.search(r"NewListColumn\(elementCol, parquet\.FieldRepetitionType_(\w+)\)", body)
        if lm:  # NewListColumn: <name> (LIST) { repeated group list { element } } (schema.go NewListColumn)
            em = re.search(r"NewDataColumn\(elementStore, parquet\.FieldRepetitionType_(\w+)\)", body)
            cm = re.search(r'AddColumn\("([\w.]+)", list\)', body)
            base = cm.group(1)
            schema += [{"path": base, "repetition": REP[lm.group(1)], "kind": "group", "at": cm.start()},
                       {"path": base + ".list", "repetition": 2, "kind": "group", "at": cm.start() + 1},
                       {"path": base + ".list.element", "repetition": REP[em.group(1)], "kind": "int32",
                        "at": cm.start() + 2}]
        schema.sort(key=lambda e: e.pop("at"))
        if not schema:
            continue
        # expected-value variables used by some tests
        exp_var = None
        loop = re.search(r"for i := (\d+); i < (\d+); i\+\+ \{\s*expected = append\(expected, int32\(i\)\)", body)
        if loop:
            exp_var = list(range(int(loop.group(1)), int(loop.group(2))))
        lit = re.search(r"var expected = \[\]interface\{\}\{([^}]*)\}", body)
        if lit:
            exp_var = _ints(lit.group(1).replace("int32", ""))
        cols = {}
        blocks = list(re.finditer(r'(\w+), err :?= row\.findDataColumn\("([\w.]+)"\)', body))
        for j, m in enumerate(blocks):
            var, col = m.group(1), m.group(2)
            blk = body[m.end():blocks[j + 1].start() if j + 1 < len(blocks) else len(body)]
            c = {"line": line_of(src, f0 + m.start())}
            c["max_def"] = int(re.search(r"uint16\((\d+)\), %s\.MaxDefinitionLevel\(\)" % var, blk).group(1))
            c["max_rep"] = int(re.search(r"uint16\((\d+)\), %s\.MaxRepetitionLevel\(\)" % var, blk).group(1))
            vm = re.search(r"Equal\(t, (\[\]interface\{\}\{[^\n]*\}|expected), %s\.data\.values\.assemble\(\)\)" % var, blk)
            c["values"] = exp_var if vm.group(1) == "expected" else _ints(vm.group(1).replace("int32", ""))
            c["def"] = _ints(re.search(r"\[\]int32\{([^}]*)\}, %s\.data\.dLevels\.toArray\(\)" % var, blk).group(1))
            c["rep"] = _ints(re.search(r"\[\]int32\{([^}]*)\}, %s\.data\.rLevels\.toArray\(\)" % var, blk).group(1))
            cols[col] = c
        out[name] = {"source": "data_store_test.go:%d" % line_of(src, f0), "schema": schema, "columns": cols}
        print("levels: %-22s %d leaves asserted" % (name, len(cols)))
    with open(os.path.join(HERE, "kat_levels.json"), "w") as f:
        json.dump({"source": "data_store_test.go:18-477", "tests": out}, f, indent=1)


if __name__ == "__main__":
    make_crash()
    make_levels()
