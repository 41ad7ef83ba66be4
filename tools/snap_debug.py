"""Debug: GPU DecompressBlock on hand-assembled / pyarrow Snappy streams, report mismatches."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "oracle")]
import oracle, pqgpu

def uv(v):
    out = bytearray()
    while True:
        b = v & 0x7f; v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v: return bytes(out)

def run(name, stream, total):
    rc, want, _ = oracle.snappy_decode(bytes(stream), total)
    try:
        got = pqgpu.DecompressBlock(pqgpu.CompressionCodec_SNAPPY, bytes(stream), total)
    except Exception as e:
        print(name, "GPU error", e, "oracle rc", rc); return
    g = np.frombuffer(got, np.uint8); w = np.frombuffer(want, np.uint8)
    bad = np.nonzero(g != w)[0]
    print(name, "oracle rc", rc, "len", len(got), len(want), "mismatches", bad.size,
          (bad[0], bad[-1]) if bad.size else "", "zeros in got", int((g == 0).sum()), flush=True)

rng = np.random.default_rng(5)
for L in (70000, 20000, 16384, 16383, 9000):
    lit = rng.integers(1, 256, L, dtype=np.uint8).tobytes()
    tail = [(min(L - 100, 68000), 40), (min(L - 200, 9000), 64), (3, 5)]
    total = L + sum(t[1] for t in tail)
    lh = L - 1
    st = uv(total) + bytes([62 << 2]) + lh.to_bytes(3, "little") + lit
    for off, ln in tail:
        st += bytes([((ln - 1) << 2) | 3]) + off.to_bytes(4, "little")
    run("lit%d+copies" % L, st, total)
    st = uv(L) + bytes([62 << 2]) + lh.to_bytes(3, "little") + lit
    run("lit%d only" % L, st, L)
    st = uv(L + 4) + bytes([62 << 2]) + lh.to_bytes(3, "little") + lit + bytes([((4 - 1) << 2) | 2]) + (2).to_bytes(2, "little")
    run("lit%d+near" % L, st, L + 4)
import pyarrow as pa
for n in (65, 8193, 70000, 300000):
    d = np.round(rng.standard_normal(n // 8 + 1), 2).tobytes()[:n]
    run("pa mixed %d" % n, pa.compress(d, codec="snappy", asbytes=True), n)
    d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    run("pa rand %d" % n, pa.compress(d, codec="snappy", asbytes=True), n)
