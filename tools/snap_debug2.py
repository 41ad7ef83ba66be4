"""Debug: replay test_snappy_block_roundtrip's call sequence, report the first mismatch."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "oracle")]
import oracle, pqgpu
import pyarrow as pa

def check(name, comp, n, want):
    got = pqgpu.DecompressBlock(pqgpu.CompressionCodec_SNAPPY, comp, n)
    g = np.frombuffer(got, np.uint8); w = np.frombuffer(want, np.uint8)
    bad = np.nonzero(g != w)[0]
    print(name, n, "mismatches", bad.size, (int(bad[0]), int(bad[-1])) if bad.size else "", "zeros", int((g == 0).sum()),
          "vs", int((w == 0).sum()), flush=True)

rng = np.random.default_rng(5)
for n in (0, 1, 5, 64, 65, 4095, 8192, 8193, 70000, 300000):
    for kind in ("rand", "rep", "mixed"):
        if kind == "rand":
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == "rep":
            data = (b"0123456789abcdefXYZ" * (n // 19 + 1))[:n]
        else:
            data = np.round(rng.standard_normal(n // 8 + 1), 2).tobytes()[:n]
        comp = pa.compress(data, codec="snappy", asbytes=True)
        check("%s" % kind, comp, n, data)
lit = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
stream = bytearray()
total = 70000 + 40 + 64 + 5
v = total
while True:
    b = v & 0x7f
    v >>= 7
    stream.append(b | (0x80 if v else 0))
    if not v:
        break
stream += bytes([62 << 2]) + (70000 - 1).to_bytes(3, "little") + lit
stream += bytes([((40 - 1) << 2) | 3]) + (68000).to_bytes(4, "little")
stream += bytes([((64 - 1) << 2) | 3]) + (9000).to_bytes(4, "little")
stream += bytes([((5 - 1) << 2) | 2]) + (3).to_bytes(2, "little")
rc, want, _ = oracle.snappy_decode(bytes(stream), total)
check("hand", bytes(stream), total, want)
check("hand again", bytes(stream), total, want)
