"""Count Snappy tokens (literals / copies) in a raw snappy block (analysis aid)."""
import sys


def tokens(b):
    i = 0
    n = 0
    while True:  # varint
        c = b[i]; i += 1
        if c < 0x80:
            break
    lit = cp = litb = cpb = 0
    while i < len(b):
        t = b[i]
        if t & 3 == 0:
            x = t >> 2
            if x < 60:
                i += 1
            else:
                e = x - 59
                x = int.from_bytes(b[i + 1:i + 1 + e], "little")
                i += 1 + e
            L = x + 1
            i += L
            lit += 1; litb += L
        else:
            L = (4 + ((t >> 2) & 7)) if t & 3 == 1 else 1 + (t >> 2)
            i += {1: 2, 2: 3, 3: 5}[t & 3]
            cp += 1; cpb += L
    return lit, litb, cp, cpb


if __name__ == "__main__":
    import numpy as np
    import pyarrow as pa
    rng = np.random.default_rng(0)
    for n in (2500, 30000, 50000):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        print("random", n, tokens(pa.compress(d, codec="snappy", asbytes=True)))
    for bw in (1, 2, 4, 8, 12, 16, 20):
        # a bit-packed hybrid run stream: header 0x7f + 63*bw bytes, repeated
        run = bytes([0x7f]) + rng.integers(0, 256, 63 * bw, dtype=np.uint8).tobytes()
        d = b"".join(bytes([0x7f]) + rng.integers(0, 256, 63 * bw, dtype=np.uint8).tobytes() for _ in range(40))
        d = bytes([bw]) + d
        print("hybrid bw", bw, len(d), tokens(pa.compress(d, codec="snappy", asbytes=True)))
