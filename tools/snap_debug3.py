"""Debug: run the GPU parity tests that precede test_snappy_block_roundtrip in-process, then it."""
import os, sys
os.environ["PQG_DEBUG_SNAPPY"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.exit(__import__("pytest").main([os.path.join(ROOT, "tests", "test_gpu_parity.py"), "-x", "-q", "-s", "-m", "gpu",
                                    "-k", "golden_fixture or row_group_subsets or snappy_block_roundtrip"]))
