"""bench.py with the earlier decode split plan (fixed 4-block chunks, 2-block chunks below 128
(sequence, kv-head) pairs, contexts of <= 4 blocks unsplit): the A/B baseline for the ~256-workgroup plan."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402


def legacy_plan(B, Hkv, max_ctx):
    nblk = max(1, (max_ctx + 63) // 64)
    if nblk <= 4:
        return nblk, 1, 4
    chunk = 2 if B * Hkv < 128 else 4
    while (nblk + chunk - 1) // chunk > 256:
        chunk += 1
    return chunk, (nblk + chunk - 1) // chunk, 4


ops.decode_split_plan = legacy_plan
sys.argv[0] = "bench.py"
import bench  # noqa: E402

sys.exit(bench.main())
