"""Option-less co-serving (bench_serving --option-less, 4 QPS, 15 s) with the round-4 prefill routes off
(ops.PREFILL_BLAS_RES = False, ops.PREFILL_BLAS_SILU_MAX_M = 0): with random-init weights the option-less output
lengths depend on when greedy decoding happens to emit EOS, so this separates a routing effect from that chaos.
    python scripts/coserve_prefill_routes_ab.py > gpurun_out/coserve_routes_off.json
"""
import sys

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import bench_serving, ops  # noqa: E402

ops.PREFILL_BLAS_RES = False
ops.PREFILL_BLAS_SILU_MAX_M = 0
bench_serving.main(["--qps", "4", "--duration", "15", "--option-less"])
