"""Does an Infinity-Cache warm-up on a side stream make the decode GEMMs cheaper?

Per weight shape (3B o / gate_up / down, 7B down), batch-1 decode GEMM timed with events:
  cold      : a 1 GiB sweep evicts the weights, then the GEMM
  warm_pf   : the sweep, then ops.prefetch(W), then the GEMM (timed alone)
  warm_gemm : the GEMM twice, the second timed (do the GEMM's own non-temporal loads leave W resident?)
  pf_us     : the prefetch kernel alone (cold)
  overlap   : sweep; stream 1 runs a busy-wait (~latency-bound attention stand-in) then the GEMM, stream 2 the
              prefetch of W forked at the same point -- total vs the same without the prefetch
    python scripts/probe_mall_prefetch.py > gpurun_out/mall.jsonl
"""
import json
import statistics

import torch

from llm_based_apache_spark_optimization_amd import ops

dev = torch.device("cuda:0")
big = torch.empty(1 << 28, dtype=torch.int32, device=dev)  # 1 GiB


def sweep():
    ops.prefetch([big], wgs=1024)


def ev():
    return torch.cuda.Event(enable_timing=True)


def med(f, n=15):
    ts = []
    for _ in range(n):
        ts.append(f())
    return round(statistics.median(ts), 2)


def run(name, N, K, M=1, wgs=512, spin=20000):
    w = ops.PackedWeight.from_dense(torch.randn(N, K, device=dev) * 0.02, "bf16")
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    wt = [w.data, w.scale]
    gemm = lambda: ops.linear(x, w, "bf16", out=out)
    pf = lambda s=None: ops.prefetch(wt, wgs=wgs)
    s2 = torch.cuda.Stream()

    def timed(pre, body):
        pre()
        a, b = ev(), ev()
        a.record()
        body()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3

    def overlap(with_pf):
        sweep()
        a, b = ev(), ev()
        a.record()
        if with_pf:
            s2.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s2):
                pf()
        torch.cuda._sleep(spin)
        gemm()
        if with_pf:
            torch.cuda.current_stream().wait_stream(s2)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3

    def spin_only():
        a, b = ev(), ev()
        a.record()
        torch.cuda._sleep(spin)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3

    def graph_overlap(with_pf):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                if with_pf:
                    s2.wait_stream(s)
                    with torch.cuda.stream(s2):
                        pf()
                torch.cuda._sleep(spin)
                gemm()
                if with_pf:
                    s.wait_stream(s2)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

        def one():
            sweep()
            a, b = ev(), ev()
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b) * 1e3
        return med(one)

    gemm(); pf(); torch.cuda.synchronize()
    res = dict(name=name, N=N, K=K, M=M, MB=round(w.nbytes / 1e6, 1), wgs=wgs,
               cold=med(lambda: timed(sweep, gemm)),
               warm_pf=med(lambda: timed(lambda: (sweep(), pf()), gemm)),
               warm_gemm=med(lambda: timed(gemm, gemm)),
               pf_us=med(lambda: timed(sweep, pf)),
               spin_us=med(spin_only),
               overlap_nopf=med(lambda: overlap(False)),
               overlap_pf=med(lambda: overlap(True)),
               graph_nopf=graph_overlap(False), graph_pf=graph_overlap(True))
    print(json.dumps(res), flush=True)


for nm, N, K in (("3b_o", 3072, 3072), ("3b_gate_up", 16384, 3072), ("3b_down", 3072, 8192),
                 ("7b_down", 4096, 11008), ("7b_gate_up", 22016, 4096)):
    run(nm, N, K)
run("3b_gate_up", 16384, 3072, wgs=128)
