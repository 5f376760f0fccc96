"""Per-launch floor of a captured decode step: graphs of 200 launches of
  empty   : ops.prefetch of 0 bytes (no memory access at all), 256 / 1024 workgroups
  resadd  : the b32 residual add (7B: 32 rows x 4096, 2 f32 slabs)
  *_gpu_side: the same replays queued behind a long busy-wait kernel, so the host has submitted every packet before
              the first one runs (the events then time the GPU side alone, not the host's submission rate)
  touch   : ops.prefetch of 2.5 MB (the residual add's bytes, no dependent chain)
timed with events over whole replays (per launch = replay / 200).
    python scripts/probe_kernel_floor.py > gpurun_out/floor.jsonl
"""
import json
import statistics

import torch

from llm_based_apache_spark_optimization_amd import ops

dev = torch.device("cuda:0")
N = 200


def graph_time(fn, reps=20, pre_sleep=False):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(N):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g.replay()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if pre_sleep:  # the GPU is busy while the host queues the replay: the events then time the GPU side only
            torch.cuda._sleep(20_000_000)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / N)
    return round(statistics.median(ts), 3)


buf = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
h = torch.randn(32, 4096, device=dev)
parts = torch.randn(2, 32, 4096, device=dev)
xn = torch.empty(32, 4096, device=dev, dtype=torch.bfloat16)
ss = torch.zeros(32, dtype=torch.int64, device=dev)
small = torch.zeros(625 * 1024, dtype=torch.int32, device=dev)  # 2.5 MB
res = {
    "empty_256wg": graph_time(lambda: ops.prefetch([buf], [0], 256)),
    "empty_1wg": graph_time(lambda: ops.prefetch([buf], [0], 1)),
    "empty_1024wg": graph_time(lambda: ops.prefetch([buf], [0], 1024)),
    "touch_2p5MB_256wg": graph_time(lambda: ops.prefetch([small], None, 256)),
    "resadd_b32_7b": graph_time(lambda: ops.res_add_ss(h, parts, xn, 32, ss)),
    "empty_256wg_gpu_side": graph_time(lambda: ops.prefetch([buf], [0], 256), pre_sleep=True),
    "resadd_b32_7b_gpu_side": graph_time(lambda: ops.res_add_ss(h, parts, xn, 32, ss), pre_sleep=True),
    "torch_add_small": graph_time(lambda: buf.add_(1)),
}
print(json.dumps(res), flush=True)
