"""bench.py's driver contract on CPU (gloo): the same launch the round-end driver uses
(``torch.distributed.run --nproc-per-node N ... bench.py --gpus N``), here with ``--cpu-rehearsal`` and a
tiny model, so the multi-rank path (replica groups, TP groups, barriers, MAX-over-ranks timing, one
JSON line from rank 0) is exercised without a GPU."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--cpu-rehearsal", "--model", "tiny-nsql", "--batch", "3", "--prompt-len", "12", "--new-tokens", "4",
        "--steps", "2", "--warmup", "1"]


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(nproc: int, extra=()):
    if nproc == 1:
        cmd = [sys.executable, "bench.py", *ARGS, *extra]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", f"--master-port={_port()}", "bench.py", "--gpus", str(nproc),
               *ARGS, *extra]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    return lines[0]


@pytest.mark.parametrize("nproc,extra,par,batch", [(1, (), "dp1", 3), (2, (), "dp2", 6), (2, ("--tp", "2"), "tp2dp1", 3),
                                                 (4, ("--tp", "2"), "tp2dp2", 6)])
def test_bench_contract_cpu(nproc, extra, par, batch):
    d = _run(nproc, extra)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == nproc and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["config"]["parallelism"] == par and d["config"]["global_batch"] == batch
    # value = whole-job output tokens / slowest rank's wall time over exactly `steps` steps
    assert abs(d["value"] - batch * 4 * 2 / (d["ms_per_step"] * 2 / 1000.0)) / d["value"] < 0.01
    assert "CPU rehearsal" in d["data"]
    # the teacher-forced decode check runs under TP too (rank 0's tokens vs the oracle on the unsharded weights)
    assert d["numerics"]["ok"] and d["numerics"]["tokens_checked"] >= 3, d["numerics"]
    if nproc > 1:  # the self-verifying communication record (which paths ran, on which devices)
        c = d["tp_comm"]
        assert c["world"] == nproc and len(c["device_per_rank"]) == nproc and c["backend"] == "gloo"
        if "--tp" in extra:
            assert c["tp"] == 2 and c["group_ranks"] == [2] and c["tp_backend"] == "gloo"
            assert c["ipc_allreduce"] is False and c["ipc_fallback"] is None  # CPU groups never try the IPC kernel
            calls = c["calls_all_ranks"]
            assert calls.get("gloo_all_reduce", 0) > 0, calls  # decode all-reduces of the row-parallel projections
            assert calls.get("gloo_all_gather_float32", 0) > 0, calls  # vocab-parallel logits
    else:
        assert "tp_comm" not in d
