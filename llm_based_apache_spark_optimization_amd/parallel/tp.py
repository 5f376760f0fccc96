"""Tensor-parallel process groups over RCCL (torch.distributed backend "nccl" is RCCL on ROCm).

Megatron-style split (SURVEY.md §2.6 P-TP): QKV and gate/up column-parallel, O and down row-parallel
followed by one all-reduce each (2 per layer), LM head vocab-parallel followed by an all-gather.
On MI355X every GPU pair has its own xGMI link, so a TP=2 replica uses exactly one link; the
decode-size all-reduce (B x d f32, 16-512 KiB) is latency-bound and is captured inside the decode
hipGraph together with the kernels around it.  On GPU groups those decode-size all-reduces run on
the one-shot IPC kernel (``custom_ar.IpcAllReduce``); RCCL keeps the large ones.
"""
from __future__ import annotations

import collections
import os
from typing import Optional

import torch
import torch.distributed as dist


class TPGroup:
    def __init__(self, group, rank: int, size: int, device: torch.device):
        self.group, self.rank, self.size, self.device = group, rank, size, device
        self._warm = False
        self.car = None  # IpcAllReduce once warmed up on a GPU group
        self.ipc_fallback = ""  # why a GPU group runs without the IPC kernel (custom_ar.maybe_ipc_allreduce)
        # collectives ISSUED per path (eager launches and graph captures; a replayed graph re-runs its captured
        # ones without coming back here): ipc_oneshot / ipc_twoshot / ipc_all_gather, <backend>_<collective>
        self.calls: collections.Counter = collections.Counter()

    def _backend(self) -> str:
        try:
            return str(dist.get_backend(self.group))
        except Exception:  # noqa: BLE001 - not initialised (unit tests of the helpers)
            return "none"

    def _ipc(self, payload_bytes: int) -> None:
        self.calls["ipc_twoshot" if self.car.mode(payload_bytes) & 2 else "ipc_oneshot"] += 1

    def describe(self) -> dict:
        """Which communication paths this rank's TP group runs (bench.py's ``tp_comm`` record): backend, ranks per
        group, the device it sits on, whether the one-shot IPC all-reduce is live (else why not), and the
        issued-collective counts per path."""
        try:
            nranks = dist.get_world_size(self.group)
        except Exception:  # noqa: BLE001
            nranks = self.size
        return {"backend": self._backend(), "group_ranks": int(nranks), "tp_rank": self.rank,
                "device": str(self.device), "device_index": self.device.index,
                "ipc_allreduce": self.car is not None,
                "ipc_bf16_payload": bool(self.car.bf16) if self.car is not None else None,
                "ipc_fallback": self.ipc_fallback or None, "calls": dict(sorted(self.calls.items()))}

    def all_reduce(self, t: torch.Tensor) -> None:
        if self.car is not None and self.car.fits(t):
            self._ipc(t.numel() * 4)
            self.car(t)
        else:
            self.calls[f"{self._backend()}_all_reduce"] += 1
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def can_fold_splitk(self, slab_numel: int) -> bool:
        """Whether split-K slabs of slab_numel f32 each can be reduced inside the one-shot all-reduce."""
        return self.car is not None and slab_numel * 4 <= self.car.max_bytes

    def reduce_parts(self, parts: torch.Tensor) -> torch.Tensor:
        """All-reduce of the sum of parts [nslab, ...] (row-parallel GEMM split-K slabs); returns the [1, ...]
        view holding the result."""
        if parts.shape[0] == 1:
            self.all_reduce(parts)
            return parts
        if self.car is not None and self.car.fits_slabs(parts):
            self._ipc(parts.numel() // parts.shape[0] * 4)
            return self.car.reduce_slabs(parts)
        red = parts[:1]
        red.add_(parts[1:].sum(0, keepdim=True))
        self.all_reduce(red)
        return red

    def reduce_add(self, parts: torch.Tensor, h: torch.Tensor, xn: torch.Tensor, ss: torch.Tensor, rows: int,
                   xf: bool = False) -> None:
        """Residual epilogue of a row-parallel projection: h[:rows] += all-reduced slab sum of parts [nslab, rows, D];
        xn = bf16(h) (fragment-major when xf); ss[:rows] += row sums of h^2 (Q24).  On the one-shot IPC kernel this is
        ONE launch (``IpcAllReduce.reduce_slabs_res``); otherwise the all-reduce, then the wide residual add."""
        from .. import ops

        D = h.shape[1]
        if (self.car is not None and parts.is_cuda and self.car.fits_slabs(parts) and D % 256 == 0
                and h.is_contiguous() and parts.shape[1] == rows):
            self._ipc(parts.numel() // parts.shape[0] * 4)
            self.car.reduce_slabs_res(parts, h[:rows], xn, ss, ops.xfrag_tiles(rows) if xf else 0)
            return
        ops.res_add_ss(h, self.reduce_parts(parts), xn, rows, ss, xf=xf)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if self.car is not None and self.car.fits(inp) and out.is_contiguous():
            self.calls["ipc_all_gather"] += 1
            self.car.all_gather(out, inp)
        else:
            self.calls[f"{self._backend()}_all_gather_{str(inp.dtype).replace('torch.', '')}"] += 1
            dist.all_gather_into_tensor(out, inp, group=self.group)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """out = rank's 1/size row block of the sum over ranks of inp (sequence-parallel prefill)."""
        self.calls[f"{self._backend()}_reduce_scatter_{str(inp.dtype).replace('torch.', '')}"] += 1
        if inp.is_cuda and dist.get_backend(self.group) == "gloo":  # gloo: CPU tensors only (test boxes)
            tmp = inp.clone()
            dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=self.group)
            out.copy_(tmp.view(self.size, -1)[self.rank].view_as(out))
            return
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group)

    def capturable(self) -> bool:
        """Whether the decode step's collectives can be captured in a hipGraph: the one-shot IPC kernel or
        RCCL can; gloo (ranks sharing one GPU on test boxes, after an IPC fallback) cannot."""
        return self.car is not None or dist.get_backend(self.group) == "nccl"

    def min_int(self, x: int) -> int:
        """Minimum of ``x`` over the group (host value; collective)."""
        on_dev = dist.get_backend(self.group) == "nccl"
        t = torch.tensor([int(x)], dtype=torch.int64, device=self.device if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return int(t.item())

    def warmup(self) -> None:
        """Initialise the communicators outside graph capture (collective over the group)."""
        if not self._warm:
            t = torch.zeros(16, device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            if self.device.type == "cuda":
                from .custom_ar import maybe_ipc_allreduce

                self.car = maybe_ipc_allreduce(self.group, self.rank, self.size, self.device)
                self.ipc_fallback = "" if self.car is not None else (maybe_ipc_allreduce.last_reason or "unavailable")
                if self.car is not None:
                    self.car(t)
                torch.cuda.synchronize(self.device)
            self._warm = True


def init_distributed(backend: Optional[str] = None) -> tuple[int, int, int]:
    """(rank, world, local_rank) from torchrun env; initialises the default group once."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def make_replica_groups(world: int, tp: int, rank: int, device: torch.device) -> tuple[int, Optional[TPGroup]]:
    """Split ``world`` ranks into world/tp replicas of ``tp`` consecutive ranks ({0,1},{2,3},... for tp=2).

    Every rank must call this (new_group is collective).  Returns (replica index, this rank's TP group).
    """
    if world % tp:
        raise ValueError(f"world {world} not divisible by tp {tp}")
    mine = None
    for r0 in range(0, world, tp):
        ranks = list(range(r0, r0 + tp))
        g = dist.new_group(ranks) if (tp > 1 and world > 1) else None
        if rank in ranks and tp > 1:
            mine = TPGroup(g, rank - r0, tp, device)
    return rank // tp, mine
