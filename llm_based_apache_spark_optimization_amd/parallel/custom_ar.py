"""One-shot all-reduce (and all-gather) over IPC-mapped peer buffers for decode-size TP messages (SURVEY.md §2.5 K15,
§2.6 P-COMM).

RCCL's generic all-reduce pays a collective launch and n-1 dependent ring hops; a TP=2 decode step
issues 64 of them (2 per layer, 7B) on B x 4096 f32 tensors of 16-512 KiB, each latency-bound on one
xGMI link.  ``IpcAllReduce`` replaces those with one kernel (``csrc/kernels/allreduce.hip``) that
pushes the tensor into every peer's receive slot over xGMI, raises per-block flags and sums locally
in rank order.  It is graph-capturable (fixed launch arguments, epochs on the device), so it sits
inside the captured decode hipGraph exactly where the RCCL call was.  Larger messages (prefill
[T, d] activations) keep using RCCL, which is bandwidth-optimal there.

The per-rank region is exchanged once through ``torch.distributed.all_gather_object`` on the TP
group (any backend), so the same code runs on one node of 8 GPUs over RCCL and in the 2/4-process
single-GPU tests over gloo.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops

log = logging.getLogger(__name__)

DEFAULT_MAX_BYTES = 8 << 20  # B=64 x d=4096 f32 all-reduces; B=32 x 64128 vocab-parallel logit gathers (3B, TP2)
DEFAULT_TIMEOUT_S = 60.0
# sums push bf16 partials (each rank rounds its contribution, its own copy too, and sums in f32 in rank order: every
# rank still gets bitwise the same result) -- half the xGMI bytes of the f32 payload; LSA_CUSTOM_AR_BF16=0 keeps f32
AR_BF16 = os.environ.get("LSA_CUSTOM_AR_BF16", "1") != "0"
# two-shot (reduce-scatter + all-gather) above this many payload bytes when the group has more than 2 ranks: each rank
# then sends (W - 1) / W of the tensor instead of the whole tensor to each of W - 1 peers (TP = 2 gains nothing from it)
AR_TWO_SHOT_MIN_BYTES = int(os.environ.get("LSA_CUSTOM_AR_TWO_SHOT_BYTES", str(128 << 10)))


class IpcUnavailable(RuntimeError):
    """The IPC regions could not be allocated, exported or mapped on some rank of the group; every rank
    then keeps RCCL for all of its collectives (the decision is collective, so the ranks never disagree
    on which path a call takes)."""


def _peer_reachable(mine: Optional[int], peer: Optional[int]) -> bool:
    """hipDeviceCanAccessPeer between two GPUs this process can see (TP ranks of a router replica see the
    replica's whole GPU list); ranks sharing one GPU, or a peer outside this process's view, pass here and
    are settled by the mapping itself."""
    if mine is None or peer is None or mine == peer:
        return True
    try:
        n = torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return True
    if not (0 <= mine < n and 0 <= peer < n):
        return True
    return bool(torch.cuda.can_device_access_peer(mine, peer))


def open_regions(group, rank: int, world: int, ext, nbytes: int,
                 device_index: Optional[int] = None) -> tuple[int, list, list]:
    """Allocate this rank's region, exchange IPC handles and map every peer's region.

    Collective over ``group`` and all-or-nothing: a failure on ANY rank (allocation, handle export, peer
    mapping -- e.g. ``hipIpcOpenMemHandle`` refused because the peer GPU is not reachable) makes every rank
    release what it mapped and raise ``IpcUnavailable``.  Returns (own base, [region ptr per rank], [opened
    peer ptrs])."""
    base, handle, why = 0, None, ""
    try:
        base = ext.ar_alloc(nbytes)
        handle = ext.ar_handle(base)
    except Exception as e:  # noqa: BLE001 - reported collectively below
        why = f"rank {rank}: region export failed: {e}"
    recs: list = [None] * world
    dist.all_gather_object(recs, (handle, device_index), group=group)
    handles = [h for h, _ in recs]
    opened, ptrs = [], []
    if not why:
        unreachable = [r for r, (_, di) in enumerate(recs) if r != rank and not _peer_reachable(device_index, di)]
        if unreachable:
            why = f"rank {rank}: no peer access to the GPUs of ranks {unreachable}"
    if not why and all(h is not None for h in handles):
        try:
            for r, h in enumerate(handles):
                if r == rank:
                    ptrs.append(base)
                    continue
                if os.environ.get("LSA_TEST_FAIL_AR_OPEN") == str(rank):  # fault injection (tests)
                    raise RuntimeError("injected ar_open failure")
                p = ext.ar_open(h)
                opened.append(p)
                ptrs.append(p)
        except Exception as e:  # noqa: BLE001
            why = f"rank {rank}: peer mapping failed: {e}"
    elif not why:
        why = "a peer could not export its region"
    verdicts: list = [None] * world
    dist.all_gather_object(verdicts, why, group=group)
    bad = [v for v in verdicts if v]
    if bad:
        for p in opened:
            try:
                ext.ar_close(p)
            except Exception:  # noqa: BLE001
                pass
        if base:
            try:
                ext.ar_free(base)
            except Exception:  # noqa: BLE001
                pass
        raise IpcUnavailable("; ".join(bad))
    return base, ptrs, opened


class IpcAllReduce:
    """In-place f32 sum over the ``world`` ranks of ``group`` for tensors up to ``max_bytes``: one-shot (every rank
    pushes its tensor to every peer) for TP = 2 and small messages, two-shot (reduce-scatter + all-gather) above
    ``two_shot_min_bytes`` with more than 2 ranks; bf16 payloads by default (``AR_BF16``)."""

    def __init__(self, group, rank: int, world: int, device: torch.device, max_bytes: int = DEFAULT_MAX_BYTES,
                 nblocks: int = 128, timeout_s: float = DEFAULT_TIMEOUT_S, bf16: Optional[bool] = None,
                 two_shot_min_bytes: Optional[int] = None):
        ext = ops.ext()
        if not 2 <= world <= ext.ar_max_world:
            raise ValueError(f"IpcAllReduce supports 2..{ext.ar_max_world} ranks, got {world}")
        self.rank, self.world, self.device = rank, world, device
        self.max_bytes = int(max_bytes)
        self.nblocks = int(nblocks)
        self.bf16 = AR_BF16 if bf16 is None else bool(bf16)
        self.two_shot_min_bytes = AR_TWO_SHOT_MIN_BYTES if two_shot_min_bytes is None else int(two_shot_min_bytes)
        with torch.cuda.device(device):
            # recv[2][world][max_bytes] + the two-shot result area res[2][max_bytes]
            self._base, ptrs, self._opened = open_regions(group, rank, world, ext,
                                                          ext.ar_header_bytes + (2 * world + 2) * self.max_bytes,
                                                          device_index=device.index)
            self.regions = torch.tensor(ptrs, dtype=torch.int64, device=device)
            self.err = torch.zeros(1, dtype=torch.int32, device=device)
            self.timeout_ticks = int(timeout_s * ext.ar_wallclock_khz() * 1000)
        # every rank has mapped every peer before anyone pushes
        dist.barrier(group=group)

    def mode(self, payload_bytes: int) -> int:
        """Kernel mode of a sum over ``payload_bytes`` of f32: bit 0 bf16 payload, bit 1 two-shot."""
        two = self.world > 2 and payload_bytes > self.two_shot_min_bytes
        return (1 if self.bf16 else 0) | (2 if two else 0)

    def fits(self, t: torch.Tensor) -> bool:
        return (t.dtype == torch.float32 and t.is_cuda and t.is_contiguous() and t.numel() % 4 == 0
                and t.numel() * 4 <= self.max_bytes and t.data_ptr() % 16 == 0)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        ops.ext().ar_run(t, None, self.regions, self.rank, self.max_bytes, self.nblocks, self.timeout_ticks, self.err,
                         mode=self.mode(t.numel() * 4))
        return t

    def fits_slabs(self, t: torch.Tensor) -> bool:
        """t = [nslab, ...] split-K slabs whose per-slab payload fits the slot."""
        return (t.dtype == torch.float32 and t.is_cuda and t.is_contiguous() and t.dim() >= 2
                and (t.numel() // t.shape[0]) % 4 == 0 and (t.numel() // t.shape[0]) * 4 <= self.max_bytes
                and t.data_ptr() % 16 == 0)

    def reduce_slabs(self, t: torch.Tensor) -> torch.Tensor:
        """Sum over ranks of each rank's slab-sum of t [nslab, ...]; the result lands in t[0] (returned
        as a [1, ...] view) — split-K partials and the TP all-reduce in one kernel."""
        ops.ext().ar_run(t, None, self.regions, self.rank, self.max_bytes, self.nblocks, self.timeout_ticks, self.err,
                         t.shape[0], mode=self.mode(t.numel() // t.shape[0] * 4))
        return t[:1]

    def reduce_slabs_res(self, t: torch.Tensor, h: torch.Tensor, xn: torch.Tensor, ss: torch.Tensor,
                         xmt: int = 0) -> None:
        """The all-reduce of ``reduce_slabs`` with the residual epilogue of a row-parallel projection fused in: h
        [rows, D] f32 += the sum over ranks of every rank's slab sum; xn = bf16(h) (fragment-major with ``xmt`` row
        tiles, else row-major); ss[rows] += row sums of h^2 (Q24 int64).  One launch where the unfused TP step ran
        an all-reduce and then a residual-add launch (D % 256 == 0)."""
        ops.ext().ar_run(t, None, self.regions, self.rank, self.max_bytes, self.nblocks, self.timeout_ticks, self.err,
                         t.shape[0], res_h=h, res_xn=xn, res_ss=ss, res_xmt=xmt,
                         mode=self.mode(t.numel() // t.shape[0] * 4))

    def all_gather(self, out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        """out[world * n] = concatenation of every rank's t[n] in rank order (same push protocol)."""
        ops.ext().ar_run(t, out, self.regions, self.rank, self.max_bytes, self.nblocks, self.timeout_ticks, self.err)
        return out

    def check(self) -> None:
        """Raise if any wait timed out since construction (a peer never arrived).  The engine reads the
        same flag at every host sync (``ModelRunner.read_rows``); a timed-out block's result is NaN."""
        if int(self.err.item()):
            raise RuntimeError("IpcAllReduce: a peer did not arrive within the timeout")

    def close(self) -> None:
        ext = ops.ext()
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            ext.ar_close(p)
        self._opened = []
        if self._base:
            ext.ar_free(self._base)
            self._base = 0


def maybe_ipc_allreduce(group, rank: int, world: int, device: torch.device) -> Optional[IpcAllReduce]:
    """The one-shot all-reduce for a GPU TP group, unless disabled (``LSA_CUSTOM_AR=0``) or unavailable.

    Unavailable includes a failure on any rank to map its peers' regions (``IpcUnavailable``): the group
    then degrades to RCCL for every collective instead of the replica dying in ``TPGroup.warmup``."""
    maybe_ipc_allreduce.last_reason = ""
    if device.type != "cuda" or world < 2 or os.environ.get("LSA_CUSTOM_AR", "1") == "0":
        maybe_ipc_allreduce.last_reason = "disabled" if device.type == "cuda" and world >= 2 else "not a GPU group"
        return None
    if world > ops.ext().ar_max_world:
        maybe_ipc_allreduce.last_reason = f"group of {world} ranks exceeds the kernel's {ops.ext().ar_max_world}"
        return None
    try:
        return IpcAllReduce(group, rank, world, device,
                            max_bytes=int(os.environ.get("LSA_CUSTOM_AR_MAX_BYTES", DEFAULT_MAX_BYTES)),
                            timeout_s=float(os.environ.get("LSA_CUSTOM_AR_TIMEOUT_S", DEFAULT_TIMEOUT_S)))
    except IpcUnavailable as e:
        log.warning("one-shot IPC all-reduce unavailable, TP group falls back to RCCL: %s", e)
        maybe_ipc_allreduce.last_reason = str(e)
        return None


maybe_ipc_allreduce.last_reason = ""
