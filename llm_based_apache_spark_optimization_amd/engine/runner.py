"""ModelRunner: one model replica (optionally one tensor-parallel shard of it) on one device.

Owns the packed weights, the paged KV cache, the RoPE tables, every decode workspace and the
device-resident decode state, and executes

* ``prefill(seqs)`` — packed variable-length prefill (eager launches; shapes change per call),
  which also commits each sequence's first generated token into its decode slot;
* ``decode(B, steps)`` — ``steps`` decode steps over slot rows ``[0, B)``, replayed from a captured
  hipGraph (``torch.cuda.CUDAGraph``) per (batch bucket, sampler mode).  The whole step — 32 layers of
  fused kernels, the TP all-reduces, LM head, token selection and the state update — runs without
  the host: positions, context lengths, finished flags and the generated tokens live on the device, so
  a graph replays for as many steps as the host wants between synchronisations.

Decode-step kernel sequence per layer (``L`` layers, B tokens):
  add_rmsnorm(+embedding | +down partials) -> gemm qkv -> rope_append (RoPE + paged KV write)
  -> attn_decode (split-KV) -> gemm o (f32 split-K slabs) [-> all_reduce] -> add_rmsnorm(+o partials)
  -> gemm gate_up (fused SiLU*up) -> gemm down (f32 slabs) [-> all_reduce]
then add_rmsnorm(final) -> gemm lm_head [-> all_gather] -> argmax/sample + commit.
"""
from __future__ import annotations


import math
import os
from typing import Optional, Sequence

import torch

from .. import ops
from ..models.llama import LlamaWeights
from ..ops import reference as ref

BLOCK = 64
REPEAT_WINDOW = 64  # repetition-penalty ring (Ollama repeat_last_n default; larger values are clamped)
# norm-free attention input in prefill (Runner._prefill_layers), off by default: measured even with the norm launch
# it removes (3B 2k TTFT 14.38 vs 14.34 ms, profiles/r5/prefill_norm_free_ab.txt)
# batch-1 decode with the residual add folded into the next GEMM's prologue (ModelRunner._decode_step_rr)
RR_DECODE = os.environ.get("LSA_RR", "1") != "0"


class TPCommError(RuntimeError):
    """A TP peer missed a one-shot all-reduce (the kernel poisoned the result with NaN and set err)."""


class ModelRunner:
    def __init__(self, weights: LlamaWeights, max_slots: int = 32, max_model_len: int = 4096,
                 num_kv_blocks: Optional[int] = None, kv_memory_fraction: float = 0.85,
                 max_new_cap: Optional[int] = None, tp=None, use_graphs: bool = True,
                 fuse_rope: Optional[bool] = None, seq_parallel: Optional[bool] = None, sp_min_tokens: Optional[int] = None,
                 kv_dtype: Optional[str] = None):
        self.w = weights
        # paged KV cache dtype: "bf16" or "fp8" (e4m3 rows with per-(token, kv-head) scales, ops.KV_FP8)
        kv_dtype = kv_dtype or ("fp8" if ops.KV_FP8 else "bf16")
        assert kv_dtype in ("bf16", "fp8"), kv_dtype
        self.kv_fp8 = kv_dtype == "fp8"
        # Megatron sequence parallelism for TP prefill (SURVEY.md §2.6 P-SP): reduce-scatter the row-parallel
        # outputs, residual + RMSNorm on T/tp rows, all-gather the bf16 normalised activations
        self.seq_parallel = True if seq_parallel is None else seq_parallel
        # SP prefill collective payload: the row-parallel GEMMs write bf16 and the reduce-scatter moves bf16 (half the
        # xGMI bytes of f32; the TP partial sums are rounded once to bf16 before the sum, as the decode all-reduce's
        # bf16 payload does); False keeps f32 slabs
        self.sp_bf16 = os.environ.get("LSA_SP_BF16", "1") != "0"
        self.sp_min_tokens = 256 if sp_min_tokens is None else sp_min_tokens
        # decode RoPE + KV append inside the attention kernel (fuse_rope=False restores the separate launch)
        self.fuse_rope = True if fuse_rope is None else fuse_rope
        self.spec = spec = weights.spec
        self.device = weights.device
        self.tp = tp
        tps = tp.size if tp is not None else 1
        self.H = spec.n_heads // tps
        self.Hkv = spec.n_kv_heads // tps
        self.D = spec.head_dim
        assert self.D == 128, "kernels are specialised for head_dim 128"
        self.d = spec.hidden
        self.L = spec.n_layers
        self.V = spec.vocab_size
        self.Vl = weights.lm_head.N
        self.ffn_l = spec.ffn // tps
        self.eps = spec.rms_eps
        self.scale = 1.0 / math.sqrt(self.D)
        self.max_slots = max_slots
        self.max_model_len = min(max_model_len, spec.max_position)
        self.max_blocks = (self.max_model_len + BLOCK - 1) // BLOCK
        self.max_new_cap = max_new_cap or self.max_model_len
        self.on_gpu = self.device.type == "cuda"
        self.use_graphs = use_graphs and self.on_gpu
        dev = self.device

        # ---------------- KV cache: [L, 2, blocks, Hkv, 64, D] bf16, or e4m3 bytes + [L, 2, blocks, Hkv, 64] f32 scales
        per_block = self.L * 2 * self.Hkv * BLOCK * ((self.D + 4) if self.kv_fp8 else self.D * 2)
        want = max_slots * self.max_blocks + 1
        if num_kv_blocks is None:
            if self.on_gpu:
                free, _ = torch.cuda.mem_get_info(dev)
                budget = int(free * kv_memory_fraction) - (1 << 30)
                num_kv_blocks = max(2, min(want, budget // per_block))
            else:
                num_kv_blocks = want
        if tp is not None and tp.size > 1:
            # every rank's arena must hold every block id the leader's scheduler hands out: ranks that size
            # their arenas from their own free memory (shared GPUs, a rebuild beside a not-yet-freed engine)
            # agree on the smallest
            num_kv_blocks = tp.min_int(num_kv_blocks)
        self.num_kv_blocks = int(num_kv_blocks)
        self.kv = torch.zeros(self.L, 2, self.num_kv_blocks, self.Hkv, BLOCK, self.D,
                              dtype=torch.uint8 if self.kv_fp8 else torch.bfloat16, device=dev)
        self.kv_scale = (torch.zeros(self.L, 2, self.num_kv_blocks, self.Hkv, BLOCK, dtype=torch.float32, device=dev)
                         if self.kv_fp8 else None)
        # one row per position the block tables can address (the kernels check this bound on the host)
        cos, sin = ref.rope_tables(self.D, self.max_blocks * BLOCK, spec.rope_theta, spec.rope_scaling, device=dev)
        self.cos, self.sin = cos.contiguous(), sin.contiguous()

        # ---------------- device decode state (one row per slot)
        S = max_slots
        i32 = dict(dtype=torch.int32, device=dev)
        self.input_ids = torch.zeros(S, **i32)
        self.positions = torch.zeros(S, **i32)
        self.gen_len = torch.zeros(S, **i32)
        self.finished = torch.ones(S, **i32)
        self.limit = torch.full((S,), self.max_new_cap, **i32)
        self.eos_on = torch.ones(S, **i32)
        self.out_tokens = torch.zeros(S, self.max_new_cap, **i32)
        self.block_tables = torch.zeros(S, self.max_blocks, **i32)
        self.temperature = torch.zeros(S, dtype=torch.float32, device=dev)
        self.top_k = torch.full((S,), 40, **i32)
        self.top_p = torch.full((S,), 0.9, dtype=torch.float32, device=dev)
        self.seeds = torch.zeros(S, dtype=torch.int64, device=dev)
        # repetition penalty (Ollama repeat_penalty / repeat_last_n): per-row ring of the context's last
        # REPEAT_WINDOW tokens, indexed by position, written by the sampling commit
        self.penalty = torch.ones(S, dtype=torch.float32, device=dev)
        self.last_n = torch.full((S,), REPEAT_WINDOW, **i32)
        self.hist = torch.full((S, REPEAT_WINDOW), -1, **i32)
        self.eos_list = list(spec.eos_ids) or [-1]
        self.eos = torch.tensor(self.eos_list, **i32)

        # ---------------- decode workspaces sized for S rows
        f32 = dict(dtype=torch.float32, device=dev)
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.h = torch.zeros(S, self.d, **f32)
        self.xn = torch.zeros(S, self.d, **bf)
        self.qkv = torch.zeros(S, (self.H + 2 * self.Hkv) * self.D, **bf)
        self.q = torch.zeros(S, self.H, self.D, **bf)
        self.attn = torch.zeros(S, self.H * self.D, **bf)
        self.act = torch.zeros(S, self.ffn_l, **bf)
        # fragment-major decode activations (ops.to_xfrag) for 16 < B <= 64 bf16 buckets: the norm,
        # attention and gate_up kernels write the next GEMM's MFMA B-fragments directly
        xr = 16 * ops.xfrag_tiles(min(S, 64))
        self.xn_f = torch.zeros(xr * self.d, **bf)
        self.attn_f = torch.zeros(xr * self.H * self.D, **bf)
        self.act_f = torch.zeros(xr * self.ffn_l, **bf)
        # W8A8 / W4A8 decode (fp8 or MXFP4 weights, ops.linear_a8 on the block-scaled fp8 MFMA, activations in the
        # xf8 layout): the norm launches write the qkv / gate_up inputs as per-row-scaled e4m3, the decode attention
        # writes the o input as e4m3 with one E8M0 scale per (row, head), and the gate_up GEMM's SiLU epilogue writes
        # the down input as e4m3 with one E8M0 scale per (row, 32 columns)
        wkind = weights.layers[0].wqkv.kind
        self.a8 = (ops.FP8_A8_DECODE and self.on_gpu and wkind in ("fp8", "mxfp4") and self.d % 128 == 0)
        # the down projection W8A8 needs whole 32-column blocks per SiLU workgroup (gate_up n-blocks % 4 == 0)
        self.a8_down_ok = self.ffn_l % 128 == 0 and (2 * self.ffn_l // 16) % 4 == 0
        # Which projections take e4m3 activations, per weight format and bucket (standalone sweeps with weights
        # streaming from HBM: profiles/r4/bench_a8_decode_{fp8,mxfp4}_mi355x.jsonl, scripts/bench_a8_decode.py):
        #   qkv: fp8 above 32 rows -- at 32 the W8A8 GEMM ties / loses to W8A16 (7B 13.3 vs 12.4 us) and the 7B b32
        #        bench did not move while the e4m3 activations cost top-1 agreement (profiles/bench_fp8a_decode_mi355x.jsonl);
        #        MXFP4 at every bucket (7B 8.0 vs 10.2 us at 1 row, 9.4 vs 11.9 at 32: no VALU e2m1 widening);
        #   gate_up: fp8 from 17 rows (7B 19.0 vs 22.7 us at 32), MXFP4 at every bucket (11.2 vs 15.7, 13.0 vs 15.5);
        #   o and down: only where it pays -- MXFP4 up to 16 rows (7B o 6.1 vs 10.0 us, down 7.9 vs 10.0 at 1 row); at 32
        #        rows they tie or lose (o 6.3 vs 6.1, down 9.6 vs 10.5 but the e4m3 SiLU output it needs costs gate_up
        #        15.3 vs 13.0 us), and fp8 never gains (7B b32 step 2.80 vs 2.60 ms with them,
        #        profiles/r4/rocprof_fp8_b32_a8all_summary.txt)
        mx = wkind == "mxfp4"
        self.a8_min_batch = 0 if mx else 32
        self.a8_mlp_min_batch = 0 if mx else 16
        self.a8_od_max_batch = 16 if mx else 0  # o / down W8A8 (W4A8) up to this bucket
        self.x8 = torch.zeros(xr * self.d if self.a8 else 1, dtype=torch.uint8, device=dev)
        self.sx8 = torch.ones(max(S, 64), **f32)
        mt64 = ops.xfrag_tiles(min(S, 64))
        self.x8o = torch.zeros(xr * self.H * self.D if self.a8 else 1, dtype=torch.uint8, device=dev)
        self.s8o = torch.full((mt64 * 64 * (self.H * self.D // 128) if self.a8 else 1,), 127, dtype=torch.uint8,
                              device=dev)
        a8d = self.a8 and self.a8_down_ok
        self.x8d = torch.zeros(xr * self.ffn_l if a8d else 1, dtype=torch.uint8, device=dev)
        self.s8d = torch.full((mt64 * 64 * (self.ffn_l // 128) if a8d else 1,), 127, dtype=torch.uint8, device=dev)
        self.o_buf = torch.zeros(8 * S * self.d, **f32)
        self.down_buf = torch.zeros(8 * S * self.d, **f32)
        self.qkv_buf = torch.zeros(8 * S * (self.H + 2 * self.Hkv) * self.D, **f32)
        self.logits_l = torch.zeros(S, self.Vl, **f32)
        self.logits = self.logits_l if tps == 1 else torch.zeros(S, self.V, **f32)
        self.gather_buf = None if tps == 1 else torch.zeros(tps * S * self.Vl, **f32)
        nsplit_max = max(4, ops.decode_split_plan(1, self.Hkv, self.max_model_len)[1])
        self.attn_ws = ops.decode_workspace(S, self.H, self.Hkv, nsplit_max, dev)
        self.amax_part = torch.zeros(S * ((self.V + 4095) // 4096), dtype=torch.int64, device=dev)
        self.cand = torch.zeros(S * ((self.V + 2047) // 2048) * 64, dtype=torch.int64, device=dev)
        # norm-free decode (TP = 1, gammas folded into wqkv / w_gate_up): the GEMMs read the raw residual
        # stream and scale rows by its RMS; the row sums of squares are produced by the embedding kernel
        # and the o / down residual epilogues into ssq[2l], ssq[2l + 1], ssq[2l + 2]
        self.fused_norm = tps == 1 and all(lw.norms_folded for lw in weights.layers)
        # ... for decode buckets up to this batch: measured on MI355X (rocprofv3 decode-step spans,
        # profiles/rocprof_fused_norm_ab.txt) the norm-free step wins at batch 1 (3B 2k explain 1788 -> 1738 us,
        # 7B 2.77 -> 2.71 ms) but loses at batch 32 for the 3B (2029 -> 2087 us: the residual epilogue's
        # last-arriver tail costs more than the norm launch it replaces); the norm launches stay above it
        # The 3B (hidden 3072) lost it again in round 2 once its o / down residual epilogues were re-measured
        # inside the step: 192 output blocks per row-parallel GEMM leave CUs idle without split-K, and split-K
        # adds the last-arriver tail (3B 2k explain 1.733 vs 1.708 ms per step norm-free vs norm launches,
        # 7B b1 2.625 vs 2.69 ms) -- so the default is per hidden size
        # (o / down as non-split residual GEMMs on the decode block's ring engine (ops.res_gemm, removed in round 4), in the norm-free
        # step at batch 32 measured slower than the split-K GEMMs + norm launches: 7B 3.77 vs 3.49 ms per step,
        # profiles/r3/res_ring_ab_mi355x.txt -- a standalone full-K stream cannot ramp 128-352 KB per CU fast
        # enough with <= 63 KB of LDS-DMA in flight per loader wave; not wired in)
        self.fused_norm_max_batch = 16 if self.d >= 4096 else 0
        self.res_cfg = None  # experiment hook: (nb, splitk, waves, div) of the norm-free step's o / down GEMMs
        self.ssq = torch.zeros(2 * self.L + 2, S, dtype=torch.int64, device=dev)  # Q24 fixed point (ops.ss_q24)
        # arrival counters of the split-K residual epilogues (one per 16 output columns; left zeroed)
        self.res_tickets = torch.zeros(max(64, self.d // 16), dtype=torch.int32, device=dev)
        # buckets that keep the norm launches (above fused_norm_max_batch): the norms as WIDE raw residual adds
        # (ops.res_add_ss: one wave per 512-column slice, Q24 row sums of squares by integer atomics) with the RMS
        # scaling moved into the qkv / gate_up GEMMs (rownorm; gammas folded into their weights) instead of one
        # 512-thread workgroup per row with a block reduction.  TP = 1; not with W8A8 inputs (their e4m3
        # quantisation needs the whole-row amax in the norm launch) or the MLP residual epilogue
        # Under TP the residual add rides in the one-shot all-reduce (TPGroup.reduce_add: the sum over ranks, h +=,
        # bf16 / fragment-major xn and the row sums in one launch), so a TP layer issues as many launches as TP = 1.
        self.wide_norm = all(lw.norms_folded for lw in weights.layers)
        # batch-1 residual-reduce step (_decode_step_rr): the qkv and gate_up GEMMs fold the residual add of the
        # previous row-parallel projection's slabs into their prologue (ops.linear_rr), so a layer issues 5 launches
        # (qkv, attention, o, gate_up, down) and no residual-add launch; TP = 1, bf16 weights, gammas folded
        self._plan_rr()
        self.zero_slab = torch.zeros(1, 1, self.d, **f32)  # layer 0's "previous projection" in the W8A8 RR step
        self.h_alt = torch.zeros(1, self.d, **f32)  # the residual stream's second buffer (h_out never aliases h)
        self.graphs: dict = {}
        self._pending_bt: dict = {}  # slot -> block-table row of a prompt still being prefilled in chunks
        if self.tp is not None and self.tp.size > 1 and self.on_gpu:
            self.tp.warmup()  # communicators (RCCL + the one-shot IPC all-reduce) before any launch
            if not self.tp.capturable():  # gloo without the IPC kernel (test boxes): eager decode steps
                self.use_graphs = False

    # ------------------------------------------------------------------------------------ helpers
    def _kv_scales(self, l: int):
        """(ks, vs) scale tensors of layer l's fp8 cache, None for a bf16 cache."""
        return (self.kv_scale[l, 0], self.kv_scale[l, 1]) if self.kv_fp8 else None

    def _reduce_add(self, parts: torch.Tensor, h: torch.Tensor, xn: torch.Tensor, ss: torch.Tensor, B: int,
                    xf: bool) -> None:
        """Wide residual add of a row-parallel projection's split-K slabs (+ the TP all-reduce, fused on the IPC
        kernel): h[:B] += sum; xn = bf16(h); ss[:B] += row sums of h^2."""
        if self.tp is None or self.tp.size == 1:
            ops.res_add_ss(h, parts, xn, B, ss, xf=xf)
        else:
            self.tp.reduce_add(parts, self.h, xn, ss, B, xf=xf)

    def _reduce_parts(self, parts: torch.Tensor) -> torch.Tensor:
        """TP all-reduce of a row-parallel GEMM's split-K slabs; returns what the next add_rmsnorm sums."""
        if self.tp is None or self.tp.size == 1:
            return parts
        return self.tp.reduce_parts(parts)

    def _splitk(self, M: int, K: int, N: Optional[int] = None, tp_reduced: bool = True, xf: bool = False) -> int:
        if not self.on_gpu:
            return 1
        if M > 64:  # prefill: split-K on small tile grids; TP prefill reduces single slabs over RCCL
            return 1 if (self.tp is not None and self.tp.size > 1) else ops.tile_splitk(
                M, N or self.d, K, self.w.layers[0].wo.kind)
        if tp_reduced and self.tp is not None and self.tp.size > 1 and not self.tp.can_fold_splitk(M * self.d):
            return 1  # RCCL reduces one slab; the one-shot kernel folds split-K slabs into the all-reduce
        return ops.pick_gemm_config(M, N or self.d, K, "f32", xf=xf, kind=self.w.layers[0].wo.kind)[1]

    def a8_plan(self, B: int) -> tuple[bool, bool, bool, bool]:
        """Which decode projections run W8A8 / W4A8 (e4m3 activations) at bucket B: (qkv, gate_up, o, down)."""
        if not self.a8 or B > 64:
            return (False, False, False, False)
        qkv, gu, od = B > self.a8_min_batch, B > self.a8_mlp_min_batch, B <= self.a8_od_max_batch
        return (qkv, gu, od, gu and od and self.a8_down_ok)

    def _plan_rr(self) -> None:
        """rr_a8 / rr_decode from the current a8 buckets (``set_a8_buckets`` re-plans)."""
        lw0 = self.w.layers[0]
        # quantised weights whose batch-1 step runs all four projections W8A8 / W4A8 (MXFP4): the qkv / gate_up GEMMs
        # quantise their own residual-reduced input (ops.linear_a8_rr), so the two quantising norm launches go too
        self.rr_a8 = all(self.a8_plan(1)) and ops.rr_a8_supported(lw0.wqkv, self.d) and ops.rr_a8_supported(
            lw0.w_gate_up, self.d) and self._a8_splitk_b1() <= 4  # the prologue sums at most 4 slabs
        tps = 1 if self.tp is None else self.tp.size
        self.rr_decode = (RR_DECODE and tps == 1 and self.wide_norm and (self.rr_a8 or (
            ops.rr_supported(lw0.wqkv, self.d) and ops.rr_supported(lw0.w_gate_up, self.d))))

    def set_a8_buckets(self, min_batch: int, mlp_min_batch: int, od_max_batch: int) -> None:
        """Re-plan which decode buckets run W8A8 / W4A8 (``a8_plan``) and the batch-1 residual-reduce step; drops
        captured graphs."""
        self.a8_min_batch, self.a8_mlp_min_batch, self.a8_od_max_batch = min_batch, mlp_min_batch, od_max_batch
        self._plan_rr()
        self.graphs.clear()

    def _a8_splitk_b1(self) -> int:
        """The larger split-K of the batch-1 W8A8 / W4A8 o and down GEMMs (the slabs a residual-reduce prologue sums;
        e.g. MXFP4 Llama-3.2-3B picks 8 and keeps the norm-launch step)."""
        kind = self.w.layers[0].wqkv.kind
        if kind not in ("fp8", "mxfp4"):
            return 1
        ak = "fp8a" if kind == "fp8" else "fp4a"
        return max(ops.pick_gemm_config(1, self.d, K, "f32", xf=True, kind=ak)[1] for K in (self.H * self.D, self.ffn_l))

    def oracle_plan(self, B: int) -> dict:
        """a8_plan(B) as the numerics oracle's ``decode_a8`` dict (models/llama.py reference_forward), plus ``rr``:
        the batch-1 residual-reduce step of fp8 / MXFP4 weights quantises the qkv / gate_up inputs per 32-block
        (E8M0) from the raw residual and applies the RMS row scale after the GEMM (_decode_step_rr)."""
        plan = dict(zip(("qkv", "gate_up", "o", "down"), self.a8_plan(B)))
        plan["rr"] = B == 1 and self.rr_decode and self.rr_a8
        return plan

    def use_xfrag(self, B: int) -> bool:
        """Fragment-major activations pay off once a decode batch spans >1 row tile (B > 16):
        measured 8-20 % faster GEMMs at B = 32 (scripts/bench_xf.py); bf16 and fp8 weights."""
        return self.on_gpu and 16 < B <= 64 and self.w.layers[0].wqkv.kind in ("bf16", "fp8", "mxfp4")

    def _lm_head(self, xn: torch.Tensor, M: int, xf: bool = False) -> torch.Tensor:
        """logits [M, V] (f32) for the normalised rows xn [M, d] (fragment-major when xf)."""
        loc = self.logits_l[:M] if M <= self.max_slots else torch.empty(M, self.Vl, dtype=torch.float32,
                                                                         device=self.device)
        if xf:
            ops.linear_xf(xn, M, self.w.lm_head, "f32", out=loc, splitk=1)
        else:
            ops.linear(xn, self.w.lm_head, "f32", out=loc, splitk=1)
        return self._gather_logits(loc, M)

    def _gather_logits(self, loc: torch.Tensor, M: int) -> torch.Tensor:
        """vocab-parallel logits -> full [M, V] (all-gather over the TP group)."""
        if self.tp is None or self.tp.size == 1:
            return loc
        tps = self.tp.size
        gb = self.gather_buf[: tps * M * self.Vl] if M <= self.max_slots else torch.empty(
            tps * M * self.Vl, dtype=torch.float32, device=self.device)
        self.tp.all_gather(gb, loc.reshape(-1))
        full = self.logits[:M] if M <= self.max_slots else torch.empty(M, self.V, dtype=torch.float32,
                                                                      device=self.device)
        full.view(M, tps, self.Vl).copy_(gb.view(tps, M, self.Vl).transpose(0, 1))
        return full

    # ------------------------------------------------------------------------------------ decode
    def ctx_plan(self, B: int, max_ctx: Optional[int] = None) -> tuple[int, int]:
        """Split-KV grid plan for a decode run whose contexts stay <= max_ctx.  Contexts are rounded up to
        a power-of-two tier (>= 256) so only a few plans (= captured graphs) exist per bucket.  Any plan is
        correct for any context (the kernel widens its splits); the tier only avoids launching split
        workgroups that short contexts leave empty: B = 32 at ctx 200 costs 24 us planned for 512 keys,
        31 us for 4096 and 42 us for 8192 (scripts/attn_scaling.py)."""
        t = self.max_model_len if max_ctx is None else min(self.max_model_len, max(256, max_ctx))
        tier = 256
        while tier < t:
            tier *= 2
        tier = min(tier, self.max_model_len)
        return tuple(ops.decode_split_plan(B, self.Hkv, tier))

    def _decode_step(self, B: int, sample: bool, plan: Optional[tuple] = None) -> None:
        a8, a8m, a8o, a8d = self.a8_plan(B)  # qkv / gate_up / o / down W8A8 (W4A8)
        if B == 1 and self.rr_decode and (self.rr_a8 or not (a8 or a8m or a8o)):
            return self._decode_step_rr(sample, plan)
        if self.fused_norm and B <= self.fused_norm_max_batch and not (a8 or a8m or a8o):
            return self._decode_step_fused(B, sample, plan)
        w, d = self.w, self.d
        ids, pos, bt = self.input_ids[:B], self.positions[:B], self.block_tables[:B]
        h = self.h[:B]
        # e4m3 activations live in the xf8 layout: every GEMM input of the step is then fragment-major
        xf = self.step_xfrag(B)
        ak = "fp8a" if w.layers[0].wo.kind == "fp8" else "fp4a"
        sk_o = (self._splitk(B, self.H * self.D, xf=xf) if not a8o else
                ops.pick_gemm_config(B, d, self.H * self.D, "f32", xf=True, kind=ak)[1])
        sk_d = (self._splitk(B, self.ffn_l, xf=xf) if not a8d else
                ops.pick_gemm_config(B, d, self.ffn_l, "f32", xf=True, kind=ak)[1])
        nqkv = (self.H + 2 * self.Hkv) * self.D
        sk_q = (ops.pick_gemm_config(B, nqkv, d, "f32", xf=True, kind=ak)[1] if a8
                else self._splitk(B, d, nqkv, tp_reduced=False, xf=xf))
        q8 = dict(x8=self.x8, sx8=self.sx8) if a8 else {}
        q8m = dict(x8=self.x8, sx8=self.sx8) if a8m else {}
        # each side of the layer: a wide residual add + row scale in the next GEMM unless that GEMM runs W8A8 (its
        # e4m3 input comes from the quantising norm launch)
        wna = self.wide_norm and not a8
        wnm = self.wide_norm and not a8m
        # the embedding launch writes raw rows + row sums and zeroes every later accumulator whenever any side uses them
        # (layer 0's qkv then row-scales, whatever its later layers do)
        raw0 = wna or wnm
        ssq = self.ssq
        rn_a = lambda l: dict(rownorm=(ssq[2 * l], self.eps)) if (wna or (l == 0 and raw0)) else {}  # noqa: E731
        assert not (a8 and wna), "a W8A8 qkv input comes from the quantising norm launch"
        rn_m = lambda l: dict(rownorm=(ssq[2 * l + 1], self.eps)) if wnm else {}  # noqa: E731
        o_parts = self.o_buf[: sk_o * B * d].view(sk_o, B, d)
        d_parts = self.down_buf[: sk_d * B * d].view(sk_d, B, d)
        qkv_parts = self.qkv_buf[: sk_q * B * nqkv].view(sk_q, B, nqkv)
        plan = plan or ops.decode_split_plan(B, self.Hkv, self.max_model_len)
        ws = self.attn_ws
        if xf:  # every GEMM input lives in the fragment-major layout, written by its producer
            xn, attn, act = self.xn_f, self.attn_f, self.act_f

            def lin(x, wt, epi, **kw):
                return ops.linear_xf(x, B, wt, epi, **kw)
        else:
            xn, attn, act = self.xn[:B], self.attn[:B], self.act[:B]
            lin = ops.linear
        for l, lw in enumerate(w.layers):
            if l == 0 and raw0:
                ops.add_rmsnorm(h, lw.attn_norm, self.eps, xn, ids=ids, emb=w.embed, rows=B, xf=xf,
                                ss_out=ssq.view(-1), ss_ld=self.max_slots, ss_nzero=2 * self.L, **q8)
            elif l == 0:
                ops.add_rmsnorm(h, lw.attn_norm, self.eps, xn, ids=ids, emb=w.embed, rows=B, xf=xf, **q8)
            elif wna:
                self._reduce_add(d_parts, h, xn, ssq[2 * l], B, xf)
            else:
                ops.add_rmsnorm(h, lw.attn_norm, self.eps, xn, parts=self._reduce_parts(d_parts), rows=B, xf=xf, **q8)
            # QKV as f32 split-K slabs; the attention kernel sums them, applies RoPE and appends the new
            # token's k/v to the paged cache itself (no separate rope/append launch)
            if a8:  # (layer 0 after a raw embedding launch: its e4m3 rows are un-normalised -> row scale)
                ops.linear_a8(self.x8, self.sx8, B, lw.wqkv, "f32", out=qkv_parts, splitk=sk_q, **rn_a(l))
            else:
                lin(xn, lw.wqkv, "f32", out=qkv_parts, splitk=sk_q, **rn_a(l))
            kc, vc = self.kv[l, 0], self.kv[l, 1]
            if not self.fuse_rope:
                ops.rope_append(qkv_parts, pos, None, bt, self.cos, self.sin, self.q[:B], kc, vc, self.H, self.Hkv,
                                kv_scales=self._kv_scales(l))
            fr = self.fuse_rope
            ops.attn_decode(self.q[:B], kc, vc, bt, pos, self.H, self.Hkv, self.scale,
                            (self.x8o if a8o else attn) if xf else attn.view(B, self.H, self.D), workspace=ws,
                            plan=plan, xf=xf, qkv_parts=qkv_parts if fr else None, cos=self.cos if fr else None,
                            sin=self.sin if fr else None, kv_scales=self._kv_scales(l),
                            out_s8=self.s8o if a8o else None)
            if a8o:
                ops.linear_a8(self.x8o, None, B, lw.wo, "f32", out=o_parts, splitk=sk_o, s8=self.s8o)
            else:
                lin(attn, lw.wo, "f32", out=o_parts, splitk=sk_o)
            if wnm:
                self._reduce_add(o_parts, h, xn, ssq[2 * l + 1], B, xf)
            else:
                ops.add_rmsnorm(h, lw.mlp_norm, self.eps, xn, parts=self._reduce_parts(o_parts), rows=B, xf=xf, **q8m)
            if a8m:
                ops.linear_a8(self.x8, self.sx8, B, lw.w_gate_up, "silu", out=self.x8d if a8d else act,
                              out_s8=self.s8d if a8d else None)
            else:
                lin(xn, lw.w_gate_up, "silu", out=act, **rn_m(l))
            if a8d:
                ops.linear_a8(self.x8d, None, B, lw.w_down, "f32", out=d_parts, splitk=sk_d, s8=self.s8d)
            else:
                lin(act, lw.w_down, "f32", out=d_parts, splitk=sk_d)
        ops.add_rmsnorm(h, w.final_norm, self.eps, xn, parts=self._reduce_parts(d_parts), rows=B, xf=xf)
        self._decode_tail(B, sample, xn, xf)

    def _decode_step_fused(self, B: int, sample: bool, plan: Optional[tuple] = None) -> None:
        """Norm-free decode step (TP = 1): 5 launches per layer instead of 7.

          embed (+ row sum of squares)  ->  per layer:
            gemm qkv (rows scaled by rsqrt(ss/d + eps), f32 split-K slabs) -> attn_decode (RoPE + KV append)
            -> gemm o (residual epilogue: h += y, x = bf16(h), ss += h^2)
            -> gemm gate_up (row-scaled, SiLU*up) -> gemm down (residual epilogue)
          -> final RMSNorm -> lm_head -> token commit
        """
        w, d = self.w, self.d
        ids, pos, bt = self.input_ids[:B], self.positions[:B], self.block_tables[:B]
        h = self.h[:B]
        xf = self.use_xfrag(B)
        nqkv = (self.H + 2 * self.Hkv) * self.D
        sk_q = self._splitk(B, d, nqkv, tp_reduced=False, xf=xf)
        # the residual-epilogue GEMMs run their own tuned split (ops/gemm_tuning.json "res" entries; the
        # f32 pick where none is tuned)
        sk_o = ops.pick_gemm_config(B, d, self.H * self.D, "res", xf=xf, kind=w.layers[0].wo.kind)[1]
        sk_d = ops.pick_gemm_config(B, d, self.ffn_l, "res", xf=xf, kind=w.layers[0].w_down.kind)[1]
        rc = {}
        if self.res_cfg is not None:  # experiment override (bench.py --set res_cfg=(nb,splitk,waves,div))
            nb_, sk_o, wv_, dv_ = self.res_cfg
            sk_d = sk_o
            rc = dict(nb=nb_, waves=wv_, div=dv_)
        qkv_parts = self.qkv_buf[: sk_q * B * nqkv].view(sk_q, B, nqkv)
        o_parts = self.o_buf[: sk_o * B * d].view(sk_o, B, d)
        d_parts = self.down_buf[: sk_d * B * d].view(sk_d, B, d)
        plan = plan or ops.decode_split_plan(B, self.Hkv, self.max_model_len)
        ws = self.attn_ws
        ssq, S, tk = self.ssq, self.max_slots, self.res_tickets
        if xf:
            xn, attn, act = self.xn_f, self.attn_f, self.act_f

            def lin(x, wt, epi, **kw):
                return ops.linear_xf(x, B, wt, epi, **kw)
        else:
            xn, attn, act = self.xn[:B], self.attn[:B], self.act[:B]
            lin = ops.linear
        ops.add_rmsnorm(h, w.layers[0].attn_norm, self.eps, xn, ids=ids, emb=w.embed, rows=B, xf=xf,
                        ss_out=ssq.view(-1), ss_ld=S, ss_nzero=2 * self.L)
        for l, lw in enumerate(w.layers):
            lin(xn, lw.wqkv, "f32", out=qkv_parts, splitk=sk_q, rownorm=(ssq[2 * l], self.eps))
            kc, vc = self.kv[l, 0], self.kv[l, 1]
            ops.attn_decode(self.q[:B], kc, vc, bt, pos, self.H, self.Hkv, self.scale,
                            attn if xf else attn.view(B, self.H, self.D), workspace=ws, plan=plan, xf=xf,
                            qkv_parts=qkv_parts, cos=self.cos, sin=self.sin, kv_scales=self._kv_scales(l))
            lin(attn, lw.wo, "res", out=o_parts, splitk=sk_o, res=(h, xn, ssq[2 * l + 1], tk), **rc)
            lin(xn, lw.w_gate_up, "silu", out=act, rownorm=(ssq[2 * l + 1], self.eps))
            lin(act, lw.w_down, "res", out=d_parts, splitk=sk_d, res=(h, xn, ssq[2 * l + 2], tk), **rc)
        ops.add_rmsnorm(h, w.final_norm, self.eps, xn, rows=B, xf=xf, write_h=False)
        self._decode_tail(B, sample, xn, xf)

    def _decode_step_rr(self, sample: bool, plan: Optional[tuple] = None) -> None:
        """Batch-1 decode step with the residual adds folded into the GEMM prologues (TP = 1, bf16, gammas folded):
        5 launches per layer.

          embed (raw h, bf16(h), sum h^2)  ->  per layer:
            gemm qkv  (layer 0: bf16 x, row-scaled slabs; later layers ops.linear_rr: x = h + sum(down slabs) formed
                       in the prologue, h_out = x, sum x^2 -> ssq[l], unscaled f32 slabs)
            -> attn_decode (slab sum, RMS row scale from ssq[l], RoPE, KV append, split-KV attention)
            -> gemm o (f32 split-K slabs)
            -> gemm gate_up (ops.linear_rr: x = h + sum(o slabs), its own full-row RMS scale, SiLU * up)
            -> gemm down (f32 split-K slabs)
          -> final RMSNorm (h + down slabs) -> lm_head -> token commit
        The residual stream alternates between self.h and self.h_alt (a prologue's other workgroups still read the
        buffer the column-0 workgroups replace).
        With fp8 / MXFP4 weights (``rr_a8``) every projection runs W8A8 / W4A8: qkv and gate_up quantise their
        residual-reduced input themselves (ops.linear_a8_rr; layer 0's qkv reduces the embedding row with a zero
        slab), attention writes the o input as e4m3 + E8M0 per head, gate_up the down input as e4m3 + E8M0 per 32."""
        w, d, B = self.w, self.d, 1
        ids, pos, bt = self.input_ids[:1], self.positions[:1], self.block_tables[:1]
        nqkv = (self.H + 2 * self.Hkv) * self.D
        a8 = self.rr_a8
        if a8:
            ak = "fp8a" if w.layers[0].wqkv.kind == "fp8" else "fp4a"
            sk_q = ops.rr_config(nqkv, d, "f32", w.layers[0].wqkv.kind)[1]
            sk_o = ops.pick_gemm_config(1, d, self.H * self.D, "f32", xf=True, kind=ak)[1]
            sk_d = ops.pick_gemm_config(1, d, self.ffn_l, "f32", xf=True, kind=ak)[1]
        else:
            sk_q = ops.rr_config(nqkv, d, "f32", w.layers[0].wqkv.kind)[1] if self.on_gpu else 1
            sk_o = self._splitk(1, self.H * self.D)
            sk_d = self._splitk(1, self.ffn_l)
        assert sk_o <= 4 and sk_d <= 4, "the residual-reduce prologue sums at most 4 slabs"
        qkv_parts = self.qkv_buf[: sk_q * nqkv].view(sk_q, 1, nqkv)
        o_parts = self.o_buf[: sk_o * d].view(sk_o, 1, d)
        d_parts = self.down_buf[: sk_d * d].view(sk_d, 1, d)
        plan = plan or ops.decode_split_plan(1, self.Hkv, self.max_model_len)
        ssq = self.ssq
        hs = (self.h[:1], self.h_alt)
        cur = 0
        xn, attn, act = self.xn[:1], self.attn[:1], self.act[:1]
        ops.add_rmsnorm(hs[0], w.layers[0].attn_norm, self.eps, xn, ids=ids, emb=w.embed, rows=1,
                        ss_out=ssq.view(-1), ss_ld=self.max_slots, ss_nzero=self.L)
        for l, lw in enumerate(w.layers):
            if a8:  # the qkv input (embedding row | h + down slabs) quantised in the GEMM's prologue
                ops.linear_a8_rr(hs[cur], self.zero_slab if l == 0 else d_parts, hs[1 - cur], lw.wqkv, "f32",
                                 out=qkv_parts, ss_out=ssq[l + 1], eps=self.eps, splitk=sk_q)
                cur = 1 - cur
                rn = (ssq[l + 1], self.eps, d)
            elif l == 0:
                ops.linear(xn, lw.wqkv, "f32", out=qkv_parts, splitk=sk_q, rownorm=(ssq[0], self.eps))
                rn = None
            else:
                ops.linear_rr(hs[cur], d_parts, hs[1 - cur], lw.wqkv, "f32", out=qkv_parts, ss_out=ssq[l + 1],
                              eps=self.eps, splitk=sk_q)
                cur = 1 - cur
                rn = (ssq[l + 1], self.eps, d)
            kc, vc = self.kv[l, 0], self.kv[l, 1]
            if a8:
                ops.attn_decode(self.q[:1], kc, vc, bt, pos, self.H, self.Hkv, self.scale, self.x8o, workspace=self.attn_ws,
                                plan=plan, xf=True, qkv_parts=qkv_parts, cos=self.cos, sin=self.sin,
                                kv_scales=self._kv_scales(l), out_s8=self.s8o, rownorm=rn)
                ops.linear_a8(self.x8o, None, 1, lw.wo, "f32", out=o_parts, splitk=sk_o, s8=self.s8o)
                ops.linear_a8_rr(hs[cur], o_parts, hs[1 - cur], lw.w_gate_up, "silu", out=self.x8d, out_s8=self.s8d,
                                 eps=self.eps)
                cur = 1 - cur
                ops.linear_a8(self.x8d, None, 1, lw.w_down, "f32", out=d_parts, splitk=sk_d, s8=self.s8d)
                continue
            ops.attn_decode(self.q[:1], kc, vc, bt, pos, self.H, self.Hkv, self.scale, attn.view(1, self.H, self.D),
                            workspace=self.attn_ws, plan=plan, qkv_parts=qkv_parts, cos=self.cos, sin=self.sin,
                            kv_scales=self._kv_scales(l), rownorm=rn)
            ops.linear(attn, lw.wo, "f32", out=o_parts, splitk=sk_o)
            ops.linear_rr(hs[cur], o_parts, hs[1 - cur], lw.w_gate_up, "silu", out=act, eps=self.eps)
            cur = 1 - cur
            ops.linear(act, lw.w_down, "f32", out=d_parts, splitk=sk_d)
        ops.add_rmsnorm(hs[cur], w.final_norm, self.eps, xn, parts=d_parts, rows=1, write_h=False)
        self._decode_tail(B, sample, xn, False)

    def _decode_tail(self, B: int, sample: bool, xn, xf: bool) -> None:
        logits = self._lm_head(xn, B, xf)
        st = (self.out_tokens[:B], self.gen_len[:B], self.input_ids[:B], self.positions[:B], self.finished[:B])
        if sample:
            ops.sample_commit(logits, self.hist[:B], self.penalty[:B], self.temperature[:B], self.top_k[:B],
                              self.top_p[:B], self.seeds[:B], *st, self.eos, self.limit[:B], self.eos_on[:B],
                              workspace=(self.amax_part, self.cand) if self.on_gpu else None,
                              last_n=self.last_n[:B])
        else:
            ops.argmax_commit(logits, *st, self.eos, self.limit[:B], self.eos_on[:B],
                              part=self.amax_part if self.on_gpu else None)

    def final_hidden(self, B: int) -> torch.Tensor:
        """[B, d] bf16: the final-norm output rows of the last decode step (what the lm_head read), in row order
        whatever layout the step's bucket used (the numerics check of tied-embedding models reads it)."""
        if self.step_xfrag(B):
            return ops.from_xfrag(self.xn_f, B, self.d)
        return self.xn[:B]

    def step_xfrag(self, B: int) -> bool:
        """Whether the decode step of bucket B hands its activations on in the fragment-major layouts (use_xfrag,
        or -- any W8A8 / W4A8 projection -- the xf8 one, which forces it at any batch)."""
        a8, a8m, a8o, _ = self.a8_plan(B)
        return self.use_xfrag(B) or a8 or a8m or a8o

    def bucket(self, n: int) -> int:
        b = 1
        while b < n:
            b *= 2
        return min(b, self.max_slots) if n <= self.max_slots else self.max_slots

    def capture(self, B: int, sample: bool, plan: Optional[tuple] = None) -> None:
        """Capture the decode-step graph of (bucket, sampling mode, split plan).  (Several steps per graph were
        measured no faster -- no idle time at graph boundaries, profiles/decode_b32_normfree_spg_ab_mi355x.txt.)"""
        plan = tuple(plan or self.ctx_plan(B))
        key = (B, sample, plan)
        if key in self.graphs:
            return
        if self.tp is not None and self.tp.size > 1:
            self.tp.warmup()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            # state must not change during capture: kernels are recorded, not executed
            with torch.cuda.graph(g, stream=s):
                self._decode_step(B, sample, plan)
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graphs[key] = g

    def count_step_kernels(self, B: int, sample: bool = False) -> int:
        """Kernel launches of one captured decode step of bucket B (a throw-away capture whose graph is kept and
        walked with hipGraphGetNodes): the launch-count check of the fused TP step (tests/test_tp_launches_gpu.py)."""
        import ctypes

        assert self.use_graphs, "needs graph capture"
        plan = tuple(self.ctx_plan(B))
        if self.tp is not None and self.tp.size > 1:
            self.tp.warmup()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self._decode_step(B, sample, plan)
        torch.cuda.current_stream(self.device).wait_stream(s)
        lib = ctypes.CDLL("libamdhip64.so")
        graph = ctypes.c_void_p(g.raw_cuda_graph())
        n = ctypes.c_size_t(0)
        assert lib.hipGraphGetNodes(graph, None, ctypes.byref(n)) == 0
        nodes = (ctypes.c_void_p * n.value)()
        assert lib.hipGraphGetNodes(graph, nodes, ctypes.byref(n)) == 0
        kernels = 0
        for nd in nodes:
            t = ctypes.c_int(-1)
            assert lib.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t)) == 0
            kernels += t.value == 0  # hipGraphNodeTypeKernel
        g.reset()
        return kernels

    def buckets(self) -> list[int]:
        out, b = [], 1
        while b < self.max_slots:
            out.append(b)
            b *= 2
        return out + [self.max_slots]

    def plans(self, B: int) -> list[tuple]:
        """Distinct split plans over the context tiers 256, 512, ... max_model_len."""
        out, t = [], 256
        while True:
            p = self.ctx_plan(B, t)
            if p not in out:
                out.append(p)
            if t >= self.max_model_len:
                return out
            t *= 2

    def capture_all(self, sample_modes: Sequence[bool] = (False, True)) -> None:
        """Capture every (bucket, sampling mode, context tier) decode graph up front, so a server never
        pays a capture inside a request."""
        if not self.use_graphs:
            return
        for b in self.buckets():
            for sm in sample_modes:
                for p in self.plans(b):
                    self.capture(b, sm, p)
        torch.cuda.synchronize(self.device)

    def decode(self, B: int, steps: int, sample: bool = False, max_ctx: Optional[int] = None) -> None:
        """Run ``steps`` decode steps over slot rows [0, B) (B a bucket size); ``max_ctx`` bounds every
        row's context length during the run (picks the graph planned for that tier)."""
        plan = tuple(self.ctx_plan(B, max_ctx))
        if not self.use_graphs:
            for _ in range(steps):
                self._decode_step(B, sample, plan)
            return
        self.capture(B, sample, plan)
        g = self.graphs[(B, sample, plan)]
        for _ in range(steps):
            g.replay()

    # ------------------------------------------------------------------------------------ slots
    def set_slot(self, slot: int, blocks: Sequence[int], limit: int, temperature: float = 0.0, top_k: int = 40,
                 top_p: float = 0.9, seed: int = 0, eos_on: bool = True, repeat_penalty: float = 1.0,
                 repeat_last_n: int = REPEAT_WINDOW, prompt_ids: Sequence[int] = (), defer_table: bool = False) -> None:
        """``defer_table``: the slot's block table stays out of the decode-visible table until its prompt's
        final prefill chunk commits (chunked-prefill interleave: decode runs in between must not append
        the idle row's k/v into the blocks the prompt is being written to)."""
        self.set_slots([dict(slot=slot, blocks=blocks, limit=limit, temperature=temperature, top_k=top_k, top_p=top_p,
                             seed=seed, eos_on=eos_on, repeat_penalty=repeat_penalty, repeat_last_n=repeat_last_n,
                             prompt_ids=prompt_ids, defer_table=defer_table)])

    def set_slots(self, entries: Sequence[dict]) -> None:
        """``set_slot`` for every admitted request at once (keyword dicts of set_slot's arguments): the per-slot
        parameters travel host -> device in ONE pinned int32 + one f32 + one int64 transfer and land with one
        index_copy per state tensor, instead of ~11 tiny copies / fills per slot (a 32-request bench round's
        admission was ~350 small launches of host time with the GPU idle)."""
        if not entries:
            return
        n, W, mb = len(entries), REPEAT_WINDOW, self.max_blocks
        ints = torch.zeros(n, mb + 5, dtype=torch.int32)  # block-table row | limit top_k eos_on last_n visible
        flts = torch.zeros(n, 3, dtype=torch.float32)     # temperature top_p penalty
        seeds = torch.zeros(n, dtype=torch.int64)
        hist = None
        for i, e in enumerate(entries):
            blocks = list(e["blocks"])
            ints[i, : len(blocks)] = torch.tensor(blocks, dtype=torch.int32)
            last_n = max(0, min(int(e.get("repeat_last_n", REPEAT_WINDOW)), W))
            ints[i, mb:] = torch.tensor([min(int(e["limit"]), self.max_new_cap), int(e.get("top_k", 40)),
                                         1 if e.get("eos_on", True) else 0, last_n,
                                         0 if e.get("defer_table", False) else 1], dtype=torch.int32)
            flts[i] = torch.tensor([float(e.get("temperature", 0.0)), float(e.get("top_p", 0.9)),
                                    float(e.get("repeat_penalty", 1.0))])
            seeds[i] = int(e.get("seed", 0))
            if float(e.get("repeat_penalty", 1.0)) != 1.0:  # seed the ring with the prompt's last tokens (p -> p % W)
                if hist is None:
                    hist = torch.full((n, W), -1, dtype=torch.int32)
                ids = list(e.get("prompt_ids", ()))
                for p in range(max(0, len(ids) - W), len(ids)):
                    hist[i, p % W] = int(ids[p])
        if self.on_gpu:
            ints, flts, seeds = ints.pin_memory(), flts.pin_memory(), seeds.pin_memory()
        dv = ints.to(self.device, non_blocking=True)
        fv = flts.to(self.device, non_blocking=True)
        sv = seeds.to(self.device, non_blocking=True)
        slots = [int(e["slot"]) for e in entries]
        idx = torch.tensor(slots, dtype=torch.long).to(self.device, non_blocking=True)
        visible = ints[:, mb + 4].tolist()
        for i, sl in enumerate(slots):
            if visible[i]:
                self._pending_bt.pop(sl, None)
            else:
                self._pending_bt[sl] = dv[i, :mb].clone()
        self.block_tables.index_copy_(0, idx, dv[:, :mb] * dv[:, mb + 4:mb + 5])  # deferred rows stay zero
        self.limit.index_copy_(0, idx, dv[:, mb])
        self.top_k.index_copy_(0, idx, dv[:, mb + 1])
        self.eos_on.index_copy_(0, idx, dv[:, mb + 2])
        self.last_n.index_copy_(0, idx, dv[:, mb + 3])
        self.temperature.index_copy_(0, idx, fv[:, 0])
        self.top_p.index_copy_(0, idx, fv[:, 1])
        self.penalty.index_copy_(0, idx, fv[:, 2])
        self.seeds.index_copy_(0, idx, sv)
        if hist is not None:
            hv = hist.pin_memory() if self.on_gpu else hist
            hsel = torch.tensor([i for i, e in enumerate(entries) if float(e.get("repeat_penalty", 1.0)) != 1.0],
                                dtype=torch.long)
            self.hist.index_copy_(0, idx[hsel.to(self.device)], hv[hsel].to(self.device, non_blocking=True))

    def extend_tables(self, entries: Sequence[tuple]) -> None:
        """Lazy KV growth (engine._grow_kv): rewrite the decode-visible block-table rows of running slots,
        ``entries`` = [(slot, blocks)], whose tables gained blocks -- one pinned transfer + one index_copy for all
        of them, between decode runs (a captured graph reads the table from device memory at every replay)."""
        if not entries:
            return
        mb = self.max_blocks
        rows = torch.zeros(len(entries), mb, dtype=torch.int32)
        for i, (_, blocks) in enumerate(entries):
            assert len(blocks) <= mb, "block table longer than max_model_len"
            rows[i, : len(blocks)] = torch.tensor(list(blocks), dtype=torch.int32)
        if self.on_gpu:
            rows = rows.pin_memory()
        idx = torch.tensor([int(sl) for sl, _ in entries], dtype=torch.long)
        for sl, _ in entries:
            assert int(sl) not in self._pending_bt, "growing a slot whose prompt is still being prefilled"
        self.block_tables.index_copy_(0, idx.to(self.device, non_blocking=True), rows.to(self.device, non_blocking=True))

    def set_eos(self, ids: Sequence[int]) -> None:
        """Replace the stop-token set (same length keeps captured graphs valid; otherwise recapture)."""
        ids = list(ids) or [-1]
        if len(ids) != self.eos.numel():
            self.graphs.clear()
            self.eos = torch.tensor(ids, dtype=torch.int32, device=self.device)
        else:
            self.eos.copy_(torch.tensor(ids, dtype=torch.int32))
        self.eos_list = ids

    def release_slot(self, slot: int) -> None:
        self._pending_bt.pop(slot, None)
        self.finished[slot] = 1
        self.positions[slot] = 0
        self.gen_len[slot] = 0
        self.block_tables[slot].zero_()

    # ------------------------------------------------------------------------------------ prefill
    def prefill(self, seqs: list[tuple[int, Sequence[int], int]], sample_any: bool = False) -> None:
        """Prefill ``seqs`` = [(slot, token_ids, start_pos)] and commit each first token into its slot.

        ``start_pos`` > 0 continues a chunked prefill (the cache already holds positions < start_pos);
        only the final chunk of a prompt should be passed with ``commit=True`` semantics — a chunk whose
        prompt continues is passed through ``prefill_chunk``.
        """
        self._prefill(seqs, commit=True, sample_any=sample_any)

    def prefill_chunk(self, seqs: list[tuple[int, Sequence[int], int]]) -> None:
        self._prefill(seqs, commit=False)

    def _prefill(self, seqs, commit: bool, sample_any: bool = False) -> None:
        dev, w, d = self.device, self.w, self.d
        n = len(seqs)
        lens = [len(t) for _, t, _ in seqs]
        T = sum(lens)
        cu = [0]
        for x in lens:
            cu.append(cu[-1] + x)
        toks, pos, tseq = [], [], []
        for i, (_, t, p0) in enumerate(seqs):
            toks.extend(int(x) for x in t)
            pos.extend(range(p0, p0 + len(t)))
            tseq.extend([i] * len(t))
        ctx = [p0 + len(t) for _, t, p0 in seqs]
        slots = [s for s, _, _ in seqs]
        host = torch.tensor(toks + pos + tseq + cu + ctx + [c - 1 for c in cu[1:]], dtype=torch.int32)
        if self.on_gpu:
            host = host.pin_memory()
        dv = host.to(dev, non_blocking=True)
        o = 0
        ids = dv[o:o + T]; o += T
        posd = dv[o:o + T]; o += T
        tsd = dv[o:o + T]; o += T
        cud = dv[o:o + n + 1]; o += n + 1
        ctxd = dv[o:o + n]; o += n
        last = dv[o:o + n]
        slot_t = torch.tensor(slots, dtype=torch.long, device=dev)
        bt = self.block_tables.index_select(0, slot_t)
        for i, sl in enumerate(slots):  # deferred tables: prefill writes through them; the commit publishes
            pend = self._pending_bt.get(sl)
            if pend is not None:
                bt[i].copy_(pend)
                if commit:
                    self.block_tables[sl].copy_(pend)
                    del self._pending_bt[sl]
        work = None
        self._cu_host = cu  # host offsets: the prefill attention kernel choice (ops._prefill_kernel)
        # fp8 cache: the bf16 scratch every layer's prefill attention widens its blocks into (ops.kv8_scratch)
        self._kv8_scratch = ops.kv8_scratch(ctx, self.Hkv, dev) if (self.kv_fp8 and self.on_gpu) else None
        if self.on_gpu:
            work = ops.prefill_plan(cu, ctx=ctx, heads=self.H, device=dev)

        tps = self.tp.size if self.tp is not None else 1
        if self.seq_parallel and tps > 1 and T >= self.sp_min_tokens:
            xl = self._prefill_layers_sp(T, ids, posd, tsd, bt, cud, ctxd, last, work, n, commit)
        else:
            xl = self._prefill_layers(T, ids, posd, tsd, bt, cud, ctxd, last, work, n, commit)
        if not commit:
            return
        logits = self._lm_head(xl, n)
        # commit the first generated token of each sequence into its slot row
        i32 = dict(dtype=torch.int32, device=dev)
        out_t = torch.zeros(n, self.max_new_cap, **i32)
        gl = torch.zeros(n, **i32)
        iid = torch.zeros(n, **i32)
        pp = ctxd - 1
        fin = torch.zeros(n, **i32)
        lim = self.limit.index_select(0, slot_t)
        eon = self.eos_on.index_select(0, slot_t)
        if sample_any:
            hist = self.hist.index_select(0, slot_t)
            ops.sample_commit(logits, hist, self.penalty.index_select(0, slot_t),
                              self.temperature.index_select(0, slot_t),
                              self.top_k.index_select(0, slot_t), self.top_p.index_select(0, slot_t),
                              self.seeds.index_select(0, slot_t), out_t, gl, iid, pp, fin, self.eos, lim, eon,
                              last_n=self.last_n.index_select(0, slot_t))
            self.hist.index_copy_(0, slot_t, hist)
        else:
            ops.argmax_commit(logits, out_t, gl, iid, pp, fin, self.eos, lim, eon)
        self.out_tokens.index_copy_(0, slot_t, out_t)
        self.gen_len.index_copy_(0, slot_t, gl)
        self.input_ids.index_copy_(0, slot_t, iid)
        self.positions.index_copy_(0, slot_t, pp)
        self.finished.index_copy_(0, slot_t, fin)

    def _prefill_layers(self, T, ids, posd, tsd, bt, cud, ctxd, last, work, n, commit):
        """Prefill layer stack with full-sequence residuals; returns the last rows' normalised states."""
        dev, w, d = self.device, self.w, self.d
        f32 = dict(dtype=torch.float32, device=dev)
        bf = dict(dtype=torch.bfloat16, device=dev)
        h = torch.empty(T, d, **f32)
        qkv = torch.empty(T, (self.H + 2 * self.Hkv) * self.D, **bf)
        q = torch.empty(T, self.H, self.D, **bf)
        sk_o = self._splitk(T, self.H * self.D)
        sk_d = self._splitk(T, self.ffn_l)
        d_parts = None
        # TP = 1: o / down accumulate into the f32 residual in the stream-K GEMM's epilogue (ops.linear_res), so the
        # norms after them read h alone (no f32 slab written by the GEMM and read back by the add)
        # (stream-K tile kernels: T > 64 rows; shorter chunks take the skinny split-K GEMMs, whose f32 slabs the next
        # add_rmsnorm sums).  The round-5 norm-free variant (the down epilogue also writing bf16(h) + row sums, the qkv
        # GEMM scaling its rows) measured a tie and was removed in round 6 (ARCHITECTURE.md section 4)
        tp1 = self.tp is None or self.tp.size == 1
        res_o = tp1 and T > 64 and ops.res_supported(w.layers[0].wo)
        res_d = tp1 and T > 64 and ops.res_supported(w.layers[0].w_down)
        # fragment-major activations (ops.to_xfrag, ceil(T / 16) row tiles): the norms, the attention and the gate_up
        # SiLU epilogue write every stream-K GEMM input in the order the GEMM stages it, one contiguous KiB per MFMA
        # fragment (ops.PREFILL_XF)
        xfp = res_o and res_d and ops.PREFILL_XF
        rows = T if xfp else None
        mt16 = 16 * ops.xfrag_tiles(T)
        xn = torch.empty(mt16 * d, **bf) if xfp else torch.empty(T, d, **bf)
        attn = torch.empty(mt16 * self.H * self.D, **bf) if xfp else torch.empty(T, self.H * self.D, **bf)
        act = torch.empty(mt16 * (w.layers[0].w_gate_up.N // 2), **bf) if xfp else None
        for l, lw in enumerate(w.layers):
            if l == 0:
                ops.add_rmsnorm(h, lw.attn_norm, self.eps, xn, ids=ids, emb=w.embed, rows=rows, xf=xfp)
            else:
                ops.add_rmsnorm(h, lw.attn_norm, self.eps, xn, parts=d_parts, write_h=not res_d, rows=rows, xf=xfp)
            self._prefill_attention(xn, lw, l, qkv, q, attn, posd, tsd, bt, cud, ctxd, work, T, xfp)
            if res_o:
                ops.linear_res(attn, lw.wo, h, rows=rows)
                ops.add_rmsnorm(h, lw.mlp_norm, self.eps, xn, write_h=False, rows=rows, xf=xfp)
            else:
                o_parts = ops.linear(attn, lw.wo, "f32", splitk=sk_o)
                if not self.on_gpu:
                    o_parts = o_parts.view(1, T, d)
                o_parts = self._reduce_parts(o_parts)
                ops.add_rmsnorm(h, lw.mlp_norm, self.eps, xn, parts=o_parts)
            sk_g = self._splitk(T, self.d, lw.w_gate_up.N)
            if xfp:
                ops.linear_sk(xn, lw.w_gate_up, "silu", act, rows=T, xf_out=True)
            elif sk_g > 1:  # small tile grid: f32 split-K slabs, then silu(gate) * up over the slabs
                act = ops.silu_parts(ops.linear(xn, lw.w_gate_up, "f32", splitk=sk_g),
                                     torch.empty(T, lw.w_gate_up.N // 2, **bf))
            else:
                act = ops.linear(xn, lw.w_gate_up, "silu")
            if res_d:
                ops.linear_res(act, lw.w_down, h, rows=rows)
                d_parts = None
            else:
                d_parts = ops.linear(act, lw.w_down, "f32", splitk=sk_d)
                if not self.on_gpu:
                    d_parts = d_parts.view(1, T, d)
                d_parts = self._reduce_parts(d_parts)
        if not commit:
            return None
        xl = torch.empty(n, d, **bf)
        ops.add_rmsnorm(h, w.final_norm, self.eps, xl, parts=d_parts, row_idx=last, write_h=False)
        return xl

    def _prefill_attention(self, xn, lw, l, qkv, q, attn, posd, tsd, bt, cud, ctxd, work, T, xf=False):
        """qkv projection + RoPE + KV-cache append + causal attention of one prefill layer.  xf: xn and attn are
        flat fragment-major buffers of T rows (``_prefill_layers``)."""
        kc, vc = self.kv[l, 0], self.kv[l, 1]
        kvs = self._kv_scales(l)
        rows = T if xf else None
        out = attn if xf else attn.view(T, self.H, self.D)
        akw = dict(work=work, cu_list=self._cu_host, kv_scales=kvs, kv8_scratch_=self._kv8_scratch, xf=xf)
        if self.on_gpu and ops.rope_fusable(lw.wqkv, self.kv_fp8, T) and bt.shape[1] > 0:
            # RoPE + the KV-cache append in the qkv GEMM's epilogue: no qkv round trip, no rope_append launch
            ops.linear_rope(xn, lw.wqkv, posd, tsd, bt, self.cos, self.sin, q, kc, vc, self.H, self.Hkv, rows=rows)
            ops.attn_prefill(q, kc, vc, bt, cud, ctxd, self.H, self.Hkv, self.scale, out, **akw)
            return
        sk_q = self._splitk(T, self.d, (self.H + 2 * self.Hkv) * self.D)
        if xf:
            ops.linear_sk(xn, lw.wqkv, "bf16", qkv, rows=T)
            ops.rope_append(qkv, posd, tsd, bt, self.cos, self.sin, q, kc, vc, self.H, self.Hkv, kv_scales=kvs)
        elif sk_q > 1:  # small tile grid: f32 split-K slabs, summed by rope_append while it rotates
            parts = ops.linear(xn, lw.wqkv, "f32", splitk=sk_q)
            ops.rope_append(parts, posd, tsd, bt, self.cos, self.sin, q, kc, vc, self.H, self.Hkv, kv_scales=kvs)
        else:
            ops.linear(xn, lw.wqkv, "bf16", out=qkv)
            ops.rope_append(qkv, posd, tsd, bt, self.cos, self.sin, q, kc, vc, self.H, self.Hkv, kv_scales=kvs)
        ops.attn_prefill(q, kc, vc, bt, cud, ctxd, self.H, self.Hkv, self.scale, out, **akw)

    def _prefill_layers_sp(self, T, ids, posd, tsd, bt, cud, ctxd, last, work, n, commit):
        """Sequence-parallel prefill under TP: rank r owns rows [r*Tl, (r+1)*Tl) of the residual stream.
        Row-parallel outputs (O, down; [Tp, d], bf16 when ``sp_bf16`` else f32) are reduce-scattered instead of
        all-reduced, the residual add + RMSNorm runs on the local Tl rows only (in f32), and the bf16 normalised
        rows are all-gathered for the next column-parallel GEMM: with bf16 payloads both collectives move half the
        bytes of an f32 all-reduce's phases, and 1/tp of the norm work.  Rows past T (padding to a multiple of tp)
        are row-independent garbage that is never read back."""
        dev, w, d, tp = self.device, self.w, self.d, self.tp
        f32 = dict(dtype=torch.float32, device=dev)
        bf = dict(dtype=torch.bfloat16, device=dev)
        tps, r = tp.size, tp.rank
        Tl = (T + tps - 1) // tps
        Tp = Tl * tps
        ids_p = ids if Tp == T else torch.cat([ids, torch.zeros(Tp - T, dtype=ids.dtype, device=dev)])
        ids_l = ids_p[r * Tl:(r + 1) * Tl]
        h_l = torch.empty(Tl, d, **f32)
        xn_l = torch.empty(Tl, d, **bf)
        xn_full = torch.empty(Tp, d, **bf)
        xn = xn_full[:T]
        pay = dict(dtype=torch.bfloat16 if self.sp_bf16 else torch.float32, device=dev)
        epi = "bf16" if self.sp_bf16 else "f32"
        full = torch.zeros(Tp, d, **pay)  # row-parallel GEMM output (padding rows stay zero)
        loc = torch.empty(Tl, d, **f32)
        loc_p = torch.empty(Tl, d, **pay) if self.sp_bf16 else loc

        def rs():  # reduce-scatter of the row-parallel output into this rank's f32 residual slab
            tp.reduce_scatter(loc_p, full)
            if loc_p is not loc:
                loc.copy_(loc_p)

        qkv = torch.empty(T, (self.H + 2 * self.Hkv) * self.D, **bf)
        q = torch.empty(T, self.H, self.D, **bf)
        attn = torch.empty(T, self.H * self.D, **bf)
        parts = loc.view(1, Tl, d)
        for l, lw in enumerate(w.layers):
            if l == 0:
                ops.add_rmsnorm(h_l, lw.attn_norm, self.eps, xn_l, ids=ids_l, emb=w.embed)
            else:
                ops.add_rmsnorm(h_l, lw.attn_norm, self.eps, xn_l, parts=parts)
            tp.all_gather(xn_full.view(-1), xn_l.view(-1))
            self._prefill_attention(xn, lw, l, qkv, q, attn, posd, tsd, bt, cud, ctxd, work, T)
            ops.linear(attn, lw.wo, epi, out=full, splitk=1)
            rs()
            ops.add_rmsnorm(h_l, lw.mlp_norm, self.eps, xn_l, parts=parts)
            tp.all_gather(xn_full.view(-1), xn_l.view(-1))
            act = ops.linear(xn, lw.w_gate_up, "silu")
            ops.linear(act, lw.w_down, epi, out=full, splitk=1)
            rs()
        if not commit:
            return None
        ops.add_rmsnorm(h_l, w.final_norm, self.eps, xn_l, parts=parts)
        tp.all_gather(xn_full.view(-1), xn_l.view(-1))
        return xn_full.index_select(0, last.long())

    # ------------------------------------------------------------------------------------ readback
    def read_rows(self, slots: Sequence[int]):
        """(finished, gen_len, tokens) for ``slots`` (one device->host sync)."""
        idx = torch.tensor(list(slots), dtype=torch.long, device=self.device)
        n = idx.numel()
        parts = [self.finished.index_select(0, idx), self.gen_len.index_select(0, idx)]
        car = getattr(self.tp, "car", None) if self.tp is not None else None
        if car is not None:
            parts.append(car.err)  # one-shot all-reduce timeout flag, read in the same transfer
        host = torch.cat(parts).cpu()
        if car is not None and int(host[2 * n]):
            raise TPCommError("tensor-parallel all-reduce: a peer did not arrive within the timeout; "
                              "this replica's outputs since the last sync are invalid")
        return host[:n], host[n:2 * n], idx

    def tokens_of(self, slot: int, n: int) -> list[int]:
        return self.out_tokens[slot, :n].tolist()

    def tokens_of_many(self, slots: Sequence[int], ns: Sequence[int]) -> list[list[int]]:
        """``tokens_of`` for several rows in one device -> host transfer."""
        if not slots:
            return []
        m = max(ns)
        idx = torch.tensor(list(slots), dtype=torch.long, device=self.device)
        rows = self.out_tokens[:, :m].index_select(0, idx).cpu().tolist()
        return [r[:k] for r, k in zip(rows, ns)]
