"""Llama-family weights in the layouts the gfx950 kernels stream, plus tensor-parallel sharding.

Per layer: ``wqkv`` (fused q|k|v rows, column-parallel), ``wo`` (row-parallel), ``w_gate_up``
(gate/up interleaved per 16 rows for the fused SiLU epilogue, column-parallel), ``w_down``
(row-parallel), two RMSNorm vectors.  Embedding is replicated; the LM head is vocab-parallel.

Sources: seeded random init directly on the device (the benchmark path: the reference's models are
Ollama GGUF blobs we cannot download), a HuggingFace-format state dict (``from_hf_state_dict``),
or safetensors files (``load_safetensors_dir``).  ``kind='fp8'`` quantises every projection to
e4m3fn with per-output-channel scales at load time (BASELINE config 5).
"""
from __future__ import annotations

import dataclasses
import math
import glob
import json
import os
from typing import Optional

import torch

from .. import ops
from .spec import ModelSpec, spec_from_hf_config


# RMSNorm gammas folded into the following projections at load time (FOLD_NORMS = False keeps them apart):
# rmsnorm(x) * g @ W^T == rmsnorm(x) @ (W * g)^T, so wqkv / w_gate_up carry the attention / MLP norm
# weights and the stored norm vectors are ones.  The decode path then needs no norm launch at all: the
# GEMMs read the raw residual stream and scale their output rows by its RMS (engine/runner.py fused path).
FOLD_NORMS = True


@dataclasses.dataclass
class LayerWeights:
    wqkv: ops.PackedWeight
    wo: ops.PackedWeight
    w_gate_up: ops.PackedWeight
    w_down: ops.PackedWeight
    attn_norm: torch.Tensor
    mlp_norm: torch.Tensor
    norms_folded: bool = False


@dataclasses.dataclass
class LlamaWeights:
    spec: ModelSpec
    embed: torch.Tensor  # [V, d] bf16 (replicated)
    layers: list
    final_norm: torch.Tensor
    lm_head: ops.PackedWeight  # [V / tp, d]
    tp_rank: int = 0
    tp_size: int = 1

    @property
    def device(self) -> torch.device:
        return self.embed.device

    def nbytes(self) -> int:
        n = self.embed.numel() * 2 + self.lm_head.nbytes
        for lw in self.layers:
            n += lw.wqkv.nbytes + lw.wo.nbytes + lw.w_gate_up.nbytes + lw.w_down.nbytes
        return n


def _shard_rows(w: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    n = w.shape[0] // size
    return w[rank * n:(rank + 1) * n]


def _shard_cols(w: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    n = w.shape[1] // size
    return w[:, rank * n:(rank + 1) * n]


def check_tp(spec: ModelSpec, tp: int) -> None:
    if spec.n_kv_heads % tp or spec.n_heads % tp:
        raise ValueError(f"{spec.name}: heads {spec.n_heads}/{spec.n_kv_heads} not divisible by tp={tp}")
    if spec.ffn % (16 * tp) or spec.vocab_size % (16 * tp):
        raise ValueError(f"{spec.name}: ffn/vocab not divisible by 16*tp={16 * tp}")


def pack_layer(spec: ModelSpec, wq, wk, wv, wo, wg, wu, wd, an, mn, rank=0, tp=1, kind="bf16") -> LayerWeights:
    """HF-layout layer tensors -> packed, TP-sharded LayerWeights on wq's device."""
    hd = spec.head_dim
    hq, hk = spec.n_heads // tp, spec.n_kv_heads // tp
    q = wq.view(spec.n_heads, hd, -1)[rank * hq:(rank + 1) * hq].reshape(hq * hd, -1)
    k = wk.view(spec.n_kv_heads, hd, -1)[rank * hk:(rank + 1) * hk].reshape(hk * hd, -1)
    v = wv.view(spec.n_kv_heads, hd, -1)[rank * hk:(rank + 1) * hk].reshape(hk * hd, -1)
    wqkv = torch.cat([q, k, v], 0)
    wo_s = _shard_cols(wo, rank, tp)
    gu = ops.interleave_gate_up(_shard_rows(wg, rank, tp), _shard_rows(wu, rank, tp))
    wd_s = _shard_cols(wd, rank, tp)
    an, mn = an.to(torch.bfloat16), mn.to(torch.bfloat16)
    if FOLD_NORMS:
        wqkv = (wqkv.float() * an.float()[None, :]).to(torch.bfloat16)
        gu = (gu.float() * mn.float()[None, :]).to(torch.bfloat16)
        an, mn = torch.ones_like(an), torch.ones_like(mn)
    P = ops.PackedWeight.from_dense
    return LayerWeights(P(wqkv.contiguous(), kind), P(wo_s.contiguous(), kind), P(gu.contiguous(), kind),
                        P(wd_s.contiguous(), kind), an.contiguous(),
                        mn.contiguous(), norms_folded=FOLD_NORMS)


def init_random(spec: ModelSpec, device="cpu", seed: int = 0, kind: str = "bf16", std: float = 0.02,
                tp_rank: int = 0, tp_size: int = 1) -> LlamaWeights:
    """Seeded random-init weights generated on ``device`` (identical across TP ranks / DP replicas)."""
    check_tp(spec, tp_size)
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    d, hd = spec.hidden, spec.head_dim

    def rnd(*shape, s=std):
        return (torch.randn(*shape, generator=g, device=dev, dtype=torch.float32) * s).to(torch.bfloat16)

    def ones(n):
        return (1.0 + 0.1 * torch.randn(n, generator=g, device=dev)).to(torch.bfloat16)

    embed = rnd(spec.vocab_size, d, s=1.0)
    layers = []
    for _ in range(spec.n_layers):
        wq = rnd(spec.n_heads * hd, d)
        wk = rnd(spec.n_kv_heads * hd, d)
        wv = rnd(spec.n_kv_heads * hd, d)
        wo = rnd(d, spec.n_heads * hd)
        wg = rnd(spec.ffn, d)
        wu = rnd(spec.ffn, d)
        wd = rnd(d, spec.ffn)
        layers.append(pack_layer(spec, wq, wk, wv, wo, wg, wu, wd, ones(d), ones(d), tp_rank, tp_size, kind))
        del wq, wk, wv, wo, wg, wu, wd
    final_norm = ones(d)
    head = embed if spec.tie_embeddings else rnd(spec.vocab_size, d)
    lm_head = ops.PackedWeight.from_dense(_shard_rows(head, tp_rank, tp_size).contiguous(), kind)
    return LlamaWeights(spec, embed, layers, final_norm, lm_head, tp_rank, tp_size)


def from_hf_state_dict(spec: ModelSpec, sd: dict, device="cpu", kind: str = "bf16", tp_rank: int = 0,
                       tp_size: int = 1) -> LlamaWeights:
    """HF LlamaForCausalLM / MistralForCausalLM state dict -> LlamaWeights."""
    check_tp(spec, tp_size)
    dev = torch.device(device)

    def t(name):
        return sd[name].to(device=dev, dtype=torch.bfloat16)

    layers = []
    for i in range(spec.n_layers):
        p = f"model.layers.{i}."
        layers.append(pack_layer(
            spec, t(p + "self_attn.q_proj.weight"), t(p + "self_attn.k_proj.weight"), t(p + "self_attn.v_proj.weight"),
            t(p + "self_attn.o_proj.weight"), t(p + "mlp.gate_proj.weight"), t(p + "mlp.up_proj.weight"),
            t(p + "mlp.down_proj.weight"), t(p + "input_layernorm.weight"), t(p + "post_attention_layernorm.weight"),
            tp_rank, tp_size, kind))
    embed = t("model.embed_tokens.weight").contiguous()
    head = embed if (spec.tie_embeddings or "lm_head.weight" not in sd) else t("lm_head.weight")
    lm_head = ops.PackedWeight.from_dense(_shard_rows(head, tp_rank, tp_size).contiguous(), kind)
    return LlamaWeights(spec, embed, layers, t("model.norm.weight").contiguous(), lm_head, tp_rank, tp_size)


def load_safetensors_dir(path: str, device="cpu", kind="bf16", name: Optional[str] = None,
                         template: Optional[str] = None, tp_rank=0, tp_size=1) -> LlamaWeights:
    """Load an HF checkpoint directory (config.json + *.safetensors) with the safe loader.  The prompt
    template follows the served name when it is a known model (a duckdb-nsql checkpoint served as
    ``duckdb-nsql`` keeps the Ollama duckdb-nsql template), else ``template`` or raw."""
    from safetensors.torch import load_file

    from .spec import get_spec

    with open(os.path.join(path, "config.json")) as f:
        cfg = json.load(f)
    if template is None:
        try:
            template = get_spec(name).template if name else "raw"
        except KeyError:
            template = "raw"
    spec = spec_from_hf_config(cfg, name or os.path.basename(path.rstrip("/")), template)
    sd = {}
    for fn in sorted(glob.glob(os.path.join(path, "*.safetensors"))):
        sd.update(load_file(fn))
    return from_hf_state_dict(spec, sd, device, kind, tp_rank, tp_size)


@torch.no_grad()
def reference_forward(w: LlamaWeights, ids, layer_dtype=torch.float32, act_quant_rows: int = 0,
                      decode_a8=False, decode_a8_mlp: Optional[bool] = None,
                      kv_fp8: bool = False, return_hidden: bool = False):
    """fp32 causal forward of one sequence over the weights exactly as packed (``dense()`` undoes the
    fragment shuffle and the fp8 quantisation, so an fp8 model is compared against its own dequantised
    weights): logits [T, V] f32.  The numerics oracle for the engine at production shapes
    (tests/test_prod_shapes_gpu.py); plain PyTorch, one layer's dense weights alive at a time.

    ``act_quant_rows``: fp8 models run prefill GEMMs W8A8 (ops.linear, M > 64: per-token e4m3 activations);
    the first ``act_quant_rows`` rows (the prompt, when its prefill batch had > 64 tokens) get the same
    per-token activation rounding before the projections.  Decode rows keep bf16 activations (W8A16), or with
    ``decode_a8`` (the W8A8 decode GEMMs of fragment-major buckets, ops.linear_a8) the qkv / gate_up inputs of
    the rows past the prompt are rounded per row to e4m3 from the f32 norm output (as add_rmsnorm's fp8
    output does), o / down inputs stay bf16.  ``decode_a8_mlp`` (default: = decode_a8) sets the gate_up input
    separately (the engine runs gate_up W8A8 from a smaller batch than qkv).  ``decode_a8`` may also be a dict
    {qkv, gate_up, o, down} of the projections the engine runs W8A8 / W4A8 (ModelRunner.a8_plan): the o input is
    then rounded to e4m3 with one E8M0 scale per (row, head) from the f32 attention output, the down input with one
    per (row, 32 columns) from the f32 SiLU product (ops.quantize_blocks_fp8, as the kernels write them); fp8 and
    MXFP4 weights alike; its ``rr`` key (ModelRunner.oracle_plan: the batch-1 residual-reduce step) rounds the qkv /
    gate_up inputs per (row, 32 columns) with E8M0 scales from the raw residual instead, the RMS row scale applied
    after the GEMM (ops.linear_a8_rr).  ``kv_fp8``: the engine's fp8 KV
    cache (ops.KV_FP8) -- every rotated key and value row is rounded per (token, kv-head) to e4m3 with its
    amax / 448 scale (ops.reference.quant_kv_rows) before attention.  ``return_hidden``: (logits, the final
    normalised hidden states [T, d] the lm_head reads)."""
    from ..ops import reference as ref

    spec, dev = w.spec, w.device
    ids = torch.as_tensor(ids, dtype=torch.long, device=dev)
    T, hd = ids.numel(), spec.head_dim
    H, Hkv = spec.n_heads // w.tp_size, spec.n_kv_heads // w.tp_size
    G = H // Hkv
    cos, sin = ref.rope_tables(hd, T, spec.rope_theta, spec.rope_scaling, device=dev)
    cos, sin = cos.unsqueeze(1), sin.unsqueeze(1)

    def norm(x, g):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + spec.rms_eps) * g.float()

    def rope(x):
        lo, hi = x[..., : hd // 2], x[..., hd // 2:]
        return torch.cat([lo * cos - hi * sin, hi * cos + lo * sin], dim=-1)

    def bf(x):  # the kernels hand activations between ops in bf16
        return x.to(torch.bfloat16).float()

    aq = act_quant_rows if w.layers[0].wqkv.kind == "fp8" else 0

    def q8(x):  # W8A8 prefill rows: per-token e4m3 with amax / 448 scales (ops.quantize_rows_fp8)
        if aq <= 0:
            return x
        head = x[:aq]
        amax = head.abs().amax(1, keepdim=True)
        s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
        head = (head / s).to(torch.float8_e4m3fn).float() * s
        return torch.cat([head, x[aq:]], 0)

    fp8w = w.layers[0].wqkv.kind == "fp8"
    if isinstance(decode_a8, dict):
        qw = w.layers[0].wqkv.kind in ("fp8", "mxfp4")
        da8, da8m = bool(decode_a8.get("qkv")) and qw, bool(decode_a8.get("gate_up")) and qw
        da8o, da8d = bool(decode_a8.get("o")) and qw, bool(decode_a8.get("down")) and qw
    else:
        da8 = decode_a8 and fp8w
        da8m = (decode_a8 if decode_a8_mlp is None else decode_a8_mlp) and fp8w
        da8o = da8d = False

    def qblk(x, raw, on, blk):  # o / down inputs of the decode rows: block-scaled e4m3 from the f32 values
        if not on or aq >= T:
            return x
        from ..ops import dequant_blocks_fp8, quantize_blocks_fp8
        return torch.cat([x[:aq], dequant_blocks_fp8(*quantize_blocks_fp8(raw[aq:], blk))], 0)

    def e4m3_rows(x):
        amax = x.abs().amax(1, keepdim=True)
        s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
        return (x / s).to(torch.float8_e4m3fn).float() * s

    rr = isinstance(decode_a8, dict) and bool(decode_a8.get("rr"))

    def qin(xn, on, hraw, g):  # qkv / gate_up input from the f32 norm output
        x = q8(bf(xn))
        if on and aq < T:
            if rr:  # residual-reduce step: e4m3 per 32-block of the raw residual, RMS row scale after the GEMM
                from ..ops import dequant_blocks_fp8, quantize_blocks_fp8
                hr = hraw[aq:]
                rs = torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + spec.rms_eps)
                return torch.cat([x[:aq], dequant_blocks_fp8(*quantize_blocks_fp8(hr, 32)) * rs * g.float()], 0)
            x = torch.cat([x[:aq], e4m3_rows(xn[aq:])], 0)
        return x

    h = w.embed[ids].float()
    mask = torch.full((T, T), float("-inf"), device=dev).triu(1)
    for lw in w.layers:
        x = qin(norm(h, lw.attn_norm), da8, h, lw.attn_norm)
        qkv = x @ lw.wqkv.dense().float().t()
        q = qkv[:, : H * hd].view(T, H, hd)
        k = qkv[:, H * hd:(H + Hkv) * hd].view(T, Hkv, hd)
        v = qkv[:, (H + Hkv) * hd:].view(T, Hkv, hd)
        if kv_fp8:
            q, k, v = bf(rope(q)), ref.dequant_kv_rows(*ref.quant_kv_rows(rope(k))), ref.dequant_kv_rows(*ref.quant_kv_rows(v))
        else:
            q, k, v = bf(rope(q)), bf(rope(k)), bf(v)
        k, v = k.repeat_interleave(G, 1), v.repeat_interleave(G, 1)
        s = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(hd) + mask
        a32 = torch.einsum("hqk,khd->qhd", s.softmax(-1), v).reshape(T, H * hd)
        a = qblk(bf(a32), a32, da8o, 128)
        h = h + q8(a) @ lw.wo.dense().float().t()
        x = qin(norm(h, lw.mlp_norm), da8m, h, lw.mlp_norm)
        gu = (x @ lw.w_gate_up.dense().float().t()).view(T, -1, 2, 16)
        act32 = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(T, -1)
        act = qblk(bf(act32), act32, da8d, 32)
        h = h + q8(act) @ lw.w_down.dense().float().t()
    x = bf(norm(h, w.final_norm))
    logits = x @ w.lm_head.dense().float().t()
    return (logits, x) if return_hidden else logits
