"""Plain-PyTorch fp32 reference of every fused op in ``csrc/kernels`` (the numerics oracle).

Each function here has exactly the signature and in-place semantics of its HIP counterpart in
``ops/__init__.py`` so that (a) the GPU tests compare the kernel against this file op-by-op and (b) the
whole engine can step on CPU for the CPU-only test suite.  Nothing here is used on a GPU tensor in
production: ``ops`` refuses to fall back when the extension is missing on a GPU box.
"""
from __future__ import annotations

import math

import torch

BLOCK = 64  # tokens per KV-cache block (kernels assume 64)


def linear(x: torch.Tensor, w: torch.Tensor, epi: str = "bf16", splitk: int = 1) -> torch.Tensor:
    """x [M,K] @ w[N,K]^T.  epi: bf16 | f32 | silu (w rows interleaved gate/up per 16)."""
    y = x.float() @ w.float().t()
    if epi == "f32":
        return y
    if epi == "silu":
        M, N = y.shape
        y4 = y.view(M, N // 32, 2, 16)
        g, u = y4[:, :, 0, :].reshape(M, N // 2), y4[:, :, 1, :].reshape(M, N // 2)
        return (torch.nn.functional.silu(g) * u).to(torch.bfloat16)
    return y.to(torch.bfloat16)


def add_rmsnorm(h, w, eps, xn, parts=None, ids=None, emb=None, row_idx=None, write_h=True):
    rows = xn.shape[0]
    idx = row_idx.long() if row_idx is not None else torch.arange(rows, device=h.device)
    if ids is not None:
        v = emb[ids.long()[idx]].float()
    else:
        v = h[idx].float()
    if parts is not None:
        v = v + parts[:, idx].float().sum(0)
    if write_h:
        h[idx] = v
    inv = torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + eps)
    xn.copy_((v * inv * w.float()).to(torch.bfloat16))
    return xn


def rope_tables(head_dim: int, max_pos: int, theta: float, scaling: dict | None = None, device="cpu"):
    """cos/sin [max_pos, head_dim/2] f32 with optional llama3 frequency scaling."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling["low_freq_factor"], scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        smooth = (old / wl - lo) / (hi - lo)
        mid = (1 - smooth) * scaled / factor + smooth * scaled
        is_mid = (wl >= hi_wl) & (wl <= lo_wl)
        inv = torch.where(is_mid, mid, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def _slots(pos, tok_seq, block_tables):
    seq = tok_seq.long() if tok_seq is not None else torch.arange(pos.shape[0], device=pos.device)
    p = pos.long()
    blk = block_tables.long()[seq, p // BLOCK]
    return blk, p % BLOCK


# fp8 KV cache rows (csrc/kernels/common.h kv8_inv / LSA_KV8_RMAX): e4m3(x * (448 / amax)) with scale amax * (1/448)
KV8_RMAX = torch.tensor(1.0 / 448.0, dtype=torch.float32)


def quant_kv_rows(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """x f32 [..., 128] -> (e4m3 bytes as uint8 [..., 128], f32 scales [...]) per row of 128 values."""
    x = x.float()
    a = x.abs().amax(-1)
    inv = torch.where(a > 0, torch.tensor(448.0, dtype=torch.float32, device=x.device) / a.clamp_min(1e-38),
                      torch.zeros_like(a))
    q = (x * inv.unsqueeze(-1)).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8)
    return q, a * KV8_RMAX.to(x.device)


def dequant_kv_rows(q: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    return q.view(torch.float8_e4m3fn).float() * sc.float().unsqueeze(-1)


# The fp8 cache tensors keep the [.., 64 tokens, 128] shape but store each (block, kv-head) tile in token-pair order
# (csrc/kernels/common.h kv8_off): the 8-byte chunk c of tokens 2p and 2p + 1 side by side, so one 16-byte lane load
# in decode attention carries two keys.  Scales stay in token order.
def kv8_physical(logical: torch.Tensor) -> torch.Tensor:
    """token-order e4m3 bytes [..., 64, 128] -> the cache's token-pair order (same shape)."""
    sh = logical.shape
    return logical.reshape(*sh[:-2], 32, 2, 16, 8).transpose(-3, -2).reshape(sh)


def kv8_logical(physical: torch.Tensor) -> torch.Tensor:
    """the cache's token-pair order [..., 64, 128] -> token-order e4m3 bytes (same shape)."""
    sh = physical.shape
    return physical.reshape(*sh[:-2], 32, 16, 2, 8).transpose(-3, -2).reshape(sh)


def rope_append(qkv, pos, tok_seq, block_tables, cos_t, sin_t, q_out, kc, vc, H, Hkv, kv_scales=None):
    if qkv.dtype == torch.float32 and qkv.dim() == 3:  # f32 split-K slabs [S, T, n]
        qkv = qkv.sum(0)
    T = qkv.shape[0]
    D = 128
    x = qkv.float().view(T, H + 2 * Hkv, D)
    p = pos.long()
    c = cos_t[p].unsqueeze(1)
    s = sin_t[p].unsqueeze(1)
    qk = x[:, : H + Hkv]
    lo, hi = qk[..., :64], qk[..., 64:]
    rot = torch.cat([lo * c - hi * s, hi * c + lo * s], dim=-1)
    q_out.copy_(rot[:, :H].to(torch.bfloat16).view_as(q_out))
    blk, off = _slots(pos, tok_seq, block_tables)
    if kv_scales is not None:  # fp8 cache: quantise each (token, kv-head) row
        ks, vs = kv_scales
        k8, ksc = quant_kv_rows(rot[:, H:])
        v8, vsc = quant_kv_rows(x[:, H + Hkv:])
        ub = blk.unique()
        idx = torch.searchsorted(ub, blk)
        for cache, rows in ((kc, k8), (vc, v8)):
            tiles = kv8_logical(cache[ub])
            tiles[idx, :, off] = rows
            cache[ub] = kv8_physical(tiles)
        ks[blk, :, off] = ksc
        vs[blk, :, off] = vsc
        return
    kc[blk, :, off] = rot[:, H:].to(kc.dtype)
    vc[blk, :, off] = x[:, H + Hkv:].to(vc.dtype)


def _gather_kv(cache, table_row, n, scales=None):
    nb = (n + BLOCK - 1) // BLOCK
    blocks = cache[table_row[:nb].long()]  # [nb, Hkv, 64, D]
    if scales is not None:
        blocks = dequant_kv_rows(kv8_logical(blocks), scales[table_row[:nb].long()])
    return blocks.permute(1, 0, 2, 3).reshape(cache.shape[1], nb * BLOCK, cache.shape[3])[:, :n]


def attn_decode(q, kc, vc, block_tables, pos, H, Hkv, scale, out, kv_scales=None):
    B = pos.shape[0]
    G = H // Hkv
    ks, vs = kv_scales if kv_scales is not None else (None, None)
    for b in range(B):
        n = int(pos[b]) + 1
        k = _gather_kv(kc, block_tables[b], n, ks).float().repeat_interleave(G, 0)
        v = _gather_kv(vc, block_tables[b], n, vs).float().repeat_interleave(G, 0)
        s = torch.einsum("hd,hnd->hn", q[b].float(), k) * scale
        o = torch.einsum("hn,hnd->hd", s.softmax(-1), v)
        out[b] = o.to(out.dtype).view_as(out[b])
    return out


def attn_prefill(q, kc, vc, block_tables, cu_q, ctx_lens, H, Hkv, scale, out, kv_scales=None):
    G = H // Hkv
    ks, vs = kv_scales if kv_scales is not None else (None, None)
    cu = cu_q.tolist()
    for sq in range(len(cu) - 1):
        q0, q1 = cu[sq], cu[sq + 1]
        ql = q1 - q0
        if ql == 0:
            continue
        n = int(ctx_lens[sq])
        k = _gather_kv(kc, block_tables[sq], n, ks).float().repeat_interleave(G, 0)
        v = _gather_kv(vc, block_tables[sq], n, vs).float().repeat_interleave(G, 0)
        qq = q[q0:q1].float().transpose(0, 1)  # [H, ql, D]
        s = torch.einsum("hqd,hnd->hqn", qq, k) * scale
        qpos = torch.arange(n - ql, n, device=q.device).view(ql, 1)
        kpos = torch.arange(n, device=q.device).view(1, n)
        s = s.masked_fill(kpos > qpos, float("-inf"))
        o = torch.einsum("hqn,hnd->hqd", s.softmax(-1), v)
        out[q0:q1] = o.transpose(0, 1).to(out.dtype).view_as(out[q0:q1])
    return out


def commit(tok, out_tokens, gen_len, input_ids, positions, finished, eos, limit=None, eos_on=None, hist=None):
    eos_set = set(eos.tolist()) if eos is not None else set()
    max_new = out_tokens.shape[1]
    for b in range(tok.shape[0]):
        if int(finished[b]):
            continue
        n = int(gen_len[b])
        t = int(tok[b])
        if n < max_new:
            out_tokens[b, n] = t
        gen_len[b] = n + 1
        input_ids[b] = t
        if hist is not None:  # position-indexed ring of the context's last tokens
            hist[b, (int(positions[b]) + 1) % hist.shape[1]] = t
        lim = min(max_new, int(limit[b])) if limit is not None else max_new
        use_eos = bool(int(eos_on[b])) if eos_on is not None else True
        if n + 1 >= lim or (use_eos and t in eos_set):
            finished[b] = 1
        else:
            positions[b] += 1


def argmax_commit(logits, out_tokens, gen_len, input_ids, positions, finished, eos, limit=None, eos_on=None):
    commit(logits.float().argmax(-1), out_tokens, gen_len, input_ids, positions, finished, eos, limit, eos_on)


def sample_probs(logits_row: torch.Tensor, temperature: float, top_k: int, top_p: float, topk_cap: int = 64):
    """Distribution the sampler draws from (top-k capped at 64, nucleus within it)."""
    k = top_k if 0 < top_k <= topk_cap else topk_cap
    vals, idx = logits_row.float().topk(min(topk_cap, logits_row.numel()))
    vals, idx = vals[:k], idx[:k]
    p = torch.softmax(vals / temperature, -1)
    before = torch.cumsum(p, 0) - p
    keep = before < top_p
    keep[0] = True
    p = torch.where(keep, p, torch.zeros_like(p))
    return idx, p / p.sum()


def repeat_penalty(row, hist_row, pen, pos, last_n):
    """llama.cpp/Ollama repetition penalty on one row of logits over the distinct tokens at context
    positions (pos - last_n, pos] of the position-indexed ring ``hist_row``."""
    W = hist_row.numel()
    n = min(W if last_n is None else int(last_n), W, pos + 1)
    for t in {int(hist_row[(pos - i) % W]) for i in range(n)}:
        if 0 <= t < row.numel():
            row[t] = row[t] / pen if row[t] > 0 else row[t] * pen
    return row


_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def pack_seed(key: int, offset: int = 0) -> int:
    """Device seed word of a request: the stream key (low 40 bits) and the draw-counter offset (high 24 bits, the
    tokens a preempted request already generated), as sampling.hip unpacks it."""
    assert 0 <= offset < (1 << 23), offset
    return (offset << 40) | (int(key) & ((1 << 40) - 1))


def draw_seed(packed: int, gen_len: int) -> int:
    """Generator seed of draw gen_len of a request (the host twin of sampling.hip's keyed counter): the scrambled
    key plus the counter, so nearby keys give unrelated streams and the offset continues a resumed stream."""
    packed &= _M64
    key, off = packed & ((1 << 40) - 1), packed >> 40
    return _mix64((_mix64(key) + 0x9E3779B97F4A7C15 * (off + gen_len + 1)) & _M64) & ((1 << 63) - 1)


def sample_commit(logits, hist, penalty, temperature, top_k, top_p, seeds, out_tokens, gen_len, input_ids,
                  positions, finished, eos, limit=None, eos_on=None, generator: torch.Generator | None = None,
                  last_n=None):
    B = logits.shape[0]
    toks = torch.empty(B, dtype=torch.long)
    for b in range(B):
        row = logits[b].float().clone()
        if hist is not None and penalty is not None and float(penalty[b]) != 1.0:
            row = repeat_penalty(row, hist[b].cpu(), float(penalty[b]), int(positions[b]),
                                 None if last_n is None else int(last_n[b]))
        T = float(temperature[b])
        if T <= 0:
            toks[b] = int(row.argmax())
            continue
        idx, p = sample_probs(row, T, int(top_k[b]), float(top_p[b]))
        # draw g of a row comes from (seed key, g + offset) alone (one generator per row: a generator shared across
        # rows made a row's draws depend on the rows sampled before it in the batch)
        g = generator if generator is not None else torch.Generator().manual_seed(draw_seed(int(seeds[b]), int(gen_len[b])))
        toks[b] = int(idx[torch.multinomial(p.cpu(), 1, generator=g)])
    commit(toks, out_tokens, gen_len, input_ids, positions, finished, eos, limit, eos_on, hist=hist)
