"""Fused operators of the decode engine.

GPU tensors run the hand-written gfx950 kernels of ``csrc/kernels`` through the in-tree extension
``_lsa_hip``; there is no silent fallback — if the extension is missing while a GPU tensor is passed,
the op raises.  CPU tensors run ``ops.reference`` (the fp32 oracle the GPU tests compare against) so
the engine and its scheduler can be exercised on a machine without a GPU.

Weights are held as :class:`PackedWeight`: on the GPU in the MFMA fragment-major layout
(``shuffle_weight``) or fp8-e4m3fn with per-channel scales (``quantize_fp8``); on the CPU as the
plain ``[N, K]`` matrix.
"""
from __future__ import annotations

import dataclasses
import importlib
import importlib.util
import json
import math
import os
from typing import NamedTuple, Optional

import torch

from . import reference as ref

_ext = None
_ext_err: Optional[BaseException] = None

EPI = {"bf16": 0, "f32": 1, "silu": 2, "res": 3}


def ext():
    """The compiled gfx950 extension (raises if it cannot be loaded)."""
    global _ext, _ext_err
    if _ext is None and _ext_err is None:
        try:
            alt = os.environ.get("LSA_HIP_SO")  # experiment knob: an alternative build of the same extension
            if alt:
                spec = importlib.util.spec_from_file_location("_lsa_hip", alt)
                _ext = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(_ext)
            else:
                _ext = importlib.import_module(__name__ + "._lsa_hip")
        except BaseException as e:  # noqa: BLE001 - record and re-raise on use
            _ext_err = e
    if _ext is None:
        raise RuntimeError(
            "gfx950 extension _lsa_hip is not built/loadable; run "
            "`python -m llm_based_apache_spark_optimization_amd.ops.build`"
        ) from _ext_err
    if not BUILD_INFO:
        _check_provenance()
    return _ext


# build provenance of the loaded extension (ops/build.py writes _lsa_hip.provenance.json next to the .so): the
# sources hash it was built from, its own hash, and whether both still match the tree -- a stale .so (kernels
# edited, not rebuilt) fails loudly on load instead of silently running old kernels (LSA_ALLOW_STALE_EXT=1 to
# override, e.g. for A/B builds)
BUILD_INFO: dict = {}


def _check_provenance() -> None:
    import hashlib

    from . import build as _b

    so = getattr(_ext, "__file__", "") or ""
    info = {"so": os.path.basename(so)}
    try:
        rec = json.loads(_b.PROVENANCE.read_text())
    except (OSError, ValueError):
        rec = None
    info["provenance"] = rec
    if rec is not None and so and os.path.abspath(so) == str(_b.HIP_EXT):
        try:
            with open(so, "rb") as f:
                info["so_match"] = hashlib.sha256(f.read()).hexdigest()[:16] == rec.get("so_sha256")
        except OSError:
            info["so_match"] = False
        try:
            info["sources_match"] = _b.sources_sha() == rec.get("sources_sha")
        except OSError:  # sources not shipped with this tree
            info["sources_match"] = None
    BUILD_INFO.update(info)
    if (info.get("so_match") is False or info.get("sources_match") is False) and \
            os.environ.get("LSA_ALLOW_STALE_EXT") != "1":
        raise RuntimeError(f"_lsa_hip.so does not match its sources / provenance record ({info}); rebuild with "
                           "`python -m llm_based_apache_spark_optimization_amd.ops.build`")


def hip_available() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ----------------------------------------------------------------------------------- weights
def shuffle_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> fragment-major [N/16, K/32, 64 lanes, 8]: lane = 16*((k%32)//8) + n%16."""
    N, K = w.shape
    assert N % 16 == 0 and K % 32 == 0, (N, K)
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()


def unshuffle_weight(wf: torch.Tensor, N: int, K: int) -> torch.Tensor:
    return wf.reshape(N // 16, K // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(N, K)


def interleave_gate_up(wg: torch.Tensor, wu: torch.Tensor) -> torch.Tensor:
    """Stack gate and up rows interleaved per 16 so one skinny-GEMM wave owns matching pairs."""
    F, K = wg.shape
    return torch.stack([wg.view(F // 16, 16, K), wu.view(F // 16, 16, K)], dim=1).reshape(2 * F, K)


def pack_fp8(q: torch.Tensor) -> torch.Tensor:
    """e4m3fn bytes [N, K] -> the fragment layout [N/16, K/64, 64 lanes, 16 B], lane = 16 g + r holding
    W[16 nb + r][64 kb + 16 g .. + 15]."""
    N, K = q.shape
    assert N % 16 == 0 and K % 64 == 0, (N, K)
    return q.view(torch.uint8).reshape(N // 16, 16, K // 64, 4, 16).permute(0, 2, 3, 1, 4).contiguous()


def quantize_fp8(w: torch.Tensor):
    """Per-output-channel e4m3fn quantisation -> (packed uint8 [N/16, K/64, 64, 16], scale f32 [N])."""
    N, K = w.shape
    assert N % 16 == 0 and K % 64 == 0, (N, K)
    wf = w.float()
    scale = (wf.abs().amax(dim=1) / 448.0).clamp(min=1e-12)
    q = (wf / scale[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    return pack_fp8(q), scale


def dequantize_fp8(packed: torch.Tensor, scale: torch.Tensor, N: int, K: int) -> torch.Tensor:
    q = packed.reshape(N // 16, K // 64, 4, 16, 16).permute(0, 3, 1, 2, 4).reshape(N, K)
    return q.view(torch.float8_e4m3fn).float() * scale[:, None]


# MXFP4 (OCP MX): e2m1 elements, one E8M0 power-of-two scale per 32 consecutive k (csrc/kernels/gemm_fp4.hip)
FP4_VALUES = (0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0)
_FP4_EDGES = (0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5.0)  # midpoints of the e2m1 magnitude grid


def quantize_mxfp4(w: torch.Tensor):
    """[N, K] -> (e2m1 codes uint8 [N, K] (sign in bit 3), E8M0 scale bytes uint8 [N, K/32]): per 32-element block
    scale 2^(floor(log2 amax) - 2) (e2m1 emax = 2, OCP MX), elements rounded to the e2m1 grid, saturated at 6."""
    N, K = w.shape
    assert K % 32 == 0, K
    wf = w.float().view(N, K // 32, 32)
    amax = wf.abs().amax(-1)
    e = (torch.floor(torch.log2(amax.clamp(min=2.0 ** -125))) - 2).clamp(-126, 127)
    e = torch.where(amax > 0, e, torch.full_like(e, -127))
    v = wf / torch.exp2(e.clamp(min=-126))[..., None]
    mag = torch.bucketize(v.abs().clamp(max=6.0), torch.tensor(_FP4_EDGES, device=w.device))
    codes = (mag | ((v < 0).to(mag.dtype) << 3)).to(torch.uint8).view(N, K)
    return codes, (e + 127).to(torch.uint8)


def pack_mxfp4(codes: torch.Tensor, sbytes: torch.Tensor):
    """codes [N, K], scale bytes [N, K/32] -> the gemm_fp4 layouts: Wq [N/16, K/128, 64 lanes, 16 B] (lane = 16 g + r
    holds W[16 nb + r][128 kb + 32 g .. + 31], element 2i in the low nibble of byte i) and S [N/16, ceil(K/512), 64, 4]
    (the lane's scale byte of four consecutive 128-k steps in one word)."""
    N, K = codes.shape
    assert N % 16 == 0 and K % 128 == 0, (N, K)
    c = codes.view(N, K // 2, 2)
    packed = (c[..., 0] | (c[..., 1] << 4)).contiguous()
    wq = packed.view(N // 16, 16, K // 128, 4, 16).permute(0, 2, 3, 1, 4).reshape(N // 16, K // 128, 64, 16)
    kb = K // 128
    kb4 = (kb + 3) // 4
    sl = sbytes.view(N // 16, 16, kb, 4).permute(0, 2, 3, 1).reshape(N // 16, kb, 64)
    sp = torch.zeros(N // 16, kb4 * 4, 64, dtype=torch.uint8, device=codes.device)
    sp[:, :kb] = sl
    return wq, sp.view(N // 16, kb4, 4, 64).permute(0, 1, 3, 2).contiguous()


def dequantize_mxfp4(wq: torch.Tensor, sw: torch.Tensor, N: int, K: int) -> torch.Tensor:
    """The exact f32 values the gemm_fp4 kernels multiply with (e2m1 value x 2^(e - 127))."""
    kb = K // 128
    packed = wq.reshape(N // 16, kb, 4, 16, 16).permute(0, 3, 1, 2, 4).reshape(N, K // 2)
    codes = torch.stack([packed & 15, packed >> 4], dim=-1).view(N, K).long()
    vals = torch.tensor(FP4_VALUES, device=wq.device)[codes & 7] * (1.0 - 2.0 * (codes >> 3).float())
    sb = sw.reshape(N // 16, -1, 64, 4).permute(0, 1, 3, 2).reshape(N // 16, -1, 64)[:, :kb]
    sb = sb.reshape(N // 16, kb, 4, 16).permute(0, 3, 1, 2).reshape(N, K // 32).float()
    scale = torch.where(sb > 0, torch.exp2(sb - 127.0), torch.zeros_like(sb))
    return (vals.view(N, K // 32, 32) * scale[..., None]).view(N, K)


@dataclasses.dataclass
class PackedWeight:
    """A linear layer's weight in the layout its kernel streams."""

    N: int
    K: int
    kind: str  # "dense" (CPU reference) | "bf16" (fragment layout) | "fp8" | "mxfp4"
    data: torch.Tensor
    scale: Optional[torch.Tensor] = None

    @staticmethod
    def from_dense(w: torch.Tensor, kind: str = "bf16") -> "PackedWeight":
        N, K = w.shape
        if not w.is_cuda:
            return PackedWeight(N, K, "dense", w.to(torch.bfloat16).contiguous())
        if kind == "fp8":
            q, s = quantize_fp8(w)
            return PackedWeight(N, K, "fp8", q, s.contiguous())
        if kind == "mxfp4":
            wq, sw = pack_mxfp4(*quantize_mxfp4(w))
            return PackedWeight(N, K, "mxfp4", wq, sw)
        wb = w.to(torch.bfloat16)
        return PackedWeight(N, K, "bf16", shuffle_weight(wb))

    def dense(self) -> torch.Tensor:
        if self.kind == "dense":
            return self.data
        if self.kind == "bf16":
            return unshuffle_weight(self.data, self.N, self.K)
        if self.kind == "mxfp4":
            return dequantize_mxfp4(self.data, self.scale, self.N, self.K).to(torch.bfloat16)
        return dequantize_fp8(self.data, self.scale, self.N, self.K).to(torch.bfloat16)

    @property
    def nbytes(self) -> int:
        return self.data.numel() * self.data.element_size() + (
            self.scale.numel() * self.scale.element_size() if self.scale is not None else 0)


def pick_nb_splitk(M: int, N: int, K: int, epi: str) -> tuple[int, int]:
    """Skinny-GEMM decomposition (from scripts/bench_gemm.py sweeps on MI355X).

    M <= 16: one 16-row block per wave-group (x traffic is negligible), split-K until >= 1024
    workgroups.  M > 16: 4 blocks (64 rows) per workgroup so each activation fragment feeds 4 MFMAs,
    split-K until >= 256 workgroups.  Only the f32 epilogue (partial slabs summed by the consumer)
    can split K.
    """
    nbt = N // 16
    if M <= 16:
        nb, target = 1, 1024
    else:
        nb, target = (4 if M <= 32 else 2), 256
    if epi == "silu":
        nb = max(nb, 2)
    while nb > 1 and nbt % nb:
        nb //= 2
    splitk = 1
    if epi == "f32" and M <= 64:
        while (nbt // nb) * splitk < target and splitk < 8 and K // (32 * splitk * 2) >= 16:
            splitk *= 2
    return nb, splitk


# ----------------------------------------------------------------------------------- tuning
_TUNING_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_tuning.json")
_tuning: Optional[dict] = None


# experiment overrides of tuning entries (in-pipeline A/Bs: bench.py --set 'ops.TUNING_OVERRIDES={"key": {...}}'),
# consulted before the measured table; empty in production
TUNING_OVERRIDES: dict = {}


def _tuning_table() -> dict:
    """Measured best decode-GEMM configs on MI355X ({"NxK:epi:s|m": {nb, splitk, waves, div}}),
    produced by scripts/bench_gemm.py (median of 3 interleaved runs per config)."""
    global _tuning
    if _tuning is None:
        try:
            with open(_TUNING_PATH) as f:
                _tuning = json.load(f)
        except (OSError, ValueError):
            _tuning = {}
    return {**_tuning, **TUNING_OVERRIDES} if TUNING_OVERRIDES else _tuning


def pick_gemm_config(M: int, N: int, K: int, epi: str, xf: bool = False,
                     kind: str = "bf16") -> tuple[int, int, int, int]:
    """(nb, splitk, waves, div) for a decode GEMM: the tuning table when it has the shape (entries
    measured with fragment-major activations carry a ':xf' suffix, fp8-weight entries ':fp8'), else
    the heuristic below (div 4, 4-wave workgroups won most measured shapes)."""
    if kind == "mxfp4":  # W4A16 decode GEMM (gemm_fp4.hip): its own sweep entries (scripts/bench_fp4_decode.py)
        b = 1
        while b < M:
            b *= 2
        e = _tuning_table().get(f"{N}x{K}:{epi}:b{b}:fp4") or _tuning_table().get(
            f"{N}x{K}:{'f32' if epi == 'res' else epi}:b{b}:fp4")
        if e is not None and M <= 64:
            return e["nb"], e["splitk"], e["waves"], 4
        nbt = N // 16
        nb = 2 if M <= 16 else (8 if M <= 32 else 2)
        while nb > 1 and nbt % nb:
            nb //= 2
        if epi == "silu":
            nb = max(nb, 2)
        sk, target = 1, (512 if M <= 16 else 256)
        if epi in ("f32", "res"):
            while (nbt // nb) * sk < target and sk < 8 and K // (128 * sk * 2) >= 4:
                sk *= 2
        return nb, sk, 4, 4
    if kind in ("fp8a", "fp4a"):  # W8A8 / W4A8 decode GEMM: its own sweep entries, else the 16-bit-activation
        # kernel's (nb, splitk) at default knobs; 'silu8' = the e4m3 SiLU output (whole 32-column blocks: nb % 4 == 0)
        b = 1
        while b < M:
            b *= 2
        e = _tuning_table().get(f"{N}x{K}:{epi}:b{b}:{kind}")
        if e is not None:
            return e["nb"], e["splitk"], e["waves"], e["div"]
        if epi == "silu8":
            nbt = N // 16
            nb = 8 if (M <= 16 and nbt % 8 == 0 and nbt // 8 >= 256) else 4
            assert nbt % nb == 0, f"e4m3 SiLU output needs N / 16 % 4 == 0 (N = {N})"
            return nb, 1, 4, 4
        nb, sk, _, _ = pick_gemm_config(M, N, K, epi, xf=xf, kind="fp8" if kind == "fp8a" else "mxfp4")
        return (2 if (M > 32 and nb > 2) else nb), sk, 4, 4
    if epi == "res":  # the residual epilogue runs the f32-slab main loop (split-K with a last-arriver finish):
        # its own measured entries (scripts/bench_res_epi.py --tune) first, else the f32 entries
        b = 1
        while b < M:
            b *= 2
        e = _tuning_table().get(f"{N}x{K}:res:b{b}" + (":fp8" if kind == "fp8" else ""))
        if e is not None and M <= 64 and not (M > 32 and e["nb"] > 2):
            return e["nb"], e["splitk"], e["waves"], e["div"]
        epi = "f32"
    if M <= 64:
        key = f"{N}x{K}:{epi}:{'s' if M <= 16 else 'm'}"
        tab = _tuning_table()
        e = None
        # per-batch-bucket entries (power-of-two M) where a sweep beat the s/m entry by > 3 %
        # (scripts/bench_gemm_buckets.py, profiles/gemm_buckets_mi355x.jsonl)
        b = 1
        while b < M:
            b *= 2
        e = tab.get(f"{N}x{K}:{epi}:b{b}" + (":fp8" if kind == "fp8" else ":xf" if xf else ""))
        if e is None and kind == "fp8":
            e = tab.get(key + ":fp8")
        fp8_entry = e is not None and kind == "fp8"
        if e is None and xf:
            e = tab.get(key + ":xf")
        e = e if e is not None else tab.get(key)
        if e is not None and not (M > 32 and e["nb"] > 2):
            if kind == "fp8" and not fp8_entry:  # a bf16 entry's nb / split only; fp8 knobs at their defaults
                return e["nb"], e["splitk"], 4, 4
            return e["nb"], e["splitk"], e["waves"], e["div"]
    nb, sk = pick_nb_splitk(M, N, K, epi)
    return nb, sk, 4, 4


# ----------------------------------------------------------------------------------- linear
_dq_scratch: dict = {}


def _fp8_depth(div) -> int:
    """fp8 skinny GEMM chunk depth from a config tuple's 4th field: entries measured for fp8 store the
    depth (1 | 2) there; the bf16 'div' defaults (4) mean the shallow default."""
    return 2 if div == 2 else 1


SS_SCALE = float(1 << 24)


def ss_q24(v: torch.Tensor) -> torch.Tensor:
    """f32 sums of squares -> the kernels' int64 Q24 fixed point (truncating, like the device conversion)."""
    return (v.float() * SS_SCALE).to(torch.int64)


def ss_float(q: torch.Tensor) -> torch.Tensor:
    return q.double().div(SS_SCALE).float()


def _epi_kw(rownorm, res, xmt: int) -> dict:
    """Keyword arguments of the kernels' decode epilogue extensions (csrc/kernels/lsa_epi.h).

    rownorm = (ss, eps): the input rows are the UN-normalised residual stream (RMSNorm gamma folded into
    the weight): output row m is scaled by rsqrt(ss[m] / K + eps).  Row sums of squares (``ss``, ``ss_out``)
    are int64 Q24 fixed point (value * 2^24, ``SS_SCALE``): the kernels add them with integer atomics, so the
    total does not depend on workgroup arrival order and batched decoding stays deterministic.
    res = (h, xout, ss_out[, tickets]) with epi='res': h += y (f32 [M, N]); xout = bf16(h) (fragment-major
    when the call is linear_xf, else row-major [M, N]); ss_out[m] += sum_n h[m, n]^2 (the next GEMM's
    rownorm).  With ``tickets`` (int32, >= N/16 zeroed counters) the GEMM may split K: the splits publish
    f32 partials into ``out`` ([splitk, M, N]) and the last to arrive finishes each column."""
    kw = {}
    if rownorm is not None:
        kw["rowss"], kw["eps"] = rownorm[0], float(rownorm[1])
    if res is not None:
        kw["h"], kw["xout"], kw["ss_out"] = res[:3]
        kw["xmt"] = xmt
        if len(res) > 3 and res[3] is not None:
            kw["tickets"] = res[3]
    return kw


def _res_split(res, splitk: int, out, M: int, N: int, device):
    """(splitk, out) of a residual-epilogue call: split-K needs the ticket counters and a slab buffer."""
    if len(res) < 4 or res[3] is None or splitk <= 1:
        return 1, res[0]
    if out is None:
        out = torch.empty(splitk, M, N, device=device, dtype=torch.float32)
    return splitk, out


def _epi_ref(y: torch.Tensor, M: int, K: int, epi: str, rownorm, res, xf: bool):
    """CPU semantics of the epilogue extensions on a reference result y (f32 [M, N] or bf16 silu output
    computed from row-scaled inputs)."""
    h, xout, ss_out = res[:3]
    hn = h[:M].float() + y.float()
    h[:M].copy_(hn)
    x16 = hn.to(torch.bfloat16)
    if xf:
        f = to_xfrag(x16)
        xout.view(-1)[: f.numel()].copy_(f)
    else:
        xout.view(-1)[: x16.numel()].copy_(x16.reshape(-1))
    ss_out[:M] += ss_q24(hn.pow(2).sum(1))


# ----------------------------------------------------------------------------------- prefill GEMM (M > 64)
# Every prefill projection runs on the stream-K 256^2 MFMA kernel (csrc/kernels/gemm_tile256.hip): a persistent grid
# of one workgroup per CU, whole tiles for the full rounds and K-range shares of the rest, partial tiles summed by the
# last workgroup to arrive.  Its workspace (partial slots + tickets) is per (device, HIP stream): co-served engines
# prefill on their own streams and must not share tickets.
_sk_ws: dict = {}
# fewest K-tiles (64 deep) a workgroup's stream-K share may hold: below it the grid shrinks instead (fewer partial
# tiles, each summed from fewer contributors)
SK_MIN_SHARE = int(os.environ.get("LSA_SK_MIN_SHARE", "8"))
_SK_EPI = {"bf16": 0, "f32": 1, "silu": 2, "res": 3}


def _sk_workspace(device) -> tuple:
    dev = torch.device(device)
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    got = _sk_ws.get(key)
    if got is None:
        ncu = num_cus(dev)
        e = ext()
        ws = torch.empty(e.gemm_sk_ws_bytes(ncu) // 4, device=dev, dtype=torch.float32)
        tk = torch.zeros(e.gemm_sk_tickets(ncu), device=dev, dtype=torch.int32)
        got = _sk_ws[key] = (ws, tk, ncu)
    return got


# stream-K tile configurations (gemm_tile256.hip kSkCfgs, same order; + 8 = whole tiles only):
# (BM, BN, BK, waves per workgroup; 4 = two workgroups per CU)
SK_CFGS = ((256, 256, 64, 8), (256, 192, 64, 8), (256, 128, 64, 8), (128, 256, 64, 8), (128, 192, 64, 8),
           (128, 128, 64, 8), (128, 192, 64, 4), (128, 128, 64, 4))


def sk_cfg_pairs(cfg: int) -> bool:
    """Whether a configuration's waves hold an even n-block count (the SiLU epilogue pairs gate / up n-blocks)."""
    _, bn, _, nw = SK_CFGS[cfg & 7]
    return (bn // 16 // (nw // 2)) % 2 == 0


def sk_cfg_tag(cfg: int) -> str:
    """Name of a stream-K configuration code (bench arms, the tuning table): e.g. 128x192, 128x192w4dp."""
    bm, bn, bk, nw = SK_CFGS[cfg & 7]
    return f"{bm}x{bn}" + ("k128" if bk == 128 else "") + ("w4" if nw == 4 else "") + ("dp" if cfg & 8 else "")


_SK_TUNING_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_sk_tuning.json")
_sk_tuning: Optional[dict] = None
_SK_BUCKETS = (128, 256, 300, 512, 1024, 2048, 4096)


def sk_config(M: int, N: int, K: int, epi: str) -> int:
    """Tile configuration for a prefill GEMM: the measured table (scripts/bench_prefill_gemm.py --grid ->
    scripts/make_sk_tuning.py -> gemm_sk_tuning.json; the nearest measured M in log scale), else -1 (the kernel's
    tile-shape cost model)."""
    global _sk_tuning
    if _sk_tuning is None:
        try:
            with open(_SK_TUNING_PATH) as f:
                _sk_tuning = json.load(f)
        except (OSError, ValueError):
            _sk_tuning = {}
    b = min(_SK_BUCKETS, key=lambda c: abs(math.log2(c) - math.log2(max(M, 1))))
    e = _sk_tuning.get(f"{N}x{K}:{'res' if epi in ('res', 'f32') else epi}:m{b}")
    return int(e["cfg"]) if e is not None else -1


def gemm_sk(x: torch.Tensor, wf: torch.Tensor, N: int, out: torch.Tensor, epi: str,
            min_share: Optional[int] = None, cfg: Optional[int] = None, rows: Optional[int] = None,
            xf_out: bool = False) -> torch.Tensor:
    """out (epi 'bf16' / 'f32' / 'silu') or h (epi 'res': h[:M] += x @ W^T) from the stream-K prefill GEMM over the
    fragment-layout bf16 weight ``wf``.  cfg: None = the measured table (``sk_config``), -1 = the kernel's
    tile-shape cost model, else an SK_CFGS index (+ 8: whole tiles only).  rows: x is a flat buffer in the
    fragment-major layout (``to_xfrag``) of that many rows; xf_out: the SiLU output is written in it."""
    M, K = (rows, wf.numel() // N) if rows is not None else x.shape
    if cfg is None:
        cfg = sk_config(M, N, K, epi)
    ws, tk, ncu = _sk_workspace(x.device)
    ext().gemm_sk(x, wf, N, out, _SK_EPI[epi], ws, tk, ncu, SK_MIN_SHARE if min_share is None else min_share, cfg,
                  (1 if rows is not None else 0) + (2 if xf_out else 0), rows or 0)
    return out


def linear_sk(x: torch.Tensor, w: PackedWeight, epi: str, out: torch.Tensor, rows: Optional[int] = None,
              xf_out: bool = False) -> torch.Tensor:
    """Prefill projection (M > 64) on the stream-K kernel into ``out`` (epi 'bf16' | 'silu'), with fragment-major
    activations: rows = x is a flat ``to_xfrag`` buffer of that many rows; xf_out = the SiLU output is written in
    that layout too (flat, >= xfrag_tiles(rows) * 16 * N / 2), the down projection's input."""
    M = rows if rows is not None else x.shape[0]
    if not _gpu(x):
        y = ref.linear(from_xfrag(x, M, w.K) if rows is not None else x, w.dense(), epi)
        f = to_xfrag(y) if xf_out else y
        out.view(-1)[: f.numel()].copy_(f.reshape(-1))
        return out
    wf = w.data if w.kind == "bf16" else _dequant_scratch(w, x.device)
    return gemm_sk(x, wf, w.N, out, epi, rows=rows, xf_out=xf_out)


def linear_res(x: torch.Tensor, w: PackedWeight, h: torch.Tensor, rows: Optional[int] = None) -> torch.Tensor:
    """h[:M] += x @ W^T in f32 (prefill o / down, M > 64, TP = 1): the residual add rides in the GEMM epilogue, so the
    norm after it reads h alone.  bf16 weights, or quantised ones through their bf16 dequantisation scratch; W8A8
    fp8 prefill keeps its slab path (``res_supported``).  rows: x is fragment-major (``to_xfrag``) with that many."""
    M = rows if rows is not None else x.shape[0]
    if not _gpu(x):
        xr = from_xfrag(x, M, w.K) if rows is not None else x
        h[:M] += ref.linear(xr, w.dense(), "f32")
        return h
    wf = w.data if w.kind == "bf16" else _dequant_scratch(w, x.device)
    return gemm_sk(x, wf, w.N, h, "res", rows=rows)


def linear_rope(x: torch.Tensor, w: PackedWeight, pos, tok_seq, block_tables, cos_t, sin_t, q_out, kc, vc,
                H: int, Hkv: int, rows: Optional[int] = None) -> None:
    """The prefill qkv projection with RoPE and the paged bf16 KV-cache append fused into the GEMM epilogue (M > 64,
    bf16 cache): q_out [T, H, 128] = rotated q, the cache gets rotated k and v at each token's slot.  CPU: the
    unfused reference (bf16 qkv, then ``rope_append``).  rows: x is fragment-major (``to_xfrag``) with that many."""
    M = rows if rows is not None else x.shape[0]
    if not _gpu(x):
        qkv = linear(from_xfrag(x, M, w.K) if rows is not None else x, w, "bf16")
        return ref.rope_append(qkv, pos, tok_seq, block_tables, cos_t, sin_t, q_out, kc, vc, H, Hkv)
    wf = w.data if w.kind == "bf16" else _dequant_scratch(w, x.device)
    ws, tk, ncu = _sk_workspace(x.device)
    ext().gemm_sk_rope(x, wf, ws, tk, ncu, SK_MIN_SHARE, rope_config(M, w.N, w.K), pos, tok_seq,
                       block_tables, cos_t, sin_t, q_out, kc, vc, H, Hkv, 1 if rows is not None else 0, rows or 0)


def rope_config(M: int, N: int, K: int) -> int:
    """Tile configuration of the RoPE-epilogue qkv GEMM: the table's measured "rope" entry (scripts/rope_cfg_sweep.py,
    profiles/r5/rope_cfg_sweep_mi355x.jsonl: the bf16 entry's 192-column tile widened to 256 columns ran the 3B qkv at
    4096 rows in 185 us vs 147.5 us on 128 x 256), else the bf16 entry."""
    sk_config(M, N, K, "bf16")  # loads the table
    b = min(_SK_BUCKETS, key=lambda c: abs(math.log2(c) - math.log2(max(M, 1))))
    e = (_sk_tuning or {}).get(f"{N}x{K}:rope:m{b}")
    return int(e["cfg"]) if e is not None else sk_config(M, N, K, "bf16")


def rope_fusable(w: PackedWeight, kv_fp8: bool, M: int = 1 << 30) -> bool:
    """Whether the prefill qkv projection of M rows takes the fused RoPE / cache-append epilogue (``linear_rope``):
    bf16 cache, weights the stream-K kernel reads (bf16, or quantised ones through their bf16 dequantisation; the
    W8A8 fp8 prefill keeps its split-K path), and at least ROPE_FUSED_MIN_M rows."""
    return not kv_fp8 and res_supported(w) and ROPE_FUSED and M >= ROPE_FUSED_MIN_M


# The fused epilogue needs a whole-head (256-column) tile.  In the engine (rocprofv3 / scripts/ttft_ab.py,
# profiles/r5/ttft_ab_mi355x.jsonl, profiles/r5/rocprof_b32_gaps.txt) it wins where the qkv round trip it removes is
# large -- the 7B b32 bench prefill, 4096 rows: 361 us fused vs 320 + 65 (rope_append) -- and loses below, where the
# 192-column tile plus the separate launch is faster (3B 2k TTFT 14.41 vs 14.30 ms, 7B 300-token 11.29 vs 10.96 ms)
ROPE_FUSED = os.environ.get("LSA_ROPE_FUSED", "1") != "0"
ROPE_FUSED_MIN_M = int(os.environ.get("LSA_ROPE_FUSED_MIN_M", "4096"))


def res_supported(w: PackedWeight) -> bool:
    """Whether ``linear_res`` takes this weight (everything but W8A8 fp8 prefill, whose fp8 tile kernel writes
    split-K slabs)."""
    return RES_FUSED and not (w.kind == "fp8" and FP8_W8A8 and w.K % 128 == 0)


# prefill o / down: residual add in the GEMM epilogue (1) or an f32 GEMM output summed by the next add_rmsnorm (0)
RES_FUSED = os.environ.get("LSA_RES_FUSED", "1") != "0"
# TP = 1 prefill with every stream-K GEMM input in the fragment-major layout (engine.runner._prefill_layers): the
# producers (add_rmsnorm, the prefill attention, the gate_up SiLU epilogue) write it, the GEMM stages each MFMA
# fragment as one contiguous KiB instead of 16 half-lines
PREFILL_XF = os.environ.get("LSA_PREFILL_XF", "1") != "0"


def linear(x: torch.Tensor, w: PackedWeight, epi: str = "bf16", out: Optional[torch.Tensor] = None,
           splitk: Optional[int] = None, nb: Optional[int] = None, waves: Optional[int] = None,
           div: Optional[int] = None, rownorm=None, res=None, _xf: bool = False) -> torch.Tensor:
    """y = x @ W^T with a fused epilogue.  epi='f32' returns [splitk, M, N] partial slabs.
    rownorm / res (epi='res'): the decode epilogue extensions, see ``_epi_kw``."""
    M, K = x.shape
    assert K == w.K, (K, w.K)
    assert (epi == "res") == (res is not None), "epi='res' needs res=(h, xout, ss_out)"
    if not _gpu(x):
        if rownorm is not None:  # scale the rows before the product (the kernels scale the output rows)
            x = (x.float() * torch.rsqrt(ss_float(rownorm[0][:M]) / K + rownorm[1])[:, None]).to(x.dtype)
        if epi == "res":
            _epi_ref(ref.linear(x, w.dense(), "f32"), M, K, epi, rownorm, res, _xf)
            return res[0]
        y = ref.linear(x, w.dense(), epi)
        if epi == "f32":
            y = y.unsqueeze(0)
        if out is not None:
            out.view(-1)[: y.numel()].copy_(y.reshape(-1))
            return out
        return y
    if M > 64 and epi in ("bf16", "f32", "silu") and not (w.kind == "fp8" and FP8_W8A8 and K % 128 == 0):
        # prefill: the stream-K tile kernel (epi 'f32' returns one [1, M, N] slab whatever splitk asked for)
        assert rownorm is None and res is None, "epilogue extensions are decode-only (M <= 64)"
        if out is None:
            out = torch.empty(*((1, M, w.N) if epi == "f32" else (M, w.N // 2 if epi == "silu" else w.N)),
                              device=x.device, dtype=torch.float32 if epi == "f32" else torch.bfloat16)
        wf = w.data if w.kind == "bf16" else _dequant_scratch(w, x.device)
        return gemm_sk(x, wf, w.N, out, epi)
    nb0, sk0, wv0, dv0 = pick_gemm_config(M, w.N, K, epi, kind=w.kind)
    nb = nb0 if nb is None else nb
    if M > 64:  # prefill tile kernels: split-K (f32 slabs) only where the tile grid is small
        assert rownorm is None and res is None, "epilogue extensions are decode-only (M <= 64)"
        splitk = (tile_splitk(M, w.N, K, w.kind) if splitk is None else splitk) if epi == "f32" else 1
    splitk = sk0 if splitk is None else splitk
    waves = wv0 if waves is None else waves
    div = dv0 if div is None else div
    if epi == "res":
        splitk, out = _res_split(res, splitk, out, M, w.N, x.device)
    if out is None:
        if epi == "f32":
            out = torch.empty(splitk, M, w.N, device=x.device, dtype=torch.float32)
        else:
            out = torch.empty(M, w.N // 2 if epi == "silu" else w.N, device=x.device, dtype=torch.bfloat16)
    e = ext()
    kw = _epi_kw(rownorm, res, 0)
    if w.kind == "bf16":
        e.gemm(x, w.data, w.N, out, EPI[epi], nb, splitk, waves, div, **kw)
    elif w.kind == "fp8":
        if M <= 64:  # fp8 knobs: waves, and the tuning entry's "div" field is the chunk depth (1 | 2)
            e.fp8_gemm(x, w.data, w.scale, w.N, out, EPI[epi], nb, splitk, waves, _fp8_depth(div), **kw)
        else:  # W8A8 on the block-scaled fp8 MFMA: per-token activation scales, no weight dequantisation
            x8, sx = quantize_rows_fp8(x)
            e.fp8_gemm_t256(x8, sx, w.data, w.scale, w.N, out, EPI[epi], splitk)
    elif w.kind == "mxfp4":  # W4A16 decode GEMM, e2m1 -> bf16 in registers (v_cvt_scalef32_pk_bf16_fp4)
        e.fp4_gemm(x, w.data, w.scale, w.N, out, EPI[epi], nb, splitk, waves, **kw)
    else:
        raise ValueError(f"weight kind {w.kind} on GPU")
    return out


FP8_W8A8 = os.environ.get("LSA_FP8_W8A8", "1") != "0"


def _dequant_scratch(w: PackedWeight, device) -> torch.Tensor:
    """One layer's weight dequantised to the bf16 fragment layout in a scratch (prefill of quantised models: one
    pass over 0.5-1 byte per weight, then the bf16 tile GEMM).  One scratch per (device, HIP stream): co-served
    engines prefill on their own streams (client.py), and a scratch shared across streams would let one stream's
    dequant overwrite the weights another stream's GEMM is still reading.  A regrown scratch is freed on the same
    stream that used it, so the caching allocator orders its reuse behind that stream's pending kernels."""
    key = (torch.device(device), torch.cuda.current_stream(device).cuda_stream)
    buf = _dq_scratch.get(key)
    if buf is None or buf.numel() < w.N * w.K:
        buf = torch.empty(w.N * w.K, device=device, dtype=torch.bfloat16)
        _dq_scratch[key] = buf
    if w.kind == "mxfp4":
        ext().fp4_dequant(w.data, w.scale, w.N, w.K, buf)
    else:
        ext().fp8_dequant(w.data, w.scale, w.N, w.K, buf)
    return buf[: w.N * w.K]


def quantize_rows_fp8(x: torch.Tensor):
    """Per-token fp8: (x8 [M, K] uint8 e4m3fn bits, sx [M] f32) with x ~= e4m3(x / sx) * sx, sx = amax / 448."""
    M, K = x.shape
    if not _gpu(x):
        xf = x.float()
        sx = (xf.abs().amax(1) / 448.0).clamp(min=1e-30)
        sx = torch.where(xf.abs().amax(1) > 0, sx, torch.ones_like(sx))
        q = (xf / sx[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
        return q.view(torch.uint8), sx
    x8 = torch.empty(M, K, device=x.device, dtype=torch.uint8)
    sx = torch.empty(M, device=x.device, dtype=torch.float32)
    ext().quant_rows_fp8(x, x8, sx)
    return x8, sx


def fp8_tile_splitk(M: int, N: int, K: int) -> int:
    """Split-K of a W8A8 prefill GEMM (f32 slab epilogue) on the 256^2 fp8 tile kernel: doubled until the
    grid has >= 256 workgroups, at most 8 slabs and >= 4 K-tiles (512 of K) per slab."""
    tiles = ((M + 255) // 256) * ((N // 16 + 15) // 16)
    if tiles >= 128:
        return 1
    sk = 1
    while tiles * sk < 256 and sk < 8 and (K // 128) // (sk * 2) >= 4:
        sk *= 2
    return sk


def tile_splitk(M: int, N: int, K: int, kind: str = "bf16") -> int:
    """Split-K (f32 slabs) of a prefill GEMM (M > 64): only the W8A8 fp8 tile kernel splits K (``fp8_tile_splitk``);
    every other prefill projection runs on the stream-K kernel, which balances the K ranges itself."""
    if kind == "fp8" and FP8_W8A8 and K % 128 == 0:
        return fp8_tile_splitk(M, N, K)
    return 1


_NUM_CUS: dict = {}


def num_cus(device) -> int:
    idx = torch.device(device).index or 0
    if idx not in _NUM_CUS:
        _NUM_CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _NUM_CUS[idx]


def xfrag_tiles(M: int) -> int:
    """Row tiles (16 rows each) of the fragment-major activation layout for M rows: decode (M <= 64) rounds up to
    1 | 2 | 4 tiles (the skinny kernels' MT), prefill (M > 64) to ceil(M / 16) (the stream-K GEMM's xf operands)."""
    return 1 if M <= 16 else (2 if M <= 32 else (4 if M <= 64 else (M + 15) // 16))


def to_xfrag(x: torch.Tensor) -> torch.Tensor:
    """[M, K] -> fragment-major activations Xf[K/32][MT][64 lanes][8] (lane = 16*((k%32)/8) + m%16,
    rows >= M zero): one MFMA B-fragment per (k-step, row tile) is 1 KiB lane-linear."""
    M, K = x.shape
    mt = xfrag_tiles(M)
    xp = torch.zeros(mt * 16, K, dtype=x.dtype, device=x.device)
    xp[:M] = x
    return xp.view(mt, 16, K // 32, 4, 8).permute(2, 0, 3, 1, 4).contiguous().view(-1)


def from_xfrag(xf: torch.Tensor, M: int, K: int) -> torch.Tensor:
    mt = xfrag_tiles(M)
    return xf[: mt * 16 * K].view(K // 32, mt, 4, 16, 8).permute(1, 3, 0, 2, 4).reshape(mt * 16, K)[:M]


def linear_xf(xf: torch.Tensor, M: int, w: PackedWeight, epi: str = "bf16", out: Optional[torch.Tensor] = None,
              splitk: Optional[int] = None, nb: Optional[int] = None, waves: Optional[int] = None,
              div: Optional[int] = None, rownorm=None, res=None) -> torch.Tensor:
    """``linear`` with the activations in the fragment-major layout (``to_xfrag``), M <= 64, bf16 or fp8 weights.
    epi='silu' writes its [M, N/2] output in the fragment-major layout too (the next GEMM's input);
    for that epilogue ``out`` is a flat buffer of at least xfrag_tiles(M) * 16 * N/2 elements.
    epi='res' writes its bf16 copy of the residual in the fragment-major layout."""
    if not _gpu(xf) or w.kind not in ("bf16", "fp8", "mxfp4"):
        if epi != "silu":
            return linear(from_xfrag(xf, M, w.K), w, epi, out, splitk, nb, waves, div, rownorm, res, _xf=True)
        y = to_xfrag(linear(from_xfrag(xf, M, w.K), w, epi, None, splitk, nb, waves, div, rownorm))
        if out is None:
            return y
        out.view(-1)[: y.numel()].copy_(y)
        return out
    nb0, sk0, wv0, dv0 = pick_gemm_config(M, w.N, w.K, epi, xf=True, kind=w.kind)
    nb = nb0 if nb is None else nb
    splitk = sk0 if splitk is None else splitk
    waves = wv0 if waves is None else waves
    div = dv0 if div is None else div
    if epi == "res":
        splitk, out = _res_split(res, splitk, out, M, w.N, xf.device)
    if out is None:
        if epi == "f32":
            out = torch.empty(splitk, M, w.N, device=xf.device, dtype=torch.float32)
        elif epi == "silu":
            out = torch.zeros(xfrag_tiles(M) * 16 * (w.N // 2), device=xf.device, dtype=torch.bfloat16)
        else:
            out = torch.empty(M, w.N, device=xf.device, dtype=torch.bfloat16)
    kw = _epi_kw(rownorm, res, xfrag_tiles(M))
    if w.kind == "fp8":
        ext().fp8_gemm_xf(xf, M, w.K, w.data, w.scale, w.N, out, EPI[epi], nb, splitk, waves, _fp8_depth(div), **kw)
    elif w.kind == "mxfp4":
        ext().fp4_gemm_xf(xf, M, w.K, w.data, w.scale, w.N, out, EPI[epi], nb, splitk, waves, **kw)
    else:
        ext().gemm_xf(xf, M, w.K, w.data, w.N, out, EPI[epi], nb, splitk, waves, div, **kw)
    return out


# ----------------------------------------------------------------------------------- W8A8 decode
# LSA_FP8_A8=0 keeps the W8A16 decode GEMMs for the qkv / gate_up projections of fp8 models
FP8_A8_DECODE = os.environ.get("LSA_FP8_A8", "1") != "0"


def to_xf8(x8: torch.Tensor, mt: int) -> torch.Tensor:
    """uint8 [M, K] e4m3 bytes -> the flat xf8 layout X8[K/128][mt][64 lanes][32 B] of the W8A8 / W4A8 decode GEMM
    (csrc/kernels/gemm_fp8a.hip, common.h xf8_off; lane 16 g + r: row 16 t + r at k = 128 s + 16 g .. +15 and
    128 s + 64 + 16 g .. +15 -- the MFMA's own K order for an 8-bit operand), rows >= M zero."""
    M, K = x8.shape
    full = torch.zeros(16 * mt, K, dtype=torch.uint8, device=x8.device)
    full[:M] = x8
    v = full.view(mt, 16, K // 128, 2, 4, 16)  # t, r, s, h, g, e
    return v.permute(2, 0, 4, 1, 3, 5).contiguous().view(-1)  # s, t, g, r, h, e


def from_xf8(x8f: torch.Tensor, M: int, K: int) -> torch.Tensor:
    mt = xfrag_tiles(M)
    v = x8f.view(-1)[: mt * 16 * K].view(K // 128, mt, 4, 16, 2, 16)  # s, t, g, r, h, e
    return v.permute(1, 3, 0, 4, 2, 5).reshape(16 * mt, K)[:M]


def to_xs8(s: torch.Tensor, mt: int) -> torch.Tensor:
    """E8M0 bytes [M, K/32] (one per row and 32-column block) -> the block-scale layout S8[K/128][mt][64 lanes]
    (common.h xs8_off), rows >= M = 127 (2^0)."""
    M, nb32 = s.shape
    full = torch.full((16 * mt, nb32), 127, dtype=torch.uint8, device=s.device)
    full[:M] = s
    return full.view(mt, 16, nb32 // 4, 4).permute(2, 0, 3, 1).contiguous().view(-1)  # s, t, g, r


def from_xs8(s8: torch.Tensor, M: int, K: int) -> torch.Tensor:
    mt = xfrag_tiles(M)
    v = s8.view(-1)[: mt * 64 * (K // 128)].view(K // 128, mt, 4, 16)  # s, t, g, r
    return v.permute(1, 3, 0, 2).reshape(16 * mt, K // 32)[:M]


def e8m0_for_amax(amax: torch.Tensor) -> torch.Tensor:
    """E8M0 exponent (int32) of the smallest power of two s with amax / s <= 448, clamped to [1, 253] -- the host
    twin of common.h e8m0_for_amax (same f32 bit arithmetic)."""
    b = (amax.float() * (1.0 / 448.0)).contiguous().view(torch.int32)
    e = (b >> 23) + ((b & 0x7FFFFF) != 0).to(torch.int32)
    return e.clamp(1, 253)


def quantize_blocks_fp8(x: torch.Tensor, blk: int = 32):
    """[M, K] -> (e4m3 bytes [M, K] uint8, E8M0 bytes [M, K/32] uint8): one power-of-two scale per row and block of
    ``blk`` (32 | 128) consecutive columns (a 128-block's byte repeated for its four 32-blocks) -- what the decode
    attention (blk 128: per head) and the W8A8 SiLU epilogue (blk 32) write for the next W8A8 / W4A8 GEMM."""
    M, K = x.shape
    xf = x.float().view(M, K // blk, blk)
    e = e8m0_for_amax(xf.abs().amax(-1))
    inv = torch.exp2(127.0 - e.float())
    q = (xf * inv[..., None]).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8).view(M, K)
    return q, e.to(torch.uint8).repeat_interleave(blk // 32, dim=1)


def dequant_blocks_fp8(x8: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """(e4m3 bytes [M, K], E8M0 [M, K/32]) -> f32 [M, K]."""
    M, K = x8.shape
    v = x8.view(torch.float8_e4m3fn).float().view(M, K // 32, 32)
    return (v * torch.exp2(s.float() - 127.0)[..., None]).view(M, K)


def quantize_xf8(x: torch.Tensor, mt: Optional[int] = None, out: Optional[torch.Tensor] = None,
                 sx: Optional[torch.Tensor] = None):
    """(x8 flat xf8 bytes, sx [M] f32): per-row e4m3 activations (scale amax / 448) for ``linear_a8``."""
    M, K = x.shape
    mt = mt or xfrag_tiles(M)
    if out is None:
        out = torch.zeros(mt * 16 * K, dtype=torch.uint8, device=x.device)
    if sx is None:
        sx = torch.empty(M, dtype=torch.float32, device=x.device)
    if not _gpu(x):
        q, s = quantize_rows_fp8(x)
        out.view(-1)[: mt * 16 * K].copy_(to_xf8(q, mt))
        sx[:M].copy_(s)
        return out, sx
    ext().quant_xf8(x, mt, out, sx)
    return out, sx


def quantize_xf8_blocks(x: torch.Tensor, blk: int = 32, mt: Optional[int] = None, out: Optional[torch.Tensor] = None,
                        s8: Optional[torch.Tensor] = None):
    """(x8 flat xf8 bytes, s8 flat block scales): block-scaled e4m3 activations (``quantize_blocks_fp8``) in the
    layouts ``linear_a8(..., s8=)`` reads."""
    M, K = x.shape
    mt = mt or xfrag_tiles(M)
    if out is None:
        out = torch.zeros(mt * 16 * K, dtype=torch.uint8, device=x.device)
    if s8 is None:
        s8 = torch.full((mt * 64 * (K // 128),), 127, dtype=torch.uint8, device=x.device)
    if not _gpu(x):
        q, s = quantize_blocks_fp8(x, blk)
        out.view(-1)[: mt * 16 * K].copy_(to_xf8(q, mt))
        s8.view(-1)[: mt * 64 * (K // 128)].copy_(to_xs8(s, mt))
        return out, s8
    ext().quant_xf8_blocks(x.contiguous(), mt, blk, out, s8)
    return out, s8


def xf8_dequant(x8: torch.Tensor, M: int, K: int, sx: Optional[torch.Tensor] = None,
                s8: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The f32 [M, K] activations a W8A8 / W4A8 GEMM multiplies: xf8 bytes x per-row sx x per-block E8M0."""
    v = from_xf8(x8, M, K).view(torch.float8_e4m3fn).float()
    if s8 is not None:
        v = (v.view(M, K // 32, 32) * torch.exp2(from_xs8(s8, M, K).float() - 127.0)[..., None]).view(M, K)
    if sx is not None:
        v = v * sx[:M, None].float()
    return v


def linear_a8(x8: torch.Tensor, sx: Optional[torch.Tensor], M: int, w: PackedWeight, epi: str = "f32",
              out: Optional[torch.Tensor] = None, splitk: Optional[int] = None, nb: Optional[int] = None,
              waves: Optional[int] = None, div: Optional[int] = None, rownorm=None, xfo: bool = True,
              s8: Optional[torch.Tensor] = None, out_s8: Optional[torch.Tensor] = None) -> torch.Tensor:
    """W8A8 / W4A8 decode GEMM (M <= 64; fp8 or MXFP4 weights): out = (x8 . scales) @ w^T with the activations in
    the xf8 layout on the block-scaled fp8 MFMA.  Activation scales: per-row f32 ``sx`` (``quantize_xf8`` / the
    fp8 output of ``add_rmsnorm``) and / or per-block E8M0 ``s8`` (``quantize_xf8_blocks`` / the e4m3 outputs of
    ``attn_decode(out_s8=)`` and of this GEMM's SiLU epilogue).  epi 'f32' -> [splitk, M, N] slabs; 'silu' -> bf16
    [M, N/2] in the fragment-major layout (``xfo``) or row-major, or -- ``out_s8`` given -- e4m3 xf8 bytes in
    ``out`` with one E8M0 scale per (row, 32 columns) in ``out_s8`` (nb a multiple of 4)."""
    assert epi in ("f32", "silu")
    assert sx is not None or s8 is not None
    f8o = epi == "silu" and out_s8 is not None
    if not _gpu(x8):
        xd = xf8_dequant(x8, M, w.K, sx, s8)
        if rownorm is not None:
            xd = xd * torch.rsqrt(ss_float(rownorm[0][:M]) / w.K + rownorm[1])[:, None]
        y = xd @ w.dense().float().t()
        if epi == "f32":
            sk = splitk or 1
            o = out if out is not None else torch.empty(sk, M, w.N)
            o.view(-1)[: sk * M * w.N].zero_()
            o.view(sk, M, w.N)[0].copy_(y)
            return o
        F = w.N // 2
        y3 = y.view(M, F // 16, 2, 16)
        act = (torch.nn.functional.silu(y3[:, :, 0]) * y3[:, :, 1]).reshape(M, F)
        if f8o:
            q, s = quantize_blocks_fp8(act, 32)
            mt = xfrag_tiles(M)
            out.view(-1)[: mt * 16 * F].copy_(to_xf8(q, mt))
            out_s8.view(-1)[: mt * 64 * (F // 128)].copy_(to_xs8(s, mt))
            return out
        act = act.to(torch.bfloat16)
        act = to_xfrag(act) if xfo else act
        if out is None:
            return act
        out.view(-1)[: act.numel()].copy_(act.view(-1))
        return out
    assert w.kind in ("fp8", "mxfp4"), "linear_a8 runs fp8 / MXFP4 weights"
    kind = "fp8a" if w.kind == "fp8" else "fp4a"
    nb0, sk0, wv0, dv0 = pick_gemm_config(M, w.N, w.K, "silu8" if f8o else epi, xf=True, kind=kind)
    nb = nb0 if nb is None else nb
    splitk = sk0 if splitk is None else splitk
    waves = wv0 if waves is None else waves
    div = dv0 if div is None else div
    if out is None:
        if epi == "f32":
            out = torch.empty(splitk, M, w.N, device=x8.device, dtype=torch.float32)
        else:
            out = torch.zeros((xfrag_tiles(M) * 16 if xfo else M) * (w.N // 2), device=x8.device, dtype=torch.bfloat16)
    kw = _epi_kw(rownorm, None, 0)
    fp4 = w.kind == "mxfp4"
    ext().a8_gemm(x8, s8, sx, M, w.K, w.data, None if fp4 else w.scale, w.scale if fp4 else None, w.N, out, out_s8,
                  EPI[epi], nb, splitk, waves, _fp8_depth(div), 2 if f8o else (1 if xfo else 0), **kw)
    return out


def rr_config(N: int, K: int, epi: str, kind: str = "bf16") -> tuple[int, int, int, int]:
    """(nb, splitk, waves, div) of a batch-1 residual-reduce GEMM (``linear_rr`` / ``linear_a8_rr``): the measured
    "NxK:epi:b1:rr[:kind]" entry of the tuning table (scripts/sweep_rr_b1.py -- the prologue re-reads the residual
    slice once per workgroup, so the best n-block width differs from the plain kernel's), else the plain kernel's
    pick.  kind: 'bf16' or the weight kind ('fp8' / 'mxfp4': the W8A8 / W4A8 kernel)."""
    a8 = kind in ("fp8", "mxfp4")
    e = _tuning_table().get(f"{N}x{K}:{epi}:b1:rr" + (f":{kind}" if a8 else ""))
    if e is not None:
        return e["nb"], (1 if epi == "silu" else e["splitk"]), e["waves"], e["div"]
    if a8:
        ak = "fp8a" if kind == "fp8" else "fp4a"
        nb, sk, wv, dv = pick_gemm_config(1, N, K, "silu8" if epi == "silu" else epi, xf=True, kind=ak)
    else:
        nb, sk, wv, dv = pick_gemm_config(1, N, K, epi, kind=kind)
    return nb, (1 if epi == "silu" else sk), wv, dv


def linear_a8_rr(h: torch.Tensor, parts: torch.Tensor, h_out: torch.Tensor, w: PackedWeight, epi: str,
                 out: Optional[torch.Tensor] = None, out_s8: Optional[torch.Tensor] = None,
                 ss_out: Optional[torch.Tensor] = None, eps: float = 1e-5, splitk: Optional[int] = None,
                 nb: Optional[int] = None, waves: Optional[int] = None, div: Optional[int] = None) -> torch.Tensor:
    """Batch-1 W8A8 / W4A8 decode projection (fp8 or MXFP4 weights) with the residual add AND the activation
    quantisation in its prologue (gemm_fp8a.hip RR): x = h + sum_s parts[s] (h_out <- x), quantised to e4m3 with one
    E8M0 scale per 32 k -- no quantising norm launch before it.  The RMSNorm gamma is folded into W; the row scale
    r = rsqrt(mean(x^2) + eps) is applied
      * epi='silu' (gate_up): in the epilogue from the workgroup's own full-row sum; the output is the down
        projection's e4m3 input in the xf8 layout (``out``) with one E8M0 per 32 columns (``out_s8``);
      * epi='f32' (qkv): not here -- [splitk, 1, N] f32 slabs of W @ q(x), and sum x^2 goes to ss_out[0] (Q24) for
        the slab consumer (``attn_decode(rownorm=...)``)."""
    K = w.K
    assert epi in ("f32", "silu") and parts.dim() == 3 and parts.shape[1] == 1
    nb0, sk0, wv0, dv0 = rr_config(w.N, K, epi, w.kind)
    splitk = 1 if epi == "silu" else (sk0 if splitk is None else splitk)
    nb, waves, div = nb0 if nb is None else nb, wv0 if waves is None else waves, dv0 if div is None else div
    if not _gpu(h):
        x = h.view(-1)[:K].float() + parts.float().sum(0).view(-1)
        h_out.view(-1)[:K].copy_(x)
        q, s = quantize_blocks_fp8(x.view(1, K), 32)
        y = dequant_blocks_fp8(q, s) @ w.dense().float().t()
        if epi == "f32":
            ss_out.view(-1)[:1] += ss_q24(x.pow(2).sum().view(1))
            o = out if out is not None else torch.empty(splitk, 1, w.N)
            o.view(-1)[: splitk * w.N].zero_()
            o.view(splitk, 1, w.N)[0].copy_(y)
            return o
        y = y * torch.rsqrt(x.pow(2).sum() / K + eps)
        F = w.N // 2
        y3 = y.view(1, F // 16, 2, 16)
        act = (torch.nn.functional.silu(y3[:, :, 0]) * y3[:, :, 1]).reshape(1, F)
        qa, sa = quantize_blocks_fp8(act, 32)
        out.view(-1)[: 16 * F].copy_(to_xf8(qa, 1))
        out_s8.view(-1)[: 64 * (F // 128)].copy_(to_xs8(sa, 1))
        return out
    assert w.kind in ("fp8", "mxfp4"), "linear_a8_rr runs fp8 / MXFP4 weights"
    if out is None:
        assert epi == "f32"
        out = torch.empty(splitk, 1, w.N, device=h.device, dtype=torch.float32)
    fp4 = w.kind == "mxfp4"
    ext().a8_gemm_rr(h.view(-1)[:K], parts, h_out.view(-1), w.data, None if fp4 else w.scale, w.scale if fp4 else None,
                     w.N, out, out_s8, EPI[epi], nb, splitk, waves, _fp8_depth(div), ss_out=ss_out, eps=float(eps))
    return out


def rr_a8_supported(w: PackedWeight, K: int, splitk: int = 1) -> bool:
    """Whether a batch-1 W8A8 / W4A8 GEMM can take the residual-reduce prologue (``linear_a8_rr``): K slices that
    fit the kernel's LDS image (gemm_fp8a.hip A8_RR_KMAX)."""
    return w.kind in ("fp8", "mxfp4") and K % 128 == 0 and (K // 128 + splitk - 1) // splitk * 128 <= 8192


# ----------------------------------------------------------------------------------- norms / rope
def add_rmsnorm(h: torch.Tensor, w: torch.Tensor, eps: float, xn: torch.Tensor,
                parts: Optional[torch.Tensor] = None, ids: Optional[torch.Tensor] = None,
                emb: Optional[torch.Tensor] = None, row_idx: Optional[torch.Tensor] = None,
                write_h: bool = True, rows: Optional[int] = None, xf: bool = False,
                ss_out: Optional[torch.Tensor] = None, ss_ld: int = 0, ss_nzero: int = 0,
                x8: Optional[torch.Tensor] = None, sx8: Optional[torch.Tensor] = None) -> torch.Tensor:
    """h[r] (= emb[ids[r]]) (+= sum parts[:, r]); xn[m] = rmsnorm(h[row_idx[m]]) * w.
    xf=True: xn is a flat buffer receiving the fragment-major layout (``to_xfrag``) of ``rows`` rows.
    ss_out (raw mode, the norm folded into the next GEMMs): xn = bf16(h) un-normalised, ss_out[m] = sum h^2,
    and ss_out[k * ss_ld + m] = 0 for k = 1..ss_nzero (the accumulators of the later residual epilogues).
    x8 / sx8: the same rows also as per-row-scaled e4m3 in the xf8 layout (``linear_a8`` input; quantised from
    the f32 values, before the bf16 rounding of xn)."""
    assert x8 is None or xf, "the fp8 output rides on the fragment-major (xf) decode layout"
    if x8 is not None and not _gpu(h):
        add_rmsnorm(h, w, eps, xn, parts, ids, emb, row_idx, write_h, rows, xf, ss_out, ss_ld, ss_nzero)
        n = rows if rows is not None else xn.shape[0]
        xr = from_xfrag(xn, n, w.numel()) if xf else xn[:n]
        quantize_xf8(xr, xfrag_tiles(n), x8, sx8)
        return xn
    if rows is None:
        assert not xf, "xf output needs rows"
        rows = xn.shape[0]
    if ss_out is not None and not _gpu(h):
        tmp = torch.empty(rows, w.numel(), dtype=torch.bfloat16, device=h.device)
        ref.add_rmsnorm(h, torch.ones_like(w), eps, tmp, parts, ids, emb, row_idx, write_h)
        hv = h[:rows].float()
        raw = hv.to(torch.bfloat16)
        if xf:
            f = to_xfrag(raw)
            xn.view(-1)[: f.numel()].copy_(f)
        else:
            xn[:rows].copy_(raw)
        ss_out[:rows] = ss_q24(hv.pow(2).sum(1))
        for k in range(1, ss_nzero + 1):
            ss_out[k * ss_ld: k * ss_ld + rows] = 0
        return xn
    if not _gpu(h):
        if not xf:
            return ref.add_rmsnorm(h, w, eps, xn, parts, ids, emb, row_idx, write_h)
        tmp = torch.empty(rows, w.numel(), dtype=torch.bfloat16, device=h.device)
        ref.add_rmsnorm(h, w, eps, tmp, parts, ids, emb, row_idx, write_h)
        f = to_xfrag(tmp)
        xn.view(-1)[: f.numel()].copy_(f)
        return xn
    nparts = parts.shape[0] if parts is not None else 0
    stride = parts.stride(0) if parts is not None else 0
    ext().add_rmsnorm(h, parts, nparts, stride, ids, emb, row_idx, write_h, w, eps, xn, rows,
                      xfrag_tiles(rows) if (xf or x8 is not None) else 0, ss_out, ss_ld, ss_nzero, x8, sx8)
    return xn


def prefetch(tensors, nbytes=None, wgs: int = 512) -> None:
    """Infinity-Cache warm-up: stream (the first ``nbytes[k]`` bytes of) up to four tensors through the memory
    hierarchy with allocating loads and no stores, so the next kernel reading them hits the 256 MiB die-level cache.
    Issued on a side stream of the captured decode step (``ModelRunner.prefetch_plan``).  No-op off the GPU."""
    tensors = [t for t in tensors if t is not None]
    if not tensors or not _gpu(tensors[0]):
        return
    nb = list(nbytes) if nbytes is not None else [-1] * len(tensors)
    ext().prefetch(tensors, [int(b) for b in nb], int(wgs))


def rr_supported(w: PackedWeight, K: int, splitk: int = 1) -> bool:
    """Whether a batch-1 decode GEMM can take the residual-reduce prologue (``linear_rr``): bf16 weights and a K slice
    per split that fits the kernel's LDS image (gemm.hip RR_KMAX)."""
    return w.kind in ("bf16", "dense") and K % 32 == 0 and (K // 32 + splitk - 1) // splitk * 32 <= 8192


def linear_rr(h: torch.Tensor, parts: torch.Tensor, h_out: torch.Tensor, w: PackedWeight, epi: str,
              out: Optional[torch.Tensor] = None, ss_out: Optional[torch.Tensor] = None, eps: float = 1e-5,
              splitk: Optional[int] = None, nb: Optional[int] = None, waves: Optional[int] = None,
              div: Optional[int] = None) -> torch.Tensor:
    """Batch-1 decode projection with the residual add folded into its prologue (gemm.hip RR; lsa_epi.h LsaRr).

    x = h + sum_s parts[s] (h: f32 [1, K] residual stream, parts: f32 [S, 1, K] split-K slabs of the previous
    row-parallel projection); h_out <- x (the next residual stream, a different buffer than h).  The RMSNorm gamma is
    folded into W (``norms_folded``); the RMS row scale r = rsqrt(mean(x^2) + eps) is applied
      * epi='silu': in the epilogue (splitk 1; each workgroup reduces the whole row itself) -> bf16 [1, N/2];
      * epi='f32': NOT here -- the output is [splitk, 1, N] f32 slabs of W @ bf16(x), and sum x^2 is added to
        ss_out[0] (Q24 int64, must be zero on entry) for the slab consumer (``attn_decode(rownorm=...)``).
    Replaces the ``res_add_ss`` launch between the two projections (one kernel boundary less per layer side)."""
    K = w.K
    assert epi in ("f32", "silu") and h.numel() >= K and parts.dim() == 3 and parts.shape[1] == 1
    nb0, sk0, wv0, dv0 = rr_config(w.N, K, epi, w.kind)
    splitk = 1 if epi == "silu" else (sk0 if splitk is None else splitk)
    nb = nb0 if nb is None else nb
    if not _gpu(h):
        x = h.view(-1)[:K].float() + parts.float().sum(0).view(-1)
        h_out.view(-1)[:K].copy_(x)
        xb = x.to(torch.bfloat16).view(1, K)
        if epi == "silu":
            r = torch.rsqrt(x.pow(2).sum() / K + eps)
            y = ref.linear(xb, w.dense(), "f32") * r
            g, u = y.view(-1, 2, 16)[:, 0].reshape(1, -1), y.view(-1, 2, 16)[:, 1].reshape(1, -1)
            res = (torch.nn.functional.silu(g) * u).to(torch.bfloat16)
            if out is None:
                return res
            out.view(-1)[: res.numel()].copy_(res.view(-1))
            return out
        assert ss_out is not None
        ss_out.view(-1)[:1] += ss_q24(x.pow(2).sum().view(1))
        y = ref.linear(xb, w.dense(), "f32").unsqueeze(0)
        if out is None:
            return y
        out.view(-1)[: y.numel()].copy_(y.reshape(-1))
        return out
    waves = wv0 if waves is None else waves
    div = dv0 if div is None else div
    if out is None:
        out = (torch.empty(splitk, 1, w.N, device=h.device, dtype=torch.float32) if epi == "f32" else
               torch.empty(1, w.N // 2, device=h.device, dtype=torch.bfloat16))
    ext().gemm_rr(h.view(-1)[:K], parts, h_out.view(-1), w.data, w.N, out, EPI[epi], nb, splitk, waves, div,
                  ss_out=ss_out, eps=float(eps))
    return out


def res_add_ss(h: torch.Tensor, parts: Optional[torch.Tensor], xn: torch.Tensor, rows: int, ss_out: torch.Tensor,
               xf: bool = False) -> torch.Tensor:
    """Residual add of the folded-norm decode step (the RMSNorm gammas live in the next GEMM's weight, which scales
    its output rows by rsqrt(ss / d + eps), ``linear(..., rownorm=(ss_out, eps))``):
    h[:rows] += sum_s parts[s];  xn = bf16(h) (fragment-major when xf);  ss_out[:rows] += sum h^2 (Q24 int64).
    ss_out must be zero on entry.  One wave per 512-column slice on the GPU (norm_rope.hip res_add_ss_kernel)."""
    D = h.shape[1]
    if not _gpu(h):
        hv = h[:rows].float()
        if parts is not None:
            hv = hv + parts[:, :rows].float().sum(0)
        h[:rows].copy_(hv)
        x16 = hv.to(torch.bfloat16)
        if xf:
            f = to_xfrag(x16)
            xn.view(-1)[: f.numel()].copy_(f)
        else:
            xn[:rows].copy_(x16)
        ss_out[:rows] += ss_q24(hv.pow(2).sum(1))
        return xn
    nparts = parts.shape[0] if parts is not None else 0
    stride = parts.stride(0) if parts is not None else 0
    ext().res_add_ss(h, parts, nparts, stride, xn, rows, D, xfrag_tiles(rows) if xf else 0, ss_out)
    return xn


def rope_append(qkv, pos, tok_seq, block_tables, cos_t, sin_t, q_out, kc, vc, H, Hkv, kv_scales=None):
    """RoPE of q / k and the paged-cache append of k / v.  kv_scales = (ks, vs): fp8 cache (``KV_FP8``), kc / vc
    are uint8 e4m3 bytes and every (token, kv-head) row is stored with its own f32 scale."""
    if not _gpu(qkv):
        return ref.rope_append(qkv, pos, tok_seq, block_tables, cos_t, sin_t, q_out, kc, vc, H, Hkv, kv_scales)
    ks, vs = kv_scales if kv_scales is not None else (None, None)
    ext().rope_append(qkv, pos, tok_seq, block_tables, cos_t, sin_t, q_out, kc, vc, H, Hkv, ks, vs)


def silu_parts(parts: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out [M, F] = silu(gate) * up from f32 split-K slabs [S, M, 2F] of the interleaved gate_up GEMM."""
    if not _gpu(parts):
        S, M, N = parts.shape
        y = parts.float().sum(0).view(M, N // 32, 2, 16)
        g, u = y[:, :, 0, :].reshape(M, N // 2), y[:, :, 1, :].reshape(M, N // 2)
        out.copy_((torch.nn.functional.silu(g) * u).to(out.dtype))
        return out
    ext().silu_parts(parts, out)
    return out


def silu_mul(g: torch.Tensor, u: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if out is None:
        out = torch.empty_like(g)
    if not _gpu(g):
        out.copy_((torch.nn.functional.silu(g.float()) * u.float()).to(out.dtype))
        return out
    ext().silu_mul(g, u, out)
    return out


# ----------------------------------------------------------------------------------- attention
# fp8 KV cache (LSA_KV_FP8=1 or ModelRunner(kv_dtype="fp8")): the paged cache holds e4m3 bytes with one f32 scale
# per (token, kv-head) row of 128 values (amax / 448) -- half the bytes of the memory-bound decode attention and
# twice the tokens per GiB of cache.  Decode attention reads the bytes directly; prefill widens the blocks it
# attends to into a bf16 scratch per layer (kv8_dequant).  Off by default: it is a lossy cache (relative error
# ~2^-4 per element), checked against the oracle's own fp8-cache emulation (models.llama.reference_forward kv_fp8).
KV_FP8 = os.environ.get("LSA_KV_FP8", "0") == "1"


def kv8_scratch(ctx: list[int], Hkv: int, device) -> tuple:
    """(ko, vo, table) for ``attn_prefill``'s fp8 path: compact bf16 scratch of every block the sequences with
    contexts ``ctx`` attend to (sequence i's block j at i * mb + j) and the matching [n, mb] block table."""
    mb = max(1, max((c + 63) // 64 for c in ctx))
    n = len(ctx)
    ko = torch.empty(n * mb, Hkv, 64, 128, dtype=torch.bfloat16, device=device)
    vo = torch.empty_like(ko)
    table = torch.arange(n * mb, dtype=torch.int32, device=device).view(n, mb)
    return ko, vo, table


# experiment overrides of the split-KV decode plan, {(B, Hkv): (chunk_blocks, nsplit, unsplit_max)} (in-engine A/Bs,
# scripts/ab_rr_cfg.py "plan:B:Hkv" keys); empty in production
DECODE_PLAN_OVERRIDES: dict = {}


def decode_split_plan(B: int, Hkv: int, max_ctx: int) -> tuple[int, int, int]:
    """(chunk_blocks, nsplit, unsplit_max) grid plan of split-KV decode for contexts up to max_ctx.  The
    kernel picks each sequence's own split from its length (csrc/kernels/attention.hip eff_split):
    <= unsplit_max blocks run unsplit, longer contexts are cut into nsplit pieces of at least chunk_blocks
    blocks, so a sequence shorter than max_ctx uses fewer, equally long splits.

    Measured on MI355X (scripts/bench_attn.py, profiles/attn_split_plans_mi355x.jsonl): the best grid is
    about 256 workgroups, i.e. one per CU of (sequence, kv-head) pairs x splits.  At >= 256 pairs (7B at
    batch >= 8, 3B at batch >= 32) every context runs unsplit (3B B=32 ctx 2048: 77.2 -> 46.4 us, 7B B=32
    ctx 512: 53.9 -> 44.6 us vs the earlier fixed 4-block chunks); 64 pairs -> 4 splits (3B B=8 ctx 2048:
    31.8 -> 16.8 us); 8 pairs (3B at batch 1) -> up to 32 splits of >= 2 blocks (17 at 2k context).
    Contexts of <= 4 blocks run unsplit (a combine costs more than it spreads), except on grids of <= 8
    pairs, where one block per split still wins (3B B=1 ctx 200: 8.65 -> 7.32 us)."""
    if (B, Hkv) in DECODE_PLAN_OVERRIDES:
        return tuple(DECODE_PLAN_OVERRIDES[(B, Hkv)])
    nblk = max(1, (max_ctx + 63) // 64)
    pairs = max(1, B * Hkv)
    if nblk <= 4:  # every sequence runs unsplit (eff_split): no empty split workgroups, no combine
        if pairs <= 8 and nblk > 1:
            return 1, nblk, 0
        return nblk, 1, 4
    nsplit = min(max(1, round(256 / pairs)), (nblk + 1) // 2, 256)
    if nsplit <= 1:
        return nblk, 1, 4
    return 2, nsplit, 4


def decode_workspace(B: int, H: int, Hkv: int, nsplit: int, device) -> tuple:
    """(opart, mlpart, counters) for split-KV decode: per-split partial outputs / (max, sum) pairs and the
    per-(sequence, kv-head) arrival tickets of the in-kernel combine (must start zeroed; the kernel
    leaves them zeroed)."""
    return (torch.empty(B * H * max(nsplit, 1) * 128, device=device, dtype=torch.float32),
            torch.empty(B * H * max(nsplit, 1) * 2, device=device, dtype=torch.float32),
            torch.zeros(B * Hkv, device=device, dtype=torch.int32))


def attn_decode(q, kc, vc, block_tables, pos, H, Hkv, scale, out, workspace=None, plan=None, xf=False,
                qkv_parts=None, cos=None, sin=None, kv_scales=None, out_s8=None, rownorm=None):
    """q [B,H,128] vs paged cache, context = pos + 1.  workspace = decode_workspace(...) for split-KV.
    xf=True: out is a flat buffer receiving the fragment-major layout of the [B, H*128] output.
    qkv_parts ([S, B, (H+2Hkv)*128] f32 split-K slabs of the QKV projection) + cos/sin: RoPE and the
    KV-cache append of the new token are fused in (``q`` is then only a [B, H, 128] scratch buffer).
    kv_scales = (ks, vs): fp8 cache (see ``KV_FP8``).
    out_s8 (xf only): ``out`` is a uint8 buffer receiving the output as e4m3 in the xf8 layout with one E8M0 scale
    per (row, head) in ``out_s8`` -- the input of a W8A8 / W4A8 o projection (``linear_a8(s8=)``).
    rownorm = (ss, eps, hidden): the slabs are the projection of UN-normalised rows (``linear_rr``); row b's q / k / v
    are scaled by rsqrt(ss[b] / hidden + eps) (ss Q24 int64) before RoPE."""
    B = pos.shape[0]
    assert out_s8 is None or xf, "the e4m3 attention output lives in the xf8 layout"
    assert rownorm is None or qkv_parts is not None, "rownorm scales the fused-RoPE slabs"
    if not _gpu(pos):
        if rownorm is not None:
            r = torch.rsqrt(ss_float(rownorm[0][:B]) / rownorm[2] + rownorm[1])
            qkv_parts = qkv_parts[:, :B].sum(0, keepdim=True) * r.view(1, B, 1)
        if qkv_parts is not None:
            ref.rope_append(qkv_parts, pos, None, block_tables, cos, sin, q, kc, vc, H, Hkv, kv_scales)
        if out_s8 is not None:
            tmp = torch.empty(B, H, q.shape[-1], dtype=torch.bfloat16, device=q.device)
            ref.attn_decode(q, kc, vc, block_tables, pos, H, Hkv, scale, tmp, kv_scales)
            quantize_xf8_blocks(tmp.view(B, -1), 128, xfrag_tiles(B), out, out_s8)
            return out
        if not xf:
            return ref.attn_decode(q, kc, vc, block_tables, pos, H, Hkv, scale, out, kv_scales)
        tmp = torch.empty(B, H, q.shape[-1], dtype=torch.bfloat16, device=q.device)
        ref.attn_decode(q, kc, vc, block_tables, pos, H, Hkv, scale, tmp, kv_scales)
        f = to_xfrag(tmp.view(B, -1))
        out.view(-1)[: f.numel()].copy_(f)
        return out
    plan = plan if plan is not None else decode_split_plan(B, Hkv, block_tables.shape[1] * 64)
    chunk, nsplit = plan[0], plan[1]
    unsplit_max = plan[2] if len(plan) > 2 else 4
    if workspace is None:
        workspace = decode_workspace(B, H, Hkv, nsplit, q.device)
    opart, mlpart, counters = workspace
    ks, vs = kv_scales if kv_scales is not None else (None, None)
    ext().attn_decode(q, kc, vc, block_tables, pos, H, Hkv, scale, chunk, nsplit, out, opart, mlpart, counters,
                      xfrag_tiles(B) if xf else 0, qkv_parts, cos, sin, unsplit_max, ks, vs, out_s8=out_s8,
                      **({} if rownorm is None else dict(rowss=rownorm[0], eps=float(rownorm[1]),
                                                          hidden=int(rownorm[2]))))
    return out


# prefill attention kernel: "32" = 32 x 32 MFMA tiles, 128 query rows per workgroup (attention_prefill32.hip);
# "16" = the 16 x 16 kernel of attention.hip (64 rows per workgroup); "auto" = 32 when the longest packed
# sequence has >= 512 rows (measured, scripts/bench_attn_prefill.py: 7B 2k 146 -> 119 us, 3B 2k 118 -> 115 us,
# 8k 1051 -> 1021 us), else 16 (32 x 128-token prompts: 28 vs 31 us, twice the work items)
PREFILL_ATTN = "auto"


def _prefill_kernel(cu_q: list) -> str:
    if PREFILL_ATTN != "auto":
        return PREFILL_ATTN
    longest = max((cu_q[i + 1] - cu_q[i] for i in range(len(cu_q) - 1)), default=0)
    return "32" if longest >= 512 else "16"


def prefill_qblock(cu_q: Optional[list] = None) -> int:
    k = _prefill_kernel(cu_q or [0])
    return 128 if k == "32" else ext().prefill_qblock


def prefill_work(cu_q: list[int], qblock: Optional[int] = None, ctx: Optional[list[int]] = None,
                 kernel: Optional[str] = None, heads: int = 32) -> list:
    """Work items of the prefill attention kernel for packed sequences (cu_q offsets; ``ctx`` = per-sequence
    context length after this prefill, default = the chunk length, i.e. no cached prefix).

    16-row kernel: (seq, q_start) per workgroup, heaviest (latest) query blocks first.
    32-row kernel ('32'): NG items (seq, q_start, t0, t1) per workgroup -- the key tiles [t0, t1) = the whole causal
    range of a 128-row query block; NG = 2 pairs a heavy block with a light one (``_pair_blocks``).  (Cutting heavy
    blocks into KV-split pieces -- merged by a second launch, in LDS, or in the same launch through write-through
    partials -- was built three times and measured slower each time: profiles/attn_prefill_kv_split_mi355x.jsonl,
    profiles/attn_prefill_halves_mi355x.jsonl, profiles/r5/attn_prefill_kv_split_inlaunch_ab_mi355x.jsonl: a CU is
    throughput-bound on one busy group, so halving the longest chain only moves work between groups.)"""
    kernel = kernel or _prefill_kernel(cu_q)
    if qblock is None:
        qblock = 128 if kernel == "32" else ext().prefill_qblock
    items = []
    for s in range(len(cu_q) - 1):
        ql = cu_q[s + 1] - cu_q[s]
        pos0 = (ctx[s] - ql) if ctx is not None else 0
        for qs in range(0, ql, qblock):
            items.append(((pos0 + min(qs + qblock, ql) + 63) // 64, s, qs))
    items.sort(key=lambda t: -t[0])
    if kernel != "32":
        return [(s, qs) for _, s, qs in items]
    units = [(s, qs, 0, nt) for nt, s, qs in items]
    empty = (-1, 0, 0, 0)
    n = len(units)
    longest = max(cu_q[i + 1] - cu_q[i] for i in range(len(cu_q) - 1))
    if not _pair_blocks(n, heads, longest, qblock):
        return units
    out = []
    for i in range((n + 1) // 2):
        j = n - 1 - i
        b = units[j] if j > i else empty
        out.append(units[i] + b)
    return out


class PrefillPlan(NamedTuple):
    """Device-side plan of one prefill attention call (``prefill_plan``)."""
    kernel: str
    work: torch.Tensor  # int32 [n_workgroups, 2 | 4 * NG]


def prefill_plan(cu_q: list[int], ctx: Optional[list[int]] = None, heads: int = 32, device=None,
                 kernel: Optional[str] = None) -> PrefillPlan:
    """Work items of the prefill attention kernel for packed sequences, on ``device``."""
    kernel = kernel or _prefill_kernel(cu_q)
    rows = prefill_work(cu_q, ctx=ctx, kernel=kernel, heads=heads)
    w = torch.tensor(rows, dtype=torch.int32)
    if device is not None:
        w = w.to(device, non_blocking=True)
    return PrefillPlan(kernel, w)


# auto | 1 | 0 -- heavy/light paired query blocks in the 32-row prefill kernel
PREFILL_PAIR = "auto"


def _pair_blocks(n_items: int, heads: int, longest: int, qblock: int) -> bool:
    """Pair when every single block would be resident at once (<= 2 per CU on 256 CUs: the dispatch order
    then fixes which blocks share a CU, and heavy ones can land together) or for very long sequences; with
    more blocks than slots the hardware's dynamic dispatch balances them better (scripts/bench_attn_prefill.py,
    profiles/attn_prefill_pairing_mi355x.jsonl: 7B 2k 103 -> 89 us paired, 3B 2k 97 -> 84, 3B 8k 730 -> 695;
    4 x 1k 3B single 83 vs paired 90)."""
    if PREFILL_PAIR != "auto":
        return PREFILL_PAIR == "1"
    return n_items * heads <= 512 or longest >= 32 * qblock


def attn_prefill(q, kc, vc, block_tables, cu_q, ctx_lens, H, Hkv, scale, out, work=None, cu_list=None,
                 kv_scales=None, kv8_scratch_=None, xf: bool = False):
    """Causal prefill attention of packed sequences (cu_q offsets) over the paged cache.  ``work``: the
    ``prefill_plan`` of the same offsets (or None: planned here from ``cu_list`` / the device offsets).
    kv_scales = (ks, vs): fp8 cache -- the attended blocks are widened into ``kv8_scratch_`` (= kv8_scratch(ctx,
    ...), built from the host context list; made here when not given) and the bf16 kernels run on that.
    xf: ``out`` is a flat buffer receiving the fragment-major layout (``to_xfrag``) of the [T, H * 128] rows -- the
    o projection's stream-K input."""
    T = q.shape[0]
    if not _gpu(q):
        if not xf:
            return ref.attn_prefill(q, kc, vc, block_tables, cu_q, ctx_lens, H, Hkv, scale, out, kv_scales)
        tmp = ref.attn_prefill(q, kc, vc, block_tables, cu_q, ctx_lens, H, Hkv, scale, torch.empty_like(q), kv_scales)
        f = to_xfrag(tmp.reshape(T, -1))
        out.view(-1)[: f.numel()].copy_(f)
        return out
    if kv_scales is not None:
        ko, vo, table = kv8_scratch_ if kv8_scratch_ is not None else kv8_scratch(ctx_lens.tolist(), Hkv, q.device)
        ext().kv8_dequant(kc, vc, kv_scales[0], kv_scales[1], block_tables, ctx_lens, table.shape[1], ko, vo)
        kc, vc, block_tables = ko, vo, table
    cu = cu_list if cu_list is not None else cu_q.tolist()
    plan = work if isinstance(work, PrefillPlan) else None
    if plan is None:
        plan = (prefill_plan(cu, ctx=ctx_lens.tolist(), heads=H, device=q.device) if work is None
                else PrefillPlan(_prefill_kernel(cu), work))
    ext().attn_prefill(q, kc, vc, block_tables, cu_q, ctx_lens, plan.work, H, Hkv, scale, out,
                       1 if plan.kernel == "32" else 0, xfrag_tiles(T) if xf else 0)
    return out


# ----------------------------------------------------------------------------------- sampling
def _row_defaults(B, out_tokens, limit, eos_on):
    dev = out_tokens.device
    if limit is None:
        limit = torch.full((B,), out_tokens.shape[1], dtype=torch.int32, device=dev)
    if eos_on is None:
        eos_on = torch.ones(B, dtype=torch.int32, device=dev)
    return limit, eos_on


def argmax_commit(logits, out_tokens, gen_len, input_ids, positions, finished, eos, limit=None, eos_on=None,
                  part=None):
    """Greedy token + in-place decode-state update (see kernels/sampling.hip)."""
    B, V = logits.shape
    limit, eos_on = _row_defaults(B, out_tokens, limit, eos_on)
    if not _gpu(logits):
        return ref.argmax_commit(logits, out_tokens, gen_len, input_ids, positions, finished, eos, limit, eos_on)
    if part is None:
        part = torch.empty(B * ((V + 4095) // 4096), device=logits.device, dtype=torch.int64)
    ext().argmax_commit(logits, part, out_tokens, gen_len, input_ids, positions, finished, eos, limit, eos_on)


def sample_commit(logits, hist, penalty, temperature, top_k, top_p, seeds, out_tokens, gen_len, input_ids,
                  positions, finished, eos, limit=None, eos_on=None, workspace=None, last_n=None):
    """Temperature / top-k / top-p draw (+ optional repetition penalty) + decode-state update.

    ``hist`` [B, W] int32 is the ring of each row's last W context tokens (token at position p in column
    p % W, -1 = empty); with it, rows whose ``penalty`` != 1 have the logits of the distinct tokens among
    their last ``last_n`` (<= W, default W) positions penalised (Ollama ``repeat_penalty`` /
    ``repeat_last_n``), and the committed token is written into the ring.  ``logits`` is modified."""
    B, V = logits.shape
    limit, eos_on = _row_defaults(B, out_tokens, limit, eos_on)
    if not _gpu(logits):
        return ref.sample_commit(logits, hist, penalty, temperature, top_k, top_p, seeds, out_tokens, gen_len,
                                 input_ids, positions, finished, eos, limit, eos_on, last_n=last_n)
    if workspace is None:
        part = torch.empty(B * ((V + 4095) // 4096), device=logits.device, dtype=torch.int64)
        cand = torch.empty(B * ((V + 2047) // 2048) * 64, device=logits.device, dtype=torch.int64)
    else:
        part, cand = workspace
    ext().sample_commit(logits, part, cand, hist, penalty, last_n, temperature, top_k, top_p, seeds, out_tokens,
                        gen_len, input_ids, positions, finished, eos, limit, eos_on)
