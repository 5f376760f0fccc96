"""Persistent decode block (ops.decode_block) alone at the 7B / 3B decode shapes: us per launch and the weight
stream's effective bandwidth, over a sweep of tile plans and grid sizes.  Weights rotate over 4 layer copies
(> MALL) so they stream from HBM.  One JSON line per (shape, B, cfg, nwg).

    python scripts/bench_decode_block.py [Bs] [cfg;cfg..] [nwg,nwg..] [--stamps]

--stamps: also one stamped launch per point (after 3 unstamped ones): per phase boundary the min / median / max
over workgroups of the wall-clock time since the earliest workgroup start (us).
      cfg = nbo,nbg,nbd,nbq      ("-": ops.decode_block_cfg(B))
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"7b": (4096, 4096, 11008, 12288), "3b": (3072, 3072, 8192, 5120)}
_pos = [a for a in sys.argv[1:] if not a.startswith("--")]
Bs = [int(v) for v in _pos[0].split(",")] if len(_pos) > 0 else [1, 8, 32, 64]
CFGS = [tuple(int(x) for x in c.split(",")) for c in _pos[1].split(";")] if len(_pos) > 1 and _pos[1] != "-" else [None]
NWGS = [int(v) for v in _pos[2].split(",")] if len(_pos) > 2 else [0]
STAMPS = "--stamps" in sys.argv
NAMES = ["start", "prologue", "o_done", "o_complete", "gu_done", "gu_complete", "down_done", "down_complete", "qkv_done"]


def main():
    ncu = ops.num_cus(dev)
    for name, (d, hd, ffn, nq) in SHAPES.items():
        layers = []
        for i in range(4):
            mk = lambda n, k: ops.PackedWeight.from_dense(torch.randn(n, k, device=dev).mul_(k ** -0.5).to(torch.bfloat16))
            layers.append((mk(d, hd), mk(2 * ffn, d), mk(d, ffn), mk(nq, d)))
        wbytes = 2 * (d * hd + 2 * ffn * d + d * ffn + nq * d)
        for B in Bs:
            attn = torch.randn(64 * hd, device=dev).to(torch.bfloat16)
            h = torch.randn(64, d, device=dev)
            x = torch.zeros(64 * d, device=dev, dtype=torch.bfloat16)
            act = torch.zeros(64 * ffn, device=dev, dtype=torch.bfloat16)
            qout = torch.empty(64 * nq, device=dev)
            ss = torch.zeros(2, 64, device=dev, dtype=torch.long)
            cnt = torch.zeros(64, ops.DECODE_BLOCK_CNT_INTS, device=dev, dtype=torch.int32)
            err = torch.zeros(1, device=dev, dtype=torch.int32)
            for cfg in CFGS:
                c = cfg or ops.decode_block_cfg(B)
                for nwg in NWGS:
                    n = nwg or ncu

                    def run(i):
                        wo, wgu, wd, wq = layers[i % 4]
                        ops.decode_block(attn, wo, h, x, ss[0], ss[1], wgu, act, wd, wq, qout, B, 1e-5, cnt[i % 64],
                                         err, cfg=c, nwg=n)

                    try:
                        for i in range(8):
                            cnt.zero_(); ss.zero_()
                            run(i)
                        torch.cuda.synchronize()
                        ts = []
                        for rep in range(3):
                            cnt.zero_(); ss.zero_()
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record()
                            for i in range(64):
                                run(i)
                            e1.record()
                            torch.cuda.synchronize()
                            ts.append(e0.elapsed_time(e1) * 1000 / 64)
                        us = sorted(ts)[1]
                        rec = {"shape": name, "B": B, "cfg": list(c), "nwg": n, "us": round(us, 2),
                               "TBps": round(wbytes / us / 1e6, 2), "err": int(err[0])}
                    except Exception as e:  # noqa: BLE001 - an unsupported plan is a result, not a crash
                        rec = {"shape": name, "B": B, "cfg": list(c), "nwg": n, "error": str(e)[:200]}
                    if STAMPS and "us" in rec:
                        st = torch.zeros(n, 16, device=dev, dtype=torch.long)
                        cnt.zero_(); ss.zero_()
                        for i in range(3):
                            run(i)
                        wo, wgu, wd, wq = layers[3]
                        ops.decode_block(attn, wo, h, x, ss[0], ss[1], wgu, act, wd, wq, qout, B, 1e-5, cnt[3], err,
                                         cfg=c, nwg=n, stamps=st)
                        torch.cuda.synchronize()
                        st = st.cpu()
                        st = st[st[:, 0] > 0]  # the launcher clamps the grid to the co-resident capacity
                        khz = ops.ext().ar_wallclock_khz()
                        t0 = int(st[:, 0].min())
                        us = (st[:, :9] - t0).double() * 1000.0 / khz
                        rec["stamps_us"] = {k: [round(float(us[:, i].min()), 1), round(float(us[:, i].median()), 1),
                                                round(float(us[:, i].max()), 1)] for i, k in enumerate(NAMES)}
                        rec["o_drained_us"] = [round(float(v), 1) for v in
                                               ((st[:, 13] - t0).double() * 1000.0 / khz).quantile(
                                                   torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64)).tolist()]
                        rec["items"] = {k: [int(st[:, 9 + i].min()), int(st[:, 9 + i].max())]
                                        for i, k in enumerate(["o", "gu", "down", "qkv"])}
                    print(json.dumps(rec), flush=True)
                    if int(err[0]):
                        return


if __name__ == "__main__":
    main()
