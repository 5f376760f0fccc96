"""Decode-step timeline from a rocprofv3 kernel_trace.csv: per decode step (delimited by the
argmax/sample commit kernel) the wall span, the summed kernel time and the idle gap between kernels."""
import csv
import statistics
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
steps, cur = [], []
for r in rows:
    cur.append(r)
    if "commit_kernel" in r[2]:
        steps.append(cur)
        cur = []
spans, busy, nk = [], [], []
for st in steps[2:]:  # skip the first (warm-up / prefill) ones
    if len(st) < 8:
        continue
    s0, s1 = st[0][0], st[-1][1]
    spans.append((s1 - s0) / 1e3)
    busy.append(sum(e - s for s, e, _ in st) / 1e3)
    nk.append(len(st))
# graph boundary: idle time between one step's commit kernel and the next step's first kernel
between = [(b[0][0] - a[-1][1]) / 1e3 for a, b in zip(steps[2:], steps[3:]) if len(a) >= 8 and len(b) >= 8]
if spans:
    med = statistics.median
    print(f"decode steps {len(spans)}: span {med(spans):.1f} us, kernel-busy {med(busy):.1f} us, "
          f"gaps {med(spans) - med(busy):.1f} us over {int(med(nk))} kernels "
          f"({(med(spans) - med(busy)) / max(1, med(nk)):.2f} us/kernel)")
if between:
    print(f"between steps (commit end -> next step's first kernel): median {statistics.median(between):.1f} us, "
          f"mean {statistics.mean(between):.1f} us over {len(between)} boundaries")

# round level: idle stretches > 20 us anywhere in the trace (host work between a round's decode run and the next
# round's prefill, prefill host preparation, result read-back), with the kernels on either side
idle = []
for a, b in zip(rows, rows[1:]):
    g = (b[0] - a[1]) / 1e3
    if g > 20:
        idle.append((g, a[2][:48], b[2][:48]))
if idle:
    tot = sum(g for g, _, _ in idle)
    print(f"idle stretches > 20 us: {len(idle)}, total {tot / 1e3:.2f} ms over a {(rows[-1][1] - rows[0][0]) / 1e6:.1f} ms trace")
    by = {}
    for g, a, b in idle:
        k = (a, b)
        c, s = by.get(k, (0, 0.0))
        by[k] = (c + 1, s + g)
    for (a, b), (c, s) in sorted(by.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {c:4d} x {s / c:9.1f} us  after {a}  before {b}")
# prefill segments: from the first engine prefill kernel (stream-K GEMM, prefill attention, rope/append) to the commit
# kernel that ends the prefill; kernel-busy = every kernel in that window; per-kernel totals of the median one.  Vendor
# GEMMs (Cijk_*) inside a segment are counted and reported; outside them (the bench's fp32 numerics oracle) they are not
# engine work.  ("gemm_sk_kernel", not "gemm_sk": the decode GEMV is gemm_skinny_kernel.)
PRE = ("gemm_sk_kernel", "attn_prefill", "rope_append")
seg, segs = [], []
for r in rows:
    if seg or any(p in r[2] for p in PRE):
        seg.append(r)
        if "commit_kernel" in r[2]:
            segs.append(seg)
            seg = []
if segs:
    spans = sorted(((s[-1][1] - s[0][0]) / 1e3, i) for i, s in enumerate(segs))
    med_span, mi = spans[len(spans) // 2]
    ms = segs[mi]
    busy = sum(e - s for s, e, _ in ms) / 1e3
    print(f"prefill segments {len(segs)}: median span {med_span:.0f} us, its kernel time {busy:.0f} us "
          f"({len(ms)} kernels, {med_span - busy:.0f} us idle)")
    by = {}
    for s, e, n in ms:
        k = n[:60]
        c, t = by.get(k, (0, 0.0))
        by[k] = (c + 1, t + (e - s) / 1e3)
    for k, (c, t) in sorted(by.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"  {t:8.1f} us  {c:4d} x {t / c:7.1f}  {k}")
    vendor = sum(1 for sg in segs for r in sg if "Cijk" in r[2])
    print(f"vendor (Cijk_*) kernels inside the {len(segs)} prefill segments: {vendor}")
