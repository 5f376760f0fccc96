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
