"""Where one bench step's time goes, from a rocprofv3 kernel_trace.csv of ``bench.py``: per timed step,
prefill (first prefill-GEMM launch -> first decode commit) vs decode (commit -> last commit), the decode
step period, the idle gap between decode graph replays, and the per-layer decode kernel sequence."""
import csv
import statistics
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
commits = [i for i, r in enumerate(rows) if "commit_kernel" in r[2]]
period = [(rows[b][1] - rows[a][1]) / 1e3 for a, b in zip(commits, commits[1:]) if 100 < b - a < 400]
gap = [(rows[a + 1][0] - rows[a][1]) / 1e3 for a, b in zip(commits, commits[1:]) if 100 < b - a < 400]
# generate() calls: a prefill GEMM (256^2 / 128^2 tile kernel) after a decode commit starts a new call
starts, last_commit = [], True
for i, r in enumerate(rows):
    if "commit_kernel" in r[2]:
        last_commit = True
    elif ("gemm_sk" in r[2] or "gemm_t256" in r[2]) and last_commit:
        starts.append(i)
        last_commit = False
for k, s0 in enumerate(starts):
    s1 = starts[k + 1] if k + 1 < len(starts) else len(rows)
    cs = [c for c in commits if s0 < c < s1]
    if len(cs) < 16:
        continue
    pre = (rows[cs[0]][1] - rows[s0][0]) / 1e6
    dec = (rows[cs[-1]][1] - rows[cs[0]][1]) / 1e6
    print(f"generate() #{k}: prefill {pre:.1f} ms (from the first prefill GEMM), decode {dec:.1f} ms over "
          f"{len(cs)} commits ({100 * pre / (pre + dec):.1f} % prefill)")
a, b = commits[len(commits) // 2], commits[len(commits) // 2 + 1]
print("one decode step, first 8 kernels (us):")
for i in range(a + 1, min(b, a + 9)):
    print(f"  {(rows[i][1] - rows[i][0]) / 1e3:8.2f}  {rows[i][2][:70]}")
