"""Condense a rocprofv3 kernel_stats.csv: short kernel names, total ms, % and avg us."""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':60s} {'calls':>7s} {'total_ms':>9s} {'pct':>6s} {'avg_us':>8s}")
for r in rows:
    n = r["Name"]
    n = re.sub(r"\(.*", "", n) if not n.startswith("void at::") else "torch:" + re.sub(r"<.*", "", n[5:])[:50]
    n = n.replace("void ", "")
    print(f"{n[:60]:60s} {r['Calls']:>7s} {float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f} {float(r['AverageNs'])/1e3:8.2f}")
