"""Per-kernel HBM read traffic from a rocprofv3 `--pmc <counter> --kernel-trace` run.

    python scripts/pmc_bw.py <rocprofv3 output dir> [COUNTER [BYTES_PER_UNIT]] > profiles/pmc_bw_<tag>.txt

COUNTER defaults to FETCH_SIZE with BYTES_PER_UNIT 2048: the counter is KiB per dispatch, and on gfx950 it
reports exactly half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md § HBM: 128-B requests
tallied at 64 B), so it is doubled.  Checked on this code base: the 7B gate_up weight stream (180.4 MB) reads
as 93.2 MiB-units -> 186 MB.  TCC_EA0_RDREQ_sum (L2 -> memory read requests) with BYTES_PER_UNIT 128 is the
raw-counter fallback.

Joins counter_collection.csv (FETCH_SIZE per dispatch, KiB) with kernel_trace.csv (start/end ns) on the
dispatch id and prints, per kernel name: calls, mean duration, mean bytes fetched from HBM/MALL and the
achieved read rate (bytes / kernel time), sorted by total time.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def _one(pattern: str) -> str:
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        sys.exit(f"no file matches {pattern}")
    return hits[0]


def _col(row: dict, *names: str) -> str:
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(f"none of {names} in {sorted(row)}")


def main(root: str, counter: str = "FETCH_SIZE", unit: float = 2048.0) -> None:
    kt = _one(os.path.join(root, "**", "*kernel_trace.csv"))
    cc = _one(os.path.join(root, "**", "*counter_collection.csv"))
    dur = {}
    with open(kt) as f:
        for r in csv.DictReader(f):
            d = _col(r, "Dispatch_Id", "Correlation_Id")
            dur[d] = (_col(r, "Kernel_Name"), int(_col(r, "End_Timestamp")) - int(_col(r, "Start_Timestamp")))
    fetch = defaultdict(float)
    names = {}
    with open(cc) as f:
        for r in csv.DictReader(f):
            if _col(r, "Counter_Name") != counter:
                continue
            d = _col(r, "Dispatch_Id", "Correlation_Id")
            fetch[d] += float(_col(r, "Counter_Value"))
            names[d] = _col(r, "Kernel_Name")
    agg = defaultdict(lambda: [0, 0.0, 0.0])  # calls, ns, KiB
    for d, kib in fetch.items():
        if d in dur:
            name, ns = dur[d]
        else:  # PMC runs serialise dispatches; fall back to the counter row's own name without a time
            name, ns = names[d], 0
        a = agg[name.split("(")[0][:70]]
        a[0] += 1
        a[1] += ns
        a[2] += kib
    print(f"# {kt}\n# {counter} x {unit:g} B per dispatch (bytes the L2 fetched from HBM / Infinity Cache) vs kernel time")
    print(f"{'kernel':72s} {'calls':>7s} {'avg_us':>8s} {'avg_MB':>8s} {'TB/s':>6s}")
    for name, (n, ns, kib) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        us = ns / n / 1e3
        mb = kib * unit / n / 1e6
        tbps = (mb * 1e6) / (us * 1e-6) / 1e12 if us > 0 else float("nan")
        print(f"{name:72s} {n:7d} {us:8.2f} {mb:8.2f} {tbps:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *(float(a) for a in sys.argv[3:4]))
