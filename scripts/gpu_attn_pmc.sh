#!/bin/bash
# PMC counters of the prefill attention kernel (3B 2k explain case), one counter group per pass.
export TMPDIR=/tmp
O=gpurun_out/apmc
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $O/avail.txt | sort -u > $O/sq_counters.txt || true
export LSA_ATTN_CASES=3b_explain_2k
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/p1 -o run -- python3 scripts/bench_attn_prefill.py > $O/p1.log 2>&1 || { echo "pass1 failed"; tail -n 20 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $O/p2 -o run -- python3 scripts/bench_attn_prefill.py > $O/p2.log 2>&1 || { echo "pass2 failed"; tail -n 20 $O/p2.log; }
for d in p1 p2; do f=$(find $O/$d -name "*counter_collection.csv" | head -1); [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if "attn_prefill32" not in r.get("Kernel_Name", ""): continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(agg): print(k, agg[k] / max(1, n[k]) , "per dispatch (avg over", n[k], ")")
PY
done
find $O -name "*.csv" -size +5M -delete
