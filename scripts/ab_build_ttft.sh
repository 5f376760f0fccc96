#!/bin/bash
# Cross-build A/B of time to first token (scripts/ttft_knob_ab.py, knob 'none'): the loaded in-tree build vs an
# alternative build of the same extension (LSA_HIP_SO), processes in turns so drift hits both arms alike.
# Usage: scripts/ab_build_ttft.sh <variant.so> [turns] [rounds] [cases]   -> gpurun_out/ab_build_ttft.log
set -e -o pipefail
alt=$1; turns=${2:-3}; rounds=${3:-5}; cases=${4:-0,1,2}
mkdir -p gpurun_out
for i in $(seq "$turns"); do
  LSA_HIP_SO=$alt timeout -k 10 240 python -u scripts/ttft_knob_ab.py none "$rounds" "$cases" | sed "s/^/{\"arm\": \"alt\", \"turn\": $i, \"r\": /; s/$/}/" >> gpurun_out/ab_build_ttft.log
  timeout -k 10 240 python -u scripts/ttft_knob_ab.py none "$rounds" "$cases" | sed "s/^/{\"arm\": \"tree\", \"turn\": $i, \"r\": /; s/$/}/" >> gpurun_out/ab_build_ttft.log
done
