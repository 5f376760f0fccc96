#!/bin/bash
# Build alternative copies of the gfx950 extension for A/B experiments on the GPU box:
#   scripts/build_variants.sh name1="-DFOO=1" name2="-DFOO=2" ...
# each lands in variants/<name>.so (top level: ./build is gpurun-ignored) (load it with LSA_HIP_SO=...); the in-tree default build is
# restored at the end.  "head=" builds the committed HEAD sources (git worktree under build/).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants variants
for spec in "$@"; do
  name="${spec%%=*}"; flags="${spec#*=}"
  if [ "$name" = head ]; then
    rm -rf build/head_wt; git worktree prune
    git worktree add -f --detach build/head_wt HEAD > /dev/null
    (cd build/head_wt && LSA_HIP_EXTRA="$flags" python -m llm_based_apache_spark_optimization_amd.ops.build > /dev/null)
    cp build/head_wt/llm_based_apache_spark_optimization_amd/ops/_lsa_hip.so variants/head.so
    git worktree remove --force build/head_wt
  else
    LSA_HIP_EXTRA="$flags" python -m llm_based_apache_spark_optimization_amd.ops.build > /dev/null
    cp llm_based_apache_spark_optimization_amd/ops/_lsa_hip.so "variants/$name.so"
  fi
  echo "built variants/$name.so"
done
python -m llm_based_apache_spark_optimization_amd.ops.build > /dev/null
