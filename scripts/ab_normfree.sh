set -o pipefail
mkdir -p gpurun_out/ab_nf
for rep in 1 2; do
for arm in 0 16; do
  timeout -k 10 300 python bench.py --model llama3.2 --batch 1 --prompt-len 2048 --new-tokens 128 --steps 3 --warmup 1 --no-extras --set fused_norm_max_batch=$arm > gpurun_out/ab_nf/ex_${arm}_$rep.log 2>&1 || exit 3
  tail -1 gpurun_out/ab_nf/ex_${arm}_$rep.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('explain nf=$arm rep $rep', d['value'], d['decode_device_ms_per_step'], d['numerics']['ok'])"
done
for arm in 0 32; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-extras --set fused_norm_max_batch=$arm > gpurun_out/ab_nf/b32_${arm}_$rep.log 2>&1 || exit 4
  tail -1 gpurun_out/ab_nf/b32_${arm}_$rep.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('b32 nf=$arm rep $rep', d['value'], d['decode_device_ms_per_step'], d['numerics']['ok'])"
done
done
