set -e
mkdir -p gpurun_out
timeout -k 10 300 python -c "
import torch,time
t=time.time()
print(torch.cuda.is_available(), torch.cuda.device_count(), torch.cuda.get_device_name(0))
p=torch.cuda.get_device_properties(0); print(p)
print(p.gcnArchName, p.multi_processor_count, p.total_memory/2**30)
a=torch.randn(8192,8192,device='cuda',dtype=torch.bfloat16)
torch.cuda.synchronize()
for _ in range(3): c=a@a
torch.cuda.synchronize(); t=time.time()
for _ in range(10): c=a@a
torch.cuda.synchronize(); dt=(time.time()-t)/10
print('bf16 8k gemm TF', 2*8192**3/dt/1e12)
x=torch.empty(2**30,dtype=torch.uint8,device='cuda'); y=torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); t=time.time()
for _ in range(10): y.copy_(x)
torch.cuda.synchronize(); dt=(time.time()-t)/10
print('copy GB/s', 2*2**30/dt/1e9)
" > gpurun_out/envprobe.txt 2>&1
rocm-smi --showtopo >> gpurun_out/envprobe.txt 2>&1 || true
nproc >> gpurun_out/envprobe.txt
