set -x
nproc; free -g; df -h . /tmp /dev/shm; echo TMPDIR=$TMPDIR; pwd
timeout -k 10 300 python -c "
import torch,time
t=time.time(); print(torch.cuda.is_available(), torch.cuda.device_count(), torch.cuda.get_device_name(0)); 
p=torch.cuda.get_device_properties(0); print(p); print('mem', torch.cuda.mem_get_info())
x=torch.randn(1<<28, device='cuda'); torch.cuda.synchronize()
s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
for _ in range(3):
  s.record(); y=x*2; e.record(); torch.cuda.synchronize(); print('copy GB/s', 2*x.numel()*4/s.elapsed_time(e)/1e6)
import torch.distributed as dist; print('nccl', dist.is_nccl_available())
"
