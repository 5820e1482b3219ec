#!/bin/bash
# Exploratory probe of a GPU box: PCI ids, KFD topology, amd-smi, netns capability.
out=gpurun_out/probe
mkdir -p $out
{
echo "== id"; id
echo "== uname"; uname -a
echo "== amdgpu pci"; for d in /sys/bus/pci/drivers/amdgpu/*:*; do echo "$d -> $(readlink -f $d)"; cat $d/vendor $d/device $d/numa_node 2>/dev/null | tr '\n' ' '; echo; done
echo "== class/net"; for n in /sys/class/net/*; do echo "$n -> $(readlink -f $n)"; cat $n/address $n/mtu $n/operstate 2>/dev/null|tr '\n' ' '; echo; readlink -f $n/device/driver 2>/dev/null; done
echo "== infiniband"; ls -la /sys/class/infiniband 2>&1
echo "== kfd nodes"; for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "-- $n"; cat $n/properties 2>&1 | grep -E 'gpu_id|simd_count|location_id|domain|drm_render_minor|vendor_id|device_id|io_links_count|num_xcc|hive_id|unique_id|max_engine|local_mem' ; cat $n/gpu_id 2>/dev/null; for l in $n/io_links/*; do echo "   link $l: $(cat $l/properties 2>/dev/null | tr '\n' ' ')"; done; done
echo "== amd-smi"; timeout 60 amd-smi list 2>&1 | head -40; timeout 60 amd-smi topology 2>&1 | head -60; timeout 60 amd-smi xgmi 2>&1 | head -60; timeout 60 amd-smi static -a 2>&1 | head -80
echo "== rocm-smi"; timeout 60 rocm-smi --showtopo 2>&1 | head -60
echo "== unshare"; unshare -rn sh -c 'echo inside-userns; cat /proc/self/uid_map' 2>&1
python3 - <<'PY' 2>&1
import socket
try:
    s=socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(0x88cc)); print("AF_PACKET ok (no userns)")
except Exception as e: print("AF_PACKET fail", e)
PY
echo "== nproc/mem"; nproc; free -g
echo "== env"; env | grep -E 'HSA|HIP|ROCR|GPU|NCCL|RCCL|OMP|CUDA' | sort
} > $out/probe.txt 2>&1
timeout -k 10 300 python3 -c "
import torch, time, torch.distributed as dist, os
print(torch.__version__, torch.version.hip, torch.cuda.device_count(), torch.cuda.get_device_name(0))
p=torch.cuda.get_device_properties(0); print(p)
os.environ.setdefault('MASTER_ADDR','127.0.0.1'); os.environ.setdefault('MASTER_PORT','29511')
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda:0'))
x=torch.ones(256<<20, dtype=torch.bfloat16, device='cuda')
for i in range(3): dist.all_reduce(x)
torch.cuda.synchronize(); t=time.time()
for i in range(10): dist.all_reduce(x)
torch.cuda.synchronize(); dt=(time.time()-t)/10
print('1-rank allreduce 512MiB: %.3f ms algbw %.1f GB/s'%(dt*1e3, x.numel()*2/dt/1e9))
dist.destroy_process_group()
" >> $out/probe.txt 2>&1
echo done
