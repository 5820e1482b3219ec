#!/bin/bash
# What RCCL itself sees on the box: topology dump (NCCL_TOPO_DUMP_FILE) after a 1-rank init,
# with INIT/NET/GRAPH logging, so the generated NCCL_TOPO_FILE can match its XML dialect.
set -o pipefail
mkdir -p gpurun_out/topo
export TMPDIR=/tmp
cat > /tmp/dump.py <<'PY'
import os, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29561")
d = torch.device("cuda", 0); torch.cuda.set_device(d)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=d)
x = torch.ones(1024, device=d); dist.all_reduce(x); torch.cuda.synchronize()
dist.destroy_process_group(); print("ok", x[0].item())
PY
NCCL_TOPO_DUMP_FILE=$PWD/gpurun_out/topo/rccl_auto.xml NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,NET,GRAPH \
  timeout -k 10 120 python3 /tmp/dump.py > gpurun_out/topo/auto.log 2>&1 || { tail -30 gpurun_out/topo/auto.log; exit 1; }
tail -3 gpurun_out/topo/auto.log
ls /dev/infiniband 2>&1 | head -3
ls /sys/class/infiniband 2>&1 | head -10
for n in /sys/class/net/*; do echo "$(basename $n) $(readlink -f $n/device 2>/dev/null)"; done > gpurun_out/topo/netdevs.txt
for d in /sys/bus/pci/drivers/amdgpu/0000*; do b=$(basename $d); echo "$b $(cat $d/class) $(cat $d/max_link_speed) $(cat $d/max_link_width) $(readlink -f $d)"; done > gpurun_out/topo/gpus.txt
python3 -c 'import network_operator_amd.agent as a, json; print(json.dumps(a.native().discover("/sys/"), indent=1))' > gpurun_out/topo/discover.json 2>&1
head -c 4000 gpurun_out/topo/rccl_auto.xml
