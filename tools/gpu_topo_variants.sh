#!/bin/bash
# RCCL's handling of the generated NCCL_TOPO_FILE and of variants, on the real box:
#   file     - as the agent writes it
#   xgmi     - plus <gpu><xgmi target=peer/></gpu> for the 7 peers outside the job (why the
#              agent leaves xGMI links to RCCL)
#   rocm     - the same file through /opt/rocm's RCCL (native netop-rccl-bench)
set -o pipefail
mkdir -p gpurun_out/topo_variants
export TMPDIR=/tmp
O=gpurun_out/topo_variants
python3 -c 'import network_operator_amd.agent as a; open("'$O'/file.xml","w").write(a.native().rccl_topo_xml("/sys/"))' || exit 1
python3 - <<'PY' || exit 1
import re, network_operator_amd.agent as a
x = open("gpurun_out/topo_variants/file.xml").read()
n = a.native()
xg = n.read_xgmi("/sys/")
gpus = xg["gpus"]
out = x
for g in gpus:
    peers = "".join(f'<xgmi target="{p}" count="1" tclass="0x120000"/>' for p in gpus if p != g)
    out = re.sub(rf'(<pci busid="{g}"[^>]*)/>', rf'\1><gpu>{peers}</gpu></pci>', out)
open("gpurun_out/topo_variants/xgmi.xml", "w").write(out)
PY
cat > /tmp/init.py <<'PY'
import torch, torch.distributed as dist
d = torch.device("cuda", 0); torch.cuda.set_device(d)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=d)
x = torch.ones(4096, device=d); dist.all_reduce(x); torch.cuda.synchronize()
dist.destroy_process_group(); print("init+allreduce ok")
PY
for v in file xgmi; do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + RANDOM % 300)) NCCL_TOPO_FILE=$PWD/$O/$v.xml NCCL_TOPO_DUMP_FILE=$PWD/$O/dump_$v.xml \
    NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,GRAPH \
    timeout -k 10 120 python3 /tmp/init.py > $O/$v.log 2>&1; rc=$?
  echo "variant $v: rc=$rc"; grep -iE "error|warn|topology file|init\+allreduce" $O/$v.log | head -8
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done
NCCL_TOPO_FILE=$PWD/$O/file.xml NCCL_TOPO_DUMP_FILE=$PWD/$O/dump_rocm.xml NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT \
  timeout -k 10 120 network_operator_amd/_lib/netop-rccl-bench -o all_reduce -g 1 -b 1048576 -e 1048576 -n 5 -w 2 > $O/rocm.log 2>&1; echo "variant rocm: rc=$?"
grep -iE "version|topology file|error" $O/rocm.log | head -5
head -30 $O/dump_file.xml
