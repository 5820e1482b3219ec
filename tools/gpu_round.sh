#!/bin/bash
# One GPU-box session, the driver's way (no build on the box: the in-tree .so files travel):
# GPU tests, smoke, 1-GPU bench, xGMI probe + counters, rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
# The driver's launcher path (torchrun's agent store carries the agent's artifacts to the ranks).
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_torchrun.log 2>&1 || { tail -20 gpurun_out/bench_torchrun.log; exit 1; }
grep '^{' gpurun_out/bench_torchrun.log | tail -1 | head -c 600; echo
timeout -k 10 300 network_operator_amd/_lib/netop-xgmi-probe --bytes=268435456 --iters=10 > gpurun_out/xgmi_probe.json 2>&1 || { cat gpurun_out/xgmi_probe.json; exit 1; }
cat gpurun_out/xgmi_probe.json
timeout -k 10 120 network_operator_amd/_lib/netop-xgmi-counters > gpurun_out/xgmi_counters.json 2>&1 && head -c 1500 gpurun_out/xgmi_counters.json && echo
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
echo PROF OK
find $GRAFT_REPO_ROOT/gpurun_out/prof -name '*stats*'
# The default-route refusal on the box's own kernel (unprivileged dry runs).
cd $GRAFT_REPO_ROOT && bash tools/gpu_uplink.sh && tail -2 gpurun_out/box_uplink.log
