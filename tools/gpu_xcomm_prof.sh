#!/bin/bash
# rocprofv3 kernel stats of the multi-process xGMI all-reduce: two rank processes on the one
# GPU of the box, each under its own profiler (no launcher in between), 256 MiB, both algorithms.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29655 WORLD_SIZE=2 PYTHONPATH=$R
cd /tmp
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_xcomm_r$r -o xcomm \
    --output-format csv -- python3 -m network_operator_amd.parallel.xgmi_comm --worker --bytes 268435456 \
    --min-bytes 268435456 --iters 10 --warmup 2 --devices 0,0 --timeout 100 > $R/gpurun_out/xcomm_prof_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
grep -h '^{' $R/gpurun_out/xcomm_prof_r0.log || tail -20 $R/gpurun_out/xcomm_prof_r0.log
[ $rc -eq 0 ] || { tail -20 $R/gpurun_out/xcomm_prof_r1.log; exit $rc; }
find $R/gpurun_out/prof_xcomm_r0 -name '*kernel_stats.csv' -exec cut -c1-220 {} \;
