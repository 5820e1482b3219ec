#!/bin/bash
# The driver's 1-GPU bench line, as the driver runs it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_line.json')); print(json.dumps(d['node_ready_gpu_side'])[:1500])"
