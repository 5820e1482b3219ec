#!/bin/bash
# The n-way bf16 sum kernel's rate on local HBM (the direct all-reduce's reduce step).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/sum_rate_box.py > gpurun_out/sum_rate.json 2> gpurun_out/sum_rate.err || { tail -20 gpurun_out/sum_rate.err; exit 1; }
cat gpurun_out/sum_rate.json
