#!/bin/bash
# The n-way bf16 sum's tuning sweep on one GPU (local HBM), 256 MiB per buffer.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 network_operator_amd/_lib/netop-sum-tune 256 10 > gpurun_out/sum_tune.jsonl 2> gpurun_out/sum_tune.err || { tail -5 gpurun_out/sum_tune.err; exit 1; }
wc -l gpurun_out/sum_tune.jsonl
