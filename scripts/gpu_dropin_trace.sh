#!/bin/bash
# Kernel + copy trace of the batcher under one synchronous caller: the per-batch kernel chain and
# the idle gaps (small-batch latency budget).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/dtrace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/dtrace/prof -o run -- $R/tools/dropin_bench --mode sync --threads ${THREADS:-1} --seconds 1 > $R/gpurun_out/dtrace/out.json 2> $R/gpurun_out/dtrace/prof.err || { tail -5 $R/gpurun_out/dtrace/prof.err; exit 1; }
cd $R
cat gpurun_out/dtrace/out.json
python scripts/trace_gaps.py gpurun_out/dtrace/prof/run_kernel_trace.csv 40
