#!/bin/bash
# Round-6 end-of-round evidence, part B: rocprofv3 --kernel-trace --stats of config 3 and the memory-side
# request counters by size (scripts/gpu_pmc_req.sh: two separate --pmc passes) of configs 3, 5conc, 2 and 5.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash scripts/gpu_run.sh r06_final_b prof=3 prof=5conc || exit 1
for c in 3 5conc 2 5; do
  bash scripts/gpu_pmc_req.sh r06_final_c$c python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-host-path > gpurun_out/r06_final_b/pmc_$c.log 2>&1 || { tail -20 gpurun_out/r06_final_b/pmc_$c.log; exit 1; }
  rm -rf gpurun_out/pmcreq_r06_final_c$c/rd gpurun_out/pmcreq_r06_final_c$c/wr
done
echo "B OK"
