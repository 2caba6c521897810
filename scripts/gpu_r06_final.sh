#!/bin/bash
# Round-6 end-of-round evidence, part A: GPU suite, smoke and every config's bench line (gpurun_out/r06_final).
# Part B (scripts/gpu_r06_final_b.sh): rocprofv3 kernel stats of config 3 and request-size PMC of the shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_run.sh r06_final tests smoke bench=3 bench=2 bench=5 bench=5conc bench=4 bench=4cm bench=3lim
