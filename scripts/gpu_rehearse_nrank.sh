#!/bin/bash
# Rehearsal of bench.py's N-rank path on a one-GPU box (from gpurun): N ranks on cuda:0 over gloo
# (SENTINEL_BENCH_ONE_DEVICE=1) -- sharding, barriers, max-over-ranks timing and the snapshot
# all-gathers, not RCCL; the numbers are not results (N ranks share one GPU).
# usage: bash scripts/gpu_rehearse_nrank.sh TAG N [CONFIG]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; N=$2; CFG=${3:-3}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
SENTINEL_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --config $CFG --steps 5 --warmup 2 \
  > $O/rehearse_${CFG}_$N.json 2> $O/rehearse_${CFG}_$N.err || { tail -30 $O/rehearse_${CFG}_$N.err; exit 1; }
python scripts/bench_brief.py $O/rehearse_${CFG}_$N.json
