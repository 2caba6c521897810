#!/bin/bash
# A/B of variant libraries on one bench config (from gpurun): the in-tree build, then each
# _variants/lib_<name>.so through SENTINEL_LIB.  usage: bash scripts/gpu_ab_lib.sh TAG CONFIG NAME [NAME ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; CFG=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/base.json 2> $O/base.err || { tail -5 $O/base.err; exit 1; }
echo "base $(python scripts/bench_brief.py $O/base.json)"
for V in "$@"; do
  SENTINEL_LIB=$R/_variants/lib_$V.so timeout -k 10 300 python -u bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/$V.json 2> $O/$V.err || { tail -5 $O/$V.err; exit 1; }
  echo "$V $(python scripts/bench_brief.py $O/$V.json)"
done
