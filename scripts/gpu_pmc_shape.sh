#!/bin/bash
# PMC traffic of one bench workload shape: separate FETCH_SIZE and WRITE_SIZE passes (never combined
# with trace domains), summarised with the shape recorded, written to profiles/pmc/<TAG>.json so
# bench.py quotes `roofline.traffic` for exactly this shape (on the box; the copy that comes back is
# gpurun_out/pmc_<TAG>/summary.json -> commit it as profiles/pmc/<TAG>.json).
# usage (from gpurun): bash scripts/gpu_pmc_shape.sh TAG [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O $R/profiles/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-host-path "$@" > $O/bench_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-host-path "$@" > $O/bench_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
cd $R
python scripts/pmc_summary.py $O $O/bench_fetch.json > $O/summary.json && cp $O/summary.json profiles/pmc/$TAG.json && python -c "
import json; d=json.load(open('$O/summary.json')); print(d['shape']); [print(k, round(v['traffic_bytes_avg']/1e6,1), 'MB') for k,v in d['kernels'].items() if k.startswith('k_')]"
