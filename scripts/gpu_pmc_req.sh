#!/bin/bash
# Memory-side request counters of one command, by request size (round 5): two separate rocprofv3 --pmc
# passes (4 TCC counters each at most; never combined with trace domains), summarised by
# scripts/pmc_summary.py --req into gpurun_out/pmcreq_<TAG>/summary.json (commit it under profiles/pmc/).
#   read pass:  TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
#   write pass: TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_BUBBLE_sum
# usage (from gpurun): bash scripts/gpu_pmc_req.sh TAG <program> [args...]
#   e.g. bash scripts/gpu_pmc_req.sh calib tools/pmc_calib
#        bash scripts/gpu_pmc_req.sh c3 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-host-path
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/pmcreq_$TAG
mkdir -p $O
P=$1; shift
case $P in
  python|python3) P=$(command -v python3); S=$1; shift; case $S in /*) ;; *) S=$R/$S ;; esac; set -- "$S" "$@" ;;
  /*) ;;
  *) P=$R/$P ;;
esac
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
  --output-format csv -d $O/rd -o run -- $P "$@" > $O/rd.out 2> $O/rd.err || { tail -20 $O/rd.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_BUBBLE_sum \
  --output-format csv -d $O/wr -o run -- $P "$@" > $O/wr.out 2> $O/wr.err || { tail -20 $O/wr.err; exit 1; }
cd $R
python scripts/pmc_summary.py --req $O $O/rd.out > $O/summary.json && python - <<PY
import json
d = json.load(open("$O/summary.json"))
for k, v in d["kernels"].items():
    print(f"{k[:40]:40s} disp {v['dispatches']:3d}  read {v['read_bytes_avg']/1e6:9.2f} MB  write {v['write_bytes_avg']/1e6:9.2f} MB  "
          f"rd32/64/128 {v['rdreq_32b_avg']:.3g}/{v['rdreq_64b_avg']:.3g}/{v['rdreq_128b_avg']:.3g} rdreq {v['rdreq_avg']:.3g} "
          f"wr {v['wrreq_avg']:.3g} wr64 {v['wrreq_64b_avg']:.3g} bubble {v['bubble_avg']:.3g}")
PY
