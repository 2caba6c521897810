# Quick bench check on one MI355X: the default bench line and the N=8 per-rank shape.
# Usage (from gpurun): bash scripts/gpu_baseline.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-base}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 180 python -u bench.py --flows 125000 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_125k.json 2> $O/bench_125k.err || { tail -20 $O/bench_125k.err; exit 1; }
cat $O/bench_125k.json
