# rocprofv3 kernel stats of config 4 (exact param path): every kernel of the timed steps, including
# the slot-table maintenance the bench's per-kernel list does not name.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r02_prof4}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_4.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(r["Name"][:70], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms", round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
