#!/bin/bash
# One parametrised GPU session (from gpurun): each step has its own time limit, the chain stops at
# the first failure, results go under gpurun_out/<TAG>/.
# usage: bash scripts/gpu_run.sh TAG STEP [STEP ...]
#   tests[=<pytest selector>]    pytest -m gpu (default: the whole tests/ dir)
#   bench=<config>[,<args>]      bench.py --config <config> --steps 20 --warmup 3 <args, commas -> spaces>
#   prof=<config>[,<args>]       rocprofv3 --kernel-trace --stats of a short bench run of that config
#   pmc=<tag>,<config>[,<args>]  separate FETCH_SIZE / WRITE_SIZE passes -> profiles/pmc/<tag>.json
#   smoke                        __graft_entry__.smoke()
#   stream                       scripts/host_stream_study.py under rocprofv3 kernel + memory-copy trace
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
n=0
for S in "$@"; do
  n=$((n + 1))
  case $S in
    tests*)
      SEL=${S#tests}; SEL=${SEL#=}; SEL=${SEL:-tests}
      echo "== tests $SEL"
      timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_$n.log 2>&1
      rc=$?; tail -3 $O/tests_$n.log
      [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests_$n.log | head -30; exit $rc; } ;;
    smoke)
      echo "== smoke"
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench=*)
      A=${S#bench=}; C=${A%%,*}; X=""; [ "$A" != "$C" ] && X=${A#*,}; X=${X//,/ }
      echo "== bench $C $X"
      timeout -k 10 400 python -u bench.py --config $C --steps 20 --warmup 3 $X > $O/bench_${C}_$n.json 2> $O/bench_${C}_$n.err || { tail -20 $O/bench_${C}_$n.err; exit 1; }
      python scripts/bench_brief.py $O/bench_${C}_$n.json ;;
    prof=*)
      A=${S#prof=}; C=${A%%,*}; X=""; [ "$A" != "$C" ] && X=${A#*,}; X=${X//,/ }
      echo "== rocprof $C $X"
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${C}_$n -o run -- python $R/bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-host-path $X > $O/prof_${C}_$n.json 2> $O/prof_${C}_$n.err ) || { tail -20 $O/prof_${C}_$n.err; exit 1; }
      python scripts/trace_summary.py $O/prof_${C}_$n/run_kernel_trace.csv warmup:2,profile:3,timed:10 > $O/prof_${C}_$n/summary.json 2>/dev/null
      head -c 1500 $O/prof_${C}_$n/run_kernel_stats.csv; echo ;;
    pmc=*)
      A=${S#pmc=}; T=${A%%,*}; B=${A#*,}; C=${B%%,*}; X=""; [ "$B" != "$C" ] && X=${B#*,}; X=${X//,/ }
      echo "== pmc $T ($C $X)"
      bash scripts/gpu_pmc_shape.sh $T --config $C $X || exit 1 ;;
    stream)
      echo "== host stream study"
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/stream_$n -o run -- python $R/scripts/host_stream_study.py > $O/stream_$n.log 2> $O/stream_$n.err ) || { tail -20 $O/stream_$n.err; exit 1; }
      cat $O/stream_$n.log ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "RUN OK"
