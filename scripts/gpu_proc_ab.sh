# Config 4 (and 2): per-key process kernel variants by env (SENTINEL_PROCESS = reg (default) / group / thread).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/proc_ab
mkdir -p $O
for C in 4 2; do
  for P in reg group thread; do
    SENTINEL_PROCESS=$P timeout -k 10 240 python -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > $O/b_${C}_$P.json 2> $O/b_${C}_$P.err || { tail -20 $O/b_${C}_$P.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${C}_$P.json'));print('$C $P', round(d['value']/1e9,3), d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
  done
done
echo AB OK
