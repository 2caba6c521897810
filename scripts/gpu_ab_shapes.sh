set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06g_abs; mkdir -p $O; cd $R
for F in 500000 250000 125000; do
  for V in base single7 single6; do
    L=""; [ $V != base ] && L=$R/_variants/lib_$V.so
    SENTINEL_LIB=$L timeout -k 10 180 python -u bench.py --flows $F --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/${V}_$F.json 2> $O/${V}_$F.err || { tail -5 $O/${V}_$F.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${V}_$F.json')); print($F, '$V', round(d['value']/1e9,2), d['p99_batch_ms'], d['kernels'].get('part_fused'), d.get('parity_mismatches'))"
  done
done
