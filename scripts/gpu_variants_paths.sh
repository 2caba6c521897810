set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/variants
for p in ${PATHS:-auto partition sorted}; do
  SENTINEL_FLOW_PATH=$p timeout -k 10 300 python -u scripts/bench_variants.py > gpurun_out/variants/$p.jsonl 2> gpurun_out/variants/$p.err || { tail -5 gpurun_out/variants/$p.err; exit 1; }
  cat gpurun_out/variants/$p.jsonl
done
