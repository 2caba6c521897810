# k_pp_cm_block cost diagnostics (SENTINEL_CM_DIAG bits: 1 no window reads, 2 no walk, 4 no block load/store, 8 no key list)
# The variable changes results, so only a -DSENTINEL_DIAG_CM_ENV build reads it: build one on the CPU side first
#   python -c "from sentinel_amd import build as B; B.build(defines=['SENTINEL_DIAG_CM_ENV'])"
# and rebuild the release library (B.build(force=True)) afterwards.
mkdir -p gpurun_out/cmdiag
for d in ${DIAGS:-0 1 2 3 4 6 7 8}; do
  SENTINEL_CM_DIAG=$d timeout -k 10 200 python -u bench.py --config 4cm --steps 10 --warmup 3 --no-cpu-baseline --latency-batches 10 > gpurun_out/cmdiag/d$d.log 2>&1 || exit 1
done
