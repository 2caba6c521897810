# SQ / TCC counter passes over a short bench run (one pass per counter group, each time-limited).
# Usage (from gpurun): bash scripts/gpu_pmc_sq.sh TAG   -> gpurun_out/TAG/sq{1,2,3}
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sq}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P3="SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/sq$i -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} > /dev/null 2> $O/sq$i.err || { tail -5 $O/sq$i.err; exit 1; }
done
cd $R && python scripts/pmc_sq_summary.py $O && rm -rf $O/sq1 $O/sq2 $O/sq3
