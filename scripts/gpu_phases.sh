# Per-workgroup phase stamps of k_part_half (diagnostic build) at the 1M and 125k flow shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-phases}
O=gpurun_out/$TAG
mkdir -p $O
for F in 1000000 125000; do
  SENTINEL_LIB=$GRAFT_REPO_ROOT/sentinel_amd/libsentinel_diag.so DIAG_FLOWS=$F timeout -k 10 120 python -u scripts/diag_phases.py > $O/phases_$F.txt 2>&1 || { tail -5 $O/phases_$F.txt; exit 1; }
  echo "F=$F"; grep -v amdgpu.ids $O/phases_$F.txt
done
