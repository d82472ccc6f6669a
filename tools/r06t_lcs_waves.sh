# round 6: LCS sweep pace vs sweeping waves a workgroup (GX_LCS_WAVES) and workgroups (GX_LCS_WGS)
mkdir -p gpurun_out
for cfg in "5 2" "4 3" "4 4" "2 5" "2 8" "1 10" "1 16"; do
  set -- $cfg
  echo "waves=$1 wgs=$2"
  GX_LCS_WAVES=$1 GX_LCS_WGS=$2 timeout -k 10 120 python3 tools/lcs_trace.py || exit 1
done > gpurun_out/r06t_waves.log 2>&1
