# the first calls of a context, by LVLIP_WARM_BYTES (round 6 diagnosis)
cd $GRAFT_REPO_ROOT || exit 1
for W in 0 4096 1048576 67108864; do
  echo "== LVLIP_WARM_BYTES=$W" >> gpurun_out/first.log
  LVLIP_WARM_BYTES=$W LVLIP_FRAME_TRACE=1 timeout -k 10 120 python scripts/first_call_diag.py >> gpurun_out/first.log 2>&1 || exit 1
done
