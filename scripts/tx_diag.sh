set -e
cd $GRAFT_REPO_ROOT
echo '[]' > gpurun_out/req.json
for W in 1048576 8388608; do
 for IM in 32768 0; do
  echo "== W=$W inline_max=$IM" >> gpurun_out/txdiag.log
  LVLIP_CPU_MAX=0 LVLIP_FRAME_TRACE=1 LVLIP_INLINE_MAX=$IM timeout -k 10 120 python tests/ref_tx_batch_child.py gpurun_out/req.json gpurun_out/o.json oracle/_ref/libref_txq.so gpu "{\"write_bytes\": $W, \"send_next\": 0, \"time\": true, \"hold\": true}" >> gpurun_out/txdiag.log 2>&1
  python -c "import json; print(json.load(open('gpurun_out/o.json'))['time'])" >> gpurun_out/txdiag.log
 done
done
