# round 6: the GPU side's wait inside level-ip's stack (16K-frame RX bursts,
# replies held, threshold 0): the default piece policy against spinning
# waits, no direct pieces, and one whole piece; each call traced
cd $GRAFT_REPO_ROOT || exit 1
O='{"time": [16384], "kinds": "ok", "seed": 3, "hold": 1}'
for k in 1 2; do
  for V in default BLOCK_MIN=0 DIRECT_MAX=0 FIRST_PIECE=67108864; do
    E=""; [ $V != default ] && E="LVLIP_$V"
    echo "== $V" >> gpurun_out/wait_ab.log
    env $E LVLIP_CPU_MAX=0 LVLIP_FRAME_TRACE=1 timeout -k 10 200 python tests/ref_scale_child.py gpurun_out/wab.json oracle/_ref/libref_rxtxq.so batched "$O" 2>&1 | grep "mode 0 n 16384" >> gpurun_out/wait_ab.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/wab.json'))['time']['16384']; print('wall_us_per_frame', d['wall_us_per_frame'])" >> gpurun_out/wait_ab.log
  done
done
