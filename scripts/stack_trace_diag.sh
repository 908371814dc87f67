# round 6: where the GPU side's time goes inside level-ip's stack: RX bursts
# of 4 096 and 16 384 echo requests, replies held, threshold 0, each library
# call's host steps traced (LVLIP_FRAME_TRACE=1); plain skbs, then a slab
cd $GRAFT_REPO_ROOT || exit 1
for lib in libref_rxtxq.so libref_rxtxq_slab.so; do
  slab=0; [ $lib = libref_rxtxq_slab.so ] && slab=1073741824
  echo "== $lib" >> gpurun_out/stack_trace.log
  LVLIP_CPU_MAX=0 LVLIP_FRAME_TRACE=1 timeout -k 10 200 python tests/ref_scale_child.py gpurun_out/st.json oracle/_ref/$lib batched \
    "{\"time\": [4096, 16384], \"kinds\": \"ok\", \"seed\": 3, \"hold\": 1, \"slab\": $slab}" >> gpurun_out/stack_trace.log 2>&1 || exit 1
  python -c "import json; print(json.dumps(json.load(open('gpurun_out/st.json'))['time']))" >> gpurun_out/stack_trace.log
done
