# round 6 A/B: the density rule's span ratio (LVLIP_SPAN_RATIO 2 against 3)
# inside level-ip's stack: RX bursts with replies held, skb buffers in a
# registered slab, GPU side; the CPU side beside them; three alternations
cd $GRAFT_REPO_ROOT || exit 1
O='{"time": [4096, 16384, 65536], "kinds": "ok", "seed": 3, "hold": 1, "slab": 1073741824}'
for k in 1 2 3; do
  for R in 2 3; do
    LVLIP_CPU_MAX=0 LVLIP_SPAN_RATIO=$R timeout -k 10 200 python tests/ref_scale_child.py gpurun_out/ab.json oracle/_ref/libref_rxtxq_slab.so batched "$O" || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json'))['time']; print(json.dumps({'ratio': $R, 'side': 'gpu', 'us_per_frame': {n: d[n]['wall_us_per_frame'] for n in d}, 'h2d': {n: d[n]['flush']['h2d_bytes'] for n in d}}))" >> gpurun_out/span_ab.jsonl
  done
  LVLIP_CPU_MAX=1073741824 timeout -k 10 200 python tests/ref_scale_child.py gpurun_out/ab.json oracle/_ref/libref_rxtxq_slab.so batched "$O" || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab.json'))['time']; print(json.dumps({'side': 'cpu', 'us_per_frame': {n: d[n]['wall_us_per_frame'] for n in d}}))" >> gpurun_out/span_ab.jsonl
done
