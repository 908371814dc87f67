# round 6: the GPU suite on the current tree, then the composition timing three times
cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || exit 1
for k in 1 2 3; do
  timeout -k 10 300 python scripts/compose_timing.py > gpurun_out/r06_compose_w$k.json 2> gpurun_out/compose_w$k.log || exit 1
done
