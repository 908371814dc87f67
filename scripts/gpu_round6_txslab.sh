# round 6: the TX slab tests, then the composition timing twice more
cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ref_tx_batch.py > gpurun_out/txslab_tests.log 2>&1 || exit 1
for k in 1 2 3; do
  timeout -k 10 400 python scripts/compose_timing.py > gpurun_out/r06_compose_d$k.json 2> gpurun_out/compose_d$k.log || exit 1
done
