cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_dispatch_gpu.py tests/test_skb_gpu.py tests/test_skb_list.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6_t1.log 2>&1 && \
timeout -k 10 500 python -u bench.py --crossover --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6_cross.json 2> gpurun_out/r6_cross.log
