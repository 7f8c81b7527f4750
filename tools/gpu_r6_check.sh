mkdir -p gpurun_out/u6e
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_engine_gpu.py -k "dataflow or fused_hash_rounds" > gpurun_out/u6e/t0.log 2>&1 &&
UTTT_TOWER_DEFER=1 timeout -k 10 150 python -u tools/diag/tower_ab.py gpurun_out/u6e/tower_ab_defer1.json 1370,2740,4096 3 10 > gpurun_out/u6e/ab1.log 2>&1 &&
UTTT_TOWER_DEFER=0 timeout -k 10 150 python -u tools/diag/tower_ab.py gpurun_out/u6e/tower_ab_defer0.json 1370,2740,4096 3 10 > gpurun_out/u6e/ab0.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/u6e/bench.log 2>&1 &&
UTTT_NN_TOWER=layers UTTT_ROUND_DISPATCHES=3 timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/u6e/bench_old.log 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_engine_gpu.py tests/test_dropins_gpu.py > gpurun_out/u6e/t.log 2>&1
