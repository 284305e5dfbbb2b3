set -o pipefail
mkdir -p gpurun_out/vc1
timeout -k 10 300 python -u -m pytest tests/test_gpu_value_codes.py tests/test_gpu_sell.py -x -q --timeout 120 --timeout-method thread > gpurun_out/vc1/pytest.log 2>&1 || { tail -40 gpurun_out/vc1/pytest.log; exit 1; }
tail -2 gpurun_out/vc1/pytest.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/vc1/bench.log 2>&1 || { tail -20 gpurun_out/vc1/bench.log; exit 1; }
tail -1 gpurun_out/vc1/bench.log
CGX_VALUE_CODES=0 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/vc1/bench_novc.log 2>&1 || { tail -20 gpurun_out/vc1/bench_novc.log; exit 1; }
tail -1 gpurun_out/vc1/bench_novc.log
