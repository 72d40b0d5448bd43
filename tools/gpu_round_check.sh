set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1_pytest.log 2>&1 && echo pytest ok &&
timeout -k 10 300 python -u bench.py > gpurun_out/t1_bench_c2.json 2> gpurun_out/t1_bench_c2.err && echo bench c2 ok &&
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/t1_bench_c3.json 2> gpurun_out/t1_bench_c3.err && echo c3 ok &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/t1_bench_c5.json 2> gpurun_out/t1_bench_c5.err && echo c5 ok
