set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_monitor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t3_pytest.log 2>&1 && echo tests ok &&
timeout -k 10 120 python -u tools/monitor_run.py frozen_n_65536_k_32768 --batch 4096 --json gpurun_out/t3_mon_c3.json > gpurun_out/t3_mon_c3.txt 2>&1 && echo c3 ok &&
timeout -k 10 120 python -u tools/monitor_run.py frozen_n_262144_k_131072 --batch 512 --json gpurun_out/t3_mon_c5.json > gpurun_out/t3_mon_c5.txt 2>&1 && echo c5 ok &&
timeout -k 10 120 python -u tools/monitor_run.py frozen_n_65536_k_32768 --batch 8 > gpurun_out/t3_mon_c3_b8.txt 2>&1 && echo c3b8 ok
