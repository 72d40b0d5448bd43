set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 8 512; do timeout -k 10 200 python tools/op_latency_probe.py frozen_n_262144_k_131072 --batch $b --out gpurun_out/probe_c5_b$b.json; done
timeout -k 10 200 python tools/op_latency_probe.py frozen_n_65536_k_32768 --batch 4096 --out gpurun_out/probe_c3_b4096.json
