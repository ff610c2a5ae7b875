set -o pipefail
mkdir -p gpurun_out/r4tun2
timeout -k 10 200 python -u scripts/bench_tunnel.py > gpurun_out/r4tun2/noloss.json 2> gpurun_out/r4tun2/noloss.err && timeout -k 10 200 python -u scripts/bench_tunnel.py --loss 3 > gpurun_out/r4tun2/loss3.json 2> gpurun_out/r4tun2/loss3.err && cat gpurun_out/r4tun2/*.json
