set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --rank-proxy 8 --no-cpu-baseline > gpurun_out/r06i_proxy8_bench.json
timeout -k 10 300 python3 bench.py --moist --no-cpu-baseline > gpurun_out/r06i_aquaplanet_bench.json
timeout -k 10 400 python3 bench.py --npx 361 --no-cpu-baseline --steps 5 --kernel-report gpurun_out/r06i_c360l72_kernel_events.json > gpurun_out/r06i_c360l72_bench.json
