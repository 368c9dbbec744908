#!/bin/bash
# Round profile on the gpurun box: bench line, rocprofv3 kernel stats, and the two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for per-kernel HBM traffic.
#   usage: tools/profile_round.sh rNN [extra bench args]
R=${1:?round tag}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
# the traced runs use one stream so every launch of a kernel runs unoverlapped, as in the
# bench's roofline pass (the bench line itself times the default three streams)
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --streams 1 $*"
exec_steps=(
  "bench:300:python3 bench.py --kernel-report gpurun_out/${R}_kernels.json $* > gpurun_out/${R}_bench.json"
  "ktrace:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_kt -o run -- $B"
  "pmc_fetch:500:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${R}_pmc_f -o run -- $B"
  "pmc_write:500:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${R}_pmc_w -o run -- $B"
)
bash tools/gpu_steps.sh "${exec_steps[@]}"
