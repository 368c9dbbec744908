#!/bin/bash
# SQ / TA PMC passes of the Riemann solver kernels (tools/riem_bench.py), one run per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python3 tools/riem_bench.py --reps 2"
timeout -k 10 120 $B > gpurun_out/riem_bench.log 2>&1 || exit $?
run() { timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmcr_$1 -o run -- $B > gpurun_out/pmcr_$1.log 2>&1 || exit $?; }
run a "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS"
run b "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum"
