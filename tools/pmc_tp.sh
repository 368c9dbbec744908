#!/bin/bash
# SQ / TA PMC passes of the isolated fv_tp_2d kernel (tools/tp_bench.py), one run per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python3 tools/tp_bench.py --cfgs=-1 --reps 3"
run() { timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmc_$1 -o run -- $B > gpurun_out/pmc_$1.log 2>&1 || exit $?; }
run a "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES"
run b "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVES TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
run c "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_WAVEFRONTS_sum"
