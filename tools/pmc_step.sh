#!/bin/bash
# Occupancy / issue PMC passes of the whole C180 L72 step (single stream), one run per pass,
# plus a kernel trace (VGPR / LDS per kernel).  tools/pmc_step_summary.py reduces them.
#   usage: tools/pmc_step.sh TAG [extra bench args]
R=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --streams 1 $*"
run() { timeout -s KILL 240 rocprofv3 $2 --output-format csv -d gpurun_out/${R}_$1 -o run -- $B > gpurun_out/${R}_$1.log 2>&1 || exit $?; }
run kt "--kernel-trace --stats"
run sqa "--pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_WAVES"
run sqb "--pmc SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"
run tcc "--pmc TCC_HIT_sum TCC_MISS_sum"
run fetch "--pmc FETCH_SIZE"
run write "--pmc WRITE_SIZE"
