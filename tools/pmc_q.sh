#!/bin/bash
# SQ counters (two separate --pmc passes) of one bench step: instruction mix, wave cycles and
# stall buckets per kernel.  usage: tools/pmc_q.sh TAG [extra bench args]
T=${1:-pmcq}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/${T}_a -o run -- $B > gpurun_out/${T}_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_BUSY_CYCLES --output-format csv -d gpurun_out/${T}_b -o run -- $B > gpurun_out/${T}_b.log 2>&1 || exit 1
