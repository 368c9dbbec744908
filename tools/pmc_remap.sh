cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing"
for v in 0 1; do
GTFV3_REMAP_SCRATCH=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/pmcm_a$v -o run -- $B > /dev/null 2>&1 || exit 1
GTFV3_REMAP_SCRATCH=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcm_f$v -o run -- $B > /dev/null 2>&1 || exit 1
done
