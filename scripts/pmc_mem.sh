# Memory-pipe counters per kernel (two --pmc passes, no tracing domains): SQ issue/wait split, TA busy,
# TD busy, L1 (TCP) accesses and L1->L2 read requests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_mem1 gpurun_out/prof_mem2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
   --output-format csv -d "$R/gpurun_out/prof_mem1" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-timing > gpurun_out/prof_mem1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum \
   --output-format csv -d "$R/gpurun_out/prof_mem2" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-timing > gpurun_out/prof_mem2.log 2>&1 || exit $?
echo done
