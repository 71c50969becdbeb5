# Kernel trace + two SQ counter passes over a short bench run (one --pmc pass per counter set, no tracing
# domains).  usage: bash scripts/prof_sq.sh TAG [bench args...]; outputs under gpurun_out/TAG_{kt,sqa,sqb}.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-prof}; shift
ARGS=${*:-"--steps 5 --warmup 2"}
B="python3 $R/bench.py $ARGS --cpu-seconds 0 --no-timing"
rm -rf gpurun_out/${TAG}_kt gpurun_out/${TAG}_sqa gpurun_out/${TAG}_sqb
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_kt" -o run -- $B \
    > gpurun_out/${TAG}_kt.log 2>&1 || { echo "kt failed rc=$?"; tail -5 gpurun_out/${TAG}_kt.log; exit 1; }
echo "kt ok"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$R/gpurun_out/${TAG}_sqa" -o run -- $B \
    > gpurun_out/${TAG}_sqa.log 2>&1 || { echo "sqa failed rc=$?"; tail -5 gpurun_out/${TAG}_sqa.log; exit 1; }
echo "sqa ok"
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY \
    SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv \
    -d "$R/gpurun_out/${TAG}_sqb" -o run -- $B \
    > gpurun_out/${TAG}_sqb.log 2>&1 || { echo "sqb failed rc=$?"; tail -5 gpurun_out/${TAG}_sqb.log; exit 1; }
echo "sqb ok"
find gpurun_out/${TAG}_kt gpurun_out/${TAG}_sqa gpurun_out/${TAG}_sqb -name '*.csv' | head
