# Round profile of the default bench step: kernel trace + stats, FETCH_SIZE pass, WRITE_SIZE pass, two SQ passes.
# One --pmc pass per counter set, nothing else traced in a PMC pass.  Outputs under gpurun_out/TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-prof}; shift
ARGS=${*:-""}
B="python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-timing --host-api-frames 0 --no-c3 $ARGS"
O=gpurun_out/$TAG
rm -rf $O; mkdir -p $O
run() { local name=$1; shift; timeout -s KILL 240 rocprofv3 "$@" --output-format csv -d "$R/$O/$name" -o run -- $B \
          > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }; echo "$name ok"; }
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sqa --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
run sqb --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
