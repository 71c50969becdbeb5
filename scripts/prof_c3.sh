# C3 all-pairs kernels (k_bf_tile + k_bf_merge): kernel trace + one SQ pass over a short bench run that includes the C3
# block (one step of the front end, then 2000x2000 single and 64-problem batched launches).  Outputs gpurun_out/TAG.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-c3prof}
B="python3 $R/bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-timing --host-api-frames 0"
O=gpurun_out/$TAG; rm -rf $O; mkdir -p $O
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt" -o run -- $B > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
echo kt ok
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d "$R/$O/sq" -o run -- $B > $O/sq.log 2>&1 || { echo "sq failed"; tail -5 $O/sq.log; exit 1; }
echo sq ok
