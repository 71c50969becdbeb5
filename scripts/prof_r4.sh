# Profile of the bench's timed command (round 4: the bench steps only -- --alone-reps 0 and every side block off, so the
# trace holds exactly STEPS steps and launches_per_step is exact): kernel trace + stats (-> kernel_share.json: the dominant kernel),
# FETCH_SIZE and WRITE_SIZE passes (-> pmc_traffic.json, per-step HBM bytes per kernel family), two SQ passes
# (-> sq_summary.json, VALU per step).  One --pmc pass per counter set, nothing else traced in a PMC pass.
# usage: bash scripts/prof_r4.sh TAG [bench args]; outputs under gpurun_out/TAG/ (copy the summaries to profiles/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-prof}; shift
ARGS=${*:-""}
CFG=kitti; ROWS=375; COLS=1242
case "$ARGS" in *euroc*) CFG=euroc; ROWS=480; COLS=752;; esac
B="python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --alone-reps 0 $ARGS"
STEPS=28   # 3 store-fill steps + 5 warmup + 20 timed, every one the same kernels
IMG=${IMG:-512}   # images per extractor launch: 2 x bench --batch (default 256)
O=gpurun_out/$TAG
rm -rf $O; mkdir -p $O
run() { local name=$1; shift; timeout -s KILL 240 rocprofv3 "$@" --output-format csv -d "$R/$O/$name" -o run -- $B \
          > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }; echo "$name ok"; }
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sqa --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
run sqb --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
python3 scripts/kernel_share.py $O/kt/run_kernel_trace.csv $TAG $STEPS --config $CFG --batch-images $IMG --out $O/kernel_share.json || exit 1
DOM=$(python3 -c "import json; print(json.load(open('$O/kernel_share.json'))['dominant'].split('<')[0])") || exit 1
python3 scripts/pmc_summary.py $O $TAG $IMG $ROWS $COLS $DOM $STEPS $O || exit 1
python3 scripts/sq_summary.py $O $O/sq_summary.json $CFG $IMG $STEPS || exit 1
cp $O/kt/run_kernel_stats.csv $O/${TAG}_kernel_stats.csv
grep -o '"stage_ms_per_step": {[^}]*}' $O/kt.log > $O/live_stages_under_rocprof.txt || true
