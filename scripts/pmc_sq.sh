# SQ counters for the kernels (one --pmc pass per counter set, no tracing domains).
# PMC="..." overrides the counter list; OUT names the output directory under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
PMC=${PMC:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"}
OUT=${OUT:-prof_sq}
rm -rf gpurun_out/$OUT
timeout -k 10 300 rocprofv3 --pmc $PMC \
   --output-format csv -d "$R/gpurun_out/$OUT" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-timing > gpurun_out/$OUT.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/$OUT.log; exit $rc
