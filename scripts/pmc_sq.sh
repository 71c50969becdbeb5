# SQ counters for the extractor kernels (one --pmc pass, no tracing domains)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_sq
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
   --output-format csv -d "$R/gpurun_out/prof_sq" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-timing > gpurun_out/prof_sq.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/prof_sq.log; exit $rc
