# Kernel trace of the bench step, pipelined (default) and serial (ORBX_PIPELINE=0: isolated kernel durations).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-kt}; shift
B="python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-timing --host-api-frames 0 --no-c3 $*"
for mode in 1 0; do
  O=gpurun_out/${TAG}_p$mode; rm -rf $O
  ORBX_PIPELINE=$mode timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O" -o run -- $B > $O.log 2>&1 \
    || { echo "kt p$mode failed"; tail -5 $O.log; exit 1; }
  echo "== pipeline=$mode"; python3 scripts/kt_split.py $O/run_kernel_trace.csv 16
done
