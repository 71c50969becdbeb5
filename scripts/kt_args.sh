# Kernel traces of the bench step under several argument sets: scripts/kt_args.sh TAG "args A" "args B" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
i=0
for a in "$@"; do
  i=$((i+1))
  O=gpurun_out/${TAG}_$i; rm -rf $O
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O" -o run -- \
      python3 $R/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-timing --host-api-frames 0 --no-c3 $a > $O.log 2>&1 \
    || { echo "kt [$a] failed"; tail -5 $O.log; exit 1; }
  echo "== [$a]"; python3 scripts/kt_timeline.py $O/run_kernel_trace.csv | head -30
done
