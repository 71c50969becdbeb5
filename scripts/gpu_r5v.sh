# What each stage costs the step (diagnostics: stages left out).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
for a in "" "--diag-skip keyframes" "--no-tracking" "--no-fuse" "--no-tri" "--diag-skip stereo"; do
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd --host-fed-steps 0 --alone-reps 0 $a \
      > gpurun_out/r5v.log 2>&1 || { echo "[$a] failed"; tail -3 gpurun_out/r5v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r5v.log').read().strip().splitlines()[-1]); print('r$r [$a]', d['value'], d['ms_per_step'])"
done; done
