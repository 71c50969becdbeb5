set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/r3k_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"stage_ms_per_step": {[^}]*}' gpurun_out/r3k_bench.log | head -4; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_r3.sh r3k_prof || exit $?
grep -o '"stage_ms_per_step": {[^}]*}' gpurun_out/r3k_prof/kt.log
