set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_cd.py tests/test_bench_contract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r3f_pytest.log; [ $rc -eq 0 ] || exit $rc
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP=$OMP_NUM_THREADS"
timeout -k 10 400 python -u bench.py > gpurun_out/r3f_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 4000 gpurun_out/r3f_bench.log; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_r3.sh r3f_prof
