set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 30"
for k in 1 3 1 3; do
  timeout -k 10 300 python -u bench.py $B --input-sets $k > gpurun_out/r3o_k$k.log 2>&1 || exit $?
  echo "sets $k: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r3o_k$k.log | tr '\n' ' ')"
done
