# Host-API A/B of environment switches in one GPU call (bash scripts/hapi_ab2_r4.sh TAG "VAR=v ..." ...): native
# per-call bench (300 frames) for each whitespace-free switch list, two rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; shift
for rep in 1 2; do
  i=0
  for sw in "$@"; do
    i=$((i+1))
    env $sw timeout -k 10 120 build/host_api_bench multiagent_orb_slam2_amd/liborbx.so 300 > gpurun_out/${T}_${i}_$rep.log 2>&1 || exit $?
    echo "$sw: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['frames_per_s'], d['frame_ms']['median'], d['frame_ms']['p95'], d['extract_left_ms']['median'], d['extract_right_ms']['median'], d['slowest'][0][:2])" gpurun_out/${T}_${i}_$rep.log)"
  done
done
