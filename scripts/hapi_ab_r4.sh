# Host-API A/B in one GPU call: the native per-call bench under several environments (bash scripts/hapi_ab_r4.sh TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4hab}
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 120 build/host_api_bench multiagent_orb_slam2_amd/liborbx.so 300 > gpurun_out/${T}_$n.log 2>&1 || return $?
  echo "$n: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['frames_per_s'], d['frame_ms'], d['extract_left_ms'], d['extract_right_ms'], d['stereo_ms'])" gpurun_out/${T}_$n.log)"
}
for rep in ${REPS:-1 2}; do
  run graph$rep ORBX_NONE=1 || exit $?
  run nopc$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit $?
  run nograph$rep ORBX_HOST_GRAPH=0 || exit $?
done
