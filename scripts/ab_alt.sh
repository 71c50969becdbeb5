# Alternating A/B of library builds on the default bench (no CPU / C3 / host-API / CD / host-fed legs; the serial
# roofline_alone block kept): each lib runs ROUNDS times in the order A B A B ..., so box drift hits both alike.
# usage: ROUNDS=2 bash scripts/ab_alt.sh TAG product build/x/liborbx.so ...   (AB_ENV="A=1" for every run)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
TAG=$1; shift
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    L=""; [ "$lib" != product ] && L="ORBX_LIB=$lib"
    log=gpurun_out/${TAG}_${i}_r$r.log
    env $L $AB_ENV timeout -k 10 200 python bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd --host-fed-steps 0 \
        $AB_ARGS > $log 2>&1 || { echo "[$lib] failed"; tail -3 $log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
a=d.get('roofline_alone',{}).get('stage_ms_alone',{})
print('r$r [$lib]', d['value'], d['ms_per_step'], 'alone', {k: round(v, 3) for k, v in a.items()})"
  done
done
