# A/B of bench arguments (one short bench run each, no CPU baseline).  usage: bash scripts/ab_args.sh TAG "ARGS1" "ARGS2" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --host-api-frames 0 --no-c3 $a \
      > gpurun_out/${TAG}_arg$i.log 2>&1 || { echo "run $i ($a) failed"; tail -5 gpurun_out/${TAG}_arg$i.log; exit 1; }
  python3 - "$a" gpurun_out/${TAG}_arg$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"{sys.argv[1]:40s} {d['value']:9.0f} fps {d['ms_per_step']:.3f} ms/step host {d['host_enqueue_ms_per_step']:.3f} " +
      " ".join(f"{k}={v:.3f}" for k, v in d.get("stage_ms_per_step", {}).items()))
PY
done
