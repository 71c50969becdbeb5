# Kernel trace + stats of the bench step exactly as the driver's bench measures it (per-stage HIP-event timing on),
# without the CPU / C3 / host-API legs (their kernels would mix into the per-kernel averages): scripts/kt_bench.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-ktb}; shift
O=gpurun_out/$TAG; rm -rf $O
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O" -o run -- \
    python3 $R/bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 "$@" > $O.log 2>&1 || { echo "kt failed"; tail -5 $O.log; exit 1; }
tail -1 $O.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms_per_launch'])"
python3 - "$O/run_kernel_trace.csv" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].split("::")[-1]
    g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
    d[(n, g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for (n, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:30]:
    print(f"{n:26s} grid {g:9d} n {len(v):4d} avg {sum(v) / len(v) / 1e3:8.1f} us")
PY
