# kernel trace of the bench with every stage on one stream (ORBX_PIPELINE=0): per-kernel serial durations and the
# idle gaps between consecutive kernels of a step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-kts}; shift
O=gpurun_out/$TAG; rm -rf $O
ORBX_PIPELINE=0 timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$R/$O" -o run -- \
    python3 $R/bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd --host-fed-steps 0 --steps 10 "$@" > $O.log 2>&1 || { echo "kt failed"; tail -5 $O.log; exit 1; }
python3 - "$O/run_kernel_trace.csv" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].split("::")[-1]
    g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
    d[(n, g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = 0
for (n, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(f"{n:34s} grid {g:9d} n {len(v):4d} avg {sum(v) / len(v) / 1e3:8.1f} us")
# last 5 steps: busy vs wall
t0, t1 = int(rows[len(rows) // 2]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
busy, last = 0, t0
for r in rows[len(rows) // 2:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    s = max(s, last)
    if e > s: busy += e - s; last = e
print(f"second half: wall {(t1 - t0) / 1e6:.3f} ms, kernel-busy {busy / 1e6:.3f} ms")
PY
