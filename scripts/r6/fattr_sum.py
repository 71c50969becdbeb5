"""k_fast_wave SQ counters per build of scripts/r6/fattr.sh (per dispatch, averaged over the pass's dispatches)."""
import collections
import csv
import glob
import json
import sys

base = sys.argv[1]
res = {}
for v in ("product", "fattr1", "fattr2", "fattr3"):
    f = glob.glob(f"{base}/{v}/**/run_counter_collection.csv", recursive=True) or glob.glob(f"{base}/{v}*counter_collection.csv")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "", 1).replace("orbx::", "")
        if not k.startswith("k_fast_wave"):
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    out = {}
    for k, d in agg.items():
        c = {m: d[m] / n[(k, m)] for m in d}
        c["conflict_per_lds_inst"] = round(c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_INSTS_LDS"], 1), 3)
        c["lds_inst_per_wave"] = round(c["SQ_INSTS_LDS"] / max(c["SQ_WAVES"], 1), 1)
        c["conflict_cycles_per_wave"] = round(c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_WAVES"], 1), 1)
        out[k] = {m: round(x, 3) for m, x in c.items()}
    res[v] = out
    for k, c in sorted(out.items()):
        print(v, k, "conf/lds", c["conflict_per_lds_inst"], "lds/wave", c["lds_inst_per_wave"], "conf cyc/wave",
              c["conflict_cycles_per_wave"], "waves", c["SQ_WAVES"])
json.dump(res, open(f"{base}/fattr_summary.json", "w"), indent=1)
