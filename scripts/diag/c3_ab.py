import sys, os, json
sys.path.insert(0, os.getcwd())
import torch, bench
import multiagent_orb_slam2_amd as pkg
print(os.environ.get("ORBX_LIB"), json.dumps({k: v["us_per_launch"] for k, v in bench.c3_bench(pkg, torch.device("cuda", 0)).items() if isinstance(v, dict) and "us_per_launch" in v}))
