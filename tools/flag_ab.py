"""Interleaved A/B of module switches on the bench's main training line (graph replay, 30 x
1024): each arm sets kernels.<FLAG>["on"] values, runs the bench leg in a fresh process, two
rounds.   python tools/flag_ab.py "COLSUM_ONCE=0,DEFER_WGRAD=0" "COLSUM_ONCE=1,DEFER_WGRAD=0" ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = """
import sys
sys.path.insert(0, {root!r})
from ensemble_svs_with_interactions_amd import kernels as K
for kv in {arm!r}.split(","):
    if kv:
        k, v = kv.split("=")
        getattr(K, k)["on"] = bool(int(v))
sys.argv = ["bench.py", "--steps", "20", "--warmup", "3", "--no-cpu-baseline", "--no-synth",
            "--no-sf0", "--no-census", "--no-config2", "--no-shapes", "--no-real-data",
            "--no-transformer"]
import bench
bench.main()
"""
for rep in range(2):
    for arm in sys.argv[1:]:
        out = subprocess.run([sys.executable, "-c", RUN.format(root=ROOT, arm=arm)], cwd=ROOT,
                             capture_output=True, text=True, timeout=400)
        if out.returncode:
            print(out.stderr[-2000:])
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print(f"arm=[{arm}] {d['ms_per_step']:.3f} ms", flush=True)
