"""Interleaved A/B of module switches on the bench's main training line (graph replay, 30 x
1024): each arm sets kernels.<FLAG>["on"] values or calls C-ABI switches (ensvs_*=value), runs
the bench leg in a fresh process, two rounds.
  python tools/flag_ab.py [--sf0] "COLSUM_ONCE=0,DEFER_WGRAD=0" "ensvs_ardec_coop_set_tile_seqs=32" \
      "diffsinger.SKIP_GEMM=0" "ensvs_set_p8=1" ...
--sf0: time the recipe-default SeparateF0 leg instead (its ms_per_step); --tf: the tier-2
Transformer leg."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = """
import sys
sys.path.insert(0, {root!r})
from ensemble_svs_with_interactions_amd import kernels as K
from ensemble_svs_with_interactions_amd._lib import call
for kv in {arm!r}.split(","):
    if kv:
        k, v = kv.split("=")
        if k.startswith("ensvs_"):  # integer arguments separated by ':'
            call(k, *[int(x) for x in v.split(":")])
        else:  # [module.]FLAG[:key] of the package (default module kernels, key "on")
            import importlib
            k, key = k.split(":") if ":" in k else (k, "on")
            mod, flag = k.rsplit(".", 1) if "." in k else ("kernels", k)
            getattr(importlib.import_module("ensemble_svs_with_interactions_amd." + mod),
                    flag)[key] = bool(int(v))
sys.argv = ["bench.py", "--steps", "20", "--warmup", "3", "--no-cpu-baseline", "--no-synth",
            "--no-census", "--no-config2", "--no-shapes", "--no-real-data",
            ] + ([] if {tf!r} else ["--no-transformer"]) + ([] if {sf0!r} else ["--no-sf0"])
import bench
bench.main()
"""
SF0 = "--sf0" in sys.argv[1:]
TF = "--tf" in sys.argv[1:]
ARMS = [a for a in sys.argv[1:] if a not in ("--sf0", "--tf")]
for rep in range(2):
    for arm in ARMS:
        out = subprocess.run([sys.executable, "-c", RUN.format(root=ROOT, arm=arm, sf0=SF0, tf=TF)], cwd=ROOT,
                             capture_output=True, text=True, timeout=400)
        if out.returncode:
            print(out.stderr[-2000:])
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        leg = "separate_f0" if SF0 else ("transformer" if TF else None)
        ms = d[leg]["ms_per_step"] if leg else d["ms_per_step"]
        print(f"arm=[{arm}] {ms:.3f} ms" + (f" ({leg})" if leg else ""), flush=True)
