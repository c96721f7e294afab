"""Queue / stream attribution of the inference part of a kernel trace (dev tool):
kernels after the last Adam launch, counted per (hardware queue, stream) and per kernel.
  python3 tools/trace_queues.py TRACE_CSV"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:30],
             r["Queue_Id"], r["Stream_Id"]) for r in rows)
last = max((i for i, k in enumerate(ks) if "adam_kernel" in k[2]), default=-1)
inf = ks[last + 1:]
print("inference kernels per (queue, stream):",
      collections.Counter((k[3], k[4]) for k in inf).most_common(12))
c = collections.Counter((k[3], k[4], k[2]) for k in inf
                        if any(s in k[2] for s in ("dual", "p_sample", "ardec", "lstm")))
for key, n in c.most_common(14):
    print(n, key)
