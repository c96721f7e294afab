"""Per-kernel VGPR / AGPR / scratch of a HIP source compiled for gfx950 (dev tool).
   python tools/kernel_regs.py ensemble_svs_with_interactions_amd/csrc/gemm.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                "-Iensemble_svs_with_interactions_amd/csrc", "-Iinclude", "--cuda-device-only",
                "-S", "-o", "/tmp/kregs.s", src], check=True, stderr=subprocess.DEVNULL)
s = open("/tmp/kregs.s").read()
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    get = lambda k: (re.search(k + r" (\d+)", body) or [None, "-"])[1]  # noqa: E731
    print(f"{name[:78]:78s} vgpr {get('next_free_vgpr'):>4} accoff {get('accum_offset'):>4} "
          f"scratch {get('private_segment_fixed_size'):>4}")
