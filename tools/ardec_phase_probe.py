"""Per-phase sensitivity of the cooperative AR-decoder forward step (dev tool): times the modes
of tools/ardec_phase_probe.hip (the full step, then one phase removed at a time) at the bench
workload (H = 256, 30 sequences x 1024 frames = 256 AR steps) and prints us per AR step.
  python tools/ardec_phase_probe.py     (builds tools/libardec_probe.so)"""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libardec_probe.so")
CSRC = os.path.join(os.path.dirname(HERE), "ensemble_svs_with_interactions_amd", "csrc")
INC = os.path.join(os.path.dirname(HERE), "include")
MODES = ["full step", "no global stores", "no global input loads", "no MFMA",
         "no slab h loads", "no feat_out reduction", "publish without drain", "hand-off only"]


def build():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-shared", "-I", CSRC, "-I", INC, "-o", SO,
                    os.path.join(HERE, "ardec_phase_probe.hip")], check=True)


def main():
    if not os.path.exists(SO):
        build()
    lib = ctypes.CDLL(SO)
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.probe_launch.argtypes = [ci] + [vp] * 6 + [ci, ci] + [vp] * 7
    lib.probe_work_bytes.restype = ctypes.c_longlong
    H, B, T = 256, 30, 1024
    Tr = T // 4
    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(1)
    gx = torch.randn(B * Tr, 4 * H, device=dev, generator=g) * 0.5
    ofx = torch.randn(B * Tr, 4, device=dev, generator=g) * 0.3
    wp = (torch.randn(4 * H * H, device=dev, generator=g) * 0.05).half()
    wih = torch.randn(4 * H, device=dev, generator=g) * 0.05
    wfo = torch.randn(4, H + 130, device=dev, generator=g) * 0.05
    mask = torch.ones(B * Tr, device=dev)
    lf0 = torch.empty(B * T, device=dev)
    sg = torch.empty(B * Tr, 4 * H, device=dev)
    sc = torch.empty(B * Tr, H, device=dev)
    sh = torch.empty(B * Tr, H, device=dev)
    so = torch.empty(B * Tr, 4, device=dev)
    work = torch.zeros(lib.probe_work_bytes(), dtype=torch.uint8, device=dev)
    for mode, name in enumerate(MODES):
        def run():
            r = lib.probe_launch(mode, gx.data_ptr(), ofx.data_ptr(), wp.data_ptr(), wih.data_ptr(),
                                 wfo.data_ptr(), mask.data_ptr(), B, T, lf0.data_ptr(),
                                 sg.data_ptr(), sc.data_ptr(), sh.data_ptr(), so.data_ptr(),
                                 work.data_ptr(), st)
            assert r == 0, r
        for _ in range(2):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        print(f"mode {mode} {name:24s} {us:8.1f} us/launch {us / Tr:6.2f} us/AR step", flush=True)


if __name__ == "__main__":
    sys.exit(main())
