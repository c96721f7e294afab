"""Per-phase sensitivity of the MFMA LSTM recurrence step (dev tool): times the modes of
tools/lstm_phase_probe.hip (full step, then one phase removed at a time) at the bench workload
(30 sequences x 1024 steps, both directions) and prints ns per recurrent step.
  python tools/lstm_phase_probe.py     (builds tools/liblstm_probe.so first if missing)"""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liblstm_probe.so")
MODES = ["full step", "no MFMA", "no activations", "no global I/O", "no LDS h/dG read",
         "loop + barrier only", "flush only", "chunk loads only", "flush without stores"]


def build():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-shared", "-o", SO, os.path.join(HERE, "lstm_phase_probe.hip")], check=True)


def main():
    if not os.path.exists(SO):
        build()
    lib = ctypes.CDLL(SO)
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.probe_launch.argtypes = [ci, ci, ci, vp, vp, ci, ci, vp, vp, vp]
    B, T = 30, 1024
    st = torch.cuda.current_stream().cuda_stream
    for H in (64, 128):
        gx = torch.randn(B * T, 8 * H, device="cuda") * 0.3
        dy = torch.randn(B * T, 2 * H, device="cuda") * 0.1
        y = torch.empty(B * T, 2 * H, device="cuda")
        sv = torch.rand(B * T * 10 * H, device="cuda")
        dg = torch.empty(B * T, 8 * H, device="cuda")
        wf = (torch.randn(2 * 4 * H * H, device="cuda") * 0.05).half()
        wb = (torch.randn(2 * 4 * H * H, device="cuda") * 0.05).bfloat16()
        for bwd in (0, 1):
            for mode, name in enumerate(MODES):
                args = ((dy, wb, sv, dg) if bwd else (gx, wf, y, sv))

                def run():
                    r = lib.probe_launch(H, mode, bwd, args[0].data_ptr(), args[1].data_ptr(), B,
                                         T, args[2].data_ptr(), args[3].data_ptr(), st)
                    assert r == 0, r
                for _ in range(2):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 5 * 1e3
                print(f"H={H:3d} {'bwd' if bwd else 'fwd'} mode {mode} {name:22s} "
                      f"{us:8.1f} us/launch {us * 1e3 / T:7.1f} ns/step", flush=True)


if __name__ == "__main__":
    sys.exit(main())
