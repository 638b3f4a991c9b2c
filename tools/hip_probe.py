#!/usr/bin/env python3
"""Does the C-ABI library find the GPU on its own (no torch in the process)?
  python tools/hip_probe.py            # libtdec.so alone
  python tools/hip_probe.py --torch    # torch imported (and its HIP runtime loaded) first
Prints the tdec_create result, the HIP runtime the process mapped and the
device-visibility environment."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    if "--torch" in sys.argv:
        import torch
        print("torch sees", torch.cuda.device_count(), "device(s)")
    from modulations_amd import _native as _n
    from modulations_amd import dvb_rcs2_turbo as M
    print({k: v for k, v in os.environ.items() if "VISIBLE" in k or k.startswith(("HSA_", "HIP_", "ROCR"))})
    c = M.DVBRCS2_Turbo(48, "1/3")
    try:
        c.handle
        print("tdec_create: OK")
    except _n.TdecError as e:
        print("tdec_create:", e)
    with open("/proc/self/maps") as f:
        libs = sorted({ln.split()[-1] for ln in f if "amdhip" in ln or "hsa-runtime" in ln})
    print("\n".join(libs))


if __name__ == "__main__":
    main()
