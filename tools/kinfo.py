#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / SGPR / scratch / LDS of a built library's gfx950 code object.
   python tools/kinfo.py modulations_amd/lib/libtdec.so [kernel-name-filter]"""
import os
import re
import subprocess
import sys
import tempfile


def main(lib, flt=""):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "co.o")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
        subprocess.run(["/opt/rocm/llvm/bin/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        txt = subprocess.run(["/opt/rocm/llvm/bin/llvm-readelf", "--notes", co], capture_output=True,
                             text=True).stdout
    for blk in txt.split("- .agpr_count")[1:]:
        blk = ".agpr_count" + blk
        m = re.search(r"\.name:\s+(\S+)", blk)
        name = m.group(1) if m else "?"
        if flt not in name:
            continue

        def g(k):
            m = re.search(r"\.%s:\s+(\S+)" % k, blk)
            return m.group(1) if m else "?"
        print(f"{name[:90]:90s} vgpr={g('vgpr_count')} agpr={g('agpr_count')} sgpr={g('sgpr_count')} "
              f"scratch={g('private_segment_fixed_size')} lds={g('group_segment_fixed_size')} "
              f"vspill={g('vgpr_spill_count')} sspill={g('sgpr_spill_count')}")


if __name__ == "__main__":
    main(*sys.argv[1:])
