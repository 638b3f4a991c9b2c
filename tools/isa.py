#!/usr/bin/env python3
"""Disassemble one kernel of a built library's gfx950 code object and count
its instruction mnemonics.   python tools/isa.py lib.so kernel-substring [--dump out.s]"""
import collections
import os
import re
import subprocess
import sys
import tempfile


def main(lib, flt, *rest):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "co.o")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
        subprocess.run(["/opt/rocm/llvm/bin/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        txt = subprocess.run(["/opt/rocm/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", co],
                             capture_output=True, text=True).stdout
    funcs = re.split(r"\n(?=[0-9a-f]+ <)", txt)
    for f in funcs:
        head = f.split("\n")[0]
        if flt not in head:
            continue
        ins = [l.strip().split()[0] for l in f.split("\n")[1:] if l.strip() and not l.strip().startswith(";")
               and not l.strip().endswith(":")]
        c = collections.Counter(ins)
        print(head, len(ins), "instructions")
        for k, v in c.most_common(40):
            print(f"  {k:28s} {v}")
        if "--dump" in rest:
            open(rest[rest.index("--dump") + 1], "w").write(f)
        break


if __name__ == "__main__":
    main(*sys.argv[1:])
