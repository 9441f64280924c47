"""Disassemble one kernel of a built object or library (development tool).
Usage: python tools/isa.py FILE.o|.so 'kernel-name-regex' > out.s"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main(path, pat):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "-C", co],
                             capture_output=True, text=True).stdout
    rx = re.compile(pat)
    on = False
    for line in txt.splitlines():
        if line and not line.startswith(" ") and line.endswith(">:"):
            on = bool(rx.search(line))
        if on:
            print(line)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
