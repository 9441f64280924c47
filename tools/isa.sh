#!/bin/bash
# Development tool: disassemble one kernel of a built library.  Usage: tools/isa.sh LIB.so KERNEL_SUBSTRING > out.s
set -e
LIB=$(readlink -f "$1"); PAT="$2"
D=$(mktemp -d)
cp "$LIB" "$D/lib.so"
( cd "$D" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading lib.so >/dev/null 2>&1 )
for f in "$D"/lib.so.*hipv4*; do /opt/rocm/lib/llvm/bin/llvm-objdump -d "$f"; done > "$D/dis.s"
L0=$(grep -n "^[0-9a-f]* <.*$PAT" "$D/dis.s" | head -1 | cut -d: -f1)
awk -v s="$L0" 'NR>=s' "$D/dis.s" | awk '/^[0-9a-f]+ <_Z/ && NR>1 {exit} {print}'
rm -rf "$D"
