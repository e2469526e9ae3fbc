#!/bin/bash
# CPU-only reproducer of the ROCm 7.2 (amdclang / llc, gfx950) miscompile that round 2 worked around in decode():
# the select form of the tuple zeroing (k.dport = l4_ok ? dport : 0, PPE_TUPLE_SELECT=1) loses dport for packets
# that fail syn_check.  Steps: device IR of the select build at -O3 (correct: a switch on the status with cases
# 255 and 17 to one block, the merge phi takes 0 only on the default edge), the C1 PART kernel extracted
# textually, llc -O3 for gfx950, and the lowered switch's LeafBlock printed: it zeroes the dport register for every
# lane with status != 255 before testing status == 17, and the later block restores only sport.
set -e
K=_ZN12_GLOBAL__N_119ppe_classify_kernelILi1ELi1ELi512ELb0ELb1EEEv9ppe_kargs
D=${1:-/tmp/ppe_select_repro}
mkdir -p $D
cd "$(dirname "$0")/../packet-process-engine_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -Icsrc -DPPE_TUPLE_SELECT=1 \
  --offload-device-only -emit-llvm -S csrc/ppe_kernels.hip -o $D/all.ll 2>/dev/null
python3 - "$D" "$K" <<'PY'
import sys
d, name = sys.argv[1], sys.argv[2]
lines = open(f"{d}/all.ll").read().split("\n")
out, i = [], 0
while i < len(lines):
    if lines[i].startswith("define "):
        j = i
        while lines[j] != "}":
            j += 1
        if name in lines[i]:
            out.extend(lines[i:j + 1])
        i = j + 1
        continue
    out.append(lines[i])
    i += 1
open(f"{d}/kernel.ll", "w").write("\n".join(out))
PY
echo "== IR: the status switch and the merge phis (dport = %first phi)"
grep -n -A12 "switch i32 .*, label" $D/kernel.ll | grep -B2 -A12 "i32 17, label" | head -20
/opt/rocm/lib/llvm/bin/llc -O3 -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 $D/kernel.ll -o $D/kernel.s
echo "== ISA: the lowered switch (LeafBlock runs for every lane with status != 255, including status 17)"
grep -n -B6 -A14 "%LeafBlock" $D/kernel.s | head -40
