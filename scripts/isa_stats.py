#!/usr/bin/env python3
"""Static ISA statistics of fr::chunk_kernel (build container, no GPU): compile fr_kernels.hip for gfx950,
extract the kernel, report its resources and the instruction mix of its tile loop (the innermost loop
that issues the wave-tile buffer loads) and of the whole kernel.  A quick CPU-side check of a kernel
edit before it is timed on the GPU.   usage: python scripts/isa_stats.py [extra hipcc flags...]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "frender_amd", "csrc", "fr_kernels.hip")
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    "--cuda-device-only", "-S", "-o", os.path.join(d, "k.s"), *sys.argv[1:], src], check=True,
                   stderr=subprocess.DEVNULL)
    asm = open(os.path.join(d, "k.s")).read()
m = re.search(r"^_ZN2fr12chunk_kernelILb0EEEvNS_8ScanArgsE:[^\n]*\n(.*?)s_endpgm", asm, re.S | re.M)
body = m.group(1).splitlines()
npos = asm.find(".name:           _ZN2fr12chunk_kernelILb0EEEvNS_8ScanArgsE")
lo = asm.rfind("\n  - .", 0, npos)
hi = asm.find("\n  - .", npos)
md = asm[lo:hi if hi > 0 else None]
def field(k):
    x = re.search(rf"\.{k}:\s+(\d+)", md)
    return int(x.group(1)) if x else None
ins = [l.strip().split()[0] for l in body if l.strip() and not l.strip().startswith((";", ".")) and not l.startswith(".")]
def mix(lines):
    c = collections.Counter(lines)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    return valu, c
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
# the tile loop: the backward branch with the most buffer_load_dwordx4 inside
best = None
for i, l in enumerate(body):
    mm = re.search(r"s_(?:c?branch\w*)\s+(\.LBB\d+_\d+)", l)
    if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
        seg = body[labels[mm.group(1)]:i + 1]
        n = sum("buffer_load_dwordx4" in x for x in seg)
        if n and (best is None or n > best[0] or (n == best[0] and len(seg) < best[2])):
            best = (n, labels[mm.group(1)], len(seg), i)
tv, tc = mix(ins)
print(f"vgpr {field('vgpr_count')} vgpr_spill {field('vgpr_spill_count')} sgpr {field('sgpr_count')} "
      f"sgpr_spill {field('sgpr_spill_count')} scratch {field('private_segment_fixed_size')} lds {field('group_segment_fixed_size')}")
print(f"kernel: {len(ins)} instructions, {tv} VALU, readlane {tc['v_readlane_b32']} writelane {tc['v_writelane_b32']}")
if best:
    seg = [l.strip().split()[0] for l in body[best[1]:best[3] + 1] if l.strip() and not l.strip().startswith((";", "."))]
    lv, lc = mix(seg)
    print(f"tile loop (lines {best[1]}-{best[3]}): {len(seg)} instructions, {lv} VALU, readlane {lc['v_readlane_b32']} "
          f"writelane {lc['v_writelane_b32']} scratch {sum(v for k, v in lc.items() if k.startswith('scratch'))} "
          f"waitcnt {lc['s_waitcnt']} calls {lc['s_swappc_b64']}")
    print("  top: " + ", ".join(f"{k} {v}" for k, v in lc.most_common(14)))
