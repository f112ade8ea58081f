#!/usr/bin/env python3
"""Static VALU count of one kernel's ISA (CPU only: hipcc -S for gfx950).

    python tools/valu_count.py twemproxy_amd/csrc/nc_md5_kernels.hip \
        _Z20nc_md5_direct_kernelILb0ELb0ELi0EEvPKhPKmmPjmj [--blocks]

Prints the function's VALU instruction total, the part in blocks of more than
200 VALU (the unrolled hash steps) and the rest (padding, bookkeeping), and
with --blocks each basic block's VALU count and its last instruction, so a
change to a round's bookkeeping can be counted before a GPU A/B. md5's time
follows its dynamic SQ_INSTS_VALU; this is the static view.
"""
import re
import subprocess
import sys


def main() -> int:
    src, kern = sys.argv[1], sys.argv[2]
    show = "--blocks" in sys.argv[3:]
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-Iinclude",
                    "-Itwemproxy_amd/csrc", "-S", "--cuda-device-only", src, "-o", "/tmp/valu_count.s"],
                   check=True, stderr=subprocess.DEVNULL)
    s = open("/tmp/valu_count.s").read()
    a = s.index(kern + ":")
    b = s.index(".Lfunc_end", a)
    blocks, cur = [], None
    for line in s[a:b].split("\n"):
        t = line.strip()
        if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", t):
            cur = [t.split()[0], []]
            blocks.append(cur)
            continue
        if cur is None or not t or t.startswith(";") or t.startswith("."):
            continue
        cur[1].append(t)
    total = big = 0
    for name, ins in blocks:
        v = sum(1 for i in ins if i.startswith("v_"))
        total += v
        big += v if v > 200 else 0
        if show:
            print(f"{name:14s} valu={v:4d} last={ins[-1] if ins else ''}")
    print(f"valu total {total}, in step blocks {big}, other {total - big}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
