#!/usr/bin/env python3
"""Static check of hand-counted vmcnt pipelines in a kernel's ISA (.s).

Builds each kernel's basic-block graph (labels, s_branch / s_cbranch_*,
fall-through) and explores it path-sensitively: the state is the queue of
outstanding VMEM operations (youngest last, each with the VGPRs it will
write) plus the SGPR pairs known to hold 0 or -1 (from `s_mov_b64`), which
prunes the `s_and_b64 vcc, exec, s[..]` / `s_cbranch_vcc*` edges hipcc
emits for loop exits. States are deduplicated per block; `s_waitcnt
vmcnt(N)` keeps the N youngest.
Any instruction that reads or writes a VGPR which may still be the
destination of an outstanding INLINE-ASM load is reported: it reads garbage,
or its result is overwritten later by the load's return. hipcc tracks its own
loads, so only asm loads (between ;;#ASMSTART/;;#ASMEND) are checked.

    python tools/check_vmcnt.py twemproxy_amd/csrc/build/nc_gpuhash_kernels.s [kernel-substring]
"""
import re
import sys

LOAD = re.compile(r"^\s*(global_load_\w+|buffer_load_\w+|scratch_load_\w+|flat_load_\w+)\s+(v\[\d+:\d+\]|v\d+)")
VMEM_NODEST = re.compile(r"^\s*(global_store_\w+|buffer_store_\w+|scratch_store_\w+|global_load_lds_\w+|"
                         r"buffer_load_\w+.*\blds\b|global_atomic_\w+)")
WAIT = re.compile(r"s_waitcnt\s+.*vmcnt\((\d+)\)")
VREG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")
LABEL = re.compile(r"^(\.?L\w+|\.LBB\w+):")
BRANCH = re.compile(r"^\s*(s_branch|s_cbranch_\w+)\s+(\S+)")
MAXQ = 64


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse_blocks(lines):
    """-> list of blocks [label, [(lineno, text, in_asm)], succ-labels]"""
    blocks = []
    cur = ["<entry>", [], []]
    in_asm = False
    for no, raw in lines:
        if ";;#ASMSTART" in raw:
            in_asm = True
            continue
        if ";;#ASMEND" in raw:
            in_asm = False
            continue
        lm = LABEL.match(raw.strip())
        if lm:
            if cur[1] or cur[0] == "<entry>":
                cur[2].append(lm.group(1))  # fall-through
                blocks.append(cur)
            else:
                cur[2].append(lm.group(1))
                blocks.append(cur)
            cur = [lm.group(1), [], []]
            continue
        line = raw.split(";")[0].rstrip()
        s = line.strip()
        if not s or s.startswith("."):
            continue
        cur[1].append((no, s, in_asm))
        b = BRANCH.match(s)
        if b:
            cur[2].append(b.group(2))
            if b.group(1) == "s_branch":
                blocks.append(cur)
                cur = ["<dead@%d>" % no, [], []]
            else:  # conditional: ends the block, falls through to a new one
                nxt = "<ft@%d>" % no
                cur[2].append(nxt)
                blocks.append(cur)
                cur = [nxt, [], []]
            continue
        if s.startswith(("s_endpgm", "s_setpc")):
            blocks.append(cur)
            cur = ["<dead@%d>" % no, [], []]
    blocks.append(cur)
    return blocks


def transfer(insts, q, report):
    q = list(q)
    for no, s, asm in insts:
        w = WAIT.search(s)
        if w:
            n = int(w.group(1))
            if len(q) > n:
                q = q[len(q) - n:]
            continue
        if s.startswith("s_waitcnt"):
            continue
        m = LOAD.match(s)
        if m and " lds" not in s:
            used = regs(s[m.end():])
            dest = regs(m.group(2))
            for d, a in q:
                if a and (d & (used | dest)):
                    report(no, s, d & (used | dest))
                    break
            q.append((frozenset(dest), asm))
        elif VMEM_NODEST.match(s):
            used = regs(s)
            for d, a in q:
                if a and (d & used):
                    report(no, s, d & used)
                    break
            q.append((frozenset(), asm))
        elif s.startswith(("v_", "ds_", "s_")):
            used = regs(s)
            if used:
                for d, a in q:
                    if a and (d & used):
                        report(no, s, d & used)
                        break
        if len(q) > MAXQ:
            q = q[-MAXQ:]
    return tuple(q)


SMOV = re.compile(r"^s_mov_b64\s+(s\[\d+:\d+\]),\s*(-1|0)$")
VCCAND = re.compile(r"^s_(and|andn2)_b64\s+vcc,\s*(exec,\s*(s\[\d+:\d+\])|(s\[\d+:\d+\]),\s*exec)$")
SDEF = re.compile(r"^s_\w+\s+(s\[\d+:\d+\]|s\d+)")


def sregs(text):
    out = set()
    for m in re.finditer(r"s\[(\d+):(\d+)\]|\bs(\d+)\b", text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def consts_step(consts, s):
    """update the known-constant SGPR pairs for one scalar instruction"""
    m = SMOV.match(s)
    d = SDEF.match(s)
    if d:
        dead = sregs(d.group(1))
        consts = {k: v for k, v in consts.items() if not (sregs(k) & dead)}
    if m:
        consts[m.group(1)] = int(m.group(2))
    return consts


def successors(block, consts, vcc_known):
    """prune a conditional vcc branch whose vcc value is known"""
    succ = list(block[2])
    if not block[1]:
        return succ
    last = block[1][-1][1]
    b = BRANCH.match(last)
    if b and b.group(1) in ("s_cbranch_vccnz", "s_cbranch_vccz") and vcc_known is not None:
        taken = (vcc_known != 0) == (b.group(1) == "s_cbranch_vccnz")
        # block[2]: [fallthrough?, target] in textual order of discovery
        tgt = b.group(2)
        return [tgt] if taken else [x for x in succ if x != tgt]
    return succ


def run_block(insts, q, consts, report):
    q = list(q)
    consts = dict(consts)
    vcc_known = None
    for no, s, asm in insts:
        if s.startswith("s_"):
            vm = VCCAND.match(s)
            if vm:
                reg = vm.group(3) or vm.group(4)
                vcc_known = None
                if reg in consts:
                    v = consts[reg]
                    vcc_known = (1 if v == -1 else 0) if vm.group(1) == "and" else (0 if v == -1 else 1)
            elif "vcc" in s.split(",")[0] and not s.startswith("s_cbranch"):
                vcc_known = None
            consts = consts_step(consts, s)
        q = list(transfer([(no, s, asm)], tuple(q), report))
    return tuple(q), consts, vcc_known


def check(lines, name):
    blocks = parse_blocks(lines)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    seen = set()
    reps = {}

    def rep(no, s, r):
        reps.setdefault(no, (s, r))

    work = [(0, (), ())]
    steps = 0
    while work and steps < 200000:
        steps += 1
        i, q, cs = work.pop()
        key = (i, q, cs)
        if key in seen:
            continue
        seen.add(key)
        out, consts, vk = run_block(blocks[i][1], q, dict(cs), rep)
        ncs = tuple(sorted(consts.items()))
        for sname in successors(blocks[i], consts, vk):
            j = idx.get(sname)
            if j is not None:
                work.append((j, out, ncs))
    if work:
        print(f"{name}: exploration bound hit ({steps} steps)")
    for no in sorted(reps):
        s, r = reps[no]
        print(f"{name}:{no}: '{s[:70]}' touches v{sorted(r)} of an in-flight asm load")
    return len(reps)


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    text = open(path).read().splitlines()
    kernels = []
    cur = None
    for i, l in enumerate(text, 1):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            cur = [m.group(1), []]
            kernels.append(cur)
        elif cur is not None:
            if l.startswith("\t.section") or l.startswith("\t.size") or re.match(r"^\s*\.Lfunc_end", l):
                cur = None
                continue
            cur[1].append((i, l))
    total = 0
    for name, body in kernels:
        if want and want not in name:
            continue
        total += check(body, name[-40:])
    print(f"{total} report(s)")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
