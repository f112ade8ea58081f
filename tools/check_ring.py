#!/usr/bin/env python3
"""Static check of the wave ring's hand-counted VMEM queue (nc_hash_kernel_wr,
twemproxy_amd/csrc/nc_gpuhash_kernels.hip) in its gfx950 ISA (.s).

The ring waits with constant counts: wait_vm<kWaitOff> (offsets of tile
j + DS have landed) and wait_vm<kWaitSlab> (slab j has landed), with
kWaitOff = (DO - DS) * kIter and kWaitSlab = DS * kIter, which is right only
if every iteration issues exactly kIter = P + NOFF + 1 + NST ring operations
(inline-asm LDS-DMAs, dummies and stores) in the order issue_off ->
wait_off -> issue_slab (P) -> wait_slab -> ... stores. For every ring
instantiation in the code object this walks every path of the kernel's
basic-block graph and checks, counting only inline-asm VMEM instructions
(hipcc's own loads, e.g. the global reader of a tile too long for its slot,
only make the waits more conservative):

  - entry -> first wait_off:          (DO - DS) * kIter + NOFF + 1 ring ops
  - wait_off -> next wait_off:        kIter
  - wait_off -> the wait_slab after:  P
  - every asm vmcnt wait in the kernel is one of those two (or the final 0)

Template arguments come from the mangled name. exec is tracked as known
non-empty or unknown: non-empty at entry, after a restore (s_or_b64 exec, ...)
and on entering an if body (s_and_saveexec / s_and_b64 exec) — the ring
guards its DMAs with lane predicates that always hold for lane 0 (or every
lane), so a wave never skips one — and unknown after s_andn2 / s_xor into
exec (divergent loop exits, else arms).
With exec known non-empty, s_cbranch_execz falls through and
s_cbranch_execnz is taken (hipcc uses both as plain jumps there).

    python tools/check_ring.py twemproxy_amd/csrc/build/nc_gpuhash_kernels.s [kernel-substring]
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from check_vmcnt import BRANCH, VCCAND, consts_step, parse_blocks, successors  # noqa: E402

VMEM = re.compile(r"^(global_|buffer_|scratch_|flat_)\w+")
WAIT = re.compile(r"^s_waitcnt\s+.*vmcnt\((\d+)\)")
EXECW = re.compile(r"^s_(or|and_saveexec|or_saveexec|mov|andn2|and|xor|andn2_saveexec|xor_saveexec)_b64\s+exec\b")
ARGS = re.compile(r"nc_hash_kernel_wrI((?:Li(?:n?\d+)E){8})")


def ring_params(name):
    m = ARGS.search(name)
    if not m:
        return None
    v = [int(x.replace("n", "-")) for x in re.findall(r"Li(n?\d+)E", m.group(1))]
    mode, var, p, ds, do, dist, wpw, tk = v
    noff = 2 if tk == 256 else 1
    nst = tk // 64
    kiter = p + noff + 1 + nst
    return {"P": p, "DS": ds, "DO": do, "TK": tk, "NOFF": noff, "kIter": kiter,
            "wOff": (do - ds) * kiter, "wSlab": ds * kiter}


def check_kernel(body, name, k):
    blocks = parse_blocks(body)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    cap = k["kIter"] + k["wOff"] + k["NOFF"] + 2
    reports = {}

    def rep(no, msg):
        reports.setdefault(no, msg)

    # state: ops since the last wait_off (or entry), ops since that wait_off
    # for the slab check (None once checked / before any), seen a wait_off?
    start = (0, 0, None, False, (), True)
    seen = set()
    work = [(0, start)]
    steps = 0
    while work and steps < 400000:
        steps += 1
        i, st = work.pop()
        if (i, st) in seen:
            continue
        seen.add((i, st))
        c_off, _unused, c_slab, had_off, cs, exec_nz = st
        consts, vcc_known = dict(cs), None
        for no, s, asm in blocks[i][1]:
            e = EXECW.match(s)
            if e:
                exec_nz = e.group(1) in ("or", "and", "and_saveexec", "or_saveexec", "mov")
            if s.startswith("s_"):  # known-constant SGPR pairs prune hipcc's flag branches (check_vmcnt.py)
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
            w = WAIT.match(s)
            if w and asm:
                n = int(w.group(1))
                if n == 0:
                    continue
                is_off = n == k["wOff"] and (c_off == (k["kIter"] if had_off else k["wOff"] + k["NOFF"] + 1))
                is_slab = n == k["wSlab"] and c_slab is not None and c_slab == k["P"]
                if is_slab and not (is_off and c_slab is None):
                    c_slab = None
                    continue
                if is_off:
                    c_off, c_slab, had_off = 0, 0, True
                    continue
                want = (f"wait_off after {k['kIter'] if had_off else k['wOff'] + k['NOFF'] + 1} ring ops"
                        f" or wait_slab after {k['P']}")
                rep(no, f"vmcnt({n}) after {c_off} ring ops since the last wait_off "
                        f"({c_slab} since it for the slab); expected {want}")
                continue
            if asm and VMEM.match(s):
                c_off = min(c_off + 1, cap)
                if c_slab is not None:
                    c_slab = min(c_slab + 1, cap)
        nst = (c_off, 0, c_slab, had_off, tuple(sorted(consts.items())), exec_nz)
        last = blocks[i][1][-1][1] if blocks[i][1] else ""
        b = BRANCH.match(last)
        succ = successors(blocks[i], consts, vcc_known)
        if b and exec_nz and b.group(1) == "s_cbranch_execz":
            succ = [x for x in succ if x != b.group(2)]  # exec non-empty: falls through
        elif b and exec_nz and b.group(1) == "s_cbranch_execnz":
            succ = [b.group(2)]  # exec non-empty: taken
        for sname in succ:
            j = idx.get(sname)
            if j is not None:
                work.append((j, nst))
    if work:
        rep(0, f"exploration bound hit ({steps} steps)")
    for no in sorted(reports):
        print(f"{name}:{no}: {reports[no]}")
    return len(reports)


def kernels(path, want=""):
    text = open(path).read().splitlines()
    out, cur = [], None
    for i, line in enumerate(text, 1):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = [m.group(1), []]
            out.append(cur)
        elif cur is not None:
            if line.startswith("\t.section") or line.startswith("\t.size") or re.match(r"^\s*\.Lfunc_end", line):
                cur = None
                continue
            cur[1].append((i, line))
    return [(n, b) for n, b in out if "nc_hash_kernel_wr" in n and want in n]


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    total = nk = 0
    for name, body in kernels(path, want):
        k = ring_params(name)
        if k is None:
            continue
        nk += 1
        total += check_kernel(body, name[-48:], k)
    print(f"{nk} ring kernel(s), {total} report(s)")
    return 1 if total or nk == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
