"""Instruction mix per basic block of one kernel in a hipcc -S listing.

usage: asm_mix.py FILE.s KERNEL_SUBSTRING [min_block_instrs]
Categories: VALU (v_*, split pk / f64 / other), SALU (s_* minus waitcnt/nop/branch),
LDS (ds_*), VMEM (global_/buffer_), waits/nops, branches.
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(m):
    if m.startswith("v_"):
        if m.startswith("v_pk_"):
            return "v_pk"
        if "_f64" in m:
            return "v_f64"
        if m.startswith("v_accvgpr"):
            return "v_acc"
        return "v_other"
    if m.startswith("ds_"):
        return "lds"
    if m.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if m in ("s_waitcnt", "s_nop") or m.startswith("s_waitcnt"):
        return "wait"
    if m.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if m.startswith("s_"):
        return "salu"
    return "other"


def main(path, kname, min_n=0):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kname in l
                 and l.rstrip().endswith(tuple(":")) or (l.startswith("_Z") and kname in l))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = Counter()
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
        if m:
            cur = m.group(1) + m.group(2)
            blocks[cur] = Counter()
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        mn = s.split()[0]
        blocks[cur][classify(mn)] += 1
        blocks[cur]["_all"] += 1
        if mn.startswith("v_"):
            blocks[cur]["~" + mn] += 1
    tot = Counter()
    for b, c in blocks.items():
        tot.update(c)
        if c["_all"] >= min_n:
            print("%-60s %6d  " % (b[:60], c["_all"]) + " ".join(
                "%s=%d" % (k, c[k]) for k in ("v_pk", "v_f64", "v_other", "v_acc", "salu",
                                              "lds", "vmem", "wait", "branch")))
    print("TOTAL", tot["_all"], {k: v for k, v in tot.items() if not k.startswith("~")})
    top = sorted(((v, k) for k, v in tot.items() if k.startswith("~")), reverse=True)[:40]
    print(" ".join("%s:%d" % (k[1:], v) for v, k in top))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 0)
