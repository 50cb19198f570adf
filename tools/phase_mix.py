#!/usr/bin/env python3
"""Per-phase instruction mix of a register-tile kernel from its listing (analysis builds
with -DMHF_PHASE_MARKS: tile.hip.h MHF_PHASE): every instruction between two
';@mhf-phase NAME' markers, in listing order, is counted to NAME (the tile loop is
straight-line code per phase; blocks of the loop's other paths land in the phase they
follow). Usage: python tools/phase_mix.py FILE.s KERNEL_SUBSTRING"""
import collections
import re
import sys


def kind(op):
    if op.startswith("v_pk_"):
        return "v_pk"
    if op.startswith("v_accvgpr"):
        return "acc"
    if op.startswith("v_") and ("f64" in op):
        return "v_f64"
    if op.startswith("v_"):
        return "v_other"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_"):
        return "vmem"
    return "other"


def main(path, ksub):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(ksub), l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    phase = "prologue"
    cnt = collections.OrderedDict()
    for l in lines[start:end]:
        t = l.strip()
        m = re.search(r";@mhf-phase (.+)$", t)
        if m:
            phase = m.group(1).strip()
            continue
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        cnt.setdefault(phase, collections.Counter())[kind(op)] += 1
    cols = ["v_pk", "v_f64", "v_other", "acc", "salu", "lds", "vmem", "wait", "nop", "branch"]
    print("| phase | VALU | " + " | ".join(cols) + " |")
    print("|---|---|" + "---|" * len(cols))
    for ph, c in cnt.items():
        valu = c["v_pk"] + c["v_f64"] + c["v_other"] + c["acc"]
        print("| %s | %d | " % (ph, valu) + " | ".join(str(c[k]) for k in cols) + " |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
