"""Static check of the scalar-table pipeline in a hipcc -S listing (spectral_lane.hip.inc).

A block requested by `s_load_dwordx16 s[a:b]` is in flight until the next
`s_waitcnt lgkmcnt(0)`; no instruction in between may read or write any of s[a..b]
(LLVM does not know the asm load completes late). Linear scan per kernel; prints the
violations and the pipeline statistics.
usage: check_sload_pipeline.py FILE.s [KERNEL_SUBSTRING]
"""
import re
import sys

REG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")


def sregs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main(path, kname=""):
    bad = 0
    loads = waits = 0
    cur = None
    inflight = {}   # reg -> line number of the load
    for no, raw in enumerate(open(path), 1):
        line = raw.split(";")[0].strip()
        if raw.startswith("_Z") and raw.rstrip().endswith(":") or raw.startswith("_Z") and ": ;" in raw:
            cur = raw.split(":")[0]
            inflight.clear()
            continue
        if kname and (cur is None or kname not in cur):
            continue
        if not line or line.startswith(".") or line.endswith(":"):
            continue
        op = line.split()[0]
        if op == "s_waitcnt" and "lgkmcnt(0)" in line:
            inflight.clear()
            waits += 1
            continue
        used = sregs(line[len(op):])
        hit = used & set(inflight)
        if hit:
            bad += 1
            print("%s:%d: %s touches in-flight s%s (loaded at line %d)"
                  % (path, no, line, sorted(hit), inflight[min(hit)]))
        if op.startswith("s_load_dword"):
            dst = line[len(op):].split(",")[0]
            for r in sregs(dst):
                inflight[r] = no
            loads += 1
    print("scalar loads %d, lgkmcnt(0) waits %d, violations %d" % (loads, waits, bad))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
