#!/usr/bin/env python3
"""Static instruction counts per basic block of one kernel in a device assembly file (hipcc --cuda-device-only -S),
with loop back-edges marked, to cost a visit loop by instruction class.
Usage: tools/isa_blocks.py FILE.s KERNEL_SUBSTRING [--min N]"""
import re
import sys


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 1
    text = open(path).read()
    syms = [m.group(1) for m in re.finditer(r"^(\S*" + re.escape(name) + r"\S*):(\s|$)", text, re.M)]
    if not syms:
        sys.exit(f"no kernel matching {name}")
    sym = syms[0]
    i = text.index(sym + ":")
    j = text.index(".Lfunc_end", i)
    lines = text[i:j].splitlines()[1:]
    blocks, order = {}, []
    cur = "entry"
    blocks[cur] = {"n": {}, "targets": [], "line": 0}
    order.append(cur)
    for k, ln in enumerate(lines):
        s = ln.split(";")[0].strip()
        if not s or s.startswith("."):
            if re.match(r"^\.LBB\S+:", s):
                cur = s[:-1]
                blocks[cur] = {"n": {}, "targets": [], "line": k}
                order.append(cur)
            continue
        if s.endswith(":"):
            continue
        op = s.split()[0]
        c = classify(op)
        blocks[cur]["n"][c] = blocks[cur]["n"].get(c, 0) + 1
        if c == "branch":
            t = s.split()[-1]
            blocks[cur]["targets"].append(t)
    pos = {b: n for n, b in enumerate(order)}
    print(f"{sym[:90]}")
    cols = ["valu", "salu", "smem", "lds", "vmem", "branch", "wait"]
    print(f"{'block':14s} " + " ".join(f"{c:>6s}" for c in cols) + "  back-edges")
    for b in order:
        n = blocks[b]["n"]
        tot = sum(n.values())
        if tot < mn:
            continue
        back = [t for t in blocks[b]["targets"] if t in pos and pos[t] <= pos[b]]
        print(f"{b:14s} " + " ".join(f"{n.get(c, 0):6d}" for c in cols) + ("  -> " + ",".join(back) if back else ""))


if __name__ == "__main__":
    main()
