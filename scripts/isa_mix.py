"""Instruction mix of one kernel in a hipcc -S listing, per loop body.

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S -o k.s hq_kernels.hip
    python scripts/isa_mix.py k.s cost16w_kernelILi0ELb1

A loop is a label that a later s_cbranch/s_branch jumps back to; its body is the
text between the label and that branch.  Used to see where VALU issue goes
(DESIGN.md "Performance log").
"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r"^(_Z\S*%s\S*):(.*?)^\.Lfunc_end" % re.escape(key), s, re.S | re.M)
    if not m:
        sys.exit("kernel not found")
    lines = m.group(2).split("\n")
    labels = {}
    for i, ln in enumerate(lines):
        lm = re.match(r"^(\.LBB\w+):", ln)
        if lm:
            labels[lm.group(1)] = i
    total = collections.Counter()
    loops = []
    for i, ln in enumerate(lines):
        om = re.match(r"\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|scratch_\w+)", ln)
        if om:
            total[om.group(1)] += 1
        bm = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", ln)
        if bm and bm.group(1) in labels and labels[bm.group(1)] < i:
            loops.append((labels[bm.group(1)], i, bm.group(1)))
    print("whole kernel: %d instructions" % sum(total.values()))
    for a, b, name in loops:
        c = collections.Counter()
        for ln in lines[a:b + 1]:
            om = re.match(r"\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|scratch_\w+)", ln)
            if om:
                c[om.group(1)] += 1
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print("\nloop %s lines %d-%d: %d instr, %d VALU" % (name, a, b, sum(c.values()), valu))
        for k, v in c.most_common(18):
            print("   %-26s %d" % (k, v))


if __name__ == "__main__":
    main()
