#!/usr/bin/env python3
"""Does the compiler keep a wave's claim broadcast in the same loop as the claim?

Reads a gfx950 assembly listing (hipcc --save-temps) and, for every kernel with a claim atomic
(`*_atomic_add`), reports the innermost loop of the atomic (the compiler's own `Loop Header` /
`in Loop: Header=` block annotations) and whether any `ds_bpermute_b32` -- the `__shfl(k, 0)`
that broadcasts lane 0's claim -- sits directly in that loop.

A correct compile has the broadcast in the claim's loop.  The miscompile (heavy
pixels) moves it into an inner loop the atomic is outside of, whose back edge zeroes the claim
register and whose exit mask is `lane == 0`: after the first body, lanes 1..63 re-run the claim
check without lane 0 and render claim 0 again, forever.  Exit status 1 when a kernel shows it."""
import re
import sys


def blocks(path):
    """(kernel, label, innermost loop header or None, parent loop headers, is a loop header,
    instruction lines) per basic block"""
    kernel, label, loop, parents, header, lines = None, None, None, [], False, []
    for line in open(path):
        k = re.match(r"^(_Z\w+):", line)
        b = re.match(r"^(?:\.LBB(\d+_\d+):|; %bb\.(\d+):)", line)
        if k or b:
            if kernel and label:
                yield kernel, label, loop, parents, header, lines
            if k:
                kernel = k.group(1)
            label = (b.group(1) or ("bb" + b.group(2))) if b else None
            loop, parents, header, lines = None, [], False, []
            m = re.search(r"in Loop: Header=BB(\d+_\d+)", line)
            if m:
                loop = m.group(1)
            continue
        if re.search(r"=>\s*This (?:Inner )?Loop Header", line):
            loop, header = label, True
        m = re.search(r"Parent Loop BB(\d+_\d+)", line)
        if m and not lines:
            parents.append(m.group(1))
        m = re.search(r"in Loop: Header=BB(\d+_\d+)", line)
        if m and not lines:
            loop = m.group(1)
        if line.startswith("\t") and not line.lstrip().startswith(";"):
            lines.append(line.strip())
    if kernel and label:
        yield kernel, label, loop, parents, header, lines


def scan(path):
    """kernel -> (claim loop, [inner loops of it whose header broadcasts a register that the loop's
    own blocks zero: the split's signature])"""
    atomic_loop, bl = {}, []
    for kernel, label, loop, parents, header, lines in blocks(path):
        bl.append((kernel, label, loop, parents, header, lines))
        for ins in lines:
            if re.match(r"(global|flat|buffer)_atomic_add\b", ins) and loop is not None:
                atomic_loop.setdefault(kernel, loop)
    out = {}
    for kernel, a in atomic_loop.items():
        split = []
        for k2, label, loop, parents, header, lines in bl:
            if k2 != kernel or not header or a not in parents:
                continue
            srcs = set()
            for ins in lines:
                m = re.match(r"ds_bpermute_b32 v\d+, v\d+, (v\d+)", ins) or re.match(r"v_readfirstlane_b32 s\d+, (v\d+)", ins)
                if m:
                    srcs.add(m.group(1))
            zeroed = {r for k3, _l, lp, _p, _h, ls in bl if k3 == kernel and lp == label
                      for ins in ls for r in srcs if ins == f"v_mov_b32_e32 {r}, 0"}
            if zeroed:
                split.append(label)
        out[kernel] = (a, split)
    return out


if __name__ == "__main__":
    res = scan(sys.argv[1])
    bad = False
    for k, (a, split) in sorted(res.items()):
        print(f"{k}: claim atomic in loop BB{a}; claim re-broadcast by an inner loop: "
              + (", ".join("BB" + s for s in split) + "  <-- SPLIT" if split else "none"))
        bad |= bool(split)
    sys.exit(1 if bad else 0)
