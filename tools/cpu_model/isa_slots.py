"""Scratch-slot check over one function of a gfx950 assembly listing (hipcc --cuda-device-only -S):
splits the function into basic blocks, builds the branch CFG, and for every scratch slot that is
both stored and loaded reports whether a load is reachable from the entry without passing a store
to the same slot (a spill reloaded before it was spilled would read whatever the wave slot's
previous occupant left).  Also lists loads of slots the function never stores that are reachable
without a call (objects written by a callee, e.g. tok_build's Huff tables) — path-insensitive, so
these are candidates, not findings.  DESIGN.md §4, the r02 profiling-build failure.

usage: isa_slots.py LISTING.s FUNCTION_SYMBOL
"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    name = sys.argv[2]
    i = s.find(name + ":")
    j = s.find(".Lfunc_end", i)
    lines = s[i:j].splitlines()
    blocks, cur = [], []
    for k, l in enumerate(lines):
        t = l.strip()
        if re.match(r"^(\.LBB\w+):", t):
            if cur:
                blocks.append(cur)
            cur = [(k, t)]
            continue
        cur.append((k, t))
        if re.match(r"s_(cbranch_\w+|branch|endpgm|setpc)", t):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    labels = {}
    for bi, b in enumerate(blocks):
        m = re.match(r"^(\.LBB\w+):", b[0][1])
        if m:
            labels[m.group(1)] = bi
    succ = {}
    for bi, b in enumerate(blocks):
        last = b[-1][1]
        ss = []
        m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\w+)", last)
        if m:
            ss.append(labels[m.group(2)])
            if m.group(1) != "branch" and bi + 1 < len(blocks):
                ss.append(bi + 1)
        elif not last.startswith("s_endpgm") and bi + 1 < len(blocks):
            ss.append(bi + 1)
        succ[bi] = ss

    def block_of(line):
        for bi, b in enumerate(blocks):
            if b[0][0] <= line <= b[-1][0]:
                return bi

    def reach_avoiding(target_line, avoid_lines):
        tb = block_of(target_line)
        avoid = set(block_of(x) for x in avoid_lines)
        seen, st = set(), [0]
        while st:
            x = st.pop()
            if x in seen:
                continue
            seen.add(x)
            if x == tb:
                return True
            if x in avoid:
                continue
            st.extend(succ[x])
        return False

    stores, loads = {}, {}
    for k, l in enumerate(lines):
        m = re.search(r"scratch_store_\w+ off, v[\[\]\d:]+, off(?: offset:(\d+))?", l)
        if m:
            stores.setdefault(int(m.group(1) or 0), []).append(k)
        m = re.search(r"scratch_load_\w+ v[\[\]\d:]+, off, off(?: offset:(\d+))?", l)
        if m:
            loads.setdefault(int(m.group(1) or 0), []).append(k)
    print("stores by slot offset:", stores)
    for off, ls in sorted(loads.items()):
        if off in stores:
            for L in ls:
                print("slot %d: load at line %d reachable from the entry without a store: %s"
                      % (off, L, reach_avoiding(L, stores[off])))
    calls = [k for k, l in enumerate(lines) if "s_swappc" in l]
    for off, ls in sorted(loads.items()):
        if off not in stores:
            for L in ls:
                if reach_avoiding(L, calls):
                    print("slot %d (written by a callee): load at line %d reachable without a call" % (off, L))


if __name__ == "__main__":
    main()
