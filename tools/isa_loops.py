"""List the loops of a kernel in a hipcc --save-temps .s file with the
s_waitcnt / global_load / ds instructions inside each (to check that the RX
pipeline keeps counted vmcnt waits).  Usage: isa_loops.py file.s kernel_substring"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    s = open(path).read()
    names = [n for n in re.findall(r"^([A-Za-z_]\w*):", s, re.M) if pat in n]
    name = names[0]
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].split("\n")
    labels = {}
    for k, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = k
    loops = set()
    for k, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            loops.add((labels[m.group(1)], k))
    print(name)
    for a, b in sorted(loops):
        ins = [body[x].strip() for x in range(a, b + 1)]
        loads = sum(1 for x in ins if x.startswith(("global_load", "buffer_load")))
        waits = [x.split(";")[0].strip() for x in ins if x.startswith("s_waitcnt") and "vmcnt" in x]
        nins = sum(1 for x in ins if x and not x.startswith((";", ".")))
        print(f"  loop {body[a].split(':')[0]} lines {a}-{b} instr {nins} vmem_loads {loads} vm_waits {waits}")


if __name__ == "__main__":
    main()
