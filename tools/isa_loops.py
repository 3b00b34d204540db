"""Instruction mix of a kernel's loops in a device assembly file (hipcc --cuda-device-only -S).

    python tools/isa_loops.py <file.s> <kernel-name regex>

For every backward branch (a loop) prints its size and counts: MFMA, other VALU, LDS reads / writes, buffer loads,
SALU, waitcnt, barriers. Static counts per loop iteration (not dynamic)."""
import re
import sys
from collections import Counter


def main():
    path, pat = sys.argv[1], re.compile(sys.argv[2])
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat.search(l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S*:", l)}
    print(lines[start].split(":")[0])
    for i, l in enumerate(body):
        m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\S+)|\s+s_branch\s+(\.LBB\S+)", l)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        j = labels.get(tgt)
        if j is None or j >= i:
            continue
        c = Counter()
        for ins in body[j:i + 1]:
            s = ins.strip()
            if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
                continue
            op = s.split()[0]
            if op.startswith("v_mfma"):
                c["mfma"] += 1
            elif op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("ds_read") or op.startswith("ds_load"):
                c["ds_read"] += 1
            elif op.startswith("ds_write") or op.startswith("ds_store"):
                c["ds_write"] += 1
            elif op.startswith("buffer_load") or op.startswith("global_load"):
                c["vmem_load"] += 1
            elif op.startswith("s_waitcnt"):
                c["waitcnt"] += 1
            elif op == "s_barrier":
                c["barrier"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            else:
                c["other:" + op] += 1
        print(f"  loop {tgt} lines {j}-{i}: " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
