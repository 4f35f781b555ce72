"""Wait states between each MFMA and the first VALU read of its result, from a .s file.

For every `v_mfma*` writing v[a:b], scan forward (straight-line, until a
branch/label) to the first VALU instruction that reads one of v[a..b]; the gap
is counted the way the hardware counts wait states: 1 per instruction issued
in between, N + 1 for `s_nop N`.  Prints the histogram of gaps per kernel and
the smallest ones with their instruction pair (tools/microbench/mfma_raw.hip
measures how many the hardware needs).

    python tools/debug/mfma_read_gap.py file.s [kernel-substring]
"""
import re
import sys
from collections import Counter

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def split_ops(line):
    ins = line.split(";")[0].strip()
    if not ins or ins.endswith(":") or ins.startswith("."):
        return None, None, None
    op = ins.split()[0]
    rest = ins[len(op):]
    parts = [p.strip() for p in rest.split(",")]
    return op, parts[0] if parts else "", ",".join(parts[1:])


def analyse(lines):
    gaps = []
    for i, line in enumerate(lines):
        op, dst, src = split_ops(line)
        if not op or not op.startswith("v_mfma"):
            continue
        written = regs(dst)
        ws = 0
        for j in range(i + 1, min(i + 400, len(lines))):
            op2, d2, s2 = split_ops(lines[j])
            if op2 is None:
                if lines[j].strip().endswith(":"):
                    break
                continue
            if op2.startswith("s_cbranch") or op2 in ("s_branch", "s_endpgm", "s_setpc_b64"):
                break
            if op2.startswith("s_nop"):
                ws += int(d2 or 0) + 1
                continue
            reads = regs(s2) if not op2.startswith(("global_store", "buffer_store", "ds_write")) else regs(d2 + "," + s2)
            if op2.startswith("v_") and not op2.startswith("v_mfma") and reads & written:
                gaps.append((ws, line.strip(), lines[j].strip()))
                break
            if op2.startswith("v_mfma") and regs(d2) & written:
                break  # overwritten / accumulated by another MFMA first
            ws += 1
    return gaps


def main():
    text = open(sys.argv[1]).read().splitlines()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    kernels = {}
    cur = None
    for line in text:
        m = re.match(r"^(\S+):\s*(;.*)?$", line)
        if m and not line.startswith((".", "\t")) and not m.group(1).startswith((".L", "$")):
            cur = m.group(1)
            kernels[cur] = []
        elif cur:
            kernels[cur].append(line)
    for name, body in kernels.items():
        if want not in name:
            continue
        gaps = analyse(body)
        if not gaps:
            continue
        hist = Counter(g[0] for g in gaps)
        print(f"{name[:90]}: {len(gaps)} MFMA->VALU reads, gap histogram {dict(sorted(hist.items()))}")
        for ws, a, b in sorted(gaps)[:3]:
            print(f"    {ws:2d} wait states: {a}  ->  {b}")


if __name__ == "__main__":
    main()
