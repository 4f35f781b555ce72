"""Wait states between each VMEM store and the first later write of its data or address VGPRs.

    python tools/debug/store_data_gap.py file.s [kernel-substring]

For every global_store_dwordx2/x3/x4 (data > 32 bits) prints the gap (1 per
instruction, N + 1 per s_nop N) to the first instruction that writes one of
its data VGPRs, as a histogram per kernel plus the tightest pairs.
"""
import re
import sys
from collections import Counter

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from mfma_read_gap import regs, split_ops  # noqa: E402


def analyse(lines):
    gaps = []
    for i, line in enumerate(lines):
        op, dst, src = split_ops(line)
        if not op or not op.startswith(("global_store_dwordx", "buffer_store_dwordx")):
            continue
        parts = [p.strip() for p in line.split(";")[0].split(None, 1)[1].split(",")]
        data = regs(parts[1])
        ws = 0
        for j in range(i + 1, min(i + 200, len(lines))):
            op2, d2, s2 = split_ops(lines[j])
            if op2 is None:
                if lines[j].strip().endswith(":"):
                    break
                continue
            if op2.startswith("s_cbranch") or op2 in ("s_branch", "s_endpgm"):
                break
            if op2.startswith("s_nop"):
                ws += int(d2 or 0) + 1
                continue
            if op2.startswith("v_") and regs(d2) & data:
                gaps.append((ws, line.strip(), lines[j].strip()))
                break
            ws += 1
    return gaps


def main():
    text = open(sys.argv[1]).read().splitlines()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    kernels, cur = {}, None
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
        print(f"{name[:80]}: {len(gaps)} store-data rewrites, gap histogram {dict(sorted(hist.items()))}")
        for ws, a, b in sorted(gaps)[:4]:
            print(f"    {ws:2d}: {a}  ->  {b}")


if __name__ == "__main__":
    main()
