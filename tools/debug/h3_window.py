"""Debug: the instruction window of the round-1 f16x3 miscompute.

    python tools/debug/h3_window.py [--asm path.s]

Builds (or reads) the device assembly of mano_kernels_h3.hip in the failing
configuration -- SLP vectorizer on, no_pack transparent (-DMANO_H3_NO_PACK=0)
-- and, for every `v_pk_fma_f32 vD, vS, s[a:b], 0 op_sel_hi:[1,1,0]` (the
packed unscale of the LBS output) in each blend_skin_h3 instantiation, lists
every instruction from its issue to the first reader of vD, marking:
  W-src  writes a register of vS (the packed op's source pair)
  W-sgpr writes s[a:b]
  R-dst  reads vD (the consumer: the window ends there)
  vmem / lds / mfma   the instruction class
and the number of vector-memory ops issued since the last vmcnt wait (the
wave's outstanding VMEM work at that point).  Output: one JSON object per
window, so the failing (rest_verts: kVposed) and passing instantiations can
be compared line by line."""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(REPO, "mano-hand_amd", "csrc", "mano_kernels_h3.hip")
PK = re.compile(r"^\s*v_pk_fma_f32 v\[(\d+):(\d+)\], v\[(\d+):(\d+)\], s\[(\d+):(\d+)\], 0 op_sel_hi:\[1,1,0\]")


def build_asm(out="/tmp/h3pack.s"):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-DMANO_DIAGNOSTIC_BUILD=1", "-DMANO_H3_NO_PACK=0", "--cuda-device-only", "-S",
                    "-o", out, SRC], check=True, capture_output=True)
    return out


def regs(text, kind):
    """Register numbers of `kind` ('v' or 's') named in an operand string."""
    out = set()
    for a, b in re.findall(rf"\b{kind}\[(\d+):(\d+)\]", text):
        out |= set(range(int(a), int(b) + 1))
    for a in re.findall(rf"\b{kind}(\d+)\b", text):
        out.add(int(a))
    return out


def split_ops(line):
    """(mnemonic, dst operand text, src operand text) of one instruction."""
    code = line.split(";")[0].strip()
    if not code or code.endswith(":") or code.startswith("."):
        return None
    parts = code.split(None, 1)
    mn = parts[0]
    ops = parts[1] if len(parts) > 1 else ""
    fields = [f.strip() for f in re.split(r",(?![^\[]*\])", ops)]
    if mn.startswith(("global_store", "buffer_store", "ds_write", "s_waitcnt", "s_barrier", "s_nop",
                      "s_cbranch", "s_branch")) or not fields or not fields[0]:
        return mn, "", ops
    return mn, fields[0], ", ".join(fields[1:])


def windows(asm_path):
    lines = open(asm_path).read().splitlines()
    func, out = None, []
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            func = m.group(1)
            continue
        pm = PK.match(l)
        if not pm or func is None or "blend_skin_h3" not in func:
            continue
        d = set(range(int(pm.group(1)), int(pm.group(2)) + 1))
        src = set(range(int(pm.group(3)), int(pm.group(4)) + 1))
        sg = set(range(int(pm.group(5)), int(pm.group(6)) + 1))
        # VMEM ops outstanding: issued since the last vmcnt wait, walking back
        back = 0
        for j in range(i - 1, 0, -1):
            t = lines[j].strip()
            if t.startswith("s_waitcnt") and "vmcnt" in t:
                break
            if re.match(r"(global_|buffer_|flat_)", t):
                back += 1
            if re.match(r"^_Z\S+:", lines[j]):
                break
        win, vm = [], back
        for j in range(i + 1, min(i + 200, len(lines))):
            ops = split_ops(lines[j])
            if ops is None:
                continue
            mn, dst, srcs = ops
            tags = []
            if mn.startswith("s_waitcnt") and "vmcnt" in srcs:
                vm = int(re.search(r"vmcnt\((\d+)\)", srcs).group(1))
            if re.match(r"(global_|buffer_|flat_)", mn):
                vm += 1
                tags.append("vmem")
            if mn.startswith("ds_"):
                tags.append("lds")
            if mn.startswith("v_mfma"):
                tags.append("mfma")
            if dst and regs(dst, "v") & src:
                tags.append("W-src")
            if dst and regs(dst, "s") & sg:
                tags.append("W-sgpr")
            reads = regs(srcs, "v") | (regs(dst, "v") if mn.startswith(("global_store", "buffer_store")) else set())
            if mn.startswith(("global_store", "buffer_store", "ds_write")):
                reads |= regs(srcs, "v")
            hit = bool(reads & d)
            if hit:
                tags.append("R-dst")
            win.append({"inst": lines[j].split(";")[0].strip(), "tags": tags, "vmem_outstanding_max": vm})
            if hit:
                break
        out.append({"function": func, "line": i + 1, "pk_fma": l.strip(), "vmem_outstanding_at_issue": back,
                    "window": win})
    return out


if __name__ == "__main__":
    path = sys.argv[sys.argv.index("--asm") + 1] if "--asm" in sys.argv else build_asm()
    for w in windows(path):
        print(json.dumps(w))
