"""Disassembly checks of the built gfx950 library (no HIP runtime needed).

    python tools/isa_scan.py [--json] [path/to/libmano_hip.so]

1. No packed fp32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) in any
   kernel: the SLP-packed unscale of the f16x3 rest_verts kernels misexecuted
   (DESIGN.md §4), and packed fp32 is the slower form beside MFMAs.
2. skin_pair's hand-counted vmcnt protocol (mano_skin_quad.hip, memory
   wave): the step's `s_waitcnt vmcnt(N)`, N = (kAhead - 1) * (3 + kDmaOps),
   is correct only if the unit awaited is the DMA group issued 3 + kDmaOps
   vector-memory ops earlier (5 + kDmaOps in the in-place instantiations:
   the tail's two partial stores).  On every control-flow path into each such wait
   the disassembly must end with: a DMA group (buffer_load ... lds, the awaited
   unit), at least 3 other vector-memory ops (the stores), then exactly
   kDmaOps LDS-DMA ops (the next unit), so at least N younger ops cover the
   awaited group.  A compiler or flag change that reorders or drops one of
   these ops fails here, on the CPU, instead of racing on the GPU.
   (`s_cbranch_execz` is taken as not taken: every exec-masked DMA of the
   memory wave keeps lane 0 active.)
3. No repeated store data: a run of 4 or more vector-memory stores of the
   same data register(s) with no write to them in between is flagged.  The
   toolchain pitfall of round 3 (`__builtin_bit_cast(unsigned, v[r])` of an
   `ext_vector_type` element compiles to element 0 for every r: sixteen
   `buffer_store_dword v0, ...` at different offsets) has this
   shape; storing one value to many places is nowhere in the design.
   (tests/native/bitcast_pitfall.hip is a two-kernel fixture: the pitfall and
   its fix; tests/test_codegen.py checks that the rule tells them apart.)

Used by tools/codegen_report.py at build time and by tests/test_gpu_codegen.py
on the library the GPU tests load (run in a child process started before the
tests initialise HIP)."""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "mano-hand_amd", "mano_amd", "libmano_hip.so")
LLVM = "/opt/rocm/llvm/bin"
PACKED_FP32 = re.compile(r"\bv_pk_(fma|mul|add)_f32\b")
# skin_pair memory wave: VMEM ops per LDS-DMA of a unit = 4 rows + 3
# transform sweeps (+ 1 translation load with kTrans), kAhead = 2.
SKIN_PAIR = re.compile(r"skin_pair_kernelILb([01])ELb([01])ELb([01])E(?:Lb([01])E)?")
# stores per step: 3 sweeps (+ the in-place tail's b32 and b64 pieces, kInPlace)
K_AHEAD, N_STORES, N_ROWS, N_TR = 2, 3, 4, 3
N_STORES_IN_PLACE = 5


def disassemble(lib=LIB):
    """llvm-objdump -d of every gfx950 code object in the library's fat binary."""
    work = tempfile.mkdtemp()
    try:
        fat = os.path.join(work, "fatbin.bin")
        subprocess.run([shutil.which("objcopy") or "objcopy", f"--dump-section=.hip_fatbin={fat}", lib],
                       check=True)
        data = open(fat, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        out = []
        for k, a in enumerate(starts):
            b = starts[k + 1] if k + 1 < len(starts) else len(data)
            part, co = os.path.join(work, f"b{k}.bin"), os.path.join(work, f"b{k}.co")
            open(part, "wb").write(data[a:b])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                            f"--output={co}"], check=True)
            out.append(subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co],
                                      check=True, capture_output=True, text=True).stdout)
        return "\n".join(out)
    finally:
        shutil.rmtree(work, ignore_errors=True)


_FUNC = re.compile(r"^([0-9a-f]+) <(\S+)>:$")
_INST = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<(\S+)\+0x([0-9a-f]+)>\s*$")


def functions(asm):
    """{name: [(addr, mnemonic, operands, target_addr or None)]} per function."""
    funcs, cur, base = {}, None, 0
    for line in asm.splitlines():
        m = _FUNC.match(line)
        if m:
            base, cur = int(m.group(1), 16), m.group(2)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = _INST.match(line)
        if not m:
            continue
        tgt = None
        t = _TARGET.search(line)
        if t and m.group(1).startswith(("s_branch", "s_cbranch")):
            tgt = base + int(t.group(2), 16) if t.group(1) == cur else None
        funcs[cur].append((int(m.group(3), 16), m.group(1), m.group(2).strip(), tgt))
    return funcs


def _vmem_kind(mn, ops):
    """'dma' (LDS-DMA), 'vmem' (other vector-memory op) or None."""
    if mn.startswith(("buffer_", "global_", "flat_", "scratch_")):
        if mn.startswith(("buffer_load", "global_load")) and re.search(r"\blds\b", ops):
            return "dma"
        if mn.startswith(("buffer_wbl2", "buffer_inv")):
            return None
        return "vmem"
    return None


_SREG = r"s\[\d+:\d+\]"


def _flow_step(mn, ops, consts, vcc):
    """The structurizer's flow variables, tracked along a path: an SGPR pair
    set to a constant (s_mov_b64 s[a:b], -1 / 0) and `s_andn2_b64 vcc, exec,
    s[a:b]` of a known pair (vcc nonzero iff the pair is 0 -- exec is never 0
    here: every exec-masked region of the memory wave keeps lane 0).  An
    if / else whose arms the compiler emitted as two guarded blocks (the
    second skipped through such a vcc) then has exactly one arm on every
    path the scan follows.  Any other write to a tracked register forgets
    it.  Returns (consts, vcc) after the instruction; vcc is True / False /
    None (unknown)."""
    parts = [p.strip() for p in ops.split(",")] if ops else []
    dst = parts[0] if parts else ""
    m = re.fullmatch(_SREG, dst) if mn == "s_mov_b64" else None
    if m and len(parts) > 1 and parts[1] in ("-1", "0"):
        return dict(consts, **{dst: int(parts[1])}), (None if dst == "vcc" else vcc)
    if mn == "s_andn2_b64" and dst == "vcc" and len(parts) == 3 and parts[1] == "exec" and parts[2] in consts:
        return consts, consts[parts[2]] == 0
    # any write that touches a tracked pair (the pair itself, one of its
    # halves or a wider range) forgets it
    written = _sgprs(dst)
    if written:
        consts = {k: v for k, v in consts.items() if not (_sgprs(k) & written)}
    if dst == "vcc" or dst.startswith("vcc"):
        vcc = None
    return consts, vcc


def _sgprs(op):
    """The SGPR numbers an operand names (s7 -> {7}, s[44:45] -> {44, 45})."""
    m = re.fullmatch(r"s(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def check_vmcnt_protocol(insts, n_dma, n_wait, n_stores=N_STORES):
    """Every path from the function entry to each `s_waitcnt vmcnt(n_wait)`
    must end with [dma]+ [other]{>=n_stores} [dma]{n_dma} (see the module
    docstring).  Paths that the structurizer's flow variables rule out
    (`_flow_step`) are not followed.  Returns (n_waits_found, [failure
    strings])."""
    idx = {a: i for i, (a, _, _, _) in enumerate(insts)}
    waits = {i for i, (_, mn, ops, _) in enumerate(insts)
             if mn == "s_waitcnt" and re.search(rf"\bvmcnt\({n_wait}\)", ops)}
    keep = n_dma + n_stores + 8
    failures, seen, stack = [], set(), [(0, (), (), None)]
    while stack:
        i, tail, cst, vcc = stack.pop()
        consts = dict(cst)
        while i < len(insts):
            state = (i, tail, tuple(sorted(consts.items())), vcc)
            if state in seen:
                break
            seen.add(state)
            a, mn, ops, tgt = insts[i]
            if i in waits:
                k = len(tail)
                last = tail[k - n_dma:] if k >= n_dma else ()
                j = k - n_dma
                n_other = 0
                while j - 1 >= 0 and tail[j - 1] != "dma":
                    n_other += 1
                    j -= 1
                ok = (len(last) == n_dma and all(x == "dma" for x in last)
                      and (k - n_dma - 1 < 0 or tail[k - n_dma - 1] != "dma")
                      and n_other >= n_stores and j - 1 >= 0 and tail[j - 1] == "dma")
                if not ok:
                    failures.append(f"wait at 0x{a:x}: ops before it {list(tail)}")
            kind = _vmem_kind(mn, ops)
            if kind:
                tail = (tail + (kind,))[-keep:]
            if mn == "s_endpgm":
                break
            if mn == "s_branch":
                if tgt is None or tgt not in idx:
                    failures.append(f"unresolved branch at 0x{a:x}")
                    break
                i = idx[tgt]
                continue
            if mn in ("s_cbranch_vccnz", "s_cbranch_vccz") and vcc is not None:
                if tgt is None or tgt not in idx:
                    failures.append(f"unresolved branch at 0x{a:x}")
                    break
                if vcc == (mn == "s_cbranch_vccnz"):   # taken: the only feasible successor
                    i = idx[tgt]
                    continue
                i += 1
                continue
            if mn.startswith("s_cbranch") and mn != "s_cbranch_execz":
                if tgt is None or tgt not in idx:
                    failures.append(f"unresolved branch at 0x{a:x}")
                    break
                stack.append((idx[tgt], tail, tuple(sorted(consts.items())), vcc))
            consts, vcc = _flow_step(mn, ops, consts, vcc)
            i += 1
    return len(waits), failures


_VREG = re.compile(r"^(?:v(\d+)|v\[(\d+):(\d+)\]|a(\d+)|a\[(\d+):(\d+)\])$")


def _regs(op):
    """VGPR / AGPR numbers named by one operand ('v5', 'v[4:7]', 'a3'), else ()."""
    m = _VREG.match(op.strip())
    if not m:
        return ()
    if m.group(1):
        return (("v", int(m.group(1))),)
    if m.group(2):
        return tuple(("v", r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    if m.group(4):
        return (("a", int(m.group(4))),)
    return tuple(("a", r) for r in range(int(m.group(5)), int(m.group(6)) + 1))


def _store_data(mn, ops):
    """Data registers of a vector-memory store (buffer_store: first operand;
    global / flat / scratch_store: second), else None."""
    if not re.match(r"(buffer|global|flat|scratch)_store", mn):
        return None
    parts = [p.strip() for p in ops.split(",")]
    k = 0 if mn.startswith("buffer_") else 1
    return _regs(parts[k]) if len(parts) > k else None


def repeated_store_data(insts, min_run=4):
    """Rule 3 over one function's [(mnemonic, operands)] in program order:
    [(data registers, count)] for each run of >= min_run stores of the same
    data registers with no instruction writing any of them in between."""
    live, hits = {}, []
    for mn, ops in insts:
        data = _store_data(mn, ops)
        if data:
            live[data] = live.get(data, 0) + 1
            if live[data] == min_run:
                hits.append(data)
            continue
        if mn.startswith(("s_", "buffer_", "global_", "flat_", "scratch_", "ds_write", "ds_store")) and \
                not mn.startswith(("buffer_load", "global_load", "flat_load", "scratch_load")):
            continue   # writes no VGPR / AGPR
        first = ops.split(",")[0] if ops else ""
        dst = set(_regs(first))
        if dst:
            live = {k: v for k, v in live.items() if not dst.intersection(k)}
    return [(d, live.get(d, min_run)) for d in hits]


def asm_functions(text):
    """{name: [(mnemonic, operands)]} from `hipcc -S` output or objdump -d."""
    if re.search(r"^[0-9a-f]+ <\S+>:$", text, re.M):
        return {k: [(mn, ops) for _, mn, ops, _ in v] for k, v in functions(text).items()}
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+([a-z_][\w.]*)\s*(.*?)\s*(?:;.*)?$", line)
        if m and not m.group(1).startswith("."):
            funcs[cur].append((m.group(1), m.group(2)))
        if line.strip() == "s_endpgm":
            cur = None
    return funcs


def scan_repeated_stores(text):
    """{function: ["<regs> stored N times"]} for every function rule 3 flags."""
    out = {}
    for name, insts in asm_functions(text).items():
        hits = repeated_store_data(insts)
        if hits:
            out[name] = [f"{','.join(f'{k}{r}' for k, r in d)} stored {n} times" for d, n in hits]
    return out


def scan(lib=LIB):
    asm = disassemble(lib)
    funcs = functions(asm)
    pairs = {}
    for name, insts in funcs.items():
        m = SKIN_PAIR.search(name)
        if not m:
            continue
        trans = m.group(1) == "1"
        in_place = m.group(4) == "1"
        n_dma = N_ROWS + N_TR + (1 if trans else 0)
        n_st = N_STORES_IN_PLACE if in_place else N_STORES
        n_wait = (K_AHEAD - 1) * (n_st + n_dma)
        n_found, fails = check_vmcnt_protocol(insts, n_dma, n_wait, n_st)
        pairs[name] = {"trans": trans, "h3": m.group(2) == "1", "in_place": in_place, "dma_ops": n_dma,
                       "vmcnt": n_wait, "waits": n_found, "failures": fails[:5], "ok": n_found > 0 and not fails}
    packed = [l.strip() for l in asm.splitlines() if PACKED_FP32.search(l)]
    return asm, {"packed_fp32": len(packed), "packed_fp32_examples": packed[:5],
                 "skin_pair_vmcnt": pairs,
                 "repeated_store_data": scan_repeated_stores(asm),
                 "mfma": {op: len(re.findall(rf"\b{op}\b", asm))
                          for op in sorted(set(re.findall(r"\bv_mfma_\w+", asm)))}}


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--json"]
    _, rep = scan(*args)
    print(json.dumps(rep) if "--json" in sys.argv else json.dumps(rep, indent=1))
