"""Disassemble every gfx950 code object of the built library and count the
instructions the design keeps out of it: packed fp32 VALU and
scalar-cache stores.  Writes <lib>.codegen.json next to the library; run by
__graft_entry__.build() and `make`, read by tests/test_codegen.py.

    python tools/codegen_report.py [path/to/libmano_hip.so]

(Disassembly runs here, at build time, in a process without the HIP runtime:
child processes of a process that has loaded the runtime make it crash later
in this container.)"""
import hashlib
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
WATCH = {
    "packed_fp32": re.compile(r"\bv_pk_(fma|mul|add)_f32\b"),
    "scalar_store": re.compile(r"\b(s_store_dword\w*|s_buffer_store\w*|s_scratch_store\w*|s_dcache_wb\w*|s_dcache_discard\w*|s_atomic_\w*|s_buffer_atomic_\w*)\b"),
}


def disassemble(lib):
    fat_dir = tempfile.mkdtemp()
    try:
        fat = os.path.join(fat_dir, "fatbin.bin")
        subprocess.run([shutil.which("objcopy"), f"--dump-section=.hip_fatbin={fat}", lib], check=True)
        data = open(fat, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        out = []
        for k, a in enumerate(starts):
            b = starts[k + 1] if k + 1 < len(starts) else len(data)
            part, co = os.path.join(fat_dir, f"b{k}.bin"), os.path.join(fat_dir, f"b{k}.co")
            open(part, "wb").write(data[a:b])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                            f"--output={co}"], check=True)
            out.append(subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co],
                                      check=True, capture_output=True, text=True).stdout)
        return "\n".join(out)
    finally:
        shutil.rmtree(fat_dir, ignore_errors=True)


def main(lib=LIB):
    asm = disassemble(lib)
    report = {
        "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
        "mfma": {m: n for m, n in sorted(
            {op: len(re.findall(rf"\b{op}\b", asm)) for op in set(re.findall(r"\bv_mfma_\w+", asm))}.items())},
        "counts": {k: len(rx.findall(asm)) for k, rx in WATCH.items()},
        "examples": {k: [l.strip() for l in asm.splitlines() if rx.search(l)][:5] for k, rx in WATCH.items()},
    }
    with open(lib + ".codegen.json", "w") as f:
        json.dump(report, f, indent=1)
    print(json.dumps({k: report[k] for k in ("mfma", "counts")}))


if __name__ == "__main__":
    main(*sys.argv[1:])
