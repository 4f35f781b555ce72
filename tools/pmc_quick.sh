#!/bin/bash
# Quick PMC look at the fused forward: stall breakdown + MFMA busy + clock.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcq
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d $OUT/a -o p --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu "$@" > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES -d $OUT/b -o p --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu "$@" > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmcq/*/*counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        k = n.split('(')[0].split('::')[-1][:40]
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in acc.items():
    if 'mano' not in k and 'kernel' not in k: continue
    a = {c: sum(v)/len(v) for c, v in d.items()}
    print(k)
    for c, v in sorted(a.items()): print(f"   {c:28s} {v:.4g}")
    if 'GRBM_GUI_ACTIVE' in a and 'SQ_VALU_MFMA_BUSY_CYCLES' in a:
        cyc = a['GRBM_GUI_ACTIVE'] / 8
        print(f"   -> MFMA busy per SIMD {a['SQ_VALU_MFMA_BUSY_CYCLES']/1024/cyc:.2%} of {cyc:.0f} cycles")
PY
