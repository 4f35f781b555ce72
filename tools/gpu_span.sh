set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/span
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -8 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu --path unfused --steps 100 --warmup 200 > $OUT/bench_unfused.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/span/bench_unfused.log").read().strip().splitlines()[-1])
for k, v in d["kernels"].items():
    print(k, round(v["ms"], 4), {x: round(v[x], 3) for x in ("frac", "achieved_GBs") if x in v})
PY
