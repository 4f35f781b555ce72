set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/ab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu > $OUT/bench$i.log 2>&1 || exit $?
python -c "
import json; d = json.loads(open('$OUT/bench$i.log').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), 'M hands/s', {k: round(v['ms'],4) for k, v in d['kernels'].items()})"; done
