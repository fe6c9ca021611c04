set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out
bash tools/gpu_run.sh tests || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sort-bench --no-sweep > $O/b18.json 2> $O/b18.err || { tail -5 $O/b18.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/b18.json')); fr=d['frame']
print('fps', d['value'], 'serial', fr['serial_ms_per_frame'], fr['stage_ms'])
print('facade', json.dumps(fr.get('cpp_facade')))"
for c in c3 v2 v7; do timeout -k 10 120 python tools/valu_account.py $c > $O/valu_$c.txt 2>&1 || { tail -5 $O/valu_$c.txt; exit 1; }; cat $O/valu_$c.txt; done
