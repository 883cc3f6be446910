set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/s30_c5.jsonl
for r in 1 2; do
for V in "" rc26 rc24; do
WPT_LIB_VARIANT=$V timeout -k 10 300 python tools/session_rate.py c5 --reps 1 "" 2>gpurun_out/s30_err_$V.txt | grep -v summary | sed "s/^{/{\"variant\": \"$V\", /" >> gpurun_out/s30_c5.jsonl || { echo FAIL $V; tail -3 gpurun_out/s30_err_$V.txt; }
done
done
python3 -c "
import json,statistics
r={}
for l in open('gpurun_out/s30_c5.jsonl'):
    d=json.loads(l); r.setdefault(d['variant'],[]).append(round(d['Mray/s']))
for k,v in r.items(): print('c5', k or 'base', v)"
: > gpurun_out/s30_init.jsonl
for V in "" rc26; do
WPT_LIB_VARIANT=$V timeout -k 10 300 python tools/session_rate.py init --reps 2 "" 2>/dev/null | tail -1 | sed "s/^/init $V /" || exit 1
done
