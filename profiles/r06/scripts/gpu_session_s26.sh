set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/s26_c3.jsonl
for r in 1 2 3 4; do
for V in "" glds; do
WPT_LIB_VARIANT=$V timeout -k 10 300 python tools/session_rate.py c3 --reps 1 "" 2>/dev/null | grep -v summary | sed "s/^{/{\"variant\": \"$V\", /" >> gpurun_out/s26_c3.jsonl || { echo FAIL $V; exit 1; }
done
done
python3 -c "
import json
r={}
for l in open('gpurun_out/s26_c3.jsonl'):
    d=json.loads(l); r.setdefault(d['variant'],[]).append(round(d['Mray/s']))
print(r)"
for V in "" glds; do
WPT_LIB_VARIANT=$V timeout -k 10 300 python tools/session_rate.py c5 --reps 1 "" 2>/dev/null | tail -1 | sed "s/^/c5 $V /" || exit 1
WPT_LIB_VARIANT=$V timeout -k 10 300 python tools/session_rate.py init --reps 2 "" 2>/dev/null | tail -1 | sed "s/^/init $V /" || exit 1
done
