set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/s29_c3.jsonl
for r in 1 2 3 4; do
for V in "" lb12 lb20 m28 m36; do
WPT_LIB_VARIANT=$V timeout -k 10 300 python tools/session_rate.py c3 --reps 1 "" 2>/dev/null | grep -v summary | sed "s/^{/{\"variant\": \"$V\", /" >> gpurun_out/s29_c3.jsonl || { echo FAIL $V; exit 1; }
done
done
python3 -c "
import json,statistics
r={}; crc={}
for l in open('gpurun_out/s29_c3.jsonl'):
    d=json.loads(l); r.setdefault(d['variant'],[]).append(round(d['Mray/s'])); crc.setdefault(d['variant'],set()).add(d['crc'])
for k,v in r.items(): print(k or 'base', statistics.median(v), v, crc[k])"
