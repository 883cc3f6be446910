set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/s35_c3.jsonl
for r in 1 2 3 4; do
for Q in 4 8; do
GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python tools/session_rate.py c3 --reps 1 "" 2>/dev/null | grep -v summary | sed "s/^{/{\"hwq\": $Q, /" >> gpurun_out/s35_c3.jsonl || { echo FAIL $Q; exit 1; }
done
done
python3 -c "
import json
r={}
for l in open('gpurun_out/s35_c3.jsonl'):
    d=json.loads(l); r.setdefault(d['hwq'],[]).append(round(d['Mray/s']))
print(r)"
