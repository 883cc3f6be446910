set -o pipefail
timeout -k 10 300 python tools/probe_tails.py c5 4000 > gpurun_out/probe_c5_last.json 2> gpurun_out/probe_c5_last.err || { echo PROBEFAIL; tail -5 gpurun_out/probe_c5_last.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/probe_c5_last.json'))
print({k:v for k,v in d.items() if not isinstance(v,(list,dict))})"
