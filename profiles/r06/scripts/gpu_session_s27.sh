set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/probe_tails.py c5 4000 > gpurun_out/probe_c5_final.json 2> gpurun_out/probe_c5_final.err || { echo PROBEFAIL; tail -5 gpurun_out/probe_c5_final.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/probe_c5_final.json'));print(d['compute_s'], d['launches_recorded'], d['gpu_wide'])"
