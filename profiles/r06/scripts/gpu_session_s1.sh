set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/session_rate.py c3 --reps 2 "chain=1,stagger=0" "chain=1,stagger=1,grid_pct=75" "chain=1,stagger=1,grid_pct=100" "chain=1,stagger=2,grid_pct=100" "chain=1,stagger=0,grid_pct=60" > gpurun_out/chain2_ab_c3.jsonl 2> gpurun_out/chain2_ab_c3.err || { echo ABFAIL; tail -5 gpurun_out/chain2_ab_c3.err; exit 1; }
tail -1 gpurun_out/chain2_ab_c3.jsonl
bash tools/profile_init.sh base "" && python3 -c "import json;d=json.load(open('gpurun_out/prof_init_base/phases.json'));print(d['window_ms'],d['queues_running_ms'],list(d['alone_ms'].items())[:6])"
