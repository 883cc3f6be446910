set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for t in 8 4; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --no-serial-step --opt pixel_tile=$t > gpurun_out/s23_t${t}_$i.json 2> gpurun_out/s23_t${t}_$i.err || { echo FAIL $t; tail -3 gpurun_out/s23_t${t}_$i.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/s23_t${t}_$i.json'));print('tile $t rep $i', round(d['value'],1), round(d['ms_per_step'],2))"
done
done
timeout -k 10 600 python tools/session_rate.py c3 --reps 3 "pixel_tile=8" "pixel_tile=4" > gpurun_out/s23_c3.jsonl 2> gpurun_out/s23_c3.err || exit 1
tail -1 gpurun_out/s23_c3.jsonl
