# Round 5, twenty-ninth GPU session: museum kernel stats + counters (BVH4
# walk with the f64 torus test), to see what bounds its traversal.
set -o pipefail
bash tools/profile.sh r05museum --config museum --steps 1 --warmup 0 --no-cpu-baseline --no-serial-step --no-secondary || exit 1
python3 - <<'PY'
import json, csv, glob
d = json.load(open('gpurun_out/prof_r05museum/pmc_summary.json'))
for k, v in d.items():
    if any(x in k for x in ('extend', 'shadow', 'shade')):
        print(k, {a: (round(b, 3) if isinstance(b, float) else b) for a, b in v.items() if not isinstance(b, dict)})
for f in glob.glob('gpurun_out/prof_r05museum/trace/**/*kernel_stats.csv', recursive=True):
    for x in list(csv.DictReader(open(f)))[:8]:
        print(x['Name'][:60], x['Calls'], round(float(x['AverageNs']) / 1e3, 1))
PY
