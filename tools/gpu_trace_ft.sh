# Kernel trace of one C3 step with the fast tree on extension rays, one lane
# (standalone kernel durations, incl. every exact drain launch).
# Usage: bash tools/gpu_trace_ft.sh NAME [bench args...]  (env, e.g. WPT_LIB_VARIANT, passes through)
export TMPDIR=/tmp
N=$1; shift
O=gpurun_out/tr_$N
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-serial-step --no-secondary --opt traversal=ft --opt ft_max_leaf=1 --opt ft_ctrav=0 --opt lanes=1 "$@" > $O/trace.log 2>&1 || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
echo "== $N $*"
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print(f"{k:60s} n={len(v):4d} sum={sum(v)/1e3:8.2f} ms  each(us)=" + " ".join(f"{x:.0f}" for x in v[:12]))
PY
