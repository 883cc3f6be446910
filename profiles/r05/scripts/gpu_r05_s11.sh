# Round 5, eleventh GPU session: evidence for the final build (leaf batching
# on): kernel trace + PMC passes of the C3 bench workload (tools/profile.sh,
# full-instantiation keys), the wave-timeline probes of C3 and C5.
set -o pipefail
mkdir -p gpurun_out/r05
bash tools/profile.sh r05final || exit 1
timeout -k 10 300 python -u tools/probe_tails.py c3 64 > gpurun_out/r05/probe3_c3.json 2> gpurun_out/r05/probe3_c3.err || exit 1
timeout -k 10 300 python -u tools/probe_tails.py c5 1500 > gpurun_out/r05/probe3_c5.json 2> gpurun_out/r05/probe3_c5.err || exit 1
echo s11-done
