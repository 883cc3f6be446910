# GPU suite on the working tree's product, then a same-session A/B against
# the committed build (variant head: make variant V=head from git HEAD), C3 and C5.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/t_new.log 2>&1; rc=$?
tail -1 gpurun_out/t_new.log; grep -E "^FAILED|^E " gpurun_out/t_new.log | head -20
[ $rc -eq 0 ] || exit 1
AB_STEPS=4 bash tools/ab.sh new= head=WPT_LIB_VARIANT=head new2= head2=WPT_LIB_VARIANT=head c5=--config=c5 c5h=WPT_LIB_VARIANT=head,--config=c5 ${AB_EXTRA}
for f in new head new2 head2 c5 c5h; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'],{k:round(v['value']) for k,v in (d.get('secondary') or {}).items()})"; done
