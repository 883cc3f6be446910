# Round 5, twenty-second GPU session: the device error sum with tighter
# speculation bands (+-1 % candidates, +-0.2 % re-sum marking; session 21's
# +-10 % marked too many chunks to pack): chunk statistics of a C5 session,
# then C5 twice and the C3 line against variant hsum.
set -o pipefail
mkdir -p gpurun_out/r05/dsum3
timeout -k 10 300 python -u -m pytest tests/test_gpu_seqsum.py tests/test_gpu_parity.py -x -q -k "seqsum or device_chunk or c5_settings or adaptive or init_defaults" --timeout 250 --timeout-method thread > gpurun_out/r05/dsum3/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/dsum3/tests.log; exit 1; }
tail -1 gpurun_out/r05/dsum3/tests.log
timeout -k 10 300 python -u -c "
import wpt_loader, json
pkg = wpt_loader.load(); itf = pkg.interface
W, H = 1920, 1080
itf.init(W, H, 2, *pkg.scenes.scene_camera(2)); itf.store_mesh(1, pkg.scenes.triangle_cloud(100000))
itf.update_settings(2, 2, 1, 1, 0); itf.set_render_options(8, 0xBABABEBE, 0)
itf.compute(W * H * 1024); itf.sync(); st = itf.stats()
print(json.dumps({k: st[k] for k in ('sum_chunks', 'sum_resummed', 'sum_fetched')}))
itf.shutdown()
" > gpurun_out/r05/dsum3/chunk_stats.json 2> gpurun_out/r05/dsum3/chunk_stats.err || { echo STATSFAIL; tail -5 gpurun_out/r05/dsum3/chunk_stats.err; exit 1; }
cat gpurun_out/r05/dsum3/chunk_stats.json
AB_STEPS=4 bash tools/ab.sh c5=--config=c5 c5h=WPT_LIB_VARIANT=hsum,--config=c5 c5b=--config=c5 c5hb=WPT_LIB_VARIANT=hsum,--config=c5 base= h=WPT_LIB_VARIANT=hsum || exit 1
for n in c5 c5h c5b c5hb base h; do cp gpurun_out/ab_$n.json gpurun_out/r05/dsum3/; done
python -c "
import json
for n in ['base','h']:
    d=json.load(open('gpurun_out/r05/dsum3/ab_'+n+'.json')); print(n, round(d['value']), {k:round(x['value']) for k,x in (d.get('secondary') or {}).items()})
"
